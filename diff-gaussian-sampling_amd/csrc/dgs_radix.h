// dgs_radix.h -- the binning's stable LSD radix sort of (key, u32 value) pairs (gfx950).
//
// One launch per 8-bit digit place plus one histogram launch per sort, and NO zero-fill
// launches of its own: the digit histograms, tile tickets and look-back states live in one
// scratch region the caller zero-fills together with its other regions (ZeroList), so a
// two-place sort is 3 launches.  rocprim's onesweep (which this replaces in the binning) adds
// a histogram memset, a histogram-scan kernel and two memsets per place: 9 launches of >= 5 us
// each for the binning's 2-place sorts, more than the passes' own work at these sizes.
//
// A place (k_rs_pass): a block takes the next tile of kRsTile items in ticket order (so every
// tile's predecessors are running or done and the look-back terminates), ranks its keys
// stably -- per wave, 8 ballots find the lanes holding the same digit; per-wave running counts
// in LDS order the items (wave chunks are contiguous: the order is wave, item, lane = index
// order) -- publishes its per-digit counts, looks back per digit (one thread per digit) for
// the exclusive prefix over earlier tiles, scatters the tile into LDS in digit order and
// writes it out in runs of equal digits.  Look-back words are 8-byte {flag, count} granules
// under relaxed agent-scope atomics, no fences (see k_fused_scan in dgs_scan.h).
#pragma once
#include <algorithm>
#include <cstdint>

#include "dgs_internal.h"

namespace dgs {

constexpr int kRsBits = 8, kRsBins = 1 << kRsBits;
#ifndef DGS_RS_ITEMS
#define DGS_RS_ITEMS 16
#endif
constexpr int kRsThreads = 256, kRsWaves = kRsThreads / kWave, kRsItems = DGS_RS_ITEMS;
constexpr int kRsTile = kRsThreads * kRsItems;  // 4096 items (16 per thread), each wave a contiguous 1024
static_assert(kRsThreads == kRsBins, "one thread per digit in the look-back");
constexpr uint64_t kRsAgg = 1ull << 62, kRsPre = 2ull << 62, kRsVal = (1ull << 62) - 1;

// Host plan of one sort of n items over key bits [0, bits): scratch = [zeroed: histograms
// u32[kRsHistCopies][places][256], tickets u32[64], states u64[places][tiles][256]] [tmp keys
// u32[n]] [tmp values u32[n]].  zero_bytes from the start must be zero before the sort.  The
// histograms are kept in one copy per XCD (block b adds to copy b % 8: one word takes only ~88
// atomic adds per us) and summed by the passes.
constexpr int kRsHistCopies = 8;
struct RadixPlan {
    int64_t n = 0, tiles = 0;
    int places = 0;
    size_t o_tickets = 0, o_states = 0, zero_bytes = 0, o_tkeys = 0, o_tvals = 0, bytes = 0;
};

inline RadixPlan radix_plan(int64_t n, int bits) {
    RadixPlan p;
    p.n = n;
    p.places = n > 0 ? (std::max(bits, 1) + kRsBits - 1) / kRsBits : 0;
    p.tiles = (n + kRsTile - 1) / kRsTile;
    size_t o = align_up(4 * (size_t)kRsHistCopies * p.places * kRsBins, 256);
    p.o_tickets = o;
    o += 256;
    p.o_states = o;
    o = align_up(o + 8 * (size_t)p.places * (size_t)p.tiles * kRsBins, 256);
    p.zero_bytes = o;
    p.o_tkeys = o;
    o = align_up(o + 4 * (size_t)std::max<int64_t>(n, 1), 256);
    p.o_tvals = o;
    o = align_up(o + 4 * (size_t)std::max<int64_t>(n, 1), 256);
    p.bytes = o;
    return p;
}

__device__ __forceinline__ uint32_t rs_digit(uint32_t key, int shift) { return (key >> shift) & (kRsBins - 1); }

// All places' digit counts in one read of the keys (LDS histograms, one global add per bin).
// ndev (optional, device): the item count is min(n, *ndev) -- a sort sized by a capacity whose
// exact count only the device knows (the graph-capturable binning).
template <typename KT>
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(int64_t n, const KT *__restrict__ keys, int places,
                                                        uint32_t *__restrict__ hist, const int64_t *__restrict__ ndev) {
    __shared__ uint32_t h[4 * kRsBins];
    if (ndev) n = min(n, max(sload(ndev), (int64_t)0));
    for (int i = threadIdx.x; i < places * kRsBins; i += kRsThreads) h[i] = 0u;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * kRsThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kRsThreads) {
        const uint32_t k = keys[i];
        for (int p = 0; p < places; ++p) atomicAdd(&h[p * kRsBins + rs_digit(k, p * kRsBits)], 1u);
    }
    __syncthreads();
    uint32_t *hc = hist + (size_t)(blockIdx.x & (kRsHistCopies - 1)) * places * kRsBins;
    for (int i = threadIdx.x; i < places * kRsBins; i += kRsThreads)
        if (h[i]) atomicAdd(&hc[i], h[i]);
}

// exclusive scan over the block of one value per thread
__device__ __forceinline__ uint32_t rs_block_excl(uint32_t x, uint32_t *wsum) {
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint32_t inc = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, kWave);
        if (lane >= d) inc += y;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int i = 0; i < kRsWaves; ++i)
        if (i < w) pre += wsum[i];
    __syncthreads();
    return pre + inc - x;
}

// One digit place: kin/vin -> kout/vout, stable by digit (key >> shift) & 255.  hist: this
// place's global digit counts; states: this place's [tiles][256] look-back words; ticket: this
// place's tile counter (both zero before the launch).  grid = tiles.  A look-back that waits
// implausibly long (a broken invariant, never expected) gives up and sets *err instead of
// hanging the device.
// Extra: called as extra(position, value) for every item the pass writes (the last place of a
// sort may scatter a payload gathered by value, e.g. the samples' pair rows); RsNone: nothing.
struct RsNone {
    __device__ __forceinline__ void operator()(uint32_t, uint32_t) const {}
};

template <typename KT, class Extra>
__global__ __launch_bounds__(kRsThreads) void k_rs_pass(int64_t n, const KT *__restrict__ kin, KT *__restrict__ kout,
                                                        const uint32_t *__restrict__ vin, uint32_t *__restrict__ vout,
                                                        int shift, const uint32_t *__restrict__ hist, int hstride,
                                                        unsigned long long *__restrict__ states,
                                                        uint32_t *__restrict__ ticket, uint32_t *__restrict__ err,
                                                        Extra extra, const int64_t *__restrict__ ndev) {
    __shared__ uint32_t sk[kRsTile], sv[kRsTile];
    if (ndev) n = min(n, max(sload(ndev), (int64_t)0));  // (tiles past it publish empty counts)
    __shared__ uint32_t cnt[kRsWaves][kRsBins];
    __shared__ uint32_t s_tstart[kRsBins], s_delta[kRsBins];
    __shared__ uint32_t wsum[kRsWaves];
    __shared__ int s_tile;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    if (tid == 0) s_tile = (int)atomicAdd(ticket, 1u);
#pragma unroll
    for (int q = 0; q < kRsWaves; ++q) cnt[q][tid] = 0u;
    uint32_t gcount = 0;  // (the histogram's copies, hstride words apart)
#pragma unroll
    for (int q = 0; q < kRsHistCopies; ++q) gcount += hist[q * hstride + tid];
    const uint32_t gbase = rs_block_excl(gcount, wsum);  // (its barriers also publish s_tile / cnt)
    const int64_t tile = s_tile;
    const int64_t base = tile * kRsTile;
    const int64_t cb = base + (int64_t)w * (kRsItems * kWave) + lane;

    uint32_t key[kRsItems], val[kRsItems], rank[kRsItems];
#pragma unroll
    for (int k = 0; k < kRsItems; ++k) {
        const int64_t i = cb + (int64_t)k * kWave;
        const bool ok = i < n;
        key[k] = ok ? (uint32_t)kin[i] : 0u;
        val[k] = ok ? (vin ? vin[i] : (uint32_t)i) : 0u;  // (vin null: the values are the input positions)
    }
    const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < kRsItems; ++k) {
        const bool ok = cb + (int64_t)k * kWave < n;
        const uint32_t d = rs_digit(key[k], shift);
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < kRsBits; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        uint32_t c0 = 0u;
        if (ok) c0 = cnt[w][d];
        rank[k] = c0 + (uint32_t)__popcll(peers & lt);
        // the highest lane of each digit group advances the wave's count (after every lane's read)
        if (ok && (peers >> lane) == 1ull) cnt[w][d] = c0 + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // per digit (thread = digit): the tile's count, the waves' exclusive offsets
    uint32_t tot = 0;
#pragma unroll
    for (int q = 0; q < kRsWaves; ++q) {
        const uint32_t c = cnt[q][tid];
        cnt[q][tid] = tot;
        tot += c;
    }
    unsigned long long *st = states + tile * kRsBins + tid;
    __hip_atomic_store(st, (tile == 0 ? kRsPre : kRsAgg) | (unsigned long long)tot, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tstart = rs_block_excl(tot, wsum);
    uint64_t pre = 0;
    if (tile > 0) {
        uint32_t spins = 0;
        for (int64_t j = tile - 1; j >= 0;) {
            const unsigned long long v =
                __hip_atomic_load(states + j * kRsBins + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((v & ~kRsVal) == 0ull) {  // not yet published: spin
                if (++spins > (1u << 22)) {
                    atomicOr(err, 1u);
                    break;
                }
                continue;
            }
            pre += v & kRsVal;
            if (v & kRsPre) break;
            --j;
        }
        __hip_atomic_store(st, kRsPre | (pre + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_tstart[tid] = tstart;
    s_delta[tid] = gbase + (uint32_t)pre - tstart;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRsItems; ++k) {
        if (cb + (int64_t)k * kWave < n) {
            const uint32_t d = rs_digit(key[k], shift);
            const uint32_t pos = s_tstart[d] + cnt[w][d] + rank[k];
            sk[pos] = key[k];
            sv[pos] = val[k];
        }
    }
    __syncthreads();
    const int cnt_tile = n - base < kRsTile ? (int)(n - base) : kRsTile;
    for (int i = tid; i < cnt_tile; i += kRsThreads) {
        const uint32_t kk = sk[i];
        const uint32_t o = s_delta[rs_digit(kk, shift)] + (uint32_t)i;
        const uint32_t v = sv[i];
        if ((int64_t)o >= n) continue;  // (only after a look-back gave up: the sort has failed, err is set)
        kout[o] = (KT)kk;
        vout[o] = v;
        extra(o, v);
    }
}

// The sort of n <= p.n items: keys kin (KT) / values vin -> kout / vout, stable, over the key
// bits the plan was made for (vin null: the values are the input positions 0 .. n - 1).  scratch: p.bytes, its first p.zero_bytes zero-filled beforehand
// (once: a plan's scratch serves one sort).  The look-back's give-up word is tickets[63].
// hist_ready: the keys' producer has already added their digit counts into the plan's
// histograms (radix_hist; dgs_preprocess.hip's RsHist), so the histogram launch is skipped.
template <typename KT, class Extra = RsNone>
static hipError_t radix_sort(const RadixPlan &p, int64_t n, char *scratch, const KT *kin, KT *kout,
                             const uint32_t *vin, uint32_t *vout, hipStream_t s, bool hist_ready = false,
                             Extra extra = Extra{}, const int64_t *ndev = nullptr) {
    if (n <= 0) return hipSuccess;
    if (n > p.n) return hipErrorInvalidValue;
    uint32_t *hist = reinterpret_cast<uint32_t *>(scratch);
    uint32_t *tickets = reinterpret_cast<uint32_t *>(scratch + p.o_tickets);
    uint32_t *err = tickets + 63;
    const int64_t tiles = (n + kRsTile - 1) / kRsTile;
    unsigned long long *states = reinterpret_cast<unsigned long long *>(scratch + p.o_states);
    KT *tk = reinterpret_cast<KT *>(scratch + p.o_tkeys);
    uint32_t *tv = reinterpret_cast<uint32_t *>(scratch + p.o_tvals);
    const unsigned hb = (unsigned)(tiles < 1024 ? tiles : 1024);
    if (!hist_ready) k_rs_hist<KT><<<hb, kRsThreads, 0, s>>>(n, kin, p.places, hist, ndev);
    const KT *ki = kin;
    const uint32_t *vi = vin;
    for (int q = 0; q < p.places; ++q) {
        const bool to_out = ((p.places - 1 - q) & 1) == 0;  // the last place writes kout / vout
        KT *ko = to_out ? kout : tk;
        uint32_t *vo = to_out ? vout : tv;
        if (q == p.places - 1)  // (the last place: the payload too)
            k_rs_pass<KT, Extra><<<(unsigned)tiles, kRsThreads, 0, s>>>(
                n, ki, ko, vi, vo, q * kRsBits, hist + q * kRsBins, p.places * kRsBins,
                states + (size_t)q * p.tiles * kRsBins, tickets + q, err, extra, ndev);
        else
            k_rs_pass<KT, RsNone><<<(unsigned)tiles, kRsThreads, 0, s>>>(
                n, ki, ko, vi, vo, q * kRsBits, hist + q * kRsBins, p.places * kRsBins,
                states + (size_t)q * p.tiles * kRsBins, tickets + q, err, RsNone{}, ndev);
        ki = ko;
        vi = vo;
    }
    return hipGetLastError();
}

}  // namespace dgs
