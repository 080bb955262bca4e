// dgs_scan.h -- device-wide primitives of the binning and the neighbour search (gfx950):
// a stable LSD radix sort of (key, u32 value) pairs on rocprim's onesweep algorithm, and
// exclusive / inclusive prefix sums.  Both are chosen to keep the code objects small: the
// first call of a HIP module loads every kernel it holds, and the generic library entry points
// (hipcub::DeviceScan, rocprim::radix_sort_pairs with its block-sort and merge-sort branches)
// instantiated ~450 kernels, 2/3 of the preprocess code object (first call 20 ms -> 6.4 ms).
#pragma once
#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>

#include "dgs_internal.h"

namespace dgs {

// The branch rocprim::radix_sort_pairs takes for large inputs, called directly
// (rocprim::detail::radix_sort_onesweep_impl).
template <typename KT>
static hipError_t onesweep_pairs(void *tmp, size_t &bytes, const KT *kin, KT *kout, const uint32_t *vin,
                                 uint32_t *vout, size_t n, unsigned b0, unsigned b1, hipStream_t s) {
    if (n == 0) {  // (rocprim's block-sort branch returns here)
        if (tmp == nullptr) bytes = 4;
        return hipSuccess;
    }
    bool in_output = true;
    return rocprim::detail::radix_sort_onesweep_impl<rocprim::default_config, false>(
        tmp, bytes, kin, static_cast<KT *>(nullptr), kout, vin, static_cast<uint32_t *>(nullptr), vout, n,
        in_output, rocprim::identity_decomposer{}, b0, b1, s, false, false);
}

// Exclusive prefix sums of one or two count arrays of length n: tile sums, one block scanning
// them, then a downsweep (3 launches for both arrays).  Replaces hipcub::DeviceScan, whose ~210
// kernel instantiations were a third of this code object.
constexpr int kScanItems = 8, kScanTile = kBlock * kScanItems;

static inline int64_t scan_tiles(int64_t n) { return (n + kScanTile - 1) / kScanTile; }
template <typename T>
static inline size_t scan_scratch_bytes(int64_t n) { return sizeof(T) * 2 * (size_t)std::max<int64_t>(scan_tiles(n), 1); }

// exclusive scan of x over the block; total = the block's sum
template <typename T>
__device__ __forceinline__ T block_excl_scan(T x, T &total) {
    __shared__ T wsum[kWavesPerBlock];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    T inc = x;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const T y = __shfl_up(inc, d, kWave);
        if (lane >= d) inc += y;
    }
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    T pre = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < kWavesPerBlock; ++i) {
        if (i < w) pre += wsum[i];
        total += wsum[i];
    }
    __syncthreads();
    return pre + inc - x;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scan_reduce(int64_t n, const T *__restrict__ a, const T *__restrict__ b,
                                                        T *__restrict__ part) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    T sa = 0, sb = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + k * kBlock + threadIdx.x;
        if (i < n) {
            sa += a[i];
            if (b) sb += b[i];
        }
    }
    T ta, tb = 0;
    (void)block_excl_scan(sa, ta);
    if (b) (void)block_excl_scan(sb, tb);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = ta;
        if (b) part[gridDim.x + blockIdx.x] = tb;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scan_parts(int64_t nt, int arrays, T *__restrict__ part) {
    for (int r = 0; r < arrays; ++r) {
        T carry = 0;
        for (int64_t c0 = 0; c0 < nt; c0 += kBlock) {
            const int64_t i = c0 + threadIdx.x;
            const T x = i < nt ? part[r * nt + i] : (T)0;
            T tot;
            const T e = block_excl_scan(x, tot);
            if (i < nt) part[r * nt + i] = carry + e;
            carry += tot;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scan_down(int64_t n, const T *__restrict__ a, T *__restrict__ ao,
                                                      const T *__restrict__ b, T *__restrict__ bo,
                                                      const T *__restrict__ part, bool inclusive) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    for (int r = 0; r < (b ? 2 : 1); ++r) {
        const T *in = r ? b : a;
        T *out = r ? bo : ao;
        T carry = part[r * (int64_t)gridDim.x + blockIdx.x];
        for (int k = 0; k < kScanItems; ++k) {
            const int64_t i = base + k * kBlock + threadIdx.x;
            const T x = i < n ? in[i] : (T)0;
            T tot;
            const T e = block_excl_scan(x, tot);
            if (i < n) out[i] = carry + e + (inclusive ? x : (T)0);
            carry += tot;
        }
    }
}

// ao = exclusive (inclusive) scan of a, bo = of b (b may be null); part: scan_scratch_bytes<T>(n)
template <typename T>
static void scan_excl(int64_t n, const T *a, T *ao, const T *b, T *bo, T *part, hipStream_t s,
                      bool inclusive = false) {
    if (n <= 0) return;
    const int64_t nt = scan_tiles(n);
    k_scan_reduce<T><<<(unsigned)nt, kBlock, 0, s>>>(n, a, b, part);
    k_scan_parts<T><<<1, kBlock, 0, s>>>(nt, b ? 2 : 1, part);
    k_scan_down<T><<<(unsigned)nt, kBlock, 0, s>>>(n, a, ao, b, bo, part, inclusive);
}

// ---- single-pass exclusive scan with decoupled look-back, fused with its producer and consumer
// A chain "per-element counts -> exclusive scan -> per-element outputs" in ONE launch (the
// three-kernel scan above plus the two kernels around it were five launches of ~5 us each, most
// of their time launch overhead at the binning's sizes).  Tiles of kBlock * ITEMS elements are
// taken in ticket order (atomic counter), so every tile's predecessors are running or done and
// the look-back always terminates; wave 0 looks back 64 tiles at a time.  A look-back word is
// one 8-byte {flag, value} granule written and polled with RELAXED agent-scope atomics (sc1
// stores / loads, served past the non-coherent per-XCD L2s): the value travels in the flag's
// own word, so no fence is needed -- an agent-scope release is a write-back of the XCD's whole
// L2 and an acquire an L1 invalidate (MI355X_MICROARCH.md), and with them this scan took ~200 us.  NA (1 or 2) arrays of
// unsigned counts are scanned side by side.  ITEMS = 1 where the consumer does real work per
// element (unit lists), more where it is a plain store.
//   prod(i, v[NA])            : the counts of element i
//   cons(i, v[NA], excl[NA])  : the outputs of element i given its exclusive prefixes
//   last(total[NA])           : once, by the block holding element n - 1 (totals, counters)
// state: fused_scan_state_words(n, NA, ITEMS) 64-bit words, ZERO-FILLED before the launch.
constexpr uint64_t kFuseAgg = 1ull << 62, kFusePre = 2ull << 62, kFuseVal = (1ull << 62) - 1;

static inline int64_t fused_scan_tiles(int64_t n, int items) { return (n + (int64_t)kBlock * items - 1) / ((int64_t)kBlock * items); }
static inline size_t fused_scan_state_words(int64_t n, int NA, int items) {
    return 1 + (size_t)NA * std::max<int64_t>(fused_scan_tiles(n, items), 1);
}

template <int NA, int ITEMS, class Prod, class Cons, class Last>
__global__ __launch_bounds__(kBlock) void k_fused_scan(int64_t n, unsigned long long *__restrict__ state, Prod prod,
                                                       Cons cons, Last last) {
    __shared__ int tile_s;
    __shared__ uint64_t pre_s[NA], tot_s[NA];
    if (threadIdx.x == 0) tile_s = (int)atomicAdd(reinterpret_cast<unsigned int *>(state), 1u);
    __syncthreads();
    const int tile = tile_s;
    unsigned long long *st = state + 1;
    const int64_t i0 = ((int64_t)tile * kBlock + threadIdx.x) * ITEMS;  // blocked: ITEMS per thread
    uint64_t v[ITEMS][NA], sum[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) sum[a] = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        uint64_t x[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) x[a] = 0;
        if (i0 + k < n) prod(i0 + k, x);
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            v[k][a] = x[a];
            sum[a] += x[a];
        }
    }
    uint64_t excl[NA], agg[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) excl[a] = block_excl_scan<uint64_t>(sum[a], agg[a]);
    if (threadIdx.x < kWave) {  // wave 0: publish the aggregate, look back, publish the prefix
        const int lane = threadIdx.x;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            if (lane == 0)
                __hip_atomic_store(&st[(int64_t)tile * NA + a], (tile == 0 ? kFusePre : kFuseAgg) | agg[a],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint64_t pre = 0;
            for (int j = tile - 1; j >= 0; j -= kWave) {
                const int jj = j - lane;  // lane 0 = the nearest predecessor
                uint64_t w = kFusePre;    // (before tile 0: a zero prefix)
                if (jj >= 0)
                    do {
                        w = __hip_atomic_load(&st[(int64_t)jj * NA + a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } while ((w & ~kFuseVal) == 0);
                const uint64_t pm = __ballot((w & kFusePre) != 0);
                const int stop = pm ? __builtin_ctzll(pm) : kWave;  // lanes <= stop contribute
                uint64_t c = lane <= stop ? (w & kFuseVal) : 0;
#pragma unroll
                for (int off = kWave / 2; off > 0; off >>= 1) c += __shfl_xor(c, off);
                pre += c;
                if (pm) break;
            }
            if (lane == 0) {
                if (tile > 0)
                    __hip_atomic_store(&st[(int64_t)tile * NA + a], kFusePre | (pre + agg[a]), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                pre_s[a] = pre;
                tot_s[a] = pre + agg[a];
            }
        }
    }
    __syncthreads();
    uint64_t run[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) run[a] = pre_s[a] + excl[a];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (i0 + k < n) cons(i0 + k, v[k], run);
#pragma unroll
        for (int a = 0; a < NA; ++a) run[a] += v[k][a];
    }
    if (n > 0 && (int64_t)tile == (n - 1) / ((int64_t)kBlock * ITEMS) && threadIdx.x == 0) {
        uint64_t t[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) t[a] = tot_s[a];
        last(t);
    }
}

template <int NA, int ITEMS, class Prod, class Cons, class Last>
static hipError_t fused_scan(int64_t n, unsigned long long *state, Prod prod, Cons cons, Last last, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_fused_scan<NA, ITEMS><<<(unsigned)fused_scan_tiles(n, ITEMS), kBlock, 0, s>>>(n, state, prod, cons, last);
    return hipGetLastError();
}

}  // namespace dgs
