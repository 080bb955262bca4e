// dgs_aggregate.hip -- neighbour aggregation (gfx950).
//
// Replaces aggregate_neighbors.cu (kr4b/diff-gaussian-sampling):
//   findCollisions + preprocess (18-127, 323-367) -> dgs_agg_preprocess
//   aggregateNeighbors        (129-208, 369-415) -> dgs_agg_forward
//   aggregateNeighborsBackward (210-321, 417-475) -> dgs_agg_backward
//
// Neighbour lists.  The reference tests every (i, j) pair into a P x P bool matrix (1 TB at
// P = 1M).  Here the Gaussians are radix-sorted into a uniform grid whose cell is at least
// twice the largest search radius 0.2 * radius, packed in cell order as {x, y, r, id}, and one
// wave per row walks the cells that can hold a neighbour -- the direct neighbourhood and, per
// axis, the images at +2k that the reference's one-sided torus wrap
// `min(dx, |2 - fmod(|dx|, 2)|)` can bring close (only a positive dx wraps) -- evaluating the
// reference predicate bit-exactly.  Pass 1 counts; pass 2 collects the row's neighbours in LDS,
// bitonic-sorts them into the reference's ascending-j slot order and writes the slots.  Rows
// with more neighbours than the wave's LDS holds are emitted in id windows.
//
// Forward.  One wave per row, lanes over slots.  The reference adds transform^T * embedded
// into the output for every slot (2 L^2 FLOP per slot); here each lane accumulates
// a[j] += dw (emb + fac * features[idx][j]) over its slots, one cross-lane reduce-scatter per
// row forms a, and out = transform^T a (same sum, different rounding order).
//
// Backward.  One wave per row.  Per slot the reference's j-loops collapse onto two row sums,
// S1 = sum_j st[j] and S2 = sum_j st[j] features[idx][j] (st = transform dL_row):
// sum_j te_j = dc (emb S1 + fac S2), and the distance-transform / frequency terms need only
// dcw S1 and dcw S2.  Query gradients and the row's a are reduced in registers; transform's
// gradient is A^T dL over the rows' a (a second, small kernel); the neighbours' feature and
// key gradients are scattered with float atomics as in the reference; the distance-transform
// and frequency gradients are per-lane LDS partials, flushed once per wave.

#include <algorithm>
#include <vector>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "dgs_internal.h"
#include "dgs_render.h"
#include "dgs_scan.h"

namespace dgs {

constexpr int kAggNMax = 2048;  // neighbour ids a wave sorts at once (wave_sort_keys: <= 32 per lane)
constexpr int kAggMaxCells = 1 << 24;

struct AggGeom {
    int D;
    int nc[2];     // grid cells per axis
    double lo[2];  // grid origin (min of the valid means)
    double hi[2];  // max of the valid means
    double cs;     // cell size
    float rmax;    // max 0.2 * radius over valid Gaussians
};

// float <-> order-preserving uint (min/max atomics on floats of any sign)
__device__ __forceinline__ uint32_t f2o(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
static inline float o2f(uint32_t o) {
    const uint32_t b = (o & 0x80000000u) ? (o & 0x7fffffffu) : ~o;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}

// aggregate_neighbors.cu:29-34: r = radii * 0.2 (double literal, rounded to float); r < 1e-6
// takes no part.
__device__ __forceinline__ float agg_r(float radius) { return (float)((double)radius * 0.2); }
__device__ __forceinline__ bool agg_valid(float r) { return (double)r >= 1e-6; }

// stats: kAggStatCopies copies of [rmax, min[2], max[2]] (order-preserving u32 codes), kAggStatStride
// words apart; a wave reduces its lanes first and block b adds to copy b % 8 (one word takes only
// ~88 atomic ops per us: one atomic per lane on five words was the kernel's whole cost).
constexpr int kAggStatCopies = 8, kAggStatStride = 32;
__global__ void k_agg_prep(int P, int D, const float *__restrict__ means, const float *__restrict__ radii,
                           uint32_t *__restrict__ stats) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[5] = {0u, 0xffffffffu, 0xffffffffu, 0u, 0u};
    if (i < P) {
        const float r = agg_r(radii[i]);
        if (agg_valid(r)) {
            v[0] = f2o(r);
            for (int d = 0; d < D; ++d) {
                const uint32_t m = f2o(means[(int64_t)i * D + d]);
                v[1 + d] = m;
                v[3 + d] = m;
            }
        }
    }
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        v[0] = max(v[0], (uint32_t)__shfl_xor((int)v[0], off));
        for (int d = 0; d < 2; ++d) {
            v[1 + d] = min(v[1 + d], (uint32_t)__shfl_xor((int)v[1 + d], off));
            v[3 + d] = max(v[3 + d], (uint32_t)__shfl_xor((int)v[3 + d], off));
        }
    }
    if ((threadIdx.x & (kWave - 1)) == 0 && v[0] != 0u) {
        uint32_t *st = stats + (blockIdx.x & (kAggStatCopies - 1)) * kAggStatStride;
        atomicMax(&st[0], v[0]);
        for (int d = 0; d < D; ++d) {
            atomicMin(&st[1 + d], v[1 + d]);
            atomicMax(&st[3 + d], v[3 + d]);
        }
    }
}

__device__ __forceinline__ int agg_cell_1d(const AggGeom &g, int d, double x) {
    const double c = floor((x - g.lo[d]) / g.cs);
    return c < 0.0 ? 0 : (c >= (double)g.nc[d] ? g.nc[d] - 1 : (int)c);
}

__global__ void k_agg_keys(int P, AggGeom g, const float *__restrict__ means, const float *__restrict__ radii,
                           uint32_t *__restrict__ keys, uint32_t *__restrict__ ids) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    uint32_t key = (uint32_t)(g.nc[0] * g.nc[1]);  // not a neighbour of anything: sorts last
    if (agg_valid(agg_r(radii[i]))) {
        const int cx = agg_cell_1d(g, 0, means[(int64_t)i * g.D]);
        const int cy = g.D == 2 ? agg_cell_1d(g, 1, means[(int64_t)i * 2 + 1]) : 0;
        key = (uint32_t)(cy * g.nc[0] + cx);
    }
    keys[i] = key;
    ids[i] = (uint32_t)i;
}

// Candidates packed in cell order as {x, y, r, id}.
__global__ void k_agg_pack(int P, int D, const uint32_t *__restrict__ ids, const float *__restrict__ means,
                           const float *__restrict__ radii, float4 *__restrict__ cand) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= P) return;
    const uint32_t j = ids[t];
    cand[t] = make_float4(means[(int64_t)j * D], D == 2 ? means[(int64_t)j * D + 1] : 0.0f, agg_r(radii[j]),
                          __uint_as_float(j));
}

// cstart[c] = first sorted position whose key is >= c, for c in [0, ncells].
__global__ void k_agg_cell_start(int ncells, int P, const uint32_t *__restrict__ keys, int32_t *__restrict__ cstart) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c > ncells) return;
    int lo = 0, hi = P;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < (uint32_t)c) lo = mid + 1;
        else hi = mid;
    }
    cstart[c] = lo;
}

// min(dx, |2 - fmod(|dx|, 2)|) of the reference (aggregate_neighbors.cu:43-46), evaluated there
// in double and rounded to float.  fmod is exact, 2 - r rounds once, and rounding is monotonic
// (so min commutes with it): this float evaluation is bit-identical.
__device__ __forceinline__ float torus_dx(float dx) {
    const float ax = fabsf(dx);
    const float r = ax < 2.0f ? ax : fmodf(ax, 2.0f);
    return fminf(dx, fabsf(2.0f - r));
}

// findCollisions' predicate (aggregate_neighbors.cu:36-53): float, no contraction.
__device__ __forceinline__ bool agg_collides(int D, float mix, float miy, float ri, float4 cj) {
    DGS_NO_CONTRACT
    if (!agg_valid(cj.z)) return false;
    const float dx = torus_dx(cj.x - mix);
    float dist = dx * dx;
    if (D == 2) {
        const float dy = torus_dx(cj.y - miy);
        dist = dist + dy * dy;
    }
    const float radius = ri + cj.z;
    return !(dist > radius * radius);
}

// Per-axis candidate cell ranges of a row: the direct window [m - R, m + R] and the images
// [m + 2k - R, m + 2k] (k >= 1) that a positive dx can wrap onto, widened by a rounding
// tolerance and merged into disjoint ranges.
struct AxisRanges {
    int n;
    int lo[8], hi[8];
};

__device__ inline void agg_axis_ranges(const AggGeom &g, int d, float m, float R, AxisRanges &out) {
    out.n = 0;
    for (int k = 0;; ++k) {
        const double tol = 1e-5 * (1.0 + fabs((double)m) + 2.0 * k);
        const double a = (double)m + 2.0 * k - R - tol;
        const double b = (double)m + (k == 0 ? (double)R : 2.0 * k) + tol;
        if (a > g.hi[d]) break;
        if (b < g.lo[d]) continue;
        const int c0 = agg_cell_1d(g, d, a), c1 = agg_cell_1d(g, d, b);
        if (out.n > 0 && c0 <= out.hi[out.n - 1] + 1) {
            out.hi[out.n - 1] = max(out.hi[out.n - 1], c1);
        } else if (out.n == 8) {  // pathological spread: the whole axis
            out.n = 1;
            out.lo[0] = 0;
            out.hi[0] = g.nc[d] - 1;
            return;
        } else {
            out.lo[out.n] = c0;
            out.hi[out.n] = c1;
            ++out.n;
        }
    }
}

// Visit every candidate of row i: wave-uniform loops over cell ranges, lanes over members;
// f(j, ok) is called by every lane (ok = the lane holds a neighbour j).
template <class Fn>
__device__ inline void agg_for_candidates(const AggGeom &g, float mix, float miy, float ri,
                                          const float4 *__restrict__ cand, const int32_t *__restrict__ cstart,
                                          int lane, Fn f) {
    const float R = ri + g.rmax;
    AxisRanges ax, ay;
    agg_axis_ranges(g, 0, mix, R, ax);
    if (g.D == 2) {
        agg_axis_ranges(g, 1, miy, R, ay);
    } else {
        ay.n = 1;
        ay.lo[0] = ay.hi[0] = 0;
    }
    for (int ry = 0; ry < ay.n; ++ry)
        for (int cy = ay.lo[ry]; cy <= ay.hi[ry]; ++cy)
            for (int rx = 0; rx < ax.n; ++rx) {
                // the cells of one x range are contiguous in the sorted order
                const int row = cy * g.nc[0];
                const int b = cstart[row + ax.lo[rx]], e = cstart[row + ax.hi[rx] + 1];
                for (int t0 = b; t0 < e; t0 += kWave) {
                    const int t = t0 + lane;
                    bool ok = false;
                    uint32_t j = 0;
                    if (t < e) {
                        const float4 c = cand[t];
                        j = __float_as_uint(c.w);
                        ok = agg_collides(g.D, mix, miy, ri, c);
                    }
                    f(j, ok);
                }
            }
}

__global__ __launch_bounds__(kBlock) void k_agg_count(int P, AggGeom g, const float *__restrict__ means,
                                                      const float *__restrict__ radii,
                                                      const float4 *__restrict__ cand,
                                                      const int32_t *__restrict__ cstart,
                                                      const uint32_t *__restrict__ order,
                                                      int64_t *__restrict__ counts) {
    const int lane = threadIdx.x & (kWave - 1);
    const int stride = gridDim.x * kWavesPerBlock;
    for (int w = wave_unit_index(P); w < P; w += stride) {
        const int i = (int)order[w];  // rows in cell order: concurrent waves share neighbours in L2
        int64_t n = 0;
        const float ri = agg_r(radii[i]);
        if (agg_valid(ri)) {
            const float mix = means[(int64_t)i * g.D], miy = g.D == 2 ? means[(int64_t)i * 2 + 1] : 0.0f;
            agg_for_candidates(g, mix, miy, ri, cand, cstart, lane,
                               [&](uint32_t, bool ok) { n += __popcll(__ballot(ok)); });
        }
        if (lane == 0) counts[i] = n;
    }
}

// X[d] of aggregate_neighbors.cu:91-101 (fmod(X, 2.0) -+ 2.0 in double: exact as in torus_dx).
__device__ __forceinline__ float agg_wrap(float x) {
    if (fabsf(x) > 1.0f) return x >= 0.0f ? fmodf(x, 2.0f) - 2.0f : fmodf(x, 2.0f) + 2.0f;
    return x;
}

// One slot of aggregate_neighbors.cu:84-119: X, power with the neighbour's conic, scaled X,
// density; index -1 and density 0 when power > 0.  Returns the density added to the total.
__device__ __forceinline__ float agg_slot(int D, float mix, float miy, float inv_r, const float *mj,
                                          const float *con, int64_t j, int64_t *idx_out, float *X_out,
                                          float *dens_out) {
    DGS_NO_CONTRACT
    const float X0 = agg_wrap(mj[0] - mix);
    const float X1 = D == 2 ? agg_wrap(mj[1] - miy) : 0.0f;
    float power;
    if (D == 1) {
        power = (float)(-0.5 * (double)con[0] * (double)X0 * (double)X0);
    } else {
        const float a = con[0] * X0 * X0 + con[2] * X1 * X1;
        const float b = con[1] * X0 * X1;
        power = (float)(-0.5 * (double)a - (double)b);
    }
    X_out[0] = X0 * inv_r;
    if (D == 2) X_out[1] = X1 * inv_r;
    if (power > 0.0f) {
        *idx_out = -1;
        *dens_out = 0.0f;
        return 0.0f;
    }
    const float dn = expf(power);
    *idx_out = j;
    *dens_out = dn;
    return dn;
}

// LDS hand-off between the lanes of one wave.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Ascending bitonic sort of n (a power of two) keys in this wave's LDS region.
__device__ inline void wave_bitonic(uint32_t *s, int n, int lane) {
    for (int k = 2; k <= n; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            const int lj = __builtin_ctz(jj);
            for (int t = lane; t < (n >> 1); t += kWave) {
                const int i = ((t >> lj) << (lj + 1)) | (t & (jj - 1)), l = i + jj;
                const uint32_t a = s[i], b = s[l];
                const bool up = (i & k) == 0;
                if ((a > b) == up) {
                    s[i] = b;
                    s[l] = a;
                }
            }
            wave_sync_lds();
        }
}

// The same ascending bitonic network with the keys in registers: element e = lane * R + r
// (R = n / 64 consecutive keys per lane).  Partners closer than R are in the lane's own
// registers; farther ones are lane ^ (j / R), exchanged with one cross-lane permute per
// register.  Two thirds of the 66 stages of n = 2048 stay in registers, and no stage waits on
// LDS banks (the LDS network was ~40 % of k_agg_fill).
// One stage (K, J compile-time) of the network.
template <int R, int K, int J>
__device__ __forceinline__ void reg_bitonic_stage(uint32_t (&v)[R], int lane) {
    const int e0 = lane * R;
    if constexpr (J < R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r & J) continue;
            const bool asc = ((e0 + r) & K) == 0;
            const uint32_t a = v[r], b = v[r | J];
            const bool sw = (a > b) == asc;
            v[r] = sw ? b : a;
            v[r | J] = sw ? a : b;
        }
    } else {
        constexpr int LX = J / R;
        const bool keep_min = ((lane & LX) == 0) == ((e0 & K) == 0);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v[r], LX);
            v[r] = keep_min ? min(v[r], o) : max(v[r], o);
        }
    }
    if constexpr (J > 1) reg_bitonic_stage<R, K, J / 2>(v, lane);
}

template <int R, int K = 2>
__device__ __forceinline__ void reg_bitonic(uint32_t (&v)[R], int lane) {
    reg_bitonic_stage<R, K, K / 2>(v, lane);
    if constexpr (K < R * kWave) reg_bitonic<R, K * 2>(v, lane);
}

template <int R>
__device__ __forceinline__ void reg_bitonic_lds(uint32_t *s, int lane) {
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = s[lane * R + r];
    reg_bitonic<R>(v, lane);
    wave_sync_lds();
#pragma unroll
    for (int r = 0; r < R; ++r) s[lane * R + r] = v[r];
    wave_sync_lds();
}

// Ascending sort of s[0, np2) (np2 a power of two, 64 <= np2 <= kAggNMax) in registers.
__device__ inline void wave_sort_keys(uint32_t *s, int np2, int lane) {
    switch (np2) {
    case 64: reg_bitonic_lds<1>(s, lane); break;
    case 128: reg_bitonic_lds<2>(s, lane); break;
    case 256: reg_bitonic_lds<4>(s, lane); break;
    case 512: reg_bitonic_lds<8>(s, lane); break;
    case 1024: reg_bitonic_lds<16>(s, lane); break;
    default: reg_bitonic_lds<32>(s, lane); break;
    }
}

__device__ __forceinline__ float wave_sum(float v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__global__ __launch_bounds__(kBlock) void k_agg_fill(int P, AggGeom g, const float *__restrict__ means,
                                                     const float *__restrict__ conics,
                                                     const float *__restrict__ radii,
                                                     const float4 *__restrict__ cand,
                                                     const int32_t *__restrict__ cstart,
                                                     const uint32_t *__restrict__ order,
                                                     const int64_t *__restrict__ ranges,
                                                     int64_t *__restrict__ indices, float *__restrict__ dists,
                                                     float *__restrict__ densities,
                                                     float *__restrict__ inv_total, int regsort) {
    __shared__ uint32_t buf[kWavesPerBlock][kAggNMax];
    const int lane = threadIdx.x & (kWave - 1);
    uint32_t *s = buf[threadIdx.x >> 6];
    const int stride = gridDim.x * kWavesPerBlock;
    const int D = g.D, S = D * (D + 1) / 2;
    for (int w = wave_unit_index(P); w < P; w += stride) {
        const int i = (int)order[w];
        const int64_t start = i == 0 ? 0 : ranges[i - 1], end = ranges[i];
        // aggregate_neighbors.cu:73-74 (0.333 and 1.0 / (r + 1e-6) in double)
        const float my_radius = (float)((double)radii[i] * 0.333);
        const float inv_r = (float)(1.0 / ((double)my_radius + 1e-6));
        const float ri = agg_r(radii[i]);
        const float mix = means[(int64_t)i * D], miy = D == 2 ? means[(int64_t)i * 2 + 1] : 0.0f;
        float total = 0.0f;
        int64_t slot = start;
        uint32_t lo = 0;
        while (slot < end) {
            // collect the neighbours with id in [lo, hi), halving the window until they fit
            uint32_t hi = (uint32_t)P;
            int n;
            for (;;) {
                n = 0;
                agg_for_candidates(g, mix, miy, ri, cand, cstart, lane, [&](uint32_t j, bool ok) {
                    const bool take = ok && j >= lo && j < hi;
                    const uint64_t bal = __ballot(take);
                    const int pos = n + (int)__popcll(bal & ((1ull << lane) - 1ull));
                    if (take && pos < kAggNMax) s[pos] = j;
                    n += (int)__popcll(bal);
                });
                if (n <= kAggNMax) break;
                hi = lo + (hi - lo) / 2;
            }
            int np2 = kWave;  // register network: at least one key per lane
            while (np2 < n) np2 <<= 1;
            for (int t = n + lane; t < np2; t += kWave) s[t] = 0xffffffffu;
            wave_sync_lds();
            if (regsort) wave_sort_keys(s, np2, lane);
            else wave_bitonic(s, np2, lane);
            for (int t0 = 0; t0 < n; t0 += kWave) {
                const int t = t0 + lane;
                float dv = 0.0f;
                if (t < n) {
                    const int64_t j = s[t], o = slot + t;
                    dv = agg_slot(D, mix, miy, inv_r, means + j * D, conics + j * S, j, &indices[o], &dists[o * D],
                                  &densities[o]);
                }
                total += wave_sum(dv);  // 64 slots at a time, in slot order
            }
            slot += n;
            lo = hi;
            wave_sync_lds();
        }
        if (lane == 0) inv_total[i] = (float)(1.0 / ((double)total + 1e-6));
    }
}

// --------------------------------------------------------------------- forward / backward
struct AggArgs {
    int P, D, L, K, E;
    const float *features, *transform, *queries, *keys, *freq, *dt;
    const int64_t *indices, *ranges;
    const float *dists, *densities, *inv_total;
    float *weights, *embeddings, *factors;  // forward: written; backward: read
    float *out;                             // forward
    const float *dL;                        // backward
    float *arows;                           // backward scratch: a of every row [P][L]
    float *dfeat, *dq, *dkeys, *dfreq, *ddt;
    const int32_t *order;  // optional row order (spatial, from dgs_agg_preprocess); NULL = 0..P-1
    float *strows;         // transposed backward (dgs_agg_backward_tr): st = transform dL of every row [P][L]
    float4 *ct;            // ... and per slot (c, te, row as int bits, 0) for the per-neighbour sum,
    const int32_t *rstart; // at rstart[row] + (slot - the row's first slot): rows in spatial order
    int expt;              // profiling experiments (DGS_AGG_EXPT): bit 0 skips the scatter, bit 1 the
                           // distance-transform terms -- results are then wrong; 0 in production
};

__device__ __forceinline__ int agg_row(const AggArgs &A, int w) { return A.order ? A.order[w] : w; }

// sin / cos of the reference's double argument frequencies * M_PI * X (aggregate_neighbors.cu
// :181-182 evaluate sin/cos in double and round to float): quadrant reduction in double, then
// float minimax polynomials on |r| <= pi/4 (Cephes sinf/cosf coefficients; < 1 ulp there, so
// within ~2 ulp of the correctly rounded double result).
__device__ __forceinline__ void ref_sincos(float f, float X, float *s, float *c) {
    const double arg = (double)f * M_PI * (double)X;
    if (!(fabs(arg) < 1e6)) {
        *s = (float)sin(arg);
        *c = (float)cos(arg);
        return;
    }
    const double n = rint(arg * M_2_PI);
    double rd = fma(-n, 1.5707963267948966, arg);
    rd = fma(-n, 6.123233995736766e-17, rd);
    const float r = (float)rd, z = r * r;
    const float sr = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z, r, r);
    const float cp = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    const float cr = fmaf(cp * z, z, -0.5f * z) + 1.0f;
    const int q = (int)n & 3;
    const float a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;
    *s = (q & 2) ? -a : a;
    *c = ((q + 1) & 2) ? -b : b;
}

// embedding / factor of one slot (aggregate_neighbors.cu:176-193).
__device__ __forceinline__ void agg_embed(int D, int F, int E, const float *__restrict__ freq,
                                          const float *__restrict__ dt, const float *X, float *emb, float *fac) {
    const int stride = (E - 1) / D;
    float e0 = 0.0f, f0 = 0.0f;
    for (int d = 0; d < D; ++d)
        for (int e = 0; e < F; ++e) {
            float sn, cs;
            ref_sincos(freq[e], X[d], &sn, &cs);
            const int a = d * stride + e * 2;
            e0 += dt[a] * sn;
            e0 += dt[a + 1] * cs;
            f0 += dt[E + a] * sn;
            f0 += dt[E + a + 1] * cs;
        }
    *emb = e0 + dt[E - 1];
    *fac = f0 + dt[2 * E - 1];
}

// Wave sum of y over the lane pairs (l, l ^ 32) / 16-lane row pairs, every lane keeping the sum.
__device__ __forceinline__ float swap_add32(float y) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(y), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap_add16(float y) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int N>
__device__ __forceinline__ void rs_stage(float (&x)[16], int lane, int bit, int ctrl) {
    const bool hi = (lane & bit) != 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float keep = hi ? x[i + N] : x[i];
        const float send = hi ? x[i] : x[i + N];
        x[i] = keep + rs_partner(send, ctrl);
    }
}

// NB per-lane partial sums (consumed) -> lane l holds the wave total of value l % NB.  NB = 64
// is reduce_scatter64; NB = 32 / 16 fold the lane halves (and quarters) first and keep only NB
// registers live.
template <int NB>
__device__ __forceinline__ float reduce_row(float (&acc)[NB], int lane) {
    if constexpr (NB == 64) {
        return reduce_scatter64(acc, lane);
    } else {
        float x[16];
        if constexpr (NB == 32) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float a = swap_add32(acc[i]), b = swap_add32(acc[i + 16]);
                const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
                x[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
            }
        } else {
            static_assert(NB == 16, "NB is 16, 32 or 64");
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = swap_add16(swap_add32(acc[i]));
        }
        rs_stage<8>(x, lane, 8, 0x140);
        rs_stage<4>(x, lane, 4, 0x141);
        rs_stage<2>(x, lane, 2, 0x4e);
        rs_stage<1>(x, lane, 1, 0xb1);
        return x[0];
    }
}

// NB (16, 32 or 64): features per pass; L > 64 takes several passes over the row.
template <int NB>
__global__ __launch_bounds__(kBlock) void k_agg_forward(AggArgs A) {
    __shared__ float arow[kWavesPerBlock][256];
    const int lane = threadIdx.x & (kWave - 1);
    float *ar = arow[threadIdx.x >> 6];
    const int stride = gridDim.x * kWavesPerBlock;
    const int D = A.D, L = A.L, K = A.K, E = A.E, F = (E - 1) / D / 2;
    for (int w = wave_unit_index(A.P); w < A.P; w += stride) {
        const int i = agg_row(A, w);
        const int64_t start = i == 0 ? 0 : A.ranges[i - 1], end = A.ranges[i];
        const float inv = A.inv_total[i];
        const float *q = A.queries + (int64_t)i * K;
        for (int fb = 0; fb == 0 || fb < L; fb += NB) {  // one pass even without features
            float acc[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) acc[t] = 0.0f;
            for (int64_t s = start + lane; s < end; s += kWave) {
                const int64_t idx = A.indices[s];
                if (idx < 0) {
                    if (fb == 0) A.weights[s] = A.embeddings[s] = A.factors[s] = 0.0f;
                    continue;
                }
                const float *key = A.keys + idx * K;
                float weight = 0.0f;
                for (int k = 0; k < K; ++k) weight += q[k] * key[k];
                const float X[2] = {A.dists[s * D], D == 2 ? A.dists[s * D + 1] : 0.0f};
                float emb, fac;
                agg_embed(D, F, E, A.freq, A.dt, X, &emb, &fac);
                if (fb == 0) {
                    A.weights[s] = weight;
                    A.embeddings[s] = emb;
                    A.factors[s] = fac;
                }
                const float dw = inv * A.densities[s] * weight;
                const float dwf = dw * fac, dwe = dw * emb;
                const float *feat = A.features + idx * L + fb;
                if (fb + NB <= L) {
#pragma unroll
                    for (int t = 0; t < NB; ++t) acc[t] += dwe + dwf * feat[t];
                } else {
#pragma unroll
                    for (int t = 0; t < NB; ++t)
                        if (fb + t < L) acc[t] += dwe + dwf * feat[t];
                }
            }
            const float r = reduce_row<NB>(acc, lane);
            if (lane < NB && fb + lane < L) ar[fb + lane] = r;
        }
        wave_sync_lds();
        for (int k = lane; k < L; k += kWave) {
            float o = 0.0f;
            for (int j = 0; j < L; ++j) o += A.transform[j * L + k] * ar[j];
            A.out[(int64_t)i * L + k] = o;
        }
        wave_sync_lds();
    }
}

// Dynamic LDS per wave (kAggBwdLds): NV x 64 per-lane partials of the shared arrays (ddt[2E],
// dfreq[F]), st[256], and the batch's (neighbour, dcw * fac, te) for the scatter.
constexpr int kAggStash = 256 + 3 * kWave;
__host__ __device__ constexpr int agg_bwd_lds_floats(int NV) { return NV * kWave + kAggStash; }

template <int NB>
__global__ __launch_bounds__(kBlock) void k_agg_backward(AggArgs A) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x >> 6;
    const int D = A.D, L = A.L, K = A.K, E = A.E, F = (E - 1) / D / 2, dstride = (E - 1) / D;
    const int NV = 2 * E + F;
    float *base = lds + w * agg_bwd_lds_floats(NV);
    float *part = base + lane;  // value v of this lane: part[v * 64]
    float *st = base + NV * kWave;
    int *sm = reinterpret_cast<int *>(st + 256);
    float *sc = st + 256 + kWave, *ste = st + 256 + 2 * kWave;
    for (int v = 0; v < NV; ++v) part[v * kWave] = 0.0f;
    const int stride = gridDim.x * kWavesPerBlock;
    const int LK = max(L, K);
    // scatter layout: G = L + K lanes per neighbour row (dfeat row, then dkeys row), spp rows
    // per atomic instruction, so one instruction covers whole rows instead of 64 scattered words
    const int G = L + K, spp = G <= kWave ? kWave / max(G, 1) : 1;
    const int sub = G <= kWave ? lane / max(G, 1) : 0;
    for (int wr = wave_unit_index(A.P); wr < A.P; wr += stride) {
        const int i = agg_row(A, wr);
        const int64_t start = i == 0 ? 0 : A.ranges[i - 1], end = A.ranges[i];
        const float inv = A.inv_total[i];
        const float *q = A.queries + (int64_t)i * K, *g = A.dL + (int64_t)i * L;
        // summed_transform (aggregate_neighbors.cu:257-262)
        for (int j = lane; j < L; j += kWave) {
            float v = 0.0f;
            for (int k = 0; k < L; ++k) v += A.transform[j * L + k] * g[k];
            st[j] = v;
        }
        wave_sync_lds();
        float S1 = 0.0f;
        for (int j = 0; j < L; ++j) S1 += st[j];
        for (int fb = 0; fb == 0 || fb < LK; fb += NB) {
            float acc_a[NB], acc_q[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) acc_a[t] = acc_q[t] = 0.0f;
            for (int64_t s0 = start; s0 < end; s0 += kWave) {
                const int64_t s = s0 + lane;
                const int64_t idx = s < end ? A.indices[s] : -1;
                float c = 0.0f, te = 0.0f;
                if (idx >= 0) {
                    const float *feat = A.features + idx * L, *key = A.keys + idx * K;
                    const float dc = A.densities[s] * inv;
                    const float dcw = dc * A.weights[s];
                    const float emb = A.embeddings[s], fac = A.factors[s];
                    float S2 = 0.0f;
                    for (int j = 0; j < L; ++j) S2 += st[j] * feat[j];
                    te = (dc * emb) * S1 + (dc * fac) * S2;  // sum_j te_j
                    c = dcw * fac;
                    const float dwe = dcw * emb, dwf = dcw * fac;
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        if (fb + t < L) acc_a[t] += dwe + dwf * feat[fb + t];
                        if (fb + t < K) acc_q[t] += key[fb + t] * te;
                    }
                    if (fb == 0 && !(A.expt & 2)) {
                        // distance-transform and frequency terms (aggregate_neighbors.cu:270-295)
                        const float t1 = dcw * S1, t2 = dcw * S2;
                        for (int d = 0; d < D; ++d) {
                            const float Xd = A.dists[s * D + d];
                            const double px = M_PI * (double)Xd;
                            for (int e = 0; e < F; ++e) {
                                float sn, cs;
                                ref_sincos(A.freq[e], Xd, &sn, &cs);
                                const int a = d * dstride + e * 2;
                                part[a * kWave] += t1 * sn;
                                part[(a + 1) * kWave] += t1 * cs;
                                part[(E + a) * kWave] += t2 * sn;
                                part[(E + a + 1) * kWave] += t2 * cs;
                                const float f0 =
                                    (float)((double)cs * px * ((double)A.dt[a] * t1 + (double)A.dt[E + a] * t2));
                                const float f1 = (float)((double)-sn * px *
                                                         ((double)A.dt[a + 1] * t1 + (double)A.dt[E + a + 1] * t2));
                                part[(2 * E + e) * kWave] += f0 + f1;
                            }
                        }
                        part[(E - 1) * kWave] += t1;
                        part[(2 * E - 1) * kWave] += t2;
                    }
                }
                if (fb != 0 || (A.expt & 1)) continue;
                // neighbour gradients (aggregate_neighbors.cu:296-319):
                //   dfeat[idx][j] += dcw fac st[j],  dkeys[idx][k] += q[k] te
                sm[lane] = (int)idx;
                sc[lane] = c;
                ste[lane] = te;
                wave_sync_lds();
                const int nb = (int)min<int64_t>(kWave, end - s0);
                for (int b = 0; b < nb; b += spp) {
                    const int sl = b + sub;
                    const int m = (sub < spp && sl < nb) ? sm[sl] : -1;
                    if (m >= 0) {
                        for (int t = G <= kWave ? lane - sub * G : lane; t < G; t += kWave) {
                            if (t < L) atomicAdd(&A.dfeat[(int64_t)m * L + t], sc[sl] * st[t]);
                            else atomicAdd(&A.dkeys[(int64_t)m * K + (t - L)], ste[sl] * q[t - L]);
                        }
                    }
                }
                wave_sync_lds();
            }
            const float ra = reduce_row<NB>(acc_a, lane);
            if (lane < NB && fb + lane < L) A.arows[(int64_t)i * L + fb + lane] = ra;
            const float rq = reduce_row<NB>(acc_q, lane);
            if (lane < NB && fb + lane < K) A.dq[(int64_t)i * K + fb + lane] = rq;
        }
        wave_sync_lds();
    }
    for (int v = 0; v < NV; ++v) {
        const float x = wave_sum(part[v * kWave]);
        if (lane == 0) atomicAdd(v < 2 * E ? &A.ddt[v] : &A.dfreq[v - 2 * E], x);
    }
}

// ---------------------------------------------------------- staged fast path (L, K <= 64)
// In the lane-per-slot form every lane gathers its own neighbour row, so one load instruction
// touches 64 cache lines and the vector memory pipe (not HBM, not the ALUs) bounds the kernels.
// Here a batch's 64 neighbour rows are first copied into LDS with coalesced 16-byte pieces
// (consecutive lanes take consecutive pieces of one row: 4 lanes per 64-byte row at L = 16),
// then each slot lane reads its row from LDS.
struct AggStage {
    int SL, SK;      // LDS row strides (floats) of the staged feature / key rows
    int vf, vk;      // rows may be moved in 16-byte pieces (width % 4 == 0, base 16-byte aligned)
    int per_wave;    // LDS floats per wave
};

// Up to U pieces of a row array per lane per round: all U loads are issued before the first LDS
// write, so a round costs one memory latency (the loop form waited on every load).
template <int U>
__device__ __forceinline__ void stage_round(const float *__restrict__ src, int W, int vec, const int *sm, int npieces,
                                            float *dst, int SW, int lane, int p0) {
    if (vec) {
        const int PW = W >> 2;
        const float inv = 1.0f / (float)max(PW, 1);
        float4 v[U];
        int off[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int p = p0 + u * kWave + lane;
            off[u] = -1;
            v[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (p < npieces) {
                const int r = (int)(((float)p + 0.5f) * inv), q = p - r * PW;
                const int m = sm[r];
                if (m >= 0) {
                    v[u] = *reinterpret_cast<const float4 *>(src + (int64_t)m * W + 4 * q);
                    off[u] = r * SW + 4 * q;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (off[u] >= 0) *reinterpret_cast<float4 *>(dst + off[u]) = v[u];
    } else {
        const float inv = 1.0f / (float)max(W, 1);
        float v[4 * U];
        int off[4 * U];
#pragma unroll
        for (int u = 0; u < 4 * U; ++u) {
            const int p = p0 + u * kWave + lane;
            off[u] = -1;
            v[u] = 0.0f;
            if (p < npieces) {
                const int r = (int)(((float)p + 0.5f) * inv), q = p - r * W;
                const int m = sm[r];
                if (m >= 0) {
                    v[u] = src[(int64_t)m * W + q];
                    off[u] = r * SW + q;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4 * U; ++u)
            if (off[u] >= 0) dst[off[u]] = v[u];
    }
}

// Stage the batch's neighbour rows of features and keys (nb rows, sm[r] < 0 skipped).
__device__ __forceinline__ void stage_rows2(const AggArgs &A, const AggStage &G, const int *sm, int nb, float *sf,
                                            float *sk, int lane) {
    const int nf = nb * (G.vf ? A.L >> 2 : A.L), nk = nb * (G.vk ? A.K >> 2 : A.K);
    const int sf_step = (G.vf ? 4 : 16) * kWave, sk_step = (G.vk ? 4 : 16) * kWave;
    for (int pf = 0, pk = 0; pf < nf || pk < nk; pf += sf_step, pk += sk_step) {
        if (pf < nf) stage_round<4>(A.features, A.L, G.vf, sm, nf, sf, G.SL, lane, pf);
        if (pk < nk) stage_round<4>(A.keys, A.K, G.vk, sm, nk, sk, G.SK, lane, pk);
    }
}

__device__ __forceinline__ float dot_row(const float *__restrict__ q, const float *row, int K) {
    float v = 0.0f;
    for (int k = 0; k < K; ++k) v += q[k] * row[k];
    return v;
}
// The same sum, order and roundings for a compile-time length: the LDS row is then read as
// 16-byte pieces (a lane's row at a stride of SK floats; the runtime loop's 4-byte reads at that
// stride were 4-way bank conflicts, PMC SQ_LDS_BANK_CONFLICT).
template <int N>
__device__ __forceinline__ float dot_fixed(const float *__restrict__ q, const float *row) {
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < N; ++k) v += q[k] * row[k];
    return v;
}

// Pipelined staging (L, K <= 16, 16-byte rows: at most 4 pieces of each row array per lane):
// the next batch's pieces are loaded into registers before the current batch's arithmetic
// and written to LDS after it, so the gather latency overlaps the arithmetic (the
// synchronous form left the waves parked on s_waitcnt for ~70 % of their cycles, PMC
// SQ_WAIT_ANY).
struct Pieces {
    float4 f[4], k[4];
};

__device__ __forceinline__ void piece_rq(int p, int PW, int &r, int &q) {
    r = (int)(((float)p + 0.5f) / (float)PW);
    q = p - r * PW;
}

__device__ __forceinline__ void pieces_load(const AggArgs &A, const int *sm, int nb, int lane, Pieces &pc) {
    const int PF = A.L >> 2, PK = A.K >> 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int p = u * kWave + lane;
        int r, q;
        pc.f[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        piece_rq(p, PF, r, q);
        if (r < nb) {
            const int m = sm[r];
            if (m >= 0) pc.f[u] = *reinterpret_cast<const float4 *>(A.features + (int64_t)m * A.L + 4 * q);
        }
        pc.k[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        piece_rq(p, PK, r, q);
        if (r < nb) {
            const int m = sm[r];
            if (m >= 0) pc.k[u] = *reinterpret_cast<const float4 *>(A.keys + (int64_t)m * A.K + 4 * q);
        }
    }
}

__device__ __forceinline__ void pieces_store(const AggArgs &A, const AggStage &G, const Pieces &pc, float *sf,
                                             float *sk, int lane) {
    const int PF = A.L >> 2, PK = A.K >> 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int p = u * kWave + lane;
        int r, q;
        piece_rq(p, PF, r, q);
        if (r < kWave) *reinterpret_cast<float4 *>(sf + r * G.SL + 4 * q) = pc.f[u];
        piece_rq(p, PK, r, q);
        if (r < kWave) *reinterpret_cast<float4 *>(sk + r * G.SK + 4 * q) = pc.k[u];
    }
}

// NB = L rounded up to 16 / 32 / 64; K <= 64.
template <int NB, bool PIPE>
__global__ __launch_bounds__(kBlock) void k_agg_forward_s(AggArgs A, AggStage G) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x & (kWave - 1);
    float *base = lds + (threadIdx.x >> 6) * G.per_wave;
    int *sm = reinterpret_cast<int *>(base);
    float *sf = base + kWave, *sk = sf + kWave * G.SL, *ar = sk + kWave * G.SK;
    const int stride = gridDim.x * kWavesPerBlock;
    const int D = A.D, L = A.L, K = A.K, E = A.E, F = (E - 1) / D / 2;
    for (int w = wave_unit_index(A.P); w < A.P; w += stride) {
        const int i = agg_row(A, w);
        const int64_t start = i == 0 ? 0 : A.ranges[i - 1], end = A.ranges[i];
        const float inv = A.inv_total[i];
        const float *q = A.queries + (int64_t)i * K;
        float acc[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) acc[t] = 0.0f;
        // the streamed per-slot inputs are loaded one batch ahead (their HBM latency then
        // overlaps the current batch's row staging and arithmetic)
        int64_t idx_n = -1;
        float X0_n = 0.0f, X1_n = 0.0f, dn_n = 0.0f;
        auto fetch = [&](int64_t sp) {
            idx_n = -1;
            if (sp < end) {
                idx_n = A.indices[sp];
                X0_n = A.dists[sp * D];
                X1_n = D == 2 ? A.dists[sp * D + 1] : 0.0f;
                dn_n = A.densities[sp];
            }
        };
        // one slot of the batch: weight, embedding, factor and the lane's share of a
        auto slot = [&](int64_t s, int64_t idx, const float *X, float dn) {
            if (idx >= 0) {
                const float weight = K == NB ? dot_fixed<NB>(q, sk + lane * G.SK) : dot_row(q, sk + lane * G.SK, K);
                float emb, fac;
                agg_embed(D, F, E, A.freq, A.dt, X, &emb, &fac);
                A.weights[s] = weight;
                A.embeddings[s] = emb;
                A.factors[s] = fac;
                const float dw = inv * dn * weight;
                const float dwf = dw * fac, dwe = dw * emb;
                const float *feat = sf + lane * G.SL;
                if (L == NB) {
#pragma unroll
                    for (int t = 0; t < NB; ++t) acc[t] += dwe + dwf * feat[t];
                } else {
#pragma unroll
                    for (int t = 0; t < NB; ++t)
                        if (t < L) acc[t] += dwe + dwf * feat[t];
                }
            } else if (s < end) {
                A.weights[s] = A.embeddings[s] = A.factors[s] = 0.0f;
            }
        };
        fetch(start + lane);
        if constexpr (PIPE) {
            Pieces pc;
            int64_t idx = idx_n;
            float X[2] = {X0_n, X1_n}, dn = dn_n;
            sm[lane] = (int)idx;
            wave_sync_lds();
            pieces_load(A, sm, (int)min<int64_t>(kWave, end - start), lane, pc);
            fetch(start + kWave + lane);
            wave_sync_lds();
            pieces_store(A, G, pc, sf, sk, lane);
            wave_sync_lds();
            for (int64_t s0 = start; s0 < end; s0 += kWave) {
                const int64_t s = s0 + lane;
                const bool more = s0 + kWave < end;
                const int64_t idx_x = idx_n;
                const float Xx[2] = {X0_n, X1_n}, dn_x = dn_n;
                if (more) {  // the next batch's rows into registers, its successor's streams
                    sm[lane] = (int)idx_x;
                    wave_sync_lds();
                    pieces_load(A, sm, (int)min<int64_t>(kWave, end - s0 - kWave), lane, pc);
                    fetch(s + 2 * kWave);
                }
                slot(s, idx, X, dn);
                wave_sync_lds();
                if (more) {
                    pieces_store(A, G, pc, sf, sk, lane);
                    wave_sync_lds();
                }
                idx = idx_x;
                X[0] = Xx[0];
                X[1] = Xx[1];
                dn = dn_x;
            }
        } else {
        for (int64_t s0 = start; s0 < end; s0 += kWave) {
            const int64_t s = s0 + lane;
            const int nb = (int)min<int64_t>(kWave, end - s0);
            const int64_t idx = idx_n;
            float X[2] = {X0_n, X1_n};
            const float dn = dn_n;
            fetch(s + kWave);
            sm[lane] = (int)idx;
            wave_sync_lds();
            stage_rows2(A, G, sm, nb, sf, sk, lane);
            wave_sync_lds();
            slot(s, idx, X, dn);
            wave_sync_lds();
        }
        }
        const float r = reduce_row<NB>(acc, lane);
        if (lane < L) ar[lane] = r;
        wave_sync_lds();
        for (int k = lane; k < L; k += kWave) {
            float o = 0.0f;
            for (int j = 0; j < L; ++j) o += A.transform[j * L + k] * ar[j];
            A.out[(int64_t)i * L + k] = o;
        }
        wave_sync_lds();
    }
}

// Backward, L and K <= 64 (NB = max(L, K) rounded up).  Per-wave LDS: the staged rows, the
// batch's (neighbour, dcw * fac, te), st[64], and the shared-array partials: every value is
// first summed over the lane quartet (l, l^16, l^32, l^48) and kept by lanes 0..15 (NV x 16).
// TR (dgs_agg_backward_tr): instead of scattering the neighbours' feature / key gradients with
// float atomics, every slot's two factors (c, te) and its row go to A.ct (16-byte coalesced stores,
// rows laid out in spatial order) and every row's st to A.strows; k_agg_tgather then sums them per
// neighbour.
template <int NB, bool COMBO, bool PIPE, bool TR>
__global__ __launch_bounds__(kBlock) void k_agg_backward_s(AggArgs A, AggStage G) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x & (kWave - 1);
    const int D = A.D, L = A.L, K = A.K, E = A.E, F = (E - 1) / D / 2, dstride = (E - 1) / D;
    const int NV = 2 * E + F;
    float *base = lds + (threadIdx.x >> 6) * G.per_wave;
    int *sm = reinterpret_cast<int *>(base);
    float *sc = base + kWave, *ste = sc + kWave, *st = ste + kWave;
    float *sf = st + kWave, *sk = sf + kWave * G.SL, *s1 = sk + kWave * G.SK, *s2 = s1 + kWave;
    float *sx0 = s2 + kWave, *sx1 = sx0 + kWave, *pbase = sx1 + kWave, *part = pbase + (lane & 15);
    for (int v = lane; v < NV * 16; v += kWave) pbase[v] = 0.0f;
    // distance-transform / frequency terms: lane = (slot group cg, combination cc = (d, e)); each
    // lane keeps its five sums in registers for the wave's lifetime (DF <= 64; otherwise the
    // per-slot `put` reduction below)
    const int DF = D * F, DFe = max(DF, 1);
    constexpr bool combo_path = COMBO;  // host: COMBO == (D * F <= 64)
    const int GR = kWave / DFe, cg = lane / DFe, cc = lane - cg * DFe;
    const bool cact = combo_path && cg < GR;
    const int cd = DF > 0 ? cc / F : 0, ce = DF > 0 ? cc - cd * F : 0, ca = cd * dstride + 2 * ce;
    float cfr = 0.0f, c_a0 = 0.0f, c_a1 = 0.0f, c_b0 = 0.0f, c_b1 = 0.0f;
    if (cact && DF > 0) {
        cfr = A.freq[ce];
        c_a0 = A.dt[ca];
        c_a1 = A.dt[ca + 1];
        c_b0 = A.dt[E + ca];
        c_b1 = A.dt[E + ca + 1];
    }
    float a_ts = 0.0f, a_tc = 0.0f, a_us = 0.0f, a_uc = 0.0f, a_fr = 0.0f, a_t1 = 0.0f, a_t2 = 0.0f;
    const int stride = gridDim.x * kWavesPerBlock;
    const int G2 = L + K, spp = kWave / max(G2, 1), sub = lane / max(G2, 1), tl = lane - sub * G2;
    const bool keep = lane < 16;
    auto put = [&](int v, float x) {  // part[v] += x summed over the lane quartet
        x = swap_add16(swap_add32(x));
        if (keep) part[v * 16] += x;
    };
    for (int wr = wave_unit_index(A.P); wr < A.P; wr += stride) {
        const int i = agg_row(A, wr);
        const int64_t start = i == 0 ? 0 : A.ranges[i - 1], end = A.ranges[i];
        const float inv = A.inv_total[i];
        const float *q = A.queries + (int64_t)i * K, *g = A.dL + (int64_t)i * L;
        // summed_transform (aggregate_neighbors.cu:257-262)
        if (lane < L) {
            float v = 0.0f;
            for (int k = 0; k < L; ++k) v += A.transform[lane * L + k] * g[k];
            st[lane] = v;
            if constexpr (TR) A.strows[(int64_t)i * L + lane] = v;
        }
        // this lane's factor in the scatter: st[t] for a feature lane, q[t - L] for a key lane
        wave_sync_lds();
        const float coef = (sub < spp && tl < G2) ? (tl < L ? st[tl] : q[tl - L]) : 0.0f;
        float S1 = 0.0f;
        for (int j = 0; j < L; ++j) S1 += st[j];
        float acc_a[NB], acc_q[NB];
#pragma unroll
        for (int t = 0; t < NB; ++t) acc_a[t] = acc_q[t] = 0.0f;
        int64_t idx_n = -1;  // streamed per-slot inputs, one batch ahead (see the forward)
        float dn_n = 0.0f, wt_n = 0.0f, emb_n = 0.0f, fac_n = 0.0f, X0_n = 0.0f, X1_n = 0.0f;
        auto fetch = [&](int64_t sp) {
            idx_n = -1;
            if (sp < end) {
                idx_n = A.indices[sp];
                dn_n = A.densities[sp];
                wt_n = A.weights[sp];
                emb_n = A.embeddings[sp];
                fac_n = A.factors[sp];
                X0_n = A.dists[sp * D];
                X1_n = D == 2 ? A.dists[sp * D + 1] : 0.0f;
            }
        };
        fetch(start + lane);
        Pieces pc;  // PIPE: the next batch's row pieces, loaded during this batch's scatter
        int *snext = reinterpret_cast<int *>(sx0);
        if constexpr (PIPE) {
            snext[lane] = (int)idx_n;
            wave_sync_lds();
            pieces_load(A, snext, (int)min<int64_t>(kWave, end - start), lane, pc);
            wave_sync_lds();
            pieces_store(A, G, pc, sf, sk, lane);
            wave_sync_lds();
        }
        for (int64_t s0 = start; s0 < end; s0 += kWave) {
            const int64_t s = s0 + lane;
            const int nb = (int)min<int64_t>(kWave, end - s0);
            const int64_t idx = idx_n;
            const float dn = dn_n, wt = wt_n, emb = emb_n, fac = fac_n;
            const float Xs[2] = {X0_n, X1_n};
            fetch(s + kWave);
            sm[lane] = (int)idx;
            wave_sync_lds();
            if constexpr (!PIPE) {
                stage_rows2(A, G, sm, nb, sf, sk, lane);
                wave_sync_lds();
            }
            const bool more = PIPE && s0 + kWave < end;
            float c = 0.0f, te = 0.0f, t1 = 0.0f, t2 = 0.0f;
            if (idx >= 0) {
                const float *feat = sf + lane * G.SL, *key = sk + lane * G.SK;
                const float dc = dn * inv;
                const float dcw = dc * wt;
                float S2 = 0.0f;
                if (L == NB) {  // (16-byte LDS reads of the lane's row: see dot_fixed)
#pragma unroll
                    for (int j = 0; j < NB; ++j) S2 += st[j] * feat[j];
                } else {
                    for (int j = 0; j < L; ++j) S2 += st[j] * feat[j];
                }
                te = (dc * emb) * S1 + (dc * fac) * S2;  // sum_j te_j
                c = dcw * fac;
                const float dwe = dcw * emb, dwf = dcw * fac;
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    if (t < L) acc_a[t] += dwe + dwf * feat[t];
                    if (t < K) acc_q[t] += key[t] * te;
                }
                t1 = dcw * S1;
                t2 = dcw * S2;
            }
            // distance-transform and frequency terms (aggregate_neighbors.cu:270-295)
            if constexpr (COMBO) {
              if (!(A.expt & 2)) {
                s1[lane] = t1;
                s2[lane] = t2;
                sx0[lane] = Xs[0];
                sx1[lane] = Xs[1];
                wave_sync_lds();
                if (cact) {
                    for (int sl = cg; sl < nb; sl += GR) {
                        const float u1 = s1[sl], u2 = s2[sl];
                        if (cc == 0) {
                            a_t1 += u1;
                            a_t2 += u2;
                        }
                        if (DF > 0) {
                            const float Xd = cd ? sx1[sl] : sx0[sl];
                            float sn, cs;
                            ref_sincos(cfr, Xd, &sn, &cs);
                            a_ts += u1 * sn;
                            a_tc += u1 * cs;
                            a_us += u2 * sn;
                            a_uc += u2 * cs;
                            const double px = M_PI * (double)Xd;
                            const float f0 = (float)((double)cs * px * ((double)c_a0 * u1 + (double)c_b0 * u2));
                            const float f1 = (float)((double)-sn * px * ((double)c_a1 * u1 + (double)c_b1 * u2));
                            a_fr += f0 + f1;
                        }
                    }
                }
              }
            } else if (!(A.expt & 2)) {
                for (int d = 0; d < D; ++d) {
                    const float Xd = idx >= 0 ? Xs[d] : 0.0f;
                    const double px = M_PI * (double)Xd;
                    for (int e = 0; e < F; ++e) {
                        float sn = 0.0f, cs = 0.0f;
                        if (idx >= 0) ref_sincos(A.freq[e], Xd, &sn, &cs);
                        const int a = d * dstride + e * 2;
                        put(a, t1 * sn);
                        put(a + 1, t1 * cs);
                        put(E + a, t2 * sn);
                        put(E + a + 1, t2 * cs);
                        const float f0 = (float)((double)cs * px * ((double)A.dt[a] * t1 + (double)A.dt[E + a] * t2));
                        const float f1 =
                            (float)((double)-sn * px * ((double)A.dt[a + 1] * t1 + (double)A.dt[E + a + 1] * t2));
                        put(2 * E + e, f0 + f1);
                    }
                }
                put(E - 1, t1);
                put(2 * E - 1, t2);
            }
            if (more) {  // issue the next batch's row loads; they land during the scatter
                wave_sync_lds();
                snext[lane] = (int)idx_n;
                wave_sync_lds();
                pieces_load(A, snext, (int)min<int64_t>(kWave, end - s0 - kWave), lane, pc);
            }
            // neighbour gradients (aggregate_neighbors.cu:296-319), a whole neighbour row
            // (dfeat row, then dkeys row) per G2 lanes of one atomic instruction
            if constexpr (TR) {
                if (s < end) A.ct[A.rstart[i] + (s - start)] = make_float4(c, te, __int_as_float(i), 0.0f);
            } else if (!(A.expt & 1)) {
                sc[lane] = c;
                ste[lane] = te;
                wave_sync_lds();
                if (spp > 0) {
                    for (int b = 0; b < nb; b += spp) {
                        const int sl = b + sub;
                        const int m = (sub < spp && sl < nb) ? sm[sl] : -1;
                        if (m >= 0) {
                            if (tl < L) atomicAdd(&A.dfeat[(int64_t)m * L + tl], sc[sl] * coef);
                            else atomicAdd(&A.dkeys[(int64_t)m * K + (tl - L)], ste[sl] * coef);
                        }
                    }
                } else {  // L + K > 64: one neighbour row per pass
                    for (int sl = 0; sl < nb; ++sl) {
                        const int m = sm[sl];
                        if (m < 0) continue;
                        for (int t = lane; t < G2; t += kWave) {
                            if (t < L) atomicAdd(&A.dfeat[(int64_t)m * L + t], sc[sl] * st[t]);
                            else atomicAdd(&A.dkeys[(int64_t)m * K + (t - L)], ste[sl] * q[t - L]);
                        }
                    }
                }
            }
            wave_sync_lds();
            if (more) {
                pieces_store(A, G, pc, sf, sk, lane);
                wave_sync_lds();
            }
        }
        const float ra = reduce_row<NB>(acc_a, lane);
        if (lane < L) A.arows[(int64_t)i * L + lane] = ra;
        const float rq = reduce_row<NB>(acc_q, lane);
        if (lane < K) A.dq[(int64_t)i * K + lane] = rq;
        wave_sync_lds();
    }
    wave_sync_lds();
    if constexpr (COMBO) {
        float *cp = pbase;  // 7 x 64 per-lane sums (the put area is unused on this path)
        const float vals[7] = {a_ts, a_tc, a_us, a_uc, a_fr, a_t1, a_t2};
#pragma unroll
        for (int v = 0; v < 7; ++v) cp[v * kWave + lane] = vals[v];
        wave_sync_lds();
        if (lane < DFe) {
            float sum[7];
#pragma unroll
            for (int v = 0; v < 7; ++v) {
                sum[v] = 0.0f;
                for (int g2 = 0; g2 < GR; ++g2) sum[v] += cp[v * kWave + g2 * DFe + lane];
            }
            if (DF > 0) {
                atomicAdd(&A.ddt[ca], sum[0]);
                atomicAdd(&A.ddt[ca + 1], sum[1]);
                atomicAdd(&A.ddt[E + ca], sum[2]);
                atomicAdd(&A.ddt[E + ca + 1], sum[3]);
                atomicAdd(&A.dfreq[ce], sum[4]);
            }
            if (lane == 0) {
                atomicAdd(&A.ddt[E - 1], sum[5]);
                atomicAdd(&A.ddt[2 * E - 1], sum[6]);
            }
        }
    } else {
        for (int v = lane; v < NV; v += kWave) {
            float x = 0.0f;
            for (int l = 0; l < 16; ++l) x += part[v * 16 + l - (lane & 15)];
            atomicAdd(v < 2 * E ? &A.ddt[v] : &A.dfreq[v - 2 * E], x);
        }
    }
}

// dL_dtransform = A^T dL over the rows' a (aggregate_neighbors.cu:301-304, summed over slots).
__global__ __launch_bounds__(kBlock) void k_agg_dtrans(int P, int L, const float *__restrict__ arows,
                                                       const float *__restrict__ dL, float *__restrict__ dtrans) {
    const int64_t per = ((int64_t)P + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * per, r1 = min<int64_t>(P, r0 + per);
    if (r0 >= r1) return;
    for (int e = threadIdx.x; e < L * L; e += blockDim.x) {
        const int j = e / L, k = e - j * L;
        float acc = 0.0f;
        for (int64_t i = r0; i < r1; ++i) acc += arows[i * L + j] * dL[i * L + k];
        atomicAdd(&dtrans[e], acc);
    }
}

// Transposition keys, one wave per row (spatial order): slot s of row i names neighbour
// j = indices[s] (key P for index -1: sorted last, in no row's range); its value is the slot's
// position in the spatial-order record array, rstart[i] + (s - the row's first slot).  The
// records of neighbouring rows are then near each other, and the per-neighbour sum, which visits
// rows in spatial order, reads them from a moving window that stays in the last-level cache.
__global__ __launch_bounds__(kBlock) void k_agg_tkeys(int P, const int64_t *__restrict__ indices,
                                                      const int64_t *__restrict__ ranges,
                                                      const int32_t *__restrict__ order,
                                                      const int32_t *__restrict__ rstart, uint32_t *__restrict__ keys,
                                                      uint32_t *__restrict__ vals) {
    const int lane = threadIdx.x & (kWave - 1);
    const int stride = gridDim.x * kWavesPerBlock;
    for (int w = wave_unit_index(P); w < P; w += stride) {
        const int i = order ? order[w] : w;
        const int64_t start = i == 0 ? 0 : ranges[i - 1], end = ranges[i];
        const uint32_t r0 = (uint32_t)rstart[i];
        for (int64_t s = start + lane; s < end; s += kWave) {
            const int64_t j = indices[s];
            keys[s] = (j >= 0 && j < P) ? (uint32_t)j : (uint32_t)P;
            vals[s] = r0 + (uint32_t)(s - start);
        }
    }
}

// Row lengths in spatial order (the scan of these gives the rows' record offsets).
__global__ void k_agg_rowlen(int P, const int64_t *__restrict__ ranges, const int32_t *__restrict__ order,
                             int32_t *__restrict__ len) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= P) return;
    const int i = order ? order[w] : w;
    len[w] = (int32_t)(ranges[i] - (i == 0 ? 0 : ranges[i - 1]));
}

__global__ void k_agg_rowstart(int P, const int32_t *__restrict__ excl, const int32_t *__restrict__ order,
                               int32_t *__restrict__ rstart) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= P) return;
    rstart[order ? order[w] : w] = excl[w];
}

// tstart[j] = first sorted position whose key is >= j, j in [0, P] (int32: length < 2^31).
__global__ void k_agg_tstart(int P, int64_t n, const uint32_t *__restrict__ keys, int32_t *__restrict__ tstart) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j > P) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < (uint32_t)j) lo = mid + 1;
        else hi = mid;
    }
    tstart[j] = (int32_t)lo;
}

// Per-neighbour sum of the feature / key gradients (the transposed form of
// aggregate_neighbors.cu:303 and 315): for row j, over its incoming slots (i -> j) in slot order,
//   dL/dfeatures[j] = sum c * st_i,   dL/dkeys[j] = sum te * q_i
// (c = dcw * factor, te = sum over the features of summed_transform * embedded, both from the slot's
// row pass).  One wave per row (spatial order: the rows i of neighbouring j share L2).  A batch's 64
// slot records sit in LDS; GR lanes per slot (L + K <= GR: feature lanes, then key lanes), 64 / GR
// slots per step, gather the slot's st_i / q_i row pieces (one 64-byte segment per 16 lanes).  The
// batch pipeline: this batch's row loads are issued first, then the next batch's record (its slot
// id came one batch earlier) and the slot id of the batch after, so the row loads' waits never wait
// for the random record loads (vector-memory counters retire in issue order).  No atomics: every
// gradient row is written once, in a fixed order.
template <int GR>
__global__ __launch_bounds__(kBlock) void k_agg_tgather(int P, int L, int K, const int32_t *__restrict__ tstart,
                                                        const uint32_t *__restrict__ tslot,
                                                        const float4 *__restrict__ ct,
                                                        const float *__restrict__ strows,
                                                        const float *__restrict__ queries,
                                                        const int32_t *__restrict__ order, float *__restrict__ dfeat,
                                                        float *__restrict__ dkeys) {
    constexpr int SPP = kWave / GR, NS = kWave / SPP;  // steps per full batch
    constexpr int CH = NS < 16 ? NS : 16, NCH = NS / CH;  // steps per chunk (registers), chunks
    __shared__ float4 srec[kWavesPerBlock][2][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    float4 (*rec)[kWave] = srec[threadIdx.x >> 6];
    const int sub = lane / GR, t = lane - sub * GR;
    const bool fl = t < L, kl = !fl && t < L + K;
    const float *base = fl ? strows + t : queries + (t - L);
    const int rs = fl ? L : K;
    const int stride = gridDim.x * kWavesPerBlock;
    for (int w = wave_unit_index(P); w < P; w += stride) {
        const int j = order ? order[w] : w;
        const int kb = tstart[j], ke = tstart[j + 1];
        float acc = 0.0f;
        // batch 0's record, batch 1's slot id
        if (kb + lane < ke) rec[0][lane] = ct[tslot[kb + lane]];
        uint32_t sid = (kb + kWave + lane < ke) ? tslot[kb + kWave + lane] : 0u;
        wave_sync_lds();
        int cur = 0;
        for (int k0 = kb; k0 < ke; k0 += kWave) {
            const int nb = min(kWave, ke - k0);
            const bool more = k0 + kWave + lane < ke;
            float4 nrec = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
            for (int ch = 0; ch < NCH; ++ch) {
                if (ch * CH * SPP >= nb) break;
                float2 e[CH];
                float v[CH];
#pragma unroll
                for (int u = 0; u < CH; ++u) {
                    const float4 r = rec[cur][min((ch * CH + u) * SPP + sub, nb - 1)];
                    e[u] = make_float2(fl ? r.x : r.y, r.z);
                }
#pragma unroll
                for (int u = 0; u < CH; ++u) v[u] = (fl || kl) ? base[(int64_t)__float_as_int(e[u].y) * rs] : 0.0f;
                if (ch == NCH - 1 || (ch + 1) * CH * SPP >= nb) {
                    // the next batch's record and the slot id of the batch after, issued after
                    // this batch's last row loads: their waits never wait for these
                    if (more) nrec = ct[sid];
                    sid = (k0 + 2 * kWave + lane < ke) ? tslot[k0 + 2 * kWave + lane] : 0u;
                }
#pragma unroll
                for (int u = 0; u < CH; ++u)
                    if ((ch * CH + u) * SPP + sub < nb) acc = fmaf(e[u].x, v[u], acc);
            }
            if (more) rec[cur ^ 1][lane] = nrec;
            wave_sync_lds();
            cur ^= 1;
        }
        if constexpr (SPP >= 4) acc += __shfl_xor(acc, 16);
        if constexpr (SPP >= 2) acc += __shfl_xor(acc, 32);
        if (sub == 0) {
            if (fl) dfeat[(int64_t)j * L + t] = acc;
            else if (kl) dkeys[(int64_t)j * K + (t - L)] = acc;
        }
    }
}

}  // namespace dgs

using namespace dgs;

static unsigned agg_elem_blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + kBlock - 1) / kBlock); }
static unsigned agg_row_blocks(int P) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((P + kWavesPerBlock - 1) / kWavesPerBlock, 1 << 20));
}

extern "C" int dgs_agg_preprocess(int P, int D, const float *means, const float *conics, const float *radii,
                                  int64_t *ranges, float *inv_total, int32_t *row_order, dgs_alloc_fn alloc,
                                  void *alloc_ctx, int64_t *length, dgs_stream_t stream, int debug) {
    if (D != 1 && D != 2) return fail(DGS_ERR_ARG, "aggregate: only D = 1 or D = 2 is supported");
    if (P < 0 || !alloc || !length) return fail(DGS_ERR_ARG, "dgs_agg_preprocess: bad arguments");
    *length = 0;
    if (P == 0) return DGS_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    auto scratch = [&](size_t n) { return alloc(alloc_ctx, DGS_BUF_SCRATCH, std::max<size_t>(n, 16)); };
    constexpr size_t kStatWords = (size_t)kAggStatCopies * kAggStatStride;
    uint32_t *stats = static_cast<uint32_t *>(scratch(4 * kStatWords));
    if (!stats) return fail(DGS_ERR_ALLOC, "aggregate: scratch allocation failed");
    static const std::vector<uint32_t> init = [] {
        std::vector<uint32_t> v(kStatWords, 0u);
        for (int q = 0; q < kAggStatCopies; ++q) v[q * kAggStatStride + 1] = v[q * kAggStatStride + 2] = 0xffffffffu;
        return v;
    }();
    DGS_TRY_HIP(hipMemcpyAsync(stats, init.data(), 4 * kStatWords, hipMemcpyHostToDevice, s));
    k_agg_prep<<<agg_elem_blocks(P), kBlock, 0, s>>>(P, D, means, radii, stats);
    DGS_LAUNCH_CHECK(s, debug);
    std::vector<uint32_t> hs(kStatWords);
    DGS_TRY_HIP(hipMemcpyAsync(hs.data(), stats, 4 * kStatWords, hipMemcpyDeviceToHost, s));
    DGS_TRY_HIP(hipStreamSynchronize(s));
    uint32_t h[5] = {0u, 0xffffffffu, 0xffffffffu, 0u, 0u};
    for (int q = 0; q < kAggStatCopies; ++q) {
        const uint32_t *c = &hs[(size_t)q * kAggStatStride];
        h[0] = std::max(h[0], c[0]);
        for (int d = 0; d < 2; ++d) {
            h[1 + d] = std::min(h[1 + d], c[1 + d]);
            h[3 + d] = std::max(h[3 + d], c[3 + d]);
        }
    }

    AggGeom g;
    g.D = D;
    const bool any = h[0] != 0;
    g.rmax = any ? o2f(h[0]) : 0.0f;
    for (int d = 0; d < 2; ++d) {
        g.lo[d] = (any && d < D) ? (double)o2f(h[1 + d]) : 0.0;
        g.hi[d] = (any && d < D) ? (double)o2f(h[3 + d]) : 0.0;
    }
    // cell >= 2 rmax (a row's direct window spans at most three cells); at most kAggMaxCells
    double cell = std::max(2.0 * (double)g.rmax, 1e-6);
    for (;;) {
        int64_t tot = 1;
        for (int d = 0; d < 2; ++d) {
            g.nc[d] = d < D ? (int)std::min<double>((g.hi[d] - g.lo[d]) / cell + 1.0, 1 << 24) : 1;
            tot *= g.nc[d];
        }
        if (tot <= kAggMaxCells) break;
        cell *= 2.0;
    }
    g.cs = cell;
    const int ncells = g.nc[0] * g.nc[1];

    uint32_t *keys = static_cast<uint32_t *>(scratch(4 * (size_t)P));
    uint32_t *keys_s = static_cast<uint32_t *>(scratch(4 * (size_t)P));
    uint32_t *ids = static_cast<uint32_t *>(scratch(4 * (size_t)P));
    uint32_t *ids_s = static_cast<uint32_t *>(scratch(4 * (size_t)P));
    float4 *cand = static_cast<float4 *>(scratch(16 * (size_t)P));
    int32_t *cstart = static_cast<int32_t *>(scratch(4 * ((size_t)ncells + 1)));
    int64_t *counts = static_cast<int64_t *>(scratch(8 * (size_t)P));
    if (!keys || !keys_s || !ids || !ids_s || !cand || !cstart || !counts)
        return fail(DGS_ERR_ALLOC, "aggregate: scratch allocation failed");
    size_t tsort = 0, tscan = 0;
    int bits = 1;
    while (bits < 32 && (1u << bits) <= (uint32_t)ncells) ++bits;
    DGS_TRY_HIP(onesweep_pairs<uint32_t>(nullptr, tsort, keys, keys_s, ids, ids_s, (size_t)P, 0u, (unsigned)bits, s));
    tscan = scan_scratch_bytes<int64_t>(P);
    size_t tb = std::max(tsort, tscan);
    void *tmp = scratch(tb);
    if (!tmp) return fail(DGS_ERR_ALLOC, "aggregate: scratch allocation failed");

    k_agg_keys<<<agg_elem_blocks(P), kBlock, 0, s>>>(P, g, means, radii, keys, ids);
    DGS_LAUNCH_CHECK(s, debug);
    DGS_TRY_HIP(onesweep_pairs<uint32_t>(tmp, tb, keys, keys_s, ids, ids_s, (size_t)P, 0u, (unsigned)bits, s));
    k_agg_pack<<<agg_elem_blocks(P), kBlock, 0, s>>>(P, D, ids_s, means, radii, cand);
    DGS_LAUNCH_CHECK(s, debug);
    k_agg_cell_start<<<agg_elem_blocks((int64_t)ncells + 1), kBlock, 0, s>>>(ncells, P, keys_s, cstart);
    DGS_LAUNCH_CHECK(s, debug);
    const unsigned wblocks = agg_row_blocks(P);
    k_agg_count<<<wblocks, kBlock, 0, s>>>(P, g, means, radii, cand, cstart, ids_s, counts);
    DGS_LAUNCH_CHECK(s, debug);
    scan_excl<int64_t>(P, counts, ranges, nullptr, nullptr, static_cast<int64_t *>(tmp), s, true);
    DGS_LAUNCH_CHECK(s, debug);
    int64_t len = 0;
    DGS_TRY_HIP(hipMemcpyAsync(&len, ranges + (P - 1), sizeof(len), hipMemcpyDeviceToHost, s));
    DGS_TRY_HIP(hipStreamSynchronize(s));
    *length = len;
    int64_t *indices =
        static_cast<int64_t *>(alloc(alloc_ctx, DGS_BUF_AGG_INDICES, std::max<size_t>(8 * (size_t)len, 16)));
    float *dists = static_cast<float *>(alloc(alloc_ctx, DGS_BUF_AGG_DISTS, std::max<size_t>(4 * (size_t)len * D, 16)));
    float *dens = static_cast<float *>(alloc(alloc_ctx, DGS_BUF_AGG_DENSITIES, std::max<size_t>(4 * (size_t)len, 16)));
    if (!indices || !dists || !dens) return fail(DGS_ERR_ALLOC, "aggregate: output allocation failed");
    k_agg_fill<<<wblocks, kBlock, 0, s>>>(P, g, means, conics, radii, cand, cstart, ids_s, ranges, indices, dists,
                                          dens, inv_total,
        std::getenv("DGS_AGG_LDSSORT") ? 0 : 1);
    DGS_LAUNCH_CHECK(s, debug);
    if (row_order) DGS_TRY_HIP(hipMemcpyAsync(row_order, ids_s, 4 * (size_t)P, hipMemcpyDeviceToDevice, s));
    return DGS_OK;
}

static int agg_check(int P, int D, int L, int K, int E) {
    if (D != 1 && D != 2) return fail(DGS_ERR_ARG, "aggregate: only D = 1 or D = 2 is supported");
    if (P < 0 || L < 0 || K < 0) return fail(DGS_ERR_ARG, "aggregate: negative size");
    if (E < 1) return fail(DGS_ERR_ARG, "aggregate: distance_transform needs at least 2 entries");
    if (L > 256) return fail(DGS_ERR_ARG, "aggregate: at most 256 features are supported");
    return DGS_OK;
}

static int agg_nb(int m) { return m <= 16 ? 16 : (m <= 32 ? 32 : 64); }

// Staged-row LDS layout: strides padded to a multiple of 4 floats plus 4 (16-byte aligned rows,
// staggered banks).
static AggStage agg_stage(int L, int K, const float *features, const float *keys, int extra) {
    AggStage G;
    G.SL = ((L + 3) & ~3) + 4;
    G.SK = ((K + 3) & ~3) + 4;
    G.vf = (L % 4 == 0) && (reinterpret_cast<uintptr_t>(features) % 16 == 0);
    G.vk = (K % 4 == 0) && (reinterpret_cast<uintptr_t>(keys) % 16 == 0);
    G.per_wave = kWave * (G.SL + G.SK) + extra;
    return G;
}

extern "C" size_t dgs_agg_workspace_size(int P, int L) { return 4 * (size_t)std::max(P, 0) * std::max(L, 0) + 256; }

extern "C" int dgs_agg_forward(int P, int D, int L, int K, int E, const float *features, const float *transform,
                               const float *queries, const float *keys, const float *frequencies,
                               const float *distance_transform, const int64_t *indices, const int64_t *ranges,
                               const float *dists, const float *densities, const float *inv_total,
                               const int32_t *row_order, float *weights, float *embeddings, float *factors, float *out,
                               dgs_stream_t stream, int debug) {
    int rc = agg_check(P, D, L, K, E);
    if (rc) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (P == 0) return DGS_OK;
    AggArgs A{};
    A.P = P, A.D = D, A.L = L, A.K = K, A.E = E;
    A.features = features, A.transform = transform, A.queries = queries, A.keys = keys;
    A.freq = frequencies, A.dt = distance_transform, A.indices = indices, A.ranges = ranges;
    A.dists = dists, A.densities = densities, A.inv_total = inv_total;
    A.weights = weights, A.embeddings = embeddings, A.factors = factors, A.out = out, A.order = row_order;
    const unsigned nb = agg_row_blocks(P);
    if (L <= 64 && K <= 64) {
        const AggStage G = agg_stage(L, K, features, keys, 2 * kWave + 64 /* sm, ar */);
        const size_t lds = sizeof(float) * (size_t)kWavesPerBlock * G.per_wave;
        const bool pipe = L <= 16 && K <= 16 && G.vf && G.vk && !std::getenv("DGS_AGG_NOPIPE");
        switch (agg_nb(std::max(L, 1))) {
        case 16:
            if (pipe) k_agg_forward_s<16, true><<<nb, kBlock, lds, s>>>(A, G);
            else k_agg_forward_s<16, false><<<nb, kBlock, lds, s>>>(A, G);
            break;
        case 32: k_agg_forward_s<32, false><<<nb, kBlock, lds, s>>>(A, G); break;
        default: k_agg_forward_s<64, false><<<nb, kBlock, lds, s>>>(A, G); break;
        }
    } else {
        switch (agg_nb(std::min(std::max(L, 1), 64))) {
        case 16: k_agg_forward<16><<<nb, kBlock, 0, s>>>(A); break;
        case 32: k_agg_forward<32><<<nb, kBlock, 0, s>>>(A); break;
        default: k_agg_forward<64><<<nb, kBlock, 0, s>>>(A); break;
        }
    }
    DGS_LAUNCH_CHECK(s, debug);
    return DGS_OK;
}

static int agg_backward_impl(int P, int D, int L, int K, int E, const float *features, const float *transform,
                             const float *queries, const float *keys, const float *frequencies,
                             const float *distance_transform, const int64_t *indices, const int64_t *ranges,
                             const float *dists, const float *densities, const float *weights,
                             const float *embeddings, const float *factors, const float *inv_total,
                             const int32_t *row_order, const int32_t *tstart, const uint32_t *tslot,
                             const int32_t *rstart, int64_t length, const float *dL_dout, float *dL_dfeatures, float *dL_dtransform, float *dL_dqueries,
                             float *dL_dkeys, float *dL_dfrequencies, float *dL_ddistance_transform,
                             void *workspace, size_t workspace_bytes, dgs_stream_t stream, int debug) {
    int rc = agg_check(P, D, L, K, E);
    if (rc) return rc;
    const bool tr = tstart != nullptr;
    const size_t need = tr ? dgs_agg_workspace_size_tr(P, L, length) : dgs_agg_workspace_size(P, L);
    if (workspace_bytes < need || (!workspace && P > 0))
        return fail(DGS_ERR_ARG, "dgs_agg_backward: workspace smaller than dgs_agg_workspace_size");
    if (tr && (L + K > kWave || !tslot || !rstart || length < 0 || length >= ((int64_t)1 << 31)))
        return fail(DGS_ERR_ARG, "dgs_agg_backward_tr: needs L + K <= 64, tslot, rstart and 0 <= length < 2^31");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int F = (E - 1) / D / 2;
    const int NV = 2 * E + F;
    const bool staged = L <= 64 && K <= 64;
    const AggStage G = agg_stage(L, K, features, keys,
                                 8 * kWave + std::max(NV * 16, 7 * kWave) /* sm sc ste st s1 s2 sx0 sx1, sums */);
    const size_t lds = sizeof(float) * (size_t)kWavesPerBlock * (staged ? G.per_wave : agg_bwd_lds_floats(NV));
    const bool pipe = staged && L <= 16 && K <= 16 && G.vf && G.vk && !std::getenv("DGS_AGG_NOPIPE");
    if (lds > 160 * 1024) return fail(DGS_ERR_ARG, "aggregate backward: distance_transform too long for LDS");
    auto zero = [&](float *p, size_t n) { return n ? hipMemsetAsync(p, 0, sizeof(float) * n, s) : hipSuccess; };
    if (!tr) {  // (the transposed path writes every row of these)
        DGS_TRY_HIP(zero(dL_dfeatures, (size_t)P * L));
        DGS_TRY_HIP(zero(dL_dkeys, (size_t)P * K));
    }
    DGS_TRY_HIP(zero(dL_dtransform, (size_t)L * L));
    DGS_TRY_HIP(zero(dL_dqueries, (size_t)P * K));
    DGS_TRY_HIP(zero(dL_dfrequencies, (size_t)F));
    DGS_TRY_HIP(zero(dL_ddistance_transform, 2 * (size_t)E));
    if (P == 0) return DGS_OK;
    AggArgs A{};
    A.P = P, A.D = D, A.L = L, A.K = K, A.E = E;
    A.features = features, A.transform = transform, A.queries = queries, A.keys = keys;
    A.freq = frequencies, A.dt = distance_transform, A.indices = indices, A.ranges = ranges;
    A.dists = dists, A.densities = densities, A.inv_total = inv_total;
    A.weights = const_cast<float *>(weights), A.embeddings = const_cast<float *>(embeddings);
    A.factors = const_cast<float *>(factors);
    A.dL = dL_dout, A.arows = static_cast<float *>(workspace);
    A.dfeat = dL_dfeatures, A.dq = dL_dqueries, A.dkeys = dL_dkeys, A.dfreq = dL_dfrequencies;
    A.ddt = dL_ddistance_transform, A.order = row_order;
    if (tr) {
        A.strows = A.arows + (size_t)P * L;
        const size_t ct_off = ((sizeof(float) * 2 * (size_t)P * L + 15) / 16) * 16;
        A.ct = reinterpret_cast<float4 *>(static_cast<char *>(workspace) + ct_off);
        A.rstart = rstart;
    }
    if (const char *e = getenv("DGS_AGG_EXPT")) A.expt = atoi(e);
    // few enough waves that each flushes its shared-array partials after many rows
    const unsigned nb = std::min(agg_row_blocks(P), 2048u);
    if (staged) {
        const bool combo = D * F <= kWave;
#define DGS_AGG_BWD(NB_, CO_, PI_)                                                  \
    do {                                                                            \
        if (tr) k_agg_backward_s<NB_, CO_, PI_, true><<<nb, kBlock, lds, s>>>(A, G);  \
        else k_agg_backward_s<NB_, CO_, PI_, false><<<nb, kBlock, lds, s>>>(A, G);    \
    } while (0)
        switch (agg_nb(std::max(std::max(L, K), 1)) * 2 + (combo ? 1 : 0)) {
        case 33:
            if (pipe) DGS_AGG_BWD(16, true, true);
            else DGS_AGG_BWD(16, true, false);
            break;
        case 32: DGS_AGG_BWD(16, false, false); break;
        case 65: DGS_AGG_BWD(32, true, false); break;
        case 64: DGS_AGG_BWD(32, false, false); break;
        case 129: DGS_AGG_BWD(64, true, false); break;
        default: DGS_AGG_BWD(64, false, false); break;
        }
#undef DGS_AGG_BWD
    } else {
        switch (agg_nb(std::min(std::max(std::max(L, K), 1), 64))) {
        case 16: k_agg_backward<16><<<nb, kBlock, lds, s>>>(A); break;
        case 32: k_agg_backward<32><<<nb, kBlock, lds, s>>>(A); break;
        default: k_agg_backward<64><<<nb, kBlock, lds, s>>>(A); break;
        }
    }
    DGS_LAUNCH_CHECK(s, debug);
    if (tr && L + K > 0) {
        const unsigned gb = agg_row_blocks(P);
        const int gr = L + K <= 16 ? 16 : (L + K <= 32 ? 32 : 64);
        if (gr == 16)
            k_agg_tgather<16><<<gb, kBlock, 0, s>>>(P, L, K, tstart, tslot, A.ct, A.strows, queries, row_order,
                                                    dL_dfeatures, dL_dkeys);
        else if (gr == 32)
            k_agg_tgather<32><<<gb, kBlock, 0, s>>>(P, L, K, tstart, tslot, A.ct, A.strows, queries, row_order,
                                                    dL_dfeatures, dL_dkeys);
        else
            k_agg_tgather<64><<<gb, kBlock, 0, s>>>(P, L, K, tstart, tslot, A.ct, A.strows, queries, row_order,
                                                    dL_dfeatures, dL_dkeys);
        DGS_LAUNCH_CHECK(s, debug);
    }
    if (L > 0) {
        const unsigned tb = (unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, ((int64_t)P + 255) / 256));
        k_agg_dtrans<<<tb, kBlock, 0, s>>>(P, L, A.arows, dL_dout, dL_dtransform);
        DGS_LAUNCH_CHECK(s, debug);
    }
    return DGS_OK;
}

extern "C" size_t dgs_agg_workspace_size_tr(int P, int L, int64_t length) {
    const size_t rows = ((sizeof(float) * 2 * (size_t)std::max(P, 0) * std::max(L, 0) + 15) / 16) * 16;
    return rows + 16 * (size_t)std::max<int64_t>(length, 0) + 256;
}

extern "C" int dgs_agg_backward(int P, int D, int L, int K, int E, const float *features, const float *transform,
                                const float *queries, const float *keys, const float *frequencies,
                                const float *distance_transform, const int64_t *indices, const int64_t *ranges,
                                const float *dists, const float *densities, const float *weights,
                                const float *embeddings, const float *factors, const float *inv_total,
                                const int32_t *row_order, const float *dL_dout, float *dL_dfeatures, float *dL_dtransform, float *dL_dqueries,
                                float *dL_dkeys, float *dL_dfrequencies, float *dL_ddistance_transform,
                                void *workspace, size_t workspace_bytes, dgs_stream_t stream, int debug) {
    return agg_backward_impl(P, D, L, K, E, features, transform, queries, keys, frequencies, distance_transform,
                             indices, ranges, dists, densities, weights, embeddings, factors, inv_total, row_order,
                             nullptr, nullptr, nullptr, 0, dL_dout, dL_dfeatures, dL_dtransform, dL_dqueries, dL_dkeys,
                             dL_dfrequencies, dL_ddistance_transform, workspace, workspace_bytes, stream, debug);
}

extern "C" int dgs_agg_backward_tr(int P, int D, int L, int K, int E, const float *features, const float *transform,
                                   const float *queries, const float *keys, const float *frequencies,
                                   const float *distance_transform, const int64_t *indices, const int64_t *ranges,
                                   const float *dists, const float *densities, const float *weights,
                                   const float *embeddings, const float *factors, const float *inv_total,
                                   const int32_t *row_order, const int32_t *tstart, const uint32_t *tslot,
                                   const int32_t *rstart, int64_t length, const float *dL_dout, float *dL_dfeatures, float *dL_dtransform,
                                   float *dL_dqueries, float *dL_dkeys, float *dL_dfrequencies,
                                   float *dL_ddistance_transform, void *workspace, size_t workspace_bytes,
                                   dgs_stream_t stream, int debug) {
    if (!tstart) return fail(DGS_ERR_ARG, "dgs_agg_backward_tr: tstart is NULL");
    return agg_backward_impl(P, D, L, K, E, features, transform, queries, keys, frequencies, distance_transform,
                             indices, ranges, dists, densities, weights, embeddings, factors, inv_total, row_order,
                             tstart, tslot, rstart, length, dL_dout, dL_dfeatures, dL_dtransform, dL_dqueries, dL_dkeys,
                             dL_dfrequencies, dL_ddistance_transform, workspace, workspace_bytes, stream, debug);
}

extern "C" int dgs_agg_transpose(int P, int64_t length, const int64_t *indices, const int64_t *ranges,
                                 const int32_t *row_order, int32_t *tstart, uint32_t *tslot, int32_t *rstart,
                                 dgs_alloc_fn alloc, void *alloc_ctx, dgs_stream_t stream, int debug) {
    if (P < 0 || length < 0 || length >= ((int64_t)1 << 31) || !tstart || !rstart || !ranges ||
        (!tslot && length > 0) || !alloc)
        return fail(DGS_ERR_ARG, "dgs_agg_transpose: bad arguments (length must be < 2^31)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (P == 0) return DGS_OK;
    auto scratch = [&](size_t n) { return alloc(alloc_ctx, DGS_BUF_SCRATCH, std::max<size_t>(n, 16)); };
    int32_t *len = static_cast<int32_t *>(scratch(4 * (size_t)P));
    int32_t *excl = static_cast<int32_t *>(scratch(4 * (size_t)P));
    int32_t *part = static_cast<int32_t *>(scratch(scan_scratch_bytes<int32_t>(P)));
    if (!len || !excl || !part) return fail(DGS_ERR_ALLOC, "dgs_agg_transpose: scratch allocation failed");
    k_agg_rowlen<<<agg_elem_blocks(P), kBlock, 0, s>>>(P, ranges, row_order, len);
    scan_excl<int32_t>(P, len, excl, nullptr, nullptr, part, s);
    k_agg_rowstart<<<agg_elem_blocks(P), kBlock, 0, s>>>(P, excl, row_order, rstart);
    DGS_LAUNCH_CHECK(s, debug);
    if (length == 0) {
        DGS_TRY_HIP(hipMemsetAsync(tstart, 0, sizeof(int32_t) * ((size_t)P + 1), s));
        return DGS_OK;
    }
    uint32_t *keys = static_cast<uint32_t *>(scratch(4 * (size_t)length));
    uint32_t *keys_s = static_cast<uint32_t *>(scratch(4 * (size_t)length));
    uint32_t *vals = static_cast<uint32_t *>(scratch(4 * (size_t)length));
    if (!keys || !keys_s || !vals) return fail(DGS_ERR_ALLOC, "dgs_agg_transpose: scratch allocation failed");
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= (unsigned long long)P) ++bits;
    size_t tb = 0;
    DGS_TRY_HIP(onesweep_pairs<uint32_t>(nullptr, tb, keys, keys_s, vals, tslot, (size_t)length, 0u, (unsigned)bits, s));
    void *tmp = scratch(tb);
    if (!tmp) return fail(DGS_ERR_ALLOC, "dgs_agg_transpose: scratch allocation failed");
    k_agg_tkeys<<<agg_row_blocks(P), kBlock, 0, s>>>(P, indices, ranges, row_order, rstart, keys, vals);
    DGS_LAUNCH_CHECK(s, debug);
    DGS_TRY_HIP(onesweep_pairs<uint32_t>(tmp, tb, keys, keys_s, vals, tslot, (size_t)length, 0u, (unsigned)bits, s));
    DGS_LAUNCH_CHECK(s, debug);
    k_agg_tstart<<<agg_elem_blocks((int64_t)P + 1), kBlock, 0, s>>>(P, length, keys_s, tstart);
    DGS_LAUNCH_CHECK(s, debug);
    return DGS_OK;
}

// ------------------------------------------------------------------------- warm-up
// A no-op launch: the first launch of any kernel of this translation unit loads its code object
// (rocprim's kernels included) onto the device; dgs_warmup does it for every unit up front.
__global__ void k_warm_aggregate() {}
namespace dgs {
hipError_t warm_aggregate(hipStream_t s) {
    k_warm_aggregate<<<1, 1, 0, s>>>();
    return hipGetLastError();
}
}  // namespace dgs
