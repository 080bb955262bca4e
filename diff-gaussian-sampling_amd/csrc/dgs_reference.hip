// dgs_reference.hip -- the call-time path of the render calls (see dgs_reference.h).
//
// k_verify        : the call's means / conics / samples against the binning's copies -> flag
// k_ref_forward   : renderCUDA (forward.cu:87-166) on the reference's pair set: unit = (tile,
//                   64 of its samples in sorted order), lane = sample, the tile's Gaussian list
//                   walked in ascending id (the reference's per-thread order) with wave-uniform
//                   scalar loads of the CALL-TIME means / conics / values
// k_ref_backward  : renderCUDA backward (backward.cu:26-106): unit = (tile, 64 entries of its
//                   list), lane = Gaussian (call-time parameters), the tile's samples
//                   wave-uniform; per lane one float atomic per gradient component per unit into
//                   the internal-order sums that k_finalize permutes to caller order
// Both run only when the flag is set (they exit at once otherwise); the fine-cell kernels of
// dgs_sample.hip exit when it is set.  The arithmetic per pair is the reference's: the exact
// period-2 wrap (ref_wrap), the literal power (ref_power), `power > 0 -> skip`, expf.
#include "dgs_reference.h"

namespace dgs {

static inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// ------------------------------------------------------------------------------ verify
__global__ void k_verify(const char *__restrict__ gb, const char *__restrict__ sb, int64_t nm,
                         int64_t nc, int64_t ns, const uint32_t *__restrict__ means,
                         const uint32_t *__restrict__ conics, const uint32_t *__restrict__ samples,
                         int vec, uint32_t *__restrict__ flag) {
    const Header *h = reinterpret_cast<const Header *>(gb);
    const uint32_t *cp[3] = {reinterpret_cast<const uint32_t *>(gb + sload(&h->o_mcopy)),
                             reinterpret_cast<const uint32_t *>(gb + sload(&h->o_ccopy)),
                             reinterpret_cast<const uint32_t *>(sb + sload(&h->o_scopy))};
    const uint32_t *in[3] = {means, conics, samples};
    const int64_t n[3] = {nm, nc, ns};
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    bool diff = false;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        int64_t done = 0;
        if (vec & (1 << r)) {  // 16-byte aligned input: 4 words per load
            const int64_t n4 = n[r] >> 2;
            const uint4 *a = reinterpret_cast<const uint4 *>(in[r]), *b = reinterpret_cast<const uint4 *>(cp[r]);
            for (int64_t i = t; i < n4; i += st) {
                const uint4 x = a[i], y = b[i];
                diff |= (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
            }
            done = n4 << 2;
        }
        for (int64_t i = done + t; i < n[r]; i += st) diff |= in[r][i] != cp[r][i];
    }
    if (__any(diff) && (threadIdx.x & (kWave - 1)) == 0) atomicOr(flag, 1u);
}

int verify_inputs(const char *gb, const char *sb, int P, int D, int N, const float *means,
                  const float *conics, const float *samples, uint32_t *flag, hipStream_t s, int debug) {
    const int S = D * (D + 1) / 2;
    const int64_t nm = (int64_t)P * D, nc = (int64_t)P * S, ns = (int64_t)N * D;
    int vec = 0;
    if ((reinterpret_cast<uintptr_t>(means) & 15) == 0) vec |= 1;
    if ((reinterpret_cast<uintptr_t>(conics) & 15) == 0) vec |= 2;
    if ((reinterpret_cast<uintptr_t>(samples) & 15) == 0) vec |= 4;
    const int64_t words = std::max(std::max(nm, nc), ns) / 4 + 1;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid_for(words), 2048));
    k_verify<<<blocks, kBlock, 0, s>>>(gb, sb, nm, nc, ns, reinterpret_cast<const uint32_t *>(means),
                                       reinterpret_cast<const uint32_t *>(conics),
                                       reinterpret_cast<const uint32_t *>(samples), vec, flag);
    DGS_LAUNCH_CHECK(s, debug);
    return DGS_OK;
}

// ---------------------------------------------------------------------- call-time path
// The tile of a unit: the last t with prefix[t] <= unit (prefix[T] = the unit count).
__device__ __forceinline__ int tile_of_unit(const uint32_t *prefix, int T, uint32_t unit) {
    int lo = 0, hi = T - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sload(&prefix[mid]) <= unit) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <int D>
__device__ __forceinline__ void ref_displacement(const float *m, const float *s, float *X) {
    X[0] = ref_wrap(m[0] - s[0]);  // forward.cu:144-157 (X = mean - sample, then the wrap)
    X[1] = D == 2 ? ref_wrap(m[1] - s[1]) : 0.0f;
}

template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock) void k_ref_forward(const char *__restrict__ gbuf, const char *__restrict__ sbuf,
                                                        const float *__restrict__ means,
                                                        const float *__restrict__ values,
                                                        const float *__restrict__ conics,
                                                        const float *__restrict__ samples,
                                                        const uint32_t *__restrict__ flag, const Outs outs,
                                                        int C, int cbase) {
    if (sload(flag) == 0u) return;  // the binned tensors were passed: the fine-cell kernels did it
    using Tr = Traits<FN, D>;
    constexpr int U = Tr::U, S = Tr::S;
    const Bins bins = resolve(gbuf, sbuf);
    const int T = sload(&bins.h->T);
    const uint32_t *gst = bins.rtab + kRtGStart * (T + 1), *sst = bins.rtab + kRtSStart * (T + 1);
    const uint32_t *fu = bins.rtab + kRtFwdUnits * (T + 1);
    const uint32_t nunits = sload(&fu[T]);
    const int lane = threadIdx.x & (kWave - 1);
    const int nch = min(CB, C - cbase);
    const uint32_t w0 = blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t unit = w0; unit < nunits; unit += gridDim.x * kWavesPerBlock) {
        const int t = tile_of_unit(fu, T, unit);
        const uint32_t sb = sload(&sst[t]), se = sload(&sst[t + 1]);
        const uint32_t j = sb + (unit - sload(&fu[t])) * kRefUnit + lane;
        const bool active = j < se;
        const int64_t sid = bins.sorted_sid[active ? j : sb];
        const float s[2] = {samples[sid * D], D == 2 ? samples[sid * D + 1] : 0.0f};
        float acc[U][CB];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) acc[u][ch] = 0.0f;
        const uint32_t ge = sload(&gst[t + 1]);
        for (uint32_t e = sload(&gst[t]); e < ge; ++e) {  // ascending Gaussian id, as the reference
            const int64_t g = sload(&bins.rlist[e]);
            float m[2], c[3] = {0.0f, 0.0f, 0.0f}, v[CB];
            m[0] = sload(&means[g * D]);
            m[1] = D == 2 ? sload(&means[g * D + 1]) : 0.0f;
#pragma unroll
            for (int k = 0; k < S; ++k) c[k] = sload(&conics[g * S + k]);
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) v[ch] = ch < nch ? sload(&values[g * C + cbase + ch]) : 0.0f;
            float X[2];
            ref_displacement<D>(m, s, X);
            const float p = ref_power<FN, D>(X, c);
            if (!(p > 0.0f)) fwd_terms<FN, D, CB, float>(X, c, expf(p), v, acc);  // forward.cu:228
        }
        if (active) {
#pragma unroll
            for (int ui = 0; ui < U; ++ui)
#pragma unroll
                for (int ch = 0; ch < CB; ++ch)
                    if (ch < nch) store_unique<FN, D, false>(outs, sid, ui, C, cbase + ch, acc[ui][ch]);
        }
    }
}

// One function f of the call's mask: this sample's dL (summed over symmetric components) and
// the reference's per-pair gradient terms, into that function's accumulators.
template <int f, int D, int CB>
__device__ __forceinline__ void ref_bwd_fn(const DLs &dls, int64_t sid, int C, int cbase, int nch,
                                           const float *X, const float *c, float G, const float *v,
                                           float *gm, float *gv, float *gc) {
    constexpr int U = Traits<f, D>::U, K = Traits<f, D>::K;
    float dl[U][CB];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) dl[u][ch] = 0.0f;
    const float *d = dls.p[f] + sid * K * C + cbase;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int ch = 0; ch < CB; ++ch)
            if (ch < nch) dl[unique_fk(f, D, k)][ch] += sload(&d[k * C + ch]);
    bwd_terms<f, D, CB, float>(X, c, G, v, dl, gm, gv, gc);
}

template <int f, int D, int CB>
__device__ __forceinline__ void ref_bwd_finish_fn(const float *c, const float *v, float *gm, float *gc) {
    if constexpr (f == 0 && CB == 1 && DGS_VFACTOR) {  // v-factored moments (bwd_terms)
#pragma unroll
        for (int d = 0; d < 2; ++d) gm[d] *= v[0];
#pragma unroll
        for (int k = 0; k < 3; ++k) gc[k] *= v[0];
    }
    bwd_finish<f, D>(c, gm, gc);
}

template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock) void k_ref_backward(const char *__restrict__ gbuf, const char *__restrict__ sbuf,
                                                         const float *__restrict__ means,
                                                         const float *__restrict__ values,
                                                         const float *__restrict__ conics,
                                                         const float *__restrict__ samples,
                                                         const uint32_t *__restrict__ flag, const DLs dls,
                                                         float *__restrict__ acc, int P, int C, int cbase) {
    if (sload(flag) == 0u) return;
    constexpr int M = fn_mask(FN), S = D * (D + 1) / 2;
    const Bins bins = resolve(gbuf, sbuf);
    const int T = sload(&bins.h->T);
    const uint32_t *gst = bins.rtab + kRtGStart * (T + 1), *sst = bins.rtab + kRtSStart * (T + 1);
    const uint32_t *bu = bins.rtab + kRtBwdUnits * (T + 1);
    const int32_t *inv = bins.perm + P;
    const uint32_t nunits = sload(&bu[T]);
    const int lane = threadIdx.x & (kWave - 1);
    const int nch = min(CB, C - cbase);
    const uint32_t w0 = blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t unit = w0; unit < nunits; unit += gridDim.x * kWavesPerBlock) {
        const int t = tile_of_unit(bu, T, unit);
        const uint32_t eb = sload(&gst[t]), ee = sload(&gst[t + 1]);
        const uint32_t e = eb + (unit - sload(&bu[t])) * kRefUnit + lane;
        const bool active = e < ee;
        const int64_t g = bins.rlist[active ? e : eb];
        const float m[2] = {means[g * D], D == 2 ? means[g * D + 1] : 0.0f};
        float c[3] = {0.0f, 0.0f, 0.0f}, v[CB];
#pragma unroll
        for (int k = 0; k < S; ++k) c[k] = conics[g * S + k];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) v[ch] = ch < nch ? values[g * C + cbase + ch] : 0.0f;
        float gm[4][2], gv[4][CB], gc[4][3];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            gm[f][0] = gm[f][1] = gc[f][0] = gc[f][1] = gc[f][2] = 0.0f;
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) gv[f][ch] = 0.0f;
        }
        const uint32_t se = sload(&sst[t + 1]);
        for (uint32_t j = sload(&sst[t]); j < se; ++j) {  // the tile's samples, wave-uniform
            const int64_t sid = sload(&bins.sorted_sid[j]);
            const float s[2] = {sload(&samples[sid * D]), D == 2 ? sload(&samples[sid * D + 1]) : 0.0f};
            float X[2];
            ref_displacement<D>(m, s, X);
            const float p = ref_power<FN, D>(X, c);
            if (p > 0.0f) continue;  // backward.cu:114/133/...: power > 0 -> skip
            const float G = expf(p);
            if constexpr ((M & 1) != 0) ref_bwd_fn<0, D, CB>(dls, sid, C, cbase, nch, X, c, G, v, gm[0], gv[0], gc[0]);
            if constexpr ((M & 2) != 0) ref_bwd_fn<1, D, CB>(dls, sid, C, cbase, nch, X, c, G, v, gm[1], gv[1], gc[1]);
            if constexpr ((M & 4) != 0) ref_bwd_fn<2, D, CB>(dls, sid, C, cbase, nch, X, c, G, v, gm[2], gv[2], gc[2]);
            if constexpr ((M & 8) != 0) ref_bwd_fn<3, D, CB>(dls, sid, C, cbase, nch, X, c, G, v, gm[3], gv[3], gc[3]);
        }
        if (!active) continue;
        if constexpr ((M & 1) != 0) ref_bwd_finish_fn<0, D, CB>(c, v, gm[0], gc[0]);
        if constexpr ((M & 2) != 0) ref_bwd_finish_fn<1, D, CB>(c, v, gm[1], gc[1]);
        if constexpr ((M & 4) != 0) ref_bwd_finish_fn<2, D, CB>(c, v, gm[2], gc[2]);
        if constexpr ((M & 8) != 0) ref_bwd_finish_fn<3, D, CB>(c, v, gm[3], gc[3]);
        float sm[2] = {0.0f, 0.0f}, sc[3] = {0.0f, 0.0f, 0.0f}, sv[CB];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) sv[ch] = 0.0f;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            if (!(M & (1 << f))) continue;
            sm[0] += gm[f][0]; sm[1] += gm[f][1];
            sc[0] += gc[f][0]; sc[1] += gc[f][1]; sc[2] += gc[f][2];
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) sv[ch] += gv[f][ch];
        }
        const int64_t i = inv[g];  // internal index: k_finalize permutes to caller order
#pragma unroll
        for (int d = 0; d < D; ++d) atomicAdd(acc + (int64_t)d * P + i, sm[d]);
#pragma unroll
        for (int k = 0; k < S; ++k) atomicAdd(acc + (int64_t)(D + k) * P + i, sc[k]);
#pragma unroll
        for (int ch = 0; ch < CB; ++ch)
            if (ch < nch) atomicAdd(acc + (int64_t)(D + S + cbase + ch) * P + i, sv[ch]);
    }
}

// Persistent grids: the work is known only on the device; when the flag is clear every block
// exits after one scalar load.
static unsigned ref_blocks(int64_t units) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((units + kWavesPerBlock - 1) / kWavesPerBlock, 1024));
}

template <int FN, int D, int CB>
int ref_forward(const RefCall &a) {
    const int64_t cap = a.N / kRefUnit + (a.N + 1);  // >= the device-side unit count
    k_ref_forward<FN, D, CB><<<ref_blocks(cap), kBlock, 0, a.s>>>(a.gb, a.sb, a.means, a.values, a.conics,
                                                                  a.samples, a.flag, a.outs, a.C, a.cbase);
    DGS_LAUNCH_CHECK(a.s, a.debug);
    return DGS_OK;
}

template <int FN, int D, int CB>
int ref_backward(const RefCall &a) {
    const int64_t cap = a.R / kRefUnit + (a.R + 1);
    k_ref_backward<FN, D, CB><<<ref_blocks(cap), kBlock, 0, a.s>>>(a.gb, a.sb, a.means, a.values, a.conics,
                                                                   a.samples, a.flag, a.dls, a.acc, a.P,
                                                                   a.C, a.cbase);
    DGS_LAUNCH_CHECK(a.s, a.debug);
    return DGS_OK;
}

#define DGS_REF_INST(FN, D, CB)                            \
    template int ref_forward<FN, D, CB>(const RefCall &);  \
    template int ref_backward<FN, D, CB>(const RefCall &);
#define DGS_REF_INST_CB(FN, D) \
    DGS_REF_INST(FN, D, 1) DGS_REF_INST(FN, D, 2) DGS_REF_INST(FN, D, 4) DGS_REF_INST(FN, D, 8) DGS_REF_INST(FN, D, 16)
DGS_REF_INST_CB(0, 1) DGS_REF_INST_CB(0, 2)
DGS_REF_INST_CB(1, 1) DGS_REF_INST_CB(1, 2)
DGS_REF_INST_CB(2, 1) DGS_REF_INST_CB(2, 2)
DGS_REF_INST_CB(3, 1) DGS_REF_INST_CB(3, 2)
DGS_REF_INST(kMulti + 3, 2, 1) DGS_REF_INST(kMulti + 5, 2, 1) DGS_REF_INST(kMulti + 6, 2, 1)
DGS_REF_INST(kMulti + 7, 2, 1) DGS_REF_INST(kMulti + 9, 2, 1) DGS_REF_INST(kMulti + 10, 2, 1)
DGS_REF_INST(kMulti + 11, 2, 1) DGS_REF_INST(kMulti + 12, 2, 1) DGS_REF_INST(kMulti + 13, 2, 1)
DGS_REF_INST(kMulti + 14, 2, 1) DGS_REF_INST(kMulti + 15, 2, 1)

}  // namespace dgs

// ------------------------------------------------------------------------- warm-up
// A no-op launch: the first launch of any kernel of this translation unit loads its code object
// (rocprim's kernels included) onto the device; dgs_warmup does it for every unit up front.
__global__ void k_warm_reference() {}
namespace dgs {
hipError_t warm_reference(hipStream_t s) {
    k_warm_reference<<<1, 1, 0, s>>>();
    return hipGetLastError();
}
}  // namespace dgs
