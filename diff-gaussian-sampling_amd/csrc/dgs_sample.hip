// dgs_sample.hip -- forward and backward sampling kernels (gfx950).
//
// Replaces FORWARD::render / BACKWARD::render (forward.cu:87-166, 277-345;
// backward.cu:26-106, 418-501) and the per-call host glue of sample_points.cu:100-372.
//
// Work decomposition (one wave64 per work unit, 4 independent waves per 256-thread block):
//   forward : unit = (fine cell, up to 128 of its samples).  Lane l holds samples l and l+64
//             and evaluates both with packed fp32 ops (v_pk_*; a unit of <= 64 samples runs
//             the one-sample-per-lane instance).  The cell's Gaussian list is walked
//             wave-uniformly: each Gaussian's packed row comes in through the scalar cache
//             (s_load) into SGPRs, so the per-pair work is pure VALU and the accumulation
//             stays in registers (no atomics, no global RMW per pair).
//   backward: unit = (fine cell, up to 64 entries of its Gaussian list).  Lane = Gaussian.
//             The cell's samples (position + dL/dout) are walked wave-uniformly through the
//             scalar cache, two at a time with packed ops where the sample rows are small
//             enough to be stored as interleaved pairs; every lane accumulates its own
//             Gaussian's gradient in registers and issues one atomic add per gradient
//             component at the end of the unit.  Gaussians are renumbered spatially at
//             preprocess, so a wave's 64 lanes add to nearly contiguous addresses.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>

#include "dgs_reference.h"

namespace dgs {

static inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// --------------------------------------------------------------------------- packing
template <int FN, int D, int CB>
__global__ void k_pack_gauss(int P, const char *__restrict__ gbuf, const float *__restrict__ values, int C,
                             int cbase, float *__restrict__ rows, uint32_t *__restrict__ flag_zero) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (flag_zero && i == 0) *flag_zero = 0u;  // the call's input check (k_verify) runs next
    if (i >= P) return;
    // means / conics were packed in internal order at binning (coalesced here); only the
    // values are gathered through perm
    const Header *h = reinterpret_cast<const Header *>(gbuf);
    const int32_t *perm = reinterpret_cast<const int32_t *>(gbuf + h->o_perm);
    const float2 mm = reinterpret_cast<const float2 *>(gbuf + h->o_gmean)[i];
    const float4 cc = reinterpret_cast<const float4 *>(gbuf + h->o_gcon)[i];
    constexpr int RS = grow_stride<FN, D, CB>(), B = Traits<FN, D>::GBASE;
    const float c[3] = {cc.x, cc.y, cc.z};
    float out[RS];
#pragma unroll
    for (int k = 0; k < RS; ++k) out[k] = 0.0f;
    if constexpr (D == 2) {
        out[0] = mm.x;
        out[1] = mm.y;
        out[2] = -0.5f * kLog2e * c[0];
        out[3] = -kLog2e * c[1];
        out[4] = -0.5f * kLog2e * c[2];
        if constexpr (Traits<FN, D>::CONIC) { out[5] = c[0]; out[6] = c[1]; out[7] = c[2]; }
    } else {
        out[0] = mm.x;
        out[1] = -0.5f * kLog2e * c[0];
        if constexpr (Traits<FN, D>::CONIC) out[2] = c[0];
    }
    if (CB > 0 && cbase < C) {
        const int64_t g = perm[i];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) {
            const int gc = cbase + ch;
            out[B + ch] = gc < C ? values[g * C + gc] : 0.0f;
        }
    }
    float *row = rows + i * RS;
#pragma unroll
    for (int k = 0; k < RS; k += 4)
        *reinterpret_cast<float4 *>(row + k) = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
}

// Sample rows of the backward.  Packed layout (kPairRows): samples j = 2p, 2p+1 share the
// pair row p, field-interleaved [f0(2p) f0(2p+1) f1(2p) f1(2p+1) ...], so that a wave-uniform
// s_load puts each field of both samples into an aligned SGPR pair (a packed-op operand).
template <int FN, int D, int CB>
__host__ __device__ constexpr bool pair_rows() { return srow_stride<FN, D, CB>() <= 16; }

constexpr int kSrowPad = 16;
template <int FN, int D, int CB>
__global__ void k_pack_samples(int N, const char *__restrict__ gbuf, const char *__restrict__ sbuf,
                               const DLs dls, int C, int cbase, float *__restrict__ rows,
                               float4 *__restrict__ acc_zero, int64_t acc_n4, uint32_t *__restrict__ flag_zero) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // the gradient sums' zero-fill and the call's input-check word (k_verify runs next), folded
    // into this launch (first channel block only)
    if (flag_zero && j == 0) *flag_zero = 0u;
    if (acc_zero)
        for (int64_t k = j; k < acc_n4; k += (int64_t)gridDim.x * blockDim.x) acc_zero[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr bool PK = pair_rows<FN, D, CB>();
    // (scalar layout: kSrowPad zero rows after the last sample, read by k_backward_mx's last steps)
    if (j >= (PK ? (int64_t)(N + 1) / 2 * 2 : (int64_t)N + kSrowPad)) return;
    constexpr int M = fn_mask(FN), RSS = srow_stride<FN, D, CB>();
    float out[RSS];
#pragma unroll
    for (int k = 0; k < RSS; ++k) out[k] = 0.0f;
    if (j < N) {  // j == N (odd N, packed): the zero second half of the last pair
        const Header *h = reinterpret_cast<const Header *>(gbuf);
        const int32_t *sorted = reinterpret_cast<const int32_t *>(sbuf + h->o_sorted);
        const int64_t sid = sorted[j];
        // coordinates from the binning's sorted pair rows (coalesced); only dL is gathered
        const float *fr = reinterpret_cast<const float *>(sbuf + h->o_fsrows) + (j >> 1) * (2 * D) + (j & 1);
        out[0] = fr[0];
        if constexpr (D == 2) out[1] = fr[2];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            if (!(M & (1 << f))) continue;
            const int K = fn_k(f, D);
            const float *d = dls.p[f] + sid * K * C;
            if constexpr (bwd_mom<FN, D, CB>()) {  // moment form (C = 1): pre-scaled coefficients
                float hs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < K; ++k) hs[unique_fk(f, D, k)] += d[k];
                mom_coef(f, hs, &out[D + mask_foff(M, f)]);
            } else {  // dL summed over symmetric components, [U][CB]
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const int u = unique_fk(f, D, k);
#pragma unroll
                    for (int ch = 0; ch < CB; ++ch) {
                        const int gc = cbase + ch;
                        if (gc < C) out[D + u * CB + ch] += d[k * C + gc];
                    }
                }
            }
        }
    }
    if constexpr (PK) {
        float *row = rows + (j >> 1) * (2 * RSS) + (j & 1);
#pragma unroll
        for (int k = 0; k < RSS; ++k) row[2 * k] = out[k];
    } else {
        float *row = rows + j * RSS;
#pragma unroll
        for (int k = 0; k < RSS; k += 4)
            *reinterpret_cast<float4 *>(row + k) = make_float4(out[k], out[k + 1], out[k + 2], out[k + 3]);
    }
}

// ------------------------------------------------------------------- pair probability
// Fast path: no torus wrap in this (Gaussian, cell) entry and a well-conditioned PD conic, so
// power <= 0 is guaranteed and G = 2^(power*log2e) is one v_exp_f32.  General path: the
// reference's exact wrap and, for other conics, the reference-literal power with its
// `power > 0 -> skip` rule (forward.cu:228) and an accurate expf.
template <int D, typename V>
__device__ __forceinline__ V fast_prob(const V *X, const float *k) {
    if constexpr (D == 2) return vexp2(vfma(X[0], vfma(bc<V>(k[0]), X[0], k[1] * X[1]), k[2] * X[1] * X[1]));
    else return vexp2(k[0] * X[0] * X[0]);
}

template <int FN, int D>
__device__ __forceinline__ float general_prob(float *X, const float *c, const float *k, bool wrap,
                                              bool unsafe) {
    if (wrap) {
        X[0] = ref_wrap(X[0]);
        if constexpr (D == 2) X[1] = ref_wrap(X[1]);
    }
    if (unsafe) {
        const float p = ref_power<FN, D>(X, c);
        return p > 0.0f ? 0.0f : expf(p);
    }
    return fast_prob<D, float>(X, k);
}

template <int FN, int D>
__device__ __forceinline__ f2 general_prob(f2 *X, const float *c, const float *k, bool wrap,
                                           bool unsafe) {
    float Xa[2] = {X[0].x, D == 2 ? X[1].x : 0.0f}, Xb[2] = {X[0].y, D == 2 ? X[1].y : 0.0f};
    const float Ga = general_prob<FN, D>(Xa, c, k, wrap, unsafe);
    const float Gb = general_prob<FN, D>(Xb, c, k, wrap, unsafe);
    X[0] = f2{Xa[0], Xb[0]};
    if constexpr (D == 2) X[1] = f2{Xa[1], Xb[1]};
    return f2{Ga, Gb};
}

// Raw conic of a Gaussian row (FN != gaussian keeps it in the row).
template <int FN, int D, int RS>
__device__ __forceinline__ void row_conic(const float (&r)[RS], float *c) {
    if constexpr (Traits<FN, D>::CONIC) {
        if constexpr (D == 2) { c[0] = r[5]; c[1] = r[6]; c[2] = r[7]; }
        else { c[0] = r[2]; c[1] = c[2] = 0.0f; }
    } else {
        c[0] = c[1] = c[2] = 0.0f;
    }
}

// ------------------------------------------------------------------- forward kernels
// A forward unit is (cell, pair-aligned block of up to 64 sorted samples); the samples it
// writes are those of the block that belong to the cell.
struct FwdUnit {
    int cell, sb, lo, hi;  // block start (even), written sample range [lo, hi)
};

__device__ __forceinline__ FwdUnit fwd_unit_at(const Bins &bins, int unit) {
    const uint2 u = sload(&bins.fwd_units[unit]);
    FwdUnit f;
    f.cell = (int)u.x;
    f.sb = (int)u.y;
    f.lo = max(f.sb, sload(&bins.cell_sbeg[f.cell]));
    f.hi = min(f.sb + kFwdUnit, sload(&bins.cell_send[f.cell]));
    return f;
}

// Centre of a cell's sample bounding box: preprocess classified each kGeneral entry's wrap
// shift as constant over exactly that box (plus rounding margin), so the shift at the centre
// is the shift of every sample of the cell.  (The nominal cell may reach past the last
// sample and across a wrap breakpoint; its centre would not do.)
template <int D>
__device__ __forceinline__ void cell_center(const Bins &bins, int cell, float *ctr) {
    const float4 b = sload(&bins.cell_box[cell]);
    ctr[0] = 0.5f * (b.x + b.z);
    ctr[1] = 0.5f * (b.y + b.w);
}

// (a) Transposed form (small accumulators, U * CB <= 4).  Lane = Gaussian of the cell list,
// 64 at a time (rows by vector gather); the block's samples are wave-uniform, read in order
// as packed pair rows [s0(2p) s0(2p+1) s1(2p) s1(2p+1)] through the scalar cache, and the
// pair math is packed fp32.  Every lane keeps a partial sum per (sample, component) over the
// whole cell list; one cross-lane reduce-scatter per pass then leaves sum (sample, comp) =
// value l in lane l.  Row delivery per pair is negligible here (the lane-per-sample form is
// bound by the scalar cache's random-row throughput, tools/ubench.hip).

#ifndef DGS_BWD_PIPE
// backward pair loop: the next batch of pair rows in flight during this one; 2 (round 6): two
// batch buffers in turn, no register copy of the look-ahead batch per iteration (-3 %)
#define DGS_BWD_PIPE 2
#endif
#ifndef DGS_BWD_PRIO
// backward wave priority (round 6, -1 % on top of DGS_BWD_PIPE 2): s_setprio 3 while a wave is not in
// its pair loop -- kernel entry and header loads (3), each unit's dependent unit -> entry -> row
// loads (1), the finish and the atomics (2) -- and 0 inside it, so a wave waiting on its setup
// chain issues its loads ahead of the VALU-bound waves instead of behind them
#define DGS_BWD_PRIO 3
#endif
#ifndef DGS_FWD_SUB
#define DGS_FWD_SUB 1  // D = 2 transposed forward over the sub-cell lists (k_forward_s)
#endif
#ifndef DGS_FWD_FULL
#define DGS_FWD_FULL 1  // whole passes take the explicitly pipelined pair-row loads
#endif
#ifndef DGS_MULTI_T
#define DGS_MULTI_T 1  // fused form: transposed forward (else lane-per-sample)
#endif
template <int FN, int D, int CB>
__host__ __device__ constexpr bool fwd_transposed() {
    return Traits<FN, D>::U * CB <= 4 || (is_multi(FN) && DGS_MULTI_T);
}

// The pass's first `np` (<= NP, wave-uniform) sample pairs against the lane's Gaussian.
// WRAP: some lane's entry crosses the torus seam.  Its wrap (forward.cu:149-157) is a
// constant even shift over the cell (preprocess sends the other seam entries to the general
// path), subtracted exactly: sh = 0 for every other lane.
template <int FN, int D, int CB, bool WRAP>
__device__ __forceinline__ void fwd_t_pair(const float *pr, const float *m, const float *sh, const float *c,
                                           const float *kk, const float *v, f2 (&acc)[Traits<FN, D>::U][CB]) {
    f2 X[2] = {m[0] - f2{pr[0], pr[1]}, D == 2 ? m[1] - f2{pr[2], pr[3]} : bc<f2>(0.0f)};
    if constexpr (WRAP) {
        X[0] = X[0] - sh[0];
        if constexpr (D == 2) X[1] = X[1] - sh[1];
    }
    fwd_terms<FN, D, CB, f2>(X, c, fast_prob<D, f2>(X, kk), v, acc);
}

// s_waitcnt lgkmcnt(0) (gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0)
#define DGS_WAIT_LGKM0() __builtin_amdgcn_s_waitcnt(0xC07F)

template <int FN, int D, int CB, int NP, bool WRAP, bool FULL>
__device__ __forceinline__ void fwd_t_pairs(const float *__restrict__ fsrows, int p0, int np,
                                            const float *m, const float *sh, const float *c,
                                            const float *kk, const float *v,
                                            f2 (&acc)[NP][Traits<FN, D>::U][CB]) {
    constexpr int LW = 16;  // (x8 loads measured 6x slower: the unrolled pass stopped interleaving)
    constexpr int PRF = 2 * D, PPL = LW / PRF;  // floats per pair row, pairs per s_load_dwordx16
    if constexpr (FULL) {
        // A whole pass (np == NP): the next block of pair rows is in flight while this one is
        // evaluated.  Scalar loads complete out of order, so a block can only be waited for
        // with lgkmcnt(0); the wait is therefore placed explicitly BEFORE the next block's load
        // is issued, and scheduling barriers keep the compiler from hoisting the loads (with a
        // variable pass length it turned the exits into a cascade that issued them all first).
        constexpr int NB = NP / PPL;
        static_assert(NP % PPL == 0, "full passes are whole load blocks");
        F32s<LW> cur = sload_f<LW>(fsrows + (int64_t)p0 * PRF);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            F32s<LW> nxt;
            DGS_WAIT_LGKM0();
            __builtin_amdgcn_sched_barrier(0);
            if (b + 1 < NB) nxt = sload_f<LW>(fsrows + (int64_t)(p0 + (b + 1) * PPL) * PRF);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < PPL; ++j)
                fwd_t_pair<FN, D, CB, WRAP>(&cur.v[j * PRF], m, sh, c, kk, v, acc[b * PPL + j]);
            __builtin_amdgcn_sched_barrier(0);
            if (b + 1 < NB) cur = nxt;
        }
    } else {
#pragma unroll
        for (int q = 0; q < NP; q += PPL) {
            if (q >= np) break;
            const F32s<LW> sr = sload_f<LW>(fsrows + (int64_t)(p0 + q) * PRF);
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                if (q + j < NP) fwd_t_pair<FN, D, CB, WRAP>(&sr.v[j * PRF], m, sh, c, kk, v, acc[q + j]);
            }
        }
    }
}

// Cell-list entries [eb, ee) against the pass's sample pairs, 64 Gaussians (lanes) at a time.
template <int RS>
__device__ __forceinline__ void load_grow(const float *__restrict__ grows, uint32_t ent, float (&r)[RS]) {
    const float *grow = grows + (int64_t)(ent & kIdMask) * RS;
#pragma unroll
    for (int k = 0; k < RS; k += 4) {
        const float4 qv = *reinterpret_cast<const float4 *>(grow + k);
        r[k] = qv.x; r[k + 1] = qv.y; r[k + 2] = qv.z; r[k + 3] = qv.w;
    }
}

// One group: the lane's row r (entry ent; `active` = a real entry) against the pass's pairs.
template <int FN, int D, int CB, int NP, bool FLAGGED, bool FULL>
__device__ __forceinline__ void fwd_t_group(const float *__restrict__ fsrows, float (&r)[grow_stride<FN, D, CB>()],
                                            uint32_t ent, bool active, int p0, int np, const float *ctr,
                                            f2 (&acc)[NP][Traits<FN, D>::U][CB]) {
    constexpr int RS = grow_stride<FN, D, CB>(), B = Traits<FN, D>::GBASE;
    // a padding lane, or a kUnsafe entry (done by the tail pass), adds exactly 0.  Flagged
    // groups zero the whole row (an unsafe conic may overflow); a padding lane of a flag-free
    // group holds a copy of a well-conditioned row (finite terms), so zero values suffice.
    if constexpr (FLAGGED) {  // (kUnsafe: the tail pass)
        if (!active || (ent & kUnsafe)) {
#pragma unroll
            for (int k = 0; k < RS; ++k) r[k] = 0.0f;
        }
    } else {
        if (!active) {
#pragma unroll
            for (int k = B; k < RS; ++k) r[k] = 0.0f;
        }
    }
    float c[3];
    row_conic<FN, D, RS>(r, c);
    const float m[2] = {r[0], D == 2 ? r[1] : 0.0f};
    float sh[2] = {0.0f, 0.0f};  // the lane's constant wrap shift (kGeneral entries)
    if constexpr (FLAGGED) {
        if (active && (ent & (kGeneral | kUnsafe)) == kGeneral) {
#pragma unroll
            for (int d = 0; d < D; ++d) sh[d] = wrap_shift_f(m[d] - ctr[d]);
        }
    }
    fwd_t_pairs<FN, D, CB, NP, FLAGGED, FULL>(fsrows, p0, np, m, sh, c, &r[D], &r[B], acc);
}

// Software-pipelined over the groups: group g + 1's rows and group g + 2's entries are in
// flight while group g is evaluated (each group otherwise starts with two dependent memory
// round trips, entry then row).
template <int FN, int D, int CB, int NP, bool FLAGGED, bool FULL>
__device__ __forceinline__ void fwd_t_groups(const Bins &bins, const float *__restrict__ grows,
                                             const float *__restrict__ fsrows, int eb, int ee,
                                             int p0, int np, int lane, const float *ctr,
                                             f2 (&acc)[NP][Traits<FN, D>::U][CB]) {
    constexpr int RS = grow_stride<FN, D, CB>();
    if (eb >= ee) return;
    const int last = ee - 1;
    uint32_t e_cur = bins.entries[min(eb + lane, last)];
    uint32_t e_nxt = bins.entries[min(eb + kWave + lane, last)];
    float r_cur[RS];
    load_grow<RS>(grows, e_cur, r_cur);
    for (int g0 = eb; g0 < ee; g0 += kWave) {
        float r_nxt[RS];
        load_grow<RS>(grows, e_nxt, r_nxt);  // (a clamped, valid row past the list's end)
        const uint32_t e_nn = bins.entries[min(g0 + 2 * kWave + lane, last)];
        fwd_t_group<FN, D, CB, NP, FLAGGED, FULL>(fsrows, r_cur, e_cur, g0 + lane < ee, p0, np, ctr, acc);
#pragma unroll
        for (int k = 0; k < RS; ++k) r_cur[k] = r_nxt[k];
        e_cur = e_nxt;
        e_nxt = e_nn;
    }
}

template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock) void k_forward_t(const char *__restrict__ gbuf,
                                                      const char *__restrict__ sbuf,
                                                      const float *__restrict__ grows,
                                                      const Outs outs, int C, int cbase,
                                                      const uint32_t *__restrict__ dirty) {
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    using Tr = Traits<FN, D>;
    constexpr int U = Tr::U, K = Tr::K, UC = U * CB, RS = grow_stride<FN, D, CB>(), B = Tr::GBASE;
    constexpr int NP = 32 / UC, NS = 2 * NP;  // sample pairs / samples per pass
    static_assert(NP >= 1 && NS * UC <= 64, "accumulator does not fit the reduce-scatter");
    const Bins bins = resolve(gbuf, sbuf);
    const float *__restrict__ fsrows = bins.fsrows;
    const int nunits = sload(&bins.counts[kNumFwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1);
    const int nch = min(CB, C - cbase);
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const FwdUnit fu = fwd_unit_at(bins, unit);
        // every entry but the kUnsafe ones (added by k_forward<..., TAIL = true>)
        const int gb = sload(&bins.cell_gbeg[fu.cell]), ge = sload(&bins.cell_gend[fu.cell]);
        const int gm = sload(&bins.cell_gmid[fu.cell]);
        float ctr[2];
        cell_center<D>(bins, fu.cell, ctr);
        for (int ps = fu.sb; ps < fu.hi; ps += NS) {
            const int np = min(NP, (fu.hi - ps + 1) >> 1);
            f2 acc[NP][U][CB];
#pragma unroll
            for (int q = 0; q < NP; ++q)
#pragma unroll
                for (int a = 0; a < U; ++a)
#pragma unroll
                    for (int ch = 0; ch < CB; ++ch) acc[q][a][ch] = bc<f2>(0.0f);
            // flag-free prefix [gb, gm), then the flagged suffix [gm, ge) (seam wraps; the kUnsafe
            // entries there are left to the tail pass)
            constexpr bool kFullOk = DGS_FWD_FULL && NP % (8 / D) == 0;
            if (kFullOk && np == NP) {  // whole pass: pipelined pair-row loads
                fwd_t_groups<FN, D, CB, NP, false, kFullOk>(bins, grows, fsrows, gb, gm, ps >> 1, np, lane, ctr, acc);
                if (gm < ge)
                    fwd_t_groups<FN, D, CB, NP, true, kFullOk>(bins, grows, fsrows, gm, ge, ps >> 1, np, lane, ctr, acc);
            } else {
                fwd_t_groups<FN, D, CB, NP, false, false>(bins, grows, fsrows, gb, gm, ps >> 1, np, lane, ctr, acc);
                if (gm < ge)
                    fwd_t_groups<FN, D, CB, NP, true, false>(bins, grows, fsrows, gm, ge, ps >> 1, np, lane, ctr, acc);
            }
            // value index = (2 * pair + half) * UC + (u * CB + ch)
            float x[64];
#pragma unroll
            for (int i = 0; i < 64; ++i) x[i] = 0.0f;
#pragma unroll
            for (int q = 0; q < NP; ++q)
#pragma unroll
                for (int a = 0; a < U; ++a)
#pragma unroll
                    for (int ch = 0; ch < CB; ++ch) {
                        x[(2 * q) * UC + a * CB + ch] = acc[q][a][ch].x;
                        x[(2 * q + 1) * UC + a * CB + ch] = acc[q][a][ch].y;
                    }
            const float sum = reduce_scatter64(x, lane);
            const int slot = lane / UC, comp = lane - slot * UC;
            const int j = ps + slot, ui = comp / CB, ch = comp - ui * CB;
            if (lane < NS * UC && j >= fu.lo && j < fu.hi && ch < nch) {
                store_unique<FN, D, false>(outs, bins.sorted_sid[j], ui, C, cbase + ch, sum);
            }
        }
    }
}

// (a') Sub-cell form (D = 2; SURVEY 8d: W_cand towards W_live).  The transposed kernel over the
// sub units: a unit is (sub-cell, up to kSubPairs sample pairs) and walks the sub list -- the
// entries of its cell whose cut meets the sub-cell's sample box -- instead of the whole cell
// list.  The pass's first 16 pair rows are loaded once per pass, before the group loop, and stay
// in SGPRs for every group (no scalar load, hence no out-of-order lgkmcnt(0) wait, for them
// inside the loop).  Arithmetic, order per lane and the reduce-scatter are those of (a).
// The first HB (DGS_FWD_HB = 2) blocks of 4 pair rows are hoisted (at 4 blocks, 64 SGPRs, the kernel spilled SGPRs into VGPR lanes: a
// v_readlane per dword inside the loop); the pass's later blocks, needed by the larger sub-cells
// only, are loaded where they are used.
template <int FN, int D, int CB, int NPH, int HB, bool WRAP>
__device__ __forceinline__ void fwd_s_pairs(const F32s<16> (&hr)[HB], const float *__restrict__ prow, int np,
                                            const float *m, const float *sh, const float *c, const float *kk,
                                            const float *v, f2 (&acc)[NPH][Traits<FN, D>::U][CB]) {
    constexpr int PRF = 2 * D, PPL = 16 / PRF, NB = (NPH + PPL - 1) / PPL;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b * PPL >= np) break;  // wave-uniform: the rest of the pass is padding
        F32s<16> t;
        if (b < HB) t = hr[b < HB ? b : 0];
        else t = sload_f<16>(prow + (int64_t)b * PPL * PRF);
#pragma unroll
        for (int j = 0; j < PPL; ++j)
            if (b * PPL + j < NPH)
                fwd_t_pair<FN, D, CB, WRAP>(&t.v[j * PRF], m, sh, c, kk, v, acc[b * PPL + j]);
    }
}

#ifndef DGS_FWD_UNROLL
#define DGS_FWD_UNROLL 1  // sub-cell forward: list-walk unroll (register renaming instead of copies)
#endif
#ifndef DGS_FWD_HB
#define DGS_FWD_HB 2  // sub-cell forward: blocks of 4 pair rows hoisted into SGPRs for the list walk (4: SGPR spills, 2.7 % slower)
#endif
#ifndef DGS_FWD_PRIO
#define DGS_FWD_PRIO 0  // tuning: s_setprio 3 for a sub unit's setup, 0 for its list walk
#endif
#ifndef DGS_FWD_LDS
#define DGS_FWD_LDS 0  // sub-cell forward: the pass's pair rows staged in LDS (else hoisted into SGPRs)
#endif
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v4f lds_cf4;

// The LDS form: the pass's pair rows sit in the wave's LDS slot; each block of 4 pairs reads its
// 4 rows (broadcast ds_read_b128, in order, so counted waits) right before its arithmetic.  The
// slot address is re-laundered per group so the compiler cannot hoist the reads out of the list
// walk (hoisted, they would need 4 VGPRs per pair for the whole walk).
template <int FN, int D, int CB, int NPH, bool WRAP>
__device__ __forceinline__ void fwd_l_pairs(uint32_t slot, int np, const float *m, const float *sh, const float *c,
                                            const float *kk, const float *v, f2 (&acc)[NPH][Traits<FN, D>::U][CB]) {
    constexpr int PPL = 4, NB = (NPH + PPL - 1) / PPL;
    // One block of rows in flight: block b + 1 is read while block b is evaluated, into the other
    // of two register buffers (compile-time parity: no copies).  Its address is laundered through
    // the previous block's last sum, so the compiler can neither hoist the reads of the whole
    // pass to the front (a cascade holding every row in VGPRs) nor out of the list walk.
    float dep = 0.0f;
    v4f buf[2][PPL];
    {
        uint32_t sl = slot;
        asm volatile("" : "+v"(sl));
        lds_cf4 *rows = (lds_cf4 *)(size_t)sl;
#pragma unroll
        for (int j = 0; j < PPL; ++j) buf[0][j] = rows[j];
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b * PPL < np) {  // wave-uniform
            if (b + 1 < NB && (b + 1) * PPL < np) {
                uint32_t sl = slot;
                asm volatile("" : "+v"(sl) : "v"(dep));
                lds_cf4 *rows = (lds_cf4 *)(size_t)sl;
#pragma unroll
                for (int j = 0; j < PPL; ++j) buf[(b + 1) & 1][j] = rows[(b + 1) * PPL + j];
            }
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                const v4f q = buf[b & 1][j];
                const float pr[4] = {q[0], q[1], q[2], q[3]};
                if (b * PPL + j < NPH) fwd_t_pair<FN, D, CB, WRAP>(pr, m, sh, c, kk, v, acc[b * PPL + j]);
            }
            dep = acc[min(b * PPL + PPL - 1, NPH - 1)][0][0].x;
        }
    }
}

// FLAGGED: every lane but the kUnsafe ones (the tail pass), with the lane's constant wrap shift.
template <int FN, int D, int CB, int NPH, int HB, bool FLAGGED>
__device__ __forceinline__ void fwd_s_group(const F32s<16> (&hr)[HB], const float *__restrict__ prow, uint32_t slot,
                                            float (&r)[grow_stride<FN, D, CB>()],
                                            uint32_t ent, bool active, int np, const float *ctr,
                                            f2 (&acc)[NPH][Traits<FN, D>::U][CB]) {
    constexpr int RS = grow_stride<FN, D, CB>(), B = Traits<FN, D>::GBASE;
    bool on = active;
    if constexpr (FLAGGED) {
        on = active && !(ent & kUnsafe);
        if (!on) {
#pragma unroll
            for (int k = 0; k < RS; ++k) r[k] = 0.0f;
        }
    } else {
        if (!active) {
#pragma unroll
            for (int k = B; k < RS; ++k) r[k] = 0.0f;
        }
    }
    float c[3];
    row_conic<FN, D, RS>(r, c);
    const float m[2] = {r[0], D == 2 ? r[1] : 0.0f};
    float sh[2] = {0.0f, 0.0f};
    if constexpr (FLAGGED) {
        if (on && (ent & kGeneral)) {
#pragma unroll
            for (int d = 0; d < D; ++d) sh[d] = wrap_shift_f(m[d] - ctr[d]);
        }
    }
    if constexpr (DGS_FWD_LDS) {
        fwd_l_pairs<FN, D, CB, NPH, FLAGGED>(slot, np, m, sh, c, &r[D], &r[B], acc);
    } else {
        fwd_s_pairs<FN, D, CB, NPH, HB, FLAGGED>(hr, prow, np, m, sh, c, &r[D], &r[B], acc);
    }
}

template <int FN, int D, int CB, int NPH, int HB, bool FLAGGED>
__device__ __forceinline__ void fwd_s_groups(const uint32_t *__restrict__ ents, const float *__restrict__ grows,
                                             const F32s<16> (&hr)[HB], const float *__restrict__ prow, uint32_t slot,
                                             int eb, int ee, int np, int lane,
                                             const float *ctr, f2 (&acc)[NPH][Traits<FN, D>::U][CB]) {
    constexpr int RS = grow_stride<FN, D, CB>();
    if (eb >= ee) return;
    const int last = ee - 1;
    uint32_t e_cur = ents[min(eb + lane, last)];
    uint32_t e_nxt = ents[min(eb + kWave + lane, last)];
    float r_cur[RS];
    load_grow<RS>(grows, e_cur, r_cur);
#if DGS_FWD_UNROLL > 1
#pragma unroll DGS_FWD_UNROLL
#endif
    for (int g0 = eb; g0 < ee; g0 += kWave) {
        float r_nxt[RS];
        load_grow<RS>(grows, e_nxt, r_nxt);
        const uint32_t e_nn = ents[min(g0 + 2 * kWave + lane, last)];
        // flagged groups with no lane for this pass (all kUnsafe: the tail pass) are skipped
        bool work = true;
        if constexpr (FLAGGED) {
            const bool act = g0 + lane < ee;
            work = __builtin_amdgcn_readfirstlane((uint32_t)(__ballot(act && (e_cur & kUnsafe) == 0) != 0ull)) != 0u;
        }
        if (work)
            fwd_s_group<FN, D, CB, NPH, HB, FLAGGED>(hr, prow, slot, r_cur, e_cur, g0 + lane < ee, np, ctr, acc);
#pragma unroll
        for (int k = 0; k < RS; ++k) r_cur[k] = r_nxt[k];
        e_cur = e_nxt;
        e_nxt = e_nn;
    }
}

// Per sub unit the sub list [lbeg, lthin): its flag-free part, then its flagged part [lmid, lthin)
// (lthin = lend: no entry carries the round-4 kThin flag since round 6).
template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock) void k_forward_s(const char *__restrict__ gbuf,
                                                      const char *__restrict__ sbuf,
                                                      const float *__restrict__ grows,
                                                      const Outs outs, int C, int cbase,
                                                      const uint32_t *__restrict__ dirty) {
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    using Tr = Traits<FN, D>;
    constexpr int U = Tr::U, UC = U * CB;
    constexpr int NP0 = 32 / UC, NPH = NP0 < kSubPairs ? NP0 : kSubPairs, NS = 2 * NPH;
    constexpr int PRF = 2 * D, PPL = 16 / PRF, NB = (NPH + PPL - 1) / PPL, HB = NB < DGS_FWD_HB ? NB : DGS_FWD_HB;
    static_assert(D == 2 && NPH >= 1 && NS * UC <= 64, "sub-cell form: D = 2, reduce-scatter width");
    const Bins bins = resolve(gbuf, sbuf);
    const float *__restrict__ fsrows = bins.fsrows;
    const int nunits = sload(&bins.counts[kNumFwdSubUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1);
    const int nch = min(CB, C - cbase);
    __shared__ v4f srows[kWavesPerBlock][kSubPairs];  // DGS_FWD_LDS: each wave's pass rows
    const int wv = threadIdx.x >> 6;
    const uint32_t slot = (uint32_t)(size_t)(lds_cf4 *)(&srows[wv][0]);  // (addrspacecast: the LDS offset)
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
#if DGS_FWD_PRIO
        __builtin_amdgcn_s_setprio(3);  // (the unit's loads issue first; 0 again for the list walk)
#endif
        const uint2 u = sload(&bins.fsub_units[unit]);
        const int sc = (int)u.x, cell = sc / kSubPerCell, sb = (int)u.y;
        const int lo = max(sb, sload(&bins.sub_sbeg[sc]));
        const int hi = min(sb + 2 * kSubPairs, sload(&bins.sub_send[sc]));
        const int gb = sload(&bins.sub_lbeg[sc]), gm = sload(&bins.sub_lmid[sc]), ge = sload(&bins.sub_lend[sc]);
        const int gt = sload(&bins.sub_lthin[sc]);
        (void)ge;
        float ctr[2];
        cell_center<D>(bins, cell, ctr);
        for (int ps = sb; ps < hi; ps += NS) {
            // (provably wave-uniform: the block exits become scalar compares, not lane masks held in SGPRs)
            const int np = __builtin_amdgcn_readfirstlane(min(NPH, (hi - ps + 1) >> 1));
            const float *prow = fsrows + (int64_t)(ps >> 1) * PRF;
            F32s<16> hr[DGS_FWD_LDS ? 1 : HB];  // the pass's first pair rows, in SGPRs for the whole list walk
            if constexpr (DGS_FWD_LDS) {
                if (lane < NPH) srows[wv][lane] = reinterpret_cast<const v4f *>(prow)[lane];
            } else {
#pragma unroll
                for (int b = 0; b < HB; ++b) hr[b] = sload_f<16>(prow + (int64_t)b * PPL * PRF);
            }
            f2 acc[NPH][U][CB];
#pragma unroll
            for (int q = 0; q < NPH; ++q)
#pragma unroll
                for (int a = 0; a < U; ++a)
#pragma unroll
                    for (int ch = 0; ch < CB; ++ch) acc[q][a][ch] = bc<f2>(0.0f);
            constexpr int HBX = DGS_FWD_LDS ? 1 : HB;
#if DGS_FWD_PRIO
            __builtin_amdgcn_s_setprio(0);
#endif
            fwd_s_groups<FN, D, CB, NPH, HBX, false>(bins.sub_ent, grows, hr, prow, slot, gb, gm, np, lane, ctr, acc);
#ifdef DGS_TIMING_TWICE
            fwd_s_groups<FN, D, CB, NPH, HBX, false>(bins.sub_ent, grows, hr, prow, slot, gb, gm, np, lane, ctr, acc);
#endif
            if (gm < gt)
                fwd_s_groups<FN, D, CB, NPH, HBX, true>(bins.sub_ent, grows, hr, prow, slot, gm, gt, np, lane, ctr, acc);
            float x[64];
#pragma unroll
            for (int i = 0; i < 64; ++i) x[i] = 0.0f;
#pragma unroll
            for (int q = 0; q < NPH; ++q)
#pragma unroll
                for (int a = 0; a < U; ++a)
#pragma unroll
                    for (int ch = 0; ch < CB; ++ch) {
                        x[(2 * q) * UC + a * CB + ch] = acc[q][a][ch].x;
                        x[(2 * q + 1) * UC + a * CB + ch] = acc[q][a][ch].y;
                    }
            const float sum = reduce_scatter64(x, lane);
            const int slot = lane / UC, comp = lane - slot * UC;
            const int j = ps + slot, ui = comp / CB, ch = comp - ui * CB;
            if (lane < NS * UC && j >= lo && j < hi && ch < nch) {
                store_unique<FN, D, false>(outs, bins.sorted_sid[j], ui, C, cbase + ch, sum);
            }
        }
    }
}

// (b) Lane-per-sample form (wide accumulators, U * CB > 4): lane = sample of the block, the
// cell's Gaussian rows are walked wave-uniformly through the scalar cache.
template <int FN, int D, int CB, bool UNSAFE_ONLY>
__device__ __forceinline__ void fwd_accumulate(const Bins &bins, const float *__restrict__ grows,
                                               const float4 *__restrict__ crows, int eb, int ee,
                                               int gm, float s0, float s1,
                                               float (&acc)[Traits<FN, D>::U][CB]) {
    using Tr = Traits<FN, D>;
    constexpr int RS = grow_stride<FN, D, CB>(), B = Tr::GBASE;
    constexpr int NB = fwd_batch<RS>();
    const char *gbase = reinterpret_cast<const char *>(grows);
    // (1) flag-free entries in full batches: NB entries, then NB rows in flight, then math
    const int fe = min(ee, gm);
    int e0 = eb;
    for (; e0 + NB <= fe; e0 += NB) {
        const U32s<NB> E = sload_u<NB>(bins.entries + e0);
        F32s<RS> rows[NB];
#pragma unroll
        for (int q = 0; q < NB; ++q)  // 32-bit byte offset: folds into the s_load (soffset)
            rows[q] = sload_f<RS>(reinterpret_cast<const float *>(gbase + E.v[q] * (uint32_t)(RS * 4)));
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const float(&r)[RS] = rows[q].v;
            float c[3];
            row_conic<FN, D, RS>(r, c);
            float X[2] = {r[0] - s0, D == 2 ? r[1] - s1 : 0.0f};
            const float G = fast_prob<D, float>(X, &r[D]);
            fwd_terms<FN, D, CB, float>(X, c, G, &r[B], acc);
        }
    }
    // (2) the rest one by one: fast tail, then the flagged entries (wrap / unsafe conic)
    for (; e0 < ee; ++e0) {
        const uint32_t e = sload(&bins.entries[e0]);
        if (UNSAFE_ONLY && !(e & kUnsafe)) continue;
        const uint32_t id = e & kIdMask;
        const F32s<RS> row = sload_f<RS>(reinterpret_cast<const float *>(gbase + id * (uint32_t)(RS * 4)));
        const float(&r)[RS] = row.v;
        float c[3];
        row_conic<FN, D, RS>(r, c);
        float X[2] = {r[0] - s0, D == 2 ? r[1] - s1 : 0.0f};
        float G;
        if (!(e & kSlow)) {
            G = fast_prob<D, float>(X, &r[D]);
        } else {
            const bool lit = (e & kUnsafe) != 0;  // the reference-literal power
            if (lit) {
                const float4 cr = sload(&crows[id]);
                c[0] = cr.x; c[1] = cr.y; c[2] = cr.z;
            }
            G = general_prob<FN, D>(X, c, &r[D], (e & kGeneral) != 0, lit);
        }
        fwd_terms<FN, D, CB, float>(X, c, G, &r[B], acc);
    }
}

// TAIL = true: only the unsafe-conic entries (all in the flagged tail [gm, ge) of a list),
// added onto the transposed kernel's output, which covered every other entry.
template <int FN, int D, int CB, bool TAIL>
__global__ __launch_bounds__(kBlock) void k_forward(const char *__restrict__ gbuf,
                                                    const char *__restrict__ sbuf,
                                                    const float *__restrict__ grows,
                                                    const float *__restrict__ samples,
                                                    const Outs outs, int C, int cbase,
                                                    const uint32_t *__restrict__ dirty) {
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    constexpr int U = Traits<FN, D>::U, K = Traits<FN, D>::K;
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumFwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1);
    const int nch = min(CB, C - cbase);
    if (TAIL && sload(&bins.counts[kNumUnsafe]) == 0) return;  // no unsafe entry anywhere
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const FwdUnit fu = fwd_unit_at(bins, unit);
        if (TAIL && sload(&bins.cell_gmid[fu.cell]) == sload(&bins.cell_gend[fu.cell])) continue;
        const int j = fu.sb + lane;
        const bool active = j >= fu.lo && j < fu.hi;
        const int64_t sid = bins.sorted_sid[active ? j : fu.lo];
        const float s0 = samples[sid * D], s1 = D == 2 ? samples[sid * D + 1] : 0.0f;
        const int gb = sload(&bins.cell_gbeg[fu.cell]), ge = sload(&bins.cell_gend[fu.cell]);
        const int gm = sload(&bins.cell_gmid[fu.cell]);
        float acc[U][CB];
#pragma unroll
        for (int a = 0; a < U; ++a)
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) acc[a][ch] = 0.0f;
        fwd_accumulate<FN, D, CB, TAIL>(bins, grows, bins.gcon, TAIL ? gm : gb, ge, gm, s0, s1, acc);
        if (active) {
#pragma unroll
            for (int ui = 0; ui < U; ++ui)
#pragma unroll
                for (int ch = 0; ch < CB; ++ch)
                    if (ch < nch) store_unique<FN, D, TAIL>(outs, sid, ui, C, cbase + ch, acc[ui][ch]);
        }
    }
}

// (c) Matrix-core form (wide accumulators, CB >= 8).  For a unit's samples the forward is
// out[s][u][ch] = sum_g A_u[s][g] v[g][ch] with A_u = G t_u (the exponent and the terms of
// forward.cu:225-332): a [samples x Gaussians] by [Gaussians x channels] product.  A_u comes
// from the VALU (one pair per lane per step), the product from v_mfma_f32_16x16x4_f32, whose
// f32 accumulation is an exact fmaf chain.  Unit = (cell, 64 samples) as in k_forward.  A
// 4-Gaussian step gives 16-lane group kq = lane >> 4 the list entry e + kq; lane col = lane & 15
// evaluates samples 16 b + col (b = 0..3) against it and holds channel col of its values (the
// B operand); accumulator tile b ends with samples 16 b + 4 kq + r (r = 0..3), channel col.
// The Gaussian rows arrive by vector loads (a 16-lane group shares one row), so neither the
// scalar cache's random-row rate (the lane-per-sample form's bound) nor a per-pass
// re-walk of the list (the transposed form's) is paid.
#ifndef DGS_QFORM
#define DGS_QFORM 1
#endif
#ifndef DGS_FWD_MX
#define DGS_FWD_MX 1
#endif
template <int FN, int D, int CB>
__host__ __device__ constexpr bool fwd_mfma() {
    return DGS_FWD_MX && !is_multi(FN) && CB >= 8;
}

template <int FN, int D, int CB, bool FLAGGED>
__device__ __forceinline__ void fwd_mx_groups(const Bins &bins, const float *__restrict__ grows, int eb, int ee,
                                              int kq, int col, const float (&sx)[4], const float (&sy)[4],
                                              const float *ctr, f32x4_t (&acc)[Traits<FN, D>::U][4]) {
    constexpr int U = Traits<FN, D>::U, RS = grow_stride<FN, D, CB>(), B = Traits<FN, D>::GBASE;
    constexpr int HB = (B + 3) / 4 * 4;  // row head (mean, exponent coefficients, conic) in float4s
    if (eb >= ee) return;
    const int last = ee - 1;
    const float one = 1.0f;
    // software-pipelined: the next step group's rows and the one after's entries are in flight
    // while a group is evaluated (each group otherwise starts with two dependent round trips)
    auto load_ent = [&](int e, uint32_t (&en)[4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) en[t] = bins.entries[min(e + 4 * t + kq, last)];
    };
    auto load_rows = [&](const uint32_t (&en)[4], float (&h)[4][HB], float (&v)[4]) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float *row = grows + (int64_t)(en[t] & kIdMask) * RS;
#pragma unroll
            for (int k = 0; k < HB; k += 4) {
                const float4 q = *reinterpret_cast<const float4 *>(row + k);
                h[t][k] = q.x; h[t][k + 1] = q.y; h[t][k + 2] = q.z; h[t][k + 3] = q.w;
            }
            v[t] = (CB >= 16 || col < CB) ? row[B + (CB >= 16 ? col : min(col, CB - 1))] : 0.0f;
        }
    };
    uint32_t ent[4], ent_n[4];
    float hd[4][HB], vv[4];
    load_ent(eb, ent);
    load_rows(ent, hd, vv);
    load_ent(eb + 16, ent_n);
    for (int e0 = eb; e0 < ee; e0 += 16) {
        float hd_n[4][HB], vv_n[4];
        uint32_t ent_nn[4];
        load_rows(ent_n, hd_n, vv_n);
        load_ent(e0 + 32, ent_nn);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            bool act = e0 + 4 * t + kq < ee;
            float sh[2] = {0.0f, 0.0f};
            if constexpr (FLAGGED) {
                act = act && !(ent[t] & kUnsafe);  // unsafe conics: the tail pass
                if (act && (ent[t] & kGeneral)) {
#pragma unroll
                    for (int d = 0; d < D; ++d) sh[d] = wrap_shift_f(hd[t][d] - ctr[d]);
                }
            }
            float c[3];
            row_conic<FN, D, HB>(hd[t], c);
            const float bv = act ? vv[t] : 0.0f;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                float X[2] = {hd[t][0] - sx[b], D == 2 ? hd[t][1] - sy[b] : 0.0f};
                if constexpr (FLAGGED) {  // fl(m - s) - shift: exact (see fwd_t_pairs)
                    X[0] = X[0] - sh[0];
                    if constexpr (D == 2) X[1] = X[1] - sh[1];
                }
                const float G = fast_prob<D, float>(X, &hd[t][D]);
                float tu[U][1];
#pragma unroll
                for (int u = 0; u < U; ++u) tu[u][0] = 0.0f;
                fwd_terms<FN, D, 1, float>(X, c, G, &one, tu);
#pragma unroll
                for (int u = 0; u < U; ++u)
                    acc[u][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(act ? tu[u][0] : 0.0f, bv, acc[u][b], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int k = 0; k < HB; ++k) hd[t][k] = hd_n[t][k];
            vv[t] = vv_n[t];
            ent[t] = ent_n[t];
            ent_n[t] = ent_nn[t];
        }
    }
}

template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock) void k_forward_mx(const char *__restrict__ gbuf,
                                                       const char *__restrict__ sbuf,
                                                       const float *__restrict__ grows,
                                                       const Outs outs, int C, int cbase,
                                                       const uint32_t *__restrict__ dirty) {
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    constexpr int U = Traits<FN, D>::U;
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumFwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1), col = lane & 15, kq = lane >> 4;
    const int nch = min(CB, C - cbase);
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const FwdUnit fu = fwd_unit_at(bins, unit);
        float sx[4], sy[4];  // samples 16 b + col
#pragma unroll
        for (int b = 0; b < 4; ++b) {  // samples outside the cell: a valid one (not stored)
            int j = fu.sb + 16 * b + col;
            j = (j >= fu.lo && j < fu.hi) ? j : fu.lo;
            const float *pr = bins.fsrows + (int64_t)(j >> 1) * (2 * D) + (j & 1);
            sx[b] = pr[0];
            sy[b] = D == 2 ? pr[2] : 0.0f;
        }
        const int gb = sload(&bins.cell_gbeg[fu.cell]), ge = sload(&bins.cell_gend[fu.cell]);
        const int gm = sload(&bins.cell_gmid[fu.cell]);
        float ctr[2];
        cell_center<D>(bins, fu.cell, ctr);
        f32x4_t acc[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[u][b] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
        fwd_mx_groups<FN, D, CB, false>(bins, grows, gb, gm, kq, col, sx, sy, ctr, acc);
        if (gm < ge) fwd_mx_groups<FN, D, CB, true>(bins, grows, gm, ge, kq, col, sx, sy, ctr, acc);
        if (col < nch) {
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = fu.sb + 16 * b + 4 * kq + r;
                    if (j >= fu.lo && j < fu.hi) {
                        const int64_t sid = bins.sorted_sid[j];
#pragma unroll
                        for (int u = 0; u < U; ++u) store_unique<FN, D, false>(outs, sid, u, C, cbase + col, acc[u][b][r]);
                    }
                }
        }
    }
}

// ------------------------------------------------------------------ backward kernel
// MODE 0: fast path; 1: plus the lane's constant torus-wrap shift sh (kGeneral entries);
// 2: the fully general per-pair path (some lane has a kUnsafe entry).
template <int FN, int D, int CB, int MODE, typename V>
__device__ __forceinline__ void bwd_sample(const V *srow, const float *m, const float *sh,
                                           const float *c, const float *kk, const float *v,
                                           bool wrap, bool unsafe, V *acc) {
    constexpr int U = Traits<FN, D>::U;
    V dl[U][CB];
#pragma unroll
    for (int a = 0; a < U; ++a)
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) dl[a][ch] = srow[D + a * CB + ch];
    V X[2] = {m[0] - srow[0], D == 2 ? m[1] - srow[1] : bc<V>(0.0f)};
    if constexpr (MODE == 1) {
        X[0] = X[0] - sh[0];
        if constexpr (D == 2) X[1] = X[1] - sh[1];
    }
    if constexpr (FN == 0 && D == 2 && CB == 1 && MODE != 2 && DGS_QFORM && DGS_VFACTOR) {
        // gaussian, C = 1: the exponent from the quadratic monomials q = (X0^2, X0 X1, X1^2)
        // that the conic moments need anyway -- 15 packed ops per two pairs instead of 16
        const V q0 = X[0] * X[0], q1 = X[0] * X[1], q2 = X[1] * X[1];
        const V e = vexp2(vfma(bc<V>(kk[2]), q2, vfma(bc<V>(kk[1]), q1, kk[0] * q0)));
        const V t = e * dl[0][0];
        V *gm = acc, *gv = acc + 2, *gc = acc + 3;
        gv[0] += t;
        gm[0] = vfma(t, X[0], gm[0]);
        gm[1] = vfma(t, X[1], gm[1]);
        gc[0] = vfma(t, q0, gc[0]);
        gc[1] = vfma(t, q1, gc[1]);
        gc[2] = vfma(t, q2, gc[2]);
        return;
    }
    V G;
    if constexpr (MODE == 2) G = general_prob<FN, D>(X, c, kk, wrap, unsafe);
    else G = fast_prob<D, V>(X, kk);
    if constexpr (bwd_mom<FN, D, CB>()) bwd_mom_terms<FN, V>(X, c, G, &srow[D], acc);
    else bwd_terms<FN, D, CB, V>(X, c, G, v, dl, acc, acc + 2, acc + 2 + CB);
}

// One sample pair (packed layout) as RSS f2 fields; `drop` = 1 / 2 zeroes the dL fields of the
// first / second sample (a pair straddling the cell boundary: the foreign sample then adds 0).
template <int RSS, int D>
__device__ __forceinline__ void pair_fields(const float *p, f2 (&f)[RSS], int drop) {
#pragma unroll
    for (int k = 0; k < RSS; ++k) {
        float a = p[2 * k], b = p[2 * k + 1];
        if (k >= D) {
            a = drop == 1 ? 0.0f : a;
            b = drop == 2 ? 0.0f : b;
        }
        f[k] = f2{a, b};
    }
}

// The cell's samples [sb, se), wave-uniform through the scalar cache.
//   scalar layout: NB sample rows per batch, then the tail one by one;
//   pair layout  : pairs (2p, 2p+1) covering [sb, se), packed; the boundary pairs are masked.
template <int FN, int D, int CB, int MODE, typename V>
__device__ __forceinline__ void bwd_loop(int sb, int se, const float *__restrict__ srows,
                                         const float *m, const float *sh, const float *c, const float *kk,
                                         const float *v, bool wrap, bool unsafe, V *acc) {
    constexpr int RSS = srow_stride<FN, D, CB>();
    if constexpr (sizeof(V) == 4) {
        constexpr int NB = bwd_batch<RSS>();
        int j0 = sb;
        for (; j0 + NB <= se; j0 += NB) {
            const F32s<NB * RSS> sr = sload_f<NB * RSS>(srows + (int64_t)j0 * RSS);
#pragma unroll
            for (int q = 0; q < NB; ++q)
                bwd_sample<FN, D, CB, MODE, V>(&sr.v[q * RSS], m, sh, c, kk, v, wrap, unsafe, acc);
        }
        for (; j0 < se; ++j0) {
            const F32s<RSS> sr = sload_f<RSS>(srows + (int64_t)j0 * RSS);
            bwd_sample<FN, D, CB, MODE, V>(sr.v, m, sh, c, kk, v, wrap, unsafe, acc);
        }
    } else {
        constexpr int PR = 2 * RSS, NB = bwd_batch<PR>();
        int p = sb >> 1;
        const int pe = (se + 1) >> 1;
        const int pf = (se & 1) ? pe - 1 : pe;  // end of the pairs fully inside [sb, se)
        f2 f[RSS];
        if (sb & 1) {
            const F32s<PR> sr = sload_f<PR>(srows + (int64_t)p * PR);
            pair_fields<RSS, D>(sr.v, f, 1);
            bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
            ++p;
        }
        if constexpr (DGS_BWD_PIPE == 2) {
            // two batch buffers in turn (no register copy of the look-ahead batch per iteration)
            if (p + NB <= pf) {
                const int plast = pf - NB;
                F32s<NB * PR> b0 = sload_f<NB * PR>(srows + (int64_t)p * PR), b1;
                for (;;) {
                    DGS_WAIT_LGKM0();
                    __builtin_amdgcn_sched_barrier(0);
                    b1 = sload_f<NB * PR>(srows + (int64_t)min(p + NB, plast) * PR);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        pair_fields<RSS, D>(&b0.v[q * PR], f, 0);
                        bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    p += NB;
                    if (p + NB > pf) break;
                    DGS_WAIT_LGKM0();
                    __builtin_amdgcn_sched_barrier(0);
                    b0 = sload_f<NB * PR>(srows + (int64_t)min(p + NB, plast) * PR);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        pair_fields<RSS, D>(&b1.v[q * PR], f, 0);
                        bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    p += NB;
                    if (p + NB > pf) break;
                }
                DGS_WAIT_LGKM0();  // (the last look-ahead, unused)
            }
        } else if constexpr (DGS_BWD_PIPE) {
            // The next batch of pair rows is in flight while this one is evaluated.  Scalar loads
            // complete out of order, so each batch is waited for with lgkmcnt(0) BEFORE the next
            // one is issued; scheduling barriers keep the compiler from moving the load across.
            // (The look-ahead address is clamped to the last full batch: always in bounds.)
            if (p + NB <= pf) {
                const int plast = pf - NB;
                F32s<NB * PR> cur = sload_f<NB * PR>(srows + (int64_t)p * PR);
                for (; p + NB <= pf; p += NB) {
                    DGS_WAIT_LGKM0();
                    __builtin_amdgcn_sched_barrier(0);
                    const F32s<NB * PR> nxt = sload_f<NB * PR>(srows + (int64_t)min(p + NB, plast) * PR);
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        pair_fields<RSS, D>(&cur.v[q * PR], f, 0);
                        bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    cur = nxt;
                }
                DGS_WAIT_LGKM0();  // (the last look-ahead, unused)
            }
        } else {
            for (; p + NB <= pf; p += NB) {
                const F32s<NB * PR> sr = sload_f<NB * PR>(srows + (int64_t)p * PR);
#pragma unroll
                for (int q = 0; q < NB; ++q) {
                    pair_fields<RSS, D>(&sr.v[q * PR], f, 0);
                    bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
                }
            }
        }
        for (; p < pf; ++p) {
            const F32s<PR> sr = sload_f<PR>(srows + (int64_t)p * PR);
            pair_fields<RSS, D>(sr.v, f, 0);
            bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
        }
        if (se & 1) {
            const F32s<PR> sr = sload_f<PR>(srows + (int64_t)(pe - 1) * PR);
            pair_fields<RSS, D>(sr.v, f, 2);
            bwd_sample<FN, D, CB, MODE, V>(f, m, sh, c, kk, v, wrap, unsafe, acc);
        }
    }
}

// A lane's register sums -> its finished gradient sums (moment form or v-factored terms).
template <int FN, int D, int CB, typename V>
__device__ __forceinline__ void bwd_finish_sums(const V *ra, const float *c, float vB, float (&sm)[2], float (&sc)[3],
                                                float (&sv)[CB]) {
    if constexpr (bwd_mom<FN, D, CB>()) {
        float sum[kMomAcc];
#pragma unroll
        for (int k = 0; k < kMomAcc; ++k) sum[k] = hsum(ra[k]);
        bwd_mom_finish(c, vB, sum, sm, sc, sv[0]);
    } else {
        const V *gm = ra, *gv = ra + 2, *gc = ra + 2 + CB;
        sm[0] = hsum(gm[0]); sm[1] = hsum(gm[1]);
#pragma unroll
        for (int k = 0; k < 3; ++k) sc[k] = hsum(gc[k]);
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) sv[ch] = hsum(gv[ch]);
        if constexpr (FN == 0 && CB == 1 && DGS_VFACTOR) {  // v-factored moments (bwd_terms)
#pragma unroll
            for (int d = 0; d < 2; ++d) sm[d] *= vB;
#pragma unroll
            for (int k = 0; k < 3; ++k) sc[k] *= vB;
        }
        bwd_finish<FN, D>(c, sm, sc);
    }
}

// The gradient sums of one lane's Gaussian (entry ent, row r, conic cr) over the samples
// [sb, se) of `cell` (sorted order), finished into sm[D], sc[S], sv[CB].  The mode (fast /
// constant wrap shift / general) is chosen for the whole wave from its active lanes' flags.
template <int FN, int D, int CB>
__device__ __forceinline__ void bwd_sums(const Bins &bins, const float *__restrict__ srows, int cell, int sb, int se,
                                         uint32_t ent, bool active, const float (&r)[grow_stride<FN, D, CB>()],
                                         float4 cr, float (&sm)[2], float (&sc)[3], float (&sv)[CB]) {
    using Tr = Traits<FN, D>;
    using V = typename std::conditional<pair_rows<FN, D, CB>(), f2, float>::type;
    constexpr int B = Tr::GBASE;
    const bool wrap = (ent & kGeneral) != 0;
    const bool unsafe = (ent & kUnsafe) != 0;  // (mode 2: the literal power)
    const float c[3] = {cr.x, cr.y, cr.z};
    const float m[2] = {r[0], D == 2 ? r[1] : 0.0f};
    // register accumulators: [gm(2) gv(CB) gc(3)], or the kMomAcc sums of the moment form
    constexpr int NA = bwd_mom<FN, D, CB>() ? kMomAcc : 2 + CB + 3;
    V ra[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) ra[k] = bc<V>(0.0f);
    float sh[2] = {0.0f, 0.0f};
    if (__any(active && (ent & kUnsafe))) {
        bwd_loop<FN, D, CB, 2, V>(sb, se, srows, m, sh, c, &r[D], &r[B], wrap, unsafe, ra);
    } else if (__any(active && wrap)) {
        if (active && wrap) {
            float ctr[2];
            cell_center<D>(bins, cell, ctr);
#pragma unroll
            for (int d = 0; d < D; ++d) sh[d] = wrap_shift_f(m[d] - ctr[d]);
        }
        bwd_loop<FN, D, CB, 1, V>(sb, se, srows, m, sh, c, &r[D], &r[B], false, false, ra);
    } else {
        bwd_loop<FN, D, CB, 0, V>(sb, se, srows, m, sh, c, &r[D], &r[B], false, false, ra);
#ifdef DGS_TIMING_TWICE  // (timing build only: the pair loop twice -- its cost by difference)
        bwd_loop<FN, D, CB, 0, V>(sb, se, srows, m, sh, c, &r[D], &r[B], false, false, ra);
#endif
    }
    bwd_finish_sums<FN, D, CB, V>(ra, c, r[B], sm, sc, sv);
}

// The slot row width of a Gaussian's sums (k_bwd_esum): [dm(D) dc(S) dv(CB)] padded to 2 floats
// (8-byte pieces: 24-byte rows at D = 2, C = 1, where 4-float padding wrote and read 32).
template <int FN, int D, int CB>
__host__ __device__ constexpr int esum_stride() {
    return (D + Traits<FN, D>::S + CB + 1) / 2 * 2;
}

// DGS_BWD_STAMPS builds (tuning only): per-unit wave-time sums of k_backward's phases (s_memtime,
// lane 0 of each wave): [0] setup (unit, entry, rows landed), [1] the pair loop and the finish,
// [2] the stores / atomics, [3] units; read back with dgs_debug_bwd_stamps.
#ifndef DGS_BWD_STAMPS
#define DGS_BWD_STAMPS 0
#endif
#if DGS_BWD_STAMPS
constexpr int kStampCopies = 1024;  // (one word per slot took every wave's atomics: ~88 per us)
__device__ unsigned long long g_bwd_stamps[kStampCopies][8];
#define BWD_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define BWD_ADD(slot, a, b) \
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_bwd_stamps[blockIdx.x % kStampCopies][slot], (unsigned long long)((b) - (a)))
#else
#define BWD_STAMP(v)
#define BWD_ADD(slot, a, b)
#endif

// A lane's finished sums for list position pos (Gaussian id): sort-path entries (the sorted part
// of the list: scattered ids, one cache line per lane and atomic) store them in their
// Gaussian-major slot (k_bwd_esum adds them up); the others add them with one atomic each.
template <int FN, int D, int CB>
__device__ __forceinline__ void bwd_store(const Bins &bins, float *__restrict__ acc, int P, int vrow0, int cell, int pos,
                                          int64_t id, bool active, const float (&sm)[2], const float (&sc)[3],
                                          const float (&sv)[CB], float *__restrict__ esums) {
    constexpr int S = Traits<FN, D>::S, SSW = esum_stride<FN, D, CB>();
    const bool slot = esums != nullptr && pos >= sload(&bins.cell_gsort[cell]);
    if (active && slot) {
        float row[SSW];
#pragma unroll
        for (int k = 0; k < SSW; ++k) row[k] = 0.0f;
#pragma unroll
        for (int d = 0; d < D; ++d) row[d] = sm[d];
#pragma unroll
        for (int k = 0; k < S; ++k) row[D + k] = sc[k];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) row[D + S + ch] = sv[ch];
        float2 *o = reinterpret_cast<float2 *>(esums + (int64_t)bins.esum_q[pos] * SSW);
#pragma unroll
        for (int k = 0; k < SSW / 2; ++k) o[k] = make_float2(row[2 * k], row[2 * k + 1]);
    } else if (active) {
#pragma unroll
        for (int d = 0; d < D; ++d) atomicAdd(acc + (int64_t)d * P + id, sm[d]);
#pragma unroll
        for (int k = 0; k < S; ++k) atomicAdd(acc + (int64_t)(D + k) * P + id, sc[k]);
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) atomicAdd(acc + (int64_t)(vrow0 + ch) * P + id, sv[ch]);
    }
}

// One backward unit: (cell, <= 64 entries of its list), lane = Gaussian (entry ent, row r,
// conic cr), the cell's samples wave-uniform; one atomicAdd per gradient component per lane
// (a slot store for the sorted part, below).
template <int FN, int D, int CB>
__device__ __forceinline__ void bwd_unit(const Bins &bins, const float *__restrict__ srows,
                                         float *__restrict__ acc, int P, int vrow0, uint2 u,
                                         uint32_t ent, const float (&r)[grow_stride<FN, D, CB>()],
                                         float4 cr, int lane, float *__restrict__ esums) {
    const int cell = (int)u.x, eb = (int)u.y;
    const int ee = min(eb + kWave, sload(&bins.cell_gend[cell]));
    const bool active = eb + lane < ee;
    const int64_t id = ent & kIdMask;
    const int sb = sload(&bins.cell_sbeg[cell]), se = sload(&bins.cell_send[cell]);
    float sm[2], sc[3], sv[CB];
#if DGS_BWD_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    BWD_STAMP(ts1);
    bwd_sums<FN, D, CB>(bins, srows, cell, sb, se, ent, active, r, cr, sm, sc, sv);
#if DGS_BWD_PRIO > 1
    __builtin_amdgcn_s_setprio(3);  // (2: the finish and the atomics too -- the wave's slot frees sooner)
#endif
    BWD_STAMP(ts2);
    BWD_ADD(1, ts1, ts2);
    bwd_store<FN, D, CB>(bins, acc, P, vrow0, cell, eb + lane, id, active, sm, sc, sv, esums);
#if DGS_BWD_STAMPS
#if DGS_BWD_STAMPS > 1  // (2: wait for the atomics too -- they are fire-and-forget otherwise)
    __builtin_amdgcn_s_waitcnt(0);
#endif
    BWD_STAMP(ts3);
    BWD_ADD(2, ts2, ts3);
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_bwd_stamps[blockIdx.x % kStampCopies][3], 1ull);
#endif
}

// The lane's entry of unit u (clamped to the unit's last entry for padding lanes).
#ifndef DGS_BWD_ENTRY_FREE
#define DGS_BWD_ENTRY_FREE 0  // 1: clamp to the list end E instead (no wait for cell_gend first)
#endif
__device__ __forceinline__ uint32_t bwd_entry(const Bins &bins, uint2 u, int lane) {
#if DGS_BWD_ENTRY_FREE
    // (padding lanes read the next cells' entries: valid rows, never stored -- bwd_unit's `active`)
    return bins.entries[min((int64_t)u.y + lane, sload(&bins.h->E) - 1)];
#else
    const int ee = min((int)u.y + kWave, sload(&bins.cell_gend[u.x]));
    return bins.entries[min((int)u.y + lane, ee - 1)];
#endif
}

// One wave per unit (exact grid from the preprocess hint; grid-strided otherwise).  A
// persistent, software-pipelined form (rows of unit k + 1 in flight during unit k) measured
// 5-15 % slower: the hardware's dynamic wave dispatch balances the uneven units better.
template <int FN, int D, int CB>
#ifndef DGS_BWD_WAVES
#define DGS_BWD_WAVES 5  // (launch bound: >= 5 waves per SIMD, <= 96 VGPRs; the kernel holds 68: 7 waves)
#endif
__global__ __launch_bounds__(kBlock, DGS_BWD_WAVES) void k_backward(const char *__restrict__ gbuf,
                                                     const char *__restrict__ sbuf,
                                                     const float *__restrict__ grows,
                                                     const float *__restrict__ srows,
                                                     float *__restrict__ acc, int P, int vrow0,
                                                     const uint32_t *__restrict__ dirty, float *__restrict__ esums) {
#if DGS_BWD_PRIO > 2
    __builtin_amdgcn_s_setprio(3);  // (3: from the kernel's entry, its header loads included)
#endif
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    constexpr int RS = grow_stride<FN, D, CB>();
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumBwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1);
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        BWD_STAMP(ts0);
#if DGS_BWD_PRIO
        __builtin_amdgcn_s_setprio(3);  // (the unit's loads issue first; bwd_unit drops it again)
#endif
        const uint2 u = sload(&bins.bwd_units[unit]);
        const uint32_t ent = bwd_entry(bins, u, lane);
        float r[RS];
        load_grow<RS>(grows, ent, r);
#if DGS_BWD_STAMPS
        __builtin_amdgcn_s_waitcnt(0);
        BWD_STAMP(tsl);
        BWD_ADD(0, ts0, tsl);
#endif
        bwd_unit<FN, D, CB>(bins, srows, acc, P, vrow0, u, ent, r, bins.gcon[ent & kIdMask], lane, esums);
    }
}

// (b) Matrix-core backward (gaussian, D = 2, CB = 16: BASELINE config 2's C = 16).  Per pair
// (s, g) the gaussian backward is
//   dL/dG = sum_c dl[s][c] v[g][c]                      (16 MACs: a [samples x channels] x
//                                                          [channels x Gaussians] product)
//   dv[g][c] += G dl[s][c]                              (16 MACs: [channels x samples] x
//                                                          [samples x Gaussians])
//   moments of t = G dL/dG over X, X X^T                (the VALU: exponent, exp, 5 FMAs)
// In k_backward both contractions run on the VALU: ~32 of the ~47 operations per pair.  Here
// they run on v_mfma_f32_16x16x4_f32 (exact f32: an fmaf chain), beside the VALU work of other
// waves and of the wave's own next step (separate pipes, MI355X_MICROARCH.md).
// A wave takes a unit's entries 16 at a time: lane (q = lane >> 4, col = lane & 15) holds
// Gaussian col, and a 16-sample step gives it samples 4q + i (i = 0..3) -- the C/D layout of
// the first product, whose K index runs over the channels c = 4q + j of the operands' 4
// steps j.  The second product's K index (samples) is then taken as s = 4q + j, so its B
// operand of step j is exactly register j of the VALU's G: no cross-lane movement per pair.
// Its result leaves dv[c = 4q + i][col] in register i.  MODE as in k_backward: 0 fast, 1 the
// lanes' constant wrap shifts, 2 some entry of the unit is unsafe (the literal power, per pair).
#ifndef DGS_BWD_MX
#define DGS_BWD_MX 1
#endif
template <int FN, int D, int CB>
__host__ __device__ constexpr bool bwd_mfma() {
    return DGS_BWD_MX && FN == 0 && D == 2 && CB == 16;
}

#ifndef DGS_BWD_MX_NG
#define DGS_BWD_MX_NG 4  // 16-entry groups per pass over the samples (4: the whole unit at once)
#endif

// One 16-sample step's operands of lane (q, col): samples s0 + 4q + i (position; dl[.][col], the
// second product's A) and sample s0 + col (dl[.][4q + j], the first product's A).  Rows past the
// cell are the next cell's, or k_pack_samples' zero rows past N: finite, and their G is 0.
struct MxStep {
    float2 xy[4];
    float a2[4];
    float2 a1[2];
};
template <int D>
__device__ __forceinline__ void mx_load(const float *__restrict__ ps, const float *__restrict__ pc, int col, int rss,
                                        MxStep &st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        st.xy[i] = *reinterpret_cast<const float2 *>(ps + i * rss);
        st.a2[i] = ps[i * rss + D + col];
    }
    st.a1[0] = reinterpret_cast<const float2 *>(pc)[0];
    st.a1[1] = reinterpret_cast<const float2 *>(pc)[1];
}

// Entries [eg, eg + 16 NG) of the unit (clamped to ee - 1; lanes past ee are not stored).
template <int FN, int D, int CB, int NG, int MODE>
__device__ __forceinline__ void bwd_mx_pass(const Bins &bins, const float *__restrict__ grows,
                                            const float *__restrict__ srows, float *__restrict__ acc, int P,
                                            int vrow0, int cell, int sb, int se, int eg, int ee, int q, int col,
                                            const float *ctr, float *__restrict__ esums) {
    constexpr int RSS = srow_stride<FN, D, CB>(), RS = grow_stride<FN, D, CB>(), B = Traits<FN, D>::GBASE;
    constexpr int S = Traits<FN, D>::S, SSW = esum_stride<FN, D, CB>();
    static_assert(D == 2 && CB == 16 && RS % 4 == 0 && RSS % 2 == 0, "matrix-core backward layout");
    int pos[NG];
    uint32_t ent[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        pos[g] = min(eg + 16 * g + col, ee - 1);
        ent[g] = bins.entries[pos[g]];
    }
    float4 hd[NG];  // m0 m1 k0 k1
    float k2[NG], bv[NG][4], sh0[NG], sh1[NG];  // bv: the first product's B, step j: v[col][4q + j]
    float4 cr[NG];  // raw conics (the finish; MODE 2: the literal power)
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const float *grow = grows + (int64_t)(ent[g] & kIdMask) * RS;
        hd[g] = *reinterpret_cast<const float4 *>(grow);
        k2[g] = grow[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[g][j] = grow[B + 4 * q + j];
        if constexpr (MODE == 2) cr[g] = bins.gcon[ent[g] & kIdMask];
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        sh0[g] = sh1[g] = 0.0f;
        if constexpr (MODE == 1) {
            if (ent[g] & kGeneral) {
                sh0[g] = wrap_shift_f(hd[g].x - ctr[0]);
                sh1[g] = wrap_shift_f(hd[g].y - ctr[1]);
            }
        }
    }
    float mom[NG][5];  // sum t X0, t X1, t X0^2, t X0 X1, t X1^2
    f32x4_t gv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int k = 0; k < 5; ++k) mom[g][k] = 0.0f;
        gv[g] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
    }
    const float *ps = srows + (int64_t)(sb + 4 * q) * RSS;
    const float *pc = srows + (int64_t)(sb + col) * RSS + D + 4 * q;
    MxStep cur, nxt;
    mx_load<D>(ps, pc, col, RSS, cur);
#ifdef DGS_TIMING_TWICE  // (timing build only: the step loop twice -- its cost by difference)
    for (int rep = 0; rep < 2; ++rep) {
    ps = srows + (int64_t)(sb + 4 * q) * RSS;
    pc = srows + (int64_t)(sb + col) * RSS + D + 4 * q;
    mx_load<D>(ps, pc, col, RSS, cur);
#endif
    for (int base = sb; base < se; base += 16) {
        ps += 16 * RSS;
        pc += 16 * RSS;
        if (base + 16 < se) mx_load<D>(ps, pc, col, RSS, nxt);  // (the next step's rows in flight)
        const float a1[4] = {cur.a1[0].x, cur.a1[0].y, cur.a1[1].x, cur.a1[1].y};
        f32x4_t dg[NG];  // dL/dG of (sample base + 4q + i, Gaussian col of group g)
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            dg[g] = f32x4_t{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < 4; ++j) dg[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], bv[g][j], dg[g], 0, 0, 0);
        }
        bool ok[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) ok[i] = base + 4 * q + i < se;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            float G[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float X0 = hd[g].x - cur.xy[i].x, X1 = hd[g].y - cur.xy[i].y;
                if constexpr (MODE == 1) {  // fl(m - s) - shift: exact (see fwd_t_pairs)
                    X0 = X0 - sh0[g];
                    X1 = X1 - sh1[g];
                }
                float e;
                if constexpr (MODE == 2) {  // (the reference's wrap of X and, for unsafe conics, its power)
                    float X[2] = {X0, X1};
                    const float c[3] = {cr[g].x, cr[g].y, cr[g].z}, kk[3] = {hd[g].z, hd[g].w, k2[g]};
                    e = general_prob<FN, D>(X, c, kk, (ent[g] & kGeneral) != 0, (ent[g] & kUnsafe) != 0);
                    X0 = X[0];
                    X1 = X[1];
                }
                const float q0 = X0 * X0, q1 = X0 * X1, q2 = X1 * X1;
                if constexpr (MODE != 2) e = fast_exp2(fmaf(k2[g], q2, fmaf(hd[g].w, q1, hd[g].z * q0)));
                G[i] = ok[i] ? e : 0.0f;
                const float t = G[i] * dg[g][i];
                mom[g][0] = fmaf(t, X0, mom[g][0]);
                mom[g][1] = fmaf(t, X1, mom[g][1]);
                mom[g][2] = fmaf(t, q0, mom[g][2]);
                mom[g][3] = fmaf(t, q1, mom[g][3]);
                mom[g][4] = fmaf(t, q2, mom[g][4]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) gv[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur.a2[j], G[j], gv[g], 0, 0, 0);
        }
        cur = nxt;
    }
#ifdef DGS_TIMING_TWICE
    }
#endif
    const int gsort = esums != nullptr ? sload(&bins.cell_gsort[cell]) : 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        // the moments over the four sample quarters (lanes col + 16 q), then the gradient sums
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            mom[g][k] += __shfl_xor(mom[g][k], 16);
            mom[g][k] += __shfl_xor(mom[g][k], 32);
        }
        const int64_t id = ent[g] & kIdMask;
        if constexpr (MODE != 2) cr[g] = bins.gcon[id];
        const float c[3] = {cr[g].x, cr[g].y, cr[g].z};
        float sm[2] = {mom[g][0], mom[g][1]}, sc[3] = {mom[g][2], mom[g][3], mom[g][4]};
        bwd_finish<FN, D>(c, sm, sc);
        if (eg + 16 * g + col >= ee) continue;
#ifdef DGS_TIMING_NO_STORE  // (timing build only: no stores -- their cost by difference)
        if (sm[0] != 1.2345e-30f) continue;
#endif
        if (esums != nullptr && pos[g] >= gsort) {  // (the row of bwd_store: [dm dc dv pad])
            float *o = esums + (int64_t)bins.esum_q[pos[g]] * SSW;
            if (q == 0) {
                o[0] = sm[0]; o[1] = sm[1];
#pragma unroll
                for (int k = 0; k < S; ++k) o[D + k] = sc[k];
                if constexpr (SSW > D + S + CB) o[SSW - 1] = 0.0f;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) o[D + S + 4 * q + i] = gv[g][i];
        } else {
            if (q == 0) {
#pragma unroll
                for (int d = 0; d < D; ++d) atomicAdd(acc + (int64_t)d * P + id, sm[d]);
#pragma unroll
                for (int k = 0; k < S; ++k) atomicAdd(acc + (int64_t)(D + k) * P + id, sc[k]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) atomicAdd(acc + (int64_t)(vrow0 + 4 * q + i) * P + id, gv[g][i]);
        }
    }
}

#ifndef DGS_BWD_MX_WAVES
#define DGS_BWD_MX_WAVES 3  // (launch bound: >= 3 waves per SIMD, <= 168 VGPRs; 2 waves at the free allocation: +9 %)
#endif
template <int FN, int D, int CB>
__global__ __launch_bounds__(kBlock, DGS_BWD_MX_WAVES) void k_backward_mx(const char *__restrict__ gbuf, const char *__restrict__ sbuf,
                                                        const float *__restrict__ grows,
                                                        const float *__restrict__ srows, float *__restrict__ acc,
                                                        int P, int vrow0, const uint32_t *__restrict__ dirty,
                                                        float *__restrict__ esums) {
    if (sload(dirty)) return;  // call-time tensors differ from the binned ones: dgs_reference.hip
    constexpr int NG = DGS_BWD_MX_NG;
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumBwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    const int lane = threadIdx.x & (kWave - 1), q = lane >> 4, col = lane & 15;
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const uint2 u = sload(&bins.bwd_units[unit]);
        const int cell = (int)u.x, eb = (int)u.y;
        const int ee = min(eb + kWave, sload(&bins.cell_gend[cell]));
        const uint32_t ent = bwd_entry(bins, u, lane);
        const bool active = eb + lane < ee;
        const int sb = sload(&bins.cell_sbeg[cell]), se = sload(&bins.cell_send[cell]);
        if (__any(active && (ent & kUnsafe))) {
            for (int eg = eb; eg < ee; eg += 16)  // (one group at a time: the general path's registers)
                bwd_mx_pass<FN, D, CB, 1, 2>(bins, grows, srows, acc, P, vrow0, cell, sb, se, eg, ee, q, col, nullptr,
                                             esums);
        } else if (__any(active && (ent & kGeneral))) {
            float ctr[2];
            cell_center<D>(bins, cell, ctr);
            for (int eg = eb; eg < ee; eg += 16 * NG)
                bwd_mx_pass<FN, D, CB, NG, 1>(bins, grows, srows, acc, P, vrow0, cell, sb, se, eg, ee, q, col, ctr,
                                              esums);
        } else {
            for (int eg = eb; eg < ee; eg += 16 * NG)
                bwd_mx_pass<FN, D, CB, NG, 0>(bins, grows, srows, acc, P, vrow0, cell, sb, se, eg, ee, q, col, nullptr,
                                              esums);
        }
    }
}

// The sort-path entries' sums (k_backward's slots), per Gaussian in slot order -- its entries'
// order of k_fine_fill -- added to the atomics' sums (plain adds: k_backward has finished).
// (kEsumLanes lanes per Gaussian stride over its slots, slot rows side by side, then a
// shuffle reduction: one thread per Gaussian walked ~24 rows serially in thin fields)
constexpr int kEsumLanes = 8;
template <int FN, int D, int CB>
__global__ void k_bwd_esum(int P, const char *__restrict__ gbuf, const float *__restrict__ esums,
                           float *__restrict__ acc, int vrow0, const uint32_t *__restrict__ dirty) {
    if (sload(dirty)) return;  // (k_backward wrote no slot)
    constexpr int S = Traits<FN, D>::S, SSW = esum_stride<FN, D, CB>();
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = t / kEsumLanes;
    const int sub = (int)(t & (kEsumLanes - 1));
    const Header *h = reinterpret_cast<const Header *>(gbuf);
    const uint32_t *goff = reinterpret_cast<const uint32_t *>(gbuf + h->o_goff);
    uint32_t q0 = 0, q1 = 0;
    if (i < P) {
        q0 = goff[i];
        q1 = goff[i + 1];
    }
    float sum[SSW];
#pragma unroll
    for (int k = 0; k < SSW; ++k) sum[k] = 0.0f;
    for (uint32_t q = q0 + sub; q < q1; q += kEsumLanes) {
        const float2 *rw = reinterpret_cast<const float2 *>(esums + (int64_t)q * SSW);
#pragma unroll
        for (int k = 0; k < SSW / 2; ++k) {
            const float2 x = rw[k];
            sum[2 * k] += x.x; sum[2 * k + 1] += x.y;
        }
    }
#pragma unroll
    for (int off = kEsumLanes / 2; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < SSW; ++k) sum[k] += __shfl_xor(sum[k], off);
    if (i >= P || sub != 0 || q0 >= q1) return;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[(int64_t)d * P + i] += sum[d];
#pragma unroll
    for (int k = 0; k < S; ++k) acc[(int64_t)(D + k) * P + i] += sum[D + k];
#pragma unroll
    for (int ch = 0; ch < CB; ++ch) acc[(int64_t)(vrow0 + ch) * P + i] += sum[D + S + ch];
}

// Internal (spatial) order -> caller order: thread = caller id g gathers its six sums from
// internal index inv[g] (the stores are coalesced; scattered 4-byte stores were 2-3x slower).
__global__ void k_finalize(int P, int D, int C, const char *__restrict__ gbuf,
                           const float *__restrict__ acc, float *__restrict__ dmeans,
                           float *__restrict__ dvalues, float *__restrict__ dconics) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= P) return;
    const Header *h = reinterpret_cast<const Header *>(gbuf);
    const int32_t *inv = reinterpret_cast<const int32_t *>(gbuf + h->o_perm) + P;
    const int64_t i = inv[g];
    const int S = D * (D + 1) / 2;
    for (int d = 0; d < D; ++d) dmeans[g * D + d] = acc[(int64_t)d * P + i];
    for (int k = 0; k < S; ++k) dconics[g * S + k] = acc[(int64_t)(D + k) * P + i];
    for (int ch = 0; ch < C; ++ch) dvalues[g * C + ch] = acc[(int64_t)(D + S + ch) * P + i];
}

// D = 2, C = 1: the six sums go through an AoS row per Gaussian (internal order, coalesced
// transpose), then each caller id gathers one 32-byte row: 1 random sector per Gaussian
// instead of 6 (k_finalize, 75 us at 1M Gaussians, was bound by those random sectors).
__global__ void k_soa_to_rows(int P, const float *__restrict__ acc, float4 *__restrict__ rows) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    rows[2 * i] = make_float4(acc[i], acc[P + i], acc[2 * (int64_t)P + i], acc[3 * (int64_t)P + i]);
    rows[2 * i + 1] = make_float4(acc[4 * (int64_t)P + i], acc[5 * (int64_t)P + i], 0.0f, 0.0f);
}

__global__ void k_finalize_rows(int P, const char *__restrict__ gbuf, const float4 *__restrict__ rows,
                                float *__restrict__ dmeans, float *__restrict__ dvalues,
                                float *__restrict__ dconics) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= P) return;
    const Header *h = reinterpret_cast<const Header *>(gbuf);
    const int64_t i = (reinterpret_cast<const int32_t *>(gbuf + h->o_perm) + P)[g];
    const float4 a = rows[2 * i], b = rows[2 * i + 1];
    dmeans[2 * g] = a.x;
    dmeans[2 * g + 1] = a.y;
    dconics[3 * g] = a.z;
    dconics[3 * g + 1] = a.w;
    dconics[3 * g + 2] = b.x;
    dvalues[g] = b.y;
}

// ------------------------------------------------------------- diagnostic pair count
template <int D>
__global__ __launch_bounds__(kBlock) void k_count(const char *__restrict__ gbuf,
                                                  const char *__restrict__ sbuf,
                                                  const float *__restrict__ grows,
                                                  const float *__restrict__ samples, float thr,
                                                  unsigned long long *__restrict__ counts) {
    constexpr int RS = grow_stride<0, D, 1>();
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumFwdUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const FwdUnit fu = fwd_unit_at(bins, unit);
        const int gb = sload(&bins.cell_gbeg[fu.cell]), ge = sload(&bins.cell_gend[fu.cell]);
        const int j = fu.sb + (threadIdx.x & (kWave - 1));
        const bool active = j >= fu.lo && j < fu.hi;
        const int64_t sid = bins.sorted_sid[active ? j : fu.lo];
        const float s0 = samples[sid * D], s1 = D == 2 ? samples[sid * D + 1] : 0.0f;
        unsigned long long live = 0;
        for (int e = gb; e < ge; ++e) {
            const int64_t id = sload(&bins.entries[e]) & kIdMask;
            const float *row = grows + id * RS;
            const float4 cr = sload(&bins.gcon[id]);
            const float c[3] = {cr.x, cr.y, cr.z};
            float X[2] = {ref_wrap(sload(row) - s0), D == 2 ? ref_wrap(sload(row + 1) - s1) : 0.0f};
            const float p = ref_power<0, D>(X, c);
            live += (p >= thr && p <= 0.0f) ? 1ull : 0ull;
        }
        if (active) {
            atomicAdd(&counts[0], (unsigned long long)(ge - gb));
            atomicAdd(&counts[1], live);
        }
    }
}

// W_cand / W_live over the sub lists (D = 2, k_forward_s): per sub unit, every sample of the unit
// against every entry of its sub list (the kUnsafe entries of the cell are the tail pass's, a
// handful, not counted).
__global__ __launch_bounds__(kBlock) void k_count_s(const char *__restrict__ gbuf, const char *__restrict__ sbuf,
                                                    const float *__restrict__ grows,
                                                    const float *__restrict__ samples, float thr,
                                                    unsigned long long *__restrict__ counts) {
    constexpr int RS = grow_stride<0, 2, 1>();
    const Bins bins = resolve(gbuf, sbuf);
    const int nunits = sload(&bins.counts[kNumFwdSubUnits]);
    const int stride = gridDim.x * kWavesPerBlock;
    for (int unit = wave_unit_index(nunits); unit < nunits; unit += stride) {
        const uint2 u = sload(&bins.fsub_units[unit]);
        const int sc = (int)u.x, sb = (int)u.y;
        const int lo = max(sb, sload(&bins.sub_sbeg[sc])), hi = min(sb + 2 * kSubPairs, sload(&bins.sub_send[sc]));
        const int gb = sload(&bins.sub_lbeg[sc]), ge = sload(&bins.sub_lend[sc]);
        const int j = sb + (threadIdx.x & (kWave - 1));
        const bool active = j >= lo && j < hi;
        const int64_t sid = bins.sorted_sid[active ? j : lo];
        const float s0 = samples[sid * 2], s1 = samples[sid * 2 + 1];
        unsigned long long live = 0, cand = 0;
        for (int e = gb; e < ge; ++e) {
            const uint32_t ent = sload(&bins.sub_ent[e]);
            if (ent & kUnsafe) continue;
            const int64_t id = ent & kIdMask;
            const float *row = grows + id * RS;
            const float4 cr = sload(&bins.gcon[id]);
            const float c[3] = {cr.x, cr.y, cr.z};
            float X[2] = {ref_wrap(sload(row) - s0), ref_wrap(sload(row + 1) - s1)};
            const float p = ref_power<0, 2>(X, c);
            live += (p >= thr && p <= 0.0f) ? 1ull : 0ull;
            ++cand;
        }
        if (active) {
            atomicAdd(&counts[0], cand);
            atomicAdd(&counts[1], live);
        }
    }
}

// ------------------------------------------------------------------ kernel timing
// Optional HIP-event brackets around the render kernels (bench.py: the dominant kernel's
// average duration on the stream it runs on).  Off by default.
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_tev[2];

struct KernelTimer {
    int which;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(int w, hipStream_t st, uint32_t opts) : which(w), s(st) {
        if (opts & DGS_SAMPLE_GRAPH_CAPTURE) return;  // (no events inside a captured graph)
        std::lock_guard<std::mutex> lk(g_tmu);
        if (!g_timing) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { a = b = nullptr; return; }
        (void)hipEventRecord(a, s);
    }
    ~KernelTimer() {
        if (!a) return;
        (void)hipEventRecord(b, s);
        std::lock_guard<std::mutex> lk(g_tmu);
        g_tev[which].push_back({a, b});
    }
};

// ------------------------------------------------------------------ host dispatch
static int channel_block(int C) { return C <= 1 ? 1 : C <= 2 ? 2 : C <= 4 ? 4 : C <= 8 ? 8 : 16; }
static int grow_stride_rt(int FN, int D, int CB) {
    const bool conic = (fn_mask(FN) & ~1) != 0;
    const int base = D == 2 ? (conic ? 8 : 5) : (conic ? 3 : 2);
    return (base + CB + 3) / 4 * 4;
}
static int srow_stride_rt(int FN, int D, int CB) {
    const int M = fn_mask(FN);
    return is_multi(FN) ? (D + mask_sum(M, D, 2) + 3) / 4 * 4 : (D + mask_sum(M, D, 1) * CB + 3) / 4 * 4;
}
static size_t a256(size_t x) { return align_up(x, 256); }

struct WsLayout {
    size_t grows, srows, acc, flag, total;  // flag: 256 B after the sums (the call's input check)
};
static WsLayout ws_layout(int FN, int P, int D, int N, int C, bool backward) {
    const int CB = channel_block(C), nblk = (C + CB - 1) / CB;
    WsLayout w;
    w.grows = a256((size_t)P * grow_stride_rt(FN, D, CB) * 4 + 64);
    // pair rows: N rounded up to even; scalar rows: kSrowPad zero rows after the last
    w.srows = backward ? a256(((size_t)N + kSrowPad) * srow_stride_rt(FN, D, CB) * 4 + 64) : 0;
    w.acc = backward ? a256((size_t)(D + D * (D + 1) / 2 + nblk * CB) * P * 4) : 0;
    w.flag = w.grows + w.srows + w.acc;
    w.total = w.flag + 256;
    return w;
}

// The backward's slot-sum region (k_bwd_esum), behind the workspace layout: wanted where the
// binning's sort path holds >= 1/4 of the entries (thin fields: ~70 %; the headline: 2 %, where the
// slot pass costs more than the scattered atomics it replaces), for one channel block (the sums
// of a multi-block C accumulate over the blocks: atomics).  The caller provides it by sizing the
// workspace with dgs_sample_workspace_size_binned; a smaller workspace takes the atomics.
static size_t slot_region_bytes(int FN, int D, int C, const void *gb, size_t gbytes, const void *sb, size_t sbytes) {
    UnitHint h;
    const int CB = channel_block(C);
    if (C > CB || !hint_get(gb, gbytes, sb, sbytes, &h) || h.Es <= 0 || 4 * h.Es < h.E) return 0;
    const int S = D * (D + 1) / 2;
    (void)FN;
    return a256(sizeof(float) * (size_t)((D + S + CB + 1) / 2 * 2) * (size_t)h.Es);  // (esum_stride)
}

// Grid size in blocks: exact (from the preprocess hint) or a persistent-size fallback; the
// kernels grid-stride over the device-side unit count either way.
static unsigned unit_blocks(const void *gb, size_t gbytes, const void *sb, size_t sbytes, bool bwd,
                            int units_per_block = kWavesPerBlock, bool sub = false) {
    UnitHint h;
    int64_t units;
    if (hint_get(gb, gbytes, sb, sbytes, &h)) {
        units = sub ? h.nfsub : bwd ? h.nbwd : h.nfwd;
    } else {
        units = 256 * 8 * kWavesPerBlock;  // 8 blocks per CU, striding
    }
    int64_t blocks = (units + units_per_block - 1) / units_per_block;
    static const int64_t cap = [] {  // DGS_BLOCKS_PER_CU: persistent grid (tuning)
        const char *e = std::getenv("DGS_BLOCKS_PER_CU");
        return e ? (int64_t)std::atoi(e) * 256 : (int64_t)0;
    }();
    if (cap > 0 && blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    if (blocks > (1 << 30)) blocks = 1 << 30;
    return (unsigned)blocks;
}

struct Call {
    int FN, P, D, N, C;
    uint32_t opts;  // dgs_sample_flag bits
    const float *means, *values, *conics, *samples;
    DLs dls;
    const char *gb, *sb;
    size_t gbytes, sbytes;
    Outs outs;
    float *dm, *dv, *dc;
    char *ws;
    size_t wsbytes;
    hipStream_t s;
    int debug;
};

// The call-time path's arguments (dgs_reference.h).
// cbox: the workspace's Gaussian-row region (>= 16 P bytes), idle on the call-time path.
static RefCall ref_call(const Call &a, float *acc, const uint32_t *flag, int cbase, float *cbox) {
    UnitHint h;
    const int64_t R = hint_get(a.gb, a.gbytes, a.sb, a.sbytes, &h) ? h.R : (int64_t)1 << 40;
    return RefCall{a.gb, a.sb, a.means, a.values, a.conics, a.samples, a.dls, a.outs, acc, flag,
                   a.P, a.N, a.C, cbase, R, a.s, a.debug, reinterpret_cast<float4 *>(cbox)};
}

// The word the render kernels test for "the call's inputs differ from the binned ones": the
// call's own check word, or -- when the caller vouches for its inputs (DGS_SAMPLE_INPUTS_BINNED)
// -- the binning header's always-zero word (no check, no call-time launches).
static uint32_t *dirty_word(const Call &a, uint32_t *flag) {
    if (!(a.opts & DGS_SAMPLE_INPUTS_BINNED)) return flag;
    return reinterpret_cast<uint32_t *>(const_cast<char *>(a.gb) + offsetof(Header, zero));
}

template <int FN, int D, int CB>
static int run_forward(const Call &a) {
    const WsLayout w = ws_layout(FN, a.P, D, a.N, a.C, false);
    float *grows = reinterpret_cast<float *>(a.ws);
    const bool binned = (a.opts & DGS_SAMPLE_INPUTS_BINNED) != 0;
    // rows of an earlier call on this workspace (one channel block: the rows hold all of C)
    const bool rows_valid = (a.opts & DGS_SAMPLE_ROWS_VALID) && a.C <= CB;
    uint32_t *const check = reinterpret_cast<uint32_t *>(a.ws + w.flag);
    uint32_t *const flag = dirty_word(a, check);
    const unsigned blocks = unit_blocks(a.gb, a.gbytes, a.sb, a.sbytes, false);
    const unsigned sub_blocks = unit_blocks(a.gb, a.gbytes, a.sb, a.sbytes, false, kWavesPerBlock, true);
    constexpr bool T = fwd_transposed<FN, D, CB>(), MX = !T && fwd_mfma<FN, D, CB>();
    UnitHint hint;  // without a hint (foreign buffers) the tail pass runs unconditionally
    hint.nunsafe = -1;
    const bool hinted = hint_get(a.gb, a.gbytes, a.sb, a.sbytes, &hint);
    const bool has_unsafe = !hinted || hint.nunsafe != 0;
    if (!binned)  // (the call-time path's tile lists, at the binning's first such call)
        if (int rc = ensure_ref_lists(a.gb, a.gbytes, a.sb, a.sbytes, a.s, a.debug)) return rc;
    for (int cbase = 0; cbase < a.C; cbase += CB) {
        if (!rows_valid) {
            k_pack_gauss<FN, D, CB><<<grid_for(a.P), kBlock, 0, a.s>>>(a.P, a.gb, a.values, a.C, cbase, grows,
                                                                       cbase == 0 && !binned ? flag : nullptr);
            DGS_LAUNCH_CHECK(a.s, a.debug);
        } else if (!binned) {
            DGS_TRY_HIP(hipMemsetAsync(flag, 0, 4, a.s));
        }
        if (cbase == 0 && !binned) {  // were the binned means / conics / samples passed? (device-side flag)
            const int rc = verify_inputs(a.gb, a.sb, a.P, D, a.N, a.means, a.conics, a.samples, flag, a.s, a.debug);
            if (rc) return rc;
        }
        {
            KernelTimer t(0, a.s, a.opts);  // (the main pass and the thin / tail passes behind it)
            if constexpr (T && D == 2 && DGS_FWD_SUB)  // sub-cell lists (units from the sub-unit hint)
                k_forward_s<FN, D, CB><<<sub_blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows, a.outs, a.C, cbase, flag);
            else if constexpr (T)
                k_forward_t<FN, D, CB><<<blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows, a.outs, a.C, cbase, flag);
            else if constexpr (MX)
                k_forward_mx<FN, D, CB><<<blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows, a.outs, a.C, cbase, flag);
            else
                k_forward<FN, D, CB, false><<<blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows,
                                                                          a.samples, a.outs, a.C, cbase, flag);
            DGS_LAUNCH_CHECK(a.s, a.debug);
            if constexpr (T || MX) {
                if (has_unsafe) {  // unsafe-conic entries, same stream: after the main pass
                    // (grid-strided over a capped grid: it exits at once when the device-side
                    // unsafe count is 0, which the host does not know without a sync)
                    const unsigned tb = hint.nunsafe > 0 ? blocks : std::min(blocks, 1024u);
                    k_forward<FN, D, CB, true><<<tb, kBlock, 0, a.s>>>(a.gb, a.sb, grows, a.samples, a.outs, a.C,
                                                                       cbase, flag);
                    DGS_LAUNCH_CHECK(a.s, a.debug);
                }
            }
        }
        // the call-time path (exits at once unless the inputs differ from the binned ones)
        if (!binned) {  // (the Gaussian rows are not read on this path: the cuts go there)
            const RefCall rc_ = ref_call(a, nullptr, flag, cbase, grows);
            int rc = ref_boxes<D>(rc_);
            if (!rc) rc = ref_forward<FN, D, CB>(rc_);
            if (rc) return rc;
        }
    }
    return DGS_OK;
}

template <int FN, int D, int CB>
static int run_backward(const Call &a) {
    const WsLayout w = ws_layout(FN, a.P, D, a.N, a.C, true);
    float *grows = reinterpret_cast<float *>(a.ws);
    float *srows = reinterpret_cast<float *>(a.ws + w.grows);
    float *acc = reinterpret_cast<float *>(a.ws + w.grows + w.srows);
    const bool binned = (a.opts & DGS_SAMPLE_INPUTS_BINNED) != 0;
    const bool rows_valid = (a.opts & DGS_SAMPLE_ROWS_VALID) && a.C <= CB;
    uint32_t *const check = reinterpret_cast<uint32_t *>(a.ws + w.flag);
    uint32_t *const flag = dirty_word(a, check);
    constexpr int S = D * (D + 1) / 2;
    const unsigned blocks = unit_blocks(a.gb, a.gbytes, a.sb, a.sbytes, true);
    // the sort-path entries' slots (one channel block: the sums of a multi-block C accumulate
    // over the blocks, so those keep the atomics; buffers without a hint keep them too)
    // Only where the sort path holds a large share of the entries (thin fields: 70 %): at the
    // headline (2 %) the slot pass costs more than the few scattered atomics it replaces.
    // (the caller's workspace: no allocation here, graph capture included)
    const size_t slot_bytes = slot_region_bytes(FN, D, a.C, a.gb, a.gbytes, a.sb, a.sbytes);
    float *const esums = slot_bytes > 0 && a.wsbytes >= w.total + slot_bytes
                             ? reinterpret_cast<float *>(a.ws + w.total) : nullptr;
    if (!binned)
        if (int rc = ensure_ref_lists(a.gb, a.gbytes, a.sb, a.sbytes, a.s, a.debug)) return rc;
    for (int cbase = 0; cbase < a.C; cbase += CB) {
        if (!rows_valid) {
            k_pack_gauss<FN, D, CB><<<grid_for(a.P), kBlock, 0, a.s>>>(a.P, a.gb, a.values, a.C, cbase, grows,
                                                                       nullptr);
            DGS_LAUNCH_CHECK(a.s, a.debug);
        }
        // sample rows (+ the zero-fill of the sums and of the check word, first block only)
        k_pack_samples<FN, D, CB><<<grid_for(a.N + kSrowPad), kBlock, 0, a.s>>>(
            a.N, a.gb, a.sb, a.dls, a.C, cbase, srows, cbase == 0 ? reinterpret_cast<float4 *>(acc) : nullptr,
            (int64_t)(w.acc / 16), cbase == 0 && !binned ? flag : nullptr);
        DGS_LAUNCH_CHECK(a.s, a.debug);
        if (cbase == 0 && !binned) {
            const int rc = verify_inputs(a.gb, a.sb, a.P, D, a.N, a.means, a.conics, a.samples, flag, a.s, a.debug);
            if (rc) return rc;
        }
        // dm/dc accumulate over all channel blocks (dL_dG is a sum over channels)
        {
            KernelTimer t(1, a.s, a.opts);
            if constexpr (bwd_mfma<FN, D, CB>())
                k_backward_mx<FN, D, CB><<<blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows, srows, acc, a.P, D + S + cbase,
                                                                      flag, esums);
            else
                k_backward<FN, D, CB><<<blocks, kBlock, 0, a.s>>>(a.gb, a.sb, grows, srows, acc, a.P, D + S + cbase,
                                                                   flag, esums);
            if (esums)
                k_bwd_esum<FN, D, CB><<<grid_for((int64_t)a.P * kEsumLanes), kBlock, 0, a.s>>>(a.P, a.gb, esums, acc,
                                                                                             D + S + cbase, flag);
        }
        DGS_LAUNCH_CHECK(a.s, a.debug);
        if (!binned) {  // (after k_backward, the last reader of the Gaussian rows)
            const RefCall rc_ = ref_call(a, acc, flag, cbase, grows);
            int rc = ref_boxes<D>(rc_);
            if (!rc) rc = ref_backward<FN, D, CB>(rc_);
            if (rc) return rc;
        }
    }
    if constexpr (D == 2 && CB == 1 && grow_stride<FN, D, CB>() >= 8) {
        if (a.C == 1) {  // the Gaussian-row region is free again: AoS rows there
            float4 *rows = reinterpret_cast<float4 *>(a.ws);
            k_soa_to_rows<<<grid_for(a.P), kBlock, 0, a.s>>>(a.P, acc, rows);
            DGS_LAUNCH_CHECK(a.s, a.debug);
            k_finalize_rows<<<grid_for(a.P), kBlock, 0, a.s>>>(a.P, a.gb, rows, a.dm, a.dv, a.dc);
            DGS_LAUNCH_CHECK(a.s, a.debug);
            return DGS_OK;
        }
    }
    k_finalize<<<grid_for(a.P), kBlock, 0, a.s>>>(a.P, D, a.C, a.gb, acc, a.dm, a.dv, a.dc);
    DGS_LAUNCH_CHECK(a.s, a.debug);
    return DGS_OK;
}

template <int FN, int D>
static int dispatch_cb(const Call &a, bool bwd) {
    switch (channel_block(a.C)) {
    case 1: return bwd ? run_backward<FN, D, 1>(a) : run_forward<FN, D, 1>(a);
    case 2: return bwd ? run_backward<FN, D, 2>(a) : run_forward<FN, D, 2>(a);
    case 4: return bwd ? run_backward<FN, D, 4>(a) : run_forward<FN, D, 4>(a);
    case 8: return bwd ? run_backward<FN, D, 8>(a) : run_forward<FN, D, 8>(a);
    default: return bwd ? run_backward<FN, D, 16>(a) : run_forward<FN, D, 16>(a);
    }
}

template <int FN>
static int dispatch_d(const Call &a, bool bwd) {
    return a.D == 1 ? dispatch_cb<FN, 1>(a, bwd) : dispatch_cb<FN, 2>(a, bwd);
}

// Fused masks (two or more functions; D = 2, C = 1): one instantiation per mask.
template <int M>
static int run_multi(const Call &a, bool bwd) {
    return bwd ? run_backward<kMulti + M, 2, 1>(a) : run_forward<kMulti + M, 2, 1>(a);
}
static int dispatch_multi(const Call &a, bool bwd) {
    switch (fn_mask(a.FN)) {
    case 3: return run_multi<3>(a, bwd);
    case 5: return run_multi<5>(a, bwd);
    case 6: return run_multi<6>(a, bwd);
    case 7: return run_multi<7>(a, bwd);
    case 9: return run_multi<9>(a, bwd);
    case 10: return run_multi<10>(a, bwd);
    case 11: return run_multi<11>(a, bwd);
    case 12: return run_multi<12>(a, bwd);
    case 13: return run_multi<13>(a, bwd);
    case 14: return run_multi<14>(a, bwd);
    default: return run_multi<15>(a, bwd);
    }
}

static int dispatch(const Call &a, bool bwd) {
    if (is_multi(a.FN)) return dispatch_multi(a, bwd);
    switch (a.FN) {
    case DGS_GAUSSIAN: return dispatch_d<0>(a, bwd);
    case DGS_DERIVATIVE: return dispatch_d<1>(a, bwd);
    case DGS_LAPLACIAN: return dispatch_d<2>(a, bwd);
    default: return dispatch_d<3>(a, bwd);
    }
}

static int validate(int FN, int P, int D, int N, int C, const void *gb, size_t gbytes,
                    const void *sb, size_t sbytes, size_t need, size_t have) {
    if (FN < 0 || (FN > 3 && !is_multi(FN))) return fail(DGS_ERR_ARG, "unknown sampling function");
    if (is_multi(FN) && (fn_mask(FN) < 1 || fn_mask(FN) > 15)) return fail(DGS_ERR_ARG, "function mask must be in 1..15");
    if (is_multi(FN) && (D != 2 || C != 1))
        return fail(DGS_ERR_ARG, "the fused form supports D = 2, C = 1 (call the per-function entry points)");
    if (D != 1 && D != 2) return fail(DGS_ERR_ARG, "only D = 1 or D = 2 is supported");
    if (P < 0 || N < 0 || C < 0) return fail(DGS_ERR_ARG, "negative size");
    if (P == 0 || N == 0 || C == 0) return DGS_OK;
    if ((uint64_t)P * grow_stride_rt(FN, D, channel_block(C)) * 4 >= (1ull << 32))
        return fail(DGS_ERR_ARG, "Gaussian rows exceed 4 GiB (32-bit scalar offsets)");
    if (!gb || !sb || gbytes < kHeaderBytes || sbytes < kHeaderBytes)
        return fail(DGS_ERR_BUFFER, "binning buffers missing or too small (run preprocess first)");
    if (have < need) return fail(DGS_ERR_ARG, "workspace too small");
    // The kernels index perm / rows / samples by the binned sizes: a call with other sizes than
    // the buffers were built for is an error (checked on the host against the preprocess record;
    // buffers from elsewhere have none and are trusted, as in the reference).
    UnitHint h;
    if (hint_get(gb, gbytes, sb, sbytes, &h) && (h.P != P || h.D != D || h.N != N))
        return fail(DGS_ERR_ARG, "P / D / N differ from the ones the binning buffers were built for (P " +
                                     std::to_string(h.P) + ", D " + std::to_string(h.D) + ", N " +
                                     std::to_string(h.N) + ")");
    return DGS_OK;
}

}  // namespace dgs

using namespace dgs;

extern "C" size_t dgs_sample_workspace_size(int function, int P, int D, int N, int C, int backward) {
    if (function < 0 || (function > 3 && !is_multi(function))) return 256;
    if (P <= 0 || N <= 0 || C <= 0 || (D != 1 && D != 2)) return 256;
    return ws_layout(function, P, D, N, C, backward != 0).total;
}

static int mask_code(int mask);
extern "C" size_t dgs_sample_workspace_size_binned(int mask, int P, int D, int N, int C, int backward,
                                                  const void *binning, size_t binning_bytes,
                                                  const void *sample_binning, size_t sample_binning_bytes) {
    const int FN = mask_code(mask);
    if (FN < 0) return 256;
    const size_t base = dgs_sample_workspace_size(FN, P, D, N, C, backward);
    if (!backward || P <= 0 || N <= 0 || C <= 0 || (D != 1 && D != 2)) return base;
    return base + slot_region_bytes(FN, D, C, binning, binning_bytes, sample_binning, sample_binning_bytes);
}

// ------------------------------------------------------------------ entry points
// One traversal of the pairs for every function of `mask` (bit f = dgs_function f): the
// forward writes each function's output, the backward takes each function's dL and returns
// the gradients of the summed loss.  A single-bit mask is the per-function path.
static int mask_code(int mask) {
    if (mask < 1 || mask > 15) return -1;
    for (int f = 0; f < 4; ++f)
        if (mask == (1 << f)) return f;
    return kMulti + mask;
}

extern "C" size_t dgs_sample_workspace_size_multi(int mask, int P, int D, int N, int C, int backward) {
    const int FN = mask_code(mask);
    return FN < 0 ? 256 : dgs_sample_workspace_size(FN, P, D, N, C, backward);
}

extern "C" int dgs_sample_forward_ex(int mask, int P, int D, int N, int C, const float *means,
                                     const float *values, const float *conics, const float *samples,
                                     const void *binning, size_t binning_bytes, const void *sample_binning,
                                     size_t sample_binning_bytes, float *const *outs, void *workspace,
                                     size_t workspace_bytes, const dgs_sample_options *opts, dgs_stream_t stream,
                                     int debug) {
    const int FN = mask_code(mask);
    if (FN < 0) return fail(DGS_ERR_ARG, "function mask must be in 1..15");
    const size_t need = dgs_sample_workspace_size(FN, P, D, N, C, 0);
    int rc = validate(FN, P, D, N, C, binning, binning_bytes, sample_binning, sample_binning_bytes,
                      need, workspace_bytes);
    if (rc || P == 0 || N == 0 || C == 0) return rc;
    Outs o{{nullptr, nullptr, nullptr, nullptr}};
    for (int f = 0; f < 4; ++f) {
        if (!(mask & (1 << f))) continue;
        if (!outs || !outs[f]) return fail(DGS_ERR_ARG, "missing output pointer for a function of the mask");
        o.p[f] = outs[f];
    }
    // (debug: always the device-side input check)
    const uint32_t flags = opts && !debug ? opts->flags : 0u;
    if ((flags & DGS_SAMPLE_GRAPH_CAPTURE) && !(flags & DGS_SAMPLE_INPUTS_BINNED))
        return fail(DGS_ERR_ARG, "DGS_SAMPLE_GRAPH_CAPTURE requires DGS_SAMPLE_INPUTS_BINNED (the binned tensors)");
    Call a{FN, P, D, N, C, flags, means, values, conics, samples, DLs{{nullptr, nullptr, nullptr, nullptr}},
           static_cast<const char *>(binning), static_cast<const char *>(sample_binning),
           binning_bytes, sample_binning_bytes, o, nullptr, nullptr, nullptr,
           static_cast<char *>(workspace), workspace_bytes, reinterpret_cast<hipStream_t>(stream), debug};
    return dispatch(a, false);
}

extern "C" int dgs_sample_backward_ex(int mask, int P, int D, int N, int C, const float *means,
                                      const float *values, const float *conics, const float *samples,
                                      const float *const *dL_douts, const void *binning, size_t binning_bytes,
                                      const void *sample_binning, size_t sample_binning_bytes, float *dL_dmeans,
                                      float *dL_dvalues, float *dL_dconics, void *workspace, size_t workspace_bytes,
                                      const dgs_sample_options *opts, dgs_stream_t stream, int debug) {
    const int FN = mask_code(mask);
    if (FN < 0) return fail(DGS_ERR_ARG, "function mask must be in 1..15");
    const size_t need = dgs_sample_workspace_size(FN, P, D, N, C, 1);
    int rc = validate(FN, P, D, N, C, binning, binning_bytes, sample_binning, sample_binning_bytes,
                      need, workspace_bytes);
    if (rc) return rc;
    DLs d{{nullptr, nullptr, nullptr, nullptr}};
    for (int f = 0; f < 4 && P > 0 && N > 0 && C > 0; ++f) {
        if (!(mask & (1 << f))) continue;
        if (!dL_douts || !dL_douts[f]) return fail(DGS_ERR_ARG, "missing dL_dout for a function of the mask");
        d.p[f] = dL_douts[f];
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (P == 0 || N == 0 || C == 0) {
        // sample_points.cu:165-167: zero gradients
        const int S = D * (D + 1) / 2;
        if (P > 0) {
            DGS_TRY_HIP(hipMemsetAsync(dL_dmeans, 0, sizeof(float) * (size_t)P * D, s));
            DGS_TRY_HIP(hipMemsetAsync(dL_dconics, 0, sizeof(float) * (size_t)P * S, s));
            if (C > 0) DGS_TRY_HIP(hipMemsetAsync(dL_dvalues, 0, sizeof(float) * (size_t)P * C, s));
        }
        return DGS_OK;
    }
    const uint32_t flags = opts && !debug ? opts->flags : 0u;
    if ((flags & DGS_SAMPLE_GRAPH_CAPTURE) && !(flags & DGS_SAMPLE_INPUTS_BINNED))
        return fail(DGS_ERR_ARG, "DGS_SAMPLE_GRAPH_CAPTURE requires DGS_SAMPLE_INPUTS_BINNED (the binned tensors)");
    Call a{FN, P, D, N, C, flags, means, values, conics, samples, d,
           static_cast<const char *>(binning), static_cast<const char *>(sample_binning),
           binning_bytes, sample_binning_bytes, Outs{{nullptr, nullptr, nullptr, nullptr}},
           dL_dmeans, dL_dvalues, dL_dconics, static_cast<char *>(workspace), workspace_bytes, s, debug};
    return dispatch(a, true);
}

extern "C" int dgs_sample_forward(int function, int P, int D, int N, int C, const float *means,
                                  const float *values, const float *conics, const float *samples,
                                  const void *binning, size_t binning_bytes,
                                  const void *sample_binning, size_t sample_binning_bytes,
                                  float *out, void *workspace, size_t workspace_bytes,
                                  dgs_stream_t stream, int debug) {
    if (function < 0 || function > 3) return fail(DGS_ERR_ARG, "unknown sampling function");
    float *outs[4] = {nullptr, nullptr, nullptr, nullptr};
    outs[function] = out;
    return dgs_sample_forward_ex(1 << function, P, D, N, C, means, values, conics, samples, binning, binning_bytes,
                                 sample_binning, sample_binning_bytes, outs, workspace, workspace_bytes, nullptr,
                                 stream, debug);
}

extern "C" int dgs_sample_backward(int function, int P, int D, int N, int C, const float *means,
                                   const float *values, const float *conics, const float *samples,
                                   const float *dL_dout, const void *binning, size_t binning_bytes,
                                   const void *sample_binning, size_t sample_binning_bytes,
                                   float *dL_dmeans, float *dL_dvalues, float *dL_dconics,
                                   void *workspace, size_t workspace_bytes, dgs_stream_t stream,
                                   int debug) {
    if (function < 0 || function > 3) return fail(DGS_ERR_ARG, "unknown sampling function");
    const float *dls[4] = {nullptr, nullptr, nullptr, nullptr};
    dls[function] = dL_dout;
    return dgs_sample_backward_ex(1 << function, P, D, N, C, means, values, conics, samples, dls, binning,
                                  binning_bytes, sample_binning, sample_binning_bytes, dL_dmeans, dL_dvalues,
                                  dL_dconics, workspace, workspace_bytes, nullptr, stream, debug);
}

extern "C" int dgs_sample_forward_multi(int mask, int P, int D, int N, int C, const float *means,
                                        const float *values, const float *conics, const float *samples,
                                        const void *binning, size_t binning_bytes,
                                        const void *sample_binning, size_t sample_binning_bytes,
                                        float *const *outs, void *workspace, size_t workspace_bytes,
                                        dgs_stream_t stream, int debug) {
    return dgs_sample_forward_ex(mask, P, D, N, C, means, values, conics, samples, binning, binning_bytes,
                                 sample_binning, sample_binning_bytes, outs, workspace, workspace_bytes, nullptr,
                                 stream, debug);
}

extern "C" int dgs_sample_backward_multi(int mask, int P, int D, int N, int C, const float *means,
                                         const float *values, const float *conics, const float *samples,
                                         const float *const *dL_douts, const void *binning,
                                         size_t binning_bytes, const void *sample_binning,
                                         size_t sample_binning_bytes, float *dL_dmeans,
                                         float *dL_dvalues, float *dL_dconics, void *workspace,
                                         size_t workspace_bytes, dgs_stream_t stream, int debug) {
    return dgs_sample_backward_ex(mask, P, D, N, C, means, values, conics, samples, dL_douts, binning,
                                  binning_bytes, sample_binning, sample_binning_bytes, dL_dmeans, dL_dvalues,
                                  dL_dconics, workspace, workspace_bytes, nullptr, stream, debug);
}

extern "C" int dgs_count_pairs(int P, int D, int N, const float *means, const float *conics,
                               const float *samples, const void *binning, size_t binning_bytes,
                               const void *sample_binning, size_t sample_binning_bytes, float thr,
                               int64_t *counts, void *workspace, size_t workspace_bytes,
                               dgs_stream_t stream) {
    counts[0] = counts[1] = 0;
    const size_t need = dgs_sample_workspace_size(0, P, D, N, 1, 0) + 256;
    int rc = validate(0, P, D, N, 1, binning, binning_bytes, sample_binning, sample_binning_bytes,
                      need, workspace_bytes);
    if (rc || P == 0 || N == 0) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const char *gb = static_cast<const char *>(binning), *sb = static_cast<const char *>(sample_binning);
    const WsLayout w = ws_layout(0, P, D, N, 1, false);
    float *grows = static_cast<float *>(workspace);
    unsigned long long *dcnt = reinterpret_cast<unsigned long long *>(
        static_cast<char *>(workspace) + need - 256);
    DGS_TRY_HIP(hipMemsetAsync(dcnt, 0, 16, s));
    const unsigned blocks = unit_blocks(gb, binning_bytes, sb, sample_binning_bytes, false);
    if (D == 2) {
        k_pack_gauss<0, 2, 1><<<grid_for(P), kBlock, 0, s>>>(P, gb, conics, 0, 0, grows, nullptr);
        if (DGS_FWD_SUB)
            k_count_s<<<unit_blocks(gb, binning_bytes, sb, sample_binning_bytes, false, kWavesPerBlock, true), kBlock, 0,
                        s>>>(gb, sb, grows, samples, thr, dcnt);
        else
            k_count<2><<<blocks, kBlock, 0, s>>>(gb, sb, grows, samples, thr, dcnt);
    } else {
        k_pack_gauss<0, 1, 1><<<grid_for(P), kBlock, 0, s>>>(P, gb, conics, 0, 0, grows, nullptr);
        k_count<1><<<blocks, kBlock, 0, s>>>(gb, sb, grows, samples, thr, dcnt);
    }
    DGS_TRY_HIP(hipGetLastError());
    unsigned long long h[2];
    DGS_TRY_HIP(hipMemcpyAsync(h, dcnt, sizeof(h), hipMemcpyDeviceToHost, s));
    DGS_TRY_HIP(hipStreamSynchronize(s));
    counts[0] = (int64_t)h[0];
    counts[1] = (int64_t)h[1];
    return DGS_OK;
}

extern "C" int dgs_inputs_match(int P, int D, int N, const float *means, const float *conics,
                                const float *samples, const void *binning, size_t binning_bytes,
                                const void *sample_binning, size_t sample_binning_bytes, int *match,
                                dgs_stream_t stream) {
    if (!match) return fail(DGS_ERR_ARG, "dgs_inputs_match: match pointer required");
    *match = 1;
    int rc = validate(0, P, D, N, 1, binning, binning_bytes, sample_binning, sample_binning_bytes, 0, 0);
    if (rc || P == 0 || N == 0) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t *flag = nullptr;
    note_internal_alloc();  // (a diagnostic: 4 bytes of stream-ordered scratch, dgs.h)
    DGS_TRY_HIP(hipMallocAsync(&flag, 4, s));
    struct FreeGuard {  // (freed on every path, the error paths included)
        uint32_t *p;
        hipStream_t s;
        ~FreeGuard() { (void)hipFreeAsync(p, s); }
    } guard{flag, s};
    DGS_TRY_HIP(hipMemsetAsync(flag, 0, 4, s));
    rc = verify_inputs(static_cast<const char *>(binning), static_cast<const char *>(sample_binning), P, D, N,
                       means, conics, samples, flag, s, 0);
    if (rc) return rc;
    uint32_t h = 0;
    DGS_TRY_HIP(hipMemcpyAsync(&h, flag, 4, hipMemcpyDeviceToHost, s));
    DGS_TRY_HIP(hipStreamSynchronize(s));
    *match = h ? 0 : 1;
    return DGS_OK;
}

// Tuning hook: k_backward's phase sums of a DGS_BWD_STAMPS build (reset after reading).
extern "C" int dgs_debug_bwd_stamps(unsigned long long *out8) {
#if DGS_BWD_STAMPS
    std::vector<unsigned long long> all((size_t)dgs::kStampCopies * 8, 0ull);
    DGS_TRY_HIP(hipMemcpyFromSymbol(all.data(), HIP_SYMBOL(dgs::g_bwd_stamps), all.size() * 8));
    for (int k = 0; k < 8; ++k) {
        out8[k] = 0;
        for (int c = 0; c < dgs::kStampCopies; ++c) out8[k] += all[(size_t)c * 8 + k];
    }
    std::fill(all.begin(), all.end(), 0ull);
    DGS_TRY_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dgs::g_bwd_stamps), all.data(), all.size() * 8));
    return DGS_OK;
#else
    (void)out8;
    return fail(DGS_ERR_ARG, "not a DGS_BWD_STAMPS build");
#endif
}

extern "C" void dgs_timing_enable(int on) {
    std::lock_guard<std::mutex> lk(g_tmu);
    g_timing = on != 0;
}

// Sums the recorded durations of kernel `which` (0 = forward render, 1 = backward render),
// waiting for their events, and clears the record.  Returns the number of launches.
extern "C" int dgs_timing_read(int which, double *total_ms) {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
    {
        std::lock_guard<std::mutex> lk(g_tmu);
        if (which < 0 || which > 1) return -1;
        ev.swap(g_tev[which]);
    }
    double tot = 0.0;
    for (auto &p : ev) {
        float ms = 0.0f;
        (void)hipEventSynchronize(p.second);
        if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) tot += ms;
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    *total_ms = tot;
    return (int)ev.size();
}

// ------------------------------------------------------------------------- warm-up
// A no-op launch: the first launch of any kernel of this translation unit loads its code object
// (rocprim's kernels included) onto the device; dgs_warmup does it for every unit up front.
__global__ void k_warm_sample() {}
namespace dgs {
hipError_t warm_sample(hipStream_t s) {
    k_warm_sample<<<1, 1, 0, s>>>();
    return hipGetLastError();
}
}  // namespace dgs
