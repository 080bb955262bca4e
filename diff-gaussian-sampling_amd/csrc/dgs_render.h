// dgs_render.h -- per-pair math of the four sampling functions (forward and backward) and
// the packed row formats of the render kernels.
//
// Row formats (fp32, written per call by the pack kernels; read wave-uniformly through the
// scalar cache in the forward, per lane in the backward):
//   Gaussian row  D=2: [m0 m1 k0 k1 k2 (c0 c1 c2) v0..v(CB-1)]   (c only for FN != gaussian)
//                 D=1: [m0 k0 (c0) v0..]                           padded to RS = 4k floats
//     k = conic * (-log2 e) * {1/2, 1, 1/2}: power * log2(e) = X0 (k0 X0 + k1 X1) + k2 X1^2
//   Conic row:    [c0 c1 c2 0] / [c0 0 0 0]  (unsafe/general paths and the backward)
//   Sample row (backward): [s0 (s1) dLsym[U][CB]], dL summed over symmetric components.
#pragma once

#include "dgs_internal.h"

namespace dgs {

constexpr float kLog2e = 1.4426950408889634f;

#ifndef DGS_VFACTOR
#define DGS_VFACTOR 1  // backward, gaussian, C = 1: moments of G dL, scaled by v per unit
#endif

// Function codes: 0..3 = gaussian, derivative, laplacian, third (dgs_function); kMulti + mask
// = the fused form that evaluates every function of `mask` (bit f = function f) in one
// traversal of the pairs (D = 2, C = 1; dgs_sample_forward_multi).
constexpr int kMulti = 16;
__host__ __device__ constexpr bool is_multi(int FN) { return FN >= kMulti; }
__host__ __device__ constexpr int fn_mask(int FN) { return FN >= kMulti ? FN - kMulti : 1 << FN; }
__host__ __device__ constexpr int fn_k(int f, int D) { return f == 0 ? 1 : f == 1 ? D : f == 2 ? D * D : D * D * D; }
__host__ __device__ constexpr int fn_u(int f, int D) { return D == 1 ? 1 : f + 1; }
// sample-row coefficient fields of the moment-form backward (mom_coef)
__host__ __device__ constexpr int fn_mfields(int f) { return f == 0 ? 1 : f == 1 ? 2 : f == 2 ? 5 : 6; }
__host__ __device__ constexpr int mask_sum(int M, int D, int what) {  // 0: K, 1: U, 2: fields
    int s = 0;
    for (int f = 0; f < 4; ++f)
        if (M & (1 << f)) s += what == 0 ? fn_k(f, D) : what == 1 ? fn_u(f, D) : fn_mfields(f);
    return s;
}
// first unique component / coefficient field of function f in a mask's block
__host__ __device__ constexpr int mask_uoff(int M, int D, int f) { return mask_sum(M & ((1 << f) - 1), D, 1); }
__host__ __device__ constexpr int mask_foff(int M, int f) { return mask_sum(M & ((1 << f) - 1), 2, 2); }

template <int FN, int D>
struct Traits {
    static constexpr int M = fn_mask(FN);
    static constexpr int K = mask_sum(M, D, 0);  // output components (summed over the mask)
    static constexpr int U = mask_sum(M, D, 1);  // unique components
    static constexpr int S = D * (D + 1) / 2;
    static constexpr bool CONIC = (M & ~1) != 0;  // a function other than gaussian: raw conic in the row
    static constexpr int GBASE = D == 2 ? (CONIC ? 8 : 5) : (CONIC ? 3 : 2);  // first value slot
};

// expanded component k of function f -> its unique term (forward.cu:288-291, 322-329)
__host__ __device__ constexpr int unique_fk(int f, int D, int k) {
    if (D == 1 || f <= 1) return k;
    if (f == 2) return k == 0 ? 0 : (k == 3 ? 2 : 1);
    return k == 0 ? 0 : (k == 7 ? 3 : ((k == 1 || k == 2 || k == 4) ? 1 : 2));
}
template <int FN, int D>
__host__ __device__ constexpr int unique_of(int k) { return unique_fk(FN, D, k); }

template <int FN, int D, int CB>
__host__ __device__ constexpr int grow_stride() { return (Traits<FN, D>::GBASE + CB + 3) / 4 * 4; }
template <int FN, int D, int CB>
__host__ __device__ constexpr int srow_stride() {
    return is_multi(FN) ? (D + mask_sum(fn_mask(FN), D, 2) + 3) / 4 * 4 : (D + Traits<FN, D>::U * CB + 3) / 4 * 4;
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---------------------------------------------------------------------------------------
// Lane values: `float` (one pair per lane) or `f2` (two pairs per lane).  The per-pair math
// below is written once over V; with V = f2 the compiler emits packed fp32 VALU ops
// (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32, wave-uniform operands broadcast from SGPR
// pairs with op_sel), which is what the 157 TFLOP/s fp32 vector peak of MI355X counts.  Each
// component goes through exactly the operations of the scalar form, so results are
// bit-identical to V = float.
// ---------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

template <typename V> __device__ __forceinline__ V bc(float x);
template <> __device__ __forceinline__ float bc<float>(float x) { return x; }
template <> __device__ __forceinline__ f2 bc<f2>(float x) { return f2{x, x}; }

__device__ __forceinline__ float vexp2(float x) { return fast_exp2(x); }
__device__ __forceinline__ f2 vexp2(f2 x) { return f2{fast_exp2(x.x), fast_exp2(x.y)}; }

__device__ __forceinline__ float lo(float x) { return x; }
__device__ __forceinline__ float lo(f2 x) { return x.x; }
__device__ __forceinline__ float hsum(float x) { return x; }
__device__ __forceinline__ float hsum(f2 x) { return x.x + x.y; }

// Batch sizes of the wave-uniform scalar loads: the batch's rows occupy SGPRs (<= ~64).
template <int RS>
__host__ __device__ constexpr int fwd_batch() { return RS <= 8 ? 8 : RS <= 16 ? 4 : 2; }
template <int RSS>
__host__ __device__ constexpr int bwd_batch() { return RSS <= 4 ? 8 : RSS <= 8 ? 4 : RSS <= 16 ? 2 : 1; }

template <int N> struct U32s { uint32_t v[N]; };
template <int N> struct F32s { float v[N]; };

// N consecutive wave-uniform dwords as whole vector loads from the constant address space:
// one s_load_dwordx{4,8,16} per 4/8/16 dwords.  (Element-wise loads get shrunk to the dwords
// actually used -- e.g. a 6-of-8-dword row became x4 + x2 -- doubling the scalar-cache
// requests, which were the forward kernel's bottleneck.)
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ V sload_vec(const void *p) {
    return *(const __attribute__((address_space(4))) V *)(p);
}

template <int N>
__device__ __forceinline__ F32s<N> sload_f(const float *p) {
    static_assert(N % 4 == 0, "rows are padded to 4 dwords");
    F32s<N> r;
    int k = 0;
#pragma unroll
    for (; k + 16 <= N; k += 16) {
        const f32x16_t v = sload_vec<f32x16_t>(p + k);
#pragma unroll
        for (int i = 0; i < 16; ++i) r.v[k + i] = v[i];
    }
#pragma unroll
    for (; k + 8 <= N; k += 8) {
        const f32x8_t v = sload_vec<f32x8_t>(p + k);
        // Mark all 8 dwords live (no instruction is emitted): otherwise the load is shrunk
        // to the dwords the caller reads (x4 + x2 for a 6-dword row), two requests instead of one.
        asm volatile("" ::"s"(v));
#pragma unroll
        for (int i = 0; i < 8; ++i) r.v[k + i] = v[i];
    }
#pragma unroll
    for (; k + 4 <= N; k += 4) {
        const f32x4_t v = sload_vec<f32x4_t>(p + k);
#pragma unroll
        for (int i = 0; i < 4; ++i) r.v[k + i] = v[i];
    }
    return r;
}
template <int N>
__device__ __forceinline__ U32s<N> sload_u(const uint32_t *p) {
    static_assert(N == 8 || N == 4 || N == 2, "entry batches of 2, 4 or 8");
    U32s<N> r;
    if constexpr (N == 8) {
        const u32x8_t v = sload_vec<u32x8_t>(p);
#pragma unroll
        for (int i = 0; i < 8; ++i) r.v[i] = v[i];
    } else if constexpr (N == 4) {
        const u32x4_t v = sload_vec<u32x4_t>(p);
#pragma unroll
        for (int i = 0; i < 4; ++i) r.v[i] = v[i];
    } else {
        r.v[0] = sload(p);
        r.v[1] = sload(p + 1);
    }
    return r;
}

// dL of each function (indexed by function code; the fused form reads those of its mask)
struct DLs {
    const float *p[4];
};
// Output of each function (indexed by function code)
struct Outs {
    float *p[4];
};

// Stores (ADD: adds) the sum x of unique component ui (over the mask's functions), channel
// ch, of sample sid into every output component of its function that maps to it.
template <int FN, int D, bool ADD>
__device__ __forceinline__ void store_unique(const Outs &outs, int64_t sid, int ui, int C, int ch,
                                             float x) {
    constexpr int M = fn_mask(FN);
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        if (!(M & (1 << f))) continue;
        const int o = mask_uoff(M, D, f), K = fn_k(f, D);
        if (ui < o || ui >= o + fn_u(f, D)) continue;
        float *p = outs.p[f] + sid * K * C + ch;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (unique_fk(f, D, k) == ui - o) {
                if (ADD) p[k * C] += x;
                else p[k * C] = x;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Cross-lane reduce-scatter of a wave: every lane holds 64 partial sums v[0..63]; afterwards
// lane l holds v[l] summed over all 64 lanes (returned).  Six halving stages, each adding a
// lane's kept half to its partner's copy of the same half: distance 32 and 16 with the gfx950
// half-swap instructions (v_permlane32_swap / v_permlane16_swap move a whole register half
// between lane halves), distance 8/4/2/1 inside 16-lane rows with DPP (row_mirror,
// row_half_mirror, quad_perm xor 2 / xor 1).  At every stage the lane whose partner-distance
// bit is set keeps the upper half, so the surviving index equals the lane id.  ~140 VALU ops
// per 64 x 64 sums; the order of the additions is fixed (deterministic).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float rs_partner(float x, int ctrl) {
    switch (ctrl) {  // the DPP control must be a constant at the builtin
    case 0x140: return __builtin_amdgcn_update_dpp(0.0f, x, 0x140, 0xf, 0xf, false);  // row_mirror
    case 0x141: return __builtin_amdgcn_update_dpp(0.0f, x, 0x141, 0xf, 0xf, false);  // row_half_mirror
    case 0x4e: return __builtin_amdgcn_update_dpp(0.0f, x, 0x4e, 0xf, 0xf, false);    // quad_perm xor 2
    default: return __builtin_amdgcn_update_dpp(0.0f, x, 0xb1, 0xf, 0xf, false);      // quad_perm xor 1
    }
}

template <int N>
__device__ __forceinline__ void rs_dpp_stage(float (&x)[64], int lane, int bit, int ctrl) {
    // x[0..2N) -> x[0..N): keep own half, add the partner's copy of it
    const bool hi = (lane & bit) != 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const float keep = hi ? x[i + N] : x[i];
        const float send = hi ? x[i] : x[i + N];
        x[i] = keep + rs_partner(send, ctrl);
    }
}

__device__ __forceinline__ float reduce_scatter64(float (&x)[64], int lane) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {  // distance 32: lanes >= 32 keep values 32..63
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[i]), __float_as_uint(x[i + 32]), false, false);
        x[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // distance 16: odd 16-lane rows keep the upper half
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[i]), __float_as_uint(x[i + 16]), false, false);
        x[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    rs_dpp_stage<8>(x, lane, 8, 0x140);
    rs_dpp_stage<4>(x, lane, 4, 0x141);
    rs_dpp_stage<2>(x, lane, 2, 0x4e);
    rs_dpp_stage<1>(x, lane, 1, 0xb1);
    return x[0];
}

// Reference-literal power (forward.cu:227/234/246/256, backward.cu:113/132/...): float
// products without contraction, double scaling, rounded once to float.
template <int FN, int D>
__device__ __forceinline__ float ref_power(const float *X, const float *c) {
    DGS_NO_CONTRACT
    if constexpr (D == 1) {
        if constexpr (FN == 0) return (float)(-0.5 * (double)c[0] * (double)X[0] * (double)X[0]);
        else {
            const float x1 = rmul(c[0], X[0]);
            return (float)(-0.5 * (double)x1 * (double)X[0]);
        }
    } else {
        // gaussian: c0*X0*X0 + c2*X1*X1; others: x1*X0 + x2*X1 with x1 = c0*X0 -- same ops
        const float a = radd(rmul(rmul(c[0], X[0]), X[0]), rmul(rmul(c[2], X[1]), X[1]));
        const float b = rmul(rmul(c[1], X[0]), X[1]);
        return (float)(-0.5 * (double)a - (double)b);
    }
}

// ---------------------------------------------------------------------------------------
// Forward (forward.cu:225-332): acc[U][CB] += v * G * term_u
// ---------------------------------------------------------------------------------------
template <int FN, int D, int CB, typename V>
__device__ __forceinline__ void fwd_terms(const V *X, const float *c, V G, const float *v,
                                          V (&acc)[Traits<FN, D>::U][CB]) {
    constexpr int M = fn_mask(FN), UT = Traits<FN, D>::U;
    static_assert(!is_multi(FN) || D == 2, "the fused form is D = 2 only");
    if constexpr (M == 1) {
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) acc[0][ch] = vfma(bc<V>(v[ch]), G, acc[0][ch]);
    } else {
    V t[UT];
    if constexpr (D == 1) {
        const V x1 = c[0] * X[0];
        if constexpr (FN == 1) t[0] = x1;
        else if constexpr (FN == 2) t[0] = x1 * x1 - c[0];
        else t[0] = 3.0f * c[0] * x1 - x1 * x1 * x1;  // 2 c x1 - x1^3 + c x1
    } else {
        const V a1 = vfma(bc<V>(c[1]), X[1], c[0] * X[0]);
        const V a2 = vfma(bc<V>(c[1]), X[0], c[2] * X[1]);
        if constexpr ((M & 1) != 0) t[mask_uoff(M, D, 0)] = bc<V>(1.0f);
        if constexpr ((M & 2) != 0) {
            constexpr int o = mask_uoff(M, D, 1);
            t[o] = a1; t[o + 1] = a2;
        }
        if constexpr ((M & 4) != 0) {
            constexpr int o = mask_uoff(M, D, 2);
            t[o] = vfma(a1, a1, bc<V>(-c[0]));
            t[o + 1] = vfma(a1, a2, bc<V>(-c[1]));
            t[o + 2] = vfma(a2, a2, bc<V>(-c[2]));
        }
        if constexpr ((M & 8) != 0) {
            constexpr int o = mask_uoff(M, D, 3);
            const V a11 = a1 * a1, a22 = a2 * a2;
            t[o] = a1 * (3.0f * c[0] - a11);
            t[o + 1] = vfma(bc<V>(2.0f * c[1]), a1, a2 * (c[0] - a11));
            t[o + 2] = vfma(bc<V>(2.0f * c[1]), a2, a1 * (c[2] - a22));
            t[o + 3] = a2 * (3.0f * c[2] - a22);
        }
    }
#pragma unroll
    for (int ch = 0; ch < CB; ++ch) {
        const V vg = v[ch] * G;
#pragma unroll
        for (int u = 0; u < UT; ++u) acc[u][ch] = vfma(vg, t[u], acc[u][ch]);
    }
    }
}

// ---------------------------------------------------------------------------------------
// Backward (backward.cu:108-416).  Lane = Gaussian, so every accumulator is per lane.
// The gaussian function accumulates moments (gm/gc are linear in them, converted in the
// epilogue); the others accumulate the reference's per-pair terms.
//   gm[D], gc[S]: mean / conic gradient accumulators, gv[CB]: value gradient
//   dl[U][CB]: this sample's dL/dout summed over symmetric components (wave-uniform)
// ---------------------------------------------------------------------------------------
template <int FN, int D, int CB, typename V>
__device__ __forceinline__ void bwd_terms(const V *X, const float *c, V G, const float *v,
                                          const V (&dl)[Traits<FN, D>::U][CB], V *gm, V *gv,
                                          V *gc) {
    constexpr int U = Traits<FN, D>::U;
    V Gu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        V s = bc<V>(0.0f);
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) s = vfma(bc<V>(v[ch]), dl[u][ch], s);
        Gu[u] = s;  // dL_dG (per unique component), reference's dL_dG* sums
    }
    if constexpr (FN == 0) {
        // moments: gm = -[A (sum t X)], gc = -1/2 sum t X X^T (off-diagonal -sum t X0 X1).
        // CB = 1: t = v * (G dL) -- the moments accumulate w = G dL (also the values gradient)
        // and k_backward scales them by v once per unit (one op per pair fewer).
        V t;
        if constexpr (CB == 1 && DGS_VFACTOR) {
            t = G * dl[0][0];
            gv[0] += t;
        } else {
#pragma unroll
            for (int ch = 0; ch < CB; ++ch) gv[ch] = vfma(G, dl[0][ch], gv[ch]);
            t = G * Gu[0];
        }
        const V tx = t * X[0];
        gm[0] += tx;                              // sum t X0
        gc[0] = vfma(tx, X[0], gc[0]);            // sum t X0^2
        if constexpr (D == 2) {
            const V ty = t * X[1];
            gm[1] += ty;                          // sum t X1
            gc[1] = vfma(tx, X[1], gc[1]);        // sum t X0 X1
            gc[2] = vfma(ty, X[1], gc[2]);        // sum t X1^2
        }
    } else if constexpr (D == 1) {
        const V x1 = c[0] * X[0];
        const V GdLdG = G * Gu[0];
        V f, dmx, dcc;
        if constexpr (FN == 1) {
            f = x1;
            dmx = (x1 * x1 - c[0]);
            dcc = X[0] - 0.5f * X[0] * X[0] * x1;
        } else if constexpr (FN == 2) {
            f = x1 * x1 - c[0];
            dmx = x1 * x1 * x1 - 3.0f * c[0] * x1;
            dcc = 2.0f * x1 * X[0] - 0.5f * (x1 * x1 - c[0]) * X[0] * X[0] - 1.0f;
        } else {
            f = 3.0f * c[0] * x1 - x1 * x1 * x1;
            dmx = 6.0f * c[0] * x1 * x1 - x1 * x1 * x1 * x1 - 3.0f * c[0] * c[0];
            // backward.cu:322-325, reproduced literally (not the true derivative)
            dcc = 2.0f * X[0] * X[0] - 2.0f * x1 * x1 * X[0] - 0.5f * (2.0f * X[0] * x1 - X[0]) * X[0] * X[0]
                + 0.5f * (x1 * x1 - c[0]) * x1 * X[0] * X[0];
        }
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) gv[ch] = vfma(f * dl[0][ch], G, gv[ch]);
        gm[0] = vfma(-dmx, GdLdG, gm[0]);
        gc[0] = vfma(dcc, GdLdG, gc[0]);
    } else {
    const V X0 = X[0], X1 = X[1];
    const V a1 = vfma(bc<V>(c[1]), X1, c[0] * X0);
    const V a2 = vfma(bc<V>(c[1]), X0, c[2] * X1);
    if constexpr (FN == 1) {
        const V Gx = Gu[0], Gy = Gu[1];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch) gv[ch] = vfma(vfma(a1, dl[0][ch], a2 * dl[1][ch]), G, gv[ch]);
        const V gx = vfma(a1, Gx, a2 * Gy);
        const V axy = vfma(a1, a2, bc<V>(-c[1]));
        const V dLdx = vfma(vfma(a1, a1, bc<V>(-c[0])), Gx, axy * Gy) * G;
        const V dLdy = vfma(vfma(a2, a2, bc<V>(-c[2])), Gy, axy * Gx) * G;
        gm[0] -= dLdx;
        gm[1] -= dLdy;
        gc[0] = vfma(vfma(X0, Gx, -0.5f * X0 * X0 * gx), G, gc[0]);
        gc[1] = vfma(X1 * Gx + X0 * Gy - X0 * X1 * gx, G, gc[1]);
        gc[2] = vfma(vfma(X1, Gy, -0.5f * X1 * X1 * gx), G, gc[2]);
    } else if constexpr (FN == 2) {
        const V dxx = vfma(a1, a1, bc<V>(-c[0])), dxy = vfma(a1, a2, bc<V>(-c[1])),
                dyy = vfma(a2, a2, bc<V>(-c[2]));
        const V Gxx = Gu[0], Sxy = Gu[1], Gyy = Gu[2];
#pragma unroll
        for (int ch = 0; ch < CB; ++ch)
            gv[ch] = vfma(dxx * dl[0][ch] + dxy * dl[1][ch] + dyy * dl[2][ch], G, gv[ch]);
        const V dLdx = ((a1 * a1 * a1 - 3.0f * c[0] * a1) * Gxx
                            + (a1 * a2 * a1 - c[1] * a1 - (c[1] * a1 + c[0] * a2)) * Sxy
                            + (a2 * a2 * a1 - c[2] * a1 - 2.0f * c[1] * a2) * Gyy) * G;
        const V dLdy = ((a1 * a1 * a2 - c[0] * a2 - 2.0f * c[1] * a1) * Gxx
                            + (a1 * a2 * a2 - c[1] * a2 - (c[2] * a1 + c[1] * a2)) * Sxy
                            + (a2 * a2 * a2 - 3.0f * c[2] * a2) * Gyy) * G;
        gm[0] -= dLdx;
        gm[1] -= dLdy;
        const V xx_cxx = -0.5f * dxx * X0 * X0 + 2.0f * a1 * X0 - 1.0f;
        const V xy_cxx = -0.5f * dxy * X0 * X0 + a2 * X0;
        const V yy_cxx = -0.5f * dyy * X0 * X0;
        const V xx_cxy = -dxx * X0 * X1 + 2.0f * a1 * X1;
        const V xy_cxy = -dxy * X0 * X1 + a2 * X1 + a1 * X0 - 1.0f;
        const V yy_cxy = -dyy * X0 * X1 + 2.0f * a2 * X0;
        const V xx_cyy = -0.5f * dxx * X1 * X1;
        const V xy_cyy = -0.5f * dxy * X1 * X1 + a1 * X1;
        const V yy_cyy = -0.5f * dyy * X1 * X1 + 2.0f * a2 * X1 - 1.0f;
        gc[0] = vfma(xx_cxx * Gxx + xy_cxx * Sxy + yy_cxx * Gyy, G, gc[0]);
        gc[1] = vfma(xx_cxy * Gxx + xy_cxy * Sxy + yy_cxy * Gyy, G, gc[1]);
        gc[2] = vfma(xx_cyy * Gxx + xy_cyy * Sxy + yy_cyy * Gyy, G, gc[2]);
    } else {
    // third, D == 2
    const V a11 = a1 * a1, a22 = a2 * a2, a12 = a1 * a2;
    const V dxxx = 3.0f * c[0] * a1 - a11 * a1;
    const V dxxy = 2.0f * c[1] * a1 - a11 * a2 + c[0] * a2;
    const V dxyy = 2.0f * c[1] * a2 - a1 * a22 + c[2] * a1;
    const V dyyy = 3.0f * c[2] * a2 - a22 * a2;
    const V Gxxx = Gu[0], S1 = Gu[1], S2 = Gu[2], Gyyy = Gu[3];
#pragma unroll
    for (int ch = 0; ch < CB; ++ch)
        gv[ch] = vfma(dxxx * dl[0][ch] + dxxy * dl[1][ch] + dxyy * dl[2][ch] + dyyy * dl[3][ch], G, gv[ch]);
    const V xxy_dx = 2.0f * a12 * c[0] + a11 * c[1] - 3.0f * c[0] * c[1];
    const V xyy_dx = 2.0f * a12 * c[1] + a22 * c[0] - c[2] * c[0] - 2.0f * c[1] * c[1];
    const V dLdx = ((dxxx * a1 - 3.0f * c[0] * c[0] + 3.0f * a11 * c[0]) * Gxxx
                        + (dxxy * a1 + xxy_dx) * S1 + (dxyy * a1 + xyy_dx) * S2
                        + (dyyy * a1 - 3.0f * c[2] * c[1] + 3.0f * a22 * c[1]) * Gyyy) * G;
    const V xxy_dy = 2.0f * a12 * c[1] + a11 * c[2] - c[0] * c[2] - 2.0f * c[1] * c[1];
    const V xyy_dy = 2.0f * a12 * c[2] + a22 * c[1] - 3.0f * c[2] * c[1];
    const V dLdy = ((dxxx * a2 - 3.0f * c[0] * c[1] + 3.0f * a11 * c[1]) * Gxxx
                        + (dxxy * a2 + xxy_dy) * S1 + (dxyy * a2 + xyy_dy) * S2
                        + (dyyy * a2 - 3.0f * c[2] * c[2] + 3.0f * a22 * c[2]) * Gyyy) * G;
    gm[0] -= dLdx;
    gm[1] -= dLdy;
    const V v0 = -0.5f * dxxx * X0 * X0 + 3.0f * c[0] * X0 + 3.0f * a1 - 3.0f * a11 * X0;
    const V v1 = -0.5f * dxxy * X0 * X0 + 2.0f * c[1] * X0 - 2.0f * a12 * X0 + a2;
    const V v2 = -0.5f * dxyy * X0 * X0 - a22 * X0 + c[2] * X0;
    const V v3 = -0.5f * dyyy * X0 * X0;
    const V w0 = -dxxx * X0 * X1 + 3.0f * c[0] * X1 - 3.0f * a11 * X1;
    const V w1 = -dxxy * X0 * X1 + 2.0f * c[1] * X1 + 2.0f * a1 - 2.0f * a12 * X1 - a11 * X0 + c[0] * X0;
    const V w2 = -dxyy * X0 * X1 + 2.0f * c[1] * X0 + 2.0f * a2 - a22 * X1 - 2.0f * a12 * X0 + c[2] * X1;
    const V w3 = -dyyy * X0 * X1 + 3.0f * c[2] * X0 - 3.0f * a22 * X0;
    const V z0 = -0.5f * dxxx * X1 * X1;
    const V z1 = -0.5f * dxxy * X1 * X1 - a11 * X1 + c[0] * X1;
    const V z2 = -0.5f * dxyy * X1 * X1 + 2.0f * c[1] * X1 - 2.0f * a12 * X1 + a1;
    const V z3 = -0.5f * dyyy * X1 * X1 + 3.0f * c[2] * X1 + 3.0f * a2 - 3.0f * a22 * X1;
    gc[0] = vfma(v0 * Gxxx + v1 * S1 + v2 * S2 + v3 * Gyyy, G, gc[0]);
    gc[1] = vfma(w0 * Gxxx + w1 * S1 + w2 * S2 + w3 * Gyyy, G, gc[1]);
    gc[2] = vfma(z0 * Gxxx + z1 * S1 + z2 * S2 + z3 * Gyyy, G, gc[2]);
    }
    }
}

// ---------------------------------------------------------------------------------------
// Moment form of the derivative / laplacian / third backward (D = 2, C = 1).
//
// Every output is v G(X) t_u(a, c) with a = A X (forward.cu:225-332), so with the sample's
// dL summed over symmetric components, h_u, the pair's loss is L = v G phi, phi = sum_u h_u t_u.
// Writing g = d phi / d a and e_i = d phi / d c_i (explicit c only), the reference's gradients
// (backward.cu:108-416, the autograd of the forward) are
//   dL/dv  = G phi
//   dL/dm  = v G (A g - phi A X)                         = v A (G g - G phi X)
//   dL/dc0 = v G (-1/2 X0^2 phi + g0 X0 + e0)
//   dL/dc1 = v G (-X0 X1 phi + g0 X1 + g1 X0 + e1)       (c1 is both off-diagonal entries)
//   dL/dc2 = v G (-1/2 X1^2 phi + g1 X1 + e2)
// A and v are per Gaussian, so the pair loop accumulates kMomAcc sums per lane
//   [S G phi | S G g0 | S G g1 | S G phi X0 | S G phi X1 | S G phi X0X0 | X0X1 | X1X1 |
//    S G (g0 X0 + e0) | S G (g0 X1 + g1 X0 + e1) | S G (g1 X1 + e2)]
// and bwd_mom_finish contracts them once per unit.  The sample row carries pre-scaled h
// coefficients (k_pack_samples, mom_coef): derivative [h0 h1], laplacian [h0 h1 h2 2h0 2h2],
// third [3h0 h1 2h1 h2 2h2 3h3].  For the third, phi is evaluated as (a.g + 2 c.e) / 3
// (Euler's identity on the cubic and linear parts of phi: a.g = 3 cubic + linear, and the
// linear part is c.e).
// Per pair: 34 / 43 / 54 VALU ops against 46 / 103 / 140 for the reference-literal terms.
// The fused form (FN = kMulti + mask) sums phi, g and e over the mask's functions: all four
// cost ~75 ops per pair against 34 + 43 + 54 + 16 in four separate passes.
// ---------------------------------------------------------------------------------------
#ifndef DGS_HMOM
#define DGS_HMOM 1
#endif
constexpr int kMomAcc = 11;

template <int FN, int D, int CB>
__host__ __device__ constexpr bool bwd_mom() {
    return is_multi(FN) || (DGS_HMOM && D == 2 && CB == 1 && FN >= 1);
}

// Sample-row coefficients of function f (after s0, s1) from its h (dL summed over symmetric
// components): gaussian [h], derivative [h0 h1], laplacian [h0 h1 h2 2h0 2h2],
// third [3h0 h1 2h1 h2 2h2 3h3].
__host__ __device__ inline void mom_coef(int f, const float *h, float *o) {
    if (f == 0) { o[0] = h[0]; }
    else if (f == 1) { o[0] = h[0]; o[1] = h[1]; }
    else if (f == 2) { o[0] = h[0]; o[1] = h[1]; o[2] = h[2]; o[3] = 2.0f * h[0]; o[4] = 2.0f * h[2]; }
    else { o[0] = 3.0f * h[0]; o[1] = h[1]; o[2] = 2.0f * h[1]; o[3] = h[2]; o[4] = 2.0f * h[2]; o[5] = 3.0f * h[3]; }
}

// One pair of the moment form for the functions of mask M (the fused form sums phi, g and e
// over them: the loss of a fused call is the sum of the functions' losses).
template <int FN, typename V>
__device__ __forceinline__ void bwd_mom_terms(const V *X, const float *c, V G, const V *f, V *acc) {
    constexpr int M = fn_mask(FN);
    const V X0 = X[0], X1 = X[1];
    const V a1 = vfma(bc<V>(c[1]), X1, c[0] * X0);
    const V a2 = vfma(bc<V>(c[1]), X0, c[2] * X1);
    V phi = bc<V>(0.0f), g0 = bc<V>(0.0f), g1 = bc<V>(0.0f);
    V e0 = bc<V>(0.0f), e1 = bc<V>(0.0f), e2 = bc<V>(0.0f);
    constexpr bool HAS_E = (M & 12) != 0;
    if constexpr ((M & 1) != 0) phi = f[mask_foff(M, 0)];
    if constexpr ((M & 2) != 0) {
        const V *h = f + mask_foff(M, 1);
        phi = vfma(h[0], a1, vfma(h[1], a2, phi));
        g0 = h[0];
        g1 = h[1];
    }
    if constexpr ((M & 4) != 0) {
        const V *h = f + mask_foff(M, 2);
        const V t0 = vfma(a1, a1, bc<V>(-c[0])), t1 = vfma(a1, a2, bc<V>(-c[1])),
                t2 = vfma(a2, a2, bc<V>(-c[2]));
        phi = vfma(h[2], t2, vfma(h[1], t1, vfma(h[0], t0, phi)));
        g0 = vfma(h[3], a1, vfma(h[1], a2, g0));
        g1 = vfma(h[4], a2, vfma(h[1], a1, g1));
        e0 = -h[0];
        e1 = -h[1];
        e2 = -h[2];
    }
    if constexpr ((M & 8) != 0) {
        const V *h = f + mask_foff(M, 3);
        const V p = vfma(-a1, a1, bc<V>(c[0])), r = vfma(-a1, a2, bc<V>(c[1])),
                s = vfma(-a2, a2, bc<V>(c[2]));
        const V q0 = vfma(h[3], s, vfma(h[2], r, h[0] * p));
        const V q1 = vfma(h[5], s, vfma(h[4], r, h[1] * p));
        const V E0 = vfma(h[0], a1, h[1] * a2);
        const V E1 = vfma(h[2], a1, h[4] * a2);
        const V E2 = vfma(h[3], a1, h[5] * a2);
        const V l = vfma(bc<V>(c[2]), E2, vfma(bc<V>(c[1]), E1, c[0] * E0));
        // 3 phi_third = a.g + 2 c.e (Euler's identity, see above)
        phi = vfma(vfma(bc<V>(2.0f), l, vfma(a2, q1, a1 * q0)), bc<V>(1.0f / 3.0f), phi);
        g0 += q0;
        g1 += q1;
        e0 += E0;
        e1 += E1;
        e2 += E2;
    }
    const V t = G * phi, u0 = G * g0, u1 = G * g1;
    const V tx = t * X0, ty = t * X1;
    acc[0] += t;
    acc[1] += u0;
    acc[2] += u1;
    acc[3] += tx;
    acc[4] += ty;
    acc[5] = vfma(tx, X0, acc[5]);
    acc[6] = vfma(tx, X1, acc[6]);
    acc[7] = vfma(ty, X1, acc[7]);
    acc[8] = vfma(u0, X0, acc[8]);
    acc[9] = vfma(u1, X0, vfma(u0, X1, acc[9]));
    acc[10] = vfma(u1, X1, acc[10]);
    if constexpr (HAS_E) {
        acc[8] = vfma(G, e0, acc[8]);
        acc[9] = vfma(G, e1, acc[9]);
        acc[10] = vfma(G, e2, acc[10]);
    }
}

// Sums -> (dmeans, dconics, dvalues) of one Gaussian (c: conic, v: value).
__device__ __forceinline__ void bwd_mom_finish(const float *c, float v, const float *s, float *gm,
                                               float *gc, float &gv) {
    gv = s[0];
    const float M0 = s[1] - s[3], M1 = s[2] - s[4];
    gm[0] = v * fmaf(c[0], M0, c[1] * M1);
    gm[1] = v * fmaf(c[1], M0, c[2] * M1);
    gc[0] = v * fmaf(-0.5f, s[5], s[8]);
    gc[1] = v * (s[9] - s[6]);
    gc[2] = v * fmaf(-0.5f, s[7], s[10]);
}

// Epilogue of the gaussian moment form: convert moments to gradients.
template <int FN, int D>
__device__ __forceinline__ void bwd_finish(const float *c, float *gm, float *gc) {
    if constexpr (FN != 0) {
        return;
    } else if constexpr (D == 1) {
        gm[0] = -c[0] * gm[0];
        gc[0] = -0.5f * gc[0];
    } else {
    const float sx = gm[0], sy = gm[1];
    gm[0] = -fmaf(c[0], sx, c[1] * sy);
    gm[1] = -fmaf(c[1], sx, c[2] * sy);
    gc[0] = -0.5f * gc[0];
    gc[1] = -gc[1];
    gc[2] = -0.5f * gc[2];
    }
}

}  // namespace dgs
