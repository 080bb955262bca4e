/*
 * oracle.c -- CPU restatement of the kr4b/diff-gaussian-sampling sampler path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or as the timed CPU
 * baseline).  The product path (diff_gaussian_sampling + libdgs.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned".  The reference is CUDA-only (nvcc, cub, cooperative
 * groups, an un-vendored glm submodule) and cannot be built or run in this image, and it
 * ships no tests, fixtures or golden vectors.  This restatement is
 * instead pinned by (a) autograd: every backward formula equals torch.autograd of the
 * matching forward (except the reference's own D=1 third-derivative conic gradient,
 * backward.cu:322-325, which is reproduced literally and pinned by a literal transcription
 * test), (b) closed-form known answers, and (c) torch's own CUDA-path arithmetic for the
 * tile grid (tests/test_gpu_parity.py::test_tile_grid_matches_torch_cuda_semantics).
 *
 * Arithmetic is literal: float where the reference uses FLOAT, double where the reference's
 * double literals promote (e.g. `-0.5 * (...)`, `3.0 * sqrt(...)`), expf/sqrtf/floorf for the
 * CUDA float overloads of exp/sqrt/floor.
 *
 * FMA CONTRACTION MODELS (ORC_FMAD, one library per model; oracle/Makefile):
 *   0  liboracle.so            gcc -ffp-contract=off: every product and sum rounded on its own
 *                              (the model the GPU path and the parity tests are built against);
 *   1  liboracle_fmad.so       clang -ffp-contract=fast -mfma: nvcc's default --fmad=true (the
 *                              reference's setup.py:30 passes no --fmad=false) modelled by LLVM's
 *                              own DAG contraction of the same expressions (NVVM is LLVM-based):
 *                              every a*b +- c whose product feeds one add is fused; where both
 *                              operands of an add are products (SUM2), LLVM fuses the LEFT one;
 *   2  liboracle_fmad_alt.so   as 1, but every SUM2 site fuses the RIGHT product (the other legal
 *                              choice of a contracting compiler at `a*b +- c*d`).
 * The reference's atomicAdd(ptr, term) cannot fuse its addend: ACC() keeps the term rounded in
 * every model.  Nothing here is the nvcc binary: the models bracket what it can do
 * (tools/contraction_study.py, profiles/r05_contraction.json).
 *
 * Every function cites the reference file:line it follows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_TILE 0.51f /* config.h:18 BLOCK_SIZE */

#include "oracle_fmad.h"

int orc_fmad_model(void) { return ORC_FMAD; }

typedef struct {
    int P, D, N;
    int grid[2];
    int T;
    float off[2];
    int64_t R;        /* num_rendered: sum of tiles_touched (sampler_impl.cu:253-257) */
    int64_t *gstart;  /* [T+1] CSR over tiles of the per-tile Gaussian lists         */
    int32_t *glist;   /* ascending gid inside each tile (unique (tile<<32|gid) keys) */
    int64_t *sstart;  /* [T+1] CSR over tiles of the per-tile sample lists           */
    int32_t *slist;   /* ascending sid inside each tile                              */
    int32_t *skey;    /* [N] sample tile key (may be >= T: never rendered)           */
    uint32_t *ranges; /* [2T] reference-layout uint2 ranges (sampler_impl.cu:134-151) */
    uint32_t *sranges;
} orc_bins;

/* float -> int as the CUDA cvt.rzi/rmi.s32.f32 instructions do it: saturating, NaN -> 0. */
static int sat_int(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

/* sample_points.cu:70-74.  min/max over samples, then
 *   tile_grid = ceil((max - min + 1e-6f) / BLOCK_SIZE)
 * evaluated by torch on the CUDA device.  ATen's div_true_kernel_cuda turns division by a
 * CPU scalar into a multiplication by the opmath (float) reciprocal, so the CUDA result is
 * ceil(ext * (1.0f / 0.51f)); tests pin this against torch's own GPU op. */
void orc_tile_grid(int N, int D, const float *samples, int *grid, float *off) {
    for (int d = 0; d < 2; ++d) { grid[d] = 1; off[d] = 0.0f; }
    for (int d = 0; d < D; ++d) {
        float mn = samples[d], mx = samples[d];
        for (int i = 1; i < N; ++i) {
            float v = samples[(int64_t)i * D + d];
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
        volatile float ext = (mx - mn) + 1e-6f;
        volatile float inv = 1.0f / ORC_TILE;
        volatile float q = ext * inv;
        grid[d] = (int)ceilf(q);
        off[d] = mn;
    }
}

/* forward.cu:52-61 -- radius of the 3-sigma box; returns 0 when the Gaussian is skipped. */
static float ref_radius(int D, const float *cov) {
    if (D == 1) return (float)(3.0 * (double)sqrtf(cov[0]));
    float det = SUM2(cov[0], cov[2], -cov[1], cov[1]); /* forward.cu:55 */
    if (det == 0.0f) return 0.0f;
    float mid = 0.5f * (cov[0] + cov[2]);
    float disc = FMA(mid, mid, -det); /* forward.cu:59 */
    double floor_disc = fmax(1e-6, (double)disc); /* CUDA max(double, float) */
    float lambda = (float)((double)mid + sqrt(floor_disc));
    return (float)(3.0 * (double)sqrtf(lambda));
}

/* auxiliary.h:21-31 (TORUS branch) */
static void ref_rect(int D, const float *p, float r, const float *off, int *rmin, int *rmax) {
    for (int i = 0; i < D; ++i) {
        float lo = ((p[i] - off[i]) - r) / ORC_TILE;
        float hi = ((p[i] - off[i]) + r) / ORC_TILE;
        rmin[i] = sat_int(floorf(lo));
        rmax[i] = sat_int(ceilf(hi));
    }
}

/* forward.cu:24-83 -- tiles touched; radius stored only when touched != 0. */
static uint32_t ref_touched(int D, const float *mean, const float *cov, const int *grid,
                            const float *off, float *radius_out) {
    *radius_out = 0.0f;
    if (D == 2) {
        float det = SUM2(cov[0], cov[2], -cov[1], cov[1]);
        if (det == 0.0f) return 0;
    }
    float r = ref_radius(D, cov);
    int rmin[2], rmax[2];
    ref_rect(D, mean, r, off, rmin, rmax);
    int t0 = rmax[0] - rmin[0];
    if (t0 > grid[0]) t0 = grid[0];
    uint32_t touched;
    if (D == 1) {
        touched = (uint32_t)t0;
    } else {
        int t1 = rmax[1] - rmin[1];
        if (t1 > grid[1]) t1 = grid[1];
        touched = (uint32_t)(t1 * t0);
    }
    if (touched == 0) return 0;
    *radius_out = r;
    return touched;
}

static int wrap_tile(int x, int g) { return x < 0 ? (g + (x % g)) : (x % g); } /* sampler_impl.cu:88-89 */

/* sampler_impl.cu:54-129 -- enumerate the tile keys of one Gaussian, in emission order. */
static int ref_keys(int D, const float *mean, float r, const int *grid, const float *off,
                    uint32_t *keys) {
    int rmin[2], rmax[2], n = 0;
    ref_rect(D, mean, r, off, rmin, rmax);
    if (rmax[0] - rmin[0] >= grid[0]) { rmin[0] = 0; rmax[0] = grid[0]; }
    if (D == 1) {
        for (int x = rmin[0]; x < rmax[0]; ++x) keys[n++] = (uint32_t)wrap_tile(x, grid[0]);
        return n;
    }
    if (rmax[1] - rmin[1] >= grid[1]) { rmin[1] = 0; rmax[1] = grid[1]; }
    for (int y = rmin[1]; y < rmax[1]; ++y)
        for (int x = rmin[0]; x < rmax[0]; ++x)
            keys[n++] = (uint32_t)(wrap_tile(y, grid[1]) * grid[0] + wrap_tile(x, grid[0]));
    return n;
}

/* sampler_impl.cu:155-189 -- sample tile key (clamped to [0, grid], not grid-1). */
static uint32_t ref_sample_key(int D, const float *s, const int *grid, const float *off) {
    uint32_t tile[2] = {0, 0};
    for (int i = 0; i < D; ++i) {
        int t = sat_int((s[i] - off[i]) / ORC_TILE);
        if (t < 0) t = 0;
        if (t > grid[i]) t = grid[i];
        tile[i] = (uint32_t)t;
    }
    return D == 1 ? tile[0] : tile[1] * (uint32_t)grid[0] + tile[0];
}

void orc_free(orc_bins *b) {
    if (!b) return;
    free(b->gstart); free(b->glist); free(b->sstart); free(b->slist); free(b->skey);
    free(b->ranges); free(b->sranges); free(b);
}

/* sample_points.cu:38-98 + sampler_impl.cu:216-330.  grid/off may be given (sharded runs
 * use the global grid); pass grid == NULL to derive them from `samples` as the reference
 * does.  Writes radii[P].  Returns NULL on allocation failure. */
orc_bins *orc_bin(int P, int D, int N, const float *means, const float *covs,
                  const float *samples, const int *grid_in, const float *off_in, float *radii) {
    orc_bins *b = (orc_bins *)calloc(1, sizeof(orc_bins));
    if (!b) return NULL;
    b->P = P; b->D = D; b->N = N;
    if (grid_in) {
        b->grid[0] = grid_in[0]; b->grid[1] = D == 2 ? grid_in[1] : 1;
        b->off[0] = off_in[0]; b->off[1] = D == 2 ? off_in[1] : 0.0f;
    } else {
        orc_tile_grid(N, D, samples, b->grid, b->off);
    }
    b->T = D == 1 ? b->grid[0] : b->grid[0] * b->grid[1];
    const int T = b->T, S = D * (D + 1) / 2;
    b->gstart = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    b->sstart = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    b->ranges = (uint32_t *)calloc((size_t)2 * T, sizeof(uint32_t));
    b->sranges = (uint32_t *)calloc((size_t)2 * T, sizeof(uint32_t));
    b->skey = (int32_t *)calloc((size_t)N + 1, sizeof(int32_t));
    uint32_t *keys = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)T + 1));
    if (!b->gstart || !b->sstart || !b->ranges || !b->sranges || !b->skey || !keys) {
        free(keys); orc_free(b); return NULL;
    }
    /* pass 1: radii, R, per-tile counts */
    int64_t *gcount = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    for (int g = 0; g < P; ++g) {
        float r;
        uint32_t touched = ref_touched(D, means + (int64_t)g * D, covs + (int64_t)g * S,
                                       b->grid, b->off, &r);
        radii[g] = r;
        b->R += touched;
        if (r > 0.0f) {
            int n = ref_keys(D, means + (int64_t)g * D, r, b->grid, b->off, keys);
            for (int k = 0; k < n; ++k)
                if (keys[k] < (uint32_t)T) gcount[keys[k]]++;
        }
    }
    for (int t = 0; t < T; ++t) b->gstart[t + 1] = b->gstart[t] + gcount[t];
    b->glist = (int32_t *)malloc(sizeof(int32_t) * ((size_t)b->gstart[T] + 1));
    memset(gcount, 0, sizeof(int64_t) * ((size_t)T + 1));
    /* pass 2: fill -- gid-ascending scan gives the (tile<<32 | gid) sorted order per tile */
    for (int g = 0; g < P; ++g) {
        if (!(radii[g] > 0.0f)) continue;
        int n = ref_keys(D, means + (int64_t)g * D, radii[g], b->grid, b->off, keys);
        for (int k = 0; k < n; ++k)
            if (keys[k] < (uint32_t)T) b->glist[b->gstart[keys[k]] + gcount[keys[k]]++] = g;
    }
    /* samples */
    int64_t *scount = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    for (int i = 0; i < N; ++i) {
        uint32_t k = ref_sample_key(D, samples + (int64_t)i * D, b->grid, b->off);
        b->skey[i] = (int32_t)k;
        if (k < (uint32_t)T) scount[k]++;
    }
    for (int t = 0; t < T; ++t) b->sstart[t + 1] = b->sstart[t] + scount[t];
    b->slist = (int32_t *)malloc(sizeof(int32_t) * ((size_t)b->sstart[T] + 1));
    memset(scount, 0, sizeof(int64_t) * ((size_t)T + 1));
    for (int i = 0; i < N; ++i) {
        uint32_t k = (uint32_t)b->skey[i];
        if (k < (uint32_t)T) b->slist[b->sstart[k] + scount[k]++] = i;
    }
    /* identifyTileRanges (sampler_impl.cu:134-151): empty tiles keep (0,0) */
    for (int t = 0; t < T; ++t) {
        if (b->gstart[t + 1] > b->gstart[t]) {
            b->ranges[2 * t] = (uint32_t)b->gstart[t];
            b->ranges[2 * t + 1] = (uint32_t)b->gstart[t + 1];
        }
        if (b->sstart[t + 1] > b->sstart[t]) {
            b->sranges[2 * t] = (uint32_t)b->sstart[t];
            b->sranges[2 * t + 1] = (uint32_t)b->sstart[t + 1];
        }
    }
    free(gcount); free(scount); free(keys);
    return b;
}

int orc_T(const orc_bins *b) { return b->T; }
int64_t orc_R(const orc_bins *b) { return b->R; }
void orc_grid(const orc_bins *b, int *grid, float *off) {
    grid[0] = b->grid[0]; grid[1] = b->grid[1]; off[0] = b->off[0]; off[1] = b->off[1];
}
void orc_ranges(const orc_bins *b, uint32_t *ranges, uint32_t *sranges) {
    memcpy(ranges, b->ranges, sizeof(uint32_t) * 2 * (size_t)b->T);
    memcpy(sranges, b->sranges, sizeof(uint32_t) * 2 * (size_t)b->T);
}
void orc_sample_keys(const orc_bins *b, int32_t *keys) {
    memcpy(keys, b->skey, sizeof(int32_t) * (size_t)b->N);
}
int64_t orc_tile_gaussians(const orc_bins *b, int t, int32_t *out) {
    int64_t n = b->gstart[t + 1] - b->gstart[t];
    if (out) memcpy(out, b->glist + b->gstart[t], sizeof(int32_t) * (size_t)n);
    return n;
}

/* forward.cu:149-157 / backward.cu:89-97 -- period-2 torus wrap of one displacement. */
static float ref_wrap(float x) {
    if (fabsf(x) > 1.0) {
        if (x >= 0) x = (float)(fmod((double)x, 2.0) - 2.0);
        else x = (float)(fmod((double)x, 2.0) + 2.0);
    }
    return x;
}

enum { F_GAUSS = 0, F_DERIV = 1, F_LAPL = 2, F_THIRD = 3 };

static int out_comps(int fn, int D) {
    int k = 1;
    for (int i = 0; i < fn; ++i) k *= D;
    return k;
}

/* forward.cu:168-275 -- one pair's contribution, accumulated into o[comp*C + ch].  Contraction
 * sites (ORC_FMAD): the exponent's float sum (forward.cu:177,199,223,252: SUM2), a1/a2 and the
 * laplacian terms (FMA), and every `out += values*alpha*t` (forward.cu:182 ff.: FMA into out). */
static void fwd_pair(int fn, int D, int C, const float *X, const float *c, const float *v, float *o) {
    if (D == 1) {
        float x1 = c[0] * X[0];
        float power = fn == F_GAUSS ? (float)(-0.5 * c[0] * X[0] * X[0]) : (float)(-0.5 * x1 * X[0]);
        if (power > 0.0) return;
        float a = expf(power);
        for (int ch = 0; ch < C; ++ch) {
            float va = v[ch] * a;
            switch (fn) {
            case F_GAUSS: o[ch] = FMA(v[ch], a, o[ch]); break;
            case F_DERIV: o[ch] = FMA(va, x1, o[ch]); break;
            case F_LAPL: o[ch] = FMA(va, FMA(x1, x1, -c[0]), o[ch]); break;
            default: {
                double t = 2.0 * c[0] * x1 - (double)(x1 * x1 * x1) + (double)(c[0] * x1);
#if ORC_FMAD
                o[ch] = (float)fma((double)va, t, (double)o[ch]);
#else
                o[ch] = (float)((double)o[ch] + (double)va * t);
#endif
            }
            }
        }
        return;
    }
    float power;
    float x1 = c[0] * X[0], x2 = c[2] * X[1];
    if (fn == F_GAUSS)
        power = (float)(-0.5 * (double)SUM2(c[0] * X[0], X[0], c[2] * X[1], X[1]) - (double)(c[1] * X[0] * X[1]));
    else
        power = (float)(-0.5 * (double)SUM2(x1, X[0], x2, X[1]) - (double)(c[1] * X[0] * X[1]));
    if (power > 0.0) return;
    float a = expf(power);
    float a1 = FMA(c[1], X[1], x1), a2 = FMA(c[1], X[0], x2);
    float t[4];
    switch (fn) {
    case F_GAUSS: break;
    case F_DERIV: t[0] = a1; t[1] = a2; break;
    case F_LAPL: t[0] = FMA(a1, a1, -c[0]); t[1] = FMA(a1, a2, -c[1]); t[2] = FMA(a2, a2, -c[2]); break;
    default:
        t[0] = (float)(3.0 * c[0] * a1 - (double)(a1 * a1 * a1));
        t[1] = (float)(2.0 * c[1] * a1 - (double)(a1 * a1 * a2) + (double)(c[0] * a2));
        t[2] = (float)(2.0 * c[1] * a2 - (double)(a1 * a2 * a2) + (double)(c[2] * a1));
        t[3] = (float)(3.0 * c[2] * a2 - (double)(a2 * a2 * a2));
    }
    /* expanded component -> unique term: laplacian [xx,xy,yx,yy]; third [xxx,xxy,xyx,xyy,yxx,yxy,yyx,yyy] */
    static const int lap_map[4] = {0, 1, 1, 2};
    static const int third_map[8] = {0, 1, 1, 2, 1, 2, 2, 3};
    for (int ch = 0; ch < C; ++ch) {
        float va = v[ch] * a;
        switch (fn) {
        case F_GAUSS: o[ch] = FMA(v[ch], a, o[ch]); break;
        case F_DERIV: o[ch] = FMA(va, t[0], o[ch]); o[C + ch] = FMA(va, t[1], o[C + ch]); break;
        case F_LAPL: for (int k = 0; k < 4; ++k) o[k * C + ch] = FMA(va, t[lap_map[k]], o[k * C + ch]); break;
        default: for (int k = 0; k < 8; ++k) o[k * C + ch] = FMA(va, t[third_map[k]], o[k * C + ch]);
        }
    }
}

/* backward.cu:108-416 (oracle_bwd_body.h): bwd_pair (float sums) and bwd_pair64 (exact sums) */
#define BWD_T float
#define BWD_FN(name) name
#include "oracle_bwd_body.h"
#undef BWD_T
#undef BWD_FN
#define BWD_T double
#define BWD_FN(name) name##64
#include "oracle_bwd_body.h"
#undef BWD_T
#undef BWD_FN

static void displacement(int D, const float *m, const float *s, float *X) {
    for (int k = 0; k < D; ++k) X[k] = ref_wrap(m[k] - s[k]);
}

/* forward.cu:87-166 (render) for samples `sub` (NULL = all); out is [N][K][C], accumulated
 * in ascending-gid order exactly like the reference's per-thread loop.  Samples whose key
 * is >= T are never rendered (left untouched). */
void orc_forward(const orc_bins *b, int fn, int C, const float *means, const float *values,
                 const float *conics, const float *samples, float *out, int nsub, const int32_t *sub) {
    const int D = b->D, S = D * (D + 1) / 2, K = out_comps(fn, D);
    int count = sub ? nsub : b->N;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        float *o = out + (int64_t)sid * K * C;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            fwd_pair(fn, D, C, X, conics + (int64_t)g * S, values + (int64_t)g * C, o);
        }
    }
}

/* backward.cu:26-106 -- gradient accumulation (serial order; the reference's atomic order
 * is nondeterministic).  Grads are accumulated into dmeans[P][D], dvalues[P][C], dconics[P][S]
 * (caller zero-initialises).  Only samples in `sub` contribute (NULL = all). */
void orc_backward(const orc_bins *b, int fn, int C, const float *means, const float *values,
                  const float *conics, const float *samples, const float *dL_dout, float *dmeans,
                  float *dvalues, float *dconics, int nsub, const int32_t *sub) {
    const int D = b->D, S = D * (D + 1) / 2, K = out_comps(fn, D);
    int count = sub ? nsub : b->N;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        const float *dL = dL_dout + (int64_t)sid * K * C;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            bwd_pair(fn, D, C, X, conics + (int64_t)g * S, values + (int64_t)g * C, dL,
                     dmeans + (int64_t)g * D, dvalues + (int64_t)g * C, dconics + (int64_t)g * S);
        }
    }
}

/* orc_backward with exact (double) sums of the same float per-pair terms: the value around
 * which every atomic order of the reference scatters; the GPU parity tests' gradient reference.  Grads are accumulated into dmeans[P][D], dvalues[P][C], dconics[P][S]
 * (caller zero-initialises).  Only samples in `sub` contribute (NULL = all). */
void orc_backward64(const orc_bins *b, int fn, int C, const float *means, const float *values,
                    const float *conics, const float *samples, const float *dL_dout, double *dmeans,
                    double *dvalues, double *dconics, int nsub, const int32_t *sub) {
    const int D = b->D, S = D * (D + 1) / 2, K = out_comps(fn, D);
    int count = sub ? nsub : b->N;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        const float *dL = dL_dout + (int64_t)sid * K * C;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            bwd_pair64(fn, D, C, X, conics + (int64_t)g * S, values + (int64_t)g * C, dL,
                     dmeans + (int64_t)g * D, dvalues + (int64_t)g * C, dconics + (int64_t)g * S);
        }
    }
}

/* Diagnostic: pairs of the reference pair set with power >= thr (W_live for thr = -104) and
 * the total pair count (W_ref), over samples `sub` (NULL = all). */
void orc_count_pairs(const orc_bins *b, const float *means, const float *conics, const float *samples,
                     double thr, int nsub, const int32_t *sub, int64_t *w_ref, int64_t *w_live) {
    const int D = b->D, S = D * (D + 1) / 2;
    int count = sub ? nsub : b->N;
    int64_t ref = 0, live = 0;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            const float *c = conics + (int64_t)g * S;
            double p = D == 1 ? -0.5 * c[0] * X[0] * X[0]
                              : -0.5 * ((double)c[0] * X[0] * X[0] + (double)c[2] * X[1] * X[1]) - (double)c[1] * X[0] * X[1];
            ref++;
            if (p >= thr && p <= 0.0) live++;
        }
    }
    *w_ref = ref;
    *w_live = live;
}

/* A-PRIORI BOUND of the exponent's evaluation order.  The reference
 * evaluates power = -0.5 (c0 X0 X0 + c2 X1 X1) - c1 X0 X1 (forward.cu:177, 199, 223, 252;
 * backward.cu:110 ff.) in SOME fp32 operation order: unfused (gcc), contracted by nvcc's default
 * --fmad=true in either of its legal ways, or -- on the GPU path -- pre-scaled by log2(e) and
 * summed with FMAs.  Every such order rounds each of the three terms through at most
 * ORC_ORDER_OPS operations (the coefficient's scaling, two products, two sums, the final
 * rounding), so |power_any - power_exact| <= gamma_k * M, M = 0.5|c0 X0^2| + |c1 X0 X1| +
 * 0.5|c2 X1^2| (standard floating-point summation analysis; gamma_k = k u / (1 - k u), u = 2^-24).
 * Every output and gradient term of the pair is exp(power) times factors that do not depend on
 * power, so the term moves by at most |term| (exp(gamma_k M) - 1) ~ |term| gamma_k M.  The bound
 * of an element is the sum of that over its pairs -- it depends only on the reference's
 * expression and the inputs, not on any GPU result.  The thin-Gaussian parity tests state
 *   |gpu - ref| <= 1e-5 |ref| + 1e-6 max|ref| + B.
 * (At well-conditioned conics M ~ |power| and B is far below the 8c bound; cancellation at
 * rho^2 -> 1 makes M >> |power|: there no order is "the reference's".) */
#define ORC_ORDER_OPS 6

static double pair_mag(int D, const float *X, const float *c) {
    if (D == 1) return 0.5 * fabs((double)c[0] * X[0] * X[0]);
    return 0.5 * fabs((double)c[0] * X[0] * X[0]) + fabs((double)c[1] * X[0] * X[1]) + 0.5 * fabs((double)c[2] * X[1] * X[1]);
}

static double order_gamma(void) {
    const double u = ldexp(1.0, -24), k = ORC_ORDER_OPS;
    return k * u / (1.0 - k * u);
}

/* bound[N][K][C] (double, caller zero-initialises): the forward's per-element B. */
void orc_forward_bound(const orc_bins *b, int fn, int C, const float *means, const float *values,
                       const float *conics, const float *samples, double *bound, int nsub, const int32_t *sub) {
    const int D = b->D, S = D * (D + 1) / 2, K = out_comps(fn, D);
    const double gam = order_gamma();
    float *tmp = (float *)malloc(sizeof(float) * (size_t)K * C);
    int count = sub ? nsub : b->N;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        double *o = bound + (int64_t)sid * K * C;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            const float *c = conics + (int64_t)g * S;
            memset(tmp, 0, sizeof(float) * (size_t)K * C);
            fwd_pair(fn, D, C, X, c, values + (int64_t)g * C, tmp); /* this pair's terms */
            const double e = expm1(gam * pair_mag(D, X, c));
            for (int k = 0; k < K * C; ++k) o[k] += fabs((double)tmp[k]) * e;
        }
    }
    free(tmp);
}

/* The gradients' per-element B (dmeans[P][D], dvalues[P][C], dconics[P][S], double, caller
 * zero-initialises): the same per-pair rule over the pair's float gradient terms. */
void orc_backward_bound(const orc_bins *b, int fn, int C, const float *means, const float *values,
                        const float *conics, const float *samples, const float *dL_dout, double *dmeans,
                        double *dvalues, double *dconics, int nsub, const int32_t *sub) {
    const int D = b->D, S = D * (D + 1) / 2, K = out_comps(fn, D);
    const double gam = order_gamma();
    double *tv = (double *)malloc(sizeof(double) * (size_t)C);
    int count = sub ? nsub : b->N;
    for (int q = 0; q < count; ++q) {
        int sid = sub ? sub[q] : q;
        uint32_t t = (uint32_t)b->skey[sid];
        if (t >= (uint32_t)b->T) continue;
        const float *dL = dL_dout + (int64_t)sid * K * C;
        for (int64_t j = b->gstart[t]; j < b->gstart[t + 1]; ++j) {
            int g = b->glist[j];
            float X[2];
            displacement(D, means + (int64_t)g * D, samples + (int64_t)sid * D, X);
            const float *c = conics + (int64_t)g * S;
            double tm[2] = {0.0, 0.0}, tc[3] = {0.0, 0.0, 0.0};
            memset(tv, 0, sizeof(double) * (size_t)C);
            bwd_pair64(fn, D, C, X, c, values + (int64_t)g * C, dL, tm, tv, tc); /* this pair's terms */
            const double e = expm1(gam * pair_mag(D, X, c));
            for (int k = 0; k < D; ++k) dmeans[(int64_t)g * D + k] += fabs(tm[k]) * e;
            for (int k = 0; k < C; ++k) dvalues[(int64_t)g * C + k] += fabs(tv[k]) * e;
            for (int k = 0; k < S; ++k) dconics[(int64_t)g * S + k] += fabs(tc[k]) * e;
        }
    }
    free(tv);
}
