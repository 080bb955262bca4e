/*
 * dgs_volume.h -- C ABI of the D = 3 Gaussian sampler, in libdgs.so.
 *
 * Beyond the reference: its device functions have no D = 3 branch (forward.cu:164-275,
 * backward.cu:108-416), its radius is 0 there (forward.cu:52-61) and its sample keys are left
 * uninitialised (sampler_impl.cu:177-182), so at D = 3 it renders nothing.  This path is the
 * reference's per-pair arithmetic carried to three dimensions:
 *   X_d   = mean_d - sample_d, wrapped as forward.cu:149-157 does per axis (period 2)
 *   power = -0.5f * (c00 X0 X0 + c11 X1 X1 + c22 X2 X2) - (c01 X0 X1 + c02 X0 X2 + c12 X1 X2),
 *           conics packed [c00 c01 c02 c11 c12 c22] (the reference's D(D+1)/2 row-major
 *           upper triangle, sample_points.cu:40); a pair with power > 0 is skipped
 *   a     = A X;  outputs v G t with G = expf(power) and
 *           gaussian t = 1, derivative t_i = a_i, laplacian t_ij = a_i a_j - A_ij,
 *           third t_ijk = A_ij a_k + A_ik a_j + A_jk a_i - a_i a_j a_k
 *           (the D = 2 expressions of forward.cu:164-275 in index form)
 * summed over EVERY Gaussian (no tile truncation: a pair is left out only when its
 * contribution is exactly 0 in fp32, i.e. X^T A X > 210 for a well-conditioned positive-
 * definite conic; other Gaussians are evaluated against every sample).
 *
 * Same conventions as dgs.h: device pointers, fp32 row-major, asynchronous on `stream`
 * except dgs_volume_preprocess (one host sync), buffers from the caller.
 */
#ifndef DGS_VOLUME_H_INCLUDED
#define DGS_VOLUME_H_INCLUDED

#include "dgs.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Binning of a D = 3 field: Gaussians and samples sorted into one uniform grid of cells no
 * smaller than the largest exact-zero cut half-width.  means[P][3], conics[P][6], samples[N][3].
 * The opaque buffer (DGS_BUF_BINNING) is requested through `alloc`; scratch as DGS_BUF_SCRATCH.
 * Synchronises `stream` once (bounds, to size the grid).  forward/backward must be given the
 * same means, conics and samples (re-bin when they change): every forward / backward /
 * count_pairs call compares its tensors bitwise with the binned ones on the device (no sync)
 * and, on a difference, writes NaN to every output, as for a stale buffer (count_pairs
 * returns DGS_ERR_BUFFER).  The buffer holds the flag word these calls reset and set, so the
 * calls on one binning must be ordered (one stream, or events between streams): two
 * concurrent calls could clear each other's flag. */
int dgs_volume_preprocess(int P, int N, const float *means, const float *conics,
                          const float *samples, dgs_alloc_fn alloc, void *alloc_ctx,
                          dgs_stream_t stream, int debug);

/* Workspace bytes of dgs_volume_backward (0 for the forward). */
size_t dgs_volume_workspace_size(int function, int P, int N, int C, int backward);

/* out[N][3^function][C] (every entry written; symmetric entries repeated, as the reference's
 * D = 2 outputs are). */
int dgs_volume_forward(int function, int P, int N, int C, const float *means, const float *values,
                       const float *conics, const float *samples, const void *binning,
                       size_t binning_bytes, float *out, dgs_stream_t stream, int debug);

/* dL_dout[N][3^function][C]; writes (overwrites) dL_dmeans[P][3], dL_dvalues[P][C],
 * dL_dconics[P][6]. */
int dgs_volume_backward(int function, int P, int N, int C, const float *means, const float *values,
                        const float *conics, const float *samples, const float *dL_dout,
                        const void *binning, size_t binning_bytes, float *dL_dmeans,
                        float *dL_dvalues, float *dL_dconics, void *workspace,
                        size_t workspace_bytes, dgs_stream_t stream, int debug);

/* Diagnostic (not on any reference API): counts[0] = pairs the forward evaluates (candidates
 * inside their own cut box), counts[1] = live pairs (G = expf(power) > 0).  Host, syncs;
 * DGS_ERR_BUFFER when the inputs differ from the binned ones. */
int dgs_volume_count_pairs(int P, int N, const float *means, const float *conics, const float *samples,
                           const void *binning, size_t binning_bytes, int64_t *counts, dgs_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* DGS_VOLUME_H_INCLUDED */
