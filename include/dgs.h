/*
 * dgs.h -- C ABI of the MI355X-native differentiable Gaussian sampler (libdgs.so).
 *
 * Plain pointers, sizes and a HIP stream; no torch types.  Every device pointer is global
 * memory on the current HIP device; every array is dense row-major fp32 unless stated.
 * All entry points are asynchronous on `stream` except where a host value is returned
 * (dgs_tile_grid, dgs_preprocess).  The binning, sampling and aggregation entry points allocate
 * no device memory on their own: buffers come from the caller through `dgs_alloc_fn`
 * (mirroring the reference's resize_functional lambdas, sample_points.cu:29-35) or as explicit
 * workspaces.  The exceptions use small stream-ordered scratch and are counted by
 * dgs_internal_allocations(): dgs_tile_grid (its min/max partials), dgs_inputs_match and
 * dgs_volume_count_pairs (diagnostics), and the first call-time-path use of a binning (a
 * forward / backward WITHOUT DGS_SAMPLE_INPUTS_BINNED sorts the reference tile lists once).
 * The preprocess reads its one host value back into pinned host memory allocated once per host
 * thread.
 *
 * Each function names the reference interface it replaces.  The torch extension
 * diff_gaussian_sampling._C (csrc/torch_ext.cpp) maps the 12 pybind entry points of the
 * reference (ext.cpp:19-32) onto these functions; INTEGRATION.md shows the ctypes binding.
 *
 * Return value: DGS_OK (0) or a dgs_status code; dgs_last_error() describes the failure
 * (thread-local).  With debug != 0 every launch is followed by a stream synchronisation
 * and a HIP error check, as the reference's CHECK_CUDA(…, debug) does (auxiliary.h:33-40).
 */
#ifndef DGS_H_INCLUDED
#define DGS_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *dgs_stream_t; /* == hipStream_t; NULL = default stream */

enum dgs_status {
    DGS_OK = 0,
    DGS_ERR_ARG = 1,     /* invalid argument (shape, dimension, size)                */
    DGS_ERR_HIP = 2,     /* HIP runtime / kernel error                               */
    DGS_ERR_ALLOC = 3,   /* the allocation callback returned NULL                    */
    DGS_ERR_BUFFER = 4   /* an opaque binning buffer is missing, stale or corrupted  */
};

/* CudaSampler::Function (sampler.h:23) */
enum dgs_function { DGS_GAUSSIAN = 0, DGS_DERIVATIVE = 1, DGS_LAPLACIAN = 2, DGS_THIRD = 3 };

/* Which buffer the allocation callback is asked for. */
enum dgs_buffer {
    DGS_BUF_BINNING = 0,        /* opaque Gaussian-side binning state (returned to Python) */
    DGS_BUF_SAMPLE_BINNING = 1, /* opaque sample-side binning state (returned to Python)   */
    DGS_BUF_RANGES = 2,         /* uint2[T] + 8 B, reference layout (sample_points.cu:76)  */
    DGS_BUF_SAMPLE_RANGES = 3,  /* uint2[T] + 8 B, reference layout (sample_points.cu:77)  */
    DGS_BUF_SCRATCH = 4,        /* temporary, released by the caller after the call        */
    DGS_BUF_AGG_INDICES = 5,    /* int64[length] neighbour ids (dgs_agg_preprocess)        */
    DGS_BUF_AGG_DISTS = 6,      /* float[length][D] scaled displacements                   */
    DGS_BUF_AGG_DENSITIES = 7   /* float[length] densities                                 */
};

/* Returns device memory of at least `bytes` bytes (16-byte aligned), or NULL on failure.
 * DGS_BUF_SCRATCH is requested several times per call.  Within one call the other kinds may be
 * requested more than once too: dgs_preprocess sizes its lists before its host sync from the
 * previous call's sizes and asks again if they do not fit, and dgs_preprocess_auto bins a
 * second time when its grid guess was wrong.  The LAST pointer returned for a kind is the one
 * the call's results live in; the earlier ones of that kind are unused once the call returns
 * (a torch caller simply drops them; an arena caller should size for two of each). */
typedef void *(*dgs_alloc_fn)(void *ctx, int which, size_t bytes);

const char *dgs_last_error(void);
int dgs_version(void);

/* Loads every code object of the library onto the current device (one no-op launch per
 * translation unit; synchronises `stream`).  Optional: otherwise the first call of each kind
 * pays its unit's load (a training loop calls it once at start-up; bench.py reports it). */
int dgs_warmup(dgs_stream_t stream);

/* Tile grid of the reference host glue (sample_points.cu:70-74), computed on the device with
 * torch's CUDA-path arithmetic: grid[d] = ceil((max_d - min_d + 1e-6f) * (1.0f / 0.51f)),
 * offset[d] = min_d.  Synchronises `stream`; grid_out/offset_out are host arrays of D. */
int dgs_tile_grid(int N, int D, const float *samples, int *grid_out, float *offset_out,
                  dgs_stream_t stream);

/* Binning: replaces PreprocessCUDA (sample_points.cu:38-98) and
 * CudaSampler::Sampler::preprocess (sampler_impl.cu:216-330).
 *   means[P][D], covariances[P][S], conics[P][S], samples[N][D]   (S = D(D+1)/2, D in {1,2})
 *   grid[D], grid_offset[D]: host arrays (dgs_tile_grid, or the global grid of a sharded run)
 *   radii[P]: out, reference radii (0 for skipped Gaussians)
 *   num_rendered: out (host), the reference's R = sum of tiles touched
 * Buffers are requested through `alloc`.  Synchronises `stream` once (to size the lists).
 * The forward/backward calls read the means, conics and samples they are given, as the
 * reference does (forward.cu:136-145): inputs that differ from the binned ones are detected on
 * the device and take the reference's tile pair set (dgs_reference.hip). */
int dgs_preprocess(int P, int D, int N, const float *means, const float *covariances,
                   const float *conics, const float *samples, const int *grid,
                   const float *grid_offset, float *radii, dgs_alloc_fn alloc, void *alloc_ctx,
                   int64_t *num_rendered, dgs_stream_t stream, int debug);

/* The ABI this header describes (dgs_version() returns it).  11: dgs_bin_options starts with
 * struct_size and flags; dgs_binning_info writes 6 values.  12: dgs_bin_options.samples_binned,
 * dgs_preprocess_auto_ex, dgs_sample_reuse_count. */
#define DGS_ABI_VERSION 12

/* dgs_bin_options.flags */
enum {
    /* the capturable binning ORs its status into *status_device instead of storing it: a
     * status word allocated once, outside the captured step, then records every overflow of
     * every replay until the caller clears it (diff_gaussian_sampling.BinningStatusMonitor) */
    DGS_BIN_STATUS_STICKY = 1,
    /* the capturable binning with samples_binned: the caller guarantees that the samples hold, at
     * every replay, the values they had when samples_binned's binning was made (a training loop's
     * fixed collocation points), and keeps that buffer allocated as long as the graph.  The
     * captured binning then copies the sample side instead of sorting the samples at every replay,
     * and status bit 8 (the samples' own grid) is not computed. */
    DGS_BIN_SAMPLES_FIXED = 2
};

/* Options of dgs_preprocess_ex (zero-initialise, set struct_size = sizeof(dgs_bin_options), then
 * set what is wanted; a struct of another size -- a caller built against another ABI -- is
 * refused with DGS_ERR_ARG). */
typedef struct dgs_bin_options {
    uint32_t struct_size;
    uint32_t flags; /* DGS_BIN_STATUS_STICKY, DGS_BIN_SAMPLES_FIXED */
    /* device uint8[P] or NULL.  Gaussians with present[g] == 0 are left out of the binning the
     * way a det == 0 Gaussian is (radius 0, no tiles, no pairs; radii[g] = 0 and they do not
     * count in num_rendered).  A rank of a spatially sharded run bins only the rows it holds
     * current copies of (diff_gaussian_sampling.distributed.SpatialShardedGaussianSampler). */
    const uint8_t *present;
    /* > 0: the area (D = 2; a length at D = 1, domain units) the samples actually occupy.  The
     * fine cells are then sized for the density N / sample_area instead of N / (T tiles): a
     * shard's points fill only part of the global tile grid.  Results do not depend on it
     * beyond float summation order; 0 = the whole grid. */
    double sample_area;
    /* > 0: the GRAPH-CAPTURABLE binning (replaces the syncs of
     * sampler_impl.cu:257 and sample_points.cu:74).  No host synchronisation and no host read of a
     * device value, so the call can be captured into a HIP graph and replayed (a training loop's
     * re-binning after every optimizer step).  The lists are sized from these capacities -- e.g.
     * the previous binning's sizes plus slack (dgs_binning_info out[1], out[5]); the grid is the
     * one passed to dgs_preprocess_ex.  *num_rendered (host) is set to -1;
     *   num_rendered_device (int64, device): R;
     *   status_device (uint32, device): 0, or bits 1: entries > capacity_E, 2: sort-path entries
     *   > capacity_Es, 4: R > capacity_R, 8: the samples' own tile grid (sample_points.cu:70-74)
     *   differs from the one passed.
     * A non-zero status marks the binning invalid (the lists were clamped into the capacities):
     * sample calls on it leave binned outputs at zero, never access memory out of bounds; re-bin
     * eagerly or with larger capacities.  capacity_Es <= capacity_E, capacity_R > 0. */
    int64_t capacity_E, capacity_Es, capacity_R;
    int64_t *num_rendered_device;
    uint32_t *status_device;
    /* The sample_binning buffer of an earlier binning by this process (still allocated) of the
     * SAME samples -- the same pointer, N and D, contents unchanged since -- or NULL.  When this
     * call's tile grid and fine cells are that binning's, the sample side (the sorted samples,
     * the fine cells' and sub-cells' sample ranges and boxes) is copied from it instead of
     * recomputed: the samples' sort, cell keys and boxes, ~0.15 ms of a 1M x 2M binning, are
     * skipped.  Results are bit-identical either way.  The caller vouches for the contents (the
     * torch layer: the samples tensor's identity and version counter); otherwise it is
     * ignored.  With the capturable form (capacity_E > 0) only under DGS_BIN_SAMPLES_FIXED: a
     * replay cannot see whether the captured samples changed. */
    const void *samples_binned;
    size_t samples_binned_bytes;
} dgs_bin_options;

/* dgs_preprocess with options (NULL = dgs_preprocess). */
int dgs_preprocess_ex(int P, int D, int N, const float *means, const float *covariances,
                      const float *conics, const float *samples, const int *grid,
                      const float *grid_offset, const dgs_bin_options *opts, float *radii,
                      dgs_alloc_fn alloc, void *alloc_ctx, int64_t *num_rendered,
                      dgs_stream_t stream, int debug);

/* dgs_preprocess with the tile grid of the reference host glue (sample_points.cu:70-74)
 * computed on the device (dgs_tile_grid's arithmetic) instead of passed in: the reference's
 * PreprocessCUDA as a whole.  Per sample set (the samples pointer, N and D; 8 sets remembered)
 * the call either speculates -- bins with the set's previous grid while the device computes
 * this call's, both read back at the binning's one host sync, re-binning only on a miss -- or
 * reads the grid first (one small extra sync, then one binning).  A set speculates after two
 * consecutive calls found the same grid, and a miss returns it to read-first: fixed samples
 * pay one sync per call, resampled points (whose min, the offset, moves) one extra small one,
 * and never a second binning after their first miss.
 * grid_out[D] / offset_out[D] (host): the grid used.  Replaces PreprocessCUDA
 * (sample_points.cu:38-98) + Sampler::preprocess (sampler_impl.cu:216-330). */
int dgs_preprocess_auto(int P, int D, int N, const float *means, const float *covariances,
                        const float *conics, const float *samples, float *radii, dgs_alloc_fn alloc,
                        void *alloc_ctx, int64_t *num_rendered, int *grid_out, float *offset_out,
                        dgs_stream_t stream, int debug);

/* dgs_preprocess_auto with options: present / sample_area as in dgs_preprocess_ex, and
 * samples_binned -- when that binning's grid was its samples' own (a dgs_preprocess_auto[_ex]
 * binning), it is this call's grid too, so no grid pass or speculation runs and the sample side
 * is copied (dgs_bin_options.samples_binned).  capacity_E must be 0.  NULL = dgs_preprocess_auto. */
int dgs_preprocess_auto_ex(int P, int D, int N, const float *means, const float *covariances,
                           const float *conics, const float *samples, const dgs_bin_options *opts, float *radii,
                           dgs_alloc_fn alloc, void *alloc_ctx, int64_t *num_rendered, int *grid_out,
                           float *offset_out, dgs_stream_t stream, int debug);

/* Diagnostics: the binnings of this process that copied their sample side from an earlier one
 * (dgs_bin_options.samples_binned). */
int64_t dgs_sample_reuse_count(void);

/* Spatial sharding (diff_gaussian_sampling.distributed.SupportExchange): for
 * each Gaussian, bit r of mask_out[g] is set when rank r's point range extents[r] = [lo, hi]
 * along the sharding axis (y at D = 2, x at D = 1) meets the Gaussian's exact-zero cut
 * X^T A X <= 210 or one of its torus images (period 2, forward.cu:149-157), i.e. when rank r's
 * partial gradient for it can be non-zero; owner_out[g] is the rank nearest its mean among the
 * ranks it touches (the nearest of all ranks when it touches none; first on ties).
 * extents: host array [W][2]; 1 <= W <= 32. */
int dgs_exchange_sets(int P, int D, const float *means, const float *conics, int W,
                      const double *extents, uint32_t *mask_out, int32_t *owner_out,
                      dgs_stream_t stream);

/* Workspace bytes needed by dgs_sample_forward (backward == 0) or dgs_sample_backward. */
size_t dgs_sample_workspace_size(int function, int P, int D, int N, int C, int backward);

/* The workspace bytes a call on THIS binning can use to full effect (mask as in
 * dgs_sample_forward_ex): for a backward whose binning sends >= 1/4 of its entries through the
 * sort path (thin / anisotropic fields) that adds a per-entry slot-sum region (the entries'
 * partial gradients are stored and summed per Gaussian in order, instead of scattered float
 * atomics).  A workspace of dgs_sample_workspace_size bytes is still valid (the atomics then).
 * >= dgs_sample_workspace_size_multi(mask, ...); buffers this process did not bin: the same. */
size_t dgs_sample_workspace_size_binned(int mask, int P, int D, int N, int C, int backward,
                                        const void *binning, size_t binning_bytes,
                                        const void *sample_binning, size_t sample_binning_bytes);

/* Stream-ordered allocations the library has made on its own since load (see the top of this
 * file: none on the binning / sampling hot path). */
int64_t dgs_internal_allocations(void);

/* Forward: replaces SampleGaussians{,Derivative,Laplacian,Third}CUDA (sample_points.cu:100-143,
 * 198-296), CudaSampler::Sampler::forward (sampler_impl.cu:333-364) and FORWARD::render
 * (forward.cu:277-345).  out[N][K][C], K = D^function, must be zero-filled by the caller
 * (samples outside every tile stay 0, as in the reference).
 * The first forward / backward of a binning that may take the call-time path (every call
 * without DGS_SAMPLE_INPUTS_BINNED) also sorts that path's tile lists -- the reference's
 * point_list, sampler_impl.cu:265-283 -- on `stream` (stream-ordered scratch); later calls on
 * other streams wait for that sort.  A binning's calls otherwise only read it. */
int dgs_sample_forward(int function, int P, int D, int N, int C, const float *means,
                       const float *values, const float *conics, const float *samples,
                       const void *binning, size_t binning_bytes, const void *sample_binning,
                       size_t sample_binning_bytes, float *out, void *workspace,
                       size_t workspace_bytes, dgs_stream_t stream, int debug);

/* Backward: replaces SampleGaussians*BackwardCUDA (sample_points.cu:145-196, 298-372),
 * CudaSampler::Sampler::backward (sampler_impl.cu:368-405) and BACKWARD::render
 * (backward.cu:418-501).  dL_dout[N][K][C]; writes (overwrites) dL_dmeans[P][D],
 * dL_dvalues[P][C], dL_dconics[P][S]. */
int dgs_sample_backward(int function, int P, int D, int N, int C, const float *means,
                        const float *values, const float *conics, const float *samples,
                        const float *dL_dout, const void *binning, size_t binning_bytes,
                        const void *sample_binning, size_t sample_binning_bytes,
                        float *dL_dmeans, float *dL_dvalues, float *dL_dconics, void *workspace,
                        size_t workspace_bytes, dgs_stream_t stream, int debug);

/* Fused functions (not on the reference API): one traversal of the
 * binned pairs for every function of `mask` (bit f set = dgs_function f, mask in 1..15), as
 * the Physics-Informed-GS loss calls several of the four per step.  Each result equals the
 * per-function entry point's within the parity tolerance.
 *   forward : outs[f] = out of function f (as dgs_sample_forward; zero-filled by the caller),
 *             for every f in mask (the other entries are ignored and may be NULL)
 *   backward: dL_douts[f] = dL/d out of function f for every f in mask; writes the gradients
 *             of the summed loss, sum_f <dL_douts[f], out_f>
 * Two or more functions need D = 2 and C = 1 (DGS_ERR_ARG otherwise: call the per-function
 * entry points and add their gradients); a single-bit mask is the per-function path. */
size_t dgs_sample_workspace_size_multi(int mask, int P, int D, int N, int C, int backward);
int dgs_sample_forward_multi(int mask, int P, int D, int N, int C, const float *means,
                             const float *values, const float *conics, const float *samples,
                             const void *binning, size_t binning_bytes, const void *sample_binning,
                             size_t sample_binning_bytes, float *const *outs, void *workspace,
                             size_t workspace_bytes, dgs_stream_t stream, int debug);
int dgs_sample_backward_multi(int mask, int P, int D, int N, int C, const float *means,
                              const float *values, const float *conics, const float *samples,
                              const float *const *dL_douts, const void *binning,
                              size_t binning_bytes, const void *sample_binning,
                              size_t sample_binning_bytes, float *dL_dmeans, float *dL_dvalues,
                              float *dL_dconics, void *workspace, size_t workspace_bytes,
                              dgs_stream_t stream, int debug);

/* Per-call options of dgs_sample_forward_ex / dgs_sample_backward_ex (not on the reference API;
 * zero-initialise, then set what is wanted).  `flags` is a bit set of dgs_sample_flag:
 *   DGS_SAMPLE_INPUTS_BINNED: the caller vouches that means, conics and samples are bitwise the
 *     tensors the binning was built from (e.g. the same tensor objects, unmodified since: the
 *     torch extension checks object identity and autograd version counters).  The call then
 *     skips the device-side comparison with the binned copies and the call-time path of
 *     dgs_reference.hip (forward.cu:136-145 reads the passed tensors; the comparison exists only
 *     to detect a difference).  Wrong if the tensors were changed: leave it unset when unsure.
 *   DGS_SAMPLE_ROWS_VALID: `workspace` comes from an earlier call on the same binning with the
 *     same function mask, C <= 16 and the same means / conics / values (unmodified since), whose
 *     Gaussian-row region (offset 0) the earlier call packed: the rows are reused, not repacked.
 *     A forward followed by its backward shares one workspace of the backward's size this way.
 *     A backward leaves the region overwritten (its finalize reuses it): never reuse after one.
 *   DGS_SAMPLE_GRAPH_CAPTURE: the call is being captured into a HIP graph (stream capture):
 *     it then enqueues kernels only -- no timing events -- and requires DGS_SAMPLE_INPUTS_BINNED (the
 *     call-time path's first use builds tile lists behind a host-side record; DGS_ERR_ARG
 *     without it).  A replay re-reads means, values, conics, samples and dL from the captured
 *     addresses; values and dL may change between replays.  means / conics / samples may change
 *     only when the graph also holds their re-binning: a capturable dgs_preprocess_ex (capacity
 *     options above) captured before the sample calls (tests/graph_child.py: rebin_step).
 */
enum dgs_sample_flag { DGS_SAMPLE_INPUTS_BINNED = 1, DGS_SAMPLE_ROWS_VALID = 2, DGS_SAMPLE_GRAPH_CAPTURE = 4 };
typedef struct dgs_sample_options {
    uint32_t flags;
} dgs_sample_options;

/* The multi-function entry points with options (opts NULL = no flags).  mask as in
 * dgs_sample_forward_multi (a single-bit mask is the per-function path, C any). */
int dgs_sample_forward_ex(int mask, int P, int D, int N, int C, const float *means,
                          const float *values, const float *conics, const float *samples,
                          const void *binning, size_t binning_bytes, const void *sample_binning,
                          size_t sample_binning_bytes, float *const *outs, void *workspace,
                          size_t workspace_bytes, const dgs_sample_options *opts, dgs_stream_t stream,
                          int debug);
int dgs_sample_backward_ex(int mask, int P, int D, int N, int C, const float *means,
                           const float *values, const float *conics, const float *samples,
                           const float *const *dL_douts, const void *binning, size_t binning_bytes,
                           const void *sample_binning, size_t sample_binning_bytes, float *dL_dmeans,
                           float *dL_dvalues, float *dL_dconics, void *workspace, size_t workspace_bytes,
                           const dgs_sample_options *opts, dgs_stream_t stream, int debug);

/* Diagnostics (not on the reference API): counts, over the pairs the forward evaluates,
 * W_cand (candidate pairs after culling) and W_live (pairs with power >= thr, the survey's
 * live-pair count for thr = -104).  counts[0] = W_cand, counts[1] = W_live (host, syncs). */
int dgs_count_pairs(int P, int D, int N, const float *means, const float *conics,
                    const float *samples, const void *binning, size_t binning_bytes,
                    const void *sample_binning, size_t sample_binning_bytes, float thr,
                    int64_t *counts, void *workspace, size_t workspace_bytes,
                    dgs_stream_t stream);

/* Diagnostics (not on the reference API): host-known facts of a binning this process made (no
 * device work): out[0] = num_rendered R, out[1] = fine (Gaussian, cell) entries E, out[2] = the
 * entries that take the reference-literal per-pair path (conics that are not positive definite,
 * wrap breakpoints, fallback cells), out[3] = fine cells, out[4] = 0 (round 4's kThin entries;
 * the literal-order thin pass was removed in round 6), out[5] = sort-path entries (the
 * capturable binning's capacity_Es).  A capturable binning reports its capacities for R / E and
 * -1 for the device-only counts.  DGS_ERR_BUFFER for buffers this process did not bin.
 * out must hold 6 values. */
int dgs_binning_info(const void *binning, size_t binning_bytes, const void *sample_binning,
                     size_t sample_binning_bytes, int64_t *out);

/* Diagnostic: do means / conics / samples equal (bitwise) the tensors the binning was built
 * from?  *match = 1: forward / backward take the binned fine-cell path; 0: they take the
 * call-time path (the reference reads these tensors at every call, forward.cu:136-145,
 * backward.cu:76-85, while its tile lists come from preprocess).  Host, syncs. */
int dgs_inputs_match(int P, int D, int N, const float *means, const float *conics,
                     const float *samples, const void *binning, size_t binning_bytes,
                     const void *sample_binning, size_t sample_binning_bytes, int *match,
                     dgs_stream_t stream);

/* ---- neighbour aggregation (aggregate_neighbors.{h,cu}) ------------------------------- */

/* Neighbour lists: replaces AggregateNeighborsPreprocessCUDA (aggregate_neighbors.cu:323-367)
 * with its kernels findCollisions (18-55) and preprocess (57-127), without the P x P matrix.
 *   means[P][D], conics[P][S], radii[P]   (D in {1,2})
 *   ranges[P]: out, int64 inclusive cumsum of the per-row neighbour counts
 *   inv_total[P]: out, 1 / (sum of the row's densities + 1e-6)
 *   row_order[P]: optional out (NULL = not wanted), a permutation of the rows in spatial (grid
 *     cell) order.  Passed to dgs_agg_forward / dgs_agg_backward it only changes the order in
 *     which rows are scheduled -- concurrent rows then share their neighbours in L2 -- never a
 *     result; any permutation of 0..P-1 is valid there.
 *   length: out (host), ranges[P-1] (0 when P == 0)
 * indices (int64, -1 where the exponent is positive), dists [length][D] and densities [length]
 * are requested through `alloc` (DGS_BUF_AGG_*), slots in ascending neighbour id per row;
 * every slot is written.  Synchronises `stream` twice (grid bounds, list length). */
int dgs_agg_preprocess(int P, int D, const float *means, const float *conics, const float *radii,
                       int64_t *ranges, float *inv_total, int32_t *row_order, dgs_alloc_fn alloc,
                       void *alloc_ctx, int64_t *length, dgs_stream_t stream, int debug);

/* Forward: replaces AggregateNeighborsCUDA (aggregate_neighbors.cu:369-415) and its kernel
 * aggregateNeighbors (129-208).  E = len(distance_transform) / 2, F = (E-1)/D/2 frequencies.
 *   features[P][L] (L <= 256), transform[L][L], queries/keys[P][K]
 *   row_order[P]: optional (NULL = 0..P-1), see dgs_agg_preprocess
 *   weights/embeddings/factors[length]: out (0 at index -1); out[P][L]: out (overwritten) */
int dgs_agg_forward(int P, int D, int L, int K, int E, const float *features, const float *transform,
                    const float *queries, const float *keys, const float *frequencies,
                    const float *distance_transform, const int64_t *indices, const int64_t *ranges,
                    const float *dists, const float *densities, const float *inv_total,
                    const int32_t *row_order, float *weights, float *embeddings, float *factors,
                    float *out, dgs_stream_t stream, int debug);

/* Workspace bytes needed by dgs_agg_backward. */
size_t dgs_agg_workspace_size(int P, int L);

/* Backward: replaces AggregateNeighborsBackwardCUDA (aggregate_neighbors.cu:417-475) and its
 * kernel aggregateNeighborsBackward (210-321).  Writes (overwrites) the six gradients, shaped as
 * features, transform, queries, keys, frequencies[F], distance_transform[2E]. */
int dgs_agg_backward(int P, int D, int L, int K, int E, const float *features,
                     const float *transform, const float *queries, const float *keys,
                     const float *frequencies, const float *distance_transform,
                     const int64_t *indices, const int64_t *ranges, const float *dists,
                     const float *densities, const float *weights, const float *embeddings,
                     const float *factors, const float *inv_total, const int32_t *row_order,
                     const float *dL_dout,
                     float *dL_dfeatures, float *dL_dtransform, float *dL_dqueries,
                     float *dL_dkeys, float *dL_dfrequencies, float *dL_ddistance_transform,
                     void *workspace, size_t workspace_bytes, dgs_stream_t stream, int debug);

/* The neighbour lists transposed (CSR -> CSC of the slot matrix): for every row j, the slots
 * (i -> j) that name j, in ascending slot order: tslot[tstart[j] .. tstart[j + 1]) (slots with
 * index -1 come after tstart[P]).  Each entry is the slot's position in a record array whose rows
 * follow row_order (NULL = 0..P-1): row i's slots are at rstart[i] + 0, 1, ...  No reference
 * counterpart: it turns the reference's scatter of the neighbours' feature / key gradients
 * (aggregate_neighbors.cu:303, 315 -- float atomics, here the float-atomic rate bounded the
 * backward) into a per-row sum, so the backward writes every gradient once.
 * ranges / row_order: as from dgs_agg_preprocess.  tstart[P + 1], tslot[length], rstart[P]: out.
 * Scratch (12 bytes per slot) through `alloc` (DGS_BUF_SCRATCH).  length < 2^31. */
int dgs_agg_transpose(int P, int64_t length, const int64_t *indices, const int64_t *ranges,
                      const int32_t *row_order, int32_t *tstart, uint32_t *tslot, int32_t *rstart,
                      dgs_alloc_fn alloc, void *alloc_ctx, dgs_stream_t stream, int debug);

/* Workspace bytes of dgs_agg_backward_tr (L + K <= 64; larger widths take dgs_agg_backward). */
size_t dgs_agg_workspace_size_tr(int P, int L, int64_t length);

/* dgs_agg_backward with the transposed lists of dgs_agg_transpose (same indices, ranges and
 * row_order): identical
 * gradients up to float summation order, with no float atomics on the features / keys
 * gradients (each row sums its incoming slots in slot order: deterministic). */
int dgs_agg_backward_tr(int P, int D, int L, int K, int E, const float *features,
                        const float *transform, const float *queries, const float *keys,
                        const float *frequencies, const float *distance_transform,
                        const int64_t *indices, const int64_t *ranges, const float *dists,
                        const float *densities, const float *weights, const float *embeddings,
                        const float *factors, const float *inv_total, const int32_t *row_order,
                        const int32_t *tstart, const uint32_t *tslot, const int32_t *rstart,
                        int64_t length, const float *dL_dout,
                        float *dL_dfeatures, float *dL_dtransform, float *dL_dqueries,
                        float *dL_dkeys, float *dL_dfrequencies, float *dL_ddistance_transform,
                        void *workspace, size_t workspace_bytes, dgs_stream_t stream, int debug);

/* ---- the dense sharded path's collective (the reference is single-GPU) ---- */

/* RCCL communicators for callers without torch.distributed.  RCCL (librccl.so.1) is loaded on
 * first use.  dgs_comm_unique_id writes dgs_comm_id_bytes() bytes (ncclUniqueId) on one rank,
 * which the caller distributes; every rank then calls dgs_comm_init (ncclCommInitRank). */
size_t dgs_comm_id_bytes(void);
int dgs_comm_unique_id(void *id_out);
int dgs_comm_init(void **comm_out, int nranks, const void *id, int rank);
int dgs_comm_destroy(void *comm);

/* Sums the packed per-Gaussian gradients [dmeans | dvalues | dconics] (device float[count], in
 * place) over the communicator's ranks: the one all-reduce of query-point sharding (each rank's
 * backward is a partial sum over its points).  chunk_elems > 0 issues it as back-to-back chunks
 * (RCCL pipelines them; a caller can start optimizer work on the first chunks early).  comm: a
 * communicator of dgs_comm_init (an ncclComm_t of the same RCCL library).  Asynchronous on
 * `stream`. */
int dgs_allreduce_grads(float *grads, size_t count, void *comm, size_t chunk_elems, dgs_stream_t stream);

/* Benchmark support: bracket every forward (which = 0) / backward (which = 1) render-kernel
 * launch with HIP events on its stream.  dgs_timing_read waits for the recorded events, adds
 * their durations into *total_ms, clears the record and returns the launch count. */
void dgs_timing_enable(int on);
int dgs_timing_read(int which, double *total_ms);

#ifdef __cplusplus
}
#endif

#endif /* DGS_H_INCLUDED */
