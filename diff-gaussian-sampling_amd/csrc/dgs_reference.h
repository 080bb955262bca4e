// dgs_reference.h -- the call-time path of the render calls (dgs_reference.hip).
//
// The reference bins at preprocess but reads means, conics and samples from the tensors passed
// to every forward / backward call (forward.cu:136-145, backward.cu:76-85).  The fine-cell
// kernels evaluate a culled pair set and packed rows built from the BINNED tensors, so each
// call first compares its tensors with the copies the binning kept (k_verify, a device-side
// flag: no host sync).  When any differs, the fine-cell kernels exit at once and the kernels
// here evaluate the reference's own pair set -- every Gaussian of a tile's list (its
// point_list, kept by the binning) against every sample of the tile -- with the call-time
// tensors and the reference-literal per-pair arithmetic.  When the inputs match (the normal
// case: GaussianSampler passes the binned tensors) these kernels exit at once.
#pragma once

#include "dgs_render.h"

namespace dgs {

struct RefCall {
    const char *gb, *sb;
    const float *means, *values, *conics, *samples;
    DLs dls;         // backward: dL/dout of each function of the call
    Outs outs;       // forward: the outputs (zero-filled by the caller, written here)
    float *acc;      // backward: SoA gradient sums in internal order (k_finalize permutes them)
    const uint32_t *flag;  // non-zero: the call-time tensors differ from the binned ones
    int P, N, C, cbase;
    int64_t R;       // num_rendered (sizes the backward's grid)
    hipStream_t s;
    int debug;
    float4 *cbox;    // P float4 of the caller's workspace (its Gaussian-row region, idle on this
                     // path) for the call-time cuts (ref_boxes); null: tested from means / conics
};

// The call-time cut of every Gaussian (caller order) into a.cbox: {m0, m1, e0, e1}, e = the cut's
// half-widths (ref_may_touch's, rounded up to fp32; +inf: never culled).  Exits at once unless
// *a.flag is set.  Run after the fine-cell kernels, which read that region when the flag is clear.
template <int D>
int ref_boxes(const RefCall &a);

// Compares the call's means / conics / samples with the binning's copies; ORs 1 into *flag on
// any difference (bitwise).  The flag must be zeroed earlier on the stream.
int verify_inputs(const char *gb, const char *sb, int P, int D, int N, const float *means,
                  const float *conics, const float *samples, uint32_t *flag, hipStream_t s, int debug);

template <int FN, int D, int CB>
int ref_forward(const RefCall &a);
template <int FN, int D, int CB>
int ref_backward(const RefCall &a);

}  // namespace dgs
