// dgs_internal.h -- shared definitions of libdgs.so (MI355X / gfx950).
//
// Opaque buffer layouts, the reference-literal arithmetic used by the binning kernels, the
// fine-cell geometry used for exact culling, and small host helpers.  See DESIGN.md.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <string>

#include "dgs.h"

#define DGS_NO_CONTRACT _Pragma("clang fp contract(off)")

namespace dgs {

// ---------------------------------------------------------------------------------------
// Constants (config.h:18-20, forward.cu:21)
// ---------------------------------------------------------------------------------------
constexpr float kTile = 0.51f;         // BLOCK_SIZE
constexpr uint32_t kMagic = 0x44475342u;  // "DGSB"
constexpr uint32_t kVersion = DGS_ABI_VERSION;  // (the binning header's version too)
// Fine-list entry = internal Gaussian id | flags.  Entries of a cell are sorted so that the
// flagged ones come last (the render kernels then see whole flag-free batches).
constexpr uint32_t kGeneral = 0x80000000u;  // per-pair exact torus wrap needed in this cell
constexpr uint32_t kUnsafe = 0x40000000u;   // conic not positive definite, a wrap breakpoint in the
                                            // cell, or a fallback cell: the per-pair literal path
constexpr uint32_t kThin = 0x20000000u;     // reserved (round 4's literal-order thin pass; no entry carries it)
                                            // (rho^2 >= 0.82): packed, the unfused reference's exponent order
constexpr uint32_t kSlow = kGeneral | kUnsafe | kThin;
constexpr uint32_t kIdMask = 0x1fffffffu;
constexpr int64_t kMaxGaussians = (int64_t)kIdMask;
// Culling threshold on q = X^T A X.  power = -q/2 < -105 makes expf(power) exactly +0 in
// fp32 (e^-105 < half of the smallest subnormal), so every forward and backward term of such
// a pair is exactly zero in the reference (all of them carry the factor G); culling them
// is result-preserving.
constexpr double kQCut = 210.0;
constexpr double kCellSlack = 1e-3;  // fraction of a fine cell tolerated outside its bounds
constexpr int kWave = 64;
// Forward work unit: a block of up to 32 sample PAIRS of one cell, pair-aligned in the sorted
// sample order (pairs (2p, 2p+1) are packed fp32 operands; a pair may straddle a cell edge,
// its foreign sample is evaluated but not written).
constexpr int kFwdUnit = kWave;
// Sub-cells (D = 2): every fine cell is split 2 x 2 at its nominal mid-lines; samples are sorted
// by (cell, sub-cell), and the forward walks per sub-cell the entries of its cell whose cut
// meets the sub-cell's sample box (sub lists), in units of up to kSubPairs sample pairs.  The
// backward keeps the cell lists: their one flush per (cell, Gaussian), in ascending-id runs, is
// what the float atomics allow.
constexpr int kSubPerCell = 4;
#ifndef DGS_SUB_PAIRS
#define DGS_SUB_PAIRS 24
#endif
constexpr int kSubPairs = DGS_SUB_PAIRS;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

// ---------------------------------------------------------------------------------------
// Opaque buffer layout.  Gaussian-side buffer (DGS_BUF_BINNING):
//   [header 256 B][counts int32[4]][perm int32[P]][cell_gbeg int32[ncells]]
//   [cell_gmid int32[ncells]][cell_gend int32[ncells]][entries uint32[E]][bwd_units uint2[bwd_cap]]
//   [gmean float2[P]][gcon float4[P]]  (means / conics in internal order, packed at binning)
//   [mcopy float[P*D]][ccopy float[P*S]]  (the binned means / conics as passed, caller order)
//   [rlist uint32[R]]  the reference's point_list: every tile's Gaussian ids, ascending
//                      (sampler_impl.cu:265-283), the pair set of the call-time path -- built
//                      at the binning's first call that may take that path (ensure_ref_lists)
//   [rref u32[P] f32[P]] tile-list offsets (caller order), radii (internal order) for that build
//   [rtab uint32[4][T+1]]  per tile: Gaussian-list start (rlist), sample start (sorted order),
//                      and the prefix counts of the call-time path's forward / backward units
// A cell's list is [gbeg, gend); its flag-free entries come first, [gbeg, gmid).
// Sample-side buffer (DGS_BUF_SAMPLE_BINNING):
//   [header copy][sorted_sid int32[N]][cell_sbeg int32[ncells]][cell_send int32[ncells]]
//   [fwd_units uint2[fwd_cap]][cell_box float4[ncells]]
//   [fsrows: sample pair rows [s0(2p) s0(2p+1) (s1(2p) s1(2p+1))] in sorted order, + slack]
//   [scopy float[N*D]]  (the binned samples as passed, caller order)
// The fine-cell lists are built from the binned means / conics / samples.  The reference reads
// means / conics / samples at every forward / backward call (forward.cu:136-145,
// backward.cu:76-85) and only its tile lists from preprocess; each call therefore compares its
// tensors with the copies (k_verify) and, if any differs, takes the call-time path instead
// (dgs_reference.hip: the reference's tile pair set, the passed tensors).
// ---------------------------------------------------------------------------------------
struct Header {
    uint32_t magic, version;
    int32_t P, D, N, T;
    int32_t grid[2];
    float off[2];
    int32_t n;       // fine cells per tile axis
    int32_t CT;      // cells per tile = n^D + 1 (the last one is the tile's unculled fallback cell)
    int32_t ncells;  // T * CT
    int32_t pad0;
    int64_t R;       // num_rendered (reference count)
    int64_t E;       // fine (Gaussian, cell) entries
    int64_t fwd_cap, bwd_cap;
    uint64_t o_counts, o_perm, o_cell_gbeg, o_cell_gend, o_entries, o_bwd_units, g_bytes;
    uint64_t o_sorted, o_cell_sbeg, o_cell_send, o_fwd_units, s_bytes;
    uint64_t stamp;  // identical in both buffers of one preprocess call
    uint64_t o_cell_gmid;
    uint64_t o_cell_box;  // sample buffer: per-cell bounding box of the cell's samples
    uint64_t o_gmean, o_gcon, o_fsrows;
    uint64_t o_mcopy, o_ccopy, o_rlist, o_rtab, o_scopy;
    // sub-cells (D = 2; empty at D = 1): sample side [sub_sbeg/send int32[4 ncells]]
    // [sub_box float4[4 ncells]] [fsub_units uint2[fsub_cap]]; Gaussian side
    // [sub_lbeg/lmid/lend int32[4 ncells]] [sub_ent uint32[Esub_cap]]
    uint64_t o_sub_sbeg, o_sub_send, o_sub_box, o_fsub_units;
    uint64_t o_sub_lbeg, o_sub_lmid, o_sub_lend, o_sub_ent;
    int64_t fsub_cap, esub_cap;
    uint32_t zero[4];  // always 0: the "inputs differ" word of calls whose inputs the caller vouches for
    uint64_t o_rref;   // (rlist's inputs: tile-list offsets u32[P] by caller id, radii f32[P] by internal id)
    // the sorted part of the cell lists (sort-path entries): per list position its Gaussian-major
    // slot q (esum_q u32[E]), per cell where that part begins (cell_gsort i32[ncells]), per
    // internal id its first slot (goff u32[P + 1]); the backward stores those entries' sums in
    // slot order and k_bwd_esum adds them per Gaussian (no scattered atomics)
    uint64_t o_esum_q, o_cell_gsort, o_goff;
    int64_t Es;        // sort-path entries
    uint64_t o_sub_lthin;  // per sub list: where its kThin entries begin (int32[4 ncells]; = lend without any)
};
constexpr size_t kHeaderBytes = 512;
static_assert(sizeof(Header) <= kHeaderBytes, "header too large");
enum RefTab { kRtGStart = 0, kRtSStart = 1, kRtFwdUnits = 2, kRtBwdUnits = 3 };
constexpr int kRefUnit = 64;  // call-time path: samples (forward) / list entries (backward) per unit

enum Counter { kNumFwdUnits = 0, kNumBwdUnits = 1, kNumUnsafe = 2, kNumFwdSubUnits = 3 };

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Layout {  // byte offsets, computed on the host
    uint64_t o_counts, o_perm, o_cell_gbeg, o_cell_gmid, o_cell_gend, o_entries, o_bwd_units, g_bytes;
    uint64_t o_gmean, o_gcon, o_mcopy, o_ccopy, o_rlist, o_rtab, o_rref, o_esum_q, o_cell_gsort, o_goff;
    uint64_t o_sub_lbeg, o_sub_lmid, o_sub_lend, o_sub_ent, o_sub_lthin;
    uint64_t o_sorted, o_cell_sbeg, o_cell_send, o_fwd_units, o_cell_box, o_fsrows, o_scopy, s_bytes;
    uint64_t o_sub_sbeg, o_sub_send, o_sub_box, o_fsub_units;
};

// Forward sample pair rows: N rounded up to a pair, plus slack for a pass's wide scalar loads
// (up to 32 pairs + one x16 load past the last pair).
inline size_t fsrows_bytes(int64_t N, int D) { return ((size_t)N + 1) * D * 4 + 36 * 16; }

// Sub-list capacity: an entry is in at most every sub-list of its cell (D = 2).
inline int64_t esub_cap_of(int D, int64_t E) { return D == 2 ? kSubPerCell * E : 0; }
inline int64_t fsub_cap_of(int D, int64_t N, int64_t ncells) {
    // per non-empty sub-cell: ceil(pairs / kSubPairs) <= its samples / (2 kSubPairs) + 2
    return D == 2 ? (N + 1) / 2 / kSubPairs + 2 * std::min<int64_t>(kSubPerCell * ncells, N) + 1 : 0;
}

inline Layout make_layout(int D, int64_t P, int64_t N, int64_t T, int64_t R, int64_t ncells, int64_t E,
                          int64_t fwd_cap, int64_t bwd_cap) {
    const int64_t nsub = D == 2 ? kSubPerCell * ncells : 0;
    const int S = D * (D + 1) / 2;
    Layout L;
    size_t o = kHeaderBytes;
    L.o_counts = o;    o = align_up(o + 16, 256);
    L.o_perm = o;      o = align_up(o + 8 * (size_t)P, 256);  // perm[P], then its inverse[P]
    L.o_cell_gbeg = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_cell_gmid = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_cell_gend = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_entries = o;   o = align_up(o + 4 * (size_t)E + 64, 256);  // slack: 8-entry scalar loads
    L.o_bwd_units = o; o = align_up(o + 8 * (size_t)bwd_cap, 256);
    L.o_gmean = o;     o = align_up(o + 8 * (size_t)P, 256);
    L.o_gcon = o;      o = align_up(o + 16 * (size_t)P, 256);
    L.o_mcopy = o;     o = align_up(o + 4 * (size_t)P * D, 256);
    L.o_ccopy = o;     o = align_up(o + 4 * (size_t)P * S, 256);
    L.o_rlist = o;     o = align_up(o + 4 * (size_t)R + 64, 256);
    L.o_rtab = o;      o = align_up(o + 16 * ((size_t)T + 1), 256);
    L.o_rref = o;      o = align_up(o + 8 * (size_t)P, 256);
    L.o_esum_q = o;    o = align_up(o + 4 * (size_t)E + 64, 256);
    L.o_cell_gsort = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_goff = o;      o = align_up(o + 4 * ((size_t)P + 1), 256);
    L.o_sub_lbeg = o;  o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_lmid = o;  o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_lend = o;  o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_lthin = o; o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_ent = o;   o = align_up(o + 4 * (size_t)esub_cap_of(D, E) + 64, 256);
    L.g_bytes = o;
    o = kHeaderBytes;
    L.o_sorted = o;    o = align_up(o + 4 * (size_t)N, 256);
    L.o_cell_sbeg = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_cell_send = o; o = align_up(o + 4 * (size_t)ncells, 256);
    L.o_fwd_units = o; o = align_up(o + 8 * (size_t)fwd_cap, 256);
    L.o_cell_box = o;  o = align_up(o + 16 * (size_t)ncells, 256);
    L.o_fsrows = o;    o = align_up(o + fsrows_bytes(N, 2), 256);
    L.o_scopy = o;     o = align_up(o + 4 * (size_t)N * D, 256);
    L.o_sub_sbeg = o;  o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_send = o;  o = align_up(o + 4 * (size_t)nsub, 256);
    L.o_sub_box = o;   o = align_up(o + 16 * (size_t)nsub, 256);
    L.o_fsub_units = o; o = align_up(o + 8 * (size_t)fsub_cap_of(D, N, ncells), 256);
    L.s_bytes = o;
    return L;
}

// Device view of both buffers.
struct Bins {
    const Header *h;
    const int32_t *counts;
    const int32_t *perm;
    const int32_t *cell_gbeg, *cell_gmid, *cell_gend;
    const uint32_t *entries;
    const uint2 *bwd_units;
    const int32_t *sorted_sid;
    const int32_t *cell_sbeg, *cell_send;
    const uint2 *fwd_units;
    const float4 *cell_box;  // [min0 min1 max0 max1] of each cell's samples
    const float2 *gmean;     // means in internal order ({m, 0} at D = 1)
    const float4 *gcon;      // conics in internal order ({c0, c1, c2, 0}; {c0, 0, 0, 0} at D = 1)
    const float *fsrows;     // sample pair rows in sorted order
    const uint32_t *rlist;   // reference tile lists (ascending Gaussian id per tile)
    const uint32_t *rtab;    // [4][T+1] per-tile tables of the call-time path (RefTab)
    const int32_t *sub_sbeg, *sub_send;  // sample range per sub-cell (cell * 4 + sub)
    const float4 *sub_box;
    const uint2 *fsub_units;             // (sub-cell, pair-aligned first sample)
    const int32_t *sub_lbeg, *sub_lmid, *sub_lend;
    const int32_t *sub_lthin;            // [lmid, lthin) flagged, [lthin, lend) kThin
    const uint32_t *sub_ent;             // sub lists: entries of the cell list, flagged last
    const uint32_t *esum_q;              // sorted-part list position -> Gaussian-major slot
    const int32_t *cell_gsort;           // first sorted-part position of each cell list
};

// Uniform (wave-invariant) loads through the constant address space: with a wave-uniform
// address hipcc emits s_load_* into SGPRs (no VGPRs, no LDS, no vector-memory slot).
template <typename T>
__device__ __forceinline__ T sload(const T *p) {
    return *(const __attribute__((address_space(4))) T *)(p);
}
template <>
__device__ __forceinline__ float4 sload<float4>(const float4 *p) {
    const float *f = reinterpret_cast<const float *>(p);
    return make_float4(sload(f), sload(f + 1), sload(f + 2), sload(f + 3));
}
template <>
__device__ __forceinline__ uint2 sload<uint2>(const uint2 *p) {
    const uint64_t v = *(const __attribute__((address_space(4))) uint64_t *)(p);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}

__device__ __forceinline__ Bins resolve(const char *gb, const char *sb) {
    Bins B;
    B.h = reinterpret_cast<const Header *>(gb);
    const uint64_t o_counts = sload(&B.h->o_counts), o_perm = sload(&B.h->o_perm);
    const uint64_t o_gbeg = sload(&B.h->o_cell_gbeg), o_gend = sload(&B.h->o_cell_gend);
    const uint64_t o_gmid = sload(&B.h->o_cell_gmid);
    const uint64_t o_ent = sload(&B.h->o_entries), o_bu = sload(&B.h->o_bwd_units);
    const uint64_t o_sorted = sload(&B.h->o_sorted), o_sbeg = sload(&B.h->o_cell_sbeg);
    const uint64_t o_send = sload(&B.h->o_cell_send), o_fu = sload(&B.h->o_fwd_units);
    const uint64_t o_box = sload(&B.h->o_cell_box);
    const uint64_t o_gmean = sload(&B.h->o_gmean), o_gcon = sload(&B.h->o_gcon);
    const uint64_t o_fsrows = sload(&B.h->o_fsrows);
    const uint64_t o_rlist = sload(&B.h->o_rlist), o_rtab = sload(&B.h->o_rtab);
    B.counts = reinterpret_cast<const int32_t *>(gb + o_counts);
    B.perm = reinterpret_cast<const int32_t *>(gb + o_perm);
    B.cell_gbeg = reinterpret_cast<const int32_t *>(gb + o_gbeg);
    B.cell_gend = reinterpret_cast<const int32_t *>(gb + o_gend);
    B.cell_gmid = reinterpret_cast<const int32_t *>(gb + o_gmid);
    B.entries = reinterpret_cast<const uint32_t *>(gb + o_ent);
    B.bwd_units = reinterpret_cast<const uint2 *>(gb + o_bu);
    B.sorted_sid = reinterpret_cast<const int32_t *>(sb + o_sorted);
    B.cell_sbeg = reinterpret_cast<const int32_t *>(sb + o_sbeg);
    B.cell_send = reinterpret_cast<const int32_t *>(sb + o_send);
    B.fwd_units = reinterpret_cast<const uint2 *>(sb + o_fu);
    B.cell_box = reinterpret_cast<const float4 *>(sb + o_box);
    B.gmean = reinterpret_cast<const float2 *>(gb + o_gmean);
    B.gcon = reinterpret_cast<const float4 *>(gb + o_gcon);
    B.fsrows = reinterpret_cast<const float *>(sb + o_fsrows);
    B.rlist = reinterpret_cast<const uint32_t *>(gb + o_rlist);
    B.rtab = reinterpret_cast<const uint32_t *>(gb + o_rtab);
    B.sub_sbeg = reinterpret_cast<const int32_t *>(sb + sload(&B.h->o_sub_sbeg));
    B.sub_send = reinterpret_cast<const int32_t *>(sb + sload(&B.h->o_sub_send));
    B.sub_box = reinterpret_cast<const float4 *>(sb + sload(&B.h->o_sub_box));
    B.fsub_units = reinterpret_cast<const uint2 *>(sb + sload(&B.h->o_fsub_units));
    B.sub_lbeg = reinterpret_cast<const int32_t *>(gb + sload(&B.h->o_sub_lbeg));
    B.sub_lmid = reinterpret_cast<const int32_t *>(gb + sload(&B.h->o_sub_lmid));
    B.sub_lend = reinterpret_cast<const int32_t *>(gb + sload(&B.h->o_sub_lend));
    B.sub_lthin = reinterpret_cast<const int32_t *>(gb + sload(&B.h->o_sub_lthin));
    B.sub_ent = reinterpret_cast<const uint32_t *>(gb + sload(&B.h->o_sub_ent));
    B.esum_q = reinterpret_cast<const uint32_t *>(gb + sload(&B.h->o_esum_q));
    B.cell_gsort = reinterpret_cast<const int32_t *>(gb + sload(&B.h->o_cell_gsort));
    return B;
}

// Wave index of this thread, provably uniform (readfirstlane), with the bijective XCD-aware
// block remap (cdna_hip_programming.md T1): consecutive units -- neighbouring cells that
// share Gaussians -- run on one XCD and share its L2.  Kernels grid-stride by
// gridDim.x * kWavesPerBlock from here.
__device__ __forceinline__ int wave_unit_index(int nunits) {
    // The remap is a bijection on the first nb blocks, nb = the blocks the device-side unit
    // count needs (the launch may be larger: preprocess hands the host only capacities), so
    // the working blocks stay spread over all 8 XCDs; surplus blocks map to themselves and
    // exit.  With nunits > the grid's waves (grid-strided use) every block is remapped.
    const int need = (nunits + kWavesPerBlock - 1) / kWavesPerBlock;
    const int nb = min((int)gridDim.x, need), b = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (b >= nb) return b * kWavesPerBlock + w;
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    const int bb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    return bb * kWavesPerBlock + w;
}

// The same remap at block granularity (one unit per block; kernels stride by gridDim.x).
__device__ __forceinline__ int block_unit_index() {
    const int nb = gridDim.x, b = blockIdx.x;
    const int xcd = b & 7, q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// ---------------------------------------------------------------------------------------
// Reference-literal arithmetic (binning).  hipcc inlines the __f*_rn intrinsics into plain
// operators, which -ffp-contract=fast would then fuse into FMAs (measured: 28 % of 1e5
// determinants differed by an ulp), so every function here also turns contraction off.
// ---------------------------------------------------------------------------------------
// float -> int like CUDA's cvt.{rzi,rmi,rpi}.s32.f32: saturating, NaN -> 0.
__host__ __device__ inline int sat_int(float v) {
    if (v != v) return 0;
    if (v >= 2147483647.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

// IEEE single operations, never fused.  Not the __f*_rn intrinsics: they are OCML bitcode
// whose instructions carry `contract` flags and fuse after inlining whatever the caller's
// pragma.  sqrt and division go through double: double rounding through 53 >= 2*24+2 bits
// is innocuous for + - * / sqrt, and the device's f64 sqrt is correctly rounded while its
// f32 sqrt is not (tools/diag_radius.hip: 16 % of 1e5 results one ulp off).
__device__ __forceinline__ float rsub(float a, float b) { DGS_NO_CONTRACT return a - b; }
__device__ __forceinline__ float radd(float a, float b) { DGS_NO_CONTRACT return a + b; }
__device__ __forceinline__ float rmul(float a, float b) { DGS_NO_CONTRACT return a * b; }
__device__ __forceinline__ float rdiv(float a, float b) { return (float)((double)a / (double)b); }
__device__ __forceinline__ float rsqrt_cr(float a) { return (float)__builtin_sqrt((double)a); }

// forward.cu:52-61 (called only when not skipped by det == 0)
__device__ inline float ref_radius(int D, const float *cov) {
    DGS_NO_CONTRACT
    if (D == 1) return (float)(3.0 * (double)rsqrt_cr(cov[0]));
    const float det = rsub(rmul(cov[0], cov[2]), rmul(cov[1], cov[1]));
    const float mid = rmul(0.5f, radd(cov[0], cov[2]));
    const float disc = rsub(rmul(mid, mid), det);
    const double fl = fmax(1e-6, (double)disc);
    const float lambda = (float)((double)mid + sqrt(fl));
    return (float)(3.0 * (double)rsqrt_cr(lambda));
}

// auxiliary.h:21-31 (TORUS)
__device__ inline void ref_rect(int D, const float *p, float r, const float *off, int *rmin,
                                int *rmax) {
    DGS_NO_CONTRACT
    for (int i = 0; i < D; ++i) {
        const float d = rsub(p[i], off[i]);
        rmin[i] = sat_int(floorf(rdiv(rsub(d, r), kTile)));
        rmax[i] = sat_int(ceilf(rdiv(radd(d, r), kTile)));
    }
}

// forward.cu:24-83: returns tiles touched and the stored radius (0 = Gaussian skipped).
__device__ inline uint32_t ref_touched(int D, const float *mean, const float *cov,
                                       const int *grid, const float *off, float *radius) {
    DGS_NO_CONTRACT
    *radius = 0.0f;
    if (D == 2) {
        const float det = rsub(rmul(cov[0], cov[2]), rmul(cov[1], cov[1]));
        if (det == 0.0f) return 0;
    }
    const float r = ref_radius(D, cov);
    int rmin[2], rmax[2];
    ref_rect(D, mean, r, off, rmin, rmax);
    int t0 = rmax[0] - rmin[0];
    t0 = t0 < grid[0] ? t0 : grid[0];
    uint32_t touched;
    if (D == 1) {
        touched = (uint32_t)t0;
    } else {
        int t1 = rmax[1] - rmin[1];
        t1 = t1 < grid[1] ? t1 : grid[1];
        touched = (uint32_t)(t1 * t0);
    }
    if (touched == 0) return 0;
    *radius = r;
    return touched;
}

// The fast paths evaluate the exponent in their own operation order (pre-scaled k, FMAs).  With
// rho = |c1| / sqrt(c0 c2), max over X of (c0 X0^2 + 2 |c1 X0 X1| + c2 X1^2) / X^T A X
// = (1 + rho) / (1 - rho): cancellation amplifies the fp32 rounding of the exponent's terms by
// up to that factor, in ANY operation order -- the reference's own included.  nvcc's default
// --fmad=true (setup.py:30 passes no --fmad=false) fuses the reference's a*b + c*d exponent sum
// (forward.cu:177 ff.), and for thin Gaussians (rho^2 >= 0.82, axis ratio >= ~10) the fused and
// unfused reference differ by 1-2x the 1e-5 parity bound in the forward and 4-6x in the
// gradients (tools/contraction_study.py, profiles/r05_contraction.json): no operation order is
// "the reference's" there.  So thin conics take the fast paths like every other PD conic, under
// the stated bound of tests/test_gpu_parity.py (an a-priori bound on the exponent's
// rounding in any operation order).  (Round 4's kThin literal-order pass was removed in round 6.)
// Past rho^2 = kRho2Max (axis ratio ~89, amplification A = (1 + rho) / (1 - rho) ~8000) a conic
// is treated as not positive definite: up to there the fp32 exponent of a pair beyond the cut
// (X^T A X > 210, power < -105) is below -104.5 in any operation order (|error| <= ~3e-7 x A x 210
// = 0.5; expf is +0 below -103.97), so culling it drops an exact +0; past it the rounding could
// leave a subnormal term.  (0.999 -- A ~4000 -- left the axis-ratio-25 field's 107 thinnest
// Gaussians, rho^2 up to 0.99925, unculled: ~1500 literal-path entries each, +0.19 ms per forward.)
constexpr double kRho2Max = 0.9995;
// Not positive definite, too ill-conditioned (above), or not finite: kUnsafe, the per-pair
// literal path with the exact wrap and the reference's `power > 0 -> skip` (forward.cu:228).
__host__ __device__ inline bool conic_unsafe(int D, float c0f, float c1f, float c2f) {
    const double c0 = c0f, c1 = c1f, c2 = c2f;
    if (D == 1) return !(c0 >= 0.0 && c0 < INFINITY);
    return !(c0 > 0.0 && c2 > 0.0 && c0 < INFINITY && c2 < INFINITY && fabs(c1) < INFINITY &&
             c1 * c1 < kRho2Max * (c0 * c2));
}
// Positive definite but ill-conditioned, rho^2 = c1^2 / (c0 c2) >= 0.82 (D = 2): kept off the
// binning's gather path in -DDGS_THIN_GATHER=0 builds only (a tuning knob).
__host__ __device__ inline bool conic_thin(int D, float c0f, float c1f, float c2f) {
    if (D != 2 || conic_unsafe(D, c0f, c1f, c2f)) return false;
    const double c0 = c0f, c1 = c1f, c2 = c2f;
    return !(c1 * c1 < 0.82 * c0 * c2);
}

__host__ __device__ inline int wrap_tile(int x, int g) { return x < 0 ? (g + (x % g)) : (x % g); }

// sampler_impl.cu:54-129: the tile-key rectangle of one Gaussian (after the full-range rule).
struct KeyRect {
    int x0, x1, y0, y1;
};
__device__ inline KeyRect ref_key_rect(int D, const float *mean, float r, const int *grid,
                                       const float *off) {
    int rmin[2], rmax[2];
    ref_rect(D, mean, r, off, rmin, rmax);
    KeyRect k;
    if (rmax[0] - rmin[0] >= grid[0]) { rmin[0] = 0; rmax[0] = grid[0]; }
    k.x0 = rmin[0]; k.x1 = rmax[0];
    k.y0 = 0; k.y1 = 1;
    if (D == 2) {
        if (rmax[1] - rmin[1] >= grid[1]) { rmin[1] = 0; rmax[1] = grid[1]; }
        k.y0 = rmin[1]; k.y1 = rmax[1];
    }
    return k;
}
__device__ inline uint32_t key_of(int D, int x, int y, const int *grid) {
    if (D == 1) return (uint32_t)wrap_tile(x, grid[0]);
    return (uint32_t)(wrap_tile(y, grid[1]) * grid[0] + wrap_tile(x, grid[0]));
}

// sampler_impl.cu:155-189
__device__ inline uint32_t ref_sample_key(int D, const float *s, const int *grid,
                                          const float *off) {
    DGS_NO_CONTRACT
    uint32_t tile[2] = {0, 0};
    for (int i = 0; i < D; ++i) {
        int t = sat_int(rdiv(rsub(s[i], off[i]), kTile));
        t = t < 0 ? 0 : t;
        t = t > grid[i] ? grid[i] : t;
        tile[i] = (uint32_t)t;
    }
    return D == 1 ? tile[0] : tile[1] * (uint32_t)grid[0] + tile[0];
}

// forward.cu:149-157: exact period-2 wrap of one displacement (general path only).
__device__ __forceinline__ float ref_wrap(float x) {
    DGS_NO_CONTRACT
    if (fabsf(x) > 1.0f) {
        const float ax = fabsf(x);
        // |x| in (1, 2): fmod(x, 2) == x, so the result x -/+ 2 is exact in float.
        float r = ax < 2.0f ? ax : fmodf(ax, 2.0f);
        r = r - 2.0f;  // correctly rounded, same as the double computation rounded once
        x = x >= 0.0f ? r : -r;
    }
    return x;
}

// The even shift the reference's wrap applies to a displacement x (X' = x - shift): 0 for
// |x| <= 1, else sign(x) * 2 (floor(|x| / 2) + 1) -- fmod(x, 2) -/+ 2 in closed form.  On an
// interval of x that crosses none of the breakpoints |x| = 1, 2, 4, ... the shift is constant,
// and fl(m - s) - shift is then exact (Sterbenz), i.e. bit-identical to the reference.
__host__ __device__ inline double wrap_shift(double x) {
    const double ax = fabs(x);
    if (!(ax > 1.0)) return 0.0;
    return copysign(2.0 * (floor(ax * 0.5) + 1.0), x);
}
__device__ __forceinline__ float wrap_shift_f(float x) {
    const float ax = fabsf(x);
    return ax > 1.0f ? copysignf(2.0f * (floorf(ax * 0.5f) + 1.0f), x) : 0.0f;
}

// ref_wrap in closed form, branch-free and exact: fmod(|x|, 2) = |x| - 2 trunc(|x| / 2) is
// representable, so every step below is exact except the final `- 2`, which rounds once,
// like the reference's double expression rounded to float.  Identity for |x| <= 1.
__device__ __forceinline__ float wrap_exact(float x) {
    DGS_NO_CONTRACT
    const float ax = fabsf(x);
    const float f = ax - 2.0f * truncf(0.5f * ax);
    const float w = f - 2.0f;
    return ax > 1.0f ? (x >= 0.0f ? w : -w) : x;
}

// ---------------------------------------------------------------------------------------
// Fine-cell geometry.  Every reference tile is cut into n x n (D=2) or n (D=1) fine cells
// plus one unculled fallback cell for samples that lie outside their tile's nominal area
// (the reference's clamp-to-grid aliasing, sampler_impl.cu:169).  Cell id = tile*CT + local.
// ---------------------------------------------------------------------------------------
struct Geom {
    int D, T, n, CT, ncells;
    int grid[2];
    float off[2];
    double fs;   // fine cell size = 0.51f / n
    double ifs;  // 1 / fs (the binning's cell indices multiply by it: no fp64 divisions)
};

__device__ inline uint32_t sample_cell(const Geom &G, const float *s) {
    DGS_NO_CONTRACT
    const uint32_t key = ref_sample_key(G.D, s, G.grid, G.off);
    if (key >= (uint32_t)G.T) return (uint32_t)G.ncells;  // never rendered
    const int tx = G.D == 1 ? (int)key : (int)(key % (uint32_t)G.grid[0]);
    const int ty = G.D == 1 ? 0 : (int)(key / (uint32_t)G.grid[0]);
    const int tc[2] = {tx, ty};
    int f[2] = {0, 0};
    for (int i = 0; i < G.D; ++i) {
        const double d = (double)rsub(s[i], G.off[i]);
        const double u = (d - (double)tc[i] * (double)kTile) / G.fs;
        int fi = (int)floor(u);
        if (fi < 0) {
            if (u >= -kCellSlack) fi = 0;
            else return key * (uint32_t)G.CT + (uint32_t)(G.CT - 1);
        } else if (fi >= G.n) {
            if (u <= G.n + kCellSlack) fi = G.n - 1;
            else return key * (uint32_t)G.CT + (uint32_t)(G.CT - 1);
        }
        f[i] = fi;
    }
    return key * (uint32_t)G.CT + (uint32_t)(f[1] * G.n + f[0]);
}

// (cell, sub-cell) key = cell * 4 + sub: at D = 2 the sub-cell of a fine cell is the quadrant of
// its nominal square (bit 0: x in the upper half, bit 1: y); the fallback cell and D = 1 use
// sub 0.  Never-rendered samples: ncells * 4.
__device__ inline uint32_t sample_cell_sub(const Geom &G, const float *s) {
    DGS_NO_CONTRACT
    const uint32_t cell = sample_cell(G, s);
    if (cell >= (uint32_t)G.ncells) return (uint32_t)G.ncells * kSubPerCell;
    const uint32_t local = cell % (uint32_t)G.CT;
    if (G.D != 2 || local == (uint32_t)(G.CT - 1)) return cell * kSubPerCell;
    const uint32_t tile = cell / (uint32_t)G.CT;
    const int tc[2] = {(int)(tile % (uint32_t)G.grid[0]), (int)(tile / (uint32_t)G.grid[0])};
    const int f[2] = {(int)(local % (uint32_t)G.n), (int)(local / (uint32_t)G.n)};
    uint32_t sub = 0;
    for (int i = 0; i < 2; ++i) {
        const double d = (double)rsub(s[i], G.off[i]);
        const double u = (d - (double)tc[i] * (double)kTile) / G.fs - (double)f[i];
        if (u >= 0.5) sub |= 1u << i;
    }
    return cell * kSubPerCell + sub;
}

// ---------------------------------------------------------------------------------------
// Host-side launch hints.  preprocess records the exact work-unit counts of the buffers it
// created; forward/backward size their grids from them.  The kernels grid-stride over the
// device-side counts, so a missing or stale hint only costs speed, never correctness.
// ---------------------------------------------------------------------------------------
struct UnitHint {
    const void *gbuf, *sbuf;
    size_t gbytes, sbytes;
    int64_t nfwd, nbwd, nfsub, ncells;
    int64_t nunsafe;  // kUnsafe entries (the forward's tail pass)
    int64_t nthin;    // kThin entries (the forward's thin pass)
    int32_t P, D, N;  // the problem the buffers were built for (validate() checks calls against it)
    int64_t R;        // num_rendered (sizes the call-time path's backward grid)
    int64_t E;        // fine (Gaussian, cell) entries
    int64_t Es;       // of which sort-path entries (the backward's slot sums)
    Header hdr;       // the header preprocess wrote (ensure_ref_lists reads its geometry / offsets)
    bool ref_built;   // rlist built (ensure_ref_lists), ref_done recorded after its build
    bool capture = false;  // a graph-capturable binning: R / E / nunsafe are on the device only
    bool own_grid = false;  // the grid was the samples' own (dgs_preprocess_auto[_ex])
    hipEvent_t ref_done;
};
void hint_put(const UnitHint &h);
bool hint_get(const void *gbuf, size_t gbytes, const void *sbuf, size_t sbytes, UnitHint *out);
// The newest binning whose sample buffer is (sbuf, sbytes) (dgs_bin_options.samples_binned).
bool hint_by_sbuf(const void *sbuf, size_t sbytes, UnitHint *out);
// The call-time path's tile lists (rlist) of a binning: built on `s` at the first call that may
// take that path (any call not flagged DGS_SAMPLE_INPUTS_BINNED); later calls on another stream
// wait for that build.  Buffers without a hint (not made by this process) are rebuilt per call.
int ensure_ref_lists(const void *gbuf, size_t gbytes, const void *sbuf, size_t sbytes, hipStream_t s, int debug);
// Counts the library's own stream-ordered allocations (dgs_internal_allocations, dgs.h): the
// diagnostics, dgs_tile_grid and the call-time path's first use; the hot path makes none.
void note_internal_alloc();

// ---------------------------------------------------------------------------------------
// Host-side error state
// ---------------------------------------------------------------------------------------
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
int check_hip(hipError_t e, const char *what);

}  // namespace dgs

#define DGS_TRY_HIP(expr)                                                        \
    do {                                                                         \
        int _rc = ::dgs::check_hip((expr), #expr);                               \
        if (_rc) return _rc;                                                     \
    } while (0)

// Launch check; with debug, synchronise and surface asynchronous faults (auxiliary.h:33-40).
#define DGS_LAUNCH_CHECK(stream, debug)                                          \
    do {                                                                         \
        DGS_TRY_HIP(hipGetLastError());                                          \
        if (debug) DGS_TRY_HIP(hipStreamSynchronize(stream));                    \
    } while (0)
