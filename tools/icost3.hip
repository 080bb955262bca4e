// icost3.hip -- do f32 MFMAs (v_mfma_f32_16x16x4_f32) and f32 VALU work execute together on one
// gfx950 SIMD?  Per-wave instruction mixes at a fixed occupancy, timed with HIP events; prints
// SIMD-cycles per loop iteration at a nominal 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 -o tools/icost3 tools/icost3.hip && tools/icost3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

// MODE 0: NM MFMAs (4 independent accumulators) and NV v_fma_f32 (8 independent chains) per
// iteration in every wave; MODE 1: waves 0-3 of the 512-thread block the MFMAs only, waves 4-7
// (the same four SIMDs: two waves each) the VALU only.
template <int NM, int NV, int MODE>
__global__ __launch_bounds__(512) void k(float *out, int iters, float a, float b) {
    f32x4 acc[4];
    float y[8];
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int i = 0; i < 8; ++i) y[i] = threadIdx.x * 1e-3f + i;
    const int w = threadIdx.x >> 6;
    const bool dom = MODE == 0 || w < 4, dov = MODE == 0 || w >= 4;
    const float x = threadIdx.x * 1e-3f;
    for (int it = 0; it < iters; ++it) {
        if (dom) {
#pragma unroll
            for (int i = 0; i < NM; ++i) acc[i & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, a, acc[i & 3], 0, 0, 0);
        }
        if (dov) {
#pragma unroll
            for (int i = 0; i < NV; ++i) y[i & 7] = __builtin_fmaf(y[i & 7], a, b);
        }
    }
    float s = 0;
    for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    for (int i = 0; i < 8; ++i) s += y[i];
    if (s == 1234.5f) out[threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, iters = 20000;
    float *out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, int bpc, auto f) {
        const int blocks = cus * bpc;
        f(blocks);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) f(blocks);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double waves_per_simd = (double)blocks * 8 / (cus * 4);
        // SIMD-cycles per iteration of ONE wave, times the waves sharing the SIMD: cycles per
        // SIMD per (waves_per_simd iterations)
        const double cyc = ms * 1e-3 * 2.4e9 / iters;
        printf("%-44s waves/SIMD %.0f: %.3f ms, %.1f SIMD-cycles per iteration of all its waves\n", name,
               waves_per_simd, ms, cyc);
    };
#define RUN(NM, NV, MODE, BPC)                                                                     \
    run(#NM " mfma + " #NV " fma, mode " #MODE, BPC,                                                \
        [&](int blocks) { k<NM, NV, MODE><<<blocks, 512>>>(out, iters, 0.999f, 1e-3f); })
    for (int bpc : {1, 2, 3}) {
        RUN(8, 0, 0, bpc);
        RUN(0, 96, 0, bpc);
        RUN(8, 96, 0, bpc);
        RUN(8, 96, 1, bpc);
        RUN(8, 48, 0, bpc);
    }
    return 0;
}
