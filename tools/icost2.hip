// icost2.hip -- does v_exp_f32 overlap packed fp32 VALU work on gfx950?  Per-wave instruction
// mixes at full occupancy (8 blocks x 256 threads per CU, independent chains), timed with HIP
// events; prints SIMD-cycles per loop iteration at a nominal 2.4 GHz.
//   hipcc --offload-arch=gfx950 -O3 -o tools/icost2 tools/icost2.hip && tools/icost2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

// NPK packed FMAs (over 8 independent f2 chains) and NEX v_exp_f32 (over 4 independent float
// chains) per iteration.
template <int NPK, int NEX>
__global__ __launch_bounds__(256) void k(float *out, int iters, float a, float b) {
    f2 y[8];
    float x[4];
    for (int i = 0; i < 8; ++i) y[i] = f2{threadIdx.x * 1e-3f + i, threadIdx.x * 1e-3f - i};
    for (int i = 0; i < 4; ++i) x[i] = -1e-3f * threadIdx.x - i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NPK; ++i) y[i & 7] = __builtin_elementwise_fma(y[i & 7], f2{a, a}, f2{b, b});
#pragma unroll
        for (int i = 0; i < NEX; ++i) x[i & 3] = __builtin_amdgcn_exp2f(x[i & 3]) - 2.0f;
    }
    float s = 0;
    for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y;
    for (int i = 0; i < 4; ++i) s += x[i];
    if (s == 1234.5f) out[threadIdx.x] = s;
}

// The same, but the exp chain consumes and feeds the packed chains (the pair loop's shape:
// p -> exp -> t -> accumulators), NCH independent pair-pairs per iteration.
template <int NCH>
__global__ __launch_bounds__(256) void kpair(float *out, int iters, float a, float b) {
    f2 acc[NCH][6], X[NCH][2];
    for (int c = 0; c < NCH; ++c) {
        for (int i = 0; i < 6; ++i) acc[c][i] = f2{0.f, 0.f};
        X[c][0] = f2{threadIdx.x * 1e-4f + c, threadIdx.x * 2e-4f};
        X[c][1] = f2{threadIdx.x * -1e-4f, c * 1e-3f};
    }
    const f2 k0 = f2{-0.7f, -0.7f}, k1 = f2{0.1f, 0.1f}, k2 = f2{-0.5f, -0.5f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const f2 x0 = X[c][0] - f2{a, b}, x1 = X[c][1] - f2{b, a};
            const f2 q0 = x0 * x0, q1 = x0 * x1, q2 = x1 * x1;
            const f2 p = __builtin_elementwise_fma(k2, q2, __builtin_elementwise_fma(k1, q1, k0 * q0));
            const f2 e = f2{__builtin_amdgcn_exp2f(p.x), __builtin_amdgcn_exp2f(p.y)};
            const f2 t = e * f2{a, a};
            acc[c][0] += t;
            acc[c][1] = __builtin_elementwise_fma(t, x0, acc[c][1]);
            acc[c][2] = __builtin_elementwise_fma(t, x1, acc[c][2]);
            acc[c][3] = __builtin_elementwise_fma(t, q0, acc[c][3]);
            acc[c][4] = __builtin_elementwise_fma(t, q1, acc[c][4]);
            acc[c][5] = __builtin_elementwise_fma(t, q2, acc[c][5]);
            X[c][0] = X[c][0] + f2{1e-7f, 1e-7f};
        }
    }
    float s = 0;
    for (int c = 0; c < NCH; ++c)
        for (int i = 0; i < 6; ++i) s += acc[c][i].x + acc[c][i].y;
    if (s == 1234.5f) out[threadIdx.x] = s;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus * 8, iters = 20000;
    float *out;
    hipMalloc(&out, 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, double per_iter_insts, auto f) {
        f();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) f();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double waves_per_simd = (double)blocks * 4 / (cus * 4);
        const double cyc = ms * 1e-3 * 2.4e9 / (waves_per_simd * iters);
        printf("%-28s %.3f ms  %.2f SIMD-cycles per wave-iteration (%.0f insts)\n", name, ms, cyc, per_iter_insts);
    };
#define RUN(A, B) run(#A " pk_fma + " #B " exp", A + B, [&] { k<A, B><<<blocks, 256>>>(out, iters, 0.999f, 1e-3f); })
    RUN(8, 0);
    RUN(16, 0);
    RUN(0, 4);
    RUN(0, 8);
    RUN(8, 2);
    RUN(16, 2);
    RUN(16, 4);
    RUN(15, 2);
    RUN(8, 4);
    run("pair loop x1 (15pk+2exp)", 17, [&] { kpair<1><<<blocks, 256>>>(out, iters, 0.999f, 1e-3f); });
    run("pair loop x2", 34, [&] { kpair<2><<<blocks, 256>>>(out, iters, 0.999f, 1e-3f); });
    run("pair loop x4", 68, [&] { kpair<4><<<blocks, 256>>>(out, iters, 0.999f, 1e-3f); });
    return 0;
}
