// icost.hip -- per-instruction VALU throughput on gfx950 (wave64, 8 blocks x 256 threads per
// CU, independent accumulators): v_fma_f32, v_pk_fma_f32, v_exp_f32 and mixes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/icost tools/icost.hip && tools/icost
// Results are quoted in DESIGN.md section 5.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int K>
__global__ __launch_bounds__(256) void k(float *out, int iters, float a, float b) {
    float x[8]; f2 y[8];
    for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x * 1e-3f + i; y[i] = f2{x[i], x[i] + 1}; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (K == 0) x[i] = fmaf(x[i], a, b);
            if constexpr (K == 1) y[i] = __builtin_elementwise_fma(y[i], f2{a, a}, f2{b, b});
            if constexpr (K == 2) x[i] = __builtin_amdgcn_exp2f(x[i]);
            if constexpr (K == 3) { x[i] = fmaf(x[i], a, b); y[i] = __builtin_elementwise_fma(y[i], f2{a, a}, f2{b, b}); }
            if constexpr (K == 4) { x[i] = __builtin_amdgcn_exp2f(x[i]); y[i] = __builtin_elementwise_fma(y[i], f2{a, a}, f2{b, b}); }
            if constexpr (K == 5) y[i] = y[i] * f2{a, a} + y[i];
        }
    }
    float s = 0; for (int i = 0; i < 8; ++i) s += x[i] + y[i].x + y[i].y;
    if (s == 1234.5f) out[threadIdx.x] = s;
}
int main() {
    hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
    int cus = p.multiProcessorCount, blocks = cus * 8; float *out; hipMalloc(&out, 4096);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const char *names[] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "fma + pk_fma", "exp + pk_fma", "pk_mul+pk_add"};
    auto run = [&](int K, auto f) {
        f(); hipDeviceSynchronize(); hipEventRecord(e0); for (int r = 0; r < 3; ++r) f(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
        double insts = (double)blocks * 4 * 20000 * 8;  // wave-instructions (per kind)
        printf("%-16s %.3f ms  %.2f SIMD-cycles per wave-instruction (2.4 GHz)\n", names[K], ms, ms * 1e-3 * 2.4e9 * cus * 4 / insts);
    };
    run(0, [&] { k<0><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
    run(1, [&] { k<1><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
    run(2, [&] { k<2><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
    run(3, [&] { k<3><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
    run(4, [&] { k<4><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
    run(5, [&] { k<5><<<blocks, 256>>>(out, 20000, 0.999f, 1e-3f); });
}
