// ubench.hip -- microbenchmarks for the render kernels' building blocks on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip && tools/ubench
// Each kernel runs 7 blocks x 256 threads per CU; reported: cycles per (wave, item) at the
// measured clock, i.e. how many SIMD cycles one wave's work item costs when every SIMD is full.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f32x8_t __attribute__((ext_vector_type(8)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <typename V>
__device__ __forceinline__ V vexp2(V x);
template <> __device__ __forceinline__ float vexp2<float>(float x) { return __builtin_amdgcn_exp2f(x); }
template <> __device__ __forceinline__ f2 vexp2<f2>(f2 x) { return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ f32x8_t sload8(const float *p) {
    const f32x8_t v = *(const __attribute__((address_space(4))) f32x8_t *)(p);
    asm volatile("" ::"s"(v));
    return v;
}

// (1) the forward's pair math with the Gaussian rows delivered by:
//   MODE 0: SGPRs loaded once (no per-row delivery: the VALU bound; samples drift per iteration)
//   MODE 1: one s_load_dwordx8 per row (scalar-cache hits)
//   MODE 2: one s_load_dwordx16 per two adjacent rows
//   MODE 3: LDS broadcast, two ds_read_b128 per row (all lanes one address)
template <typename V, int MODE>
__global__ __launch_bounds__(256) void k_pairs(const float *__restrict__ table, int iters, float *out) {
    __shared__ float lds[1024 * 8];
    const int lane = threadIdx.x & 63;
    if constexpr (MODE == 3) {
        for (int i = threadIdx.x; i < 1024 * 8; i += 256) lds[i] = table[i];
        __syncthreads();
    }
    V s0, s1;
    if constexpr (sizeof(V) == 8) { s0 = V{lane * 1e-3f, lane * 2e-3f}; s1 = V{lane * 3e-3f, lane * 4e-3f}; }
    else { s0 = lane * 1e-3f; s1 = lane * 3e-3f; }
    V acc = s0 * 0.0f, acc2 = acc;
    float r0[8][8];
    if constexpr (MODE == 0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f32x8_t v = sload8(table + q * 8);
#pragma unroll
            for (int k = 0; k < 8; ++k) r0[q][k] = v[k];
        }
    }
    for (int it = 0; it < iters; ++it) {
        float r[8][8];
        const int base = (it * 8) & 1023;
        if constexpr (MODE == 0) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
#pragma unroll
                for (int k = 0; k < 8; ++k) r[q][k] = r0[q][k];
            s0 += 1e-7f;
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const f32x8_t v = sload8(table + (base + q) * 8);
#pragma unroll
                for (int k = 0; k < 8; ++k) r[q][k] = v[k];
            }
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                typedef float f32x16_t __attribute__((ext_vector_type(16)));
                const f32x16_t v = *(const __attribute__((address_space(4))) f32x16_t *)(table + (base + q) * 8);
                asm volatile("" ::"s"(v));
#pragma unroll
                for (int k = 0; k < 8; ++k) { r[q][k] = v[k]; r[q + 1][k] = v[8 + k]; }
            }
        } else {
            const int ub = __builtin_amdgcn_readfirstlane(base);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float4 x = *reinterpret_cast<const float4 *>(&lds[(ub + q) * 8]);
                const float4 y = *reinterpret_cast<const float4 *>(&lds[(ub + q) * 8 + 4]);
                r[q][0] = x.x; r[q][1] = x.y; r[q][2] = x.z; r[q][3] = x.w;
                r[q][4] = y.x; r[q][5] = y.y; r[q][6] = y.z; r[q][7] = y.w;
            }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const V X0 = r[q][0] - s0, X1 = r[q][1] - s1;
            const V p = vfma(X0, vfma(V(r[q][2]), X0, r[q][3] * X1), r[q][4] * X1 * X1);
            const V G = vexp2(p);
            if (q & 1) acc2 = vfma(V(r[q][5]), G, acc2);
            else acc = vfma(V(r[q][5]), G, acc);
        }
    }
    acc += acc2;
    float o;
    if constexpr (sizeof(V) == 8) o = acc.x + acc.y; else o = acc;
    if (o == 12345.0f) out[threadIdx.x] = o;
}

// (1b) transposed forward body: lane = Gaussian (row in VGPRs), samples wave-uniform from
// sequential s_load_dwordx16 of packed pair rows [s0a s0b s1a s1b] (4 pairs per load), the
// lane accumulates a per-sample partial sum in acc[NP] (f2).  Item = one sample pair.
// PF: issue the next load right after the wait for the current one (one load in flight).
template <int NP, bool PF>
__global__ __launch_bounds__(256) void k_transposed(const float *__restrict__ table, const float *__restrict__ srows,
                                                    int iters, float *out) {
    typedef float f32x16_t __attribute__((ext_vector_type(16)));
    const int lane = threadIdx.x & 63;
    const float m0 = table[lane * 8], m1 = table[lane * 8 + 1], k0 = -table[lane * 8 + 2] * 100.f,
                k1 = table[lane * 8 + 3], k2 = -table[lane * 8 + 4] * 100.f, v = table[lane * 8 + 5];
    f2 acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = f2{0.f, 0.f};
    constexpr int NL = NP / 4;
    for (int it = 0; it < iters; ++it) {
        const float *sr = srows + ((it * NP * 4) & 4095);
        f32x16_t q = *(const __attribute__((address_space(4))) f32x16_t *)(sr);
#pragma unroll
        for (int b = 0; b < NL; ++b) {
            f32x16_t qn;
            if constexpr (PF) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (b + 1 < NL) qn = *(const __attribute__((address_space(4))) f32x16_t *)(sr + (b + 1) * 16);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const f2 s0 = f2{q[4 * j], q[4 * j + 1]}, s1 = f2{q[4 * j + 2], q[4 * j + 3]};
                const f2 X0 = m0 - s0, X1 = m1 - s1;
                const f2 p = vfma(X0, vfma(f2{k0, k0}, X0, k1 * X1), k2 * X1 * X1);
                acc[b * 4 + j] = vfma(f2{v, v}, vexp2(p), acc[b * 4 + j]);
            }
            if constexpr (PF) { if (b + 1 < NL) q = qn; }
            else if (b + 1 < NL) q = *(const __attribute__((address_space(4))) f32x16_t *)(sr + (b + 1) * 16);
        }
    }
    float o = 0.f;
#pragma unroll
    for (int p = 0; p < NP; ++p) o += acc[p].x + acc[p].y;
    if (o == 12345.0f) out[threadIdx.x] = o;
}

// (2) scalar-load throughput: each wave streams s_load_dwordx8 rows by an index array
// (entries) -- the forward's access pattern without its math.  SPAN = table rows touched.
__global__ __launch_bounds__(256) void k_sload(const float *__restrict__ table, const unsigned *__restrict__ ids,
                                               int iters, unsigned mask, float *out) {
    float acc = 0.0f;
    const int w = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 7919;
    for (int it = 0; it < iters; ++it) {
        f32x8_t v[8];
        const unsigned base = (unsigned)(w + it * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = sload8(table + ((base + q * 131) & mask) * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q][0];
    }
    if (acc == 12345.0f) out[threadIdx.x] = acc;
}

int main() {
    int dev = 0;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    const int blocks = cus * 7;
    const int waves = blocks * 4;
    const size_t trows = 1 << 22;  // 128 MiB of 32-byte rows
    std::vector<float> h(trows * 8);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-4f - 0.05f;
    float *table, *out;
    CHECK(hipMalloc(&table, h.size() * 4));
    CHECK(hipMalloc(&out, 4096));
    CHECK(hipMemcpy(table, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    const double ghz = prop.clockRate * 1e-6;
    auto run = [&](const char *name, auto launch, double items_per_wave) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        for (int r = 0; r < 5; ++r) launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        ms /= 5;
        // SIMD-cycles per item = time * clock * (SIMDs) / (waves * items)
        const double cyc = ms * 1e-3 * ghz * 1e9 * (cus * 4) / (waves * items_per_wave);
        printf("%-34s %8.3f ms  %7.2f SIMD-cycles per wave-item (at %.2f GHz nominal)\n", name, ms, cyc, ghz);
        return 0;
    };
    const int it = 2000;
    run("pairs f32 rows in SGPRs (VALU bound)", [&] { k_pairs<float, 0><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f2  rows in SGPRs (VALU bound)", [&] { k_pairs<f2, 0><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f32 s_load x8 per row", [&] { k_pairs<float, 1><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f2  s_load x8 per row", [&] { k_pairs<f2, 1><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f32 s_load x16 per 2 rows", [&] { k_pairs<float, 2><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f2  s_load x16 per 2 rows", [&] { k_pairs<f2, 2><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f32 LDS broadcast rows", [&] { k_pairs<float, 3><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("pairs f2  LDS broadcast rows", [&] { k_pairs<f2, 3><<<blocks, 256>>>(table, it, out); }, it * 8.0);
    run("transposed f2 acc32", [&] { k_transposed<32, false><<<blocks, 256>>>(table, table + 64 * 8, it / 4, out); }, it / 4 * 32.0);
    run("transposed f2 acc32 prefetch", [&] { k_transposed<32, true><<<blocks, 256>>>(table, table + 64 * 8, it / 4, out); }, it / 4 * 32.0);
    run("transposed f2 acc16", [&] { k_transposed<16, false><<<blocks, 256>>>(table, table + 64 * 8, it / 2, out); }, it / 2 * 16.0);
    run("transposed f2 acc16 prefetch", [&] { k_transposed<16, true><<<blocks, 256>>>(table, table + 64 * 8, it / 2, out); }, it / 2 * 16.0);
    const unsigned masks[] = {255u, 4095u, 65535u, (1u << 20) - 1, (1u << 22) - 1};
    for (unsigned m : masks) {
        char name[64];
        snprintf(name, sizeof name, "s_load_x8 rows, %u KiB span", (unsigned)(((size_t)m + 1) * 32 / 1024));
        run(name, [&] { k_sload<<<blocks, 256>>>(table, nullptr, it / 4, m, out); }, it / 4 * 8.0);
    }
    return 0;
}
