// Checks reduce_scatter64 against a serial per-value sum (run on the GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include "dgs_render.h"
__global__ void k(const float *in, float *out) {
    const int lane = threadIdx.x & 63;
    float x[64];
    for (int i = 0; i < 64; ++i) x[i] = in[lane * 64 + i];
    out[lane] = dgs::reduce_scatter64(x, lane);
}
int main() {
    float h[4096], r[64];
    for (int i = 0; i < 4096; ++i) h[i] = (float)((i * 7919) % 1000) * 0.001f - 0.5f + (i % 64);
    float *din, *dout;
    if (hipMalloc(&din, sizeof h) || hipMalloc(&dout, 256)) return 2;
    if (hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice)) return 2;
    k<<<1, 64>>>(din, dout);
    if (hipMemcpy(r, dout, 256, hipMemcpyDeviceToHost)) return 2;
    int bad = 0;
    for (int j = 0; j < 64; ++j) {
        double s = 0; for (int l = 0; l < 64; ++l) s += h[l * 64 + j];
        if (std::fabs(r[j] - s) > 1e-3 * (1 + std::fabs(s))) { if (bad < 5) printf("lane %d: got %f want %f\n", j, r[j], s); ++bad; }
    }
    printf("reduce_scatter64: %s (%d bad)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 1 : 0;
}
