// Diagnostic: each step of the reference-radius arithmetic on the device, fed the host's
// inputs, against the host (IEEE, no contraction).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>
#pragma clang fp contract(off)

__global__ void k(int n, const float* in, double* out) {
#pragma clang fp contract(off)
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* c = in + 8 * i;  // c0 c1 c2 mid det lambda  (host values)
    const double fl = (double)in[8 * i + 6] ;
    out[8 * i + 0] = __fsub_rn(__fmul_rn(c[0], c[2]), __fmul_rn(c[1], c[1]));   // det
    out[8 * i + 1] = __fsub_rn(__fmul_rn(c[3], c[3]), c[4]);                     // disc
    out[8 * i + 2] = sqrt(fl);                                                     // double sqrt
    out[8 * i + 3] = __fsqrt_rn(c[5]);                                             // float sqrt
    out[8 * i + 4] = __fdiv_rn(c[0], 0.51f);                                       // division
    out[8 * i + 5] = (float)(3.0 * (double)c[5]);
}

int main() {
    const int n = 100000;
    std::mt19937 g(1);
    std::uniform_real_distribution<float> u(0.5f, 1.5f), th(0.0f, 3.14159f);
    std::vector<float> in(8 * n);
    std::vector<double> ref(8 * n);
    for (int i = 0; i < n; ++i) {
        float h = 0.0632f, s0 = h * u(g), s1 = h * u(g), t = th(g);
        float cc = cosf(t), ss = sinf(t);
        float* c = &in[8 * i];
        c[0] = cc * cc * s0 * s0 + ss * ss * s1 * s1;
        c[1] = cc * ss * (s0 * s0 - s1 * s1);
        c[2] = ss * ss * s0 * s0 + cc * cc * s1 * s1;
        volatile float a = c[0] * c[2], b = c[1] * c[1];
        float det = a - b;
        volatile float sm = c[0] + c[2];
        float mid = 0.5f * sm;
        volatile float mm = mid * mid;
        float disc = mm - det;
        double fl = fmax(1e-6, (double)disc);
        float lambda = (float)((double)mid + sqrt(fl));
        c[3] = mid; c[4] = det; c[5] = lambda; c[6] = (float)fl;
        volatile float dv = c[0] / 0.51f;
        ref[8 * i + 0] = det; ref[8 * i + 1] = disc; ref[8 * i + 2] = sqrt((double)(float)fl);
        ref[8 * i + 3] = sqrtf(lambda); ref[8 * i + 4] = dv; ref[8 * i + 5] = (float)(3.0 * (double)lambda);
    }
    float* dc; double* dout;
    (void)hipMalloc(&dc, 32 * n); (void)hipMalloc(&dout, 64 * n);
    (void)hipMemcpy(dc, in.data(), 32 * n, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(n, dc, dout);
    std::vector<double> o(8 * n);
    (void)hipMemcpy(o.data(), dout, 64 * n, hipMemcpyDeviceToHost);
    const char* names[6] = {"det", "disc", "dsqrt", "fsqrt_rn", "fdiv_rn", "3*x"};
    for (int k2 = 0; k2 < 6; ++k2) {
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += ref[8 * i + k2] != o[8 * i + k2];
        printf("%s mismatches %d / %d\n", names[k2], bad, n);
    }
    return 0;
}
