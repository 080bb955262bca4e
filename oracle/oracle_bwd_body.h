/*
 * oracle_bwd_body.h -- one pair's gradient contributions (backward.cu:108-416), instantiated twice
 * by oracle.c:
 *   BWD_T = float : the reference's literal float accumulation (`+=` of each float term);
 *   BWD_T = double: the same float terms, summed exactly to double -- the value every order of
 *                   the reference's float atomics scatters around (backward.cu: atomicAdd).
 * Contraction sites (oracle.c ORC_FMAD): the exponent's float sum (SUM2), a1/a2 and the
 * a*a - c terms (FMA), the per-channel sums `dL_dG += values*dL` (FMA), the float a*b + c*d
 * sums of the gradient terms (SUM2 / FMA chains, left to right as written).  Double-promoted
 * expressions are left to the contracting compiler of models 1/2 (oracle/Makefile); their
 * products of floats are mostly exact in double.  ACC: the atomicAdd operand, rounded on its own.
 * TEST INFRASTRUCTURE ONLY (see oracle.c).
 */
#define ACC(dst, term) ((dst) += (BWD_T)orc_rounded((float)(term)))
/* backward.cu:108-416 -- one pair's gradient contributions (literal formulas, including the
 * reference's D=1 third-derivative conic gradient at backward.cu:322-325). */
static void BWD_FN(bwd_pair)(int fn, int D, int C, const float *X, const float *c, const float *v,
                     const float *dL /* [K][C] of this sample */, BWD_T *gm, BWD_T *gv, BWD_T *gc) {
    if (D == 1) {
        float x1 = c[0] * X[0];
        float power = fn == F_GAUSS ? (float)(-0.5 * c[0] * X[0] * X[0]) : (float)(-0.5 * x1 * X[0]);
        if (power > 0.0) return;
        float G = expf(power);
        float dLdG = 0.0f;
        for (int ch = 0; ch < C; ++ch) {
            float d = dL[ch];
            switch (fn) {
            case F_GAUSS: ACC(gv[ch], G * d); break;
            case F_DERIV: ACC(gv[ch], x1 * d * G); break;
            case F_LAPL: { float gx = FMA(x1, x1, -c[0]) * d; ACC(gv[ch], gx * G); } break;
            default: { float gx = (float)((3.0 * c[0] * x1 - (double)(x1 * x1 * x1)) * d); ACC(gv[ch], gx * G); }
            }
            dLdG = FMA(v[ch], d, dLdG);
        }
        switch (fn) {
        case F_GAUSS: {
            float gdx = G * X[0];
            float dG = gdx * c[0];
            float dLdx = dLdG * dG;
            ACC(gm[0], -dLdx);
            ACC(gc[0], (float)(-0.5 * gdx * X[0] * dLdG));
        } break;
        case F_DERIV: {
            float dLdx = FMA(x1, x1, -c[0]) * dLdG * G;
            ACC(gm[0], -dLdx);
            ACC(gc[0], (float)(((double)X[0] - 0.5 * X[0] * X[0] * x1) * dLdG * G));
        } break;
        case F_LAPL: {
            float dLdx = (float)(((double)(x1 * x1 * x1) - 3.0 * c[0] * x1) * dLdG * G);
            float dVdc = (float)((2.0 * x1 * X[0] - 0.5 * FMA(x1, x1, -c[0]) * X[0] * X[0] - 1.0) * dLdG * G);
            ACC(gm[0], -dLdx);
            ACC(gc[0], dVdc);
        } break;
        default: {
            float dLdx = (float)((6.0 * c[0] * x1 * x1 - (double)(x1 * x1 * x1 * x1) - 3.0 * c[0] * c[0]) * dLdG * G);
            /* backward.cu:322-325: not the true derivative; reproduced literally */
            float dVdc = (float)((2.0 * X[0] * X[0] - 2.0 * x1 * x1 * X[0] - 0.5 * (2.0 * X[0] * x1 - X[0]) * X[0] * X[0]
                                  + 0.5 * FMA(x1, x1, -c[0]) * x1 * X[0] * X[0]) * dLdG * G);
            ACC(gm[0], -dLdx);
            ACC(gc[0], dVdc);
        }
        }
        return;
    }
    float x1 = c[0] * X[0], x2 = c[2] * X[1];
    float power;
    if (fn == F_GAUSS)
        power = (float)(-0.5 * (double)SUM2(c[0] * X[0], X[0], c[2] * X[1], X[1]) - (double)(c[1] * X[0] * X[1]));
    else
        power = (float)(-0.5 * (double)SUM2(x1, X[0], x2, X[1]) - (double)(c[1] * X[0] * X[1]));
    if (power > 0.0) return;
    float G = expf(power);
    float a1 = FMA(c[1], X[1], x1), a2 = FMA(c[1], X[0], x2);
    if (fn == F_GAUSS) {
        float dLdG = 0.0f;
        for (int ch = 0; ch < C; ++ch) { ACC(gv[ch], G * dL[ch]); dLdG = FMA(v[ch], dL[ch], dLdG); }
        float gdx = G * X[0], gdy = G * X[1];
        ACC(gm[0], -dLdG * SUM2(gdx, c[0], gdy, c[1]));
        ACC(gm[1], -dLdG * SUM2(gdx, c[1], gdy, c[2]));
        ACC(gc[0], (float)(-0.5 * gdx * X[0] * dLdG));
        ACC(gc[1], -gdy * X[0] * dLdG);
        ACC(gc[2], (float)(-0.5 * gdy * X[1] * dLdG));
        return;
    }
    if (fn == F_DERIV) {
        float Gx = 0.0f, Gy = 0.0f;
        for (int ch = 0; ch < C; ++ch) {
            float dx = dL[ch], dy = dL[C + ch];
            float gx = SUM2(a1, dx, a2, dy);
            ACC(gv[ch], gx * G);
            Gx = FMA(v[ch], dx, Gx);
            Gy = FMA(v[ch], dy, Gy);
        }
        float gx = SUM2(a1, Gx, a2, Gy);
        float dLdx = SUM2(FMA(a1, a1, -c[0]), Gx, FMA(a1, a2, -c[1]), Gy) * G;
        float dLdy = SUM2(FMA(a2, a2, -c[2]), Gy, FMA(a1, a2, -c[1]), Gx) * G;
        ACC(gm[0], -dLdx);
        ACC(gm[1], -dLdy);
        ACC(gc[0], (float)(((double)(X[0] * Gx) - 0.5 * X[0] * X[0] * gx) * G));
        ACC(gc[1], FMA(-(X[0] * X[1]), gx, SUM2(X[1], Gx, X[0], Gy)) * G);
        ACC(gc[2], (float)(((double)(X[1] * Gy) - 0.5 * X[1] * X[1] * gx) * G));
        return;
    }
    if (fn == F_LAPL) {
        float dxx = FMA(a1, a1, -c[0]), dxy = FMA(a1, a2, -c[1]), dyy = FMA(a2, a2, -c[2]);
        float Gxx = 0.0f, Gxy = 0.0f, Gyx = 0.0f, Gyy = 0.0f;
        for (int ch = 0; ch < C; ++ch) {
            float d0 = dL[ch], d1 = dL[C + ch], d2 = dL[2 * C + ch], d3 = dL[3 * C + ch];
            float g = FMA(dyy, d3, FMA(dxy, d2, SUM2(dxx, d0, dxy, d1)));
            ACC(gv[ch], g * G);
            Gxx = FMA(v[ch], d0, Gxx); Gxy = FMA(v[ch], d1, Gxy);
            Gyx = FMA(v[ch], d2, Gyx); Gyy = FMA(v[ch], d3, Gyy);
        }
        float dLdx = (float)(((double)(a1 * a1 * a1) - 3.0 * c[0] * a1) * Gxx
                             + (double)((a1 * a2 * a1 - c[1] * a1 - FMA(c[1], a1, c[0] * a2)) * (Gxy + Gyx))
                             + ((double)(a2 * a2 * a1 - c[2] * a1) - 2.0 * c[1] * a2) * Gyy) * G;
        float dLdy = (float)(((double)(a1 * a1 * a2 - c[0] * a2) - 2.0 * c[1] * a1) * Gxx
                             + (double)((a1 * a2 * a2 - c[1] * a2 - FMA(c[2], a1, c[1] * a2)) * (Gxy + Gyx))
                             + ((double)(a2 * a2 * a2) - 3.0 * c[2] * a2) * Gyy) * G;
        ACC(gm[0], -dLdx);
        ACC(gm[1], -dLdy);
        float S = Gxy + Gyx;
        float xx_cxx = (float)(-0.5 * dxx * X[0] * X[0] + 2.0 * a1 * X[0] - 1.0);
        float xy_cxx = (float)(-0.5 * dxy * X[0] * X[0] + (double)(a2 * X[0]));
        float yy_cxx = (float)(-0.5 * dyy * X[0] * X[0]);
        float xx_cxy = (float)((double)(-dxx * X[0] * X[1]) + 2.0 * a1 * X[1]);
        float xy_cxy = FMA(a1, X[0], SUM2(-dxy * X[0], X[1], a2, X[1])) - 1.0f;
        float yy_cxy = (float)((double)(-dyy * X[0] * X[1]) + 2.0 * a2 * X[0]);
        float xx_cyy = (float)(-0.5 * dxx * X[1] * X[1]);
        float xy_cyy = (float)(-0.5 * dxy * X[1] * X[1] + (double)(a1 * X[1]));
        float yy_cyy = (float)(-0.5 * dyy * X[1] * X[1] + 2.0 * a2 * X[1] - 1.0);
        ACC(gc[0], FMA(yy_cxx, Gyy, SUM2(xx_cxx, Gxx, xy_cxx, S)) * G);
        ACC(gc[1], FMA(yy_cxy, Gyy, SUM2(xx_cxy, Gxx, xy_cxy, S)) * G);
        ACC(gc[2], FMA(yy_cyy, Gyy, SUM2(xx_cyy, Gxx, xy_cyy, S)) * G);
        return;
    }
    /* third, D == 2 (backward.cu:329-415) */
    float dxxx = (float)(3.0 * c[0] * a1 - (double)(a1 * a1 * a1));
    float dxxy = (float)(2.0 * c[1] * a1 - (double)(a1 * a1 * a2) + (double)(c[0] * a2));
    float dxyy = (float)(2.0 * c[1] * a2 - (double)(a1 * a2 * a2) + (double)(c[2] * a1));
    float dyyy = (float)(3.0 * c[2] * a2 - (double)(a2 * a2 * a2));
    float Gk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int ch = 0; ch < C; ++ch) {
        const float *d = dL + ch;
        float g = SUM2(dxxx, d[0], dxxy, d[C]);
        g = FMA(dxxy, d[2 * C], g);
        g = FMA(dxyy, d[3 * C], g);
        g = FMA(dxxy, d[4 * C], g);
        g = FMA(dxyy, d[5 * C], g);
        g = FMA(dxyy, d[6 * C], g);
        g = FMA(dyyy, d[7 * C], g);
        ACC(gv[ch], g * G);
        for (int k = 0; k < 8; ++k) Gk[k] = FMA(v[ch], d[k * C], Gk[k]);
    }
    float S1 = Gk[1] + Gk[2] + Gk[4], S2 = Gk[3] + Gk[5] + Gk[6];
    float xxy_dx = (float)(2.0 * a1 * a2 * c[0] + (double)(a1 * a1 * c[1]) - 3.0 * c[0] * c[1]);
    float xyy_dx = (float)(2.0 * a1 * a2 * c[1] + (double)(a2 * a2 * c[0]) - (double)(c[2] * c[0]) - 2.0 * c[1] * c[1]);
    /* left-to-right sum in double: each float term is promoted on its own */
    float dLdx = (float)((((double)(dxxx * a1) - 3.0 * c[0] * c[0] + 3.0 * a1 * a1 * c[0]) * Gk[0]
                          + (double)(FMA(dxxy, a1, xxy_dx) * Gk[1]) + (double)(FMA(dxxy, a1, xxy_dx) * Gk[2])
                          + (double)(FMA(dxyy, a1, xyy_dx) * Gk[3]) + (double)(FMA(dxxy, a1, xxy_dx) * Gk[4])
                          + (double)(FMA(dxyy, a1, xyy_dx) * Gk[5]) + (double)(FMA(dxyy, a1, xyy_dx) * Gk[6])
                          + ((double)(dyyy * a1) - 3.0 * c[2] * c[1] + 3.0 * a2 * a2 * c[1]) * Gk[7]) * G);
    float xxy_dy = (float)(2.0 * a1 * a2 * c[1] + (double)(a1 * a1 * c[2]) - (double)(c[0] * c[2]) - 2.0 * c[1] * c[1]);
    float xyy_dy = (float)(2.0 * a1 * a2 * c[2] + (double)(a2 * a2 * c[1]) - 3.0 * c[2] * c[1]);
    float dLdy = (float)((((double)(dxxx * a2) - 3.0 * c[0] * c[1] + 3.0 * a1 * a1 * c[1]) * Gk[0]
                          + (double)(FMA(dxxy, a2, xxy_dy) * Gk[1]) + (double)(FMA(dxxy, a2, xxy_dy) * Gk[2])
                          + (double)(FMA(dxyy, a2, xyy_dy) * Gk[3]) + (double)(FMA(dxxy, a2, xxy_dy) * Gk[4])
                          + (double)(FMA(dxyy, a2, xyy_dy) * Gk[5]) + (double)(FMA(dxyy, a2, xyy_dy) * Gk[6])
                          + ((double)(dyyy * a2) - 3.0 * c[2] * c[2] + 3.0 * a2 * a2 * c[2]) * Gk[7]) * G);
    ACC(gm[0], -dLdx);
    ACC(gm[1], -dLdy);
    float X0 = X[0], X1 = X[1];
    float v_cxx[4], v_cxy[4], v_cyy[4];
    v_cxx[0] = (float)(-0.5 * dxxx * X0 * X0 + 3.0 * c[0] * X0 + 3.0 * a1 - 3.0 * a1 * a1 * X0);
    v_cxx[1] = (float)(-0.5 * dxxy * X0 * X0 + 2.0 * c[1] * X0 - 2.0 * a1 * a2 * X0 + a2);
    v_cxx[2] = (float)(-0.5 * dxyy * X0 * X0 - (double)(a2 * a2 * X0) + (double)(c[2] * X0));
    v_cxx[3] = (float)(-0.5 * dyyy * X0 * X0);
    v_cxy[0] = (float)((double)(-dxxx * X0 * X1) + 3.0 * c[0] * X1 - 3.0 * a1 * a1 * X1);
    v_cxy[1] = (float)((double)(-dxxy * X0 * X1) + 2.0 * c[1] * X1 + 2.0 * a1 - 2.0 * a1 * a2 * X1 - (double)(a1 * a1 * X0) + (double)(c[0] * X0));
    v_cxy[2] = (float)((double)(-dxyy * X0 * X1) + 2.0 * c[1] * X0 + 2.0 * a2 - (double)(a2 * a2 * X1) - 2.0 * a1 * a2 * X0 + (double)(c[2] * X1));
    v_cxy[3] = (float)((double)(-dyyy * X0 * X1) + 3.0 * c[2] * X0 - 3.0 * a2 * a2 * X0);
    v_cyy[0] = (float)(-0.5 * dxxx * X1 * X1);
    v_cyy[1] = (float)(-0.5 * dxxy * X1 * X1 - (double)(a1 * a1 * X1) + (double)(c[0] * X1));
    v_cyy[2] = (float)(-0.5 * dxyy * X1 * X1 + 2.0 * c[1] * X1 - 2.0 * a1 * a2 * X1 + a1);
    v_cyy[3] = (float)(-0.5 * dyyy * X1 * X1 + 3.0 * c[2] * X1 + 3.0 * a2 - 3.0 * a2 * a2 * X1);
    ACC(gc[0], FMA(v_cxx[3], Gk[7], FMA(v_cxx[2], S2, SUM2(v_cxx[0], Gk[0], v_cxx[1], S1))) * G);
    ACC(gc[1], FMA(v_cxy[3], Gk[7], FMA(v_cxy[2], S2, SUM2(v_cxy[0], Gk[0], v_cxy[1], S1))) * G);
    ACC(gc[2], FMA(v_cyy[3], Gk[7], FMA(v_cyy[2], S2, SUM2(v_cyy[0], Gk[0], v_cyy[1], S1))) * G);
}
#undef ACC
