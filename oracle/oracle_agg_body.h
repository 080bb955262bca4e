/*
 * oracle_agg_body.h -- the aggregate forward / backward of oracle_agg.c, instantiated twice:
 *   AGG_T = float : the reference's literal float accumulation (aggregate_neighbors.cu order);
 *   AGG_T = double: the same per-slot float quantities (weights, embeddings, factors, dw, ...),
 *                   with every accumulated product and sum exact to double -- the value the
 *                   reference's formula has before its own float summation rounds it.
 * TEST INFRASTRUCTURE ONLY (see oracle.c).
 */
/* aggregateNeighbors, aggregate_neighbors.cu:129-208.  E = distance_transform.size / 2. */
void AGG_FN(orc_agg_forward)(int P, int D, int L, int K, int E, const float *features,
                     const float *transform, const float *queries, const float *keys,
                     const float *frequencies, const float *dt, const int64_t *indices,
                     const int64_t *ranges, const float *dists, const float *densities,
                     const float *inv_total, float *weights, float *embeddings, float *factors,
                     AGG_T *out) {
    const int F = (E - 1) / D / 2, stride = (E - 1) / D;
    for (int i = 0; i < P; ++i) {
        const float *q = queries + (int64_t)i * K;
        const int64_t start = i == 0 ? 0 : ranges[i - 1], end = ranges[i];
        AGG_T *o = out + (int64_t)i * L;
        for (int64_t s = start; s < end; ++s) {
            const int64_t idx = indices[s];
            if (idx == -1) continue;
            const float *feat = features + idx * L, *key = keys + idx * K, *X = dists + s * D;
            float weight = 0.0f;
            for (int k = 0; k < K; ++k) weight += q[k] * key[k];
            weights[s] = weight;
            float emb = 0.0f, fac = 0.0f;
            for (int d = 0; d < D; ++d)
                for (int e = 0; e < F; ++e) {
                    const float sn = (float)sin((double)frequencies[e] * M_PI * (double)X[d]);
                    const float cs = (float)cos((double)frequencies[e] * M_PI * (double)X[d]);
                    emb += dt[d * stride + e * 2 + 0] * sn;
                    emb += dt[d * stride + e * 2 + 1] * cs;
                    fac += dt[E + d * stride + e * 2 + 0] * sn;
                    fac += dt[E + d * stride + e * 2 + 1] * cs;
                }
            emb += dt[E - 1];
            fac += dt[2 * E - 1];
            embeddings[s] = emb;
            factors[s] = fac;
            const float dw = inv_total[i] * densities[s] * weight;
            const float dwf = dw * fac, dwe = dw * emb;
            for (int j = 0; j < L; ++j) {
                const float embedded = dwe + dwf * feat[j];
                for (int k = 0; k < L; ++k) o[k] += AGG_MUL(transform[j * L + k], embedded);
            }
        }
    }
}

/* aggregateNeighborsBackward, aggregate_neighbors.cu:210-321 (atomics in serial order). */
void AGG_FN(orc_agg_backward)(int P, int D, int L, int K, int E, const float *features,
                      const float *transform, const float *queries, const float *keys,
                      const float *frequencies, const float *dt, const int64_t *indices,
                      const int64_t *ranges, const float *dists, const float *densities,
                      const float *weights, const float *embeddings, const float *factors,
                      const float *inv_total, const float *dL, AGG_T *dfeat, AGG_T *dtrans,
                      AGG_T *dq, AGG_T *dkeys, AGG_T *dfreq, AGG_T *ddt) {
    const int F = (E - 1) / D / 2, stride = (E - 1) / D;
    float st[1024];
    for (int i = 0; i < P; ++i) {
        const float *q = queries + (int64_t)i * K, *g = dL + (int64_t)i * L;
        const int64_t start = i == 0 ? 0 : ranges[i - 1], end = ranges[i];
        for (int j = 0; j < L; ++j) {
            st[j] = 0.0f;
            for (int k = 0; k < L; ++k) st[j] += transform[j * L + k] * g[k];
        }
        for (int64_t s = start; s < end; ++s) {
            const int64_t idx = indices[s];
            if (idx == -1) continue;
            const float *feat = features + idx * L, *key = keys + idx * K, *X = dists + s * D;
            const float dc = densities[s] * inv_total[i];
            const float dcw = dc * weights[s];
            for (int d = 0; d < D; ++d)
                for (int e = 0; e < F; ++e) {
                    const float sn = (float)sin((double)frequencies[e] * M_PI * (double)X[d]);
                    const float cs = (float)cos((double)frequencies[e] * M_PI * (double)X[d]);
                    const int a = d * stride + e * 2;
                    for (int j = 0; j < L; ++j) {
                        const float dct = dcw * st[j];
                        ddt[a + 0] += AGG_MUL(dct, sn);
                        ddt[E + a + 0] += AGG_MUL3(dct, sn, feat[j]);
                        dfreq[e] += (AGG_T)((double)cs * M_PI * (double)X[d] * (double)dct *
                                            (double)(dt[a + 0] + dt[E + a + 0] * feat[j]));
                        ddt[a + 1] += AGG_MUL(dct, cs);
                        ddt[E + a + 1] += AGG_MUL3(dct, cs, feat[j]);
                        dfreq[e] += (AGG_T)((double)-sn * M_PI * (double)X[d] * (double)dct *
                                            (double)(dt[a + 1] + dt[E + a + 1] * feat[j]));
                    }
                }
            const float dce = dc * embeddings[s], dcf = dc * factors[s];
            for (int j = 0; j < L; ++j) {
                const float dct = dcw * st[j];
                ddt[E - 1] += dct;
                ddt[2 * E - 1] += AGG_MUL(dct, feat[j]);
                dfeat[idx * L + j] += AGG_MUL(dct, factors[s]);
                const float embedded = dce + dcf * feat[j];
                const float we = weights[s] * embedded;
                for (int k = 0; k < L; ++k) dtrans[j * L + k] += AGG_MUL(we, g[k]);
                const float te = st[j] * embedded;
                for (int k = 0; k < K; ++k) {
                    dq[(int64_t)i * K + k] += AGG_MUL(key[k], te);
                    dkeys[idx * K + k] += AGG_MUL(q[k], te);
                }
            }
        }
    }
}
