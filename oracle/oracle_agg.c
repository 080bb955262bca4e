/*
 * oracle_agg.c -- CPU restatement of the reference's neighbour aggregation
 * (aggregate_neighbors.cu, kr4b/diff-gaussian-sampling).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.c): used by tests/ as the checker of the HIP path.
 * PARITY STATUS: "parity unpinned" -- the reference is CUDA-only and ships no fixtures; this
 * restatement is pinned by torch autograd of its forward (tests/test_oracle_agg.py) and by
 * hand-checked predicate cases (asymmetric torus wrap, radius skip, power > 0 slots).
 *
 * FLOAT = float as in the reference (config.h:20); double where its double literals promote
 * (`radii * 0.2`, `1.0 / (r + 1e-6)`, `-0.5 * ...`, `fmod(x, 2.0)`, `frequencies * M_PI * X`,
 * `sin`/`cos` of that double).  Atomic float accumulations of the reference are serial here.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle_fmad.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* findCollisions, aggregate_neighbors.cu:18-50: is j a neighbour of i? */
static int agg_collides(int D, const float *means, const float *radii, int i, int j) {
    const float my_radius = (float)((double)radii[i] * 0.2);
    if ((double)my_radius < 1e-6) return 0;
    const float other_radius = (float)((double)radii[j] * 0.2);
    if ((double)other_radius < 1e-6) return 0;
    float dist = 0.0f;
    for (int d = 0; d < D; ++d) {
        float dx = means[(int64_t)j * D + d] - means[(int64_t)i * D + d];
        /* TORUS: min(dx, abs(2.0 - fmod(abs(dx), 2.0))) -- only a positive dx can shrink */
        const double w = fabs(2.0 - fmod((double)fabsf(dx), 2.0));
        dx = (float)fmin((double)dx, w);
        dist = FMA(dx, dx, dist); /* aggregate_neighbors.cu:44: contracted under --fmad=true */
    }
    const float radius = my_radius + other_radius;
    return !(dist > radius * radius);
}

/* Pass 1: neighbour counts per row (the reference's bool_indices.sum(-1)). */
void orc_agg_counts(int P, int D, const float *means, const float *radii, int64_t *counts) {
    for (int i = 0; i < P; ++i) {
        int64_t n = 0;
        for (int j = 0; j < P; ++j) n += agg_collides(D, means, radii, i, j);
        counts[i] = n;
    }
}

/* The same for the rows rows[0..nrows) only (a bounded check of a large problem). */
void orc_agg_counts_rows(int P, int D, const float *means, const float *radii, int nrows,
                         const int32_t *rows, int64_t *counts) {
    for (int r = 0; r < nrows; ++r) {
        int64_t n = 0;
        for (int j = 0; j < P; ++j) n += agg_collides(D, means, radii, rows[r], j);
        counts[r] = n;
    }
}

/* Pass 2: preprocess, aggregate_neighbors.cu:52-127.  ranges = inclusive cumsum of counts;
 * indices pre-filled with -1, dists / densities with 0 (the host glue at 336-341). */
static void agg_fill_row(int P, int D, const float *means, const float *conics,
                         const float *radii, int i, int64_t start, int64_t *indices, float *dists,
                         float *densities, float *inv_total_i) {
    const int S = D * (D + 1) / 2;
    {
        const float my_radius = (float)((double)radii[i] * 0.333);
        const float my_inv_radius = (float)(1.0 / ((double)my_radius + 1e-6));
        float total = 0.0f;
        int64_t current = -1;
        for (int j = 0; j < P; ++j) {
            if (!agg_collides(D, means, radii, i, j)) continue;
            current += 1;
            const float *con = conics + (int64_t)j * S;
            float *X = dists + (start + current) * D;
            for (int d = 0; d < D; ++d) {
                X[d] = means[(int64_t)j * D + d] - means[(int64_t)i * D + d];
                if (fabsf(X[d]) > 1.0f) {
                    if (X[d] >= 0) X[d] = (float)(fmod((double)X[d], 2.0) - 2.0);
                    else X[d] = (float)(fmod((double)X[d], 2.0) + 2.0);
                }
            }
            float power;
            if (D == 1) {
                power = (float)(-0.5 * con[0] * X[0] * X[0]);
            } else {
                power = (float)(-0.5 * (double)SUM2(con[0] * X[0], X[0], con[2] * X[1], X[1])
                                - (double)(con[1] * X[0] * X[1]));
            }
            for (int d = 0; d < D; ++d) X[d] *= my_inv_radius;
            if (power > 0) continue;
            densities[start + current] = expf(power);
            indices[start + current] = j;
            total += densities[start + current];
        }
        *inv_total_i = (float)(1.0 / ((double)total + 1e-6));
    }
}

void orc_agg_fill(int P, int D, const float *means, const float *conics, const float *radii,
                  const int64_t *ranges, int64_t *indices, float *dists, float *densities,
                  float *inv_total) {
    for (int i = 0; i < P; ++i)
        agg_fill_row(P, D, means, conics, radii, i, i == 0 ? 0 : ranges[i - 1], indices, dists,
                     densities, inv_total + i);
}

/* Rows rows[0..nrows) only, into compact lists: row r's slots start at ranges[r - 1]
 * (ranges = inclusive cumsum of orc_agg_counts_rows). */
void orc_agg_fill_rows(int P, int D, const float *means, const float *conics, const float *radii,
                       int nrows, const int32_t *rows, const int64_t *ranges, int64_t *indices,
                       float *dists, float *densities, float *inv_total) {
    for (int r = 0; r < nrows; ++r)
        agg_fill_row(P, D, means, conics, radii, rows[r], r == 0 ? 0 : ranges[r - 1], indices,
                     dists, densities, inv_total + r);
}

#define AGG_T float
#define AGG_FN(n) n
#define AGG_MUL(a, b) ((a) * (b))
#define AGG_MUL3(a, b, c) ((a) * (b) * (c))
#include "oracle_agg_body.h"
#undef AGG_T
#undef AGG_FN
#undef AGG_MUL
#undef AGG_MUL3

/* Exact-accumulation twins (orc_agg_forward64 / orc_agg_backward64): double outputs. */
#define AGG_T double
#define AGG_FN(n) n##64
#define AGG_MUL(a, b) ((double)(a) * (double)(b))
#define AGG_MUL3(a, b, c) ((double)(a) * (double)(b) * (double)(c))
#include "oracle_agg_body.h"
