/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * Never linked into the product library.
 *
 * CPU restatement of the reference codebook search:
 *   torch.argmin(torch.cdist(flat, embed, compute_mode='donot_use_mm_for_euclid_dist'), dim=1)
 *   (reference vqvae/layers.py:700-702), followed by the gather embed[idx] (layers.py:703),
 *   the straight-through value inputs + (q - inputs) (layers.py:720) and the squared
 *   error behind mse_loss(q, inputs) (layers.py:716).
 *
 * Exact arithmetic of torch's CPU cdist kernel (pinned bitwise by SURVEY.md §0.3 /
 * Appendix B and by tests/golden/vq_kat.npz "dist" arrays):
 *   acc = 0; B = 4*floor(D/4)
 *   d in [0,B):  t = x-e; acc = fl(acc + fl(t*t))       (no FMA, in order)
 *   d in [B,D):  t = x-e; acc = fmaf(t, t, acc)          (FMA tail)
 *   dist = sqrtf(acc); idx = first k with minimal dist    (strict <)
 * Built with -ffp-contract=off so the compiler cannot fuse the first loop.
 */
#include <math.h>
#include <stdint.h>

static float row_dist(const float *x, const float *e, int d) {
    const int b = 4 * (d / 4);
    float acc = 0.0f;
    for (int i = 0; i < b; ++i) {
        const float t = x[i] - e[i];
        const float p = t * t;
        acc = acc + p;
    }
    for (int i = b; i < d; ++i) {
        const float t = x[i] - e[i];
        acc = fmaf(t, t, acc);
    }
    return sqrtf(acc);
}

/* dist may be NULL; otherwise n*k floats. */
void vq_oracle_cdist(const float *z, int64_t n, int d, const float *e, int k, float *dist) {
    for (int64_t r = 0; r < n; ++r)
        for (int c = 0; c < k; ++c)
            dist[r * k + c] = row_dist(z + r * d, e + (int64_t)c * d, d);
}

/*
 * idx[n]; zst[n*d] = fl(x + fl(q - x)) (may be NULL); returns sum over rows of (q-x)^2
 * accumulated in double (the reference's mean reduction order is ATen-internal: tolerance).
 */
double vq_oracle_nearest(const float *z, int64_t n, int d, const float *e, int k,
                         int64_t *idx, float *zst) {
    double sq = 0.0;
    for (int64_t r = 0; r < n; ++r) {
        const float *x = z + r * d;
        float best = INFINITY;
        int bi = 0;
        for (int c = 0; c < k; ++c) {
            const float dv = row_dist(x, e + (int64_t)c * d, d);
            if (dv < best) { best = dv; bi = c; }
        }
        /* NaN rows: torch.argmin returns the NaN's index; keep 0 like an all-NaN row */
        idx[r] = bi;
        const float *q = e + (int64_t)bi * d;
        for (int i = 0; i < d; ++i) {
            const float diff = q[i] - x[i];
            if (zst) zst[r * d + i] = x[i] + diff;
            sq += (double)diff * (double)diff;
        }
    }
    return sq;
}
