/* CPU ORACLE in C — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).
 *
 * A plain C restatement of the reference hot path, used (a) as a fast checker
 * at sizes where the numpy/Python oracle is too slow and (b) as the timed CPU
 * baseline in bench.py.  Never linked into the product library.
 *
 * Built with -ffp-contract=off so every a*b+c rounds twice, like the
 * reference's NumPy / Python float arithmetic.  pow() is glibc's, the same
 * routine Python's float ** calls in the reference.
 *
 *   oracle_gae        agilerl/components/rollout_buffer.py:413-481
 *   oracle_per_*      agilerl/components/segment_tree.py:81-156,
 *                     agilerl/components/replay_buffer.py:311-428
 *   oracle_ppo_loss   agilerl/algorithms/ppo.py:868-902 (+ torch autograd rules)
 *   oracle_c51        agilerl/algorithms/dqn_rainbow.py:313-367
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* GAE / MC over P independent (T, N) time-major blocks. */
void oracle_gae(const float *r, const uint8_t *done, const float *v, const float *last_v,
                const uint8_t *last_done, int64_t P, int64_t T, int64_t N, double gamma,
                double lam, int use_gae, float *adv, float *ret, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t col = 0; col < P * N; ++col) {
        const int64_t p = col / N, n = col % N;
        const int64_t base = p * T * N + n;
        const float g32 = (float)gamma;
        const double gl = gamma * lam;
        if (use_gae) {
            double c = 0.0;
            for (int64_t t = T - 1; t >= 0; --t) {
                double nnt, gv;
                if (t == T - 1) {
                    nnt = 1.0 - (double)last_done[col];
                    gv = gamma * (double)last_v[col];
                } else {
                    nnt = 1.0 - (double)done[base + (t + 1) * N];
                    gv = (double)(g32 * v[base + (t + 1) * N]);
                }
                const double delta = ((double)r[base + t * N] + gv * nnt) - (double)v[base + t * N];
                c = delta + (gl * nnt) * c;
                const float a = (float)c;
                adv[base + t * N] = a;
                ret[base + t * N] = a + v[base + t * N];
            }
        } else {
            double c = (double)last_v[col] * (1.0 - (double)last_done[col]);
            for (int64_t t = T - 1; t >= 0; --t) {
                c = (double)r[base + t * N] + (gamma * c) * (1.0 - (double)done[base + t * N]);
                const float rt = (float)c;
                ret[base + t * N] = rt;
                adv[base + t * N] = rt - v[base + t * N];
            }
        }
    }
}

/* ---- segment trees (1-indexed heaps of 2*cap doubles) ------------------- */
static void set_leaf(double *sum, double *mn, int64_t cap, int64_t idx, double val) {
    int64_t k = idx + cap;
    sum[k] = val;
    mn[k] = val;
    k >>= 1;
    while (k >= 1) {
        sum[k] = sum[2 * k] + sum[2 * k + 1];
        const double a = mn[2 * k], b = mn[2 * k + 1];
        mn[k] = (b < a) ? b : a; /* Python min(a, b): returns a unless b < a */
        k >>= 1;
    }
}

/* update_priorities: in order, floor 1e-5, leaf = p**alpha; returns new max. */
double oracle_per_update(double *sum, double *mn, int64_t cap, const int64_t *idx,
                         const float *pri, int64_t n, double alpha, double max_priority) {
    for (int64_t i = 0; i < n; ++i) {
        double p = (double)pri[i];
        if (p < 1e-5) p = 1e-5;
        set_leaf(sum, mn, cap, idx[i], pow(p, alpha));
        if (p > max_priority) max_priority = p;
    }
    return max_priority;
}

/* add: n inserts at max priority starting at *tree_ptr (ring of max_size). */
void oracle_per_add(double *sum, double *mn, int64_t cap, int64_t max_size, int64_t *tree_ptr,
                    int64_t n, double alpha, double max_priority) {
    const double pa = pow(max_priority, alpha);
    for (int64_t i = 0; i < n; ++i) {
        set_leaf(sum, mn, cap, *tree_ptr, pa);
        *tree_ptr = (*tree_ptr + 1) % max_size;
    }
}

/* proportional sampling; returns number of assert violations (ub > sum+1e-5). */
int64_t oracle_per_sample(const double *sum, int64_t cap, const float *u, int64_t B, int64_t *out) {
    const double total = sum[1];
    const double segment = total / (double)B;
    int64_t bad = 0;
    for (int64_t i = 0; i < B; ++i) {
        const double a = segment * (double)i;
        const double b = segment * (double)(i + 1);
        double ub = (double)u[i] * (b - a) + a;
        if (!(ub >= 0.0 && ub <= total + 1e-5)) ++bad;
        int64_t k = 1;
        while (k < cap) {
            const double left = sum[2 * k];
            if (left > ub) {
                k = 2 * k;
            } else {
                ub -= left;
                k = 2 * k + 1;
            }
        }
        out[i] = k - cap;
    }
    return bad;
}

void oracle_per_weights(const double *sum, const double *mn, int64_t cap, const int64_t *idx,
                        int64_t B, int64_t size, double beta, float *w) {
    const double p_min = mn[1] / sum[1];
    const double max_w = pow(p_min * (double)size, -beta);
    for (int64_t i = 0; i < B; ++i) {
        const double ps = sum[cap + idx[i]] / sum[1];
        const double wt = pow(ps * (double)size, -beta);
        w[i] = (float)(wt / max_w);
    }
}

/* ---- PPO clipped loss fwd+bwd over nmb contiguous minibatches of b ------ */
void oracle_ppo_loss(const float *logp, const float *old_logp, const float *adv, const float *ret,
                     const float *old_v, const float *v, const float *H, int64_t b, int64_t nmb,
                     double clip, double vf, double ent, float *g_logp, float *g_v, float *g_H,
                     double *loss_out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t m = 0; m < nmb; ++m) {
        double pg = 0, vl = 0, es = 0;
        const double lo = 1.0 - clip, hi = 1.0 + clip, inv_b = 1.0 / (double)b;
        for (int64_t j = m * b; j < (m + 1) * b; ++j) {
            const double ratio = exp((double)logp[j] - (double)old_logp[j]);
            const double A = adv[j];
            const double rc = ratio < lo ? lo : (ratio > hi ? hi : ratio);
            const double p1 = -A * ratio, p2 = -A * rc;
            pg += p1 > p2 ? p1 : p2;
            const double g1 = p1 > p2 ? 1.0 : (p1 == p2 ? 0.5 : 0.0);
            const double g2 = p2 > p1 ? 1.0 : (p1 == p2 ? 0.5 : 0.0);
            const double inr = (ratio >= lo && ratio <= hi) ? 1.0 : 0.0;
            g_logp[j] = (float)((g1 * -A + g2 * -A * inr) * inv_b * ratio);
            const double dv = (double)v[j] - (double)old_v[j];
            const double dvc = dv < -clip ? -clip : (dv > clip ? clip : dv);
            const double vc = (double)old_v[j] + dvc;
            const double eu = (double)v[j] - (double)ret[j], ec = vc - (double)ret[j];
            const double lu = eu * eu, lc = ec * ec;
            vl += lu > lc ? lu : lc;
            const double gu = lu > lc ? 1.0 : (lu == lc ? 0.5 : 0.0);
            const double gc = lc > lu ? 1.0 : (lu == lc ? 0.5 : 0.0);
            const double inv = (dv >= -clip && dv <= clip) ? 1.0 : 0.0;
            g_v[j] = (float)(vf * 0.5 * inv_b * (gu * 2.0 * eu + gc * 2.0 * ec * inv));
            g_H[j] = (float)(-ent * inv_b);
            es += H[j];
        }
        loss_out[m] = pg * inv_b + vf * 0.5 * vl * inv_b - ent * es * inv_b;
    }
}

/* ---- C51 projection + loss, one row at a time --------------------------- */
void oracle_c51(const float *q_next, const float *tdist, const float *logp_cur, const int64_t *act,
                const float *r, const float *d, const float *support, int64_t B, int64_t A,
                int64_t Z, double vmin, double vmax, double gamma, float *proj, float *loss) {
    const float dz = (float)((vmax - vmin) / (double)(Z - 1));
    const float fvmin = (float)vmin, fvmax = (float)vmax, g = (float)gamma;
    for (int64_t i = 0; i < B; ++i) {
        int64_t as = 0;
        float best = q_next[i * A];
        for (int64_t a = 1; a < A; ++a)
            if (q_next[i * A + a] > best) { best = q_next[i * A + a]; as = a; }
        const float *p = tdist + (i * A + as) * Z;
        float *row = proj + i * Z;
        for (int64_t z = 0; z < Z; ++z) row[z] = 0.0f;
        const float k = (1.0f - d[i]) * g;
        int64_t Ls[1024], Us[1024];
        float bs[1024];
        for (int64_t z = 0; z < Z; ++z) {
            float tz = r[i] + k * support[z];
            tz = tz < fvmin ? fvmin : (tz > fvmax ? fvmax : tz);
            const float b = (tz - fvmin) / dz;
            int64_t L = (int64_t)floorf(b), U = (int64_t)ceilf(b);
            if (U > 0 && U == L) L -= 1;
            if (Z - 1 > L && U == L) U += 1;
            Ls[z] = L; Us[z] = U; bs[z] = b;
        }
        for (int64_t z = 0; z < Z; ++z) row[Ls[z]] += p[z] * ((float)Us[z] - bs[z]);
        for (int64_t z = 0; z < Z; ++z) row[Us[z]] += p[z] * (bs[z] - (float)Ls[z]);
        double s = 0.0;
        const float *lp = logp_cur + (i * A + act[i]) * Z;
        for (int64_t z = 0; z < Z; ++z) s += (double)row[z] * (double)lp[z];
        loss[i] = (float)(-s);
    }
}

/* libm pow, element-wise: what the reference's Python ``float ** float``
 * calls (replay_buffer.py:322 leaves, :399-406 IS weights).  The checker of
 * the device restatement of glibc's pow (agilerl_amd/csrc/libm_pow.h). */
void oracle_pow(const double *x, const double *y, double *out, int64_t n) {
    for (int64_t i = 0; i < n; ++i) out[i] = pow(x[i], y[i]);
}
