/* ccd_oracle.c -- sequential C restatement of lcmap-pyccd ccd.detect (TEST INFRASTRUCTURE ONLY).
 *
 * ORACLE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load the
 * library built from this file (oracle/libccdoracle.so), and only as the checker or as the
 * timed CPU baseline.  The product (lcmap-firebird_amd/) never links or calls it.
 *
 * It restates, module for module, the same pyccd algorithm as oracle/ccd_ref.py (see that
 * file's header for provenance: reference call site ccdc/pyccd.py:168, pinned dependency
 * lcmap-pyccd 2018.03.12.dev-ncompare.b2 from setup.py:32 / requirements-dev.txt:1, which is
 * absent here), but independently of the GPU kernels' formulation:
 *   * Lasso = scikit-learn 0.18 cd_fast.enet_coordinate_descent, residual-update form (the GPU
 *     uses the equivalent Gram form), on the centred n x 7 design of models/lasso.py;
 *   * robust_fit.RLM least squares = min-norm lstsq via one-sided Jacobi SVD (numpy uses LAPACK
 *     gelsd; the GPU uses 5x5 normal equations);
 *   * medians / argsorts = full sorts (the GPU uses counting selection).
 * Parity status: pinned against ccd_ref.py golden vectors (tests/golden) which are themselves
 * pinned only by the reference's boundary tests -- see DESIGN.md "Oracle".
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ccdgpu.h"

#define NB 7

typedef struct {
    double coef[7];
    double intercept;
    double rmse;
    double *resid; /* length n (owned by caller scratch) */
    int n;
    int sweeps;
} fit_t;

typedef struct {
    int64_t *v;
    int n, cap;
} segvec_t;

typedef struct {
    const ccdgpu_params *p;
    int n;               /* sorted observations */
    const int64_t *t;    /* sorted dates */
    const double *basis; /* [n][6] cos/sin of w*t, 2wt, 3wt (coefficient_matrix) */
    int16_t *obs;        /* [7][n] sorted, thermal converted */
    uint8_t *mask;       /* [n] processing mask */
    int *idx;            /* compacted indices (period) */
    int m;
    int peek;
    int overflow; /* adaptive peek exceeded CCDGPU_MAX_PEEK */
    double chg_thr;
    double vario[NB];
    /* scratch */
    double *X, *Xc, *yc, *R, *y;
    double *resid_store; /* [7][n] residuals of the current models over their fit window */
    fit_t models[NB];
    /* output */
    ccdgpu_segment *segs;
    int nseg, segcap;
    int64_t fits, sweeps;
    int32_t qs_deep; /* argsort parts past numpy 1.17's introsort depth limit (ccdoracle_np_argsort) */
} pix_t;

/* ------------------------------------------------------------------ small helpers */
static int cmp_double(const void *a, const void *b) {
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static double median_sorted(const double *s, int n) {
    if (n <= 0) return NAN;
    if (n & 1) return s[n / 2];
    return (s[n / 2 - 1] + s[n / 2]) / 2.0;
}

static double median_inplace(double *v, int n) {
    qsort(v, (size_t)n, sizeof(double), cmp_double);
    return median_sorted(v, n);
}

static inline double period(const pix_t *P, int i) { return (double)P->t[P->idx[i]]; }
static inline int64_t period_i(const pix_t *P, int i) { return P->t[P->idx[i]]; }
static inline double spec(const pix_t *P, int b, int i) { return (double)P->obs[(size_t)b * P->n + P->idx[i]]; }

static void mask_remove(pix_t *P, int j) { /* change.update_processing_mask(mask, j) */
    P->mask[P->idx[j]] = 0;
    memmove(P->idx + j, P->idx + j + 1, sizeof(int) * (size_t)(P->m - j - 1));
    P->m -= 1;
}

/* chi-square(5) cdf and its inverse by bisection (scipy chi2.ppf stand-in for ncompare). */
static double chi2_5_cdf(double x) {
    if (x <= 0) return 0.0;
    return erf(sqrt(x / 2.0)) - sqrt(2.0 * x / M_PI) * exp(-x / 2.0) * (1.0 + x / 3.0);
}
static double chi2_5_ppf(double p) {
    double lo = 0.0, hi = 400.0;
    for (int i = 0; i < 200; ++i) {
        double mid = 0.5 * (lo + hi);
        if (chi2_5_cdf(mid) < p) lo = mid; else hi = mid;
    }
    return 0.5 * (lo + hi);
}

/* ------------------------------------------------------------------ numpy argsort (quicksort) */
/* np.argsort(v) with numpy's default kind='quicksort' as the pinned reference image runs it:
 * lcmap-pyccd's detect (ccd/__init__.py: argsort of the dates) and change.find_closest_doy
 * (argsort of the day-of-year distances) call it, and their tie order decides which of equal
 * dates is kept (mask_duplicate_values keeps the first) and which of equally close observations
 * enter the comparison rmse.  The Dockerfile:4 conda image (Python 3.6, scikit-learn 0.18) carries
 * a numpy < 1.17, whose aquicksort_<type> (numpy/core/src/npysort/quicksort.c.src) is restated
 * here: median-of-3 pivot swapped to pr - 1, Sedgewick's partition (both scans stop on keys equal
 * to the pivot), the larger part pushed, the smaller continued, insertion sort of parts of at
 * most 16 (SMALL_QUICKSORT 15).  numpy 1.17 added a heapsort fallback for a part popped more than
 * 2 floor(log2 n) partitions deep (introsort); *deep counts the parts that would have taken it
 * (none on any input of the suite or the tiles -- tests/test_oracle.py).  numpy >= 1.25 sorts
 * with x86-simd-sort on AVX-512 machines, another tie order.
 * v: keys; tosort: 0..n-1 on entry, the argsort on return.  num > 0: only the parts overlapping
 * positions [0, num) are sorted -- positions [0, num) end exactly as in the full sort (parts are
 * disjoint ranges, each permuted only within itself). */
#define NP_SMALL_QUICKSORT 15
#define NP_QS_STACK 128
static int np_msb(int n) {
    int d = 0;
    while (n >>= 1) d++;
    return d;
}
/* [0] closest-DOY selections over more than 24 fit observations, [1] of them with ties across
   the 24th position, [2] of those where the stable rule would take another set, [3] argsort
   parts past numpy 1.17's depth limit (summed at the end of each pixel) */
static int64_t g_qs_stats[4];
void ccdoracle_argsort_stats(int64_t *out, int32_t reset) {
    for (int i = 0; i < 4; ++i) {
        out[i] = __atomic_load_n(&g_qs_stats[i], __ATOMIC_RELAXED);
        if (reset) __atomic_store_n(&g_qs_stats[i], 0, __ATOMIC_RELAXED);
    }
}

/* numpy's pairwise summation of a contiguous float64 array (np.sum / add.reduce,
   numpy/core/src/umath/loops.c.src pairwise_sum_DOUBLE): below 8 terms in order; up to 128
   eight running sums then ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) and the remainder in
   order; above, the halves (n / 2 rounded down to a multiple of 8) summed recursively. */
double ccdoracle_np_pairwise_sum(const double *a, int32_t n) {
    if (n < 8) {
        double res = 0.;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        int i;
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int n2 = n / 2;
        n2 -= n2 % 8;
        return ccdoracle_np_pairwise_sum(a, n2) + ccdoracle_np_pairwise_sum(a + n2, n - n2);
    }
}
static double np_pairwise_sum(const double *a, int n) { return ccdoracle_np_pairwise_sum(a, n); }

void ccdoracle_np_argsort(const double *v, int32_t *tosort, int32_t n, int32_t num, int32_t *deep) {
    int32_t *pl = tosort, *pr = tosort + n - 1;
    int32_t *stack[NP_QS_STACK], **sptr = stack;
    int depth[NP_QS_STACK / 2], *psdepth = depth;
    int cdepth = np_msb(n) * 2;
    const int32_t *lim = num > 0 ? tosort + num : tosort + n;  /* parts starting here are skipped */
    if (n <= 1) return;
    for (;;) {
        if (cdepth < 0 && deep) ++*deep;
        while ((pr - pl) > NP_SMALL_QUICKSORT) {
            int32_t *pm = pl + ((pr - pl) >> 1), *pi, *pj, *pk, t;
            double vp;
            if (v[*pm] < v[*pl]) { t = *pm; *pm = *pl; *pl = t; }
            if (v[*pr] < v[*pm]) { t = *pr; *pr = *pm; *pm = t; }
            if (v[*pm] < v[*pl]) { t = *pm; *pm = *pl; *pl = t; }
            vp = v[*pm];
            pi = pl;
            pj = pr - 1;
            t = *pm; *pm = *pj; *pj = t;
            for (;;) {
                do ++pi; while (v[*pi] < vp);
                do --pj; while (vp < v[*pj]);
                if (pi >= pj) break;
                t = *pi; *pi = *pj; *pj = t;
            }
            pk = pr - 1;
            t = *pi; *pi = *pk; *pk = t;
            /* push largest partition on stack (a part starting at or past lim is dropped) */
            if (pi - pl < pr - pi) {
                if (pi + 1 < lim) { *sptr++ = pi + 1; *sptr++ = pr; *psdepth++ = cdepth - 1; }
                pr = pi - 1;
            } else {
                if (pl < lim) { *sptr++ = pl; *sptr++ = pi - 1; *psdepth++ = cdepth - 1; }
                pl = pi + 1;
            }
            --cdepth;
            if (pl >= lim) break;
        }
        if (pl < lim) {
            for (int32_t *pi = pl + 1; pi <= pr; ++pi) {  /* insertion sort */
                const int32_t vi = *pi;
                const double vv = v[vi];
                int32_t *pj = pi, *pk = pi - 1;
                while (pj > pl && vv < v[*pk]) *pj-- = *pk--;
                *pj = vi;
            }
        }
        if (sptr == stack) break;
        pr = *(--sptr);
        pl = *(--sptr);
        cdepth = *(--psdepth);
    }
}

/* ------------------------------------------------------------------ Lasso (models/lasso.py) */
/* sklearn 0.18 enet_coordinate_descent, beta = 0, cyclic, on centred X (n x p col-major). */
static int enet_cd(const double *X, const double *y, int n, int p, double alpha, int max_iter,
                   double tol, double *w, double *R) {
    double norm_cols[7];
    for (int j = 0; j < p; ++j) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += X[(size_t)j * n + i] * X[(size_t)j * n + i];
        norm_cols[j] = s;
        w[j] = 0.0;
    }
    double yy = 0;
    for (int i = 0; i < n; ++i) { R[i] = y[i]; yy += y[i] * y[i]; }
    const double d_w_tol = tol;
    tol *= yy;
    int n_iter;
    for (n_iter = 0; n_iter < max_iter; ++n_iter) {
        double w_max = 0.0, d_w_max = 0.0;
        for (int ii = 0; ii < p; ++ii) {
            if (norm_cols[ii] == 0.0) continue;
            const double *Xi = X + (size_t)ii * n;
            double w_ii = w[ii];
            if (w_ii != 0.0) for (int i = 0; i < n; ++i) R[i] += w_ii * Xi[i];
            double tmp = 0;
            for (int i = 0; i < n; ++i) tmp += Xi[i] * R[i];
            double a = fabs(tmp) - alpha;
            w[ii] = (a > 0 ? (tmp > 0 ? a : -a) : 0.0) / norm_cols[ii];
            if (w[ii] != 0.0) for (int i = 0; i < n; ++i) R[i] -= w[ii] * Xi[i];
            double d = fabs(w[ii] - w_ii);
            if (d > d_w_max) d_w_max = d;
            if (fabs(w[ii]) > w_max) w_max = fabs(w[ii]);
        }
        if (w_max == 0.0 || d_w_max / w_max < d_w_tol || n_iter == max_iter - 1) {
            double dual = 0, rr = 0, ry = 0, l1 = 0;
            for (int j = 0; j < p; ++j) {
                double s = 0;
                for (int i = 0; i < n; ++i) s += X[(size_t)j * n + i] * R[i];
                if (fabs(s) > dual) dual = fabs(s);
                l1 += fabs(w[j]);
            }
            for (int i = 0; i < n; ++i) { rr += R[i] * R[i]; ry += R[i] * y[i]; }
            double cst, gap;
            if (dual > alpha) {
                cst = alpha / dual;
                gap = 0.5 * (rr + rr * cst * cst);
            } else {
                cst = 1.0;
                gap = rr;
            }
            gap += alpha * l1 - cst * ry;
            if (gap < tol) break;
        }
    }
    return (n_iter < max_iter ? n_iter : max_iter - 1) + 1;
}

/* models/lasso.fitted_model for all 7 bands over compacted window [a, b) with k coefficients. */
static void fit_models(pix_t *P, int a, int b, int k) {
    const ccdgpu_params *p = P->p;
    const int n = b - a;
    double *X = P->X, *Xc = P->Xc;
    double xoff[7];
    for (int i = 0; i < n; ++i) {
        const double *bs = P->basis + (size_t)P->idx[a + i] * 6;
        X[0 * (size_t)n + i] = period(P, a + i);
        X[1 * (size_t)n + i] = bs[0];
        X[2 * (size_t)n + i] = bs[1];
        X[3 * (size_t)n + i] = k >= 6 ? bs[2] : 0.0;
        X[4 * (size_t)n + i] = k >= 6 ? bs[3] : 0.0;
        X[5 * (size_t)n + i] = k >= 8 ? bs[4] : 0.0;
        X[6 * (size_t)n + i] = k >= 8 ? bs[5] : 0.0;
    }
    for (int j = 0; j < 7; ++j) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += X[(size_t)j * n + i];
        xoff[j] = s / n;
        for (int i = 0; i < n; ++i) Xc[(size_t)j * n + i] = X[(size_t)j * n + i] - xoff[j];
    }
    for (int band = 0; band < NB; ++band) {
        fit_t *f = &P->models[band];
        double ys = 0;
        for (int i = 0; i < n; ++i) { P->y[i] = spec(P, band, a + i); ys += P->y[i]; }
        double yoff = ys / n;
        for (int i = 0; i < n; ++i) P->yc[i] = P->y[i] - yoff;
        f->sweeps = enet_cd(Xc, P->yc, n, 7, p->lasso_alpha * n, p->lasso_max_iter, p->lasso_tol,
                            f->coef, P->R);
        double dot = 0;
        for (int j = 0; j < 7; ++j) dot += xoff[j] * f->coef[j];
        f->intercept = yoff - dot;
        f->resid = P->resid_store + (size_t)band * P->n;
        f->n = n;
        double ss = 0;
        for (int i = 0; i < n; ++i) {
            double pr = 0;
            for (int j = 0; j < 7; ++j) pr += X[(size_t)j * n + i] * f->coef[j];
            pr += f->intercept;
            double r = P->y[i] - pr;
            f->resid[i] = r;
            ss += r * r;
        }
        f->rmse = sqrt(ss / (n - (p->rmse_dof ? k : 0)));
        P->fits += 1;
        P->sweeps += f->sweeps;
    }
}

/* lasso.predict at compacted obs i (coefficient_matrix(..., 8) @ coef + intercept) */
static double predict_at(const pix_t *P, const fit_t *f, int i) {
    const double *bs = P->basis + (size_t)P->idx[i] * 6;
    double x[7] = {period(P, i), bs[0], bs[1], bs[2], bs[3], bs[4], bs[5]};
    double s = 0;
    for (int j = 0; j < 7; ++j) s += x[j] * f->coef[j];
    return s + f->intercept;
}

/* ------------------------------------------------------------------ robust_fit.py (RLM) */
/* min-norm least squares via one-sided Jacobi SVD; also returns row leverages if h != NULL. */
static void lstsq_svd(const double *A, const double *y, int n, int p, double *x, double *h) {
    double *W = (double *)malloc(sizeof(double) * (size_t)n * p);
    double V[5][5];
    memcpy(W, A, sizeof(double) * (size_t)n * p);
    for (int i = 0; i < p; ++i)
        for (int j = 0; j < p; ++j) V[i][j] = (i == j);
    for (int sweep = 0; sweep < 60; ++sweep) {
        int rotated = 0;
        for (int i = 0; i < p - 1; ++i)
            for (int j = i + 1; j < p; ++j) {
                double alpha = 0, beta = 0, gamma = 0;
                double *wi = W + (size_t)i * n, *wj = W + (size_t)j * n;
                for (int r = 0; r < n; ++r) {
                    alpha += wi[r] * wi[r];
                    beta += wj[r] * wj[r];
                    gamma += wi[r] * wj[r];
                }
                if (fabs(gamma) <= 1e-15 * sqrt(alpha * beta) || gamma == 0.0) continue;
                rotated = 1;
                double zeta = (beta - alpha) / (2.0 * gamma);
                double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
                for (int r = 0; r < n; ++r) {
                    double a0 = wi[r], b0 = wj[r];
                    wi[r] = c * a0 - s * b0;
                    wj[r] = s * a0 + c * b0;
                }
                for (int r = 0; r < p; ++r) {
                    double a0 = V[r][i], b0 = V[r][j];
                    V[r][i] = c * a0 - s * b0;
                    V[r][j] = s * a0 + c * b0;
                }
            }
        if (!rotated) break;
    }
    double sig[5], smax = 0;
    for (int i = 0; i < p; ++i) {
        double s = 0;
        for (int r = 0; r < n; ++r) s += W[(size_t)i * n + r] * W[(size_t)i * n + r];
        sig[i] = sqrt(s);
        if (sig[i] > smax) smax = sig[i];
    }
    const double cutoff = 2.220446049250313e-16 * (n > p ? n : p) * smax;
    for (int j = 0; j < p; ++j) x[j] = 0;
    if (h) for (int r = 0; r < n; ++r) h[r] = 0;
    for (int i = 0; i < p; ++i) {
        if (sig[i] <= cutoff) continue;
        double uy = 0;
        for (int r = 0; r < n; ++r) uy += W[(size_t)i * n + r] / sig[i] * y[r];
        for (int j = 0; j < p; ++j) x[j] += V[j][i] * uy / sig[i];
        if (h)
            for (int r = 0; r < n; ++r) {
                double u = W[(size_t)i * n + r] / sig[i];
                h[r] += u * u;
            }
    }
    free(W);
}

static void rlm_fit(const double *X, const double *y, int n, int p, double *coef, double *scratch) {
    double *h = scratch, *adj = scratch + n, *r = scratch + 2 * n, *Xw = scratch + 3 * n,
           *yw = scratch + 3 * n + (size_t)5 * n, *tmp = yw + n;
    double coef0[5];
    lstsq_svd(X, y, n, p, coef, h);
    for (int i = 0; i < n; ++i) {
        double hh = h[i] < 0.9999 ? h[i] : 0.9999;
        adj[i] = 1.0 / sqrt(1.0 - hh);
    }
    double ym = 0, yv = 0;
    for (int i = 0; i < n; ++i) ym += y[i];
    ym /= n;
    for (int i = 0; i < n; ++i) yv += (y[i] - ym) * (y[i] - ym);
    const double ystd = sqrt(yv / n);
    int iteration = 1, converged = 0;
    while (!converged && iteration < 5) {
        memcpy(coef0, coef, sizeof(double) * p);
        for (int i = 0; i < n; ++i) {
            double pr = 0;
            for (int j = 0; j < p; ++j) pr += X[(size_t)j * n + i] * coef0[j];
            r[i] = (y[i] - pr) * adj[i];
            tmp[i] = fabs(r[i]);
        }
        qsort(tmp, (size_t)n, sizeof(double), cmp_double);
        double mad = median_sorted(tmp + 4, n - 4) / 0.6745;
        double scale = 2.220446049250313e-16 * ystd;
        if (mad > scale) scale = mad;
        for (int i = 0; i < n; ++i) {
            double u = r[i] / scale;
            double q = u / 4.685;
            double wgt = fabs(u) < 4.685 ? (1 - q * q) * (1 - q * q) : 0.0;
            double sw = sqrt(wgt);
            for (int j = 0; j < p; ++j) Xw[(size_t)j * n + i] = X[(size_t)j * n + i] * sw;
            yw[i] = y[i] * sw;
        }
        lstsq_svd(Xw, yw, n, p, coef, NULL);
        iteration += 1;
        converged = 1;
        for (int j = 0; j < p; ++j)
            if (coef[j] - coef0[j] > 1e-8) converged = 0;
    }
}

/* models/tmask.tmask over compacted window [a, b): outlier flags in out[0..b-a) */
static int tmask(pix_t *P, int a, int b, uint8_t *out) {
    const ccdgpu_params *p = P->p;
    const int n = b - a;
    const double w = 2.0 * M_PI / p->avg_days_yr;
    const double oc = w / ceil((period(P, b - 1) - period(P, a)) / p->avg_days_yr);
    const int ncol = (oc == w) ? 3 : 5;
    double *X = (double *)malloc(sizeof(double) * (size_t)n * 5);
    double *y = (double *)malloc(sizeof(double) * (size_t)n);
    double *scratch = (double *)malloc(sizeof(double) * (size_t)n * 12);
    for (int i = 0; i < n; ++i) {
        const double *bs = P->basis + (size_t)P->idx[a + i] * 6;
        double t = period(P, a + i);
        X[0 * (size_t)n + i] = bs[0];
        X[1 * (size_t)n + i] = bs[1];
        if (ncol == 5) {
            X[2 * (size_t)n + i] = cos(oc * t);
            X[3 * (size_t)n + i] = sin(oc * t);
            X[4 * (size_t)n + i] = 1.0;
        } else {
            X[2 * (size_t)n + i] = 1.0;
        }
        out[i] = 0;
    }
    int count = 0;
    for (int band = 0; band < NB; ++band) {
        if (!((p->tmask_bands >> band) & 1u)) continue;
        for (int i = 0; i < n; ++i) y[i] = spec(P, band, a + i);
        double coef[5];
        rlm_fit(X, y, n, ncol, coef, scratch);
        const double thr = P->vario[band] * p->t_const;
        for (int i = 0; i < n; ++i) {
            double pr = 0;
            for (int j = 0; j < ncol; ++j) pr += X[(size_t)j * n + i] * coef[j];
            pr += 0.0;
            if (fabs(pr - y[i]) > thr) out[i] = 1;
        }
    }
    for (int i = 0; i < n; ++i) count += out[i];
    free(X); free(y); free(scratch);
    return count;
}

/* ------------------------------------------------------------------ change.py */
static int num_coefs(const ccdgpu_params *p, int n) {
    double span = (double)n / p->num_obs_factor;
    if (span < p->coef_mid) return p->coef_min;
    if (span < p->coef_max) return p->coef_mid;
    return p->coef_max;
}

static int stable(pix_t *P, int a, int b) {
    const ccdgpu_params *p = P->p;
    double ss = 0;
    for (int band = 0; band < NB; ++band) {
        if (!((p->detection_bands >> band) & 1u)) continue;
        const fit_t *f = &P->models[band];
        double rn = P->vario[band] > f->rmse ? P->vario[band] : f->rmse;
        double slope = f->coef[0] * (period(P, b - 1) - period(P, a));
        double v = (fabs(slope) + fabs(f->resid[0]) + fabs(f->resid[b - a - 1])) / rn;
        ss += v * v;
    }
    return sqrt(ss) < P->chg_thr;
}

static void emit(pix_t *P, int64_t sday, int64_t eday, int64_t bday, int count, double chprob,
                 int curve_qa, const double *mags) {
    if (P->nseg == P->segcap) {
        P->segcap = P->segcap ? 2 * P->segcap : 16;
        P->segs = (ccdgpu_segment *)realloc(P->segs, sizeof(ccdgpu_segment) * (size_t)P->segcap);
    }
    ccdgpu_segment *s = &P->segs[P->nseg++];
    memset(s, 0, sizeof(*s));
    s->start_day = (int32_t)sday;
    s->end_day = (int32_t)eday;
    s->break_day = (int32_t)bday;
    s->observation_count = count;
    s->curve_qa = curve_qa;
    s->change_probability = chprob;
    for (int b = 0; b < NB; ++b) {
        s->magnitude[b] = mags ? mags[b] : 0.0;
        s->rmse[b] = P->models[b].rmse;
        s->intercept[b] = P->models[b].intercept;
        for (int j = 0; j < 7; ++j) s->coef[b][j] = P->models[b].coef[j];
    }
}

static void catch_(pix_t *P, int a, int b, int curve_qa) {
    fit_models(P, a, b, P->p->coef_min);
    int64_t bday = (b < P->m) ? period_i(P, b) : period_i(P, P->m - 1);
    emit(P, period_i(P, a), period_i(P, b - 1), bday, b - a, 0.0, curve_qa, NULL);
}

/* change magnitude of residual columns r[7][k] (only detection bands are read) */
static void magnitudes(const pix_t *P, const double r[NB][CCDGPU_MAX_PEEK], int k, const double *comp,
                       double *mag) {
    for (int j = 0; j < k; ++j) {
        double s = 0;
        for (int band = 0; band < NB; ++band) {
            if (!((P->p->detection_bands >> band) & 1u)) continue;
            double rm = P->vario[band] > comp[band] ? P->vario[band] : comp[band];
            double v = r[band][j] / rm;
            s += v * v;
        }
        mag[j] = s;
    }
}

static int initialize(pix_t *P, int *wa, int *wb) {
    const ccdgpu_params *p = P->p;
    int a = *wa, b = *wb;
    uint8_t *out = (uint8_t *)malloc((size_t)P->n + 1);
    int ok = 0;
    while (b + p->meow_size < P->m) {
        if (period(P, b - 1) - period(P, a) < p->day_delta) { b += 1; continue; }
        int cnt = tmask(P, a, b, out);
        if (cnt == b - a) { b += 1; continue; }
        /* enough time / samples after the Tmask removal */
        int first = -1, last = -1, kept = 0;
        for (int i = 0; i < b - a; ++i)
            if (!out[i]) { if (first < 0) first = i; last = i; ++kept; }
        if (period(P, a + last) - period(P, a + first) < p->day_delta || kept < p->meow_size) {
            b += 1;
            continue;
        }
        if (cnt) {
            for (int i = b - a - 1; i >= 0; --i) if (out[i]) mask_remove(P, a + i);
            b -= cnt;
        }
        fit_models(P, a, b, 4);
        if (!stable(P, a, b)) { a += 1; b += 1; continue; }
        ok = 1;
        break;
    }
    free(out);
    *wa = a;
    *wb = b;
    return ok;
}

static void lookback(pix_t *P, int *wa, int *wb, int prev) {
    const ccdgpu_params *p = P->p;
    int a = *wa, b = *wb;
    double r[NB][CCDGPU_MAX_PEEK], comp[NB], mag[CCDGPU_MAX_PEEK];
    for (int band = 0; band < NB; ++band) comp[band] = P->models[band].rmse;
    while (a > prev) {
        int lo; /* peek obs are a-1 down to lo (inclusive) */
        if (a - prev > P->peek) lo = a - P->peek + 1;
        else if (a - P->peek <= 0) lo = 0;
        else lo = prev;
        int k = a - lo;
        for (int j = 0; j < k; ++j)
            for (int band = 0; band < NB; ++band)
                r[band][j] = spec(P, band, a - 1 - j) - predict_at(P, &P->models[band], a - 1 - j);
        magnitudes(P, r, k, comp, mag);
        double mn = mag[0];
        for (int j = 1; j < k; ++j) if (mag[j] < mn) mn = mag[j];
        if (mn > P->chg_thr) break;
        if (mag[0] > p->outlier_threshold) {
            mask_remove(P, a - 1);
            a -= 1;
            b -= 1;
            continue;
        }
        a -= 1;
    }
    *wa = a;
    *wb = b;
}

static int cmp_key(const void *x, const void *y) {
    const double *a = (const double *)x, *b = (const double *)y;
    if (a[0] < b[0]) return -1;
    if (a[0] > b[0]) return 1;
    return (a[1] > b[1]) - (a[1] < b[1]);
}

static void lookforward(pix_t *P, int *wa, int *wb) {
    const ccdgpu_params *p = P->p;
    int a = *wa, b = *wb;
    int fa = a, fb = b;
    int have = 0, change = 0, nc = p->coef_min;
    double fit_span = period(P, b - 1) - period(P, a);
    double r[NB][CCDGPU_MAX_PEEK], comp[NB], mag[CCDGPU_MAX_PEEK];
    double *keys = (double *)malloc(sizeof(double) * 2 * (size_t)P->n);
    int32_t *cord = (int32_t *)malloc(sizeof(int32_t) * ((size_t)P->n + 1)), cidx[24];
    int peek_start = b;
    while (b + P->peek < P->m || !have) {
        nc = num_coefs(p, b - a);
        peek_start = b;
        const int k = P->peek;
        double model_span = period(P, b - 1) - period(P, a);
        if (!have || b - a < 24) {
            fa = a; fb = b;
            fit_span = period(P, b - 1) - period(P, a);
            fit_models(P, fa, fb, nc);
            have = 1;
            for (int band = 0; band < NB; ++band) comp[band] = P->models[band].rmse;
        } else {
            if (model_span >= 1.33 * fit_span) {
                fa = a; fb = b;
                fit_span = period(P, b - 1) - period(P, a);
                fit_models(P, fa, fb, nc);
            }
            /* find_closest_doy(period, peek.stop - 1, fit_window, 24): argsort(d_yr)[:24] */
            const int64_t ref = period_i(P, b + k - 1);
            const int nf = fb - fa;
            const int take = nf < 24 ? nf : 24;
            if (p->argsort_stable) {
                for (int i = 0; i < nf; ++i) {
                    double d = (double)(period_i(P, fa + i) - ref);
                    keys[2 * i] = fabs(rint(d / 365.25) * 365.25 - d);
                    keys[2 * i + 1] = i;
                }
                qsort(keys, (size_t)nf, 2 * sizeof(double), cmp_key);
                for (int j = 0; j < take; ++j) cidx[j] = (int32_t)keys[2 * j + 1];
            } else {
                for (int i = 0; i < nf; ++i) {
                    double d = (double)(period_i(P, fa + i) - ref);
                    keys[i] = fabs(rint(d / 365.25) * 365.25 - d);
                    cord[i] = i;
                }
                ccdoracle_np_argsort(keys, cord, nf, 24, &P->qs_deep);
                for (int j = 0; j < take; ++j) cidx[j] = cord[j];
                if (nf > 24) {  /* exposure statistics (ccdoracle_argsort_stats) */
                    const double kk = keys[cord[23]];
                    int lt = 0, le = 0;
                    for (int i = 0; i < nf; ++i) { lt += keys[i] < kk; le += keys[i] <= kk; }
                    __atomic_add_fetch(&g_qs_stats[0], 1, __ATOMIC_RELAXED);
                    if (le > 24) {
                        /* ties straddle the 24th position: does the stable rule (lowest fit
                           indices of the tied entries) take another set? */
                        int need = 24 - lt, diff = 0, seen = 0;
                        for (int i = 0; i < nf && seen < need; ++i)
                            if (keys[i] == kk) {
                                int in = 0;
                                for (int j = lt; j < 24; ++j) in |= cord[j] == i;
                                diff |= !in;
                                ++seen;
                            }
                        __atomic_add_fetch(&g_qs_stats[1], 1, __ATOMIC_RELAXED);
                        if (diff) __atomic_add_fetch(&g_qs_stats[2], 1, __ATOMIC_RELAXED);
                    }
                }
            }
            /* euclidean_norm(residual[closest]) / 4: numpy's pairwise sum of the squares in
               argsort order (math_utils.euclidean_norm = np.sum(v ** 2) ** .5) */
            for (int band = 0; band < NB; ++band) {
                double sq[24];
                for (int j = 0; j < take; ++j) {
                    double e = P->models[band].resid[cidx[j]];
                    sq[j] = e * e;
                }
                comp[band] = sqrt(np_pairwise_sum(sq, take)) / 4.0;
            }
        }
        for (int j = 0; j < k; ++j)
            for (int band = 0; band < NB; ++band)
                r[band][j] = spec(P, band, b + j) - predict_at(P, &P->models[band], b + j);
        magnitudes(P, r, k, comp, mag);
        double mn = mag[0];
        for (int j = 1; j < k; ++j) if (mag[j] < mn) mn = mag[j];
        if (mn > P->chg_thr) { change = 1; break; }
        if (mag[0] > p->outlier_threshold) { mask_remove(P, b); continue; }
        b += 1;
    }
    /* result: magnitudes = median of the last peek residuals per band */
    double mags[NB], tmp[CCDGPU_MAX_PEEK];
    for (int band = 0; band < NB; ++band) {
        for (int j = 0; j < P->peek; ++j) tmp[j] = r[band][j];
        mags[band] = median_inplace(tmp, P->peek);
    }
    emit(P, period_i(P, a), period_i(P, b - 1), period_i(P, peek_start), b - a, (double)change, nc, mags);
    free(keys);
    free(cord);
    *wa = a;
    *wb = b;
}

/* math_utils.adjusted_variogram over the compacted series */
static void variogram(pix_t *P) {
    const int m = P->m;
    if (m < 2) { for (int b = 0; b < NB; ++b) P->vario[b] = NAN; return; }
    double *buf = (double *)malloc(sizeof(double) * (size_t)m);
    int lag = 0;
    for (int k = 1; k < m; ++k) {
        int cnt = 0;
        for (int i = 0; i + k < m; ++i) cnt += (period_i(P, i + k) - period_i(P, i)) > 30;
        if (2 * cnt >= m - k) { lag = k; break; }
    }
    for (int b = 0; b < NB; ++b) {
        int c = 0;
        if (lag == 0) {
            for (int i = 0; i + 1 < m; ++i) buf[c++] = fabs(spec(P, b, i + 1) - spec(P, b, i));
        } else {
            for (int i = 0; i + lag < m; ++i)
                if (period_i(P, i + lag) - period_i(P, i) > 30) buf[c++] = fabs(spec(P, b, i + lag) - spec(P, b, i));
        }
        P->vario[b] = median_inplace(buf, c);
    }
    free(buf);
}

static void standard_procedure(pix_t *P) {
    const ccdgpu_params *p = P->p;
    const int meow = p->meow_size;
    variogram(P);
    P->peek = p->peek_size;
    P->chg_thr = p->change_threshold;
    if (p->adaptive_peek && P->m >= 2) {
        double *d = (double *)malloc(sizeof(double) * (size_t)P->m);
        for (int i = 0; i + 1 < P->m; ++i) d[i] = (double)(period_i(P, i + 1) - period_i(P, i));
        double delta = median_inplace(d, P->m - 1);
        free(d);
        double adj = rint((double)p->peek_size * 16.0 / delta);
        if (adj > p->peek_size) {
            /* as the kernel (include/ccdgpu.h CCDGPU_MAX_PEEK): a peek past 96 is reported
               (CCDGPU_EOVERFLOW), the pixel finishes with the largest supported peek */
            if (adj > CCDGPU_MAX_PEEK) P->overflow = 1;
            P->peek = adj > CCDGPU_MAX_PEEK ? CCDGPU_MAX_PEEK : (int)adj;
            double pt = 1.0 - pow(1.0 - p->change_probability, (double)p->peek_size / P->peek);
            P->chg_thr = chi2_5_ppf(pt);
        }
    }
    int a = 0, b = meow, prev = 0, start = 1, nres = 0;
    while (b <= P->m - meow) {
        if (nres > 0) start = 0;
        if (!initialize(P, &a, &b)) break;
        if (a > prev) lookback(P, &a, &b, prev);
        if (a - prev > P->peek && start) {
            catch_(P, prev, a, p->curve_qa_start);
            nres++;
            start = 0;
        }
        if (b + P->peek > P->m) break;
        lookforward(P, &a, &b);
        nres++;
        prev = b;
        a = b;
        b = b + meow;
    }
    if (prev + P->peek < P->m) catch_(P, prev, P->m, p->curve_qa_end);
}

/* ------------------------------------------------------------------ qa.py */
static int qabitval(const ccdgpu_params *p, unsigned v) {
#define BIT(o) ((v >> (o)) & 1u)
    if (BIT(p->qa_fill)) return p->qa_fill;
    if (BIT(p->qa_cloud)) return p->qa_cloud;
    if (BIT(p->qa_shadow)) return p->qa_shadow;
    if (BIT(p->qa_snow)) return p->qa_snow;
    if (BIT(p->qa_water)) return p->qa_water;
    if (BIT(p->qa_clear)) return p->qa_clear;
    if (BIT(p->qa_cirrus1) && BIT(p->qa_cirrus2)) return p->qa_clear;
    if (BIT(p->qa_occlusion)) return p->qa_clear;
    return -1;
#undef BIT
}

static int detect_pixel(const ccdgpu_params *p, int n, const int64_t *t, const double *basis,
                        const int32_t *order, const int16_t *spectra_in, const uint16_t *qa_in,
                        size_t band_stride, ccdgpu_segment **segs, int *nseg, uint32_t *mask_bits,
                        int32_t *proc, double *probs, int64_t *fits, int64_t *sweeps) {
    pix_t P;
    memset(&P, 0, sizeof(P));
    P.p = p;
    P.n = n;
    P.t = t;
    P.basis = basis;
    P.obs = (int16_t *)malloc(sizeof(int16_t) * 7 * (size_t)n);
    P.mask = (uint8_t *)calloc((size_t)n, 1);
    P.idx = (int *)malloc(sizeof(int) * (size_t)n);
    int *cls = (int *)malloc(sizeof(int) * (size_t)n);
    int rc = 0;
    for (int i = 0; i < n; ++i) {
        for (int b = 0; b < NB; ++b) P.obs[(size_t)b * n + i] = spectra_in[b * band_stride + order[i]];
        unsigned q = qa_in[order[i]];
        cls[i] = p->qa_bitpacked ? qabitval(p, q) : (int)q;
        if (cls[i] < 0) rc = CCDGPU_EQA;
    }
    if (rc) goto done;
    {
        int c_clear = 0, c_water = 0, c_snow = 0, c_cloud = 0, c_total = 0;
        for (int i = 0; i < n; ++i) {
            c_clear += cls[i] == p->qa_clear;
            c_water += cls[i] == p->qa_water;
            c_snow += cls[i] == p->qa_snow;
            c_cloud += cls[i] == p->qa_cloud;
            c_total += cls[i] != p->qa_fill;
        }
        const int cw = c_clear + c_water;
        probs[0] = (double)c_cloud / (double)c_total;
        probs[1] = (double)c_snow / (cw + c_snow + 0.01);
        probs[2] = (double)c_water / (cw + c_snow + 0.01);
        int procedure;
        if (!((double)cw / (double)c_total >= p->clear_pct_threshold))
            procedure = ((double)c_snow / (cw + c_snow + 0.01) >= p->snow_pct_threshold)
                            ? CCDGPU_PROC_PERMANENT_SNOW : CCDGPU_PROC_INSUFFICIENT_CLEAR;
        else
            procedure = CCDGPU_PROC_STANDARD;
        *proc = procedure;
        if (procedure == CCDGPU_PROC_STANDARD && p->kelvin_to_celsius)
            for (int i = 0; i < n; ++i)
                P.obs[6 * (size_t)n + i] = (int16_t)(P.obs[6 * (size_t)n + i] * 10 - 27315);
        /* standard_procedure_filter (+ snow / insufficient-clear variants) */
        int64_t last_kept = INT64_MIN;
        for (int i = 0; i < n; ++i) {
            int cw_i = cls[i] == p->qa_clear || cls[i] == p->qa_water;
            int th = P.obs[6 * (size_t)n + i] > p->thermal_min && P.obs[6 * (size_t)n + i] < p->thermal_max;
            int sat = 1;
            for (int b = 0; b < 6; ++b) {
                int16_t v = P.obs[(size_t)b * n + i];
                if (!(v > 0 && v < 10000)) sat = 0;
            }
            int keep = cw_i && th && sat;
            if (procedure == CCDGPU_PROC_PERMANENT_SNOW) keep = keep || cls[i] == p->qa_snow;
            if (keep) {
                if (t[i] == last_kept) keep = 0; /* mask_duplicate_values: first of repeated dates */
                else last_kept = t[i];
            }
            P.mask[i] = (uint8_t)keep;
        }
        if (procedure == CCDGPU_PROC_INSUFFICIENT_CLEAR) {
            int c = 0;
            double *g = (double *)malloc(sizeof(double) * (size_t)n + 8);
            for (int i = 0; i < n; ++i) if (P.mask[i]) g[c++] = P.obs[1 * (size_t)n + i];
            if (c > 0) {
                double med = median_inplace(g, c) + p->median_green_filter;
                for (int i = 0; i < n; ++i)
                    if (P.mask[i] && !(P.obs[1 * (size_t)n + i] < med)) P.mask[i] = 0;
            }
            free(g);
        }
        P.m = 0;
        for (int i = 0; i < n; ++i) if (P.mask[i]) P.idx[P.m++] = i;
        const size_t nn = (size_t)n + 8;
        P.X = (double *)malloc(sizeof(double) * 7 * nn);
        P.Xc = (double *)malloc(sizeof(double) * 7 * nn);
        P.yc = (double *)malloc(sizeof(double) * nn);
        P.y = (double *)malloc(sizeof(double) * nn);
        P.R = (double *)malloc(sizeof(double) * nn);
        P.resid_store = (double *)malloc(sizeof(double) * 7 * nn);
        if (procedure == CCDGPU_PROC_STANDARD) {
            standard_procedure(&P);
        } else if (P.m >= p->meow_size) {
            fit_models(&P, 0, P.m, p->coef_min);
            emit(&P, t[0], t[n - 1], 0, P.m, 0.0,
                 procedure == CCDGPU_PROC_PERMANENT_SNOW ? p->curve_qa_persist_snow : p->curve_qa_insuf_clear,
                 NULL);
        }
        for (int i = 0; i < n; ++i)
            if (P.mask[i]) mask_bits[i >> 5] |= 1u << (i & 31);
        free(P.X); free(P.Xc); free(P.yc); free(P.y); free(P.R); free(P.resid_store);
    }
done:
    if (!rc && P.overflow) rc = CCDGPU_EOVERFLOW;
    *segs = P.segs;
    *nseg = P.nseg;
    *fits += P.fits;
    if (P.qs_deep) __atomic_add_fetch(&g_qs_stats[3], P.qs_deep, __ATOMIC_RELAXED);
    *sweeps += P.sweeps;
    free(P.obs); free(P.mask); free(P.idx); free(cls);
    return rc;
}

/* ------------------------------------------------------------------ public oracle entry */
typedef struct { int64_t d; int32_t i; } di_t;
static int cmp_di(const void *x, const void *y) {
    const di_t *a = (const di_t *)x, *b = (const di_t *)y;
    if (a->d != b->d) return (a->d > b->d) - (a->d < b->d);
    return (a->i > b->i) - (a->i < b->i);
}

void ccdoracle_params_default(ccdgpu_params *p) {
    memset(p, 0, sizeof(*p));
    p->meow_size = 12; p->peek_size = 6; p->day_delta = 365;
    p->coef_min = 4; p->coef_mid = 6; p->coef_max = 8; p->num_obs_factor = 3;
    p->detection_bands = 0x3E; p->tmask_bands = 0x12;
    p->lasso_max_iter = 1000;
    p->thermal_min = -9320; p->thermal_max = 7070; p->median_green_filter = 400;
    p->curve_qa_start = 14; p->curve_qa_end = 24; p->curve_qa_insuf_clear = 44; p->curve_qa_persist_snow = 54;
    p->qa_fill = 0; p->qa_clear = 1; p->qa_water = 2; p->qa_shadow = 3; p->qa_snow = 4; p->qa_cloud = 5;
    p->qa_cirrus1 = 8; p->qa_cirrus2 = 9; p->qa_occlusion = 10;
    p->qa_bitpacked = 1; p->adaptive_peek = 1; p->rmse_dof = 0; p->kelvin_to_celsius = 1;
    p->avg_days_yr = 365.2425; p->change_probability = 0.99;
    p->change_threshold = 15.086272469388987; p->outlier_threshold = 35.888186879610423;
    p->t_const = 4.42; p->lasso_alpha = 1.0; p->lasso_tol = 1e-4;
    p->clear_pct_threshold = 0.25; p->snow_pct_threshold = 0.75;
}

double ccdoracle_chi2_5_ppf(double p) { return chi2_5_ppf(p); }

/* Same layout contract as ccdgpu_detect_batch (include/ccdgpu.h). Returns 0, CCDGPU_EOVERFLOW (a
   pixel's adaptive peek exceeds CCDGPU_MAX_PEEK) or CCDGPU_EQA. */
int ccdoracle_detect_batch(const ccdgpu_params *p, int32_t n_pix, int32_t n_obs, const int64_t *dates,
                           const int16_t *spectra, const uint16_t *qa, ccdgpu_result *out, int32_t n_threads) {
    memset(out, 0, sizeof(*out));
    out->n_pix = n_pix;
    out->n_obs = n_obs;
    out->error_pixel = -1;
    out->mask_words = (n_obs + 31) / 32;
    di_t *srt = (di_t *)malloc(sizeof(di_t) * (size_t)(n_obs > 0 ? n_obs : 1));
    if (p->argsort_stable) {
        for (int i = 0; i < n_obs; ++i) { srt[i].d = dates[i]; srt[i].i = i; }
        qsort(srt, (size_t)n_obs, sizeof(di_t), cmp_di);
    } else {  /* ccd.detect: indices = np.argsort(dates) (numpy quicksort) */
        double *dk = (double *)calloc((size_t)(n_obs > 0 ? n_obs : 1), sizeof(double));
        int32_t *ord = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_obs > 0 ? n_obs : 1));
        for (int i = 0; i < n_obs; ++i) { dk[i] = (double)dates[i]; ord[i] = i; }
        ccdoracle_np_argsort(dk, ord, n_obs, 0, NULL);
        for (int i = 0; i < n_obs; ++i) { srt[i].d = dates[ord[i]]; srt[i].i = ord[i]; }
        free(dk);
        free(ord);
    }
    out->sorted_dates = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n_obs + 1));
    out->sort_index = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_obs + 1));
    double *basis = (double *)malloc(sizeof(double) * 6 * (size_t)(n_obs + 1));
    const double w = 2.0 * M_PI / p->avg_days_yr;
    for (int i = 0; i < n_obs; ++i) {
        out->sorted_dates[i] = srt[i].d;
        out->sort_index[i] = srt[i].i;
        double w12 = w * (double)srt[i].d, w34 = 2.0 * w12, w56 = 3.0 * w12;
        basis[6 * i + 0] = cos(w12); basis[6 * i + 1] = sin(w12);
        basis[6 * i + 2] = cos(w34); basis[6 * i + 3] = sin(w34);
        basis[6 * i + 4] = cos(w56); basis[6 * i + 5] = sin(w56);
    }
    free(srt);
    out->mask_bits = (uint32_t *)calloc((size_t)n_pix * out->mask_words + 1, sizeof(uint32_t));
    out->procedure = (int32_t *)calloc((size_t)n_pix + 1, sizeof(int32_t));
    out->probs = (double *)calloc((size_t)n_pix * 3 + 1, sizeof(double));
    out->seg_offsets = (int64_t *)calloc((size_t)n_pix + 1, sizeof(int64_t));
    ccdgpu_segment **psegs = (ccdgpu_segment **)calloc((size_t)n_pix + 1, sizeof(void *));
    int *pn = (int *)calloc((size_t)n_pix + 1, sizeof(int));
    int err_pix = -1, ovf_pix = -1;
    int64_t fits = 0, sweeps = 0;
    (void)n_threads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads > 0 ? n_threads : 1) reduction(+ : fits, sweeps)
    for (int px = 0; px < n_pix; ++px) {
        int rc = detect_pixel(p, n_obs, out->sorted_dates, basis, out->sort_index,
                              spectra + (size_t)px * n_obs, qa + (size_t)px * n_obs,
                              (size_t)n_pix * n_obs, &psegs[px], &pn[px],
                              out->mask_bits + (size_t)px * out->mask_words, &out->procedure[px],
                              out->probs + 3 * (size_t)px, &fits, &sweeps);
        if (rc == CCDGPU_EQA) {
#pragma omp critical
            if (err_pix < 0 || px < err_pix) err_pix = px;
        } else if (rc == CCDGPU_EOVERFLOW) {
#pragma omp critical
            if (ovf_pix < 0 || px < ovf_pix) ovf_pix = px;
        }
    }
    int64_t tot = 0;
    for (int px = 0; px < n_pix; ++px) { out->seg_offsets[px] = tot; tot += pn[px]; }
    out->seg_offsets[n_pix] = tot;
    out->n_seg = tot;
    out->segments = (ccdgpu_segment *)malloc(sizeof(ccdgpu_segment) * (size_t)(tot + 1));
    for (int px = 0; px < n_pix; ++px) {
        for (int s = 0; s < pn[px]; ++s) {
            psegs[px][s].pixel = px;
            out->segments[out->seg_offsets[px] + s] = psegs[px][s];
        }
        free(psegs[px]);
    }
    free(psegs); free(pn); free(basis);
    out->error_pixel = err_pix;
    out->seconds_kernel = (double)fits;   /* oracle: reports fit/sweep counters here */
    out->seconds_total = (double)sweeps;
    if (ovf_pix >= 0) return CCDGPU_EOVERFLOW;
    return err_pix >= 0 ? CCDGPU_EQA : 0;
}

void ccdoracle_result_free(ccdgpu_result *r) {
    free(r->seg_offsets); free(r->segments); free(r->mask_bits); free(r->procedure);
    free(r->probs); free(r->sorted_dates); free(r->sort_index);
    memset(r, 0, sizeof(*r));
}
