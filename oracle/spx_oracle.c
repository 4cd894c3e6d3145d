/*
 * ORACLE -- plain-C restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library (oracle/build/libspx_oracle.so via oracle/c_oracle.py), as the
 * checker or as the timed single-core CPU baseline.  The product never links it.
 *
 * Restates (paths relative to the reference repository root):
 *   spxo_bin_mean     src/binning.py:170-231                      (bit-exact)
 *   spxo_gap_average  src/average_spectrum_clustering.py:26-103   (stable sort ->
 *                     equal to numpy up to the order of tied m/z, i.e. within 1e-12)
 *   spxo_medoid       src/most_similar_representative.py:13-19, 60-111 with OpenMS
 *                     XQuestScores::xCorrelationPrescore restated (PARITY UNPINNED
 *                     at the xcorr boundary).  mode 1 builds
 *                     OpenMS's two dense f64 ion tables per pair (the reference's
 *                     cost model); mode 0 intersects sorted bin sets (same result).
 *   spxo_pairwise_sum numpy pairwise summation (the .sum() of :98-100).
 * Pinned against the fixtures in tests/golden by tests/test_oracle_golden.py.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: IEEE sub/div, no FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { ST_OK = 0, ST_MIXED_CHARGE = 1, ST_NO_GAP = 2, ST_EMPTY = 3 };

/* ------------------------------------------------------------ pairwise sum */
static double pw_rec(const double *a, int64_t n, int64_t stride) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i * stride];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int k = 0; k < 8; ++k) r[k] = a[k * stride];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int k = 0; k < 8; ++k) r[k] += a[(i + k) * stride];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i * stride];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pw_rec(a, n2, stride) + pw_rec(a + n2 * stride, n - n2, stride);
}

double spxo_pairwise_sum(const double *a, int64_t n) { return 0.0 + pw_rec(a, n, 1); }

/* ---------------------------------------------------------------- bin-mean */
static int cmp_i64(const void *x, const void *y) {
  int64_t a = *(const int64_t *)x, b = *(const int64_t *)y;
  return (a > b) - (a < b);
}

/* out_off[C+1] is filled; out_mz/out_int need capacity >= total valid peaks. */
int spxo_bin_mean(int64_t C, const int64_t *cluster_off, const int64_t *spec_off, const double *mz,
                  const double *inten, const double *prec, const int32_t *charge, double minimum,
                  double maximum, double binsize, int apply_quorum, int64_t *out_off, double *out_mz,
                  double *out_int, double *out_prec, int32_t *out_charge, int32_t *status) {
  int64_t n_bins = (int64_t)((maximum - minimum) / binsize) + 1;
  float *acc_i = (float *)calloc((size_t)n_bins, sizeof(float));
  float *acc_m = (float *)calloc((size_t)n_bins, sizeof(float));
  int32_t *cnt = (int32_t *)calloc((size_t)n_bins, sizeof(int32_t));
  int64_t *stamp = (int64_t *)malloc((size_t)n_bins * sizeof(int64_t));
  int64_t max_p = 0;
  for (int64_t c = 0; c < C; ++c) {
    int64_t p = spec_off[cluster_off[c + 1]] - spec_off[cluster_off[c]];
    if (p > max_p) max_p = p;
  }
  int64_t *touched = (int64_t *)malloc((size_t)(max_p + 1) * sizeof(int64_t));
  if (!acc_i || !acc_m || !cnt || !stamp || !touched) return -1;
  for (int64_t b = 0; b < n_bins; ++b) stamp[b] = -1;
  out_off[0] = 0;
  for (int64_t c = 0; c < C; ++c) {
    int64_t s0 = cluster_off[c], s1 = cluster_off[c + 1], n = s1 - s0, nt = 0;
    int32_t quorum = apply_quorum ? (int32_t)((double)n * 0.25) + 1 : 1;
    for (int64_t s = s0; s < s1; ++s) {
      /* reverse scan: the first hit of a bin is the file-order LAST peak (numpy last-wins) */
      for (int64_t k = spec_off[s + 1] - 1; k >= spec_off[s]; --k) {
        double m = mz[k];
        if (!(m >= minimum && m < maximum)) continue;
        int64_t b = (int64_t)((m - minimum) / binsize);
        if (stamp[b] == s) continue;
        if (stamp[b] < s0) touched[nt++] = b;  /* first touch in this cluster */
        stamp[b] = s;
        cnt[b] += 1;
        acc_i[b] = (float)((double)acc_i[b] + inten[k]);
        acc_m[b] = (float)((double)acc_m[b] + m);
      }
    }
    qsort(touched, (size_t)nt, sizeof(int64_t), cmp_i64);
    int mixed = 0;
    for (int64_t s = s0 + 1; s < s1; ++s) mixed |= charge[s] != charge[s0];
    int64_t o = out_off[c];
    if (mixed || n == 0) {
      status[c] = mixed ? ST_MIXED_CHARGE : ST_EMPTY;
      out_prec[c] = NAN;
      out_charge[c] = 0;
    } else {
      for (int64_t t = 0; t < nt; ++t) {
        int64_t b = touched[t];
        double mi = (double)acc_i[b] / (double)cnt[b];
        if (cnt[b] >= quorum && !isnan(mi)) {
          out_int[o] = mi;
          out_mz[o] = acc_m[b] == 0.0f ? NAN : (double)acc_m[b] / (double)cnt[b];
          ++o;
        }
      }
      out_prec[c] = (0.0 + pw_rec(prec + s0, n, 1)) / (double)n;
      out_charge[c] = charge[s0];
      status[c] = ST_OK;
    }
    out_off[c + 1] = o;
    for (int64_t t = 0; t < nt; ++t) {
      int64_t b = touched[t];
      acc_i[b] = 0.0f;
      acc_m[b] = 0.0f;
      cnt[b] = 0;
    }
  }
  free(acc_i); free(acc_m); free(cnt); free(stamp); free(touched);
  return 0;
}

/* ------------------------------------------------------------- gap-average */
typedef struct { double mz, it; int64_t idx; } peak_t;

static int cmp_peak(const void *x, const void *y) {
  const peak_t *a = (const peak_t *)x, *b = (const peak_t *)y;
  const int an = isnan(a->mz), bn = isnan(b->mz);
  if (an != bn) return an - bn;  /* np.argsort: NaN last */
  if (a->mz < b->mz) return -1;
  if (a->mz > b->mz) return 1;
  return (a->idx > b->idx) - (a->idx < b->idx);
}

int spxo_gap_average(int64_t C, const int64_t *cluster_off, const int64_t *spec_off, const double *mz,
                     const double *inten, double mz_accuracy, double dyn_range, double min_fraction,
                     int64_t *out_off, double *out_mz, double *out_int, int32_t *status) {
  int64_t max_p = 0;
  for (int64_t c = 0; c < C; ++c) {
    int64_t p = spec_off[cluster_off[c + 1]] - spec_off[cluster_off[c]];
    if (p > max_p) max_p = p;
  }
  peak_t *pk = (peak_t *)malloc((size_t)(max_p + 1) * sizeof(peak_t));
  double *cm = (double *)malloc((size_t)(max_p + 1) * sizeof(double));
  double *ci = (double *)malloc((size_t)(max_p + 1) * sizeof(double));
  int64_t *bnd = (int64_t *)malloc((size_t)(max_p + 2) * sizeof(int64_t));
  if (!pk || !cm || !ci || !bnd) return -1;
  out_off[0] = 0;
  for (int64_t c = 0; c < C; ++c) {
    int64_t s0 = cluster_off[c], s1 = cluster_off[c + 1], n = s1 - s0;
    int64_t p0 = spec_off[s0], N = spec_off[s1] - p0, o = out_off[c], o0 = o;
    status[c] = ST_OK;
    if (n == 0) {
      status[c] = ST_NO_GAP;
    } else if (n == 1) {
      for (int64_t k = 0; k < N; ++k) { out_mz[o] = mz[p0 + k]; out_int[o] = inten[p0 + k]; ++o; }
    } else {
      for (int64_t k = 0; k < N; ++k) { pk[k].mz = mz[p0 + k]; pk[k].it = inten[p0 + k]; pk[k].idx = k; }
      qsort(pk, (size_t)N, sizeof(peak_t), cmp_peak);
      int64_t m = 0;  /* number of gaps */
      for (int64_t k = 0; k + 1 < N; ++k)
        if (pk[k + 1].mz - pk[k].mz >= mz_accuracy) bnd[1 + m++] = k + 1;
      if (m == 0) {
        status[c] = ST_NO_GAP;
      } else {
        double sm = 0.0, si = 0.0;
        for (int64_t k = 0; k < N; ++k) { sm += pk[k].mz; si += pk[k].it; cm[k] = sm; ci[k] = si; }
        bnd[0] = 0;
        int64_t nb;
        if (m == 1) { nb = 3; bnd[2] = N; }                   /* [0,s0) [s0,N)            */
        else { nb = m + 1; bnd[m] = N; }                       /* last two groups merged   */
        double min_len = min_fraction * (double)n;
        for (int64_t g = 0; g + 1 < nb; ++g) {
          int64_t a = bnd[g], b = bnd[g + 1];
          if ((double)(b - a) < min_len) continue;
          double sum_m = a > 0 ? cm[b - 1] - cm[a - 1] : cm[b - 1];
          double sum_i = a > 0 ? ci[b - 1] - ci[a - 1] : ci[b - 1];
          out_mz[o] = sum_m / (double)(b - a);
          out_int[o] = sum_i / (double)n;
          ++o;
        }
      }
    }
    if (status[c] == ST_OK) {
      if (o == o0) {
        status[c] = ST_EMPTY;
      } else {
        double mx = out_int[o0];
        for (int64_t k = o0 + 1; k < o; ++k) if (isnan(out_int[k]) || out_int[k] > mx) mx = out_int[k];
        double thr = mx / dyn_range;
        int64_t w = o0;
        for (int64_t k = o0; k < o; ++k)
          if (out_int[k] >= thr) { out_mz[w] = out_mz[k]; out_int[w] = out_int[k]; ++w; }
        o = w;
      }
    }
    if (status[c] != ST_OK) o = o0;
    out_off[c + 1] = o;
  }
  free(pk); free(cm); free(ci); free(bnd);
  return 0;
}

/* ------------------------------------------------------------------ medoid */
/* OpenMS XQuestScores::xCorrelationPrescore, restated: dense binary ion tables. */
static double xcorr_dense(const double *a, int64_t na, const double *b, int64_t nb, double tol,
                          double **t1, double **t2, int64_t *cap) {
  if (na == 0 || nb == 0) return 0.0;
  double maxion = a[na - 1] > b[nb - 1] ? a[na - 1] : b[nb - 1];
  int64_t size = (int64_t)ceil(maxion / tol) + 1;
  int64_t need = size;
  for (int64_t i = 0; i < na; ++i) { int64_t p = (int64_t)ceil(a[i] / tol); if (p + 1 > need) need = p + 1; }
  for (int64_t i = 0; i < nb; ++i) { int64_t p = (int64_t)ceil(b[i] / tol); if (p + 1 > need) need = p + 1; }
  if (need > *cap) {
    *t1 = (double *)realloc(*t1, (size_t)need * sizeof(double));
    *t2 = (double *)realloc(*t2, (size_t)need * sizeof(double));
    *cap = need;
  }
  memset(*t1, 0, (size_t)need * sizeof(double));
  memset(*t2, 0, (size_t)need * sizeof(double));
  for (int64_t i = 0; i < na; ++i) (*t1)[(int64_t)ceil(a[i] / tol)] = 1.0;
  for (int64_t i = 0; i < nb; ++i) (*t2)[(int64_t)ceil(b[i] / tol)] = 1.0;
  double dot = 0.0;
  for (int64_t i = 0; i < need; ++i) dot += (*t1)[i] * (*t2)[i];
  double peaks = (double)(na < nb ? na : nb);
  return dot / peaks;
}

static int64_t unique_bins(const double *a, int64_t na, double tol, int64_t *out) {
  for (int64_t i = 0; i < na; ++i) out[i] = (int64_t)ceil(a[i] / tol);
  qsort(out, (size_t)na, sizeof(int64_t), cmp_i64);
  int64_t u = 0;
  for (int64_t i = 0; i < na; ++i) if (u == 0 || out[u - 1] != out[i]) out[u++] = out[i];
  return u;
}

/* rep[c] = global spectrum index (-1 for an empty cluster); totals[S] optional. */
int spxo_medoid(int64_t C, const int64_t *cluster_off, const int64_t *spec_off, const double *mz,
                double tol, int dense_tables, int64_t *rep, double *totals) {
  double *t1 = NULL, *t2 = NULL;
  int64_t cap = 0, max_n = 0, max_p = 0;
  for (int64_t c = 0; c < C; ++c) {
    int64_t n = cluster_off[c + 1] - cluster_off[c];
    if (n > max_n) max_n = n;
  }
  int64_t S = C ? cluster_off[C] : 0;
  for (int64_t s = 0; s < S; ++s) if (spec_off[s + 1] - spec_off[s] > max_p) max_p = spec_off[s + 1] - spec_off[s];
  double *D = (double *)malloc((size_t)(max_n * max_n + 1) * sizeof(double));
  int64_t *bins = (int64_t *)malloc((size_t)((dense_tables ? 0 : spec_off[S]) + 1) * sizeof(int64_t));
  int64_t *nbin = (int64_t *)malloc((size_t)(max_n + 1) * sizeof(int64_t));
  int64_t *boff = (int64_t *)malloc((size_t)(max_n + 1) * sizeof(int64_t));
  if (!D || !bins || !nbin || !boff) return -1;
  for (int64_t c = 0; c < C; ++c) {
    int64_t s0 = cluster_off[c], n = cluster_off[c + 1] - s0;
    if (n == 0) { rep[c] = -1; continue; }
    if (n == 1) { rep[c] = s0; if (totals) totals[s0] = 0.0; continue; }
    if (!dense_tables) {
      int64_t off = 0;
      for (int64_t i = 0; i < n; ++i) {
        int64_t s = s0 + i;
        boff[i] = off;
        nbin[i] = unique_bins(mz + spec_off[s], spec_off[s + 1] - spec_off[s], tol, bins + off);
        off += nbin[i];
      }
    }
    memset(D, 0, (size_t)(n * n) * sizeof(double));
    for (int64_t i = 0; i < n; ++i) {
      int64_t si = s0 + i, pi = spec_off[si + 1] - spec_off[si];
      for (int64_t j = i; j < n; ++j) {
        int64_t sj = s0 + j, pj = spec_off[sj + 1] - spec_off[sj];
        double x;
        if (dense_tables) {
          x = xcorr_dense(mz + spec_off[si], pi, mz + spec_off[sj], pj, tol, &t1, &t2, &cap);
        } else if (pi == 0 || pj == 0) {
          x = 0.0;
        } else {
          const int64_t *a = bins + boff[i], *b = bins + boff[j];
          int64_t ia = 0, ib = 0, cnt = 0;
          while (ia < nbin[i] && ib < nbin[j]) {
            if (a[ia] < b[ib]) ++ia;
            else if (a[ia] > b[ib]) ++ib;
            else { ++cnt; ++ia; ++ib; }
          }
          x = (double)cnt / (double)(pi < pj ? pi : pj);
        }
        D[i * n + j] = 1.0 - x;
      }
    }
    int64_t best = 0;
    double best_t = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      double t = ((0.0 + pw_rec(D + i * n, n, 1)) + (0.0 + pw_rec(D + i, n, n))) / (double)n;
      if (totals) totals[s0 + i] = t;
      if (i == 0 || t < best_t) { best = i; best_t = t; }
    }
    rep[c] = s0 + best;
  }
  free(t1); free(t2); free(D); free(bins); free(nbin); free(boff);
  return 0;
}
