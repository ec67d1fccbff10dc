/* CPU oracle, C restatement: the reference's dense per-window scan, OpenMP over windows.
 *
 * TEST INFRASTRUCTURE ONLY (like oracle/sfs_oracle.py): only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load it, as a checker or as the timed CPU baseline.  The product
 * path never does.  It is pinned to the numpy oracle (tests/test_oracle_c.py), which is pinned to
 * the reference's golden vectors.  The sums scipy's p[-1] rule reads are numpy's pairwise sums
 * (np_sum); the T sums are plain loops (last-ulp differences, far inside the 1e-10 tolerance).
 *
 * What it restates, per window, the way the reference computes it (dense grids, O(grid) work per
 * window as in twoDSFS_class.py):
 *   fixed-bp windows ............ combined_scan's loop, twoDSFS_class.py:843-949 (window start 1,
 *                                 advanced by ws * ((pos - start) // ws); empty windows emit nothing)
 *   2D SFS with the joint fold .. calculate_2d_sfs, :140-232 (fold when alt1 + alt2 > n1p + n2p,
 *                                 ties not folded; (0,0) skipped)
 *   1D SFS, fold ................ calculate_1d_sfs / fold_1d_sfs, :398-463 (raw alt counts, alt 0
 *                                 skipped, minor = min(f, 2*pop_size - f))
 *   T2D / T1D ................... calculate_likelihood_2D / _1D, :478-537, :625-684: bins[1:-1],
 *                                 None (NaN here) on N == 0 or B == 0, then
 *                                 2 * (multinomial.logpmf(x; N, x/N) - multinomial.logpmf(x; N, p_bg))
 *                                 with scipy's p[-1] <- 1 - sum(p[:-1]) when |.| > 1e-15 (NaN when
 *                                 the adjusted p is negative); the gammaln terms cancel, so
 *                                 T = 2 * sum_{x_k > 0} x_k (ln p_fg,k - ln p_bg,k)
 *   backgrounds ................. per chromosome (combined_scan, :820-841): the whole chromosome's
 *                                 folded 2D and 1D spectra
 * The stale-carry / last-window quirks (Q6, Q9) are host post-pass rules and are not restated. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int n1p, n2p, n1, n2;      /* individuals, haploid sample sizes */
  int g2;                    /* (n1 + 1) * (n2 + 1): 2D grid bins */
} Grid;

/* one SNP into the dense grids (the reference's per-SNP loop bodies) */
static void add_snp(const Grid* G, uint32_t c, int64_t* h2, int64_t* h1a, int64_t* h1b) {
  int r1 = c & 0xff, a1 = (c >> 8) & 0xff, r2 = (c >> 16) & 0xff, a2 = (int)(c >> 24);
  if (a1) h1a[a1 < G->n1 ? a1 : G->n1]++;   /* raw alt counts (alt > 2 pop_size: a KeyError there) */
  if (a2) h1b[a2 < G->n2 ? a2 : G->n2]++;
  if (a1 + a2 > G->n1p + G->n2p) { a1 = r1; a2 = r2; }
  if (a1 == 0 && a2 == 0) return;
  if (a1 > G->n1 || a2 > G->n2) return;    /* outside the grid: a ValueError there */
  h2[a1 * (G->n2 + 1) + a2]++;
}

/* numpy's float64 sum of a contiguous array (pairwise_sum, numpy/_core/src/umath/loops_utils.h.src):
 * sequential below 8, eight accumulators up to 128, halves (at a multiple of 8) above.  scipy's
 * p[-1] rule compares 1 - sum(p[:-1]) with 1e-15, so the order matters (a plain sum over 2,599
 * bins can land below -1e-15 and turn the window's T into NaN) */
static double np_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return np_sum(a, n2) + np_sum(a + n2, n - n2);
}

/* bins[1:-1] of a dense spectrum x (n bins) against background b: the CLR T, NaN for None.
 * scratch: n doubles */
static double clr(const int64_t* x, const double* lpb, double badj_lp, int n, double* scratch) {
  /* inner bins 1 .. n-2; the last inner bin takes scipy's adjusted p (badj_lp: its log, or NAN
   * when the adjustment made it negative) */
  int64_t N = 0;
  for (int k = 1; k < n - 1; ++k) N += x[k];
  if (N == 0) return NAN;
  if (isnan(badj_lp)) return NAN;
  const double lN = log((double)N);
  /* p_fg = x / N, its own last-bin adjustment */
  for (int k = 1; k < n - 1; ++k) scratch[k - 1] = (double)x[k] / (double)N;
  const double s = np_sum(scratch, n - 3);
  double pf_last = (double)x[n - 2] / (double)N;
  const double fadj = 1.0 - s;
  if (fabs(fadj) > 1e-15) pf_last = fadj;
  if (pf_last < 0.0) return NAN;
  double t = 0.0;
  for (int k = 1; k < n - 2; ++k)
    if (x[k]) t += (double)x[k] * ((log((double)x[k]) - lN) - lpb[k]);
  if (x[n - 2]) t += (double)x[n - 2] * (log(pf_last) - badj_lp);
  return 2.0 * t;
}

/* background logs over bins[1:-1] with scipy's adjustment of the last inner bin; B == 0: NaN */
static void bg_logs(const int64_t* b, int n, double* lpb, double* last_lp) {
  int64_t B = 0;
  for (int k = 1; k < n - 1; ++k) B += b[k];
  if (B == 0) { *last_lp = NAN; return; }
  double* pv = (double*)malloc(sizeof(double) * (size_t)n);
  for (int k = 1; k < n - 1; ++k) {
    const double p = (double)b[k] / (double)B;
    pv[k - 1] = p;
    lpb[k] = log(p);   /* -inf for an empty background bin: T = +inf where the window has SNPs */
  }
  const double s = np_sum(pv, n - 3);
  free(pv);
  const double adj = 1.0 - s;
  double pl = (double)b[n - 2] / (double)B;
  if (fabs(adj) > 1e-15) pl = adj;
  *last_lp = pl < 0.0 ? NAN : log(pl);
}

static void fold1(const int64_t* h, int n, int64_t* f) {   /* n = 2 pop_size: keys 0..n */
  memset(f, 0, sizeof(int64_t) * (size_t)(n / 2 + 1));
  for (int k = 0; k <= n; ++k) f[k < n - k ? k : n - k] += h[k];
}

/* Fixed-bp windows of every chromosome with per-chromosome backgrounds.  Outputs per window (in
 * scan order): chromosome, window start, SNP range [b, e), T2D, T1D_p1, T1D_p2 (NaN = None).
 * Returns 0, or -1 when cap < the number of windows (*nwin = the number needed). */
int oracle_scan_bp(const uint32_t* counts, const uint32_t* pos, const int64_t* chrom_off, int nchrom, int n1p,
                   int n2p, uint32_t ws, int nthreads, int64_t cap, int64_t* nwin, int32_t* w_chrom,
                   uint32_t* w_start, int64_t* w_b, int64_t* w_e, double* t2d, double* t1a, double* t1b) {
  Grid G;
  G.n1p = n1p; G.n2p = n2p; G.n1 = 2 * n1p; G.n2 = 2 * n2p; G.g2 = (G.n1 + 1) * (G.n2 + 1);
  /* windows (the reference's loop; sequential, cheap) */
  int64_t nw = 0;
  for (int c = 0; c < nchrom; ++c) {
    const int64_t s = chrom_off[c], e = chrom_off[c + 1];
    if (s == e) continue;
    int64_t start = 1, b = s;
    for (int64_t i = s; i < e; ++i) {
      const int64_t q = pos[i];
      if (q < start + (int64_t)ws) continue;
      if (i > b) {
        if (nw < cap) { w_chrom[nw] = c; w_start[nw] = (uint32_t)start; w_b[nw] = b; w_e[nw] = i; }
        ++nw;
      }
      start += (int64_t)ws * ((q - start) / (int64_t)ws);
      b = i;
    }
    if (nw < cap) { w_chrom[nw] = c; w_start[nw] = (uint32_t)start; w_b[nw] = b; w_e[nw] = e; }
    ++nw;
  }
  *nwin = nw;
  if (nw > cap) return -1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  /* per-chromosome backgrounds: log tables of the 2D and both folded 1D spectra */
  const int f1n = n1p + 1, f2n = n2p + 1;
  double* lp2 = (double*)malloc(sizeof(double) * (size_t)nchrom * G.g2);
  double* lpa = (double*)malloc(sizeof(double) * (size_t)nchrom * f1n);
  double* lpb = (double*)malloc(sizeof(double) * (size_t)nchrom * f2n);
  double* last = (double*)malloc(sizeof(double) * (size_t)nchrom * 3);
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < nchrom; ++c) {
    int64_t* h2 = (int64_t*)calloc((size_t)G.g2, sizeof(int64_t));
    int64_t* h1a = (int64_t*)calloc((size_t)G.n1 + 1, sizeof(int64_t));
    int64_t* h1b = (int64_t*)calloc((size_t)G.n2 + 1, sizeof(int64_t));
    int64_t* fa = (int64_t*)calloc((size_t)f1n, sizeof(int64_t));
    int64_t* fb = (int64_t*)calloc((size_t)f2n, sizeof(int64_t));
    for (int64_t i = chrom_off[c]; i < chrom_off[c + 1]; ++i) add_snp(&G, counts[i], h2, h1a, h1b);
    fold1(h1a, G.n1, fa);
    fold1(h1b, G.n2, fb);
    bg_logs(h2, G.g2, lp2 + (size_t)c * G.g2, last + 3 * c);
    bg_logs(fa, f1n, lpa + (size_t)c * f1n, last + 3 * c + 1);
    bg_logs(fb, f2n, lpb + (size_t)c * f2n, last + 3 * c + 2);
    free(h2); free(h1a); free(h1b); free(fa); free(fb);
  }
  /* windows: dense grids per window, as the reference builds them */
#pragma omp parallel
  {
    int64_t* h2 = (int64_t*)malloc(sizeof(int64_t) * (size_t)G.g2);
    int64_t* h1a = (int64_t*)malloc(sizeof(int64_t) * ((size_t)G.n1 + 1));
    int64_t* h1b = (int64_t*)malloc(sizeof(int64_t) * ((size_t)G.n2 + 1));
    int64_t* fa = (int64_t*)malloc(sizeof(int64_t) * (size_t)f1n);
    int64_t* fb = (int64_t*)malloc(sizeof(int64_t) * (size_t)f2n);
    double* scr = (double*)malloc(sizeof(double) * (size_t)G.g2);
#pragma omp for schedule(dynamic, 16)
    for (int64_t w = 0; w < nw; ++w) {
      const int c = w_chrom[w];
      memset(h2, 0, sizeof(int64_t) * (size_t)G.g2);
      memset(h1a, 0, sizeof(int64_t) * ((size_t)G.n1 + 1));
      memset(h1b, 0, sizeof(int64_t) * ((size_t)G.n2 + 1));
      for (int64_t i = w_b[w]; i < w_e[w]; ++i) add_snp(&G, counts[i], h2, h1a, h1b);
      fold1(h1a, G.n1, fa);
      fold1(h1b, G.n2, fb);
      t2d[w] = clr(h2, lp2 + (size_t)c * G.g2, last[3 * c], G.g2, scr);
      t1a[w] = clr(fa, lpa + (size_t)c * f1n, last[3 * c + 1], f1n, scr);
      t1b[w] = clr(fb, lpb + (size_t)c * f2n, last[3 * c + 2], f2n, scr);
    }
    free(h2); free(h1a); free(h1b); free(fa); free(fb); free(scr);
  }
  free(lp2); free(lpa); free(lpb); free(last);
  return 0;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
