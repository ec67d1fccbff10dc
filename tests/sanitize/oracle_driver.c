/* Sanitizer driver for the C restatement of the oracle (oracle/sfs_oracle_c.c): built with
 * -fsanitize=address,undefined together with it, scans a seeded synthetic stream (several
 * chromosomes, an empty one, a one-SNP one, missing calls) with 1 and 4 OpenMP threads, checks that
 * both agree bit for bit and prints a digest.  Test infrastructure only.  usage: oracle_driver */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_scan_bp(const uint32_t* counts, const uint32_t* pos, const int64_t* chrom_off, int nchrom, int n1p,
                   int n2p, uint32_t ws, int nthreads, int64_t cap, int64_t* nwin, int32_t* w_chrom,
                   uint32_t* w_start, int64_t* w_b, int64_t* w_e, double* t2d, double* t1a, double* t1b);

static uint64_t st = 12345;
static uint32_t rnd(void) { st = st * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(st >> 33); }

int main(void) {
  const int nchrom = 4, n1p = 9, n2p = 7;
  const int64_t len[4] = {30000, 0, 1, 12000};
  int64_t off[5] = {0};
  for (int c = 0; c < nchrom; ++c) off[c + 1] = off[c] + len[c];
  const int64_t n = off[nchrom];
  uint32_t* counts = malloc(sizeof(uint32_t) * (size_t)n);
  uint32_t* pos = malloc(sizeof(uint32_t) * (size_t)n);
  for (int c = 0; c < nchrom; ++c) {
    uint32_t q = 0;
    for (int64_t i = off[c]; i < off[c + 1]; ++i) {
      q += 1 + rnd() % 90;
      pos[i] = q;
      const uint32_t m1 = 2 * n1p - rnd() % 2, m2 = 2 * n2p - rnd() % 2;   /* a missing call now and then */
      const uint32_t a1 = rnd() % (m1 + 1), a2 = rnd() % (m2 + 1);
      counts[i] = (m1 - a1) | (a1 << 8) | ((m2 - a2) << 16) | (a2 << 24);
    }
  }
  double digest = 0.0;
  int64_t nw1 = 0;
  double* res[2][3];
  for (int t = 0; t < 2; ++t) {
    int64_t nw = 0;
    oracle_scan_bp(counts, pos, off, nchrom, n1p, n2p, 5000, 1, 0, &nw, NULL, NULL, NULL, NULL, NULL, NULL, NULL);
    int32_t* wc = malloc(sizeof(int32_t) * (size_t)nw);
    uint32_t* ws = malloc(sizeof(uint32_t) * (size_t)nw);
    int64_t* wb = malloc(sizeof(int64_t) * (size_t)nw);
    int64_t* we = malloc(sizeof(int64_t) * (size_t)nw);
    for (int k = 0; k < 3; ++k) res[t][k] = malloc(sizeof(double) * (size_t)nw);
    int64_t got = 0;
    if (oracle_scan_bp(counts, pos, off, nchrom, n1p, n2p, 5000, t ? 4 : 1, nw, &got, wc, ws, wb, we, res[t][0], res[t][1],
                       res[t][2]) != 0 || got != nw) {
      fprintf(stderr, "scan failed\n");
      return 1;
    }
    nw1 = nw;
    free(wc); free(ws); free(wb); free(we);
  }
  for (int64_t w = 0; w < nw1; ++w)
    for (int k = 0; k < 3; ++k) {
      const double a = res[0][k][w], b = res[1][k][w];
      if (!(a == b || (isnan(a) && isnan(b)))) { fprintf(stderr, "thread counts disagree at %lld\n", (long long)w); return 1; }
      if (!isnan(a)) digest += a;
    }
  printf("windows=%lld digest=%.17g\n", (long long)nw1, digest);
  for (int t = 0; t < 2; ++t) for (int k = 0; k < 3; ++k) free(res[t][k]);
  free(counts); free(pos);
  return 0;
}
