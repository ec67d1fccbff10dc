// sfs2d.hip -- MI355X (gfx950) kernels + C ABI for the windowed 2D-SFS composite-likelihood scan.
//
// Reference path (uricchio/2DSFS-scan, scripts/src/twoDSFS_class.py): for every genomic window,
// calculate_2d_sfs (140-232) + fold_1d_sfs(calculate_1d_sfs) (398-463) and the multinomial
// log-likelihood ratios calculate_likelihood_2D (625-684) / _1D (478-537) against a background SFS.
// The reference builds dense dict grids per window and calls scipy.stats.multinomial.logpmf twice.
// Here the statistic is evaluated in its sparse closed form over the bins the window touches:
//
//   T = 2 * ( sum_{k: x_k>0} x_k * (ln x_k - lp_k)  -  N ln N ),   lp_k = ln(b_k / B)
//
// (gammaln terms cancel between the two logpmf calls), with the reference's value semantics kept
// exactly: T = 0.0 exactly when x_k/N == b_k/B bitwise on every touched bin (then both logpmf
// calls return the same double), +inf when a touched bin has b_k == 0 (xlogy(x, 0) = -inf),
// NaN when scipy's p[-1] <- 1 - sum(p[:-1]) replacement makes the background's last inner
// proportion negative (emulated bit-exactly with numpy's pairwise summation order), and
// None-conditions (N == 0 or B == 0) reported through counts/flags.
//
// Kernels (all fp64 arithmetic, integer histograms):
//   k_bg_seg      one pass over SNP tiles: per-chromosome background histograms (LDS-privatised,
//                 flushed with device-scope atomics into REPL replicas) + fixed-bp window
//                 segmentation (first/last SNP of every window slot).            reads 8 B/SNP
//   k_bg_finalize one workgroup per background: replica sum, fold, B sums, proportions,
//                 log-proportion tables, numpy-exact p[-1] adjustment.          O(grid) per bg
//   k_scan        the hot loop: one wavefront (small grids) or one workgroup (large grids) per
//                 window; SNP counts streamed with coalesced dword loads; the window's 2D and two
//                 folded 1D histograms built in LDS (u16-packed 2D bins), then an atomic
//                 take-and-clear pass in which the single owner lane of each touched bin adds
//                 x*(ln x - lp_k); wavefront shuffle reductions; one 64-B record per window.
//                                                                               reads 4 B/SNP
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sfs2d.h"

namespace {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
constexpr int LNX_N = 1 << 20;  // ln(k) table for k < LNX_N (window bin counts / window totals)
constexpr int REPL = 8;        // replicas of the per-chromosome background histograms
constexpr int PW_MAX_LEAVES = 256;

enum : uint32_t { ERR_KEY = 1u, ERR_GRID = 2u };
enum : uint32_t { BGF_B2_ZERO = 1u, BGF_B1A_ZERO = 2u, BGF_B1B_ZERO = 4u, BGF_NAN2 = 8u, BGF_NAN1A = 16u, BGF_NAN1B = 32u,
                  BGF_FLOATV = 64u };

// x_k / N == b_k / B bitwise (then scipy's two logpmf calls see identical proportions and T is
// exactly 0.0).  Integer backgrounds: exact cross-multiplication (all products < 2^53, and for
// x*B < 2^52 distinct rationals cannot round to the same double); normalised backgrounds: the
// reference's own division.
__device__ __forceinline__ bool prop_ok(uint32_t x, double N, double v, double B, bool floatv) {
  return floatv ? ((double)x / N == v) : ((double)x * B == v * N);
}

struct KParams {
  int n1p, n2p, n1, n2;  // diploid sizes and haploid sample sizes
  int nb2;               // (n1+1)*(n2+1) 2D bins
  int nh;                // background histogram words per chromosome: nb2 + (n1+1) + (n2+1)
  int h1a, h1b;          // offsets of the unfolded 1D histograms inside a background histogram
  int nt;                // table entries per background: nb2 + (n1p+1) + (n2p+1)
  int t1a, t1b;          // offsets of the folded 1D tables
  int fold;
  int ann_want;          // -1: no variant_type filter
  int has_start, has_end;
  long long start_pos, end_pos;
  unsigned int ws;       // bp window size (fixed-bp) or SNPs per window
  int nchrom;
};

struct Tile {   // k_bg_seg work item: SNPs [begin, end) of one chromosome
  uint32_t chrom, begin, end, pad;
};

struct Chunk {  // k_scan work item: window slots [slot_lo, slot_hi) of one chromosome
  uint32_t chrom, kind, slot_lo, slot_hi;
  uint32_t wid_lo, pad0, pad1, pad2;
};

struct PL {     // per-bin background table entry
  double lp;    // log of the proportion scipy uses (p[-1] adjusted on the last inner bin)
  double v;     // integer backgrounds: the count b_k; normalised (float) backgrounds: p_k = b_k / B
};

struct BgHead {
  double B2, B1a, B1b;
  uint32_t flags, pad;
};

static_assert(sizeof(sfs2d_window) == 64, "window record must be 64 bytes");

// Diagnostic build only (-DSFS2D_STAMPS): wall-clock stamps (s_memrealtime, 100 MHz) of block 0 at
// phase boundaries, read back with sfs2d__debug_stamps.  The shipped library executes none.
#ifdef SFS2D_STAMPS
__device__ unsigned long long g_stamps[64];
#define STAMP(i)                                                                   \
  do {                                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[i] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------
// device helpers

__device__ __forceinline__ bool snp_pass(const KParams& P, uint32_t p, const uint16_t* ann, uint32_t i) {
  bool ok = true;
  if (P.has_start) ok &= (long long)p >= P.start_pos;   // twoDSFS_class.py:179-180
  if (P.has_end) ok &= (long long)p <= P.end_pos;       // :181-182
  if (P.ann_want >= 0) ok &= (int)ann[i] == P.ann_want;  // :185-187
  return ok;
}

// 2D bin after the joint fold (twoDSFS_class.py:197-217): -1 when skipped ((0,0) or filtered).
__device__ __forceinline__ int bin2d(const KParams& P, uint32_t c, bool pass, uint32_t& err) {
  int r1 = c & 0xff, a1 = (c >> 8) & 0xff, r2 = (c >> 16) & 0xff, a2 = c >> 24;
  int x1 = a1, x2 = a2;
  if (P.fold && a1 + a2 > P.n1p + P.n2p) { x1 = r1; x2 = r2; }
  if (!pass || (x1 | x2) == 0) return -1;
  if (x1 > P.n1 || x2 > P.n2) { err |= ERR_GRID; return -1; }
  return x1 * (P.n2 + 1) + x2;
}

// raw alt count of one population, -1 when skipped (alt == 0 or filtered) (calculate_1d_sfs:428-433)
__device__ __forceinline__ int alt_raw(int a, int n, bool pass, uint32_t& err) {
  if (!pass || a == 0) return -1;
  if (a > n) { err |= ERR_KEY; return -1; }
  return a;
}

// folded inner 1D bin: min(a, 2n - a) restricted to 1..pop_size-1 (bins[1:-1], :486-488), else -1
__device__ __forceinline__ int fold_inner(int a, int n, int np_) {
  if (a < 0) return -1;
  int f = min(a, n - a);
  return (f >= 1 && f <= np_ - 1) ? f : -1;
}

__device__ __forceinline__ uint32_t wid_of(uint32_t p, uint32_t ws) { return p ? (p - 1u) / ws : 0u; }

__device__ __forceinline__ double lnx_of(const double* lnx, uint32_t x) {
  return x < (uint32_t)LNX_N ? lnx[x] : log((double)x);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

// LDS histogram primitives: 16-bit bins packed two per dword, or plain 32-bit bins
template <bool P16>
__device__ __forceinline__ void h_add(uint32_t* h, int k) {
  if (P16) atomicAdd(&h[k >> 1], 1u << ((k & 1) << 4));
  else atomicAdd(&h[k], 1u);
}

template <bool P16>
__device__ __forceinline__ uint32_t h_take(uint32_t* h, int k) {  // read-and-clear; one lane gets x
  if (P16) {
    int sh = (k & 1) << 4;
    uint32_t old = atomicAnd(&h[k >> 1], ~(0xffffu << sh));
    return (old >> sh) & 0xffffu;
  }
  return atomicExch(&h[k], 0u);
}

template <int G>
__device__ __forceinline__ void group_sync() {
  if (G == WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

// group-wide sums; G == 256 uses a small LDS scratch of 4 waves x 8 doubles
template <int G>
__device__ __forceinline__ double group_sum_d(double v, double* red, int slot) {
  v = wave_sum_d(v);
  if (G == WAVE) return v;
  int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) red[w * 8 + slot] = v;
  __syncthreads();
  double t = red[slot] + red[8 + slot] + red[16 + slot] + red[24 + slot];
  __syncthreads();
  return t;
}

template <int G>
__device__ __forceinline__ unsigned long long group_sum_u64(unsigned long long v, unsigned long long* red, int slot) {
  v = wave_sum_u64(v);
  if (G == WAVE) return v;
  int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) red[w * 8 + slot] = v;
  __syncthreads();
  unsigned long long t = red[slot] + red[8 + slot] + red[16 + slot] + red[24 + slot];
  __syncthreads();
  return t;
}

// T from the owner-lane sum: T = 2*(S - N ln N), with the reference's special values
__device__ __forceinline__ double clr_value(double S, uint32_t N, bool prop, bool nan_bg, const double* lnx) {
  if (nan_bg) return __builtin_nan("");
  if (prop) return 0.0;
  double n = (double)N;
  return 2.0 * (S - n * lnx_of(lnx, N));
}

// ------------------------------------------------------------------------------------------
// K0: ln table

__global__ void k_init_lnx(double* lnx) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < LNX_N) lnx[i] = i ? log((double)i) : 0.0;
}

// ------------------------------------------------------------------------------------------
// K1: background histograms + fixed-bp window segmentation

constexpr int BLOCK1 = 512;   // k_bg_seg workgroup

template <bool DO_BG, bool DO_SEG, bool LDS_HIST>
__global__ __launch_bounds__(BLOCK1) void k_bg_seg(KParams P, const uint32_t* __restrict__ counts,
                                                   const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                                   const Tile* __restrict__ tiles, const long long* __restrict__ chrom_off,
                                                   const unsigned long long* __restrict__ slot_base,
                                                   uint32_t* __restrict__ repl, uint2* __restrict__ slots,
                                                   uint32_t* __restrict__ err_word) {
  extern __shared__ uint32_t sh_hist[];
  STAMP(20);
  const Tile t = tiles[blockIdx.x];
  uint32_t* gh = repl + ((size_t)(blockIdx.x % REPL) * P.nchrom + t.chrom) * (size_t)P.nh;
  uint32_t* H = LDS_HIST ? sh_hist : gh;
  if (DO_BG && LDS_HIST) {
    for (int k = threadIdx.x; k < P.nh; k += BLOCK1) sh_hist[k] = 0u;
    __syncthreads();
  }
  const long long cb = chrom_off[t.chrom], ce = chrom_off[t.chrom + 1];
  const unsigned long long sbase = DO_SEG ? slot_base[t.chrom] : 0ull;
  const bool pos_filter = P.has_start || P.has_end;
  const bool need_pos = DO_SEG || pos_filter;
  const int lane = threadIdx.x & (WAVE - 1);
  uint32_t err = 0;

  // one 16-B vector = 4 consecutive SNPs; elements outside [t.begin, t.end) are masked
  auto process = [&](uint32_t i0, const uint4& cv, const uint4& pv, uint32_t pprev, uint32_t pnext) {
    const uint32_t cc[4] = {cv.x, cv.y, cv.z, cv.w};
    const uint32_t pp[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = i0 + k;
      if (i < t.begin || i >= t.end) continue;
      const uint32_t c = cc[k];
      const uint32_t p = pp[k];
      if (DO_BG) {
        bool pass = true;
        if (pos_filter) pass = snp_pass(P, p, ann, i);
        else if (P.ann_want >= 0) pass = (int)ann[i] == P.ann_want;
        const int k2 = bin2d(P, c, pass, err);
        const int a1 = alt_raw((c >> 8) & 0xff, P.n1, pass, err);
        const int a2 = alt_raw(c >> 24, P.n2, pass, err);
        if (k2 >= 0) atomicAdd(&H[k2], 1u);
        if (a1 >= 0) atomicAdd(&H[P.h1a + a1], 1u);
        if (a2 >= 0) atomicAdd(&H[P.h1b + a2], 1u);
      }
      if (DO_SEG) {
        // window id (pos-1)//ws: the reference's start += ws*((pos-start)//ws) from start=1 (:894, :948)
        const uint32_t w = wid_of(p, P.ws);
        const uint32_t qp = k ? pp[k - 1] : pprev;
        const uint32_t qn = k < 3 ? pp[k + 1] : pnext;
        const bool first = ((long long)i == cb) || (wid_of(qp, P.ws) != w);
        const bool last = ((long long)i + 1 == ce) || (wid_of(qn, P.ws) != w);
        const unsigned long long s = sbase + w;
        if (first) slots[s].x = i + 1u;  // 0 = unset; the scan kernel clears what it consumed
        if (last) slots[s].y = i + 1u;
      }
    }
  };
  // neighbours of a vector's first / last SNP: from the adjacent lanes, else from memory
  auto neighbours = [&](uint32_t i0, const uint4& pv, uint32_t& pprev, uint32_t& pnext) {
    pprev = __shfl_up(pv.w, 1, WAVE);
    pnext = __shfl_down(pv.x, 1, WAVE);
    if (lane == 0 && (long long)i0 > cb && i0 > 0) pprev = pos[i0 - 1];
    if ((lane == WAVE - 1 || i0 + 4 >= t.end) && (long long)i0 + 4 < ce) pnext = pos[i0 + 4];
  };

  STAMP(21);
  // two vectors per thread in flight per step (8 SNPs, 32 B of counts + positions)
  constexpr uint32_t STEP = 8 * BLOCK1;
  const uint32_t ab = t.begin & ~3u;
  for (uint32_t base = ab; base < t.end; base += STEP) {
    const uint32_t ia = base + 4 * threadIdx.x, ib = ia + 4 * BLOCK1;
    const bool la = ia < t.end, lb = ib < t.end;
    const uint4 ca = la ? *reinterpret_cast<const uint4*>(counts + ia) : make_uint4(0, 0, 0, 0);
    const uint4 cbv = lb ? *reinterpret_cast<const uint4*>(counts + ib) : make_uint4(0, 0, 0, 0);
    const uint4 pa = (need_pos && la) ? *reinterpret_cast<const uint4*>(pos + ia) : make_uint4(0, 0, 0, 0);
    const uint4 pb = (need_pos && lb) ? *reinterpret_cast<const uint4*>(pos + ib) : make_uint4(0, 0, 0, 0);
    uint32_t pva = 0, pna = 0, pvb = 0, pnb = 0;
    if (DO_SEG) {
      neighbours(ia, pa, pva, pna);
      neighbours(ib, pb, pvb, pnb);
    }
    process(ia, ca, pa, pva, pna);
    process(ib, cbv, pb, pvb, pnb);
  }
  STAMP(22);
  if (err) atomicOr(err_word, err);
  if (DO_BG && LDS_HIST) {
    __syncthreads();
    for (int k = threadIdx.x; k < P.nh; k += BLOCK1) {
      const uint32_t v = sh_hist[k];
      if (v) atomicAdd(&gh[k], v);
    }
  }
  STAMP(23);
}

// ------------------------------------------------------------------------------------------
// K2: background tables.  One workgroup per background.

// numpy pairwise_sum leaf (numpy/_core/src/umath/loops_utils.h.src): n < 8 sequential from 0.0,
// n <= 128: eight strided accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) + tail.
// `a` is a generic pointer (LDS or global), element i at a[i * stride].
__device__ double np_leaf_sum(const double* a, int stride, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i * stride];
    return r;
  }
  double r0 = a[0], r1 = a[stride], r2 = a[2 * stride], r3 = a[3 * stride];
  double r4 = a[4 * stride], r5 = a[5 * stride], r6 = a[6 * stride], r7 = a[7 * stride];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    const double* q = a + (size_t)i * stride;
    r0 += q[0]; r1 += q[stride]; r2 += q[2 * stride]; r3 += q[3 * stride];
    r4 += q[4 * stride]; r5 += q[5 * stride]; r6 += q[6 * stride]; r7 += q[7 * stride];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[(size_t)i * stride];
  return res;
}

constexpr int FBLOCK = 1024;            // k_bg_finalize workgroup
constexpr int FIN_LDS_BINS = 12288;     // backgrounds with nt <= this keep values / proportions in LDS

// One workgroup per background.  from_repl: per-chromosome background from the k_bg_seg replicas
// (summed, folded, and cleared for the next run); else bgval was uploaded (supplied background).
// The values v, then the proportions p (overwriting v), live in LDS when they fit.
__global__ __launch_bounds__(FBLOCK) void k_bg_finalize(KParams P, int from_repl, int integer_values,
                                                        uint32_t* __restrict__ repl, double* __restrict__ bgval,
                                                        PL* __restrict__ tab, BgHead* __restrict__ head,
                                                        const int2* __restrict__ pw_leaves, int pw_nleaves,
                                                        const short* __restrict__ pw_prog, int pw_nprog) {
  extern __shared__ double v_lds[];
  __shared__ double red[3][FBLOCK / WAVE];
  __shared__ uint32_t u1[2 * 256 + 2];
  __shared__ double leafsum[PW_MAX_LEAVES];
  __shared__ short prog_s[2 * PW_MAX_LEAVES];
  __shared__ double padj1[2];
  __shared__ double pw_stack[32];
  __shared__ double Bs[3];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const bool in_lds = P.nt <= FIN_LDS_BINS;
  double* gv = bgval + (size_t)b * P.nt;
  double* V = in_lds ? v_lds : gv;
  PL* T = tab + (size_t)b * P.nt;

  STAMP(0);
  for (int i = tid; i < pw_nprog; i += FBLOCK) prog_s[i] = pw_prog[i];
  if (from_repl) {
    // replica sum with all REPL loads of a bin in flight; 1D spectra are folded:
    // folded[f] = u[f] + u[2n - f] (f < n), folded[n] = u[n] (fold_1d_sfs, :446-463)
    const size_t rstride = (size_t)P.nchrom * P.nh;
    for (int k = tid; k < P.nh; k += FBLOCK) {
      uint32_t* q = repl + (size_t)b * P.nh + k;
      uint32_t x[REPL];
#pragma unroll
      for (int r = 0; r < REPL; ++r) x[r] = q[r * rstride];
      uint32_t s = 0;
#pragma unroll
      for (int r = 0; r < REPL; ++r) { s += x[r]; if (x[r]) q[r * rstride] = 0u; }
      if (k < P.nb2) V[k] = (double)s;
      else u1[k - P.nb2] = s;
    }
    __syncthreads();
    for (int f = tid; f <= P.n1p; f += FBLOCK)
      V[P.t1a + f] = (double)u1[f] + (f < P.n1p ? (double)u1[P.n1 - f] : 0.0);
    for (int f = tid; f <= P.n2p; f += FBLOCK)
      V[P.t1b + f] = (double)u1[(P.n1 + 1) + f] + (f < P.n2p ? (double)u1[(P.n1 + 1) + P.n2 - f] : 0.0);
  } else if (in_lds) {
    for (int k = tid; k < P.nt; k += FBLOCK) V[k] = gv[k];
  }
  __syncthreads();

  STAMP(1);
  // inner sums B over bins[1:-1]: exact for integer values in any order; for normalised
  // (float) values the reference's builtin sum() is sequential, so one lane adds in order.
  const int M2 = P.nb2 - 2, M1a = P.n1p - 1, M1b = P.n2p - 1;
  if (integer_values) {
    double s2 = 0.0, sa = 0.0, sb = 0.0;
    for (int k = tid; k < M2; k += FBLOCK) s2 += V[1 + k];
    for (int k = tid; k < M1a; k += FBLOCK) sa += V[P.t1a + 1 + k];
    for (int k = tid; k < M1b; k += FBLOCK) sb += V[P.t1b + 1 + k];
    s2 = wave_sum_d(s2); sa = wave_sum_d(sa); sb = wave_sum_d(sb);
    if ((tid & (WAVE - 1)) == 0) {
      red[0][tid / WAVE] = s2; red[1][tid / WAVE] = sa; red[2][tid / WAVE] = sb;
    }
    __syncthreads();
    if (tid < 3) {
      double t = 0.0;
      for (int w = 0; w < FBLOCK / WAVE; ++w) t += red[tid][w];
      Bs[tid] = t;
    }
  } else if (tid == 0) {
    double s2 = 0.0, sa = 0.0, sb = 0.0;
    for (int k = 0; k < M2; ++k) s2 += V[1 + k];
    for (int k = 0; k < M1a; ++k) sa += V[P.t1a + 1 + k];
    for (int k = 0; k < M1b; ++k) sb += V[P.t1b + 1 + k];
    Bs[0] = s2; Bs[1] = sa; Bs[2] = sb;
  }
  __syncthreads();
  const double B2 = Bs[0], B1a = Bs[1], B1b = Bs[2];
  STAMP(2);

  // proportions p = v / B (Python true division == IEEE division here) and their logs; p
  // overwrites v for the pairwise p[:-1] sums below
  for (int k = tid; k < P.nt; k += FBLOCK) {
    const double B = k < P.nb2 ? B2 : (k < P.t1b ? B1a : B1b);
    const double val = V[k];
    const double p = (B != 0.0) ? val / B : 0.0;
    PL e;
    e.lp = log(p);
    e.v = integer_values ? val : p;
    T[k] = e;
    V[k] = p;
  }
  __syncthreads();
  STAMP(3);

  // scipy multinomial._process_parameters: p[-1] <- 1 - sum(p[:-1]) when |.| > 1e-15, and the
  // whole logpmf is NaN if any p < 0.  sum(p[:-1]) is numpy's pairwise sum over the inner bins
  // except the last: the 2D tree plan (leaves + postfix program) comes from the host.
  if (tid < pw_nleaves) {
    const int2 lf = pw_leaves[tid];
    leafsum[tid] = np_leaf_sum(V + 1 + lf.x, 1, lf.y);
  } else if (tid == PW_MAX_LEAVES && M1a >= 1) {
    padj1[0] = 1.0 - np_leaf_sum(V + P.t1a + 1, 1, M1a - 1);
  } else if (tid == PW_MAX_LEAVES + WAVE && M1b >= 1) {
    padj1[1] = 1.0 - np_leaf_sum(V + P.t1b + 1, 1, M1b - 1);
  }
  __syncthreads();
  STAMP(4);
  if (tid == 0) {
    uint32_t flags = integer_values ? 0u : BGF_FLOATV;
    if (B2 == 0.0) flags |= BGF_B2_ZERO;
    if (B1a == 0.0) flags |= BGF_B1A_ZERO;
    if (B1b == 0.0) flags |= BGF_B1B_ZERO;
    if (M2 >= 1 && B2 != 0.0) {
      // postfix evaluation; the stack lives in LDS (a runtime-indexed private array would be scratch)
      int sp = 0;
      for (int i = 0; i < pw_nprog; ++i) {
        const short op = prog_s[i];
        if (op >= 0) pw_stack[sp++] = leafsum[op];
        else { const double r = pw_stack[--sp]; pw_stack[sp - 1] = pw_stack[sp - 1] + r; }
      }
      const double S = sp ? pw_stack[0] : 0.0;
      const double padj = 1.0 - S;
      if (padj < -1e-15) flags |= BGF_NAN2;
      else if (fabs(padj) > 1e-15) T[1 + M2 - 1].lp = log(padj);
    }
    if (M1a >= 1 && B1a != 0.0) {
      const double padj = padj1[0];
      if (padj < -1e-15) flags |= BGF_NAN1A;
      else if (fabs(padj) > 1e-15) T[P.t1a + M1a].lp = log(padj);
    }
    if (M1b >= 1 && B1b != 0.0) {
      const double padj = padj1[1];
      if (padj < -1e-15) flags |= BGF_NAN1B;
      else if (fabs(padj) > 1e-15) T[P.t1b + M1b].lp = log(padj);
    }
    BgHead h;
    h.B2 = B2; h.B1a = B1a; h.B1b = B1b; h.flags = flags; h.pad = 0;
    head[b] = h;
    STAMP(5);
  }
}

// ------------------------------------------------------------------------------------------
// K3: the window scan

struct WinOut {
  uint32_t snp_count, n2, n2_all, n1a, n1b;
  double t2d, t1a, t1b;
};

// Evaluate one window [begin, end) against background `bg` with a group of G lanes.
// H2: 2D histogram (u16-packed when P16), H1: two folded 1D histograms (u32).
template <int G, bool P16>
__device__ __forceinline__ WinOut eval_window(const KParams& P, const uint32_t* __restrict__ counts,
                                              const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                              uint32_t begin, uint32_t end, const PL* __restrict__ T,
                                              const BgHead& hb, const double* __restrict__ lnx, uint32_t* H2,
                                              uint32_t* H1, double* redd, unsigned long long* redu,
                                              uint32_t& err) {
  const int lane = threadIdx.x & (G - 1);
  const bool need_pos = P.has_start || P.has_end;
  const int last2 = P.nb2 - 1;   // bin (n1, n2): counted in n2_all, excluded from T2D (bins[1:-1])
  uint32_t* H1a = H1;
  uint32_t* H1b = H1 + (P.n1p + 1);
  const PL* T2 = T;
  const PL* T1a = T + P.t1a;
  const PL* T1b = T + P.t1b;

  // ---- phase A: histogram the window
  uint32_t c_var = 0, c2 = 0, c2all = 0, c1a = 0, c1b = 0;
  for (uint32_t i = begin + lane; i < end; i += G) {
    const uint32_t c = counts[i];
    const uint32_t p = need_pos ? pos[i] : 0u;
    const bool var_ok = P.ann_want < 0 || (int)ann[i] == P.ann_want;
    const bool pass = var_ok && (!need_pos || snp_pass(P, p, ann, i));
    c_var += var_ok;
    const int k2 = bin2d(P, c, pass, err);
    const int f1 = fold_inner(alt_raw((c >> 8) & 0xff, P.n1, pass, err), P.n1, P.n1p);
    const int f2 = fold_inner(alt_raw(c >> 24, P.n2, pass, err), P.n2, P.n2p);
    if (k2 >= 0) {
      ++c2all;
      if (k2 != last2) { ++c2; h_add<P16>(H2, k2); }
    }
    if (f1 >= 0) { ++c1a; atomicAdd(&H1a[f1], 1u); }
    if (f2 >= 0) { ++c1b; atomicAdd(&H1b[f2], 1u); }
  }
  group_sync<G>();
  const unsigned long long r0 = group_sum_u64<G>((unsigned long long)c2 | ((unsigned long long)c2all << 32), redu, 0);
  const unsigned long long r1 = group_sum_u64<G>((unsigned long long)c1a | ((unsigned long long)c1b << 32), redu, 1);
  const unsigned long long r2 = group_sum_u64<G>((unsigned long long)c_var, redu, 2);
  WinOut o;
  o.n2 = (uint32_t)r0; o.n2_all = (uint32_t)(r0 >> 32);
  o.n1a = (uint32_t)r1; o.n1b = (uint32_t)(r1 >> 32);
  o.snp_count = (uint32_t)r2;
  const double N2 = (double)o.n2, N1a = (double)o.n1a, N1b = (double)o.n1b;

  // ---- phase B: take-and-clear; the owner lane of each touched bin adds x*(ln x - lp_k)
  double s2 = 0.0, sa = 0.0, sb = 0.0;
  bool q2 = true, qa = true, qb = true;   // x_k/N == p_k bitwise on every touched bin
  for (uint32_t i = begin + lane; i < end; i += G) {
    const uint32_t c = counts[i];
    const uint32_t p = need_pos ? pos[i] : 0u;
    const bool pass = (P.ann_want < 0 || (int)ann[i] == P.ann_want) && (!need_pos || snp_pass(P, p, ann, i));
    uint32_t e2 = 0;
    const int k2 = bin2d(P, c, pass, e2);
    const int f1 = fold_inner(alt_raw((c >> 8) & 0xff, P.n1, pass, e2), P.n1, P.n1p);
    const int f2 = fold_inner(alt_raw(c >> 24, P.n2, pass, e2), P.n2, P.n2p);
    if (k2 >= 0 && k2 != last2) {
      const uint32_t x = h_take<P16>(H2, k2);
      if (x) {
        const PL t = T2[k2];
        s2 += (double)x * (lnx_of(lnx, x) - t.lp);
        q2 &= prop_ok(x, N2, t.v, hb.B2, hb.flags & BGF_FLOATV);
      }
    }
    if (f1 >= 0) {
      const uint32_t x = atomicExch(&H1a[f1], 0u);
      if (x) {
        const PL t = T1a[f1];
        sa += (double)x * (lnx_of(lnx, x) - t.lp);
        qa &= prop_ok(x, N1a, t.v, hb.B1a, hb.flags & BGF_FLOATV);
      }
    }
    if (f2 >= 0) {
      const uint32_t x = atomicExch(&H1b[f2], 0u);
      if (x) {
        const PL t = T1b[f2];
        sb += (double)x * (lnx_of(lnx, x) - t.lp);
        qb &= prop_ok(x, N1b, t.v, hb.B1b, hb.flags & BGF_FLOATV);
      }
    }
  }
  s2 = group_sum_d<G>(s2, redd, 0);
  sa = group_sum_d<G>(sa, redd, 1);
  sb = group_sum_d<G>(sb, redd, 2);
  const unsigned long long qbits = group_sum_u64<G>((unsigned long long)(!q2) | ((unsigned long long)(!qa) << 21) |
                                                    ((unsigned long long)(!qb) << 42), redu, 3);
  const bool all2 = (qbits & 0x1fffffull) == 0, alla = ((qbits >> 21) & 0x1fffffull) == 0,
             allb = (qbits >> 42) == 0;
  o.t2d = clr_value(s2, o.n2, all2, hb.flags & BGF_NAN2, lnx);
  o.t1a = clr_value(sa, o.n1a, alla, hb.flags & BGF_NAN1A, lnx);
  o.t1b = clr_value(sb, o.n1b, allb, hb.flags & BGF_NAN1B, lnx);
  return o;
}

__device__ __forceinline__ uint32_t bg_zero_flags(const BgHead& hb) {
  return ((hb.flags & BGF_B2_ZERO) ? SFS2D_W_BG2_ZERO : 0u) | ((hb.flags & BGF_B1A_ZERO) ? SFS2D_W_BG1A_ZERO : 0u) |
         ((hb.flags & BGF_B1B_ZERO) ? SFS2D_W_BG1B_ZERO : 0u);
}

__device__ __forceinline__ void write_rec(sfs2d_window* o, uint32_t chrom, uint32_t wid, uint32_t b, uint32_t e,
                                          const WinOut& w, uint32_t flags) {
  sfs2d_window r;
  r.chrom = chrom; r.wid = wid; r.begin = b; r.end = e;
  r.snp_count = w.snp_count; r.n2 = w.n2; r.n2_all = w.n2_all; r.n1a = w.n1a; r.n1b = w.n1b;
  r.flags = flags;
  r.t2d = w.t2d; r.t1d_p1 = w.t1a; r.t1d_p2 = w.t1b;
  *o = r;
}

// first index j in [cb, e) such that SNPs j..e-1 share the fixed-bp window of SNP e-1.
// Wave-level (every wave of the group computes the same answer).
__device__ uint32_t window_begin_back(const uint32_t* __restrict__ pos, long long cb, uint32_t e, uint32_t ws) {
  const int lane = threadIdx.x & (WAVE - 1);
  const uint32_t w = wid_of(pos[e - 1], ws);
  long long hi = (long long)e - 1;   // pos[hi] is in the window
  while (true) {
    const long long j = hi - 1 - lane;
    const bool out = (j < cb) || (wid_of(pos[j], ws) != w);
    const unsigned long long m = __ballot(out);
    if (m) return (uint32_t)(hi - __builtin_ctzll(m));
    hi -= WAVE;
  }
}

// Per-element bins of the window's first 512 SNPs, kept in registers between the two phases:
// bits 0-15 inner 2D bin (0xffff none), 16-23 / 24-31 folded inner 1D bins (0xff none).
__device__ __forceinline__ uint32_t pack_bins(int k2, int f1, int f2) {
  return (uint32_t)(k2 < 0 ? 0xffff : k2) | ((uint32_t)(f1 < 0 ? 0xff : f1) << 16) |
         ((uint32_t)(f2 < 0 ? 0xff : f2) << 24);
}

template <int G, bool P16>
__global__ __launch_bounds__(BLOCK) void k_scan(KParams P, const uint32_t* __restrict__ counts,
                                                const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                                const Chunk* __restrict__ chunks, const long long* __restrict__ chrom_off,
                                                uint2* __restrict__ slots, const PL* __restrict__ tab,
                                                const BgHead* __restrict__ head, int bg_per_chrom,
                                                const double* __restrict__ lnx, sfs2d_window* __restrict__ out,
                                                uint32_t* __restrict__ err_word, int mode_bp, long long extra_rec) {
  extern __shared__ uint32_t lds[];
  constexpr int NG = BLOCK / G;
  const int g = threadIdx.x / G;
  const int lane = threadIdx.x & (G - 1);
  const int h2w = P16 ? (P.nb2 + 1) / 2 : P.nb2;
  const int h1w = (P.n1p + 1) + (P.n2p + 1);
  const int per = h2w + h1w;
  uint32_t* H2 = lds + g * per;
  uint32_t* H1 = H2 + h2w;
  double* redd = reinterpret_cast<double*>(lds + NG * per + ((NG * per) & 1));
  unsigned long long* redu = reinterpret_cast<unsigned long long*>(redd + 32);

  for (int k = lane; k < per; k += G) H2[k] = 0u;
  group_sync<G>();

  const Chunk ch = chunks[blockIdx.x];
  uint32_t err = 0;
  const long long cb = chrom_off[ch.chrom];
  const PL* T = tab + (bg_per_chrom ? (size_t)ch.chrom * P.nt : 0);
  const BgHead hb = head[bg_per_chrom ? ch.chrom : 0];

  if (ch.kind == 0) {
    for (uint32_t s = ch.slot_lo + g; s < ch.slot_hi; s += NG) {
      const uint32_t wid = ch.wid_lo + (s - ch.slot_lo);
      uint32_t b, e;
      if (mode_bp) {
        const uint2 sr = slots[s];
        if (sr.x == 0u) {   // empty fixed-bp slot
          if (lane == 0) {
            sfs2d_window r;
            memset(&r, 0, sizeof(r));
            r.chrom = ch.chrom; r.wid = wid; r.flags = SFS2D_W_EMPTY;
            out[s] = r;
          }
          continue;
        }
        b = sr.x - 1u;
        e = sr.y;
      } else {
        b = (uint32_t)(cb + (long long)wid * P.ws);
        e = b + P.ws;
      }
      const WinOut w = eval_window<G, P16>(P, counts, pos, ann, b, e, T, hb, lnx, H2, H1, redd, redu, err);
      if (lane == 0) {
        write_rec(out + s, ch.chrom, wid, b, e, w, bg_zero_flags(hb));
        if (mode_bp) slots[s] = make_uint2(0u, 0u);   // leave the slot table clean for the next run
      }
    }
  }
  if (err) atomicOr(err_word, err);
}

// ------------------------------------------------------------------------------------------
// K3 (small grids): one wavefront per window, windows software-pipelined.
//
// Per window: the first 512 SNPs arrive as two 16-B loads per lane (issued while the previous
// window finishes), their bins are kept in registers (pack_bins) between the histogram pass and
// the take pass, longer windows stream further 512-SNP chunks.  In the take pass every lane
// gathers table entries and ln x for all its elements at once (no load behind a branch), then
// the owner lanes accumulate.  Counts come from ballots; only three fp64 sums are reduced.

struct Win {
  uint32_t b, e;
  uint4 v0, v1;   // first chunk (SNPs [b & ~3, +512))
  bool has;
};

__device__ __forceinline__ uint4 ld4(const uint32_t* __restrict__ a, uint32_t i, uint32_t e) {
  return i < e ? *reinterpret_cast<const uint4*>(a + i) : make_uint4(0, 0, 0, 0);
}

// Branch-free classification of one SNP (same rules as bin2d / alt_raw / fold_inner).
struct Cls {
  int k2, g1, g2;          // 2D bin, folded 1D bins
  bool v2, in2, v1a, v1b;  // inner 2D bin / any 2D bin (incl. (n1,n2)) / inner folded 1D bins
};

__device__ __forceinline__ Cls classify_bf(const KParams& P, uint32_t c, bool pass, uint32_t& err) {
  const int r1 = c & 0xff, a1 = (c >> 8) & 0xff, r2 = (c >> 16) & 0xff, a2 = c >> 24;
  const bool sw = P.fold & (a1 + a2 > P.n1p + P.n2p);
  const int x1 = sw ? r1 : a1, x2 = sw ? r2 : a2;
  const bool nz = (x1 | x2) != 0;
  const bool oob = (x1 > P.n1) | (x2 > P.n2);
  const bool ka = a1 > P.n1, kb = a2 > P.n2;
  err |= (pass & nz & oob) ? ERR_GRID : 0u;
  err |= (pass & (ka | kb)) ? ERR_KEY : 0u;
  Cls r;
  r.k2 = x1 * (P.n2 + 1) + x2;
  r.in2 = pass & nz & !oob;
  r.v2 = r.in2 & (r.k2 != P.nb2 - 1);
  r.g1 = min(a1, P.n1 - a1);
  r.g2 = min(a2, P.n2 - a2);
  r.v1a = pass & (a1 != 0) & !ka & (r.g1 >= 1) & (r.g1 <= P.n1p - 1);
  r.v1b = pass & (a2 != 0) & !kb & (r.g2 >= 1) & (r.g2 <= P.n2p - 1);
  return r;
}

// Take pass over 8 elements for histogram h (0: 2D, 1: pop1 1D, 2: pop2 1D): LDS take-and-clear
// (skipped elements hit the lane's private trash word), then every table / ln-x gather is issued
// before any is used.  Called in a runtime loop over h so that only one histogram's 8 gathers are
// live at a time (the compiler otherwise interleaves all three and runs out of registers).
template <bool P16>
__device__ __forceinline__ double take_accumulate(int h, const uint32_t (&bins)[8], uint32_t* W, uint32_t trash,
                                                  int toff, const PL* __restrict__ T, const double* __restrict__ lnx) {
  const uint32_t shift = h == 0 ? 0u : (h == 1 ? 16u : 24u);
  const uint32_t msk = h == 0 ? 0xffffu : 0xffu;
  uint32_t x[8];
  int kk[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t k = (bins[j] >> shift) & msk;
    const bool valid = k != msk;
    uint32_t xv;
    if (P16 && h == 0) {
      const uint32_t sh = (k & 1) << 4;
      const uint32_t old = atomicAnd(&W[valid ? (k >> 1) : trash], valid ? ~(0xffffu << sh) : 0u);
      xv = valid ? (old >> sh) & 0xffffu : 0u;
    } else {
      const uint32_t old = atomicExch(&W[valid ? (uint32_t)toff + k : trash], 0u);
      xv = valid ? old : 0u;
    }
    x[j] = xv;
    kk[j] = xv ? (int)k : 0;
  }
  double lp[8], lx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lp[j] = T[kk[j]].lp;
    lx[j] = lnx[x[j]];          // x < LNX_N: windows of >= LNX_N SNPs take the exact path
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += x[j] ? (double)x[j] * (lx[j] - lp[j]) : 0.0;
  return s;
}

// |T| this small may be an exactly proportional window (reference: T == 0.0 exactly, which its
// truthiness guard reads as False): such windows are re-evaluated with the exact bin-by-bin test.
__device__ __forceinline__ bool suspect_zero(double S, uint32_t N, const double* lnx) {
  const double n = (double)N;
  return N && fabs(2.0 * (S - n * lnx[N])) <= 1e-9 * (n + 1.0);
}

__device__ __forceinline__ double clr_fast(double S, uint32_t N, bool nan_bg, const double* lnx) {
  return nan_bg ? __builtin_nan("") : 2.0 * (S - (double)N * lnx[N]);
}

constexpr int TRASH = WAVE;   // lane-private scratch words after each wave's histograms

template <bool P16>
__global__ __launch_bounds__(BLOCK) void k_scan_w(KParams P, const uint32_t* __restrict__ counts,
                                                  const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                                  const Chunk* __restrict__ chunks, const long long* __restrict__ chrom_off,
                                                  uint2* __restrict__ slots, const PL* __restrict__ tab,
                                                  const BgHead* __restrict__ head, int bg_per_chrom,
                                                  const double* __restrict__ lnx, sfs2d_window* __restrict__ out,
                                                  uint32_t* __restrict__ err_word, int mode_bp) {
  extern __shared__ uint32_t lds[];
  STAMP(10);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & (WAVE - 1);
  const int h2w = P16 ? (P.nb2 + 1) / 2 : P.nb2;
  const int core = h2w + (P.n1p + 1) + (P.n2p + 1);
  uint32_t* W = lds + wv * (core + TRASH);    // [2D bins | 1D pop1 | 1D pop2 | trash x 64]
  const int t1a = h2w, t1b = h2w + P.n1p + 1;
  const uint32_t trash = (uint32_t)(core + lane);
  for (int k = lane; k < core + TRASH; k += WAVE) W[k] = 0u;

  const Chunk ch = chunks[blockIdx.x];
  const long long cb = chrom_off[ch.chrom];
  const PL* T = tab + (bg_per_chrom ? (size_t)ch.chrom * P.nt : 0);
  const BgHead hb = head[bg_per_chrom ? ch.chrom : 0];
  const bool filt = P.ann_want >= 0 || P.has_start || P.has_end;
  const bool posf = P.has_start || P.has_end;
  const uint32_t zflags = bg_zero_flags(hb);
  uint32_t err = 0;
  group_sync<WAVE>();

  auto bounds = [&](uint32_t s, uint2 sr, Win& w) {
    if (mode_bp) {
      w.has = sr.x != 0u;
      w.b = sr.x - 1u;
      w.e = sr.y;
    } else {
      w.has = true;
      w.b = (uint32_t)(cb + (long long)(ch.wid_lo + (s - ch.slot_lo)) * P.ws);
      w.e = w.b + P.ws;
    }
    if (w.has) {
      const uint32_t i0 = (w.b & ~3u) + 4 * lane;
      w.v0 = ld4(counts, i0, w.e);
      w.v1 = ld4(counts, i0 + 4 * WAVE, w.e);
    }
  };
  // element -> (pass, variant ok); filters read ann / pos at a clamped (always valid) index
  auto passes = [&](uint32_t i, const Win& w, bool& var_ok) -> bool {
    const bool valid = (i >= w.b) & (i < w.e);
    var_ok = valid;
    if (!filt) return valid;
    const uint32_t ic = min(max(i, w.b), w.e - 1);
    var_ok = valid & ((P.ann_want < 0) | ((int)ann[ic] == P.ann_want));
    bool ok = var_ok;
    if (posf) {
      const long long p = (long long)pos[ic];
      ok = ok & (!P.has_start | (p >= P.start_pos)) & (!P.has_end | (p <= P.end_pos));
    }
    return ok;
  };

  uint32_t s = ch.slot_lo + wv;
  if (s >= ch.slot_hi) return;
  Win cur;
  STAMP(11);
  bounds(s, mode_bp ? slots[s] : make_uint2(0, 0), cur);
  int it = 0;
  for (; s < ch.slot_hi; s += BLOCK / WAVE, ++it) {
    const uint32_t sn = s + BLOCK / WAVE;
    const bool more = sn < ch.slot_hi;
    const uint2 srn = (mode_bp && more) ? slots[sn] : make_uint2(0, 0);
    const uint32_t wid = ch.wid_lo + (s - ch.slot_lo);
    uint32_t nvar = 0, nlast = 0, n2 = 0, n1a = 0, n1b = 0;
    uint32_t kb[8];
    const uint32_t a0 = cur.b & ~3u;
    if (cur.has) {
      // ---- histogram pass
      for (uint32_t base = a0; base < cur.e; base += 8 * WAVE) {
        const uint32_t i0 = base + 4 * lane, i1 = i0 + 4 * WAVE;
        const uint4 c0 = base == a0 ? cur.v0 : ld4(counts, i0, cur.e);
        const uint4 c1 = base == a0 ? cur.v1 : ld4(counts, i1, cur.e);
        const uint32_t cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t i = (j < 4 ? i0 : i1) + (j & 3);
          bool var_ok;
          const bool pass = passes(i, cur, var_ok);
          const Cls r = classify_bf(P, cc[j], pass, err);
          if (filt) nvar += __popcll(__ballot(var_ok));
          if (!P.fold) nlast += __popcll(__ballot(r.in2 & !r.v2));
          n2 += __popcll(__ballot(r.v2));
          if (base == a0) kb[j] = r.v2 ? (uint32_t)r.k2 : 0xffffu;
          if (P16) atomicAdd(&W[r.v2 ? (uint32_t)(r.k2 >> 1) : trash], 1u << ((r.k2 & 1) << 4));
          else atomicAdd(&W[r.v2 ? (uint32_t)r.k2 : trash], 1u);
          atomicAdd(&W[r.v1a ? (uint32_t)(t1a + r.g1) : trash], 1u);
          atomicAdd(&W[r.v1b ? (uint32_t)(t1b + r.g2) : trash], 1u);
          __builtin_amdgcn_sched_barrier(0);   // one element at a time: keeps its lane masks short-lived
        }
      }
    }
    if (it == 0) STAMP(12);
    // next window: slot record is in, issue its first chunk now (overlaps the take pass)
    Win nxt;
    nxt.has = false;
    if (more) bounds(sn, srn, nxt);
    if (cur.has) {
      group_sync<WAVE>();
      if (!filt) nvar = cur.e - cur.b;
      double s2 = 0.0, sa = 0.0, sb = 0.0;
      for (uint32_t base = a0; base < cur.e; base += 8 * WAVE) {
        uint32_t bins[8];
        if (base == a0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bins[j] = kb[j];
        } else {
          const uint32_t i0 = base + 4 * lane, i1 = i0 + 4 * WAVE;
          const uint4 c0 = ld4(counts, i0, cur.e), c1 = ld4(counts, i1, cur.e);
          const uint32_t cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
          uint32_t e2 = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t i = (j < 4 ? i0 : i1) + (j & 3);
            bool var_ok;
            const Cls r = classify_bf(P, cc[j], passes(i, cur, var_ok), e2);
            bins[j] = r.v2 ? (uint32_t)r.k2 : 0xffffu;
          }
        }
        s2 += take_accumulate<P16>(0, bins, W, trash, 0, T, lnx);
      }
      // the folded 1D spectra have pop_size-1 inner bins: one lane per bin reads and clears it
      auto bin_pass = [&](int toff, int np_, const PL* Th, uint32_t& N) -> double {
        double acc = 0.0;
        uint32_t cnt = 0;
        for (int k = 1 + lane; k <= np_ - 1; k += WAVE) {
          const uint32_t x = W[toff + k];
          W[toff + k] = 0u;
          const double lp = Th[x ? k : 0].lp;
          acc += x ? (double)x * (lnx[x] - lp) : 0.0;
          cnt += x;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, WAVE);
        N = cnt;
        return wave_sum_d(acc);
      };
      if (it == 0) STAMP(13);
      sa = bin_pass(t1a, P.n1p, T + P.t1a, n1a);
      sb = bin_pass(t1b, P.n2p, T + P.t1b, n1b);
      s2 = wave_sum_d(s2);
      WinOut w;
      if (cur.e - cur.b >= (uint32_t)LNX_N || suspect_zero(s2, n2, lnx) || suspect_zero(sa, n1a, lnx) ||
          suspect_zero(sb, n1b, lnx)) {
        // rare: exact re-evaluation with the bin-by-bin proportionality test
        w = eval_window<WAVE, P16>(P, counts, pos, ann, cur.b, cur.e, T, hb, lnx, W, W + t1a, nullptr, nullptr, err);
        if (lane == 0) atomicAdd(err_word + 1, 1u);   // statistics: windows that took the exact path
      } else {
        w.snp_count = nvar; w.n2_all = n2 + nlast; w.n2 = n2; w.n1a = n1a; w.n1b = n1b;
        w.t2d = clr_fast(s2, n2, hb.flags & BGF_NAN2, lnx);
        w.t1a = clr_fast(sa, n1a, hb.flags & BGF_NAN1A, lnx);
        w.t1b = clr_fast(sb, n1b, hb.flags & BGF_NAN1B, lnx);
      }
      if (lane == 0) {
        write_rec(out + s, ch.chrom, wid, cur.b, cur.e, w, zflags);
        if (mode_bp) slots[s] = make_uint2(0u, 0u);   // leave the slot table clean for the next run
      }
      if (it == 0) STAMP(14);
    } else if (lane == 0) {
      sfs2d_window r;
      memset(&r, 0, sizeof(r));
      r.chrom = ch.chrom; r.wid = wid; r.flags = SFS2D_W_EMPTY;
      out[s] = r;
    }
    cur = nxt;
  }
  STAMP(15);
  if (err) atomicOr(err_word, err);
}

// Q9 helper (combined_scan's final block, twoDSFS_class.py:951-989): the window before the last
// one, evaluated against the LAST window's chromosome background.  One workgroup, launched only
// for plans with SFS2D_F_PREV_EXTRA.
template <int G, bool P16>
__global__ __launch_bounds__(BLOCK) void k_scan_extra(KParams P, const uint32_t* __restrict__ counts,
                                                      const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                                      uint32_t chrom_last, const long long* __restrict__ chrom_off,
                                                      const PL* __restrict__ tab, const BgHead* __restrict__ head,
                                                      int bg_per_chrom, const double* __restrict__ lnx,
                                                      sfs2d_window* __restrict__ out, uint32_t* __restrict__ err_word,
                                                      long long extra_rec) {
  extern __shared__ uint32_t lds[];
  constexpr int NG = BLOCK / G;
  const int g = threadIdx.x / G;
  const int lane = threadIdx.x & (G - 1);
  const int h2w = P16 ? (P.nb2 + 1) / 2 : P.nb2;
  const int per = h2w + (P.n1p + 1) + (P.n2p + 1);
  uint32_t* H2 = lds + g * per;
  uint32_t* H1 = H2 + h2w;
  double* redd = reinterpret_cast<double*>(lds + NG * per + ((NG * per) & 1));
  unsigned long long* redu = reinterpret_cast<unsigned long long*>(redd + 32);
  for (int k = lane; k < per; k += G) H2[k] = 0u;
  group_sync<G>();
  if (g != 0) return;
  uint32_t err = 0;
  const long long cb = chrom_off[chrom_last];
  const PL* T = tab + (bg_per_chrom ? (size_t)chrom_last * P.nt : 0);
  const BgHead hb = head[bg_per_chrom ? chrom_last : 0];
  const long long ce = chrom_off[chrom_last + 1];
  const uint32_t bl = window_begin_back(pos, cb, (uint32_t)ce, P.ws);
  WinOut w;
  memset(&w, 0, sizeof(w));
  uint32_t pb = 0, pe = 0, pc = chrom_last, flags = SFS2D_W_EXTRA | bg_zero_flags(hb);
  if (bl > 0) {
    pe = bl;
    int c2 = (int)chrom_last;
    while (c2 > 0 && chrom_off[c2] >= (long long)pe) --c2;
    pc = (uint32_t)c2;
    pb = window_begin_back(pos, chrom_off[c2], pe, P.ws);
    w = eval_window<G, P16>(P, counts, pos, ann, pb, pe, T, hb, lnx, H2, H1, redd, redu, err);
  } else {
    flags |= SFS2D_W_EMPTY;
  }
  if (lane == 0) write_rec(out + extra_rec, pc, bl, pb, pe, w, flags);
  if (err) atomicOr(err_word, err);
}


// ------------------------------------------------------------------------------------------
// host side

void pw_plan(int lo, int n, std::vector<int2>& leaves, std::vector<short>& prog) {
  // numpy pairwise_sum recursion: n <= 128 -> leaf; else split at n2 = n/2 - (n/2 % 8)
  if (n <= 128) {
    prog.push_back((short)leaves.size());
    leaves.push_back(make_int2(lo, n));
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  pw_plan(lo, n2, leaves, prog);
  pw_plan(lo + n2, n - n2, leaves, prog);
  prog.push_back(-1);
}

}  // namespace

struct sfs2d_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  double* d_lnx = nullptr;
  std::string err;
};

struct sfs2d_data {
  sfs2d_ctx* ctx = nullptr;
  bool owned = false;
  uint32_t* counts = nullptr;
  uint32_t* pos = nullptr;
  uint16_t* ann = nullptr;
  long long* d_chrom_off = nullptr;
  int64_t n = 0;
  int32_t nchrom = 0;
  std::vector<int64_t> chrom_off;
  std::vector<uint32_t> last_pos;
  std::vector<uint32_t> host_pos;   // upload path only: exact window-length bound for u16 bins
  bool ann_owned = false;
  bool strict = true;   // positions strictly increasing within each chromosome
};

struct sfs2d_plan {
  sfs2d_ctx* ctx = nullptr;
  const sfs2d_data* data = nullptr;
  sfs2d_params prm{};
  KParams K{};
  int nbg = 0;
  bool do_bg = false, do_seg = false, lds_hist = true, bg_ready = false;
  int G = 64;
  bool p16 = true;
  size_t scan_lds = 0, bg_lds = 0;
  int64_t nslots = 0, nrec = 0, extra_rec = -1;
  uint32_t last_chrom = 0;
  std::vector<Tile> tiles;
  std::vector<Chunk> chunks;
  Tile* d_tiles = nullptr;
  Chunk* d_chunks = nullptr;
  unsigned long long* d_slot_base = nullptr;
  uint2* d_slots = nullptr;
  uint32_t* d_repl = nullptr;
  double* d_bgval = nullptr;
  PL* d_tab = nullptr;
  BgHead* d_head = nullptr;
  int2* d_leaves = nullptr;
  short* d_prog = nullptr;
  int nleaves = 0, nprog = 0;
  sfs2d_window* d_out = nullptr;
  uint32_t* d_err = nullptr;
  sfs2d_window* last_out = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // live timing ring: events around each kernel of every run while timing is on
  bool timing = false;
  std::vector<hipEvent_t> tev;   // 4 per run
  int tcount = 0;
};

namespace {

int set_err(sfs2d_ctx* ctx, int code, const std::string& m) {
  if (ctx) ctx->err = m;
  return code;
}

#define HIPCHK(ctx, call)                                                                         \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return set_err((ctx), SFS2D_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_));      \
  } while (0)

template <typename T>
int dalloc(sfs2d_ctx* ctx, T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return set_err(ctx, SFS2D_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  return 0;
}

void plan_free(sfs2d_plan* p) {
  hipFree(p->d_tiles); hipFree(p->d_chunks); hipFree(p->d_slot_base); hipFree(p->d_slots);
  hipFree(p->d_repl); hipFree(p->d_bgval); hipFree(p->d_tab); hipFree(p->d_head);
  hipFree(p->d_leaves); hipFree(p->d_prog); hipFree(p->d_out); hipFree(p->d_err);
  for (auto& e : p->ev) if (e) hipEventDestroy(e);
  for (auto& e : p->tev) if (e) hipEventDestroy(e);
}

template <int G, bool P16>
hipError_t launch_scan(sfs2d_plan* pl, sfs2d_window* out) {
  const sfs2d_data* d = pl->data;
  if (G == WAVE) {
    hipLaunchKernelGGL((k_scan_w<P16>), dim3((unsigned)pl->chunks.size()), dim3(BLOCK), pl->scan_lds,
                       pl->ctx->stream, pl->K, d->counts, d->pos, d->ann, pl->d_chunks, d->d_chrom_off,
                       pl->d_slots, pl->d_tab, pl->d_head, pl->prm.bg_mode == SFS2D_BG_PER_CHROM ? 1 : 0,
                       pl->ctx->d_lnx, out, pl->d_err, pl->prm.window_mode == SFS2D_WINDOW_BP ? 1 : 0);
    return hipGetLastError();
  }
  hipLaunchKernelGGL((k_scan<G, P16>), dim3((unsigned)pl->chunks.size()), dim3(BLOCK), pl->scan_lds,
                     pl->ctx->stream, pl->K, d->counts, d->pos, d->ann, pl->d_chunks, d->d_chrom_off,
                     pl->d_slots, pl->d_tab, pl->d_head, pl->prm.bg_mode == SFS2D_BG_PER_CHROM ? 1 : 0,
                     pl->ctx->d_lnx, out, pl->d_err, pl->prm.window_mode == SFS2D_WINDOW_BP ? 1 : 0,
                     (long long)pl->extra_rec);
  return hipGetLastError();
}

template <bool B, bool S, bool L>
hipError_t launch_bgseg1(sfs2d_plan* pl) {
  const sfs2d_data* d = pl->data;
  hipLaunchKernelGGL((k_bg_seg<B, S, L>), dim3((unsigned)pl->tiles.size()), dim3(BLOCK1), L ? pl->bg_lds : 0,
                     pl->ctx->stream, pl->K, d->counts, d->pos, d->ann, pl->d_tiles, d->d_chrom_off,
                     pl->d_slot_base, pl->d_repl, pl->d_slots, pl->d_err);
  return hipGetLastError();
}

hipError_t launch_bgseg(sfs2d_plan* pl) {
  if (pl->tiles.empty()) return hipSuccess;
  if (pl->do_bg && pl->do_seg) return pl->lds_hist ? launch_bgseg1<true, true, true>(pl) : launch_bgseg1<true, true, false>(pl);
  if (pl->do_bg) return pl->lds_hist ? launch_bgseg1<true, false, true>(pl) : launch_bgseg1<true, false, false>(pl);
  if (pl->do_seg) return launch_bgseg1<false, true, false>(pl);
  return hipSuccess;
}

hipError_t launch_finalize(sfs2d_plan* pl, int from_repl, int integer_values) {
  const size_t lds = pl->K.nt <= FIN_LDS_BINS ? sizeof(double) * pl->K.nt : 0;
  hipLaunchKernelGGL(k_bg_finalize, dim3(pl->nbg), dim3(FBLOCK), lds, pl->ctx->stream, pl->K, from_repl, integer_values,
                     pl->d_repl, pl->d_bgval, pl->d_tab, pl->d_head, pl->d_leaves, pl->nleaves, pl->d_prog, pl->nprog);
  return hipGetLastError();
}

template <int G, bool P16>
hipError_t launch_extra(sfs2d_plan* pl, sfs2d_window* out) {
  const sfs2d_data* d = pl->data;
  hipLaunchKernelGGL((k_scan_extra<G, P16>), dim3(1), dim3(BLOCK), pl->scan_lds, pl->ctx->stream, pl->K, d->counts,
                     d->pos, d->ann, pl->last_chrom, d->d_chrom_off, pl->d_tab, pl->d_head,
                     pl->prm.bg_mode == SFS2D_BG_PER_CHROM ? 1 : 0, pl->ctx->d_lnx, out, pl->d_err,
                     (long long)pl->extra_rec);
  return hipGetLastError();
}

hipError_t launch_scan_any(sfs2d_plan* pl, sfs2d_window* out) {
  hipError_t e = hipSuccess;
  if (!pl->chunks.empty()) {
    if (pl->G == 64) e = pl->p16 ? launch_scan<64, true>(pl, out) : launch_scan<64, false>(pl, out);
    else e = pl->p16 ? launch_scan<256, true>(pl, out) : launch_scan<256, false>(pl, out);
  }
  if (e == hipSuccess && pl->extra_rec >= 0) {
    if (pl->G == 64) e = pl->p16 ? launch_extra<64, true>(pl, out) : launch_extra<64, false>(pl, out);
    else e = pl->p16 ? launch_extra<256, true>(pl, out) : launch_extra<256, false>(pl, out);
  }
  return e;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI

extern "C" {

int sfs2d_abi_version(void) { return SFS2D_ABI_VERSION; }

const char* sfs2d_last_error(const sfs2d_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int sfs2d_ctx_create(int device, sfs2d_ctx** out) {
  if (!out) return SFS2D_E_ARG;
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return SFS2D_E_HIP;
  if (device < 0 || device >= ndev) return SFS2D_E_ARG;
  sfs2d_ctx* c = new sfs2d_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SFS2D_E_HIP;
  }
  c->stream = c->own;
  if (dalloc(c, &c->d_lnx, LNX_N)) { hipStreamDestroy(c->own); delete c; return SFS2D_E_NOMEM; }
  hipLaunchKernelGGL(k_init_lnx, dim3(LNX_N / 256), dim3(256), 0, c->stream, c->d_lnx);
  if (hipStreamSynchronize(c->stream) != hipSuccess) { hipFree(c->d_lnx); hipStreamDestroy(c->own); delete c; return SFS2D_E_HIP; }
  *out = c;
  return 0;
}

int sfs2d_ctx_destroy(sfs2d_ctx* ctx) {
  if (!ctx) return SFS2D_E_ARG;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  hipFree(ctx->d_lnx);
  hipStreamDestroy(ctx->own);
  delete ctx;
  return 0;
}

int sfs2d_ctx_set_stream(sfs2d_ctx* ctx, void* stream) {
  if (!ctx) return SFS2D_E_ARG;
  ctx->stream = stream ? (hipStream_t)stream : ctx->own;
  return 0;
}

static int data_meta(sfs2d_ctx* ctx, sfs2d_data* d, const int64_t* chrom_off, int32_t nchrom, int64_t n) {
  if (nchrom < 0 || n < 0 || n > 0xfffffff0ll) return set_err(ctx, SFS2D_E_ARG, "bad n / nchrom");
  if (nchrom > 0 && !chrom_off) return set_err(ctx, SFS2D_E_ARG, "chrom_off is NULL");
  d->chrom_off.assign(chrom_off, chrom_off + nchrom + 1);
  if (nchrom == 0) d->chrom_off.assign(1, 0);
  if (d->chrom_off.front() != 0 || d->chrom_off.back() != n) return set_err(ctx, SFS2D_E_ARG, "chrom_off must span [0, n]");
  for (int c = 0; c < nchrom; ++c)
    if (d->chrom_off[c + 1] < d->chrom_off[c]) return set_err(ctx, SFS2D_E_ARG, "chrom_off not monotone");
  d->n = n;
  d->nchrom = nchrom;
  if (dalloc(ctx, &d->d_chrom_off, (size_t)nchrom + 1)) return SFS2D_E_NOMEM;
  HIPCHK(ctx, hipMemcpy(d->d_chrom_off, d->chrom_off.data(), sizeof(long long) * (nchrom + 1), hipMemcpyHostToDevice));
  return 0;
}

int sfs2d_data_upload(sfs2d_ctx* ctx, const uint32_t* counts, const uint32_t* pos, const uint16_t* ann_id, int64_t n,
                      const int64_t* chrom_off, int32_t nchrom, sfs2d_data** out) {
  if (!ctx || !out || (n > 0 && (!counts || !pos))) return set_err(ctx, SFS2D_E_ARG, "null argument");
  *out = nullptr;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  sfs2d_data* d = new sfs2d_data();
  d->ctx = ctx;
  d->owned = true;
  int rc = data_meta(ctx, d, chrom_off, nchrom, n);
  // padded: the kernels issue aligned 16-B loads that may run up to 15 bytes past element n-1
  const size_t npad = ((size_t)n + 3) / 4 * 4 + 64;
  if (!rc) rc = dalloc(ctx, &d->counts, npad);
  if (!rc) rc = dalloc(ctx, &d->pos, npad);
  if (!rc) rc = dalloc(ctx, &d->ann, npad);
  if (!rc && (hipMemset(d->counts, 0, npad * 4) != hipSuccess || hipMemset(d->pos, 0, npad * 4) != hipSuccess))
    rc = set_err(ctx, SFS2D_E_HIP, "hipMemset");
  if (rc) { hipFree(d->counts); hipFree(d->pos); hipFree(d->ann); hipFree(d->d_chrom_off); delete d; return rc; }
  hipError_t e = hipSuccess;
  if (n) {
    e = hipMemcpy(d->counts, counts, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d->pos, pos, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
      if (ann_id) e = hipMemcpy(d->ann, ann_id, sizeof(uint16_t) * n, hipMemcpyHostToDevice);
      else e = hipMemset(d->ann, 0, sizeof(uint16_t) * n);
    }
  }
  if (e != hipSuccess) {
    hipFree(d->counts); hipFree(d->pos); hipFree(d->ann); hipFree(d->d_chrom_off); delete d;
    return set_err(ctx, SFS2D_E_HIP, std::string("upload: ") + hipGetErrorString(e));
  }
  d->last_pos.assign(nchrom, 0);
  d->host_pos.assign(pos, pos + n);
  for (int c = 0; c < nchrom; ++c) {
    int64_t s = d->chrom_off[c], t = d->chrom_off[c + 1];
    if (t > s) d->last_pos[c] = pos[t - 1];
    for (int64_t i = s + 1; i < t; ++i)
      if (pos[i] <= pos[i - 1]) { d->strict = false; break; }
  }
  *out = d;
  return 0;
}

int sfs2d_data_wrap_device(sfs2d_ctx* ctx, const uint32_t* d_counts, const uint32_t* d_pos, const uint16_t* d_ann_id,
                           int64_t n, const int64_t* chrom_off, const uint32_t* chrom_last_pos, int32_t nchrom,
                           sfs2d_data** out) {
  if (!ctx || !out || (n > 0 && (!d_counts || !d_pos)) || (nchrom > 0 && !chrom_last_pos))
    return set_err(ctx, SFS2D_E_ARG, "null argument");
  *out = nullptr;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  sfs2d_data* d = new sfs2d_data();
  d->ctx = ctx;
  d->owned = false;
  int rc = data_meta(ctx, d, chrom_off, nchrom, n);
  if (rc) { hipFree(d->d_chrom_off); delete d; return rc; }
  if (((uintptr_t)d_counts & 15) || ((uintptr_t)d_pos & 15)) {
    hipFree(d->d_chrom_off); delete d;
    return set_err(ctx, SFS2D_E_ARG, "device arrays must be 16-byte aligned (and readable to round_up(n, 4))");
  }
  d->counts = const_cast<uint32_t*>(d_counts);
  d->pos = const_cast<uint32_t*>(d_pos);
  if (d_ann_id) {
    d->ann = const_cast<uint16_t*>(d_ann_id);
  } else {
    if (dalloc(ctx, &d->ann, (size_t)n + 1) || hipMemset(d->ann, 0, sizeof(uint16_t) * (n + 1)) != hipSuccess) {
      hipFree(d->d_chrom_off); delete d; return SFS2D_E_NOMEM;
    }
    d->ann_owned = true;
  }
  d->last_pos.assign(chrom_last_pos, chrom_last_pos + nchrom);
  d->strict = true;   // contract: positions strictly increasing within each chromosome
  *out = d;
  return 0;
}

int sfs2d_data_free(sfs2d_data* d) {
  if (!d) return SFS2D_E_ARG;
  hipSetDevice(d->ctx->device);
  if (d->owned) { hipFree(d->counts); hipFree(d->pos); }
  if (d->owned || d->ann_owned) hipFree(d->ann);
  hipFree(d->d_chrom_off);
  delete d;
  return 0;
}

static int make_kparams(sfs2d_ctx* ctx, const sfs2d_params* prm, int nchrom, KParams* K) {
  if (!prm) return set_err(ctx, SFS2D_E_ARG, "params is NULL");
  if (prm->n1p < 1 || prm->n2p < 1 || 2 * prm->n1p > 255 || 2 * prm->n2p > 255)
    return set_err(ctx, SFS2D_E_ARG, "pop sizes must satisfy 1 <= pop_size and 2*pop_size <= 255 (u8 counts)");
  if (prm->window_mode != SFS2D_WINDOW_BP && prm->window_mode != SFS2D_WINDOW_SNPS)
    return set_err(ctx, SFS2D_E_ARG, "bad window_mode");
  if (prm->window < 1 || prm->window > 0xffffffffll) return set_err(ctx, SFS2D_E_ARG, "window must be in [1, 2^32)");
  if (prm->bg_mode != SFS2D_BG_PER_CHROM && prm->bg_mode != SFS2D_BG_SUPPLIED) return set_err(ctx, SFS2D_E_ARG, "bad bg_mode");
  K->n1p = prm->n1p; K->n2p = prm->n2p; K->n1 = 2 * prm->n1p; K->n2 = 2 * prm->n2p;
  K->nb2 = (K->n1 + 1) * (K->n2 + 1);
  K->h1a = K->nb2; K->h1b = K->nb2 + K->n1 + 1; K->nh = K->h1b + K->n2 + 1;
  K->t1a = K->nb2; K->t1b = K->nb2 + K->n1p + 1; K->nt = K->t1b + K->n2p + 1;
  K->fold = prm->fold ? 1 : 0;
  K->ann_want = prm->ann_want;
  K->has_start = prm->has_start ? 1 : 0; K->has_end = prm->has_end ? 1 : 0;
  K->start_pos = prm->start_pos; K->end_pos = prm->end_pos;
  K->ws = (unsigned)prm->window;
  K->nchrom = nchrom;
  return 0;
}

int sfs2d_plan_create(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, sfs2d_plan** out) {
  if (!ctx || !data || !prm || !out) return set_err(ctx, SFS2D_E_ARG, "null argument");
  *out = nullptr;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  KParams K;
  int rc = make_kparams(ctx, prm, data->nchrom, &K);
  if (rc) return rc;
  sfs2d_plan* pl = new sfs2d_plan();
  pl->ctx = ctx; pl->data = data; pl->prm = *prm; pl->K = K;
  const bool bp = prm->window_mode == SFS2D_WINDOW_BP;
  pl->do_seg = bp;
  pl->do_bg = prm->bg_mode == SFS2D_BG_PER_CHROM;
  pl->nbg = pl->do_bg ? std::max(1, data->nchrom) : 1;
  const int nc = data->nchrom;

  // window slots + scan chunks
  std::vector<unsigned long long> slot_base(nc + 1, 0);
  uint32_t last_c = 0;
  bool any = false;
  for (int c = 0; c < nc; ++c) {
    const int64_t len = data->chrom_off[c + 1] - data->chrom_off[c];
    int64_t ns = 0;
    if (len > 0) {
      if (bp) ns = (int64_t)(data->last_pos[c] ? (data->last_pos[c] - 1u) / (uint32_t)prm->window : 0u) + 1;
      else ns = len / prm->window;
      last_c = (uint32_t)c;
      any = true;
    }
    slot_base[c + 1] = slot_base[c] + ns;
  }
  pl->nslots = (int64_t)slot_base[nc];
  if (pl->nslots > 0x7fffffffll) { delete pl; return set_err(ctx, SFS2D_E_ARG, "too many window slots (window too small)"); }
  pl->extra_rec = ((prm->flags & SFS2D_F_PREV_EXTRA) && bp && any) ? pl->nslots : -1;
  pl->nrec = pl->nslots + (pl->extra_rec >= 0 ? 1 : 0);

  // LDS strategy: a wavefront per window with u16-packed 2D bins for small grids, a workgroup per
  // window for large ones; u16 bins need < 65536 SNPs of one window in one bin.
  bool p16_ok;
  if (!bp) {
    p16_ok = prm->window <= 65535;
  } else if (data->strict && prm->window <= 65535) {
    p16_ok = true;   // unique positions: a window of ws bp holds at most ws SNPs
  } else if (!data->host_pos.empty() || data->n == 0) {
    // exact longest window run from the host copy of the positions
    int64_t longest = 0;
    for (int c = 0; c < nc; ++c) {
      int64_t run = 0;
      uint32_t pw = 0xffffffffu;
      for (int64_t i = data->chrom_off[c]; i < data->chrom_off[c + 1]; ++i) {
        const uint32_t p = data->host_pos[i];
        const uint32_t w = p ? (p - 1u) / (uint32_t)prm->window : 0u;
        run = (w == pw) ? run + 1 : 1;
        pw = w;
        longest = std::max(longest, run);
      }
    }
    p16_ok = longest <= 65535;
  } else {
    p16_ok = false;
  }
  pl->p16 = p16_ok;
  pl->G = (K.nb2 <= 8192) ? 64 : 256;
  const int h2w = pl->p16 ? (K.nb2 + 1) / 2 : K.nb2;
  const int per = h2w + (K.n1p + 1) + (K.n2p + 1);
  const int ng = BLOCK / pl->G;
  pl->scan_lds = (size_t)(ng * (per + TRASH) + 2) * 4 + 32 * 8 + 32 * 8;
  if (pl->scan_lds > 160 * 1024) {
    delete pl;
    return set_err(ctx, SFS2D_E_ARG, "2D grid too large for LDS with 32-bit bins (windows of >= 65536 SNPs)");
  }
  // slots per workgroup: enough workgroups to fill 256 CUs several times, then longer chunks
  uint32_t CH;
  if (pl->G == 64) {
    const int64_t per_wave = (pl->nslots + 4 * 1024 - 1) / (4 * 1024);
    CH = (uint32_t)(4 * std::max<int64_t>(1, std::min<int64_t>(8, per_wave)));
  } else {
    CH = 2;
  }
  for (int c = 0; c < nc; ++c) {
    for (unsigned long long s = slot_base[c]; s < slot_base[c + 1]; s += CH) {
      Chunk ch{};
      ch.chrom = (uint32_t)c; ch.kind = 0; ch.slot_lo = (uint32_t)s;
      ch.slot_hi = (uint32_t)std::min<unsigned long long>(s + CH, slot_base[c + 1]);
      ch.wid_lo = (uint32_t)(s - slot_base[c]);
      pl->chunks.push_back(ch);
    }
  }
  pl->last_chrom = last_c;

  // background / segmentation tiles (never crossing a chromosome)
  if (pl->do_bg || pl->do_seg) {
    const int64_t n = data->n;
    // ~1000+ tiles for big inputs (several workgroups per CU), >= 4096 SNPs each (flush amortised)
    int64_t T = std::max<int64_t>(4096, std::min<int64_t>(65536, (n / 768 + 4095) / 4096 * 4096));
    for (int c = 0; c < nc; ++c)
      for (int64_t s = data->chrom_off[c]; s < data->chrom_off[c + 1]; s += T) {
        Tile t{};
        t.chrom = (uint32_t)c; t.begin = (uint32_t)s;
        t.end = (uint32_t)std::min<int64_t>(s + T, data->chrom_off[c + 1]);
        pl->tiles.push_back(t);
      }
  }
  pl->bg_lds = (size_t)K.nh * 4;
  pl->lds_hist = pl->bg_lds <= 150 * 1024;

  // numpy pairwise plan over the 2D inner bins except the last (p[:-1] of bins[1:-1])
  std::vector<int2> leaves;
  std::vector<short> prog;
  if (K.nb2 - 3 > 0) pw_plan(0, K.nb2 - 3, leaves, prog);
  pl->nleaves = (int)leaves.size();
  pl->nprog = (int)prog.size();
  if (pl->nleaves > PW_MAX_LEAVES) { delete pl; return set_err(ctx, SFS2D_E_ARG, "grid too large for the pairwise plan"); }

  hipStream_t st = ctx->stream;
  rc = 0;
  rc = rc ? rc : dalloc(ctx, &pl->d_tiles, pl->tiles.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_chunks, pl->chunks.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_slot_base, (size_t)nc + 1);
  rc = rc ? rc : dalloc(ctx, &pl->d_slots, (size_t)pl->nslots + 1);
  rc = rc ? rc : dalloc(ctx, &pl->d_repl, pl->do_bg ? (size_t)REPL * nc * K.nh : 1);
  rc = rc ? rc : dalloc(ctx, &pl->d_bgval, (size_t)pl->nbg * K.nt);
  rc = rc ? rc : dalloc(ctx, &pl->d_tab, (size_t)pl->nbg * K.nt);
  rc = rc ? rc : dalloc(ctx, &pl->d_head, (size_t)pl->nbg);
  rc = rc ? rc : dalloc(ctx, &pl->d_leaves, leaves.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_prog, prog.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_out, (size_t)pl->nrec);
  rc = rc ? rc : dalloc(ctx, &pl->d_err, 4);
  if (rc) { plan_free(pl); delete pl; return rc; }
  hipError_t e = hipSuccess;
#define PCPY(dst, v) if (e == hipSuccess && !(v).empty()) e = hipMemcpyAsync(dst, (v).data(), sizeof((v)[0]) * (v).size(), hipMemcpyHostToDevice, st)
  PCPY(pl->d_tiles, pl->tiles);
  PCPY(pl->d_chunks, pl->chunks);
  PCPY(pl->d_slot_base, slot_base);
  PCPY(pl->d_leaves, leaves);
  PCPY(pl->d_prog, prog);
#undef PCPY
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_slots, 0, sizeof(uint2) * ((size_t)pl->nslots + 1), st);
  if (e == hipSuccess && pl->do_bg) e = hipMemsetAsync(pl->d_repl, 0, sizeof(uint32_t) * (size_t)REPL * nc * K.nh, st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_err, 0, 4 * sizeof(uint32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_out, 0, sizeof(sfs2d_window) * (size_t)pl->nrec, st);
  for (auto& ev : pl->ev) if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    plan_free(pl); delete pl;
    return set_err(ctx, SFS2D_E_HIP, std::string("plan setup: ") + hipGetErrorString(e));
  }
  if (pl->lds_hist && pl->bg_lds > 64 * 1024) {
    if (pl->do_bg && pl->do_seg) hipFuncSetAttribute((const void*)k_bg_seg<true, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->bg_lds);
    if (pl->do_bg) hipFuncSetAttribute((const void*)k_bg_seg<true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->bg_lds);
  }
  hipFuncSetAttribute((const void*)k_bg_finalize, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)(sizeof(double) * FIN_LDS_BINS));
  if (pl->scan_lds > 64 * 1024) {
    hipFuncSetAttribute((const void*)k_scan<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan<256, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan<256, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan_extra<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan_extra<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan_extra<256, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
    hipFuncSetAttribute((const void*)k_scan_extra<256, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->scan_lds);
  }
  pl->bg_ready = false;
  *out = pl;
  return 0;
}

int64_t sfs2d_plan_num_records(const sfs2d_plan* pl) { return pl ? pl->nrec : -1; }

int sfs2d_plan_set_background(sfs2d_plan* pl, const double* bg2d, const double* bg1a, const double* bg1b) {
  if (!pl || !bg2d || !bg1a || !bg1b) return set_err(pl ? pl->ctx : nullptr, SFS2D_E_ARG, "null argument");
  sfs2d_ctx* ctx = pl->ctx;
  if (pl->prm.bg_mode != SFS2D_BG_SUPPLIED) return set_err(ctx, SFS2D_E_ARG, "plan does not take a supplied background");
  const KParams& K = pl->K;
  std::vector<double> v(K.nt);
  std::memcpy(v.data(), bg2d, sizeof(double) * K.nb2);
  std::memcpy(v.data() + K.t1a, bg1a, sizeof(double) * (K.n1p + 1));
  std::memcpy(v.data() + K.t1b, bg1b, sizeof(double) * (K.n2p + 1));
  bool integer_values = true;
  for (double x : v)
    if (!(x == std::floor(x)) || std::fabs(x) > 9.0e15) { integer_values = false; break; }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemcpyAsync(pl->d_bgval, v.data(), sizeof(double) * K.nt, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, launch_finalize(pl, 0, integer_values ? 1 : 0));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  pl->bg_ready = true;
  return 0;
}

int sfs2d_plan_run_phase(sfs2d_plan* pl, int phase, sfs2d_window* out_dev) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  hipEvent_t* te = nullptr;
  if (pl->timing && phase == 0 && pl->tcount * 4 < (int)pl->tev.size()) te = &pl->tev[(size_t)pl->tcount * 4];
  if (!pl->do_bg && !pl->bg_ready && phase != 1)
    return set_err(ctx, SFS2D_E_ARG, "supplied-background plan run before sfs2d_plan_set_background");
  if (te) HIPCHK(ctx, hipEventRecord(te[0], ctx->stream));
  if (phase == 0 || phase == 1) {
    HIPCHK(ctx, launch_bgseg(pl));
  }
  if (te) HIPCHK(ctx, hipEventRecord(te[1], ctx->stream));
  if (phase == 0 || phase == 2) {
    if (pl->do_bg) HIPCHK(ctx, launch_finalize(pl, 1, 1));
    if (te) HIPCHK(ctx, hipEventRecord(te[2], ctx->stream));
    sfs2d_window* out = out_dev ? out_dev : pl->d_out;
    HIPCHK(ctx, launch_scan_any(pl, out));
    pl->last_out = out;
  }
  if (te) {
    HIPCHK(ctx, hipEventRecord(te[3], ctx->stream));
    pl->tcount++;
  }
  return 0;
}

int sfs2d_plan_set_timing(sfs2d_plan* pl, int max_runs) {
  if (!pl || max_runs < 0) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  for (auto& e : pl->tev) if (e) hipEventDestroy(e);
  pl->tev.assign((size_t)max_runs * 4, nullptr);
  for (auto& e : pl->tev) HIPCHK(ctx, hipEventCreate(&e));
  pl->tcount = 0;
  pl->timing = max_runs > 0;
  return 0;
}

int sfs2d_plan_timing_read(sfs2d_plan* pl, int* nruns, double* ms_k1, double* ms_k2, double* ms_k3) {
  if (!pl || !nruns) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  double t[3] = {0, 0, 0};
  for (int r = 0; r < pl->tcount; ++r) {
    hipEvent_t* te = &pl->tev[(size_t)r * 4];
    HIPCHK(ctx, hipEventSynchronize(te[3]));
    for (int k = 0; k < 3; ++k) {
      float ms = 0;
      HIPCHK(ctx, hipEventElapsedTime(&ms, te[k], te[k + 1]));
      t[k] += ms;
    }
  }
  *nruns = pl->tcount;
  const double d = pl->tcount ? pl->tcount : 1;
  if (ms_k1) *ms_k1 = t[0] / d;
  if (ms_k2) *ms_k2 = t[1] / d;
  if (ms_k3) *ms_k3 = t[2] / d;
  return 0;
}

int sfs2d_plan_run(sfs2d_plan* pl, sfs2d_window* out_dev) { return sfs2d_plan_run_phase(pl, 0, out_dev); }

int sfs2d_plan_bg_buffer(sfs2d_plan* pl, void** dev_ptr, int64_t* nbytes) {
  if (!pl || !dev_ptr || !nbytes) return SFS2D_E_ARG;
  *dev_ptr = pl->d_repl;
  *nbytes = pl->do_bg ? (int64_t)REPL * pl->data->nchrom * pl->K.nh * 4 : 0;
  return 0;
}

int sfs2d_plan_check(sfs2d_plan* pl) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  uint32_t e = 0;
  HIPCHK(ctx, hipMemcpyAsync(&e, pl->d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (e) {
    HIPCHK(ctx, hipMemsetAsync(pl->d_err, 0, 4, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (e & ERR_KEY) return set_err(ctx, SFS2D_E_KEY, "allele count above 2*pop_size (reference: KeyError in calculate_1d_sfs)");
    return set_err(ctx, SFS2D_E_GRID, "folded 2D bin outside the (2n1+1)x(2n2+1) grid");
  }
  return 0;
}

// diagnostic: stamps of a -DSFS2D_STAMPS build (returns SFS2D_E_ARG in the shipped build)
int sfs2d__debug_stamps(unsigned long long* out64) {
#ifdef SFS2D_STAMPS
  if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 64) != hipSuccess) return SFS2D_E_HIP;
  return 0;
#else
  (void)out64;
  return SFS2D_E_ARG;
#endif
}

int sfs2d_plan_stats(sfs2d_plan* pl, uint32_t* exact_windows) {
  if (!pl || !exact_windows) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  HIPCHK(ctx, hipMemcpyAsync(exact_windows, pl->d_err + 1, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int sfs2d_plan_read(sfs2d_plan* pl, sfs2d_window* out_host, int64_t cap, int64_t* nrec_out) {
  if (!pl || !nrec_out) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  *nrec_out = pl->nrec;
  if (cap < pl->nrec) return set_err(ctx, SFS2D_E_CAP, "output capacity too small");
  if (pl->nrec && !out_host) return SFS2D_E_ARG;
  const sfs2d_window* src = pl->last_out ? pl->last_out : pl->d_out;
  if (pl->nrec)
    HIPCHK(ctx, hipMemcpyAsync(out_host, src, sizeof(sfs2d_window) * pl->nrec, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  return 0;
}

int sfs2d_plan_time(sfs2d_plan* pl, int iters, double* ms_run, double* ms_k1, double* ms_k2, double* ms_k3) {
  if (!pl || iters < 1) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  hipStream_t st = ctx->stream;
  double t1 = 0, t2 = 0, t3 = 0, tall = 0;
  for (int it = 0; it < iters; ++it) {
    HIPCHK(ctx, hipEventRecord(pl->ev[0], st));
    HIPCHK(ctx, launch_bgseg(pl));
    HIPCHK(ctx, hipEventRecord(pl->ev[1], st));
    if (pl->do_bg) HIPCHK(ctx, launch_finalize(pl, 1, 1));
    HIPCHK(ctx, hipEventRecord(pl->ev[2], st));
    HIPCHK(ctx, launch_scan_any(pl, pl->d_out));
    HIPCHK(ctx, hipEventRecord(pl->ev[3], st));
    HIPCHK(ctx, hipEventSynchronize(pl->ev[3]));
    float a = 0, b = 0, c = 0, d = 0;
    hipEventElapsedTime(&a, pl->ev[0], pl->ev[1]);
    hipEventElapsedTime(&b, pl->ev[1], pl->ev[2]);
    hipEventElapsedTime(&c, pl->ev[2], pl->ev[3]);
    hipEventElapsedTime(&d, pl->ev[0], pl->ev[3]);
    t1 += a; t2 += b; t3 += c; tall += d;
  }
  pl->last_out = pl->d_out;
  if (ms_run) *ms_run = tall / iters;
  if (ms_k1) *ms_k1 = t1 / iters;
  if (ms_k2) *ms_k2 = t2 / iters;
  if (ms_k3) *ms_k3 = t3 / iters;
  return 0;
}

int sfs2d_plan_destroy(sfs2d_plan* pl) {
  if (!pl) return SFS2D_E_ARG;
  hipSetDevice(pl->ctx->device);
  hipStreamSynchronize(pl->ctx->stream);
  plan_free(pl);
  delete pl;
  return 0;
}

int sfs2d_bg_hist(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int32_t chrom, int64_t* h2d,
                  int64_t* h1a, int64_t* h1b) {
  if (!ctx || !data || !prm || !h2d || !h1a || !h1b) return set_err(ctx, SFS2D_E_ARG, "null argument");
  if (chrom < -1 || chrom >= data->nchrom) return set_err(ctx, SFS2D_E_ARG, "chrom out of range");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  KParams K;
  int rc = make_kparams(ctx, prm, data->nchrom, &K);
  if (rc) return rc;
  // one pseudo-chromosome: all tiles accumulate into background 0
  sfs2d_plan pl;
  pl.ctx = ctx; pl.data = data; pl.prm = *prm; pl.K = K; pl.K.nchrom = 1;
  pl.do_bg = true; pl.do_seg = false;
  pl.bg_lds = (size_t)K.nh * 4;
  pl.lds_hist = pl.bg_lds <= 150 * 1024;
  const int c0 = chrom < 0 ? 0 : chrom, c1 = chrom < 0 ? data->nchrom : chrom + 1;
  const int64_t T = 16384;
  for (int c = c0; c < c1; ++c)
    for (int64_t s = data->chrom_off[c]; s < data->chrom_off[c + 1]; s += T) {
      Tile t{};
      t.chrom = 0; t.begin = (uint32_t)s; t.end = (uint32_t)std::min<int64_t>(s + T, data->chrom_off[c + 1]);
      pl.tiles.push_back(t);
    }
  // chrom_off for pseudo-chromosome 0 is only read by segmentation (disabled)
  std::vector<uint32_t> hist((size_t)REPL * K.nh, 0);
  rc = 0;
  rc = rc ? rc : dalloc(ctx, &pl.d_tiles, pl.tiles.size());
  rc = rc ? rc : dalloc(ctx, &pl.d_repl, (size_t)REPL * K.nh);
  rc = rc ? rc : dalloc(ctx, &pl.d_err, 1);
  hipError_t e = hipSuccess;
  if (!rc) {
    if (!pl.tiles.empty()) e = hipMemcpyAsync(pl.d_tiles, pl.tiles.data(), sizeof(Tile) * pl.tiles.size(), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(pl.d_repl, 0, sizeof(uint32_t) * REPL * K.nh, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(pl.d_err, 0, 4, ctx->stream);
    if (e == hipSuccess && pl.lds_hist && pl.bg_lds > 64 * 1024)
      hipFuncSetAttribute((const void*)k_bg_seg<true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.bg_lds);
    if (e == hipSuccess) e = launch_bgseg(&pl);
    if (e == hipSuccess) e = hipMemcpyAsync(hist.data(), pl.d_repl, sizeof(uint32_t) * REPL * K.nh, hipMemcpyDeviceToHost, ctx->stream);
    uint32_t err = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&err, pl.d_err, 4, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && err) rc = (err & ERR_KEY) ? set_err(ctx, SFS2D_E_KEY, "allele count above 2*pop_size")
                                                     : set_err(ctx, SFS2D_E_GRID, "folded 2D bin outside the grid");
  }
  hipFree(pl.d_tiles); hipFree(pl.d_repl); hipFree(pl.d_err);
  pl.d_tiles = nullptr; pl.d_repl = nullptr; pl.d_err = nullptr;
  if (e != hipSuccess) return set_err(ctx, SFS2D_E_HIP, std::string("bg_hist: ") + hipGetErrorString(e));
  if (rc) return rc;
  for (int k = 0; k < K.nh; ++k) {
    int64_t s = 0;
    for (int r = 0; r < REPL; ++r) s += hist[(size_t)r * K.nh + k];
    if (k < K.nb2) h2d[k] = s;
    else if (k < K.h1b) h1a[k - K.h1a] = s;
    else h1b[k - K.h1b] = s;
  }
  return 0;
}

int sfs2d_scan(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* params, const double* bg2d,
               const double* bg1a, const double* bg1b, sfs2d_window* out_host, int64_t cap, int64_t* nrec_out) {
  sfs2d_plan* pl = nullptr;
  int rc = sfs2d_plan_create(ctx, data, params, &pl);
  if (rc) return rc;
  if (params->bg_mode == SFS2D_BG_SUPPLIED) rc = sfs2d_plan_set_background(pl, bg2d, bg1a, bg1b);
  if (!rc) rc = sfs2d_plan_run(pl, nullptr);
  if (!rc) rc = sfs2d_plan_check(pl);
  if (!rc) rc = sfs2d_plan_read(pl, out_host, cap, nrec_out);
  else if (nrec_out) *nrec_out = pl->nrec;
  std::string keep = ctx->err;
  sfs2d_plan_destroy(pl);
  ctx->err = keep;
  return rc;
}

}  // extern "C"
