// sfs2d_kernels.hpp -- gfx950 (MI355X) device code of the windowed 2D-SFS composite-likelihood scan.
//
// Reference path (uricchio/2DSFS-scan, scripts/src/twoDSFS_class.py): per genomic window,
// calculate_2d_sfs (140-232) + fold_1d_sfs(calculate_1d_sfs) (398-463) and the multinomial
// log-likelihood ratios calculate_likelihood_2D (625-684) / _1D (478-537) against a background SFS.
// The reference builds dense dict grids per window and calls scipy.stats.multinomial.logpmf twice.
// Here the statistic is evaluated in its sparse closed form over the bins the window touches:
//
//   T = 2 * ( sum_{k: x_k>0} x_k * (ln x_k - lp_k)  -  N ln N ),   lp_k = ln(b_k / B)
//
// (the gammaln terms of the two logpmf calls cancel), keeping the reference's value semantics:
// T = 0.0 exactly when x_k/N == b_k/B bitwise on every touched bin (both logpmf calls then see
// identical proportions), +inf when a touched bin has b_k == 0 (xlogy(x, 0) = -inf), NaN when
// scipy's p[-1] <- 1 - sum(p[:-1]) replacement makes the background's last inner proportion
// negative (emulated with numpy's pairwise summation order), and the None conditions (N == 0 or
// B == 0) reported through counts / flags.
//
// For the 2D spectrum the fast path sums per SNP instead of per bin: with r_i the number of
// earlier SNPs of the window in SNP i's bin (returned by the LDS histogram atomic itself),
//   sum_k x_k ln x_k = sum_i D(r_i),  D(r) = (r+1) ln(r+1) - r ln r     (telescoping)
//   sum_k x_k lp_k   = sum_i lp_{k(i)}
// so each SNP adds D(r_i) - lp_{k(i)} with no second pass over the histogram.
//
//   k_prep        one pass over SNP tiles (counts + positions, 8 B/SNP): filters and the joint fold
//                 applied once, per-SNP packed bins written (4 B/SNP), per-chromosome background
//                 histograms (LDS-privatised, flushed into REPL replicas) and inner 2D sums,
//                 fixed-bp segmentation of the window slots.
//   k_bg_slice    per-chromosome background tables, many workgroups per background: each slice of
//                 2D bins sums its replicas, writes proportions / logs and its numpy pairwise leaves;
//                 one block per background folds the 1D spectra; the last block to finish combines
//                 the leaves (numpy's tree) and applies scipy's p[-1] rule.
//   k_bg_finalize one workgroup per supplied background (set once per plan, float or integer).
//   k_scan_w      the hot loop (small grids): one wavefront per window, 8 per workgroup sharing the
//                 background's log-proportion table and the D / x ln x tables in LDS; bins streamed
//                 with 16-B loads; one fp64 DPP reduction per spectrum; one 64-B record per window.
//   k_scan_gw     large grids: k_scan_w's loop in one-wavefront workgroups, tables read from L2.
//   k_scan_g      grids too large for k_scan_gw: one workgroup per window (exact evaluation).
//   k_scan_extra  combined_scan's final-window helper (quirk Q9).
#pragma once

#include <type_traits>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "sfs2d.h"

namespace sfs2dk {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;        // k_scan_g / k_scan_extra workgroup
constexpr int SBLOCK = 512;       // k_scan_w workgroup (8 wavefronts, one window each)
constexpr int BLOCK1 = 512;       // k_prep workgroup
constexpr int FBLOCK = 1024;      // k_bg_finalize workgroup
constexpr int KBLOCK = 512;       // k_bg_slice workgroup
constexpr int LNX_N = 1 << 20;    // ln(k) table for k < LNX_N (bin counts / window totals)
constexpr int LNT = 512;          // D(r) and x ln x tables staged in LDS by k_scan_w
constexpr int LNF = 256;          // k_scan_w: x ln x entries in LDS (x < LNF; the 1D pass and the flush, per window)
// Fst's reciprocals (1/n, 1/(n(n-1))) in LDS (k_scan_w) for n <= 2 max(n1p, n2p): an even
// count of double2
__host__ __device__ inline int wl_rtn(int n1p, int n2p) { return 2 * (n1p > n2p ? n1p : n2p) + 2; }
constexpr int RCPN = 512;         // (1/k, 1/(k(k-1))) for k < 512 (Fst: called allele counts ref + alt <= 510), after the LNT tables
#ifndef SFS2D_ABL   // ablation builds (timing only, results wrong): bit 0 no 2D atomic, 1 no 1D atomics, 2 no D / lp
#define SFS2D_ABL 0  // reads, 3 no record stores, 4 no Fst table reads, 5 no 1D end pass, 8 no per-window wave
#endif              // sums, 9 no batched finish; k_prep's common step: 6 no LDS histogram atomics, 7 loads only
                    // (no classification, histograms or segmentation); round 6's position-byte probes (10, 11:
                    // profiles/r06h_prep_position_bytes.txt) are not kept
constexpr int REPL = 4;           // replicas of the per-chromosome background histograms
constexpr int PW_MAX_LEAVES = 1024;  // numpy pairwise leaves (64-128 values each): grids up to 255 x 255 (u8 counts)
constexpr int LEAVES_PER_SLICE = 4;
constexpr int FIN_LDS_BINS = 12288;  // backgrounds with nt <= this keep values / proportions in LDS
constexpr int TRASH = WAVE;       // lane-private scratch words after each wave's histograms
// replicas of the folded 1D window histograms (lane & 3).  Round 6, k_scan_w on config 3 with Fst:
// 4 / 2 / 1 replicas 131.8-132.7 / 142.8-142.9 / 173.6-174.0 us (profiles/r06m_scan_r1_sb_ab.txt)
constexpr int R1 = 4;
#ifndef SFS2D_GW_R1
#define SFS2D_GW_R1 1
#endif
// ... in k_scan_gw: one copy (less LDS per wavefront, more of them per CU; measured 1 / 2 / 4:
// sims scan kernel 1.55 / 1.56 / 1.63 ms per 500 replicates, config 5 13.8 / 17.7 / 14.4 us)
constexpr int R1GW = SFS2D_GW_R1;

// sum (and clear) the RR replicas of one 1D bin word group (RR consecutive words, 4 * RR-B aligned)
template <int RR>
__device__ __forceinline__ uint32_t take_replicas(uint32_t* p, uint32_t shift) {
  if (RR == 4) {
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint4 v = *q;
    *q = make_uint4(0, 0, 0, 0);
    return (v.x >> shift) + (v.y >> shift) + (v.z >> shift) + (v.w >> shift);
  } else if (RR == 2) {
    uint2* q = reinterpret_cast<uint2*>(p);
    const uint2 v = *q;
    *q = make_uint2(0, 0);
    return (v.x >> shift) + (v.y >> shift);
  } else {
    const uint32_t v = *p;
    *p = 0u;
    return v >> shift;
  }
}
constexpr int FUSED_VCNT = 2 * (1536 + 256) + 16;   // k_scan_w fused prologue: word offset of the counts

enum : uint32_t { ERR_KEY = 1u, ERR_GRID = 2u, ERR_OVF = 4u };   // OVF: summed background rows >= 2^32
enum : uint32_t {
  BGF_B2_ZERO = 1u, BGF_B1A_ZERO = 2u, BGF_B1B_ZERO = 4u, BGF_NAN2 = 8u, BGF_NAN1A = 16u, BGF_NAN1B = 32u,
  BGF_FLOATV = 64u
};

// per-SNP packed bins written by k_prep:
//   bits 0-15  inner 2D bin k = x1*(n2+1)+x2 after the fold (0 = none: (0,0) is never counted)
//   bits 16-22 folded inner 1D bin of pop1 (1..pop_size-1; 0 = none)
//   bits 23-29 folded inner 1D bin of pop2
//   bit  30    annotation matches variant_type (count_snps)
//   bit  31    counted in the 2D SFS in its last bin (n1, n2), which bins[1:-1] excludes
constexpr uint32_t B_VAR = 1u << 30, B_LAST = 1u << 31;

struct KParams {
  int n1p, n2p, n1, n2;  // diploid sizes and haploid sample sizes
  int nb2;               // (n1+1)*(n2+1) 2D bins
  int nh;                // background histogram words per chromosome: nb2 + (n1+1) + (n2+1), rounded up to 4
  int h1a, h1b;          // offsets of the unfolded 1D histograms inside a background histogram
  int nt;                // table entries per background: nb2 + (n1p+1) + (n2p+1)
  int t1a, t1b;          // offsets of the folded 1D tables
  int fold;
  int ann_want;          // -1: no variant_type filter
  int has_start, has_end;
  long long start_pos, end_pos;
  int fold_thr;          // joint fold when alt1 + alt2 > fold_thr (n1p + n2p; INT_MAX without folding)
  unsigned int ws;       // bp window size (fixed-bp) or SNPs per window
  unsigned int wmag;     // (p-1)/ws as a multiply-high: q = (t + ((n - t) >> wsh1)) >> wsh2, t = mulhi(n, wmag)
  int wsh1, wsh2;
  int nchrom;
  int fst_e;             // Fst fixed point: sums of 2^fst_e-scaled terms (|term| <= 1), chosen per plan so
  double fst_scale;      // that the most SNPs a window can hold cannot overflow int64 (fst_fixed)
  uint32_t nm1;          // the data set's last SNP index (counts-reading scans clamp their row loads to it)
  uint32_t kmul;         // bytes (n2+1, 0, 1, 0): the 2D key x1*(n2+1) + x2 as one byte dot product
  uint32_t n12, lim12;   // u16 pairs (n1, n2), (n1p-1, n2p-1): both folded 1D bins in packed 16-bit ops
  int rtn;               // Fst's (1/n, 1/(n(n-1))) entries in LDS (k_scan_w): n up to the data's
                         // largest called count (even; >= wl_rtn(n1p, n2p))
  int ntri;              // k_scan_gw TRI (folded counts plans, n1 = n2 = n): the reachable 2D bins
                         // x1 + x2 <= n, (n+1)(n+2)/2 of them, stored as a triangle (0: full grid)
  int jnt;               // k_prep (counts plans, LDS histogram): the joint (alt1, alt2) histogram, see prep_tile
  int lnl;               // k_scan_gw: ln(x) for x < LNL in the wave's LDS (when it costs no occupancy)
};
constexpr int LNL = 512;   // k_scan_gw's LDS ln table (window totals and 1D bin counts below it)

struct Tile {   // k_prep work item: SNPs [begin, end) of chromosome chrom = [cb, ce), slots from sbase
  uint32_t chrom, begin, end, cb, ce, sbase, nslots, pad1;   // nslots: the chromosome's window slots
};

constexpr int SCAN_PAD = 512;   // readable words past the end of the per-SNP bins (k_scan_w prefetch)
constexpr int CTR_POOLS = 8;     // k_scan_w dynamic window pools per chromosome
constexpr int CTR_STRIDE = 16;   // one 64-B line per pool counter
#ifndef SFS2D_PREP_PREFETCH
#define SFS2D_PREP_PREFETCH 2
#endif
#ifndef SFS2D_FST_LDS
#define SFS2D_FST_LDS 256
#endif
#ifndef SFS2D_FST_R
#define SFS2D_FST_R 4
#endif
constexpr int FST_LDS = SFS2D_FST_LDS;             // k_prep: windows per tile accumulated in LDS (others: global)
constexpr int FST_R = SFS2D_FST_R;                 // ... in FST_R interleaved copies (lane & 3) to spread same-window atomics
constexpr int FST_E_MAX = 48;   // Fst sums as int64 fixed point (deterministic atomics): at most 2^48 per unit
// k_prep's fast path converts a lane's sum of up to 4 SNP terms (|term| <= 1) at once: fst_fixed's
// |x * scale| < 2^51 must hold for that sum
static_assert(4.0 * (double)(1ll << FST_E_MAX) < (double)(1ll << 51), "fst_fixed range: 4 terms at the largest scale");

struct Chunk {  // k_scan work item: window slots [slot_lo, slot_hi) of one chromosome
  uint32_t chrom, slot_lo, slot_hi, wid_lo, cb;
  // k_scan_w (slot_lo..slot_hi = the whole chromosome, wid_lo = 0): wavefront w's first window is
  // slot_lo + first + w; the windows from slot_lo + nstatic on are taken dynamically from `npool`
  // interleaved pools (pool p: nstatic + p + npool * j), this workgroup drawing from pool `pool`
  uint32_t first, nstatic, pool;   // pool: npool | pool << 16
};

struct PL {     // per-bin background table entry
  double lp;    // log of the proportion scipy uses (p[-1] adjusted on the last inner bin)
  double v;     // integer backgrounds: the count b_k; normalised (float) backgrounds: p_k = b_k / B
};

struct BgHead {
  double B2, B1a, B1b;
  uint32_t flags, pad;
};

struct Bg1D {   // k_bg_slice: the 1D block's results for the tail
  double B1a, B1b;
  uint32_t flags, pad;
};

struct WinOut {
  uint32_t snp_count, n2, n2_all, n1a, n1b;
  double t2d, t1a, t1b;
};

static_assert(sizeof(sfs2d_window) == 64, "window record must be 64 bytes");
static_assert(sizeof(Tile) == 32 && sizeof(Chunk) == 32, "work items are 32 bytes");

// Diagnostic build only (-DSFS2D_STAMPS): wall-clock stamps (s_memrealtime, 100 MHz) of block 0 at
// phase boundaries, read back with sfs2d__debug_stamps.  The shipped library executes none.
#ifdef SFS2D_STAMPS
__device__ unsigned long long g_stamps[64];
__device__ unsigned long long g_blk[2][4096][2];   // per-block start / end (k_prep, k_scan_w)
#define BLK_STAMP(k, e)                                                                          \
  do {                                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_blk[k][blockIdx.x][e] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define STAMP(i)                                                                                 \
  do {                                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[i] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
#define TSTAMP(i)   /* thread 0 of whichever block runs it (a kernel's one tail block) */       \
  do {                                                                                           \
    if (threadIdx.x == 0) g_stamps[i] = __builtin_amdgcn_s_memrealtime();                        \
  } while (0)
__device__ unsigned long long g_wv[4096 * 8][2];   // k_scan_w per wavefront: end, windows scanned
__device__ unsigned long long g_bgs[1024][2];      // k_bg_slice per block (x + y * gridDim.x): start, work done
#define BGS_STAMP(e)                                                                             \
  do {                                                                                           \
    const unsigned bi = blockIdx.x + blockIdx.y * gridDim.x;                                     \
    if (threadIdx.x == 0 && bi < 1024) g_bgs[bi][e] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#define WV_STAMP(n)                                                                              \
  do {                                                                                           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) {                                          \
      g_wv[blockIdx.x * 8 + (threadIdx.x >> 6)][0] = __builtin_amdgcn_s_memrealtime();           \
      g_wv[blockIdx.x * 8 + (threadIdx.x >> 6)][1] = (n);                                        \
    }                                                                                            \
  } while (0)
#else
#define WV_STAMP(n) \
  do {              \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#define TSTAMP(i) \
  do {            \
  } while (0)
#define BLK_STAMP(k, e) \
  do {                  \
  } while (0)
#define BGS_STAMP(e) \
  do {               \
  } while (0)
#endif

// Diagnostic build only (-DSFS2D_MARK): assembly comments delimiting regions of the scan loop
#ifdef SFS2D_MARK
#define MARK(n) asm volatile("; MARK " #n)
#else
#define MARK(n) \
  do {          \
  } while (0)
#endif

// ------------------------------------------------------------------------------------------ helpers

__device__ __forceinline__ uint32_t wid_of(uint32_t p, uint32_t ws) { return p ? (p - 1u) / ws : 0u; }

// the same window id with the division replaced by a multiply-high (host-side magic numbers)
__device__ __forceinline__ uint32_t wid_fast(const KParams& P, uint32_t p) {
  const uint32_t n = p - min(p, 1u);   // p - 1, and 0 for p = 0 (wid_of(0) = 0), without a branch
  const uint32_t t = __umulhi(n, P.wmag);
  return (t + ((n - t) >> P.wsh1)) >> P.wsh2;
}

// q = n / ws with the host-side magic numbers (fixed-SNP-count window ids)
__device__ __forceinline__ uint32_t div_fast(const KParams& P, uint32_t n) {
  const uint32_t t = __umulhi(n, P.wmag);
  return (t + ((n - t) >> P.wsh1)) >> P.wsh2;
}

// ln x for counts past the table (>= 2^20 SNPs in one bin): out of line, so that log's constants
// are not kept in registers across the loops that can reach it
__device__ __noinline__ double log_u32(uint32_t x) { return log((double)x); }

__device__ __forceinline__ double lnx_of(const double* lnx, uint32_t x) {
  return x < (uint32_t)LNX_N ? lnx[x] : log_u32(x);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

__device__ __forceinline__ uint32_t wave_sum_u(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}

// fp64 wave sum on the DPP path (xor-1 and xor-2 quad permutes, row half-mirror, row mirror: every
// lane then holds its 16-lane row's sum) and four readlanes; the result is wave-uniform and its
// rounding order is fixed (deterministic).  All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xffffffffull), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((int)(u & 0xffffffffull), l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// s2 = sum of a over the wave; sa / sb = sums of b over lanes 0-31 / 32-63
__device__ __forceinline__ void wave_sum_dpp_halves(double a, double b, double& s2, double& sa, double& sb) {
  a += dpp_d<0xB1>(a);  b += dpp_d<0xB1>(b);
  a += dpp_d<0x4E>(a);  b += dpp_d<0x4E>(b);
  a += dpp_d<0x141>(a); b += dpp_d<0x141>(b);
  a += dpp_d<0x140>(a); b += dpp_d<0x140>(b);
  s2 = (readlane_d(a, 0) + readlane_d(a, 16)) + (readlane_d(a, 32) + readlane_d(a, 48));
  sa = readlane_d(b, 0) + readlane_d(b, 16);
  sb = readlane_d(b, 32) + readlane_d(b, 48);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_d<0x141>(v);   // row_half_mirror
  v += dpp_d<0x140>(v);   // row_mirror
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// the same for u32 (per-lane packed 16-bit counters: the fields do not carry into each other as
// long as every field's total stays below 65536)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}

__device__ __forceinline__ uint32_t wave_sum_dpp_u(uint32_t v) {
  v += dpp_u<0xB1>(v);
  v += dpp_u<0x4E>(v);
  v += dpp_u<0x141>(v);
  v += dpp_u<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// x_k / N == b_k / B bitwise.  Integer backgrounds: exact cross-multiplication (all products
// < 2^53, and for x*B < 2^52 distinct rationals cannot round to the same double); normalised
// backgrounds: the reference's own division.
__device__ __forceinline__ bool prop_ok(uint32_t x, double N, double v, double B, bool floatv) {
  return floatv ? ((double)x / N == v) : ((double)x * B == v * N);
}

__device__ __forceinline__ uint4 ld4(const uint32_t* __restrict__ a, uint32_t i, uint32_t e) {
  return i < e ? *reinterpret_cast<const uint4*>(a + i) : make_uint4(0, 0, 0, 0);
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

__device__ __forceinline__ void write_empty(sfs2d_window* o, uint32_t chrom, uint32_t wid) {
  sfs2d_window r;
  memset(&r, 0, sizeof(r));
  r.chrom = chrom; r.wid = wid; r.flags = SFS2D_W_EMPTY;
  *o = r;
}

// One SNP: filters (position: twoDSFS_class.py:179-182; variant_type: 185-187), the joint fold on
// individual counts (197-206; ties not folded), the (0,0) skip (212-213), raw 1D alt counts
// (428-433) and their fold against 2*pop_size (446-463), restricted to the inner bins that
// bins[1:-1] keeps (486-488, 635).  Returns the packed bins word (see B_VAR / B_LAST).
// k2all / u1a / u1b: the unfolded background histogram words to count (-1: none).
__device__ __forceinline__ uint32_t classify(const KParams& P, uint32_t c, bool var_ok, bool pos_ok, uint32_t& err,
                                            int& k2all, int& u1a, int& u1b) {
  const int r1 = c & 0xff, a1 = (c >> 8) & 0xff, r2 = (c >> 16) & 0xff, a2 = c >> 24;
  const bool pass = var_ok & pos_ok;
  const bool sw = a1 + a2 > P.fold_thr;
  const int x1 = sw ? r1 : a1, x2 = sw ? r2 : a2;
  const bool nz = (x1 | x2) != 0;
  const bool oob = (x1 > P.n1) | (x2 > P.n2);
  const bool ka = a1 > P.n1, kb = a2 > P.n2;
  err |= (pass & nz & oob) ? ERR_GRID : 0u;           // out-of-grid key: unsupported (documented)
  err |= (pass & (ka | kb)) ? ERR_KEY : 0u;            // reference: KeyError in calculate_1d_sfs
  const int k2 = x1 * (P.n2 + 1) + x2;
  const bool in2 = pass & nz & !oob;
  const bool last = in2 & (k2 == P.nb2 - 1);
  const int g1 = min(a1, P.n1 - a1), g2 = min(a2, P.n2 - a2);
  const bool v1a = pass & (a1 != 0) & !ka & (g1 >= 1) & (g1 <= P.n1p - 1);
  const bool v1b = pass & (a2 != 0) & !kb & (g2 >= 1) & (g2 <= P.n2p - 1);
  k2all = in2 ? k2 : -1;
  u1a = (pass & (a1 != 0) & !ka) ? a1 : -1;
  u1b = (pass & (a2 != 0) & !kb) ? a2 : -1;
  return (uint32_t)((in2 & !last) ? k2 : 0) | ((uint32_t)(v1a ? g1 : 0) << 16) | ((uint32_t)(v1b ? g2 : 0) << 23) |
         (var_ok ? B_VAR : 0u) | (last ? B_LAST : 0u);
}

// a wave-uniform value held in a VGPR: k_prep's per-SNP code reads a dozen parameters, and as
// scalars they (with the lane masks of four unrolled SNPs) overflow the SGPR file into v_readlane
// reloads inside the loop
__device__ __forceinline__ int vreg(int x) {
  int r;
  asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(x));
  return r;
}
__device__ __forceinline__ unsigned int vreg(unsigned int x) { return (unsigned int)vreg((int)x); }

// classify() for counts inside the grid (r1 + a1 <= n1 and r2 + a2 <= n2, so no out-of-grid key and
// no KeyError): the same word from fewer, branch-free operations.  x1 = x2 = 0 iff k2 = 0; with
// a1 <= n1, 1 <= min(a1, n1 - a1) <= n1p - 1 is exactly the v1a condition of classify().
__device__ __forceinline__ uint32_t classify_fast(const KParams& P, uint32_t c, bool var_ok, bool pos_ok, int& k2all,
                                                 int& u1a, int& u1b) {
  const uint32_t r1 = c & 0xffu, a1 = (c >> 8) & 0xffu, r2 = (c >> 16) & 0xffu, a2 = c >> 24;
  const bool pass = var_ok & pos_ok;
  const bool sw = (int)(a1 + a2) > P.fold_thr;
  const uint32_t x1 = sw ? r1 : a1, x2 = sw ? r2 : a2;
  const uint32_t k2 = x1 * (uint32_t)(P.n2 + 1) + x2;
  const bool in2 = pass & (k2 != 0u);
  const bool last = in2 & (k2 == (uint32_t)(P.nb2 - 1));
  const uint32_t g1 = min(a1, (uint32_t)P.n1 - a1), g2 = min(a2, (uint32_t)P.n2 - a2);
  const bool v1a = pass & (g1 - 1u < (uint32_t)(P.n1p - 1));
  const bool v1b = pass & (g2 - 1u < (uint32_t)(P.n2p - 1));
  k2all = in2 ? (int)k2 : -1;
  u1a = (pass & (a1 != 0u)) ? (int)a1 : -1;
  u1b = (pass & (a2 != 0u)) ? (int)a2 : -1;
  return ((in2 & !last) ? k2 : 0u) | ((v1a ? g1 : 0u) << 16) | ((v1b ? g2 : 0u) << 23) | (var_ok ? B_VAR : 0u) |
         (last ? B_LAST : 0u);
}

// The bins word of one SNP straight from its packed counts, for the scan kernels of plans without a
// position / variant_type filter ("counts" plans: k_prep writes no bins, the scans classify the
// counts they stream).  Exactly classify()'s word wherever the plan runs without error: counts whose
// key leaves the grid, or above 2*pop_size, make k_prep raise (ERR_GRID / ERR_KEY), and here only
// keep the LDS indices in range (the key is clamped into the excluded last bin).
//   a1 + a2 (one byte dot product) > n1p + n2p -> the fold swaps ref / alt in both populations: the
//   (x1, x2) bytes are then bytes 0 and 2 of the counts, else bytes 1 and 3; k2 = x1 (n2+1) + x2 as
//   one more dot product.
__device__ __forceinline__ uint32_t cls_word(const KParams& P, uint32_t c) {
  const bool sw = (int)__builtin_amdgcn_udot4(c, 0x01000100u, 0u, false) > P.fold_thr;
  const uint32_t x = sw ? c : (c >> 8);
  const uint32_t nb2m1 = (uint32_t)P.nb2 - 1u;
  const uint32_t k2 = min(__builtin_amdgcn_udot4(x, P.kmul, 0u, false), nb2m1);
  const uint32_t a1 = __builtin_amdgcn_ubfe(c, 8, 8), a2 = c >> 24;
  const uint32_t g1 = min(a1, (uint32_t)P.n1 - a1), g2 = min(a2, (uint32_t)P.n2 - a2);
  const uint32_t f1 = g1 - 1u < (uint32_t)(P.n1p - 1) ? g1 : 0u, f2 = g2 - 1u < (uint32_t)(P.n2p - 1) ? g2 : 0u;
  return (k2 == nb2m1 ? B_LAST : k2) | (f1 << 16) | (f2 << 23) | B_VAR;
}

// cls_word's fields without the packing, for the scan kernels' SNP rows: the inner 2D key k2 (0: in no
// inner bin; the excluded last bin and clamped out-of-grid keys included) and both folded inner 1D
// bins, the latter in packed u16 arithmetic (v_perm, v_pk_sub / v_pk_min, a saturating v_pk_sub for the
// range test: 7 operations for the two populations)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ void cls_fields(const KParams& P, uint32_t c, uint32_t& k2, uint32_t& g1, uint32_t& g2,
                                           uint32_t* ktri = nullptr) {
  const bool sw = (int)__builtin_amdgcn_udot4(c, 0x01000100u, 0u, false) > P.fold_thr;
  const uint32_t x = sw ? c : (c >> 8);
  const uint32_t kk = __builtin_amdgcn_udot4(x, P.kmul, 0u, false);
  k2 = kk < (uint32_t)P.nb2 - 1u ? kk : 0u;
  if (ktri) {   // (k_scan_gw TRI) the triangle index, clamped into it (counts outside the grid are an error)
    const uint32_t x1 = x & 0xffu;
    *ktri = min(kk - ((x1 * (x1 - 1u)) >> 1), (uint32_t)P.ntri - 1u);
  }
  const u16x2 a = as_u16x2(__builtin_amdgcn_perm(0u, c, 0x0c030c01u));      // (a1, a2)
  const u16x2 g = __builtin_elementwise_min(a, as_u16x2(P.n12) - a);         // min(a, n - a)
  // 1 <= g <= n_p - 1 <=> lim - (g - 1) > 0 (saturating); keep g there, 0 elsewhere
  const u16x2 v = __builtin_elementwise_sub_sat(as_u16x2(P.lim12), g - (u16x2){1, 1});
  const uint32_t gv = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(g, v * (u16x2){0xffff, 0xffff}));
  g1 = gv & 0xffffu;
  g2 = gv >> 16;
}

// k_scan_w's per-SNP classification: cls_fields' k2, and both folded 1D bins packed (u16 pairs, times BS)
// with no range test -- the excluded bins 0 (fixed in the population) and n_p (MAF 1/2) are counted like the
// others and dropped at the window's end; counts above 2 pop_size (an error k_prep reports) clamp to n_p
template <uint32_t BS>   // gp in bytes: the bins times BS (the LDS bytes per 1D bin)
__device__ __forceinline__ void cls_k2g(const KParams& P, uint32_t c, uint32_t& k2, uint32_t& gp) {
  const bool sw = (int)__builtin_amdgcn_udot4(c, 0x01000100u, 0u, false) > P.fold_thr;
  const uint32_t x = sw ? c : (c >> 8);
  const uint32_t kk = __builtin_amdgcn_udot4(x, P.kmul, 0u, false);
  k2 = kk < (uint32_t)P.nb2 - 1u ? kk : 0u;
  const u16x2 a = as_u16x2(__builtin_amdgcn_perm(0u, c, 0x0c030c01u));      // (a1, a2)
  const u16x2 g = __builtin_elementwise_min(a, as_u16x2(P.n12) - a);         // min(a, n - a)
  const u16x2 np = {(unsigned short)P.n1p, (unsigned short)P.n2p};
  gp = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(g, np) * (u16x2){(unsigned short)BS, (unsigned short)BS});
}

// the per-SNP source of the scan kernels: the bins k_prep wrote, or (CNT) the counts, classified
template <bool CNT>
__device__ __forceinline__ uint32_t snp_word(const KParams& P, const uint32_t* __restrict__ src, uint32_t i) {
  return CNT ? cls_word(P, src[i]) : src[i];
}

// counts plans: a window's rows as a buffer resource based at its first SNP b, covering [b, e) (and
// not past the data set's last SNP): the range check returns 0 past the window's end -- an SNP in no
// spectrum with no called allele -- so the rows need no masking, no clamp and no per-row address
// arithmetic (the rows sit in the loads' immediate offsets).  b, e are wave-uniform: scalar work.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t window_rows(const uint32_t* counts, uint32_t b, uint32_t e, uint32_t nm1) {
  const uint32_t left = min(min(e, nm1 + 1u) - b, 0x3fffffffu);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(counts + b), (short)0, (int)(left * 4u), 0x00020000);
}

__device__ __forceinline__ uint32_t bin_k2(uint32_t w) { return w & 0xffffu; }
__device__ __forceinline__ uint32_t bin_g1(uint32_t w) { return (w >> 16) & 0x7fu; }
__device__ __forceinline__ uint32_t bin_g2(uint32_t w) { return (w >> 23) & 0x7fu; }

// ------------------------------------------------------------------------------------------ K0

// ln k for k < LNX_N; F(x) = x ln x for x < LNT; D(r) = F(r+1) - F(r) for r < LNT-1 and
// D(LNT-1) = 0 (k_scan_w adds the ranks from LNT-1 on per bin, as F(x) - F(LNT-1))
__global__ void k_init_lnx(double* lnx, double* dtab, double* ftab, double* rtab) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < LNX_N) lnx[i] = i ? log((double)i) : 0.0;
  if (i < RCPN) {   // Fst: (1/n, 1/(n(n-1))) per called allele count n; 0 below n = 2 (not in the set)
    rtab[2 * i] = i >= 2 ? 1.0 / (double)i : 0.0;
    rtab[2 * i + 1] = i >= 2 ? 1.0 / ((double)i * (double)(i - 1)) : 0.0;
  }
  if (i < LNT) {
    const double a = i ? (double)i * log((double)i) : 0.0;
    const double b = (double)(i + 1) * log((double)(i + 1));
    dtab[i] = i < LNT - 1 ? b - a : 0.0;
    ftab[i] = a;
  }
}

// the largest called allele counts r1 + a1 / r2 + a2 over a data set (sfs2d_data_wrap_device: whether a
// counts plan may skip validating the counts) and whether some SNP has < 2 called alleles in a population
// (whether Fst summed in the scan must mask such SNPs); m[3] zeroed by the caller
__global__ __launch_bounds__(256) void k_max_called(const uint32_t* __restrict__ counts, unsigned long long n,
                                                    uint32_t* __restrict__ m) {
  uint32_t m1 = 0, m2 = 0;
  bool low = false;   // m[2]: some SNP with < 2 called alleles in a population
  for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (unsigned long long)gridDim.x * 256) {
    const uint32_t c = counts[i];
    const uint32_t n1c = __builtin_amdgcn_udot4(c, 0x00000101u, 0u, false), n2c = __builtin_amdgcn_udot4(c, 0x01010000u, 0u, false);
    m1 = max(m1, n1c);
    m2 = max(m2, n2c);
    low |= min(n1c, n2c) < 2u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    m1 = max(m1, (uint32_t)__shfl_xor((int)m1, o, WAVE));
    m2 = max(m2, (uint32_t)__shfl_xor((int)m2, o, WAVE));
  }
  const bool any_low = __ballot(low) != 0ull;
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    atomicMax(&m[0], m1);
    atomicMax(&m[1], m2);
    if (any_low) atomicMax(&m[2], 1u);
  }
}

// ------------------------------------------------------------------------------------------ background rows
// A plan's per-chromosome background histograms as int64 rows (the multi-GPU exchange, sfs2d/dist.py):
// row c = [nb2 2D bins | n1+1 unfolded pop-1 | n2+1 unfolded pop-2 | inner 2D sum] = SFS2D_BG_ROW_WORDS.
// get: the REPL replicas of this run's k_prep pass summed (read only); set: the summed rows of every
// rank back into replica 0 (the others and the padding zeroed) and the inner sums, before the scan.
// Grid (ceil(W / 256), nchrom).
__global__ __launch_bounds__(256) void k_bg_rows_get(KParams P, const uint32_t* __restrict__ repl, unsigned long long rs,
                                                     const uint32_t* __restrict__ bsum, long long* __restrict__ rows,
                                                     long long stride) {
  const int c = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
  const int W = P.h1b + P.n2 + 2;
  if (k >= W) return;
  long long v;
  if (k == W - 1) {
    v = (long long)bsum[c];
  } else {
    const uint32_t* q = repl + (size_t)c * P.nh + k;
    v = 0;
#pragma unroll
    for (int r = 0; r < REPL; ++r) v += (long long)q[(size_t)r * rs];
  }
  rows[(size_t)c * stride + k] = v;
}

__global__ __launch_bounds__(256) void k_bg_rows_set(KParams P, uint32_t* __restrict__ repl, unsigned long long rs,
                                                     uint32_t* __restrict__ bsum, const long long* __restrict__ rows,
                                                     long long stride, uint32_t* __restrict__ err_word) {
  const int c = blockIdx.y, k = blockIdx.x * 256 + threadIdx.x;
  const int W = P.h1b + P.n2 + 2;
  if (k >= P.nh && k != W - 1) return;
  const long long v = k < W ? rows[(size_t)c * stride + k] : 0;
  if (v < 0 || v > 0xffffffffll) atomicOr(err_word, ERR_OVF);
  if (k == W - 1) {
    bsum[c] = (uint32_t)v;
    if (k >= P.nh) return;
  }
  uint32_t* q = repl + (size_t)c * P.nh + k;
  q[0] = k < W - 1 ? (uint32_t)v : 0u;
#pragma unroll
  for (int r = 1; r < REPL; ++r) q[(size_t)r * rs] = 0u;
}

// ------------------------------------------------------------------------------------------ K1

// Per-SNP Fst terms (see fst_terms below for the definition) from the raw counts.  Hudson's terms in
// the form num = A1 + A2 - 2 p1 p2, den = p1 + p2 - 2 p1 p2 with p = a / n and
// A = p^2 - p(1-p)/(n-1) = a(a-1) / (n(n-1)); rt[n] = (1/n, 1/(n(n-1))) (0 for n < 2).  A SNP outside
// the set takes a = 0 (num = den = 0).
__device__ __forceinline__ void fst_snp(uint32_t c, bool member, const double2* rt, double& num, double& den) {
  const uint32_t r1 = c & 0xffu, a1 = (c >> 8) & 0xffu, r2 = (c >> 16) & 0xffu, a2 = c >> 24;
  const uint32_t n1c = r1 + a1, n2c = r2 + a2;             // u8 counts: n <= 510 < RCPN
  const bool ok = member & (n1c >= 2u) & (n2c >= 2u);
  const uint32_t b1 = ok ? a1 : 0u, b2 = ok ? a2 : 0u;
  const double2 q1 = rt[n1c], q2 = rt[n2c];
  const double p1 = (double)b1 * q1.x, p2 = (double)b2 * q2.x;
  const double A1 = (double)__umul24(b1, b1 - 1u) * q1.y, A2 = (double)__umul24(b2, b2 - 1u) * q2.y;
  const double m = p1 * p2;
  num = fma(-2.0, m, A1 + A2);
  den = fma(-2.0, m, p1 + p2);
}

// x * scale rounded to the nearest integer, |x * scale| < 2^51 (the magic-number conversion:
// 1.5 * 2^52 pins the exponent, the low mantissa bits then hold the integer); scale <= 2^FST_E_MAX
// and the Fst terms are within [-1, 1]
__device__ __forceinline__ unsigned long long fst_fixed(double x, double scale) {
  const double y = fma(x, scale, 6755399441055744.0);
  return (unsigned long long)(__double_as_longlong(y) - 0x4338000000000000ll);
}

// k_prep's work on one tile t (work item ti: its replica is ti % REPL), by a 512-thread workgroup whose
// dynamic LDS starts at sh_hist
template <bool DO_BG, bool DO_SEG, bool LDS_HIST, bool DO_BINS, bool FILT, bool FST>
__device__ __forceinline__ void prep_tile(const KParams& P, const Tile t, uint32_t ti, uint32_t* sh_hist,
                                          const uint32_t* __restrict__ counts, const uint32_t* __restrict__ pos,
                                          const uint16_t* __restrict__ ann, uint32_t* __restrict__ repl,
                                          uint2* __restrict__ slots, uint32_t* __restrict__ bins,
                                          uint32_t* __restrict__ bcount, uint32_t* __restrict__ err_word, int hr,
                                          const double2* __restrict__ rcp_g, unsigned long long* __restrict__ fsum) {
  // repl / bcount: this run's parity buffers.  LDS histogram: hr interleaved copies of every word
  // (lane & (hr-1) picks one), which spreads the many same-bin atomics of a wavefront over banks.
  __shared__ uint32_t sh_b2;
  // FST: per-window sums of the Fst terms, int64 fixed point (num, den) for the tile's first
  // FST_LDS windows (FST_R copies each), the rest straight to the global per-slot sums
  __shared__ unsigned long long sh_fst[FST ? 2 * FST_R * FST_LDS : 1];
  // the fast path's called counts are in the grid (n <= 2*pop_size <= 254): half the table in LDS;
  // the exact path (any u8 counts, n <= 510) reads the global table
  __shared__ double2 sh_rcp[FST ? RCPN / 2 : 1];
  __shared__ uint32_t sh_wlo;
  // JNT (P.jnt = nb2 words, plans whose k_prep only histograms and segments): the common step counts
  // every SNP once in the joint histogram of its unfolded alt counts (alt1, alt2), laid out as the 2D
  // grid, and a folded SNP once more in the 2D histogram at its (ref1, ref2) key: 1 + (folded) LDS
  // atomics per SNP instead of 3 (2D key, both unfolded 1D spectra).  The tile's end derives both 1D
  // spectra as the joint histogram's margins and adds its bins with alt1 + alt2 <= fold_thr -- the
  // unfolded SNPs' 2D keys -- to the 2D histogram (the edge steps' process() counts the three directly)
  constexpr bool JNT = DO_BG && LDS_HIST && !DO_BINS && !FST;
  const bool jnt = JNT && P.jnt != 0;
  STAMP(20);
  BLK_STAMP(0, 0);
  uint32_t* gh = repl + ((size_t)(ti % REPL) * P.nchrom + t.chrom) * (size_t)P.nh;
  const int lane0 = threadIdx.x & (WAVE - 1);
  const int hsh = LDS_HIST ? (hr == 4 ? 2 : 0) : 0;
  const int rep = lane0 & (hr - 1);
  const int trash = P.nh * hr + lane0;   // LDS word after the histogram (64 of them)
  if (FST) {
    for (int k = threadIdx.x; k < 2 * FST_R * FST_LDS; k += BLOCK1) sh_fst[k] = 0ull;
    for (int k = threadIdx.x; k < RCPN / 2; k += BLOCK1) sh_rcp[k] = rcp_g[k];
    if (threadIdx.x == 0) sh_wlo = DO_SEG ? wid_fast(P, pos[t.begin]) : div_fast(P, t.begin - t.cb);
  }
  if (DO_BG) {
    if (LDS_HIST)
      for (int k = threadIdx.x; k < P.nh * hr + WAVE + (JNT ? P.jnt : 0); k += BLOCK1) sh_hist[k] = 0u;
    if (threadIdx.x == 0) sh_b2 = 0u;
  }
  if (DO_SEG) {
    // the slot table is rewritten every run, so that no kernel needs to clear it after reading (the
    // scans' scattered 8-B stores, one per window): this tile first clears, with coalesced stores, the
    // slots strictly between its first SNP's window and the next tile's first SNP's window (from slot 0
    // in a chromosome's first tile, to the chromosome's last slot in its last one).  Only this tile's
    // SNPs fall in those windows (it writes their ends below, after the barrier); the windows at the
    // edges hold SNPs of two tiles and get both ends written by them, so no tile clears them.
    const uint32_t wf = wid_fast(P, pos[t.begin]);
    const uint32_t lo = t.begin == t.cb ? 0u : wf + 1u;
    const uint32_t hi = t.end == t.ce ? t.nslots : wid_fast(P, pos[t.end]);
    for (uint32_t s = lo + threadIdx.x; s < hi; s += BLOCK1)
      if (s != wf) slots[(size_t)t.sbase + s] = make_uint2(0u, 0u);
  }
  if (DO_BG || FST || DO_SEG) __syncthreads();
  const uint32_t wlo = FST ? sh_wlo : 0u;
  // fixed-point add of one lane's (num, den) pair into window wid of this chromosome
  const int frep = threadIdx.x & (FST_R - 1);
  auto fst_add = [&](uint32_t wid, double num, double den) {
    const unsigned long long qn = fst_fixed(num, P.fst_scale), qd = fst_fixed(den, P.fst_scale);
    if ((qn | qd) == 0ull) return;
    const uint32_t j = wid - wlo;
    if (j < (uint32_t)FST_LDS) {
      atomicAdd(&sh_fst[2 * (j * FST_R + frep)], qn);
      atomicAdd(&sh_fst[2 * (j * FST_R + frep) + 1], qd);
    } else {
      atomicAdd(&fsum[2 * ((size_t)t.sbase + wid)], qn);
      atomicAdd(&fsum[2 * ((size_t)t.sbase + wid) + 1], qd);
    }
  };
  // FILT: a position or variant_type filter is set (kept out of the common kernel: its uniform
  // flags would otherwise occupy scalar registers throughout the loop)
  const bool pos_filter = FILT && (P.has_start || P.has_end);
  const bool need_pos = DO_SEG || pos_filter;
  const bool filt = FILT && P.ann_want >= 0;
  const int lane = threadIdx.x & (WAVE - 1);
  uint32_t err = 0, b2 = 0;
  STAMP(21);

  // one 16-B vector = 4 consecutive SNPs; elements outside [t.begin, t.end) are masked.
  // wprev / wnext: window ids of the SNPs just before / after the vector.
  // EDGE: the step reaches past the tile (elements outside [t.begin, t.end) are masked);
  // FAST: no lane of the wave holds counts outside the grid (classify_fast)
  KParams Q = P;   // the per-SNP parameters as VGPR copies (vreg)
  Q.n1 = vreg(P.n1); Q.n2 = vreg(P.n2); Q.n1p = vreg(P.n1p); Q.n2p = vreg(P.n2p); Q.nb2 = vreg(P.nb2);
  Q.fold_thr = vreg(P.fold_thr); Q.h1a = vreg(P.h1a); Q.h1b = vreg(P.h1b);
  Q.wmag = vreg(P.wmag); Q.wsh1 = vreg(P.wsh1); Q.wsh2 = vreg(P.wsh2);
  auto process = [&](auto EDGE_C, auto FAST_C, uint32_t i0, const uint4& cv, const uint4& pv, const uint2& av,
                     uint32_t wprev, uint32_t wnext) {
    constexpr bool EDGE = decltype(EDGE_C)::value, FAST = decltype(FAST_C)::value;
    const uint32_t cc[4] = {cv.x, cv.y, cv.z, cv.w};
    const uint32_t pp[4] = {pv.x, pv.y, pv.z, pv.w};
    const uint32_t aa[4] = {av.x & 0xffffu, av.x >> 16, av.y & 0xffffu, av.y >> 16};
    uint32_t w[4];
    if (DO_SEG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = wid_fast(Q, pp[k]);
    }
    uint32_t bw[4];
    uint32_t segcode = 0;   // bit 2k: SNP k opens a window, bit 2k+1: it closes one
    // Fst: the terms of the four SNPs; one fixed-point add for the lane when they share a window
    uint32_t fw[4];
    bool fm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t i = i0 + k;
      const bool in = EDGE ? (i >= t.begin) & (i < t.end) : true;
      bool var_ok = in, pos_ok = true;
      if (filt) var_ok = in & ((int)aa[k] == P.ann_want);
      if (pos_filter) {
        const long long p = (long long)pp[k];
        pos_ok = (!P.has_start | (p >= P.start_pos)) & (!P.has_end | (p <= P.end_pos));
      }
      int k2all, u1a, u1b;
      bw[k] = FAST ? classify_fast(Q, cc[k], var_ok, pos_ok, k2all, u1a, u1b)
                   : classify(P, cc[k], var_ok, pos_ok, err, k2all, u1a, u1b);
      if (FST) {
        fw[k] = DO_SEG ? w[k] : div_fast(Q, i - t.cb);
        fm[k] = in & (k2all >= 0) & (DO_SEG | (fw[k] < t.nslots));   // fixed-SNP windows: the tail is dropped
      }
      if (DO_BG) {
        if (LDS_HIST) {
          // no branches: skipped SNPs add to the lane's trash word (keeps exec masks, and the
          // scalar registers they take, out of the unrolled loop)
          atomicAdd(&sh_hist[(in & (k2all >= 0)) ? (k2all << hsh) + rep : trash], 1u);
          atomicAdd(&sh_hist[(in & (u1a >= 0)) ? ((Q.h1a + u1a) << hsh) + rep : trash], 1u);
          atomicAdd(&sh_hist[(in & (u1b >= 0)) ? ((Q.h1b + u1b) << hsh) + rep : trash], 1u);
        } else if (in) {
          if (k2all >= 0) atomicAdd(&gh[k2all], 1u);
          if (u1a >= 0) atomicAdd(&gh[P.h1a + u1a], 1u);
          if (u1b >= 0) atomicAdd(&gh[P.h1b + u1b], 1u);
        }
        b2 += (in & (bin_k2(bw[k]) != 0)) ? 1u : 0u;
      }
      if (DO_SEG) {
        // window id (pos-1)//ws: the reference's start += ws*((pos-start)//ws) from start=1 (:894, :948)
        const uint32_t qp = k ? w[k - 1] : wprev;
        const uint32_t qn = k < 3 ? w[k + 1] : wnext;
        const bool first = in & ((i == t.cb) | (qp != w[k]));
        const bool last = in & ((i + 1 == t.ce) | (qn != w[k]));
        segcode |= (first ? 1u : 0u) << (2 * k) | (last ? 2u : 0u) << (2 * k);
      }
      __builtin_amdgcn_sched_barrier(0);   // one SNP at a time: its lane masks die before the next
    }
    if (FST) {   // per SNP (edge steps: masked SNPs may carry any window id)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double nk, dk;
        fst_snp(cc[k], fm[k], rcp_g, nk, dk);
        if (fm[k]) fst_add(fw[k], nk, dk);
      }
    }
    // window boundaries are rare: one divergent pass over the set bits
    if (DO_SEG && segcode) {
      for (uint32_t c = segcode; c; c &= c - 1) {
        const int bit = __builtin_ctz(c), k = bit >> 1;
        const uint32_t wk = k == 0 ? w[0] : k == 1 ? w[1] : k == 2 ? w[2] : w[3];
        uint32_t* sl = reinterpret_cast<uint32_t*>(slots + ((size_t)t.sbase + wk));
        sl[bit & 1] = i0 + k + 1u;   // .x = first + 1, .y = last + 1 (0: an empty slot)
      }
    }
    if (DO_BINS) {
      if (!EDGE || (i0 >= t.begin && i0 + 4 <= t.end)) {
        *reinterpret_cast<uint4*>(bins + i0) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i0 + k >= t.begin && i0 + k < t.end) bins[i0 + k] = bw[k];
      }
    }
  };

  // one 16-B vector of counts (+ positions) per thread per step; loads are clamped into the tile
  // (lanes past its end re-read its last vector, masked) so that no load sits behind a branch; the
  // lanes at the wave edges fetch their neighbour positions in the same batch
  // The common step (not a tile's first or last, every count inside the grid, no filter): classify_fast
  // inline with precomputed LDS byte offsets, and window-boundary bookkeeping only in lanes whose
  // neighbours differ.  Everything else goes through process() above.
  constexpr bool FASTOK = !FILT && (!DO_BG || LDS_HIST);
  const uint32_t s2 = (uint32_t)hsh + 2u;                        // bin -> byte offset shift
  uint32_t* const hist_l = sh_hist + rep;                        // this lane's histogram copy
  uint32_t* const h1a_l = hist_l + ((uint32_t)P.h1a << hsh);
  uint32_t* const h1b_l = hist_l + ((uint32_t)P.h1b << hsh);
  uint32_t* const trash_p = sh_hist + trash;
  uint32_t* const jh_l = sh_hist + P.nh * hr + WAVE;             // JNT: the joint histogram
  const uint32_t n2p1 = vreg(P.n2 + 1), nb2m1 = vreg(P.nb2 - 1), n1pm1 = vreg(P.n1p - 1), n2pm1 = vreg(P.n2p - 1);
  auto process_fast = [&](uint32_t i0, const uint4& cv, const uint4& pv, uint32_t wprev, uint32_t wnext) {
    const uint32_t cc[4] = {cv.x, cv.y, cv.z, cv.w};
    const uint32_t pp[4] = {pv.x, pv.y, pv.z, pv.w};
    uint32_t w[4], bw[4];
    if (DO_SEG) {
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = wid_fast(Q, pp[k]);
    }
    uint32_t fw[4];
    bool fm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t c = cc[k];
      if (JNT && jnt) {
        if (!(SFS2D_ABL & 64)) {
          const uint32_t ka = __builtin_amdgcn_udot4(c >> 8, Q.kmul, 0u, false);   // a1 (n2+1) + a2
          const uint32_t kr = __builtin_amdgcn_udot4(c, Q.kmul, 0u, false);        // r1 (n2+1) + r2
          const bool sw = (int)__builtin_amdgcn_udot4(c, 0x01000100u, 0u, false) > Q.fold_thr;
          atomicAdd(ka ? (uint32_t*)((char*)jh_l + (ka << 2)) : trash_p, 1u);
          atomicAdd((sw & (kr != 0u)) ? (uint32_t*)((char*)hist_l + (kr << 2)) : trash_p, 1u);
        }
        continue;
      }
      const uint32_t r1 = c & 0xffu, a1 = (c >> 8) & 0xffu, r2 = (c >> 16) & 0xffu, a2 = c >> 24;
      const bool sw = (int)(a1 + a2) > Q.fold_thr;
      const uint32_t x1 = sw ? r1 : a1, x2 = sw ? r2 : a2;
      const uint32_t k2 = __umul24(x1, n2p1) + x2;                 // 0 iff (x1, x2) = (0, 0)
      const bool in2 = k2 != 0u, last = k2 == nb2m1;
      const uint32_t g1 = min(a1, (uint32_t)Q.n1 - a1), g2 = min(a2, (uint32_t)Q.n2 - a2);
      const uint32_t f1 = g1 - 1u < n1pm1 ? g1 : 0u, f2 = g2 - 1u < n2pm1 ? g2 : 0u;
      bw[k] = (last ? B_LAST : k2) | (f1 << 16) | (f2 << 23) | B_VAR;
      if (DO_BG && !(SFS2D_ABL & 64)) {
        atomicAdd(in2 ? (uint32_t*)((char*)hist_l + (k2 << s2)) : trash_p, 1u);
        atomicAdd(a1 ? (uint32_t*)((char*)h1a_l + (a1 << s2)) : trash_p, 1u);
        atomicAdd(a2 ? (uint32_t*)((char*)h1b_l + (a2 << s2)) : trash_p, 1u);
        b2 += (in2 & !last) ? 1u : 0u;
      }
      if (FST) {
        fw[k] = DO_SEG ? w[k] : div_fast(Q, i0 + k - t.cb);
        fm[k] = in2 & (DO_SEG | (fw[k] < t.nslots));
      }
    }
    if (FST) {
      // the lane's four SNPs in order, one running (num, den) pair per window: a fixed-point add
      // whenever the window changes (rare) and one at the end
      double sn = 0.0, sd = 0.0;
      uint32_t wc = fw[0];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        double nk, dk;
        fst_snp(cc[k], fm[k], sh_rcp, nk, dk);
        if (k && fw[k] != wc) {
          fst_add(wc, sn, sd);
          sn = 0.0; sd = 0.0; wc = fw[k];
        }
        sn += nk; sd += dk;
      }
      fst_add(wc, sn, sd);
    }
    // window boundaries: ids are non-decreasing along the tile, so a lane holds one iff its
    // neighbours' ids differ (rare)
    if (DO_SEG && wprev != wnext) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t qp = k ? w[k - 1] : wprev, qn = k < 3 ? w[k + 1] : wnext;
        uint32_t* sl = reinterpret_cast<uint32_t*>(slots + ((size_t)t.sbase + w[k]));
        if (qp != w[k]) sl[0] = i0 + k + 1u;   // .x = first + 1, .y = last + 1
        if (qn != w[k]) sl[1] = i0 + k + 1u;
      }
    }
    if (DO_BINS) *reinterpret_cast<uint4*>(bins + i0) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
  };

  constexpr uint32_t STEP = 4 * BLOCK1;
  const uint32_t ab = t.begin & ~3u, alast = (t.end - 1u) & ~3u;
  // (a segmentation-only pass -- a supplied background, no bins, no Fst -- reads no counts)
  constexpr bool NEED_C = DO_BG || DO_BINS || FST;
  // the step's vectors (and the wave-edge neighbour positions) are loaded one step ahead: HBM-sized
  // streams keep two steps of loads in flight per wave (SFS2D_PREP_PREFETCH=0 at compile time: one)
  struct StepIn {
    uint4 c, p;
    uint2 a;
    uint32_t xp, xn;
  };
  // counts / positions through buffer resources covering the tile's vectors [ab, alast + 4): a load past
  // them (the last step's lanes beyond the tile, the unconditional reload of the step after the last)
  // returns 0 with no memory access -- clamped to the last vector instead, those re-reads cost small
  // tiles (config 2: 4,096 SNPs, two steps) half as many bytes again in fetches
  const uint32_t tbytes = (alast + 4u - ab) * 4u;
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(counts + ab), (short)0, (int)tbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(pos + ab), (short)0, (int)tbytes, 0x00020000);
  auto load_step = [&](uint32_t base) {
    StepIn x;
    const uint32_t ia = base + 4 * threadIdx.x;
    const int off = (int)((ia - ab) * 4u);
    x.c = NEED_C ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(crs, off, 0, 0)) : make_uint4(0, 0, 0, 0);
    x.p = need_pos ? __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(prs, off, 0, 0)) : make_uint4(0, 0, 0, 0);
    x.a = filt ? *reinterpret_cast<const uint2*>(ann + min(ia, alast)) : make_uint2(0, 0);
    x.xp = 0;
    x.xn = 0;
    if (DO_SEG) {   // neighbour positions at the wave edges and past the tile end
      // (buffer loads on the chromosome's positions, issued by every lane, out of range -- 0, no
      // access -- where no neighbour is needed: no branch around them, so the count of loads in
      // flight is the same on every path and a step waits only for its own buffer)
      const __amdgpu_buffer_rsrc_t pr =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(pos + t.cb), (short)0, (int)((t.ce - t.cb) * 4u), 0x00020000);
      const uint32_t none = (t.ce - t.cb) * 4u;
      const bool edge_next = lane == WAVE - 1 || ia + 4 >= t.end;
      const uint32_t op = (lane == 0 && ia > t.cb) ? (min(ia, alast + 4u) - 1u - t.cb) * 4u : none;
      const uint32_t on = (edge_next && ia + 4 < t.ce) ? (ia + 4u - t.cb) * 4u : none;
      x.xp = __builtin_amdgcn_raw_buffer_load_b32(pr, (int)op, 0, 0);
      x.xn = __builtin_amdgcn_raw_buffer_load_b32(pr, (int)on, 0, 0);
    }
    return x;
  };
  // one step of the tile: the SNPs [base, base + STEP), from its loaded vectors
  auto body = [&](uint32_t base, const StepIn& cur) {
    const uint32_t ia = base + 4 * threadIdx.x;
    const uint4 ca = cur.c, pa = cur.p;
    const uint2 aav = cur.a;
    uint32_t wpa = 0, wna = 0;
    if (DO_SEG) {
      const uint32_t xa_prev = cur.xp, xa_next = cur.xn;
      const bool edge_next = lane == WAVE - 1 || ia + 4 >= t.end;
      wpa = __shfl_up(wid_fast(P, pa.w), 1, WAVE);
      wna = __shfl_down(wid_fast(P, pa.x), 1, WAVE);
      if (lane == 0) wpa = wid_fast(P, xa_prev);
      if (edge_next) wna = wid_fast(P, xa_next);
    }
    // counts outside the grid (r + a > n: an error or an out-of-grid key) take the exact classify()
    // (called allele counts r + a by byte dot products)
    auto nc1 = [](uint32_t c) { return __builtin_amdgcn_udot4(c, 0x00000101u, 0u, false); };
    auto nc2 = [](uint32_t c) { return __builtin_amdgcn_udot4(c, 0x01010000u, 0u, false); };
    const bool bad = (int)(max(max(nc1(ca.x), nc1(ca.y)), max(nc1(ca.z), nc1(ca.w))) > (uint32_t)P.n1) |
                     (int)(max(max(nc2(ca.x), nc2(ca.y)), max(nc2(ca.z), nc2(ca.w))) > (uint32_t)P.n2);
    // the masked edge path: a step reaching outside the tile (only a chromosome's first / last tile
    // has unaligned ends: the host puts tile edges on multiples of 4 SNPs) or holding the
    // chromosome's first or last SNP (window starts / ends there whatever the neighbours' ids)
    const bool edge = base < t.begin || base + STEP > t.end || base <= t.cb || base + STEP >= t.ce;   // block-uniform
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (!FASTOK || edge || __ballot(bad)) process(T_{}, F_{}, ia, ca, pa, aav, wpa, wna);   // exact, masked
    else {
#ifdef SFS2D_MARK
      asm volatile("; HOT_BEGIN");
#endif
      if (SFS2D_ABL & 128) asm volatile("" ::"v"(ca.x), "v"(ca.y), "v"(ca.z), "v"(ca.w), "v"(pa.x), "v"(pa.w), "v"(wpa), "v"(wna));
      else process_fast(ia, ca, pa, wpa, wna);
#ifdef SFS2D_MARK
      asm volatile("; HOT_END");
#endif
    }
  };
#if SFS2D_PREP_PREFETCH >= 2
  // two steps of loads in flight per wave: two buffers in turn (loop unrolled by two, so that no
  // buffer is copied while its loads are pending), each reloaded for the step after next once its
  // step is done.  The reloads are unconditional (past the tile they re-read its last vector, never
  // used): with a path-independent count of loads in flight the compiler waits for exactly the
  // buffer a step needs (vmcnt(n)), not for all of them
  StepIn bufA = load_step(ab), bufB = load_step(ab + STEP);
  for (uint32_t base = ab; base < t.end; base += 2 * STEP) {
    body(base, bufA);
    bufA = load_step(base + 2 * STEP);
    if (base + STEP >= t.end) break;
    body(base + STEP, bufB);
    bufB = load_step(base + 3 * STEP);
  }
#else
  StepIn nxt = load_step(ab);
  for (uint32_t base = ab; base < t.end; base += STEP) {
#if SFS2D_PREP_PREFETCH
    const StepIn cur = nxt;
    if (base + STEP < t.end) nxt = load_step(base + STEP);   // block-uniform
#else
    const StepIn cur = base == ab ? nxt : load_step(base);
#endif
    body(base, cur);
  }
#endif
  STAMP(22);
  if (err) atomicOr(err_word, err);
  if (DO_BG && !jnt) {
    b2 = wave_sum_u(b2);
    if (lane == 0 && b2) atomicAdd(&sh_b2, b2);
  }
  if (DO_BG || FST) __syncthreads();
  if (JNT && jnt) {
    // the joint histogram's margins into the 1D spectra, its unfolded keys into the 2D bins; the inner
    // 2D count (bins 1 .. nb2-2) from the finished tile histogram (edge-step SNPs included)
    const uint32_t n2p1 = (uint32_t)P.n2 + 1u;
    uint32_t bs = 0;
    for (int k = threadIdx.x; k < P.nb2; k += BLOCK1) {
      const uint32_t j = jh_l[k];
      const uint32_t x1 = (uint32_t)k / n2p1, x2 = (uint32_t)k - x1 * n2p1;
      if (j) {
        if (x1) atomicAdd(&sh_hist[P.h1a + (int)x1], j);
        if (x2) atomicAdd(&sh_hist[P.h1b + (int)x2], j);
      }
      const uint32_t v = sh_hist[k] + ((int)(x1 + x2) <= P.fold_thr ? j : 0u);
      if (k) sh_hist[k] = v;
      if (k >= 1 && k <= P.nb2 - 2) bs += v;
    }
    bs = wave_sum_u(bs);
    if (lane == 0 && bs) atomicAdd(&sh_b2, bs);
    __syncthreads();
  }
  if (FST)
    for (int j = threadIdx.x; j < FST_LDS; j += BLOCK1) {
      unsigned long long qn = 0, qd = 0;
#pragma unroll
      for (int r = 0; r < FST_R; ++r) {
        qn += sh_fst[2 * (j * FST_R + r)];
        qd += sh_fst[2 * (j * FST_R + r) + 1];
      }
      if (qn | qd) {
        atomicAdd(&fsum[2 * ((size_t)t.sbase + wlo + j)], qn);
        atomicAdd(&fsum[2 * ((size_t)t.sbase + wlo + j) + 1], qd);
      }
    }
  if (DO_BG) {
    if (LDS_HIST)
      for (int k = threadIdx.x; k < P.nh; k += BLOCK1) {
        uint32_t v;
        if (hr == 4) {
          const uint4 q = *reinterpret_cast<const uint4*>(sh_hist + 4 * k);
          v = q.x + q.y + q.z + q.w;
        } else {
          v = sh_hist[k];
        }
        if (v) atomicAdd(&gh[k], v);
      }
    if (threadIdx.x == 0 && sh_b2) atomicAdd(&bcount[t.chrom], sh_b2);
  }
  STAMP(23);
  BLK_STAMP(0, 1);
}

template <bool DO_BG, bool DO_SEG, bool LDS_HIST, bool DO_BINS, bool FILT, bool FST>
__global__ __launch_bounds__(BLOCK1) void k_prep(KParams P, const uint32_t* __restrict__ counts,
                                                 const uint32_t* __restrict__ pos, const uint16_t* __restrict__ ann,
                                                 const Tile* __restrict__ tiles, uint32_t* __restrict__ repl,
                                                 uint2* __restrict__ slots, uint32_t* __restrict__ bins,
                                                 uint32_t* __restrict__ bcount, uint32_t* __restrict__ err_word,
                                                 int hr, const double2* __restrict__ rcp_g,
                                                 unsigned long long* __restrict__ fsum) {
  extern __shared__ uint32_t sh_hist[];
  prep_tile<DO_BG, DO_SEG, LDS_HIST, DO_BINS, FILT, FST>(P, tiles[blockIdx.x], blockIdx.x, sh_hist, counts, pos, ann,
                                                         repl, slots, bins, bcount, err_word, hr, rcp_g, fsum);
}


// Fst per fixed-bp window, one wavefront per window (windows wave_id, wave_id + nwaves, ...): the
// window's SNPs from its slot record (k_prep's segmentation), membership from the packed bins (in
// the 2D SFS, the excluded last bin included), terms by fst_snp, fp64 lane sums in a fixed order and
// one DPP reduction (deterministic).  Used instead of k_prep's per-SNP fixed-point sums where the
// GPU has idle capacity: extra workgroups of k_bg_slice (sliced plans), or k_fst_win alone.
// CNT: membership from the counts themselves (counts plans write no bins)
template <bool CNT>
__device__ __forceinline__ void fst_windows(const KParams& P, const uint32_t* __restrict__ counts,
                                            const uint32_t* __restrict__ bins, const uint2* __restrict__ slots,
                                            const double2* __restrict__ rt, double* __restrict__ fst_out,
                                            uint32_t nslots, uint32_t wave_id, uint32_t nwaves) {
  const int lane = threadIdx.x & (WAVE - 1);
  for (uint32_t s = wave_id; s < nslots; s += nwaves) {
    const uint2 sr = slots[s];
    if (sr.x == 0u) {
      if (lane == 0) fst_out[s] = __builtin_nan("");
      continue;
    }
    const uint32_t b = sr.x - 1u, e = sr.y;
    double sn = 0.0, sd = 0.0;
    // rows of 64 SNPs, eight rows' loads in flight at a time (a window is ~6 rows at 20 kb)
    for (uint32_t r0 = b; r0 < e; r0 += 8 * WAVE) {
      uint32_t c[8], w[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t i = r0 + 64 * j + lane;
        c[j] = i < e ? counts[i] : 0u;
        if (!CNT) w[j] = i < e ? bins[i] : 0u;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        double nk, dk;
        const uint32_t wj = CNT ? cls_word(P, c[j]) : w[j];   // (counts 0 past e: outside the set)
        fst_snp(c[j], (bin_k2(wj) != 0u) | ((wj & B_LAST) != 0u), rt, nk, dk);
        sn += nk;
        sd += dk;
      }
    }
    double tn, ta, tb;
    wave_sum_dpp_halves(sn, sd, tn, ta, tb);
    const double td = ta + tb;
    if (lane == 0) fst_out[s] = td != 0.0 ? tn / td : __builtin_nan("");
  }
}

template <bool CNT>
__global__ __launch_bounds__(256) void k_fst_win(KParams P, const uint32_t* __restrict__ counts,
                                                 const uint32_t* __restrict__ bins, const uint2* __restrict__ slots,
                                                 const double2* __restrict__ rt, double* __restrict__ fst_out,
                                                 uint32_t nslots) {
  __shared__ double2 rl[RCPN];   // the (1/n, 1/(n(n-1))) table in LDS, as in k_bg_slice's Fst workgroups
  for (int k = threadIdx.x; k < RCPN; k += 256) rl[k] = rt[k];
  __syncthreads();
  fst_windows<CNT>(P, counts, bins, slots, rl, fst_out, nslots, blockIdx.x * 4u + (threadIdx.x >> 6), gridDim.x * 4u);
}

// ------------------------------------------------------------------------------------------ K2

// numpy pairwise_sum leaf (numpy/_core/src/umath/loops_utils.h.src): n < 8 sequential from 0.0,
// n <= 128: eight strided accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) + tail.
__device__ double np_leaf_sum(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a[i]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
    r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return res;
}

// the same leaf with its eight accumulators on eight lanes (r = lane within the group of 8): each
// accumulator is its own sequential sum, so the result is bitwise np_leaf_sum's
__device__ __forceinline__ double np_leaf_sum8(const double* a, int n, int r, double* acc8) {
  if (n >= 8) {
    double x = a[r];
    for (int i = 8 + r; i < n - (n % 8); i += 8) x += a[i];
    acc8[r] = x;
  }
  __syncthreads();
  double res = 0.0;
  if (r == 0) {
    if (n < 8) {
      for (int i = 0; i < n; ++i) res += a[i];
    } else {
      res = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
      for (int i = n - (n % 8); i < n; ++i) res += a[i];
    }
  }
  return res;
}

// proportion and log entry of one background bin
__device__ __forceinline__ double put_bin(PL* T, double* LP, int k, double v, double B, int integer_values) {
  const double p = (B != 0.0) ? v / B : 0.0;
  PL e;
  e.lp = log(p);
  e.v = integer_values ? v : p;
  T[k] = e;
  LP[k] = e.lp;
  return p;
}

// scipy multinomial._process_parameters on one spectrum: p[-1] <- 1 - sum(p[:-1]) when
// |.| > 1e-15; the whole logpmf is NaN when that p is < 0
__device__ __forceinline__ uint32_t adjust_last(PL* T, double* LP, int klast, double padj, uint32_t nan_flag) {
  if (padj < -1e-15) return nan_flag;
  if (fabs(padj) > 1e-15) {
    T[klast].lp = log(padj);
    LP[klast] = T[klast].lp;
  }
  return 0u;
}

// Per-run per-chromosome backgrounds (integer counts).  grid = (nslices + 1, nbg): blocks
// [0, nslices) own 2D bin ranges aligned to numpy's pairwise leaves, block nslices folds the 1D
// spectra; the last block of a background to finish combines the leaves and writes its head.
// The replicas, the inner-sum counters and the completion counter are left zeroed.
// slices[s] = {kb, ke, leaf_lo, leaf_hi}; leaves[j] = {offset into p[1:], n}; nodes: numpy's tree
// (children ids into [leaves | nodes] and the node's level, ordered by height: children first).
__global__ __launch_bounds__(KBLOCK) void k_bg_slice(KParams P, uint32_t* __restrict__ repl,
                                                     uint32_t* __restrict__ bcount, PL* __restrict__ tab,
                                                     double* __restrict__ LPg, BgHead* __restrict__ head,
                                                     double* __restrict__ leafsum, Bg1D* __restrict__ bg1d,
                                                     uint32_t* __restrict__ done, const int4* __restrict__ slices,
                                                     int nslices, const int2* __restrict__ leaves, int nleaves,
                                                     const int4* __restrict__ nodes, int nnodes, int nlevels, int tail,
                                                     int nfst, const uint32_t* __restrict__ counts,
                                                     const uint32_t* __restrict__ bins, const uint2* __restrict__ slots,
                                                     const double2* __restrict__ rt, double* __restrict__ fst_out,
                                                     uint32_t nslots) {
  // tail == 0: no last-block combination -- the scan kernel combines the leaf sums itself (its
  // prologue), and bcount is a per-run parity buffer cleared by the scan kernel
  __shared__ double pv[4 * 128 + 8];
  __shared__ double acc8[KBLOCK > 2 * PW_MAX_LEAVES ? KBLOCK : 2 * PW_MAX_LEAVES];   // (also the tail's leaf tree)
  __shared__ uint32_t u1[2 * 256 + 2];
  __shared__ double red[KBLOCK / WAVE][2];
  __shared__ int last_blk;
  const int b = blockIdx.y;
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  BGS_STAMP(0);
  if (s > nslices) {   // the extra workgroups (background 0's row only): Fst per window, using the
                       // GPU while this kernel's table blocks wait on memory
    if (b == 0) {
      // the (1/n, 1/(n(n-1))) table in LDS (acc8 is free here): its look-ups follow each SNP's count
      // load, and L2 round trips there were on the window's critical path
      double2* rl = reinterpret_cast<double2*>(acc8);
      for (int k = tid; k < RCPN; k += KBLOCK) rl[k] = rt[k];
      __syncthreads();
      const uint32_t wid0 = (uint32_t)(s - nslices - 1) * (KBLOCK / WAVE) + (tid >> 6);
      if (bins == counts)   // a counts plan (no bins): membership from the counts
        fst_windows<true>(P, counts, bins, slots, rl, fst_out, nslots, wid0, (uint32_t)nfst * (KBLOCK / WAVE));
      else
        fst_windows<false>(P, counts, bins, slots, rl, fst_out, nslots, wid0, (uint32_t)nfst * (KBLOCK / WAVE));
    }
    return;
  }
  const size_t rstride = (size_t)P.nchrom * P.nh;
  uint32_t* R = repl + (size_t)b * P.nh;
  PL* T = tab + (size_t)b * P.nt;
  double* LP = LPg + (size_t)b * P.nt;
  STAMP(0);

  if (s < nslices) {
    const int4 sl = slices[s];
    const double B2 = (double)bcount[b];
    // replica sums (all REPL loads of a bin in flight), proportions, logs
    for (int k = sl.x + tid; k < sl.y; k += KBLOCK) {
      uint32_t x[REPL];
#pragma unroll
      for (int r = 0; r < REPL; ++r) x[r] = R[k + r * rstride];
      uint32_t sum = 0;
#pragma unroll
      for (int r = 0; r < REPL; ++r) {
        sum += x[r];
        if (x[r]) R[k + r * rstride] = 0u;
      }
      pv[k - sl.x] = put_bin(T, LP, k, (double)sum, B2, 1);
    }
    __syncthreads();
    STAMP(1);
    // numpy pairwise leaves over p[1 : nb2-2] (eight lanes per leaf)
    const int g = tid >> 3, r = tid & 7;
    const int j = sl.z + g;
    if (j < sl.w) {
      const int2 lf = leaves[j];
      const double* a = pv + (1 + lf.x - sl.x);
      if (lf.y >= 8) {
        double x = a[r];
        for (int i = 8 + r; i < lf.y - (lf.y % 8); i += 8) x += a[i];
        acc8[tid] = x;
      }
    }
    __syncthreads();
    if (j < sl.w && r == 0) {
      const int2 lf = leaves[j];
      const double* a = pv + (1 + lf.x - sl.x);
      const double* q = acc8 + tid;
      double res = 0.0;
      if (lf.y < 8) {
        for (int i = 0; i < lf.y; ++i) res += a[i];
      } else {
        res = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
        for (int i = lf.y - (lf.y % 8); i < lf.y; ++i) res += a[i];
      }
      leafsum[(size_t)b * nleaves + j] = res;
    }
    STAMP(2);
  } else {
    // the 1D spectra: replica sums of the unfolded histograms, fold_1d_sfs (:446-463), inner sums
    const int nu = P.nh - P.nb2;
    for (int k = tid; k < nu; k += KBLOCK) {
      uint32_t x[REPL];
#pragma unroll
      for (int r = 0; r < REPL; ++r) x[r] = R[P.nb2 + k + r * rstride];
      uint32_t sum = 0;
#pragma unroll
      for (int r = 0; r < REPL; ++r) {
        sum += x[r];
        if (x[r]) R[P.nb2 + k + r * rstride] = 0u;
      }
      u1[k] = sum;
    }
    __syncthreads();
    // folded[f] = u[f] + u[2n - f] (f < n), folded[n] = u[n]; inner sums over f = 1 .. n-1
    double fa = 0.0, fb = 0.0, sa = 0.0, sb = 0.0;
    if (tid <= P.n1p) {
      fa = (double)u1[tid] + (tid < P.n1p ? (double)u1[P.n1 - tid] : 0.0);
      if (tid >= 1 && tid <= P.n1p - 1) sa = fa;
    }
    if (tid <= P.n2p) {
      fb = (double)u1[P.n1 + 1 + tid] + (tid < P.n2p ? (double)u1[P.n1 + 1 + P.n2 - tid] : 0.0);
      if (tid >= 1 && tid <= P.n2p - 1) sb = fb;
    }
    sa = wave_sum_d(sa);
    sb = wave_sum_d(sb);
    if (lane == 0) { red[tid / WAVE][0] = sa; red[tid / WAVE][1] = sb; }
    __syncthreads();
    double B1a = 0.0, B1b = 0.0;
    for (int w = 0; w < KBLOCK / WAVE; ++w) { B1a += red[w][0]; B1b += red[w][1]; }
    // proportions; p kept in LDS for the p[:-1] sums
    if (tid <= P.n1p) pv[tid] = put_bin(T, LP, P.t1a + tid, fa, B1a, 1);
    if (tid <= P.n2p) pv[256 + tid] = put_bin(T, LP, P.t1b + tid, fb, B1b, 1);
    __syncthreads();
    if (tid == 0) {
      uint32_t flags = 0;
      const int M1a = P.n1p - 1, M1b = P.n2p - 1;
      if (B1a == 0.0) flags |= BGF_B1A_ZERO;
      if (B1b == 0.0) flags |= BGF_B1B_ZERO;
      if (M1a >= 1 && B1a != 0.0)
        flags |= adjust_last(T, LP, P.t1a + M1a, 1.0 - np_leaf_sum(pv + 1, M1a - 1), BGF_NAN1A);
      if (M1b >= 1 && B1b != 0.0)
        flags |= adjust_last(T, LP, P.t1b + M1b, 1.0 - np_leaf_sum(pv + 256 + 1, M1b - 1), BGF_NAN1B);
      Bg1D o;
      o.B1a = B1a; o.B1b = B1b; o.flags = flags; o.pad = 0;
      bg1d[b] = o;
    }
  }

  BGS_STAMP(1);
  if (!tail) return;
  // completion: the last block of this background combines (threadfence-reduction pattern)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (tid == 0) last_blk = atomicAdd(&done[b], 1u) == (uint32_t)nslices;
  __syncthreads();
  if (!last_blk) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  TSTAMP(3);
  // numpy's tree over the leaf sums, by the whole block: leaves and nodes loaded in parallel, then
  // one level per barrier (children before parents; each node = left + right, the serial order's
  // sums exactly).  (One thread walking leaves and nodes took 18.6 us on a 201 x 151 grid.)
  double* node = acc8;   // leaves then internal nodes (<= 2 * PW_MAX_LEAVES entries)
  static_assert(2 * PW_MAX_LEAVES <= 4 * KBLOCK, "tree nodes per thread");
  uint32_t bc = 0u;
  Bg1D o1{};
  if (tid == 0) { bc = bcount[b]; o1 = bg1d[b]; }
  int4 nd[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = tid + r * KBLOCK;
    nd[r] = i < nnodes ? nodes[i] : make_int4(0, 0, -1, 0);
    if (i < nleaves) node[i] = leafsum[(size_t)b * nleaves + i];
  }
  __syncthreads();
  for (int l = 0; l < nlevels; ++l) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (nd[r].z == l) node[nleaves + tid + r * KBLOCK] = node[nd[r].x] + node[nd[r].y];
    __syncthreads();
  }
  if (tid == 0) {
    const double B2 = (double)bc;
    const Bg1D o = o1;
    uint32_t flags = o.flags;
    if (B2 == 0.0) flags |= BGF_B2_ZERO;
    const int M2 = P.nb2 - 2;
    if (M2 >= 1 && B2 != 0.0) {
      const double S = (nleaves + nnodes) ? node[nleaves + nnodes - 1] : 0.0;
      flags |= adjust_last(T, LP, M2, 1.0 - S, BGF_NAN2);
    }
    BgHead h;
    h.B2 = B2; h.B1a = o.B1a; h.B1b = o.B1b; h.flags = flags; h.pad = 0;
    head[b] = h;
    bcount[b] = 0u;
    done[b] = 0u;
    TSTAMP(4);
  }
}

// One workgroup per supplied background (sfs2d_plan_set_background; once per plan).  Values v,
// then the proportions p (overwriting v), live in LDS when nt <= FIN_LDS_BINS.
__global__ __launch_bounds__(FBLOCK) void k_bg_finalize(KParams P, int integer_values, const double* __restrict__ bgval,
                                                        double* __restrict__ scratch, PL* __restrict__ tab,
                                                        double* __restrict__ LPg, BgHead* __restrict__ head,
                                                        const int2* __restrict__ pw_leaves, int pw_nleaves,
                                                        const int4* __restrict__ pw_nodes, int pw_nnodes) {
  extern __shared__ double v_lds[];
  __shared__ double red[FBLOCK / WAVE];
  __shared__ double node[2 * PW_MAX_LEAVES];
  __shared__ double Bs[3];
  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  const bool in_lds = P.nt <= FIN_LDS_BINS;
  double* V = in_lds ? v_lds : scratch;
  PL* T = tab;
  double* LP = LPg;
  const int M2 = P.nb2 - 2, M1a = P.n1p - 1, M1b = P.n2p - 1;
  double s2 = 0.0;
  for (int k = tid; k < P.nt; k += FBLOCK) {
    const double x = bgval[k];
    V[k] = x;
    if (k >= 1 && k <= M2) s2 += x;
  }
  __syncthreads();
  // inner sums B over bins[1:-1]: exact for integer values in any order; for normalised (float)
  // values the reference's builtin sum() is sequential, so one lane adds them in order
  if (integer_values) {
    s2 = wave_sum_d(s2);
    if (lane == 0) red[tid / WAVE] = s2;
    if (tid < WAVE) {
      double sa = 0.0, sb = 0.0;
      for (int k = tid; k < M1a; k += WAVE) sa += V[P.t1a + 1 + k];
      for (int k = tid; k < M1b; k += WAVE) sb += V[P.t1b + 1 + k];
      sa = wave_sum_d(sa);
      sb = wave_sum_d(sb);
      if (tid == 0) { Bs[1] = sa; Bs[2] = sb; }
    }
    __syncthreads();
    if (tid == 0) {
      double t = 0.0;
      for (int w = 0; w < FBLOCK / WAVE; ++w) t += red[w];
      Bs[0] = t;
    }
  } else if (tid == 0) {
    double a = 0.0, sa = 0.0, sb = 0.0;
    for (int k = 0; k < M2; ++k) a += V[1 + k];
    for (int k = 0; k < M1a; ++k) sa += V[P.t1a + 1 + k];
    for (int k = 0; k < M1b; ++k) sb += V[P.t1b + 1 + k];
    Bs[0] = a; Bs[1] = sa; Bs[2] = sb;
  }
  __syncthreads();
  const double B2 = Bs[0], B1a = Bs[1], B1b = Bs[2];
  for (int k = tid; k < P.nt; k += FBLOCK) {
    const double B = k < P.nb2 ? B2 : (k < P.t1b ? B1a : B1b);
    V[k] = put_bin(T, LP, k, V[k], B, integer_values);
  }
  __syncthreads();
  if (tid < pw_nleaves) {
    const int2 lf = pw_leaves[tid];
    node[tid] = np_leaf_sum(V + 1 + lf.x, lf.y);
  }
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < pw_nnodes; ++i) {
      const int4 ab = pw_nodes[i];
      node[pw_nleaves + i] = node[ab.x] + node[ab.y];
    }
    uint32_t flags = integer_values ? 0u : BGF_FLOATV;
    if (B2 == 0.0) flags |= BGF_B2_ZERO;
    if (B1a == 0.0) flags |= BGF_B1A_ZERO;
    if (B1b == 0.0) flags |= BGF_B1B_ZERO;
    if (M2 >= 1 && B2 != 0.0) {
      const int nn = pw_nleaves + pw_nnodes;
      flags |= adjust_last(T, LP, M2, 1.0 - (nn ? node[nn - 1] : 0.0), BGF_NAN2);
    }
    if (M1a >= 1 && B1a != 0.0) flags |= adjust_last(T, LP, P.t1a + M1a, 1.0 - np_leaf_sum(V + P.t1a + 1, M1a - 1), BGF_NAN1A);
    if (M1b >= 1 && B1b != 0.0) flags |= adjust_last(T, LP, P.t1b + M1b, 1.0 - np_leaf_sum(V + P.t1b + 1, M1b - 1), BGF_NAN1B);
    BgHead h;
    h.B2 = B2; h.B1a = B1a; h.B1b = B1b; h.flags = flags; h.pad = 0;
    head[0] = h;
  }
}

// ------------------------------------------------------------------------------------------ K3

template <int G>
__device__ __forceinline__ void group_sync() {
  if (G == WAVE) {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

// group-wide sums; G > WAVE uses a small LDS scratch (G/64 waves x 8 slots)
template <int G>
__device__ __forceinline__ double group_sum_d(double v, double* red, int slot) {
  v = wave_sum_d(v);
  if (G == WAVE) return v;
  const int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) red[w * 8 + slot] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < G / WAVE; ++i) t += red[i * 8 + slot];
  __syncthreads();
  return t;
}

template <int G>
__device__ __forceinline__ unsigned long long group_sum_u64(unsigned long long v, unsigned long long* red, int slot) {
  v = wave_sum_u64(v);
  if (G == WAVE) return v;
  const int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) red[w * 8 + slot] = v;
  __syncthreads();
  unsigned long long t = 0;
  for (int i = 0; i < G / WAVE; ++i) t += red[i * 8 + slot];
  __syncthreads();
  return t;
}

// T from the owner-lane sum: T = 2*(S - N ln N), with the reference's special values
__device__ __forceinline__ double clr_value(double S, uint32_t N, bool prop, bool nan_bg, const double* lnx) {
  if (nan_bg) return __builtin_nan("");
  if (prop) return 0.0;
  return 2.0 * (S - (double)N * lnx_of(lnx, N));
}

template <bool P16>
__device__ __forceinline__ void h2_add(uint32_t* h, uint32_t k) {
  if (P16) atomicAdd(&h[k >> 1], 1u << ((k & 1) << 4));
  else atomicAdd(&h[k], 1u);
}

template <bool P16>
__device__ __forceinline__ uint32_t h2_take(uint32_t* h, uint32_t k) {  // read-and-clear; one lane gets x
  if (P16) {
    const uint32_t sh = (k & 1) << 4;
    return (atomicAnd(&h[k >> 1], ~(0xffffu << sh)) >> sh) & 0xffffu;
  }
  return atomicExch(&h[k], 0u);
}

// Exact evaluation of one window [b, e) by a group of G lanes: per element take-and-clear with the
// bin-by-bin proportionality test.  Used for large grids, for windows whose fast-path |T| is ~0
// (possibly exactly proportional), for windows of >= LNX_N SNPs, and for the Q9 helper.
// S1: word stride of the 1D histograms (k_scan_w keeps R1 replicas per bin; this uses the first).
// Background table views for eval_exact: lp(k) and v(k) (the count, or p for normalised backgrounds)
struct TabGlobal {   // the PL table written by k_bg_slice / k_bg_finalize
  const PL* T;
  __device__ __forceinline__ PL at(int k) const { return T[k]; }
};

struct TabLocal {    // k_bg_slice's table with the log proportions from LDS (the workgroup's own p[-1] rule)
  const PL* T;
  const double* LPl;
  __device__ __forceinline__ PL at(int k) const {
    PL e = T[k];
    e.lp = LPl[k];
    return e;
  }
};
struct TabFused {    // k_scan_w's own table: lp in LDS, counts summed from this run's replicas
  const double* LPl;
  const uint32_t* R;   // this chromosome's replica 0; replica r at R + r * rs
  size_t rs;
  int nb2, n1, n2, n1p, h1a, h1b, t1a, t1b;
  __device__ __forceinline__ uint32_t u(int k) const {
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < REPL; ++r) s += R[k + r * rs];
    return s;
  }
  __device__ __forceinline__ PL at(int k) const {
    PL e;
    e.lp = LPl[k];
    if (k < nb2) {
      e.v = (double)u(k);
    } else if (k < t1b) {
      const int f = k - t1a;   // fold_1d_sfs: u[f] + u[2n - f] (f < n)
      e.v = (double)u(h1a + f) + (f < n1p ? (double)u(h1a + n1 - f) : 0.0);
    } else {
      const int f = k - t1b, n2p = n2 / 2;
      e.v = (double)u(h1b + f) + (f < n2p ? (double)u(h1b + n2 - f) : 0.0);
    }
    return e;
  }
};

template <int G, bool P16, int S1, bool CNT, class Tab>
__device__ __forceinline__ WinOut eval_exact(const KParams& P, const uint32_t* __restrict__ bins, uint32_t b,
                                             uint32_t e, const Tab& T, const BgHead& hb,
                                             const double* __restrict__ lnx, uint32_t* H2, uint32_t* H1a,
                                             uint32_t* H1b, double* redd, unsigned long long* redu) {
  const int lane = threadIdx.x & (G - 1);
  const bool floatv = hb.flags & BGF_FLOATV;
  uint32_t c_var = 0, c2 = 0, c_last = 0, c1a = 0, c1b = 0;
  for (uint32_t i = b + lane; i < e; i += G) {
    const uint32_t w = snp_word<CNT>(P, bins, i);
    const uint32_t k2 = bin_k2(w), g1 = bin_g1(w), g2 = bin_g2(w);
    c_var += (w & B_VAR) ? 1u : 0u;
    c_last += (w & B_LAST) ? 1u : 0u;
    if (k2) { ++c2; h2_add<P16>(H2, k2); }
    if (g1) { ++c1a; atomicAdd(&H1a[g1 * S1], 1u); }
    if (g2) { ++c1b; atomicAdd(&H1b[g2 * S1], 1u); }
  }
  if (G == WAVE) __threadfence();   // (k_scan_gw passes a histogram in global memory: adds land before the takes)
  group_sync<G>();
  const unsigned long long r0 = group_sum_u64<G>((unsigned long long)c2 | ((unsigned long long)c_last << 32), redu, 0);
  const unsigned long long r1 = group_sum_u64<G>((unsigned long long)c1a | ((unsigned long long)c1b << 32), redu, 1);
  const unsigned long long r2 = group_sum_u64<G>((unsigned long long)c_var, redu, 2);
  WinOut o;
  o.n2 = (uint32_t)r0;
  o.n2_all = o.n2 + (uint32_t)(r0 >> 32);
  o.n1a = (uint32_t)r1;
  o.n1b = (uint32_t)(r1 >> 32);
  o.snp_count = (uint32_t)r2;
  const double N2 = (double)o.n2, N1a = (double)o.n1a, N1b = (double)o.n1b;
  double s2 = 0.0, sa = 0.0, sb = 0.0;
  bool q2 = true, qa = true, qb = true;   // x_k/N == p_k bitwise on every touched bin
  for (uint32_t i = b + lane; i < e; i += G) {
    const uint32_t w = snp_word<CNT>(P, bins, i);
    const uint32_t k2 = bin_k2(w), g1 = bin_g1(w), g2 = bin_g2(w);
    if (k2) {
      const uint32_t x = h2_take<P16>(H2, k2);
      if (x) {
        const PL t = T.at(k2);
        s2 += (double)x * (lnx_of(lnx, x) - t.lp);
        q2 &= prop_ok(x, N2, t.v, hb.B2, floatv);
      }
    }
    if (g1) {
      const uint32_t x = atomicExch(&H1a[g1 * S1], 0u);
      if (x) {
        const PL t = T.at(P.t1a + g1);
        sa += (double)x * (lnx_of(lnx, x) - t.lp);
        qa &= prop_ok(x, N1a, t.v, hb.B1a, floatv);
      }
    }
    if (g2) {
      const uint32_t x = atomicExch(&H1b[g2 * S1], 0u);
      if (x) {
        const PL t = T.at(P.t1b + g2);
        sb += (double)x * (lnx_of(lnx, x) - t.lp);
        qb &= prop_ok(x, N1b, t.v, hb.B1b, floatv);
      }
    }
  }
  s2 = group_sum_d<G>(s2, redd, 0);
  sa = group_sum_d<G>(sa, redd, 1);
  sb = group_sum_d<G>(sb, redd, 2);
  const unsigned long long bad = group_sum_u64<G>((unsigned long long)(!q2) | ((unsigned long long)(!qa) << 21) |
                                                  ((unsigned long long)(!qb) << 42), redu, 3);
  o.t2d = clr_value(s2, o.n2, (bad & 0x1fffffull) == 0, hb.flags & BGF_NAN2, lnx);
  o.t1a = clr_value(sa, o.n1a, ((bad >> 21) & 0x1fffffull) == 0, hb.flags & BGF_NAN1A, lnx);
  o.t1b = clr_value(sb, o.n1b, (bad >> 42) == 0, hb.flags & BGF_NAN1B, lnx);
  return o;
}

// |T| this small may be an exactly proportional window (reference: T == 0.0 exactly, which its
// truthiness guard reads as False): such windows are re-evaluated on the exact path.
__device__ __forceinline__ bool suspect_zero(double t, uint32_t N) {
  return N && fabs(t) <= 1e-9 * ((double)N + 1.0);
}

// Hudson's Fst (Bhatia et al. 2013, ratio of averages) over the SNPs entering the window's 2D SFS
// (filters passed, (0,0) excluded, the (n1,n2) bin included) with >= 2 called alleles in each
// population: p_i = alt_i / (ref_i + alt_i) on the raw counts,
//   num = (p1 - p2)^2 - p1(1-p1)/(n1c-1) - p2(1-p2)/(n2c-1),  den = p1(1-p2) + p2(1-p1),
// Fst = sum num / sum den (NaN when no SNP qualifies or sum den == 0).  Not in the reference (its
// published Fst is pixy's Weir-Cockerham, joined in R): parity is pinned to oracle.window_fst.
// k_prep sums the terms per window slot (fst_snp, int64 fixed point); the scan kernels turn the
// sums into the value and clear them for the next run.
__device__ __forceinline__ double fst_take(unsigned long long* fsum, size_t s) {
  const long long qn = (long long)fsum[2 * s], qd = (long long)fsum[2 * s + 1];
  fsum[2 * s] = 0ull;
  fsum[2 * s + 1] = 0ull;
  return qd != 0 ? (double)qn / (double)qd : __builtin_nan("");
}

struct Win {
  uint32_t b, e;
  uint32_t u[8];   // bins of this lane's first 8 SNPs, b + lane + 64 j (0 past e)
  bool has;
};

// F(x) = x ln x from the LDS table (N entries), the global ln table beyond it
template <int N = LNT>
__device__ __forceinline__ double xlnx(uint32_t x, const double* Ft, const double* lnx) {
  return x < (uint32_t)N ? Ft[x] : (double)x * lnx[x];
}

// The fused prologue of k_scan_w (kept out of line: it runs once per workgroup and its registers
// must not count against the window loop's).  Builds the chromosome's background table from this
// run's replicas -- the k_bg_slice computation -- in LDS (LPl), using the histogram area HB as
// scratch; clears this workgroup's share of the other parity's replicas; the chromosome's first
// workgroup (writer) also writes the global tables.  The head lands in *hb_out (LDS).
__device__ __forceinline__ void fused_table(int nb2, int nh, int nt, int n1p, int n2p, int n1, int n2,
                                            int t1a, int t1b, int nchrom, uint32_t chrom, bool writer,
                                                      int bg, const uint32_t* __restrict__ Rc, size_t rs,
                                                      uint32_t* __restrict__ repl, uint32_t* __restrict__ bcount,
                                                      int par, PL* __restrict__ tab, double* __restrict__ LPg,
                                                      BgHead* __restrict__ head, double* LPl, uint32_t* HB,
                                                      const int2* __restrict__ leaves, int nleaves,
                                                      const int4* __restrict__ nodes, int nnodes, int nlevels,
                                                      const double* __restrict__ lnx, BgHead* hb_out,
                                                      double* lsum, uint32_t* vcnt) {
  __shared__ double sh_misc[8];
  __shared__ double sh_lnb[3];
  __shared__ uint32_t sh_flags;
  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  BgHead hb;
  PL* T = tab + (size_t)bg * nt;
  double* LP = LPg + (size_t)bg * nt;
  // scratch in the histogram area: u1 words, 1D p, leaf accumulators, leaf sums
  double* scr = reinterpret_cast<double*>(HB);
  uint32_t* u1 = HB;                 // [0, 512) words
  double* p1a = scr + 264;           // 128
  double* p1b = scr + 392;           // 128
  double* acc8 = scr + 512;          // 8 per leaf (<= 128 leaves)
  // lsum: leaf sums and tree nodes (nleaves + nnodes); vcnt: the table's counts (2D, then folded 1D),
  // nt words -- both in HB past acc8 (fixed offsets)
  const double B2 = (double)bcount[(size_t)par * nchrom + chrom];
  const int4 my_node = tid < nnodes ? nodes[tid] : make_int4(0, 0, -1, 0);
  const int2 my_leaf = tid < nleaves ? leaves[tid] : make_int2(0, 0);   // this thread's leaf to combine
  const int gl = (tid - 2 * WAVE) >> 3;                                   // waves 2..7: accumulator group
  const int2 acc_leaf = (tid >= 2 * WAVE && gl < nleaves) ? leaves[gl] : make_int2(0, 0);
  // replica sums, four words per 16-B load, every load of a round in flight; 2D words become
  // proportions (LPl holds p until the log pass), 1D words go to u1
  constexpr int QJ = 2;   // 16-B rows per thread per round
  for (int q0 = tid; q0 < nh / 4; q0 += QJ * SBLOCK) {
    uint4 x[QJ][REPL];
#pragma unroll
    for (int j = 0; j < QJ; ++j)
#pragma unroll
      for (int r = 0; r < REPL; ++r) {
        const int q = q0 + j * SBLOCK;
        x[j][r] = q < nh / 4 ? *reinterpret_cast<const uint4*>(Rc + r * rs + 4 * q) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
    for (int j = 0; j < QJ; ++j) {
      const int q = q0 + j * SBLOCK;
      if (q >= nh / 4) continue;
      uint32_t sm[4] = {0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < REPL; ++r) {
        sm[0] += x[j][r].x; sm[1] += x[j][r].y; sm[2] += x[j][r].z; sm[3] += x[j][r].w;
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = 4 * q + c;
        if (k < nb2) {
          const double v = (double)sm[c];
          LPl[k] = (B2 != 0.0) ? v / B2 : 0.0;
          vcnt[k] = sm[c];
          if (writer) T[k].v = v;
        } else {
          u1[k - nb2] = sm[c];
        }
      }
    }
  }
  __syncthreads();
  STAMP(16);
  // 1D spectra (wave 0: pop1, wave 1: pop2): fold_1d_sfs (:446-463), inner sums, proportions
  if (wv < 2) {
    const int np_ = wv ? n2p : n1p, n_ = wv ? n2 : n1, off = wv ? n1 + 1 : 0, t0 = wv ? t1b : t1a;
    double f[2], sf = 0.0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = lane + WAVE * j;
      f[j] = 0.0;
      if (k <= np_) f[j] = (double)u1[off + k] + (k < np_ ? (double)u1[off + n_ - k] : 0.0);
      if (k >= 1 && k <= np_ - 1) sf += f[j];
    }
    const double B1 = wave_sum_d(sf);
    double* p1 = wv ? p1b : p1a;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = lane + WAVE * j;
      if (k <= np_) {
        const double p = (B1 != 0.0) ? f[j] / B1 : 0.0;
        p1[k] = p;
        LPl[t0 + k] = p;
        vcnt[t0 + k] = (uint32_t)f[j];
        if (writer) T[t0 + k].v = f[j];
      }
    }
    if (lane == 0) sh_misc[1 + wv] = B1;
  } else {
    // 2D numpy pairwise leaves over p[1 : nb2-2], eight lanes per leaf
    for (int g = (tid - 2 * WAVE) >> 3; g < nleaves; g += (SBLOCK - 2 * WAVE) / 8) {
      const int r = tid & 7;
      const int2 lf = g == gl ? acc_leaf : leaves[g];
      if (lf.y >= 8) {
        const double* a = LPl + 1 + lf.x;
        double x = a[r];
        for (int i = 8 + r; i < lf.y - (lf.y % 8); i += 8) x += a[i];
        acc8[g * 8 + r] = x;
      }
    }
  }
  __syncthreads();
  if (tid < nleaves) {
    const int2 lf = my_leaf;
    const double* a = LPl + 1 + lf.x;
    const double* q = acc8 + tid * 8;
    double res = 0.0;
    if (lf.y < 8) {
      for (int i = 0; i < lf.y; ++i) res += a[i];
    } else {
      res = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
      for (int i = lf.y - (lf.y % 8); i < lf.y; ++i) res += a[i];
    }
    lsum[tid] = res;
  }
  if (tid == 4 * WAVE && n1p >= 2) sh_misc[3] = 1.0 - np_leaf_sum(p1a + 1, n1p - 2);
  if (tid == 5 * WAVE && n2p >= 2) sh_misc[4] = 1.0 - np_leaf_sum(p1b + 1, n2p - 2);
  __syncthreads();
  STAMP(17);
  // numpy's tree over the leaves, one level of equal-height nodes at a time (lsum holds the
  // leaves, then the nodes; children always precede parents)
  for (int l = 0; l < nlevels; ++l) {
    if (my_node.z == l) lsum[nleaves + tid] = lsum[my_node.x] + lsum[my_node.y];
    __syncthreads();
  }
  STAMP(18);
  if (tid == 0) {
    const double S = (nleaves + nnodes) ? lsum[nleaves + nnodes - 1] : 0.0;
    const double B1a = sh_misc[1], B1b = sh_misc[2];
    uint32_t flags = 0;
    if (B2 == 0.0) flags |= BGF_B2_ZERO;
    if (B1a == 0.0) flags |= BGF_B1A_ZERO;
    if (B1b == 0.0) flags |= BGF_B1B_ZERO;
    // bit 8/9/10: replace the last inner lp of 2D / pop1 / pop2 with log(padj)
    const double pa[3] = {1.0 - S, sh_misc[3], sh_misc[4]};
    const bool on[3] = {nb2 - 2 >= 1 && B2 != 0.0, n1p - 1 >= 1 && B1a != 0.0, n2p - 1 >= 1 && B1b != 0.0};
    const uint32_t nanf[3] = {BGF_NAN2, BGF_NAN1A, BGF_NAN1B};
    for (int q = 0; q < 3; ++q) {
      if (!on[q]) continue;
      if (pa[q] < -1e-15) flags |= nanf[q];
      else if (fabs(pa[q]) > 1e-15) flags |= 256u << q;
    }
    sh_misc[0] = 1.0 - S;
    sh_lnb[0] = log(B2);
    sh_lnb[1] = log(B1a);
    sh_lnb[2] = log(B1b);
    sh_flags = flags;
  }
  __syncthreads();
  const uint32_t flags = sh_flags;
  const int kl[3] = {nb2 - 2, t1a + n1p - 1, t1b + n2p - 1};
  const double pad[3] = {sh_misc[0], sh_misc[3], sh_misc[4]};
  // lp = ln v - ln B, ln v from the ln table (p = v / B stayed in LPl only for numpy's sums above);
  // the replaced last inner bins take log(padj).  Same value as log(v / B) to a few ulp.
  const double lnB[3] = {sh_lnb[0], sh_lnb[1], sh_lnb[2]};
  const double ninf = -__builtin_inf();
  constexpr int LB = 6;   // bins per thread per round, all table loads in flight together
  for (int k0 = tid; k0 < nt; k0 += LB * SBLOCK) {
    uint32_t v[LB];
    double lv[LB];
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int k = k0 + j * SBLOCK;
      v[j] = k < nt ? vcnt[k] : 0u;
    }
#pragma unroll
    for (int j = 0; j < LB; ++j) lv[j] = lnx[v[j] < (uint32_t)LNX_N ? v[j] : 0u];
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const int k = k0 + j * SBLOCK;
      if (k >= nt) continue;
      const int sp = k < nb2 ? 0 : (k < t1b ? 1 : 2);
      double lp = v[j] == 0u ? ninf : (v[j] < (uint32_t)LNX_N ? lv[j] : log((double)v[j])) - lnB[sp];
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (k == kl[q] && (flags & (256u << q))) lp = log(pad[q]);
      LPl[k] = lp;
      if (writer) { T[k].lp = lp; LP[k] = lp; }
    }
  }
  STAMP(19);
  hb.B2 = B2; hb.B1a = sh_misc[1]; hb.B1b = sh_misc[2]; hb.flags = flags & 0xffu; hb.pad = 0;
  if (writer && tid == 0) head[bg] = hb;
  if (tid == 0) *hb_out = hb;
  __syncthreads();   // scratch reads done before the histogram area is zeroed
}

// K3 for small grids.  Workgroup LDS: [lp table of the chunk's background (nt doubles, rounded up
// to even) | D | F | per wave: 2D bins (u16-packed when P16) | R1 x folded pop1 1D | R1 x pop2 1D |
// 64 trash words].
// FUSED (per-chromosome backgrounds): the workgroup builds its chromosome's table in the prologue
// from this run's k_prep replicas (the k_bg_slice computation, in the histogram area as scratch),
// clears its share of the other parity's replicas for the next run, and the first workgroup of a
// chromosome also writes the global tables (k_scan_extra and callers read them).  Otherwise the
// table comes from k_bg_finalize's output.
// Per window (one wavefront): pass over its bins (first 512 prefetched with the previous window):
// per-lane counters give every count, the 2D atomic returns the SNP's rank r in its bin and the
// SNP adds D(r) - lp_k; the 1D atomics land in lane-&3 replicas; then one lane per 1D bin adds
// x ln x - x lp; the touched 2D words are cleared; DPP sums; one record.
// k_scan_gw (grids too large for the table in LDS): one-wavefront workgroups whose LDS holds
// only the wave's histograms; lp, D and F are read from the global tables (L2-resident: one
// table per background, read by every window).  The 2D bins are u8-packed (101 x 101: 10 KB per
// wave, 12 waves per CU instead of 7 with u16): a rank of 255 means the byte wrapped, and such a
// window is re-evaluated exactly on a u32 histogram in global memory (gscr: nscr slots of nb2
// words, then nscr lock words; a slot is taken with a CAS, so every resident wave finds one).
#define SCAN_W_ARGS                                                                                           \
  KParams P, const uint32_t *__restrict__ bins, const Chunk *__restrict__ chunks, uint2 *__restrict__ slots,  \
      PL *__restrict__ tab, double *__restrict__ LPg, BgHead *__restrict__ head, int bg_per_chrom,            \
      const double *__restrict__ lnx, const double *__restrict__ dfg, sfs2d_window *__restrict__ out,          \
      uint32_t *__restrict__ err_word, int mode_bp, uint32_t *__restrict__ repl, uint32_t *__restrict__ bcount, \
      int par, const int2 *__restrict__ leaves, int nleaves, const int4 *__restrict__ nodes, int nnodes,       \
      int nlevels, int write_chrom, unsigned long long *__restrict__ fsum, double *__restrict__ fst_out,       \
      uint32_t *__restrict__ ctr, int cpar, const double *__restrict__ leafsum, const Bg1D *__restrict__ bg1d, \
      int sliced, uint32_t *__restrict__ gscr, int nscr
#define SCAN_W_PASS                                                                                           \
  P, bins, chunks, slots, tab, LPg, head, bg_per_chrom, lnx, dfg, out, err_word, mode_bp, repl, bcount, par,  \
      leaves, nleaves, nodes, nnodes, nlevels, write_chrom, fsum, fst_out, ctr, cpar, leafsum, bg1d, sliced,  \
      gscr, nscr

__device__ __forceinline__ void wave_sum3(double a, double b, double c, double& sa, double& sb, double& sc);

// TRI (counts plans, folded, n1 = n2 = n): the wave's u8 2D histogram holds only the bins a folded key
// can reach, x1 + x2 <= n (the fold swaps to the reference alleles when a1 + a2 > n, and r1 + r2 <=
// 2n - (a1 + a2) then), as a triangle: bin (x1, x2) at x1 (n + 1) - x1 (x1 - 1) / 2 + x2 = k2 -
// x1 (x1 - 1) / 2.  101 x 101: 5.2 instead of 10.2 KB per wave.  The tables (lp, the exact path's
// global histogram) keep the full index k2.
template <bool P16, bool FST, bool CNT, bool TRI = false>
__device__ __forceinline__ void scan_gw_body(double* ldsd, SCAN_W_ARGS) {
  STAMP(10);
  BLK_STAMP(1, 0);
  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  const Chunk ch = chunks[blockIdx.x];
  const int bg = bg_per_chrom ? (int)ch.chrom : 0;

  // the tables in global memory (L2-resident): the background's lp table, D and F; LDS holds the wave's
  // histograms only: u8-packed 2D bins | RG x folded pop-1 1D | RG x pop-2 1D | 64 lane trash words
  const double* LPl = LPg + (size_t)bg * P.nt;
  const double* Dt = dfg;       // LNT
  const double* Ft = Dt + LNT;  // LNT
  static_assert(!TRI || CNT, "the triangle index needs the counts (x1)");
  const int h2w = (((TRI ? P.ntri : P.nb2) + 3) / 4 + 3) & ~3;
  constexpr int RG = R1GW;   // 1D replicas
  const int h1w = RG * (P.n1p + 1), h1wb = RG * (P.n2p + 1);
  const int per = h2w + h1w + h1wb + TRASH;
  uint32_t* W = reinterpret_cast<uint32_t*>(ldsd);
  // P.lnl: ln(x) for x < LNL after the histograms, copied from the global ln table at the start: the window's
  // end reads ln of its totals and 1D counts from LDS instead of an L2 round trip per window
  double* LNLt = reinterpret_cast<double*>(W + ((per + 1) & ~1));
  uint32_t* H1a = W + h2w;
  uint32_t* H1b = H1a + h1w;
  const uint32_t trash = (uint32_t)(h2w + h1w + h1wb + lane);   // word offset from W
  const uint32_t rep = lane & (RG - 1);

  // the first window's slot record is fetched before the table work.  The rows are loaded
  // unconditionally, range-checked (a window that is not there -- live false, or an empty slot -- reads a
  // 0-byte range: zeros, no memory access): no branch join around them for the wait counters to merge,
  // which made later waits wait for them
  auto bounds = [&](uint32_t s, uint2 sr, Win& w, bool live) {
    if (mode_bp) {
      w.has = live && sr.x != 0u;
      w.b = sr.x - 1u;
      w.e = sr.y;
    } else {
      w.has = live;
      w.b = ch.cb + (ch.wid_lo + (s - ch.slot_lo)) * P.ws;
      w.e = w.b + P.ws;
    }
    const __amdgpu_buffer_rsrc_t rr = window_rows(bins, w.has ? w.b : 0u, w.has ? w.e : 0u, P.nm1);
    // (the lane's byte offset made opaque here: hoisted out of the window loop, the eight row offsets
    // were kept live as eight VGPRs -- spilled elsewhere -- instead of one base + immediate offsets)
    uint32_t lo = (uint32_t)lane * 4u;
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (int j = 0; j < 8; ++j) w.u[j] = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)lo + 256 * j, 0, 0);
  };
  // window schedule: one static window per wavefront, then the chromosome's pool counters (an
  // atomic is always one window ahead of its use, so its latency hides under a window's work)
  uint32_t s = ch.slot_lo + ch.first;
  const bool active = s < ch.slot_hi;
  const uint2 sr0 = (active && mode_bp) ? slots[s] : make_uint2(0, 0);   // in flight during the table work
  const uint32_t npool = ch.pool & 0xffffu, pool = ch.pool >> 16;
  const bool dyn = ch.slot_lo + ch.nstatic < ch.slot_hi;
  const uint32_t dbase = ch.slot_lo + ch.nstatic + pool;
  uint32_t* myctr = ctr + (((size_t)cpar * P.nchrom + ch.chrom) * CTR_POOLS + pool) * CTR_STRIDE;
  uint32_t gq = 0;
  if (active && dyn && lane == 0) gq = atomicAdd(myctr, 1u);
  if (blockIdx.x == 0)   // the other parity's counters, for the next run
    for (int k = tid; k < P.nchrom * CTR_POOLS; k += WAVE) ctr[((size_t)(1 - cpar) * P.nchrom * CTR_POOLS + k) * CTR_STRIDE] = 0u;

  const BgHead hb = head[bg];
  for (int k = lane; k < per / 4; k += WAVE) reinterpret_cast<uint4*>(W)[k] = make_uint4(0, 0, 0, 0);
  if (P.lnl)
    for (int k = lane; k < LNL; k += WAVE) LNLt[k] = lnx[k];
  __syncthreads();
  const bool filt = P.ann_want >= 0;
  const bool half1d = P.n1p <= 33 && P.n2p <= 33;
  const uint32_t zflags = bg_zero_flags(hb);
  const bool nan2 = hb.flags & BGF_NAN2, nan1a = hb.flags & BGF_NAN1A, nan1b = hb.flags & BGF_NAN1B;

  if (!active) return;
  const double Dreg = lane < 63 ? dfg[lane] : 0.0;   // D(lane), lane 63: 0 (ranks from 63 on)
  const double f63 = Ft[63];                          // F(63) (bins past 63 SNPs)
  // the background's 1D terms of this lane's inner bins (the window's end: x ln x - x lp per bin)
  const bool in1h = half1d && 1 + (lane & 31) <= (lane < 32 ? P.n1p : P.n2p) - 1;
  double lp1a[2] = {0.0, 0.0}, lp1b[2] = {0.0, 0.0};
  if (half1d) {
    if (in1h) lp1a[0] = LPl[(lane < 32 ? P.t1a : P.t1b) + 1 + (lane & 31)];
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = 1 + lane + WAVE * j;
      if (k <= P.n1p - 1) lp1a[j] = LPl[P.t1a + k];
      if (k <= P.n2p - 1) lp1b[j] = LPl[P.t1b + k];
    }
  }
  const uint32_t one1 = 1u;                         // 1D increment
  uint32_t* const H1a_l = H1a + rep;            // this lane's replica column of the 1D histograms
  uint32_t* const H1b_l = H1b + rep;
  uint32_t* const T_l = W + trash;
  // the 1D atomics' LDS byte addresses from opaque per-lane bases (one v_lshl_add per bin)
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  uint32_t a1b = (uint32_t)(uintptr_t)((lds_u32*)H1a_l), a2b = (uint32_t)(uintptr_t)((lds_u32*)H1b_l);
  uint32_t atr = (uint32_t)(uintptr_t)((lds_u32*)T_l);
  asm volatile("" : "+v"(a1b), "+v"(a2b), "+v"(atr));
  Win cur;
  bounds(s, sr0, cur, true);
  STAMP(11);
  int it = 0;
  uint32_t sn = ch.slot_hi;
  for (; s < ch.slot_hi; s = sn, ++it) {
    sn = ch.slot_hi;
    if (dyn) {
      const uint32_t j = __builtin_amdgcn_readfirstlane(gq);
      sn = dbase + npool * j < ch.slot_hi ? dbase + npool * j : ch.slot_hi;
      if (sn < ch.slot_hi && lane == 0) gq = atomicAdd(myctr, 1u);
    }
    const bool more = sn < ch.slot_hi;
    const uint2 srn = (mode_bp && more) ? slots[sn] : make_uint2(0, 0);
    const uint32_t wid = ch.wid_lo + (s - ch.slot_lo);
    if (!cur.has) {
      if (lane == 0) write_empty(out + s, ch.chrom, wid);
      if (FST && lane == 0) fst_out[s] = __builtin_nan("");
      Win nxt;
      nxt.has = false;
      bounds(sn, make_uint2(__builtin_amdgcn_readfirstlane(srn.x), __builtin_amdgcn_readfirstlane(srn.y)), nxt, more);
      cur = nxt;
      continue;
    }
    // SNP j of this lane is b + lane + 64 j: steps (rows) of 64 SNPs in pairs (SNPs past e are w = 0,
    // i.e. excluded).  Counters are wave-uniform ballot counts.  Excluded SNPs (k2 = 0) add 0 to the
    // lane's trash word and take rank 0 and lp 0; 1D increments outside the inner bins land there too.
    const uint32_t nsnp = cur.e - cur.b;
    const int lim = (int)nsnp - lane;

    double acc2 = 0.0;
    uint32_t n2 = 0, nlast = 0, n1a = 0, n1b = 0, nvar = 0;
    bool ovf = false;   // some u8 bin of this lane wrapped
    bool big = false;   // some bin of this lane passed rank 63 (its later ranks added 0; see below)
    // the 2D words of the last 8 steps (a shift register: computed values, no loads, so its moves never
    // wait), cleared after a window of <= 6 steps; initially the lane's trash word
    uint32_t kw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) kw[j] = trash;
    // A pair of rows in two halves, software-pipelined as in k_scan_w: issue() classifies, issues the
    // LDS atomics and the lp loads from the global table; finish() turns the returned ranks and lp
    // into D(r) - lp_k.  The loops issue pair j before they finish pair j - 2: a pair's atomics and its
    // L2 round trip for lp return under the next pair's work.
    struct PairSt { uint32_t ov[2], xs[2], kk[2]; double lp[2]; };
    auto issue = [&](uint32_t w0, uint32_t w1, int j) {
      PairSt st;
      // SNPs past e are excluded (unconditional: cheaper than a guard; CNT: the window-ranged loads
      // returned 0 there)
      if (!CNT) {
        w0 = 64 * j < lim ? w0 : 0u;
        w1 = 64 * (j + 1) < lim ? w1 : 0u;
      }
      const uint32_t ww[2] = {w0, w1};   // (CNT: counts; 0 past e, in no spectrum)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t w = ww[q];
        uint32_t k2, g1, g2, kh;   // kh: the bin's index in the LDS histogram
        if (CNT) cls_fields(P, w, k2, g1, g2, TRI ? &kh : nullptr);
        else { k2 = bin_k2(w); g1 = bin_g1(w); g2 = bin_g2(w); }
        if (!TRI) kh = k2;
        n2 += 64u - (uint32_t)__popcll(__ballot(k2 == 0u));   // (the compare the selects below use)
        n1a += __popcll(__ballot(g1 != 0u));
        n1b += __popcll(__ballot(g2 != 0u));
        // (the global table, whose bin 0 is not zeroed: excluded SNPs read D's last entry, 0, instead --
        // an address select here, not a select of the loaded value in finish(), which the scheduler
        // hoisted next to the load and so waited for the gather on the spot)
        st.lp[q] = *(k2 ? LPl + k2 : Dt + (LNT - 1));
        const uint32_t word = k2 ? (kh >> 2) : trash;   // (u8 bins: four to a word)
        // the byte's shift: the hardware reads shift operands' low five bits, so kh << 3 serves
        // without a mask (the bins word's low bits are k2's)
        const uint32_t wk = CNT ? kh : w;
        const uint32_t sh = wk << 3;
        uint32_t one2 = 1u;
        asm("v_lshlrev_b32 %0, %1, 1" : "=v"(one2) : "v"(sh));
        st.ov[q] = atomicAdd(&W[word], k2 ? one2 : 0u);
        st.xs[q] = sh;
        st.kk[q] = k2;
        kw[q] = kw[q + 2]; kw[q + 2] = kw[q + 4]; kw[q + 4] = kw[q + 6]; kw[q + 6] = word;
        const uint32_t u1 = g1 ? a1b + g1 * (4u * RG) : atr, u2 = g2 ? a2b + g2 * (4u * RG) : atr;
        __hip_atomic_fetch_add((lds_u32*)(uintptr_t)u1, one1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add((lds_u32*)(uintptr_t)u2, one1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      return st;
    };
    // dlook(): the pair's D(r) look-ups, issued as soon as its ranks are in (lane shuffles, before
    // the next pair's atomics, so that waiting for them is not waiting for those too -- LDS operations
    // complete in order); finish(): D(r) - lp_k into the sum
    auto dlook = [&](const PairSt& st, double (&d)[2]) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        // (the trash word's low byte counts 1D increments: excluded SNPs take rank 0)
        const uint32_t r = __builtin_amdgcn_ubfe(st.ov[q], st.xs[q], 8);
        const uint32_t rk = st.kk[q] ? r : 0u;
        ovf |= (st.kk[q] != 0u) & (r == 255u);
        // D(r) for r < 63 from the lanes' registers, lane 63 holding 0: ranks from 63 on add 0 here and
        // the window's end adds F(x) - F(63) for each bin past 63 (a global read of D for them, even
        // in a branch never taken, put a wait for every outstanding load -- the next pair's lp gathers
        // and rows -- into every pair; config 4's bins never pass ~20 SNPs)
        d[q] = __shfl(Dreg, (int)min(rk, 63u));
        big |= rk >= 63u;
      }
    };
    auto finish = [&](const PairSt& st, const double (&d)[2]) {
#pragma unroll
      for (int q = 0; q < 2; ++q) acc2 += d[q] - st.lp[q];
    };
    // The pairs as a rolled loop, two per trip in fixed slots A / B (a pending pair carried through a
    // branch join is copied there, and a copy of registers with loads in flight waits for them: unrolled
    // with the window's length tests, every pair waited for the lp gathers it had just issued -- an L2
    // round trip per pair).  Pair 0 first, then trips of two: the pair count is rounded up to odd (a
    // padding pair's rows are past the window's end, zeros: excluded SNPs).  Rows are buffer loads
    // (range-checked: 0 past the end), two pairs ahead; pairs 0-2 came with the window (bounds()).
    const __amdgpu_buffer_rsrc_t rr = window_rows(bins, cur.b, cur.e, P.nm1);
    uint32_t ro = (uint32_t)lane * 4u;
    asm volatile("" : "+v"(ro));   // (one base + the loads' immediate offsets)
    auto row = [&](int r) -> uint32_t { return __builtin_amdgcn_raw_buffer_load_b32(rr, (int)ro + 256 * r, 0, 0); };
    const int npair = (((int)nsnp + 2 * WAVE - 1) / (2 * WAVE)) | 1;
    PairSt B = issue(cur.u[0], cur.u[1], 0);
    double dB[2], dA[2];
    dlook(B, dB);
    uint32_t x0 = cur.u[2], x1 = cur.u[3], y0 = cur.u[4], y1 = cur.u[5];
    // (scheduling barriers keep each pair's finish after the next pair's issue: hoisted to the loop's
    // top, it waited there for everything in flight)
    for (int p = 1; p < npair; p += 2) {
      const PairSt A = issue(x0, x1, 2 * p);
      x0 = row(2 * p + 4);
      x1 = row(2 * p + 5);
      __builtin_amdgcn_sched_barrier(0);
      finish(B, dB);
      dlook(A, dA);
      __builtin_amdgcn_sched_barrier(0);
      B = issue(y0, y1, 2 * p + 2);
      y0 = row(2 * p + 6);
      y1 = row(2 * p + 7);
      __builtin_amdgcn_sched_barrier(0);
      finish(A, dA);
      dlook(B, dB);
      __builtin_amdgcn_sched_barrier(0);
    }
    finish(B, dB);
    if (!P.fold || filt) {   // rare settings: unfolded (SNPs in the excluded last 2D bin), variant_type filter
      for (uint32_t i0 = cur.b; i0 < cur.e; i0 += WAVE) {   // wave-uniform trip count
        const uint32_t w = i0 + lane < cur.e ? snp_word<CNT>(P, bins, i0 + lane) : 0u;
        nlast += __popcll(__ballot((w & B_LAST) != 0u));
        nvar += __popcll(__ballot((w & B_VAR) != 0u));
      }
    }
    if (!filt) nvar = nsnp;
    // The window's end issues its global loads -- ln of the totals and of the 1D counts (F(x) = x * ln x,
    // the F table's own values) -- before the next window's rows, unconditionally (no branch joins) and
    // with the 1D background terms in registers, so that no wait here is a wait for those rows (loads
    // complete in order; the rows then get the rest of this window's end to arrive)
    auto lnld = [&](uint32_t x) { return lnx[min(x, (uint32_t)LNX_N - 1u)]; };
    // ln of the totals from the global table only when the LDS copy is absent or too short (wave-uniform;
    // the 1D counts are checked below)
    const bool lq0 = P.lnl && (n2 | n1a | n1b) < (uint32_t)LNL;
    double ln2 = 0.0, ln1a = 0.0, ln1b = 0.0;
    if (!lq0) { ln2 = lnld(n2); ln1a = lnld(n1a); ln1b = lnld(n1b); }
    ulonglong2 fq = make_ulonglong2(0ull, 0ull);   // this window's Fst sums (k_prep), used at the end
    if (FST && lane == 0) fq = reinterpret_cast<const ulonglong2*>(fsum)[s];
    if (it == 0) STAMP(12);
    group_sync<WAVE>();
    // 1D spectra: one lane per folded inner bin reads (and clears) its replicas; with <= 32 inner bins
    // per population, lanes 0-31 take population 1 and lanes 32-63 population 2 (acca)
    constexpr uint32_t S1 = 0u;   // (the 1D counts fill their words)
    uint32_t xa[2] = {0u, 0u}, xb[2] = {0u, 0u};
    if (half1d) {
      if (in1h) xa[0] = take_replicas<RG>((lane < 32 ? H1a : H1b) + (1 + (lane & 31)) * RG, S1);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = 1 + lane + WAVE * j;
        if (k <= P.n1p - 1) xa[j] = take_replicas<RG>(H1a + k * RG, S1);
        if (k <= P.n2p - 1) xb[j] = take_replicas<RG>(H1b + k * RG, S1);
      }
    }
    double la[2], lb[2];
    if (lq0 && __ballot((xa[0] | xa[1] | xb[0] | xb[1]) >= (uint32_t)LNL) == 0ull) {
      ln2 = LNLt[n2]; ln1a = LNLt[n1a]; ln1b = LNLt[n1b];
#pragma unroll
      for (int j = 0; j < 2; ++j) { la[j] = LNLt[xa[j]]; lb[j] = LNLt[xb[j]]; }
    } else {
      if (lq0) { ln2 = lnld(n2); ln1a = lnld(n1a); ln1b = lnld(n1b); }
#pragma unroll
      for (int j = 0; j < 2; ++j) { la[j] = lnld(xa[j]); lb[j] = lnld(xb[j]); }
    }
    __builtin_amdgcn_sched_barrier(0);
    // next window: its slot record is in, issue its first rows now (the record made wave-uniform
    // here: its load, issued at the window's start, was otherwise waited for right there)
    Win nxt;
    nxt.has = false;
    bounds(sn, make_uint2(__builtin_amdgcn_readfirstlane(srn.x), __builtin_amdgcn_readfirstlane(srn.y)), nxt, more);
    __builtin_amdgcn_sched_barrier(0);
    const double fn2 = __dmul_rn((double)n2, ln2), fn1a = __dmul_rn((double)n1a, ln1a), fn1b = __dmul_rn((double)n1b, ln1b);
    // x ln x - x lp per inner bin (x = 0: 0, whatever lp -- -inf for an empty background bin)
    double acca = 0.0, accb = 0.0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {   // (half1d: j = 1 adds 0)
      acca += xa[j] ? __dmul_rn((double)xa[j], la[j]) - (double)xa[j] * lp1a[j] : 0.0;
      accb += xb[j] ? __dmul_rn((double)xb[j], lb[j]) - (double)xb[j] * lp1b[j] : 0.0;
    }
    // (consumed here, before any branch: a load's register first used behind a branch join made the
    // wait there conservative -- a wait for the rows just issued)
    asm volatile("" ::"v"(acca), "v"(accb), "v"(fn2), "v"(fn1a), "v"(fn1b), "v"(fq.x), "v"(fq.y));
    // bins with x > 63 SNPs (u8: x <= 254, or the window is re-evaluated exactly below) add
    // F(x) - F(63) (read before the clear; ln x computed, not loaded: no global load after the rows)
    if (__ballot(big) != 0ull) {
      for (int k = lane; k < h2w; k += WAVE) {
        const uint32_t v = W[k];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t x = (v >> (8 * b)) & 0xffu;
          if (x > 63u) acc2 += __dmul_rn((double)x, log((double)x)) - f63;
        }
      }
    }
    // clear the 2D words this window touched (<= 6 steps: all in kw, with trash words)
    if (nsnp <= 6 * WAVE) {
#pragma unroll
      for (int j = 0; j < 8; ++j) W[kw[j]] = 0u;
    } else {
      uint4* q = reinterpret_cast<uint4*>(W);
      for (int k = lane; k < h2w / 4; k += WAVE) q[k] = make_uint4(0, 0, 0, 0);
    }
    if (it == 0) STAMP(13);
    double s2, sa, sb;
    if (half1d) {
      wave_sum_dpp_halves(acc2, acca, s2, sa, sb);
    } else {
      wave_sum3(acc2, acca, accb, s2, sa, sb);
    }
    WinOut w;
    w.snp_count = nvar; w.n2_all = n2 + nlast; w.n2 = n2; w.n1a = n1a; w.n1b = n1b;
    w.t2d = 2.0 * (s2 - fn2);
    w.t1a = 2.0 * (sa - fn1a);
    w.t1b = 2.0 * (sb - fn1b);
    const bool wrapped = __ballot(ovf) != 0ull;
    if (wrapped || cur.e - cur.b >= 65536u || suspect_zero(w.t2d, n2) || suspect_zero(w.t1a, n1a) ||
        suspect_zero(w.t1b, n1b)) {
      // rare: exact re-evaluation with the bin-by-bin proportionality test (histograms are clean)
      group_sync<WAVE>();
      {
        // a u32 histogram in global memory: take a free slot (nscr >= resident waves)
        uint32_t* lock = gscr + (size_t)nscr * P.nb2;
        uint32_t slot = blockIdx.x % (uint32_t)nscr;
        for (;;) {
          uint32_t got = 1u;
          if (lane == 0) got = atomicCAS(&lock[slot], 0u, 1u);
          if (__builtin_amdgcn_readfirstlane(got) == 0u) break;
          slot = slot + 1u == (uint32_t)nscr ? 0u : slot + 1u;
        }
        w = eval_exact<WAVE, false, RG, CNT>(P, bins, cur.b, cur.e, TabGlobal{tab + (size_t)bg * P.nt}, hb, lnx,
                                        gscr + (size_t)slot * P.nb2, H1a, H1b, nullptr, nullptr);
        __threadfence();   // the slot's words are clean again before it is released
        if (lane == 0) atomicExch(&lock[slot], 0u);
      }
      if (lane == 0) atomicAdd(err_word + 1, 1u);   // statistics: windows that took the exact path
    } else {
      if (nan2) w.t2d = __builtin_nan("");
      if (nan1a) w.t1a = __builtin_nan("");
      if (nan1b) w.t1b = __builtin_nan("");
    }
    if (FST && lane == 0) {
      fst_out[s] = fq.y != 0 ? (double)(long long)fq.x / (double)(long long)fq.y : __builtin_nan("");
      reinterpret_cast<ulonglong2*>(fsum)[s] = make_ulonglong2(0ull, 0ull);
    }
    if (lane == 0) {
      write_rec(out + s, ch.chrom, wid, cur.b, cur.e, w, zflags);
    }
    group_sync<WAVE>();
    if (it == 0) STAMP(14);
    cur = nxt;
  }
  STAMP(15);
  WV_STAMP(it);
#ifdef SFS2D_STAMPS
  __builtin_amdgcn_s_barrier();   // diagnostic build only: the block's end is its last active wave's
#endif
  BLK_STAMP(1, 1);
}

// fp64 wave sums on the DPP path without update_dpp's old-value copies (every lane of these
// patterns has a source lane); the rounding order of wave_sum_dpp / wave_sum_dpp_halves
template <int CTRL>
__device__ __forceinline__ double mdpp_d(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(u & 0xffffffffull), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ void wave_sum2_halves(double a, double b, double& s2, double& sa, double& sb) {
  a += mdpp_d<0xB1>(a);  b += mdpp_d<0xB1>(b);
  a += mdpp_d<0x4E>(a);  b += mdpp_d<0x4E>(b);
  a += mdpp_d<0x141>(a); b += mdpp_d<0x141>(b);
  a += mdpp_d<0x140>(a); b += mdpp_d<0x140>(b);
  s2 = (readlane_d(a, 0) + readlane_d(a, 16)) + (readlane_d(a, 32) + readlane_d(a, 48));
  sa = readlane_d(b, 0) + readlane_d(b, 16);
  sb = readlane_d(b, 32) + readlane_d(b, 48);
}
__device__ __forceinline__ double wave_sum1(double v) {
  v += mdpp_d<0xB1>(v);
  v += mdpp_d<0x4E>(v);
  v += mdpp_d<0x141>(v);
  v += mdpp_d<0x140>(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// fp64 wave sums replicated in every lane: the row sums by DPP, then across rows and halves by the
// gfx950 lane swaps (v_permlane16_swap / v_permlane32_swap); a fixed tree, so deterministic
__device__ __forceinline__ double swap16_d(double v, bool upper) {
  const unsigned long long u = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)(u & 0xffffffffull), (uint32_t)(u & 0xffffffffull), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  const uint32_t l = upper ? lo[1] : lo[0], h = upper ? hi[1] : hi[0];
  return __longlong_as_double((long long)(((unsigned long long)h << 32) | l));
}
__device__ __forceinline__ double swap32_d(double v, bool upper) {
  const unsigned long long u = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)(u & 0xffffffffull), (uint32_t)(u & 0xffffffffull), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  const uint32_t l = upper ? lo[1] : lo[0], h = upper ? hi[1] : hi[0];
  return __longlong_as_double((long long)(((unsigned long long)h << 32) | l));
}
// row (16-lane) sums in every lane of the row
__device__ __forceinline__ double row_sum_d(double v) {
  v += mdpp_d<0xB1>(v);    // quad_perm [1,0,3,2]
  v += mdpp_d<0x4E>(v);    // quad_perm [2,3,0,1]
  v += mdpp_d<0x141>(v);   // row_half_mirror
  v += mdpp_d<0x140>(v);   // row_mirror
  return v;
}
// (permlane16_swap(v, v): result 0 holds the even rows' values in both rows of a pair, result 1 the odd
// rows'; permlane32_swap(v, v): result 0 the lower half's in both halves, result 1 the upper half's)
__device__ __forceinline__ double wave_sum_all(double v) {
  v = row_sum_d(v);
  v = swap16_d(v, false) + swap16_d(v, true);
  return swap32_d(v, false) + swap32_d(v, true);
}
// sums of lanes 0-31 (a) and 32-63 (b), both in every lane
__device__ __forceinline__ void wave_sum_halves_all(double v, double& a, double& b) {
  v = row_sum_d(v);
  v = swap16_d(v, false) + swap16_d(v, true);
  a = swap32_d(v, false);
  b = swap32_d(v, true);
}

// the window's five fp64 sums at once, as a reduce-scatter: each lane swap exchanges halves of two
// values (one swap and one add per pair of values instead of per value), and the DPP row steps add two
// interleaved values (even lanes one, odd lanes the other).  In: a (summed over the wave), h (summed over
// lanes 0-31 and over lanes 32-63 separately), f1, f2 (over the wave).  Out, in the lane's own register:
// lane 0 sum(a), lane 16 sum(f1), lane 32 sum(f2), lane 33 sum(h, lanes 0-31), lane 48 sum(h, lanes
// 32-63).  A fixed tree: deterministic.  (Separate replicated sums took ~70 VALU instructions per window,
// this ~35.)
__device__ __forceinline__ void swap32_pair(double x, double y, double& xo, double& yo) {
  const unsigned long long u = __double_as_longlong(x), v = __double_as_longlong(y);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)v, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(v >> 32), false, false);
  xo = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));   // [x lo | y lo]
  yo = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));   // [x hi | y hi]
}
__device__ __forceinline__ void swap16_pair(double x, double y, double& xo, double& yo) {
  const unsigned long long u = __double_as_longlong(x), v = __double_as_longlong(y);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)v, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(v >> 32), false, false);
  xo = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));   // rows x0 y0 x2 y2
  yo = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));   // rows x1 y1 x3 y3
}
__device__ __forceinline__ double wave_sum5(double a, double h, double f1, double f2, uint32_t lane) {
  double x, y;
  swap32_pair(a, f2, x, y);
  const double r1 = x + y;                       // lanes 0-31: a, 32-63: f2 (32-lane partials)
  swap32_pair(f1, h, x, y);
  const double r2 = lane < 32 ? x + y : y;       // lanes 0-31: f1 partial, 32-63: h (own, upper half)
  const double r3 = x;                           // lanes 32-63: h of lanes 0-31
  swap16_pair(r1, r2, x, y);
  const double q = x + y;                        // rows: a, f1, f2, h upper (16-lane partials)
  swap16_pair(r3, r3, x, y);
  const double t = x + y;                        // rows 2, 3: h lower
  const bool odd = lane & 1u;
  double z = odd ? t : q;
  z += mdpp_d<0xB1>(odd ? q : t);                // quad_perm [1,0,3,2]: even lanes q, odd lanes t
  z += mdpp_d<0x4E>(z);                          // quad_perm [2,3,0,1]
  z += mdpp_d<0x124>(z);                         // row_ror:4 (keeps lane parity)
  z += mdpp_d<0x128>(z);                         // row_ror:8
  return z;
}

// three fp64 wave sums (k_scan_gw's 2D and two whole-wave 1D sums), reduce-scatter as wave_sum5: a, b
// exchanged in one lane swap (lanes 0-31 then hold a's partials, 32-63 b's), c folded in both halves,
// one 16-lane swap (rows: a, c, b, c), DPP row steps, three readlanes -- ~27 VALU instructions instead of
// ~69 for three wave_sum_dpp
__device__ __forceinline__ void wave_sum3(double a, double b, double c, double& sa, double& sb, double& sc) {
  double x, y;
  swap32_pair(a, b, x, y);
  const double r1 = x + y;
  swap32_pair(c, c, x, y);
  const double r2 = x + y;
  swap16_pair(r1, r2, x, y);
  double q = x + y;
  q += mdpp_d<0xB1>(q);    // quad_perm [1,0,3,2]
  q += mdpp_d<0x4E>(q);    // quad_perm [2,3,0,1]
  q += mdpp_d<0x124>(q);   // row_ror:4
  q += mdpp_d<0x128>(q);   // row_ror:8
  sa = readlane_d(q, 0);
  sc = readlane_d(q, 16);
  sb = readlane_d(q, 32);
}

// v_writelane_b32 (the LLVM intrinsic: this clang has no builtin for it): lane l (uniform) of `old`
// takes the uniform value v; the compiler puts the lane select in M0
extern "C" __device__ int sfs2d_llvm_writelane(int v, int l, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ uint32_t wlane(uint32_t v, int l, uint32_t old) {
  return (uint32_t)sfs2d_llvm_writelane((int)__builtin_amdgcn_readfirstlane((int)v), l, (int)old);
}


// dst[0, n) = src[0, n) into LDS by the whole workgroup, eight 8-B loads of a thread in flight at once
__device__ __forceinline__ void lds_copy_d(double* dst, const double* __restrict__ src, int n) {
  constexpr int U = 8;
  for (int k0 = threadIdx.x; k0 < n; k0 += U * SBLOCK) {
    double v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = k0 + j * SBLOCK < n ? src[k0 + j * SBLOCK] : 0.0;
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (k0 + j * SBLOCK < n) dst[k0 + j * SBLOCK] = v[j];
  }
}

// K3 for small grids (nb2 <= 8192: the background table in LDS).  Workgroup: 8 wavefronts sharing
// one chromosome's table (prologue: copied from k_bg_slice's output and finished -- "sliced" -- or
// built from this run's replicas -- "fused"); each wavefront scans one window at a time: a static
// first window, then windows from the chromosome's pool counters (the atomic one window ahead of
// its use), the next window's slot record and first 8 rows of bins in flight while the current one
// is finished.  Per window only the per-SNP work and the wave sums run; what is wave-uniform -- the
// T values, the zero / NaN rules, the Fst value, the 64-B record -- is evaluated per lane for a
// batch of windows at once (flush), the rare exact re-evaluations included.  (Measured on config 3:
// the loop is VALU-issue and LDS-latency bound at 4 waves per SIMD; the batched finish took it from
// 405 to ~330 VALU instructions per window.)
// FST: 0 no Fst; 1 k_prep's fixed-point sums of the slot, read and cleared; 2 (counts plans) Hudson's
// terms summed here, per SNP of the rows the window streams anyway (fst_snp on the counts in registers,
// membership = an inner 2D bin; the unfolded last bin in the rare pass), fp64 lane sums in a fixed order
// and two wave sums per window: k_prep then runs without the Fst work (DESIGN.md "Fst placement");
// 3: as 2, for data sets where some SNP has < 2 called alleles in a population (those SNPs masked out)
template <bool P16, bool FUSED, int FST, bool CNT>
// (wgi: the work item -- chunks[wgi] -- and nwg the items of the launch: k_scan_w's block index and grid)
__device__ __forceinline__ void scan_w_small(double* ldsd, uint32_t wgi, uint32_t nwg, SCAN_W_ARGS) {
  constexpr bool FSTIN = FST >= 2;
  constexpr bool FMASK = FST == 3;
  static_assert(!FSTIN || CNT, "Fst in the scan reads the counts");
  constexpr int DT = LNT;   // D(r) entries in LDS
  constexpr int R1U = R1;
  constexpr int NWV = SBLOCK / WAVE;
  // windows per batch (see flush; LDS-limited: the 2 KB of the retired trash words; 16 with two 1D
  // replicas instead of four measured 1-2 us faster than 8 with two: not worth the replicas)
  constexpr int SB = 8;
  __shared__ BgHead sh_hb;
  __shared__ double sh_bd[NWV][3][SB];      // batch: the three sums of window j
  __shared__ uint32_t sh_bu[NWV][5][SB];    // batch: slot, begin, n2 | n2_all, n1a | n1b, nsnp | nvar
  __shared__ unsigned long long sh_bf[NWV][FST ? 2 : 1][SB];   // batch (FST): the slot's Fst sums (FST 2: fp64 bits)
  STAMP(10);
  BLK_STAMP(1, 0);
  const int tid = threadIdx.x;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & (WAVE - 1);
  const Chunk ch = chunks[wgi];
  const int bg = bg_per_chrom ? (int)ch.chrom : 0;

  // LDS: lp table (nt, rounded up to even: the histograms are 16-B aligned) | D (LNT) | F (LNF) |
  // FSTIN: Fst's (1/n, 1/(n(n-1))) for n < P.rtn | histograms
  double* LPl = ldsd;
  double* Dt = LPl + ((P.nt + 1) & ~1);   // DT
  double* Ft = Dt + DT;                   // LNF
  double2* RT = reinterpret_cast<double2*>(Ft + LNF);
  // FSTIN: rtn (1/n, 1/(n(n-1))) pairs
  const int rtn = FSTIN ? P.rtn : 0;
  uint32_t* HB = reinterpret_cast<uint32_t*>(RT + rtn);
  const int h2w = P16 ? ((P.nb2 + 1) / 2 + 3) & ~3 : (P.nb2 + 3) & ~3;
  const int h1w = R1 * (P.n1p + 1), h1wb = R1 * (P.n2p + 1);
  const int per = (h2w + h1w + h1wb + 3) & ~3;   // (16-B rows; no trash words: SNPs outside the 2D SFS skip the atomic)
  uint32_t* W = HB + wv * per;
  uint32_t* H1a = W + h2w;
  uint32_t* H1b = H1a + h1w;
  const uint32_t rep = lane & (R1U - 1);

  // a window's first 8 rows, loaded unconditionally and range-checked (a window that is not there --
  // live false, or an empty slot -- reads a 0-byte range: zeros, no memory access): issued behind a
  // branch, the join made the wait counters merge conservatively, and the row loop waited for the next
  // window's rows as well as this window's
  auto bounds = [&](uint32_t s, uint2 sr, Win& w, bool live) {
    if (mode_bp) {
      w.has = live && sr.x != 0u;
      w.b = sr.x - 1u;
      w.e = sr.y;
    } else {
      w.has = live;
      w.b = ch.cb + (ch.wid_lo + (s - ch.slot_lo)) * P.ws;
      w.e = w.b + P.ws;
    }
    // (counts: 0 past the window's end; bins: masked in the row loop anyway)
    const __amdgpu_buffer_rsrc_t rr = window_rows(bins, w.has ? w.b : 0u, w.has ? w.e : 0u, P.nm1);
    // (the lane's byte offset made opaque here: hoisted out of the window loop, the eight row offsets
    // were kept live as eight VGPRs -- spilled elsewhere -- instead of one base + immediate offsets)
    uint32_t lo = (uint32_t)lane * 4u;
    asm volatile("" : "+v"(lo));
#pragma unroll
    for (int j = 0; j < 8; ++j) w.u[j] = __builtin_amdgcn_raw_buffer_load_b32(rr, (int)lo + 256 * j, 0, 0);
  };
  // window schedule: one static window per wavefront, then the chromosome's pool counters (an
  // atomic is always one window ahead of its use, so its latency hides under a window's work)
  uint32_t s = ch.slot_lo + ch.first + wv;
  const bool active = s < ch.slot_hi;
  const uint2 sr0 = (active && mode_bp) ? slots[s] : make_uint2(0, 0);   // in flight during the table work
  const uint32_t npool = ch.pool & 0xffffu, pool = ch.pool >> 16;
  const bool dyn = ch.slot_lo + ch.nstatic < ch.slot_hi;
  const uint32_t dbase = ch.slot_lo + ch.nstatic + pool;
  uint32_t* myctr = ctr + (((size_t)cpar * P.nchrom + ch.chrom) * CTR_POOLS + pool) * CTR_STRIDE;
  uint32_t gq1 = 0, gq = 0;   // two pool atomics in flight from the start (the schedule runs two ahead)
  if (active && dyn && lane == 0) {
    gq1 = atomicAdd(myctr, 1u);
    gq = atomicAdd(myctr, 1u);
  }
  if (wgi == 0)   // the other parity's counters, for the next run
    for (int k = tid; k < P.nchrom * CTR_POOLS; k += SBLOCK) ctr[((size_t)(1 - cpar) * P.nchrom * CTR_POOLS + k) * CTR_STRIDE] = 0u;

  // table copies with every load of a thread in flight at once (a load-wait-store loop paid one
  // L2/MALL round trip per element: ~4 us of config 2's ~10)
  // the prologue's global loads in flight together (each dependent round trip to L2 / MALL cost ~1 us
  // of config 2's ~4 us prologue): the D / F tables (two doubles per thread), and for sliced plans the
  // leaf sums, the tree nodes and the head's inputs, then the lp table
  static_assert(LNT == SBLOCK && LNF <= SBLOCK, "one D and at most one F double per thread");
  const double dfv0 = dfg[tid], dfv1 = tid < LNF ? dfg[LNT + tid] : 0.0;
  const double2 rtv = (FSTIN && tid < rtn) ? reinterpret_cast<const double2*>(dfg + 2 * LNT)[tid] : make_double2(0.0, 0.0);
  auto stage_fst = [&]() {   // Fst's LDS table
    if (FSTIN && tid < rtn) RT[tid] = rtv;
  };
  BgHead hb;
  const size_t rs = (size_t)P.nchrom * P.nh;     // replica stride
  const uint32_t* Rc = repl + (size_t)par * REPL * rs + (size_t)ch.chrom * P.nh;
  if (!FUSED) {
    double lsv = 0.0;
    int4 my_node = make_int4(0, 0, -1, 0);
    uint32_t bc = 0u;
    Bg1D o{};
    if (sliced) {
      if (tid < nleaves) lsv = leafsum[(size_t)bg * nleaves + tid];
      if (tid < nnodes) my_node = nodes[tid];
      if (tid == 0) { bc = bcount[(size_t)par * P.nchrom + bg]; o = bg1d[bg]; }
    }
    lds_copy_d(LPl, LPg + (size_t)bg * P.nt, P.nt);
    if (tid < DT) Dt[tid] = dfv0;
    if (tid < LNF) Ft[tid] = dfv1;
    stage_fst();
    if (sliced) {
      // this run's per-chromosome table from k_bg_slice (proportions, logs, 1D part final) and its
      // leaf sums: numpy's tree over the leaves, then scipy's p[-1] rule on the 2D table -- the
      // combination k_bg_slice's last block would do, here in every workgroup (no grid-wide
      // completion step between the kernels).  Scratch: the histogram area (zeroed below).
      const bool writer = ch.first == 0 && (int)ch.chrom == write_chrom;
      double* lsum = reinterpret_cast<double*>(HB);
      if (tid < nleaves) lsum[tid] = lsv;
      __syncthreads();
      for (int l = 0; l < nlevels; ++l) {
        if (my_node.z == l) lsum[nleaves + tid] = lsum[my_node.x] + lsum[my_node.y];
        __syncthreads();
      }
      if (tid == 0) {
        const double B2 = (double)bc;
        uint32_t flags = o.flags;
        if (B2 == 0.0) flags |= BGF_B2_ZERO;
        const int M2 = P.nb2 - 2;
        if (M2 >= 1 && B2 != 0.0) {
          const double S = (nleaves + nnodes) ? lsum[nleaves + nnodes - 1] : 0.0;
          const double padj = 1.0 - S;
          if (padj < -1e-15) {
            flags |= BGF_NAN2;
          } else if (fabs(padj) > 1e-15) {
            const double l2 = log(padj);
            LPl[M2] = l2;
            if (writer) { tab[(size_t)bg * P.nt + M2].lp = l2; LPg[(size_t)bg * P.nt + M2] = l2; }
          }
        }
        BgHead h;
        h.B2 = B2; h.B1a = o.B1a; h.B1b = o.B1b; h.flags = flags; h.pad = 0;
        sh_hb = h;
        if (writer) head[bg] = h;
      }
      if (wgi == 0)   // the other parity's inner sums, for the next run
        for (int c = tid; c < P.nchrom; c += SBLOCK) bcount[(size_t)(1 - par) * P.nchrom + c] = 0u;
      __syncthreads();
      hb = sh_hb;
    } else {
      hb = head[bg];
    }
  } else {
    if (tid < DT) Dt[tid] = dfv0;
    if (tid < LNF) Ft[tid] = dfv1;
    stage_fst();
    fused_table(P.nb2, P.nh, P.nt, P.n1p, P.n2p, P.n1, P.n2, P.t1a, P.t1b, P.nchrom, ch.chrom,
                ch.first == 0 && (int)ch.chrom == write_chrom, bg,
                Rc, rs, repl, bcount, par, tab, LPg, head, LPl, HB, leaves, nleaves, nodes, nnodes, nlevels, lnx,
                &sh_hb, reinterpret_cast<double*>(HB) + 1536, HB + FUSED_VCNT);
    hb = sh_hb;
  }
  for (int k = lane; k < per / 4; k += WAVE) reinterpret_cast<uint4*>(W)[k] = make_uint4(0, 0, 0, 0);
  if (tid == 0) LPl[0] = 0.0;   // bin 0 ((0,0), never counted): SNPs outside the 2D SFS read it and add 0
  __syncthreads();
  if (FUSED) {
    // the other parity's replicas and inner sums: zeroed for the next run, a slice per workgroup
    // (after the last barrier: nothing waits for these stores)
    uint32_t* Ro = repl + (size_t)(1 - par) * REPL * rs;
    const size_t tot = (size_t)REPL * rs, share = (tot + nwg - 1) / nwg;
    const size_t lo = (size_t)wgi * share, hi = lo + share < tot ? lo + share : tot;
    for (size_t k = lo + tid; k < hi; k += SBLOCK) Ro[k] = 0u;
    if (wgi == 0)
      for (int c = tid; c < P.nchrom; c += SBLOCK) bcount[(size_t)(1 - par) * P.nchrom + c] = 0u;
  }
  if (!active) return;
  const bool filt = P.ann_want >= 0;
  const bool half1d = P.n1p <= 31 && P.n2p <= 31;   // bins 0..n_p of each population on lanes 0-31 / 32-63
  const uint32_t zflags = bg_zero_flags(hb);
  const bool nan2 = hb.flags & BGF_NAN2, nan1a = hb.flags & BGF_NAN1A, nan1b = hb.flags & BGF_NAN1B;
  uint32_t* const H1a_l = H1a + rep;   // this lane's replica column of the 1D histograms
  uint32_t* const H1b_l = H1b + rep;
  const uint32_t one1 = P16 ? 0x10000u : 1u;   // 1D increment (P16: upper halves, see the window loop)
  // the 1D atomics' LDS byte addresses: per-lane bases kept opaque, so that a bin's address is one
  // v_lshl_add (the compiler otherwise re-splits base + replica + bin into three operations)
  typedef __attribute__((address_space(3))) uint32_t lds_u32;
  uint32_t a1b = (uint32_t)(uintptr_t)((lds_u32*)H1a_l), a2b = (uint32_t)(uintptr_t)((lds_u32*)H1b_l);
  asm volatile("" : "+v"(a1b), "+v"(a2b));
  uint32_t awb = (uint32_t)(uintptr_t)((lds_u32*)W);   // the wave's 2D words (LDS byte address, uniform)
  asm volatile("" : "+s"(awb));
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) d2v lds_d2;   // (16-B aligned: one ds_read_b128)
  const uint32_t rtb = (uint32_t)(uintptr_t)((lds_d2*)RT);   // Fst's reciprocals (LDS byte address)
  // ---- batched finish.  Lane j of the B* registers holds the j-th window this wavefront has
  // scanned since the last flush (slot, SNP range, counts, the three sums); per window only the
  // sums' wave reductions run, and the T values, the zero / NaN rules, the Fst value and the 64-B
  // record of up to 64 windows are computed per lane, in one pass (flush)
  uint32_t jb = 0;
  // lane j holds ln of window j's totals (n2, n1a, n1b), loaded by that lane alone at the window's end:
  // the batched finish then reads no global table (x ln x for x >= LNF came from the global ln table there,
  // an L2 round trip per finish; config 3's totals are ~300-450).  Overlapped config-3 step 0.1808-0.1810
  // vs 0.1822-0.1825 ms (profiles/r06r_scan_finish_ln_prefetch_ab.txt)
  double fl2 = 0.0, fla = 0.0, flb = 0.0;
  auto flush = [&]() {
    MARK(30);
    if (SFS2D_ABL & 512) { jb = 0; return; }
    // (the lane id and the batch addresses recomputed here: kept live across the window loop they
    // were spilled, and their scratch reloads put an L2 round trip in front of every flush)
    uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(ln));
    const bool mine = ln < jb;
    const int jl = ln & (SB - 1);
    const double B2 = sh_bd[wv][0][jl], Ba = sh_bd[wv][1][jl], Bb = sh_bd[wv][2][jl];
    const uint32_t Bs = sh_bu[wv][0][jl], Bsb = sh_bu[wv][1][jl], Bn2 = sh_bu[wv][2][jl], Bn1 = sh_bu[wv][3][jl],
                   Bnv = sh_bu[wv][4][jl];
    const uint32_t nsnp = Bnv & 0xffffu;
    const bool empty = nsnp == 0u;   // a slot with no SNP
    const uint32_t wid = ch.wid_lo + (Bs - ch.slot_lo);
    const uint32_t Bse = Bsb + nsnp;
    WinOut w;
    w.snp_count = Bnv >> 16; w.n2 = Bn2 & 0xffffu; w.n2_all = Bn2 >> 16; w.n1a = Bn1 & 0xffffu; w.n1b = Bn1 >> 16;
    // F(x) = x ln x of the window's totals from the ln values this lane loaded at the window's end
    // (__dmul_rn: the F table's own rounding, k_init_lnx)
    w.t2d = 2.0 * (B2 - __dmul_rn((double)w.n2, fl2));
    w.t1a = 2.0 * (Ba - __dmul_rn((double)w.n1a, fla));
    w.t1b = 2.0 * (Bb - __dmul_rn((double)w.n1b, flb));
    // |T| this small may be an exactly proportional window: the exact evaluation below
    const bool exact = mine && !empty &&
                       (nsnp == 0xffffu || suspect_zero(w.t2d, w.n2) ||
                        suspect_zero(w.t1a, w.n1a) || suspect_zero(w.t1b, w.n1b));
    if (nan2) w.t2d = __builtin_nan("");
    if (nan1a) w.t1a = __builtin_nan("");
    if (nan1b) w.t1b = __builtin_nan("");
    if (empty) { w.t2d = 0.0; w.t1a = 0.0; w.t1b = 0.0; }   // (counts 0: write_empty's record)
    if (mine && !exact)
      if (!(SFS2D_ABL & 8)) write_rec(out + Bs, ch.chrom, wid, empty ? 0u : Bsb, empty ? 0u : Bse, w, empty ? SFS2D_W_EMPTY : zflags);
    if (mine) {
      if (FSTIN) {   // the window's own sums
        const double fx = __longlong_as_double((long long)sh_bf[wv][0][jl]);
        const double fy = __longlong_as_double((long long)sh_bf[wv][FST ? 1 : 0][jl]);
        fst_out[Bs] = fy != 0.0 ? fx / fy : __builtin_nan("");
      } else if (FST) {   // k_prep's fixed-point sums of the slot (read in the window), cleared for the next run
        const long long fx = (long long)sh_bf[wv][0][jl], fy = (long long)sh_bf[wv][FST ? 1 : 0][jl];
        fst_out[Bs] = fy != 0 ? (double)fx / (double)fy : __builtin_nan("");
        reinterpret_cast<ulonglong2*>(fsum)[Bs] = make_ulonglong2(0ull, 0ull);
      }
    }
      if (mine && mode_bp && !FSTIN) {
        // the slot is cleared after its read although k_prep rewrites the table every run: without this
        // store the overlapped Fst-free config-3 pass measured 0.194-0.197 vs 0.162-0.174 ms per pass
        // (profiles/r05r_scan_slot_store_ab.txt).  With Fst in the scan it is left out: no difference in
        // time (profiles/r06g_scan_ablation_noclr.txt) and 8 B fewer scattered writes per window
        uint32_t z = 0u;
        asm volatile("" : "+v"(z));   // (a literal 0 here was taken from a spilled register)
        slots[Bs] = make_uint2(z, z);
      }
    MARK(31);
    // rare: exact re-evaluation with the bin-by-bin proportionality test (the histograms are clean)
    for (unsigned long long m = __ballot(exact); m; m &= m - 1) {
      const int l = __builtin_ctzll(m);
      const uint32_t xs = __builtin_amdgcn_readlane(Bs, l), xb = __builtin_amdgcn_readlane(Bsb, l);
      // (a saturated size: the window's end from its slot record, still in place)
      const uint32_t xn = __builtin_amdgcn_readlane(Bnv, l) & 0xffffu;
      const uint32_t xe = xn != 0xffffu ? xb + xn : (mode_bp ? slots[xs].y : xb + P.ws);
      WinOut x;
      if (FUSED) {
        x = eval_exact<WAVE, P16, R1, CNT>(P, bins, xb, xe,
                                      TabFused{LPl, Rc, rs, P.nb2, P.n1, P.n2, P.n1p, P.h1a, P.h1b, P.t1a, P.t1b}, hb,
                                      lnx, W, H1a, H1b, nullptr, nullptr);
      } else {
        x = eval_exact<WAVE, P16, R1, CNT>(P, bins, xb, xe, TabLocal{tab + (size_t)bg * P.nt, LPl}, hb, lnx, W, H1a, H1b,
                                      nullptr, nullptr);
      }
      if (lane == 0) {
        write_rec(out + xs, ch.chrom, ch.wid_lo + (xs - ch.slot_lo), xb, xe, x, zflags);
        atomicAdd(err_word + 1, 1u);   // statistics: windows that took the exact path
      }
      group_sync<WAVE>();
    }
    jb = 0;
  };
  // window jb of the batch: its integers (lane 0)
  auto put_u = [&](uint32_t slot, uint32_t b, uint32_t nsnp, uint32_t n2, uint32_t n1a, uint32_t n1b, uint32_t nvar,
                   uint32_t nlast) {
    sh_bu[wv][0][jb] = slot;
    sh_bu[wv][1][jb] = b;
    sh_bu[wv][2][jb] = min(n2, 0xffffu) | (min(n2 + nlast, 0xffffu) << 16);
    sh_bu[wv][3][jb] = min(n1a, 0xffffu) | (min(n1b, 0xffffu) << 16);
    sh_bu[wv][4][jb] = min(nsnp, 0xffffu) | (min(nvar, 0xffffu) << 16);
  };
  auto put = [&](uint32_t slot, uint32_t b, uint32_t nsnp, uint32_t n2, uint32_t n1a, uint32_t n1b, uint32_t nvar,
                 uint32_t nlast, double s2, double sa, double sb, ulonglong2 fq) {
    if (lane == 0) {
      sh_bd[wv][0][jb] = s2; sh_bd[wv][1][jb] = sa; sh_bd[wv][2][jb] = sb;
      if (FST) { sh_bf[wv][0][jb] = fq.x; sh_bf[wv][FST ? 1 : 0][jb] = fq.y; }
      put_u(slot, b, nsnp, n2, n1a, n1b, nvar, nlast);
    }
  };
  // the sums from wave_sum5's lanes (FSTIN: the Fst sums too; FST 1: k_prep's, lane 0)
  // put5's store: the five lanes wave_sum5 leaves the sums in each store to their own batch array
  // (one store, the lane's LDS address computed here and kept opaque: per-lane selects in the loop
  // became a branch tree)
  typedef __attribute__((address_space(3))) double lds_f64;
  constexpr unsigned long long OWN5 = 1ull | (1ull << 33) | (1ull << 48) | (FSTIN ? (1ull << 16) | (1ull << 32) : 0ull);
  uint32_t sdst;
  {
    double* d = lane == 0 ? &sh_bd[wv][0][0] : lane == 33 ? &sh_bd[wv][1][0] : lane == 48 ? &sh_bd[wv][2][0]
              : lane == 16 ? reinterpret_cast<double*>(&sh_bf[wv][0][0])
                           : reinterpret_cast<double*>(&sh_bf[wv][FST ? 1 : 0][0]);
    sdst = (uint32_t)(uintptr_t)((lds_f64*)d);
  }
  asm volatile("" : "+v"(sdst));
  auto put5 = [&](double v, ulonglong2 fq) {
    if ((OWN5 >> lane) & 1ull) ((lds_f64*)(uintptr_t)(sdst + 8u * jb))[0] = v;
    if (FST == 1 && lane == 0) { sh_bf[wv][0][jb] = fq.x; sh_bf[wv][FST ? 1 : 0][jb] = fq.y; }
  };


  // the schedule runs two windows ahead: at window i's start the rows of window i+1 are issued (its slot
  // record arrived during window i-1), window i+2's slot record is loaded (its pool index arrived during
  // window i-1) and the pool atomic for window i+3 issued -- a window's rows get a whole window's time to
  // arrive from HBM, and nothing in the row loop waits on a global load (Fst from LDS)
  auto pool_slot = [&](uint32_t g) -> uint32_t {
    const uint32_t j = __builtin_amdgcn_readfirstlane(g);
    return dyn && dbase + npool * j < ch.slot_hi ? dbase + npool * j : ch.slot_hi;
  };
  Win cur;
  bounds(s, sr0, cur, true);
  uint32_t s1 = pool_slot(gq1);
  uint2 sr1 = (mode_bp && s1 < ch.slot_hi) ? slots[s1] : make_uint2(0, 0);
  uint2 srs = make_uint2(0, 0);   // the slot record of window s, for the rows issued after a flush
  STAMP(11);
  int it = 0;
  for (;;) {
  while (s < ch.slot_hi) {
    // the batch's last window prefetches nothing: the flush after it (with the rare exact
    // evaluations) then runs with no rows in flight and no row registers live
    const bool fill = jb + 1u < (uint32_t)SB;   // (prefetching here too, the finish with rows in flight, measured
                                                // slower: 127 VGPRs, profiles/r06u_scan_prefetch_across_finish_ab.txt)
    const bool more = s1 < ch.slot_hi;
    const uint2 sr1u = make_uint2(__builtin_amdgcn_readfirstlane(sr1.x), __builtin_amdgcn_readfirstlane(sr1.y));
    Win nxt;
    nxt.has = false;
    bounds(s1, sr1u, nxt, more && fill);
    const uint32_t s2 = more ? pool_slot(gq) : ch.slot_hi;
    const uint2 sr2 = (mode_bp && s2 < ch.slot_hi) ? slots[s2] : make_uint2(0, 0);
    if (s2 < ch.slot_hi && lane == 0) gq = atomicAdd(myctr, 1u);
    if (!cur.has) {
      put(s, 0u, 0u, 0u, 0u, 0u, 0u, 0u, 0.0, 0.0, 0.0, make_ulonglong2(0ull, 0ull));   // (no SNP: no Fst sums)
      ++jb;
      cur = nxt;
      s = s1; srs = sr1u;
      s1 = s2; sr1 = sr2;
      if (!fill) break;
      continue;
    }
    // SNP j of this lane is b + lane + 64 j: rows of 64 SNPs in pairs, the first 8 rows from the
    // prefetched registers (a row wholly past e is skipped; SNPs past e are w = 0, outside every
    // spectrum).  Per SNP: the 2D LDS atomic (u16 halves) returns the SNP's rank r in its bin and the
    // SNP adds D(r) - lp_k (telescoping: sum_k x_k ln x_k = sum_i D(r_i)); the folded 1D bins are
    // counted in lane & 3 replicas, every SNP slot in one bin of each (the excluded bins 0 and n_p too:
    // dropped at the window's end, which derives n1a / n1b from them).  An SNP outside the 2D spectrum
    // skips the 2D atomic and takes rank 0: D(0) = 0, LPl[0] = 0 (it used to add 0 to a lane-private
    // trash word: 2 KB of LDS per workgroup, now the batch's).  n2 is a wave-uniform ballot count.
    const uint32_t nsnp = cur.e - cur.b;
    const int lim = (int)nsnp - lane;
    const bool clampd = nsnp > (uint32_t)(LNT - 1);   // some rank may pass the D table
    double acc2 = 0.0;
    // FSTIN: this lane's sums of A1 + A2, p1 + p2 and p1 p2 (fst_snp's num = A1 + A2 - 2 p1 p2,
    // den = p1 + p2 - 2 p1 p2, summed per part).  Every SNP takes part: those outside the 2D SFS --
    // bin (0,0) or, folded, both populations fixed for the alternative allele, and the unfolded last
    // bin -- have num = den = 0, as have SNPs with fewer than 2 called alleles in either population
    // (both populations read table entry 0)
    double fA = 0.0, fP = 0.0, fM = 0.0;
    uint32_t n2 = 0, n1a = 0, n1b = 0, nlast = 0, nvar = 0;
    uint32_t kw[8];   // the 2D words of the first 8 rows, cleared after the window
    // FSTIN: the pair's (p, A) of both populations, p = a / n and A = a (a - 1) / (n (n - 1)) from the
    // LDS reciprocals (1/n, 1/(n(n-1))) (0 for n < 2): no global loads in the row loop, so that the next
    // window's rows, issued at this window's start, are never waited for here (loads complete in order).
    // (FMASK: a = 0 in both populations of an SNP without >= 2 called alleles in both -- a data set
    // without such SNPs skips the test: a population alone below n = 2 reads (0, 0))
    auto fst_load = [&](uint32_t w0, uint32_t w1, double2 (&fq)[4]) {
      if (FSTIN) {
        const uint32_t ww[2] = {w0, w1};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint32_t w = ww[q];
          const uint32_t n1c = __builtin_amdgcn_udot4(w, 0x00000101u, 0u, false);
          const uint32_t n2c = __builtin_amdgcn_udot4(w, 0x01010000u, 0u, false);
          uint32_t a1 = __builtin_amdgcn_ubfe(w, 8, 8), a2 = w >> 24;
          if (FMASK) {
            const bool ok = min(n1c, n2c) >= 2u;
            a1 = ok ? a1 : 0u;
            a2 = ok ? a2 : 0u;
          }
          // (a and a (a - 1) converted here: an LDS table of them, two more LDS reads per SNP, made the
          // pass slower -- 143 -> 158 us on config 3: the loop's LDS pipe is the busier one)
          d2v r1, r2;
          if (SFS2D_ABL & 16) {
            r1.x = (double)n1c; r1.y = (double)n1c; r2.x = (double)n2c; r2.y = (double)n2c;
          } else {
            r1 = *(const lds_d2*)(uintptr_t)(rtb + 16u * n1c);
            r2 = *(const lds_d2*)(uintptr_t)(rtb + 16u * n2c);
          }
          fq[2 * q] = make_double2((double)a1 * r1.x, (double)__umul24(a1, a1 - 1u) * r1.y);
          fq[2 * q + 1] = make_double2((double)a2 * r2.x, (double)__umul24(a2, a2 - 1u) * r2.y);
        }
      }
    };
    // SNPs past the window's end: w = 0 (unconditional: a guard on the window's last rows cost more
    // selects than the masking itself); w = 0 is in no spectrum and has no called allele
    auto pair = [&](uint32_t w0, uint32_t w1, int j, bool keep, const double2 (&fq)[4]) {
      const uint32_t ww[2] = {w0, w1};   // (CNT: counts)
      uint32_t rk[2], kk[2], ov[2], xs[2];
      bool in2[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint32_t w = ww[q];
        uint32_t k2, gp;   // gp: the folded 1D bins of both populations (u16 pair; excluded ones included)
        if (CNT) cls_k2g<4 * R1>(P, w, k2, gp);
        else { k2 = bin_k2(w); gp = (bin_g1(w) | (bin_g2(w) << 16)) * (4u * R1); }
        in2[q] = k2 != 0u;   // (one compare: the ballot, the atomic's exec mask, the rank's select)
        n2 += __popcll(__ballot(in2[q]));
        // low five bits: (k2 & 1) << 4, the u16 half's shift
        const uint32_t x = (CNT ? k2 : w) << 4;
        const uint32_t word = P16 ? (k2 >> 1) : k2;   // (k2 = 0: word 0, cleared after the window anyway)
        // (v_lshlrev_b32 / v_bfe_u32 read the shift's low five bits: no mask; C's << would need one)
        uint32_t one2 = 1u;
        if (P16) asm("v_lshlrev_b32 %0, %1, 1" : "=v"(one2) : "v"(x));
        // an SNP outside the 2D SFS skips the atomic (exec mask; its rank is 0 below): no trash word,
        // fewer lanes in the LDS atomic.  (The address before the branch: one v_lshl_add.)
        const uint32_t wa = awb + word * 4u;
        uint32_t o = one2;   // (any value: lanes outside take rank 0; one2's register, dead after the atomic)
        if (in2[q] && !(SFS2D_ABL & 1))
          o = __hip_atomic_fetch_add((lds_u32*)(uintptr_t)wa, one2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ov[q] = o;
        xs[q] = x;
        kk[q] = k2;
        if (keep) kw[(j + q) & 7] = word;
        // every SNP slot adds to one bin of each folded 1D spectrum (no range test, no trash select: the
        // window's end drops bins 0 and n_p and counts n1a / n1b from them)
        // (bin 0 -- the fixed SNPs and every padding slot -- counted by ballot with its atomics on lane-private
        // words measured slower: profiles/r06p_scan_bin0_ballot_ab.txt)
        const uint32_t u1 = a1b + (gp & 0xffffu), u2 = a2b + (gp >> 16);
        if (!(SFS2D_ABL & 2)) {
          __hip_atomic_fetch_add((lds_u32*)(uintptr_t)u1, one1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add((lds_u32*)(uintptr_t)u2, one1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (FSTIN) {   // (SNPs past e: counts 0, no called allele, terms 0)
        // five fp64 operations per SNP on the table's (p, A) (computed from (1/n, 1/(n(n-1))) they took
        // ~20 VALU instructions in a VALU-bound loop; an LDS table measured slower: the loop's LDS pipe
        // is busy, profiles/r03k_fst_scan.txt)
        // (the window's first pair assigns: "x + 0.0" is no identity in fp64 (-0.0), so the adds to the
        // zero-initialised sums would stay in the code)
        const double a0 = fq[0].y + fq[1].y, a1 = fq[2].y + fq[3].y;
        const double p0 = fq[0].x + fq[1].x, p1 = fq[2].x + fq[3].x;
        if (j == 0) {
          fA = a0 + a1;
          fP = p0 + p1;
          fM = fma(fq[2].x, fq[3].x, fq[0].x * fq[1].x);
        } else {
          fA += a0 + a1;
          fP += p0 + p1;
          fM = fma(fq[2].x, fq[3].x, fma(fq[0].x, fq[1].x, fM));
        }
      }
      // the ranks once both SNPs' atomics are issued (extracted right after its own atomic, each rank's
      // wait held the other SNP's work back: two LDS round trips per pair instead of one)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        rk[q] = in2[q] ? (P16 ? __builtin_amdgcn_ubfe(ov[q], xs[q], 16) : ov[q]) : 0u;
      double d[2], lp[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        // D[LNT-1] = 0: ranks past the table add 0 (clampd windows); elsewhere rank < nsnp <= LNT-1 and
        // the min is a no-op, cheaper than selecting it per window
        d[q] = (SFS2D_ABL & 4) ? (double)rk[q] : Dt[min(rk[q], (uint32_t)LNT - 1u)];
        lp[q] = (SFS2D_ABL & 4) ? (double)kk[q] : LPl[kk[q]];
      }
      const double t = (d[0] - lp[0]) + (d[1] - lp[1]);
      acc2 = j == 0 ? t : acc2 + t;
    };
    MARK(19);
#pragma unroll
    for (int j = 0; j < 8; j += 2)
      if (64 * j < (int)nsnp) {
        // (CNT: the loads past the window's end returned 0)
        const uint32_t w0 = (CNT || 64 * j < lim) ? cur.u[j] : 0u, w1 = (CNT || 64 * (j + 1) < lim) ? cur.u[j + 1] : 0u;
        double2 fq[4];
        fst_load(w0, w1, fq);
        pair(w0, w1, j, true, fq);
      }
    MARK(20);
    if (nsnp > 8 * WAVE) {   // rows 8 on (windows of > 512 SNPs), streamed one pair ahead
      const uint32_t* qb = bins + cur.b;
      uint32_t ln = (uint32_t)lane;
      asm volatile("" : "+v"(ln));   // (else bins + lane is hoisted out of the window loop and spilled)
      if (CNT) {   // buffer loads (range-checked: no clamp), rows masked in pair()
        const __amdgpu_buffer_rsrc_t rr = window_rows(bins, cur.b, cur.e, P.nm1);
        int vo = (int)(ln * 4u) + 256 * 8;
        uint32_t x0 = __builtin_amdgcn_raw_buffer_load_b32(rr, vo, 0, 0), x1 = __builtin_amdgcn_raw_buffer_load_b32(rr, vo + 256, 0, 0);
        for (int j = 8; 64 * j < (int)nsnp; j += 2) {
          const uint32_t w0 = x0, w1 = x1;   // (0 past the window's end)
          double2 fq[4];
          fst_load(w0, w1, fq);
          vo += 512;
          x0 = __builtin_amdgcn_raw_buffer_load_b32(rr, vo, 0, 0);
          x1 = __builtin_amdgcn_raw_buffer_load_b32(rr, vo + 256, 0, 0);
          pair(w0, w1, j, false, fq);
        }
        // the last prefetch, consumed here: left in flight, its registers' reuse after the join of this
        // (rare) path with the common one put a wait for every outstanding load -- the next window's rows
        // included -- into every window
        asm volatile("" ::"v"(x0), "v"(x1));
      } else {
        uint32_t x0 = 64 * 8 < lim ? qb[ln + 64 * 8] : 0u, x1 = 64 * 9 < lim ? qb[ln + 64 * 9] : 0u;
        for (int j = 8; 64 * j < (int)nsnp; j += 2) {
          const uint32_t w0 = 64 * j < lim ? x0 : 0u, w1 = 64 * (j + 1) < lim ? x1 : 0u;
          x0 = 64 * (j + 2) < lim ? qb[ln + 64u * (j + 2)] : 0u;
          x1 = 64 * (j + 3) < lim ? qb[ln + 64u * (j + 3)] : 0u;
          double2 fq[4];
          pair(w0, w1, j, false, fq);
        }
      }
    }
    MARK(22);
    if (!P.fold || filt) {   // rare settings: unfolded (SNPs in the excluded last 2D bin), variant_type filter
      for (uint32_t i0 = cur.b; i0 < cur.e; i0 += WAVE) {   // wave-uniform trip count
        const uint32_t w = i0 + lane < cur.e ? snp_word<CNT>(P, bins, i0 + lane) : 0u;
        nlast += __popcll(__ballot((w & B_LAST) != 0u));
        nvar += __popcll(__ballot((w & B_VAR) != 0u));
      }
    }
    if (!filt) nvar = nsnp;
    ulonglong2 fq = make_ulonglong2(0ull, 0ull);   // this window's Fst sums (k_prep): their latency under the window
    if (FST == 1 && lane == 0) fq = reinterpret_cast<const ulonglong2*>(fsum)[s];
    if (it == 0) STAMP(12);
    MARK(23);
    group_sync<WAVE>();
    // bins with x > LNT-1 SNPs: the ranks from LNT-1 on add F(x) - F(LNT-1) (read before the clear)
    if (clampd) {
      constexpr uint32_t L1 = LNT - 1;
      const double fl = (double)L1 * lnx[L1];   // F(LNT-1), as k_init_lnx's table entry
      for (int k = lane; k < h2w; k += WAVE) {
        const uint32_t v = W[k];
        const uint32_t xa = P16 ? (v & 0xffffu) : v, xb = P16 ? (v >> 16) : 0u;
        if (xa > L1) acc2 += (double)xa * lnx_of(lnx, xa) - fl;
        if (xb > L1) acc2 += (double)xb * lnx_of(lnx, xb) - fl;
      }
    }
    // clear the 2D words this window counted: its rows are then dead
    if (nsnp <= 8 * WAVE) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (64 * j < (int)nsnp) W[kw[j]] = 0u;
    } else {
      uint4* q = reinterpret_cast<uint4*>(W);
      for (int k = lane; k < h2w / 4; k += WAVE) q[k] = make_uint4(0, 0, 0, 0);
    }
    MARK(24);
    // 1D spectra: one lane per folded inner bin reads (and clears) its R1 replicas; with <= 32 inner
    // bins per population, lanes 0-31 take population 1 and lanes 32-63 population 2 (acca)
    // (every SNP slot of the rows -- 128 per pair, masked ones included -- is counted in one bin of each
    // spectrum: n1a / n1b = slots - bin 0 - bin n_p)
    double acca = 0.0, accb = 0.0;
    constexpr uint32_t S1 = P16 ? 16u : 0u;
    // (counting only the live slots -- a partial row's live lanes, no row past the end -- measured 1%
    // slower: its uniform tests cost more than the same-address atomics of the padding)
    const uint32_t slots = 128u * ((nsnp + 127u) / 128u);
    // folded bin k (<= n_p) of a population's spectrum, its replicas read and cleared
    auto take1 = [&](uint32_t* H, int k) -> uint32_t {
      if (SFS2D_ABL & 32) return (uint32_t)k;
      return take_replicas<R1U>(H + k * R1, S1);
    };
    if (half1d) {
      const bool pa = lane < 32;
      const int k = lane & 31, np = pa ? P.n1p : P.n2p;
      uint32_t x = 0;
      if (k <= np) {
        x = take1(pa ? H1a : H1b, k);
        if (k >= 1 && k < np && x) acca = xlnx<LNF>(x, Ft, lnx) - (double)x * LPl[(pa ? P.t1a : P.t1b) + k];
      }
      n1a = slots - (uint32_t)__builtin_amdgcn_readlane((int)x, 0) - (uint32_t)__builtin_amdgcn_readlane((int)x, P.n1p);
      n1b = slots - (uint32_t)__builtin_amdgcn_readlane((int)x, 32) -
            (uint32_t)__builtin_amdgcn_readlane((int)x, 32 + P.n2p);
    } else {
      uint32_t xa[2] = {0u, 0u}, xb[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = lane + WAVE * j;
        if (k <= P.n1p) {
          const uint32_t x = take1(H1a, k);
          xa[j] = x;
          if (k >= 1 && k < P.n1p && x) acca += xlnx<LNF>(x, Ft, lnx) - (double)x * LPl[P.t1a + k];
        }
        if (k <= P.n2p) {
          const uint32_t x = take1(H1b, k);
          xb[j] = x;
          if (k >= 1 && k < P.n2p && x) accb += xlnx<LNF>(x, Ft, lnx) - (double)x * LPl[P.t1b + k];
        }
      }
      const uint32_t ea = P.n1p >= WAVE ? (uint32_t)__builtin_amdgcn_readlane((int)xa[1], P.n1p - WAVE)
                                        : (uint32_t)__builtin_amdgcn_readlane((int)xa[0], P.n1p);
      const uint32_t eb = P.n2p >= WAVE ? (uint32_t)__builtin_amdgcn_readlane((int)xb[1], P.n2p - WAVE)
                                        : (uint32_t)__builtin_amdgcn_readlane((int)xb[0], P.n2p);
      n1a = slots - (uint32_t)__builtin_amdgcn_readlane((int)xa[0], 0) - ea;
      n1b = slots - (uint32_t)__builtin_amdgcn_readlane((int)xb[0], 0) - eb;
    }
    if (it == 0) STAMP(13);
    MARK(25);
    // the sums, replicated in every lane (fixed trees: deterministic), into lane jb of the batch
    if (half1d) {
      const double m2 = 2.0 * fM;
      const double v = (SFS2D_ABL & 256) ? acc2 + acca + (FSTIN ? fA - m2 + fP : 0.0)
                                         : wave_sum5(acc2, acca, FSTIN ? fA - m2 : 0.0, FSTIN ? fP - m2 : 0.0, (uint32_t)lane);
      MARK(26);
      put5(v, fq);
      if (lane == 0) put_u(s, cur.b, nsnp, n2, n1a, n1b, nvar, nlast);
      if ((uint32_t)lane == jb) {
        fl2 = lnx[min(n2, 0xffffu)];
        fla = lnx[min(n1a, 0xffffu)];
        flb = lnx[min(n1b, 0xffffu)];
      }
    } else {
      const double s2 = wave_sum_all(acc2);
      const double sa = wave_sum_all(acca), sb = wave_sum_all(accb);
      if (FSTIN) {
        const double m2 = 2.0 * fM;
        fq = make_ulonglong2((unsigned long long)__double_as_longlong(wave_sum_all(fA - m2)),
                             (unsigned long long)__double_as_longlong(wave_sum_all(fP - m2)));
      }
      MARK(26);
      put(s, cur.b, nsnp, n2, n1a, n1b, nvar, nlast, s2, sa, sb, fq);
      if ((uint32_t)lane == jb) {
        fl2 = lnx[min(n2, 0xffffu)];
        fla = lnx[min(n1a, 0xffffu)];
        flb = lnx[min(n1b, 0xffffu)];
      }
    }
    ++jb;
    group_sync<WAVE>();
    if (it == 0) STAMP(14);
    MARK(28);
    ++it;
    cur = nxt;
    s = s1; srs = sr1u;
    s1 = s2; sr1 = sr2;
    if (!fill) break;
  }
  if (jb) flush();   // (a full batch, or the wavefront's last windows)
  if (s >= ch.slot_hi) break;
  bounds(s, srs, cur, true);   // the next batch's first window
  }
  STAMP(15);
  WV_STAMP(it);
#ifdef SFS2D_STAMPS
  __builtin_amdgcn_s_barrier();   // diagnostic build only: the block's end is its last active wave's
#endif
  BLK_STAMP(1, 1);
}

// CNT: `bins` is the counts array (counts plans): every scan classifies the counts it streams
template <bool P16, bool FUSED, int FST, bool CNT>
__global__ __launch_bounds__(SBLOCK) __attribute__((amdgpu_waves_per_eu(4))) void k_scan_w(SCAN_W_ARGS) {
  extern __shared__ double ldsd[];
  scan_w_small<P16, FUSED, FST, CNT>(ldsd, blockIdx.x, gridDim.x, SCAN_W_PASS);
}

// K3 for large grids, one wavefront per window (LDS: the wave's histograms only)
template <bool P16, bool FST, bool CNT, bool TRI = false>
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(4))) void k_scan_gw(SCAN_W_ARGS) {
  extern __shared__ double ldsd[];
  scan_gw_body<P16, FST, CNT, TRI>(ldsd, SCAN_W_PASS);
}

// K3 for large grids: one workgroup per window, exact evaluation.
template <bool P16, bool FST, bool CNT>
__global__ __launch_bounds__(BLOCK) void k_scan_g(KParams P, const uint32_t* __restrict__ bins,
                                                  const Chunk* __restrict__ chunks, uint2* __restrict__ slots,
                                                  const PL* __restrict__ tab, const BgHead* __restrict__ head,
                                                  int bg_per_chrom, const double* __restrict__ lnx,
                                                  sfs2d_window* __restrict__ out, int mode_bp,
                                                  unsigned long long* __restrict__ fsum, double* __restrict__ fst_out) {
  extern __shared__ uint32_t lds[];
  const int h2w = P16 ? (P.nb2 + 1) / 2 : P.nb2;
  const int core = h2w + (P.n1p + 1) + (P.n2p + 1);
  uint32_t* H2 = lds;
  uint32_t* H1a = H2 + h2w;
  uint32_t* H1b = H1a + (P.n1p + 1);
  double* redd = reinterpret_cast<double*>(lds + core + TRASH + ((core + TRASH) & 1));
  unsigned long long* redu = reinterpret_cast<unsigned long long*>(redd + 32);
  for (int k = threadIdx.x; k < core; k += BLOCK) H2[k] = 0u;
  __syncthreads();
  const Chunk ch = chunks[blockIdx.x];
  const int bg = bg_per_chrom ? (int)ch.chrom : 0;
  const PL* T = tab + (size_t)bg * P.nt;
  const BgHead hb = head[bg];
  for (uint32_t s = ch.slot_lo; s < ch.slot_hi; ++s) {
    const uint32_t wid = ch.wid_lo + (s - ch.slot_lo);
    uint32_t b, e;
    if (mode_bp) {
      const uint2 sr = slots[s];
      __syncthreads();
      if (sr.x == 0u) {
        if (threadIdx.x == 0) write_empty(out + s, ch.chrom, wid);
        if (FST && threadIdx.x == 0) fst_out[s] = __builtin_nan("");
        continue;
      }
      b = sr.x - 1u;
      e = sr.y;
    } else {
      b = ch.cb + wid * P.ws;
      e = b + P.ws;
    }
    const WinOut w = eval_exact<BLOCK, P16, 1, CNT>(P, bins, b, e, TabGlobal{T}, hb, lnx, H2, H1a, H1b, redd, redu);
    if (FST && threadIdx.x == 0) fst_out[s] = fst_take(fsum, s);
    if (threadIdx.x == 0) {
      write_rec(out + s, ch.chrom, wid, b, e, w, bg_zero_flags(hb));
    }
  }
}

// first index j in [cb, e) such that SNPs j..e-1 share the fixed-bp window of SNP e-1 (per wave)
__device__ uint32_t window_begin_back(const uint32_t* __restrict__ pos, long long cb, uint32_t e, uint32_t ws) {
  const int lane = threadIdx.x & (WAVE - 1);
  const uint32_t w = wid_of(pos[e - 1], ws);
  long long hi = (long long)e - 1;   // pos[hi] is in the window
  while (true) {
    const long long j = hi - 1 - lane;
    const bool outside = (j < cb) || (wid_of(pos[j], ws) != w);
    const unsigned long long m = __ballot(outside);
    if (m) return (uint32_t)(hi - __builtin_ctzll(m));
    hi -= WAVE;
  }
}

// Q9 helper (combined_scan's final block, twoDSFS_class.py:951-989): the window before the last
// one, evaluated against the LAST window's chromosome background.  One wavefront; launched only
// for plans with SFS2D_F_PREV_EXTRA.
template <bool P16, bool CNT>
__global__ __launch_bounds__(WAVE) void k_scan_extra(KParams P, const uint32_t* __restrict__ bins,
                                                     const uint32_t* __restrict__ pos, uint32_t chrom_last,
                                                     const long long* __restrict__ chrom_off,
                                                     const PL* __restrict__ tab, const BgHead* __restrict__ head,
                                                     int bg_per_chrom, const double* __restrict__ lnx,
                                                     sfs2d_window* __restrict__ out, long long extra_rec) {
  extern __shared__ uint32_t lds[];
  const int h2w = P16 ? (P.nb2 + 1) / 2 : P.nb2;
  const int core = h2w + (P.n1p + 1) + (P.n2p + 1);
  uint32_t* H2 = lds;
  uint32_t* H1a = H2 + h2w;
  uint32_t* H1b = H1a + (P.n1p + 1);
  for (int k = threadIdx.x; k < core; k += WAVE) H2[k] = 0u;
  group_sync<WAVE>();
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
    w = eval_exact<WAVE, P16, 1, CNT>(P, bins, pb, pe, TabGlobal{T}, hb, lnx, H2, H1a, H1b, nullptr, nullptr);
  } else {
    flags |= SFS2D_W_EMPTY;
  }
  if (threadIdx.x == 0) write_rec(out + extra_rec, pc, bl, pb, pe, w, flags);
}


// ------------------------------------------------------------------------------------------ multi-resolution

// Fixed-bp window slots of a plan attached to another plan's k_prep pass (several window sizes from
// one read of the SNP stream; the reference script runs 20 kb, 500 kb and SNP-count scans over the
// same data, twoDSFS_class.py:1923-2032).  One thread per slot: window j of chromosome c holds the
// SNPs with (pos-1)//ws == j (pos 0 -> window 0, as wid_of), found by binary search on the sorted
// positions: slot = (first + 1, last + 1), (0, 0) when empty -- what k_prep's segmentation writes.
__device__ __forceinline__ uint32_t lower_bound_pos(const uint32_t* __restrict__ pos, uint32_t lo, uint32_t hi,
                                                    unsigned long long v) {
  while (lo < hi) {
    const uint32_t mid = lo + ((hi - lo) >> 1);
    if ((unsigned long long)pos[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_slots_bp(const uint32_t* __restrict__ pos, const long long* __restrict__ chrom_off,
                                                  const uint32_t* __restrict__ slot_base, int nchrom, uint32_t ws,
                                                  uint32_t nslots, uint2* __restrict__ slots) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= nslots) return;
  int lo = 0, hi = nchrom;   // chromosome c with slot_base[c] <= s < slot_base[c+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (slot_base[mid] <= s) lo = mid;
    else hi = mid;
  }
  const uint32_t j = s - slot_base[lo];
  const uint32_t cb = (uint32_t)chrom_off[lo], ce = (uint32_t)chrom_off[lo + 1];
  const uint32_t b = j ? lower_bound_pos(pos, cb, ce, (unsigned long long)j * ws + 1ull) : cb;
  const uint32_t e = lower_bound_pos(pos, b, ce, (unsigned long long)(j + 1) * ws + 1ull);
  slots[s] = b < e ? make_uint2(b + 1u, e) : make_uint2(0u, 0u);
}

// The slot table of a fixed-bp counts plan that has no other k_prep work (a supplied background, no Fst
// sums: scan_chooseChr / scan_precomputed_BG / sims_scan.process_window over real replicate VCFs): window j
// of chromosome c is [B_j, B_{j+1}) with B_j the first SNP of c whose pos > j ws (lower_bound of j ws + 1,
// pos 0 in window 0 as wid_of), found by binary search on the resident sorted positions instead of
// k_prep's segmentation pass over every position.  One thread per slot searches B_j; B_{j+1} comes from
// the next lane (the same chromosome's next window), a second search only in a wave's last lane.  A
// wave's 64 windows share the searches' upper levels (one broadcast line each); per window the search
// touches ~6 lines of positions (its deep levels) against the window's whole position run for k_prep
// (config 4: 358 SNPs = 11 lines).  Writes what k_prep's segmentation writes: (first + 1, last + 1),
// (0, 0) for an empty window.
__global__ __launch_bounds__(256) void k_slots_search(const uint32_t* __restrict__ pos,
                                                      const long long* __restrict__ chrom_off,
                                                      const uint32_t* __restrict__ slot_base, int nchrom, uint32_t ws,
                                                      uint32_t nslots, uint2* __restrict__ slots) {
  // (starting from interpolated guesses -- galloping out of the index the chromosome's position range
  // predicts -- measured slower: 0.75-0.77 vs 0.64 ms per config-4 generation; bisection's upper levels are
  // lines the wave shares, profiles/r06z_slot_search_guess_ab.txt)
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  const uint32_t sc = min(s, nslots - 1u);   // (lanes past the end search too: their neighbours read them)
  int lo = 0, hi = nchrom;                   // chromosome c with slot_base[c] <= sc < slot_base[c+1]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (slot_base[mid] <= sc) lo = mid;
    else hi = mid;
  }
  const uint32_t j = sc - slot_base[lo], ns = slot_base[lo + 1] - slot_base[lo];
  const uint32_t cb = (uint32_t)chrom_off[lo], ce = (uint32_t)chrom_off[lo + 1];
  auto lb = [&](uint32_t a, unsigned long long v) -> uint32_t { return lower_bound_pos(pos, a, ce, v); };
  const uint32_t b = j ? lb(cb, (unsigned long long)j * ws + 1ull) : cb;
  uint32_t e = __shfl_down(b, 1, WAVE);
  const bool lastw = j + 1u == ns;
  if (lastw) e = ce;
  else if ((threadIdx.x & (WAVE - 1)) == WAVE - 1 || s + 1u >= nslots)
    e = lb(b, (unsigned long long)(j + 1u) * ws + 1ull);
  if (s < nslots) slots[s] = b < e ? make_uint2(b + 1u, e) : make_uint2(0u, 0u);
}

// Fst sums of an attached fixed-bp plan whose window is m times the base plan's: window j of
// chromosome c is base windows [j*m, (j+1)*m) of c, and the base's int64 fixed-point sums add
// exactly (the same value as k_prep accumulating the attached windows directly).
__global__ __launch_bounds__(256) void k_fst_agg(const unsigned long long* __restrict__ bsum,
                                                 const uint32_t* __restrict__ bslot_base,
                                                 const uint32_t* __restrict__ slot_base, int nchrom, uint32_t m,
                                                 uint32_t nslots, int shift, unsigned long long* __restrict__ fsum) {
  const uint32_t s = blockIdx.x * 256u + threadIdx.x;
  if (s >= nslots) return;
  int lo = 0, hi = nchrom;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (slot_base[mid] <= s) lo = mid;
    else hi = mid;
  }
  const uint32_t j = s - slot_base[lo];
  const uint32_t b0 = bslot_base[lo] + j * m, b1 = min(b0 + m, bslot_base[lo + 1]);
  // the base's sums, rounded to this plan's coarser fixed point (its windows may hold more SNPs)
  const long long half = shift ? 1ll << (shift - 1) : 0ll;
  unsigned long long qn = 0, qd = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    qn += (unsigned long long)(((long long)bsum[2 * (size_t)b] + half) >> shift);
    qd += (unsigned long long)(((long long)bsum[2 * (size_t)b + 1] + half) >> shift);
  }
  fsum[2 * (size_t)s] = qn;
  fsum[2 * (size_t)s + 1] = qd;
}

// ------------------------------------------------------------------------------------------ synthetic sims data

// BASELINE config 4 (sims_scan.likelihood_scan at scale: thousands of replicates x 2,000 windows,
// Poisson(358.5) SNPs per window) generated in HBM instead of parsed from VCFs.  Counter-based
// Philox4x32-10 keyed by (seed) with counter (global SNP index, call, generation): every SNP's draws
// are independent of launch geometry, and the host twin (sfs2d.synth.sims_host) reproduces them bit
// for bit -- only correctly rounded IEEE operations (mul, add, div, sqrt, floor; no contraction:
// the _rn intrinsics) and integer table look-ups.
//   position: window w, SNP j of k_w: w*ws + 1 + floor((j + u) * ws / k_w)  (strictly increasing)
//   ancestral f: u^3 or 1 - u^3 (a U-shaped spectrum); per population f_i = clip(f + 0.1 (u - 1/2))
//   missing alleles: Binomial(2 n_i, miss) by inverse-CDF table (u32 thresholds from the host)
//   alt_i ~ normal approximation of Binomial(m_i, f_i): floor(m f + sqrt(m f (1-f)) z + 1/2) clipped
//   to [0, m], z = (sum of 4 uniforms - 2) * sqrt(3); ref_i = m_i - alt_i
struct SynthP {
  unsigned long long seed;
  uint32_t gen, nwin, ws, n1, n2, nm1, nm2;   // n1 / n2 = 2 * pop size; nm = miss-table length
};

__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x, p1 = (unsigned long long)0xCD9E8D57u * c.z;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    c = make_uint4(h1 ^ c.y ^ k.x, l1, h0 ^ c.w ^ k.y, l0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ double u01(uint32_t x) { return __dmul_rn(__dadd_rn((double)x, 0.5), 2.3283064365386963e-10); }

__device__ __forceinline__ uint32_t synth_alt(double f, uint32_t m, uint4 z4) {
  const double z = __dmul_rn(__dadd_rn(__dadd_rn(__dadd_rn(u01(z4.x), u01(z4.y)), __dadd_rn(u01(z4.z), u01(z4.w))), -2.0),
                             1.7320508075688772);
  const double mf = __dmul_rn((double)m, f);
  const double sd = __dsqrt_rn(__dmul_rn(mf, __dadd_rn(1.0, -f)));
  const double x = floor(__dadd_rn(__dadd_rn(mf, __dmul_rn(sd, z)), 0.5));
  return x <= 0.0 ? 0u : (x >= (double)m ? m : (uint32_t)x);
}

__device__ __forceinline__ uint32_t synth_miss(const uint32_t* __restrict__ tab, uint32_t nt, uint32_t x) {
  uint32_t k = 0;   // smallest k with x < tab[k] (tab: cumulative thresholds, last = 0xffffffff)
  while (k + 1 < nt && x >= tab[k]) ++k;
  return k;
}

__global__ __launch_bounds__(256) void k_synth_sims(SynthP S, const unsigned long long* __restrict__ woff,
                                                    unsigned long long nwtot, const uint32_t* __restrict__ mt1,
                                                    const uint32_t* __restrict__ mt2, uint32_t* __restrict__ counts,
                                                    uint32_t* __restrict__ pos) {
  const int lane = threadIdx.x & (WAVE - 1);
  const unsigned long long nwaves = (unsigned long long)gridDim.x * 4u;
  const uint2 key = make_uint2((uint32_t)S.seed, (uint32_t)(S.seed >> 32));
  for (unsigned long long w = blockIdx.x * 4ull + (threadIdx.x >> 6); w < nwtot; w += nwaves) {
    const unsigned long long o = woff[w], k = woff[w + 1] - o;
    const uint32_t wl = (uint32_t)(w % S.nwin);
    for (unsigned long long j = lane; j < k; j += WAVE) {
      const unsigned long long g = o + j;
      const uint4 a = philox4x32(make_uint4((uint32_t)g, (uint32_t)(g >> 32), 0u, S.gen), key);
      const uint4 b = philox4x32(make_uint4((uint32_t)g, (uint32_t)(g >> 32), 1u, S.gen), key);
      const uint4 z1 = philox4x32(make_uint4((uint32_t)g, (uint32_t)(g >> 32), 2u, S.gen), key);
      const uint4 z2 = philox4x32(make_uint4((uint32_t)g, (uint32_t)(g >> 32), 3u, S.gen), key);
      const double u = u01(a.x);
      const double u3 = __dmul_rn(__dmul_rn(u, u), u);
      const double f = (b.w & 1u) ? u3 : __dadd_rn(1.0, -u3);
      const double f1 = fmin(1.0, fmax(0.0, __dadd_rn(f, __dmul_rn(0.1, __dadd_rn(u01(a.z), -0.5)))));
      const double f2 = fmin(1.0, fmax(0.0, __dadd_rn(f, __dmul_rn(0.1, __dadd_rn(u01(a.w), -0.5)))));
      const uint32_t m1 = S.n1 - synth_miss(mt1, S.nm1, b.x), m2 = S.n2 - synth_miss(mt2, S.nm2, b.y);
      const uint32_t a1 = synth_alt(f1, m1, z1), a2 = synth_alt(f2, m2, z2);
      counts[g] = (m1 - a1) | (a1 << 8) | ((m2 - a2) << 16) | (a2 << 24);
      const double t = __dmul_rn(__dadd_rn((double)j, u01(b.z)), (double)S.ws);
      pos[g] = wl * S.ws + 1u + (uint32_t)floor(__ddiv_rn(t, (double)k));
    }
  }
}

// the slot table of a fixed-bp plan over generated replicates from the generator's window offsets
// (sfs2d_data_synth_sims placed window w's SNPs [woff[w], woff[w+1]) in window w): slot w = (first + 1,
// last + 1) as k_prep's segmentation writes it, (0, 0) for a window without SNPs
__global__ __launch_bounds__(256) void k_slots_synth(const unsigned long long* __restrict__ woff, unsigned long long nw,
                                                     uint2* __restrict__ slots) {
  for (unsigned long long w = (unsigned long long)blockIdx.x * 256 + threadIdx.x; w < nw;
       w += (unsigned long long)gridDim.x * 256) {
    const unsigned long long a = woff[w], b = woff[w + 1];
    slots[w] = b > a ? make_uint2((uint32_t)a + 1u, (uint32_t)b) : make_uint2(0u, 0u);
  }
}

}  // namespace sfs2dk
