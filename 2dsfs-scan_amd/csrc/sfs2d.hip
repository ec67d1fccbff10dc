// sfs2d.hip -- host side + C ABI of the MI355X (gfx950) windowed 2D-SFS composite-likelihood scan.
//
// Device code lives in sfs2d_kernels.hpp (see its header for the statistic and the kernels).
// One run of a plan enqueues, on the context's stream:
//   k_prep         counts + positions (8 B/SNP) -> packed per-SNP bins (4 B/SNP), per-chromosome
//                  background histograms + inner sums, fixed-bp segmentation of the window slots
//   k_bg_slice     per-chromosome background tables (skipped for supplied backgrounds)
//   k_scan_w / _g  bins (4 B/SNP) -> one 64-B record per window slot
//   k_scan_extra   combined_scan's final-window helper (only with SFS2D_F_PREV_EXTRA)
// All device state a run touches (slot table, background replicas and counters, LDS) is left
// zeroed by the run itself, so plans replay without memsets.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "sfs2d.h"
#include "sfs2d_kernels.hpp"

using namespace sfs2dk;

namespace {

// numpy pairwise_sum recursion over n elements: n <= 128 -> leaf (np_leaf_sum), else split at
// n2 = n/2 - (n/2 % 8).  Leaves are numbered left to right; internal nodes get ids nleaves + i
// sorted by height (children before parents, the root last), with level = height - 1, so that a
// node can be combined as soon as its level is reached (same sums, same order inside each node).
struct PwTree {
  std::vector<int2> leaves;   // {offset, n}
  std::vector<int4> nodes;    // {child a, child b, level, 0} (leaf ids < nleaves, node ids >= nleaves)
  int nlevels = 0;
};

int pw_build(int lo, int n, PwTree& t, std::vector<int2>& raw, std::vector<int>& height) {
  // returns a provisional id: >= 0 leaf, < 0 internal node -(i+1)
  if (n <= 128) {
    t.leaves.push_back(make_int2(lo, n));
    return (int)t.leaves.size() - 1;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  const int a = pw_build(lo, n2, t, raw, height);
  const int b = pw_build(lo + n2, n - n2, t, raw, height);
  auto h = [&](int id) { return id >= 0 ? 0 : height[-id - 1]; };
  raw.push_back(make_int2(a, b));
  height.push_back(std::max(h(a), h(b)) + 1);
  return -(int)raw.size();
}

PwTree pw_plan(int n) {
  PwTree t;
  std::vector<int2> raw;
  std::vector<int> height;
  if (n > 0) pw_build(0, n, t, raw, height);
  const int L = (int)t.leaves.size();
  std::vector<int> order(raw.size());
  for (size_t i = 0; i < raw.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return height[x] < height[y]; });
  std::vector<int> newid(raw.size());
  for (size_t i = 0; i < order.size(); ++i) newid[order[i]] = L + (int)i;
  auto remap = [&](int id) { return id >= 0 ? id : newid[-id - 1]; };
  for (int i : order) {
    t.nodes.push_back(make_int4(remap(raw[i].x), remap(raw[i].y), height[i] - 1, 0));
    t.nlevels = std::max(t.nlevels, height[i]);
  }
  return t;
}

// (p-1)/ws as a multiply-high (Granlund-Montgomery, 33-bit magic): q = (t + ((n-t) >> s1)) >> s2
void div_magic(uint32_t d, uint32_t* m, int* s1, int* s2) {
  if (d <= 1) { *m = 0; *s1 = 0; *s2 = 0; return; }
  int l = 0;
  while ((1ull << l) < d) ++l;   // ceil(log2 d)
  *m = (uint32_t)((((unsigned __int128)1 << 32) * (((unsigned __int128)1 << l) - d)) / d + 1);
  *s1 = 1;
  *s2 = l - 1;
}

}  // namespace

// the stream the library enqueues on: the ctx's current one (sfs2d_ctx_set_stream)
#define CTX_STREAM(c) ((c)->stream)

struct sfs2d_ctx {
  int device = 0;
  int ncu = 256;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  double* d_lnx = nullptr;
  double* d_df = nullptr;   // D(r), F(x) (LNT each), then (1/k, 1/(k(k-1))) pairs (RCPN)
  hipEvent_t stagger = nullptr;   // sfs2d_plan_run_streams: the first run's k_prep, awaited by the second stream
  std::string err;
  std::mutex err_mu;
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
  // the largest called allele counts r + a of population 1 / 2 over the data set: counts plans with a
  // supplied background run no pass that validates the counts (k_prep reads none), so they need
  // max_nc1 <= n1 and max_nc2 <= n2 -- then no SNP can raise KeyError (a > 2 pop_size) or leave the
  // grid after the fold; otherwise the plan takes the bins pipeline, whose k_prep raises the error
  uint32_t max_nc1 = 0xffffffffu, max_nc2 = 0xffffffffu;
  // some SNP has fewer than 2 called alleles in a population (unknown: true): Fst summed in the scan
  // must then drop such SNPs explicitly (k_scan_w<..., 3, ...>); without any, the unmasked terms are exact
  bool low_nc = true;
  // sfs2d_data_synth_sims: the generator's window offsets (SNP index of window w's first SNP, nwin + 1
  // entries; w = replicate * win_per_chrom + window), its window length and windows per replicate --
  // fixed-bp plans of that window length take their slot table from them instead of k_prep's
  // segmentation pass over the positions (the generator placed window w's SNPs in its own window)
  unsigned long long* d_win_off = nullptr;
  uint32_t win_bp = 0, win_per_chrom = 0;
};

struct sfs2d_plan {
  sfs2d_ctx* ctx = nullptr;
  const sfs2d_data* data = nullptr;
  sfs2d_params prm{};
  KParams K{};
  int nbg = 0;
  bool do_bg = false, do_seg = false, lds_hist = true, bg_ready = false;
  bool seg_synth = false;   // fixed-bp slots from the generator's window offsets (slots_only)
  bool seg_search = false;  // fixed-bp slots by binary search on the positions, k_slots_search (slots_only)
  bool fused = false;       // per-chromosome tables built inside k_scan_w (parity-alternating replicas)
  bool sliced = false;      // per-chromosome tables by k_bg_slice without its tail; k_scan_w combines
                            // the leaf sums (parity-alternating inner sums)
  bool cnt = false;         // counts plan (no position / variant_type filter): k_prep writes no per-SNP bins,
                            // the scan kernels classify the counts themselves (12 B/SNP per pass instead of 20)
  bool fst = false;         // SFS2D_F_FST: Fst per slot into d_fst
  double* d_fst = nullptr;      // where runs write Fst: d_fst_own, or the caller's (sfs2d_plan_set_fst_out)
  double* d_fst_own = nullptr;
  unsigned long long* d_fsum = nullptr;   // k_prep's per-slot Fst sums (int64 fixed point), cleared by the scan
  int hr = 1;               // k_prep LDS histogram copies per word
  uint64_t runs = 0;        // completed runs (the replica parity of a fused plan)
  int G = 64;               // 64: k_scan_w; 256: large grids (k_scan_gw when gw, else k_scan_g)
  bool gw = false;
  uint32_t* d_gscr = nullptr;   // k_scan_gw: nscr u32 histograms (nb2 words) + nscr lock words, for exact re-evaluations
  int nscr = 0;
  bool p16 = true;
  size_t scan_lds = 0, bg_lds = 0, extra_lds = 0;
  int64_t nslots = 0, nrec = 0, extra_rec = -1;
  uint32_t last_chrom = 0;
  std::vector<Tile> tiles;
  std::vector<Chunk> chunks;
  std::vector<int4> slices;
  Tile* d_tiles = nullptr;
  Chunk* d_chunks = nullptr;
  uint2* d_slots = nullptr;
  uint32_t* d_repl = nullptr;
  uint32_t* d_bcount = nullptr;   // per-chromosome inner 2D sums (k_prep -> k_bg_slice)
  uint32_t* d_done = nullptr;     // per-background completion counters of k_bg_slice
  uint32_t* d_ctr = nullptr;      // k_scan_w window pool counters, 2 parities x nchrom x CTR_POOLS lines
  double* d_bgval = nullptr;
  PL* d_tab = nullptr;
  double* d_lp = nullptr;         // log proportions alone (k_scan_w stages them in LDS)
  BgHead* d_head = nullptr;
  Bg1D* d_bg1d = nullptr;
  double* d_leafsum = nullptr;
  int2* d_leaves = nullptr;
  int4* d_nodes = nullptr;
  int4* d_slices = nullptr;
  int nleaves = 0, nnodes = 0, nlevels = 0;
  uint32_t* d_bins = nullptr;     // packed per-SNP bins written by k_prep, read by the scan kernels
  sfs2d_window* d_out = nullptr;
  uint32_t* d_err = nullptr;
  sfs2d_window* last_out = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // live timing ring: events around each kernel of every run while timing is on
  bool timing = false;
  std::vector<hipEvent_t> tev;   // 6 per sampled run (start / end of k_prep, k_bg_slice, the scan)
  int tcount = 0;
  int tmax = 0;                  // samples of the current timing session (<= tev.size() / 6)
  int tevery = 1;                // sample every tevery-th run
  int tmask = 7;                 // kernels with events: bit 0 k_prep, 1 k_bg_slice, 2 the scan kernel
  int64_t tseen = 0;             // runs since timing was set
  hipEvent_t* tpend = nullptr;   // a sampled run's events between its phase 1 and phase 2
  // events of the run being enqueued: k_prep start/stop, scan start/stop (null: not sampled).  They
  // go into the kernels' own dispatch packets (hipExtLaunchKernelGGL), so they stamp the kernel's
  // start and end as the command processor sees them -- the durations rocprofv3 reports.
  hipEvent_t kev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // multi-resolution (sfs2d_plan_attach): an attached plan shares its base's k_prep pass (bins,
  // background replicas, inner sums); the base's run scans every attached plan before its own
  std::vector<unsigned long long> slot_base_h;   // window slots per chromosome (prefix sums)
  uint32_t* d_slot_base = nullptr;
  sfs2d_plan* base = nullptr;
  std::vector<sfs2d_plan*> attached;
  uint32_t fst_m = 0;             // attached Fst: base windows per window (their sums add)
  bool fst_win = false;           // Fst by window kernels (fst_windows) instead of k_prep's sums
  bool fst_scan = false;          // Fst summed by k_scan_w itself (counts plans, small grids): k_prep has no Fst work
  bool fst_mask = true;           // Fst in the scan: the data set has SNPs with < 2 called alleles (k_scan_w FST 3 / 5)
  int nfst = 0;                   // k_bg_slice's extra Fst workgroups
};

namespace {

int set_err(sfs2d_ctx* ctx, int code, const std::string& m) {
  if (ctx) {   // (callers may use several ctx objects from several threads)
    std::lock_guard<std::mutex> g(ctx->err_mu);
    ctx->err = m;
  }
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
  if (p->base) {   // shared with the base plan
    p->d_bins = nullptr;
    p->d_repl = nullptr;
    p->d_bcount = nullptr;
    if (p->sliced) {
      p->d_tab = nullptr; p->d_lp = nullptr; p->d_head = nullptr; p->d_leafsum = nullptr; p->d_bg1d = nullptr;
    } else if (p->do_bg && p->G != WAVE) {
      p->d_tab = nullptr; p->d_lp = nullptr; p->d_head = nullptr;
    }
  }
  hipFree(p->d_slot_base);
  hipFree(p->d_tiles); hipFree(p->d_chunks); hipFree(p->d_slots); hipFree(p->d_repl); hipFree(p->d_bcount); hipFree(p->d_ctr);
  hipFree(p->d_done); hipFree(p->d_bgval); hipFree(p->d_tab); hipFree(p->d_lp); hipFree(p->d_head);
  hipFree(p->d_bg1d); hipFree(p->d_leafsum); hipFree(p->d_leaves); hipFree(p->d_nodes); hipFree(p->d_slices);
  hipFree(p->d_out); hipFree(p->d_err); hipFree(p->d_bins); hipFree(p->d_fst_own); hipFree(p->d_fsum); hipFree(p->d_gscr);
  for (auto& e : p->ev) if (e) hipEventDestroy(e);
  for (auto& e : p->tev) if (e) hipEventDestroy(e);
}

// replica parity of the current run (an attached plan reads its base's k_prep output)
int plan_par(const sfs2d_plan* pl) {
  return (pl->fused || pl->sliced) ? (int)((pl->base ? pl->base->runs : pl->runs) & 1) : 0;
}
// replica parity: only fused plans alternate replicas (k_bg_slice clears what it reads)
int repl_par(const sfs2d_plan* pl) { return pl->fused ? plan_par(pl) : 0; }

// what the scan kernels stream per SNP: the bins k_prep wrote, or (counts plans) the counts themselves
const uint32_t* scan_src(const sfs2d_plan* pl) { return pl->cnt ? pl->data->counts : pl->d_bins; }

template <bool P16, bool FUSED, int FST, bool CNT>
void launch_scan_w(sfs2d_plan* pl, sfs2d_window* out, int per_chrom, int bp) {
  hipExtLaunchKernelGGL((k_scan_w<P16, FUSED, FST, CNT>), dim3((unsigned)pl->chunks.size()), dim3(SBLOCK), pl->scan_lds,
                     CTX_STREAM(pl->ctx), pl->kev[4], pl->kev[5], 0, pl->K, scan_src(pl), pl->d_chunks, pl->d_slots, pl->d_tab, pl->d_lp, pl->d_head,
                     per_chrom, pl->ctx->d_lnx, pl->ctx->d_df, out, pl->d_err, bp, pl->d_repl, pl->d_bcount,
                     plan_par(pl), pl->d_leaves, pl->nleaves, pl->d_nodes, pl->nnodes, pl->nlevels,
                     pl->extra_rec >= 0 ? (int)pl->last_chrom : -1, pl->d_fsum, pl->d_fst, pl->d_ctr,
                     (int)(pl->runs & 1), pl->d_leafsum, pl->d_bg1d, pl->sliced ? 1 : 0, nullptr, 0);
}

template <bool P16, bool FST, bool CNT>
void launch_scan_g(sfs2d_plan* pl, sfs2d_window* out, int per_chrom, int bp) {
  hipExtLaunchKernelGGL((k_scan_g<P16, FST, CNT>), dim3((unsigned)pl->chunks.size()), dim3(BLOCK), pl->scan_lds,
                     CTX_STREAM(pl->ctx), pl->kev[4], pl->kev[5], 0, pl->K, scan_src(pl), pl->d_chunks, pl->d_slots, pl->d_tab, pl->d_head, per_chrom,
                     pl->ctx->d_lnx, out, bp, pl->d_fsum, pl->d_fst);
}

template <bool P16, bool FST, bool CNT, bool TRI = false>
void launch_scan_gw(sfs2d_plan* pl, sfs2d_window* out, int per_chrom, int bp) {
  hipExtLaunchKernelGGL((k_scan_gw<P16, FST, CNT, TRI>), dim3((unsigned)pl->chunks.size()), dim3(WAVE), pl->scan_lds,
                     CTX_STREAM(pl->ctx), pl->kev[4], pl->kev[5], 0, pl->K, scan_src(pl), pl->d_chunks, pl->d_slots, pl->d_tab, pl->d_lp, pl->d_head,
                     per_chrom, pl->ctx->d_lnx, pl->ctx->d_df, out, pl->d_err, bp, pl->d_repl, pl->d_bcount,
                     0, pl->d_leaves, pl->nleaves, pl->d_nodes, pl->nnodes, pl->nlevels, -1, pl->d_fsum, pl->d_fst,
                     pl->d_ctr, (int)(pl->runs & 1), pl->d_leafsum, pl->d_bg1d, 0, pl->d_gscr, pl->nscr);
}

template <bool P16, bool CNT>
hipError_t launch_scan_c(sfs2d_plan* pl, sfs2d_window* out) {
  const int per_chrom = pl->prm.bg_mode == SFS2D_BG_PER_CHROM ? 1 : 0;
  const int bp = pl->prm.window_mode == SFS2D_WINDOW_BP ? 1 : 0;
  if (pl->gw) {
    if (CNT && pl->K.ntri) {
      if (pl->fst) launch_scan_gw<P16, true, CNT, CNT>(pl, out, per_chrom, bp);
      else launch_scan_gw<P16, false, CNT, CNT>(pl, out, per_chrom, bp);
    } else if (pl->fst) {
      launch_scan_gw<P16, true, CNT>(pl, out, per_chrom, bp);
    } else {
      launch_scan_gw<P16, false, CNT>(pl, out, per_chrom, bp);
    }
  } else if (pl->G == WAVE) {
    if constexpr (CNT) {
      if (pl->fst_scan) {
        if (pl->fst_mask) {
          if (pl->fused) launch_scan_w<P16, true, 3, CNT>(pl, out, per_chrom, bp);
          else launch_scan_w<P16, false, 3, CNT>(pl, out, per_chrom, bp);
        } else {
          if (pl->fused) launch_scan_w<P16, true, 2, CNT>(pl, out, per_chrom, bp);
          else launch_scan_w<P16, false, 2, CNT>(pl, out, per_chrom, bp);
        }
        return hipGetLastError();
      }
    }
    if (pl->fused) {
      if (pl->fst && !pl->fst_win) launch_scan_w<P16, true, true, CNT>(pl, out, per_chrom, bp);
      else launch_scan_w<P16, true, false, CNT>(pl, out, per_chrom, bp);
    } else {
      if (pl->fst && !pl->fst_win) launch_scan_w<P16, false, true, CNT>(pl, out, per_chrom, bp);
      else launch_scan_w<P16, false, false, CNT>(pl, out, per_chrom, bp);
    }
  } else {
    if (pl->fst) launch_scan_g<P16, true, CNT>(pl, out, per_chrom, bp);
    else launch_scan_g<P16, false, CNT>(pl, out, per_chrom, bp);
  }
  return hipGetLastError();
}

template <bool P16>
hipError_t launch_scan(sfs2d_plan* pl, sfs2d_window* out) {
  return pl->cnt ? launch_scan_c<P16, true>(pl, out) : launch_scan_c<P16, false>(pl, out);
}

template <bool B, bool S, bool L, bool N, bool F, bool FS>
hipError_t launch_prep3(sfs2d_plan* pl) {
  const sfs2d_data* d = pl->data;
  const int par = plan_par(pl);
  hipExtLaunchKernelGGL((k_prep<B, S, L, N, F, FS>), dim3((unsigned)pl->tiles.size()), dim3(BLOCK1),
                     (B && L) ? pl->bg_lds : 0, CTX_STREAM(pl->ctx), pl->kev[0], pl->kev[1], 0, pl->K, d->counts, d->pos, d->ann, pl->d_tiles,
                     pl->d_repl + (size_t)repl_par(pl) * REPL * pl->K.nchrom * pl->K.nh, pl->d_slots, pl->d_bins,
                     pl->d_bcount + (size_t)par * pl->K.nchrom, pl->d_err, L ? pl->hr : 1,
                     reinterpret_cast<const double2*>(pl->ctx->d_df + 2 * LNT), pl->d_fsum);
  return hipGetLastError();
}

template <bool B, bool S, bool L, bool N, bool F>
hipError_t launch_prep2(sfs2d_plan* pl) {
  // Fst sums with a plan's pass (the bins pass, or a counts plan's bins-less one); not in sfs2d_bg_hist
  if (pl->fst && !pl->fst_win && !pl->fst_scan && (N || pl->cnt)) return launch_prep3<B, S, L, N, F, true>(pl);
  return launch_prep3<B, S, L, N, F, false>(pl);
}

template <bool B, bool S, bool L, bool N>
hipError_t launch_prep1(sfs2d_plan* pl) {
  const bool f = pl->K.ann_want >= 0 || pl->K.has_start || pl->K.has_end;
  return f ? launch_prep2<B, S, L, N, true>(pl) : launch_prep2<B, S, L, N, false>(pl);
}

// k_prep for a plan run: a counts plan's pass stores no bins (and is skipped when it has nothing to do:
// supplied background, SNP-count windows, no Fst sums)
hipError_t launch_prep_cnt(sfs2d_plan* pl) {
  const bool L = pl->lds_hist;
  const bool fs = pl->fst && !pl->fst_win && !pl->fst_scan;
  if (pl->do_bg && pl->do_seg)
    return L ? launch_prep1<true, true, true, false>(pl) : launch_prep1<true, true, false, false>(pl);
  if (pl->do_bg) return L ? launch_prep1<true, false, true, false>(pl) : launch_prep1<true, false, false, false>(pl);
  if (pl->do_seg) return launch_prep1<false, true, false, false>(pl);
  if (fs) return launch_prep1<false, false, false, false>(pl);
  return hipSuccess;
}

// whether a run takes its slot table from the generator's window offsets or a binary search on the
// positions instead of k_prep (seg_synth / seg_search; k_prep's Fst sums or an attached plan's use of its
// pass keep k_prep)
bool slots_only(const sfs2d_plan* pl) {
  return (pl->seg_synth || pl->seg_search) && pl->attached.empty() && !(pl->fst && !pl->fst_win && !pl->fst_scan);
}

hipError_t launch_slots_only(sfs2d_plan* pl) {
  const unsigned long long nw = (unsigned long long)pl->nslots;
  // (the k_prep timing slot: this is the run's segmentation stage)
  if (nw && pl->seg_synth)
    hipExtLaunchKernelGGL(k_slots_synth, dim3((unsigned)std::min<unsigned long long>(8192, (nw + 255) / 256)), dim3(256),
                          0, CTX_STREAM(pl->ctx), pl->kev[0], pl->kev[1], 0, pl->data->d_win_off, nw, pl->d_slots);
  else if (nw)
    hipExtLaunchKernelGGL(k_slots_search, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, CTX_STREAM(pl->ctx),
                          pl->kev[0], pl->kev[1], 0, pl->data->pos, pl->data->d_chrom_off, pl->d_slot_base,
                          pl->data->nchrom, (uint32_t)pl->prm.window, (uint32_t)nw, pl->d_slots);
  return hipGetLastError();
}

// whether a plan run launches k_prep at all
bool prep_runs(const sfs2d_plan* pl) {
  return !pl->tiles.empty() && (!pl->cnt || pl->do_bg || pl->do_seg || (pl->fst && !pl->fst_win && !pl->fst_scan));
}

hipError_t launch_prep(sfs2d_plan* pl, bool bins) {
  if (pl->tiles.empty()) return hipSuccess;
  const bool L = pl->lds_hist;
  if (!bins) return L ? launch_prep1<true, false, true, false>(pl) : launch_prep1<true, false, false, false>(pl);
  if (pl->cnt) return launch_prep_cnt(pl);
  if (pl->do_bg && pl->do_seg)
    return L ? launch_prep1<true, true, true, true>(pl) : launch_prep1<true, true, false, true>(pl);
  if (pl->do_bg) return L ? launch_prep1<true, false, true, true>(pl) : launch_prep1<true, false, false, true>(pl);
  if (pl->do_seg) return launch_prep1<false, true, false, true>(pl);
  return launch_prep1<false, false, false, true>(pl);
}

// per-run per-chromosome backgrounds
hipError_t launch_bg_slices(sfs2d_plan* pl) {
  hipExtLaunchKernelGGL(k_bg_slice, dim3((unsigned)pl->slices.size() + 1 + (unsigned)pl->nfst, (unsigned)pl->nbg), dim3(KBLOCK), 0,
                     CTX_STREAM(pl->ctx), pl->kev[2], pl->kev[3], 0, pl->K, pl->d_repl, pl->d_bcount + (size_t)plan_par(pl) * pl->K.nchrom, pl->d_tab,
                     pl->d_lp, pl->d_head, pl->d_leafsum, pl->d_bg1d, pl->d_done, pl->d_slices, (int)pl->slices.size(),
                     pl->d_leaves, pl->nleaves, pl->d_nodes, pl->nnodes, pl->nlevels, pl->sliced ? 0 : 1, pl->nfst,
                     pl->data->counts, scan_src(pl), pl->d_slots, reinterpret_cast<const double2*>(pl->ctx->d_df + 2 * LNT),
                     pl->d_fst, (uint32_t)pl->nslots);
  return hipGetLastError();
}

// one supplied background (values uploaded to d_bgval)
hipError_t launch_finalize(sfs2d_plan* pl, int integer_values) {
  const size_t lds = pl->K.nt <= FIN_LDS_BINS ? sizeof(double) * pl->K.nt : 0;
  hipLaunchKernelGGL(k_bg_finalize, dim3(1), dim3(FBLOCK), lds, CTX_STREAM(pl->ctx), pl->K, integer_values, pl->d_bgval,
                     pl->d_bgval, pl->d_tab, pl->d_lp, pl->d_head, pl->d_leaves, pl->nleaves, pl->d_nodes, pl->nnodes);
  return hipGetLastError();
}

template <bool P16, bool CNT>
hipError_t launch_extra(sfs2d_plan* pl, sfs2d_window* out) {
  const sfs2d_data* d = pl->data;
  hipLaunchKernelGGL((k_scan_extra<P16, CNT>), dim3(1), dim3(WAVE), pl->extra_lds, CTX_STREAM(pl->ctx), pl->K, scan_src(pl),
                     d->pos, pl->last_chrom, d->d_chrom_off, pl->d_tab, pl->d_head,
                     pl->prm.bg_mode == SFS2D_BG_PER_CHROM ? 1 : 0, pl->ctx->d_lnx, out, (long long)pl->extra_rec);
  return hipGetLastError();
}

hipError_t launch_scan_any(sfs2d_plan* pl, sfs2d_window* out) {
  hipError_t e = hipSuccess;
  if (!pl->chunks.empty()) e = pl->p16 ? launch_scan<true>(pl, out) : launch_scan<false>(pl, out);
  if (e == hipSuccess && pl->extra_rec >= 0)
    e = pl->p16 ? (pl->cnt ? launch_extra<true, true>(pl, out) : launch_extra<true, false>(pl, out))
                : (pl->cnt ? launch_extra<false, true>(pl, out) : launch_extra<false, false>(pl, out));
  return e;
}

// one attached plan inside its base's run: its window slots (fixed bp: binary search on the
// positions), its Fst sums (from the base's), then its scan against the base's k_prep output
hipError_t launch_attached(sfs2d_plan* a) {
  const sfs2d_data* d = a->data;
  const uint32_t ns = (uint32_t)a->nslots;
  if (!ns) { a->runs++; return hipSuccess; }
  const dim3 g((ns + 255) / 256);
  if (a->prm.window_mode == SFS2D_WINDOW_BP)
    hipLaunchKernelGGL(k_slots_bp, g, dim3(256), 0, CTX_STREAM(a->ctx), d->pos, d->d_chrom_off, a->d_slot_base,
                       d->nchrom, (uint32_t)a->prm.window, ns, a->d_slots);
  if (a->fst_m)
    hipLaunchKernelGGL(k_fst_agg, g, dim3(256), 0, CTX_STREAM(a->ctx), a->base->d_fsum, a->base->d_slot_base,
                       a->d_slot_base, d->nchrom, a->fst_m, ns,
                       std::max(0, a->base->K.fst_e - a->K.fst_e), a->d_fsum);
  if (a->fst_win) {   // before the scan clears the slots
    const dim3 gf((unsigned)std::min<uint32_t>(2048u, (ns + 3u) / 4u));
    if (a->cnt)
      hipLaunchKernelGGL(k_fst_win<true>, gf, dim3(256), 0, CTX_STREAM(a->ctx), a->K, d->counts, scan_src(a), a->d_slots,
                         reinterpret_cast<const double2*>(a->ctx->d_df + 2 * LNT), a->d_fst, ns);
    else
      hipLaunchKernelGGL(k_fst_win<false>, gf, dim3(256), 0, CTX_STREAM(a->ctx), a->K, d->counts, scan_src(a), a->d_slots,
                         reinterpret_cast<const double2*>(a->ctx->d_df + 2 * LNT), a->d_fst, ns);
  }
  const hipError_t e = launch_scan_any(a, a->d_out);
  a->last_out = a->d_out;
  a->runs++;
  return e;
}

}  // namespace

// ------------------------------------------------------------------------------------------ C ABI

extern "C" {

// an ablation build (-DSFS2D_ABL=..., timing only, wrong results) reports a negative version, which the
// loaders refuse (sfs2d/_lib.py) unless SFS2D_ALLOW_ABLATION=1 is set by the timing tool
int sfs2d_abi_version(void) { return SFS2D_ABL ? -SFS2D_ABL : SFS2D_ABI_VERSION; }

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
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) c->ncu = prop.multiProcessorCount;
  if (dalloc(c, &c->d_lnx, LNX_N) || dalloc(c, &c->d_df, 2 * LNT + 2 * RCPN)) {
    hipFree(c->d_lnx); hipStreamDestroy(c->own); delete c; return SFS2D_E_NOMEM;
  }
  hipLaunchKernelGGL(k_init_lnx, dim3(LNX_N / 256), dim3(256), 0, c->stream, c->d_lnx, c->d_df, c->d_df + LNT,
                     c->d_df + 2 * LNT);
  if (hipStreamSynchronize(c->stream) != hipSuccess) {
    hipFree(c->d_lnx); hipFree(c->d_df); hipStreamDestroy(c->own); delete c; return SFS2D_E_HIP;
  }
  *out = c;
  return 0;
}

int sfs2d_ctx_destroy(sfs2d_ctx* ctx) {
  if (!ctx) return SFS2D_E_ARG;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(CTX_STREAM(ctx));
  hipFree(ctx->d_lnx);
  hipFree(ctx->d_df);
  if (ctx->stagger) hipEventDestroy(ctx->stagger);
  hipStreamDestroy(ctx->own);
  delete ctx;
  return 0;
}

// NULL is the HIP null stream (ordered with the process's blocking streams), not the ctx's own: a
// caller passing its default stream's handle (torch's is 0) gets the ordering it expects
int sfs2d_ctx_set_stream(sfs2d_ctx* ctx, void* stream) {
  if (!ctx) return SFS2D_E_ARG;
  ctx->stream = (hipStream_t)stream;
  return 0;
}

int sfs2d_ctx_get_stream(const sfs2d_ctx* ctx, void** stream) {
  if (!ctx || !stream) return SFS2D_E_ARG;
  *stream = (void*)ctx->stream;
  return 0;
}

int sfs2d_ctx_use_own_stream(sfs2d_ctx* ctx) {
  if (!ctx) return SFS2D_E_ARG;
  ctx->stream = ctx->own;
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
  {
    uint32_t m1 = 0, m2 = 0;
    bool low = false;
    for (int64_t i = 0; i < n; ++i) {
      const uint32_t c = counts[i];
      const uint32_t n1c = (c & 0xffu) + ((c >> 8) & 0xffu), n2c = ((c >> 16) & 0xffu) + (c >> 24);
      m1 = std::max(m1, n1c);
      m2 = std::max(m2, n2c);
      low |= std::min(n1c, n2c) < 2u;
    }
    d->max_nc1 = m1;
    d->max_nc2 = m2;
    d->low_nc = low;
  }
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
  if (((uintptr_t)d_counts & 15) || ((uintptr_t)d_pos & 15) || ((uintptr_t)d_ann_id & 7)) {
    hipFree(d->d_chrom_off); delete d;
    return set_err(ctx, SFS2D_E_ARG, "device arrays must be 16-byte aligned (and readable to round_up(n, 4))");
  }
  d->counts = const_cast<uint32_t*>(d_counts);
  d->pos = const_cast<uint32_t*>(d_pos);
  if (d_ann_id) {
    d->ann = const_cast<uint16_t*>(d_ann_id);
  } else {
    const size_t na = ((size_t)n + 3) / 4 * 4 + 64;
    if (dalloc(ctx, &d->ann, na) || hipMemset(d->ann, 0, sizeof(uint16_t) * na) != hipSuccess) {
      hipFree(d->d_chrom_off); delete d; return SFS2D_E_NOMEM;
    }
    d->ann_owned = true;
  }
  d->last_pos.assign(chrom_last_pos, chrom_last_pos + nchrom);
  d->strict = true;   // contract: positions strictly increasing within each chromosome
  if (n > 0) {   // the largest called counts (see max_nc1), one pass over the caller's counts
    uint32_t* d_m = nullptr;
    uint32_t hm[3] = {0, 0, 0};
    hipError_t e = hipMalloc((void**)&d_m, 3 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(d_m, 0, 3 * sizeof(uint32_t), CTX_STREAM(ctx));
    if (e == hipSuccess) {
      const unsigned grid = (unsigned)std::min<int64_t>(4096, (n + 1023) / 1024);
      hipLaunchKernelGGL(k_max_called, dim3(grid), dim3(256), 0, CTX_STREAM(ctx), d->counts, (unsigned long long)n, d_m);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(hm, d_m, sizeof(hm), hipMemcpyDeviceToHost, CTX_STREAM(ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(CTX_STREAM(ctx));
    hipFree(d_m);
    if (e != hipSuccess) {
      if (d->ann_owned) hipFree(d->ann);
      hipFree(d->d_chrom_off); delete d;
      return set_err(ctx, SFS2D_E_HIP, std::string("wrap_device: ") + hipGetErrorString(e));
    }
    d->max_nc1 = hm[0];
    d->max_nc2 = hm[1];
    d->low_nc = hm[2] != 0u;
  } else {
    d->max_nc1 = d->max_nc2 = 0;
    d->low_nc = false;
  }
  *out = d;
  return 0;
}

int sfs2d_data_synth_sims(sfs2d_ctx* ctx, const sfs2d_synth_params* sp, const uint16_t* win_snps,
                          const uint32_t* miss_cdf1, int32_t nm1, const uint32_t* miss_cdf2, int32_t nm2,
                          sfs2d_data** out) {
  if (!ctx || !sp || !out || !miss_cdf1 || !miss_cdf2 || nm1 < 1 || nm2 < 1 ||
      (sp->n_replicates && sp->n_windows && !win_snps))
    return set_err(ctx, SFS2D_E_ARG, "null argument");
  if (sp->n1p < 1 || sp->n2p < 1 || 2 * sp->n1p > 255 || 2 * sp->n2p > 255 || sp->window_bp < 1 ||
      (unsigned long long)sp->n_windows * sp->window_bp > 0xffffffffull)
    return set_err(ctx, SFS2D_E_ARG, "bad synthetic parameters");
  *out = nullptr;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const uint64_t nw = (uint64_t)sp->n_replicates * sp->n_windows;
  std::vector<unsigned long long> woff(nw + 1, 0);
  std::vector<int64_t> coff(sp->n_replicates + 1, 0);
  for (uint64_t w = 0; w < nw; ++w) {
    if (win_snps[w] > sp->window_bp) return set_err(ctx, SFS2D_E_ARG, "more SNPs than bp in a window");
    woff[w + 1] = woff[w] + win_snps[w];
  }
  for (uint32_t r = 0; r < sp->n_replicates; ++r) coff[r + 1] = (int64_t)woff[(uint64_t)(r + 1) * sp->n_windows];
  const int64_t n = (int64_t)woff[nw];
  sfs2d_data* d = new sfs2d_data();
  d->ctx = ctx;
  d->owned = true;
  int rc = data_meta(ctx, d, coff.data(), (int32_t)sp->n_replicates, n);
  if (rc) { hipFree(d->d_chrom_off); delete d; return rc; }
  const size_t np = ((size_t)n + 3) / 4 * 4 + 64;   // readable to round_up(n, 4) (+ k_scan_w overhang)
  unsigned long long* d_woff = nullptr;
  uint32_t* d_mt = nullptr;
  if (dalloc(ctx, &d->counts, np) || dalloc(ctx, &d->pos, np) || dalloc(ctx, &d->ann, np) ||
      dalloc(ctx, &d_woff, nw + 1) || dalloc(ctx, &d_mt, (size_t)nm1 + nm2)) {
    hipFree(d->counts); hipFree(d->pos); hipFree(d->ann); hipFree(d_woff); hipFree(d->d_chrom_off); delete d;
    return SFS2D_E_NOMEM;
  }
  hipError_t e = hipMemsetAsync(d->ann, 0, sizeof(uint16_t) * np, CTX_STREAM(ctx));
  if (e == hipSuccess) e = hipMemsetAsync(d->counts, 0, sizeof(uint32_t) * np, CTX_STREAM(ctx));
  if (e == hipSuccess) e = hipMemsetAsync(d->pos, 0, sizeof(uint32_t) * np, CTX_STREAM(ctx));
  if (e == hipSuccess) e = hipMemcpyAsync(d_woff, woff.data(), sizeof(unsigned long long) * (nw + 1), hipMemcpyHostToDevice, CTX_STREAM(ctx));
  if (e == hipSuccess) e = hipMemcpyAsync(d_mt, miss_cdf1, sizeof(uint32_t) * nm1, hipMemcpyHostToDevice, CTX_STREAM(ctx));
  if (e == hipSuccess) e = hipMemcpyAsync(d_mt + nm1, miss_cdf2, sizeof(uint32_t) * nm2, hipMemcpyHostToDevice, CTX_STREAM(ctx));
  if (e == hipSuccess && nw) {
    SynthP S;
    S.seed = sp->seed; S.gen = sp->generation; S.nwin = sp->n_windows; S.ws = sp->window_bp;
    S.n1 = 2u * (uint32_t)sp->n1p; S.n2 = 2u * (uint32_t)sp->n2p; S.nm1 = (uint32_t)nm1; S.nm2 = (uint32_t)nm2;
    const unsigned grid = (unsigned)std::min<uint64_t>(16384, (nw + 3) / 4);
    hipLaunchKernelGGL(k_synth_sims, dim3(grid), dim3(256), 0, CTX_STREAM(ctx), S, d_woff, (unsigned long long)nw,
                       d_mt, d_mt + nm1, d->counts, d->pos);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(CTX_STREAM(ctx));
  hipFree(d_mt);
  if (e != hipSuccess) {
    hipFree(d_woff);
    hipFree(d->counts); hipFree(d->pos); hipFree(d->ann); hipFree(d->d_chrom_off); delete d;
    return set_err(ctx, SFS2D_E_HIP, std::string("synthetic data: ") + hipGetErrorString(e));
  }
  d->d_win_off = d_woff;   // the window offsets stay: fixed-bp plans of window_bp read their slots from them
  d->win_bp = sp->window_bp;
  d->win_per_chrom = sp->n_windows;
  d->last_pos.assign(sp->n_replicates, sp->n_windows * sp->window_bp);   // upper bound: trailing slots stay empty
  d->strict = true;
  d->max_nc1 = 2u * (uint32_t)sp->n1p;   // k_synth_sims: ref + alt + missing = 2 pop_size
  d->max_nc2 = 2u * (uint32_t)sp->n2p;
  *out = d;
  return 0;
}

int sfs2d_data_read(const sfs2d_data* d, uint32_t* counts, uint32_t* pos, int64_t n) {
  if (!d || n != d->n) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = d->ctx;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  if (counts && n) HIPCHK(ctx, hipMemcpy(counts, d->counts, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost));
  if (pos && n) HIPCHK(ctx, hipMemcpy(pos, d->pos, sizeof(uint32_t) * (size_t)n, hipMemcpyDeviceToHost));
  return 0;
}

int sfs2d_data_free(sfs2d_data* d) {
  if (!d) return SFS2D_E_ARG;
  hipSetDevice(d->ctx->device);
  if (d->owned) { hipFree(d->counts); hipFree(d->pos); }
  if (d->owned || d->ann_owned) hipFree(d->ann);
  hipFree(d->d_chrom_off);
  hipFree(d->d_win_off);
  delete d;
  return 0;
}

static int make_kparams(sfs2d_ctx* ctx, const sfs2d_params* prm, int nchrom, KParams* K) {
  *K = KParams{};   // (every field defined: e.g. ntri stays 0 unless a plan takes k_scan_gw's triangle)
  if (!prm) return set_err(ctx, SFS2D_E_ARG, "params is NULL");
  if (prm->n1p < 1 || prm->n2p < 1 || 2 * prm->n1p > 255 || 2 * prm->n2p > 255)
    return set_err(ctx, SFS2D_E_ARG, "pop sizes must satisfy 1 <= pop_size and 2*pop_size <= 255 (u8 counts)");
  if (prm->window_mode != SFS2D_WINDOW_BP && prm->window_mode != SFS2D_WINDOW_SNPS)
    return set_err(ctx, SFS2D_E_ARG, "bad window_mode");
  if (prm->window < 1 || prm->window > 0xffffffffll) return set_err(ctx, SFS2D_E_ARG, "window must be in [1, 2^32)");
  if (prm->bg_mode != SFS2D_BG_PER_CHROM && prm->bg_mode != SFS2D_BG_SUPPLIED) return set_err(ctx, SFS2D_E_ARG, "bad bg_mode");
  K->n1p = prm->n1p; K->n2p = prm->n2p; K->n1 = 2 * prm->n1p; K->n2 = 2 * prm->n2p;
  K->nb2 = (K->n1 + 1) * (K->n2 + 1);
  K->h1a = K->nb2; K->h1b = K->nb2 + K->n1 + 1; K->nh = (K->h1b + K->n2 + 1 + 3) & ~3;   // 16-B rows
  K->t1a = K->nb2; K->t1b = K->nb2 + K->n1p + 1; K->nt = K->t1b + K->n2p + 1;
  K->rtn = wl_rtn(K->n1p, K->n2p);   // (plans: widened to the data's largest called count)
  K->fold = prm->fold ? 1 : 0;
  K->fold_thr = prm->fold ? K->n1p + K->n2p : 0x7fffffff;
  K->ann_want = prm->ann_want;
  K->has_start = prm->has_start ? 1 : 0; K->has_end = prm->has_end ? 1 : 0;
  K->start_pos = prm->start_pos; K->end_pos = prm->end_pos;
  K->ws = (unsigned)prm->window;
  div_magic(K->ws, &K->wmag, &K->wsh1, &K->wsh2);
  K->nchrom = nchrom;
  K->fst_e = 40;   // plan_create narrows this to the plan's windows
  K->fst_scale = std::ldexp(1.0, K->fst_e);
  return 0;
}

static int plan_create(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int force_sliced,
                       sfs2d_plan** out);

int sfs2d_plan_create(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, sfs2d_plan** out) {
  return plan_create(ctx, data, prm, -1, out);
}

// force_sliced: -1 choose (windows per wave), 0 fused, 1 sliced (attached plans follow their base)
static int plan_create(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int force_sliced,
                       sfs2d_plan** out) {
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
  pl->slot_base_h = slot_base;
  // counts plan: no filter (the scan kernels classify counts without positions / annotations)
  pl->cnt = prm->ann_want < 0 && !prm->has_start && !prm->has_end;
  // a supplied background: no k_prep pass reads (and validates) the counts of a counts plan, so one is
  // taken only when no SNP can raise an error (max_nc1 / max_nc2); else the bins pipeline's k_prep
  // classifies every SNP and reports KeyError / out-of-grid keys as the reference raises them
  if (pl->cnt && prm->bg_mode != SFS2D_BG_PER_CHROM &&
      !(data->max_nc1 <= (uint32_t)K.n1 && data->max_nc2 <= (uint32_t)K.n2))
    pl->cnt = false;
  // generated replicates (sfs2d_data_synth_sims) scanned with the generator's window length: slot s of
  // replicate c is the generator's window c * win_per_chrom + w, whose SNPs it placed in that window
  // ((pos - 1) / ws == w), so the slot table is the window offsets (k_slots_synth) -- when every
  // replicate holds SNPs (the slot numbering skips empty chromosomes) and the plan has no other k_prep
  // work (a counts plan with a supplied background; see slots_only).
  // Any other fixed-bp counts plan with a supplied background (no k_prep histograms) takes its slots by
  // binary search on the resident positions (k_slots_search) instead of k_prep's segmentation pass.
  // SFS2D_SEG=prep forces k_prep's segmentation, SFS2D_SEG=search the search (never the generator's
  // offsets: what a real replicate VCF gets); both are selected by tests/test_synth_device.py
  const char* seg_ev = std::getenv("SFS2D_SEG");
  const bool seg_prep = seg_ev && std::strcmp(seg_ev, "prep") == 0, seg_srch = seg_ev && std::strcmp(seg_ev, "search") == 0;
  if (bp && data->d_win_off && (uint32_t)prm->window == data->win_bp && pl->cnt && !pl->do_bg &&
      pl->nslots == (int64_t)nc * (int64_t)data->win_per_chrom) {
    bool all = true;
    for (int c = 0; c < nc && all; ++c) all = data->chrom_off[c + 1] > data->chrom_off[c];
    pl->seg_synth = all && !seg_prep && !seg_srch;
  }
  // (Not with per-chromosome backgrounds, whose k_prep runs anyway: there a search before a counts-only
  // k_prep cost more than the positions it saved k_prep -- config 3: k_prep 83.5 -> 64.5 us but one pass
  // 0.214 -> 0.225 ms, the overlapped step 0.184 -> 0.191 ms, config 2 2.4e8 -> 2.0e8 windows/s; as extra
  // blocks of k_prep itself, concurrent with its tiles: 0.185 -> 0.193 ms; profiles/r06e_*, r06f_*.)
  pl->seg_search = bp && pl->cnt && !pl->do_bg && !pl->seg_synth && !seg_prep;
  pl->K.nm1 = data->n > 0 ? (uint32_t)(data->n - 1) : 0u;
  pl->K.kmul = (uint32_t)(pl->K.n2 + 1) | (1u << 16);
  pl->K.n12 = (uint32_t)pl->K.n1 | ((uint32_t)pl->K.n2 << 16);
  pl->K.lim12 = (uint32_t)(pl->K.n1p - 1) | ((uint32_t)(pl->K.n2p - 1) << 16);
  {   // Fst's reciprocals in LDS cover the data's largest called count: the reference counts SNPs whose
      // r + a exceeds 2 pop_size as long as the key stays in the grid (u8 counts: n <= 510)
    const uint32_t mx = std::min<uint32_t>(510u, std::max(data->max_nc1, data->max_nc2));
    pl->K.rtn = std::max(wl_rtn(K.n1p, K.n2p), (int)((mx + 2u) & ~1u));
  }
  if (pl->nslots > 0x7fffffffll) { delete pl; return set_err(ctx, SFS2D_E_ARG, "too many window slots (window too small)"); }
  pl->extra_rec = ((prm->flags & SFS2D_F_PREV_EXTRA) && bp && any) ? pl->nslots : -1;
  pl->nrec = pl->nslots + (pl->extra_rec >= 0 ? 1 : 0);

  // LDS strategy: a wavefront per window with u16-packed 2D bins for small grids, a workgroup per
  // window for large ones; u16 bins need < 65536 SNPs of one window in one bin.
  // (maxsnp: the most SNPs any window can hold, bounding the Fst fixed-point sums)
  int64_t maxc = 0;
  for (int c = 0; c < nc; ++c) maxc = std::max<int64_t>(maxc, data->chrom_off[c + 1] - data->chrom_off[c]);
  int64_t maxsnp = maxc;
  if (!bp || data->strict) maxsnp = std::min<int64_t>(maxc, prm->window);
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
    maxsnp = std::min(maxsnp, longest);
  } else {
    p16_ok = false;
  }
  pl->p16 = p16_ok;
  {
    // Fst fixed point 2^e: maxsnp terms of |x| <= 1 stay below 2^62 (e = 46 for 20 kb windows)
    int b = 0;
    while (b < 62 && (int64_t(1) << b) <= maxsnp) ++b;   // bit length of maxsnp
    pl->K.fst_e = std::max(8, std::min(FST_E_MAX, 61 - b));
    pl->K.fst_scale = std::ldexp(1.0, pl->K.fst_e);
  }
  pl->G = (K.nb2 <= 8192) ? 64 : 256;
  {
    const int core = (pl->p16 ? (K.nb2 + 1) / 2 : K.nb2) + (K.n1p + 1) + (K.n2p + 1);
    pl->extra_lds = (size_t)core * 4;
    if (pl->G == WAVE) {
      // k_scan_w: lp table (even-rounded) + D + F tables (+ Fst's reciprocals when Fst is asked for: the
      // scan may sum it), then 8 per-wave histogram blocks (also the fused prologue's scratch: u1 words,
      // 1D proportions, leaf accumulators and sums)
      const int h2w = pl->p16 ? (((K.nb2 + 1) / 2 + 3) & ~3) : ((K.nb2 + 3) & ~3);
      const int per = (h2w + R1 * (K.n1p + 1) + R1 * (K.n2p + 1) + 3) & ~3;   // (no trash words: scan_w_small)
      const size_t hist_words = std::max<size_t>((size_t)(SBLOCK / WAVE) * per, (size_t)FUSED_VCNT + K.nt + 16);
      const size_t rt = (prm->flags & SFS2D_F_FST) ? 2 * (size_t)pl->K.rtn : 0;
      pl->scan_lds = sizeof(double) * (size_t)(((K.nt + 1) & ~1) + LNT + LNF + rt) + hist_words * 4;
      // with the static LDS of the variant that uses most (the batched finish's per-wave arrays, Fst);
      // grids whose workgroup does not fit the 160 KB (e.g. 81 x 81) take the large-grid kernels
      hipFuncAttributes fa{};
      const size_t stat = hipFuncGetAttributes(&fa, (const void*)k_scan_w<true, true, true, true>) == hipSuccess
                              ? fa.sharedSizeBytes : 4096;
      if (pl->scan_lds + stat > 160 * 1024) pl->G = 256;
    }
    if (pl->G != WAVE) {
      pl->scan_lds = (size_t)(core + TRASH + 2) * 4 + 32 * 8 + 32 * 8;
      // k_scan_gw (a wavefront per window, tables from L2) when its one-wave workgroups, whose LDS
      // holds only the wave's histograms, still leave >= 2 wavefronts per CU (101 x 101: 7);
      // otherwise k_scan_g (a workgroup per window).  SFS2D_GW=0/1 forces one.
      // u8-packed 2D bins; counts plans with folded square grids keep only the reachable triangle
      // (k_scan_gw TRI: x1 + x2 <= n; 101 x 101: 5,151 of 10,201 bins -- half the LDS per wave).
      // x1 + x2 <= n holds only when every SNP's called counts r + a are <= 2 pop_size (then a folded
      // key has r1 + r2 <= 2n - (a1 + a2) < n); the reference counts any in-grid key
      // (twoDSFS_class.py:198-217), so data with a larger called count (max_nc1 / max_nc2, known at
      // upload) keep the full k2-indexed grid
      if (pl->cnt && prm->fold && K.n1 == K.n2 && data->max_nc1 <= (uint32_t)K.n1 && data->max_nc2 <= (uint32_t)K.n2)
        K.ntri = pl->K.ntri = (K.n1 + 1) * (K.n1 + 2) / 2;
      const int h2w = (((K.ntri ? K.ntri : K.nb2) + 3) / 4 + 3) & ~3;
      size_t gw_lds = (size_t)(h2w + R1GW * (K.n1p + 1) + R1GW * (K.n2p + 1) + TRASH) * 4;
      int occ = 0;
      if (gw_lds <= 160 * 1024) {
        const hipFuncAttribute A = hipFuncAttributeMaxDynamicSharedMemorySize;
        if (gw_lds > 64 * 1024)
          for (const void* f : {(const void*)k_scan_gw<true, false, false>, (const void*)k_scan_gw<false, false, false>,
                                (const void*)k_scan_gw<true, true, false>, (const void*)k_scan_gw<false, true, false>,
                                (const void*)k_scan_gw<true, false, true>, (const void*)k_scan_gw<false, false, true>,
                                (const void*)k_scan_gw<true, true, true>, (const void*)k_scan_gw<false, true, true>,
                                (const void*)k_scan_gw<true, false, true, true>, (const void*)k_scan_gw<false, false, true, true>,
                                (const void*)k_scan_gw<true, true, true, true>, (const void*)k_scan_gw<false, true, true, true>})
            hipFuncSetAttribute(f, A, (int)gw_lds);
        const hipError_t oe =
            K.ntri ? (pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<true, true, true, true>, WAVE, gw_lds)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<false, true, true, true>, WAVE, gw_lds))
                   : (pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<true, true, true>, WAVE, gw_lds)
                              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<false, true, true>, WAVE, gw_lds));
        if (oe != hipSuccess) occ = 0;
        // the LDS ln table (KParams::lnl) when it costs no workgroup per CU (config 4's 101 x 101 triangle:
        // 16 one-wave workgroups either way; config 5's 201 x 151 grid would lose one)
        {
          const size_t lds2 = gw_lds + 8 + (size_t)LNL * 8;
          int occ2 = 0;
          const bool big = lds2 > 64 * 1024 && lds2 <= 160 * 1024;
          if (big)
            for (const void* f : {(const void*)k_scan_gw<true, false, false>, (const void*)k_scan_gw<false, false, false>,
                                  (const void*)k_scan_gw<true, true, false>, (const void*)k_scan_gw<false, true, false>,
                                  (const void*)k_scan_gw<true, false, true>, (const void*)k_scan_gw<false, false, true>,
                                  (const void*)k_scan_gw<true, true, true>, (const void*)k_scan_gw<false, true, true>,
                                  (const void*)k_scan_gw<true, false, true, true>, (const void*)k_scan_gw<false, false, true, true>,
                                  (const void*)k_scan_gw<true, true, true, true>, (const void*)k_scan_gw<false, true, true, true>})
              hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds2);
          const hipError_t oe2 =
              lds2 > 160 * 1024 ? hipErrorInvalidValue
              : K.ntri ? (pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_scan_gw<true, true, true, true>, WAVE, lds2)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_scan_gw<false, true, true, true>, WAVE, lds2))
                       : (pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_scan_gw<true, true, true>, WAVE, lds2)
                                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_scan_gw<false, true, true>, WAVE, lds2));
          const char* lev = std::getenv("SFS2D_LNL");
          if (oe2 == hipSuccess && occ2 == occ && occ >= 2 && !(lev && lev[0] == '0')) {
            gw_lds = lds2;
            K.lnl = pl->K.lnl = 1;
          }
          (void)hipGetLastError();
        }
        pl->gw = occ >= 2;   // measured on 201 x 151 with u16 bins (2 per CU): 22 vs 32 us for k_scan_g
        if (const char* ev = std::getenv("SFS2D_GW")) pl->gw = occ >= 1 && ev[0] == '1';
      }
      if (pl->gw) pl->scan_lds = gw_lds;
    }
  }
  if (pl->scan_lds > 160 * 1024) {
    delete pl;
    return set_err(ctx, SFS2D_E_ARG, "2D grid too large for LDS with 32-bit bins (windows of >= 65536 SNPs)");
  }
  // per-chromosome backgrounds on the small-grid path: k_bg_slice (many workgroups per background)
  // then k_scan_w copies the table and combines the leaf sums in its prologue ("sliced"); the fused
  // alternative (every scan workgroup sums the replicas and builds the table itself) is kept for
  // comparison (SFS2D_FUSED=1): it is ~2x longer per workgroup
  // for the small-grid path.  Which wins depends on windows per wavefront: with about one window
  // each (1e6-SNP chromosome: 2.8k windows on 4k resident wavefronts) the table build IS the
  // kernel's critical path and the sliced path is ~5% faster per run; with tens of windows each
  // (config 3: 34) the fused prologue is amortised and its loop variant is faster.
  // SFS2D_FUSED=0/1 forces one.
  const bool small = pl->do_bg && pl->G == WAVE;
  const double wpw = (double)pl->nslots / (2.0 * ctx->ncu * (SBLOCK / WAVE));   // windows per resident wave
  pl->sliced = small && wpw < 4.0;
  if (const char* ev = std::getenv("SFS2D_FUSED")) pl->sliced = small && ev[0] == '0';
  if (force_sliced >= 0) pl->sliced = small && force_sliced == 1;
  pl->fused = small && !pl->sliced;
  // Fst of sliced fixed-bp plans: by extra k_bg_slice workgroups (the GPU is mostly idle during
  // that latency-bound kernel) instead of k_prep's per-SNP sums (config 2: k_prep -3 us)
  pl->fst = (prm->flags & SFS2D_F_FST) != 0;
  // Fst of counts plans on the small-grid path is summed by k_scan_w over the rows it streams
  // (fst_scan): k_prep then has no Fst work and stays bandwidth-bound (config 3: 147 -> 83 us) while
  // the scan, bound by its LDS pipe and VALU issue, grows (143 -> 210 us; an LDS copy of the
  // reciprocal table: 262 us).  One pass alone is ~2% slower than with k_prep's sums, but passes
  // overlapped on streams gain (config 2, 3 streams: 14.0 -> 12.8 us per pass; config 3, 2 streams
  // capped at 1 scan workgroup per CU: 293 -> 281 us), and an attached plan can then have Fst on any
  // window (profiles/r03k_fst_scan.txt).  SFS2D_FST_SCAN=0: k_prep's fixed-point sums / k_bg_slice's
  // Fst workgroups instead (attached Fst then needs fixed-bp windows the base's divide)
  pl->fst_scan = false;
  if (pl->fst && pl->cnt && pl->G == WAVE && !pl->gw) {
    const char* ev = std::getenv("SFS2D_FST_SCAN");
    pl->fst_scan = !(ev && ev[0] == '0');
    if (pl->fst_scan) {   // its variant's static LDS must fit beside the dynamic
      hipFuncAttributes fa{};
      const void* f = pl->p16 ? (const void*)k_scan_w<true, true, 2, true> : (const void*)k_scan_w<false, true, 2, true>;
      if (hipFuncGetAttributes(&fa, f) != hipSuccess || pl->scan_lds + fa.sharedSizeBytes > 160 * 1024) pl->fst_scan = false;
    }
  }
  const PwTree pw = pw_plan(K.nb2 - 3);
  pl->fst_mask = data->low_nc;
  pl->fst_win = pl->sliced && bp && pl->fst && !pl->fst_scan;
  pl->nfst = pl->fst_win ? (int)std::min<int64_t>(1024, std::max<int64_t>(1, (pl->nslots + 7) / 8)) : 0;   // ~1 window per wave
  if (pl->scan_lds > 64 * 1024) {
    const int lds = (int)pl->scan_lds;
    const hipFuncAttribute A = hipFuncAttributeMaxDynamicSharedMemorySize;
    for (const void* f : {(const void*)k_scan_w<true, true, false, false>, (const void*)k_scan_w<false, true, false, false>,
                          (const void*)k_scan_w<true, false, false, false>, (const void*)k_scan_w<false, false, false, false>,
                          (const void*)k_scan_w<true, true, true, false>, (const void*)k_scan_w<false, true, true, false>,
                          (const void*)k_scan_w<true, false, true, false>, (const void*)k_scan_w<false, false, true, false>,
                          (const void*)k_scan_w<true, true, false, true>, (const void*)k_scan_w<false, true, false, true>,
                          (const void*)k_scan_w<true, false, false, true>, (const void*)k_scan_w<false, false, false, true>,
                          (const void*)k_scan_w<true, true, true, true>, (const void*)k_scan_w<false, true, true, true>,
                          (const void*)k_scan_w<true, false, true, true>, (const void*)k_scan_w<false, false, true, true>,
                          (const void*)k_scan_w<true, true, 2, true>, (const void*)k_scan_w<false, true, 2, true>,
                          (const void*)k_scan_w<true, false, 2, true>, (const void*)k_scan_w<false, false, 2, true>,
                          (const void*)k_scan_w<true, true, 3, true>, (const void*)k_scan_w<false, true, 3, true>,
                          (const void*)k_scan_w<true, false, 3, true>, (const void*)k_scan_w<false, false, 3, true>,
                          (const void*)k_scan_g<true, false, false>, (const void*)k_scan_g<false, false, false>,
                          (const void*)k_scan_g<true, true, false>, (const void*)k_scan_g<false, true, false>,
                          (const void*)k_scan_g<true, false, true>, (const void*)k_scan_g<false, false, true>,
                          (const void*)k_scan_g<true, true, true>, (const void*)k_scan_g<false, true, true>})
      hipFuncSetAttribute(f, A, lds);
  }
  if (pl->extra_lds > 64 * 1024) {
    for (const void* f : {(const void*)k_scan_extra<true, false>, (const void*)k_scan_extra<false, false>,
                          (const void*)k_scan_extra<true, true>, (const void*)k_scan_extra<false, true>})
      hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl->extra_lds);
  }

  // scan work items.  k_scan_w: about one workgroup per resident slot (one dispatch wave, no
  // tail), shared among the chromosomes by window count; each wavefront takes one static window,
  // then windows from its chromosome's pool counters until they run dry (windows cost up to ~3x
  // each other, so static chunks left the slowest workgroups 2x behind the median).
  // k_scan_g: two windows per workgroup.
  if (pl->G == WAVE || pl->gw) {
    int occ = 0;
    // (the grid is one dispatch wave of resident workgroups: occupancy of the variant that runs)
    hipError_t oe;
    if (pl->gw && K.ntri)
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<true, true, true, true>, WAVE, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<false, true, true, true>, WAVE, pl->scan_lds);
    else if (pl->gw)
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<true, true, true>, WAVE, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_gw<false, true, true>, WAVE, pl->scan_lds);
    else if (pl->fst_scan && pl->fused)
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<true, true, 2, true>, SBLOCK, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<false, true, 2, true>, SBLOCK, pl->scan_lds);
    else if (pl->fst_scan)
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<true, false, 2, true>, SBLOCK, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<false, false, 2, true>, SBLOCK, pl->scan_lds);
    else if (pl->fused)
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<true, true, true, true>, SBLOCK, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<false, true, true, true>, SBLOCK, pl->scan_lds);
    else
      oe = pl->p16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<true, false, true, true>, SBLOCK, pl->scan_lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_scan_w<false, false, true, true>, SBLOCK, pl->scan_lds);
    if (oe != hipSuccess || occ < 1) occ = 1;
    if (prm->scan_wgs_per_cu > 0 && (int)prm->scan_wgs_per_cu < occ) occ = (int)prm->scan_wgs_per_cu;
    int64_t cap = (int64_t)occ * ctx->ncu;
    if (pl->gw) pl->nscr = (int)cap;   // one exact-path histogram per resident wavefront
    if (const char* ev = std::getenv("SFS2D_WGS")) cap = std::max<int64_t>(1, std::atoll(ev));   // tuning
    const double S = (double)std::max<unsigned long long>(1, slot_base[nc] - slot_base[0]);
    const uint32_t NW = pl->gw ? 1u : (uint32_t)(SBLOCK / WAVE);   // wavefronts per workgroup
    int64_t gw_win = 64;   // k_scan_gw: windows per workgroup of a small chromosome
    if (const char* ev = std::getenv("SFS2D_GWWIN")) gw_win = std::max<int64_t>(1, std::atoll(ev));   // tuning
    std::vector<double> order;
    for (int c = 0; c < nc; ++c) {
      const uint32_t ns = (uint32_t)(slot_base[c + 1] - slot_base[c]);
      if (!ns) continue;
      const uint32_t wmax = (ns + NW - 1) / NW;
      int64_t want = std::llround(cap * (ns / S));
      // k_scan_gw has no table prologue: many small chromosomes (sims batches: thousands of
      // replicates) get ~64 windows per workgroup instead of one workgroup each, which would leave
      // the last dispatch wave's workgroups running alone
      if (pl->gw) want = std::max<int64_t>(want, (ns + gw_win - 1) / gw_win);
      const uint32_t nwg = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(wmax, want));
      uint32_t npool = std::min<uint32_t>(nwg, CTR_POOLS);
      if (const char* ev = std::getenv("SFS2D_POOLS")) npool = std::max(1u, std::min<uint32_t>(npool, (uint32_t)std::atoi(ev)));   // tuning
      for (uint32_t k = 0; k < nwg; ++k) {
        Chunk ch{};
        ch.chrom = (uint32_t)c; ch.slot_lo = (uint32_t)slot_base[c]; ch.slot_hi = (uint32_t)slot_base[c + 1];
        ch.wid_lo = 0; ch.cb = (uint32_t)data->chrom_off[c];
        ch.first = k * NW; ch.nstatic = nwg * NW; ch.pool = npool | ((k % npool) << 16);
        pl->chunks.push_back(ch);
        order.push_back((k + 0.5) / nwg);
      }
    }
    // spread every chromosome's workgroups evenly over the grid: the first ~ncu workgroups are the
    // older of the two on their CU (issue priority), so a chromosome made only of younger ones
    // finished ~25% later than one of older ones; mixed, each pool drains at the common rate
    std::vector<size_t> idx(pl->chunks.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return order[a] < order[b]; });
    std::vector<Chunk> sorted(idx.size());
    for (size_t i = 0; i < idx.size(); ++i) sorted[i] = pl->chunks[idx[i]];
    pl->chunks.swap(sorted);
  } else {
    constexpr uint32_t CH = 2;
    for (int c = 0; c < nc; ++c)
      for (unsigned long long s = slot_base[c]; s < slot_base[c + 1]; s += CH) {
        Chunk ch{};
        ch.chrom = (uint32_t)c; ch.slot_lo = (uint32_t)s;
        ch.slot_hi = (uint32_t)std::min<unsigned long long>(s + CH, slot_base[c + 1]);
        ch.wid_lo = (uint32_t)(s - slot_base[c]);
        ch.cb = (uint32_t)data->chrom_off[c];
        ch.nstatic = ch.slot_hi - ch.slot_lo; ch.pool = 1;
        pl->chunks.push_back(ch);
      }
  }
  pl->last_chrom = last_c;

  // k_prep tiles (never crossing a chromosome); k_prep always runs (it writes the per-SNP bins)
  int64_t tileT = 0;
  {
    const int64_t n = data->n;
    // ~1000+ tiles for big inputs (several workgroups per CU), >= 4096 SNPs each (flush amortised)
    // (with k_prep's Fst sums, <= 32k SNPs per tile keep a tile's windows in its LDS sums down to
    // ~128-SNP windows; every tile flushes its LDS histogram, so no smaller tiles than that otherwise)
    const bool kfst_t = (prm->flags & SFS2D_F_FST) && !pl->fst_win && !pl->fst_scan;
    const int64_t Tmax = kfst_t ? 32768 : 65536;
    int64_t T = std::max<int64_t>(4096, std::min<int64_t>(Tmax, (n / 768 + 4095) / 4096 * 4096));
    if (const char* ev = std::getenv("SFS2D_TILE")) T = std::max<int64_t>(2048, std::atoll(ev) & ~int64_t(3));   // tuning
    tileT = T;
    // tile edges on absolute multiples of 4 SNPs (T is): only a chromosome's first and last step
    // take k_prep's masked edge path, every interior step of every tile the fast one
    for (int c = 0; c < nc; ++c)
      for (int64_t s = data->chrom_off[c]; s < data->chrom_off[c + 1];) {
        const int64_t e = std::min<int64_t>((s & ~int64_t(3)) + T, data->chrom_off[c + 1]);
        Tile t{};
        t.chrom = (uint32_t)c; t.begin = (uint32_t)s;
        t.end = (uint32_t)e;
        s = e;
        t.cb = (uint32_t)data->chrom_off[c]; t.ce = (uint32_t)data->chrom_off[c + 1];
        t.sbase = (uint32_t)slot_base[c];
        t.nslots = (uint32_t)(slot_base[c + 1] - slot_base[c]);
        pl->tiles.push_back(t);
      }
  }
  // one LDS copy per histogram word: four interleaved copies (lane & 3, fewer same-address atomics)
  // cost more in zeroing and flushing than they saved (k_prep config 2 10.3 vs 10.9 us, config 3
  // 183 vs 187 us)
  pl->hr = 1;
  pl->bg_lds = ((size_t)K.nh * pl->hr + WAVE) * 4;   // + 64 lane trash words
  {
    // the LDS histogram must fit beside the static LDS of the k_prep variant that will run: the Fst
    // variant (Fst not taken from k_bg_slice) holds ~20 KB of window sums and reciprocals, so e.g.
    // pop_size 95 / 95 (148 KB of histogram) takes the global-atomic histogram with Fst
    const bool kfst = (prm->flags & SFS2D_F_FST) && !pl->fst_win && !pl->fst_scan;
    hipFuncAttributes fa{};
    const hipError_t ae = kfst ? hipFuncGetAttributes(&fa, (const void*)k_prep<true, true, true, true, false, true>)
                               : hipFuncGetAttributes(&fa, (const void*)k_prep<true, true, true, true, false, false>);
    const size_t stat = ae == hipSuccess ? fa.sharedSizeBytes : (kfst ? 24 * 1024 : 1024);
    pl->lds_hist = pl->bg_lds + stat <= 160 * 1024;
    // k_prep's joint (alt1, alt2) histogram (prep_tile, JNT): counts plans whose k_prep only histograms
    // and segments, with tiles of >= 16k SNPs (its margins pass at the tile's end cost config 2's 4k-SNP
    // tiles more than the atomics saved: 2.25e8 vs 2.32-2.46e8 windows/s, profiles/r06i_prep_joint_hist.txt),
    // while the LDS stays <= 64 KB (nb2 words more).  SFS2D_JNT=0: three atomics per SNP; =1: the joint
    // histogram whatever the tile size (tests)
    const char* jev = std::getenv("SFS2D_JNT");
    const size_t jl = pl->bg_lds + (size_t)K.nb2 * 4;
    const bool jwant = jev ? jev[0] == '1' : tileT >= 16384;
    if (pl->lds_hist && pl->cnt && !kfst && jl + stat <= 64 * 1024 && jwant) {
      pl->K.jnt = K.nb2;
      pl->bg_lds = jl;
    }
  }
  if (pl->lds_hist && pl->bg_lds > 64 * 1024) {
    const hipFuncAttribute A = hipFuncAttributeMaxDynamicSharedMemorySize;
    const int lds = (int)pl->bg_lds;
    hipError_t e = hipSuccess;
    auto set = [&](const void* f) { if (e == hipSuccess) e = hipFuncSetAttribute(f, A, lds); };
    set((const void*)k_prep<true, true, true, true, false, false>);
    set((const void*)k_prep<true, false, true, true, false, false>);
    set((const void*)k_prep<true, true, true, true, true, false>);
    set((const void*)k_prep<true, false, true, true, true, false>);
    set((const void*)k_prep<true, true, true, true, false, true>);
    set((const void*)k_prep<true, false, true, true, false, true>);
    set((const void*)k_prep<true, true, true, true, true, true>);
    set((const void*)k_prep<true, false, true, true, true, true>);
    set((const void*)k_prep<true, false, true, false, false, false>);   // (the histogram-only pass)
    set((const void*)k_prep<true, false, true, false, true, false>);
    set((const void*)k_prep<true, true, true, false, false, false>);    // (counts plans: no bins)
    set((const void*)k_prep<true, true, true, false, false, true>);
    set((const void*)k_prep<true, false, true, false, false, true>);
    if (e != hipSuccess) {   // the large dynamic LDS was refused: the global-atomic histogram instead
      (void)hipGetLastError();
      pl->lds_hist = false;
    }
  }
  hipFuncSetAttribute((const void*)k_bg_finalize, hipFuncAttributeMaxDynamicSharedMemorySize,
                      (int)(sizeof(double) * FIN_LDS_BINS));

  // numpy pairwise plan over the 2D inner bins except the last (p[:-1] of bins[1:-1]) and the
  // k_bg_slice bin ranges: LEAVES_PER_SLICE leaves each, the first from bin 0, the last to nb2
  pl->nleaves = (int)pw.leaves.size();
  pl->nnodes = (int)pw.nodes.size();
  pl->nlevels = pw.nlevels;
  if (pl->nleaves > PW_MAX_LEAVES) { delete pl; return set_err(ctx, SFS2D_E_ARG, "grid too large for the pairwise plan"); }
  const int lps = LEAVES_PER_SLICE;   // (1 / 2 / 4 leaves per slice measure the same, tools/lps_probe.sh)
  for (int j = 0; j < pl->nleaves; j += lps) {
    const int jl = std::min(pl->nleaves, j + lps);
    const int kb = j == 0 ? 0 : 1 + pw.leaves[j].x;
    const int ke = jl == pl->nleaves ? K.nb2 : 1 + pw.leaves[jl].x;
    pl->slices.push_back(make_int4(kb, ke, j, jl));
  }
  if (pl->slices.empty()) pl->slices.push_back(make_int4(0, K.nb2, 0, 0));

  hipStream_t st = CTX_STREAM(ctx);
  rc = 0;
  rc = rc ? rc : dalloc(ctx, &pl->d_tiles, pl->tiles.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_chunks, pl->chunks.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_slots, (size_t)pl->nslots + 1);
  const size_t nrepl = pl->do_bg ? (size_t)(pl->fused ? 2 : 1) * REPL * nc * K.nh : 1;
  rc = rc ? rc : dalloc(ctx, &pl->d_repl, nrepl);
  rc = rc ? rc : dalloc(ctx, &pl->d_bcount, (size_t)2 * std::max(1, nc));
  rc = rc ? rc : dalloc(ctx, &pl->d_done, (size_t)pl->nbg);
  const size_t nctr = (size_t)2 * std::max(1, nc) * CTR_POOLS * CTR_STRIDE;
  rc = rc ? rc : dalloc(ctx, &pl->d_ctr, nctr);
  const size_t ngscr = pl->gw ? (size_t)pl->nscr * (K.nb2 + 1) : 0;
  if (pl->gw) rc = rc ? rc : dalloc(ctx, &pl->d_gscr, ngscr);
  rc = rc ? rc : dalloc(ctx, &pl->d_bgval, (size_t)pl->nbg * K.nt);
  rc = rc ? rc : dalloc(ctx, &pl->d_tab, (size_t)pl->nbg * K.nt);
  rc = rc ? rc : dalloc(ctx, &pl->d_lp, (size_t)pl->nbg * K.nt);
  rc = rc ? rc : dalloc(ctx, &pl->d_head, (size_t)pl->nbg);
  rc = rc ? rc : dalloc(ctx, &pl->d_bg1d, (size_t)pl->nbg);
  rc = rc ? rc : dalloc(ctx, &pl->d_leafsum, (size_t)pl->nbg * std::max(1, pl->nleaves));
  rc = rc ? rc : dalloc(ctx, &pl->d_leaves, pw.leaves.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_nodes, pw.nodes.size());
  rc = rc ? rc : dalloc(ctx, &pl->d_slices, pl->slices.size());
  const size_t nbins = pl->cnt ? 4 : ((size_t)data->n + 3) / 4 * 4 + SCAN_PAD;   // k_scan_w's step loads overhang n
  rc = rc ? rc : dalloc(ctx, &pl->d_bins, nbins);
  rc = rc ? rc : dalloc(ctx, &pl->d_out, (size_t)pl->nrec);
  rc = rc ? rc : dalloc(ctx, &pl->d_err, 4);
  if (pl->fst) rc = rc ? rc : dalloc(ctx, &pl->d_fst, (size_t)pl->nslots + 1);
  pl->d_fst_own = pl->d_fst;
  if (pl->seg_search && !rc) {   // k_slots_search's slot bases per chromosome (u32: nslots < 2^31)
    std::vector<uint32_t> sb(pl->slot_base_h.begin(), pl->slot_base_h.end());
    rc = dalloc(ctx, &pl->d_slot_base, sb.size());
    if (!rc && hipMemcpy(pl->d_slot_base, sb.data(), sizeof(uint32_t) * sb.size(), hipMemcpyHostToDevice) != hipSuccess)
      rc = set_err(ctx, SFS2D_E_HIP, "slot bases upload");
  }
  if (pl->fst) rc = rc ? rc : dalloc(ctx, &pl->d_fsum, 2 * ((size_t)pl->nslots + 1));
  if (rc) { plan_free(pl); delete pl; return rc; }
  hipError_t e = hipSuccess;
#define PCPY(dst, v) if (e == hipSuccess && !(v).empty()) e = hipMemcpyAsync(dst, (v).data(), sizeof((v)[0]) * (v).size(), hipMemcpyHostToDevice, st)
  PCPY(pl->d_tiles, pl->tiles);
  PCPY(pl->d_chunks, pl->chunks);
  PCPY(pl->d_leaves, pw.leaves);
  PCPY(pl->d_nodes, pw.nodes);
  PCPY(pl->d_slices, pl->slices);
#undef PCPY
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_slots, 0, sizeof(uint2) * ((size_t)pl->nslots + 1), st);
  if (e == hipSuccess && pl->do_bg) e = hipMemsetAsync(pl->d_repl, 0, sizeof(uint32_t) * nrepl, st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_bcount, 0, sizeof(uint32_t) * 2 * std::max(1, nc), st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_done, 0, sizeof(uint32_t) * pl->nbg, st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_ctr, 0, sizeof(uint32_t) * nctr, st);
  if (e == hipSuccess && pl->gw) e = hipMemsetAsync(pl->d_gscr, 0, sizeof(uint32_t) * ngscr, st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_err, 0, 4 * sizeof(uint32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_bins, 0, sizeof(uint32_t) * nbins, st);
  if (e == hipSuccess && pl->fst) e = hipMemsetAsync(pl->d_fsum, 0, sizeof(unsigned long long) * 2 * ((size_t)pl->nslots + 1), st);
  if (e == hipSuccess) e = hipMemsetAsync(pl->d_out, 0, sizeof(sfs2d_window) * (size_t)pl->nrec, st);
  for (auto& ev : pl->ev) if (e == hipSuccess) e = hipEventCreate(&ev);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    plan_free(pl); delete pl;
    return set_err(ctx, SFS2D_E_HIP, std::string("plan setup: ") + hipGetErrorString(e));
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
  HIPCHK(ctx, hipMemcpyAsync(pl->d_bgval, v.data(), sizeof(double) * K.nt, hipMemcpyHostToDevice, CTX_STREAM(ctx)));
  HIPCHK(ctx, launch_finalize(pl, integer_values ? 1 : 0));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  pl->bg_ready = true;
  return 0;
}

int sfs2d_plan_run_phase(sfs2d_plan* pl, int phase, sfs2d_window* out_dev) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  if (pl->base) return set_err(ctx, SFS2D_E_ARG, "an attached plan runs with its base plan (sfs2d_plan_attach)");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // a sampled run split into phases 1 and 2 (sfs2d_plan_run_streams' staggered first run) keeps
  // its events from phase 1 to phase 2 (tpend)
  hipEvent_t* te = nullptr;
  if (phase == 2) {
    te = pl->tpend;
    pl->tpend = nullptr;
  } else if (pl->timing && (pl->tseen++ % pl->tevery) == 0 && pl->tcount < pl->tmax) {
    te = &pl->tev[(size_t)pl->tcount * 6];
  }
  if (!pl->do_bg && !pl->bg_ready && phase != 1)
    return set_err(ctx, SFS2D_E_ARG, "supplied-background plan run before sfs2d_plan_set_background");
  // sampled runs: each kernel carries its start / end events in its own dispatch packet; a kernel
  // this run does not launch gets both events recorded in the stream instead (duration ~0)
  for (int k = 0; k < 6; ++k) pl->kev[k] = (te && ((pl->tmask >> (k / 2)) & 1)) ? te[k] : nullptr;
  auto mark = [&](int k) -> int {
    if (te && ((pl->tmask >> (k / 2)) & 1)) {
      HIPCHK(ctx, hipEventRecord(te[k], CTX_STREAM(ctx)));
      HIPCHK(ctx, hipEventRecord(te[k + 1], CTX_STREAM(ctx)));
    }
    return 0;
  };
  int rc = 0;
  if (phase == 0 || phase == 1) {
    if (slots_only(pl)) {
      HIPCHK(ctx, launch_slots_only(pl));
      if (pl->nslots == 0 && (rc = mark(0))) return rc;
    } else {
      HIPCHK(ctx, launch_prep(pl, true));
      if (!prep_runs(pl) && (rc = mark(0))) return rc;
    }
  }
  if (phase == 0 || phase == 2) {
    if (pl->do_bg && !pl->fused) HIPCHK(ctx, launch_bg_slices(pl));
    else if ((rc = mark(2))) return rc;
    for (sfs2d_plan* a : pl->attached) HIPCHK(ctx, launch_attached(a));   // before the base clears its state
    sfs2d_window* out = out_dev ? out_dev : pl->d_out;
    if (pl->chunks.empty() && (rc = mark(4))) return rc;
    HIPCHK(ctx, launch_scan_any(pl, out));
    pl->last_out = out;
    pl->runs++;
  }
  for (auto& e : pl->kev) e = nullptr;
  if (te && phase == 1) pl->tpend = te;   // (counted when its phase 2 has run)
  else if (te) pl->tcount++;
  return 0;
}

int sfs2d_plan_grids(const sfs2d_plan* pl, int64_t* prep_threads, int64_t* scan_threads) {
  if (!pl) return SFS2D_E_ARG;
  if (prep_threads) *prep_threads = (int64_t)pl->tiles.size() * BLOCK1;
  if (scan_threads) *scan_threads = (int64_t)pl->chunks.size() * (pl->G == WAVE ? SBLOCK : pl->gw ? WAVE : BLOCK);
  return 0;
}

const char* sfs2d_plan_scan_kernel(const sfs2d_plan* pl) {
  if (!pl) return nullptr;
  if (pl->gw) return "k_scan_gw";
  return pl->G == WAVE ? "k_scan_w" : "k_scan_g";
}

int sfs2d_plan_set_timing(sfs2d_plan* pl, int max_runs) { return sfs2d_plan_set_timing_sampled(pl, max_runs, 1); }

int sfs2d_plan_set_timing_sampled(sfs2d_plan* pl, int max_runs, int every) {
  return sfs2d_plan_set_timing_kernels(pl, max_runs, every, 7);
}

int sfs2d_plan_set_timing_kernels(sfs2d_plan* pl, int max_runs, int every, int kernel_mask) {
  if (!pl || max_runs < 0 || every < 1 || (kernel_mask & ~7) || !kernel_mask) return SFS2D_E_ARG;
  pl->tevery = every;
  pl->tmask = kernel_mask;
  pl->tseen = 0;
  sfs2d_ctx* ctx = pl->ctx;
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  // the event ring only grows (turning timing off keeps it): re-arming a sampled loop then costs no
  // event creation -- hundreds of hipEventCreate calls right before a timed loop left the GPU idle for
  // milliseconds first
  if ((size_t)max_runs * 6 > pl->tev.size()) {
    for (auto& e : pl->tev) if (e) hipEventDestroy(e);
    pl->tev.assign((size_t)max_runs * 6, nullptr);
    for (auto& e : pl->tev) HIPCHK(ctx, hipEventCreate(&e));
  }
  pl->tmax = max_runs;
  pl->tcount = 0;
  pl->tpend = nullptr;
  pl->timing = max_runs > 0;
  return 0;
}

int sfs2d_plan_timing_read(sfs2d_plan* pl, int* nruns, double* ms_k1, double* ms_k2, double* ms_k3) {
  if (!pl || !nruns) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  double t[3] = {0, 0, 0};
  const int klast = (pl->tmask & 4) ? 2 : (pl->tmask & 2) ? 1 : 0;   // the run's last recorded event pair
  for (int r = 0; r < pl->tcount; ++r) {
    hipEvent_t* te = &pl->tev[(size_t)r * 6];
    HIPCHK(ctx, hipEventSynchronize(te[2 * klast + 1]));
    for (int k = 0; k < 3; ++k) {
      if (!((pl->tmask >> k) & 1)) continue;
      float ms = 0;
      HIPCHK(ctx, hipEventElapsedTime(&ms, te[2 * k], te[2 * k + 1]));
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

int sfs2d_plan_run_many(sfs2d_plan* pl, int nruns, sfs2d_window* out_dev) {
  if (!pl || nruns < 0) return SFS2D_E_ARG;
  for (int i = 0; i < nruns; ++i) {
    const int rc = sfs2d_plan_run_phase(pl, 0, out_dev);
    if (rc) return rc;
  }
  return 0;
}

int sfs2d_plan_run_streams(sfs2d_plan* const* plans, void* const* streams, sfs2d_window* const* outs, int nplans,
                           int nruns) {
  if (!plans || !streams || nplans < 1 || nruns < 0) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = plans[0] ? plans[0]->ctx : nullptr;
  if (!ctx) return SFS2D_E_ARG;
  for (int k = 0; k < nplans; ++k) {
    if (!plans[k] || plans[k]->ctx != ctx) return set_err(ctx, SFS2D_E_ARG, "plans must share one ctx");
    for (int j = 0; j < k; ++j)
      if (plans[j] == plans[k]) return set_err(ctx, SFS2D_E_ARG, "a plan may appear once (its per-run state is not shareable)");
  }
  // run i: plan i % nplans on stream i % nplans.  The plans' per-run state (bins, replicas, slots,
  // counters) is their own, so consecutive runs on different streams overlap.  (One host thread
  // enqueues: config 2 with 3 streams is not host-bound -- 10.7 us of enqueue per pass vs 14.5 us on
  // the GPU; a thread per stream gained 1.5% at 400 passes and lost its thread starts in 20-pass runs,
  // profiles/r02i_enqueue_probe.txt)
  // The streams start staggered: the second stream's first run waits for the first run's k_prep, so
  // that from the start one stream's bandwidth-bound k_prep runs beside the other's latency-bound scan
  // (started together, the two k_preps competed and then the two scans, and the streams kept that
  // phase: config 3's 20-step bench loop 0.184 vs 0.190-0.198 ms per pass, without Fst 0.165 vs 0.181;
  // profiles/r05u_stream_stagger_ab.txt).  Not for plans with attached plans: their longer passes
  // settled into a worse phase staggered (20 kb + 500 kb: 0.328-0.331 vs 0.285-0.286 ms per step).
  // Chaining every run's k_prep after the previous run's k_prep (and its scan after the previous scan)
  // measured slower: 0.1852-0.1857 (0.238-0.248) vs 0.1821-0.1828 ms (profiles/r06l_stream_chain_ab.txt).
  // About one 20-run loop in eight settles into a slower phase (0.19-0.216 ms per run, the scans of both
  // streams overlapping more); the k_prep chain never did in 8 runs but costs ~2% in the typical one, a
  // chained start made the slow phase likelier (5 of 8), the scan chain is far slower
  // (profiles/r06v_*, r06w_*, r06x_*)
  bool stagger = nplans >= 2 && nruns >= 2;
  for (int k = 0; k < nplans; ++k) stagger = stagger && plans[k]->attached.empty();
  if (stagger && !ctx->stagger) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->stagger, hipEventDisableTiming));
  hipStream_t saved = CTX_STREAM(ctx);
  int rc = 0;
  for (int i = 0; i < nruns && !rc; ++i) {
    const int k = i % nplans;
    ctx->stream = (hipStream_t)streams[k];   // (NULL: the null stream, as sfs2d_ctx_set_stream)
    if (stagger && i == 0) {
      rc = sfs2d_plan_run_phase(plans[k], 1, outs ? outs[k] : nullptr);
      if (!rc && hipEventRecord(ctx->stagger, ctx->stream) != hipSuccess) rc = set_err(ctx, SFS2D_E_HIP, "stagger event");
      if (!rc) rc = sfs2d_plan_run_phase(plans[k], 2, outs ? outs[k] : nullptr);
      continue;
    }
    if (stagger && i == 1 && hipStreamWaitEvent(ctx->stream, ctx->stagger, 0) != hipSuccess)
      rc = set_err(ctx, SFS2D_E_HIP, "stagger wait");
    if (!rc) rc = sfs2d_plan_run_phase(plans[k], 0, outs ? outs[k] : nullptr);
  }
  ctx->stream = saved;
  return rc;
}

// A run_streams sequence captured into HIP graphs, one per stream (each a chain of its plans' runs), and
// replayed with one hipGraphLaunch per stream: short passes (config 2's 1e6-SNP chromosome, ~12 us of
// GPU time per pass) are host-bound when each of their three launches is enqueued on its own.  One graph
// holding all the streams' chains as parallel branches (forked and joined through events) measured 6-9x
// slower than run_streams (0.066-0.107 vs 0.0117 ms per pass, profiles/r06ad_*): the replay does not
// overlap the branches the way independent streams do.  The runs' kernel arguments (parity-selected
// buffers, output pointers) are fixed at capture: every plan runs an even number of times per replay, so
// its buffer parity is the same before and after each replay, and a replay refuses to start when a plan
// ran an odd number of times since the capture.
struct sfs2d_graph {
  sfs2d_ctx* ctx = nullptr;
  std::vector<hipStream_t> streams;
  std::vector<hipGraph_t> graphs;
  std::vector<hipGraphExec_t> execs;
  std::vector<sfs2d_plan*> plans;
  std::vector<int64_t> par;
};

static void graph_free(sfs2d_graph* g) {
  for (auto& x : g->execs) if (x) hipGraphExecDestroy(x);
  for (auto& x : g->graphs) if (x) hipGraphDestroy(x);
  delete g;
}

int sfs2d_graph_create(sfs2d_plan* const* plans, void* const* streams, sfs2d_window* const* outs, int nplans,
                       int nruns, sfs2d_graph** out) {
  if (!plans || !streams || !out || nplans < 1 || nruns < 1) return SFS2D_E_ARG;
  *out = nullptr;
  sfs2d_ctx* ctx = plans[0] ? plans[0]->ctx : nullptr;
  if (!ctx) return SFS2D_E_ARG;
  if (nruns % (2 * nplans))
    return set_err(ctx, SFS2D_E_ARG, "a graph holds an even number of runs of every plan (nruns % (2 * nplans) == 0)");
  for (int k = 0; k < nplans; ++k) {
    if (!plans[k] || plans[k]->ctx != ctx) return set_err(ctx, SFS2D_E_ARG, "plans must share one ctx");
    for (int j = 0; j < k; ++j)
      if (plans[j] == plans[k]) return set_err(ctx, SFS2D_E_ARG, "a plan may appear once (its per-run state is not shareable)");
    if (plans[k]->timing) return set_err(ctx, SFS2D_E_ARG, "a plan with timing on cannot be captured");
    if (plans[k]->base) return set_err(ctx, SFS2D_E_ARG, "an attached plan runs with its base plan (sfs2d_plan_attach)");
    if (!streams[k]) return set_err(ctx, SFS2D_E_ARG, "graph capture needs non-null streams");
  }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  sfs2d_graph* g = new sfs2d_graph;
  g->ctx = ctx;
  for (int k = 0; k < nplans; ++k) {
    hipStream_t s = (hipStream_t)streams[k];
    if (std::find(g->streams.begin(), g->streams.end(), s) == g->streams.end()) g->streams.push_back(s);
  }
  hipStream_t saved = CTX_STREAM(ctx);
  int rc = 0;
  hipError_t e = hipSuccess;
  for (hipStream_t s : g->streams) {
    // run i of the sequence is plan i % nplans on its stream: this stream's chain, in sequence order
    e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) break;
    ctx->stream = s;
    for (int i = 0; i < nruns && !rc; ++i) {
      const int k = i % nplans;
      if ((hipStream_t)streams[k] == s) rc = sfs2d_plan_run_phase(plans[k], 0, outs ? outs[k] : nullptr);
    }
    hipGraph_t gr = nullptr;
    e = hipStreamEndCapture(s, &gr);
    g->graphs.push_back(gr);
    hipGraphExec_t x = nullptr;
    if (!rc && e == hipSuccess) e = hipGraphInstantiate(&x, gr, nullptr, nullptr, 0);
    g->execs.push_back(x);
    if (rc || e != hipSuccess) break;
  }
  ctx->stream = saved;
  if (rc || e != hipSuccess) {
    graph_free(g);
    return rc ? rc : set_err(ctx, SFS2D_E_HIP, std::string("graph capture: ") + hipGetErrorString(e));
  }
  for (int k = 0; k < nplans; ++k) {
    g->plans.push_back(plans[k]);
    g->par.push_back(plans[k]->runs & 1);
  }
  *out = g;
  return 0;
}

int sfs2d_graph_launch(sfs2d_graph* g, int nlaunch) {
  if (!g || nlaunch < 0) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = g->ctx;
  for (size_t k = 0; k < g->plans.size(); ++k)
    if ((g->plans[k]->runs & 1) != g->par[k])
      return set_err(ctx, SFS2D_E_ARG, "a captured plan ran an odd number of times since the capture");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  for (int i = 0; i < nlaunch; ++i)
    for (size_t j = 0; j < g->execs.size(); ++j) HIPCHK(ctx, hipGraphLaunch(g->execs[j], g->streams[j]));
  return 0;
}

int sfs2d_graph_destroy(sfs2d_graph* g) {
  if (!g) return SFS2D_E_ARG;
  hipSetDevice(g->ctx->device);
  for (hipStream_t s : g->streams) hipStreamSynchronize(s);   // (no replay in flight)
  graph_free(g);
  return 0;
}

int sfs2d_plan_bg_buffer(sfs2d_plan* pl, void** dev_ptr, int64_t* nbytes) {
  if (!pl || !dev_ptr || !nbytes) return SFS2D_E_ARG;
  // the replica buffer the next run's k_prep accumulates into (fused plans alternate two)
  *dev_ptr = pl->d_repl + (size_t)repl_par(pl) * REPL * pl->data->nchrom * pl->K.nh;
  *nbytes = pl->do_bg ? (int64_t)REPL * pl->data->nchrom * pl->K.nh * 4 : 0;
  return 0;
}

int sfs2d_plan_bg_words(const sfs2d_plan* pl, int64_t* replicas, int64_t* nchrom, int64_t* bins) {
  if (!pl || !replicas || !nchrom || !bins) return SFS2D_E_ARG;
  *replicas = pl->do_bg ? REPL : 0;
  *nchrom = pl->do_bg ? pl->data->nchrom : 0;
  *bins = pl->do_bg ? pl->K.nh : 0;
  return 0;
}

int sfs2d_plan_bg_exchange(sfs2d_plan* pl, uint32_t* host_repl, uint32_t* host_sums, int to_device) {
  if (!pl || !host_repl || !host_sums) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  if (!pl->do_bg) return set_err(ctx, SFS2D_E_ARG, "plan has no per-chromosome backgrounds");
  if (pl->base) return set_err(ctx, SFS2D_E_ARG, "exchange the base plan's backgrounds");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // this run's buffers: the replicas k_prep accumulated into and the per-chromosome inner 2D sums
  // (the parities of sfs2d_plan_run_phase(plan, 1) of the run in progress)
  uint32_t* r = pl->d_repl + (size_t)repl_par(pl) * REPL * pl->data->nchrom * pl->K.nh;
  uint32_t* b = pl->d_bcount + (size_t)plan_par(pl) * pl->K.nchrom;
  const size_t nr = (size_t)REPL * pl->data->nchrom * pl->K.nh * 4, nb = (size_t)pl->K.nchrom * 4;
  hipStream_t st = CTX_STREAM(ctx);
  if (to_device) {
    HIPCHK(ctx, hipMemcpyAsync(r, host_repl, nr, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemcpyAsync(b, host_sums, nb, hipMemcpyHostToDevice, st));
  } else {
    HIPCHK(ctx, hipMemcpyAsync(host_repl, r, nr, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipMemcpyAsync(host_sums, b, nb, hipMemcpyDeviceToHost, st));
  }
  HIPCHK(ctx, hipStreamSynchronize(st));
  return 0;
}

int sfs2d_plan_bg_rows_dev(sfs2d_plan* pl, int64_t* d_rows, int64_t row_stride) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  if (!pl->do_bg) return set_err(ctx, SFS2D_E_ARG, "plan has no per-chromosome backgrounds");
  if (pl->base) return set_err(ctx, SFS2D_E_ARG, "exchange the base plan's backgrounds");
  const int W = pl->K.h1b + pl->K.n2 + 2;
  if (!d_rows || row_stride < W) return set_err(ctx, SFS2D_E_ARG, "rows: null or stride < SFS2D_BG_ROW_WORDS");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int nc = pl->data->nchrom;
  if (nc == 0) return 0;
  const size_t rs = (size_t)nc * pl->K.nh;
  hipLaunchKernelGGL(k_bg_rows_get, dim3((unsigned)((W + 255) / 256), (unsigned)nc), dim3(256), 0, CTX_STREAM(ctx), pl->K,
                     pl->d_repl + (size_t)repl_par(pl) * REPL * rs, (unsigned long long)rs,
                     pl->d_bcount + (size_t)plan_par(pl) * pl->K.nchrom, (long long*)d_rows, (long long)row_stride);
  HIPCHK(ctx, hipGetLastError());
  return 0;
}

int sfs2d_plan_bg_rows_set_dev(sfs2d_plan* pl, const int64_t* d_rows, int64_t row_stride) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  if (!pl->do_bg) return set_err(ctx, SFS2D_E_ARG, "plan has no per-chromosome backgrounds");
  if (pl->base) return set_err(ctx, SFS2D_E_ARG, "exchange the base plan's backgrounds");
  const int W = pl->K.h1b + pl->K.n2 + 2;
  if (!d_rows || row_stride < W) return set_err(ctx, SFS2D_E_ARG, "rows: null or stride < SFS2D_BG_ROW_WORDS");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int nc = pl->data->nchrom;
  if (nc == 0) return 0;
  const size_t rs = (size_t)nc * pl->K.nh;
  const int nk = std::max(W, pl->K.nh);
  hipLaunchKernelGGL(k_bg_rows_set, dim3((unsigned)((nk + 255) / 256), (unsigned)nc), dim3(256), 0, CTX_STREAM(ctx), pl->K,
                     pl->d_repl + (size_t)repl_par(pl) * REPL * rs, (unsigned long long)rs,
                     pl->d_bcount + (size_t)plan_par(pl) * pl->K.nchrom, (const long long*)d_rows, (long long)row_stride,
                     pl->d_err);
  HIPCHK(ctx, hipGetLastError());
  return 0;
}

int sfs2d_plan_fst_buffer(sfs2d_plan* pl, void** dev_ptr, int64_t* nslots) {
  if (!pl || !dev_ptr || !nslots) return SFS2D_E_ARG;
  if (!pl->fst) return set_err(pl->ctx, SFS2D_E_ARG, "plan was created without SFS2D_F_FST");
  *dev_ptr = pl->d_fst;
  *nslots = pl->nslots;
  return 0;
}

int sfs2d_plan_set_fst_out(sfs2d_plan* pl, double* d_fst) {
  if (!pl) return SFS2D_E_ARG;
  if (!pl->fst) return set_err(pl->ctx, SFS2D_E_ARG, "plan was created without SFS2D_F_FST");
  if (pl->base) return set_err(pl->ctx, SFS2D_E_ARG, "an attached plan's Fst buffer is its own");
  pl->d_fst = d_fst ? d_fst : pl->d_fst_own;
  return 0;
}

int sfs2d_plan_fst_read(sfs2d_plan* pl, double* out_host, int64_t cap) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  if (!pl->fst) return set_err(ctx, SFS2D_E_ARG, "plan was created without SFS2D_F_FST");
  if (cap < pl->nslots) return set_err(ctx, SFS2D_E_CAP, "output capacity too small");
  if (pl->nslots && !out_host) return SFS2D_E_ARG;
  if (pl->nslots)
    HIPCHK(ctx, hipMemcpyAsync(out_host, pl->d_fst, sizeof(double) * pl->nslots, hipMemcpyDeviceToHost, CTX_STREAM(ctx)));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  return 0;
}

int sfs2d_plan_check(sfs2d_plan* pl) {
  if (!pl) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  uint32_t e = 0;
  HIPCHK(ctx, hipMemcpyAsync(&e, pl->d_err, 4, hipMemcpyDeviceToHost, CTX_STREAM(ctx)));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  if (e) {
    HIPCHK(ctx, hipMemsetAsync(pl->d_err, 0, 4, CTX_STREAM(ctx)));
    HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
    if (e & ERR_OVF) return set_err(ctx, SFS2D_E_ARG, "summed background histograms overflow uint32");
    if (e & ERR_KEY) return set_err(ctx, SFS2D_E_KEY, "allele count above 2*pop_size (reference: KeyError in calculate_1d_sfs)");
    return set_err(ctx, SFS2D_E_GRID, "folded 2D bin outside the (2n1+1)x(2n2+1) grid");
  }
  return 0;
}

// diagnostic: stamps of a -DSFS2D_STAMPS build (returns SFS2D_E_ARG in the shipped build)
int sfs2d__debug_stamps(unsigned long long* out64) {
#ifdef SFS2D_STAMPS
  // 64 phase stamps, then per-block (start, end) of k_prep and k_scan_w (2 x 4096 x 2), then per wave,
  // then k_bg_slice per block
  if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 64) != hipSuccess) return SFS2D_E_HIP;
  if (hipMemcpyFromSymbol(out64 + 64, HIP_SYMBOL(g_blk), sizeof(unsigned long long) * 2 * 4096 * 2) != hipSuccess)
    return SFS2D_E_HIP;
  // then k_scan_w per wavefront (end, windows): 4096 x 8 x 2
  if (hipMemcpyFromSymbol(out64 + 64 + 2 * 4096 * 2, HIP_SYMBOL(g_wv), sizeof(unsigned long long) * 4096 * 8 * 2) != hipSuccess)
    return SFS2D_E_HIP;
  // then k_bg_slice per block (start, work done): 1024 x 2
  if (hipMemcpyFromSymbol(out64 + 64 + 2 * 4096 * 2 + 4096 * 8 * 2, HIP_SYMBOL(g_bgs), sizeof(unsigned long long) * 1024 * 2) != hipSuccess)
    return SFS2D_E_HIP;
  return 0;
#else
  (void)out64;
  return SFS2D_E_ARG;
#endif
}

int sfs2d_plan_stats(sfs2d_plan* pl, uint32_t* exact_windows) {
  if (!pl || !exact_windows) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  HIPCHK(ctx, hipMemcpyAsync(exact_windows, pl->d_err + 1, 4, hipMemcpyDeviceToHost, CTX_STREAM(ctx)));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
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
    HIPCHK(ctx, hipMemcpyAsync(out_host, src, sizeof(sfs2d_window) * pl->nrec, hipMemcpyDeviceToHost, CTX_STREAM(ctx)));
  HIPCHK(ctx, hipStreamSynchronize(CTX_STREAM(ctx)));
  return 0;
}

int sfs2d_plan_time(sfs2d_plan* pl, int iters, double* ms_run, double* ms_k1, double* ms_k2, double* ms_k3) {
  if (!pl || iters < 1) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = pl->ctx;
  hipStream_t st = CTX_STREAM(ctx);
  double t1 = 0, t2 = 0, t3 = 0, tall = 0;
  for (int it = 0; it < iters; ++it) {
    HIPCHK(ctx, hipEventRecord(pl->ev[0], st));
    HIPCHK(ctx, slots_only(pl) ? launch_slots_only(pl) : launch_prep(pl, true));
    HIPCHK(ctx, hipEventRecord(pl->ev[1], st));
    if (pl->do_bg && !pl->fused) HIPCHK(ctx, launch_bg_slices(pl));
    for (sfs2d_plan* a : pl->attached) HIPCHK(ctx, launch_attached(a));
    HIPCHK(ctx, hipEventRecord(pl->ev[2], st));
    HIPCHK(ctx, launch_scan_any(pl, pl->d_out));
    pl->runs++;
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
  hipStreamSynchronize(CTX_STREAM(pl->ctx));
  for (sfs2d_plan* a : pl->attached) {   // attached plans go with their base
    a->base = pl;
    plan_free(a);
    delete a;
  }
  pl->attached.clear();
  if (pl->base) {
    auto& v = pl->base->attached;
    v.erase(std::remove(v.begin(), v.end(), pl), v.end());
  }
  plan_free(pl);
  delete pl;
  return 0;
}

int sfs2d_plan_attach(sfs2d_plan* base, const sfs2d_params* prm, sfs2d_plan** out) {
  if (!base || !prm || !out) return SFS2D_E_ARG;
  sfs2d_ctx* ctx = base->ctx;
  *out = nullptr;
  if (base->base) return set_err(ctx, SFS2D_E_ARG, "attach to a base plan, not to an attached one");
  const bool large = base->do_bg && base->G != WAVE;   // tables from the base's k_bg_slice (with its tail)
  if (!base->fused && !base->sliced && !large)
    return set_err(ctx, SFS2D_E_ARG, "attached plans need a per-chromosome-background base plan");
  const sfs2d_params& b = base->prm;
  if (prm->n1p != b.n1p || prm->n2p != b.n2p || (prm->fold != 0) != (b.fold != 0) || prm->bg_mode != b.bg_mode ||
      prm->ann_want != b.ann_want || prm->has_start != b.has_start || prm->has_end != b.has_end ||
      (prm->has_start && prm->start_pos != b.start_pos) || (prm->has_end && prm->end_pos != b.end_pos))
    return set_err(ctx, SFS2D_E_ARG, "an attached plan may differ from its base only in the window and flags");
  const bool bp = prm->window_mode == SFS2D_WINDOW_BP;
  sfs2d_plan* a = nullptr;
  int rc = plan_create(ctx, base->data, prm, base->sliced ? 1 : 0, &a);
  if (rc) return rc;
  if (a->fused != base->fused || a->sliced != base->sliced || a->G != base->G || a->cnt != base->cnt) {
    plan_free(a); delete a;
    return set_err(ctx, SFS2D_E_ARG, "attached plan would take a different kernel path than its base");
  }
  // Fst of an attached plan: its own scan's sums (fst_scan), else the base's k_prep sums added per
  // attached window (fused bases) or k_fst_win on the attached slots (sliced bases)
  uint32_t m = 0;
  if ((prm->flags & SFS2D_F_FST) && !a->fst_scan) {
    const bool base_bp = b.window_mode == SFS2D_WINDOW_BP;
    const char* why = nullptr;
    if (!bp) why = "attached Fst needs fixed-bp windows";
    else if (!base->sliced && (!(b.flags & SFS2D_F_FST) || base->fst_scan || !base_bp || prm->window % b.window != 0))
      why = "attached Fst needs a fixed-bp Fst base plan whose window divides this one's";
    if (why) { plan_free(a); delete a; return set_err(ctx, SFS2D_E_ARG, why); }
    if (!base->sliced) m = (uint32_t)(prm->window / b.window);
  }
  HIPCHK(ctx, hipSetDevice(ctx->device));
  hipFree(a->d_bins); hipFree(a->d_repl); hipFree(a->d_bcount);
  a->d_bins = base->d_bins;
  a->d_repl = base->d_repl;
  a->d_bcount = base->d_bcount;
  if (base->sliced) {   // the base's k_bg_slice tables (the attached scans combine the same leaf sums)
    hipFree(a->d_tab); hipFree(a->d_lp); hipFree(a->d_head); hipFree(a->d_leafsum); hipFree(a->d_bg1d);
    a->d_tab = base->d_tab;
    a->d_lp = base->d_lp;
    a->d_head = base->d_head;
    a->d_leafsum = base->d_leafsum;
    a->d_bg1d = base->d_bg1d;
  } else if (large) {   // the base's finished per-chromosome tables
    hipFree(a->d_tab); hipFree(a->d_lp); hipFree(a->d_head);
    a->d_tab = base->d_tab;
    a->d_lp = base->d_lp;
    a->d_head = base->d_head;
  }
  a->base = base;
  a->fst_m = m;
  a->fst_win = base->sliced && (prm->flags & SFS2D_F_FST) && !a->fst_scan;   // k_fst_win on the attached slots
  a->nfst = 0;
  rc = 0;
  std::vector<uint32_t> sb(a->slot_base_h.begin(), a->slot_base_h.end());
  rc = rc ? rc : dalloc(ctx, &a->d_slot_base, sb.size());
  if (m && !base->d_slot_base) {
    std::vector<uint32_t> bsb(base->slot_base_h.begin(), base->slot_base_h.end());
    rc = rc ? rc : dalloc(ctx, &base->d_slot_base, bsb.size());
    if (!rc && hipMemcpy(base->d_slot_base, bsb.data(), sizeof(uint32_t) * bsb.size(), hipMemcpyHostToDevice) != hipSuccess)
      rc = SFS2D_E_HIP;
  }
  if (!rc && hipMemcpy(a->d_slot_base, sb.data(), sizeof(uint32_t) * sb.size(), hipMemcpyHostToDevice) != hipSuccess)
    rc = SFS2D_E_HIP;
  if (rc) { plan_free(a); delete a; return rc == SFS2D_E_HIP ? set_err(ctx, rc, "attach: copy") : rc; }
  base->attached.push_back(a);
  *out = a;
  return 0;
}

static int bg_hist_impl(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int32_t chrom, int64_t* h2d,
                        int64_t* h1a, int64_t* h1b, int64_t* d_row);

int sfs2d_bg_hist(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int32_t chrom, int64_t* h2d,
                  int64_t* h1a, int64_t* h1b) {
  if (!ctx || !data || !prm || !h2d || !h1a || !h1b) return set_err(ctx, SFS2D_E_ARG, "null argument");
  return bg_hist_impl(ctx, data, prm, chrom, h2d, h1a, h1b, nullptr);
}

int sfs2d_bg_hist_dev(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int32_t chrom, int64_t* d_row) {
  if (!ctx || !data || !prm || !d_row) return set_err(ctx, SFS2D_E_ARG, "null argument");
  return bg_hist_impl(ctx, data, prm, chrom, nullptr, nullptr, nullptr, d_row);
}

// d_row: the histograms as one device row (k_bg_rows_get's layout) instead of host arrays
static int bg_hist_impl(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* prm, int32_t chrom, int64_t* h2d,
                        int64_t* h1a, int64_t* h1b, int64_t* d_row) {
  if (chrom < -1 || chrom >= data->nchrom) return set_err(ctx, SFS2D_E_ARG, "chrom out of range");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  KParams K;
  int rc = make_kparams(ctx, prm, data->nchrom, &K);
  if (rc) return rc;
  // one pseudo-chromosome: all tiles accumulate into background 0
  sfs2d_plan pl;
  pl.ctx = ctx; pl.data = data; pl.prm = *prm; pl.K = K; pl.K.nchrom = 1;
  pl.do_bg = true; pl.do_seg = false;
  pl.bg_lds = ((size_t)K.nh + WAVE) * 4;
  pl.lds_hist = pl.bg_lds <= 150 * 1024;
  const int c0 = chrom < 0 ? 0 : chrom, c1 = chrom < 0 ? data->nchrom : chrom + 1;
  const int64_t T = 16384;
  for (int c = c0; c < c1; ++c)
    for (int64_t s = data->chrom_off[c]; s < data->chrom_off[c + 1];) {   // (edges on multiples of 4, as plans)
      const int64_t e = std::min<int64_t>((s & ~int64_t(3)) + T, data->chrom_off[c + 1]);
      Tile t{};
      t.chrom = 0; t.begin = (uint32_t)s; t.end = (uint32_t)e;
      t.cb = (uint32_t)data->chrom_off[c]; t.ce = (uint32_t)data->chrom_off[c + 1];
      pl.tiles.push_back(t);
      s = e;
    }
  // chrom_off for pseudo-chromosome 0 is only read by segmentation (disabled)
  std::vector<uint32_t> hist((size_t)REPL * K.nh, 0);
  rc = 0;
  rc = rc ? rc : dalloc(ctx, &pl.d_tiles, pl.tiles.size());
  rc = rc ? rc : dalloc(ctx, &pl.d_repl, (size_t)REPL * K.nh);
  rc = rc ? rc : dalloc(ctx, &pl.d_bcount, 1);
  rc = rc ? rc : dalloc(ctx, &pl.d_err, 1);
  hipError_t e = hipSuccess;
  if (!rc) {
    if (!pl.tiles.empty()) e = hipMemcpyAsync(pl.d_tiles, pl.tiles.data(), sizeof(Tile) * pl.tiles.size(), hipMemcpyHostToDevice, CTX_STREAM(ctx));
    if (e == hipSuccess) e = hipMemsetAsync(pl.d_repl, 0, sizeof(uint32_t) * REPL * K.nh, CTX_STREAM(ctx));
    if (e == hipSuccess) e = hipMemsetAsync(pl.d_err, 0, 4, CTX_STREAM(ctx));
    if (e == hipSuccess) e = hipMemsetAsync(pl.d_bcount, 0, 4, CTX_STREAM(ctx));
    if (e == hipSuccess && pl.lds_hist && pl.bg_lds > 64 * 1024)
      hipFuncSetAttribute((const void*)k_prep<true, false, true, false, false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.bg_lds),
      hipFuncSetAttribute((const void*)k_prep<true, false, true, false, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pl.bg_lds);
    if (e == hipSuccess) e = launch_prep(&pl, false);
    if (e == hipSuccess && d_row) {
      const int W = K.h1b + K.n2 + 2;
      hipLaunchKernelGGL(k_bg_rows_get, dim3((unsigned)((W + 255) / 256), 1u), dim3(256), 0, CTX_STREAM(ctx), pl.K,
                         pl.d_repl, (unsigned long long)K.nh, pl.d_bcount, (long long*)d_row, (long long)W);
      e = hipGetLastError();
    } else if (e == hipSuccess) {
      e = hipMemcpyAsync(hist.data(), pl.d_repl, sizeof(uint32_t) * REPL * K.nh, hipMemcpyDeviceToHost, CTX_STREAM(ctx));
    }
    uint32_t err = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&err, pl.d_err, 4, hipMemcpyDeviceToHost, CTX_STREAM(ctx));
    if (e == hipSuccess) e = hipStreamSynchronize(CTX_STREAM(ctx));
    if (e == hipSuccess && err) rc = (err & ERR_KEY) ? set_err(ctx, SFS2D_E_KEY, "allele count above 2*pop_size")
                                                     : set_err(ctx, SFS2D_E_GRID, "folded 2D bin outside the grid");
  }
  hipFree(pl.d_tiles); hipFree(pl.d_repl); hipFree(pl.d_err); hipFree(pl.d_bcount);
  pl.d_tiles = nullptr; pl.d_repl = nullptr; pl.d_err = nullptr; pl.d_bcount = nullptr;
  if (e != hipSuccess) return set_err(ctx, SFS2D_E_HIP, std::string("bg_hist: ") + hipGetErrorString(e));
  if (rc || d_row) return rc;
  for (int k = 0; k < K.h1b + K.n2 + 1; ++k) {
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
