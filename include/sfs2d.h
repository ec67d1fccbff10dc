/*
 * sfs2d.h -- C ABI of the MI355X windowed 2D-SFS composite-likelihood scan.
 *
 * Drop-in boundary for the hot path of uricchio/2DSFS-scan: the per-window 2D-SFS + folded
 * 1D-SFS accumulation and the T2D / T1D multinomial log-likelihood ratios against a
 * background SFS (scripts/src/twoDSFS_class.py, scripts/sims_scan.py).  The reference has no
 * FFI layer -- its boundary is the Python class `LikelihoodInference_jointSFS`
 * (twoDSFS_class.py:20-33) -- so these entry points are what that class's methods bind through
 * ctypes:
 *
 *   sfs2d_data_upload / _wrap_device  <- the SNP dict built by make_data_dict_vcf (36-138),
 *                                        packed into SoA (sorted as in combined_scan 828-835)
 *   sfs2d_bg_hist                     <- calculate_2d_sfs (140-232) + calculate_1d_sfs (398-444)
 *                                        over a whole chromosome / data set (background SFS)
 *   sfs2d_plan_create + sfs2d_plan_run <- the window loop of combined_scan (787-991),
 *                                        scan_chooseChr (993), scan_precomputed_BG (1161),
 *                                        scan_*_bySNPs (1303, 1422), sims_scan.process_window (451):
 *                                        per window calculate_2d_sfs + fold_1d_sfs(calculate_1d_sfs)
 *                                        + calculate_likelihood_2D (625-684) / _1D (478-537)
 *   sfs2d_scan                        <- one-shot plan_create + plan_run + copy-out
 *
 * Conventions: every call returns 0 on success or a negative SFS2D_E* code; the message is
 * available from sfs2d_last_error(ctx).  Nothing throws or aborts across the ABI.  The caller
 * owns every host buffer; the library owns the device buffers inside ctx / data / plan.
 * One ctx per GPU; calls on one ctx must be serialised by the caller.  All work is enqueued on
 * the ctx's HIP stream (sfs2d_ctx_set_stream to share a stream with another runtime).
 */
#ifndef SFS2D_H
#define SFS2D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 5-6): sfs2d_ctx_set_stream(ctx, NULL) selects the HIP null stream (1: the ctx's own),
 * sfs2d_ctx_use_own_stream / sfs2d_ctx_get_stream added, the sfs2d_dist_* entry points removed;
 * sfs2d_graph_* added (round 6, additive) */
#define SFS2D_ABI_VERSION 2

/* status codes */
#define SFS2D_OK 0
#define SFS2D_E_ARG (-1)       /* invalid argument (sizes, modes, null pointers) */
#define SFS2D_E_HIP (-2)       /* HIP runtime error (message has the HIP string) */
#define SFS2D_E_NOMEM (-3)     /* device allocation failed */
#define SFS2D_E_KEY (-4)       /* an alt count > 2*pop_size: the reference raises KeyError (calculate_1d_sfs:433) */
#define SFS2D_E_GRID (-5)      /* a folded 2D bin lies outside the (2n1+1)x(2n2+1) grid */
#define SFS2D_E_CAP (-6)       /* output capacity too small (*nwin_out holds the needed size) */

/* window modes */
#define SFS2D_WINDOW_BP 0      /* fixed-bp windows, window id (pos-1)//ws per chromosome (twoDSFS_class.py:894, 948) */
#define SFS2D_WINDOW_SNPS 1    /* fixed SNP-count windows, incomplete tail dropped (1515-1535) */

/* background modes */
#define SFS2D_BG_PER_CHROM 0   /* each chromosome's own SNPs form its background (combined_scan 809-825) */
#define SFS2D_BG_SUPPLIED 1    /* one background for all windows (scan_chooseChr / precomputed / sims) */

/* plan flags */
#define SFS2D_F_PREV_EXTRA 1u  /* also evaluate the previous window's 1D SFSs against the LAST window's
                                  chromosome background (combined_scan final block, 951-989, quirk Q9) */

#define SFS2D_F_FST 2u         /* also compute Hudson's Fst per window slot (not in the reference),
                                  read with sfs2d_plan_fst_read / sfs2d_plan_fst_buffer */

/* window record flags */
#define SFS2D_W_EMPTY 0x80000000u  /* slot holds no SNP (fixed-bp slot between SNPs): not a window */
#define SFS2D_W_BG2_ZERO 0x1u      /* background 2D inner sum == 0  -> None / ZeroDivisionError */
#define SFS2D_W_BG1A_ZERO 0x2u
#define SFS2D_W_BG1B_ZERO 0x4u
#define SFS2D_W_EXTRA 0x40000000u  /* record is the Q9 helper (see SFS2D_F_PREV_EXTRA) */

typedef struct sfs2d_ctx sfs2d_ctx;
typedef struct sfs2d_data sfs2d_data;
typedef struct sfs2d_plan sfs2d_plan;
typedef struct sfs2d_graph sfs2d_graph;

typedef struct {
  int32_t n1p, n2p;       /* pop1_size, pop2_size: diploid individuals (twoDSFS_class.py:22); grid (2n1p+1)x(2n2p+1) */
  int32_t fold;           /* joint 2D fold: swap ref/alt in both pops if alt1+alt2 > n1p+n2p (197-206) */
  int32_t window_mode;    /* SFS2D_WINDOW_BP / SFS2D_WINDOW_SNPS */
  int64_t window;         /* window size in bp, or SNPs per window */
  int32_t bg_mode;        /* SFS2D_BG_PER_CHROM / SFS2D_BG_SUPPLIED */
  int32_t ann_want;       /* variant_type filter: annotation id to keep, -1 = no filter (185-187, 291-302) */
  int32_t has_start, has_end; /* SFS position filter start_position / end_position (179-182) */
  int64_t start_pos, end_pos;
  uint32_t flags;         /* SFS2D_F_* */
  uint32_t scan_wgs_per_cu; /* 0: the scan kernel's grid is one resident wave of workgroups (all that fit);
                               k > 0: at most k workgroups per CU -- leaves CUs to the next pass's k_prep
                               when independent passes overlap on several streams (sfs2d_plan_run_streams) */
} sfs2d_params;

/* one record per window slot (64 bytes) */
typedef struct {
  uint32_t chrom;         /* chromosome index in the data set's (sorted) chromosome list */
  uint32_t wid;           /* window index within the chromosome: (pos-1)//ws, or SNP-window ordinal */
  uint32_t begin, end;    /* SNP index range [begin, end) in the data set */
  uint32_t snp_count;     /* count_snps (291-302): SNPs in the window matching variant_type */
  uint32_t n2;            /* 2D foreground total over inner bins bins[1:-1] (N of T2D) */
  uint32_t n2_all;        /* 2D foreground total over all bins (scan_*_bySNPs skip test, 1376/1496) */
  uint32_t n1a, n1b;      /* folded 1D foreground totals over inner bins 1..pop_size-1 */
  uint32_t flags;         /* SFS2D_W_* */
  double t2d, t1d_p1, t1d_p2; /* NaN-boxed "None" is not used: validity = n>0 and !BG*_ZERO */
} sfs2d_window;

/* context */
int sfs2d_ctx_create(int device, sfs2d_ctx** out);
int sfs2d_ctx_destroy(sfs2d_ctx* ctx);
const char* sfs2d_last_error(const sfs2d_ctx* ctx);
/* Stream the ctx enqueues on.  sfs2d_ctx_set_stream(ctx, s): the caller's HIP stream s; NULL is the
 * HIP null stream (the legacy default stream: ordered with every blocking stream of the process, e.g.
 * torch's default stream), never a private one.  sfs2d_ctx_use_own_stream: the ctx's own non-blocking
 * stream (the state after sfs2d_ctx_create), which NOTHING orders against the caller's streams --
 * synchronise before handing buffers across.  The class state these replace is the reference object's
 * (twoDSFS_class.py:21-33): one ctx per GPU, calls serialised by the caller. */
int sfs2d_ctx_set_stream(sfs2d_ctx* ctx, void* hip_stream);
int sfs2d_ctx_use_own_stream(sfs2d_ctx* ctx);
/* the HIP stream the ctx currently enqueues on (NULL = the null stream; after sfs2d_ctx_create or
 * sfs2d_ctx_use_own_stream, the handle of the ctx's own stream) -- e.g. to pass it to
 * sfs2d_plan_run_streams or to order a caller's stream after the ctx's work */
int sfs2d_ctx_get_stream(const sfs2d_ctx* ctx, void** hip_stream);
/* SFS2D_ABI_VERSION of the loaded library (negative: an ablation build for timing experiments, whose
 * results are wrong -- loaders must refuse it) */
int sfs2d_abi_version(void);

/* data set: packed SNPs in scan order (sorted by chromosome string, then position) */
int sfs2d_data_upload(sfs2d_ctx* ctx, const uint32_t* counts, const uint32_t* pos, const uint16_t* ann_id,
                      int64_t n, const int64_t* chrom_off, int32_t nchrom, sfs2d_data** out);
/* wrap caller-owned DEVICE arrays (no copy); chrom_off / chrom_last_pos are HOST arrays */
int sfs2d_data_wrap_device(sfs2d_ctx* ctx, const uint32_t* d_counts, const uint32_t* d_pos,
                           const uint16_t* d_ann_id, int64_t n, const int64_t* chrom_off,
                           const uint32_t* chrom_last_pos, int32_t nchrom, sfs2d_data** out);
int sfs2d_data_free(sfs2d_data* data);

/* Synthetic sims replicates generated in HBM (BASELINE config 4: sims_scan.likelihood_scan's
 * replicate VCFs, sims_scan.py:593-644, at thousands of replicates).  Each replicate is one
 * chromosome of n_windows fixed windows of window_bp; win_snps[r * n_windows + w] (host) SNPs in
 * window w of replicate r (the caller draws them, e.g. Poisson(358.5)); per-SNP values from a
 * counter-based Philox stream keyed by seed and generation (the model is in sfs2d_kernels.hpp;
 * the host twin sfs2d.synth.sims_host reproduces it bit for bit).  miss_cdf1 / miss_cdf2: u32
 * inverse-CDF thresholds of the missing-allele counts of each population (nm entries, the last
 * 0xffffffff).  The data set owns its arrays. */
typedef struct {
  uint64_t seed;
  uint32_t generation, n_replicates, n_windows, window_bp;
  int32_t n1p, n2p;   /* diploid pop sizes: counts <= 2 * pop size */
} sfs2d_synth_params;
int sfs2d_data_synth_sims(sfs2d_ctx* ctx, const sfs2d_synth_params* sp, const uint16_t* win_snps,
                          const uint32_t* miss_cdf1, int32_t nm1, const uint32_t* miss_cdf2, int32_t nm2,
                          sfs2d_data** out);
/* copy a data set's packed counts / positions to host (n = the data set's SNP count; NULL skips) */
int sfs2d_data_read(const sfs2d_data* data, uint32_t* counts, uint32_t* pos, int64_t n);

/* Background SFS histograms of chromosome `chrom` (-1: all SNPs of the data set), with the
 * params' filters (position, variant_type, fold).  h2d: (2n1p+1)*(2n2p+1) int64, row-major
 * (alt1, alt2); h1a / h1b: UNFOLDED 1D spectra of raw alt counts, 2*pop_size+1 int64 each. */
int sfs2d_bg_hist(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* params, int32_t chrom,
                  int64_t* h2d, int64_t* h1a, int64_t* h1b);

/* The same histograms as ONE int64 row on the device (d_row: SFS2D_BG_ROW_WORDS int64), laid out
 * [2D bins | unfolded pop-1 spectrum | unfolded pop-2 spectrum | inner 2D sum (bins[1:-1])]: the
 * multi-GPU calculate_2d_sfs / calculate_1d_sfs (sfs2d/dist.py sharded_bg_hist) all-reduce these
 * rows over the ranks without a host copy.  Enqueued on the ctx stream; synchronises to report
 * SFS2D_E_KEY / SFS2D_E_GRID (the row is then undefined). */
#define SFS2D_BG_ROW_WORDS(n1p, n2p) ((2 * (n1p) + 1) * (2 * (n2p) + 1) + 2 * (n1p) + 2 * (n2p) + 3)
int sfs2d_bg_hist_dev(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* params, int32_t chrom,
                      int64_t* d_row);

/* Plans: everything that depends only on (data, params) is built once; plan_run enqueues the pass's
 * kernels (k_prep, k_bg_slice, the scan) with inputs and outputs resident in HBM. */
int sfs2d_plan_create(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* params, sfs2d_plan** out);
/* number of output records the plan writes (window slots, +1 when SFS2D_F_PREV_EXTRA) */
int64_t sfs2d_plan_num_records(const sfs2d_plan* plan);
/* SFS2D_BG_SUPPLIED: background values (host doubles, integer or normalised): bg2d has
 * (2n1p+1)*(2n2p+1) entries, bg1a / bg1b have n1p+1 / n2p+1 entries read at keys 1..pop_size-1
 * (folded or, for the sims path, unfolded spectra: quirk Q7). */
int sfs2d_plan_set_background(sfs2d_plan* plan, const double* bg2d, const double* bg1a, const double* bg1b);
/* enqueue the scan; out_dev: device buffer of sfs2d_plan_num_records records (NULL = plan-owned) */
int sfs2d_plan_run(sfs2d_plan* plan, sfs2d_window* out_dev);
/* enqueue `nruns` back-to-back runs (no host work in between; benchmarks and batch replays) */
int sfs2d_plan_run_many(sfs2d_plan* plan, int nruns, sfs2d_window* out_dev);
/* enqueue `nruns` runs round-robin over `nplans` distinct plans of one ctx: run i is plans[i % nplans]
 * on streams[i % nplans] (NULL = the HIP null stream, as sfs2d_ctx_set_stream) into outs[i % nplans]
 * (outs NULL or an entry NULL = plan-owned).  Independent scans (replicates, data sets, repeated
 * passes) overlap across the streams; each plan's own runs stay ordered on its stream.  The
 * ctx stream is unchanged after.  The runs are only enqueued: synchronise the passed streams before
 * sfs2d_plan_read / _check / _fst_read / _destroy of these plans (those synchronise the ctx stream
 * only). */
int sfs2d_plan_run_streams(sfs2d_plan* const* plans, void* const* streams, sfs2d_window* const* outs, int nplans,
                           int nruns);
/* the same run sequence captured once into HIP graphs, one per distinct stream (that stream's runs in
 * sequence order), and replayed by sfs2d_graph_launch: one hipGraphLaunch per stream and replay instead of
 * a launch per kernel (short passes are host-bound otherwise).  nruns must be a multiple of 2 * nplans
 * (every plan runs an even number of times per replay, so its buffer parity is unchanged); streams
 * non-null; no plan with timing on or attached.  The outputs are fixed at capture.  Replays run on the
 * capture streams, each after that stream's earlier work, without run_streams' staggered start.  A launch
 * fails with SFS2D_E_ARG when a captured plan ran an odd number of times since the capture.  Not a
 * reference interface: repeated scans of the same data (the bench's loops; replicate loops as
 * sims_scan.py:593-644). */
int sfs2d_graph_create(sfs2d_plan* const* plans, void* const* streams, sfs2d_window* const* outs, int nplans,
                       int nruns, sfs2d_graph** out);
int sfs2d_graph_launch(sfs2d_graph* graph, int nlaunch);
int sfs2d_graph_destroy(sfs2d_graph* graph);
/* copy the last run's records to host (synchronises the stream) */
int sfs2d_plan_read(sfs2d_plan* plan, sfs2d_window* out_host, int64_t cap, int64_t* nrec_out);
/* device pointers of the plan's per-chromosome background histogram replicas (uint32), for a
 * multi-GPU all-reduce between sfs2d_plan_run_phase(plan, 1) and (plan, 2). */
int sfs2d_plan_bg_buffer(sfs2d_plan* plan, void** dev_ptr, int64_t* nbytes);
/* Multi-GPU split of a chromosome over ranks (sfs2d/dist.py): between sfs2d_plan_run_phase(plan, 1)
 * (k_prep: this rank's part of every chromosome's background histograms) and (plan, 2) (tables and
 * scan), every rank reads its partial histograms -- replicas x nchrom x bins uint32 words, laid out
 * [replica][chromosome][bin] (the consumer sums the replicas), and nchrom uint32 per-chromosome inner
 * 2D sums (sizes: sfs2d_plan_bg_words) -- sums them over the ranks (the SURVEY 8(e) all-reduce) and
 * writes the totals back (to_device = 1).  Synchronous.  Replaces the whole-chromosome background
 * loops of calculate_2d_sfs / calculate_1d_sfs (twoDSFS_class.py:140-232, 398-444) when one
 * chromosome's SNPs are held by several ranks.  Plans without per-chromosome backgrounds: all 0. */
int sfs2d_plan_bg_words(const sfs2d_plan* plan, int64_t* replicas, int64_t* nchrom, int64_t* bins);
int sfs2d_plan_bg_exchange(sfs2d_plan* plan, uint32_t* host_repl, uint32_t* host_sums, int to_device);
/* The device-resident form of that exchange (no host copy; the SURVEY 8(e) all-reduce runs on the
 * rows in HBM, RCCL over xGMI): after sfs2d_plan_run_phase(plan, 1), _bg_rows_dev writes the plan's
 * per-chromosome partial histograms as int64 rows (row c at d_rows + c * row_stride, row_stride >=
 * SFS2D_BG_ROW_WORDS; layout of sfs2d_bg_hist_dev); after the all-reduce, _bg_rows_set_dev writes the
 * summed rows back (sums >= 2^32: SFS2D_E_ARG from sfs2d_plan_check), then sfs2d_plan_run_phase(plan, 2).
 * Both are enqueued on the ctx stream (order the collective against it). */
int sfs2d_plan_bg_rows_dev(sfs2d_plan* plan, int64_t* d_rows, int64_t row_stride);
int sfs2d_plan_bg_rows_set_dev(sfs2d_plan* plan, const int64_t* d_rows, int64_t row_stride);
/* Fst of the last run per window slot (NaN: no qualifying SNP / empty slot); plans with SFS2D_F_FST */
int sfs2d_plan_fst_read(sfs2d_plan* plan, double* out_host, int64_t cap);
int sfs2d_plan_fst_buffer(sfs2d_plan* plan, void** dev_ptr, int64_t* nslots);
/* Fst output of the following runs: a caller-owned device buffer of >= nslots doubles (NULL = the plan-owned
 * buffer again), as sfs2d_plan_run's out_dev is for the records -- consecutive runs of one plan can keep their
 * Fst columns apart (e.g. each pass's table gathered while the next pass runs: bench.py at N > 1).  Attached
 * plans keep their own buffer. */
int sfs2d_plan_set_fst_out(sfs2d_plan* plan, double* d_fst);
int sfs2d_plan_run_phase(sfs2d_plan* plan, int phase, sfs2d_window* out_dev);
/* Multi-resolution: attach to `base` (a per-chromosome-background plan on the small-grid path) a
 * plan over the same data whose params differ only in window_mode / window / flags.  The base's
 * run then makes ONE k_prep pass over the SNP stream (background histograms, per-SNP bins, the
 * base's segmentation and Fst sums) and scans every attached plan from it before its own scan:
 * fixed-bp windows get their slots by binary search on the resident positions, SNP-count windows
 * need none; SFS2D_F_FST on an attached plan needs a fixed-bp Fst base whose window divides the
 * attached window (the base's per-window int64 fixed-point sums add exactly).  The reference
 * script scans the same data at 20 kb, 500 kb and 500 / 300 SNPs (twoDSFS_class.py:1923-2032).
 * An attached plan is not run on its own (its run calls fail); read it with sfs2d_plan_read /
 * sfs2d_plan_fst_read after the base's run.  Destroying the base destroys its attached plans. */
int sfs2d_plan_attach(sfs2d_plan* base, const sfs2d_params* params, sfs2d_plan** out);
/* launch geometry (threads per grid) of k_prep and of the scan kernel: matches the Grid_Size column
 * of rocprofv3 kernel traces, so profiles can be joined to a plan */
int sfs2d_plan_grids(const sfs2d_plan* plan, int64_t* prep_threads, int64_t* scan_threads);
/* name of the scan kernel the plan launches ("k_scan_w", "k_scan_gw", "k_scan_g"; the
 * prefix of its rocprofv3 kernel name), NULL for a null plan */
const char* sfs2d_plan_scan_kernel(const sfs2d_plan* plan);
/* cumulative number of windows re-evaluated on the exact path (|T| ~ 0: proportionality test) */
int sfs2d_plan_stats(sfs2d_plan* plan, uint32_t* exact_windows);
/* last run's error word (0 = ok, else SFS2D_E_KEY / SFS2D_E_GRID, or SFS2D_E_ARG for summed background
 * rows that overflow); synchronises */
int sfs2d_plan_check(sfs2d_plan* plan);
/* live timing: every `every`-th of the following runs (up to `max_samples` of them) launches k_prep
 * and the scan kernel with start/stop events in their own dispatch packets (hipExtLaunchKernelGGL):
 * kernel start/end timestamps, the durations rocprofv3 --kernel-trace reports; no extra packets
 * between kernels.  sfs2d_plan_timing_read averages the sampled runs' per-kernel durations */
int sfs2d_plan_set_timing(sfs2d_plan* plan, int max_runs);   /* = sampled(plan, max_runs, 1) */
int sfs2d_plan_set_timing_sampled(sfs2d_plan* plan, int max_samples, int every);
/* the same for a subset of the kernels: bit 0 k_prep, bit 1 k_bg_slice, bit 2 the scan kernel (an event
 * pair costs queue time: the bench times only the scan kernel inside its timed loop); the kernels
 * left out read 0 in sfs2d_plan_timing_read */
int sfs2d_plan_set_timing_kernels(sfs2d_plan* plan, int max_samples, int every, int kernel_mask);
/* average device time per kernel over the sampled runs (synchronises): k1 = k_prep, k2 = k_bg_slice
 * (0 when the plan does not launch it), k3 = the window scan kernel (k_scan_w / k_scan_gw / k_scan_g) */
int sfs2d_plan_timing_read(sfs2d_plan* plan, int* nruns, double* ms_k1, double* ms_k2, double* ms_k3);
/* standalone timing loop: average device time per kernel over `iters` runs */
int sfs2d_plan_time(sfs2d_plan* plan, int iters, double* ms_per_run, double* ms_k1, double* ms_k2, double* ms_k3);
int sfs2d_plan_destroy(sfs2d_plan* plan);

/* one-shot convenience: plan + run + read (+ supplied background when bg2d != NULL) */
int sfs2d_scan(sfs2d_ctx* ctx, const sfs2d_data* data, const sfs2d_params* params, const double* bg2d,
               const double* bg1a, const double* bg1b, sfs2d_window* out_host, int64_t cap, int64_t* nrec_out);

#ifdef __cplusplus
}
#endif
#endif /* SFS2D_H */
