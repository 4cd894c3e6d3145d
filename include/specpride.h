/*
 * specpride.h -- C-ABI of the MI355X consensus/representative-spectrum engine
 * (libspecpride_hip.so, built from specpride_amd/csrc for gfx950).
 *
 * The reference (timosachsenberg/specpride) has no FFI: its hot path is three
 * Python functions.  Each entry point below replaces one of them for a whole
 * batch of clusters at once; the Python shims in specpride_amd/ keep the
 * reference's own names and call these through ctypes.
 *
 *   spx_bin_mean     <- src/binning.py:170-231  RepresentativeSpectrumCreator.combine_bin_mean
 *                       (called per cluster from binning.py:291-297)
 *   spx_gap_average  <- src/average_spectrum_clustering.py:26-103  average_spectrum
 *                       + precursor helpers :106-148 (called from :151-165)
 *   spx_medoid       <- src/most_similar_representative.py:13-19 distance() and the
 *                       per-cluster medoid loop :60-111
 *   spx_bin_mean_medoid <- both of the above in one pass (the configs[4] pipeline step)
 *   spx_xcorr_distance <- src/most_similar_representative.py:13-19 distance() per pair
 *   spx_binned_cosine  <- src/benchmark.py:10-38  bin_proc / cos_dist / average_cos_dist
 *                       (representative vs its cluster members)
 *   spx_best_score   <- src/best_spectrum.py:67-100  get_best_representative
 *                       (called per cluster from best_spectrum():170-174)
 *   spx_compact_peaks   (packing helper for the shims' output writers)
 *   spx_wire_pack / spx_wire_unpack  (9-byte consensus peaks for the multi-GPU gather to rank 0)
 *   spx_copy_h2d / spx_copy_d2h  (host transfers of pageable batches: the reference
 *                       holds its spectra in host memory, binning.py:122-167)
 *
 * Conventions
 *   - Every array pointer inside spx_csr / outputs is a DEVICE pointer (HBM),
 *     owned by the caller.  The library owns nothing but the workspace contents
 *     while a call runs; size the workspace with the *_workspace_size queries.
 *   - Work is enqueued on `stream` (a hipStream_t, passed as void*; NULL = the
 *     default stream) and is asynchronous.  Entry points are reentrant (no
 *     global mutable state) and never allocate or synchronise, so they can be
 *     captured into a hipGraph.  The caller selects the device.
 *   - Return value: SPX_SUCCESS or a negative spx_error.  Per-cluster outcomes
 *     are reported in `status[c]` (spx_status) -- the shims raise the
 *     reference's exception type for the first failing cluster in order.
 *   - Peak outputs use the cluster's INPUT peak range as capacity: cluster c
 *     writes count[c] peaks at out->mz/inten[spec_off[cluster_off[c]] + k], so
 *     the out arrays have n_peaks entries and no planning pass is needed.
 */
#ifndef SPECPRIDE_H_
#define SPECPRIDE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPX_ABI_VERSION 2

typedef enum spx_error {
  SPX_SUCCESS = 0,
  SPX_EINVAL = -1,   /* bad argument (null pointer, inconsistent sizes) */
  SPX_EHIP = -2,     /* a HIP launch/runtime call failed */
  SPX_ENOSPACE = -3  /* workspace smaller than the matching *_workspace_size */
} spx_error;

typedef enum spx_status {
  SPX_OK = 0,
  SPX_MIXED_CHARGE = 1, /* binning.py:205-206 AssertionError / :131 ValueError   */
  SPX_NO_GAP = 2,       /* average_spectrum_clustering.py:69 IndexError          */
  SPX_EMPTY = 3,        /* average_spectrum_clustering.py:95 ValueError (max())  */
  SPX_NON_FINITE = 4,   /* spx_best_score: only NaN scores (gap-average carries NaN/inf as the reference does) */
  SPX_UNRESOLVED = 100  /* outside the engine's limits            */
} spx_status;

/* Cluster-segmented CSR batch (device pointers).  Clusters are [cluster_off[c],
 * cluster_off[c+1]) in spectra; spectra are [spec_off[s], spec_off[s+1]) in peaks;
 * peaks in file order (not re-sorted).  rt may be NULL except for spx_gap_average. */
typedef struct spx_csr {
  int64_t n_clusters, n_spectra, n_peaks;
  const int64_t *cluster_off; /* [n_clusters + 1] */
  const int64_t *spec_off;    /* [n_spectra + 1]  */
  const double *mz;           /* [n_peaks] */
  const double *inten;        /* [n_peaks] */
  const double *prec_mz;      /* [n_spectra] */
  const int32_t *charge;      /* [n_spectra] */
  const double *rt;           /* [n_spectra] or NULL */
} spx_csr;

/* Host-side facts about the batch that size the workspace (any upper bound works). */
typedef struct spx_batch_info {
  int64_t max_cluster_peaks;   /* max over clusters of its peak count */
  int64_t max_cluster_spectra; /* max over clusters of its spectrum count */
  double max_mz_span;          /* max over clusters of (max m/z - min m/z); 0 = 5000 Da */
} spx_batch_info;

typedef struct spx_peaks_out {
  double *mz;     /* [n_peaks] capacity, see "Peak outputs" above */
  double *inten;  /* [n_peaks] */
  int64_t *count; /* [n_clusters] peaks written per cluster */
} spx_peaks_out;

/* ---- bin-mean: RepresentativeSpectrumCreator.combine_bin_mean(peaklists,
 *      minimum=100, maximum=2000, binsize=0.02, apply_peak_quorum=True) ---- */
typedef struct spx_bin_params {
  double minimum, maximum, binsize;
  int32_t apply_peak_quorum;
} spx_bin_params;

size_t spx_bin_mean_workspace_size(const spx_csr *csr, const spx_bin_params *params,
                                   const spx_batch_info *info);
/* prec_out[c] = np.mean(precursor m/z), charge_out[c] = charge of the cluster. */
int spx_bin_mean(const spx_csr *csr, const spx_bin_params *params, const spx_batch_info *info,
                 spx_peaks_out *out, double *prec_out, int32_t *charge_out, int32_t *status,
                 void *workspace, size_t workspace_bytes, void *stream);
/* spx_bin_mean in two halves, for a caller that reads the statuses anyway (the
 * per-cluster shim, binning.py:291-297, which copies every result back):
 *   stage 1: the register and wide kernels (and the global kernel for unsorted
 *            spectra) -- every cluster of <= 128 spectra and <= 4,096 distinct bins;
 *            the others keep status SPX_UNRESOLVED;
 *   stage 2: the chain for those (kept-bin fold, segmented fold, split path), on
 *            the SAME workspace, untouched since stage 1;
 *   stage 0: both (= spx_bin_mean).
 * Stage 1 alone is a memset and 3 kernels instead of 21 kernels: a one-cluster
 * call costs about 100 us less when no cluster needs stage 2. */
int spx_bin_mean_stage(const spx_csr *csr, const spx_bin_params *params, const spx_batch_info *info,
                       spx_peaks_out *out, double *prec_out, int32_t *charge_out, int32_t *status,
                       void *workspace, size_t workspace_bytes, void *stream, int stage);

/* ---- gap-average: average_spectrum(spectra, title, pepmass, rtinseconds, charge,
 *      mz_accuracy=0.01, dyn_range=1000, min_fraction=0.5) + precursor helpers ---- */
typedef enum spx_pepmass_mode { SPX_PEPMASS_LOWER_MEDIAN = 0, SPX_PEPMASS_NAIVE_AVERAGE = 1,
                                SPX_PEPMASS_NEUTRAL_AVERAGE = 2 } spx_pepmass_mode;
typedef enum spx_rt_mode { SPX_RT_MEDIAN = 0, SPX_RT_MASS_LOWER_MEDIAN = 1 } spx_rt_mode;

typedef struct spx_gap_params {
  double mz_accuracy, dyn_range, min_fraction;
  double proton;        /* pyteomics nist_mass['H+'][0][0] = 1.00727646677 */
  int32_t pepmass_mode; /* spx_pepmass_mode */
  int32_t rt_mode;      /* spx_rt_mode */
} spx_gap_params;

/* The workspace holds the global kernel's scratch slices and, when
 * info->max_cluster_peaks > 16,384, an arena of at most 1 GiB for the giant-cluster
 * pipeline (clusters past 16,384 peaks, tiled over the whole grid).
 * NaN / +-inf m/z or intensities give what the reference's numpy arithmetic gives
 * (NaN sorts last, inf - inf = NaN in the cumsum differences, np.max propagates
 * NaN): such a cluster is OK, possibly with NaN/inf values or no peaks, never an
 * error status (average_spectrum_clustering.py:59-98).
 * With clusters past 65,536 peaks in the batch, the giants' pipeline runs on a second
 * stream the library owns (one per device; spx_bin_mean's kept-bin fold of clusters past
 * 128 spectra and spx_medoid's large path use it the same way), forked from `stream` by an event and
 * joined back to it before the call returns: the call stays ordered on `stream`,
 * hipGraph capture of `stream` included. */
size_t spx_gap_average_workspace_size(const spx_csr *csr, const spx_gap_params *params,
                                      const spx_batch_info *info);
int spx_gap_average(const spx_csr *csr, const spx_gap_params *params, const spx_batch_info *info,
                    spx_peaks_out *out, double *pepmass_out, int32_t *charge_out, double *rt_out,
                    int32_t *status, void *workspace, size_t workspace_bytes, void *stream);

/* ---- medoid: most_similar_representative.py distance(s1, s2, 'xcorr') with
 *      XQuestScores().xCorrelationPrescore(s1, s2, 0.1) + argmin of summed distance ---- */
typedef struct spx_medoid_params {
  double tolerance;   /* 0.1 at most_similar_representative.py:15 */
  int32_t large_path; /* 1: run the large-cluster (MFMA Gram) passes for clusters the
                         small-cluster kernel defers; 0: skip them (their rep[c] is then
                         SPX_REP_DEFERRED).  0 saves ~11 small launches per call when
                         spx_medoid_needs_large_path() says no cluster is large by size. */
} spx_medoid_params;

/* rep[c] codes besides a spectrum index */
#define SPX_REP_EMPTY (-1)      /* empty cluster */
#define SPX_REP_RANGE (-2)      /* m/z range > 4.2M bins (> 420k Da at tol 0.1) */
#define SPX_REP_ARENA (-3)      /* workspace arena exhausted: grow it (extra clusters below), re-run */
#define SPX_REP_DEFERRED (-4)   /* deferred to the large path, skipped (params.large_path = 0) */

/* Needs the HOST copies of the offsets: the large-cluster arena is sized from them.
 * `extra` (nullable, n_extra entries) lists clusters to budget a full arena share for on
 * top of the ones large by size -- the clusters a previous call reported SPX_REP_ARENA
 * for (small clusters deferred at run time: m/z >= 3276.8 at tol 0.1, > 1,984 distinct
 * bins).  Budgeting them makes the re-run's arena sufficient. */
size_t spx_medoid_workspace_size(const int64_t *host_cluster_off, const int64_t *host_spec_off,
                                 int64_t n_clusters, const int64_t *extra, int64_t n_extra);
/* 1 if some cluster takes the large path by size alone (n > 64 spectra or > 12,288
 * peaks): then params.large_path must be 1.  0: only run-time deferrals are possible. */
int spx_medoid_needs_large_path(const int64_t *host_cluster_off, const int64_t *host_spec_off,
                                int64_t n_clusters);
/* rep[c] = global index of the chosen spectrum, or an SPX_REP_* code (< 0);
 * totals (nullable) [n_spectra] = the reference's total_dist per spectrum. */
int spx_medoid(const spx_csr *csr, const spx_medoid_params *params, int64_t *rep, double *totals,
               void *workspace, size_t workspace_bytes, void *stream);

/* ---- the headline step in one pass: spx_bin_mean + spx_medoid over the same batch
 *      (SURVEY.md §8(d) configs[4], "medoid + binned consensus").  Each cluster's
 *      bin-mean and medoid register bodies run back to back in one workgroup
 *      (bin_mean_medoid_kernel), then each method's own leftover chain; every output
 *      equals the two separate calls'.  The workspaces are the two calls' own
 *      (spx_bin_mean_workspace_size / spx_medoid_workspace_size). */
int spx_bin_mean_medoid(const spx_csr *csr, const spx_bin_params *bin_params, const spx_batch_info *info,
                        spx_peaks_out *out, double *prec_out, int32_t *charge_out, int32_t *status,
                        void *bin_workspace, size_t bin_workspace_bytes, const spx_medoid_params *medoid_params,
                        int64_t *rep, double *totals, void *medoid_workspace, size_t medoid_workspace_bytes,
                        void *stream);
/* spx_bin_mean_medoid in two halves (ABI 2, round 6):
 *   stage 1: the fused register pass alone (bin_mean_medoid_kernel); the clusters either
 *            register body hands on stay on its list.  With `handoff` (a DEVICE int32[2],
 *            nullable) it also writes how many: [0] bin-mean, [1] medoid;
 *   stage 2: both leftover chains (the 21 bin-mean and 1-12 medoid kernels that take
 *            what the register bodies could not), on the SAME workspaces, untouched
 *            since stage 1;
 *   stage 0: both (= spx_bin_mean_medoid).
 * Which clusters a register body hands on depends only on the batch and the parameters,
 * so a caller that saw both counts at 0 after stage 1 may run the same (unchanged) batch
 * with stage 1 alone and skip ~22 launches that would find their lists empty; results
 * are then identical to stage 0.  Any other caller runs stage 2 (or stage 0). */
int spx_bin_mean_medoid_stage(const spx_csr *csr, const spx_bin_params *bin_params, const spx_batch_info *info,
                              spx_peaks_out *out, double *prec_out, int32_t *charge_out, int32_t *status,
                              void *bin_workspace, size_t bin_workspace_bytes,
                              const spx_medoid_params *medoid_params, int64_t *rep, double *totals,
                              void *medoid_workspace, size_t medoid_workspace_bytes, void *stream, int stage,
                              int32_t *handoff);

/* distance(spec1, spec2, 'xcorr') = 1 - xCorrelationPrescore for n_pairs (global
 * spectrum index) pairs: out[p] for pairs[2p], pairs[2p+1].  The per-call API
 * behind most_similar_representative.distance (:13-19); not the batched path. */
int spx_xcorr_distance(const spx_csr *csr, const spx_medoid_params *params, const int64_t *pairs,
                       int64_t n_pairs, double *out, void *stream);

/* ---- binned cosine: benchmark.cos_dist(representative, member) for every member of
 *      every cluster + average_cos_dist per cluster (benchmark.py:10-38) ---- */
typedef struct spx_cosine_params {
  double mz_space; /* benchmark.py:7-8: 1.000508 * .005 */
} spx_cosine_params;

/* Cluster c's representative is the peak list [rep_off[c], rep_off[c+1]) of
 * rep_mz / rep_inten (device arrays; e.g. the compacted bin-mean output); its
 * members are the cluster's spectra in csr.  cos_out [n_spectra] = cos_dist per
 * member, avg_out [n_clusters] = average_cos_dist (0.0 for no members).
 * status[c]: SPX_EMPTY if the representative or a member has no peaks (the
 * reference's mz[-1] raises IndexError; NaN outputs).  Representatives of up to
 * 512 peaks are sorted in LDS; longer ones (max_rep_peaks = an upper bound on
 * every representative's length) in a global workspace slice, so any length is
 * evaluated; SPX_UNRESOLVED only if a representative exceeds max_rep_peaks. */
size_t spx_binned_cosine_workspace_size(int64_t n_clusters, int64_t max_rep_peaks);
int spx_binned_cosine(const spx_csr *csr, const int64_t *rep_off, const double *rep_mz, const double *rep_inten,
                      const spx_cosine_params *params, double *cos_out, double *avg_out, int32_t *status,
                      int64_t max_rep_peaks, void *workspace, size_t workspace_bytes, void *stream);

/* ---- best spectrum: best_spectrum.get_best_representative(cluster, scores) for every
 *      cluster: scores.idxmax() over the cluster's members (best_spectrum.py:97-100) ---- */

/* Only csr->n_clusters / n_spectra / cluster_off are read (no peaks).  Per spectrum
 * (device arrays [n_spectra]): score = the max non-NaN PSM score of its USI (NaN if
 * every PSM score is NaN), rank = the USI's position among the sorted distinct score
 * USIs (the order of get_scores()' sort_index, best_spectrum.py:64), -1 = no PSM.
 * best[c] = global index of the member with the highest score, ties to the lowest
 * rank (idxmax = first maximum in sorted-USI order); -1 if none.  status[c]:
 * SPX_EMPTY if no member has a PSM (the reference's ValueError, :98-99), SPX_NON_FINITE
 * if every matching score is NaN (pandas' idxmax returns NaN -> KeyError). */
int spx_best_score(const spx_csr *csr, const double *score, const int64_t *rank, int64_t *best, int32_t *status,
                   void *stream);

/* Pack the per-cluster outputs densely: dst[out_off[c] + k] = src[spec_off[cluster_off[c]] + k]
 * for k < count[c]; out_off is the exclusive prefix sum of count (device array [C+1]). */
int spx_compact_peaks(const spx_csr *csr, const spx_peaks_out *src, const int64_t *out_off,
                      double *dst_mz, double *dst_inten, void *stream);

/* Wire format of the multi-GPU gather (csrc/wire.hip; shard.StepGatherer): bin-mean
 * consensus peaks (mz, inten)[n] (dense, device) -> mi[2n] (f32 bin sums M, I) and
 * count[n] (count_bytes = 1 or 2 bytes each, max_count <= 255 or <= 65,535: at least the
 * batch's largest cluster size), 9 or 10 bytes a peak instead of 16; spx_wire_unpack
 * rebuilds the doubles bit for bit (mz = M == 0 ? NaN : f64(M)/c, inten = f64(I)/c,
 * binning.py:211-218).  A peak no count <= max_count rebuilds exactly (not a bin-mean
 * output) is sent as NaN and counted in *n_fail (device int32, zeroed by the caller).
 * The inputs are meant to be spx_bin_mean outputs: a peak whose rebuild fails costs
 * max_count exact tests (the search cannot stop early), so pass the batch's real largest
 * cluster size as max_count, not the 65,535 bound. */
int spx_wire_pack(const double *mz, const double *inten, int64_t n, int32_t max_count, float *mi, void *count,
                  int32_t count_bytes, int32_t *n_fail, void *stream);
int spx_wire_unpack(const float *mi, const void *count, int32_t count_bytes, int64_t n, double *mz, double *inten,
                    void *stream);

/* Host <-> device copies of batches in PAGEABLE host memory (SURVEY.md §8(d) tier 2).
 * The bytes are staged through a process-wide pool of pinned buffers by several host
 * threads, each chunk's DMA (on `stream`) overlapping the next chunk's staging copy.
 * Unlike the compute entry points these use host threads and a staging pool that is
 * allocated on first use and shared (calls are serialised).  spx_copy_h2d returns once
 * the source has been consumed; the device copy is ordered on `stream`.  spx_copy_d2h
 * returns with dst_host complete (after the work already on `stream`). */
int spx_copy_h2d(void *dst_device, const void *src_host, size_t nbytes, void *stream);
int spx_copy_d2h(void *dst_host, const void *src_device, size_t nbytes, void *stream);

int spx_abi_version(void);
const char *spx_last_error(void); /* thread-local text of the last failure */

/* Diagnostics (bench.py's per-kernel rooflines).  spx_profile_enable(1) brackets the
 * launches of bin_mean_reg_kernel, medoid_reg_kernel, the medoid Gram kernel ("medoid_gram_kernel"),
 * gap_average_lds_kernel, gap_average_wide_kernel and bin_mean_medoid_kernel with HIP events on the caller's
 * stream (and resets the sums); spx_profile_read syncs on them and returns the summed
 * duration and the launch count of one kernel.  Off by default: nothing recorded. */
int spx_profile_enable(int on);
int spx_profile_read(const char *kernel, double *total_ms, int64_t *launches);
/* The large-cluster medoid Gram's MFMA operand encoding of its 0/1 bin rows: 4 = FP4
 * e2m1 (v_mfma_f32_32x32x64_f8f6f4, ~10 POPS dense), 8 = i8 (v_mfma_i32_32x32x32_i8,
 * ~5 POPS dense); the counts are exact either way.  bench.py prices the Gram's MFMA
 * roofline against the peak of the encoding the library was built with. */
int spx_medoid_gram_operand_bits(void);

#ifdef __cplusplus
}
#endif
#endif /* SPECPRIDE_H_ */
