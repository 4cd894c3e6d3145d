// One pass of the headline step over a cluster: bin-mean consensus AND medoid
// representative (SURVEY.md §8(d) configs[4]: "medoid + binned consensus").
//
// The two register kernels run back to back inside ONE workgroup per cluster:
// bin_mean_reg_path (bin_mean.hip; binning.py:170-231), then medoid_small_body
// (medoid.hip; most_similar_representative.py:13-19, :60-111) over the same
// cluster, their LDS states overlaid (they never live at once).  The bodies and
// their hand-off lists are the separate kernels' own, so every result is
// bit-identical to spx_bin_mean + spx_medoid.
//
// Why fuse: bin-mean streams 16 B per peak and is bound by the traffic it issues;
// the medoid reads 8 B per peak and spends most of its lifetime in LDS-bound
// latency chains (rows, pairs, pairwise sums).  As two kernels, each fills the
// chip alone.  Fused, one CU holds workgroups in both kinds of phases at once,
// and the medoid's m/z read finds the cluster just read by the bin-mean (L2 /
// Infinity Cache) instead of HBM.
#include "bin_mean.hip"
#include "medoid.hip"

namespace spx {

#ifndef SPX_FU_MINW
#define SPX_FU_MINW 5  // waves per SIMD: the bin-mean body's 96 VGPRs
#endif

union FusedSmem {
  BinHeadSmem b;
  MedoidRegSmem<MD_BLOCK, MR_UMAX, MD_KWMAX> m;
};
static_assert(BM_BLOCK == MD_BLOCK, "one workgroup shape for both bodies");

__global__ __launch_bounds__(BM_BLOCK, SPX_FU_MINW) void bin_mean_medoid_kernel(
    CsrView v, BinMeanParams PB, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    StripedList bm_rest, MedoidParams PM, int64_t* rep, double* totals_out, StripedList md_wide) {
  __shared__ FusedSmem L;
  const int64_t c = blockIdx.x;
  // bin-mean first: its phase A streams the cluster's m/z, which the medoid's
  // first pass then re-reads from cache
  const int32_t st = bin_mean_head_path(v, PB, L.b, c, out, prec_out, charge_out);
  if (threadIdx.x == 0) {  // bin_mean_reg_kernel's hand-off, verbatim
    if (st != kNotHere) status[c] = st;
    if (st == kNotHere || st == kDeferred) striped_push(bm_rest, (int32_t)c);
  }
  __syncthreads();  // the bin-mean LDS is dead: the medoid's takes its place
  medoid_small_body<MD_BLOCK, MR_UMAX, MD_KWMAX>(v, PM, rep, totals_out, L.m, c, [&](int64_t cc, int64_t, int) {
    rep[cc] = -4;  // medoid_reg_kernel's hand-off, verbatim
    striped_push(md_wide, (int32_t)cc);
  });
}

// The hand-off counts of one fused pass (spx_bin_mean_medoid_stage, stage 1): the
// clusters each register body left on its list -- out[0] bin-mean (for
// bin_mean_wide_kernel), out[1] medoid (for medoid_wide_kernel).  Both zero: the
// leftover chains (stage 2) have nothing to do for this batch.
__global__ __launch_bounds__(kWave) void handoff_count_kernel(const int32_t* bm_counts, const int32_t* md_counts,
                                                              int32_t* out) {
  const int l = threadIdx.x;
  const int32_t a = wave_sum(bm_counts[l * kListLine]);
  const int32_t b = wave_sum(md_counts[l * kListLine]);
  if (l == 0) {
    out[0] = a;
    out[1] = b;
  }
}

}  // namespace spx
