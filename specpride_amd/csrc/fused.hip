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
// chip alone.  Fused, one CU holds workgroups in both kinds of phases at once.
// Since round 6 the pass reads each m/z ONCE for both methods: the bin-mean's phase
// A computes the medoid's ceil(mz/tol) bin beside its own from the same load and
// phase B ranks it, so the medoid's bit rows come from registers (medoid_from_codes)
// and its own m/z pass, offsets search and flat-layout bookkeeping are gone for every
// cluster the register path completes.
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

// The medoid of a cluster the fused register path has binned (bin_mean_reg_path_t<true>
// returned kOk with every medoid bin inside [0, 32,768)): the codes hold this lane's
// peak of spectrum j -- peak 63 * wave + lane, lanes 0..62 own one each -- as its
// medoid column (the rank of ceil(mz/tol) among the cluster's occupied medoid bins),
// two spectra's columns per register after phase C.  P3 sets each spectrum's bit row straight from those registers
// (the spectrum of a peak is its step j: no offsets search), then medoid_tail runs
// P4..P6 exactly as medoid_small_body does, so rep and totals are the same bits
// (most_similar_representative.py:13-19, :60-111).  K > 64 * MD_KWMAX columns hands the
// cluster on as the register kernel would.
template <class Defer>
__device__ __forceinline__ void medoid_from_codes(const CsrView& v, int64_t* rep, double* totals_out,
                                                  MedoidRegSmem<MD_BLOCK, MR_UMAX, MD_KWMAX>& L, int64_t c,
                                                  const int32_t (&code)[BR_NMAX], const MdSide& md,
                                                  const Defer& defer) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c];
  const int n = (int)(v.cluster_off[c + 1] - s0);
  if (n <= 1) {
    if (tid == 0) {
      rep[c] = n == 1 ? s0 : -1;
      if (totals_out && n == 1) totals_out[s0] = 0.0;
    }
    return;
  }
  const int KW = ((md.K + 63) / 64) | 1;  // odd row stride, as medoid_small_body's
  if (KW > MD_KWMAX) {
    if (tid == 0) defer(c, s0, n);
    return;
  }
  // spectrum offsets (lane j < n: spectrum j's start; lane n: spectrum n-1's end)
  if (tid <= n) L.soff[tid] = tid < n ? md.rlo : md.rhi;
  for (int w = tid; w < n * KW; w += MD_BLOCK) L.u.a.rows[w] = 0ull;
  __syncthreads();
  const uint32_t swz_nw = 2u * (uint32_t)KW;  // 32-bit words per row
  const uint32_t swz_m = swz_nw >= 32u ? 31u : (1u << (31 - __clz((int)swz_nw))) - 1u;  // 2^k - 1 < swz_nw
  const int fpos = wid * (kWave - 1) + lane;
  const bool owner = lane < kWave - 1;
  reg_steps(n, [&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    const int len = __builtin_amdgcn_readlane(md.rhi, j) - __builtin_amdgcn_readlane(md.rlo, j);
    if (owner & (fpos < len)) {
      // phase C packed the columns of spectra 2k, 2k+1 into code[2k] (low, high half);
      // a last even spectrum (n odd) keeps its (slot, column) code
      uint32_t col;
      if constexpr (j & 1) col = (uint32_t)code[j - 1] >> 16;
      else col = j + 1 < n ? (uint32_t)code[j] & 0xFFFFu : (uint32_t)code[j] >> 16;
      // the register kernel's P3 word swizzle (a bijection per bit position)
      uint32_t wq = (col >> 5) + (col & swz_m);
      wq = min(wq, wq - swz_nw);
      atomicOr(reinterpret_cast<uint32_t*>(&L.u.a.rows[__mul24(j, KW)]) + wq, 1u << (col & 31));
    }
  });
  SPX_STAMP2(-1, 5);
  medoid_tail<MD_BLOCK, MR_UMAX, MD_KWMAX>(L, n, KW, s0, c, rep, totals_out);
}

__global__ __launch_bounds__(BM_BLOCK, SPX_FU_MINW) void bin_mean_medoid_kernel(
    CsrView v, BinMeanParams PB, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    StripedList bm_rest, MedoidParams PM, int64_t* rep, double* totals_out, StripedList md_wide) {
  __shared__ FusedSmem L;
  const int64_t c = blockIdx.x;
  SPX_STAMP2(-1, 0);
  // bin-mean first: its phase A reads each m/z once for BOTH methods' bins
  int32_t code[BR_NMAX];
  MdSide md{PM.tol, PM.inv_tol, 1, 0, 0, 0};
  const int32_t st = bin_mean_reg_path_t<true>(v, PB, L.b, c, out, prec_out, charge_out, code, &md);
  if (threadIdx.x == 0) {  // bin_mean_reg_kernel's hand-off, verbatim
    if (st != kNotHere) status[c] = st;
    if (st == kNotHere || st == kDeferred) striped_push(bm_rest, (int32_t)c);
  }
  SPX_STAMP2(-1, 4);
  __syncthreads();  // the bin-mean LDS is dead: the medoid's takes its place
  auto defer = [&](int64_t cc, int64_t, int) {
    rep[cc] = -4;  // medoid_reg_kernel's hand-off, verbatim
    striped_push(md_wide, (int32_t)cc);
  };
  if (st == kOk && !md.out) {  // uniform
    medoid_from_codes(v, rep, totals_out, L.m, c, code, md, defer);
  } else {
    // the register path stopped before its codes were complete (more than 50 spectra,
    // a long / unsorted / NaN spectrum, mixed charges, > 1,536 bins) or a medoid bin is
    // out of its range: the medoid's own body, which reads the m/z itself
    medoid_small_body<MD_BLOCK, MR_UMAX, MD_KWMAX>(v, PM, rep, totals_out, L.m, c, defer);
  }
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
