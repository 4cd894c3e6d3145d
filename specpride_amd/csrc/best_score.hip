// Score-based representative: the highest-scoring member of every cluster
// (reference: src/best_spectrum.py:67-100 get_best_representative, driven by
// best_spectrum():151-175; restated in oracle/np_oracle.py best_score).
//
// The reference filters the USI-sorted MaxQuant score Series to the cluster's
// members (:97) and takes idxmax (:100): the FIRST maximum in sorted-USI order,
// NaN scores skipped.  The host folds that join into two per-spectrum arrays:
//   score[s]  max non-NaN PSM score of spectrum s's USI (NaN if all are NaN)
//   rank[s]   position of the USI among the sorted distinct score USIs, or -1
//             when the USI has no PSM (it is not in the filtered Series)
// so the device work is a segmented argmax over (score desc, rank asc).
//
// One wave per cluster: lanes stride over the members, then a shuffle-xor
// reduction of (score, rank, index).  HBM-bound: 16 B per spectrum
// (score + rank) + 8 B cluster offset + 12 B of output per cluster.
#include "spx_device.hpp"

namespace spx {

constexpr int BEST_WAVES = 4;

// (a better than b) under the reference's idxmax order; rank < 0 = no entry
__device__ __forceinline__ bool best_better(double sa, int64_t ra, double sb, int64_t rb) {
  if (ra < 0) return false;
  if (rb < 0) return true;
  const bool na = sa != sa, nb = sb != sb;
  if (na != nb) return nb;          // a real score beats NaN (skipna)
  if (!na && sa != sb) return sa > sb;
  return ra < rb;                   // equal (or both NaN): first in sorted-USI order
}

__global__ __launch_bounds__(BEST_WAVES * kWave) void best_score_kernel(int64_t C, const int64_t* __restrict__ cluster_off,
                                                                       const double* __restrict__ score,
                                                                       const int64_t* __restrict__ rank,
                                                                       int64_t* __restrict__ best,
                                                                       int32_t* __restrict__ status) {
  const int64_t c = (int64_t)blockIdx.x * BEST_WAVES + wave_id();
  if (c >= C) return;  // wave-uniform
  const int lane = lane_id();
  const int64_t s0 = cluster_off[c], s1 = cluster_off[c + 1];
  double bs = 0.0;
  int64_t br = -1, bi = -1;
  for (int64_t s = s0 + lane; s < s1; s += kWave) {
    const int64_t r = rank[s];
    const double v = score[s];
    if (best_better(v, r, bs, br)) { bs = v; br = r; bi = s; }
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const double os = __shfl_xor(bs, o, kWave);
    const int64_t orr = __shfl_xor(br, o, kWave);
    const int64_t oi = __shfl_xor(bi, o, kWave);
    if (best_better(os, orr, bs, br)) { bs = os; br = orr; bi = oi; }
  }
  if (lane == 0) {
    // no PSM for any member: ValueError (:98-99); only NaN scores: pandas'
    // idxmax returns NaN and spectra[nan] raises KeyError
    const int32_t st = br < 0 ? kEmpty : (bs != bs ? kNonFinite : kOk);
    best[c] = st == kOk ? bi : -1;
    status[c] = st;
  }
}

}  // namespace spx
