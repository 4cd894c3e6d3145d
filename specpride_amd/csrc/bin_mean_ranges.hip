// bin_mean_ranges_kernel (SPX_BIN_KERNEL=9, experimental): bin-mean with wave-private
// bin ranges, the run boundaries found in the flat first pass (reference:
// src/binning.py:170-231, combine_bin_mean; semantics in SURVEY.md Appendix A.1).
//
// Measured: 4.78 ms vs 2.97 ms for bin_mean_lds_kernel on the bench batch.  Without
// the binary search of variant 7 and without any per-spectrum barrier it is still
// slower: each wave walks all n spectra itself, and every step carries more LDS
// round trips (run bounds, offsets, rank, read-modify-write) than variant 0's,
// so the per-step LDS chain -- not the barrier -- is what bounds the fold.
// Kept as a parity-tested variant.
//
// bin_mean_wave_kernel (variant 7) showed that wave-private bin ranges keep the
// reference's spectrum-ordered float32 fold without a per-spectrum barrier (a
// wave's LDS operations execute in program order), but it found each wave's
// run of each spectrum by a binary search -- ~8 dependent global loads per
// cluster.  Here the boundaries B1 <= B2 <= B3 are fixed BEFORE the first pass
// (the bins of spectrum 0's quartile peaks, so the ranges follow the cluster's
// m/z distribution), and the first pass, which already computes every peak's
// bin, also records where each spectrum's bins cross each boundary:
//   prologue  offsets, precursors, charge check; B_w from spectrum 0; a bitmap of
//             spectrum-start positions
//   phase 1   flat, coalesced: bin key of every peak, occupied-bin bitmap; the
//             previous peak's key (shuffle; lane 0 loads its predecessor) and the
//             start bit give the crossings prev < B_w <= key, stored as
//             run[w][j] = offset in spectrum j (j by a search over the offsets,
//             ~3 crossings per spectrum)
//   phase 2   popcount prefix -> slots in bin order; counters zeroed
//   phase 3   wave w walks the spectra in file order over its run [run[w-1][j],
//             run[w][j]) -- the last peak of each bin in the spectrum (numpy
//             fancy-index "+=" keeps the last, binning.py:197-199) updates its
//             slot (count, then I = f32(f64(I)+it), M = f32(f64(M)+mz)); no
//             barrier until the output phase
//   phase 4   bin_mean_lds_kernel's: kept slots (count >= int(0.25 n)+1) in bin
//             order, means, np.mean of the precursors
// A key inversion inside a spectrum (unsorted m/z; the crossings are then not a
// partition) or a NaN m/z defers the cluster to bin_mean_global_kernel, as do
// > 128 spectra, a spectrum longer than 255 peaks, > 12,288 peaks, > BM_WMAX
// bitmap words and > BM_DCAP occupied bins.
#include "bin_mean.hip"

namespace spx {

constexpr int BR_NMAX = 128;                 // spectra per cluster
constexpr int BR_PMAX = 12288;               // peaks per cluster (start bitmap)
constexpr int BR_SMAX = 255;                 // peaks per spectrum (u8 run offsets)
constexpr int BR_NW = BM_BLOCK / kWave;      // waves = ranges
constexpr int BR_PF = 8;                     // spectra in flight per wave (phase 3 ring)

struct BinMeanRangesSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  uint8_t cnt[BM_DCAP];                      // <= 128 spectra per slot
  float acc_i[BM_DCAP];
  float acc_m[BM_DCAP];
  unsigned long long sbits[BR_PMAX / 64];    // bit r: a spectrum starts at peak r
  uint8_t run[BR_NW - 1][BR_NMAX];           // run[w-1][j]: first peak of spectrum j with key >= B_w
  int32_t soff[BR_NMAX + 1];
  double prec[BR_NMAX];
  int32_t bound[BR_NW];
  int votes[2 * BR_NW];
  int tmp[BR_NW + 1];
};

__device__ __forceinline__ int32_t br_key(double m, const BinMeanParams& P) {
  if (in_range(m, P)) return bin_small(m, P);
  return m < P.minimum ? -1 : 0x7fffffff;
}

// last spectrum j with soff[j] <= r (the one holding peak r; empty spectra skipped)
__device__ __forceinline__ int br_spectrum_of(const int32_t* soff, int n, int r) {
  int lo = 0, hi = n;  // soff[lo] <= r < soff[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (soff[mid] <= r) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_ranges_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                   double* prec_out, int32_t* charge_out,
                                                                   int32_t* status, int32_t* deferred,
                                                                   int32_t* n_deferred) {
  __shared__ BinMeanRangesSmem L;
  const int64_t c = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  auto finish = [&](int32_t st) {
    if (tid == 0) {
      status[c] = st;
      if (st == kDeferred) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
  };
  if (n == 0) {
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    finish(kEmpty);
    return;
  }
  if (s1 - s0 > BR_NMAX || p1 - p0 > BR_PMAX || P.n_words > BM_WMAX) { finish(kDeferred); return; }
  const int np = (int)(p1 - p0);
  const char* __restrict__ mzb = reinterpret_cast<const char*>(v.mz + p0);
  const char* __restrict__ itb = reinterpret_cast<const char*>(v.inten + p0);
  auto ld = [](const char* base, int r) { return *reinterpret_cast<const double*>(base + (uint32_t)r * 8u); };

  // prologue
  for (int j = tid; j <= n; j += BM_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
  for (int j = tid; j < n; j += BM_BLOCK) L.prec[j] = v.prec_mz[s0 + j];
  const int32_t z0 = v.charge[s0];
  int mixed = 0;
  for (int64_t s = s0 + 1 + tid; s < s1; s += BM_BLOCK) mixed |= v.charge[s] != z0;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.bitmap[w] = 0ull;
  for (int w = tid; w < (np + 63) / 64; w += BM_BLOCK) L.sbits[w] = 0ull;
  if (tid >= 1 && tid < BR_NW) {  // B_w: the key of spectrum 0's peak at w/4 of its length
    const int len0 = (int)(v.spec_off[s0 + 1] - p0);
    L.bound[tid] = len0 > 0 ? br_key(ld(mzb, (tid * len0) / BR_NW), P) : 0x7fffffff;
  }
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 1)) {  // binning.py:205-206
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    finish(kMixedCharge);
    return;
  }
  int irregular = 0;  // a spectrum longer than BR_SMAX
  for (int j = tid; j < n; j += BM_BLOCK) {
    const int a = L.soff[j], e = L.soff[j + 1];
    irregular |= e - a > BR_SMAX;
    if (a < e) atomicOr(&L.sbits[a >> 6], 1ull << (a & 63));
    L.run[0][j] = (uint8_t)(e - a);  // no crossing: the range's run is empty (at the end)
    L.run[1][j] = (uint8_t)(e - a);
    L.run[2][j] = (uint8_t)(e - a);
  }
  if (tid == 0) {  // sort B1 <= B2 <= B3 (spectrum 0 may be unsorted)
    int32_t b1 = L.bound[1], b2 = L.bound[2], b3 = L.bound[3], t;
    if (b1 > b2) { t = b1; b1 = b2; b2 = t; }
    if (b2 > b3) { t = b2; b2 = b3; b3 = t; }
    if (b1 > b2) { t = b1; b1 = b2; b2 = t; }
    L.bound[1] = b1; L.bound[2] = b2; L.bound[3] = b3;
  }
  if (block_any<BM_BLOCK, true>(irregular, L.votes, 0)) { finish(kDeferred); return; }
  const int32_t B1 = L.bound[1], B2 = L.bound[2], B3 = L.bound[3];

  // phase 1: bitmap + run boundaries (8 m/z loads in flight per thread, plus lane 0's predecessors)
  constexpr int U1 = 8;
  for (int r0 = tid; r0 < np; r0 += U1 * BM_BLOCK) {
    double m[U1], mp[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int r = r0 + u * BM_BLOCK;
      m[u] = ld(mzb, r < np ? r : 0);
      mp[u] = (lane == 0 && r > 0 && r < np) ? ld(mzb, r - 1) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int r = r0 + u * BM_BLOCK;
      if (r - lane >= np) break;  // wave-uniform: the rest of the batch is past the cluster
      const bool valid = r < np;
      const int32_t key = valid ? br_key(m[u], P) : 0x7fffffff;
      int32_t kp = __shfl_up(key, 1, kWave);
      if (lane == 0) kp = r > 0 ? br_key(mp[u], P) : -2;
      const unsigned long long sw = L.sbits[(r - lane) >> 6];  // this wave's 64 positions
      if (valid && ((sw >> lane) & 1ull)) kp = -2;             // a spectrum starts here
      if (valid && key >= 0 && key != 0x7fffffff) atomicOr(&L.bitmap[key >> 6], 1ull << (key & 63));
      const bool x1 = valid && kp < B1 && key >= B1, x2 = valid && kp < B2 && key >= B2,
                 x3 = valid && kp < B3 && key >= B3;
      if (x1 || x2 || x3) {
        const int j = br_spectrum_of(L.soff, n, r);
        const uint8_t off = (uint8_t)(r - L.soff[j]);
        if (x1) L.run[0][j] = off;
        if (x2) L.run[1][j] = off;
        if (x3) L.run[2][j] = off;
      }
    }
  }
  lds_barrier();

  // phase 2: compact slots in bin order
  const int D = bitmap_prefix<BM_BLOCK>(L.bitmap, L.wprefix, P.n_words, L.tmp);
  if (D > BM_DCAP) { finish(kDeferred); return; }
  for (int d = tid; d < D; d += BM_BLOCK) {
    L.cnt[d] = 0;
    L.acc_i[d] = 0.0f;
    L.acc_m[d] = 0.0f;
  }
  lds_barrier();

  // phase 3: wave-private ordered accumulation
  int bad = 0;
  if (np > 0) {
    struct Pk { double m, it, mn; };
    auto run_a = [&](int j) -> int { return wid == 0 ? 0 : (int)L.run[wid - 1][j]; };
    auto run_e = [&](int j) -> int { return wid == BR_NW - 1 ? L.soff[j + 1] - L.soff[j] : (int)L.run[wid][j]; };
    auto fetch = [&](int j) {  // first chunk of spectrum j's run (j clamped)
      const int jj = j < n ? j : n - 1;
      const int sa = L.soff[jj], se = L.soff[jj + 1];
      const int k = sa + run_a(jj) + lane;
      Pk q;
      q.m = ld(mzb, k < se ? k : 0);
      q.it = ld(itb, k < se ? k : 0);
      q.mn = (lane == kWave - 1 && k + 1 < se) ? ld(mzb, k + 1) : 0.0;
      return q;
    };
    // one chunk: lane l = peak a0 + l of the spectrum (offsets relative to its start sa)
    auto chunk = [&](const Pk& q, int a0, int e, int len) {
      const int t = a0 + lane;
      const bool active = t < e, has_next = t + 1 < len;
      const int32_t key = br_key(q.m, P);
      int32_t kn = __shfl_down(key, 1, kWave);
      if (lane == kWave - 1) kn = br_key(q.mn, P);
      bad |= active && ((q.m != q.m) || (has_next && key > kn));
      if (active && (!has_next || kn != key) && key >= 0 && key != 0x7fffffff) {
        const int slot = bitmap_rank(L.bitmap, L.wprefix, (int64_t)key);
        L.cnt[slot] = (uint8_t)(L.cnt[slot] + 1);
        L.acc_i[slot] = (float)((double)L.acc_i[slot] + q.it);
        L.acc_m[slot] = (float)((double)L.acc_m[slot] + q.m);
      }
    };
    Pk R[BR_PF];
#pragma unroll
    for (int j = 0; j < BR_PF; ++j) R[j] = fetch(j);
    for (int jb = 0; jb < n; jb += BR_PF) {
#pragma unroll
      for (int u = 0; u < BR_PF; ++u) {
        const int j = jb + u;
        if (j < n) {  // wave-uniform
          const int sa = L.soff[j], len = L.soff[j + 1] - sa;
          const int a = run_a(j), e = run_e(j);
          bad |= a > e;  // crossings out of order: an unsorted spectrum
          const Pk q = R[u];
          R[u] = fetch(j + BR_PF);
          chunk(q, a, e, len);
          for (int a0 = a + kWave; a0 < e; a0 += kWave) {  // runs longer than a wave
            const int k = sa + a0 + lane;
            Pk r;
            r.m = ld(mzb, k < sa + len ? k : 0);
            r.it = ld(itb, k < sa + len ? k : 0);
            r.mn = (lane == kWave - 1 && k + 1 < sa + len) ? ld(mzb, k + 1) : 0.0;
            chunk(r, a0, e, len);
          }
        }
      }
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 1)) { finish(kDeferred); return; }

  // phase 4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (D + BM_BLOCK - 1) / BM_BLOCK;
  const int d0 = tid * per;
  int mine = 0;
  for (int q = 0; q < per; ++q) {
    const int d = d0 + q;
    if (d < D && L.cnt[d] >= quorum && !isnan(L.acc_i[d])) ++mine;
  }
  int total;
  int o = block_exclusive_scan<BM_BLOCK>(mine, L.tmp, total);
  for (int q = 0; q < per; ++q) {
    const int d = d0 + q;
    if (d < D && L.cnt[d] >= quorum) {
      const double cn = (double)L.cnt[d];
      const double mi = (double)L.acc_i[d] / cn;
      if (isnan(mi)) continue;
      out.inten[p0 + o] = mi;
      out.mz[p0 + o] = L.acc_m[d] == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)L.acc_m[d] / cn;
      ++o;
    }
  }
  if (tid == 0) {
    out.count[c] = total;
    charge_out[c] = z0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return L.prec[j]; }, n) / (double)n;  // np.mean, binning.py:224
  }
  finish(kOk);
}

}  // namespace spx
