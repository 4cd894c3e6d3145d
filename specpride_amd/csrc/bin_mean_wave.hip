// bin_mean_wave_kernel (SPX_BIN_KERNEL=7, experimental): bin-mean with wave-private
// bin ranges and no per-spectrum barrier (reference: src/binning.py:170-231,
// combine_bin_mean; semantics in SURVEY.md Appendix A.1).
//
// Measured: 4.55 ms vs 2.97 ms for bin_mean_lds_kernel on the bench batch.  The
// binary search of phase 2b is a chain of ~8 dependent global loads per
// cluster, and at ~5 clusters per CU that latency is not hidden; the phase-4
// walk is bin_mean_fast_kernel's slow one.  Kept as a parity-tested variant.
//
// The float32 sums of combine_bin_mean are ORDER-dependent: bin b's
// I = f32(f64(I) + it) runs over the spectra in file order.  bin_mean_lds_kernel
// honours that with one block barrier per spectrum; every step then waits on a
// read-modify-write round trip plus a 4-wave barrier.  Here the order is kept
// without barriers: the cluster's occupied bins are split into 4 contiguous
// ranges, and wave w alone owns range w.  A wave issues its LDS operations in
// program order and the LDS executes one wave's operations in order, so wave w
// walking the spectra in file order IS the reference's accumulation order for
// its bins -- the waves never wait for each other until the output phase.
//
//   phase 1  (flat, all peaks) occupied-bin bitmap in LDS (bin_mean_lds_kernel)
//   phase 2  popcount prefix -> slots in ascending bin order; the bins of slots
//            D/4, D/2, 3D/4 become the range boundaries B1 <= B2 <= B3
//   phase 2b waves 1..3: per spectrum, the first peak whose bin >= B_w
//            (binary search, lane j = spectrum j; spectra are m/z-sorted)
//   phase 3  wave w, spectra in file order: its run of the spectrum, 64 peaks per
//            step, loads prefetched through an 8-deep register ring.  The last
//            peak of each bin in the spectrum (numpy fancy-index "+=" keeps the
//            last, binning.py:197-199; neighbour compare, valid for sorted keys)
//            updates its slot: (I, M) as one float2, ds_read_b64 + ds_write_b64
//   phase 4  kept bins in bin order: count >= int(0.25 n)+1 (binning.py:181-183),
//            mz = f64(M)/count, int = f64(I)/count (binning.py:209-222)
//
// Counts are not stored: every m/z summed into bin b lies in
// [min + b*binsize, min + (b+1)*binsize), so count = round(M / (min + b*binsize))
// exactly while 128*binsize/min + 128^2 * 2^-23 < 0.45 (host-checked: 0.03 for
// the reference's 100 / 0.02; other parameters take bin_mean_lds_kernel).
// Deferred to bin_mean_global_kernel: > 128 spectra, > 65,535 peaks, > BM_WMAX
// bitmap words or > BM_DCAP occupied bins, a key inversion inside a spectrum
// (unsorted m/z) or a NaN m/z.
// HBM traffic: m/z read in phase 1 (phase 2b/3 re-read it from L2/MALL),
// intensity once in phase 3, 16 B per output peak, offsets.
#include "bin_mean.hip"

namespace spx {

constexpr int BW_NMAX = 128;   // spectra per cluster
constexpr int BW_PF = 8;       // spectra in flight per wave (register ring)
constexpr int BW_NW = BM_BLOCK / kWave;

struct BinMeanWaveSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  float2 acc[BM_DCAP];                 // (I, M) per slot
  uint16_t run[BW_NW - 1][BW_NMAX];    // run[w-1][j]: first peak of spectrum j with bin >= B_w (rel. p0)
  int32_t soff[BW_NMAX + 1];           // spectrum offsets relative to the cluster's first peak
  double prec[BW_NMAX];
  int32_t bound[BW_NW];                // B_1..B_3 (bound[0] unused)
  int votes[2 * BW_NW];
  int tmp[BW_NW + 1];
};

// bin key of an m/z: its bin when in range, -1 below the minimum, INT_MAX at or
// above the maximum (and NaN), so keys of a sorted spectrum are non-decreasing
__device__ __forceinline__ int32_t bw_key(double m, const BinMeanParams& P) {
  if (in_range(m, P)) return bin_small(m, P);
  return m < P.minimum ? -1 : 0x7fffffff;
}

// the bit index of the r-th set bit of w (0-based, r < popcount(w))
__device__ __forceinline__ int select_bit(unsigned long long w, int r) {
  for (int i = 0; i < r; ++i) w &= w - 1ull;
  return __ffsll((long long)w) - 1;
}

struct BwPeak {
  double m, it, mn;  // this lane's m/z and intensity; lane 63: the m/z after the chunk
};

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_wave_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                 double* prec_out, int32_t* charge_out,
                                                                 int32_t* status, int32_t* deferred,
                                                                 int32_t* n_deferred) {
  __shared__ BinMeanWaveSmem L;
  const int64_t c = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n = s1 - s0;
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
  if (n > BW_NMAX || p1 - p0 > 0xFFFF || P.n_words > BM_WMAX) { finish(kDeferred); return; }

  for (int j = tid; j <= n; j += BM_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
  for (int j = tid; j < n; j += BM_BLOCK) L.prec[j] = v.prec_mz[s0 + j];
  const int32_t z0 = v.charge[s0];
  int mixed = 0;
  for (int64_t s = s0 + 1 + tid; s < s1; s += BM_BLOCK) mixed |= v.charge[s] != z0;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.bitmap[w] = 0ull;
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 1)) {  // binning.py:205-206
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    finish(kMixedCharge);
    return;
  }

  // phase 1: occupied-bin bitmap (16 independent loads in flight per thread)
  constexpr int U1 = 16;
  for (int64_t k0 = p0 + tid; k0 < p1; k0 += U1 * BM_BLOCK) {
    double m[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int64_t k = k0 + (int64_t)u * BM_BLOCK;
      m[u] = v.mz[k < p1 ? k : p0];
    }
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      if (k0 + (int64_t)u * BM_BLOCK < p1 && in_range(m[u], P)) {
        const int32_t b = bin_small(m[u], P);
        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
      }
    }
  }
  lds_barrier();

  // phase 2: slots in bin order, then the wave range boundaries
  const int D = bitmap_prefix<BM_BLOCK>(L.bitmap, L.wprefix, P.n_words, L.tmp);
  if (D > BM_DCAP) { finish(kDeferred); return; }
  for (int d = tid; d < D; d += BM_BLOCK) L.acc[d] = make_float2(0.0f, 0.0f);
  {
    const int per = (P.n_words + BM_BLOCK - 1) / BM_BLOCK;
    if (tid == 0)
      for (int w = 1; w < BW_NW; ++w) L.bound[w] = 0x7fffffff;  // D == 0: ranges 1..3 empty
    lds_barrier();
    for (int k = 0; k < per; ++k) {
      const int wd = tid * per + k;
      if (wd >= P.n_words) break;
      const unsigned long long bits = L.bitmap[wd];
      const int lo = L.wprefix[wd], cnt = __popcll(bits);
      for (int w = 1; w < BW_NW; ++w) {
        const int r = (w * D) / BW_NW;
        if (r < D && r >= lo && r < lo + cnt) L.bound[w] = wd * 64 + select_bit(bits, r - lo);
      }
    }
  }
  lds_barrier();

  // phase 2b: each wave's first peak per spectrum (wave 0 starts at the spectrum start)
  if (wid > 0) {
    const int32_t B = L.bound[wid];
    for (int j = lane; j < n; j += kWave) {
      int lo = L.soff[j], hi = L.soff[j + 1];
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (bw_key(v.mz[p0 + mid], P) < B) lo = mid + 1;
        else hi = mid;
      }
      L.run[wid - 1][j] = (uint16_t)lo;
    }
  }
  lds_barrier();

  // phase 3: wave-private ordered accumulation
  int bad = 0;
  if (p1 > p0) {
    const double* __restrict__ mzc = v.mz + p0;
    const double* __restrict__ itc = v.inten + p0;
    auto run_a = [&](int j) -> int { return wid == 0 ? L.soff[j] : (int)L.run[wid - 1][j]; };
    auto run_e = [&](int j) -> int { return wid == BW_NW - 1 ? L.soff[j + 1] : (int)L.run[wid][j]; };
    // first chunk of spectrum j's run (j clamped: past-the-end fetches are discarded)
    auto fetch = [&](int j) {
      const int jj = j < n ? j : (int)n - 1;
      const int a = run_a(jj), se = L.soff[jj + 1];
      const int k = a + lane;
      BwPeak q;
      q.m = mzc[k < se ? k : 0];
      q.it = itc[k < se ? k : 0];
      q.mn = (lane == kWave - 1 && k + 1 < se) ? mzc[k + 1] : 0.0;
      return q;
    };
    // one chunk: lanes k = a0 + lane of the run [a0, e) of a spectrum ending at se
    auto chunk = [&](const BwPeak& q, int a0, int e, int se) {
      const int k = a0 + lane;
      const bool active = k < e, has_next = k + 1 < se;
      const int32_t key = bw_key(q.m, P);
      int32_t kn = __shfl_down(key, 1, kWave);
      if (lane == kWave - 1) kn = bw_key(q.mn, P);
      bad |= active && ((q.m != q.m) || (has_next && key > kn));
      if (active && (!has_next || kn != key) && key >= 0 && key != 0x7fffffff) {
        const int slot = bitmap_rank(L.bitmap, L.wprefix, (int64_t)key);
        float2 a = L.acc[slot];
        a.x = (float)((double)a.x + q.it);
        a.y = (float)((double)a.y + q.m);
        L.acc[slot] = a;
      }
    };
    BwPeak R[BW_PF];
#pragma unroll
    for (int j = 0; j < BW_PF; ++j) R[j] = fetch(j);
    for (int jb = 0; jb < n; jb += BW_PF) {
#pragma unroll
      for (int u = 0; u < BW_PF; ++u) {
        const int j = jb + u;
        if (j < n) {  // wave-uniform
          const int a = run_a(j), e = run_e(j), se = L.soff[j + 1];
          bad |= a > e;  // boundaries out of order: an unsorted spectrum
          const BwPeak q = R[u];
          R[u] = fetch(j + BW_PF);
          chunk(q, a, e, se);
          for (int a0 = a + kWave; a0 < e; a0 += kWave) {  // runs longer than a wave
            const int k = a0 + lane;
            BwPeak r;
            r.m = mzc[k < se ? k : 0];
            r.it = itc[k < se ? k : 0];
            r.mn = (lane == kWave - 1 && k + 1 < se) ? mzc[k + 1] : 0.0;
            chunk(r, a0, e, se);
          }
        }
      }
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 0)) { finish(kDeferred); return; }

  // phase 4: kept bins in bin order (each thread: a contiguous run of bitmap words)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (P.n_words + BM_BLOCK - 1) / BM_BLOCK;
  auto kept = [&](int wd, int bit, float2& a, double& cn) {
    a = L.acc[L.wprefix[wd] + __popcll(L.bitmap[wd] & ((1ull << bit) - 1ull))];
    const double lo = P.minimum + (double)(wd * 64 + bit) * P.binsize;
    cn = (double)(uint32_t)((double)a.y / lo + 0.5);
    return cn >= (double)quorum && !isnan(a.x);
  };
  int mine = 0;
  for (int k = 0; k < per; ++k) {
    const int wd = tid * per + k;
    if (wd >= P.n_words) break;
    for (unsigned long long bits = L.bitmap[wd]; bits; bits &= bits - 1ull) {
      float2 a;
      double cn;
      mine += kept(wd, __ffsll((long long)bits) - 1, a, cn);
    }
  }
  int total;
  int o = block_exclusive_scan<BM_BLOCK>(mine, L.tmp, total);
  for (int k = 0; k < per; ++k) {
    const int wd = tid * per + k;
    if (wd >= P.n_words) break;
    for (unsigned long long bits = L.bitmap[wd]; bits; bits &= bits - 1ull) {
      float2 a;
      double cn;
      if (kept(wd, __ffsll((long long)bits) - 1, a, cn)) {
        out.inten[p0 + o] = (double)a.x / cn;
        out.mz[p0 + o] = (double)a.y / cn;
        ++o;
      }
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
