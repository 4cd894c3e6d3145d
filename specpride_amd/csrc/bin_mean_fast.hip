// bin_mean_fast_kernel (SPX_BIN_KERNEL=8, experimental; reference: src/binning.py:170-231,
// combine_bin_mean; semantics in SURVEY.md Appendix A.1) -- bin_mean_lds_kernel's
// algorithm with the per-peak VALU work cut down.
//
// Measured (profiles/r01_v9_phases.json): 3.99 ms vs 2.99 ms for
// bin_mean_lds_kernel on the bench batch -- phase 3 2.26 vs 1.93 ms (fewer VALU
// instructions, but 64-bit LDS read-modify-writes and the lane-63 loads lengthen
// the per-spectrum chain) and phase 4 1.27 vs 0.26 ms (divergent per-word
// walk with a divide per kept bin).  Kept as a parity-tested variant.
//
// Profiling bin_mean_lds_kernel (rocprofv3 --pmc, profiles/r01_v7_pmc_summary.txt)
// showed it VALU-issue bound, not HBM- or latency-bound: ~2.1 wave64 VALU
// instructions per peak against ~1 wave-instruction per clock per CU, and a
// deeper register ring did not move it.  This kernel keeps the same phases
// and the same spectrum-ordered float32 fold, and removes instructions:
//   * every peak load is a buffer_load through a per-cluster descriptor
//     (base = the cluster's first peak, range = its peaks): the per-lane
//     voffset is a constant, the spectrum start goes in soffset (an SGPR), so
//     addressing costs no VALU; lanes past the cluster read 0.0 (hardware
//     range check), which is below the minimum and so never binned
//   * (I, M) accumulate as one float2 (ds_read_b64 / ds_write_b64) and the
//     count is not stored: every m/z summed into bin b lies in
//     [min + b*binsize, min + (b+1)*binsize), so count = round(M / (min + b*binsize))
//     exactly while 128*binsize/min + 128^2 * 2^-23 < 0.45 (host-checked, 0.03 for
//     the reference's 100 / 0.02; other parameters run bin_mean_lds_kernel)
//   * a wave's lane 63 loads its successor peak itself (one exec-masked load)
//     instead of exchanging keys between waves through LDS
// Phases: 1 occupied-bin bitmap (flat over the cluster's peaks), 2 popcount
// prefix -> slots in bin order, 3 spectra in file order (lane t = peak t; the
// last peak of each bin in the spectrum -- numpy fancy-index "+=" keeps the
// last, binning.py:197-199 -- updates its slot; slots of spectrum j are looked
// up while spectrum j-1's updates drain; one LDS-only barrier per spectrum),
// 4 kept bins (count >= int(0.25 n)+1, binning.py:181-183) in bin order.
// Deferred to bin_mean_global_kernel: > 128 spectra, a spectrum longer than
// 256 peaks, > 65,535 peaks, > BM_WMAX bitmap words or > BM_DCAP occupied bins,
// a key inversion inside a spectrum (unsorted m/z) or a NaN m/z.
#include "bin_mean.hip"

namespace spx {

constexpr int BF8_NMAX = 128;
#ifndef SPX_BF8_PF
#define SPX_BF8_PF 8
#endif
constexpr int BF8_PF = SPX_BF8_PF;  // spectra in flight per thread (rolling register ring)

struct BinMeanFastSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  float2 acc[BM_DCAP];  // (I, M) per slot
  int32_t soff[BF8_NMAX + 1];
  double prec[BF8_NMAX];
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

// bin key: the bin when in range, -1 below the minimum, INT_MAX at/above the
// maximum (and NaN): non-decreasing along a sorted spectrum
__device__ __forceinline__ int32_t bf_key(double m, const BinMeanParams& P) {
  if (in_range(m, P)) return bin_small(m, P);
  return m < P.minimum ? -1 : 0x7fffffff;
}

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_fast_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                 double* prec_out, int32_t* charge_out,
                                                                 int32_t* status, int32_t* deferred,
                                                                 int32_t* n_deferred) {
  __shared__ BinMeanFastSmem L;
  const int64_t c = blockIdx.x;
  const int tid = threadIdx.x, lane = lane_id();
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
  if (n > BF8_NMAX || p1 - p0 > 0xFFFF || P.n_words > BM_WMAX) { finish(kDeferred); return; }
  const int np = (int)(p1 - p0);
  // per-cluster descriptors from wave-uniform values only (no waterfall loops)
  const __amdgpu_buffer_rsrc_t rmz = bf_rsrc(v.mz + p0, np);
  const __amdgpu_buffer_rsrc_t rit = bf_rsrc(v.inten + p0, np);

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

  // phase 1: occupied-bin bitmap; 16 loads in flight per thread, out-of-range
  // lanes read 0.0 (< minimum) and drop out with the range test
  constexpr int U1 = 16;
  int irregular = 0;  // a spectrum longer than the block: generic kernel
  for (int j = tid; j < n; j += BM_BLOCK) irregular |= (L.soff[j + 1] - L.soff[j]) > BM_BLOCK;
  for (int k0 = 0; k0 < np; k0 += U1 * BM_BLOCK) {
    double m[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) m[u] = bf_load(rmz, tid * 8, (k0 + u * BM_BLOCK) * 8);
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      if (in_range(m[u], P)) {
        const int32_t b = bin_small(m[u], P);
        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
      }
    }
  }
  if (block_any<BM_BLOCK, true>(irregular, L.votes, 0)) { finish(kDeferred); return; }

  // phase 2: compact slots in bin order
  const int D = bitmap_prefix<BM_BLOCK>(L.bitmap, L.wprefix, P.n_words, L.tmp);
  if (D > BM_DCAP) { finish(kDeferred); return; }
  for (int d = tid; d < D; d += BM_BLOCK) L.acc[d] = make_float2(0.0f, 0.0f);
  lds_barrier();

  // phase 3: spectra in file order, lane t = peak t, software-pipelined by one
  // spectrum: step j looks up spectrum j's slots while spectrum j-1's update runs
  int bad = 0;
  if (!(P.ablate & 1)) {  // (profiling: SPX_ABLATE=1 skips phase 3)
    struct Pk { double m, it, mn; };
    const int vo = tid * 8;
    auto fetch = [&](int j) {
      const int so = __builtin_amdgcn_readfirstlane(L.soff[j < n ? j : (int)n - 1] * 8);
      Pk q;
      q.m = bf_load(rmz, vo, so);
      q.it = bf_load(rit, vo, so);
      q.mn = lane == kWave - 1 ? bf_load(rmz, vo + 8, so) : 0.0;
      return q;
    };
    Pk R[BF8_PF];
#pragma unroll
    for (int j = 0; j < BF8_PF; ++j) R[j] = fetch(j);
    int pslot = -1;  // spectrum j-1's pending update
    double pm = 0.0, pit = 0.0;
    for (int jb = 0; jb < n; jb += BF8_PF) {
#pragma unroll
      for (int u = 0; u < BF8_PF; ++u) {
        const int j = jb + u;
        if (j < n) {  // uniform
          const int len = L.soff[j + 1] - L.soff[j];
          const Pk q = R[u];
          R[u] = fetch(j + BF8_PF);
          const bool active = tid < len, has_next = tid + 1 < len;
          const int32_t key = bf_key(q.m, P);
          int32_t kn = __shfl_down(key, 1, kWave);
          if (lane == kWave - 1) kn = bf_key(q.mn, P);
          bad |= active && ((q.m != q.m) || (has_next && key > kn));
          int slot = -1;
          if (active && (!has_next || kn != key) && key >= 0 && key != 0x7fffffff)
            slot = bitmap_rank(L.bitmap, L.wprefix, (int64_t)key);
          if (pslot >= 0) {
            float2 a = L.acc[pslot];
            a.x = (float)((double)a.x + pit);
            a.y = (float)((double)a.y + pm);
            L.acc[pslot] = a;
          }
          lds_barrier();
          pslot = slot;
          pm = q.m;
          pit = q.it;
        }
      }
    }
    if (pslot >= 0) {
      float2 a = L.acc[pslot];
      a.x = (float)((double)a.x + pit);
      a.y = (float)((double)a.y + pm);
      L.acc[pslot] = a;
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 1)) { finish(kDeferred); return; }

  if (P.ablate & 2) {  // (profiling: SPX_ABLATE=2 skips phase 4)
    if (tid == 0) out.count[c] = 0;
    finish(kOk);
    return;
  }
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
