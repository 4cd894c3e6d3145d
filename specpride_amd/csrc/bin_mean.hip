// Segmented bin-mean consensus (reference: src/binning.py:170-231, combine_bin_mean;
// exact semantics restated in SURVEY.md Appendix A.1 and oracle/np_oracle.py).
//
// One 256-thread workgroup (4 waves) per cluster.  The reference's dense
// 95,001-bin float32 histogram does not fit LDS, so the cluster is processed
// as a sparse, *ordered* histogram:
//
//   phase 1  (all peaks in parallel)  mark every occupied bin in an LDS bitmap
//            (1 bit per bin, 95,001 bins = 11.9 KB; ds_or_b64)
//   phase 2  exclusive popcount prefix per 64-bit word -> each occupied bin gets a
//            compact slot id in ASCENDING bin order (D slots, D << #bins)
//   phase 3  spectra in file order, peaks of one spectrum in parallel: the last
//            peak of the spectrum in each bin (numpy fancy-index "+=" keeps the
//            last, binning.py:197-199) updates its slot:
//               cnt += 1;  I = f32(f64(I) + inten);  M = f32(f64(M) + mz)
//            Spectrum order is the reference's float32 accumulation order, so the
//            result is bit-exact; a barrier separates consecutive spectra.
//            "Last in bin" is a neighbour compare for m/z-sorted spectra (the
//            MGF norm); an unsorted spectrum (voted block-wide) takes an
//            owner-tag path (LDS atomicMax of the peak position per slot).
//   phase 4  slots with cnt >= int(0.25 n)+1 and a non-NaN mean are written in
//            slot (= bin) order: mz = f64(M)/cnt, int = f64(I)/cnt.
//
// Bins are trunc(fl((mz - min)/binsize)) computed exactly (spx_device.hpp).
// Clusters that do not fit the LDS budget (bins, distinct bins, > 128 spectra)
// are appended to a deferred list and finished by bin_mean_global_kernel, the
// same body with its state in a per-workgroup global scratch slice.
//
// HBM traffic per cluster: mz + inten once from HBM (16 B/peak; phase 3 re-reads
// the m/z that phase 1 pulled into L2/MALL), 16 B per output peak, offsets.
#pragma once
#include <utility>

#include "spx_device.hpp"

namespace spx {

struct BinMeanParams {
  double minimum, maximum, binsize, inv_binsize;
  int32_t apply_quorum;
  int32_t n_words;  // ceil(n_bins / 64)
};

template <class PrefixT, class CountT = uint32_t>
struct BinMeanState {
  unsigned long long* bitmap;
  PrefixT* wprefix;
  CountT* cnt;
  float* acc_i;
  float* acc_m;
  uint32_t* owner;
  int32_t* soff;  // LDS copy of the spectrum offsets (nullptr: read spec_off)
  double* prec;   // LDS copy of the precursor m/z (nullptr: read prec_mz)
  int* votes;
  int32_t* xch;
  int dcap;
  int nmax;  // clusters with more spectra are deferred (leaf-only pairwise mean)
};

#ifndef SPX_BM_MINW
#define SPX_BM_MINW 4  // __launch_bounds__ minimum waves per SIMD for bin_mean_lds_kernel (the leftovers)
#endif
#ifndef SPX_BR_MINW
#define SPX_BR_MINW 5  // the same for bin_mean_reg_kernel (50 register codes)
#endif
#ifndef SPX_BM_PF
#define SPX_BM_PF 10  // spectra in flight per thread in the fast path's register ring
#endif

constexpr int BM_BLOCK = 256;
// fast path: wave w's lanes 0..62 own peaks 63w..63w+62 of the spectrum; lane 63
// loads peak 63w+63 (owned by wave w+1's lane 0) only to hand lane 62 its key
constexpr int BM_FASTLEN = 4 * 63;
constexpr int BM_WMAX = 1536;  // 98,304 bins
constexpr int BM_DCAP = 1536;  // distinct occupied bins per cluster
constexpr int BM_NMAX = 128;

struct BinMeanSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  uint16_t cnt[BM_DCAP];       // <= BM_NMAX spectra per slot
  float acc_i[BM_DCAP];
  float acc_m[BM_DCAP];
  double prec[BM_NMAX];       // precursor m/z (np.mean at the end, from LDS)
  int32_t soff[BM_NMAX + 1];  // the cluster's spectrum offsets, relative to its first peak
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
  int flag;
};

struct PeakLane {
  double m, it, mn;  // m/z, intensity, m/z of the next peak in the spectrum
  bool active, has_next;
};

__device__ __forceinline__ bool in_range(double m, const BinMeanParams& P) {
  return m >= P.minimum && m < P.maximum;
}

__device__ __forceinline__ int64_t bin_of(double m, const BinMeanParams& P) {
  return trunc_div_exact(m - P.minimum, P.binsize, P.inv_binsize);
}

// the LDS paths cap the bin count at 64 * BM_WMAX < 2^17: the cheap exact form applies
__device__ __forceinline__ int32_t bin_small(double m, const BinMeanParams& P) {
  return trunc_div_small(m - P.minimum, P.binsize, P.inv_binsize);
}

__device__ __forceinline__ PeakLane load_lane(const CsrView& v, int64_t k, int64_t e) {
  PeakLane L;
  L.active = k < e;
  L.has_next = k + 1 < e;
  L.m = L.active ? v.mz[k] : 0.0;
  L.it = L.active ? v.inten[k] : 0.0;
  L.mn = L.has_next ? v.mz[k + 1] : 0.0;
  return L;
}

template <class PrefixT, class CountT>
__device__ __forceinline__ void accumulate(const BinMeanState<PrefixT, CountT>& S, int slot, double m, double it) {
  S.cnt[slot] += (CountT)1;
  S.acc_i[slot] = (float)((double)S.acc_i[slot] + it);
  S.acc_m[slot] = (float)((double)S.acc_m[slot] + m);
}

// Processes one spectrum chunk lane on the sorted path.
template <class PrefixT, class CountT>
__device__ __forceinline__ void sorted_lane(const BinMeanState<PrefixT, CountT>& S, const BinMeanParams& P,
                                            const PeakLane& L) {
  if (!L.active || !in_range(L.m, P)) return;
  const int64_t b = bin_of(L.m, P);
  if (L.has_next && in_range(L.mn, P) && bin_of(L.mn, P) == b) return;  // a later peak owns the bin
  accumulate(S, bitmap_rank(S.bitmap, S.wprefix, b), L.m, L.it);
}

// Phase 4 of the LDS paths: slots with cnt >= quorum and a non-NaN mean, written
// in slot (= bin) order as mz = f64(M)/cnt, int = f64(I)/cnt (binning.py:209-222).
// Slots are striped over the block (slot j*256 + tid): conflict-free LDS reads and
// coalesced stores.  A slot's output position = kept slots before it = kept in
// earlier stripes + kept in earlier waves of its stripe + earlier lanes of its wave
// (ballot).  Per-(stripe, wave) counts go to `wcnt` (the dead bitmap): one barrier.
// Returns the number of peaks written.
template <int BLOCK = BM_BLOCK, class Cnt, class AccI, class AccM>
__device__ __forceinline__ int emit_striped_f(const Cnt& cnt, const AccI& acc_i, const AccM& acc_m, int* wcnt,
                                              int D, uint32_t quorum, double* __restrict__ omz,
                                              double* __restrict__ oint) {
  constexpr int NW = BLOCK / kWave;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int per = (D + BLOCK - 1) / BLOCK;  // <= 32 stripes
  const unsigned long long below = (1ull << lane) - 1ull;
  uint32_t keep = 0u;  // bit j: slot j*256 + tid is emitted
  for (int j = 0; j < per; ++j) {
    const int d = j * BLOCK + tid;
    const bool k = d < D && (uint32_t)cnt(d) >= quorum && !isnan(acc_i(d));  // cnt >= 1: mean NaN iff sum NaN
    const unsigned long long b = __ballot(k);
    if (lane == 0) wcnt[j * NW + wid] = __popcll(b);
    keep |= (uint32_t)k << j;
  }
  lds_barrier();
  int base = 0;
  for (int j = 0; j < per; ++j) {
    int tot = 0, before = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const int x = wcnt[j * NW + w];
      tot += x;
      before += w < wid ? x : 0;
    }
    const bool k = (keep >> j) & 1u;
    const unsigned long long b = __ballot(k);
    if (k) {
      const int d = j * BLOCK + tid;
      const int o = base + before + __popcll(b & below);
      const double cn = (double)cnt(d);
      const float si = acc_i(d), sm = acc_m(d);
      oint[o] = (double)si / cn;
      omz[o] = sm == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)sm / cn;
    }
    base += tot;
  }
  return base;
}
template <int BLOCK = BM_BLOCK, class CountT, class AccI, class AccM>
__device__ __forceinline__ int emit_striped(const CountT* cnt, const AccI& acc_i, const AccM& acc_m, int* wcnt,
                                            int D, uint32_t quorum, double* __restrict__ omz,
                                            double* __restrict__ oint) {
  return emit_striped_f<BLOCK>([&](int d) { return (uint32_t)cnt[d]; }, acc_i, acc_m, wcnt, D, quorum, omz, oint);
}

template <bool kSmall, class PrefixT, class CountT>
__device__ __forceinline__ int32_t bin_mean_body(const CsrView& v, const BinMeanParams& P, const BinMeanState<PrefixT, CountT>& S,
                                 int64_t c, const PeaksOut& out, double* prec_out, int32_t* charge_out,
                                 int* tmp, int* flag) {
  const int tid = threadIdx.x;
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n = s1 - s0;
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  if (n == 0) {
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kEmpty;
  }
  if (n > S.nmax || P.n_words > (kSmall ? BM_WMAX : 0x7fffffff)) return kDeferred;

  // spectrum boundaries, from LDS when the cluster is small enough
  if constexpr (kSmall) {
    for (int64_t j = tid; j <= n; j += BM_BLOCK) S.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
    for (int64_t j = tid; j < n; j += BM_BLOCK) S.prec[j] = v.prec_mz[s0 + j];
  }
  auto spec_a = [&](int64_t s) -> int64_t {
    if constexpr (kSmall) return p0 + S.soff[s - s0];
    else return v.spec_off[s];
  };
  auto spec_e = [&](int64_t s) -> int64_t {
    if constexpr (kSmall) return p0 + S.soff[s - s0 + 1];
    else return v.spec_off[s + 1];
  };

  // charge check (binning.py:205-206) -- nothing is emitted for a mixed cluster
  const int32_t z0 = v.charge[s0];
  int mixed = 0;
  for (int64_t s = s0 + 1 + tid; s < s1; s += BM_BLOCK) mixed |= v.charge[s] != z0;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) S.bitmap[w] = 0ull;
  // (a full barrier on the global path: the bitmap zeroing must land before
  // any wave's phase-1 atomicOr; hip's __syncthreads_or orders LDS only)
  if (block_any<BM_BLOCK, kSmall>(mixed, S.votes, 1)) {
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kMixedCharge;
  }

  // phase 1: occupied-bin bitmap (16 independent loads in flight per thread)
  int irregular = 0;  // a spectrum longer than the block: no fast path
  if constexpr (kSmall) {
    for (int64_t j = tid; j < n; j += BM_BLOCK) irregular |= (S.soff[j + 1] - S.soff[j]) > BM_FASTLEN;
  }
  constexpr int U1 = 16;
  if (kSmall && p1 - p0 < (int64_t(1) << 28)) {
    // 32-bit cluster-relative byte offsets from a wave-uniform base (saddr loads)
    const char* __restrict__ mzb = reinterpret_cast<const char*>(v.mz + p0);
    const int np = (int)(p1 - p0);
    for (int r0 = tid; r0 < np; r0 += U1 * BM_BLOCK) {
      double m[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const int r = r0 + u * BM_BLOCK;
        m[u] = *reinterpret_cast<const double*>(mzb + (uint32_t)(r < np ? r : 0) * 8u);
      }
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        if (r0 + u * BM_BLOCK < np && in_range(m[u], P)) {
          const int32_t b = bin_small(m[u], P);
          atomicOr(&S.bitmap[b >> 6], 1ull << (b & 63));
        }
      }
    }
  } else
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
        const int64_t b = kSmall ? (int64_t)bin_small(m[u], P) : bin_of(m[u], P);
        atomicOr(&S.bitmap[b >> 6], 1ull << (b & 63));
      }
    }
  }
  // (the vote is also the barrier between phase-1 ORs and phase-2 reads: always taken)
  const int irregular_any = block_any<BM_BLOCK, kSmall>(irregular, S.votes, 0);
  const bool fast = kSmall && !irregular_any && p1 > p0;

  // phase 2: compact slot ids in bin order
  const int D = bitmap_prefix<BM_BLOCK>(S.bitmap, S.wprefix, P.n_words, tmp);
  if (D > S.dcap) return kDeferred;
  for (int d = tid; d < D; d += BM_BLOCK) {
    S.cnt[d] = 0u;
    S.acc_i[d] = 0.0f;
    S.acc_m[d] = 0.0f;
  }
  if (tid == 0) *flag = 0;  // owner tags not yet initialised
  __syncthreads();

  // phase 3: ordered accumulation, one spectrum at a time
  int64_t slow_from = s0;
  if (fast) {
    // Fast path (every spectrum <= BM_FASTLEN = 252 peaks).  Wave w's lanes
    // 0..62 own peaks 63w..63w+62 of the spectrum; lane 63 loads peak 63w+63
    // (owned by wave w+1's lane 0) only to hand lane 62 its key.  Each lane
    // computes ONE bin key (-1 below min, INT_MAX at or above max) and its slot,
    // and takes its neighbour's key by a DPP move.  If keys are non-decreasing
    // inside every spectrum, equal bins are contiguous and "last peak of its
    // bin" is a neighbour compare; a key inversion or a NaN anywhere defers the
    // whole cluster to the generic kernel.
    // Software-pipelined by one spectrum: iteration j first issues the
    // accumulator reads of spectrum j-1's read-modify-write, computes spectrum
    // j's keys and slots (no shared state) while they are in flight, then
    // writes j-1's sums; one LDS-only barrier per spectrum orders the updates.
    if constexpr (kSmall) {
      // the ring also carries the spectrum's length, so a step reads no offsets
      struct Pk { double m, it; int len; };
      // 32-bit cluster-relative offsets from a wave-uniform base: the loads take
      // the saddr + 32-bit voffset form, no 64-bit address arithmetic per fetch
      const double* __restrict__ mzc = v.mz + p0;
      const double* __restrict__ itc = v.inten + p0;
      const int lane = lane_id();
      const int fpos = wave_id() * (kWave - 1) + lane;  // this lane's peak in every spectrum
      auto fetch = [&](int64_t j) {
        const int jj = (int)(j < n ? j : n - 1);
        const int a = S.soff[jj], e = S.soff[jj + 1];
        const uint32_t k = (uint32_t)(a + fpos);
        const uint32_t idx = k < (uint32_t)e ? k : 0u;
        Pk q;
        q.len = e - a;
        const uint32_t bo = idx * 8u;  // < 2^19: cluster-relative byte offset
        q.m = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(mzc) + bo);
        q.it = *reinterpret_cast<const double*>(reinterpret_cast<const char*>(itc) + bo);
        return q;
      };
      int bad = 0;
      // Rolling register ring: slot j holds spectrum jb + j and is refilled with
      // spectrum jb + j + PF right after it is read, so every load has PF steps
      // to land.  (A double buffer copied at the end of each batch would make
      // the copy wait for the whole next batch's loads: s_waitcnt vmcnt(0).)
      constexpr int PF = SPX_BM_PF;
      Pk R[PF];
#pragma unroll
      for (int j = 0; j < PF; ++j) R[j] = fetch(j);
      // spectrum j - 1 in flight: its slot (or -1) and values
      int pslot = -1;
      double pm = 0.0, pit = 0.0;
      for (int64_t jb = 0; jb < n; jb += PF) {
#pragma unroll
        for (int j = 0; j < PF; ++j) {
          if (jb + j < n) {  // uniform
            const int64_t js = jb + j;
            // spectrum j - 1's accumulator reads first (every lane; non-owners
            // read slot 0 and discard)
            const int ps = pslot >= 0 ? pslot : 0;
            const float e_ai = S.acc_i[ps], e_am = S.acc_m[ps];
            const CountT e_cn = S.cnt[ps];
            const Pk q = R[j];
            const int len = q.len;
            const bool active = fpos < len && lane < kWave - 1, has_next = fpos + 1 < len;
            const bool inr = fpos < len && in_range(q.m, P);  // lane 63 too: its key is lane 62's neighbour
            R[j] = fetch(js + PF);
            bad |= active && (q.m != q.m);
            int32_t key = q.m < P.minimum ? -1 : 0x7fffffff;
            int slot = -1;
            if (inr) {
              key = bin_small(q.m, P);
              slot = bitmap_rank(S.bitmap, S.wprefix, (int64_t)key);
            }
            const int32_t kn = wave_next(key, 0x7fffffff);
            bool last = true;
            if (active && has_next) {
              bad |= key > kn;
              last = kn != key;
            }
            if (pslot >= 0) {  // finish spectrum j - 1
              S.cnt[pslot] = (CountT)(e_cn + 1u);
              S.acc_i[pslot] = (float)((double)e_ai + pit);
              S.acc_m[pslot] = (float)((double)e_am + pm);
            }
            lds_barrier();
            pslot = (active && last) ? slot : -1;
            pm = q.m;
            pit = q.it;
          }
        }
      }
      if (pslot >= 0) accumulate(S, pslot, pm, pit);
      if (block_any<BM_BLOCK, true>(bad, S.votes, 1)) return kDeferred;  // generic kernel redoes it
      slow_from = s1;
    }
  }
  for (int64_t s = slow_from; s < s1; ++s) {
    const int64_t a = spec_a(s), e = spec_e(s);
    int unsorted = 0;
    for (int64_t k = a + tid; k < e; k += BM_BLOCK) {
      const PeakLane L = load_lane(v, k, e);
      unsorted |= L.active && L.has_next && !(L.m <= L.mn);
    }
    if (!block_any<BM_BLOCK, kSmall>(unsorted, S.votes, (int)((s - s0) & 1))) {
      for (int64_t k = a + tid; k < e; k += BM_BLOCK) sorted_lane(S, P, load_lane(v, k, e));
      continue;
    }
    // unsorted spectrum: the highest file position per slot wins (tags grow
    // monotonically through the cluster, so stale tags never win)
    if (S.owner == nullptr) return kDeferred;  // LDS kernel: no tag array, generic kernel
    if (*flag == 0) {
      for (int d = tid; d < D; d += BM_BLOCK) S.owner[d] = 0u;
      __syncthreads();
      if (tid == 0) *flag = 1;
    }
    for (int64_t k = a + tid; k < e; k += BM_BLOCK) {
      const double m = v.mz[k];
      if (in_range(m, P)) atomicMax(&S.owner[bitmap_rank(S.bitmap, S.wprefix, bin_of(m, P))], (uint32_t)(k - p0 + 1));
    }
    __syncthreads();
    for (int64_t k = a + tid; k < e; k += BM_BLOCK) {
      const double m = v.mz[k];
      if (!in_range(m, P)) continue;
      const int slot = bitmap_rank(S.bitmap, S.wprefix, bin_of(m, P));
      if (S.owner[slot] == (uint32_t)(k - p0 + 1)) accumulate(S, slot, m, v.inten[k]);
    }
  }
  __syncthreads();

  // phase 4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (D + BM_BLOCK - 1) / BM_BLOCK;
  int total;
  if constexpr (kSmall) {
    total = emit_striped(S.cnt, [&](int d) { return S.acc_i[d]; }, [&](int d) { return S.acc_m[d]; },
                         reinterpret_cast<int*>(S.bitmap), D, quorum, out.mz + p0,
                         out.inten + p0);
  } else {
    const int d0 = tid * per;
    int mine = 0;
    for (int j = 0; j < per; ++j) {
      const int d = d0 + j;
      if (d < D && S.cnt[d] >= quorum && !isnan(S.acc_i[d])) ++mine;  // cnt >= 1: mean NaN iff sum NaN
    }
    int o = block_exclusive_scan<BM_BLOCK>(mine, tmp, total);
    for (int j = 0; j < per; ++j) {
      const int d = d0 + j;
      if (d < D && S.cnt[d] >= quorum) {
        const double cn = (double)S.cnt[d];
        const double mi = (double)S.acc_i[d] / cn;
        if (isnan(mi)) continue;
        out.inten[p0 + o] = mi;
        out.mz[p0 + o] = S.acc_m[d] == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)S.acc_m[d] / cn;
        ++o;
      }
    }
  }
  if (tid == 0) {
    out.count[c] = total;
    charge_out[c] = z0;
    // np.mean of the precursor list (binning.py:224): pairwise sum / n
    const double* pr = kSmall ? S.prec : v.prec_mz + s0;
    const double sum = kSmall ? pw_sum_small([&](int64_t j) { return pr[j]; }, n)
                              : pw_sum([&](int64_t j) { return pr[j]; }, n);
    prec_out[c] = sum / (double)n;
  }
  return kOk;
}

// ------------------------------------------------------------------------
// Register-code fast path (clusters of <= BR_NMAX m/z-sorted spectra of <= 252
// peaks: every U{2..50} cluster of the configs).  Lane mapping as the body's
// fast path: wave w's lanes 0..62 own peaks 63w..63w+62 of each spectrum, lane
// 63 loads peak 63w+63 only to hand lane 62 its neighbour key.  Each peak's
// bin, its "last in bin" flag and its slot are computed ONCE and kept in
// registers (one u32 per spectrum per lane), so the spectrum-serial fold is
// only the read-modify-write itself:
//   A  spectra in order, no barriers (waves stream independently): m/z, exact
//      bin, DPP neighbour key -> last-in-bin (numpy fancy-index "+=" keeps the
//      last, binning.py:197-199), occupancy bitmap (32-bit LDS atomics), and
//      code[j] = bin of the contribution (-1: none)
//   B  popcount prefix -> slot per bin in ascending order; codes -> slots
//   C  spectra in order: I = f32(f64(I) + inten), M = f32(f64(M) + mz) and the
//      count of each contribution's slot (one 16-B LDS record) -- the reference's
//      float32 accumulation order (binning.py:198-199); one LDS-only barrier per
//      spectrum
// The step masks never live in SGPRs across phases (the codes are opaque to the
// compiler after A): 50 kept masks spilled SGPRs into VGPR lanes and cost ~10%.
//   D  quorum + ordered output (emit_striped), precursor mean
// A key inversion or NaN inside a spectrum sends the cluster to the generic
// kernel.  Returns kNotHere when the cluster does not fit this path.
#ifndef SPX_BR_NMAX
#define SPX_BR_NMAX 50
#endif
constexpr int BR_NMAX = SPX_BR_NMAX;  // spectra per cluster: one code VGPR each
#ifndef SPX_BR_PFA
#define SPX_BR_PFA 8
#endif
#ifndef SPX_BR_PFC
#define SPX_BR_PFC 3
#endif
constexpr int BR_PFA = SPX_BR_PFA;    // phase-A m/z loads in flight per lane
constexpr int BR_PFC = SPX_BR_PFC;    // phase-C (m/z, intensity) loads in flight per lane
#ifndef SPX_BR_KM
#define SPX_BR_KM 8
#endif
// Spectra whose m/z phase A keeps in registers for phase C (no re-read for them):
// 8 with a 3-deep phase-C ring fit the 96 VGPRs of 5 waves/SIMD (100k clusters:
// none 2.24, 6 2.20, 8 2.14 ms); 12 or 20 at 4 waves/SIMD measured 2.28 / 2.23 ms
// (fewer clusters in flight)
constexpr int BR_KM = SPX_BR_KM;
#ifndef SPX_BR_PFA_MD
#define SPX_BR_PFA_MD 6  // the fused pass's phase-A ring depth (8: 11.32 ms, 6: 11.16 at KM 4; configs[4])
#endif
#ifndef SPX_BR_KM_MD
#define SPX_BR_KM_MD 4  // the same for the fused pass (phase A holds its medoid bins too: 8 spilled, 12.37 ms; 6: 12.29; 4: 11.32; 2: 11.17)
#endif
#ifndef SPX_BR_BG
#define SPX_BR_BG 4  // phase-B steps whose LDS reads issue together (8: 2 VGPRs spilled)
#endif
constexpr int BR_W32 = 2 * BM_WMAX;   // 32-bit occupancy words
// phases C-D accumulator of one slot: (intensity, m/z) sums and the contribution count
struct alignas(16) BinAcc {
  float i, m;
  uint32_t n, pad;
};

// LDS of the register path.  The occupancy bitmap (32-bit words + per-word rank
// prefix) is dead once every code is a slot, so the accumulators overlay it.
// The fused pass (bin_mean_medoid_kernel) also keeps the medoid's union bitmap of
// ceil(mz/tol) bins (< 32,768: most_similar_representative.py:15) and its u16 prefix
// in the slack of phases A-B (the accumulators of C-D need more LDS than A-B).
constexpr int BR_MDW32 = 1024;  // 32-bit words of the medoid's bins (32,768 bins)
struct BinRegSmem {
  union alignas(16) {
    struct {
      // + one dummy word per lane past the bitmap: bits 0, prefix BM_DCAP + lane, so
      // a lane's no-contribution code maps to its own dummy accumulator record
      uint32_t bits[BR_W32 + kWave];
      uint16_t pre[BR_W32 + kWave];
      alignas(16) uint32_t mdbits[BR_MDW32];  // fused pass only
      uint16_t mdpre[BR_MDW32];
    } b;                         // phases A-B
    BinAcc acc[BM_DCAP + kWave];  // phases C-D; [BM_DCAP + lane]: dummies
  } u;
  double prec[BR_NMAX];
  int wcnt[(BM_DCAP / BM_BLOCK) * (BM_BLOCK / kWave)];  // emit: kept slots per (stripe, wave)
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};
constexpr int32_t kNotHere = -1;

// Exclusive popcount prefix over ALL BR_W32 occupancy words (BR_W32 / 256 = 12
// contiguous words per thread): three ds_read_b128 per thread -- the 48-B lane
// stride puts each 16-lane group on 16 distinct 16-B bank slots, conflict-free --
// and the u16 prefixes written as three quads.  Words past the batch's bin range
// are zero (the set-up clears all BR_W32).  Returns the number of occupied bins.
constexpr int BR_WPT = BR_W32 / BM_BLOCK;
static_assert(BR_WPT == 12, "reg_prefix reads three b128 quads per thread");
__device__ __forceinline__ int reg_prefix_arrays(const uint32_t* bits, uint16_t* pre, int* tmp) {
  const uint4* src = reinterpret_cast<const uint4*>(bits) + threadIdx.x * (BR_WPT / 4);
  uint32_t w[BR_WPT];
#pragma unroll
  for (int k = 0; k < BR_WPT / 4; ++k) {
    const uint4 q = src[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
  int local = 0;
#pragma unroll
  for (int k = 0; k < BR_WPT; ++k) local += __popc(w[k]);
  int total;
  int base = block_exclusive_scan<BM_BLOCK, int, true, false>(local, tmp, total);
  uint2* dst = reinterpret_cast<uint2*>(pre) + threadIdx.x * (BR_WPT / 4);
#pragma unroll
  for (int k = 0; k < BR_WPT / 4; ++k) {
    uint32_t p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { p[i] = (uint32_t)base; base += __popc(w[4 * k + i]); }
    dst[k] = make_uint2(p[0] | (p[1] << 16), p[2] | (p[3] << 16));
  }
  lds_barrier();
  return total;
}
__device__ __forceinline__ int reg_prefix(BinRegSmem& L) { return reg_prefix_arrays(L.u.b.bits, L.u.b.pre, L.tmp); }

// reg_prefix and the medoid's bitmap prefix (4 contiguous words per thread) in ONE
// block scan: each count is <= the cluster's peaks (<= 50 x 252 = 12,600), so the two
// local sums travel packed, bin-mean in the low and the medoid in the high 16 bits.
// Returns the bin-mean's occupied bins; *md_total the medoid's (its column count K).
__device__ __forceinline__ int reg_prefix_md(BinRegSmem& L, int* md_total) {
  const uint4* src = reinterpret_cast<const uint4*>(L.u.b.bits) + threadIdx.x * (BR_WPT / 4);
  uint32_t w[BR_WPT];
#pragma unroll
  for (int k = 0; k < BR_WPT / 4; ++k) {
    const uint4 q = src[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
  static_assert(BR_MDW32 == 4 * BM_BLOCK, "one b128 of medoid words per thread");
  const uint4 mq = reinterpret_cast<const uint4*>(L.u.b.mdbits)[threadIdx.x];
  const uint32_t mw[4] = {mq.x, mq.y, mq.z, mq.w};
  int local = 0, mlocal = 0;
#pragma unroll
  for (int k = 0; k < BR_WPT; ++k) local += __popc(w[k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) mlocal += __popc(mw[k]);
  int total;
  const int packed = block_exclusive_scan<BM_BLOCK, int, true, false>(local | (mlocal << 16), L.tmp, total);
  int base = packed & 0xFFFF, mbase = (int)((uint32_t)packed >> 16);
  uint2* dst = reinterpret_cast<uint2*>(L.u.b.pre) + threadIdx.x * (BR_WPT / 4);
#pragma unroll
  for (int k = 0; k < BR_WPT / 4; ++k) {
    uint32_t p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { p[i] = (uint32_t)base; base += __popc(w[4 * k + i]); }
    dst[k] = make_uint2(p[0] | (p[1] << 16), p[2] | (p[3] << 16));
  }
  uint32_t mp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { mp[i] = (uint32_t)mbase; mbase += __popc(mw[i]); }
  reinterpret_cast<uint2*>(L.u.b.mdpre)[threadIdx.x] = make_uint2(mp[0] | (mp[1] << 16), mp[2] | (mp[3] << 16));
  lds_barrier();
  *md_total = (int)((uint32_t)total >> 16);
  return total & 0xFFFF;
}

// What the fused pass's register path hands the medoid (bin_mean_reg_path_t<true>):
// the medoid's tolerance in, and out: `out` (a peak's ceil(mz/tol) outside
// [0, 32,768): the medoid reads the m/z itself), K (its occupied bins) and this lane's
// spectrum [rlo, rhi) (lane j: spectrum min(j, n-1)), relative to the cluster's first peak.
struct MdSide {
  double tol, inv_tol;
  int out, K;
  int32_t rlo, rhi;
};

// the register path's step loops: n <= BR_NMAX steps, uniform early exit
template <class F>
__device__ __forceinline__ void reg_steps(int n, F&& f) {
  unrolled_while(n, f, std::make_integer_sequence<int, BR_NMAX>{});
}

// kMd (the fused pass, bin_mean_medoid_kernel): phase A also computes each peak's
// medoid bin ceil(mz/tol) from the same m/z load and ORs it into the medoid's union
// bitmap; phase B turns it into the medoid's column (its rank among the cluster's
// occupied medoid bins).  code[j] then carries the bin-mean slot in its low and the
// medoid column in its high 16 bits, so the medoid builds its bit rows from registers
// (medoid_from_codes, fused.hip) and never reads the m/z again.  kMd = false is the
// register kernel's own path, unchanged.
template <bool kMd>
__device__ __forceinline__ int32_t bin_mean_reg_path_t(const CsrView& v, const BinMeanParams& P, BinRegSmem& L,
                                                       int64_t c, const PeaksOut& out, double* prec_out,
                                                       int32_t* charge_out, int32_t (&code)[BR_NMAX], MdSide* md) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  // spectra whose m/z phase A keeps for phase C (the fused pass needs registers for
  // its medoid bins in phase A)
  constexpr int KM = kMd ? SPX_BR_KM_MD : BR_KM;
  constexpr int PFA = kMd ? SPX_BR_PFA_MD : BR_PFA;  // phase-A ring depth
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n64 = s1 - s0;
  if (n64 < 1 || n64 > BR_NMAX || P.n_words > BM_WMAX) return kNotHere;
  const int n = (int)n64;
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  if (p1 == p0 || p1 - p0 >= (int64_t(1) << 28)) return kNotHere;
  // lane j of every wave: spectrum j's [lo, hi) relative to p0, charge, precursor
  const int jl = lane < n ? lane : n - 1;
  const int32_t rlo = (int32_t)(v.spec_off[s0 + jl] - p0), rhi = (int32_t)(v.spec_off[s0 + jl + 1] - p0);
  const int32_t z0 = v.charge[s0];
  const bool mine = lane < n;
  const int32_t zl = v.charge[s0 + jl];
  const double pl = v.prec_mz[s0 + jl];
  if (__ballot(mine & ((rhi - rlo) > BM_FASTLEN)) != 0ull) return kNotHere;  // uniform (same in every wave)
  if (__ballot(mine & (zl != z0)) != 0ull) {  // binning.py:205-206: nothing emitted
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kMixedCharge;
  }
  if (wid == 0 && mine) L.prec[lane] = pl;
  if constexpr (kMd) {
    md->rlo = rlo;
    md->rhi = rhi;
    reinterpret_cast<uint4*>(L.u.b.mdbits)[tid] = make_uint4(0u, 0u, 0u, 0u);
  }
  {
    uint4* z = reinterpret_cast<uint4*>(L.u.b.bits) + tid * (BR_WPT / 4);
#pragma unroll
    for (int k = 0; k < BR_WPT / 4; ++k) z[k] = make_uint4(0u, 0u, 0u, 0u);
    if (tid < kWave) {  // the dummy words (phase C's accumulators overwrote them)
      L.u.b.bits[BR_W32 + tid] = 0u;
      L.u.b.pre[BR_W32 + tid] = (uint16_t)(BM_DCAP + tid);
    }
  }
  lds_barrier();
  SPX_STAMP2(1, -1);

  const int fpos = wid * (kWave - 1) + lane;  // this lane's peak in every spectrum
  const bool owner = lane < kWave - 1;
  // Buffer descriptors over the cluster's peaks.  A lane past its spectrum's end
  // reads the next spectrum's peak, or 0 past the cluster's end (out of the
  // descriptor's range: no fault), so the offsets need no select; spectra past
  // the cluster's last (j >= n, a ring's tail prefetch) re-read the last one.
  // The ring's loads are unconditional (a conditional load makes its ring
  // register a merge of two values, which compiles to a wait right after issue).
  const __amdgpu_buffer_rsrc_t rmz = bf_rsrc(v.mz + p0, (int)(p1 - p0));
  const __amdgpu_buffer_rsrc_t rit = bf_rsrc(v.inten + p0, (int)(p1 - p0));
  auto boffb = [&](int j) -> int {  // byte offset of this lane's peak of spectrum j
    const int jj = j < n ? j : n - 1;
    return (__builtin_amdgcn_readlane(rlo, jj) + fpos) * 8;
  };

  // ---- A: bins, last-in-bin, occupancy, codes (branch-free per lane)
  double mk[KM > 0 ? KM : 1];  // m/z of spectra 0..BR_KM-1, kept from phase A
  uint32_t* bm32 = L.u.b.bits;
  int bad = 0, mdout = 0;
  {
    // ring slot: this lane's m/z of spectrum j and the spectrum's length (read
    // once, when the load is issued)
    double ra[PFA];
    int rl[PFA];
    auto fetch = [&](int j, double& m, int& len) __attribute__((always_inline)) {
      const int jj = j < n ? j : n - 1;
      const int a = __builtin_amdgcn_readlane(rlo, jj), e = __builtin_amdgcn_readlane(rhi, jj);
      const int k = a + fpos;
      len = e - a;
      m = bf_load(rmz, k * 8, 0);
    };
#pragma unroll
    for (int j = 0; j < BR_NMAX; ++j) code[j] = -1;
    auto body = [&](auto jc, const double m, const int len) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      if constexpr (j < KM) mk[j] = m;
      const bool act = fpos < len;
      const bool inr = act & (m >= P.minimum) & (m < P.maximum);
      const int32_t kb = bin_small(m, P);  // used only where inr
      // inactive lanes (past the spectrum's end) carry INT_MAX: the last active
      // peak's neighbour then always differs from it, and never sorts below it
      const int32_t key = inr ? kb : ((act & (m < P.minimum)) ? -1 : 0x7fffffff);
      const int32_t kn = wave_next(key, 0x7fffffff);
      bad |= (int)(owner & act & ((m != m) | (key > kn)));
      const bool valid = owner & inr & (kn != key);  // the last peak of its bin (binning.py:197-199)
      // a lane without a contribution ORs 0 into a word of its own (same-address
      // LDS atomics serialise; distinct words do not)
      atomicOr(&bm32[valid ? key >> 5 : lane], valid ? 1u << (key & 31) : 0u);
      if constexpr (kMd) {
        // the medoid's bin of the same peak, ceil(mz / tol) exactly (md_bin): the
        // reciprocal product where it is certain, else the division (~1 peak in 10^7)
        const bool mact = owner & act;
        const double q = m * md->inv_tol;
        const double t = ceil(q);
        const double f = t - q;
        uint32_t mb = (uint32_t)__double2int_rz(t);
        if (__builtin_expect(mact & !((f > kDivBand) & (f < 1.0 - kDivBand) & (mb < 32u * BR_MDW32)), 0)) {
          const int64_t bb = ceil_div_exact(m, md->tol, md->inv_tol);
          const bool in = bb >= 0 && bb < 32 * BR_MDW32;
          mdout |= !in;
          mb = in ? (uint32_t)bb : 0u;
        }
        // no peak here: 0 ORed into a word of the lane's own (same-address atomics serialise)
        atomicOr(&L.u.b.mdbits[mact ? mb >> 5 : lane], mact ? 1u << (mb & 31) : 0u);
        // bin-mean bin in the low 17 bits (0x1FFFF: no contribution), medoid bin above
        code[j] = (valid ? key : 0x1FFFF) | (int32_t)((mact ? mb : 0u) << 17);
      } else {
        code[j] = valid ? key : -1;
      }
      // opaque to the compiler: phase B must not keep each step's 64-bit valid mask
      // live instead (50 SGPR pairs: spills)
      asm volatile("" : "+v"(code[j]));
    };
#pragma unroll
    for (int j = 0; j < PFA; ++j) fetch(j, ra[j], rl[j]);
    reg_steps(n, [&](auto jc) __attribute__((always_inline)) {
      constexpr int j = decltype(jc)::value;
      const double m = ra[j % PFA];
      const int len = rl[j % PFA];
      fetch(j + PFA, ra[j % PFA], rl[j % PFA]);
      body(jc, m, len);
    });
  }
  // phase C's first (m/z, intensity) loads go out now and land during phase B
  // (whose barriers are LDS-only, so they stay in flight)
  double rm[BR_PFC], ri[BR_PFC];
#pragma unroll
  for (int j = 0; j < BR_PFC; ++j) {
    const int bo = boffb(j);
    if (j >= KM) rm[j] = bf_load(rmz, bo, 0);
    ri[j] = bf_load(rit, bo, 0);
  }
  if constexpr (kMd) {
    // one barrier for both votes: bit 0 bin-mean's (unsorted / NaN), bit 1 the medoid's
    const int w = (__ballot(bad) != 0ull ? 1 : 0) | (__ballot(mdout) != 0ull ? 2 : 0);
    if (lane == 0) L.votes[wid] = w;
    lds_barrier();
    int r = 0;
#pragma unroll
    for (int k = 0; k < BM_BLOCK / kWave; ++k) r |= L.votes[k];
    md->out = r >> 1;
    if (r & 1) return kDeferred;  // generic kernel redoes it
  } else {
    if (block_any<BM_BLOCK, true>(bad, L.votes, 0)) return kDeferred;  // generic kernel redoes it
  }
  SPX_STAMP2(2, 1);

  // ---- B: slots in bin order, codes -> slots (the contribution count rides
  // phase C's read-modify-write)
  int D;
  if constexpr (kMd) D = reg_prefix_md(L, &md->K);
  else D = reg_prefix(L);
  if (D > BM_DCAP) return kDeferred;
  // Every step is the same two LDS reads and a popcount -- no branch: a code
  // without contribution (-1: word 0x7FFFFFF, clamped to this lane's dummy word,
  // bit 31 of an all-zero word) ranks to BM_DCAP + lane -- and a group of
  // SPX_BR_BG steps issues its reads before the first use (one step at a time, each read
  // waited for, was ~5k cycles of this phase).
  {
    constexpr int G = SPX_BR_BG;
    int nn = __builtin_amdgcn_readfirstlane(n);
#pragma unroll
    for (int j0 = 0; j0 < BR_NMAX; j0 += G) {
      asm volatile("" : "+s"(nn));  // one uniform guard per group, evaluated in place
      if (j0 < nn) {
        uint32_t wb[G], wp[G], mwb[G], mwp[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
          if (j0 + q < BR_NMAX) {
            const uint32_t lo = kMd ? (uint32_t)code[j0 + q] & 0x1FFFFu : (uint32_t)code[j0 + q];
            const uint32_t w = min(lo >> 5, (uint32_t)(BR_W32 + lane));
            wb[q] = L.u.b.bits[w];
            wp[q] = L.u.b.pre[w];
            if constexpr (kMd) {
              const uint32_t mw = (uint32_t)code[j0 + q] >> 22;  // the medoid bin's word
              mwb[q] = L.u.b.mdbits[mw];
              mwp[q] = L.u.b.mdpre[mw];
            }
          }
        }
#pragma unroll
        for (int q = 0; q < G; ++q) {
          if (j0 + q < BR_NMAX) {
            const uint32_t b = (uint32_t)code[j0 + q];
            const int32_t slot = (int32_t)wp[q] + __popc(wb[q] & ((1u << (b & 31)) - 1u));
            if constexpr (kMd) {
              // the medoid column: rank of the bin among the cluster's medoid bins
              const uint32_t mb = b >> 17;
              const uint32_t col = mwp[q] + __popc(mwb[q] & ((1u << (mb & 31)) - 1u));
              code[j0 + q] = slot | (int32_t)(col << 16);
            } else {
              code[j0 + q] = slot;
            }
          }
        }
      }
    }
  }
  lds_barrier();  // the bitmap is dead: the accumulators take its place
  for (int d = tid; d < D; d += BM_BLOCK) L.u.acc[d] = BinAcc{0.0f, 0.0f, 0u, 0u};
  lds_barrier();
  SPX_STAMP2(3, 2);

  // ---- C: the ordered fold (spectrum order per slot = the reference's order)
  reg_steps(n, [&](auto jc) __attribute__((always_inline)) {
    constexpr int j = decltype(jc)::value;
    double m;
    const double it = ri[j % BR_PFC];
    if constexpr (j < KM) m = mk[j];
    else m = rm[j % BR_PFC];
    const int bo = boffb(j + BR_PFC);
    if constexpr (j + BR_PFC >= KM) rm[j % BR_PFC] = bf_load(rmz, bo, 0);
    ri[j % BR_PFC] = bf_load(rit, bo, 0);
    const int slot = kMd ? code[j] & 0xFFFF : code[j];
    if constexpr (kMd && (j & 1)) {
      // both slots used: spectra j-1 and j's medoid columns share code[j-1] (low, high
      // half) from here on, so code[j] is dead through phase D (registers for the emit)
      code[j - 1] = (int32_t)(((uint32_t)code[j - 1] >> 16) | ((uint32_t)code[j] & 0xFFFF0000u));
    }
    BinAcc a = L.u.acc[slot];
    a.i = (float)((double)a.i + it);
    a.m = (float)((double)a.m + m);
    a.n += 1u;
    L.u.acc[slot] = a;
    lds_barrier();
  });
  SPX_STAMP2(4, 3);

  // ---- D: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int total = emit_striped_f([&](int d) { return L.u.acc[d].n; }, [&](int d) { return L.u.acc[d].i; },
                                   [&](int d) { return L.u.acc[d].m; }, L.wcnt, D, quorum, out.mz + p0,
                                   out.inten + p0);
  if (tid == 0) {
    out.count[c] = total;
    charge_out[c] = z0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return L.prec[j]; }, n) / (double)n;  // np.mean (binning.py:224)
  }
  return kOk;
}

using BinHeadSmem = BinRegSmem;
__device__ __forceinline__ int32_t bin_mean_head_path(const CsrView& v, const BinMeanParams& P, BinHeadSmem& L,
                                                      int64_t c, const PeaksOut& out, double* prec_out,
                                                      int32_t* charge_out) {
  int32_t code[BR_NMAX];
  return bin_mean_reg_path_t<false>(v, P, L, c, out, prec_out, charge_out, code, nullptr);
}

// Register-code kernel: one workgroup per cluster.  Clusters this path does not
// take (kNotHere) and kDeferred ones (unsorted, NaN, too many distinct bins) go
// to the striped `rest` list of the wide kernel (which hands the unsorted ones on
// to the global kernel).
__global__ __launch_bounds__(BM_BLOCK, SPX_BR_MINW) void bin_mean_reg_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                             double* prec_out, int32_t* charge_out,
                                                                             int32_t* status, StripedList rest) {
  __shared__ BinHeadSmem L;
  const int64_t c = blockIdx.x;
  SPX_STAMP(0);
  const int32_t st = bin_mean_head_path(v, P, L, c, out, prec_out, charge_out);
  SPX_STAMP(6);
  if (threadIdx.x == 0) {
    if (st != kNotHere) status[c] = st;
    if (st == kNotHere || st == kDeferred) striped_push(rest, (int32_t)c);
  }
}

// The LDS body (bin_mean_body<true>: its own fast path for <= 128 spectra) over
// the clusters the register kernel left, grid-stride over the list.
__global__ __launch_bounds__(BM_BLOCK, SPX_BM_MINW) void bin_mean_lds_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                double* prec_out, int32_t* charge_out,
                                                                int32_t* status, const int32_t* list,
                                                                const int32_t* n_list, int32_t* deferred,
                                                                int32_t* n_deferred) {
  __shared__ BinMeanSmem L;
  BinMeanState<uint16_t, uint16_t> S;
  S.bitmap = L.bitmap;
  S.wprefix = L.wprefix;
  S.cnt = L.cnt;
  S.acc_i = L.acc_i;
  S.acc_m = L.acc_m;
  S.owner = nullptr;
  S.soff = L.soff;
  S.prec = L.prec;
  S.votes = L.votes;
  S.xch = nullptr;
  S.dcap = BM_DCAP;
  S.nmax = BM_NMAX;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = list[i];
    const int32_t st = bin_mean_body<true>(v, P, S, c, out, prec_out, charge_out, L.tmp, &L.flag);
    if (threadIdx.x == 0) {
      status[c] = st;
      if (st == kDeferred) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
    __syncthreads();
  }
}

// Scratch slice of the deferred path, every array 256-B aligned.
struct BinSliceLayout {
  int64_t bitmap, wprefix, cnt, acc_i, acc_m, owner, total;
};
__host__ __device__ inline BinSliceLayout bin_slice_layout(int64_t n_words, int64_t dcap) {
  BinSliceLayout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t at = o; o += (bytes + 255) & ~int64_t(255); return at; };
  L.bitmap = take(n_words * 8);
  L.wprefix = take(n_words * 4);
  L.cnt = take(dcap * 4);
  L.acc_i = take(dcap * 4);
  L.acc_m = take(dcap * 4);
  L.owner = take(dcap * 4);
  L.total = o;
  return L;
}

// Deferred clusters: same body, state in global scratch (slice per workgroup).
__global__ __launch_bounds__(BM_BLOCK) void bin_mean_global_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                   double* prec_out, int32_t* charge_out,
                                                                   int32_t* status, const int32_t* deferred,
                                                                   const int32_t* n_deferred, char* scratch,
                                                                   int64_t slice_bytes, int dcap) {
  __shared__ int tmp[BM_BLOCK / kWave + 1];
  __shared__ int votes[2 * (BM_BLOCK / kWave)];
  __shared__ int flag;
  char* base = scratch + (int64_t)blockIdx.x * slice_bytes;
  const BinSliceLayout Lo = bin_slice_layout(P.n_words, dcap);
  BinMeanState<uint32_t, uint32_t> S;
  S.bitmap = reinterpret_cast<unsigned long long*>(base + Lo.bitmap);
  S.wprefix = reinterpret_cast<uint32_t*>(base + Lo.wprefix);
  S.cnt = reinterpret_cast<uint32_t*>(base + Lo.cnt);
  S.acc_i = reinterpret_cast<float*>(base + Lo.acc_i);
  S.acc_m = reinterpret_cast<float*>(base + Lo.acc_m);
  S.owner = reinterpret_cast<uint32_t*>(base + Lo.owner);
  S.soff = nullptr;
  S.prec = nullptr;
  S.votes = votes;
  S.xch = nullptr;
  S.dcap = dcap;
  S.nmax = 0x7fffffff;
  const int32_t nd = *n_deferred;
  for (int32_t i = blockIdx.x; i < nd; i += gridDim.x) {
    const int64_t c = deferred[i];
    const int32_t st = bin_mean_body<false>(v, P, S, c, out, prec_out, charge_out, tmp, &flag);
    if (threadIdx.x == 0) status[c] = st;
    __syncthreads();
  }
}

// bytes of one fallback slice
__host__ int64_t bin_mean_slice_bytes(int32_t n_words, int64_t dcap) { return bin_slice_layout(n_words, dcap).total; }

}  // namespace spx
