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
#include "spx_device.hpp"

namespace spx {

struct BinMeanParams {
  double minimum, maximum, binsize, inv_binsize;
  int32_t apply_quorum;
  int32_t n_words;  // ceil(n_bins / 64)
  int32_t ablate;   // profiling only (SPX_ABLATE): 1 skip phase 3, 2 skip phase 4
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
#define SPX_BM_MINW 5  // __launch_bounds__ minimum waves per SIMD for bin_mean_lds_kernel (LDS allows 5)
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

template <bool kSmall, class PrefixT, class CountT>
__device__ int32_t bin_mean_body(const CsrView& v, const BinMeanParams& P, const BinMeanState<PrefixT, CountT>& S,
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
  int64_t slow_from = (P.ablate & 1) ? s1 : s0;
  if (fast && !(P.ablate & 1)) {
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

  if (P.ablate & 2) {
    if (tid == 0) out.count[c] = 0;
    return kOk;
  }
  // phase 4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (D + BM_BLOCK - 1) / BM_BLOCK;
  int total;
  if constexpr (kSmall) {
    // Slots striped over the block (slot j*256 + tid): conflict-free LDS reads and
    // coalesced stores.  A slot's output position = kept slots before it = kept in
    // earlier stripes + kept in earlier waves of its stripe + earlier lanes of its
    // wave (ballot).  Per-(stripe, wave) counts go to the dead bitmap: one barrier.
    constexpr int NW = BM_BLOCK / kWave;
    int* wcnt = reinterpret_cast<int*>(S.bitmap);  // [per][NW], per <= BM_DCAP / BM_BLOCK
    const int lane = lane_id(), wid = wave_id();
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t keep = 0u;  // bit j: slot j*256 + tid is emitted
    for (int j = 0; j < per; ++j) {
      const int d = j * BM_BLOCK + tid;
      const bool k = d < D && S.cnt[d] >= quorum && !isnan(S.acc_i[d]);  // cnt >= 1: mean NaN iff sum NaN
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
        const int d = j * BM_BLOCK + tid;
        const int o = base + before + __popcll(b & below);
        const double cn = (double)S.cnt[d];
        out.inten[p0 + o] = (double)S.acc_i[d] / cn;
        out.mz[p0 + o] = S.acc_m[d] == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)S.acc_m[d] / cn;
      }
      base += tot;
    }
    total = base;
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

__global__ __launch_bounds__(BM_BLOCK, SPX_BM_MINW) void bin_mean_lds_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                double* prec_out, int32_t* charge_out,
                                                                int32_t* status, int32_t* deferred,
                                                                int32_t* n_deferred) {
  __shared__ BinMeanSmem L;
  const int64_t c = blockIdx.x;
  BinMeanState<uint16_t, uint16_t> S{L.bitmap, L.wprefix, L.cnt, L.acc_i, L.acc_m, nullptr, L.soff, L.prec, L.votes, nullptr,
                           BM_DCAP, BM_NMAX};
  const int32_t st = bin_mean_body<true>(v, P, S, c, out, prec_out, charge_out, L.tmp, &L.flag);
  if (threadIdx.x == 0) {
    status[c] = st;
    if (st == kDeferred) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
  }
}

// ------------------------------------------------------------------------
// bin_mean_list_kernel: the per-cluster fast path (one workgroup per cluster).
//
// No spectrum-serial loop: the reference's float32 accumulation order (spectrum
// order within each bin) is rebuilt as an explicit per-bin list instead.
//   P1  every peak once (flat, coalesced; <= 48 peaks per thread kept in
//       registers): exact bin, LDS occupancy bitmap, and "last peak of its bin
//       in its spectrum" (numpy fancy-index "+=" keeps the last,
//       binning.py:197-199) = the next peak of the same spectrum has another
//       bin -- a neighbour compare, valid because keys are checked to be
//       non-decreasing inside every spectrum (else the cluster is deferred).
//   P2  popcount prefix -> compact slots in ascending bin order.
//   P3a each last peak sets bit s (its spectrum) of smask[slot]:
//       count(slot) = popcount(smask[slot]) = the reference's n[b].
//   P3b one block scan: kept slots (count >= int(0.25 n)+1) in bin order and
//       their list offsets.
//   P3c each last peak of a kept slot writes its position to
//       list[off[slot] + popcount(smask[slot] & below(s))]: the slot's list is in
//       spectrum order by construction (no atomics, no sort).
//   P3d one thread per kept slot folds I = f32(f64(I) + it), M = f32(f64(M) + mz)
//       along its list (the reference's order) and writes the means.
// Deferred to bin_mean_global_kernel (the generic spectrum-serial body): more
// than 64 spectra or BL_PCAP peaks, empty spectra, NaN m/z or non-finite means,
// a key inversion inside a spectrum (unsorted), > BL_DCAP slots or > BL_LCAP kept
// contributions.
constexpr int BL_UMAX = 48;                  // peaks per thread
constexpr int BL_PCAP = BL_UMAX * BM_BLOCK;  // 12,288 peaks per cluster
constexpr int BL_LCAP = 10240;               // kept (spectrum, bin) contributions
constexpr int BL_DCAP = 1536;                // occupied bins (slots)
constexpr int BL_NMAX = 64;                  // spectra (one u64 mask per slot)
constexpr int BL_SW = BL_PCAP / 64;          // spectrum-start bitmap words
constexpr uint16_t BL_DROP = 0xFFFFu;
constexpr int BL_PB = 16;                    // P1 loads in flight per thread

struct BinListSmem {
  union {
    struct {
      unsigned long long bitmap[BM_WMAX];
      uint16_t wprefix[BM_WMAX];
    } b;                      // P1..P3a
    uint16_t list[BL_LCAP];   // P3c..P3d (peak offsets within the cluster)
  } u;
  unsigned long long smask[BL_DCAP];
  uint16_t loff[BL_DCAP];     // list offset of a kept slot (BL_DROP: below quorum)
  uint16_t kslot[BL_DCAP];    // slot of the j-th kept slot (= output order)
  unsigned long long sbits[BL_SW];  // bit r: peak r starts spectrum >= 1
  uint8_t spre[BL_SW];              // spectra started before word w
  int32_t xch[BL_UMAX * (BM_BLOCK / kWave)];  // lane-0 key of (iteration, wave)
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
  long long tmp64[BM_BLOCK / kWave + 1];
};

// register entry: P1 holds (bin | flags), P3a on (slot | spectrum << 16 | flags)
constexpr uint32_t BL_IN = 1u << 31;    // peak exists and min <= mz < max
constexpr uint32_t BL_LAST = 1u << 30;  // last peak of its bin in its spectrum
constexpr uint32_t BL_NXT = 1u << 29;   // lane 63 only: the next peak is in the same spectrum
constexpr uint32_t BL_HI = 1u << 28;    // out of range at/above maximum (key INT_MAX; else -1)
constexpr uint32_t BL_VAL = (1u << 28) - 1u;

__device__ __forceinline__ void bl_finish_empty(const PeaksOut& out, double* prec_out, int32_t* charge_out, int64_t c) {
  out.count[c] = 0;
  prec_out[c] = __longlong_as_double(0x7ff8000000000000ll);
  charge_out[c] = 0;
}

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_list_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                 double* prec_out, int32_t* charge_out,
                                                                 int32_t* status, int32_t* deferred,
                                                                 int32_t* n_deferred) {
  __shared__ BinListSmem L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  constexpr int NW = BM_BLOCK / kWave;
  const int64_t c = blockIdx.x;
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  const int np = (int)(p1 - p0);
  auto defer = [&]() {
    if (tid == 0) {
      status[c] = kDeferred;
      deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
  };
  if (n == 0) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kEmpty; }
    return;
  }
  if (n > BL_NMAX || p1 - p0 > BL_PCAP || P.n_words > BM_WMAX) { defer(); return; }

  // P0: charge check (binning.py:205-206), zero the bitmaps, spectrum starts
  const int32_t z0 = v.charge[s0];
  int mixed = 0, empty_spec = 0;
  if (tid < n) {
    mixed = v.charge[s0 + tid] != z0;
    empty_spec = v.spec_off[s0 + tid + 1] == v.spec_off[s0 + tid];
  }
  const int nsw = (np + 63) / 64;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.u.b.bitmap[w] = 0ull;
  for (int w = tid; w < nsw; w += BM_BLOCK) L.sbits[w] = 0ull;
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 0)) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kMixedCharge; }
    return;
  }
  if (tid >= 1 && tid < n) {
    const int r = (int)(v.spec_off[s0 + tid] - p0);
    if (r < np) atomicOr(&L.sbits[r >> 6], 1ull << (r & 63));
  }
  if (block_any<BM_BLOCK, true>(empty_spec, L.votes, 1)) { defer(); return; }

  // P1: one exact bin per peak, bitmap, neighbour keys.  Loads are issued in
  // batches of BL_PB (all in flight together), then the batch is processed.
  uint32_t ent[BL_UMAX];
  int bad = 0;
#pragma unroll
  for (int u = 0; u < BL_UMAX; ++u) ent[u] = 0u;
#pragma unroll
  for (int u0 = 0; u0 < BL_UMAX; u0 += BL_PB) {
    if (u0 * BM_BLOCK < np) {  // uniform
      double mb[BL_PB];
#pragma unroll
      for (int q = 0; q < BL_PB; ++q) {
        const int r = (u0 + q) * BM_BLOCK + tid;
        mb[q] = v.mz[p0 + (r < np ? r : 0)];
      }
#pragma unroll
      for (int q = 0; q < BL_PB; ++q) {
        const int u = u0 + q;
        if (u * BM_BLOCK < np) {  // uniform
          const int r = u * BM_BLOCK + tid;
          const bool valid = r < np;
          const double m = mb[q];
          bad |= valid && (m != m);
          int32_t key = m < P.minimum ? -1 : 0x7fffffff;
          const bool inr = valid && in_range(m, P);
          if (inr) {
            const int64_t b = bin_of(m, P);
            key = (int32_t)b;
            atomicOr(&L.u.b.bitmap[b >> 6], 1ull << (b & 63));
          }
          const int32_t kn = __shfl_down(key, 1, kWave);
          if (lane == 0) L.xch[u * NW + wid] = key;
          const int rn = r + 1;
          const bool same = valid && rn < np && !((L.sbits[rn >> 6] >> (rn & 63)) & 1ull);
          uint32_t e = inr ? (BL_IN | (uint32_t)key) : (key == 0x7fffffff ? BL_HI : 0u);
          if (lane < kWave - 1) {
            bad |= same && key > kn;
            if (!(same && kn == key)) e |= BL_LAST;
          } else if (same) {
            e |= BL_NXT;  // decided after the barrier from the next wave's lane-0 key
          } else {
            e |= BL_LAST;
          }
          ent[u] = e;
        }
      }
    }
  }
  // spectra started before each start-bit word (wave 0; n <= 64 fits a u8)
  if (wid == 0) {
    int carry = 0;
    for (int w0 = 0; w0 < nsw; w0 += kWave) {
      const int w = w0 + lane;
      const int pc = w < nsw ? __popcll(L.sbits[w]) : 0;
      int inc = pc;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(inc, o, kWave);
        if (lane >= o) inc += t;
      }
      if (w < nsw) L.spre[w] = (uint8_t)(carry + inc - pc);
      carry += __shfl(inc, kWave - 1, kWave);
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 0)) { defer(); return; }

  // P2: compact slots in bin order
  const int D = bitmap_prefix<BM_BLOCK>(L.u.b.bitmap, L.u.b.wprefix, P.n_words, L.tmp);
  if (D > BL_DCAP) { defer(); return; }
  for (int d = tid; d < D; d += BM_BLOCK) L.smask[d] = 0ull;
  lds_barrier();

  // P3a: spectrum masks per slot; lane 63 resolves its cross-wave neighbour
#pragma unroll
  for (int u = 0; u < BL_UMAX; ++u) {
    if (u * BM_BLOCK < np) {
      uint32_t e = ent[u];
      if (e & BL_NXT) {
        const int32_t kx = wid < NW - 1 ? L.xch[u * NW + wid + 1] : L.xch[(u + 1) * NW];
        const int32_t key = (e & BL_IN) ? (int32_t)(e & BL_VAL) : ((e & BL_HI) ? 0x7fffffff : -1);
        bad |= key > kx;
        if (kx != key) e |= BL_LAST;
      }
      if (e & BL_IN) {
        const int r = u * BM_BLOCK + tid;
        const int slot = bitmap_rank(L.u.b.bitmap, L.u.b.wprefix, (int64_t)(e & BL_VAL));
        const int sp = (int)L.spre[r >> 6] + __popcll(L.sbits[r >> 6] & ((2ull << (r & 63)) - 1ull));
        if (e & BL_LAST) atomicOr(&L.smask[slot], 1ull << sp);
        e = (e & (BL_IN | BL_LAST)) | (uint32_t)slot | ((uint32_t)sp << 16);
      }
      ent[u] = e;
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 1)) { defer(); return; }
  if (P.ablate & 1) {
    if (tid == 0) { out.count[c] = 0; status[c] = kOk; }
    return;
  }

  // P3b: kept slots in bin order and their list offsets (one 64-bit scan)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (D + BM_BLOCK - 1) / BM_BLOCK;
  const int d0 = tid * per;
  long long mine = 0;
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
    if (d < D) {
      const uint32_t cn = (uint32_t)__popcll(L.smask[d]);
      if (cn >= quorum) mine += (1ll << 32) | (long long)cn;
    }
  }
  long long tot;
  long long ex = block_exclusive_scan<BM_BLOCK>(mine, L.tmp64, tot);
  const int K = (int)(tot >> 32), LN = (int)(tot & 0xffffffffll);
  if (LN > BL_LCAP) { defer(); return; }
  int kj = (int)(ex >> 32), lo = (int)(ex & 0xffffffffll);
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
    if (d < D) {
      const uint32_t cn = (uint32_t)__popcll(L.smask[d]);
      if (cn >= quorum) {
        L.loff[d] = (uint16_t)lo;
        L.kslot[kj] = (uint16_t)d;
        lo += (int)cn;
        ++kj;
      } else {
        L.loff[d] = BL_DROP;
      }
    }
  }
  lds_barrier();  // also: the bitmap (aliased by the list) is dead from here

  // P3c: spectrum-ordered lists of the kept slots
#pragma unroll
  for (int u = 0; u < BL_UMAX; ++u) {
    if (u * BM_BLOCK < np) {
      const uint32_t e = ent[u];
      if ((e & BL_IN) && (e & BL_LAST)) {
        const int slot = (int)(e & 0xffffu), sp = (int)((e >> 16) & 0xffu);
        const uint16_t base = L.loff[slot];
        if (base != BL_DROP)
          L.u.list[base + __popcll(L.smask[slot] & ((1ull << sp) - 1ull))] = (uint16_t)(u * BM_BLOCK + tid);
      }
    }
  }
  lds_barrier();

  // P3d: the reference's float32 folds, one thread per kept slot, means out
  int nonfinite = 0;
  if (!(P.ablate & 2)) {
    for (int j = tid; j < K; j += BM_BLOCK) {
      const int d = L.kslot[j];
      const int base = L.loff[d], cn = __popcll(L.smask[d]);
      float am = 0.0f, ai = 0.0f;
      // gathers in batches of 8 (16 loads in flight), folded in list order
      for (int e0 = 0; e0 < cn; e0 += 8) {
        double mm[8], ii[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = e0 + q < cn ? e0 + q : cn - 1;
          const int64_t k = p0 + L.u.list[base + e];
          mm[q] = v.mz[k];
          ii[q] = v.inten[k];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (e0 + q < cn) {
            ai = (float)((double)ai + ii[q]);
            am = (float)((double)am + mm[q]);
          }
        }
      }
      const double cnd = (double)cn;
      const double mi = (double)ai / cnd;
      nonfinite |= isnan(mi);
      out.inten[p0 + j] = mi;
      out.mz[p0 + j] = am == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)am / cnd;
    }
  }
  // a NaN mean would be dropped by the reference (binning.py:209-222): the
  // generic path redoes such clusters with that filter
  if (block_any<BM_BLOCK, true>(nonfinite, L.votes, 0)) { defer(); return; }
  if (tid == 0) {
    out.count[c] = (P.ablate & 2) ? 0 : K;
    charge_out[c] = z0;
    const double* pr = v.prec_mz + s0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return pr[j]; }, n) / (double)n;  // np.mean, n <= 64
    status[c] = kOk;
  }
}

// ------------------------------------------------------------------------
// bin_mean_fold_kernel (variant 2): bins computed ONCE, spectrum-serial fold
// with a trivial per-step body.
//   P1  flat pass over the cluster's peaks (<= 48 per thread, in registers):
//       exact bin (trunc_div_small), LDS occupancy bitmap, and "last peak of its
//       bin in its spectrum" from the neighbour's key (shuffle; lane 63 reads
//       the next wave's lane-0 key after the barrier).  Keys must be
//       non-decreasing inside every spectrum (else: deferred).
//   P2  popcount prefix -> compact slots in ascending bin order.
//   P3a every register entry becomes a u16 code: slot if the peak is the last
//       of its bin in its spectrum, else NONE.
//   P3  codes go to LDS (aliasing the dead bitmap) in spectrum-aligned chunks
//       of <= BF_CODES peaks; the fold walks spectra in file order: lane t
//       reads its code and, if it owns a slot, does the reference's
//       cnt += 1; I = f32(f64(I) + it); M = f32(f64(M) + mz) (binning.py:197-199).
//       m/z and intensity come through an 8-spectrum register prefetch ring; one
//       LDS-only barrier per spectrum.
//   P4  quorum filter and ordered output, as the other kernels.
constexpr int BF_CODES = 7680;  // u16 codes per chunk (= bitmap + prefix bytes)
constexpr uint16_t BF_NONE = 0xFFFFu;
constexpr int BF_PB = 8;  // P1 loads in flight per thread

struct BinFoldSmem {
  union {
    struct {
      unsigned long long bitmap[BM_WMAX];
      uint16_t wprefix[BM_WMAX];
    } b;                       // P1..P3a
    uint16_t code[BF_CODES];   // P3 (per chunk)
  } u;
  uint32_t cnt[BM_DCAP];
  float acc_i[BM_DCAP];
  float acc_m[BM_DCAP];
  int32_t soff[BL_NMAX + 1];
  unsigned long long sbits[BL_SW];
  int32_t xch[BL_UMAX * (BM_BLOCK / kWave)];
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

__global__ __launch_bounds__(BM_BLOCK, 4) void bin_mean_fold_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                 double* prec_out, int32_t* charge_out,
                                                                 int32_t* status, int32_t* deferred,
                                                                 int32_t* n_deferred) {
  static_assert(sizeof(BinFoldSmem::u) >= BF_CODES * 2, "codes alias the bitmap");
  __shared__ BinFoldSmem L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  constexpr int NW = BM_BLOCK / kWave;
  const int64_t c = blockIdx.x;
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  const int np = (int)(p1 - p0);
  auto defer = [&]() {
    if (tid == 0) {
      status[c] = kDeferred;
      deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
  };
  if (n == 0) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kEmpty; }
    return;
  }
  if (n > BL_NMAX || p1 - p0 > BL_PCAP || P.n_words > BM_WMAX) { defer(); return; }

  // P0: charge check (binning.py:205-206), spectrum offsets and starts, zeroing
  const int32_t z0 = v.charge[s0];
  int mixed = 0, longspec = 0;
  if (tid <= n) L.soff[tid] = (int32_t)(v.spec_off[s0 + tid] - p0);
  if (tid < n) mixed = v.charge[s0 + tid] != z0;
  const int nsw = (np + 63) / 64;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.u.b.bitmap[w] = 0ull;
  for (int w = tid; w < nsw; w += BM_BLOCK) L.sbits[w] = 0ull;
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 0)) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kMixedCharge; }
    return;
  }
  if (tid >= 1 && tid < n) {
    const int r = L.soff[tid];
    if (r < np) atomicOr(&L.sbits[r >> 6], 1ull << (r & 63));  // empty spectra share a bit: harmless here
  }
  if (tid < n) longspec = L.soff[tid + 1] - L.soff[tid] > BF_CODES;
  if (block_any<BM_BLOCK, true>(longspec, L.votes, 1)) { defer(); return; }

  // P1
  uint32_t ent[BL_UMAX];
  int bad = 0;
#pragma unroll
  for (int u = 0; u < BL_UMAX; ++u) ent[u] = 0u;
#pragma unroll
  for (int u0 = 0; u0 < BL_UMAX; u0 += BF_PB) {
    if (u0 * BM_BLOCK < np) {  // uniform
      double mb[BF_PB];
#pragma unroll
      for (int q = 0; q < BF_PB; ++q) {
        const int r = (u0 + q) * BM_BLOCK + tid;
        mb[q] = v.mz[p0 + (r < np ? r : 0)];
      }
#pragma unroll
      for (int q = 0; q < BF_PB; ++q) {
        const int u = u0 + q;
        if (u * BM_BLOCK < np) {  // uniform
          const int r = u * BM_BLOCK + tid;
          const bool valid = r < np;
          const double m = mb[q];
          bad |= valid && (m != m);
          const bool inr = valid && in_range(m, P);
          int32_t key = m < P.minimum ? -1 : 0x7fffffff;
          if (inr) {
            key = trunc_div_small(m - P.minimum, P.binsize, P.inv_binsize);
            atomicOr(&L.u.b.bitmap[key >> 6], 1ull << (key & 63));
          }
          const int32_t kn = __shfl_down(key, 1, kWave);
          if (lane == 0) L.xch[u * NW + wid] = key;
          const int rn = r + 1;
          const bool same = valid && rn < np && !((L.sbits[rn >> 6] >> (rn & 63)) & 1ull);
          uint32_t e = inr ? (BL_IN | (uint32_t)key) : (key == 0x7fffffff ? BL_HI : 0u);
          if (lane < kWave - 1) {
            bad |= same && key > kn;
            if (!(same && kn == key)) e |= BL_LAST;
          } else if (same) {
            e |= BL_NXT;
          } else {
            e |= BL_LAST;
          }
          ent[u] = e;
        }
      }
    }
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 0)) { defer(); return; }

  // P2
  const int D = bitmap_prefix<BM_BLOCK>(L.u.b.bitmap, L.u.b.wprefix, P.n_words, L.tmp);
  if (D > BM_DCAP) { defer(); return; }
  for (int d = tid; d < D; d += BM_BLOCK) {
    L.cnt[d] = 0u;
    L.acc_i[d] = 0.0f;
    L.acc_m[d] = 0.0f;
  }

  // P3a: entry -> code (slot of a last peak, else BF_NONE), two u16 codes per register
  uint32_t pk[BL_UMAX / 2];
#pragma unroll
  for (int u = 0; u < BL_UMAX; ++u) {
    uint32_t cd = BF_NONE;
    if (u * BM_BLOCK < np) {
      uint32_t e = ent[u];
      if (e & BL_NXT) {
        const int32_t kx = wid < NW - 1 ? L.xch[u * NW + wid + 1] : L.xch[(u + 1) * NW];
        const int32_t key = (e & BL_IN) ? (int32_t)(e & BL_VAL) : ((e & BL_HI) ? 0x7fffffff : -1);
        bad |= key > kx;
        if (kx != key) e |= BL_LAST;
      }
      if ((e & BL_IN) && (e & BL_LAST))
        cd = (uint32_t)bitmap_rank(L.u.b.bitmap, L.u.b.wprefix, (int64_t)(e & BL_VAL));
    }
    if (u & 1) pk[u >> 1] |= cd << 16;
    else pk[u >> 1] = cd;
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 1)) { defer(); return; }
  if (P.ablate & 1) {
    if (tid == 0) { out.count[c] = 0; status[c] = kOk; }
    return;
  }

  // P3: chunks of whole spectra, codes to LDS, spectrum-serial fold
  constexpr int PF = 4;
  auto fetch = [&](int j, double& m, double& it) {
    const int jj = j < n ? j : n - 1;
    const int a = L.soff[jj], e = L.soff[jj + 1];
    const int k = a + tid < e ? a + tid : 0;
    m = v.mz[p0 + k];
    it = v.inten[p0 + k];
  };
  double Am[PF], Ai[PF], Bm[PF], Bi[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) fetch(j, Am[j], Ai[j]);
  int sa = 0;
  while (sa < n) {  // uniform
    int sb = sa + 1;
    while (sb < n && L.soff[sb + 1] - L.soff[sa] <= BF_CODES) ++sb;
    const int ka = L.soff[sa], kb = L.soff[sb];
#pragma unroll
    for (int u = 0; u < BL_UMAX; ++u) {
      const int r = u * BM_BLOCK + tid;
      if (u * BM_BLOCK < np && r >= ka && r < kb) L.u.code[r - ka] = (uint16_t)(pk[u >> 1] >> (16 * (u & 1)));
    }
    lds_barrier();
    for (int jb = sa; jb < sb; ++jb) {
      // ring: Am/Ai hold spectra [jr, jr + PF) where jr = jb - (jb % PF) relative to 0
      const int q = jb % PF;
      if (q == 0) {
#pragma unroll
        for (int j = 0; j < PF; ++j) fetch(jb + PF + j, Bm[j], Bi[j]);
      }
      double m = 0.0, it = 0.0;
#pragma unroll
      for (int j = 0; j < PF; ++j)
        if (j == q) { m = Am[j]; it = Ai[j]; }
      const int a = L.soff[jb], e = L.soff[jb + 1];
      if (a + tid < e) {
        const uint16_t cd = L.u.code[a - ka + tid];
        if (cd != BF_NONE) {
          L.cnt[cd] += 1u;
          L.acc_i[cd] = (float)((double)L.acc_i[cd] + it);
          L.acc_m[cd] = (float)((double)L.acc_m[cd] + m);
        }
      }
      for (int k = a + BM_BLOCK + tid; k < e; k += BM_BLOCK) {  // spectra longer than the block
        const uint16_t cd = L.u.code[k - ka];
        if (cd != BF_NONE) {
          L.cnt[cd] += 1u;
          L.acc_i[cd] = (float)((double)L.acc_i[cd] + v.inten[p0 + k]);
          L.acc_m[cd] = (float)((double)L.acc_m[cd] + v.mz[p0 + k]);
        }
      }
      if (q == PF - 1) {
#pragma unroll
        for (int j = 0; j < PF; ++j) { Am[j] = Bm[j]; Ai[j] = Bi[j]; }
      }
      lds_barrier();
    }
    sa = sb;
  }
  __syncthreads();

  if (P.ablate & 2) {
    if (tid == 0) { out.count[c] = 0; status[c] = kOk; }
    return;
  }
  // P4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int per = (D + BM_BLOCK - 1) / BM_BLOCK;
  const int d0 = tid * per;
  int mine = 0;
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
    if (d < D && L.cnt[d] >= quorum && !isnan(L.acc_i[d])) ++mine;
  }
  int total;
  int o = block_exclusive_scan<BM_BLOCK>(mine, L.tmp, total);
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
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
    const double* pr = v.prec_mz + s0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return pr[j]; }, n) / (double)n;  // np.mean, n <= 64
    status[c] = kOk;
  }
}

// ------------------------------------------------------------------------
// bin_mean_hash_kernel (variant 3): ONE pass over the cluster's peaks.
//
// The two-pass LDS kernels first stream every m/z to build the occupied-bin
// bitmap (slot = rank of the bin), then stream m/z and intensity again for the
// ordered fold: 24 B of loads per peak.  Here the per-cluster accumulators live
// in an LDS hash table keyed by bin, so the fold starts with the first spectrum
// and every peak is loaded exactly once (16 B per peak, the algorithmic minimum).
//   * spectra in file order through a BH_PF-deep register prefetch ring.  Wave w
//     takes peaks 63w .. 63w+63 of a 252-peak chunk: lane 63 duplicates the next
//     wave's lane 0, so every participating lane finds its successor's key in its
//     own wave (one DPP move) -- no cross-wave exchange; lane 63 never updates.
//   * key = exact trunc(fl((mz - min)/binsize)) (spx_device.hpp); the last peak of
//     each run of equal keys in a spectrum is the one numpy's fancy-index "+="
//     keeps (binning.py:197-199)
//   * table: H bins in groups of 4 (one ds_read_b128 per probe), hashed home
//     group, double-hashed probing over groups; a new bin is claimed by LDS
//     compare-and-swap.  Groups fill left to right, so the first word of a group
//     that is the bin OR empty ends a search.  Counts (u16) and float32
//     accumulators (I, M) in parallel arrays.
//   * update: count += 1; I = f32(f64(I) + it); M = f32(f64(M) + mz) -- the
//     reference's float32 accumulation in spectrum order (one LDS-only barrier
//     per spectrum; bins are unique inside a step, so updates never collide)
//   * end: kept slots (count >= int(0.25 n)+1, mean not NaN) go to an occupancy
//     bitmap (aliasing the accumulators) whose popcount prefix gives each its
//     output position in ascending bin order (binning.py:209-222)
// Deferred to bin_mean_global_kernel: > BM_NMAX spectra, > BM_WMAX bitmap
// words, a key inversion inside a spectrum (unsorted; NaN next to in-range
// peaks), a full table.
constexpr uint32_t BH_EMPTY = 0xFFFFFFFFu;  // never a bin (< 2^17)
constexpr int BH_PF = 8;                    // spectra in flight per lane
constexpr int BH_CHUNK = 4 * (kWave - 1);   // peaks per block step (252)
constexpr int BH_MAXITER = 64;              // probe iterations before a cluster is deferred (table full)

template <int H>
struct BinHashSmem {
  uint32_t key[H];      // bin, or BH_EMPTY
  uint32_t cnt2[H / 2];  // u16 counts, two per word (ds_add_u32 on the right half)
  union {
    float2 acc[H];  // (I, M) float32 running sums
    struct {
      unsigned long long bitmap[BM_WMAX];
      uint16_t wprefix[BM_WMAX];
    } b;  // output ordering (after the fold)
  } u;
  double prec[BM_NMAX];
  int32_t soff[BM_NMAX + 1 + 2 * BH_PF];  // spectrum offsets relative to the cluster's first peak (+ end pad)
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

// home group and probe stride (odd: the sequence visits every group) of a bin.
// Adjacent bins (a jittered peak straddling a bin edge) land far apart.
template <int H>
__device__ __forceinline__ uint32_t bh_home(uint32_t key) {
  constexpr int LG = __builtin_ctz(H / 4);
  return __umul24(key, 0x9E3779u) >> (24 - LG) & (H / 4 - 1);
}
__device__ __forceinline__ uint32_t bh_stride(uint32_t key) { return (__umul24(key, 0x85EBCAu) >> 12) | 1u; }

// First word of a group that is `key` or empty (-1: neither; the group is full
// of other bins).  Sets hit when it is `key`.
__device__ __forceinline__ int bh_find4(const uint4& k, uint32_t key, bool& hit) {
  const bool m0 = k.x == key, m1 = k.y == key, m2 = k.z == key, m3 = k.w == key;
  const bool s0 = m0 | (k.x == BH_EMPTY), s1 = m1 | (k.y == BH_EMPTY), s2 = m2 | (k.z == BH_EMPTY),
             s3 = m3 | (k.w == BH_EMPTY);
  hit = m0 | m1 | m2 | m3;
  return s0 ? 0 : s1 ? 1 : s2 ? 2 : s3 ? 3 : -1;
}

// (S: any LDS layout with members key[H], cnt2[H/2] and u.acc[H])
template <class S>
__device__ __forceinline__ void bh_count_add(S& L, int slot) {
  atomicAdd(&L.cnt2[slot >> 1], 1u << (16 * (slot & 1)));  // ds_add_u32, no return
}
template <class S>
__device__ __forceinline__ void bh_count_set1(S& L, int slot) {
  reinterpret_cast<uint16_t*>(L.cnt2)[slot] = 1;
}
template <class S>
__device__ __forceinline__ uint32_t bh_count(const S& L, int slot) {
  return reinterpret_cast<const uint16_t*>(L.cnt2)[slot];
}

// Slow path of one update: the bin's home group is full of other bins, or
// another lane of this step claimed the empty word first.  Continue the probe
// sequence; returns false if the table is full.
template <int H, class S>
__device__ __forceinline__ bool bh_slow_update(S& L, uint32_t key, uint32_t g, double m, double it) {
  constexpr uint32_t G = H / 4;
  const uint32_t stride = bh_stride(key);
#pragma unroll 1
  for (int iter = 0; iter < BH_MAXITER; ++iter) {
    const uint4 k4 = *reinterpret_cast<const uint4*>(&L.key[g * 4]);
    bool hit;
    const int e = bh_find4(k4, key, hit);
    if (e < 0) {
      g = (g + stride) & (G - 1);
      continue;
    }
    const int slot = (int)g * 4 + e;
    if (hit) {
      const float2 a = L.u.acc[slot];
      bh_count_add(L, slot);
      L.u.acc[slot] = make_float2((float)((double)a.x + it), (float)((double)a.y + m));
      return true;
    }
    if (atomicCAS(&L.key[slot], BH_EMPTY, key) == BH_EMPTY) {
      bh_count_set1(L, slot);
      L.u.acc[slot] = make_float2((float)(0.0 + it), (float)(0.0 + m));
      return true;
    }
    // lost the claim: re-read the same group
  }
  return false;
}

// One lane's peak t of a spectrum of `len` peaks, one fold step (see
// bin_mean_hash_kernel).  A NaN m/z gets key -1: excluded, as numpy's
// (mz >= min) & (mz < max) excludes it (binning.py:191-192); next to in-range
// peaks it reads as an inversion and defers the cluster.  badm collects (per
// wave) lanes that saw a key inversion or a full table.
template <int H, class S>
__device__ __forceinline__ void bh_fold_peak(S& L, const BinMeanParams& P, int lane, int t, int len,
                                             double m, double it, uint64_t& badm) {
  const int32_t b = bin_small(m, P);
  const int32_t key = !(m >= P.minimum) ? -1 : (m < P.maximum ? b : 0x7fffffff);
  const int32_t kn = wave_next(key, 0x7fffffff);
  const bool active = (t < len) & (lane < kWave - 1), has_next = t + 1 < len;
  badm |= __ballot(active & has_next & (key > kn));
  const bool part = active & !(has_next & (kn == key)) & ((uint32_t)key < 0x7fffffffu) & !(P.ablate & 16);
  // probe the home group (every lane: harmless for non-participants)
  const uint32_t uk = (uint32_t)key & 0x1FFFFu;
  const uint32_t g = bh_home<H>(uk);
  const uint4 k4 = *reinterpret_cast<const uint4*>(&L.key[g * 4]);
  bool hit;
  const int e = bh_find4(k4, uk, hit);
  // one more round trip: the accumulators of the found slot and, for a new
  // bin, the claim of the group's first empty word, in flight together
  const int slot = (int)g * 4 + (e < 0 ? 0 : e);
  const float2 a = L.u.acc[slot];  // speculative for non-hits
  const bool ins = part & !hit & (e >= 0) & !(P.ablate & 4);
  uint32_t old = 0u;
  if (ins) old = atomicCAS(&L.key[slot], BH_EMPTY, uk);
  const bool upd = part & hit & !(P.ablate & 8);
  const bool fresh = ins & (old == BH_EMPTY);
  if (upd) bh_count_add(L, slot);
  if (fresh) bh_count_set1(L, slot);
  if (upd | fresh) {
    const float ax = fresh ? 0.0f : a.x, ay = fresh ? 0.0f : a.y;
    L.u.acc[slot] = make_float2((float)((double)ax + it), (float)((double)ay + m));
  }
  if (part & !hit & !fresh & !(P.ablate & 4)) {
    if (!bh_slow_update<H>(L, uk, g, m, it)) badm |= 1ull << lane;
  }
}

template <int H>
__global__ __launch_bounds__(BM_BLOCK) void bin_mean_hash_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                 double* prec_out, int32_t* charge_out,
                                                                 int32_t* status, int32_t* deferred,
                                                                 int32_t* n_deferred) {
  static_assert(sizeof(float2) * H >= sizeof(unsigned long long) * BM_WMAX + sizeof(uint16_t) * BM_WMAX,
                "the ordering bitmap aliases the accumulators");
  constexpr int SPT = H / BM_BLOCK;  // table slots per thread at the end
  static_assert(SPT % 4 == 0, "whole key groups per thread");
  static_assert(BH_PF + 1 <= kWave, "one lane per ring offset");
  __shared__ BinHashSmem<H> L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t c = blockIdx.x;
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  auto defer = [&]() {
    if (tid == 0) {
      status[c] = kDeferred;
      deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
  };
  if (n == 0) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kEmpty; }
    return;
  }
  if (n > BM_NMAX || P.n_words > BM_WMAX) { defer(); return; }
  const int64_t p0 = v.spec_off[s0];
  const double* __restrict__ mzc = v.mz + p0;
  const double* __restrict__ itc = v.inten + p0;

  // P0: offsets (padded with the end offset) and precursors to LDS, charge
  // check (binning.py:205-206), empty table
  const int32_t z0 = v.charge[s0];
  int mixed = 0, longspec = 0;
  // padded with the end offset up to n + 2 BH_PF: the ring reads the offsets of the turn after the last
  for (int j = tid; j <= n + 2 * BH_PF; j += BM_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + (j < n ? j : n)] - p0);
  for (int j = tid; j < n; j += BM_BLOCK) {
    L.prec[j] = v.prec_mz[s0 + j];
    mixed |= v.charge[s0 + j] != z0;
    longspec |= v.spec_off[s0 + j + 1] - v.spec_off[s0 + j] > BH_CHUNK;
  }
#pragma unroll
  for (int q = 0; q < SPT / 4; ++q)
    reinterpret_cast<uint4*>(L.key)[tid + q * BM_BLOCK] = make_uint4(BH_EMPTY, BH_EMPTY, BH_EMPTY, BH_EMPTY);
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 0)) {
    if (tid == 0) { bl_finish_empty(out, prec_out, charge_out, c); status[c] = kMixedCharge; }
    return;
  }
  longspec = block_any<BM_BLOCK, true>(longspec, L.votes, 1);  // also: offsets and empty table visible

  // P1: the ordered fold, one spectrum per step
  const int t0 = (kWave - 1) * wid + lane;  // this lane's peak in a chunk
  // a peak by cluster-relative index: 32-bit byte offsets from a scalar base
  auto ld = [&](const double* base, int k) __attribute__((always_inline)) {
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + (uint32_t)k * 8u);
  };
  uint64_t badm = 0;  // lanes that saw a key inversion (wave mask)
  auto peak = [&](int t, int len, double m, double it) __attribute__((always_inline)) {
    bh_fold_peak<H>(L, P, lane, t, len, m, it, badm);
  };
  const bool any_peaks = v.spec_off[s1] > p0;  // else nothing to fold (and no peak to clamp loads to)
  if (!any_peaks) {
  } else if (longspec) {
    // a spectrum longer than a chunk: no ring (the extra chunks of a step
    // would sit between the ring's loads and their uses)
    for (int j = 0; j < n; ++j) {
      const int a = __builtin_amdgcn_readfirstlane(L.soff[j]);
      const int len = __builtin_amdgcn_readfirstlane(L.soff[j + 1]) - a;
      for (int tb = 0; tb < len; tb += BH_CHUNK) {
        const int t = tb + t0;
        const int k = a + (t < len ? t : 0);
        peak(t, len, ld(mzc, k), ld(itc, k));
      }
      lds_barrier();
    }
  } else {
    // The ring.  Every refill is unconditional (past the last spectrum it
    // reads one line), so no ring register is ever a merge of a load and
    // another value: the compiler waits with a counted vmcnt and BH_PF
    // spectra stay in flight across the LDS-only barriers.  The offsets of a
    // ring turn are read once (lane i: offset jb + i) and handed out by readlane.
    // The ring registers are defined in ONE place (the loop body; the first
    // turn, jb = -BH_PF, only fills), so the allocator keeps each in one
    // register pair with no copies at the loop header.
    double Rm[BH_PF], Ri[BH_PF];
    int Rl[BH_PF];
    for (int jb = -BH_PF; jb < n; jb += BH_PF) {
      const int offs = L.soff[jb + BH_PF + (lane < BH_PF + 1 ? lane : 0)];  // next turn's offsets (padded)
#pragma unroll
      for (int q = 0; q < BH_PF; ++q) {
        const bool live = jb >= 0 && jb + q < n;  // uniform
        if (live) peak(t0, Rl[q], Rm[q], Ri[q]);
        const int a = __builtin_amdgcn_readlane(offs, q);
        const int len = __builtin_amdgcn_readlane(offs, q + 1) - a;
        const int k = len ? a + (t0 < len ? t0 : 0) : 0;
        Rm[q] = ld(mzc, k);
        Ri[q] = ld(itc, k);
        Rl[q] = len;
        if (live) lds_barrier();
      }
    }
  }
  if (block_any<BM_BLOCK, true>(badm != 0, L.votes, 0)) { defer(); return; }
  if (P.ablate & 2) {
    if (tid == 0) { out.count[c] = 0; status[c] = kOk; }
    return;
  }

  // P2: kept slots (binning.py:209-222) into registers; thread owns SPT slots
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  int32_t kk[SPT];
  float ka[SPT], kb[SPT];
  uint32_t kn[SPT];
#pragma unroll
  for (int q = 0; q < SPT; ++q) {
    const int s = tid * SPT + q;
    const uint32_t w = L.key[s];
    const uint32_t cn = bh_count(L, s);
    const float2 a = L.u.acc[s];
    // cnt >= 1, so the mean is NaN iff the float32 sum is
    const bool keep = w != BH_EMPTY && cn >= quorum && !isnan(a.x);
    kk[q] = keep ? (int32_t)w : -1;
    ka[q] = a.x;
    kb[q] = a.y;
    kn[q] = cn;
  }
  lds_barrier();  // accumulators dead: the bitmap takes their place
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.u.b.bitmap[w] = 0ull;
  lds_barrier();
#pragma unroll
  for (int q = 0; q < SPT; ++q)
    if (kk[q] >= 0) atomicOr(&L.u.b.bitmap[kk[q] >> 6], 1ull << (kk[q] & 63));
  lds_barrier();
  const int K = bitmap_prefix<BM_BLOCK>(L.u.b.bitmap, L.u.b.wprefix, P.n_words, L.tmp);
  if (!(P.ablate & 32)) {
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
      if (kk[q] >= 0) {
        const int o = bitmap_rank(L.u.b.bitmap, L.u.b.wprefix, (int64_t)kk[q]);
        const double cnd = (double)kn[q];
        out.inten[p0 + o] = (double)ka[q] / cnd;
        out.mz[p0 + o] = kb[q] == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)kb[q] / cnd;
      }
    }
  }
  if (tid == 0) {
    out.count[c] = K;
    charge_out[c] = z0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return L.prec[j]; }, n) / (double)n;  // np.mean (binning.py:224)
    status[c] = kOk;
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
