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
