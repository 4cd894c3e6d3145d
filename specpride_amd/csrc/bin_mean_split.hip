// Bin-mean for the clusters the register and LDS kernels cannot hold (more than
// 128 spectra, more than 1,536 distinct bins, spectra of any length): the
// cluster's bin axis is split into word-aligned RANGES of <= BM_DCAP occupied
// bins, and one workgroup per range folds the whole cluster in spectrum order
// restricted to its bins (reference: src/binning.py:170-231).  Bins of different
// ranges never interact -- the reference's per-bin sums are independent -- so a
// 5,000-spectrum cluster runs on dozens of workgroups instead of one.
//
//   bin_mean_split_plan_kernel  (one workgroup per deferred cluster)
//       occupancy bitmap in LDS, word popcounts -> ranges (block scan), the
//       mixed-charge check; clusters this path cannot take go on to the
//       global-scratch kernel's list
//   bin_mean_split_fold_kernel  (one workgroup per range)
//       1: the range's occupancy bits from the cluster's peaks, slot prefix
//       2: spectra in order (register ring of the next spectra's peaks): exact bin,
//          last-in-bin by the DPP neighbour key, f32(f64(acc) + v) per slot; a key
//          inversion or NaN flags the cluster (the global kernel redoes it)
//       3: quorum, the range's kept bins in bin order at p0 + (occupied bins of
//          earlier ranges)
//   bin_mean_split_emit_kernel  (one workgroup per planned cluster)
//       ranges' outputs moved together (an in-place left shift), count, charge,
//       np.mean of the precursors; flagged clusters go to the global list
#pragma once
#include "bin_mean.hip"

namespace spx {

constexpr int SP_NMAX = 8192;                        // spectra per cluster (offsets staged in LDS)
constexpr int SP_CAPW = BM_DCAP - 64;                // occupied bins before a range closes (+ one word)
constexpr int SP_PF = 8;                             // spectra in flight per lane
constexpr int SP_POS = 4 * (kWave - 1);              // positions owned per chunk (252)

struct SplitRange {
  int32_t cl;         // planned-cluster index (-1: dropped)
  int32_t w0, w1;     // bitmap words [w0, w1)
  int32_t slot_base;  // occupied bins in earlier ranges (the output offset in the capacity layout)
  int32_t kept;       // bins this range emitted
  int32_t pad;
};
struct SplitCluster {
  int64_t c;
  int32_t first, nr;  // its ranges
  int32_t bad;        // set by a fold: unsorted or NaN -> global kernel
  int32_t pad;
};

struct SplitPlanSmem {
  unsigned long long bits[BM_WMAX];
  int open_w[BM_WMAX];  // opening word of range r
  int open_e[BM_WMAX];  // occupied bins before it
  int tmp[BM_BLOCK / kWave + 1];
  int votes[2 * (BM_BLOCK / kWave)];
  int base, slot;
};

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_split_plan_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    const int32_t* deferred, const int32_t* n_deferred, SplitCluster* scl, int32_t* n_scl, SplitRange* ranges,
    int32_t* n_ranges, int32_t range_cap, int32_t* glist, int32_t* n_glist) {
  __shared__ SplitPlanSmem L;
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t i = blockIdx.x; i < nd; i += gridDim.x) {
    const int64_t c = deferred[i];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n = s1 - s0;
    const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
    if (n < 1 || n > SP_NMAX || P.n_words > BM_WMAX || p1 - p0 >= (int64_t(1) << 31)) {
      if (tid == 0) glist[atomicAdd(n_glist, 1)] = (int32_t)c;
      continue;
    }
    // mixed charges (binning.py:205-206): nothing emitted
    const int32_t z0 = v.charge[s0];
    int mixed = 0;
    for (int64_t s = s0 + 1 + tid; s < s1; s += BM_BLOCK) mixed |= v.charge[s] != z0;
    for (int w = tid; w < P.n_words; w += BM_BLOCK) L.bits[w] = 0ull;
    if (block_any<BM_BLOCK, true>(mixed, L.votes, 0)) {
      if (tid == 0) {
        out.count[c] = 0;
        prec_out[c] = __longlong_as_double(0x7ff8000000000000ll);
        charge_out[c] = 0;
        status[c] = kMixedCharge;
      }
      lds_barrier();  // every wave has read the votes before the next cluster's vote reuses them
      continue;
    }
    // occupancy of the whole cluster (any order, NaN not in range)
    for (int64_t k0 = p0 + tid; k0 < p1; k0 += 8 * BM_BLOCK) {
      double m[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t k = k0 + (int64_t)u * BM_BLOCK;
        m[u] = v.mz[k < p1 ? k : p0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (k0 + (int64_t)u * BM_BLOCK < p1 && in_range(m[u], P)) {
          const int32_t b = bin_small(m[u], P);
          atomicOr(&L.bits[b >> 6], 1ull << (b & 63));
        }
      }
    }
    lds_barrier();
    // ranges: word w opens a range when floor(occupied-before-w / SP_CAPW) steps
    // (so a range holds < SP_CAPW + 64 <= BM_DCAP occupied bins)
    const int nw = P.n_words;
    const int per = (nw + BM_BLOCK - 1) / BM_BLOCK, w0 = tid * per;
    int cnt_local = 0;
    for (int k = 0; k < per; ++k)
      if (w0 + k < nw) cnt_local += __popcll(L.bits[w0 + k]);
    int tot;
    int excl = block_exclusive_scan<BM_BLOCK, int, true>(cnt_local, L.tmp, tot);
    // word 0 opens range 0; word w > 0 opens a range when the band of the occupied
    // bins before it, floor(excl / SP_CAPW), differs from word w-1's (so a range
    // holds < SP_CAPW + 64 <= BM_DCAP occupied bins)
    auto opens_at = [&](int w, int e, int pc_prev) { return w == 0 || (e / SP_CAPW) != ((e - pc_prev) / SP_CAPW); };
    int opens = 0;
    {
      int e = excl, pc_prev = (w0 > 0 && w0 < nw) ? __popcll(L.bits[w0 - 1]) : 0;
      for (int k = 0; k < per; ++k) {
        const int w = w0 + k;
        if (w >= nw) break;
        opens += opens_at(w, e, pc_prev);
        pc_prev = __popcll(L.bits[w]);
        e += pc_prev;
      }
    }
    int nr;
    int ropen = block_exclusive_scan<BM_BLOCK, int, true>(opens, L.tmp, nr);
    // a cluster without in-range peaks needs no range (its output is empty)
    if (tot == 0) nr = 0;
    if (tid == 0) L.base = nr > 0 ? atomicAdd(n_ranges, nr) : -1;
    lds_barrier();
    const int base = L.base;
    if (base >= 0 && base + nr > range_cap) {
      // out of range records: the global kernel takes the cluster; the records it
      // reserved below the cap are marked dropped, so the fold (which walks every
      // record under min(n_ranges, range_cap)) never reads one left unwritten
      for (int r = base + tid; r < range_cap; r += BM_BLOCK) {
        SplitRange R;
        R.cl = -1;
        R.w0 = R.w1 = R.slot_base = R.kept = R.pad = 0;
        ranges[r] = R;
      }
      if (tid == 0) glist[atomicAdd(n_glist, 1)] = (int32_t)c;
      lds_barrier();
      continue;
    }
    // openings (word, occupied bins before it) in LDS, then one record per range
    {
      int e = excl, r = ropen, pc_prev = (w0 > 0 && w0 < nw) ? __popcll(L.bits[w0 - 1]) : 0;
      for (int k = 0; k < per; ++k) {
        const int w = w0 + k;
        if (w >= nw) break;
        if (opens_at(w, e, pc_prev)) {
          L.open_w[r] = w;
          L.open_e[r] = e;
          ++r;
        }
        pc_prev = __popcll(L.bits[w]);
        e += pc_prev;
      }
    }
    if (tid == 0) L.slot = atomicAdd(n_scl, 1);
    lds_barrier();
    const int32_t slot = L.slot;
    for (int r = tid; r < nr; r += BM_BLOCK) {
      SplitRange R;
      R.cl = slot;
      R.w0 = L.open_w[r];
      R.w1 = r + 1 < nr ? L.open_w[r + 1] : nw;
      R.slot_base = L.open_e[r];
      R.kept = 0;
      R.pad = 0;
      ranges[base + r] = R;
    }
    if (tid == 0) {
      SplitCluster S;
      S.c = c;
      S.first = base;
      S.nr = nr;
      S.bad = 0;
      S.pad = 0;
      scl[slot] = S;
    }
    lds_barrier();  // the LDS is reused by the next cluster
  }
}

struct SplitFoldSmem {
  uint32_t bits[2 * BM_WMAX];  // the range's words as 32-bit halves
  uint16_t pre[2 * BM_WMAX];
  float2 acc[BM_DCAP];
  uint32_t cnt[BM_DCAP];
  int32_t soff[SP_NMAX + 1];
  int wcnt[(BM_DCAP / BM_BLOCK) * (BM_BLOCK / kWave)];
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_split_fold_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                       SplitCluster* scl, SplitRange* ranges,
                                                                       const int32_t* n_ranges, int32_t range_cap) {
  __shared__ SplitFoldSmem L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int32_t total = min(*n_ranges, range_cap);
  for (int32_t ri = blockIdx.x; ri < total; ri += gridDim.x) {
    const SplitRange R = ranges[ri];
    if (R.cl < 0) continue;
    const SplitCluster S = scl[R.cl];
    const int64_t c = S.c;
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int n = (int)(s1 - s0);
    const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
    const int np = (int)(p1 - p0);
    const int nw32 = 2 * (R.w1 - R.w0);
    const int32_t klo = R.w0 * 64, khi = R.w1 * 64;  // the range's bins [klo, khi)
    for (int j = tid; j <= n; j += BM_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
    for (int w = tid; w < nw32; w += BM_BLOCK) L.bits[w] = 0u;
    lds_barrier();
    // 1: the range's occupied bins
    const double* __restrict__ mzc = v.mz + p0;
    const double* __restrict__ itc = v.inten + p0;
    for (int r0 = tid; r0 < np; r0 += 8 * BM_BLOCK) {
      double m[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = r0 + u * BM_BLOCK;
        m[u] = mzc[r < np ? r : 0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (r0 + u * BM_BLOCK < np && in_range(m[u], P)) {
          const int32_t b = bin_small(m[u], P);
          if (b >= klo && b < khi) atomicOr(&L.bits[(b - klo) >> 5], 1u << (b & 31));
        }
      }
    }
    lds_barrier();
    const int D = bitmap_prefix32<BM_BLOCK>(L.bits, L.pre, nw32, L.tmp);
    for (int d = tid; d < D; d += BM_BLOCK) {
      L.acc[d] = make_float2(0.0f, 0.0f);
      L.cnt[d] = 0u;
    }
    lds_barrier();

    // 2: the ordered fold.  Lane mapping of the register kernel: wave w's lanes
    // 0..62 own positions 63w..63w+62 of a 252-position chunk, lane 63 reads the
    // next position only for its neighbour key.  The work items are the (spectrum,
    // chunk) pairs in order (a spectrum of > 252 peaks takes several); a fetch
    // cursor runs SP_PF items ahead of the consumer, so every item's peaks are in
    // flight SP_PF steps before they are used.  One barrier after each spectrum.
    const int fpos = wid * (kWave - 1) + lane;
    const bool owner = lane < kWave - 1;
    struct Pk { double m, it; };
    // kLong: some spectrum exceeds one chunk.  Otherwise every item is a whole
    // spectrum and the cursor is just the spectrum index (cheaper per step).
    int maxlen = 0;
    for (int j = tid; j < n; j += BM_BLOCK) maxlen = max(maxlen, L.soff[j + 1] - L.soff[j]);
    const bool any_long = block_any<BM_BLOCK, true>(maxlen > SP_POS, L.votes, 1);
    int bad = 0;
    auto fold = [&](auto long_tag) __attribute__((always_inline)) {
      constexpr bool kLong = decltype(long_tag)::value;
      // uniform item cursors: spectrum j, chunk start c0
      auto next_item = [&](int& j, int& c0) __attribute__((always_inline)) {
        if constexpr (kLong) {
          const int len = j < n ? L.soff[j + 1] - L.soff[j] : 0;
          c0 += SP_POS;
          if (c0 >= len) { ++j; c0 = 0; }
        } else {
          ++j;
        }
      };
      auto fetch = [&](int j, int c0) __attribute__((always_inline)) -> Pk {
        const int jj = j < n ? j : n - 1;
        const int a = L.soff[jj], e = L.soff[jj + 1];
        const int k = a + c0 + fpos;
        const int idx = (j < n && k < e) ? k : 0;
        return Pk{mzc[idx], itc[idx]};
      };
      Pk ring[SP_PF];
      int fj = 0, fc = 0;  // fetch cursor
#pragma unroll
      for (int q = 0; q < SP_PF; ++q) {
        ring[q] = fetch(fj, fc);
        next_item(fj, fc);
      }
      int cj = 0, cc = 0;  // consume cursor
      while (cj < n) {  // uniform
#pragma unroll
        for (int q = 0; q < SP_PF; ++q) {
          if (cj < n) {  // uniform
            const int len = L.soff[cj + 1] - L.soff[cj];
            const Pk pk = ring[q];
            ring[q] = fetch(fj, fc);
            next_item(fj, fc);
            const int pos = cc + fpos;
            const bool act = pos < len;
            const bool inr = act && in_range(pk.m, P);
            const int32_t kb = bin_small(inr ? pk.m : P.minimum, P);
            const int32_t key = inr ? kb : ((act && pk.m < P.minimum) ? -1 : 0x7fffffff);
            const int32_t kn = wave_next(key, 0x7fffffff);
            bad |= (int)(owner && act && ((pk.m != pk.m) || key > kn));
            if (owner && inr && kn != key && key >= klo && key < khi) {
              const uint32_t b = (uint32_t)(key - klo), w = b >> 5;
              const int slot = (int)L.pre[w] + __popc(L.bits[w] & ((1u << (b & 31)) - 1u));
              float2 s = L.acc[slot];
              s.x = (float)((double)s.x + pk.it);
              s.y = (float)((double)s.y + pk.m);
              L.acc[slot] = s;
              L.cnt[slot] += 1u;
            }
            const int pj = cj;
            next_item(cj, cc);
            if (cj != pj) lds_barrier();  // spectrum pj's updates before the next spectrum's
          }
        }
      }
    };
    if (any_long)
      fold(std::true_type{});
    else
      fold(std::false_type{});
    if (block_any<BM_BLOCK, true>(bad, L.votes, 0)) {
      if (tid == 0) atomicOr(&scl[R.cl].bad, 1);
      continue;
    }
    // 3: this range's kept bins, in bin order, at p0 + slot_base
    const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
    const int kept = emit_striped(L.cnt, [&](int d) { return L.acc[d].x; }, [&](int d) { return L.acc[d].y; },
                                  L.wcnt, D, quorum, out.mz + p0 + R.slot_base, out.inten + p0 + R.slot_base);
    if (tid == 0) ranges[ri].kept = kept;
    lds_barrier();
  }
}

__global__ __launch_bounds__(BM_BLOCK) void bin_mean_split_emit_kernel(CsrView v, BinMeanParams P, PeaksOut out,
                                                                       double* prec_out, int32_t* charge_out,
                                                                       int32_t* status, const SplitCluster* scl,
                                                                       const int32_t* n_scl, const SplitRange* ranges,
                                                                       int32_t* glist, int32_t* n_glist) {
  const int tid = threadIdx.x;
  const int32_t ns = *n_scl;
  for (int32_t i = blockIdx.x; i < ns; i += gridDim.x) {
    const SplitCluster S = scl[i];
    const int64_t c = S.c;
    if (S.bad) {
      if (tid == 0) glist[atomicAdd(n_glist, 1)] = (int32_t)c;
      continue;
    }
    const int64_t s0 = v.cluster_off[c], n = v.cluster_off[c + 1] - s0;
    const int64_t p0 = v.spec_off[s0];
    // ranges' kept blocks moved together in order (destination <= source): per
    // 256-element chunk, read, barrier, write
    int64_t dst = 0;
    for (int r = 0; r < S.nr; ++r) {
      const SplitRange R = ranges[S.first + r];
      const int64_t src = R.slot_base;
      if (src != dst) {
        for (int64_t o = 0; o < R.kept; o += BM_BLOCK) {
          const int64_t k = o + tid;
          double a = 0.0, b = 0.0;
          if (k < R.kept) { a = out.mz[p0 + src + k]; b = out.inten[p0 + src + k]; }
          __syncthreads();
          if (k < R.kept) { out.mz[p0 + dst + k] = a; out.inten[p0 + dst + k] = b; }
          __syncthreads();
        }
      }
      dst += R.kept;
    }
    if (tid == 0) {
      out.count[c] = dst;
      charge_out[c] = v.charge[s0];
      prec_out[c] = pw_sum([&](int64_t j) { return v.prec_mz[s0 + j]; }, n) / (double)n;  // np.mean (binning.py:224)
      status[c] = kOk;
    }
  }
}

}  // namespace spx
