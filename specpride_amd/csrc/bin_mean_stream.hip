// bin_mean_stream_kernel: the default bin-mean kernel (reference: src/binning.py:170-231,
// combine_bin_mean; semantics in SURVEY.md Appendix A.1).
//
// Why a persistent kernel.  One workgroup per cluster (bin_mean_lds_kernel,
// bin_mean_hash_kernel) is latency-bound, not bandwidth-bound: every cluster
// starts with a dependent chain (cluster_off -> spec_off -> first peaks) and a
// mean cluster holds only ~83 KB, so at the 5 workgroups per CU the LDS allows,
// most of a workgroup's life is spent waiting on that chain.  Here each
// workgroup owns ONE contiguous range of clusters (range_plan_kernel: cut so
// every range has about the same weight peaks + 64 spectra + 1024 clusters)
// and walks its spectra as a single stream:
//   * spectra in file order through an 8-deep register ring (lane t = peak t of
//     the spectrum, 252 peaks per step: wave w takes peaks 63w..63w+63, lane 63
//     duplicating the next wave's lane 0 so every lane finds its successor's key
//     inside its own wave).  The ring never drains at a cluster boundary: the
//     spectra after the current cluster's last one are the next cluster's first.
//   * the spectrum offsets, precursor m/z and charges the ring needs come in
//     lane-distributed vectors two turns ahead; cluster ends come from a
//     64-cluster window of cluster_off held in one register.
//   * the fold is bin_mean_hash_kernel's: per-cluster LDS hash table keyed by
//     bin, the last peak of each run of equal keys in a spectrum (numpy's
//     fancy-index "+=" keeps the last, binning.py:197-199) does
//     count += 1; I = f32(f64(I) + it); M = f32(f64(M) + mz)
//     in spectrum order, one LDS-only barrier per spectrum.
//   * at a cluster end the table is drained (kept bins, quorum int(0.25 n)+1,
//     binning.py:181-183, 209-222, ordered by a popcount prefix over a bin
//     bitmap aliasing the accumulators), reset, and the stream continues.
// Every barrier is LDS-only (lds_barrier), so the ring's loads stay in flight
// through the drain.  HBM traffic: 16 B per peak read once, 20 B per spectrum,
// 16 B per output peak.
// Deferred to bin_mean_global_kernel (exact generic path): > BM_NMAX spectra,
// a spectrum longer than 252 peaks, a key inversion inside a spectrum
// (unsorted m/z, or NaN next to in-range peaks), a full table.
#include "bin_mean.hip"

#ifndef SPX_BS_PF
#define SPX_BS_PF 7
#endif

namespace spx {

constexpr int BS_BLOCKS_PER_CU = 5;  // LDS: 5 x 30 KB tables per CU
constexpr int BS_H = 2048;           // table slots per workgroup
constexpr int BS_PF = SPX_BS_PF;     // ring depth: spectra in flight per workgroup
constexpr int BS_PLAN_MAX = 8192;    // workgroups the plan buffer can describe

// Range weight of the clusters before c (non-decreasing in c, < W for c < C).
__device__ __forceinline__ int64_t range_weight(const CsrView& v, int64_t c) {
  const int64_t s = v.cluster_off[c];
  return (v.spec_off[s] - v.spec_off[v.cluster_off[0]]) + 64 * (s - v.cluster_off[0]) + 1024 * c;
}

// plan[b] = first cluster of workgroup b (plan[G] = C): cluster c belongs to
// workgroup floor(weight(c) * G / W), so every workgroup gets a contiguous
// range of about W / G.
__global__ __launch_bounds__(256) void range_plan_kernel(CsrView v, int32_t G, int32_t* plan) {
  const int64_t C = v.n_clusters;
  const int64_t W = range_weight(v, C);
  auto blk = [&](int64_t c) -> int64_t { return c == C ? G : (W > 0 ? range_weight(v, c) * G / W : 0); };
  for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c <= C; c += (int64_t)gridDim.x * 256) {
    const int64_t bc = blk(c), bp = c == 0 ? -1 : blk(c - 1);
    for (int64_t b = bp + 1; b <= bc; ++b) plan[b] = (int32_t)c;
  }
}

// Block exclusive scan with LDS-only barriers (keeps register prefetches in flight).
template <int BLOCK, class T>
__device__ __forceinline__ T block_exclusive_scan_lds(T v, T* tmp, T& total) {
  constexpr int NW = BLOCK / kWave;
  const T inc = wave_inclusive_sum(v);
  if (lane_id() == kWave - 1) tmp[wave_id()] = inc;
  lds_barrier();
  T base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const T t = tmp[w];
    base += (w < wave_id()) ? t : T(0);
    tot += t;
  }
  total = tot;
  return base + inc - v;
}


// Lane-distributed look-ahead of one turn, ONE register: lane i of lanes 0..15
// holds the low word of spectrum (j0 + i)'s start offset (relative to the
// workgroup's first peak after subtracting its low word), lanes 16..31 its
// charge, lanes 32..47 / 48..63 the low / high word of its precursor m/z.
// Spectra past the stream end are clamped to it.
__device__ __forceinline__ uint32_t stream_ahead(const CsrView& v, int64_t S0, int64_t S1, int64_t j0) {
  const int l = lane_id(), f = l >> 4, i = l & 15;
  const int64_t s = S0 + j0 + i < S1 ? S0 + j0 + i : S1;
  const int64_t sp = s < S1 ? s : S1 - 1;  // S1 > S0 here
  const uint32_t* p = f == 0   ? reinterpret_cast<const uint32_t*>(v.spec_off + s)
                      : f == 1 ? reinterpret_cast<const uint32_t*>(v.charge + sp)
                               : reinterpret_cast<const uint32_t*>(v.prec_mz + sp) + (f - 2);
  return *p;
}
__device__ __forceinline__ int ahead_off(uint32_t A, int q, uint32_t pb_lo) {
  return (int)(__builtin_amdgcn_readlane(A, q) - pb_lo);
}
__device__ __forceinline__ int32_t ahead_z(uint32_t A, int q) { return (int32_t)__builtin_amdgcn_readlane(A, 16 + q); }
__device__ __forceinline__ double ahead_prec(uint32_t A, int q) {
  const uint32_t lo = __builtin_amdgcn_readlane(A, 32 + q), hi = __builtin_amdgcn_readlane(A, 48 + q);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// numpy's pairwise sum (spx_device.hpp pw_sum_small) of x[0..n), n <= 128, by
// one whole wave with two registers per lane: lane k < 8 runs accumulator k,
// shuffles combine them ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) (IEEE addition is
// commutative, so either lane's order gives the same bits), lane 0 adds the
// sequential tail.  The result is valid on lane 0.
__device__ __forceinline__ double pw_sum_wave(const double* x, int n) {
  const int lane = lane_id();
  double r = 0.0;
  if (n < 8) {
    if (lane == 0)
      for (int j = 0; j < n; ++j) r += x[j];
    return 0.0 + r;
  }
  const int lim = n - n % 8;
  if (lane < 8) {
    r = x[lane];
    for (int j = 8 + lane; j < lim; j += 8) r += x[j];
  }
  r += __shfl_xor(r, 1, kWave);
  r += __shfl_xor(r, 2, kWave);
  r += __shfl_xor(r, 4, kWave);
  if (lane == 0)
    for (int j = lim; j < n; ++j) r += x[j];
  return 0.0 + r;
}

__device__ double g_spx_zero_peak[2];  // load target of a workgroup with no peaks at all

// LDS of one workgroup (30 KB: 5 per CU).  During the drain, key + cnt2 (12 KB
// = BM_WMAX u64 words at H = 2048) hold the ordering bitmap of the kept bins;
// the accumulators stay untouched until their slot's output is written.
template <int H>
struct alignas(16) BinStreamSmem {
  uint32_t key[H];       // bin, or BH_EMPTY
  uint32_t cnt2[H / 2];  // u16 counts, two per word
  struct {
    float2 acc[H];       // (I, M) float32 running sums
  } u;
  union {
    double prec[BM_NMAX];    // fold: precursor m/z of the cluster's spectra (np.mean at the drain's start)
    uint16_t pre[BM_WMAX];   // drain: kept bins before each bitmap word
  } v;
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};


template <int H>
__global__ __launch_bounds__(BM_BLOCK, BS_BLOCKS_PER_CU) void bin_mean_stream_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    int32_t* deferred, int32_t* n_deferred, const int32_t* plan) {
  constexpr int SPT = H / BM_BLOCK;  // table slots per thread in the drain
  static_assert(SPT == 8, "drain reads two uint4 of keys per thread");
  static_assert(sizeof(uint32_t) * H * 3 / 2 == sizeof(uint64_t) * BM_WMAX, "the bitmap is key + cnt2");
  __shared__ BinStreamSmem<H> L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t cb0 = plan[blockIdx.x], cb1 = plan[blockIdx.x + 1];
  if (cb0 >= cb1) return;
  const int64_t S0 = v.cluster_off[cb0], S1 = v.cluster_off[cb1];
  const int64_t NS = S1 - S0;
  const int64_t PB = NS > 0 ? v.spec_off[S0] : 0;
  const bool has_peaks = NS > 0 && v.spec_off[S1] > PB;
  // peak k of the workgroup's range: 32-bit offsets from a scalar base (the
  // host keeps a range below 2^28 peaks)
  const double* __restrict__ mzb = has_peaks ? v.mz + PB : g_spx_zero_peak;
  const double* __restrict__ itb = has_peaks ? v.inten + PB : g_spx_zero_peak;
  auto ld64 = [](const double* base, uint32_t k) __attribute__((always_inline)) {
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + k * 8u);
  };

  // empty table
#pragma unroll
  for (int q = 0; q < SPT / 4; ++q)
    reinterpret_cast<uint4*>(L.key)[tid + q * BM_BLOCK] = make_uint4(BH_EMPTY, BH_EMPTY, BH_EMPTY, BH_EMPTY);

  // cluster window: lane i holds cluster_off[cwb + i] - S0 (clamped at cb1)
  int32_t cwb = (int32_t)cb0 + 1;
  auto load_window = [&](int32_t base) __attribute__((always_inline)) {
    const int64_t cc = base + lane < cb1 ? base + lane : cb1;
    return (int32_t)(v.cluster_off[cc] - S0);
  };
  int32_t cw = load_window(cwb);
  auto cluster_end = [&](int32_t cl) __attribute__((always_inline)) {  // stream index where cluster cl ends
    if (cl + 1 - cwb >= kWave) {  // calls come in non-decreasing cl
      cwb = cl + 1;
      cw = load_window(cwb);
    }
    return __builtin_amdgcn_readlane(cw, cl + 1 - cwb);
  };

  // The stream is cut into TURNS of <= BS_PF spectra that never cross a cluster
  // end: turn = (ts, tl) spectra [ts, ts + tl) of cluster c = [cs, ce).
  struct Turn {
    int32_t ts, tl, c, cs, ce;
  };
  auto next_turn = [&](const Turn& t) __attribute__((always_inline)) {
    Turn r;
    r.ts = t.ts + t.tl;
    r.c = t.c;
    r.cs = t.cs;
    r.ce = t.ce;
    while (r.c < (int32_t)cb1 && r.ce <= r.ts) {  // past the cluster's end (empty clusters included)
      ++r.c;
      r.cs = r.ts;
      r.ce = r.c < (int32_t)cb1 ? cluster_end(r.c) : r.ts;
    }
    r.tl = r.c < (int32_t)cb1 ? (r.ce - r.ts < BS_PF ? r.ce - r.ts : BS_PF) : 0;
    return r;
  };

  int32_t z0 = 0;
  int64_t cp0 = 0;
  int mixed = 0, vpar = 0;
  uint64_t badm = 0;  // lanes that saw a key inversion / full table (this wave)

  auto emit_empty = [&](int64_t cl) __attribute__((always_inline)) {
    if (tid == 0) {
      bl_finish_empty(out, prec_out, charge_out, cl);
      status[cl] = kEmpty;
    }
  };
  auto finish = [&](int64_t c, int n) __attribute__((always_inline)) {
    // the cluster's last fold step ended with a barrier: the table is complete
    const int bad = block_any<BM_BLOCK, true>(badm != 0, L.votes, vpar) | (n > BM_NMAX);
    vpar ^= 1;
    badm = 0;
    unsigned long long* const bitmap = reinterpret_cast<unsigned long long*>(L.key);  // key + cnt2, during the drain
    if (mixed | bad) {  // uniform: nothing is emitted, the table is reset
      if (tid == 0) {
        if (mixed) {
          bl_finish_empty(out, prec_out, charge_out, c);
          status[c] = kMixedCharge;
        } else {
          status[c] = kDeferred;
          deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
        }
      }
    } else {
      // np.mean of the precursors (binning.py:224) before the prefix overwrites them
      double pmean = 0.0;
      if (tid == 0) pmean = pw_sum_small([&](int64_t j) { return L.v.prec[j]; }, n) / (double)n;
      // drain: thread t owns slots 8t .. 8t+7
      const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
      const uint4 k0 = reinterpret_cast<const uint4*>(L.key)[2 * tid];
      const uint4 k1 = reinterpret_cast<const uint4*>(L.key)[2 * tid + 1];
      const uint4 cq = reinterpret_cast<const uint4*>(L.cnt2)[tid];
      const uint32_t kw[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
      const uint32_t cw2[4] = {cq.x, cq.y, cq.z, cq.w};
      int32_t kk[SPT];
#pragma unroll
      for (int q = 0; q < SPT; ++q) {
        const uint32_t cn = (cw2[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
        // cnt >= 1, so the mean is NaN iff the float32 sum is
        const bool keep = kw[q] != BH_EMPTY && cn >= quorum && !isnan(L.u.acc[SPT * tid + q].x);
        kk[q] = keep ? (int32_t)kw[q] : -1;
      }
      lds_barrier();  // keys and counts read: the ordering bitmap takes their place
#pragma unroll
      for (int q = 0; q < 3; ++q) reinterpret_cast<uint4*>(bitmap)[tid + q * BM_BLOCK] = make_uint4(0u, 0u, 0u, 0u);
      lds_barrier();
#pragma unroll
      for (int q = 0; q < SPT; ++q)
        if (kk[q] >= 0) atomicOr(&bitmap[kk[q] >> 6], 1ull << (kk[q] & 63));
      lds_barrier();
      // exclusive popcount prefix per word (BM_WMAX / BM_BLOCK = 6 words per thread)
      int K;
      {
        constexpr int WPT = BM_WMAX / BM_BLOCK;
        int pc[WPT], sum = 0;
#pragma unroll
        for (int r = 0; r < WPT; ++r) {
          pc[r] = __popcll(bitmap[WPT * tid + r]);
          sum += pc[r];
        }
        int base = block_exclusive_scan_lds<BM_BLOCK>(sum, L.tmp, K);
#pragma unroll
        for (int r = 0; r < WPT; ++r) {
          L.v.pre[WPT * tid + r] = (uint16_t)base;
          base += pc[r];
        }
      }
      lds_barrier();
      if (!(P.ablate & 32)) {
#pragma unroll
        for (int q = 0; q < SPT; ++q) {
          if (kk[q] >= 0) {
            const int o = bitmap_rank(bitmap, L.v.pre, (int64_t)kk[q]);
            const uint32_t cn = (cw2[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
            const float2 a = L.u.acc[SPT * tid + q];
            const double cnd = (double)cn;
            out.inten[cp0 + o] = (double)a.x / cnd;
            out.mz[cp0 + o] = a.y == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)a.y / cnd;
          }
        }
      }
      if (tid == 0) {
        out.count[c] = K;
        charge_out[c] = z0;
        prec_out[c] = pmean;
        status[c] = kOk;
      }
      lds_barrier();  // bitmap reads done: the keys are reset below
    }
#pragma unroll
    for (int q = 0; q < SPT / 4; ++q)
      reinterpret_cast<uint4*>(L.key)[2 * tid + q] = make_uint4(BH_EMPTY, BH_EMPTY, BH_EMPTY, BH_EMPTY);
    lds_barrier();  // empty table before the next cluster's first step
  };
  const int t0 = (kWave - 1) * wid + lane;  // this lane's peak in a step
  Turn cur{0, 0, (int32_t)cb0, 0, (int32_t)cb0 < (int32_t)cb1 ? cluster_end((int32_t)cb0) : 0};
  cur = next_turn(cur);
  for (int64_t cl = cb0; cl < cur.c; ++cl) emit_empty(cl);  // leading empty clusters
  if (cur.tl > 0) {
    Turn nx = next_turn(cur), nn = next_turn(nx);
    const uint32_t pb_lo = (uint32_t)PB;
    uint32_t A0 = stream_ahead(v, S0, S1, cur.ts), A1 = stream_ahead(v, S0, S1, nx.ts);
    double Rm[BS_PF], Ri[BS_PF];
    int Rl[BS_PF];
    // refill slot q with spectrum q of turn t (offsets from A; len 0 past the turn)
    auto refill = [&](int q, const Turn& t, uint32_t A) __attribute__((always_inline)) {
      const int a = ahead_off(A, q, pb_lo);
      const int len = q < t.tl ? ahead_off(A, q + 1, pb_lo) - a : 0;
      const uint32_t k = len > 0 ? (uint32_t)(a + (t0 < len ? t0 : 0)) : 0u;
      Rm[q] = ld64(mzb, k);
      Ri[q] = ld64(itb, k);
      Rl[q] = len;
    };
#pragma unroll
    for (int q = 0; q < BS_PF; ++q) refill(q, cur, A0);
    lds_barrier();  // empty table visible
    while (cur.tl > 0) {  // uniform
      const uint32_t A2 = stream_ahead(v, S0, S1, nn.ts);  // offsets for the next turn's refills
      if (cur.ts == cur.cs) {  // first turn of a cluster
        z0 = ahead_z(A0, 0);
        cp0 = PB + ahead_off(A0, 0, pb_lo);
        mixed = 0;
      }
#pragma unroll
      for (int q = 0; q < BS_PF; ++q) {
        const bool live = q < cur.tl;  // uniform
        if (live) {
          mixed |= ahead_z(A0, q) != z0;
          const int jc = cur.ts - cur.cs + q;  // spectrum index inside the cluster
          if (tid == 0 && jc < BM_NMAX) L.v.prec[jc] = ahead_prec(A0, q);
          if (Rl[q] > BH_CHUNK) badm |= 1ull;  // peaks past the step width: generic path
          bh_fold_peak<H>(L, P, lane, t0, Rl[q], Rm[q], Ri[q], badm);
        }
        refill(q, nx, A1);  // unconditional: BS_PF spectra stay in flight (counted vmcnt)
        if (live) lds_barrier();
      }
      if (cur.ts + cur.tl == cur.ce) {  // the turn ends its cluster
        finish(cur.c, cur.ce - cur.cs);
        for (int64_t cl = cur.c + 1; cl < nx.c; ++cl) emit_empty(cl);  // empty clusters in between
      }
      cur = nx;
      nx = nn;
      nn = next_turn(nn);
      A0 = A1;
      A1 = A2;
    }
  } else {
    for (int64_t cl = cur.c; cl < cb1; ++cl) emit_empty(cl);
  }
}

// ------------------------------------------------------------------------
// bin_mean_stream2_kernel (variant 6): the persistent stream with the
// bitmap-rank fold instead of the hash table.  Per cluster the stream carries
// two passes of turns:
//   A  (<= 2 BS_PF spectra per turn, no barriers): every in-range peak sets its
//      bin in an LDS occupancy bitmap (ds_or_b64); at the cluster's last A-turn
//      a popcount prefix gives each occupied bin its slot, in ascending bin order
//   B  (<= BS_PF spectra per turn, one LDS-only barrier per spectrum): the last
//      peak of each run of equal bins in a spectrum (binning.py:197-199) does
//      count += 1; I = f32(f64(I) + it); M = f32(f64(M) + mz) at slot
//      rank(bin) = pre[w] + popcount(word & below) -- two LDS reads, no probing
// The drain walks the slots (already in bin order): quorum (binning.py:181-183),
// a block scan for the output positions (binning.py:209-222), and re-zeroes the
// bitmap.  A-turns read m/z only (the ring's second register set carries the
// second half of the turn's spectra); B-turns read m/z and intensity.  The
// A-pass m/z is re-read by the B-pass a few microseconds later (L2 / MALL).
// Deferred: > BM_NMAX spectra, > BM_DCAP distinct bins, a spectrum longer than
// 252 peaks, a key inversion inside a spectrum.
struct alignas(16) BinStream2Smem {
  unsigned long long bitmap[BM_WMAX];  // occupied bins of the cluster (A), rank base (B)
  uint16_t pre[BM_WMAX];               // occupied bins before each word
  uint32_t cnt2[BM_DCAP / 2];          // u16 counts, two per word
  float2 acc[BM_DCAP];                 // (I, M) float32 running sums, slot = rank of the bin
  double prec[BM_NMAX];                // precursor m/z of the cluster's spectra
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

__global__ __launch_bounds__(BM_BLOCK, BS_BLOCKS_PER_CU) void bin_mean_stream2_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    int32_t* deferred, int32_t* n_deferred, const int32_t* plan) {
  constexpr int WPT = BM_WMAX / BM_BLOCK;  // bitmap words per thread (6)
  constexpr int SPT2 = BM_DCAP / BM_BLOCK; // slots per thread in the drain (6)
  constexpr int PFA = 2 * BS_PF;           // spectra per A-turn
  static_assert(PFA <= 15, "A-turn offsets fit lanes 0..15 of the look-ahead");
  __shared__ BinStream2Smem L;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t cb0 = plan[blockIdx.x], cb1 = plan[blockIdx.x + 1];
  if (cb0 >= cb1) return;
  const int64_t S0 = v.cluster_off[cb0], S1 = v.cluster_off[cb1];
  const int64_t NS = S1 - S0;
  const int64_t PB = NS > 0 ? v.spec_off[S0] : 0;
  const bool has_peaks = NS > 0 && v.spec_off[S1] > PB;
  const double* __restrict__ mzb = has_peaks ? v.mz + PB : g_spx_zero_peak;
  const double* __restrict__ itb = has_peaks ? v.inten + PB : g_spx_zero_peak;
  auto ld64 = [](const double* base, uint32_t k) __attribute__((always_inline)) {
    return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(base) + k * 8u);
  };

#pragma unroll
  for (int r = 0; r < WPT; ++r) L.bitmap[WPT * tid + r] = 0ull;

  int32_t cwb = (int32_t)cb0 + 1;
  auto load_window = [&](int32_t base) __attribute__((always_inline)) {
    const int64_t cc = base + lane < cb1 ? base + lane : cb1;
    return (int32_t)(v.cluster_off[cc] - S0);
  };
  int32_t cw = load_window(cwb);
  auto cluster_end = [&](int32_t cl) __attribute__((always_inline)) {
    if (cl + 1 - cwb >= kWave) {
      cwb = cl + 1;
      cw = load_window(cwb);
    }
    return __builtin_amdgcn_readlane(cw, cl + 1 - cwb);
  };

  // turns: phase 0 = A (bitmap), 1 = B (fold); spectra [ts, ts + tl) of cluster c = [cs, ce)
  struct Turn {
    int32_t ts, tl, c, cs, ce, ph;
  };
  auto a_len = [](int32_t e, int32_t s) { return e - s < PFA ? e - s : PFA; };
  auto b_len = [](int32_t e, int32_t s) { return e - s < BS_PF ? e - s : BS_PF; };
  auto next_turn = [&](const Turn& t) __attribute__((always_inline)) {
    Turn r = t;
    const int32_t e = t.ts + t.tl;
    if (t.tl == 0) return r;  // past the end
    if (t.ph == 0) {
      if (e < t.ce) { r.ts = e; r.tl = a_len(t.ce, e); }
      else { r.ph = 1; r.ts = t.cs; r.tl = b_len(t.ce, t.cs); }
      return r;
    }
    if (e < t.ce) { r.ts = e; r.tl = b_len(t.ce, e); return r; }
    r.ph = 0;
    r.ts = e;
    while (r.c < (int32_t)cb1 && r.ce <= r.ts) {  // next non-empty cluster
      ++r.c;
      r.cs = r.ts;
      r.ce = r.c < (int32_t)cb1 ? cluster_end(r.c) : r.ts;
    }
    r.tl = r.c < (int32_t)cb1 ? a_len(r.ce, r.ts) : 0;
    return r;
  };

  int32_t z0 = 0;
  int64_t cp0 = 0;
  int mixed = 0, vpar = 0, D = 0;
  uint64_t badm = 0;

  auto emit_empty = [&](int64_t cl) __attribute__((always_inline)) {
    if (tid == 0) {
      bl_finish_empty(out, prec_out, charge_out, cl);
      status[cl] = kEmpty;
    }
  };
  // end of the A-pass: slots in bin order; the B-pass accumulators zeroed
  auto slots = [&](int n) __attribute__((always_inline)) {
    lds_barrier();  // every bit set
    int pc[WPT], sum = 0;
#pragma unroll
    for (int r = 0; r < WPT; ++r) {
      pc[r] = __popcll(L.bitmap[WPT * tid + r]);
      sum += pc[r];
    }
    int base = block_exclusive_scan_lds<BM_BLOCK>(sum, L.tmp, D);
#pragma unroll
    for (int r = 0; r < WPT; ++r) {
      L.pre[WPT * tid + r] = (uint16_t)base;
      base += pc[r];
    }
    if (D > BM_DCAP) badm |= 1ull;  // (uniform) too many distinct bins: generic path
#pragma unroll
    for (int r = 0; r < SPT2; ++r) {
      const int d = SPT2 * tid + r;
      if (d < D) L.acc[d] = make_float2(0.0f, 0.0f);
    }
#pragma unroll
    for (int r = 0; r < BM_DCAP / 2 / BM_BLOCK; ++r) {
      const int w = (BM_DCAP / 2 / BM_BLOCK) * tid + r;
      if (2 * w < D) L.cnt2[w] = 0u;
    }
    (void)n;
    lds_barrier();
  };
  // end of the B-pass: outputs, then the bitmap is zeroed for the next cluster
  auto finish = [&](int64_t c, int n) __attribute__((always_inline)) {
    const int bad = block_any<BM_BLOCK, true>(badm != 0, L.votes, vpar) | (n > BM_NMAX);
    vpar ^= 1;
    badm = 0;
    if (mixed | bad) {
      if (tid == 0) {
        if (mixed) {
          bl_finish_empty(out, prec_out, charge_out, c);
          status[c] = kMixedCharge;
        } else {
          status[c] = kDeferred;
          deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
        }
      }
    } else {
      const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
      // thread t: slots SPT2 t .. SPT2 t + SPT2 - 1 (bin order)
      int kept = 0;
      uint32_t keep_bits = 0;
#pragma unroll 1
      for (int r = 0; r < SPT2; ++r) {
        const int d = SPT2 * tid + r;
        if (d < D) {
          const uint32_t cn = reinterpret_cast<const uint16_t*>(L.cnt2)[d];
          const bool k = cn >= quorum && !isnan(L.acc[d].x);  // cnt >= 1: mean NaN iff sum NaN
          keep_bits |= (uint32_t)k << r;
          kept += k;
        }
      }
      int K;
      int o = block_exclusive_scan_lds<BM_BLOCK>(kept, L.tmp, K);
      if (!(P.ablate & 32)) {
#pragma unroll 1  // one slot at a time: the f64 divides stay out of the ring's registers
        for (int r = 0; r < SPT2; ++r) {
          if ((keep_bits >> r) & 1u) {
            const int d = SPT2 * tid + r;
            const double cnd = (double)reinterpret_cast<const uint16_t*>(L.cnt2)[d];
            const float2 a = L.acc[d];
            out.inten[cp0 + o] = (double)a.x / cnd;
            out.mz[cp0 + o] = a.y == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)a.y / cnd;
            ++o;
          }
        }
      }
      if (wid == 0) {
        const double psum = pw_sum_wave(L.prec, n);  // np.mean (binning.py:224)
        if (tid == 0) {
          out.count[c] = K;
          charge_out[c] = z0;
          prec_out[c] = psum / (double)n;
          status[c] = kOk;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < WPT; ++r) L.bitmap[WPT * tid + r] = 0ull;
    lds_barrier();  // bitmap clear, drain reads done
  };

  const int t0 = (kWave - 1) * wid + lane;
  // a virtual, finished B-turn of the cluster before cb0: next_turn opens the first non-empty one
  Turn cur{-1, 1, (int32_t)cb0 - 1, 0, 0, 1};
  cur = next_turn(cur);
  for (int64_t cl = cb0; cl < cur.c; ++cl) emit_empty(cl);
  if (cur.tl > 0) {
    Turn nx = next_turn(cur), nn = next_turn(nx);
    const uint32_t pb_lo = (uint32_t)PB;
    uint32_t A0 = stream_ahead(v, S0, S1, cur.ts), A1 = stream_ahead(v, S0, S1, nx.ts);
    double Rm[BS_PF], Ri[BS_PF];
    int Rl[BS_PF], Rl2[BS_PF];
    // slot q of turn t: A -> Rm = m/z of spectrum q, Ri = m/z of spectrum q + BS_PF;
    //                   B -> Rm = m/z, Ri = intensity of spectrum q
    auto refill = [&](int q, const Turn& t, uint32_t A) __attribute__((always_inline)) {
      const int a = ahead_off(A, q, pb_lo);
      const int len = q < t.tl ? ahead_off(A, q + 1, pb_lo) - a : 0;
      const uint32_t k = len > 0 ? (uint32_t)(a + (t0 < len ? t0 : 0)) : 0u;
      const int q2 = t.ph == 0 ? q + BS_PF : q;
      const int a2 = ahead_off(A, q2, pb_lo);
      const int len2 = q2 < t.tl ? ahead_off(A, q2 + 1, pb_lo) - a2 : 0;
      const uint32_t k2 = len2 > 0 ? (uint32_t)(a2 + (t0 < len2 ? t0 : 0)) : 0u;
      Rm[q] = ld64(mzb, k);
      Ri[q] = ld64(t.ph == 0 ? mzb : itb, k2);
      Rl[q] = len;
      Rl2[q] = len2;
    };
    auto mark = [&](double m, int len) __attribute__((always_inline)) {
      if (t0 < len && lane < kWave - 1 && in_range(m, P)) {
        const int32_t b = bin_small(m, P);
        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
      }
    };
#pragma unroll
    for (int q = 0; q < BS_PF; ++q) refill(q, cur, A0);
    lds_barrier();  // zeroed bitmap visible
    while (cur.tl > 0) {  // uniform
      const uint32_t A2 = stream_ahead(v, S0, S1, nn.ts);
      const bool isA = cur.ph == 0;  // uniform
      if (!isA && cur.ts == cur.cs) {  // first B-turn of a cluster
        z0 = ahead_z(A0, 0);
        cp0 = PB + ahead_off(A0, 0, pb_lo);
        mixed = 0;
      }
      const bool upd_ok = D <= BM_DCAP;  // uniform
      // one unrolled body for both passes, so each ring register has ONE definition
#pragma unroll
      for (int q = 0; q < BS_PF; ++q) {
        const bool live = q < cur.tl;  // uniform
        if (isA) {
          if (live) {
            if (Rl[q] > BH_CHUNK) badm |= 1ull;
            mark(Rm[q], Rl[q]);
          }
          if (q + BS_PF < cur.tl) {
            if (Rl2[q] > BH_CHUNK) badm |= 1ull;
            mark(Ri[q], Rl2[q]);
          }
        } else if (live) {
          mixed |= ahead_z(A0, q) != z0;
          const int jc = cur.ts - cur.cs + q;
          if (tid == 0 && jc < BM_NMAX) L.prec[jc] = ahead_prec(A0, q);
          const double m = Rm[q], it = Ri[q];
          const int len = Rl[q];
          const int32_t b = bin_small(m, P);
          const int32_t key = !(m >= P.minimum) ? -1 : (m < P.maximum ? b : 0x7fffffff);
          const int32_t kn = wave_next(key, 0x7fffffff);
          const bool active = (t0 < len) & (lane < kWave - 1), has_next = t0 + 1 < len;
          badm |= __ballot(active & has_next & (key > kn));
          const bool part = active & !(has_next & (kn == key)) & ((uint32_t)key < 0x7fffffffu) & upd_ok &
                            !(P.ablate & 16);
          if (part) {
            int slot = bitmap_rank(L.bitmap, L.pre, (int64_t)key);
            slot = slot < BM_DCAP ? slot : BM_DCAP - 1;  // only a deferred cluster's absent bin gets here
            const float2 acc = L.acc[slot];
            atomicAdd(&L.cnt2[slot >> 1], 1u << (16 * (slot & 1)));
            L.acc[slot] = make_float2((float)((double)acc.x + it), (float)((double)acc.y + m));
          }
        }
        refill(q, nx, A1);
        if (!isA && live) lds_barrier();
      }
      if (cur.ts + cur.tl == cur.ce) {
        if (isA) {
          slots(cur.ce - cur.cs);
        } else {
          finish(cur.c, cur.ce - cur.cs);
          for (int64_t cl = cur.c + 1; cl < nx.c; ++cl) emit_empty(cl);
        }
      }
      cur = nx;
      nx = nn;
      nn = next_turn(nn);
      A0 = A1;
      A1 = A2;
    }
  }
}

}  // namespace spx
