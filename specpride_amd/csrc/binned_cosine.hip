// Binned-cosine evaluation of a representative against its cluster members
// (reference: src/benchmark.py:10-38, bin_proc / cos_dist / average_cos_dist;
// restated in oracle/np_oracle.py and pinned by tests/golden/binned_cosine.npz).
//
// The reference densifies both spectra on the edges
//   np.arange(-s/2, max_mz, s), s = 1.000508 * 0.005, max_mz = max(last m/z of the pair)
// (~400k bins), sums intensities per bin (scipy binned_statistic: np.digitize,
// a value "on" the rightmost edge -- x >= e_last and np.around(x, 8) ==
// np.around(e_last, 8) -- shifted into the last bin, outliers dropped), and
// takes cos = A.B / sqrt(A.A * B.B) (0 if either is all zero).  Only bins a
// spectrum occupies contribute, so everything here is sparse:
//   * edges exactly as numpy's DOUBLE_fill writes them: e0 = start,
//     e1 = start + s, e_i = start + i * (e1 - e0); a peak's bin k is the exact
//     #edges <= x minus 1 (a divide for the estimate, then edge compares)
//   * the representative (<= CS_RCAP peaks) is stable-rank-sorted by bin in LDS,
//     its runs summed in input order (np.bincount's order), and the prefix of
//     A_b^2 over runs kept, so each pair's cut (bins <= L-2, L = len(edges))
//     gives A.A with one binary search
//   * one wave per member: each peak's bin (cut and on-edge rule of this pair),
//     A.B = sum_q I_q * A'_{bin(q)} by binary search over the runs, B.B from the
//     member's own runs of equal bins (sums in input order; an unsorted member
//     takes an O(m^2) pass instead)
//   * average_cos_dist = the sequential mean over the members in order.
// Dot products are summed in a different order than BLAS's ddot: values agree
// with the reference to ~1e-15 relative (the north star asks 1e-5).
#include "spx_device.hpp"

namespace spx {

struct CosParams {
  double s, start, e1, d;  // np.arange(start, stop, s) = start, e1, start + i * d
  double p10;              // 10**decimals of scipy's on-edge rounding
  double inv_d;            // 1 / d: the bin estimate (edge compares make it exact)
};

constexpr int CS_BLOCK = 256;
// 512 representative peaks in LDS and 1,024-bin run buckets: 25.9 KB, 6 workgroups
// per CU.  The kernel is latency-bound (a wave walks its members chunk by chunk), so
// occupancy is what pays: 1,024 peaks / 256-bin buckets (55 KB, 2 per CU) measured
// 14.6 ms per 100k clusters, 640 peaks (4 per CU) 8.0 ms, this 6.15 ms.  Longer
// representatives take the global-scratch kernel.
#ifndef SPX_CS_RCAP
#define SPX_CS_RCAP 512
#endif
constexpr int CS_RCAP = SPX_CS_RCAP;  // representative peaks held in LDS
constexpr int CS_NW = CS_BLOCK / kWave;
#ifndef SPX_CS_BSH
#define SPX_CS_BSH 10
#endif
constexpr int CS_BSH = SPX_CS_BSH;                 // run-index buckets of 2^CS_BSH bins (1,024: ~5.1 Da)
constexpr int CS_BMAX = (1 << 19) >> CS_BSH;       // buckets held in LDS: bins < 524,288 (m/z < ~2,620)
static_assert(CS_BMAX % CS_BLOCK == 0, "whole buckets per thread");

// Representative state: LDS arrays (cap = CS_RCAP) in the main kernel, a
// per-workgroup global scratch slice (cap = the largest deferred
// representative) in binned_cosine_global_kernel.
struct CosState {
  int32_t* sk;    // representative peak bins, input order (rank sort input)
  int32_t* pk;    // ... sorted by (bin, index)
  double* pI;     //     their intensities
  int32_t* pidx;  //     their input index
  int32_t* rb;    // runs of equal bins: bin,
  int32_t* rs;    //   first sorted position [cap + 1],
  double* rA;     //   A_b (summed in input order),
  double* rA2;    //   exclusive prefix of A_b^2 [cap + 1]
  int cap;
};

struct CosShared {               // LDS of both kernels
  int32_t bst[CS_BMAX];          // first run with a bin >= t << CS_BSH, per bucket t
  int32_t wk[CS_NW][kWave];      // per-wave member scratch: bins,
  double wI[CS_NW][kWave];       //   intensities
  double tmpd[CS_NW + 1];
  int tmp[CS_NW + 1];
  int nruns;
};

struct CosSmem {
  union {  // the rank sort's input is dead once the runs are written
    int32_t sk[CS_RCAP];
    int32_t rb[CS_RCAP];
  };
  int32_t pk[CS_RCAP], pidx[CS_RCAP], rs[CS_RCAP + 1];
  double pI[CS_RCAP], rA[CS_RCAP], rA2[CS_RCAP + 1];
  CosShared sh;
};

__device__ __forceinline__ double cs_edge(const CosParams& P, int64_t i) {
  return i == 0 ? P.start : (i == 1 ? P.e1 : P.start + (double)i * P.d);
}

// k with e_k <= x < e_{k+1} over the unbounded edge sequence; -1 below e_0 or NaN.
// The reciprocal product is only an estimate; the exact edge compares settle it.
__device__ __forceinline__ int64_t cs_bin(const CosParams& P, double x) {
  if (!(x >= P.start)) return -1;
  int64_t k = (int64_t)((x - P.start) * P.inv_d);
  if (k > 0 && cs_edge(P, k) > x) --k;
  if (k > 0 && cs_edge(P, k) > x) --k;
  while (cs_edge(P, k + 1) <= x) ++k;
  return k;
}

// np.around(x, decimals) for decimals > 0: rint(x * 10**d) / 10**d
__device__ __forceinline__ double np_around(double x, double p10) { return rint(x * p10) / p10; }

// first run index with a bin > b (runs sorted by bin), over [0, nr)
__device__ __forceinline__ int runs_upper(const int32_t* rb, int nr, int64_t b) {
  int lo = 0, hi = nr;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)rb[mid] <= b) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// One cluster: the representative's runs, then one wave per member.  Returns
// false (nothing written) if the representative exceeds S.cap.
__device__ bool cos_body(const CsrView& v, const CosParams& P, const CosState& S, CosShared& L, int64_t c,
                         const int64_t* rep_off, const double* rep_mz, const double* rep_int, double* cos_out,
                         double* avg_out, int32_t* status) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  const int64_t r0 = rep_off[c];
  const int R = (int)(rep_off[c + 1] - r0);
  const double nan = __longlong_as_double(0x7ff8000000000000ll);
  if (n == 0) {  // average_cos_dist of no members (benchmark.py:36-38)
    if (tid == 0) { avg_out[c] = 0.0; status[c] = kOk; }
    return true;
  }
  // an empty spectrum: the reference's mz[-1] raises IndexError (benchmark.py:20)
  int empty = R == 0;
  for (int j = tid; j < n; j += CS_BLOCK) empty |= v.spec_off[s0 + j + 1] == v.spec_off[s0 + j];
  const bool any_empty = __syncthreads_or(empty);
  if (any_empty) {
    for (int j = tid; j < n; j += CS_BLOCK) cos_out[s0 + j] = nan;
    if (tid == 0) { avg_out[c] = nan; status[c] = kEmpty; }
    return true;
  }
  if (R > S.cap) return false;

  // representative: bins, stable rank sort by (bin, index), runs, prefix of A^2
  for (int i = tid; i < R; i += CS_BLOCK) {
    const int64_t k = cs_bin(P, rep_mz[r0 + i]);
    S.sk[i] = k > 0x7ffffffe ? 0x7ffffffe : (int32_t)k;
  }
  __syncthreads();
  // an m/z-sorted representative (the consensus outputs are) is already in
  // (bin, index) order: the stable rank sort is the identity
  int inv = 0;
  for (int i = tid + 1; i < R; i += CS_BLOCK) inv |= S.sk[i] < S.sk[i - 1];
  const bool sorted = !__syncthreads_or(inv);
  for (int i = tid; i < R; i += CS_BLOCK) {
    const int32_t k = S.sk[i];
    int rank = i;
    if (!sorted) {
      rank = 0;
      for (int j = 0; j < R; ++j) {
        const int32_t kj = S.sk[j];
        rank += kj < k || (kj == k && j < i);
      }
    }
    S.pk[rank] = k;
    S.pI[rank] = rep_int[r0 + i];
    S.pidx[rank] = i;
  }
  __syncthreads();
  {
    const int PER = (R + CS_BLOCK - 1) / CS_BLOCK;  // contiguous chunk per thread: runs in order
    int heads = 0;
    for (int u = 0; u < PER; ++u) {
      const int r = PER * tid + u;
      heads += r < R && (r == 0 || S.pk[r] != S.pk[r - 1]);
    }
    int nr;
    int id = block_exclusive_scan<CS_BLOCK>(heads, L.tmp, nr);
    for (int u = 0; u < PER; ++u) {
      const int r = PER * tid + u;
      if (r < R && (r == 0 || S.pk[r] != S.pk[r - 1])) {
        double A = 0.0;  // np.bincount: out[bin] = 0.0, then += w in input order
        for (int q = r; q < R && S.pk[q] == S.pk[r]; ++q) A += S.pI[q];
        S.rb[id] = S.pk[r];
        S.rs[id] = r;
        S.rA[id] = A;
        ++id;
      }
    }
    if (tid == 0) { L.nruns = nr; S.rs[nr] = R; }
    __syncthreads();
    const int PR = (nr + CS_BLOCK - 1) / CS_BLOCK;
    double sq = 0.0;
    for (int u = 0; u < PR; ++u) {
      const int r = PR * tid + u;
      if (r < nr && S.rb[r] >= 0) sq += S.rA[r] * S.rA[r];
    }
    double tot;
    double pre = block_exclusive_scan<CS_BLOCK>(sq, L.tmpd, tot);
    for (int u = 0; u < PR; ++u) {
      const int r = PR * tid + u;
      if (r < nr) {
        S.rA2[r] = pre;
        if (S.rb[r] >= 0) pre += S.rA[r] * S.rA[r];
      }
    }
    if (tid == 0) S.rA2[nr] = tot;
    // bucket t: the first run with a bin >= t << CS_BSH (runs are sorted by bin)
    {
      // CS_BMAX / CS_BLOCK consecutive buckets per thread: one binary search for the
      // first, then a forward walk (runs are sparse: ~0-1 steps per bucket)
      constexpr int TPT = CS_BMAX / CS_BLOCK;
      const int t0 = tid * TPT;
      const int64_t b0 = (int64_t)t0 << CS_BSH;
      int lo = 0, hi = nr;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)S.rb[mid] < b0) lo = mid + 1;
        else hi = mid;
      }
#pragma unroll
      for (int k = 0; k < TPT; ++k) {
        const int64_t bk = (int64_t)(t0 + k) << CS_BSH;
        while (lo < nr && (int64_t)S.rb[lo] < bk) ++lo;
        L.bst[t0 + k] = lo;
      }
    }
    __syncthreads();
  }
  const int NR = L.nruns;
  const double rep_last = rep_mz[r0 + R - 1];  // rep.mz[-1] (benchmark.py:20)

  // members: one wave each
  for (int j = wid; j < n; j += CS_NW) {
    const int64_t a = v.spec_off[s0 + j], e = v.spec_off[s0 + j + 1];
    // the member's first chunk is loaded with its last m/z, before the pair's cut is
    // worked out, and every chunk loads the next one ahead (one HBM latency per member
    // instead of one per chunk)
    double xq, Iq;
    {
      const int64_t k0 = a + lane;
      xq = k0 < e ? v.mz[k0] : 0.0;
      Iq = k0 < e ? v.inten[k0] : 0.0;
    }
    const double mem_last = v.mz[e - 1];
    const double max_mz = mem_last > rep_last ? mem_last : rep_last;  // max(rep.mz[-1], member.mz[-1])
    const int64_t Lc = (int64_t)ceil((max_mz - P.start) / P.s);      // len(np.arange(...))
    const int64_t kc = Lc - 2;                                          // the last bin
    const double e_last = cs_edge(P, Lc - 1), rl = np_around(e_last, P.p10);
    // representative under this pair's cut: A.A and the on-edge extra of bin kc
    const int ic = runs_upper(S.rb, NR, kc);  // runs with a bin <= kc
    double extra = 0.0;
    bool has_extra = false;
    if (ic < NR && (int64_t)S.rb[ic] == kc + 1) {
      for (int q = S.rs[ic]; q < S.rs[ic + 1]; ++q) {
        const double x = rep_mz[r0 + S.pidx[q]];
        if (x >= e_last && np_around(x, P.p10) == rl) {
          extra += S.pI[q];
          has_extra = true;
        }
      }
    }
    const bool kc_run = ic > 0 && (int64_t)S.rb[ic - 1] == kc;
    const double A_kc = (kc_run ? S.rA[ic - 1] : 0.0) + extra;  // A'_{kc}
    double aa = S.rA2[ic];
    if (has_extra) aa = S.rA2[kc_run ? ic - 1 : ic] + A_kc * A_kc;
    auto lookup = [&](int64_t b) -> double {
      if (b == kc) return A_kc;
      if ((b >> CS_BSH) < CS_BMAX) {  // bucket start, then a short forward walk
        int u = L.bst[b >> CS_BSH];
        while (u < NR && (int64_t)S.rb[u] < b) ++u;
        return (u < NR && (int64_t)S.rb[u] == b) ? S.rA[u] : 0.0;
      }
      const int u = runs_upper(S.rb, NR, b);
      return (u > 0 && (int64_t)S.rb[u - 1] == b) ? S.rA[u - 1] : 0.0;
    };
    auto mem_bin = [&](double x) -> int64_t {
      const int64_t k = cs_bin(P, x);
      if (k >= 0 && k <= kc) return k;
      if (k > kc && x >= e_last && np_around(x, P.p10) == rl) return kc;  // on the rightmost edge
      return -1;
    };
    const int m = (int)(e - a);
    double ab = 0.0, bb = 0.0;
    int64_t carry_b = -1, lastb = -1, last_raw = -1;
    double carry_s = 0.0;
    bool unsorted = false;
    for (int ch = 0; ch < m; ch += kWave) {
      const int q = ch + lane;
      const bool in = q < m;
      const double x = in ? xq : 0.0, I = in ? Iq : 0.0;
      {
        const int qn = q + kWave;
        xq = qn < m ? v.mz[a + qn] : 0.0;
        Iq = qn < m ? v.inten[a + qn] : 0.0;
      }
      const int64_t bm = in ? mem_bin(x) : -1;
      if (bm >= 0) ab += I * lookup(bm);
      // runs need every valid bin >= the previous valid one, and a repeated bin
      // right after its predecessor (an invalid peak between two equal bins
      // would split np.bincount's single sum)
      int64_t prev, raw_before, cmax, lraw;
      if (kc < 0x7ffffff0) {  // uniform: every bin fits 32 bits -- DPP, no LDS round trips
        const int32_t b32 = (int32_t)bm;
        const int32_t p32 = wave_scan_dpp(b32, (int32_t)0x80000000, [](int32_t x, int32_t y) { return x > y ? x : y; });
        prev = (int32_t)__builtin_amdgcn_update_dpp(-1, p32, 0x138, 0xF, 0xF, false);  // wave_shr:1
        raw_before = (int32_t)__builtin_amdgcn_update_dpp(-1, b32, 0x138, 0xF, 0xF, false);
        cmax = __builtin_amdgcn_readlane(p32, kWave - 1);
        lraw = __builtin_amdgcn_readlane(b32, kWave - 1);
      } else {
        int64_t pm = bm;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
          const int64_t t = __shfl_up(pm, o, kWave);
          if (lane >= o) pm = pm > t ? pm : t;
        }
        prev = __shfl_up(pm, 1, kWave);
        raw_before = __shfl_up(bm, 1, kWave);
        cmax = __shfl(pm, kWave - 1, kWave);
        lraw = __shfl(bm, kWave - 1, kWave);
      }
      if (lane == 0) { prev = -1; raw_before = last_raw; }
      prev = prev > lastb ? prev : lastb;
      unsorted |= __ballot(bm >= 0 && (bm < prev || (bm == prev && raw_before != bm))) != 0ull;
      lastb = cmax > lastb ? cmax : lastb;
      last_raw = lraw;
      if (unsorted) continue;  // (uniform) B.B by the O(m^2) pass below
      // runs of equal bins, summed in input order; the last one may continue
      L.wk[wid][lane] = (int32_t)bm;
      L.wI[wid][lane] = I;
      wave_lds_sync();
      const int64_t before = lane == 0 ? carry_b : (int64_t)L.wk[wid][lane - 1];
      const bool head = bm >= 0 && bm != before;
      const bool cont = lane == 0 && bm >= 0 && bm == carry_b;  // continues the open run
      int64_t new_carry_b = -1;
      double new_carry_s = 0.0;
      if (carry_b >= 0 && !(__ballot(cont) & 1ull) && lane == 0) bb += carry_s * carry_s;  // open run closed
      if (head || cont) {
        double s = cont ? carry_s : 0.0;
        int qq = lane;
        while (qq < kWave && L.wk[wid][qq] == (int32_t)bm) s += L.wI[wid][qq++];
        if (qq == kWave && ch + kWave < m) {
          new_carry_b = bm;
          new_carry_s = s;
        } else {
          bb += s * s;
        }
      }
      const unsigned long long cm = __ballot(new_carry_b >= 0);
      if (cm) {
        const int cl = __ffsll((long long)cm) - 1;
        carry_b = readlane64(new_carry_b, cl);
        carry_s = readlane_f64(new_carry_s, cl);
      } else {
        carry_b = -1;
        carry_s = 0.0;
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (unsorted) {  // B.B = sum_q I_q * (sum of I over the member's peaks in q's bin)
      bb = 0.0;
      for (int ch = 0; ch < m; ch += kWave) {
        const int q = ch + lane;
        const double I = q < m ? v.inten[a + q] : 0.0;
        const int64_t bm = q < m ? mem_bin(v.mz[a + q]) : -1;
        double sb = 0.0;
        for (int ch2 = 0; ch2 < m; ch2 += kWave) {
          const int q2 = ch2 + lane;
          L.wk[wid][lane] = q2 < m ? (int32_t)mem_bin(v.mz[a + q2]) : -1;
          L.wI[wid][lane] = q2 < m ? v.inten[a + q2] : 0.0;
          wave_lds_sync();
          for (int t = 0; t < kWave; ++t)
            if (bm >= 0 && L.wk[wid][t] == (int32_t)bm) sb += L.wI[wid][t];
          __builtin_amdgcn_wave_barrier();
        }
        if (bm >= 0) bb += I * sb;
      }
    } else if (carry_b >= 0 && lane == 0) {
      bb += carry_s * carry_s;
    }
    ab = wave_sum_f64(ab);
    bb = wave_sum_f64(bb);
    if (lane == 0) cos_out[s0 + j] = (aa == 0.0 || bb == 0.0) ? 0.0 : ab / sqrt(aa * bb);
  }
  __syncthreads();
  if (tid == 0) {  // average_cos_dist: sequential sum in member order (benchmark.py:33-36)
    double sum = 0.0;
    for (int j = 0; j < n; ++j) sum += cos_out[s0 + j];
    avg_out[c] = sum / (double)n;
    status[c] = kOk;
  }
  return true;
}

// Clusters whose representative fits LDS; larger ones go to `deferred`.
__global__ __launch_bounds__(CS_BLOCK) void binned_cosine_kernel(CsrView v, CosParams P, const int64_t* rep_off,
                                                                 const double* rep_mz, const double* rep_int,
                                                                 double* cos_out, double* avg_out, int32_t* status,
                                                                 int32_t* deferred, int32_t* n_deferred) {
  __shared__ CosSmem L;
  CosState S;
  S.sk = L.sk; S.pk = L.pk; S.pI = L.pI; S.pidx = L.pidx; S.rb = L.rb; S.rs = L.rs; S.rA = L.rA; S.rA2 = L.rA2;
  S.cap = CS_RCAP;
  const int64_t c = blockIdx.x;
  if (!cos_body(v, P, S, L.sh, c, rep_off, rep_mz, rep_int, cos_out, avg_out, status) && threadIdx.x == 0) {
    status[c] = kDeferred;
    deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
  }
}

// Bytes of one scratch slice for representatives of up to `cap` peaks.
__host__ __device__ inline int64_t cos_slice_bytes(int64_t cap) {
  return 5 * ((4 * (cap + 1) + 255) & ~int64_t(255)) + 3 * ((8 * (cap + 1) + 255) & ~int64_t(255));
}

// The deferred clusters (representative > CS_RCAP peaks): the same body with the
// representative's arrays in a per-workgroup global scratch slice.
__global__ __launch_bounds__(CS_BLOCK) void binned_cosine_global_kernel(
    CsrView v, CosParams P, const int64_t* rep_off, const double* rep_mz, const double* rep_int, double* cos_out,
    double* avg_out, int32_t* status, const int32_t* deferred, const int32_t* n_deferred, char* scratch, int cap) {
  __shared__ CosShared L;
  char* base = scratch + (int64_t)blockIdx.x * cos_slice_bytes(cap);
  const int64_t s4 = (4 * ((int64_t)cap + 1) + 255) & ~int64_t(255), s8 = (8 * ((int64_t)cap + 1) + 255) & ~int64_t(255);
  CosState S;
  S.sk = reinterpret_cast<int32_t*>(base);
  S.pk = reinterpret_cast<int32_t*>(base + s4);
  S.pidx = reinterpret_cast<int32_t*>(base + 2 * s4);
  S.rb = reinterpret_cast<int32_t*>(base + 3 * s4);
  S.rs = reinterpret_cast<int32_t*>(base + 4 * s4);
  S.pI = reinterpret_cast<double*>(base + 5 * s4);
  S.rA = reinterpret_cast<double*>(base + 5 * s4 + s8);
  S.rA2 = reinterpret_cast<double*>(base + 5 * s4 + 2 * s8);
  S.cap = cap;
  const int32_t nd = *n_deferred;
  for (int32_t i = blockIdx.x; i < nd; i += gridDim.x) {
    const int64_t c = deferred[i];
    if (!cos_body(v, P, S, L, c, rep_off, rep_mz, rep_int, cos_out, avg_out, status) && threadIdx.x == 0)
      status[c] = kDeferred;  // longer than the workspace was sized for
    __syncthreads();
  }
}

}  // namespace spx
