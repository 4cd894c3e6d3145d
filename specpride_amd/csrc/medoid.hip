// Most-similar (medoid) representative (reference: src/most_similar_representative.py:13-19
// distance(), :60-111 the per-cluster loop; OpenMS XQuestScores::xCorrelationPrescore
// restated in SURVEY.md Appendix A.3 / oracle/np_oracle.py).
//
// xcorr(a, b) = |B_a ∩ B_b| / min(#peaks a, #peaks b), B = {ceil(mz / tol)} (0 if
// either spectrum is empty); d = 1 - xcorr; D = upper triangle of d INCLUDING
// the diagonal (lower triangle 0); total_i = (pairwise_sum(row i) +
// pairwise_sum(col i)) / n with numpy's pairwise-summation tree; representative
// = lowest index among the minima.  Every integer (bins, |B_a ∩ B_b|, peak counts)
// is exact and the f64 epilogue follows the reference's operation order, so the
// chosen index is bit-exact.
//
// Small clusters (n <= 64): medoid_reg_kernel, one 256-thread workgroup per
// cluster, all state in LDS (bit-packed rows over the compact bin columns, the
// bit-packed Gram by AND + popcount).  Large clusters (n > 64, or an LDS
// overflow) go to a deferred list and through the grid-parallel passes and the
// MFMA Gram kernel below, with state in a bump-allocated global arena.
#pragma once
#include <type_traits>

#include "spx_device.hpp"

namespace spx {

struct MedoidParams {
  double tol, inv_tol;
};

constexpr int MD_BLOCK = 256;
constexpr int MD_NMAX = 64;
// 27 row words (<= 1,728 occupied bins) and 72 VGPRs: 22.6 KB of LDS, 7 workgroups
// per CU (31 words / 6 per CU: 1.55 -> 1.48 ms at 100k clusters); a cluster with
// more distinct bins takes the large path
#ifndef SPX_MD_KWMAX
#define SPX_MD_KWMAX 27
#endif
#ifndef SPX_MD_MINW
#define SPX_MD_MINW 7
#endif
#ifndef SPX_MD_MFMA_NMIN
#define SPX_MD_MFMA_NMIN 32  // ... for clusters of more spectra than this
#endif
constexpr int MD_KWMAX = SPX_MD_KWMAX;  // row words (odd stride): <= 64 * MD_KWMAX occupied bins per small cluster


__device__ __forceinline__ int64_t md_bin(double m, const MedoidParams& P) {
  return ceil_div_exact(m, P.tol, P.inv_tol);
}

// d(i,j) exactly as 1.0 - XQuestScores::xCorrelationPrescore(...)
__device__ __forceinline__ double md_dist(uint32_t c, int64_t pi, int64_t pj) {
  const double x = (pi == 0 || pj == 0) ? 0.0 : (double)c / (double)(pi < pj ? pi : pj);
  return 1.0 - x;
}

// d(i,j) = 1 - c/q, q = min(p_i, p_j), with the quotient from q's reciprocal r = fl(1/q)
// and one exact fma remainder step: equal to the IEEE quotient fl(c/q) for every
// 0 <= c <= q <= 65,536 (all 2.1e9 pairs checked on the host), so the distances --
// and with them the totals and representatives -- are md_dist's bit for bit.
__device__ __forceinline__ double md_dist_r(uint32_t c, int pi, double ri, int pj, double rj) {
  const int q = pi < pj ? pi : pj;
  const double cd = (double)c, qd = (double)q;
  const double r = pi < pj ? ri : rj;
  const double y = cd * r;
  const double x = __builtin_fma(__builtin_fma(-y, qd, cd), r, y);
  return (pi == 0 || pj == 0) ? 1.0 : 1.0 - x;
}
// Both pairwise sums of thread i (row i: j >= i; column i: j <= i) in one pass
// over j, for n <= 128 (numpy's leaf regime).  f(j) returns d(i, j) = d(j, i).
template <class F>
__device__ __forceinline__ void dual_pw_leaf(const F& f, int n, int i, double& row, double& col) {
  if (n < 8) {
    double r = 0.0, cc = 0.0;
    for (int j = 0; j < n; ++j) {
      const double d = f(j);
      r += j >= i ? d : 0.0;
      cc += j <= i ? d : 0.0;
    }
    row = 0.0 + r;
    col = 0.0 + cc;
    return;
  }
  double r[8], cc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double d = f(k);
    r[k] = k >= i ? d : 0.0;
    cc[k] = k <= i ? d : 0.0;
  }
  int j = 8;
  const int lim = n - (n % 8);
  for (; j < lim; j += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double d = f(j + k);
      r[k] += (j + k) >= i ? d : 0.0;
      cc[k] += (j + k) <= i ? d : 0.0;
    }
  }
  double rs = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  double cs = ((cc[0] + cc[1]) + (cc[2] + cc[3])) + ((cc[4] + cc[5]) + (cc[6] + cc[7]));
  for (; j < n; ++j) {
    const double d = f(j);
    rs += j >= i ? d : 0.0;
    cs += j <= i ? d : 0.0;
  }
  row = 0.0 + rs;
  col = 0.0 + cs;
}

// spectrum (local index) holding cluster-relative peak k, from LDS offsets
__device__ __forceinline__ int spectrum_of(const int32_t* soff, int n, int32_t k) {
  int lo = 0, hi = n;  // soff[lo] <= k < soff[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (soff[mid] <= k) lo = mid; else hi = mid;
  }
  return lo;
}

typedef int md_i32x8 __attribute__((ext_vector_type(8)));
typedef float md_f32x16 __attribute__((ext_vector_type(16)));

// One 32-bin half of a 64-bin row word as an FP4 e2m1 MFMA operand (1.0 = nibble
// 0b0010): lane half fh takes bins 32fh..32fh+31, dword g nibble p = bin 32fh + g + 4p
// (the same k order for A and B, so the dot products are the bit-AND popcounts).
__device__ __forceinline__ md_i32x8 md_frag4(uint64_t w, int fh) {
  const uint32_t c = (uint32_t)(w >> (32 * fh));
  md_i32x8 f;
  f[0] = (int)((c << 1) & 0x22222222u);
  f[1] = (int)(c & 0x22222222u);
  f[2] = (int)((c >> 1) & 0x22222222u);
  f[3] = (int)((c >> 2) & 0x22222222u);
  f[4] = f[5] = f[6] = f[7] = 0;
  return f;
}

// --------------------------------------------------------- small clusters
// Per deferred cluster state of the large path (zero-initialised at deferral).
struct MedoidMeta {
  unsigned long long lo_key, hi_key;  // bin range, order-preserving keys (atomicMax; 0 = none)
  int64_t c, s0, blo;
  int64_t p0, np;  // the cluster's peaks (medoid_units_kernel)
  int64_t l1_off, l2_off, rows_off, rowsT_off, cmat_off, leaf_off, lsum_off, tot_off;  // arena byte offsets
  int32_t n, nw1, B1, KW, L, tiles, units, ok;
};

// Appends cluster c to the deferred list; rep[c] = -4 until the large path
// (if the call runs it) writes the result.
__device__ __forceinline__ void md_defer(int64_t c, int64_t s0, int n, int32_t* deferred, int32_t* n_deferred,
                                         MedoidMeta* meta, int64_t* rep) {
  rep[c] = -4;
  const int32_t slot = atomicAdd(n_deferred, 1);
  deferred[slot] = (int32_t)c;
  MedoidMeta M = {};
  M.c = c;
  M.s0 = s0;
  M.n = n;
  meta[slot] = M;
}

// ---------------------------------------------------------- small clusters
// medoid_reg_kernel: every m/z read from HBM exactly ONCE (8 B per peak, the algorithmic minimum) and the
// per-peak LDS traffic cut to four operations:
//   P1  flat coalesced pass over the cluster's peaks (peak r = u*256 + tid,
//       8 loads in flight per thread): absolute bin ceil(mz/tol) < 32,768, kept
//       in registers as packed u16 (<= MR_UMAX per thread), union bitmap in LDS
//       (32-bit LDS atomics).  Branch-free per batch of 8: the
//       reciprocal product's ceil where certain and in range, one "bad" mask
//       settled by md_bin's exact divide once per batch.  The xcorr is a set
//       intersection: no range pass, and unsorted spectra need no special path.
//   P2  popcount prefix -> K compact columns (a u16 prefix per
//       32-bit occupancy word)
//   P3  bit-packed rows from the register bins: column = rank (a u16 prefix and
//       one bfe + popcount), spectrum = the slice's spectrum-end word and its
//       prefix handed out by readlane, counted by two v_mbcnt; rows
//       set by 32-bit LDS atomics into words swizzled per bit position
//       (a spectrum's neighbouring columns -- consecutive lanes --
//       no longer serialise on one word)
//   P4  pair counts: past 32 spectra on the matrix cores (FP4 0/1 Gram tiles, one
//       per wave), else one thread per pair i <= j by AND + popcount;
//       then d_ij = 1 - c_ij/min(p_i, p_j) (exact reciprocal form, md_dist_r) into
//       the reference's n x n matrix (upper triangle incl. the diagonal, zeros
//       below: most_similar_representative.py:91-93), aliasing the dead bitmap and rows
//   P5  totals with numpy's pairwise tree (:98-100): one lane per spectrum, wave 0
//       the rows, wave 1 the columns (8 strided accumulators combined
//       ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), sequential tail), total = (row + col)/n
//   P6  lowest index of the minimum (:103-110), wave 0 straight from P5's registers
// Deferred (to the wide kernel, then the large path): n > 64, > MR_UMAX*256 peaks, a bin outside
// [0, 65,536), > 64 * MD_KWMAX distinct bins.
constexpr int MR_UMAX = 48;                  // peaks per thread (12,288 per cluster)
constexpr int MR_PMAX = MR_UMAX * MD_BLOCK;
constexpr int MR_WMAX = 512;                 // union-bitmap words: bins < 32,768 (m/z < 3,276.8 at 0.1)
constexpr int MR_TRI = MD_NMAX * (MD_NMAX + 1) / 2;  // packed upper triangle of the distance matrix

// The wide variant (medoid_wide_kernel): what the register kernel defers for its
// peak or bin caps alone (n <= 64 still) -- 512 threads, 64 peaks per thread
// (32,768 per cluster), 95 row words (<= 6,080 occupied bins): 59 KB of LDS, two
// workgroups per CU.  600-peak spectra reach it from n ~ 20 on.
constexpr int MW_BLOCK = 512;
constexpr int MW_UMAX = 64;
constexpr int MW_PMAX = MW_UMAX * MW_BLOCK;
constexpr int MW_KWMAX = 95;

template <int BLOCK, int UMAX, int KWMAX>
struct MedoidRegSmem {
  union {
    struct {
      // occupancy words and their exclusive popcount prefixes in two dense arrays:
      // word w's 32-bit halves sit on banks 2w, 2w+1 and its prefix on bank w, so
      // the ORs and rank reads spread over every bank (a 16-B {word, prefix}
      // record put them on 16 of 32 and 8 of 32 banks)
      unsigned long long bits[MR_WMAX];
      uint32_t pre[MR_WMAX];
      unsigned long long rows[MD_NMAX * KWMAX];
      unsigned long long sbits[UMAX * BLOCK / 64];  // bit r: peak r starts spectrum >= 1 (ends a spectrum)
      uint8_t spre[UMAX * BLOCK / 64];              // spectra started (ended) before word w
    } a;                                         // P0..P4a
    double d[MR_TRI];                            // P4b..P5: d(i, j), j >= i, row-major packed
    struct {
      double d[MR_TRI];
      double col[MD_NMAX];                       // P5: column sums, past d
    } t;
  } u;
  int32_t soff[MD_NMAX + 1];
  double totals[MD_NMAX];
  int tmp[BLOCK / kWave + 1];
  long long red[4];
  int votes[2 * (BLOCK / kWave)];
};

// P4..P6 of a small cluster whose bit rows (n rows of KW words, swizzled as P3
// sets them) are in L.u.a.rows and whose spectrum offsets are in L.soff: the pair
// counts, the reference's distance matrix, the pairwise-tree totals and the
// lowest-index argmin.  Shared by medoid_small_body and the fused pass's
// medoid_from_codes (fused.hip), so both give the same bits.
template <int BLOCK, int UMAX, int KWMAX>
__device__ __forceinline__ void medoid_tail(MedoidRegSmem<BLOCK, UMAX, KWMAX>& L, int n, int KW, int64_t s0,
                                            int64_t c, int64_t* rep, double* totals_out) {
  constexpr int PMAX = UMAX * BLOCK;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  // each spectrum's exact reciprocal for P4's quotients (totals is free until P5;
  // spectra here hold at most PMAX <= 65,536 peaks, md_dist_r's checked range)
  static_assert(PMAX <= 65536, "md_dist_r's exact range");
  if (tid < n) {
    const int p = L.soff[tid + 1] - L.soff[tid];
    L.totals[tid] = p > 0 ? 1.0 / (double)p : 0.0;
  }
  __syncthreads();
  SPX_STAMP2(4, -1);

  auto row_start = [&](int i) { return i * n - (i * (i - 1)) / 2; };
  // the matrix cores for the register kernel's P4; the wide kernel (up to 95 row words,
  // 128 VGPRs) keeps the AND + popcount pairs: there the sequential MFMA chain measured
  // slower (600-peak spectra, medoid_shapes: 1.12 -> 1.37 ms)
  // and only for clusters of more than SPX_MD_MFMA_NMIN spectra: below, one wave holds
  // the one 32 x 32 tile and its epilogue while the pairs spread over the whole workgroup
  // (stamps, configs[4]: P4 n 41-50 14.4k -> 11.7k cycles, n 11-25 5.7k -> 8.7k)
  bool mfma_p4 = false;
  if constexpr (BLOCK == MD_BLOCK) mfma_p4 = n > SPX_MD_MFMA_NMIN;  // uniform
  if (mfma_p4) {
  // P4 on the matrix cores: c_ij = |B_i ∩ B_j| = the Gram of the 0/1 rows, one
  // 32 x 32 tile per wave -- (0,0) for n <= 32; (0,0), (0,1), (1,1) for n <= 64 --
  // one v_mfma_f32_32x32x64_f8f6f4 per 64-bin row word (FP4 0/1 operands at unit
  // scale: the f32 sums of <= 2^24 ones are the integer counts), then
  // d_ij = 1 - c_ij / min(p_i, p_j) into the packed upper triangle
  {
    const int fr = lane & 31, fh = lane >> 5;
    const int ntile = n > 32 ? 3 : 1;
    const bool work = wid < ntile;  // wave-uniform
    const int ta = wid == 2 ? 1 : 0, tb = wid == 0 ? 0 : 1;
    md_f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
    if (work) {
      const int ra = ta * 32 + fr, rb = tb * 32 + fr;
      const unsigned long long* pa = L.u.a.rows + (ra < n ? ra : 0) * KW;
      const unsigned long long* pb = L.u.a.rows + (rb < n ? rb : 0) * KW;
      const unsigned long long ma = ra < n ? ~0ull : 0ull, mb = rb < n ? ~0ull : 0ull;
      unsigned long long wa = pa[0] & ma, wb = pb[0] & mb;  // one word ahead
      for (int w = 0; w < KW; ++w) {
        const int wn = w + 1 < KW ? w + 1 : w;
        const unsigned long long na = pa[wn] & ma, nb = pb[wn] & mb;
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(md_frag4(wa, fh), md_frag4(wb, fh), acc, 4, 4, 0, 0,
                                                              0, 0);
        wa = na;
        wb = nb;
      }
    }
    __syncthreads();  // rows dead: the distance matrix takes their place
    if (work) {
      // C/D layout (32x32): col = lane & 31, row = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5)
      const int j = tb * 32 + fr;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = ta * 32 + (q & 3) + 8 * (q >> 2) + 4 * fh;
        if (i <= j && j < n) {
          const uint32_t cnt = (uint32_t)acc[q];
          L.u.d[row_start(i) + j - i] =
              md_dist_r(cnt, L.soff[i + 1] - L.soff[i], L.totals[i], L.soff[j + 1] - L.soff[j], L.totals[j]);
        }
      }
    }
  }
  } else {
    // P4: every pair i <= j of the row-major upper triangle (row i starts at
    // i*n - i*(i-1)/2; recovered by a float sqrt + integer fix-up); counts in
    // registers until the rows are dead
    constexpr int PPT = (MD_NMAX * (MD_NMAX + 1) / 2 + BLOCK - 1) / BLOCK;  // pairs per thread (9)
    const int NP = n * (n + 1) / 2;
    uint32_t pc[PPT];
    int pij[PPT];
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      const int p = tid + q * BLOCK;
      pc[q] = 0u;
      pij[q] = -1;
      if (p < NP) {
        const float b2 = 2.0f * n + 1.0f;
        int i = (int)((b2 - sqrtf(b2 * b2 - 8.0f * (float)p)) * 0.5f);
        i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
        while (i > 0 && row_start(i) > p) --i;
        while (i + 1 < n && row_start(i + 1) <= p) ++i;
        const int j = i + (p - row_start(i));
        uint32_t cnt = 0;
        for (int w = 0; w < KW; ++w) cnt += (uint32_t)__popcll(L.u.a.rows[i * KW + w] & L.u.a.rows[j * KW + w]);
        pc[q] = cnt;
        pij[q] = i << 8 | j;
      }
    }
    __syncthreads();  // rows dead: the distance matrix takes their place
#pragma unroll
    for (int q = 0; q < PPT; ++q) {
      if (pij[q] >= 0) {
        const int i = pij[q] >> 8, j = pij[q] & 0xff;
        L.u.d[row_start(i) + j - i] =
            md_dist_r(pc[q], L.soff[i + 1] - L.soff[i], L.totals[i], L.soff[j + 1] - L.soff[j], L.totals[j]);
      }
    }
  }
  __syncthreads();
  // D(a, b) of the reference's dense matrix: the upper triangle incl. the
  // diagonal, zeros below (most_similar_representative.py:91-93)

  SPX_STAMP2(5, 6);
  // P5: totals, one lane per spectrum (n <= 64): wave 0 sums row i, wave 1 column i, each
  // with numpy's leaf order -- 8 strided accumulators over j < lim = n - n % 8 (in order),
  // combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the sequential tail; n < 8 is all
  // tail.  D's zeros (below the diagonal) are skipped: adding +0.0 to a sum of d >= 0
  // changes nothing.  (16 lanes per spectrum and 4 rounds of 16 spectra measured slower.)
  const bool colside = wid == 1;
  const int i5 = lane;
  const bool valid5 = i5 < n;
  double sum = 0.0;
  if (tid < 2 * kWave) {  // waves 0 and 1
    const int i = i5;
    const bool valid = valid5;
    const int lim = n >= 8 ? n - n % 8 : 0;
    auto term = [&](int j) -> double {
      const bool use = valid && (colside ? j <= i : j >= i);
      return use ? (colside ? L.u.d[row_start(j) + i - j] : L.u.d[row_start(i) + j - i]) : 0.0;
    };
    double r[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = 0.0;
    for (int j0 = 0; j0 < lim; j0 += 8) {  // uniform
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = term(j0 + k);
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] += v[k];
    }
    sum = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int j = lim; j < n; ++j) sum += term(j);  // the sequential tail
    sum = 0.0 + sum;
    if (colside && valid) L.u.t.col[i] = sum;
  }
  lds_barrier();  // every wave
  if (wid == 0 && valid5) {
    const double t = (sum + L.u.t.col[i5]) / (double)n;  // (row + col) / n
    L.totals[i5] = t;
    if (totals_out) totals_out[s0 + i5] = t;
    sum = t;  // wave 0 keeps lane i's total for P6
  }
  // P6 straight from wave 0's registers (lane i holds total i): no barrier, no LDS
  SPX_STAMP2(6, -1);
  if (wid == 0) {
    double t = valid5 ? sum : __longlong_as_double(0x7ff0000000000000ll);
    int idx = tid < n ? tid : 0x7fffffff;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const double t2 = __shfl_xor(t, o, kWave);
      const int i2 = __shfl_xor(idx, o, kWave);
      if (t2 < t || (t2 == t && i2 < idx)) { t = t2; idx = i2; }
    }
    if (tid == 0) rep[c] = s0 + idx;
  }
  SPX_STAMP2(7, 7);
}

// The small-cluster body for one cluster c: BLOCK threads, <= UMAX peaks per
// thread, <= 64 * KWMAX occupied bins.  defer() hands a cluster past those caps on.
template <int BLOCK, int UMAX, int KWMAX, class Defer>
__device__ __forceinline__ void medoid_small_body(const CsrView& v, const MedoidParams& P, int64_t* rep,
                                                  double* totals_out, MedoidRegSmem<BLOCK, UMAX, KWMAX>& L,
                                                  int64_t c, const Defer& defer) {
  constexpr int PMAX = UMAX * BLOCK;
  constexpr int NWV = BLOCK / kWave;
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  SPX_STAMP(0);
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  if (s1 - s0 > MD_NMAX) {
    if (tid == 0) defer(c, s0, n);
    return;
  }
  if (n <= 1) {
    if (tid == 0) {
      rep[c] = n == 1 ? s0 : -1;
      if (totals_out && n == 1) totals_out[s0] = 0.0;
    }
    return;
  }
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  const int np = (int)(p1 - p0);
  if (p1 - p0 > PMAX) {
    if (tid == 0) defer(c, s0, n);
    return;
  }
  const double* __restrict__ mzc = v.mz + p0;

  // P0: offsets, spectrum start bits, empty bitmap.  Bins are absolute
  // ceil(mz/tol) in [0, 65,536) (m/z < 6,553.6 at tol 0.1): the xcorr is a set
  // intersection, so neither a range pass nor sorted spectra are needed.
  const int nsw = (np + 63) / 64;
  for (int w = tid; w < nsw; w += BLOCK) L.u.a.sbits[w] = 0ull;
  if (tid <= n) L.soff[tid] = (int32_t)(v.spec_off[s0 + tid] - p0);
  for (int w = tid; w < MR_WMAX; w += BLOCK) L.u.a.bits[w] = 0ull;
  __syncthreads();
  if (tid < kWave) {  // n <= 64: wave 0 holds every spectrum
    const bool empty_spec = tid < n && L.soff[tid + 1] == L.soff[tid];
    // the whole wave votes (a ballot inside `if (tid == 0)` would see lane 0 only)
    const unsigned long long any_empty = __ballot(empty_spec);
    if (tid == 0) L.red[1] = any_empty != 0ull;
  }
  for (int j = 1 + tid; j < n; j += BLOCK) {
    const int r = L.soff[j];
    // end bits: peak r - 1 closes spectrum j - 1 (r >= 1 unless spectrum 0 is
    // empty, and then the binary search decides)
    if (r >= 1 && r < np) atomicOr(&L.u.a.sbits[(r - 1) >> 6], 1ull << ((r - 1) & 63));
  }
  __syncthreads();
  const bool has_empty = L.red[1] != 0;
  if (tid < kWave) {  // prefix of start bits (<= 192 words, one wave)
    int carry = 0;
    for (int w0 = 0; w0 < nsw; w0 += kWave) {
      const int w = w0 + tid;
      const int c1 = w < nsw ? __popcll(L.u.a.sbits[w]) : 0;
      const int inc = wave_inclusive_sum(c1);
      if (w < nsw) L.u.a.spre[w] = (uint8_t)(carry + inc - c1);
      carry += __shfl(inc, kWave - 1, kWave);
    }
  }

  SPX_STAMP(1);
  // P1: one read of every m/z; bins packed two per register.  Batches of 8
  // loads per thread, double-buffered (batch b+1 in flight while b is binned).
  // The batch count is a compile-time constant per size class, so every load
  // is unconditional: no ring register is ever a merge of a load and another
  // value, and the compiler waits with counted vmcnt.
  uint32_t bins[UMAX / 2];
  int outside = 0;
  constexpr uint32_t kBins = (uint32_t)MR_WMAX * 64u;
  constexpr int NB = UMAX / 8;
  auto pass1 = [&](auto nbt_c) __attribute__((always_inline)) {
    constexpr int NBT = decltype(nbt_c)::value;
    double mb[2][8];
#pragma unroll
    for (int bt = 0; bt <= NBT; ++bt) {
      if (bt < NBT) {  // issue batch bt
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int r = (bt * 8 + q) * BLOCK + tid;
          mb[bt & 1][q] = mzc[r < np ? r : 0];
        }
      }
      if (bt > 0) {  // bin batch bt - 1
        const int pb = bt - 1;
        uint32_t* const bits32 = reinterpret_cast<uint32_t*>(L.u.a.bits);
        uint32_t bad = 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int u = pb * 8 + q;
          const int r = u * BLOCK + tid;
          uint32_t b = 0u;
          if (r < np) {
            // the reciprocal product's ceil, when it is certain and inside the
            // bitmap (|q| >= 2^24 saturates out of it); anything else -- a quotient
            // near an integer, NaN, a bin outside [0, kBins) -- is settled below
            const double qt = mb[pb & 1][q] * P.inv_tol;
            const double t = ceil(qt);
            const double f = t - qt;
            const uint32_t bf = (uint32_t)__double2int_rz(t);
            const bool ok = (f > kDivBand) & (f < 1.0 - kDivBand) & (bf < kBins);
            bad |= (uint32_t)!ok << q;
            // no bin yet: 0 ORed into a word of the lane's own (same-address LDS
            // atomics serialise); 32-bit halves of the occupancy words likewise
            b = ok ? bf : (uint32_t)lane << 5;
            atomicOr(bits32 + (b >> 5), ok ? 1u << (b & 31) : 0u);
          }
          if (u & 1) bins[u >> 1] |= b << 16;
          else bins[u >> 1] = b;
        }
        if (__builtin_expect(bad != 0u, 0)) {  // ~1 peak in 10^7: md_bin's exact divide decides
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if ((bad >> q) & 1u) {
              const int u = pb * 8 + q;
              const int64_t bb = md_bin(mb[pb & 1][q], P);
              if (bb < 0 || bb >= (int64_t)kBins) {
                outside = 1;
              } else {
                const uint32_t b = (uint32_t)bb, s = 16 * (u & 1);
                atomicOr(bits32 + (b >> 5), 1u << (b & 31));
                bins[u >> 1] = (bins[u >> 1] & ~(0xFFFFu << s)) | (b << s);
              }
            }
          }
        }
      } else if (bt > 0) {
        const int pb = bt - 1;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int u = pb * 8 + q;
          const int r = u * BLOCK + tid;
          uint32_t b = 0u;
          if (r < np) {
            const int64_t bb = md_bin(mb[pb & 1][q], P);
            if (bb < 0 || bb >= (int64_t)kBins) {
              outside = 1;
            } else {
              b = (uint32_t)bb;
              // 32-bit half of the occupancy word (same-address LDS atomics serialise)
              atomicOr(reinterpret_cast<uint32_t*>(&L.u.a.bits[b >> 6]) + ((b >> 5) & 1), 1u << (b & 31));
            }
          }
          if (u & 1) bins[u >> 1] |= b << 16;
          else bins[u >> 1] = b;
        }
      }
    }
  };
  switch ((np + 8 * BLOCK - 1) / (8 * BLOCK)) {  // uniform size class
    case 0: break;
    case 1: pass1(std::integral_constant<int, 1>{}); break;
    case 2: pass1(std::integral_constant<int, 2>{}); break;
    case 3: pass1(std::integral_constant<int, 3>{}); break;
    case 4: pass1(std::integral_constant<int, 4>{}); break;
    case 5: pass1(std::integral_constant<int, 5>{}); break;
    case 6: pass1(std::integral_constant<int, (NB < 6 ? NB : 6)>{}); break;
    case 7: pass1(std::integral_constant<int, (NB < 7 ? NB : 7)>{}); break;
    default: pass1(std::integral_constant<int, NB>{}); break;
  }
  static_assert(NB >= 5 && NB <= 8, "size classes above cover 40..64 peaks per thread");
  if (block_any<BLOCK, true>(outside, L.votes, 0)) {  // m/z out of the LDS bitmap's range: general path
    if (tid == 0) defer(c, s0, n);
    return;
  }
  SPX_STAMP(2);
  // P2: compact columns (exclusive popcount prefix into the records)
  int K;
  {
    // all MR_WMAX records (P0 cleared them), RPT
    // contiguous per thread, read unconditionally: the reads pipeline
    // per 32-bit word: a u16 prefix (K <= 32,768) in the same 2 KB
    constexpr int RPT = 2 * MR_WMAX / BLOCK;
    const int w0 = tid * RPT;
    const uint32_t* const bits32 = reinterpret_cast<const uint32_t*>(L.u.a.bits);
    uint16_t* const pre16 = reinterpret_cast<uint16_t*>(L.u.a.pre);
    uint32_t b[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) b[k] = bits32[w0 + k];
    int local = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) local += __popc(b[k]);
    int base = block_exclusive_scan<BLOCK, int, true>(local, L.tmp, K);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      pre16[w0 + k] = (uint16_t)base;
      base += __popc(b[k]);
    }
  }
  // row stride KW is odd: lanes reading rows j, j+1, ... at one word hit
  // different LDS banks (an even stride of u64s would fold them together)
  const int KW = ((K + 63) / 64) | 1;
  if (KW > KWMAX) {
    if (tid == 0) defer(c, s0, n);
    return;
  }
  SPX_STAMP(3);
  // P3: bit-packed rows from the register bins
  for (int w = tid; w < n * KW; w += BLOCK) L.u.a.rows[w] = 0ull;
  // start-bit word NWV*u + wid and its prefix for slice u, lane u holds them
  unsigned long long my_sw = 0ull;
  int my_sp = 0;
  {
    const int w = NWV * lane + wid;
    if (lane < UMAX && w < nsw) { my_sw = L.u.a.sbits[w]; my_sp = L.u.a.spre[w]; }
  }
  __syncthreads();
  const uint32_t swz_nw = 2u * (uint32_t)KW;  // 32-bit words per row
  const uint32_t swz_m = swz_nw >= 32u ? 31u : (1u << (31 - __clz((int)swz_nw))) - 1u;  // 2^k - 1 < swz_nw
#pragma unroll
  for (int u = 0; u < UMAX; ++u) {
    if (u * BLOCK < np) {  // uniform
      const int r = u * BLOCK + tid;
      const uint32_t swlo = __builtin_amdgcn_readlane((uint32_t)my_sw, u);
      const uint32_t swhi = __builtin_amdgcn_readlane((uint32_t)(my_sw >> 32), u);
      const int spw = __builtin_amdgcn_readlane(my_sp, u);
      if (r < np) {
        const uint32_t b = (bins[u >> 1] >> (16 * (u & 1))) & 0xFFFFu;
        // rank in a 32-bit word: its u16 prefix + the popcount of the bits below b
        const uint32_t w32 = b >> 5;
        const int col = (int)reinterpret_cast<const uint16_t*>(L.u.a.pre)[w32] +
                        __popc(__builtin_amdgcn_ubfe(reinterpret_cast<const uint32_t*>(L.u.a.bits)[w32], 0u, b & 31u));
        // empty spectra share a start bit: then the binary search
        const unsigned long long sw = ((unsigned long long)swhi << 32) | swlo;
        // spectra closed before peak r: the word's prefix + its end bits below this
        // lane (peak r is bit `lane` of its word) -- two v_mbcnt
        (void)sw;
        const int sp = has_empty ? spectrum_of(L.soff, n, r)
                                 : (int)__builtin_amdgcn_mbcnt_hi(swhi, __builtin_amdgcn_mbcnt_lo(swlo, (uint32_t)spw));
        // 32-bit halves: consecutive peaks of a spectrum share a row word, and
        // same-address LDS atomics serialise -- half as many per address
        // word (col/32 + (col & m)) mod NW32: a bijection per bit position, so P4's
        // row-AND popcounts and Gram sums are unchanged, while neighbouring columns of a
        // spectrum -- consecutive lanes -- land in different words (a shared word
        // serialises the LDS atomic: ~6 lanes per word unswizzled)
        uint32_t wq = (uint32_t)(col >> 5) + ((uint32_t)col & swz_m);
        wq = min(wq, wq - swz_nw);
        atomicOr(reinterpret_cast<uint32_t*>(&L.u.a.rows[__mul24(sp, KW)]) + wq, 1u << (col & 31));
      }
    }
  }
  medoid_tail<BLOCK, UMAX, KWMAX>(L, n, KW, s0, c, rep, totals_out);
}

// Register kernel: one 256-thread workgroup per cluster.  Clusters past its caps
// go to the wide kernel's list.
// Whether a cluster goes to the large path by its size alone (spx_api.hip's
// medoid_large_by_size): more than MD_NMAX spectra, or more peaks than the wide kernel holds.
__device__ __forceinline__ bool md_large_by_size(const CsrView& v, int64_t s0, int n) {
  return n > MD_NMAX || v.spec_off[s0 + n] - v.spec_off[s0] > MW_PMAX;
}

// The medoid intake (spx_medoid, round 6): every cluster large by size deferred up front
// into a list of its own, so its large path runs on the call's second stream BESIDE the
// register and wide kernels; the register kernel (own = 1) leaves those clusters alone.
__global__ __launch_bounds__(256) void medoid_intake_kernel(CsrView v, int64_t* rep, int32_t* deferred,
                                                            int32_t* n_deferred, MedoidMeta* meta) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < v.n_clusters;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s0 = v.cluster_off[c];
    const int n = (int)(v.cluster_off[c + 1] - s0);
    if (md_large_by_size(v, s0, n)) md_defer(c, s0, n, deferred, n_deferred, meta, rep);
  }
}

__global__ __launch_bounds__(MD_BLOCK, SPX_MD_MINW) void medoid_reg_kernel(CsrView v, MedoidParams P, int64_t* rep,
                                                              double* totals_out, StripedList wide, int own) {
  __shared__ MedoidRegSmem<MD_BLOCK, MR_UMAX, MD_KWMAX> L;
  auto defer = [&](int64_t c, int64_t s0, int n) {
    if (own && md_large_by_size(v, s0, n)) return;  // the intake's (its rep is the large path's to write)
    // every leftover via the wide kernel, which passes n > 64 straight on (one
    // list target here keeps the kernel's register budget)
    rep[c] = -4;
    striped_push(wide, (int32_t)c);
  };
  medoid_small_body<MD_BLOCK, MR_UMAX, MD_KWMAX>(v, P, rep, totals_out, L, (int64_t)blockIdx.x, defer);
}

// Wide kernel: the register kernel's leftovers, grid-stride; what it cannot hold
// (n > 64 first of all) goes on to the large path.
__global__ __launch_bounds__(MW_BLOCK, 4) void medoid_wide_kernel(CsrView v, MedoidParams P, int64_t* rep,
                                                                  double* totals_out, StripedList wide,
                                                                  int32_t* deferred, int32_t* n_deferred,
                                                                  MedoidMeta* meta) {
  __shared__ MedoidRegSmem<MW_BLOCK, MW_UMAX, MW_KWMAX> L;
  __shared__ int32_t lbase[kListStripes + 1];
  const int32_t nw = striped_prefix(wide, lbase);
  for (int32_t i = blockIdx.x; i < nw; i += gridDim.x) {
    medoid_small_body<MW_BLOCK, MW_UMAX, MW_KWMAX>(v, P, rep, totals_out, L, (int64_t)striped_at(wide, lbase, i),
                                                  [&](int64_t c, int64_t s0, int n) {
      md_defer(c, s0, n, deferred, n_deferred, meta, rep);
    });
    __syncthreads();  // the LDS is reused by the next cluster
  }
}

// ------------------------------------------------------------ large path
// Clusters the LDS kernel defers (n > 64, or too many bins/peaks) go through
// grid-parallel passes over ONE bump-allocated arena (one workgroup per
// cluster only for the small planning steps):
//   range   (grid)   bin range; allocates the level-1 bitmap
//   l1      (grid)   level-1 occupancy (one bit per 64-bin block), LDS-staged
//   plan1   (WG/cl)  level-1 prefix; allocates the level-2 words
//   l2      (grid)   level-2 occupancy (one bit per occupied bin)
//   plan2   (WG/cl)  level-2 prefix -> K compact columns; allocates rows, counts,
//                    numpy's leaf segmentation and leaf sums
//   scan    (1 WG)   Gram-tile, leaf-unit and transpose-tile bases over the deferred clusters
//   fill    (grid)   bit rows, 1 bit per occupied column (the OpenMS binary
//                    ion table, compacted)
//   xpose   (grid)   bit rows row-major -> word-major (64 x 64-word LDS tiles)
//   gram    (MFMA)   c_ij = |B_i ∩ B_j|, v_mfma_i32_32x32x32_i8 on 0/1 bytes
//                    expanded in registers, one 64 x 64 tile per wave
//   leaves  (grid)   numpy pairwise-tree leaf sums of row i and column i
//   combine (WG/cl)  the tree over the leaf sums -> totals, lowest-index argmin
constexpr int MD_L1WORDS = 1024;  // level-1 bits: 65,536 blocks = 4.2M bins
constexpr int MD_L2LDS = 4096;    // level-2 words staged in LDS (else global atomics)
constexpr int MD_GT = 128;        // rows padded to a multiple
constexpr int MD_WT = 64;         // register Gram: one wave's 64-row output tile
#ifndef SPX_GR_NB
#define SPX_GR_NB 2
#endif
constexpr int MD_GR_NB = SPX_GR_NB;  // 32-column MFMA blocks per wave tile (64 x 128 measured: no faster)
constexpr int MD_WTN = 32 * MD_GR_NB;  // wave tile columns

// Wave tiles of a cluster: 64-row blocks ti against MD_WTN-column blocks tj that
// reach the upper triangle (tj * MD_WTN + MD_WTN - 1 >= ti * 64).
__host__ __device__ __forceinline__ int md_gr_first_tj(int ti) { return (ti * MD_WT) / MD_WTN; }
__host__ __device__ __forceinline__ int64_t md_gr_tiles(int n) {
  const int T = (n + MD_WT - 1) / MD_WT, TN = (n + MD_WTN - 1) / MD_WTN;
  int64_t t = 0;
  for (int ti = 0; ti < T; ++ti) t += TN - md_gr_first_tj(ti);
  return t;
}

constexpr int MD_GRIDX = 64;      // blocks per cluster in the grid-parallel passes

__host__ __device__ __forceinline__ int64_t md_align(int64_t b) { return (b + 255) & ~int64_t(255); }
__host__ __device__ __forceinline__ int64_t md_l1_bytes() { return md_align((int64_t)MD_L1WORDS * 12); }
__host__ __device__ __forceinline__ int64_t md_max_leaves(int64_t n) { return n / 32 + 2; }

__device__ __forceinline__ unsigned long long md_key(int64_t b) {
  return (unsigned long long)b ^ 0x8000000000000000ull;
}
__device__ __forceinline__ int64_t md_unkey(unsigned long long k) { return (int64_t)(k ^ 0x8000000000000000ull); }

struct MedoidTables {  // views into the arena
  const unsigned long long* l1;
  const uint32_t* l1pre;
  const unsigned long long* l2;
  const uint32_t* l2pre;
  __device__ __forceinline__ int column(int64_t rel) const {
    const int bs = bitmap_rank(l1, l1pre, rel >> 6);
    return (int)l2pre[bs] + __popcll(l2[bs] & ((1ull << (rel & 63)) - 1ull));
  }
};

__device__ __forceinline__ MedoidTables md_tables(const char* arena, const MedoidMeta& M) {
  MedoidTables T;
  T.l1 = reinterpret_cast<const unsigned long long*>(arena + M.l1_off);
  T.l1pre = reinterpret_cast<const uint32_t*>(arena + M.l1_off + (int64_t)MD_L1WORDS * 8);
  T.l2 = reinterpret_cast<const unsigned long long*>(arena + M.l2_off);
  T.l2pre = reinterpret_cast<const uint32_t*>(arena + M.l2_off + (int64_t)M.B1 * 8);
  return T;
}

__device__ __forceinline__ int64_t md_bump(unsigned long long* bump, int64_t bytes, int64_t cap) {
  const int64_t b = (int64_t)atomicAdd(bump, (unsigned long long)bytes);
  return b + bytes > cap ? -1 : b;
}

// which deferred cluster owns work item t (base[lo] <= t < base[lo + 1], skipping empties)
__device__ __forceinline__ int md_owner(const int64_t* base, int nd, int64_t t) {
  int lo = 0, hi = nd;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (base[mid] <= t) lo = mid; else hi = mid;
  }
  while (lo + 1 < nd && base[lo + 1] <= t) ++lo;
  return lo;
}

// Units of the three peak passes (range, level 1, level 2): per deferred cluster its
// peak range and ceil(peaks / MD_PU) units of MD_PU peaks (one at least: unit 0 also
// allocates the level-1 bitmap), exclusive-scanned into pk_base (one workgroup).  A
// flat grid over units keeps every block on one unit of 64 peaks per thread, where a
// fixed 64 blocks per cluster gave the 442 clusters of configs[3] ~4 peaks per thread
// per cluster and a dependent meta -> offsets -> m/z chain for each.
constexpr int MD_PU = 16384;

__global__ __launch_bounds__(MD_BLOCK) void medoid_units_kernel(CsrView v, MedoidMeta* meta, const int32_t* n_deferred,
                                                                int64_t* pk_base) {
  __shared__ int64_t tmp[MD_BLOCK / kWave + 1];
  const int32_t nd = *n_deferred;
  int64_t cu = 0;
  for (int32_t i0 = 0; i0 < nd; i0 += MD_BLOCK) {  // uniform
    const int32_t i = i0 + (int32_t)threadIdx.x;
    int64_t units = 0;
    if (i < nd) {
      const int64_t s0 = meta[i].s0;
      const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s0 + meta[i].n];
      meta[i].p0 = p0;
      meta[i].np = p1 - p0;
      units = p1 > p0 ? (p1 - p0 + MD_PU - 1) / MD_PU : 1;
    }
    int64_t tot;
    const int64_t e = block_exclusive_scan<MD_BLOCK>(units, tmp, tot);
    if (i < nd) pk_base[i] = cu + e;
    cu += tot;
  }
  if (threadIdx.x == 0) pk_base[nd] = cu;
}

// a unit's peaks [k0, k1) and its cluster
__device__ __forceinline__ int md_unit(const int64_t* pk_base, int nd, const MedoidMeta* meta, int64_t u, int64_t& r,
                                       int64_t& k0, int64_t& k1) {
  const int o = md_owner(pk_base, nd, u);
  r = u - pk_base[o];
  const int64_t p0 = meta[o].p0, p1 = p0 + meta[o].np;
  k0 = p0 + r * MD_PU;
  k1 = k0 + MD_PU < p1 ? k0 + MD_PU : p1;
  return o;
}

// f(k, m) for every peak k of [k0, k1): thread tid takes k0 + tid + j * MD_BLOCK,
// eight m/z loads in flight at a time
template <class F>
__device__ __forceinline__ void md_unit_peaks(const CsrView& v, int64_t k0, int64_t k1, const F& f) {
  for (int64_t kb = k0 + threadIdx.x; kb < k1; kb += 8 * MD_BLOCK) {
    double m[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int64_t k = kb + (int64_t)q * MD_BLOCK;
      m[q] = k < k1 ? v.mz[k] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (kb + (int64_t)q * MD_BLOCK < k1) f(m[q]);
  }
}

// f(m, active) for every lane on every round of [k0, k1) (uniform: the whole wave
// calls f, lanes past k1 with active = false), eight m/z loads in flight at a time
template <class F>
__device__ __forceinline__ void md_unit_peaks_all(const CsrView& v, int64_t k0, int64_t k1, const F& f) {
  for (int64_t kb = k0; kb < k1; kb += 8 * MD_BLOCK) {  // uniform
    double m[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int64_t k = kb + (int64_t)q * MD_BLOCK + threadIdx.x;
      m[q] = k < k1 ? v.mz[k] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) f(m[q], kb + (int64_t)q * MD_BLOCK + threadIdx.x < k1);
  }
}

// Pass 1: bin range of every deferred cluster (wave-reduced atomics on
// order-preserving keys; lo is stored complemented so both are maxima).
// Unit 0 of a cluster also allocates and zeroes its level-1 bitmap.
__global__ __launch_bounds__(MD_BLOCK) void medoid_range_kernel(CsrView v, MedoidParams P, const int32_t* n_deferred,
                                                                MedoidMeta* meta, const int64_t* pk_base, char* arena,
                                                                unsigned long long* bump, int64_t arena_bytes) {
  __shared__ int64_t base_sh;
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  const int64_t total = pk_base[nd];
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {  // uniform
    int64_t r, k0, k1;
    const int o = md_unit(pk_base, nd, meta, u, r, k0, k1);
    MedoidMeta* M = meta + o;
    if (r == 0) {
      if (tid == 0) base_sh = md_bump(bump, md_l1_bytes(), arena_bytes);
      __syncthreads();
      const int64_t base = base_sh;
      if (base >= 0) {
        unsigned long long* l1 = reinterpret_cast<unsigned long long*>(arena + base);
        for (int w = tid; w < MD_L1WORDS; w += MD_BLOCK) l1[w] = 0ull;
      }
      if (tid == 0) M->l1_off = base;
      __syncthreads();
    }
    long long lo = 0x7fffffffffffffffll, hi = -0x7fffffffffffffffll - 1;
    md_unit_peaks(v, k0, k1, [&](double m) {
      const long long b = md_bin(m, P);
      lo = b < lo ? b : lo;
      hi = b > hi ? b : hi;
    });
#pragma unroll
    for (int o2 = kWave / 2; o2 > 0; o2 >>= 1) {
      const long long l2 = __shfl_xor(lo, o2, kWave), h2 = __shfl_xor(hi, o2, kWave);
      lo = l2 < lo ? l2 : lo;
      hi = h2 > hi ? h2 : hi;
    }
    if (lane_id() == 0 && lo <= hi) {
      atomicMax(&M->hi_key, md_key(hi));
      atomicMax(&M->lo_key, ~md_key(lo));
    }
  }
}

__device__ __forceinline__ bool md_range(const MedoidMeta& M, int64_t& blo, int& nw1) {
  if (M.hi_key == 0ull) { blo = 0; nw1 = 0; return true; }  // no peaks at all
  blo = md_unkey(~M.lo_key);
  const int64_t bhi = md_unkey(M.hi_key);
  const int64_t nblk = ((bhi - blo) >> 6) + 1;
  const int64_t w = (nblk + 63) / 64;
  nw1 = w > MD_L1WORDS ? -1 : (int)w;
  return w <= MD_L1WORDS;
}

// Pass 2: level-1 occupancy, staged in LDS, merged with one atomicOr per word.
__global__ __launch_bounds__(MD_BLOCK) void medoid_l1_kernel(CsrView v, MedoidParams P, const int32_t* n_deferred,
                                                             const MedoidMeta* meta, const int64_t* pk_base,
                                                             char* arena) {
  __shared__ unsigned long long l1s[MD_L1WORDS];
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  const int64_t total = pk_base[nd];
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {  // uniform
    int64_t r, k0, k1;
    const MedoidMeta M = meta[md_unit(pk_base, nd, meta, u, r, k0, k1)];
    int64_t blo;
    int nw1;
    if (M.l1_off < 0 || !md_range(M, blo, nw1) || nw1 == 0 || k0 >= k1) continue;
    for (int w = tid; w < nw1; w += MD_BLOCK) l1s[w] = 0ull;
    __syncthreads();
    // neighbouring peaks fall in the same 64-bin block or the next: ~40 lanes of a
    // wave OR into one level-1 word, so each run of lanes with one 32-bit word
    // ORs its bits together first and its last lane issues the atomic
    uint32_t* const l1s32 = reinterpret_cast<uint32_t*>(l1s);
    md_unit_peaks_all(v, k0, k1, [&](double m, bool act) {
      const int64_t blk = act ? (md_bin(m, P) - blo) >> 6 : 0;
      const uint32_t key = act ? (uint32_t)(blk >> 5) : 0xFFFFFFFEu;
      uint32_t val = act ? 1u << (blk & 31) : 0u;
      if (wave_or_runs(key, val) && act) atomicOr(&l1s32[key], val);
    });
    __syncthreads();
    unsigned long long* l1 = reinterpret_cast<unsigned long long*>(arena + M.l1_off);
    for (int w = tid; w < nw1; w += MD_BLOCK)
      if (l1s[w]) atomicOr(&l1[w], l1s[w]);
    __syncthreads();
  }
}

// Plan 1 (one workgroup per cluster): level-1 prefix, allocate + zero level 2.
__global__ __launch_bounds__(MD_BLOCK) void medoid_plan1_kernel(const int32_t* n_deferred, MedoidMeta* meta,
                                                                char* arena, unsigned long long* bump,
                                                                int64_t arena_bytes, int64_t* rep) {
  __shared__ unsigned long long l1s[MD_L1WORDS];
  __shared__ uint32_t pre[MD_L1WORDS];
  __shared__ int tmp[MD_BLOCK / kWave + 1];
  __shared__ int64_t base_sh;
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    MedoidMeta* M = meta + di;
    int64_t blo;
    int nw1;
    const bool fits = md_range(*M, blo, nw1);
    if (M->l1_off < 0 || !fits) {  // > 4.2M bins (-2) or arena exhausted (-3): reported, not approximated
      if (tid == 0) rep[M->c] = fits ? -3 : -2;
      continue;
    }
    const unsigned long long* l1 = reinterpret_cast<const unsigned long long*>(arena + M->l1_off);
    for (int w = tid; w < nw1; w += MD_BLOCK) l1s[w] = l1[w];
    __syncthreads();
    const int B1 = bitmap_prefix<MD_BLOCK>(l1s, pre, nw1, tmp);
    uint32_t* l1pre = reinterpret_cast<uint32_t*>(arena + M->l1_off + (int64_t)MD_L1WORDS * 8);
    for (int w = tid; w < nw1; w += MD_BLOCK) l1pre[w] = pre[w];
    if (tid == 0) base_sh = md_bump(bump, md_align((int64_t)B1 * 12 + 8), arena_bytes);
    __syncthreads();
    const int64_t base = base_sh;
    if (base < 0) {
      if (tid == 0) { rep[M->c] = -3; M->l1_off = -1; }
      __syncthreads();
      continue;
    }
    unsigned long long* l2 = reinterpret_cast<unsigned long long*>(arena + base);
    for (int w = tid; w < B1; w += MD_BLOCK) l2[w] = 0ull;
    if (tid == 0) { M->blo = blo; M->nw1 = nw1; M->B1 = B1; M->l2_off = base; }
    __syncthreads();
  }
}

// Pass 3: level-2 occupancy (LDS-staged when the cluster's level-2 fits).
__global__ __launch_bounds__(MD_BLOCK) void medoid_l2_kernel(CsrView v, MedoidParams P, const int32_t* n_deferred,
                                                             const MedoidMeta* meta, const int64_t* pk_base,
                                                             char* arena) {
  __shared__ unsigned long long l2s[MD_L2LDS];
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  const int64_t total = pk_base[nd];
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {  // uniform
    int64_t r, k0, k1;
    const MedoidMeta M = meta[md_unit(pk_base, nd, meta, u, r, k0, k1)];
    if (M.l1_off < 0 || M.l2_off == 0 || M.B1 == 0 || k0 >= k1) continue;
    const MedoidTables T = md_tables(arena, M);
    unsigned long long* l2 = reinterpret_cast<unsigned long long*>(arena + M.l2_off);
    const bool staged = M.B1 <= MD_L2LDS;
    if (staged) {
      for (int w = tid; w < M.B1; w += MD_BLOCK) l2s[w] = 0ull;
      __syncthreads();
    }
    md_unit_peaks(v, k0, k1, [&](double m) {
      const int64_t rel = md_bin(m, P) - M.blo;
      const int bs = bitmap_rank(T.l1, T.l1pre, rel >> 6);
      if (staged) atomicOr(&l2s[bs], 1ull << (rel & 63));
      else atomicOr(&l2[bs], 1ull << (rel & 63));
    });
    if (staged) {
      __syncthreads();
      for (int w = tid; w < M.B1; w += MD_BLOCK)
        if (l2s[w]) atomicOr(&l2[w], l2s[w]);
      __syncthreads();
    }
  }
}

// Plan 2 (one workgroup per cluster): level-2 prefix -> K columns; allocate
// rows (bit-packed, KW multiple of 8 words, rows padded to Gram tiles), the
// count matrix, numpy's leaf segmentation of [0, n) and the leaf sums.
__global__ __launch_bounds__(MD_BLOCK) void medoid_plan2_kernel(const int32_t* n_deferred, MedoidMeta* meta,
                                                                char* arena, unsigned long long* bump,
                                                                int64_t arena_bytes, int64_t* rep) {
  __shared__ int tmp[MD_BLOCK / kWave + 1];
  __shared__ int64_t base_sh;
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    MedoidMeta* M = meta + di;
    if (M->l1_off < 0) continue;
    int K = 0;
    if (M->B1 > 0) {
      unsigned long long* l2 = reinterpret_cast<unsigned long long*>(arena + M->l2_off);
      uint32_t* l2pre = reinterpret_cast<uint32_t*>(arena + M->l2_off + (int64_t)M->B1 * 8);
      K = bitmap_prefix<MD_BLOCK>(l2, l2pre, M->B1, tmp);
    }
    const int n = M->n;
    const int KW = ((K + 63) / 64 + 7) / 8 * 8 > 0 ? ((K + 63) / 64 + 7) / 8 * 8 : 8;
    const int T = (n + MD_GT - 1) / MD_GT;
    const int64_t maxL = md_max_leaves(n);
    const int64_t rows_b = md_align((int64_t)T * MD_GT * KW * 8);
    const int64_t cmat_b = md_align((int64_t)n * n * 4);
    const int64_t leaf_b = md_align((2 * maxL + 1) * 4);        // leaf starts, leaf node ids
    const int64_t lsum_b = md_align(2 * (2 * maxL) * (int64_t)n * 8);  // node values, row and column
    const int64_t tot_b = md_align((int64_t)n * 8);
    const int64_t rowsT_b = rows_b;  // the word-major copy the Gram kernel reads
    if (tid == 0) base_sh = md_bump(bump, rows_b + rowsT_b + cmat_b + leaf_b + lsum_b + tot_b, arena_bytes);
    __syncthreads();
    const int64_t base = base_sh;
    if (base < 0) {
      if (tid == 0) rep[M->c] = -3;
      __syncthreads();
      continue;
    }
    if (tid == 0) {
      // numpy's recursion over [0, n) (split at h = len/2 - (len/2) % 8 down to
      // leaves of <= 128), numbered in post-order: leaf k's start and node id, and
      // (implicitly) the internal nodes that complete right after it -- the
      // ancestors below its deepest left turn.  Each leaf is found by a descent
      // from the root in registers (no stack: a stack in LDS or scratch made this
      // walk a memory round trip per step).  medoid_combine_kernel runs the same
      // post-order as a stack machine over the ids.
      int32_t* start = reinterpret_cast<int32_t*>(arena + base + rows_b + rowsT_b + cmat_b);  // [maxL + 1]
      int32_t* lnode = start + (maxL + 1);                                           // [maxL]
      int nl = 0, nid = 0;
      for (int64_t pos = 0; pos < n;) {
        int64_t lo = 0, len = n;
        int depth = 0, lastleft = -1;
        while (len > 128) {
          int64_t h = len / 2;
          h -= h % 8;
          if (pos < lo + h) {
            len = h;
            lastleft = depth;
          } else {
            lo += h;
            len -= h;
          }
          ++depth;
        }
        start[nl] = (int32_t)lo;
        lnode[nl++] = nid++;
        nid += depth - 1 - lastleft;  // the internal nodes this leaf completes
        pos = lo + len;
      }
      start[nl] = n;
      M->KW = KW;
      M->L = nl;
      M->rows_off = base;
      M->rowsT_off = base + rows_b;
      M->cmat_off = base + rows_b + rowsT_b;
      M->leaf_off = M->cmat_off + cmat_b;
      M->lsum_off = M->leaf_off + leaf_b;
      M->tot_off = M->lsum_off + lsum_b;
      M->tiles = md_gr_tiles(n);
      M->units = ((n + MD_BLOCK - 1) / MD_BLOCK) * nl;
      M->ok = 1;
    }
    __syncthreads();
  }
}

// Exclusive scans of Gram tiles and leaf units over the deferred clusters (one workgroup).
#ifndef SPX_MD_XP_ROWS
#define SPX_MD_XP_ROWS 32  // transpose tiles of 32 rows x 64 words (16.6 KB of LDS: 9 workgroups per CU)
#endif
constexpr int MD_XPR = SPX_MD_XP_ROWS;
__device__ __forceinline__ int64_t md_xpose_tiles(const MedoidMeta& M) {  // MD_XPR x 64-word transpose tiles
  return (int64_t)((M.n + MD_GT - 1) / MD_GT * MD_GT / MD_XPR) * ((M.KW + 63) / 64);
}

__global__ __launch_bounds__(MD_BLOCK) void medoid_scan_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                               int64_t* tile_base, int64_t* unit_base,
                                                               int64_t* chunk_base, int64_t* xpose_base,
                                                               int64_t* row_base) {
  __shared__ int64_t tmp[MD_BLOCK / kWave + 1];
  const int32_t nd = *n_deferred;
  int64_t ct = 0, cu = 0, cc = 0, cx = 0, cr = 0;
  for (int32_t i0 = 0; i0 < nd; i0 += MD_BLOCK) {
    const int32_t i = i0 + threadIdx.x;
    const bool ok = i < nd && meta[i].ok;
    int64_t tot;
    const int64_t et = block_exclusive_scan<MD_BLOCK>(ok ? (int64_t)meta[i].tiles : 0, tmp, tot);
    if (i < nd) tile_base[i] = ct + et;
    ct += tot;
    const int64_t eu = block_exclusive_scan<MD_BLOCK>(ok ? (int64_t)meta[i].units : 0, tmp, tot);
    if (i < nd) unit_base[i] = cu + eu;
    cu += tot;
    const int64_t ec =
        block_exclusive_scan<MD_BLOCK>(ok ? (int64_t)((meta[i].n + MD_BLOCK - 1) / MD_BLOCK) : 0, tmp, tot);
    if (i < nd) chunk_base[i] = cc + ec;
    cc += tot;
    const int64_t ex = block_exclusive_scan<MD_BLOCK>(ok ? md_xpose_tiles(meta[i]) : int64_t(0), tmp, tot);
    if (i < nd) xpose_base[i] = cx + ex;
    cx += tot;
    const int64_t er =
        block_exclusive_scan<MD_BLOCK>(ok ? (int64_t)((meta[i].n + MD_GT - 1) / MD_GT * MD_GT) : 0, tmp, tot);
    if (i < nd) row_base[i] = cr + er;
    cr += tot;
  }
  if (threadIdx.x == 0) {
    tile_base[nd] = ct;
    unit_base[nd] = cu;
    chunk_base[nd] = cc;
    xpose_base[nd] = cx;
    row_base[nd] = cr;
  }
}


// Bit rows, one wave per (padded) row: zero the row's words, drain the stores,
// then OR in one bit per peak (peaks may be unsorted; duplicates are idempotent).
constexpr int MD_FILL_KW = 512;  // row words a wave builds in LDS (4 KB; 32,768 columns)
constexpr int MD_FILL_U = 4;     // 64-peak chunks of a spectrum whose loads go out together

__global__ __launch_bounds__(MD_BLOCK) void medoid_fill_kernel(CsrView v, MedoidParams P, const MedoidMeta* meta,
                                                               const int32_t* n_deferred, const int64_t* row_base,
                                                               char* arena) {
  const int32_t nd = *n_deferred;
  constexpr int W = MD_BLOCK / kWave;
  // One wave per row.  A row of at most MD_FILL_KW words is built in the wave's
  // LDS slice (no zeroing round trip through memory, no global atomics) and then
  // written with plain coalesced stores; the peaks of up to MD_FILL_U chunks
  // issue their m/z loads, then their level-1 and level-2 rank loads, together
  // (three dependent round trips per 256 peaks instead of three per 64).
  __shared__ unsigned long long lrow[W][MD_FILL_KW];
  unsigned long long* L = lrow[wave_id()];
  // Every padded row of every deferred cluster, as one flat list (row_base: the
  // exclusive scan of the padded row counts); wave q takes the contiguous run
  // [q * per, (q + 1) * per), so the owner changes rarely and a giant's rows are
  // spread over the whole grid instead of one y-slot of blocks (the old
  // 64 x 32 grid walked the clusters 32 at a time: the n = 5,000 ones held it).
  const int64_t total = row_base[nd];
  const int64_t nwaves = (int64_t)gridDim.x * gridDim.y * W;
  const int64_t per = (total + nwaves - 1) / nwaves;
  const int64_t q = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * W + wave_id();
  const int64_t g0 = q * per, g1 = g0 + per < total ? g0 + per : total;
  int o = g0 < total ? md_owner(row_base, nd, g0) : 0;
  for (int64_t g = g0; g < g1; ++g) {  // uniform per wave
    while (g >= row_base[o + 1]) ++o;
    const MedoidMeta M = meta[o];
    if (!M.ok) continue;
    const int r = (int)(g - row_base[o]);
    const MedoidTables Tb = md_tables(arena, M);
    unsigned long long* rows = reinterpret_cast<unsigned long long*>(arena + M.rows_off);
    if (M.KW <= MD_FILL_KW) {  // uniform
        unsigned long long* row = rows + (int64_t)r * M.KW;
        for (int w = lane_id(); w < M.KW; w += kWave) L[w] = 0ull;
        if (r < M.n) {
          const int64_t a = v.spec_off[M.s0 + r], e = v.spec_off[M.s0 + r + 1];
          for (int64_t k0 = a; k0 < e; k0 += MD_FILL_U * kWave) {
            double m[MD_FILL_U];
#pragma unroll
            for (int u = 0; u < MD_FILL_U; ++u) {
              const int64_t k = k0 + u * kWave + lane_id();
              m[u] = v.mz[k < e ? k : a];
            }
            int64_t rel[MD_FILL_U];
            unsigned long long w1[MD_FILL_U];
            uint32_t p1[MD_FILL_U];
#pragma unroll
            for (int u = 0; u < MD_FILL_U; ++u) {
              rel[u] = md_bin(m[u], P) - M.blo;
              const int64_t b1 = rel[u] >> 6;  // level-1 bit = the 64-bin block
              w1[u] = Tb.l1[b1 >> 6];
              p1[u] = Tb.l1pre[b1 >> 6];
            }
            unsigned long long w2[MD_FILL_U];
            uint32_t p2[MD_FILL_U];
#pragma unroll
            for (int u = 0; u < MD_FILL_U; ++u) {
              const int64_t b1 = rel[u] >> 6;
              const int bs = (int)p1[u] + __popcll(w1[u] & ((1ull << (b1 & 63)) - 1ull));
              w2[u] = Tb.l2[bs];
              p2[u] = Tb.l2pre[bs];
            }
#pragma unroll
            for (int u = 0; u < MD_FILL_U; ++u) {
              const int64_t k = k0 + u * kWave + lane_id();
              if (k < e) {
                const int col = (int)p2[u] + __popcll(w2[u] & ((1ull << (rel[u] & 63)) - 1ull));
                atomicOr(&L[col >> 6], 1ull << (col & 63));
              }
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int w = lane_id(); w < M.KW; w += kWave) row[w] = L[w];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next row's zeroing after these reads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      continue;
    }
    {
      unsigned long long* row = rows + (int64_t)r * M.KW;
      for (int w = lane_id(); w < M.KW; w += kWave) row[w] = 0ull;
      if (r >= M.n) continue;
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): zeros land before the ORs
      const int64_t a = v.spec_off[M.s0 + r], e = v.spec_off[M.s0 + r + 1];
      for (int64_t k = a + lane_id(); k < e; k += kWave) {
        const int col = Tb.column(md_bin(v.mz[k], P) - M.blo);
        atomicOr(&row[col >> 6], 1ull << (col & 63));
      }
    }
  }
}

typedef int md_i32x4 __attribute__((ext_vector_type(4)));
typedef int md_i32x16 __attribute__((ext_vector_type(16)));

// 64 bins (one u64 row word) -> 64 bytes of 0/1 in 4 x 16 B.  Byte p of dword
// g (g < 8: low word) holds bin g + 8p -- a fixed permutation of the k axis,
// identical for the A and B operands, so the dot products are unchanged.
#ifndef SPX_GR_PF
#define SPX_GR_PF 4
#endif
#ifndef SPX_GR_MINW
#define SPX_GR_MINW 3  // 3 waves per SIMD (167 unified registers, the accumulators in VGPRs)
#endif
constexpr int MD_GR_PF = SPX_GR_PF;  // words in flight per lane (divides 8: KW is a multiple of 8)
// The 0/1 operands as FP4 e2m1 (1.0 = nibble 0b0010) through
// v_mfma_f32_32x32x64_f8f6f4 (the MX-scaled instruction at unit scale): one MFMA per
// 64-bin word and (a, b) block instead of two, from half the expansion VALU (a
// 32-bin half word -> 4 dwords of 8 nibbles, 2 ops each).  Products are 1.0 or 0,
// the f32 accumulation of at most 2^24 of them is exact, so the counts are the
// integer ones.  Peak: the FP4 dense rate (~10 POPS), twice the i8 one.

// Bit rows, row-major [npad][KW] -> word-major [KW][npad] (64 x 64-word tiles
// through LDS: both sides coalesced), for the register Gram's loads.
__global__ __launch_bounds__(MD_BLOCK) void medoid_transpose_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                                    const int64_t* xpose_base, char* arena) {
  // tile = MD_XPR rows x 64 words: read as rows (lane = word), written as words (lane = row)
  __shared__ unsigned long long tile[MD_XPR][65];
  constexpr int RS = MD_BLOCK / 64;      // rows per read step
  constexpr int WS = MD_BLOCK / MD_XPR;  // words per write step
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  const int64_t total = xpose_base[nd];
  for (int64_t g = blockIdx.x; g < total; g += gridDim.x) {  // every tile of every cluster, flat
    const int o = md_owner(xpose_base, nd, g);
    const MedoidMeta M = meta[o];
    const int npad = (M.n + MD_GT - 1) / MD_GT * MD_GT, KW = M.KW;
    const unsigned long long* rows = reinterpret_cast<const unsigned long long*>(arena + M.rows_off);
    unsigned long long* rowsT = reinterpret_cast<unsigned long long*>(arena + M.rowsT_off);
    const int tw = (KW + 63) / 64;
    const int t = (int)(g - xpose_base[o]);
    const int r0 = (t / tw) * MD_XPR, w0 = (t % tw) * 64;
    {
      const int x = tid & 63, y0 = tid >> 6;
#pragma unroll
      for (int y = y0; y < MD_XPR; y += RS)
        tile[y][x] = w0 + x < KW ? rows[(int64_t)(r0 + y) * KW + w0 + x] : 0ull;
    }
    __syncthreads();
    {
      const int x = tid % MD_XPR, y0 = tid / MD_XPR;
#pragma unroll
      for (int y = y0; y < 64; y += WS)
        if (w0 + y < KW) rowsT[(int64_t)(w0 + y) * npad + r0 + x] = tile[x][y];
    }
    __syncthreads();
  }
}
__global__ __launch_bounds__(MD_BLOCK, SPX_GR_MINW) void medoid_gram_reg_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                                   const int64_t* tile_base, char* arena) {
  const int lane = lane_id();
  const int fr = lane & 31, fh = lane >> 5;
  __shared__ uint32_t tr[MD_BLOCK / kWave][32][33];
  const int32_t nd = *n_deferred;
  const int64_t total = tile_base[nd];
  const int64_t wstride = (int64_t)gridDim.x * (MD_BLOCK / kWave);
  for (int64_t t = (int64_t)blockIdx.x * (MD_BLOCK / kWave) + wave_id(); t < total; t += wstride) {
    const int o = md_owner(tile_base, nd, t);
    const MedoidMeta M = meta[o];
    int64_t r = t - tile_base[o];
    const int TN = (M.n + MD_WTN - 1) / MD_WTN;
    int ti = 0;
    while (r >= TN - md_gr_first_tj(ti)) { r -= TN - md_gr_first_tj(ti); ++ti; }
    const int tj = md_gr_first_tj(ti) + (int)r;
    const int KW = M.KW;
    const int64_t npad = (int64_t)((M.n + MD_GT - 1) / MD_GT) * MD_GT;
    const unsigned long long* rows = reinterpret_cast<const unsigned long long*>(arena + M.rowsT_off);
    // rows this lane loads: A blocks 0/1 (64-row tile), B blocks 0..NB-1 (zero past npad)
    const unsigned long long* pa = rows + ti * MD_WT + fr;
    const unsigned long long* pb = rows + (int64_t)tj * MD_WTN + fr;
    bool bok[MD_GR_NB];
#pragma unroll
    for (int b = 0; b < MD_GR_NB; ++b) bok[b] = (int64_t)tj * MD_WTN + b * 32 < npad;

    md_f32x16 acc[2][MD_GR_NB];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < MD_GR_NB; ++b)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[a][b][q] = 0;

    constexpr int NR = 2 + MD_GR_NB;  // rows per lane
    unsigned long long ring[MD_GR_PF][NR];
    auto load = [&](int w, unsigned long long* dst) __attribute__((always_inline)) {
      const int64_t wo = (int64_t)(w < KW ? w : 0) * npad;  // unconditional (clamped)
      dst[0] = pa[wo];
      dst[1] = pa[wo + 32];
#pragma unroll
      for (int b = 0; b < MD_GR_NB; ++b) dst[2 + b] = pb[wo + (bok[b] ? b * 32 : 0)];
    };
#pragma unroll
    for (int q = 0; q < MD_GR_PF; ++q) load(q, ring[q]);
    // lane half fh takes bins 32fh..32fh+31 of the word: dword g, nibble p = bin
    // 32fh + g + 4p (the same k order for A and B)
    auto frag4 = [&](uint64_t w) __attribute__((always_inline)) {
      const uint32_t c = (uint32_t)(w >> (32 * fh));
      md_i32x8 f;
      f[0] = (int)((c << 1) & 0x22222222u);
      f[1] = (int)(c & 0x22222222u);
      f[2] = (int)((c >> 1) & 0x22222222u);
      f[3] = (int)((c >> 2) & 0x22222222u);
      f[4] = f[5] = f[6] = f[7] = 0;
      return f;
    };
    for (int w0 = 0; w0 < KW; w0 += MD_GR_PF) {  // KW is a multiple of 8
#pragma unroll
      for (int q = 0; q < MD_GR_PF; ++q) {
        unsigned long long cur[NR];
#pragma unroll
        for (int k = 0; k < NR; ++k) cur[k] = ring[q][k];
        load(w0 + q + MD_GR_PF, ring[q]);
        {
          md_i32x8 fa[2], fb[MD_GR_NB];
#pragma unroll
          for (int a = 0; a < 2; ++a) fa[a] = frag4(cur[a]);
#pragma unroll
          for (int b = 0; b < MD_GR_NB; ++b) fb[b] = frag4(cur[2 + b]);
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < MD_GR_NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[a], fb[b], acc[a][b], 4, 4, 0, 0, 0, 0);
        }
      }
    }
    // C/D layout (32x32): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
    uint32_t* cmat = reinterpret_cast<uint32_t*>(arena + M.cmat_off);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < MD_GR_NB; ++b) {
        const int i0 = ti * MD_WT + a * 32, j0 = tj * MD_WTN + b * 32;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int i = i0 + (q & 3) + 8 * (q >> 2) + 4 * fh;
          const int j = j0 + fr;
          if (i < M.n && j < M.n && i <= j) {
            const uint32_t cnt = (uint32_t)acc[a][b][q];
            cmat[(int64_t)i * M.n + j] = cnt;  // row i: the lanes write consecutive j
          }
        }
        // the mirrored entries (j, i): through a wave-private 32 x 33 LDS tile so
        // that the lanes write consecutive columns of each row j (the direct
        // column store put every lane on its own cache line: 19% of the kernel)
        uint32_t(*T)[33] = tr[wave_id()];
#pragma unroll
        for (int q = 0; q < 16; ++q) T[fr][(q & 3) + 8 * (q >> 2) + 4 * fh] = (uint32_t)acc[a][b][q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int jl = 2 * rr + fh, j = j0 + jl, i = i0 + fr;
          if (i < M.n && j < M.n && i <= j) cmat[(int64_t)j * M.n + i] = T[jl][fr];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next block's writes after these reads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
  }
}

template <class F>
__device__ __forceinline__ void dual_leaf_at(const F& f, int lo, int m, int i, double& row, double& col) {
  if (m < 8) {
    double r = 0.0, cc = 0.0;
    for (int j = lo; j < lo + m; ++j) {
      const double d = f(j);
      r += j >= i ? d : 0.0;
      cc += j <= i ? d : 0.0;
    }
    row = r;
    col = cc;
    return;
  }
  double r[8], cc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double d = f(lo + k);
    r[k] = lo + k >= i ? d : 0.0;
    cc[k] = lo + k <= i ? d : 0.0;
  }
  int j = 8;
  const int lim = m - (m % 8);
  for (; j < lim; j += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int jj = lo + j + k;
      const double d = f(jj);
      r[k] += jj >= i ? d : 0.0;
      cc[k] += jj <= i ? d : 0.0;
    }
  }
  double rs = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  double cs = ((cc[0] + cc[1]) + (cc[2] + cc[3])) + ((cc[4] + cc[5]) + (cc[6] + cc[7]));
  for (; j < m; ++j) {
    const int jj = lo + j;
    const double d = f(jj);
    rs += jj >= i ? d : 0.0;
    cs += jj <= i ? d : 0.0;
  }
  row = rs;
  col = cs;
}


// dual_leaf_at over column i of the count matrix (colp = cmat + i, row stride n) with
// the loads separated from the arithmetic: 16 counts in flight per lane, then the
// distances g(j, c) in j order.  Same sums: the 8 accumulators start at +0.0 instead
// of the first term, which is exact for the distances' values (+0.0 <= d, or NaN).
template <class G>
__device__ __forceinline__ void dual_leaf_cols(const uint32_t* colp, int64_t n, const G& g, int lo, int m, int i,
                                               double& row, double& col) {
  auto acc = [&](int jj, uint32_t c, double& r, double& cc) __attribute__((always_inline)) {
    const double d = g(jj, c);
    r += jj >= i ? d : 0.0;
    cc += jj <= i ? d : 0.0;
  };
  if (m < 8) {
    double r = 0.0, cc = 0.0;
    uint32_t cv[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) cv[q] = q < m ? colp[(int64_t)(lo + q) * n] : 0u;
#pragma unroll
    for (int q = 0; q < 7; ++q)
      if (q < m) acc(lo + q, cv[q], r, cc);
    row = r;
    col = cc;
    return;
  }
  double r[8], cc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) r[k] = cc[k] = 0.0;
  const int lim = m - (m % 8);
  int j = 0;
  for (; j + 16 <= lim; j += 16) {  // uniform
    uint32_t cv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) cv[q] = colp[(int64_t)(lo + j + q) * n];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc(lo + j + q, cv[q], r[q & 7], cc[q & 7]);
  }
  if (j < lim) {  // one round of 8 left
    uint32_t cv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) cv[q] = colp[(int64_t)(lo + j + q) * n];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc(lo + j + q, cv[q], r[q], cc[q]);
    j += 8;
  }
  double rs = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  double cs = ((cc[0] + cc[1]) + (cc[2] + cc[3])) + ((cc[4] + cc[5]) + (cc[6] + cc[7]));
  {  // the sequential tail (< 8 terms)
    uint32_t cv[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) cv[q] = j + q < m ? colp[(int64_t)(lo + j + q) * n] : 0u;
#pragma unroll
    for (int q = 0; q < 7; ++q)
      if (j + q < m) acc(lo + j + q, cv[q], rs, cs);
  }
  row = rs;
  col = cs;
}
constexpr int MD_LEAF_MAX = 128;  // a numpy pairwise leaf holds at most 128 terms

// Leaf sums, grid-stride over (cluster, leaf, 256-wide chunk of i): thread i
// reads column i of the symmetric count matrix (coalesced across i).  With
// Each wave first writes the leaf's spectrum sizes and their
// reciprocals into its own LDS slice (no workgroup barrier: a wave's LDS
// operations complete in order), and the j loop reads them back as broadcasts:
// one division per spectrum and lane instead of one per (i, j).  Clusters whose
// spectra reach 65,536 peaks keep the division.
#ifndef SPX_MD_LEAF_MINW
#define SPX_MD_LEAF_MINW 5  // 86 VGPRs, no spills: 5 waves/SIMD (301 vs 318 us on configs[3] at 4)
#endif
__global__ __launch_bounds__(MD_BLOCK, SPX_MD_LEAF_MINW) void medoid_leaves_kernel(CsrView v, const MedoidMeta* meta,
                                                                 const int32_t* n_deferred, const int64_t* unit_base,
                                                                 char* arena) {
  __shared__ double rj_s[MD_BLOCK / kWave][MD_LEAF_MAX];
  __shared__ int pj_s[MD_BLOCK / kWave][MD_LEAF_MAX];
  const int32_t nd = *n_deferred;
  const int64_t total = unit_base[nd];
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {
    const int o = md_owner(unit_base, nd, u);
    const MedoidMeta M = meta[o];
    const int n = M.n;
    const int nch = (n + MD_BLOCK - 1) / MD_BLOCK;
    const int64_t r = u - unit_base[o];
    const int leaf = (int)(r / nch), ch = (int)(r % nch);
    const int i = ch * MD_BLOCK + threadIdx.x;
    const int32_t* ls = reinterpret_cast<const int32_t*>(arena + M.leaf_off);
    const int lo = ls[leaf], m = ls[leaf + 1] - lo;
    const uint32_t* cmat = reinterpret_cast<const uint32_t*>(arena + M.cmat_off);
    const int64_t* so = v.spec_off + M.s0;
    double row, col;
    if (m <= MD_LEAF_MAX) {  // uniform
      double* R = rj_s[wave_id()];
      int* Pp = pj_s[wave_id()];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // the previous unit's reads of the slice are done
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      int big = 0;
      for (int t = lane_id(); t < m; t += kWave) {
        const int64_t p = so[lo + t + 1] - so[lo + t];
        big |= p > 65536;
        Pp[t] = (int)p;
        R[t] = p > 0 ? 1.0 / (double)p : 0.0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int64_t pi64 = i < n ? so[i + 1] - so[i] : 0;
      big |= pi64 > 65536;
      if (__ballot(big) == 0ull) {  // uniform per wave: every quotient in the checked range
        if (i >= n) continue;
        const int pi = (int)pi64;
        const double ri = pi > 0 ? 1.0 / (double)pi : 0.0;
        dual_leaf_cols(cmat + i, n, [&](int j, uint32_t c) { return md_dist_r(c, pi, ri, Pp[j - lo], R[j - lo]); }, lo,
                       m, i, row, col);
      } else {
        if (i >= n) continue;
        dual_leaf_at([&](int j) { return md_dist(cmat[(int64_t)j * n + i], pi64, so[j + 1] - so[j]); }, lo, m, i,
                     row, col);
      }
    } else
    {
      if (i >= n) continue;
      const int64_t pi = so[i + 1] - so[i];
      dual_leaf_at([&](int j) { return md_dist(cmat[(int64_t)j * n + i], pi, so[j + 1] - so[j]); }, lo, m, i, row,
                   col);
    }
    const int32_t node = ls[md_max_leaves(n) + 1 + leaf];
    double* lsum = reinterpret_cast<double*>(arena + M.lsum_off);
    lsum[(int64_t)node * n + i] = row;
    lsum[(int64_t)(2 * M.L - 1 + node) * n + i] = col;
  }
}

// Totals = (tree(row leaves) + tree(column leaves)) / n (most_similar_representative.py:98-100):
// grid-stride over (cluster, 256-wide chunk of i); thread i runs the cluster's
// post-order stack machine over its leaf sums (coalesced across i).
__global__ __launch_bounds__(MD_BLOCK) void medoid_combine_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                                  const int64_t* chunk_base, char* arena,
                                                                  double* totals_out) {
  // The node ids are the post-order (plan2), so the tree is evaluated as a stack
  // machine over ids 0..2L-2: a leaf pushes its two sums (read from memory,
  // independent loads), an internal node pops right and left and pushes left +
  // right -- numpy's additions in numpy's order.  The stack lives in LDS (uniform
  // depth, one slot per thread): no dependent round trip through memory per node.
  // Depth <= log2(n / 128) + 2: 12 for the n whose n x n count matrix fits 288 GB.
  constexpr int kDepth = 16;
  __shared__ double stk[kDepth][2][MD_BLOCK];
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  const int64_t total = chunk_base[nd];
  for (int64_t u = blockIdx.x; u < total; u += gridDim.x) {
    const int o = md_owner(chunk_base, nd, u);
    const MedoidMeta M = meta[o];
    const int n = M.n;
    const int i = (int)(u - chunk_base[o]) * MD_BLOCK + tid;
    if (i >= n) continue;
    const double* row = reinterpret_cast<const double*>(arena + M.lsum_off) + i;
    const double* col = row + (int64_t)(2 * M.L - 1) * n;
    const int32_t* lnode = reinterpret_cast<const int32_t*>(arena + M.leaf_off) + (md_max_leaves(n) + 1);
    int sp = 0, kl = 0;
    for (int id = 0; id <= 2 * M.L - 2; ++id) {  // uniform
      if (kl < M.L && lnode[kl] == id) {
        stk[sp][0][tid] = row[(int64_t)id * n];
        stk[sp][1][tid] = col[(int64_t)id * n];
        ++sp;
        ++kl;
      } else {
        --sp;
        stk[sp - 1][0][tid] = stk[sp - 1][0][tid] + stk[sp][0][tid];
        stk[sp - 1][1][tid] = stk[sp - 1][1][tid] + stk[sp][1][tid];
      }
    }
    const double t = ((0.0 + stk[0][0][tid]) + (0.0 + stk[0][1][tid])) / (double)n;
    reinterpret_cast<double*>(arena + M.tot_off)[i] = t;
    if (totals_out) totals_out[M.s0 + i] = t;
  }
}

// Lowest-index argmin of the totals (most_similar_representative.py:103-110), one workgroup per cluster.
__global__ __launch_bounds__(MD_BLOCK) void medoid_argmin_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                                 const char* arena, int64_t* rep) {
  __shared__ double bt_sh[MD_BLOCK / kWave];
  __shared__ int bi_sh[MD_BLOCK / kWave];
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    const MedoidMeta M = meta[di];
    if (!M.ok) continue;
    const double* tot = reinterpret_cast<const double*>(arena + M.tot_off);
    double best_t = __longlong_as_double(0x7ff0000000000000ll);
    int best_i = 0x7fffffff;
    for (int i = tid; i < M.n; i += MD_BLOCK) {
      const double t = tot[i];
      if (t < best_t) { best_t = t; best_i = i; }
    }
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const double t2 = __shfl_xor(best_t, o, kWave);
      const int i2 = __shfl_xor(best_i, o, kWave);
      if (t2 < best_t || (t2 == best_t && i2 < best_i)) { best_t = t2; best_i = i2; }
    }
    if (lane_id() == 0) { bt_sh[wave_id()] = best_t; bi_sh[wave_id()] = best_i; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < MD_BLOCK / kWave; ++w)
        if (bt_sh[w] < best_t || (bt_sh[w] == best_t && bi_sh[w] < best_i)) { best_t = bt_sh[w]; best_i = bi_sh[w]; }
      rep[M.c] = M.s0 + best_i;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------- pair distances
// distance(spec1, spec2) of most_similar_representative.py:13-19 for arbitrary
// (global) spectrum pairs: one workgroup per pair.  |B_a ∩ B_b| = popcount of the
// AND of the two spectra's bin bitmaps in LDS (bins [0, XC_BINS): m/z < 6,553.6 at
// tol 0.1); a pair with a bin outside that range falls back to one wave's
// O(p_a * (p_a + p_b)) scan (first occurrence in a, membership in b).
constexpr int XC_BLOCK = 256;
constexpr int XC_BINS = 1 << 16;
constexpr int XC_W = XC_BINS / 32;

__global__ __launch_bounds__(XC_BLOCK) void xcorr_pairs_kernel(CsrView v, MedoidParams P,
                                                               const int64_t* __restrict__ pairs, int64_t n_pairs,
                                                               double* __restrict__ out) {
  __shared__ uint32_t bma[XC_W], bmb[XC_W];
  __shared__ int votes[2 * (XC_BLOCK / kWave)];
  __shared__ uint32_t part[XC_BLOCK / kWave];
  const int tid = threadIdx.x;
  for (int64_t p = blockIdx.x; p < n_pairs; p += gridDim.x) {
    const int64_t sa = pairs[2 * p], sb = pairs[2 * p + 1];
    const int64_t a0 = v.spec_off[sa], a1 = v.spec_off[sa + 1], b0 = v.spec_off[sb], b1 = v.spec_off[sb + 1];
    for (int w = tid; w < XC_W; w += XC_BLOCK) { bma[w] = 0u; bmb[w] = 0u; }
    __syncthreads();
    int outside = 0;
    for (int64_t k = a0 + tid; k < a1; k += XC_BLOCK) {
      const int64_t bk = md_bin(v.mz[k], P);
      if (bk < 0 || bk >= XC_BINS) outside = 1;
      else atomicOr(&bma[bk >> 5], 1u << (bk & 31));
    }
    for (int64_t k = b0 + tid; k < b1; k += XC_BLOCK) {
      const int64_t bk = md_bin(v.mz[k], P);
      if (bk < 0 || bk >= XC_BINS) outside = 1;
      else atomicOr(&bmb[bk >> 5], 1u << (bk & 31));
    }
    if (block_any<XC_BLOCK, false>(outside, votes, 0)) {
      if (wave_id() == 0) {  // the scan, one wave
        uint32_t cnt = 0;
        for (int64_t ka = a0 + lane_id(); ka < a1; ka += kWave) {
          const int64_t bk = md_bin(v.mz[ka], P);
          bool first = true;
          for (int64_t kk = a0; kk < ka && first; ++kk) first = md_bin(v.mz[kk], P) != bk;
          if (!first) continue;
          bool found = false;
          for (int64_t kb = b0; kb < b1 && !found; ++kb) found = md_bin(v.mz[kb], P) == bk;
          cnt += found;
        }
        cnt = wave_sum(cnt);
        if (lane_id() == 0) out[p] = md_dist(cnt, a1 - a0, b1 - b0);
      }
    } else {
      uint32_t cnt = 0;
      for (int w = tid; w < XC_W; w += XC_BLOCK) cnt += (uint32_t)__popc(bma[w] & bmb[w]);
      cnt = wave_sum(cnt);
      if (lane_id() == 0) part[wave_id()] = cnt;
      __syncthreads();
      if (tid == 0) {
        uint32_t c = 0;
        for (int w = 0; w < XC_BLOCK / kWave; ++w) c += part[w];
        out[p] = md_dist(c, a1 - a0, b1 - b0);
      }
    }
    __syncthreads();
  }
}

}  // namespace spx
