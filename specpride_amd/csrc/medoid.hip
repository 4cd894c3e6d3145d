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
// Small clusters (n <= 64): one 256-thread workgroup per cluster, all in LDS.
//   1  min/max bin of the cluster, union bitmap of occupied bins (ds_or_b64)
//   2  popcount prefix -> compact column id per occupied bin (K columns)
//   3  per spectrum a bit-packed row over the K columns ("densified" bin matrix)
//   4  all pairs i <= j: c_ij = sum_w popcount(row_i[w] & row_j[w])  (64 bin
//      pairs per AND+2xBCNT: the bit-packed Gram is cheaper than unpacking)
//   5  thread i: both pairwise sums over j in one pass, total_i
//   6  first argmin
// Large clusters (n > 64, or an LDS overflow) go to a deferred list and run
// through medoid_build -> medoid_tile_scan -> medoid_gram -> medoid_totals with
// state in a bump-allocated global scratch.
#include "spx_device.hpp"

namespace spx {

struct MedoidParams {
  double tol, inv_tol;
  int32_t ablate;  // profiling only (SPX_ABLATE): 16 skip rows+pairs, 32 skip totals
};

constexpr int MD_BLOCK = 256;
constexpr int MD_NMAX = 64;
constexpr int MD_WMAX = 1024;    // union-bitmap words: bin range <= 65,536 (6,553 Da at 0.1)
constexpr int MD_KWMAX = 31;     // row words (odd stride): <= 1,984 occupied bins per small cluster
constexpr int MD_PMAX = 16384;   // peaks per small cluster (spectrum-start bitmap)
constexpr int MD_TILE = 64;      // Gram tile (large path)
constexpr int MD_KCHUNK = 32;    // u64 words per LDS stage (large path)

struct MedoidSmem {
  unsigned long long bitmap[MD_WMAX];
  uint16_t wprefix[MD_WMAX];
  unsigned long long rows[MD_NMAX * MD_KWMAX];
  uint16_t cmat[MD_NMAX * MD_NMAX];
  int32_t soff[MD_NMAX + 1];
  unsigned long long sbits[MD_PMAX / 64];  // bit k set: peak k starts spectrum >= 1
  uint8_t spre[MD_PMAX / 64];              // spectra started before word w
  double totals[MD_NMAX];
  int tmp[MD_BLOCK / kWave + 1];
  long long red[2 * (MD_BLOCK / kWave)];
};

__device__ __forceinline__ int64_t md_bin(double m, const MedoidParams& P) {
  return ceil_div_exact(m, P.tol, P.inv_tol);
}

// d(i,j) exactly as 1.0 - XQuestScores::xCorrelationPrescore(...)
__device__ __forceinline__ double md_dist(uint32_t c, int64_t pi, int64_t pj) {
  const double x = (pi == 0 || pj == 0) ? 0.0 : (double)c / (double)(pi < pj ? pi : pj);
  return 1.0 - x;
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

// Block min/max of the cluster's bins -> (lo, hi); returns false if no peak.
__device__ bool cluster_bin_range(const CsrView& v, int64_t p0, int64_t p1, const MedoidParams& P,
                                  long long* red, int64_t& lo, int64_t& hi) {
  long long l = 0x7fffffffffffffffll, h = -0x7fffffffffffffffll;
  for (int64_t k = p0 + threadIdx.x; k < p1; k += MD_BLOCK) {
    const long long b = md_bin(v.mz[k], P);
    l = b < l ? b : l;
    h = b > h ? b : h;
  }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    const long long lo2 = __shfl_xor(l, o, kWave), hi2 = __shfl_xor(h, o, kWave);
    l = lo2 < l ? lo2 : l;
    h = hi2 > h ? hi2 : h;
  }
  if (lane_id() == 0) { red[wave_id()] = l; red[MD_BLOCK / kWave + wave_id()] = h; }
  __syncthreads();
  l = red[0];
  h = red[MD_BLOCK / kWave];
  for (int w = 1; w < MD_BLOCK / kWave; ++w) {
    l = red[w] < l ? red[w] : l;
    h = red[MD_BLOCK / kWave + w] > h ? red[MD_BLOCK / kWave + w] : h;
  }
  __syncthreads();
  lo = l;
  hi = h;
  return p1 > p0;
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

// --------------------------------------------------------- small clusters
__global__ __launch_bounds__(MD_BLOCK) void medoid_small_kernel(CsrView v, MedoidParams P, int64_t* rep,
                                                                double* totals_out, int32_t* deferred,
                                                                int32_t* n_deferred) {
  __shared__ MedoidSmem L;
  const int tid = threadIdx.x;
  const int64_t c = blockIdx.x;
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  const int n = (int)(s1 - s0);
  if (s1 - s0 > MD_NMAX) {
    if (tid == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
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
  if (p1 - p0 > MD_PMAX) {
    if (tid == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    return;
  }
  const int nsw = (int)((p1 - p0 + 63) / 64);
  for (int w = tid; w < nsw; w += MD_BLOCK) L.sbits[w] = 0ull;
  // bin range from each spectrum's first and last peak (m/z-sorted spectra);
  // pass 1 verifies every bin falls inside and defers the cluster otherwise
  long long blo = 0x7fffffffffffffffll, bhi = -0x7fffffffffffffffll;
  if (tid <= n) L.soff[tid] = (int32_t)(v.spec_off[s0 + tid] - p0);
  if (tid < n) {
    const int64_t a = v.spec_off[s0 + tid], e = v.spec_off[s0 + tid + 1];
    if (e > a) {
      blo = md_bin(v.mz[a], P);
      bhi = md_bin(v.mz[e - 1], P);
    }
  }
  if (tid < kWave) {  // n <= 64: wave 0 holds every spectrum
    const bool empty_spec = tid < n && v.spec_off[s0 + tid + 1] == v.spec_off[s0 + tid];
    const unsigned long long any_empty = __ballot(empty_spec);
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const long long l2 = __shfl_xor(blo, o, kWave), h2 = __shfl_xor(bhi, o, kWave);
      blo = l2 < blo ? l2 : blo;
      bhi = h2 > bhi ? h2 : bhi;
    }
    if (tid == 0) { L.red[0] = blo; L.red[1] = bhi; L.red[2] = any_empty != 0ull; }
  }
  __syncthreads();
  blo = L.red[0];
  bhi = L.red[1];
  const bool has_empty = L.red[2] != 0;
  const bool any = p1 > p0;
  const int64_t nw = any ? (bhi - blo) / 64 + 1 : 0;
  if (nw > MD_WMAX || (any && bhi < blo)) {
    if (tid == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    return;
  }
  // spectrum of a peak in O(1): a start bit at every spectrum boundary and a
  // per-word count of the boundaries before it
  for (int j = 1 + tid; j < n; j += MD_BLOCK) {
    const int r = L.soff[j];
    if (r < p1 - p0) atomicOr(&L.sbits[r >> 6], 1ull << (r & 63));
  }
  // 1: union bitmap (8 loads in flight per thread)
  for (int w = tid; w < nw; w += MD_BLOCK) L.bitmap[w] = 0ull;
  __syncthreads();
  if (tid < kWave) {  // prefix of start bits (<= 256 words, one wave)
    int carry = 0;
    for (int w0 = 0; w0 < nsw; w0 += kWave) {
      const int w = w0 + tid;
      const int c1 = w < nsw ? __popcll(L.sbits[w]) : 0;
      const int inc = wave_inclusive_sum(c1);
      if (w < nsw) L.spre[w] = (uint8_t)(carry + inc - c1);
      carry += __shfl(inc, kWave - 1, kWave);
    }
  }
  int outside = 0;
  for (int64_t k0 = p0 + tid; k0 < p1; k0 += 8 * MD_BLOCK) {
    double m[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + (int64_t)u * MD_BLOCK;
      m[u] = k < p1 ? v.mz[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (k0 + (int64_t)u * MD_BLOCK >= p1) continue;
      const int64_t b = md_bin(m[u], P) - blo;
      if (b < 0 || b >= nw * 64) { outside = 1; continue; }
      atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
    }
  }
  if (__syncthreads_or(outside)) {  // an unsorted spectrum: general path
    if (tid == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    return;
  }
  // 2: compact columns
  const int K = bitmap_prefix<MD_BLOCK>(L.bitmap, L.wprefix, (int)nw, L.tmp);
  // row stride KW is odd: lanes reading rows j, j+1, ... at one word hit
  // different LDS banks (an even stride of u64s would fold them together)
  const int KW = ((K + 63) / 64) | 1;
  if (KW > MD_KWMAX) {
    if (tid == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    return;
  }
  // 3: bit-packed rows
  for (int w = tid; w < n * KW; w += MD_BLOCK) L.rows[w] = 0ull;
  __syncthreads();
  if (P.ablate & 16) { if (tid == 0) rep[c] = s0; return; }
  for (int64_t k0 = p0 + tid; k0 < p1; k0 += 8 * MD_BLOCK) {
    double m[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + (int64_t)u * MD_BLOCK;
      m[u] = k < p1 ? v.mz[k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + (int64_t)u * MD_BLOCK;
      if (k >= p1) continue;
      const int col = bitmap_rank(L.bitmap, L.wprefix, md_bin(m[u], P) - blo);
      const int r = (int)(k - p0);
      // empty spectra share a start bit: then fall back to the binary search
      const int sp = has_empty ? spectrum_of(L.soff, n, r)
                               : (int)L.spre[r >> 6] + __popcll(L.sbits[r >> 6] & ((2ull << (r & 63)) - 1ull));
      atomicOr(&L.rows[sp * KW + (col >> 6)], 1ull << (col & 63));
    }
  }
  __syncthreads();
  // 4: shared-bin counts for every pair i <= j: pair p of the row-major upper
  // triangle, row i starting at i*n - i*(i-1)/2 (recovered by a float sqrt +
  // integer fix-up: no idle half, no integer division per pair)
  if (P.ablate & 64) { if (tid == 0) rep[c] = s0; return; }
  const int NP = n * (n + 1) / 2;
  auto row_start = [&](int i) { return i * n - (i * (i - 1)) / 2; };
  for (int p = tid; p < NP; p += MD_BLOCK) {
    const float b2 = 2.0f * n + 1.0f;
    int i = (int)((b2 - sqrtf(b2 * b2 - 8.0f * (float)p)) * 0.5f);
    i = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    while (i > 0 && row_start(i) > p) --i;
    while (i + 1 < n && row_start(i + 1) <= p) ++i;
    const int j = i + (p - row_start(i));
    uint32_t cnt = 0;
    for (int w = 0; w < KW; ++w) cnt += (uint32_t)__popcll(L.rows[i * KW + w] & L.rows[j * KW + w]);
    L.cmat[i * n + j] = (uint16_t)cnt;
    L.cmat[j * n + i] = (uint16_t)cnt;
  }
  __syncthreads();
  // 5: totals (most_similar_representative.py:98-100)
  if (P.ablate & 32) { if (tid == 0) rep[c] = s0; return; }
  if (tid < n) {
    const int i = tid;
    const int64_t pi = L.soff[i + 1] - L.soff[i];
    double row, col;
    dual_pw_leaf([&](int j) { return md_dist(L.cmat[i * n + j], pi, L.soff[j + 1] - L.soff[j]); }, n, i, row, col);
    const double t = (row + col) / (double)n;
    L.totals[i] = t;
    if (totals_out) totals_out[s0 + i] = t;
  }
  __syncthreads();
  // 6: first index of the minimum (:103-110)
  if (tid == 0) {
    int best = 0;
    double bt = L.totals[0];
    for (int i = 1; i < n; ++i)
      if (L.totals[i] < bt) { bt = L.totals[i]; best = i; }
    rep[c] = s0 + best;
  }
}

// ------------------------------------------------------------ large path
struct MedoidMeta {
  int64_t c, s0, rows_off, cmat_off;  // byte offsets into scratch
  int32_t n, KW, tiles, ok;
};

// One workgroup per deferred cluster.  Compact column ids come from a
// two-level occupancy bitmap so any bin range works: level 1 (LDS) has one bit
// per block of 64 bins, level 2 (arena) one u64 word per OCCUPIED block; the
// column of bin b is prefix2[block slot] + popcount(word & below(b)).  Rows and
// the count matrix are bump-allocated from the same arena.
constexpr int MD_L1WORDS = 1024;  // level-1 bits: 65,536 blocks = 4.2M bins

__global__ __launch_bounds__(MD_BLOCK) void medoid_build_kernel(CsrView v, MedoidParams P, const int32_t* deferred,
                                                                const int32_t* n_deferred, MedoidMeta* meta,
                                                                char* scratch, unsigned long long* bump,
                                                                int64_t scratch_bytes, int64_t* rep) {
  __shared__ unsigned long long l1[MD_L1WORDS];
  __shared__ uint32_t l1pre[MD_L1WORDS];
  __shared__ int tmp[MD_BLOCK / kWave + 1];
  __shared__ long long red[2 * (MD_BLOCK / kWave)];
  __shared__ unsigned long long base_sh;
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    const int64_t c = deferred[di];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int n = (int)(s1 - s0);
    const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
    int64_t blo, bhi;
    const bool any = cluster_bin_range(v, p0, p1, P, red, blo, bhi);
    const int64_t nblk = any ? ((bhi - blo) >> 6) + 1 : 0;
    const int64_t nw1 = (nblk + 63) / 64;
    MedoidMeta M{c, s0, 0, 0, n, 0, 0, 0};
    if (nw1 > MD_L1WORDS) {  // > 4.2M bins: reported, not approximated
      if (tid == 0) { meta[di] = M; rep[c] = -2; }
      continue;
    }
    // level 1
    for (int w = tid; w < nw1; w += MD_BLOCK) l1[w] = 0ull;
    __syncthreads();
    for (int64_t k = p0 + tid; k < p1; k += MD_BLOCK) {
      const int64_t blk = (md_bin(v.mz[k], P) - blo) >> 6;
      atomicOr(&l1[blk >> 6], 1ull << (blk & 63));
    }
    __syncthreads();
    const int B1 = bitmap_prefix<MD_BLOCK>(l1, l1pre, (int)nw1, tmp);
    // arena: level-2 words + their prefix, then rows and counts (sized after K)
    const int64_t l2_bytes = (((int64_t)B1 * 12) + 255) & ~int64_t(255);
    if (tid == 0) base_sh = atomicAdd(bump, (unsigned long long)l2_bytes);
    __syncthreads();
    const int64_t l2_base = (int64_t)base_sh;
    if (l2_base + l2_bytes > scratch_bytes) {
      if (tid == 0) { meta[di] = M; rep[c] = -3; }
      __syncthreads();
      continue;
    }
    unsigned long long* l2 = reinterpret_cast<unsigned long long*>(scratch + l2_base);
    uint32_t* l2pre = reinterpret_cast<uint32_t*>(scratch + l2_base + (int64_t)B1 * 8);
    for (int w = tid; w < B1; w += MD_BLOCK) l2[w] = 0ull;
    __syncthreads();
    auto block_slot = [&](int64_t rel) { return bitmap_rank(l1, l1pre, rel >> 6); };
    for (int64_t k = p0 + tid; k < p1; k += MD_BLOCK) {
      const int64_t rel = md_bin(v.mz[k], P) - blo;
      atomicOr(&l2[block_slot(rel)], 1ull << (rel & 63));
    }
    __syncthreads();
    const int K = bitmap_prefix<MD_BLOCK>(l2, l2pre, B1, tmp);
    auto column = [&](int64_t rel) {
      const int bs = block_slot(rel);
      return (int)l2pre[bs] + __popcll(l2[bs] & ((1ull << (rel & 63)) - 1ull));
    };
    const int KW = (K + 63) / 64 > 0 ? (K + 63) / 64 : 1;
    const int T = (n + MD_TILE - 1) / MD_TILE;
    // rows padded to whole tiles so the Gram kernel never reads past them
    const int64_t rows_bytes = (int64_t)T * MD_TILE * KW * 8;
    const int64_t cmat_bytes = (((int64_t)n * n * 4) + 255) & ~int64_t(255);
    __syncthreads();
    if (tid == 0) base_sh = atomicAdd(bump, (unsigned long long)(rows_bytes + cmat_bytes));
    __syncthreads();
    const int64_t base = (int64_t)base_sh;
    if (base + rows_bytes + cmat_bytes > scratch_bytes) {
      if (tid == 0) { meta[di] = M; rep[c] = -3; }
      __syncthreads();
      continue;
    }
    unsigned long long* rows = reinterpret_cast<unsigned long long*>(scratch + base);
    for (int64_t w = tid; w < (int64_t)T * MD_TILE * KW; w += MD_BLOCK) rows[w] = 0ull;
    __syncthreads();
    for (int64_t s = s0; s < s1; ++s) {
      const int64_t a = v.spec_off[s], e = v.spec_off[s + 1];
      unsigned long long* row = rows + (s - s0) * KW;
      for (int64_t k = a + tid; k < e; k += MD_BLOCK) {
        const int col = column(md_bin(v.mz[k], P) - blo);
        atomicOr(&row[col >> 6], 1ull << (col & 63));
      }
    }
    if (tid == 0) {
      M.rows_off = base;
      M.cmat_off = base + rows_bytes;
      M.KW = KW;
      M.tiles = T * (T + 1) / 2;
      M.ok = 1;
      meta[di] = M;
    }
    __syncthreads();
  }
}

// Exclusive scan of Gram tiles over the deferred clusters (one workgroup).
__global__ __launch_bounds__(MD_BLOCK) void medoid_tile_scan_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                                    int64_t* tile_base) {
  __shared__ int64_t tmp[MD_BLOCK / kWave + 1];
  const int32_t nd = *n_deferred;
  int64_t carry = 0;
  for (int32_t i0 = 0; i0 < nd; i0 += MD_BLOCK) {
    const int32_t i = i0 + threadIdx.x;
    const int64_t t = (i < nd && meta[i].ok) ? meta[i].tiles : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<MD_BLOCK>(t, tmp, tot);
    if (i < nd) tile_base[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) tile_base[nd] = carry;
}

// 64x64 tile of c_ij = popcount(row_i & row_j) per workgroup, grid-stride over
// all tiles of all deferred clusters.  Thread (ty, tx) owns rows 4ty..4ty+3 x
// columns 4tx..4tx+3; row words staged through LDS in 32-word chunks (rows
// padded to 33 words: conflict-free column reads).
__global__ __launch_bounds__(MD_BLOCK) void medoid_gram_kernel(const MedoidMeta* meta, const int32_t* n_deferred,
                                                               const int64_t* tile_base, char* scratch) {
  __shared__ unsigned long long As[MD_TILE][MD_KCHUNK + 1];
  __shared__ unsigned long long Bs[MD_TILE][MD_KCHUNK + 1];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int32_t nd = *n_deferred;
  const int64_t total = tile_base[nd];
  for (int64_t t = blockIdx.x; t < total; t += gridDim.x) {
    int lo = 0, hi = nd;  // tile_base[lo] <= t < tile_base[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (tile_base[mid] <= t) lo = mid; else hi = mid;
    }
    while (lo + 1 < nd && tile_base[lo + 1] <= t) ++lo;  // skip empty entries
    const MedoidMeta M = meta[lo];
    int64_t r = t - tile_base[lo];
    const int T = (M.n + MD_TILE - 1) / MD_TILE;
    int ti = 0;
    while (r >= T - ti) { r -= T - ti; ++ti; }
    const int tj = ti + (int)r;
    const unsigned long long* rows = reinterpret_cast<const unsigned long long*>(scratch + M.rows_off);
    uint32_t* cmat = reinterpret_cast<uint32_t*>(scratch + M.cmat_off);
    uint32_t acc[4][4] = {};
    for (int w0 = 0; w0 < M.KW; w0 += MD_KCHUNK) {
      const int wn = M.KW - w0 < MD_KCHUNK ? M.KW - w0 : MD_KCHUNK;
      for (int e = tid; e < MD_TILE * MD_KCHUNK; e += MD_BLOCK) {
        const int rr = e / MD_KCHUNK, ww = e % MD_KCHUNK;
        const bool in = ww < wn;
        As[rr][ww] = in ? rows[((int64_t)ti * MD_TILE + rr) * M.KW + w0 + ww] : 0ull;
        Bs[rr][ww] = in ? rows[((int64_t)tj * MD_TILE + rr) * M.KW + w0 + ww] : 0ull;
      }
      __syncthreads();
      for (int w = 0; w < wn; ++w) {
        unsigned long long a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { a[q] = As[4 * ty + q][w]; b[q] = Bs[4 * tx + q][w]; }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[q][u] += (uint32_t)__popcll(a[q] & b[u]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = ti * MD_TILE + 4 * ty + q, j = tj * MD_TILE + 4 * tx + u;
        if (i < M.n && j < M.n) {
          cmat[(int64_t)i * M.n + j] = acc[q][u];
          cmat[(int64_t)j * M.n + i] = acc[q][u];
        }
      }
  }
}

// Totals and argmin, one workgroup per deferred cluster.  Thread i walks
// column i of the symmetric count matrix (coalesced across threads) and
// evaluates numpy's pairwise tree for row i (j >= i) and column i (j <= i).
__global__ __launch_bounds__(MD_BLOCK) void medoid_totals_kernel(CsrView v, const MedoidMeta* meta,
                                                                 const int32_t* n_deferred, const char* scratch,
                                                                 int64_t* rep, double* totals_out) {
  __shared__ double bt_sh[MD_BLOCK / kWave];
  __shared__ int bi_sh[MD_BLOCK / kWave];
  const int tid = threadIdx.x;
  const int32_t nd = *n_deferred;
  for (int32_t di = blockIdx.x; di < nd; di += gridDim.x) {
    const MedoidMeta M = meta[di];
    if (!M.ok) continue;
    const int n = M.n;
    const uint32_t* cmat = reinterpret_cast<const uint32_t*>(scratch + M.cmat_off);
    const int64_t* so = v.spec_off + M.s0;
    double best_t = __longlong_as_double(0x7ff0000000000000ll);
    int best_i = 0x7fffffff;
    for (int i = tid; i < n; i += MD_BLOCK) {
      const int64_t pi = so[i + 1] - so[i];
      auto drow = [&](int64_t j) {
        return j >= i ? md_dist(cmat[j * n + i], pi, so[j + 1] - so[j]) : 0.0;
      };
      auto dcol = [&](int64_t j) {
        return j <= i ? md_dist(cmat[j * n + i], pi, so[j + 1] - so[j]) : 0.0;
      };
      const double t = (pw_sum(drow, n) + pw_sum(dcol, n)) / (double)n;
      if (totals_out) totals_out[M.s0 + i] = t;
      if (t < best_t) { best_t = t; best_i = i; }
    }
    // block argmin, lowest index on ties
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
// (global) spectrum pairs: one wave per pair.  |B_a ∩ B_b| counts the distinct
// bins of a (first occurrence in a) that occur in b.  O(p_a * (p_a + p_b)) per
// pair: this is the per-call API, not the batched medoid path.
__global__ __launch_bounds__(256) void xcorr_pairs_kernel(CsrView v, MedoidParams P, const int64_t* __restrict__ pairs,
                                                          int64_t n_pairs, double* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * 4 + wave_id();
  if (p >= n_pairs) return;
  const int64_t sa = pairs[2 * p], sb = pairs[2 * p + 1];
  const int64_t a0 = v.spec_off[sa], a1 = v.spec_off[sa + 1], b0 = v.spec_off[sb], b1 = v.spec_off[sb + 1];
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

}  // namespace spx
