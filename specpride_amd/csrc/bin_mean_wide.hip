// Bin-mean for the clusters the register kernel does not take: up to 128
// spectra of ANY length and up to BW_DCAP distinct bins (reference:
// src/binning.py:170-231, combine_bin_mean).  One 256-thread
// workgroup per cluster, grid-stride over the register kernel's leftovers:
//
//   set-up  spectrum offsets and precursors into LDS, the mixed-charge vote
//           (binning.py:205-206), the occupancy bitmap cleared
//   1  one flat coalesced pass over the cluster's m/z (16 loads in flight per
//      thread, any order): occupied bins into the LDS bitmap
//   2  popcount prefix -> every occupied bin's slot, in ascending bin order
//   3  the ordered fold over WORK ITEMS = (spectrum, 252-position chunk) in file
//      order, a register ring BW_PF items deep: wave w's lanes 0..62 own positions
//      63w..63w+62 of the chunk and lane 63 reads position 63w+63 only to hand lane
//      62 its neighbour key (for the last wave that is the NEXT chunk's first
//      peak), so "last peak of its bin in the spectrum" (numpy fancy-index +=,
//      binning.py:197-199) is one DPP compare; the slot is the bin's rank; the
//      update is f32(f64(acc) + v) (binning.py:198-199).  Software-pipelined by
//      one item (item i's slots are computed while item i-1's accumulator reads
//      are in flight).  Chunks of one spectrum touch distinct slots, so the one
//      LDS-only barrier per step is taken only where a new spectrum begins -- the
//      reference's spectrum order per bin is all the fold has to keep
//   4  quorum int(0.25 n) + 1 and the striped ordered emit (emit_striped), the
//      precursor np.mean (numpy's pairwise tree)
//
// HBM traffic: the m/z twice (phase 3 re-reads what phase 1 pulled toward the
// caches), the intensities once.  A key inversion or NaN inside a spectrum
// (unsorted input) sends the cluster on to the split path / global kernel, as
// does a cluster with more than BW_DCAP distinct bins or BM_NMAX spectra.
#pragma once
#include "bin_mean.hip"

namespace spx {

#ifndef SPX_BW_DCAP
#define SPX_BW_DCAP 4096
#endif
#ifndef SPX_BW_PF
#define SPX_BW_PF 8
#endif
#ifndef SPX_BW_MINW
#define SPX_BW_MINW 2
#endif
constexpr int BW_DCAP = SPX_BW_DCAP;  // distinct occupied bins per cluster (10 B of LDS each)
constexpr int BW_PF = SPX_BW_PF;      // items in flight per lane
constexpr int BW_CHUNK = 4 * (kWave - 1);  // positions per item (252)
static_assert(BW_DCAP % BM_BLOCK == 0 && BW_DCAP / BM_BLOCK <= 32, "emit_striped keeps one bit per stripe");

struct BinWideSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  float acc_i[BW_DCAP];
  float acc_m[BW_DCAP];
  uint16_t cnt[BW_DCAP];  // <= BM_NMAX contributions per slot
  double prec[BM_NMAX];
  int32_t soff[BM_NMAX + 1];
  int wcnt[(BW_DCAP / BM_BLOCK) * (BM_BLOCK / kWave)];
  int votes[2 * (BM_BLOCK / kWave)];
  int tmp[BM_BLOCK / kWave + 1];
};

// Uniform cursor over a cluster's work items: spectrum j, chunk start c0.
// Empty spectra have no item.  Past the last item j == n.
struct ItemCursor {
  int j, c0;
};

__device__ __forceinline__ int bw_len(const BinWideSmem& L, int j) { return L.soff[j + 1] - L.soff[j]; }

__device__ __forceinline__ void bw_skip_empty(const BinWideSmem& L, int n, ItemCursor& q) {
  while (q.j < n && bw_len(L, q.j) == 0) ++q.j;
}

// the next item; past the last one the cursor stays at j == n (null items)
__device__ __forceinline__ void bw_next(const BinWideSmem& L, int n, ItemCursor& q) {
  if (q.j >= n) return;
  q.c0 += BW_CHUNK;
  if (q.c0 >= bw_len(L, q.j)) {
    ++q.j;
    q.c0 = 0;
    bw_skip_empty(L, n, q);
  }
}

__device__ __forceinline__ int32_t bin_mean_wide_body(const CsrView& v, const BinMeanParams& P, BinWideSmem& L,
                                                      int64_t c, const PeaksOut& out, double* prec_out,
                                                      int32_t* charge_out) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n64 = s1 - s0;
  if (n64 == 0) {
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kEmpty;
  }
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1];
  if (n64 > BM_NMAX || P.n_words > BM_WMAX || p1 - p0 >= (int64_t(1) << 28)) return kDeferred;
  const int n = (int)n64;
  const int np = (int)(p1 - p0);
  for (int j = tid; j <= n; j += BM_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
  for (int j = tid; j < n; j += BM_BLOCK) L.prec[j] = v.prec_mz[s0 + j];
  const int32_t z0 = v.charge[s0];
  int mixed = 0;
  for (int j = 1 + tid; j < n; j += BM_BLOCK) mixed |= v.charge[s0 + j] != z0;
  for (int w = tid; w < P.n_words; w += BM_BLOCK) L.bitmap[w] = 0ull;
  if (block_any<BM_BLOCK, true>(mixed, L.votes, 0)) {  // binning.py:205-206: nothing emitted
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kMixedCharge;
  }

  // 1: occupancy from one flat pass (every in-range bin has a last peak)
  const char* __restrict__ mzb = reinterpret_cast<const char*>(v.mz + p0);
  constexpr int U1 = 16;
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
        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
      }
    }
  }
  lds_barrier();

  // 2: slots in bin order
  const int D = bitmap_prefix<BM_BLOCK, uint16_t, true>(L.bitmap, L.wprefix, P.n_words, L.tmp);
  if (D > BW_DCAP) return kDeferred;
  for (int d = tid; d < D; d += BM_BLOCK) {
    L.cnt[d] = 0;
    L.acc_i[d] = 0.0f;
    L.acc_m[d] = 0.0f;
  }
  lds_barrier();

  // 3: the ordered fold over the work items
  const int fpos = wid * (kWave - 1) + lane;  // this lane's position in every chunk
  const bool owner = lane < kWave - 1;
  const __amdgpu_buffer_rsrc_t rmz = bf_rsrc(v.mz + p0, np);
  const __amdgpu_buffer_rsrc_t rit = bf_rsrc(v.inten + p0, np);
  struct Pk {
    double m, it;
  };
  // item (j, c0) -> this lane's peak; j == n (past the end) reads out of range: 0
  auto fetch = [&](const ItemCursor& q) __attribute__((always_inline)) {
    const int jj = q.j < n ? q.j : n - 1;
    const int a = L.soff[jj], e = L.soff[jj + 1];
    const int k = a + q.c0 + fpos;
    const int bo = (q.j < n && k < e) ? k * 8 : np * 8;
    return Pk{bf_load(rmz, bo, 0), bf_load(rit, bo, 0)};
  };
  ItemCursor fq{0, 0}, cq{0, 0};  // fetch and consume cursors (uniform)
  bw_skip_empty(L, n, fq);
  bw_skip_empty(L, n, cq);
  Pk ring[BW_PF];
#pragma unroll
  for (int q = 0; q < BW_PF; ++q) {
    ring[q] = fetch(fq);
    bw_next(L, n, fq);
  }
  int bad = 0, pslot = -1, pj = -1;
  double pm = 0.0, pit = 0.0;
  // whole groups of BW_PF steps: past the last item the steps are null items
  // (nothing active, one extra barrier), so no step is guarded and no ring
  // register is ever a merge of a fresh load and an old value
  while (cq.j < n) {  // uniform
#pragma unroll
    for (int q = 0; q < BW_PF; ++q) {
      // item i-1's accumulator reads first (every lane; non-owners read slot 0)
      const int ps = pslot >= 0 ? pslot : 0;
      const float e_ai = L.acc_i[ps], e_am = L.acc_m[ps];
      const uint16_t e_cn = L.cnt[ps];
      const Pk pk = ring[q];
      ring[q] = fetch(fq);
      bw_next(L, n, fq);
      const int len = cq.j < n ? bw_len(L, cq.j) : 0;
      const int pos = cq.c0 + fpos;
      const bool act = pos < len;
      const bool inr = act && in_range(pk.m, P);
      int32_t key = (act && pk.m < P.minimum) ? -1 : 0x7fffffff;
      int slot = -1;
      if (inr) {
        key = bin_small(pk.m, P);
        slot = bitmap_rank(L.bitmap, L.wprefix, (int64_t)key);
      }
      const int32_t kn = wave_next(key, 0x7fffffff);
      bad |= (int)(owner && act && ((pk.m != pk.m) || key > kn));
      const bool last = kn != key;
      if (pslot >= 0) {  // finish item i-1
        L.cnt[pslot] = (uint16_t)(e_cn + 1u);
        L.acc_i[pslot] = (float)((double)e_ai + pit);
        L.acc_m[pslot] = (float)((double)e_am + pm);
      }
      // a new spectrum may touch item i-1's slots: its writes land first
      if (cq.j != pj) lds_barrier();
      pj = cq.j;
      pslot = (owner && inr && last) ? slot : -1;
      pm = pk.m;
      pit = pk.it;
      bw_next(L, n, cq);
    }
  }
  if (pslot >= 0) {
    L.cnt[pslot] = (uint16_t)(L.cnt[pslot] + 1u);
    L.acc_i[pslot] = (float)((double)L.acc_i[pslot] + pit);
    L.acc_m[pslot] = (float)((double)L.acc_m[pslot] + pm);
  }
  if (block_any<BM_BLOCK, true>(bad, L.votes, 1)) return kDeferred;  // unsorted / NaN: the general paths

  // 4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int total = emit_striped(L.cnt, [&](int d) { return L.acc_i[d]; }, [&](int d) { return L.acc_m[d]; },
                                 L.wcnt, D, quorum, out.mz + p0, out.inten + p0);
  if (tid == 0) {
    out.count[c] = total;
    charge_out[c] = z0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return L.prec[j]; }, n) / (double)n;  // np.mean (binning.py:224)
  }
  return kOk;
}

// The register kernel's leftovers, grid-stride over the list.
__global__ __launch_bounds__(BM_BLOCK, SPX_BW_MINW) void bin_mean_wide_kernel(CsrView v, BinMeanParams P,
                                                                              PeaksOut out, double* prec_out,
                                                                              int32_t* charge_out, int32_t* status,
                                                                              const int32_t* list,
                                                                              const int32_t* n_list,
                                                                              int32_t* deferred,
                                                                              int32_t* n_deferred) {
  __shared__ BinWideSmem L;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = list[i];
    const int32_t st = bin_mean_wide_body(v, P, L, c, out, prec_out, charge_out);
    if (threadIdx.x == 0) {
      status[c] = st;
      if (st == kDeferred) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
    }
    lds_barrier();  // the LDS is reused by the next cluster
  }
}

}  // namespace spx
