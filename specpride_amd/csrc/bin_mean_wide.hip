// Bin-mean for the clusters the register kernel does not take: up to 128
// spectra of ANY length and up to BW_DCAP distinct bins (reference:
// src/binning.py:170-231, combine_bin_mean).  One 512-thread
// workgroup per cluster, grid-stride over the register kernel's leftovers:
//
//   set-up  spectrum offsets and precursors into LDS, the mixed-charge vote
//           (binning.py:205-206), the occupancy bitmap cleared
//   1  one flat coalesced pass over the cluster's m/z (16 loads in flight per
//      thread, any order): occupied bins into the LDS bitmap
//   2  popcount prefix -> every occupied bin's slot, in ascending bin order
//   3  the ordered fold over WORK ITEMS = (spectrum, 504-position chunk) in file
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
// (unsorted input) sends the cluster to the global kernel; one with more than
// BW_DCAP distinct bins, BM_NMAX spectra or BW_IMAX work items to the segmented
// fold (bin_mean_seg.hip).
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
#define SPX_BW_MINW 4
#endif
#ifndef SPX_BW_BLOCK
#define SPX_BW_BLOCK 512
#endif
constexpr int32_t kUnsortedW = -2;  // (internal) a key inversion or NaN: straight to the global kernel
constexpr int BW_DCAP = SPX_BW_DCAP;  // distinct occupied bins per cluster (10 B of LDS each)
constexpr int BW_PF = SPX_BW_PF;      // items in flight per lane
constexpr int BW_BLOCK = SPX_BW_BLOCK;  // threads per workgroup (8 waves: 2 workgroups per CU = 4 waves per SIMD)
constexpr int BW_CHUNK = (BW_BLOCK / kWave) * (kWave - 1);  // positions per item (504)
static_assert(BW_DCAP % BW_BLOCK == 0 && BW_DCAP / BW_BLOCK <= 32, "emit_striped keeps one bit per stripe");
static_assert(BM_NMAX <= BW_BLOCK, "one thread per spectrum lays out the work items");

#ifndef SPX_BW_IMAX
#define SPX_BW_IMAX 1024
#endif
constexpr int BW_IMAX = SPX_BW_IMAX;  // work items per cluster (the table in LDS)

struct BinWideSmem {
  unsigned long long bitmap[BM_WMAX];
  uint16_t wprefix[BM_WMAX];
  float2 acc[BW_DCAP];    // (intensity, m/z) sums: one b64 read + one b64 write per contribution
  uint16_t cnt[BW_DCAP];  // <= BM_NMAX contributions per slot
  // work item i: x = cluster-relative index of its first position, y = positions
  // left in its spectrum from there, bit 31 of y: the item starts a spectrum;
  // entries past the last item are null ({0, 0}: nothing active)
  int2 item[BW_IMAX + BW_PF];
  double prec[BM_NMAX];
  int32_t soff[BM_NMAX + 1];
  int wcnt[(BW_DCAP / BW_BLOCK) * (BW_BLOCK / kWave)];
  int votes[2 * (BW_BLOCK / kWave)];
  int tmp[BW_BLOCK / kWave + 1];
};

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
  if (n64 > BM_NMAX || P.n_words > BM_WMAX || p1 - p0 >= (int64_t(1) << 28)) return kDeferred;  // bin_mean_past_wide
  const int n = (int)n64;
  const int np = (int)(p1 - p0);
  for (int j = tid; j <= n; j += BW_BLOCK) L.soff[j] = (int32_t)(v.spec_off[s0 + j] - p0);
  for (int j = tid; j < n; j += BW_BLOCK) L.prec[j] = v.prec_mz[s0 + j];
  const int32_t z0 = v.charge[s0];
  int mixed = 0;
  for (int j = 1 + tid; j < n; j += BW_BLOCK) mixed |= v.charge[s0 + j] != z0;
  for (int w = tid; w < P.n_words; w += BW_BLOCK) L.bitmap[w] = 0ull;
  if (block_any<BW_BLOCK, true>(mixed, L.votes, 0)) {  // binning.py:205-206: nothing emitted
    if (tid == 0) { out.count[c] = 0; prec_out[c] = __longlong_as_double(0x7ff8000000000000ll); charge_out[c] = 0; }
    return kMixedCharge;
  }

  // 1: occupancy from one flat pass (every in-range bin has a last peak)
  const char* __restrict__ mzb = reinterpret_cast<const char*>(v.mz + p0);
  constexpr int U1 = 16;
  for (int r0 = tid; r0 < np; r0 += U1 * BW_BLOCK) {
    double m[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int r = r0 + u * BW_BLOCK;
      m[u] = *reinterpret_cast<const double*>(mzb + (uint32_t)(r < np ? r : 0) * 8u);
    }
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      if (r0 + u * BW_BLOCK < np && in_range(m[u], P)) {
        const int32_t b = bin_small(m[u], P);
        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
      }
    }
  }
  lds_barrier();

  // 2: slots in bin order
  const int D = bitmap_prefix<BW_BLOCK, uint16_t, true>(L.bitmap, L.wprefix, P.n_words, L.tmp);
  if (D > BW_DCAP) return kDeferred;
  for (int d = tid; d < D; d += BW_BLOCK) {
    L.cnt[d] = 0;
    L.acc[d] = make_float2(0.0f, 0.0f);
  }
  // the work items: ceil(len / BW_CHUNK) per spectrum, in file order (thread j < n <= 128
  // lays out spectrum j's; empty spectra have none)
  int ni;
  {
    const int len = tid < n ? L.soff[tid + 1] - L.soff[tid] : 0;
    const int mine = (len + BW_CHUNK - 1) / BW_CHUNK;
    const int base = block_exclusive_scan<BW_BLOCK, int, true>(mine, L.tmp, ni);
    if (ni <= BW_IMAX) {
      for (int k = 0; k < mine; ++k)
        L.item[base + k] = make_int2(L.soff[tid] + k * BW_CHUNK, (len - k * BW_CHUNK) | (k == 0 ? (int)0x80000000 : 0));
      if (tid < BW_PF) L.item[ni + tid] = make_int2(0, 0);
    }
  }
  if (ni > BW_IMAX) return kDeferred;
  lds_barrier();

  // 3: the ordered fold over the work items
  const int fpos = wid * (kWave - 1) + lane;  // this lane's position in every chunk
  const bool owner = lane < kWave - 1;
  const __amdgpu_buffer_rsrc_t rmz = bf_rsrc(v.mz + p0, np);
  const __amdgpu_buffer_rsrc_t rit = bf_rsrc(v.inten + p0, np);
  struct Pk {
    double m, it;
    int rem;  // positions left in the spectrum (bit 31: a new spectrum)
  };
  // item i -> this lane's peak (past the spectrum or a null item: out of the
  // descriptor's range, the load returns 0)
  auto fetch = [&](int i) __attribute__((always_inline)) {
    const int2 d = L.item[i];
    const int rem = d.y & 0x7fffffff;
    const int bo = fpos < rem ? (d.x + fpos) * 8 : np * 8;
    return Pk{bf_load(rmz, bo, 0), bf_load(rit, bo, 0), d.y};
  };
  Pk ring[BW_PF];
#pragma unroll
  for (int q = 0; q < BW_PF; ++q) ring[q] = fetch(q);
  int bad = 0, pslot = -1;
  double pm = 0.0, pit = 0.0;
  // whole groups of BW_PF steps (the table's null tail): no step is guarded, so
  // no ring register is ever a merge of a fresh load and an old value
  for (int i0 = 0; i0 < ni; i0 += BW_PF) {  // uniform
#pragma unroll
    for (int q = 0; q < BW_PF; ++q) {
      // item i-1's accumulator reads first (every lane; non-owners read slot 0)
      const int ps = pslot >= 0 ? pslot : 0;
      const float2 e_a = L.acc[ps];
      const uint16_t e_cn = L.cnt[ps];
      const Pk pk = ring[q];
      const int inext = i0 + q + BW_PF;
      ring[q] = fetch(inext < ni ? inext : ni);  // past the end: the null entry
      const int rem = __builtin_amdgcn_readfirstlane(pk.rem);
      const bool act = fpos < (rem & 0x7fffffff);
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
        L.acc[pslot] = make_float2((float)((double)e_a.x + pit), (float)((double)e_a.y + pm));
      }
      // a new spectrum may touch item i-1's slots: its writes land first
      if (rem < 0) lds_barrier();
      pslot = (owner && inr && last) ? slot : -1;
      pm = pk.m;
      pit = pk.it;
    }
  }
  if (pslot >= 0) {
    L.cnt[pslot] = (uint16_t)(L.cnt[pslot] + 1u);
    const float2 a = L.acc[pslot];
    L.acc[pslot] = make_float2((float)((double)a.x + pit), (float)((double)a.y + pm));
  }
  if (block_any<BW_BLOCK, true>(bad, L.votes, 1)) return kUnsortedW;  // unsorted / NaN: the global kernel

  // 4: quorum filter and ordered output (binning.py:181-183, 209-222)
  const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)n * 0.25) + 1u : 1u;
  const int total = emit_striped<BW_BLOCK>(L.cnt, [&](int d) { return L.acc[d].x; }, [&](int d) { return L.acc[d].y; },
                                 L.wcnt, D, quorum, out.mz + p0, out.inten + p0);
  if (tid == 0) {
    out.count[c] = total;
    charge_out[c] = z0;
    prec_out[c] = pw_sum_small([&](int64_t j) { return L.prec[j]; }, n) / (double)n;  // np.mean (binning.py:224)
  }
  return kOk;
}

// Whether the wide kernel hands cluster c on by its size alone (bin_mean_wide_body's first
// test): more than BM_NMAX spectra, a bin space past BM_WMAX words, 2^28 peaks or more.
__device__ __forceinline__ bool bin_mean_past_wide(const CsrView& v, const BinMeanParams& P, int64_t c) {
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
  if (s1 == s0) return false;
  return s1 - s0 > BM_NMAX || P.n_words > BM_WMAX || v.spec_off[s1] - v.spec_off[s0] >= (int64_t(1) << 28);
}

// The bin-mean intake (round 6): every cluster the wide kernel would hand on by its size
// (the skewed law's clusters of more than 128 spectra) listed up front, so that the kept-bin
// fold of those clusters runs on the call's second stream BESIDE the register and wide
// kernels instead of after them; the wide kernel (owned = 1) then leaves them alone.
__global__ __launch_bounds__(256) void bin_mean_intake_kernel(CsrView v, BinMeanParams P, int32_t* list,
                                                              int32_t* n_list) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < v.n_clusters;
       c += (int64_t)gridDim.x * blockDim.x)
    if (bin_mean_past_wide(v, P, c)) list[atomicAdd(n_list, 1)] = (int32_t)c;
}

// The register kernel's leftovers, grid-stride over the list.
__global__ __launch_bounds__(BW_BLOCK, SPX_BW_MINW) void bin_mean_wide_kernel(CsrView v, BinMeanParams P,
                                                                              PeaksOut out, double* prec_out,
                                                                              int32_t* charge_out, int32_t* status,
                                                                              StripedList list,
                                                                              int32_t* deferred,
                                                                              int32_t* n_deferred, int32_t* glist,
                                                                              int32_t* n_glist, int owned) {
  __shared__ BinWideSmem L;
  __shared__ int32_t lbase[kListStripes + 1];
  const int32_t nl = striped_prefix(list, lbase);
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = striped_at(list, lbase, i);
    if (owned && bin_mean_past_wide(v, P, c)) continue;  // uniform: the intake's (bin_mean_intake_kernel)
    const int32_t st = bin_mean_wide_body(v, P, L, c, out, prec_out, charge_out);
    if (threadIdx.x == 0) {
      if (st == kUnsortedW) {
        status[c] = kDeferred;
        glist[atomicAdd(n_glist, 1)] = (int32_t)c;
      } else {
        status[c] = st;
        if (st == kDeferred) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
      }
    }
    lds_barrier();  // the LDS is reused by the next cluster
  }
}

}  // namespace spx
