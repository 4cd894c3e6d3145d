// Bin-mean for the clusters past the wide kernel -- more than 128 spectra (the
// configs[3] long tail, up to 5,000 spectra and ~1M peaks) or more than BW_DCAP
// distinct bins -- as a grid-parallel SEGMENTED FOLD (reference:
// src/binning.py:170-231).
//
// The reference's per-bin accumulation f32(f64(acc) + v) runs in spectrum order
// and does not reassociate, so each bin's contributions must meet in that order.
// Instead of walking the cluster's spectra one after another (a serial chain as
// long as the cluster), the contributions are sorted by (bin, spectrum) with a
// stable counting sort and every bin is then folded by one thread over its own
// contiguous segment:
//
//   setup    (WG per cluster)   mixed-charge check; bitmap from the arena;
//                               work items = blocks of SG_SB = 64 spectra
//   occupy   (grid, per block)  occupied bins (LDS bitmap per block, ORed into
//                               the cluster's) and the sortedness / NaN check
//   prefix   (WG per cluster)   bin -> slot (popcount prefix); the D-sized tables
//   mask     (grid, per block)  mask[b][slot] bit s: the block's spectrum s holds
//                               the last peak of that bin (numpy fancy-index +=
//                               keeps the last, binning.py:197-199)
//   count    (grid, per slot)   boff[b][slot] = contributions of earlier blocks;
//                               tot[slot]
//   scan     (WG per cluster)   seg[slot] = contributions of earlier slots
//   place    (grid, per block)  value of (s, slot) -> seg[slot] + boff[b][slot] +
//                               popcount(mask[b][slot] below s): spectrum order
//   fold     (grid, per slot)   one thread per bin over its segment, in order
//   emit     (WG per cluster)   quorum, ordered output, count, charge, np.mean
//
// Every table lives in a bump-allocated arena of the workspace; a cluster that
// does not fit goes on to the bin-range split path, an unsorted or NaN one to
// the global kernel.  HBM traffic per peak: m/z three times, the intensity once,
// 16 B of contribution written and read back, plus the (block x slot) tables.
#pragma once
#include "bin_mean.hip"

namespace spx {

constexpr int SG_SB = 64;      // spectra per block (one bit each in a u64 mask)
constexpr int SG_BLOCK = 256;  // threads per workgroup
constexpr int SG_TILE = 256;   // slots per fold / count workgroup
enum : int32_t { kSegOk = 0, kSegBad = 1, kSegNoRoom = 2, kSegDone = 3 };

struct SegMeta {
  int64_t c, p0;
  int32_t n, nb;       // spectra, blocks
  int32_t D, state;    // occupied bins; kSeg*
  int32_t task0, tile0;  // first block task, first slot tile
  int64_t bm, pre;       // arena offsets: bitmap (n_words u64), prefix (n_words u32)
  int64_t mask, boff;    // mask[b * D + slot] u64, boff[b * D + slot] u16
  int64_t seg, vals;     // seg[slot] u32 (D + 1), contributions (m/z, intensity) f64 x 2
  int64_t res, keep;     // res[slot] (m/z mean, intensity mean) f64 x 2, keep[slot] u32 (D + 1)
};

__device__ __forceinline__ int64_t seg_align(int64_t b) { return (b + 255) & ~int64_t(255); }

// bump allocation from the arena; -1 when it is exhausted
__device__ __forceinline__ int64_t seg_alloc(unsigned long long* bump, int64_t bytes, int64_t cap) {
  const unsigned long long o = atomicAdd(bump, (unsigned long long)seg_align(bytes));
  return (int64_t)o + seg_align(bytes) <= cap ? (int64_t)o : -1;
}

// setup: one workgroup per deferred cluster (grid-stride over the list)
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_setup_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    const int32_t* list, const int32_t* n_list, SegMeta* meta, char* arena, unsigned long long* bump, int64_t cap,
    int32_t* task_cl, int32_t* n_tasks) {
  __shared__ int votes[2 * (SG_BLOCK / kWave)];
  __shared__ int64_t s_bm;
  __shared__ int32_t s_task0;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = list[i];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int n = (int)(s1 - s0);
    const int32_t z0 = v.charge[s0];
    int mixed = 0;
    for (int64_t s = s0 + 1 + tid; s < s1; s += SG_BLOCK) mixed |= v.charge[s] != z0;
    const bool mix = block_any<SG_BLOCK, false>(mixed, votes, 0);
    SegMeta M = {};
    M.c = c;
    M.p0 = v.spec_off[s0];
    M.n = n;
    M.nb = (n + SG_SB - 1) / SG_SB;
    if (mix) {  // binning.py:205-206: nothing emitted
      if (tid == 0) {
        out.count[c] = 0;
        prec_out[c] = __longlong_as_double(0x7ff8000000000000ll);
        charge_out[c] = 0;
        status[c] = kMixedCharge;
        M.state = kSegDone;
        M.task0 = 0;
        M.nb = 0;
        meta[i] = M;
      }
      __syncthreads();
      continue;
    }
    const int64_t P_c = v.spec_off[s1] - M.p0;
    // the tables' limits: the LDS bitmap of a block, u16 block offsets, u32 segments
    const bool fits = P.n_words <= BM_WMAX && n <= 65535 && P_c < (int64_t(1) << 28);
    if (tid == 0) {
      s_bm = fits ? seg_alloc(bump, (int64_t)P.n_words * 12, cap) : -1;
      s_task0 = s_bm >= 0 ? atomicAdd(n_tasks, M.nb) : 0;
    }
    __syncthreads();
    const int64_t bm = s_bm;
    M.bm = bm;
    M.pre = bm + (int64_t)P.n_words * 8;
    M.task0 = s_task0;
    if (bm < 0) {
      M.state = kSegNoRoom;
      M.nb = 0;
    } else {
      unsigned long long* B = reinterpret_cast<unsigned long long*>(arena + bm);
      for (int w = tid; w < P.n_words; w += SG_BLOCK) B[w] = 0ull;
      for (int k = tid; k < M.nb; k += SG_BLOCK) task_cl[M.task0 + k] = i;
    }
    if (tid == 0) meta[i] = M;
    __syncthreads();
  }
}

// The block's spectra, one wave per spectrum at a time, in GROUPS of 4 x 63
// peaks (lane j of chunk q owns peak g0 + 63q + j, j < 63; lane 63 reads the next
// peak only to hand lane 62 its key): bin, last-in-bin by the DPP neighbour key
// (numpy fancy-index += keeps the last, binning.py:197-199), the sortedness / NaN
// check.  The next group's loads are issued before the current one is processed.
// f(k, key, last, spectrum-in-block) for every in-range peak.  Returns "bad".
constexpr int SG_GQ = 4;                       // chunks per group
constexpr int SG_GROUP = SG_GQ * (kWave - 1);  // peaks per group (252)

// walk_block: the same walk for any block of nsb spectra whose offsets (relative
// to the cluster's first peak p0) are in LDS; kInten also streams the
// intensities alongside.  f(k, key, last, spectrum-in-block, m/z, intensity).
// SG_WR groups are in flight per wave: a ring of register groups, unrolled so
// every slot is a fixed register set, each refilled with the group SG_WR ahead.
constexpr int SG_WR = 2;  // ring slots (one group in flight + the one processed)

struct NoChunkHook {
  __device__ void operator()(int) const {}
};

// chunk(sl): after each 63-peak chunk of spectrum sl, every lane of the wave (uniform)
template <bool kInten, class F, class C = NoChunkHook>
__device__ __forceinline__ int walk_block(const CsrView& v, const BinMeanParams& P, int64_t p0, int nsb,
                                          const int32_t* soff, F&& f, C&& chunk = C{}) {
  constexpr int NW = SG_BLOCK / kWave;
  const int lane = lane_id(), wid = wave_id();
  // buffer loads over the block's peaks: a position past its spectrum reads the
  // descriptor's end and returns 0 -- no guarded load, so no register is a merge
  // of a load and a constant and the ring stays in flight (counted vmcnt)
  const int npb = soff[nsb];  // < 2^28 (the setups' limit)
  const __amdgpu_buffer_rsrc_t rmz = bf_rsrc(v.mz + p0, npb);
  const __amdgpu_buffer_rsrc_t rit = bf_rsrc(v.inten + p0, npb);
  const bool owner = lane < kWave - 1;
  auto skip = [&](int& s) { while (s < nsb && soff[s + 1] == soff[s]) s += NW; };
  // the group after (sl, g0): the next 252 peaks of the spectrum or the wave's
  // next non-empty spectrum; past the end it stays there
  auto advance = [&](int& sl, int& g0) __attribute__((always_inline)) {
    if (sl >= nsb) return;
    g0 += SG_GROUP;
    if (g0 >= soff[sl + 1] - soff[sl]) {
      sl += NW;
      g0 = 0;
      skip(sl);
    }
  };
  auto load = [&](int s, int g, double* m, double* x) __attribute__((always_inline)) {
    const int a = s < nsb ? soff[s] : 0, e = s < nsb ? soff[s + 1] : 0;
#pragma unroll
    for (int q = 0; q < SG_GQ; ++q) {
      const int k = a + g + q * (kWave - 1) + lane;
      const int bo = (k < e ? k : npb) * 8;
      m[q] = bf_load(rmz, bo, 0);
      if constexpr (kInten) x[q] = bf_load(rit, bo, 0);
    }
  };
  int csl[SG_WR], cg[SG_WR];
  double cm[SG_WR][SG_GQ], cx[SG_WR][SG_GQ];
  csl[0] = wid;
  cg[0] = 0;
  skip(csl[0]);
#pragma unroll
  for (int r = 1; r < SG_WR; ++r) {
    csl[r] = csl[r - 1];
    cg[r] = cg[r - 1];
    advance(csl[r], cg[r]);
  }
#pragma unroll
  for (int r = 0; r < SG_WR; ++r) load(csl[r], cg[r], cm[r], cx[r]);
  int bad = 0;
  while (csl[0] < nsb) {  // uniform
#pragma unroll
    for (int r = 0; r < SG_WR; ++r) {
      if (csl[r] < nsb) {  // uniform; cursors ascend, so past one end all are
        const int sl = csl[r];
        const int a = soff[sl], e = soff[sl + 1];
        const int g0 = cg[r];
        double m_[SG_GQ], x_[SG_GQ];
#pragma unroll
        for (int q = 0; q < SG_GQ; ++q) {
          m_[q] = cm[r][q];
          if constexpr (kInten) x_[q] = cx[r][q];
        }
        // refill this slot with the group SG_WR ahead (after the newest cursor)
        const int prev = (r + SG_WR - 1) % SG_WR;
        int nsl = csl[prev], ng = cg[prev];
        advance(nsl, ng);
        load(nsl, ng, cm[r], cx[r]);
        csl[r] = nsl;
        cg[r] = ng;
#pragma unroll
        for (int q = 0; q < SG_GQ; ++q) {
          const int k = a + g0 + q * (kWave - 1) + lane;
          const bool act = k < e;
          const double m = m_[q];
          const bool inr = act && in_range(m, P);
          const int32_t key = inr ? bin_small(m, P) : ((act && m < P.minimum) ? -1 : 0x7fffffff);
          const int32_t kn = wave_next(key, 0x7fffffff);
          bad |= (int)(owner && act && ((m != m) || key > kn));
          if (owner && inr) f(p0 + k, key, kn != key, sl, m, kInten ? x_[q] : 0.0);
          chunk(sl);
        }
      }
    }
  }
  return bad;
}

template <class F>
__device__ __forceinline__ int seg_walk_block(const CsrView& v, const BinMeanParams& P, const SegMeta& M, int b,
                                              const int32_t* soff, F&& f) {
  const int nsb = min(M.n - b * SG_SB, SG_SB);  // spectra in this block
  return walk_block<false>(v, P, M.p0, nsb, soff, [&](int64_t k, int32_t key, bool last, int s, double, double) {
    f(k, key, last, s);
  });
}

// the block's spectrum offsets (relative to the cluster's first peak) into LDS
__device__ __forceinline__ void seg_block_offsets(const CsrView& v, const SegMeta& M, int b, int32_t* soff) {
  const int64_t s0 = v.cluster_off[M.c] + (int64_t)b * SG_SB;
  const int nsb = min(M.n - b * SG_SB, SG_SB);
  for (int j = threadIdx.x; j <= nsb; j += SG_BLOCK) soff[j] = (int32_t)(v.spec_off[s0 + j] - M.p0);
}

// occupancy: one workgroup per (cluster, block) task
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_occupy_kernel(CsrView v, BinMeanParams P, SegMeta* meta,
                                                                       char* arena, const int32_t* task_cl,
                                                                       const int32_t* n_tasks) {
  __shared__ unsigned long long bits[BM_WMAX];
  __shared__ int32_t soff[SG_SB + 1];
  __shared__ int votes[2 * (SG_BLOCK / kWave)];
  const int tid = threadIdx.x;
  const int32_t nt = *n_tasks;
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = task_cl[t];
    const SegMeta M = meta[i];
    for (int w = tid; w < P.n_words; w += SG_BLOCK) bits[w] = 0ull;
    seg_block_offsets(v, M, t - M.task0, soff);
    lds_barrier();
    const int bad = seg_walk_block(v, P, M, t - M.task0, soff, [&](int64_t, int32_t key, bool, int) {
      atomicOr(&bits[key >> 6], 1ull << (key & 63));
    });
    if (block_any<SG_BLOCK, true>(bad, votes, 0) && tid == 0) atomicOr(&meta[i].state, kSegBad);
    unsigned long long* B = reinterpret_cast<unsigned long long*>(arena + M.bm);
    for (int w = tid; w < P.n_words; w += SG_BLOCK)
      if (bits[w]) atomicOr(&B[w], bits[w]);
    lds_barrier();
  }
}

// prefix: one workgroup per cluster -- slots, then the D-sized tables
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_prefix_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    const int32_t* n_list, SegMeta* meta, char* arena, unsigned long long* bump, int64_t cap, int32_t* tile_cl,
    int32_t* n_tiles) {
  __shared__ int tmp[SG_BLOCK / kWave + 1];
  __shared__ SegMeta sM;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    SegMeta M = meta[i];
    if (M.state != kSegOk) {
      __syncthreads();
      continue;
    }
    const unsigned long long* B = reinterpret_cast<const unsigned long long*>(arena + M.bm);
    uint32_t* pre = reinterpret_cast<uint32_t*>(arena + M.pre);
    const int D = bitmap_prefix<SG_BLOCK, uint32_t>(B, pre, P.n_words, tmp);
    if (tid == 0) {
      M.D = D;
      const int64_t nbD = (int64_t)M.nb * D;
      const int64_t P_c = v.spec_off[v.cluster_off[M.c + 1]] - M.p0;  // contributions <= peaks
      const int64_t bytes = seg_align(nbD * 8) + seg_align(nbD * 2) + seg_align((int64_t)(D + 1) * 4) +
                            seg_align(P_c * 16) + seg_align((int64_t)D * 16) + seg_align((int64_t)(D + 1) * 4);
      const int64_t base = D > 0 ? seg_alloc(bump, bytes, cap) : 0;
      if (D == 0) {
        // no in-range peak: an empty consensus (count 0), charge and np.mean as usual
        const int64_t s0 = v.cluster_off[M.c];
        out.count[M.c] = 0;
        charge_out[M.c] = v.charge[s0];
        prec_out[M.c] = pw_sum([&](int64_t j) { return v.prec_mz[s0 + j]; }, M.n) / (double)M.n;
        status[M.c] = kOk;
        M.state = kSegDone;
      } else if (base < 0) {
        M.state = kSegNoRoom;
      } else {
        M.mask = base;
        M.boff = M.mask + seg_align(nbD * 8);
        M.seg = M.boff + seg_align(nbD * 2);
        M.vals = M.seg + seg_align((int64_t)(D + 1) * 4);
        M.res = M.vals + seg_align(P_c * 16);
        M.keep = M.res + seg_align((int64_t)D * 16);
        const int nt = (D + SG_TILE - 1) / SG_TILE;
        M.tile0 = atomicAdd(n_tiles, nt);
      }
      sM = M;
    }
    __syncthreads();
    M = sM;
    if (M.state == kSegOk) {
      const int nt = (M.D + SG_TILE - 1) / SG_TILE;
      for (int k = tid; k < nt; k += SG_BLOCK) tile_cl[M.tile0 + k] = i;
    }
    if (tid == 0) meta[i] = M;
    __syncthreads();
  }
}

__device__ __forceinline__ int seg_slot(const SegMeta& M, const char* arena, int32_t key) {
  const unsigned long long* B = reinterpret_cast<const unsigned long long*>(arena + M.bm);
  const uint32_t* pre = reinterpret_cast<const uint32_t*>(arena + M.pre);
  return bitmap_rank(B, pre, (int64_t)key);
}

// ---- block-local slots: the block's own occupied bins, ranked in LDS, so the
// mask and place passes work on LDS arrays instead of global atomics / lookups
#ifndef SPX_SG_LCAP
#define SPX_SG_LCAP 3072
#endif
constexpr int SG_LCAP = SPX_SG_LCAP;  // block-local occupied bins held in LDS (more: the global-atomic form)

struct SegBlockSmem {
  unsigned long long bits[BM_WMAX];
  uint16_t lpre[BM_WMAX];
  unsigned long long lmask[SG_LCAP];  // mask pass: bit s = spectrum s of the block contributes
  uint32_t lbase[SG_LCAP];            // place pass: the slot's segment position of the block's first
  int32_t soff[SG_SB + 1];
  int tmp[SG_BLOCK / kWave + 1];
};

// walk 1 + prefix: the block's occupied bins and their local ranks; returns D_b
__device__ __forceinline__ int seg_local_slots(const CsrView& v, const BinMeanParams& P, const SegMeta& M, int b,
                                               SegBlockSmem& L) {
  const int tid = threadIdx.x;
  for (int w = tid; w < P.n_words; w += SG_BLOCK) L.bits[w] = 0ull;
  seg_block_offsets(v, M, b, L.soff);
  lds_barrier();
  seg_walk_block(v, P, M, b, L.soff, [&](int64_t, int32_t key, bool last, int) {
    if (last) atomicOr(&L.bits[key >> 6], 1ull << (key & 63));
  });
  lds_barrier();
  return bitmap_prefix<SG_BLOCK, uint16_t, true>(L.bits, L.lpre, P.n_words, L.tmp);
}

// f(local slot, bin) for every occupied bin of the block (thread per bitmap word)
template <class F>
__device__ __forceinline__ void seg_for_local_slots(const BinMeanParams& P, const SegBlockSmem& L, F&& f) {
  for (int w = threadIdx.x; w < P.n_words; w += SG_BLOCK) {
    unsigned long long x = L.bits[w];
    int ls = L.lpre[w];
    while (x) {
      const int bit = __ffsll((long long)x) - 1;
      x &= x - 1ull;
      f(ls++, w * 64 + bit);
    }
  }
}

// mask: one workgroup per (cluster, block) task -- mask[b][slot] bit s: spectrum
// s of block b holds the last peak of that bin
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_mask_kernel(CsrView v, BinMeanParams P,
                                                                     const SegMeta* meta, char* arena,
                                                                     const int32_t* task_cl,
                                                                     const int32_t* n_tasks) {
  __shared__ SegBlockSmem L;
  const int tid = threadIdx.x;
  const int32_t nt = *n_tasks;
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = task_cl[t];
    const SegMeta M = meta[i];
    if (M.state != kSegOk) continue;  // uniform
    const int b = t - M.task0;
    unsigned long long* mask = reinterpret_cast<unsigned long long*>(arena + M.mask) + (int64_t)b * M.D;
    for (int d = tid; d < M.D; d += SG_BLOCK) mask[d] = 0ull;
    const int Db = seg_local_slots(v, P, M, b, L);
    if (Db <= SG_LCAP) {
      for (int ls = tid; ls < Db; ls += SG_BLOCK) L.lmask[ls] = 0ull;
      lds_barrier();
      seg_walk_block(v, P, M, b, L.soff, [&](int64_t, int32_t key, bool last, int s) {
        if (last) atomicOr(&L.lmask[bitmap_rank(L.bits, L.lpre, (int64_t)key)], 1ull << s);
      });
      __syncthreads();  // the LDS masks are complete and the row's zeros have landed
      seg_for_local_slots(P, L, [&](int ls, int32_t key) { mask[seg_slot(M, arena, key)] = L.lmask[ls]; });
    } else {  // a block with more distinct bins than LDS holds: global atomics
      __syncthreads();
      seg_walk_block(v, P, M, b, L.soff, [&](int64_t, int32_t key, bool last, int s) {
        if (last) atomicOr(&mask[seg_slot(M, arena, key)], 1ull << s);
      });
    }
    __syncthreads();  // the LDS is reused by the next task
  }
}

// count: one thread per slot -- contributions of earlier blocks (boff) and the total
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_count_kernel(const SegMeta* meta, char* arena,
                                                                      const int32_t* tile_cl,
                                                                      const int32_t* n_tiles) {
  constexpr int U = 8;  // mask loads in flight per thread
  const int32_t nt = *n_tiles;
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = tile_cl[t];
    const SegMeta M = meta[i];
    if (M.state != kSegOk) continue;
    const int d = (t - M.tile0) * SG_TILE + threadIdx.x;
    if (d >= M.D) continue;
    const unsigned long long* mask = reinterpret_cast<const unsigned long long*>(arena + M.mask) + d;
    uint16_t* boff = reinterpret_cast<uint16_t*>(arena + M.boff) + d;
    uint32_t run = 0;
    for (int b0 = 0; b0 < M.nb; b0 += U) {
      unsigned long long x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = b0 + u < M.nb ? mask[(int64_t)(b0 + u) * M.D] : 0ull;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (b0 + u < M.nb) boff[(int64_t)(b0 + u) * M.D] = (uint16_t)run;
        run += (uint32_t)__popcll(x[u]);
      }
    }
    reinterpret_cast<uint32_t*>(arena + M.seg)[d] = run;
  }
}

// scan: one workgroup per cluster -- seg[slot] = contributions of earlier slots
// (thread t scans the contiguous run t*per .. (t+1)*per, its loads batched)
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_scan_kernel(const int32_t* n_list, const SegMeta* meta,
                                                                     char* arena) {
  __shared__ uint32_t tmp[SG_BLOCK / kWave + 1];
  constexpr int U = 8;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const SegMeta M = meta[i];
    if (M.state != kSegOk) continue;  // uniform
    uint32_t* seg = reinterpret_cast<uint32_t*>(arena + M.seg);
    const int per = (M.D + SG_BLOCK - 1) / SG_BLOCK, d0 = tid * per, d1 = min(M.D, d0 + per);
    uint32_t local = 0;
    for (int k0 = d0; k0 < d1; k0 += U) {
      uint32_t x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = k0 + u < d1 ? seg[k0 + u] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) local += x[u];
    }
    uint32_t total;
    uint32_t base = block_exclusive_scan<SG_BLOCK, uint32_t>(local, tmp, total);
    for (int k0 = d0; k0 < d1; k0 += U) {
      uint32_t x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = k0 + u < d1 ? seg[k0 + u] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (k0 + u < d1) seg[k0 + u] = base;
        base += x[u];
      }
    }
    if (tid == 0) seg[M.D] = total;
    __syncthreads();
  }
}

// place: one workgroup per (cluster, block) task -- each contribution into its
// bin's segment at seg[slot] + boff[b][slot] + popcount(mask[b][slot] below s),
// i.e. in spectrum order
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_place_kernel(CsrView v, BinMeanParams P,
                                                                      const SegMeta* meta, char* arena,
                                                                      const int32_t* task_cl,
                                                                      const int32_t* n_tasks) {
  __shared__ SegBlockSmem L;
  const int32_t nt = *n_tasks;
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = task_cl[t];
    const SegMeta M = meta[i];
    if (M.state != kSegOk) continue;  // uniform
    const int b = t - M.task0;
    const unsigned long long* mask = reinterpret_cast<const unsigned long long*>(arena + M.mask) + (int64_t)b * M.D;
    const uint16_t* boff = reinterpret_cast<const uint16_t*>(arena + M.boff) + (int64_t)b * M.D;
    const uint32_t* seg = reinterpret_cast<const uint32_t*>(arena + M.seg);
    double2* vals = reinterpret_cast<double2*>(arena + M.vals);
    const int Db = seg_local_slots(v, P, M, b, L);
    if (Db <= SG_LCAP) {
      seg_for_local_slots(P, L, [&](int ls, int32_t key) {
        const int d = seg_slot(M, arena, key);
        L.lbase[ls] = seg[d] + boff[d];
        L.lmask[ls] = mask[d];
      });
      lds_barrier();
      seg_walk_block(v, P, M, b, L.soff, [&](int64_t k, int32_t key, bool last, int s) {
        if (!last) return;
        const int ls = bitmap_rank(L.bits, L.lpre, (int64_t)key);
        const uint32_t pos = L.lbase[ls] + (uint32_t)__popcll(L.lmask[ls] & ((1ull << s) - 1ull));
        vals[pos] = make_double2(v.mz[k], v.inten[k]);
      });
    } else {
      seg_walk_block(v, P, M, b, L.soff, [&](int64_t k, int32_t key, bool last, int s) {
        if (!last) return;
        const int d = seg_slot(M, arena, key);
        const uint32_t pos = seg[d] + boff[d] + (uint32_t)__popcll(mask[d] & ((1ull << s) - 1ull));
        vals[pos] = make_double2(v.mz[k], v.inten[k]);
      });
    }
    __syncthreads();  // the LDS is reused by the next task
  }
}

// fold: one thread per slot over its segment, in spectrum order (binning.py:198-199),
// loads issued SG_FU ahead of the (serial) f32 accumulation; then the quorum
// (:181-183) and the means (:209-222)
constexpr int SG_FU = 8;
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_fold_kernel(BinMeanParams P, const SegMeta* meta,
                                                                     char* arena, const int32_t* tile_cl,
                                                                     const int32_t* n_tiles) {
  const int32_t nt = *n_tiles;
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = tile_cl[t];
    const SegMeta M = meta[i];
    if (M.state != kSegOk) continue;
    const int d = (t - M.tile0) * SG_TILE + threadIdx.x;
    if (d >= M.D) continue;
    const uint32_t* seg = reinterpret_cast<const uint32_t*>(arena + M.seg);
    const double2* vals = reinterpret_cast<const double2*>(arena + M.vals);
    const uint32_t a = seg[d], e = seg[d + 1];
    float si = 0.0f, sm = 0.0f;
    double2 ring[SG_FU];
#pragma unroll
    for (int u = 0; u < SG_FU; ++u) ring[u] = vals[min(a + u, e - 1)];  // e > a: every slot has a contribution
    for (uint32_t k0 = a; k0 < e; k0 += SG_FU) {
#pragma unroll
      for (int u = 0; u < SG_FU; ++u) {
        const double2 x = ring[u];
        ring[u] = vals[min(k0 + u + SG_FU, e - 1)];  // (clamped: the tail re-reads the last)
        if (k0 + u < e) {
          si = (float)((double)si + x.y);
          sm = (float)((double)sm + x.x);
        }
      }
    }
    const uint32_t cnt = e - a;
    const uint32_t quorum = P.apply_quorum ? (uint32_t)((double)M.n * 0.25) + 1u : 1u;
    const bool keep = cnt >= quorum && !isnan(si);  // cnt >= 1: mean NaN iff sum NaN
    reinterpret_cast<uint32_t*>(arena + M.keep)[d] = keep ? 1u : 0u;
    const double cn = (double)cnt;
    reinterpret_cast<double2*>(arena + M.res)[d] =
        make_double2(sm == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)sm / cn, (double)si / cn);
  }
}

// numpy's pairwise mean of x[0..n) by a whole workgroup: the leaves (<= 128
// elements, numpy's recursion) found by descending from the root (thread 0, no
// stack), summed 8 lanes per leaf, then combined in numpy's order by a post-order
// stack machine over the leaves' root paths (thread 0, the stack in LDS).  More
// than SG_MAXLEAF leaves: thread 0 alone (pw_sum).
constexpr int SG_MAXLEAF = SG_BLOCK;
struct PwSmem {
  int64_t lo[SG_MAXLEAF];
  int32_t len[SG_MAXLEAF];
  uint32_t path[SG_MAXLEAF];  // left (0) / right (1) turns from the root, the last turn in bit 0
  int32_t depth[SG_MAXLEAF];
  double sum[SG_MAXLEAF];
  double stk[40];
  int nleaf;
};

__device__ double seg_pw_mean(const double* x, int64_t n, PwSmem& S) {
  const int tid = threadIdx.x;
  if (tid == 0) {
    int k = 0;
    int64_t p = 0;
    while (p < n && k <= SG_MAXLEAF) {
      int64_t l = 0, m = n;
      uint32_t path = 0;
      int d = 0;
      while (m > 128) {  // split [l, l+m) at h = m/2 - (m/2)%8 (pw_tree)
        int64_t h = m / 2;
        h -= h % 8;
        if (p < l + h) {
          m = h;
          path <<= 1;
        } else {
          l += h;
          m -= h;
          path = (path << 1) | 1u;
        }
        ++d;
      }
      if (k < SG_MAXLEAF) {
        S.lo[k] = l;
        S.len[k] = (int32_t)m;
        S.path[k] = path;
        S.depth[k] = d;
      }
      ++k;
      p = l + m;
    }
    S.nleaf = k;
  }
  __syncthreads();
  const int nl = S.nleaf;
  if (nl > SG_MAXLEAF) {  // thread 0, serially
    double r = 0.0;
    if (tid == 0) r = pw_sum([&](int64_t j) { return x[j]; }, n) / (double)n;
    return r;
  }
  // the leaf sums, 8 lanes per leaf: lane i holds numpy's i-th strided partial
  // sum (its <= 16 loads issued at once), combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
  // by xor shuffles, then the sequential tail (pw_leaf)
  for (int base = 0; base < nl; base += SG_BLOCK / 8) {  // uniform
    const int l = base + tid / 8, i = tid & 7;
    const bool act = l < nl;
    const int64_t l0 = act ? S.lo[l] : 0;
    const int64_t m = act ? S.len[l] : 0;
    const int64_t lim = m - (m % 8);
    double r = 0.0;
    if (m >= 8) {
      double xs[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) xs[t] = x[l0 + min<int64_t>(i + 8 * t, m - 1)];  // (clamped: m <= 128)
      r = xs[0];
#pragma unroll
      for (int t = 1; t < 16; ++t)
        if (8 * t < lim) r += xs[t];
    }
    r += xor_f64<1>(r);
    r += xor_f64<2>(r);
    r += xor_f64<4>(r);
    if (act && i == 0) {
      if (m < 8) {
        r = 0.0;
        for (int64_t j = 0; j < m; ++j) r += x[l0 + j];
      } else {
        for (int64_t j = lim; j < m; ++j) r += x[l0 + j];
      }
      S.sum[l] = r;
    }
  }
  __syncthreads();
  double r = 0.0;
  if (tid == 0) {
    // post-order: a leaf (or a finished subtree) that is a right child joins its
    // left sibling on the stack: left + right, as pw_tree adds them
    int sp = 0;
    for (int k = 0; k < nl; ++k) {
      double v = S.sum[k];
      uint32_t path = S.path[k];
      for (int d = S.depth[k]; d > 0 && (path & 1u); --d) {
        v = S.stk[--sp] + v;
        path >>= 1;
      }
      S.stk[sp++] = v;
    }
    r = (0.0 + S.stk[0]) / (double)n;
  }
  return r;
}

// emit: one workgroup per cluster -- kept slots in bin order, count, charge, np.mean
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_seg_emit_kernel(CsrView v, PeaksOut out, double* prec_out,
                                                                     int32_t* charge_out, int32_t* status,
                                                                     const int32_t* n_list, const SegMeta* meta,
                                                                     char* arena, int32_t* split_list,
                                                                     int32_t* n_split, int32_t* glist,
                                                                     int32_t* n_glist) {
  __shared__ uint32_t tmp[SG_BLOCK / kWave + 1];
  __shared__ PwSmem pws;
  constexpr int U = 8;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const SegMeta M = meta[i];
    if (M.state != kSegOk) {  // uniform
      if (tid == 0) {
        if (M.state == kSegBad) glist[atomicAdd(n_glist, 1)] = (int32_t)M.c;  // unsorted / NaN
        if (M.state == kSegNoRoom) split_list[atomicAdd(n_split, 1)] = (int32_t)M.c;  // arena full
      }
      continue;
    }
    const uint32_t* keep = reinterpret_cast<const uint32_t*>(arena + M.keep);
    const double2* res = reinterpret_cast<const double2*>(arena + M.res);
    const int per = (M.D + SG_BLOCK - 1) / SG_BLOCK, d0 = tid * per, d1 = min(M.D, d0 + per);
    uint32_t local = 0;
    for (int k0 = d0; k0 < d1; k0 += U) {
      uint32_t x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = k0 + u < d1 ? keep[k0 + u] : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) local += x[u];
    }
    uint32_t total;
    uint32_t o = block_exclusive_scan<SG_BLOCK, uint32_t>(local, tmp, total);
    for (int d = d0; d < d1; ++d) {
      if (keep[d]) {
        const double2 r = res[d];
        out.mz[M.p0 + o] = r.x;
        out.inten[M.p0 + o] = r.y;
        ++o;
      }
    }
    const int64_t s0 = v.cluster_off[M.c];
    const double pm = seg_pw_mean(v.prec_mz + s0, M.n, pws);  // np.mean (binning.py:224)
    if (tid == 0) {
      out.count[M.c] = total;
      charge_out[M.c] = v.charge[s0];
      prec_out[M.c] = pm;
      status[M.c] = kOk;
    }
    __syncthreads();
  }
}

}  // namespace spx
