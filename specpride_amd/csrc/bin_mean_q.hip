// Bin-mean for the clusters past the wide kernel when the peak quorum applies
// (the reference's default, binning.py:181-183): a KEPT-BIN fold (reference:
// src/binning.py:170-231).
//
// A bin survives only with at least int(0.25 n) + 1 contributions, so in a large
// cluster the bins that need a sum are few (the peptide's fragment bins) and
// every one of them is hit by a quarter of the spectra or more, while the noise
// bins -- most of the distinct bins -- only need a count.  So:
//
//   setup  (WG per cluster)  mixed-charge check (binning.py:205-206); the bin
//                            window [lo, hi] from each spectrum's first and last
//                            peak; blocks of sb <= 64 spectra with sb * longest
//                            spectrum <= Q_LCAP
//   tally  (grid, per block) last-peak-of-its-bin per spectrum (numpy fancy-index
//                            += keeps the last, binning.py:197-199) counted per
//                            bin in LDS; one dense u8 row per block over the
//                            window; the sortedness / NaN check
//   count  (grid, per tile)  column sums of the rows: kept[bin] = count >= quorum
//                            (a ballot per 64 bins: the kept bitmap)
//   plan   (WG per cluster)  kept bin -> its rank k; the dense value table V[k][s]
//                            (K x n, 16 B) and the presence masks P[k][block]
//   place  (grid, per block) (m/z, intensity) of spectrum s's last peak in kept
//                            bin k -> V[k][s]; P[k][block] bit s
//   fold   (wave per kept bin) the f32(f64(acc) + v) chain in spectrum order
//                            (binning.py:198-199): the wave loads 64 spectra's
//                            entries at once and folds the present ones in order
//                            by lane broadcast -- the chain is as long as the
//                            cluster, so a lane-per-bin fold would wait on memory
//   emit   (WG per cluster)  kept bins with a non-NaN intensity mean, in bin
//                            order; count, charge, np.mean of the precursors
//
// A cluster that does not fit (no quorum, a wide bin space, more than Q_KCAP
// kept bins, an exhausted arena) goes on to the segmented fold, an unsorted or
// NaN one to the global kernel.  HBM traffic per peak: m/z three times (tally
// twice, place once), the intensity once; 16 B written and read back per kept
// contribution; the u8 rows (one byte per bin and block).
#pragma once
#include "bin_mean_seg.hip"

namespace spx {

#ifndef SPX_Q_LCAP
#define SPX_Q_LCAP 16384
#endif
constexpr int Q_LCAP = SPX_Q_LCAP;  // block-local occupied bins (u8 counts packed four to an LDS word)
constexpr int Q_KCAP = 2048;        // kept bins per cluster (place's LDS presence masks)
constexpr int Q_TILEW = 16;         // bitmap words (1,024 bins) per count workgroup
enum : int32_t { kQOk = 0, kQBad = 1, kQNoFit = 2, kQDone = 3 };

struct QMeta {
  int64_t c, p0;
  int32_t n, nb, sb, state;      // spectra, blocks, spectra per block, kQ*
  int32_t lo_w, nw, task0, tile0;  // window words [lo_w, lo_w + nw); first block task, first count tile
  int32_t unit0, K, pad0, pad1;  // first fold unit (wave), kept bins
  int64_t rows, kbits, kpre;     // arena offsets: rows[b][bin] u8, kept bitmap (nw u64), its prefix (nw u32)
  int64_t vals, pbits, res;      // V[k][s] (m/z, intensity), P[k][b] u64, res[k] (m/z mean, intensity mean)
};

__device__ __forceinline__ unsigned long long uniform_u64(unsigned long long x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// window key of a spectrum's first / last m/z: below the range -> 0, past it ->
// the last bin (a NaN lands on 0; the tally's walk flags it)
__device__ __forceinline__ int32_t q_window_key(double m, const BinMeanParams& P) {
  if (!(m >= P.minimum)) return 0;
  if (m >= P.maximum) return P.n_words * 64 - 1;
  return bin_small(m, P);
}

// setup: one workgroup per cluster of the list (grid-stride)
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_setup_kernel(
    CsrView v, BinMeanParams P, PeaksOut out, double* prec_out, int32_t* charge_out, int32_t* status,
    const int32_t* list, const int32_t* n_list, QMeta* meta, char* arena, unsigned long long* bump, int64_t cap,
    int32_t* task_cl, int32_t* n_tasks, int32_t task_cap, int32_t* tile_cl, int32_t* n_tiles, int32_t tile_cap,
    int enabled) {
  __shared__ int votes[2 * (SG_BLOCK / kWave)];
  __shared__ int red[3];
  __shared__ QMeta sM;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = list[i];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int n = (int)(s1 - s0);
    const int32_t z0 = v.charge[s0];
    int mixed = 0;
    for (int64_t s = s0 + 1 + tid; s < s1; s += SG_BLOCK) mixed |= v.charge[s] != z0;
    if (tid == 0) { red[0] = 0; red[1] = 0x7fffffff; red[2] = -1; }
    const bool mix = block_any<SG_BLOCK, false>(mixed, votes, 0);
    QMeta M = {};
    M.c = c;
    M.p0 = v.spec_off[s0];
    M.n = n;
    if (mix) {  // binning.py:205-206: nothing emitted
      if (tid == 0) {
        out.count[c] = 0;
        prec_out[c] = __longlong_as_double(0x7ff8000000000000ll);
        charge_out[c] = 0;
        status[c] = kMixedCharge;
        M.state = kQDone;
        meta[i] = M;
      }
      __syncthreads();
      continue;
    }
    // longest spectrum and the bin window (first / last peak of each spectrum)
    int maxlen = 0, lok = 0x7fffffff, hik = -1;
    for (int64_t s = s0 + tid; s < s1; s += SG_BLOCK) {
      const int64_t a = v.spec_off[s], e = v.spec_off[s + 1];
      if (e > a) {
        maxlen = max(maxlen, (int)min<int64_t>(e - a, 0x7fffffff));
        lok = min(lok, q_window_key(v.mz[a], P));
        hik = max(hik, q_window_key(v.mz[e - 1], P));
      }
    }
    atomicMax(&red[0], maxlen);
    atomicMin(&red[1], lok);
    atomicMax(&red[2], hik);
    __syncthreads();
    if (tid == 0) {
      const int64_t P_c = v.spec_off[s1] - M.p0;
      maxlen = red[0];
      lok = red[1];
      hik = red[2];
      if (hik < lok) { lok = 0; hik = 0; }  // every spectrum empty: an empty window
      M.sb = max(1, min(SG_SB, Q_LCAP / max(maxlen, 1)));
      M.nb = (n + M.sb - 1) / M.sb;
      M.lo_w = lok >> 6;
      M.nw = (hik >> 6) - M.lo_w + 1;
      const bool fits = enabled && P.apply_quorum && P.n_words <= BM_WMAX && n <= 65535 && maxlen <= Q_LCAP &&
                        P_c < (int64_t(1) << 31);
      const int64_t W = (int64_t)M.nw * 64;
      const int64_t bytes = seg_align((int64_t)M.nb * W) + seg_align((int64_t)M.nw * 8) + seg_align((int64_t)M.nw * 4);
      const int64_t base = fits ? seg_alloc(bump, bytes, cap) : -1;
      const int ntl = (M.nw + Q_TILEW - 1) / Q_TILEW;
      M.task0 = base >= 0 ? atomicAdd(n_tasks, M.nb) : 0;
      M.tile0 = base >= 0 ? atomicAdd(n_tiles, ntl) : 0;
      if (base < 0 || M.task0 + M.nb > task_cap || M.tile0 + ntl > tile_cap) {
        M.state = kQNoFit;
      } else {
        M.state = kQOk;
        M.rows = base;
        M.kbits = base + seg_align((int64_t)M.nb * W);
        M.kpre = M.kbits + seg_align((int64_t)M.nw * 8);
      }
      sM = M;
    }
    __syncthreads();
    M = sM;
    if (M.state == kQOk) {
      for (int k = tid; k < M.nb; k += SG_BLOCK) task_cl[M.task0 + k] = i;
      const int ntl = (M.nw + Q_TILEW - 1) / Q_TILEW;
      for (int k = tid; k < ntl; k += SG_BLOCK) tile_cl[M.tile0 + k] = i;
    }
    if (tid == 0) meta[i] = M;
    __syncthreads();
  }
}

// block b's spectrum offsets (relative to the cluster's first peak) into LDS;
// returns the block's spectrum count
__device__ __forceinline__ int q_block_offsets(const CsrView& v, const QMeta& M, int b, int32_t* soff) {
  const int64_t s0 = v.cluster_off[M.c] + (int64_t)b * M.sb;
  const int nsb = min(M.n - b * M.sb, M.sb);
  for (int j = threadIdx.x; j <= nsb; j += SG_BLOCK) soff[j] = (int32_t)(v.spec_off[s0 + j] - M.p0);
  return nsb;
}

struct QTallySmem {
  unsigned long long bits[BM_WMAX];
  uint16_t lpre[BM_WMAX];
  uint32_t lcnt[Q_LCAP / 4];  // u8 spectrum counts of the block's occupied bins, four per word
  int32_t soff[SG_SB + 1];
  int votes[2 * (SG_BLOCK / kWave)];
  int tmp[SG_BLOCK / kWave + 1];
};

// tally: one workgroup per (cluster, block) task -- rows[b][bin] = spectra of the
// block whose last peak of that bin exists (0..sb)
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_tally_kernel(CsrView v, BinMeanParams P, QMeta* meta,
                                                                    char* arena, const int32_t* task_cl,
                                                                    const int32_t* n_tasks, int32_t task_cap) {
  __shared__ QTallySmem L;
  const int tid = threadIdx.x;
  const int32_t nt = min(*n_tasks, task_cap);
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = task_cl[t];
    const QMeta M = meta[i];
    if (M.state != kQOk) continue;  // uniform
    const int b = t - M.task0;
    const int32_t base = M.lo_w * 64, W = M.nw * 64;
    for (int w = tid; w < M.nw; w += SG_BLOCK) L.bits[w] = 0ull;
    const int nsb = q_block_offsets(v, M, b, L.soff);
    lds_barrier();
    int oob = 0;
    int bad = walk_block<false>(v, P, M.p0, nsb, L.soff, [&](int64_t, int32_t key, bool last, int, double, double) {
      const uint32_t r = (uint32_t)(key - base);
      if (r >= (uint32_t)W) oob = 1;  // outside the window: only an unsorted spectrum does that
      else if (last) atomicOr(&L.bits[r >> 6], 1ull << (r & 63));
    });
    if (block_any<SG_BLOCK, true>(bad | oob, L.votes, 0)) {
      if (tid == 0) atomicOr(&meta[i].state, kQBad);
      __syncthreads();
      continue;
    }
    const int Db = bitmap_prefix<SG_BLOCK, uint16_t, true>(L.bits, L.lpre, M.nw, L.tmp);  // <= sb * maxlen <= Q_LCAP
    for (int w = tid; w < (Db + 3) / 4; w += SG_BLOCK) L.lcnt[w] = 0u;
    lds_barrier();
    walk_block<false>(v, P, M.p0, nsb, L.soff, [&](int64_t, int32_t key, bool last, int, double, double) {
      if (last) {
        const int r = bitmap_rank(L.bits, L.lpre, (int64_t)(key - base));
        atomicAdd(&L.lcnt[r >> 2], 1u << ((r & 3) * 8));
      }
    });
    lds_barrier();
    // the dense row, 16 bins per store
    uint4* row = reinterpret_cast<uint4*>(arena + M.rows + (int64_t)b * W);
    for (int c16 = tid; c16 < M.nw * 4; c16 += SG_BLOCK) {
      const int w = c16 >> 2, sh = (c16 & 3) * 16;
      const unsigned long long word = L.bits[w];
      uint32_t x = (uint32_t)(word >> sh) & 0xFFFFu;
      int r = (int)L.lpre[w] + __popcll(word & ((1ull << sh) - 1ull));
      unsigned long long lo = 0ull, hi = 0ull;
      while (x) {
        const int j = __ffs((int)x) - 1;
        x &= x - 1u;
        const unsigned long long cn = (L.lcnt[r >> 2] >> ((r & 3) * 8)) & 0xFFu;
        if (j < 8) lo |= cn << (j * 8);
        else hi |= cn << ((j - 8) * 8);
        ++r;
      }
      row[c16] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
    }
    __syncthreads();  // the LDS is reused by the next task
  }
}

// count: one workgroup per (cluster, Q_TILEW words) tile; wave per bitmap word,
// lane per bin: the column sum over the blocks' rows against the quorum
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_count_kernel(const QMeta* meta, char* arena,
                                                                    const int32_t* tile_cl, const int32_t* n_tiles,
                                                                    int32_t tile_cap) {
  constexpr int U = 8;  // row loads in flight per lane
  const int lane = lane_id(), wid = wave_id();
  const int32_t nt = min(*n_tiles, tile_cap);
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = tile_cl[t];
    const QMeta M = meta[i];
    if (M.state != kQOk) continue;
    const int64_t W = (int64_t)M.nw * 64;
    const uint32_t quorum = (uint32_t)((double)M.n * 0.25) + 1u;  // binning.py:181-183
    for (int w = (t - M.tile0) * Q_TILEW + wid; w < min(M.nw, (t - M.tile0 + 1) * Q_TILEW); w += SG_BLOCK / kWave) {
      const uint8_t* col = reinterpret_cast<const uint8_t*>(arena + M.rows) + w * 64 + lane;
      uint32_t tot = 0;
      for (int b0 = 0; b0 < M.nb; b0 += U) {
        uint32_t x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = b0 + u < M.nb ? col[(int64_t)(b0 + u) * W] : 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) tot += x[u];
      }
      const unsigned long long kept = __ballot(tot >= quorum);
      if (lane == 0) reinterpret_cast<unsigned long long*>(arena + M.kbits)[w] = kept;
    }
  }
}

// plan: one workgroup per cluster -- kept ranks, the value table and the fold units
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_plan_kernel(const int32_t* n_list, QMeta* meta, char* arena,
                                                                   unsigned long long* bump, int64_t cap,
                                                                   int32_t* unit_cl, int32_t* n_units,
                                                                   int32_t unit_cap) {
  __shared__ int tmp[SG_BLOCK / kWave + 1];
  __shared__ QMeta sM;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    QMeta M = meta[i];
    if (M.state != kQOk) continue;  // uniform
    const unsigned long long* kb = reinterpret_cast<const unsigned long long*>(arena + M.kbits);
    uint32_t* kp = reinterpret_cast<uint32_t*>(arena + M.kpre);
    const int K = bitmap_prefix<SG_BLOCK, uint32_t>(kb, kp, M.nw, tmp);
    if (tid == 0) {
      M.K = K;
      if (K > Q_KCAP) {
        M.state = kQNoFit;
      } else if (K > 0) {
        const int64_t bytes = seg_align((int64_t)K * M.n * 16) + seg_align((int64_t)K * M.nb * 8) +
                              seg_align((int64_t)K * 16);
        const int64_t base = seg_alloc(bump, bytes, cap);
        M.unit0 = base >= 0 ? atomicAdd(n_units, K) : 0;
        if (base < 0 || M.unit0 + K > unit_cap) {
          M.state = kQNoFit;
        } else {
          M.vals = base;
          M.pbits = M.vals + seg_align((int64_t)K * M.n * 16);
          M.res = M.pbits + seg_align((int64_t)K * M.nb * 8);
        }
      }
      sM = M;
    }
    __syncthreads();
    M = sM;
    if (M.state == kQOk)
      for (int k = tid; k < M.K; k += SG_BLOCK) unit_cl[M.unit0 + k] = i;
    if (tid == 0) meta[i] = M;
    __syncthreads();
  }
}

struct QPlaceSmem {
  unsigned long long kb[BM_WMAX];
  uint16_t kp[BM_WMAX];
  unsigned long long lmask[Q_KCAP];  // bit s: spectrum s of the block has kept bin k
  int32_t soff[SG_SB + 1];
};

// place: one workgroup per (cluster, block) task -- V[k][s] and P[k][b]
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_place_kernel(CsrView v, BinMeanParams P, const QMeta* meta,
                                                                    char* arena, const int32_t* task_cl,
                                                                    const int32_t* n_tasks, int32_t task_cap) {
  __shared__ QPlaceSmem L;
  const int tid = threadIdx.x;
  const int32_t nt = min(*n_tasks, task_cap);
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = task_cl[t];
    const QMeta M = meta[i];
    if (M.state != kQOk || M.K == 0) continue;  // uniform
    const int b = t - M.task0;
    const int32_t base = M.lo_w * 64, W = M.nw * 64;
    const unsigned long long* kb = reinterpret_cast<const unsigned long long*>(arena + M.kbits);
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(arena + M.kpre);
    for (int w = tid; w < M.nw; w += SG_BLOCK) {
      L.kb[w] = kb[w];
      L.kp[w] = (uint16_t)kp[w];  // K <= Q_KCAP
    }
    for (int k = tid; k < M.K; k += SG_BLOCK) L.lmask[k] = 0ull;
    const int nsb = q_block_offsets(v, M, b, L.soff);
    __syncthreads();
    double2* V = reinterpret_cast<double2*>(arena + M.vals);
    const int sb0 = b * M.sb;
    walk_block<true>(v, P, M.p0, nsb, L.soff, [&](int64_t, int32_t key, bool last, int s, double m, double it) {
      const uint32_t r = (uint32_t)(key - base);
      if (!last || r >= (uint32_t)W) return;
      const unsigned long long word = L.kb[r >> 6];
      if (!((word >> (r & 63)) & 1ull)) return;  // a bin under the quorum
      const int k = (int)L.kp[r >> 6] + __popcll(word & ((1ull << (r & 63)) - 1ull));
      V[(int64_t)k * M.n + sb0 + s] = make_double2(m, it);
      atomicOr(&L.lmask[k], 1ull << s);
    });
    lds_barrier();
    unsigned long long* Pb = reinterpret_cast<unsigned long long*>(arena + M.pbits);
    for (int k = tid; k < M.K; k += SG_BLOCK) Pb[(int64_t)k * M.nb + b] = L.lmask[k];
    __syncthreads();  // the LDS is reused by the next task
  }
}

// fold: one wave per kept bin (grid-stride over the units) -- block by block, the
// lanes load the block's sb entries of V[k] at once (the next block's while this
// one is folded) and the present ones are folded in spectrum order by broadcast
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_fold_kernel(const QMeta* meta, char* arena,
                                                                   const int32_t* unit_cl, const int32_t* n_units,
                                                                   int32_t unit_cap) {
  constexpr int NW = SG_BLOCK / kWave;
  const int lane = lane_id();
  const int32_t nu = min(*n_units, unit_cap);
  for (int32_t u = blockIdx.x * NW + wave_id(); u < nu; u += gridDim.x * NW) {  // uniform per wave
    const int i = unit_cl[u];
    const QMeta M = meta[i];
    const int k = u - M.unit0;
    const double2* Vk = reinterpret_cast<const double2*>(arena + M.vals) + (int64_t)k * M.n;
    const unsigned long long* Pk = reinterpret_cast<const unsigned long long*>(arena + M.pbits) + (int64_t)k * M.nb;
    const int last_s = M.n - 1;
    double2 x = Vk[min(lane, last_s)];
    unsigned long long mask = Pk[0];
    float si = 0.0f, sm = 0.0f;
    uint32_t cnt = 0;
    for (int b = 0; b < M.nb; ++b) {
      const int bn = min(b + 1, M.nb - 1);
      const double2 xn = Vk[min(bn * M.sb + lane, last_s)];  // (entries of absent spectra are never used)
      const unsigned long long mn = Pk[bn];
      unsigned long long m = uniform_u64(mask);
      cnt += (uint32_t)__popcll(m);
      while (m) {
        const int j = __builtin_ctzll(m);
        m &= m - 1ull;
        const double xi = readlane_f64(x.y, j), xm = readlane_f64(x.x, j);
        si = (float)((double)si + xi);
        sm = (float)((double)sm + xm);
      }
      x = xn;
      mask = mn;
    }
    if (lane == 0) {
      const double cn = (double)cnt;  // >= the quorum
      reinterpret_cast<double2*>(arena + M.res)[k] =
          make_double2(sm == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)sm / cn, (double)si / cn);
    }
  }
}

// emit: one workgroup per cluster -- kept bins whose intensity mean is not NaN,
// in bin order (binning.py:209-222); count, charge, np.mean (:224).  Clusters
// that did not fit go to the segmented fold's list, unsorted / NaN ones to the
// global kernel's.
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_emit_kernel(CsrView v, PeaksOut out, double* prec_out,
                                                                   int32_t* charge_out, int32_t* status,
                                                                   const int32_t* n_list, const QMeta* meta,
                                                                   char* arena, int32_t* seg_list, int32_t* n_seg,
                                                                   int32_t* glist, int32_t* n_glist) {
  __shared__ uint32_t tmp[SG_BLOCK / kWave + 1];
  __shared__ int64_t leaf_lo[SG_MAXLEAF], leaf_len[SG_MAXLEAF];
  __shared__ double leaf_sum[SG_MAXLEAF];
  __shared__ int nleaf;
  constexpr int PER = Q_KCAP / SG_BLOCK;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const QMeta M = meta[i];
    if (M.state != kQOk) {  // uniform
      if (tid == 0) {
        if (M.state == kQBad) glist[atomicAdd(n_glist, 1)] = (int32_t)M.c;
        if (M.state == kQNoFit) seg_list[atomicAdd(n_seg, 1)] = (int32_t)M.c;
      }
      continue;
    }
    const double2* res = reinterpret_cast<const double2*>(arena + M.res);
    const int k0 = tid * PER;
    double2 r[PER];
    uint32_t local = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      r[q] = k0 + q < M.K ? res[k0 + q] : make_double2(0.0, __longlong_as_double(0x7ff8000000000000ll));
      local += isnan(r[q].y) ? 0u : 1u;
    }
    uint32_t total;
    uint32_t o = block_exclusive_scan<SG_BLOCK, uint32_t>(local, tmp, total);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      if (!isnan(r[q].y)) {
        out.mz[M.p0 + o] = r[q].x;
        out.inten[M.p0 + o] = r[q].y;
        ++o;
      }
    }
    const int64_t s0 = v.cluster_off[M.c];
    const double pm = seg_pw_mean(v.prec_mz + s0, M.n, leaf_lo, leaf_len, leaf_sum, &nleaf);  // np.mean (binning.py:224)
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
