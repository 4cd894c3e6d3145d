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
constexpr int QF_LONG = 1024;       // clusters of at least this many spectra fold first (the longest chains)
enum : int32_t { kQOk = 0, kQBad = 1, kQNoFit = 2, kQDone = 3 };

struct QMeta {
  int64_t c, p0;
  int32_t n, nb, sb, state;      // spectra, blocks, spectra per block, kQ*
  int32_t lo_w, nw, task0, tile0;  // window words [lo_w, lo_w + nw); first block task, first count tile
  int32_t unit0, K, G, pad;      // first fold unit, kept bins, 64-bin groups of them (the fold units)
  int64_t rows, kbits, kpre;     // arena offsets: rows[b][bin] u8, kept bitmap (nw u64), its prefix (nw u32)
  int64_t vals, pres, res;       // V[s][k] (m/z, intensity; rows of 64 G), presence P[g][s] u64, res[k]
  double prec;                   // np.mean of the precursors (binning.py:224)
};

// OR over the wave, every lane gets it
__device__ __forceinline__ unsigned long long wave_or_u64(unsigned long long x) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) x |= __shfl_xor(x, o, kWave);
  return x;
}

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
  __shared__ PwSmem pws;
  const int tid = threadIdx.x;
  const int32_t nl = *n_list;
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = list[i];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int n = (int)(s1 - s0);
    const int32_t z0 = v.charge[s0];
    // the charges, the longest spectrum and the bin window (first / last peak of each
    // spectrum) in ONE pass, QS_U spectra per thread per round with their loads issued
    // together: a 5,000-spectrum cluster is 3 rounds of two dependent loads (the charges
    // used to take a pass of their own before it, and the window pass 4 spectra a round)
    constexpr int QS_U = 8;
    int mixed = 0, maxlen = 0, lok = 0x7fffffff, hik = -1;
    if (tid == 0) { red[0] = 0; red[1] = 0x7fffffff; red[2] = -1; }
    for (int64_t r0 = s0 + tid; r0 < s1; r0 += QS_U * SG_BLOCK) {
      int64_t a[QS_U], e[QS_U];
      int32_t z[QS_U];
#pragma unroll
      for (int u = 0; u < QS_U; ++u) {
        const int64_t sp = min(r0 + u * SG_BLOCK, s1 - 1);  // (clamped: a repeat)
        a[u] = v.spec_off[sp];
        e[u] = v.spec_off[sp + 1];
        z[u] = v.charge[sp];
      }
      double mf[QS_U], ml[QS_U];
#pragma unroll
      for (int u = 0; u < QS_U; ++u) {
        mf[u] = e[u] > a[u] ? v.mz[a[u]] : 0.0;
        ml[u] = e[u] > a[u] ? v.mz[e[u] - 1] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < QS_U; ++u) {
        mixed |= z[u] != z0;
        if (r0 + u * SG_BLOCK < s1 && e[u] > a[u]) {
          maxlen = max(maxlen, (int)min<int64_t>(e[u] - a[u], 0x7fffffff));
          lok = min(lok, q_window_key(mf[u], P));
          hik = max(hik, q_window_key(ml[u], P));
        }
      }
    }
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
    atomicMax(&red[0], maxlen);
    atomicMin(&red[1], lok);
    atomicMax(&red[2], hik);
    const double pm = seg_pw_mean(v.prec_mz + s0, n, pws);  // (barriers inside)
    if (tid == 0) {
      M.prec = pm;
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
                        P_c < (int64_t(1) << 28);
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

// bit i of a 16-bit value -> bit 4 i
__device__ __forceinline__ unsigned long long spread4(uint32_t x) {
  unsigned long long y = x & 0xFFFFu;
  y = (y | (y << 24)) & 0x000000FF000000FFull;
  y = (y | (y << 12)) & 0x000F000F000F000Full;
  y = (y | (y << 6)) & 0x0303030303030303ull;
  y = (y | (y << 3)) & 0x1111111111111111ull;
  return y;
}

// count: one workgroup per (cluster, Q_TILEW words) tile; a wave per 4 bitmap
// words, 4 bins per lane (u32 row loads): the column sums over the blocks' rows
// against the quorum, kept words assembled from the four ballots
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_count_kernel(const QMeta* meta, char* arena,
                                                                    const int32_t* tile_cl, const int32_t* n_tiles,
                                                                    int32_t tile_cap) {
  constexpr int U = 8;  // row loads in flight per lane
  static_assert(Q_TILEW == 4 * (SG_BLOCK / kWave), "a wave per 4 words");
  const int lane = lane_id(), wid = wave_id();
  const int32_t nt = min(*n_tiles, tile_cap);
  for (int32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const int i = tile_cl[t];
    const QMeta M = meta[i];
    if (M.state != kQOk) continue;
    const int w0 = (t - M.tile0) * Q_TILEW + 4 * wid;  // this wave's first word
    if (w0 >= M.nw) continue;                          // uniform per wave
    const int64_t W4 = (int64_t)M.nw * 16;              // row length in u32
    const uint32_t quorum = (uint32_t)((double)M.n * 0.25) + 1u;  // binning.py:181-183
    const int q4 = w0 * 16 + lane;                      // this lane's u32 (bins 4 q4 .. 4 q4 + 3)
    const bool inw = q4 < W4;
    const uint32_t* col = reinterpret_cast<const uint32_t*>(arena + M.rows) + (inw ? q4 : 0);
    uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
    for (int b0 = 0; b0 < M.nb; b0 += U) {
      uint32_t x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) x[u] = col[(int64_t)min(b0 + u, M.nb - 1) * W4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t y = b0 + u < M.nb ? x[u] : 0u;
        t0 += y & 0xFFu;
        t1 += (y >> 8) & 0xFFu;
        t2 += (y >> 16) & 0xFFu;
        t3 += y >> 24;
      }
    }
    const unsigned long long k0 = __ballot(inw && t0 >= quorum), k1 = __ballot(inw && t1 >= quorum);
    const unsigned long long k2 = __ballot(inw && t2 >= quorum), k3 = __ballot(inw && t3 >= quorum);
    if (lane < 4 && w0 + lane < M.nw) {  // word w0 + lane: lanes 16 lane .. 16 lane + 15
      const int sh = 16 * lane;
      reinterpret_cast<unsigned long long*>(arena + M.kbits)[w0 + lane] =
          spread4((uint32_t)(k0 >> sh)) | (spread4((uint32_t)(k1 >> sh)) << 1) |
          (spread4((uint32_t)(k2 >> sh)) << 2) | (spread4((uint32_t)(k3 >> sh)) << 3);
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
      M.G = (K + 63) / 64;
      if (K > Q_KCAP) {
        M.state = kQNoFit;
      } else if (K > 0) {
        const int64_t Kp = (int64_t)M.G * 64;
        const int64_t bytes = seg_align((int64_t)M.n * Kp * 16) + seg_align((int64_t)M.G * M.n * 8) +
                              seg_align((int64_t)K * 16);
        const int64_t base = seg_alloc(bump, bytes, cap);
        // long chains first (the front half of unit_cl), the rest from the back
        const bool lng = M.n >= QF_LONG;
        M.unit0 = base >= 0 ? atomicAdd(&n_units[lng ? 0 : 1], M.G) : 0;
        if (base < 0 || M.unit0 + M.G > (lng ? unit_cap / 2 : unit_cap - unit_cap / 2)) {
          M.state = kQNoFit;
        } else {
          M.vals = base;
          M.pres = M.vals + seg_align((int64_t)M.n * Kp * 16);
          M.res = M.pres + seg_align((int64_t)M.G * M.n * 8);
        }
      }
      sM = M;
    }
    __syncthreads();
    M = sM;
    if (M.state == kQOk)
      for (int g = tid; g < M.G; g += SG_BLOCK) unit_cl[M.n >= QF_LONG ? M.unit0 + g : unit_cap - 1 - (M.unit0 + g)] = i;
    if (tid == 0) meta[i] = M;
    __syncthreads();
  }
}

struct QPlaceSmem {
  unsigned long long kb[BM_WMAX];
  uint16_t kp[BM_WMAX];
  unsigned long long lp[SG_SB * (Q_KCAP / 64)];  // presence of spectrum s in group g: lp[s * G + g]
  int32_t soff[SG_SB + 1];
};

// place: one workgroup per (cluster, block) task -- V[s][k] (a spectrum's kept
// peaks are consecutive k: contiguous stores) and P[g][s]
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
    const int64_t Kp = (int64_t)M.G * 64;
    const unsigned long long* kb = reinterpret_cast<const unsigned long long*>(arena + M.kbits);
    const uint32_t* kp = reinterpret_cast<const uint32_t*>(arena + M.kpre);
    for (int w = tid; w < M.nw; w += SG_BLOCK) {
      L.kb[w] = kb[w];
      L.kp[w] = (uint16_t)kp[w];  // K <= Q_KCAP
    }
    const int nsb = q_block_offsets(v, M, b, L.soff);
    for (int e = tid; e < nsb * M.G; e += SG_BLOCK) L.lp[e] = 0ull;
    __syncthreads();
    double2* V = reinterpret_cast<double2*>(arena + M.vals);
    const int sb0 = b * M.sb;
    // a chunk's kept peaks are ascending kept ranks of one spectrum, mostly in one
    // 64-bin group: their presence bits are ORed across the wave per group and
    // merged by one lane (only this wave writes spectrum s's words) -- 63 LDS
    // atomics on one word would serialise
    int my_g = -1;
    unsigned long long my_bit = 0ull;
    walk_block<true>(
        v, P, M.p0, nsb, L.soff,
        [&](int64_t, int32_t key, bool last, int s, double m, double it) {
          const uint32_t r = (uint32_t)(key - base);
          if (!last || r >= (uint32_t)W) return;
          const unsigned long long word = L.kb[r >> 6];
          if (!((word >> (r & 63)) & 1ull)) return;  // a bin under the quorum
          const int k = (int)L.kp[r >> 6] + __popcll(word & ((1ull << (r & 63)) - 1ull));
          V[(int64_t)(sb0 + s) * Kp + k] = make_double2(m, it);
          my_g = k >> 6;
          my_bit = 1ull << (k & 63);
        },
        [&](int s) {
          unsigned long long pending = __ballot(my_g >= 0);
          while (pending) {  // uniform
            const int l0 = __builtin_ctzll(pending);
            const int g = __builtin_amdgcn_readlane(my_g, l0);
            const bool sel = my_g == g;
            const unsigned long long w = wave_or_u64(sel ? my_bit : 0ull);
            if (lane_id() == l0) L.lp[s * M.G + g] |= w;
            pending &= ~__ballot(sel);
          }
          my_g = -1;
        });
    lds_barrier();
    unsigned long long* Pg = reinterpret_cast<unsigned long long*>(arena + M.pres);
    for (int e = tid; e < nsb * M.G; e += SG_BLOCK) {
      const int g = e / nsb, s = e - g * nsb;  // consecutive threads: consecutive spectra of one group
      Pg[(int64_t)g * M.n + sb0 + s] = L.lp[s * M.G + g];
    }
    __syncthreads();  // the LDS is reused by the next task
  }
}

// fold: one workgroup per 64-bin group of a cluster's kept bins (grid-stride over
// the units).  Lane j of wave 0 owns kept bin 64 g + j and runs its
// f32(f64(acc) + v) chain over the spectra in order (binning.py:198-199);
// waves 1..4 stream the rows V[s][64 g .. 64 g + 63] (1 KB each) and the presence
// words into an LDS ring with LDS-DMA loads, QF_NS - 1 stages of QF_TS spectra
// ahead, so the chain -- as long as the cluster -- never waits on HBM latency.
#ifndef SPX_QF_TS
#define SPX_QF_TS 16
#endif
#ifndef SPX_QF_NS
#define SPX_QF_NS 8
#endif
constexpr int QF_TS = SPX_QF_TS;             // spectra per stage
constexpr int QF_NS = SPX_QF_NS;             // ring stages (QF_NS x QF_TS KB of rows)
constexpr int QF_LOADERS = 4;                // loader waves
constexpr int QF_RPW = QF_TS / QF_LOADERS;   // rows per loader wave per stage
constexpr int QF_BLOCK = (QF_LOADERS + 1) * kWave;
static_assert(QF_TS % QF_LOADERS == 0 && 2 * QF_TS <= kWave, "rows split evenly; presence: 2 x u32 per spectrum");

struct QFoldSmem {
  double2 v[QF_NS][QF_TS][kWave];
  uint32_t p[QF_NS][kWave];  // presence words of the stage's spectra (lanes 0..2 QF_TS - 1)
};

__device__ __forceinline__ void q_glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}
__device__ __forceinline__ void q_glds4(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 4, 0, 0);
}

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt left open)
template <int N>
__device__ __forceinline__ void q_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | 0x0F70);
}
// at most `stages` stages of G loads each still in flight (past what vmcnt can
// count: wait for all)
template <int G, int K = 0>
__device__ __forceinline__ void q_wait_stages(int stages) {
  if constexpr (K * G < 64 && K <= 16) {
    if (stages == K) q_wait_vm<K * G>();
    else q_wait_stages<G, K + 1>(stages);
  } else {
    q_wait_vm<0>();
  }
}

__global__ __launch_bounds__(QF_BLOCK, 1) void bin_mean_q_fold_kernel(const QMeta* meta, char* arena,
                                                                      const int32_t* unit_cl, const int32_t* n_units,
                                                                      int32_t unit_cap) {
  __shared__ QFoldSmem L;
  const int lane = lane_id(), wid = wave_id();
  // the long-chain units first (front of unit_cl), then the others (from the back)
  const int32_t n_long = min(n_units[0], unit_cap / 2);
  const int32_t nu = n_long + min(n_units[1], unit_cap - unit_cap / 2);
  for (int32_t u = blockIdx.x; u < nu; u += gridDim.x) {
    const int32_t j = u < n_long ? u : u - n_long;
    const int i = unit_cl[u < n_long ? u : unit_cap - 1 - j];
    const QMeta M = meta[i];
    const int g = j - M.unit0;
    const int n = M.n;
    const int64_t Kp = (int64_t)M.G * 64;
    const int nst = (n + QF_TS - 1) / QF_TS;
    const double2* Vg = reinterpret_cast<const double2*>(arena + M.vals) + (int64_t)g * 64 + lane;
    const uint32_t* Pg = reinterpret_cast<const uint32_t*>(arena + M.pres) + (int64_t)g * n * 2;
    // loader wave w (1..4) issues rows w-1, w-1+4, ... of a stage; wave 1 also the
    // presence words (2 x u32 per spectrum: lanes 0..31; 32..63 repeat them)
    auto issue = [&](int st) __attribute__((always_inline)) {
      const int slot = st % QF_NS;
      const int sbase = st * QF_TS;
#pragma unroll
      for (int r = 0; r < QF_RPW; ++r) {
        const int row = (wid - 1) + r * QF_LOADERS;
        const int sp = min(sbase + row, n - 1);  // rows past the cluster: never folded
        q_glds16(Vg + (int64_t)sp * Kp, &L.v[slot][row][0]);
      }
      if (wid == 1) {
        const int sp = min(sbase + ((lane & 31) >> 1), n - 1);
        q_glds4(Pg + (int64_t)sp * 2 + (lane & 1), &L.p[slot][0]);
      }
    };
    if (wid > 0)
      for (int st = 0; st < min(QF_NS - 1, nst); ++st) issue(st);
    float si = 0.0f, sm = 0.0f;
    uint32_t cnt = 0;
    for (int t = 0; t < nst; ++t) {  // uniform
      if (wid > 0) {  // stage t landed: stages t+1 .. t+NS-2 may stay in flight
        const int ahead = min(QF_NS - 2, nst - 1 - t);
        if (wid == 1) q_wait_stages<QF_RPW + 1>(ahead);
        else q_wait_stages<QF_RPW>(ahead);
      }
      __builtin_amdgcn_s_barrier();
      if (wid > 0) {
        if (t + QF_NS - 1 < nst) issue(t + QF_NS - 1);  // into the slot folded in iteration t - 1
      } else {
        const int slot = t % QF_NS;
        const int steps = min(QF_TS, n - t * QF_TS);  // uniform
        // the stage's words and entries read first (stale ones past `steps` are
        // never used), then the chain with selects: no branch between LDS reads
        uint32_t pl[QF_TS], ph[QF_TS];
        double2 x[QF_TS];
#pragma unroll
        for (int j = 0; j < QF_TS; ++j) {
          pl[j] = L.p[slot][2 * j];
          ph[j] = L.p[slot][2 * j + 1];
          x[j] = L.v[slot][j][lane];
        }
#pragma unroll
        for (int j = 0; j < QF_TS; ++j) {
          const uint32_t w = lane < 32 ? pl[j] : ph[j];
          const bool pr = j < steps && ((w >> (lane & 31)) & 1u);
          const float ni = (float)((double)si + x[j].y);
          const float nm = (float)((double)sm + x[j].x);
          si = pr ? ni : si;
          sm = pr ? nm : sm;
          cnt += pr ? 1u : 0u;
        }
      }
    }
    if (wid == 0 && g * 64 + lane < M.K) {
      const double cn = (double)cnt;  // >= the quorum
      reinterpret_cast<double2*>(arena + M.res)[g * 64 + lane] =
          make_double2(sm == 0.0f ? __longlong_as_double(0x7ff8000000000000ll) : (double)sm / cn, (double)si / cn);
    }
    __syncthreads();  // the ring is reused by the next unit (every load has landed: vmcnt(0) above)
  }
}

// emit: one workgroup per cluster -- kept bins whose intensity mean is not NaN,
// in bin order (binning.py:209-222); count, charge, np.mean (:224, from setup).
// Clusters that did not fit go to the segmented fold's list, unsorted / NaN ones
// to the global kernel's.
__global__ __launch_bounds__(SG_BLOCK) void bin_mean_q_emit_kernel(CsrView v, PeaksOut out, double* prec_out,
                                                                   int32_t* charge_out, int32_t* status,
                                                                   const int32_t* n_list, const QMeta* meta,
                                                                   char* arena, int32_t* seg_list, int32_t* n_seg,
                                                                   int32_t* glist, int32_t* n_glist) {
  __shared__ uint32_t tmp[SG_BLOCK / kWave + 1];
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
    if (tid == 0) {
      out.count[M.c] = total;
      charge_out[M.c] = v.charge[v.cluster_off[M.c]];
      prec_out[M.c] = M.prec;
      status[M.c] = kOk;
    }
  }
}

}  // namespace spx
