// Gap-average consensus (reference: src/average_spectrum_clustering.py:26-103,
// average_spectrum; precursor helpers :106-148; semantics in SURVEY.md A.2 and
// oracle/np_oracle.py gap_average_cluster).
//
// The reference pools the cluster's peaks, argsorts them by m/z, splits where
// the sorted gap is >= mz_accuracy, keeps groups holding >= min_fraction*n
// peaks (the last two true groups merged: the ind_list[1:-1] loop, :79) and
// averages them through cumulative-sum differences, then applies a dynamic
// range filter.  A full segmented sort is not needed to reproduce that
// exactly: with buckets k = floor(mz / mz_accuracy),
//   * two consecutive sorted peaks in one bucket differ by < mz_accuracy unless
//     the bucket's own span reaches mz_accuracy (checked per bucket; such a
//     cluster is deferred, never approximated);
//   * the sorted gap between two consecutive occupied buckets is exactly
//     fl(min(next) - max(prev)) -- the same f64 subtraction np.diff performs.
// So group boundaries and group counts are exact (integer/bit-exact), and only
// the group sums differ from the reference's cumsum differences by rounding
// (within 1e-12 relative; the parity bar is 1e-5).  The sums are accumulated
// as 64-bit fixed point (scale 2^e per cluster from max|value| * #peaks), so
// LDS integer atomics make them order-independent and run-to-run deterministic.
//
//   1  block reduce: min/max m/z, max |intensity|, finiteness
//   2  bucket bitmap (ds_or_b64) -> exclusive popcount prefix -> slot ids
//   3  per peak: slot count, min and max m/z (u64 order keys, ds_min/max_u64)
//   4  per slot: in-bucket span check, gap flags, block scan -> group ids
//   5  per peak: fixed-point m/z and intensity sums per emitted group
//   6  per group: min_fraction filter, values, dynamic-range filter, ordered write
//
// n == 1 passes the spectrum through (original order) with only the dynamic
// range filter (:88-98).  Precursor m/z / charge / RT per cluster follow the
// CLI's --pepmass / --rt choices (:106-148, :190-195).
#include "spx_device.hpp"

// The stamps build leaves the gap-average kernels unstamped unless asked
// (-DSPX_STAMPS_GA): with stamp 0, the LDS kernel trips an "illegal VGPR to SGPR
// copy" in this compiler (ROCm 7.2), so build with -DSPX_GA_STAMP_MASK=0xFE
#if defined(SPX_STAMPS) && !defined(SPX_STAMPS_GA)
#define SPX_GA_STAMP(k) do { } while (0)
#else
#ifndef SPX_GA_STAMP_MASK
#define SPX_GA_STAMP_MASK 0xFF  // diagnostic builds: the stamps recorded
#endif
#define SPX_GA_STAMP(k)                                   \
  do {                                                    \
    if constexpr (((SPX_GA_STAMP_MASK) >> (k)) & 1) SPX_STAMP(k); \
  } while (0)
#endif

namespace spx {

struct GapParams {
  double mz_accuracy, dyn_range, min_fraction, proton;
  double bucket_w, inv_bucket_w;  // mz_accuracy (LDS path) or mz_accuracy/2 (global path)
  int32_t pepmass_mode;  // 0 lower_median, 1 naive_average, 2 neutral_average
  int32_t rt_mode;       // 0 median, 1 mass_lower_median
};


constexpr int GA_BLOCK = 512;  // 2 workgroups per CU (LDS): 16 waves
constexpr int GA_NW = GA_BLOCK / kWave;
#ifndef SPX_GA_UM
#define SPX_GA_UM 20
#endif
constexpr int GA_UM = SPX_GA_UM;  // m/z values per thread held in registers (10,240 per cluster: n <= 51 at ~200 peaks)
#ifndef SPX_GA_WMAXN
#define SPX_GA_WMAXN 65536  // the wide kernel hands clusters of more peaks than this to the giant pipeline (0: none)
#endif
// the giant intake (spx_gap_average, round 6): every cluster of more than GA_OWN_N peaks
// is registered up front and its pipeline runs on the call's second stream; those of more
// than GA_OWN_LO while its table has room (16,384 for all giants measured 15 ms on skewed
// configs[3] instead of 1.63: past the 256 records the global kernel takes them)
constexpr int64_t GA_OWN_N = 65536;
constexpr int64_t GA_OWN_LO = 32768;
#ifndef SPX_GA_WUM
#define SPX_GA_WUM 20
#endif
// the wide kernel's (40 spilled 135 VGPRs even at its 256-VGPR budget)
constexpr int GA_WUM = SPX_GA_WUM;
constexpr int GA_WMAX = 3584;  // 229,376 buckets (2,293 Da at 0.01)
constexpr int GA_DCAP = 1536;  // occupied buckets per cluster
static_assert(GA_WMAX % GA_BLOCK == 0, "the LDS bitmap is whole words per thread");

// Exclusive popcount prefix over ALL of an LDS bitmap of BLOCK * WPT u64 words
// (words past the cluster's range are zero): each thread's WPT contiguous words
// are read unconditionally (the reads pipeline: one wait, not one per word) --
// the 8*WPT-B lane stride is bank-conflict-free for odd WPT -- then one block
// scan and the u16 prefixes.  Returns the number of set bits.
template <int BLOCK, int WPT>
__device__ __forceinline__ int bitmap_prefix_fixed(const unsigned long long* bm, uint16_t* pref, int* tmp) {
  const int w0 = threadIdx.x * WPT;
  unsigned long long w[WPT];
#pragma unroll
  for (int k = 0; k < WPT; ++k) w[k] = bm[w0 + k];
  int local = 0;
#pragma unroll
  for (int k = 0; k < WPT; ++k) local += __popcll(w[k]);
  int total;
  int base = block_exclusive_scan<BLOCK, int, true>(local, tmp, total);
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    pref[w0 + k] = (uint16_t)base;
    base += __popcll(w[k]);
  }
  lds_barrier();
  return total;
}

template <class PrefixT>
struct GapState {
  unsigned long long* bitmap;
  PrefixT* wprefix;
  uint32_t* cnt;        // per slot count, later its emitted group id
  uint32_t* gcnt;       // per emitted group count
  uint64_t* kmin;       // per slot min m/z key, later group fixed-point m/z sum
  uint64_t* kmax;       // per slot max m/z key, later group fixed-point intensity sum
  int wcap, dcap;
  uint32_t* flags = nullptr;  // global scratch only: per emitted group, the non-finite classes it holds
};

template <int DCAP>
struct GapSmemT {
  unsigned long long bitmap[GA_WMAX];
  uint16_t wprefix[GA_WMAX];
  uint32_t cnt[DCAP];
  uint32_t gcnt[DCAP];
  uint64_t kmin[DCAP];
  uint64_t kmax[DCAP];
  int tmp[GA_BLOCK / kWave + 1];
  int votes[2 * GA_NW];
  double red[GA_BLOCK / kWave * 3];
  int prank[2 * GA_NW * kWave];  // per-wave partial precursor ranks (mass, RT); n > 64: the rank stage
  long long sel[4];              // n > 64: prec_select_block's picks
};
using GapSmem = GapSmemT<GA_DCAP>;
static_assert(sizeof(GapSmem::prank) >= GA_BLOCK * sizeof(double), "the rank stage fits the prank words");
static_assert(GA_BLOCK * sizeof(double) >= (264 + GA_BLOCK / 64 + 1) * 4, "the radix select's words fit the stage");
static_assert(GA_BLOCK >= 256, "one thread per radix bucket");
// The wide kernel (what the LDS kernel defers for its bucket cap: spectra of hundreds of
// peaks give clusters thousands of occupied 0.01-Da buckets): 4,608 slots, 147 KB of
// LDS, one workgroup per CU
constexpr int GA_WDCAP = 4608;

__device__ __forceinline__ double nan_d() { return __longlong_as_double(0x7ff8000000000000ll); }

// ------------------------------------------------------ precursor summary
struct PrecSummary {
  double pepmass, rt;
  int32_t charge, status;
};

// numpy-compatible "less" for argsort/median ranks: NaN sorts last.
__device__ __forceinline__ bool lt_nan_last(double a, double b) { return a < b || (!isnan(a) && isnan(b)); }

// Clusters of <= 64 spectra (every config's common case): lane i holds
// spectrum i's charge, neutral mass and RT, loaded once; ranks and sums walk
// the other lanes' values by readlane (uniform index) -- no memory traffic in
// the O(n^2) rank loops.  Same arithmetic and order as the general path below.
// Lane i's spectrum fields (one load each).
struct PrecLanes {
  int32_t z;
  double pm, rt;
};
__device__ __forceinline__ PrecLanes prec_lanes(const CsrView& v, int64_t s0, int64_t n) {
  const int lane = lane_id();
  const bool valid = lane < n;
  return PrecLanes{valid ? v.charge[s0 + lane] : 0, valid ? v.prec_mz[s0 + lane] : 0.0, valid ? v.rt[s0 + lane] : 0.0};
}

// Stable ranks of lane i's neutral mass and RT among the cluster's n <= 64
// spectra, counted over j = j0, j0 + dj, ... only: the LDS kernel splits the O(n^2)
// comparisons over its 8 waves (j0 = wave, dj = 8) and sums the partial ranks.
struct PrecRanks {
  int m, r;
};
__device__ __forceinline__ PrecRanks prec_ranks(const PrecLanes& pl, int n, const GapParams& P, int j0, int dj) {
  const int lane = lane_id();
  const double z = (double)pl.z;
  const double mi = pl.pm * z - z * P.proton;  // (m*c - c*H), no contraction
  const double ri = pl.rt;
  PrecRanks k{0, 0};
  for (int j = j0; j < n; j += dj) {
    const double mj = readlane_f64(mi, j);
    k.m += lt_nan_last(mj, mi) || (!lt_nan_last(mi, mj) && j < lane);
  }
  if (P.rt_mode == 0) {
    for (int j = j0; j < n; j += dj) {
      const double rj = readlane_f64(ri, j);
      k.r += lt_nan_last(rj, ri) || (!lt_nan_last(ri, rj) && j < lane);
    }
  }
  return k;
}

// ranks: the summed partial ranks, or nullptr to count them here
__device__ PrecSummary precursor_summary_wave(const PrecLanes& pl, int n, const GapParams& P,
                                              const PrecRanks* ranks = nullptr) {
  PrecSummary R;
  const int lane = lane_id();
  const double H = P.proton;
  const bool valid = lane < n;
  const int32_t zi = pl.z;
  const double z = (double)zi;
  const double pm = pl.pm;
  const double mi = pm * z - z * H;  // (m*c - c*H), no contraction
  const double ri = pl.rt;
  const PrecRanks K = ranks ? *ranks : prec_ranks(pl, n, P, 0, 1);
  // lower-median index of the neutral masses: rank == (n-1)//2
  const int want = (n - 1) / 2;
  const int rank = K.m;
  const unsigned long long hit = __ballot(valid && rank == want);
  const int lm = hit ? __ffsll((long long)hit) - 1 : 0;
  double rt_lo = 0.0, rt_hi = 0.0;
  if (P.rt_mode == 0) {  // np.median
    const int rr = K.r;
    const unsigned long long h1 = __ballot(valid && rr == (n - 1) / 2), h2 = __ballot(valid && rr == n / 2);
    rt_lo = readlane_f64(ri, __ffsll((long long)h1) - 1);
    rt_hi = readlane_f64(ri, __ffsll((long long)h2) - 1);
  }
  R.status = kOk;
  if (P.pepmass_mode == 0) {
    const int32_t zl = __builtin_amdgcn_readlane(zi, lm);
    R.pepmass = (readlane_f64(mi, lm) + (double)zl * H) / (double)zl;
    R.charge = zl;
  } else if (P.pepmass_mode == 1) {
    double s = 0.0;
    int mixed = 0;
    const int32_t z0 = __builtin_amdgcn_readlane(zi, 0);
    for (int i = 0; i < n; ++i) {
      s += readlane_f64(pm, i);
      mixed |= __builtin_amdgcn_readlane(zi, i) != z0;
    }
    R.pepmass = s / (double)n;
    R.charge = z0;
    if (mixed) R.status = kMixedCharge;
  } else {
    double sm = 0.0;
    int64_t sz = 0;
    for (int i = 0; i < n; ++i) {
      sm += readlane_f64(mi, i);
      sz += __builtin_amdgcn_readlane(zi, i);
    }
    const int32_t zz = (int32_t)rint((double)sz / (double)n);
    R.pepmass = (sm / (double)n + (double)zz * H) / (double)zz;
    R.charge = zz;
  }
  if (P.rt_mode == 1) {
    R.rt = readlane_f64(ri, lm);
  } else {
    R.rt = (n & 1) ? rt_lo : (0.0 + rt_lo + rt_hi) / 2.0;
    if (__ballot(valid && isnan(ri)) != 0ull) R.rt = nan_d();  // np.median: any NaN -> NaN
  }
  return R;
}

// Run by one whole wave.  Ranks are stable (ties by index), which is what
// numpy's argsort returns for n <= 16 and for tie-free input.
// sel (optional): the ranks' picks, computed block-wide by prec_select_block --
// sel[0] the lower-median mass index, sel[1] / sel[2] the RT ranks (n-1)//2 and n//2.
__device__ PrecSummary precursor_summary(const CsrView& v, int64_t s0, int64_t n, const GapParams& P,
                                         const long long* sel = nullptr) {
  if (n <= kWave) return precursor_summary_wave(prec_lanes(v, s0, n), (int)n, P);
  PrecSummary R;
  const int lane = lane_id();
  const double H = P.proton;
  auto mass = [&](int64_t i) {
    const double z = (double)v.charge[s0 + i];
    return v.prec_mz[s0 + i] * z - z * H;  // (m*c - c*H), no contraction
  };
  // lower-median index of the neutral masses: rank == (n-1)//2
  const int64_t want = (n - 1) / 2;
  int64_t lm = sel ? (int64_t)sel[0] : -1;
  for (int64_t i0 = 0; !sel && i0 < n; i0 += kWave) {
    const int64_t i = i0 + lane;
    int64_t rank = -1;
    if (i < n) {
      const double mi = mass(i);
      rank = 0;
      for (int64_t j = 0; j < n; ++j) {
        const double mj = mass(j);
        rank += lt_nan_last(mj, mi) || (!lt_nan_last(mi, mj) && j < i);
      }
    }
    const unsigned long long hit = __ballot(rank == want);
    if (hit && lm < 0) lm = i0 + __ffsll((long long)hit) - 1;
  }
  // median RT (np.median): middle element(s) of the sorted values
  double rt_lo = 0.0, rt_hi = 0.0;
  const int64_t k_lo = (n - 1) / 2, k_hi = n / 2;
  if (P.rt_mode == 0 && sel) {
    rt_lo = v.rt[s0 + sel[1]];
    rt_hi = v.rt[s0 + sel[2]];
  } else if (P.rt_mode == 0) {
    for (int64_t i0 = 0; i0 < n; i0 += kWave) {
      const int64_t i = i0 + lane;
      int64_t rank = -1;
      double ri = 0.0;
      if (i < n) {
        ri = v.rt[s0 + i];
        rank = 0;
        for (int64_t j = 0; j < n; ++j) {
          const double rj = v.rt[s0 + j];
          rank += lt_nan_last(rj, ri) || (!lt_nan_last(ri, rj) && j < i);
        }
      }
      const unsigned long long h1 = __ballot(rank == k_lo), h2 = __ballot(rank == k_hi);
      if (h1) rt_lo = __shfl(ri, __ffsll((long long)h1) - 1, kWave);
      if (h2) rt_hi = __shfl(ri, __ffsll((long long)h2) - 1, kWave);
    }
  }
  R.status = kOk;
  if (P.pepmass_mode == 0) {
    const int32_t z = v.charge[s0 + lm];
    R.pepmass = (mass(lm) + (double)z * H) / (double)z;
    R.charge = z;
  } else if (P.pepmass_mode == 1) {
    double s = 0.0;
    int mixed = 0;
    for (int64_t i = 0; i < n; ++i) {
      s += v.prec_mz[s0 + i];
      mixed |= v.charge[s0 + i] != v.charge[s0];
    }
    R.pepmass = s / (double)n;
    R.charge = v.charge[s0];
    if (mixed) R.status = kMixedCharge;
  } else {
    double sm = 0.0;
    int64_t sz = 0;
    for (int64_t i = 0; i < n; ++i) {
      sm += mass(i);
      sz += v.charge[s0 + i];
    }
    const int32_t z = (int32_t)rint((double)sz / (double)n);
    R.pepmass = (sm / (double)n + (double)z * H) / (double)z;
    R.charge = z;
  }
  if (P.rt_mode == 1) {
    R.rt = v.rt[s0 + lm];
  } else {
    R.rt = (n & 1) ? rt_lo : (0.0 + rt_lo + rt_hi) / 2.0;
    bool rt_nan = false;  // np.median: any NaN -> NaN (NaN ranks last, so it is rarely a middle pick)
    for (int64_t i0 = 0; i0 < n && !rt_nan; i0 += kWave)
      rt_nan = __ballot(i0 + lane < n && isnan(v.rt[s0 + (i0 + lane < n ? i0 + lane : 0)])) != 0ull;
    if (rt_nan) R.rt = nan_d();
  }
  return R;
}

// The O(n^2) stable ranks of precursor_summary for n > 64, spread over the whole
// block instead of one wave (the skewed law's n = 5,000 giants spent ~58 ms of a
// 78 ms batch in the one-wave loops): each thread ranks its i's against every j,
// the j's staged through `stage` (GA_BLOCK doubles of LDS).  Same comparisons, so
// the same picks: sel[0] = the lower-median mass index, sel[1] / sel[2] = the RT
// ranks (n-1)//2 and n//2 (rt_mode 0).  Ranks are unique (ties by index), so each
// pick has one writer.  Call with the whole block; ends with a barrier.
// lt_nan_last as an unsigned order: -0 and +0 equal, every NaN one key above +inf
__device__ __forceinline__ uint64_t prec_key(double x) {
  if (isnan(x)) return ~0ull;
  return f64_order_key(x == 0.0 ? 0.0 : x);
}

// The index whose stable rank (lt_nan_last, ties by index) is `want`, for large n:
// an 8-pass radix select over prec_key (8-bit digits, LDS histogram) finds the
// want-th smallest key K and how many of K's equal keys precede the pick, then one
// ordered scan over the K's finds it by index.  O(n) per pass instead of O(n^2):
// the same element as prec_select_block's rank loops.  ws: 320 words of LDS.
// Call with the whole block; every thread gets the index.
template <class F>
__device__ int64_t prec_radix_select(F value, int64_t n, int64_t want, uint32_t* ws) {
  const int tid = threadIdx.x;
  uint32_t* hist = ws;                                          // 256 counts
  unsigned long long* ctl = reinterpret_cast<unsigned long long*>(ws + 256);  // digit, rank left, pick
  int* tmp = reinterpret_cast<int*>(ws + 264);                  // GA_NW + 1 scan words
  uint64_t prefix = 0;
  int64_t rem = want;
  for (int shift = 56; shift >= 0; shift -= 8) {
    const uint64_t hmask = shift == 56 ? 0ull : (~0ull << (shift + 8));
    if (tid < 256) hist[tid] = 0u;
    __syncthreads();
    for (int64_t i = tid; i < n; i += GA_BLOCK) {
      const uint64_t k = prec_key(value(i));
      if ((k & hmask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid < kWave) {
      const uint32_t h0 = hist[4 * tid], h1 = hist[4 * tid + 1], h2 = hist[4 * tid + 2], h3 = hist[4 * tid + 3];
      const int64_t s = (int64_t)h0 + h1 + h2 + h3;
      const int64_t inc = wave_inclusive_sum<int64_t, false>(s);
      int64_t c = inc - s;
      if (c <= rem && rem < inc) {  // one lane: the digit is in its 4 bins
        int q = 0;
        if (rem >= c + h0) { c += h0; q = 1; }
        if (q == 1 && rem >= c + h1) { c += h1; q = 2; }
        if (q == 2 && rem >= c + h2) { c += h2; q = 3; }
        ctl[0] = (unsigned long long)(4 * tid + q);
        ctl[1] = (unsigned long long)(rem - c);
      }
    }
    __syncthreads();
    prefix |= (uint64_t)ctl[0] << shift;
    rem = (int64_t)ctl[1];
  }
  // K = prefix; the pick is the rem-th (0-based) element with key K in index order
  int64_t base = 0;
  for (int64_t i0 = 0; i0 < n && base <= rem; i0 += GA_BLOCK) {  // uniform
    const int64_t i = i0 + tid;
    const int f = i < n && prec_key(value(i)) == prefix;
    int tot;
    const int o = block_exclusive_scan<GA_BLOCK, int>(f, tmp, tot);
    if (f && base + o == rem) ctl[2] = (unsigned long long)i;
    base += tot;
  }
  __syncthreads();
  const int64_t pick = (int64_t)ctl[2];
  __syncthreads();  // ctl is reused by the next call
  return pick;
}

// Past this many spectra the precursor picks take the radix select
constexpr int64_t GA_RADIX_N = 512;

__device__ void prec_select_block(const CsrView& v, int64_t s0, int64_t n, const GapParams& P, double* stage,
                                  long long* sel) {
  const int tid = threadIdx.x;
  const double H = P.proton;
  if (n > GA_RADIX_N) {
    uint32_t* ws = reinterpret_cast<uint32_t*>(stage);
    const int64_t m = prec_radix_select([&](int64_t i) {
      const double z = (double)v.charge[s0 + i];
      return v.prec_mz[s0 + i] * z - z * H;  // (m*c - c*H), no contraction: precursor_summary's mass
    }, n, (n - 1) / 2, ws);
    int64_t r0 = 0, r1 = 0;
    if (P.rt_mode == 0) {
      auto rt = [&](int64_t i) { return v.rt[s0 + i]; };
      r0 = prec_radix_select(rt, n, (n - 1) / 2, ws);
      r1 = prec_radix_select(rt, n, n / 2, ws);
    }
    if (tid == 0) { sel[0] = m; sel[1] = r0; sel[2] = r1; }
    __syncthreads();
    return;
  }
  auto pass = [&](auto value, int64_t want0, int64_t want1, long long* out0, long long* out1) {
    for (int64_t i0 = 0; i0 < n; i0 += GA_BLOCK) {  // uniform
      const int64_t i = i0 + tid;
      const double xi = i < n ? value(i) : 0.0;
      int64_t rank = 0;
      for (int64_t j0 = 0; j0 < n; j0 += GA_BLOCK) {  // uniform
        __syncthreads();  // the previous chunk is consumed
        stage[tid] = j0 + tid < n ? value(j0 + tid) : 0.0;
        __syncthreads();
        const int m = (int)(n - j0 < GA_BLOCK ? n - j0 : GA_BLOCK);
        for (int k = 0; k < m; ++k) {
          const double xj = stage[k];
          rank += lt_nan_last(xj, xi) || (!lt_nan_last(xi, xj) && j0 + k < i);
        }
      }
      if (i < n && rank == want0) *out0 = i;
      if (out1 && i < n && rank == want1) *out1 = i;
    }
  };
  pass([&](int64_t i) {
    const double z = (double)v.charge[s0 + i];
    return v.prec_mz[s0 + i] * z - z * H;  // (m*c - c*H), no contraction: precursor_summary's mass
  }, (n - 1) / 2, -1, &sel[0], nullptr);
  if (P.rt_mode == 0) pass([&](int64_t i) { return v.rt[s0 + i]; }, (n - 1) / 2, n / 2, &sel[1], &sel[2]);
  __syncthreads();
}

// Every peak of [p0, p1) once, GA_BATCH loads in flight per thread (indices
// clamped, so each load is unconditional): f(k, mz[k], inten[k]).  kInten
// false skips the intensity loads (f sees 0.0).
constexpr int GA_BATCH = 8;
template <bool kInten, class F>
__device__ __forceinline__ void gap_peaks(const CsrView& v, int64_t p0, int64_t p1, F f) {
  for (int64_t k0 = p0 + threadIdx.x; k0 < p1; k0 += GA_BATCH * GA_BLOCK) {
    double m[GA_BATCH], it[GA_BATCH];
#pragma unroll
    for (int u = 0; u < GA_BATCH; ++u) {
      const int64_t k = k0 + (int64_t)u * GA_BLOCK;
      const int64_t kk = k < p1 ? k : p0;
      m[u] = v.mz[kk];
      it[u] = kInten ? v.inten[kk] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < GA_BATCH; ++u) {
      const int64_t k = k0 + (int64_t)u * GA_BLOCK;
      if (k < p1) f(k, m[u], it[u]);
    }
  }
}

// ------------------------------------------------- per-slot / per-group steps
// Shared by gap_body and the giant-cluster pipeline (kL: LDS state, LDS-only
// barriers; otherwise global scratch and full barriers).
template <bool kL>
__device__ __forceinline__ void gap_bar() {
  if constexpr (kL) lds_barrier();
  else __syncthreads();
}

// 4: gaps between consecutive occupied buckets -> emitted group per slot (cnt[d]
// becomes slot d's group, gcnt the group counts), the group-sum words zeroed.
// kOk with E groups, kDeferred (a bucket spans mz_accuracy) or kNoGap.
template <bool kL, class PrefixT>
__device__ __forceinline__ int32_t gap_groups(const GapState<PrefixT>& S, const GapParams& P, int D, int* tmp,
                                              int* votes, int& E) {
  const int tid = threadIdx.x;
  auto bar = []() __attribute__((always_inline)) { gap_bar<kL>(); };
  if constexpr (!kL) {
    // Global scratch: each thread's contiguous chunk of D / 512 slots (below) makes
    // every load a 64-line gather, one dependent round trip per slot (0.87 ms for a
    // 380k-slot giant).  Here: a coalesced sweep for the totals, then rounds of
    // 8 contiguous slots per thread with a running carry of the gaps before them.
    constexpr int CH = 8;
    const double acc = P.mz_accuracy;
    auto key = [&](const uint64_t* a, int d) { return f64_from_order_key(a[d]); };
    int my_gaps = 0, split = 0;
    for (int d = tid; d < D; d += GA_BLOCK) {
      const double mx = key(S.kmax, d);
      split |= (mx - key(S.kmin, d)) >= acc;  // a gap could hide inside the bucket
      if (d + 1 < D) my_gaps += (key(S.kmin, d + 1) - mx) >= acc;
    }
    if (block_any<GA_BLOCK, kL>(split, votes, 1)) return kDeferred;
    int m_gaps;
    block_exclusive_scan<GA_BLOCK, int, kL>(my_gaps, tmp, m_gaps);
    if (m_gaps == 0) return kNoGap;
    E = m_gaps >= 2 ? m_gaps : 2;
    int carry = 0;  // gaps before this round's first slot
    for (int r0 = 0; r0 < D; r0 += GA_BLOCK * CH) {  // uniform
      const int db = r0 + tid * CH;
      int f[CH], mine = 0;
#pragma unroll
      for (int k = 0; k < CH; ++k) {  // f[k]: a gap between slots d - 1 and d
        const int d = db + k;
        f[k] = d > 0 && d < D && (key(S.kmin, d) - key(S.kmax, d - 1)) >= acc;
        mine += f[k];
      }
      int tot;
      int g = carry + block_exclusive_scan<GA_BLOCK, int, kL>(mine, tmp, tot);
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int d = db + k;
        if (d < D) {
          g += f[k];
          const int eg = m_gaps >= 2 ? min(g, m_gaps - 1) : g;
          if (const uint32_t k_cnt = S.cnt[d]) atomicAdd(&S.gcnt[eg], k_cnt);  // giants count in pass 5
          S.cnt[d] = (uint32_t)eg;
        }
      }
      carry += tot;
    }
    bar();
    for (int e = tid; e < E; e += GA_BLOCK) { S.kmin[e] = 0ull; S.kmax[e] = 0ull; }
    bar();
    return kOk;
  }
  const int per = (D + GA_BLOCK - 1) / GA_BLOCK;
  const int d0 = tid * per;
  int my_gaps = 0, split = 0;
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
    if (d >= D) break;
    const double mn = f64_from_order_key(S.kmin[d]), mx = f64_from_order_key(S.kmax[d]);
    split |= (mx - mn) >= P.mz_accuracy;  // a gap could hide inside the bucket
    if (d + 1 < D) my_gaps += (f64_from_order_key(S.kmin[d + 1]) - mx) >= P.mz_accuracy;
  }
  if (block_any<GA_BLOCK, kL>(split, votes, 1)) return kDeferred;
  int m_gaps;
  int g = block_exclusive_scan<GA_BLOCK, int, kL>(my_gaps, tmp, m_gaps);
  if (m_gaps == 0) return kNoGap;
  E = m_gaps >= 2 ? m_gaps : 2;
  for (int j = 0; j < per; ++j) {
    const int d = d0 + j;
    if (d >= D) break;
    const int eg = m_gaps >= 2 ? min(g, m_gaps - 1) : g;
    atomicAdd(&S.gcnt[eg], S.cnt[d]);
    const bool gap_after = d + 1 < D &&
        (f64_from_order_key(S.kmin[d + 1]) - f64_from_order_key(S.kmax[d])) >= P.mz_accuracy;
    S.cnt[d] = (uint32_t)eg;
    g += gap_after;
  }
  bar();
  for (int e = tid; e < E; e += GA_BLOCK) { S.kmin[e] = 0ull; S.kmax[e] = 0ull; }
  bar();
  return kOk;
}

// 6: min_fraction filter, dynamic range, ordered output of cluster c's E groups
// (fixed-point sums at scales 2^sc_m / 2^sc_i): kOk or kEmpty.
template <bool kL, class PrefixT>
__device__ __forceinline__ int32_t gap_emit(const GapState<PrefixT>& S, const GapParams& P, int64_t c, int64_t n,
                                            int64_t N, int64_t p0, int E, int sc_m, int sc_i, const PeaksOut& out,
                                            int* tmp, double* red, int* votes) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const double min_len = P.min_fraction * (double)n;
  const int gper = (E + GA_BLOCK - 1) / GA_BLOCK;
  const int e0 = tid * gper;
  auto isum = [&](int e) -> double { return ldexp((double)(int64_t)S.kmax[e], -sc_i); };
  double gmax = -__longlong_as_double(0x7ff0000000000000ll);
  int anyg = 0;
  for (int j = 0; j < gper; ++j) {
    const int e = e0 + j;
    if (e < E && (double)S.gcnt[e] >= min_len) {
      gmax = fmax(gmax, isum(e) / (double)n);
      anyg = 1;
    }
  }
  gmax = wave_max_dpp(gmax);
  if (lane == 0) red[wid] = gmax;
  if (!block_any<GA_BLOCK, kL>(anyg, votes, 1)) return kEmpty;
  for (int w = 0; w < GA_BLOCK / kWave; ++w) gmax = fmax(gmax, red[w]);
  const double thr = gmax / P.dyn_range;
  int mine = 0;
  for (int j = 0; j < gper; ++j) {
    const int e = e0 + j;
    if (e < E && (double)S.gcnt[e] >= min_len && isum(e) / (double)n >= thr) ++mine;
  }
  int total;
  int o = block_exclusive_scan<GA_BLOCK, int, kL>(mine, tmp, total);
  for (int j = 0; j < gper; ++j) {
    const int e = e0 + j;
    if (e >= E || (double)S.gcnt[e] < min_len) continue;
    const double iv = isum(e) / (double)n;
    if (!(iv >= thr)) continue;
    SPX_GUARD(o < N, "gap out c=%ld o=%d N=%ld\n", (long)c, o, (long)N)
    out.mz[p0 + o] = ldexp((double)(int64_t)S.kmin[e], -sc_m) / (double)S.gcnt[e];
    out.inten[p0 + o] = iv;
    ++o;
  }
  if (tid == 0) out.count[c] = total;
  return kOk;
}

// --------------------------------------------------------------- the body
template <int UM, bool kDeferBig, class PrefixT>
__device__ int32_t gap_body(const CsrView& v, const GapParams& P, const GapState<PrefixT>& S, int64_t c,
                            const PeaksOut& out, int* tmp, double* red, int* votes, const PrecLanes* pl = nullptr,
                            int* prank = nullptr) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  // LDS state (the LDS kernel): barriers order LDS only, so register loads in
  // flight survive them; global-scratch state (the fallback kernel): full barriers
  constexpr bool kL = std::is_same<PrefixT, uint16_t>::value;
  auto bar = [&]() __attribute__((always_inline)) {
    if constexpr (kL) lds_barrier();
    else __syncthreads();
  };
  auto any = [&](int pred, int parity) __attribute__((always_inline)) {
    return block_any<GA_BLOCK, kL>(pred, votes, parity);
  };
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n = s1 - s0;
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1], N = p1 - p0;
  if (n == 0) return kNoGap;

  // The cluster's m/z values are read from HBM ONCE into registers when they
  // fit (<= UM per thread: 10,240 peaks); passes 2-3 run from registers, pass 2's bucket per peak is kept for
  // pass 3 and pass 3's slot for pass 5 (a u32 each).  Intensities are needed
  // only by passes 1 and 5 and are streamed there (8 loads in flight), so the
  // register budget holds twice as many peaks as m/z + intensity pairs would.
  // Larger clusters re-read per pass (the LDS kernel hands them to the wide one
  // before reading anything).
  if constexpr (kDeferBig) {
    // the LDS kernel: to the wide kernel unread.  Tested on an opaque copy of N: the
    // compiler must not learn that the streamed path below is dead (knowing it, it
    // schedules the register path into 4 spilled VGPRs: 16.7 -> 17.2 ms, configs[4])
    int64_t Nd = N;
    asm volatile("" : "+s"(Nd));
    if (Nd > (int64_t)UM * GA_BLOCK) return kDeferred;
  }
  const bool inreg = N <= (int64_t)UM * GA_BLOCK;  // uniform
  // hybrid (not the LDS kernel, which hands such clusters on): the first UM * BLOCK
  // peaks are register-resident and tagged like a small cluster's, only the tail is
  // re-read per pass (600-peak spectra: clusters of 10,800 to 30,000 peaks)
  constexpr bool kHy = !kDeferBig;
  const bool hyb = kHy && !inreg;  // uniform
  const bool regs = inreg || hyb;
  const int64_t ptail = p0 + (int64_t)UM * GA_BLOCK;
  double rm[UM];
  uint32_t tags[UM];  // per register peak: pass 2's bucket, then pass 3's slot (for pass 5)
#pragma unroll
  for (int q = 0; q < UM; ++q) tags[q] = 0u;
  if (regs) {
#pragma unroll
    for (int u0 = 0; u0 < UM; u0 += 8) {
      // a batch of rows no peak reaches is not loaded (uniform; the batch's loads stay
      // together)
      const bool live = (int64_t)u0 * GA_BLOCK < N;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = u0 + q;
        if (u < UM) {
          const int64_t k = p0 + (int64_t)u * GA_BLOCK + tid;
          const int64_t kk = k < p1 ? k : (N > 0 ? p0 : 0);
          if (live) rm[u] = N > 0 ? v.mz[kk] : 0.0;
          else rm[u] = 0.0;
        }
      }
    }
  }
  if (prank && pl && n <= kWave) {  // uniform: every wave's share of the precursor ranks
    const PrecRanks k = prec_ranks(*pl, (int)n, P, wid, GA_NW);
    prank[wid * kWave + lane] = k.m;
    prank[(GA_NW + wid) * kWave + lane] = k.r;
  }
  SPX_GA_STAMP(1);
  // f(m, it, tag, reg) over every peak; kInten false passes it = 0 and loads none;
  // reg (a std::bool_constant) is true for a register peak, whose tag is live
  auto peaks_g = [&](auto inten_c, auto tagout_c, auto f) __attribute__((always_inline)) {
    constexpr bool kInten = decltype(inten_c)::value;
    constexpr bool kTagOut = decltype(tagout_c)::value;
    if (regs) {
      if (N == 0) return;  // uniform: no peaks (and the batch may hold none to load)
#pragma unroll
      for (int u0 = 0; u0 < UM; u0 += 8) {
        if ((int64_t)u0 * GA_BLOCK >= N) break;  // uniform: no peak in rows u0.. (their tags stay 0)
        double itb[8];
        if constexpr (kInten) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int64_t k = p0 + (int64_t)(u0 + q) * GA_BLOCK + tid;
            itb[q] = (u0 + q < UM) ? v.inten[k < p1 ? k : p0] : 0.0;
          }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int u = u0 + q;
          if (u < UM) {
            const int64_t k = p0 + (int64_t)u * GA_BLOCK + tid;
            int32_t tag = (int32_t)tags[u];
            if (k < p1) f(rm[u], kInten ? itb[q] : 0.0, tag, std::true_type{});
            if constexpr (kTagOut) tags[u] = (uint32_t)tag;
          }
        }
      }
      if constexpr (kHy) {
        if (hyb) {
          gap_peaks<kInten>(v, ptail, p1, [&](int64_t, double m, double it) {
            int32_t tag = 0;
            f(m, it, tag, std::false_type{});
          });
        }
      }
    } else {
      gap_peaks<kInten>(v, p0, p1, [&](int64_t, double m, double it) {
        int32_t tag = 0;
        f(m, it, tag, std::false_type{});
      });
    }
  };
  auto peaks = [&](auto f) __attribute__((always_inline)) { peaks_g(std::true_type{}, std::false_type{}, f); };
  auto peaks_m_tag = [&](auto f) __attribute__((always_inline)) { peaks_g(std::false_type{}, std::true_type{}, f); };
  // passes 3 and 5 take a register peak's bucket / slot from its tag

  double lo = __longlong_as_double(0x7ff0000000000000ll), hi = -lo, imax = 0.0;
  int bad = 0;
  // The wide kernel (LDS state, m/z in registers, one workgroup per CU: its
  // latencies are not covered by a second workgroup): the intensities are needed
  // only for max |intensity| (pass 5's fixed-point scale) and their finiteness,
  // so they are streamed DURING the bucket pass instead of in a pass of their
  // own, and the bitmap is zeroed while the m/z loads land.  (In the LDS kernel,
  // two per CU, the same order measured 16.68 -> 17.18 ms: its pass-1 loads had
  // overlapped the m/z loads; profiles/r04_ab_gap_early.txt.)
  const bool early = kL && !kDeferBig && inreg && n > 1 && N >= 2;  // uniform
  if (early) {
#pragma unroll
    for (int k = 0; k < GA_WMAX / GA_BLOCK; ++k) S.bitmap[k * GA_BLOCK + tid] = 0ull;
    // 1a: m/z extrema and finiteness from registers
#pragma unroll
    for (int u = 0; u < UM; ++u) {
      if (p0 + (int64_t)u * GA_BLOCK + tid < p1) {
        bad |= !isfinite(rm[u]);
        lo = fmin(lo, rm[u]);
        hi = fmax(hi, rm[u]);
      }
    }
    if (any(bad, 0)) return kNonFinite;
  } else {
    // 1: extrema and finiteness
    peaks([&](double m, double it, int32_t& tag, auto) {
      bad |= !isfinite(m) || !isfinite(it);
      lo = fmin(lo, m);
      hi = fmax(hi, m);
      imax = fmax(imax, fabs(it));
    });
    if (any(bad, 0)) return kNonFinite;
  }
  SPX_GA_STAMP(2);

  if (n == 1) {
    // passthrough + dynamic-range filter on the raw spectrum (:88-98)
    double mx = -__longlong_as_double(0x7ff0000000000000ll);
    for (int64_t k = p0 + tid; k < p1; k += GA_BLOCK) mx = fmax(mx, v.inten[k]);
    mx = wave_max_dpp(mx);
    if (lane == 0) red[wid] = mx;
    bar();
    mx = red[0];
    for (int w = 1; w < GA_BLOCK / kWave; ++w) mx = fmax(mx, red[w]);
    bar();
    if (N == 0) return kEmpty;
    const double thr = mx / P.dyn_range;
    int64_t base = 0;
    for (int64_t k0 = p0; k0 < p1; k0 += GA_BLOCK) {
      const int64_t k = k0 + tid;
      const int keep = k < p1 && v.inten[k] >= thr;
      int tot;
      const int o = block_exclusive_scan<GA_BLOCK, int, kL>(keep, tmp, tot);
      if (keep) {
        out.mz[p0 + base + o] = v.mz[k];
        out.inten[p0 + base + o] = v.inten[k];
      }
      base += tot;
    }
    if (tid == 0) out.count[c] = base;
    return kOk;
  }
  if (N < 2) return kNoGap;  // np.diff of < 2 values is empty -> ind_list[0] IndexError

  lo = wave_min_dpp(lo);
  hi = wave_max_dpp(hi);
  imax = wave_max_dpp(imax);
  if (lane == 0) { red[wid] = lo; red[GA_NW + wid] = hi; red[2 * GA_NW + wid] = imax; }
  bar();
  for (int w = 0; w < GA_BLOCK / kWave; ++w) {
    lo = fmin(lo, red[w]);
    hi = fmax(hi, red[GA_NW + w]);
    imax = fmax(imax, red[2 * GA_NW + w]);
  }
  const int64_t kb = floor_div_exact(lo, P.bucket_w, P.inv_bucket_w);
  const int64_t ke = floor_div_exact(hi, P.bucket_w, P.inv_bucket_w);
  const int64_t nw = (ke - kb) / 64 + 1;
  if (nw > S.wcap) return kDeferred;

  // 2: occupied buckets
  if (early) {
    // 1b + 2: the buckets of the register m/z, one batch of intensity loads in
    // flight behind each batch of bucket work; the block's max |intensity| and
    // the intensities' finiteness ride the barrier before the prefix
    imax = 0.0;
#pragma unroll
    for (int u0 = 0; u0 < UM; u0 += 8) {
      double itb[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t k = p0 + (int64_t)(u0 + q) * GA_BLOCK + tid;
        itb[q] = (u0 + q < UM) ? v.inten[k < p1 ? k : p0] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = u0 + q;
        if (u < UM && p0 + (int64_t)u * GA_BLOCK + tid < p1) {
          const int64_t bk = floor_div_exact(rm[u], P.bucket_w, P.inv_bucket_w) - kb;
          tags[u] = (uint32_t)bk;
          atomicOr(&S.bitmap[bk >> 6], 1ull << (bk & 63));
        }
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = u0 + q;
        if (u < UM && p0 + (int64_t)u * GA_BLOCK + tid < p1) {
          bad |= !isfinite(itb[q]);
          imax = fmax(imax, fabs(itb[q]));
        }
      }
    }
    imax = wave_max_dpp(imax);
    const bool wbad = __ballot(bad) != 0ull;
    if (lane == 0) { red[2 * GA_NW + wid] = imax; votes[GA_NW + wid] = wbad; }
    bar();
    int nf = 0;
    for (int w = 0; w < GA_NW; ++w) {
      imax = fmax(imax, red[2 * GA_NW + w]);
      nf |= votes[GA_NW + w];
    }
    if (nf) return kNonFinite;
  } else {
    if constexpr (kL) {  // the whole LDS bitmap (the fixed-size prefix reads all of it)
#pragma unroll
      for (int k = 0; k < GA_WMAX / GA_BLOCK; ++k) S.bitmap[k * GA_BLOCK + tid] = 0ull;
    } else {
      for (int w = tid; w < nw; w += GA_BLOCK) S.bitmap[w] = 0ull;
    }
    bar();
    auto pass2 = [&](double m, double, int32_t& tag, auto) __attribute__((always_inline)) {
      const int64_t b = floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb;
      tag = (int32_t)b;
      SPX_GUARD(b >= 0 && b < nw * 64, "gap bitmap c=%ld b=%ld nw=%ld\n", (long)c, (long)b, (long)nw)
      atomicOr(&S.bitmap[b >> 6], 1ull << (b & 63));
    };
    if (regs && N > 0) {  // uniform
#pragma unroll
      for (int u0 = 0; u0 < UM; u0 += 8) {
        if ((int64_t)u0 * GA_BLOCK >= N) break;  // uniform
        // the reciprocal product's floor for all 8 rows (a lane past the cluster bins its
        // clamped copy of peak 0: never used); where it is not certain, one divide below
        uint32_t badm = 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int u = u0 + q;
          if (u < UM) {
            const double qv = rm[u] * P.inv_bucket_w;
            const double t = floor(qv);
            const double fr = qv - t;
            const bool sure = (fabs(qv) < kDivFastLimit) & (fr > kDivBand) & (fr < 1.0 - kDivBand);
            badm |= (uint32_t)!sure << q;
            tags[u] = (uint32_t)((int64_t)__double2int_rz(t) - kb);
          }
        }
        if (__builtin_expect(badm != 0u, 0)) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int u = u0 + q;
            if (u < UM && ((badm >> q) & 1u)) tags[u] = (uint32_t)((int64_t)floor(rm[u] / P.bucket_w) - kb);
          }
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int u = u0 + q;
          if (u < UM && p0 + (int64_t)u * GA_BLOCK + tid < p1) {
            const int32_t b = (int32_t)tags[u];
            SPX_GUARD(b >= 0 && b < nw * 64, "gap bitmap c=%ld b=%d nw=%ld\n", (long)c, b, (long)nw)
            atomicOr(&S.bitmap[b >> 6], 1ull << (b & 63));
          }
        }
      }
      if constexpr (kHy) {
        if (hyb) {
          gap_peaks<false>(v, ptail, p1, [&](int64_t, double m, double) {
            int32_t tag = 0;
            pass2(m, 0.0, tag, std::false_type{});
          });
        }
      }
    } else {
      peaks_m_tag(pass2);
    }
    bar();
  }
  int D;
  if constexpr (kL) D = bitmap_prefix_fixed<GA_BLOCK, GA_WMAX / GA_BLOCK>(S.bitmap, S.wprefix, tmp);
  else D = bitmap_prefix<GA_BLOCK, PrefixT, kL>(S.bitmap, S.wprefix, (int)nw, tmp);
  if (D > S.dcap) return kDeferred;
  SPX_GA_STAMP(3);
  for (int d = tid; d < D; d += GA_BLOCK) {
    S.cnt[d] = 0u;
    S.gcnt[d] = 0u;
    S.kmin[d] = ~0ull;
    S.kmax[d] = 0ull;
  }
  bar();

  // 3: per-slot count and m/z extent
  auto pass3 = [&](double m, double it, int32_t& tag, auto reg_c) __attribute__((always_inline)) {
    const int64_t b = decltype(reg_c)::value ? (int64_t)tag : floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb;
    const int slot = bitmap_rank(S.bitmap, S.wprefix, b);
    tag = slot;
    const uint64_t key = f64_order_key(m);
    SPX_GUARD(slot >= 0 && slot < D, "gap slot c=%ld slot=%d D=%d\n", (long)c, slot, D)
    atomicAdd(&S.cnt[slot], 1u);
    atomicMin(reinterpret_cast<unsigned long long*>(&S.kmin[slot]), (unsigned long long)key);
    atomicMax(reinterpret_cast<unsigned long long*>(&S.kmax[slot]), (unsigned long long)key);
  };
  peaks_m_tag(pass3);
  bar();

  SPX_GA_STAMP(4);
  int E;
  if (const int32_t st = gap_groups<kL>(S, P, D, tmp, votes, E); st != kOk) return st;
  SPX_GA_STAMP(5);
  // 5: fixed-point group sums (exact integer adds: order-independent)
  int ex_m, ex_i;
  frexp(fmax(fabs(lo), fabs(hi)) * (double)N, &ex_m);
  frexp(imax * (double)N, &ex_i);
  const int sc_m = 61 - ex_m, sc_i = 61 - ex_i;
  peaks([&](double m, double it, int32_t& tag, auto reg_c) {
    const int slot = decltype(reg_c)::value
                         ? tag
                         : bitmap_rank(S.bitmap, S.wprefix, floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb);
    const uint32_t eg = S.cnt[slot];
    SPX_GUARD(slot >= 0 && slot < D && (int)eg < E, "gap eg c=%ld slot=%d eg=%u E=%d\n", (long)c, slot, eg, E)
    atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmin[eg]), (unsigned long long)__double2ll_rn(ldexp(m, sc_m)));
    atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmax[eg]), (unsigned long long)__double2ll_rn(ldexp(it, sc_i)));
  });
  bar();

  SPX_GA_STAMP(6);
  return gap_emit<kL>(S, P, c, n, N, p0, E, sc_m, sc_i, out, tmp, red, votes);
}

template <class PrefixT>
__device__ __forceinline__ void gap_finish(const CsrView& v, const GapParams& P, int64_t c, int32_t st,
                                           const PeaksOut& out, double* prec_out, int32_t* charge_out,
                                           double* rt_out, int32_t* status, const PrecLanes* pl = nullptr,
                                           const int* prank = nullptr, double* stage = nullptr,
                                           long long* sel = nullptr) {
  const int64_t s0 = v.cluster_off[c], n = v.cluster_off[c + 1] - s0;
  if (st == kDeferred) return;
  const bool big = n > kWave && stage != nullptr;  // uniform
  if (big) prec_select_block(v, s0, n, P, stage, sel);
  if (wave_id() == 0) {
    PrecSummary R{nan_d(), nan_d(), 0, kOk};
    if (prank && pl && n > 0 && n <= kWave) {
      PrecRanks K{0, 0};
      const int lane = lane_id();
#pragma unroll
      for (int w = 0; w < GA_NW; ++w) {
        K.m += prank[w * kWave + lane];
        K.r += prank[(GA_NW + w) * kWave + lane];
      }
      R = precursor_summary_wave(*pl, (int)n, P, &K);
    } else if (n > 0) {
      R = (pl && n <= kWave) ? precursor_summary_wave(*pl, (int)n, P)
                             : precursor_summary(v, s0, n, P, big ? sel : nullptr);
    }
    if (lane_id() == 0) {
      // the reference computes the precursor first (:161-163): its error wins
      const int32_t fin = R.status != kOk ? R.status : st;
      prec_out[c] = R.pepmass;
      charge_out[c] = R.charge;
      rt_out[c] = R.rt;
      status[c] = fin;
      if (fin != kOk) out.count[c] = 0;
    }
  }
}

__global__ __launch_bounds__(GA_BLOCK, 4) void gap_average_lds_kernel(CsrView v, GapParams P, PeaksOut out,
                                                                   double* prec_out, int32_t* charge_out,
                                                                   double* rt_out, int32_t* status,
                                                                   StripedList deferred, int64_t own_n,
                                                                   int64_t own_lo) {
  __shared__ GapSmem L;
  const int64_t c = blockIdx.x;
  SPX_GA_STAMP(0);
  GapState<uint16_t> S{L.bitmap, L.wprefix, L.cnt, L.gcnt, L.kmin, L.kmax, GA_WMAX, GA_DCAP};
  const int64_t ps0 = v.cluster_off[c], pn = v.cluster_off[c + 1] - ps0;
  PrecLanes pl{0, 0.0, 0.0};
  if (pn <= kWave) pl = prec_lanes(v, ps0, pn);
  // a cluster past the register capacity goes to the wide kernel unread: streamed
  // here it would only be deferred after its bitmap pass (600-peak spectra from n ~ 18)
  const int32_t st = gap_body<GA_UM, true>(v, P, S, c, out, L.tmp, L.red, L.votes, &pl, L.prank);
  if (st == kDeferred || st == kNonFinite) {  // non-finite: the global kernel's gap_body_nf
    // a cluster of more than own_n peaks belongs to the giant intake (gap_giant_intake_kernel,
    // on the call's second stream): its status is the giant pipeline's to write; one of more
    // than own_lo MAY be the intake's (the wide kernel checks), so its status is left alone
    const int64_t pN = (own_n > 0 && pn >= 2) ? v.spec_off[ps0 + pn] - v.spec_off[ps0] : 0;
    if (own_n > 0 && pN > own_n) return;  // uniform
    if (threadIdx.x == 0) {
      if (!(own_lo > 0 && pN > own_lo)) status[c] = kDeferred;
      striped_push(deferred, (int32_t)c);
    }
    return;
  }
  gap_finish<uint16_t>(v, P, c, st, out, prec_out, charge_out, rt_out, status, &pl, L.prank,
                       reinterpret_cast<double*>(L.prank), L.sel);
  SPX_GA_STAMP(7);
}

// The LDS kernel's leftovers (striped list), grid-stride, one 147 KB workgroup per
// CU; what this one cannot hold either (a bucket range past the bitmap, more than
// GA_WDCAP buckets, a bucket spanning mz_accuracy) goes on to the global kernel.
__global__ __launch_bounds__(GA_BLOCK, 1) void gap_average_wide_kernel(CsrView v, GapParams P, PeaksOut out,
                                                                    double* prec_out, int32_t* charge_out,
                                                                    double* rt_out, int32_t* status,
                                                                    StripedList list, int32_t* deferred,
                                                                    int32_t* n_deferred, int64_t own_n,
                                                                    const uint8_t* owned) {
  __shared__ GapSmemT<GA_WDCAP> L;
  __shared__ int32_t lbase[kListStripes + 1];
  const int32_t nl = striped_prefix(list, lbase);
  GapState<uint16_t> S{L.bitmap, L.wprefix, L.cnt, L.gcnt, L.kmin, L.kmax, GA_WMAX, GA_WDCAP};
  for (int32_t i = blockIdx.x; i < nl; i += gridDim.x) {
    const int64_t c = striped_at(list, lbase, i);
    const int64_t ps0 = v.cluster_off[c], pn = v.cluster_off[c + 1] - ps0;
    const int64_t pN = pn >= 2 ? v.spec_off[ps0 + pn] - v.spec_off[ps0] : 0;
    if (own_n > 0 && pN > own_n) continue;  // uniform: the giant intake's
    if (owned && owned[c]) continue;        // uniform: taken by the intake's second tier
    if (SPX_GA_WMAXN > 0 && pN > (int64_t)SPX_GA_WMAXN) {  // uniform
      // too many peaks for one CU (the hybrid path re-reads its tail every pass): to the
      // global kernel, which hands it to the giant pipeline spread over the grid
      if (threadIdx.x == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
      continue;
    }
    PrecLanes pl{0, 0.0, 0.0};
    if (pn <= kWave) pl = prec_lanes(v, ps0, pn);
    const int32_t st = gap_body<GA_WUM, false>(v, P, S, c, out, L.tmp, L.red, L.votes, &pl, L.prank);
    if (st == kDeferred || st == kNonFinite) {
      if (threadIdx.x == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;  // status stays kDeferred
    } else {
      gap_finish<uint16_t>(v, P, c, st, out, prec_out, charge_out, rt_out, status, &pl, L.prank,
                           reinterpret_cast<double*>(L.prank), L.sel);
    }
    __syncthreads();  // the LDS is reused by the next cluster
  }
}

// Scratch slice of the deferred path: every array starts 256-B aligned (the
// 64-bit atomics on kmin/kmax fault on a misaligned address).
struct GapSliceLayout {
  int64_t bitmap, wprefix, cnt, gcnt, kmin, kmax, flags, chunks, total;
};
constexpr int GA_GCH = 8 * GA_BLOCK;  // slots per chunk of the giants' flat step-4 passes
__host__ __device__ inline GapSliceLayout gap_slice_layout(int wcap, int dcap) {
  GapSliceLayout L;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t at = o; o += (bytes + 255) & ~int64_t(255); return at; };
  L.bitmap = take((int64_t)wcap * 8);
  L.wprefix = take((int64_t)wcap * 4);
  L.cnt = take((int64_t)dcap * 4);
  L.gcnt = take((int64_t)dcap * 4);
  L.kmin = take((int64_t)dcap * 8);
  L.kmax = take((int64_t)dcap * 8);
  L.flags = take((int64_t)dcap * 4);
  L.chunks = take(((int64_t)dcap / GA_GCH + 2) * 4);  // step 4's per-chunk gap counts, then bases
  L.total = o;
  return L;
}

// ------------------------------------------------------- giant clusters
// A cluster of more than GA_GIANT_N peaks (the skewed law's n = 5,000 giants hold
// ~1.1M) is too much for one workgroup: the global kernel hands it to a pipeline
// whose per-peak passes (1 extrema, 2 bitmap, 3 slot extrema, 5 group sums) spread
// the cluster's peaks over the whole grid in tiles, with the per-slot and
// per-group steps (prefix, 4 gaps, 6 emit + precursor) one workgroup per giant in
// between.  Same integer atomics, same group structure, same fixed-point sums:
// the results equal gap_body's.  Each giant works in its own slice of an arena
// (slots for min(N, buckets in range)), taken by the global kernel's hand-off;
// a giant the arena or the record table cannot take stays in the global kernel.
constexpr int64_t GA_GIANT_N = 16384;
constexpr int GA_GMAX = 256;                      // giant records per call
constexpr int64_t GA_TILE = 2 * GA_BATCH * GA_BLOCK;  // peaks per tile
// The global kernel's giants (more than 16,384 peaks, deferred by the wide kernel; with
// the intake, the skewed law's mid-size clusters of a few hundred spectra) are few: their
// pipeline takes smaller tiles, so its per-tile passes spread over more workgroups
constexpr int64_t GA_TILE_LATE = 2048;
#ifndef SPX_GA_GGRID
#define SPX_GA_GGRID 512  // skewed configs[3] gap-average: 1024 4.21 ms, 512 3.77-3.79, 256 3.78-3.80, 4096 6.05
#endif
constexpr int GA_GIANT_GRID = SPX_GA_GGRID;       // tile kernels' workgroups
constexpr int GA_GAGG = 2560;                     // groups pass 5 sums in LDS first (50 KB)
// More groups than that (the skewed law's giants: 6.5k-59k, mostly noise groups of
// one peak): an open-addressing LDS table of HCAP groups per tile (a tile of ~40
// spectra touches ~1-2k groups), flushed to the slice after each tile -- one global
// add per (tile, group) instead of per peak.  A peak whose probe runs past
// GA_HPROBE slots adds globally.  Integer adds, so the totals do not change.
constexpr int GA_HCAP = 2048;
constexpr int GA_HPROBE = 16;

struct GapGiant {  // zeroed by the call's memset
  unsigned long long lo_inv, hi_key, imax_key;  // ~order key of the min m/z, order keys of max m/z, max |intensity|
  long long off;                                // its arena slice
  int32_t c, dcap, ok, bad, status, D, E, pad;  // pad: step 4a's "a bucket spans mz_accuracy" flag
  unsigned long long gmax_key;  // step 6a: order key of the largest kept group intensity
  int32_t gany, gnan;           // step 6a: some group has >= min_fraction spectra; one of them a NaN intensity
  // non-finite values (round 6: such a giant takes the tiled passes too; average_spectrum_clustering.py:59-98
  // as gap_body_nf restates it): any NaN/inf m/z or intensity; the -inf, +inf and NaN m/z counts; the true
  // groups' count M (the -inf group, the finite gaps' groups, the +inf boundary) and the -inf group's b0
  int32_t nf, n_ninf, n_pinf, n_nan, M, b0;
};

// Pass 5 of a giant with more groups than the LDS pre-sum holds: each tile's hashed
// (group -> sums) table is written as plain records, grouped by chunk of GA_GAGG groups,
// into the partials arena (instead of three memory-side atomics per entry), and
// gap_giant_reduce_kernel sums each (giant, chunk)'s records in LDS.  The sums are
// fixed-point integers, so any order gives the same totals.
struct GapPartial {
  uint32_t e, c;            // group, peaks
  unsigned long long m, i;  // fixed-point m/z and intensity sums
};
constexpr int GA_PCH = 2 * kWave - 1;  // chunks of GA_GAGG groups a tile's records can be sorted into (more: atomics)

struct GiantArgs {
  CsrView v;
  GapParams P;
  GapGiant* giants;
  const int32_t* n_giant;
  int gmax;
  char* arena;
  int wcap;
  double* out_mz;     // step 6 over the flat grid: the consensus outputs
  double* out_int;
  int64_t* out_count;
  char* part;                      // pass 5's partials arena
  long long part_cap;              // its bytes
  unsigned long long* part_used;   // bump pointer (zeroed by the call's memset)
  long long* tile_off;             // per flat (giant, tile) index: its records' byte offset, -1 = atomics
  int64_t tile;                    // peaks per tile (GA_TILE; the global kernel's few giants: GA_TILE_LATE)
};

__device__ __forceinline__ GapState<uint32_t> gap_slice_state(char* base, int wcap, int dcap) {
  const GapSliceLayout Lo = gap_slice_layout(wcap, dcap);
  GapState<uint32_t> S;
  S.bitmap = reinterpret_cast<unsigned long long*>(base + Lo.bitmap);
  S.wprefix = reinterpret_cast<uint32_t*>(base + Lo.wprefix);
  S.cnt = reinterpret_cast<uint32_t*>(base + Lo.cnt);
  S.gcnt = reinterpret_cast<uint32_t*>(base + Lo.gcnt);
  S.kmin = reinterpret_cast<uint64_t*>(base + Lo.kmin);
  S.kmax = reinterpret_cast<uint64_t*>(base + Lo.kmax);
  S.flags = reinterpret_cast<uint32_t*>(base + Lo.flags);
  S.wcap = wcap;
  S.dcap = dcap;
  return S;
}

// ------------------------------------------------------ non-finite clusters
// A cluster holding a NaN or +-inf m/z or intensity: gap_body reports it
// (kNonFinite) and the LDS and wide kernels hand it on, so only the global kernel
// and the giant pipeline's last step run this body.  It reproduces what the
// reference's own arithmetic does with such values (average_spectrum_clustering.py:59-98):
//  * np.argsort puts -inf first, then the finite m/z, then +inf, NaN last;
//  * np.diff >= acc holds from -inf to anything finite or +inf and from a finite
//    m/z to +inf, never across a NaN difference (inf - inf, x - NaN): the -inf
//    peaks are true group 0, the +inf and NaN peaks join the last true group;
//  * a cumsum difference cm[e-1] - cm[s-1] is finite while everything up to the
//    group's end is, +-inf when the group brings the first inf of one sign, and
//    NaN otherwise (inf - inf, NaN) -- per column from the group's classes and the
//    OR of the classes of the groups before it (nf_value);
//  * np.max propagates NaN: a kept NaN intensity makes the threshold NaN and
//    nothing is kept (no error).
// The finite m/z take gap_body's buckets and slots; sums are the same fixed point
// over the finite values.  Global scratch (S.flags), full barriers.
constexpr uint32_t NF_MZ_NINF = 1u, NF_MZ_PINF = 2u, NF_MZ_NAN = 4u;  // intensity classes: << 3

// 0 finite, 1 +inf, 2 -inf, 3 NaN: a cumsum over values of these classes
__device__ __forceinline__ int nf_state(uint32_t f) {
  f &= 7u;
  if ((f & NF_MZ_NAN) || (f & 3u) == 3u) return 3;
  return (f & NF_MZ_PINF) ? 1 : ((f & NF_MZ_NINF) ? 2 : 0);
}
// cm[e-1] - cm[s-1] (or cm[e-1] alone for s = 0) from the classes before the group (pre)
// and in it (grp); `fin` is the value when everything up to the group's end is finite
__device__ __forceinline__ double nf_value(uint32_t pre, uint32_t grp, double fin) {
  const int a = nf_state(pre | grp);
  if (a == 0) return fin;
  if (a == 3 || nf_state(pre) != 0) return nan_d();
  const double inf = __longlong_as_double(0x7ff0000000000000ll);
  return a == 1 ? inf : -inf;
}

__device__ int32_t gap_body_nf(const CsrView& v, const GapParams& P, const GapState<uint32_t>& S, int64_t c,
                               const PeaksOut& out, int* tmp, double* red, int* votes, uint32_t* ored) {
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1], n = s1 - s0;
  const int64_t p0 = v.spec_off[s0], p1 = v.spec_off[s1], N = p1 - p0;
  const double INF = __longlong_as_double(0x7ff0000000000000ll);
  if (n == 0) return kNoGap;
  auto emit_kept = [&](auto keep_at, auto mz_at, auto it_at, int64_t count) {  // ordered compaction
    int64_t base = 0;
    for (int64_t k0 = 0; k0 < count; k0 += GA_BLOCK) {  // uniform
      const int64_t k = k0 + tid;
      const int keep = k < count && keep_at(k);
      int tot;
      const int o = block_exclusive_scan<GA_BLOCK, int>(keep, tmp, tot);
      if (keep) {
        out.mz[p0 + base + o] = mz_at(k);
        out.inten[p0 + base + o] = it_at(k);
      }
      base += tot;
    }
    if (tid == 0) out.count[c] = base;
  };
  if (n == 1) {  // passthrough + the dynamic-range filter (:88-98), NaN-propagating max
    double mx = -INF;
    int nanf = 0;
    for (int64_t k = p0 + tid; k < p1; k += GA_BLOCK) {
      const double it = v.inten[k];
      nanf |= isnan(it);
      mx = fmax(mx, it);
    }
    mx = wave_max_dpp(mx);
    if (lane == 0) red[wid] = mx;
    const int any_nan = block_any<GA_BLOCK, false>(nanf, votes, 0);
    for (int w = 0; w < GA_NW; ++w) mx = fmax(mx, red[w]);
    __syncthreads();
    if (N == 0) return kEmpty;
    const double thr = any_nan ? nan_d() : mx / P.dyn_range;
    emit_kept([&](int64_t k) { return v.inten[p0 + k] >= thr; }, [&](int64_t k) { return v.mz[p0 + k]; },
              [&](int64_t k) { return v.inten[p0 + k]; }, N);
    return kOk;
  }
  if (N < 2) return kNoGap;

  // 1: the finite m/z extent, max |finite intensity|, the non-finite m/z classes
  double lo = INF, hi = -INF, imax = 0.0;
  int cn = 0, cp = 0, cq = 0;
  gap_peaks<true>(v, p0, p1, [&](int64_t, double m, double it) {
    if (isfinite(m)) {
      lo = fmin(lo, m);
      hi = fmax(hi, m);
    } else if (isnan(m)) {
      ++cq;
    } else if (m > 0.0) {
      ++cp;
    } else {
      ++cn;
    }
    if (isfinite(it)) imax = fmax(imax, fabs(it));
  });
  lo = wave_min_dpp(lo);
  hi = wave_max_dpp(hi);
  imax = wave_max_dpp(imax);
  if (lane == 0) { red[wid] = lo; red[GA_NW + wid] = hi; red[2 * GA_NW + wid] = imax; }
  int n_ninf, n_pinf, n_nan;
  block_exclusive_scan<GA_BLOCK, int>(cn, tmp, n_ninf);  // its barriers order red too
  block_exclusive_scan<GA_BLOCK, int>(cp, tmp, n_pinf);
  block_exclusive_scan<GA_BLOCK, int>(cq, tmp, n_nan);
  for (int w = 0; w < GA_NW; ++w) {
    lo = fmin(lo, red[w]);
    hi = fmax(hi, red[GA_NW + w]);
    imax = fmax(imax, red[2 * GA_NW + w]);
  }
  __syncthreads();
  const int64_t Nf = N - n_ninf - n_pinf - n_nan;

  // 2-4 over the finite m/z: buckets, slots, their extents, the finite gaps
  int D = 0, fin_gaps = 0;
  int64_t kb = 0;
  const double acc = P.mz_accuracy;
  auto key = [&](const uint64_t* a, int d) { return f64_from_order_key(a[d]); };
  if (Nf > 0) {  // uniform
    kb = floor_div_exact(lo, P.bucket_w, P.inv_bucket_w);
    const int64_t nw = (floor_div_exact(hi, P.bucket_w, P.inv_bucket_w) - kb) / 64 + 1;
    if (nw > S.wcap) return kDeferred;
    for (int64_t w = tid; w < nw; w += GA_BLOCK) S.bitmap[w] = 0ull;
    __syncthreads();
    gap_peaks<false>(v, p0, p1, [&](int64_t, double m, double) {
      if (isfinite(m)) {
        const int64_t b = floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb;
        atomicOr(&S.bitmap[b >> 6], 1ull << (b & 63));
      }
    });
    __syncthreads();
    D = bitmap_prefix<GA_BLOCK, uint32_t, false>(S.bitmap, S.wprefix, (int)nw, tmp);
    if (D > S.dcap) return kDeferred;
    for (int d = tid; d < D; d += GA_BLOCK) {
      S.cnt[d] = 0u;
      S.kmin[d] = ~0ull;
      S.kmax[d] = 0ull;
    }
    __syncthreads();
    gap_peaks<false>(v, p0, p1, [&](int64_t, double m, double) {
      if (isfinite(m)) {
        const int slot = bitmap_rank(S.bitmap, S.wprefix, floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb);
        const uint64_t k = f64_order_key(m);
        atomicAdd(&S.cnt[slot], 1u);
        atomicMin(reinterpret_cast<unsigned long long*>(&S.kmin[slot]), (unsigned long long)k);
        atomicMax(reinterpret_cast<unsigned long long*>(&S.kmax[slot]), (unsigned long long)k);
      }
    });
    __syncthreads();
    int split = 0, my_gaps = 0;
    for (int d = tid; d < D; d += GA_BLOCK) {
      const double mx = key(S.kmax, d);
      split |= (mx - key(S.kmin, d)) >= acc;  // a gap could hide inside the bucket
      if (d + 1 < D) my_gaps += (key(S.kmin, d + 1) - mx) >= acc;
    }
    if (block_any<GA_BLOCK, false>(split, votes, 1)) return kDeferred;
    block_exclusive_scan<GA_BLOCK, int>(my_gaps, tmp, fin_gaps);
  }
  // the boundaries: after the -inf peaks, the finite gaps, before the +inf peaks
  const int b0 = (n_ninf > 0 && (Nf > 0 || n_pinf > 0)) ? 1 : 0;
  const int be = (n_pinf > 0 && Nf > 0) ? 1 : 0;
  const int M = b0 + fin_gaps + be;
  if (M == 0) return kNoGap;
  const int E = M >= 2 ? M : 2;
  if (E > S.dcap) return kDeferred;
  auto emitted = [&](int g) { return M >= 2 ? min(g, M - 1) : g; };  // the last two true groups merged (:79)
  for (int e = tid; e < E; e += GA_BLOCK) {
    S.gcnt[e] = 0u;
    S.flags[e] = 0u;
  }
  __syncthreads();
  // each finite slot's emitted group (rounds of 8 contiguous slots, as gap_groups)
  constexpr int CH = 8;
  int carry = 0;
  for (int r0 = 0; r0 < D; r0 += GA_BLOCK * CH) {  // uniform
    const int db = r0 + tid * CH;
    int f[CH], mine = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int d = db + k;
      f[k] = d > 0 && d < D && (key(S.kmin, d) - key(S.kmax, d - 1)) >= acc;
      mine += f[k];
    }
    int tot;
    int g = b0 + carry + block_exclusive_scan<GA_BLOCK, int>(mine, tmp, tot);
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int d = db + k;
      if (d < D) {
        g += f[k];
        const int eg = emitted(g);
        atomicAdd(&S.gcnt[eg], S.cnt[d]);
        S.cnt[d] = (uint32_t)eg;
      }
    }
    carry += tot;
  }
  __syncthreads();
  for (int e = tid; e < E; e += GA_BLOCK) { S.kmin[e] = 0ull; S.kmax[e] = 0ull; }
  __syncthreads();

  // 5: fixed-point sums of the finite values, the non-finite m/z's counts, the classes
  int ex_m, ex_i;
  frexp(Nf > 0 ? fmax(fabs(lo), fabs(hi)) * (double)N : 0.0, &ex_m);
  frexp(imax * (double)N, &ex_i);
  const int sc_m = 61 - ex_m, sc_i = 61 - ex_i;
  gap_peaks<true>(v, p0, p1, [&](int64_t, double m, double it) {
    uint32_t fl = 0u;
    int eg;
    if (isfinite(m)) {
      eg = (int)S.cnt[bitmap_rank(S.bitmap, S.wprefix, floor_div_exact(m, P.bucket_w, P.inv_bucket_w) - kb)];
      atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmin[eg]), (unsigned long long)__double2ll_rn(ldexp(m, sc_m)));
    } else {
      eg = emitted(m == -INF ? 0 : M);  // -inf: group 0; +inf and NaN: the last true group
      atomicAdd(&S.gcnt[eg], 1u);
      fl = isnan(m) ? NF_MZ_NAN : (m > 0.0 ? NF_MZ_PINF : NF_MZ_NINF);
    }
    if (isfinite(it))
      atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmax[eg]), (unsigned long long)__double2ll_rn(ldexp(it, sc_i)));
    else
      fl |= (isnan(it) ? NF_MZ_NAN : (it > 0.0 ? NF_MZ_PINF : NF_MZ_NINF)) << 3;
    if (fl) atomicOr(&S.flags[eg], fl);
  });
  __syncthreads();

  // 6: values in group order (classes of the groups before each one), min_fraction,
  // the NaN-propagating max, the dynamic-range filter, ordered output
  const int gper = (E + GA_BLOCK - 1) / GA_BLOCK;
  const int e0 = tid * gper;
  uint32_t mine = 0u;
  for (int j = 0; j < gper && e0 + j < E; ++j) mine |= S.flags[e0 + j];
  ored[tid] = mine;
  __syncthreads();
  uint32_t pre = 0u;
  for (int t = 0; t < tid; ++t) pre |= ored[t];
  const double min_len = P.min_fraction * (double)n;
  auto values = [&](int e, uint32_t pf, double& vm, double& vi) {
    const uint32_t gf = S.flags[e];
    vm = nf_value(pf, gf, ldexp((double)(int64_t)S.kmin[e], -sc_m) / (double)S.gcnt[e]);
    vi = nf_value(pf >> 3, gf >> 3, ldexp((double)(int64_t)S.kmax[e], -sc_i) / (double)n);
  };
  double gmax = -INF;
  int anyg = 0, gnan = 0;
  {
    uint32_t pf = pre;
    for (int j = 0; j < gper && e0 + j < E; ++j) {
      const int e = e0 + j;
      double vm, vi;
      values(e, pf, vm, vi);
      pf |= S.flags[e];
      if ((double)S.gcnt[e] >= min_len) {
        anyg = 1;
        if (isnan(vi)) gnan = 1;
        else gmax = fmax(gmax, vi);
      }
    }
  }
  gmax = wave_max_dpp(gmax);
  if (lane == 0) red[wid] = gmax;
  const int any_kept = block_any<GA_BLOCK, false>(anyg, votes, 0);
  const int any_nan = block_any<GA_BLOCK, false>(gnan, votes, 1);
  for (int w = 0; w < GA_NW; ++w) gmax = fmax(gmax, red[w]);
  __syncthreads();
  if (!any_kept) return kEmpty;
  const double thr = any_nan ? nan_d() : gmax / P.dyn_range;  // NaN: nothing passes `>=`
  int cntk = 0;
  {
    uint32_t pf = pre;
    for (int j = 0; j < gper && e0 + j < E; ++j) {
      const int e = e0 + j;
      double vm, vi;
      values(e, pf, vm, vi);
      pf |= S.flags[e];
      cntk += (double)S.gcnt[e] >= min_len && vi >= thr;
    }
  }
  int total;
  int o = block_exclusive_scan<GA_BLOCK, int>(cntk, tmp, total);
  {
    uint32_t pf = pre;
    for (int j = 0; j < gper && e0 + j < E; ++j) {
      const int e = e0 + j;
      double vm, vi;
      values(e, pf, vm, vi);
      pf |= S.flags[e];
      if ((double)S.gcnt[e] >= min_len && vi >= thr) {
        out.mz[p0 + o] = vm;
        out.inten[p0 + o] = vi;
        ++o;
      }
    }
  }
  if (tid == 0) out.count[c] = total;
  return kOk;
}

// The giant's m/z extent as gap_body's pass 1 leaves it (lo, hi, imax; kb, nw)
struct GiantExtent {
  double lo, hi, imax;
  int64_t kb, nw;
};
__device__ __forceinline__ GiantExtent giant_extent(const GapGiant& H, const GapParams& P) {
  GiantExtent X;
  X.lo = f64_from_order_key(~H.lo_inv);
  X.hi = f64_from_order_key(H.hi_key);
  X.imax = f64_from_order_key(H.imax_key);
  X.kb = floor_div_exact(X.lo, P.bucket_w, P.inv_bucket_w);
  X.nw = (floor_div_exact(X.hi, P.bucket_w, P.inv_bucket_w) - X.kb) / 64 + 1;
  return X;
}

// A giant's tiles in tile pass `pass` (0: not in it); the tile passes and the pass-5
// reduction index the (giant, tile) pairs by the same prefix of these counts.
__device__ __forceinline__ int64_t giant_tiles(const GiantArgs& A, const GapGiant& H, int pass) {
  if (!H.ok) return 0;
  if (pass > 1) {
    if (H.bad || H.status != kOk) return 0;
    if (H.hi_key == 0ull) return 0;  // no finite m/z (step 0 sends it to gap_body_nf)
    if (giant_extent(H, A.P).nw > A.wcap) return 0;  // the prefix step defers it
  }
  const int64_t p0 = A.v.spec_off[A.v.cluster_off[H.c]], p1 = A.v.spec_off[A.v.cluster_off[H.c + 1]];
  return (p1 - p0 + A.tile - 1) / A.tile;
}

// The per-peak passes over every giant's tiles: PASS 1 extrema (and the slices'
// bitmaps zeroed), 2 bucket bitmap, 3 slot m/z extent, 5 group sums and counts.
// The (giant, tile) pairs of all giants form one index space, striped over the grid.
template <int PASS>
__global__ __launch_bounds__(GA_BLOCK) void gap_giant_tiles_kernel(GiantArgs A) {
  __shared__ double red[GA_NW * 3];
  __shared__ int votes[2 * GA_NW];
  constexpr bool kH3 = PASS == 3 || PASS == 2;
  // pass 2 (kH3 too): agg_m holds the hashed words' OR-ed bits
  // pass 5: group sums (agg_m, agg_i); pass 3 (kH3): the hashed slots' min / max m/z keys
  __shared__ unsigned long long agg_m[PASS == 5 ? GA_GAGG : (kH3 ? GA_HCAP : 1)];
  __shared__ unsigned long long agg_i[PASS == 5 ? GA_GAGG : (kH3 && PASS == 3 ? GA_HCAP : 1)];
  __shared__ uint32_t agg_c[PASS == 5 ? GA_GAGG : 1];
  __shared__ uint32_t hkey[PASS == 5 || kH3 ? GA_HCAP : 1];  // group / slot + 1 (0: empty)
  const int tid = threadIdx.x, lane = lane_id(), wid = wave_id();
  const int ng = min(*A.n_giant, A.gmax);
  auto peaks_of = [&](const GapGiant& H, int64_t& p0, int64_t& p1) {
    p0 = A.v.spec_off[A.v.cluster_off[H.c]];
    p1 = A.v.spec_off[A.v.cluster_off[H.c + 1]];
  };
  // a giant's tiles in this pass (0: not in it)
  auto tiles_of = [&](const GapGiant& H) -> int64_t { return giant_tiles(A, H, PASS); };
  if constexpr (kH3) {
    for (int h = tid; h < GA_HCAP; h += GA_BLOCK) {
      hkey[h] = 0u;
      agg_m[h] = PASS == 3 ? ~0ull : 0ull;
      if constexpr (PASS == 3) agg_i[h] = 0ull;
    }
    lds_barrier();
  }
  if constexpr (PASS == 1) {
    for (int g = 0; g < ng; ++g) {
      if (!A.giants[g].ok) continue;
      unsigned long long* bm = gap_slice_state(A.arena + A.giants[g].off, A.wcap, A.giants[g].dcap).bitmap;
      for (int64_t w = (int64_t)blockIdx.x * GA_BLOCK + tid; w < A.wcap; w += (int64_t)gridDim.x * GA_BLOCK)
        bm[w] = 0ull;
    }
  }
  int g = 0, cur = -1, E = 0, sc_m = 0, sc_i = 0, Mg = 0;
  bool agg = false, hashed = false, nfg = false;
  int64_t gbase = 0, gtiles = ng > 0 ? tiles_of(A.giants[0]) : 0, p0 = 0, p1 = 0, kb = 0;
  // passes 2 and 3 take the tiles in a scattered order (t = u * P mod T): consecutive
  // workgroups then work on different giants instead of 512 neighbouring tiles of one,
  // whose per-tile flushes all hit the same template slots of one slice at once
  // (round 6, with passes 3 and 5 flushing plain records: the scattered order is still
  // the fastest for every pass -- skewed configs[3] 1.865 ms; sequential pass 5 1.90,
  // sequential 3 and 5 1.99, sequential 3 only 1.96)
  constexpr bool kPerm = PASS == 1 || PASS == 2 || PASS == 3 || PASS == 5;
  __shared__ long long tpre[kPerm ? GA_GMAX + 1 : 1];
  __shared__ long long ttmp[kPerm ? GA_NW + 1 : 1];
  long long tT = 0, tP = 1;
  if constexpr (kPerm) {
    const int64_t tc = tid < ng ? tiles_of(A.giants[tid]) : 0;
    long long tot;
    const long long e = block_exclusive_scan<GA_BLOCK, long long>((long long)tc, ttmp, tot);
    if (tid < ng) tpre[tid] = e;
    if (tid == 0) tpre[ng] = tot;
    __syncthreads();
    tT = tpre[ng];
    // a multiplier coprime to T (T < 2^31 tiles)
    const long long cands[4] = {40503, 65521, 7919, 1};
    for (int q = 0; q < 4; ++q) {
      long long a = cands[q], b = tT > 0 ? tT : 1;
      while (b) { const long long r = a % b; a = b; b = r; }
      if (a == 1) { tP = cands[q]; break; }
    }
  }
  GapState<uint32_t> S{};
  __shared__ int pcnt[PASS == 5 || PASS == 3 ? 2 * kWave : 1];  // passes 3, 5: records per chunk, then cursors
  __shared__ long long poff;
  __shared__ int pocc;
  // the hashed table after tile u: its occupied entries (pass 5: group sums; pass 3: slot
  // m/z extents) as records sorted by chunk of GA_GAGG groups / slots (the partials arena;
  // gap_giant_reduce_kernel folds them) or, when the arena is full or the giant has too
  // many chunks, as global atomics; the table emptied
  auto hflush = [&](int64_t u) __attribute__((always_inline)) {
    if constexpr (PASS == 5 || PASS == 3) {
      const int nch = (E + GA_GAGG - 1) / GA_GAGG;
      for (int k = tid; k <= GA_PCH; k += GA_BLOCK) pcnt[k] = 0;
      lds_barrier();
      if (nch <= GA_PCH) {
        for (int h = tid; h < GA_HCAP; h += GA_BLOCK) {
          const uint32_t k = hkey[h];
          if (k) atomicAdd(&pcnt[(k - 1u) / GA_GAGG], 1);
        }
      }
      lds_barrier();
      if (tid < kWave) {  // chunk starts (exclusive prefix) for the record header and the LDS cursors
        const int a = pcnt[2 * tid], b = pcnt[2 * tid + 1];
        const int inc = wave_inclusive_sum(a + b);
        const int occ = __shfl(inc, kWave - 1, kWave);  // the tile's occupied entries
        pcnt[2 * tid] = inc - a - b;
        pcnt[2 * tid + 1] = inc - b;
        if (tid == 0) {
          long long off = -1;
          if (nch <= GA_PCH && occ > 0) {
            const long long bytes = ((long long)(nch + 1) * 4 + 15) / 16 * 16 + (long long)occ * sizeof(GapPartial);
            const long long at = (long long)atomicAdd(A.part_used, (unsigned long long)bytes);
            if (at + bytes <= A.part_cap) off = at;
          }
          poff = off;
          pocc = occ;
          A.tile_off[u] = off;
        }
      }
      lds_barrier();
      const long long off = poff;
      const int occ = pocc;
      uint32_t* hdr = off >= 0 ? reinterpret_cast<uint32_t*>(A.part + off) : nullptr;
      GapPartial* rec = off >= 0 ? reinterpret_cast<GapPartial*>(A.part + off + ((long long)(nch + 1) * 4 + 15) / 16 * 16)
                                 : nullptr;
      if (off >= 0)
        for (int k = tid; k <= nch; k += GA_BLOCK) hdr[k] = (uint32_t)(k < nch ? pcnt[k] : occ);
      lds_barrier();  // the header read its starts before the cursors move
      for (int h = tid; h < GA_HCAP; h += GA_BLOCK) {
        const uint32_t k = hkey[h];
        if (k) {
          const uint32_t e = k - 1u;
          if constexpr (PASS == 5) {
            if (off >= 0) {
              const int pos = atomicAdd(&pcnt[e / GA_GAGG], 1);
              rec[pos] = GapPartial{e, agg_c[h], agg_m[h], agg_i[h]};
            } else {
              atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmin[e]), agg_m[h]);
              atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmax[e]), agg_i[h]);
              atomicAdd(&S.gcnt[e], agg_c[h]);
            }
            agg_m[h] = 0ull;
            agg_i[h] = 0ull;
            agg_c[h] = 0u;
          } else {
            if (off >= 0) {
              const int pos = atomicAdd(&pcnt[e / GA_GAGG], 1);
              rec[pos] = GapPartial{e, 0u, agg_m[h], agg_i[h]};
            } else {
              atomicMin(reinterpret_cast<unsigned long long*>(&S.kmin[e]), agg_m[h]);
              atomicMax(reinterpret_cast<unsigned long long*>(&S.kmax[e]), agg_i[h]);
            }
            agg_m[h] = ~0ull;
            agg_i[h] = 0ull;
          }
          hkey[h] = 0u;
        }
      }
      lds_barrier();
    }
  };
  auto flush = [&]() __attribute__((always_inline)) {  // PASS 5: the LDS sums of giant `cur`
    if constexpr (PASS == 5) {
      if (agg) {
        lds_barrier();
        for (int e = tid; e < E; e += GA_BLOCK) {
          if (agg_c[e]) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmin[e]), agg_m[e]);
            atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmax[e]), agg_i[e]);
            atomicAdd(&S.gcnt[e], agg_c[e]);
          }
        }
        lds_barrier();
      }
    }
  };
  for (int64_t u0 = blockIdx.x;; u0 += gridDim.x) {  // uniform
    int64_t u = u0;
    if constexpr (kPerm) {
      if (u0 >= tT) break;
      u = (int64_t)(((unsigned long long)u0 * (unsigned long long)tP) % (unsigned long long)tT);
      int lo = 0, hi = ng;  // the giant with tpre[g] <= u < tpre[g + 1]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tpre[mid] <= u) lo = mid; else hi = mid;
      }
      while (lo + 1 < ng && tpre[lo + 1] <= u) ++lo;
      g = lo;
      gbase = tpre[g];
      gtiles = tpre[g + 1] - tpre[g];
    } else
    {
      while (g < ng && u >= gbase + gtiles) {
        gbase += gtiles;
        if (++g < ng) gtiles = tiles_of(A.giants[g]);
      }
      if (g >= ng) break;
    }
    const GapGiant& H = A.giants[g];
    if (g != cur) {  // this workgroup's first tile of giant g
      flush();
      cur = g;
      peaks_of(H, p0, p1);
      S = gap_slice_state(A.arena + H.off, A.wcap, H.dcap);
      if constexpr (PASS > 1) {
        const GiantExtent X = giant_extent(H, A.P);
        kb = X.kb;
        if constexpr (PASS == 3) E = H.D;  // hflush's records are per slot
        if constexpr (PASS == 5) {
          const int64_t N = p1 - p0;
          int ex_m, ex_i;
          frexp(fmax(fabs(X.lo), fabs(X.hi)) * (double)N, &ex_m);
          frexp(X.imax * (double)N, &ex_i);
          sc_m = 61 - ex_m;
          sc_i = 61 - ex_i;
          nfg = H.nf != 0;
          Mg = H.M;
          // few groups: this workgroup's sums and counts in LDS first, one global add
          // per group at the end (integer adds: the same totals)
          E = H.E;
          agg = E <= GA_GAGG;
          hashed = !agg;
          if (agg) {
            for (int e = tid; e < E; e += GA_BLOCK) { agg_m[e] = 0ull; agg_i[e] = 0ull; agg_c[e] = 0u; }
            lds_barrier();
          } else if (hashed) {
            for (int h = tid; h < GA_HCAP; h += GA_BLOCK) { hkey[h] = 0u; agg_m[h] = 0ull; agg_i[h] = 0ull; agg_c[h] = 0u; }
            lds_barrier();
          }
        }
      }
    }
    const int64_t t0 = p0 + (u - gbase) * A.tile, t1 = min(p1, t0 + A.tile);
    if constexpr (PASS == 1) {
      // the FINITE m/z extent and max |finite intensity| (gap_body_nf's pass 1); a
      // non-finite m/z is counted by class, and any non-finite value flags the giant
      double lo = __longlong_as_double(0x7ff0000000000000ll), hi = -lo, imax = 0.0;
      int bad = 0, cn = 0, cp = 0, cq = 0;
      gap_peaks<true>(A.v, t0, t1, [&](int64_t, double m, double it) {
        if (isfinite(m)) {
          lo = fmin(lo, m);
          hi = fmax(hi, m);
        } else {
          cq += isnan(m);
          cp += m == __longlong_as_double(0x7ff0000000000000ll);
          cn += m == -__longlong_as_double(0x7ff0000000000000ll);
        }
        if (isfinite(it)) imax = fmax(imax, fabs(it));
        else bad = 1;
      });
      bad |= cn | cp | cq;
      if (cn | cp | cq) {  // rare: per thread, straight to the giant's counters
        GapGiant& Hc = A.giants[g];
        if (cn) atomicAdd(&Hc.n_ninf, cn);
        if (cp) atomicAdd(&Hc.n_pinf, cp);
        if (cq) atomicAdd(&Hc.n_nan, cq);
      }
      lo = wave_min_dpp(lo);
      hi = wave_max_dpp(hi);
      imax = wave_max_dpp(imax);
      if (lane == 0) { red[wid] = lo; red[GA_NW + wid] = hi; red[2 * GA_NW + wid] = imax; }
      const int anybad = block_any<GA_BLOCK, true>(bad, votes, 0);  // its barrier orders red too
      if (tid == 0) {
        for (int w = 1; w < GA_NW; ++w) {
          lo = fmin(lo, red[w]);
          hi = fmax(hi, red[GA_NW + w]);
          imax = fmax(imax, red[2 * GA_NW + w]);
        }
        GapGiant& Hw = A.giants[g];
        if (anybad) atomicOr(&Hw.nf, 1);
        if (lo <= hi) {
          atomicMax(&Hw.lo_inv, ~(unsigned long long)f64_order_key(lo));
          atomicMax(&Hw.hi_key, (unsigned long long)f64_order_key(hi));
        }
        atomicMax(&Hw.imax_key, (unsigned long long)f64_order_key(imax));
      }
      lds_barrier();  // red and votes are reused by the next tile
    } else if (PASS == 2 || PASS == 3) {
      // passes 2-3 in batches of GA_BATCH peaks per thread: every global read a
      // batch needs (bitmap words; ranks, then the slots' extrema) goes out before
      // its first atomic -- an atomic in between would order each read behind it
      for (int64_t k0 = t0 + tid; k0 < t1; k0 += GA_BATCH * GA_BLOCK) {
        double m[GA_BATCH];
#pragma unroll
        for (int q = 0; q < GA_BATCH; ++q) {
          const int64_t k = k0 + (int64_t)q * GA_BLOCK;
          m[q] = A.v.mz[k < t1 ? k : t0];
        }
        // a non-finite m/z takes no bucket (its index 0 is never used)
        int64_t b[GA_BATCH];
#pragma unroll
        for (int q = 0; q < GA_BATCH; ++q)
          b[q] = isfinite(m[q]) ? floor_div_exact(m[q], A.P.bucket_w, A.P.inv_bucket_w) - kb : 0;
        if constexpr (PASS == 2 && kH3) {
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) {
            if (k0 + (int64_t)q * GA_BLOCK >= t1 || !isfinite(m[q])) continue;
            const uint32_t wi = (uint32_t)(b[q] >> 6);
            const unsigned long long bit = 1ull << (b[q] & 63);
            const uint32_t want = wi + 1u;
            uint32_t h = (wi * 2654435761u) >> (32 - 11);  // log2(GA_HCAP) = 11
            bool done = false;
            for (int probe = 0; probe < GA_HPROBE; ++probe, h = (h + 1u) & (GA_HCAP - 1)) {
              uint32_t k = hkey[h];
              if (k == 0u) {
                const uint32_t old = atomicCAS(&hkey[h], 0u, want);
                k = old == 0u ? want : old;
              }
              if (k == want) {
                if (!(agg_m[h] & bit)) atomicOr(&agg_m[h], bit);
                done = true;
                break;
              }
            }
            if (!done && !(S.bitmap[wi] & bit)) atomicOr(&S.bitmap[wi], bit);  // a long probe: globally
          }
        } else if constexpr (PASS == 2) {
          unsigned long long w[GA_BATCH];
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) w[q] = S.bitmap[b[q] >> 6];
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) {
            const unsigned long long bit = 1ull << (b[q] & 63);
            if (k0 + (int64_t)q * GA_BLOCK < t1 && !(w[q] & bit)) atomicOr(&S.bitmap[b[q] >> 6], bit);
          }
        } else if constexpr (kH3) {
          int slot[GA_BATCH];
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) slot[q] = bitmap_rank(S.bitmap, S.wprefix, b[q]);
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) {
            if (k0 + (int64_t)q * GA_BLOCK >= t1 || !isfinite(m[q])) continue;
            const unsigned long long key = f64_order_key(m[q]);
            const uint32_t want = (uint32_t)slot[q] + 1u;
            uint32_t h = ((uint32_t)slot[q] * 2654435761u) >> (32 - 11);  // log2(GA_HCAP) = 11
            bool done = false;
            for (int probe = 0; probe < GA_HPROBE; ++probe, h = (h + 1u) & (GA_HCAP - 1)) {
              uint32_t k = hkey[h];
              if (k == 0u) {
                const uint32_t old = atomicCAS(&hkey[h], 0u, want);
                k = old == 0u ? want : old;
              }
              if (k == want) {
                atomicMin(&agg_m[h], key);
                atomicMax(&agg_i[h], key);
                done = true;
                break;
              }
            }
            if (!done) {  // a long probe: the slot's extent globally
              unsigned long long* kmin = reinterpret_cast<unsigned long long*>(&S.kmin[slot[q]]);
              unsigned long long* kmax = reinterpret_cast<unsigned long long*>(&S.kmax[slot[q]]);
              if (key < *kmin) atomicMin(kmin, key);
              if (key > *kmax) atomicMax(kmax, key);
            }
          }
        } else {
          int slot[GA_BATCH];
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) slot[q] = bitmap_rank(S.bitmap, S.wprefix, b[q]);
          unsigned long long lo[GA_BATCH], hi[GA_BATCH];
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) {
            lo[q] = reinterpret_cast<const unsigned long long*>(S.kmin)[slot[q]];
            hi[q] = reinterpret_cast<const unsigned long long*>(S.kmax)[slot[q]];
          }
#pragma unroll
          for (int q = 0; q < GA_BATCH; ++q) {
            if (k0 + (int64_t)q * GA_BLOCK >= t1) continue;
            const unsigned long long key = f64_order_key(m[q]);
            if (key < lo[q]) atomicMin(reinterpret_cast<unsigned long long*>(&S.kmin[slot[q]]), key);
            if (key > hi[q]) atomicMax(reinterpret_cast<unsigned long long*>(&S.kmax[slot[q]]), key);
          }
        }
      }
      if constexpr (PASS == 3) {
        hflush(u);  // the tile's slot extents: records for gap_giant_reduce_kernel<3>
      } else if constexpr (kH3) {  // the tile's bitmap words to the slice
        lds_barrier();
        for (int h = tid; h < GA_HCAP; h += GA_BLOCK) {
          const uint32_t k = hkey[h];
          if (k) {
            atomicOr(&S.bitmap[k - 1u], agg_m[h]);
            agg_m[h] = 0ull;
            hkey[h] = 0u;
          }
        }
        lds_barrier();
      }
    } else {
      gap_peaks<PASS == 5>(A.v, t0, t1, [&](int64_t, double m, double it) {
        const int64_t b = isfinite(m) ? floor_div_exact(m, A.P.bucket_w, A.P.inv_bucket_w) - kb : 0;
        // bits and extrema only grow / shrink, so a stale read that says "no
        // change" is still right: the atomic is issued only when it can matter
        if constexpr (PASS == 2) {
          const unsigned long long bit = 1ull << (b & 63);
          if (!(S.bitmap[b >> 6] & bit)) atomicOr(&S.bitmap[b >> 6], bit);
        } else if constexpr (PASS == 3) {  // the counts come with pass 5's group sums
          const int slot = bitmap_rank(S.bitmap, S.wprefix, b);
          const unsigned long long key = f64_order_key(m);
          unsigned long long* kmin = reinterpret_cast<unsigned long long*>(&S.kmin[slot]);
          unsigned long long* kmax = reinterpret_cast<unsigned long long*>(&S.kmax[slot]);
          if (key < *kmin) atomicMin(kmin, key);
          if (key > *kmax) atomicMax(kmax, key);
        } else {
          uint32_t eg;
          unsigned long long qm = 0ull, qi = 0ull;
          if (!nfg || isfinite(m)) {
            eg = S.cnt[bitmap_rank(S.bitmap, S.wprefix, b)];
            qm = (unsigned long long)__double2ll_rn(ldexp(m, sc_m));
          } else {  // -inf: true group 0; +inf, NaN: the last true group (gap_body_nf)
            eg = (uint32_t)min(m < 0.0 ? 0 : Mg, E - 1);
          }
          if (!nfg || isfinite(it)) qi = (unsigned long long)__double2ll_rn(ldexp(it, sc_i));
          if (nfg) {  // the classes of the group's non-finite m/z and intensities
            uint32_t fl = 0u;
            if (!isfinite(m)) fl = isnan(m) ? NF_MZ_NAN : (m > 0.0 ? NF_MZ_PINF : NF_MZ_NINF);
            if (!isfinite(it)) fl |= (isnan(it) ? NF_MZ_NAN : (it > 0.0 ? NF_MZ_PINF : NF_MZ_NINF)) << 3;
            if (fl) atomicOr(&S.flags[eg], fl);
          }
          if (agg) {
            atomicAdd(&agg_m[eg], qm);
            atomicAdd(&agg_i[eg], qi);
            atomicAdd(&agg_c[eg], 1u);
            return;
          }
          if (hashed) {
            const uint32_t want = eg + 1u;
            uint32_t h = (eg * 2654435761u) >> (32 - 11);  // log2(GA_HCAP) = 11
            for (int probe = 0; probe < GA_HPROBE; ++probe, h = (h + 1u) & (GA_HCAP - 1)) {
              uint32_t k = hkey[h];
              if (k == 0u) {
                const uint32_t old = atomicCAS(&hkey[h], 0u, want);
                k = old == 0u ? want : old;
              }
              if (k == want) {
                atomicAdd(&agg_m[h], qm);
                atomicAdd(&agg_i[h], qi);
                atomicAdd(&agg_c[h], 1u);
                return;
              }
            }
          }
          atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmin[eg]), qm);
          atomicAdd(reinterpret_cast<unsigned long long*>(&S.kmax[eg]), qi);
          atomicAdd(&S.gcnt[eg], 1u);
        }
      });
      if constexpr (PASS == 5) {
        if (hashed) hflush(u);  // uniform: the giant's mode
      }
    }
  }
  flush();
}

// Passes 3b / 5b: the partial records of the tile passes (gap_giant_tiles_kernel's
// hflush), one workgroup per (giant, chunk of GA_GAGG slots / groups): every tile's
// records of that chunk folded in LDS -- pass 3 the slots' min / max m/z keys, pass 5 the
// groups' fixed-point sums and counts -- then into the slice's words (the tiles that fell
// back to global atomics folded theirs already).  Integer min / max / sums: the same
// words as the atomics gave.
template <int PASS>
__global__ __launch_bounds__(GA_BLOCK) void gap_giant_reduce_kernel(GiantArgs A) {
  static_assert(PASS == 3 || PASS == 5, "passes 3 (slot extents) and 5 (group sums)");
  __shared__ unsigned long long sm[GA_GAGG], si[GA_GAGG];
  __shared__ uint32_t sc[GA_GAGG];
  __shared__ long long tpre[GA_GMAX + 1], cpre[GA_GMAX + 1];
  __shared__ long long ttmp[GA_NW + 1];
  __shared__ long long rs_off[GA_BLOCK];  // per tile of the current batch: its records' byte offset
  __shared__ int rs_a[GA_BLOCK], rs_b[GA_BLOCK];  // and this chunk's record range
  const int tid = threadIdx.x;
  const int ng = min(*A.n_giant, A.gmax);
  long long tc = 0, cc = 0;
  if (PASS == 3 && blockIdx.x == 0 && tid == 0) *A.part_used = 0ull;  // the arena is pass 5's next
  if (tid < ng) {
    const GapGiant& H = A.giants[tid];
    tc = giant_tiles(A, H, PASS);
    const int NE = PASS == 5 ? H.E : H.D;
    const long long nch = (NE + GA_GAGG - 1) / GA_GAGG;
    // the giants whose tiles wrote records (pass 5: the hashed ones, past the LDS pre-sum)
    cc = (tc > 0 && (PASS == 3 || NE > GA_GAGG) && nch <= GA_PCH) ? nch : 0;
  }
  long long tot;
  const long long te = block_exclusive_scan<GA_BLOCK, long long>(tc, ttmp, tot);
  if (tid < ng) tpre[tid] = te;
  const long long ce = block_exclusive_scan<GA_BLOCK, long long>(cc, ttmp, tot);
  if (tid < ng) cpre[tid] = ce;
  if (tid == 0) cpre[ng] = tot;
  __syncthreads();
  for (long long w = blockIdx.x; w < cpre[ng]; w += gridDim.x) {  // uniform
    int lo = 0, hi = ng;  // the giant with cpre[g] <= w < cpre[g + 1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (cpre[mid] <= w) lo = mid; else hi = mid;
    }
    while (lo + 1 < ng && cpre[lo + 1] <= w) ++lo;
    const int g = lo;
    const GapGiant& H = A.giants[g];
    const int k = (int)(w - cpre[g]);
    const int NE = PASS == 5 ? H.E : H.D;
    const int nch = (NE + GA_GAGG - 1) / GA_GAGG;
    const int e0 = k * GA_GAGG, ne = min(NE - e0, GA_GAGG);
    for (int e = tid; e < ne; e += GA_BLOCK) { sm[e] = PASS == 5 ? 0ull : ~0ull; si[e] = 0ull; sc[e] = 0u; }
    __syncthreads();
    const long long tiles = giant_tiles(A, H, PASS);
    const long long hbytes = ((long long)(nch + 1) * 4 + 15) / 16 * 16;
    // GA_BLOCK tiles at a time: thread t reads tile t's offset and this chunk's record
    // range (one dependent chain for all of them), then every wave folds whole runs
    for (long long t0 = 0; t0 < tiles; t0 += GA_BLOCK) {  // uniform
      const long long t = t0 + tid;
      long long off = -1;
      int a = 0, b = 0;
      if (t < tiles) {
        off = A.tile_off[tpre[g] + t];
        if (off >= 0) {
          const uint32_t* hdr = reinterpret_cast<const uint32_t*>(A.part + off);
          a = (int)hdr[k];
          b = (int)hdr[k + 1];
        }
      }
      rs_off[tid] = off + hbytes;
      rs_a[tid] = a;
      rs_b[tid] = off >= 0 ? b : a;
      __syncthreads();
      const int nt = (int)min<long long>(GA_BLOCK, tiles - t0);
      for (int q = wave_id(); q < nt; q += GA_NW) {  // wave-uniform
        const GapPartial* rec = reinterpret_cast<const GapPartial*>(A.part + rs_off[q]);
        for (int r = rs_a[q] + lane_id(); r < rs_b[q]; r += kWave) {
          const GapPartial R = rec[r];
          const int e = (int)R.e - e0;
          if constexpr (PASS == 5) {
            atomicAdd(&sm[e], R.m);
            atomicAdd(&si[e], R.i);
            atomicAdd(&sc[e], R.c);
          } else {
            atomicMin(&sm[e], R.m);
            atomicMax(&si[e], R.i);
          }
        }
      }
      __syncthreads();  // the run table is refilled
    }
    const GapState<uint32_t> S = gap_slice_state(A.arena + H.off, A.wcap, H.dcap);
    for (int e = tid; e < ne; e += GA_BLOCK) {
      if constexpr (PASS == 5) {
        if (sc[e]) {
          S.kmin[e0 + e] += sm[e];
          S.kmax[e0 + e] += si[e];
          S.gcnt[e0 + e] += sc[e];
        }
      } else if (sm[e] != ~0ull) {
        S.kmin[e0 + e] = min((unsigned long long)S.kmin[e0 + e], sm[e]);
        S.kmax[e0 + e] = max((unsigned long long)S.kmax[e0 + e], si[e]);
      }
    }
    __syncthreads();  // sm/si/sc are zeroed for the next chunk
  }
}

// The per-giant steps, a workgroup per giant: STEP 0 the bitmap prefix (and the
// slots zeroed), 4 the gaps and groups, 6 the emit, precursor and status.
template <int STEP>
__global__ __launch_bounds__(GA_BLOCK) void gap_giant_step_kernel(GiantArgs A, PeaksOut out, double* prec_out,
                                                                 int32_t* charge_out, double* rt_out,
                                                                 int32_t* status, int32_t* unresolved) {
  static_assert(STEP == 0 || STEP == 6, "steps 4 and 6a-d run over the flat grid (gap_giant_groups_kernel)");
  __shared__ int tmp[GA_NW + 1];
  __shared__ int votes[2 * GA_NW];
  __shared__ double red[GA_NW * 3];
  __shared__ double stage[GA_BLOCK];
  __shared__ long long sel[4];
  const int tid = threadIdx.x;
  const int ng = min(*A.n_giant, A.gmax);
  for (int g = blockIdx.x; g < ng; g += gridDim.x) {
    GapGiant& H = A.giants[g];
    if (!H.ok) continue;  // uniform
    const int64_t c = H.c;
    const GapState<uint32_t> S = gap_slice_state(A.arena + H.off, A.wcap, H.dcap);
    int32_t st = H.bad ? kNonFinite : H.status;
    if constexpr (STEP == 0) {
      if (st != kOk) continue;
      if (H.hi_key == 0ull) {  // uniform: every m/z non-finite -- one workgroup in step 6 (gap_body_nf)
        __syncthreads();
        if (tid == 0) H.bad = 1;
        continue;
      }
      const GiantExtent X = giant_extent(H, A.P);
      int D = 0;
      if (X.nw > S.wcap) {
        st = kDeferred;
      } else {
        D = bitmap_prefix<GA_BLOCK, uint32_t, false>(S.bitmap, S.wprefix, (int)X.nw, tmp);
        if (D > S.dcap) st = kDeferred;
      }
      if (st == kOk) {
        for (int d = tid; d < D; d += GA_BLOCK) {
          S.cnt[d] = 0u;
          S.gcnt[d] = 0u;
          S.kmin[d] = ~0ull;
          S.kmax[d] = 0ull;
        }
      }
      if (tid == 0) { H.D = D; H.status = st; }
    } else {
      const int64_t s0 = A.v.cluster_off[c], n = A.v.cluster_off[c + 1] - s0;
      const int64_t p0 = A.v.spec_off[s0], N = A.v.spec_off[A.v.cluster_off[c + 1]] - p0;
      if (H.bad) {  // NaN / inf: one workgroup runs the whole giant in its slice
        st = gap_body_nf(A.v, A.P, S, c, out, tmp, red, votes, reinterpret_cast<uint32_t*>(stage));
        __syncthreads();
      } else if (st == kOk) {
        // the groups were emitted by gap_giant_groups_kernel<4..7>
        (void)n;
        (void)N;
        (void)p0;
        st = H.gany ? kOk : kEmpty;
      }
      if (st == kDeferred) {
        if (tid == 0) { status[c] = kDeferred; atomicAdd(unresolved, 1); }
      } else {
        gap_finish<uint32_t>(A.v, A.P, c, st, out, prec_out, charge_out, rt_out, status, nullptr, nullptr, stage,
                             sel);
      }
    }
    __syncthreads();  // the LDS is reused by the next giant
  }
}

// Step 4 of the giants over a flat (giant, chunk of GA_GCH slots) space instead of one
// workgroup per giant (whose 56 rounds of block scans over a 229k-slot giant made it a
// latency chain, 0.24 ms for the skewed configs[3] batch): (a) per chunk, the gaps
// inside it and any bucket wider than mz_accuracy; (b) per giant, the chunks' exclusive
// bases, the group count E and the status; (c) per chunk, each slot's emitted group
// and the group counts; (d) per chunk of E, the group-sum words zeroed (after (c) has
// read every slot's extent).  The same gaps, groups and counts as gap_groups<false>.
// LDS prefix over the giants of their chunk counts (of D slots, or of E groups);
// pre[ng] = the total.  Call with the whole workgroup.
__device__ __forceinline__ int giant_chunk_prefix(const GiantArgs& A, int* pre, int* tmp, bool of_groups) {
  const int ng = min(*A.n_giant, A.gmax);
  const int t = threadIdx.x;
  int cnt = 0;
  if (t < ng) {
    const GapGiant& H = A.giants[t];
    if (H.ok && !H.bad && H.status == kOk) cnt = ((of_groups ? H.E : H.D) + GA_GCH - 1) / GA_GCH;
  }
  int total;
  const int e = block_exclusive_scan<GA_BLOCK, int>(cnt, tmp, total);
  if (t < ng) pre[t] = e;
  if (t == 0) pre[ng] = total;
  __syncthreads();
  return ng;
}
__device__ __forceinline__ int giant_chunk_owner(const int* pre, int ng, int t) {
  int lo = 0, hi = ng;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (pre[mid] <= t) lo = mid; else hi = mid;
  }
  while (lo + 1 < ng && pre[lo + 1] <= t) ++lo;
  return lo;
}

template <int PART>
__global__ __launch_bounds__(GA_BLOCK) void gap_giant_groups_kernel(GiantArgs A) {
  static_assert(GA_GMAX <= GA_BLOCK, "one thread per giant record");
  __shared__ int pre[GA_GMAX + 1];
  __shared__ int tmp[GA_NW + 1];
  __shared__ int votes[2 * GA_NW];
  __shared__ uint32_t nf_prev, nf_wave[GA_NW];  // steps 6a-d of a giant with non-finite values
  const int tid = threadIdx.x;
  const double acc = A.P.mz_accuracy;
  auto key = [&](const uint64_t* a, int d) { return f64_from_order_key(a[d]); };
  if constexpr (PART == 6) {  // (6c) one workgroup per giant: the kept groups' output bases, the count
    const int ng = min(*A.n_giant, A.gmax);
    for (int g = blockIdx.x; g < ng; g += gridDim.x) {
      GapGiant& H = A.giants[g];
      if (!H.ok || H.bad || H.status != kOk || !H.gany) continue;  // uniform
      const GapSliceLayout Lo = gap_slice_layout(A.wcap, H.dcap);
      int* ch = reinterpret_cast<int*>(A.arena + H.off + Lo.chunks);
      const int nch = (H.E + GA_GCH - 1) / GA_GCH;
      if (tid < kWave) {
        int carry = 0;
        for (int k0 = 0; k0 < nch; k0 += kWave) {
          const int k = k0 + tid;
          const int x = k < nch ? ch[k] : 0;
          const int inc = wave_inclusive_sum(x);
          if (k < nch) ch[k] = carry + inc - x;
          carry += __shfl(inc, kWave - 1, kWave);
        }
        if (tid == 0) A.out_count[H.c] = carry;
      }
    }
    return;
  } else if constexpr (PART == 1) {  // (b) one workgroup per giant: the chunk bases, E, the status
    const int ng = min(*A.n_giant, A.gmax);
    for (int g = blockIdx.x; g < ng; g += gridDim.x) {
      GapGiant& H = A.giants[g];
      if (!H.ok || H.bad || H.status != kOk) continue;  // uniform
      const GapSliceLayout Lo = gap_slice_layout(A.wcap, H.dcap);
      int* ch = reinterpret_cast<int*>(A.arena + H.off + Lo.chunks);
      const int nch = (H.D + GA_GCH - 1) / GA_GCH;
      if (tid < kWave) {
        int carry = 0;
        for (int k0 = 0; k0 < nch; k0 += kWave) {
          const int k = k0 + tid;
          const int x = k < nch ? ch[k] : 0;
          const int inc = wave_inclusive_sum(x);
          if (k < nch) ch[k] = carry + inc - x;
          carry += __shfl(inc, kWave - 1, kWave);
        }
        if (tid == 0) {
          // the true groups' boundaries: after the -inf peaks, the finite gaps, before the
          // +inf peaks (gap_body_nf; 0 and 0 for a finite giant)
          const int b0 = H.n_ninf > 0 ? 1 : 0, be = H.n_pinf > 0 ? 1 : 0;
          const int M = b0 + carry + be;
          H.M = M;
          H.b0 = b0;
          if (H.pad) H.status = kDeferred;  // a bucket spans mz_accuracy
          else if (M == 0) H.status = kNoGap;
          else if ((M >= 2 ? M : 2) > H.dcap) H.status = kDeferred;  // the group words hold dcap
          else H.E = M >= 2 ? M : 2;
        }
      }
    }
    return;
  } else {
    const int ng = giant_chunk_prefix(A, pre, tmp, PART >= 3);
    const int total = pre[ng];
    for (int t = blockIdx.x; t < total; t += gridDim.x) {  // uniform
      const int g = giant_chunk_owner(pre, ng, t);
      GapGiant& H = A.giants[g];
      const int k = t - pre[g];
      const GapState<uint32_t> S = gap_slice_state(A.arena + H.off, A.wcap, H.dcap);
      const GapSliceLayout Lo = gap_slice_layout(A.wcap, H.dcap);
      int* ch = reinterpret_cast<int*>(A.arena + H.off + Lo.chunks);
      const int D = H.D;
      const int db = k * GA_GCH + tid * 8;
      if constexpr (PART == 3) {  // (d) the group-sum words
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = db + q;
          if (e < H.E) { S.kmin[e] = 0ull; S.kmax[e] = 0ull; S.flags[e] = 0u; }
        }
        continue;
      }
      if constexpr (PART >= 4) {  // step 6 over chunks of the E groups (gap_emit's three sweeps)
        const int64_t c = H.c;
        const int64_t s0 = A.v.cluster_off[c], n = A.v.cluster_off[c + 1] - s0;
        const int64_t p0 = A.v.spec_off[s0], N = A.v.spec_off[A.v.cluster_off[c + 1]] - p0;
        const GiantExtent X = giant_extent(H, A.P);
        int ex_m, ex_i;
        frexp(fmax(fabs(X.lo), fabs(X.hi)) * (double)N, &ex_m);
        frexp(X.imax * (double)N, &ex_i);
        const int sc_m = 61 - ex_m, sc_i = 61 - ex_i;
        const double min_len = A.P.min_fraction * (double)n;
        const int E = H.E;
        auto isum = [&](int e) -> double { return ldexp((double)(int64_t)S.kmax[e], -sc_i); };
        // a giant with non-finite values (round 6): each group's values are what the
        // reference's cumsum differences give (nf_value, gap_body_nf's step 6), from the
        // classes of the groups before it -- the chunks before this one and this chunk's
        // groups before the thread's first
        const bool nfg = H.nf != 0;  // uniform
        uint32_t pf = 0u;
        if (nfg) {
          if (tid == 0) nf_prev = 0u;
          __syncthreads();
          uint32_t a = 0u;
          for (int e = tid; e < k * GA_GCH && e < E; e += GA_BLOCK) a |= S.flags[e];
          if (a) atomicOr(&nf_prev, a);
          uint32_t own = 0u;
#pragma unroll
          for (int q = 0; q < 8; ++q) own |= db + q < E ? S.flags[db + q] : 0u;
          uint32_t x = own;  // the wave's inclusive OR scan
#pragma unroll
          for (int o = 1; o < kWave; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, kWave);
            if (lane_id() >= o) x |= y;
          }
          uint32_t ex_or = __shfl_up(x, 1, kWave);
          if (lane_id() == 0) ex_or = 0u;
          if (lane_id() == kWave - 1) nf_wave[wave_id()] = x;
          __syncthreads();
          pf = nf_prev | ex_or;
          for (int w = 0; w < wave_id(); ++w) pf |= nf_wave[w];
        }
        auto values = [&](int e, uint32_t pre, double& vm, double& vi) {
          const double fm = ldexp((double)(int64_t)S.kmin[e], -sc_m) / (double)S.gcnt[e];
          const double fi = isum(e) / (double)n;
          if (!nfg) {
            vm = fm;
            vi = fi;
          } else {
            const uint32_t gf = S.flags[e];
            vm = nf_value(pre, gf, fm);
            vi = nf_value(pre >> 3, gf >> 3, fi);
          }
        };
        if constexpr (PART == 4) {  // (6a) the largest kept group intensity, any kept group
          double gm = -__longlong_as_double(0x7ff0000000000000ll);
          int anyg = 0, gn = 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int e = db + q;
            if (e < E && (double)S.gcnt[e] >= min_len) {
              double vm, vi;
              values(e, pf, vm, vi);
              if (isnan(vi)) gn = 1;  // np.max propagates NaN: nothing is kept
              else gm = fmax(gm, vi);
              anyg = 1;
            }
            if (nfg && e < E) pf |= S.flags[e];
          }
          gm = wave_max_dpp(gm);
          const unsigned long long any_w = __ballot(anyg);
          const unsigned long long nan_w = __ballot(gn);
          if (lane_id() == 0 && any_w) {
            atomicMax(&H.gmax_key, f64_order_key(gm));
            atomicOr(&H.gany, 1);
          }
          if (lane_id() == 0 && nan_w) atomicOr(&H.gnan, 1);
          continue;
        }
        if (!H.gany) continue;  // uniform: kEmpty (the per-giant step reports it)
        // a kept NaN intensity makes the threshold NaN: nothing passes `>=`
        const double thr = H.gnan ? nan_d() : f64_from_order_key(H.gmax_key) / A.P.dyn_range;
        int keep[8], mine = 0;
        double kvm[8], kvi[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = db + q;
          keep[q] = 0;
          if (e < E) {
            values(e, pf, kvm[q], kvi[q]);
            keep[q] = (double)S.gcnt[e] >= min_len && kvi[q] >= thr;
            if (nfg) pf |= S.flags[e];
          }
          mine += keep[q];
        }
        int tot;
        const int ex = block_exclusive_scan<GA_BLOCK, int>(mine, tmp, tot);
        if constexpr (PART == 5) {  // (6b) kept groups per chunk
          if (tid == 0) ch[k] = tot;
        } else {  // (6d) the kept groups in order
          int o = ch[k] + ex;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if (keep[q]) {
              SPX_GUARD(o < N, "giant out c=%ld o=%d N=%ld\n", (long)c, o, (long)N)
              A.out_mz[p0 + o] = kvm[q];
              A.out_int[p0 + o] = kvi[q];
              ++o;
            }
          }
        }
        __syncthreads();
        continue;
      }
      int f[8], mine = 0, split = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // f[q]: a gap between slots d - 1 and d
        const int d = db + q;
        f[q] = d > 0 && d < D && (key(S.kmin, d) - key(S.kmax, d - 1)) >= acc;
        mine += f[q];
        if constexpr (PART == 0) split |= d < D && (key(S.kmax, d) - key(S.kmin, d)) >= acc;
      }
      int tot;
      const int ex = block_exclusive_scan<GA_BLOCK, int>(mine, tmp, tot);
      if constexpr (PART == 0) {  // (a)
        if (block_any<GA_BLOCK, false>(split, votes, 1) && tid == 0) atomicOr(&H.pad, 1);
        if (tid == 0) ch[k] = tot;
      } else {  // (c)
        int gg = H.b0 + ch[k] + ex;
        const int E = H.E;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int d = db + q;
          if (d < D) {
            gg += f[q];
            const int eg = min(gg, E - 1);
            if (const uint32_t k_cnt = S.cnt[d]) atomicAdd(&S.gcnt[eg], k_cnt);  // giants count in pass 5
            S.cnt[d] = (uint32_t)eg;
          }
        }
      }
      __syncthreads();  // tmp / votes reused by the next chunk
    }
  }
}

// A giant's record and arena slice (the global kernel's hand-off and the intake's): 1 if
// taken, 0 if the record table or the arena is full (the cluster then stays where it is).
__device__ __forceinline__ int giant_register(int64_t c, int64_t N, GapGiant* giants, int32_t* n_giant, int gmax,
                                              unsigned long long* arena_used, long long arena_bytes, int wcap) {
  const int g = atomicAdd(n_giant, 1);
  if (g >= gmax) return 0;
  const int dg = (int)(N < (int64_t)wcap * 64 ? N : (int64_t)wcap * 64);  // D <= both
  const long long need = (long long)gap_slice_layout(wcap, dg).total;
  const long long off = (long long)atomicAdd(arena_used, (unsigned long long)need);
  if (off + need > arena_bytes) return 0;
  GapGiant& H = giants[g];
  H.c = (int32_t)c;
  H.dcap = dg;
  H.off = off;
  H.ok = 1;
  return 1;
}

// The giant intake (round 6): clusters of at least 2 spectra registered as giants up
// front, so their pipeline runs on the call's second stream BESIDE the LDS and wide
// kernels instead of after them.  TIER 0 takes every cluster of more than own_n peaks --
// what the LDS and wide kernels only pass on (one the table or the arena cannot take goes
// on the global kernel's list, which the main stream reads after the intake).  TIER 1,
// launched after it, takes clusters of (own_lo, own_n] peaks while the table has room --
// the skewed law's clusters of a few hundred spectra, whose 0.01-Da buckets often outgrow
// the wide kernel's LDS, which would then hand them on after reading them -- and marks
// them in `owned`, which the wide kernel reads (after the intake) to leave them alone.
template <int TIER>
__global__ __launch_bounds__(256) void gap_giant_intake_kernel(CsrView v, int64_t own_n, int64_t own_lo,
                                                               GapGiant* giants, int32_t* n_giant, int gmax,
                                                               unsigned long long* arena_used, long long arena_bytes,
                                                               int wcap, int32_t* deferred, int32_t* n_deferred,
                                                               uint8_t* owned) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < v.n_clusters;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    if (s1 - s0 < 2) continue;
    const int64_t N = v.spec_off[s1] - v.spec_off[s0];
    if (TIER == 0 ? N <= own_n : (N <= own_lo || N > own_n)) continue;
    if (TIER == 1 && *n_giant >= gmax) continue;  // (a stale read only costs a failed registration)
    if (giant_register(c, N, giants, n_giant, gmax, arena_used, arena_bytes, wcap)) owned[c] = 1;
    else if (TIER == 0) deferred[atomicAdd(n_deferred, 1)] = (int32_t)c;
  }
}

__global__ __launch_bounds__(GA_BLOCK) void gap_average_global_kernel(CsrView v, GapParams P, PeaksOut out,
                                                                      double* prec_out, int32_t* charge_out,
                                                                      double* rt_out, int32_t* status,
                                                                      const int32_t* deferred,
                                                                      const int32_t* n_deferred, char* scratch,
                                                                      int64_t slice_bytes, int wcap, int dcap,
                                                                      int32_t* unresolved, GapGiant* giants,
                                                                      int32_t* n_giant, int gmax,
                                                                      unsigned long long* arena_used,
                                                                      long long arena_bytes) {
  __shared__ int tmp[GA_BLOCK / kWave + 1];
  __shared__ int votes[2 * GA_NW];
  __shared__ double red[GA_BLOCK / kWave * 3];
  __shared__ double stage[GA_BLOCK];
  __shared__ long long sel[4];
  __shared__ int handed;
  const GapState<uint32_t> S = gap_slice_state(scratch + (int64_t)blockIdx.x * slice_bytes, wcap, dcap);
  const int32_t nd = *n_deferred;
  for (int32_t i = blockIdx.x; i < nd; i += gridDim.x) {
    const int64_t c = deferred[i];
    const int64_t s0 = v.cluster_off[c], s1 = v.cluster_off[c + 1];
    const int64_t N = v.spec_off[s1] - v.spec_off[s0];
    if (s1 - s0 >= 2 && N > GA_GIANT_N) {  // uniform: hand it to the giant pipeline if it fits
      if (threadIdx.x == 0) handed = giant_register(c, N, giants, n_giant, gmax, arena_used, arena_bytes, wcap);
      __syncthreads();
      const int h = handed;
      __syncthreads();
      if (h) continue;
    }
    int32_t st = gap_body<GA_UM, false>(v, P, S, c, out, tmp, red, votes);
    if (st == kNonFinite) {
      __syncthreads();
      st = gap_body_nf(v, P, S, c, out, tmp, red, votes, reinterpret_cast<uint32_t*>(stage));
    }
    if (st == kDeferred) {
      // bucket range beyond the scratch, or a bucket spanning >= mz_accuracy:
      // reported, never approximated (the host re-runs it through the sort path)
      if (threadIdx.x == 0) { status[c] = kDeferred; atomicAdd(unresolved, 1); }
    } else {
      gap_finish<uint32_t>(v, P, c, st, out, prec_out, charge_out, rt_out, status, nullptr, nullptr, stage, sel);
    }
    __syncthreads();
  }
}

__host__ int64_t gap_slice_bytes(int wcap, int dcap) { return gap_slice_layout(wcap, dcap).total; }

}  // namespace spx
