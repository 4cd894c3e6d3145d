// Shared device-side helpers for the specpride gfx950 kernels.
//
// Everything here is written for CDNA4: 64-lane wavefronts, 256-thread
// workgroups (4 waves, one per SIMD), LDS-resident per-cluster state.  Exact
// IEEE f64 arithmetic is required on the parity path (bin indices, masses,
// precursor means): the library is compiled with -ffp-contract=off and these
// helpers never use fast-math intrinsics.
#pragma once
#include <utility>

#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#ifdef SPX_DEBUG
#include <stdio.h>
// Debug builds only: report an out-of-range index instead of touching memory.
#define SPX_GUARD(cond, ...)        \
  if (!(cond)) {                    \
    printf(__VA_ARGS__);            \
  } else
#else
#define SPX_GUARD(cond, ...)
#endif

namespace spx {

constexpr int kWave = 64;

// Diagnostic builds only (-DSPX_STAMPS, tools/stamps.py): thread 0 of each
// workgroup records the shader clock at phase boundaries, stamps[block * 8 + k].
// Product builds compile SPX_STAMP to nothing.
#ifdef SPX_STAMPS
__device__ unsigned long long* g_spx_stamps;
#define SPX_STAMP(k)                                                                           \
  do {                                                                                         \
    if (threadIdx.x == 0 && g_spx_stamps)                                                      \
      g_spx_stamps[(size_t)blockIdx.x * 8 + (k)] = (unsigned long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define SPX_STAMP(k) \
  do {               \
  } while (0)
#endif
// A stamp that the fused pass's diagnostic build (-DSPX_STAMPS -DSPX_STAMPS_FU) records at
// index `fu` instead of `other` (-1: none), so its eight slots span both methods' phases.
#ifdef SPX_STAMPS_FU
#define SPX_STAMP2(other, fu) \
  do {                        \
    if ((fu) >= 0) SPX_STAMP((fu) < 0 ? 0 : (fu)); \
  } while (0)
#else
#define SPX_STAMP2(other, fu) \
  do {                        \
    if ((other) >= 0) SPX_STAMP((other) < 0 ? 0 : (other)); \
  } while (0)
#endif

// ----------------------------------------------------------------- CSR views
struct CsrView {
  int64_t n_clusters, n_spectra, n_peaks;
  const int64_t* __restrict__ cluster_off;
  const int64_t* __restrict__ spec_off;
  const double* __restrict__ mz;
  const double* __restrict__ inten;
  const double* __restrict__ prec_mz;
  const int32_t* __restrict__ charge;
  const double* __restrict__ rt;
};

// Per-cluster peak output, written at the cluster's own input peak offset
// (capacity of cluster c = its input peak count, so no planning pass).
struct PeaksOut {
  double* __restrict__ mz;
  double* __restrict__ inten;
  int64_t* __restrict__ count;
};

enum : int32_t { kOk = 0, kMixedCharge = 1, kNoGap = 2, kEmpty = 3, kNonFinite = 4, kDeferred = 100 };

// ------------------------------------------------------------ buffer loads
__device__ __forceinline__ double bf_load(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}

// buffer descriptor over n doubles at p, built from readfirstlane'd halves so
// the compiler sees it wave-uniform (readfirstlane returns int: zero-extend the
// low half, a sign-extended one would corrupt the base's upper bits)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bf_rsrc(const double* p, int n) {
  const uint64_t a = (uint64_t)p;
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(lo | (hi << 32)), (short)0,
                                           __builtin_amdgcn_readfirstlane(n * 8), 0x00020000);
}


// --------------------------------------------------------- wave primitives
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
// lane i receives lane i+1's value (DPP wave_shl:1, a VALU op: no LDS round
// trip as __shfl_down's ds_bpermute costs); lane 63 receives `old`.  Call with
// the whole wave active.
__device__ __forceinline__ int32_t wave_next(int32_t x, int32_t old) {
  return __builtin_amdgcn_update_dpp(old, x, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ int wave_id() { return threadIdx.x / kWave; }

// ---- DPP wave reductions / scans (no LDS round trip, unlike __shfl's ds_bpermute).
// GFX9 DPP controls: row_shr:n = 0x110 + n, row_bcast:15 = 0x142, row_bcast:31 = 0x143.
// Lanes whose DPP source is outside the row (or whose row is masked off) get `old`
// (the identity), so each step is x = op(x, shifted) (Hillis-Steele).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64(double old, double x) {
  const uint64_t o = (uint64_t)__double_as_longlong(old), v = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = dpp_u32<CTRL, ROWMASK>((uint32_t)o, (uint32_t)v);
  const uint32_t hi = dpp_u32<CTRL, ROWMASK>((uint32_t)(o >> 32), (uint32_t)(v >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// inclusive scan over the wave (lane 63 holds the total)
template <class T, class Op>
__device__ __forceinline__ T wave_scan_dpp(T x, T ident, Op op) {
  auto step = [&](auto ctrl_c, auto mask_c) __attribute__((always_inline)) {
    constexpr int C = decltype(ctrl_c)::value, M = decltype(mask_c)::value;
    if constexpr (sizeof(T) == 8) {
      x = op(x, dpp_f64<C, M>(ident, x));
    } else {
      x = op(x, (T)dpp_u32<C, M>((uint32_t)ident, (uint32_t)x));
    }
  };
  step(std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xA>{});
  step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xC>{});
  return x;
}

// OR of `val` over each run of consecutive lanes holding the same `key` (a segmented
// Hillis-Steele scan on the DPP steps of wave_scan_dpp); true on the lane that ends
// its run, which then holds the OR of the run.  Lanes of one key that are not
// contiguous end runs of their own (each a correct partial OR).  Keys must differ
// from 0xFFFFFFFF; call with the whole wave active.  This turns a wave's LDS atomic
// ORs into one word from many lanes (which serialise) into one atomic per run.
__device__ __forceinline__ bool wave_or_runs(uint32_t key, uint32_t& val) {
  auto step = [&](auto ctrl_c, auto mask_c) __attribute__((always_inline)) {
    constexpr int C = decltype(ctrl_c)::value, M = decltype(mask_c)::value;
    const uint32_t k2 = dpp_u32<C, M>(0xFFFFFFFFu, key), v2 = dpp_u32<C, M>(0u, val);
    if (k2 == key) val |= v2;
  };
  step(std::integral_constant<int, 0x111>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x112>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x114>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x118>{}, std::integral_constant<int, 0xF>{});
  step(std::integral_constant<int, 0x142>{}, std::integral_constant<int, 0xA>{});
  step(std::integral_constant<int, 0x143>{}, std::integral_constant<int, 0xC>{});
  return (uint32_t)wave_next((int32_t)key, -1) != key;
}

// Inclusive wave scan: DPP for 32-bit integers (kDpp), else ds_bpermute shuffles.
// The register bin-mean kernel measured 1% faster with the shuffle form (its
// LDS round trips overlap the surrounding VALU work), the others 2-3% faster
// with DPP (A/B, tools/gpu/ab.sh).
template <class T, bool kDpp = true>
__device__ __forceinline__ T wave_inclusive_sum(T x) {
  if constexpr (kDpp && std::is_integral<T>::value && sizeof(T) == 4) {
    return wave_scan_dpp(x, T(0), [](T a, T b) { return a + b; });
  } else {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      T y = __shfl_up(x, o, kWave);
      if (lane_id() >= o) x += y;
    }
    return x;
  }
}

// f(integral_constant<int, J>) for J = 0, 1, ... while J < n (n <= sizeof...(Js)):
// a compile-time-unrolled loop with a uniform early exit.  Register arrays are
// indexed by the constant J, and after the exit nothing is merged back (a
// prefetch ring read inside f never becomes a phi of a fresh load and an old
// value, which would compile to a wait for the load right after issuing it).
template <class F, int... Js>
__device__ __forceinline__ void unrolled_while(int n, F&& f, std::integer_sequence<int, Js...>) {
  // each step re-reads n through an empty asm: the compiler cannot evaluate the
  // 64 uniform guards up front (64 live SGPR pairs, which spill)
  int nn = __builtin_amdgcn_readfirstlane(n);
  auto more = [&](int j) __attribute__((always_inline)) {
    asm volatile("" : "+s"(nn));
    return j < nn;
  };
  (void)((more(Js) ? (f(std::integral_constant<int, Js>{}), true) : false) && ...);
}

// ------------------------------------------------------ striped cluster lists
// A per-cluster kernel hands the clusters it does not take to the next kernel
// through a list.  One append counter for the whole grid serialises every
// workgroup on one L2 atomic: 20,000 workgroups deferring 600-peak clusters spent
// 230 us in the register bin-mean kernel that way (~10 ns per append).  Appends
// spread over kListStripes counters, one 256-B line apart; stripe k = c mod
// kListStripes holds its entries at items[k * cap, k * cap + count_k).
constexpr int kListStripes = kWave;  // the consumer's prefix is one wave scan
constexpr int kListLine = 64;        // int32 per counter: 256 B apart
constexpr int64_t kListCountBytes = (int64_t)kListStripes * kListLine * 4;
struct StripedList {
  int32_t* items;
  int32_t* counts;  // counts[k * kListLine]
  int32_t cap;      // entries per stripe: ceil(C / kListStripes)
};
__host__ __device__ inline int32_t striped_cap(int64_t C) {
  return (int32_t)((C + kListStripes - 1) / kListStripes);
}
__device__ __forceinline__ void striped_push(const StripedList& L, int32_t c) {
  const int k = c & (kListStripes - 1);
  L.items[(int64_t)k * L.cap + atomicAdd(&L.counts[k * kListLine], 1)] = c;
}
// The stripes' exclusive prefix into base[0..kListStripes] (LDS) by the first
// wave, then a barrier: call with the whole workgroup.  Returns the entries.
__device__ __forceinline__ int32_t striped_prefix(const StripedList& L, int32_t* base) {
  if (threadIdx.x < kWave) {
    const int32_t inc = wave_inclusive_sum((int32_t)L.counts[threadIdx.x * kListLine]);
    base[threadIdx.x + 1] = inc;
    if (threadIdx.x == 0) base[0] = 0;
  }
  __syncthreads();
  return base[kListStripes];
}
// entry i (< the total) of the list: stripe k with base[k] <= i < base[k + 1]
__device__ __forceinline__ int32_t striped_at(const StripedList& L, const int32_t* base, int32_t i) {
  int lo = 0, hi = kListStripes;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (base[mid] <= i) lo = mid; else hi = mid;
  }
  return L.items[(int64_t)lo * L.cap + (i - base[lo])];
}

template <class T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}

// lane l receives lane l ^ K's value: DPP quad_perm for K = 1, 2 (no LDS), ds_swizzle's
// bit mode for K = 4, 8, 16 (no address VGPR), ds_bpermute for K = 32
template <int K>
__device__ __forceinline__ double xor_f64(double x) {
  if constexpr (K == 32) {
    return __shfl_xor(x, 32, kWave);
  } else {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    int lo = (int)(uint32_t)u, hi = (int)(uint32_t)(u >> 32);
    if constexpr (K == 1) {
      lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
      hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
    } else if constexpr (K == 2) {
      lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
      hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false);
    } else {
      static_assert(K == 4 || K == 8 || K == 16, "swizzle xor within 32 lanes");
      lo = __builtin_amdgcn_ds_swizzle(lo, 0x001F | (K << 10));  // and 0x1F, xor K
      hi = __builtin_amdgcn_ds_swizzle(hi, 0x001F | (K << 10));
    }
    return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
  }
}

// wave_sum's butterfly (xor 32, 16, ..., 1: the same additions in the same order,
// so the same bits) with DPP/swizzle moves for all but the first step
__device__ __forceinline__ double wave_sum_f64(double x) {
  x += xor_f64<32>(x);
  x += xor_f64<16>(x);
  x += xor_f64<8>(x);
  x += xor_f64<4>(x);
  x += xor_f64<2>(x);
  x += xor_f64<1>(x);
  return x;
}

__device__ __forceinline__ double wave_max(double x) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) {
    double y = __shfl_xor(x, o, kWave);
    x = (y > x || (y != y)) ? y : x;  // NaN propagates like numpy max
  }
  return x;
}

__device__ __forceinline__ double wave_min_d(double x) {
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) x = fmin(x, __shfl_xor(x, o, kWave));
  return x;
}

// lane l's value, broadcast (l uniform: v_readlane into scalar registers)
__device__ __forceinline__ int64_t readlane64(int64_t x, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)x >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
  return __longlong_as_double(readlane64(__double_as_longlong(x), l));
}

// wave-wide min (fmin: NaN-ignoring) / max (NaN-propagating, like numpy max),
// broadcast to every lane; DPP, not ds_bpermute
__device__ __forceinline__ double wave_min_dpp(double x) {
  return readlane_f64(wave_scan_dpp(x, __longlong_as_double(0x7ff0000000000000ll),
                                    [](double a, double b) { return fmin(a, b); }), kWave - 1);
}
__device__ __forceinline__ double wave_max_dpp(double x) {
  return readlane_f64(wave_scan_dpp(x, -__longlong_as_double(0x7ff0000000000000ll),
                                    [](double a, double b) { return (b > a || (b != b)) ? b : a; }), kWave - 1);
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a release/acquire
// fence on ALL address spaces: its release waits for every outstanding global
// load (vmcnt), which drains any prefetch in flight.  Steps that exchange data
// only through LDS use this instead, so register prefetches survive it.
// The LDS-scoped fences only pin the compiler's ordering (on gfx950 they emit
// no wait); the explicit lgkmcnt(0) makes this wave's LDS writes complete
// before the barrier releases the other waves.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: vmcnt/expcnt left alone
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Block exclusive scan of one int per thread.  `tmp` holds BLOCK/64 + 1 ints
// in LDS.  Returns the exclusive prefix; `total` receives the block sum.
// kLdsOnly: LDS-only barriers (register prefetches in flight survive them).
template <int BLOCK, class T, bool kLdsOnly = false, bool kDpp = true>
__device__ __forceinline__ T block_exclusive_scan(T v, T* tmp, T& total) {
  static_assert(BLOCK % kWave == 0, "block must be whole waves");
  constexpr int NW = BLOCK / kWave;
  T inc = wave_inclusive_sum<T, kDpp>(v);
  if (lane_id() == kWave - 1) tmp[wave_id()] = inc;
  if constexpr (kLdsOnly) lds_barrier();
  else __syncthreads();
  T base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    T t = tmp[w];
    base += (w < wave_id()) ? t : T(0);
    tot += t;
  }
  if constexpr (kLdsOnly) lds_barrier();
  else __syncthreads();
  total = tot;
  return base + inc - v;
}

// Block-wide OR with ONE barrier: wave ballot, one LDS word per wave, barrier,
// read.  `votes` holds 2 x (BLOCK/64) ints; alternate `parity` between
// consecutive calls so a fast wave's next vote cannot overwrite a word a slow
// wave is still reading.  (hip's __syncthreads_or costs three barriers.)
// kLdsOnly: the barrier may ignore global memory (all shared state is in LDS);
// otherwise it is a full __syncthreads() (state in global scratch).
template <int BLOCK, bool kLdsOnly = true>
__device__ __forceinline__ int block_any(int pred, int* votes, int parity) {
  constexpr int NW = BLOCK / kWave;
  const int w = __ballot(pred) != 0ull;
  if (lane_id() == 0) votes[parity * NW + wave_id()] = w;
  if constexpr (kLdsOnly) lds_barrier();
  else __syncthreads();
  int r = 0;
#pragma unroll
  for (int k = 0; k < NW; ++k) r |= votes[parity * NW + k];
  return r;
}

// ------------------------------------------------------ exact bin indexing
// trunc(fl((m - lo) / w)) and ceil(fl(m / w)) exactly as numpy / OpenMS compute
// them (IEEE subtract + correctly rounded divide), without paying a f64 divide
// per peak.  Exact trunc/floor/ceil of fl(x / w) via the reciprocal product q = x * (1/w):
// for |q| < 2^24, q is within 2^-27 of fl(x / w), so outside a 2^-24 band
// around an integer q's integer part is the answer (32-bit conversion); inside
// the band, or for larger quotients, the correctly rounded division decides.
constexpr double kDivFastLimit = 0x1p24;
constexpr double kDivBand = 0x1p-24;

__device__ __forceinline__ int64_t trunc_div_exact(double x, double w, double inv_w) {
  const double q = x * inv_w;
  const double t = trunc(q);
  const double f = fabs(q - t);
  if (fabs(q) < kDivFastLimit && f > kDivBand && f < 1.0 - kDivBand) return (int64_t)(int32_t)t;
  return (int64_t)trunc(x / w);
}

// trunc(fl(x / w)) for 0 <= x / w < 2^17 (the LDS bin-mean paths).  There the
// reciprocal product q is within 2^-34 of fl(x / w), so outside a 2^-30 band
// around an integer its integer part is the answer; inside the band (1 peak in
// ~10^8 for arbitrary m/z) the correctly rounded division decides.
__device__ __forceinline__ int32_t trunc_div_small(double x, double w, double inv_w) {
  const double q = x * inv_w;
  const double t = trunc(q);
  const double f = q - t;
  if (f > 0x1p-30 && f < 1.0 - 0x1p-30) return (int32_t)t;
  return (int32_t)trunc(x / w);
}

__device__ __forceinline__ int64_t floor_div_exact(double x, double w, double inv_w) {
  const double q = x * inv_w;
  const double t = floor(q);
  const double f = q - t;
  if (fabs(q) < kDivFastLimit && f > kDivBand && f < 1.0 - kDivBand) return (int64_t)(int32_t)t;
  return (int64_t)floor(x / w);
}

__device__ __forceinline__ int64_t ceil_div_exact(double x, double w, double inv_w) {
  const double q = x * inv_w;
  const double t = ceil(q);
  const double f = t - q;
  if (fabs(q) < kDivFastLimit && f > kDivBand && f < 1.0 - kDivBand) return (int64_t)(int32_t)t;
  return (int64_t)ceil(x / w);
}

// ceil_div_exact's fast half alone, for loops that batch the rare division:
// the answer when *sure, else the caller divides (ceil_div_exact).
__device__ __forceinline__ int32_t ceil_div_fast(double x, double inv_w, bool& sure) {
  const double q = x * inv_w;
  const double t = ceil(q);
  const double f = t - q;
  sure = fabs(q) < kDivFastLimit && f > kDivBand && f < 1.0 - kDivBand;
  return __double2int_rz(t);  // saturating conversion: no UB where !sure
}

// f64 <-> order-preserving u64 (for LDS atomic min/max on doubles)
__device__ __forceinline__ uint64_t f64_order_key(double x) {
  uint64_t u = __double_as_longlong(x);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double f64_from_order_key(uint64_t k) {
  uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double(u);
}

// ------------------------------------------------ numpy pairwise summation
// The reduction numpy's add.reduce (np.mean, pandas .sum()) evaluates on a
// float64 vector: n < 8 sequential; n <= 128 eight strided partial sums
// combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a sequential tail; larger n
// split at n2 = n/2 - (n/2)%8 and recursed.  f(j) yields element j.
template <class F>
__device__ __forceinline__ double pw_leaf(const F& f, int64_t lo, int64_t n) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += f(lo + i);
    return r;
  }
  double r0 = f(lo + 0), r1 = f(lo + 1), r2 = f(lo + 2), r3 = f(lo + 3);
  double r4 = f(lo + 4), r5 = f(lo + 5), r6 = f(lo + 6), r7 = f(lo + 7);
  int64_t i = 8;
  const int64_t lim = n - (n % 8);
  for (; i < lim; i += 8) {
    r0 += f(lo + i + 0); r1 += f(lo + i + 1); r2 += f(lo + i + 2); r3 += f(lo + i + 3);
    r4 += f(lo + i + 4); r5 += f(lo + i + 5); r6 += f(lo + i + 6); r7 += f(lo + i + 7);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += f(lo + i);
  return res;
}

// Leaf-only form (n <= 128), usable in kernels that must not touch scratch.
template <class F>
__device__ __forceinline__ double pw_sum_small(const F& f, int64_t n) {
  return 0.0 + pw_leaf(f, 0, n);
}

// numpy's recursion over [0, n) unrolled onto an explicit stack (depth <= 40):
// leaf(lo, m) returns the sum of the leaf segment [lo, lo + m), m <= 128; the
// leaves are visited left to right.  Returns 0.0 + tree (np.add.reduce).
template <class L>
__device__ double pw_tree(const L& leaf, int64_t n) {
  if (n <= 128) return 0.0 + leaf(0, n);
  int64_t lo[40], len[40];
  double left[40];
  int state[40];
  int sp = 0;
  lo[0] = 0; len[0] = n; state[0] = 0;
  for (;;) {
    const int64_t m = len[sp];
    if (m <= 128) {
      double val = leaf(lo[sp], m);
      for (;;) {
        if (sp == 0) return 0.0 + val;
        --sp;
        if (state[sp] == 1) {
          left[sp] = val;
          state[sp] = 2;
          int64_t h = len[sp] / 2;
          h -= h % 8;
          lo[sp + 1] = lo[sp] + h;
          len[sp + 1] = len[sp] - h;
          state[sp + 1] = 0;
          ++sp;
          break;
        }
        val = left[sp] + val;
      }
    } else {
      int64_t h = m / 2;
      h -= h % 8;
      state[sp] = 1;
      lo[sp + 1] = lo[sp];
      len[sp + 1] = h;
      state[sp + 1] = 0;
      ++sp;
    }
  }
}

// General form of numpy's pairwise sum of f(0..n-1).
template <class F>
__device__ double pw_sum(const F& f, int64_t n) {
  return pw_tree([&](int64_t lo, int64_t m) { return pw_leaf(f, lo, m); }, n);
}

// Population count below bit `b` of a u64 bitmap with a per-word exclusive
// prefix: the rank of bin b among the set bits (= its compact slot id).
template <class PrefixT>
__device__ __forceinline__ int bitmap_rank(const unsigned long long* bm, const PrefixT* pref, int64_t b) {
  const int64_t w = b >> 6;
  const unsigned long long mask = (1ull << (b & 63)) - 1ull;
  return (int)pref[w] + __popcll(bm[w] & mask);
}

// The same over 32-bit words, LDS-only barriers.
template <int BLOCK, class PrefixT>
__device__ int bitmap_prefix32(const uint32_t* bm, PrefixT* pref, int nw, int* tmp) {
  const int per = (nw + BLOCK - 1) / BLOCK;
  const int w0 = threadIdx.x * per;
  int local = 0;
  for (int k = 0; k < per; ++k) {
    const int w = w0 + k;
    if (w < nw) local += __popc(bm[w]);
  }
  int total;
  int base = block_exclusive_scan<BLOCK, int, true, false>(local, tmp, total);
  for (int k = 0; k < per; ++k) {
    const int w = w0 + k;
    if (w < nw) {
      pref[w] = (PrefixT)base;
      base += __popc(bm[w]);
    }
  }
  lds_barrier();
  return total;
}

// Exclusive popcount prefix over `nw` bitmap words, in place into `pref`;
// returns the total number of set bits.  Whole block participates.
template <int BLOCK, class PrefixT, bool kLdsOnly = false>
__device__ int bitmap_prefix(const unsigned long long* bm, PrefixT* pref, int nw, int* tmp) {
  const int per = (nw + BLOCK - 1) / BLOCK;
  const int w0 = threadIdx.x * per;
  int local = 0;
  for (int k = 0; k < per; ++k) {
    int w = w0 + k;
    if (w < nw) local += __popcll(bm[w]);
  }
  int total;
  int base = block_exclusive_scan<BLOCK, int, kLdsOnly>(local, tmp, total);
  for (int k = 0; k < per; ++k) {
    int w = w0 + k;
    if (w < nw) {
      pref[w] = (PrefixT)base;
      base += __popcll(bm[w]);
    }
  }
  if constexpr (kLdsOnly) lds_barrier();
  else __syncthreads();
  return total;
}

}  // namespace spx
