// Wire format of the multi-GPU gather (shard.StepGatherer: every rank's consensus
// peaks travel to rank 0 over xGMI each step; north_star: "RCCL ... to gather
// representatives and consensus peaks back to rank 0").
//
// A bin-mean consensus peak is (fl(f64(M) / c), fl(f64(I) / c)): the float32 bin sums
// M, I of binning.py:198-199 over the c spectra that hit the bin, divided in f64
// (binning.py:211-218; M == 0 gives NaN, :216).  Those two doubles are 16 bytes; the
// gather sends M and I as f32 plus a count c' instead -- 9 bytes (10 past 255
// spectra per cluster) -- and rank 0 rebuilds the doubles with the same division,
// bit for bit.  The link to rank 0 is what bounds the strong-scaled step (xGMI is
// point-to-point: rank 0 takes 7/8 of the batch's consensus peaks over its 7 links),
// so 16 -> 9 bytes is 1.78x less time on it.
//
// The engine's outputs do not carry c.  It is not needed: pack searches the
// smallest c' <= cmax whose f32(x * c') divides back to exactly x for BOTH values.
// The true count always qualifies: x = M / c (1 + d1), fl(x * c) = M (1 + d1)(1 + d2)
// with |d1|, |d2| <= 2^-53, and an f32 M is the only f32 within that relative
// distance, so f32(fl(x * c)) = M and fl(M / c) = x.  Any other c' that passes
// the same exact test rebuilds the same bits, which is all the wire needs (c' is
// typically the odd part of c: M / 2^k is exact in f32).  A cheap filter skips the
// exact test for most c': fl(x * c') must lie within 4 f64 ulps of an f32, i.e.
// its low 29 mantissa bits near 0 or 2^29 (f32 subnormals, zeros and non-finite
// values go straight to the exact test).  A peak no c' <= cmax rebuilds (input
// that is not a bin-mean output) is counted in *n_fail and sent as NaN.
#pragma once
#include "spx_device.hpp"

namespace spx {

constexpr uint64_t kCanonNaN = 0x7ff8000000000000ull;

__device__ __forceinline__ bool near_f32(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint32_t e = (uint32_t)(b >> 52) & 0x7ffu;
  if (e < 1023 - 126 || e == 0x7ffu) return true;  // f32 subnormal / zero range, inf, NaN: exact test
  const uint32_t low = (uint32_t)b & 0x1fffffffu;  // the 29 mantissa bits an f32 does not hold
  return low <= 4u || low >= 0x1fffffffu - 3u;
}

// rank 0's rebuild of one value (shared by pack's exact test and unpack)
__device__ __forceinline__ double wire_mz(float m, uint32_t c) {
  return m == 0.0f ? __longlong_as_double((long long)kCanonNaN) : (double)m / (double)c;
}
__device__ __forceinline__ double wire_int(float i, uint32_t c) { return (double)i / (double)c; }
__device__ __forceinline__ bool same_bits(double a, double b) {
  return __double_as_longlong(a) == __double_as_longlong(b);
}

template <class CT>
__global__ __launch_bounds__(256) void wire_pack_kernel(const double* __restrict__ mz, const double* __restrict__ inten,
                                                        int64_t n, uint32_t cmax, float2* __restrict__ mi,
                                                        CT* __restrict__ cnt, int32_t* __restrict__ n_fail) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const double xm = mz[k], xi = inten[k];
    const bool mnan = (uint64_t)__double_as_longlong(xm) == kCanonNaN;
    float M = 0.0f, I = __int_as_float(0x7fc00000);
    uint32_t c = 0u;
    for (uint32_t cc = 1; cc <= cmax; ++cc) {
      const double ym = xm * (double)cc, yi = xi * (double)cc;
      if (!near_f32(yi) || (!mnan && !near_f32(ym))) continue;
      const float Mc = mnan ? 0.0f : (float)ym, Ic = (float)yi;
      if (same_bits(wire_int(Ic, cc), xi) && (mnan || (Mc != 0.0f && same_bits(wire_mz(Mc, cc), xm)))) {
        M = Mc;
        I = Ic;
        c = cc;
        break;
      }
    }
    if (c == 0u) {
      atomicAdd(n_fail, 1);
      M = __int_as_float(0x7fc00000);
    }
    mi[k] = make_float2(M, I);
    cnt[k] = (CT)c;
  }
}

template <class CT>
__global__ __launch_bounds__(256) void wire_unpack_kernel(const float2* __restrict__ mi, const CT* __restrict__ cnt,
                                                          int64_t n, double* __restrict__ mz,
                                                          double* __restrict__ inten) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const float2 v = mi[k];
    const uint32_t c = (uint32_t)cnt[k];
    mz[k] = wire_mz(v.x, c);
    inten[k] = wire_int(v.y, c);
  }
}

}  // namespace spx
