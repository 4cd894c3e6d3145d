// Streaming-shape calibration (profiling aid, not part of the engine): how fast
// can the cluster-segmented CSR be READ with the access shapes the bin-mean /
// medoid kernels use?  Each kernel reads m/z + intensity (f64) of every peak
// once and keeps a checksum, nothing else.
//   0 flat        grid-stride over both arrays (the chip's streaming ceiling)
//   1 cl_flat     one 256-thread block per cluster, peak r = u*256 + tid, 8 in flight
//   2 cl_ring     one block per cluster, lane t = peak t of spectrum j, 8-deep
//                 register ring, LDS-only barrier per spectrum (the fold's shape)
//   3 cl_ring_nb  as 2 without the per-spectrum barrier
//   4 cl_mz       as 1 but m/z only (the bitmap pass)
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ unsigned long long bits(double x) { return (unsigned long long)__double_as_longlong(x); }

__global__ __launch_bounds__(256) void k_flat(const double* __restrict__ mz, const double* __restrict__ it, int64_t n,
                                              unsigned long long* out) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s ^= bits(mz[i]) + bits(it[i]);
  if (s == 0x123456789ull) out[0] = s;
}

__global__ __launch_bounds__(256) void k_cl_flat(const int64_t* __restrict__ coff, const int64_t* __restrict__ soff,
                                                 const double* __restrict__ mz, const double* __restrict__ it,
                                                 int with_int, unsigned long long* out) {
  const int64_t c = blockIdx.x;
  const int64_t p0 = soff[coff[c]], p1 = soff[coff[c + 1]];
  const int np = (int)(p1 - p0);
  unsigned long long s = 0;
  for (int r0 = 0; r0 < np; r0 += 8 * 256) {
    double a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + u * 256 + threadIdx.x;
      const int k = r < np ? r : 0;
      a[u] = mz[p0 + k];
      b[u] = with_int ? it[p0 + k] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s ^= bits(a[u]) + bits(b[u]);
  }
  if (s == 0x123456789ull) out[c] = s;
}

template <bool kBarrier>
__global__ __launch_bounds__(256) void k_cl_ring(const int64_t* __restrict__ coff, const int64_t* __restrict__ soff,
                                                 const double* __restrict__ mz, const double* __restrict__ it,
                                                 unsigned long long* out) {
  __shared__ int so[130];
  const int64_t c = blockIdx.x;
  const int64_t s0 = coff[c], s1 = coff[c + 1];
  const int n = (int)(s1 - s0);
  const int64_t p0 = soff[s0];
  if (n > 128) return;
  for (int j = threadIdx.x; j <= n; j += 256) so[j] = (int)(soff[s0 + j] - p0);
  __syncthreads();
  constexpr int PF = 8;
  auto fetch = [&](int j, double& m, double& x) {
    const int jj = j < n ? j : n - 1;
    const int a = so[jj], e = so[jj + 1];
    const int k = a + (int)threadIdx.x < e ? a + (int)threadIdx.x : a;
    m = mz[p0 + k];
    x = it[p0 + k];
  };
  double M[PF], X[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(q, M[q], X[q]);
  unsigned long long s = 0;
  int jb = 0;
  for (; jb + PF <= n; jb += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      s ^= bits(M[q]) + bits(X[q]);
      fetch(jb + q + PF, M[q], X[q]);
      if (kBarrier) lds_barrier();
    }
  }
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (jb + q < n) s ^= bits(M[q]) + bits(X[q]);
  if (s == 0x123456789ull) out[c] = s;
}

extern "C" int stream_shape(int kind, const void* coff, const void* soff, const void* mz, const void* it,
                            int64_t n_clusters, int64_t n_peaks, void* out, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto C = dim3((unsigned)n_clusters);
  switch (kind) {
    case 0: hipLaunchKernelGGL(k_flat, dim3(8192), dim3(256), 0, s, (const double*)mz, (const double*)it, n_peaks,
                               (unsigned long long*)out); break;
    case 1: hipLaunchKernelGGL(k_cl_flat, C, dim3(256), 0, s, (const int64_t*)coff, (const int64_t*)soff,
                               (const double*)mz, (const double*)it, 1, (unsigned long long*)out); break;
    case 2: hipLaunchKernelGGL(k_cl_ring<true>, C, dim3(256), 0, s, (const int64_t*)coff, (const int64_t*)soff,
                               (const double*)mz, (const double*)it, (unsigned long long*)out); break;
    case 3: hipLaunchKernelGGL(k_cl_ring<false>, C, dim3(256), 0, s, (const int64_t*)coff, (const int64_t*)soff,
                               (const double*)mz, (const double*)it, (unsigned long long*)out); break;
    case 4: hipLaunchKernelGGL(k_cl_flat, C, dim3(256), 0, s, (const int64_t*)coff, (const int64_t*)soff,
                               (const double*)mz, (const double*)it, 0, (unsigned long long*)out); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
