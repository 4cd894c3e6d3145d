// FETCH_SIZE calibration (profiling aid, not part of the engine): stream a
// known number of bytes with the same access widths the engine kernels use
// (8 B/lane f64 loads, and 16 B/lane), so rocprofv3's FETCH_SIZE can be
// converted to bytes for those widths on gfx950 (MI355X_MICROARCH.md: only the
// 16 B/lane case is documented, as exactly 1/2).
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void calib_read_b64(const double* __restrict__ a, int64_t n, double* out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += a[i];
  if (s == 1.2345e300) out[0] = s;  // never true: keeps the loads
}

__global__ void calib_read_b128(const double2* __restrict__ a, int64_t n2, double* out) {
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1.2345e300) out[0] = s;
}

extern "C" int calib_read(const void* a, int64_t bytes, int width, void* out, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (width == 8)
    hipLaunchKernelGGL(calib_read_b64, dim3(4096), dim3(256), 0, s, (const double*)a, bytes / 8, (double*)out);
  else
    hipLaunchKernelGGL(calib_read_b128, dim3(4096), dim3(256), 0, s, (const double2*)a, bytes / 16, (double*)out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
