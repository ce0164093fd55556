// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the engine's
// kernels use (MI355X_MICROARCH.md §HBM calibrates only 16-B-per-lane streams).
// Each kernel moves a known byte count through HBM once: a coalesced grid-stride
// read of a 1 GiB buffer (four times the 256 MiB last-level cache, so nothing is
// served on-die) with 2-, 4-, 8- or 16-byte loads per lane, and coalesced stores
// of 4, 8 and 16 bytes per lane.  Run under rocprofv3 --pmc FETCH_SIZE, then
// WRITE_SIZE (separate passes); scripts/fetch_calib.py divides the known bytes by
// the counters.
//   hipcc -O3 --offload-arch=gfx950 -o build/fetch_calib scripts/ubench/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__device__ __forceinline__ unsigned fold(unsigned short v) { return v; }
__device__ __forceinline__ unsigned fold(unsigned v) { return v; }
__device__ __forceinline__ unsigned fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ unsigned fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// the result is stored only when it equals a value the data never folds to (the
// buffer is zero-filled), so the kernel writes nothing but cannot be elided
template <typename T>
__global__ void k_read(const T* __restrict__ p, size_t n, unsigned magic, unsigned* out) {
  unsigned acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) acc ^= fold(p[i]);
  if (acc == magic) out[threadIdx.x] = acc;
}

template <typename T>
__global__ void k_write(T* __restrict__ p, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  T v;
  memset(&v, 0x5A, sizeof(T));
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = v;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* buf = nullptr;
  unsigned* out = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&out, 4096));
  CHK(hipMemset(buf, 0, bytes));
  CHK(hipDeviceSynchronize());
  const dim3 g(256 * 8 * 4), b(256);
  // names are what scripts/fetch_calib.py matches
  hipLaunchKernelGGL(k_read<unsigned short>, g, b, 0, 0, (const unsigned short*)buf, bytes / 2, 0xDEADBEEFu, out);
  hipLaunchKernelGGL(k_read<unsigned>, g, b, 0, 0, (const unsigned*)buf, bytes / 4, 0xDEADBEEFu, out);
  hipLaunchKernelGGL(k_read<uint2>, g, b, 0, 0, (const uint2*)buf, bytes / 8, 0xDEADBEEFu, out);
  hipLaunchKernelGGL(k_read<uint4>, g, b, 0, 0, (const uint4*)buf, bytes / 16, 0xDEADBEEFu, out);
  hipLaunchKernelGGL(k_write<unsigned>, g, b, 0, 0, (unsigned*)buf, bytes / 4);
  hipLaunchKernelGGL(k_write<uint2>, g, b, 0, 0, (uint2*)buf, bytes / 8);
  hipLaunchKernelGGL(k_write<uint4>, g, b, 0, 0, (uint4*)buf, bytes / 16);
  CHK(hipGetLastError());
  CHK(hipDeviceSynchronize());
  printf("{\"bytes_per_kernel\": %zu}\n", bytes);
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
