// Micro-benchmark: what a kernel boundary costs on this GPU.
// Times (a) a small streaming kernel back-to-back, (b) a kernel with three
// dependent loads per thread, (c) an empty kernel, each averaged over many
// launches on one stream (HIP events), and (d) the same streaming kernel
// launched 64 times inside ONE kernel via a grid-stride repeat.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}

__global__ void k_stream(const int* __restrict__ a, int* __restrict__ b, long long* __restrict__ c, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { b[i] = a[i] + 1; c[i] = a[i]; }
}

__global__ void k_chain(const int* __restrict__ idx, const int* __restrict__ v, int* __restrict__ out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { int x = idx[i]; int y = idx[x]; int z = v[y]; out[i] = z; }
}

__global__ void k_atom1(int* ctr, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(ctr, 1);
}
__global__ void k_atomb(int* ctr, int n, int per) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&ctr[i / per], 1);
}
__global__ void k_atomb_ret(int* ctr, int n, int per, int* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = atomicAdd(&ctr[i / per], 1);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const int n = 100000;
  int *a, *b, *idx, *v, *o; long long* c;
  CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&c, n * 8));
  CK(hipMalloc(&idx, n * 4)); CK(hipMalloc(&v, n * 4)); CK(hipMalloc(&o, n * 4));
  std::vector<int> h(n);
  for (int i = 0; i < n; i++) h[i] = (int)((i * 2654435761u) % n);
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(a, 0, n * 4));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int it = 200;
  dim3 g((n + 255) / 256), blk(256);
  for (int w = 0; w < 20; w++) hipLaunchKernelGGL(k_stream, g, blk, 0, s, a, b, c, n);
  CK(hipStreamSynchronize(s));
  float ms;
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("empty kernel        : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_empty, g, blk, 0, s);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("empty 391x256 grid  : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_stream, g, blk, 0, s, a, b, c, n);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("stream 100k (1.6MB) : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_chain, g, blk, 0, s, idx, v, o, n);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("3-level gather 100k : %.2f us per launch\n", ms * 1000 / it);
  int* ctr; CK(hipMalloc(&ctr, 4096 * 4)); CK(hipMemset(ctr, 0, 4096 * 4));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_atom1, g, blk, 0, s, ctr, n);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("100k atomicAdd, 1 address          : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_atomb, g, blk, 0, s, ctr, n, 139);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("100k atomicAdd, 720 addresses      : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_atomb_ret, g, blk, 0, s, ctr, n, 139, o);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("100k atomicAdd w/ return, 720 addr : %.2f us per launch\n", ms * 1000 / it);
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < it; r++) hipLaunchKernelGGL(k_atomb_ret, g, blk, 0, s, ctr, n, 16, o);
  CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  printf("100k atomicAdd w/ return, 6250 addr: %.2f us per launch\n", ms * 1000 / it);
  // single launch timing with events around each (as the engine's profiler does)
  float tot = 0;
  for (int r = 0; r < 50; r++) {
    CK(hipEventRecord(e0, s));
    hipLaunchKernelGGL(k_stream, g, blk, 0, s, a, b, c, n);
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    tot += ms;
  }
  printf("stream, event-bracketed single launch: %.2f us\n", tot * 1000 / 50);
  return 0;
}
