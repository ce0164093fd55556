// Microbenchmark: the latency floor of the direct rounds kernel's frontier hand-off
// (hge_rounds_direct.hip) -- 8-byte {epoch, value} granules, relaxed agent-scope
// stores, polled with relaxed agent-scope loads and s_sleep(1), as the kernel does.
//   mode 0 (2 workgroups on different CUs): ping-pong; one hop = half a round trip.
//   mode 1 (G workgroups of 1024 threads, one per CU, like the kernel): every round
//     each workgroup publishes its granule, then each of its 16 waves polls its own
//     G/16 granules until all carry the round's epoch, then a workgroup barrier --
//     the kernel's per-round hand-off with no select, no fetch and no member rows.
// Prints ns per hop (mode 0) and ns / shader cycles per round (mode 1); the
// kernel's measured ~8.5 us per round at 256/10M minus this is the work.
//   granule_hop [G] [rounds]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

typedef __attribute__((address_space(1))) unsigned long long gu64_t;

__device__ __forceinline__ void put(gu64_t* g, unsigned long long v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long get(const gu64_t* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bounded spins: a block that is not resident makes the others give up (err)
__global__ void __launch_bounds__(64) k_pingpong(unsigned long long* gran, int iters, int* err,
                                                 unsigned long long* cyc) {
  gu64_t* g = (gu64_t*)gran;
  const int me = blockIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int e = 1; e <= iters; e++) {
    if (me == 0) {
      if (threadIdx.x == 0) put(g, (unsigned long long)e);
      unsigned spins = 0;
      while (get(g + 1) != (unsigned long long)e) {
        if (++spins > (1u << 22)) { if (threadIdx.x == 0) atomicOr(err, 1); return; }
        __builtin_amdgcn_s_sleep(1);
      }
    } else {
      unsigned spins = 0;
      while (get(g) != (unsigned long long)e) {
        if (++spins > (1u << 22)) { if (threadIdx.x == 0) atomicOr(err, 1); return; }
        __builtin_amdgcn_s_sleep(1);
      }
      if (threadIdx.x == 0) put(g + 1, (unsigned long long)e);
    }
  }
  if (threadIdx.x == 0) cyc[me] = __builtin_amdgcn_s_memtime() - t0;
}

__global__ void __launch_bounds__(1024) k_allgather(unsigned long long* gran, int G, int iters, int* err,
                                                    unsigned long long* cyc) {
  gu64_t* g = (gu64_t*)gran;
  const int c = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int e = 1; e <= iters; e++) {
    gu64_t* gr = g + (size_t)(e & 1) * G;  // double-buffered by round parity, as the kernel
    if (threadIdx.x == 0) put(gr + c, ((unsigned long long)e << 32) | (unsigned)c);
    // wave w polls granules d = 16 w .. 16 w + 15 (lanes 0-15)
    const int d = wave * 16 + lane;
    unsigned spins = 0;
    bool fail = false;
    for (;;) {
      bool ok = true;
      if (lane < 16 && d < G) ok = (unsigned)(get(gr + d) >> 32) == (unsigned)e;
      if (__all(ok)) break;
      if (++spins > (1u << 22)) { fail = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (fail && lane == 0) atomicOr(err, 1);
    __syncthreads();
    if (fail) break;
  }
  if (threadIdx.x == 0) cyc[c] = __builtin_amdgcn_s_memtime() - t0;
}

int main(int argc, char** argv) {
  int G = argc > 1 ? atoi(argv[1]) : 256;
  const int iters = argc > 2 ? atoi(argv[2]) : 4000;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  if (G > ncu) G = ncu;  // one workgroup per CU must fit
  if (G > 256) G = 256;
  unsigned long long *gran, *cyc;
  int* err;
  CK(hipMalloc(&gran, 2 * 256 * 8));
  CK(hipMalloc(&cyc, 256 * 8));
  CK(hipMalloc(&err, 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms0 = 0, ms1 = 0;
  int herr = 0;
  unsigned long long hc[256];
  for (int rep = 0; rep < 2; rep++) {  // the first pass warms clocks and code objects
    CK(hipMemset(gran, 0, 2 * 256 * 8));
    CK(hipMemset(err, 0, 4));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_pingpong, dim3(2), dim3(64), 0, 0, gran, iters, err, cyc);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms0, a, b));
  }
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc, cyc, 16, hipMemcpyDeviceToHost));
  const double hop_ns = ms0 * 1e6 / iters / 2, hop_cyc = (double)hc[0] / iters / 2;
  const int err0 = herr;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipMemset(gran, 0, 2 * 256 * 8));
    CK(hipMemset(err, 0, 4));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_allgather, dim3(G), dim3(1024), 0, 0, gran, G, iters, err, cyc);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms1, a, b));
  }
  CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc, cyc, 8 * (size_t)G, hipMemcpyDeviceToHost));
  double cmax = 0;
  for (int i = 0; i < G; i++) cmax = hc[i] > cmax ? (double)hc[i] : cmax;
  printf("{\"hop_ns\": %.1f, \"hop_memtime_ticks\": %.1f, \"pingpong_err\": %d, \"workgroups\": %d, "
         "\"round_ns\": %.1f, \"round_memtime_ticks\": %.1f, \"allgather_err\": %d, \"rounds\": %d}\n",
         hop_ns, hop_cyc, err0, G, ms1 * 1e6 / iters, cmax / iters, herr, iters);
  return 0;
}
