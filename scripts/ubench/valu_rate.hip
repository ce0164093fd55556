// Microbenchmark: issue rate of the probe's packed 16-bit triple
// (v_pk_sub_u16 clamp, v_pk_min_u16, v_pk_add_u16) vs a 32-bit SWAR triple
// (v_sub_u32, v_and_b32, v_bcnt_u32_b32), 16 waves per CU (the rounds kernel's
// occupancy), cycles per wave-instruction per SIMD from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void __launch_bounds__(1024) kbench(uint32_t* out, uint64_t* cyc, int iters) {
  uint32_t a0 = threadIdx.x * 7 + 1, a1 = a0 * 3, a2 = a0 ^ 0x5555, a3 = a0 + 99;
  uint32_t m0 = 0x00030003u, m1 = 0x00050001u, one = 0x00010001u;
  uint32_t acc0 = 0, acc1 = 0, d0, d1;
  __syncthreads();
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if constexpr (MODE == 0) {
        asm volatile("v_pk_sub_u16 %0, %4, %6 clamp\n\t"
                     "v_pk_sub_u16 %1, %5, %7 clamp\n\t"
                     "v_pk_min_u16 %0, %0, %8\n\t"
                     "v_pk_min_u16 %1, %1, %8\n\t"
                     "v_pk_add_u16 %2, %2, %0\n\t"
                     "v_pk_add_u16 %3, %3, %1"
                     : "=&v"(d0), "=&v"(d1), "+v"(acc0), "+v"(acc1)
                     : "v"(a0), "v"(a1), "v"(m0), "v"(m1), "v"(one));
      } else {
        asm volatile("v_sub_u32 %0, %4, %6\n\t"
                     "v_sub_u32 %1, %5, %7\n\t"
                     "v_and_b32 %0, %0, %8\n\t"
                     "v_and_b32 %1, %1, %8\n\t"
                     "v_bcnt_u32_b32 %2, %0, %2\n\t"
                     "v_bcnt_u32_b32 %3, %1, %3"
                     : "=&v"(d0), "=&v"(d1), "+v"(acc0), "+v"(acc1)
                     : "v"(a2), "v"(a3), "v"(m0), "v"(m1), "v"(one));
      }
    }
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 + acc1;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  uint64_t* cyc;
  hipMalloc(&out, sizeof(uint32_t) * ncu * 1024);
  hipMalloc(&cyc, sizeof(uint64_t) * ncu);
  const int iters = 4096;
  uint64_t h[1024];
  for (int mode = 0; mode < 2; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      if (mode == 0) kbench<0><<<ncu, 1024>>>(out, cyc, iters);
      else kbench<1><<<ncu, 1024>>>(out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(uint64_t) * ncu, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < ncu; i++) s += (double)h[i];
    s /= ncu;
    // per SIMD: 4 waves x iters x 8 x 6 instructions
    const double instr = 4.0 * iters * 8 * 6;
    printf("mode %s: %.2f cycles per wave-instruction per SIMD (%.0f cycles/block)\n",
           mode == 0 ? "pk16 (sub clamp, min, add)" : "swar32 (sub, and, bcnt)", s / instr, s);
  }
  return 0;
}
