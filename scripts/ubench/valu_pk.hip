// Issue cost of the VALU forms the strongly-see counts can use (gfx950), one
// workgroup of 1024 threads per CU (4 waves per SIMD, the rounds kernel's shape):
// cycles per wave-instruction per SIMD for 8 independent streams of each form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ void __launch_bounds__(1024) kb(uint32_t* out, uint64_t* cyc, int iters, uint32_t seed) {
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  const uint32_t b = seed * 0x9E3779B9u, one = 0x00010001u;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#define OP(j)                                                                                 \
    if constexpr (K == 0) asm volatile("v_pk_sub_u16 %0, %0, %1 clamp" : "+v"(a##j) : "v"(b)); \
    if constexpr (K == 1) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a##j) : "v"(one));      \
    if constexpr (K == 2) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a##j) : "v"(b));        \
    if constexpr (K == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##j) : "v"(b));           \
    if constexpr (K == 4) asm volatile("v_sub_u16 %0, %0, %1 clamp" : "+v"(a##j) : "v"(b));     \
    if constexpr (K == 5) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##j) : "v"(b), "v"(one)); \
    if constexpr (K == 6) asm volatile("v_dot2_u32_u16 %0, %0, %1, %0" : "+v"(a##j) : "v"(one));
    for (int u = 0; u < 8; u++) { REP8(OP) }
#undef OP
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 1024 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out; uint64_t* cyc;
  hipMalloc(&out, 4 * 1024 * ncu);
  hipMalloc(&cyc, 8 * ncu);
  const char* names[] = {"v_pk_sub_u16 clamp", "v_pk_min_u16", "v_pk_add_u16", "v_add_u32", "v_sub_u16 clamp", "v_perm_b32", "v_dot2_u32_u16"};
  const int iters = 2000;
  for (int k = 0; k < 7; k++) {
    for (int rep = 0; rep < 2; rep++) {
      switch (k) {
        case 0: kb<0><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 1: kb<1><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 2: kb<2><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 3: kb<3><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 4: kb<4><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 5: kb<5><<<ncu, 1024>>>(out, cyc, iters, 7); break;
        case 6: kb<6><<<ncu, 1024>>>(out, cyc, iters, 7); break;
      }
    }
    hipDeviceSynchronize();
    uint64_t c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // per SIMD: 4 waves x iters x 64 instructions
    printf("%-22s %.2f cycles per wave-instruction per SIMD (block 0: %llu cycles)\n", names[k],
           (double)c / (4.0 * iters * 64), (unsigned long long)c);
  }
  return 0;
}
