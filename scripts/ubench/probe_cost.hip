// Microbenchmark of one strongly-see probe of the direct rounds kernel at N = 256
// (1024 threads = 256 members x 4 parts, 32 packed words per thread): cycles per
// probe for the full probe and with parts removed, to see what bounds it.
//   mode 0: LDS slice reads + packed compares + DPP sum + ballot + barrier + read
//   mode 1: no LDS slice reads (compares on registers)
//   mode 2: no compares (LDS reads summed with one add per word)
//   mode 3: barrier + counter exchange only
//   mode 4: slice read by 8 lanes + v_readlane broadcast (single-part waves)
//   mode 5: mode 0 with 4-word asm blocks and 4 accumulators
//   mode 6: two positions per probe (independent chains interleaved), per position
//   mode 7: 8-bit SWAR compares (16 words: (la | 0x80..) - m, & 0x80.., bcnt)
//   mode 8: mode 0 with 32-bit ops in place of the packed ones (sub, min, add)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int BS = 1024, CW = 32, PS = CW + 4, RS = 4 * PS, W = 64;

template <int MODE>
__global__ void __launch_bounds__(1024) kprobe(uint32_t* out, uint64_t* cyc, int iters) {
  __shared__ uint32_t ring[W * RS];
  __shared__ int cntw[32][16];
  const int tid = threadIdx.x, part = tid & 3;
  for (int i = tid; i < W * RS; i += BS) ring[i] = i * 2654435761u;
  uint32_t mw[CW];
#pragma unroll
  for (int k = 0; k < CW; k++) mw[k] = (tid * 31 + k) * 0x00010001u;
  __syncthreads();
  int p = 17, tot = 0;
  const uint32_t ones = 0x00010001u;
  const uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; it++) {
    uint32_t acc0 = 0, acc1 = 0;
    if constexpr (MODE == 0 || MODE == 1 || MODE == 2) {
      const uint32_t* src = ring + (p & (W - 1)) * RS + part * PS;
      uint32_t la[CW];
#pragma unroll
      for (int k = 0; k < CW; k += 4) {
        if constexpr (MODE == 1) {
          la[k] = mw[k] ^ p; la[k + 1] = mw[k + 1] + p; la[k + 2] = mw[k + 2] - p; la[k + 3] = mw[k + 3] | p;
        } else {
          const uint4 q = *(const uint4*)(src + k);
          la[k] = q.x; la[k + 1] = q.y; la[k + 2] = q.z; la[k + 3] = q.w;
        }
      }
      if constexpr (MODE == 2) {
#pragma unroll
        for (int k = 0; k < CW; k++) acc0 += la[k];
      } else {
#pragma unroll
        for (int k = 0; k < CW; k += 2) {
          uint32_t d0, d1;
          asm volatile("v_pk_sub_u16 %0, %4, %6 clamp\n\tv_pk_sub_u16 %1, %5, %7 clamp\n\t"
                       "v_pk_min_u16 %0, %0, %8\n\tv_pk_min_u16 %1, %1, %8\n\t"
                       "v_pk_add_u16 %2, %2, %0\n\tv_pk_add_u16 %3, %3, %1"
                       : "=&v"(d0), "=&v"(d1), "+v"(acc0), "+v"(acc1)
                       : "v"(la[k]), "v"(la[k + 1]), "v"(mw[k]), "v"(mw[k + 1]), "v"(ones));
        }
      }
    } else if constexpr (MODE == 5 || MODE == 6) {
      constexpr int NPOS = MODE == 6 ? 2 : 1;
      uint32_t accs[NPOS][4];
#pragma unroll
      for (int q = 0; q < NPOS; q++)
#pragma unroll
        for (int a = 0; a < 4; a++) accs[q][a] = 0;
#pragma unroll
      for (int k = 0; k < CW; k += 4) {
#pragma unroll
        for (int q = 0; q < NPOS; q++) {
          const uint32_t* src = ring + ((p + 7 * q) & (W - 1)) * RS + part * PS;
          const uint4 v = *(const uint4*)(src + k);
          uint32_t d0, d1, d2, d3;
          asm volatile("v_pk_sub_u16 %0, %8, %12 clamp\n\tv_pk_sub_u16 %1, %9, %13 clamp\n\t"
                       "v_pk_sub_u16 %2, %10, %14 clamp\n\tv_pk_sub_u16 %3, %11, %15 clamp\n\t"
                       "v_pk_min_u16 %0, %0, %16\n\tv_pk_min_u16 %1, %1, %16\n\t"
                       "v_pk_min_u16 %2, %2, %16\n\tv_pk_min_u16 %3, %3, %16\n\t"
                       "v_pk_add_u16 %4, %4, %0\n\tv_pk_add_u16 %5, %5, %1\n\t"
                       "v_pk_add_u16 %6, %6, %2\n\tv_pk_add_u16 %7, %7, %3"
                       : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(accs[q][0]), "+v"(accs[q][1]),
                         "+v"(accs[q][2]), "+v"(accs[q][3])
                       : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(mw[k]), "v"(mw[k + 1]), "v"(mw[k + 2]),
                         "v"(mw[k + 3]), "v"(ones));
        }
      }
      acc0 = accs[0][0] + accs[0][1];
      acc1 = accs[0][2] + accs[0][3];
      if constexpr (NPOS == 2) acc0 += accs[1][0] ^ accs[1][1] ^ accs[1][2] ^ accs[1][3];
    } else if constexpr (MODE == 7) {
      const uint32_t* src = ring + (p & (W - 1)) * RS + part * PS;
      const uint32_t hb = 0x80808080u;
#pragma unroll
      for (int k = 0; k < CW / 2; k += 4) {
        const uint4 v = *(const uint4*)(src + k);
        uint32_t d0, d1, d2, d3;
        asm volatile("v_sub_u32 %0, %6, %10\n\tv_sub_u32 %1, %7, %11\n\t"
                     "v_sub_u32 %2, %8, %12\n\tv_sub_u32 %3, %9, %13\n\t"
                     "v_and_b32 %0, %0, %14\n\tv_and_b32 %1, %1, %14\n\t"
                     "v_and_b32 %2, %2, %14\n\tv_and_b32 %3, %3, %14\n\t"
                     "v_bcnt_u32_b32 %4, %0, %4\n\tv_bcnt_u32_b32 %5, %1, %5\n\t"
                     "v_bcnt_u32_b32 %4, %2, %4\n\tv_bcnt_u32_b32 %5, %3, %5"
                     : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(acc0), "+v"(acc1)
                     : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(mw[k]), "v"(mw[k + 1]), "v"(mw[k + 2]),
                       "v"(mw[k + 3]), "v"(hb));
      }
    } else if constexpr (MODE == 8) {
      const uint32_t* src = ring + (p & (W - 1)) * RS + part * PS;
#pragma unroll
      for (int k = 0; k < CW; k += 4) {
        const uint4 v = *(const uint4*)(src + k);
        uint32_t d0, d1, d2, d3;
        asm volatile("v_sub_u32 %0, %6, %10\n\tv_sub_u32 %1, %7, %11\n\t"
                     "v_sub_u32 %2, %8, %12\n\tv_sub_u32 %3, %9, %13\n\t"
                     "v_min_u32 %0, %0, %14\n\tv_min_u32 %1, %1, %14\n\t"
                     "v_min_u32 %2, %2, %14\n\tv_min_u32 %3, %3, %14\n\t"
                     "v_add_u32 %4, %4, %0\n\tv_add_u32 %5, %5, %1\n\t"
                     "v_add_u32 %4, %4, %2\n\tv_add_u32 %5, %5, %3"
                     : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(acc0), "+v"(acc1)
                     : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(mw[k]), "v"(mw[k + 1]), "v"(mw[k + 2]),
                       "v"(mw[k + 3]), "v"(ones));
      }
    } else if constexpr (MODE == 4) {
      // single-part waves: lanes 0..7 read the uniform slice, readlane to SGPRs
      const int wpart = (tid >> 6) >> 2;
      const uint32_t* src = ring + (p & (W - 1)) * RS + wpart * PS;
      const int lane = tid & 63;
      uint4 q = make_uint4(0, 0, 0, 0);
      if (lane < CW / 4) q = *(const uint4*)(src + 4 * lane);
#pragma unroll
      for (int k = 0; k < CW; k += 2) {
        const uint32_t s0 = __builtin_amdgcn_readlane(k % 4 == 0 ? q.x : q.z, k / 4);
        const uint32_t s1 = __builtin_amdgcn_readlane(k % 4 == 0 ? q.y : q.w, k / 4);
        uint32_t d0, d1;
        asm volatile("v_pk_sub_u16 %0, %4, %6 clamp\n\tv_pk_sub_u16 %1, %5, %7 clamp\n\t"
                     "v_pk_min_u16 %0, %0, %8\n\tv_pk_min_u16 %1, %1, %8\n\t"
                     "v_pk_add_u16 %2, %2, %0\n\tv_pk_add_u16 %3, %3, %1"
                     : "=&v"(d0), "=&v"(d1), "+v"(acc0), "+v"(acc1)
                     : "s"(s0), "s"(s1), "v"(mw[k]), "v"(mw[k + 1]), "v"(ones));
      }
    }
    int cnt = (int)(acc0 & 0xFFFF) + (int)(acc0 >> 16) + (int)(acc1 & 0xFFFF) + (int)(acc1 >> 16);
    cnt += __builtin_amdgcn_mov_dpp(cnt, 0xB1, 0xF, 0xF, false);
    cnt += __builtin_amdgcn_mov_dpp(cnt, 0x4E, 0xF, 0xF, false);
    const uint64_t b = __ballot(part == 0 && cnt >= 300);
    const int slot = it & 31;
    if ((tid & 63) == 0) cntw[slot][tid >> 6] = (int)__builtin_popcountll(b);
    __syncthreads();
    int r = 0;
#pragma unroll
    for (int w = 0; w < 16; w += 4) {
      const int4 q = *(const int4*)&cntw[slot][w];
      r += q.x + q.y + q.z + q.w;
    }
    tot += r;
    p = (p * 5 + r + 3) & 63;
  }
  const uint64_t t1 = __builtin_readcyclecounter();
  out[blockIdx.x * BS + tid] = tot;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
double run(int ncu, uint32_t* out, uint64_t* cyc, int iters) {
  for (int r = 0; r < 2; r++) {
    kprobe<MODE><<<ncu, BS>>>(out, cyc, iters);
    hipDeviceSynchronize();
  }
  uint64_t h[1024];
  hipMemcpy(h, cyc, sizeof(uint64_t) * ncu, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < ncu; i++) s += (double)h[i];
  return s / ncu / iters;
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  uint64_t* cyc;
  (void)hipMalloc(&out, sizeof(uint32_t) * ncu * BS);
  (void)hipMalloc(&cyc, sizeof(uint64_t) * ncu);
  const int iters = 2000;
  printf("mode 0 full probe:            %.0f cycles\n", run<0>(ncu, out, cyc, iters));
  printf("mode 1 no LDS slice reads:    %.0f cycles\n", run<1>(ncu, out, cyc, iters));
  printf("mode 2 no packed compares:    %.0f cycles\n", run<2>(ncu, out, cyc, iters));
  printf("mode 3 barrier+exchange only: %.0f cycles\n", run<3>(ncu, out, cyc, iters));
  printf("mode 4 readlane broadcast:    %.0f cycles\n", run<4>(ncu, out, cyc, iters));
  printf("mode 5 4-word blocks, 4 acc:  %.0f cycles\n", run<5>(ncu, out, cyc, iters));
  printf("mode 6 two positions:         %.0f cycles (both)\n", run<6>(ncu, out, cyc, iters));
  printf("mode 7 8-bit SWAR, 16 words:  %.0f cycles\n", run<7>(ncu, out, cyc, iters));
  printf("mode 8 32-bit ops, 32 words:  %.0f cycles\n", run<8>(ncu, out, cyc, iters));
  return 0;
}
