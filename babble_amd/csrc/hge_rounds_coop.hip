// hge_rounds_coop.hip — DivideRounds for wide hashgraphs (N > 32): the
// frontier recurrence evaluated by one co-resident workgroup per chain.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

// ---------------------------------------------------------------------------
// Rounds for wide hashgraphs: the frontier recurrence of DESIGN.md §4.2,
//   C_{r+1}[c] = SM-th smallest over d of fss_c(C_r[d]),
//   fss_c(m)   = SM-th smallest over i of FD[(i, FD[m][i])][c],
// evaluated for the N members of round r only (never for every event).  One
// workgroup per target chain c (cooperative launch, all co-resident); thread
// d computes fss_c(m_d) from N gathers of FDT[c][i][u] (u = FD[m_d][i], the
// member rows staged through LDS 64 columns at a time).  Every gathered value
// is a chain-c position >= C_r[c] (a descendant of a round->=r event has
// round >= r), so both selections are 64-bin histograms relative to C_r[c]
// with an exact bisection fallback past the window.
// ---------------------------------------------------------------------------
// count of the gathered values <= t for thread d (exact; used past the window)
__device__ int fss_count_le(const Tables& t, const int32_t* FDT, int c, int d, int Pd, int t_) {
  const int N = t.N;
  const int32_t* fdm = t.FD + rowoff(t, d, Pd);
  int cnt = 0;
  for (int i = 0; i < N; i++) {
    const int u = fdm[i];
    if (u == INF32) continue;
    const int v = FDT[((size_t)c * N + i) * t.ccap + u];
    cnt += (v <= t_) ? 1 : 0;
  }
  return cnt;
}

// Hand-off between workgroups: only the frontier itself.  Each workgroup
// publishes C_{r+1}[c] as one 8-byte granule {epoch, value} with a relaxed
// agent-scope (write-through, sc1) store, and every workgroup's wave 0 polls
// the N granules of the round with relaxed agent-scope loads until all tags
// match ("the data is the flag": cdna_hip_programming.md Guideline 16, R2).
// No grid barrier, no release/acquire fence: every other load of the kernel
// reads tables written by earlier kernels (FD, FDT), so the L2-resident rows
// stay cached across rounds.  Granules are double-buffered by round parity:
// a workgroup can only publish round r+2 after every workgroup published
// r+1, which each does after it finished reading round r.
// Member rows FD[(d, C_r[d])] are staged through LDS as uint16 (chain
// positions < 65535, checked by the host), CW columns at a time.
// The kernel also emits the strongly-see bits of the next round's frontier
// event of chain c against this round's members (ssc), which k_witness_bits
// turns into the vote adjacency without an N-wide compare per pair:
// y = C_{r+1}[c] strongly sees m_d  <=>  pos(y) >= fss_c(m_d).
typedef __attribute__((address_space(1))) unsigned long long gu64_t;

__global__ void __launch_bounds__(256) k_rounds_coop(Tables t, const int32_t* FDT, const int32_t* olen,
                                                     const int32_t* len, int32_t* rstate, int rlo,
                                                     int Rprev, uint64_t* gran, int32_t* err,
                                                     uint64_t* ssc, uint64_t* dbg) {
  // HGE_STAMPS diagnostics (workgroup 0, thread 0): cycles per section
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_t = 0, st_u = 0;
#define CSUB(k)                                                \
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0) {            \
    const uint64_t now_ = stamp();        \
    if ((k) > 4) st_acc[(k)] += now_ - st_u;                   \
    st_u = now_;                                               \
  }
#define CSTAMP(k)                                              \
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0) {            \
    const uint64_t now_ = stamp();        \
    if ((k) > 0) st_acc[(k) - 1] += now_ - st_t;               \
    st_t = now_;                                               \
  }
  constexpr int NB = 64;  // histogram bins (window above C_r[c])
  constexpr int CW = 64;  // member-row columns staged per chunk
  constexpr int RS = 33;  // LDS row stride in words (odd: conflict-free per-thread rows)
  __shared__ int sP[256];
  __shared__ uint32_t sU[256 * RS];  // sU[d][ii] as uint16 pairs: member rows, CW columns
  __shared__ uint32_t sH[256 * RS];  // sH[d][b/2]: per-thread histograms, two 16-bit bins per word
  __shared__ uint32_t sH2[NB];
  constexpr int WIN = 64;            // FDT window per column i: positions [wb_i, wb_i + WIN)
  __shared__ uint16_t sW[CW][WIN];
  __shared__ int sWb[CW];
  __shared__ int s_sel, s_exact, s_cnt, s_nxt, s_stop;
  const int N = t.N, SM = t.SM, NW = t.NW;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int lenc = len[c];
  gu64_t* gr[2] = {(gu64_t*)gran, (gu64_t*)(gran + N)};
  if (tid < N) {
    int P = t.C[(size_t)rlo * N + tid];
    if (rlo == 0 && olen[tid] == 0 && len[tid] > 0) P = 0;
    sP[tid] = P;
    if (c == 0 && rlo == 0 && olen[tid] == 0 && len[tid] > 0) t.C[tid] = 0;
  }
  __syncthreads();
  for (int r = rlo;; r++) {
    if (r + 1 >= t.Rcap) {
      if (c == 0 && tid == 0) rstate[1] = 1;
      break;
    }
    CSTAMP(0);
    const int Pc = sP[c];
    // thread = (member d, part): TPM = 256 / NPOW threads share member d's columns
    const int NPOW = N <= 64 ? 64 : N <= 128 ? 128 : 256;
    const int TPM = 256 / NPOW;
    const int d = tid & (NPOW - 1), part = tid / NPOW;
    const bool lead = part == 0;
    const int Pd = (d < N) ? sP[d] : INF32;
    const bool dact = d < N && Pd != INF32 && Pc != INF32;
    if (lead)
      for (int w = 0; w < NB / 2; w++) sH[d * RS + w] = 0;
    if (tid < NB) sH2[tid] = 0;
    for (int i0 = 0; i0 < N; i0 += CW) {
      const int ni = min(CW, N - i0);
      __syncthreads();
      CSUB(4);
      // member rows FD[(dd, C_r[dd])][i0, i0 + CW): 4 ints per load, coalesced
      constexpr int Q = CW / 4;
      constexpr int PER = 256 * Q / 256;  // N <= 256 rows
      int4 vv[PER];
#pragma unroll
      for (int m = 0; m < PER; m++) {
        const int item = tid + m * 256;
        const int dd = item / Q, q = item - (item / Q) * Q;
        vv[m] = make_int4(INF32, INF32, INF32, INF32);
        if (dd < N && sP[dd] != INF32 && 4 * q < ni) {
          const int32_t* row = t.FD + rowoff(t, dd, sP[dd]) + i0 + 4 * q;
          if ((N & 3) == 0) {
            vv[m] = *(const int4*)row;
          } else {
            vv[m].x = row[0];
            if (4 * q + 1 < ni) vv[m].y = row[1];
            if (4 * q + 2 < ni) vv[m].z = row[2];
            if (4 * q + 3 < ni) vv[m].w = row[3];
          }
        }
      }
      if (tid < CW) sWb[tid] = INF32;
      __syncthreads();
      CSUB(5);
      // pack to uint16 and take the per-column minimum (window base): lanes
      // l, l+16, l+32, l+48 of a wave hold the same 4 columns
      int4 mn = make_int4(INF32, INF32, INF32, INF32);
#pragma unroll
      for (int m = 0; m < PER; m++) {
        const int item = tid + m * 256;
        const int dd = item / Q, q = item - (item / Q) * Q;
        if (dd < N) {
          const int4 w = vv[m];
          mn.x = min(mn.x, w.x);
          mn.y = min(mn.y, w.y);
          mn.z = min(mn.z, w.z);
          mn.w = min(mn.w, w.w);
          const uint32_t a = (uint32_t)(w.x == INF32 ? 0xFFFF : w.x) |
                             ((uint32_t)(w.y == INF32 ? 0xFFFF : w.y) << 16);
          const uint32_t b = (uint32_t)(w.z == INF32 ? 0xFFFF : w.z) |
                             ((uint32_t)(w.w == INF32 ? 0xFFFF : w.w) << 16);
          sU[dd * RS + 2 * q] = a;
          sU[dd * RS + 2 * q + 1] = b;
        }
      }
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        mn.x = min(mn.x, __shfl_xor(mn.x, o));
        mn.y = min(mn.y, __shfl_xor(mn.y, o));
        mn.z = min(mn.z, __shfl_xor(mn.z, o));
        mn.w = min(mn.w, __shfl_xor(mn.w, o));
      }
      if ((tid & 63) < Q) {
        const int q = tid & 63;
        if (mn.x != INF32) atomicMin(&sWb[4 * q], mn.x);
        if (mn.y != INF32) atomicMin(&sWb[4 * q + 1], mn.y);
        if (mn.z != INF32) atomicMin(&sWb[4 * q + 2], mn.z);
        if (mn.w != INF32) atomicMin(&sWb[4 * q + 3], mn.w);
      }
      __syncthreads();
      CSUB(6);
      // FDT windows: column i's member values sit just above their minimum
      const int32_t* fdt = FDT + ((size_t)c * N + i0) * t.ccap;
      {
        constexpr int WPER = CW * WIN / 256;
        int wv[WPER];
#pragma unroll
        for (int m = 0; m < WPER; m++) {
          const int item = tid + m * 256;
          const int ii = item / WIN, k = item - (item / WIN) * WIN;
          const int wb = min(sWb[ii], t.ccap - WIN);
          wv[m] = (ii < ni && sWb[ii] != INF32) ? fdt[(size_t)ii * t.ccap + wb + k] : INF32;
        }
#pragma unroll
        for (int m = 0; m < WPER; m++) {
          const int item = tid + m * 256;
          const int ii = item / WIN, k = item - (item / WIN) * WIN;
          sW[ii][k] = (wv[m] == INF32) ? 0xFFFF : (uint16_t)wv[m];
        }
      }
      __syncthreads();
      // effective window base (clamped inside the table; INF32 = no window)
      if (tid < CW && sWb[tid] != INF32) sWb[tid] = min(sWb[tid], t.ccap - WIN);
      __syncthreads();
      CSUB(7);
      if (dact) {
        // branch-free: all LDS reads of a batch issue back to back, window
        // misses become predicated global loads, empty values add 0.  Part p
        // of member d takes columns ii = p + TPM * k.
        const uint16_t* myu = (const uint16_t*)(sU + d * RS);
        constexpr int KB = 16;
        for (int ib = part; ib < ni; ib += KB * TPM) {
          int uu[KB], wv[KB], gv[KB];
#pragma unroll
          for (int k = 0; k < KB; k++) {
            const int ii = ib + k * TPM;
            uu[k] = (ii < ni) ? (int)myu[ii] : 0xFFFF;
          }
#pragma unroll
          for (int k = 0; k < KB; k++) {
            const int ii = min(ib + k * TPM, CW - 1);
            const int off = uu[k] - sWb[ii];
            const bool inw = uu[k] != 0xFFFF && (unsigned)off < (unsigned)WIN;
            wv[k] = sW[ii][inw ? off : 0];
            if (!inw) wv[k] = -1;
          }
#pragma unroll
          for (int k = 0; k < KB; k++) {
            const bool need = uu[k] != 0xFFFF && wv[k] < 0;
            gv[k] = need ? fdt[(size_t)(ib + k * TPM) * t.ccap + uu[k]] : INF32;
          }
#pragma unroll
          for (int k = 0; k < KB; k++) {
            int v = (wv[k] >= 0) ? (wv[k] == 0xFFFF ? INF32 : wv[k]) : gv[k];
            if (uu[k] == 0xFFFF) v = INF32;
            const bool fin = v != INF32;
            const int b = fin ? min(max(v - Pc, 0), NB - 1) : 0;
            atomicAdd(&sH[d * RS + (b >> 1)], fin ? (1u << ((b & 1) * 16)) : 0u);
          }
        }
      }
    }
    __syncthreads();
    CSTAMP(1);
    // first level: fss_c(m_d) = SM-th smallest gathered value (branch-free bin scan)
    int fss = INF32;
    if (dact && lead) {
      uint32_t hw[NB / 2];
#pragma unroll
      for (int w = 0; w < NB / 2; w++) hw[w] = sH[d * RS + w];
      int cum = 0, b = NB;
#pragma unroll
      for (int w = 0; w < NB / 2; w++) {
        const int lo = hw[w] & 0xFFFF, hi = hw[w] >> 16;
        if (b == NB && cum + lo >= SM) b = 2 * w;
        cum += lo;
        if (b == NB && cum + hi >= SM) b = 2 * w + 1;
        cum += hi;
      }
      if (b == NB) {
        fss = INF32;  // fewer than SM finite values
      } else if (b < NB - 1) {
        fss = Pc + b;
      } else {
        // past the window: bisection on the exact count
        int lo = Pc + NB - 1, hi = lenc;
        if (hi <= lo || fss_count_le(t, FDT, c, d, Pd, hi - 1) < SM) {
          fss = INF32;
        } else {
          while (lo < hi - 1) {
            const int mid = lo + (hi - 1 - lo) / 2;
            if (fss_count_le(t, FDT, c, d, Pd, mid) >= SM) hi = mid + 1;
            else lo = mid + 1;
          }
          fss = lo;
        }
      }
      if (fss >= lenc) fss = INF32;
    }
    const int fss_raw = fss;  // strongly seen by every position >= fss_raw
    if (fss != INF32 && d == c) fss = max(fss, Pc + 1);  // x never strongly sees itself
    // second level: SM-th smallest over the members (wave-0 prefix scan of 64 bins)
    if (fss != INF32) atomicAdd(&sH2[min(max(fss - Pc, 0), NB - 1)], 1u);
    __syncthreads();
    CSTAMP(2);
    if (tid < 64) {
      int v = (int)sH2[tid];
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o);
        if (tid >= o) v += y;
      }
      const uint64_t m = __ballot(v >= SM);
      if (tid == 0) {
        const int b = m ? __builtin_ctzll(m) : NB;
        s_sel = (b < NB - 1) ? Pc + b : INF32;
        s_exact = (b == NB - 1) ? 1 : 0;
      }
    }
    __syncthreads();
    if (s_exact) {
      int lo = Pc + NB - 1, hi = lenc;
      while (lo < hi) {
        const int mid = lo + (hi - lo) / 2;
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        if (fss != INF32 && fss <= mid) atomicAdd(&s_cnt, 1);
        __syncthreads();
        const int cnt = s_cnt;
        __syncthreads();
        if (cnt >= SM) hi = mid;
        else lo = mid + 1;
      }
      if (tid == 0) s_sel = lo < lenc ? lo : INF32;
      __syncthreads();
    }
    if (tid == 0) {
      const int cur = (r + 1 < Rprev) ? t.C[(size_t)(r + 1) * N + c] : INF32;
      int nxt = INF32;
      if (Pc != INF32) nxt = (cur != INF32) ? cur : (s_sel < lenc ? s_sel : INF32);
      if (nxt != INF32 && cur == INF32) t.C[(size_t)(r + 1) * N + c] = nxt;
      s_nxt = nxt;
      // publish: epoch = r - rlo + 1 (never 0: the buffer is zeroed before launch)
      const uint64_t g = ((uint64_t)(uint32_t)(r - rlo + 1) << 32) | (uint32_t)nxt;
      __hip_atomic_store(gr[(r + 1) & 1] + c, (unsigned long long)g, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int nxt = s_nxt;
    // strongly-see bits of C_{r+1}[c] against the members of round r
    if (nxt != INF32) {
      const uint64_t bits = __ballot(lead && d < N && fss_raw != INF32 && fss_raw <= nxt);
      if ((tid & 63) == 0 && (tid >> 6) < NW)
        ssc[((size_t)(r + 1) * N + c) * NW + (tid >> 6)] = bits;
    }
    CSTAMP(3);
    // collect C_{r+1}: wave 0 polls the N granules of epoch r - rlo + 1
    if (tid < 64) {
      const unsigned ep = (unsigned)(r - rlo + 1);
      gu64_t* g = gr[(r + 1) & 1];
      unsigned spins = 0;
      bool any = false, fail = false;
      for (;;) {
        bool ok = true;
        any = false;
        for (int dd = tid; dd < N; dd += 64) {
          const unsigned long long x =
              __hip_atomic_load(g + dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (unsigned)(x >> 32) == ep;
          const int P = (int)(uint32_t)x;
          sP[dd] = P;
          any |= (P != INF32);
        }
        if (__all(ok)) break;
        if (++spins > (1u << 24)) {  // never a normal wait: co-residency failure
          fail = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      any = __ballot(any) != 0;
      if (tid == 0) {
        s_stop = fail ? 2 : (any ? 0 : 1);
        if (fail) atomicOr(err, 1);
      }
    }
    __syncthreads();
    CSTAMP(4);
    if (s_stop) {
      if (s_stop == 1 && c == 0 && tid == 0) rstate[0] = max(rstate[0], r + 1);
      break;
    }
  }
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0)
    for (int q = 0; q < 8; q++) dbg[q] += st_acc[q];
#undef CSTAMP
}

}  // namespace hge
