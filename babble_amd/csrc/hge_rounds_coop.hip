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

// LDS of one workgroup of the frontier recurrence
struct CoopLDS {
  int sP[256];                 // the frontier C_r (one position per chain)
  uint32_t sU[256 * 33];       // sU[d][ii] as uint16 pairs: member rows, CW columns
  uint32_t sH[32 * 256];       // sH[b/2][d]: per-member histograms, two 16-bit bins per word
                               // (bin-major: a half-wave of members never shares a bank)
  uint32_t sH2[64];
  uint16_t sW[64][64];         // FDT window per column i: positions [wb_i, wb_i + WIN)
  int sWb[64];
  int s_sel, s_exact, s_cnt, s_nxt, s_stop, s_hit;
  uint64_t s_hash;
};

// One step of the recurrence for target chain c = the workgroup's chain, from
// the frontier in L.sP: returns C_{r+1}[c] before the end-of-chain clamp
// (valid in thread 0) and, per thread, fss_c(m_d) before the own-chain clamp
// (INF32 for threads that hold no member).  The result is a function of
// L.sP alone, which is what lets speculative walkers merge (below).
template <int BS, int KB>
__device__ __forceinline__ int coop_select(const Tables& t, const int32_t* FDT, int c, int lenc,
                                           CoopLDS& L, int& fss_out, uint64_t* sacc = nullptr) {
  // HGE_STAMPS: cycles per section into sacc[4..7] (loads, pack, windows, gathers), sacc[8] (select)
  uint64_t su = sacc ? stamp() : 0;
#define SSUB(k)                          \
  if (sacc) {                            \
    const uint64_t now_ = stamp();       \
    sacc[(k)] += now_ - su;              \
    su = now_;                           \
  }
  constexpr int NB = 64;  // histogram bins (window above C_r[c])
  constexpr int CW = 64;  // member-row columns staged per chunk
  constexpr int RS = 33;  // LDS row stride in words (odd: conflict-free per-thread rows)
  constexpr int WIN = 64;
  const int N = t.N, SM = t.SM;
  const int tid = threadIdx.x;
  const int Pc = L.sP[c];
  // thread = (member d, part): TPM = BS / NPOW threads share member d's columns
  const int NPOW = N <= 64 ? 64 : N <= 128 ? 128 : 256;
  const int TPM = BS / NPOW;
  const int d = tid & (NPOW - 1), part = tid / NPOW;
  const bool lead = part == 0;
  const int Pd = (d < N) ? L.sP[d] : INF32;
  const bool dact = d < N && Pd != INF32 && Pc != INF32;
  if (lead)
    for (int w = 0; w < NB / 2; w++) L.sH[w * 256 + d] = 0;
  if (tid < NB) L.sH2[tid] = 0;
  for (int i0 = 0; i0 < N; i0 += CW) {
    const int ni = min(CW, N - i0);
    __syncthreads();
    SSUB(8);
    // member rows FD[(dd, C_r[dd])][i0, i0 + CW): 4 ints per load, coalesced
    constexpr int Q = CW / 4;
    constexpr int PER = 256 * Q / BS;  // N <= 256 rows
    int4 vv[PER];
#pragma unroll
    for (int m = 0; m < PER; m++) {
      const int item = tid + m * BS;
      const int dd = item / Q, q = item - (item / Q) * Q;
      vv[m] = make_int4(INF32, INF32, INF32, INF32);
      if (dd < N && L.sP[dd] != INF32 && 4 * q < ni) {
        const int32_t* row = t.FD + rowoff(t, dd, L.sP[dd]) + i0 + 4 * q;
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
    if (tid < CW) L.sWb[tid] = INF32;
    __syncthreads();
    SSUB(4);
    // pack to uint16 and take the per-column minimum (window base): lanes
    // l, l+16, l+32, l+48 of a wave hold the same 4 columns
    int4 mn = make_int4(INF32, INF32, INF32, INF32);
#pragma unroll
    for (int m = 0; m < PER; m++) {
      const int item = tid + m * BS;
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
        L.sU[dd * RS + 2 * q] = a;
        L.sU[dd * RS + 2 * q + 1] = b;
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
      if (mn.x != INF32) atomicMin(&L.sWb[4 * q], mn.x);
      if (mn.y != INF32) atomicMin(&L.sWb[4 * q + 1], mn.y);
      if (mn.z != INF32) atomicMin(&L.sWb[4 * q + 2], mn.z);
      if (mn.w != INF32) atomicMin(&L.sWb[4 * q + 3], mn.w);
    }
    __syncthreads();
    SSUB(5);
    // FDT windows: column i's member values sit just above their minimum
    const int32_t* fdt = FDT + ((size_t)c * N + i0) * t.ccap;
    {
      constexpr int WPER = CW * WIN / BS;
      int wv[WPER];
#pragma unroll
      for (int m = 0; m < WPER; m++) {
        const int item = tid + m * BS;
        const int ii = item / WIN, k = item - (item / WIN) * WIN;
        const int wb = min(L.sWb[ii], t.ccap - WIN);
        wv[m] = (ii < ni && L.sWb[ii] != INF32) ? fdt[(size_t)ii * t.ccap + wb + k] : INF32;
      }
#pragma unroll
      for (int m = 0; m < WPER; m++) {
        const int item = tid + m * BS;
        const int ii = item / WIN, k = item - (item / WIN) * WIN;
        L.sW[ii][k] = (wv[m] == INF32) ? 0xFFFF : (uint16_t)wv[m];
      }
    }
    __syncthreads();
    // effective window base (clamped inside the table; INF32 = no window)
    if (tid < CW && L.sWb[tid] != INF32) L.sWb[tid] = min(L.sWb[tid], t.ccap - WIN);
    __syncthreads();
    SSUB(6);
    if (dact) {
      // branch-free: all LDS reads of a batch issue back to back, window
      // misses become predicated global loads, empty values add 0.  Part p
      // of member d takes columns ii = p + TPM * k.
      const uint16_t* myu = (const uint16_t*)(L.sU + d * RS);
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
          const int off = uu[k] - L.sWb[ii];
          const bool inw = uu[k] != 0xFFFF && (unsigned)off < (unsigned)WIN;
          wv[k] = L.sW[ii][inw ? off : 0];
          if (!inw) wv[k] = -1;
        }
        if (sacc) {  // HGE_STAMPS: batches of wave 0, and those with a window miss
          bool miss = false;
#pragma unroll
          for (int k = 0; k < KB; k++) miss |= uu[k] != 0xFFFF && wv[k] < 0;
          sacc[10] += 1;
          sacc[9] += __ballot(miss) ? 1 : 0;
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
          atomicAdd(&L.sH[(b >> 1) * 256 + d], fin ? (1u << ((b & 1) * 16)) : 0u);
        }
      }
    }
  }
  __syncthreads();
  SSUB(7);
  // first level: fss_c(m_d) = SM-th smallest gathered value (branch-free bin scan)
  int fss = INF32;
  if (dact && lead) {
    uint32_t hw[NB / 2];
#pragma unroll
    for (int w = 0; w < NB / 2; w++) hw[w] = L.sH[w * 256 + d];
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
  if (fss != INF32) atomicAdd(&L.sH2[min(max(fss - Pc, 0), NB - 1)], 1u);
  __syncthreads();
  if (tid < 64) {
    int v = (int)L.sH2[tid];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o);
      if (tid >= o) v += y;
    }
    const uint64_t m = __ballot(v >= SM);
    if (tid == 0) {
      const int b = m ? __builtin_ctzll(m) : NB;
      L.s_sel = (b < NB - 1) ? Pc + b : INF32;
      L.s_exact = (b == NB - 1) ? 1 : 0;
    }
  }
  __syncthreads();
  if (L.s_exact) {
    int lo = Pc + NB - 1, hi = lenc;
    while (lo < hi) {
      const int mid = lo + (hi - lo) / 2;
      if (tid == 0) L.s_cnt = 0;
      __syncthreads();
      if (fss != INF32 && fss <= mid) atomicAdd(&L.s_cnt, 1);
      __syncthreads();
      const int cnt = L.s_cnt;
      __syncthreads();
      if (cnt >= SM) hi = mid;
      else lo = mid + 1;
    }
    if (tid == 0) L.s_sel = lo < lenc ? lo : INF32;
    __syncthreads();
  }
  SSUB(8);
#undef SSUB
  fss_out = fss_raw;
  return L.s_sel;
}


// 1024 threads: four waves per SIMD (the gather loop is issue/latency-bound at
// one); gather batches of 8 columns keep it within 128 VGPRs
constexpr int COOP_BS = 1024;
constexpr int COOP_SPEC_BS = 512;  // walkers: 512 threads, 2 per CU
__global__ void __launch_bounds__(COOP_BS) k_rounds_coop(Tables t, const int32_t* FDT, const int32_t* olen,
                                                     const int32_t* len, int32_t* rstate, int rlo,
                                                     const int32_t* rlo_dev, int Rprev, uint64_t* gran,
                                                     int32_t* err, uint64_t* ssc, uint64_t* dbg) {
  // rlo_dev: the first round to recompute, read here (INF32: nothing to do)
  if (rlo_dev) {
    rlo = *rlo_dev;
    if (rlo == INF32) return;
  }
  // HGE_STAMPS diagnostics (workgroup 0, thread 0): cycles per section
  __shared__ uint64_t st_acc[11];  // thread 0 only: kept out of every lane's registers
  uint64_t st_t = 0;
  if (threadIdx.x < 11) st_acc[threadIdx.x] = 0;
#define CSTAMP(k)                                              \
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0) {            \
    const uint64_t now_ = stamp();        \
    if ((k) > 0) st_acc[(k) - 1] += now_ - st_t;               \
    st_t = now_;                                               \
  }
  __shared__ CoopLDS L;
  const int N = t.N, NW = t.NW;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int lenc = len[c];
  gu64_t* gr[2] = {(gu64_t*)gran, (gu64_t*)(gran + N)};
  if (tid < N) {
    int P = t.C[(size_t)rlo * N + tid];
    if (rlo == 0 && olen[tid] == 0 && len[tid] > 0) P = 0;
    L.sP[tid] = P;
    if (c == 0 && rlo == 0 && olen[tid] == 0 && len[tid] > 0) t.C[tid] = 0;
  }
  __syncthreads();
  for (int r = rlo;; r++) {
    if (r + 1 >= t.Rcap) {
      if (c == 0 && tid == 0) rstate[1] = 1;
      break;
    }
    CSTAMP(0);
    int fss_raw;
    coop_select<COOP_BS, 8>(t, FDT, c, lenc, L, fss_raw, (dbg && blockIdx.x == 0 && tid == 0) ? st_acc : nullptr);
    CSTAMP(2);
    if (tid == 0) {
      const int Pc = L.sP[c];
      const int cur = (r + 1 < Rprev) ? t.C[(size_t)(r + 1) * N + c] : INF32;
      int nxt = INF32;
      if (Pc != INF32) nxt = (cur != INF32) ? cur : (L.s_sel < lenc ? L.s_sel : INF32);
      if (nxt != INF32 && cur == INF32) t.C[(size_t)(r + 1) * N + c] = nxt;
      L.s_nxt = nxt;
      // publish: epoch = r - rlo + 1 (never 0: the buffer is zeroed before launch)
      const uint64_t g = ((uint64_t)(uint32_t)(r - rlo + 1) << 32) | (uint32_t)nxt;
      __hip_atomic_store(gr[(r + 1) & 1] + c, (unsigned long long)g, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int nxt = L.s_nxt;
    // strongly-see bits of C_{r+1}[c] against the members of round r
    if (nxt != INF32) {
      const uint64_t bits = __ballot(fss_raw != INF32 && fss_raw <= nxt);
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
          L.sP[dd] = P;
          any |= (P != INF32);
        }
        if (__all(ok)) break;
        if (++spins > (1u << 21)) {  // never a normal wait (~2 s): co-residency failure
          fail = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      any = __ballot(any) != 0;
      if (tid == 0) {
        L.s_stop = fail ? 2 : (any ? 0 : 1);
        if (fail) {  // the host falls back to k_round_step32
          atomicOr(err, 1);
          atomicOr(rstate + 1, 4);  // the downstream kernels stand down, as on overflow
        }
      }
    }
    __syncthreads();
    CSTAMP(4);
    if (L.s_stop) {
      if (L.s_stop == 1 && c == 0 && tid == 0) rstate[0] = max(rstate[0], r + 1);
      break;
    }
  }
  if (dbg && blockIdx.x == 0 && threadIdx.x == 0)
    for (int q = 0; q < 11; q++) dbg[q] += st_acc[q];
#undef CSTAMP
}

// ---------------------------------------------------------------------------
// Speculative walkers for wide hashgraphs (fresh state).  The recurrence
// C_{r+1} = F(C_r) is evaluated by coop_select as a function of the frontier
// row alone, so two walks that ever hold the same row coincide from then on
// (the N <= 32 form is hge_walk_spec.hip).  Walker w (N workgroups, all
// walkers co-resident in one cooperative grid) starts at the true C_0 for
// w = 0 and at floor(len_c * w / nw) on every chain otherwise.  Its rows are
// the hand-off itself: H[w][j][c] = (tag << 32) | C_j[c], written once per
// launch with relaxed agent-scope stores (tag = launch epoch, bit 31 = "this
// workgroup saw a merge"), polled by every workgroup of the walker.
// Merge test: walker w-1 looks its newest row up in walker w's hash table
// (workgroup 0 of walker w inserts each completed row) and verifies the whole
// row word by word.  A hit sets the flag bit on the next row, so every
// workgroup of the walker stops after the same row.  Stale or not-yet-visible
// words never carry the current tag: a race can only delay a merge.
// ---------------------------------------------------------------------------
struct CoopSpec {
  uint64_t* H;          // [nw][Hcap][N] tagged rows
  uint64_t* SSCH;       // [nw][Hcap][N][NW] strongly-see bits of row j vs row j-1
  uint64_t* TT;         // [nw][TS] hash -> row: (tag << 32) | (hash16 << 16) | row
  unsigned long long* mrg;  // [nw] min over hits of (row << 32) | (walker offset << 16) | row there
  int32_t* hn;          // [2 nw]: rows written (incl. the terminal row), natural end flag
  int nw, Hcap, TS;
  uint32_t epoch;       // 1 .. 2^31-1, new per launch
  int64_t events;       // events inserted (time-cut guesses)
  int guess;            // walker w >= 1 starts at: 0 = len_c * w / nw on every chain,
                        // 1 = the time cut events * w / nw, 2 = 0 for odd w, 1 for even w
};

__device__ __forceinline__ uint64_t coop_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int BS>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4, 4))) k_rounds_coop_spec(Tables t, const int32_t* FDT,
                                                          const int32_t* olen, const int32_t* len,
                                                          CoopSpec sp, int32_t* err) {
  __shared__ CoopLDS L;
  const int N = t.N, NW = t.NW;
  const int w = blockIdx.x / N, c = blockIdx.x - w * N, tid = threadIdx.x;
  const int lenc = len[c];
  const uint32_t ep = sp.epoch;
  gu64_t* Hw = (gu64_t*)(sp.H + (size_t)w * sp.Hcap * N);
  gu64_t* Tw = (gu64_t*)(sp.TT + (size_t)w * sp.TS);
  if (tid < N) {
    const int ld = len[tid];
    int P;
    if (w == 0) {
      P = t.C[tid];
      if (olen[tid] == 0 && ld > 0) P = 0;
    } else if (sp.guess == 0 || (sp.guess == 2 && (w & 1))) {
      P = ld > 0 ? (int)((int64_t)ld * w / sp.nw) : INF32;
    } else {
      // time cut: the first event of chain tid inserted at or after T (ids are
      // insertion order, increasing along a chain); none = an ended chain
      const int64_t T = sp.events * w / sp.nw;
      const int32_t* ch = t.chain + (size_t)tid * t.ccap;
      int lo = 0, hi = ld;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)ch[mid] < T) lo = mid + 1;
        else hi = mid;
      }
      P = lo < ld ? lo : INF32;
    }
    L.sP[tid] = P;
    if (tid == c)
      __hip_atomic_store(Hw + c, ((unsigned long long)ep << 32) | (uint32_t)P, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) L.s_hit = 0;
  __syncthreads();
  for (int j = 0;; j++) {
    if (j + 1 >= sp.Hcap) {  // history full: rows 0..j
      if (c == 0 && tid == 0) {
        sp.hn[w] = j + 1;
        sp.hn[sp.nw + w] = 0;
      }
      break;
    }
    int fss_raw;
    coop_select<BS, 8>(t, FDT, c, lenc, L, fss_raw);
    if (tid == 0) {
      const int Pc = L.sP[c];
      const int nxt = (Pc != INF32 && L.s_sel < lenc) ? L.s_sel : INF32;
      L.s_nxt = nxt;
      const uint32_t tag = ep | (L.s_hit ? 0x80000000u : 0u);
      __hip_atomic_store(Hw + (size_t)(j + 1) * N + c, ((unsigned long long)tag << 32) | (uint32_t)nxt,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    {
      const int nxt = L.s_nxt;
      const uint64_t bits = __ballot(nxt != INF32 && fss_raw != INF32 && fss_raw <= nxt);
      if ((tid & 63) == 0 && (tid >> 6) < NW)
        sp.SSCH[(((size_t)w * sp.Hcap + j + 1) * N + c) * NW + (tid >> 6)] = bits;
    }
    // collect row j+1, its hash, and the merge flags
    if (tid < 64) {
      gu64_t* g = Hw + (size_t)(j + 1) * N;
      unsigned spins = 0;
      bool any = false, fail = false, flag = false;
      uint64_t h = 0;
      for (;;) {
        bool ok = true;
        any = false;
        flag = false;
        h = 0;
        for (int dd = tid; dd < N; dd += 64) {
          const unsigned long long x =
              __hip_atomic_load(g + dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t tg = (uint32_t)(x >> 32);
          ok &= (tg & 0x7FFFFFFFu) == ep;
          flag |= (tg >> 31) != 0;
          const int P = (int)(uint32_t)x;
          L.sP[dd] = P;
          any |= (P != INF32);
          h += coop_mix(((uint64_t)dd << 32) | (uint32_t)P);
        }
        if (__all(ok)) break;
        if (++spins > (1u << 21)) {  // never a normal wait (~2 s): co-residency failure
          fail = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      any = __ballot(any) != 0;
      flag = __ballot(flag) != 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) h += __shfl_xor(h, o);
      if (tid == 0) {
        L.s_stop = fail ? 2 : (!any ? 1 : (flag ? 3 : 0));
        L.s_hash = h;
        if (fail) atomicOr(err, 1);
      }
    }
    __syncthreads();
    const int stop = L.s_stop;
    if (stop) {
      if (c == 0 && tid == 0) {
        sp.hn[w] = j + 2;
        sp.hn[sp.nw + w] = stop == 1 ? 1 : 0;
      }
      break;
    }
    const uint64_t h = L.s_hash;
    const uint32_t h16 = (uint32_t)(h >> 48);
    // workgroup 0 files row j+1 in this walker's table (single writer)
    if (c == 0 && tid == 0 && j + 1 <= 0xFFFF) {
      const uint32_t mask = (uint32_t)sp.TS - 1;
      for (uint32_t k = 0, s = (uint32_t)h & mask; k < (uint32_t)sp.TS; k++, s = (s + 1) & mask) {
        const unsigned long long x = __hip_atomic_load(Tw + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(x >> 32) == ep) continue;
        __hip_atomic_store(Tw + s, ((unsigned long long)ep << 32) | ((unsigned long long)h16 << 16) | (uint32_t)(j + 1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    // merge test: against walker w+1 every step, w+2 and w+3 on alternate
    // steps (a guessed walker can follow a trajectory that never meets the
    // true one); one probe window of 64 slots
    const int toff = (j & 1) ? 1 : ((j & 2) ? 2 : 3);
    if (tid < 64 && w + toff < sp.nw) {
      gu64_t* Tn = (gu64_t*)(sp.TT + (size_t)(w + toff) * sp.TS);
      gu64_t* Hn = (gu64_t*)(sp.H + (size_t)(w + toff) * sp.Hcap * N);
      const uint32_t mask = (uint32_t)sp.TS - 1;
      const unsigned long long x =
          __hip_atomic_load(Tn + (((uint32_t)h + tid) & mask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool occ = (uint32_t)(x >> 32) == ep;
      const uint64_t emp = __ballot(!occ);
      const int run = emp ? __builtin_ctzll(emp) : 64;  // slots before the first empty one
      uint64_t cand = __ballot(occ && tid < run && ((uint32_t)(x >> 16) & 0xFFFF) == h16);
      int hit = -1;
      while (cand && hit < 0) {
        const int l = __builtin_ctzll(cand);
        cand &= cand - 1;
        const int k = __shfl((int)(x & 0xFFFF), l);
        bool ok = true;
        for (int dd = tid; dd < N; dd += 64) {
          const unsigned long long y =
              __hip_atomic_load(Hn + (size_t)k * N + dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok &= (((uint32_t)(y >> 32)) & 0x7FFFFFFFu) == ep && (int)(uint32_t)y == L.sP[dd];
        }
        if (__all(ok)) hit = k;
      }
      if (tid == 0 && hit >= 0) {
        L.s_hit = 1;
        atomicMin(sp.mrg + w, ((unsigned long long)(j + 1) << 32) | ((uint32_t)toff << 16) | (uint32_t)hit);
      }
    }
    __syncthreads();
  }
}

// Join: follow the merges from walker 0 (true by construction) and copy the
// true rows into C and ssc with global round numbers.  Sets rstate[0] (round
// count) on a natural end, rstate[1] on rounds-table overflow, and *resume to
// the round the sequential kernel must continue from (-1 = none).
__global__ void __launch_bounds__(256) k_coop_join(Tables t, CoopSpec sp, uint64_t* ssc,
                                                   int32_t* rstate, int32_t* resume) {
  constexpr int MS = 64;
  __shared__ int sv[MS], ss[MS], se[MS], sG[MS], sE2[MS];
  __shared__ int s_n;
  const int N = t.N, NW = t.NW;
  if (threadIdx.x == 0) {
    int n = 0, v = 0, s = 0, G = 0, res = -1, R = -1;
    for (int it = 0; it < 4 * sp.nw + 4 && n < MS; it++) {
      const unsigned long long m = sp.mrg[v];
      const int hn = sp.hn[v];
      if (m != ~0ull) {
        const int r = (int)(m >> 32), b = (int)(m & 0xFFFF), v2 = v + (int)((m >> 16) & 0xFFFF);
        if (s >= r) {  // row s of v is row b + s - r of v2
          const int s2 = b + (s - r);
          if (s2 < sp.hn[v2] - (sp.hn[sp.nw + v2] ? 1 : 0)) {
            v = v2;
            s = s2;
            continue;
          }
          sv[n] = v; ss[n] = s; se[n] = s + 1; sG[n] = G; sE2[n] = s; n++;
          res = G;
          break;
        }
        sv[n] = v; ss[n] = s; se[n] = r; sG[n] = G; sE2[n] = r; n++;
        G += r - s;
        v = v2;
        s = b;
        continue;
      }
      if (sp.hn[sp.nw + v]) {  // natural end: row hn-1 is the empty frontier
        sv[n] = v; ss[n] = s; se[n] = hn - 1; sG[n] = G; sE2[n] = hn - 2; n++;
        R = G + (hn - 1 - s);
      } else {  // capacity: the sequential walk resumes from the last row
        sv[n] = v; ss[n] = s; se[n] = hn; sG[n] = G; sE2[n] = hn - 1; n++;
        res = G + (hn - 1 - s);
      }
      break;
    }
    if (R < 0 && res < 0) {  // unreachable (each step advances v): resume from the last true row
      res = G;
      if (n < MS) { sv[n] = v; ss[n] = s; se[n] = s + 1; sG[n] = G; sE2[n] = s; n++; }
    }
    // rows the rounds table cannot hold: report the overflow, copy nothing
    if ((R >= 0 && R >= t.Rcap) || (R < 0 && res >= t.Rcap)) {
      n = 0;
      res = -1;
      R = -1;
      if (blockIdx.x == 0) rstate[1] = 1;
    }
    if (blockIdx.x == 0) {
      if (R >= 0) rstate[0] = R;
      *resume = res;
    }
    s_n = n;
  }
  __syncthreads();
  const int n = s_n;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int q = 0; q < n; q++) {
    const int v = sv[q], s = ss[q], e = se[q], G = sG[q], e2 = sE2[q];
    const uint64_t* Hv = sp.H + (size_t)v * sp.Hcap * N;
    for (size_t i = i0; i < (size_t)(e - s) * N; i += stride) {
      const int j = s + (int)(i / N), c = (int)(i % N);
      const int P = (int)(uint32_t)Hv[(size_t)j * N + c];
      if (P != INF32) t.C[(size_t)(G + j - s) * N + c] = P;
    }
    if (e2 > s) {
      const uint64_t* Sv = sp.SSCH + (size_t)v * sp.Hcap * N * NW;
      for (size_t i = i0; i < (size_t)(e2 - s) * N * NW; i += stride) {
        const size_t jj = i / ((size_t)N * NW), rem = i % ((size_t)N * NW);
        const int j = s + 1 + (int)jj, c = (int)(rem / NW);
        const int P = (int)(uint32_t)Hv[(size_t)j * N + c];
        if (P != INF32)
          ssc[((size_t)(G + j - s) * N + c) * NW + rem % NW] = Sv[((size_t)j * N + c) * NW + rem % NW];
      }
    }
  }
}

template __global__ void k_rounds_coop_spec<512>(Tables, const int32_t*, const int32_t*, const int32_t*,
                                                 CoopSpec, int32_t*);
template __global__ void k_rounds_coop_spec<1024>(Tables, const int32_t*, const int32_t*, const int32_t*,
                                                  CoopSpec, int32_t*);

}  // namespace hge
