// hge_wide.hip — coordinate and round kernels for wide hashgraphs (N > 32).
//
// The chunked coordinate pipeline of hge_kernels.hip keeps N x N head tables
// and per-chunk records in LDS, which stops fitting past N = 64.  Here the
// coordinates are built from bandwidth-friendly passes instead:
//
//   1. lastAncestors by chain-prefix sweeps.  Along a creator chain,
//      InitEventCoordinates (hashgraph.go:399-463) is a prefix max:
//        LA[(j,k)] = max(own(j,k), LA[(j,k-1)], LA[op(j,k)]).
//      A sweep recomputes every new row from the CURRENT table (in place,
//      segments of SEG positions per workgroup, carry = the stored row before
//      the segment).  Every value ever stored is a lower bound of the true
//      one and the update is monotone, so a sweep that changes nothing has
//      reached the fixed point, which for an acyclic recurrence is unique:
//      the exact table.  ~10-20 sweeps (SURVEY §7 "windowed Jacobi").
//      Each sweep streams op rows and own rows: coalesced 4N-byte rows.
//   2. LA -> LAT (chain j, column c, position k) by a tiled LDS transpose.
//   3. firstDescendants as runs (UpdateAncestorFirstDescendant,
//      hashgraph.go:466-494): chain-j event k is the first chain-j descendant
//      of chain-c positions (LAT[j][c][k-1], LAT[j][c][k]], so
//      FDT[j][c][q] = k there: contiguous runs, coalesced writes.
//   4. FDT -> FD rows (the layout every reader uses) by a tiled transpose.
//
// Rounds for N > 32 use a cooperative kernel: one workgroup per chain, one
// grid barrier per round (k_rounds_coop below).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

// LA[(j, k)] = -1 for the new positions k in [olen_j, len_j) of every chain
__global__ void k_la_clear(Tables t, const int32_t* olen, const int32_t* len) {
  const int j = blockIdx.y;
  const int N = t.N;
  const int64_t lo = (int64_t)olen[j] * N, hi = (int64_t)len[j] * N;
  int32_t* base = t.LA + (size_t)j * t.ccap * N;
  for (int64_t e = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < hi;
       e += (int64_t)gridDim.x * blockDim.x)
    base[e] = -1;
}

// One in-place sweep.  G = 256/NP segments per workgroup, NP threads (columns)
// per segment.  segs[s] = (chain, first position).
template <int NP>
__global__ void __launch_bounds__(256) k_la_sweep(Tables t, const int2* segs, int nseg, int SEG,
                                                  const int32_t* len, int32_t* changed) {
  constexpr int G = 256 / NP;
  constexpr int SEGMAX = 64;
  __shared__ int64_t s_off[G][SEGMAX];
  const int N = t.N;
  const int g = threadIdx.x / NP, i = threadIdx.x - (threadIdx.x / NP) * NP;
  const int sidx = blockIdx.x * G + g;
  const bool valid = sidx < nseg;
  int j = 0, k0 = 0, k1 = 0;
  if (valid) {
    const int2 sg = segs[sidx];
    j = sg.x;
    k0 = sg.y;
    k1 = min(k0 + SEG, len[j]);
  }
  for (int kk = i; kk < SEG; kk += NP) {
    int64_t off = -1;
    if (valid && k0 + kk < k1) {
      const int x = t.chain[(size_t)j * t.ccap + k0 + kk];
      const int o = t.op[x];
      if (o >= 0) off = (int64_t)rowoff(t, t.creator[o], t.index[o]);
    }
    s_off[g][kk] = off;
  }
  __syncthreads();
  const bool act = valid && i < N;
  bool ch = false;
  if (act) {
    int v = (k0 > 0) ? t.LA[rowoff(t, j, k0 - 1) + i] : -1;
    for (int kb = k0; kb < k1; kb += 8) {
      int a[8], old[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int k = kb + u;
        a[u] = -1;
        old[u] = -1;
        if (k < k1) {
          const int64_t off = s_off[g][k - k0];
          if (off >= 0) a[u] = t.LA[off + i];
          old[u] = t.LA[rowoff(t, j, k) + i];
        }
      }
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int k = kb + u;
        if (k < k1) {
          v = max(v, a[u]);
          if (i == j) v = max(v, k);
          const int nv = max(v, old[u]);
          v = nv;
          if (nv != old[u]) {
            t.LA[rowoff(t, j, k) + i] = nv;
            ch = true;
          }
        }
      }
    }
  }
  if (__ballot(ch) && (threadIdx.x & 63) == __builtin_ctzll(__ballot(ch))) atomicOr(changed, 1);
}

// Tiled transposes through LDS (64 x 64 tiles, 256 threads).
//   mode 0: LA[(j,k)][c] -> LAT[j][c][k] for k in [klo_j, len_j)
//   mode 1: FDT[j][c][q] -> FD[(c,q)][j] for q in [qlo_c, len_c)
// grid: (tiles along positions, tiles along the N columns, chain)
__global__ void __launch_bounds__(256) k_transpose(Tables t, const int32_t* LAT_or_FDT, int32_t* out,
                                                   const int32_t* plo, const int32_t* len, int mode) {
  __shared__ int32_t tile[64][65];
  const int N = t.N;
  const size_t ccap = t.ccap;
  const int a = blockIdx.z;  // mode 0: chain j; mode 1: source chain c
  const int p0 = plo[a] + blockIdx.x * 64;
  const int pend = len[a];
  if (p0 >= pend) return;
  const int c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  if (mode == 0) {
    // read rows (j, p) columns [c0, c0+64): row-major, coalesced along c
    for (int r = ty; r < 64; r += 4) {
      const int p = p0 + r, c = c0 + tx;
      tile[r][tx] = (p < pend && c < N) ? t.LA[rowoff(t, a, p) + c] : 0;
    }
    __syncthreads();
    // write LAT[a][c][p]: coalesced along p
    int32_t* LAT = out;
    for (int r = ty; r < 64; r += 4) {
      const int c = c0 + r, p = p0 + tx;
      if (c < N && p < pend) LAT[((size_t)a * N + c) * ccap + p] = tile[tx][r];
    }
  } else {
    // read FDT[j][a][q] for j in [c0, c0+64): coalesced along q
    const int32_t* FDT = LAT_or_FDT;
    for (int r = ty; r < 64; r += 4) {
      const int jj = c0 + r, q = p0 + tx;
      tile[r][tx] = (jj < N && q < pend) ? FDT[((size_t)jj * N + a) * ccap + q] : 0;
    }
    __syncthreads();
    // write FD[(a, q)][j]: coalesced along j
    for (int r = ty; r < 64; r += 4) {
      const int q = p0 + r, jj = c0 + tx;
      if (q < pend && jj < N) t.FD[rowoff(t, a, q) + jj] = tile[tx][r];
    }
  }
}

// FDT[j][c][q] = INF32 for the new positions q in [olen_c, len_c)
__global__ void k_fdt_clear(Tables t, int32_t* FDT, const int32_t* olen, const int32_t* len) {
  const int c = blockIdx.y, j = blockIdx.z;
  const int lo = olen[c], hi = len[c];
  int32_t* row = FDT + ((size_t)j * t.N + c) * t.ccap;
  for (int q = lo + blockIdx.x * blockDim.x + threadIdx.x; q < hi; q += gridDim.x * blockDim.x)
    row[q] = INF32;
}

// runs: chain-j event k (new) is the first chain-j descendant of chain-c
// positions (LAT[j][c][k-1], LAT[j][c][k]]
__global__ void k_fdt_runs(Tables t, const int32_t* LAT, int32_t* FDT, const int32_t* olen,
                           const int32_t* len) {
  const int c = blockIdx.y, j = blockIdx.z;
  const int k = olen[j] + blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len[j]) return;
  const size_t base = ((size_t)j * t.N + c) * t.ccap;
  const int hi = LAT[base + k];
  const int lo = k > 0 ? LAT[base + k - 1] : -1;
  int32_t* row = FDT + base;
  for (int q = lo + 1; q <= hi; q++) row[q] = k;
}

// lowest chain-c position whose FD row a new event can change:
// min over chains j with old events of LA[(j, olen_j - 1)][c] + 1
__global__ void k_fd_qlo(Tables t, const int32_t* olen, const int32_t* len, int32_t* qlo) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= t.N) return;
  int m = olen[c];  // the new positions themselves
  for (int j = 0; j < t.N; j++) {
    if (len[j] == olen[j]) continue;  // chain j got no new event
    const int ol = olen[j];
    const int v = ol > 0 ? t.LA[rowoff(t, j, ol - 1) + c] + 1 : 0;
    m = min(m, v);
  }
  qlo[c] = max(0, m);
}

}  // namespace hge

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
// with an exact bisection fallback past the window.  One grid barrier per
// round publishes C_{r+1}.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned target) {
  __syncthreads();
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 26)) {  // ~seconds: a co-residency failure, never a normal wait
        ok = 0;
        break;
      }
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

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

__global__ void __launch_bounds__(256) k_rounds_coop(Tables t, const int32_t* FDT, const int32_t* olen,
                                                     const int32_t* len, int32_t* rstate, int rlo,
                                                     int Rprev, unsigned* bar, int32_t* err) {
  constexpr int NB = 64;  // histogram bins
  __shared__ int sP[256];
  __shared__ uint16_t sU[64][256];       // member rows, 64 columns at a time: sU[i - i0][d]
  __shared__ uint32_t sH[NB / 2][256];    // per-thread histograms, two 16-bit bins per word
  __shared__ uint32_t sH2[NB];
  __shared__ int s_any, s_sel, s_lo, s_hi, s_cnt;
  const int N = t.N, SM = t.SM;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int G = gridDim.x;
  const int lenc = len[c];
  if (tid < N) {
    int P = t.C[(size_t)rlo * N + tid];
    if (rlo == 0 && olen[tid] == 0 && len[tid] > 0) P = 0;
    sP[tid] = P;
    if (c == 0 && rlo == 0 && olen[tid] == 0 && len[tid] > 0) t.C[tid] = 0;
  }
  __syncthreads();
  unsigned nbar = 0;
  for (int r = rlo;; r++) {
    if (r + 1 >= t.Rcap) {
      if (c == 0 && tid == 0) rstate[1] = 1;
      break;
    }
    const int Pc = sP[c];
    for (int w = tid; w < (NB / 2) * 256; w += 256) (&sH[0][0])[w] = 0;
    if (tid < NB) sH2[tid] = 0;
    const int d = tid;
    const int Pd = (d < N) ? sP[d] : INF32;
    const bool dact = d < N && Pd != INF32 && Pc != INF32;
    int nfin = 0;  // finite gathered values of thread d
    for (int i0 = 0; i0 < N; i0 += 64) {
      const int ni = min(64, N - i0);
      __syncthreads();
      // stage u = FD[(d', P_d')][i0 + ii]: rows are contiguous, 64 columns per row
      for (int item = tid; item < N * 64; item += 256) {
        const int dd = item >> 6, ii = item & 63;
        const int P = sP[dd];
        int u = INF32;
        if (ii < ni && P != INF32) u = t.FD[rowoff(t, dd, P) + i0 + ii];
        sU[ii][dd] = (u == INF32) ? 0xFFFF : (uint16_t)u;
      }
      __syncthreads();
      if (dact) {
        const int32_t* fdt = FDT + ((size_t)c * N + i0) * t.ccap;
        for (int ib = 0; ib < ni; ib += 16) {
          int v[16];
#pragma unroll
          for (int k = 0; k < 16; k++) {
            v[k] = INF32;
            if (ib + k < ni) {
              const int u = sU[ib + k][d];
              if (u != 0xFFFF) v[k] = fdt[(size_t)(ib + k) * t.ccap + u];
            }
          }
#pragma unroll
          for (int k = 0; k < 16; k++) {
            if (v[k] == INF32) continue;
            nfin++;
            const int b = min(max(v[k] - Pc, 0), NB - 1);
            atomicAdd(&sH[b >> 1][d], 1u << ((b & 1) * 16));
          }
        }
      }
    }
    __syncthreads();
    // first level: fss_c(m_d) = SM-th smallest gathered value
    int fss = INF32;
    if (dact && nfin >= SM) {
      int cum = 0, b = 0;
      for (; b < NB; b++) {
        cum += (sH[b >> 1][d] >> ((b & 1) * 16)) & 0xFFFF;
        if (cum >= SM) break;
      }
      if (b < NB - 1) {
        fss = Pc + b;
      } else {
        // past the window: bisection on the exact count
        int lo = Pc + NB - 1, hi = lenc;  // answer in [lo, hi) or INF
        if (fss_count_le(t, FDT, c, d, Pd, hi - 1) < SM) {
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
      if (fss != INF32 && d == c) fss = max(fss, Pc + 1);  // x never strongly sees itself
      if (fss >= lenc) fss = INF32;
    }
    // second level: SM-th smallest fss over the members
    if (fss != INF32) atomicAdd(&sH2[min(max(fss - Pc, 0), NB - 1)], 1u);
    __syncthreads();
    if (tid == 0) {
      int cum = 0, b = 0, sel = INF32;
      for (; b < NB; b++) {
        cum += sH2[b];
        if (cum >= SM) break;
      }
      if (b < NB - 1) sel = Pc + b;
      s_sel = sel;
      s_lo = (b == NB - 1) ? 1 : 0;  // exact selection needed
    }
    __syncthreads();
    if (s_lo) {
      // exact: bisection over the member values with block counts
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
    }
    nbar++;
    if (!grid_barrier(bar, nbar * (unsigned)G)) {
      if (tid == 0) atomicOr(err, 1);
      return;
    }
    if (tid == 0) s_any = 0;
    __syncthreads();
    if (tid < N) {
      const int P = t.C[(size_t)(r + 1) * N + tid];
      sP[tid] = P;
      if (P != INF32) s_any = 1;
    }
    __syncthreads();
    if (!s_any) {
      if (c == 0 && tid == 0) rstate[0] = max(rstate[0], r + 1);
      break;
    }
  }
}

}  // namespace hge
