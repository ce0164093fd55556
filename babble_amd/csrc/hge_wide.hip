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
