// hge_wide32.hip — the wide path (N > 32) past 65,534 events per chain.
//
// The wide kernels keep chain positions as uint16: the packed lastAncestors table
// (LA16 = LA + 1), the rounds walk's LA + 2 / FD + 1 encodings and theta's packed
// columns.  The reference has no such cap (hashgraph.go:328-363), so when a chain
// reaches it the engine switches, for good, to int32 positions (to_wide32 in
// hge_engine.hip): the int32 sweeps and transposes of the N <= 32 path (their
// kernels take any N), and the three kernels below in place of the packed ones.
// They are plain and slow next to the packed path; they keep a long-running node
// accepting honest events with results identical to the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

// LA16 (LA + 1 as uint16 pairs) -> int32 LA rows for the positions [0, upto_c) of
// every chain c (the events with coordinates at the switch).  grid (position
// tiles of 256 / N-column passes, chain)
__global__ void k_la16_to_la32(Tables t, const uint32_t* LA16, const int32_t* upto) {
  const int c = blockIdx.y, N = t.N;
  const int n = upto[c];
  const size_t rowlen = (size_t)N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)n * N;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(e / N), col = (int)(e - (e / N) * N);
    const size_t row = (size_t)c * t.ccap + p;
    const uint32_t w = LA16[row * (size_t)t.NW2 + (col >> 1)];
    t.LA[row * rowlen + col] = (int)((w >> ((col & 1) << 4)) & 0xFFFFu) - 1;
  }
}

// the round-r frontier member of chain d (the rounds walk's row-0 rule: a chain
// whose first event is new starts round 0 at position 0)
__device__ __forceinline__ int w32_member(const Tables& t, const int32_t* olen, const int32_t* len, int r, int d) {
  if (r == 0 && olen[d] == 0 && len[d] > 0) return 0;
  return t.C[(size_t)r * t.N + d];
}

// StronglySee((c, p), m) for the member of thread d (hashgraph.go:189-208):
// #{i : LA[(c,p)][i] >= FD[m][i]} >= SM, the LA row staged in LDS by the caller
__device__ __forceinline__ bool w32_ss(const Tables& t, const int* sla, int d, int md) {
  if (md == INF32) return false;
  const size_t frow = (size_t)d * t.ccap + md;
  int n = 0;
  for (int i = 0; i < t.N; i++) n += sla[i] >= fd_at(t, frow, i) ? 1 : 0;
  return n >= t.SM;
}

// One round of the frontier recurrence with int32 positions:
// C_{r+1}[c] = min { p >= C_r[c] : #{d : StronglySee((c, p), m_d)} >= SM }, block c,
// thread d = member d (blockDim.x >= N).  Rows from an earlier batch (r + 1 < Rprev,
// not INF) stand (a new event cannot change a kept row); the strongly-see bits of
// the chosen row against the round-r members go to ssc as in the packed walk.
// alive = 1 if some chain has a row r + 1.  The host launches it round by round.
__global__ void __launch_bounds__(256) k_round_step32(Tables t, const int32_t* olen, const int32_t* len, int r,
                                                      int Rprev, uint64_t* ssc, int32_t* alive) {
  __shared__ int sla[256];
  __shared__ int s_cnt;
  const int N = t.N, NW = t.NW;
  const int c = blockIdx.x, d = threadIdx.x;
  const int Pc = w32_member(t, olen, len, r, c);
  if (r == 0 && d == 0 && Pc == 0 && t.C[c] != 0) t.C[c] = 0;
  const int md = d < N ? w32_member(t, olen, len, r, d) : INF32;
  const int lenc = len[c];
  const int cur = (r + 1 < Rprev) ? t.C[(size_t)(r + 1) * N + c] : INF32;
  // count(p) >= SM at p?  (block-uniform result)
  auto probe = [&](int p, bool& mine) -> bool {
    __syncthreads();
    if (d < N) sla[d] = la_row(t, (size_t)c * t.ccap + p, d);
    if (d == 0) s_cnt = 0;
    __syncthreads();
    mine = d < N && w32_ss(t, sla, d, md);
    const uint64_t b = __ballot(mine);
    if ((d & 63) == 0) atomicAdd(&s_cnt, (int)__popcll(b));
    __syncthreads();
    return s_cnt >= t.SM;
  };
  int nxt = INF32;
  bool mine = false;
  if (Pc != INF32 && Pc < lenc) {
    if (cur != INF32) {
      nxt = cur;
    } else {
      // exponential then binary search for the first passing position (monotone in p)
      int lo = Pc, step = 1, hi = -1;
      for (int p = Pc;; step <<= 1, p = min(Pc + step - 1, lenc - 1)) {
        if (probe(p, mine)) {
          hi = p;
          break;
        }
        lo = p + 1;
        if (p == lenc - 1) break;
      }
      if (hi >= 0) {
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (probe(mid, mine)) hi = mid;
          else lo = mid + 1;
        }
        nxt = hi;
      }
    }
  }
  if (nxt != INF32) {
    probe(nxt, mine);  // the bits of the chosen row
    if (d == 0 && cur == INF32) t.C[(size_t)(r + 1) * N + c] = nxt;
    const uint64_t b = __ballot(mine);
    if ((d & 63) == 0 && (d >> 6) < NW) ssc[((size_t)(r + 1) * N + c) * NW + (d >> 6)] = b;
    if (d == 0) atomicOr(alive, 1);
  }
}

// theta for N > 64 with int32 positions (k_seg_theta_wide's packed columns hold
// uint16): thread = creator cx, the (|fws|/2 + 1)-th largest LA[w][cx] over the
// segment's famous witnesses w by bisection over [min, max], rows read from HBM.
template <int NWT>
__global__ void __launch_bounds__(256) k_seg_theta32(Tables t, const int32_t* seg_round, const int32_t* segoff,
                                                     const int32_t* segcnt, int nr, const uint64_t* seg_fws,
                                                     int32_t* theta) {
  __shared__ int s_row[256];
  __shared__ int s_nf;
  const int N = t.N, tid = threadIdx.x;
  for (int q = blockIdx.x; q < nr; q += gridDim.x) {
    const int cnt = segcnt[q];
    for (int l = 0; l < cnt; l++) {
      const int sg = segoff[q] + l;
      const int i = seg_round[sg];
      uint64_t fw[NWT];
      int nfw = 0;
#pragma unroll
      for (int w = 0; w < NWT; w++) {
        fw[w] = seg_fws[(size_t)sg * NWT + w];
        nfw += __popcll(fw[w]);
      }
      const int d = tid;
      if (d < N && ((fw[d >> 6] >> (d & 63)) & 1ull)) {
        int rank = __popcll(fw[d >> 6] & ((1ull << (d & 63)) - 1));
#pragma unroll
        for (int w = 0; w < NWT; w++) rank += w < (d >> 6) ? __popcll(fw[w]) : 0;
        const int x = t.W[(size_t)i * N + d];
        s_row[rank] = d * t.ccap + t.index[x];
      }
      if (tid == 0) s_nf = nfw;
      __syncthreads();
      const int nf = s_nf, cx = tid;
      if (cx < N) {
        int th = (int)0x80000000;
        if (nf > 0) {
          int vmin = INT32_MAX, vmax = INT32_MIN;
          for (int k = 0; k < nf; k++) {
            const int v = la_row(t, (size_t)s_row[k], cx);
            vmin = min(vmin, v);
            vmax = max(vmax, v);
          }
          const int kk = nf / 2 + 1;  // k-th largest = largest v with count(>= v) >= kk
          int lo = vmin, hi = vmax;
          while (lo < hi) {
            const int mid = lo + (int)(((int64_t)hi - lo + 1) >> 1);
            int c2 = 0;
            for (int k = 0; k < nf; k++) c2 += la_row(t, (size_t)s_row[k], cx) >= mid ? 1 : 0;
            if (c2 >= kk) lo = mid;
            else hi = mid - 1;
          }
          th = lo;
        }
        theta[(size_t)sg * N + cx] = th;
      }
      __syncthreads();
    }
  }
}

}  // namespace hge
