// hge_coords_win.hip — lastAncestors (InitEventCoordinates, hashgraph.go:399-463)
// for 32 < N <= 256 by windowed exact propagation in insertion order.
//
// Column c of LA is a scalar propagation over the DAG in insertion
// (topological) order:  LA[x][c] = max(LA[sp(x)][c], LA[op(x)][c], [creator(x)
// == c] index(x)).  The only state it needs at any point of the order is the LA
// row of every chain's current head (its last inserted event): N rows of N
// uint16, 128 KB at N = 256 -- one workgroup's LDS.  So a workgroup walks a
// window of consecutive insertion ids exactly, with no global dependence chain:
//   * k_lw_plan cuts the ids into chunks of 64 and gives every event a level
//     inside its chunk: above its self-parent, its other-parent when that is in
//     the chunk, and every earlier event of the chunk that reads the head row
//     this event replaces (so an other-parent head is still in LDS when read);
//     the chunk's events are stored sorted by level;
//   * a level is one read phase (self and other-parent head rows from LDS, all
//     N columns of up to 1024 / (N/2) events at once, packed u16 max), a
//     barrier, one write phase (the head row in LDS and the packed row to HBM:
//     2N coalesced bytes per event), a barrier.
// Windows run in parallel, each starting from the head rows at its first id as
// they are stored at that moment (the windows before it are being computed
// concurrently; in the first pass a new head row of another window is taken as
// its own column only, so nothing unwritten is ever read).  Every stored value
// is a lower bound of the exact one and every input only grows, so repeating
// the pass converges to the exact table (the unique fixed point, as for the
// sweeps of hge_coords.hip), and a pass that changes no row proves it.  A
// window's rows stop depending on its starting rows after the information
// horizon (the gossip spreading time, a few thousand ids), so a later pass
// recomputes a window only until its running head rows equal the previous
// pass's (compared through per-row sums: rows only grow, so equal sums mean
// equal rows) and skips windows whose starting rows did not change.  Random
// gossip converges in three passes, the last one a no-op, against ~20 Jacobi
// sweeps of the whole table.
//
// An other-parent that was not its chain's head when the event was inserted
// ("risky": possible in general DAGs, never in the synthetic gossip) is read
// from HBM; a chunk holding one drains its stores before each barrier, and a
// window with one after its convergence point is recomputed to its end.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

constexpr int LW_K = 64;          // ids per chunk (one wave plans a chunk)
constexpr int LW_RISKY = 1;       // other-parent not the head of its chain at insertion
constexpr int LW_INWIN = 2;       // other-parent inside the event's window
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

// wpos[w][c] = first chain-c position whose id is >= the window's first id
// (the head before the window is wpos - 1); risky[w] = -1; zero[0, nzero) = 0
__global__ void k_lw_pos(Tables t, int64_t n0, int WN, int G, const int32_t* len, int32_t* wpos,
                         int32_t* risky, int32_t* zero, int nzero) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nzero) zero[i] = 0;
  if (i < G) risky[i] = -1;
  if (i >= G * t.N) return;
  const int w = i / t.N, c = i - w * t.N;
  const int64_t s0 = n0 + (int64_t)w * WN;
  const int32_t* ch = t.chain + (size_t)c * t.ccap;
  int lo = 0, hi = len[c];
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)ch[mid] < s0) lo = mid + 1;
    else hi = mid;
  }
  wpos[i] = lo;
}

// One wave per chunk of 64 ids.  plan[id - n0] for the chunk's ids, sorted by
// level: {creator | level << 16 | flags << 24, index, opc, opp} (opc = -1: no
// other-parent).  risky[w] = the last risky id of window w.
__device__ __forceinline__ void lw_plan_chunk(const Tables& t, int64_t n0, int64_t n1, int WN, const int32_t* len,
                                              int4* plan, int32_t* risky, int64_t cs) {
  const int lane = threadIdx.x & 63;
  if (cs >= n1) return;  // wave-uniform
  const int64_t e = cs + lane;
  const bool v = e < n1;
  const int64_t wst = n0 + ((cs - n0) / WN) * WN;
  int a = 0, k = 0, opc = -1, opp = -1, flags = 0;
  int keysp = -2, keyop = -3;  // (chain << 16 | position) of the self- and other-parent
  uint64_t pred = 0;           // lanes this event must follow
  if (v) {
    a = t.creator[e];
    k = t.index[e];
    if (k > 0) {
      const int s = t.chain[(size_t)a * t.ccap + k - 1];
      if (s >= cs) pred |= 1ull << (s - cs);
      keysp = (a << 16) | (k - 1);
    }
    const int o = t.op[e];
    if (o >= 0) {
      opc = t.creator[o];
      opp = t.index[o];
      keyop = (opc << 16) | opp;
      if (o >= cs) pred |= 1ull << (o - cs);
      if (o >= wst) flags |= LW_INWIN;
      if (opp + 1 < len[opc] && (int64_t)t.chain[(size_t)opc * t.ccap + opp + 1] < e) flags |= LW_RISKY;
    }
  }
  // earlier readers of the head this event replaces (its self-parent as their other-parent)
  for (int q = 0; q < 63; q++) {
    const int kq = __builtin_amdgcn_readlane(keyop, q);
    if (q < lane && kq == keysp) pred |= 1ull << q;
  }
  // levels in lane (= id) order: every predecessor has a lower lane
  int lvl = 0;
  for (int q = 0; q < 63; q++) {
    const int lq = __builtin_amdgcn_readlane(lvl, q);
    if ((pred >> q) & 1ull) lvl = max(lvl, lq + 1);
  }
  int maxl = v ? lvl : 0;
  for (int off = 32; off >= 1; off >>= 1) maxl = max(maxl, __shfl_xor(maxl, off));
  int rank = 0, base = 0;
  const uint64_t lt = (1ull << lane) - 1;
  for (int L = 0; L <= maxl; L++) {
    const uint64_t m = __ballot(v && lvl == L);
    if (v && lvl == L) rank = base + __builtin_popcountll(m & lt);
    base += __builtin_popcountll(m);
  }
  if (v) plan[cs - n0 + rank] = make_int4(a | (lvl << 16) | (flags << 24), k, opc, opp);
  const uint64_t rm = __ballot(v && (flags & LW_RISKY));
  if (rm && lane == 63 - __builtin_clzll(rm)) atomicMax(&risky[(cs - n0) / WN], (int32_t)e);
}
__global__ void __launch_bounds__(256) k_lw_plan(Tables t, int64_t n0, int64_t n1, int WN,
                                                 const int32_t* len, int4* plan, int32_t* risky) {
  lw_plan_chunk(t, n0, n1, WN, len, plan, risky, n0 + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * LW_K);
}

// WPT consecutive packed words of an LDS row / to HBM (16-, 8- or 4-byte accesses)
template <int WPT>
__device__ __forceinline__ void lw_lds_read(const uint32_t* p, uint32_t (&v)[WPT]) {
  if constexpr (WPT == 4) {
    const uint4 q = *(const uint4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else if constexpr (WPT == 2) {
    const uint2 q = *(const uint2*)p;
    v[0] = q.x; v[1] = q.y;
  } else {
    v[0] = *p;
  }
}
template <int WPT>
__device__ __forceinline__ void lw_lds_write(uint32_t* p, const uint32_t (&v)[WPT]) {
  if constexpr (WPT == 4) *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
  else if constexpr (WPT == 2) *(uint2*)p = make_uint2(v[0], v[1]);
  else *p = v[0];
}
template <int WPT>
__device__ __forceinline__ void lw_global_write(uint32_t* p, const uint32_t (&v)[WPT]) {
  lw_lds_write<WPT>(p, v);
}

// One pass over every window (one workgroup each).  pass 1 computes every new row;
// pass > 1 recomputes a window from its current starting rows until its running
// head rows equal the previous pass's.  rsum[plan slot] = sum of the row's 16-bit
// values (LA + 1); initbuf[w] = the starting rows a pass used; prev / changed:
// the previous pass's changed flag (0: converged, return at once) and this pass's.
// plan_here (one window, an online call): the window's 16 waves plan its chunks
// first (k_lw_plan's work; the plan and the risky id are block-visible after the
// barrier), one launch less
template <int NPOW>
__global__ void __launch_bounds__(1024) k_la_win(Tables t, int4* plan, int64_t n0, int64_t n1, int WN,
                                                 const int32_t* wpos, const int32_t* olen, uint32_t* initbuf,
                                                 int32_t* risky, uint32_t* rsum, int pass,
                                                 const int32_t* prev, int32_t* changed, const int32_t* plan_len) {
  constexpr int RWW = NPOW / 2;         // packed words per (padded) row
  constexpr int WPT = NPOW / 64;         // words per thread: 32 threads per event
  constexpr int TPE = RWW / WPT;         // = 32
  constexpr int SL = 1024 / TPE;         // events per read/write phase (32)
  constexpr int MAXI = (LW_K + SL - 1) / SL;
  static_assert(TPE == 32, "half a wave per event");
  __shared__ uint32_t s_st[NPOW * RWW] __attribute__((aligned(16)));  // head rows [chain][word]
  __shared__ int s_hp[NPOW], s_ol[NPOW];
  __shared__ int4 s_ev[LW_K];
  __shared__ uint32_t s_sum[LW_K];
  __shared__ int s_lvoff[LW_K + 1];
  __shared__ uint32_t s_dirty[NPOW / 32];
  __shared__ int s_nlv, s_wait;
  if (prev && *prev == 0) return;  // converged: the flag stays 0
  if (plan_len) {
    for (int64_t cs = n0 + (int64_t)(threadIdx.x >> 6) * LW_K; cs < n1; cs += (int64_t)(blockDim.x >> 6) * LW_K)
      lw_plan_chunk(t, n0, n1, WN, plan_len, plan, risky, cs);
    __syncthreads();
  }
  const int N = t.N, W = t.NW2;
  const int w = blockIdx.x;
  const int64_t s0 = n0 + (int64_t)w * WN;
  if (s0 >= n1) return;
  const int64_t s1 = min(n1, s0 + (int64_t)WN);
  const int tid = threadIdx.x;
  const int slot = tid / TPE, wd0 = (tid - (tid / TPE) * TPE) * WPT;  // first owned word
  if (tid < NPOW / 32) s_dirty[tid] = 0;
  __syncthreads();
  // starting rows: the heads before s0 as stored (pass 1: a new row of another
  // window is not written yet, take its own column only)
  uint32_t* ib = initbuf + (size_t)w * N * W;
  // the head positions first, then every thread's row words with all their loads in
  // flight (a loop with a dependent pair of loads per word was ~45 us per online call
  // at N = 256, where one window holds the whole batch)
  for (int c = tid; c < NPOW; c += 1024) {
    s_hp[c] = c < N ? wpos[(size_t)w * N + c] - 1 : -1;
    s_ol[c] = c < N ? olen[c] : 0;
  }
  __syncthreads();
  constexpr int PERT = NPOW * RWW / 1024;
  uint32_t sv0[PERT];
#pragma unroll
  for (int k = 0; k < PERT; k++) {
    const int i = tid + k * 1024;
    const int c = i / RWW, q = i - (i / RWW) * RWW;
    uint32_t val = 0;
    if (c < N && q < W) {
      const int hp = s_hp[c];
      if (hp >= 0) {
        if (hp < s_ol[c] || pass > 1) val = t.LA16[((size_t)c * t.ccap + hp) * W + q];
        else val = (q == (c >> 1)) ? (uint32_t)(hp + 1) << ((c & 1) * 16) : 0u;
      }
    }
    sv0[k] = val;
  }
#pragma unroll
  for (int k = 0; k < PERT; k++) {
    const int i = tid + k * 1024;
    const int c = i / RWW, q = i - (i / RWW) * RWW;
    if (c < N && q < W) {
      if (pass > 1 && ib[(size_t)c * W + q] != sv0[k]) atomicOr(&s_dirty[c >> 5], 1u << (c & 31));
      ib[(size_t)c * W + q] = sv0[k];
    }
    s_st[i] = sv0[k];
  }
  const int rl = risky[w];  // last risky id of the window (-1: none)
  __syncthreads();
  if (pass > 1) {
    bool clean = rl < s0;
    for (int q = 0; q < NPOW / 32; q++) clean &= s_dirty[q] == 0;
    if (clean) return;  // same starting rows, nothing to revisit: the rows stand
  }
  // the chunk's plan entries (and, pass > 1, the previous pass's row sums) one chunk ahead
  int4 nx = make_int4(-1, 0, -1, 0);
  uint32_t nxs = 0, cur_s = 0;
  if (tid < LW_K && s0 + tid < s1) {
    nx = plan[s0 - n0 + tid];
    if (pass > 1) nxs = rsum[s0 - n0 + tid];
  }
  bool anyc = false;
  for (int64_t cs = s0; cs < s1; cs += LW_K) {
    const int ne = (int)min((int64_t)LW_K, s1 - cs);
    if (tid < LW_K) {
      s_ev[tid] = nx;
      s_sum[tid] = 0;
      cur_s = nxs;
      // level boundaries of the sorted entries (wave 0)
      const int lv = tid < ne ? (nx.x >> 16) & 0xFF : 0x7FFF;
      const int lp = __shfl(lv, tid > 0 ? tid - 1 : 0);
      const bool start = tid < ne && (tid == 0 || lv != lp);
      const uint64_t m = __ballot(start);
      if (start) s_lvoff[__builtin_popcountll(m & ((1ull << tid) - 1))] = tid;
      const bool rw = tid < ne && ((nx.x >> 24) & (LW_RISKY | LW_INWIN)) == (LW_RISKY | LW_INWIN);
      const bool wt = __ballot(rw) != 0;
      if (tid == 0) {
        s_nlv = __builtin_popcountll(m);
        s_lvoff[__builtin_popcountll(m)] = ne;
        s_wait = wt ? 1 : 0;
      }
      const int64_t nc = cs + LW_K + tid;
      nx = make_int4(-1, 0, -1, 0);
      if (nc < s1) nx = plan[nc - n0];
    }
    __syncthreads();
    if (pass > 1 && cs > s0) {
      // the previous chunk left every head row as the previous pass had it and no
      // risky event follows: the rest of the window is unchanged
      bool clean = rl < cs;
      for (int q = 0; q < NPOW / 32; q++) clean &= s_dirty[q] == 0;
      if (clean) break;
    }
    const bool wt = s_wait != 0;
    if (wt) {  // a risky read of this chunk may need rows stored by earlier chunks
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    const int nlv = s_nlv;
    for (int L = 0; L < nlv; L++) {
      const int lo = s_lvoff[L], hi = s_lvoff[L + 1];
      uint32_t nv[MAXI][WPT];
#pragma unroll
      for (int i = 0; i < MAXI; i++) {
        const int j = lo + slot + i * SL;
        if (lo + i * SL < hi && j < hi) {
          const int4 en = s_ev[j];
          const int a = en.x & 0xFFFF, k = en.y, opc = en.z, opp = en.w;
          uint32_t v[WPT], o[WPT];
          lw_lds_read<WPT>(&s_st[a * RWW + wd0], v);
#pragma unroll
          for (int u = 0; u < WPT; u++) o[u] = 0;
          if (opc >= 0) {
            if (s_hp[opc] == opp) {
              lw_lds_read<WPT>(&s_st[opc * RWW + wd0], o);
            } else {
              const uint32_t* src = t.LA16 + ((size_t)opc * t.ccap + opp) * W;
#pragma unroll
              for (int u = 0; u < WPT; u++) {
                const int q = wd0 + u;
                if (q >= W) continue;
                if (opp < s_ol[opc]) o[u] = src[q];  // an old, final row
                else if ((en.x >> 24) & LW_INWIN)     // written by this workgroup this pass
                  o[u] = __hip_atomic_load(src + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (pass == 1) o[u] = (q == (opc >> 1)) ? (uint32_t)(opp + 1) << ((opc & 1) * 16) : 0u;
                else o[u] = src[q];  // another window's row: a lower bound
              }
            }
          }
#pragma unroll
          for (int u = 0; u < WPT; u++) {
            uint32_t x = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, v[u]),
                                                                               __builtin_bit_cast(u16x2_t, o[u])));
            if (wd0 + u == (a >> 1))
              x = __builtin_bit_cast(uint32_t,
                                     __builtin_elementwise_max(__builtin_bit_cast(u16x2_t, x),
                                                               __builtin_bit_cast(u16x2_t, (uint32_t)(k + 1) << ((a & 1) * 16))));
            nv[i][u] = x;
          }
        }
      }
      __syncthreads();  // every read of this level's head rows is done
#pragma unroll
      for (int i = 0; i < MAXI; i++) {
        if (lo + i * SL >= hi) break;  // wave-uniform
        const int j = lo + slot + i * SL;
        uint32_t s = 0;
        if (j < hi) {
          const int4 en = s_ev[j];
          const int a = en.x & 0xFFFF, k = en.y;
          lw_lds_write<WPT>(&s_st[a * RWW + wd0], nv[i]);
          uint32_t* dst = t.LA16 + ((size_t)a * t.ccap + k) * W + wd0;
          if (W == RWW) {
            lw_global_write<WPT>(dst, nv[i]);
          } else {
#pragma unroll
            for (int u = 0; u < WPT; u++)
              if (wd0 + u < W) dst[u] = nv[i][u];
          }
          if (wd0 == 0) s_hp[a] = k;
#pragma unroll
          for (int u = 0; u < WPT; u++) s += (nv[i][u] & 0xFFFFu) + (nv[i][u] >> 16);
        }
        // sum over the event's 32 lanes: rows of 16 by DPP (quad_perm xor 1, xor 2,
        // row_half_mirror, row_mirror), then the two rows by readlane (no LDS permutes)
        int r = (int)s;
        r += __builtin_amdgcn_mov_dpp(r, 0xB1, 0xF, 0xF, false);
        r += __builtin_amdgcn_mov_dpp(r, 0x4E, 0xF, 0xF, false);
        r += __builtin_amdgcn_mov_dpp(r, 0x141, 0xF, 0xF, false);
        r += __builtin_amdgcn_mov_dpp(r, 0x140, 0xF, 0xF, false);
        const uint32_t lo2 = (uint32_t)(__builtin_amdgcn_readlane(r, 0) + __builtin_amdgcn_readlane(r, 16));
        const uint32_t hi2 = (uint32_t)(__builtin_amdgcn_readlane(r, 32) + __builtin_amdgcn_readlane(r, 48));
        const uint32_t tot = (tid & 32) ? hi2 : lo2;
        if ((tid & 31) == 0 && j < hi) s_sum[j] = tot;  // one half-wave per event: no atomics
      }
      if (wt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // rows a risky read may need
      __syncthreads();
    }
    // chunk end (wave 0): row sums, changed rows, the head rows' dirty bits
    if (tid < LW_K) {
      const int4 en = s_ev[tid];
      const bool v = tid < ne;
      const int a = v ? (en.x & 0xFFFF) : -1, k = en.y;
      const uint32_t sm = s_sum[tid];
      bool chg = v;
      if (pass > 1) {
        chg = v && sm != cur_s;
        bool last = v;  // the chain's last event in this chunk sets its dirty bit
        for (int q = 0; q < LW_K; q++) {
          const int aq = __builtin_amdgcn_readlane(a, q), kq = __builtin_amdgcn_readlane(k, q);
          if (aq == a && kq > k) last = false;
        }
        if (last) {
          if (chg) atomicOr(&s_dirty[a >> 5], 1u << (a & 31));
          else atomicAnd(&s_dirty[a >> 5], ~(1u << (a & 31)));
        }
      }
      if (chg) rsum[cs - n0 + tid] = sm;
      anyc |= __ballot(chg) != 0;
      // the next chunk's previous-pass sums (its plan entries have arrived)
      if (pass > 1) {
        const int64_t nc = cs + LW_K + tid;
        nxs = nc < s1 ? rsum[nc - n0] : 0u;
      }
    }
  }
  if (tid == 0 && anyc) *changed = 1;
}

}  // namespace hge
