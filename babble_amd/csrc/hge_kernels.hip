// hge_kernels.hip — CDNA4 (gfx950) kernels of the hashgraph ordering engine.
//
// The reference (mpitid/babble hashgraph.go) evaluates everything lazily per
// event pair behind LRU caches.  Here every schedule-independent quantity is
// computed in bulk over dense, chain-major HBM tables, and the schedule-
// dependent part (DecideFame / DecideRoundReceived, which depend on WHEN
// RunConsensus is called) is replayed exactly, but in parallel over
// (round, call) pairs.  DESIGN.md derives each reformulation; the parity tests
// check them against the Go-faithful oracle.
//
// Tables (N participants; a "row" is N int32 over participants):
//   LA[c][p][:]  lastAncestors index row of the event at chain c position p
//   FD[c][p][:]  firstDescendants index row (INF32 = unset)
//   chain[c][p]  event id at (c, p); ids are dense in insertion order
//   C[r][c]      first position on chain c whose round is >= r (INF32 = none yet)
//   W[r][c]      witness of round r created by c (-1 none)
//   ssb/seeb[r][c][NW]  strongly-see / see bitsets of witness W[r][c] over the
//                slots of round r-1
//   fame[r][c]   0 undefined, 1 true, 2 false (persisted across calls)
#include <hip/hip_runtime.h>
#include <stdint.h>

#define INF32 0x7FFFFFFF

namespace hge {

struct Tables {
  int N, NW, SM, ccap, Rcap;
  int NW2;           // packed uint16 words per LA16 row (ceil(N / 2))
  uint32_t* LA16;    // [N][ccap][NW2]: (LA + 1) as uint16 pairs, the N > 32 sweeps' table
  const int32_t* creator;
  const int32_t* index;
  const int32_t* sp;
  const int32_t* op;
  const int64_t* ts;
  const uint64_t* S;
  const uint8_t* coin;
  const int32_t* ntx;
  int32_t* chain;
  int2* opcp;     // [N][ccap]: (creator, index) of the other-parent, (-1, -1) if none
  int64_t* tsch;  // [N][ccap]: timestamp of the event at (chain, position)
  // N > 16: [N][ccap][N] timestamp of the event at FD[(c, p)][j] minus that of (c, p) itself
  // (0: none; INT32_MIN: outside int32, the row's 64-column tile flagged in FDTW)
  int32_t* FDTD;
  uint8_t* FDTW;  // N > 16: [N][ccap][ceil(N / 64)]: 1 = the tile holds an out-of-range delta
  int32_t* WLA;   // N > 16: [Rcap][N][N] LA[(d, C[r][d])][cx] at [r][cx][d]
  // N > 192, N % 4 == 0, uint16 positions: the same rows as LA + 1 (0: none) in place of
  // WLA (the median reads a lane's 4 thresholds with one 8-byte load)
  uint16_t* WLA16;
  uint16_t* WLR;  // N > 64, packed path: [Rcap][N][N] LA + 1 of the same rows, row-major [r][d][cx] (theta)
  int32_t* LA;
  int32_t* FD;
  // N > 128, N % 4 == 0, uint16 positions (hge_engine.hip fdt16): the firstDescendants
  // rows as uint16 FD + 1 (0xFFFF = none; the rounds walk's packed member format),
  // [N][ccap][N]; FD is then null and every reader goes through fd_at
  uint16_t* FD16;
  int32_t* round;
  uint8_t* wit;
  int32_t* C;
  int32_t* W;
  uint64_t* ssb;
  uint64_t* seeb;
  uint8_t* fame;
  int32_t* rcnt;  // events per round
};

__device__ __forceinline__ size_t rowoff(const Tables& t, int c, int p) {
  return ((size_t)c * t.ccap + p) * (size_t)t.N;
}

// XCD-aware block order: the dispatcher deals workgroup ids round-robin to the 8
// XCDs (each with its own L2), so neighbouring ids -- which a kernel gives
// neighbouring work that shares rows -- land on different L2s and every XCD
// fetches every shared row.  xcd_block maps the id to one of 8 contiguous ranges
// of the grid, one per XCD (a bijection on [0, nb) for any nb).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}


// lastAncestors[row][col], row = chain * ccap + position.  N > 32 keeps only the
// packed table (LA16 = LA + 1 as uint16 pairs, chains below 65,535 events): the
// int32 rows are not materialised, every reader unpacks.  Past that length the
// engine switches to the int32 rows (LA16 = null: hge_engine.hip, to_wide32).
__device__ __forceinline__ int la_row(const Tables& t, size_t row, int col) {
  if (t.LA16) {
    const uint32_t w = t.LA16[row * (size_t)t.NW2 + (col >> 1)];
    return (int)((w >> ((col & 1) << 4)) & 0xFFFFu) - 1;
  }
  return t.LA[row * (size_t)t.N + col];
}
// firstDescendants[row][col] (row = chain * ccap + position; INF32 = none)
__device__ __forceinline__ int fd_at(const Tables& t, size_t row, int col) {
  if (t.FD16) {
    const uint32_t v = t.FD16[row * (size_t)t.N + col];
    return v == 0xFFFFu ? INF32 : (int)v - 1;
  }
  return t.FD[row * (size_t)t.N + col];
}
__device__ __forceinline__ int la_at(const Tables& t, int c, int p, int col) {
  return la_row(t, (size_t)c * t.ccap + p, col);
}

__global__ void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void k_iota(int32_t* p, int64_t n, int32_t base) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = base + (int32_t)i;
}

// lowest round among the candidate events (DecideRoundReceived starts above it)
__global__ void k_min_round(const int32_t* round, const int32_t* cand, int n, int32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int v = INF32;
  if (i < n) v = round[cand[i]];
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0 && v != INF32) atomicMin(out, v);
}

// k_min_round over the ids [lo, hi)
__global__ void k_min_round_range(const int32_t* round, int lo, int hi, int32_t* out) {
  const int i = lo + blockIdx.x * blockDim.x + threadIdx.x;
  int v = INF32;
  if (i < hi) v = round[i];
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  if ((threadIdx.x & 63) == 0 && v != INF32) atomicMin(out, v);
}

// exclusive scan of a small int array by one block (n <= ~64k): per-thread
// contiguous runs, a wave scan by shuffles and one scan of the 16 wave totals
// (two barriers; a Hillis-Steele over 1024 partials took 20)
// scat (non-null): also und[out[i]] = scat[i] for every i with in[i] != 0 (the
// undetermined list's compaction, k_scatter_und's work)
// n <= 16,384 (scan_large's case): the input is loaded coalesced into LDS (padded one
// word per 16: the per-thread runs read it without bank conflicts), each thread scans
// its contiguous run there, and the positions go back out coalesced.  (Runs loaded
// straight from HBM put 64 cache lines behind every load instruction: ~10 us at
// 10k entries.)  scat: flags in[] are 0 / 1 (the compaction's case).
constexpr int SCAN_LDS = 16384;
// sv: SCAN_LDS + SCAN_LDS / 16 ints of LDS (the caller's: k_order_call lends its sort pool)
__device__ __forceinline__ void scan_small_core(const int32_t* in, int32_t* out, int n, int32_t* total,
                                                const int32_t* scat, int32_t* und, int* sv) {
  __shared__ int wsum[16];
  const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (n + T - 1) / T;
  const int lo = min(n, tid * per), hi = min(n, lo + per);
  const bool lds = n <= SCAN_LDS && T == 1024;  // block-uniform
  auto P = [](int i) { return i + (i >> 4); };
  int s = 0;
  if (lds) {
    constexpr int K = SCAN_LDS / 1024;
    int rv[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = tid + 1024 * k;
      rv[k] = i < n ? in[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = tid + 1024 * k;
      if (i < n) sv[P(i)] = rv[k];
    }
    __syncthreads();
    for (int i = lo; i < hi; i++) s += sv[P(i)];
  } else {
    for (int i = lo; i < hi; i++) s += in[i];
  }
  int inc = s;  // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  if (wv == 0) {
    int v = lane < T / 64 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane < T / 64) wsum[lane] = v;  // inclusive totals of the waves
  }
  __syncthreads();
  int run = (wv > 0 ? wsum[wv - 1] : 0) + inc - s;
  const int tot = wsum[T / 64 - 1];
  if (lds) {
    for (int i = lo; i < hi; i++) {  // the run's exclusive positions, in place
      const int v = sv[P(i)];
      sv[P(i)] = run;
      run += v;
    }
    __syncthreads();
    constexpr int K = SCAN_LDS / 1024;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const int i = tid + 1024 * k;
      if (i < n) {
        const int o = sv[P(i)];
        out[i] = o;
        if (scat) {
          const int nx = i + 1 < n ? sv[P(i + 1)] : tot;
          if (nx != o) und[o] = scat[i];
        }
      }
    }
  } else {
    for (int i = lo; i < hi; i++) {
      const int v = in[i];
      out[i] = run;
      if (scat && v) und[run] = scat[i];
      run += v;
    }
  }
  if (tid == T - 1 && total) *total = tot;
}
__device__ __forceinline__ void scan_small_body(const int32_t* in, int32_t* out, int n, int32_t* total,
                                                const int32_t* scat, int32_t* und) {
  __shared__ int sv[SCAN_LDS + SCAN_LDS / 16];
  scan_small_core(in, out, n, total, scat, und, sv);
}
__global__ void __launch_bounds__(1024) k_scan_small(const int32_t* in, int32_t* out, int n, int32_t* total) {
  scan_small_body(in, out, n, total, nullptr, nullptr);
}

// multi-block exclusive scan: 1024 elements per 256-thread block
__global__ void __launch_bounds__(256) k_scan_blocks(const int32_t* in, int32_t* out, int n,
                                                     int32_t* partial) {
  __shared__ int ws[256];
  const int tid = threadIdx.x;
  const int base = blockIdx.x * 1024 + tid * 4;
  int v[4];
#pragma unroll
  for (int j = 0; j < 4; j++) v[j] = (base + j < n) ? in[base + j] : 0;
  const int s = v[0] + v[1] + v[2] + v[3];
  ws[tid] = s;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int add = (tid >= off) ? ws[tid - off] : 0;
    __syncthreads();
    ws[tid] += add;
    __syncthreads();
  }
  int run = ws[tid] - s;  // exclusive
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (tid == 255) partial[blockIdx.x] = ws[255];
}

__global__ void k_scan_add(int32_t* out, int n, const int32_t* partial_scanned) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += partial_scanned[i / 1024];
}

// A small batch's event fields uploaded as one packed record per event (one copy
// instead of eight; hge_engine.hip upload()), unpacked by k_chain_fill.
struct UpEv {
  int32_t creator, index, sp, op, ntx, coin;
  int64_t ts;
  uint64_t S[4];
};
struct UpDst {
  int32_t *creator, *index, *sp, *op, *ntx;
  int64_t* ts;
  uint64_t* S;
  uint8_t* coin;
};

// a batch's results header: out[0, n) = 0, out[3] = *lcr when given
__global__ void k_out_init(int32_t* out, int n, const int32_t* lcr) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (i == 3 && lcr) ? *lcr : 0;
}

// chain table: chain[c][index] = id for the new events.  up (non-null): the new
// events' fields arrive packed (record x - n0) and are unpacked into their tables
// here; an other-parent inside the batch is read from its record (its table entry
// is being written by another thread)
__device__ __forceinline__ void chain_fill_one(const Tables& t, int x, int n0, const UpEv* up, const UpDst& dst) {
  int cx, ix, o;
  int64_t ts;
  if (up) {
    const UpEv r = up[x - n0];
    cx = r.creator;
    ix = r.index;
    o = r.op;
    ts = r.ts;
    dst.creator[x] = cx;
    dst.index[x] = ix;
    dst.sp[x] = r.sp;
    dst.op[x] = o;
    dst.ntx[x] = r.ntx;
    dst.ts[x] = ts;
    dst.coin[x] = (uint8_t)r.coin;
#pragma unroll
    for (int k = 0; k < 4; k++) dst.S[4 * (size_t)x + k] = r.S[k];
  } else {
    cx = t.creator[x];
    ix = t.index[x];
    o = t.op[x];
    ts = t.ts[x];
  }
  const size_t at = (size_t)cx * t.ccap + ix;
  t.chain[at] = x;
  t.tsch[at] = ts;
  int2 oc = make_int2(-1, -1);
  if (o >= 0) {
    if (up && o >= n0) oc = make_int2(up[o - n0].creator, up[o - n0].index);
    else oc = make_int2(t.creator[o], t.index[o]);
  }
  t.opcp[at] = oc;
}

__global__ void k_chain_fill(Tables t, int n0, int n1, const UpEv* up, UpDst dst) {
  const int x = n0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (x < n1) chain_fill_one(t, x, n0, up, dst);
}

// HGE_STAMPS diagnostics: shader-clock stamp, ordered with the code around it
__device__ __forceinline__ uint64_t stamp() {
  uint64_t v;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
  return v;
}

// ---------------------------------------------------------------------------
// Rounds via first-strong-seer rows (the fast path).
// fss_c(w) = first position on chain c whose event strongly sees w
//          = SM-th smallest over i of FD[i][FD[w][i]][c]
// (x on chain c sees w's first descendant on chain i iff pos(x) >= that FD
// entry, and strongly seeing w is seeing >= SM of them).  Then, with C_r the
// round-r frontier (first position per chain with round >= r),
//   C_{r+1}[c] = SM-th smallest over d of fss_c(C_r[d]),
// the own-chain term clamped to C_r[c] + 1 (x never strongly sees itself;
// this only matters for N = 1).  DESIGN.md §Rounds proves both steps.
// ---------------------------------------------------------------------------
// k-th smallest (1-based, k <= NPC) of NPC register values: a fully unrolled
// bitonic network (constant indices keep everything in VGPRs), then a select
template <int NPC>
__device__ __forceinline__ int select_kth(int (&v)[NPC], int k) {
#pragma unroll
  for (int size = 2; size <= NPC; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int i = 0; i < NPC; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const int a = v[i], b = v[j];
          v[i] = up ? min(a, b) : max(a, b);
          v[j] = up ? max(a, b) : min(a, b);
        }
      }
    }
  }
  int r = v[0];
#pragma unroll
  for (int i = 1; i < NPC; i++) r = (i == k - 1) ? v[i] : r;
  return r;
}

// one lane per (event w, target chain c); events of chain cw from position lo[cw].
// Lane i of an event loads w's first descendant z_i on chain i and then the
// whole FD row of (i, z_i) with vector loads; an LDS transpose hands lane c the
// column c of those rows, FD[(i, z_i)][c] over i.
// FSS16 (non-null: the LDS walk) receives uint16 rows padded to NPC columns
// (INF and the padding = 0xFFFF) with the own-chain entry already clamped to
// pw + 1 (an event never strongly sees itself); otherwise int32 rows of N.
template <int NPC>
__global__ void __launch_bounds__(256) k_fss(Tables t, const int32_t* lo, const int32_t* off,
                                             int total_arg, int32_t* FSS, uint16_t* FSS16,
                                             const int32_t* total_dev) {
  constexpr int EPB = 256 / NPC;  // events per block and pass
  __shared__ int s_off[NPC + 1], s_lo[NPC];
  __shared__ int tr[EPB][NPC][NPC + 1];
  const int N = t.N;
  const int tid = threadIdx.x;
  // total_dev (non-null): the count written by k_frontier_start on the device (an
  // online call's walk; the grid loops over it, sized by the host without a readback)
  const int total = total_dev ? *total_dev : total_arg;
  if (tid <= N) s_off[tid] = off[tid];
  if (tid < N) s_lo[tid] = lo[tid];
  __syncthreads();
  const int e = tid / NPC, c = tid - (tid / NPC) * NPC;
  for (int b = blockIdx.x; b * EPB < total; b += gridDim.x) {
    const int ev = b * EPB + e;
    const bool valid = ev < total;
    int cw = 0;
    if (valid)
      while (s_off[cw + 1] <= ev) cw++;
    const int pw = valid ? s_lo[cw] + (ev - s_off[cw]) : 0;
    // row of (c, z_c): FD[(c, z_c)][0..N)
    const int z = (valid && c < N) ? t.FD[rowoff(t, cw, pw) + c] : INF32;
    int* row = tr[e][c];
    if (z == INF32) {
#pragma unroll
      for (int j = 0; j < NPC; j++) row[j] = INF32;
    } else {
      const int32_t* src = t.FD + rowoff(t, c, z);
      if (N == NPC) {
#pragma unroll
        for (int j = 0; j < NPC; j += 4) {
          const int4 q4 = *(const int4*)(src + j);
          row[j] = q4.x;
          row[j + 1] = q4.y;
          row[j + 2] = q4.z;
          row[j + 3] = q4.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < NPC; j++) row[j] = j < N ? src[j] : INF32;
      }
    }
    __syncthreads();
    if (valid) {
      int v[NPC];
#pragma unroll
      for (int i = 0; i < NPC; i++) v[i] = tr[e][i][c];
      int f = (c < N) ? select_kth<NPC>(v, t.SM) : INF32;
      if (FSS16) {
        if (c == cw && f != INF32) f = max(f, pw + 1);
        FSS16[((size_t)cw * t.ccap + pw) * NPC + c] = (f == INF32) ? 0xFFFF : (uint16_t)f;
      } else if (c < N) {
        FSS[rowoff(t, cw, pw) + c] = f;
      }
    }
    __syncthreads();  // tr is reused by the next pass
  }
}

// the sequential frontier walk: one wave, lane = chain
template <int NPC>
__global__ void __launch_bounds__(64) k_rounds_fss(Tables t, const int32_t* FSS,
                                                   const int32_t* olen, const int32_t* len,
                                                   int32_t* rstate, int rlo) {
  const int N = t.N, SM = t.SM;
  const int c = threadIdx.x;
  const bool act = c < N;
  const int ln = act ? len[c] : 0;
  const int ol = act ? olen[c] : 0;
  int P = act ? t.C[(size_t)rlo * N + c] : INF32;
  if (act && rlo == 0 && ol == 0 && ln > 0) {
    P = 0;
    t.C[c] = 0;
  }
  int r = rlo;
  for (;; r++) {
    if (r + 1 >= t.Rcap) {
      if (c == 0) rstate[1] = 1;
      return;
    }
    int v[NPC];
#pragma unroll
    for (int d = 0; d < NPC; d++) {
      const int Pd = __builtin_amdgcn_readlane(P, d);
      v[d] = INF32;
      if (d < N && act && Pd != INF32) v[d] = FSS[rowoff(t, d, Pd) + c];
    }
    const int cur = act ? t.C[(size_t)(r + 1) * N + c] : INF32;
    int nxt = INF32;
    if (act && P != INF32) {
#pragma unroll
      for (int d = 0; d < NPC; d++)
        if (d == c) v[d] = max(v[d], P + 1);
      const int sel = select_kth<NPC>(v, SM);
      nxt = cur != INF32 ? cur : (sel < ln ? sel : INF32);
      if (cur == INF32 && nxt != INF32) t.C[(size_t)(r + 1) * N + c] = nxt;
    }
    const uint64_t any = __ballot(act && nxt != INF32);
    P = nxt;
    if (!any) break;
  }
  if (c == 0) rstate[0] = max(rstate[0], r + 1);
}

// ---------------------------------------------------------------------------
// The frontier walk (C_{r+1}[c] = SM-th smallest over d of fss_c(C_r[d])).
// Every step depends on the previous one, so the walk is latency-bound and
// runs in ONE wave with no barriers: lane (c, q) = chain c, quarter q of the
// d range (LPC lanes per chain, VPL = NPC/LPC values per lane).  A step is
// one LDS read of the members' block rows, VPL LDS gathers of uint16 fss
// values (0xFFFF = none), an all-ascending bitonic network over the NPC values
// of each chain whose in-lane stages are register min/max and whose
// cross-lane stages are DPP quad permutes, and the owner lane's LDS stores.
// Global traffic is taken out of the step: all 16 waves stage blocks of uint16
// fss rows [P_d, P_d + B) of every chain into LDS (chain positions < 65535,
// checked by the host) together with the already-known C rows of the next RB
// rounds; the walk buffers its C rows in LDS and they are flushed at the next
// restage.  Row B of every chain's block is all 0xFFFF: an absent member
// (no frontier event) gathers from it, so a gather address is one shift-add of
// the member's block row.  The own-chain clamp (an event never strongly sees
// itself) is folded into the rows by k_fss.
// ---------------------------------------------------------------------------
// lane l reads lane l ^ X within its quad (X in 1..3): quad_perm DPP
template <int X>
__device__ __forceinline__ int dpp_flip(int v) {
  static_assert(X >= 1 && X <= 3, "quad permutes only");
  constexpr int ctrl = (0 ^ X) | ((1 ^ X) << 2) | ((2 ^ X) << 4) | ((3 ^ X) << 6);
  return __builtin_amdgcn_mov_dpp(v, ctrl, 0xF, 0xF, false);
}

// the same with the distance as a value (constant after unrolling)
__device__ __forceinline__ int dpp_flip(int x, int v) {
  return x == 1 ? dpp_flip<1>(v) : x == 2 ? dpp_flip<2>(v) : dpp_flip<3>(v);
}

// packed uint16 pairs (v_pk_min_u16 / v_pk_max_u16)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pmin(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t pmax(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t hswap(uint32_t a) { return __builtin_amdgcn_alignbit(a, a, 16); }
// (lo of a, hi of b)
__device__ __forceinline__ uint32_t lohi(uint32_t a, uint32_t b) {
  return (a & 0xFFFFu) | (b & 0xFFFF0000u);
}
// in-register compare-exchange of the two halves (lo gets the min)
__device__ __forceinline__ uint32_t cx_half(uint32_t r) {
  const uint32_t sw = hswap(r);
  return lohi(pmin(r, sw), pmax(r, sw));
}
// cross-lane stage: lower lanes keep the minima, upper lanes the maxima
__device__ __forceinline__ uint32_t cx_lane(bool lower, uint32_t a, uint32_t o) {
  return lower ? pmin(a, o) : pmax(a, o);
}

// All-ascending bitonic sort of the 16 values of one chain held by 4 lanes
// (lane quarter q, values e = 4q + k) as two packed registers R0 = (v0, v2),
// R1 = (v1, v3): stride-1 compare-exchanges are one packed min/max pair, the
// stride-2 ones exchange register halves.  Returns the value of element k.
__device__ __forceinline__ int net16_packed(uint32_t R0, uint32_t R1, int q, int k) {
  uint32_t a, b, o0, o1;
  // size 2 (flip k^1 = stride 1)
  a = pmin(R0, R1); b = pmax(R0, R1); R0 = a; R1 = b;
  // size 4: flip k^3 -> pairs (0,3), (1,2)
  {
    const uint32_t s1 = hswap(R1);
    const uint32_t mn = pmin(R0, s1), mx = pmax(R0, s1);
    R0 = lohi(mn, mx);
    R1 = __builtin_amdgcn_alignbit(mx, mn, 16);  // (mn.hi, mx.lo)
  }
  a = pmin(R0, R1); b = pmax(R0, R1); R0 = a; R1 = b;  // stride 1
  // size 8: flip across lanes q^1 (partner element e^7: its v[3-k])
  {
    const bool lower = (q & 1) == 0;
    o0 = hswap((uint32_t)dpp_flip<1>((int)R1));  // (p.v3, p.v1)
    o1 = hswap((uint32_t)dpp_flip<1>((int)R0));  // (p.v2, p.v0)
    R0 = cx_lane(lower, R0, o0);
    R1 = cx_lane(lower, R1, o1);
  }
  R0 = cx_half(R0); R1 = cx_half(R1);                   // stride 2
  a = pmin(R0, R1); b = pmax(R0, R1); R0 = a; R1 = b;  // stride 1
  // size 16: flip across lanes q^3
  {
    const bool lower = (q & 2) == 0;
    o0 = hswap((uint32_t)dpp_flip<3>((int)R1));
    o1 = hswap((uint32_t)dpp_flip<3>((int)R0));
    R0 = cx_lane(lower, R0, o0);
    R1 = cx_lane(lower, R1, o1);
  }
  // stride 4: across lanes q^1, same slot
  {
    const bool lower = (q & 1) == 0;
    o0 = (uint32_t)dpp_flip<1>((int)R0);
    o1 = (uint32_t)dpp_flip<1>((int)R1);
    R0 = cx_lane(lower, R0, o0);
    R1 = cx_lane(lower, R1, o1);
  }
  R0 = cx_half(R0); R1 = cx_half(R1);                   // stride 2
  a = pmin(R0, R1); b = pmax(R0, R1); R0 = a; R1 = b;  // stride 1
  const uint32_t r = (k & 1) ? R1 : R0;
  return (int)((k & 2) ? (r >> 16) : (r & 0xFFFFu));
}

template <int NPC, int LPC, int B>
__device__ __forceinline__ void rounds_walk_body(const Tables& t, const uint16_t* FSS,
                                                 const int32_t* olen, const int32_t* len,
                                                 int32_t* rstate, int rlo_arg, int Rprev,
                                                 uint64_t* dbg, const int32_t* rlo_dev) {
  // rlo_dev (non-null): the round to resume from, written by k_walk_join (-1: the
  // speculative walk completed and there is nothing left to walk)
  // (k_frontier_start's INF32: no new event needs a round; an online call reads
  // its first round this way, without a host round trip)
  const int rlo = rlo_dev ? *rlo_dev : rlo_arg;
  if (rlo < 0 || rlo == INF32) return;
  constexpr int VPL = NPC / LPC;
  constexpr int RB = 64;       // C rows buffered per restage
  constexpr int Q8 = NPC / 8;  // int4 loads per fss row
  constexpr int BR = B + 1;    // block rows per chain: B staged + the 0xFFFF row
  static_assert(NPC * LPC == 64, "one wave walks");
  uint64_t wst[4] = {0, 0, 0, 0}, wt = 0;  // HGE_STAMPS: restage cycles, walk cycles, restages, steps
  int pf = 0;                              // prefetch sink (kept live below)
  __shared__ __attribute__((aligned(16))) uint16_t blk[NPC * BR * NPC];  // [d][row][c]
  __shared__ __attribute__((aligned(16))) int sA[NPC];  // member block rows (B = absent)
  __shared__ int sP[NPC], sBase[NPC], sLen[NPC], sC[RB * NPC];
  __shared__ int s_r, s_done, s_nr;
  const int N = t.N, SM = t.SM;
  const int tid = threadIdx.x, T = blockDim.x;
  if (tid < NPC) {
    const int c = tid;
    int P = INF32, ln = 0;
    if (c < N) {
      ln = len[c];
      P = t.C[(size_t)rlo * N + c];
      if (rlo == 0 && olen[c] == 0 && ln > 0) {
        P = 0;
        t.C[c] = 0;
      }
    }
    sP[c] = P;
    sLen[c] = ln;
  }
  for (int i = tid; i < NPC * NPC; i += T) blk[((i / NPC) * BR + B) * NPC + (i % NPC)] = 0xFFFF;
  if (tid == 0) {
    s_r = rlo;
    s_done = 0;
  }
  __syncthreads();
  for (;;) {
    const int r0 = s_r;
    if (dbg && tid == 0) wt = stamp();
    // ---- restage: uint16 fss rows [P_d, P_d + B) of every chain, 8 values per
    //      int4; all loads of a thread are in flight before the first LDS store
    constexpr int ITEMS = NPC * B * Q8;
    constexpr int PER = (ITEMS + 1023) / 1024;  // launched with 1024 threads
    int4 vals[PER];
#pragma unroll
    for (int m = 0; m < PER; m++) {
      const int item = tid + m * 1024;
      const int d = item / (B * Q8);
      const int rem = item - d * (B * Q8);
      const int k = rem / Q8, q8 = rem - k * Q8;
      int4 w = make_int4(-1, -1, -1, -1);  // 0xFFFF x 8
      if (item < ITEMS && d < N && sP[d] != INF32 && sP[d] + k < sLen[d])
        w = *(const int4*)(FSS + ((size_t)d * t.ccap + sP[d] + k) * NPC + 8 * q8);
      vals[m] = w;
    }
#pragma unroll
    for (int m = 0; m < PER; m++) {
      const int item = tid + m * 1024;
      if (item >= ITEMS) break;
      const int d = item / (B * Q8);
      const int rem = item - d * (B * Q8);
      const int k = rem / Q8, q8 = rem - k * Q8;
      *(int4*)&blk[(d * BR + k) * NPC + 8 * q8] = vals[m];
    }
    // the next RB rounds' C rows as stored before this kernel (rows < Rprev)
    for (int item = tid; item < RB * NPC; item += T) {
      const int q = item / NPC, c = item - q * NPC;
      const int rr = r0 + 1 + q;
      sC[item] = (c < N && rr < Rprev && rr < t.Rcap) ? t.C[(size_t)rr * N + c] : INF32;
    }
    if (tid < NPC) {
      sBase[tid] = sP[tid];
      sA[tid] = sP[tid] == INF32 ? B : 0;
    }
    __syncthreads();
    if (dbg && tid == 0) {
      const uint64_t now = stamp();
      wst[0] += now - wt;
      wt = now;
      wst[2]++;
    }
    // ---- wave 0 walks from LDS only
    if (tid < 64) {
      const int lane = tid;
      const int c = lane / LPC, q = lane - (lane / LPC) * LPC;
      const bool act = c < N;
      const int ln = sLen[c];
      const int base_c = sBase[c];
      const int qo = (SM - 1) / VPL, ko = (SM - 1) - qo * VPL;
      const bool owner = act && q == qo;
      // byte offset of (member d = q*VPL + k, row 0, column c)
      int gb[VPL];
#pragma unroll
      for (int k = 0; k < VPL; k++) gb[k] = 2 * (((q * VPL + k) * BR) * NPC + c);
      int myP = sP[c];  // the owner's frontier position, kept in a register
      int r = r0;
      bool done = false;
      const int rcap1 = t.Rcap - 1;
      const int rend = min(r0 + RB, rcap1);  // C buffer full / rounds table full
      for (;;) {
        if (r >= rend) {
          if (r >= rcap1) {
            if (lane == 0) rstate[1] = 1;
            done = true;
          }
          break;
        }
        int Av[VPL], v[VPL];
#pragma unroll
        for (int k = 0; k < VPL; k++) Av[k] = sA[q * VPL + k];
        // the already-known C value of round r+1, read together with the members
        const int cur = sC[(r - r0) * NPC + c];
#pragma unroll
        for (int k = 0; k < VPL; k++)
          v[k] = *(const uint16_t*)((const char*)blk + gb[k] + Av[k] * (2 * NPC));
        // keep every gather in flight before the first comparator waits on one
        __builtin_amdgcn_sched_barrier(0);
        int sel;
        if constexpr (NPC == 16 && VPL == 4) {
          sel = net16_packed((uint32_t)v[0] | ((uint32_t)v[2] << 16),
                             (uint32_t)v[1] | ((uint32_t)v[3] << 16), q, ko);
        } else {
          // all-ascending bitonic network over the NPC values of chain c (LPC lanes
          // x VPL values): each merge starts with a flip (partner e ^ (size - 1))
          // followed by half-cleaners (partner e ^ stride), so every in-lane
          // comparator is static and a cross-lane one needs only the lane's
          // position in its pair
#pragma unroll
          for (int size = 2; size <= NPC; size <<= 1) {
            if (size <= VPL) {
#pragma unroll
              for (int k = 0; k < VPL; k++) {
                const int k2 = k ^ (size - 1);
                if (k2 > k) {
                  const int a = v[k], b = v[k2];
                  v[k] = min(a, b);
                  v[k2] = max(a, b);
                }
              }
            } else {
              const bool lower = (q & ((size >> 1) / VPL)) == 0;
              int o[VPL];
#pragma unroll
              for (int k = 0; k < VPL; k++) o[k] = dpp_flip(size / VPL - 1, v[VPL - 1 - k]);
#pragma unroll
              for (int k = 0; k < VPL; k++) v[k] = lower ? min(v[k], o[k]) : max(v[k], o[k]);
            }
#pragma unroll
            for (int stride = size >> 2; stride > 0; stride >>= 1) {
              if (stride < VPL) {
#pragma unroll
                for (int k = 0; k < VPL; k++) {
                  const int k2 = k ^ stride;
                  if (k2 > k) {
                    const int a = v[k], b = v[k2];
                    v[k] = min(a, b);
                    v[k2] = max(a, b);
                  }
                }
              } else {
                const bool lower = (q & (stride / VPL)) == 0;
#pragma unroll
                for (int k = 0; k < VPL; k++) {
                  const int o = dpp_flip(stride / VPL, v[k]);
                  v[k] = lower ? min(v[k], o) : max(v[k], o);
                }
              }
            }
          }
          sel = v[0];
#pragma unroll
          for (int k = 1; k < VPL; k++) sel = (k == ko) ? v[k] : sel;
        }
        // branch-free owner update: no LDS read between the network and the store
        // (ln < 0xFFFF, so sel < ln also rules out the 0xFFFF "none")
        const int cand = sel < ln ? sel : INF32;
        const int nxt = myP == INF32 ? INF32 : (cur != INF32 ? cur : cand);
        myP = nxt;
        const int rowA = nxt == INF32 ? B : nxt - base_c;  // B: the 0xFFFF row
        if (owner) {
          sP[c] = nxt;
          sA[c] = min(rowA, B);
          sC[(r - r0) * NPC + c] = nxt;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // stop when no chain has a frontier event left, or when one leaves its block
        const bool alive_l = owner && nxt != INF32;
        const uint64_t alive = __builtin_amdgcn_ballot_w64(alive_l);
        const uint64_t lv = __builtin_amdgcn_ballot_w64(alive_l && rowA >= B);
        if (alive == 0 || lv != 0) {
          if (alive == 0) done = true;
          else r++;
          break;
        }
        r++;
      }
      if (lane == 0) {
        s_nr = r - r0 + (done ? 1 : 0);  // C rows r0+1 .. r0+s_nr were produced
        s_r = r;
        s_done = done;
        if (done && !rstate[1]) rstate[0] = max(rstate[0], r + 1);
      }
    } else {
      // the other waves pull the rows after every block ([base + B, base + 2B))
      // into this XCD's L2 while wave 0 walks: the next block of a chain starts
      // inside its current one, so the next restage hits L2
      constexpr int RPL = 128 / (2 * NPC);  // fss rows per 128-byte line
      constexpr int LPCH = B / RPL;         // lines per chain block
      for (int item = tid - 64; item < NPC * LPCH; item += T - 64) {
        const int d = item / LPCH, k = (item - d * LPCH) * RPL;
        if (d < N && sBase[d] != INF32 && sBase[d] + B + k < sLen[d])
          pf ^= *(const int*)(FSS + ((size_t)d * t.ccap + sBase[d] + B + k) * NPC);
      }
    }
    __syncthreads();
    if (dbg && tid == 0) {
      const uint64_t now = stamp();
      wst[1] += now - wt;
      wt = now;
      wst[3] += s_nr;
    }
    // ---- flush the walked C rows (rows < Rprev are rewritten with their own values)
    const int nr = min(s_nr, RB);
    for (int item = tid; item < nr * NPC; item += T) {
      const int qq = item / NPC, c = item - qq * NPC;
      const int v = sC[item];
      if (c < N && v != INF32) t.C[(size_t)(r0 + 1 + qq) * N + c] = v;
    }
    const bool fin = s_done;
    __syncthreads();
    if (dbg && tid == 0) wst[0] += stamp() - wt;
    if (fin) break;
  }
  if (dbg && tid == 0)
    for (int q = 0; q < 4; q++) dbg[q] += wst[q];
  if (pf == 0x7fffffff && tid == 1 && rlo < 0) rstate[2] = pf;  // never true: keeps the prefetch
}

// frontier start: r_lo and the first position per chain that can be a member
// lo_off (non-null): the k_fss rows of the walk from r_lo, [0, N) the start
// positions, [N, 2N] their prefix offsets (the candidates' count last), written here
// so that an online call at N <= 32 needs no host round trip for them
// zbar / zgran (non-null): the wide rounds walk's hand-off flags and its 2 ngran
// granules, zeroed here in place of two memsets
__device__ __forceinline__ void frontier_start_body(const Tables& t, const int32_t* olen, const int32_t* len,
                                                    int32_t* out, int32_t* lo_off, int32_t* zbar,
                                                    uint64_t* zgran, int ngran) {
  if (zbar && threadIdx.x < 2) zbar[threadIdx.x] = 0;
  if (zgran)
    for (int i = threadIdx.x; i < ngran; i += blockDim.x) zgran[i] = 0;
  __shared__ int s_rlo;
  const int N = t.N;
  if (threadIdx.x == 0) s_rlo = INF32;
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    const int ol = olen[c], ln = len[c];
    if (ln > ol) atomicMin(&s_rlo, ol == 0 ? 0 : t.round[t.chain[(size_t)c * t.ccap + ol - 1]]);
  }
  __syncthreads();
  const int rlo = s_rlo;
  if (threadIdx.x == 0) out[0] = rlo;
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    int p = INF32;
    if (rlo != INF32) {
      p = t.C[(size_t)rlo * N + c];
      if (rlo == 0 && olen[c] == 0 && len[c] > 0) p = 0;
    }
    out[1 + c] = p == INF32 ? len[c] : p;
    if (lo_off) lo_off[c] = p == INF32 ? len[c] : p;
  }
  if (lo_off && threadIdx.x == 0) {
    int tot = 0;
    for (int c = 0; c < N; c++) {
      lo_off[N + c] = tot;
      if (rlo != INF32) {
        const int p = t.C[(size_t)rlo * N + c];
        const int s0 = (rlo == 0 && olen[c] == 0 && len[c] > 0) ? 0 : (p == INF32 ? len[c] : p);
        tot += max(0, len[c] - s0);
      }
    }
    lo_off[2 * N] = tot;
  }
}
__global__ void k_frontier_start(Tables t, const int32_t* olen, const int32_t* len,
                                 int32_t* out /* [0] rlo, [1..N] start positions */,
                                 int32_t* lo_off, int32_t* zbar, uint64_t* zgran, int ngran) {
  frontier_start_body(t, olen, len, out, lo_off, zbar, zgran, ngran);
}

// round(x) = max r with C[r][cx] <= px; witness iff C[round][cx] == px
// (consecutive events share a round: the per-round counts and the new-witness
// slots are aggregated per wave before touching global atomics)
// und_app (non-null: DivideRounds of an online call): the new ids are appended to the
// undetermined list there too (in place of a k_iota launch)
__device__ __forceinline__ void round_assign_item(const Tables& t, int x, int n0, int n1, const int32_t* rstate,
                                                  int32_t* newwit, int32_t* nnewwit, int32_t* und_app) {
  if (rstate[1]) return;  // the rounds table overflowed: the host grows it and walks again
  const int R = rstate[0];
  const bool valid = x < n1;
  if (und_app && valid) und_app[x - n0] = x;
  const int N = t.N;
  const int lane = threadIdx.x & 63;
  int lo = 0;
  bool w = false;
  if (valid) {
    const int cx = t.creator[x], px = t.index[x];
    int hi = R - 1;  // C[0][cx] == 0 <= px
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (t.C[(size_t)mid * N + cx] <= px) lo = mid;
      else hi = mid - 1;
    }
    t.round[x] = lo;
    w = (t.C[(size_t)lo * N + cx] == px);
    t.wit[x] = w ? 1 : 0;
    if (w) t.W[(size_t)lo * N + cx] = x;
  }
  uint64_t pending = __ballot(valid);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const int r = __shfl(lo, leader);
    const uint64_t same = __ballot(valid && lo == r);
    if (lane == leader) atomicAdd(&t.rcnt[r], __popcll(same));
    pending &= ~same;
  }
  const uint64_t wm = __ballot(w);
  if (wm) {
    const int leader = __builtin_ctzll(wm);
    int base = 0;
    if (lane == leader) base = atomicAdd(nnewwit, __popcll(wm));
    base = __shfl(base, leader);
    if (w) newwit[base + __popcll(wm & ((1ull << lane) - 1))] = x;
  }
}
__global__ void k_round_assign(Tables t, int n0, int n1, const int32_t* rstate, int32_t* newwit,
                               int32_t* nnewwit, int32_t* und_app) {
  round_assign_item(t, n0 + blockIdx.x * blockDim.x + threadIdx.x, n0, n1, rstate, newwit, nnewwit, und_app);
}
// k_round_assign's work appended to a single-block rounds walk (an online call at
// N <= 32: one launch less); n1 <= n0: none
struct RoundAssign {
  int n0, n1;
  int32_t* newwit;
  int32_t* nnewwit;
  int32_t* und_app;
  // minw (non-null): k_round_tail's work too -- the new witnesses' bitsets (groups of
  // G lanes), the first witness of rounds [r_from, R) (r_from < 0: the walk's first
  // round, rlo_dev[0]; the rows below it are unchanged since the last batch), the
  // round count, overflow flag and hand-off error (0), and the lowest round over
  // und[0, n_und) and the ids [lo, hi), final at minw[Rcap + 2]
  int32_t* minw;
  int G;
  const int32_t* und;
  int n_und, lo, hi, r_from;
  const int32_t* rlo_dev;
};

// The same from a fresh state, by frontier ranges: chain c's positions
// [C[r][c], C[r+1][c]) are exactly its round-r events (rounds never decrease
// along a chain) and the first of them is the witness.  One thread per
// (round, chain) over the Rcap rows (R from the device).
__global__ void k_round_ranges(Tables t, const int32_t* len, const int32_t* rstate,
                               int32_t* newwit, int32_t* nnewwit) {
  if (rstate[1]) return;
  const int R = rstate[0];
  const int N = t.N;
  const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int r = (int)(item / N), c = (int)(item - (item / N) * N);
  const int lane = threadIdx.x & 63;
  int lo = INF32, hi = 0;
  if (r < R) {
    lo = t.C[(size_t)r * N + c];
    hi = min(r + 1 < R ? t.C[(size_t)(r + 1) * N + c] : INF32, len[c]);
  }
  const bool any = lo != INF32 && lo < hi;
  int w = -1;
  if (any) {
    const int32_t* ch = t.chain + (size_t)c * t.ccap;
    for (int p = lo; p < hi; p++) {
      const int x = ch[p];
      t.round[x] = r;
      t.wit[x] = p == lo ? 1 : 0;
    }
    w = ch[lo];
    t.W[(size_t)r * N + c] = w;
  }
  // per-round counts: one atomic per distinct round in the wave
  {
    const int cnt = any ? hi - lo : 0;
    uint64_t pending = __ballot(cnt > 0);
    while (pending) {
      const int leader = __builtin_ctzll(pending);
      const int rl = __shfl(r, leader);
      const uint64_t same = __ballot(cnt > 0 && r == rl);
      int part = (cnt > 0 && r == rl) ? cnt : 0;
      for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
      if (lane == leader) atomicAdd(&t.rcnt[rl], part);
      pending &= ~same;
    }
  }
  const uint64_t wm = __ballot(any);
  if (wm) {
    const int leader = __builtin_ctzll(wm);
    int base = 0;
    if (lane == leader) base = atomicAdd(nnewwit, __popcll(wm));
    base = __shfl(base, leader);
    if (any) newwit[base + __popcll(wm & ((1ull << lane) - 1))] = w;
  }
}

// first witness id per round (monotone increasing in r); rounds [r0, R)
// minw[r] = the lowest witness id of round r: one wave per round, lanes over the
// creators (a thread per round looping over N creators was latency-bound: ~27 us
// per online call at N = 256)
// mr (an online call's candidates, few): the grid's last mr blocks also take the
// lowest round over und[0, n_und) and the ids [lo, hi), each over its slice, and
// store their partial minima at minw[Rcap+4+b] (the host folds them: in place of
// k_min_round / k_min_round_range; one block looping over ~10k gathers was ~15 us)
__device__ __forceinline__ void round_minw_body(const Tables& t, int r0, const int32_t* rstate, int32_t* minw,
                                                const int32_t* err_in, int mr, const int32_t* und, int n_und,
                                                int lo, int hi, int bid, int nblocks) {
  if (mr && bid >= nblocks - mr) {
    __shared__ int s_m;
    const int b = bid - (nblocks - mr);
    if (threadIdx.x == 0) s_m = INF32;
    __syncthreads();
    int m = INF32;
    const int tot = n_und + (hi - lo);
    constexpr int U = 8;
    for (int i0 = b * 256 * U + threadIdx.x; i0 < tot; i0 += mr * 256 * U) {
      int id[U];
#pragma unroll
      for (int k = 0; k < U; k++) {
        const int i = i0 + k * 256;
        id[k] = i < n_und ? und[min(i, n_und - 1)] : lo + (i - n_und);
      }
      int rv[U];
#pragma unroll
      for (int k = 0; k < U; k++) rv[k] = i0 + k * 256 < tot ? t.round[id[k]] : INF32;
#pragma unroll
      for (int k = 0; k < U; k++) m = min(m, rv[k]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMin(&s_m, m);
    __syncthreads();
    if (threadIdx.x == 0) minw[t.Rcap + 4 + b] = s_m;
    return;
  }
  const int r = r0 + bid * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  // the round count and overflow flag ride along at minw[Rcap..Rcap+1], the next
  // batch's lowest candidate round at [Rcap+2] (INF32 here when k_min_round* lower it
  // after this kernel) and the rounds walk's hand-off error flag at [Rcap+3]: one
  // readback for all of them
  if (bid == 0 && threadIdx.x == 0) {
    minw[t.Rcap] = rstate[0];
    minw[t.Rcap + 1] = rstate[1];
    minw[t.Rcap + 2] = INF32;
    minw[t.Rcap + 3] = err_in ? *err_in : 0;
  }
  if (rstate[1] || r >= rstate[0]) return;
  int m = INF32;
  for (int c = lane; c < t.N; c += 64) {
    const int w = t.W[(size_t)r * t.N + c];
    if (w >= 0) m = min(m, w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
  if (lane == 0) minw[r] = m;
}

// strongly-see / see bitsets of each new witness y (round j >= 1) over the
// slots of round j-1: StronglySee (hashgraph.go:189-208), See (:149-154)
// ssc (wide path): strongly-see bits already produced by k_rounds_coop.
// One group of G lanes (G = N rounded up to a power of two, at most 64) per
// (witness, 64-slot word): the group's ballots ARE the word, stored by its
// first lane (no global atomics: same-address atomics serialise at memory).
__device__ __forceinline__ void witness_bits_body(const Tables& t, const int32_t* newwit, const int32_t* pnnew,
                                                  const uint64_t* ssc, int G, int bid, int nblocks) {
  const int N = t.N, NW = t.NW;
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);
  const uint64_t gm = G == 64 ? ~0ull : ((1ull << G) - 1) << (lane & ~(G - 1));
  const int gshift = G == 64 ? 0 : (lane & ~(G - 1));
  // grid-stride over whole groups (the count lives on the device)
  const int64_t total = (int64_t)(*pnnew) * NW * G;
  for (int64_t item = (int64_t)bid * blockDim.x + threadIdx.x; item < total;
       item += (int64_t)nblocks * blockDim.x) {
    const int64_t grp = item / G;
    const int y = newwit[grp / NW];
    const int wd = (int)(grp - (grp / NW) * NW);
    const int d = wd * 64 + gl;
    const int j = t.round[y];
    const int cy = t.creator[y];
    bool see = false, ss = false;
    if (j > 0 && d < N) {
      const int w = t.W[(size_t)(j - 1) * N + d];
      if (w >= 0) {
        const size_t lrow = (size_t)cy * t.ccap + t.index[y];
        see = la_row(t, lrow, d) >= t.index[w];
        if (ssc) {
          ss = (ssc[((size_t)j * N + cy) * NW + wd] >> (d & 63)) & 1ull;
        } else {
          const size_t frow = (size_t)d * t.ccap + t.index[w];
          int c = 0;
          for (int i = 0; i < N; i++) c += (la_row(t, lrow, i) >= fd_at(t, frow, i)) ? 1 : 0;
          ss = c >= t.SM;
        }
      }
    }
    const uint64_t bsee = (__ballot(see) & gm) >> gshift;
    const uint64_t bss = (__ballot(ss) & gm) >> gshift;
    if (gl == 0 && j > 0) {
      const size_t off = ((size_t)j * N + cy) * NW + wd;
      t.seeb[off] = bsee;
      t.ssb[off] = bss;
    }
  }
}

// the rounds step's tail in one launch: blocks [0, nb_wb) k_witness_bits' work,
// the rest k_round_minw's (they are independent; one launch less per call)
__global__ void __launch_bounds__(256) k_round_tail(Tables t, const int32_t* newwit, const int32_t* pnnew,
                                                    const uint64_t* ssc, int G, int nb_wb, const int32_t* rstate,
                                                    int32_t* minw, const int32_t* err_in, int mr, const int32_t* und,
                                                    int n_und, int lo, int hi) {
  if ((int)blockIdx.x < nb_wb) witness_bits_body(t, newwit, pnnew, ssc, G, blockIdx.x, nb_wb);
  else round_minw_body(t, 0, rstate, minw, err_in, mr, und, n_und, lo, hi, blockIdx.x - nb_wb, gridDim.x - nb_wb);
}

template <int NPC, int LPC, int B>
__global__ void __launch_bounds__(1024) k_rounds_walk(Tables t, const uint16_t* FSS,
                                                      const int32_t* olen, const int32_t* len,
                                                      int32_t* rstate, int rlo_arg, int Rprev,
                                                      uint64_t* dbg, const int32_t* rlo_dev, RoundAssign ra) {
  rounds_walk_body<NPC, LPC, B>(t, FSS, olen, len, rstate, rlo_arg, Rprev, dbg, rlo_dev);
  if (ra.n1 > ra.n0) {
    __syncthreads();  // the walk's C rows and round count (global) are visible to the block
    for (int b = ra.n0; b < ra.n1; b += blockDim.x)
      round_assign_item(t, b + (int)threadIdx.x, ra.n0, ra.n1, rstate, ra.newwit, ra.nnewwit, ra.und_app);
  }
  if (!ra.minw) return;
  __shared__ int s_mr;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
  if (tid == 0) s_mr = INF32;
  __syncthreads();  // the new witnesses, their count and rounds
  witness_bits_body(t, ra.newwit, ra.nnewwit, nullptr, ra.G, 0, 1);
  const int R = rstate[0], ov = rstate[1];
  int32_t* minw = ra.minw;
  if (tid == 0) {
    minw[t.Rcap] = R;
    minw[t.Rcap + 1] = ov;
    minw[t.Rcap + 3] = 0;
  }
  if (!ov) {
    int r0 = ra.r_from >= 0 ? ra.r_from : *ra.rlo_dev;
    r0 = max(0, r0);
    for (int r = r0 + wv; r < R; r += nwv) {
      int m = INF32;
      for (int c = lane; c < t.N; c += 64) {
        const int w = t.W[(size_t)r * t.N + c];
        if (w >= 0) m = min(m, w);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
      if (lane == 0) minw[r] = m;
    }
  }
  int m = INF32;
  const int tot = ra.n_und + (ra.hi - ra.lo);
  for (int i = tid; i < tot; i += blockDim.x) m = min(m, t.round[i < ra.n_und ? ra.und[i] : ra.lo + (i - ra.n_und)]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
  if (lane == 0 && m != INF32) atomicMin(&s_mr, m);
  __syncthreads();
  if (tid == 0) minw[t.Rcap + 2] = s_mr;
}

// ---------------------------------------------------------------------------
// DecideFame (hashgraph.go:598-664) for one (round i, call c) pair and one
// witness slot x of round i: the votes of this call are rebuilt from scratch
// (hashgraph.go:599), y iterates in canonical (ascending creator) order, a
// decision breaks the y loop leaving later y without a vote (read as "no" at
// j+1), and the LAST decision over j is what SetFame leaves.  Output per
// (pair, slot): 0 no decision in this call, 1 famous, 2 not famous.
// ---------------------------------------------------------------------------
// (N % 64 == 0 takes k_fame_decide_blk below: one pair per block, rows in LDS.)
template <int NWT>
__device__ __forceinline__ void fame_decide_item(const Tables& t, int item, const int32_t* pr_round,
                                                 const int32_t* pr_off, const int32_t* pr_cf, int nrounds,
                                                 int p0, int npairs, const int64_t* nc, const int32_t* Rc,
                                                 uint8_t* dec) {
  const int N = t.N, SM = t.SM;
  if (item >= (npairs - p0) * N) return;
  int p = item / N;
  const int xd = item - p * N;
  p += p0;
  int lo = 0, hi = nrounds - 1;  // last round with pr_off <= p
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pr_off[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  const int i = pr_round[lo];
  const int c = pr_cf[lo] + (p - pr_off[lo]);
  const int64_t n = nc[c];
  const int R = Rc[c];
  uint8_t out = 0;
  const int x = t.W[(size_t)i * N + xd];
  // R <= i + 2: no round j in [i + 2, R) votes, so no decision (the See votes of
  // round i + 1 are not even read)
  if (x >= 0 && x < n && R > i + 2) {
    uint64_t votes[NWT], cur[NWT];
#pragma unroll
    for (int w = 0; w < NWT; w++) votes[w] = 0;
    // the witness rows are read in chunks of DC slots with every load of a chunk
    // in flight before the first use (the d loops are latency chains otherwise)
    constexpr int DC = 16;
    // diff == 1: vote = See(y, x)
    for (int d0 = 0; d0 < N; d0 += DC) {
      int ys[DC];
      uint64_t sb[DC];
#pragma unroll
      for (int u = 0; u < DC; u++) {
        const int d = d0 + u;
        ys[u] = d < N ? t.W[(size_t)(i + 1) * N + d] : -1;
        sb[u] = d < N ? t.seeb[((size_t)(i + 1) * N + d) * NWT + (xd >> 6)] : 0;
      }
#pragma unroll
      for (int u = 0; u < DC; u++) {
        const int d = d0 + u;
        if (ys[u] >= 0 && ys[u] < n && ((sb[u] >> (xd & 63)) & 1ull))
          votes[d >> 6] |= 1ull << (d & 63);
      }
    }
    for (int j = i + 2; j < R; j++) {
      const int diff = j - i;
      bool brk = false;  // DecideFame's break leaves the y loop of this j only
      const bool coinr = (diff % N) == 0;
#pragma unroll
      for (int w = 0; w < NWT; w++) cur[w] = 0;
      for (int d0 = 0; d0 < N && !brk; d0 += DC) {
        int ys[DC];
        uint64_t ss[DC][NWT];
#pragma unroll
        for (int u = 0; u < DC; u++) {
          const int d = d0 + u;
          ys[u] = d < N ? t.W[(size_t)j * N + d] : -1;
#pragma unroll
          for (int w = 0; w < NWT; w++) ss[u][w] = d < N ? t.ssb[((size_t)j * N + d) * NWT + w] : 0;
        }
#pragma unroll
        for (int u = 0; u < DC; u++) {
          const int d = d0 + u;
          const int y = ys[u];
          if (brk || y < 0 || y >= n) continue;
          int yays = 0, tot = 0;
#pragma unroll
          for (int w = 0; w < NWT; w++) {
            yays += __popcll(ss[u][w] & votes[w]);
            tot += __popcll(ss[u][w]);
          }
          const int nays = tot - yays;
          const bool v = yays >= nays;
          const int tt = v ? yays : nays;
          if (!coinr) {
            if (tt >= SM) {
              out = v ? 1 : 2;  // the last decision over j is what SetFame leaves
              brk = true;        // later y of this j cast no vote
              continue;
            }
            if (v) cur[d >> 6] |= 1ull << (d & 63);
          } else {
            const bool vv = (tt >= SM) ? v : (t.coin[y] != 0);
            if (vv) cur[d >> 6] |= 1ull << (d & 63);
          }
        }
      }
#pragma unroll
      for (int w = 0; w < NWT; w++) votes[w] = cur[w];
    }
  }
  dec[(size_t)p * N + xd] = out;
}
template <int NWT>
__global__ void k_fame_decide(Tables t, const int32_t* pr_round, const int32_t* pr_off,
                              const int32_t* pr_cf, int nrounds, int p0, int npairs,
                              const int64_t* nc, const int32_t* Rc, uint8_t* dec) {
  // pairs [p0, npairs): a part of a split replay decides the pairs of its rounds only
  // (pr_* then start at its first round; pair indices stay absolute)
  // (XCD-aware order: neighbouring pairs read the same rounds' witness rows)
  const int item = (int)xcd_block(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x;
  fame_decide_item<NWT>(t, item, pr_round, pr_off, pr_cf, nrounds, p0, npairs, nc, Rc, dec);
}

// k_fame_decide for N = 64 * NWT, one (round i, call c) pair per block of N
// threads (thread = witness slot x of round i): the rows every lane of the pair
// reads -- round j's witnesses W[j][.], their strongly-see bitsets ssb[j][.] and
// coins -- are staged in LDS once per j by one coalesced load of the block, and
// the y loop reads them as LDS broadcasts (the per-lane k_fame_decide reads them
// as chains of scalar loads, 8 slots at a time).  Same decisions, same output.
template <int NWT>
// plist (non-null): block b decides pair plist[b] (a widened window's new pairs only)
__global__ void __launch_bounds__(256) k_fame_decide_blk(Tables t, const int32_t* pr_round, const int32_t* pr_off,
                                                         const int32_t* pr_cf, int nrounds, int p0, int npairs,
                                                         const int64_t* nc, const int32_t* Rc, uint8_t* dec,
                                                         const int32_t* plist) {
  __shared__ int sY[64 * NWT];    // witness y of slot d, -1 if none or not yet inserted at call c
  __shared__ int sTot[64 * NWT];  // |ssb[y]|: the same for every lane
  __shared__ uint64_t sS[64 * NWT][NWT];
  __shared__ uint8_t sCoin[64 * NWT];
  const int N = t.N, SM = t.SM;
  const int p = plist ? plist[blockIdx.x] : p0 + (int)xcd_block(blockIdx.x, gridDim.x);  // (XCD-aware)
  if (p >= npairs) return;
  const int xd = threadIdx.x;
  int lo = 0, hi = nrounds - 1;  // last round with pr_off <= p
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pr_off[mid] <= p) lo = mid;
    else hi = mid - 1;
  }
  const int i = pr_round[lo];
  const int c = pr_cf[lo] + (p - pr_off[lo]);
  const int64_t n = nc[c];
  const int R = Rc[c];
  const int x = t.W[(size_t)i * N + xd];
  const bool act = x >= 0 && x < n;
  if (R <= i + 2) {  // no round j in [i + 2, R) votes: no decision (block-uniform)
    dec[(size_t)p * N + xd] = 0;
    return;
  }
  auto stage = [&](int j, const uint64_t* bits) {
    __syncthreads();  // every lane is done with the previous round's rows
    const int y = t.W[(size_t)j * N + xd];
    sY[xd] = (y >= 0 && y < n) ? y : -1;
    int tot = 0;
#pragma unroll
    for (int w = 0; w < NWT; w++) {
      const uint64_t b = bits[((size_t)j * N + xd) * NWT + w];
      sS[xd][w] = b;
      tot += __popcll(b);
    }
    sTot[xd] = tot;
    sCoin[xd] = y >= 0 ? t.coin[y] : 0;
    __syncthreads();
  };
  uint64_t votes[NWT], cur[NWT];
#pragma unroll
  for (int w = 0; w < NWT; w++) votes[w] = 0;
  // diff == 1: vote = See(y, x)
  stage(i + 1, t.seeb);
  if (act)
    for (int d = 0; d < N; d++) {
      if (sY[d] >= 0 && ((sS[d][xd >> 6] >> (xd & 63)) & 1ull)) votes[d >> 6] |= 1ull << (d & 63);
    }
  uint8_t out = 0;
  for (int j = i + 2; j < R; j++) {
    stage(j, t.ssb);
    if (!act) continue;
    const int diff = j - i;
    const bool coinr = (diff % N) == 0;
#pragma unroll
    for (int w = 0; w < NWT; w++) cur[w] = 0;
    for (int d = 0; d < N; d++) {
      if (sY[d] < 0) continue;
      int yays = 0;
#pragma unroll
      for (int w = 0; w < NWT; w++) yays += __popcll(sS[d][w] & votes[w]);
      const int nays = sTot[d] - yays;
      const bool v = yays >= nays;
      const int tt = v ? yays : nays;
      if (!coinr) {
        if (tt >= SM) {
          out = v ? 1 : 2;  // the last decision over j is what SetFame leaves
          break;            // later y of this j cast no vote
        }
        if (v) cur[d >> 6] |= 1ull << (d & 63);
      } else {
        const bool vv = (tt >= SM) ? v : (sCoin[d] != 0);
        if (vv) cur[d >> 6] |= 1ull << (d & 63);
      }
    }
#pragma unroll
    for (int w = 0; w < NWT; w++) votes[w] = cur[w];
  }
  dec[(size_t)p * N + xd] = act ? out : 0;
}

// LCR_c = max(LCR_start, prefix max of Lc); c_last(i) = first call with LCR >= i;
// coverage check of each round's speculative window.
// rfail (non-null): rfail[ri] = 1 when round ri's window ended before its decision
__device__ __forceinline__ void lcr_scan_body(const int32_t* Lc, int ncalls, int lcr_start, int32_t* LCR,
                                              const int32_t* pr_round, const int32_t* pr_cf,
                                              const int32_t* pr_len, int nrounds, int32_t* clast,
                                              int32_t* flags, int32_t* rfail = nullptr) {
  __shared__ int wm[16];
  const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (ncalls + T - 1) / T;
  const int lo = min(ncalls, tid * per), hi = min(ncalls, lo + per);
  int m = -1;
  for (int i = lo; i < hi; i++) m = max(m, Lc[i]);
  // exclusive max-scan over the threads' partial maxima: wave shuffles, then one
  // scan of the 16 wave maxima (two barriers; a Hillis-Steele over 1024 took twenty)
  int inc = m;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc = max(inc, y);
  }
  if (lane == 63) wm[wv] = inc;
  __syncthreads();
  if (wv == 0) {
    int v = lane < T / 64 ? wm[lane] : -1;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v = max(v, y);
    }
    if (lane < T / 64) wm[lane] = v;
  }
  __syncthreads();
  const int ex = __shfl_up(inc, 1, 64);  // the wave's prefix before this thread
  int run = max(lcr_start, max(wv > 0 ? wm[wv - 1] : -1, lane > 0 ? ex : -1));
  for (int i = lo; i < hi; i++) {
    run = max(run, Lc[i]);
    LCR[i] = run;
  }
  __syncthreads();
  if (tid == 0) {
    const int fin = LCR[ncalls - 1];
    flags[1] = fin;
    int a = 0, b = ncalls - 1;  // first call where LCR reached its final value
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (LCR[mid] >= fin) b = mid;
      else a = mid + 1;
    }
    flags[2] = a;
  }
  for (int ri = tid; ri < nrounds; ri += T) {
    const int i = pr_round[ri];
    int a = 0, b = ncalls;  // first c with LCR[c] >= i
    while (a < b) {
      const int mid = (a + b) >> 1;
      if (LCR[mid] >= i) b = mid;
      else a = mid + 1;
    }
    clast[ri] = a;
    const int ce = pr_cf[ri] + pr_len[ri] - 1;
    bool bad = false;
    if (pr_len[ri] > 0) bad = a < ncalls ? a > ce : ce < ncalls - 1;
    if (bad) atomicOr(&flags[0], 1);
    if (rfail) rfail[ri] = bad ? 1 : 0;
  }
}
__global__ void __launch_bounds__(1024) k_lcr_scan(const int32_t* Lc, int ncalls, int lcr_start,
                                                   int32_t* LCR, const int32_t* pr_round,
                                                   const int32_t* pr_cf, const int32_t* pr_len,
                                                   int nrounds, int32_t* clast, int32_t* flags,
                                                   int32_t* rfail) {
  lcr_scan_body(Lc, ncalls, lcr_start, LCR, pr_round, pr_cf, pr_len, nrounds, clast, flags, rfail);
}

// a widened DecideFame batch: every round's decisions of the previous layout
// (old_off / old_len pairs of N slots) copied to the start of its new range (new_off);
// the widened rounds' new pairs are then decided alone (k_fame_decide_blk's plist)
// (also L_c = -1 over the ncalls calls and the four flags zeroed: the pass's control
// block keeps them otherwise)
__global__ void __launch_bounds__(256) k_dec_relayout(const uint8_t* old_dec, uint8_t* new_dec, const int32_t* old_off,
                                                      const int32_t* old_len, const int32_t* new_off, int N,
                                                      int32_t* Lc, int ncalls, int32_t* flags) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ncalls; i += gridDim.x * blockDim.x) Lc[i] = -1;
  if (blockIdx.x == 0 && threadIdx.x < 4) flags[threadIdx.x] = 0;
  const int ri = blockIdx.x;
  const size_t n = (size_t)old_len[ri] * N;
  const uint8_t* src = old_dec + (size_t)old_off[ri] * N;
  uint8_t* dst = new_dec + (size_t)new_off[ri] * N;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// persisted fame after the batch: decisions up to c_last(i); one lane per
// (processed round, witness slot), coalesced over the slots
__device__ __forceinline__ void fame_persist_body(const Tables& t, const int32_t* pr_round, const int32_t* pr_off,
                                                  const int32_t* pr_cf, const int32_t* pr_len, int nrounds,
                                                  const int32_t* clast, const uint8_t* dec, int bid) {
  const int N = t.N;
  const int64_t item = (int64_t)bid * blockDim.x + threadIdx.x;
  const int ri = (int)(item / N), d = (int)(item - (item / N) * N);
  if (ri >= nrounds) return;
  const int i = pr_round[ri];
  const int qend = min(pr_len[ri], clast[ri] - pr_cf[ri] + 1);
  uint8_t f = t.fame[(size_t)i * N + d];
  for (int q = 0; q < qend; q++) {
    const uint8_t o = dec[(size_t)(pr_off[ri] + q) * N + d];
    if (o) f = o;
  }
  t.fame[(size_t)i * N + d] = f;
}
__global__ void k_fame_persist(Tables t, const int32_t* pr_round, const int32_t* pr_off, const int32_t* pr_cf,
                               const int32_t* pr_len, int nrounds, const int32_t* clast, const uint8_t* dec) {
  fame_persist_body(t, pr_round, pr_off, pr_cf, pr_len, nrounds, clast, dec, blockIdx.x);
}

// ---------------------------------------------------------------------------
// N <= 64: the per-round scans below run one G-lane group per round (lane =
// witness slot d, G = 16/32/64) instead of one thread per round, so the N-wide
// inner loops become one coalesced load and a masked ballot per step.
// ---------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ uint64_t group_mask(int lane) {
  return (G == 64) ? ~0ull : (((1ull << G) - 1) << (lane & ~(G - 1)));
}

template <int G>
__device__ __forceinline__ int group_min(int v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// k_fame_timeline with one group per processed round (G lanes; a lane holds
// SPL witness slots d + 64k when N > 64)
template <int G, int SPL>
__device__ __forceinline__ void fame_timeline_group(const Tables& t, int64_t gthread, const int32_t* pr_round,
                                                    const int32_t* pr_off, const int32_t* pr_cf,
                                                    const int32_t* pr_len, int nrounds, const int64_t* nc,
                                                    const uint8_t* dec, uint8_t* decbit, int32_t* Lc) {
  static_assert(SPL == 1 || G == 64, "several slots per lane need full-wave groups");
  const int N = t.N;
  const int lane = threadIdx.x & 63, d = lane & (G - 1);
  const int ri = (int)(gthread / G);
  const uint64_t gm = group_mask<G>(lane);
  const bool valid = ri < nrounds;  // uniform per group
  const int i = valid ? pr_round[ri] : 0;
  bool known[SPL];
  int x[SPL];
#pragma unroll
  for (int k = 0; k < SPL; k++) {
    const int sl = d + 64 * k;
    known[k] = false;
    x[k] = -1;
    if (valid && sl < N) {
      known[k] = t.fame[(size_t)i * N + sl] != 0;
      x[k] = t.W[(size_t)i * N + sl];
    }
  }
  const int len = valid ? pr_len[ri] : 0;
  const int poff = valid ? pr_off[ri] : 0, cf = valid ? pr_cf[ri] : 0;
  // the window's loads go out QC calls at a time before the sequential scan uses them
  constexpr int QC = 8;
  int64_t nq[QC];
  uint8_t oq[QC][SPL];
  for (int q = 0; q < len; q++) {
    const int u = q & (QC - 1);
    if (u == 0) {
#pragma unroll
      for (int kq = 0; kq < QC; kq++) {
        const bool in = q + kq < len;
        nq[kq] = in ? nc[cf + q + kq] : 0;
#pragma unroll
        for (int k = 0; k < SPL; k++) {
          const int sl = d + 64 * k;
          oq[kq][k] = (in && sl < N) ? dec[(size_t)(poff + q + kq) * N + sl] : 0;
        }
      }
    }
    const int p = poff + q, c = cf + q;
    int64_t n = nq[0];
#pragma unroll
    for (int kq = 1; kq < QC; kq++) n = (u == kq) ? nq[kq] : n;
    uint64_t und = 0;
#pragma unroll
    for (int k = 0; k < SPL; k++) {
      uint8_t o = oq[0][k];
#pragma unroll
      for (int kq = 1; kq < QC; kq++) o = (u == kq) ? oq[kq][k] : o;
      if (o) known[k] = true;
      und |= __ballot(x[k] >= 0 && x[k] < n && !known[k]) & gm;
    }
    if (d == 0) {
      decbit[p] = und == 0 ? 1 : 0;
      if (und == 0) atomicMax(&Lc[c], i);
    }
  }
}
template <int G, int SPL>
__global__ void __launch_bounds__(256) k_fame_timeline_g(Tables t, const int32_t* pr_round,
                                                         const int32_t* pr_off, const int32_t* pr_cf,
                                                         const int32_t* pr_len, int nrounds,
                                                         const int64_t* nc, const uint8_t* dec,
                                                         uint8_t* decbit, int32_t* Lc) {
  fame_timeline_group<G, SPL>(t, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, pr_round, pr_off, pr_cf, pr_len,
                              nrounds, nc, dec, decbit, Lc);
}

// An online call's DecideFame at N < 64 in ONE launch (in place of k_fame_decide,
// k_fame_timeline_g and k_lcr_scan, plus k_out_init's results header): one block of
// 1024 threads, the three stages behind block barriers (their grids were one or two
// blocks each for a single call).  out (non-null): the header zeroed with the new
// LastConsensusRound at out[3].
// DECIDE false (N >= 64, where k_fame_decide_blk decides the pairs with a block per
// pair): the timeline, LCR and header only.
struct FameCall {
  const int32_t *pr_round, *pr_off, *pr_cf, *pr_len;
  int nrounds, npairs;
  const int64_t* nc;
  const int32_t* Rc;
  uint8_t *dec, *decbit;
  int32_t* Lc;
  int ncalls, lcr_start;
  int32_t *LCR, *clast, *flags, *out;
  int nout;
};
template <int G, int SPL, bool DECIDE>
__device__ __forceinline__ void fame_call_body(const Tables& t, const FameCall& f) {
  const int32_t *pr_round = f.pr_round, *pr_off = f.pr_off, *pr_cf = f.pr_cf, *pr_len = f.pr_len;
  const int nrounds = f.nrounds, npairs = f.npairs, ncalls = f.ncalls, lcr_start = f.lcr_start, nout = f.nout;
  const int64_t* nc = f.nc;
  const int32_t* Rc = f.Rc;
  uint8_t *dec = f.dec, *decbit = f.decbit;
  int32_t *Lc = f.Lc, *LCR = f.LCR, *clast = f.clast, *flags = f.flags, *out = f.out;
  const int tid = threadIdx.x;
  if (DECIDE) {
    for (int it = tid; it < npairs * t.N; it += blockDim.x)
      fame_decide_item<1>(t, it, pr_round, pr_off, pr_cf, nrounds, 0, npairs, nc, Rc, dec);
    __syncthreads();  // the decisions (global) are visible to the block
  }
  for (int64_t b = 0; b < (int64_t)nrounds * G; b += blockDim.x)
    fame_timeline_group<G, SPL>(t, b + tid, pr_round, pr_off, pr_cf, pr_len, nrounds, nc, dec, decbit, Lc);
  __syncthreads();
  lcr_scan_body(Lc, ncalls, lcr_start, LCR, pr_round, pr_cf, pr_len, nrounds, clast, flags);
  if (out) {
    __syncthreads();
    for (int i = tid; i < nout; i += blockDim.x) out[i] = i == 3 ? flags[1] : 0;
  }
}
template <int G, int SPL, bool DECIDE>
__global__ void __launch_bounds__(1024) k_fame_call(Tables t, FameCall f) {
  fame_call_body<G, SPL, DECIDE>(t, f);
}

// ---------------------------------------------------------------------------
// Round-state segments for DecideRoundReceived (hashgraph.go:676-721): for each
// round i, the calls at which (WitnessesDecided, famous set) changes.  State
// changes only when a witness of round i becomes visible (its call of arrival)
// or, while the round is processed by DecideFame, when a decision lands.
// ---------------------------------------------------------------------------
struct SegInfo {
  const int32_t* pr_index;  // [rounds rr_lo..] -> index into pr_* arrays or -1
  const int32_t* pr_off;
  const int32_t* pr_cf;
  const int32_t* pr_len;
  const int32_t* clast;
  const uint8_t* dec;
};

// first call of the batch at which witness W[r][d] is visible (INF32: none / later)
// vis[x] = first call whose event count exceeds x (ncalls: none; the readers take
// a null table as 0 everywhere: one call that sees every event), for the
// events [0, nev): a block takes 256 consecutive events and binary-searches
// them in an LDS window of the calls from the first one that sees its first
// event (the global search is the fallback past the window)
// out (non-null): the blocks past the events' also zero the results header
// out[0, nout) with out[3] = *lcr when given (k_out_init's work, one launch less)
__global__ void __launch_bounds__(256) k_visibility(const int64_t* nc, int ncalls, int nev,
                                                    int32_t* vis, int32_t* out, int nout, const int32_t* lcr) {
  __shared__ int64_t s_nc[256];
  __shared__ int s_c0;
  const int tid = threadIdx.x;
  const int nvb = (nev + 255) >> 8;
  if ((int)blockIdx.x >= nvb) {
    const int i = ((int)blockIdx.x - nvb) * 256 + tid;
    if (i < nout) out[i] = (i == 3 && lcr) ? *lcr : 0;
    return;
  }
  const int x0 = blockIdx.x * 256;
  auto upper = [&](int64_t x, int lo, int hi) {
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (nc[mid] > x) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  if (tid == 0) s_c0 = upper(x0, 0, ncalls);
  __syncthreads();
  const int c0 = s_c0;
  s_nc[tid] = c0 + tid < ncalls ? nc[c0 + tid] : INT64_MAX;
  __syncthreads();
  const int x = x0 + tid;
  if (x >= nev) return;
  int lo = 0, hi = 256;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (s_nc[mid] > x) hi = mid;
    else lo = mid + 1;
  }
  vis[x] = lo < 256 ? min(c0 + lo, ncalls) : upper(x, c0 + 256, ncalls);
}

// One group per round (G lanes, SPL witness slots per lane when N > 64): the
// witness arrivals come from the visibility table, the segments of round q are
// written straight into [segoff[q], segoff[q+1]) (a per-round capacity the host
// sized from the bound N + 2 + processed fame calls), and for N <= 64 each
// segment's theta row is computed by the same group as it is found (lane =
// witness slot, then = creator); wider hashgraphs take k_seg_theta_wide.
template <int G, int SPL>
__device__ __forceinline__ void segments_group(const Tables& t, int64_t gthread, int rr_lo, int nr, int ncalls,
                                               const int32_t* vis, const SegInfo& si, const int32_t* segoff,
                                               int32_t* segcnt, int32_t* seg_call, int32_t* seg_round,
                                               uint8_t* seg_dec, uint64_t* seg_fws, int32_t* theta) {
  static_assert(SPL == 1 || G == 64, "several slots per lane need full-wave groups");
  const int N = t.N;
  const int lane = threadIdx.x & 63, d = lane & (G - 1);
  const int qi = (int)(gthread / G);
  const uint64_t gm = group_mask<G>(lane);
  const int gshift = (G == 64) ? 0 : (lane & ~(G - 1));
  const bool valid = qi < nr;  // uniform per group
  const int i = rr_lo + (valid ? qi : 0);
  int a[SPL];
  bool known[SPL], val[SPL], slot[SPL];
  int row = -1;  // chain-major lastAncestors row of witness d (theta, SPL == 1)
#pragma unroll
  for (int k = 0; k < SPL; k++) {
    const int sl = d + 64 * k;
    slot[k] = valid && sl < N;
    a[k] = INF32;
    known[k] = val[k] = false;
    if (slot[k]) {
      const int x = t.W[(size_t)i * N + sl];
      if (x >= 0) {
        const int vx = vis ? vis[x] : 0;  // null: one call that sees every event
        if (vx < ncalls) a[k] = vx;
      }
      if (SPL == 1 && x >= 0) row = sl * t.ccap + t.index[x];
      const uint8_t f = t.fame[(size_t)i * N + sl];  // persisted BEFORE this batch's update
      known[k] = f != 0;
      val[k] = f == 1;
    }
  }
  const int pi = valid ? si.pr_index[qi] : -1;
  const int cf = pi >= 0 ? si.pr_cf[pi] : INF32;
  const int wl = pi >= 0 ? min(si.pr_len[pi], si.clast[pi] - cf + 1) : 0;  // processed calls
  const int poff = pi >= 0 ? si.pr_off[pi] : 0;
  int prevdec = -1, nseg = 0;
  uint64_t prevf[SPL];
#pragma unroll
  for (int k = 0; k < SPL; k++) prevf[k] = 0;
  const int base = valid ? segoff[qi] : 0;
  int c = valid ? 0 : INF32;
  while (c < ncalls) {
    int mn = INF32;
#pragma unroll
    for (int k = 0; k < SPL; k++) mn = min(mn, (slot[k] && a[k] > c) ? a[k] : INF32);
    int nxt = group_min<G>(mn);
    uint64_t bp = 0, und = 0, fws[SPL];
    bool same = true;
#pragma unroll
    for (int k = 0; k < SPL; k++) {
      const bool pres = slot[k] && a[k] <= c;
      if (c >= cf && c - cf < wl && slot[k]) {
        const uint8_t o = si.dec[(size_t)(poff + (c - cf)) * N + d + 64 * k];
        if (o) {
          known[k] = true;
          val[k] = (o == 1);
        }
      }
      bp |= __ballot(pres) & gm;
      und |= __ballot(pres && !known[k]) & gm;
      fws[k] = (__ballot(pres && known[k] && val[k]) & gm) >> gshift;
      same = same && fws[k] == prevf[k];
    }
    const bool decided = und == 0;
    if (bp && (prevdec != (int)decided || !same)) {
      const int sidx = base + nseg;
      if (d == 0) {
        seg_call[sidx] = c;
        seg_round[sidx] = i;
        seg_dec[sidx] = decided ? 1 : 0;
#pragma unroll
        for (int k = 0; k < SPL; k++) seg_fws[(size_t)sidx * SPL + k] = fws[k];
      }
      if (SPL == 1) {
        // theta of the segment, lane = creator cx: the (|fws|/2 + 1)-th largest
        // LA[w][cx] over its famous witnesses w (INT_MIN pads sort lowest)
        const int cx = d;
        int v[G];
#pragma unroll
        for (int dd = 0; dd < G; dd++) {
          const int rd = __shfl(row, gshift + dd);
          v[dd] = (((fws[0] >> dd) & 1ull) && cx < N) ? la_row(t, (size_t)rd, cx) : (int)0x80000000;
        }
        const int nf = __popcll(fws[0]);
        const int th = nf ? select_kth<G>(v, G - (nf / 2 + 1) + 1) : (int)0x80000000;
        if (cx < N) theta[(size_t)sidx * N + cx] = th;
      }
      nseg++;
      prevdec = decided;
#pragma unroll
      for (int k = 0; k < SPL; k++) prevf[k] = fws[k];
    }
    // next change point: an arrival, or the next call DecideFame processes round i
    if (c + 1 >= cf && c + 1 - cf < wl) nxt = min(nxt, c + 1);
    else if (c + 1 < cf && wl > 0) nxt = min(nxt, cf);
    if (nxt <= c) nxt = c + 1;
    c = nxt;
  }
  if (valid && d == 0) segcnt[qi] = nseg;
}
template <int G, int SPL>
__global__ void __launch_bounds__(256) k_segments_1p(Tables t, int rr_lo, int nr, int ncalls,
                                                     const int32_t* vis, SegInfo si,
                                                     const int32_t* segoff, int32_t* segcnt,
                                                     int32_t* seg_call, int32_t* seg_round,
                                                     uint8_t* seg_dec, uint64_t* seg_fws,
                                                     int32_t* theta) {
  segments_group<G, SPL>(t, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, rr_lo, nr, ncalls, vis, si, segoff,
                         segcnt, seg_call, seg_round, seg_dec, seg_fws, theta);
}

// theta for N > 64: one 256-thread block per (round, segment stride), thread =
// creator cx.  The famous witnesses' lastAncestors values of column cx (from WLA,
// which k_witness_la has written for the batch's rounds before this kernel) are
// staged in LDS as uint16 (position + 1; chains are < 65535 long on the wide path),
// then each thread bisects the value domain of its column for the (|fws|/2 + 1)-th
// largest.
template <int NWT>
__global__ void __launch_bounds__(1024) k_seg_theta_wide(Tables t, const int32_t* seg_round,
                                                         const int32_t* segoff, const int32_t* segcnt,
                                                         int nr, const uint64_t* seg_fws,
                                                         int32_t* theta, uint64_t* dbg) {
  // [famous k / 8][cx]: 8 values of a column per 16 bytes, as uint16 pairs
  __shared__ uint4 sv[32][256];
  __shared__ int s_row[256];
  __shared__ int s_nf;
  __shared__ int s_vmin[256], s_vmax[256];
  const int N = t.N;
  const int tid = threadIdx.x;
  // blocks (x, y): rounds x, x + gridDim.x, ... (grid-stride) and, of each round's
  // segments [segoff[q], segoff[q] + segcnt[q]), those l = y, y + gridDim.y, ...
  // (an online call decides a few rounds of a few segments each: one block per
  // round left them serial, ~90 us per call at N = 256)
  for (int q = blockIdx.x; q < nr; q += gridDim.x) {
    const int cnt = segcnt[q];
    for (int l = blockIdx.y; l < cnt; l += gridDim.y) {
      // HGE_STAMPS diagnostics (block (0, 0), thread 0): cycles of the row list,
      // the staging and the bisection into dbg[12..14], segments into dbg[15]
      const bool stmp = dbg && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0;
      uint64_t ts0 = stmp ? __builtin_amdgcn_s_memtime() : 0, ts1 = 0, ts2 = 0;
      const int sg = segoff[q] + l;
      const int i = seg_round[sg];
      // the famous witnesses' rows, in ascending creator order: thread d places
      // its own at its rank (a serial walk here was a chain of dependent loads)
      if (tid < 256) {
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
          s_row[rank] = d;  // the famous witness of chain d: its row is WLR[i][d][.]
        }
        if (tid == 0) s_nf = nfw;
        s_vmin[tid] = 65535;
        s_vmax[tid] = 0;
      }
      __syncthreads();
      if (stmp) ts1 = __builtin_amdgcn_s_memtime();
      const int nf = s_nf, ng = (nf + 7) >> 3;
      // staging (thread = column cx, quarter pa of the 8-row groups g = pa + 4 u): the
      // famous witnesses' LA + 1 values of column cx from WLR[i][d][cx], the round's
      // frontier rows written row-major by k_witness_la (the witness of round i on
      // chain d sits at C[i][d]); a wave reads 64 consecutive columns of one row, and
      // a thread's loads go out 32 at a time.  (Round 3 gathered the
      // witnesses' own LA16 rows, one page each: ~160k cycles per segment of
      // dependent latencies at N = 256, 80 us per online call.)
      {
        const int cx = tid & 255, pa = tid >> 8;
        if (cx < N) {
          const uint16_t* wr = t.WLR + (size_t)i * N * N + cx;
          int vmin = 65535, vmax = 0;
#pragma unroll 1
          for (int hb = 0; hb < 2; hb++) {  // two batches of 32 loads in flight (registers)
            if (8 * (pa + 16 * hb) >= nf) break;
            uint32_t v[32];
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
              for (int e = 0; e < 8; e++) {
                const int k = 8 * (pa + 4 * (u + 4 * hb)) + e;
                v[8 * u + e] = wr[(size_t)s_row[k < nf ? k : 0] * N];
              }
#pragma unroll
            for (int u = 0; u < 4; u++) {
              const int g = pa + 4 * (u + 4 * hb);
              if (g < ng) {
                uint32_t w[4];
#pragma unroll
                for (int e = 0; e < 8; e += 2) {
                  const int k = 8 * g + e;
                  const int a = k < nf ? (int)v[8 * u + e] : -1;
                  const int b = k + 1 < nf ? (int)v[8 * u + e + 1] : -1;
                  if (a >= 0) { vmin = min(vmin, a); vmax = max(vmax, a); }
                  if (b >= 0) { vmin = min(vmin, b); vmax = max(vmax, b); }
                  w[e >> 1] = (uint32_t)max(a, 0) | ((uint32_t)max(b, 0) << 16);
                }
                sv[g][cx] = make_uint4(w[0], w[1], w[2], w[3]);
              }
            }
          }
          if (nf > 0) {
            atomicMin(&s_vmin[cx], vmin);
            atomicMax(&s_vmax[cx], vmax);
          }
        }
      }
      __syncthreads();
      if (stmp) ts2 = __builtin_amdgcn_s_memtime();
      // bisection (thread = column cx = tid / 4, quarter pb = tid % 4 of the groups,
      // a quad per column: the counts are summed by two DPP quad permutes).  The
      // column's values span a few dozen positions (the famous witnesses of one round
      // see chain cx up to about the same point): bisect [min, max], not [0, 65535].
      // Values are LA + 1 (0: no ancestor on chain cx), never counted for mid >= 1.
      {
        const int cx = tid >> 2, pb = tid & 3;
        int th = (int)0x80000000;
        if (nf > 0 && cx < N) {
          const int kk = nf / 2 + 1;  // k-th largest = largest v with count(>= v) >= kk
          int lo = s_vmin[cx], hi = s_vmax[cx];
          while (lo < hi) {  // quad-uniform (one column)
            const int mid = (lo + hi + 1) >> 1;
            // v >= mid <=> v -sat (mid - 1) != 0: packed saturating subtract, min 1, add
            const uint32_t m1 = (uint32_t)(mid - 1) * 0x00010001u, one = 0x00010001u;
            uint32_t acc0 = 0, acc1 = 0;
            for (int g = pb; g < ng; g += 4) {
              const uint4 x = sv[g][cx];
              uint32_t d0, d1, d2, d3;
              asm("v_pk_sub_u16 %0, %6, %10 clamp\n\t"
                  "v_pk_sub_u16 %1, %7, %10 clamp\n\t"
                  "v_pk_sub_u16 %2, %8, %10 clamp\n\t"
                  "v_pk_sub_u16 %3, %9, %10 clamp\n\t"
                  "v_pk_min_u16 %0, %0, %11\n\t"
                  "v_pk_min_u16 %1, %1, %11\n\t"
                  "v_pk_min_u16 %2, %2, %11\n\t"
                  "v_pk_min_u16 %3, %3, %11\n\t"
                  "v_pk_add_u16 %4, %4, %0\n\t"
                  "v_pk_add_u16 %5, %5, %1\n\t"
                  "v_pk_add_u16 %4, %4, %2\n\t"
                  "v_pk_add_u16 %5, %5, %3"
                  : "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "+v"(acc0), "+v"(acc1)
                  : "v"(x.x), "v"(x.y), "v"(x.z), "v"(x.w), "v"(m1), "v"(one));
            }
            int c2 = (int)(acc0 & 0xFFFFu) + (int)(acc0 >> 16) + (int)(acc1 & 0xFFFFu) + (int)(acc1 >> 16);
            c2 += __builtin_amdgcn_mov_dpp(c2, 0xB1, 0xF, 0xF, false);  // quad_perm xor 1
            c2 += __builtin_amdgcn_mov_dpp(c2, 0x4E, 0xF, 0xF, false);  // quad_perm xor 2
            if (c2 >= kk) lo = mid;
            else hi = mid - 1;
          }
          th = lo - 1;
        }
        if (cx < N && pb == 0) theta[(size_t)sg * N + cx] = th;
      }
      if (stmp) {
        const uint64_t ts3 = __builtin_amdgcn_s_memtime();
        dbg[12] += ts1 - ts0;
        dbg[13] += ts2 - ts1;
        dbg[14] += ts3 - ts2;
        dbg[15] += 1;
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------
// DecideRoundReceived + MedianTimestamp (hashgraph.go:676-721, 762-770) for
// every candidate event (undetermined at batch start, or new): the first call
// c >= arrival(x) and, within it, the lowest round i > round(x) that is decided
// at c and whose famous witnesses see x by strict majority.
// ---------------------------------------------------------------------------
template <int NWT>
__device__ __forceinline__ void round_received_item(const Tables& t, int q, const int32_t* cand, int ncand,
                                                    const int32_t* vis, int ncalls, int call_lo, int rr_lo,
                                                    int R_last, const int32_t* segoff, const int32_t* segcnt,
                                                    const int32_t* seg_call, const uint8_t* seg_dec,
                                                    const uint64_t* seg_fws, const int32_t* theta,
                                                    int32_t* recv_call, int32_t* rr_out, int64_t* cts_out,
                                                    int32_t* bseg_out) {
  if (q >= ncand) return;
  const int N = t.N;
  const int x = cand[q];
  const int cx = t.creator[x], ix = t.index[x];
  const int rx = t.round[x];
  // first call at which x is visible
  const int c0 = max(call_lo, vis ? vis[x] : 0);  // null: one call that sees every event
  int best = INF32, rr = -1, bseg = -1;
  for (int i = rx + 1; i < R_last; i++) {
    const int qi = i - rr_lo;
    const int so = segoff[qi], sc = segcnt[qi];
    if (sc == 0) continue;
    if (seg_call[so] >= best) break;
    for (int k = 0; k < sc; k++) {
      const int sstart = seg_call[so + k];
      const int send = (k + 1 < sc) ? seg_call[so + k + 1] : ncalls;
      if (send <= c0) continue;
      if (sstart >= best) break;
      if (seg_dec[so + k] && ix <= theta[(size_t)(so + k) * N + cx]) {
        const int f = max(sstart, c0);
        if (f < best) {
          best = f;
          rr = i;
          bseg = so + k;
        }
        break;
      }
    }
  }
  if (rr < 0 || best >= ncalls) {
    recv_call[q] = -1;
    return;
  }
  if (bseg_out) {  // wide: the median is taken by k_median_wave
    recv_call[q] = best;
    rr_out[q] = rr;
    bseg_out[q] = bseg;
    return;
  }
  // median of the oldest-self-ancestor-to-see timestamps (OSA(w,x) = FD[x][cw]),
  // N <= 16 (wider hashgraphs take k_median_wave): every gather of a level is
  // issued before the next level needs it, then an int64 register sort
  constexpr int M = 16;
  const uint64_t fw = seg_fws[(size_t)bseg * NWT];
  const int32_t* fdx = t.FD + rowoff(t, cx, ix);
  int wid[M], wix[M], fd[M];
#pragma unroll
  for (int d = 0; d < M; d++) {
    const bool fam = d < N && ((fw >> d) & 1ull);
    wid[d] = fam ? t.W[(size_t)rr * N + d] : -1;
    fd[d] = d < N ? fdx[d] : 0;
  }
#pragma unroll
  for (int d = 0; d < M; d++) wix[d] = wid[d] >= 0 ? t.index[wid[d]] : 0;
  int osa[M];
#pragma unroll
  for (int d = 0; d < M; d++) {
    const bool seen = wid[d] >= 0 && la_at(t, d, wix[d], cx) >= ix;
    osa[d] = seen ? t.chain[(size_t)d * t.ccap + fd[d]] : -1;
  }
  int64_t tv[M];
  int m = 0;
#pragma unroll
  for (int d = 0; d < M; d++) {
    tv[d] = osa[d] >= 0 ? t.ts[osa[d]] : INT64_MAX;
    m += osa[d] >= 0 ? 1 : 0;
  }
  // ascending bitonic sort (the unseen INT64_MAX pads go last), upper median
#pragma unroll
  for (int size = 2; size <= M; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int i = 0; i < M; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const int64_t u = tv[i], w = tv[j];
          const bool sw = up ? (w < u) : (u < w);
          tv[i] = sw ? w : u;
          tv[j] = sw ? u : w;
        }
      }
    }
  }
  int64_t med = tv[0];
#pragma unroll
  for (int i = 1; i < M; i++) med = (i == m / 2) ? tv[i] : med;
  recv_call[q] = best;
  rr_out[q] = rr;
  cts_out[q] = med;
}
template <int NWT>
__global__ void k_round_received(Tables t, const int32_t* cand, int ncand, const int32_t* vis,
                                 int ncalls, int call_lo, int rr_lo, int R_last,
                                 const int32_t* segoff, const int32_t* segcnt,
                                 const int32_t* seg_call, const uint8_t* seg_dec,
                                 const uint64_t* seg_fws, const int32_t* theta,
                                 int32_t* recv_call, int32_t* rr_out, int64_t* cts_out,
                                 int32_t* bseg_out) {
  round_received_item<NWT>(t, blockIdx.x * blockDim.x + threadIdx.x, cand, ncand, vis, ncalls, call_lo, rr_lo,
                           R_last, segoff, segcnt, seg_call, seg_dec, seg_fws, theta, recv_call, rr_out, cts_out,
                           bseg_out);
}

// The upper median over 32-bit order-preserving images (int32 timestamp offsets ^
// 0x80000000), a byte at a time (radix 256) from the top byte of max - min: per
// digit one LDS histogram of the live values (the wave's own 256 bins), a wave scan
// of the bins and the bin that holds rank kk; the live set narrows to that bin and
// the select ends once one value is left.  A 20-24-bit span takes three digits; the
// bit-at-a-time select it replaced took twenty-odd steps (6.27 -> 6.0 ms at 256/10M).
// hist: the wave's 256 ints in LDS.  Returns the image.
// Wave-wide inclusive scans by DPP row shifts and row broadcasts (VALU, no LDS
// crossbar): row_shr 1/2/4/8 scan each 16-lane row, row_bcast15 / row_bcast31 carry
// rows 0 -> 1, 2 -> 3 and rows 0-1 -> 2-3.  A lane whose source is outside its row
// (or a row the mask leaves out) takes the identity.  Every lane of the wave must be
// active (EXEC full): an inactive source lane would read as the identity, not its
// value.  row_bcast15/31 exist on GFX9-family targets (CDNA) only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "HGE_DPP_SCAN needs the GFX9-family DPP row broadcasts (CDNA; built for gfx950)"
#endif
#define HGE_DPP_SCAN(x, op, id)                                                        \
  do {                                                                                 \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x111, 0xf, 0xf, false));         \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x112, 0xf, 0xf, false));         \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x114, 0xf, 0xf, false));         \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x118, 0xf, 0xf, false));         \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x142, 0xa, 0xf, false));         \
    x = op(x, __builtin_amdgcn_update_dpp((id), (x), 0x143, 0xc, 0xf, false));         \
  } while (0)
__device__ __forceinline__ int dpp_add(int a, int b) { return a + b; }
__device__ __forceinline__ int dpp_umin(int a, int b) { return (int)min((uint32_t)a, (uint32_t)b); }
__device__ __forceinline__ int dpp_umax(int a, int b) { return (int)max((uint32_t)a, (uint32_t)b); }

template <int VPL>
__device__ __forceinline__ uint32_t wave_upper_median32_r8(const uint32_t (&v)[VPL], const bool (&in)[VPL],
                                                           int* hist) {
  const int lane = threadIdx.x & 63;
  int n = 0;
  uint32_t mn = ~0u, mx = 0;
#pragma unroll
  for (int k = 0; k < VPL; k++) {
    n += __popcll(__ballot(in[k]));
    if (in[k]) {
      mn = min(mn, v[k]);
      mx = max(mx, v[k]);
    }
  }
  int smn = (int)mn, smx = (int)mx;
  HGE_DPP_SCAN(smn, dpp_umin, -1);
  HGE_DPP_SCAN(smx, dpp_umax, 0);
  mn = (uint32_t)__builtin_amdgcn_readlane(smn, 63);  // lane 63: the whole wave
  if (n == 0) return mn;  // no value (a candidate that is not stored)
  const uint32_t span = (uint32_t)__builtin_amdgcn_readlane(smx, 63) - mn;
  int kk = n / 2;  // 0-based rank of the upper median
  uint32_t vr[VPL];
  bool live[VPL];
#pragma unroll
  for (int k = 0; k < VPL; k++) {
    vr[k] = v[k] - mn;
    live[k] = in[k];
  }
  uint32_t pre = 0;
  for (int sft = span ? (31 - __builtin_clz(span)) / 8 * 8 : 0;; sft -= 8) {
    // the live values' digits: one histogram (bins 4l .. 4l + 3 belong to lane l)
    *(int4*)&hist[4 * lane] = make_int4(0, 0, 0, 0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < VPL; k++)
      if (live[k]) atomicAdd(&hist[(vr[k] >> sft) & 255u], 1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int4 b = *(const int4*)&hist[4 * lane];
    const int tot = b.x + b.y + b.z + b.w;
    int inc = tot;  // inclusive scan of the lanes' totals
    HGE_DPP_SCAN(inc, dpp_add, 0);
    const int ex = inc - tot;
    const uint64_t hit = __ballot(ex <= kk && kk < inc);
    const int L = (int)__builtin_ctzll(hit);
    // in lane L: the bin of rank kk and the rank within it
    int r = kk - ex, dg = 0, cnt = b.x;
    if (r >= b.x) {
      r -= b.x;
      dg = 1;
      cnt = b.y;
      if (r >= b.y) {
        r -= b.y;
        dg = 2;
        cnt = b.z;
        if (r >= b.z) {
          r -= b.z;
          dg = 3;
          cnt = b.w;
        }
      }
    }
    const uint32_t digit = (uint32_t)(4 * L + __builtin_amdgcn_readlane(dg, L));
    kk = __builtin_amdgcn_readlane(r, L);
    const int nbin = __builtin_amdgcn_readlane(cnt, L);
    pre |= digit << sft;
#pragma unroll
    for (int k = 0; k < VPL; k++) live[k] = live[k] && ((vr[k] >> sft) & 255u) == digit;
    if (nbin == 1 || sft == 0) {
      if (sft == 0) return mn + pre;
      // the one live value: its low bits too
#pragma unroll
      for (int k = 0; k < VPL; k++) {
        const uint64_t m = __ballot(live[k]);
        if (m) return mn + (uint32_t)__builtin_amdgcn_readlane((int)vr[k], (int)__builtin_ctzll(m));
      }
    }
    __builtin_amdgcn_wave_barrier();  // every lane has read the bins before they are cleared
  }
}

// Upper median (element len/2 of the sorted list, MedianTimestamp,
// hashgraph.go:762-770) of the wave's values v[k] where in[k]: a bitwise radix
// select over the order-preserving uint64 image (ts ^ sign bit), skipping the
// high bits every candidate shares.  Wave-uniform result.
template <int VPL>
__device__ __forceinline__ int64_t wave_upper_median(const uint64_t (&v)[VPL], const bool (&in)[VPL]) {
  int n = 0;
  uint64_t mn = ~0ull, mx = 0;
#pragma unroll
  for (int k = 0; k < VPL; k++) {
    n += __popcll(__ballot(in[k]));
    if (in[k]) {
      mn = min(mn, v[k]);
      mx = max(mx, v[k]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (uint64_t)__shfl_xor((long long)mn, o));
    mx = max(mx, (uint64_t)__shfl_xor((long long)mx, o));
  }
  int kk = n / 2;  // 0-based rank of the upper median
  const bool narrow = __builtin_amdgcn_readfirstlane((int)(mx - mn < (1ull << 32))) != 0;
  if (narrow && n > 0) {
    // the values span < 2^32: radix-select the 32-bit offsets from the minimum
    // with the live sets as wave masks (scalar registers), two vector
    // instructions per value word and bit
    uint32_t vr[VPL];
    uint64_t lm[VPL];
#pragma unroll
    for (int k = 0; k < VPL; k++) {
      vr[k] = (uint32_t)(v[k] - mn);
      lm[k] = __ballot(in[k]);
    }
    const uint32_t span = __builtin_amdgcn_readfirstlane((uint32_t)(mx - mn));  // wave-uniform
    uint32_t pre = 0;
    int nlive = n;
    for (int b = span ? 31 - __builtin_clz(span) : -1; b >= 0; b--) {
      uint64_t bm[VPL];
      int c0 = 0;
#pragma unroll
      for (int k = 0; k < VPL; k++) {
        bm[k] = __ballot((vr[k] >> b) & 1u);
        c0 += __popcll(lm[k] & ~bm[k]);
      }
      const bool one = kk >= c0;
      if (one) {
        kk -= c0;
        pre |= 1u << b;
        nlive -= c0;
      } else {
        nlive = c0;
      }
#pragma unroll
      for (int k = 0; k < VPL; k++) lm[k] &= one ? bm[k] : ~bm[k];
      if (nlive == 1) {
        // one value left with this prefix: it is the answer (kk == 0), low bits and all
#pragma unroll
        for (int k = 0; k < VPL; k++)
          if (lm[k]) {
            const uint32_t w = (uint32_t)__shfl((int)vr[k], (int)__builtin_ctzll(lm[k]));
            return (int64_t)((mn + w) ^ 0x8000000000000000ull);
          }
      }
    }
    return (int64_t)((mn + pre) ^ 0x8000000000000000ull);
  }
  uint64_t prefix = mn;
  const uint64_t diff = mn ^ mx;
  if (diff) {
    const int top = 63 - __builtin_clzll(diff);
    prefix = (mn >> (top + 1)) << (top + 1);  // shared high bits
    bool live[VPL];
#pragma unroll
    for (int k = 0; k < VPL; k++) live[k] = in[k];
    int nlive = n;
    for (int b = top; b >= 0; b--) {
      int c0 = 0;
#pragma unroll
      for (int k = 0; k < VPL; k++) c0 += __popcll(__ballot(live[k] && !((v[k] >> b) & 1ull)));
      const bool one = kk >= c0;
      if (one) {
        kk -= c0;
        prefix |= 1ull << b;
        nlive -= c0;
      } else {
        nlive = c0;
      }
#pragma unroll
      for (int k = 0; k < VPL; k++) live[k] = live[k] && (((v[k] >> b) & 1ull) == (one ? 1ull : 0ull));
      if (nlive == 1) {
        // one value left with this prefix: it is the answer (kk == 0), low bits and all
        // (~8 bits in for distinct values instead of every bit below the top one)
#pragma unroll
        for (int k = 0; k < VPL; k++) {
          const uint64_t m = __ballot(live[k]);
          if (m) return (int64_t)((uint64_t)__shfl((long long)v[k], (int)__builtin_ctzll(m)) ^ 0x8000000000000000ull);
        }
      }
    }
  }
  return (int64_t)(prefix ^ 0x8000000000000000ull);
}

// The round-r frontier rows transposed, for every round a received event can
// have: WLA[r][cx][d] = LA[(d, C[r][d])][cx] (-1: chain d has no event of round
// >= r).  The witness of round r on chain d sits at C[r][d]; w_d sees x iff
// index(x) <= WLA[r][creator(x)][d].  64 x 64 tiles through LDS.
__global__ void __launch_bounds__(256) k_witness_la(Tables t, int rr_lo) {
  __shared__ int32_t tile[64][65];
  const int N = t.N;
  const int rr = rr_lo + blockIdx.z;
  const int d0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  // all 16 frontier positions, then all 16 row values, each batch in flight
  // together (a loop with one dependent pair of loads per row was ~12 us per online
  // call at N = 256: the rows sit in different pages)
  int pw[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int d = d0 + ty + 4 * k;
    pw[k] = d < N ? t.C[(size_t)rr * N + d] : INF32;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int d = d0 + ty + 4 * k, cx = c0 + tx;
    const bool on = d < N && cx < N && pw[k] != INF32;
    const int v = la_at(t, on ? d : 0, on ? pw[k] : 0, on ? cx : 0);
    tile[ty + 4 * k][tx] = on ? v : -1;
    // the row-major copy (theta's staging reads a famous witness's row coalesced)
    if (t.WLR && d < N && cx < N) t.WLR[((size_t)rr * N + d) * N + cx] = (uint16_t)((on ? v : -1) + 1);
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int cx = c0 + r, d = d0 + tx;
    if (cx < N && d < N) {
      if (t.WLA16) t.WLA16[((size_t)rr * N + cx) * N + d] = (uint16_t)(tile[tx][r] + 1);
      else t.WLA[((size_t)rr * N + cx) * N + d] = tile[tx][r];
    }
  }
}

// MedianTimestamp (hashgraph.go:762-770) for wide hashgraphs: one wave per
// received event.  Lane l holds the timestamps of the famous witnesses
// d = l, l+64, ... that see x (OSA(w, x) = FD[x][cw], its timestamp offset FDTD[x][cw]);
// the upper median (element len/2 of the sorted list) is found by a radix-256
// select over the order-preserving uint32 image of the int32 offsets
// (wave_upper_median32_r8; base + the median offset), or of the int64 timestamps
// for a row flagged in FDTW (wave_upper_median).
// Every per-witness input is a coalesced row: the "sees x" thresholds
// WLA[rr][cx][.] (k_witness_la) and the timestamp offsets FDTD[x][.] (k_fd_transpose_ts),
// instead of 2N scattered gathers per event.
// events per k_median_wave wave (the grid is sized from it)
constexpr int MED_EPW = 1;
template <int VPL>
__global__ void __launch_bounds__(256) k_median_wave(Tables t, const int32_t* cand, int ncand,
                                                     const int32_t* recv_call, const int32_t* rr_in,
                                                     const int32_t* bseg, const uint64_t* seg_fws,
                                                     int64_t* cts_out) {
  // MW_E events per wave (candidates q0 + e * nw, nw = the grid's wave count; 1 measured
  // fastest once the select became cheap: 6.36 vs 6.62 ms at 2, 8.19 at 3): all
  // their loads are in flight together before the first select
  constexpr int MW_E = MED_EPW;
  __shared__ __attribute__((aligned(16))) int s_mhist[4][256];  // each wave's select bins
  const int nw = gridDim.x * 4;
  // (the XCD-aware order of k_fame_decide measured 0.2 ms slower here, and a
  // chain-major order -- a threshold row shared by consecutive waves -- 10.4 vs 6.0 ms)
  const int q0 = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int N = t.N, NW = t.NW;
  int qe[MW_E], ixe[MW_E];
  bool live[MW_E];
  uint64_t fw[MW_E][VPL];
  int th[MW_E][VPL];
  int64_t ts[MW_E][VPL];   // exact timestamps (wide rows only)
  int32_t off[MW_E][VPL];  // offsets from x's own timestamp
  int64_t bse[MW_E];
  int wde[MW_E];
#pragma unroll
  for (int e = 0; e < MW_E; e++) {
    const int q = q0 + e * nw;
    const int qq = q < ncand ? q : ncand - 1;  // valid indices; the result is not stored
    const int x = cand ? cand[qq] : qq;
    const int rc = recv_call[qq], rr0 = rr_in[qq], sg0 = bseg[qq];
    const int cx = t.creator[x], ix = t.index[x];
    // an event not received (rc < 0) runs through with valid indices and is not
    // stored: no branch between these loads and the row loads below
    live[e] = q < ncand && rc >= 0;
    const int rr = live[e] ? rr0 : 0, sg = live[e] ? sg0 : 0;
    qe[e] = q;
    ixe[e] = ix;
    const size_t rw = (size_t)cx * t.ccap + ix;
    const int32_t* tdr = t.FDTD + rw * N;
    // the FD timestamps as int32 offsets from x's own timestamp; a row with an offset
    // outside int32 (flagged per 64-column tile) gathers the exact ones instead
    const int NT = (N + 63) >> 6;
    int wide = 0;
    if (NT == 4) {
      wide = *(const int32_t*)(t.FDTW + rw * 4);  // one aligned load for the 4 tiles
    } else {
      for (int k = 0; k < NT; k++) wide |= t.FDTW[rw * NT + k];
    }
    bse[e] = t.ts[x];
    wde[e] = __builtin_amdgcn_readfirstlane(wide);
    if (VPL == 4 && t.WLA16) {
      // lane l takes witnesses d = 4l .. 4l + 3: its thresholds in one 8-byte load
      // (LA + 1 as uint16), its offsets in one 16-byte load, one fame word.  Lanes past
      // N / 4 (N < 256) load the last group again and are masked out below (d >= N).
      const int l4 = min(lane, (N >> 2) - 1);
      const uint2 tw = *(const uint2*)(t.WLA16 + ((size_t)rr * N + cx) * N + 4 * l4);
      const int4 ow = *(const int4*)(tdr + 4 * l4);
      const uint64_t f = seg_fws[(size_t)sg * NW + (lane >> 4)];
      const uint32_t u[4] = {tw.x & 0xFFFFu, tw.x >> 16, tw.y & 0xFFFFu, tw.y >> 16};
      const int32_t o4[4] = {ow.x, ow.y, ow.z, ow.w};
#pragma unroll
      for (int k = 0; k < VPL; k++) {
        fw[e][k] = f;
        th[e][k] = (int)u[k & 3] - 1;
        off[e][k] = o4[k & 3];
      }
    } else {
      const int32_t* thr = t.WLA + ((size_t)rr * N + cx) * N;
#pragma unroll
      for (int k = 0; k < VPL; k++) {
        const int dd = min(lane + 64 * k, N - 1);
        fw[e][k] = seg_fws[(size_t)sg * NW + (k < NW ? k : 0)];
        th[e][k] = thr[dd];
        off[e][k] = tdr[dd];
      }
    }
    if (wde[e]) {
#pragma unroll
      for (int k = 0; k < VPL; k++) {
        const int dd = VPL == 4 && t.WLA16 ? min(4 * lane + k, N - 1) : min(lane + 64 * k, N - 1);
        const int f = fd_at(t, rw, dd);
        ts[e][k] = f != INF32 ? t.tsch[(size_t)dd * t.ccap + f] : 0;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < MW_E; e++) {
    bool in[VPL];
#pragma unroll
    for (int k = 0; k < VPL; k++) {
      const int d = VPL == 4 && t.WLA16 ? 4 * lane + k : lane + 64 * k;
      in[k] = d < N && ((fw[e][k] >> (d & 63)) & 1ull) && th[e][k] >= ixe[e];
    }
    int64_t med;
    if (!wde[e]) {  // int32 offsets: the median of (base + o) is base + the median of o
      uint32_t v[VPL];
#pragma unroll
      for (int k = 0; k < VPL; k++) v[k] = in[k] ? ((uint32_t)off[e][k] ^ 0x80000000u) : ~0u;
      med = bse[e] + (int64_t)(int32_t)(wave_upper_median32_r8<VPL>(v, in, s_mhist[threadIdx.x >> 6]) ^ 0x80000000u);
    } else {
      uint64_t v[VPL];
#pragma unroll
      for (int k = 0; k < VPL; k++) v[k] = in[k] ? ((uint64_t)ts[e][k] ^ 0x8000000000000000ull) : ~0ull;
      med = wave_upper_median<VPL>(v, in);
    }
    if (lane == 0 && live[e]) cts_out[qe[e]] = med;
  }
}

// ---------------------------------------------------------------------------
// FindOrder sort (hashgraph.go:744-745, consensus_sorter.go:36-59): key
// (call, roundReceived, consensusTimestamp, S) with S compared as an unsigned
// 256-bit integer (the whitening PRN is identically 0), id as a final tie-break.
// ---------------------------------------------------------------------------
struct OKey {
  uint64_t a;  // call << 32 | rr
  uint64_t b;  // cts ^ sign
  uint64_t s0, s1, s2, s3;
  uint32_t id;
  uint32_t pad;
};

__device__ __forceinline__ bool okless(const OKey& x, const OKey& y) {
  if (x.a != y.a) return x.a < y.a;
  if (x.b != y.b) return x.b < y.b;
  if (x.s0 != y.s0) return x.s0 < y.s0;
  if (x.s1 != y.s1) return x.s1 < y.s1;
  if (x.s2 != y.s2) return x.s2 < y.s2;
  if (x.s3 != y.s3) return x.s3 < y.s3;
  return x.id < y.id;
}

// flags for compaction: received (and committing) vs still undetermined; with
// call_counts, the events each call receives (the order's call buckets)
__global__ void k_recv_flags(const int32_t* recv_call, int ncand, int32_t* f_recv,
                             int32_t* f_und, int commit, int32_t* call_counts) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int rc = q < ncand ? recv_call[q] : -1;
  const bool r = rc >= 0;
  if (q < ncand) {
    if (f_recv) f_recv[q] = r;
    // -1: not received (stays undetermined); below -1: another part's (split replay)
    f_und[q] = commit ? rc == -1 : 1;
  }
  if (!call_counts) return;
  // neighbouring candidates are mostly received by the same call: one atomic
  // per distinct call in the wave
  const int lane = threadIdx.x & 63;
  uint64_t pending = __ballot(r);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const int c = __shfl(rc, leader);
    const uint64_t same = __ballot(r && rc == c);
    if (lane == leader) atomicAdd(&call_counts[c], __popcll(same));
    pending &= ~same;
  }
}

// ---------------------------------------------------------------------------
// FindOrder's sort as call buckets: a counting sort by call (k_recv_flags
// counts, one scan gives the bucket ends), the keys scattered into their
// bucket in any order, then one workgroup per call sorts its bucket by
// (rr, cts, S, id): an LDS bitonic index sort up to 512 keys, larger buckets
// as 512-key chunks merged pairwise (merge path) through global scratch.
// ---------------------------------------------------------------------------
// (also records roundReceived / consensusTimestamp and sums the transactions,
// as k_set_rr does outside a committing batch)
// candidate q's key into its call's bucket (a slot per wave and call by one atomic);
// returns the wave's transaction count (every lane)
__device__ __forceinline__ unsigned long long bucket_key_item(const Tables& t, int q, const int32_t* cand, int ncand,
                                                              const int32_t* recv_call, const int32_t* rr,
                                                              const int64_t* cts, int32_t* bpos, OKey* keys,
                                                              int32_t* ev_rr, int64_t* ev_cts) {
  const int lane = threadIdx.x & 63;
  const int rc = q < ncand ? recv_call[q] : -1;
  const bool rec = rc >= 0;
  const int x = rec ? cand[q] : 0;
  unsigned long long tx = rec ? (unsigned long long)t.ntx[x] : 0;
  for (int o = 32; o > 0; o >>= 1) tx += __shfl_xor(tx, o);
  int slot = 0;
  uint64_t pending = __ballot(rec);
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const int c = __shfl(rc, leader);
    const uint64_t same = __ballot(rec && rc == c);
    int base = 0;
    if (lane == leader) base = atomicAdd(&bpos[c], __popcll(same));
    base = __shfl(base, leader);
    if (rec && rc == c) slot = base + __popcll(same & ((1ull << lane) - 1));
    pending &= ~same;
  }
  if (rec) {
    ev_rr[x] = rr[q];
    ev_cts[x] = cts[q];
    OKey k;
    k.a = ((uint64_t)(uint32_t)rc << 32) | (uint32_t)rr[q];
    k.b = (uint64_t)cts[q] ^ 0x8000000000000000ull;
    k.s0 = t.S[4 * (size_t)x];
    k.s1 = t.S[4 * (size_t)x + 1];
    k.s2 = t.S[4 * (size_t)x + 2];
    k.s3 = t.S[4 * (size_t)x + 3];
    k.id = (uint32_t)x;
    k.pad = 0;
    keys[slot] = k;
  }
  return tx;
}

__global__ void k_bucket_keys(Tables t, const int32_t* cand, int ncand, const int32_t* recv_call,
                              const int32_t* rr, const int64_t* cts, int32_t* bpos, OKey* keys,
                              int32_t* ev_rr, int64_t* ev_cts, unsigned long long* ntx_sum) {
  // ntx_sum: one partial per block (launched with 256 threads; summed by the host, no
  // global atomics)
  __shared__ unsigned long long s_tx[4];
  const unsigned long long tx = bucket_key_item(t, blockIdx.x * blockDim.x + threadIdx.x, cand, ncand, recv_call,
                                                rr, cts, bpos, keys, ev_rr, ev_cts);
  if ((threadIdx.x & 63) == 0) s_tx[threadIdx.x >> 6] = tx;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long bt = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) bt += s_tx[w];
    ntx_sum[blockIdx.x] = bt;
  }
}

__device__ __forceinline__ OKey okey_inf() {
  OKey inf;
  inf.a = inf.b = inf.s0 = inf.s1 = inf.s2 = inf.s3 = ~0ull;
  inf.id = 0xFFFFFFFFu;
  inf.pad = 0;
  return inf;
}

// first index i in [0, la] of A such that A[i..] and B[k-i..] split the merged
// prefix of length k (keys are unique)
__device__ int merge_corank(const OKey* A, int la, const OKey* B, int lb, int k) {
  int lo = max(0, k - lb), hi = min(k, la);
  while (lo < hi) {
    const int i = (lo + hi) >> 1;  // take i from A, k - i from B
    if (okless(A[i], B[k - i - 1])) lo = i + 1;
    else hi = i;
  }
  return lo;
}

// barrier after a bitonic stage of stride cur followed by one of stride nxt: with
// i = pair index = thread (+ k * blockDim), a stride <= 64 keeps a wave's pairs
// inside its own 128 slots [128w, 128w + 128), so two such stages in a row need
// only the wave's own LDS order (no block barrier: 10 of 55 stages at 1,024 keys
// keep one)
__device__ __forceinline__ void bitonic_sync(int cur, int nxt) {
  if (cur <= 64 && nxt <= 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    __syncthreads();
  }
}

// LDS chunk of keys as structure-of-arrays (conflict-free per field) sorted
// through a uint16 index permutation: a compare-exchange reads two indices and
// the fields up to the first difference, and swaps only the indices.
template <int CH>
struct SortChunk {
  uint64_t a[CH], b[CH], s0[CH], s1[CH], s2[CH], s3[CH];
  uint32_t id[CH];
  uint16_t ix[CH];
  __device__ void put(int i, const OKey& k) {
    a[i] = k.a;
    b[i] = k.b;
    s0[i] = k.s0;
    s1[i] = k.s1;
    s2[i] = k.s2;
    s3[i] = k.s3;
    id[i] = k.id;
    ix[i] = (uint16_t)i;
  }
  __device__ OKey get(int i) const {
    OKey k;
    k.a = a[i];
    k.b = b[i];
    k.s0 = s0[i];
    k.s1 = s1[i];
    k.s2 = s2[i];
    k.s3 = s3[i];
    k.id = id[i];
    k.pad = 0;
    return k;
  }
  __device__ bool less(int x, int y) const {
    if (a[x] != a[y]) return a[x] < a[y];
    if (b[x] != b[y]) return b[x] < b[y];
    if (s0[x] != s0[y]) return s0[x] < s0[y];
    if (s1[x] != s1[y]) return s1[x] < s1[y];
    if (s2[x] != s2[y]) return s2[x] < s2[y];
    if (s3[x] != s3[y]) return s3[x] < s3[y];
    return id[x] < id[y];
  }
  // bitonic sort of ix[0, P) (P a power of two <= CH) by the whole block
  __device__ void sort(int P) {
    const int tid = threadIdx.x, T = blockDim.x;
    for (int size = 2; size <= P; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int i = tid; i < P / 2; i += T) {
          const int lo = 2 * stride * (i / stride) + (i % stride);
          const int hi = lo + stride;
          const bool up = ((lo & size) == 0);
          const int x = ix[lo], y = ix[hi];
          if (less(y, x) == up) {
            ix[lo] = (uint16_t)y;
            ix[hi] = (uint16_t)x;
          }
        }
        bitonic_sync(stride, stride > 1 ? stride >> 1 : size);
      }
    }
  }
};

// bucket offsets (exclusive scan of the per-call counts, total = events
// received) and the list of non-empty buckets, by one block
__device__ __forceinline__ void bucket_list_body(const int32_t* cnt, int n, int32_t* off, int32_t* total,
                                                 int32_t* list, int32_t* nlist) {
  // per-thread contiguous runs, wave scans by shuffles, one scan of the 16 wave
  // totals: two barriers (a Hillis-Steele over the 1024 partials took twenty)
  __shared__ int ws[16], wn[16];
  const int T = blockDim.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (n + T - 1) / T;
  const int lo = min(n, tid * per), hi = min(n, lo + per);
  int s = 0, ne = 0;
  for (int i = lo; i < hi; i++) {
    const int v = cnt[i];
    s += v;
    ne += v > 0 ? 1 : 0;
  }
  int is = s, in = ne;  // inclusive over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int a = __shfl_up(is, o, 64), b = __shfl_up(in, o, 64);
    if (lane >= o) {
      is += a;
      in += b;
    }
  }
  if (lane == 63) {
    ws[wv] = is;
    wn[wv] = in;
  }
  __syncthreads();
  if (wv == 0) {
    int a = lane < T / 64 ? ws[lane] : 0, b = lane < T / 64 ? wn[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int x = __shfl_up(a, o, 64), y = __shfl_up(b, o, 64);
      if (lane >= o) {
        a += x;
        b += y;
      }
    }
    if (lane < T / 64) {
      ws[lane] = a;
      wn[lane] = b;
    }
  }
  __syncthreads();
  int run = (wv > 0 ? ws[wv - 1] : 0) + is - s, pos = (wv > 0 ? wn[wv - 1] : 0) + in - ne;
  for (int i = lo; i < hi; i++) {
    const int v = cnt[i];
    off[i] = run;
    run += v;
    if (v > 0) list[pos++] = i;
  }
  if (tid == T - 1) {
    *total = ws[T / 64 - 1];
    *nlist = wn[T / 64 - 1];
  }
}
__global__ void __launch_bounds__(1024) k_bucket_list(const int32_t* cnt, int n, int32_t* off, int32_t* total,
                                                      int32_t* list, int32_t* nlist) {
  bucket_list_body(cnt, n, off, total, list, nlist);
}
// An online call (a few calls, <= 16k candidates): k_recv_flags' work folded in as
// well.  Block 0 counts the received events per call in LDS, stores the counts and
// builds the call buckets from them; block 1 writes the undetermined flags
// (recv_call == -1), then scans and compacts them.  Each block reads back only
// global data it wrote itself, after a barrier.
__global__ void __launch_bounds__(1024) k_recv_list_und(const int32_t* recv_call, int ncand, int32_t* cnt,
                                                        int ncalls, int32_t* off, int32_t* total, int32_t* list,
                                                        int32_t* nlist, int32_t* f_und, int32_t* upos,
                                                        int32_t* nund, const int32_t* cand, int32_t* und) {
  constexpr int MAXC = 8;
  if (blockIdx.x == 0) {
    __shared__ int s_cnt[MAXC];
    if (threadIdx.x < MAXC) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    for (int q = threadIdx.x; q < ncand; q += blockDim.x) {
      const int rc = recv_call[q];
      if (rc >= 0) atomicAdd(&s_cnt[rc], 1);
    }
    __syncthreads();
    if ((int)threadIdx.x < ncalls) cnt[threadIdx.x] = s_cnt[threadIdx.x];
    __syncthreads();
    bucket_list_body(cnt, ncalls, off, total, list, nlist);
  } else {
    for (int q = threadIdx.x; q < ncand; q += blockDim.x) f_und[q] = recv_call[q] == -1 ? 1 : 0;
    __syncthreads();
    scan_small_body(f_und, upos, ncand, nund, cand, und);
  }
}

// an online call's two single-block steps after k_recv_flags in one launch: block 0
// the call buckets (k_bucket_list), block 1 the new undetermined list's scan and
// compaction (k_scan_small + k_scatter_und; fl.size <= 16k)
__global__ void __launch_bounds__(1024) k_list_und(const int32_t* cnt, int n, int32_t* off, int32_t* total,
                                                   int32_t* list, int32_t* nlist, const int32_t* f_und,
                                                   int32_t* upos, int ncand, int32_t* nund, const int32_t* cand,
                                                   int32_t* und) {
  if (blockIdx.x == 0) bucket_list_body(cnt, n, off, total, list, nlist);
  else scan_small_body(f_und, upos, ncand, nund, cand, und);
}

// keys per bucket that k_bucket_sort_big sorts whole in LDS (k_bucket_sort leaves them to it)
constexpr int BIG_SORT = 8192;

constexpr int SORT_CH = 512;  // keys per LDS chunk (k_bucket_sort)
__device__ void bucket_sort_one(int b, const int32_t* bend, const int32_t* bcnt, OKey* keys,
                                OKey* tmp, int32_t* ids_out, bool skip_big, SortChunk<SORT_CH>& sc) {
  constexpr int CH = SORT_CH;
  const int n = bcnt[b];
  if (n == 0 || (skip_big && n > CH && n <= 2 * BIG_SORT)) return;
  const int start = bend[b] - n;
  const int tid = threadIdx.x, T = blockDim.x;
  if (n == 1) {
    if (tid == 0) ids_out[start] = (int32_t)keys[start].id;
    return;
  }
  if (n <= CH) {
    int P = 2;
    while (P < n) P <<= 1;
    for (int i = tid; i < P; i += T) sc.put(i, i < n ? keys[start + i] : okey_inf());
    __syncthreads();
    sc.sort(P);
    for (int i = tid; i < n; i += T) ids_out[start + i] = (int32_t)sc.id[sc.ix[i]];
    return;
  }
  // large bucket (past 2 * BIG_SORT, or every one with HGE_BIG_SORT=0): sorted
  // CH-key chunks, then pairwise merges (ping-pong)
  OKey* src = keys + start;
  OKey* dst = tmp + start;
  for (int c0 = 0; c0 < n; c0 += CH) {
    const int m = min(CH, n - c0);
    for (int i = tid; i < CH; i += T) sc.put(i, i < m ? src[c0 + i] : okey_inf());
    __syncthreads();
    sc.sort(CH);
    for (int i = tid; i < m; i += T) src[c0 + i] = sc.get(sc.ix[i]);
    __syncthreads();
  }
  for (int run = CH; run < n; run <<= 1) {
    for (int a0 = 0; a0 < n; a0 += 2 * run) {
      const int la = min(run, n - a0);
      const int lb = max(0, min(run, n - a0 - run));
      const OKey* A = src + a0;
      const OKey* B = A + la;
      const int len = la + lb;
      const int k0 = (int)((int64_t)len * tid / T), k1 = (int)((int64_t)len * (tid + 1) / T);
      int i = merge_corank(A, la, B, lb, k0), j = k0 - i;
      for (int k = k0; k < k1; k++) {
        const bool takeA = j >= lb || (i < la && okless(A[i], B[j]));
        dst[a0 + k] = takeA ? A[i++] : B[j++];
      }
    }
    __syncthreads();
    OKey* sw = src;
    src = dst;
    dst = sw;
  }
  for (int i = tid; i < n; i += T) ids_out[start + i] = (int32_t)src[i].id;
}

// one block per non-empty bucket (grid-stride over the list)
__global__ void __launch_bounds__(256) k_bucket_sort(const int32_t* bend, const int32_t* bcnt,
                                                     const int32_t* list, const int32_t* nlist,
                                                     OKey* keys, OKey* tmp, int32_t* ids_out, int skip_big) {
  __shared__ SortChunk<SORT_CH> sc;
  for (int li = blockIdx.x; li < *nlist; li += gridDim.x) {
    bucket_sort_one(list[li], bend, bcnt, keys, tmp, ids_out, skip_big != 0, sc);
    __syncthreads();
  }
}

// Buckets of 513 .. BIG_SORT keys -- in a replay nearly every key sits in one: the
// call that decides a round's fame receives that round's ~EPR events at once
// (3,448 at N = 256; 256/2M: 422 calls of 2-4k keys, 68 of 4-8k, 4 larger,
// scripts/analysis/call_buckets.py).  One 1024-thread block sorts such a bucket
// whole in LDS: a bitonic index sort over (rr, cts, the top 32 bits of S) -- the
// call is the bucket's -- 18 bytes per key, 147 KB at 8,192 keys; keys equal on
// those bits are ordered by the full key from HBM.  k_bucket_sort's 512-key
// chunks + pairwise merges through global scratch moved ~50x the keys' bytes for
// such buckets (25 GB per 256/10M replay, rocprofv3 PMC).
// bitonic index sort of K[0, n) (n <= BIG_SORT) in LDS by (rr, cts, the top 32 bits
// of S), then the full key from HBM on ties; ix[0, n) = the sorted local indices
__device__ void big_bitonic(const OKey* K, int n, uint64_t* sb, uint32_t* sr, uint32_t* ss, uint16_t* ix) {
  const int tid = threadIdx.x, T = blockDim.x;
  int P = 1024;
  while (P < n) P <<= 1;
  for (int i = tid; i < P; i += T) {
    if (i < n) {
      const OKey k = K[i];
      sr[i] = (uint32_t)k.a;  // rr (the call is the bucket's)
      sb[i] = k.b;
      ss[i] = (uint32_t)(k.s0 >> 32);
    } else {
      sr[i] = 0xFFFFFFFFu;
      sb[i] = ~0ull;
      ss[i] = 0xFFFFFFFFu;
    }
    ix[i] = (uint16_t)i;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P / 2; i += T) {
        const int lo = 2 * stride * (i / stride) + (i % stride);
        const int hi = lo + stride;
        const bool up = ((lo & size) == 0);
        const int x = ix[lo], y = ix[hi];
        bool yl;  // key y < key x
        if (sr[x] != sr[y]) yl = sr[y] < sr[x];
        else if (sb[x] != sb[y]) yl = sb[y] < sb[x];
        else if (ss[x] != ss[y]) yl = ss[y] < ss[x];
        else if (x >= n || y >= n) yl = y < x;  // padding (only padding ties padding)
        else yl = okless(K[y], K[x]);          // equal leading bits: the full key
        if (yl == up) {
          ix[lo] = (uint16_t)y;
          ix[hi] = (uint16_t)x;
        }
      }
      bitonic_sync(stride, stride > 1 ? stride >> 1 : size);
    }
  }
}

// Buckets of BIG_SORT + 1 .. 2 * BIG_SORT keys (a call that receives more than one
// round's worth: 33 calls of 8-16k keys at 256/10M) are two halves sorted in LDS
// the same way, then one merge-path pass over their index lists (scratch: the
// bucket's slice of tmp), each thread placing nb / 1024 outputs from its co-rank.
// one bucket of 513 .. 2 * BIG_SORT keys (block-uniform)
__device__ void bucket_sort_big_one(int b, int nb, const int32_t* bend, const OKey* keys, OKey* tmp,
                                    int32_t* ids_out, uint64_t* sb, uint32_t* sr, uint32_t* ss, uint16_t* ix) {
  const int tid = threadIdx.x, T = blockDim.x;
  {
    const OKey* K = keys + (bend[b] - nb);
    int32_t* out = ids_out + (bend[b] - nb);
    if (nb <= BIG_SORT) {
      big_bitonic(K, nb, sb, sr, ss, ix);
      for (int i = tid; i < nb; i += T) out[i] = (int32_t)K[ix[i]].id;
      __syncthreads();
      return;
    }
    int32_t* S = (int32_t*)(tmp + (bend[b] - nb));  // 4 of the 48 scratch bytes per key
    const int na = (nb + 1) >> 1, nbb = nb - na;
    big_bitonic(K, na, sb, sr, ss, ix);
    for (int i = tid; i < na; i += T) S[i] = ix[i];
    __syncthreads();
    big_bitonic(K + na, nbb, sb, sr, ss, ix);
    for (int i = tid; i < nbb; i += T) S[na + i] = na + ix[i];
    __syncthreads();
    const int32_t* A = S;
    const int32_t* B = S + na;
    const int k0 = (int)((int64_t)nb * tid / T), k1 = (int)((int64_t)nb * (tid + 1) / T);
    int lo = max(0, k0 - nbb), hi = min(k0, na);
    while (lo < hi) {  // co-rank: take i from A, k0 - i from B
      const int i = (lo + hi) >> 1;
      if (okless(K[A[i]], K[B[k0 - i - 1]])) lo = i + 1;
      else hi = i;
    }
    int i = lo, j = k0 - lo;
    for (int k = k0; k < k1; k++) {
      const bool takeA = j >= nbb || (i < na && okless(K[A[i]], K[B[j]]));
      out[k] = (int32_t)K[takeA ? A[i++] : B[j++]].id;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(1024) k_bucket_sort_big(const int32_t* bend, const int32_t* bcnt,
                                                          const int32_t* list, const int32_t* nlist,
                                                          const OKey* keys, OKey* tmp, int32_t* ids_out) {
  __shared__ uint64_t sb[BIG_SORT];
  __shared__ uint32_t sr[BIG_SORT], ss[BIG_SORT];
  __shared__ uint16_t ix[BIG_SORT];
  for (int li = blockIdx.x; li < *nlist; li += gridDim.x) {
    const int b = list[li];
    const int nb = bcnt[b];
    if (nb <= 512 || nb > 2 * BIG_SORT) continue;  // block-uniform
    bucket_sort_big_one(b, nb, bend, keys, tmp, ids_out, sb, sr, ss, ix);
  }
}

// A few buckets (an online call's one): both sorts in one launch of 1024-thread
// blocks, each bucket to the path its size takes, the two paths' LDS as one pool
// (one launch in place of k_bucket_sort + k_bucket_sort_big)
__global__ void __launch_bounds__(1024) k_bucket_sort_all(const int32_t* bend, const int32_t* bcnt,
                                                          const int32_t* list, const int32_t* nlist,
                                                          OKey* keys, OKey* tmp, int32_t* ids_out) {
  constexpr size_t BIG_LDS = (size_t)BIG_SORT * (8 + 4 + 4 + 2);
  constexpr size_t POOL = BIG_LDS > sizeof(SortChunk<SORT_CH>) ? BIG_LDS : sizeof(SortChunk<SORT_CH>);
  __shared__ __attribute__((aligned(16))) unsigned char pool[POOL];
  uint64_t* sb = (uint64_t*)pool;
  uint32_t* sr = (uint32_t*)(pool + (size_t)BIG_SORT * 8);
  uint32_t* ss = (uint32_t*)(pool + (size_t)BIG_SORT * 12);
  uint16_t* ix = (uint16_t*)(pool + (size_t)BIG_SORT * 16);
  SortChunk<SORT_CH>& sc = *(SortChunk<SORT_CH>*)pool;
  for (int li = blockIdx.x; li < *nlist; li += gridDim.x) {
    const int b = list[li];
    const int nb = bcnt[b];
    if (nb > 512 && nb <= 2 * BIG_SORT) bucket_sort_big_one(b, nb, bend, keys, tmp, ids_out, sb, sr, ss, ix);
    else bucket_sort_one(b, bend, bcnt, keys, tmp, ids_out, false, sc);
    __syncthreads();
  }
}

__global__ void k_scatter_und(const int32_t* cand, int ncand, const int32_t* f_und,
                              const int32_t* pos, int32_t* und) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= ncand || !f_und[q]) return;
  und[pos[q]] = cand[q];
}

__global__ void k_set_rr(Tables t, const int32_t* cand, int ncand, const int32_t* recv_call,
                         const int32_t* rr, const int64_t* cts, int32_t* ev_rr, int64_t* ev_cts,
                         unsigned long long* ntx_sum, int commit) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const bool rec = q < ncand && recv_call[q] >= 0;
  unsigned long long tx = 0;
  if (rec) {
    const int x = cand[q];
    ev_rr[x] = rr[q];
    ev_cts[x] = cts[q];
    tx = (unsigned long long)t.ntx[x];
  }
  if (!commit) return;
  // one atomic per wave
  for (int o = 32; o > 0; o >>= 1) tx += __shfl_xor(tx, o);
  if ((threadIdx.x & 63) == 0 && tx) atomicAdd(ntx_sum, tx);
}

// ---------------------------------------------------------------------------
// One hashgraph split across GPUs: part p commits the events its
// calls [c_lo, c_hi] receive.  A candidate received before c_lo is the previous
// part's (-2: neither ordered nor left here); one received after c_hi, or not at
// all, is left (-1).  A left candidate below `guard` (the next part's first
// candidate) is one no part covers: the flag makes the whole split fall back.
// ---------------------------------------------------------------------------
__global__ void k_split_filter(const int32_t* cand, int ncand, int32_t* recv_call, int c_lo, int c_hi,
                               int32_t guard, int32_t* flag) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  bool bad = false;
  if (q < ncand) {
    int rc = recv_call[q];
    if (rc >= 0 && rc < c_lo) rc = -2;
    else if (rc > c_hi) rc = -1;
    recv_call[q] = rc;
    bad = rc == -1 && cand[q] < guard;
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

// Slot of a part in the order exchange (int32 words): header [nord, nleft, flag,
// 0, ntx lo, ntx hi, 0, 0], the counts of its calls, then ids, rr, cts (int64)
// and the left (undetermined) ids, each region `cap` entries.
struct SplitSlot {
  int64_t counts, ids, rr, cts, left, words;
  __host__ __device__ static SplitSlot make(int ncalls_max, int64_t cap) {
    SplitSlot s;
    s.counts = 8;
    s.ids = (s.counts + ncalls_max + 1) & ~(int64_t)1;
    s.rr = s.ids + cap;
    s.cts = (s.rr + cap + 1) & ~(int64_t)1;
    s.left = s.cts + 2 * cap;
    s.words = (s.left + cap + 1) & ~(int64_t)1;
    return s;
  }
};

// pack this part's results into its slot (one grid over max(nord, nleft, ncalls));
// block 0 also sums the per-block transaction partials and writes the header
__global__ void k_split_pack(const int32_t* cnt, const int32_t* call_counts, int c_lo, int ncalls_p,
                             const int32_t* ids, const int32_t* left, const int32_t* ev_rr,
                             const int64_t* ev_cts, const unsigned long long* ntx_part, int ntxb,
                             const int32_t* flag, SplitSlot L, int32_t* slot) {
  const int nord = cnt[0], nleft = cnt[1];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nord; i += stride) {
    const int x = ids[i];
    slot[L.ids + i] = x;
    slot[L.rr + i] = ev_rr[x];
    ((int64_t*)(slot + L.cts))[i] = ev_cts[x];
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nleft; i += stride)
    slot[L.left + i] = left[i];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ncalls_p; i += stride)
    slot[L.counts + i] = call_counts[c_lo + i];
  if (blockIdx.x == 0) {
    __shared__ unsigned long long s_tx[256];
    unsigned long long tx = 0;
    for (int b = threadIdx.x; b < ntxb; b += blockDim.x) tx += ntx_part[b];
    s_tx[threadIdx.x] = tx;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long tot = 0;
      for (int k = 0; k < (int)blockDim.x; k++) tot += s_tx[k];
      slot[0] = nord;
      slot[1] = nleft;
      slot[2] = *flag;
      slot[3] = 0;
      slot[4] = (int32_t)(uint32_t)tot;
      slot[5] = (int32_t)(uint32_t)(tot >> 32);
      slot[6] = slot[7] = 0;
    }
  }
}

// every part's ordered ids into one list (part g's at off[g]) and their round
// received / consensus timestamp into the event tables
__global__ void k_split_unpack(const int32_t* buf, SplitSlot L, int nparts, const int64_t* off,
                               int32_t* ids_out, int32_t* ev_rr, int64_t* ev_cts) {
  const int g = blockIdx.y;
  const int32_t* slot = buf + (size_t)g * L.words;
  const int nord = slot[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nord;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int x = slot[L.ids + i];
    ids_out[off[g] + i] = x;
    ev_rr[x] = slot[L.rr + i];
    ev_cts[x] = ((const int64_t*)(slot + L.cts))[i];
  }
  (void)nparts;
}

// LastCommitedRoundEvents = RoundEvents(LCR-1) at the call that set LCR
// (hashgraph.go:666-673): events of round r minus those inserted after that
// call (ids >= n_from).  *out starts at 0.
__global__ void k_lcre(Tables t, int n_from, int n1, int r, int32_t* out) {
  const int x = n_from + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(out, t.rcnt[r]);
  if (x < n1 && t.round[x] == r) atomicSub(out, 1);
}

// k_lcre with the new LastConsensusRound L = flags[1] and its call flags[2] read
// on the device: nothing unless L > lcr_old; the blocks before the call's event
// count n_c stand down
__device__ __forceinline__ void lcre_dev_body(const Tables& t, const int64_t* nc, const int32_t* flags, int lcr_old,
                                              int n_lo, int n1, int32_t* out, int bid) {
  const int L = flags[1];
  if (L <= lcr_old || L < 1) return;
  const int r = L - 1;
  const int n_from = (int)min<int64_t>(nc[flags[2]], (int64_t)n1);
  if (bid == 0 && threadIdx.x == 0) atomicAdd(out, t.rcnt[r]);
  const int x = n_lo + bid * blockDim.x + threadIdx.x;
  if (x >= n_from && x < n1 && t.round[x] == r) atomicSub(out, 1);
}
// k_fame_persist (blocks [0, nb_fp)) and the LCR round count (lcre_dev_body, the rest) in one launch: the
// persisted fame and the LCR round's event count read and write disjoint tables
__global__ void k_fame_persist_lcre(Tables t, const int32_t* pr_round, const int32_t* pr_off, const int32_t* pr_cf,
                                    const int32_t* pr_len, int nrounds, const int32_t* clast, const uint8_t* dec,
                                    int nb_fp, const int64_t* nc, const int32_t* flags, int lcr_old, int n_lo,
                                    int n1, int32_t* out) {
  if ((int)blockIdx.x < nb_fp) fame_persist_body(t, pr_round, pr_off, pr_cf, pr_len, nrounds, clast, dec, blockIdx.x);
  else lcre_dev_body(t, nc, flags, lcr_old, n_lo, n1, out, blockIdx.x - nb_fp);
}

// An online call's DecideRoundReceived / FindOrder at N <= 16 in ONE launch (in place
// of k_segments_1p, k_round_received, k_recv_list_und, k_bucket_keys,
// k_bucket_sort_all and k_fame_persist_lcre): one block of 1024 threads, the stages
// behind block barriers, the same bodies as those kernels (one call that sees every
// event; the host checks the candidate count against the LDS scan and sort).  Wider
// hashgraphs (front = 0) run the segments, theta, round received and the median as
// their own grids and this kernel from the call's bucket on.
struct OrderCall {
  SegInfo si;  // segments
  int rr_lo, nr;
  const int32_t* segoff;
  int32_t *segcnt, *seg_call, *seg_round;
  uint8_t* seg_dec;
  uint64_t* seg_fws;
  int32_t* theta;
  const int32_t* cand;  // round received and the median
  int ncand, R_last;
  int32_t *recv, *rr;
  int64_t* cts;
  int32_t *cnt, *bpos, *total, *blist, *nblist;  // the call's bucket
  int32_t *f_und, *upos, *nund, *und_out;        // the new undetermined list
  OKey *k1, *k2;                                 // keys and the sort
  int32_t* ev_rr;
  int64_t* ev_cts;
  unsigned long long* ntx;
  int ntxb;
  int32_t* ids;
  const int32_t* pr;  // persisted fame (nrounds > 0) and the LCR round's count
  int nrounds;
  const int32_t* clast;
  const uint8_t* dec;
  const int64_t* nc;
  const int32_t* flags;
  int lcr_old, n_lo, n1;
  int32_t* lcre_out;
  int front;  // 1: the segments and round received here too (N <= 16); 0: from the stage kernels
};
constexpr size_t OC_BIG_LDS = (size_t)BIG_SORT * (8 + 4 + 4 + 2);
constexpr size_t OC_POOL = OC_BIG_LDS > sizeof(SortChunk<SORT_CH>) ? OC_BIG_LDS : sizeof(SortChunk<SORT_CH>);
static_assert(OC_POOL >= sizeof(int) * (SCAN_LDS + SCAN_LDS / 16), "the scan borrows the sort pool");
template <int G>
__device__ __forceinline__ void order_call_body(const Tables& t, const OrderCall& o, unsigned char* pool) {
  __shared__ int s_cnt;
  __shared__ unsigned long long s_tx[16];
  const int tid = threadIdx.x, T = blockDim.x;
  if (o.front) {
    // the round-state segments of the batch's rounds (theta inline)
    for (int64_t b = 0; b < (int64_t)o.nr * G; b += T)
      segments_group<G, 1>(t, b + tid, o.rr_lo, o.nr, 1, nullptr, o.si, o.segoff, o.segcnt, o.seg_call,
                           o.seg_round, o.seg_dec, o.seg_fws, o.theta);
    __syncthreads();
    // round received and the median timestamp (inline at N <= 16)
    for (int q = tid; q < o.ncand; q += T)
      round_received_item<1>(t, q, o.cand, o.ncand, nullptr, 1, 0, o.rr_lo, o.R_last, o.segoff, o.segcnt,
                             o.seg_call, o.seg_dec, o.seg_fws, o.theta, o.recv, o.rr, o.cts, nullptr);
  }
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  // the call's received count and its bucket (k_recv_list_und's block 0)
  int c = 0;
  for (int q = tid; q < o.ncand; q += T) c += o.recv[q] >= 0 ? 1 : 0;
  for (int s2 = 32; s2 > 0; s2 >>= 1) c += __shfl_xor(c, s2);
  if ((tid & 63) == 0 && c) atomicAdd(&s_cnt, c);
  for (int q = tid; q < o.ncand; q += T) o.f_und[q] = o.recv[q] == -1 ? 1 : 0;
  __syncthreads();
  if (tid == 0) o.cnt[0] = s_cnt;
  __syncthreads();
  bucket_list_body(o.cnt, 1, o.bpos, o.total, o.blist, o.nblist);
  __syncthreads();
  // the new undetermined list in candidate order (its block 1)
  scan_small_core(o.f_und, o.upos, o.ncand, o.nund, o.cand, o.und_out, (int*)pool);
  __syncthreads();
  // keys into the bucket, the transactions summed
  unsigned long long tx = 0;
  for (int b = 0; b < o.ncand; b += T)
    tx += bucket_key_item(t, b + tid, o.cand, o.ncand, o.recv, o.rr, o.cts, o.bpos, o.k1, o.ev_rr, o.ev_cts);
  if ((tid & 63) == 0) s_tx[tid >> 6] = tx;
  __syncthreads();
  if (tid == 0) {
    unsigned long long bt = 0;
    for (int w = 0; w < T / 64; w++) bt += s_tx[w];
    o.ntx[0] = bt;
  }
  for (int i = 1 + tid; i < o.ntxb; i += T) o.ntx[i] = 0;
  __syncthreads();
  // the sort (k_bucket_sort_all's path for the bucket's size)
  {
    uint64_t* sb = (uint64_t*)pool;
    uint32_t* sr = (uint32_t*)(pool + (size_t)BIG_SORT * 8);
    uint32_t* ss = (uint32_t*)(pool + (size_t)BIG_SORT * 12);
    uint16_t* ix = (uint16_t*)(pool + (size_t)BIG_SORT * 16);
    SortChunk<SORT_CH>& sc = *(SortChunk<SORT_CH>*)pool;
    const int nl = *o.nblist;
    for (int li = 0; li < nl; li++) {
      const int b = o.blist[li];
      const int nb = o.cnt[b];
      if (nb > 512 && nb <= 2 * BIG_SORT) bucket_sort_big_one(b, nb, o.bpos, o.k1, o.k2, o.ids, sb, sr, ss, ix);
      else bucket_sort_one(b, o.bpos, o.cnt, o.k1, o.k2, o.ids, false, sc);
      __syncthreads();
    }
  }
  // the persisted fame, read above by the segments as it was before this call, and
  // RoundEvents(LCR - 1) (k_fame_persist_lcre)
  if (o.nrounds > 0) {
    const int np = o.nrounds;
    for (int b = 0; (int64_t)b * T < (int64_t)np * t.N; b++)
      fame_persist_body(t, o.pr, o.pr + np, o.pr + 2 * np, o.pr + 3 * np, np, o.clast, o.dec, b);
    for (int b = 0; b == 0 || b * T < o.n1 - o.n_lo; b++)
      lcre_dev_body(t, o.nc, o.flags, o.lcr_old, o.n_lo, o.n1, o.lcre_out, b);
  }
}
template <int G>
__global__ void __launch_bounds__(1024) k_order_call(Tables t, OrderCall o) {
  __shared__ __attribute__((aligned(16))) unsigned char pool[OC_POOL];
  order_call_body<G>(t, o, pool);
}
// the whole consensus part of an online call at N <= 16 in one launch: DecideFame,
// LCR and the header (fame_call_body), then the order (order_call_body, front = 1)
template <int G>
__global__ void __launch_bounds__(1024) k_consensus_call(Tables t, FameCall f, OrderCall o) {
  __shared__ __attribute__((aligned(16))) unsigned char pool[OC_POOL];
  fame_call_body<G, 1, true>(t, f);
  __syncthreads();  // decisions, LCR and the header (global) are visible to the block
  order_call_body<G>(t, o, pool);
}

// An online call's consensus at N <= 16 with its control built on the device
// (k_consensus_call's stages after a prologue): the round count and the candidates'
// lowest round are read where the rounds walk left them (rstate, minw[Rcap + 2]), so
// the host enqueues the whole call without a round trip in the middle.  The single
// call's DecideFame windows are one pair per round lcr+1 .. R-2 (consensus_batch's
// enumeration for one call); the rounds DecideRoundReceived examines are
// [mnr + 1, R), with their segment capacities.  Buffers are sized by the host from
// R <= R_before + new events.
struct DynCall {
  int lcr, ncand, Rcap;
  int64_t n_c;
  const int32_t* rstate;
  const int32_t* minw;
  int64_t* c_nc;
  int32_t *c_Rc, *c_Lc, *c_flags, *c_pr, *c_pidx, *c_sgo;
  uint8_t *dec, *decbit;
  int32_t *LCR, *clast, *out;
  OrderCall o;  // buffers; its round scalars and control pointers are filled here
};
template <int G>
__global__ void __launch_bounds__(1024) k_consensus_dyn(Tables t, DynCall dc) {
  __shared__ __attribute__((aligned(16))) unsigned char pool[OC_POOL];
  __shared__ int s_R, s_rrlo, s_nr, s_nround;
  const int tid = threadIdx.x, T = blockDim.x, N = t.N;
  if (tid == 0) {
    const int R = dc.rstate[0];
    const int mnr = dc.minw[dc.Rcap + 2];
    const int rr_lo = mnr >= INF32 - 1 ? INF32 : mnr + 1;  // (INF32: no candidate)
    s_R = R;
    s_rrlo = rr_lo;
    s_nr = max(0, R - rr_lo);
    s_nround = max(0, R - 2 - dc.lcr);
    dc.c_nc[0] = dc.n_c;
    dc.c_Rc[0] = R;
    dc.c_Lc[0] = -1;
    for (int i = 0; i < 4; i++) dc.c_flags[i] = 0;
  }
  __syncthreads();
  const int R = s_R, rr_lo = s_rrlo, nr = s_nr, nround = s_nround;
  int32_t* pr = dc.c_pr;
  for (int k = tid; k < nround; k += T) {
    pr[k] = dc.lcr + 1 + k;
    pr[nround + k] = k;
    pr[2 * nround + k] = 0;
    pr[3 * nround + k] = 1;
  }
  for (int q = tid; q < nr; q += T) {
    const int k = rr_lo + q - (dc.lcr + 1);
    dc.c_pidx[q] = k >= 0 && k < nround ? k : -1;
  }
  __syncthreads();
  if (tid == 0) {
    int slot = 0;
    for (int q = 0; q < nr; q++) {
      dc.c_sgo[q] = slot;
      slot += N + 2 + (dc.c_pidx[q] >= 0 ? 1 : 0);
    }
    dc.c_sgo[nr] = slot;
  }
  __syncthreads();
  FameCall f{};
  f.pr_round = pr;
  f.pr_off = pr + nround;
  f.pr_cf = pr + 2 * nround;
  f.pr_len = pr + 3 * nround;
  f.nrounds = nround;
  f.npairs = nround;
  f.nc = dc.c_nc;
  f.Rc = dc.c_Rc;
  f.dec = dc.dec;
  f.decbit = dc.decbit;
  f.Lc = dc.c_Lc;
  f.ncalls = 1;
  f.lcr_start = dc.lcr;
  f.LCR = dc.LCR;
  f.clast = dc.clast;
  f.flags = dc.c_flags;
  f.out = dc.out;
  f.nout = 9;
  if (nround > 0) {
    fame_call_body<G, 1, true>(t, f);
  } else {
    for (int i = tid; i < 9; i += T) dc.out[i] = i == 3 ? dc.lcr : 0;  // no new LastConsensusRound
  }
  __syncthreads();
  OrderCall o = dc.o;
  o.rr_lo = rr_lo;
  o.nr = nr;
  o.R_last = R;
  o.segoff = dc.c_sgo;
  o.si.pr_index = dc.c_pidx;
  o.si.pr_off = nround ? pr + nround : nullptr;
  o.si.pr_cf = nround ? pr + 2 * nround : nullptr;
  o.si.pr_len = nround ? pr + 3 * nround : nullptr;
  o.si.clast = nround ? dc.clast : nullptr;
  o.si.dec = nround ? dc.dec : nullptr;
  o.pr = pr;
  o.nrounds = nround;
  o.clast = dc.clast;
  o.dec = dc.dec;
  o.flags = dc.c_flags;
  o.nc = dc.c_nc;
  o.front = nr > 0 ? 1 : 0;
  if (nr == 0)
    for (int q = tid; q < o.ncand; q += T) o.recv[q] = -1;  // no round can receive
  order_call_body<G>(t, o, pool);
}

// fresh consensus state: C = INF, W = -1, bitsets / fame / counts = 0, rr = -1
__global__ void k_reset_rounds(Tables t, int64_t nrow, int64_t nbits, int64_t nev,
                               int32_t* rr) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrow; i += stride) {
    t.C[i] = INF32;
    t.W[i] = -1;
    t.fame[i] = 0;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbits; i += stride) {
    t.ssb[i] = 0;
    t.seeb[i] = 0;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nev; i += stride) rr[i] = -1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.Rcap; i += stride)
    t.rcnt[i] = 0;
}

// ---------------------------------------------------------------------------
// MedianTimestamp's source (hashgraph.go:762-770): the event whose Body.Timestamp
// becomes x's consensus timestamp.  The candidates are OldestSelfAncestorToSee(w, x)
// = (d, FD[x][d]) for the famous witnesses w = W[rr][d] of x's round received that
// see x (hashgraph.go:704-709); the source is one whose timestamp is the median.
// Several may share that instant in different zones: Go's sort.Sort over a list
// built in map order leaves which one lands at len/2 unspecified, and the lowest
// creator d is returned here.  Fame of a round at or below LastConsensusRound is
// final, so the persisted fame table gives the set the median used.  One wave per
// event, lane = d; -1 for an event with no round received.
__global__ void __launch_bounds__(256) k_cts_source(Tables t, const int32_t* ids, int n, const int32_t* rr,
                                                    const int64_t* cts, int32_t* out) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= n) return;  // wave-uniform
  const int x = ids[q];
  const int r = rr[x];
  int src = -1;
  if (r >= 0) {
    const int cx = t.creator[x], ix = t.index[x];
    const int64_t c = cts[x];
    for (int d0 = 0; d0 < t.N; d0 += 64) {
      const int d = d0 + lane;
      bool hit = false;
      int p = 0;
      if (d < t.N) {
        const int w = t.W[(size_t)r * t.N + d];
        if (w >= 0 && t.fame[(size_t)r * t.N + d] == 1 && la_at(t, d, t.index[w], cx) >= ix) {
          p = fd_at(t, (size_t)cx * t.ccap + ix, d);
          hit = p != INF32 && t.tsch[(size_t)d * t.ccap + p] == c;
        }
      }
      const uint64_t b = __ballot(hit);
      if (b) {
        const int l = __ffsll((unsigned long long)b) - 1;
        src = t.chain[(size_t)(d0 + l) * t.ccap + __shfl(p, l)];
        break;
      }
    }
  }
  if (lane == 0) out[q] = src;
}

}  // namespace hge
