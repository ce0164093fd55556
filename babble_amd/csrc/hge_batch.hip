// hge_batch.hip — many independent small hashgraphs replayed together
// (BASELINE config 5: a Monte Carlo batch of 32-participant graphs with
// Byzantine forkers).  C ABI: hge_batch_* in include/hge.h.
//
// The single-graph engine (hge_engine.hip) sizes its grids from one graph and
// makes a few host round trips per replay; driving 1,024 of them means ~50k
// launches per batch from host threads (58M ev/s, the
// host bound).  Here every stage is ONE launch over the whole batch, and the
// graph's whole call schedule runs inside the consensus kernel:
//
//   kb_coords     lastAncestors rows in insertion order (hashgraph.go:399-463), one
//                 256-thread workgroup per graph: runs of mutually independent
//                 events computed together, a row the max of its parents' rows
//                 (from an LDS ring of the chunk or a snapshot of the chain heads).
//   kb_fd         firstDescendants in run layout FDT[j][c][p], one wave per (graph,
//                 chain j): chain-j event k is the first chain-j descendant of
//                 chain-c positions (LA[(j,k-1)][c], LA[(j,k)][c]] (hashgraph.go:466-494);
//   kb_fdrows     ... transposed to rows FD[c][p][j] through LDS tiles.
//   kb_front      Round / Witness of every event (hashgraph.go:220-305) by the round
//                 frontier: C_{r+1}[c] = the SM-th smallest over the round-r
//                 members d of the first position of chain c that strongly sees d,
//                 one 1024-thread workgroup per graph; each witness's strongly-see /
//                 see bitsets over the previous round's witnesses (the vote adjacency
//                 of DecideFame).
//   kb_consensus  for every call point in order, one 4-wave workgroup per graph:
//                 DivideRounds' bookkeeping, DecideFame (hashgraph.go:598-664: lane
//                 = voter y, witnesses x over the waves, a vote set a 64-bit mask,
//                 the `break` as the first y whose tally reaches SM, missing votes as
//                 nays, coin rounds), DecideRoundReceived (hashgraph.go:676-721: x is
//                 seen by more than half of the famous witnesses iff index(x) <=
//                 theta(round, creator(x)), the (|F|/2+1)-th largest lastAncestor of
//                 the famous witnesses), MedianTimestamp (:762-770) and the
//                 ConsensusSorter sort of the call's batch (consensus_sorter.go:36-59,
//                 PRN = 0) in LDS.
//
// Everything on the path is integer; results are bit-exact with the oracle
// (tests/test_gpu_batch.py, tests/test_gpu_mc.py: every graph's full-state digest).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hge.h"

namespace hgb {

constexpr int32_t INF = 0x7fffffff;

struct GDesc {
  int64_t eo;    // first event of the graph in the per-event pools
  int32_t E;     // accepted events
  int32_t co;    // first call in the per-call pools
  int32_t K;     // calls
  int32_t ro;    // first round row in the per-round pools
  int32_t Rcap;  // rounds the graph may reach (E / SM + 2)
  int32_t pad;
};

// batch tables (device pointers); per-graph blocks are addressed through GDesc
struct BT {
  int N, SM, ccap;
  const GDesc* gd;
  const int32_t *cr, *ix, *sp, *op, *oc, *ntx, *clen;  // oc: the other-parent's creator
  const int64_t* ts;
  const uint64_t* S;  // 4 limbs per event, most significant first
  const uint8_t* coin;
  const int32_t* chain;  // [g][N][ccap] local event ids
  const int64_t* tsch;   // [g][N][ccap] timestamps in chain layout
  const int64_t* calls;  // accepted-event count at each call point
  int32_t* LA;           // [eo + x][N] lastAncestors (positions; -1 none)
  int32_t* FDT;          // [g][j][c][ccap] firstDescendants in run layout (INF none)
  int32_t* FD;           // [g][c][p][N] firstDescendants rows of chain positions (INF none)
  const uint64_t* Sch;   // [g][c][p] limb 0 of S in chain layout (the sort key)
  const int32_t* ntxch;  // [g][c][p] transaction counts in chain layout
  int32_t* round;
  uint8_t* wit;
  int32_t* rr;
  int64_t* cts;
  int32_t *W, *WIX, *WFD;      // [ro + r][N] witness id / its index, [ro + r][N][N] its FD row
  uint8_t* WCOIN;              // [ro + r][N] the witness's coin (middleBit)
  uint64_t *ssb, *seeb;        // [ro + r][N] bitsets over round r-1's witness creators
  int8_t* fame;                // [ro + r][N] 0 undefined, 1 true, 2 false (persisted)
  int32_t *rcnt, *ver, *thv;   // [ro + r] events in the round so far, fame/witness version, theta's version
  int32_t* th;                 // [ro + r][N] receive thresholds
  int32_t *U, *Ur, *Ucp;       // [eo + k] undetermined list past LDS: id, round, creator << 24 | index
  int32_t* order;              // [eo + k] consensus order
  int64_t* counts;             // [co + c] batch size of call c
  int64_t* scal;               // [g][8] R, LCR, LCRE, transactions, ordered, undetermined, error
  int32_t* krr;                // [2 eo + k] sort scratch for call batches past the LDS keys
  int64_t* kct;
  uint64_t* ks0;
  int32_t* kid;
  uint64_t* dbg;               // diagnostics: per-graph section cycles (null: off)
  // the bulk call schedule (hge_batch_bulk.hip)
  const int32_t* glist;  // kb_consensus: the graphs it replays (null: every graph)
  const int32_t* cg;     // [co + c] the graph of each call
  int32_t *Rc, *xcall;   // [co + c] Rounds() after call c's DivideRounds; [eo + x] x's insertion call
  int32_t* rfirst;       // [ro + r] the first call with R_c >= r (r <= the last call's R)
  uint64_t* arr;         // [eo + k] the witnesses in insertion order: call << 32 | round << 8 | creator
  uint64_t* Dp;          // [((co + c) * NS + s) * 2 + {0, 1}], NS <= BNS DecideFame's decided / famous masks
  int32_t* gx;           // [g][16] per-graph internals (GX_*)
  int4* ivh;             // [(ro + r) * BVCAP + k] receive intervals: first call, end call, theta slot
  uint64_t* ivF;         // ... and their famous witnesses
  int32_t *nivl, *fsuf;  // [ro + r] intervals per round; the suffix minimum of their first starts
  int32_t *thp, *thR;    // [g * BICAP + s][N] receive thresholds; [g * BICAP + s] their round
  uint64_t* thF;         // [g * BICAP + s] their famous witnesses
  // chain layout [g][c][p] (kb_receive's lanes are consecutive positions of a chain)
  int32_t* roundch;      // rounds
  int32_t *rcall, *rrank;  // the call that receives the event (-1 none), its slot in that call's bucket
  int32_t* rrch;         // round received
  int32_t* rslot;        // the receiving interval's threshold slot (-1 none)
  int64_t* ctsch;        // consensus timestamps
  int32_t *bcnt, *boff;  // [co + c] call buckets: size, offset
  int4* wl;              // the non-empty buckets (graph, size, offset in the graph's order)
  int32_t* wlc;          // their count
  int64_t* gctx;         // [g] ConsensusTransactions
  int2* cinf;            // [eo + x] kb_levels' records for kb_coords
};

__device__ __forceinline__ int rl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return (uint64_t)hi << 32 | lo;
}
__device__ __forceinline__ int64_t rl64s(int64_t v, int l) { return (int64_t)rl64((uint64_t)v, l); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int wave_max(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_min(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
// mutable per-graph state in global memory is written and read by different
// lanes of the graph's wave: device-coherent loads bypass a stale L1 line
template <typename T>
__device__ __forceinline__ T ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, typename V>
__device__ __forceinline__ void st(T* p, V v) {
  __hip_atomic_store(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wsync() { __builtin_amdgcn_wave_barrier(); }
// a workgroup barrier ordering LDS accesses only: no wait for outstanding global stores
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ---------------------------------------------------------------------------
// A graph's work is a dependent chain (insertion order, rounds, the call schedule),
// so each kernel below gives one graph one workgroup and hides its latency inside
// it: the chain's independent steps spread over the waves, the next chunk's loads
// issued before the current one is consumed, and the consensus kernel's state of
// the last RW rounds (witnesses, vote bitsets, fame, thresholds) and the
// undetermined list kept in LDS.

// lastAncestors (InitEventCoordinates, hashgraph.go:399-463): in insertion order,
// LA[x] = max(LA[sp], LA[op]) with LA[x][creator] = index.  The events go in chunks of
// 64.  kb_levels gives every event of every chunk, all graphs at once, its level inside
// its chunk (one above its in-chunk parents) and its parents' row sources; kb_coords
// (one workgroup per graph) then walks the chunks, one step per level.
//
// kb_levels: one wave per (graph, chunk), lane = event.  A parent's row source is a
// row of the chunk's LDS ring (the parent is in the chunk), the chain head as of the
// chunk's start (the parent is its chain's last event before the chunk: the
// self-parent always is, admission "Self-parent not last known", hashgraph.go:390-393,
// and the other-parent nearly always), or HBM.  cinf[x] = {srcA | srcB << 8 |
// level << 16 | last << 23 | levels << 24, creator | index << 8}; last: x is its
// chain's last event in the chunk (its row becomes that chain's head).
__global__ __launch_bounds__(256) void kb_levels(BT t) {
  const int g = blockIdx.y, lane = threadIdx.x & 63;
  const GDesc d = t.gd[g];
  const int base = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (base >= d.E) return;
  const int N = t.N, cc = t.ccap, i = base + lane;
  const bool on = i < d.E;
  const int sp = on ? t.sp[d.eo + i] : -1, op = on ? t.op[d.eo + i] : -1;
  const int cr = on ? t.cr[d.eo + i] : 0, oc = on ? t.oc[d.eo + i] : 0, ix = on ? t.ix[d.eo + i] : 0;
  const int32_t* chg = t.chain + (int64_t)g * N * cc;
  const int32_t* lng = t.clen + (int64_t)g * N;
  // the event after position q of chain c (INF: none)
  auto next = [&](int c, int q) { return q + 1 < lng[c] ? chg[(int64_t)c * cc + q + 1] : INF; };
  auto src = [&](int p, int c) -> int {
    if (p < 0) return -1;
    if (p >= base) return p - base;
    return next(c, t.ix[d.eo + p]) >= base ? 64 + c : -2;
  };
  const int sa = src(sp, cr), sb = src(op, oc);
  const bool last = on && next(cr, ix) >= base + 64;
  const int ps = on && sp >= base ? sp - base : -1, po = on && op >= base ? op - base : -1;
  int lvl = 0;
  while (true) {  // parents precede their children: settles after the chunk's depth
    const int x = __shfl(lvl, ps < 0 ? 0 : ps), y = __shfl(lvl, po < 0 ? 0 : po);
    const int nl = max(ps >= 0 ? x + 1 : 0, po >= 0 ? y + 1 : 0);
    const bool ch = nl != lvl;
    lvl = nl;
    if (!ballot(ch)) break;
  }
  const int nlev = wave_max(on ? lvl : 0) + 1;
  if (on)
    t.cinf[d.eo + i] = make_int2((sa & 0xFF) | (sb & 0xFF) << 8 | lvl << 16 | (last ? 1 << 23 : 0) | nlev << 24,
                                 cr | ix << 8);
}

// kb_coords: one workgroup per graph (SPLIT = 1) or per (graph, 1/SPLIT of the columns:
// every column's recurrence is independent of the others), NT threads; thread (s, k) owns column k of the
// chunk's events s, s + SL, ... (SL = NT / NM), their kb_levels records in registers
// (the next chunk's loaded while this one runs).  A step computes one level: every
// event of it reads its parents' rows from LDS (ring or heads) or HBM and writes its
// own; one LDS-scoped barrier per step (the row stores to HBM are never waited for
// inside a chunk).  After the chunk the chains' last events' rows become the heads,
// behind a full barrier (which also completes the chunk's HBM stores).
// LV = false (past two graphs per CU: the chip is full, and kb_levels' extra pass
// measured 1.04 -> 1.42 ms at 1,024 graphs), the earlier form: wave 0 levels each chunk
// itself, and a step computes up to SL events of one level together (their rows depend
// only on rows already final).  The parents' row sources are found the same way (the
// heads' ids kept in LDS); wave 0 loads the next chunk's event records while this
// chunk's steps run.
template <int NM, int NT, bool LV, int SPLIT = 1>
__global__ __launch_bounds__(NT) void kb_coords(BT t) {
  if constexpr (LV) {
  constexpr int CPW = NM / SPLIT, SL = NT / CPW, EPT = 64 / SL;
  static_assert(EPT >= 1 && SL * EPT == 64, "slots tile the chunk");
  const GDesc d = t.gd[blockIdx.x / SPLIT];
  const int part = blockIdx.x % SPLIT;
  const int N = t.N, tid = threadIdx.x, s = tid / CPW, kl = tid - (tid / CPW) * CPW, k = part * CPW + kl;
  // rows 0..63: the chunk's ring; 64 + c: chain c's head row as of the chunk's start
  // (this workgroup's CPW columns: the recurrence is column by column)
  __shared__ int32_t rows[64 + NM][CPW];
  for (int i = tid; i < NM * CPW; i += NT) rows[64 + i / CPW][i - (i / CPW) * CPW] = -1;
  __syncthreads();
  int32_t* LA = t.LA + d.eo * N;
  const int2* ci = t.cinf + d.eo;
  int2 nx[EPT];
  int nlv = 0;
  auto fetch = [&](int b) {
#pragma unroll
    for (int u = 0; u < EPT; u++) {
      const int e = b + s + SL * u;
      nx[u] = e < d.E ? ci[e] : make_int2(0, 0);
    }
    nlv = b < d.E ? ci[b].x >> 24 : 0;  // the chunk's level count (its first event's record)
  };
  fetch(0);
  for (int base = 0; base < d.E; base += 64) {
    int2 in[EPT];
#pragma unroll
    for (int u = 0; u < EPT; u++) in[u] = nx[u];
    const int nlev = nlv;
    if (base + 64 < d.E) fetch(base + 64);
    int val[EPT];
    for (int l = 0; l < nlev; l++) {
#pragma unroll
      for (int u = 0; u < EPT; u++) {
        const int e = s + SL * u;
        if (base + e < d.E && k < N && ((in[u].x >> 16) & 63) == l) {
          const int sa = (int)(int8_t)(in[u].x & 0xFF), sb = (int)(int8_t)((in[u].x >> 8) & 0xFF);
          const int a = sa >= 0 ? rows[sa][kl] : sa == -1 ? -1 : ld(&LA[(int64_t)t.sp[d.eo + base + e] * N + k]);
          const int b = sb >= 0 ? rows[sb][kl] : sb == -1 ? -1 : ld(&LA[(int64_t)t.op[d.eo + base + e] * N + k]);
          const int v = k == (in[u].y & 0xFF) ? in[u].y >> 8 : max(a, b);
          val[u] = v;
          rows[e][kl] = v;
          LA[(int64_t)(base + e) * N + k] = v;
        }
      }
      lds_barrier();
    }
    // the heads after the chunk (every read of the old heads is behind the last barrier)
#pragma unroll
    for (int u = 0; u < EPT; u++)
      if (base + s + SL * u < d.E && k < N && (in[u].x >> 23 & 1)) rows[64 + (in[u].y & 0xFF)][kl] = val[u];
    __syncthreads();  // also: the chunk's row stores are complete before the next one reads HBM
  }
  } else {
  constexpr int SL = NT / NM;  // event slots per step
  const GDesc d = t.gd[blockIdx.x];
  const int N = t.N, tid = threadIdx.x, s = tid / NM, k = tid - (tid / NM) * NM;
  // rows 0..63: the chunk's ring; 64 + c: chain c's head row as of the chunk's start
  __shared__ int32_t rows[64 + NM][NM];
  __shared__ int32_t headid[NM];
  // per event of the chunk: its parents' row sources (a row of `rows`, -1 none,
  // -2 HBM), creator, index; the parents' ids for the HBM case
  __shared__ int4 einfo[64];
  __shared__ int32_t msp[64], mop[64];
  __shared__ int32_t ord[64];     // the chunk's events by level
  __shared__ int32_t gst[130];    // the steps: ord[gst[i] .. gst[i + 1])
  __shared__ int32_t clast[NM];   // the chunk's last event per chain (-1)
  __shared__ int s_ng;
  for (int i = tid; i < NM * NM; i += NT) rows[64 + i / NM][i - (i / NM) * NM] = -1;
  if (tid < NM) headid[tid] = -1;
  __syncthreads();
  int32_t* LA = t.LA + d.eo * N;
  // wave 0 holds the next chunk's event records (loaded while this chunk's steps run)
  int nsp = -1, nop = -1, ncr = 0, noc = 0, nix = 0;
  auto fetch = [&](int b) {
    const int i = b + tid;
    const bool on = i < d.E;
    nsp = on ? t.sp[d.eo + i] : -1;
    nop = on ? t.op[d.eo + i] : -1;
    ncr = on ? t.cr[d.eo + i] : 0;
    noc = on ? t.oc[d.eo + i] : 0;
    nix = on ? t.ix[d.eo + i] : 0;
  };
  if (tid < 64) fetch(0);
  for (int base = 0; base < d.E; base += 64) {
    const int cnt = min(64, d.E - base);
    if (tid < 64) {
      const int sp = nsp, op = nop, cr = ncr, oc = noc;
      const bool on = base + tid < d.E;
      auto src = [&](int p, int c) -> int {
        return p < 0 ? -1 : p >= base ? p - base : headid[c] == p ? 64 + c : -2;
      };
      einfo[tid] = make_int4(src(sp, cr), src(op, oc), cr, nix);
      msp[tid] = sp;
      mop[tid] = op;
      if (tid < NM) clast[tid] = -1;
      wsync();
      if (on) atomicMax(&clast[cr], tid);
      // levels inside the chunk: one above the in-chunk parents (parents precede
      // their children, so the passes settle after the chunk's depth); the events of
      // a level are independent and take the steps of that level, SL at a time
      const int ps = on && sp >= base ? sp - base : -1, po = on && op >= base ? op - base : -1;
      int lvl = 0;
      while (true) {
        const int a = __shfl(lvl, ps < 0 ? 0 : ps), b = __shfl(lvl, po < 0 ? 0 : po);
        const int nl = max(ps >= 0 ? a + 1 : 0, po >= 0 ? b + 1 : 0);
        const bool ch = nl != lvl;
        lvl = nl;
        if (!ballot(ch)) break;
      }
      const int maxl = wave_max(on ? lvl : 0);
      const uint64_t below = tid ? (~0ull >> (64 - tid)) : 0ull;
      int pos = 0, ng = 0;
      for (int l = 0; l <= maxl; l++) {
        const uint64_t m = ballot(on && lvl == l);
        const int c_l = __popcll(m);
        if (on && lvl == l) ord[pos + __popcll(m & below)] = tid;
        for (int q = 0; q < c_l; q += SL) {
          if (tid == 0) gst[ng] = pos + q;
          ng++;
        }
        pos += c_l;
      }
      if (tid == 0) {
        gst[ng] = cnt;
        s_ng = ng;
      }
      if (base + 64 < d.E) fetch(base + 64);
    }
    __syncthreads();
    const int ng = s_ng;
    for (int gi = 0; gi < ng; gi++) {
      const int q0 = gst[gi], q1 = gst[gi + 1];
      const bool on = q0 + s < q1 && k < N;
      if (on) {
        const int e = ord[q0 + s];
        const int4 ei = einfo[e];
        const int a = ei.x >= 0 ? rows[ei.x][k] : ei.x == -1 ? -1 : ld(&LA[(int64_t)msp[e] * N + k]);
        const int b = ei.y >= 0 ? rows[ei.y][k] : ei.y == -1 ? -1 : ld(&LA[(int64_t)mop[e] * N + k]);
        const int val = k == ei.z ? ei.w : max(a, b);
        rows[e][k] = val;
        LA[(int64_t)(base + e) * N + k] = val;
      }
      lds_barrier();
    }
    // the heads after the chunk
    if (k < N)
      for (int c = s; c < N; c += SL) {
        const int l = clast[c];
        if (l >= 0) rows[64 + c][k] = rows[l][k];
      }
    if (tid < N && clast[tid] >= 0) headid[tid] = base + clast[tid];
    __syncthreads();  // also: the chunk's row stores are complete before the next one reads HBM
  }
  }
}


// The per-replay resets of the pooled tables in one launch (14 stream fills cost ~5 µs
// of launch each, ~70 µs of a 128-graph replay): segment k gets its 4-byte pattern,
// 16-byte stores over its whole 16-byte units, then the tail bytes.
struct ClrSeg {
  void* p;
  uint64_t bytes;
  uint32_t pat;
};
struct ClrList {
  ClrSeg s[16];
  int n;
};
__global__ __launch_bounds__(256) void kb_clear(ClrList L) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
  for (int k = 0; k < L.n; k++) {
    const ClrSeg sg = L.s[k];
    const uint64_t n16 = sg.bytes >> 4;
    const uint4 v = make_uint4(sg.pat, sg.pat, sg.pat, sg.pat);
    uint4* q = (uint4*)sg.p;
    for (uint64_t i = tid; i < n16; i += nth) q[i] = v;
    for (uint64_t b = (n16 << 4) + tid; b < sg.bytes; b += nth) ((uint8_t*)sg.p)[b] = (uint8_t)sg.pat;
  }
}

// ---------------------------------------------------------------------------
// firstDescendants in run layout (UpdateAncestorFirstDescendant, hashgraph.go:466-494):
// chain-j event k is the first chain-j descendant of the chain-c positions
// (LA[(j,k-1)][c], LA[(j,k)][c]]; positions no chain-j event sees keep INF
// (MaxInt64).  One wave per (graph, chain j, slice of FCW columns): lane r holds row
// k0 + r of chain j (the slice's columns, registers); for each column c the 64 rows'
// runs tile one contiguous range of chain c's positions, so the stores of a column
// are contiguous across the lanes.  The next 64 rows' loads are in flight meanwhile.
// (Slices of 16 columns: a wave holding all 32 columns took 176 VGPRs, two waves per SIMD.)
constexpr int FCW = 16;
template <int NM>
__global__ __launch_bounds__(64 * (NM / FCW)) void kb_fd(BT t) {
  constexpr int NS_ = NM / FCW;
  // a (graph, chain) per workgroup, one wave per slice: the slices read the same LA rows
  // (one 128-byte line at N = 32) together on one CU instead of on two XCDs
  const int N = t.N, cc = t.ccap, lane = threadIdx.x & 63;
  const int w = blockIdx.x * NS_ + (threadIdx.x >> 6), g = w / (N * NS_), j = (w / NS_) % N, c0 = (w % NS_) * FCW;
  if (c0 >= N) return;
  const GDesc d = t.gd[g];
  const int32_t* LA = t.LA + d.eo * N;
  const int lenc = lane < N ? t.clen[g * N + lane] : 0;  // lane c's chain length (the INF tails)
  {
    const int lenj = t.clen[g * N + j];
    const int32_t* ch = t.chain + ((int64_t)g * N + j) * cc;
    int32_t* outj = t.FDT + ((int64_t)g * N + j) * N * cc;  // + c * cc + p
    const bool vec = (N & 3) == 0 && c0 + FCW <= N;  // 16-byte aligned slices
    int row[FCW], nrow[FCW];
    int carry[FCW];  // the last row's value of column c0 + c before the chunk (uniform)
#pragma unroll
    for (int c = 0; c < FCW; c++) carry[c] = -1;
    auto load = [&](int k0, int (&v)[FCW]) {
      const bool ok = k0 + lane < lenj;
      const int x = ok ? ch[k0 + lane] : 0;
      const int32_t* r = LA + (int64_t)x * N + c0;
      if (vec) {
#pragma unroll
        for (int c = 0; c < FCW; c += 4) {
          const int4 q = ok ? *(const int4*)(r + c) : make_int4(-1, -1, -1, -1);
          v[c] = q.x;
          v[c + 1] = q.y;
          v[c + 2] = q.z;
          v[c + 3] = q.w;
        }
      } else {
#pragma unroll
        for (int c = 0; c < FCW; c++) v[c] = ok && c0 + c < N ? r[c] : -1;
      }
    };
    if (lenj > 0) load(0, row);
    for (int k0 = 0; k0 < lenj; k0 += 64) {
      const bool more = k0 + 64 < lenj;
      if (more) load(k0 + 64, nrow);
      const bool ok = k0 + lane < lenj;
      const int last = min(64, lenj - k0) - 1;  // the chunk's last valid lane
#pragma unroll
      for (int c = 0; c < FCW; c++) {
        if (c0 + c < N) {
          const int up = __shfl_up(row[c], 1);
          const int a = lane == 0 ? carry[c] : up;  // positions (a, b] take k0 + lane
          const int b = ok ? row[c] : a;
          int32_t* out = outj + (int64_t)(c0 + c) * cc;
          for (int p = a + 1; p <= b; p++) out[p] = k0 + lane;
          carry[c] = rl(row[c], last);
        }
      }
      if (more) {
#pragma unroll
        for (int c = 0; c < FCW; c++) row[c] = nrow[c];
      }
    }
    // chain c's positions no chain-j event sees: one coalesced sweep per column
#pragma unroll
    for (int c = 0; c < FCW; c++) {
      if (c0 + c < N) {
        const int lc = rl(lenc, c0 + c);
        int32_t* out = outj + (int64_t)(c0 + c) * cc;
        for (int p = carry[c] + 1 + lane; p < lc; p += 64) out[p] = INF;
      }
    }
  }
}

// firstDescendants as rows in chain layout: FD[g][c][p][j] = FDT[j][c][p], through an
// LDS tile of 64 positions x N chains per step.  One workgroup per (graph, chain c).
template <int NM>
__global__ __launch_bounds__(256) void kb_fdrows(BT t) {
  const int g = blockIdx.x / t.N, c = blockIdx.x % t.N;
  const int N = t.N, cc = t.ccap, tid = threadIdx.x;
  __shared__ int32_t tile[NM][65];
  const int len = t.clen[g * N + c];
  for (int p0 = 0; p0 < len; p0 += 64) {
    for (int e = tid; e < N * 64; e += 256) {  // read along positions
      const int j = e >> 6, p = e & 63;
      tile[j][p] = p0 + p < len ? t.FDT[(((int64_t)g * N + j) * N + c) * cc + p0 + p] : INF;
    }
    __syncthreads();
    for (int e = tid; e < N * 64; e += 256) {  // write event rows
      const int p = e / N, j = e % N;
      if (p0 + p < len) t.FD[(((int64_t)g * N + c) * cc + p0 + p) * N + j] = tile[j][p];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Round / Witness by the round frontier, one 1024-thread workgroup per graph.
// Round(x) is a function of x's ancestry alone: the witnesses x strongly sees are
// its ancestors, so "the witnesses of the parent round inserted so far"
// (hashgraph.go:263-285) are all it can count.  With C_r[c] the first position of
// chain c whose round is >= r (rounds never decrease along a chain):
//   round(x) >= r + 1  <=>  x strongly sees >= SM of the members (d, C_r[d]),
//   fss_c(w) = the first position of chain c that strongly sees w
//            = SM-th smallest over i of FD[(i, FD[w][i])][c]
//     (x on chain c sees w's first descendant on chain i iff pos(x) >= that entry;
//     StronglySee counts those i, hashgraph.go:189-208),
//   C_{r+1}[c] = SM-th smallest over d of fss_c(C_r[d])  (the own-chain term at
//     least C_r[c] + 1: an event never strongly sees itself; matters at N = 1).
// The single-graph engine walks the same recurrence (k_fss / k_rounds_fss,
// hge_kernels.hip).  Per round: thread (member d, chain c) gathers the N rows
// FD[(i, FD[w_d][i])] at column c (one 128-byte row per half wave) and selects;
// then chain c's thread selects over the members.  Chain c's round-r events are
// the positions [C_r[c], C_{r+1}[c]), the first of them the witness; a witness's
// strongly-see bits over round r-1's witnesses are fss_c(w) <= its position, its
// see bits LA[x][d] >= index(w) (the vote adjacency of DecideFame).
template <int M>
__device__ __forceinline__ int kth_smallest(const int (&v)[M], int k) {
  // bisection over the value range: the smallest t with #{v <= t} >= k (INF when
  // fewer than k values are finite); positions span a few hundred, so ~9 counting
  // passes of M compares, register-light (a bitonic network held M values plus its
  // temporaries, ~88 VGPRs in kb_front: one 1,024-thread workgroup per CU)
  int lo = INF, hi = INT32_MIN, fin = 0;
#pragma unroll
  for (int i = 0; i < M; i++) {
    if (v[i] != INF) {
      lo = min(lo, v[i]);
      hi = max(hi, v[i]);
      fin++;
    }
  }
  if (fin < k) return INF;
  while (lo < hi) {
    const int mid = lo + ((hi - lo) >> 1);
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < M; i++) cnt += v[i] <= mid;
    if (cnt >= k) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// NT: 1024 threads while the graphs fit one workgroup per CU; 512 past that, so two
// graphs share a CU (the kernel's ~88 VGPRs hold one 1024-thread workgroup per CU)
template <int NM, int NT>
__global__ __launch_bounds__(NT) void kb_front(BT t) {
  constexpr int NW = NT / 64;
  const int g = blockIdx.x;
  const GDesc d = t.gd[g];
  const int N = t.N, SM = t.SM, cc = t.ccap, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ int32_t zrow[NM][NM];     // [member d][i]: the FD row of (d, C_r[d])
  __shared__ int32_t fssL[3][NM][NM];  // [r % 3][member d][chain c]: fss_c((d, C_r[d])), INF: no member
  __shared__ int32_t Cl[3][NM];        // C_{r-1}, C_r, C_{r+1} by r mod 3 (INF: none)
  __shared__ int32_t lenL[NM];
  __shared__ int s_more;
  const int32_t* FDg = t.FD + (int64_t)g * N * cc * N;  // [c][p][N]
  const int32_t* chg = t.chain + (int64_t)g * N * cc;   // [c][p] -> id
  const int32_t* LA = t.LA + d.eo * N;
  if (tid < N) {
    const int ln = t.clen[g * N + tid];
    lenL[tid] = ln;
    Cl[0][tid] = ln > 0 ? 0 : INF;  // the first event of a chain has no parents: round 0
    Cl[2][tid] = INF;
  }
  __syncthreads();
  // round r's outputs once C_{r+1} is known: the frontier ranges' rounds and witness
  // flags, the witness rows, and (r >= 1) each witness's bits over round r-1's
  auto outputs = [&](int r) {
    const int* Cp = Cl[(r + 2) % 3];
    const int* Cc = Cl[r % 3];
    const int* Cn = Cl[(r + 1) % 3];
    const int64_t row = (int64_t)(d.ro + r) * N;
    const int per = NT / N;  // threads per chain
    if (tid < per * N) {
      const int c = tid % N, k = tid / N;
      const int lo = Cc[c], hi = min(Cn[c], lenL[c]);
      if (lo != INF)
        for (int p = lo + k; p < hi; p += per) {
          const int x = chg[(int64_t)c * cc + p];
          t.round[d.eo + x] = r;
          t.roundch[(int64_t)g * N * cc + (int64_t)c * cc + p] = r;
          t.wit[d.eo + x] = p == lo;
          if (p == lo) {
            t.W[row + c] = x;
            t.WIX[row + c] = lo;
            t.WCOIN[row + c] = t.coin[d.eo + x];
          }
        }
    }
    if (r >= 1)
      for (int c = wv; c < N; c += NW) {  // one wave per witness of round r, lane = d
        const int lo = Cc[c], hi = min(Cn[c], lenL[c]);
        if (lo == INF || lo >= hi) continue;
        bool ss = false, see = false;
        if (lane < N) {
          const int pw = Cp[lane];
          if (pw != INF && pw < min(Cc[lane], lenL[lane])) {  // (lane, pw) is a witness of round r-1
            ss = fssL[(r + 2) % 3][lane][c] <= lo;
            const int x = chg[(int64_t)c * cc + lo];
            see = LA[(int64_t)x * N + lane] >= pw;
          }
        }
        const uint64_t bss = ballot(ss), bsee = ballot(see);
        if (lane == 0) {
          t.ssb[row + c] = bss;
          t.seeb[row + c] = bsee;
        }
      }
  };
  for (int r = 0;; r++) {
    if (r >= d.Rcap) {  // never for a consistent graph (R <= E / SM + 1)
      if (tid == 0) t.scal[(int64_t)g * 8 + 6] = 1;
      return;
    }
    const int* Cc = Cl[r % 3];
    int* Cn = Cl[(r + 1) % 3];
    // the members' FD rows
    for (int e = tid; e < N * N; e += NT) {
      const int dd = e / N, i = e - (e / N) * N;
      const int P = Cc[dd];
      zrow[dd][i] = P != INF ? FDg[((int64_t)dd * cc + P) * N + i] : INF;
    }
    __syncthreads();
    // fss_c of every member (c fastest: a half wave reads one 128-byte row; reading
    // the run layout FDT here instead, with no FD rows built, took 1.82 -> 2.69 ms at
    // 1,024 graphs)
    // One (member, chain) pair per thread (N^2 <= NT): round r - 1's outputs go out
    // while this round's gathers are in flight (its chain-id loads overlap them; the
    // outputs' reads of C_{r-2} and fss(r - 2) precede the barrier after which the
    // select overwrites C_{r-2}'s slot, and fssL holds three rounds).
    const bool one = N * N <= NT;
    if (one) {
      const int e = tid, dd = e / N, c = e - (e / N) * N;
      const bool act = e < N * N && Cc[dd] != INF;
      int v[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) {
        const int z = act && i < N ? zrow[dd][i] : INF;
        v[i] = z != INF ? FDg[((int64_t)i * cc + z) * N + c] : INF;
      }
      if (r > 0) outputs(r - 1);
      int f = INF;
      if (act) {
        f = kth_smallest<NM>(v, SM);
        if (dd == c && f != INF) f = max(f, Cc[c] + 1);
      }
      if (e < N * N) fssL[r % 3][dd][c] = f;
    } else {
      for (int e = tid; e < N * N; e += NT) {
        const int dd = e / N, c = e - (e / N) * N;
        int f = INF;
        if (Cc[dd] != INF) {
          int v[NM];
#pragma unroll
          for (int i = 0; i < NM; i++) {
            const int z = i < N ? zrow[dd][i] : INF;
            v[i] = z != INF ? FDg[((int64_t)i * cc + z) * N + c] : INF;
          }
          f = kth_smallest<NM>(v, SM);
          if (dd == c && f != INF) f = max(f, Cc[c] + 1);
        }
        fssL[r % 3][dd][c] = f;
      }
    }
    __syncthreads();
    // the next frontier
    if (wv == 0) {
      int nxt = INF;
      if (lane < N && Cc[lane] != INF) {
        int v[NM];
#pragma unroll
        for (int dd = 0; dd < NM; dd++) v[dd] = dd < N ? fssL[r % 3][dd][lane] : INF;
        const int sel = kth_smallest<NM>(v, SM);
        nxt = sel < lenL[lane] ? sel : INF;
      }
      if (lane < N) Cn[lane] = nxt;
      const uint64_t any = ballot(lane < N && nxt != INF);
      if (lane == 0) s_more = any != 0;
    }
    __syncthreads();
    if (!one) outputs(r);
    if (!s_more) {  // uniform: written before the barrier above
      if (one) outputs(r);
      break;
    }
  }
}

// ---------------------------------------------------------------------------
// consensus sorter keys (consensus_sorter.go:36-59 with PRN = 0): roundReceived,
// consensus timestamp, S (4 limbs), then the id (S never ties for real signatures)
__device__ __forceinline__ bool key_less(const BT& t, int64_t eo, int ra, int64_t ca, uint64_t sa, int ia,
                                         int rb, int64_t cb, uint64_t sb, int ib) {
  if (ra != rb) return ra < rb;
  if (ca != cb) return ca < cb;
  if (sa != sb) return sa < sb;
  for (int l = 1; l < 4; l++) {
    const uint64_t a = t.S[(eo + ia) * 4 + l], b = t.S[(eo + ib) * 4 + l];
    if (a != b) return a < b;
  }
  return ia < ib;
}

// Bitonic networks over the whole workgroup.  Stage (size, stride): thread q of the
// pair loop compares a = 2q - (q & (stride - 1)) and a + stride; for stride <= 64 a
// wave's 64 pairs stay inside its own 128 slots (also on the next pass of the q
// loop, 2 blockDim slots further), so two consecutive such stages need only the
// wave's own sync; a block barrier brackets every wider stage.
__device__ __forceinline__ void stage_sync(int size, int stride) {
  const int next = stride > 1 ? stride >> 1 : size;  // the next stage's stride
  if (stride > 64 || next > 64) __syncthreads();
  else wsync();
}

// n keys (padded to a power of two with sentinels, id INF, that order after every
// key) in the graph's global scratch (device-coherent accesses: threads exchange
// keys between stages)
__device__ void sort_keys_g(const BT& t, int64_t eo, int n, int32_t* kr, int64_t* kc, uint64_t* ks, int32_t* ki) {
  const int tid = threadIdx.x, NT = blockDim.x;
  int P = 1;
  while (P < n) P <<= 1;
  for (int p = n + tid; p < P; p += NT) st(ki + p, INF);
  __threadfence_block();
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int q = tid; q < P / 2; q += NT) {
        const int a = 2 * q - (q & (stride - 1));
        const int b = a + stride;
        const bool up = (a & size) == 0;
        const int ia = ld(ki + a), ib = ld(ki + b);
        if (ia == INF && ib == INF) continue;
        int ra = 0, rb = 0;
        int64_t ca = 0, cb = 0;
        uint64_t sa = 0, sb = 0;
        if (ia != INF) {
          ra = ld(kr + a);
          ca = ld(kc + a);
          sa = ld(ks + a);
        }
        if (ib != INF) {
          rb = ld(kr + b);
          cb = ld(kc + b);
          sb = ld(ks + b);
        }
        const bool b_lt_a = ib == INF ? false : (ia == INF ? true : key_less(t, eo, rb, cb, sb, ib, ra, ca, sa, ia));
        const bool a_lt_b = ia == INF ? false : (ib == INF ? true : key_less(t, eo, ra, ca, sa, ia, rb, cb, sb, ib));
        if (up ? b_lt_a : a_lt_b) {
          st(kr + a, rb);
          st(kr + b, ra);
          st(kc + a, cb);
          st(kc + b, ca);
          st(ks + a, sb);
          st(ks + b, sa);
          st(ki + a, ib);
          st(ki + b, ia);
        }
      }
      __threadfence_block();
      stage_sync(size, stride);
    }
  }
}

// the same network in LDS over packed keys: kri = roundReceived << 16 | id (both
// below 65,535: the host checks, sentinel 0xFFFFFFFF), n padded to a power of two
// P <= the arrays' size
__device__ void sort_keys_lds(const BT& t, int64_t eo, int n, uint32_t* kri, int64_t* kc, uint64_t* ks) {
  const int tid = threadIdx.x, NT = blockDim.x;
  int P = 1;
  while (P < n) P <<= 1;
  for (int p = n + tid; p < P; p += NT) kri[p] = 0xFFFFFFFFu;
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int q = tid; q < P / 2; q += NT) {
        const int a = 2 * q - (q & (stride - 1));
        const int b = a + stride;
        const bool up = (a & size) == 0;
        const uint32_t pa = kri[a], pb = kri[b];
        const bool na = pa == 0xFFFFFFFFu, nb_ = pb == 0xFFFFFFFFu;
        if (na && nb_) continue;
        const int ra = (int)(pa >> 16), ia = (int)(pa & 0xFFFFu), rb = (int)(pb >> 16), ib = (int)(pb & 0xFFFFu);
        const int64_t ca = na ? 0 : kc[a], cb = nb_ ? 0 : kc[b];
        const uint64_t sa = na ? 0 : ks[a], sb = nb_ ? 0 : ks[b];
        const bool b_lt_a = nb_ ? false : (na ? true : key_less(t, eo, rb, cb, sb, ib, ra, ca, sa, ia));
        const bool a_lt_b = na ? false : (nb_ ? true : key_less(t, eo, ra, ca, sa, ia, rb, cb, sb, ib));
        if (up ? b_lt_a : a_lt_b) {
          kri[a] = pb;
          kri[b] = pa;
          kc[a] = cb;
          kc[b] = ca;
          ks[a] = sb;
          ks[b] = sa;
        }
      }
      stage_sync(size, stride);
    }
  }
}

// ascending bitonic sorting networks over M register values (M a power of two)
template <int M>
__device__ __forceinline__ void sort_regs32(int32_t (&v)[M]) {
#pragma unroll
  for (int size = 2; size <= M; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
      for (int i = 0; i < M; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const int32_t a = v[i], b = v[j];
          v[i] = up ? min(a, b) : max(a, b);
          v[j] = up ? max(a, b) : min(a, b);
        }
      }
}
template <int M>
__device__ __forceinline__ void sort_regs(int64_t (&v)[M]) {
#pragma unroll
  for (int size = 2; size <= M; size <<= 1)
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1)
#pragma unroll
      for (int i = 0; i < M; i++) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const int64_t a = v[i], b = v[j];
          const bool sw = up ? a > b : a < b;
          v[i] = sw ? b : a;
          v[j] = sw ? a : b;
        }
      }
}

// ---------------------------------------------------------------------------
// The graph's call schedule in order, one workgroup of NWV waves per graph.  LDS
// holds the state of the rounds [R - RW, R) (witnesses and their indexes, vote
// bitsets, coins, fame, event counts, versions, receive thresholds and famous
// masks) and the undetermined list with each event's round, creator and index;
// rounds below the window and lists past UL entries live in global memory, where
// every mutation is also written.  Per call:
//   DivideRounds    wave 0 (the other waves compute the same scalars from the same
//                   loads: R, the list length, its lowest round);
//   DecideFame      rounds i split over the waves (each round's fame is decided from
//                   the vote adjacency alone), LastConsensusRound = the highest
//                   decided round, folded through LDS;
//   thresholds      rounds split over the waves;
//   round received  the list in spans of NWV x CPW chunks of 64: pass 1 loads a
//                   span's entries into registers and finds each one's round
//                   received, a prefix over the chunks' counts places the call's
//                   batch and the remaining entries (compacted in place: a span's
//                   entries move only below its own start), pass 2 takes the median
//                   timestamps and writes both;
//   FindOrder       the batch's bitonic sort over the whole workgroup.
// OCC: workgroups per CU the register budget is sized for.  One graph per CU
// leaves the compiler its 230 VGPRs; with more graphs than two per CU, 4 per CU
// (128 VGPRs, a few spills) take the whole batch in one pass.
template <int NM, int OCC>
__global__ __launch_bounds__(256, OCC) void kb_consensus(BT t) {
  // KB: the LDS sort's capacity, a power of two (the network pads to one)
  constexpr int NWV = 4, RW = 8, UL = 1536, KB = 1024, CPW = 2, NCH = NWV * CPW, SPAN = 64 * NCH;
  const int g = t.glist ? t.glist[blockIdx.x] : blockIdx.x;
  const GDesc d = t.gd[g];
  const int N = t.N, SM = t.SM, cc = t.ccap;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, NT = NWV * 64;
  const int64_t eo = d.eo;
  const int32_t* LA = t.LA + eo * N;
  const int32_t* FDg = t.FD + (int64_t)g * N * cc * N;  // [c][p][N]
  const int64_t* tschg = t.tsch + (int64_t)g * N * cc;
  __shared__ int32_t wid[RW][NM], wix[RW][NM], thL[RW][NM];
  __shared__ uint64_t ssbL[RW][NM], seebL[RW][NM];
  __shared__ uint64_t coinL[RW], fmL[RW];
  __shared__ int8_t fameL[RW][NM];
  __shared__ int32_t rcntL[RW], verL[RW], thvL[RW];
  // the undetermined list: creator << 24 | index, and round (the id is chain[c][index])
  __shared__ int32_t Ur_s[UL], Ucp_s[UL];
  __shared__ uint32_t kri[KB];  // roundReceived << 16 | id
  __shared__ int64_t kc[KB];
  __shared__ uint64_t ks[KB];
  __shared__ int32_t cntR[NCH], cntK[NCH];  // a span's chunks: received / kept entries
  __shared__ int32_t wred[3][NWV];          // per-wave partials: decided round, thresholds changed, kept minimum
  __shared__ int64_t wtx[NWV];              // per-wave transaction counts of the call's batch
  if (t.scal[(int64_t)g * 8 + 6]) return;  // the rounds pass failed: nothing to decide
  // packed LDS keys need ids and rounds below 65,535 (else the global-scratch sort)
  const bool lds_keys = d.E < 0xFFFF && d.Rcap < 0xFFFF;
  int R = 0, lcr = -1, lcre = 0, nord = 0, nU = 0, n_prev = 0;
  int umin = INF;  // the lowest round in the undetermined list
  int64_t ctx = 0;
  uint64_t cyc[6] = {0, 0, 0, 0, 0, 0};
  uint64_t t0_ = t.dbg ? __builtin_amdgcn_s_memtime() : 0;
#define HGB_STAMP(i)                                      \
  if (t.dbg && wv == 0) {                                 \
    const uint64_t t1_ = __builtin_amdgcn_s_memtime();    \
    cyc[i] += t1_ - t0_;                                  \
    t0_ = t1_;                                            \
  }
  bool ug = false;  // the undetermined list lives in global memory
  int32_t *Urg = t.Ur + eo, *Ucpg = t.Ucp + eo;
  const int32_t* chg = t.chain + (int64_t)g * N * cc;  // [c][p] -> id
  auto uget = [&](const int32_t* ls, const int32_t* gs, int i) -> int { return ug ? ld(&gs[i]) : ls[i]; };
  auto uput = [&](int32_t* ls, int32_t* gs, int i, int v) {
    if (ug) st(&gs[i], v);
    else ls[i] = v;
  };
  // ---- round accessors: LDS for [R - RW, R), global below ----
  auto res = [&](int r) { return r >= 0 && r < R && r >= R - RW; };
  auto row = [&](int r) { return (int64_t)(d.ro + r) * N; };
  auto W_ = [&](int r, int c) -> int { return res(r) ? wid[r & (RW - 1)][c] : t.W[row(r) + c]; };
  auto WIX_ = [&](int r, int c) -> int { return res(r) ? wix[r & (RW - 1)][c] : t.WIX[row(r) + c]; };
  auto fame_ = [&](int r, int c) -> int { return res(r) ? fameL[r & (RW - 1)][c] : ld(&t.fame[row(r) + c]); };
  auto rcnt_ = [&](int r) -> int { return res(r) ? rcntL[r & (RW - 1)] : ld(&t.rcnt[d.ro + r]); };
  auto ver_ = [&](int r) -> int { return res(r) ? verL[r & (RW - 1)] : ld(&t.ver[d.ro + r]); };
  auto thv_ = [&](int r) -> int { return res(r) ? thvL[r & (RW - 1)] : ld(&t.thv[d.ro + r]); };
  // single-writer updates (lane 0 or the lane of column c of the owning wave), written through
  auto set_rcnt = [&](int r, int v) {
    if (res(r)) rcntL[r & (RW - 1)] = v;
    st(&t.rcnt[d.ro + r], v);
  };
  auto set_ver = [&](int r, int v) {
    if (res(r)) verL[r & (RW - 1)] = v;
    st(&t.ver[d.ro + r], v);
  };
  for (int c = 0; c < d.K; c++) {
    const int n_c = (int)t.calls[d.co + c];
    const int nU0 = nU, umin0 = umin;  // the list before this call's events
    int rnmin;                         // the lowest round among the call's new events
    // ---- DivideRounds (hashgraph.go:573-588): the new events join the store ----
    {
      const int nn = n_c - n_prev;
      // the first 64 new events stay in registers (K <= 64: every call's)
      const bool on0 = lane < nn;
      const int x0 = n_prev + lane;
      const int r0 = on0 ? t.round[eo + x0] : -1;
      int rmax = r0, rlo = on0 ? r0 : INF;
      for (int b0 = n_prev + 64; b0 < n_c; b0 += 64)
        if (b0 + lane < n_c) {
          const int r = t.round[eo + b0 + lane];
          rmax = max(rmax, r);
          rlo = min(rlo, r);
        }
      rmax = wave_max(rmax);
      rnmin = wave_min(rlo);
      umin = min(umin, rnmin);
      const int Rnew = nn > 0 ? max(R, rmax + 1) : R;
      const int Rold = R;
      R = Rnew;
      const bool ug_new = !ug && nU + nn > UL;  // past the LDS list: it moves to global memory for good
      if (wv == 0) {
        // rounds entering the window: their immutable rows, fresh mutable state
        for (int r = max(Rold, Rnew - RW); r < Rnew; r++) {
          const int s = r & (RW - 1);
          const bool cl = lane < N;
          const int64_t rw_ = (int64_t)(d.ro + r) * N;
          const int w = cl ? t.W[rw_ + lane] : -1;
          if (cl) {
            wid[s][lane] = w;
            wix[s][lane] = t.WIX[rw_ + lane];
            ssbL[s][lane] = t.ssb[rw_ + lane];
            seebL[s][lane] = t.seeb[rw_ + lane];
            fameL[s][lane] = 0;
          }
          const uint64_t cm = ballot(cl && w >= 0 && t.WCOIN[rw_ + lane]);
          if (lane == 0) {
            coinL[s] = cm;
            fmL[s] = 0;
            rcntL[s] = 0;
            verL[s] = 0;
            thvL[s] = -1;
          }
        }
        wsync();
        // RoundEvents counts and witness versions, one writer per round; the
        // undetermined list grows by the new events in insertion order
        if (ug_new) {
          for (int i = lane; i < nU; i += 64) {
            st(&Urg[i], Ur_s[i]);
            st(&Ucpg[i], Ucp_s[i]);
          }
          ug = true;
        }
        const int w0 = on0 ? t.wit[eo + x0] : 0;
        const int cp0 = on0 ? (t.cr[eo + x0] << 24 | t.ix[eo + x0]) : 0;
        for (int b0 = n_prev; b0 < n_c; b0 += 64) {
          const int x = b0 + lane;
          const bool on = x < n_c;
          const int r = b0 == n_prev ? r0 : (on ? t.round[eo + x] : -1);
          const int w = b0 == n_prev ? w0 : (on ? t.wit[eo + x] : 0);
          const int cp = b0 == n_prev ? cp0 : (on ? (t.cr[eo + x] << 24 | t.ix[eo + x]) : 0);
          if (on) {
            uput(Ur_s, Urg, nU + (x - n_prev), r);
            uput(Ucp_s, Ucpg, nU + (x - n_prev), cp);
          }
          uint64_t rem = ballot(on);
          while (rem) {
            const int rr0 = rl(r, __ffsll((unsigned long long)rem) - 1);
            const uint64_t same = ballot(on && r == rr0);
            const bool nw = ballot(on && r == rr0 && w) != 0;
            if (lane == 0) {
              set_rcnt(rr0, rcnt_(rr0) + __popcll(same));
              if (nw) set_ver(rr0, ver_(rr0) + 1);
            }
            rem &= ~same;
            wsync();
          }
        }
        __threadfence_block();
      }
      ug = ug || ug_new;
      nU += nn;
      n_prev = n_c;
    }
    __syncthreads();
    HGB_STAMP(0)
    // ---- DecideFame (hashgraph.go:598-664) ----
    // Lane y is a voter of round j (y = lane, or lane & 31 with two half waves at
    // N <= 32); the witnesses x of round i are spread over the waves and half
    // waves, KX per lane group.  For one x and one j every present y's yays / nays
    // come at once (popcounts of its strongly-see bits against x's votes from round
    // j-1), the y loop's `break` is the first y whose tally reaches SM (a ballot's
    // lowest bit): x's votes from round j are the v of the y before it, its fame the
    // v of that y; later j decide again and the last decision stays.  Coin rounds
    // (diff % N == 0) vote the middle bit where no supermajority.  Missing votes are
    // nays.  Per round, the waves' "changed" / "undecided" flags meet in LDS.
    int mydec = -1;
    {
      constexpr int HV = NM <= 32 ? 2 : 1, XS = NWV * HV, KX = (NM + XS - 1) / XS;
      const int h = HV == 2 ? lane >> 5 : 0, y = HV == 2 ? lane & 31 : lane;
      const int xb = wv * HV + h;
      auto half = [&](uint64_t m) -> uint64_t { return HV == 2 ? (m >> (32 * h)) & 0xFFFFFFFFull : m; };
      for (int i = lcr + 1; i < R - 1; i++) {
        bool px[KX];
        int fv[KX], fv0[KX];
        uint64_t prev[KX];
#pragma unroll
        for (int k = 0; k < KX; k++) {
          const int x = xb + XS * k;
          const int xid = x < N ? W_(i, x) : -1;
          px[k] = xid >= 0 && xid < n_c;
          fv0[k] = px[k] ? fame_(i, x) : 0;
          fv[k] = fv0[k];
          prev[k] = 0;
        }
        for (int j = i + 1; j < R; j++) {
          const int diff = j - i;
          const bool rj = res(j);
          const int sj = j & (RW - 1);
          const int yid = y < N ? W_(j, y) : -1;
          const bool py = yid >= 0 && yid < n_c;
          uint64_t yb = 0;
          bool ycoin = false;
          if (py) {
            yb = diff == 1 ? (rj ? seebL[sj][y] : t.seeb[row(j) + y]) : (rj ? ssbL[sj][y] : t.ssb[row(j) + y]);
            ycoin = rj ? (coinL[sj] >> y) & 1 : t.WCOIN[row(j) + y] != 0;
          }
          const int tot = __popcll(yb);
#pragma unroll
          for (int k = 0; k < KX; k++) {
            const int x = xb + XS * k;
            uint64_t cur;
            if (diff == 1) {
              cur = half(ballot(py && ((yb >> x) & 1)));  // setVote(y, x, See(y, x))
            } else {
              const int yays = __popcll(yb & prev[k]), nays = tot - yays;
              const bool v = yays >= nays;
              const int tt = v ? yays : nays;
              if (diff % N != 0) {  // normal round: SetFame(x, v) and break at the first tt >= SM
                const uint64_t dm = half(ballot(py && tt >= SM));
                const uint64_t vm = half(ballot(py && v));
                if (dm) {
                  const int ys = __ffsll((unsigned long long)dm) - 1;
                  if (px[k]) fv[k] = (vm >> ys) & 1 ? 1 : 2;
                  cur = vm & ((1ull << ys) - 1);
                } else {
                  cur = vm;
                }
              } else {  // coin round: the middle bit of y's hash when no supermajority
                cur = half(ballot(py && (tt >= SM ? v : ycoin)));
              }
            }
            prev[k] = cur;
          }
        }
        bool chg = false, und = false;
#pragma unroll
        for (int k = 0; k < KX; k++) {
          const int x = xb + XS * k;
          const bool ch = px[k] && fv[k] != fv0[k];
          if (ch && y == 0) {
            if (res(i)) fameL[i & (RW - 1)][x] = (int8_t)fv[k];
            st(&t.fame[row(i) + x], (int8_t)fv[k]);
          }
          chg = chg || ch;
          und = und || (px[k] && fv[k] == 0);
        }
        const uint64_t bc = ballot(chg), bu = ballot(und);
        if (lane == 0) wred[0][wv] = (bc ? 1 : 0) | (bu ? 2 : 0);
        __threadfence_block();
        __syncthreads();
        int fl = 0;
        for (int w = 0; w < NWV; w++) fl |= wred[0][w];
        if ((fl & 1) && tid == 0) set_ver(i, ver_(i) + 1);
        if (!(fl & 2)) mydec = i;  // WitnessesDecided (roundInfo.go:78-85)
        __syncthreads();           // wred[0] is the next round's
      }
    }
    {
      // setLastConsensusRound (hashgraph.go:666-673): i runs upwards from lcr + 1 and
      // every decided i is past the last one set, so the highest decided round wins
      if (mydec >= 0) {
        lcr = mydec;
        lcre = mydec >= 1 ? rcnt_(mydec - 1) : 0;
      }
    }
    __syncthreads();  // the versions set above, for the thresholds
    HGB_STAMP(1)
    // ---- DecideRoundReceived (hashgraph.go:676-721) ----
    const int rmin = umin == INF ? R : umin;
    // decided rounds past the lowest undetermined round: the famous mask and the
    // thresholds theta (kept while the round's version holds: every fame change and
    // every new witness bumps the version, so thv == ver means decided and current)
    bool thchg = false;
    for (int i = rmin + 1 + wv; i < R; i += NWV) {
      const int v = ver_(i);
      if (thv_(i) == v) continue;
      const int w = lane < N ? W_(i, lane) : -1;
      const bool pw = w >= 0 && w < n_c;
      const int f = pw ? fame_(i, lane) : 0;
      if (ballot(pw && f == 0)) continue;  // not decided
      thchg = true;
      const uint64_t fm = ballot(pw && f == 1);
      const int m = __popcll(fm);
      int th = -2;  // no famous witness: nothing is received in the round
      if (lane < N && m > 0) {
        int vals[NM];
#pragma unroll
        for (int dd = 0; dd < NM; dd++) vals[dd] = (fm >> dd) & 1 ? LA[(int64_t)rl(w, dd) * N + lane] : -1;
        const int need = m / 2 + 1;  // len(s) > len(fws)/2
        int lo = -1, hi = t.clen[g * N + lane] - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          int cnt = 0;
#pragma unroll
          for (int dd = 0; dd < NM; dd++) cnt += ((fm >> dd) & 1) && vals[dd] >= mid;
          if (cnt >= need) lo = mid;
          else hi = mid - 1;
        }
        th = lo;
      }
      if (lane < N) {
        if (res(i)) thL[i & (RW - 1)][lane] = th;
        st(&t.th[row(i) + lane], th);
      }
      wsync();
      if (lane == 0) {
        if (res(i)) {
          thvL[i & (RW - 1)] = v;
          fmL[i & (RW - 1)] = fm;
        }
        st(&t.thv[d.ro + i], v);
      }
      wsync();
    }
    if (lane == 0) wred[1][wv] = thchg;
    __threadfence_block();
    __syncthreads();
    for (int w = 0; w < NWV; w++) thchg = thchg || wred[1][w];
    HGB_STAMP(2)
    // the undetermined events in order: received ones become the call's batch (keys
    // to LDS, and to global scratch past KB), the rest stay (compacted in place).
    // With no thresholds (re)computed in this call no earlier entry can be received
    // now (a round leaving the decided state only removes candidates), so only the
    // call's new events are examined.
    // Nor can a new event be, unless some round above it is decided: then the call
    // receives nothing and the list only grew.
    bool scan = thchg;
    for (int i = rnmin == INF ? R : rnmin + 1; i < R && !scan; i++) scan = thv_(i) == ver_(i);
    const int u0 = thchg ? 0 : nU0;
    int nb = 0, nk = scan ? u0 : nU, kmin = INF;
    int64_t tx = 0;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int sb = u0; scan && sb < nU; sb += SPAN) {
      // pass 1: the span's entries (chunk k * NWV + wv of the span is this wave's k-th)
      int er[CPW], ecp[CPW], ef[CPW];
#pragma unroll
      for (int k = 0; k < CPW; k++) {
        const int e = sb + (k * NWV + wv) * 64 + lane;
        const bool on = e < nU;
        er[k] = on ? uget(Ur_s, Urg, e) : 0;
        ecp[k] = on ? uget(Ucp_s, Ucpg, e) : 0;
        int found = -1;
        if (on) {
          const int cx = ecp[k] >> 24, px = ecp[k] & 0xFFFFFF;
          for (int i = er[k] + 1; i < R; i++) {
            int th;
            if (res(i)) {
              const int s = i & (RW - 1);
              if (thvL[s] != verL[s]) continue;  // not decided (or thresholds stale: never here)
              th = thL[s][cx];
            } else {
              if (ld(&t.thv[d.ro + i]) != ld(&t.ver[d.ro + i])) continue;
              th = ld(&t.th[row(i) + cx]);
            }
            if (th != -2 && px <= th) {
              found = i;
              break;
            }
          }
        }
        ef[k] = found;
        const int nr = __popcll(ballot(found >= 0)), nkp = __popcll(ballot(on && found < 0));
        if (lane == 0) {
          cntR[k * NWV + wv] = nr;
          cntK[k * NWV + wv] = nkp;
        }
      }
      __syncthreads();
      int preR[CPW], preK[CPW], totR = 0, totK = 0;
#pragma unroll
      for (int k = 0; k < CPW; k++) preR[k] = preK[k] = 0;
      for (int q = 0; q < NCH; q++) {
#pragma unroll
        for (int k = 0; k < CPW; k++)
          if (q == k * NWV + wv) {
            preR[k] = totR;
            preK[k] = totK;
          }
        totR += cntR[q];
        totK += cntK[q];
      }
      // pass 2: medians and keys of the received entries, the kept ones compacted
#pragma unroll
      for (int k = 0; k < CPW; k++) {
        const int e = sb + (k * NWV + wv) * 64 + lane;
        const bool on = e < nU;
        const int found = ef[k];
        const int cx = ecp[k] >> 24, px = ecp[k] & 0xFFFFFF;
        const uint64_t rec = ballot(found >= 0), keep = ballot(on && found < 0);
        if (found >= 0) {
          // MedianTimestamp over OldestSelfAncestorToSee(w, x) of the famous witnesses w
          // that see x (hashgraph.go:704-709, 762-770), the upper median.  w = (d, i_w)
          // sees x iff FD[x][d] <= i_w, and FD[x][d] is then OldestSelfAncestorToSee
          const int64_t cpos = (int64_t)cx * cc + px;
          const int x = chg[cpos];
          const uint64_t s0 = t.Sch[(int64_t)g * N * cc + cpos];
          tx += t.ntxch[(int64_t)g * N * cc + cpos];
          uint64_t fm;
          if (res(found)) {
            fm = fmL[found & (RW - 1)];
          } else {
            fm = 0;
            for (int dd = 0; dd < N; dd++) {
              const int w = t.W[row(found) + dd];
              if (w >= 0 && w < n_c && ld(&t.fame[row(found) + dd]) == 1) fm |= 1ull << dd;
            }
          }
          // the timestamps as int32 offsets from x's own (a register sort of 32-bit
          // values); an offset outside int32 takes the exact 64-bit count below
          const int64_t tsx = tschg[cpos];
          int32_t vals[NM];
          int m = 0;
          bool ovf = false;
#pragma unroll
          for (int dd = 0; dd < NM; dd++) {
            const int q = dd < N && ((fm >> dd) & 1) ? FDg[cpos * N + dd] : INF;
            vals[dd] = INT32_MAX;  // fillers sort last (a real INT32_MAX ties with them)
            if (q != INF && q <= WIX_(found, dd)) {
              const int64_t o = tschg[(int64_t)dd * cc + q] - tsx;
              ovf = ovf || o < -(int64_t)INT32_MAX || o > (int64_t)INT32_MAX;
              vals[dd] = (int32_t)o;
              m++;
            }
          }
          const int want = m / 2;  // the upper median
          int64_t med = 0;
          if (!ovf) {
            sort_regs32<NM>(vals);
#pragma unroll
            for (int a = 0; a < NM; a++)
              if (a == want) med = tsx + vals[a];
          } else {
            // the value whose rank among the m timestamps covers `want`
            auto tv = [&](int dd, int64_t& v) -> bool {
              if (!((fm >> dd) & 1)) return false;
              const int q = FDg[cpos * N + dd];
              if (q == INF || q > WIX_(found, dd)) return false;
              v = tschg[(int64_t)dd * cc + q];
              return true;
            };
            for (int a = 0; a < N; a++) {
              int64_t va;
              if (!tv(a, va)) continue;
              int lt = 0, eq = 0;
              for (int b = 0; b < N; b++) {
                int64_t vb;
                if (!tv(b, vb)) continue;
                lt += vb < va;
                eq += vb == va;
              }
              if (lt <= want && want < lt + eq) {
                med = va;
                break;
              }
            }
          }
          t.rr[eo + x] = found;
          t.cts[eo + x] = med;
          const int p = nb + preR[k] + __popcll(rec & below);
          if (p < KB && lds_keys) {
            kri[p] = (uint32_t)found << 16 | (uint32_t)x;
            kc[p] = med;
            ks[p] = s0;
          } else {
            const int64_t so = 2 * eo + nord + p;
            st(&t.krr[so], found);
            st(&t.kct[so], med);
            st(&t.ks0[so], s0);
            st(&t.kid[so], x);
          }
        }
        if (on && found < 0) {
          const int p = nk + preK[k] + __popcll(keep & below);
          uput(Ur_s, Urg, p, er[k]);
          uput(Ucp_s, Ucpg, p, ecp[k]);
          kmin = min(kmin, er[k]);
        }
      }
      nb += totR;
      nk += totK;
      __threadfence_block();
      __syncthreads();  // cntR / cntK are the next span's; its entries lie past every write above
    }
    nU = nk;
    {
      const int km = wave_min(kmin);
      const int64_t tw = wave_sum64(tx);
      if (lane == 0) {
        wred[2][wv] = km;
        wtx[wv] = tw;
      }
    }
    __syncthreads();
    {
      int km = INF;
      for (int w = 0; w < NWV; w++) {
        km = min(km, wred[2][w]);
        ctx += wtx[w];
      }
      if (scan) umin = min(thchg ? INF : umin0, km);
    }
    HGB_STAMP(3)
    // ---- FindOrder (hashgraph.go:723-760): sort the batch, append it ----
    if (nb > 0) {
      if (nb <= KB && lds_keys) {
        sort_keys_lds(t, eo, nb, kri, kc, ks);
        __syncthreads();
        for (int p = tid; p < nb; p += NT) t.order[eo + nord + p] = (int32_t)(kri[p] & 0xFFFFu);
      } else {
        // past KB keys: the same network on the graph's global scratch (2E entries
        // from 2 eo: nord + the padded size stays below 2E); the first KB keys are in LDS
        const int64_t so = 2 * eo + nord;
        if (lds_keys)
          for (int p = tid; p < KB; p += NT) {
            st(&t.krr[so + p], (int32_t)(kri[p] >> 16));
            st(&t.kct[so + p], kc[p]);
            st(&t.ks0[so + p], ks[p]);
            st(&t.kid[so + p], (int32_t)(kri[p] & 0xFFFFu));
          }
        __threadfence_block();
        __syncthreads();
        sort_keys_g(t, eo, nb, t.krr + so, t.kct + so, t.ks0 + so, t.kid + so);
        __syncthreads();
        for (int p = tid; p < nb; p += NT) t.order[eo + nord + p] = ld(&t.kid[so + p]);
      }
    }
    if (tid == 0) t.counts[d.co + c] = nb;
    nord += nb;
    __syncthreads();  // kri and the window state are the next call's
    HGB_STAMP(4)
  }
#undef HGB_STAMP
  if (t.dbg && tid == 0)
    for (int i = 0; i < 5; i++) t.dbg[(int64_t)g * 8 + i] = cyc[i];
  // the undetermined list for the host
  for (int i = tid; i < nU; i += NT) {
    const int cp = uget(Ucp_s, Ucpg, i);
    t.U[eo + i] = chg[(int64_t)(cp >> 24) * cc + (cp & 0xFFFFFF)];
  }
  if (tid == 0) {
    int64_t* s = t.scal + (int64_t)g * 8;
    s[0] = R;
    s[1] = lcr;
    s[2] = lcre;
    s[3] = ctx;
    s[4] = nord;
    s[5] = nU;
  }
}

#include "hge_batch_bulk.hip"

}  // namespace hgb

// ===========================================================================
// host side
// ===========================================================================
using namespace hgb;

namespace {

struct BatchError {
  int code;
  std::string msg;
};

#define BCHK(x)                                                                                \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) throw BatchError{HGE_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

template <typename T>
struct Buf {
  T* p = nullptr;
  size_t n = 0;
  void need(size_t m) {
    if (m <= n && p) return;
    free_();
    BCHK(hipMalloc(&p, std::max<size_t>(m, 1) * sizeof(T)));
    n = m;
  }
  void free_() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace

struct hge_batch {
  int N = 0, SM = 1, device = 0, ncu = 256;
  hipStream_t st = nullptr;
  hipEvent_t ev[9] = {};
  std::string err;
  struct Graph {
    std::vector<int32_t> cr, ix, sp, op, oc, ntx;
    std::vector<int64_t> ts;
    std::vector<uint64_t> S;
    std::vector<uint8_t> coin;
    std::vector<int64_t> calls;  // accepted counts at the call points
    std::vector<std::vector<int32_t>> chain;
  };
  std::vector<Graph> gs;
  bool staged = false, ran = false;
  std::vector<GDesc> hd;
  int64_t Etot = 0;
  int64_t Ktot = 0, Rtot = 0;
  int ccap = 0;
  std::vector<int64_t> h_scal;
  static constexpr int NK = 8;  // coords, fd, fdrows, front, fame (prep + pairs), fold (+ theta), receive, order
  float kms[NK] = {};
  // device tables
  Buf<GDesc> d_gd;
  Buf<int32_t> d_cr, d_ix, d_sp, d_op, d_oc, d_ntx, d_clen, d_chain, d_LA, d_FDT, d_FD, d_round, d_rr, d_W, d_WIX,
      d_WFD;
  Buf<int32_t> d_rcnt, d_ver, d_thv, d_th, d_U, d_Ur, d_Ucp, d_order, d_krr, d_kid;
  Buf<int64_t> d_ts, d_tsch, d_calls, d_cts, d_counts, d_scal, d_kct;
  Buf<uint64_t> d_Sch;
  Buf<int32_t> d_ntxch;
  Buf<uint64_t> d_S, d_ssb, d_seeb, d_ks0;
  Buf<uint8_t> d_coin, d_wit, d_WCOIN;
  Buf<int8_t> d_fame;
  Buf<uint64_t> d_dbg;
  bool dbg_on = getenv("HGB_STAMPS") != nullptr;
  // the bulk call schedule; HGB_SERIAL=1 (test hook): every graph through kb_consensus
  bool serial = getenv("HGB_SERIAL") != nullptr;
  Buf<int32_t> d_roundch, d_rrch, d_rslot, d_glist, d_cg, d_Rc, d_rfirst, d_rrank, d_xcall, d_gx, d_nivl, d_fsuf, d_thp, d_thR, d_rcall, d_bcnt, d_boff, d_wlc;
  Buf<uint64_t> d_arr, d_Dp, d_ivF, d_thF;
  Buf<int4> d_ivh;
  Buf<int4> d_wl;
  Buf<int2> d_cinf;
  Buf<int64_t> d_gctx, d_ctsch;
  int Emax = 0;
  int64_t n_fallback = 0;  // graphs the last run replayed through kb_consensus

  void free_all() {
    d_gd.free_();
    for (auto* b : {&d_cr, &d_ix, &d_sp, &d_op, &d_oc, &d_ntx, &d_clen, &d_chain, &d_LA, &d_FDT, &d_FD, &d_round,
                    &d_rr, &d_W, &d_WIX, &d_WFD, &d_rcnt, &d_ver, &d_thv, &d_th, &d_U, &d_Ur, &d_Ucp, &d_order,
                    &d_krr, &d_kid})
      b->free_();
    for (auto* b : {&d_ts, &d_tsch, &d_calls, &d_cts, &d_counts, &d_scal, &d_kct}) b->free_();
    for (auto* b : {&d_S, &d_ssb, &d_seeb, &d_ks0, &d_Sch}) b->free_();
    d_ntxch.free_();
    for (auto* b : {&d_roundch, &d_rrch, &d_rslot, &d_glist, &d_cg, &d_Rc, &d_rfirst, &d_rrank, &d_xcall, &d_gx, &d_nivl, &d_fsuf, &d_thp, &d_thR, &d_rcall, &d_bcnt,
                    &d_boff, &d_wlc})
      b->free_();
    for (auto* b : {&d_arr, &d_Dp, &d_ivF, &d_thF}) b->free_();
    d_ivh.free_();
    d_wl.free_();
    d_cinf.free_();
    d_gctx.free_();
    d_ctsch.free_();
    d_coin.free_();
    d_wit.free_();
    d_WCOIN.free_();
    d_fame.free_();
  }

  // FromParentsLatest (hashgraph.go:366-396) and the index rule of the engine
  // (hge_engine.hip admit: index-lying events are refused, HGE_ERR_INDEX)
  int admit(Graph& G, const std::vector<int32_t>& last, const hge_event& e, int32_t sp, int32_t op) {
    const int c = e.creator;
    if (c < 0 || c >= N) return HGE_ERR_CREATOR;
    const int known = (int)G.chain[c].size();
    const int64_t E = (int64_t)G.cr.size();
    if (sp == HGE_NONE && op == HGE_NONE && known == 0) return e.index == 0 ? HGE_OK : HGE_ERR_INDEX;
    if (sp < 0 || sp >= E) return HGE_ERR_SELF_PARENT_UNKNOWN;
    if (G.cr[sp] != c) return HGE_ERR_SELF_PARENT_CREATOR;
    if (op < 0 || op >= E) return HGE_ERR_OTHER_PARENT_UNKNOWN;
    if (sp != last[c]) return HGE_ERR_SELF_PARENT_NOT_LAST;
    if (e.index != known) return HGE_ERR_INDEX;
    return HGE_OK;
  }

  int add(const hge_event* ev, int64_t n_sub, const int64_t* cp, int64_t n_calls, int32_t* status) {
    for (int64_t c = 0; c < n_calls; c++)
      if (cp[c] < 1 || cp[c] > n_sub || (c > 0 && cp[c] <= cp[c - 1]))
        throw BatchError{HGE_ERR_ARG, "hge_batch_add: call points must be strictly ascending within [1, n_sub]"};
    if (n_sub >= INT32_MAX / 2) throw BatchError{HGE_ERR_ARG, "hge_batch_add: stream too long for a batch graph"};
    gs.emplace_back();
    Graph& G = gs.back();
    G.chain.assign(N, {});
    std::vector<int32_t> last(N, -1), idmap(n_sub, -1);
    int64_t nc = 0;
    for (int64_t i = 0; i < n_sub; i++) {
      const int32_t s = ev[i].self_parent, o = ev[i].other_parent;
      const int32_t sp = s < 0 ? HGE_NONE : (s < i && idmap[s] >= 0 ? idmap[s] : HGE_UNKNOWN);
      const int32_t op = o < 0 ? HGE_NONE : (o < i && idmap[o] >= 0 ? idmap[o] : HGE_UNKNOWN);
      const int r = admit(G, last, ev[i], sp, op);
      if (r == HGE_OK) {
        const int32_t id = (int32_t)G.cr.size();
        idmap[i] = id;
        G.cr.push_back(ev[i].creator);
        G.ix.push_back(ev[i].index);
        G.sp.push_back(sp);
        G.op.push_back(op);
        G.oc.push_back(op >= 0 ? G.cr[op] : 0);
        G.ntx.push_back(ev[i].n_tx);
        G.ts.push_back(ev[i].timestamp_ns);
        for (int k = 0; k < 4; k++) {
          uint64_t v = 0;
          for (int b = 0; b < 8; b++) v = (v << 8) | ev[i].s[8 * k + b];
          G.S.push_back(v);
        }
        G.coin.push_back(ev[i].hash[16] != 0);
        G.chain[ev[i].creator].push_back(id);
        last[ev[i].creator] = id;
      }
      if (status) status[i] = r == HGE_OK ? idmap[i] : r;
      while (nc < n_calls && cp[nc] == i + 1) {
        G.calls.push_back((int64_t)G.cr.size());
        nc++;
      }
    }
    staged = false;
    ran = false;
    return (int)gs.size() - 1;
  }

  template <typename T>
  void up(Buf<T>& b, const std::vector<T>& h) {
    b.need(h.size());
    if (!h.empty()) BCHK(hipMemcpyAsync(b.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, st));
  }

  void stage() {
    if (staged) return;
    BCHK(hipSetDevice(device));
    const int G = (int)gs.size();
    hd.assign(G, GDesc{});
    Etot = Ktot = Rtot = 0;
    ccap = 1;
    for (int g = 0; g < G; g++) {
      const Graph& gr = gs[g];
      GDesc& d = hd[g];
      d.eo = Etot;
      d.E = (int32_t)gr.cr.size();
      d.co = (int32_t)Ktot;
      d.K = (int32_t)gr.calls.size();
      d.ro = (int32_t)Rtot;
      // a round r + 1 exists only once >= SM witnesses of round r do: R <= E / SM + 1
      d.Rcap = d.E / SM + 2;
      Etot += d.E;
      Ktot += d.K;
      Rtot += d.Rcap;
      for (int c = 0; c < N; c++) ccap = std::max(ccap, (int)gr.chain[c].size());
    }
    if (Rtot >= INT32_MAX || Ktot >= INT32_MAX) throw BatchError{HGE_ERR_CAPACITY, "batch too large"};
    if (ccap >= (1 << 24)) throw BatchError{HGE_ERR_CAPACITY, "batch graph with a chain of 2^24 events or more"};
    std::vector<int32_t> cr, ix, sp, op, oc, ntx, clen((size_t)G * N), chain((size_t)G * N * ccap, -1), cgv;
    Emax = 0;
    for (int g = 0; g < G; g++) {
      cgv.insert(cgv.end(), (size_t)hd[g].K, g);
      Emax = std::max(Emax, hd[g].E);
    }
    std::vector<int64_t> ts, tsch((size_t)G * N * ccap, 0), calls;
    std::vector<uint64_t> Sch((size_t)G * N * ccap, 0);
    std::vector<int32_t> ntxch((size_t)G * N * ccap, 0);
    std::vector<uint64_t> S;
    std::vector<uint8_t> coin;
    cr.reserve(Etot);
    for (int g = 0; g < G; g++) {
      const Graph& gr = gs[g];
      cr.insert(cr.end(), gr.cr.begin(), gr.cr.end());
      ix.insert(ix.end(), gr.ix.begin(), gr.ix.end());
      sp.insert(sp.end(), gr.sp.begin(), gr.sp.end());
      op.insert(op.end(), gr.op.begin(), gr.op.end());
      oc.insert(oc.end(), gr.oc.begin(), gr.oc.end());
      ntx.insert(ntx.end(), gr.ntx.begin(), gr.ntx.end());
      ts.insert(ts.end(), gr.ts.begin(), gr.ts.end());
      S.insert(S.end(), gr.S.begin(), gr.S.end());
      coin.insert(coin.end(), gr.coin.begin(), gr.coin.end());
      calls.insert(calls.end(), gr.calls.begin(), gr.calls.end());
      for (int c = 0; c < N; c++) {
        clen[(size_t)g * N + c] = (int32_t)gr.chain[c].size();
        for (size_t p = 0; p < gr.chain[c].size(); p++) {
          chain[((size_t)g * N + c) * ccap + p] = gr.chain[c][p];
          tsch[((size_t)g * N + c) * ccap + p] = gr.ts[gr.chain[c][p]];
          Sch[((size_t)g * N + c) * ccap + p] = gr.S[4 * (size_t)gr.chain[c][p]];
          ntxch[((size_t)g * N + c) * ccap + p] = gr.ntx[gr.chain[c][p]];
        }
      }
    }
    up(d_cr, cr);
    up(d_ix, ix);
    up(d_sp, sp);
    up(d_op, op);
    up(d_oc, oc);
    up(d_ntx, ntx);
    up(d_ts, ts);
    up(d_S, S);
    up(d_coin, coin);
    up(d_calls, calls);
    up(d_clen, clen);
    up(d_chain, chain);
    up(d_tsch, tsch);
    up(d_Sch, Sch);
    up(d_ntxch, ntxch);
    up(d_cg, cgv);
    d_gd.need(G);
    BCHK(hipMemcpyAsync(d_gd.p, hd.data(), sizeof(GDesc) * G, hipMemcpyHostToDevice, st));
    const size_t E1 = (size_t)std::max<int64_t>(Etot, 1);
    d_LA.need(E1 * N);
    d_FDT.need((size_t)G * N * N * ccap);
    d_FD.need((size_t)G * N * ccap * N);
    d_round.need(E1);
    d_wit.need(E1);
    d_rr.need(E1);
    d_cts.need(E1);
    d_U.need(E1);
    d_Ur.need(E1);
    d_Ucp.need(E1);
    d_order.need(E1);
    d_krr.need(2 * E1 + 64);
    d_kct.need(2 * E1 + 64);
    d_ks0.need(2 * E1 + 64);
    d_kid.need(2 * E1 + 64);
    const size_t RN = (size_t)std::max<int64_t>(Rtot, 1) * N;
    d_W.need(RN);
    d_WIX.need(RN);
    d_WFD.need(RN * N);
    d_WCOIN.need(RN);
    d_ssb.need(RN);
    d_seeb.need(RN);
    d_fame.need(RN);
    d_th.need(RN);
    d_rcnt.need(RN / N);
    d_ver.need(RN / N);
    d_thv.need(RN / N);
    d_counts.need(std::max<int64_t>(Ktot, 1));
    d_scal.need((size_t)G * 8);
    if (dbg_on) d_dbg.need((size_t)G * 8);
    const size_t K1 = (size_t)std::max<int64_t>(Ktot, 1);
    d_glist.need(G);
    d_Rc.need(K1);
    d_rfirst.need(RN / N);
    d_xcall.need(E1);
    d_arr.need(E1);
    d_Dp.need(K1 * BNS * 2);
    d_gx.need((size_t)G * 16);
    d_ivh.need(RN / N * BVCAP);
    d_ivF.need(RN / N * BVCAP);
    d_nivl.need(RN / N);
    d_fsuf.need(RN / N);
    d_thp.need((size_t)G * BICAP * N);
    d_thR.need((size_t)G * BICAP);
    d_thF.need((size_t)G * BICAP);
    const size_t CH = (size_t)G * N * ccap;
    d_roundch.need(CH);
    d_rcall.need(CH);
    d_rrank.need(CH);
    d_rrch.need(CH);
    d_rslot.need(CH);
    d_ctsch.need(CH);
    d_bcnt.need(K1);
    d_boff.need(K1);
    d_wl.need(K1);
    d_wlc.need(1);
    d_gctx.need(G);
    d_cinf.need(E1);
    BCHK(hipStreamSynchronize(st));
    staged = true;
  }

  BT tables() const {
    BT t;
    t.N = N;
    t.SM = SM;
    t.ccap = ccap;
    t.gd = d_gd.p;
    t.cr = d_cr.p;
    t.ix = d_ix.p;
    t.sp = d_sp.p;
    t.op = d_op.p;
    t.oc = d_oc.p;
    t.ntx = d_ntx.p;
    t.clen = d_clen.p;
    t.ts = d_ts.p;
    t.S = d_S.p;
    t.coin = d_coin.p;
    t.chain = d_chain.p;
    t.tsch = d_tsch.p;
    t.calls = d_calls.p;
    t.LA = d_LA.p;
    t.FDT = d_FDT.p;
    t.FD = d_FD.p;
    t.Sch = d_Sch.p;
    t.ntxch = d_ntxch.p;
    t.round = d_round.p;
    t.wit = d_wit.p;
    t.rr = d_rr.p;
    t.cts = d_cts.p;
    t.W = d_W.p;
    t.WIX = d_WIX.p;
    t.WFD = d_WFD.p;
    t.WCOIN = d_WCOIN.p;
    t.ssb = d_ssb.p;
    t.seeb = d_seeb.p;
    t.fame = d_fame.p;
    t.rcnt = d_rcnt.p;
    t.ver = d_ver.p;
    t.thv = d_thv.p;
    t.th = d_th.p;
    t.U = d_U.p;
    t.Ur = d_Ur.p;
    t.Ucp = d_Ucp.p;
    t.order = d_order.p;
    t.counts = d_counts.p;
    t.scal = d_scal.p;
    t.krr = d_krr.p;
    t.kct = d_kct.p;
    t.ks0 = d_ks0.p;
    t.kid = d_kid.p;
    t.dbg = dbg_on ? d_dbg.p : nullptr;
    t.glist = nullptr;
    t.cg = d_cg.p;
    t.Rc = d_Rc.p;
    t.rfirst = d_rfirst.p;
    t.xcall = d_xcall.p;
    t.arr = d_arr.p;
    t.Dp = d_Dp.p;
    t.gx = d_gx.p;
    t.ivh = d_ivh.p;
    t.ivF = d_ivF.p;
    t.nivl = d_nivl.p;
    t.fsuf = d_fsuf.p;
    t.thp = d_thp.p;
    t.thR = d_thR.p;
    t.thF = d_thF.p;
    t.roundch = d_roundch.p;
    t.rcall = d_rcall.p;
    t.rrank = d_rrank.p;
    t.rrch = d_rrch.p;
    t.rslot = d_rslot.p;
    t.ctsch = d_ctsch.p;
    t.bcnt = d_bcnt.p;
    t.boff = d_boff.p;
    t.wl = d_wl.p;
    t.wlc = d_wlc.p;
    t.gctx = d_gctx.p;
    t.cinf = d_cinf.p;
    return t;
  }

  template <typename K>
  void launch(K kern, int G, const BT& t, int block = 64) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(block), 0, st, t);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw BatchError{HGE_ERR_DEVICE, std::string("batch launch: ") + hipGetErrorString(e)};
  }

  template <int NM>
  void run_stages(int G, const BT& t) {
    // a workgroup of 1,024 threads per graph while two fit a CU, else 512
    // 1,024 threads per graph and the kb_levels pass while two graphs fit a CU, else
    // 512 threads levelling their own chunks
    if (G <= 2 * ncu) {
      if (Emax > 0) {
        hipLaunchKernelGGL(kb_levels, dim3((unsigned)((Emax + 255) / 256), (unsigned)G), dim3(256), 0, st, t);
        BCHK(hipGetLastError());
      }
      // the columns split over two workgroups while both still get a CU of their own
      // (128 graphs: 0.46 -> 0.43 ms; at 256 graphs, two per CU, 0.49 -> 0.51; four
      // 8-column parts: 0.45 / 0.55)
      if (2 * G <= ncu) hipLaunchKernelGGL((kb_coords<NM, 512, true, 2>), dim3(G * 2), dim3(512), 0, st, t);
      else launch(kb_coords<NM, 1024, true>, G, t, 1024);
      BCHK(hipGetLastError());
    } else {
      launch(kb_coords<NM, 512, false>, G, t, 512);
    }
    BCHK(hipEventRecord(ev[1], st));
    launch(kb_fd<NM>, G * N, t, 64 * (NM / FCW));
    BCHK(hipEventRecord(ev[2], st));
    launch(kb_fdrows<NM>, G * N, t, 256);  // rows for kb_front (kb_median reads the run layout)
    BCHK(hipEventRecord(ev[3], st));
    if (G > 2 * ncu) launch(kb_front<NM, 256>, G, t, 256);
    else if (G > ncu) launch(kb_front<NM, 512>, G, t, 512);
    else launch(kb_front<NM, 1024>, G, t, 1024);
    BCHK(hipEventRecord(ev[4], st));
    if (serial) {  // every graph through kb_consensus, after the run's readback
      for (int k = 5; k < 9; k++) BCHK(hipEventRecord(ev[k], st));
      return;
    }
    launch(kb_prep<NM>, G, t, 1024);
    if (G > 2 * ncu) hipLaunchKernelGGL((kb_pairs<NM, 2>), dim3(8, (unsigned)G), dim3(256), 0, st, t);
    else hipLaunchKernelGGL((kb_pairs<NM, 3>), dim3(8, (unsigned)G), dim3(256), 0, st, t);
    BCHK(hipGetLastError());
    BCHK(hipEventRecord(ev[5], st));
    if (G > 2 * ncu) launch((kb_fold<NM, 2>), G, t, 64);
    else launch((kb_fold<NM, 3>), G, t, 64);
    launch(kb_theta<NM>, G, t, 256);
    BCHK(hipEventRecord(ev[6], st));
    if (Emax > 0) {
      hipLaunchKernelGGL(kb_receive<NM>, dim3((unsigned)N, (unsigned)G), dim3(256), 0, st, t);
      BCHK(hipGetLastError());
      hipLaunchKernelGGL(kb_median<NM>, dim3((unsigned)(N * ((ccap + 255) / 256)), (unsigned)G), dim3(256), 0, st, t);
      BCHK(hipGetLastError());
    }
    BCHK(hipEventRecord(ev[7], st));
    launch(kb_order_prep<NM>, G, t, 1024);
    // call buckets: up to 1,024 keys one wave each (a workgroup of four while the
    // batch has few buckets), larger ones a workgroup each
    const int nbk = (int)std::min<int64_t>(std::max<int64_t>(Ktot, 1), (int64_t)ncu * 16);
    if (Ktot > 16 * (int64_t)ncu) hipLaunchKernelGGL((kb_sort<64, 0, 1024>), dim3(nbk), dim3(64), 0, st, t, 0);
    else hipLaunchKernelGGL((kb_sort<256, 0, 1024>), dim3(nbk), dim3(256), 0, st, t, 0);
    BCHK(hipGetLastError());
    hipLaunchKernelGGL((kb_sort<256, 1024, 4096>), dim3(ncu), dim3(256), 0, st, t, 1);
    BCHK(hipGetLastError());
    BCHK(hipEventRecord(ev[8], st));
  }

  int64_t run() {
    stage();
    const int G = (int)gs.size();
    if (G == 0) return 0;
    const size_t RN = (size_t)std::max<int64_t>(Rtot, 1) * N;
    const size_t E1 = (size_t)std::max<int64_t>(Etot, 1);
    const size_t K1 = (size_t)std::max<int64_t>(Ktot, 1);
    ClrList cl{};
    auto seg = [&](void* p, size_t bytes, uint32_t pat) { cl.s[cl.n++] = ClrSeg{p, (uint64_t)bytes, pat}; };
    seg(d_W.p, RN * 4, ~0u);
    seg(d_WIX.p, RN * 4, ~0u);
    seg(d_ssb.p, RN * 8, 0);
    seg(d_seeb.p, RN * 8, 0);
    seg(d_fame.p, RN, 0);
    seg(d_rcnt.p, RN / N * 4, 0);
    seg(d_ver.p, RN / N * 4, 0);
    seg(d_thv.p, RN / N * 4, ~0u);
    seg(d_rr.p, E1 * 4, ~0u);
    seg(d_cts.p, E1 * 8, 0);
    seg(d_scal.p, (size_t)G * 64, 0);
    seg(d_bcnt.p, K1 * 4, 0);
    seg(d_wlc.p, 4, 0);
    seg(d_gctx.p, (size_t)G * 8, 0);
    hipLaunchKernelGGL(kb_clear, dim3((unsigned)std::min<size_t>(2048, (E1 * 8 / 16 + 255) / 256 + 1)), dim3(256), 0, st, cl);
    BCHK(hipGetLastError());
    BT t = tables();
    BCHK(hipEventRecord(ev[0], st));
    if (N <= 32) run_stages<32>(G, t);
    else run_stages<64>(G, t);
    h_scal.resize((size_t)G * 8);
    BCHK(hipMemcpyAsync(h_scal.data(), d_scal.p, (size_t)G * 64, hipMemcpyDeviceToHost, st));
    BCHK(hipStreamSynchronize(st));
    for (int k = 0; k < NK; k++) BCHK(hipEventElapsedTime(&kms[k], ev[k], ev[k + 1]));
    // graphs the bulk fold could not hold: replayed by kb_consensus (their outputs untouched so far)
    std::vector<int32_t> fb;
    for (int g = 0; g < G; g++)
      if (serial || (h_scal[(size_t)g * 8 + 7] && !h_scal[(size_t)g * 8 + 6])) fb.push_back(g);
    n_fallback = (int64_t)fb.size();
    if (!fb.empty()) {
      BCHK(hipMemcpyAsync(d_glist.p, fb.data(), fb.size() * 4, hipMemcpyHostToDevice, st));
      t.glist = d_glist.p;
      const int F = (int)fb.size();
      float ms = 0;
      BCHK(hipEventRecord(ev[7], st));
      if (N <= 32) {
        if (F > 2 * ncu) launch(kb_consensus<32, 4>, F, t, 256);
        else launch(kb_consensus<32, 1>, F, t, 256);
      } else {
        if (F > 2 * ncu) launch(kb_consensus<64, 4>, F, t, 256);
        else launch(kb_consensus<64, 1>, F, t, 256);
      }
      BCHK(hipEventRecord(ev[8], st));
      BCHK(hipMemcpyAsync(h_scal.data(), d_scal.p, (size_t)G * 64, hipMemcpyDeviceToHost, st));
      BCHK(hipStreamSynchronize(st));
      BCHK(hipEventElapsedTime(&ms, ev[7], ev[8]));
      kms[NK - 1] += ms;
    }
    if (dbg_on) {  // section cycles of kb_consensus, summed over the graphs
      std::vector<uint64_t> hd_((size_t)G * 8);
      BCHK(hipMemcpy(hd_.data(), d_dbg.p, (size_t)G * 64, hipMemcpyDeviceToHost));
      double sum[5] = {};
      for (int g = 0; g < G; g++)
        for (int i = 0; i < 5; i++) sum[i] += (double)hd_[(size_t)g * 8 + i];
      fprintf(stderr, "[hgb stamps] per graph cycles: divide %.0f fame %.0f thresholds %.0f receive %.0f order %.0f\n",
              sum[0] / G, sum[1] / G, sum[2] / G, sum[3] / G, sum[4] / G);
    }
    int64_t tot = 0;
    for (int g = 0; g < G; g++) {
      if (h_scal[(size_t)g * 8 + 6])
        throw BatchError{HGE_ERR_INTERNAL, "batch graph " + std::to_string(g) + ": round capacity exceeded"};
      tot += h_scal[(size_t)g * 8 + 4];
    }
    ran = true;
    return tot;
  }

  template <typename T>
  void down(T* host, const T* dev, size_t n) {
    if (host && n) BCHK(hipMemcpy(host, dev, n * sizeof(T), hipMemcpyDeviceToHost));
  }
};

#define BGUARD_BEGIN try {
#define BGUARD_END(b)                 \
  }                                   \
  catch (BatchError & e) {            \
    (b)->err = e.msg;                 \
    return e.code;                    \
  }                                   \
  catch (std::exception & e) {        \
    (b)->err = e.what();              \
    return HGE_ERR_INTERNAL;          \
  }

extern "C" {

int hge_batch_create(int32_t n_participants, int32_t device, hge_batch** out) {
  if (!out || n_participants < 1 || n_participants > 64) return HGE_ERR_ARG;
  hge_batch* b = new hge_batch();
  b->N = n_participants;
  b->SM = 2 * n_participants / 3 + 1;  // hashgraph.go:78-80
  b->device = device;
  try {
    BCHK(hipSetDevice(device));
    BCHK(hipDeviceGetAttribute(&b->ncu, hipDeviceAttributeMultiprocessorCount, device));
    BCHK(hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking));
    for (auto& e : b->ev) BCHK(hipEventCreate(&e));
  } catch (BatchError& e) {
    delete b;
    return e.code;
  }
  *out = b;
  return HGE_OK;
}

void hge_batch_destroy(hge_batch* b) {
  if (!b) return;
  if (b->st) (void)hipStreamSynchronize(b->st);
  b->free_all();
  for (auto& e : b->ev)
    if (e) (void)hipEventDestroy(e);
  if (b->st) (void)hipStreamDestroy(b->st);
  delete b;
}

const char* hge_batch_last_error(hge_batch* b) { return b ? b->err.c_str() : "null handle"; }

int hge_batch_add(hge_batch* b, const hge_event* ev, int64_t n_sub, const int64_t* call_points, int64_t n_calls,
                  int32_t* status_out, int32_t* graph_out) {
  if (!b) return HGE_ERR_ARG;
  BGUARD_BEGIN
  if (n_sub < 0 || (n_sub > 0 && !ev) || n_calls < 0 || (n_calls > 0 && !call_points))
    throw BatchError{HGE_ERR_ARG, "hge_batch_add: bad argument"};
  const int g = b->add(ev, n_sub, call_points, n_calls, status_out);
  if (graph_out) *graph_out = g;
  return HGE_OK;
  BGUARD_END(b)
}

int hge_batch_stage(hge_batch* b) {
  if (!b) return HGE_ERR_ARG;
  BGUARD_BEGIN
  b->stage();
  return HGE_OK;
  BGUARD_END(b)
}

int hge_batch_run(hge_batch* b, int64_t* n_ordered) {
  if (!b) return HGE_ERR_ARG;
  BGUARD_BEGIN
  const int64_t m = b->run();
  if (n_ordered) *n_ordered = m;
  return HGE_OK;
  BGUARD_END(b)
}

int32_t hge_batch_graphs(hge_batch* b) { return b ? (int32_t)b->gs.size() : -1; }

int hge_batch_info(hge_batch* b, int32_t g, int64_t* info) {
  if (!b || !info || g < 0 || g >= (int)b->gs.size()) return HGE_ERR_ARG;
  if (!b->ran) {
    b->err = "hge_batch_info: no replay yet (hge_batch_run)";
    return HGE_ERR_ARG;
  }
  const int64_t* s = &b->h_scal[(size_t)g * 8];
  info[0] = (int64_t)b->gs[g].cr.size();
  info[1] = (int64_t)b->gs[g].calls.size();
  for (int k = 0; k < 6; k++) info[2 + k] = s[k];
  return HGE_OK;
}

int hge_batch_results(hge_batch* b, int32_t g, int32_t* order, int64_t* counts, int32_t* round, uint8_t* witness,
                      int32_t* rr, int64_t* cts, int8_t* fame, int32_t* undetermined) {
  if (!b || g < 0 || g >= (int)b->gs.size()) return HGE_ERR_ARG;
  BGUARD_BEGIN
  if (!b->ran) throw BatchError{HGE_ERR_ARG, "hge_batch_results: no replay yet (hge_batch_run)"};
  const GDesc& d = b->hd[g];
  const int64_t* s = &b->h_scal[(size_t)g * 8];
  const int N = b->N;
  b->down(order, b->d_order.p + d.eo, (size_t)s[4]);
  b->down(counts, b->d_counts.p + d.co, (size_t)d.K);
  b->down(round, b->d_round.p + d.eo, (size_t)d.E);
  b->down(witness, b->d_wit.p + d.eo, (size_t)d.E);
  b->down(rr, b->d_rr.p + d.eo, (size_t)d.E);
  b->down(cts, b->d_cts.p + d.eo, (size_t)d.E);
  b->down(undetermined, b->d_U.p + d.eo, (size_t)s[5]);
  if (fame && s[0] > 0) {
    const size_t RN = (size_t)s[0] * N;
    std::vector<int32_t> w(RN);
    std::vector<int8_t> f(RN);
    b->down(w.data(), b->d_W.p + (size_t)d.ro * N, RN);
    b->down(f.data(), b->d_fame.p + (size_t)d.ro * N, RN);
    for (size_t k = 0; k < RN; k++) fame[k] = w[k] >= 0 ? f[k] : (int8_t)-1;
  }
  return HGE_OK;
  BGUARD_END(b)
}

int64_t hge_batch_fallbacks(hge_batch* b) { return b ? b->n_fallback : -1; }

int hge_batch_kernel_ms(hge_batch* b, float* ms, int32_t cap) {
  if (!b || (!ms && cap > 0)) return HGE_ERR_ARG;
  for (int k = 0; k < hge_batch::NK && k < cap; k++) ms[k] = b->kms[k];
  return hge_batch::NK;
}

}  // extern "C"

// diagnostics (not part of the C ABI): graph g's lastAncestors (which 0) or
// firstDescendants (which 1) rows after a run, E x N int32 into out
extern "C" int hgb_debug_rows(hge_batch* b, int32_t g, int32_t which, int32_t* out) {
  if (!b || !out || g < 0 || g >= (int)b->gs.size() || !b->ran) return HGE_ERR_ARG;
  BGUARD_BEGIN
  const GDesc& d = b->hd[g];
  if (which == 2)  // the run layout FDT[j][c][p], N x N x ccap
    b->down(out, b->d_FDT.p + (size_t)g * b->N * b->N * b->ccap, (size_t)b->N * b->N * b->ccap);
  else
    b->down(out, b->d_LA.p + d.eo * b->N, (size_t)d.E * b->N);
  return HGE_OK;
  BGUARD_END(b)
}
