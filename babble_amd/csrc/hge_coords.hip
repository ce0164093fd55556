// hge_coords.hip — coordinate kernels (InitEventCoordinates +
// UpdateAncestorFirstDescendant) of the hashgraph ordering engine, all N.
//
// The DAG is ~E / (N/3.7) levels deep (18.6k levels at 16/100k), so the
// coordinates are built from a few bandwidth-friendly passes instead of a
// level-by-level walk:
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
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

// LA[(j, k)] = -1 for the new positions k in [olen_j, len_j) of every chain;
// also zeroes the sweeps' changed flags (zero[0, nzero)) in place of a memset
__global__ void k_la_clear(Tables t, const int32_t* olen, const int32_t* len, int32_t* zero,
                           int nzero) {
  const int j = blockIdx.y;
  const int N = t.N;
  if (j == 0 && blockIdx.x == 0)
    for (int i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0;
  const int64_t lo = (int64_t)olen[j] * N, hi = (int64_t)len[j] * N;
  int32_t* base = t.LA + (size_t)j * t.ccap * N;
  for (int64_t e = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < hi;
       e += (int64_t)gridDim.x * blockDim.x)
    base[e] = -1;
}

// One in-place sweep.  G = 256/NP segments per workgroup, NP threads (columns)
// per segment.  segs[s] = (chain, first position).
// prev: the previous sweep's changed flag (nullptr for the first): sweeps are
// queued in groups without a host round trip, and once one changes nothing
// the rest of its group return at once.
// A sweep is a chain of dependent memory latencies, not of bytes at small N:
// the other-parent coordinates come from the chain-major opcp table (one load,
// staged in LDS), and each lane then has all U loads of a batch in flight
// (op rows and own rows) before it folds them, so a 64-position segment costs
// three latencies (opcp, two batches) plus the fold.
template <int NP>
__global__ void __launch_bounds__(256) k_la_sweep(Tables t, const int2* segs, int nseg, int SEG,
                                                  const int32_t* len, const int32_t* prev,
                                                  int32_t* changed) {
  constexpr int G = 256 / NP;
  constexpr int SEGMAX = 64;
  constexpr int U = 32;  // loads in flight per lane and batch
  __shared__ int64_t s_off[G][SEGMAX];
  if (prev && *prev == 0) return;  // converged: the flag stays 0
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
      const int2 o = t.opcp[(size_t)j * t.ccap + k0 + kk];
      if (o.x >= 0) off = (int64_t)rowoff(t, o.x, o.y);
    }
    s_off[g][kk] = off;
  }
  __syncthreads();
  const bool act = valid && i < N;
  bool ch = false;
  if (act) {
    const size_t own0 = rowoff(t, j, k0) + i;
    int v = (k0 > 0) ? t.LA[own0 - N] : -1;
    for (int kb = k0; kb < k1; kb += U) {
      int a[U], old[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = kb + u;
        a[u] = -1;
        old[u] = -1;
        if (k < k1) {
          const int64_t off = s_off[g][k - k0];
          if (off >= 0) a[u] = t.LA[off + i];
          old[u] = t.LA[own0 + (size_t)(k - k0) * N];
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = kb + u;
        if (k < k1) {
          v = max(v, a[u]);
          if (i == j) v = max(v, k);
          const int nv = max(v, old[u]);
          v = nv;
          if (nv != old[u]) {
            t.LA[own0 + (size_t)(k - k0) * N] = nv;
            ch = true;
          }
        }
      }
    }
  }
  // a plain store: every writer stores 1 (same-address atomics serialise at memory)
  if (__ballot(ch) && (threadIdx.x & 63) == __builtin_ctzll(__ballot(ch))) *changed = 1;
}

// lastAncestors of a small batch of new events [n0, n1) (an online call at N <= 32)
// in ONE exact pass: no fixed-point sweeps, so no host round trip for their
// convergence flags.  The same recurrence as k_la_sweep, in insertion order (a
// parent is inserted before its child):
//   phase 1 (all lanes, NP per event): the max of the rows of the event's chain
//     predecessor and other-parent that existed before the batch, with its own
//     column; the batch indices of the parents inserted in it;
//   phase 2 (the first NP lanes of wave 0, lane = column): the events in order,
//     folding their in-batch parents' rows from LDS (two LDS reads per event);
//   phase 3: the rows to LA, coalesced.
// lowest chain-c position whose FD row a new event can change:
// min over chains j with old events of LA[(j, olen_j - 1)][c] + 1
// grid N blocks (chain c), thread j = chain j: one load per thread and a block
// min (a thread looping over the N chains was a chain of 256 dependent-latency
// loads: ~40 us per online call at N = 256)
__device__ __forceinline__ void fd_qlo_body(const Tables& t, const int32_t* olen, const int32_t* len, int32_t* qlo,
                                            int c) {
  __shared__ int s_m;
  const int j = threadIdx.x;
  if (j == 0) s_m = olen[c];  // the new positions themselves
  __syncthreads();
  if (j < t.N && len[j] != olen[j]) {  // chain j got a new event
    const int ol = olen[j];
    const int v = ol > 0 ? la_at(t, j, ol - 1, c) + 1 : 0;
    atomicMin(&s_m, v);
  }
  __syncthreads();
  if (j == 0) qlo[c] = max(0, s_m);
}
// m * NP <= LASEQ_MAX (the host checks; larger batches take the sweeps).
constexpr int LASEQ_MAX = 8192;
// It also fills the chain table for the batch first (k_chain_fill's work: one
// launch less per online call); the barrier makes those global writes visible to
// the block.
// qlo (non-null): blocks 1 .. N take k_fd_qlo's work for chain blockIdx.x - 1 (it
// reads only the old events' LA rows; one launch less per online call)
// fst (non-null): the grid's last block takes k_frontier_start's work (the rounds
// walk's first round and k_fss rows, written to fst / fst_lo; it reads only the old
// events' rounds and the C rows: one launch less per online call)
// fdt (non-null, N <= 16): the firstDescendants of the batch written here too, in
// place of k_la16_rows_runs + k_transpose (two launches less per online call): the new
// positions' FD rows and FDT entries start as none, then chain-j event k is the first
// chain-j descendant of chain-c positions (LA[(j, k-1)][c], LA[(j, k)][c]] -- the same
// runs, stored straight into both layouts (FDT stays the runs table later batches
// transpose from)
template <int NP>
__global__ void __launch_bounds__(256) k_la_seq(Tables t, int n0, int n1, const UpEv* up, UpDst dst,
                                                const int32_t* qolen, const int32_t* qlen, int32_t* qlo,
                                                int32_t* fst, int32_t* fst_lo, int32_t* fdt) {
  __shared__ int rows[LASEQ_MAX];
  __shared__ int2 par[LASEQ_MAX / NP];
  if (fst && blockIdx.x == gridDim.x - 1) {
    frontier_start_body(t, qolen, qlen, fst, fst_lo, nullptr, nullptr, 0);
    return;
  }
  if (blockIdx.x > 0) {
    fd_qlo_body(t, qolen, qlen, qlo, blockIdx.x - 1);
    return;
  }
  constexpr int G = 256 / NP;
  const int N = t.N, m = n1 - n0;
  const int tid = threadIdx.x, i = tid % NP;
  for (int x = n0 + tid; x < n1; x += 256) chain_fill_one(t, x, n0, up, dst);
  __syncthreads();
  for (int e = tid / NP; e < m; e += G) {
    const int x = n0 + e;
    const int cx = t.creator[x], px = t.index[x];
    const int s = px > 0 ? t.chain[(size_t)cx * t.ccap + px - 1] : -1;
    const int2 oc = t.opcp[(size_t)cx * t.ccap + px];
    const int o = oc.x >= 0 ? t.chain[(size_t)oc.x * t.ccap + oc.y] : -1;
    int v = -1;
    if (i < N) {
      if (s >= 0 && s < n0) v = t.LA[rowoff(t, cx, px - 1) + i];
      if (o >= 0 && o < n0) v = max(v, t.LA[rowoff(t, oc.x, oc.y) + i]);
      if (i == cx) v = max(v, px);
    }
    rows[e * NP + i] = v;
    if (i == 0) par[e] = make_int2(s >= n0 ? s - n0 : -1, o >= n0 ? o - n0 : -1);
  }
  __syncthreads();
  if (tid < NP) {
    for (int e = 0; e < m; e++) {
      const int2 pp = par[e];
      const int a = pp.x >= 0 ? rows[pp.x * NP + i] : -1;
      const int b = pp.y >= 0 ? rows[pp.y * NP + i] : -1;
      rows[e * NP + i] = max(rows[e * NP + i], max(a, b));
    }
  }
  __syncthreads();
  for (int e = tid / NP; e < m; e += G) {
    const int x = n0 + e;
    if (i < N) t.LA[rowoff(t, t.creator[x], t.index[x]) + i] = rows[e * NP + i];
  }
  if (!fdt) return;
  const size_t ccap = t.ccap;
  for (int e = tid / NP; e < m; e += G) {  // thread i: chain j = i of the new position
    const int x = n0 + e, cx = t.creator[x], px = t.index[x];
    if (i < N) {
      t.FD[rowoff(t, cx, px) + i] = INF32;
      fdt[((size_t)i * N + cx) * ccap + px] = INF32;
    }
  }
  __syncthreads();  // (global, block scope) the runs below overwrite some of them
  for (int e = tid / NP; e < m; e += G) {  // thread i: column c = i
    const int x = n0 + e, j = t.creator[x], k = t.index[x];
    if (i < N) {
      const int2 pp = par[e];
      int lo = -1;
      if (k > 0) lo = pp.x >= 0 ? rows[pp.x * NP + i] : t.LA[rowoff(t, j, k - 1) + i];
      const int hi = rows[e * NP + i];
      for (int q = lo + 1; q <= hi; q++) {
        t.FD[rowoff(t, i, q) + j] = k;
        fdt[((size_t)j * N + i) * ccap + q] = k;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Packed 16-bit sweeps (N > 32 while every chain holds at most 65,534 events; past
// that the engine switches to the int32 tables for good, hge_wide32.hip):
// the fixed-point sweeps run on LA16, a table of (LA + 1) as uint16 pairs
// (NW2 = ceil(N / 2) words per row, -1 -> 0), so every sweep streams half the
// bytes of the int32 sweep; k_la16_rows_runs then writes the int32 LA rows and
// the FDT runs from it in one pass.  Same segments, order and fixed-point argument
// as k_la_sweep: max over packed halves is max over each column.
// ---------------------------------------------------------------------------
__device__ __forceinline__ size_t rowoff16(const Tables& t, int c, int p) {
  return ((size_t)c * t.ccap + p) * (size_t)t.NW2;
}

// also resets the segments' last-changed sweeps (dirty[0, ndirty) = -2: none yet)
__global__ void k_la_clear16(Tables t, const int32_t* olen, const int32_t* len, int32_t* zero, int nzero,
                             int32_t* dirty, int ndirty) {
  const int j = blockIdx.y;
  const int W = t.NW2;
  if (j == 0 && blockIdx.x == 0)
    for (int i = threadIdx.x; i < nzero; i += blockDim.x) zero[i] = 0;
  if (dirty && j == (int)gridDim.y - 1 && blockIdx.x == 0)
    for (int i = threadIdx.x; i < ndirty; i += blockDim.x) dirty[i] = -2;
  const int64_t lo = (int64_t)olen[j] * W, hi = (int64_t)len[j] * W;
  uint32_t* base = t.LA16 + (size_t)j * t.ccap * W;
  for (int64_t e = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < hi;
       e += (int64_t)gridDim.x * blockDim.x)
    base[e] = 0u;
}

//
// Segment skipping (dirty != nullptr): dirty[s] = the last sweep in which
// segment s (chain-major numbering: segbase[c] + (p - olen[c]) / SEG) changed a
// row.  Sweep `sweep` recomputes a segment only if one of its inputs -- the
// segment before it on its chain, or a segment holding one of its other
// parents -- changed in the previous sweep or so far in this one (dirty >=
// sweep - 1).  Every change to an input is then followed by a recomputation
// that reads it, so the fixed point and its detection are unchanged; rows
// below olen are final and never dirty.
template <int NP>  // NP lanes (packed words) per segment
__global__ void __launch_bounds__(256) k_la_sweep16(Tables t, const int2* segs, int nseg, int SEG,
                                                    const int32_t* len, const int32_t* prev,
                                                    int32_t* changed, const int32_t* olen,
                                                    const int32_t* segbase, int32_t* dirty, int sweep) {
  constexpr int G = 256 / NP;
  constexpr int SEGMAX = 64;
  constexpr int U = 32;  // loads in flight per lane and batch
  __shared__ int64_t s_off[G][SEGMAX];
  __shared__ int s_need[G];
  if (prev && *prev == 0) return;  // converged: the flag stays 0
  const int W = t.NW2;
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
  const bool skip = dirty != nullptr && sweep > 0;
  int sid = 0;
  if (skip) {
    if (valid) sid = segbase[j] + (k0 - olen[j]) / SEG;
    // the segment before this one on its chain
    if (i == 0) s_need[g] = valid && k0 > olen[j] && dirty[sid - 1] >= sweep - 1;
    __syncthreads();
  }
  for (int kk = i; kk < SEG; kk += NP) {
    int64_t off = -1;
    if (valid && k0 + kk < k1) {
      const int2 o = t.opcp[(size_t)j * t.ccap + k0 + kk];
      if (o.x >= 0) {
        off = (int64_t)rowoff16(t, o.x, o.y);
        if (skip) {
          const int ol = olen[o.x];
          if (o.y >= ol && dirty[segbase[o.x] + (o.y - ol) / SEG] >= sweep - 1) s_need[g] = 1;
        }
      }
    }
    s_off[g][kk] = off;
  }
  __syncthreads();
  const bool act = valid && i < W && (!skip || s_need[g]);
  bool ch = false;
  if (act) {
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    // the own column j lives in word j / 2, half j & 1
    const bool ownw = i == (j >> 1);
    const int own_shift = (j & 1) * 16;
    const size_t own0 = rowoff16(t, j, k0) + i;
    u16x2 v = (k0 > 0) ? __builtin_bit_cast(u16x2, t.LA16[own0 - W]) : u16x2{0, 0};
    for (int kb = k0; kb < k1; kb += U) {
      uint32_t a[U], old[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = kb + u;
        a[u] = 0;
        old[u] = 0;
        if (k < k1) {
          const int64_t off = s_off[g][k - k0];
          if (off >= 0) a[u] = t.LA16[off + i];
          old[u] = t.LA16[own0 + (size_t)(k - k0) * W];
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int k = kb + u;
        if (k < k1) {
          v = __builtin_elementwise_max(v, __builtin_bit_cast(u16x2, a[u]));
          if (ownw) v = __builtin_elementwise_max(v, __builtin_bit_cast(u16x2, (uint32_t)(k + 1) << own_shift));
          const u16x2 nv = __builtin_elementwise_max(v, __builtin_bit_cast(u16x2, old[u]));
          v = nv;
          const uint32_t nw = __builtin_bit_cast(uint32_t, nv);
          if (nw != old[u]) {
            t.LA16[own0 + (size_t)(k - k0) * W] = nw;
            ch = true;
          }
        }
      }
    }
  }
  const uint64_t bal = __ballot(ch);
  if (bal && (threadIdx.x & 63) == __builtin_ctzll(bal)) *changed = 1;
  if (dirty) {
    // one lane per (wave, segment) with a change: NP = 32 puts two segments in a wave
    const int lane = threadIdx.x & 63;
    const uint64_t grp = NP >= 64 ? ~0ull : (0xFFFFFFFFull << (lane & 32));
    if ((bal & grp) && lane == __builtin_ctzll(bal & grp)) {
      if (!skip) sid = segbase[j] + (k0 - olen[j]) / SEG;
      dirty[sid] = sweep;
    }
  }
}

// N > 32: the FDT runs from LA16 tiles (a transpose to LAT + k_fdt_runs without the
// LAT table in between; the int32 LA rows are never materialised): chain-j event k
// (new) is the first chain-j descendant of chain-c positions
// (LA[(j, k-1)][c], LA[(j, k)][c]], written as FDT[j][c][q] = k; the new chain-c
// positions past LA[(j, len_j - 1)][c] get INF32 (no chain-j descendant yet);
// every other new position lies in a new event's run.  Tile: positions
// [p0, p0 + 64) of chain j (from plo_j = olen_j - 1: the row before the first
// new event is the first run's lower bound) x columns [c0, c0 + 64).
// FT = int32_t (INF32 = none) or uint16_t (0xFFFF = none; N > 128, FD transpose only).
// L32: the tile from the int32 LA rows (N <= 32, or a wide hashgraph past the uint16
// positions), in place of round 3's transpose to a LAT table and a runs kernel over it.
template <typename FT, bool L32 = false>
__global__ void __launch_bounds__(256) k_la16_rows_runs(Tables t, FT* FDT, const int32_t* plo,
                                                        const int32_t* olen, const int32_t* len) {
  constexpr FT FINF = sizeof(FT) == 2 ? (FT)0xFFFF : (FT)INF32;
  __shared__ int32_t tile[65][65];  // row 0: position p0 - 1; row 1 + r: position p0 + r
  const int N = t.N;
  const size_t ccap = t.ccap;
  // XCD-aware tile order (xcd_block): neighbouring position tiles of a (chain, column
  // tile) write neighbouring q ranges of the same 64 FDT rows, and now run on one XCD,
  // whose L2 merges the cache lines they share instead of writing partial lines from two
  const int64_t gxy = (int64_t)gridDim.x * gridDim.y;
  const int64_t lb = xcd_block(blockIdx.x + (int64_t)gridDim.x * blockIdx.y + gxy * blockIdx.z, gxy * gridDim.z);
  const int bz = (int)(lb / gxy), by = (int)((lb - bz * gxy) / gridDim.x), bx = (int)(lb - bz * gxy - (int64_t)by * gridDim.x);
  const int j = bz;
  const int lj = len[j], oj = olen[j];
  const int p0 = plo[j] + bx * 64;
  const int c0 = by * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  if (lj == 0) {  // empty chain: every new position of every chain c has no chain-j descendant
    if (bx == 0)
      for (int cc = ty; cc < 64; cc += 4) {
        const int c = c0 + cc;
        if (c >= N) continue;
        FT* row = FDT + ((size_t)j * N + c) * ccap;
        for (int q = olen[c] + tx; q < len[c]; q += 64) row[q] = FINF;
      }
    return;
  }
  if (p0 >= lj) return;
  // rows p0 - 1 .. p0 + 63: 32 packed words = 64 columns; lanes 0..31 take one word of
  // row r, lanes 32..63 the same word of row r + 1.  All of a thread's loads are
  // issued before the first LDS store (the loop as written compiled to one load and a
  // vmcnt(0) wait per row pair: nine serial memory latencies per tile)
  if constexpr (L32) {
    // 65 rows x 64 columns, lane = column: 17 loads per thread, all in flight
    constexpr int NIT = 17;  // 256 * 17 >= 65 * 64
    int xv[NIT];
#pragma unroll
    for (int i = 0; i < NIT; i++) {
      const int idx = (int)threadIdx.x + 256 * i, rr = idx >> 6, c = c0 + (idx & 63);
      const int p = p0 - 1 + rr;
      const bool ok = rr < 65 && p >= 0 && p < lj && c < N;
      xv[i] = ok ? t.LA[((size_t)j * ccap + p) * N + c] : -1;
    }
#pragma unroll
    for (int i = 0; i < NIT; i++) {
      const int idx = (int)threadIdx.x + 256 * i, rr = idx >> 6;
      if (rr < 65) tile[rr][idx & 63] = xv[i];
    }
  } else {
    constexpr int NIT = 9;  // r = 2 ty + 8 i < 66
    uint32_t xv[NIT];
#pragma unroll
    for (int i = 0; i < NIT; i++) {
      const int rr = 2 * ty + 8 * i + (tx >> 5), w = tx & 31;
      const int p = p0 - 1 + rr, c = c0 + 2 * w;
      const bool ok = rr < 65 && p >= 0 && p < lj && c < N;
      xv[i] = ok ? t.LA16[rowoff16(t, j, ok ? p : 0) + (ok ? (c >> 1) : 0)] : 0u;  // 0: -1 after unpacking
    }
#pragma unroll
    for (int i = 0; i < NIT; i++) {
      const int rr = 2 * ty + 8 * i + (tx >> 5), w = tx & 31;
      if (rr < 65) {
        tile[rr][2 * w] = (int)(xv[i] & 0xFFFFu) - 1;
        tile[rr][2 * w + 1] = (int)(xv[i] >> 16) - 1;
      }
    }
  }
  __syncthreads();
  // runs: wave ty takes columns ty, ty + 4, ...; lane = position k = p0 + tx.  (Writing
  // each column's contiguous q range with consecutive lanes, bisecting for the event
  // of each q, measured no faster: 7.4 vs 6.7-7.3 ms at 256/10M.)
  const int k = p0 + tx;
  const bool isnew = k >= oj && k < lj;
  const bool lasttile = lj - 1 < p0 + 64;
  for (int cc = ty; cc < 64; cc += 4) {
    const int c = c0 + cc;
    if (c >= N) break;
    FT* row = FDT + ((size_t)j * N + c) * ccap;
    if (isnew) {
      const int hi = tile[tx + 1][cc];
      const int lo = k > 0 ? tile[tx][cc] : -1;
      for (int q = lo + 1; q <= hi; q++) row[q] = (FT)k;
    }
    if (lasttile) {
      const int tail0 = max(olen[c], tile[lj - p0][cc] + 1);
      for (int q = tail0 + tx; q < len[c]; q += 64) row[q] = FINF;
    }
  }
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
  const int pend = len[a];
  const int c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  // position tiles past the grid loop (the host sizes it without reading plo)
  for (int p0 = plo[a] + blockIdx.x * 64; p0 < pend; p0 += gridDim.x * 64) {
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
  __syncthreads();
  }
}

// k_transpose mode 1 plus the timestamps (N > 16, the wide median):
// FDT[j][c][q] -> FD[(c, q)][j] and FDTD[(c, q)][j] = ts of the event (j, FD) - ts of
// (c, q), as int32 (half the bytes of the timestamps themselves; a row tile with an
// offset outside int32 is flagged in FDTW and the median gathers exact timestamps).
// The timestamp gathers sit in the read phase, where a wave walks one chain j
// along q and FD is non-decreasing: neighbouring lanes read neighbouring tsch
// cells of that chain (a few cache lines per wave), not one chain per lane.
// tlo/thi (a split part, may be null): the timestamp rows are written for chain
// positions [tlo_c, thi_c) only -- the part's own candidates; FD rows for all.
template <typename FT>
__global__ void __launch_bounds__(256) k_fd_transpose_ts(Tables t, const FT* FDT, const int32_t* plo,
                                                         const int32_t* len, const int32_t* tlo,
                                                         const int32_t* thi) {
  __shared__ int32_t tile[64][65];
  __shared__ int32_t toff[64][65];  // the offsets (INT32_MIN: outside int32)
  const int N = t.N;
  const size_t ccap = t.ccap;
  // grid (chain, column tile, position tiles): consecutive workgroups take the same
  // positions of different source chains, whose first descendants (and so the
  // timestamps gathered) lie in the same stretch of each chain j -- L2 hits
  // instead of one re-read per source chain.  Position tiles past gridDim.z loop.
  // (in XCD-aware order: the neighbouring source chains of a position tile run on one
  // XCD, so the gathers they share hit its L2)
  const int64_t nbk = (int64_t)gridDim.x * gridDim.y * gridDim.z;
  const int64_t lb = xcd_block(blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z), nbk);
  const int bx = (int)(lb % gridDim.x), by = (int)((lb / gridDim.x) % gridDim.y), bz = (int)(lb / ((int64_t)gridDim.x * gridDim.y));
  const int a = bx;  // source chain c
  const int pend = len[a];
  const int ts0 = tlo ? tlo[a] : 0, ts1 = thi ? thi[a] : pend;
  const int c0 = by * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  // uint16 runs: tiles start at a multiple of 4 positions, so a lane reads 4 of them
  // with one 8-byte load (the rows below plo it re-writes hold their final values)
  const int pb = sizeof(FT) == 2 ? (plo[a] & ~3) : plo[a];
  for (int p0 = pb + bz * 64; p0 < pend; p0 += gridDim.z * 64) {
    if constexpr (sizeof(FT) == 2) {
      // read phase: thread i takes row jj = c0 + (i >> 4) + 16 h, positions
      // p0 + 4 (i & 15) .. + 3 (16 lanes per 128-byte row segment, 4 rows per wave)
      __shared__ int64_t s_own[64];
      if (threadIdx.x < 64) s_own[threadIdx.x] = t.tsch[(size_t)a * ccap + min(p0 + (int)threadIdx.x, pend - 1)];
      const int qd = threadIdx.x & 15, r0 = threadIdx.x >> 4;
      uint2 w[4];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int jj = c0 + r0 + 16 * h, q = p0 + 4 * qd;
        w[h] = (jj < N && q < pend) ? *(const uint2*)(FDT + ((size_t)jj * N + a) * ccap + q) : make_uint2(~0u, ~0u);
      }
      int kv[16];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const uint32_t lo = w[h].x, hi = w[h].y;
        const uint32_t u[4] = {lo & 0xFFFFu, lo >> 16, hi & 0xFFFFu, hi >> 16};
#pragma unroll
        for (int e = 0; e < 4; e++) kv[4 * h + e] = (u[e] == 0xFFFFu || p0 + 4 * qd + e >= pend) ? INF32 : (int)u[e];
      }
      int64_t tv[16];
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int jj = c0 + r0 + 16 * h;
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int qq = p0 + 4 * qd + e;
          const bool tson = qq >= ts0 && qq < ts1;
          tv[4 * h + e] = tson && kv[4 * h + e] != INF32 ? t.tsch[(size_t)(jj < N ? jj : 0) * ccap + kv[4 * h + e]] : 0;
        }
      }
      __syncthreads();  // s_own
#pragma unroll
      for (int h = 0; h < 4; h++) {
        const int r = r0 + 16 * h;
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int col = 4 * qd + e;
          const int k = kv[4 * h + e];
          const int qq = p0 + col;
          tile[r][col] = k;
          const int64_t dlt = tv[4 * h + e] - s_own[col];
          const bool esc = dlt < -(int64_t)INT32_MAX || dlt > (int64_t)INT32_MAX;
          toff[r][col] = (k == INF32 || qq < ts0 || qq >= ts1) ? 0 : (esc ? INT32_MIN : (int32_t)dlt);
        }
      }
    } else {
    // read phase: lane tx walks row q = p0 + tx (its own timestamp is one load), all
    // 16 FDT loads of a thread in flight, then all 16 timestamp gathers
    const int64_t own = t.tsch[(size_t)a * ccap + min(p0 + tx, pend - 1)];
    constexpr int CH = 16;  // rows in flight per thread
#pragma unroll
    for (int h = 0; h < 16; h += CH) {
      int kv[CH];
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const int jj = c0 + ty + 4 * (h + i), q = p0 + tx;
        if (jj < N && q < pend) {
          const FT f = FDT[((size_t)jj * N + a) * ccap + q];
          kv[i] = (sizeof(FT) == 2 && f == (FT)0xFFFF) ? INF32 : (int)f;
        } else {
          kv[i] = INF32;
        }
      }
      int64_t tv[CH];
      const bool tson = p0 + tx >= ts0 && p0 + tx < ts1;
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const int jj = c0 + ty + 4 * (h + i);
        tv[i] = tson ? t.tsch[(size_t)(jj < N ? jj : 0) * ccap + (kv[i] != INF32 ? kv[i] : 0)] : own;
      }
#pragma unroll
      for (int i = 0; i < CH; i++) {
        tile[ty + 4 * (h + i)][tx] = kv[i];
        const int64_t d = tv[i] - own;  // offset from the row event's own timestamp
        const bool esc = d < -(int64_t)INT32_MAX || d > (int64_t)INT32_MAX;
        toff[ty + 4 * (h + i)][tx] = kv[i] == INF32 ? 0 : (esc ? INT32_MIN : (int32_t)d);
      }
    }
    }
    __syncthreads();
    const int NT = (N + 63) >> 6;
    for (int r = ty; r < 64; r += 4) {  // wave ty writes rows r: the 64 columns of one row each time
      const int q = p0 + r, jj = c0 + tx;
      const bool tsrow = q >= ts0 && q < ts1;  // wave-uniform
      bool esc = false;
      if (q < pend && jj < N) {
        const size_t o = rowoff(t, a, q) + jj;
        const int32_t dv = toff[tx][r];
        esc = dv == INT32_MIN;  // a real offset lies in [-INT32_MAX, INT32_MAX]
        // streaming stores: 20 GB per 256/10M replay, read back only by later kernels
        // (7.24-7.28 vs 7.40-7.41 ms in a same-box A/B; the runs kernel's scattered short
        // runs need the L2 to merge their lines: 18.9 vs 6.55 ms with streaming stores)
        if constexpr (sizeof(FT) == 2) {  // uint16 runs: the FD rows packed (FD + 1, 0xFFFF = none)
          const int f = tile[tx][r];
          __builtin_nontemporal_store((uint16_t)(f == INF32 ? 0xFFFFu : (uint32_t)f + 1), t.FD16 + o);
        } else {
          __builtin_nontemporal_store(tile[tx][r], t.FD + o);
        }
        if (tsrow) __builtin_nontemporal_store(dv, t.FDTD + o);
      }
      const bool any = __ballot(esc) != 0;
      if (tx == 0 && q < pend && tsrow) t.FDTW[((size_t)a * ccap + q) * NT + by] = any ? 1 : 0;
    }
    __syncthreads();
  }
}

// the uint16 tables widened to int32 at the switch to int32 positions: runs
// (0xFFFF -> INF32, else the value) and FD rows (0xFFFF -> INF32, else value - 1)
__global__ void k_fdt16_to32(const uint16_t* src, int32_t* dst, size_t n, int bias) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i] == 0xFFFFu ? INF32 : (int32_t)src[i] - bias;
}

__global__ void __launch_bounds__(256) k_fd_qlo(Tables t, const int32_t* olen, const int32_t* len, int32_t* qlo) {
  fd_qlo_body(t, olen, len, qlo, blockIdx.x);
}
// k_chain_fill (blocks [0, nfb)) and k_fd_qlo (the N blocks after) in one launch:
// the row bounds read only the old events' LA rows, which the batch leaves alone
// fst (non-null): the last block takes k_frontier_start's work for the wide rounds
// walk (its first round, zeroed hand-off flags and granules; old rows only)
__global__ void __launch_bounds__(256) k_chain_fill_qlo(Tables t, int n0, int n1, const UpEv* up, UpDst dst, int nfb,
                                                        const int32_t* olen, const int32_t* len, int32_t* qlo,
                                                        int32_t* fst, int32_t* zbar, uint64_t* zgran, int ngran) {
  if (fst && blockIdx.x == gridDim.x - 1) {
    frontier_start_body(t, olen, len, fst, nullptr, zbar, zgran, ngran);
  } else if ((int)blockIdx.x < nfb) {
    const int x = n0 + blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n1) chain_fill_one(t, x, n0, up, dst);
  } else {
    fd_qlo_body(t, olen, len, qlo, blockIdx.x - nfb);
  }
}

}  // namespace hge
