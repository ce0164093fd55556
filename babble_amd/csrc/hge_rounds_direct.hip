// hge_rounds_direct.hip — DivideRounds for wide hashgraphs (N > 32) by batched
// strongly-see tiles: the frontier recurrence of DESIGN.md §4.2 evaluated
// directly on the coordinate rows, one co-resident workgroup per chain.
//
//   C_{r+1}[c] = min { p >= C_r[c] : #{d : StronglySee((c, p), m_d)} >= SM },
//   StronglySee(x, m) = #{i : LA[x][i] >= FD[m][i]} >= SM   (hashgraph.go:180-208)
//
// where m_d = (d, C_r[d]) are the round-r frontier members.  StronglySee is
// monotone along a chain (LA rows only grow), so the first position is found
// by bisection over a window of candidate rows of chain c.
//
// Per round and workgroup (target chain c):
//   * thread (d, part) holds its slice of member row FD[m_d] in registers as
//     packed uint16 (FD + 1, 0xFFFF = unset / no member);
//   * the candidate rows LA[(c, p)], p in [C_r[c], C_r[c] + W), sit in LDS as
//     packed uint16 (LA + 2), staged while the previous round's hand-off was in
//     flight (they are chain c's own rows: known as soon as C_{r+1}[c] is);
//   * a probe of position p is one pass of packed saturating subtractions
//     (la + 2 -sat m + 1 > 0  <=>  la >= m) over the member slice, a sum over
//     the TPM lanes of a member, a wave ballot of the members that pass and
//     one LDS add per wave: a W x N x N strongly-see tile costs log2(W) + 1
//     probes, all compares on registers and LDS (no gathers).
// The strongly-see bits of the selected event against every member (ssc: the
// vote adjacency k_witness_bits consumes) are one more probe.
//
// The frontier hand-off between workgroups is the granule protocol of
// hge_rounds_coop.hip (8-byte {epoch, value} granules, relaxed agent-scope
// stores and loads, double-buffered by round parity; cdna_hip_programming.md
// Guideline 16, R2).  Chain positions must fit uint16 with room for the +2
// encoding: the engine runs this kernel only while every chain holds at most
// 65,534 events; a longer chain switches it to int32 positions for good
// (hge_wide32.hip, k_round_step32).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hge {

// section stamps (HGE_STAMPS) are compiled in only with -DHGE_DIR_STAMPS: the
// accumulators otherwise cost registers (and spills) in the round loop
#ifdef HGE_DIR_STAMPS
constexpr bool kDirStamps = true;
#else
constexpr bool kDirStamps = false;
#endif
constexpr int DIR_MAXP = 16;  // probe counters per window (2 + log2(W) are used)
constexpr int DIR_CH = 32;    // rows per fetch chunk (a round advances ~EPR/N ~ 14 rows)

template <int BS, int NPOW>
struct DirGeo {
  // candidate rows staged per window: 64 for 1024-thread workgroups (one per CU), 32 for
  // 512-thread ones (two per CU, e.g. two walkers of one hashgraph side by side)
  static constexpr int W = BS >= 1024 ? 64 : 32;
  static constexpr int TPM = BS / NPOW;       // threads per member
  static constexpr int CPT = NPOW / TPM;      // columns per thread (NPOW^2 / BS)
  static constexpr int CW = CPT / 2;          // packed words per thread
  static constexpr int VW = (CW % 4 == 0) ? 4 : 2;  // words per LDS read (b128 / b64)
  static constexpr int PS = CW + VW;          // LDS words per (row, part): parts on distinct banks
  static constexpr int RS = TPM * PS;         // LDS words per candidate row
  static constexpr int WIN_INTS = W * NPOW;      // ints of a full window (N = NPOW)
  static constexpr int PREF = (DIR_CH * NPOW / 4 + BS - 1) / BS;  // int4 per thread and chunk
  static constexpr int MBW = NPOW / 2;        // staged member row: packed words
  static constexpr int MVW = (CW % 4 == 0) ? 4 : 2;  // MB words per thread chunk (16 / 8 bytes)
};

template <int BS, int NPOW>
struct DirLDS {
  int sP[256];
  uint32_t sLA[DirGeo<BS, NPOW>::W * DirGeo<BS, NPOW>::RS] __attribute__((aligned(16)));
  int sCnt[DIR_MAXP];
  int sCntW[DIR_MAXP][BS / 64] __attribute__((aligned(16)));  // per-wave passing members of a probe
  int sHist[DirGeo<BS, NPOW>::W / 2];  // members by first passing offset (dir_select_pm)
  uint32_t sBits[8];
  int sFlag[2];          // per round parity: 1 = some member exists, 2 = some chain below stopcut, 4 = hand-off failed
  int s_stamp;          // HGE_STAMPS: thread 0 accumulates probe phases into sdbg
  uint64_t sdbg[2];     // [0] count (LDS reads + VALU), [1] reduce + barrier + read
};

__device__ __forceinline__ uint32_t dir_pack_la(int a, int b) {
  return (uint32_t)(a + 2) | ((uint32_t)(b + 2) << 16);
}
__device__ __forceinline__ uint32_t dir_pack_fd(int a, int b) {
  const uint32_t lo = a == INF32 ? 0xFFFFu : (uint32_t)(a + 1);
  const uint32_t hi = b == INF32 ? 0xFFFFu : (uint32_t)(b + 1);
  return lo | (hi << 16);
}

// The candidate rows live in an LDS ring of W rows: row p of chain c sits in
// slot p % W, and the ring holds [lo, lo + W) for the current lo.  Moving
// the window from lo to lo' only fetches rows [max(lo + W, lo'), lo' + W): ~EPR/N
// rows per round instead of W.
// dir_fetch: rows [p0, p0 + min(nr, DIR_CH)) of chain c into registers (8-byte slices of
// the contiguous chain-major packed rows; rows >= lenc become "no row").  N % 4 == 0
// (the host takes the gather path of hge_rounds_coop.hip otherwise).
template <int BS, int NPOW>
__device__ __forceinline__ void dir_fetch(const Tables& t, int c, int p0, int nr, int lenc,
                                          uint2 (&v)[DirGeo<BS, NPOW>::PREF]) {
  using G = DirGeo<BS, NPOW>;
  const int N = t.N;
  nr = min(nr, DIR_CH);
  const int have = (p0 == INF32 || nr <= 0) ? 0 : max(0, min(nr, lenc - p0));
  if (have == 0) return;  // block-uniform
  // the packed rows (LA + 1 as uint16 pairs, N / 2 words per row): 4 columns = 8 bytes
  const uint32_t* base = t.LA16 + ((size_t)c * t.ccap + p0) * (size_t)t.NW2;
  // unconditional loads (rows past `have` re-read the last fetched row; dir_store
  // drops them): no value select behind each load, so all of them stay in flight
  const int qmax = have * N / 4 - 1;
#pragma unroll
  for (int m = 0; m < G::PREF; m++) {
    const int q = min((int)threadIdx.x + m * BS, qmax);  // 4-column group in the fetched rows
    v[m] = *(const uint2*)(base + 2 * (size_t)q);
  }
}

// the fetched rows [p0, p0 + nr) -> their ring slots (caller syncs before a
// probe); rows at or past lenc are stored as "no row" (0: never >= a member value)
template <int BS, int NPOW>
__device__ __forceinline__ void dir_store(const Tables& t, DirLDS<BS, NPOW>& L, int p0, int nr, int lenc,
                                          uint2 (&v)[DirGeo<BS, NPOW>::PREF]) {
  using G = DirGeo<BS, NPOW>;
  const int N = t.N;
  if (p0 == INF32 || nr <= 0) return;
  nr = min(nr, DIR_CH);
  const int have = max(0, min(nr, lenc - p0));
#pragma unroll
  for (int m = 0; m < G::PREF; m++) {
    const int q = threadIdx.x + m * BS;
    const int row = (4 * q) / N;
    if (row >= nr) continue;
    // LA16 + 1 per half = the LA + 2 encoding (LA <= 65,533: no carry); a row past the
    // chain's end is "no row" (0)
    const bool hv = row < have;
    // the 4 columns lie in one part (CPT is a multiple of 4).  Columns past N are
    // never written: their member values are 0xFFFF, which no row value passes.
    const int col = 4 * q - row * N;
    const int part = col / G::CPT, w = (col - part * G::CPT) / 2;
    const int slot = (p0 + row) & (DirGeo<BS, NPOW>::W - 1);
    uint2* dst = (uint2*)(L.sLA + slot * G::RS + part * G::PS + w);
    *dst = hv ? make_uint2(v[m].x + 0x00010001u, v[m].y + 0x00010001u) : make_uint2(0u, 0u);
  }
}

// rows [p0, p0 + nr) into their ring slots, chunk by chunk (caller syncs before a probe)
template <int BS, int NPOW>
__device__ __forceinline__ void dir_load(const Tables& t, DirLDS<BS, NPOW>& L, int c, int p0, int nr, int lenc,
                                         uint2 (&v)[DirGeo<BS, NPOW>::PREF]) {
  if (p0 == INF32) return;
  for (int q = 0; q < nr; q += DIR_CH) {
    dir_fetch<BS, NPOW>(t, c, p0 + q, nr - q, lenc, v);
    dir_store<BS, NPOW>(t, L, p0 + q, nr - q, lenc, v);
  }
}

// member slice of thread (d, part) for the first round: FD[(d, Pd)][part * CPT, +CPT)
// packed (FD + 1); N % 4 == 0, so every int4 is wholly inside or past the row
template <int BS, int NPOW>
__device__ __forceinline__ void dir_members_fd(const Tables& t, int d, int part, int Pd,
                                               uint32_t (&mw)[DirGeo<BS, NPOW>::CW]) {
  using G = DirGeo<BS, NPOW>;
  const int N = t.N;
  const int c0 = part * G::CPT;
  const bool act = d < N && Pd != INF32;
  if (t.FD16) {  // the rows are stored packed already (FD + 1, 0xFFFF = none)
    const uint16_t* row = t.FD16 + rowoff(t, act ? d : 0, act ? Pd : 0);
#pragma unroll
    for (int k = 0; k < G::CW / 2; k++) {
      uint2 a = *(const uint2*)(row + min(c0 + 4 * k, N - 4));
      if (!act || c0 + 4 * k >= N) a = make_uint2(~0u, ~0u);
      mw[2 * k] = a.x;
      mw[2 * k + 1] = a.y;
    }
    return;
  }
  const int32_t* row = t.FD + rowoff(t, act ? d : 0, act ? Pd : 0);
#pragma unroll
  for (int k = 0; k < G::CW / 2; k++) {
    // unconditional loads from a valid address, then the select
    int4 a = *(const int4*)(row + min(c0 + 4 * k, N - 4));
    if (!act || c0 + 4 * k >= N) a = make_int4(INF32, INF32, INF32, INF32);
    mw[2 * k] = dir_pack_fd(a.x, a.y);
    mw[2 * k + 1] = dir_pack_fd(a.z, a.w);
  }
}

// Member rows after the first round come from the staging block MB[parity]:
// the workgroup of chain d packs its next frontier row FD[(d, C_{r+1}[d])] there
// (wave 0, write-through 8-byte stores, vmcnt(0), then the granule).  MB is laid
// out by consuming thread, chunk-major: word (k * BS + tid) * MVW + s holds word
// k * MVW + s of thread tid's slice, so load k of a wave reads one contiguous
// 64 * 4 * MVW bytes (a row-major block made every wave load touch 64 cache
// lines for 16 bytes each: TA-bound, ~13k cycles per round at N = 256).  The
// granule poll is the flag; every load of the block is an sc1 load, as the
// granule protocol requires (MI355X_MICROARCH.md, Valid forms, row 1).
template <int BS, int NPOW>
__device__ __forceinline__ void dir_members_mb(const uint32_t* mb, uint32_t (&mw)[DirGeo<BS, NPOW>::CW]) {
  using G = DirGeo<BS, NPOW>;
  constexpr int MVW = G::MVW;
  // buffer_load sc1 (aux bit 4; the table row allows 4-, 8- and 16-byte loads of
  // 8-byte sc1 stores); 8-byte loads run at 0.54-0.70x the 16-byte rate
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)mb, 0, BS * G::CW * 4, 0x00020000);
#pragma unroll
  for (int k = 0; k < G::CW / MVW; k++) {
    const int off = (k * BS + (int)threadIdx.x) * MVW * 4;
    if constexpr (MVW == 4) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
      mw[4 * k] = x.x;
      mw[4 * k + 1] = x.y;
      mw[4 * k + 2] = x.z;
      mw[4 * k + 3] = x.w;
    } else {
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 16);
      mw[2 * k] = x.x;
      mw[2 * k + 1] = x.y;
    }
  }
}

// wave 0 of chain c's workgroup: stage FD[(c, p)] (p = INF32: no member) into MB,
// read from HBM after the pick.  (Round 3 staged every window row's FD row in LDS
// ahead of the pick so the stage read LDS: ~10 GB of the kernel's traffic per
// 256/10M replay for no measured time, 24.57-24.68 vs 24.62-24.69 ms in a
// same-box A/B, profiles/r04/abfd_*.)
// Lane l packs columns 4l .. 4l + 3 into row words 2l, 2l + 1 (one part, one chunk).
template <int BS, int NPOW>
__device__ __forceinline__ void dir_stage_member(const Tables& t, uint32_t* mb, int c, int p) {
  using G = DirGeo<BS, NPOW>;
  constexpr int MVW = G::MVW;
  const int lane = threadIdx.x;  // < 64
  const int N = t.N;
  if (4 * lane < NPOW) {
    unsigned long long x;
    if (t.FD16) {  // stored packed already
      uint2 a = make_uint2(~0u, ~0u);
      if (p != INF32 && 4 * lane < N) a = *(const uint2*)(t.FD16 + rowoff(t, c, p) + 4 * lane);
      x = (unsigned long long)a.x | ((unsigned long long)a.y << 32);
    } else {
      int4 a = make_int4(INF32, INF32, INF32, INF32);
      if (p != INF32 && 4 * lane < N) a = *(const int4*)(t.FD + rowoff(t, c, p) + 4 * lane);
      x = (unsigned long long)dir_pack_fd(a.x, a.y) | ((unsigned long long)dir_pack_fd(a.z, a.w) << 32);
    }
    const int w = 2 * lane, part = w / G::CW, wp = w - part * G::CW;
    const int k = wp / MVW, sub = wp - k * MVW;
    const size_t word = ((size_t)k * BS + (size_t)c * G::TPM + part) * MVW + sub;
    __hip_atomic_store((gu64_t*)(mb + word), x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// strongly-see count of candidate position p (in the ring) against this
// thread's member slice, summed over the member's TPM lanes
template <int BS, int NPOW>
__device__ __forceinline__ int dir_count(const DirLDS<BS, NPOW>& L, int p, int part,
                                         const uint32_t (&mw)[DirGeo<BS, NPOW>::CW]) {
  using G = DirGeo<BS, NPOW>;
  const uint32_t* src = L.sLA + (p & (DirGeo<BS, NPOW>::W - 1)) * G::RS + part * G::PS;
  uint32_t acc0 = 0, acc1 = 0;
  const uint32_t ones = 0x00010001u;
  static_assert(G::CW % 2 == 0, "member slices are whole word pairs");
  static_assert(G::CW % G::VW == 0, "LDS reads cover whole slices");
  // one LDS read of VW words, then its word pairs: only VW row words are live at a
  // time (a 512-thread workgroup holds 64 member words per thread)
#pragma unroll
  for (int k0 = 0; k0 < G::CW; k0 += G::VW) {
    uint32_t la[G::VW];
    if constexpr (G::VW == 4) {
      const uint4 q = *(const uint4*)(src + k0);
      la[0] = q.x;
      la[1] = q.y;
      la[2] = q.z;
      la[3] = q.w;
    } else {
      const uint2 q = *(const uint2*)(src + k0);
      la[0] = q.x;
      la[1] = q.y;
    }
#pragma unroll
    for (int k = 0; k < G::VW; k += 2) {
      // (la + 2) -sat (m + 1) is nonzero <=> la >= m (v_pk_sub_u16 clamp saturates at 0);
      // min(., 1) per half, then a packed add: 3 VALU ops per 2 columns.  Two words per
      // asm statement and two accumulators (no dependent chain, and the compiler's
      // hazard padding between asm statements falls on every other word pair at most)
      uint32_t d0, d1;
      asm("v_pk_sub_u16 %0, %4, %6 clamp\n\t"
          "v_pk_sub_u16 %1, %5, %7 clamp\n\t"
          "v_pk_min_u16 %0, %0, %8\n\t"
          "v_pk_min_u16 %1, %1, %8\n\t"
          "v_pk_add_u16 %2, %2, %0\n\t"
          "v_pk_add_u16 %3, %3, %1"
          : "=&v"(d0), "=&v"(d1), "+v"(acc0), "+v"(acc1)
          : "v"(la[k]), "v"(la[k + 1]), "v"(mw[k0 + k]), "v"(mw[k0 + k + 1]), "v"(ones));
    }
  }
  int cnt = (int)(acc0 & 0xFFFFu) + (int)(acc0 >> 16) + (int)(acc1 & 0xFFFFu) + (int)(acc1 >> 16);
  // sum over the member's TPM consecutive lanes by DPP (no LDS permutes): quad_perm
  // xor 1 and xor 2, then row_half_mirror (quads of an 8) and row_mirror (8s of a row)
  if constexpr (G::TPM > 1) cnt += __builtin_amdgcn_mov_dpp(cnt, 0xB1, 0xF, 0xF, false);
  if constexpr (G::TPM > 2) cnt += __builtin_amdgcn_mov_dpp(cnt, 0x4E, 0xF, 0xF, false);
  if constexpr (G::TPM > 4) cnt += __builtin_amdgcn_mov_dpp(cnt, 0x141, 0xF, 0xF, false);
  if constexpr (G::TPM > 8) cnt += __builtin_amdgcn_mov_dpp(cnt, 0x140, 0xF, 0xF, false);
  static_assert(G::TPM <= 16, "a member's lanes lie in one DPP row");
  return cnt;
}

// one probe: number of members strongly seen by candidate position p; `pass` =
// this thread's member is strongly seen
template <int BS, int NPOW>
__device__ __forceinline__ int dir_probe(const Tables& t, DirLDS<BS, NPOW>& L, int p, int part, int slot,
                                         const uint32_t (&mw)[DirGeo<BS, NPOW>::CW], bool& pass) {
  const bool st = kDirStamps && L.s_stamp && threadIdx.x == 0;
  const uint64_t t0 = st ? stamp() : 0;
  const int cnt = dir_count<BS, NPOW>(L, p, part, mw);
  pass = cnt >= t.SM;
  const uint64_t t1 = st ? stamp() : 0;
  // each wave stores its own count (no same-address LDS atomics serialising the
  // waves ahead of the barrier), then every thread sums the BS / 64 counts
  const uint64_t b = __ballot(part == 0 && pass);
  if ((threadIdx.x & 63) == 0) L.sCntW[slot][threadIdx.x >> 6] = (int)__builtin_popcountll(b);
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < BS / 64; w += 4) {
    const int4 q = *(const int4*)&L.sCntW[slot][w];
    r += q.x + q.y + q.z + q.w;
  }
  if (st) {
    L.sdbg[0] += t1 - t0;
    L.sdbg[1] += stamp() - t1;
  }
  return r;
}

// Probe bisection for the first passing row at or after window offset a (the
// fallback of dir_select: rare).  Every probe counts all members at one row (a
// barrier each); the window's last row is probed first, and when it fails the
// next window is loaded.  pb = this thread's member pass flag at the returned row.
template <int BS, int NPOW>
__device__ int dir_probe_search(const Tables& t, int c, int lenc, DirLDS<BS, NPOW>& L, int part,
                                const uint32_t (&mw)[DirGeo<BS, NPOW>::CW], int& slot,
                                uint2 (&pv)[DirGeo<BS, NPOW>::PREF], int& lo, bool& pb, int a) {
  constexpr int W = DirGeo<BS, NPOW>::W;
  const int SM = t.SM;
  for (;;) {
    const int last = min(W, lenc - lo) - 1;
    if (a <= last) {
      bool ps;
      int b = last;
      if (dir_probe<BS, NPOW>(t, L, lo + b, part, slot++, mw, ps) >= SM) {
        pb = ps;
        while (a < b) {
          const int mid = (a + b) >> 1;
          if (dir_probe<BS, NPOW>(t, L, lo + mid, part, slot++, mw, ps) >= SM) {
            b = mid;
            pb = ps;
          } else {
            a = mid + 1;
          }
        }
        return lo + a;
      }
    }
    if (lo + W >= lenc) return INF32;
    // the answer lies past the window: the whole next window, fresh counters
    lo += W;
    __syncthreads();  // every thread has read this window's counters
    dir_load<BS, NPOW>(t, L, c, lo, W, lenc, pv);
    if (threadIdx.x < DIR_MAXP) L.sCnt[threadIdx.x] = 0;
    slot = 0;
    __syncthreads();
    a = 0;
  }
}

// C_{r+1}[c] before the end-of-chain clamp (INF32 = none yet) from the frontier
// in L.sP, the member slice mw and the window staged at lo (== L.sP[c]).
//
// Per member, not per probe: C_{r+1}[c] - lo is the SM-th smallest of the
// members' first passing offsets T_d = min{k : StronglySee((c, lo + k), m_d)}
// (StronglySee is monotone along the chain, so "count(k) >= SM" <=> "at least
// SM members have T_d <= k").  The TPM lanes of member d bisect T_d over the
// first half of the window on their own -- log2(W/2) counts of their slice
// against rows of the LDS ring, summed over the member's lanes by DPP, no
// barrier between steps -- and one LDS histogram of the T_d plus a wave prefix
// scan gives the SM-th smallest.  The last offset searched, e = min(W/2, rows
// left on the chain) - 1, also stands for "later" (not verified), so an answer
// there (or none) falls back to probe bisection from e on (dir_probe_search).  Round 2's probe bisection paid
// a workgroup barrier, an LDS count exchange and a ballot per probe (five to
// six per round, ~2.5k cycles each at N = 256); the counts here are the same
// N^2 compares per step, with one barrier per round.
// pb = this thread's member is strongly seen by the returned row.
template <int BS, int NPOW>
__device__ int dir_select(const Tables& t, int c, int lenc, DirLDS<BS, NPOW>& L, int d, int part,
                          const uint32_t (&mw)[DirGeo<BS, NPOW>::CW], int& slot,
                          uint2 (&pv)[DirGeo<BS, NPOW>::PREF], int& lo, bool& pb) {
  constexpr int H = DirGeo<BS, NPOW>::W / 2;
  constexpr int STEPS = H == 32 ? 5 : H == 16 ? 4 : 3;
  static_assert((1 << STEPS) == H, "window half is a power of two");
  const int SM = t.SM;
  if (lo == INF32 || lo >= lenc) return INF32;
  // bisect over real rows only: the ring's "no row" entries past the chain's end
  // fail every count, which would break the monotonicity the bisection needs
  const int e = min(H - 1, lenc - lo - 1);
  const bool st = kDirStamps && L.s_stamp && threadIdx.x == 0;
  const uint64_t t0 = st ? stamp() : 0;
  int a = 0, b = e;
#pragma unroll
  for (int s = 0; s < STEPS; s++) {
    const int mid = (a + b) >> 1;
    if (dir_count<BS, NPOW>(L, lo + mid, part, mw) >= SM) b = mid;
    else a = mid + 1;
  }
  // a == b == T_d, exact below e (e stands for "e or later"); members past N do not count
  if (part == 0 && d < t.N) atomicAdd(&L.sHist[a], 1);
  uint64_t t1 = 0;
  if (st) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    t1 = stamp();
  }
  __syncthreads();
  if (st) {  // HGE_STAMPS: [9] this wave's steps, [10] the wait for the other waves
    L.sdbg[0] += t1 - t0;
    L.sdbg[1] += stamp() - t1;
  }
  // every wave: inclusive prefix over the H bins (DPP, HGE_DPP_SCAN: no LDS
  // permutes on the round's critical path), the first bin reaching SM
  const int lane = threadIdx.x & 63;
  int v = lane < H ? L.sHist[lane] : 0;
  HGE_DPP_SCAN(v, dpp_add, 0);
  const uint64_t ge = __ballot(lane < H && v >= SM);
  const int ks = ge ? (int)__builtin_ctzll(ge) : H;
  if (ks < e) {
    pb = a <= ks;
    return lo + ks;
  }
  return dir_probe_search<BS, NPOW>(t, c, lenc, L, part, mw, slot, pv, lo, pb, e);
}

template <int BS, int NPOW>
__global__ void __launch_bounds__(BS, 4) k_rounds_direct(Tables t, const int32_t* olen, const int32_t* len,
                                                      int32_t* rstate, int rlo, const int32_t* rlo_dev,
                                                      int Rprev, uint64_t* gran,
                                                      int32_t* err, uint64_t* ssc, uint32_t* mbuf,
                                                      uint64_t* dbg, const int32_t* start, int32_t* hist,
                                                      int hmax, const int32_t* stopcut, int extra, int stall_ep) {
  // History mode (hist != nullptr; a walker of the cross-GPU split, babble_amd/dist.py):
  // the walk starts at the frontier `start` (rlo = 0, Rprev = 0), writes frontier
  // row j to hist[j * N + c] instead of C, the ssc bits of row j to ssc row j, and
  // stops after row hmax - 1 (rstate[1] = 1), `extra` rows after its frontier
  // first reached stopcut on every chain (the next walker's start; rstate[1] = 2),
  // or at the empty frontier; rstate[0] = rows written.
  // stall_ep > 0 (tests, HGE_TEST_HANDOFF_STALL): at hand-off epoch stall_ep chain 0
  // does not publish and every workgroup gives up at once, as on a timed-out poll, so
  // the other chains' rows of that round are written and chain 0's is not.
  using G = DirGeo<BS, NPOW>;
  // rlo_dev: the first round to recompute, read here (INF32: nothing to do)
  if (rlo_dev) {
    rlo = *rlo_dev;
    if (rlo == INF32) return;
  }
  // HGE_STAMPS diagnostics (workgroup 0, thread 0): cycles per section into dbg[0..8]
  // (6 = probes; 7, 8 = member-load issue and arrival inside section 0)
  uint64_t st_t = 0, st_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const bool stamping = kDirStamps && dbg && blockIdx.x == 0 && threadIdx.x == 0;
#define DSTAMP(k)                  \
  if (stamping) {                  \
    const uint64_t now_ = stamp(); \
    st_acc[(k)] += now_ - st_t;    \
    st_t = now_;                   \
  }
#define DSTAMP_START                \
  if (stamping) st_t = stamp();
  __shared__ DirLDS<BS, NPOW> L;
  const int N = t.N, NW = t.NW;
  const int c = blockIdx.x, tid = threadIdx.x;
  const int d = tid / G::TPM, part = tid - d * G::TPM;
  const int lenc = len[c];
  gu64_t* gr[2] = {(gu64_t*)gran, (gu64_t*)(gran + N)};
  uint32_t* mbp[2] = {mbuf, mbuf + (size_t)NPOW * G::MBW};
  if (tid < N) {
    int P;
    if (hist) {
      P = start[tid];
      if (c == 0) hist[tid] = P;
    } else {
      P = t.C[(size_t)rlo * N + tid];
      if (rlo == 0 && olen[tid] == 0 && len[tid] > 0) P = 0;
      if (c == 0 && rlo == 0 && olen[tid] == 0 && len[tid] > 0) t.C[tid] = 0;
    }
    L.sP[tid] = P;
  }
  if (tid == 0) {
    L.s_stamp = stamping ? 1 : 0;
    L.sdbg[0] = L.sdbg[1] = 0;
  }
  __syncthreads();
  const int rcap = hist ? hmax : t.Rcap;
  int extra_left = -1;  // history mode: rows still to walk after passing stopcut
  uint2 pv[G::PREF];
  int lo = L.sP[c];
  dir_load<BS, NPOW>(t, L, c, lo, DirGeo<BS, NPOW>::W, lenc, pv);
  int f0 = INF32, fn = 0;  // rows fetched for the next round: [f0, f0 + fn)
  // members of the first round from the FD table; later rounds' members are loaded
  // by each wave right after its own poll of the previous round (below)
  uint32_t mw[G::CW];
  dir_members_fd<BS, NPOW>(t, d, part, d < N ? L.sP[d] : INF32, mw);
  for (int r = rlo;; r++) {
    if (r + 1 >= rcap) {
      if (c == 0 && tid == 0) {
        rstate[1] = 1;
        if (hist) rstate[0] = r + 1;  // rows written
      }
      break;
    }
    DSTAMP_START
    if (d >= N) {
#pragma unroll
      for (int k = 0; k < G::CW; k++) mw[k] = 0xFFFFFFFFu;
    }
    if (tid < DIR_MAXP) L.sCnt[tid] = 0;
    if (tid < 8) L.sBits[tid] = 0;
    if (tid < DirGeo<BS, NPOW>::W / 2) L.sHist[tid] = 0;
    if (tid == 0) L.sFlag[(r + 1) & 1] = 0;  // read after the previous round's poll barrier
    __syncthreads();  // window stored, counters clear
    DSTAMP(0);
    const int Pc = L.sP[c];
    const int cur = (r + 1 < Rprev) ? t.C[(size_t)(r + 1) * N + c] : INF32;
    int slot = 0;
    int nxt = INF32;
    bool pb = false, have_bits = false;
    if (Pc != INF32) {
      if (cur != INF32) {
        nxt = cur;
      } else {
        const int s = dir_select<BS, NPOW>(t, c, lenc, L, d, part, mw, slot, pv, lo, pb);
        nxt = s < lenc ? s : INF32;
        have_bits = nxt != INF32;
      }
    }
    DSTAMP(1);
    if (stamping) st_acc[6] += slot;
    // publish C_{r+1}[c]: wave 0 stages the next member row, drains its stores,
    // then lane 0 stores the granule
    const bool stall = stall_ep > 0 && r - rlo + 1 == stall_ep;
    if (tid < 64 && !(stall && c == 0)) {
      dir_stage_member<BS, NPOW>(t, mbp[(r + 1) & 1], c, nxt);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid == 0) {
        if (hist) hist[(size_t)(r + 1) * N + c] = nxt;
        else if (nxt != INF32 && cur == INF32) t.C[(size_t)(r + 1) * N + c] = nxt;
        const uint64_t g = ((uint64_t)(uint32_t)(r - rlo + 1) << 32) | (uint32_t)nxt;
        __hip_atomic_store(gr[(r + 1) & 1] + c, (unsigned long long)g, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // strongly-see bits of C_{r+1}[c] against the members of round r
    if (nxt != INF32) {
      if (!have_bits) {  // a frontier row kept from an earlier batch: one more probe
        if (nxt < lo || nxt >= lo + DirGeo<BS, NPOW>::W) {
          __syncthreads();
          lo = nxt;
          dir_load<BS, NPOW>(t, L, c, lo, DirGeo<BS, NPOW>::W, lenc, pv);
          __syncthreads();
        }
        pb = dir_count<BS, NPOW>(L, nxt, part, mw) >= t.SM;
      }
      if (part == 0 && d < N && pb) atomicOr(&L.sBits[d >> 5], 1u << (d & 31));
      __syncthreads();  // also: every wave is done with this round's window
      if (tid < NW)
        ssc[((size_t)(r + 1) * N + c) * NW + tid] =
            (uint64_t)L.sBits[2 * tid] | ((uint64_t)L.sBits[2 * tid + 1] << 32);
    }
    DSTAMP(2);
    // the rows the next round's window [nxt, nxt + W) lacks, into their ring slots
    // (slots of rows below nxt: no wave reads them again; fn > 0 only if nxt is
    // a row, and then the barrier above has passed)
    if (nxt == INF32) {
      f0 = INF32;
      fn = 0;
    } else {
      f0 = (lo != INF32 && nxt < lo + DirGeo<BS, NPOW>::W) ? lo + DirGeo<BS, NPOW>::W : nxt;
      fn = nxt + DirGeo<BS, NPOW>::W - f0;
    }
    lo = nxt;
    dir_fetch<BS, NPOW>(t, c, f0, fn, lenc, pv);
    dir_store<BS, NPOW>(t, L, f0, fn, lenc, pv);
    if (fn > DIR_CH) {  // rare: the LA rows past the first chunk (the FD rows are in flight)
      for (int q = DIR_CH; q < fn; q += DIR_CH) {
        dir_fetch<BS, NPOW>(t, c, f0 + q, fn - q, lenc, pv);
        dir_store<BS, NPOW>(t, L, f0 + q, fn - q, lenc, pv);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's FD rows have landed
    DSTAMP(3);
    // collect C_{r+1}: every wave polls the granules (epoch r - rlo + 1) of its OWN
    // members and, once they match, loads their staged rows for the next round
    // right away -- the rows of early chains load while the late ones are still
    // being selected (round 2's single polling wave let the whole 128 KB block
    // load only after the slowest chain had published).  Each wave loads only
    // bytes whose flags it polled itself (MI355X_MICROARCH.md, Valid forms, row 1).
    {
      const unsigned ep = (unsigned)(r - rlo + 1);
      const gu64_t* g = gr[(r + 1) & 1];
      unsigned spins = 0;
      bool fail = false;
      int P = INF32;
      for (;;) {
        bool ok = true;
        if (d < N) {
          const unsigned long long x = __hip_atomic_load(g + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = (unsigned)(x >> 32) == ep;
          P = (int)(uint32_t)x;
        }
        if (__all(ok)) break;
        if (stall || ++spins > (1u << 21)) {  // never a normal wait (~2 s): co-residency failure
          fail = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (part == 0 && d < N) L.sP[d] = P;
      const bool any = __ballot(d < N && P != INF32) != 0;
      const bool notpast = stopcut && __ballot(part == 0 && d < N && P < stopcut[d]) != 0;  // INF32 passes
      if ((threadIdx.x & 63) == 0 && (any || notpast || fail))
        atomicOr(&L.sFlag[(r + 1) & 1], (any ? 1 : 0) | (notpast ? 2 : 0) | (fail ? 4 : 0));
      if (fail && (threadIdx.x & 63) == 0) {  // the host falls back to k_round_step32
        atomicOr(err, 1);
        atomicOr(rstate + 1, 4);  // the downstream kernels stand down, as on overflow
      }
      if (!fail) dir_members_mb<BS, NPOW>(mbp[(r + 1) & 1], mw);
    }
    __syncthreads();  // every wave has polled (and stored its window rows)
    DSTAMP(4);
    const int fl = L.sFlag[(r + 1) & 1];
    const int stop = (fl & 4) ? 2 : ((fl & 1) ? 0 : 1);
    if (stop) {
      if (stop == 1 && c == 0 && tid == 0) rstate[0] = hist ? r + 2 : max(rstate[0], r + 1);
      break;
    }
    if (stopcut) {
      if (extra_left < 0 && !(fl & 2)) extra_left = extra;
      if (extra_left >= 0 && extra_left-- == 0) {
        if (c == 0 && tid == 0) {
          rstate[0] = r + 2;  // rows 0 .. r + 1
          rstate[1] = 2;
        }
        break;
      }
    }
  }
  if (stamping) {
    for (int q = 0; q < 9; q++) dbg[q] += st_acc[q];
    dbg[9] += L.sdbg[0];
    dbg[10] += L.sdbg[1];
  }
#undef DSTAMP
#undef DSTAMP_START
}

template __global__ void k_rounds_direct<1024, 64>(Tables, const int32_t*, const int32_t*, int32_t*, int, const int32_t*, int,
    uint64_t*, int32_t*, uint64_t*, uint32_t*, uint64_t*, const int32_t*, int32_t*, int, const int32_t*, int, int);
template __global__ void k_rounds_direct<1024, 128>(Tables, const int32_t*, const int32_t*, int32_t*, int, const int32_t*, int,
    uint64_t*, int32_t*, uint64_t*, uint32_t*, uint64_t*, const int32_t*, int32_t*, int, const int32_t*, int, int);
template __global__ void k_rounds_direct<1024, 256>(Tables, const int32_t*, const int32_t*, int32_t*, int, const int32_t*, int,
    uint64_t*, int32_t*, uint64_t*, uint32_t*, uint64_t*, const int32_t*, int32_t*, int, const int32_t*, int, int);

}  // namespace hge
