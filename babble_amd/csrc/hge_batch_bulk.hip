// hge_batch_bulk.hip — the batch engine's call schedule in bulk (included by
// hge_batch.hip inside namespace hgb; the CPU model of these stages is
// tests/bulk_model.py, checked against the oracle by tests/test_bulk_model.py).
//
// kb_consensus walks a graph's call points in order, one workgroup per graph, so
// a GPU holding fewer graphs than CUs waits on each graph's ~11 us per call.  But
// once kb_front has every event's round and witness flag (a function of the
// event's ancestry alone), RunConsensus (node/core.go:179-202) at call c depends on
// the earlier calls only through the persisted fame and LastConsensusRound:
//   kb_prep     R_c, each event's insertion call, the witnesses in insertion order;
//   kb_pairs    DecideFame's decisions for round i at call c (hashgraph.go:598-664;
//               `votes` is rebuilt every call, so they depend on the witnesses
//               present at c alone), one wave per (call, i = R_c - 2 - s), s < NS;
//   kb_fold     per graph, one wave over the calls in order: arrivals set the
//               present-witness masks, rounds LCR+1 .. R_c-2 take their pair's
//               decisions (a pair outside the window is decided inline), then
//               setLastConsensusRound (:666-673); each round's (decided, famous set)
//               state over the calls as intervals;
//   kb_theta    per interval, the receive threshold per creator (the (|F|/2+1)-th
//               largest lastAncestor index over the famous witnesses F: x is seen by
//               more than half of them iff index(x) <= theta, :696-712);
//   kb_receive  per event, the first call at which a round above it has a decided
//               interval that sees it, the lowest such round at that call
//               (DecideRoundReceived, :676-721), and MedianTimestamp (:762-770);
//   kb_order_prep / kb_sort   per call, the received events (FindOrder, :723-760)
//               sorted by (roundReceived, timestamp, S, id) (consensus_sorter.go:36-59,
//               PRN = 0), the undetermined list, the scalars.
// A graph the fold cannot hold (more than 64 * FRS rounds, an interval table past
// its capacity) is flagged in scal[7] and replayed by kb_consensus.

constexpr int BNS = 3;      // at most BNS DecideFame pairs per call kept: rounds R_c - 2 - s, s < NS <= BNS
constexpr int BVCAP = 4;    // receive intervals per round
constexpr int BICAP = 512;  // receive intervals per graph
constexpr int FRS = 4;      // rounds per lane in kb_fold (64 * FRS rounds)

// per-graph internals, t.gx[g * 16 + k]
enum { GX_NARR = 0, GX_LCR = 2, GX_LCRC = 3, GX_NIV = 4, GX_MISS = 5, GX_RF = 6, GX_NLAST = 7 };

// inclusive block scans over blockDim.x threads (a multiple of 64), s_w: blockDim.x / 64 ints
__device__ __forceinline__ int block_scan_add(int v, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int pre = 0, tot = 0;
  for (int w = 0; w < nw; w++) {
    const int s = s_w[w];
    tot += s;
    if (w < wv) pre += s;
  }
  __syncthreads();
  total = tot;
  return x + pre;
}
__device__ __forceinline__ int block_scan_max(int v, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x = max(x, y);
  }
  if (lane == 63) s_w[wv] = x;
  __syncthreads();
  int pre = INT32_MIN, tot = INT32_MIN;
  for (int w = 0; w < nw; w++) {
    const int s = s_w[w];
    tot = max(tot, s);
    if (w < wv) pre = max(pre, s);
  }
  __syncthreads();
  total = tot;
  return max(x, pre);
}

// R_c, the insertion call of every event and the witnesses in insertion order
// (arrival call << 32 | round << 8 | creator).  One 1024-thread workgroup per graph.
template <int NM>
__global__ __launch_bounds__(1024) void kb_prep(BT t) {
  const int g = blockIdx.x;
  const GDesc d = t.gd[g];
  const int tid = threadIdx.x, NT = 1024;
  __shared__ int s_w[16], s_pm[1024];
  int32_t* gx = t.gx + (int64_t)g * 16;
  if (t.scal[(int64_t)g * 8 + 6]) return;  // the rounds pass failed
  const int K = d.K;
  const int n_last = K > 0 ? (int)t.calls[d.co + K - 1] : 0;
  int carry = -1;  // the highest round so far
  for (int c0 = 0; c0 < K; c0 += NT) {
    const int c = c0 + tid;
    int mx = -1;
    if (c < K) {
      const int lo = c ? (int)t.calls[d.co + c - 1] : 0, hi = (int)t.calls[d.co + c];
      for (int x = lo; x < hi; x++) {
        t.xcall[d.eo + x] = c;
        mx = max(mx, t.round[d.eo + x]);
      }
    }
    int tot;
    const int pm = max(block_scan_max(mx, s_w, tot), carry);
    if (c < K) t.Rc[d.co + c] = pm + 1;
    // rfirst[r] = the first call with R_c >= r, for r <= R of the last call
    s_pm[tid] = pm;
    __syncthreads();
    const int prv = tid ? s_pm[tid - 1] : carry;
    if (c < K)
      for (int r = prv + 2; r <= pm + 1; r++) t.rfirst[d.ro + r] = c;
    carry = max(carry, tot);
    __syncthreads();
  }
  for (int x = n_last + tid; x < d.E; x += NT) t.xcall[d.eo + x] = K;
  __threadfence_block();
  __syncthreads();
  int base = 0;
  for (int x0 = 0; x0 < n_last; x0 += NT) {
    const int x = x0 + tid;
    const bool w = x < n_last && t.wit[d.eo + x];
    int tot;
    const int inc = block_scan_add(w ? 1 : 0, s_w, tot);
    if (w) {
      const uint32_t rc = (uint32_t)t.round[d.eo + x] << 8 | (uint32_t)t.cr[d.eo + x];
      t.arr[d.eo + base + inc - 1] = (uint64_t)(uint32_t)ld(&t.xcall[d.eo + x]) << 32 | rc;
    }
    base += tot;
  }
  if (tid == 0) {
    gx[GX_NARR] = base;
    gx[GX_NLAST] = n_last;
    gx[GX_RF] = K > 0 ? carry + 1 : 0;
  }
}

// DecideFame for round i at a call that holds n_c events and R rounds
// (hashgraph.go:598-664), lane = witness x of round i; at NM <= 32 the two half
// waves decide two calls at once (n_c, R: the lane's half's call; i is shared).
// Per voting round j: x's votes of round j-1 are a bit mask `prev` over its
// witnesses; the voters y of round j go in ascending creator order (the canonical
// witness order), each with yays = |ss(y) & prev|, nays = |ss(y)| - yays (missing
// votes are nays).  At diff = 1 a vote is See(y, x); in a normal round the first y
// whose tally reaches SM decides x (SetFame, `break`: no later y votes); in a coin
// round (diff % N == 0) y votes v on a supermajority, else its middle bit.  The last
// deciding j wins.  dec: the present witnesses decided at this call, val: their
// values (1 = famous), for the lane's half.
template <int NM, typename Src>
__device__ void fame_pair(const BT& t, const Src& src, int i, int n_c, int R, uint64_t& dec_out,
                          uint64_t& val_out) {
  constexpr int HV = NM <= 32 ? 2 : 1;
  const int lane = threadIdx.x & 63, N = t.N, SM = t.SM;
  const int x = HV == 2 ? (lane & 31) : lane, h = HV == 2 ? lane >> 5 : 0;
  const int Rw = HV == 2 ? max(R, __shfl_xor(R, 32)) : R;  // the wave's last round
  const int wxi = x < N ? src.W(i, x) : -1;
  const bool xp = x < N && wxi >= 0 && wxi < n_c;
  uint64_t prev = 0;
  int fv = 0;
  for (int j = i + 1; j < Rw; j++) {
    const bool act = j < R;
    const int diff = j - i;
    // round j's witness rows, lane y holding voter y's (read back by readlane: the
    // voter loop makes no memory access)
    const int wl = x < N ? src.W(j, x) : -1;
    const uint64_t bl = x < N ? (diff == 1 ? src.see(j, x) : src.ss(j, x)) : 0;
    const bool cl = x < N && diff % N == 0 && src.coin(j, x);
    const uint64_t cm = ballot(cl);
    uint64_t cur = 0;
    if (diff == 1) {
      for (int y = 0; y < N; y++) {
        const int wy = rl(wl, y);
        const bool py = act && wy >= 0 && wy < n_c;
        if (py && ((rl64(bl, y) >> x) & 1)) cur |= 1ull << y;  // setVote(y, x, See(y, x))
      }
    } else if (diff % N != 0) {  // normal round
      bool dh = false;
      for (int y = 0; y < N; y++) {
        const int wy = rl(wl, y);
        const bool py = act && wy >= 0 && wy < n_c && !dh;
        const uint64_t yb = rl64(bl, y);
        const int yays = __popcll(yb & prev), nays = __popcll(yb) - yays;
        const bool v = yays >= nays;
        if (py && (v ? yays : nays) >= SM) {  // SetFame(x, v), break
          fv = v ? 1 : 2;
          dh = true;
        } else if (py && v) {
          cur |= 1ull << y;
        }
      }
    } else {  // coin round: the middle bit of y's hash when no supermajority
      for (int y = 0; y < N; y++) {
        const int wy = rl(wl, y);
        const bool py = act && wy >= 0 && wy < n_c;
        const uint64_t yb = rl64(bl, y);
        const int yays = __popcll(yb & prev), nays = __popcll(yb) - yays;
        const bool v = yays >= nays;
        if (py && ((v ? yays : nays) >= SM ? v : ((cm >> y) & 1))) cur |= 1ull << y;
      }
    }
    if (act) prev = cur;
  }
  const uint64_t db = ballot(xp && fv != 0), vb = ballot(xp && fv == 1);
  dec_out = HV == 2 ? (db >> (32 * h)) & 0xFFFFFFFFull : db;
  val_out = HV == 2 ? (vb >> (32 * h)) & 0xFFFFFFFFull : vb;
}

// the witness rows in HBM
struct GSrc {
  const BT& t;
  int64_t ro;
  int N;
  __device__ int W(int j, int y) const { return t.W[(ro + j) * N + y]; }
  __device__ uint64_t see(int j, int y) const { return t.seeb[(ro + j) * N + y]; }
  __device__ uint64_t ss(int j, int y) const { return t.ssb[(ro + j) * N + y]; }
  __device__ bool coin(int j, int y) const { return t.WCOIN[(ro + j) * N + y] != 0; }
};
// rounds i0 .. i0 + NS staged in LDS
template <int NM>
struct LSrc {
  const int32_t (*w)[NM];
  const uint64_t (*se)[NM];
  const uint64_t (*sS)[NM];
  const uint8_t (*co)[NM];
  int i0;
  __device__ int W(int j, int y) const { return w[j - i0][y]; }
  __device__ uint64_t see(int j, int y) const { return se[j - i0][y]; }
  __device__ uint64_t ss(int j, int y) const { return sS[j - i0][y]; }
  __device__ bool coin(int j, int y) const { return co[j - i0][y] != 0; }
};

// DecideFame's pairs by round: workgroup (k, g) takes graph g's rounds i = k, k +
// gridDim.x, ..., stages the witness rows of rounds i .. i + NS in LDS and decides
// round i at every call whose window holds it (R_c in [i + 3, i + 1 + NS], a
// range of calls: R_c never decreases), one wave per call.  Round R_c - 2 (s = 0)
// sees one voting round only (diff = 1 sets votes, decides nothing): no pair.
// NS = 3 while two graphs fit a CU; past that NS = 2 (s = 2 is ~3 pairs per graph,
// computed inline by kb_fold, cheaper than a third of kb_pairs' work once the chip is full).
template <int NM, int NS>
__global__ __launch_bounds__(256) void kb_pairs(BT t) {
  constexpr int RB = NS + 1;
  const int g = blockIdx.y;
  if (t.scal[(int64_t)g * 8 + 6]) return;
  const GDesc d = t.gd[g];
  const int N = t.N, tid = threadIdx.x, wv = tid >> 6;
  const int Rf = t.gx[(int64_t)g * 16 + GX_RF];
  __shared__ int32_t sW[RB][NM];
  __shared__ uint64_t sSee[RB][NM], sSs[RB][NM];
  __shared__ uint8_t sCo[RB][NM];
  const LSrc<NM> src{sW, sSee, sSs, sCo, 0};
  for (int i = blockIdx.x; i <= Rf - 2; i += gridDim.x) {
    for (int e = tid; e < RB * N; e += 256) {
      const int jj = e / N, y = e - (e / N) * N, j = i + jj;
      if (j < Rf) {
        const int64_t rj = (int64_t)(d.ro + j) * N + y;
        sW[jj][y] = t.W[rj];
        sSee[jj][y] = t.seeb[rj];
        sSs[jj][y] = t.ssb[rj];
        sCo[jj][y] = t.WCOIN[rj];
      } else {
        sW[jj][y] = -1;
      }
    }
    // s = 0 (j = i + 1 only: votes, no decision) is never computed
    const int lo = i + 3 <= Rf ? t.rfirst[d.ro + i + 3] : d.K;
    const int hi = i + 2 + NS <= Rf ? t.rfirst[d.ro + i + 2 + NS] : d.K;
    __syncthreads();
    LSrc<NM> sr = src;
    sr.i0 = i;
    // one call per half wave (NM <= 32), per wave at NM = 64
    constexpr int HV = NM <= 32 ? 2 : 1;
    const int h = HV == 2 ? (tid & 63) >> 5 : 0;
    for (int c0 = lo + HV * wv; c0 < hi; c0 += 4 * HV) {
      const int c = c0 + h;
      const bool okc = c < hi;
      const int R = okc ? t.Rc[d.co + c] : i + 1;  // (no voting round: nothing decided)
      const int n_c = okc ? (int)t.calls[d.co + c] : 0;
      uint64_t dec, val;
      fame_pair<NM>(t, sr, i, n_c, R, dec, val);
      if (okc && (tid & (64 / HV - 1)) == 0) {
        const int64_t p = (int64_t)(d.co + c) * NS + (R - 2 - i);
        t.Dp[2 * p] = dec;
        t.Dp[2 * p + 1] = val;
      }
    }
    __syncthreads();
  }
}

// The calls in order, one wave per graph, visiting only the calls where DecideFame
// has a round to decide: i in [LCR+1, R_c-3] (round R_c - 2 meets one voting round
// and decides nothing, nor was it decided at an earlier call: R never decreases), so
// from call c the next such call is the first with R >= LCR + 4 (rfirst).  Lane l
// keeps rounds l, l + 64, ... (FRS slots): decided and famous masks.  A round's
// present witnesses at call c come from its witnesses' arrival calls (LDS).
// Each round has at most one receive interval: a round is decided only while
// processed (i > LCR), and deciding it sets LCR >= i, so it is never processed again;
// the next witness to arrive (fame undefined) ends the interval for good.  So the
// interval [c, next arrival) with famous set F is written when the round is decided,
// and setLastConsensusRound (hashgraph.go:666-673) follows the loop's highest
// decided round.
template <int NM, int NS>
__global__ __launch_bounds__(64) void kb_fold(BT t) {
  constexpr int RL = 64 * FRS;  // rounds held
  const int g = blockIdx.x;
  const GDesc d = t.gd[g];
  const int lane = threadIdx.x, N = t.N, K = d.K;
  int32_t* gx = t.gx + (int64_t)g * 16;
  if (t.scal[(int64_t)g * 8 + 6]) return;
  const int Rf = gx[GX_RF], narr = gx[GX_NARR];
  if (Rf > RL || Rf * N > RL * 32) {
    if (lane == 0) t.scal[(int64_t)g * 8 + 7] = 1;
    return;
  }
  __shared__ int32_t wc[RL * 32];  // [r][creator]: the call its witness arrives at (K: none)
  __shared__ int32_t rfl[RL + 1];  // rfirst
  for (int e = lane; e < Rf * N; e += 64) wc[e] = K;
  for (int r = lane; r <= Rf; r += 64) rfl[r] = r >= 3 ? t.rfirst[d.ro + r] : 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  wsync();
  for (int k = lane; k < narr; k += 64) {
    const uint64_t a = t.arr[d.eo + k];
    wc[(int)((a >> 8) & 0xFFFFFF) * N + (int)(a & 0xFF)] = (int)(a >> 32);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  wsync();
  uint64_t dfn[FRS], vl[FRS];
  int fst[FRS];
#pragma unroll
  for (int q = 0; q < FRS; q++) {
    dfn[q] = vl[q] = 0;
    fst[q] = INF;
  }
  int LCR = -1, lcr_call = -1, nth = 0, miss = 0;
  int c = -1, c0 = -INF, Rreg = 0, Nreg = 0;
  uint64_t Dd[NS], Dv[NS];
  while (true) {
    const int need = LCR + 4;  // the next call with a round to decide has R >= LCR + 4
    if (need > Rf) break;
    c = max(c + 1, rfl[need]);
    if (c >= K) break;
    if (c >= c0 + 64) {  // the next 64 calls' R, sizes and pairs, lane l holding call c0 + l
      c0 = c;
      const int cl = c0 + lane;
      const bool on = cl < K;
      Rreg = on ? t.Rc[d.co + cl] : 0;
      Nreg = on ? (int)t.calls[d.co + cl] : 0;
#pragma unroll
      for (int s = 0; s < NS; s++) {
        const int64_t p = ((int64_t)(d.co + cl)) * NS + s;
        const bool ok = on && s > 0 && Rreg - 2 - s >= 0;
        Dd[s] = ok ? t.Dp[2 * p] : 0;
        Dv[s] = ok ? t.Dp[2 * p + 1] : 0;
      }
    }
    const int cc = c - c0, R = rl(Rreg, cc);
    int newL = -1;
    for (int i = LCR + 1; i <= R - 3; i++) {
      const int s = R - 2 - i;
      uint64_t dec = 0, v = 0;
      if (s < NS) {
#pragma unroll
        for (int q = 0; q < NS; q++)
          if (q == s) {
            dec = rl64(Dd[q], cc);
            v = rl64(Dv[q], cc);
          }
      } else {
        fame_pair<NM>(t, GSrc{t, (int64_t)d.ro, N}, i, rl(Nreg, cc), R, dec, v);
        miss++;
      }
      const int wci = lane < N ? wc[i * N + lane] : K;
      const uint64_t pres = ballot(lane < N && wci <= c);
      uint64_t df = 0, vv = 0;
#pragma unroll
      for (int q = 0; q < FRS; q++)
        if (q == (i >> 6)) {
          if (lane == (i & 63)) {
            dfn[q] |= dec;
            vl[q] = (vl[q] & ~dec) | v;
          }
          df = rl64(dfn[q], i & 63);
          vv = rl64(vl[q], i & 63);
        }
      if ((pres & ~df) == 0) {  // WitnessesDecided (roundInfo.go:78-85)
        newL = i;
        const uint64_t F = pres & vv;
        if (F) {  // the receive interval [c, the next arrival)
          const int ce = wave_min(lane < N && wci > c ? wci : K);
          if (nth < BICAP) {
            if (lane == 0) {
              const int64_t iv = (int64_t)(d.ro + i) * BVCAP;
              t.ivh[iv] = make_int4(c, ce, nth, 0);
              t.ivF[iv] = F;
              t.thR[(int64_t)g * BICAP + nth] = i;
              t.thF[(int64_t)g * BICAP + nth] = F;
            }
#pragma unroll
            for (int q = 0; q < FRS; q++)
              if (q == (i >> 6) && lane == (i & 63)) fst[q] = c;
          }
          nth++;
        }
      }
    }
    if (newL >= 0) {
      LCR = newL;
      lcr_call = c;
    }
  }
  if (nth > BICAP) {
    if (lane == 0) t.scal[(int64_t)g * 8 + 7] = 1;
    return;
  }
  // per round: interval count, the suffix minimum of the first intervals' starts
  // (kb_receive stops once no higher round can receive earlier), the fame row
  int carry = INF;
#pragma unroll
  for (int q = FRS - 1; q >= 0; q--) {
    int v = fst[q];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_down(v, o);
      if (lane + o < 64) v = min(v, u);
    }
    v = min(v, carry);
    carry = rl(v, 0);
    const int r = q * 64 + lane;
    if (r < Rf) {
      t.nivl[d.ro + r] = fst[q] != INF ? 1 : 0;
      t.fsuf[d.ro + r] = v;
      if (dfn[q])
        for (int x = 0; x < N; x++)
          if ((dfn[q] >> x) & 1) t.fame[(int64_t)(d.ro + r) * N + x] = (int8_t)((vl[q] >> x) & 1 ? 1 : 2);
    }
  }
  if (lane == 0) {
    gx[GX_LCR] = LCR;
    gx[GX_LCRC] = lcr_call;
    gx[GX_NIV] = nth;
    gx[GX_MISS] = miss;
  }
}

// the receive thresholds of every interval: one wave per interval, lane = creator
template <int NM>
__global__ __launch_bounds__(256) void kb_theta(BT t) {
  const int g = blockIdx.x;
  const GDesc d = t.gd[g];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, N = t.N;
  if (t.scal[(int64_t)g * 8 + 6] || t.scal[(int64_t)g * 8 + 7]) return;
  const int nth = t.gx[(int64_t)g * 16 + GX_NIV];
  const int32_t* LA = t.LA + d.eo * N;
  for (int s = wv; s < nth; s += 4) {
    const int r = t.thR[(int64_t)g * BICAP + s];
    const uint64_t F = t.thF[(int64_t)g * BICAP + s];
    const int m = __popcll(F), need = m / 2 + 1;  // len(s) > len(fws)/2
    const int w = lane < N ? t.W[(int64_t)(d.ro + r) * N + lane] : -1;
    int32_t vals[NM];
#pragma unroll
    for (int dd = 0; dd < NM; dd++)
      vals[dd] = (F >> dd) & 1 && lane < N ? LA[(int64_t)rl(w, dd) * N + lane] : INT32_MIN;
    sort_regs32<NM>(vals);
    int th = INT32_MIN;
#pragma unroll
    for (int a = 0; a < NM; a++)
      if (a == NM - need) th = vals[a];
    if (lane < N) t.thp[((int64_t)g * BICAP + s) * N + lane] = th;
  }
}

// One thread per chain position (events below the last call): the event's receiving
// call and round, then the median timestamp over OldestSelfAncestorToSee(w, x) of the
// famous witnesses w that see x (w = (d, i_w) sees x iff FD[x][d] <= i_w, and the
// chain-d event at FD[x][d] is then OldestSelfAncestorToSee), the upper median len/2.
// One workgroup per (chain, graph): the graph's call points and receive intervals and
// the chain's thresholds are staged in LDS, so the search is LDS reads.  Lanes take
// consecutive positions of the chain, whose first descendants on chain d never
// decrease: the timestamp gathers of a wave stay on a few lines.
constexpr int RKL = 2048;  // call points staged in LDS
constexpr int RRL = 128;   // rounds of receive intervals staged in LDS
template <int NM>
__global__ __launch_bounds__(256) void kb_receive(BT t) {
  const int g = blockIdx.y, c = blockIdx.x;
  if (t.scal[(int64_t)g * 8 + 6] || t.scal[(int64_t)g * 8 + 7]) return;
  const GDesc d = t.gd[g];
  const int N = t.N, cc = t.ccap, tid = threadIdx.x, lane = tid & 63;
  const int len = t.clen[g * N + c];
  if (len == 0) return;
  __shared__ int32_t s_calls[RKL];
  __shared__ int32_t s_fsuf[RRL], s_niv[RRL];
  __shared__ int4 s_ivh[RRL * BVCAP];
  __shared__ int32_t s_th[BICAP];
  const int32_t* gx = t.gx + (int64_t)g * 16;
  const int n_last = gx[GX_NLAST], Rf = gx[GX_RF], nth = gx[GX_NIV];
  const int K = d.K, KS = min(K, RKL), RS = min(Rf, RRL);
  for (int k = tid; k < KS; k += 256) s_calls[k] = (int)t.calls[d.co + k];
  for (int r = tid; r < RS; r += 256) {
    s_fsuf[r] = t.fsuf[d.ro + r];
    s_niv[r] = t.nivl[d.ro + r];
  }
  for (int e = tid; e < RS * BVCAP; e += 256) s_ivh[e] = t.ivh[(int64_t)d.ro * BVCAP + e];
  for (int k = tid; k < nth; k += 256) s_th[k] = t.thp[((int64_t)g * BICAP + k) * N + c];
  __syncthreads();
  auto call_at = [&](int k) -> int { return k < RKL ? s_calls[k] : (int)t.calls[d.co + k]; };
  const int64_t cb = (int64_t)g * N * cc, eo = d.eo;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int p = tid; p - lane < len; p += 256) {  // (whole waves iterate together)
  const int64_t cpos = (int64_t)c * cc + p;
  const int x = p < len ? t.chain[cb + cpos] : -1;
  const bool on = x >= 0 && x < n_last;
  int best_c = INF, bi = -1, bslot = -1;
  if (on) {
    const int r = t.roundch[cb + cpos];
    int cl = 0;  // x's insertion call: the first call with more than x events
    for (int hi = K - 1; cl < hi;) {
      const int mid = (cl + hi) >> 1;
      if (call_at(mid) > x) hi = mid;
      else cl = mid + 1;
    }
    for (int i = r + 1; i < Rf; i++) {
      const bool li = i < RRL;
      if ((li ? s_fsuf[i] : t.fsuf[d.ro + i]) >= best_c) break;
      const int n = li ? s_niv[i] : t.nivl[d.ro + i];
      for (int k = 0; k < n; k++) {
        const int64_t iv = (int64_t)(d.ro + i) * BVCAP + k;
        const int4 hv = li ? s_ivh[i * BVCAP + k] : t.ivh[iv];
        if (hv.y <= cl) continue;
        const int cand = max(hv.x, cl);
        if (cand >= best_c) break;
        if (p <= s_th[hv.z]) {
          best_c = cand;
          bi = i;
          bslot = hv.z;
          break;
        }
      }
    }
  }
  // the call bucket's slot: one atomic per distinct call in the wave (a wave's
  // consecutive positions are mostly received at the same call)
  {
    // group the lanes by call (ballots only), then every group's first lane adds the
    // group's size at once: the atomics of one wave are in flight together
    uint64_t todo = ballot(bi >= 0), mine = 0;
    while (todo) {
      const int lead = __ffsll((unsigned long long)todo) - 1;
      const int cv = rl(best_c, lead);
      const uint64_t same = ballot(bi >= 0 && best_c == cv);
      if (bi >= 0 && best_c == cv) mine = same;
      todo &= ~same;
    }
    const int lead = mine ? __ffsll((unsigned long long)mine) - 1 : lane;
    int base = 0;
    if (mine && lane == lead) base = atomicAdd(&t.bcnt[d.co + best_c], __popcll(mine));
    base = __shfl(base, lead);
    const int rank = mine ? base + __popcll(mine & below) : -1;
    if (p < len) {
      t.rcall[cb + cpos] = bi >= 0 ? best_c : -1;
      t.rrank[cb + cpos] = rank;
    }
  }
  if (p < len) t.rslot[cb + cpos] = bi >= 0 ? bslot : -1;
  }  // positions
}

// MedianTimestamp (hashgraph.go:762-770) of every received event, one thread per chain
// position (kb_receive's layout: the timestamp gathers of a wave stay on few lines):
// the upper median (len/2) over OldestSelfAncestorToSee(w, x) of the famous witnesses
// w of the receiving interval that see x (w = (d, i_w) sees x iff FD[x][d] <= i_w,
// and the chain-d event at FD[x][d] is then OldestSelfAncestorToSee).
template <int NM>
__global__ __launch_bounds__(256) void kb_median(BT t) {
  const int g = blockIdx.y;
  if (t.scal[(int64_t)g * 8 + 6] || t.scal[(int64_t)g * 8 + 7]) return;
  const GDesc d = t.gd[g];
  const int N = t.N, cc = t.ccap, lane = threadIdx.x & 63;
  const int nb = (cc + 255) >> 8;  // position blocks per chain
  const int c = blockIdx.x / nb, p = (blockIdx.x - c * nb) * 256 + threadIdx.x;
  const int len = t.clen[g * N + c];
  if (p - lane >= len) return;  // whole waves
  const int64_t cb = (int64_t)g * N * cc, cpos = (int64_t)c * cc + p, eo = d.eo;
  const int slot = p < len ? t.rslot[cb + cpos] : -1;
  const int bi = slot >= 0 ? t.thR[(int64_t)g * BICAP + slot] : -1;
  const uint64_t bF = slot >= 0 ? t.thF[(int64_t)g * BICAP + slot] : 0;
  const int x = slot >= 0 ? t.chain[cb + cpos] : -1;
  int64_t tx = 0;
  if (bi >= 0) {
    // FD[x][dd] from the run layout FDT[g][dd][c][p]: a wave's lanes are consecutive
    // positions p, so each dd is one coalesced load (no FD rows are built)
    const int32_t* FDc = t.FDT + (int64_t)g * N * N * cc + (int64_t)c * cc + p;  // + dd * N * cc
    const int64_t NC = (int64_t)N * cc;
    const int64_t* tschg = t.tsch + cb;
    const int32_t* wixr = t.WIX + (int64_t)(d.ro + bi) * N;
    const int64_t tsx = tschg[cpos];
    // the row, the witnesses' positions and the gathers, MB witnesses at a time (each
    // batch's loads in flight together; a compiler barrier between batches keeps the
    // register footprint to one batch)
    int32_t vals[NM];
    int m = 0;
    bool ovf = false;
    const bool vec = (N & 3) == 0;  // 16-byte aligned rows
    constexpr int MB = 16;
#pragma unroll
    for (int b0 = 0; b0 < NM; b0 += MB) {
      int32_t fd[MB], wx[MB];
#pragma unroll
      for (int k = 0; k < MB; k++) fd[k] = b0 + k < N ? FDc[(b0 + k) * NC] : INF;
      if (vec) {
#pragma unroll
        for (int k = 0; k < MB; k += 4) {
          const int4 w = b0 + k < N ? *(const int4*)(wixr + b0 + k) : make_int4(-1, -1, -1, -1);
          wx[k] = w.x;
          wx[k + 1] = w.y;
          wx[k + 2] = w.z;
          wx[k + 3] = w.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < MB; k++) wx[k] = b0 + k < N ? wixr[b0 + k] : -1;
      }
      int64_t tq[MB];
      bool in[MB];
#pragma unroll
      for (int k = 0; k < MB; k++) {
        const int dd = b0 + k;
        in[k] = dd < N && ((bF >> dd) & 1) && fd[k] != INF && fd[k] <= wx[k];
        tq[k] = tschg[(int64_t)dd * cc + (in[k] ? fd[k] : 0)];
      }
#pragma unroll
      for (int k = 0; k < MB; k++) {
        const int64_t o = tq[k] - tsx;
        ovf = ovf || (in[k] && (o < -(int64_t)INT32_MAX || o > (int64_t)INT32_MAX));
        vals[b0 + k] = in[k] ? (int32_t)o : INT32_MAX;  // fillers sort last (a real INT32_MAX ties with them)
        m += in[k];
      }
      asm volatile("" ::: "memory");
    }
    const int32_t* wix = wixr;
    const int want = m / 2;
    int64_t med = 0;
    if (!ovf) {
      sort_regs32<NM>(vals);
#pragma unroll
      for (int a = 0; a < NM; a++)
        if (a == want) med = tsx + vals[a];
    } else {  // the value whose rank among the m timestamps covers `want`, exact in 64 bits
      auto tv = [&](int dd, int64_t& v) -> bool {
        if (!((bF >> dd) & 1)) return false;
        const int q = FDc[dd * NC];
        if (q == INF || q > wix[dd]) return false;
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
    t.rr[eo + x] = bi;
    t.cts[eo + x] = med;
    t.rrch[cb + cpos] = bi;
    t.ctsch[cb + cpos] = med;
    tx += t.ntxch[cb + cpos];
  }
  tx = wave_sum64(tx);
  if (lane == 0 && tx) atomicAdd((unsigned long long*)&t.gctx[g], (unsigned long long)tx);
}

// Per graph: the call buckets' offsets (the per-call batch sizes), the received
// events' keys scattered into their buckets, the undetermined list in insertion
// order, LastCommitedRoundEvents and the scalars.  One 1024-thread workgroup.
template <int NM>
__global__ __launch_bounds__(1024) void kb_order_prep(BT t) {
  const int g = blockIdx.x;
  if (t.scal[(int64_t)g * 8 + 6] || t.scal[(int64_t)g * 8 + 7]) return;
  const GDesc d = t.gd[g];
  const int tid = threadIdx.x, NT = 1024;
  const int64_t eo = d.eo;
  __shared__ int s_w[16];
  const int32_t* gx = t.gx + (int64_t)g * 16;
  const int K = d.K, n_last = gx[GX_NLAST];
  int carry = 0;
  for (int c0 = 0; c0 < K; c0 += NT) {
    const int c = c0 + tid;
    const int v = c < K ? t.bcnt[d.co + c] : 0;
    int tot;
    const int inc = block_scan_add(v, s_w, tot);
    if (c < K) {
      t.boff[d.co + c] = carry + inc - v;
      t.counts[d.co + c] = v;
      if (v > 0) {
        const int k = atomicAdd(t.wlc, 1);
        t.wl[k] = make_int4(g, v, carry + inc - v, 0);
      }
    }
    carry += tot;
  }
  const int nord = carry;
  __threadfence_block();
  __syncthreads();
  // the received events' keys into their buckets, from the chain layout (a chain's
  // consecutive positions received at one call hold consecutive slots)
  {
    const int N = t.N, cc = t.ccap;
    const int64_t cb = (int64_t)g * N * cc;
    for (int e = tid; e < N * cc; e += NT) {
      const int c = e / cc, p = e - (e / cc) * cc;
      if (p >= t.clen[g * N + c]) continue;
      {
        const int64_t cp = cb + e;
        const int rc = t.rcall[cp];
        if (rc < 0) continue;
        const int pos = ld(&t.boff[d.co + rc]) + t.rrank[cp];
        const int64_t so = 2 * eo + pos;
        t.krr[so] = t.rrch[cp];
        t.kct[so] = t.ctsch[cp];
        t.ks0[so] = t.Sch[cp];
        t.kid[so] = t.chain[cp];
      }
    }
  }
  // the undetermined list (UndeterminedEvents keeps insertion order)
  int base = 0;
  for (int x0 = 0; x0 < n_last; x0 += NT) {
    const int x = x0 + tid;
    const bool u = x < n_last && t.rr[eo + x] < 0;
    int tot;
    const int inc = block_scan_add(u ? 1 : 0, s_w, tot);
    if (u) t.U[eo + base + inc - 1] = x;
    base += tot;
  }
  // LastCommitedRoundEvents: RoundEvents(LCR - 1) at the call that set LCR (hashgraph.go:666-673)
  const int L = gx[GX_LCR], lc = gx[GX_LCRC];
  int cnt = 0;
  if (L >= 1) {
    const int lim = (int)t.calls[d.co + lc];
    for (int x = tid; x < lim; x += NT) cnt += t.round[eo + x] == L - 1;
  }
  int lcre;
  block_scan_add(cnt, s_w, lcre);
  if (tid == 0) {
    int64_t* s = t.scal + (int64_t)g * 8;
    s[0] = gx[GX_RF];
    s[1] = L;
    s[2] = lcre;
    s[3] = t.gctx[g];
    s[4] = nord;
    s[5] = base;
  }
}

// The call buckets' sorts (a work list over the whole batch): an ascending bitonic
// network whose merge stages compare mirrored pairs, so slots past the bucket act as
// +infinity and need no storage.  A bucket's keys (rr, cts, S, id) sort on an
// order-preserving 64-bit prefix held in LDS with a 16-bit index:
// (rr - rmin) << 60 | (cts - cmin) << 32 | S >> 32 when the bucket's rounds span
// under 16 and its timestamps under 2^28 ns (else the prefix is 0); equal prefixes
// compare the full key from HBM (consensus_sorter.go:36-59, PRN = 0).
// kb_sort<TPB, LO, CAP> takes the buckets of LO < n <= CAP keys, TPB threads per
// bucket (one wave while the batch has many buckets, four while it has few); the
// largest class sorts buckets past CAP on their full keys in HBM.
__device__ __forceinline__ void bitonic_pair(int q, int size, int stride, int& a, int& b) {
  if (stride == size >> 1) {  // merge: mirrored pairs
    const int blk = q / stride, i = q - blk * stride;
    a = blk * size + i;
    b = blk * size + size - 1 - i;
  } else {
    a = 2 * q - (q & (stride - 1));
    b = a + stride;
  }
}
__device__ __forceinline__ int64_t wave_min64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (int64_t)__shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int64_t wave_max64(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor(v, o));
  return v;
}
template <int TPB, int LO, int CAP>
__global__ __launch_bounds__(TPB) void kb_sort(BT t, int last) {
  __shared__ uint64_t lk[CAP];
  __shared__ uint16_t lx[CAP];
  __shared__ int s_red[4][4];
  __shared__ int64_t s_red64[4][2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nw = ld(t.wlc);
  auto sync = [&](bool block) {
    if (TPB == 64 || !block) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      wsync();
    } else {
      __syncthreads();
    }
  };
  for (int w = blockIdx.x; w < nw; w += gridDim.x) {
    const int4 gc = t.wl[w];
    const int g = gc.x, n = gc.y, base = gc.z;
    if (n <= LO || (n > CAP && !last)) continue;
    const int64_t eo = t.gd[g].eo, so = 2 * eo + base;
    int P = 1;
    while (P < n) P <<= 1;
    auto full_less = [&](int a, int b) -> bool {
      return key_less(t, eo, t.krr[so + a], t.kct[so + a], t.ks0[so + a], t.kid[so + a], t.krr[so + b],
                      t.kct[so + b], t.ks0[so + b], t.kid[so + b]);
    };
    if (n <= CAP) {
      int rmn = INT32_MAX, rmx = INT32_MIN;
      int64_t cmn = INT64_MAX, cmx = INT64_MIN;
      for (int k = tid; k < n; k += TPB) {
        const int r = t.krr[so + k];
        const int64_t c = t.kct[so + k];
        rmn = min(rmn, r);
        rmx = max(rmx, r);
        cmn = min(cmn, c);
        cmx = max(cmx, c);
      }
      rmn = wave_min(rmn);
      rmx = wave_max(rmx);
      cmn = wave_min64(cmn);
      cmx = wave_max64(cmx);
      if (TPB > 64) {
        if (lane == 0) {
          s_red[wv][0] = rmn;
          s_red[wv][1] = rmx;
          s_red64[wv][0] = cmn;
          s_red64[wv][1] = cmx;
        }
        __syncthreads();
        for (int k = 0; k < TPB / 64; k++) {
          rmn = min(rmn, s_red[k][0]);
          rmx = max(rmx, s_red[k][1]);
          cmn = min(cmn, s_red64[k][0]);
          cmx = max(cmx, s_red64[k][1]);
        }
      }
      const bool fits = rmx - rmn < 16 && cmx - cmn < ((int64_t)1 << 28);
      for (int k = tid; k < n; k += TPB) {
        lk[k] = fits ? ((uint64_t)(t.krr[so + k] - rmn) << 60) | ((uint64_t)(t.kct[so + k] - cmn) << 32) |
                           (t.ks0[so + k] >> 32)
                     : 0;
        lx[k] = (uint16_t)k;
      }
      sync(true);
      for (int size = 2; size <= P; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int q = tid; q < P / 2; q += TPB) {
            int a, b;
            bitonic_pair(q, size, stride, a, b);
            if (b >= n) continue;
            const uint64_t ka = lk[a], kb = lk[b];
            const int xa = lx[a], xb = lx[b];
            if (kb < ka || (kb == ka && full_less(xb, xa))) {
              lk[a] = kb;
              lk[b] = ka;
              lx[a] = (uint16_t)xb;
              lx[b] = (uint16_t)xa;
            }
          }
          const int next = stride > 1 ? stride >> 1 : size;  // the next stage's stride
          sync(stride > 64 || next > 64);
        }
      sync(true);
      for (int k = tid; k < n; k += TPB) t.order[eo + base + k] = t.kid[so + lx[k]];
      sync(true);  // the LDS keys are the next bucket's
    } else {
      for (int size = 2; size <= P; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int q = tid; q < P / 2; q += TPB) {
            int a, b;
            bitonic_pair(q, size, stride, a, b);
            if (b >= n) continue;
            const int ra = ld(t.krr + so + a), rb = ld(t.krr + so + b);
            const int ia = ld(t.kid + so + a), ib = ld(t.kid + so + b);
            const int64_t ca = ld(t.kct + so + a), cb = ld(t.kct + so + b);
            const uint64_t sa = ld(t.ks0 + so + a), sb = ld(t.ks0 + so + b);
            if (key_less(t, eo, rb, cb, sb, ib, ra, ca, sa, ia)) {
              st(t.krr + so + a, rb);
              st(t.krr + so + b, ra);
              st(t.kid + so + a, ib);
              st(t.kid + so + b, ia);
              st(t.kct + so + a, cb);
              st(t.kct + so + b, ca);
              st(t.ks0 + so + a, sb);
              st(t.ks0 + so + b, sa);
            }
          }
          __threadfence_block();
          __syncthreads();
        }
      }
      for (int k = tid; k < n; k += TPB) t.order[eo + base + k] = ld(t.kid + so + k);
      __syncthreads();
    }
  }
}
