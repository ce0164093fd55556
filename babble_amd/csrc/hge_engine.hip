// hge_engine.hip — host side of the MI355X hashgraph engine (C ABI in include/hge.h).
//
// Orchestrates the kernels of hge_kernels.hip over one HIP stream.  The host
// keeps only control state: the FromParentsLatest admission check (O(1) per
// event over per-creator chain tails, hashgraph.go:366-396), the consensus log
// and a handful of scalars (Rounds(), LastConsensusRound, ...).  Every table
// the ordering path reads lives in HBM.
//
// A "batch" is the unit of device work: it absorbs the events inserted since
// the previous batch and replays a list of RunConsensus calls (each at an
// event count n_c).  The online API runs one call per batch; hge_replay runs a
// whole schedule in one batch.  Both produce identical results (tests).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hge.h"
#include "hge_kernels.hip"
#include "hge_wide32.hip"
#include "hge_coords.hip"
#include "hge_coords_win.hip"
#include "hge_rounds_coop.hip"
#include "hge_rounds_direct.hip"
#include "hge_walk_spec.hip"

using namespace hge;

#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      throw EngineError(HGE_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
    }                                                                                \
  } while (0)

// every launch is checked: a launch the runtime refuses (e.g. too much LDS)
// must fail the call, never leave a table silently unwritten
#define KLAUNCH(kern, ...)                                                             \
  do {                                                                                 \
    hp.launches++;                                                                     \
    prof_begin(#kern);                                                                 \
    hipLaunchKernelGGL(kern, __VA_ARGS__);                                             \
    const hipError_t le_ = hipGetLastError();                                          \
    if (le_ != hipSuccess)                                                             \
      throw EngineError(HGE_ERR_DEVICE, std::string("launch " #kern ": ") + hipGetErrorString(le_)); \
    prof_end();                                                                        \
  } while (0)

namespace {

struct EngineError {
  int code;
  std::string msg;
  EngineError(int c, std::string m) : code(c), msg(std::move(m)) {}
};

template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  void free_() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  // grow without preserving contents
  void need(size_t m) {
    if (m <= n) return;
    free_();
    size_t cap = std::max<size_t>(m, 64);
    HIPCHK(hipMalloc(&p, cap * sizeof(T)));
    n = cap;
  }
  // grow preserving contents [0, keep)
  void grow_keep(size_t m, size_t keep, hipStream_t st, int fill_byte = -1) {
    if (m <= n) return;
    size_t cap = std::max<size_t>(m, n + n / 2);
    T* q = nullptr;
    HIPCHK(hipMalloc(&q, cap * sizeof(T)));
    if (fill_byte >= 0) HIPCHK(hipMemsetAsync(q, fill_byte, cap * sizeof(T), st));
    if (p && keep) HIPCHK(hipMemcpyAsync(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    free_();
    p = q;
    n = cap;
  }
};

inline int div_up(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
static const int32_t kInf = INF32;

}  // namespace

struct hge_engine {
  int N = 0, NW = 1, SM = 1;
  int device = 0;
  hipStream_t st = nullptr;
  std::string err;

  // ---- host control state ----
  std::vector<int32_t> h_creator, h_index, h_sp, h_op, h_ntx;
  std::vector<int64_t> h_ts;
  std::vector<uint64_t> h_S;
  std::vector<uint8_t> h_coin;
  std::vector<int32_t> chain_len, chain_last;
  int64_t n_events = 0;     // accepted (host)
  int64_t n_dev = 0;        // uploaded
  int64_t n_coords = 0;     // coordinates + rounds computed
  int64_t n_divided = 0;    // visible to DecideFame / FindOrder (DivideRounds)
  std::vector<int32_t> coords_len;  // chain lengths at n_coords
  std::vector<int32_t> h_lens;      // staging for the chain-length upload

  int R = 0;                // Store.Rounds()
  int R_set = 0;            // rounds recorded by hge_set_round (Store.SetRound)
  std::vector<std::vector<int32_t>> h_chain;  // participantEventsCache: ids per creator
  int64_t cache_size = 0;   // Store.CacheSize() for the rolling views (0 = unbounded)
  int32_t chain_limit = INT32_MAX;  // longest chain of the uint16 wide path (then: to_wide32)
  int32_t chain_limit0 = INT32_MAX;
  // N > 32 past chain_limit: int32 positions for good (hge_wide32.hip); pending until
  // the next coordinate step converts the packed table
  bool wide32 = false, wide32_pending = false;
  int w32_done = 0;
  // an internal failure that left the host and device state apart: every later
  // consensus call refuses (HGE_ERR_INTERNAL) until a new stream (hge_replay_prepare)
  std::string failed;  // to_wide32's progress: 1 the runs widened, 2 the FD rows, 4 the int32 LA table allocated
  // test hook (HGE_TEST_W32_FAIL=k): to_wide32 fails once after its stage k (1 the int32
  // LA table allocated, 2 the runs widened, 3 the FD rows widened)
  int test_w32_fail = getenv("HGE_TEST_W32_FAIL") ? atoi(getenv("HGE_TEST_W32_FAIL")) : 0;
  int lcr = -1;             // LastConsensusRound (-1 nil)
  int lcre = 0;             // LastCommitedRoundEvents
  int64_t ctx = 0;          // ConsensusTransactions
  std::vector<int32_t> consensus;  // the consensus log (unbounded)
  // A replay delivers its order to host memory inside hge_replay_run: one DMA copy from
  // the results block into a pinned buffer sized at hge_replay_prepare (pin_ord), the
  // log's last cons_pin_n ids.  Readers take it from there (hge_replay_order: a view,
  // hge_replay_fetch: one copy); the log's vector gets them on first use
  // (consensus_sync), outside the replay.
  int32_t* pin_ord = nullptr;
  int32_t* pin_ord_dev = nullptr;  // its device-side address (the sorts write there)
  size_t pin_ord_cap = 0;
  int64_t cons_pin_n = 0;
  bool lazy_order = false;
  int64_t consensus_size() const { return (int64_t)consensus.size() + cons_pin_n; }
  void consensus_sync() {
    if (!cons_pin_n) return;
    consensus.insert(consensus.end(), pin_ord, pin_ord + cons_pin_n);
    cons_pin_n = 0;
  }
  void ensure_pin_ord(size_t n) {
    if (n <= pin_ord_cap && pin_ord) return;
    consensus_sync();
    if (pin_ord) HIPCHK(hipHostFree(pin_ord));
    pin_ord = nullptr;
    pin_ord_dev = nullptr;
    pin_ord_cap = 0;
    HIPCHK(hipHostMalloc((void**)&pin_ord, std::max<size_t>(n, 1) * 4, hipHostMallocDefault));
    pin_ord_cap = std::max<size_t>(n, 1);
    void* dp = nullptr;
    pin_ord_dev = hipHostGetDevicePointer(&dp, pin_ord, 0) == hipSuccess ? (int32_t*)dp : nullptr;
  }
  int64_t n_und = 0;

  // replay staging
  std::vector<int64_t> replay_calls;  // n_c per call (accepted counts)
  std::vector<int64_t> replay_counts;

  // ---- device tables ----
  int64_t Ecap = 0;
  int ccap = 0, Rcap = 0;
  DBuf<int32_t> d_creator, d_index, d_sp, d_op, d_ntx, d_round, d_rr, d_und;
  DBuf<int64_t> d_ts, d_cts;
  DBuf<uint64_t> d_S;
  DBuf<uint8_t> d_coin, d_wit;
  DBuf<int32_t> d_chain, d_LA, d_FD, d_FSS;
  DBuf<int32_t> s_w32, s_w32a;  // to_wide32 / rounds_step32 scratch
  DBuf<uint32_t> d_LA16;  // N > 32: the sweeps' packed (LA + 1) table (hge_coords.hip)
  DBuf<int2> d_opcp;  // [N][ccap] other-parent coordinates (k_chain_fill)
  DBuf<int64_t> d_tsch;  // [N][ccap] timestamps in chain layout (k_chain_fill)
  DBuf<int32_t> d_C, d_W, d_rcnt, d_minw;
  DBuf<uint64_t> d_ssb, d_seeb;
  DBuf<uint8_t> d_fame;
  // scratch
  DBuf<int32_t> s_small, s_newwit;
  DBuf<int32_t> s_LCR, s_clast;
  DBuf<uint8_t> s_dec, s_decbit;
  DBuf<int32_t> s_segcnt, s_segcall, s_seground, s_theta;
  DBuf<uint8_t> s_segdec;
  DBuf<uint64_t> s_segfws;
  DBuf<int32_t> s_recv, s_rr, s_fund, s_upos, s_und2, s_bpos, s_vis;
  bool vis_all = false;  // this batch: one call seeing every event (no visibility table)
  DBuf<int64_t> s_cts;
  DBuf<unsigned char> s_keys, s_keys2;
  DBuf<int32_t> s_part, s_fst, s_relay, s_rfail;
  DBuf<uint8_t> s_dec2;  // selective fame widening: the new layout's decisions
  bool fst_fused = false;  // this batch's k_la_seq ran k_frontier_start's block
  bool fd_direct = false;  // this batch's k_la_seq wrote the FD rows (N <= 16)
  bool asg_fused = false;  // this attempt's rounds walk assigned the new events' rounds
  bool tail_fused = false;  // ... and did k_round_tail's work
  bool minw_full = true;    // d_minw's rows are stale: the next rounds tail recomputes all
  // coordinate sweeps: transposed tables and scratch
  int n_sweeps = 0;
  DBuf<int32_t> d_FDT, s_chg, s_bar, s_dirty;
  DBuf<int32_t> s_src;  // hge_consensus_timestamp_sources: ids, then their sources
  // windowed lastAncestors (hge_coords_win.hip): chunk plans, row sums, starting rows
  DBuf<int4> s_lwplan;
  DBuf<uint32_t> s_lwsum, s_lwinit;
  DBuf<int32_t> s_lwpos, s_lwrisky;
  int ncu_cache = 0;
  int n_cu() {
    if (!ncu_cache) HIPCHK(hipDeviceGetAttribute(&ncu_cache, hipDeviceAttributeMultiprocessorCount, device));
    return ncu_cache;
  }
  DBuf<int32_t> d_FDTD;  // N > 16: timestamp offsets at the FD positions (the wide median)
  DBuf<uint8_t> d_FDTW;  // N > 16: per (row, 64-column tile) out-of-range flags of d_FDTD
  DBuf<int32_t> d_WLA;   // N > 16: round frontier rows transposed (k_witness_la)
  DBuf<uint16_t> d_WLR;  // N > 64, packed path: the same rows row-major as LA + 1 (theta)
  DBuf<uint64_t> d_ssc, s_gran;
  DBuf<int32_t> s_bseg;
  DBuf<uint64_t> s_H;                // speculative walk: epoch-tagged histories
  DBuf<int32_t> s_hn, s_hres;        // rows written + progress hints, merge results
  uint32_t walk_epoch = 0;
  int walk_chk[2] = {448, 2};        // checker threads, poll pause
  bool coop_checked = false;
  int coop_nb = 0, coop_ncu = 0, coop_spec_nb = -1, coop_spec_bs = 0;
  const void* coop_spec_fn() const {
    return coop_spec_bs == 1024 ? (const void*)k_rounds_coop_spec<1024> : (const void*)k_rounds_coop_spec<512>;
  }
  DBuf<uint64_t> s_cH, s_cS, s_cT, s_cM;  // speculative wide walk: rows, ssc bits, tables, merges
  DBuf<uint32_t> s_mb;                    // direct rounds: staged member rows (two parity blocks)
  DBuf<int32_t> s_cn;
  uint32_t coop_epoch = 0;

  hipEvent_t ev[8] = {};
  // per-kernel HIP-event timing on the engine stream (hge_set_profiling)
  bool prof_on = false;
  std::vector<hipEvent_t> prof_pool;
  std::vector<std::pair<std::string, int>> prof_rec;
  std::vector<std::string> prof_names;
  std::vector<double> prof_ms;
  std::vector<int64_t> prof_cnt;
  int R_div = 0;            // Rounds() as seen by the consensus calls (DivideRounds)
  std::vector<int32_t> h_minw;  // first witness id per round (read back by coords)
  // consensus control block (one upload) and results block (one readback)
  DBuf<int32_t> s_cctl, s_out;
  std::vector<int32_t> h_cctl;
  int64_t* c_nc = nullptr;
  int32_t *c_Rc = nullptr, *c_Lc = nullptr, *c_flags = nullptr, *c_pr = nullptr, *c_pidx = nullptr;
  int32_t* c_sgo = nullptr;
  const int32_t* segoff_p = nullptr;  // segment offsets used by k_round_received
  // coordinates control block (coords): pointers into s_kctl
  DBuf<int32_t> s_kctl;
  std::vector<int32_t> h_kctl;
  std::vector<int2> h_segs;
  bool qlo_fused = false;  // k_fd_qlo ran with k_chain_fill (coords_a)
  int32_t *k_rs = nullptr, *k_len = nullptr, *k_plo = nullptr, *k_qlo = nullptr, *k_lo = nullptr;
  int2* k_segs = nullptr;
  int32_t* k_segbase = nullptr;
  int32_t* k_fd = nullptr;  // split: the candidates' chain positions [lo N, hi N)
  int32_t* k_risky1 = nullptr;  // la_windows_run's one-window risky id (-1 as uploaded)
  bool und_fresh = false;  // the candidate list is every event of a fresh replay
  float stage_ms[7] = {};

  Tables tables() const {
    Tables t;
    t.N = N;
    t.NW = NW;
    t.SM = SM;
    t.ccap = ccap;
    t.Rcap = Rcap;
    t.creator = d_creator.p;
    t.index = d_index.p;
    t.sp = d_sp.p;
    t.op = d_op.p;
    t.ts = d_ts.p;
    t.S = d_S.p;
    t.coin = d_coin.p;
    t.ntx = d_ntx.p;
    t.chain = d_chain.p;
    t.opcp = d_opcp.p;
    t.tsch = d_tsch.p;
    t.LA = d_LA.p;
    t.NW2 = (N + 1) / 2;
    t.LA16 = sweep16() ? d_LA16.p : nullptr;  // null: int32 rows (la_row)
    t.FD = fdt16() ? nullptr : d_FD.p;
    t.FD16 = fdt16() ? (uint16_t*)d_FD.p : nullptr;
    t.FDTD = d_FDTD.p;
    t.FDTW = d_FDTW.p;
    t.WLA = wla16() ? nullptr : d_WLA.p;
    t.WLA16 = wla16() ? (uint16_t*)d_WLA.p : nullptr;
    t.WLR = (N > 64 && !wide32) ? d_WLR.p : nullptr;
    t.round = d_round.p;
    t.wit = d_wit.p;
    t.C = d_C.p;
    t.W = d_W.p;
    t.ssb = d_ssb.p;
    t.seeb = d_seeb.p;
    t.fame = d_fame.p;
    t.rcnt = d_rcnt.p;
    return t;
  }

  // ------------------------------------------------------------------------
  void init(int n, int64_t cap, int dev) {
    N = n;
    NW = (N + 63) / 64;
    SM = 2 * N / 3 + 1;  // hashgraph.go:78-80
    device = dev;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    chain_len.assign(N, 0);
    chain_last.assign(N, -1);
    h_chain.assign(N, {});
    // the wide kernels keep chain positions as uint16 (LA16, the rounds walk, theta):
    // a longer chain switches the engine to int32 positions (to_wide32).
    // HGE_CHAIN_LIMIT (tests) lowers the switch point.
    chain_limit = N > 32 ? 0xFFFE : INT32_MAX;
    if (const char* cl = getenv("HGE_CHAIN_LIMIT")) chain_limit = std::max(1, std::min(chain_limit, atoi(cl)));
    chain_limit0 = chain_limit;
    coords_len.assign(N, 0);
    // chain tables: a creator's chain is ~cap/N long (binomial, sd ~ sqrt(cap/N));
    // rounds: a round spans >= ~4N events in gossip.  Both grow on demand.
    const int64_t c0 = std::max<int64_t>(cap, 1024);
    ensure_events(c0);
    ensure_ccap(c0 / N + c0 / (8 * N) + 64);
    ensure_rcap(c0 / (2 * N) + 64);
    s_small.need(16);
  }

  void prof_begin(const char* name) {
    if (!prof_on) return;
    const int slot = (int)prof_rec.size() * 2;
    while ((int)prof_pool.size() < slot + 2) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      prof_pool.push_back(e);
    }
    HIPCHK(hipEventRecord(prof_pool[slot], st));
    prof_rec.push_back({name, slot});
  }
  void prof_end() {
    if (!prof_on) return;
    HIPCHK(hipEventRecord(prof_pool[prof_rec.back().second + 1], st));
  }
  void prof_collect() {
    if (prof_rec.empty()) return;
    HIPCHK(hipStreamSynchronize(st));
    for (auto& r : prof_rec) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, prof_pool[r.second], prof_pool[r.second + 1]));
      size_t k = 0;
      while (k < prof_names.size() && prof_names[k] != r.first) k++;
      if (k == prof_names.size()) {
        prof_names.push_back(r.first);
        prof_ms.push_back(0);
        prof_cnt.push_back(0);
      }
      prof_ms[k] += ms;
      prof_cnt[k] += 1;
    }
    prof_rec.clear();
  }

  // diagnostic stamps (HGE_STAMPS=1): per-section cycle counters of some kernels
  DBuf<uint64_t> s_dbg;
  bool dbg_on = getenv("HGE_STAMPS") != nullptr;
  uint64_t* dbg_p() {
    if (!dbg_on) return nullptr;
    if (!s_dbg.p) {
      s_dbg.need(16);
      HIPCHK(hipMemset(s_dbg.p, 0, 16 * 8));
    }
    return s_dbg.p;
  }
  void dbg_dump() {
    if (!dbg_on || !s_dbg.p) return;
    uint64_t v[16];
    readback(v, s_dbg.p, 16);
    fprintf(stderr, "[hge stamps]");
    for (int i = 0; i < 16; i++) fprintf(stderr, " %llu", (unsigned long long)v[i]);
    fprintf(stderr, "\n");
  }

  void destroy() {
    if (st) (void)hipStreamSynchronize(st);
    if (getenv("HGE_HOST_PHASES") && hp.calls) {
      const double c = (double)hp.calls;
      fprintf(stderr,
              "{\"hge_host_phases\": {\"calls\": %lld, \"launches_per_call\": %.2f, \"copies_per_call\": %.2f, "
              "\"insert_us\": %.2f, \"consensus_us\": %.2f, \"sync_wait_us\": %.2f}}\n",
              (long long)hp.calls, hp.launches / c, hp.copies / c, hp.insert_ns / c / 1e3, hp.call_ns / c / 1e3,
              hp.wait_ns / c / 1e3);
    }
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : prof_pool) (void)hipEventDestroy(e);
    prof_pool.clear();
    DBuf<int32_t>* i32s[] = {&d_creator, &d_index,  &d_sp,    &d_op,     &d_ntx,     &d_round,
                             &d_rr,      &d_und,    &d_chain, &d_LA,     &d_FD,      &d_C,
                             &d_W,       &d_rcnt,   &d_minw,  &s_small,  &s_newwit,  &s_LCR,
                             &s_clast,   &s_segcnt, &s_segcall, &s_seground, &s_theta,
                             &s_recv,    &s_rr,     &s_bpos,  &s_fund,   &s_upos,    &s_vis,
                             &s_und2,    &s_part,   &s_fst,    &d_FSS,
                             &d_FDT,     &s_chg,    &s_bar,   &s_bseg,   &s_kctl,    &s_cctl,
                             &s_out,     &s_hn,     &s_hres,  &s_dirty,  &d_WLA,     &s_lwpos,
                             &s_lwrisky, &s_src,    &s_relay, &s_rfail};
    for (auto* b : i32s) b->free_();
    s_dec2.free_();
    s_lwplan.free_();
    d_WLR.free_();
    s_xbuf.free_();
    s_sord.free_();
    s_soff.free_();
    s_lwsum.free_();
    s_lwinit.free_();
    d_ts.free_();
    d_FDTD.free_();
    d_FDTW.free_();
    d_cts.free_();
    s_cts.free_();
    d_S.free_();
    d_ssb.free_();
    d_seeb.free_();
    s_H.free_();
    s_wdbg.free_();
    s_segfws.free_();
    d_coin.free_();
    d_wit.free_();
    d_fame.free_();
    s_dec.free_();
    s_decbit.free_();
    s_segdec.free_();
    s_keys.free_();
    s_keys2.free_();
    d_opcp.free_();
    d_tsch.free_();
    d_LA16.free_();
    d_ssc.free_();
    s_gran.free_();
    s_cH.free_();
    s_cS.free_();
    s_cT.free_();
    s_cM.free_();
    s_cn.free_();
    s_mb.free_();
    s_hist.free_();
    s_hstate.free_();
    s_hssc.free_();
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    pin_cap = pin_used = 0;
    if (pin_ord) (void)hipHostFree(pin_ord);
    pin_ord = nullptr;
    pin_ord_dev = nullptr;
    pin_ord_cap = 0;
    cons_pin_n = 0;
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
  }

  void ensure_events(int64_t m) {
    if (m <= Ecap) return;
    int64_t cap = std::max<int64_t>(m, Ecap + Ecap / 2);
    d_creator.grow_keep(cap, n_dev, st);
    d_index.grow_keep(cap, n_dev, st);
    d_sp.grow_keep(cap, n_dev, st);
    d_op.grow_keep(cap, n_dev, st);
    d_ntx.grow_keep(cap, n_dev, st);
    d_ts.grow_keep(cap, n_dev, st);
    d_S.grow_keep(4 * cap, 4 * n_dev, st);
    d_coin.grow_keep(cap, n_dev, st);
    d_round.grow_keep(cap, n_coords, st);
    d_wit.grow_keep(cap, n_coords, st);
    d_rr.grow_keep(cap, n_coords, st, 0xFF);
    d_cts.grow_keep(cap, n_coords, st, 0);
    d_und.grow_keep(cap, n_und, st);
    Ecap = cap;
  }

  // chain-major tables [N][ccap][N]: grow to nc positions per chain, keeping contents
  // rowmajor: [N][ccap][N] (LA, FD, FSS); else [N][N][ccap] (LAT, FDT)
  template <typename T>
  void grow_chain_table(DBuf<T>& b, int64_t nc, bool keep, bool rowmajor = true) {
    T* q = nullptr;
    HIPCHK(hipMalloc(&q, sizeof(T) * (size_t)N * nc * N));
    const size_t rows = rowmajor ? N : (size_t)N * N, w = rowmajor ? N : 1;
    if (keep && ccap > 0 && b.p)
      HIPCHK(hipMemcpy2DAsync(q, sizeof(T) * nc * w, b.p, sizeof(T) * ccap * w,
                              sizeof(T) * ccap * w, rows, hipMemcpyDeviceToDevice, st));
    sync();
    b.free_();
    b.p = q;
    b.n = (size_t)N * nc * N;
  }

  void ensure_ccap(int64_t m) {
    if (m <= ccap) return;
    // a multiple of 64 positions: the uint16 run table's rows stay 8-byte aligned
    int64_t nc = (std::max<int64_t>(m, (int64_t)ccap + ccap / 2) + 63) & ~(int64_t)63;
    int32_t* chain = nullptr;
    HIPCHK(hipMalloc(&chain, sizeof(int32_t) * N * nc));
    HIPCHK(hipMemsetAsync(chain, 0xFF, sizeof(int32_t) * N * nc, st));
    if (ccap > 0)
      HIPCHK(hipMemcpy2DAsync(chain, sizeof(int32_t) * nc, d_chain.p, sizeof(int32_t) * ccap,
                              sizeof(int32_t) * ccap, N, hipMemcpyDeviceToDevice, st));
    sync();
    d_chain.free_();
    d_chain.p = chain;
    d_chain.n = (size_t)N * nc;
    int2* opcp = nullptr;
    HIPCHK(hipMalloc(&opcp, sizeof(int2) * N * nc));
    if (ccap > 0)
      HIPCHK(hipMemcpy2DAsync(opcp, sizeof(int2) * nc, d_opcp.p, sizeof(int2) * ccap,
                              sizeof(int2) * ccap, N, hipMemcpyDeviceToDevice, st));
    sync();
    d_opcp.free_();
    d_opcp.p = opcp;
    d_opcp.n = (size_t)N * nc;
    int64_t* tsch = nullptr;
    HIPCHK(hipMalloc(&tsch, sizeof(int64_t) * N * nc));
    if (ccap > 0)
      HIPCHK(hipMemcpy2DAsync(tsch, sizeof(int64_t) * nc, d_tsch.p, sizeof(int64_t) * ccap,
                              sizeof(int64_t) * ccap, N, hipMemcpyDeviceToDevice, st));
    sync();
    d_tsch.free_();
    d_tsch.p = tsch;
    d_tsch.n = (size_t)N * nc;
    if (!sweep16()) grow_chain_table(d_LA, nc, true);
    if (N > 32) {  // (kept across a switch to int32: a later stream starts packed again)
      const size_t w = (size_t)(N + 1) / 2;
      uint32_t* q = nullptr;
      HIPCHK(hipMalloc(&q, sizeof(uint32_t) * (size_t)N * nc * w));
      if (ccap > 0 && d_LA16.p)
        HIPCHK(hipMemcpy2DAsync(q, sizeof(uint32_t) * nc * w, d_LA16.p, sizeof(uint32_t) * ccap * w,
                                sizeof(uint32_t) * ccap * w, N, hipMemcpyDeviceToDevice, st));
      sync();
      d_LA16.free_();
      d_LA16.p = q;
      d_LA16.n = (size_t)N * nc * w;
    }
    if (fdt16()) {  // uint16 FD rows: a chain's block is ccap * N halves
      int32_t* q = nullptr;
      HIPCHK(hipMalloc(&q, sizeof(uint16_t) * (size_t)N * nc * N));
      if (ccap > 0 && d_FD.p)
        HIPCHK(hipMemcpy2DAsync(q, 2 * (size_t)nc * N, d_FD.p, 2 * (size_t)ccap * N, 2 * (size_t)ccap * N, N,
                                hipMemcpyDeviceToDevice, st));
      sync();
      d_FD.free_();
      d_FD.p = q;
      d_FD.n = (size_t)N * nc * N / 2;
    } else {
      grow_chain_table(d_FD, nc, true);
    }
    if (N > 16) {  // FD timestamp rows below a batch's qlo are kept
      grow_chain_table(d_FDTD, nc, true);
      const size_t NT = (size_t)(N + 63) / 64;
      uint8_t* q = nullptr;
      HIPCHK(hipMalloc(&q, (size_t)N * nc * NT));
      if (ccap > 0 && d_FDTW.p)
        HIPCHK(hipMemcpy2DAsync(q, nc * NT, d_FDTW.p, (size_t)ccap * NT, (size_t)ccap * NT, N,
                                hipMemcpyDeviceToDevice, st));
      sync();
      d_FDTW.free_();
      d_FDTW.p = q;
      d_FDTW.n = (size_t)N * nc * NT;
    }
    // first-strong-seer rows (N <= 32): int32 rows of N, or uint16 rows padded to
    // 16/32 columns for the LDS walk; rebuilt from the frontier on, never kept
    if (N <= 32) d_FSS.need((size_t)N * nc * std::max(N, 16));
    if (fdt16()) {  // uint16 runs: rows of ccap halves (the buffer keeps int32 capacity)
      int32_t* q = nullptr;
      HIPCHK(hipMalloc(&q, sizeof(int32_t) * (size_t)N * nc * N));
      if (ccap > 0 && d_FDT.p)
        HIPCHK(hipMemcpy2DAsync(q, 2 * (size_t)nc, d_FDT.p, 2 * (size_t)ccap, 2 * (size_t)ccap, (size_t)N * N,
                                hipMemcpyDeviceToDevice, st));
      sync();
      d_FDT.free_();
      d_FDT.p = q;
      d_FDT.n = (size_t)N * nc * N;
    } else {
      grow_chain_table(d_FDT, nc, true, false);  // persistent: FD in run layout
    }
    ccap = (int)nc;
  }

  void ensure_rcap(int64_t m) {
    if (m <= Rcap) return;
    int64_t nr = std::max<int64_t>(m, (int64_t)Rcap + Rcap / 2);
    const size_t oldn = (size_t)Rcap * N;
    d_C.grow_keep(nr * N, oldn, st, 0x7F);  // 0x7F7F7F7F is not INF32: fixed below
    d_W.grow_keep(nr * N, oldn, st, 0xFF);
    d_ssb.grow_keep(nr * N * NW, oldn * NW, st, 0);
    d_seeb.grow_keep(nr * N * NW, oldn * NW, st, 0);
    if (N > 32) d_ssc.grow_keep(nr * N * NW, oldn * NW, st, 0);
    d_fame.grow_keep(nr * N, oldn, st, 0);
    d_rcnt.grow_keep(nr, Rcap, st, 0);
    // + round count, overflow flag, lowest candidate round, hand-off error and up to 16
    // partial lowest rounds (k_round_minw)
    d_minw.need(nr + 20);
    minw_full = true;  // (need() does not keep the rows' first witnesses)
    // C must be INF32 beyond the old rows
    fill_i32(d_C.p + oldn, (int64_t)(nr - Rcap) * N, INF32);
    sync();
    Rcap = (int)nr;
  }

  void reset_state() {
    sync();
    failed.clear();  // a new stream (hge_reset, hge_replay_prepare)
    minw_full = true;
    cons_pin_n = 0;
    h_creator.clear();
    h_index.clear();
    h_sp.clear();
    h_op.clear();
    h_ntx.clear();
    h_ts.clear();
    h_S.clear();
    h_coin.clear();
    chain_len.assign(N, 0);
    chain_last.assign(N, -1);
    h_chain.assign(N, {});
    coords_len.assign(N, 0);
    n_events = n_dev = n_coords = n_divided = 0;
    up_n0 = up_n1 = -1;
    h_up.clear();
    R = 0;
    R_set = 0;
    h_minw.clear();
    lcr = -1;
    lcre = 0;
    ctx = 0;
    consensus.clear();
    n_und = 0;
    wide32 = wide32_pending = false;  // a new stream starts on the packed path
    w32_done = 0;
    chain_limit = chain_limit0;
    reset_rounds();
    HIPCHK(hipMemsetAsync(d_chain.p, 0xFF, (size_t)N * ccap * 4, st));
    sync();
  }

  // fresh per-round tables (C, W, bitsets, fame, counts) and received rounds: one launch
  void reset_rounds() {
    const int64_t nrow = (int64_t)Rcap * N, nbits = nrow * NW;
    const int64_t most = std::max<int64_t>(std::max(nbits, Ecap), Rcap);
    KLAUNCH(k_reset_rounds, dim3(std::min(div_up(most, 256), 4096)), dim3(256), 0, st, tables(), nrow,
            nbits, Ecap, d_rr.p);
  }

  // ---------------- admission (hashgraph.go:366-396) ----------------
  int admit(const hge_event& e, int32_t sp, int32_t op) {
    const int c = e.creator;
    if (c < 0 || c >= N) {
      err = "Could not find fake creator id";
      return HGE_ERR_CREATOR;
    }
    const int known = chain_len[c];
    if (sp == HGE_NONE && op == HGE_NONE && known == 0) {
      if (e.index != 0) {
        err = "Event index does not match the creator's chain position";
        return HGE_ERR_INDEX;
      }
      return HGE_OK;
    }
    if (sp < 0 || sp >= n_events) {
      err = "Self-parent not known";
      return HGE_ERR_SELF_PARENT_UNKNOWN;
    }
    if (h_creator[sp] != c) {
      err = "Self-parent has different creator";
      return HGE_ERR_SELF_PARENT_CREATOR;
    }
    if (op < 0 || op >= n_events) {
      err = "Other-parent not known";
      return HGE_ERR_OTHER_PARENT_UNKNOWN;
    }
    if (sp != chain_last[c]) {
      err = "Self-parent not last known event by creator";
      return HGE_ERR_SELF_PARENT_NOT_LAST;
    }
    if (e.index != known) {
      err = "Event index does not match the creator's chain position";
      return HGE_ERR_INDEX;
    }
    if (known >= chain_limit) {
      if (N > 32 && N <= 256 && !wide32) {  // past the uint16 positions: int32 from here on
        // the int32 LA table must fit beside what is allocated: else refuse
        // the event here (the stream stops, as at any rejection) rather than lift
        // the cap and fail at the next coordinate step
        // to_wide32's peak: the int32 LA table, plus (uint16 runs and FD rows) one
        // int32 table being widened while the other's old copy is still held
        size_t free_b = 0, total_b = 0;
        const size_t tab = sizeof(int32_t) * (size_t)N * N * (size_t)std::max(ccap, known + 2);
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b < (fdt16() ? 2 : 1) * tab + (64u << 20)) {
          err = "Chain capacity exceeded: the int32 position tables past 65,534 events per creator do not fit";
          return HGE_ERR_CAPACITY;
        }
        wide32_pending = true;
        chain_limit = INT32_MAX;
      } else {
        err = "Chain capacity exceeded: at most " + std::to_string(chain_limit) + " events per creator";
        return HGE_ERR_CAPACITY;
      }
    }
    return HGE_OK;
  }

  void append(const hge_event& e, int32_t sp, int32_t op) {
    const int64_t id = n_events++;
    h_creator.push_back(e.creator);
    h_index.push_back(e.index);
    h_sp.push_back(sp);
    h_op.push_back(op);
    h_ntx.push_back(e.n_tx);
    h_ts.push_back(e.timestamp_ns);
    for (int k = 0; k < 4; k++) {
      uint64_t v = 0;
      for (int b = 0; b < 8; b++) v = (v << 8) | e.s[8 * k + b];
      h_S.push_back(v);
    }
    h_coin.push_back(e.hash[16] != 0 ? 1 : 0);
    h_chain[e.creator].push_back((int32_t)id);
    chain_len[e.creator]++;
    chain_last[e.creator] = (int32_t)id;
  }

  // a packed upload of the events [up_n0, up_n1) waiting for k_chain_fill (upload())
  std::vector<UpEv> h_up;  // the packed records, uploaded with coords_a's control block
  int64_t up_n0 = -1, up_n1 = -1;
  void upload() {
    if (n_dev == n_events) return;
    ensure_events(n_events);
    int maxlen = 0;
    for (int c = 0; c < N; c++) maxlen = std::max(maxlen, chain_len[c]);
    ensure_ccap(maxlen + 1);
    const int64_t a = n_dev, m = n_events - n_dev;
    if (m <= 16384 && a == n_coords) {
      // a small batch (an online call): one packed record per event through the
      // pinned arena, unpacked by the coordinate step's k_chain_fill (eight copies
      // from pageable memory were ~25 us of an online call)
      std::vector<UpEv> up((size_t)m);
      if (up_n0 >= 0) throw EngineError(HGE_ERR_INTERNAL, "packed upload pending twice");
      for (int64_t i = 0; i < m; i++) {
        UpEv& r = up[(size_t)i];
        const size_t x = (size_t)(a + i);
        r.creator = h_creator[x];
        r.index = h_index[x];
        r.sp = h_sp[x];
        r.op = h_op[x];
        r.ntx = h_ntx[x];
        r.coin = h_coin[x];
        r.ts = h_ts[x];
        for (int k = 0; k < 4; k++) r.S[k] = h_S[4 * x + k];
      }
      // (they travel with the coordinate step's control block: one copy for both)
      h_up.swap(up);
      up_n0 = a;
      up_n1 = n_events;
      n_dev = n_events;
      return;
    }
    HIPCHK(hipMemcpyAsync(d_creator.p + a, h_creator.data() + a, 4 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_index.p + a, h_index.data() + a, 4 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_sp.p + a, h_sp.data() + a, 4 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_op.p + a, h_op.data() + a, 4 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_ntx.p + a, h_ntx.data() + a, 4 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_ts.p + a, h_ts.data() + a, 8 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_S.p + 4 * a, h_S.data() + 4 * a, 32 * m, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_coin.p + a, h_coin.data() + a, m, hipMemcpyHostToDevice, st));
    n_dev = n_events;
  }

  void fill_iota(int32_t* p, int64_t n, int32_t base) {
    if (n > 0) KLAUNCH(k_iota, dim3(div_up(n, 256)), dim3(256), 0, st, p, n, base);
  }

  void fill_i32(int32_t* p, int64_t n, int32_t v) {
    if (n > 0) KLAUNCH(k_fill_i32, dim3(div_up(n, 256)), dim3(256), 0, st, p, n, v);
  }

  // ---- host <-> device staging through pinned memory ----
  // A copy from pageable memory makes the runtime wait for the stream, so every
  // small control upload would be a hidden round trip.  Control data goes through
  // a pinned arena instead: uploads are enqueued without waiting, downloads are
  // queued and land in their host destinations at the next sync(), which also
  // recycles the arena (everything enqueued before it has completed).
  char* pin = nullptr;
  size_t pin_cap = 0, pin_used = 0;
  struct Pending {
    void* dst;
    size_t off, bytes;
  };
  std::vector<Pending> pending;

  char* pin_take(size_t bytes) {
    const size_t need = (bytes + 255) & ~(size_t)255;
    if (pin_used + need > pin_cap) {
      sync();
      if (need > pin_cap) {
        if (pin) HIPCHK(hipHostFree(pin));
        pin = nullptr;
        pin_cap = std::max<size_t>(need, std::max<size_t>(2 * pin_cap, 1 << 16));
        HIPCHK(hipHostMalloc((void**)&pin, pin_cap, hipHostMallocDefault));
      }
    }
    char* q = pin + pin_used;
    pin_used += need;
    return q;
  }
  void h2d(void* dev, const void* host, size_t bytes) {
    if (!bytes) return;
    char* q = pin_take(bytes);
    memcpy(q, host, bytes);
    hp.copies++;
    HIPCHK(hipMemcpyAsync(dev, q, bytes, hipMemcpyHostToDevice, st));
  }
  void d2h(void* host, const void* dev, size_t bytes) {
    if (!bytes) return;
    char* q = pin_take(bytes);
    hp.copies++;
    HIPCHK(hipMemcpyAsync(q, dev, bytes, hipMemcpyDeviceToHost, st));
    pending.push_back({host, (size_t)(q - pin), bytes});
  }
  // download into the arena itself: the returned offset stays readable after the
  // next sync() until the arena is used again (no second host copy)
  size_t d2h_pinned(const void* dev, size_t bytes) {
    char* q = pin_take(bytes);
    if (bytes) hp.copies++;
    if (bytes) HIPCHK(hipMemcpyAsync(q, dev, bytes, hipMemcpyDeviceToHost, st));
    return (size_t)(q - pin);
  }
  int64_t n_syncs = 0;  // host waits on the stream (hge_host_syncs)
  // where an online call's host time goes (HGE_HOST_PHASES=1: printed at destroy):
  // calls, launches, copies, ns spent inside hipStreamSynchronize, ns in the calls
  struct HostPhases {
    int64_t calls = 0, launches = 0, copies = 0, wait_ns = 0, call_ns = 0, insert_ns = 0;
  } hp;
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void sync() {
    n_syncs++;
    const int64_t w0 = now_ns();
    HIPCHK(hipStreamSynchronize(st));
    hp.wait_ns += now_ns() - w0;
    for (const Pending& pd : pending) memcpy(pd.dst, pin + pd.off, pd.bytes);
    pending.clear();
    pin_used = 0;
  }
  template <typename F>
  void readback(F* host, const F* dev, size_t n) {
    d2h(host, dev, n * sizeof(F));
    sync();
  }

  // ---------------- coordinates + rounds for [n_coords, n_events) ----------------
  // coordinates + rounds for [n_coords, n_events): coords_a (sweeps and
  // transposes) then coords_b (the rounds frontier and what follows).  The
  // cross-GPU split (hge_split_*) runs a walker between the two.
  bool cs_pending = false, cs_fresh = false;
  std::chrono::steady_clock::time_point w_start;
  // cross-GPU split: the joined frontier rows of the walkers (hge_split_finish)
  bool ext_on = false, ext_natural = false;
  int ext_rows = 0;
  std::vector<int32_t> ext_C;
  std::vector<uint64_t> ext_ssc;
  DBuf<int32_t> s_hist, s_hstate;
  DBuf<uint64_t> s_hssc;
  // One hashgraph sharded across GPUs by time (hge_split_plan): part
  // p owns the events [a_p, a_{p+1}) and the calls [cb_p, cb_{p+1}).  Every part
  // computes the coordinates and walks the rounds recurrence (sequential: it cannot
  // be split exactly); part p then decides the fame of the rounds whose
  // first witness it owns and commits the events its calls receive (candidates from
  // cand_lo_p, the only FD timestamp rows it writes), and the parts exchange fame
  // decisions and ordered slices through the caller's all-gather (hge_split_exchange).
  struct SplitPlan {
    int part = 0, nparts = 0;
    std::vector<int64_t> a;     // event bounds, nparts + 1
    std::vector<int32_t> cb;    // call bounds, nparts + 1
    std::vector<int64_t> clo;   // first candidate of every part
  } sp;
  bool sp_active = false;  // during hge_split_run
  bool split_on() const { return sp_active && sp.nparts > 1; }
  hge_exchange_fn x_fn = nullptr;
  void* x_ctx = nullptr;
  // measurement aid (hge_split_emulate): an unsplit replay records what every part
  // of a split contributes to the exchanges (the fame decisions of every fame
  // iteration, the order, per-call batches, round received / timestamps, the
  // undetermined list); a split part run without an exchange then takes the other
  // parts' slots from the record, so one GPU times each part of a G-way split alone
  bool rec_on = false, rec_have = false;
  std::vector<std::vector<uint8_t>> rec_dec;
  std::vector<int32_t> rec_order, rec_rr, rec_left;
  std::vector<int64_t> rec_counts, rec_cts;
  int x_iter = 0;  // fame iteration of the current batch (the record's index)
  DBuf<uint8_t> s_xbuf;
  bool emulating() const { return split_on() && !x_fn && rec_have; }
  DBuf<int32_t> s_sord;   // split: every part's ordered ids
  DBuf<int64_t> s_soff;   // split: their offsets
  // a device buffer of nparts slots of `bytes` (the caller's memory: its collectives
  // write into it), then the all-gather: this part's slot is filled and the stream drained
  void* x_buf(int64_t bytes) {
    sync();  // the caller may hand out (or move) the memory of the previous exchange
    if (emulating()) {
      s_xbuf.need((size_t)bytes * sp.nparts);
      return s_xbuf.p;
    }
    void* b = nullptr;
    if (!x_fn) throw EngineError(HGE_ERR_ARG, "split replay: no exchange (hge_split_exchange)");
    if (x_fn(x_ctx, 0, bytes, &b) != 0 || !b) throw EngineError(HGE_ERR_DEVICE, "split exchange: no buffer");
    return b;
  }
  void x_gather(int64_t bytes, void* b) {
    sync();
    if (emulating()) return;  // the caller fills the other parts' slots from the record
    if (x_fn(x_ctx, 1, bytes, &b) != 0) throw EngineError(HGE_ERR_DEVICE, "split exchange failed");
  }
  // fame rounds of part g: the pr_* indices [k_lo, k_hi) whose round's first witness
  // lies in the part's events (h_minw is ascending in the round)
  void split_rounds_of(int g, const std::vector<int32_t>& pr_round, int& k_lo, int& k_hi) const {
    const int nr = (int)pr_round.size();
    auto first_at = [&](int64_t ev) {
      int lo = 0, hi = nr;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)h_minw[pr_round[mid]] < ev) lo = mid + 1;
        else hi = mid;
      }
      return lo;
    };
    k_lo = g == 0 ? 0 : first_at(sp.a[g]);
    k_hi = g == sp.nparts - 1 ? nr : first_at(sp.a[g + 1]);
  }
  int64_t cs_n0 = 0, cs_n1 = 0;
  // the candidates' lowest round, read back with the round count (coords_b) for the
  // undetermined list of n_und = key[0] + key[2] - key[1] events after the divide
  // that raises n_divided from key[1] to key[2] (key[0] < 0: none)
  int32_t mnr_pre = 0;
  int64_t mnr_key[3] = {-1, 0, 0};
  int cs_tot0 = 0;
  void coords() {
    if (!coords_a()) return;
    coords_b();
  }
  bool coords_a() {
    fst_fused = false;
    upload();
    if (wide32_pending) to_wide32();
    const int64_t n0 = n_coords, n1 = n_events;
    if (n1 == n0) return false;
    Tables t = tables();
    // control block (one upload): round state, chain lengths, transpose bounds,
    // fss offsets of a fresh walk and the sweep segments
    // segment length: latency-bound sweeps (small N) like short segments, bandwidth-bound
    // ones (large N) long ones (fewer stale carries)
    const int SEG = N <= 32 ? 16 : 64;
    std::vector<int2>& segs = h_segs;
    segs.clear();
    // only the fixed-point sweeps read the segment list (the windowed pass and the
    // one-pass batch kernel do not): 156k segments and their sort were ~3 ms of host
    // time at the start of a 256/10M replay
    const bool sweeps = !(sweep16() && la_windows()) && !la_seq_ok(n1 - n0);
    int maxnew = 0;
    for (int c = 0; c < N; c++) {
      maxnew = std::max(maxnew, chain_len[c] - coords_len[c] + 1);
      if (sweeps)
        for (int k = coords_len[c]; k < chain_len[c]; k += SEG) segs.push_back(make_int2(c, k));
    }
    // position-major order: workgroups are dispatched roughly in index order, so
    // early positions of every chain are swept first and later segments read
    // rows already updated in this sweep (Gauss-Seidel in time order)
    if (sweeps)
      std::stable_sort(segs.begin(), segs.end(), [](const int2& a, const int2& b) { return a.y < b.y; });
    bool fresh = R == 0;
    for (int c = 0; c < N; c++) fresh = fresh && coords_len[c] == 0;
    const size_t o_len = 4, o_plo = o_len + 2 * N, o_qlo = o_plo + N, o_lo = o_qlo + N;
    const size_t o_seg = (o_lo + 2 * N + 1 + 1) & ~(size_t)1;
    const size_t o_sb = o_seg + 2 * segs.size();  // chain-major segment bases (sweep skipping)
    const size_t o_fd = o_sb + N;  // split: the chain positions of the part's candidates
    std::vector<int32_t>& kc = h_kctl;
    kc.assign(o_fd + 2 * N + 1, 0);
    kc[o_fd + 2 * N] = -1;  // the one-window lastAncestors pass's risky id (la_windows_run)
    if (split_on()) {
      // FD timestamp rows (the median's input) of the ids [cand_lo, the part's end)
      const int64_t A = sp.clo[sp.part], B = sp.a[sp.part + 1];
      for (int c = 0; c < N; c++) {
        const std::vector<int32_t>& ch = h_chain[c];
        kc[o_fd + c] = (int)(std::lower_bound(ch.begin(), ch.end(), (int32_t)A) - ch.begin());
        kc[o_fd + N + c] = (int)(std::lower_bound(ch.begin(), ch.end(), (int32_t)B) - ch.begin());
      }
    }
    kc[0] = R;  // rstate: {R, overflow}, new-witness count
    int tot0 = 0;
    for (int c = 0; c < N; c++) {
      kc[o_len + c] = coords_len[c];
      kc[o_len + N + c] = chain_len[c];
      kc[o_plo + c] = std::max(coords_len[c] - 1, 0);
      kc[o_lo + N + c] = tot0;  // fresh walk: fss rows from position 0 (qlo = 0 too)
      tot0 += chain_len[c];
    }
    for (int c = 0, b = 0; c < N; c++) {
      kc[o_sb + c] = b;
      b += div_up(chain_len[c] - coords_len[c], SEG);
    }
    kc[o_lo + 2 * N] = tot0;
    if (!segs.empty()) memcpy(&kc[o_seg], segs.data(), sizeof(int2) * segs.size());
    // the packed event records (an online call's upload) ride in the same copy
    const bool packed = up_n0 == n0 && up_n1 == n1;
    const size_t o_up = (kc.size() + 3) & ~(size_t)3;  // 16-byte aligned
    const size_t up_words = packed ? (sizeof(UpEv) * h_up.size() + 3) / 4 : 0;
    if (packed) {
      static_assert(sizeof(UpEv) % 4 == 0, "records are whole words");
      kc.resize(o_up + up_words, 0);
      memcpy(&kc[o_up], h_up.data(), sizeof(UpEv) * h_up.size());
    }
    s_kctl.need(kc.size());
    h2d(s_kctl.p, kc.data(), 4 * kc.size());
    k_rs = s_kctl.p;
    k_len = s_kctl.p + o_len;
    k_plo = s_kctl.p + o_plo;
    k_qlo = s_kctl.p + o_qlo;
    k_lo = s_kctl.p + o_lo;
    k_segs = (int2*)(s_kctl.p + o_seg);
    k_segbase = s_kctl.p + o_sb;
    k_fd = split_on() ? s_kctl.p + o_fd : nullptr;
    k_risky1 = s_kctl.p + o_fd + 2 * N;
    {
      fill_up = packed ? (const UpEv*)(s_kctl.p + o_up) : (const UpEv*)nullptr;
      fill_dst = UpDst{d_creator.p, d_index.p, d_sp.p, d_op.p, d_ntx.p, d_ts.p, d_S.p, d_coin.p};
      up_n0 = up_n1 = -1;
      h_up.clear();
      qlo_fused = false;
      if (!la_seq_ok(n1 - n0)) {  // (k_la_seq fills the chain table itself)
        const int nfb = div_up((int)(n1 - n0), 256);
        if (!fresh && N <= 256) {  // + k_fd_qlo's blocks (coords_b)
          // + k_frontier_start's block for the wide rounds walk (rounds_coop)
          fst_fused = N > 32 && !wide32 && !frontier_fallback && !split_on() && !ext_on;
          if (fst_fused) {
            s_fst.need(N + 1);
            s_bar.need(2);
            s_gran.need(2 * (size_t)N);
          }
          KLAUNCH(k_chain_fill_qlo, dim3(nfb + N + (fst_fused ? 1 : 0)), dim3(256), 0, st, t, (int)n0, (int)n1,
                  fill_up, fill_dst, nfb, (const int32_t*)k_len, (const int32_t*)(k_len + N), k_qlo,
                  fst_fused ? s_fst.p : (int32_t*)nullptr, fst_fused ? s_bar.p : (int32_t*)nullptr,
                  fst_fused ? (uint64_t*)s_gran.p : (uint64_t*)nullptr, 2 * N);
          qlo_fused = true;
        } else {
          KLAUNCH(k_chain_fill, dim3(nfb), dim3(256), 0, st, t, (int)n0, (int)n1, fill_up, fill_dst);
        }
      }
    }
    coords_sweep(t, sweeps ? (int)segs.size() : 1, SEG, maxnew, fresh);
    cs_pending = true;
    cs_fresh = fresh;
    cs_n0 = n0;
    cs_n1 = n1;
    cs_tot0 = tot0;
    return true;
  }
  void coords_b() {
    cs_pending = false;
    const bool fresh = cs_fresh;
    const int64_t n0 = cs_n0, n1 = cs_n1;
    const int tot0 = cs_tot0;
    const int m = (int)(n1 - n0);
    Tables t = tables();
    // rounds frontier
    for (bool retry = false;; retry = true) {
      // the wide frontier grids stay on the device until the sync below: two such
      // grids on one device must not overlap (frontier_lock)
      std::unique_lock<std::mutex> flk;
      if (N > 32) flk = frontier_lock();
      int32_t rs[3] = {R, 0, 0};
      if (retry) h2d(k_rs, rs, 12);
      asg_fused = false;
      tail_fused = false;
      t = tables();
      const int NP = (N + 15) & ~15;
      if (N > 32 && (wide32 || frontier_fallback)) {
        rounds_step32();
      } else if (N > 32) {
        rounds_coop(fresh);
      } else {
        // first-strong-seer rows for every event that can still be a frontier member
        // (from a fresh state the frontier starts at round 0, position 0: no round trip)
        int maxlen = 0;
        for (int c = 0; c < N; c++) maxlen = std::max(maxlen, chain_len[c]);
        const int Rprev = R;  // C rows >= Rprev are empty before this batch
        if (!fresh && maxlen < 0xFFFF) {
          // an online call: the walk's first round, its k_fss rows and their count
          // stay on the device (k_frontier_start writes them; k_fss loops over the
          // count, k_rounds_walk stands down at INF32): no host round trip
          s_fst.need(N + 1);
          if (!fst_fused || retry)  // (else k_la_seq's last block wrote them)
            KLAUNCH(k_frontier_start, dim3(1), dim3(256), 0, st, t, k_len, k_len + N, s_fst.p, k_lo,
                    (int32_t*)nullptr, (uint64_t*)nullptr, 0);
          const int64_t guess = m + 16 * (int64_t)N;  // the grid loops past it
          // the walk's block also assigns the new events' rounds (k_round_assign's work)
          und_appended = dividing && n_divided == n0;
          s_newwit.need(m);
          RoundAssign ra{(int)n0, (int)n1, s_newwit.p, k_rs + 2,
                         und_appended ? d_und.p + n_und : (int32_t*)nullptr};
          asg_fused = true;
          // ... and k_round_tail's work (the new witnesses' bitsets, the first witness
          // of the rounds from the walk's first one, the candidates' lowest round)
          if (n_und + (n1 - n_divided) <= 65536) {
            int Gw = 1;
            while (Gw < std::min(N, 64)) Gw <<= 1;
            ra.minw = d_minw.p;
            ra.G = Gw;
            ra.und = d_und.p;
            ra.n_und = (int)n_und;
            ra.lo = (int)n_divided;
            ra.hi = (int)n1;
            ra.r_from = minw_full ? 0 : -1;
            ra.rlo_dev = s_fst.p;
            tail_fused = true;
          }
#define FSSD(NPC, LPC, B)                                                                              \
  KLAUNCH(k_fss<NPC>, dim3((unsigned)std::min<int64_t>(1024, div_up(guess * NPC, 256))), dim3(256), 0, st, t, \
          k_lo, k_lo + N, 0, (int32_t*)nullptr, (uint16_t*)d_FSS.p, (const int32_t*)(k_lo + 2 * N));          \
  KLAUNCH((k_rounds_walk<NPC, LPC, B>), dim3(1), dim3(1024), 0, st, t, (const uint16_t*)d_FSS.p, k_len,       \
          k_len + N, k_rs, 0, Rprev, dbg_p(), (const int32_t*)s_fst.p, ra);
          if (NP == 16) {
            FSSD(16, 4, 256)
          } else {
            FSSD(32, 2, 64)
          }
#undef FSSD
        } else {
        std::vector<int32_t> fst(N + 1, 0);
        if (!fresh) {
          s_fst.need(N + 1);
          KLAUNCH(k_frontier_start, dim3(1), dim3(256), 0, st, t, k_len, k_len + N, s_fst.p, (int32_t*)nullptr,
                  (int32_t*)nullptr, (uint64_t*)nullptr, 0);
          readback(fst.data(), s_fst.p, N + 1);
        }
        const int rlo = fst[0];
        if (rlo != INF32) {
          int tot = fresh ? tot0 : 0;
          if (!fresh) {
            std::vector<int32_t> lo_off(2 * N + 1);
            for (int c = 0; c < N; c++) {
              lo_off[c] = fst[1 + c];
              lo_off[N + c] = tot;
              tot += std::max(0, chain_len[c] - fst[1 + c]);
            }
            lo_off[2 * N] = tot;
            h2d(k_lo, lo_off.data(), 4 * (2 * N + 1));
          }
          if (tot > 0) {
            // the LDS walk keeps chain positions as uint16; longer chains take the
            // register walk over the global fss rows
#define FSSL(NPC, LPC, B)                                                                          \
  if (maxlen < 0xFFFF) {                                                                           \
    KLAUNCH(k_fss<NPC>, dim3(div_up((int64_t)tot * NPC, 256)), dim3(256), 0, st, t, k_lo, k_lo + N, \
            tot, (int32_t*)nullptr, (uint16_t*)d_FSS.p, (const int32_t*)nullptr);                  \
    const int nw = fresh ? spec_walkers(maxlen) : 0;                                               \
    if (nw > 1) {                                                                                  \
      const char* hc = getenv("HGE_WALK_HCAP"); /* tests: force the capacity fallback */          \
      const int Hcap = hc ? std::max(2, atoi(hc))                                                  \
                          : std::max(256, std::min(Rcap, 3 * (Rcap / nw) + 256));                  \
      if ((size_t)nw * Hcap * N > s_H.n) {                                                         \
        s_H.need((size_t)nw * Hcap * N); /* epoch 0 never matches a launch's tag */                \
        HIPCHK(hipMemsetAsync(s_H.p, 0, s_H.n * sizeof(uint64_t), st));                            \
      }                                                                                            \
      s_hres.need(4 * (size_t)nw + 1);                                                             \
      s_hn.need(2 * (size_t)nw);                                                                   \
      KLAUNCH((k_walk_spec<NPC, LPC, B>), dim3(nw), dim3(1024), 0, st, t,                         \
              (const uint16_t*)d_FSS.p, k_len + N, nw, Hcap, s_H.p, s_hn.p, s_hn.p + nw,          \
              (int4*)s_hres.p, ++walk_epoch, walk_chk[0], walk_chk[1], walk_dbg(nw));              \
      int32_t* resume = s_hres.p + 4 * nw;                                                         \
      KLAUNCH(k_walk_join, dim3(64), dim3(256), 0, st, t, (const uint64_t*)s_H.p,                    \
              (const int32_t*)s_hn.p, (const int4*)s_hres.p, nw, Hcap, k_rs, resume);              \
      KLAUNCH((k_rounds_walk<NPC, LPC, B>), dim3(1), dim3(1024), 0, st, t,                         \
              (const uint16_t*)d_FSS.p, k_len, k_len + N, k_rs, 0, 0, dbg_p(),                     \
              (const int32_t*)resume, RoundAssign{});                                              \
      if (getenv("HGE_WALK_DEBUG")) walk_debug(nw);                                               \
    } else {                                                                                       \
      KLAUNCH((k_rounds_walk<NPC, LPC, B>), dim3(1), dim3(1024), 0, st, t,                         \
              (const uint16_t*)d_FSS.p, k_len, k_len + N, k_rs, rlo, Rprev, dbg_p(),               \
              (const int32_t*)nullptr, RoundAssign{});                                             \
    }                                                                                              \
  } else {                                                                                         \
    KLAUNCH(k_fss<NPC>, dim3(div_up((int64_t)tot * NPC, 256)), dim3(256), 0, st, t, k_lo, k_lo + N, \
            tot, d_FSS.p, (uint16_t*)nullptr, (const int32_t*)nullptr);                            \
    KLAUNCH(k_rounds_fss<NPC>, dim3(1), dim3(64), 0, st, t, d_FSS.p, k_len, k_len + N, k_rs, rlo);  \
  }
            if (NP == 16) {
              FSSL(16, 4, 256)
            } else {
              FSSL(32, 2, 64)
            }
#undef FSSL
          }
        }
        }
      }
      // rounds, witnesses and the first witness of every round, then ONE round
      // trip for the round count and minw (the kernels stand down if the rounds
      // table overflowed: the loop grows it and walks again)
      t = tables();
      s_newwit.need(m);
      if (fresh) {
        s_newwit.need((size_t)Rcap * N);
        KLAUNCH(k_round_ranges, dim3(div_up((int64_t)Rcap * N, 256)), dim3(256), 0, st, t, k_len + N,
                (const int32_t*)k_rs, s_newwit.p, k_rs + 2);
      } else if (!asg_fused) {
        // DivideRounds right after (divide()) with nothing coordinated but undivided:
        // the new ids join the undetermined list here (no k_iota launch)
        und_appended = dividing && n_divided == n0;
        KLAUNCH(k_round_assign, dim3(div_up(m, 256)), dim3(256), 0, st, t, (int)n0, (int)n1,
                (const int32_t*)k_rs, s_newwit.p, k_rs + 2, und_appended ? d_und.p + n_und : (int32_t*)nullptr);
      }
      // k_witness_bits (new witnesses' see / strongly-see bitsets) and k_round_minw
      // (first witness per round, round count, the candidates' lowest round) in one
      // launch (k_round_tail)
      // the lowest round of the next batch's candidates (the undetermined list and the
      // events the next divide appends), read with the round count (a fresh replay's
      // candidates start at event 0, round 0: nothing to read); an online call's few
      // candidates are reduced by one extra block of k_round_minw
      const int64_t n_mr = n_und + (n1 - n_divided);
      const int mr = tail_fused ? 0
                     : !fresh && n_mr <= 65536 ? (int)std::max<int64_t>(1, std::min<int64_t>(16, div_up(n_mr, 2048)))
                                               : 0;
      if (!tail_fused) {
        int G = 1;
        while (G < std::min(N, 64)) G <<= 1;
        const int64_t wmax = std::min<int64_t>(m, (int64_t)Rcap * N);  // witnesses <= both
        const int nb_wb = std::max(1, std::min(div_up(wmax * NW * G, 256), 8192));
        KLAUNCH(k_round_tail, dim3(nb_wb + div_up(Rcap, 4) + mr), dim3(256), 0, st, t, s_newwit.p, k_rs + 2,
                N > 32 ? (const uint64_t*)d_ssc.p : nullptr, G, nb_wb, (const int32_t*)k_rs, d_minw.p,
                (const int32_t*)coop_err_src, mr, (const int32_t*)d_und.p, (int)n_und, (int)n_divided, (int)n1);
      }
      if (!fresh && !mr && !tail_fused) {
        if (n_und > 0)
          KLAUNCH(k_min_round, dim3(div_up(n_und, 256)), dim3(256), 0, st, d_round.p, d_und.p, (int)n_und,
                  d_minw.p + Rcap + 2);
        if (n1 > n_divided)
          KLAUNCH(k_min_round_range, dim3(div_up(n1 - n_divided, 256)), dim3(256), 0, st, d_round.p,
                  (int)n_divided, (int)n1, d_minw.p + Rcap + 2);
      }
      h_minw.resize(Rcap + 4 + mr);
      d2h(h_minw.data(), d_minw.p, 4 * ((size_t)Rcap + 4 + mr));
      sync();
      minw_full = false;  // every round's first witness is in d_minw now
      if (!fresh) {
        mnr_pre = h_minw[Rcap + 2];
        for (int b = 0; b < mr; b++) mnr_pre = std::min(mnr_pre, h_minw[Rcap + 4 + b]);
      }
      if (coop_err_check && coop_err_src) coop_err = h_minw[Rcap + 3];
      coop_err_src = nullptr;
      mnr_key[0] = fresh ? -1 : n_und;
      mnr_key[1] = n_divided;
      mnr_key[2] = n1;
      if (coop_err_check) {
        coop_err_check = false;
        if (coop_err) {
          // a wide walk's frontier hand-off timed out (its workgroups were not all
          // resident: another grid on the device, e.g. one engine per rank on a
          // shared GPU).  The kernels after it stood down; the engine walks again
          // with k_round_step32, one launch per round, which needs no co-residency,
          // and keeps that walk from here on.  Rows at and past the rounds this
          // batch started from are recomputed from scratch.
          frontier_fallback = true;
          n_frontier_fallbacks++;
          HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(d_C.p + (size_t)R * N), INF32, (size_t)(Rcap - R) * N, st));
          continue;
        }
      }
      if (h_minw[Rcap + 1]) {
        ensure_rcap((int64_t)Rcap * 2);
        continue;
      }
      R = h_minw[Rcap];
      h_minw.resize(R);
      break;
    }
    n_coords = n1;
    coords_len = chain_len;
    fst_fused = false;
    prof_collect();
  }

  // Walkers of the speculative frontier walk (hge_walk_spec.hip) for a fresh
  // state: one per ~192 positions of the shortest chain, up to 32 (HGE_WALKERS
  // overrides; 0 or 1 = the sequential walk).  Short graphs walk sequentially.
  int spec_walkers(int maxlen) {
    const char* ev = getenv("HGE_WALKERS");  // read per call: the tests vary it
    const int env = ev ? atoi(ev) : -1;
    int minlen = INT32_MAX;
    for (int c = 0; c < N; c++) minlen = std::min(minlen, chain_len[c]);
    const int nw = env >= 0 ? env : (minlen >= 4 * 192 ? std::min(32, minlen / 192) : 0);
    return std::max(0, std::min(nw, 64));
  }

  // HGE_WALK_DEBUG: per-walker rows, merge results and cycle stamps on stderr
  DBuf<uint64_t> s_wdbg;
  uint64_t* walk_dbg(int nw) {
    if (!getenv("HGE_WALK_DEBUG")) return nullptr;
    s_wdbg.need(4 * (size_t)nw);
    return s_wdbg.p;
  }
  void walk_debug(int nw) {
    std::vector<int32_t> res(4 * nw + 1), hn(nw);
    std::vector<uint64_t> wd(4 * nw);
    readback(res.data(), s_hres.p, res.size());
    readback(hn.data(), s_hn.p, hn.size());
    readback(wd.data(), s_wdbg.p, wd.size());
    fprintf(stderr, "walk: nw=%d resume=%d |", nw, res[4 * nw]);
    for (int w = 0; w < nw; w++)
      fprintf(stderr, " %d:%d[%d,%d,%d,%d](%llu/%llu/%llu)", w, hn[w], res[4 * w], res[4 * w + 1],
              res[4 * w + 2], res[4 * w + 3], (unsigned long long)wd[4 * w],
              (unsigned long long)wd[4 * w + 1], (unsigned long long)wd[4 * w + 2]);
    fprintf(stderr, "\n");
  }

  // rounds of a wide hashgraph: cooperative frontier kernel (hge_rounds_coop.hip)
  // Speculative walkers of the wide walk (fresh state, N <= 128): as many
  // N-workgroup walkers as stay co-resident, up to 8; HGE_COOP_WALKERS overrides
  // (read per call: the tests vary it; 0 or 1 = the sequential kernel alone).
  int coop_walkers() {
    // walker block size: 512 threads x 2 per CU at N <= 64, 1024 x 1 above (means over
    // seeds 1-3, profiles/r01/specbs: 113.3 vs 106.4M ev/s at 64/1M, 60.8 vs 62.9M at 128/1M)
    const int sbs = N > 64 ? 1024 : COOP_SPEC_BS;
    if (sbs != coop_spec_bs) {
      coop_spec_bs = sbs;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&coop_spec_nb, coop_spec_fn(), sbs, 0));
    }
    const int cap = (int)std::min<int64_t>(16, (int64_t)coop_spec_nb * coop_ncu / N);
    int minlen = INT32_MAX;
    for (int c = 0; c < N; c++) minlen = std::min(minlen, chain_len[c]);
    const char* ev = getenv("HGE_COOP_WALKERS");
    // above N = 128 only 2 walkers fit, and the 512-thread sequential kernel is faster
    // than 2 walkers sharing each CU (22.5 vs 33.6 ms at 256/2M, profiles/r01r_*)
    int nw = ev ? atoi(ev) : (minlen >= 1024 && N <= 128 ? 8 : 0);
    nw = std::min(nw, cap);
    return nw >= 2 ? nw : 0;
  }

  // Launch of a grid whose workgroups hand data to each other (the frontier
  // kernels).  Co-residency is checked once with the occupancy API
  // (coop_checked, coop_walkers); a plain launch of such a grid gets the same
  // residency as a cooperative one (MI355X_MICROARCH.md, Residency), and
  // hipLaunchCooperativeKernel puts the work on a separate device queue whose
  // teardown at process exit crashed under rocprofv3 (profiles/r02_exit_segv.md).
  // Every such launch first checks, for the exact kernel instantiation and block
  // size, that the whole grid fits on the device at once; a grid that cannot be
  // co-resident is refused before anything is written.  The caller holds
  // frontier_lock(): two of these grids on one device (two wide engines driven
  // by different host threads) could each hold part of the CUs and wait on each
  // other's missing workgroups, so one process runs them one at a time.  (Grids of
  // other processes on the same device are not covered: wide engines need the
  // device to themselves)
  std::vector<std::pair<std::pair<const void*, int>, int>> resident_nb;
  hipError_t launch_resident(const void* fn, dim3 grid, dim3 block, void** args) {
    const int bs = (int)(block.x * block.y * block.z);
    int nb = -1;
    for (auto& e : resident_nb)
      if (e.first.first == fn && e.first.second == bs) nb = e.second;
    if (nb < 0) {
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, bs, 0));
      resident_nb.push_back({{fn, bs}, nb});
    }
    const int64_t blocks = (int64_t)grid.x * grid.y * grid.z;
    if ((int64_t)nb * n_cu() < blocks)
      throw EngineError(HGE_ERR_DEVICE, "frontier grid of " + std::to_string(blocks) + " workgroups x " +
                                            std::to_string(bs) + " threads cannot be co-resident (" +
                                            std::to_string(nb) + " per CU x " + std::to_string(n_cu()) + " CUs)");
    return hipLaunchKernel(fn, grid, block, args, 0, st);
  }
  static std::mutex& frontier_mutex(int dev) {
    static std::mutex m[64];
    return m[dev & 63];
  }
  std::unique_lock<std::mutex> frontier_lock() { return std::unique_lock<std::mutex>(frontier_mutex(device)); }

  // Wide rounds step: strongly-see tiles on the coordinate rows
  // (hge_rounds_direct.hip) for N % 4 == 0, else the FDT-gather selection of
  // hge_rounds_coop.hip.
  bool direct_rounds() const { return (N & 3) == 0; }


  // rounds of a wide hashgraph: cooperative frontier kernel (hge_rounds_coop.hip)
  // (the caller holds frontier_lock() until the stream has drained)
  int32_t coop_err = 0;
  bool coop_err_check = false;
  const int32_t* coop_err_src = nullptr;  // the walk's error flag on the device (read with minw)
  bool frontier_fallback = false;  // k_round_step32 for good after a hand-off timeout
  int64_t n_frontier_fallbacks = 0;
  void rounds_coop(bool fresh) {
    Tables t = tables();
    s_fst.need(N + 1);
    // (the hand-off flags and granules are zeroed by k_frontier_start)
    s_bar.need(2);
    s_gran.need(2 * (size_t)N);
    if (!fst_fused || fresh)  // (else the chain fill's last block ran it)
      KLAUNCH(k_frontier_start, dim3(1), dim3(256), 0, st, t, k_len, k_len + N, s_fst.p, (int32_t*)nullptr,
              s_bar.p, (uint64_t*)s_gran.p, 2 * N);
    fst_fused = false;
    // the lowest round to recompute: read back for a fresh state (the walkers and the
    // joined rows need it on the host), else read by the frontier kernel itself,
    // which stands down at INF32 (no round trip)
    int32_t rlo = 0;
    const int32_t* rlo_dev = nullptr;
    if (fresh) {
      rlo = INF32;
      readback(&rlo, s_fst.p, 1);
      if (rlo == INF32) return;
    } else {
      rlo_dev = s_fst.p;
    }
    int Rprev = R;
    if (!coop_checked) {
      int nb = 0, ncu = 0, coop = 0;
      HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_rounds_coop, COOP_BS, 0));
      HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
      HIPCHK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, device));
      if (!coop || (int64_t)nb * ncu < N) {  // a device too small for the walk's grid
        frontier_fallback = true;
        rounds_step32();
        return;
      }
      coop_nb = nb;
      coop_ncu = ncu;
      coop_checked = true;
    }
    int maxlen = 0;
    for (int c = 0; c < N; c++) maxlen = std::max(maxlen, chain_len[c]);
    // admission switches the engine to int32 positions (to_wide32) before a chain
    // passes 65,534 events, so this packed walk never sees one; the check guards it
    if (maxlen >= 0xFFFF)
      throw EngineError(HGE_ERR_INTERNAL, "packed rounds walk reached a chain past 65,534 events");
    const int32_t* FDT = d_FDT.p;
    const int32_t* olen = k_len;
    const int32_t* len = k_len + N;
    int32_t* rstate = k_rs;
    int32_t* err = s_bar.p + 1;
    if (ext_on && fresh && rlo == 0 && Rprev == 0) {
      // frontier rows joined from the walkers of all ranks (babble_amd/dist.py)
      const int K = ext_rows;  // true rows 0 .. K-1
      if (K + 1 >= Rcap) {  // the rounds table must hold them: overflow, grow, come back
        int32_t ov[2] = {0, 1};
        h2d(rstate, ov, 8);
        return;
      }
      ext_on = false;
      h2d(d_C.p, ext_C.data(), sizeof(int32_t) * (size_t)K * N);
      if (K > 1) h2d(d_ssc.p + (size_t)N * NW, ext_ssc.data() + (size_t)N * NW, sizeof(uint64_t) * (size_t)(K - 1) * N * NW);
      if (ext_natural) {  // the walk ended: row K is the empty frontier
        int32_t rs0 = K;
        h2d(rstate, &rs0, 4);
        return;
      }
      rlo = K - 1;  // the sequential walk resumes from the last true row
    }
    const int nw = (fresh && rlo == 0 && Rprev == 0) ? coop_walkers() : 0;
    if (nw >= 2) {
      const char* hc = getenv("HGE_WALK_HCAP");  // tests: force the capacity fallback
      const int Hcap = hc ? std::max(2, std::min(0xFFFF, atoi(hc)))
                          : std::min(0xFFFF, std::min(Rcap, std::max(256, 3 * (Rcap / nw) + 256)));
      int TS = 64;
      while (TS < 2 * Hcap) TS <<= 1;
      const size_t nh = (size_t)nw * Hcap * N, nt = (size_t)nw * TS;
      const size_t hn0 = s_cH.n, tn0 = s_cT.n;  // a new allocation holds arbitrary words
      s_cH.need(nh);
      s_cT.need(nt);
      bool clear = s_cH.n != hn0 || s_cT.n != tn0;
      if (++coop_epoch >= 0x7FFFFFFFu) {  // tags wrap: clear, restart at 1
        coop_epoch = 1;
        clear = true;
      }
      if (clear) {
        HIPCHK(hipMemsetAsync(s_cH.p, 0, s_cH.n * sizeof(uint64_t), st));
        HIPCHK(hipMemsetAsync(s_cT.p, 0, s_cT.n * sizeof(uint64_t), st));
      }
      s_cS.need(nh * NW);
      s_cM.need(nw);
      s_cn.need(2 * (size_t)nw + 1);
      HIPCHK(hipMemsetAsync(s_cM.p, 0xFF, (size_t)nw * sizeof(uint64_t), st));
      int64_t nev = 0;
      for (int c = 0; c < N; c++) nev += chain_len[c];
      // guesses (measured over seeds 1-3, profiles/r01/guess128): time cuts at N <= 64,
      // alternating length/time cuts above
      const int guess = N <= 64 ? 1 : 2;
      CoopSpec cs{s_cH.p, s_cS.p, s_cT.p, (unsigned long long*)s_cM.p, s_cn.p, nw, Hcap, TS,
                  coop_epoch, nev, guess};
      void* sargs[] = {&t, &FDT, &olen, &len, &cs, &err};
      prof_begin("k_rounds_coop_spec");
      HIPCHK(launch_resident(coop_spec_fn(), dim3(nw * N), dim3(coop_spec_bs), sargs));
      prof_end();
      int32_t* resume = s_cn.p + 2 * nw;
      KLAUNCH(k_coop_join, dim3(64), dim3(256), 0, st, t, cs, d_ssc.p, rstate, resume);
      int32_t hres[2] = {0, 0};
      readback(&hres[0], err, 1);
      if (hres[0]) {  // co-residency failure: coords_b falls back to k_round_step32
        const int32_t down[2] = {Rprev, 4};
        h2d(rstate, down, 8);
        coop_err = 1;
        coop_err_check = true;
        coop_err_src = nullptr;
        return;
      }
      readback(&hres[1], resume, 1);
      if (getenv("HGE_WALK_DEBUG")) {
        std::vector<int32_t> hn(2 * nw);
        std::vector<uint64_t> mg(nw);
        readback(hn.data(), s_cn.p, hn.size());
        readback(mg.data(), s_cM.p, mg.size());
        fprintf(stderr, "coop walk: nw=%d Hcap=%d resume=%d |", nw, Hcap, hres[1]);
        for (int w = 0; w < nw; w++)
          fprintf(stderr, " %d:%d%s->(%d,w%d:%d)", w, hn[w], hn[nw + w] ? "e" : "",
                  mg[w] == ~0ull ? -1 : (int)(mg[w] >> 32),
                  mg[w] == ~0ull ? -1 : w + (int)((mg[w] >> 16) & 0xFFFF), (int)(mg[w] & 0xFFFF));
        fprintf(stderr, "\n");
      }
      if (hres[1] < 0) return;
      rlo = hres[1];
    }
    uint64_t* gran = s_gran.p;
    uint64_t* ssc = d_ssc.p;
    uint64_t* dbg = dbg_p();
    if (direct_rounds()) {
      // strongly-see tiles on the coordinate rows (hge_rounds_direct.hip)
      const int npow = N <= 64 ? 64 : N <= 128 ? 128 : 256;
      s_mb.need((size_t)npow * npow);  // two parity blocks of npow rows x npow/2 packed words
      uint32_t* mb = s_mb.p;
      const int32_t* nostart = nullptr;
      int32_t* nohist = nullptr;
      int hmax = 0, extra = 0;
      // tests: the walk stalls at this hand-off epoch (chain 0 never publishes it)
      const char* hs = getenv("HGE_TEST_HANDOFF_STALL");
      int stall_ep = hs ? atoi(hs) : 0;
      void* dargs[] = {&t, &olen, &len, &rstate, &rlo, &rlo_dev, &Rprev, &gran, &err, &ssc, &mb, &dbg,
                       &nostart, &nohist, &hmax, &nostart, &extra, &stall_ep};
      const void* fn = N <= 64 ? (const void*)k_rounds_direct<1024, 64>
                     : N <= 128 ? (const void*)k_rounds_direct<1024, 128>
                                : (const void*)k_rounds_direct<1024, 256>;
      prof_begin("k_rounds_direct");
      HIPCHK(launch_resident(fn, dim3(N), dim3(1024), dargs));
      prof_end();
    } else {
      void* args[] = {&t, &FDT, &olen, &len, &rstate, &rlo, &rlo_dev, &Rprev, &gran, &err, &ssc, &dbg};
      prof_begin("k_rounds_coop");
      HIPCHK(launch_resident((const void*)k_rounds_coop, dim3(N), dim3(COOP_BS), args));
      prof_end();
    }
    if (getenv("HGE_TEST_HANDOFF_FAIL")) {  // tests: the walk reports a hand-off timeout
      const int32_t one = 1, down = 4;
      h2d(err, &one, 4);
      h2d(rstate + 1, &down, 4);
    }
    // the hand-off error flag comes back with the round count (coords_b, k_round_minw)
    coop_err_src = s_bar.p + 1;
    coop_err_check = true;
    dbg_dump();
  }

  // N > 32: lastAncestors live in the packed 16-bit table while every chain holds at
  // most 65,534 events; a longer chain switches the engine to int32 LA rows for good
  // (to_wide32 below), which the N <= 32 path uses from the start
  bool sweep16() const { return N > 32 && !wide32; }
  // the median's threshold rows as uint16 (k_witness_la, k_median_wave's 4-witness lanes)
  bool wla16() const { return N > 192 && (N & 3) == 0 && !wide32; }

  // the switch to int32 positions (hge_wide32.hip): the int32 LA rows of every event
  // with coordinates, unpacked from LA16; from here on the N <= 32 sweeps and
  // transposes, k_round_step32 and k_seg_theta32 take the wide path's place
  // Runs at the next coordinate step after admission lifted the cap.  The pending
  // flag is cleared only once the int32 tables exist: a failed allocation leaves the
  // engine refusing every later step (the packed tables can no longer hold the
  // positions) instead of packing positions past 65,534 into uint16.
  // A retry after a failed allocation resumes where the last attempt stopped: the int32
  // LA table comes first (nothing is converted before it exists), and each uint16 table
  // widened is marked in w32_done, so a retry never reads a widened table as uint16.
  void to_wide32() {
    auto test_stop = [&](int stage) {  // HGE_TEST_W32_FAIL=stage: one failure after that stage
      if (test_w32_fail == stage) {
        test_w32_fail = 0;
        throw EngineError(HGE_ERR_DEVICE, "test: to_wide32 stopped after stage " + std::to_string(stage));
      }
    };
    if (!(w32_done & 4)) {
      grow_chain_table(d_LA, ccap, false);
      w32_done |= 4;
      test_stop(1);
    }
    if (fdt16()) {  // the runs and FD rows continue in int32 from here: widen the kept ones
      const size_t n = (size_t)N * N * ccap;
      for (int which = 0; which < 2; which++) {
        if (w32_done & (1 << which)) continue;
        DBuf<int32_t>& b = which ? d_FD : d_FDT;
        int32_t* q = nullptr;
        HIPCHK(hipMalloc(&q, sizeof(int32_t) * n));
        KLAUNCH(k_fdt16_to32, dim3((unsigned)std::min<size_t>(div_up(n, 256), 65536)), dim3(256), 0, st,
                (const uint16_t*)b.p, q, n, which);
        sync();
        b.free_();
        b.p = q;
        b.n = n;
        w32_done |= 1 << which;
        test_stop(2 + which);
      }
    }
    s_w32.need(N);
    h2d(s_w32.p, coords_len.data(), 4 * (size_t)N);
    wide32 = true;
    wide32_pending = false;
    w32_done = 0;
    Tables t = tables();
    int64_t most = 1;
    for (int c = 0; c < N; c++) most = std::max<int64_t>(most, (int64_t)coords_len[c] * N);
    KLAUNCH(k_la16_to_la32, dim3((unsigned)std::min<int64_t>(div_up(most, 256), 4096), N), dim3(256), 0, st, t,
            (const uint32_t*)d_LA16.p, (const int32_t*)s_w32.p);
  }

  // rounds with int32 positions: k_round_step32 round by round from the first round
  // to recompute, 32 launches between readbacks of their "row exists" flags
  void rounds_step32() {
    Tables t = tables();
    s_fst.need(N + 1);
    KLAUNCH(k_frontier_start, dim3(1), dim3(256), 0, st, t, k_len, k_len + N, s_fst.p, (int32_t*)nullptr,
            (int32_t*)nullptr, (uint64_t*)nullptr, 0);
    int32_t rlo = INF32;
    readback(&rlo, s_fst.p, 1);
    if (rlo == INF32) return;
    const int Rprev = R, NB = 32;
    s_w32a.need(NB);
    for (int r = rlo;;) {
      HIPCHK(hipMemsetAsync(s_w32a.p, 0, 4 * NB, st));
      int k = 0;
      for (; k < NB && r + k + 1 < Rcap; k++)
        KLAUNCH(k_round_step32, dim3(N), dim3(256), 0, st, t, (const int32_t*)k_len, (const int32_t*)(k_len + N),
                r + k, Rprev, d_ssc.p, s_w32a.p + k);
      std::vector<int32_t> alive(NB, 0);
      readback(alive.data(), s_w32a.p, NB);
      for (int q = 0; q < k; q++)
        if (!alive[q]) {  // row r + q + 1 is empty: the rounds end there
          const int32_t rs[2] = {std::max(R, r + q + 1), 0};
          h2d(k_rs, rs, 8);
          return;
        }
      r += k;
      if (k < NB) {  // the rounds table is full: grown by the caller, walked again
        const int32_t rs[2] = {R, 1};
        h2d(k_rs, rs, 8);
        return;
      }
    }
  }

  // N > 128, N % 4 == 0, uint16 positions: the FDT runs as uint16 (k_la16_rows_runs<uint16_t>,
  // k_fd_transpose_ts<uint16_t>: half the run table's bytes written and read).  Neither the
  // direct walk nor theta reads FDT; the speculative walkers (N <= 128) and the
  // FDT-gather walk (N % 4 != 0) read int32 runs.
  bool fdt16() const { return N > 128 && (N & 3) == 0 && !wide32; }

  // 32 < N <= 256: lastAncestors by windowed exact propagation (hge_coords_win.hip)
  // instead of the sweeps
  bool la_windows() const { return N > 32 && N <= 256 && !wide32; }

  // passes over windows of the new ids until one changes no row (n_sweeps = passes
  // run); one window is exact in its first pass (its starting rows are final)
  void la_windows_run(Tables t) {
    const int32_t* olen = k_len;
    const int32_t* len = k_len + N;
    const int64_t n0 = n_coords, n1 = n_events, ne = n1 - n0;
    const int npow = N <= 64 ? 64 : N <= 128 ? 128 : 256;
    // k_la_win: one 1024-thread workgroup per window (a barrier-free wave-per-slice
    // variant measured 2x slower: DESIGN.md §4.1)
    const int W = t.NW2;
    const int64_t WMIN = 4096;  // ids per window at least
    const int per_cu = npow == 256 ? 1 : 2;
    int64_t G = std::min<int64_t>((int64_t)n_cu() * per_cu, std::max<int64_t>(1, ne / WMIN));
    if (const char* g = getenv("HGE_LW_G")) G = std::max(1, atoi(g));
    int64_t WN = (div_up(ne, G) + LW_K - 1) / LW_K * LW_K;
    G = div_up(ne, WN);
    s_lwplan.need(ne);
    s_lwsum.need(ne);
    s_lwinit.need((size_t)G * N * W);
    s_lwpos.need((size_t)G * N);
    s_lwrisky.need(G);
    const int MAXP = 64;
    s_chg.need(MAXP);
    // one window (an online call): its chain start positions are the chains' old
    // lengths and its risky id starts at -1 in the control block, so k_lw_pos is not
    // needed (one launch less per call)
    const int32_t* wpos = G == 1 ? olen : s_lwpos.p;
    int32_t* risky = G == 1 ? k_risky1 : s_lwrisky.p;
    if (G > 1)
      KLAUNCH(k_lw_pos, dim3(div_up(std::max<int64_t>(G * N, MAXP), 256)), dim3(256), 0, st, t, n0, (int)WN, (int)G,
              len, s_lwpos.p, s_lwrisky.p, s_chg.p, MAXP);
    // one window: its workgroup plans its own chunks (k_la_win's plan_len)
    if (G > 1)
      KLAUNCH(k_lw_plan, dim3(div_up(div_up(ne, LW_K), 4)), dim3(256), 0, st, t, n0, n1, (int)WN, len, s_lwplan.p,
              risky);
    int p = 0;
    for (int group = G == 1 ? 1 : 3;; group = 2) {
      for (int g = 0; g < group; g++, p++) {
        if (p >= MAXP) throw EngineError(HGE_ERR_INTERNAL, "lastAncestors windows did not converge");
        const int32_t* prev = p > 0 ? s_chg.p + p - 1 : nullptr;
        const int pass = p + 1;
#define LWIN(NP)                                                                                         \
  KLAUNCH(k_la_win<NP>, dim3(G), dim3(1024), 0, st, t, s_lwplan.p, n0, n1, (int)WN, wpos, olen,          \
          s_lwinit.p, risky, s_lwsum.p, pass, prev, s_chg.p + p,                                        \
          G == 1 && p == 0 ? len : (const int32_t*)nullptr)
        if (npow == 64) LWIN(64);
        else if (npow == 128) LWIN(128);
        else LWIN(256);
#undef LWIN
      }
      if (G == 1) {
        n_sweeps = 1;
        break;
      }
      std::vector<int32_t> flags(p);
      readback(flags.data(), s_chg.p, p);
      if (!flags[p - 1]) {
        n_sweeps = (int)(std::find(flags.begin(), flags.end(), 0) - flags.begin()) + 1;
        break;
      }
    }
  }

  // coordinates: chain-prefix sweeps + transposes (hge_coords.hip)
  // the one-pass lastAncestors kernel (k_la_seq) takes batches of m new events at N <= 32
  bool la_seq_ok(int64_t m) const {
    return !sweep16() && N <= 32 && m > 0 && m * (N <= 16 ? 16 : 32) <= LASEQ_MAX && !getenv("HGE_NO_LASEQ");
  }
  const UpEv* fill_up = nullptr;  // coords_a -> the chain-table fill (packed upload or the tables)
  UpDst fill_dst{};
  void coords_sweep(Tables t, int nseg, int SEG, int maxnew, bool fresh) {
    const int32_t* olen = k_len;
    const int32_t* len = k_len + N;
    if (nseg == 0) return;
    // sweeps until one changes nothing; queued in groups, checked once per group
    // (a sweep after a quiet one returns at once); k_la_clear zeroes the flags
    const int MAXSW = 4096;
    s_chg.need(MAXSW);
    const bool p16 = sweep16();
    // skip segments whose inputs did not change in the previous sweep
    const bool SKIP = true;
    const int64_t mnew = n_events - n_coords;
    if (p16 && la_windows()) {
      la_windows_run(t);
    } else if (la_seq_ok(mnew)) {
      // a small batch (an online call): one exact pass in insertion order, the chain
      // table filled by the same kernel
      // (+ k_fd_qlo's N blocks past a fresh state: coords_b skips its launch)
      const bool q = !fresh;
      // (+ k_frontier_start's block when coords_b walks as an online call)
      int maxlen = 0;
      for (int c = 0; c < N; c++) maxlen = std::max(maxlen, chain_len[c]);
      fst_fused = q && maxlen < 0xFFFF;
      if (fst_fused) s_fst.need(N + 1);
      int32_t* fp = fst_fused ? s_fst.p : (int32_t*)nullptr;
      int32_t* fl = fst_fused ? k_lo : (int32_t*)nullptr;
      // N <= 16 past a fresh state: the batch's firstDescendants in the same launch (no
      // runs, transpose or k_fd_qlo blocks)
      fd_direct = q && N <= 16 && !getenv("HGE_NO_FD_DIRECT");
      const int nq = q && !fd_direct ? N : 0;
      const int nb = 1 + nq + (fst_fused ? 1 : 0);
      if (N <= 16)
        KLAUNCH(k_la_seq<16>, dim3(nb), dim3(256), 0, st, t, (int)n_coords, (int)n_events, fill_up,
                fill_dst, olen, len, nq ? k_qlo : (int32_t*)nullptr, fp, fl,
                fd_direct ? d_FDT.p : (int32_t*)nullptr);
      else
        KLAUNCH(k_la_seq<32>, dim3(nb), dim3(256), 0, st, t, (int)n_coords, (int)n_events, fill_up,
                fill_dst, olen, len, nq ? k_qlo : (int32_t*)nullptr, fp, fl, (int32_t*)nullptr);
      qlo_fused = q;
      n_sweeps = 1;
    } else {
    int32_t* dirty = nullptr;
    if (p16 && SKIP) {
      s_dirty.need(nseg);
      dirty = s_dirty.p;
    }
    if (p16)
      KLAUNCH(k_la_clear16, dim3(std::max(1, std::min(64, div_up((int64_t)maxnew * t.NW2, 256))), N),
              dim3(256), 0, st, t, olen, len, s_chg.p, MAXSW, dirty, nseg);
    else
      KLAUNCH(k_la_clear, dim3(std::max(1, std::min(64, div_up((int64_t)maxnew * N, 256))), N),
              dim3(256), 0, st, t, olen, len, s_chg.p, MAXSW);
    const int NPt = p16 ? (t.NW2 <= 32 ? 32 : t.NW2 <= 64 ? 64 : 128)
                        : (N <= 16 ? 16 : N <= 32 ? 32 : N <= 64 ? 64 : N <= 128 ? 128 : 256);
    int sw = 0;
    for (int group = 12;; group = 8) {
      for (int g = 0; g < group; g++, sw++) {
        if (sw >= MAXSW) throw EngineError(HGE_ERR_INTERNAL, "lastAncestors sweeps did not converge");
        const int32_t* prev = sw > 0 ? s_chg.p + sw - 1 : nullptr;
        if (p16) {
          switch (NPt) {
#define SW16(NPV)                                                                                \
  case NPV:                                                                                      \
    KLAUNCH(k_la_sweep16<NPV>, dim3(div_up(nseg, 256 / NPV)), dim3(256), 0, st, t, k_segs, nseg, \
            SEG, len, prev, s_chg.p + sw, olen, k_segbase, dirty, sw);                          \
    break;
            SW16(32)
            SW16(64)
            SW16(128)
#undef SW16
          }
        } else {
          switch (NPt) {
#define SW(NPV)                                                                                  \
  case NPV:                                                                                      \
    KLAUNCH(k_la_sweep<NPV>, dim3(div_up(nseg, 256 / NPV)), dim3(256), 0, st, t, k_segs, nseg,   \
            SEG, len, prev, s_chg.p + sw);                                                       \
    break;
            SW(16)
            SW(32)
            SW(64)
            SW(128)
            SW(256)
#undef SW
          }
        }
      }
      std::vector<int32_t> flags(sw);
      readback(flags.data(), s_chg.p, sw);
      if (!flags[sw - 1]) {
        // sweeps that did work: up to and including the first one that changed nothing
        n_sweeps = (int)(std::find(flags.begin(), flags.end(), 0) - flags.begin()) + 1;
        break;
      }
    }
    }
    if (fd_direct) {
      fd_direct = false;  // (k_la_seq wrote the FD rows and FDT runs)
      qlo_fused = false;
      return;
    }
    if (fdt16()) {
      KLAUNCH((k_la16_rows_runs<uint16_t>), dim3(div_up(maxnew + 1, 64), div_up(N, 64), N), dim3(256), 0, st, t,
              (uint16_t*)d_FDT.p, k_plo, olen, len);
    } else if (p16) {
      // LA16 -> the int32 LA rows and the FDT runs from the same tiles (no LAT)
      KLAUNCH((k_la16_rows_runs<int32_t>), dim3(div_up(maxnew + 1, 64), div_up(N, 64), N), dim3(256), 0, st, t,
              d_FDT.p, k_plo, olen, len);
    } else {
      // the int32 LA rows -> the runs of the new events (and the new positions with no
      // descendant yet) through 64 x 64 LDS tiles (one launch; round 3's LA -> LAT
      // transpose + k_fdt_runs took two and the LAT table)
      KLAUNCH((k_la16_rows_runs<int32_t, true>), dim3(div_up(maxnew + 1, 64), div_up(N, 64), N), dim3(256), 0,
              st, t, d_FDT.p, k_plo, olen, len);
    }
    // FDT -> FD rows for every chain-c position a new event can have touched
    // (from a fresh state: every row, qlo = 0 as uploaded; no round trip)
    // (the rows' lower bounds stay on the device: the transposes loop over position
    // tiles past their grid, sized here for the new positions plus a tile)
    int span = 1;
    if (!fresh) {
      if (!qlo_fused) KLAUNCH(k_fd_qlo, dim3(N), dim3(256), 0, st, t, olen, len, k_qlo);
      qlo_fused = false;
      span = maxnew + 64;
    } else {
      for (int c = 0; c < N; c++) span = std::max(span, chain_len[c]);
    }
    // (a split part writes the timestamp rows of its own candidates only)
    if (fdt16())
      KLAUNCH((k_fd_transpose_ts<uint16_t>), dim3(N, div_up(N, 64), std::min(div_up(span, 64), 65535)), dim3(256),
              0, st, t, (const uint16_t*)d_FDT.p, k_qlo, len, (const int32_t*)k_fd,
              (const int32_t*)(k_fd ? k_fd + N : nullptr));
    else if (N > 16)
      KLAUNCH((k_fd_transpose_ts<int32_t>), dim3(N, div_up(N, 64), std::min(div_up(span, 64), 65535)), dim3(256),
              0, st, t, (const int32_t*)d_FDT.p, k_qlo, len, (const int32_t*)k_fd,
              (const int32_t*)(k_fd ? k_fd + N : nullptr));
    else
      KLAUNCH(k_transpose, dim3(div_up(span, 64), div_up(N, 64), N), dim3(256), 0, st, t, d_FDT.p,
              (int32_t*)nullptr, k_qlo, len, 1);
  }

  // ---------------- one batch of consensus calls ----------------
  // calls: event counts n_c (<= n_divided), ascending.
  // Host round trips: the fame-window coverage flags, the lowest candidate round
  // of an online batch, the segment count for N > 64, and one closing readback.
  // Control data goes up as one block (s_cctl), results come back as one block
  // (s_out: counters, per-call counts, order).
  void consensus_batch(const std::vector<int64_t>& calls, bool do_fame, bool do_order,
                       bool commit, std::vector<int32_t>* order_out,
                       std::vector<int64_t>* counts_out) {
    const int ncalls = (int)calls.size();
    if (ncalls == 0) return;
    const bool tph = ncalls > 1000 && getenv("HGE_HOST_PHASES");
    int64_t tp[6] = {now_ns(), 0, 0, 0, 0, 0};
    consensus_sync();  // (the results block is reused below)
    Tables t = tables();
    x_iter = 0;
    // R_c = Rounds() after the DivideRounds of call c = #{r : minw[r] < n_c}
    // (one merge pass over the ascending calls and first witnesses: 39k binary searches
    // were ~0.5 ms of idle GPU at the start of a 256/10M replay's consensus)
    std::vector<int32_t> Rc(ncalls);
    for (int c = 0, r = 0; c < ncalls; c++) {
      if (c > 0 && calls[c] < calls[c - 1])  // (not ascending: search afresh)
        r = (int)(std::lower_bound(h_minw.begin(), h_minw.end(), calls[c],
                                   [](int32_t m, int64_t n) { return (int64_t)m < n; }) -
                  h_minw.begin());
      while (r < (int)h_minw.size() && (int64_t)h_minw[r] < calls[c]) r++;
      Rc[c] = r;
    }
    const bool fresh_und = und_fresh;
    und_fresh = false;
    const bool ord = do_order && n_und > 0;
    int ncand = (int)n_und;
    int32_t* cand = d_und.p;
    // a split part's candidates: the events [cand_lo, its end) of the fresh list (identity)
    const bool spl = split_on() && ord && fresh_und;
    if (spl) {
      cand = d_und.p + sp.clo[sp.part];
      ncand = (int)(sp.a[sp.part + 1] - sp.clo[sp.part]);
    }
    // lowest candidate round (a fresh replay's candidates include event 0, round 0)
    int32_t mnr = 0;
    const bool pre = mnr_key[0] >= 0 && !spl && n_divided == mnr_key[2] &&
                     n_und == mnr_key[0] + (mnr_key[2] - mnr_key[1]);
    mnr_key[0] = -1;
    if (ord && !fresh_und && pre) {
      mnr = mnr_pre;
    } else if (ord && (!fresh_und || spl)) {
      h2d(s_small.p + 7, &kInf, 4);
      KLAUNCH(k_min_round, dim3(div_up(ncand, 256)), dim3(256), 0, st, d_round.p, cand, ncand,
              s_small.p + 7);
      readback(&mnr, s_small.p + 7, 1);
    }
    const int rr_lo = mnr + 1;
    // a split part's calls end at its last one: later rounds receive nothing it commits
    const int R_last = spl ? Rc[sp.cb[sp.part + 1] - 1] : Rc[ncalls - 1];
    const int nr = ord ? std::max(0, R_last - rr_lo) : 0;

    // the results block's size (counters | per-call counts | order | per-block transaction
    // sums), known before DecideFame: the single-call fame kernel writes its header
    const size_t o_tx0 = (8 + (size_t)ncalls + (ord ? ncand : 0) + 1) & ~(size_t)1;
    const int ntxb0 = ord ? div_up(ncand, 256) : 0;
    bool hdr_done = false;
    bool ocall = false;  // the order's stages ran as one launch (k_order_call)
    bool fame_deferred = false;  // N <= 16: k_fame_call waits to run with the order (k_consensus_call)
    FameCall fc_pend{};
    auto fame_call_args = [&](int nrounds_, int npairs_, int ncalls_, int32_t* hdr) {
      FameCall f{};
      f.pr_round = c_pr;
      f.pr_off = c_pr + nrounds_;
      f.pr_cf = c_pr + 2 * nrounds_;
      f.pr_len = c_pr + 3 * nrounds_;
      f.nrounds = nrounds_;
      f.npairs = npairs_;
      f.nc = c_nc;
      f.Rc = c_Rc;
      f.dec = s_dec.p;
      f.decbit = s_decbit.p;
      f.Lc = c_Lc;
      f.ncalls = ncalls_;
      f.lcr_start = lcr;
      f.LCR = s_LCR.p;
      f.clast = s_clast.p;
      f.flags = c_flags;
      f.out = hdr;
      f.nout = 8 + ncalls_;
      return f;
    };
    bool otail = false;  // the order's stages from the call's bucket on ran as one launch
    tp[1] = now_ns();
    // ---- DecideFame windows (host enumeration of (round, call) pairs) + control block ----
    std::vector<int32_t> pr_round, pr_off, pr_cf, pr_len;
    int npairs = 0, nrounds = 0;
    int64_t nslot = 0;
    int lcr_new = lcr, c_set = -1;
    // every round's window reaching the last call (always so for one call: the
    // online path) cannot widen: the coverage flags stay on the device, and the new
    // LastConsensusRound comes back with the batch's closing readback
    bool lcr_dev = false;
    const int i_lo = lcr + 1;
    const int i_hi = Rc[ncalls - 1] - 2;  // processed rounds: i <= R_c - 2
    // speculative fame window: calls up to R_c <= i + 2 + SPEC, widened when a round
    // stays undecided past it (narrower windows re-dispatch more often: slower)
    // Selective widening (N >= 192 a multiple of 64, no split or record; smaller N pay
    // more for the passes' round trips than the fame work they save): every window starts
    // at SPEC = 1 and only the rounds whose decision came past their window are
    // widened and re-decided (their new pairs alone; the other rounds' decisions are
    // moved to the new layout).  At 256/10M 517 of 2,836 rounds go to SPEC = 2 and 6
    // of those to 4; a uniform SPEC = 3 decides twice the pairs.
    const bool selective = do_fame && N % 64 == 0 && N >= 192 && !split_on() && !rec_on && ncalls > 1;
    std::vector<int> spec_r;
    std::vector<int32_t> old_off, old_len;
    for (int SPEC = selective ? 1 : 3, iter = 0;; SPEC *= 2, iter++) {
      pr_round.clear();
      pr_off.clear();
      pr_cf.clear();
      pr_len.clear();
      npairs = 0;
      if (do_fame) {
        int cfp = 0;
        for (int i = i_lo; i <= i_hi; i++) {
          while (cfp < ncalls && Rc[cfp] < i + 2) cfp++;
          if (cfp >= ncalls) break;
          const int k = (int)pr_round.size();
          if (selective && iter == 0) spec_r.push_back(SPEC);
          const int sp = selective ? spec_r.at(k) : SPEC;
          // last call with R_c <= i + 2 + SPEC
          int a = cfp, b = ncalls - 1;
          while (a < b) {
            int mid = (a + b + 1) / 2;
            if (Rc[mid] <= i + 2 + sp) a = mid;
            else b = mid - 1;
          }
          pr_round.push_back(i);
          pr_off.push_back(npairs);
          pr_cf.push_back(cfp);
          pr_len.push_back(a - cfp + 1);
          npairs += a - cfp + 1;
        }
      }
      nrounds = (int)pr_round.size();
      // control block: n_c (int64), R_c, L_c = -1, flags, the four window arrays,
      // the round -> window map of the order pass
      const size_t o_Rc = 2 * (size_t)ncalls, o_Lc = o_Rc + ncalls, o_fl = o_Lc + ncalls;
      const size_t o_pr = o_fl + 4, o_pidx = o_pr + 4 * (size_t)nrounds;
      const size_t o_sgo = o_pidx + nr;  // N <= 64: per-round segment capacity offsets
      std::vector<int32_t>& cc = h_cctl;
      // a widening pass keeps the calls, R_c and their offsets (the round set is the
      // same): only the window arrays are rewritten and uploaded, L_c and the flags are
      // reset on the device (k_dec_relayout)
      const bool part = selective && iter > 0;
      if (!part) {
        cc.assign(o_sgo + nr + 1, 0);
        memcpy(cc.data(), calls.data(), 8 * (size_t)ncalls);
        memcpy(&cc[o_Rc], Rc.data(), 4 * (size_t)ncalls);
        std::fill(cc.begin() + o_Lc, cc.begin() + o_fl, -1);
      }
      if (nrounds) {
        memcpy(&cc[o_pr], pr_round.data(), 4 * (size_t)nrounds);
        memcpy(&cc[o_pr + nrounds], pr_off.data(), 4 * (size_t)nrounds);
        memcpy(&cc[o_pr + 2 * nrounds], pr_cf.data(), 4 * (size_t)nrounds);
        memcpy(&cc[o_pr + 3 * nrounds], pr_len.data(), 4 * (size_t)nrounds);
      }
      for (int q = 0; q < nr; q++) cc[o_pidx + q] = -1;
      for (int k = 0; k < nrounds; k++) {
        const int i = pr_round[k];
        if (i >= rr_lo && i < rr_lo + nr) cc[o_pidx + (i - rr_lo)] = k;
      }
      // a round's segments start at call 0, at a witness arrival (<= N distinct
      // calls), at the window start or at a processed call of its fame window
      nslot = 0;
      for (int q = 0; q < nr; q++) {
        cc[o_sgo + q] = (int32_t)nslot;
        const int k = cc[o_pidx + q];
        nslot += N + 2 + (k >= 0 ? pr_len[k] : 0);
      }
      cc[o_sgo + nr] = (int32_t)std::min<int64_t>(nslot, INF32);
      if (part) {
        h2d(s_cctl.p + o_pr, cc.data() + o_pr, 4 * (cc.size() - o_pr));
      } else {
        s_cctl.need(cc.size());
        h2d(s_cctl.p, cc.data(), 4 * cc.size());
      }
      c_nc = (int64_t*)s_cctl.p;
      c_Rc = s_cctl.p + o_Rc;
      c_Lc = s_cctl.p + o_Lc;
      c_flags = s_cctl.p + o_fl;
      c_pr = s_cctl.p + o_pr;
      c_pidx = s_cctl.p + o_pidx;
      c_sgo = s_cctl.p + o_sgo;
      if (nrounds == 0) break;
      if (!(selective && iter > 0)) s_dec.need((size_t)npairs * N);  // (a widening moves them first)
      s_decbit.need(npairs);
      s_LCR.need(ncalls);
      s_clast.need(nrounds);
      bool full = true;
      for (int k = 0; k < nrounds && full; k++) full = pr_cf[k] + pr_len[k] == ncalls;
      // one call at N < 64 (an online call): decide, timeline, LCR and the results
      // header in one single-block launch (their grids were a block or two each)
      const int Gf = group_lanes();
      const bool one = ncalls == 1 && full && !split_on() && !rec_on && (int64_t)nrounds * Gf <= 8192;
      if (one && N >= 64) {
        // the pairs by k_fame_decide_blk, then the timeline, LCR and the results header
        // in one single-block launch (in place of k_fame_timeline_g, k_lcr_scan, k_out_init)
        s_out.need(o_tx0 + 2 * (size_t)ntxb0);
        int32_t* hdr = s_out.p;
        fame_dispatch(0, t, nrounds, npairs, ncalls, &pr_round, &pr_off, true);
        const FameCall fc = fame_call_args(nrounds, npairs, ncalls, hdr);
        switch (NW) {
#define FTAIL(B)                                                                                      \
  case B:                                                                                             \
    KLAUNCH((k_fame_call<64, B, false>), dim3(1), dim3(1024), 0, st, t, fc);                           \
    break;
          FTAIL(1)
          FTAIL(2)
          FTAIL(3)
          FTAIL(4)
#undef FTAIL
          default:
            throw EngineError(HGE_ERR_INTERNAL, "unsupported N");
        }
        hdr_done = true;
        x_iter++;
        lcr_dev = true;
        break;
      }
      if (one && N < 64 && (int64_t)npairs * N <= 8192) {
        s_out.need(o_tx0 + 2 * (size_t)ntxb0);
        int32_t* hdr = s_out.p;
        fc_pend = fame_call_args(nrounds, npairs, ncalls, hdr);
#define FCALL(GG) KLAUNCH((k_fame_call<GG, 1, true>), dim3(1), dim3(1024), 0, st, t, fc_pend);
        if (Gf == 16) {
          // launched with the order's stages when they run as one block (k_consensus_call)
          fame_deferred = true;
        } else if (Gf == 32) {
          FCALL(32)
        } else {
          FCALL(64)
        }
#undef FCALL
        hdr_done = true;
        x_iter++;
        lcr_dev = true;
        break;
      }
      if (selective && iter > 0) {
        // the previous layout's decisions moved, then the widened rounds' new pairs
        s_dec2.need((size_t)npairs * N);
        std::vector<int32_t> rel(2 * (size_t)nrounds);
        std::vector<int32_t> plist;
        for (int k = 0; k < nrounds; k++) {
          rel[k] = old_off[k];
          rel[nrounds + k] = old_len[k];
          for (int q = old_len[k]; q < pr_len[k]; q++) plist.push_back(pr_off[k] + q);
        }
        s_relay.need(rel.size() + plist.size() + 1);
        h2d(s_relay.p, rel.data(), 4 * rel.size());
        if (!plist.empty()) h2d(s_relay.p + rel.size(), plist.data(), 4 * plist.size());
        KLAUNCH(k_dec_relayout, dim3(nrounds), dim3(256), 0, st, (const uint8_t*)s_dec.p, s_dec2.p,
                (const int32_t*)s_relay.p, (const int32_t*)(s_relay.p + nrounds), (const int32_t*)(c_pr + nrounds),
                N, c_Lc, ncalls, c_flags);
        std::swap(s_dec, s_dec2);
        if (!plist.empty()) {
          switch (NW) {
#define XCASE(B)                                                                                      \
  case B:                                                                                             \
    KLAUNCH((k_fame_decide_blk<B>), dim3((unsigned)plist.size()), dim3(N), 0, st, t, c_pr, c_pr + nrounds, \
            c_pr + 2 * nrounds, nrounds, 0, npairs, c_nc, c_Rc, s_dec.p,                              \
            (const int32_t*)(s_relay.p + rel.size()));                                                \
    break;
            XCASE(1)
            XCASE(2)
            XCASE(3)
            XCASE(4)
#undef XCASE
            default:
              throw EngineError(HGE_ERR_INTERNAL, "unsupported N");
          }
        }
        // the timeline over the whole layout again
        fame_dispatch(0, t, nrounds, 0, ncalls, &pr_round, &pr_off);
      } else {
        fame_dispatch(0, t, nrounds, npairs, ncalls, &pr_round, &pr_off);
      }
      if (rec_on && !split_on()) {
        rec_dec.emplace_back((size_t)npairs * N);
        readback(rec_dec.back().data(), s_dec.p, (size_t)npairs * N);
      }
      x_iter++;
      s_rfail.need(nrounds);
      KLAUNCH(k_lcr_scan, dim3(1), dim3(1024), 0, st, c_Lc, ncalls, lcr, s_LCR.p, c_pr,
              c_pr + 2 * nrounds, c_pr + 3 * nrounds, nrounds, s_clast.p, c_flags,
              selective ? s_rfail.p : (int32_t*)nullptr);
      if (full) {
        lcr_dev = true;
        break;
      }
      int32_t fl[3];
      std::vector<int32_t> rf(selective ? nrounds : 0);
      if (selective) d2h(rf.data(), s_rfail.p, 4 * (size_t)nrounds);
      readback(fl, c_flags, 3);
      if (fl[0]) {  // a round stayed undecided past its window: widen (those rounds only)
        if (selective) {
          old_off = pr_off;
          old_len = pr_len;
          for (int k = 0; k < nrounds; k++)
            if (rf[k]) spec_r[k] *= 2;
        }
        continue;
      }
      lcr_new = fl[1];
      if (lcr_new > lcr) c_set = fl[2];
      break;
    }

    tp[2] = now_ns();
    // ---- DecideRoundReceived / FindOrder ----
    bool got_order = false;
    // results block: counters | per-call counts | order | per-block transaction sums
    const size_t o_tx = o_tx0;
    const int ntxb = ntxb0;
    s_out.need(o_tx + 2 * (size_t)ntxb);
    int32_t* o_cnt = s_out.p;  // [0] received [1] undetermined [2] LCR events [4..5] tx
    int32_t* o_cc = s_out.p + 8;
    int32_t* o_ids = s_out.p + 8 + ncalls;
    // a replay's sorts write the order straight into the pinned order buffer (host
    // memory mapped into the device: the writes cross PCIe while the later buckets
    // sort; no copy after the replay)
    const bool direct = lazy_order && !order_out && !spl && pin_ord_dev;
    int32_t* ids_dst = o_ids;
    bool wrote_direct = false;  // (only the bucket sorts below write there; other paths write o_ids)
    unsigned long long* o_ntx = (unsigned long long*)(s_out.p + 4);
    // the results header zeroed, with the new LastConsensusRound (o_cnt[3]) when the
    // device holds it (one launch in place of a memset and a copy)
    // (folded into k_visibility's launch when that runs)
    const int32_t* lcr_src = lcr_dev ? (const int32_t*)(c_flags + 1) : (const int32_t*)nullptr;
    // an online call at N <= 16: the order's stages in one single-block launch
    // (k_order_call: segments, round received with its median, the call's bucket, the
    // undetermined list, keys, the sort, the persisted fame), with DecideFame's block
    // in front when it waited (k_consensus_call)
    const bool ocall_pre = ord && nr > 0 && ncalls == 1 && calls[0] >= n_coords && commit && N <= 16 && !spl &&
                           ncand <= SCAN_LDS && (int64_t)nr * group_lanes() <= 65536 &&
                           (nrounds == 0 || lcr_dev) && !getenv("HGE_NO_ORDER_CALL");
    if (fame_deferred && !ocall_pre) {
      KLAUNCH((k_fame_call<16, 1, true>), dim3(1), dim3(1024), 0, st, t, fc_pend);
      fame_deferred = false;
    }
    if (!(ord && nr > 0) && !hdr_done)
      KLAUNCH(k_out_init, dim3(div_up(8 + ncalls, 256)), dim3(256), 0, st, s_out.p, 8 + ncalls, lcr_src);
    // the single-block order kernel's arguments (k_order_call; front: the caller sets it)
    auto order_call_args = [&](const SegInfo& si) {
      s_recv.need(ncand);
      s_rr.need(ncand);
      s_cts.need(ncand);
      s_fund.need(ncand);
      s_upos.need(ncand);
      s_bpos.need(2 * (size_t)ncalls + 2);
      s_und2.need(d_und.n);
      s_keys.need((size_t)ncand * sizeof(OKey));
      s_keys2.need((size_t)ncand * sizeof(OKey));
      OrderCall oc{};
      oc.si = si;
      oc.rr_lo = rr_lo;
      oc.nr = nr;
      oc.segoff = c_sgo;
      oc.segcnt = s_segcnt.p;
      oc.seg_call = s_segcall.p;
      oc.seg_round = s_seground.p;
      oc.seg_dec = s_segdec.p;
      oc.seg_fws = s_segfws.p;
      oc.theta = s_theta.p;
      oc.cand = cand;
      oc.ncand = ncand;
      oc.R_last = R_last;
      oc.recv = s_recv.p;
      oc.rr = s_rr.p;
      oc.cts = s_cts.p;
      oc.cnt = o_cc;
      oc.bpos = s_bpos.p;
      oc.total = o_cnt;
      oc.blist = s_bpos.p + ncalls;
      oc.nblist = s_bpos.p + 2 * ncalls;
      oc.f_und = s_fund.p;
      oc.upos = s_upos.p;
      oc.nund = o_cnt + 1;
      oc.und_out = s_und2.p;
      oc.k1 = (OKey*)s_keys.p;
      oc.k2 = (OKey*)s_keys2.p;
      oc.ev_rr = d_rr.p;
      oc.ev_cts = d_cts.p;
      oc.ntx = (unsigned long long*)(s_out.p + o_tx);
      oc.ntxb = ntxb;
      oc.ids = o_ids;
      oc.pr = c_pr;
      oc.nrounds = do_fame ? nrounds : 0;
      oc.clast = s_clast.p;
      oc.dec = s_dec.p;
      oc.nc = c_nc;
      oc.flags = c_flags;
      oc.lcr_old = lcr;
      oc.n_lo = (int)std::min<int64_t>(calls[0], n_coords);
      oc.n1 = (int)n_coords;
      oc.lcre_out = o_cnt + 2;
      return oc;
    };
    // one call's bucket, undetermined list, keys, sort and persisted fame as one
    // single-block launch at any N (k_order_call, front = 0) when the order's first
    // stages ran as their own grids
    const bool otail_ok = ord && commit && ncalls == 1 && !spl && ncand <= SCAN_LDS &&
                          (!do_fame || nrounds == 0 || lcr_dev) && !getenv("HGE_NO_ORDER_CALL");
    SegInfo si_tail{};
    if (ord) {
      if (nr > 0) {
        SegInfo si;
        si.pr_index = c_pidx;
        if (nrounds > 0) {
          si.pr_off = c_pr + nrounds;
          si.pr_cf = c_pr + 2 * nrounds;
          si.pr_len = c_pr + 3 * nrounds;
          si.clast = s_clast.p;
          si.dec = s_dec.p;
        } else {
          si.pr_off = si.pr_cf = si.pr_len = si.clast = nullptr;
          si.dec = nullptr;
        }
        si_tail = si;
        s_segcnt.need(nr);
        // first call at which each event is visible (arrivals, round received); one call
        // that sees every event (an online call) needs no table: 0 for all, and the
        // header is zeroed alone (a table of every event per call grew with the stream)
        vis_all = ncalls == 1 && calls[0] >= n_coords;
        if (vis_all) {
          if (!hdr_done)
            KLAUNCH(k_out_init, dim3(div_up(8 + ncalls, 256)), dim3(256), 0, st, s_out.p, 8 + ncalls, lcr_src);
        } else {
          s_vis.need(std::max<int64_t>(n_coords, 1));
          KLAUNCH(k_visibility, dim3(div_up(n_coords, 256) + div_up(8 + ncalls, 256)), dim3(256), 0, st,
                  (const int64_t*)c_nc, ncalls, (int)n_coords, s_vis.p, s_out.p, 8 + ncalls, lcr_src);
        }
        const int32_t* visp = vis_all ? (const int32_t*)nullptr : (const int32_t*)s_vis.p;
        // one pass into per-round capacity slots (no count round trip); theta inline
        // for N <= 64, by k_seg_theta_wide above
        const int G = group_lanes();
        const size_t ns = (size_t)std::max<int64_t>(nslot, 1);
        s_segcall.need(ns);
        s_seground.need(ns);
        s_segdec.need(ns);
        s_segfws.need(ns * NW);
        s_theta.need(ns * N);
        segoff_p = c_sgo;
        ocall = ocall_pre;
        if (ocall) {
          OrderCall oc = order_call_args(si);
          oc.front = 1;
          if (fame_deferred) {
            KLAUNCH(k_consensus_call<16>, dim3(1), dim3(1024), 0, st, t, fc_pend, oc);
            fame_deferred = false;
          } else {
            KLAUNCH(k_order_call<16>, dim3(1), dim3(1024), 0, st, t, oc);
          }
          std::swap(d_und, s_und2);
          got_order = true;
        }
#define SEG1(GG, SPL)                                                                              \
  KLAUNCH((k_segments_1p<GG, SPL>), dim3(div_up((int64_t)nr * GG, 256)), dim3(256), 0, st, t,      \
          rr_lo, nr, ncalls, visp, si, (const int32_t*)c_sgo, s_segcnt.p,                          \
          s_segcall.p, s_seground.p, s_segdec.p, s_segfws.p, s_theta.p);
#define THW(B)                                                                                     \
  if (wide32)                                                                                      \
    KLAUNCH(k_seg_theta32<B>, dim3(std::min(nr, 4096)), dim3(256), 0, st, t,                       \
            (const int32_t*)s_seground.p, (const int32_t*)c_sgo, (const int32_t*)s_segcnt.p, nr,   \
            (const uint64_t*)s_segfws.p, s_theta.p);                                               \
  else                                                                                             \
    KLAUNCH(k_seg_theta_wide<B>, dim3(std::min(nr, 4096), nr < 64 ? 8 : 2), dim3(1024), 0, st, t,  \
            (const int32_t*)s_seground.p, (const int32_t*)c_sgo, (const int32_t*)s_segcnt.p, nr,   \
            (const uint64_t*)s_segfws.p, s_theta.p, dbg_p());
        // the frontier rows transposed (WLA) for the batch's rounds: theta (N > 64) and
        // the median (N > 16) read them
        const bool wla = N > 16 && R_last > rr_lo && !ocall;
        if (wla) {
          d_WLA.need((size_t)Rcap * N * N);
          if (N > 64 && !wide32) d_WLR.need((size_t)Rcap * N * N);
          Tables tw = tables();
          KLAUNCH(k_witness_la, dim3(div_up(N, 64), div_up(N, 64), R_last - rr_lo), dim3(256), 0, st, tw,
                  rr_lo);
          t = tables();
        }
        if (ocall) {
          // (k_order_call above)
        } else if (G == 16) {
          SEG1(16, 1)
        } else if (G == 32) {
          SEG1(32, 1)
        } else if (NW == 1) {
          SEG1(64, 1)
        } else if (NW == 2) {
          SEG1(64, 2)
          THW(2)
        } else if (NW == 3) {
          SEG1(64, 3)
          THW(3)
        } else {
          SEG1(64, 4)
          THW(4)
        }
#undef SEG1
#undef THW
        if (getenv("HGE_SEG_DEBUG")) {  // diagnostics: the segments theta walks this batch
          std::vector<int32_t> sc(nr);
          readback(sc.data(), s_segcnt.p, nr);
          int tot = 0, mx = 0;
          for (int v : sc) {
            tot += v;
            mx = std::max(mx, v);
          }
          fprintf(stderr, "[hge seg] calls %d rounds %d segments %d max per round %d\n", ncalls, nr, tot, mx);
          if (dbg_on && s_dbg.p) {
            uint64_t v[16];
            readback(v, s_dbg.p, 16);
            fprintf(stderr, "[hge theta] segments %llu cycles: rows %llu staging %llu bisection %llu\n",
                    (unsigned long long)v[15], (unsigned long long)v[12], (unsigned long long)v[13],
                    (unsigned long long)v[14]);
          }
        }
        // round-received per candidate
        if (!ocall) {
          s_recv.need(ncand);
          s_rr.need(ncand);
          s_cts.need(ncand);
          recv_dispatch(t, cand, ncand, ncalls, rr_lo, R_last, fresh_und, wla);
        }
      } else {
        s_recv.need(ncand);
        HIPCHK(hipMemsetAsync(s_recv.p, 0xFF, 4 * ncand, st));
      }
      if (spl) {  // keep what this part's calls receive (k_split_filter)
        const int p = sp.part;
        const int32_t guard = p + 1 < sp.nparts ? (int32_t)sp.clo[p + 1] : INT32_MIN;
        HIPCHK(hipMemsetAsync(s_small.p + 8, 0, 4, st));
        KLAUNCH(k_split_filter, dim3(div_up(ncand, 256)), dim3(256), 0, st, (const int32_t*)cand, ncand,
                s_recv.p, sp.cb[p], sp.cb[p + 1] - 1, guard, s_small.p + 8);
      }
      // compaction + the order as call buckets (the received count stays on the
      // device: o_cnt[0])
      if (!ocall && otail_ok) {
        OrderCall oc = order_call_args(si_tail);
        oc.front = 0;
        KLAUNCH(k_order_call<16>, dim3(1), dim3(1024), 0, st, t, oc);
        std::swap(d_und, s_und2);
        got_order = true;
        otail = true;
      } else if (!ocall) {
        s_fund.need(ncand);
        s_upos.need(ncand);
        s_rr.need(ncand);
        s_cts.need(ncand);
        // an online call's flags, buckets and undetermined list: one launch (k_recv_list_und below)
        const bool rlu = commit && ncand <= 16384 && ncalls <= 8;
        if (!rlu)
          KLAUNCH(k_recv_flags, dim3(div_up(ncand, 256)), dim3(256), 0, st, s_recv.p, ncand,
                  (int32_t*)nullptr, s_fund.p, commit ? 1 : 0, commit ? o_cc : (int32_t*)nullptr);
        if (!commit)
          KLAUNCH(k_set_rr, dim3(div_up(ncand, 256)), dim3(256), 0, st, t, cand, ncand, s_recv.p,
                  s_rr.p, s_cts.p, d_rr.p, d_cts.p, o_ntx, 0);
        if (commit) {
          s_bpos.need(2 * (size_t)ncalls + 2);
          int32_t* blist = s_bpos.p + ncalls;     // non-empty buckets
          int32_t* nblist = s_bpos.p + 2 * ncalls;  // their count
          // a small candidate set: the undetermined list's scan and scatter ride with the
          // call buckets (k_list_und; the list swap below is the same)
          const bool lu = ncand <= 16384;
          s_und2.need(d_und.n);
          if (rlu)
            KLAUNCH(k_recv_list_und, dim3(2), dim3(1024), 0, st, (const int32_t*)s_recv.p, (int)ncand, o_cc, ncalls,
                    s_bpos.p, o_cnt, blist, nblist, s_fund.p, s_upos.p, o_cnt + 1, cand, s_und2.p);
          else if (lu)
            KLAUNCH(k_list_und, dim3(2), dim3(1024), 0, st, (const int32_t*)o_cc, ncalls, s_bpos.p, o_cnt, blist,
                    nblist, (const int32_t*)s_fund.p, s_upos.p, (int)ncand, o_cnt + 1, cand, s_und2.p);
          else
            KLAUNCH(k_bucket_list, dim3(1), dim3(1024), 0, st, (const int32_t*)o_cc, ncalls, s_bpos.p,
                    o_cnt, blist, nblist);
          s_keys.need((size_t)ncand * sizeof(OKey));
          s_keys2.need((size_t)ncand * sizeof(OKey));
          OKey* k1 = (OKey*)s_keys.p;
          OKey* k2 = (OKey*)s_keys2.p;
          KLAUNCH(k_bucket_keys, dim3(div_up(ncand, 256)), dim3(256), 0, st, t, cand, ncand, s_recv.p,
                  s_rr.p, s_cts.p, s_bpos.p, k1, d_rr.p, d_cts.p,
                  (unsigned long long*)(s_out.p + o_tx));
          if (direct) {
            ids_dst = pin_ord_dev;
            wrote_direct = true;
          }
          if (ncalls <= 8) {
            // a few buckets (an online call): one launch, each bucket to the path its size takes
            KLAUNCH(k_bucket_sort_all, dim3(ncalls), dim3(1024), 0, st, (const int32_t*)s_bpos.p,
                    (const int32_t*)o_cc, (const int32_t*)blist, (const int32_t*)nblist, k1, k2, ids_dst);
          } else {
            // buckets of 513 .. 2 * BIG_SORT keys in LDS (k_bucket_sort_big), the rest here
            KLAUNCH(k_bucket_sort, dim3(std::min(ncalls, 2048)), dim3(256), 0, st,
                    (const int32_t*)s_bpos.p, (const int32_t*)o_cc, (const int32_t*)blist,
                    (const int32_t*)nblist, k1, k2, ids_dst, 1);
            if (ncand > 512)  // (no bucket past 512 keys otherwise)
              KLAUNCH(k_bucket_sort_big, dim3(std::min(ncalls, n_cu())), dim3(1024), 0, st,
                      (const int32_t*)s_bpos.p, (const int32_t*)o_cc, (const int32_t*)blist,
                      (const int32_t*)nblist, (const OKey*)k1, k2, ids_dst);
          }
          // new undetermined list (in candidate order), scattered into the spare list
          // (same capacity) and swapped: no device copy
          if (!lu) {
            scan_large(s_fund.p, s_upos.p, ncand, o_cnt + 1);
            KLAUNCH(k_scatter_und, dim3(div_up(ncand, 256)), dim3(256), 0, st, cand, ncand, s_fund.p, s_upos.p,
                    s_und2.p);
          }
          std::swap(d_und, s_und2);
          got_order = true;
        }
      }
    }

    if (fame_deferred) throw EngineError(HGE_ERR_INTERNAL, "DecideFame's launch left pending");
    // ---- persist fame / LCR ----
    bool lcr_up = false;
    if (do_fame && nrounds > 0 && !ocall && !otail) {
      if (lcr_dev) {
        // the persisted fame and RoundEvents(LCR - 1) as below (the new LCR and its
        // call read on the device) in one launch
        const int64_t nfrom = std::min<int64_t>(calls[0], n_coords);
        const int nb_fp = (int)div_up((int64_t)nrounds * N, 256);
        KLAUNCH(k_fame_persist_lcre, dim3(nb_fp + std::max(1, div_up(n_coords - nfrom, 256))), dim3(256), 0, st, t,
                (const int32_t*)c_pr, (const int32_t*)(c_pr + nrounds), (const int32_t*)(c_pr + 2 * nrounds),
                (const int32_t*)(c_pr + 3 * nrounds), nrounds, (const int32_t*)s_clast.p, (const uint8_t*)s_dec.p,
                nb_fp, (const int64_t*)c_nc, (const int32_t*)c_flags, lcr, (int)nfrom, (int)n_coords, o_cnt + 2);
      } else {
        fame_dispatch(1, t, nrounds, npairs, ncalls);
        if (lcr_new > lcr) {
          // RoundEvents(lcr_new - 1) at call c_set: events of that round minus the
          // ones inserted after that call
          lcr_up = true;
          const int r = lcr_new - 1;
          if (r >= 0) {
            const int64_t nfrom = std::min<int64_t>(calls[c_set], n_coords);
            KLAUNCH(k_lcre, dim3(std::max(1, div_up(n_coords - nfrom, 256))), dim3(256), 0, st, t,
                    (int)nfrom, (int)n_coords, r, o_cnt + 2);
          }
        }
      }
    }
    bool split_done = false;
    if (spl && got_order) {  // the parts' ordered slices, joined in call order
      split_commit(o_cnt, o_cc, o_ids, ntxb, (const unsigned long long*)(s_out.p + o_tx), order_out, counts_out);
      got_order = false;
      split_done = true;
    }
    tp[3] = now_ns();
    // the batch's one closing round trip (read in place from the pinned arena); a
    // replay's order stays in HBM (lazy: counters, per-call counts and transaction sums only)
    const bool lazy = got_order && lazy_order && !order_out;
    const size_t off = d2h_pinned(s_out.p, 4 * (got_order && !lazy ? o_tx + 2 * (size_t)ntxb : 8 + (size_t)ncalls));
    const size_t off_tx = lazy ? d2h_pinned(s_out.p + o_tx, 4 * 2 * (size_t)ntxb) : 0;
    sync();
    const int32_t* ho = (const int32_t*)(pin + off);
    const int32_t* htx = lazy ? (const int32_t*)(pin + off_tx) : ho + o_tx;
    const int32_t nrecv = ho[0];
    if (got_order) {
      const int32_t* ids = ho + 8 + ncalls;
      unsigned long long ntx = 0;
      for (int b2 = 0; b2 < ntxb; b2++) {
        unsigned long long v = 0;
        memcpy(&v, htx + 2 * (size_t)b2, 8);
        ntx += v;
      }
      if (lazy) {  // delivered into the pinned order buffer (sized at hge_replay_prepare)
        if ((size_t)nrecv > pin_ord_cap) throw EngineError(HGE_ERR_INTERNAL, "order buffer below the ordered count");
        const int64_t td = now_ns();
        if (!wrote_direct && nrecv) {
          HIPCHK(hipMemcpyAsync(pin_ord, o_ids, 4 * (size_t)nrecv, hipMemcpyDeviceToHost, st));
          sync();
        }
        // the delivery's wall time after the sorts (hge_stage_times [5]; ~0 when written direct)
        stage_ms[5] = (float)((now_ns() - td) / 1e6);
        cons_pin_n = nrecv;
      } else {
        consensus.insert(consensus.end(), ids, ids + nrecv);
      }
      ctx += (int64_t)ntx;
      if (order_out) order_out->insert(order_out->end(), ids, ids + nrecv);
      if (counts_out)
        for (int c = 0; c < ncalls; c++) counts_out->push_back(ho[8 + c]);
      n_und = ho[1];
    } else if (do_order && counts_out && !split_done) {
      for (int c = 0; c < ncalls; c++) counts_out->push_back(0);
    }
    if (lcr_dev && ho[3] > lcr) {
      lcr_up = true;
      lcr_new = ho[3];
    }
    if (lcr_up) {
      lcr = lcr_new;
      lcre = lcr_new - 1 >= 0 ? ho[2] : 0;
    }
    tp[4] = now_ns();
    if (tph)
      fprintf(stderr, "[hge consensus] prologue %.3f ms, fame %.3f ms (incl. syncs), order enqueue %.3f ms, closing %.3f ms\n",
              (tp[1] - tp[0]) / 1e6, (tp[2] - tp[1]) / 1e6, (tp[3] - tp[2]) / 1e6, (tp[4] - tp[3]) / 1e6);
    prof_collect();
  }

  // split replay: the parts' fame decisions (each part's pairs [P0, P1)) all-gathered
  void split_exchange_dec(const std::vector<int32_t>& pr_round, const std::vector<int32_t>& pr_off, int npairs) {
    const int G = sp.nparts, nr = (int)pr_round.size();
    std::vector<int64_t> P0(G), P1(G);
    int64_t mx = 1;
    for (int g = 0; g < G; g++) {
      int klo = 0, khi = 0;
      split_rounds_of(g, pr_round, klo, khi);
      P0[g] = klo < nr ? pr_off[klo] : npairs;
      P1[g] = khi < nr ? pr_off[khi] : npairs;
      mx = std::max(mx, P1[g] - P0[g]);
    }
    const int64_t bytes = (mx * N + 255) / 256 * 256;
    uint8_t* buf = (uint8_t*)x_buf(bytes);
    const int p = sp.part;
    if (P1[p] > P0[p])
      HIPCHK(hipMemcpyAsync(buf + (size_t)p * bytes, s_dec.p + (size_t)P0[p] * N, (size_t)(P1[p] - P0[p]) * N,
                            hipMemcpyDeviceToDevice, st));
    x_gather(bytes, buf);
    if (emulating()) {  // the other parts' decisions of this fame iteration, from the record
      const std::vector<uint8_t>& rd = rec_dec.at((size_t)x_iter);
      for (int g = 0; g < G; g++)
        if (g != p && P1[g] > P0[g]) h2d(buf + (size_t)g * bytes, rd.data() + (size_t)P0[g] * N, (size_t)(P1[g] - P0[g]) * N);
    }
    for (int g = 0; g < G; g++)
      if (g != p && P1[g] > P0[g])
        HIPCHK(hipMemcpyAsync(s_dec.p + (size_t)P0[g] * N, buf + (size_t)g * bytes, (size_t)(P1[g] - P0[g]) * N,
                              hipMemcpyDeviceToDevice, st));
  }

  // split replay: this part's ordered slice (its calls' buckets, round received,
  // consensus timestamps, left candidates) all-gathered; every part then holds the
  // whole order, the per-call batches and the undetermined list (the last part's)
  void split_commit(const int32_t* o_cnt, const int32_t* o_cc, const int32_t* o_ids, int ntxb,
                    const unsigned long long* ntx_part, std::vector<int32_t>* order_out,
                    std::vector<int64_t>* counts_out) {
    const int G = sp.nparts, p = sp.part;
    int maxcalls = 0;
    int64_t cap = 1;
    for (int g = 0; g < G; g++) {
      maxcalls = std::max(maxcalls, sp.cb[g + 1] - sp.cb[g]);
      cap = std::max(cap, sp.a[g + 1] - sp.clo[g]);
    }
    const SplitSlot L = SplitSlot::make(maxcalls, cap);
    const int64_t bytes = 4 * L.words;
    int32_t* buf = (int32_t*)x_buf(bytes);
    KLAUNCH(k_split_pack, dim3(std::min(div_up(cap, 256), 4096)), dim3(256), 0, st, o_cnt, o_cc, sp.cb[p],
            sp.cb[p + 1] - sp.cb[p], o_ids, (const int32_t*)d_und.p, (const int32_t*)d_rr.p,
            (const int64_t*)d_cts.p, ntx_part, ntxb, (const int32_t*)(s_small.p + 8), L,
            buf + (size_t)p * L.words);
    x_gather(bytes, buf);
    if (emulating()) {  // the other parts' slots from the record
      int64_t off0 = 0;
      for (int g = 0; g < G; g++) {
        int64_t nord = 0;
        for (int c = sp.cb[g]; c < sp.cb[g + 1]; c++) nord += rec_counts[c];
        if (g != p) {
          const bool last = g == G - 1;
          std::vector<int32_t> sl((size_t)L.words, 0);
          unsigned long long tx = 0;
          for (int64_t i = 0; i < nord; i++) {
            const int32_t x = rec_order[off0 + i];
            sl[L.ids + i] = x;
            sl[L.rr + i] = rec_rr[x];
            memcpy(&sl[L.cts + 2 * i], &rec_cts[x], 8);
            tx += (unsigned long long)h_ntx[x];
          }
          const int64_t nleft = last ? (int64_t)rec_left.size() : 0;
          for (int64_t i = 0; i < nleft; i++) sl[L.left + i] = rec_left[i];
          for (int c = sp.cb[g]; c < sp.cb[g + 1]; c++) sl[L.counts + (c - sp.cb[g])] = (int32_t)rec_counts[c];
          sl[0] = (int32_t)nord;
          sl[1] = (int32_t)nleft;
          sl[4] = (int32_t)(uint32_t)tx;
          sl[5] = (int32_t)(uint32_t)(tx >> 32);
          h2d(buf + (size_t)g * L.words, sl.data(), 4 * (size_t)L.words);
        }
        off0 += nord;
      }
    }
    // every part's header and call counts
    std::vector<int32_t> hd((size_t)G * L.ids);
    for (int g = 0; g < G; g++) d2h(&hd[(size_t)g * L.ids], buf + (size_t)g * L.words, 4 * (size_t)L.ids);
    sync();
    std::vector<int64_t> off(G + 1, 0);
    bool bad = false;
    unsigned long long ntx = 0;
    for (int g = 0; g < G; g++) {
      const int32_t* h0 = &hd[(size_t)g * L.ids];
      bad = bad || h0[2] != 0;
      off[g + 1] = off[g] + h0[0];
      ntx += (unsigned long long)(uint32_t)h0[4] | ((unsigned long long)(uint32_t)h0[5] << 32);
    }
    if (bad) throw EngineError(HGE_ERR_SPLIT, "split replay: an event is received outside every part's range");
    const int64_t tot = off[G];
    s_sord.need((size_t)std::max<int64_t>(tot, 1));
    s_soff.need((size_t)G + 1);
    h2d(s_soff.p, off.data(), 8 * ((size_t)G + 1));
    KLAUNCH(k_split_unpack, dim3(std::min(div_up(cap, 256), 1024), G), dim3(256), 0, st, (const int32_t*)buf, L, G,
            (const int64_t*)s_soff.p, s_sord.p, d_rr.p, d_cts.p);
    // the undetermined list: the last part's left candidates
    const int nleft = hd[(size_t)(G - 1) * L.ids + 1];
    if (nleft > 0)
      HIPCHK(hipMemcpyAsync(d_und.p, buf + (size_t)(G - 1) * L.words + L.left, 4 * (size_t)nleft,
                            hipMemcpyDeviceToDevice, st));
    const size_t po = d2h_pinned(s_sord.p, 4 * (size_t)tot);
    sync();
    const int32_t* ids = (const int32_t*)(pin + po);
    consensus.insert(consensus.end(), ids, ids + tot);
    if (order_out) order_out->insert(order_out->end(), ids, ids + tot);
    ctx += (int64_t)ntx;
    n_und = nleft;
    if (counts_out)
      for (int g = 0; g < G; g++)
        for (int c = sp.cb[g]; c < sp.cb[g + 1]; c++) counts_out->push_back(hd[(size_t)g * L.ids + 8 + (c - sp.cb[g])]);
  }

  void gather_rounds(const std::vector<int32_t>& ids, std::vector<int32_t>& out) {
    // contiguous-range copy of d_round covering all ids
    int lo = INF32, hi = -1;
    for (int v : ids) {
      lo = std::min(lo, v);
      hi = std::max(hi, v);
    }
    std::vector<int32_t> r(hi - lo + 1);
    readback(r.data(), d_round.p + lo, r.size());
    for (size_t k = 0; k < ids.size(); k++) out[k] = r[ids[k] - lo];
  }

  void scan_large(const int32_t* in, int32_t* out, int n, int32_t* total) {
    if (n <= 16384) {  // one block (an online call's candidates): one launch, not three
      KLAUNCH(k_scan_small, dim3(1), dim3(1024), 0, st, in, out, n, total);
      return;
    }
    const int nb = div_up(n, 1024);
    s_part.need(2 * (size_t)nb + 2);
    KLAUNCH(k_scan_blocks, dim3(nb), dim3(256), 0, st, in, out, n, s_part.p);
    KLAUNCH(k_scan_small, dim3(1), dim3(1024), 0, st, s_part.p, s_part.p + nb, nb, total);
    KLAUNCH(k_scan_add, dim3(div_up(n, 256)), dim3(256), 0, st, out, n, s_part.p + nb);
  }

  // lanes per round in the group-scan kernels (a lane holds NW slots when N > 64)
  int group_lanes() const { return N <= 16 ? 16 : N <= 32 ? 32 : 64; }

  // which 0: k_fame_decide (a split part: the pairs of its rounds, then the parts'
  // decisions all-gathered) and the per-round timeline; which 1: persist
  // decide_only: the pairs' decisions only (k_fame_call<.., false> takes the timeline)
  void fame_dispatch(int which, const Tables& t, int nrounds, int npairs, int ncalls,
                     const std::vector<int32_t>* pr_round = nullptr, const std::vector<int32_t>* pr_off = nullptr,
                     bool decide_only = false) {
    if (which == 1) {
      KLAUNCH(k_fame_persist, dim3(div_up((int64_t)nrounds * N, 256)), dim3(256), 0, st, t, c_pr,
              c_pr + nrounds, c_pr + 2 * nrounds, c_pr + 3 * nrounds, nrounds, s_clast.p,
              s_dec.p);
      return;
    }
    const int G = group_lanes();
    int k_lo = 0, k_hi = nrounds;
    if (split_on() && pr_round) split_rounds_of(sp.part, *pr_round, k_lo, k_hi);
    const int p0 = k_lo < nrounds && pr_off ? (*pr_off)[k_lo] : (k_lo < nrounds ? 0 : npairs);
    const int p1 = k_hi < nrounds && pr_off ? (*pr_off)[k_hi] : npairs;
    const int items = (p1 - p0) * N;
    if (items > 0) {
      switch (NW) {
#define DCASE(B)                                                                                     \
  case B:                                                                                            \
    if (N == 64 * B)                                                                                 \
      KLAUNCH((k_fame_decide_blk<B>), dim3(p1 - p0), dim3(N), 0, st, t, c_pr + k_lo,                  \
              c_pr + nrounds + k_lo, c_pr + 2 * nrounds + k_lo, k_hi - k_lo, p0, p1, c_nc, c_Rc,      \
              s_dec.p, (const int32_t*)nullptr);                                                     \
    else                                                                                             \
      KLAUNCH((k_fame_decide<B>), dim3(div_up(items, 256)), dim3(256), 0, st, t, c_pr + k_lo,         \
              c_pr + nrounds + k_lo, c_pr + 2 * nrounds + k_lo, k_hi - k_lo, p0, p1, c_nc, c_Rc,      \
              s_dec.p);                                                                              \
    break;
        DCASE(1)
        DCASE(2)
        DCASE(3)
        DCASE(4)
#undef DCASE
        default:
          throw EngineError(HGE_ERR_INTERNAL, "unsupported N");
      }
    }
    if (split_on() && pr_round) split_exchange_dec(*pr_round, *pr_off, npairs);
    if (decide_only) return;
    switch (NW) {
#define FCASE(B)                                                                                 \
  case B:                                                                                        \
    if (G == 16)                                                                                 \
      KLAUNCH((k_fame_timeline_g<16, 1>), dim3(div_up((int64_t)nrounds * 16, 256)), dim3(256), 0, \
              st, t, c_pr, c_pr + nrounds, c_pr + 2 * nrounds, c_pr + 3 * nrounds, nrounds, c_nc, \
              s_dec.p, s_decbit.p, c_Lc);                                                        \
    else if (G == 32)                                                                            \
      KLAUNCH((k_fame_timeline_g<32, 1>), dim3(div_up((int64_t)nrounds * 32, 256)), dim3(256), 0, \
              st, t, c_pr, c_pr + nrounds, c_pr + 2 * nrounds, c_pr + 3 * nrounds, nrounds, c_nc, \
              s_dec.p, s_decbit.p, c_Lc);                                                        \
    else                                                                                         \
      KLAUNCH((k_fame_timeline_g<64, B>), dim3(div_up((int64_t)nrounds * 64, 256)), dim3(256), 0, \
              st, t, c_pr, c_pr + nrounds, c_pr + 2 * nrounds, c_pr + 3 * nrounds, nrounds, c_nc, \
              s_dec.p, s_decbit.p, c_Lc);                                                        \
    break;
      FCASE(1)
      FCASE(2)
      FCASE(3)
      FCASE(4)
#undef FCASE
      default:
        throw EngineError(HGE_ERR_INTERNAL, "unsupported N");
    }
    (void)ncalls;
  }

  void recv_dispatch(const Tables& t, const int32_t* cand, int ncand, int ncalls, int rr_lo,
                     int R_last, bool fresh, bool wla_done) {
    // N > 16: the median is a wave-wide radix select (k_median_wave) over coalesced
    // rows: the round frontier rows transposed (WLA, k_witness_la, for every round a
    // candidate can receive) and the FD timestamp offsets (FDTD).  A fresh replay's
    // candidate list is the identity (candidate q = event q).
    const bool wmed = N > 16;
    const bool ident = fresh && cand == d_und.p && (int64_t)ncand == n_events;
    int32_t* bseg = nullptr;
    if (wmed) {
      s_bseg.need(ncand);
      bseg = s_bseg.p;
      if (R_last > rr_lo && !wla_done) {
        d_WLA.need((size_t)Rcap * N * N);
        if (N > 64 && !wide32) d_WLR.need((size_t)Rcap * N * N);
        Tables tw = tables();
        KLAUNCH(k_witness_la, dim3(div_up(N, 64), div_up(N, 64), R_last - rr_lo), dim3(256), 0, st, tw,
                rr_lo);
      }
    }
    switch (NW) {
#define RCASE(B)                                                                                 \
  case B:                                                                                        \
    KLAUNCH(k_round_received<B>, dim3(div_up(ncand, 256)), dim3(256), 0, st, t, cand, \
                       ncand, vis_all ? (const int32_t*)nullptr : (const int32_t*)s_vis.p, ncalls, 0, rr_lo, R_last, segoff_p, \
                       s_segcnt.p,                                                               \
                       s_segcall.p, s_segdec.p, s_segfws.p, s_theta.p, s_recv.p, s_rr.p,         \
                       s_cts.p, bseg);                                                           \
    if (wmed)                                                                                    \
      KLAUNCH(k_median_wave<B>, dim3(div_up(ncand, 4 * MED_EPW)), dim3(256), 0, st, tables(),              \
              ident ? (const int32_t*)nullptr : cand, ncand, s_recv.p, s_rr.p, bseg, s_segfws.p,  \
              s_cts.p);                                                                          \
    break;
      RCASE(1)
      RCASE(2)
      RCASE(3)
      RCASE(4)
#undef RCASE
      default:
        throw EngineError(HGE_ERR_INTERNAL, "unsupported N");
    }
  }

  // DivideRounds: everything inserted becomes visible to the consensus calls
  bool dividing = false, und_appended = false;
  void divide() {
    dividing = true;
    und_appended = false;
    try {
      coords();
    } catch (...) {
      dividing = false;
      throw;
    }
    dividing = false;
    if (n_divided < n_coords) {
      // append the newly divided events to the undetermined list (insertion order),
      // unless k_round_assign already did
      const int64_t a = n_divided, m = n_coords - n_divided;
      ensure_events(n_coords);
      if (!und_appended) KLAUNCH(k_iota, dim3(div_up(m, 256)), dim3(256), 0, st, d_und.p + n_und, m, (int32_t)a);
      n_und += m;
      n_divided = n_coords;
    }
    update_rdiv();
  }

  // An online RunConsensus at N <= 16 with ONE host round trip: the coordinate and
  // rounds launches of divide() (k_la_seq with the frontier start and the batch's FD,
  // k_fss, the rounds walk with the assignment and tail), then k_consensus_dyn, whose
  // control block the device builds from the walk's round count and the candidates'
  // lowest round; the results and the rounds' first witnesses come back together.
  // The rounds table is grown first so that the walk cannot overflow it (R grows by
  // at most one per new event).  Returns false (nothing done) when the call does not
  // fit this path.
  bool online_fast(std::vector<int32_t>& order) {
    const int64_t n0 = n_coords, n1 = n_events, m = n1 - n0;
    if (N > 16 || m <= 0 || R == 0 || cs_pending || split_on() || rec_on || ext_on || sp_active) return false;
    if (n_divided != n0 || !la_seq_ok(m) || n_und + m > 65536 || n_und + m > SCAN_LDS) return false;
    if (getenv("HGE_NO_ONLINE_FAST")) return false;
    int maxlen = 0;
    for (int c = 0; c < N; c++) maxlen = std::max(maxlen, chain_len[c]);
    if (maxlen + 1 >= 0xFFFF) return false;
    consensus_sync();
    ensure_rcap((int64_t)R + m + 4);
    // ---- divide(): coordinates and rounds, no readback
    dividing = true;
    und_appended = false;
    if (!coords_a()) {
      dividing = false;
      throw EngineError(HGE_ERR_INTERNAL, "online call: no coordinates to compute");
    }
    if (!fst_fused || !cs_pending) throw EngineError(HGE_ERR_INTERNAL, "online call: frontier start not fused");
    cs_pending = false;
    Tables t = tables();
    und_appended = true;  // (n_divided == n0: the walk's block appends the new ids)
    s_newwit.need(m);
    RoundAssign ra{(int)n0, (int)n1, s_newwit.p, k_rs + 2, d_und.p + n_und};
    int Gw = 1;
    while (Gw < std::min(N, 64)) Gw <<= 1;
    ra.minw = d_minw.p;
    ra.G = Gw;
    ra.und = d_und.p;
    ra.n_und = (int)n_und;
    ra.lo = (int)n_divided;
    ra.hi = (int)n1;
    ra.r_from = minw_full ? 0 : -1;
    ra.rlo_dev = s_fst.p;
    const int64_t guess = m + 16 * (int64_t)N;
    KLAUNCH(k_fss<16>, dim3((unsigned)std::min<int64_t>(1024, div_up(guess * 16, 256))), dim3(256), 0, st, t, k_lo,
            k_lo + N, 0, (int32_t*)nullptr, (uint16_t*)d_FSS.p, (const int32_t*)(k_lo + 2 * N));
    KLAUNCH((k_rounds_walk<16, 4, 256>), dim3(1), dim3(1024), 0, st, t, (const uint16_t*)d_FSS.p, k_len, k_len + N,
            k_rs, 0, R, dbg_p(), (const int32_t*)s_fst.p, ra);
    fst_fused = false;
    dividing = false;
    n_coords = n1;
    coords_len = chain_len;
    n_und += m;
    n_divided = n_coords;
    und_fresh = false;
    // ---- consensus of the one call, control built on the device
    const int Rmax = R + (int)m + 1;
    const int nround_max = std::max(1, Rmax - 2 - lcr), nr_max = std::max(1, Rmax);
    const int ncand = (int)n_und;
    const size_t o_Rc = 2, o_Lc = 3, o_fl = 4, o_pr = 8, o_pidx = o_pr + 4 * (size_t)nround_max;
    const size_t o_sgo = o_pidx + nr_max;
    s_cctl.need(o_sgo + nr_max + 1);
    c_nc = (int64_t*)s_cctl.p;
    c_Rc = s_cctl.p + o_Rc;
    c_Lc = s_cctl.p + o_Lc;
    c_flags = s_cctl.p + o_fl;
    c_pr = s_cctl.p + o_pr;
    c_pidx = s_cctl.p + o_pidx;
    c_sgo = s_cctl.p + o_sgo;
    s_dec.need((size_t)nround_max * N);
    s_decbit.need(nround_max);
    s_LCR.need(1);
    s_clast.need(nround_max);
    const size_t nslot = (size_t)nr_max * (N + 3);
    s_segcnt.need(nr_max);
    s_segcall.need(nslot);
    s_seground.need(nslot);
    s_segdec.need(nslot);
    s_segfws.need(nslot * NW);
    s_theta.need(nslot * N);
    const size_t o_tx = (8 + 1 + (size_t)ncand + 1) & ~(size_t)1;
    const int ntxb = div_up(ncand, 256);
    s_out.need(o_tx + 2 * (size_t)ntxb);
    s_recv.need(ncand);
    s_rr.need(ncand);
    s_cts.need(ncand);
    s_fund.need(ncand);
    s_upos.need(ncand);
    s_bpos.need(4);
    s_und2.need(d_und.n);
    s_keys.need((size_t)ncand * sizeof(OKey));
    s_keys2.need((size_t)ncand * sizeof(OKey));
    t = tables();
    DynCall dc{};
    dc.lcr = lcr;
    dc.ncand = ncand;
    dc.Rcap = Rcap;
    dc.n_c = n_divided;
    dc.rstate = k_rs;
    dc.minw = d_minw.p;
    dc.c_nc = c_nc;
    dc.c_Rc = c_Rc;
    dc.c_Lc = c_Lc;
    dc.c_flags = c_flags;
    dc.c_pr = c_pr;
    dc.c_pidx = c_pidx;
    dc.c_sgo = c_sgo;
    dc.dec = s_dec.p;
    dc.decbit = s_decbit.p;
    dc.LCR = s_LCR.p;
    dc.clast = s_clast.p;
    dc.out = s_out.p;
    OrderCall& o = dc.o;
    o.segcnt = s_segcnt.p;
    o.seg_call = s_segcall.p;
    o.seg_round = s_seground.p;
    o.seg_dec = s_segdec.p;
    o.seg_fws = s_segfws.p;
    o.theta = s_theta.p;
    o.cand = d_und.p;
    o.ncand = ncand;
    o.recv = s_recv.p;
    o.rr = s_rr.p;
    o.cts = s_cts.p;
    o.cnt = s_out.p + 8;
    o.bpos = s_bpos.p;
    o.total = s_out.p;
    o.blist = s_bpos.p + 1;
    o.nblist = s_bpos.p + 2;
    o.f_und = s_fund.p;
    o.upos = s_upos.p;
    o.nund = s_out.p + 1;
    o.und_out = s_und2.p;
    o.k1 = (OKey*)s_keys.p;
    o.k2 = (OKey*)s_keys2.p;
    o.ev_rr = d_rr.p;
    o.ev_cts = d_cts.p;
    o.ntx = (unsigned long long*)(s_out.p + o_tx);
    o.ntxb = ntxb;
    o.ids = s_out.p + 9;
    o.lcr_old = lcr;
    o.n_lo = (int)n_divided;
    o.n1 = (int)n_divided;
    o.lcre_out = s_out.p + 2;
    KLAUNCH(k_consensus_dyn<16>, dim3(1), dim3(1024), 0, st, t, dc);
    std::swap(d_und, s_und2);
    // ---- the one round trip: the results block and the rounds' first witnesses
    const size_t off = d2h_pinned(s_out.p, 4 * (o_tx + 2 * (size_t)ntxb));
    const size_t offw = d2h_pinned(d_minw.p, 4 * ((size_t)Rcap + 4));
    sync();
    const int32_t* hw = (const int32_t*)(pin + offw);
    if (hw[Rcap + 1]) {  // (unreachable: ensure_rcap covers R + m + 4) the host state has moved on: refuse later calls
      failed = "online call: rounds table overflow past its bound";
      throw EngineError(HGE_ERR_INTERNAL, failed);
    }
    R = hw[Rcap];
    h_minw.assign(hw, hw + R);
    minw_full = false;
    mnr_key[0] = -1;
    update_rdiv();
    const int32_t* ho = (const int32_t*)(pin + off);
    const int32_t nrecv = ho[0];
    const int32_t* ids = ho + 9;
    unsigned long long ntx = 0;
    for (int b2 = 0; b2 < ntxb; b2++) {
      unsigned long long v = 0;
      memcpy(&v, ho + o_tx + 2 * (size_t)b2, 8);
      ntx += v;
    }
    consensus.insert(consensus.end(), ids, ids + nrecv);
    order.insert(order.end(), ids, ids + nrecv);
    ctx += (int64_t)ntx;
    n_und = ho[1];
    if (ho[3] > lcr) {
      lcr = ho[3];
      lcre = lcr - 1 >= 0 ? ho[2] : 0;
    }
    prof_collect();
    return true;
  }

  // first witness id of every round (host copy: Rounds() as seen at any event count)
  void update_rdiv() {
    // h_minw was read back together with the round count (coords)
    h_minw.resize(R);
    if (R == 0) {
      R_div = 0;
      return;
    }
    R_div = (int)(std::lower_bound(h_minw.begin(), h_minw.end(),
                                   (int32_t)std::min<int64_t>(n_divided, INF32)) -
                  h_minw.begin());
  }
};

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
#define GUARD_BEGIN try {
#define REFUSE_IF_FAILED(h) \
  if (!(h)->failed.empty()) throw EngineError(HGE_ERR_INTERNAL, "engine state inconsistent since: " + (h)->failed);
#define GUARD_END(h)                 \
  }                                  \
  catch (EngineError & e) {          \
    (h)->err = e.msg;                \
    return e.code;                   \
  }                                  \
  catch (std::exception & e) {       \
    (h)->err = e.what();             \
    return HGE_ERR_INTERNAL;         \
  }

extern "C" {

int hge_create(int32_t n_participants, int64_t capacity_events, int32_t device, uint32_t flags,
               hge_engine** out) {
  (void)flags;
  if (!out || n_participants < 1 || n_participants > 256) return HGE_ERR_ARG;
  hge_engine* h = new hge_engine();
  try {
    h->init(n_participants, capacity_events, device);
  } catch (EngineError& e) {
    fprintf(stderr, "hge_create: %s\n", e.msg.c_str());
    h->destroy();
    delete h;
    *out = nullptr;
    return e.code;
  }
  *out = h;
  return HGE_OK;
}

void hge_destroy(hge_engine* h) {
  if (!h) return;
  h->destroy();
  delete h;
}

const char* hge_last_error(hge_engine* h) { return h ? h->err.c_str() : "null handle"; }

int hge_reset(hge_engine* h) {
  GUARD_BEGIN
  h->reset_state();
  return HGE_OK;
  GUARD_END(h)
}

int hge_insert_events(hge_engine* h, const hge_event* ev, int64_t n, int32_t* status_out,
                      int64_t* n_accepted) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
  const int64_t c0 = hge_engine::now_ns();
  int64_t acc = 0;
  int rc = HGE_OK;
  for (int64_t i = 0; i < n; i++) {
    const int32_t sp = ev[i].self_parent, op = ev[i].other_parent;
    int r = h->admit(ev[i], sp, op);
    if (r != HGE_OK) {
      if (status_out) status_out[i] = r;
      rc = r;
      break;
    }
    if (status_out) status_out[i] = (int32_t)h->n_events;
    h->append(ev[i], sp, op);
    acc++;
  }
  if (n_accepted) *n_accepted = acc;
  h->hp.insert_ns += hge_engine::now_ns() - c0;
  return rc;
  GUARD_END(h)
}

int hge_divide_rounds(hge_engine* h) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
  h->divide();
  return HGE_OK;
  GUARD_END(h)
}

int hge_decide_fame(hge_engine* h) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
    h->consensus_batch({h->n_divided}, true, false, false, nullptr, nullptr);
  return HGE_OK;
  GUARD_END(h)
}

int hge_decide_round_received(hge_engine* h) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
    h->consensus_batch({h->n_divided}, false, true, false, nullptr, nullptr);
  return HGE_OK;
  GUARD_END(h)
}

int hge_find_order(hge_engine* h, int32_t* ids_out, int64_t cap, int64_t* n_out) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
    std::vector<int32_t> order;
  h->consensus_batch({h->n_divided}, false, true, true, &order, nullptr);
  for (int64_t i = 0; i < (int64_t)order.size() && i < cap && ids_out; i++) ids_out[i] = order[i];
  if (n_out) *n_out = (int64_t)order.size();
  return HGE_OK;
  GUARD_END(h)
}

int hge_run_consensus(hge_engine* h, int32_t* ids_out, int64_t cap, int64_t* n_out) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
  const int64_t c0 = hge_engine::now_ns();
  std::vector<int32_t> order;
  if (!h->online_fast(order)) {
    h->divide();
    h->consensus_batch({h->n_divided}, true, true, true, &order, nullptr);
  }
  for (int64_t i = 0; i < (int64_t)order.size() && i < cap && ids_out; i++) ids_out[i] = order[i];
  if (n_out) *n_out = (int64_t)order.size();
  h->hp.calls++;
  h->hp.call_ns += hge_engine::now_ns() - c0;
  return HGE_OK;
  GUARD_END(h)
}

int hge_replay_prepare(hge_engine* h, const hge_event* ev, int64_t n_sub,
                       const int64_t* call_points, int64_t n_calls, int32_t* status_out) {
  GUARD_BEGIN
  if (n_sub < 0 || (n_sub > 0 && !ev) || n_calls < 0 || (n_calls > 0 && !call_points)) {
    h->err = "hge_replay_prepare: bad argument";
    return HGE_ERR_ARG;
  }
  // call points: strictly ascending submission counts in [1, n_sub]
  for (int64_t c = 0; c < n_calls; c++) {
    if (call_points[c] < 1 || call_points[c] > n_sub || (c > 0 && call_points[c] <= call_points[c - 1])) {
      h->err = "hge_replay_prepare: call points must be strictly ascending within [1, n_sub]";
      return HGE_ERR_ARG;
    }
  }
  h->reset_state();
  h->sp = hge_engine::SplitPlan();  // a plan belongs to the stream it was made for
  h->sp_active = false;
  std::vector<int32_t> idmap(n_sub, -1);
  h->replay_calls.clear();
  int64_t nc = 0;
  for (int64_t i = 0; i < n_sub; i++) {
    const int32_t s = ev[i].self_parent, o = ev[i].other_parent;
    int32_t sp = s < 0 ? HGE_NONE : (s < i && idmap[s] >= 0 ? idmap[s] : HGE_UNKNOWN);
    int32_t op = o < 0 ? HGE_NONE : (o < i && idmap[o] >= 0 ? idmap[o] : HGE_UNKNOWN);
    int r = h->admit(ev[i], sp, op);
    if (r == HGE_OK) {
      idmap[i] = (int32_t)h->n_events;
      h->append(ev[i], sp, op);
    }
    if (status_out) status_out[i] = r == HGE_OK ? idmap[i] : r;
    while (nc < n_calls && call_points[nc] == i + 1) {
      h->replay_calls.push_back(h->n_events);
      nc++;
    }
  }
  h->upload();
  h->cons_pin_n = 0;
  h->ensure_pin_ord((size_t)h->n_events);  // the replay's order is delivered here
  HIPCHK(hipStreamSynchronize(h->st));
  return HGE_OK;
  GUARD_END(h)
}

// A fresh replay in two halves: replay_begin (reset + coordinates) and
// replay_end (rounds frontier, DivideRounds/DecideFame/FindOrder at every call);
// the cross-GPU split runs the walkers and their join between the two.
static void replay_begin(hge_engine* h) {
  // fresh consensus state over the staged events (they stay resident in HBM)
  h->n_coords = h->n_divided = 0;
  h->coords_len.assign(h->N, 0);
  h->R = 0;
  h->h_minw.clear();
  h->lcr = -1;
  h->lcre = 0;
  h->ctx = 0;
  h->consensus.clear();
  h->cons_pin_n = 0;
  h->n_und = 0;
  h->ext_on = false;
  h->w_start = std::chrono::steady_clock::now();
  h->reset_rounds();
  HIPCHK(hipEventRecord(h->ev[0], h->st));
  h->coords_a();
}

static void replay_end(hge_engine* h, int64_t* n_ordered) {
  const int64_t keep = h->n_events;
  if (h->cs_pending) h->coords_b();
  HIPCHK(hipEventRecord(h->ev[1], h->st));
  const auto w1 = std::chrono::steady_clock::now();
  h->n_divided = keep;
  h->update_rdiv();
  if (keep > 0) h->fill_iota(h->d_und.p, keep, 0);
  h->n_und = keep;
  h->und_fresh = keep > 0;
  h->replay_counts.clear();
  // the consensus log (cleared above) is the replay's order, delivered to the pinned
  // order buffer in one copy (not staged through the arena into the log's vector)
  h->lazy_order = h->pin_ord_cap >= (size_t)keep;
  try {
    h->consensus_batch(h->replay_calls, true, true, true, nullptr, &h->replay_counts);
  } catch (...) {
    h->lazy_order = false;
    throw;
  }
  h->lazy_order = false;
  HIPCHK(hipEventRecord(h->ev[2], h->st));
  HIPCHK(hipEventSynchronize(h->ev[2]));
  const auto w2 = std::chrono::steady_clock::now();
  float a = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&a, h->ev[0], h->ev[1]));
  HIPCHK(hipEventElapsedTime(&b, h->ev[1], h->ev[2]));
  auto ms = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
    return (float)std::chrono::duration<double, std::milli>(y - x).count();
  };
  // [0] coordinates+rounds on the GPU, [1] their wall time, [2] consensus wall time,
  // [3] consensus on the GPU, [4] replay wall time, [5] the order's delivery to host
  // memory (wall, inside [2]), [6] GPU total
  h->stage_ms[0] = a;
  h->stage_ms[1] = ms(h->w_start, w1);
  h->stage_ms[2] = ms(w1, w2);
  h->stage_ms[3] = b;
  h->stage_ms[4] = ms(h->w_start, w2);
  h->stage_ms[6] = a + b;
  if (n_ordered) *n_ordered = h->consensus_size();
  h->dbg_dump();
}

int hge_replay_run(hge_engine* h, int64_t* n_ordered) {
  GUARD_BEGIN
  REFUSE_IF_FAILED(h)
  h->sp_active = false;
  if (h->rec_on) h->rec_dec.clear();
  replay_begin(h);
  replay_end(h, n_ordered);
  if (h->rec_on) {  // hge_split_emulate: the rest of the record
    const int64_t E = h->n_events;
    h->consensus_sync();
    h->rec_order = h->consensus;
    h->rec_counts = h->replay_counts;
    h->rec_rr.resize(E);
    h->rec_cts.resize(E);
    h->readback(h->rec_rr.data(), h->d_rr.p, (size_t)E);
    h->readback(h->rec_cts.data(), h->d_cts.p, (size_t)E);
    h->rec_left.resize(h->n_und);
    if (h->n_und) h->readback(h->rec_left.data(), h->d_und.p, (size_t)h->n_und);
    h->rec_on = false;
    h->rec_have = true;
  }
  return HGE_OK;
  GUARD_END(h)
}

// ---- cross-GPU split of one hashgraph's rounds walk (babble_amd/dist.py) ----
int hge_split_plan(hge_engine* h, int32_t part, int32_t nparts, const int64_t* ev_bounds,
                   const int32_t* call_bounds, const int64_t* cand_lo) {
  if (!h) return HGE_ERR_ARG;
  GUARD_BEGIN
  if (nparts <= 1) {
    h->sp = hge_engine::SplitPlan();
    return HGE_OK;
  }
  auto bad = [&](const char* why) {
    h->err = std::string("hge_split_plan: ") + why;
    return HGE_ERR_ARG;
  };
  if (h->N <= 32 || !h->direct_rounds() || h->wide32 || h->wide32_pending)
    return bad("needs the wide direct rounds path (N > 32, N % 4 == 0, chains below 65,535 events)");
  if (part < 0 || part >= nparts || !ev_bounds || !call_bounds || !cand_lo) return bad("bad argument");
  const int64_t E = h->n_events;
  const int ncalls = (int)h->replay_calls.size();
  if (ev_bounds[0] != 0 || ev_bounds[nparts] != E || call_bounds[0] != 0 || call_bounds[nparts] != ncalls)
    return bad("the bounds must cover the staged stream and its calls");
  for (int g = 0; g < nparts; g++) {
    if (ev_bounds[g + 1] < ev_bounds[g] || call_bounds[g + 1] <= call_bounds[g])
      return bad("bounds must ascend and every part needs a call");
    if (cand_lo[g] < 0 || cand_lo[g] > ev_bounds[g] || cand_lo[g] >= ev_bounds[g + 1])
      return bad("cand_lo[p] must lie in [0, ev_bounds[p]] below ev_bounds[p + 1]");
  }
  if (E > INT32_MAX) return bad("stream too long");
  h->sp.part = part;
  h->sp.nparts = nparts;
  h->sp.a.assign(ev_bounds, ev_bounds + nparts + 1);
  h->sp.cb.assign(call_bounds, call_bounds + nparts + 1);
  h->sp.clo.assign(cand_lo, cand_lo + nparts);
  return HGE_OK;
  GUARD_END(h)
}

int hge_split_exchange(hge_engine* h, hge_exchange_fn fn, void* ctx) {
  if (!h) return HGE_ERR_ARG;
  h->x_fn = fn;
  h->x_ctx = ctx;
  return HGE_OK;
}

int hge_split_emulate(hge_engine* h, int32_t on) {
  if (!h) return HGE_ERR_ARG;
  h->rec_on = on != 0;
  h->rec_have = false;
  h->rec_dec.clear();
  return HGE_OK;
}

int hge_split_run(hge_engine* h, int64_t* n_ordered) {
  if (!h) return HGE_ERR_ARG;
  GUARD_BEGIN
  if (h->sp.nparts <= 1) {
    h->err = "hge_split_run: no split plan (hge_split_plan)";
    return HGE_ERR_ARG;
  }
  if (!h->x_fn && !h->rec_have) {
    h->err = "hge_split_run: no exchange (hge_split_exchange) and no record (hge_split_emulate)";
    return HGE_ERR_ARG;
  }
  struct Off {  // the plan applies to this replay only
    hge_engine* h;
    ~Off() { h->sp_active = false; }
  } off{h};
  h->sp_active = true;
  replay_begin(h);
  replay_end(h, n_ordered);
  return HGE_OK;
  GUARD_END(h)
}

int hge_split_begin(hge_engine* h) {
  GUARD_BEGIN
  if (h->N <= 32 || !h->direct_rounds() || h->wide32 || h->wide32_pending) {
    h->err = "the split walk needs the wide direct rounds path (N > 32, N % 4 == 0)";
    return HGE_ERR_ARG;
  }
  h->sp_active = false;  // the walk-only split: every part computes everything else
  replay_begin(h);
  if (!h->cs_pending) {
    h->err = "nothing staged (hge_replay_prepare first)";
    return HGE_ERR_ARG;
  }
  return HGE_OK;
  GUARD_END(h)
}

int hge_frontier_guess(hge_engine* h, int32_t part, int32_t nparts, int32_t* start_out) {
  if (!h) return HGE_ERR_ARG;
  GUARD_BEGIN
  if (!start_out || nparts < 1 || part < 0 || part >= nparts) {
    h->err = "hge_frontier_guess: bad argument";
    return HGE_ERR_ARG;
  }
  // part 0: the true first frontier (every chain's first event); part p: the time
  // cut at event p * E / nparts (the first event of each chain inserted at or after it)
  // with a split plan of nparts parts: its event bound of the part
  const int64_t T = h->sp.nparts == nparts ? h->sp.a[part] : h->n_events * (int64_t)part / nparts;
  for (int c = 0; c < h->N; c++) {
    const std::vector<int32_t>& ch = h->h_chain[c];
    const size_t k = std::lower_bound(ch.begin(), ch.end(), (int32_t)T) - ch.begin();
    start_out[c] = k < ch.size() ? (int32_t)k : INF32;
  }
  return HGE_OK;
  GUARD_END(h)
}

int hge_frontier_walk(hge_engine* h, const int32_t* start, const int32_t* stopcut, int32_t extra,
                      int32_t hmax, int32_t* rows_out, uint64_t* ssc_out, int32_t* nrows,
                      int32_t* natural) {
  GUARD_BEGIN
  if (!h->cs_pending || !start || hmax < 2) return HGE_ERR_ARG;
  const int N = h->N, NW = h->NW;
  h->s_hist.need((size_t)hmax * N + N);
  h->s_hssc.need((size_t)hmax * N * NW);
  h->s_hstate.need(N + 4);
  h->h2d(h->s_hstate.p, start, 4 * (size_t)N);
  int32_t* cut = nullptr;
  if (stopcut) {
    h->s_hist.need((size_t)hmax * N + 2 * N);
    cut = h->s_hist.p + (size_t)hmax * N + N;
    h->h2d(cut, stopcut, 4 * (size_t)N);
  }
  int32_t* rstate = h->s_hstate.p + N;
  HIPCHK(hipMemsetAsync(rstate, 0, 16, h->st));
  h->s_bar.need(2);
  h->s_gran.need(2 * (size_t)N);
  HIPCHK(hipMemsetAsync(h->s_bar.p, 0, 8, h->st));
  HIPCHK(hipMemsetAsync(h->s_gran.p, 0, 16 * (size_t)N, h->st));
  const int npow = N <= 64 ? 64 : N <= 128 ? 128 : 256;
  h->s_mb.need((size_t)npow * npow);
  auto lk = h->frontier_lock();  // until the walk has drained (the sync below)
  Tables t = h->tables();
  const int32_t* olen = h->k_len;
  const int32_t* len = h->k_len + N;
  int rlo = 0, Rprev = 0;
  const int32_t* rlo_dev = nullptr;
  uint64_t* gran = h->s_gran.p;
  int32_t* err = h->s_bar.p + 1;
  uint64_t* ssc = h->s_hssc.p;
  uint32_t* mb = h->s_mb.p;
  uint64_t* dbg = nullptr;
  const int32_t* st0 = h->s_hstate.p;
  int32_t* hist = h->s_hist.p;
  int hm = hmax, ex = std::max(0, (int)extra), nostall = 0;
  void* args[] = {&t, &olen, &len, &rstate, &rlo, &rlo_dev, &Rprev, &gran, &err, &ssc, &mb, &dbg,
                  &st0, &hist, &hm, &cut, &ex, &nostall};
  const void* fn = N <= 64 ? (const void*)k_rounds_direct<1024, 64>
                 : N <= 128 ? (const void*)k_rounds_direct<1024, 128>
                            : (const void*)k_rounds_direct<1024, 256>;
  h->prof_begin("k_rounds_direct_walk");
  HIPCHK(h->launch_resident(fn, dim3(N), dim3(1024), args));
  h->prof_end();
  int32_t rs[2] = {0, 0}, e = 0;
  h->d2h(rs, rstate, 8);
  h->d2h(&e, err, 4);
  h->sync();
  if (e) throw EngineError(HGE_ERR_DEVICE, "rounds frontier hand-off timed out");
  const int n = std::max(1, std::min(rs[0], hmax));
  if (rows_out) h->readback(rows_out, h->s_hist.p, (size_t)n * N);
  if (ssc_out) h->readback(ssc_out, h->s_hssc.p, (size_t)n * N * NW);
  if (nrows) *nrows = n;
  if (natural) *natural = rs[1] == 0 ? 1 : 0;
  return HGE_OK;
  GUARD_END(h)
}

int hge_frontier_rows(hge_engine* h, int32_t from, int32_t n, int32_t* rows_out, uint64_t* ssc_out) {
  GUARD_BEGIN
  const int N = h->N, NW = h->NW;
  if (from < 0 || n < 0 || (size_t)(from + n) * N > h->s_hist.n) return HGE_ERR_ARG;
  if (rows_out && n) h->d2h(rows_out, h->s_hist.p + (size_t)from * N, 4 * (size_t)n * N);
  if (ssc_out && n) h->d2h(ssc_out, h->s_hssc.p + (size_t)from * N * NW, 8 * (size_t)n * N * NW);
  h->sync();
  return HGE_OK;
  GUARD_END(h)
}

int hge_split_finish(hge_engine* h, const int32_t* rows, const uint64_t* ssc, int32_t nrows,
                     int32_t natural, int64_t* n_ordered) {
  GUARD_BEGIN
  if (!h->cs_pending || !rows || nrows < 1 || (nrows > 1 && !ssc)) return HGE_ERR_ARG;
  const int N = h->N, NW = h->NW;
  h->ext_on = true;
  h->ext_natural = natural != 0;
  h->ext_rows = nrows;
  h->ext_C.assign(rows, rows + (size_t)nrows * N);
  h->ext_ssc.assign((size_t)nrows * N * NW, 0);
  if (nrows > 1) std::copy(ssc + (size_t)N * NW, ssc + (size_t)nrows * N * NW, h->ext_ssc.begin() + (size_t)N * NW);
  replay_end(h, n_ordered);
  return HGE_OK;
  GUARD_END(h)
}

int hge_replay_fetch(hge_engine* h, int32_t* order_out, int64_t cap, int64_t* call_counts_out) {
  GUARD_BEGIN
  if (order_out) {
    // the log's vector, then the delivered tail in the pinned buffer: one copy each
    const int64_t a = std::min<int64_t>((int64_t)h->consensus.size(), std::max<int64_t>(cap, 0));
    if (a > 0) memcpy(order_out, h->consensus.data(), 4 * (size_t)a);
    const int64_t b = std::min<int64_t>(h->cons_pin_n, std::max<int64_t>(cap - a, 0));
    // (one copy thread moves ~12 GB/s: a 40 MB order takes 8 in parallel)
    const int nt = b >= (1 << 20) ? 8 : 1;
    std::vector<std::thread> th;
    for (int k = 1; k < nt; k++)
      th.emplace_back([=] {
        const int64_t lo = b * k / nt, hi = b * (k + 1) / nt;
        memcpy(order_out + a + lo, h->pin_ord + lo, 4 * (size_t)(hi - lo));
      });
    if (b > 0) memcpy(order_out + a, h->pin_ord, 4 * (size_t)(b / nt));
    for (auto& x : th) x.join();
  }
  if (call_counts_out)
    for (size_t c = 0; c < h->replay_counts.size(); c++) call_counts_out[c] = h->replay_counts[c];
  return HGE_OK;
  GUARD_END(h)
}

int hge_replay_order(hge_engine* h, const int32_t** ids, int64_t* n) {
  if (!h || !ids || !n) return HGE_ERR_ARG;
  GUARD_BEGIN
  if (!h->consensus.empty() || !h->cons_pin_n) h->consensus_sync();  // the whole log in one place
  if (h->cons_pin_n) {
    *ids = h->pin_ord;
    *n = h->cons_pin_n;
  } else {
    *ids = h->consensus.data();
    *n = (int64_t)h->consensus.size();
  }
  return HGE_OK;
  GUARD_END(h)
}

int hge_replay(hge_engine* h, const hge_event* ev, int64_t n_sub, const int64_t* call_points,
               int64_t n_calls, int32_t* status_out, int32_t* order_out, int64_t cap,
               int64_t* n_ordered, int64_t* call_counts_out) {
  int rc = hge_replay_prepare(h, ev, n_sub, call_points, n_calls, status_out);
  if (rc) return rc;
  rc = hge_replay_run(h, n_ordered);
  if (rc) return rc;
  return hge_replay_fetch(h, order_out, cap, call_counts_out);
}

int64_t hge_event_count(hge_engine* h) { return h->n_events; }
int32_t hge_participants(hge_engine* h) { return h->N; }
int32_t hge_rounds(hge_engine* h) { return std::max(h->R_div, h->R_set); }
int32_t hge_last_consensus_round(hge_engine* h) { return h->lcr; }
int32_t hge_last_committed_round_events(hge_engine* h) { return h->lcre; }
int64_t hge_consensus_transactions(hge_engine* h) { return h->ctx; }
int64_t hge_consensus_count(hge_engine* h) { return h->consensus_size(); }
// RollingList window (common/rolling_list.go:55-67): Add rolls the list back to
// its last `size` items once it holds 2*size, so after `tot` adds it holds
static int64_t window_len(int64_t tot, int64_t size) {
  if (size <= 0 || tot <= 2 * size) return tot;
  return size + (tot - 2 * size - 1) % size + 1;
}
int64_t hge_consensus_events(hge_engine* h, int32_t* ids_out, int64_t cap) {
  try {
    h->consensus_sync();
  } catch (const EngineError& e) {
    h->err = e.msg;
    return -1;
  }
  const int64_t tot = (int64_t)h->consensus.size(), w = window_len(tot, h->cache_size);
  for (int64_t i = 0; i < w && i < cap && ids_out; i++) ids_out[i] = h->consensus[tot - w + i];
  return w;
}
int64_t hge_consensus_log(hge_engine* h, int64_t from, int32_t* ids_out, int64_t cap) {
  try {
    h->consensus_sync();
  } catch (const EngineError& e) {
    h->err = e.msg;
    return -1;
  }
  const int64_t tot = (int64_t)h->consensus.size();
  if (from < 0) from = 0;
  for (int64_t i = from; i < tot && i - from < cap && ids_out; i++) ids_out[i - from] = h->consensus[i];
  return std::max<int64_t>(0, tot - from);
}
int64_t hge_undetermined(hge_engine* h, int32_t* ids_out, int64_t cap) {
  try {
    if (ids_out && h->n_und > 0) {
      int64_t m = std::min<int64_t>(cap, h->n_und);
      h->readback(ids_out, h->d_und.p, m);
    }
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
  return h->n_und;
}
int hge_known(hge_engine* h, int32_t* counts_out) {
  for (int c = 0; c < h->N; c++) counts_out[c] = h->chain_len[c];
  return HGE_OK;
}

static int32_t read1(hge_engine* h, const int32_t* p) {
  int32_t v = -1;
  h->readback(&v, p, 1);
  return v;
}

int32_t hge_round_of(hge_engine* h, int32_t id) {
  try {
    if (id < 0 || id >= h->n_events) return -1;
    h->coords();
    return read1(h, h->d_round.p + id);
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
int32_t hge_is_witness(hge_engine* h, int32_t id) {
  try {
    if (id < 0 || id >= h->n_events) return 0;
    h->coords();
    uint8_t v = 0;
    h->readback(&v, h->d_wit.p + id, 1);
    return v;
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
int32_t hge_round_witness(hge_engine* h, int32_t round, int32_t creator) {
  try {
    if (round < 0 || round >= h->R || creator < 0 || creator >= h->N) return -1;
    int32_t w = read1(h, h->d_W.p + (size_t)round * h->N + creator);
    if (w >= h->n_divided) return -1;
    return w;
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
int32_t hge_fame(hge_engine* h, int32_t round, int32_t creator) {
  try {
    if (hge_round_witness(h, round, creator) < 0) return -1;
    uint8_t v = 0;
    h->readback(&v, h->d_fame.p + (size_t)round * h->N + creator, 1);
    return v;
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
int32_t hge_round_events(hge_engine* h, int32_t round) {
  try {
    if (round < 0 || round >= h->R) return 0;
    return read1(h, h->d_rcnt.p + round);
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
// Store.GetRound's events (RoundInfo.Events, roundInfo.go:24-60): every event of
// round r in insertion order with its witness flag (the first event of round r is
// its first witness: ids below h_minw[r] are not scanned)
int hge_round_event_ids(hge_engine* h, int32_t round, int32_t* ids_out, uint8_t* witness_out, int64_t cap,
                        int64_t* n_out) {
  if (!h || !n_out) return HGE_ERR_ARG;
  GUARD_BEGIN
  *n_out = 0;
  h->coords();
  if (round < 0 || round >= h->R || h->n_coords == 0) return HGE_OK;
  const int64_t lo = round < (int)h->h_minw.size() ? std::max<int64_t>(0, h->h_minw[round]) : 0;
  const int64_t n = h->n_coords - lo;
  if (n <= 0) return HGE_OK;
  std::vector<int32_t> rd((size_t)n);
  std::vector<uint8_t> wd((size_t)n);
  h->d2h(rd.data(), h->d_round.p + lo, 4 * (size_t)n);
  h->d2h(wd.data(), h->d_wit.p + lo, (size_t)n);
  h->sync();
  int64_t k = 0;
  for (int64_t i = 0; i < n; i++) {
    if (rd[(size_t)i] != round) continue;
    if (k < cap) {
      if (ids_out) ids_out[k] = (int32_t)(lo + i);
      if (witness_out) witness_out[k] = wd[(size_t)i];
    }
    k++;
  }
  *n_out = k;
  return HGE_OK;
  GUARD_END(h)
}

int32_t hge_round_received(hge_engine* h, int32_t id) {
  try {
    if (id < 0 || id >= h->n_events) return -1;
    return read1(h, h->d_rr.p + id);
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}
int64_t hge_consensus_timestamp(hge_engine* h, int32_t id) {
  try {
    if (id < 0 || id >= h->n_events) return 0;
    int64_t v = 0;
    h->readback(&v, h->d_cts.p + id, 1);
    return v;
  } catch (EngineError& e) {
    h->err = e.msg;
    return e.code;
  }
}

int hge_coordinates(hge_engine* h, int32_t id, int32_t* la_out, int32_t* fd_out) {
  GUARD_BEGIN
  if (id < 0 || id >= h->n_events) return HGE_ERR_ARG;
  h->coords();
  const size_t off = ((size_t)h->h_creator[id] * h->ccap + h->h_index[id]) * h->N;
  if (la_out) {
    if (h->sweep16()) {  // N > 32: unpack the LA16 row (LA + 1 as uint16 pairs)
      const size_t w = (size_t)(h->N + 1) / 2;
      std::vector<uint32_t> row(w);
      h->readback(row.data(), h->d_LA16.p + ((size_t)h->h_creator[id] * h->ccap + h->h_index[id]) * w, w);
      for (int c = 0; c < h->N; c++) la_out[c] = (int32_t)((row[c >> 1] >> ((c & 1) * 16)) & 0xFFFFu) - 1;
    } else {
      h->readback(la_out, h->d_LA.p + off, h->N);
    }
  }
  if (fd_out && h->fdt16()) {  // packed rows: FD + 1, 0xFFFF = none
    std::vector<uint16_t> row(h->N);
    h->readback(row.data(), (const uint16_t*)h->d_FD.p + off, h->N);
    for (int c = 0; c < h->N; c++) fd_out[c] = row[c] == 0xFFFFu ? INF32 : (int32_t)row[c] - 1;
    return HGE_OK;
  }
  if (fd_out) h->readback(fd_out, h->d_FD.p + off, h->N);
  return HGE_OK;
  GUARD_END(h)
}

// predicates on the materialised coordinates (hashgraph.go:83-208)
int32_t hge_ancestor(hge_engine* h, int32_t x, int32_t y) {
  if (x < 0 || x >= h->n_events || y < 0 || y >= h->n_events) return 0;
  if (x == y) return 1;
  std::vector<int32_t> la(h->N);
  if (hge_coordinates(h, x, la.data(), nullptr)) return 0;
  return la[h->h_creator[y]] >= h->h_index[y] ? 1 : 0;
}
int32_t hge_self_ancestor(hge_engine* h, int32_t x, int32_t y) {
  if (x < 0 || x >= h->n_events || y < 0 || y >= h->n_events) return 0;
  if (x == y) return 1;
  return (h->h_creator[x] == h->h_creator[y] && h->h_index[x] >= h->h_index[y]) ? 1 : 0;
}
int32_t hge_see(hge_engine* h, int32_t x, int32_t y) { return hge_ancestor(h, x, y); }
int32_t hge_strongly_see(hge_engine* h, int32_t x, int32_t y) {
  if (x < 0 || x >= h->n_events || y < 0 || y >= h->n_events) return 0;
  std::vector<int32_t> la(h->N), fd(h->N);
  if (hge_coordinates(h, x, la.data(), nullptr)) return 0;
  if (hge_coordinates(h, y, nullptr, fd.data())) return 0;
  int c = 0;
  for (int i = 0; i < h->N; i++) c += la[i] >= fd[i];
  return c >= h->SM ? 1 : 0;
}
int32_t hge_oldest_self_ancestor_to_see(hge_engine* h, int32_t x, int32_t y) {
  if (x < 0 || x >= h->n_events || y < 0 || y >= h->n_events) return -1;
  std::vector<int32_t> fd(h->N);
  if (hge_coordinates(h, y, nullptr, fd.data())) return -1;
  const int cx = h->h_creator[x];
  const int32_t a = fd[cx];
  if (a <= h->h_index[x]) {
    try {
      return read1(h, h->d_chain.p + (size_t)cx * h->ccap + a);
    } catch (EngineError& e) {
      h->err = e.msg;
      return -1;
    }
  }
  return -1;
}

// ---- Store semantics and sync-path reads ----------------------------------
int hge_set_cache_size(hge_engine* h, int64_t size) {
  if (!h || size < 0) return HGE_ERR_ARG;
  h->cache_size = size;
  return HGE_OK;
}
int64_t hge_cache_size(hge_engine* h) { return h->cache_size; }

int hge_participant_events(hge_engine* h, int32_t creator, int64_t skip, int32_t* ids_out,
                           int64_t cap, int64_t* n_out) {
  if (n_out) *n_out = 0;
  if (creator < 0 || creator >= h->N) {
    h->err = "not found";
    return HGE_ERR_NOT_FOUND;
  }
  const std::vector<int32_t>& ch = h->h_chain[creator];
  const int64_t tot = (int64_t)ch.size();
  if (skip >= tot) return HGE_OK;
  const int64_t oldest = tot - window_len(tot, h->cache_size);
  if (skip < oldest) {
    h->err = "too late";
    return HGE_ERR_TOO_LATE;
  }
  if (skip < 0) skip = 0;
  for (int64_t k = skip; k < tot && k - skip < cap && ids_out; k++) ids_out[k - skip] = ch[k];
  if (n_out) *n_out = tot - skip;
  return HGE_OK;
}

int32_t hge_participant_event(hge_engine* h, int32_t creator, int64_t index) {
  if (!h || creator < 0 || creator >= h->N) return HGE_ERR_NOT_FOUND;
  const std::vector<int32_t>& ch = h->h_chain[creator];
  const int64_t tot = (int64_t)ch.size();
  // RollingList.GetItem (common/rolling_list.go:42-53): index < oldestCached (>= 0),
  // a negative index included, is ErrTooLate
  if (index < 0 || index < tot - window_len(tot, h->cache_size)) return HGE_ERR_TOO_LATE;
  if (index >= tot) return HGE_ERR_NOT_FOUND;
  return ch[index];
}

int32_t hge_last_from(hge_engine* h, int32_t creator) {
  if (creator < 0 || creator >= h->N) return HGE_ERR_NOT_FOUND;
  return h->chain_last[creator];
}

int hge_diff(hge_engine* h, const int32_t* known, int32_t* ids_out, int64_t cap, int64_t* n_out) {
  if (n_out) *n_out = 0;
  if (!known) return HGE_ERR_ARG;
  std::vector<int32_t> ids;
  for (int c = 0; c < h->N; c++) {
    const std::vector<int32_t>& ch = h->h_chain[c];
    const int64_t tot = (int64_t)ch.size(), skip = known[c];
    if (skip >= tot) continue;
    if (skip < tot - window_len(tot, h->cache_size)) {
      h->err = "too late";
      return HGE_ERR_TOO_LATE;
    }
    for (int64_t k = std::max<int64_t>(skip, 0); k < tot; k++) ids.push_back(ch[k]);
  }
  std::sort(ids.begin(), ids.end());  // ByTopologicalOrder: ids are insertion order
  for (int64_t i = 0; i < (int64_t)ids.size() && i < cap && ids_out; i++) ids_out[i] = ids[i];
  if (n_out) *n_out = (int64_t)ids.size();
  return HGE_OK;
}

int hge_wire_info(hge_engine* h, int32_t id, int32_t* out) {
  if (id < 0 || id >= h->n_events || !out) return HGE_ERR_ARG;
  const int32_t sp = h->h_sp[id], op = h->h_op[id];
  out[0] = sp >= 0 ? h->h_index[sp] : -1;
  out[1] = op >= 0 ? h->h_creator[op] : -1;
  out[2] = op >= 0 ? h->h_index[op] : -1;
  out[3] = h->h_creator[id];
  return HGE_OK;
}

int hge_read_wire_parents(hge_engine* h, int32_t creator_id, int32_t self_parent_index,
                          int32_t other_parent_creator_id, int32_t other_parent_index,
                          int32_t* sp_out, int32_t* op_out) {
  if (creator_id < 0 || creator_id >= h->N) return HGE_ERR_NOT_FOUND;
  int32_t sp = HGE_NONE, op = HGE_NONE;
  if (self_parent_index >= 0) {
    sp = hge_participant_event(h, creator_id, self_parent_index);
    if (sp < 0) return sp;
  }
  if (other_parent_index >= 0) {
    op = hge_participant_event(h, other_parent_creator_id, other_parent_index);
    if (op < 0) return op;
  }
  if (sp_out) *sp_out = sp;
  if (op_out) *op_out = op;
  return HGE_OK;
}

// ---- bulk state reads ------------------------------------------------------
int hge_event_rounds(hge_engine* h, int32_t* round_out, uint8_t* witness_out, int64_t cap) {
  GUARD_BEGIN
  h->coords();
  const int64_t m = std::min<int64_t>(cap, h->n_events);
  if (m > 0 && round_out) h->d2h(round_out, h->d_round.p, 4 * (size_t)m);
  if (m > 0 && witness_out) h->d2h(witness_out, h->d_wit.p, (size_t)m);
  h->sync();
  return HGE_OK;
  GUARD_END(h)
}

int hge_event_received(hge_engine* h, int32_t* rr_out, int64_t* cts_out, int64_t cap) {
  GUARD_BEGIN
  const int64_t m = std::min<int64_t>(cap, h->n_events);
  if (m > 0 && rr_out) h->d2h(rr_out, h->d_rr.p, 4 * (size_t)m);
  if (m > 0 && cts_out) h->d2h(cts_out, h->d_cts.p, 8 * (size_t)m);
  h->sync();
  return HGE_OK;
  GUARD_END(h)
}

int hge_consensus_timestamp_sources(hge_engine* h, const int32_t* ids, int64_t n, int32_t* src_out) {
  if (!h || n < 0 || (n > 0 && (!ids || !src_out))) return HGE_ERR_ARG;
  GUARD_BEGIN
  if (n == 0) return HGE_OK;
  for (int64_t i = 0; i < n; i++)
    if (ids[i] < 0 || ids[i] >= h->n_events) throw EngineError(HGE_ERR_ARG, "hge_consensus_timestamp_sources: unknown id");
  h->s_src.need((size_t)n * 2);
  h->h2d(h->s_src.p, ids, 4 * (size_t)n);
  hipLaunchKernelGGL(k_cts_source, dim3((unsigned)div_up(n, 4)), dim3(256), 0, h->st, h->tables(),
                     (const int32_t*)h->s_src.p, (int)n, (const int32_t*)h->d_rr.p, (const int64_t*)h->d_cts.p,
                     h->s_src.p + n);
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) throw EngineError(HGE_ERR_DEVICE, std::string("launch k_cts_source: ") + hipGetErrorString(le));
  h->readback(src_out, h->s_src.p + n, (size_t)n);
  return HGE_OK;
  GUARD_END(h)
}

int32_t hge_fame_table(hge_engine* h, int32_t rounds, int8_t* fame_out) {
  if (!h) return HGE_ERR_ARG;
  GUARD_BEGIN
  const int R = std::min<int>(std::max(rounds, 0), std::min(h->R, h->Rcap));
  if (R == 0 || !fame_out) return 0;
  const size_t n = (size_t)R * h->N;
  std::vector<int32_t> w(n);
  std::vector<uint8_t> f(n);
  h->d2h(w.data(), h->d_W.p, 4 * n);
  h->d2h(f.data(), h->d_fame.p, n);
  h->sync();
  for (size_t i = 0; i < n; i++)
    fame_out[i] = (w[i] >= 0 && w[i] < h->n_divided) ? (int8_t)f[i] : (int8_t)-1;
  return R;
  GUARD_END(h)
}

// ---- round predicates (hashgraph.go:211-326) --------------------------------
int32_t hge_parent_round(hge_engine* h, int32_t x) {
  if (x < 0 || x >= h->n_events) return -1;
  const int32_t sp = h->h_sp[x], op = h->h_op[x];
  if (sp < 0 && op < 0) return 0;
  if (sp < 0 || op < 0) return 0;  // a missing parent (GetEvent error) reads as 0
  const int32_t a = hge_round_of(h, sp), b = hge_round_of(h, op);
  return std::max(a, b);
}

int32_t hge_round_inc(hge_engine* h, int32_t x) {
  if (x < 0 || x >= h->n_events) return 0;
  const int32_t pr = hge_parent_round(h, x);
  if (pr < 0 || hge_rounds(h) < pr + 1) return 0;
  try {
    h->coords();
    if (pr >= h->Rcap) return 0;
    std::vector<int32_t> w(h->N);
    h->readback(w.data(), h->d_W.p + (size_t)pr * h->N, h->N);
    int c = 0;
    for (int i = 0; i < h->N; i++)
      if (w[i] >= 0 && w[i] < h->n_events) c += hge_strongly_see(h, x, w[i]);
    return c >= h->SM ? 1 : 0;
  } catch (EngineError& e) {
    h->err = e.msg;
    return 0;
  }
}

int hge_round_diff(hge_engine* h, int32_t x, int32_t y, int32_t* out) {
  if (x < 0 || x >= h->n_events || y < 0 || y >= h->n_events || !out) return HGE_ERR_ARG;
  const int32_t a = hge_round_of(h, x), b = hge_round_of(h, y);
  if (a < 0 || b < 0) return HGE_ERR_INTERNAL;
  *out = a - b;
  return HGE_OK;
}

int hge_set_round(hge_engine* h, int32_t round, const int32_t* ids, const uint8_t* witness,
                  const uint8_t* fame, int32_t n) {
  GUARD_BEGIN
  if (round < 0 || n < 0 || (n > 0 && !ids)) return HGE_ERR_ARG;
  h->coords();
  h->ensure_rcap((int64_t)round + 1);
  for (int32_t i = 0; i < n; i++) {
    const int32_t x = ids[i];
    if (x < 0 || x >= h->n_events) return HGE_ERR_ARG;
    if (witness && !witness[i]) continue;
    const size_t slot = (size_t)round * h->N + h->h_creator[x];
    h->h2d(h->d_W.p + slot, &ids[i], 4);
    const uint8_t f = fame ? fame[i] : 0;
    h->h2d(h->d_fame.p + slot, &f, 1);
    h->sync();
  }
  h->R_set = std::max(h->R_set, round + 1);
  return HGE_OK;
  GUARD_END(h)
}

int hge_set_profiling(hge_engine* h, int on) {
  h->prof_on = on != 0;
  return HGE_OK;
}

int hge_reset_kernel_stats(hge_engine* h) {
  h->prof_names.clear();
  h->prof_ms.clear();
  h->prof_cnt.clear();
  return HGE_OK;
}

int hge_kernel_stats(hge_engine* h, int k, char* name, int namecap, double* total_ms,
                     int64_t* launches) {
  const int n = (int)h->prof_names.size();
  if (k < 0 || k >= n) return n;
  if (name && namecap > 0) {
    snprintf(name, namecap, "%s", h->prof_names[k].c_str());
  }
  if (total_ms) *total_ms = h->prof_ms[k];
  if (launches) *launches = h->prof_cnt[k];
  return n;
}

int32_t hge_coordinate_sweeps(hge_engine* h) { return h ? h->n_sweeps : -1; }

int64_t hge_host_syncs(hge_engine* h) { return h ? h->n_syncs : -1; }

int hge_stage_times(hge_engine* h, float* ms_out, int cap) {
  int n = std::min(cap, 7);
  for (int i = 0; i < n; i++) ms_out[i] = h->stage_ms[i];
  return n;
}

int64_t hge_frontier_fallbacks(hge_engine* h) {
  if (!h) return HGE_ERR_ARG;
  return h->n_frontier_fallbacks;
}

}  // extern "C"
