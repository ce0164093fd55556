// C++ test binary for the engine's C ABI (include/hge.h), linked against
// build/libhge.so the way a cgo shim links it (no Python, no torch).
//
//   hge_abi_test            checks that need no GPU: argument errors of
//                           hge_create and the null-handle paths.
//   hge_abi_test --gpu      the reference's consensus DAG (hashgraph_test.go:
//                           835-950, initConsensusHashgraph) through
//                           hge_insert_events + hge_run_consensus, with the
//                           answers of TestDecideFame / TestFindOrder / TestKnown
//                           (hashgraph_test.go:952-1070) and node_test.go's
//                           TestStats, plus the Store views (ParticipantEvents,
//                           Diff, wire info) and hge_replay's identical result.
// Exit status 0 = all checks passed.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "hge.h"

static int failures = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);    \
      failures++;                                                          \
    }                                                                      \
  } while (0)

// (name, creator, self-parent name, other-parent name): initConsensusHashgraph
struct Def {
  const char* name;
  int creator;
  const char* sp;
  const char* op;
};
static const Def kDag[] = {
    {"e0", 0, "", ""},       {"e1", 1, "", ""},       {"e2", 2, "", ""},
    {"e10", 1, "e1", "e0"},  {"e21", 2, "e2", "e10"}, {"e02", 0, "e0", "e21"},
    {"f1", 1, "e10", "e02"}, {"f0", 0, "e02", "f1"},  {"f2", 2, "e21", "f1"},
    {"f10", 1, "f1", "f0"},  {"f21", 2, "f2", "f10"}, {"f02", 0, "f0", "f21"},
    {"g1", 1, "f10", "f02"}, {"g0", 0, "f02", "g1"},  {"g2", 2, "f21", "g1"},
    {"g10", 1, "g1", "g0"},  {"g21", 2, "g2", "g10"}, {"g02", 0, "g0", "g21"},
    {"h1", 1, "g10", "g02"}, {"h0", 0, "g02", "h1"},  {"h2", 2, "g21", "h1"},
};
static const int kE = sizeof(kDag) / sizeof(kDag[0]);

static int find(const char* nm) {
  if (!nm[0]) return HGE_NONE;
  for (int i = 0; i < kE; i++)
    if (!strcmp(kDag[i].name, nm)) return i;
  return HGE_UNKNOWN;
}

// fixed synthetic bytes (the reference draws them from crypto/rand)
static void fill_event(hge_event& e, int i) {
  static int seq[3] = {0, 0, 0};
  memset(&e, 0, sizeof(e));
  e.creator = kDag[i].creator;
  e.index = seq[e.creator]++;
  e.self_parent = find(kDag[i].sp);
  e.other_parent = find(kDag[i].op);
  e.timestamp_ns = 1500000000000000000LL + 1000LL * i;
  const int rank[] = {0, 1, 3, 2, 4, 5};  // e0 e1 e2 e10 e21 e02 -> S rank
  e.s[0] = (uint8_t)(i < 6 ? rank[i] : 10 + i);
  for (int b = 0; b < 32; b++) e.hash[b] = (uint8_t)(i * 7 + b + 1);
  e.n_tx = (i >= 3 && i < 6) ? 1 : 0;
}

static int no_gpu_checks() {
  hge_engine* h = nullptr;
  CHECK(hge_create(0, 16, 0, 0, &h) == HGE_ERR_ARG);
  CHECK(h == nullptr);
  CHECK(hge_create(257, 16, 0, 0, &h) == HGE_ERR_ARG);
  CHECK(hge_create(4, 16, 0, 0, nullptr) == HGE_ERR_ARG);
  CHECK(std::string(hge_last_error(nullptr)) == "null handle");
  hge_destroy(nullptr);  // no-op
  return failures;
}

static int gpu_checks() {
  hge_engine* h = nullptr;
  CHECK(hge_create(3, 64, 0, 0, &h) == HGE_OK);
  if (!h) return ++failures;
  std::vector<hge_event> ev(kE);
  for (int i = 0; i < kE; i++) fill_event(ev[i], i);
  std::vector<int32_t> status(kE, -99);
  int64_t acc = 0;
  CHECK(hge_insert_events(h, ev.data(), kE, status.data(), &acc) == HGE_OK);
  CHECK(acc == kE);
  for (int i = 0; i < kE; i++) CHECK(status[i] == i);
  // a fork (second child of e1) is refused and nothing is inserted
  hge_event fork = ev[3];
  fork.timestamp_ns += 1;
  int32_t st = 0;
  CHECK(hge_insert_events(h, &fork, 1, &st, &acc) == HGE_ERR_SELF_PARENT_NOT_LAST);
  CHECK(acc == 0 && st == HGE_ERR_SELF_PARENT_NOT_LAST);
  CHECK(hge_event_count(h) == kE);

  std::vector<int32_t> ids(kE);
  int64_t n = 0;
  CHECK(hge_run_consensus(h, ids.data(), kE, &n) == HGE_OK);
  // TestFindOrder (hashgraph_test.go:1019-1047): the S tie-break is random there, so
  // positions accept {e0}, {e10, e1}, {e1, e10}, {e21, e2}, {e2, e21}, {e02}
  const char* w1[] = {"e0", "e10", "e1", "e21", "e2", "e02"};
  const char* w2[] = {"e0", "e1", "e10", "e2", "e21", "e02"};
  CHECK(n == 6);
  for (int k = 0; k < n && k < 6; k++) CHECK(ids[k] == find(w1[k]) || ids[k] == find(w2[k]));
  CHECK(hge_rounds(h) == 4);                        // TestDivideRounds on this DAG
  for (int c = 0; c < 3; c++) CHECK(hge_fame(h, 0, c) == 1);  // TestDecideFame
  CHECK(hge_round_of(h, find("g0")) == 2);
  CHECK(hge_last_consensus_round(h) == 1);          // TestStats
  CHECK(hge_consensus_count(h) == 6);
  CHECK(hge_consensus_transactions(h) == 3);
  CHECK(hge_undetermined(h, nullptr, 0) == 15);
  int32_t known[3];
  CHECK(hge_known(h, known) == HGE_OK);
  CHECK(known[0] == 7 && known[1] == 7 && known[2] == 7);  // TestKnown
  // Store views and the sync path
  std::vector<int32_t> pe(8);
  int64_t m = 0;
  CHECK(hge_participant_events(h, 1, 5, pe.data(), 8, &m) == HGE_OK);
  CHECK(m == 2 && pe[0] == find("g10") && pe[1] == find("h1"));
  CHECK(hge_last_from(h, 2) == find("h2"));
  const int32_t k2[3] = {6, 7, 5};
  CHECK(hge_diff(h, k2, pe.data(), 8, &m) == HGE_OK);
  CHECK(m == 3 && pe[0] == find("g21") && pe[1] == find("h0") && pe[2] == find("h2"));
  int32_t wi[4];
  CHECK(hge_wire_info(h, find("f1"), wi) == HGE_OK);
  CHECK(wi[0] == 1 && wi[1] == 0 && wi[2] == 1 && wi[3] == 1);  // TestInsertEvent wire info
  int32_t sp = -9, op = -9;
  CHECK(hge_read_wire_parents(h, wi[3], wi[0], wi[1], wi[2], &sp, &op) == HGE_OK);
  CHECK(sp == find("e10") && op == find("e02"));
  CHECK(hge_set_cache_size(h, 2) == HGE_OK);          // window of 2..4 items
  CHECK(hge_participant_events(h, 0, 0, pe.data(), 8, &m) == HGE_ERR_TOO_LATE);
  // the bulk replay of the same stream (one call) gives the same order
  hge_engine* r = nullptr;
  CHECK(hge_create(3, 64, 0, 0, &r) == HGE_OK);
  if (r) {
    const int64_t calls[1] = {kE};
    int64_t nord = 0, cc[1] = {0};
    std::vector<int32_t> ord(kE), rst(kE);
    CHECK(hge_replay(r, ev.data(), kE, calls, 1, rst.data(), ord.data(), kE, &nord, cc) == HGE_OK);
    CHECK(nord == 6 && cc[0] == 6);
    for (int k = 0; k < 6; k++) CHECK(ord[k] == ids[k]);
    const int64_t bad[2] = {5, 5};
    CHECK(hge_replay(r, ev.data(), kE, bad, 2, rst.data(), ord.data(), kE, &nord, cc) == HGE_ERR_ARG);
    hge_destroy(r);
  }
  hge_destroy(h);
  return failures;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && !strcmp(argv[1], "--gpu");
  no_gpu_checks();
  if (gpu) gpu_checks();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("hge_abi_test: all %s checks passed\n", gpu ? "CPU and GPU" : "CPU");
  return 0;
}
