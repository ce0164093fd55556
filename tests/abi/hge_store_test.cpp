// The standalone Store through the C ABI (include/hge.h), host only: the
// reference's store tests restated with int64 keys for event hashes.
//   TestInmemEvents            hashgraph/inmem_store_test.go:48-119
//   TestInmemRounds            hashgraph/inmem_store_test.go:121-159
//   TestParticipantEventsCache hashgraph/caches_test.go:22-90
//   TestParticipantEventsCacheEdge caches_test.go:92-131
//   RollingList / LRU semantics common/rolling_list_test.go, common/lru_test.go
// Prints "ok <n>" and exits 0, or names the first failed check and exits 1.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#include "hge.h"

static int checks = 0;
#define CHECK(cond)                                                     \
  do {                                                                  \
    checks++;                                                           \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

static std::vector<int64_t> pevents(hge_store* s, int c, int64_t skip, int* rc) {
  int64_t n = 0;
  *rc = hge_store_participant_events(s, c, skip, nullptr, 0, &n);
  std::vector<int64_t> v((size_t)n);
  if (*rc == HGE_OK && n) *rc = hge_store_participant_events(s, c, skip, v.data(), n, &n);
  return v;
}

// key of participant p's k-th event (stands for the reference's event hash)
static int64_t key(int p, int k) { return (int64_t)p * 1000 + k; }

static void inmem_events() {
  const int cacheSize = 100, testSize = 15, n = 3;
  hge_store* s = nullptr;
  CHECK(hge_store_create(n, cacheSize, &s) == HGE_OK);
  // events with no parents and any index: the store does not check them
  for (int p = 0; p < n; p++)
    for (int k = 0; k < testSize; k++) CHECK(hge_store_set_event(s, key(p, k), p) == HGE_OK);
  for (int p = 0; p < n; p++)
    for (int k = 0; k < testSize; k++) CHECK(hge_store_has_event(s, key(p, k)) == 1);
  CHECK(hge_store_has_event(s, 99999) == 0);
  for (int p = 0; p < n; p++) {
    int rc;
    std::vector<int64_t> pe = pevents(s, p, 0, &rc);
    CHECK(rc == HGE_OK);
    CHECK((int)pe.size() == testSize);
    for (int k = 0; k < testSize; k++) CHECK(pe[(size_t)k] == key(p, k));
  }
  int32_t known[3];
  CHECK(hge_store_known(s, known) == HGE_OK);
  for (int p = 0; p < n; p++) CHECK(known[p] == testSize);
  // SetEvent of a stored event adds nothing
  CHECK(hge_store_set_event(s, key(1, 3), 1) == HGE_OK);
  CHECK(hge_store_known(s, known) == HGE_OK && known[1] == testSize);
  for (int p = 0; p < n; p++)
    for (int k = 0; k < testSize; k++) CHECK(hge_store_add_consensus_event(s, key(p, k)) == HGE_OK);
  CHECK(hge_store_consensus_count(s) == n * testSize);
  std::vector<int64_t> ce((size_t)(n * testSize));
  CHECK(hge_store_consensus_events(s, ce.data(), (int64_t)ce.size()) == n * testSize);
  CHECK(ce[0] == key(0, 0) && ce.back() == key(2, testSize - 1));
  // last from, item lookups, unknown participant
  int64_t k = -1;
  int32_t found = 0;
  CHECK(hge_store_last_from(s, 2, &k, &found) == HGE_OK && found == 1 && k == key(2, testSize - 1));
  CHECK(hge_store_participant_event(s, 1, 4, &k) == HGE_OK && k == key(1, 4));
  CHECK(hge_store_participant_event(s, 1, testSize, &k) == HGE_ERR_NOT_FOUND);
  // a participant the store was not created with: ParticipantEventsCache.Add creates
  // its list (caches.go:99-106); Known reports the registered ones only
  int rc;
  pevents(s, 7, 0, &rc);
  CHECK(rc == HGE_ERR_NOT_FOUND);
  CHECK(hge_store_set_event(s, 99999, 7) == HGE_OK);
  std::vector<int64_t> p7 = pevents(s, 7, 0, &rc);
  CHECK(rc == HGE_OK && p7.size() == 1 && p7[0] == 99999);
  pevents(s, 9, 0, &rc);
  CHECK(rc == HGE_ERR_NOT_FOUND);
  CHECK(hge_store_set_event(s, 5, -1) == HGE_ERR_ARG);
  hge_store_destroy(s);
}

static void inmem_rounds() {
  const int n = 3;
  hge_store* s = nullptr;
  CHECK(hge_store_create(n, 10, &s) == HGE_OK);
  // one round whose entries are events the store never saw (witnesses here)
  std::vector<int64_t> keys = {key(0, 0), key(1, 0), key(2, 0)};
  std::vector<uint8_t> wit = {1, 1, 1}, fam = {0, 0, 0};
  CHECK(hge_store_set_round(s, 0, keys.data(), wit.data(), fam.data(), 3) == HGE_OK);
  CHECK(hge_store_rounds(s) == 1);
  std::vector<int64_t> gk(8);
  std::vector<uint8_t> gw(8), gf(8);
  int32_t m = 0;
  CHECK(hge_store_get_round(s, 0, gk.data(), gw.data(), gf.data(), 8, &m) == HGE_OK && m == 3);
  std::map<int64_t, std::pair<int, int>> got, exp;
  for (int i = 0; i < m; i++) got[gk[(size_t)i]] = {gw[(size_t)i], gf[(size_t)i]};
  for (int i = 0; i < 3; i++) exp[keys[(size_t)i]] = {wit[(size_t)i], fam[(size_t)i]};
  CHECK(got == exp);  // reflect.DeepEqual(*round, storedRound)
  CHECK(hge_store_round_witnesses(s, 0, gk.data(), 8, &m) == HGE_OK && m == 3);
  CHECK((std::set<int64_t>(gk.begin(), gk.begin() + m) == std::set<int64_t>(keys.begin(), keys.end())));
  // a RoundInfo with non-witnesses and fame: round-trips; RoundEvents counts them all
  std::vector<int64_t> k2 = {7, 8, 9, 10};
  std::vector<uint8_t> w2 = {1, 0, 1, 0}, f2 = {1, 0, 2, 0};
  CHECK(hge_store_set_round(s, 1, k2.data(), w2.data(), f2.data(), 4) == HGE_OK);
  CHECK(hge_store_rounds(s) == 2 && hge_store_round_events(s, 1) == 4);
  CHECK(hge_store_get_round(s, 1, gk.data(), gw.data(), gf.data(), 8, &m) == HGE_OK && m == 4);
  for (int i = 0; i < 4; i++) CHECK(gk[(size_t)i] == k2[(size_t)i] && gw[(size_t)i] == w2[(size_t)i] && gf[(size_t)i] == f2[(size_t)i]);
  CHECK(hge_store_round_witnesses(s, 1, gk.data(), 8, &m) == HGE_OK && m == 2);
  // SetRound of a stored round replaces it
  CHECK(hge_store_set_round(s, 1, k2.data(), w2.data(), f2.data(), 2) == HGE_OK);
  CHECK(hge_store_rounds(s) == 2 && hge_store_round_events(s, 1) == 2);
  CHECK(hge_store_get_round(s, 5, gk.data(), gw.data(), gf.data(), 8, &m) == HGE_ERR_NOT_FOUND);
  CHECK(hge_store_round_events(s, 5) == 0);
  hge_store_destroy(s);
}

// participants {alice, bob, charlie} = 0, 1, 2; item "<pk><i>" = key(p, i)
static void participant_events_cache(int testSize) {
  const int size = 10, n = 3;
  hge_store* s = nullptr;
  CHECK(hge_store_create(n, size, &s) == HGE_OK);
  for (int i = 0; i < testSize; i++)
    for (int p = 0; p < n; p++) CHECK(hge_store_set_event(s, key(p, i), p) == HGE_OK);
  int32_t known[3];
  CHECK(hge_store_known(s, known) == HGE_OK);
  for (int p = 0; p < n; p++) CHECK(known[p] == testSize);
  for (int p = 0; p < n; p++) {
    int rc;
    if (testSize == 25) {
      pevents(s, p, 0, &rc);
      CHECK(rc == HGE_OK || rc == HGE_ERR_TOO_LATE);  // "Skipping 0 elements should return ErrNotFatal"
      CHECK(rc == HGE_ERR_TOO_LATE);                   // 25 items in a 2 * 10 list: rolled at 20 to the last 10
      for (int skip : {10, 15, 27}) {
        std::vector<int64_t> v = pevents(s, p, skip, &rc);
        CHECK(rc == HGE_OK);
        const int exp = skip >= testSize ? 0 : testSize - skip;
        CHECK((int)v.size() == exp);
        for (int k = 0; k < exp; k++) CHECK(v[(size_t)k] == key(p, skip + k));
      }
      int64_t x;
      CHECK(hge_store_participant_event(s, p, 9, &x) == HGE_ERR_TOO_LATE);
      CHECK(hge_store_participant_event(s, p, 10, &x) == HGE_OK && x == key(p, 10));
      CHECK(hge_store_participant_event(s, p, -1, &x) == HGE_ERR_TOO_LATE);
    } else {  // TestParticipantEventsCacheEdge: skip == size
      std::vector<int64_t> v = pevents(s, p, size, &rc);
      CHECK(rc == HGE_OK && (int)v.size() == testSize - size);
      for (int k = 0; k < testSize - size; k++) CHECK(v[(size_t)k] == key(p, size + k));
    }
  }
  hge_store_destroy(s);
}

// common/lru.go: Add evicts the least recently used past size; Get refreshes
static void round_lru() {
  hge_store* s = nullptr;
  CHECK(hge_store_create(1, 3, &s) == HGE_OK);
  int64_t k = 1;
  uint8_t w = 1, f = 0;
  for (int r = 0; r < 3; r++) CHECK(hge_store_set_round(s, r, &k, &w, &f, 1) == HGE_OK);
  CHECK(hge_store_round_events(s, 0) == 1);  // round 0 becomes the most recent
  CHECK(hge_store_set_round(s, 3, &k, &w, &f, 1) == HGE_OK);  // evicts round 1
  CHECK(hge_store_rounds(s) == 3);
  int32_t m;
  CHECK(hge_store_get_round(s, 1, nullptr, nullptr, nullptr, 0, &m) == HGE_ERR_NOT_FOUND);
  CHECK(hge_store_get_round(s, 0, nullptr, nullptr, nullptr, 0, &m) == HGE_OK && m == 1);
  hge_store_destroy(s);
  // consensus RollingList: the last window after rolls, the total kept
  CHECK(hge_store_create(1, 4, &s) == HGE_OK);
  for (int i = 0; i < 9; i++) CHECK(hge_store_add_consensus_event(s, i) == HGE_OK);
  std::vector<int64_t> v(16);
  const int64_t nv = hge_store_consensus_events(s, v.data(), 16);
  CHECK(nv == 5 && v[0] == 4 && v[4] == 8 && hge_store_consensus_count(s) == 9);  // rolled at 8 to the last 4
  hge_store_destroy(s);
}

// cache size 0 (NewLRU(0), NewRollingList(0)) and the eventCache LRU
static void lru_edges() {
  hge_store* s = nullptr;
  CHECK(hge_store_create(2, -1, &s) == HGE_ERR_ARG);
  CHECK(hge_store_create(2, 0, &s) == HGE_OK);
  int64_t k = 7;
  uint8_t w = 1, f = 0;
  CHECK(hge_store_set_round(s, 0, &k, &w, &f, 1) == HGE_OK);  // Add evicts it at once
  CHECK(hge_store_rounds(s) == 0);
  int32_t m;
  CHECK(hge_store_get_round(s, 0, nullptr, nullptr, nullptr, 0, &m) == HGE_ERR_NOT_FOUND);
  // the eventCache keeps nothing: every SetEvent appends the key again
  CHECK(hge_store_set_event(s, 11, 1) == HGE_OK && hge_store_set_event(s, 11, 1) == HGE_OK);
  CHECK(hge_store_has_event(s, 11) == 0);
  int rc;
  std::vector<int64_t> v = pevents(s, 1, 0, &rc);
  CHECK(rc == HGE_OK && v.size() == 2);
  for (int i = 0; i < 50; i++) CHECK(hge_store_add_consensus_event(s, i) == HGE_OK);  // never rolls
  CHECK(hge_store_consensus_events(s, nullptr, 0) == 50);
  hge_store_destroy(s);
  // size 2: a key evicted from the eventCache is appended again by its next SetEvent
  CHECK(hge_store_create(1, 2, &s) == HGE_OK);
  for (int64_t key_ : {1, 2, 3}) CHECK(hge_store_set_event(s, key_, 0) == HGE_OK);  // evicts 1
  CHECK(hge_store_has_event(s, 1) == 0 && hge_store_has_event(s, 2) == 1);
  CHECK(hge_store_set_event(s, 2, 0) == HGE_OK);  // still cached: nothing appended
  CHECK(hge_store_set_event(s, 1, 0) == HGE_OK);  // evicted: appended again
  int32_t known = 0;
  CHECK(hge_store_known(s, &known) == HGE_OK && known == 4);
  hge_store_destroy(s);
}

int main() {
  lru_edges();
  inmem_events();
  inmem_rounds();
  participant_events_cache(25);
  participant_events_cache(11);
  round_lru();
  std::printf("ok %d\n", checks);
  return 0;
}
