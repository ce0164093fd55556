// The Go shim's own logic (go/hashgraph/hashgraph_hge.go, inmem_store_hge.go)
// restated in C++ over the same C ABI calls, and driven through the reference's
// store and consensus tests.  No Go toolchain exists in this image, so this is
// how the shim's host-side bookkeeping -- which the cgo type check
// (tests/test_go_shim.py) cannot see -- gets executed:
//   * the hash <-> engine id map (remember / hash / parentRef), the standalone
//     key map (key / keyToHash), SetEvent's unregistered-participant lists;
//   * the SetRound overlay: bound, GetRound is the engine's live round with the
//     SetRound copy's entries added only for hashes the engine does not know
//     (a copy must not hide fame decided after the SetRound);
//   * FindOrder: the batch as the tail of the consensus log, round received, and
//     the consensus timestamp handed back as the median's source event's own Time
//     (hge_consensus_timestamp_sources: MedianTimestamp returns
//     events[len/2].Body.Timestamp, hashgraph.go:762-770), zone included -- also
//     when several events share the instant in different zones.
// Each class mirrors one Go type method by method (names kept); a Time is
// (UnixNano, zone tag) since only those two fields matter to the lookup.
//
//   shim_replay_test          host only: TestInmemRounds (inmem_store_test.go:121-159)
//                             and the unbound Store views on the standalone store
//   shim_replay_test --gpu    bound: TestFindOrder (hashgraph_test.go:1019-1047) over
//                             initConsensusHashgraph's DAG through the shim's insert,
//                             DivideRounds / DecideFame / FindOrder, then the overlay
// Exit status 0 = all checks passed.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "hge.h"

static int failures = 0;
#define CHECK(cond)                                                     \
  do {                                                                  \
    if (!(cond)) {                                                      \
      fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      failures++;                                                       \
    }                                                                   \
  } while (0)

struct Time {
  int64_t nano = 0;
  int zone = 0;
  bool operator==(const Time& o) const { return nano == o.nano && zone == o.zone; }
};

// Event: what the shim reads of one (event.go)
struct Event {
  std::string hex, creator, self_parent, other_parent;
  Time ts;
  uint8_t s[32] = {0}, hash[32] = {0};
  int index = 0, n_tx = 0;
  int round_received = -1;
  Time consensus_ts;
};

enum Trilean { Undefined = 0, True = 1, False = 2 };
struct RoundEvent {
  bool witness = false;
  Trilean famous = Undefined;
};
typedef std::map<std::string, RoundEvent> RoundInfo;  // RoundInfo.Events

enum Err { OK = 0, ErrKeyNotFound, ErrTooLate, ErrOther };
static Err storeErr(int rc) {
  if (rc == HGE_OK) return OK;
  if (rc == HGE_ERR_TOO_LATE) return ErrTooLate;
  if (rc == HGE_ERR_NOT_FOUND) return ErrKeyNotFound;
  return ErrOther;
}

// ---- InmemStore (inmem_store_hge.go) ------------------------------------------
struct InmemStore {
  int64_t cacheSize;
  std::map<std::string, Event> events;
  std::map<std::string, int32_t> ids;
  std::vector<std::string> hashes;
  std::map<std::string, int64_t> keys;
  std::vector<std::string> keyHash;
  hge_store* st = nullptr;
  hge_engine* eng = nullptr;
  std::map<std::string, int> participants, extra;

  InmemStore(const std::map<std::string, int>& p, int64_t cache) : cacheSize(cache), participants(p) {
    CHECK(hge_store_create((int32_t)p.size(), cache, &st) == HGE_OK);
  }
  ~InmemStore() { hge_store_destroy(st); }
  void bind(hge_engine* e) { eng = e; }
  bool bound() const { return eng != nullptr; }
  void remember(const std::string& hash, int32_t id) {
    ids[hash] = id;
    while ((int32_t)hashes.size() <= id) hashes.push_back("");
    hashes[id] = hash;
  }
  std::string hash(int32_t id) const { return id < 0 || id >= (int32_t)hashes.size() ? "" : hashes[id]; }
  int64_t key(const std::string& h) {
    auto it = keys.find(h);
    if (it != keys.end()) return it->second;
    const int64_t k = (int64_t)keyHash.size();
    keys[h] = k;
    keyHash.push_back(h);
    return k;
  }
  std::string keyToHash(int64_t k) const { return k < 0 || k >= (int64_t)keyHash.size() ? "" : keyHash[k]; }
  Err GetEvent(const std::string& k, Event& out) const {
    auto it = events.find(k);
    if (it == events.end()) return ErrKeyNotFound;
    if (!bound()) {  // the eventCache LRU answers (evicted: not found; a hit refreshes)
      auto kt = keys.find(k);
      if (kt == keys.end() || !hge_store_has_event(st, kt->second)) return ErrKeyNotFound;
    }
    out = it->second;
    return OK;
  }
  Err creatorID(const std::string& p, int32_t& c) const {
    auto it = participants.find(p);
    if (it != participants.end()) {
      c = it->second;
      return OK;
    }
    auto jt = extra.find(p);
    if (jt != extra.end() && !bound()) {
      c = jt->second;
      return OK;
    }
    c = -1;
    return ErrKeyNotFound;
  }
  Err SetEvent(const Event& ev) {
    if (bound()) {
      events[ev.hex] = ev;
      return OK;
    }
    int32_t c;
    if (creatorID(ev.creator, c) != OK) {
      c = (int32_t)(participants.size() + extra.size());
      extra[ev.creator] = c;
    }
    const Err e = storeErr(hge_store_set_event(st, key(ev.hex), c));
    if (e != OK) return e;
    events[ev.hex] = ev;
    return OK;
  }
  Err ParticipantEvents(const std::string& p, int skip, std::vector<std::string>& res) {
    res.clear();
    int32_t c;
    if (Err e = creatorID(p, c)) return e;
    if (!bound()) {
      int64_t n = 0;
      if (Err e = storeErr(hge_store_participant_events(st, c, skip, nullptr, 0, &n))) return e;
      std::vector<int64_t> ks(n);
      if (n) hge_store_participant_events(st, c, skip, ks.data(), n, &n);
      for (int64_t k : ks) res.push_back(keyToHash(k));
      return OK;
    }
    int64_t n = 0;
    if (Err e = storeErr(hge_participant_events(eng, c, skip, nullptr, 0, &n))) return e;
    std::vector<int32_t> is(n);
    if (n)
      if (Err e = storeErr(hge_participant_events(eng, c, skip, is.data(), n, &n))) return e;
    for (int32_t id : is) res.push_back(hash(id));
    return OK;
  }
  Err LastFrom(const std::string& p, std::string& out) {
    int32_t c;
    if (Err e = creatorID(p, c)) return e;
    if (!bound()) {
      int64_t k = 0;
      int32_t found = 0;
      if (Err e = storeErr(hge_store_last_from(st, c, &k, &found))) return e;
      out = found ? keyToHash(k) : "";
      return OK;
    }
    out = hash(hge_last_from(eng, c));
    return OK;
  }
  std::map<int, int> Known() {
    std::map<int, int> known;
    std::vector<int32_t> counts(participants.size());
    if (counts.empty()) return known;
    if (bound()) hge_known(eng, counts.data());
    else hge_store_known(st, counts.data());
    for (size_t i = 0; i < counts.size(); i++) known[(int)i] = counts[i];
    return known;
  }
  std::vector<std::string> ConsensusEvents() {
    std::vector<std::string> res;
    if (!bound()) {
      const int64_t n = hge_store_consensus_events(st, nullptr, 0);
      std::vector<int64_t> ks(n > 0 ? n : 0);
      if (n > 0) hge_store_consensus_events(st, ks.data(), n);
      for (int64_t k : ks) res.push_back(keyToHash(k));
      return res;
    }
    const int64_t n = hge_consensus_events(eng, nullptr, 0);
    std::vector<int32_t> is(n > 0 ? n : 0);
    if (n > 0) hge_consensus_events(eng, is.data(), n);
    for (int32_t id : is) res.push_back(hash(id));
    return res;
  }
  Err AddConsensusEvent(const std::string& k) {
    if (!bound()) return storeErr(hge_store_add_consensus_event(st, key(k)));
    return ids.count(k) ? OK : ErrKeyNotFound;
  }
  bool setRound(int r, RoundInfo& ri) {
    ri.clear();
    int32_t n = 0;
    if (hge_store_get_round(st, r, nullptr, nullptr, nullptr, 0, &n) != HGE_OK) return false;
    if (n == 0) return true;
    std::vector<int64_t> ks(n);
    std::vector<uint8_t> wit(n), fame(n);
    hge_store_get_round(st, r, ks.data(), wit.data(), fame.data(), n, &n);
    for (int i = 0; i < n; i++) ri[keyToHash(ks[i])] = RoundEvent{wit[i] != 0, (Trilean)fame[i]};
    return true;
  }
  int Rounds() { return bound() ? hge_rounds(eng) : hge_store_rounds(st); }
  RoundInfo engineRound(int r) {
    RoundInfo ri;
    int64_t n = 0;
    hge_round_event_ids(eng, r, nullptr, nullptr, 0, &n);
    if (n > 0) {
      std::vector<int32_t> is(n);
      std::vector<uint8_t> wit(n);
      hge_round_event_ids(eng, r, is.data(), wit.data(), n, &n);
      for (int64_t i = 0; i < n; i++) {
        RoundEvent re{wit[i] != 0, Undefined};
        if (re.witness) {
          const Event& ev = events[hash(is[i])];
          int32_t c;
          if (creatorID(ev.creator, c) == OK) re.famous = (Trilean)hge_fame(eng, r, c);
        }
        ri[hash(is[i])] = re;
      }
    }
    return ri;
  }
  Err GetRound(int r, RoundInfo& out) {
    RoundInfo set;
    const bool have = setRound(r, set);
    if (!bound() || r < 0 || r >= Rounds()) {
      out = set;
      return have ? OK : ErrKeyNotFound;
    }
    out = engineRound(r);
    if (have)
      for (auto& kv : set)
        if (!ids.count(kv.first)) out[kv.first] = kv.second;
    return OK;
  }
  Err SetRound(int r, const RoundInfo& round) {
    std::vector<int64_t> ks;
    std::vector<uint8_t> kwit, kfame, wit, fame;
    std::vector<int32_t> is;
    for (auto& kv : round) {
      const uint8_t w = kv.second.witness ? 1 : 0;
      ks.push_back(key(kv.first));
      kwit.push_back(w);
      kfame.push_back((uint8_t)kv.second.famous);
      auto it = ids.find(kv.first);
      if (it != ids.end() && bound() && kv.second.witness) {
        is.push_back(it->second);
        wit.push_back(w);
        fame.push_back((uint8_t)kv.second.famous);
      }
    }
    Err e = storeErr(hge_store_set_round(st, r, ks.empty() ? nullptr : ks.data(), kwit.data(), kfame.data(),
                                         (int32_t)ks.size()));
    if (e != OK || !bound()) return e;
    return storeErr(hge_set_round(eng, r, is.empty() ? nullptr : is.data(), wit.data(), fame.data(),
                                  (int32_t)is.size()));
  }
  std::vector<std::string> RoundWitnesses(int r) {
    std::vector<std::string> res;
    RoundInfo ri;
    if (GetRound(r, ri) != OK) return res;
    for (auto& kv : ri)
      if (kv.second.witness) res.push_back(kv.first);
    return res;
  }
  int RoundEvents(int r) {
    RoundInfo set;
    if (!setRound(r, set) && bound()) return r < 0 || r >= Rounds() ? 0 : hge_round_events(eng, r);
    RoundInfo ri;
    return GetRound(r, ri) == OK ? (int)ri.size() : 0;
  }
};

// ---- Hashgraph (hashgraph_hge.go) ---------------------------------------------
struct Hashgraph {
  std::map<std::string, int> Participants;
  InmemStore* store;
  std::vector<std::string> UndeterminedEvents;
  int LastConsensusRound = -1;
  std::vector<std::vector<Event>> commits;  // what commitCh received
  hge_engine* eng = nullptr;

  Hashgraph(const std::map<std::string, int>& p, InmemStore* s) : Participants(p), store(s) {
    CHECK(hge_create((int32_t)p.size(), 1 << 16, 0, 0, &eng) == HGE_OK);
    hge_set_cache_size(eng, s->cacheSize);
    s->bind(eng);
  }
  ~Hashgraph() { hge_destroy(eng); }
  int32_t parentRef(const std::string& x) {
    if (x.empty()) return HGE_NONE;
    auto it = store->ids.find(x);
    return it != store->ids.end() ? it->second : HGE_UNKNOWN;
  }
  Err insert(const Event& event) {
    auto it = Participants.find(event.creator);
    if (it == Participants.end()) return ErrOther;
    hge_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.creator = it->second;
    ev.index = event.index;
    ev.self_parent = parentRef(event.self_parent);
    ev.other_parent = parentRef(event.other_parent);
    ev.timestamp_ns = event.ts.nano;
    memcpy(ev.s, event.s, 32);
    memcpy(ev.hash, event.hash, 32);
    ev.n_tx = event.n_tx;
    int32_t status = 0;
    int64_t accepted = 0;
    if (hge_insert_events(eng, &ev, 1, &status, &accepted) != HGE_OK) return ErrOther;
    store->remember(event.hex, status);
    if (Err e = store->SetEvent(event)) return e;
    UndeterminedEvents.push_back(event.hex);
    return OK;
  }
  void syncFields() { LastConsensusRound = hge_last_consensus_round(eng); }
  Err DivideRounds() { return hge_divide_rounds(eng) == HGE_OK ? OK : ErrOther; }
  Err DecideFame() {
    if (hge_decide_fame(eng) != HGE_OK) return ErrOther;
    syncFields();
    return OK;
  }
  Err FindOrder() {
    int64_t n = 0;
    if (hge_find_order(eng, nullptr, 0, &n) != HGE_OK) return ErrOther;
    const int64_t total = hge_consensus_count(eng), from = total - n;
    std::vector<Event> batch;
    if (n > 0) {
      std::vector<int32_t> is(n), src(n);
      hge_consensus_log(eng, from, is.data(), n);
      if (hge_consensus_timestamp_sources(eng, is.data(), n, src.data()) != HGE_OK) return ErrOther;
      for (int64_t q = 0; q < n; q++) {
        const std::string hex = store->hash(is[q]);
        Event ev, sev;
        if (Err e = store->GetEvent(hex, ev)) return e;
        if (Err e = store->GetEvent(store->hash(src[q]), sev)) return e;
        ev.round_received = hge_round_received(eng, is[q]);
        ev.consensus_ts = sev.ts;  // the source event's Body.Timestamp, zone included
        store->events[hex] = ev;
        batch.push_back(ev);
      }
    }
    const int64_t und = hge_undetermined(eng, nullptr, 0);
    UndeterminedEvents.clear();
    if (und > 0) {
      std::vector<int32_t> is(und);
      hge_undetermined(eng, is.data(), und);
      for (int32_t id : is) UndeterminedEvents.push_back(store->hash(id));
    }
    syncFields();
    if (!batch.empty()) commits.push_back(batch);
    return OK;
  }
};

// ---- the reference's test DAGs ----------------------------------------------
static std::string pub(int i) { return "0x04" + std::string(64, (char)('a' + i)); }
static std::string hexOf(const std::string& name) {
  // a synthetic hex hash per name ("0X" + 64 hex digits, as Event.Hex formats it)
  unsigned h = 2166136261u;
  for (char ch : name) h = (h ^ (unsigned char)ch) * 16777619u;
  char buf[80];
  snprintf(buf, sizeof buf, "0X%08X%056d", h, 0);
  return buf;
}

// TestInmemRounds (inmem_store_test.go:121-159) on the unbound store, then the
// unbound views with an unregistered participant (caches.go:99-106)
static void store_checks() {
  std::map<std::string, int> parts;
  for (int i = 0; i < 10; i++) parts[pub(i)] = i;
  InmemStore store(parts, 10);
  RoundInfo round;
  std::map<std::string, Event> events;
  for (int i = 0; i < 10; i++) {
    Event ev;
    ev.creator = pub(i);
    ev.hex = hexOf("r0:" + std::to_string(i));
    events[ev.creator] = ev;
    round[ev.hex] = RoundEvent{true, Undefined};
  }
  CHECK(store.SetRound(0, round) == OK);
  CHECK(store.Rounds() == 1);
  RoundInfo got;
  CHECK(store.GetRound(0, got) == OK);
  CHECK(got.size() == round.size());
  for (auto& kv : round) {
    CHECK(got.count(kv.first) == 1);
    CHECK(got[kv.first].witness == kv.second.witness && got[kv.first].famous == kv.second.famous);
  }
  std::vector<std::string> w = store.RoundWitnesses(0);
  CHECK(w.size() == 10);
  std::set<std::string> ws(w.begin(), w.end());
  for (auto& kv : round) CHECK(ws.count(kv.first) == 1);
  CHECK(store.RoundEvents(0) == 10);
  RoundInfo none;
  CHECK(store.GetRound(5, none) == ErrKeyNotFound);

  // SetEvent / ParticipantEvents / LastFrom / Known / ConsensusEvents, unbound
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 10; i++) {
      Event ev;
      ev.creator = pub(i);
      ev.hex = hexOf("ev:" + std::to_string(i) + ":" + std::to_string(k));
      CHECK(store.SetEvent(ev) == OK);
    }
  std::vector<std::string> pe;
  CHECK(store.ParticipantEvents(pub(3), -1, pe) == ErrTooLate);  // caches.go:57-61
  CHECK(store.ParticipantEvents(pub(3), 0, pe) == OK);
  CHECK(pe.size() == 3 && pe[0] == hexOf("ev:3:0") && pe[2] == hexOf("ev:3:2"));
  std::string last;
  CHECK(store.LastFrom(pub(7), last) == OK && last == hexOf("ev:7:2"));
  std::map<int, int> known = store.Known();
  CHECK(known.size() == 10 && known[0] == 3 && known[9] == 3);
  // a creator nobody registered gets its own list and stays out of Known
  Event stranger;
  stranger.creator = "0x04stranger";
  stranger.hex = hexOf("stranger:0");
  CHECK(store.SetEvent(stranger) == OK);
  CHECK(store.ParticipantEvents("0x04stranger", 0, pe) == OK && pe.size() == 1 && pe[0] == stranger.hex);
  CHECK(store.LastFrom("0x04stranger", last) == OK && last == stranger.hex);
  CHECK(store.Known().size() == 10);
  Event got_ev;
  CHECK(store.GetEvent(stranger.hex, got_ev) == OK && got_ev.creator == stranger.creator);
  CHECK(store.AddConsensusEvent(hexOf("ev:0:0")) == OK);
  CHECK(store.AddConsensusEvent(hexOf("ev:1:0")) == OK);
  std::vector<std::string> ce = store.ConsensusEvents();
  CHECK(ce.size() == 2 && ce[0] == hexOf("ev:0:0") && ce[1] == hexOf("ev:1:0"));
}

// initConsensusHashgraph's DAG (hashgraph_test.go:835-950)
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

static int gpu_checks() {
  std::map<std::string, int> parts;
  for (int i = 0; i < 3; i++) parts[pub(i)] = i;
  InmemStore store(parts, 1000);
  Hashgraph h(parts, &store);
  std::map<std::string, std::string> name_of;  // hex -> name
  std::map<std::string, Time> ts_of;           // name -> Time
  int seq[3] = {0, 0, 0};
  for (int i = 0; i < kE; i++) {
    Event ev;
    ev.creator = pub(kDag[i].creator);
    ev.index = seq[kDag[i].creator]++;
    ev.hex = hexOf(kDag[i].name);
    ev.self_parent = kDag[i].sp[0] ? hexOf(kDag[i].sp) : "";
    ev.other_parent = kDag[i].op[0] ? hexOf(kDag[i].op) : "";
    // every event its own zone: the consensus timestamp must come back as the
    // source event's Time, not just its instant
    ev.ts = Time{1500000000000000000LL + 1000LL * i, 100 + i};
    const int rank[] = {0, 1, 3, 2, 4, 5};
    ev.s[0] = (uint8_t)(i < 6 ? rank[i] : 10 + i);
    for (int b = 0; b < 32; b++) ev.hash[b] = (uint8_t)(i * 7 + b + 1);
    ev.n_tx = (i >= 3 && i < 6) ? 1 : 0;
    name_of[ev.hex] = kDag[i].name;
    ts_of[kDag[i].name] = ev.ts;
    CHECK(h.insert(ev) == OK);
  }
  // an event whose parent the shim cannot resolve: HGE_UNKNOWN, refused, nothing kept
  CHECK(h.parentRef(hexOf("nobody")) == HGE_UNKNOWN && h.parentRef("") == HGE_NONE);
  CHECK(store.ids.size() == (size_t)kE && store.hash(0) == hexOf("e0") && store.hash(-1).empty());
  for (int i = 0; i < kE; i++) CHECK(store.ids[hexOf(kDag[i].name)] == i);

  // SetRound overlay, set BEFORE consensus: round 1's witnesses as Undefined plus a
  // hash the engine never saw (a non-witness entry)
  RoundInfo r1;
  for (const char* w : {"f1", "f0", "f2"}) r1[hexOf(w)] = RoundEvent{true, Undefined};
  r1[hexOf("foreign")] = RoundEvent{false, Undefined};
  CHECK(store.SetRound(1, r1) == OK);

  CHECK(h.DivideRounds() == OK);
  CHECK(h.DecideFame() == OK);
  CHECK(h.FindOrder() == OK);

  // TestFindOrder: 6 consensus events, either tie order of the reference test
  std::vector<std::string> ce = store.ConsensusEvents();
  CHECK(ce.size() == 6);
  const char* exp1[] = {"e0", "e10", "e1", "e21", "e2", "e02"};
  const char* exp2[] = {"e0", "e1", "e10", "e2", "e21", "e02"};
  for (size_t i = 0; i < ce.size() && i < 6; i++) CHECK(name_of[ce[i]] == exp1[i] || name_of[ce[i]] == exp2[i]);
  CHECK(h.LastConsensusRound == 1);
  // the batch went out on commitCh with round received and the source events' Times
  CHECK(h.commits.size() == 1 && h.commits[0].size() == 6);
  std::set<int64_t> instants;
  for (auto& kv : ts_of) instants.insert(kv.second.nano);
  for (auto& ev : h.commits.empty() ? std::vector<Event>() : h.commits[0]) {
    CHECK(ev.round_received == 1);
    CHECK(instants.count(ev.consensus_ts.nano) == 1);  // one of the inserted instants
    bool same = false;
    for (auto& kv : ts_of) same = same || kv.second == ev.consensus_ts;
    CHECK(same);  // and that event's Time, zone included
    Event stored;
    CHECK(store.GetEvent(ev.hex, stored) == OK && stored.round_received == 1);
  }
  // the undetermined list: every inserted event not ordered, in insertion order
  CHECK(h.UndeterminedEvents.size() == (size_t)kE - 6);
  if (!h.UndeterminedEvents.empty()) CHECK(name_of[h.UndeterminedEvents[0]] == "f1");

  // the overlay after consensus: the engine wins for events it knows (fame decided
  // after the SetRound shows), the foreign entry stays; round 0 was never set
  RoundInfo g1;
  CHECK(store.GetRound(1, g1) == OK);
  for (int c = 0; c < 3; c++) {
    const char* w = c == 0 ? "f0" : c == 1 ? "f1" : "f2";
    CHECK(g1.count(hexOf(w)) == 1);
    // decided by the engine after the SetRound said Undefined
    CHECK(g1[hexOf(w)].witness && g1[hexOf(w)].famous != Undefined);
    CHECK(g1[hexOf(w)].famous == (Trilean)hge_fame(h.eng, 1, c));
  }
  CHECK(g1.count(hexOf("foreign")) == 1 && !g1[hexOf("foreign")].witness);
  CHECK(g1.count(hexOf("f02")) == 1 && !g1[hexOf("f02")].witness);  // divided after the SetRound
  CHECK(store.RoundEvents(1) == 7);  // 6 events of round 1 + the foreign entry
  RoundInfo g0;
  CHECK(store.GetRound(0, g0) == OK && g0.size() == 6);
  CHECK(store.RoundEvents(0) == 6);
  std::vector<std::string> w0 = store.RoundWitnesses(0);
  CHECK(w0.size() == 3);
  CHECK(store.Rounds() == 4);
  std::map<int, int> known = store.Known();
  for (int i = 0; i < 3; i++) CHECK(known[i] == 7);  // TestKnown
  std::string last;
  CHECK(store.LastFrom(pub(2), last) == OK && name_of[last] == "h2");
  std::vector<std::string> pe;
  CHECK(store.ParticipantEvents(pub(0), 4, pe) == OK && pe.size() == 3 && name_of[pe[0]] == "g0");
  return failures;
}

// GetEvent / SetEvent of a standalone store against the reference's eventCache
// (inmem_store.go:42-64, common/lru.go): with cacheSize 2 the oldest of three events
// is evicted, so GetEvent misses it and its next SetEvent appends it to the
// creator's list again, while a GetEvent hit refreshes its key; with cacheSize 0
// nothing is kept and every SetEvent appends.
static void lru_checks() {
  std::map<std::string, int> parts;
  parts[pub(0)] = 0;
  {
    InmemStore store(parts, 2);
    Event ev[3];
    for (int i = 0; i < 3; i++) {
      ev[i].creator = pub(0);
      ev[i].hex = hexOf("lru:" + std::to_string(i));
      CHECK(store.SetEvent(ev[i]) == OK);
    }
    Event got;
    CHECK(store.GetEvent(ev[0].hex, got) == ErrKeyNotFound);  // evicted by ev[2]
    CHECK(store.GetEvent(ev[2].hex, got) == OK && got.hex == ev[2].hex);
    CHECK(store.GetEvent(ev[1].hex, got) == OK);  // refreshes ev[1]: ev[2] is now the oldest
    CHECK(store.SetEvent(ev[0]) == OK);           // a miss: appended again, evicts ev[2]
    CHECK(store.GetEvent(ev[2].hex, got) == ErrKeyNotFound);
    CHECK(store.GetEvent(ev[1].hex, got) == OK);
    CHECK(store.SetEvent(ev[1]) == OK);  // a hit: not appended
    std::vector<std::string> pe;
    CHECK(store.ParticipantEvents(pub(0), 0, pe) == OK);
    CHECK(pe.size() == 4);
    if (pe.size() == 4) CHECK(pe[0] == ev[0].hex && pe[1] == ev[1].hex && pe[2] == ev[2].hex && pe[3] == ev[0].hex);
  }
  {
    InmemStore store(parts, 0);
    Event e;
    e.creator = pub(0);
    e.hex = hexOf("lru0");
    CHECK(store.SetEvent(e) == OK);
    Event got;
    CHECK(store.GetEvent(e.hex, got) == ErrKeyNotFound);
    CHECK(store.SetEvent(e) == OK);
    std::map<int, int> known = store.Known();
    CHECK(known[0] == 2);
  }
}

// The same DAG with every event at ONE instant in its own zone: every consensus
// timestamp is that instant, and its zone must be the median source's -- the
// OldestSelfAncestorToSee(w, x) of the lowest-creator famous witness w of x's round
// received that sees x (ties at the median instant resolve to the lowest creator) --
// not the zone of whichever event showed that instant first (round 4's tsByNano).
static void shared_instant_checks() {
  std::map<std::string, int> parts;
  for (int i = 0; i < 3; i++) parts[pub(i)] = i;
  InmemStore store(parts, 1000);
  Hashgraph h(parts, &store);
  const int64_t T = 1500000000000000000LL;
  std::map<int32_t, int> zone_of;  // engine id -> zone
  int seq[3] = {0, 0, 0};
  for (int i = 0; i < kE; i++) {
    Event ev;
    ev.creator = pub(kDag[i].creator);
    ev.index = seq[kDag[i].creator]++;
    ev.hex = hexOf(std::string("z") + kDag[i].name);
    ev.self_parent = kDag[i].sp[0] ? hexOf(std::string("z") + kDag[i].sp) : "";
    ev.other_parent = kDag[i].op[0] ? hexOf(std::string("z") + kDag[i].op) : "";
    ev.ts = Time{T, 100 + i};
    ev.s[0] = (uint8_t)(10 + i);
    for (int b = 0; b < 32; b++) ev.hash[b] = (uint8_t)(i * 7 + b + 1);
    CHECK(h.insert(ev) == OK);
    zone_of[i] = 100 + i;
  }
  CHECK(h.DivideRounds() == OK);
  CHECK(h.DecideFame() == OK);
  CHECK(h.FindOrder() == OK);
  CHECK(h.commits.size() == 1);
  int not_first = 0;
  for (auto& ev : h.commits.empty() ? std::vector<Event>() : h.commits[0]) {
    const int32_t x = store.ids[ev.hex];
    const int r = ev.round_received;
    int want = -1;
    for (int d = 0; d < 3 && want < 0; d++) {
      const int32_t w = hge_round_witness(h.eng, r, d);
      if (w >= 0 && hge_fame(h.eng, r, d) == 1 && hge_see(h.eng, w, x)) {
        const int32_t osa = hge_oldest_self_ancestor_to_see(h.eng, w, x);
        if (osa >= 0) want = zone_of[osa];
      }
    }
    CHECK(ev.consensus_ts.nano == T && ev.consensus_ts.zone == want);
    not_first += want != 100;
  }
  CHECK(not_first > 0);  // some source is not the first event seen at that instant
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && !strcmp(argv[1], "--gpu");
  store_checks();
  lru_checks();
  if (gpu) {
    gpu_checks();
    shared_instant_checks();
  }
  printf("%s: %d failures\n", gpu ? "shim replay (store + engine)" : "shim replay (store)", failures);
  return failures ? 1 : 0;
}
