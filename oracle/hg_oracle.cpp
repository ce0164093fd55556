// hg_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// A line-faithful CPU restatement of the reference Go hashgraph ordering path
// (mpitid/babble @ /root/reference, package `hashgraph`), used as the parity
// oracle for the HIP engine and as the single-core CPU baseline ("port") in
// bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load this library.  The product engine (babble_amd/csrc) never links
// or calls it.
//
// Structure deliberately mirrors the Go code: lazily memoised predicates with
// per-pair caches (the Go LRUs with infinite capacity), an InmemStore with a
// round map whose size is Rounds(), DecideFame's nested x/y loops with the
// `break` and the fresh `votes` map, and per-call DivideRounds / DecideFame /
// FindOrder.  Go map iteration order (RoundInfo.Witnesses()) is pluggable:
// canonical = ascending creator id (the parity contract, SURVEY.md TL;DR 6),
// or a seeded random permutation per iteration to emulate Go's randomised
// map order.
//
// Parity pinning: there are no fixed-byte golden vectors in the reference
// (keys/signatures come from crypto/rand).  This oracle is pinned by the
// reference's own known-answer tests restated as fixtures in tests/golden/
// (hashgraph_test.go, node/core_test.go, node/node_test.go assertions).
//
// Citations are /root/reference relative paths.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int64_t kMaxInt64 = INT64_MAX;     // hashgraph.go:404-406 sentinel
constexpr int64_t kZeroTime = INT64_MIN;     // Go zero time.Time (never reached)

// EventCoordinates{hash, index} — event.go:68-71. hash is the event id (-1 = "").
struct Coord {
  int hash;
  int64_t index;
};

// Event — event.go:73-88 (fields the ordering path reads).
struct Event {
  int creator = 0;
  int64_t index = 0;
  int sp = -1, op = -1;  // Body.Parents[0], [1] (-1 = "")
  int64_t ts = 0;        // Body.Timestamp (int64 ns, one location)
  uint64_t S[4] = {0, 0, 0, 0};  // signature S, most significant limb first
  bool coin = true;      // middleBit: hash[len/2] != 0 (hashgraph.go:781-790)
  int ntx = 0;
  int topo = 0;
  // wire info, event.go:195-203
  int sp_index = -1, op_creator = -1, op_index = -1, creator_id = -1;
  bool has_rr = false;
  int rr = 0;
  int64_t cts = 0;
  std::vector<Coord> la, fd;
};

// RoundEvent / RoundInfo — roundInfo.go:24-60.
enum Trilean { Undefined = 0, True = 1, False = 2 };
struct RoundEvent {
  bool witness;
  Trilean famous;
};

struct Oracle;

struct RoundInfo {
  std::unordered_map<int, RoundEvent> events;  // Events map[hash]RoundEvent
  std::vector<int> keys;                       // insertion order (for determinism)

  // roundInfo.go:53-60
  void AddEvent(int x, bool witness) {
    if (events.find(x) == events.end()) {
      events[x] = RoundEvent{witness, Undefined};
      keys.push_back(x);
    }
  }
  // roundInfo.go:62-75
  void SetFame(int x, bool f) {
    auto it = events.find(x);
    RoundEvent e;
    if (it == events.end()) {
      e = RoundEvent{true, Undefined};
      keys.push_back(x);
    } else {
      e = it->second;
    }
    e.famous = f ? True : False;
    events[x] = e;
  }
  // roundInfo.go:78-85
  bool WitnessesDecided() const {
    for (auto& kv : events)
      if (kv.second.witness && kv.second.famous == Undefined) return false;
    return true;
  }
};

struct Oracle {
  int n = 0;             // len(Participants)
  uint64_t order_seed;   // 0 = canonical (ascending creator) map order
  std::mt19937_64 rng;

  // InmemStore (inmem_store.go:20-36), infinite cache contract (SURVEY TL;DR 8)
  std::vector<Event> events;                    // eventCache
  std::vector<std::vector<int>> participant;    // participantEventsCache
  std::map<int, RoundInfo> rounds;              // roundCache; Rounds() = len
  std::vector<int> consensus;                   // consensusCache (no roll)

  // Hashgraph (hashgraph.go:30-49)
  std::vector<int> undetermined;
  bool has_lcr = false;
  int lcr = 0;
  int lcre = 0;   // LastCommitedRoundEvents
  int64_t consensus_tx = 0;
  int topological_index = 0;

  std::unordered_map<uint64_t, bool> ancestorCache, selfAncestorCache, stronglySeeCache;
  // test instrumentation (not part of the reference): how often DecideFame took
  // the coin branch, voted by coin, and re-decided an already decided witness
  // (same / changed value); read by hgo_stats
  int64_t stat_coin_evals = 0, stat_coin_votes = 0, stat_redecided = 0, stat_flipped = 0;
  std::unordered_map<uint64_t, int> oldestSelfAncestorCache;
  std::unordered_map<int, int> parentRoundCache, roundCache;

  std::string last_error;
  std::vector<int> last_batch;  // events committed by the last FindOrder

  Oracle(int n_, uint64_t seed) : n(n_), order_seed(seed), rng(seed), participant(n_) {}

  static uint64_t key(int x, int y) { return (uint64_t)(uint32_t)x << 32 | (uint32_t)y; }
  bool getEvent(int x) const { return x >= 0 && x < (int)events.size(); }
  int SuperMajority() const { return 2 * n / 3 + 1; }  // hashgraph.go:78-80

  // Go map iteration emulation for RoundInfo.Witnesses()/FamousWitnesses().
  std::vector<int> ordered(std::vector<int> v) {
    if (order_seed == 0) {
      std::sort(v.begin(), v.end(), [&](int a, int b) {
        if (events[a].creator != events[b].creator) return events[a].creator < events[b].creator;
        return a < b;
      });
    } else {
      std::shuffle(v.begin(), v.end(), rng);
    }
    return v;
  }
  // roundInfo.go:88-96
  std::vector<int> Witnesses(const RoundInfo& r) {
    std::vector<int> res;
    for (int x : r.keys)
      if (r.events.at(x).witness) res.push_back(x);
    return ordered(res);
  }
  // roundInfo.go:99-107
  std::vector<int> FamousWitnesses(const RoundInfo& r) {
    std::vector<int> res;
    for (int x : r.keys) {
      auto& e = r.events.at(x);
      if (e.witness && e.famous == True) res.push_back(x);
    }
    return ordered(res);
  }
  // inmem_store.go:107-130
  int Rounds() const { return (int)rounds.size(); }
  std::vector<int> RoundWitnesses(int r) {
    auto it = rounds.find(r);
    if (it == rounds.end()) return {};
    return Witnesses(it->second);
  }
  int RoundEvents(int r) const {
    auto it = rounds.find(r);
    if (it == rounds.end()) return 0;
    return (int)it->second.events.size();
  }

  // ---------------- predicates (hashgraph.go:82-305) ----------------
  bool Ancestor(int x, int y) {
    auto k = key(x, y);
    auto it = ancestorCache.find(k);
    if (it != ancestorCache.end()) return it->second;
    bool a = ancestor(x, y);
    ancestorCache[k] = a;
    return a;
  }
  bool ancestor(int x, int y) {  // hashgraph.go:92-114
    if (x < 0) return false;
    if (x == y) return true;
    if (!getEvent(x) || !getEvent(y)) return false;
    const Event& ex = events[x];
    const Event& ey = events[y];
    return ex.la[ey.creator].index >= ey.index;
  }
  bool SelfAncestor(int x, int y) {
    auto k = key(x, y);
    auto it = selfAncestorCache.find(k);
    if (it != selfAncestorCache.end()) return it->second;
    bool a = selfAncestor(x, y);
    selfAncestorCache[k] = a;
    return a;
  }
  bool selfAncestor(int x, int y) {  // hashgraph.go:126-146
    if (x < 0) return false;
    if (x == y) return true;
    if (!getEvent(x) || !getEvent(y)) return false;
    return events[x].creator == events[y].creator && events[x].index >= events[y].index;
  }
  bool See(int x, int y) { return Ancestor(x, y); }  // hashgraph.go:149-154
  int OldestSelfAncestorToSee(int x, int y) {
    auto k = key(x, y);
    auto it = oldestSelfAncestorCache.find(k);
    if (it != oldestSelfAncestorCache.end()) return it->second;
    int r = oldestSelfAncestorToSee(x, y);
    oldestSelfAncestorCache[k] = r;
    return r;
  }
  int oldestSelfAncestorToSee(int x, int y) {  // hashgraph.go:166-177
    if (!getEvent(x) || !getEvent(y)) return -1;
    const Coord& a = events[y].fd[events[x].creator];
    if (a.index <= events[x].index) return a.hash;
    return -1;
  }
  bool StronglySee(int x, int y) {
    auto k = key(x, y);
    auto it = stronglySeeCache.find(k);
    if (it != stronglySeeCache.end()) return it->second;
    bool s = stronglySee(x, y);
    stronglySeeCache[k] = s;
    return s;
  }
  bool stronglySee(int x, int y) {  // hashgraph.go:189-208
    if (!getEvent(x) || !getEvent(y)) return false;
    const Event& ex = events[x];
    const Event& ey = events[y];
    int c = 0;
    for (int i = 0; i < (int)ex.la.size(); i++)
      if (ex.la[i].index >= ey.fd[i].index) c++;
    return c >= SuperMajority();
  }
  int ParentRound(int x) {
    auto it = parentRoundCache.find(x);
    if (it != parentRoundCache.end()) return it->second;
    int pr = parentRound(x);
    parentRoundCache[x] = pr;
    return pr;
  }
  int parentRound(int x) {  // hashgraph.go:220-244
    if (x < 0) return -1;
    if (!getEvent(x)) return -1;
    const Event& ex = events[x];
    if (ex.sp < 0 && ex.op < 0) return 0;
    if (!getEvent(ex.sp)) return 0;
    if (!getEvent(ex.op)) return 0;
    int spRound = Round(ex.sp);
    int opRound = Round(ex.op);
    return spRound > opRound ? spRound : opRound;
  }
  bool Witness(int x) {  // hashgraph.go:247-260
    if (x < 0 || !getEvent(x)) return false;
    if (events[x].sp < 0) return true;
    return Round(x) > Round(events[x].sp);
  }
  bool RoundInc(int x) {  // hashgraph.go:263-285
    if (x < 0) return false;
    int pr = ParentRound(x);
    if (pr < 0) return false;
    if (Rounds() < pr + 1) return false;
    int c = 0;
    for (int w : RoundWitnesses(pr))
      if (StronglySee(x, w)) c++;
    return c >= SuperMajority();
  }
  int Round(int x) {
    auto it = roundCache.find(x);
    if (it != roundCache.end()) return it->second;
    int r = round(x);
    roundCache[x] = r;
    return r;
  }
  int round(int x) {  // hashgraph.go:296-305
    int r = ParentRound(x);
    if (RoundInc(x)) r++;
    return r;
  }

  // ---------------- insertion (hashgraph.go:328-494) ----------------
  // Returns new id >= 0, or a negative error code:
  //  -1 bad creator, -2 self-parent not known, -3 self-parent different creator,
  //  -4 other-parent not known, -5 self-parent not last known.
  int FromParentsLatest(const Event& e) {  // hashgraph.go:366-396
    int known = (int)participant[e.creator].size();
    if (e.sp < 0 && e.op < 0 && known == 0) return 0;
    if (!getEvent(e.sp)) { last_error = "Self-parent not known"; return -2; }
    if (events[e.sp].creator != e.creator) { last_error = "Self-parent has different creator"; return -3; }
    if (!getEvent(e.op)) { last_error = "Other-parent not known"; return -4; }
    int lastKnown = participant[e.creator].empty() ? -1 : participant[e.creator].back();
    if (e.sp != lastKnown) { last_error = "Self-parent not last known event by creator"; return -5; }
    return 0;
  }

  int InsertEvent(Event e) {  // hashgraph.go:328-363 (signature verify is host crypto, out of scope)
    if (e.creator < 0 || e.creator >= n) { last_error = "Could not find fake creator id"; return -1; }
    int err = FromParentsLatest(e);
    if (err) return err;
    e.topo = topological_index++;
    // SetWireInfo (hashgraph.go:496-524)
    e.sp_index = e.sp >= 0 ? (int)events[e.sp].index : -1;
    e.op_creator = e.op >= 0 ? events[e.op].creator : -1;
    e.op_index = e.op >= 0 ? (int)events[e.op].index : -1;
    e.creator_id = e.creator;
    int id = (int)events.size();
    InitEventCoordinates(e, id);
    // Store.SetEvent (inmem_store.go:51-65): new key -> participant list
    participant[e.creator].push_back(id);
    events.push_back(std::move(e));
    UpdateAncestorFirstDescendant(id);
    undetermined.push_back(id);
    return id;
  }

  void InitEventCoordinates(Event& e, int id) {  // hashgraph.go:399-463
    e.fd.assign(n, Coord{-1, kMaxInt64});
    e.la.assign(n, Coord{-1, -1});
    if (e.sp < 0 && e.op < 0) {
      // all -1
    } else if (e.sp < 0) {
      e.la = events[e.op].la;
    } else if (e.op < 0) {
      e.la = events[e.sp].la;
    } else {
      e.la = events[e.sp].la;
      const auto& opla = events[e.op].la;
      for (int i = 0; i < n; i++)
        if (e.la[i].index < opla[i].index) e.la[i] = opla[i];
    }
    e.fd[e.creator] = Coord{id, e.index};
    e.la[e.creator] = Coord{id, e.index};
  }

  void UpdateAncestorFirstDescendant(int id) {  // hashgraph.go:466-494
    const int c = events[id].creator;
    const int64_t index = events[id].index;
    for (int i = 0; i < n; i++) {
      int ah = events[id].la[i].hash;
      while (ah >= 0) {
        Event& a = events[ah];
        if (a.fd[c].index == kMaxInt64) {
          a.fd[c] = Coord{id, index};
          ah = a.sp;
        } else {
          break;
        }
      }
    }
  }

  // ---------------- consensus (hashgraph.go:573-760) ----------------
  void DivideRounds() {  // hashgraph.go:573-588
    for (int x : undetermined) {
      int r = Round(x);
      bool w = Witness(x);
      rounds[r].AddEvent(x, w);  // GetRound (or NewRoundInfo) + SetRound
    }
  }

  void setLastConsensusRound(int i) {  // hashgraph.go:666-673
    has_lcr = true;
    lcr = i;
    lcre = RoundEvents(i - 1);
  }

  void DecideFame() {  // hashgraph.go:598-664
    // votes[y][x] => vote(y, x); rebuilt every call (hashgraph.go:599)
    std::unordered_map<uint64_t, bool> votes;
    auto setVote = [&](int y, int x, bool v) { votes[key(y, x)] = v; };
    auto getVote = [&](int y, int x) {
      auto it = votes.find(key(y, x));
      return it != votes.end() && it->second;  // missing => false (nay)
    };
    const int start = has_lcr ? lcr + 1 : 0;  // fameLoopStart, hashgraph.go:590-595
    for (int i = start; i < Rounds() - 1; i++) {
      RoundInfo& roundInfo = rounds[i];
      for (int j = i + 1; j < Rounds(); j++) {
        for (int x : Witnesses(roundInfo)) {
          for (int y : RoundWitnesses(j)) {
            int diff = j - i;
            if (diff == 1) {
              setVote(y, x, See(y, x));
            } else {
              std::vector<int> ssWitnesses;
              for (int w : RoundWitnesses(j - 1))
                if (StronglySee(y, w)) ssWitnesses.push_back(w);
              int yays = 0, nays = 0;
              for (int w : ssWitnesses) {
                if (getVote(w, x)) yays++;
                else nays++;
              }
              bool v = false;
              int t = nays;
              if (yays >= nays) { v = true; t = yays; }
              // math.Mod(float64(diff), float64(N)) > 0  <=>  diff % N != 0 (diff > 0)
              if (diff % n != 0) {  // normal round
                if (t >= SuperMajority()) {
                  auto prev = roundInfo.events.find(x);
                  if (prev != roundInfo.events.end() && prev->second.famous != Undefined) {
                    stat_redecided++;
                    if (prev->second.famous != (v ? True : False)) stat_flipped++;
                  }
                  roundInfo.SetFame(x, v);
                  break;  // break out of y loop
                } else {
                  setVote(y, x, v);
                }
              } else {  // coin round
                stat_coin_evals++;
                if (t >= SuperMajority()) setVote(y, x, v);
                else {
                  stat_coin_votes++;
                  setVote(y, x, events[y].coin);
                }
              }
            }
          }
        }
      }
      if (roundInfo.WitnessesDecided() && (!has_lcr || i > lcr)) setLastConsensusRound(i);
    }
  }

  int64_t MedianTimestamp(const std::vector<int>& hashes) {  // hashgraph.go:762-770
    std::vector<int64_t> t;
    for (int x : hashes) t.push_back(getEvent(x) ? events[x].ts : kZeroTime);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  }

  void DecideRoundReceived() {  // hashgraph.go:676-721
    for (int x : undetermined) {
      int r = Round(x);
      for (int i = r + 1; i < Rounds(); i++) {
        RoundInfo& tr = rounds[i];
        if (!tr.WitnessesDecided()) continue;
        std::vector<int> fws = FamousWitnesses(tr);
        std::vector<int> s;
        for (int w : fws)
          if (See(w, x)) s.push_back(w);
        if ((int)s.size() > (int)fws.size() / 2) {
          Event& ex = events[x];
          ex.has_rr = true;
          ex.rr = i;
          std::vector<int> t;
          for (int a : s) t.push_back(OldestSelfAncestorToSee(a, x));
          ex.cts = MedianTimestamp(t);
          break;
        }
      }
    }
  }

  // ConsensusSorter.Less (consensus_sorter.go:36-59); PRN == 0 (SURVEY TL;DR 3).
  bool consensusLess(int a, int b) const {
    const Event& ea = events[a];
    const Event& eb = events[b];
    int irr = ea.has_rr ? ea.rr : -1, jrr = eb.has_rr ? eb.rr : -1;
    if (irr != jrr) return irr < jrr;
    if (ea.cts != eb.cts) return ea.cts < eb.cts;
    for (int k = 0; k < 4; k++)
      if (ea.S[k] != eb.S[k]) return ea.S[k] < eb.S[k];
    return a < b;  // S ties never occur for signatures; make the order total
  }

  int FindOrder() {  // hashgraph.go:723-760
    DecideRoundReceived();
    std::vector<int> newConsensus, newUndetermined;
    for (int x : undetermined) {
      if (events[x].has_rr) newConsensus.push_back(x);
      else newUndetermined.push_back(x);
    }
    undetermined.swap(newUndetermined);
    std::sort(newConsensus.begin(), newConsensus.end(),
              [&](int a, int b) { return consensusLess(a, b); });
    for (int e : newConsensus) {
      consensus.push_back(e);
      consensus_tx += events[e].ntx;
    }
    last_batch = newConsensus;
    return (int)newConsensus.size();
  }

  void RunConsensus() {  // node/core.go:179-202
    DivideRounds();
    DecideFame();
    FindOrder();
  }
};

Event makeEvent(int creator, int64_t index, int sp, int op, int64_t ts, const uint8_t* s32,
                const uint8_t* h32, int ntx) {
  Event e;
  e.creator = creator;
  e.index = index;
  e.sp = sp;
  e.op = op;
  e.ts = ts;
  for (int k = 0; k < 4; k++) {
    uint64_t v = 0;
    for (int b = 0; b < 8; b++) v = (v << 8) | (s32 ? s32[k * 8 + b] : 0);
    e.S[k] = v;
  }
  e.coin = h32 ? (h32[16] != 0) : true;
  e.ntx = ntx;
  return e;
}

}  // namespace

extern "C" {

void* hgo_create(int n, uint64_t order_seed) { return new Oracle(n, order_seed); }
void hgo_destroy(void* h) { delete (Oracle*)h; }
const char* hgo_last_error(void* h) { return ((Oracle*)h)->last_error.c_str(); }

int hgo_insert(void* h, int creator, int64_t index, int sp, int op, int64_t ts,
               const uint8_t* s32, const uint8_t* h32, int ntx) {
  return ((Oracle*)h)->InsertEvent(makeEvent(creator, index, sp, op, ts, s32, h32, ntx));
}
void hgo_divide_rounds(void* h) { ((Oracle*)h)->DivideRounds(); }
void hgo_decide_fame(void* h) { ((Oracle*)h)->DecideFame(); }
void hgo_decide_round_received(void* h) { ((Oracle*)h)->DecideRoundReceived(); }
int hgo_find_order(void* h) { return ((Oracle*)h)->FindOrder(); }
void hgo_run_consensus(void* h) { ((Oracle*)h)->RunConsensus(); }

int hgo_event_count(void* h) { return (int)((Oracle*)h)->events.size(); }
int hgo_rounds(void* h) { return ((Oracle*)h)->Rounds(); }
int hgo_last_consensus_round(void* h) {
  Oracle* o = (Oracle*)h;
  return o->has_lcr ? o->lcr : -1;
}
int hgo_last_committed_round_events(void* h) { return ((Oracle*)h)->lcre; }
int64_t hgo_consensus_transactions(void* h) { return ((Oracle*)h)->consensus_tx; }
int64_t hgo_consensus_count(void* h) { return (int64_t)((Oracle*)h)->consensus.size(); }
int64_t hgo_consensus_events(void* h, int32_t* out, int64_t cap) {
  Oracle* o = (Oracle*)h;
  int64_t m = std::min<int64_t>(cap, o->consensus.size());
  for (int64_t i = 0; i < m; i++) out[i] = o->consensus[i];
  return (int64_t)o->consensus.size();
}
int64_t hgo_undetermined(void* h, int32_t* out, int64_t cap) {
  Oracle* o = (Oracle*)h;
  int64_t m = std::min<int64_t>(cap, o->undetermined.size());
  for (int64_t i = 0; i < m; i++) out[i] = o->undetermined[i];
  return (int64_t)o->undetermined.size();
}
void hgo_known(void* h, int32_t* out) {
  Oracle* o = (Oracle*)h;
  for (int c = 0; c < o->n; c++) out[c] = (int32_t)o->participant[c].size();
}

int hgo_round(void* h, int x) { return ((Oracle*)h)->Round(x); }
int hgo_parent_round(void* h, int x) { return ((Oracle*)h)->ParentRound(x); }
int hgo_witness(void* h, int x) { return ((Oracle*)h)->Witness(x); }
int hgo_round_inc(void* h, int x) { return ((Oracle*)h)->RoundInc(x); }
int hgo_ancestor(void* h, int x, int y) { return ((Oracle*)h)->Ancestor(x, y); }
int hgo_self_ancestor(void* h, int x, int y) { return ((Oracle*)h)->SelfAncestor(x, y); }
int hgo_see(void* h, int x, int y) { return ((Oracle*)h)->See(x, y); }
int hgo_strongly_see(void* h, int x, int y) { return ((Oracle*)h)->StronglySee(x, y); }
int hgo_oldest_self_ancestor_to_see(void* h, int x, int y) {
  return ((Oracle*)h)->OldestSelfAncestorToSee(x, y);
}
// RoundInfo lookups: returns 0 Undefined, 1 True, 2 False; -1 if x not in round r.
int hgo_round_fame(void* h, int r, int x) {
  Oracle* o = (Oracle*)h;
  auto it = o->rounds.find(r);
  if (it == o->rounds.end()) return -1;
  auto e = it->second.events.find(x);
  if (e == it->second.events.end()) return -1;
  return (int)e->second.famous;
}
int hgo_round_is_witness(void* h, int r, int x) {
  Oracle* o = (Oracle*)h;
  auto it = o->rounds.find(r);
  if (it == o->rounds.end()) return -1;
  auto e = it->second.events.find(x);
  if (e == it->second.events.end()) return -1;
  return e->second.witness ? 1 : 0;
}
int hgo_round_witnesses(void* h, int r, int32_t* out, int cap) {
  Oracle* o = (Oracle*)h;
  std::vector<int> w = o->RoundWitnesses(r);
  std::sort(w.begin(), w.end());
  for (int i = 0; i < (int)w.size() && i < cap; i++) out[i] = w[i];
  return (int)w.size();
}
int hgo_round_event_count(void* h, int r) { return ((Oracle*)h)->RoundEvents(r); }
int hgo_round_received(void* h, int x) {
  Oracle* o = (Oracle*)h;
  return o->events[x].has_rr ? o->events[x].rr : -1;
}
int64_t hgo_consensus_timestamp(void* h, int x) { return ((Oracle*)h)->events[x].cts; }
// lastAncestors / firstDescendants indices (FD MaxInt64 reported as INT64_MAX).
void hgo_coords(void* h, int x, int64_t* la_idx, int32_t* la_hash, int64_t* fd_idx, int32_t* fd_hash) {
  Oracle* o = (Oracle*)h;
  for (int i = 0; i < o->n; i++) {
    if (la_idx) la_idx[i] = o->events[x].la[i].index;
    if (la_hash) la_hash[i] = o->events[x].la[i].hash;
    if (fd_idx) fd_idx[i] = o->events[x].fd[i].index;
    if (fd_hash) fd_hash[i] = o->events[x].fd[i].hash;
  }
}
void hgo_wire_info(void* h, int x, int32_t* out4) {
  Oracle* o = (Oracle*)h;
  const Event& e = o->events[x];
  out4[0] = e.sp_index;
  out4[1] = e.op_creator;
  out4[2] = e.op_index;
  out4[3] = e.creator_id;
}
// Store.SetRound for the reference tests that pre-seed rounds (hashgraph_test.go:614-742).
void hgo_set_round(void* h, int r, const int32_t* ids, const int32_t* witness, const int32_t* fame, int m) {
  Oracle* o = (Oracle*)h;
  RoundInfo ri;
  for (int i = 0; i < m; i++) {
    ri.events[ids[i]] = RoundEvent{witness[i] != 0, (Trilean)fame[i]};
    ri.keys.push_back(ids[i]);
  }
  o->rounds[r] = ri;
}

// Whole-schedule replay (the bench's CPU baseline and the fixture generator).
// Events are given in submission order; parents are submission indices (-1 = none).
// Rejected submissions are skipped (status[i] < 0) and any event naming a rejected
// parent is rejected as "not known".  RunConsensus is called after each submission
// position listed in call_points (ascending, 1-based counts of submissions).
// Outputs: status[n_sub], order[cap] (consensus order), call_counts[n_calls]
// (events committed by each call).  Returns total committed events.
// DecideFame instrumentation: {coin-branch evaluations, coin votes, re-decided
// witnesses, re-decisions that changed the fame value}
int hgo_stats(void* h, int64_t* out, int cap) {
  Oracle* o = (Oracle*)h;
  const int64_t v[4] = {o->stat_coin_evals, o->stat_coin_votes, o->stat_redecided, o->stat_flipped};
  for (int i = 0; i < cap && i < 4; i++) out[i] = v[i];
  return 4;
}

int64_t hgo_replay(void* h, int64_t n_sub, const int32_t* creator, const int32_t* index,
                   const int32_t* sp, const int32_t* op, const int64_t* ts, const uint8_t* S,
                   const uint8_t* hash, const int32_t* ntx, const int64_t* call_points,
                   int64_t n_calls, int32_t* status, int32_t* order, int64_t cap,
                   int64_t* call_counts) {
  Oracle* o = (Oracle*)h;
  std::vector<int> idmap(n_sub, -1);
  int64_t next_call = 0;
  for (int64_t i = 0; i < n_sub; i++) {
    int psp = sp[i] >= 0 ? idmap[sp[i]] : -1;
    int pop = op[i] >= 0 ? idmap[op[i]] : -1;
    // a named-but-rejected parent is an unknown hash: map it to a non-existent id
    if (sp[i] >= 0 && psp < 0) psp = INT32_MAX;
    if (op[i] >= 0 && pop < 0) pop = INT32_MAX;
    int id = o->InsertEvent(makeEvent(creator[i], index[i], psp, pop, ts[i], S + 32 * i,
                                      hash + 32 * i, ntx ? ntx[i] : 0));
    if (id >= 0) idmap[i] = id;
    if (status) status[i] = id;
    while (next_call < n_calls && call_points[next_call] == i + 1) {
      int64_t before = (int64_t)o->consensus.size();
      o->RunConsensus();
      if (call_counts) call_counts[next_call] = (int64_t)o->consensus.size() - before;
      next_call++;
    }
  }
  int64_t m = std::min<int64_t>(cap, o->consensus.size());
  for (int64_t i = 0; i < m; i++) order[i] = o->consensus[i];
  return (int64_t)o->consensus.size();
}

}  // extern "C"
