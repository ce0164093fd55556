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
// Two modes over the same store:
//  * faithful (default): the Go loops as written, with the memo caches.  The
//    bench's CPU baseline times this mode.
//  * scale (hgo_create2 flag 1; canonical witness order, no SetRound seeding):
//    the same functions computed without re-deriving what cannot change within
//    one call, so that whole 1M-10M-event streams fit in the container:
//      - the pure-memo caches (ancestor, selfAncestor, stronglySee,
//        oldestSelfAncestor) are not kept: their answers never change once both
//        events exist (SURVEY TL;DR 7), so recomputing gives the same value;
//        roundCache / parentRoundCache, whose first-computed values ARE the
//        semantics (Round depends on Rounds() when first asked), are kept as
//        dense arrays;
//      - DecideFame's `votes` map becomes, per (round i, witness x), a bitset
//        over the witnesses of round j (set only when the vote is true, as a
//        missing vote reads as false), and the ssWitnesses of (y, j-1) a bitset
//        built once per call: yays / nays are popcounts of their intersection;
//      - WitnessesDecided is a counter of undecided witness entries;
//      - DecideRoundReceived's "more than half of the famous witnesses see x"
//        is x.index <= theta(round, creator(x)), the (|F|/2+1)-th largest
//        lastAncestor index among the famous witnesses, recomputed when the
//        round's fame changes; the median is taken over the same set;
//      - optional release of the coordinates of events ordered long ago (any
//        later read of them aborts the process, so a completed run used none).
//    tests/test_oracle_scale.py checks both modes field by field, and every
//    golden regenerated in scale mode is byte-identical to the faithful one.
//
// Coordinates (event.go:68-71, EventCoordinates{hash, index}) are stored as
// 4-byte event ids and indexes; an index outside int32 is refused.
//
// Parity pinning: there are no fixed-byte golden vectors in the reference
// (keys/signatures come from crypto/rand).  This oracle is pinned by the
// reference's own known-answer tests restated as fixtures in tests/golden/
// (hashgraph_test.go, node/core_test.go, node/node_test.go assertions).
//
// Citations are /root/reference relative paths.
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr int64_t kMaxInt64 = INT64_MAX;     // hashgraph.go:404-406 sentinel
constexpr int64_t kZeroTime = INT64_MIN;     // Go zero time.Time (never reached)
constexpr int32_t kFdUnset = INT32_MAX;      // the MaxInt64 sentinel in 4 bytes
constexpr int kUnset = INT_MIN;              // dense round memo: not computed yet

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
  // lastAncestors / firstDescendants (event.go:84-85): 4 rows of n int32,
  // [la index | fd index | la event id | fd event id]; null once released.
  std::unique_ptr<int32_t[]> co;
};

// RoundEvent / RoundInfo — roundInfo.go:24-60.
enum Trilean { Undefined = 0, True = 1, False = 2 };
struct RoundEvent {
  bool witness;
  Trilean famous;
};

struct RoundInfo {
  std::unordered_map<int, RoundEvent> events;  // Events map[hash]RoundEvent
  std::vector<int> keys;                       // insertion order (for determinism)
  // derived views kept in step with `events` (read by the scale mode only)
  std::vector<int> wkeys;  // keys whose entry is a witness, in insertion order
  int undecided = 0;       // witness entries with famous == Undefined
  int version = 0;         // bumped whenever a witness entry or a fame value changes

  // roundInfo.go:53-60
  void AddEvent(int x, bool witness) {
    if (events.find(x) == events.end()) {
      events[x] = RoundEvent{witness, Undefined};
      keys.push_back(x);
      if (witness) {
        wkeys.push_back(x);
        undecided++;
        version++;
      }
    }
  }
  // roundInfo.go:62-75
  void SetFame(int x, bool f) {
    auto it = events.find(x);
    RoundEvent e;
    if (it == events.end()) {
      e = RoundEvent{true, Undefined};
      keys.push_back(x);
      wkeys.push_back(x);
    } else {
      e = it->second;
      if (e.witness && e.famous == Undefined) undecided--;
    }
    e.famous = f ? True : False;
    events[x] = e;
    version++;
  }
  // roundInfo.go:78-85
  bool WitnessesDecided() const {
    for (auto& kv : events)
      if (kv.second.witness && kv.second.famous == Undefined) return false;
    return true;
  }
};

[[noreturn]] void die(const char* what, long long v) {
  std::fprintf(stderr, "hg_oracle: %s (%lld)\n", what, v);
  std::fflush(stderr);
  std::abort();
}

struct Oracle {
  int n = 0;             // len(Participants)
  uint64_t order_seed;   // 0 = canonical (ascending creator) map order
  std::mt19937_64 rng;
  bool scale = false;    // scale mode requested (see the header)
  bool seeded = false;   // Store.SetRound was called from outside: faithful path only
  int release_lag = -1;  // scale mode: release ordered events' coordinates this many rounds behind LCR
  size_t release_next = 0;

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
  // scale mode: the same two caches, dense; `added` = DivideRounds already added x
  std::vector<int> parentRoundMemo, roundMemo;
  std::vector<uint8_t> added;
  // scale mode, DecideRoundReceived: per round, thresholds valid for `version`
  struct Theta {
    int version = -1;
    std::vector<int> famous;
    std::vector<int32_t> th;  // [creator]
  };
  std::vector<Theta> thetas;

  std::string last_error;
  std::vector<int> last_batch;  // events committed by the last FindOrder

  Oracle(int n_, uint64_t seed) : n(n_), order_seed(seed), rng(seed), participant(n_) {}

  bool fast() const { return scale && order_seed == 0 && !seeded; }

  static uint64_t key(int x, int y) { return (uint64_t)(uint32_t)x << 32 | (uint32_t)y; }
  bool getEvent(int x) const { return x >= 0 && x < (int)events.size(); }
  int SuperMajority() const { return 2 * n / 3 + 1; }  // hashgraph.go:78-80

  // coordinate rows of event x
  int32_t* co(int x) const {
    int32_t* p = events[x].co.get();
    if (!p) die("coordinates of a released event were read; raise the release lag", x);
    return p;
  }
  const int32_t* laIx(int x) const { return co(x); }
  const int32_t* fdIx(int x) const { return co(x) + n; }
  const int32_t* laId(int x) const { return co(x) + 2 * n; }
  const int32_t* fdId(int x) const { return co(x) + 3 * n; }

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
    if (fast()) return ancestor(x, y);
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
    const Event& ey = events[y];
    return laIx(x)[ey.creator] >= ey.index;
  }
  bool SelfAncestor(int x, int y) {
    if (fast()) return selfAncestor(x, y);
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
    if (fast()) return oldestSelfAncestorToSee(x, y);
    auto k = key(x, y);
    auto it = oldestSelfAncestorCache.find(k);
    if (it != oldestSelfAncestorCache.end()) return it->second;
    int r = oldestSelfAncestorToSee(x, y);
    oldestSelfAncestorCache[k] = r;
    return r;
  }
  int oldestSelfAncestorToSee(int x, int y) {  // hashgraph.go:166-177
    if (!getEvent(x) || !getEvent(y)) return -1;
    const int cx = events[x].creator;
    if (fdIx(y)[cx] <= events[x].index) return fdId(y)[cx];
    return -1;
  }
  bool StronglySee(int x, int y) {
    if (fast()) return stronglySee(x, y);
    auto k = key(x, y);
    auto it = stronglySeeCache.find(k);
    if (it != stronglySeeCache.end()) return it->second;
    bool s = stronglySee(x, y);
    stronglySeeCache[k] = s;
    return s;
  }
  bool stronglySee(int x, int y) {  // hashgraph.go:189-208
    if (!getEvent(x) || !getEvent(y)) return false;
    const int32_t* la = laIx(x);
    const int32_t* fd = fdIx(y);
    int c = 0;
    for (int i = 0; i < n; i++) c += la[i] >= fd[i];
    return c >= SuperMajority();
  }
  int ParentRound(int x) {
    if (fast() && getEvent(x)) {
      int& m = parentRoundMemo[x];
      if (m == kUnset) m = parentRound(x);
      return m;
    }
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
    if (fast()) {  // the count of RoundWitnesses(pr) x strongly sees; order-free, so from wkeys
      auto it = rounds.find(pr);
      if (it == rounds.end()) return false;
      const std::vector<int>& w = it->second.wkeys;
      const int sm = SuperMajority(), m = (int)w.size();
      int c = 0;
      for (int k = 0; k < m && c < sm && c + (m - k) >= sm; k++) c += stronglySee(x, w[k]);
      return c >= sm;
    }
    int c = 0;
    for (int w : RoundWitnesses(pr))
      if (StronglySee(x, w)) c++;
    return c >= SuperMajority();
  }
  int Round(int x) {
    if (fast() && getEvent(x)) {
      int& m = roundMemo[x];
      if (m == kUnset) {
        int r = round(x);
        roundMemo[x] = r;  // round() may grow nothing, but keep the write after it
        return r;
      }
      return m;
    }
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
  //  -4 other-parent not known, -5 self-parent not last known,
  //  -6 index outside this oracle's int32 coordinate range (not a reference error).
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
    if (e.index < INT32_MIN || e.index >= kFdUnset) {
      last_error = "Index outside the oracle's int32 coordinate range";
      return -6;
    }
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
    if (scale) {
      parentRoundMemo.push_back(kUnset);
      roundMemo.push_back(kUnset);
      added.push_back(0);
    }
    UpdateAncestorFirstDescendant(id);
    undetermined.push_back(id);
    return id;
  }

  void InitEventCoordinates(Event& e, int id) {  // hashgraph.go:399-463
    e.co.reset(new int32_t[4 * (size_t)n]);
    int32_t* la = e.co.get();
    int32_t* fd = la + n;
    int32_t* lah = la + 2 * n;
    int32_t* fdh = la + 3 * n;
    for (int i = 0; i < n; i++) {
      la[i] = -1;
      lah[i] = -1;
      fd[i] = kFdUnset;
      fdh[i] = -1;
    }
    if (e.sp < 0 && e.op < 0) {
      // all -1
    } else if (e.sp < 0) {
      std::memcpy(la, laIx(e.op), n * 4);
      std::memcpy(lah, laId(e.op), n * 4);
    } else if (e.op < 0) {
      std::memcpy(la, laIx(e.sp), n * 4);
      std::memcpy(lah, laId(e.sp), n * 4);
    } else {
      std::memcpy(la, laIx(e.sp), n * 4);
      std::memcpy(lah, laId(e.sp), n * 4);
      const int32_t* opla = laIx(e.op);
      const int32_t* oplah = laId(e.op);
      for (int i = 0; i < n; i++)
        if (la[i] < opla[i]) {
          la[i] = opla[i];
          lah[i] = oplah[i];
        }
    }
    fd[e.creator] = (int32_t)e.index;
    fdh[e.creator] = id;
    la[e.creator] = (int32_t)e.index;
    lah[e.creator] = id;
  }

  void UpdateAncestorFirstDescendant(int id) {  // hashgraph.go:466-494
    const int c = events[id].creator;
    const int32_t index = (int32_t)events[id].index;
    const int32_t* lah = laId(id);
    for (int i = 0; i < n; i++) {
      int ah = lah[i];
      while (ah >= 0) {
        int32_t* a = co(ah);
        if (a[n + c] == kFdUnset) {
          a[n + c] = index;
          a[3 * n + c] = id;
          ah = events[ah].sp;
        } else {
          break;
        }
      }
    }
  }

  // ---------------- consensus (hashgraph.go:573-760) ----------------
  void DivideRounds() {  // hashgraph.go:573-588
    if (fast()) {
      for (int x : undetermined) {
        int r = Round(x);
        bool w = Witness(x);
        if (!added[x]) {  // AddEvent of an event already in its round is a no-op
          rounds[r].AddEvent(x, w);
          added[x] = 1;
        }
      }
      return;
    }
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
    if (fast()) return DecideFameScale();
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

  // Scale mode DecideFame: the loops above with the votes of one (i, x) as a
  // bitset over round j's witnesses (bit set iff vote(y, x) was set true in this
  // call; unset and false both read as nay) and ssWitnesses(y) as a bitset over
  // round j-1's witnesses.  Rounds are contiguous here (no external SetRound),
  // so rounds[i] exists for every i < Rounds().
  void DecideFameScale() {
    const int start = has_lcr ? lcr + 1 : 0;
    const int R = Rounds();
    if (start >= R - 1) return;
    if (rounds.begin()->first != 0 || rounds.rbegin()->first != R - 1) die("rounds not contiguous", R);
    const int SM = SuperMajority();
    const int nr = R - start;
    std::vector<std::vector<int>> W(nr);
    for (int j = start; j < R; j++) W[j - start] = ordered(rounds.at(j).wkeys);
    // ssb[j][ys]: the witnesses of round j-1 that witness ys of round j strongly sees
    std::vector<std::vector<uint64_t>> ssb(nr);
    std::vector<std::vector<uint8_t>> ssOk(nr);
    auto ss = [&](int j, int ys) -> const uint64_t* {
      const int jj = j - start;
      const std::vector<int>& Wp = W[jj - 1];
      const int pw = ((int)Wp.size() + 63) / 64;
      if (ssb[jj].empty()) {
        ssb[jj].assign(W[jj].size() * (size_t)pw + 1, 0);
        ssOk[jj].assign(W[jj].size(), 0);
      }
      uint64_t* s = &ssb[jj][(size_t)ys * pw];
      if (!ssOk[jj][ys]) {
        const int y = W[jj][ys];
        for (int ws = 0; ws < (int)Wp.size(); ws++)
          if (stronglySee(y, Wp[ws])) s[ws >> 6] |= 1ull << (ws & 63);
        ssOk[jj][ys] = 1;
      }
      return s;
    };
    std::vector<uint64_t> prev, cur;
    for (int i = start; i < R - 1; i++) {
      RoundInfo& roundInfo = rounds.at(i);
      const std::vector<int>& Wi = W[i - start];
      const int nx = (int)Wi.size();
      int prevWords = 0;
      for (int j = i + 1; j < R; j++) {
        const std::vector<int>& Wj = W[j - start];
        const int ny = (int)Wj.size();
        const int cw = (ny + 63) / 64;
        const int diff = j - i;
        cur.assign((size_t)nx * cw + 1, 0);
        for (int xs = 0; xs < nx; xs++) {
          const int x = Wi[xs];
          uint64_t* cv = &cur[(size_t)xs * cw];
          const uint64_t* pv = prev.data() + (size_t)xs * prevWords;
          for (int ys = 0; ys < ny; ys++) {
            const int y = Wj[ys];
            if (diff == 1) {
              if (ancestor(y, x)) cv[ys >> 6] |= 1ull << (ys & 63);
              continue;
            }
            const uint64_t* s = ss(j, ys);
            int yays = 0, tot = 0;
            for (int k = 0; k < prevWords; k++) {
              yays += __builtin_popcountll(s[k] & pv[k]);
              tot += __builtin_popcountll(s[k]);
            }
            const int nays = tot - yays;
            bool v = false;
            int t = nays;
            if (yays >= nays) { v = true; t = yays; }
            if (diff % n != 0) {  // normal round
              if (t >= SM) {
                auto prevE = roundInfo.events.find(x);
                if (prevE != roundInfo.events.end() && prevE->second.famous != Undefined) {
                  stat_redecided++;
                  if (prevE->second.famous != (v ? True : False)) stat_flipped++;
                }
                roundInfo.SetFame(x, v);
                break;  // break out of y loop
              } else if (v) {
                cv[ys >> 6] |= 1ull << (ys & 63);
              }
            } else {  // coin round
              stat_coin_evals++;
              if (t < SM) {
                stat_coin_votes++;
                v = events[y].coin;
              }
              if (v) cv[ys >> 6] |= 1ull << (ys & 63);
            }
          }
        }
        prev.swap(cur);
        prevWords = cw;
      }
      if (roundInfo.undecided == 0 && (!has_lcr || i > lcr)) setLastConsensusRound(i);
    }
  }

  int64_t MedianTimestamp(const std::vector<int>& hashes) {  // hashgraph.go:762-770
    std::vector<int64_t> t;
    for (int x : hashes) t.push_back(getEvent(x) ? events[x].ts : kZeroTime);
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  }

  void DecideRoundReceived() {  // hashgraph.go:676-721
    if (fast()) return DecideRoundReceivedScale();
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

  // Scale mode DecideRoundReceived: See(w, x) is laIx(w)[creator(x)] >= index(x),
  // so |{w in F : See(w, x)}| > |F|/2 iff index(x) <= theta(creator(x)), the
  // (|F|/2+1)-th largest of laIx(w)[creator(x)] over the famous witnesses F.
  // The median is order-free, so F's iteration order does not matter.
  void DecideRoundReceivedScale() {
    const int R = Rounds();
    if ((int)thetas.size() < R) thetas.resize(R);
    std::vector<int32_t> col;
    auto prep = [&](int i) -> Theta& {
      RoundInfo& tr = rounds.at(i);
      Theta& T = thetas[i];
      if (T.version != tr.version) {
        T.version = tr.version;
        T.famous.clear();
        for (int w : tr.wkeys)
          if (tr.events.at(w).famous == True) T.famous.push_back(w);
        T.th.assign(n, INT32_MIN);
        const int m = (int)T.famous.size();
        if (m > 0) {
          const int need = m / 2 + 1;  // count > m/2
          col.resize(m);
          for (int c = 0; c < n; c++) {
            for (int k = 0; k < m; k++) col[k] = laIx(T.famous[k])[c];
            std::nth_element(col.begin(), col.begin() + (need - 1), col.end(), std::greater<int32_t>());
            T.th[c] = col[need - 1];
          }
        }
      }
      return T;
    };
    std::vector<int64_t> t;
    for (int x : undetermined) {
      int r = Round(x);
      Event& ex = events[x];
      const int cx = ex.creator;
      for (int i = r + 1; i < R; i++) {
        if (rounds.at(i).undecided != 0) continue;
        Theta& T = prep(i);
        if (T.famous.empty() || (int64_t)T.th[cx] < ex.index) continue;
        ex.has_rr = true;
        ex.rr = i;
        const int32_t* xfd = fdIx(x);
        const int32_t* xfdh = fdId(x);
        t.clear();
        for (int a : T.famous) {
          if ((int64_t)laIx(a)[cx] < ex.index) continue;  // !See(a, x)
          const int ca = events[a].creator;
          const int o = xfd[ca] <= events[a].index ? xfdh[ca] : -1;  // OldestSelfAncestorToSee(a, x)
          t.push_back(getEvent(o) ? events[o].ts : kZeroTime);
        }
        std::sort(t.begin(), t.end());
        ex.cts = t[t.size() / 2];
        break;
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
    if (fast() && release_lag >= 0) Release();
  }

  // Scale mode: drop the coordinates of a prefix of ordered events whose round
  // lies release_lag rounds behind LastConsensusRound.  Nothing on the path reads
  // them again in a gossip stream; a read aborts (co()), so a finished run is exact.
  void Release() {
    if (!has_lcr) return;
    while (release_next < events.size()) {
      Event& e = events[release_next];
      if (!e.has_rr || roundMemo[release_next] == kUnset || roundMemo[release_next] + release_lag >= lcr) break;
      e.co.reset();
      release_next++;
    }
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
// flags: bit 0 = scale mode (see the header; applies with order_seed 0 only)
void* hgo_create2(int n, uint64_t order_seed, int flags) {
  Oracle* o = new Oracle(n, order_seed);
  o->scale = (flags & 1) != 0;
  return o;
}
// Scale mode: release the coordinates of ordered events `lag` rounds behind LCR (-1: never).
void hgo_set_release(void* h, int lag) { ((Oracle*)h)->release_lag = lag; }
int hgo_is_scale(void* h) { return ((Oracle*)h)->fast(); }
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
  const int32_t* la = o->laIx(x);
  const int32_t* fd = o->fdIx(x);
  for (int i = 0; i < o->n; i++) {
    if (la_idx) la_idx[i] = la[i];
    if (la_hash) la_hash[i] = o->laId(x)[i];
    if (fd_idx) fd_idx[i] = fd[i] == kFdUnset ? kMaxInt64 : fd[i];
    if (fd_hash) fd_hash[i] = o->fdId(x)[i];
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
    RoundEvent e{witness[i] != 0, (Trilean)fame[i]};
    ri.events[ids[i]] = e;
    ri.keys.push_back(ids[i]);
    if (e.witness) {
      ri.wkeys.push_back(ids[i]);
      if (e.famous == Undefined) ri.undecided++;
    }
  }
  o->rounds[r] = ri;
  o->seeded = true;
}

// Bulk reads for the golden generators: Round / Witness of ids [0, E), round
// received and consensus timestamp (0 when not received), and the fame of every
// (round, creator) witness slot (-1 = no witness; 0/1/2 = Undefined/True/False).
void hgo_event_rounds(void* h, int32_t* round, uint8_t* wit) {
  Oracle* o = (Oracle*)h;
  for (int x = 0; x < (int)o->events.size(); x++) {
    round[x] = o->Round(x);
    wit[x] = o->Witness(x);
  }
}
void hgo_event_received(void* h, int32_t* rr, int64_t* cts) {
  Oracle* o = (Oracle*)h;
  for (size_t x = 0; x < o->events.size(); x++) {
    rr[x] = o->events[x].has_rr ? o->events[x].rr : -1;
    cts[x] = o->events[x].has_rr ? o->events[x].cts : 0;
  }
}
void hgo_fame_table(void* h, int8_t* out, int R) {
  Oracle* o = (Oracle*)h;
  std::memset(out, -1, (size_t)R * o->n);
  for (int r = 0; r < R; r++) {
    auto it = o->rounds.find(r);
    if (it == o->rounds.end()) continue;
    for (int w : it->second.keys) {
      const RoundEvent& e = it->second.events.at(w);
      if (e.witness) out[(size_t)r * o->n + o->events[w].creator] = (int8_t)e.famous;
    }
  }
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
