// hge_store.cpp — the standalone Store (include/hge.h, "standalone Store"): the
// containers of the reference's InmemStore for a store used without a Hashgraph
// (its own tests, tools), host-only, no device.
//
//   * participant lists: ParticipantEventsCache over RollingLists
//     (hashgraph/caches.go:27-115, common/rolling_list.go:25-67): Add appends and
//     rolls the list to its last `size` items when it holds 2 * size; Get(skip)
//     and GetItem(index) answer ErrTooLate below the oldest item kept and
//     ErrKeyNotFound past the end; Known is the total per participant;
//   * the consensus list: a RollingList of the same size (inmem_store.go:88-104);
//   * rounds: an LRU of `size` RoundInfos (inmem_store.go:106-130,
//     common/lru.go:26-171): Add inserts or replaces and moves to the front,
//     evicting the least recently used past `size`; Get moves to the front;
//     Rounds() is the LRU's length.  A RoundInfo is any set of (event, witness,
//     famous) entries -- non-witnesses and events the store never saw included.
//   * events: an LRU of `size` keys (the eventCache, inmem_store.go:28-49): SetEvent
//     appends a key to its creator's list unless GetEvent finds it, then adds it;
//     a key evicted from the LRU is appended again by its next SetEvent, as in the
//     reference.
// Events are identified by the caller's int64 keys (the Go shim's hash <-> key map);
// event bodies stay with the caller.  Cache size 0 is the reference's NewLRU(0) /
// NewRollingList(0): the LRUs (events, rounds) keep nothing, the rolling lists never
// roll.  A negative size is refused (the reference's make() panics on it).
// A creator id >= n_participants is a participant the store was not created with:
// ParticipantEventsCache.Add creates its list on first use (caches.go:99-106); Known
// reports the n_participants registered ones only (the reference writes such an
// entry over participant 0's in map order, caches.go:108-115).
#include <cstdint>
#include <list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/hge.h"

namespace {

// common/rolling_list.go: the last window of items and the total ever added
struct RollingList {
  int64_t size = 0;  // <= 0: unbounded
  int64_t tot = 0;
  std::vector<int64_t> items;
  void add(int64_t v) {
    if (size > 0 && (int64_t)items.size() >= 2 * size)  // Roll: keep items[size:]
      items.erase(items.begin(), items.begin() + size);
    items.push_back(v);
    tot++;
  }
  int64_t oldest() const { return tot - (int64_t)items.size(); }
  // GetItem (rolling_list.go:42-53)
  int get_item(int64_t index, int64_t* out) const {
    if (index < oldest()) return HGE_ERR_TOO_LATE;
    const int64_t f = index - oldest();
    if (f >= (int64_t)items.size()) return HGE_ERR_NOT_FOUND;
    *out = items[(size_t)f];
    return HGE_OK;
  }
};

struct RoundEntry {
  int64_t key;
  uint8_t witness, famous;
};

}  // namespace

struct hge_store {
  int32_t n = 0;
  int64_t size = 0;
  std::vector<RollingList> part;  // ParticipantEventsCache (lists past n: unknown participants)
  std::vector<uint8_t> has_part;  // a list exists for the participant
  RollingList consensus;          // consensusCache
  // eventCache (LRU of keys): most recent first
  std::list<int64_t> ev_lru;
  std::unordered_map<int64_t, std::list<int64_t>::iterator> ev_where;

  bool ev_get(int64_t key) {  // LRU.Get: refreshes
    auto it = ev_where.find(key);
    if (it == ev_where.end()) return false;
    ev_lru.splice(ev_lru.begin(), ev_lru, it->second);
    return true;
  }
  void ev_add(int64_t key) {  // LRU.Add
    if (ev_get(key)) return;
    ev_lru.push_front(key);
    ev_where[key] = ev_lru.begin();
    if ((int64_t)ev_lru.size() > size) {
      ev_where.erase(ev_lru.back());
      ev_lru.pop_back();
    }
  }
  // roundCache (LRU): most recent first
  std::list<std::pair<int32_t, std::vector<RoundEntry>>> lru;
  std::map<int32_t, std::list<std::pair<int32_t, std::vector<RoundEntry>>>::iterator> where;

  const std::vector<RoundEntry>* get_round(int32_t r) {  // LRU.Get: moves to the front
    auto it = where.find(r);
    if (it == where.end()) return nullptr;
    lru.splice(lru.begin(), lru, it->second);
    return &lru.front().second;
  }
  void set_round(int32_t r, std::vector<RoundEntry> v) {  // LRU.Add
    auto it = where.find(r);
    if (it != where.end()) {
      it->second->second = std::move(v);
      lru.splice(lru.begin(), lru, it->second);
      return;
    }
    lru.emplace_front(r, std::move(v));
    where[r] = lru.begin();
    if ((int64_t)lru.size() > size) {  // removeOldest (size 0: the entry just added)
      where.erase(lru.back().first);
      lru.pop_back();
    }
  }
};

extern "C" {

int hge_store_create(int32_t n_participants, int64_t cache_size, hge_store** out) {
  if (!out || n_participants < 0 || cache_size < 0) return HGE_ERR_ARG;
  hge_store* s = new hge_store();
  s->n = n_participants;
  s->size = cache_size;
  s->part.resize((size_t)n_participants);
  s->has_part.assign((size_t)n_participants, 1);
  for (auto& p : s->part) p.size = cache_size;
  s->consensus.size = cache_size;
  *out = s;
  return HGE_OK;
}

void hge_store_destroy(hge_store* s) { delete s; }

static bool known_participant(const hge_store* s, int32_t c) {
  return c >= 0 && c < (int32_t)s->part.size() && s->has_part[(size_t)c];
}

// SetEvent (inmem_store.go:51-64): a key GetEvent does not find joins its creator's
// list (created for a participant not registered, caches.go:99-106), then the
// eventCache adds it
int hge_store_set_event(hge_store* s, int64_t key, int32_t creator) {
  if (!s || creator < 0) return HGE_ERR_ARG;
  if (!s->ev_get(key)) {
    if (creator >= (int32_t)s->part.size()) {
      s->part.resize((size_t)creator + 1);
      s->has_part.resize((size_t)creator + 1, 0);
    }
    if (!s->has_part[(size_t)creator]) {
      s->part[(size_t)creator] = RollingList();
      s->part[(size_t)creator].size = s->size;
      s->has_part[(size_t)creator] = 1;
    }
    s->part[(size_t)creator].add(key);
  }
  s->ev_add(key);
  return HGE_OK;
}

// GetEvent's success (inmem_store.go:41-49; refreshes the LRU entry)
int32_t hge_store_has_event(hge_store* s, int64_t key) { return s && s->ev_get(key) ? 1 : 0; }

// ParticipantEventsCache.Get (caches.go:45-76)
int hge_store_participant_events(hge_store* s, int32_t creator, int64_t skip, int64_t* keys_out, int64_t cap,
                                 int64_t* n_out) {
  if (!s || !n_out) return HGE_ERR_ARG;
  *n_out = 0;
  if (!known_participant(s, creator)) return HGE_ERR_NOT_FOUND;
  const RollingList& pe = s->part[(size_t)creator];
  if (skip >= pe.tot) return HGE_OK;
  if (skip < pe.oldest()) return HGE_ERR_TOO_LATE;
  const int64_t start = skip - pe.oldest();
  const int64_t n = (int64_t)pe.items.size() - start;
  for (int64_t k = 0; k < n && k < cap && keys_out; k++) keys_out[k] = pe.items[(size_t)(start + k)];
  *n_out = n;
  return HGE_OK;
}

// ParticipantEventsCache.GetItem (caches.go:78-84)
int hge_store_participant_event(hge_store* s, int32_t creator, int64_t index, int64_t* key_out) {
  if (!s || !key_out) return HGE_ERR_ARG;
  if (!known_participant(s, creator)) return HGE_ERR_NOT_FOUND;
  return s->part[(size_t)creator].get_item(index, key_out);
}

// ParticipantEventsCache.GetLast (caches.go:86-97): *found = 0 for "" (no event yet)
int hge_store_last_from(hge_store* s, int32_t creator, int64_t* key_out, int32_t* found) {
  if (!s || !key_out || !found) return HGE_ERR_ARG;
  if (!known_participant(s, creator)) return HGE_ERR_NOT_FOUND;
  const RollingList& pe = s->part[(size_t)creator];
  *found = pe.items.empty() ? 0 : 1;
  if (*found) *key_out = pe.items.back();
  return HGE_OK;
}

// Known (caches.go:108-115): the total per participant
int hge_store_known(hge_store* s, int32_t* counts_out) {
  if (!s || !counts_out) return HGE_ERR_ARG;
  for (int32_t c = 0; c < s->n; c++) counts_out[c] = (int32_t)s->part[(size_t)c].tot;
  return HGE_OK;
}

int hge_store_add_consensus_event(hge_store* s, int64_t key) {
  if (!s) return HGE_ERR_ARG;
  s->consensus.add(key);
  return HGE_OK;
}

// ConsensusEvents (inmem_store.go:88-95): the last window; returns its length
int64_t hge_store_consensus_events(hge_store* s, int64_t* keys_out, int64_t cap) {
  if (!s) return HGE_ERR_ARG;
  const int64_t n = (int64_t)s->consensus.items.size();
  for (int64_t k = 0; k < n && k < cap && keys_out; k++) keys_out[k] = s->consensus.items[(size_t)k];
  return n;
}

int64_t hge_store_consensus_count(hge_store* s) { return s ? s->consensus.tot : HGE_ERR_ARG; }

// SetRound (inmem_store.go:115-118): any RoundInfo
int hge_store_set_round(hge_store* s, int32_t round, const int64_t* keys, const uint8_t* witness,
                        const uint8_t* famous, int32_t n) {
  if (!s || n < 0 || (n > 0 && (!keys || !witness || !famous))) return HGE_ERR_ARG;
  std::vector<RoundEntry> v((size_t)n);
  for (int32_t i = 0; i < n; i++) v[(size_t)i] = {keys[i], witness[i], famous[i]};
  s->set_round(round, std::move(v));
  return HGE_OK;
}

// GetRound (inmem_store.go:107-113): *n_out entries (ErrKeyNotFound if absent)
int hge_store_get_round(hge_store* s, int32_t round, int64_t* keys_out, uint8_t* witness_out,
                        uint8_t* famous_out, int32_t cap, int32_t* n_out) {
  if (!s || !n_out) return HGE_ERR_ARG;
  *n_out = 0;
  const std::vector<RoundEntry>* v = s->get_round(round);
  if (!v) return HGE_ERR_NOT_FOUND;
  *n_out = (int32_t)v->size();
  for (int32_t i = 0; i < *n_out && i < cap; i++) {
    if (keys_out) keys_out[i] = (*v)[(size_t)i].key;
    if (witness_out) witness_out[i] = (*v)[(size_t)i].witness;
    if (famous_out) famous_out[i] = (*v)[(size_t)i].famous;
  }
  return HGE_OK;
}

int32_t hge_store_rounds(hge_store* s) { return s ? (int32_t)s->lru.size() : HGE_ERR_ARG; }

// RoundWitnesses (inmem_store.go:124-130): the round's witness keys; *n_out = 0 if absent
int hge_store_round_witnesses(hge_store* s, int32_t round, int64_t* keys_out, int32_t cap, int32_t* n_out) {
  if (!s || !n_out) return HGE_ERR_ARG;
  *n_out = 0;
  const std::vector<RoundEntry>* v = s->get_round(round);
  if (!v) return HGE_OK;
  for (const RoundEntry& e : *v)
    if (e.witness) {
      if (*n_out < cap && keys_out) keys_out[*n_out] = e.key;
      (*n_out)++;
    }
  return HGE_OK;
}

// RoundEvents (inmem_store.go:132-138): entries of the round, 0 if absent
int32_t hge_store_round_events(hge_store* s, int32_t round) {
  if (!s) return HGE_ERR_ARG;
  const std::vector<RoundEntry>* v = s->get_round(round);
  return v ? (int32_t)v->size() : 0;
}

}  // extern "C"
