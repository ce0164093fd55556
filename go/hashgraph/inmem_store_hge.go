package hashgraph

// The engine-backed Store (replaces /root/reference/hashgraph/inmem_store.go
// and caches.go).
//
// A store serves two callers, like the reference's:
//   * on its own (NewInmemStore, then SetEvent / SetRound / ... directly, as the
//     reference's store tests and tools do): the standalone Store of the C ABI
//     (hge_store_*: per-participant and consensus RollingLists, an LRU of
//     RoundInfos; include/hge.h) keeps the reference's containers for events that
//     were never inserted into a hashgraph and RoundInfos with any entries;
//   * bound to a Hashgraph (NewHashgraph): the per-creator lists, Known, the
//     consensus list and the rounds live in the engine, and the views keep the
//     reference's RollingList windows and ErrTooLate for the configured cacheSize
//     (caches.go:45-97, common/rolling_list.go:42-67); consensus math itself always
//     runs with infinite caches.  A RoundInfo set with SetRound is kept in the
//     standalone containers too, so GetRound returns exactly what was set (entries
//     the engine does not know included); rounds nobody set come from the engine.
// Full Events live in an UNBOUNDED map: GetEvent never misses an inserted event
// (the reference's LRU eventCache could evict, and FindOrder's GetEvent would then
// fail; SURVEY.md TL;DR 8).

/*
#include "hge.h"
*/
import "C"

import (
	"encoding/hex"
	"fmt"
)

type InmemStore struct {
	cacheSize    int
	events       map[string]Event    // hash => full Event, never evicted
	ids          map[string]C.int32_t // hash => engine id (bound)
	hashes       []string             // engine id => hash
	keys         map[string]int64     // hash => standalone key
	keyHash      []string             // standalone key => hash
	st           *C.hge_store         // the standalone containers
	eng          *C.hge_engine        // the bound Hashgraph's engine, or nil
	participants map[string]int
	extra        map[string]int // participants SetEvent met that were not registered
}

// NewInmemStore (inmem_store.go:27-36): usable on its own at once; NewHashgraph
// binds it to its engine.
func NewInmemStore(participants map[string]int, cacheSize int) *InmemStore {
	s := &InmemStore{
		cacheSize:    cacheSize,
		events:       make(map[string]Event),
		ids:          make(map[string]C.int32_t),
		keys:         make(map[string]int64),
		participants: participants,
		extra:        make(map[string]int),
	}
	if rc := C.hge_store_create(C.int32_t(len(participants)), C.int64_t(cacheSize), &s.st); rc != C.HGE_OK {
		panic(fmt.Sprintf("hge_store_create: status %d", int(rc)))
	}
	return s
}

func (s *InmemStore) bind(eng *C.hge_engine, participants map[string]int) {
	s.eng = eng
	s.participants = participants
}

func (s *InmemStore) bound() bool {
	return s.eng != nil
}

func (s *InmemStore) remember(hash string, id C.int32_t) {
	s.ids[hash] = id
	for C.int32_t(len(s.hashes)) <= id {
		s.hashes = append(s.hashes, "")
	}
	s.hashes[id] = hash
}

// hash of an engine id; "" for negative ids (HGE_NONE, "not found")
func (s *InmemStore) hash(id C.int32_t) string {
	if id < 0 || int(id) >= len(s.hashes) {
		return ""
	}
	return s.hashes[id]
}

// standalone key of a hash (a new one for a hash never seen)
func (s *InmemStore) key(hash string) C.int64_t {
	if k, ok := s.keys[hash]; ok {
		return C.int64_t(k)
	}
	k := int64(len(s.keyHash))
	s.keys[hash] = k
	s.keyHash = append(s.keyHash, hash)
	return C.int64_t(k)
}

func (s *InmemStore) keyToHash(k C.int64_t) string {
	if k < 0 || int(k) >= len(s.keyHash) {
		return ""
	}
	return s.keyHash[k]
}

func storeErr(rc C.int) error {
	switch rc {
	case C.HGE_OK:
		return nil
	case C.HGE_ERR_TOO_LATE:
		return ErrTooLate
	case C.HGE_ERR_NOT_FOUND:
		return ErrKeyNotFound
	}
	return fmt.Errorf("hge status %d", int(rc))
}

func hexDecode(s string) ([]byte, error) {
	return hex.DecodeString(s)
}

func (s *InmemStore) CacheSize() int {
	return s.cacheSize
}

// GetEvent (inmem_store.go:42-49).  On its own the store answers as the
// reference's eventCache does, an LRU of cacheSize events: a key evicted from it
// (every key at size 0) is not found, and a lookup refreshes it (common/lru.go
// Get), so the SetEvent that follows appends it to its creator's list again.
// Bound, every event the engine holds is found.
func (s *InmemStore) GetEvent(key string) (Event, error) {
	ev, ok := s.events[key]
	if !ok {
		return Event{}, ErrKeyNotFound
	}
	if !s.bound() {
		k, known := s.keys[key]
		if !known || C.hge_store_has_event(s.st, C.int64_t(k)) == 0 {
			return Event{}, ErrKeyNotFound
		}
	}
	return ev, nil
}

// SetEvent (inmem_store.go:51-64) keeps the full Event.  Bound, the engine already
// holds its coordinates and its place in the creator's list (hge_insert_events);
// on its own, the first SetEvent of a hash appends it to its creator's list.
// A creator that is not a registered participant gets its own list, as
// ParticipantEventsCache.Add creates one (caches.go:99-106).  The event is kept
// only once the store accepted it.
func (s *InmemStore) SetEvent(event Event) error {
	key := event.Hex()
	if s.bound() {
		s.events[key] = event
		return nil
	}
	c, err := s.creatorID(event.Creator())
	if err != nil {
		c = C.int32_t(len(s.participants) + len(s.extra))
		s.extra[event.Creator()] = int(c)
	}
	if err := storeErr(C.hge_store_set_event(s.st, s.key(key), c)); err != nil {
		return err
	}
	s.events[key] = event
	return nil
}

// a registered participant's id, or the list id SetEvent gave an unregistered one
func (s *InmemStore) creatorID(participant string) (C.int32_t, error) {
	if id, ok := s.participants[participant]; ok {
		return C.int32_t(id), nil
	}
	if id, ok := s.extra[participant]; ok && !s.bound() {
		return C.int32_t(id), nil
	}
	return -1, ErrKeyNotFound
}

// ParticipantEvents (caches.go:45-76): hashes from position skip on.
func (s *InmemStore) ParticipantEvents(participant string, skip int) ([]string, error) {
	c, err := s.creatorID(participant)
	if err != nil {
		return []string{}, err
	}
	res := []string{}
	if !s.bound() {
		var n C.int64_t
		if err := storeErr(C.hge_store_participant_events(s.st, c, C.int64_t(skip), nil, 0, &n)); err != nil {
			return []string{}, err
		}
		if n == 0 {
			return res, nil
		}
		keys := make([]C.int64_t, int(n))
		C.hge_store_participant_events(s.st, c, C.int64_t(skip), &keys[0], n, &n)
		for _, k := range keys {
			res = append(res, s.keyToHash(k))
		}
		return res, nil
	}
	var n C.int64_t
	if err := storeErr(C.hge_participant_events(s.eng, c, C.int64_t(skip), nil, 0, &n)); err != nil {
		return []string{}, err
	}
	if n == 0 {
		return res, nil
	}
	ids := make([]C.int32_t, int(n))
	if err := storeErr(C.hge_participant_events(s.eng, c, C.int64_t(skip), &ids[0], n, &n)); err != nil {
		return []string{}, err
	}
	for _, id := range ids {
		res = append(res, s.hash(id))
	}
	return res, nil
}

// ParticipantEvent (caches.go:78-84)
func (s *InmemStore) ParticipantEvent(participant string, index int) (string, error) {
	c, err := s.creatorID(participant)
	if err != nil {
		return "", err
	}
	if !s.bound() {
		var k C.int64_t
		if err := storeErr(C.hge_store_participant_event(s.st, c, C.int64_t(index), &k)); err != nil {
			return "", err
		}
		return s.keyToHash(k), nil
	}
	id := C.hge_participant_event(s.eng, c, C.int64_t(index))
	if id < 0 {
		return "", storeErr(C.int(id))
	}
	return s.hash(id), nil
}

// LastFrom (caches.go:86-97): "" when the creator has no event yet.
func (s *InmemStore) LastFrom(participant string) (string, error) {
	c, err := s.creatorID(participant)
	if err != nil {
		return "", err
	}
	if !s.bound() {
		var k C.int64_t
		var found C.int32_t
		if err := storeErr(C.hge_store_last_from(s.st, c, &k, &found)); err != nil {
			return "", err
		}
		if found == 0 {
			return "", nil
		}
		return s.keyToHash(k), nil
	}
	return s.hash(C.hge_last_from(s.eng, c)), nil
}

func (s *InmemStore) Known() map[int]int {
	n := len(s.participants)
	known := make(map[int]int, n)
	if n == 0 {
		return known
	}
	counts := make([]C.int32_t, n)
	if s.bound() {
		C.hge_known(s.eng, &counts[0])
	} else {
		C.hge_store_known(s.st, &counts[0])
	}
	for i, c := range counts {
		known[i] = int(c)
	}
	return known
}

// ConsensusEvents (inmem_store.go:88-95): the rolling window of the list.
func (s *InmemStore) ConsensusEvents() []string {
	res := []string{}
	if !s.bound() {
		n := C.hge_store_consensus_events(s.st, nil, 0)
		if n <= 0 {
			return res
		}
		keys := make([]C.int64_t, int(n))
		C.hge_store_consensus_events(s.st, &keys[0], n)
		for _, k := range keys {
			res = append(res, s.keyToHash(k))
		}
		return res
	}
	n := C.hge_consensus_events(s.eng, nil, 0)
	if n <= 0 {
		return res
	}
	ids := make([]C.int32_t, int(n))
	C.hge_consensus_events(s.eng, &ids[0], n)
	for _, id := range ids {
		res = append(res, s.hash(id))
	}
	return res
}

func (s *InmemStore) ConsensusEventsCount() int {
	if !s.bound() {
		return int(C.hge_store_consensus_count(s.st))
	}
	return int(C.hge_consensus_count(s.eng))
}

// AddConsensusEvent (inmem_store.go:102-105).  Bound, the engine appends to its
// consensus list in FindOrder.
func (s *InmemStore) AddConsensusEvent(key string) error {
	if !s.bound() {
		return storeErr(C.hge_store_add_consensus_event(s.st, s.key(key)))
	}
	if _, ok := s.ids[key]; !ok {
		return ErrKeyNotFound
	}
	return nil
}

// the RoundInfo set with SetRound for round r, if any
func (s *InmemStore) setRound(r int) (RoundInfo, bool) {
	var n C.int32_t
	if C.hge_store_get_round(s.st, C.int32_t(r), nil, nil, nil, 0, &n) != C.HGE_OK {
		return *NewRoundInfo(), false
	}
	ri := NewRoundInfo()
	if n == 0 {
		return *ri, true
	}
	keys := make([]C.int64_t, int(n))
	wit := make([]C.uint8_t, int(n))
	fame := make([]C.uint8_t, int(n))
	C.hge_store_get_round(s.st, C.int32_t(r), &keys[0], &wit[0], &fame[0], n, &n)
	for i := range keys {
		ri.Events[s.keyToHash(keys[i])] = RoundEvent{Witness: wit[i] != 0, Famous: Trilean(fame[i])}
	}
	return *ri, true
}

// GetRound (inmem_store.go:107-113).  On its own: the RoundInfo set with SetRound,
// as set.  Bound: the engine's live round -- every event of the round, the
// witnesses with their current fame -- with the SetRound copy's entries added
// only for hashes the engine does not know (non-inserted events); for an event
// the engine knows, the engine wins, so fame decided and events divided after a
// SetRound show up as they do in the reference, whose Hashgraph calls SetRound on
// every update (hashgraph.go:573-588, 654-661).
func (s *InmemStore) GetRound(r int) (RoundInfo, error) {
	set, have := s.setRound(r)
	if !s.bound() || r < 0 || r >= s.Rounds() {
		if have {
			return set, nil
		}
		return *NewRoundInfo(), ErrKeyNotFound
	}
	ri := s.engineRound(r)
	if have {
		for hash, re := range set.Events {
			if _, known := s.ids[hash]; !known {
				ri.Events[hash] = re
			}
		}
	}
	return *ri, nil
}

// the engine's round r: its events, the witnesses with their fame
func (s *InmemStore) engineRound(r int) *RoundInfo {
	ri := NewRoundInfo()
	var n C.int64_t
	C.hge_round_event_ids(s.eng, C.int32_t(r), nil, nil, 0, &n)
	if n > 0 {
		ids := make([]C.int32_t, int(n))
		wit := make([]C.uint8_t, int(n))
		C.hge_round_event_ids(s.eng, C.int32_t(r), &ids[0], &wit[0], n, &n)
		for i, id := range ids {
			re := RoundEvent{Witness: wit[i] != 0}
			if re.Witness {
				ev := s.events[s.hash(id)]
				if c, err := s.creatorID(ev.Creator()); err == nil {
					re.Famous = Trilean(C.hge_fame(s.eng, C.int32_t(r), c))
				}
			}
			ri.Events[s.hash(id)] = re
		}
	}
	return ri
}

// SetRound (inmem_store.go:115-118): any RoundInfo -- non-witness entries and hashes
// the store never saw included -- round-trips through GetRound.  Bound, its
// witness entries of inserted events also go to the engine's round tables.
func (s *InmemStore) SetRound(r int, round RoundInfo) error {
	keys := []C.int64_t{}
	kwit := []C.uint8_t{}
	kfame := []C.uint8_t{}
	ids := []C.int32_t{}
	wit := []C.uint8_t{}
	fame := []C.uint8_t{}
	for hash, re := range round.Events {
		w := C.uint8_t(0)
		if re.Witness {
			w = 1
		}
		keys = append(keys, s.key(hash))
		kwit = append(kwit, w)
		kfame = append(kfame, C.uint8_t(re.Famous))
		if id, ok := s.ids[hash]; ok && s.bound() && re.Witness {
			ids = append(ids, id)
			wit = append(wit, w)
			fame = append(fame, C.uint8_t(re.Famous))
		}
	}
	var err error
	if len(keys) == 0 {
		err = storeErr(C.hge_store_set_round(s.st, C.int32_t(r), nil, nil, nil, 0))
	} else {
		err = storeErr(C.hge_store_set_round(s.st, C.int32_t(r), &keys[0], &kwit[0], &kfame[0], C.int32_t(len(keys))))
	}
	if err != nil || !s.bound() {
		return err
	}
	if len(ids) == 0 {
		return storeErr(C.hge_set_round(s.eng, C.int32_t(r), nil, nil, nil, 0))
	}
	return storeErr(C.hge_set_round(s.eng, C.int32_t(r), &ids[0], &wit[0], &fame[0], C.int32_t(len(ids))))
}

// Rounds (inmem_store.go:120-122): on its own, the RoundInfos kept (the LRU's
// length); bound, the engine's Rounds().
func (s *InmemStore) Rounds() int {
	if !s.bound() {
		return int(C.hge_store_rounds(s.st))
	}
	return int(C.hge_rounds(s.eng))
}

func (s *InmemStore) RoundWitnesses(r int) []string {
	res := []string{}
	round, err := s.GetRound(r)
	if err != nil {
		return res
	}
	return round.Witnesses()
}

// RoundEvents (inmem_store.go:132-138): len(GetRound(r).Events)
func (s *InmemStore) RoundEvents(r int) int {
	if _, have := s.setRound(r); !have && s.bound() {
		if r < 0 || r >= s.Rounds() {
			return 0
		}
		return int(C.hge_round_events(s.eng, C.int32_t(r)))
	}
	ri, err := s.GetRound(r)
	if err != nil {
		return 0
	}
	return len(ri.Events)
}

func (s *InmemStore) Close() error {
	if s.st != nil {
		C.hge_store_destroy(s.st)
		s.st = nil
	}
	return nil
}
