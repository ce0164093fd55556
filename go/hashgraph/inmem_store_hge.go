package hashgraph

// The engine-backed Store (replaces /root/reference/hashgraph/inmem_store.go
// and caches.go).
//
// * Full Events live in an UNBOUNDED map: GetEvent never misses an inserted
//   event (the reference's LRU eventCache could evict, and FindOrder's
//   GetEvent would then fail; SURVEY.md TL;DR 8).
// * The per-creator lists, Known, the consensus list and the rounds live in
//   the engine.  ParticipantEvents / ParticipantEvent / ConsensusEvents keep the
//   reference's RollingList windows and ErrTooLate for the configured
//   cacheSize (caches.go:45-97, common/rolling_list.go:42-67); consensus math
//   itself always runs with infinite caches.

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
	ids          map[string]C.int32_t // hash => engine id
	hashes       []string             // engine id => hash
	eng          *C.hge_engine
	participants map[string]int
}

// NewInmemStore (inmem_store.go:27-36).  The store is bound to its engine by NewHashgraph.
func NewInmemStore(participants map[string]int, cacheSize int) *InmemStore {
	return &InmemStore{
		cacheSize:    cacheSize,
		events:       make(map[string]Event),
		ids:          make(map[string]C.int32_t),
		participants: participants,
	}
}

func (s *InmemStore) bind(eng *C.hge_engine, participants map[string]int) {
	s.eng = eng
	s.participants = participants
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

func (s *InmemStore) GetEvent(key string) (Event, error) {
	ev, ok := s.events[key]
	if !ok {
		return Event{}, ErrKeyNotFound
	}
	return ev, nil
}

// SetEvent keeps the full Event; the engine already holds its coordinates and
// its place in the creator's list (hge_insert_events).
func (s *InmemStore) SetEvent(event Event) error {
	s.events[event.Hex()] = event
	return nil
}

func (s *InmemStore) creatorID(participant string) (C.int32_t, error) {
	id, ok := s.participants[participant]
	if !ok {
		return -1, ErrKeyNotFound
	}
	return C.int32_t(id), nil
}

// ParticipantEvents (caches.go:45-76): hashes from position skip on.
func (s *InmemStore) ParticipantEvents(participant string, skip int) ([]string, error) {
	c, err := s.creatorID(participant)
	if err != nil {
		return []string{}, err
	}
	var n C.int64_t
	if err := storeErr(C.hge_participant_events(s.eng, c, C.int64_t(skip), nil, 0, &n)); err != nil {
		return []string{}, err
	}
	res := []string{}
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
	return s.hash(C.hge_last_from(s.eng, c)), nil
}

func (s *InmemStore) Known() map[int]int {
	n := len(s.participants)
	known := make(map[int]int, n)
	if n == 0 {
		return known
	}
	counts := make([]C.int32_t, n)
	C.hge_known(s.eng, &counts[0])
	for i, c := range counts {
		known[i] = int(c)
	}
	return known
}

// ConsensusEvents (inmem_store.go:88-95): the rolling window of the list.
func (s *InmemStore) ConsensusEvents() []string {
	res := []string{}
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
	return int(C.hge_consensus_count(s.eng))
}

// AddConsensusEvent: the engine appends to its consensus list in FindOrder.
func (s *InmemStore) AddConsensusEvent(key string) error {
	if _, ok := s.ids[key]; !ok {
		return ErrKeyNotFound
	}
	return nil
}

// GetRound (inmem_store.go:107-113): the round's witnesses with their fame.
// (RoundEvents(r) counts all of the round's events.)
func (s *InmemStore) GetRound(r int) (RoundInfo, error) {
	if r < 0 || r >= s.Rounds() {
		return *NewRoundInfo(), ErrKeyNotFound
	}
	ri := NewRoundInfo()
	for c := 0; c < len(s.participants); c++ {
		w := C.hge_round_witness(s.eng, C.int32_t(r), C.int32_t(c))
		if w < 0 {
			continue
		}
		ri.Events[s.hash(w)] = RoundEvent{Witness: true,
			Famous: Trilean(C.hge_fame(s.eng, C.int32_t(r), C.int32_t(c)))}
	}
	return *ri, nil
}

// SetRound (inmem_store.go:115-118): records the round's witnesses and fame.
func (s *InmemStore) SetRound(r int, round RoundInfo) error {
	ids := []C.int32_t{}
	wit := []C.uint8_t{}
	fame := []C.uint8_t{}
	for hash, re := range round.Events {
		id, ok := s.ids[hash]
		if !ok {
			return ErrKeyNotFound
		}
		w := C.uint8_t(0)
		if re.Witness {
			w = 1
		}
		ids = append(ids, id)
		wit = append(wit, w)
		fame = append(fame, C.uint8_t(re.Famous))
	}
	if len(ids) == 0 {
		return storeErr(C.hge_set_round(s.eng, C.int32_t(r), nil, nil, nil, 0))
	}
	return storeErr(C.hge_set_round(s.eng, C.int32_t(r), &ids[0], &wit[0], &fame[0], C.int32_t(len(ids))))
}

func (s *InmemStore) Rounds() int {
	return int(C.hge_rounds(s.eng))
}

func (s *InmemStore) RoundWitnesses(r int) []string {
	res := []string{}
	for c := 0; c < len(s.participants); c++ {
		if w := C.hge_round_witness(s.eng, C.int32_t(r), C.int32_t(c)); w >= 0 {
			res = append(res, s.hash(w))
		}
	}
	return res
}

func (s *InmemStore) RoundEvents(r int) int {
	return int(C.hge_round_events(s.eng, C.int32_t(r)))
}

func (s *InmemStore) Close() error {
	return nil
}
