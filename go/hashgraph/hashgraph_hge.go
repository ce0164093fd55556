// Package hashgraph: babble's consensus package with the ordering hot path on
// the MI355X engine (libhge.so, include/hge.h).
//
// This file replaces /root/reference/hashgraph/hashgraph.go (and, with
// inmem_store_hge.go, caches.go, inmem_store.go and consensus_sorter.go).
// event.go, roundInfo.go and store.go are kept as they are.  The exported API
// (Hashgraph fields and methods, NewHashgraph, the Store interface) is
// unchanged, so node/core.go, node/node.go, net/ and proxy/ compile as before.
//
// What stays on the host, in Go: ECDSA Verify and the SHA-256 event hash
// (event.go:140-186), the hash <-> engine-id map, the full Event structs
// (Diff, ToWire, GetEventTransactions) and the commitCh send.  Everything the
// ordering path computes -- coordinates, rounds, witnesses, fame, round
// received, consensus timestamps, the consensus order -- comes from the engine.
//
// Not compiled in this repository's image (no Go toolchain); every method is a
// direct forward to one C entry point, so the shim stays mechanical.  See
// INTEGRATION.md for the build line and the semantics the caller must know.
package hashgraph

/*
#cgo LDFLAGS: -lhge
#include <stdlib.h>
#include "hge.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"math"
	"sort"
	"time"

	"github.com/Sirupsen/logrus"
)

// Hashgraph keeps the reference's exported fields (hashgraph.go:30-49).
type Hashgraph struct {
	Participants            map[string]int //[public key] => id
	ReverseParticipants     map[int]string //[id] => public key
	Store                   Store          //events (full structs) and the engine-backed views
	UndeterminedEvents      []string       //[index] => hash
	LastConsensusRound      *int           //index of last round where the fame of all witnesses has been decided
	LastCommitedRoundEvents int            //number of events in round before LastConsensusRound
	ConsensusTransactions   int            //number of consensus transactions
	commitCh                chan []Event   //channel for committing events

	eng   *C.hge_engine
	store *InmemStore // the engine-backed store (owns the hash <-> id maps)

	logger *logrus.Logger
}

// NewHashgraph (hashgraph.go:51-76).  The store must be this package's
// engine-backed InmemStore (NewInmemStore): it keeps the full Events in an
// unbounded map and answers the Store views from the engine.
func NewHashgraph(participants map[string]int, store Store, commitCh chan []Event, logger *logrus.Logger) Hashgraph {
	if logger == nil {
		logger = logrus.New()
		logger.Level = logrus.DebugLevel
	}
	reverseParticipants := make(map[int]string)
	for pk, id := range participants {
		reverseParticipants[id] = pk
	}
	s, ok := store.(*InmemStore)
	if !ok {
		panic("hashgraph: the MI355X engine needs the engine-backed *InmemStore (NewInmemStore)")
	}
	h := Hashgraph{
		Participants:        participants,
		ReverseParticipants: reverseParticipants,
		Store:               store,
		commitCh:            commitCh,
		store:               s,
		logger:              logger,
	}
	capacity := C.int64_t(s.cacheSize)
	if capacity < 1<<16 {
		capacity = 1 << 16 // a sizing hint only: the engine's tables grow
	}
	if rc := C.hge_create(C.int32_t(len(participants)), capacity, 0, 0, &h.eng); rc != C.HGE_OK {
		panic(fmt.Sprintf("hge_create: status %d", int(rc)))
	}
	// rolling views of the Store (ParticipantEvents, ConsensusEvents) follow cacheSize
	C.hge_set_cache_size(h.eng, C.int64_t(s.cacheSize))
	s.bind(h.eng, participants)
	return h
}

// Close releases the engine (device tables and stream).
func (h *Hashgraph) Close() {
	if h.eng != nil {
		C.hge_destroy(h.eng)
		h.eng = nil
	}
}

func (h *Hashgraph) SuperMajority() int {
	return 2*len(h.Participants)/3 + 1
}

func (h *Hashgraph) engineErr() error {
	return errors.New(C.GoString(C.hge_last_error(h.eng)))
}

// id of a known event hash; -1 for "" and unknown hashes
func (h *Hashgraph) id(x string) C.int32_t {
	if id, ok := h.store.ids[x]; ok {
		return id
	}
	return -1
}

// ---- predicates (hashgraph.go:83-208): a lookup error reads as false / "" ----

func (h *Hashgraph) Ancestor(x, y string) bool {
	a, b := h.id(x), h.id(y)
	return a >= 0 && b >= 0 && C.hge_ancestor(h.eng, a, b) == 1
}

func (h *Hashgraph) SelfAncestor(x, y string) bool {
	a, b := h.id(x), h.id(y)
	return a >= 0 && b >= 0 && C.hge_self_ancestor(h.eng, a, b) == 1
}

func (h *Hashgraph) See(x, y string) bool {
	return h.Ancestor(x, y)
}

func (h *Hashgraph) OldestSelfAncestorToSee(x, y string) string {
	a, b := h.id(x), h.id(y)
	if a < 0 || b < 0 {
		return ""
	}
	return h.store.hash(C.hge_oldest_self_ancestor_to_see(h.eng, a, b))
}

func (h *Hashgraph) StronglySee(x, y string) bool {
	a, b := h.id(x), h.id(y)
	return a >= 0 && b >= 0 && C.hge_strongly_see(h.eng, a, b) == 1
}

// ---- rounds (hashgraph.go:211-326) ----

func (h *Hashgraph) ParentRound(x string) int {
	a := h.id(x)
	if a < 0 {
		return -1
	}
	return int(C.hge_parent_round(h.eng, a))
}

func (h *Hashgraph) Witness(x string) bool {
	a := h.id(x)
	return a >= 0 && C.hge_is_witness(h.eng, a) == 1
}

func (h *Hashgraph) RoundInc(x string) bool {
	a := h.id(x)
	return a >= 0 && C.hge_round_inc(h.eng, a) == 1
}

func (h *Hashgraph) Round(x string) int {
	a := h.id(x)
	if a < 0 {
		return -1
	}
	return int(C.hge_round_of(h.eng, a))
}

func (h *Hashgraph) RoundDiff(x, y string) (int, error) {
	if x == "" {
		return math.MinInt64, fmt.Errorf("x is empty")
	}
	if y == "" {
		return math.MinInt64, fmt.Errorf("y is empty")
	}
	a, b := h.id(x), h.id(y)
	if a < 0 || b < 0 {
		return math.MinInt64, fmt.Errorf("event not found")
	}
	var d C.int32_t
	if C.hge_round_diff(h.eng, a, b, &d) != C.HGE_OK {
		return math.MinInt64, h.engineErr()
	}
	return int(d), nil
}

// ---- insertion (hashgraph.go:328-571) ----

// InsertEvent (hashgraph.go:328-363): Verify and the hash stay here; admission
// (FromParentsLatest), coordinates and the per-creator lists are the engine's.
func (h *Hashgraph) InsertEvent(event Event) error {
	if ok, err := event.Verify(); !ok {
		if err != nil {
			return err
		}
		return fmt.Errorf("Invalid signature")
	}
	return h.insert(&event)
}

func (h *Hashgraph) parentRef(x string) C.int32_t {
	if x == "" {
		return C.HGE_NONE
	}
	if id, ok := h.store.ids[x]; ok {
		return id
	}
	return C.HGE_UNKNOWN
}

func (h *Hashgraph) insert(event *Event) error {
	creator, ok := h.Participants[event.Creator()]
	if !ok {
		return fmt.Errorf("Could not find fake creator id")
	}
	var ev C.hge_event
	ev.creator = C.int32_t(creator)
	ev.index = C.int32_t(event.Index())
	ev.self_parent = h.parentRef(event.SelfParent())
	ev.other_parent = h.parentRef(event.OtherParent())
	ev.timestamp_ns = C.int64_t(event.Body.Timestamp.UnixNano())
	if event.S != nil {
		sb := event.S.Bytes() // big-endian; left-padded into 32 bytes
		if len(sb) > 32 {
			return fmt.Errorf("signature S longer than 32 bytes")
		}
		for i, b := range sb {
			ev.s[32-len(sb)+i] = C.uint8_t(b)
		}
	}
	hash, err := event.Hash() // SHA-256 of the body; hash[len/2] is the coin (middleBit, hashgraph.go:781-790)
	if err != nil {
		return err
	}
	for i := 0; i < 32 && i < len(hash); i++ {
		ev.hash[i] = C.uint8_t(hash[i])
	}
	ev.n_tx = C.int32_t(len(event.Body.Transactions))
	var status C.int32_t
	var accepted C.int64_t
	if rc := C.hge_insert_events(h.eng, &ev, 1, &status, &accepted); rc != C.HGE_OK {
		return h.engineErr()
	}
	hex := event.Hex()
	h.store.remember(hex, status)
	if err := h.SetWireInfo(event); err != nil {
		return err
	}
	if err := h.Store.SetEvent(*event); err != nil {
		return err
	}
	h.UndeterminedEvents = append(h.UndeterminedEvents, hex)
	return nil
}

// FromParentsLatest (hashgraph.go:366-396) is enforced by the engine at
// insertion (hge_insert_events statuses -2..-5); this dry check answers the
// same question for callers that ask before inserting.
func (h *Hashgraph) FromParentsLatest(event Event) error {
	creator, ok := h.Participants[event.Creator()]
	if !ok {
		return fmt.Errorf("Could not find fake creator id")
	}
	sp, op := event.SelfParent(), event.OtherParent()
	last := C.hge_last_from(h.eng, C.int32_t(creator))
	if sp == "" && op == "" && last == -1 {
		return nil
	}
	spID, ok := h.store.ids[sp]
	if !ok {
		return fmt.Errorf("Self-parent not known (%s)", sp)
	}
	spEv, _ := h.Store.GetEvent(sp)
	if spEv.Creator() != event.Creator() {
		return fmt.Errorf("Self-parent has different creator")
	}
	if _, ok := h.store.ids[op]; !ok {
		return fmt.Errorf("Other-parent not known (%s)", op)
	}
	if spID != last {
		return fmt.Errorf("Self-parent not last known event by creator")
	}
	return nil
}

// InitEventCoordinates (hashgraph.go:399-463): the engine computes the
// coordinates of every inserted event; for callers that build a hashgraph
// step by step (hashgraph_test.go:78-129) this inserts the event.
func (h *Hashgraph) InitEventCoordinates(event *Event) error {
	return h.insert(event)
}

// UpdateAncestorFirstDescendant (hashgraph.go:466-494): firstDescendants are
// derived in bulk on the device (hge_coords.hip); nothing to do per event.
func (h *Hashgraph) UpdateAncestorFirstDescendant(event Event) error {
	return nil
}

// Coordinates of an event as the reference's EventCoordinates
// (lastAncestors, firstDescendants; event.go:84-85).  Unset firstDescendants
// read math.MaxInt64 with an empty hash, as in the reference.
func (h *Hashgraph) Coordinates(x string) ([]EventCoordinates, []EventCoordinates, error) {
	a := h.id(x)
	n := len(h.Participants)
	if a < 0 || n == 0 {
		return nil, nil, ErrKeyNotFound
	}
	la := make([]C.int32_t, n)
	fd := make([]C.int32_t, n)
	if C.hge_coordinates(h.eng, a, &la[0], &fd[0]) != C.HGE_OK {
		return nil, nil, h.engineErr()
	}
	las := make([]EventCoordinates, n)
	fds := make([]EventCoordinates, n)
	for i := 0; i < n; i++ {
		las[i] = EventCoordinates{index: int(la[i])}
		if la[i] >= 0 {
			las[i].hash = h.store.hash(C.hge_participant_event(h.eng, C.int32_t(i), C.int64_t(la[i])))
		}
		fds[i] = EventCoordinates{index: math.MaxInt64}
		if fd[i] != math.MaxInt32 {
			fds[i] = EventCoordinates{index: int(fd[i]),
				hash: h.store.hash(C.hge_participant_event(h.eng, C.int32_t(i), C.int64_t(fd[i])))}
		}
	}
	return las, fds, nil
}

// SetWireInfo (hashgraph.go:497-524)
func (h *Hashgraph) SetWireInfo(event *Event) error {
	a := h.id(event.Hex())
	if a < 0 {
		return ErrKeyNotFound
	}
	var w [4]C.int32_t
	if C.hge_wire_info(h.eng, a, &w[0]) != C.HGE_OK {
		return h.engineErr()
	}
	event.SetWireInfo(int(w[0]), int(w[1]), int(w[2]), int(w[3]))
	return nil
}

// ReadWireInfo (hashgraph.go:526-571): (creator, index) pairs -> parent hashes.
func (h *Hashgraph) ReadWireInfo(wevent WireEvent) (*Event, error) {
	creator, ok := h.ReverseParticipants[wevent.Body.CreatorID]
	if !ok || len(creator) < 2 {
		return nil, fmt.Errorf("unknown creator id %d", wevent.Body.CreatorID)
	}
	creatorBytes, err := hexDecode(creator[2:])
	if err != nil {
		return nil, err
	}
	var sp, op C.int32_t
	rc := C.hge_read_wire_parents(h.eng, C.int32_t(wevent.Body.CreatorID),
		C.int32_t(wevent.Body.SelfParentIndex), C.int32_t(wevent.Body.OtherParentCreatorID),
		C.int32_t(wevent.Body.OtherParentIndex), &sp, &op)
	if err := storeErr(rc); err != nil {
		return nil, err
	}
	body := EventBody{
		Transactions:         wevent.Body.Transactions,
		Parents:              []string{h.store.hash(sp), h.store.hash(op)},
		Creator:              creatorBytes,
		Timestamp:            wevent.Body.Timestamp,
		Index:                wevent.Body.Index,
		selfParentIndex:      wevent.Body.SelfParentIndex,
		otherParentCreatorID: wevent.Body.OtherParentCreatorID,
		otherParentIndex:     wevent.Body.OtherParentIndex,
		creatorID:            wevent.Body.CreatorID,
	}
	return &Event{Body: body, R: wevent.R, S: wevent.S}, nil
}

// ---- consensus (hashgraph.go:573-760) ----

func (h *Hashgraph) DivideRounds() error {
	if C.hge_divide_rounds(h.eng) != C.HGE_OK {
		return h.engineErr()
	}
	return nil
}

func (h *Hashgraph) DecideFame() error {
	if C.hge_decide_fame(h.eng) != C.HGE_OK {
		return h.engineErr()
	}
	h.syncFields()
	return nil
}

func (h *Hashgraph) DecideRoundReceived() error {
	if C.hge_decide_round_received(h.eng) != C.HGE_OK {
		return h.engineErr()
	}
	return nil
}

// FindOrder (hashgraph.go:723-760): the engine commits this call's batch in
// consensus order; the shim maps ids back to Events and sends on commitCh.
func (h *Hashgraph) FindOrder() error {
	var n C.int64_t
	if C.hge_find_order(h.eng, nil, 0, &n) != C.HGE_OK { // size only: nothing is committed twice
		return h.engineErr()
	}
	// the batch is the tail of the consensus log
	total := int64(C.hge_consensus_count(h.eng))
	from := total - int64(n)
	batch := make([]Event, 0, int(n))
	if n > 0 {
		ids := make([]C.int32_t, int(n))
		srcs := make([]C.int32_t, int(n))
		C.hge_consensus_log(h.eng, C.int64_t(from), &ids[0], n)
		// MedianTimestamp returns the source event's own Body.Timestamp
		// (hashgraph.go:762-770): its location too, not only the instant
		if C.hge_consensus_timestamp_sources(h.eng, &ids[0], n, &srcs[0]) != C.HGE_OK {
			return h.engineErr()
		}
		for q, id := range ids {
			hex := h.store.hash(id)
			ev, err := h.Store.GetEvent(hex)
			if err != nil {
				return err
			}
			src, err := h.Store.GetEvent(h.store.hash(srcs[q]))
			if err != nil {
				return err
			}
			ev.SetRoundReceived(int(C.hge_round_received(h.eng, id)))
			ev.consensusTimestamp = src.Body.Timestamp
			h.store.events[hex] = ev
			batch = append(batch, ev)
		}
	}
	und := int64(C.hge_undetermined(h.eng, nil, 0))
	h.UndeterminedEvents = h.UndeterminedEvents[:0]
	if und > 0 {
		ids := make([]C.int32_t, und)
		C.hge_undetermined(h.eng, &ids[0], C.int64_t(und))
		for _, id := range ids {
			h.UndeterminedEvents = append(h.UndeterminedEvents, h.store.hash(id))
		}
	}
	h.syncFields()
	if h.commitCh != nil && len(batch) > 0 {
		h.commitCh <- batch
	}
	return nil
}

func (h *Hashgraph) syncFields() {
	if lcr := int(C.hge_last_consensus_round(h.eng)); lcr >= 0 {
		h.LastConsensusRound = &lcr
	} else {
		h.LastConsensusRound = nil
	}
	h.LastCommitedRoundEvents = int(C.hge_last_committed_round_events(h.eng))
	h.ConsensusTransactions = int(C.hge_consensus_transactions(h.eng))
}

// MedianTimestamp (hashgraph.go:762-770) over Store events (host-side helper).  Like
// the reference it indexes events[len/2], so an empty list panics there too.
func (h *Hashgraph) MedianTimestamp(eventHashes []string) time.Time {
	events := []Event{}
	for _, x := range eventHashes {
		ex, _ := h.Store.GetEvent(x)
		events = append(events, ex)
	}
	sort.Sort(ByTimestamp(events))
	return events[len(events)/2].Body.Timestamp
}

func (h *Hashgraph) ConsensusEvents() []string {
	return h.Store.ConsensusEvents()
}

// Known (hashgraph.go:777-779)
func (h *Hashgraph) Known() map[int]int {
	return h.Store.Known()
}
