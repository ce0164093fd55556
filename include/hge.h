/*
 * hge.h — C ABI of the MI355X hashgraph consensus-ordering engine.
 *
 * Drop-in boundary for babble's `hashgraph` package (mpitid/babble,
 * /root/reference/hashgraph).  A thin cgo shim (go/hashgraph/engine.go,
 * INTEGRATION.md) keeps the Go `Hashgraph` / `Store` method set and forwards
 * here; node/, net/ and proxy/ are untouched.  Plain pointers and sizes only.
 *
 * Events are identified by dense engine ids assigned in insertion order (the
 * shim keeps the hash <-> id map).  The signature check and hashing of
 * InsertEvent's front half run on host cores (hge_verify_events, hge_ingest
 * below); the consensus entry points take verified hge_event records.
 *
 * Threading: one handle is used by one thread at a time (the reference
 * serialises Core under Node.coreLock, node/node.go:167-169).
 * Errors: functions return HGE_OK or a negative hge_status; hge_last_error()
 * gives the reference's error text.
 */
#ifndef HGE_H
#define HGE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hge_engine hge_engine;

/* Status codes.  -1..-5 mirror the reference's InsertEvent errors. */
enum hge_status {
  HGE_OK = 0,
  HGE_ERR_CREATOR = -1,              /* "Could not find fake creator id"        hashgraph.go:453-456 */
  HGE_ERR_SELF_PARENT_UNKNOWN = -2,  /* "Self-parent not known"                 hashgraph.go:373-376 */
  HGE_ERR_SELF_PARENT_CREATOR = -3,  /* "Self-parent has different creator"     hashgraph.go:377-379 */
  HGE_ERR_OTHER_PARENT_UNKNOWN = -4, /* "Other-parent not known"                hashgraph.go:381-384 */
  HGE_ERR_SELF_PARENT_NOT_LAST = -5, /* "Self-parent not last known event..."   hashgraph.go:390-393 */
  /* Body.Index != position in the creator's chain.  DELIBERATE DEVIATION: the
   * reference accepts such an event and uses the claimed index in its coordinates
   * (hashgraph.go:455-460); the engine's tables are indexed by chain position, so
   * it refuses index-lying events (Byzantine input only: an honest Core always
   * creates head.Index+1, node/core.go:87-99).  INTEGRATION.md, tests. */
  HGE_ERR_INDEX = -6,
  /* device allocation failed.  (Chains have no length cap: at N > 32 a chain
   * reaching 65,534 events switches the engine from its uint16 position tables
   * to int32 ones) */
  HGE_ERR_CAPACITY = -7,
  HGE_ERR_ARG = -8,        /* bad argument */
  HGE_ERR_DEVICE = -9,     /* HIP runtime error */
  HGE_ERR_INTERNAL = -10,
  HGE_ERR_TOO_LATE = -11,  /* ErrTooLate  (store.go:22): below the rolling window  */
  HGE_ERR_NOT_FOUND = -12, /* ErrKeyNotFound (store.go:21)                         */
  HGE_ERR_SIGNATURE = -13, /* "Invalid signature"  (hashgraph.go:330-336)            */
  /* a split replay's parts did not cover the stream (walkers that never met, or an
   * event received outside every part's range): every part returns it together,
   * and the caller replays unsplit (babble_amd/dist.py).  Engine-only. */
  HGE_ERR_SPLIT = -14
};

/* Parent reference values. */
#define HGE_NONE (-1)    /* empty parent ""                                   */
#define HGE_UNKNOWN (-2) /* hash the caller could not resolve: "not known"    */

/* One event as handed over by the caller (Event, event.go:73-88). */
typedef struct hge_event {
  int32_t creator;       /* participant id (Participants[pubkey])                  */
  int32_t index;         /* Body.Index                                             */
  int32_t self_parent;   /* engine id, HGE_NONE or HGE_UNKNOWN  (Body.Parents[0])  */
  int32_t other_parent;  /* engine id, HGE_NONE or HGE_UNKNOWN  (Body.Parents[1])  */
  int64_t timestamp_ns;  /* Body.Timestamp                                         */
  uint8_t s[32];         /* signature S, unsigned big-endian (consensus tie-break) */
  uint8_t hash[32];      /* SHA-256 of the event; hash[16] is the coin bit         */
  int32_t n_tx;          /* len(Body.Transactions)                                 */
  int32_t reserved;
} hge_event;

/* ---- lifecycle ------------------------------------------------------------ */
/* NewHashgraph (hashgraph.go:51-76) + NewInmemStore (inmem_store.go:27-36).
 * capacity_events is a sizing hint: the device tables grow on demand up to HBM.
 * Consensus math always runs with the reference's infinite-cache contract
 * (SURVEY.md TL;DR 8); hge_set_cache_size only shapes the rolling views below.
 * No cap on events per creator (N > 32 switches to int32 positions past 65,534). */
int hge_create(int32_t n_participants, int64_t capacity_events, int32_t device,
               uint32_t flags, hge_engine** out);
void hge_destroy(hge_engine* h);
const char* hge_last_error(hge_engine* h);
int hge_reset(hge_engine* h); /* forget all events, keep allocations */

/* ---- ingest ---------------------------------------------------------------- */
/* InsertEvent (hashgraph.go:328-363) for n events in order.  Processing stops at
 * the first rejected event, like Core.Sync (node/core.go:137-145).  Accepted
 * events receive ids hge_event_count() .. +n_accepted-1; status_out[i] is the
 * id or a negative hge_status for the first rejection (may be NULL).  The
 * events before a rejection stay inserted: *n_accepted says how many. */
int hge_insert_events(hge_engine* h, const hge_event* ev, int64_t n, int32_t* status_out,
                      int64_t* n_accepted);

/* ---- host ingest pipeline (InsertEvent's front half) -------- */
/* Event.Verify (event.go:140-150) for n events on `threads` host threads (<= 0:
 * every core): body_hash_out[32 i] = SHA-256 of body i (EventBody.Hash, event.go:60-66:
 * the bytes are the gob encoding EventBody.Marshal produces, event.go:44-52;
 * bodies[body_off[i] .. body_off[i+1])), ok_out[i] = 1 iff sigs[64 i] = r || s
 * (big-endian) is a valid ECDSA P-256 signature of that hash under pubs[65 i], the
 * creator's uncompressed key (Body.Creator, crypto.ToECDSAPub crypto/utils.go:40-46;
 * a key that is not a curve point verifies nothing).  body_hash_out may be NULL.
 * Host code only: thread-safe, needs no engine, overlaps any device work. */
int hge_verify_events(int64_t n, const uint8_t* bodies, const int64_t* body_off, const uint8_t* pubs,
                      const uint8_t* sigs, int32_t threads, uint8_t* body_hash_out, int32_t* ok_out);
/* SHA-256 of n byte strings data[off[i] .. off[i+1]) (Event.Hash over the gob(Event)
 * bytes, event.go:169-179) into out[32 i], on `threads` host threads. */
int hge_sha256_batch(int64_t n, const uint8_t* data, const int64_t* off, int32_t threads, uint8_t* out);
/* InsertEvent with its signature check over a stream, in batches of k events with
 * RunConsensus after each batch (node/core.go:179-202), while a pool of `threads`
 * host threads verifies the next batch: the host crypto overlaps the device.  ev[i]
 * is event i's record, (bodies, body_off, sigs) as for hge_verify_events, and
 * keys[65 c] is participant c's uncompressed P-256 key: event i's signature is
 * checked under keys[65 * ev[i].creator], the key its creator id stands for.  In
 * the reference Body.Creator IS the key and the creator id is looked up from it
 * (hashgraph.go:51-76 Participants, :366-370), so a body signed by another
 * participant's key cannot pass as this creator's event: it is refused with
 * HGE_ERR_SIGNATURE here.  The caller derives ev[i] (creator, index, parents,
 * timestamp, hash) from the body it passes; the engine does not decode the body.
 * A creator id outside [0, N) is refused with HGE_ERR_CREATOR, as by
 * hge_insert_events.
 * The first event whose signature fails is refused with HGE_ERR_SIGNATURE and ends
 * the stream (the events before it stay inserted and their batch goes through
 * consensus), like InsertEvent inside Core.Sync; admission errors end it the same
 * way.  status_out[i] as for hge_insert_events; *n_accepted = events inserted;
 * times_out (may be NULL): [0] host ms spent verifying that the device did not
 * hide, [1] ms inside the insert + consensus calls, [2] wall ms. */
int hge_ingest(hge_engine* h, const hge_event* ev, int64_t n, const uint8_t* bodies, const int64_t* body_off,
               const uint8_t* keys, const uint8_t* sigs, int64_t k, int32_t threads, int32_t* status_out,
               int64_t* n_accepted, double* times_out);

/* ---- consensus (node/core.go:179-202) --------------------------------------- */
int hge_divide_rounds(hge_engine* h);          /* hashgraph.go:573-588 */
int hge_decide_fame(hge_engine* h);            /* hashgraph.go:598-664 */
int hge_decide_round_received(hge_engine* h);  /* hashgraph.go:676-721 (no commit) */
/* FindOrder (hashgraph.go:723-760): commits this call's batch in consensus order.
 * ids_out may be NULL; *n_out = batch size (ids beyond cap are dropped). */
int hge_find_order(hge_engine* h, int32_t* ids_out, int64_t cap, int64_t* n_out);
/* DivideRounds + DecideFame + FindOrder */
int hge_run_consensus(hge_engine* h, int32_t* ids_out, int64_t cap, int64_t* n_out);

/* ---- bulk replay (bench / Monte Carlo) --------------------------------------- */
/* Replays a whole submission stream on a fresh state: parents are submission
 * indices (-1 none); rejected submissions are skipped and status_out records
 * them; RunConsensus runs after each submission count in call_points (1-based,
 * strictly ascending, <= n_sub; anything else is HGE_ERR_ARG).  Results are identical to calling hge_insert_events and
 * hge_run_consensus at every call point.  order_out receives the full consensus
 * order, call_counts_out[c] the batch size of call c (both may be NULL). */
int hge_replay(hge_engine* h, const hge_event* ev, int64_t n_sub, const int64_t* call_points,
               int64_t n_calls, int32_t* status_out, int32_t* order_out, int64_t cap,
               int64_t* n_ordered, int64_t* call_counts_out);
/* Split form for timing: prepare (validate + stage in HBM) then run on the device. */
int hge_replay_prepare(hge_engine* h, const hge_event* ev, int64_t n_sub,
                       const int64_t* call_points, int64_t n_calls, int32_t* status_out);
int hge_replay_run(hge_engine* h, int64_t* n_ordered);
int hge_replay_fetch(hge_engine* h, int32_t* order_out, int64_t cap, int64_t* call_counts_out);
/* The consensus log without a copy: hge_replay_run delivers a replay's order into a
 * pinned host buffer sized at hge_replay_prepare (the batches FindOrder hands its
 * caller, hashgraph.go:744-757, all of them); *ids points at it (or at the log when
 * online calls followed) and stays valid until the next replay, consensus call or
 * hge_destroy. */
int hge_replay_order(hge_engine* h, const int32_t** ids, int64_t* n);

/* ---- a batch of independent hashgraphs (BASELINE config 5, Monte Carlo) -------- */
/* Many small hashgraphs (N <= 64 participants each) replayed together: every stage
 * is one launch over the whole batch and each graph's whole call schedule runs on
 * the device in bulk (the calls' DecideFame pairs, one fold over the calls, the
 * events' round received and medians, the call buckets' sorts), so a batch costs a
 * handful of launches however many graphs it holds (hge_batch.hip,
 * hge_batch_bulk.hip).  Per graph the semantics are
 * hge_replay's: parents are submission indices, admission (FromParentsLatest,
 * hashgraph.go:366-396, and the index rule of HGE_ERR_INDEX) happens in
 * hge_batch_add on the host, RunConsensus runs after every call point, and the
 * results are identical to hge_replay on the same stream. */
typedef struct hge_batch hge_batch;
int hge_batch_create(int32_t n_participants, int32_t device, hge_batch** out);
void hge_batch_destroy(hge_batch* b);
const char* hge_batch_last_error(hge_batch* b);
/* Admit one graph's stream (status_out[i]: the event's id in its graph, or a negative
 * hge_status) and stage it on the host; *graph_out = its index in the batch. */
int hge_batch_add(hge_batch* b, const hge_event* ev, int64_t n_sub, const int64_t* call_points, int64_t n_calls,
                  int32_t* status_out, int32_t* graph_out);
int hge_batch_stage(hge_batch* b); /* upload the added graphs to HBM (hge_batch_run does it if needed) */
int hge_batch_run(hge_batch* b, int64_t* n_ordered); /* replay every graph; *n_ordered = events ordered in all */
int32_t hge_batch_graphs(hge_batch* b);
/* After a run: info[8] = {accepted events, calls, Rounds(), LastConsensusRound (-1 nil),
 * LastCommitedRoundEvents, ConsensusTransactions, ordered events, undetermined events}. */
int hge_batch_info(hge_batch* b, int32_t g, int64_t* info);
/* Graph g's state (any pointer may be NULL; sizes from hge_batch_info): the consensus
 * order, per-call batch sizes, every event's round / witness flag / round received
 * (-1 none) / consensus timestamp (0 none), fame[Rounds()][N] (-1 no witness, 0
 * undecided, 1 famous, 2 not famous) and the undetermined list. */
int hge_batch_results(hge_batch* b, int32_t g, int32_t* order, int64_t* counts, int32_t* round, uint8_t* witness,
                      int32_t* rr, int64_t* cts, int8_t* fame, int32_t* undetermined);
/* device ms of the last run's stages (HIP events between the launches): coordinates,
 * firstDescendant runs, firstDescendant rows, rounds, DecideFame pairs, the call
 * fold and receive thresholds, round received and medians, the call buckets' order;
 * returns the count */
int hge_batch_kernel_ms(hge_batch* b, float* ms, int32_t cap);
/* graphs the last run replayed call by call (kb_consensus) because the bulk fold
 * could not hold them (more than 256 rounds, or a receive-interval table overflow) */
int64_t hge_batch_fallbacks(hge_batch* b);

/* ---- one hashgraph split across GPUs (babble_amd/dist.py) ------ */
/* Sharded replay.  Every rank stages the whole stream (hge_replay_prepare) and
 * makes the same plan: part p owns the events [ev_bounds[p], ev_bounds[p+1]) and
 * the calls [call_bounds[p], call_bounds[p+1]) (both ascending, covering the
 * staged stream and its calls).  hge_split_run replays with the plan:
 *  - every part computes the coordinates and walks the rounds frontier recurrence
 *    (DESIGN.md §4.2): the recurrence is sequential and cannot be split exactly
 *    (walkers started mid-stream rarely meet the true trajectory, §6); the
 *    firstDescendants timestamp rows are written for the part's candidates only;
 *  - DecideFame: the part decides the (round, call) pairs of the rounds whose first
 *    witness it owns, and the parts all-gather the decisions;
 *  - DecideRoundReceived / FindOrder: round received, consensus timestamp and the
 *    call buckets of the candidates [cand_lo[p], ev_bounds[p+1]) that its calls
 *    receive (cand_lo[p] <= ev_bounds[p]: events received late, from before the
 *    part's own range), then the parts all-gather their ordered slices;
 * every rank ends with the whole replay's state, identical to hge_replay_run.  A
 * candidate that no part covers makes every part return HGE_ERR_SPLIT (the caller
 * replays unsplit).  nparts <= 1 clears the plan.  N > 32 with N % 4 == 0 only.
 * The exchange: op 0 asks the caller for device memory of nparts slots of
 * bytes_per_part bytes (*buf, valid until the next op 0), op 1 all-gathers it in
 * place once this part's slot is filled and the engine stream is drained; the
 * callback returns 0, or nonzero to fail the replay.  Every part makes the same
 * calls with the same sizes (torch.distributed all_gather_into_tensor on RCCL). */
typedef int (*hge_exchange_fn)(void* ctx, int32_t op, int64_t bytes_per_part, void** buf);
int hge_split_plan(hge_engine* h, int32_t part, int32_t nparts, const int64_t* ev_bounds,
                   const int32_t* call_bounds, const int64_t* cand_lo);
int hge_split_exchange(hge_engine* h, hge_exchange_fn fn, void* ctx);
int hge_split_run(hge_engine* h, int64_t* n_ordered);
/* Measurement aid: on = 1 makes the next hge_replay_run record what every part of a
 * split contributes to the exchanges; afterwards hge_split_run without an exchange
 * (hge_split_exchange(h, NULL, NULL)) takes the other parts' slots from that record,
 * so one GPU runs and times each part of a G-way split alone (results identical to
 * the replay; scripts/analysis/split_emulate.py).  on = 0 drops the record. */
int hge_split_emulate(hge_engine* h, int32_t on);

/* Walk-only split (measured, kept for the record: DESIGN.md §6).  Every rank
 * computes everything; the rounds walk is walked by one walker per rank from its
 * own start: rank 0 from the true first frontier, rank p from the time cut at
 * p * E / nparts (hge_frontier_guess), until its rows pass `stopcut` (the next
 * rank's start) plus `extra` rows, or hmax rows.  The ranks all-gather their rows
 * (N ints each) and strongly-see bits (N * ceil(N/64) words each); the join
 * follows row equalities from rank 0's true trajectory (the recurrence is a
 * function of the row alone) and hge_split_finish installs the joined rows -- the
 * sequential walk resumes from the last joined row if the walkers did not meet
 * (at N = 256 they rarely do) -- and runs DivideRounds, DecideFame and FindOrder
 * at every call point.  Results are identical to hge_replay_run. */
int hge_split_begin(hge_engine* h);
int hge_frontier_guess(hge_engine* h, int32_t part, int32_t nparts, int32_t* start_out);
/* rows_out: hmax * N ints (row 0 = start; INT32_MAX = no event yet), ssc_out:
 * hmax * N * ceil(N/64) words (row 0 unused); *nrows rows written; *natural = 1
 * when the last row is the empty frontier (the walk ended). */
int hge_frontier_walk(hge_engine* h, const int32_t* start, const int32_t* stopcut, int32_t extra,
                      int32_t hmax, int32_t* rows_out, uint64_t* ssc_out, int32_t* nrows,
                      int32_t* natural);
/* rows [from, from + n) of the last walk (hge_frontier_walk with NULL outputs
 * keeps them on the device). */
int hge_frontier_rows(hge_engine* h, int32_t from, int32_t n, int32_t* rows_out, uint64_t* ssc_out);
/* rows: the joined true frontier rows 0 .. nrows-1 (natural: the walk ended after
 * them, i.e. Rounds() = nrows), ssc their strongly-see bits (row 0 unused). */
int hge_split_finish(hge_engine* h, const int32_t* rows, const uint64_t* ssc, int32_t nrows,
                     int32_t natural, int64_t* n_ordered);

/* ---- state queries --------------------------------------------------------- */
int64_t hge_event_count(hge_engine* h);
int32_t hge_participants(hge_engine* h);
int32_t hge_rounds(hge_engine* h);                    /* Store.Rounds()            */
int32_t hge_last_consensus_round(hge_engine* h);      /* -1 = nil                  */
int32_t hge_last_committed_round_events(hge_engine* h);
int64_t hge_consensus_transactions(hge_engine* h);
int64_t hge_consensus_count(hge_engine* h);           /* Store.ConsensusEventsCount */
/* Store.ConsensusEvents (inmem_store.go:88-95): the rolling window of the
 * consensus list (common/rolling_list.go:55-67) for the configured cache size;
 * the whole list when the cache size is 0 (unbounded).  Returns its length. */
int64_t hge_consensus_events(hge_engine* h, int32_t* ids_out, int64_t cap);
/* The unbounded consensus log from position `from` (commit stream; no window). */
int64_t hge_consensus_log(hge_engine* h, int64_t from, int32_t* ids_out, int64_t cap);
int64_t hge_undetermined(hge_engine* h, int32_t* ids_out, int64_t cap);
int hge_known(hge_engine* h, int32_t* counts_out);    /* Known(), n_participants ints */
int32_t hge_round_of(hge_engine* h, int32_t id);      /* Round(x) (after DivideRounds) */
int32_t hge_is_witness(hge_engine* h, int32_t id);    /* Witness(x)                    */
int32_t hge_round_witness(hge_engine* h, int32_t round, int32_t creator); /* id or -1 */
int32_t hge_fame(hge_engine* h, int32_t round, int32_t creator); /* 0 undef, 1 true, 2 false, -1 none */
int32_t hge_round_events(hge_engine* h, int32_t round);          /* Store.RoundEvents(r) */
/* Store.GetRound's events: every event of round r (insertion order) and its witness
 * flag; *n_out = their number (ids beyond cap are dropped). */
int hge_round_event_ids(hge_engine* h, int32_t round, int32_t* ids_out, uint8_t* witness_out, int64_t cap,
                        int64_t* n_out);
int32_t hge_round_received(hge_engine* h, int32_t id);           /* -1 = nil */
int64_t hge_consensus_timestamp(hge_engine* h, int32_t id);
/* MedianTimestamp's source (hashgraph.go:762-770: events[len(events)/2].Body.Timestamp):
 * for each id, the id of the event whose Body.Timestamp is its consensus timestamp --
 * OldestSelfAncestorToSee(w, x) for a famous witness w of x's round received that
 * sees x, at the median instant -- so a caller returns that event's own time.Time
 * (its zone included).  Among candidates sharing the instant the lowest creator is
 * chosen (the reference's sort.Sort over a map-ordered list leaves it unspecified).
 * -1 for an id with no round received. */
int hge_consensus_timestamp_sources(hge_engine* h, const int32_t* ids, int64_t n, int32_t* src_out);

/* Bulk reads for ids [0, min(cap, hge_event_count)): Round/Witness of every
 * event (DivideRounds state), and RoundReceived (-1 = nil) / consensus timestamp. */
int hge_event_rounds(hge_engine* h, int32_t* round_out, uint8_t* witness_out, int64_t cap);
int hge_event_received(hge_engine* h, int32_t* rr_out, int64_t* cts_out, int64_t cap);
/* Fame of every round slot, rounds [0, min(rounds, hge_rounds)) x n_participants,
 * row-major: hge_fame's encoding (RoundInfo.Events[w].Famous, roundInfo.go:24-36,
 * -1 = no witness of that creator in that round).  Returns the rounds written. */
int32_t hge_fame_table(hge_engine* h, int32_t rounds, int8_t* fame_out);

/* ---- Store semantics and the sync path (store.go:25-41, node/core.go:108-132) -- */
/* Store.CacheSize (inmem_store.go:38-40): size of the rolling windows of
 * ParticipantEvents / ParticipantEvent / ConsensusEvents; 0 = unbounded. */
int hge_set_cache_size(hge_engine* h, int64_t size);
int64_t hge_cache_size(hge_engine* h);
/* Store.ParticipantEvents(pk, skip) (caches.go:45-76): ids of the creator's
 * events from position `skip` on; HGE_ERR_TOO_LATE below the rolling window,
 * HGE_ERR_NOT_FOUND for an unknown creator.  *n_out = number of ids. */
int hge_participant_events(hge_engine* h, int32_t creator, int64_t skip, int32_t* ids_out,
                           int64_t cap, int64_t* n_out);
/* Store.ParticipantEvent(pk, index) (caches.go:78-84): id, or HGE_ERR_TOO_LATE /
 * HGE_ERR_NOT_FOUND. */
int32_t hge_participant_event(hge_engine* h, int32_t creator, int64_t index);
/* Store.LastFrom(pk) (caches.go:86-97): id of the creator's last event, -1 = "". */
int32_t hge_last_from(hge_engine* h, int32_t creator);
/* Core.Diff's selection (node/core.go:108-132): every event the caller knows and
 * `known` (n_participants counts) does not, in topological order (ByTopologicalOrder,
 * event.go:233-239). */
int hge_diff(hge_engine* h, const int32_t* known, int32_t* ids_out, int64_t cap, int64_t* n_out);
/* SetWireInfo (hashgraph.go:497-524): {selfParentIndex, otherParentCreatorID,
 * otherParentIndex, creatorID} of an event (WireBody, event.go:244-259). */
int hge_wire_info(hge_engine* h, int32_t id, int32_t* out4);
/* ReadWireInfo's parent resolution (hashgraph.go:526-571): (creator, index)
 * pairs -> engine ids (HGE_NONE for index -1). */
int hge_read_wire_parents(hge_engine* h, int32_t creator_id, int32_t self_parent_index,
                          int32_t other_parent_creator_id, int32_t other_parent_index,
                          int32_t* sp_out, int32_t* op_out);

/* ---- standalone Store (host only: no device, no Hashgraph) -------------------- */
/* The reference's InmemStore for a store used on its own -- its own tests and tools
 * call SetEvent / SetRound directly, with events that were never inserted into a
 * hashgraph and RoundInfos holding any entries (inmem_store_test.go:48-159,
 * caches_test.go:22-131).  Same containers: per-participant RollingLists and a
 * consensus RollingList of cache_size (ErrTooLate / ErrKeyNotFound as the
 * reference's, caches.go:45-115, common/rolling_list.go:25-67) and an LRU of
 * cache_size RoundInfos (Rounds() = its length, common/lru.go), and the eventCache as
 * an LRU of cache_size keys (SetEvent appends a key GetEvent does not find to its
 * creator's list, inmem_store.go:51-64).  cache_size 0 is the reference's NewLRU(0) /
 * NewRollingList(0): the LRUs keep nothing and the lists never roll; a negative size
 * is HGE_ERR_ARG.  A creator id >= n_participants gets its list on first use
 * (caches.go:99-106) and is left out of Known.  Events are the caller's int64 keys
 * (the shim's hash <-> key map); event bodies stay with the caller.  The engine-bound Store
 * (the hge_* views above) serves a Hashgraph; this one serves NewInmemStore until a
 * Hashgraph binds it (go/hashgraph/inmem_store_hge.go). */
typedef struct hge_store hge_store;
int hge_store_create(int32_t n_participants, int64_t cache_size, hge_store** out);
void hge_store_destroy(hge_store* s);
int hge_store_set_event(hge_store* s, int64_t key, int32_t creator);   /* SetEvent */
int32_t hge_store_has_event(hge_store* s, int64_t key);
int hge_store_participant_events(hge_store* s, int32_t creator, int64_t skip, int64_t* keys_out, int64_t cap,
                                 int64_t* n_out);                       /* ParticipantEvents */
int hge_store_participant_event(hge_store* s, int32_t creator, int64_t index, int64_t* key_out);
int hge_store_last_from(hge_store* s, int32_t creator, int64_t* key_out, int32_t* found);
int hge_store_known(hge_store* s, int32_t* counts_out);
int hge_store_add_consensus_event(hge_store* s, int64_t key);
int64_t hge_store_consensus_events(hge_store* s, int64_t* keys_out, int64_t cap);
int64_t hge_store_consensus_count(hge_store* s);
/* SetRound / GetRound: entries (key, witness, famous 0 undefined 1 true 2 false) */
int hge_store_set_round(hge_store* s, int32_t round, const int64_t* keys, const uint8_t* witness,
                        const uint8_t* famous, int32_t n);
int hge_store_get_round(hge_store* s, int32_t round, int64_t* keys_out, uint8_t* witness_out,
                        uint8_t* famous_out, int32_t cap, int32_t* n_out);
int32_t hge_store_rounds(hge_store* s);
int hge_store_round_witnesses(hge_store* s, int32_t round, int64_t* keys_out, int32_t cap, int32_t* n_out);
int32_t hge_store_round_events(hge_store* s, int32_t round);

/* ---- round predicates (hashgraph.go:211-326) --------------------------------- */
int32_t hge_parent_round(hge_engine* h, int32_t x);   /* ParentRound: -1 bad id, 0 no parents */
int32_t hge_round_inc(hge_engine* h, int32_t x);      /* RoundInc (over RoundWitnesses(pr))   */
int hge_round_diff(hge_engine* h, int32_t x, int32_t y, int32_t* out); /* RoundDiff */
/* Store.SetRound (inmem_store.go:115-118): record witness entries (and their
 * fame: 0 undefined, 1 true, 2 false) of round r; Rounds() >= r + 1 afterwards.
 * The engine's own DivideRounds writes the same tables for rounds the DAG
 * determines; the reference's round tests use SetRound in its place. */
int hge_set_round(hge_engine* h, int32_t round, const int32_t* ids, const uint8_t* witness,
                  const uint8_t* fame, int32_t n);

/* ---- test predicates (hashgraph.go:82-208) --------------------------------- */
int32_t hge_ancestor(hge_engine* h, int32_t x, int32_t y);
int32_t hge_self_ancestor(hge_engine* h, int32_t x, int32_t y);
int32_t hge_see(hge_engine* h, int32_t x, int32_t y);
int32_t hge_strongly_see(hge_engine* h, int32_t x, int32_t y);
int32_t hge_oldest_self_ancestor_to_see(hge_engine* h, int32_t x, int32_t y); /* id or -1 */
/* lastAncestors / firstDescendants indices of x (FD unset = INT32_MAX), N ints each. */
int hge_coordinates(hge_engine* h, int32_t id, int32_t* la_out, int32_t* fd_out);

/* ---- wire and hashing format: encoding/gob, hge_gob.cpp --------
 * Host only.  WireEvent (hashgraph/event.go:244-259) as babble puts it on the wire
 * (SyncResponse.Events, net/commands.go; framing net/net_transport.go:297-395), and
 * EventBody.Marshal (event.go:44-58), the bytes Sign/Verify hash.  Timestamps are
 * Go time.Time values: Unix seconds, nanoseconds, zone offset in minutes (-1 =
 * UTC; set = 0: the zero Time, omitted).  R, S: 32-byte big-endian magnitudes of
 * the non-negative signature halves (r_set / s_set = 0: nil).  Transactions of
 * event k are tx[tx_off[tx_first + j] .. tx_off[tx_first + j + 1]), j < tx_count.
 * Gob type ids are process-global in Go: first_type_id is the id the first type
 * defined takes (65 in a fresh process whose first gob type is this one). */
typedef struct {
  int64_t unix_sec;
  int32_t nsec;
  int16_t offset_min;
  int16_t set;
} hge_gob_time;
typedef struct {
  int64_t self_parent_index, other_parent_creator_id, other_parent_index, creator_id, index;
  hge_gob_time timestamp;
  uint8_t r[32], s[32];
  int32_t r_set, s_set;
  int64_t tx_first;
  int32_t tx_count, pad;
} hge_wire_event;
typedef struct {
  int32_t tx_count, n_parents;
  const uint8_t* creator;
  int64_t creator_len;
  hge_gob_time timestamp;
  int64_t index;
} hge_gob_body;
/* One encoder's stream: the type definitions, then one message per event (like
 * successive gob Encoder.Encode(WireEvent) calls).  *n_out = bytes; out = NULL
 * with cap = 0 asks for the size. */
int hge_gob_encode_wire_events(const hge_wire_event* ev, int64_t n, const uint8_t* tx, const int64_t* tx_off,
                               int32_t first_type_id, uint8_t* out, int64_t cap, int64_t* n_out);
/* Every WireEvent in a gob stream (top-level values or nested, e.g. a
 * SyncResponse's Events), any type ids, fields matched by name.  tx_off gets
 * n_tx + 1 offsets.  HGE_ERR_NOT_FOUND: a capacity was too small (the counts say
 * what is needed); HGE_ERR_ARG: not a well-formed stream of these types. */
int hge_gob_decode_wire_events(const uint8_t* buf, int64_t len, hge_wire_event* ev, int64_t cap_ev, uint8_t* tx,
                               int64_t cap_bytes, int64_t* tx_off, int64_t cap_tx, int64_t* n_ev, int64_t* n_tx,
                               int64_t* n_bytes);
/* EventBody.Marshal: a fresh encoder's stream of one EventBody (Parents: hex
 * strings parents[parent_off[k] .. parent_off[k + 1])). */
int hge_gob_encode_event_body(const hge_gob_body* body, const uint8_t* tx, const int64_t* tx_off,
                              const uint8_t* parents, const int64_t* parent_off, int32_t first_type_id,
                              uint8_t* out, int64_t cap, int64_t* n_out);

/* ---- profiling ------------------------------------------------------------- */
/* Device milliseconds of the last replay/batch by stage (HIP events on the
 * engine's stream): 0 coords, 1 rounds, 2 witness bits, 3 fame, 4 received,
 * 5 order, 6 total.  Returns the number of stages written. */
int hge_stage_times(hge_engine* h, float* ms_out, int cap);
/* lastAncestors passes the last coordinate step needed: window passes for
 * 32 < N <= 256 (hge_coords_win.hip), Jacobi sweeps otherwise (hge_coords.hip);
 * the last one confirms the fixed point (a single window needs one pass). */
int32_t hge_coordinate_sweeps(hge_engine* h);
/* Host round trips so far: the number of times the host has waited on the
 * engine's stream (each readback of a control value or result is one). */
int64_t hge_host_syncs(hge_engine* h);
/* Times the wide rounds walk (N > 32) found its frontier hand-off timed out (its
 * workgroups were not all resident, e.g. several engines sharing one GPU) and
 * walked again with the launch-per-round kernel, which the engine then keeps;
 * results are unchanged.  Replaces returning HGE_ERR_DEVICE from the replay. */
int64_t hge_frontier_fallbacks(hge_engine* h);
/* Per-kernel timing: HIP events around every launch on the engine stream. */
int hge_set_profiling(hge_engine* h, int on);
int hge_reset_kernel_stats(hge_engine* h);
/* Kernel k's name, accumulated device ms and launch count; returns the number
 * of distinct kernels recorded. */
int hge_kernel_stats(hge_engine* h, int k, char* name, int namecap, double* total_ms,
                     int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* HGE_H */
