/*
 * rbe.h — C ABI of the MI355X batched Raft step engine (libdragonboat_amd.so).
 *
 * Drop-in boundary for dragonboat's step path.  Today the node layer drives
 * one *raft.Peer per group under raftMu (node.go:79-80, 290) and
 * execEngine.execNodes calls node.stepNode() for every ready cluster
 * (execengine.go:494-503).  The engine replaces that per-group loop with one
 * batched device step over every group a GPU owns.  Each entry point below
 * names the reference interface it replaces.  The binding a Go maintainer
 * would add (cgo) is in INTEGRATION.md.
 *
 * Conventions (mirroring binding/include/dragonboat/binding.h:107-113):
 *   - every function returns int: 0 = ok, < 0 = RBE_E_* error;
 *   - plain pointers and sizes only; host buffers are caller-owned;
 *   - one handle per GPU, single-threaded per handle (Peer is not
 *     thread-safe either, node.go:1017-1018);
 *   - protocol invariant violations (plog.Panicf in the reference) do not
 *     abort the process: they set a sticky per-replica fault word
 *     (RBE_FAULT_*) that rbe_get_updates/rbe_get_views report.
 *
 * A group has n_replicas slots; slot s is node id s + 1 unless the host gives
 * the group's node ids (rbe_set_node_ids: any non-zero uint64, ascending with
 * the slots).  Every node id the ABI takes or returns is such an id; masks
 * (removed, votes) and per-slot arrays (match, next) are indexed by slot.  The
 * group of cluster id c is the engine-local index g with c = cid_base + g *
 * cid_stride, which is dragonboat's FixedPartitioner rule
 * (internal/server/partition.go:38-40) when cid_stride = number of GPUs and
 * cid_base = 1 + rank.
 */
#ifndef DRAGONBOAT_AMD_RBE_H_
#define DRAGONBOAT_AMD_RBE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RBE_ABI_VERSION 9

/* error codes */
#define RBE_OK 0
#define RBE_E_INVALID (-1)   /* bad argument / configuration */
#define RBE_E_HIP (-2)       /* a HIP runtime call failed */
#define RBE_E_NOMEM (-3)     /* device allocation failed */
#define RBE_E_NODEV (-4)     /* no usable gfx950 device */
#define RBE_E_STATE (-5)     /* call not valid in the current state */
#define RBE_E_CORRUPT (-6)   /* rbe_wire_decode: a frame failed its crc32 or does not parse */

/* sticky per-replica fault bits (see dragonboat_amd/csrc/rbe_types.h) */
#define RBE_FAULT_WINDOW 0x01u
#define RBE_FAULT_OUTBOX 0x02u
#define RBE_FAULT_ARENA 0x04u
#define RBE_FAULT_READQ 0x08u
#define RBE_FAULT_RTR 0x10u
#define RBE_FAULT_PANIC 0x20u
#define RBE_FAULT_UNSUPPORTED 0x40u
#define RBE_FAULT_DROPLIST 0x80u
/* Since ABI 9 no per-replica capacity of the planes faults a replica: a full
 * message list, entry arena, readIndex queue, ReadyToRead or dropped list and
 * the log below the in-memory ring spill into the engine's spill tiers (a page
 * pool and a round spill heap, cfg.pool_bytes / spill_bytes).  OUTBOX, ARENA,
 * READQ, RTR and DROPLIST are no longer raised; WINDOW means a log entry the
 * replica holds is missing (a launch that handed over only the LogDB's tail);
 * NOMEM that a spill tier itself is exhausted (rbe_spill_stats). */
#define RBE_FAULT_NOMEM 0x100u

/* counter slots (rbe_get_counters) */
enum rbe_counter {
  RBE_CTR_STEPS = 0,           /* replica-steps (group-steps metric) */
  RBE_CTR_COMMITTED = 1,       /* entries committed, counted once per group at its leader */
  RBE_CTR_MSG_IN = 2,
  RBE_CTR_MSG_OUT = 3,
  RBE_CTR_ENT_IN = 4,
  RBE_CTR_ENT_OUT = 5,
  RBE_CTR_READS_CONFIRMED = 6, /* ReadyToRead records (ReadIndex confirmations) */
  RBE_CTR_PROPOSALS = 7,
  RBE_CTR_READS = 8,
  RBE_CTR_QUIESCED_TICKS = 9,
  RBE_CTR_ACTIVE_TICKS = 10,
  RBE_CTR_CAMPAIGNS = 11,
  RBE_CTR_ENT_SAVED = 12,
  RBE_CTR_ENT_APPLIED = 13,
  RBE_CTR_MSG_DROPPED = 14,
  RBE_CTR_DROPPED_PROPOSALS = 15,
  RBE_CTR_DROPPED_READS = 16,
  RBE_CTR_LEADER_STEPS = 17,
  RBE_CTR_REMOTE_TOUCH = 18,
  RBE_CTR_RING_ACCESS = 19,
  RBE_CTR_FAULTS = 20,
  RBE_CTR_RQ_TOUCH = 21,
  RBE_CTR_NUM = 24
};

/*
 * Engine configuration.  Protocol fields mirror config.Config
 * (config/config.go:60-171): ElectionRTT, HeartbeatRTT, CheckQuorum, Quiesce;
 * MaxInMemLogSize is max_inmem_log_size (0 = rate limiter off).  max_entry_size mirrors
 * settings.Soft.MaxEntrySize (soft.go:226).
 */
typedef struct rbe_config {
  uint32_t abi_version;      /* RBE_ABI_VERSION */
  int32_t device;            /* HIP device ordinal */
  uint64_t n_groups;         /* groups owned by this engine */
  uint32_t n_replicas;       /* replica slots per group, 1..7 (the group's largest size) */
  uint32_t election_rtt;     /* ticks, config.ElectionRTT */
  uint32_t heartbeat_rtt;    /* ticks, config.HeartbeatRTT */
  uint32_t check_quorum;     /* config.CheckQuorum */
  uint32_t quiesce;          /* config.Quiesce */
  uint32_t ring;             /* in-memory entry window per replica (power of 2), 0 = 64 */
  uint32_t rq_cap;           /* pending ReadIndex requests per leader, 0 = 8 */
  uint32_t maxm;             /* message slots per (sender, destination) per round, 0 = 12 */
  uint32_t ecap;             /* entry slots per sender per round, 0 = 32 */
  uint32_t rtr_cap;          /* ReadyToRead slots per replica per round, 0 = 8 */
  uint32_t dri_cap;          /* dropped ReadIndex slots per replica per round, 0 = 8 */
  uint32_t trace;            /* maintain per-replica trace digests */
  uint64_t cid_base;         /* cluster id of group g = cid_base + g * cid_stride */
  uint64_t cid_stride;       /* 0 = 1 */
  uint64_t seed;             /* injected PRNG seed (election timeouts, workload) */
  uint64_t max_entry_size;   /* bytes, 0 = 64 MiB */
  /* synthetic client workload; wl_enabled = 0 disables */
  uint32_t wl_enabled;
  uint32_t wl_start_round;
  uint32_t wl_stop_round;    /* 0 = never stop */
  uint32_t wl_active_mod;    /* group active iff mix(seed, cid) % mod == 0 (1 = all) */
  uint32_t wl_read_permille; /* read with probability p/1000, else propose */
  uint32_t ext_inputs;       /* accept rbe_push_proposals / rbe_push_read_index */
  /* fault schedule (network.isolate of the current leader), 0 = off */
  uint32_t iso_period;
  uint32_t iso_len;
  uint32_t iso_mod;
  /* replica-per-GPU mode: rep_world > 1 engines each step the
   * replicas k of groups g with (g + k) % rep_world == rep_rank and exchange
   * cross-GPU messages between rounds (rbe_xchg_*); 0/1 = off */
  uint32_t rep_world;
  uint32_t rep_rank;
  /* host-driven node layer */
  uint32_t ext_apply;        /* raft.applied comes from rbe_notify_applied (peer.go:312);
                                0 = the step's committed entries count as applied */
  uint32_t in_cap;           /* proposal entries rbe_push_proposals may stage per step,
                                0 = max(1024, n_groups) */
  /* leader-transfer schedule (RequestLeaderTransfer on a seeded replica every
   * xfer_period rounds in groups selected 1 in xfer_mod), 0 = off */
  uint32_t xfer_period;
  uint32_t xfer_mod;
  uint32_t snapshot_entries;     /* config.SnapshotEntries: a node snapshot at the applied
                                    index every that many applied entries, 0 = never.
                                    With ext_apply the host's snapshot worker decides
                                    (rbe_snapshot_saved / rbe_compact) and any non-zero
                                    value only turns snapshots on.  Not with ext_commit. */
  uint32_t compaction_overhead;  /* config.CompactionOverhead: the LogDB keeps that many
                                    entries below a snapshot (compacted at the next step);
                                    a remote that needs older entries gets InstallSnapshot */
  uint64_t heap_bytes;           /* payload heap for entries with Cmd > 16 B or session
                                    fields (needs ext_inputs), 0 = none: Cmd is then at
                                    most 16 bytes and Key/ClientID/SeriesID/RespondedTo 0 */
  uint32_t ext_commit;           /* the log part of Peer.Commit (savedTo, processed, the
                                    in-memory log's applied marker) comes from rbe_commit,
                                    as the node sends it after SaveRaftState (needs
                                    ext_apply); 0 = every step commits its own Update */
  /* membership change on the device (raft.go:1135-1237): ConfigChange entries
   * (rbe_propose_config_change) add or remove voting members among the group's
   * slots; the engine's own state machine applies committed ones (their Cmd in
   * the engine's 8-byte form, cc_word in rbe_step.h) unless ext_apply, where
   * the host does (rbe_apply_config_change); 0 = ConfigChange entries fault
   * (RBE_FAULT_UNSUPPORTED) */
  uint32_t membership;
  uint32_t cc_period;        /* config-change schedule (remove / re-add a seeded voter at the
                                leader every cc_period rounds in groups selected 1 in
                                cc_mod; needs membership), 0 = off */
  uint32_t cc_mod;
  /* replica mode (rep_world > 1, n_replicas < rep_world): allocate the planes
   * of only the groups this rank steps a replica of (n_replicas of every
   * rep_world groups: 3/8 at N = 3, W = 8).  Replica and group indexes of
   * every call are then the engine's local ones; rbe_local_groups maps them
   * to the global group (n_groups stays the global count). */
  uint32_t rep_compact;
  /* voting members a group starts with (0 = n_replicas): slots (node ids)
   * 1..n_voters bootstrap the group (peer.go:378-408); the other slots are
   * nodes that join later — started with no peers and an empty log
   * (node.go:280-292 with join), taking part once an AddNode for them is
   * applied.  Fewer than n_replicas needs cfg.membership. */
  uint32_t n_voters;
  /* config.MaxInMemLogSize (config.go:118-131): the rate limiter
   * (internal/server/rate.go, raft.go:660-683, 1779-1785) over each replica's
   * in-memory log bytes; 0 (or UINT64_MAX) = off.  Rate-limited engines step
   * every ticking replica on the full handler table. */
  uint64_t max_inmem_log_size;
  /* the slots beyond n_voters whose nodes start as observers (config.IsObserver)
   * or witnesses (config.IsWitness), bit s = slot s; they take part once an
   * AddObserver / AddWitness for them is applied (raft.go:1159-1180).  Needs
   * cfg.membership. */
  uint32_t observer_slots;
  uint32_t witness_slots;
  /* Spill tiers (dragonboat_amd/csrc/rbe_spill.h): everything a replica holds
   * beyond the planes' fixed capacities.  pool_bytes: the page pool holding
   * each replica's cold log (its entries below the in-memory ring: the ILogDB
   * read path, logentry.go:144-161, 186-246; every entry above the LogDB
   * marker is kept, as dragonboat's LogDB does) and readIndex queues longer
   * than rq_cap; 0 = the larger of 8 KiB per replica (at least 64 MiB) and an
   * eighth of the device's free HBM at rbe_create, at most 32 GiB (rbe_footprint
   * counts the per-replica part).  spill_bytes: the round spill heap per round
   * parity (message lists past maxm, a message's entries past ecap — a catch-up
   * Replicate sized by MaxEntrySize, raft.go:709-740 — ReadyToReads past
   * rtr_cap, dropped ReadIndexes past dri_cap); 0 = 128 B per replica, at least
   * 16 MiB, at most 4 GiB (times rep_world: each rank allocates in its own share). */
  uint64_t pool_bytes;
  uint64_t spill_bytes;
} rbe_config;

/* Snapshot of one replica (tests, debugging, rbe_get_views). */
typedef struct rbe_replica_view {
  uint64_t term, vote, leader_id, committed, last_index, processed, saved_to, digest;
  uint32_t role, election_tick, heartbeat_tick, rand_election_timeout;
  uint32_t q_tick, q_quiesced_since, q_no_activity_since, q_exit_quiesce_tick;
  uint32_t raft_quiesce, rq_count, votes_resp, votes_granted;
  uint64_t match[8], next[8];
  uint32_t rstate[8], ractive[8];
  uint32_t events;  /* RBE_EV_* of the last round's step (0 when it made no step) */
  /* slot masks, bit s = slot s (the group's s-th node: node id s + 1, or the
   * s-th id given to rbe_set_node_ids): not in this replica's raft.remotes
   * (cfg.membership), and raft.observers / raft.witnesses */
  uint32_t removed;
  uint32_t observers, witnesses;
} rbe_replica_view;

/* Per-replica step result: the Update of peer.go:201-207 / raftpb Update
 * (raftpb/raft.go:74-110) in range form.  Entries stay in the engine's ring
 * and are fetched with rbe_get_entries. */
typedef struct rbe_update {
  uint64_t term, vote, commit;  /* pb.State (valid when flags & RBE_UF_STATE_CHANGED) */
  uint64_t save_lo, save_hi;    /* EntriesToSave = [save_lo, save_hi] */
  uint64_t apply_lo, apply_hi;  /* CommittedEntries = [apply_lo, apply_hi] */
  uint64_t digest;              /* trace digest */
  uint32_t n_messages, n_ready_to_read, n_dropped_entries, n_dropped_read_indexes;
  uint32_t fault, flags;
  uint32_t role, events;     /* events: RBE_EV_* of the step */
  uint64_t leader_id;
} rbe_update;
#define RBE_UF_STATE_CHANGED 1u
#define RBE_UF_SENT_QUIESCE 2u
#define RBE_UF_FAST_APPLY 8u      /* Update.FastApply (peer.go:209-226 setFastApply) */
#define RBE_UF_HAS_UPDATE 16u     /* the step produced an Update (Peer.HasUpdate, peer.go:253-280) */
#define RBE_UF_SNAPSHOT 32u       /* Update.Snapshot: the replica restored the snapshot an
                                     InstallSnapshot carried (rbe_get_snapshot_state) */
#define RBE_UF_APPLIED 64u        /* the applied index rbe_notify_applied reported changed for
                                     this step: the node takes an Update (with only
                                     LastApplied, if nothing else) to confirm it
                                     (node.go:907-923) */

/* server.IRaftEventListener calls of a step (internal/server/event.go;
 * raft.go:354, 1090, 1333, 1368, 1503, 1995, 2010), one bit per kind.
 * RBE_EV_LEADER_UPDATED marks a step whose leader value changed. */
#define RBE_EV_LEADER_UPDATED 1u
#define RBE_EV_CAMPAIGN_LAUNCHED 2u
#define RBE_EV_CAMPAIGN_SKIPPED 4u
#define RBE_EV_SNAPSHOT_REJECTED 8u
#define RBE_EV_REPLICATION_REJECTED 16u
#define RBE_EV_PROPOSAL_DROPPED 32u
#define RBE_EV_READ_INDEX_DROPPED 64u

/* raftpb Message (raft.pb.go:1019-1033) as emitted by the engine. */
typedef struct rbe_message {
  uint32_t type, reject;
  uint64_t to, from, cluster_id, term, log_term, log_index, commit, hint, hint_high;
  uint32_t n_entries;
  /* InstallSnapshot: the snapshot's membership (Snapshot.Membership, raft.pb.go:
   * 733-739) in the packed slot-mask form of rbe_launch_state::removed: bits
   * 0-7 the slots it does not list as voters (Addresses), 8-15 its Observers,
   * 16-23 its Witnesses, bit s = slot s of the group (its index and term are
   * log_index / log_term); 0 for every other type */
  uint32_t reserved;
} rbe_message;

/* raftpb Entry (raft.pb.go:589-598), every field: Index, Term, Type, the
 * session fields Key / ClientID / SeriesID / RespondedTo that the client
 * layer stamps on each proposal (requests.go:994-997) and Cmd.  `cmd` holds
 * the first min(cmd_len, 16) bytes; the calls that move whole Cmds take or
 * return them concatenated in a separate byte buffer.  Inside the engine an
 * entry with a Cmd longer than 16 bytes or any non-zero session field lives
 * in the payload heap (cfg.heap_bytes), which such entries require. */
typedef struct rbe_entry {
  uint64_t index, term;
  uint32_t type, cmd_len;
  uint8_t cmd[16];
  uint64_t key, client_id, series_id, responded_to;
} rbe_entry;

typedef struct rbe_ready_to_read {  /* raftpb ReadyToRead, raftpb/raft.go:52-56 */
  uint64_t index, ctx_low, ctx_high;
} rbe_ready_to_read;

typedef struct rbe_engine rbe_engine;

/* Persisted state of one replica for rbe_launch: pb.State (term, vote, commit)
 * and the tail of its LogDB, entries [last_index - n_entries + 1, last_index]
 * (the engine's in-memory window).  With cfg.snapshot_entries the LogDB may be
 * compacted: `marker` is its compaction marker (entries at or below it are
 * gone, Term(marker) = marker_term; logdb GetRange first = marker + 1) and
 * snapshot_index / snapshot_term its latest snapshot, which the state machine
 * recovers from; all four are 0 without snapshots. */
typedef struct rbe_launch_state {
  uint64_t term, vote, commit, last_index;
  uint32_t n_entries;
  /* the membership the restarted raft reads from the LogDB (logdb NodeState =
   * its latest snapshot's, raft.go:260-270): bits 0-7 the slots not in
   * Membership.Addresses, 8-15 its Observers, 16-23 its Witnesses, bit s =
   * slot s; needs cfg.membership when non-zero.  With snapshots it is also the
   * snapshot's and the state machine's membership. */
  uint32_t removed;
  uint64_t marker, marker_term, snapshot_index, snapshot_term;
} rbe_launch_state;

/* Lifecycle.  Replaces the per-group raft.Launch / newRaft (peer.go:64-86,
 * raft.go:234-289): creates every group's replicas and bootstraps them with
 * peer.go:378-408 semantics (initial = true, newNode = true). */
int rbe_create(const rbe_config* cfg, rbe_engine** out);
/* Restart replicas from persisted state between two rounds: Peer.Launch with
 * initial = false, newNode = false (peer.go:64-86) over an existing LogDB, i.e.
 * newRaft + loadState + becomeFollower(term, NoLeader) (raft.go:234-289,
 * 429-437): follower without a leader, the persisted term/vote/commit, the log
 * up to last_index, nothing applied above the LogDB's first index yet
 * (processed = firstIndex - 1 = marker, logentry.go:86-96; the state machine
 * recovers from the latest snapshot), remotes next = last + 1.  Over a
 * compacted LogDB (snapshot_entries) st[i].commit must be >= the marker
 * (loadState panics below it, raft.go:429-437) and the entries lie above it.  The node around it restarts
 * too (fresh quiesce state and tick count), and the messages in flight to and
 * from a relaunched replica are lost.  replica[i] takes st[i] and the next
 * st[i].n_entries entries of `ents`: the LogDB's entries above its marker,
 * up to last_index (the ring takes the newest cfg.ring of them, the cold log
 * the rest; a LogDB handed over only in part faults with RBE_FAULT_WINDOW when
 * the replica later needs an entry below what it was given).  The
 * entries' Cmds are concatenated in `cmd` (null: each is its rbe_entry.cmd,
 * at most 16 bytes); entries with longer Cmds or session fields go to the
 * payload heap.  Checked whole before anything changes (RBE_E_INVALID;
 * RBE_E_NOMEM when the heap has no room for them). */
int rbe_launch(rbe_engine* e, uint64_t n, const uint64_t* replica, const rbe_launch_state* st,
               const rbe_entry* ents, const uint8_t* cmd);
/* The node ids of groups [first_group, first_group + count): n_replicas per
 * group in slot order, non-zero and distinct within a group.  The engine's
 * canonical order of a group's nodes (raft.go's map iterations, SURVEY.md
 * §8c) is the slot order: Go visits the maps in random order, so every fixed
 * order is one of the reference's executions, and the per-(sender, receiver)
 * message streams do not depend on it.  The node ids of raft.Config.NodeID
 * and pb.Message From/To (config.go, raft.pb.go) that a dragonboat deployment
 * assigns; a slot beyond the initial voters (cfg.n_voters) is the id a joining
 * node will have.  Only before the first step (RBE_E_STATE after; later
 * changes go through rbe_replace_node).  Without it slot s is node s + 1. */
int rbe_set_node_ids(rbe_engine* e, uint64_t first_group, uint64_t count, const uint64_t* ids);
/* A new node in a removed node's slot, between two rounds: replica[i]'s slot
 * gets node id node_id[i] and its replica becomes that node, started as
 * dragonboat starts a node that joins a running cluster (node.go:280-292: no
 * peers, an empty LogDB, Launch with newNode; peer.go:64-86) in the slot's
 * configured kind (voter, or cfg.observer_slots / witness_slots).  The host
 * then adds it with a ConfigChange (AddNode / AddObserver / AddWitness of
 * node_id[i], raft.go:1135-1180), which any replica of the group can take: a
 * removed slot can host any number of new nodes over its life, as dragonboat
 * gives every replacement a new node id (rsm membership refuses a removed id,
 * membership.go:299-321).  Preconditions, checked whole before anything
 * changes: cfg.membership, group-per-GPU (rep_world <= 1) and no seeded
 * config-change / leader-transfer schedule (RBE_E_STATE); every replica[i]
 * in range, at most one per group (RBE_E_STATE for two), node_id[i] non-zero
 * and not the id of another slot of its group (RBE_E_INVALID); no input staged
 * for any replica of the group; and nothing in the group still refers to the
 * old node (RBE_E_STATE): every other replica has applied its RemoveNode (it
 * is in none of raft.remotes / observers / witnesses), none has it as vote,
 * leader or leader-transfer target, in a vote tally, as the sender or a
 * confirmer of a queued ReadIndex or in the rate limiter's reports, and it sent no message
 * in the last round.  Messages still addressed to the slot are dropped. */
int rbe_replace_node(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* node_id);
int rbe_destroy(rbe_engine* e);
int rbe_abi_version(void);
/* sizeof the ABI structs, in this order: rbe_config, rbe_replica_view,
 * rbe_update, rbe_message, rbe_entry, rbe_ready_to_read (a binding checks its
 * mirrors of them against these); returns how many were written */
int rbe_abi_sizes(uint64_t* out, uint32_t cap);

/* One lockstep round for every replica: the stepNode/handleEvents/getUpdate/
 * Commit sequence of node.go:1016-1067, 907-994 driven by execEngine.execNodes
 * (execengine.go:474-560), with messages of round r delivered in round r+1
 * (DESIGN.md §Round semantics).  rbe_run runs `rounds` rounds back to back
 * (HIP-graph replay when the configuration allows). */
int rbe_step(rbe_engine* e);
/* rbe_step with options: RBE_STEP_NO_TICK steps without the round's tick
 * (the host steps faster than its RTT tick, nodehost.go:1668-1684); a replica
 * with no message, client input or entry to apply then makes no step at all,
 * as handleEvents finds no event (node.go:1030-1067). */
#define RBE_STEP_NO_TICK 1u
int rbe_step_ex(rbe_engine* e, uint32_t flags);
int rbe_run(rbe_engine* e, uint32_t rounds);
int rbe_sync(rbe_engine* e);
int rbe_round(const rbe_engine* e, uint32_t* round);

/* Time `rounds` rounds with HIP events on the engine stream; *ms = elapsed.
 * A graph for that round count is captured before the first event. */
int rbe_run_timed(rbe_engine* e, uint32_t rounds, float* ms);
/* Capture (and upload) the replay graph of `rounds` rounds now, so a later
 * rbe_run / rbe_run_timed of that many rounds only launches it; a no-op when
 * the configuration steps round by round.  Synchronizes the engine stream. */
int rbe_prepare_run(rbe_engine* e, uint32_t rounds);

/* Round-pipeline kernel slots (rbe_profile_rounds, rbe_get_kernel_counters,
 * rbe_kernel_name).  The default pipeline runs k_triage /
 * k_fast_list<LEAD> / k_fast_list<FOLL> / k_full_list in slots 0-3;
 * RBE_MODE=fused runs k_round (triage + steady-state steps in one kernel) in
 * slot 0 and k_full_list in slot 3; RBE_MODE=full runs k_step in slot 3.
 * Unused slots have an empty name and zero time. */
#define RBE_KERNEL_NUM 4

/* Name of the kernel in `slot` for this engine's pipeline ("" if unused). */
int rbe_kernel_name(const rbe_engine* e, int32_t slot, char* buf, uint32_t cap);

/* Run `rounds` rounds one at a time, each pipeline kernel launched with
 * hipExtLaunchKernel and a start / stop event pair that its own dispatch
 * stamps (the kernel's execution, not the launch gaps around it);
 * ms_per_kernel[RBE_KERNEL_NUM] receives each kernel's total time. */
int rbe_profile_rounds(rbe_engine* e, uint32_t rounds, float* ms_per_kernel);

/* Host input for the next step (requires cfg.ext_inputs), the node-side events
 * of handleEvents (node.go:1030-1067).  replica = g * n_replicas + (node_id - 1).
 * Each call checks its whole batch before staging any of it (RBE_E_INVALID on a
 * bad replica/argument, nothing staged); staged input is uploaded by the next
 * rbe_step in one copy.  A replica takes one proposal batch, one ReadIndex and
 * one leader transfer per step, as the node batches them; a second one for the
 * same replica, within a batch or across calls, is RBE_E_STATE (nothing staged).
 *   rbe_propose_entries: Peer.ProposeEntries (peer.go:117-123); batch i holds
 *     n_ents[i] entries for replica[i], whole raftpb.Entry values in `ents`
 *     (Type, Key, ClientID, SeriesID, RespondedTo, cmd_len; Index and Term are
 *     the leader's to stamp, raft.go:909-920) with their Cmd bytes concatenated
 *     in `cmd`.  Without a payload heap every Cmd is at most 16 bytes and the
 *     session fields are 0; with cfg.heap_bytes an entry with a longer Cmd (at
 *     most heap_bytes / 4, the ErrPayloadTooBig analog, requests.go:989-991)
 *     or session fields is written to the heap once as a record and every
 *     replica's entry refers to it.  RBE_E_NOMEM when the step's cfg.in_cap
 *     entries are used up, or the heap has no room without overwriting a
 *     record some replica has not yet saved and applied (never lapped: the
 *     reference keeps an entry until then, inmemory.go:116-166).
 *   rbe_push_proposals: rbe_propose_entries without session fields; the
 *     entries' types and Cmd lengths in type[], cmd_len[].
 *   rbe_push_read_index: Peer.ReadIndex (peer.go:297-303), ctx_low != 0
 *     (requests.go:726).
 *   rbe_request_leader_transfer: Peer.RequestLeaderTransfer (peer.go:106-113),
 *     target in 1..n_replicas.
 *   rbe_report_unreachable: Peer.ReportUnreachableNode (peer.go:168-174).
 *   rbe_report_snapshot_status: Peer.ReportSnapshotStatus (peer.go:177-184).
 *     Unreachable / SnapshotStatus reports are delivered before the step's
 *     network messages (node.go:1207-1220 handles them in the inbox).
 *   rbe_notify_applied: Peer.NotifyRaftLastApplied (peer.go:312-315): the
 *     applied index the state machine confirmed, raft.applied, which gates
 *     campaigns (hasConfigChangeToApply, raft.go:1460-1472); needs cfg.ext_apply.
 *   rbe_set_apply_ready: whether the node can take more entries to apply
 *     (node.canHaveMoreEntriesToApply, node.go:1002-1004, the moreEntriesToApply
 *     argument of Peer.HasUpdate / GetUpdate, peer.go:201, 253, 329-331); sticky
 *     per replica, ready by default.  While not ready a step returns no
 *     CommittedEntries. */
int rbe_propose_entries(rbe_engine* e, uint64_t n, const uint64_t* replica,
                        const uint32_t* n_ents, const rbe_entry* ents, const uint8_t* cmd);
int rbe_push_proposals(rbe_engine* e, uint64_t n, const uint64_t* replica,
                       const uint32_t* n_ents, const uint32_t* type, const uint32_t* cmd_len,
                       const uint8_t* cmd);
int rbe_push_read_index(rbe_engine* e, uint64_t n, const uint64_t* replica,
                        const uint64_t* ctx_low, const uint64_t* ctx_high);
int rbe_request_leader_transfer(rbe_engine* e, uint64_t n, const uint64_t* replica,
                                const uint64_t* target);
int rbe_report_unreachable(rbe_engine* e, uint64_t n, const uint64_t* replica,
                           const uint64_t* node_id);
int rbe_report_snapshot_status(rbe_engine* e, uint64_t n, const uint64_t* replica,
                               const uint64_t* node_id, const uint8_t* reject);
int rbe_notify_applied(rbe_engine* e, uint64_t n, const uint64_t* replica,
                       const uint64_t* applied);
int rbe_set_apply_ready(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint8_t* ready);
/* Membership change (cfg.membership; RBE_E_STATE otherwise), staged like every
 * input above (one of each per replica per step):
 *   rbe_propose_config_change: Peer.ProposeConfigChange (peer.go:126-135) at
 *     replica[i]: a ConfigChange entry of type[i] (pb.ConfigChangeType:
 *     0 AddNode, 1 RemoveNode, 2 AddObserver, 3 AddWitness) for node_id[i]
 *     (1..n_replicas), proposed after the step's messages and tick, before its
 *     proposals (node.go:1030-1067 handleConfigChangeMessage); a leader with a
 *     config change pending drops it (DroppedEntries) for an empty entry.
 *   rbe_apply_config_change: Peer.ApplyConfigChange (peer.go:138-149), what the
 *     node calls once its state machine applied a committed ConfigChange
 *     (node_id 0 = NoNode: clearPendingConfigChange only); applied before the
 *     replica's next step.  Needs cfg.ext_apply (else the engine applies them).
 *   rbe_reject_config_change: Peer.RejectConfigChange (peer.go:152-157). */
int rbe_propose_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica,
                              const uint32_t* type, const uint64_t* node_id);
int rbe_apply_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica,
                            const uint64_t* node_id, const uint32_t* type);
int rbe_reject_config_change(rbe_engine* e, uint64_t n, const uint64_t* replica);
/* Host-driven snapshots (cfg.snapshot_entries with cfg.ext_apply; RBE_E_STATE
 * otherwise): the node's snapshot worker around a state machine the host
 * applies (node.go:585-692 saveSnapshotRequired / doSaveSnapshot /
 * compactSnapshot, 849-866 compactLog).  One of each per replica between two
 * steps, checked whole (RBE_E_INVALID / RBE_E_STATE, nothing staged).
 *   rbe_snapshot_saved: the state machine's snapshot of replica[i] at index[i]
 *     (at most the applied index last reported with rbe_notify_applied) of
 *     term[i], with the membership removed[i] (the packed form of
 *     rbe_launch_state::removed; null = every slot a voter; non-zero needs
 *     cfg.membership), was saved and the LogDB took it
 *     (LogReader.CreateSnapshot; one at or below the LogDB's latest is out of
 *     date and ignored).  A remote that needs entries the LogDB compacted away
 *     gets this snapshot by InstallSnapshot (raft.go:684-697).
 *   rbe_compact: compactLogTo = to[i]: the replica's next step compacts the
 *     LogDB after its Update (LogReader.Compact: only inside (marker,
 *     lastIndex] and never past the latest snapshot).
 * A replica that restores a received snapshot reports RBE_UF_SNAPSHOT; the host
 * recovers its state machine from it, reports the applied index
 * (rbe_notify_applied) and calls rbe_restore_remotes. */
int rbe_snapshot_saved(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* index,
                       const uint64_t* term, const uint32_t* removed);
int rbe_compact(rbe_engine* e, uint64_t n, const uint64_t* replica, const uint64_t* to);
/* Peer.RestoreRemotes (peer.go:159-165 → raft.go:1566 handleRestoreRemote →
 * restoreRemotes, 472-517), what the node calls once its state machine has
 * recovered from a snapshot (rsm/statemachine.go:236 via node.go:241-264):
 * replica[i]'s snapshot membership lists counts[3i] voters (Addresses),
 * counts[3i + 1] observers and counts[3i + 2] witnesses, their node ids next in
 * `ids` in that order (each a node of the group, none twice).  Before the
 * replica's next step raft's remotes / observers / witnesses become exactly
 * those, every remote restarts (match 0, next lastIndex + 1; its own match
 * lastIndex), an observer listed as a voter becomes a follower and a leader
 * the snapshot does not list steps down.  Staged like the inputs above (one per
 * replica per step; the engine's own RestoreRemotes after an InstallSnapshot
 * it restored runs first and is replaced by this one).  Needs cfg.membership
 * and cfg.ext_inputs (RBE_E_STATE). */
int rbe_restore_remotes(rbe_engine* e, uint64_t n, const uint64_t* replica,
                        const uint32_t* counts, const uint64_t* ids);

/* Results of the last round.  Replaces Peer.GetUpdate (peer.go:201-207).
 * Peer.Commit (peer.go:282-293) consumes a step's outputs at the step; its log
 * part is implicit (the step's entries count as saved and its committed
 * entries as processed) unless cfg.ext_commit, where the host sends it with
 * rbe_commit. */
int rbe_get_updates(rbe_engine* e, uint64_t first, uint64_t count, rbe_update* out);
int rbe_get_messages(rbe_engine* e, uint64_t replica, rbe_message* out, uint32_t cap,
                     uint32_t* n_out);
int rbe_get_ready_to_reads(rbe_engine* e, uint64_t replica, rbe_ready_to_read* out,
                           uint32_t cap, uint32_t* n_out);
int rbe_get_entries(rbe_engine* e, uint64_t replica, uint64_t lo, uint64_t hi,
                    rbe_entry* out);
/* Node snapshot state of replicas [first, first + count) (snapshot_entries > 0,
 * else RBE_E_STATE): eight words each — the LogDB's compaction marker and its
 * term (entries at or below it are gone: logdb.go Compact / RemoveEntriesTo),
 * the latest snapshot's index and term (CreateSnapshot, or ApplySnapshot of one
 * received), the node's reqSnapshotIndex and pending compactLogTo (node.go
 * ss, 585-605 / 849-866), the latest snapshot's membership and the state
 * machine's current one, each in the packed slot-mask form of
 * rbe_launch_state::removed (bits 0-7 the slots that are not voters, 8-15
 * observers, 16-23 witnesses, bit s = slot s; pb.Snapshot.Membership,
 * raft.pb.go:733-739; a snapshot records
 * the state machine's membership at its index, and a node that restores one
 * sends it to raft with RestoreRemotes at its next step). */
int rbe_get_snapshot_state(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* out8);

/* raftpb UpdateCommit (raftpb/raft.go:60-70). */
typedef struct rbe_update_commit {
  uint64_t processed, last_applied, stable_log_to, stable_log_term, stable_snapshot_to,
      ready_to_read;
} rbe_update_commit;
/* getUpdateCommit (peer.go:410-427) of the last round's Update of replicas
 * [first, first + count): processed = last CommittedEntries index,
 * last_applied = the applied index the step ran with (rbe_notify_applied),
 * stable_log_to / stable_log_term = the last EntriesToSave entry,
 * ready_to_read = number of ReadyToReads; all zero for a replica whose step
 * made no Update (RBE_UF_HAS_UPDATE clear); an Update carrying a Snapshot
 * (RBE_UF_SNAPSHOT) gives stable_snapshot_to = its index and processed at
 * least that index.  Needs cfg.ext_commit. */
int rbe_get_update_commits(rbe_engine* e, uint64_t first, uint64_t count, rbe_update_commit* out);
/* Peer.Commit's log part (peer.go:282-293 → entryLog.commitUpdate,
 * logentry.go:335-355; inMemory.savedLogTo / appliedLogTo, inmemory.go:
 * 108-167) for replica[i] with uc[i], as the node calls it once SaveRaftState
 * has persisted the Update (node.go:975-994): savedTo advances only to an
 * entry the in-memory log still holds with that term, processed to
 * uc.processed, the in-memory marker to uc.last_applied.  A host that lags
 * (or never) commits gets the unsaved entries and unprocessed committed
 * entries again in the next Update, as the reference's Peer does.  Staged and
 * applied before the next step, in call order; a replica takes one commit per
 * step (RBE_E_STATE for a second).  A reference panic (processed below the
 * current value or above committed; last_applied above committed or
 * processed) sets RBE_FAULT_PANIC in the replica's fault word.  Needs
 * cfg.ext_commit (RBE_E_STATE).  A non-zero stable_snapshot_to equal to the
 * index of the snapshot the replica restored (the Update's Snapshot) is
 * savedSnapshotTo (inmemory.go:168-176): later Updates stop carrying it; any
 * other value changes nothing (the reference only warns).  Until then every
 * Update of the replica carries the snapshot again (peer.go:345-347) and a
 * LogDB compaction (rbe_compact) waits.  With snapshots the engine's LogDB
 * holds every entry up to the raft log's last, as a node's does: its
 * UpdateCommit.LastApplied never passes the entries it has persisted (the
 * node saves an Update before it applies it, node.go:975-994). */
/* The Snapshot of the last round's Update of replicas [first, first + count)
 * (pb.Update.Snapshot, peer.go:345-347): four words each — index, term,
 * membership in the packed slot-mask form of rbe_launch_state::removed, 0 —
 * all zero when the Update carries none (RBE_UF_SNAPSHOT clear).  This is what
 * the node hands to LogReader.ApplySnapshot and the state machine
 * (node.go:950-965). */
int rbe_get_update_snapshots(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* out4);
int rbe_commit(rbe_engine* e, uint64_t n, const uint64_t* replica, const rbe_update_commit* uc);

/* ---- Transport wire format ------------------------
 * What a node writes on a TCP connection for Raft traffic: frames of a 2-byte
 * magic 0xAE7D, the 18-byte requestHeader (method 100, payload size, header
 * crc32, payload crc32, big endian; internal/transport/tcp.go:80-91, 149-185)
 * and a marshaled raftpb.MessageBatch (raft.pb.go:2415-2443: Messages
 * 2230-2294 with their colfer-form entries, raft_optimized.go:161-295).
 * rbe_wire_encode builds, on the device, one frame per (sender slot, receiver
 * slot, run of groups_per_batch groups) holding every message the last round
 * sent between those replicas (group order; per replica the rbe_get_outbox
 * order).  InstallSnapshot messages are left out and counted: the reference
 * streams them as snapshot chunks, never in a MessageBatch
 * (transport.go:400-403).  Entries carry every raftpb.Entry field (payload-heap
 * Cmds and session fields in full); a forwarded Propose carries its entries
 * (raft.go:1841-1853). */
typedef struct rbe_wire_frame {
  uint64_t offset, bytes;      /* frame (header included) in the encoded stream */
  uint64_t first_group;
  uint32_t src, dst;           /* sender / receiver replica slot (node id - 1) */
  uint32_t n_messages, n_groups;
} rbe_wire_frame;
typedef struct rbe_wire_config {
  uint64_t deployment_id;      /* MessageBatch.DeploymentId */
  uint32_t bin_ver;            /* MessageBatch.BinVer (raftio.RPCBinVersion) */
  uint32_t groups_per_batch;   /* 0 = every group in one batch per slot pair */
  const char* source_address[7];  /* MessageBatch.SourceAddress per sender slot (< 48 B) */
  /* replica mode (rep_world > 1): only the messages of the replicas stepped
   * here to replicas stepped by rank dst_rank (-1: by any other rank); the
   * stream for one remote engine, as a transport keeps one connection per
   * remote NodeHost.  Must be -1 with one replica set per engine. */
  int32_t dst_rank;
  uint32_t pad;
} rbe_wire_config;
/* totals = {bytes, frames, messages, InstallSnapshots left out}; the frames
 * stay in engine device memory until the next encode (rbe_wire_fetch). */
int rbe_wire_encode(rbe_engine* e, const rbe_wire_config* wc, uint64_t totals[4]);
int rbe_wire_fetch(rbe_engine* e, void* out, uint64_t cap, rbe_wire_frame* frames,
                   uint32_t frames_cap);
/* Decode back-to-back frames (host memory, as read from connections) on the
 * device: both crc32s checked per frame (readMessage, tcp.go:187-244), then
 * MessageBatch.Unmarshal (raft_optimized.go:654-1204) into records in frame
 * order.  Entry Cmd bytes are concatenated in `cmd` (rbe_entry.cmd holds the
 * first 16).  RBE_E_CORRUPT when any frame fails; RBE_E_NOMEM when a capacity
 * is short (the counts are still reported). */
int rbe_wire_decode(rbe_engine* e, const void* data, uint64_t bytes, rbe_message* msgs,
                    uint32_t cap, uint32_t* n_msgs, rbe_entry* ents, uint32_t ent_cap,
                    uint32_t* n_ents, uint8_t* cmd, uint64_t cmd_cap, uint64_t* cmd_bytes);
/* The receive side of the transport on the device (replica mode, rep_world >
 * 1): decode back-to-back frames as rbe_wire_decode does and deliver every
 * message to the next rbe_step exactly as rbe_push_messages would — the
 * records never come back to the host.  The group of a message is the one
 * whose cluster id is its ClusterId (cid_base + g * cid_stride); a response
 * from a node that is not a member is dropped (Peer.Handle, peer.go:186-198);
 * a message for a replica not stepped here, a local message type or a bad
 * entry is RBE_E_INVALID, a list over cfg.maxm messages, a sender over
 * cfg.ecap entries or a full payload heap RBE_E_NOMEM, a bad frame
 * RBE_E_CORRUPT — checked whole before anything is delivered.  All frames of
 * one round come in one call (concatenated streams of several senders are
 * fine); lists it does not name are empty.  Replaces transport.go:318-350
 * handleRequest → node.handleReceivedMessages (node.go:1030-1067). */
typedef struct rbe_wire_ingest_stats {
  uint64_t frames, messages, dropped, entries, cmd_bytes, heap_bytes;
} rbe_wire_ingest_stats;
int rbe_wire_ingest(rbe_engine* e, const void* data, uint64_t bytes, rbe_wire_ingest_stats* st);
/* The Cmd bytes of entries [lo, hi] of a replica's log, concatenated in `buf`:
 * entry lo + i occupies [offsets[i], offsets[i + 1]) (offsets has hi - lo + 2
 * slots and is filled even when `cap` is short, which returns RBE_E_NOMEM).
 * RBE_E_STATE when a heap Cmd has been overwritten by a later lap of the heap
 * (the entry is older than the heap holds, as ErrCompacted for LogDB reads).
 * Together with rbe_get_entries this is what the node reads out of
 * Update.EntriesToSave / CommittedEntries (node.go:975-977, 959-968). */
int rbe_get_entry_cmds(rbe_engine* e, uint64_t replica, uint64_t lo, uint64_t hi, uint8_t* buf,
                       uint64_t cap, uint64_t* offsets);
int rbe_get_views(rbe_engine* e, uint64_t first, uint64_t count, rbe_replica_view* out);
/* Rate limiter of replicas [first, first + count) (cfg.max_inmem_log_size):
 * Peer.RateLimited (peer.go:245-249, server/rate.go:109-137), one byte per
 * replica (1 = limited: its in-memory log or a follower report fresh within
 * two rate-limit ticks exceeds the limit), and rl.Get(), the in-memory log
 * bytes (Cmd + 80 per entry, raftpb/raft.go:311-322).  Either output may be
 * null.  RBE_E_STATE when the engine has no limiter. */
int rbe_rate_limited(rbe_engine* e, uint64_t first, uint64_t count, uint8_t* limited,
                     uint64_t* in_mem_log_size);

/* The last round's Update.Messages and Update.ReadyToReads of replicas
 * [first, first + count) in one call: compacted on the device (a count pass,
 * a scan, a write pass) and copied once into engine-owned pinned buffers.
 * Replica first + i owns messages[msg_off[i] .. msg_off[i + 1]) (per
 * destination in ascending node id, Replicate messages first, as
 * rbe_get_messages) and ready_to_reads[rtr_off[i] .. rtr_off[i + 1]).  The
 * pointers stay valid until the next rbe_collect_outputs, rbe_step/rbe_run or
 * rbe_destroy.  This is the batched read of the per-node Update the node loop
 * does after stepping every node (node.go:907-923, execengine.go:494-560). */
typedef struct rbe_outputs {
  uint64_t first, count, n_messages, n_ready_to_reads;
  const uint64_t* msg_off;              /* count + 1 */
  const rbe_message* messages;
  const uint64_t* rtr_off;              /* count + 1 */
  const rbe_ready_to_read* ready_to_reads;
} rbe_outputs;
int rbe_collect_outputs(rbe_engine* e, uint64_t first, uint64_t count, rbe_outputs* out);
/* The last round's Updates of replicas [first, first + count) that have one
 * (RBE_UF_HAS_UPDATE: Peer.HasUpdate, peer.go:253-280), compacted on the
 * device and copied once into an engine-owned pinned buffer: replica[i]'s
 * Update is updates[i], replicas ascending.  This is the node loop's read of
 * the Updates of the nodes that have one (execengine.go:494-560; a quiesced
 * node without events has none).  Valid until the next rbe_collect_updates,
 * rbe_step/rbe_run or rbe_destroy. */
typedef struct rbe_update_list {
  uint64_t first, count, n;
  const uint64_t* replica;
  const rbe_update* updates;
} rbe_update_list;
int rbe_collect_updates(rbe_engine* e, uint64_t first, uint64_t count, rbe_update_list* out);
/* The node loop's whole read after a step in one call (execengine.go:494-560,
 * node.go:888-923): the Updates of replicas [first, first + count) that have
 * one, and only for those replicas (a replica with Messages or ReadyToReads
 * always has an Update, peer.go:253-280) their ReadyToReads and Messages —
 * compacted on the device, copied once into an engine-owned pinned buffer.
 * replica[i] (ascending) has updates[i], messages[msg_off[i] .. msg_off[i+1])
 * and ready_to_reads[rtr_off[i] .. rtr_off[i+1]).  With
 * RBE_COLLECT_REMOTE_MSGS only the messages to replicas this engine does not
 * step are returned (rep_world > 1: the transport's share); the others the
 * engine delivers itself at the next step, so in group-per-GPU mode none is
 * copied.  With RBE_COLLECT_SKIP_LOCAL an Update whose only content is
 * messages the engine delivers itself (none returned under the flag above) is
 * left out: the node would have nothing to persist, apply, send or report for
 * it (no State change, entries, ReadyToReads, drops, Snapshot, applied index,
 * listener event or fault: a faulted replica's Update is always returned).
 * Valid until the next rbe_collect_step, rbe_step/rbe_run
 * or rbe_destroy. */
#define RBE_COLLECT_REMOTE_MSGS 1u
#define RBE_COLLECT_SKIP_LOCAL 2u
typedef struct rbe_step_outputs {
  uint64_t first, count, n, n_messages, n_ready_to_reads;
  const uint64_t* replica;                 /* n */
  const rbe_update* updates;               /* n */
  const uint64_t* msg_off;                 /* n + 1 */
  const rbe_message* messages;
  const uint64_t* rtr_off;                 /* n + 1 */
  const rbe_ready_to_read* ready_to_reads;
} rbe_step_outputs;
int rbe_collect_step(rbe_engine* e, uint64_t first, uint64_t count, uint32_t flags,
                     rbe_step_outputs* out);
/* rbe_collect_step in two halves, so the node layer's host work for the next
 * round (rbe_push_*) runs while the device collects this one:
 *   rbe_collect_step_begin enqueues the collection of the last round's
 *     outputs (the same records and flags as rbe_collect_step) and returns at
 *     once; the records go straight into engine-owned mapped host memory;
 *   rbe_collect_step_end waits for it and fills *out exactly as
 *     rbe_collect_step would.  When a round has more records than the buffer
 *     the engine sized from the earlier rounds, _end collects that round again
 *     synchronously (and grows the buffer).
 * Between the two no step may run (rbe_step / rbe_run: _end then returns
 * RBE_E_STATE); rbe_push_* and the other host-side calls may.  The records
 * live in one of two buffers used in turn: they stay valid through the next
 * _begin / _end pair (so the node can read them while the device runs the next
 * round) until the one after it, or rbe_destroy. */
int rbe_collect_step_begin(rbe_engine* e, uint64_t first, uint64_t count, uint32_t flags);
int rbe_collect_step_end(rbe_engine* e, rbe_step_outputs* out);
int rbe_get_counters(rbe_engine* e, uint64_t* out /* RBE_CTR_NUM */);
/* the counters one pipeline kernel (RBE_KERNEL_*) contributed */
int rbe_get_kernel_counters(rbe_engine* e, int32_t kernel, uint64_t* out /* RBE_CTR_NUM */);
int rbe_reset_counters(rbe_engine* e);
/* number of replicas whose sticky fault word holds a fault, and the OR of all
 * words */
int rbe_fault_summary(rbe_engine* e, uint64_t* n_faulty, uint32_t* fault_or);
/* The spill tiers' use (cfg.pool_bytes / spill_bytes; rbe_spill.h), after every
 * round queued: out[0] pool pages in use, out[1] pool pages, out[2] the most
 * round spill heap bytes one round used, out[3] its bytes per round parity,
 * out[4] exhaustion flags (bit 0 the pool, bits 1-2 the heap of parity 0 / 1;
 * sticky, the replicas concerned carry RBE_FAULT_NOMEM). */
int rbe_spill_stats(rbe_engine* e, uint64_t* out /* 5 */);

/* Replica-per-GPU mode (cfg.rep_world > 1).  The engine steps
 * only its own replicas; between rounds the host moves the messages of the
 * last round across ranks (the north star's RCCL all-to-all over xGMI):
 *   rbe_xchg_pack: packs the last round's records for every peer into the
 *     device buffer `buf`, laid out per peer p as stream 0 (count words),
 *     stream 1 (messages), stream 2 (Replicate entries) with cap3[t] records
 *     per stream; counts[p * 3 + t] receives the record counts
 *     (RBE_E_NOMEM if a capacity was exceeded);
 *   rbe_xchg_unpack: clears the engine's remote-sender count words of that
 *     round and scatters the received records (device pointers).
 * Record sizes come from rbe_xchg_record_bytes.  Replaces, for replicas on
 * other GPUs, the transport hop of node.go:888-905 → nodehost.go:1724. */
int rbe_xchg_record_bytes(uint64_t* out3);
/* Fixed-capacity variant without a host synchronisation (one all-to-all of
 * equal chunks per round, capturable in a graph): every peer's chunk of
 * rbe_xchg_chunk_bytes(cap3) bytes opens with a header holding its record
 * counts, so the receiver scatters what each chunk holds.
 *   rbe_xchg_pack_fixed: packs the last round's records into `buf` (rep_world
 *     chunks), enqueued on the engine stream, nothing read back;
 *   rbe_xchg_unpack_fixed: scatters a received buffer of the same layout;
 *   rbe_xchg_status: the overflow flag of the fixed exchanges since the last
 *     call, cleared by the read: set when some rank's records outgrew a chunk
 *     (every rank sees it, from the chunk headers it received).  The round's
 *     outboxes are intact until the next step: a counted exchange of the same
 *     round (rbe_xchg_pack / rbe_xchg_unpack) delivers every record again to
 *     its slot, which repairs it (dragonboat_amd/replica.py exchange_fixed);
 *   rbe_stream: the engine's HIP stream (hipStream_t), so a collective can be
 *     enqueued between pack and unpack without a host wait. */
int rbe_xchg_chunk_bytes(const uint64_t* cap3, uint64_t* bytes);
int rbe_xchg_pack_fixed(rbe_engine* e, void* buf, const uint64_t* cap3);
int rbe_xchg_unpack_fixed(rbe_engine* e, const void* recv, const uint64_t* cap3);
int rbe_xchg_status(rbe_engine* e, uint32_t* overflow);
int rbe_stream(rbe_engine* e, void** stream);
int rbe_xchg_pack(rbe_engine* e, void* buf, const uint64_t* cap3, uint32_t* counts);
int rbe_xchg_unpack(rbe_engine* e, const void* cnt_recs, uint64_t n_cnt, const void* msg_recs,
                    uint64_t n_msg, const void* ent_recs, uint64_t n_ent);
/* The isolation fault schedule (cfg.iso_period) in replica mode.  At an epoch
 * round the schedule cuts off the current leader of each selected group, and
 * no rank steps every replica of a group: before the step of an epoch round
 * each rank reads its replicas' leader bits (rbe_iso_leaders: *epoch = 1 when
 * the next step is an epoch round, then out[G] holds bit k for each replica
 * k of global group G stepped here that is a leader; cfg.n_groups bytes,
 * indexed by global group also with rep_compact), the host ORs
 * them over ranks (the bits are disjoint, so a sum all-reduce does it) and
 * hands the result back (rbe_set_iso_leaders).  rbe_step returns
 * RBE_E_STATE at an epoch round without it.  With one replica set per engine
 * the step does this itself. */
int rbe_iso_leaders(rbe_engine* e, uint8_t* out, uint32_t* epoch);
/* The engine's group count and, when global_of is non-null, the global group
 * of each local group (UINT64_MAX for the padding groups of a compacted
 * engine, which no rank steps).  Without cfg.rep_compact local = global. */
int rbe_local_groups(rbe_engine* e, uint64_t* n_local, uint64_t* global_of);
int rbe_set_iso_leaders(rbe_engine* e, const uint8_t* bits);

/* Transport boundary for replicas whose peers another engine steps (cfg.rep_world > 1:
 * the replicas of other ranks, or of other hosts behind dragonboat's transport).
 *   rbe_get_outbox: sender `replica`'s messages of the last round in raftpb form,
 *     per destination in ascending node id: the Quiesce notice (node.go:873-886),
 *     Replicate messages, the rest; each message's entries (a Replicate's, and
 *     a forwarded Propose's, raft.go:1841-1853) follow in `ents` (n_entries of
 *     them) with their whole Cmds concatenated in `cmd` (cmd_cap bytes;
 *     *cmd_bytes = the total; null skips them).  Counts beyond a capacity are
 *     reported and not written (RBE_OK; the caller compares).  RBE_E_STATE when
 *     a heap record has been overwritten.  Replaces reading Update.Messages for
 *     the transport (node.go:888-905 → nodehost.go:1724 sendMessages).
 *   rbe_push_messages: the round's inbound batch for the replicas this engine
 *     steps, delivered to the next rbe_step.  Replaces Peer.Handle (peer.go:186-198)
 *     as called by node.handleReceivedMessages (node.go:1030-1067): message i is
 *     for group group[i], from node msgs[i].from (not stepped here) to node
 *     msgs[i].to (stepped here), with msgs[i].n_entries entries taken in order from
 *     `ents` (a Replicate's: Index = LogIndex + 1 + j; a Propose's: any Index)
 *     and their Cmds concatenated in `cmd` (null: each is its rbe_entry.cmd).
 *     One call per round carries every remote message of that round; lists it
 *     does not name are empty.  Entries with Cmds over 16 bytes or session
 *     fields are written to this engine's payload heap.  RBE_E_STATE when
 *     rep_world <= 1 (every sender is local), RBE_E_NOMEM when one (sender,
 *     destination) list exceeds cfg.maxm, one sender's entries cfg.ecap, or
 *     the heap has no room. */
int rbe_get_outbox(rbe_engine* e, uint64_t replica, rbe_message* out, uint32_t cap,
                   uint32_t* n_out, rbe_entry* ents, uint32_t ent_cap, uint32_t* n_ents,
                   uint8_t* cmd, uint64_t cmd_cap, uint64_t* cmd_bytes);
int rbe_push_messages(rbe_engine* e, uint64_t n, const uint64_t* group, const rbe_message* msgs,
                      const rbe_entry* ents, const uint8_t* cmd);

/* Group-range snapshots: the complete protocol state of groups [first, first + count)
 * between two rounds (every replica's raft, remote, readIndex and log-window rows and
 * the groups' in-flight messages), laid out as in dragonboat_amd/csrc/rbe_snap.h.
 * Replaces what a restarted dragonboat node rebuilds from LogDB through Peer.Launch on
 * an existing log (peer.go:64-87, raft.go:283-330 loadState), and is the hand-off a
 * host slow path uses to run a rare handler on one group and put it back.
 *   rbe_snapshot_bytes: the size of `count` groups' header and planes (the fixed part);
 *   rbe_export_bytes: the whole snapshot of [first, first + count) as the engine stands:
 *     the fixed part, then the log section — every replica's log below its ring (the
 *     cold log, in 64-entry pages) and a readIndex queue longer than cfg.rq_cap
 *     (dragonboat_amd/csrc/rbe_spill.h) — so it grows with the logs it carries;
 *   rbe_export_groups: copies the range into `buf` (host memory, cap bytes; RBE_E_NOMEM
 *     when short), after every round already queued.  RBE_E_STATE when the range's last
 *     step left messages, entries, ReadyToReads or dropped ReadIndexes in the round
 *     spill heap (lists past cfg.maxm, entries past cfg.ecap, outputs past cfg.rtr_cap /
 *     cfg.dri_cap): step one more round and export then;
 *   rbe_import_groups: overwrites the snapshot's range (its old cold logs go back to the
 *     page pool first).  The engine must be at the snapshot's round (RBE_E_STATE
 *     otherwise), unless flags has RBE_IMPORT_RESUME and the snapshot covers every
 *     group: then the engine resumes at that round.  RBE_E_INVALID when the geometry
 *     (n, ring, capacities) differs or the log section does not match the planes;
 *     RBE_E_NOMEM when the page pool cannot take the log section. */
#define RBE_IMPORT_RESUME 0x1u
int rbe_snapshot_bytes(rbe_engine* e, uint64_t count, uint64_t* bytes);
int rbe_export_bytes(rbe_engine* e, uint64_t first, uint64_t count, uint64_t* bytes);
int rbe_export_groups(rbe_engine* e, uint64_t first, uint64_t count, void* buf, uint64_t cap);
int rbe_import_groups(rbe_engine* e, const void* buf, uint64_t bytes, uint32_t flags);

/* Device memory footprint (bytes) of a configuration, without allocating. */
int rbe_footprint(const rbe_config* cfg, uint64_t* bytes);

#ifdef __cplusplus
}
#endif

#endif /* DRAGONBOAT_AMD_RBE_H_ */
