// MI355X batched Raft step engine — struct-of-arrays layout in HBM.
//
// The per-group protocol state that dragonboat's internal/raft keeps in Go
// structs and maps (raft.go:197-232 raft, remote.go:62-69 remote,
// readindex.go:31-34 readIndex, inmemory.go:36-44 inMemory) lives here as
// planes indexed by the global replica index r = g * N + k (group g, replica
// slot k, node ID k + 1).  See DESIGN.md §Data layout for the byte budget.
#pragma once
#include <stdint.h>

namespace rbe {

typedef uint64_t u64;
typedef uint32_t u32;
typedef uint16_t u16;
typedef uint8_t u8;

// the largest group size (voting slots per group) the engine is built for
static constexpr u32 kMaxN = 7;

// raftpb MessageType, raft.pb.go:23-51
enum : u32 {
  M_LocalTick = 0, M_Election = 1, M_LeaderHeartbeat = 2, M_ConfigChangeEvent = 3,
  M_NoOP = 4, M_Ping = 5, M_Pong = 6, M_Propose = 7, M_SnapshotStatus = 8,
  M_Unreachable = 9, M_CheckQuorum = 10, M_BatchedReadIndex = 11, M_Replicate = 12,
  M_ReplicateResp = 13, M_RequestVote = 14, M_RequestVoteResp = 15,
  M_InstallSnapshot = 16, M_Heartbeat = 17, M_HeartbeatResp = 18, M_ReadIndex = 19,
  M_ReadIndexResp = 20, M_Quiesce = 21, M_SnapshotReceived = 22,
  M_LeaderTransfer = 23, M_TimeoutNow = 24, M_RateLimit = 25
};

// raft State, raft.go:63-70 (observer/witness are host slow path)
enum : u8 { R_Follower = 0, R_Candidate = 1, R_Leader = 2, R_Observer = 3, R_Witness = 4 };
// remote flow-control states, remote.go:27-32
enum : u8 { RS_Retry = 0, RS_Wait = 1, RS_Replicate = 2, RS_Snapshot = 3 };
// entry types, raft.pb.go:138-141
enum : u32 { E_Application = 0, E_ConfigChange = 1, E_Encoded = 2, E_Metadata = 3 };
// Body/Ent `type` bit 16: the entry is a payload-heap record.  Its Cmd (any
// length) and its session fields live in the engine's heap at absolute position
// `hi` as {Key, ClientID, SeriesID, RespondedTo} (kHeapHdr bytes, raft.pb.go:
// 589-598) followed by the Cmd bytes; `lo` is the record's fingerprint
// (rbe_host.h entry_fingerprint), which the trace digest folds for it.  An
// entry without the bit carries Cmd <= 16 bytes inline in lo/hi and zero
// session fields.  The entry type proper is `type & ET_TYPE_MASK`.
enum : u32 { ET_HEAP = 1u << 16, ET_TYPE_MASK = 0xFFFFu };
static constexpr u32 kHeapHdr = 32;

// sticky per-replica fault bits (the engine-side analog of plog.Panicf: the
// replica stops being trustworthy, the engine keeps running, the host sees it)
// Since round 6 no capacity of the planes is a fault: a full list, arena or
// queue spills into the spill tiers (rbe_spill.h).  F_OUTBOX / F_ARENA /
// F_READQ / F_RTR / F_DROPLIST are no longer raised; F_WINDOW means a log
// entry the engine should hold is missing (an engine bug, or a launch that
// handed over only the tail of a LogDB), and F_NOMEM that a spill tier
// itself is exhausted (an engine resource: cfg.pool_bytes / spill_bytes).
enum : u32 {
  F_WINDOW = 1u << 0,       // a log entry the replica holds is missing from the ring and the cold log
  F_OUTBOX = 1u << 1,       // (unused since round 6: full lists spill)
  F_ARENA = 1u << 2,        // (unused since round 6: full arenas spill)
  F_READQ = 1u << 3,        // (unused since round 6: the readIndex queue grows into the pool)
  F_RTR = 1u << 4,          // (unused since round 6: full ReadyToRead lists spill)
  F_PANIC = 1u << 5,        // a reference panic condition (e.g. commitTo > lastIndex)
  F_UNSUPPORTED = 1u << 6,  // a slow-path message/entry type reached the device
  F_DROPLIST = 1u << 7,     // (unused since round 6: full dropped-ReadIndex lists spill)
  F_NOMEM = 1u << 8,        // the page pool or the round spill heap is exhausted (engine resource)
};

// hot plane: everything a quiesced tick touches (32 B per replica)
struct alignas(16) Hot {
  u8 role;
  u8 flags;          // HF_* below
  u8 votes_resp;     // bit (id-1): a RequestVoteResp was counted from id (raft.votes keys)
  u8 votes_granted;  // bit (id-1): that response granted the vote (raft.votes values)
  u32 election_tick;
  u16 heartbeat_tick;
  u16 rand_et;       // randomizedElectionTimeout
  u32 q_tick;        // quiesceManager (quiesce.go:23-33)
  u32 q_quiesced_since;
  u32 q_no_activity_since;
  u32 q_exit_quiesce_tick;
  u32 rng_count;     // randomized timeouts drawn so far (injected PRNG counter)
};
enum : u8 {
  HF_RAFT_QUIESCE = 1,  // raft.quiesce
  HF_PENDING_CC = 2,    // raft.pendingConfigChange
  HF_IS_LTT = 4,        // raft.isLeaderTransferTarget
  HF_APPLY_PENDING = 8, // processed < committed after the step (apply limited by size)
  HF_FAULTED = 16,      // Upd.fault != 0 (the sticky fault word is read only then)
  HF_APPLY_HELD = 64,   // the node's apply queue is full (rbe_set_apply_ready, the
                        // moreEntriesToApply = false of node.go:908-915): the step
                        // returns no CommittedEntries
  HF_APPLIED_NEW = 32,  // the last step returned committed entries: the node's
                        // confirmedIndex lags its applied index until the next
                        // step (node.go:907-923, 1033), an event of its own
  HF_SNAP_WORK = 128,   // SnapSt has a compaction or a SnapshotStatus for the next
                        // step (snapshot_entries > 0): triage sends it to k_full
};

// Core::members / Core::mflags / Core::cc_apply bits
enum : u8 {
  MB_REMOVED = 0x7F,   // members: slots that are not in raft.remotes (bit s = slot s, kMaxN = 7)
  MB_ROLES = 0x01,     // mflags: some slot is an observer or a witness (Planes::roles)
  MB_CC_IN_LOG = 0x02, // mflags: a ConfigChange entry may sit in (processed, last_index]
  CCA_VALID = 0x80, CCA_REJECT = 0x40,  // cc_apply: node id bits 0-2, ConfigChangeType bits 3-4
  CCA_MULTI = 0x20,  // cc_apply: several ConfigChanges, in the last step's apply range (Upd::cc_acc)
};
// pb.ConfigChangeType (raft.pb.go)
enum : u32 { CC_AddNode = 0, CC_RemoveNode = 1, CC_AddObserver = 2, CC_AddWitness = 3 };

// core plane (64 B per replica)
struct alignas(16) Core {
  u64 term;
  u64 committed;   // entryLog.committed
  u64 last_index;  // entryLog.lastIndex()
  u64 processed;   // entryLog.processed == node smAppliedIndex after each step
  u64 saved_to;    // inMemory.savedTo
  u8 vote;         // node IDs are slot+1; 0 = NoNode
  u8 leader;
  u8 ltt;          // leaderTransferTarget
  u8 rq_head;      // readIndex queue ring head
  u8 rq_count;
  // membership (cfg.membership; all zero otherwise): members has a bit per
  // slot that is not a voting member of this replica's raft.remotes (the
  // group starts with every slot a voter); mflags MB_CC_IN_LOG (a ConfigChange
  // entry may sit in (processed, last_index]) and MB_ROLES; cc_apply a
  // ConfigChange for the next step (CCA_* bits: the state machine applied
  // one, or the host sent it)
  u8 members;
  u8 cc_apply;
  u8 mflags;       // MB_ROLES | MB_CC_IN_LOG (membership)
  u64 t_last;      // term of entry last_index (log-tail cache)
  u64 lead_start;  // leader: index of its no-op, the first entry of its term (raft.go:985);
                   // entries [lead_start, last_index] have term == term, earlier ones less
};

// node snapshot / LogDB compaction state (snapshot_entries > 0; 64 B per
// replica).  marker is the LogDB's compaction marker (logdb: entries at or
// below it are gone, Term(marker) = marker_term); ss_* the LogDB's latest
// snapshot (CreateSnapshot or one received by InstallSnapshot, ApplySnapshot);
// ss_req / compact_to the node's reqSnapshotIndex and compactLogTo (node.go
// 585-605, 849-866); pend / pend_rej the SnapshotStatus the transport reports
// for this replica's InstallSnapshots of the last step (bit id-1 per target).
// Membership (cfg.membership; the Core::members encoding, bit id-1 = not a
// voting member): ss_rem of the LogDB's snapshot (pb.Snapshot.Membership,
// raft.pb.go:733-739, the voters it lists), sm_rem the state machine's own
// (rsm membership: every ConfigChange it applied, or the snapshot it
// recovered from), which a new snapshot records; rr_pend = a
// RestoreRemotes(ss_rem) is due at the next step (the node calls it once the
// state machine recovered from a snapshot, rsm/statemachine.go:236 →
// peer.go:159-165).
struct alignas(16) SnapSt {
  u64 marker, marker_term;
  u64 ss_index, ss_term;
  u64 ss_req, compact_to;
  u8 pend, pend_rej;
  u8 ss_rem, sm_rem, rr_pend;
  // observers / witnesses of the snapshot's and the state machine's membership
  // (Membership.Observers / Witnesses, bit s = slot s)
  u8 ss_obs, ss_wit, sm_obs, sm_wit;
  // the snapshot restored from the last InstallSnapshot (inMemory.snapshot,
  // inmemory.go:236-246): its membership, and with ext_commit upd_ss = the
  // host has not yet committed an Update carrying it (savedSnapshotTo,
  // inmemory.go:168-176), so every Update carries it again.  Its index and term
  // are marker / marker_term: the LogDB took it (ApplySnapshot) and a
  // compaction waits until the host has committed it (node_snapshot)
  u8 upd_ss, upd_rem, upd_obs, upd_wit;
  u8 pad[3];
};

// remote slot (remote.go:62-69): match/next; state|active<<2 lives in a u8 plane
struct alignas(16) RemoteMN {
  u64 match;
  u64 next;
};

// readIndex queue entry (readindex.go:24-29): 32 B
struct alignas(16) ReadReq {
  u64 low, high;   // SystemCtx
  u64 index;
  u8 from;         // node id (0 = local)
  u8 confirmed;    // bit (id-1) per confirming node
  u8 pad[6];
};

// payload ring body (24 B): the entry fields besides Index/Term
struct Body {
  u32 type;
  u32 len;   // Cmd length, <= 16
  u64 lo, hi;  // Cmd bytes, little endian
};

// message record in a per-(sender,dest) outbox list: 64 B
struct alignas(16) Msg {
  u8 type, from, to, reject;
  u16 n_ent;
  u16 pad0;
  u32 ent_off;  // offset of the first entry in the sender's per-round arena
  u32 pad1;
  u64 term, log_term, log_index, commit, hint, hint_high;
};

// Outbox header of one sender replica for one round (16 B): the count word of
// each destination list — A (Replicate messages, front of the list) | B (the
// rest, back of the list) << 7 | Quiesce notice << 15 — stamped with the round
// that reads it (the writer's round + 1).  A sender that makes no step in a
// round (a lazily skipped quiesced tick) writes no row, and the stale row of
// that parity reads as empty, so nothing ever has to be cleared.  Six words
// serve groups of up to 7: a sender has no list to itself, so the word of
// destination slot 6 takes the sender's own index (cnt_widx).
struct alignas(16) CntRow {
  u32 stamp;
  u16 w[6];
};


// arena entry: 32 B (index implicit: log_index + 1 + i for Replicate)
struct alignas(16) Ent {
  u64 term;
  u32 type;
  u32 len;
  u64 lo, hi;
};

// per-replica step output record (Update summary).  Four
// 16-B chunks; the last one (fault, flags, events, round, message and
// ReadyToRead counts) is written by every step.  Chunks 0-2 (digest, the
// EntriesToSave / CommittedEntries ranges, drop counts) are written only when
// UF_RANGES is set in that step's flags: an untraced steady-state step with
// empty ranges and no drops (most C4 rounds) stores one chunk, not four, and a
// reader treats a record without UF_RANGES as empty ranges and no drops.
struct alignas(16) Upd {
  u64 digest;       // running trace digest (trace mode)
  u64 save_lo;      // EntriesToSave = [save_lo, save_hi] (empty if lo > hi)
  u64 save_hi;
  u64 apply_lo;     // CommittedEntries = [apply_lo, apply_hi]
  u64 apply_hi;
  u16 n_drop_ent;   // DroppedEntries
  u16 n_drop_ri;    // DroppedReadIndexes
  u32 cc_acc;       // membership: bit i = the i-th ConfigChange of the apply range was
                    // accepted by the engine's state machine (Core::cc_apply CCA_MULTI)
  u32 fault;        // sticky F_* bits
  u16 flags;        // UF_* bits
  u16 events;       // EV_* bits: IRaftEventListener calls of the step
  u32 round;        // round this record was written in (idle rounds leave it stale)
  u16 n_msgs;       // messages emitted this step (Update.Messages)
  u16 n_rtr;        // ReadyToReads
};
enum : u32 {
  UF_STATE_CHANGED = 1, UF_SENT_QUIESCE = 2, UF_HAS_UPDATE = 4,
  UF_SNAPSHOT = 0x20,  // Update.Snapshot: the step restored a snapshot from InstallSnapshot
                       // (or, with ext_commit, one the host has not committed yet): index /
                       // term SnapSt::marker / marker_term, membership SnapSt::upd_*;
                       // the same bit as RBE_UF_SNAPSHOT
  UF_APPLIED = 0x40,   // ext_apply: the state machine's applied index changed for this step,
                       // so the node takes an Update even without other content (node.go:
                       // 907-923 confirmedIndex); the same bit as RBE_UF_APPLIED
  UF_RANGES = 0x100
};
// server.IRaftEventListener (internal/server/event.go) calls a step made, one
// bit per event kind (raft.go:354, 1090, 1333, 1368, 1503, 1995, 2010).
// LeaderUpdated fires on every setLeaderID call in the reference, unchanged
// leaders included (SURVEY.md appendix trap 9); EV_LEADER_UPDATED marks a step
// whose leader value changed, the event a listener acts on (event.go:93-95).
enum : u32 {
  EV_LEADER_UPDATED = 1, EV_CAMPAIGN_LAUNCHED = 2, EV_CAMPAIGN_SKIPPED = 4,
  EV_SNAPSHOT_REJECTED = 8, EV_REPLICATION_REJECTED = 16, EV_PROPOSAL_DROPPED = 32,
  EV_READ_INDEX_DROPPED = 64
};

struct RTR {  // ReadyToRead, raftpb/raft.go:52-56
  u64 index, low, high;
};
struct DropRI {  // SystemCtx
  u64 low, high;
};

// Host-pushed input of one replica, consumed by the next step: the node-side
// events of handleEvents (node.go:1030-1067) that are not network messages
// (rbe_push_proposals / rbe_push_read_index / rbe_request_leader_transfer /
// rbe_report_unreachable / rbe_report_snapshot_status).  `flags` says which
// parts are present; a replica takes at most one of each per step, as the
// node batches them (one ReadIndex ctx per step, node.go:1379-1382; one
// proposal batch, 1091-1106; one pending transfer, 1069-1075).
enum : u32 {
  EXT_PROPOSE = 1, EXT_READ = 2, EXT_XFER = 4, EXT_UNREACH = 8, EXT_SNAPST = 16,
  EXT_APPLIED = 32,  // rbe_notify_applied changed raft.applied (an event, node.go:1033)
  EXT_CC_PROPOSE = 64,  // Peer.ProposeConfigChange: ExtIn::pad[0] = type | node id << 8
  EXT_CC_APPLY = 128,   // Peer.ApplyConfigChange / RejectConfigChange: pad[1] = a cc_apply byte
  EXT_RESTORE = 256,    // Peer.RestoreRemotes: pad[2] = the snapshot's membership (removed mask)
};
struct alignas(16) ExtIn {
  u32 flags;
  u32 n_prop;        // entries of the proposal batch (EXT_PROPOSE)
  u32 prop_off;      // its first entry in Planes::in_ents
  u8 xfer_target;    // RequestLeaderTransfer target node id (EXT_XFER)
  u8 unreach;        // ReportUnreachableNode: bit (id-1) per node (EXT_UNREACH)
  u8 snap_nodes;     // ReportSnapshotStatus: bit (id-1) per node (EXT_SNAPST)
  u8 snap_reject;    //   ... reject flag per node
  u64 ctx_low, ctx_high;  // ReadIndex SystemCtx (EXT_READ)
  u64 pad[4];
};

// counters (shared numbering with oracle/harness.h HC_*)
enum : int {
  C_STEPS = 0, C_COMMITTED = 1, C_MSG_IN = 2, C_MSG_OUT = 3, C_ENT_IN = 4, C_ENT_OUT = 5,
  C_READS_CONFIRMED = 6, C_PROPOSALS = 7, C_READS = 8, C_QUIESCED_TICKS = 9,
  C_ACTIVE_TICKS = 10, C_CAMPAIGNS = 11, C_ENT_SAVED = 12, C_ENT_APPLIED = 13,
  C_MSG_DROPPED = 14, C_DROPPED_PROPOSALS = 15, C_DROPPED_READS = 16, C_LEADER_STEPS = 17,
  C_REMOTE_TOUCH = 18, C_RING_ACCESS = 19, C_FAULTS = 20, C_RQ_TOUCH = 21,
  C_NUM = 24
};

// engine parameters (immutable for a handle)
struct Params {
  u64 n_groups;
  u64 n_rep;          // N * n_groups
  u64 cid_base;       // cluster id of group g is cid_base + g * cid_stride
  u64 cid_stride;
  u64 seed;
  u64 max_entry_size;
  u32 n;              // replica slots per group (N)
  u32 n_voters;       // slots 0..n_voters-1 bootstrap the group, the rest join later
  u32 obs_slots;      // slots (beyond n_voters) whose nodes start as observers (config.IsObserver)
  u32 wit_slots;      // ... as witnesses (config.IsWitness)
  u32 ring;           // term/payload ring entries (power of two)
  u32 rq_cap;         // readIndex queue capacity
  u32 maxm;           // message slots per (sender, dest) per round
  u32 ecap;           // arena entries per sender per round
  u32 rtr_cap;        // ReadyToRead slots per replica per round
  u32 dri_cap;        // dropped ReadIndex slots per replica per round
  u32 election_rtt;
  u32 heartbeat_rtt;
  u32 check_quorum;
  u32 quiesce;
  u32 trace;
  // workload
  u32 wl_enabled, wl_start_round, wl_stop_round, wl_active_mod, wl_read_permille;
  u32 ext_inputs;     // consume host-pushed ExtIn records
  // faults
  u32 iso_period, iso_len, iso_mod;
  u32 rep_world;      // replica-per-GPU mode when > 1 (rbe_xchg.h)
  u32 rep_rank;
  u32 ext_apply;      // applied index comes from rbe_notify_applied (raft.applied lags processed)
  u32 ext_commit;     // Peer.Commit's log part comes from rbe_commit (savedTo/processed lag)
  u32 membership;     // ConfigChange entries on the device (Core::members / cc_apply)
  u32 cc_period, cc_mod;  // config-change schedule (rbe_step.h cc_selected), 0 = off
  u32 snapshot_entries;     // config.SnapshotEntries: snapshot + compact every that many applied entries (0 = never)
  u32 compaction_overhead;  // config.CompactionOverhead: entries kept below the snapshot
  u32 in_cap;         // host-pushed proposal entries per step (Planes::in_ents)
  u64 heap_bytes;     // per-replica payload heap for commands > 16 B (0 = inline commands only)
  // leader-transfer schedule (RequestLeaderTransfer on a seeded replica), 0 = off
  u32 xfer_period;
  u32 xfer_mod;
  // replica mode with compacted planes (rbe_xchg.h rep_compact_setup): local
  // group l is global group (l / n) * rep_world + res[l % n]
  u32 rep_compact;
  u64 n_groups_glob;  // global group count (= n_groups without compaction)
  u8 res[8];          // the n residues g % rep_world of the groups this rank touches, ascending
  u64 rl_max;         // config.MaxInMemLogSize (server.NewRateLimiter); 0 = limiter off
  // spill tiers (rbe_spill.h)
  u32 pool_pages;     // pages of the page pool (cold log, readIndex queue beyond rq_cap)
  u64 spill_units;    // 16-B granules of the round spill heap, per round parity
};

// Spill tiers (rbe_spill.h).  Page pool: kPageEnts 32-B records a page (log
// entries of the cold log, or ReadReq of a readIndex queue beyond rq_cap);
// page 0 is the null page.  PoolMeta links a page into its owner's chain
// (ascending page numbers), or into a free stack.
static constexpr u32 kPageEnts = 64;
struct alignas(16) PoolMeta {
  u64 pn;         // cold log: the page's entries are [pn * kPageEnts, + kPageEnts)
  u32 prev, next;
};
// A replica's cold log: the entries evicted from its term / payload ring, in
// pages head .. tail (ascending pn); 0 = none
struct alignas(16) ColdRef {
  u32 head, tail;
  u64 tail_pn;
};
// allocation words of the spill tiers, each on its own 256-B line
struct alignas(256) SpillCtl {
  u32 bump;          // next page never handed out (starts at 1)
  u32 oom;           // sticky: bit 0 the page pool, bits 1-2 the round spill heap of parity 0 / 1
  u32 live;          // pages in use
  u32 pad0[61];
  u32 free_head[2];  // free page stacks: a round of parity p frees into [p], takes from [p ^ 1]
  u32 pad1[62];
  u64 used[2];       // round spill heap granules handed out, by round parity
  u64 pad2[30];
  u64 peak[2];       // the largest `used` a round reached (diagnostics, rbe_spill_stats)
  u64 pad3[30];
};

// The rate limiter of one replica (internal/server/rate.go:33-137, raft.go:204)
// with the raft fields only it reads: raft.tickCount (raft.go:551-564) and
// inMemory.newEntries (inmemory.go:36-44).  Follower reports are kept per node
// slot.  Allocated only when Params::rl_max enables the limiter.
struct alignas(16) RlSt {
  u64 size;        // rl.size: in-memory log bytes (Cmd + 80 per entry, raftpb/raft.go:311-322)
  u64 tick;        // rl.tick (HeartbeatTick)
  u64 tick_count;  // raft.tickCount
  u32 new_ent;     // inMemory.newEntries
  u32 fmask;       // followerSizes holds node slot s
  u64 f_tick[8];
  u64 f_size[8];
};
static constexpr u64 kRlGcTick = 2;           // rate.go:25 gcTick
static constexpr u64 kEntryInMem = 80;        // unsafe.Sizeof(pb.Entry) on 64-bit Go
static constexpr u64 kEntryNonCmd = 16 * 8;   // settings.EntryNonCmdFieldsSize (soft.go:20)


// The clock of one round: `round` numbers every rbe_step, `tclk` counts the
// ticks before it (every replica ticks together, as tickWorkerMain ticks
// every node, nodehost.go:1668-1684), `tick` says whether this round ticks.
struct Clk {
  u32 round, tclk, tick;
};

// Planes::gwake bit 0: the group is awake (rbe_step.h, group sleep)
enum : u8 { GW_AWAKE = 1 };

// Planes::prof (diagnostic builds): header [0] the wave-record counter
// (RBE_FULL_PROF), [1] the item-record counter (RBE_FULL_ITEM_PROF), [8, 32)
// the RBE_PHASE_TIMING sums (rbe_fast.h); the records follow the header
static constexpr u64 kProfHdr = 32;
static constexpr u64 kFullProfCap = 1u << 20;  // wave records (4 words each)
static constexpr u64 kFullItemCap = 1u << 19;  // item records (8 words each)

// device pointers of every plane
struct Planes {
  Hot* hot;
  Core* core;
  RemoteMN* rem;      // [n_rep * N]
  u8* rem_st;         // [n_rep * N]  state | active << 2
  ReadReq* rq;        // [n_rep * rq_cap]
  u64* term_ring;     // [ring][n_rep]
  Body* pay_ring;     // [ring][n_rep]
  CntRow* cnt[2];     // [n_rep] outbox header of each sender, by round parity
  Msg* msgs[2];       // [n_groups * N * N * maxm]
  Ent* arena[2];      // [n_rep * ecap]
  u8* iso_mask;       // [n_groups]
  u8* idle;           // [n_rep] IB_* bits: lets k_triage finish a lazily quiesced round
                      // without reading Hot (rbe_step.h, idle_byte)
  u32* iso_until;     // [n_groups]
  Upd* upd;           // [n_rep]
  RTR* rtr;           // [n_rep * rtr_cap]
  DropRI* dri;        // [n_rep * dri_cap]
  ExtIn* ext;         // [n_rep]
  Ent* in_ents;       // [in_cap] proposal entries pushed for the next step
  u64* applied;       // [n_rep] raft.applied from rbe_notify_applied (ext_apply)
  SnapSt* snp;        // [n_rep] node snapshot state (snapshot_entries > 0, else null)
  u64* rem_snap;      // [n_rep * N] remote.snapshotIndex (read only in RS_Snapshot)
  u8* gwake;          // [n_groups] GW_* bits: lets k_triage skip a sleeping group whole
                      // (rbe_step.h, group sleep)
  RlSt* rl;           // [n_rep] rate limiters (Params::rl_max != 0, else null)
  u64* imark;         // [n_rep] inMemory.markerIndex (ext_commit or rl_max, else null): the first
                      // entry the in-memory log holds (inmemory.go:36-44), which bounds
                      // what savedLogTo / appliedLogTo accept
  const u64* heap_head;  // [1] payload heap: the host's next free position after the
                         // last upload; a record at p < *heap_head - heap_bytes has been
                         // overwritten by a later lap (null without a heap)
  u64* counters;      // [C_NUM]
  // [n_groups * N] the node id of each group's slots (rbe_set_node_ids), or
  // null: slot s is node s + 1.  Only the boundary's converters read it: the
  // protocol state inside the engine names nodes by slot + 1
  const u64* node_ids;
  u32 ids_n;           // slots per group (Params::n), for indexing node_ids in kernels without Params
  // [n_rep] (membership) each replica's observers | witnesses << 8, bit s =
  // slot s: raft.observers / raft.witnesses (raft.go:206-207), read by the full
  // handler table only (Core::members has MB_ROLES while any is set)
  u16* roles;
  // diagnostic builds only (-DRBE_FULL_PROF): k_full_list's wave records
  // (rbe_debug_full_prof); null otherwise
  u64* prof;
  // spill tiers (rbe_spill.h)
  Ent* pool;          // [pool_pages * kPageEnts] page pool records
  PoolMeta* pmeta;    // [pool_pages]
  ColdRef* cold;      // [n_rep] each replica's cold log
  u8* spill[2];       // [spill_units * 16] round spill heap, by round parity
  SpillCtl* sctl;     // [1]
};

// Store audit of the fast step (scripts/store_audit.py): a host
// build of the step (tests/soa_cpu) with -DRBE_STORE_AUDIT counts every global
// store a fast step makes, per site, while g_audit_on is set (bytes in the low
// 32 bits of `bytes`; a message store puts its type above them).  Expands to
// nothing in the device build and in every default build.
enum : u32 {
  AS_MSG, AS_DRI, AS_RTR, AS_SNAP, AS_UPD, AS_UPD3, AS_CNT, AS_HOT, AS_CORE, AS_IDLE,
  AS_COLD_REF, AS_COLD_ENT, AS_COLD_META, AS_TERM, AS_PAY, AS_EXT, AS_REM, AS_REM_ST, AS_RQ,
  AS_STASH, AS_NUM
};
#if defined(RBE_STORE_AUDIT) && !defined(__HIP_DEVICE_COMPILE__)
extern bool g_audit_on;
extern u64 g_store_audit[AS_NUM][2];
void audit_store(u32 site, const void* at, u64 bytes);  // address trace (tests/soa_cpu)
#define RBE_AUDIT(site, at, bytes)                                    \
  do {                                                                \
    if (::rbe::g_audit_on) {                                          \
      ::rbe::g_store_audit[site][0]++;                                \
      ::rbe::g_store_audit[site][1] += (::rbe::u64)(bytes)&0xFFFFFFFFu; \
      ::rbe::audit_store(site, at, bytes);                            \
    }                                                                 \
  } while (0)
#else
#define RBE_AUDIT(site, at, bytes) ((void)0)
#endif

}  // namespace rbe
