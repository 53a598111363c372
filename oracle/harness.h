// ORACLE — TEST INFRASTRUCTURE ONLY (see raft_ref.h header comment).
//
// Deterministic lockstep harness around the raft restatement: it runs the
// dragonboat node step loop (node.go:1016-1067 stepNode/handleEvents,
// 1171-1205 handleReceivedMessages, 1384-1399 tick, quiesce.go) for many
// independent groups, delivering every message emitted in round r at round
// r+1, exactly as node_test.go:270-401 (step/stepNodes) drive a cluster.
// The MI355X engine implements the same round semantics on device; both are
// specified in DESIGN.md §Round semantics and must agree bit for bit.
#pragma once
#include <cstdint>
#include <vector>

#include "raft_ref.h"

namespace orc {

// Counter slots, shared numbering with the engine (include/rbe.h RBE_CTR_*).
enum HarnessCounter {
  HC_STEPS = 0,           // replica-steps with >=1 input (every replica ticks every round)
  HC_COMMITTED = 1,       // leader commit advances (entries committed, once per group)
  HC_MSG_IN = 2,          // messages handled from the inbox (incl. Quiesce)
  HC_MSG_OUT = 3,         // messages delivered to the network (after drops)
  HC_ENT_IN = 4,          // entries carried by handled messages
  HC_ENT_OUT = 5,         // entries carried by delivered messages
  HC_READS_CONFIRMED = 6, // ReadyToRead records produced
  HC_PROPOSALS = 7,       // proposals injected by the workload
  HC_READS = 8,           // ReadIndex requests injected by the workload
  HC_QUIESCED_TICKS = 9,  // QuiescedTick calls
  HC_ACTIVE_TICKS = 10,   // Tick calls
  HC_CAMPAIGNS = 11,      // campaign() calls
  HC_ENT_SAVED = 12,      // entries in EntriesToSave
  HC_ENT_APPLIED = 13,    // entries in CommittedEntries
  HC_MSG_DROPPED = 14,    // messages dropped by the fault schedule
  HC_DROPPED_PROPOSALS = 15,
  HC_DROPPED_READS = 16,
  HC_LEADER_STEPS = 17,   // replica-steps that end as leader
  HC_NUM = 24
};

struct HarnessConfig {
  u64 n_groups = 1;
  u32 n_replicas = 3;
  u64 cid_base = 1;            // cluster id of group g is cid_base + g * cid_stride
  u64 cid_stride = 1;
  u64 election_rtt = 10;
  u64 heartbeat_rtt = 1;
  bool check_quorum = false;
  bool quiesce = false;
  u64 seed = 0x5EEDD8A6ULL;
  u64 max_entry_size = DefaultMaxEntrySize;
  // workload
  u32 wl_start_round = 0;      // no client input before this round
  u32 wl_stop_round = 0;       // no client input from this round on (0 = never stop)
  u32 wl_active_mod = 1;       // group active iff mix(seed,cid) % mod == 0
  u32 wl_read_permille = 0;    // per active group per round: read w.p. p/1000 else propose
  u32 wl_enabled = 0;          // 0: no client input at all
  // fault schedule: isolate the leader(s) of selected groups
  u32 iso_period = 0;          // 0 = no faults
  u32 iso_len = 0;
  u32 iso_mod = 10;
  // tracing
  u32 trace = 1;               // compute per-replica digests
  u32 threads = 1;             // worker threads (groups partitioned cid % T)
  // leader-transfer schedule: RequestLeaderTransfer on a seeded replica
  u32 xfer_period = 0;         // 0 = off
  u32 xfer_mod = 1;
  // host-driven mode: raft.applied comes from harness_push(PUSH_APPLIED)
  u32 ext_apply = 0;
  // config.SnapshotEntries / CompactionOverhead (config/config.go): the node
  // snapshots every SnapshotEntries applied entries and compacts its LogDB to
  // snapshot index - CompactionOverhead at its next step (harness.cpp)
  u32 snapshot_entries = 0;
  u32 compaction_overhead = 0;
  // host-driven persistence: Peer.Commit's log part (entryLog.commitUpdate)
  // comes from harness_commit, the engine's rbe_commit (needs ext_apply)
  u32 ext_commit = 0;
  // membership change (raft.go:1135-1237, peer.go:126-157): committed
  // ConfigChange entries in the harness's stand-in encoding (cc_cmd) are
  // applied to raft at the node's next step (ApplyConfigChange), unless the
  // host applies them (ext_apply: PUSH_CC_APPLY / PUSH_CC_REJECT)
  u32 membership = 0;
  // config-change schedule: every cc_period-th round, in groups selected 1 in
  // cc_mod, the replica leading at round start proposes removing a seeded
  // voter (while more than two vote) or adding it back (cc_input)
  u32 cc_period = 0;
  u32 cc_mod = 1;
  // voting members a group starts with (0 = n_replicas): slots 0..n_voters-1
  // bootstrap the group, the others are nodes that join later (Launch with
  // no peers, initial = false: an empty log, no remotes) once an AddNode for
  // them is applied (needs membership)
  u32 n_voters = 0;
  // config.MaxInMemLogSize (below), then the slots (beyond n_voters) whose nodes
  // start as observers / witnesses (config.IsObserver / IsWitness): every raft's rate limiter (0 = off)
  u64 max_inmem_log_size = 0;
  u32 observer_slots = 0, witness_slots = 0;
};

// host inputs for the next round (the engine's rbe_push_* / rbe_notify_applied)
enum HarnessPush { PUSH_PROPOSE = 1, PUSH_READ = 2, PUSH_XFER = 3, PUSH_UNREACH = 4,
                   PUSH_SNAPST = 5, PUSH_APPLIED = 6, PUSH_APPLY_READY = 7,
                   PUSH_CC_PROPOSE = 8,  // a = ConfigChangeType, b = node id (ProposeConfigChange)
                   PUSH_CC_APPLY = 9,    // a = node id (0 = NoNode), b = type (ApplyConfigChange)
                   PUSH_CC_REJECT = 10,  // RejectConfigChange
                   PUSH_RESTORE = 11 };  // a = removed mask (RestoreRemotes with that membership)

struct ReplicaView {  // mirrors rbe_replica_view in include/rbe.h
  u64 term, vote, leader_id, committed, last_index, processed, saved_to, digest;
  u32 role, election_tick, heartbeat_tick, rand_election_timeout;
  u32 q_tick, q_quiesced_since, q_no_activity_since, q_exit_quiesce_tick;
  u32 raft_quiesce, rq_count, votes_resp, votes_granted;
  u64 match[8], next[8];
  u32 rstate[8], ractive[8];
  u32 events;   // EV_* bits of the last round's step (rbe_types.h)
  u32 removed;  // bit (id-1): not in this replica's raft.remotes
  u32 observers, witnesses;  // bit (id-1): raft.observers / raft.witnesses
};

// ------------------------------------------------------------ quiesce.go
// (node-side; also unit-tested against quiesce_test.go through orc_quiesce_*)
struct QuiesceManager {  // quiesce.go:23-33
  u64 tick = 0, electionTick = 0, quiescedSince = 0, noActivitySince = 0,
      exitQuiesceTick = 0;
  bool enabled = false;
  bool newFlag = false;

  bool newQuiesceState() {  // quiesce.go:39-41
    bool v = newFlag;
    newFlag = false;
    return v;
  }
  u64 threshold() const { return electionTick * 10; }  // quiesce.go:84-86
  bool quiesced() const { return enabled && quiescedSince > 0; }  // quiesce.go:57-62
  bool newToQuiesce() const {  // quiesce.go:88-93
    if (!quiesced()) return false;
    return tick - quiescedSince < electionTick;
  }
  bool justExitedQuiesce() const {  // quiesce.go:95-100
    if (quiesced()) return false;
    return tick - exitQuiesceTick < threshold();
  }
  void enterQuiesce() {  // quiesce.go:112-117
    quiescedSince = tick;
    noActivitySince = tick;
    newFlag = true;
  }
  void exitQuiesce() {  // quiesce.go:119-122
    quiescedSince = 0;
    exitQuiesceTick = tick;
  }
  u64 increaseQuiesceTick() {  // quiesce.go:43-55
    if (!enabled) return 0;
    u64 th = threshold();
    tick++;
    if (!quiesced()) {
      if (tick - noActivitySince > th) enterQuiesce();
    }
    return tick;
  }
  void recordActivity(int t) {  // quiesce.go:64-82
    if (!enabled) return;
    if (t == Heartbeat || t == HeartbeatResp) {
      if (!quiesced()) return;
      if (newToQuiesce()) return;
    }
    noActivitySince = tick;
    if (quiesced()) exitQuiesce();
  }
  void tryEnterQuiesce() {  // quiesce.go:102-110
    if (justExitedQuiesce()) return;
    if (!quiesced()) enterQuiesce();
  }
};

struct Harness;
Harness* harness_create(const HarnessConfig& cfg);
void harness_destroy(Harness* h);
void harness_run(Harness* h, u32 rounds);
// one round; tick = false steps without the tick (rbe_step_ex RBE_STEP_NO_TICK)
void harness_step(Harness* h, bool tick);
// stage host input for replica g*n+k for the next round; returns 0
int harness_push(Harness* h, int kind, u64 replica, u64 a, u64 b, const Entry* ents, u32 n);
u32 harness_round(const Harness* h);
int harness_snapshot_saved(Harness* h, u64 replica, u64 index, u64 term, u32 removed);
int harness_compact(Harness* h, u64 replica, u64 to);
void harness_views(const Harness* h, ReplicaView* out);  // n_groups*n_replicas views
// Peer.RateLimited and rl.Get() of every replica (n_groups*n_replicas each)
void harness_rate_limited(Harness* h, uint8_t* limited, u64* size);
void harness_counters(const Harness* h, u64* out);       // HC_NUM counters
u64 harness_log_term(const Harness* h, u64 g, u32 k, u64 index);  // term of entry (0 if absent)
// restart of one replica from its LogDB (Peer.Launch over an existing log; the
// engine's rbe_launch): persisted state, persisted entries, the restart itself
void harness_persisted(const Harness* h, u64 replica, u64 out4[4]);  // term, vote, commit, last
int harness_persisted_entries(const Harness* h, u64 replica, u64 lo, u64 hi, Entry* out);
// LogDB marker, marker term, snapshot index, snapshot term; node reqSnapshotIndex, compactLogTo
void harness_snapshot_state(const Harness* h, u64 replica, u64 out8[8]);
void harness_restart(Harness* h, u64 replica);
// ext_commit: the UpdateCommit of the replica's last step (zero when it made no
// Update; getUpdateCommit, peer.go:410-427), and Peer.Commit's log part with a
// host-chosen UpdateCommit (entryLog.commitUpdate, logentry.go:335-355)
void harness_update_commit(const Harness* h, u64 replica, UpdateCommit* out);
// a fresh node joins in the replica's slot (rbe_replace_node); -1 while the
// group still refers to the slot's node
int harness_replace(Harness* h, u64 replica);
// the Snapshot of the replica's last Update: index, term, packed membership, 0
void harness_update_snapshot(const Harness* h, u64 replica, u64 out4[4]);
void harness_commit(Harness* h, u64 replica, const UpdateCommit& uc);
// debugging: the messages replica `replica` receives from slot `sender` next
// round (delivered by the last round), as 10 words each: type, from, to, term,
// log_term, log_index, commit, reject, hint, number of entries; returns the count
u32 harness_inbox(const Harness* h, u64 replica, u32 sender, u64* out, u32 cap);

// shared helpers (restated independently in the engine)
u64 wl_payload_lo(u64 seed, u64 cid, u64 round);
bool wl_group_active(const HarnessConfig& c, u64 cid);
int wl_input(const HarnessConfig& c, u64 cid, u32 round);  // 0 none, 1 propose, 2 read
bool iso_selected(const HarnessConfig& c, u64 cid, u32 epoch);
u64 xfer_input(const HarnessConfig& c, u64 cid, u32 round, u32 k);  // 0 = none
bool cc_selected(const HarnessConfig& c, u64 cid, u32 round);       // a cc_period round for cid
u64 cc_target(const HarnessConfig& c, u64 cid, u32 round);          // its seeded node id
// the stand-in ConfigChange Cmd the harness and the engine share: 8 bytes, LE
// of 0xCC << 56 | type << 48 | node id (bootstrap's entries are type AddNode)
std::string cc_cmd(int type, u64 node_id);
bool cc_decode(const std::string& cmd, int* type, u64* node_id);
inline u64 hfold(u64 h, u64 x) { return splitmix64(h ^ x); }

}  // namespace orc
