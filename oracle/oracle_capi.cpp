// ORACLE — TEST INFRASTRUCTURE ONLY (see raft_ref.h header comment).
// extern "C" surface of the oracle for the Python tests (ctypes).  It exposes
// the restated raft at unit level (the access the reference's own *_test.go
// files have to raft/remote/entryLog/readIndex/Peer) and the lockstep harness.
#include <cstring>
#include <string>

#include "harness.h"
#include "raft_ref.h"

using namespace orc;

extern "C" {

typedef struct {
  uint64_t term, index, key, client_id, series_id, responded_to;
  uint32_t type, cmd_len;
  uint8_t cmd[64];
  const uint8_t* data;  // the whole Cmd when cmd_len > 64 (input only)
} orc_entry;

typedef struct {
  uint64_t index, term;
  uint32_t n_addr, n_obs, n_wit, flags;  // flags: 1 dummy, 2 witness
  uint64_t addr[8], obs[8], wit[8];
} orc_snapshot;

typedef struct {
  uint32_t type, reject;
  uint64_t to, from, cluster_id, term, log_term, log_index, commit, hint, hint_high;
  uint32_t n_entries, pad;
  orc_entry* entries;
  orc_snapshot snapshot;
} orc_msg;

typedef struct {
  uint64_t node_id, cluster_id, election, heartbeat, seed, max_entry_size;
  uint32_t check_quorum, is_observer, is_witness, quiesce;
} orc_config;

typedef struct {
  uint64_t n_groups;
  uint32_t n_replicas, check_quorum;
  uint64_t cid_base, election_rtt, heartbeat_rtt, seed, max_entry_size;
  uint32_t quiesce, wl_enabled, wl_start_round, wl_stop_round;
  uint32_t wl_active_mod, wl_read_permille, iso_period, iso_len;
  uint32_t iso_mod, trace, threads, pad;
  uint64_t cid_stride;
  uint32_t xfer_period, xfer_mod, ext_apply, snapshot_entries;
  uint32_t compaction_overhead, ext_commit;
  uint32_t membership, cc_period, cc_mod, n_voters;
  uint64_t max_inmem_log_size;
  uint32_t observer_slots, witness_slots;
} orc_harness_config;

static thread_local std::string g_err;
const char* orc_last_error() { return g_err.c_str(); }

#define GUARD_BEGIN try {
#define GUARD_END(errval)            \
  }                                  \
  catch (const std::exception& e) {  \
    g_err = e.what();                \
    return errval;                   \
  }

static Entry to_entry(const orc_entry& e) {
  Entry x;
  x.term = e.term;
  x.index = e.index;
  x.type = (int)e.type;
  x.key = e.key;
  x.client_id = e.client_id;
  x.series_id = e.series_id;
  x.responded_to = e.responded_to;
  if (e.cmd_len > 64 && e.data)
    x.cmd.assign((const char*)e.data, e.cmd_len);
  else
    x.cmd.assign((const char*)e.cmd, e.cmd_len > 64 ? 64 : e.cmd_len);
  return x;
}

static void from_entry(const Entry& x, orc_entry* e) {
  memset(e, 0, sizeof(*e));
  e->term = x.term;
  e->index = x.index;
  e->type = (uint32_t)x.type;
  e->key = x.key;
  e->client_id = x.client_id;
  e->series_id = x.series_id;
  e->responded_to = x.responded_to;
  e->cmd_len = (uint32_t)(x.cmd.size() > 64 ? 64 : x.cmd.size());
  memcpy(e->cmd, x.cmd.data(), e->cmd_len);
}

static Snapshot to_snapshot(const orc_snapshot& s) {
  Snapshot ss;
  ss.index = s.index;
  ss.term = s.term;
  for (uint32_t i = 0; i < s.n_addr && i < 8; i++) ss.membership.addresses[s.addr[i]] = "a";
  for (uint32_t i = 0; i < s.n_obs && i < 8; i++) ss.membership.observers[s.obs[i]] = "o";
  for (uint32_t i = 0; i < s.n_wit && i < 8; i++) ss.membership.witnesses[s.wit[i]] = "w";
  ss.dummy = (s.flags & 1) != 0;
  ss.witness = (s.flags & 2) != 0;
  return ss;
}

static void from_snapshot(const Snapshot& ss, orc_snapshot* s) {
  memset(s, 0, sizeof(*s));
  s->index = ss.index;
  s->term = ss.term;
  for (auto& kv : ss.membership.addresses) if (s->n_addr < 8) s->addr[s->n_addr++] = kv.first;
  for (auto& kv : ss.membership.observers) if (s->n_obs < 8) s->obs[s->n_obs++] = kv.first;
  for (auto& kv : ss.membership.witnesses) if (s->n_wit < 8) s->wit[s->n_wit++] = kv.first;
  s->flags = (ss.dummy ? 1 : 0) | (ss.witness ? 2 : 0);
}

static Message to_msg(const orc_msg* m) {
  Message x;
  x.type = (int)m->type;
  x.reject = m->reject != 0;
  x.to = m->to;
  x.from = m->from;
  x.cluster_id = m->cluster_id;
  x.term = m->term;
  x.log_term = m->log_term;
  x.log_index = m->log_index;
  x.commit = m->commit;
  x.hint = m->hint;
  x.hint_high = m->hint_high;
  for (uint32_t i = 0; i < m->n_entries; i++) x.entries.push_back(to_entry(m->entries[i]));
  x.snapshot = to_snapshot(m->snapshot);
  return x;
}

static int from_msgs(const std::vector<Message>& msgs, orc_msg* out, int cap, orc_entry* ebuf,
                     int ecap) {
  int n = 0, ne = 0;
  for (auto& x : msgs) {
    if (n >= cap) break;
    orc_msg* m = &out[n++];
    memset(m, 0, sizeof(*m));
    m->type = (uint32_t)x.type;
    m->reject = x.reject ? 1 : 0;
    m->to = x.to;
    m->from = x.from;
    m->cluster_id = x.cluster_id;
    m->term = x.term;
    m->log_term = x.log_term;
    m->log_index = x.log_index;
    m->commit = x.commit;
    m->hint = x.hint;
    m->hint_high = x.hint_high;
    m->n_entries = (uint32_t)x.entries.size();
    m->entries = ebuf ? ebuf + ne : nullptr;
    for (auto& e : x.entries) {
      if (ne < ecap && ebuf) from_entry(e, &ebuf[ne]);
      ne++;
    }
    from_snapshot(x.snapshot, &m->snapshot);
  }
  return n;
}

// ------------------------------------------------------------------ LogDB
void* orc_logdb_new() { return new TestLogDB(); }
void orc_logdb_free(void* db) { delete (TestLogDB*)db; }
int orc_logdb_append(void* db, const orc_entry* e, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(e[i]));
  return (int)((TestLogDB*)db)->Append(v);
  GUARD_END(-1)
}
void orc_logdb_set_state(void* db, uint64_t term, uint64_t vote, uint64_t commit) {
  ((TestLogDB*)db)->SetState(PState{term, vote, commit});
}
int orc_logdb_apply_snapshot(void* db, const orc_snapshot* s) {
  return (int)((TestLogDB*)db)->ApplySnapshot(to_snapshot(*s));
}
int orc_logdb_create_snapshot(void* db, const orc_snapshot* s) {
  return (int)((TestLogDB*)db)->CreateSnapshot(to_snapshot(*s));
}
int orc_logdb_compact(void* db, uint64_t index) { return (int)((TestLogDB*)db)->Compact(index); }
int orc_logdb_term(void* db, uint64_t index, uint64_t* t) { return (int)((TestLogDB*)db)->Term(index, t); }
void orc_logdb_range(void* db, uint64_t* first, uint64_t* last) {
  auto r = ((TestLogDB*)db)->GetRange();
  *first = r.first;
  *last = r.second;
}
int orc_logdb_entries(void* db, uint64_t lo, uint64_t hi, uint64_t max, orc_entry* out, int cap) {
  GUARD_BEGIN
  std::vector<Entry> v;
  Err e = ((TestLogDB*)db)->Entries(lo, hi, max, &v);
  if (e != ErrOK) return -(int)e;
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
  GUARD_END(-100)
}

// ------------------------------------------------------------------ Raft
static Config to_config(const orc_config* c) {
  Config x;
  x.nodeID = c->node_id;
  x.clusterID = c->cluster_id;
  x.electionRTT = c->election;
  x.heartbeatRTT = c->heartbeat;
  x.checkQuorum = c->check_quorum != 0;
  x.isObserver = c->is_observer != 0;
  x.isWitness = c->is_witness != 0;
  x.quiesce = c->quiesce != 0;
  x.rngSeed = c->seed;
  x.maxEntrySize = c->max_entry_size ? c->max_entry_size : DefaultMaxEntrySize;
  return x;
}

void* orc_raft_new(const orc_config* c, void* db) {
  GUARD_BEGIN
  return new Raft(to_config(c), (TestLogDB*)db);
  GUARD_END(nullptr)
}
void orc_raft_free(void* r) { delete (Raft*)r; }

int orc_raft_handle(void* r, const orc_msg* m) {
  GUARD_BEGIN
  ((Raft*)r)->Handle(to_msg(m));
  return 0;
  GUARD_END(-1)
}

// Direct handler entry for tests that bypass Handle's term gate, as the
// reference's tests do (e.g. raft_etcd_test.go:1260 sm.handleReplicateMessage).
int orc_raft_handle_direct(void* r, int which, const orc_msg* m) {
  GUARD_BEGIN
  Raft* x = (Raft*)r;
  Message msg = to_msg(m);
  switch (which) {
    case 0: x->handleReplicateMessage(msg); return 0;
    case 1: x->handleHeartbeatMessage(msg); return 0;
    case 2: x->handleNodeRequestVote(msg); return 0;
    default: g_err = "bad handler"; return -1;
  }
  GUARD_END(-1)
}

int orc_raft_num_messages(void* r) { return (int)((Raft*)r)->msgs.size(); }
int orc_raft_num_message_entries(void* r) {
  int n = 0;
  for (auto& m : ((Raft*)r)->msgs) n += (int)m.entries.size();
  return n;
}
int orc_raft_read_messages(void* r, orc_msg* out, int cap, orc_entry* ebuf, int ecap) {
  auto msgs = ((Raft*)r)->readMessages();
  return from_msgs(msgs, out, cap, ebuf, ecap);
}
// peek without consuming
int orc_raft_peek_messages(void* r, orc_msg* out, int cap, orc_entry* ebuf, int ecap) {
  return from_msgs(((Raft*)r)->msgs, out, cap, ebuf, ecap);
}

enum RaftField {
  F_TERM = 0, F_VOTE, F_STATE, F_LEADER, F_COMMITTED, F_PROCESSED, F_APPLIED, F_LAST_INDEX,
  F_FIRST_INDEX, F_ELECTION_TICK, F_HEARTBEAT_TICK, F_RAND_ET, F_ELECTION_TIMEOUT,
  F_HEARTBEAT_TIMEOUT, F_CHECK_QUORUM, F_QUIESCE, F_LTT, F_IS_LTT, F_PENDING_CC, F_NODE_ID,
  F_TICK_COUNT, F_NUM_VOTING, F_QUORUM, F_RTR_COUNT, F_DROPPED_ENTRIES, F_DROPPED_RI, F_RQ_LEN,
  F_LAST_TERM, F_TEST_CC_MODE, F_SAVED_TO, F_MARKER_INDEX, F_INMEM_LEN, F_CLUSTER_ID,
  F_NUM_REMOTES, F_NUM_OBSERVERS, F_NUM_WITNESSES, F_SHRUNK, F_HAS_INMEM_SNAPSHOT,
  F_RNG_COUNT, F_VOTES_LEN, F_MATCHED_LEN
};

uint64_t orc_raft_get(void* rp, int f) {
  Raft* r = (Raft*)rp;
  switch (f) {
    case F_TERM: return r->term;
    case F_VOTE: return r->vote;
    case F_STATE: return (uint64_t)r->state;
    case F_LEADER: return r->leaderID;
    case F_COMMITTED: return r->log.committed;
    case F_PROCESSED: return r->log.processed;
    case F_APPLIED: return r->applied;
    case F_LAST_INDEX: return r->log.lastIndex();
    case F_FIRST_INDEX: return r->log.firstIndex();
    case F_ELECTION_TICK: return r->electionTick;
    case F_HEARTBEAT_TICK: return r->heartbeatTick;
    case F_RAND_ET: return r->randomizedElectionTimeout;
    case F_ELECTION_TIMEOUT: return r->electionTimeout;
    case F_HEARTBEAT_TIMEOUT: return r->heartbeatTimeout;
    case F_CHECK_QUORUM: return r->checkQuorum;
    case F_QUIESCE: return r->quiesce;
    case F_LTT: return r->leaderTransferTarget;
    case F_IS_LTT: return r->isLeaderTransferTarget;
    case F_PENDING_CC: return r->pendingConfigChange;
    case F_NODE_ID: return r->nodeID;
    case F_TICK_COUNT: return r->tickCount;
    case F_NUM_VOTING: return r->numVotingMembers();
    case F_QUORUM: return (uint64_t)r->quorum();
    case F_RTR_COUNT: return r->readyToRead.size();
    case F_DROPPED_ENTRIES: return r->droppedEntries.size();
    case F_DROPPED_RI: return r->droppedReadIndexes.size();
    case F_RQ_LEN: return r->readIndex.queue.size();
    case F_LAST_TERM: return r->log.lastTerm();
    case F_TEST_CC_MODE: return r->testOnlyCCMode;
    case F_SAVED_TO: return r->log.inmem.savedTo;
    case F_MARKER_INDEX: return r->log.inmem.markerIndex;
    case F_INMEM_LEN: return r->log.inmem.entries.size();
    case F_CLUSTER_ID: return r->clusterID;
    case F_NUM_REMOTES: return r->remotes.size();
    case F_NUM_OBSERVERS: return r->observers.size();
    case F_NUM_WITNESSES: return r->witnesses.size();
    case F_SHRUNK: return r->log.inmem.shrunk;
    case F_HAS_INMEM_SNAPSHOT: return r->log.inmem.hasSnapshot;
    case F_RNG_COUNT: return r->rngCount;
    case F_VOTES_LEN: return r->votes.size();
    case F_MATCHED_LEN: return r->matched.size();
    default: return ~0ULL;
  }
}

int orc_raft_set(void* rp, int f, uint64_t v) {
  Raft* r = (Raft*)rp;
  switch (f) {
    case F_TERM: r->term = v; return 0;
    case F_VOTE: r->vote = v; return 0;
    case F_STATE: r->state = (int)v; return 0;
    case F_LEADER: r->leaderID = v; return 0;
    case F_COMMITTED: r->log.committed = v; return 0;
    case F_PROCESSED: r->log.processed = v; return 0;
    case F_APPLIED: r->applied = v; return 0;
    case F_ELECTION_TICK: r->electionTick = v; return 0;
    case F_HEARTBEAT_TICK: r->heartbeatTick = v; return 0;
    case F_RAND_ET: r->randomizedElectionTimeout = v; return 0;
    case F_CHECK_QUORUM: r->checkQuorum = v != 0; return 0;
    case F_QUIESCE: r->quiesce = v != 0; return 0;
    case F_LTT: r->leaderTransferTarget = v; return 0;
    case F_IS_LTT: r->isLeaderTransferTarget = v != 0; return 0;
    case F_PENDING_CC: r->pendingConfigChange = v != 0; return 0;
    case F_TEST_CC_MODE: r->testOnlyCCMode = v != 0; return 0;
    case F_SAVED_TO: r->log.inmem.savedTo = v; return 0;
    case F_MARKER_INDEX: r->log.inmem.markerIndex = v; return 0;
    case F_SHRUNK: r->log.inmem.shrunk = v != 0; return 0;
    default: return -1;
  }
}

enum RaftCall {
  C_BECOME_FOLLOWER = 0, C_BECOME_CANDIDATE, C_BECOME_LEADER, C_TICK, C_QUIESCED_TICK,
  C_RESET, C_CAMPAIGN, C_TRY_COMMIT, C_ADD_NODE, C_REMOVE_NODE, C_ADD_OBSERVER, C_ADD_WITNESS,
  C_BROADCAST_REPLICATE, C_BROADCAST_HEARTBEAT, C_SEND_REPLICATE, C_HAS_CC_TO_APPLY,
  C_LEADER_HAS_QUORUM, C_LOG_COMMIT_TO, C_LOG_MATCH_TERM, C_LOG_UP_TO_DATE, C_LOG_TRY_COMMIT,
  C_SELF_REMOVED, C_BECOME_OBSERVER, C_BECOME_WITNESS, C_SET_APPLIED_LOG_TO,
  C_HAS_COMMITTED_AT_TERM, C_PENDING_CC_COUNT, C_RESET_MATCH_ARRAY, C_SORT_MATCH_CHECK,
  C_HANDLE_VOTE_RESP, C_CAN_GRANT_VOTE, C_INMEM_TRY_RESIZE, C_INMEM_RESIZE,
  C_LOG_HAS_ENTRIES_TO_APPLY, C_LOG_FIRST_NOT_APPLIED, C_LOG_SAVED_LOG_TO, C_TIME_FOR_ELECTION,
  C_SET_RANDOMIZED_ET, C_ABORT_LT, C_LEADER_TRANSFERING, C_QUIESCED_TICK_DIRECT,
  C_NON_LEADER_TICK, C_LEADER_TICK, C_LOAD_STATE,
  // rate limiter (server/rate.go, raft.go:660-683, 1779-1785)
  C_RL_SET_MAX, C_RL_GET, C_RL_TICK, C_RL_RATE_LIMITED, C_RL_ENABLED, C_RL_INCREASE,
  C_RL_DECREASE, C_RL_SET, C_RL_SET_FOLLOWER, C_RL_FOLLOWER_COUNT, C_RL_FOLLOWER_SIZE,
  C_RL_FOLLOWER_TICK, C_RL_HEARTBEAT_TICK, C_RL_GC, C_RL_RESET_FOLLOWERS,
  C_RL_HANDLE_LEADER_RATE_LIMIT, C_RL_APPEND_ENTRIES
};

int64_t orc_raft_call(void* rp, int fn, uint64_t a, uint64_t b) {
  Raft* r = (Raft*)rp;
  GUARD_BEGIN
  switch (fn) {
    case C_BECOME_FOLLOWER: r->becomeFollower(a, b); return 0;
    case C_BECOME_CANDIDATE: r->becomeCandidate(); return 0;
    case C_BECOME_LEADER: r->becomeLeader(); return 0;
    case C_TICK: r->tick(); return 0;
    case C_QUIESCED_TICK: r->quiescedTick(); return 0;
    case C_RESET: r->reset(a); return 0;
    case C_CAMPAIGN: r->campaign(); return 0;
    case C_TRY_COMMIT: return r->tryCommit() ? 1 : 0;
    case C_ADD_NODE: r->addNode(a); return 0;
    case C_REMOVE_NODE: r->removeNode(a); return 0;
    case C_ADD_OBSERVER: r->addObserver(a); return 0;
    case C_ADD_WITNESS: r->addWitness(a); return 0;
    case C_BROADCAST_REPLICATE: r->broadcastReplicateMessage(); return 0;
    case C_BROADCAST_HEARTBEAT: r->broadcastHeartbeatMessage(); return 0;
    case C_SEND_REPLICATE: r->sendReplicateMessage(a); return 0;
    case C_HAS_CC_TO_APPLY: return r->hasConfigChangeToApply() ? 1 : 0;
    case C_LEADER_HAS_QUORUM: return r->leaderHasQuorum() ? 1 : 0;
    case C_LOG_COMMIT_TO: r->log.commitTo(a); return 0;
    case C_LOG_MATCH_TERM: return r->log.matchTerm(a, b) ? 1 : 0;
    case C_LOG_UP_TO_DATE: return r->log.upToDate(a, b) ? 1 : 0;
    case C_LOG_TRY_COMMIT: return r->log.tryCommit(a, b) ? 1 : 0;
    case C_SELF_REMOVED: return r->selfRemoved() ? 1 : 0;
    case C_BECOME_OBSERVER: r->state = Observer; r->becomeObserver(a, b); return 0;
    case C_BECOME_WITNESS: r->state = Witness; r->becomeWitness(a, b); return 0;
    case C_SET_APPLIED_LOG_TO: r->log.inmem.appliedLogTo(a); return 0;
    case C_HAS_COMMITTED_AT_TERM: return r->hasCommittedEntryAtCurrentTerm() ? 1 : 0;
    case C_PENDING_CC_COUNT: return r->getPendingConfigChangeCount();
    case C_RESET_MATCH_ARRAY: r->resetMatchValueArray(); return 0;
    case C_SORT_MATCH_CHECK: r->sortMatchValues(); return 0;
    case C_HANDLE_VOTE_RESP: return r->handleVoteResp(a, b != 0);
    case C_CAN_GRANT_VOTE: { Message m; m.from = a; m.term = b; return r->canGrantVote(m) ? 1 : 0; }
    case C_INMEM_TRY_RESIZE: r->log.inmem.tryResize(); return 0;
    case C_INMEM_RESIZE: r->log.inmem.resize(); return 0;
    case C_LOG_HAS_ENTRIES_TO_APPLY: return r->log.hasEntriesToApply() ? 1 : 0;
    case C_LOG_FIRST_NOT_APPLIED: return (int64_t)r->log.firstNotAppliedIndex();
    case C_LOG_SAVED_LOG_TO: r->log.inmem.savedLogTo(a, b); return 0;
    case C_TIME_FOR_ELECTION: return r->timeForElection() ? 1 : 0;
    case C_SET_RANDOMIZED_ET: r->setRandomizedElectionTimeout(); return 0;
    case C_ABORT_LT: r->abortLeaderTransfer(); return 0;
    case C_LEADER_TRANSFERING: return r->leaderTransfering() ? 1 : 0;
    case C_QUIESCED_TICK_DIRECT: r->quiescedTick(); return 0;
    case C_NON_LEADER_TICK: r->nonLeaderTick(); return 0;
    case C_LEADER_TICK: r->leaderTick(); return 0;
    case C_LOAD_STATE: { PState st; st.term = a; st.commit = b; r->loadState(st); return 0; }
    case C_RL_SET_MAX: r->rl.maxSize = a; return 0;  // newRateLimitedTestRaft
    case C_RL_GET: return (int64_t)r->rl.get();
    case C_RL_TICK: return (int64_t)r->rl.tick;
    case C_RL_RATE_LIMITED: return r->rl.rateLimited() ? 1 : 0;
    case C_RL_ENABLED: return r->rl.enabled() ? 1 : 0;
    case C_RL_INCREASE: r->rl.increase(a); return 0;
    case C_RL_DECREASE: r->rl.decrease(a); return 0;
    case C_RL_SET: r->rl.set(a); return 0;
    case C_RL_SET_FOLLOWER: r->rl.setFollowerState(a, b); return 0;
    case C_RL_FOLLOWER_COUNT: return (int64_t)r->rl.followerSizes.size();
    case C_RL_FOLLOWER_SIZE: {
      auto it = r->rl.followerSizes.find(a);
      return it == r->rl.followerSizes.end() ? -1 : (int64_t)it->second.second;
    }
    case C_RL_FOLLOWER_TICK: {
      auto it = r->rl.followerSizes.find(a);
      return it == r->rl.followerSizes.end() ? -1 : (int64_t)it->second.first;
    }
    case C_RL_HEARTBEAT_TICK: r->rl.heartbeatTick(); return 0;
    case C_RL_GC: r->rl.gc(); return 0;
    case C_RL_RESET_FOLLOWERS: r->rl.resetFollowerState(); return 0;
    case C_RL_HANDLE_LEADER_RATE_LIMIT: {
      Message m;
      m.type = RateLimit;
      m.from = a;
      m.hint = b;
      r->handleLeaderRateLimit(m);
      return 0;
    }
    case C_RL_APPEND_ENTRIES: {  // appendEntries of one ApplicationEntry with a b-byte Cmd
      std::vector<Entry> ents(1);
      ents[0].type = ApplicationEntry;
      ents[0].cmd.assign((size_t)b, '\0');
      r->appendEntries(ents);
      return 0;
    }
    default: g_err = "bad call"; return -1000;
  }
  GUARD_END(-999)
}

// A free-standing remote (remote.go:62-69) for the remote_test.go tables.
// st = {match, next, snapshotIndex, state, active}; returns the op's bool
// result (0/1), 0 for void ops, -999 when the reference would panic.
enum { RO_BECOME_RETRY = 0, RO_RETRY_TO_WAIT, RO_WAIT_TO_RETRY, RO_BECOME_WAIT,
       RO_BECOME_REPLICATE, RO_BECOME_SNAPSHOT, RO_TRY_UPDATE, RO_PROGRESS, RO_RESPONDED_TO,
       RO_DECREASE_TO, RO_IS_PAUSED, RO_CLEAR_PENDING_SNAPSHOT, RO_SET_ACTIVE,
       RO_SET_NOT_ACTIVE, RO_IS_ACTIVE };
int64_t orc_remote_op(uint64_t* st, int op, uint64_t a, uint64_t b) {
  GUARD_BEGIN
  Remote x;
  x.match = st[0];
  x.next = st[1];
  x.snapshotIndex = st[2];
  x.state = (int)st[3];
  x.active = st[4] != 0;
  int64_t ret = 0;
  switch (op) {
    case RO_BECOME_RETRY: x.becomeRetry(); break;
    case RO_RETRY_TO_WAIT: x.retryToWait(); break;
    case RO_WAIT_TO_RETRY: x.waitToRetry(); break;
    case RO_BECOME_WAIT: x.becomeWait(); break;
    case RO_BECOME_REPLICATE: x.becomeReplicate(); break;
    case RO_BECOME_SNAPSHOT: x.becomeSnapshot(a); break;
    case RO_TRY_UPDATE: ret = x.tryUpdate(a) ? 1 : 0; break;
    case RO_PROGRESS: x.progress(a); break;
    case RO_RESPONDED_TO: x.respondedTo(); break;
    case RO_DECREASE_TO: ret = x.decreaseTo(a, b) ? 1 : 0; break;
    case RO_IS_PAUSED: ret = x.isPaused() ? 1 : 0; break;
    case RO_CLEAR_PENDING_SNAPSHOT: x.clearPendingSnapshot(); break;
    case RO_SET_ACTIVE: x.setActive(); break;
    case RO_SET_NOT_ACTIVE: x.setNotActive(); break;
    case RO_IS_ACTIVE: ret = x.isActive() ? 1 : 0; break;
    default: g_err = "unknown remote op"; return -999;
  }
  st[0] = x.match;
  st[1] = x.next;
  st[2] = x.snapshotIndex;
  st[3] = (uint64_t)x.state;
  st[4] = x.active ? 1 : 0;
  return ret;
  GUARD_END(-999)
}

// remotes: kind 0 remotes, 1 observers, 2 witnesses
static std::map<u64, Remote>& remote_map(Raft* r, int kind) {
  return kind == 0 ? r->remotes : (kind == 1 ? r->observers : r->witnesses);
}
int orc_raft_remote_get(void* rp, int kind, uint64_t id, uint64_t* out5) {
  auto& m = remote_map((Raft*)rp, kind);
  auto it = m.find(id);
  if (it == m.end()) return 0;
  out5[0] = it->second.match;
  out5[1] = it->second.next;
  out5[2] = it->second.snapshotIndex;
  out5[3] = (uint64_t)it->second.state;
  out5[4] = it->second.active ? 1 : 0;
  return 1;
}
void orc_raft_remote_set(void* rp, int kind, uint64_t id, uint64_t match, uint64_t next,
                         uint64_t snapshotIndex, uint64_t state, uint64_t active) {
  auto& m = remote_map((Raft*)rp, kind);
  Remote& x = m[id];
  x.match = match;
  x.next = next;
  x.snapshotIndex = snapshotIndex;
  x.state = (int)state;
  x.active = active != 0;
}
void orc_raft_remote_del(void* rp, int kind, uint64_t id) { remote_map((Raft*)rp, kind).erase(id); }
void orc_raft_remote_clear(void* rp, int kind) { remote_map((Raft*)rp, kind).clear(); }
int orc_raft_remote_ids(void* rp, int kind, uint64_t* out, int cap) {
  int n = 0;
  for (auto& kv : remote_map((Raft*)rp, kind)) if (n < cap) out[n++] = kv.first;
  return n;
}
int orc_raft_votes(void* rp, uint64_t* ids, uint8_t* granted, int cap) {
  int n = 0;
  for (auto& kv : ((Raft*)rp)->votes) {
    if (n < cap) {
      ids[n] = kv.first;
      granted[n] = kv.second ? 1 : 0;
    }
    n++;
  }
  return n;
}
int orc_raft_ready_to_read(void* rp, uint64_t* out3, int cap) {
  int n = 0;
  for (auto& x : ((Raft*)rp)->readyToRead) {
    if (n < cap) {
      out3[3 * n] = x.index;
      out3[3 * n + 1] = x.ctx.low;
      out3[3 * n + 2] = x.ctx.high;
    }
    n++;
  }
  return n;
}
void orc_raft_clear_ready_to_read(void* rp) { ((Raft*)rp)->readyToRead.clear(); }
int orc_raft_dropped_ri(void* rp, uint64_t* out2, int cap) {
  int n = 0;
  for (auto& x : ((Raft*)rp)->droppedReadIndexes) {
    if (n < cap) {
      out2[2 * n] = x.low;
      out2[2 * n + 1] = x.high;
    }
    n++;
  }
  return n;
}
int orc_raft_dropped_entries(void* rp, orc_entry* out, int cap) {
  int n = 0;
  for (auto& x : ((Raft*)rp)->droppedEntries) {
    if (n < cap) from_entry(x, &out[n]);
    n++;
  }
  return n;
}
int orc_raft_readindex_queue(void* rp, uint64_t* out, int cap) {
  // per queued ctx: low, high, index, from, n_confirmed
  Raft* r = (Raft*)rp;
  int n = 0;
  for (auto& c : r->readIndex.queue) {
    if (n < cap) {
      auto& s = r->readIndex.pending[c];
      out[5 * n] = c.low;
      out[5 * n + 1] = c.high;
      out[5 * n + 2] = s.index;
      out[5 * n + 3] = s.from;
      out[5 * n + 4] = s.confirmed.size();
    }
    n++;
  }
  return n;
}
int orc_raft_matched(void* rp, uint64_t* out, int cap) {
  Raft* r = (Raft*)rp;
  int n = 0;
  for (u64 v : r->matched) if (n < cap) out[n++] = v;
  return (int)r->matched.size();
}
void orc_raft_set_matched(void* rp, const uint64_t* v, int n) {
  ((Raft*)rp)->matched.assign(v, v + n);
}

int orc_raft_log_term(void* rp, uint64_t idx, uint64_t* t) {
  GUARD_BEGIN
  return (int)((Raft*)rp)->log.term(idx, t);
  GUARD_END(-100)
}
int orc_raft_log_entries(void* rp, uint64_t start, uint64_t maxSize, orc_entry* out, int cap) {
  GUARD_BEGIN
  std::vector<Entry> v;
  Err e = ((Raft*)rp)->log.entries(start, maxSize, &v);
  if (e != ErrOK) return -(int)e;
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
  GUARD_END(-100)
}
int orc_raft_log_get_entries(void* rp, uint64_t lo, uint64_t hi, uint64_t maxSize, orc_entry* out,
                             int cap) {
  GUARD_BEGIN
  std::vector<Entry> v;
  Err e = ((Raft*)rp)->log.getEntries(lo, hi, maxSize, &v);
  if (e != ErrOK) return -(int)e;
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
  GUARD_END(-100)
}
int orc_raft_log_append(void* rp, const orc_entry* e, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(e[i]));
  ((Raft*)rp)->log.append(v);
  return 0;
  GUARD_END(-1)
}
int64_t orc_raft_log_try_append(void* rp, uint64_t index, const orc_entry* e, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(e[i]));
  return ((Raft*)rp)->log.tryAppend(index, v) ? 1 : 0;
  GUARD_END(-1)
}
int64_t orc_raft_log_conflict_index(void* rp, const orc_entry* e, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(e[i]));
  return (int64_t)((Raft*)rp)->log.getConflictIndex(v);
  GUARD_END(-1)
}
int orc_raft_log_entries_to_save(void* rp, orc_entry* out, int cap) {
  auto v = ((Raft*)rp)->log.entriesToSave();
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
}
int orc_raft_log_entries_to_apply(void* rp, orc_entry* out, int cap) {
  GUARD_BEGIN
  auto v = ((Raft*)rp)->log.entriesToApply();
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
  GUARD_END(-1)
}
int orc_raft_log_restore(void* rp, const orc_snapshot* s) {
  GUARD_BEGIN
  ((Raft*)rp)->log.restore(to_snapshot(*s));
  return 0;
  GUARD_END(-1)
}
int orc_raft_restore(void* rp, const orc_snapshot* s) {
  GUARD_BEGIN
  return ((Raft*)rp)->restore(to_snapshot(*s)) ? 1 : 0;
  GUARD_END(-1)
}
int orc_raft_restore_remotes(void* rp, const orc_snapshot* s) {
  GUARD_BEGIN
  ((Raft*)rp)->restoreRemotes(to_snapshot(*s));
  return 0;
  GUARD_END(-1)
}
int orc_raft_read_index_add(void* rp, uint64_t index, uint64_t low, uint64_t high, uint64_t from) {
  GUARD_BEGIN
  ((Raft*)rp)->readIndex.addRequest(index, SystemCtx{low, high}, from);
  return 0;
  GUARD_END(-1)
}
int orc_raft_read_index_confirm(void* rp, uint64_t low, uint64_t high, uint64_t from, int quorum,
                                uint64_t* out4, int cap) {
  GUARD_BEGIN
  auto v = ((Raft*)rp)->readIndex.confirm(SystemCtx{low, high}, from, quorum);
  int n = 0;
  for (auto& s : v) {
    if (n < cap) {
      out4[4 * n] = s.index;
      out4[4 * n + 1] = s.from;
      out4[4 * n + 2] = s.ctx.low;
      out4[4 * n + 3] = s.ctx.high;
    }
    n++;
  }
  return n;
  GUARD_END(-1)
}

// ------------------------------------------------------------------ Peer
struct PeerBox {
  Peer* p = nullptr;
  Update ud;
};
void* orc_peer_launch(const orc_config* c, void* db, const uint64_t* ids, int n, int initial,
                      int newNode) {
  GUARD_BEGIN
  std::vector<std::pair<u64, std::string>> addrs;
  for (int i = 0; i < n; i++) addrs.push_back({ids[i], "addr-" + std::to_string(ids[i])});
  PeerBox* b = new PeerBox();
  b->p = Peer::Launch(to_config(c), (TestLogDB*)db, addrs, initial != 0, newNode != 0);
  return b;
  GUARD_END(nullptr)
}
void orc_peer_free(void* pb) {
  delete ((PeerBox*)pb)->p;
  delete (PeerBox*)pb;
}
void* orc_peer_raft(void* pb) { return ((PeerBox*)pb)->p->raft; }
int orc_peer_tick(void* pb, int quiesced) {
  GUARD_BEGIN
  if (quiesced) ((PeerBox*)pb)->p->QuiescedTick();
  else ((PeerBox*)pb)->p->Tick();
  return 0;
  GUARD_END(-1)
}
int orc_peer_handle(void* pb, const orc_msg* m) {
  GUARD_BEGIN
  ((PeerBox*)pb)->p->Handle(to_msg(m));
  return 0;
  GUARD_END(-1)
}
int orc_peer_propose(void* pb, const orc_entry* e, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(e[i]));
  ((PeerBox*)pb)->p->ProposeEntries(v);
  return 0;
  GUARD_END(-1)
}
int orc_peer_read_index(void* pb, uint64_t low, uint64_t high) {
  GUARD_BEGIN
  ((PeerBox*)pb)->p->ReadIndex(SystemCtx{low, high});
  return 0;
  GUARD_END(-1)
}
int orc_peer_misc(void* pb, int fn, uint64_t a, uint64_t b) {
  Peer* p = ((PeerBox*)pb)->p;
  GUARD_BEGIN
  switch (fn) {
    case 0: p->RequestLeaderTransfer(a); return 0;
    case 1: p->ApplyConfigChange(a, (int)b); return 0;
    case 2: p->RejectConfigChange(); return 0;
    case 3: p->ReportUnreachableNode(a); return 0;
    case 4: p->ReportSnapshotStatus(a, b != 0); return 0;
    case 5: p->NotifyRaftLastApplied(a); return 0;
    case 6: return p->HasEntryToApply() ? 1 : 0;
    case 7: return p->HasUpdate(a != 0) ? 1 : 0;
    default: return -1;
  }
  GUARD_END(-1)
}
int orc_peer_propose_cc(void* pb, uint64_t nodeID, int ccType, uint64_t key) {
  GUARD_BEGIN
  Message m;
  m.type = Propose;
  Entry e;
  e.type = ConfigChangeEntry;
  e.key = key;
  e.cmd = "cc" + std::to_string(nodeID) + ":" + std::to_string(ccType);
  m.entries.push_back(e);
  ((PeerBox*)pb)->p->raft->Handle(m);  // peer.go:126-135
  return 0;
  GUARD_END(-1)
}
int orc_peer_get_update(void* pb, int moreToApply, uint64_t lastApplied, uint64_t* info) {
  PeerBox* b = (PeerBox*)pb;
  GUARD_BEGIN
  b->ud = b->p->GetUpdate(moreToApply != 0, lastApplied);
  const Update& u = b->ud;
  info[0] = u.state.term;
  info[1] = u.state.vote;
  info[2] = u.state.commit;
  info[3] = u.fast_apply;
  info[4] = u.entries_to_save.size();
  info[5] = u.committed_entries.size();
  info[6] = u.more_committed_entries;
  info[7] = u.ready_to_reads.size();
  info[8] = u.messages.size();
  info[9] = u.last_applied;
  info[10] = u.update_commit.processed;
  info[11] = u.update_commit.last_applied;
  info[12] = u.update_commit.stable_log_to;
  info[13] = u.update_commit.stable_log_term;
  info[14] = u.update_commit.stable_snapshot_to;
  info[15] = u.update_commit.ready_to_read;
  info[16] = u.dropped_entries.size();
  info[17] = u.dropped_read_indexes.size();
  info[18] = u.snapshot.index;
  return 0;
  GUARD_END(-1)
}
int orc_peer_update_entries(void* pb, int which, orc_entry* out, int cap) {
  PeerBox* b = (PeerBox*)pb;
  const std::vector<Entry>& v =
      which == 0 ? b->ud.entries_to_save : (which == 1 ? b->ud.committed_entries : b->ud.dropped_entries);
  int n = 0;
  for (auto& x : v) if (n < cap) from_entry(x, &out[n++]);
  return (int)v.size();
}
int orc_peer_update_messages(void* pb, orc_msg* out, int cap, orc_entry* ebuf, int ecap) {
  return from_msgs(((PeerBox*)pb)->ud.messages, out, cap, ebuf, ecap);
}
int orc_peer_update_rtr(void* pb, uint64_t* out3, int cap) {
  int n = 0;
  for (auto& x : ((PeerBox*)pb)->ud.ready_to_reads) {
    if (n < cap) {
      out3[3 * n] = x.index;
      out3[3 * n + 1] = x.ctx.low;
      out3[3 * n + 2] = x.ctx.high;
    }
    n++;
  }
  return n;
}
int orc_peer_commit(void* pb) {
  PeerBox* b = (PeerBox*)pb;
  GUARD_BEGIN
  b->p->Commit(b->ud);
  return 0;
  GUARD_END(-1)
}
// set a field of the last retrieved update (tests that build Updates by hand)
void orc_peer_update_set_commit(void* pb, const uint64_t* uc6) {
  UpdateCommit& u = ((PeerBox*)pb)->ud.update_commit;
  u.processed = uc6[0];
  u.last_applied = uc6[1];
  u.stable_log_to = uc6[2];
  u.stable_log_term = uc6[3];
  u.stable_snapshot_to = uc6[4];
  u.ready_to_read = uc6[5];
}

// ------------------------------------------------------------------ Harness
void* orc_harness_create(const orc_harness_config* c) {
  GUARD_BEGIN
  HarnessConfig h;
  h.n_groups = c->n_groups;
  h.n_replicas = c->n_replicas;
  h.cid_base = c->cid_base;
  h.cid_stride = c->cid_stride ? c->cid_stride : 1;
  h.election_rtt = c->election_rtt;
  h.heartbeat_rtt = c->heartbeat_rtt;
  h.check_quorum = c->check_quorum != 0;
  h.quiesce = c->quiesce != 0;
  h.seed = c->seed;
  h.max_entry_size = c->max_entry_size ? c->max_entry_size : DefaultMaxEntrySize;
  h.wl_enabled = c->wl_enabled;
  h.wl_start_round = c->wl_start_round;
  h.wl_stop_round = c->wl_stop_round;
  h.wl_active_mod = c->wl_active_mod;
  h.wl_read_permille = c->wl_read_permille;
  h.iso_period = c->iso_period;
  h.iso_len = c->iso_len;
  h.iso_mod = c->iso_mod;
  h.trace = c->trace;
  h.threads = c->threads;
  h.xfer_period = c->xfer_period;
  h.xfer_mod = c->xfer_mod ? c->xfer_mod : 1;
  h.ext_apply = c->ext_apply;
  h.snapshot_entries = c->snapshot_entries;
  h.compaction_overhead = c->compaction_overhead;
  h.ext_commit = c->ext_commit;
  h.membership = c->membership;
  h.cc_period = c->cc_period;
  h.cc_mod = c->cc_mod ? c->cc_mod : 1;
  h.n_voters = c->n_voters;
  h.observer_slots = c->observer_slots;
  h.witness_slots = c->witness_slots;
  h.max_inmem_log_size = c->max_inmem_log_size;
  return harness_create(h);
  GUARD_END(nullptr)
}
void orc_harness_destroy(void* h) { harness_destroy((Harness*)h); }
int orc_harness_step(void* h, int tick) {
  GUARD_BEGIN
  harness_step((Harness*)h, tick != 0);
  return 0;
  GUARD_END(-1)
}
int orc_harness_push(void* h, int kind, uint64_t replica, uint64_t a, uint64_t b,
                     const orc_entry* ents, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(ents[i]));
  return harness_push((Harness*)h, kind, replica, a, b, v.data(), (u32)n);
  GUARD_END(-1)
}
int orc_harness_run(void* h, uint32_t rounds) {
  GUARD_BEGIN
  harness_run((Harness*)h, rounds);
  return 0;
  GUARD_END(-1)
}
uint32_t orc_harness_round(void* h) { return harness_round((Harness*)h); }
void orc_harness_views(void* h, void* out) { harness_views((Harness*)h, (ReplicaView*)out); }
void orc_harness_rate_limited(void* h, uint8_t* limited, uint64_t* size) {
  harness_rate_limited((Harness*)h, limited, size);
}
void orc_harness_counters(void* h, uint64_t* out) { harness_counters((Harness*)h, out); }
uint64_t orc_harness_log_term(void* h, uint64_t g, uint32_t k, uint64_t idx) {
  return harness_log_term((Harness*)h, g, k, idx);
}
void orc_harness_persisted(void* h, uint64_t replica, uint64_t* out4) {
  harness_persisted((Harness*)h, replica, out4);
}
void orc_harness_snapshot_state(void* h, uint64_t replica, uint64_t* out8) {
  harness_snapshot_state((Harness*)h, replica, out8);
}
int orc_harness_persisted_entries(void* h, uint64_t replica, uint64_t lo, uint64_t hi,
                                  orc_entry* out) {
  GUARD_BEGIN
  std::vector<Entry> v(hi - lo + 1);
  if (harness_persisted_entries((Harness*)h, replica, lo, hi, v.data())) return -1;
  for (size_t i = 0; i < v.size(); i++) from_entry(v[i], &out[i]);
  return 0;
  GUARD_END(-1)
}
// ext_commit: {processed, last_applied, stable_log_to, stable_log_term,
// stable_snapshot_to, ready_to_read} of the last step / sent by the host
void orc_harness_update_commit(void* h, uint64_t replica, uint64_t* out6) {
  UpdateCommit u;
  harness_update_commit((Harness*)h, replica, &u);
  out6[0] = u.processed;
  out6[1] = u.last_applied;
  out6[2] = u.stable_log_to;
  out6[3] = u.stable_log_term;
  out6[4] = u.stable_snapshot_to;
  out6[5] = u.ready_to_read;
}
int orc_harness_replace(void* h, uint64_t replica) {
  GUARD_BEGIN
  return harness_replace((Harness*)h, replica);
  GUARD_END(-2)
}
void orc_harness_update_snapshot(void* h, uint64_t replica, uint64_t* out4) {
  harness_update_snapshot((Harness*)h, replica, out4);
}
int orc_harness_commit(void* h, uint64_t replica, const uint64_t* uc6) {
  GUARD_BEGIN
  UpdateCommit u;
  u.processed = uc6[0];
  u.last_applied = uc6[1];
  u.stable_log_to = uc6[2];
  u.stable_log_term = uc6[3];
  u.stable_snapshot_to = uc6[4];
  u.ready_to_read = uc6[5];
  harness_commit((Harness*)h, replica, u);
  return 0;
  GUARD_END(-1)
}
uint32_t orc_harness_inbox(void* h, uint64_t replica, uint32_t sender, uint64_t* out,
                           uint32_t cap) {
  return harness_inbox((Harness*)h, replica, sender, out, cap);
}
int orc_harness_snapshot_saved(void* h, uint64_t replica, uint64_t index, uint64_t term,
                               uint32_t removed) {
  GUARD_BEGIN
  return harness_snapshot_saved((Harness*)h, replica, index, term, removed);
  GUARD_END(-1)
}
int orc_harness_compact(void* h, uint64_t replica, uint64_t to) {
  GUARD_BEGIN
  return harness_compact((Harness*)h, replica, to);
  GUARD_END(-1)
}
int orc_harness_restart(void* h, uint64_t replica) {
  GUARD_BEGIN
  harness_restart((Harness*)h, replica);
  return 0;
  GUARD_END(-1)
}
int orc_view_size() { return (int)sizeof(ReplicaView); }
uint64_t orc_splitmix64(uint64_t x) { return splitmix64(x); }

}  // extern "C"

// ---------------------------------------------------------------- quiesce.go
// Unit access to the node-side quiesce manager (quiesce.go:23-123), pinned by
// quiesce_test.go (tests/test_quiesce.py).
extern "C" {
void* orc_quiesce_new(uint64_t election_tick, int enabled) {
  auto* q = new QuiesceManager();
  q->electionTick = election_tick;
  q->enabled = enabled != 0;
  return q;
}
void orc_quiesce_free(void* q) { delete (QuiesceManager*)q; }
// op: 0 increaseQuiesceTick, 1 recordActivity(a), 2 tryEnterQuiesce,
//     3 quiesced, 4 newToQuiesce, 5 quiesceThreshold, 6 tick, 7 noActivitySince,
//     8 quiescedSince, 9 exitQuiesceTick, 10 newQuiesceState, 11 set enabled(a)
uint64_t orc_quiesce_op(void* qp, int op, uint64_t a) {
  auto* q = (QuiesceManager*)qp;
  switch (op) {
    case 0: return q->increaseQuiesceTick();
    case 1: q->recordActivity((int)a); return 0;
    case 2: q->tryEnterQuiesce(); return 0;
    case 3: return q->quiesced() ? 1 : 0;
    case 4: return q->newToQuiesce() ? 1 : 0;
    case 5: return q->threshold();
    case 6: return q->tick;
    case 7: return q->noActivitySince;
    case 8: return q->quiescedSince;
    case 9: return q->exitQuiesceTick;
    case 10: return q->newQuiesceState() ? 1 : 0;
    case 11: q->enabled = a != 0; return 0;
    default: return ~0ull;
  }
}
}

// ---------------------------------------------------------------- inmemory.go
// Unit access to the in-memory entry window (inmemory.go:36-246), pinned by
// inmemory_test.go (tests/test_oracle_inmem.py).
extern "C" {
void* orc_inmem_new(uint64_t marker, const orc_entry* ents, int n, uint64_t saved_to, int shrunk) {
  auto* im = new InMemory();
  im->markerIndex = marker;
  for (int i = 0; i < n; i++) im->entries.push_back(to_entry(ents[i]));
  im->savedTo = saved_to;
  im->shrunk = shrunk != 0;
  return im;
}
void orc_inmem_free(void* h) {
  auto* im = (InMemory*)h;
  delete im->rl;  // unit handles own their limiter (op 11)
  delete im;
}
int orc_inmem_merge(void* h, const orc_entry* ents, int n) {
  GUARD_BEGIN
  std::vector<Entry> v;
  for (int i = 0; i < n; i++) v.push_back(to_entry(ents[i]));
  ((InMemory*)h)->merge(v);
  return 0;
  GUARD_END(-1)
}
// op: 0 savedLogTo(a, b), 1 appliedLogTo(a), 2 getLastIndex (-1 when !ok),
//     3 getTerm(a) (-1 when !ok), 4 markerIndex, 5 savedTo, 6 shrunk, 7 len(entries),
//     8 entries[0].Index (-1 when empty), 9 restore(Snapshot{Index: a, Term: b}), 10 resize,
//     11 attach a RateLimiter of maxSize a (newInMemory(_, server.NewRateLimiter(a))),
//     12 rl.Get(), 13 newEntries
int64_t orc_inmem_op(void* h, int op, uint64_t a, uint64_t b) {
  GUARD_BEGIN
  auto* im = (InMemory*)h;
  u64 v = 0;
  switch (op) {
    case 0: im->savedLogTo(a, b); return 0;
    case 1: im->appliedLogTo(a); return 0;
    case 2: return im->getLastIndex(&v) ? (int64_t)v : -1;
    case 3: return im->getTerm(a, &v) ? (int64_t)v : -1;
    case 4: return (int64_t)im->markerIndex;
    case 5: return (int64_t)im->savedTo;
    case 6: return im->shrunk ? 1 : 0;
    case 7: return (int64_t)im->entries.size();
    case 8: return im->entries.empty() ? -1 : (int64_t)im->entries[0].index;
    case 9: {
      Snapshot ss;
      ss.index = a;
      ss.term = b;
      im->restore(ss);
      return 0;
    }
    case 10: im->resize(); return 0;
    case 11: {
      delete im->rl;
      im->rl = new RateLimiter();
      im->rl->maxSize = a;
      return 0;
    }
    case 12: return im->rl ? (int64_t)im->rl->get() : -1;
    case 13: return im->newEntries ? 1 : 0;
    default: return -2;
  }
  GUARD_END(-3)
}
int orc_inmem_entries_to_save(void* h, orc_entry* out, int cap) {
  GUARD_BEGIN
  auto v = ((InMemory*)h)->entriesToSave();
  int n = 0;
  for (auto& e : v) {
    if (n < cap) from_entry(e, &out[n]);
    n++;
  }
  return n;
  GUARD_END(-1)
}
}

// ---------------------------------------------------------------- Update helpers
// getUpdateCommit / validateUpdate / setFastApply (peer.go:209-245, 410-427) on
// an Update built from (index, term) pairs, for peer_test.go's tables
// (tests/test_update.py).  fn 0: getUpdateCommit → out6 = {processed,
// last_applied, stable_log_to, stable_log_term, stable_snapshot_to,
// ready_to_read}; fn 1: validateUpdate (-1 = panic); fn 2: setFastApply →
// out6[0] = FastApply.
extern "C" int orc_update_fn(int fn, uint64_t commit, const uint64_t* cents, int nc,
                             const uint64_t* sents, int ns, uint64_t snap_index,
                             uint64_t last_applied, uint64_t* out6) {
  GUARD_BEGIN
  Update ud;
  ud.state.commit = commit;
  for (int i = 0; i < nc; i++) {
    Entry e;
    e.index = cents[2 * i];
    e.term = cents[2 * i + 1];
    ud.committed_entries.push_back(e);
  }
  for (int i = 0; i < ns; i++) {
    Entry e;
    e.index = sents[2 * i];
    e.term = sents[2 * i + 1];
    ud.entries_to_save.push_back(e);
  }
  ud.snapshot.index = snap_index;
  ud.last_applied = last_applied;
  if (fn == 0) {
    UpdateCommit uc = getUpdateCommit(ud);
    out6[0] = uc.processed;
    out6[1] = uc.last_applied;
    out6[2] = uc.stable_log_to;
    out6[3] = uc.stable_log_term;
    out6[4] = uc.stable_snapshot_to;
    out6[5] = uc.ready_to_read;
    return 0;
  }
  if (fn == 1) {
    validateUpdate(ud);
    return 0;
  }
  if (fn == 2) {
    ud.fast_apply = true;
    out6[0] = setFastApply(ud).fast_apply ? 1 : 0;
    return 0;
  }
  return -2;
  GUARD_END(-1)
}
