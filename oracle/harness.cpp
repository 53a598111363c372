// ORACLE — TEST INFRASTRUCTURE ONLY (see raft_ref.h header comment).
// Lockstep multi-group harness: node.go step order + quiesce.go + a
// deterministic network (DESIGN.md §Round semantics).
#include "harness.h"

#include <algorithm>
#include <cstring>
#include <thread>

namespace orc {

// ------------------------------------------------------------ workload / faults
// Restated independently on device (dragonboat_amd/csrc/workload.h).
u64 wl_payload_lo(u64 seed, u64 cid, u64 round) {
  return splitmix64(seed ^ (cid * 0xD1B54A32D192ED03ULL) ^ (round << 1));
}

bool wl_group_active(const HarnessConfig& c, u64 cid) {
  if (c.wl_active_mod <= 1) return true;
  return below(splitmix64(c.seed ^ 0xA5A5A5A5A5A5A5A5ULL ^ (cid * 0x9E3779B97F4A7C15ULL)),
               c.wl_active_mod) == 0;
}

int wl_input(const HarnessConfig& c, u64 cid, u32 round) {
  if (!c.wl_enabled) return 0;
  if (round < c.wl_start_round) return 0;
  if (c.wl_stop_round != 0 && round >= c.wl_stop_round) return 0;
  if (!wl_group_active(c, cid)) return 0;
  if (c.wl_read_permille == 0) return 1;
  u64 u = below(splitmix64(c.seed ^ (cid * 0xC2B2AE3D27D4EB4FULL) ^ ((u64)round << 20)), 1000);
  return u < c.wl_read_permille ? 2 : 1;
}

// leader-transfer schedule: at every xfer_period-th round, in groups selected
// by hash, one seeded replica (any role) gets RequestLeaderTransfer(target)
// (node.go:1069-1075 handleLeaderTransferRequest → peer.go:106-113).
u64 xfer_input(const HarnessConfig& c, u64 cid, u32 round, u32 k) {
  if (!c.xfer_period || round == 0 || round % c.xfer_period != 0) return 0;
  const u64 epoch = round / c.xfer_period;
  if (c.xfer_mod > 1 &&
      below(splitmix64(c.seed ^ (cid * 0xA24BAED4963EE407ULL) ^ (epoch << 36)), c.xfer_mod) != 0)
    return 0;
  const u64 h = splitmix64(c.seed ^ (cid * 0x9FB21C651E98DF25ULL) ^ (epoch << 12) ^ 0x5851F42DULL);
  if (below(h, c.n_replicas) != k) return 0;
  return below(splitmix64(h), c.n_replicas) + 1;
}

// config-change schedule (restated on device, rbe_step.h cc_selected/cc_target)
bool cc_selected(const HarnessConfig& c, u64 cid, u32 round) {
  if (!c.cc_period || round == 0 || round % c.cc_period != 0) return false;
  const u64 epoch = round / c.cc_period;
  return c.cc_mod <= 1 ||
         below(splitmix64(c.seed ^ (cid * 0xE7037ED1A0B428DBULL) ^ (epoch << 28)), c.cc_mod) == 0;
}
u64 cc_target(const HarnessConfig& c, u64 cid, u32 round) {
  const u64 epoch = round / c.cc_period;
  return below(splitmix64(c.seed ^ (cid * 0x8EBC6AF09C88C6E3ULL) ^ (epoch << 20) ^ 0xCC),
               c.n_replicas) + 1;
}
std::string cc_cmd(int type, u64 node_id) {
  const u64 w = 0xCC00000000000000ULL | ((u64)(type & 0xFF) << 48) | (node_id & 0xFFFFFFFFFFFFULL);
  std::string s(8, '\0');
  for (int b = 0; b < 8; b++) s[b] = (char)((w >> (8 * b)) & 0xff);
  return s;
}
bool cc_decode(const std::string& cmd, int* type, u64* node_id) {
  if (cmd.size() != 8) return false;
  u64 w = 0;
  for (int b = 0; b < 8; b++) w |= (u64)(uint8_t)cmd[b] << (8 * b);
  if ((w >> 56) != 0xCC) return false;
  *type = (int)((w >> 48) & 0xFF);
  *node_id = w & 0xFFFFFFFFFFFFULL;
  return true;
}

bool iso_selected(const HarnessConfig& c, u64 cid, u32 epoch) {
  if (c.iso_mod <= 1) return true;
  return below(splitmix64(c.seed ^ (cid * 0x94D049BB133111EBULL) ^ ((u64)epoch << 40)),
               c.iso_mod) == 0;
}

// ------------------------------------------------------------ node
struct Node {
  TestLogDB db;
  Peer* peer = nullptr;
  QuiesceManager q;
  u64 confirmedIndex = 0;
  u64 smAppliedIndex = 0;
  u64 tickCount = 0;
  u64 digest = 0;
  u32 events = 0;               // EV_* bits of the last step
  // host inputs staged for the next step (harness_push)
  bool x_prop = false, x_read = false;
  std::vector<Entry> x_ents;
  SystemCtx x_ctx;
  u64 x_xfer = 0;
  u32 x_unreach = 0, x_snap = 0, x_snap_reject = 0;
  u64 x_applied = 0;
  bool more_to_apply = true;    // node.canHaveMoreEntriesToApply (sticky, PUSH_APPLY_READY)
  // node snapshot state (node.go ss: snapshotIndex, reqSnapshotIndex, compactLogTo)
  u64 ss_index = 0, ss_req = 0, compact_to = 0;
  u32 snap_pend = 0, snap_pend_reject = 0;  // SnapshotStatus of InstallSnapshots sent
  UpdateCommit uc;              // ext_commit: getUpdateCommit of the last step's Update
  Snapshot ud_snap;             // the Snapshot of the last step's Update (empty: none)
  // a ConfigChange to apply to raft at the next step: applied by the state
  // machine (membership, a committed stand-in entry) or sent by the host
  // (each ConfigChange of an Update, in log order: node.ApplyConfigChange /
  // ConfigChangeProcessed per entry, node.go:217-277)
  struct CcApply {
    bool reject;
    int type;
    u64 node;
  };
  std::vector<CcApply> cc_q;
  // the state machine's membership (rsm membership: the ConfigChanges it
  // applied, or the snapshot it recovered from), as the slots that are not
  // voters, bit k; a snapshot records it (pb.Snapshot.Membership)
  u32 sm_rem = 0;  // packed (pack_ms): slots not in Addresses | Observers << 8 | Witnesses << 16
  // RestoreRemotes for the next step: the state machine recovered from a
  // received snapshot (rr_pend: the LogDB's snapshot), or the host calls it
  // (PUSH_RESTORE: x_rr_mask)
  bool rr_pend = false, x_rr = false;
  u32 x_rr_mask = 0;
  // host ProposeConfigChange for the next step (PUSH_CC_PROPOSE)
  bool x_cc = false;
  int x_cc_type = 0;
  u64 x_cc_node = 0;
  std::vector<Message> in[8];   // this round's inbox, per sender slot (stream order)
  std::vector<Message> nxt[8];  // next round's inbox
  ~Node() { delete peer; }
};

struct Group {
  u64 cid = 0;
  std::vector<Node*> nodes;
  u32 iso_mask = 0;
  u32 iso_until = 0;
  ~Group() {
    for (auto* n : nodes) delete n;
  }
};

struct Harness {
  HarnessConfig cfg;
  std::vector<Group*> groups;
  u32 round = 0;
  u64 counters[HC_NUM] = {0};
  ~Harness() {
    for (auto* g : groups) delete g;
  }
};

static u64 cmd_word(const std::string& s, int w) {
  u64 x = 0;
  for (int i = 0; i < 8; i++) {
    size_t p = (size_t)w * 8 + i;
    if (p < s.size()) x |= (u64)(uint8_t)s[p] << (8 * i);
  }
  return x;
}

// A Cmd longer than 16 bytes, or an entry with session fields, is folded as a
// 64-bit fingerprint and a zero word (the engine keeps such an entry as a
// payload-heap record and digests its fingerprint; dragonboat_amd/csrc/
// rbe_host.h cmd_fingerprint / entry_fingerprint, restated here).
static u64 cmd_fingerprint(const std::string& s) {
  const u64 len = s.size();
  u64 h = 0x243F6A8885A308D3ull ^ len;
  for (u64 i = 0; i < len; i += 8) h = splitmix64(h ^ cmd_word(s, (int)(i / 8)));
  return splitmix64(h ^ (len << 1));
}
static bool has_session(const Entry& e) {
  return (e.key | e.client_id | e.series_id | e.responded_to) != 0;
}
static u64 entry_fingerprint(const Entry& e) {
  u64 h = cmd_fingerprint(e.cmd);
  if (has_session(e)) {
    const u64 meta[4] = {e.key, e.client_id, e.series_id, e.responded_to};
    for (u64 i = 0; i < 4; i++) h = splitmix64(h ^ meta[i] ^ ((i + 1) << 60));
  }
  return h;
}

static u64 hash_entry(u64 h, const Entry& e) {
  h = hfold(h, e.index);
  h = hfold(h, e.term);
  h = hfold(h, (u64)e.type | ((u64)e.cmd.size() << 32));
  if (e.cmd.size() > 16 || has_session(e)) {
    h = hfold(h, entry_fingerprint(e));
    h = hfold(h, 0);
  } else {
    h = hfold(h, cmd_word(e.cmd, 0));
    h = hfold(h, cmd_word(e.cmd, 1));
  }
  return h;
}

static u64 hash_message(u64 h, const Message& m) {
  h = hfold(h, (u64)m.type | ((u64)(m.reject ? 1 : 0) << 8) | ((u64)m.entries.size() << 16));
  h = hfold(h, m.to);
  h = hfold(h, m.from);
  h = hfold(h, m.term);
  // an InstallSnapshot carries its snapshot's (index, term) where other
  // messages carry LogIndex / LogTerm (the engine's message record)
  h = hfold(h, m.type == InstallSnapshot ? m.snapshot.term : m.log_term);
  h = hfold(h, m.type == InstallSnapshot ? m.snapshot.index : m.log_index);
  h = hfold(h, m.commit);
  h = hfold(h, m.hint);
  h = hfold(h, m.hint_high);
  for (auto& e : m.entries) h = hash_entry(h, e);
  return h;
}

static std::string payload_cmd(u64 seed, u64 cid, u64 round) {
  u64 lo = wl_payload_lo(seed, cid, round);
  u64 hi = splitmix64(lo);
  std::string s(16, '\0');
  for (int i = 0; i < 8; i++) {
    s[i] = (char)((lo >> (8 * i)) & 0xff);
    s[8 + i] = (char)((hi >> (8 * i)) & 0xff);
  }
  return s;
}

static Config node_config(const HarnessConfig& cfg, u64 cid, u32 k) {
  Config c;
  c.nodeID = k + 1;
  c.isObserver = ((cfg.observer_slots >> k) & 1u) != 0;
  c.isWitness = ((cfg.witness_slots >> k) & 1u) != 0;
  c.clusterID = cid;
  c.electionRTT = cfg.election_rtt;
  c.heartbeatRTT = cfg.heartbeat_rtt;
  c.checkQuorum = cfg.check_quorum;
  c.quiesce = cfg.quiesce;
  c.rngSeed = cfg.seed;
  c.maxEntrySize = cfg.max_entry_size;
  c.maxInMemLogSize = cfg.max_inmem_log_size;
  return c;
}

// A group's membership packed as slot masks (bit k = node k + 1): bits 0-7
// the slots not in Addresses (the voters, raft.remotes), 8-15 Observers,
// 16-23 Witnesses — the engine's rbe_launch_state::removed / snapshot-state
// encoding.  pb.Membership of a packed word and back; the harness's node
// addresses are "node-<id>".
static u32 pack_ms(u32 rem, u32 obs, u32 wit) { return rem | (obs << 8) | (wit << 16); }
static Membership membership_of(u32 ms, u32 n) {
  Membership m;
  for (u32 j = 0; j < n; j++) {
    const std::string a = "node-" + std::to_string(j + 1);
    if ((ms >> (8 + j)) & 1u) m.observers[j + 1] = a;
    else if ((ms >> (16 + j)) & 1u) m.witnesses[j + 1] = a;
    else if ((ms >> j) & 1u) m.removed[j + 1] = true;
    else m.addresses[j + 1] = a;
  }
  return m;
}
static u32 removed_of(const Membership& m, u32 n) {
  u32 rem = 0, obs = 0, wit = 0;
  for (u32 j = 0; j < n; j++) {
    if (!m.addresses.count(j + 1)) rem |= 1u << j;
    if (m.observers.count(j + 1)) obs |= 1u << j;
    if (m.witnesses.count(j + 1)) wit |= 1u << j;
  }
  return pack_ms(rem, obs, wit);
}
// Whether the state machine accepts a committed ConfigChange (rsm
// membership.go:299-321 handleConfigChange), judged on the membership `ms`
// (packed) raft holds when the entry is applied: an add of a node that already
// is a voter, observer or witness is rejected — alreadyMember,
// nodeBecomingObserver / Witness, witnessBecomingNode, observerBecomingWitness
// — except AddNode of an observer (isPromotingObserver); removing the only
// voter is rejected (isDeletingOnlyNode).  A rejected one goes back to raft as
// RejectConfigChange.  (The stand-in keeps no Removed set, so re-adding a
// removed node is accepted: the membership schedule relies on it.)
static bool cc_accepted(u32 ms, int t, u64 nid, u32 n) {
  if (nid < 1 || nid > n) return true;
  const u32 b = 1u << (nid - 1), rem = ms & 0xFF, obs = (ms >> 8) & 0xFF, wit = (ms >> 16) & 0xFF;
  const u32 voters = ((1u << n) - 1u) & ~rem;
  if (t == RemoveNode) return !(voters == b);
  if (t == AddNode && (obs & b)) return true;
  return !((voters | obs | wit) & b);
}
// the state machine's membership after it applied a ConfigChange (rsm
// membership.go applyConfigChange: AddNode also promotes an observer)
static void ms_apply(u32& ms, int t, u64 nid, u32 n) {
  if (nid < 1 || nid > n) return;
  const u32 b = 1u << (nid - 1);
  u32 rem = ms & 0xFF, obs = (ms >> 8) & 0xFF, wit = (ms >> 16) & 0xFF;
  if (t == AddNode) {
    rem &= ~b;
    obs &= ~b;
  } else if (t == RemoveNode) {
    rem |= b;
    obs &= ~b;
    wit &= ~b;
  } else if (t == AddObserver) {
    obs |= b;
  } else if (t == AddWitness) {
    wit |= b;
  }
  ms = pack_ms(rem, obs, wit);
}

// the voters a node starts with (its bootstrap): the initial members for one of
// them, nobody for a node that joins later (removed masks)
static u32 boot_removed(const HarnessConfig& cfg, u32 k) {
  const u32 n = cfg.n_replicas, nv = cfg.n_voters ? cfg.n_voters : n;
  const u32 all = (1u << n) - 1u;
  return k < nv ? all & ~((1u << nv) - 1u) : all;
}

static std::vector<std::pair<u64, std::string>> node_addrs(u32 n) {
  std::vector<std::pair<u64, std::string>> addrs;
  for (u32 k = 0; k < n; k++) addrs.push_back({k + 1, "node-" + std::to_string(k + 1)});
  return addrs;
}

Harness* harness_create(const HarnessConfig& cfg) {
  if (cfg.n_replicas < 1 || cfg.n_replicas > 8) panicf("n_replicas must be 1..8");
  const u32 nv = cfg.n_voters ? cfg.n_voters : cfg.n_replicas;
  if (nv > cfg.n_replicas || (nv < cfg.n_replicas && !cfg.membership))
    panicf("n_voters must be 1..n_replicas (fewer only with membership)");
  const u32 spare = ((1u << cfg.n_replicas) - 1u) & ~((1u << nv) - 1u);
  if (((cfg.observer_slots | cfg.witness_slots) & ~spare) ||
      (cfg.observer_slots & cfg.witness_slots))
    panicf("observer / witness slots are disjoint spare slots (beyond n_voters)");
  Harness* h = new Harness();
  h->cfg = cfg;
  std::vector<std::pair<u64, std::string>> addrs;
  for (u32 k = 0; k < nv; k++) addrs.push_back({k + 1, "node-" + std::to_string(k + 1)});
  for (u64 g = 0; g < cfg.n_groups; g++) {
    Group* gr = new Group();
    gr->cid = cfg.cid_base + g * cfg.cid_stride;
    for (u32 k = 0; k < cfg.n_replicas; k++) {
      Node* n = new Node();
      const Config c = node_config(cfg, gr->cid, k);
      // node.go:280-292: the initial members bootstrap the group; the other
      // slots are nodes that join later (StartCluster with join: no peers,
      // initial = false, an empty log)
      // a node that joins later may be an observer or a witness (config.IsObserver /
      // IsWitness: newRaft starts it in that state, raft.go:274-281)
      if (k < nv) n->peer = Peer::Launch(c, &n->db, addrs, true, true);
      else n->peer = Peer::Launch(c, &n->db, {}, false, true);
      n->sm_rem = boot_removed(cfg, k);
      n->q.enabled = cfg.quiesce;
      n->q.electionTick = cfg.election_rtt * 2;  // node.go:165
      gr->nodes.push_back(n);
    }
    h->groups.push_back(gr);
  }
  return h;
}

void harness_destroy(Harness* h) { delete h; }

// One stepNode + update processing for replica k of group gr in round r.
// EV_* bits (dragonboat_amd/csrc/rbe_types.h) from the listener calls a step made
static u32 event_bits(const Events& a, const Events& b, u64 leader0, u64 leader1) {
  u32 e = 0;
  if (leader1 != leader0) e |= 1;
  if (b.campaignLaunched != a.campaignLaunched) e |= 2;
  if (b.campaignSkipped != a.campaignSkipped) e |= 4;
  if (b.snapshotRejected != a.snapshotRejected) e |= 8;
  if (b.replicationRejected != a.replicationRejected) e |= 16;
  if (b.proposalDropped != a.proposalDropped) e |= 32;
  if (b.readIndexDropped != a.readIndexDropped) e |= 64;
  return e;
}

static void step_replica(const HarnessConfig& cfg, Group* gr, u32 k, u32 r, bool tick, u64* ctr) {
  Node* nd = gr->nodes[k];
  Peer* p = nd->peer;
  Raft* R = p->raft;
  const u32 n = cfg.n_replicas;
  nd->events = 0;
  nd->uc = UpdateCommit();
  nd->ud_snap = Snapshot();
  // client input of this round: the workload goes to replicas that lead at
  // round start, host input (harness_push) to the replica it names
  const int wl = R->state == Leader ? wl_input(cfg, gr->cid, r) : 0;
  // the config-change schedule proposes at the replica leading at round start
  bool do_cc = nd->x_cc;
  int cc_type = nd->x_cc_type;
  u64 cc_node = nd->x_cc_node;
  if (!do_cc && cfg.membership && R->state == Leader && cc_selected(cfg, gr->cid, r)) {
    // the seeded node: a voter is removed (while more than two are in
    // raft.remotes) and added back; an observer slot's node is added as an
    // observer, then promoted (AddNode) and kept; a witness slot's node is
    // added as a witness and removed again (rbe_step.h cc_schedule)
    cc_node = cc_target(cfg, gr->cid, r);
    const u32 b = 1u << (cc_node - 1);
    const bool voter = R->remotes.count(cc_node) > 0;
    const bool big = R->remotes.size() > 2;
    if (cfg.observer_slots & b) {
      if (R->observers.count(cc_node)) do_cc = true, cc_type = AddNode;
      else if (!voter) do_cc = true, cc_type = AddObserver;
    } else if (cfg.witness_slots & b) {
      if (!R->witnesses.count(cc_node)) do_cc = true, cc_type = AddWitness;
      else if (big) do_cc = true, cc_type = RemoveNode;
    } else if (!voter || big) {
      do_cc = true;
      cc_type = voter ? RemoveNode : AddNode;
    }
  }
  const bool do_read = wl == 2 || nd->x_read;
  const bool do_prop = wl == 1 || nd->x_prop;
  u64 xfer = nd->x_xfer ? nd->x_xfer : xfer_input(cfg, gr->cid, r, k);
  // updateBatchedLastApplied (node.go:1010-1014): with ext_apply the state
  // machine's applied index is the host's, else the harness applies each
  // step's committed entries at once
  if (cfg.ext_apply) nd->smAppliedIndex = nd->x_applied;
  const u64 applied = nd->smAppliedIndex;
  if (!tick) {
    // a round without a tick is a step only if handleEvents finds an event
    // (node.go:1030-1067)
    bool ev = do_read || do_prop || xfer || nd->x_unreach || nd->x_snap || nd->snap_pend ||
              p->HasEntryToApply() || applied != nd->confirmedIndex || do_cc || !nd->cc_q.empty() ||
              nd->rr_pend || nd->x_rr;
    for (u32 s = 0; s < n; s++) ev = ev || !nd->in[s].empty();
    if (!ev) return;
  }
  ctr[HC_STEPS]++;
  const Events ev0 = R->events;
  const u64 leader0 = R->leaderID;
  // the step's counters start here, before the calls made between two steps
  // (the engine counts an entry a RemoveNode lets the leader commit with the step)
  const u64 committed0 = R->log.committed;
  const u64 campaigns0 = R->events.campaignLaunched;
  // Peer.RestoreRemotes (peer.go:159-165) once the state machine recovered
  // from a snapshot (rsm/statemachine.go:236 → node.go:241-264), or the
  // host's; then a ConfigChange the state machine applied (or the host sent)
  // since the last step: Peer.ApplyConfigChange / RejectConfigChange
  // (peer.go:138-157).  Direct calls under raftMu between two steps.
  if (nd->x_rr || nd->rr_pend) {
    Snapshot ss = nd->db.snapshot;
    if (nd->x_rr) ss.membership = membership_of(nd->x_rr_mask, n);
    nd->x_rr = nd->rr_pend = false;
    p->RestoreRemotes(ss);
  }
  for (const Node::CcApply& a : nd->cc_q) {
    if (a.reject) p->RejectConfigChange();
    else p->ApplyConfigChange(a.node, a.type);
  }
  nd->cc_q.clear();
  // handleEvents: updateBatchedLastApplied (node.go:1002-1006, 1032)
  p->NotifyRaftLastApplied(applied);
  // handleReadIndexRequests (node.go:1108-1118)
  u64 readReq = 0;
  if (do_read) {
    nd->q.recordActivity(ReadIndex);
    readReq = 1;
    ctr[HC_READS]++;
  }
  // host-reported Unreachable / SnapshotStatus: node-handled messages of the
  // inbox (node.go:1207-1220), delivered first, no activity recorded
  for (u32 s = 0; s < n; s++)
    if ((nd->x_unreach >> s) & 1u) p->ReportUnreachableNode(s + 1);
  {
    // the transport's outcome of last round's InstallSnapshots, then host reports
    const u32 snap = nd->x_snap | nd->snap_pend;
    const u32 rej = (nd->x_snap_reject & nd->x_snap) | (nd->snap_pend_reject & ~nd->x_snap);
    nd->snap_pend = nd->snap_pend_reject = 0;
    for (u32 s = 0; s < n; s++)
      if ((snap >> s) & 1u) p->ReportSnapshotStatus(s + 1, ((rej >> s) & 1u) != 0);
  }
  // handleReceivedMessages (node.go:1171-1205); one LocalTick per ticking round
  u64 ltCount = tick ? 1 : 0;
  for (u32 s = 0; s < n; s++) {
    for (auto& m : nd->in[s]) {
      ctr[HC_MSG_IN]++;
      ctr[HC_ENT_IN] += m.entries.size();
      if (m.type == Quiesce) {  // handleMessage, node.go:1207-1220
        nd->q.tryEnterQuiesce();
        continue;
      }
      // tryRecordNodeActivity, node.go:1161-1169
      if ((m.type == Heartbeat || m.type == HeartbeatResp) && m.hint > 0)
        nd->q.recordActivity(ReadIndex);
      else
        nd->q.recordActivity(m.type);
      p->Handle(m);
    }
    nd->in[s].clear();
  }
  if (readReq > 0) {  // batchedReadIndex, node.go:1379-1382
    SystemCtx ctx;
    if (nd->x_read) {
      ctx = nd->x_ctx;
    } else {
      ctx.low = ((u64)(r + 1) << 32) | (u64)(k + 1);
      ctx.high = gr->cid + 1;
    }
    p->ReadIndex(ctx);
  }
  // handleLocalTickMessage (node.go:1152-1159) → node.tick (1384-1399)
  if (ltCount > cfg.election_rtt) ltCount = cfg.election_rtt;
  for (u64 i = 0; i < ltCount; i++) {
    nd->tickCount++;
    nd->q.increaseQuiesceTick();
    if (nd->q.quiesced()) {
      p->QuiescedTick();
      ctr[HC_QUIESCED_TICKS]++;
    } else {
      p->Tick();
      ctr[HC_ACTIVE_TICKS]++;
    }
  }
  // handleConfigChangeMessage (node.go:1120-1142): recordActivity, then
  // Peer.ProposeConfigChange with the marshaled ConfigChange (stand-in Cmd)
  if (do_cc) {
    nd->q.recordActivity(ConfigChangeEvent);
    p->ProposeConfigChange(cc_cmd(cc_type, cc_node), 0);
  }
  // handleProposals (node.go:1091-1106)
  if (do_prop) {
    if (nd->x_prop) {
      p->ProposeEntries(nd->x_ents);
    } else {
      std::vector<Entry> ents(1);
      ents[0].type = ApplicationEntry;
      ents[0].cmd = payload_cmd(cfg.seed, gr->cid, r);
      p->ProposeEntries(ents);
    }
    ctr[HC_PROPOSALS]++;
  }
  // handleLeaderTransferRequest (node.go:1069-1075)
  if (xfer) p->RequestLeaderTransfer(xfer);
  nd->x_prop = nd->x_read = false;
  nd->x_cc = false;
  nd->x_ents.clear();
  nd->x_xfer = 0;
  nd->x_unreach = nd->x_snap = nd->x_snap_reject = 0;
  // stepNode: quiesce state (node.go:1021-1023)
  const bool sendQ = nd->q.newQuiesceState();
  // getUpdate (node.go:907-923)
  u64 msgHash = 0, nMsgs = 0, rtrHash = 0, applyHash = 0, dropHash = 0;
  auto deliver = [&](const Message& m) {
    if (m.to < 1 || m.to > n) return;  // not a member of this lockstep group
    u32 d = (u32)(m.to - 1);
    const bool dropped = ((gr->iso_mask >> k) & 1) || ((gr->iso_mask >> d) & 1);
    if (m.type == InstallSnapshot) {
      // the transport streams the snapshot and reports the outcome to the
      // sender's node, which hands it to raft at its next step
      // (ReportSnapshotStatus, peer.go:177-184; nodehost.go snapshot status)
      nd->snap_pend |= 1u << d;
      if (dropped) nd->snap_pend_reject |= 1u << d;
      else nd->snap_pend_reject &= ~(1u << d);
    }
    if (dropped) {
      ctr[HC_MSG_DROPPED]++;
      return;
    }
    ctr[HC_MSG_OUT]++;
    ctr[HC_ENT_OUT] += m.entries.size();
    gr->nodes[d]->nxt[k].push_back(m);
  };
  if (sendQ) {  // sendEnterQuiesceMessages, node.go:873-886
    for (u32 d = 0; d < n; d++) {
      if (d == k) continue;
      Message m;
      m.type = Quiesce;
      m.from = k + 1;
      m.to = d + 1;
      m.cluster_id = gr->cid;
      deliver(m);
    }
  }
  // node.getUpdate (node.go:907-923) with moreEntriesToApply from the node's
  // apply queue (canHaveMoreEntriesToApply, node.go:1002-1004)
  if (p->HasUpdate(nd->more_to_apply) || nd->confirmedIndex != nd->smAppliedIndex) {
    Update ud = p->GetUpdate(nd->more_to_apply, nd->smAppliedIndex);
    nd->confirmedIndex = nd->smAppliedIndex;
    for (auto& m : ud.messages) {
      msgHash = hash_message(msgHash, m);
      nMsgs++;
    }
    // applyRaftUpdates: the harness state machine applies immediately; a
    // ConfigChange entry is handed back to raft at the next step (membership)
    u32 raft_ms = 0;  // raft's membership as the accepted changes go by
    bool have_ms = false;
    for (auto& e : ud.committed_entries) {
      applyHash = hash_entry(applyHash, e);
      int t;
      u64 nid;
      if (cfg.membership && !cfg.ext_apply && e.type == ConfigChangeEntry &&
          cc_decode(e.cmd, &t, &nid)) {
        if (!have_ms) {
          Membership m;
          for (auto& kv : R->remotes) m.addresses[kv.first] = "";
          for (auto& kv : R->observers) m.observers[kv.first] = "";
          for (auto& kv : R->witnesses) m.witnesses[kv.first] = "";
          raft_ms = removed_of(m, n);
          have_ms = true;
        }
        const bool rej = !cc_accepted(raft_ms, t, nid, n);
        nd->cc_q.push_back(Node::CcApply{rej, t, nid});
        if (!rej) {
          ms_apply(raft_ms, t, nid, n);
          // the state machine's membership (rsm membership.go)
          ms_apply(nd->sm_rem, t, nid, n);
        }
      }
    }
    ctr[HC_ENT_APPLIED] += ud.committed_entries.size();
    // (a state machine that recovered from a snapshot at a restart skips the
    // committed entries it already holds, rsm/statemachine.go)
    if (!ud.committed_entries.empty() && !cfg.ext_apply)
      nd->smAppliedIndex = std::max(nd->smAppliedIndex, ud.committed_entries.back().index);
    // sendReplicateMessages (node.go:897-905) then, after persistence,
    // sendMessages (node.go:888-895)
    for (auto& m : ud.messages)
      if (m.type == Replicate) deliver(m);
    // processReadyToRead
    for (auto& rr : ud.ready_to_reads) {
      rtrHash = hfold(rtrHash, rr.index);
      rtrHash = hfold(rtrHash, rr.ctx.low);
      rtrHash = hfold(rtrHash, rr.ctx.high);
    }
    ctr[HC_READS_CONFIRMED] += ud.ready_to_reads.size();
    for (auto& e : ud.dropped_entries) dropHash = hash_entry(dropHash, e);
    for (auto& c : ud.dropped_read_indexes) {
      dropHash = hfold(dropHash, c.low);
      dropHash = hfold(dropHash, c.high);
    }
    ctr[HC_DROPPED_PROPOSALS] += ud.dropped_entries.size();
    ctr[HC_DROPPED_READS] += ud.dropped_read_indexes.size();
    // SaveRaftState → logreader.Append (node.go:975-977)
    nd->db.Append(ud.entries_to_save);
    if (!isEmptyState(ud.state)) nd->db.SetState(ud.state);
    ctr[HC_ENT_SAVED] += ud.entries_to_save.size();
    for (auto& m : ud.messages)
      if (m.type != Replicate) deliver(m);
    // a snapshot received through InstallSnapshot: the LogDB takes it and the
    // state machine recovers from it (node.go processSnapshot / rsm recover)
    // With ext_commit the Updates carry a restored snapshot until the host's
    // UpdateCommit names it (StableSnapshotTo); the LogDB took it the first
    // time (a later ApplySnapshot of it is ErrSnapshotOutOfDate, a soft
    // error, node.go:950-965) and nothing else happens again.
    nd->ud_snap = ud.snapshot;
    if (!isEmptySnapshot(ud.snapshot) && nd->db.ApplySnapshot(ud.snapshot) == ErrOK) {
      if (!cfg.ext_apply) nd->smAppliedIndex = ud.snapshot.index;
      nd->ss_index = ud.snapshot.index;
      // the state machine takes the snapshot's membership, and the node
      // restores raft's remotes from it at the next step (RestoreRemotes)
      nd->sm_rem = removed_of(ud.snapshot.membership, n);
      nd->rr_pend = cfg.membership && !cfg.ext_apply;  // ext_apply: the host calls it
    }
    if (!cfg.ext_commit) {
      p->Commit(ud);  // commitRaftUpdate
    } else {
      // Peer.Commit (peer.go:282-293) with its log part deferred: the step's
      // outputs are consumed here, entryLog.commitUpdate runs when the host
      // sends the UpdateCommit (harness_commit, the engine's rbe_commit)
      R->msgs.clear();
      R->droppedEntries.clear();
      R->droppedReadIndexes.clear();
      if (!isEmptyState(ud.state)) p->prevState = ud.state;
      if (ud.update_commit.ready_to_read > 0) R->readyToRead.clear();
      nd->uc = ud.update_commit;
    }
  }
  if (cfg.snapshot_entries) {
    // compactLog (node.go:849-866): the compaction a snapshot asked for, at the
    // node's next step; then saveSnapshotRequired / doSaveSnapshot /
    // compactSnapshot (node.go:585-605, 619-692) with the state machine's
    // applied index, done within the step (the lockstep definition of the
    // snapshot worker)
    // With ext_commit a compaction waits while the raft log still holds a
    // restored snapshot the host has not committed: the node runs compactLog
    // before that Commit within one step (node.go:975-999), so the log's first
    // index never moves past a snapshot it holds in memory.
    if (nd->compact_to && !R->log.inmem.hasSnapshot) {
      // ErrCompacted / ErrUnavailable: nothing to do; never past the snapshot
      if (nd->compact_to <= nd->db.snapshot.index) nd->db.Compact(nd->compact_to);
      nd->compact_to = 0;
    }
    // with ext_apply the host's snapshot worker decides (harness_snapshot_saved /
    // harness_compact, the engine's rbe_snapshot_saved / rbe_compact)
    const u64 S = cfg.snapshot_entries, la = nd->smAppliedIndex;
    if (!cfg.ext_apply && !(la <= S + nd->ss_index || la <= S + nd->ss_req)) {
      nd->ss_req = la;
      u64 t = 0;
      if (R->log.term(la, &t) == ErrOK && t != 0) {
        Snapshot ss;
        ss.index = la;
        ss.term = t;
        ss.membership = membership_of(nd->sm_rem, n);  // the state machine's at la
        if (nd->db.CreateSnapshot(ss) == ErrOK) {
          if (la > cfg.compaction_overhead) nd->compact_to = la - cfg.compaction_overhead;
          nd->ss_index = la;
        }
      }
    }
  }
  ctr[HC_CAMPAIGNS] += R->events.campaignLaunched - campaigns0;
  nd->events = event_bits(ev0, R->events, leader0, R->leaderID);
  if (R->state == Leader) {
    ctr[HC_COMMITTED] += R->log.committed - committed0;
    ctr[HC_LEADER_STEPS]++;
  }
  if (cfg.trace) {
    u64 d = nd->digest;
    d = hfold(d, r);
    d = hfold(d, (u64)R->state | ((u64)(nd->q.quiesced() ? 1 : 0) << 8) |
                     ((u64)(sendQ ? 1 : 0) << 9) | ((u64)(R->quiesce ? 1 : 0) << 10));
    d = hfold(d, R->term);
    d = hfold(d, R->vote);
    d = hfold(d, R->leaderID);
    d = hfold(d, R->log.committed);
    d = hfold(d, R->log.lastIndex());
    d = hfold(d, R->log.processed);
    d = hfold(d, R->electionTick | (R->heartbeatTick << 32));
    d = hfold(d, R->randomizedElectionTimeout);
    d = hfold(d, msgHash);
    d = hfold(d, nMsgs);
    d = hfold(d, rtrHash);
    d = hfold(d, applyHash);
    d = hfold(d, dropHash);
    nd->digest = d;
  }
}

static void run_group_round(const HarnessConfig& cfg, Group* gr, u32 r, bool tick, u64* ctr) {
  // fault schedule: isolation decided from round-start roles
  if (gr->iso_mask && r >= gr->iso_until) gr->iso_mask = 0;
  if (cfg.iso_period && r > 0 && r % cfg.iso_period == 0 &&
      iso_selected(cfg, gr->cid, r / cfg.iso_period)) {
    u32 mask = 0;
    for (u32 k = 0; k < cfg.n_replicas; k++)
      if (gr->nodes[k]->peer->raft->state == Leader) mask |= 1u << k;
    if (mask) {
      gr->iso_mask = mask;
      gr->iso_until = r + cfg.iso_len;
    }
  }
  for (u32 k = 0; k < cfg.n_replicas; k++) step_replica(cfg, gr, k, r, tick, ctr);
  for (u32 k = 0; k < cfg.n_replicas; k++) {
    Node* nd = gr->nodes[k];
    for (u32 s = 0; s < cfg.n_replicas; s++) {
      nd->in[s].swap(nd->nxt[s]);
      nd->nxt[s].clear();
    }
  }
}

static void run_rounds(Harness* h, u32 rounds, bool tick) {
  const u32 T = std::max<u32>(1, h->cfg.threads);
  const u32 r0 = h->round;
  std::vector<std::vector<u64>> ctrs(T, std::vector<u64>(HC_NUM, 0));
  auto worker = [&](u32 t) {
    for (u32 r = r0; r < r0 + rounds; r++)
      for (u64 g = t; g < h->groups.size(); g += T)
        run_group_round(h->cfg, h->groups[g], r, tick, ctrs[t].data());
  };
  if (T == 1) {
    worker(0);
  } else {
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> errs(T);
    for (u32 t = 0; t < T; t++)
      th.emplace_back([&, t]() {
        try {
          worker(t);
        } catch (...) {
          errs[t] = std::current_exception();
        }
      });
    for (auto& x : th) x.join();
    for (auto& e : errs)
      if (e) std::rethrow_exception(e);
  }
  for (u32 t = 0; t < T; t++)
    for (int i = 0; i < HC_NUM; i++) h->counters[i] += ctrs[t][i];
  h->round += rounds;
}

void harness_run(Harness* h, u32 rounds) { run_rounds(h, rounds, true); }
void harness_step(Harness* h, bool tick) { run_rounds(h, 1, tick); }

int harness_push(Harness* h, int kind, u64 replica, u64 a, u64 b, const Entry* ents, u32 n) {
  const u32 N = h->cfg.n_replicas;
  if (replica >= h->groups.size() * N) return -1;
  Node* nd = h->groups[replica / N]->nodes[replica % N];
  switch (kind) {
    case PUSH_PROPOSE:
      nd->x_prop = true;
      nd->x_ents.assign(ents, ents + n);
      return 0;
    case PUSH_READ:
      nd->x_read = true;
      nd->x_ctx.low = a;
      nd->x_ctx.high = b;
      return 0;
    case PUSH_XFER: nd->x_xfer = a; return 0;
    case PUSH_UNREACH: nd->x_unreach |= 1u << (a - 1); return 0;
    case PUSH_SNAPST:
      nd->x_snap |= 1u << (a - 1);
      if (b) nd->x_snap_reject |= 1u << (a - 1);
      else nd->x_snap_reject &= ~(1u << (a - 1));
      return 0;
    case PUSH_APPLIED: nd->x_applied = a; return 0;
    case PUSH_APPLY_READY: nd->more_to_apply = a != 0; return 0;
    case PUSH_CC_PROPOSE:
      nd->x_cc = true;
      nd->x_cc_type = (int)a;
      nd->x_cc_node = b;
      return 0;
    case PUSH_CC_APPLY:
      nd->cc_q.assign(1, Node::CcApply{false, (int)b, a});
      return 0;
    case PUSH_CC_REJECT:
      nd->cc_q.assign(1, Node::CcApply{true, 0, 0});
      return 0;
    case PUSH_RESTORE:  // a: packed membership (pack_ms)
      if (((a & 0xFF) >> N) || (((a >> 8) & 0xFF) >> N) || (((a >> 16) & 0xFF) >> N) || (a >> 24))
        return -1;
      nd->x_rr = true;
      nd->x_rr_mask = (u32)a;
      return 0;
    default: return -1;
  }
}

// Host-driven snapshots (ext_apply): the snapshot worker saved the state
// machine's snapshot at `index` and the LogDB took it (doSaveSnapshot →
// LogReader.CreateSnapshot, node.go:619-692; out of date: ignored), or asks
// the next step to compact (compactSnapshot → compactLog, node.go:849-866).
int harness_snapshot_saved(Harness* h, u64 replica, u64 index, u64 term, u32 removed) {
  const u32 N = h->cfg.n_replicas;
  if (replica >= h->groups.size() * N || index == 0 || term == 0 || ((removed & 0xFF) >> N) ||
      (((removed >> 8) & 0xFF) >> N) || (((removed >> 16) & 0xFF) >> N) || (removed >> 24))
    return -1;
  Node* nd = h->groups[replica / N]->nodes[replica % N];
  if (index > nd->x_applied) return -1;  // only what the state machine applied
  Snapshot ss;
  ss.index = index;
  ss.term = term;
  ss.membership = membership_of(removed, N);
  if (nd->db.CreateSnapshot(ss) == ErrOK) nd->ss_index = index;
  return 0;
}
int harness_compact(Harness* h, u64 replica, u64 to) {
  const u32 N = h->cfg.n_replicas;
  if (replica >= h->groups.size() * N || to == 0) return -1;
  h->groups[replica / N]->nodes[replica % N]->compact_to = to;
  return 0;
}

u32 harness_round(const Harness* h) { return h->round; }

void harness_persisted(const Harness* h, u64 replica, u64 out4[4]) {
  const u32 N = h->cfg.n_replicas;
  TestLogDB& db = h->groups[replica / N]->nodes[replica % N]->db;
  const PState st = db.state;
  out4[0] = st.term;
  out4[1] = st.vote;
  out4[2] = st.commit;
  out4[3] = db.lastIndex();
}

void harness_snapshot_state(const Harness* h, u64 replica, u64 out8[8]) {
  const u32 N = h->cfg.n_replicas;
  const Node* nd = h->groups[replica / N]->nodes[replica % N];
  out8[0] = nd->db.markerIndex;
  out8[1] = nd->db.markerTerm;
  out8[2] = nd->db.snapshot.index;
  out8[3] = nd->db.snapshot.term;
  out8[4] = nd->ss_req;
  out8[5] = nd->compact_to;
  // the LogDB's membership (NodeState): its latest snapshot's, else the bootstrap's
  out8[6] = nd->db.snapshot.index ? removed_of(nd->db.snapshot.membership, N)
                                  : boot_removed(h->cfg, (u32)(replica % N));
  out8[7] = nd->sm_rem;
}

int harness_persisted_entries(const Harness* h, u64 replica, u64 lo, u64 hi, Entry* out) {
  const u32 N = h->cfg.n_replicas;
  TestLogDB& db = h->groups[replica / N]->nodes[replica % N]->db;
  std::vector<Entry> v;
  if (db.Entries(lo, hi + 1, ~0ull, &v) != ErrOK || v.size() != hi - lo + 1) return -1;
  for (size_t i = 0; i < v.size(); i++) out[i] = v[i];
  return 0;
}

// A node restart (rbe_launch): the raft comes back through Peer.Launch over its
// LogDB (initial = newNode = false, peer.go:64-86) with the LogDB's membership
// (logdb.NodeState: its latest snapshot's, raft.go:260-270; without a snapshot
// the group's bootstrap members, all of this harness's static slots), and the
// state machine recovers that snapshot's membership too; the node around it
// starts afresh: quiesce state, tick count, apply bookkeeping, apply-queue
// state.  Messages in flight to and from the node are lost.  Host input
// already staged for it stays staged.
void harness_restart(Harness* h, u64 replica) {
  const HarnessConfig& cfg = h->cfg;
  const u32 N = cfg.n_replicas;
  Group* gr = h->groups[replica / N];
  const u32 k = (u32)(replica % N);
  Node* nd = gr->nodes[k];
  if (nd->db.snapshot.index == 0)
    nd->db.snapshot.membership = membership_of(boot_removed(cfg, k), N);
  nd->sm_rem = removed_of(nd->db.snapshot.membership, N);
  nd->rr_pend = false;
  delete nd->peer;
  // an observer slot's node that was promoted (it is in Addresses) restarts as a follower
  Config c = node_config(cfg, gr->cid, k);
  if (c.isObserver && !(nd->sm_rem & (1u << k))) c.isObserver = false;
  nd->peer = Peer::Launch(c, &nd->db, node_addrs(N), false, false);
  // a fresh quiesceManager kept on the harness's tick clock: its counters are
  // translated by the ticks before the restart (tick = noActivitySince =
  // exitQuiesceTick = t, not quiesced), which quiesce.go cannot tell apart from
  // all-zero counters (it compares only differences, and nothing can enter
  // quiesce before the first tick: justExitedQuiesce holds then)
  const u64 t = nd->q.tick;
  nd->q = QuiesceManager();
  nd->q.enabled = cfg.quiesce;
  nd->q.electionTick = cfg.election_rtt * 2;  // node.go:165
  nd->q.tick = nd->q.noActivitySince = nd->q.exitQuiesceTick = t;
  nd->tickCount = 0;
  nd->confirmedIndex = 0;
  // the state machine recovers from the LogDB's latest snapshot (rsm
  // RecoverFromSnapshot; 0 without snapshots)
  nd->smAppliedIndex = cfg.ext_apply ? nd->x_applied : nd->db.snapshot.index;
  nd->events = 0;
  nd->more_to_apply = true;
  for (u32 s = 0; s < N; s++) nd->in[s].clear();
  for (u32 j = 0; j < N; j++)
    if (j != k) gr->nodes[j]->in[k].clear();
}

// A new node in a removed node's slot (the engine's rbe_replace_node): -1
// when another node of the group still refers to the slot's node (raft.go's
// maps, vote, leader, leader-transfer target, vote tally, ReadIndex queue,
// rate-limiter reports) or a message it sent last round is still to be
// delivered; else the slot's node is a fresh one that joins the running
// cluster (node.go:280-292: Launch with no peers and newNode over an empty
// LogDB; the node around it is new too, its quiesce manager on the tick clock
// as in harness_restart) and messages to the slot are dropped.  Inside the
// harness the new node keeps the slot's node id: with nothing left that names
// the old node, that is the reference run with a new id.
int harness_replace(Harness* h, u64 replica) {
  const HarnessConfig& cfg = h->cfg;
  const u32 N = cfg.n_replicas;
  if (replica >= h->groups.size() * N) return -1;
  Group* gr = h->groups[replica / N];
  const u32 k = (u32)(replica % N);
  const u64 id = k + 1;
  for (u32 j = 0; j < N; j++) {
    if (j == k) continue;
    const Node* o = gr->nodes[j];
    const Raft* R = o->peer->raft;
    if (R->remotes.count(id) || R->observers.count(id) || R->witnesses.count(id) ||
        R->vote == id || R->leaderID == id || R->leaderTransferTarget == id || R->votes.count(id) ||
        R->rl.followerSizes.count(id))
      return -1;
    for (const auto& kv : R->readIndex.pending)
      if (kv.second.from == id || kv.second.confirmed.count(id)) return -1;
    if (!o->in[k].empty()) return -1;
  }
  Node* old = gr->nodes[k];
  const u64 t = old->q.tick;
  Node* nd = new Node();
  nd->peer = Peer::Launch(node_config(cfg, gr->cid, k), &nd->db, {}, false, true);
  nd->sm_rem = (1u << N) - 1u;  // a joining node's state machine knows no members yet
  nd->q.enabled = cfg.quiesce;
  nd->q.electionTick = cfg.election_rtt * 2;  // node.go:165
  nd->q.tick = nd->q.noActivitySince = nd->q.exitQuiesceTick = t;
  gr->nodes[k] = nd;
  delete old;
  for (u32 j = 0; j < N; j++)
    if (j != k) gr->nodes[j]->in[k].clear();
  return 0;
}

void harness_update_snapshot(const Harness* h, u64 replica, u64 out4[4]) {
  const u32 N = h->cfg.n_replicas;
  const Snapshot& ss = h->groups[replica / N]->nodes[replica % N]->ud_snap;
  out4[0] = ss.index;
  out4[1] = ss.term;
  out4[2] = isEmptySnapshot(ss) ? 0 : removed_of(ss.membership, N);
  out4[3] = 0;
}

void harness_update_commit(const Harness* h, u64 replica, UpdateCommit* out) {
  const u32 N = h->cfg.n_replicas;
  *out = h->groups[replica / N]->nodes[replica % N]->uc;
}

u32 harness_inbox(const Harness* h, u64 replica, u32 sender, u64* out, u32 cap) {
  const u32 N = h->cfg.n_replicas;
  const auto& in = h->groups[replica / N]->nodes[replica % N]->in[sender];
  u32 n = 0;
  for (const Message& m : in) {
    if (n < cap) {
      u64* o = out + 10 * n;
      o[0] = m.type;
      o[1] = m.from;
      o[2] = m.to;
      o[3] = m.term;
      o[4] = m.log_term;
      o[5] = m.log_index;
      o[6] = m.commit;
      o[7] = m.reject ? 1 : 0;
      o[8] = m.hint;
      o[9] = m.entries.size();
    }
    n++;
  }
  return n;
}

void harness_commit(Harness* h, u64 replica, const UpdateCommit& uc) {
  const u32 N = h->cfg.n_replicas;
  h->groups[replica / N]->nodes[replica % N]->peer->raft->log.commitUpdate(uc);
}

void harness_rate_limited(Harness* h, uint8_t* limited, u64* size) {
  const u32 n = h->cfg.n_replicas;
  for (u64 g = 0; g < h->groups.size(); g++)
    for (u32 k = 0; k < n; k++) {
      Peer* p = h->groups[g]->nodes[k]->peer;
      if (limited) limited[g * n + k] = p->rateLimited() ? 1 : 0;
      if (size) size[g * n + k] = p->raft->rl.get();
    }
}

void harness_views(const Harness* h, ReplicaView* out) {
  const u32 n = h->cfg.n_replicas;
  for (u64 g = 0; g < h->groups.size(); g++) {
    for (u32 k = 0; k < n; k++) {
      const Node* nd = h->groups[g]->nodes[k];
      const Raft* R = nd->peer->raft;
      ReplicaView& v = out[g * n + k];
      std::memset(&v, 0, sizeof(v));
      v.term = R->term;
      v.vote = R->vote;
      v.leader_id = R->leaderID;
      v.committed = R->log.committed;
      v.last_index = R->log.lastIndex();
      v.processed = R->log.processed;
      v.saved_to = R->log.inmem.savedTo;
      v.digest = nd->digest;
      v.role = (u32)R->state;
      v.election_tick = (u32)R->electionTick;
      v.heartbeat_tick = (u32)R->heartbeatTick;
      v.rand_election_timeout = (u32)R->randomizedElectionTimeout;
      v.q_tick = (u32)nd->q.tick;
      v.q_quiesced_since = (u32)nd->q.quiescedSince;
      v.q_no_activity_since = (u32)nd->q.noActivitySince;
      v.q_exit_quiesce_tick = (u32)nd->q.exitQuiesceTick;
      v.raft_quiesce = R->quiesce ? 1 : 0;
      v.rq_count = (u32)R->readIndex.queue.size();
      u32 resp = 0, granted = 0;
      for (auto& kv : R->votes) {
        if (kv.first >= 1 && kv.first <= 8) {
          resp |= 1u << (kv.first - 1);
          if (kv.second) granted |= 1u << (kv.first - 1);
        }
      }
      v.votes_resp = resp;
      v.votes_granted = granted;
      for (u32 s = 0; s < n; s++) {
        if (!R->remotes.count(s + 1)) v.removed |= 1u << s;
        if (R->observers.count(s + 1)) v.observers |= 1u << s;
        if (R->witnesses.count(s + 1)) v.witnesses |= 1u << s;
      }
      v.events = nd->events;
      if (R->state == Leader) {  // remotes, observers and witnesses (each slot in one)
        for (const auto* mp : {&R->remotes, &R->observers, &R->witnesses}) {
          for (auto& kv : *mp) {
            if (kv.first >= 1 && kv.first <= 8) {
              u32 s = (u32)(kv.first - 1);
              v.match[s] = kv.second.match;
              v.next[s] = kv.second.next;
              v.rstate[s] = (u32)kv.second.state;
              v.ractive[s] = kv.second.active ? 1 : 0;
            }
          }
        }
      }
    }
  }
}

void harness_counters(const Harness* h, u64* out) {
  for (int i = 0; i < HC_NUM; i++) out[i] = h->counters[i];
}

u64 harness_log_term(const Harness* h, u64 g, u32 k, u64 index) {
  const Raft* R = h->groups[g]->nodes[k]->peer->raft;
  u64 t = 0;
  if (R->log.term(index, &t) != ErrOK) return 0;
  return t;
}

}  // namespace orc
