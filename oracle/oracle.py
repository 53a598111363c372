"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding to liboracle.so, the CPU restatement of dragonboat's
internal/raft (see oracle/raft_ref.h).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this module; the product package
(dragonboat_amd) never does.

Two surfaces:
  * unit level (Raft / LogDB / Peer objects) for the transcribed reference
    known-answer tests (tests/test_oracle_*.py), shaped like the Go tests'
    newTestRaft / network helpers (internal/raft/raft_etcd_test.go:2821-3003);
  * Harness: the deterministic lockstep multi-group harness that the MI355X
    engine is checked against (tests/test_parity_*.py).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

# raftpb MessageType (raft.pb.go:23-51)
(LocalTick, Election, LeaderHeartbeat, ConfigChangeEvent, NoOP, Ping, Pong, Propose,
 SnapshotStatus, Unreachable, CheckQuorum, BatchedReadIndex, Replicate, ReplicateResp,
 RequestVote, RequestVoteResp, InstallSnapshot, Heartbeat, HeartbeatResp, ReadIndex,
 ReadIndexResp, Quiesce, SnapshotReceived, LeaderTransfer, TimeoutNow, RateLimit) = range(26)
# raft State (raft.go:63-70)
FOLLOWER, CANDIDATE, LEADER, OBSERVER, WITNESS = range(5)
# remote states (remote.go:27-32)
REMOTE_RETRY, REMOTE_WAIT, REMOTE_REPLICATE, REMOTE_SNAPSHOT = range(4)
# entry types
APPLICATION_ENTRY, CONFIG_CHANGE_ENTRY, ENCODED_ENTRY, METADATA_ENTRY = range(4)
ADD_NODE, REMOVE_NODE, ADD_OBSERVER, ADD_WITNESS = range(4)
ERR_OK, ERR_COMPACTED, ERR_UNAVAILABLE, ERR_SNAPSHOT_OUT_OF_DATE = range(4)
NO_LIMIT = (1 << 64) - 1


class OrcEntry(C.Structure):
    _fields_ = [("term", C.c_uint64), ("index", C.c_uint64), ("key", C.c_uint64),
                ("client_id", C.c_uint64), ("series_id", C.c_uint64),
                ("responded_to", C.c_uint64), ("type", C.c_uint32),
                ("cmd_len", C.c_uint32), ("cmd", C.c_uint8 * 64), ("data", C.c_void_p)]


class OrcSnapshot(C.Structure):
    _fields_ = [("index", C.c_uint64), ("term", C.c_uint64), ("n_addr", C.c_uint32),
                ("n_obs", C.c_uint32), ("n_wit", C.c_uint32), ("flags", C.c_uint32),
                ("addr", C.c_uint64 * 8), ("obs", C.c_uint64 * 8), ("wit", C.c_uint64 * 8)]


class OrcMsg(C.Structure):
    _fields_ = [("type", C.c_uint32), ("reject", C.c_uint32), ("to", C.c_uint64),
                ("from_", C.c_uint64), ("cluster_id", C.c_uint64), ("term", C.c_uint64),
                ("log_term", C.c_uint64), ("log_index", C.c_uint64), ("commit", C.c_uint64),
                ("hint", C.c_uint64), ("hint_high", C.c_uint64), ("n_entries", C.c_uint32),
                ("pad", C.c_uint32), ("entries", C.POINTER(OrcEntry)),
                ("snapshot", OrcSnapshot)]


class OrcConfig(C.Structure):
    _fields_ = [("node_id", C.c_uint64), ("cluster_id", C.c_uint64), ("election", C.c_uint64),
                ("heartbeat", C.c_uint64), ("seed", C.c_uint64), ("max_entry_size", C.c_uint64),
                ("check_quorum", C.c_uint32), ("is_observer", C.c_uint32),
                ("is_witness", C.c_uint32), ("quiesce", C.c_uint32)]


class OrcHarnessConfig(C.Structure):
    _fields_ = [("n_groups", C.c_uint64), ("n_replicas", C.c_uint32),
                ("check_quorum", C.c_uint32), ("cid_base", C.c_uint64),
                ("election_rtt", C.c_uint64), ("heartbeat_rtt", C.c_uint64),
                ("seed", C.c_uint64), ("max_entry_size", C.c_uint64),
                ("quiesce", C.c_uint32), ("wl_enabled", C.c_uint32),
                ("wl_start_round", C.c_uint32), ("wl_stop_round", C.c_uint32),
                ("wl_active_mod", C.c_uint32), ("wl_read_permille", C.c_uint32),
                ("iso_period", C.c_uint32), ("iso_len", C.c_uint32), ("iso_mod", C.c_uint32),
                ("trace", C.c_uint32), ("threads", C.c_uint32), ("pad", C.c_uint32),
                ("cid_stride", C.c_uint64), ("xfer_period", C.c_uint32),
                ("xfer_mod", C.c_uint32), ("ext_apply", C.c_uint32),
                ("snapshot_entries", C.c_uint32), ("compaction_overhead", C.c_uint32),
                ("ext_commit", C.c_uint32), ("membership", C.c_uint32),
                ("cc_period", C.c_uint32), ("cc_mod", C.c_uint32), ("n_voters", C.c_uint32),
                ("max_inmem_log_size", C.c_uint64), ("observer_slots", C.c_uint32),
                ("witness_slots", C.c_uint32)]


class ReplicaView(C.Structure):
    """Mirrors rbe_replica_view (include/rbe.h) / orc::ReplicaView."""
    _fields_ = [("term", C.c_uint64), ("vote", C.c_uint64), ("leader_id", C.c_uint64),
                ("committed", C.c_uint64), ("last_index", C.c_uint64),
                ("processed", C.c_uint64), ("saved_to", C.c_uint64), ("digest", C.c_uint64),
                ("role", C.c_uint32), ("election_tick", C.c_uint32),
                ("heartbeat_tick", C.c_uint32), ("rand_election_timeout", C.c_uint32),
                ("q_tick", C.c_uint32), ("q_quiesced_since", C.c_uint32),
                ("q_no_activity_since", C.c_uint32), ("q_exit_quiesce_tick", C.c_uint32),
                ("raft_quiesce", C.c_uint32), ("rq_count", C.c_uint32),
                ("votes_resp", C.c_uint32), ("votes_granted", C.c_uint32),
                ("match", C.c_uint64 * 8), ("next", C.c_uint64 * 8),
                ("rstate", C.c_uint32 * 8), ("ractive", C.c_uint32 * 8),
                ("events", C.c_uint32), ("removed", C.c_uint32),
                ("observers", C.c_uint32), ("witnesses", C.c_uint32)]


VIEW_FIELDS = [f[0] for f in ReplicaView._fields_ if f[0] != "pad"]
# harness_push kinds (oracle/harness.h HarnessPush)
PUSH_PROPOSE, PUSH_READ, PUSH_XFER, PUSH_UNREACH, PUSH_SNAPST, PUSH_APPLIED, PUSH_APPLY_READY = \
    range(1, 8)
PUSH_CC_PROPOSE, PUSH_CC_APPLY, PUSH_CC_REJECT, PUSH_RESTORE = 8, 9, 10, 11
# pb.ConfigChangeType (raft.pb.go): AddNode, RemoveNode, AddObserver, AddWitness
CC_ADD_NODE, CC_REMOVE_NODE, CC_ADD_OBSERVER, CC_ADD_WITNESS = 0, 1, 2, 3

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"{_LIB_PATH} missing: run `make -C oracle` or __graft_entry__.build()")
        L = C.CDLL(_LIB_PATH)
        vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int, C.c_uint32
        P = C.POINTER
        sig = {
            "orc_last_error": (C.c_char_p, []),
            "orc_logdb_new": (vp, []), "orc_logdb_free": (None, [vp]),
            "orc_logdb_append": (i32, [vp, P(OrcEntry), i32]),
            "orc_logdb_set_state": (None, [vp, u64, u64, u64]),
            "orc_logdb_apply_snapshot": (i32, [vp, P(OrcSnapshot)]),
            "orc_logdb_create_snapshot": (i32, [vp, P(OrcSnapshot)]),
            "orc_logdb_compact": (i32, [vp, u64]),
            "orc_logdb_term": (i32, [vp, u64, P(u64)]),
            "orc_logdb_range": (None, [vp, P(u64), P(u64)]),
            "orc_logdb_entries": (i32, [vp, u64, u64, u64, P(OrcEntry), i32]),
            "orc_raft_new": (vp, [P(OrcConfig), vp]), "orc_raft_free": (None, [vp]),
            "orc_raft_handle": (i32, [vp, P(OrcMsg)]),
            "orc_raft_num_messages": (i32, [vp]),
            "orc_raft_num_message_entries": (i32, [vp]),
            "orc_raft_read_messages": (i32, [vp, P(OrcMsg), i32, P(OrcEntry), i32]),
            "orc_raft_peek_messages": (i32, [vp, P(OrcMsg), i32, P(OrcEntry), i32]),
            "orc_raft_get": (u64, [vp, i32]), "orc_raft_set": (i32, [vp, i32, u64]),
            "orc_raft_call": (C.c_int64, [vp, i32, u64, u64]),
            "orc_raft_remote_get": (i32, [vp, i32, u64, P(u64)]),
            "orc_remote_op": (C.c_int64, [P(u64), i32, u64, u64]),
            "orc_raft_handle_direct": (i32, [vp, i32, P(OrcMsg)]),
            "orc_raft_remote_set": (None, [vp, i32, u64, u64, u64, u64, u64, u64]),
            "orc_raft_remote_del": (None, [vp, i32, u64]),
            "orc_raft_remote_clear": (None, [vp, i32]),
            "orc_raft_remote_ids": (i32, [vp, i32, P(u64), i32]),
            "orc_raft_votes": (i32, [vp, P(u64), P(C.c_uint8), i32]),
            "orc_raft_ready_to_read": (i32, [vp, P(u64), i32]),
            "orc_raft_clear_ready_to_read": (None, [vp]),
            "orc_raft_dropped_ri": (i32, [vp, P(u64), i32]),
            "orc_raft_dropped_entries": (i32, [vp, P(OrcEntry), i32]),
            "orc_raft_readindex_queue": (i32, [vp, P(u64), i32]),
            "orc_raft_matched": (i32, [vp, P(u64), i32]),
            "orc_raft_set_matched": (None, [vp, P(u64), i32]),
            "orc_raft_log_term": (i32, [vp, u64, P(u64)]),
            "orc_raft_log_entries": (i32, [vp, u64, u64, P(OrcEntry), i32]),
            "orc_raft_log_get_entries": (i32, [vp, u64, u64, u64, P(OrcEntry), i32]),
            "orc_raft_log_append": (i32, [vp, P(OrcEntry), i32]),
            "orc_raft_log_try_append": (C.c_int64, [vp, u64, P(OrcEntry), i32]),
            "orc_raft_log_conflict_index": (C.c_int64, [vp, P(OrcEntry), i32]),
            "orc_raft_log_entries_to_save": (i32, [vp, P(OrcEntry), i32]),
            "orc_raft_log_entries_to_apply": (i32, [vp, P(OrcEntry), i32]),
            "orc_raft_log_restore": (i32, [vp, P(OrcSnapshot)]),
            "orc_raft_restore": (i32, [vp, P(OrcSnapshot)]),
            "orc_raft_restore_remotes": (i32, [vp, P(OrcSnapshot)]),
            "orc_raft_read_index_add": (i32, [vp, u64, u64, u64, u64]),
            "orc_raft_read_index_confirm": (i32, [vp, u64, u64, u64, i32, P(u64), i32]),
            "orc_peer_launch": (vp, [P(OrcConfig), vp, P(u64), i32, i32, i32]),
            "orc_peer_free": (None, [vp]), "orc_peer_raft": (vp, [vp]),
            "orc_peer_tick": (i32, [vp, i32]), "orc_peer_handle": (i32, [vp, P(OrcMsg)]),
            "orc_peer_propose": (i32, [vp, P(OrcEntry), i32]),
            "orc_peer_read_index": (i32, [vp, u64, u64]),
            "orc_peer_misc": (i32, [vp, i32, u64, u64]),
            "orc_peer_propose_cc": (i32, [vp, u64, i32, u64]),
            "orc_peer_get_update": (i32, [vp, i32, u64, P(u64)]),
            "orc_peer_update_entries": (i32, [vp, i32, P(OrcEntry), i32]),
            "orc_peer_update_messages": (i32, [vp, P(OrcMsg), i32, P(OrcEntry), i32]),
            "orc_peer_update_rtr": (i32, [vp, P(u64), i32]),
            "orc_peer_commit": (i32, [vp]),
            "orc_peer_update_set_commit": (None, [vp, P(u64)]),
            "orc_harness_create": (vp, [P(OrcHarnessConfig)]),
            "orc_harness_destroy": (None, [vp]),
            "orc_harness_run": (i32, [vp, u32]),
            "orc_harness_step": (i32, [vp, i32]),
            "orc_harness_push": (i32, [vp, i32, u64, u64, u64, P(OrcEntry), i32]),
            "orc_harness_round": (u32, [vp]),
            "orc_harness_views": (None, [vp, vp]),
            "orc_harness_rate_limited": (None, [vp, vp, vp]),
            "orc_harness_counters": (None, [vp, P(u64)]),
            "orc_harness_log_term": (u64, [vp, u64, u32, u64]),
            "orc_harness_persisted": (None, [vp, u64, P(u64)]),
            "orc_harness_snapshot_state": (None, [vp, u64, P(u64)]),
            "orc_harness_persisted_entries": (i32, [vp, u64, u64, u64, P(OrcEntry)]),
            "orc_harness_restart": (i32, [vp, u64]),
            "orc_harness_snapshot_saved": (i32, [vp, u64, u64, u64, u32]),
            "orc_harness_compact": (i32, [vp, u64, u64]),
            "orc_harness_update_commit": (None, [vp, u64, P(u64)]),
            "orc_harness_update_snapshot": (None, [vp, u64, P(u64)]),
            "orc_harness_replace": (C.c_int, [vp, u64]),
            "orc_harness_commit": (i32, [vp, u64, P(u64)]),
            "orc_harness_inbox": (u32, [vp, u64, u32, P(u64), u32]),
            "orc_view_size": (i32, []),
            "orc_splitmix64": (u64, [u64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        assert L.orc_view_size() == C.sizeof(ReplicaView), "ReplicaView layout mismatch"
        _lib = L
    return _lib


class RaftPanic(RuntimeError):
    """A plog.Panicf / panic() of the reference, raised by the restatement."""


def _err():
    return RaftPanic(lib().orc_last_error().decode())


# ----------------------------------------------------------------- value types
@dataclass
class Entry:
    index: int = 0
    term: int = 0
    type: int = APPLICATION_ENTRY
    cmd: bytes = b""
    key: int = 0
    client_id: int = 0
    series_id: int = 0
    responded_to: int = 0

    def to_c(self, e: OrcEntry):
        e.term, e.index, e.type = self.term, self.index, self.type
        e.key, e.client_id, e.series_id, e.responded_to = (
            self.key, self.client_id, self.series_id, self.responded_to)
        e.cmd_len = len(self.cmd)
        for i, b in enumerate(self.cmd[:64]):
            e.cmd[i] = b
        if len(self.cmd) > 64:  # the whole Cmd by pointer; the caller keeps it alive
            buf = C.create_string_buffer(bytes(self.cmd), len(self.cmd))
            e.data = C.cast(buf, C.c_void_p)
            return buf
        return None

    @staticmethod
    def from_c(e: OrcEntry) -> "Entry":
        return Entry(index=e.index, term=e.term, type=e.type,
                     cmd=bytes(e.cmd[:e.cmd_len]), key=e.key, client_id=e.client_id,
                     series_id=e.series_id, responded_to=e.responded_to)


def entries_array(ents: List[Entry]):
    arr = (OrcEntry * max(1, len(ents)))()
    keep = [e.to_c(arr[i]) for i, e in enumerate(ents)]
    arr._keep = [k for k in keep if k is not None]  # Cmd buffers of long entries
    return arr


@dataclass
class Snapshot:
    index: int = 0
    term: int = 0
    addresses: List[int] = field(default_factory=list)
    observers: List[int] = field(default_factory=list)
    witnesses: List[int] = field(default_factory=list)
    dummy: bool = False
    witness: bool = False

    def to_c(self) -> OrcSnapshot:
        s = OrcSnapshot()
        s.index, s.term = self.index, self.term
        s.n_addr, s.n_obs, s.n_wit = len(self.addresses), len(self.observers), len(self.witnesses)
        for i, v in enumerate(self.addresses):
            s.addr[i] = v
        for i, v in enumerate(self.observers):
            s.obs[i] = v
        for i, v in enumerate(self.witnesses):
            s.wit[i] = v
        s.flags = (1 if self.dummy else 0) | (2 if self.witness else 0)
        return s

    @staticmethod
    def from_c(s: OrcSnapshot) -> "Snapshot":
        return Snapshot(index=s.index, term=s.term, addresses=list(s.addr[:s.n_addr]),
                        observers=list(s.obs[:s.n_obs]), witnesses=list(s.wit[:s.n_wit]),
                        dummy=bool(s.flags & 1), witness=bool(s.flags & 2))


@dataclass
class Message:
    type: int = 0
    to: int = 0
    from_: int = 0
    term: int = 0
    log_term: int = 0
    log_index: int = 0
    commit: int = 0
    reject: bool = False
    hint: int = 0
    hint_high: int = 0
    entries: List[Entry] = field(default_factory=list)
    snapshot: Snapshot = field(default_factory=Snapshot)
    cluster_id: int = 0

    def to_c(self):
        m = OrcMsg()
        m.type, m.reject, m.to, m.from_ = self.type, 1 if self.reject else 0, self.to, self.from_
        m.cluster_id, m.term, m.log_term, m.log_index = (
            self.cluster_id, self.term, self.log_term, self.log_index)
        m.commit, m.hint, m.hint_high = self.commit, self.hint, self.hint_high
        arr = entries_array(self.entries)
        m.n_entries = len(self.entries)
        m.entries = C.cast(arr, C.POINTER(OrcEntry))
        m.snapshot = self.snapshot.to_c()
        return m, arr

    @staticmethod
    def from_c(m: OrcMsg) -> "Message":
        ents = [Entry.from_c(m.entries[i]) for i in range(m.n_entries)] if m.n_entries else []
        return Message(type=m.type, to=m.to, from_=m.from_, term=m.term, log_term=m.log_term,
                       log_index=m.log_index, commit=m.commit, reject=bool(m.reject),
                       hint=m.hint, hint_high=m.hint_high, entries=ents,
                       snapshot=Snapshot.from_c(m.snapshot), cluster_id=m.cluster_id)


def msg(type, **kw) -> Message:
    if "from" in kw:
        kw["from_"] = kw.pop("from")
    return Message(type=type, **kw)


# ----------------------------------------------------------------- LogDB
class LogDB:
    """TestLogDB (internal/raft/logdb_test.go:25-177)."""

    def __init__(self):
        self.h = lib().orc_logdb_new()
        self.owned = True

    def __del__(self):
        if getattr(self, "owned", False) and self.h:
            lib().orc_logdb_free(self.h)
            self.h = None

    def append(self, ents: List[Entry]):
        arr = entries_array(ents)
        if lib().orc_logdb_append(self.h, arr, len(ents)) < 0:
            raise _err()

    def set_state(self, term=0, vote=0, commit=0):
        lib().orc_logdb_set_state(self.h, term, vote, commit)

    def apply_snapshot(self, ss: Snapshot) -> int:
        s = ss.to_c()
        return lib().orc_logdb_apply_snapshot(self.h, C.byref(s))

    def create_snapshot(self, ss: Snapshot) -> int:
        s = ss.to_c()
        return lib().orc_logdb_create_snapshot(self.h, C.byref(s))

    def compact(self, index) -> int:
        return lib().orc_logdb_compact(self.h, index)

    def term(self, index):
        t = C.c_uint64()
        err = lib().orc_logdb_term(self.h, index, C.byref(t))
        return t.value, err

    def get_range(self):
        a, b = C.c_uint64(), C.c_uint64()
        lib().orc_logdb_range(self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def entries(self, lo, hi, max_size=NO_LIMIT):
        cap = max(1, hi - lo + 1)
        out = (OrcEntry * cap)()
        n = lib().orc_logdb_entries(self.h, lo, hi, max_size, out, cap)
        if n < 0:
            return [], -n
        return [Entry.from_c(out[i]) for i in range(min(n, cap))], ERR_OK


def ents(*pairs) -> List[Entry]:
    """ents((index, term), ...) helper."""
    return [Entry(index=i, term=t) for (i, t) in pairs]


# ----------------------------------------------------------------- Raft
_FIELDS = ["term", "vote", "state", "leader_id", "committed", "processed", "applied",
           "last_index", "first_index", "election_tick", "heartbeat_tick",
           "randomized_election_timeout", "election_timeout", "heartbeat_timeout",
           "check_quorum", "quiesce", "leader_transfer_target", "is_leader_transfer_target",
           "pending_config_change", "node_id", "tick_count", "num_voting_members", "quorum",
           "ready_to_read_count", "dropped_entries_count", "dropped_read_index_count",
           "read_index_queue_len", "last_term", "test_cc_mode", "saved_to", "marker_index",
           "inmem_len", "cluster_id", "num_remotes", "num_observers", "num_witnesses",
           "shrunk", "has_inmem_snapshot", "rng_count", "votes_len", "matched_len"]
_FIELD_IDX = {n: i for i, n in enumerate(_FIELDS)}
_CALLS = ["become_follower", "become_candidate", "become_leader", "tick", "quiesced_tick",
          "reset", "campaign", "try_commit", "add_node", "remove_node", "add_observer",
          "add_witness", "broadcast_replicate", "broadcast_heartbeat", "send_replicate",
          "has_config_change_to_apply", "leader_has_quorum", "log_commit_to", "log_match_term",
          "log_up_to_date", "log_try_commit", "self_removed", "become_observer",
          "become_witness", "inmem_applied_log_to", "has_committed_entry_at_current_term",
          "pending_config_change_count", "reset_match_value_array", "sort_match_values",
          "handle_vote_resp", "can_grant_vote", "inmem_try_resize", "inmem_resize",
          "log_has_entries_to_apply", "log_first_not_applied_index", "inmem_saved_log_to",
          "time_for_election", "set_randomized_election_timeout", "abort_leader_transfer",
          "leader_transfering", "quiesced_tick_direct", "non_leader_tick", "leader_tick",
          "load_state",
          # rate limiter (server/rate.go; raft.go:660-683, 1779-1785)
          "rl_set_max", "rl_get", "rl_tick", "rl_rate_limited", "rl_enabled", "rl_increase",
          "rl_decrease", "rl_set", "rl_set_follower", "rl_follower_count", "rl_follower_size",
          "rl_follower_tick", "rl_heartbeat_tick", "rl_gc", "rl_reset_followers",
          "rl_handle_leader_rate_limit", "rl_append_entries"]
_CALL_IDX = {n: i for i, n in enumerate(_CALLS)}
KIND = {"remotes": 0, "observers": 1, "witnesses": 2}


@dataclass
class RemoteView:
    match: int
    next: int
    snapshot_index: int
    state: int
    active: bool


class Raft:
    """A restated `*raft` (raft.go:197-289)."""

    def __init__(self, handle, logdb: Optional[LogDB] = None, owned=True):
        object.__setattr__(self, "h", handle)
        object.__setattr__(self, "logdb", logdb)
        object.__setattr__(self, "owned", owned)

    @staticmethod
    def new(node_id, peers=(), election=10, heartbeat=1, logdb: Optional[LogDB] = None,
            check_quorum=False, is_observer=False, is_witness=False, seed=0x5EEDD8A6,
            cluster_id=0, max_entry_size=0, test_cc_mode=True) -> "Raft":
        """newTestRaft (raft_etcd_test.go:2981-2991)."""
        db = logdb or LogDB()
        cfg = OrcConfig(node_id=node_id, cluster_id=cluster_id, election=election,
                        heartbeat=heartbeat, seed=seed, max_entry_size=max_entry_size,
                        check_quorum=int(check_quorum), is_observer=int(is_observer),
                        is_witness=int(is_witness))
        h = lib().orc_raft_new(C.byref(cfg), db.h)
        if not h:
            raise _err()
        r = Raft(h, db)
        if r.num_remotes == 0:
            for p in peers:
                r.set_remote("remotes", p, match=0, next=1)
        if test_cc_mode:
            r.test_cc_mode = 1
        return r

    def __del__(self):
        if getattr(self, "owned", False) and self.h:
            lib().orc_raft_free(self.h)
            object.__setattr__(self, "h", None)

    def __getattr__(self, name):
        if name in _FIELD_IDX:
            return lib().orc_raft_get(self.h, _FIELD_IDX[name])
        if name in _CALL_IDX:
            idx = _CALL_IDX[name]

            def call(a=0, b=0):
                v = lib().orc_raft_call(self.h, idx, int(a), int(b))
                if v <= -999:
                    raise _err()
                return v
            return call
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if name in _FIELD_IDX:
            if lib().orc_raft_set(self.h, _FIELD_IDX[name], int(value)) != 0:
                raise AttributeError(f"field {name} is read-only")
            return
        object.__setattr__(self, name, value)

    # --- messages
    def handle(self, m: Message):
        cm, keep = m.to_c()
        if lib().orc_raft_handle(self.h, C.byref(cm)) != 0:
            raise _err()

    def handle_direct(self, which: str, m: Message):
        """Call one handler without Handle's term gate (as the Go tests do)."""
        cm, keep = m.to_c()
        idx = ["replicate", "heartbeat", "request_vote"].index(which)
        if lib().orc_raft_handle_direct(self.h, idx, C.byref(cm)) != 0:
            raise _err()

    def read_messages(self) -> List[Message]:
        n = lib().orc_raft_num_messages(self.h)
        ne = lib().orc_raft_num_message_entries(self.h)
        out = (OrcMsg * max(1, n))()
        eb = (OrcEntry * max(1, ne))()
        k = lib().orc_raft_read_messages(self.h, out, n, eb, ne)
        return [Message.from_c(out[i]) for i in range(k)]

    def peek_messages(self) -> List[Message]:
        n = lib().orc_raft_num_messages(self.h)
        ne = lib().orc_raft_num_message_entries(self.h)
        out = (OrcMsg * max(1, n))()
        eb = (OrcEntry * max(1, ne))()
        k = lib().orc_raft_peek_messages(self.h, out, n, eb, ne)
        return [Message.from_c(out[i]) for i in range(k)]

    # --- remotes
    def remote(self, id, kind="remotes") -> Optional[RemoteView]:
        o = (C.c_uint64 * 5)()
        if not lib().orc_raft_remote_get(self.h, KIND[kind], id, o):
            return None
        return RemoteView(o[0], o[1], o[2], o[3], bool(o[4]))

    def set_remote(self, kind, id, match=0, next=0, snapshot_index=0, state=REMOTE_RETRY,
                   active=False):
        lib().orc_raft_remote_set(self.h, KIND[kind], id, match, next, snapshot_index, state,
                                  1 if active else 0)

    def del_remote(self, kind, id):
        lib().orc_raft_remote_del(self.h, KIND[kind], id)

    def clear_remotes(self, kind):
        lib().orc_raft_remote_clear(self.h, KIND[kind])

    def remote_ids(self, kind="remotes") -> List[int]:
        o = (C.c_uint64 * 64)()
        n = lib().orc_raft_remote_ids(self.h, KIND[kind], o, 64)
        return list(o[:n])

    def votes(self) -> Dict[int, bool]:
        ids = (C.c_uint64 * 64)()
        g = (C.c_uint8 * 64)()
        n = lib().orc_raft_votes(self.h, ids, g, 64)
        return {ids[i]: bool(g[i]) for i in range(n)}

    def ready_to_read(self):
        o = (C.c_uint64 * (3 * 256))()
        n = lib().orc_raft_ready_to_read(self.h, o, 256)
        return [(o[3 * i], o[3 * i + 1], o[3 * i + 2]) for i in range(min(n, 256))]

    def clear_ready_to_read(self):
        lib().orc_raft_clear_ready_to_read(self.h)

    def dropped_read_indexes(self):
        o = (C.c_uint64 * 512)()
        n = lib().orc_raft_dropped_ri(self.h, o, 256)
        return [(o[2 * i], o[2 * i + 1]) for i in range(min(n, 256))]

    def dropped_entries(self) -> List[Entry]:
        out = (OrcEntry * 256)()
        n = lib().orc_raft_dropped_entries(self.h, out, 256)
        return [Entry.from_c(out[i]) for i in range(min(n, 256))]

    def read_index_queue(self):
        o = (C.c_uint64 * (5 * 256))()
        n = lib().orc_raft_readindex_queue(self.h, o, 256)
        return [tuple(o[5 * i:5 * i + 5]) for i in range(min(n, 256))]

    def read_index_add(self, index, ctx, from_):
        if lib().orc_raft_read_index_add(self.h, index, ctx[0], ctx[1], from_) != 0:
            raise _err()

    def read_index_confirm(self, ctx, from_, quorum):
        o = (C.c_uint64 * (4 * 256))()
        n = lib().orc_raft_read_index_confirm(self.h, ctx[0], ctx[1], from_, quorum, o, 256)
        if n < 0:
            raise _err()
        return [tuple(o[4 * i:4 * i + 4]) for i in range(n)]

    def matched(self):
        o = (C.c_uint64 * 64)()
        n = lib().orc_raft_matched(self.h, o, 64)
        return list(o[:n])

    def set_matched(self, vals):
        arr = (C.c_uint64 * max(1, len(vals)))(*vals)
        lib().orc_raft_set_matched(self.h, arr, len(vals))

    # --- log
    def log_term(self, index):
        t = C.c_uint64()
        err = lib().orc_raft_log_term(self.h, index, C.byref(t))
        if err < 0:
            raise _err()
        return t.value, err

    def log_entries(self, start, max_size=NO_LIMIT):
        cap = 4096
        out = (OrcEntry * cap)()
        n = lib().orc_raft_log_entries(self.h, start, max_size, out, cap)
        if n <= -100:
            raise _err()
        if n < 0:
            return [], -n
        return [Entry.from_c(out[i]) for i in range(min(n, cap))], ERR_OK

    def log_get_entries(self, lo, hi, max_size=NO_LIMIT):
        cap = 4096
        out = (OrcEntry * cap)()
        n = lib().orc_raft_log_get_entries(self.h, lo, hi, max_size, out, cap)
        if n <= -100:
            raise _err()
        if n < 0:
            return [], -n
        return [Entry.from_c(out[i]) for i in range(min(n, cap))], ERR_OK

    def log_append(self, ents: List[Entry]):
        arr = entries_array(ents)
        if lib().orc_raft_log_append(self.h, arr, len(ents)) != 0:
            raise _err()

    def log_try_append(self, index, ents: List[Entry]) -> bool:
        arr = entries_array(ents)
        v = lib().orc_raft_log_try_append(self.h, index, arr, len(ents))
        if v < 0:
            raise _err()
        return bool(v)

    def log_conflict_index(self, ents: List[Entry]) -> int:
        arr = entries_array(ents)
        v = lib().orc_raft_log_conflict_index(self.h, arr, len(ents))
        if v < 0:
            raise _err()
        return v

    def log_entries_to_save(self) -> List[Entry]:
        out = (OrcEntry * 4096)()
        n = lib().orc_raft_log_entries_to_save(self.h, out, 4096)
        return [Entry.from_c(out[i]) for i in range(min(n, 4096))]

    def log_entries_to_apply(self) -> List[Entry]:
        out = (OrcEntry * 4096)()
        n = lib().orc_raft_log_entries_to_apply(self.h, out, 4096)
        if n < 0:
            raise _err()
        return [Entry.from_c(out[i]) for i in range(min(n, 4096))]

    def restore(self, ss: Snapshot) -> bool:
        s = ss.to_c()
        v = lib().orc_raft_restore(self.h, C.byref(s))
        if v < 0:
            raise _err()
        return bool(v)

    def restore_remotes(self, ss: Snapshot):
        s = ss.to_c()
        if lib().orc_raft_restore_remotes(self.h, C.byref(s)) < 0:
            raise _err()

    def log_restore(self, ss: Snapshot):
        s = ss.to_c()
        if lib().orc_raft_log_restore(self.h, C.byref(s)) < 0:
            raise _err()


REMOTE_OPS = ["become_retry", "retry_to_wait", "wait_to_retry", "become_wait",
              "become_replicate", "become_snapshot", "try_update", "progress", "responded_to",
              "decrease_to", "is_paused", "clear_pending_snapshot", "set_active",
              "set_not_active", "is_active"]


class Remote:
    """A free-standing `remote` (remote.go:62-69) for the remote_test.go tables."""

    def __init__(self, match=0, next=0, snapshot_index=0, state=REMOTE_RETRY, active=False):
        self.st = (C.c_uint64 * 5)(match, next, snapshot_index, state, int(active))

    match = property(lambda self: self.st[0])
    next = property(lambda self: self.st[1])
    snapshot_index = property(lambda self: self.st[2])
    state = property(lambda self: self.st[3])
    active = property(lambda self: bool(self.st[4]))

    def op(self, name, a=0, b=0):
        v = lib().orc_remote_op(self.st, REMOTE_OPS.index(name), a, b)
        if v <= -999:
            raise _err()
        return v


class BlackHole:
    """blackHole peer (raft_etcd_test.go:2959-2964)."""

    def handle(self, m):
        pass

    def read_messages(self):
        return []


class Network:
    """The reference's in-process test network (raft_etcd_test.go:2821-2952).

    `network.filter` drops with unseeded math/rand only for fractional
    rates; every use here is 0 or 1, so the filter is deterministic."""

    def __init__(self, *peers, config=None):
        size = len(peers)
        ids = list(range(1, size + 1))
        self.peers = {}
        self.storage = {}
        self.dropm = {}
        self.ignorem = set()
        cfg = dict(config or {})
        for j, p in enumerate(peers):
            id = ids[j]
            if p is None:
                db = LogDB()
                self.storage[id] = db
                r = Raft.new(id, (), election=cfg.get("election", 10),
                             heartbeat=cfg.get("heartbeat", 1), logdb=db,
                             check_quorum=cfg.get("check_quorum", False))
                for pid in ids:
                    r.set_remote("remotes", pid, match=0, next=1)
                if cfg.get("post") is not None:
                    cfg["post"](r)
                self.peers[id] = r
            elif isinstance(p, Raft):
                obs = set(p.remote_ids("observers"))
                wit = set(p.remote_ids("witnesses"))
                lib().orc_raft_set  # node id is fixed at creation in the oracle
                if p.node_id != id:
                    raise ValueError("Raft passed to Network must be created with node id %d" % id)
                p.clear_remotes("remotes")
                p.clear_remotes("observers")
                p.clear_remotes("witnesses")
                for pid in ids:
                    if pid in obs:
                        p.set_remote("observers", pid)
                    elif pid in wit:
                        p.set_remote("witnesses", pid)
                    else:
                        p.set_remote("remotes", pid)
                p.reset(p.term)
                self.peers[id] = p
            else:
                self.peers[id] = p

    def send(self, *msgs: Message):
        q = list(msgs)
        while q:
            m = q.pop(0)
            p = self.peers[m.to]
            p.handle(m)
            q.extend(self.filter(p.read_messages()))

    def drop(self, frm, to, perc):
        self.dropm[(frm, to)] = perc

    def cut(self, one, other):
        self.drop(one, other, 1.0)
        self.drop(other, one, 1.0)

    def isolate(self, id):
        for i in range(len(self.peers)):
            nid = i + 1
            if nid != id:
                self.drop(id, nid, 1.0)
                self.drop(nid, id, 1.0)

    def ignore(self, t):
        self.ignorem.add(t)

    def recover(self):
        self.dropm = {}
        self.ignorem = set()

    def filter(self, msgs):
        out = []
        for m in msgs:
            if m.type in self.ignorem:
                continue
            if m.type == Election:
                raise AssertionError("unexpected msgHup")
            perc = self.dropm.get((m.from_, m.to), 0.0)
            if perc >= 1.0:
                continue
            assert perc == 0.0, "fractional drop rates are not deterministic"
            out.append(m)
        return out


# ----------------------------------------------------------------- Peer
class Peer:
    """Peer API (peer.go:58-358)."""

    def __init__(self, node_id, peers, election=10, heartbeat=1, logdb=None, initial=True,
                 new_node=True, check_quorum=False, seed=0x5EEDD8A6, cluster_id=1):
        self.logdb = logdb or LogDB()
        cfg = OrcConfig(node_id=node_id, cluster_id=cluster_id, election=election,
                        heartbeat=heartbeat, seed=seed, check_quorum=int(check_quorum))
        ids = (C.c_uint64 * max(1, len(peers)))(*peers)
        self.h = lib().orc_peer_launch(C.byref(cfg), self.logdb.h, ids, len(peers),
                                       int(initial), int(new_node))
        if not self.h:
            raise _err()
        self.raft = Raft(lib().orc_peer_raft(self.h), self.logdb, owned=False)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_peer_free(self.h)
            self.h = None

    def tick(self):
        lib().orc_peer_tick(self.h, 0)

    def quiesced_tick(self):
        lib().orc_peer_tick(self.h, 1)

    def handle(self, m: Message):
        cm, keep = m.to_c()
        if lib().orc_peer_handle(self.h, C.byref(cm)) != 0:
            raise _err()

    def propose_entries(self, ents: List[Entry]):
        arr = entries_array(ents)
        if lib().orc_peer_propose(self.h, arr, len(ents)) != 0:
            raise _err()

    def read_index(self, ctx):
        if lib().orc_peer_read_index(self.h, ctx[0], ctx[1]) != 0:
            raise _err()

    def request_leader_transfer(self, target):
        lib().orc_peer_misc(self.h, 0, target, 0)

    def apply_config_change(self, node_id, cc_type):
        if lib().orc_peer_misc(self.h, 1, node_id, cc_type) < 0:
            raise _err()

    def reject_config_change(self):
        lib().orc_peer_misc(self.h, 2, 0, 0)

    def report_unreachable_node(self, nid):
        lib().orc_peer_misc(self.h, 3, nid, 0)

    def report_snapshot_status(self, nid, reject):
        lib().orc_peer_misc(self.h, 4, nid, int(reject))

    def notify_raft_last_applied(self, v):
        lib().orc_peer_misc(self.h, 5, v, 0)

    def has_entry_to_apply(self):
        return bool(lib().orc_peer_misc(self.h, 6, 0, 0))

    def has_update(self, more_to_apply):
        return bool(lib().orc_peer_misc(self.h, 7, int(more_to_apply), 0))

    def propose_config_change(self, node_id, cc_type, key):
        if lib().orc_peer_propose_cc(self.h, node_id, cc_type, key) != 0:
            raise _err()

    def get_update(self, more_to_apply=True, last_applied=0) -> dict:
        info = (C.c_uint64 * 19)()
        if lib().orc_peer_get_update(self.h, int(more_to_apply), last_applied, info) != 0:
            raise _err()
        keys = ["term", "vote", "commit", "fast_apply", "n_entries_to_save",
                "n_committed_entries", "more_committed_entries", "n_ready_to_reads",
                "n_messages", "last_applied", "uc_processed", "uc_last_applied",
                "uc_stable_log_to", "uc_stable_log_term", "uc_stable_snapshot_to",
                "uc_ready_to_read", "n_dropped_entries", "n_dropped_read_indexes",
                "snapshot_index"]
        ud = dict(zip(keys, list(info)))

        def fetch(which, n):
            out = (OrcEntry * max(1, n))()
            lib().orc_peer_update_entries(self.h, which, out, n)
            return [Entry.from_c(out[i]) for i in range(n)]
        ud["entries_to_save"] = fetch(0, ud["n_entries_to_save"])
        ud["committed_entries"] = fetch(1, ud["n_committed_entries"])
        ud["dropped_entries"] = fetch(2, ud["n_dropped_entries"])
        n = ud["n_messages"]
        out = (OrcMsg * max(1, n))()
        eb = (OrcEntry * 4096)()
        k = lib().orc_peer_update_messages(self.h, out, n, eb, 4096)
        ud["messages"] = [Message.from_c(out[i]) for i in range(k)]
        o = (C.c_uint64 * (3 * 256))()
        k = lib().orc_peer_update_rtr(self.h, o, 256)
        ud["ready_to_reads"] = [(o[3 * i], o[3 * i + 1], o[3 * i + 2]) for i in range(k)]
        return ud

    def set_update_commit(self, processed=0, last_applied=0, stable_log_to=0,
                          stable_log_term=0, stable_snapshot_to=0, ready_to_read=0):
        arr = (C.c_uint64 * 6)(processed, last_applied, stable_log_to, stable_log_term,
                               stable_snapshot_to, ready_to_read)
        lib().orc_peer_update_set_commit(self.h, arr)

    def commit(self):
        if lib().orc_peer_commit(self.h) != 0:
            raise _err()


# ----------------------------------------------------------------- Harness
HC_NAMES = ["steps", "committed", "msg_in", "msg_out", "ent_in", "ent_out", "reads_confirmed",
            "proposals", "reads", "quiesced_ticks", "active_ticks", "campaigns", "ent_saved",
            "ent_applied", "msg_dropped", "dropped_proposals", "dropped_reads", "leader_steps"]
HC_NUM = 24


class Harness:
    """Deterministic lockstep multi-group harness (oracle/harness.h)."""

    def __init__(self, n_groups=1, n_replicas=3, cid_base=1, election_rtt=10, heartbeat_rtt=1,
                 check_quorum=False, quiesce=False, seed=0x5EEDD8A6, max_entry_size=0,
                 wl_enabled=False, wl_start_round=0, wl_stop_round=0, wl_active_mod=1,
                 wl_read_permille=0, iso_period=0, iso_len=0, iso_mod=10, trace=True,
                 threads=1, cid_stride=1, xfer_period=0, xfer_mod=1, ext_apply=False,
                 ext_inputs=False, snapshot_entries=0, compaction_overhead=0,
                 ext_commit=False, membership=False, cc_period=0, cc_mod=1,
                 max_inmem_log_size=0, n_voters=0, observer_slots=0, witness_slots=0):
        c = OrcHarnessConfig(
            n_groups=n_groups, n_replicas=n_replicas, check_quorum=int(check_quorum),
            cid_base=cid_base, election_rtt=election_rtt, heartbeat_rtt=heartbeat_rtt,
            seed=seed, max_entry_size=max_entry_size, quiesce=int(quiesce),
            wl_enabled=int(wl_enabled), wl_start_round=wl_start_round,
            wl_stop_round=wl_stop_round, wl_active_mod=wl_active_mod,
            wl_read_permille=wl_read_permille, iso_period=iso_period, iso_len=iso_len,
            iso_mod=iso_mod, trace=int(trace), threads=threads, cid_stride=cid_stride,
            xfer_period=xfer_period, xfer_mod=xfer_mod, ext_apply=int(ext_apply),
            snapshot_entries=snapshot_entries, compaction_overhead=compaction_overhead,
            ext_commit=int(ext_commit), membership=int(membership), cc_period=cc_period,
            cc_mod=cc_mod, max_inmem_log_size=max_inmem_log_size, n_voters=n_voters,
            observer_slots=observer_slots, witness_slots=witness_slots)
        self.n_groups, self.n_replicas = n_groups, n_replicas
        self.h = lib().orc_harness_create(C.byref(c))
        if not self.h:
            raise _err()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_harness_destroy(self.h)
            self.h = None

    def run(self, rounds=1):
        if lib().orc_harness_run(self.h, rounds) != 0:
            raise _err()

    def step(self, tick=True):
        """One round; tick=False is rbe_step_ex(RBE_STEP_NO_TICK)."""
        if lib().orc_harness_step(self.h, int(tick)) != 0:
            raise _err()

    def push(self, kind, replica, a=0, b=0, entries=()):
        """Stage host input for the next round (the engine's rbe_push_* calls)."""
        arr = entries_array(list(entries))
        if lib().orc_harness_push(self.h, kind, replica, a, b, arr, len(entries)) != 0:
            raise _err()

    @property
    def round(self):
        return lib().orc_harness_round(self.h)

    def views(self):
        n = self.n_groups * self.n_replicas
        arr = (ReplicaView * n)()
        lib().orc_harness_views(self.h, C.cast(arr, C.c_void_p))
        return arr

    def rate_limited(self):
        """(Peer.RateLimited per replica as numpy bool, rl.Get() as uint64)."""
        import numpy as np
        n = self.n_groups * self.n_replicas
        lim = np.zeros(max(1, n), np.uint8)
        size = np.zeros(max(1, n), np.uint64)
        lib().orc_harness_rate_limited(self.h, C.c_void_p(lim.ctypes.data),
                                       C.c_void_p(size.ctypes.data))
        return lim[:n].astype(bool), size[:n]

    def counters(self) -> Dict[str, int]:
        o = (C.c_uint64 * HC_NUM)()
        lib().orc_harness_counters(self.h, o)
        return {n: o[i] for i, n in enumerate(HC_NAMES)}

    def log_term(self, g, k, index):
        return lib().orc_harness_log_term(self.h, g, k, index)

    def persisted(self, replica):
        """(term, vote, commit, last_index) of a replica's LogDB."""
        o = (C.c_uint64 * 4)()
        lib().orc_harness_persisted(self.h, replica, o)
        return tuple(o)

    def snapshot_state(self, replica):
        """(marker, marker_term, ss_index, ss_term, ss_req, compact_to, ss_removed,
        sm_removed): the LogDB's compaction marker and snapshot, the node's
        snapshot request, the snapshot's membership and the state machine's
        (bit k: node k + 1 is not a voter)."""
        o = (C.c_uint64 * 8)()
        lib().orc_harness_snapshot_state(self.h, replica, o)
        return tuple(o)

    def persisted_entries(self, replica, lo, hi):
        arr = (OrcEntry * max(1, hi - lo + 1))()
        if lib().orc_harness_persisted_entries(self.h, replica, lo, hi, arr) != 0:
            raise _err()
        return [Entry.from_c(arr[i]) for i in range(hi - lo + 1)]

    def update_commit(self, replica):
        """ext_commit: getUpdateCommit of the replica's last step (peer.go:410-427)
        as (processed, last_applied, stable_log_to, stable_log_term,
        stable_snapshot_to, ready_to_read); zeros when it made no Update."""
        o = (C.c_uint64 * 6)()
        lib().orc_harness_update_commit(self.h, replica, o)
        return tuple(o)

    def replace(self, replica):
        """A fresh node joins in the replica's slot (rbe_replace_node); False
        while the group still refers to the slot's node."""
        rc = lib().orc_harness_replace(self.h, replica)
        if rc == -2:
            raise _err()
        return rc == 0

    def update_snapshot(self, replica):
        """The Snapshot of the replica's last Update (peer.go:345-347): (index,
        term, packed membership, 0); zeros when it carried none."""
        o = (C.c_uint64 * 4)()
        lib().orc_harness_update_snapshot(self.h, replica, o)
        return tuple(o)

    def commit(self, replica, uc):
        """ext_commit: Peer.Commit's log part with a host-chosen UpdateCommit
        (entryLog.commitUpdate, logentry.go:335-355); raises where it panics."""
        a = (C.c_uint64 * 6)(*uc)
        if lib().orc_harness_commit(self.h, replica, a) != 0:
            raise _err()

    def inbox(self, replica, sender):
        """Debugging: the messages `replica` receives from slot `sender` next
        round, as (type, from, to, term, log_term, log_index, commit, reject,
        hint, n_entries) tuples."""
        o = (C.c_uint64 * 640)()
        n = lib().orc_harness_inbox(self.h, replica, sender, o, 64)
        return [tuple(o[10 * i:10 * i + 10]) for i in range(min(n, 64))]

    def snapshot_saved(self, replica, index, term, removed=0):
        """ext_apply: the host's snapshot worker saved a snapshot and the LogDB
        took it (the engine's rbe_snapshot_saved)."""
        if lib().orc_harness_snapshot_saved(self.h, replica, index, term, removed) != 0:
            raise _err()

    def compact(self, replica, to):
        """ext_apply: compactLogTo for the replica's next step (rbe_compact)."""
        if lib().orc_harness_compact(self.h, replica, to) != 0:
            raise _err()

    def restart(self, replica):
        """Restart a replica from its LogDB (the engine's rbe_launch)."""
        if lib().orc_harness_restart(self.h, replica) != 0:
            raise _err()
