"""ctypes binding to libdragonboat_amd.so (include/rbe.h).

This is the product path: every call goes to the HIP engine on an MI355X.
There is no CPU fallback; if the library or a gfx950 device is missing,
`Engine(...)` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libdragonboat_amd.so")
RBE_ABI_VERSION = 9

COUNTER_NAMES = ["steps", "committed", "msg_in", "msg_out", "ent_in", "ent_out",
                 "reads_confirmed", "proposals", "reads", "quiesced_ticks", "active_ticks",
                 "campaigns", "ent_saved", "ent_applied", "msg_dropped", "dropped_proposals",
                 "dropped_reads", "leader_steps", "remote_touch", "ring_access", "faults",
                 "rq_touch"]
CTR_NUM = 24

FAULT_NAMES = {0x01: "WINDOW", 0x02: "OUTBOX", 0x04: "ARENA", 0x08: "READQ", 0x10: "RTR",
               0x20: "PANIC", 0x40: "UNSUPPORTED", 0x80: "DROPLIST", 0x100: "NOMEM"}


class RbeConfig(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("device", C.c_int32), ("n_groups", C.c_uint64),
                ("n_replicas", C.c_uint32), ("election_rtt", C.c_uint32),
                ("heartbeat_rtt", C.c_uint32), ("check_quorum", C.c_uint32),
                ("quiesce", C.c_uint32), ("ring", C.c_uint32), ("rq_cap", C.c_uint32),
                ("maxm", C.c_uint32), ("ecap", C.c_uint32), ("rtr_cap", C.c_uint32),
                ("dri_cap", C.c_uint32), ("trace", C.c_uint32), ("cid_base", C.c_uint64),
                ("cid_stride", C.c_uint64), ("seed", C.c_uint64),
                ("max_entry_size", C.c_uint64), ("wl_enabled", C.c_uint32),
                ("wl_start_round", C.c_uint32), ("wl_stop_round", C.c_uint32),
                ("wl_active_mod", C.c_uint32), ("wl_read_permille", C.c_uint32),
                ("ext_inputs", C.c_uint32), ("iso_period", C.c_uint32),
                ("iso_len", C.c_uint32), ("iso_mod", C.c_uint32),
                ("rep_world", C.c_uint32), ("rep_rank", C.c_uint32),
                ("ext_apply", C.c_uint32), ("in_cap", C.c_uint32),
                ("xfer_period", C.c_uint32), ("xfer_mod", C.c_uint32),
                ("snapshot_entries", C.c_uint32), ("compaction_overhead", C.c_uint32),
                ("heap_bytes", C.c_uint64), ("ext_commit", C.c_uint32),
                ("membership", C.c_uint32), ("cc_period", C.c_uint32), ("cc_mod", C.c_uint32),
                ("rep_compact", C.c_uint32), ("n_voters", C.c_uint32),
                ("max_inmem_log_size", C.c_uint64), ("observer_slots", C.c_uint32),
                ("witness_slots", C.c_uint32), ("pool_bytes", C.c_uint64),
                ("spill_bytes", C.c_uint64)]


class RbeReplicaView(C.Structure):
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


def _np_dtype(struct):
    names, formats, offsets = [], [], []
    for name, t in struct._fields_:
        names.append(name)
        base = getattr(t, "_type_", t)
        n = getattr(t, "_length_", None)
        code = np.dtype(base)
        formats.append((code, (n,)) if n else code)
        offsets.append(getattr(struct, name).offset)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets,
                     "itemsize": C.sizeof(struct)})


VIEW_DTYPE = _np_dtype(RbeReplicaView)


class RbeUpdate(C.Structure):
    _fields_ = [("term", C.c_uint64), ("vote", C.c_uint64), ("commit", C.c_uint64),
                ("save_lo", C.c_uint64), ("save_hi", C.c_uint64), ("apply_lo", C.c_uint64),
                ("apply_hi", C.c_uint64), ("digest", C.c_uint64),
                ("n_messages", C.c_uint32), ("n_ready_to_read", C.c_uint32),
                ("n_dropped_entries", C.c_uint32), ("n_dropped_read_indexes", C.c_uint32),
                ("fault", C.c_uint32), ("flags", C.c_uint32), ("role", C.c_uint32),
                ("events", C.c_uint32), ("leader_id", C.c_uint64)]


# Update flags and listener events (include/rbe.h RBE_UF_* / RBE_EV_*)
UF_STATE_CHANGED, UF_SENT_QUIESCE, UF_FAST_APPLY, UF_HAS_UPDATE, UF_SNAPSHOT = 1, 2, 8, 16, 32
UF_APPLIED = 64
EV_LEADER_UPDATED, EV_CAMPAIGN_LAUNCHED, EV_CAMPAIGN_SKIPPED, EV_SNAPSHOT_REJECTED = 1, 2, 4, 8
EV_REPLICATION_REJECTED, EV_PROPOSAL_DROPPED, EV_READ_INDEX_DROPPED = 16, 32, 64


class RbeMessage(C.Structure):
    _fields_ = [("type", C.c_uint32), ("reject", C.c_uint32), ("to", C.c_uint64),
                ("from_", C.c_uint64), ("cluster_id", C.c_uint64), ("term", C.c_uint64),
                ("log_term", C.c_uint64), ("log_index", C.c_uint64), ("commit", C.c_uint64),
                ("hint", C.c_uint64), ("hint_high", C.c_uint64), ("n_entries", C.c_uint32),
                ("reserved", C.c_uint32)]


class RbeEntry(C.Structure):
    """raftpb.Entry (raft.pb.go:589-598); cmd holds the first 16 Cmd bytes."""
    _fields_ = [("index", C.c_uint64), ("term", C.c_uint64), ("type", C.c_uint32),
                ("cmd_len", C.c_uint32), ("cmd", C.c_uint8 * 16), ("key", C.c_uint64),
                ("client_id", C.c_uint64), ("series_id", C.c_uint64),
                ("responded_to", C.c_uint64)]


SESSION_FIELDS = ("key", "client_id", "series_id", "responded_to")


def make_entry(index=0, term=0, type=0, cmd=b"", key=0, client_id=0, series_id=0,
               responded_to=0) -> RbeEntry:
    e = RbeEntry(index=index, term=term, type=type, cmd_len=len(cmd), key=key,
                 client_id=client_id, series_id=series_id, responded_to=responded_to)
    for b, x in enumerate(cmd[:16]):
        e.cmd[b] = x
    return e


def entry_fields(e: RbeEntry, cmd: Optional[bytes] = None) -> dict:
    """An RbeEntry as a dict of raftpb.Entry fields (cmd: the whole Cmd when given)."""
    return dict(index=e.index, term=e.term, type=e.type,
                cmd=cmd if cmd is not None else bytes(e.cmd[:min(16, e.cmd_len)]),
                key=e.key, client_id=e.client_id, series_id=e.series_id,
                responded_to=e.responded_to)


class RbeUpdateCommit(C.Structure):  # raftpb UpdateCommit (raftpb/raft.go:60-70)
    _fields_ = [("processed", C.c_uint64), ("last_applied", C.c_uint64),
                ("stable_log_to", C.c_uint64), ("stable_log_term", C.c_uint64),
                ("stable_snapshot_to", C.c_uint64), ("ready_to_read", C.c_uint64)]


class RbeReadyToRead(C.Structure):
    _fields_ = [("index", C.c_uint64), ("ctx_low", C.c_uint64), ("ctx_high", C.c_uint64)]


class RbeLaunchState(C.Structure):
    _fields_ = [("term", C.c_uint64), ("vote", C.c_uint64), ("commit", C.c_uint64),
                ("last_index", C.c_uint64), ("n_entries", C.c_uint32), ("removed", C.c_uint32),
                ("marker", C.c_uint64), ("marker_term", C.c_uint64),
                ("snapshot_index", C.c_uint64), ("snapshot_term", C.c_uint64)]


class RbeOutputs(C.Structure):
    _fields_ = [("first", C.c_uint64), ("count", C.c_uint64), ("n_messages", C.c_uint64),
                ("n_ready_to_reads", C.c_uint64), ("msg_off", C.POINTER(C.c_uint64)),
                ("messages", C.POINTER(RbeMessage)), ("rtr_off", C.POINTER(C.c_uint64)),
                ("ready_to_reads", C.POINTER(RbeReadyToRead))]


class RbeStepOutputs(C.Structure):
    _fields_ = [("first", C.c_uint64), ("count", C.c_uint64), ("n", C.c_uint64),
                ("n_messages", C.c_uint64), ("n_ready_to_reads", C.c_uint64),
                ("replica", C.POINTER(C.c_uint64)), ("updates", C.POINTER(RbeUpdate)),
                ("msg_off", C.POINTER(C.c_uint64)), ("messages", C.POINTER(RbeMessage)),
                ("rtr_off", C.POINTER(C.c_uint64)),
                ("ready_to_reads", C.POINTER(RbeReadyToRead))]


RBE_COLLECT_REMOTE_MSGS = 1
RBE_COLLECT_SKIP_LOCAL = 2


class RbeWireFrame(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("bytes", C.c_uint64), ("first_group", C.c_uint64),
                ("src", C.c_uint32), ("dst", C.c_uint32), ("n_messages", C.c_uint32),
                ("n_groups", C.c_uint32)]


class RbeWireConfig(C.Structure):
    _fields_ = [("deployment_id", C.c_uint64), ("bin_ver", C.c_uint32),
                ("groups_per_batch", C.c_uint32), ("source_address", C.c_char_p * 7),
                ("dst_rank", C.c_int32), ("pad", C.c_uint32)]


class RbeWireIngestStats(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("frames", "messages", "dropped", "entries",
                                          "cmd_bytes", "heap_bytes")]


def wire_config(deployment_id=0, bin_ver=0, groups_per_batch=0, source_address=(), dst_rank=-1):
    wc = RbeWireConfig(deployment_id=deployment_id, bin_ver=bin_ver,
                       groups_per_batch=groups_per_batch, dst_rank=dst_rank)
    for i, a in enumerate(source_address):
        wc.source_address[i] = a.encode()
    return wc


class RbeUpdateList(C.Structure):
    _fields_ = [("first", C.c_uint64), ("count", C.c_uint64), ("n", C.c_uint64),
                ("replica", C.POINTER(C.c_uint64)), ("updates", C.POINTER(RbeUpdate))]


MESSAGE_DTYPE = _np_dtype(RbeMessage)
UPDATE_DTYPE = _np_dtype(RbeUpdate)
RTR_DTYPE = _np_dtype(RbeReadyToRead)


# exported symbols of include/rbe.h (checked by tests/test_capi.py)
EXPORTS = ["rbe_create", "rbe_destroy", "rbe_abi_version", "rbe_abi_sizes", "rbe_step", "rbe_step_ex", "rbe_run",
           "rbe_sync", "rbe_request_leader_transfer", "rbe_report_unreachable",
           "rbe_report_snapshot_status", "rbe_notify_applied",
           "rbe_round", "rbe_run_timed", "rbe_prepare_run", "rbe_push_proposals", "rbe_push_read_index",
           "rbe_get_updates", "rbe_get_messages", "rbe_get_ready_to_reads", "rbe_get_entries",
           "rbe_get_views", "rbe_get_counters", "rbe_reset_counters", "rbe_fault_summary",
           "rbe_spill_stats",
           "rbe_footprint", "rbe_profile_rounds", "rbe_get_kernel_counters", "rbe_kernel_name",
           "rbe_xchg_record_bytes", "rbe_xchg_pack", "rbe_xchg_unpack", "rbe_get_outbox",
           "rbe_push_messages", "rbe_snapshot_bytes", "rbe_export_bytes", "rbe_export_groups", "rbe_import_groups",
           "rbe_get_entry_cmds", "rbe_set_apply_ready", "rbe_collect_outputs", "rbe_collect_updates", "rbe_launch",
           "rbe_xchg_chunk_bytes", "rbe_xchg_pack_fixed", "rbe_xchg_unpack_fixed",
           "rbe_xchg_status", "rbe_stream", "rbe_get_snapshot_state", "rbe_wire_encode",
           "rbe_wire_fetch", "rbe_wire_decode", "rbe_wire_ingest", "rbe_iso_leaders", "rbe_set_iso_leaders", "rbe_local_groups", "rbe_propose_entries", "rbe_commit",
           "rbe_get_update_commits", "rbe_get_update_snapshots", "rbe_replace_node", "rbe_propose_config_change", "rbe_apply_config_change",
           "rbe_reject_config_change", "rbe_rate_limited", "rbe_restore_remotes",
           "rbe_snapshot_saved", "rbe_compact", "rbe_set_node_ids", "rbe_collect_step",
           "rbe_collect_step_begin", "rbe_collect_step_end"]
KERNEL_SLOTS = 4

_lib = None


RBE_E_INVALID, RBE_E_NOMEM, RBE_E_STATE, RBE_E_CORRUPT = -1, -3, -5, -6
RBE_STEP_NO_TICK = 1


class EngineError(RuntimeError):
    pass


def load_library(path: Optional[str] = None):
    """Load libdragonboat_amd.so; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # RBE_LIB: an alternative build of the same ABI (A/B experiments, diagnostics)
    p = path or os.environ.get("RBE_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise EngineError(
            f"{p} is missing: the HIP engine is the only implementation; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(p)
    P = C.POINTER
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    sig = {
        "rbe_create": (i32, [P(RbeConfig), P(vp)]),
        "rbe_destroy": (i32, [vp]),
        "rbe_abi_version": (i32, []),
        "rbe_abi_sizes": (i32, [P(u64), u32]),
        "rbe_step": (i32, [vp]),
        "rbe_step_ex": (i32, [vp, u32]),
        "rbe_request_leader_transfer": (i32, [vp, u64, P(u64), P(u64)]),
        "rbe_report_unreachable": (i32, [vp, u64, P(u64), P(u64)]),
        "rbe_report_snapshot_status": (i32, [vp, u64, P(u64), P(u64), P(C.c_uint8)]),
        "rbe_notify_applied": (i32, [vp, u64, P(u64), P(u64)]),
        "rbe_set_apply_ready": (i32, [vp, u64, P(u64), P(C.c_uint8)]),
        "rbe_commit": (i32, [vp, u64, P(u64), P(RbeUpdateCommit)]),
        "rbe_propose_config_change": (i32, [vp, u64, P(u64), P(u32), P(u64)]),
        "rbe_apply_config_change": (i32, [vp, u64, P(u64), P(u64), P(u32)]),
        "rbe_reject_config_change": (i32, [vp, u64, P(u64)]),
        "rbe_restore_remotes": (i32, [vp, u64, P(u64), P(u32), P(u64)]),
        "rbe_snapshot_saved": (i32, [vp, u64, P(u64), P(u64), P(u64), P(u32)]),
        "rbe_compact": (i32, [vp, u64, P(u64), P(u64)]),
        "rbe_set_node_ids": (i32, [vp, u64, u64, P(u64)]),
        "rbe_replace_node": (i32, [vp, u64, P(u64), P(u64)]),
        "rbe_get_update_commits": (i32, [vp, u64, u64, P(RbeUpdateCommit)]),
        "rbe_get_update_snapshots": (i32, [vp, u64, u64, P(u64)]),
        "rbe_run": (i32, [vp, u32]),
        "rbe_sync": (i32, [vp]),
        "rbe_round": (i32, [vp, P(u32)]),
        "rbe_run_timed": (i32, [vp, u32, P(C.c_float)]),
        "rbe_prepare_run": (i32, [vp, u32]),
        "rbe_push_proposals": (i32, [vp, u64, P(u64), P(u32), P(u32), P(u32), P(C.c_uint8)]),
        "rbe_propose_entries": (i32, [vp, u64, P(u64), P(u32), P(RbeEntry), P(C.c_uint8)]),
        "rbe_push_read_index": (i32, [vp, u64, P(u64), P(u64), P(u64)]),
        "rbe_get_updates": (i32, [vp, u64, u64, P(RbeUpdate)]),
        "rbe_collect_updates": (i32, [vp, u64, u64, P(RbeUpdateList)]),
        "rbe_collect_step": (i32, [vp, u64, u64, u32, P(RbeStepOutputs)]),
        "rbe_collect_step_begin": (i32, [vp, u64, u64, u32]),
        "rbe_collect_step_end": (i32, [vp, P(RbeStepOutputs)]),
        "rbe_get_messages": (i32, [vp, u64, P(RbeMessage), u32, P(u32)]),
        "rbe_get_outbox": (i32, [vp, u64, P(RbeMessage), u32, P(u32), P(RbeEntry), u32, P(u32),
                                 vp, u64, P(u64)]),
        "rbe_push_messages": (i32, [vp, u64, P(u64), P(RbeMessage), P(RbeEntry), vp]),
        "rbe_get_ready_to_reads": (i32, [vp, u64, P(RbeReadyToRead), u32, P(u32)]),
        "rbe_get_entries": (i32, [vp, u64, u64, u64, P(RbeEntry)]),
        "rbe_get_entry_cmds": (i32, [vp, u64, u64, u64, vp, u64, P(u64)]),
        "rbe_get_views": (i32, [vp, u64, u64, P(RbeReplicaView)]),
        "rbe_rate_limited": (i32, [vp, u64, u64, vp, vp]),
        "rbe_get_snapshot_state": (i32, [vp, u64, u64, P(u64)]),
        "rbe_wire_encode": (i32, [vp, P(RbeWireConfig), P(u64)]),
        "rbe_wire_fetch": (i32, [vp, vp, u64, P(RbeWireFrame), u32]),
        "rbe_wire_ingest": (i32, [vp, vp, u64, P(RbeWireIngestStats)]),
        "rbe_iso_leaders": (i32, [vp, vp, P(u32)]),
        "rbe_set_iso_leaders": (i32, [vp, vp]),
        "rbe_local_groups": (i32, [vp, P(u64), vp]),
        "rbe_wire_decode": (i32, [vp, vp, u64, P(RbeMessage), u32, P(u32), P(RbeEntry), u32,
                                  P(u32), vp, u64, P(u64)]),
        "rbe_collect_outputs": (i32, [vp, u64, u64, P(RbeOutputs)]),
        "rbe_launch": (i32, [vp, u64, P(u64), P(RbeLaunchState), P(RbeEntry), vp]),
        "rbe_get_counters": (i32, [vp, P(u64)]),
        "rbe_reset_counters": (i32, [vp]),
        "rbe_fault_summary": (i32, [vp, P(u64), P(u32)]),
        "rbe_spill_stats": (i32, [vp, P(u64)]),
        "rbe_footprint": (i32, [P(RbeConfig), P(u64)]),
        "rbe_profile_rounds": (i32, [vp, u32, P(C.c_float)]),
        "rbe_get_kernel_counters": (i32, [vp, C.c_int32, P(u64)]),
        "rbe_kernel_name": (i32, [vp, C.c_int32, C.c_char_p, u32]),
        "rbe_xchg_record_bytes": (i32, [P(u64)]),
        "rbe_xchg_pack": (i32, [vp, vp, P(u64), P(u32)]),
        "rbe_xchg_unpack": (i32, [vp, vp, u64, vp, u64, vp, u64]),
        "rbe_xchg_chunk_bytes": (i32, [P(u64), P(u64)]),
        "rbe_xchg_pack_fixed": (i32, [vp, vp, P(u64)]),
        "rbe_xchg_unpack_fixed": (i32, [vp, vp, P(u64)]),
        "rbe_xchg_status": (i32, [vp, P(u32)]),
        "rbe_stream": (i32, [vp, P(vp)]),
        "rbe_snapshot_bytes": (i32, [vp, u64, P(u64)]),
        "rbe_export_bytes": (i32, [vp, u64, u64, P(u64)]),
        "rbe_export_groups": (i32, [vp, u64, u64, vp, u64]),
        "rbe_import_groups": (i32, [vp, vp, u64, u32]),
    }
    ab = path is None and os.environ.get("RBE_LIB")  # an older A/B build may lack newer calls
    for name, (res, args) in sig.items():
        if ab and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.rbe_abi_version() != RBE_ABI_VERSION:
        raise EngineError("ABI version mismatch")
    sz = (C.c_uint64 * 6)()
    mine = [C.sizeof(t) for t in (RbeConfig, RbeReplicaView, RbeUpdate, RbeMessage, RbeEntry,
                                  RbeReadyToRead)]
    if L.rbe_abi_sizes(sz, 6) != 6 or list(sz) != mine:
        raise EngineError(f"ABI struct sizes differ: library {list(sz)}, binding {mine}")
    if path is None:
        _lib = L
    return L


def make_config(n_groups: int, n_replicas: int = 3, device: int = 0, election_rtt: int = 10,
                heartbeat_rtt: int = 1, check_quorum: bool = False, quiesce: bool = False,
                ring: int = 0, rq_cap: int = 0, maxm: int = 0, ecap: int = 0, rtr_cap: int = 0,
                dri_cap: int = 0, trace: bool = False, cid_base: int = 1, cid_stride: int = 1,
                seed: int = 0x5EEDD8A6, max_entry_size: int = 0, wl_enabled: bool = False,
                wl_start_round: int = 0, wl_stop_round: int = 0, wl_active_mod: int = 1,
                wl_read_permille: int = 0, ext_inputs: bool = False, iso_period: int = 0,
                iso_len: int = 0, iso_mod: int = 10, rep_world: int = 0,
                rep_rank: int = 0, ext_apply: bool = False, in_cap: int = 0,
                xfer_period: int = 0, xfer_mod: int = 1, heap_bytes: int = 0,
                snapshot_entries: int = 0, compaction_overhead: int = 0,
                ext_commit: bool = False, membership: bool = False, cc_period: int = 0,
                cc_mod: int = 1, rep_compact: bool = False,
                max_inmem_log_size: int = 0, n_voters: int = 0, observer_slots: int = 0,
                witness_slots: int = 0, pool_bytes: int = 0, spill_bytes: int = 0) -> RbeConfig:
    return RbeConfig(abi_version=RBE_ABI_VERSION, device=device, n_groups=n_groups,
                     n_replicas=n_replicas, election_rtt=election_rtt,
                     heartbeat_rtt=heartbeat_rtt, check_quorum=int(check_quorum),
                     quiesce=int(quiesce), ring=ring, rq_cap=rq_cap, maxm=maxm, ecap=ecap,
                     rtr_cap=rtr_cap, dri_cap=dri_cap, trace=int(trace), cid_base=cid_base,
                     cid_stride=cid_stride, seed=seed, max_entry_size=max_entry_size,
                     wl_enabled=int(wl_enabled), wl_start_round=wl_start_round,
                     wl_stop_round=wl_stop_round, wl_active_mod=wl_active_mod,
                     wl_read_permille=wl_read_permille, ext_inputs=int(ext_inputs),
                     iso_period=iso_period, iso_len=iso_len, iso_mod=iso_mod,
                     rep_world=rep_world, rep_rank=rep_rank, ext_apply=int(ext_apply),
                     in_cap=in_cap, xfer_period=xfer_period, xfer_mod=xfer_mod,
                     heap_bytes=heap_bytes, snapshot_entries=snapshot_entries,
                     compaction_overhead=compaction_overhead, ext_commit=int(ext_commit),
                     membership=int(membership), cc_period=cc_period, cc_mod=cc_mod,
                     rep_compact=int(rep_compact), max_inmem_log_size=max_inmem_log_size,
                     n_voters=n_voters, observer_slots=observer_slots,
                     witness_slots=witness_slots, pool_bytes=pool_bytes,
                     spill_bytes=spill_bytes)


class InputError(EngineError):
    """An rbe_push_* / rbe_request_* / rbe_report_* / rbe_notify_applied call
    refused its batch (nothing of it was staged)."""

    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} refused the batch (rc={rc})")
        self.rc = rc


def _u64s(v):
    n = len(v)
    return (C.c_uint64 * max(1, n))(*v)


def _check_input(rc: int, what: str):
    if rc != 0:
        raise InputError(rc, what)


class SnapshotError(EngineError):
    def __init__(self, rc: int, what: str):
        super().__init__(f"{what} failed with rc={rc}")
        self.rc = rc


def _check(rc: int, what: str):
    if rc != 0:
        raise EngineError(f"{what} failed with rc={rc}")


def global_groups_call(fn, h, n_groups: int):
    out = np.zeros(max(1, n_groups), np.uint64)
    n = C.c_uint64()
    _check(fn(h, C.byref(n), out.ctypes.data), "rbe_local_groups")
    return out[:n.value]


def rate_limited_call(fn, h, n_rep: int):
    """rbe_rate_limited (or the host build's twin) over replicas [0, n_rep)."""
    lim = np.zeros(max(1, n_rep), np.uint8)
    size = np.zeros(max(1, n_rep), np.uint64)
    _check(fn(h, 0, n_rep, lim.ctypes.data, size.ctypes.data), "rbe_rate_limited")
    return lim[:n_rep].astype(bool), size[:n_rep]


def iso_leaders_call(fn, h, n_groups: int):
    """rbe_iso_leaders (or the host build's twin): None off-epoch, else the
    leader bits per group."""
    ep = C.c_uint32()
    _check(fn(h, None, C.byref(ep)), "rbe_iso_leaders")
    if not ep.value:
        return None
    out = np.zeros(n_groups, np.uint8)
    _check(fn(h, out.ctypes.data, C.byref(ep)), "rbe_iso_leaders")
    return out


def wire_ingest_call(fn, h, data: bytes) -> dict:
    """rbe_wire_ingest (or the host build's twin): the stats as a dict;
    raises InputError with the return code on a refused batch."""
    st = RbeWireIngestStats()
    _check_input(fn(h, data, len(data), C.byref(st)), "rbe_wire_ingest")
    return {f: getattr(st, f) for f, _ in RbeWireIngestStats._fields_}


def entry_cmds(fn, h, replica: int, lo: int, hi: int) -> List[bytes]:
    """Cmd bytes of entries [lo, hi] through rbe_get_entry_cmds (or the host
    build's twin): one call to size the buffer, one to fill it."""
    offs = (C.c_uint64 * (hi - lo + 2))()
    rc = fn(h, replica, lo, hi, None, 0, offs)
    if rc not in (0, RBE_E_NOMEM):
        raise EngineError(f"rbe_get_entry_cmds failed with rc={rc}")
    total = offs[hi - lo + 1]
    buf = C.create_string_buffer(max(1, total))
    _check(fn(h, replica, lo, hi, buf, total, offs), "rbe_get_entry_cmds")
    raw = buf.raw
    return [raw[offs[i]:offs[i + 1]] for i in range(hi - lo + 1)]


def outbox_call(fn, h, replica, cap, ent_cap, cmd_cap):
    """rbe_get_outbox (or the host build's twin), sized by the counts it reports."""
    arr = (RbeMessage * cap)()
    ents = (RbeEntry * ent_cap)()
    cmd = C.create_string_buffer(max(1, cmd_cap))
    n, ne, nc = C.c_uint32(), C.c_uint32(), C.c_uint64()
    _check(fn(h, replica, arr, cap, C.byref(n), ents, ent_cap, C.byref(ne), cmd, cmd_cap,
              C.byref(nc)), "rbe_get_outbox")
    if n.value > cap or ne.value > ent_cap or nc.value > cmd_cap:
        return outbox_call(fn, h, replica, max(cap, n.value), max(ent_cap, ne.value),
                           max(cmd_cap, nc.value))
    es = [ents[i] for i in range(ne.value)]
    raw, cmds, off = cmd.raw, [], 0
    for e in es:
        cmds.append(raw[off:off + e.cmd_len])
        off += e.cmd_len
    return [arr[i] for i in range(n.value)], es, cmds


def push_messages_call(fn, h, groups, msgs, ents, cmds=None):
    """rbe_push_messages (or the host build's twin); raises InputError."""
    n = len(msgs)
    g = (C.c_uint64 * max(1, n))(*groups)
    m = (RbeMessage * max(1, n))(*msgs)
    e = (RbeEntry * max(1, len(ents)))(*ents)
    buf = None
    if cmds is not None:
        blob = b"".join(cmds)
        buf = C.create_string_buffer(blob, max(1, len(blob)))
    _check_input(fn(h, n, g, m, e, buf), "rbe_push_messages")


class NodeInputs:
    """The node-layer input calls (include/rbe.h rbe_push_proposals ...
    rbe_notify_applied), marshalled once for the HIP engine and for the
    test-only host build; a subclass supplies `_input(name, *args)`."""

    # node-layer inputs for the next step (rbe.h; each call is all-or-nothing)
    def push_proposals(self, replicas, batches):
        """Peer.ProposeEntries: batches[i] is a list of entries proposed at
        replicas[i], each a Cmd byte string, an (entry_type, Cmd) pair, or an
        object with raftpb.Entry attributes (type, cmd, key, client_id,
        series_id, responded_to).  Plain entries go through rbe_push_proposals,
        a batch with entry objects through rbe_propose_entries."""
        n = len(replicas)
        counts, ents, blob = [], [], bytearray()
        full = False
        for b in batches:
            counts.append(len(b))
            for e in b:
                if isinstance(e, (bytes, bytearray)):
                    t, c, meta = 0, bytes(e), (0, 0, 0, 0)
                elif isinstance(e, tuple):
                    t, c, meta = e[0], bytes(e[1]), (0, 0, 0, 0)
                else:
                    full = True
                    t, c = e.type, bytes(e.cmd)
                    meta = tuple(getattr(e, f, 0) for f in SESSION_FIELDS)
                ents.append(make_entry(type=t, cmd=c, key=meta[0], client_id=meta[1],
                                       series_id=meta[2], responded_to=meta[3]))
                blob += c
        u32a = lambda v: (C.c_uint32 * max(1, len(v)))(*v)  # noqa: E731
        buf = (C.c_uint8 * max(1, len(blob))).from_buffer_copy(bytes(blob) or b"\0")
        if full:
            ea = (RbeEntry * max(1, len(ents)))(*ents)
            _check_input(self._input("propose_entries", n, _u64s(replicas), u32a(counts), ea,
                                     buf), "rbe_propose_entries")
            return
        _check_input(self._input("push_proposals", n, _u64s(replicas), u32a(counts),
                                 u32a([e.type for e in ents]), u32a([e.cmd_len for e in ents]),
                                 buf), "rbe_push_proposals")

    def push_read_index(self, replicas, ctxs):
        lo = [c[0] for c in ctxs]
        hi = [c[1] for c in ctxs]
        _check_input(self._input("push_read_index", len(replicas), _u64s(replicas),
                                                  _u64s(lo), _u64s(hi)), "rbe_push_read_index")

    def request_leader_transfer(self, replicas, targets):
        _check_input(self._input("request_leader_transfer", len(replicas), _u64s(replicas),
                                                          _u64s(targets)),
                     "rbe_request_leader_transfer")

    def report_unreachable(self, replicas, nodes):
        _check_input(self._input("report_unreachable", len(replicas), _u64s(replicas),
                                                     _u64s(nodes)), "rbe_report_unreachable")

    def report_snapshot_status(self, replicas, nodes, rejects):
        rej = (C.c_uint8 * max(1, len(rejects)))(*[1 if x else 0 for x in rejects])
        _check_input(self._input("report_snapshot_status", len(replicas), _u64s(replicas),
                                                         _u64s(nodes), rej),
                     "rbe_report_snapshot_status")

    def notify_applied(self, replicas, applied):
        _check_input(self._input("notify_applied", len(replicas), _u64s(replicas),
                                                 _u64s(applied)), "rbe_notify_applied")

    def launch(self, replicas, states, entries):
        """rbe_launch: restart replicas[i] from states[i] = (term, vote, commit,
        last_index[, marker, marker_term, snapshot_index, snapshot_term[,
        removed]]) (removed: bit id-1 per node the LogDB's membership does
        not list as a voter) and
        entries[i] = [(index, term, type, cmd[, key, client_id, series_id,
        responded_to]), ...], the tail of its LogDB (Peer.Launch over an
        existing log, peer.go:64-86)."""
        n = len(replicas)
        st = (RbeLaunchState * max(1, n))()
        flat = []
        for i, (s, ents) in enumerate(zip(states, entries)):
            term, vote, commit, last = s[:4]
            snap = tuple(s[4:9]) + (0,) * (9 - max(4, len(s)))
            st[i] = RbeLaunchState(term=term, vote=vote, commit=commit, last_index=last,
                                   n_entries=len(ents), marker=snap[0], marker_term=snap[1],
                                   snapshot_index=snap[2], snapshot_term=snap[3],
                                   removed=snap[4])
            flat.extend(ents)
        ea = (RbeEntry * max(1, len(flat)))()
        blob = bytearray()
        for j, x in enumerate(flat):
            idx, term, typ, cmd = x[:4]
            meta = tuple(x[4:8]) + (0,) * (8 - max(4, len(x)))
            ea[j] = make_entry(idx, term, typ, cmd, *meta)
            blob += cmd
        buf = C.create_string_buffer(bytes(blob), max(1, len(blob)))
        _check_input(self._input("launch", n, _u64s(replicas), st, ea, buf), "rbe_launch")

    def propose_config_change(self, replicas, types, nodes):
        """Peer.ProposeConfigChange (rbe_propose_config_change; cfg.membership)."""
        u32a = (C.c_uint32 * max(1, len(types)))(*types)
        _check_input(self._input("propose_config_change", len(replicas), _u64s(replicas), u32a,
                                 _u64s(nodes)), "rbe_propose_config_change")

    def apply_config_change(self, replicas, nodes, types):
        """Peer.ApplyConfigChange (rbe_apply_config_change; membership + ext_apply)."""
        u32a = (C.c_uint32 * max(1, len(types)))(*types)
        _check_input(self._input("apply_config_change", len(replicas), _u64s(replicas),
                                 _u64s(nodes), u32a), "rbe_apply_config_change")

    def restore_remotes(self, replicas, voters, observers=None, witnesses=None):
        """Peer.RestoreRemotes (rbe_restore_remotes; cfg.membership): replicas[i]'s
        snapshot membership lists the node ids voters[i], observers[i] and
        witnesses[i] (peer.go:159-165)."""
        obs = observers or [[] for _ in voters]
        wit = witnesses or [[] for _ in voters]
        n, ids = [], []
        for v, o, w in zip(voters, obs, wit):
            n += [len(v), len(o), len(w)]
            ids += list(v) + list(o) + list(w)
        u32a = (C.c_uint32 * max(1, len(n)))(*n)
        _check_input(self._input("restore_remotes", len(replicas), _u64s(replicas), u32a,
                                 _u64s(ids)), "rbe_restore_remotes")

    def set_node_ids(self, first_group, ids):
        """rbe_set_node_ids: the node ids of groups first_group.. (a list of
        n_replicas-long lists of distinct ids), before the first step."""
        flat = [x for row in ids for x in row]
        _check_input(self._input("set_node_ids", first_group, len(ids), _u64s(flat)),
                     "rbe_set_node_ids")

    def replace_node(self, replicas, node_ids):
        """rbe_replace_node: a new node (id node_ids[i]) joins in the slot of
        replicas[i], whose old node the group has removed."""
        _check_input(self._input("replace_node", len(replicas), _u64s(replicas), _u64s(node_ids)),
                     "rbe_replace_node")

    def snapshot_saved(self, replicas, indexes, terms, removed=None):
        """The host's snapshot worker saved a snapshot of its state machine and the
        LogDB took it (rbe_snapshot_saved; snapshot_entries with ext_apply):
        LogReader.CreateSnapshot in doSaveSnapshot (node.go:619-692)."""
        rem = removed if removed is not None else [0] * len(replicas)
        u32a = (C.c_uint32 * max(1, len(rem)))(*rem)
        _check_input(self._input("snapshot_saved", len(replicas), _u64s(replicas),
                                 _u64s(indexes), _u64s(terms), u32a), "rbe_snapshot_saved")

    def compact(self, replicas, to):
        """compactSnapshot's compactLogTo: the replica's next step compacts the
        LogDB to `to` (compactLog, node.go:849-866; rbe_compact)."""
        _check_input(self._input("compact", len(replicas), _u64s(replicas), _u64s(to)),
                     "rbe_compact")

    def reject_config_change(self, replicas):
        """Peer.RejectConfigChange (rbe_reject_config_change)."""
        _check_input(self._input("reject_config_change", len(replicas), _u64s(replicas)),
                     "rbe_reject_config_change")

    def commit(self, replicas, ucs):
        """Peer.Commit's log part (rbe_commit; cfg.ext_commit): ucs[i] =
        (processed, last_applied, stable_log_to, stable_log_term,
        stable_snapshot_to, ready_to_read) for replicas[i]."""
        n = len(replicas)
        arr = (RbeUpdateCommit * max(1, n))(*[RbeUpdateCommit(*u) for u in ucs])
        _check_input(self._input("commit", n, _u64s(replicas), arr), "rbe_commit")

    def set_apply_ready(self, replicas, ready):
        """node.canHaveMoreEntriesToApply per replica (sticky; ready by default)."""
        r = (C.c_uint8 * max(1, len(ready)))(*[1 if x else 0 for x in ready])
        _check_input(self._input("set_apply_ready", len(replicas), _u64s(replicas), r),
                     "rbe_set_apply_ready")


class Engine(NodeInputs):
    """One batched Raft step engine on one GPU (one rbe_engine handle)."""

    def _input(self, name, *args):
        return getattr(self.lib, "rbe_" + name)(self.h, *args)

    def __init__(self, cfg: Optional[RbeConfig] = None, **kw):
        self.lib = load_library()
        self.cfg = cfg if cfg is not None else make_config(**kw)
        h = C.c_void_p()
        _check(self.lib.rbe_create(C.byref(self.cfg), C.byref(h)), "rbe_create")
        self.h = h
        # the engine's (local) groups: fewer than cfg.n_groups with rep_compact
        ng = C.c_uint64()
        _check(self.lib.rbe_local_groups(self.h, C.byref(ng), None), "rbe_local_groups")
        self.n_groups = ng.value
        self.n_replicas = self.cfg.n_replicas
        self.n_rep = self.n_groups * self.n_replicas

    def close(self):
        if getattr(self, "h", None):
            self.lib.rbe_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # rounds
    def step(self, tick: bool = True):
        if tick:
            _check(self.lib.rbe_step(self.h), "rbe_step")
        else:
            _check(self.lib.rbe_step_ex(self.h, RBE_STEP_NO_TICK), "rbe_step_ex")

    def run(self, rounds: int):
        _check(self.lib.rbe_run(self.h, rounds), "rbe_run")

    def prepare_run(self, rounds: int):
        """Capture the replay graph of `rounds` rounds ahead of a timed run."""
        _check(self.lib.rbe_prepare_run(self.h, rounds), "rbe_prepare_run")

    def run_timed(self, rounds: int) -> float:
        ms = C.c_float()
        _check(self.lib.rbe_run_timed(self.h, rounds, C.byref(ms)), "rbe_run_timed")
        return ms.value

    def sync(self):
        _check(self.lib.rbe_sync(self.h), "rbe_sync")

    @property
    def round(self) -> int:
        r = C.c_uint32()
        _check(self.lib.rbe_round(self.h, C.byref(r)), "rbe_round")
        return r.value

    # group-range snapshots (rbe_snap.h): checkpoint/resume and slow-path hand-off
    def snapshot_bytes(self, count: Optional[int] = None) -> int:
        n = C.c_uint64()
        count = self.n_groups if count is None else count
        _check(self.lib.rbe_snapshot_bytes(self.h, count, C.byref(n)), "rbe_snapshot_bytes")
        return n.value

    def export_groups(self, first: int = 0, count: Optional[int] = None,
                      cap: Optional[int] = None) -> bytes:
        """The protocol state of groups [first, first + count) after the last
        queued round, as bytes (peer.go:64-87 / raft.go:283-330 restated)."""
        count = self.n_groups - first if count is None else count
        if cap is None:
            nb = C.c_uint64()
            _check(self.lib.rbe_export_bytes(self.h, first, count, C.byref(nb)), "rbe_export_bytes")
            n = nb.value
        else:
            n = cap
        buf = C.create_string_buffer(max(1, n))
        rc = self.lib.rbe_export_groups(self.h, first, count, buf, n)
        if rc != 0:
            raise SnapshotError(rc, "rbe_export_groups")
        return buf.raw[:n]

    def import_groups(self, snap: bytes, resume: bool = False):
        """Overwrite the snapshot's groups; `resume` moves a whole engine to
        the snapshot's round (RBE_IMPORT_RESUME)."""
        rc = self.lib.rbe_import_groups(self.h, snap, len(snap), 1 if resume else 0)
        if rc != 0:
            raise SnapshotError(rc, "rbe_import_groups")

    # outputs
    def counters(self) -> Dict[str, int]:
        o = (C.c_uint64 * CTR_NUM)()
        _check(self.lib.rbe_get_counters(self.h, o), "rbe_get_counters")
        return {n: o[i] for i, n in enumerate(COUNTER_NAMES)}

    def kernel_counters(self, kernel: int) -> Dict[str, int]:
        """Counters contributed by the kernel in one pipeline slot."""
        o = (C.c_uint64 * CTR_NUM)()
        _check(self.lib.rbe_get_kernel_counters(self.h, kernel, o), "rbe_get_kernel_counters")
        return {n: o[i] for i, n in enumerate(COUNTER_NAMES)}

    def kernel_names(self) -> List[str]:
        """Kernel in each pipeline slot ("" for an unused slot)."""
        out = []
        for i in range(KERNEL_SLOTS):
            buf = C.create_string_buffer(64)
            _check(self.lib.rbe_kernel_name(self.h, i, buf, 64), "rbe_kernel_name")
            out.append(buf.value.decode())
        return out

    def profile_rounds(self, rounds: int) -> List[float]:
        """Run `rounds` rounds with HIP events between the pipeline kernels;
        returns each slot's total milliseconds (kernel_names() order)."""
        ms = (C.c_float * KERNEL_SLOTS)()
        _check(self.lib.rbe_profile_rounds(self.h, rounds, ms), "rbe_profile_rounds")
        return list(ms)

    # replica-per-GPU exchange (dragonboat_amd/replica.py drives these)
    def xchg_pack(self, buf_ptr: int, caps):
        """Pack the last round's cross-rank records into the device buffer at
        `buf_ptr`; returns (fits, counts[peer * 3 + stream]).  When a region
        overflowed (fits False) the counts are still exact: grow and re-pack."""
        world = max(1, self.cfg.rep_world)
        cap = (C.c_uint64 * 3)(*caps)
        out = (C.c_uint32 * (3 * world))()
        rc = self.lib.rbe_xchg_pack(self.h, C.c_void_p(buf_ptr), cap, out)
        if rc not in (0, RBE_E_NOMEM):
            _check(rc, "rbe_xchg_pack")
        return rc == 0, list(out)

    def xchg_unpack(self, cnt_ptr: int, n_cnt: int, msg_ptr: int, n_msg: int, ent_ptr: int,
                    n_ent: int):
        _check(self.lib.rbe_xchg_unpack(self.h, C.c_void_p(cnt_ptr), n_cnt, C.c_void_p(msg_ptr),
                                        n_msg, C.c_void_p(ent_ptr), n_ent), "rbe_xchg_unpack")

    # fixed-capacity exchange: no host synchronisation between pack and unpack
    def xchg_pack_fixed(self, buf_ptr: int, caps):
        cap = (C.c_uint64 * 3)(*caps)
        _check(self.lib.rbe_xchg_pack_fixed(self.h, C.c_void_p(buf_ptr), cap),
               "rbe_xchg_pack_fixed")

    def xchg_unpack_fixed(self, recv_ptr: int, caps):
        cap = (C.c_uint64 * 3)(*caps)
        _check(self.lib.rbe_xchg_unpack_fixed(self.h, C.c_void_p(recv_ptr), cap),
               "rbe_xchg_unpack_fixed")

    def xchg_status(self) -> int:
        o = C.c_uint32()
        _check(self.lib.rbe_xchg_status(self.h, C.byref(o)), "rbe_xchg_status")
        return o.value

    def stream_handle(self) -> int:
        """The engine's HIP stream (hipStream_t) as an integer."""
        v = C.c_void_p()
        _check(self.lib.rbe_stream(self.h, C.byref(v)), "rbe_stream")
        return v.value or 0

    def owned(self, replica: int) -> bool:
        """Replica-per-GPU ownership: replica k of group g lives on rank (g + k) % world."""
        w = max(1, self.cfg.rep_world)
        return w == 1 or (replica // self.n_replicas + replica % self.n_replicas) % w == \
            self.cfg.rep_rank

    def reset_counters(self):
        _check(self.lib.rbe_reset_counters(self.h), "rbe_reset_counters")

    def views(self, first: int = 0, count: Optional[int] = None):
        count = self.n_rep - first if count is None else count
        arr = (RbeReplicaView * count)()
        _check(self.lib.rbe_get_views(self.h, first, count, arr), "rbe_get_views")
        return arr

    def rate_limited(self):
        """rbe_rate_limited over every replica: (Peer.RateLimited per replica as
        numpy bool, rl.Get() in-memory log bytes as numpy uint64)."""
        return rate_limited_call(self.lib.rbe_rate_limited, self.h, self.n_rep)

    def global_groups(self):
        """rbe_local_groups: the global group of each local group (numpy
        uint64; UINT64_MAX for padding groups of a compacted engine)."""
        return global_groups_call(self.lib.rbe_local_groups, self.h, self.n_groups)

    def iso_leaders(self):
        """rbe_iso_leaders: None unless the next step is an isolation epoch
        round, else this engine's leader bits per group (numpy uint8)."""
        return iso_leaders_call(self.lib.rbe_iso_leaders, self.h, self.cfg.n_groups)

    def set_iso_leaders(self, bits):
        _check(self.lib.rbe_set_iso_leaders(self.h, np.ascontiguousarray(bits, np.uint8).ctypes.data),
               "rbe_set_iso_leaders")

    def wire_ingest(self, data: bytes) -> dict:
        """rbe_wire_ingest: deliver one round's inbound frames to the next step
        on the device; returns the stats as a dict (raises InputError with the
        return code on a refused batch)."""
        return wire_ingest_call(self.lib.rbe_wire_ingest, self.h, data)

    def wire_encode(self, deployment_id=0, bin_ver=0, groups_per_batch=0, source_address=(),
                    dst_rank=-1):
        """rbe_wire_encode: the last round's outbox as framed MessageBatches in
        device memory; returns (bytes, frames, messages, InstallSnapshots left out)."""
        tot = (C.c_uint64 * 4)()
        wc = wire_config(deployment_id, bin_ver, groups_per_batch, source_address, dst_rank)
        _check(self.lib.rbe_wire_encode(self.h, C.byref(wc), tot), "rbe_wire_encode")
        return tuple(tot)

    def wire_fetch(self, totals):
        """(stream bytes, [rbe_wire_frame]) of the last rbe_wire_encode."""
        nbytes, nf = totals[0], totals[1]
        buf = C.create_string_buffer(max(1, nbytes))
        fr = (RbeWireFrame * max(1, nf))()
        _check(self.lib.rbe_wire_fetch(self.h, buf, nbytes, fr, nf), "rbe_wire_fetch")
        return buf.raw[:nbytes], [fr[i] for i in range(nf)]

    def wire_decode(self, data: bytes, cap=1 << 16, ent_cap=1 << 16, cmd_cap=1 << 20):
        """rbe_wire_decode: (messages, entries, cmd bytes); raises EngineError
        with rc RBE_E_CORRUPT on a bad frame."""
        msgs = (RbeMessage * cap)()
        ents = (RbeEntry * ent_cap)()
        cmd = C.create_string_buffer(max(1, cmd_cap))
        nm, ne, nc = C.c_uint32(), C.c_uint32(), C.c_uint64()
        rc = self.lib.rbe_wire_decode(self.h, data, len(data), msgs, cap, C.byref(nm), ents,
                                      ent_cap, C.byref(ne), cmd, cmd_cap, C.byref(nc))
        if rc == RBE_E_NOMEM:
            return self.wire_decode(data, max(cap, nm.value), max(ent_cap, ne.value),
                                    max(cmd_cap, nc.value))
        if rc != 0:
            err = EngineError(f"rbe_wire_decode failed with rc={rc}")
            err.rc = rc
            raise err
        return ([msgs[i] for i in range(nm.value)], [ents[i] for i in range(ne.value)],
                cmd.raw[:nc.value])

    def snapshot_state(self, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """[count, 8] uint64: LogDB compaction marker, its term, snapshot index,
        snapshot term, reqSnapshotIndex, pending compactLogTo, the snapshot's
        membership and the state machine's (removed masks) per replica
        (rbe_get_snapshot_state; snapshot_entries > 0)."""
        count = self.n_rep - first if count is None else count
        out = (C.c_uint64 * (8 * count))()
        _check(self.lib.rbe_get_snapshot_state(self.h, first, count, out),
               "rbe_get_snapshot_state")
        return np.frombuffer(out, dtype=np.uint64).reshape(count, 8).copy()

    def views_np(self, first: int = 0, count: Optional[int] = None) -> np.ndarray:
        """views() as a numpy structured array (zero-copy over the ctypes array)."""
        arr = self.views(first, count)
        return np.frombuffer(arr, dtype=VIEW_DTYPE)

    def updates(self, first: int = 0, count: Optional[int] = None):
        count = self.n_rep - first if count is None else count
        arr = (RbeUpdate * count)()
        _check(self.lib.rbe_get_updates(self.h, first, count, arr), "rbe_get_updates")
        return arr

    def collect_updates(self, first: int = 0, count: Optional[int] = None):
        """rbe_collect_updates: (replica ids, Updates) of the replicas in
        [first, first + count) that have an Update, as numpy arrays (copies of
        the engine's pinned buffer)."""
        count = self.n_rep - first if count is None else count
        o = RbeUpdateList()
        _check(self.lib.rbe_collect_updates(self.h, first, count, C.byref(o)),
               "rbe_collect_updates")
        if o.n == 0:
            return np.zeros(0, np.uint64), np.zeros(0, UPDATE_DTYPE)
        rep = np.frombuffer(C.string_at(C.cast(o.replica, C.c_void_p), o.n * 8), np.uint64)
        ups = np.frombuffer(C.string_at(C.cast(o.updates, C.c_void_p),
                                        o.n * UPDATE_DTYPE.itemsize), UPDATE_DTYPE)
        return rep.copy(), ups.copy()

    def update_commits(self, first: int = 0, count: Optional[int] = None):
        """getUpdateCommit of the last round's Updates (rbe_get_update_commits)
        as tuples in UpdateCommit field order."""
        count = self.n_rep - first if count is None else count
        arr = (RbeUpdateCommit * max(1, count))()
        _check(self.lib.rbe_get_update_commits(self.h, first, count, arr),
               "rbe_get_update_commits")
        return [tuple(getattr(arr[i], f) for f, _ in RbeUpdateCommit._fields_)
                for i in range(count)]

    def update_snapshots(self, first: int = 0, count: Optional[int] = None):
        """The Snapshot of the last round's Updates (rbe_get_update_snapshots):
        (index, term, packed membership, 0) per replica, zeros for none."""
        count = self.n_rep - first if count is None else count
        arr = (C.c_uint64 * (4 * max(1, count)))()
        _check(self.lib.rbe_get_update_snapshots(self.h, first, count, arr),
               "rbe_get_update_snapshots")
        return [tuple(arr[4 * i:4 * i + 4]) for i in range(count)]

    def digests(self) -> np.ndarray:
        u = self.updates()
        return np.array([x.digest for x in u], dtype=np.uint64)

    def messages(self, replica: int, cap: int = 256):
        arr = (RbeMessage * cap)()
        n = C.c_uint32()
        _check(self.lib.rbe_get_messages(self.h, replica, arr, cap, C.byref(n)),
               "rbe_get_messages")
        if n.value > cap:  # never truncate silently (outbox() raises the same way)
            return self.messages(replica, n.value)
        return [arr[i] for i in range(n.value)]

    def outbox(self, replica: int, cap: int = 256, ent_cap: int = 1024, cmd_cap: int = 1 << 20):
        """The last round's messages of `replica` in transport order, with the
        entries of its Replicate and forwarded Propose messages and their
        whole Cmds (rbe_get_outbox): (messages, entries, cmds)."""
        return outbox_call(self.lib.rbe_get_outbox, self.h, replica, cap, ent_cap, cmd_cap)

    def push_messages(self, groups, msgs, ents, cmds=None):
        """Deliver one round's inbound batch from remote senders (rbe_push_messages);
        cmds[i] is entry i's whole Cmd (None: the entries' inline cmd)."""
        push_messages_call(self.lib.rbe_push_messages, self.h, groups, msgs, ents, cmds)

    def collect_outputs(self, first: int = 0, count: Optional[int] = None):
        """rbe_collect_outputs: (msg_off, messages, rtr_off, ready_to_reads) of
        replicas [first, first + count) as numpy arrays (copies of the
        engine's pinned buffers, which the next call or step reuses)."""
        count = self.n_rep - first if count is None else count
        o = RbeOutputs()
        _check(self.lib.rbe_collect_outputs(self.h, first, count, C.byref(o)),
               "rbe_collect_outputs")

        def arr(ptr, n, dtype):
            if n == 0:
                return np.zeros(0, dtype=dtype)
            raw = C.string_at(C.cast(ptr, C.c_void_p), n * dtype.itemsize)
            return np.frombuffer(raw, dtype=dtype).copy()

        u64 = np.dtype(np.uint64)
        return (arr(o.msg_off, count + 1, u64), arr(o.messages, o.n_messages, MESSAGE_DTYPE),
                arr(o.rtr_off, count + 1, u64), arr(o.ready_to_reads, o.n_ready_to_reads, RTR_DTYPE))

    def collect_step(self, first: int = 0, count: Optional[int] = None, remote_only=False,
                     skip_local=False):
        """rbe_collect_step: (replicas, Updates, msg_off, messages, rtr_off,
        ready_to_reads) of the replicas in [first, first + count) with an
        Update, as numpy arrays (copies of the engine's pinned buffer).
        skip_local: RBE_COLLECT_SKIP_LOCAL."""
        count = self.n_rep - first if count is None else count
        o = RbeStepOutputs()
        fl = (RBE_COLLECT_REMOTE_MSGS if remote_only else 0) | (RBE_COLLECT_SKIP_LOCAL if skip_local else 0)
        _check(self.lib.rbe_collect_step(self.h, first, count, fl, C.byref(o)), "rbe_collect_step")
        return self._step_outputs(o)

    def collect_step_begin(self, first: int = 0, count: Optional[int] = None, remote_only=False,
                           skip_local=False):
        """rbe_collect_step_begin: enqueue the collection of the last round's
        outputs; collect_step_end() returns what collect_step would."""
        count = self.n_rep - first if count is None else count
        fl = (RBE_COLLECT_REMOTE_MSGS if remote_only else 0) | (RBE_COLLECT_SKIP_LOCAL if skip_local else 0)
        _check(self.lib.rbe_collect_step_begin(self.h, first, count, fl), "rbe_collect_step_begin")

    def collect_step_end(self):
        o = RbeStepOutputs()
        _check(self.lib.rbe_collect_step_end(self.h, C.byref(o)), "rbe_collect_step_end")
        return self._step_outputs(o)

    @staticmethod
    def _step_outputs(o):
        def arr(ptr, n, dtype):
            if n == 0:
                return np.zeros(0, dtype=dtype)
            raw = C.string_at(C.cast(ptr, C.c_void_p), n * dtype.itemsize)
            return np.frombuffer(raw, dtype=dtype).copy()

        u64 = np.dtype(np.uint64)
        return (arr(o.replica, o.n, u64), arr(o.updates, o.n, UPDATE_DTYPE),
                arr(o.msg_off, o.n + 1, u64), arr(o.messages, o.n_messages, MESSAGE_DTYPE),
                arr(o.rtr_off, o.n + 1, u64), arr(o.ready_to_reads, o.n_ready_to_reads, RTR_DTYPE))

    def ready_to_reads(self, replica: int, cap: int = 64):
        arr = (RbeReadyToRead * cap)()
        n = C.c_uint32()
        _check(self.lib.rbe_get_ready_to_reads(self.h, replica, arr, cap, C.byref(n)),
               "rbe_get_ready_to_reads")
        if n.value > cap:  # a list that spilled past rtr_cap: never truncate silently
            return self.ready_to_reads(replica, n.value)
        return [(arr[i].index, arr[i].ctx_low, arr[i].ctx_high) for i in range(n.value)]

    def entries(self, replica: int, lo: int, hi: int):
        """(Index, Term, Type, Cmd) of entries [lo, hi] of a replica's log window;
        a Cmd longer than 16 bytes comes from the payload heap."""
        return [(d["index"], d["term"], d["type"], d["cmd"])
                for d in self.entry_records(replica, lo, hi)]

    def entry_records(self, replica: int, lo: int, hi: int) -> List[dict]:
        """Every raftpb.Entry field of entries [lo, hi] (rbe_get_entries + the
        whole Cmds from rbe_get_entry_cmds)."""
        arr = (RbeEntry * (hi - lo + 1))()
        _check(self.lib.rbe_get_entries(self.h, replica, lo, hi, arr), "rbe_get_entries")
        cmds = self.entry_cmds(replica, lo, hi)
        return [entry_fields(e, c) for e, c in zip(arr, cmds)]

    def entry_cmds(self, replica: int, lo: int, hi: int) -> List[bytes]:
        return entry_cmds(self.lib.rbe_get_entry_cmds, self.h, replica, lo, hi)

    def spill_stats(self) -> Dict[str, int]:
        """The spill tiers' use (rbe_spill_stats): pool pages in use / total,
        the most round spill heap bytes a round used / its bytes per parity,
        exhaustion flags."""
        out = (C.c_uint64 * 5)()
        _check(self.lib.rbe_spill_stats(self.h, out), "rbe_spill_stats")
        return dict(pool_pages_used=out[0], pool_pages=out[1], spill_peak_bytes=out[2],
                    spill_bytes=out[3], oom=out[4])

    def fault_summary(self):
        n = C.c_uint64()
        o = C.c_uint32()
        _check(self.lib.rbe_fault_summary(self.h, C.byref(n), C.byref(o)), "rbe_fault_summary")
        return n.value, o.value

    def faults(self):
        """(replicas with a sticky fault word, OR of the words): the host build's name."""
        return self.fault_summary()


def xchg_chunk_bytes(caps) -> int:
    """Bytes of one peer's chunk in the fixed-capacity exchange layout."""
    o = C.c_uint64()
    _check(load_library().rbe_xchg_chunk_bytes((C.c_uint64 * 3)(*caps), C.byref(o)),
           "rbe_xchg_chunk_bytes")
    return o.value


def xchg_record_bytes() -> List[int]:
    o = (C.c_uint64 * 3)()
    _check(load_library().rbe_xchg_record_bytes(o), "rbe_xchg_record_bytes")
    return list(o)


def footprint(cfg: RbeConfig) -> int:
    b = C.c_uint64()
    _check(load_library().rbe_footprint(C.byref(cfg), C.byref(b)), "rbe_footprint")
    return b.value
