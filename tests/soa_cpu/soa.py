"""TEST-ONLY wrapper of libsoa_cpu.so (host build of the device step function).

Never imported by the dragonboat_amd package; see soa_cpu.cpp.
"""
import ctypes as C
import os

from dragonboat_amd.engine import (CTR_NUM, COUNTER_NAMES, NodeInputs, RbeEntry, RbeMessage,
                                   RbeReplicaView, RbeUpdateCommit, RbeWireFrame, entry_cmds,
                                   entry_fields, make_config, outbox_call, push_messages_call,
                                   RbeWireIngestStats, global_groups_call, iso_leaders_call,
                                   rate_limited_call, wire_ingest_call)

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        # SOA_LIB: a variant build of the host tier (A/B knobs of the steps)
        p = os.environ.get("SOA_LIB") or os.path.join(_HERE, "libsoa_cpu.so")
        if not os.path.exists(p):
            raise RuntimeError(f"{p} missing: run __graft_entry__.build()")
        L = C.CDLL(p)
        L.soa_create.restype = C.c_void_p
        L.soa_create.argtypes = [C.c_void_p]
        L.soa_destroy.argtypes = [C.c_void_p]
        L.soa_run.argtypes = [C.c_void_p, C.c_uint32]
        L.soa_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.soa_views.argtypes = [C.c_void_p, C.c_void_p]
        L.soa_snapshot_state.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.soa_wire_encode.restype = C.c_int64
        L.soa_wire_encode.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                      C.POINTER(C.c_char_p), C.c_void_p, C.c_uint64,
                                      C.POINTER(RbeWireFrame), C.POINTER(C.c_uint32), C.c_int32]
        L.soa_rate_limited.restype = C.c_int
        L.soa_rate_limited.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                       C.c_void_p]
        L.soa_local_groups.restype = C.c_int
        L.soa_local_groups.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_void_p]
        L.soa_iso_leaders.restype = C.c_int
        L.soa_iso_leaders.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint32)]
        L.soa_set_iso_leaders.restype = C.c_int
        L.soa_set_iso_leaders.argtypes = [C.c_void_p, C.c_void_p]
        L.soa_wire_ingest.restype = C.c_int
        L.soa_wire_ingest.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64,
                                      C.POINTER(RbeWireIngestStats)]
        L.soa_spill_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.soa_set_full_only.argtypes = [C.c_void_p, C.c_int]
        L.soa_set_staged.argtypes = [C.c_void_p, C.c_int]
        L.soa_slow_total.restype = C.c_uint64
        L.soa_slow_total.argtypes = [C.c_void_p]
        L.soa_sleeping_groups.restype = C.c_uint64
        L.soa_sleeping_groups.argtypes = [C.c_void_p]
        P = C.POINTER
        L.soa_get_outbox.restype = C.c_int
        L.soa_get_outbox.argtypes = [C.c_void_p, C.c_uint64, P(RbeMessage), C.c_uint32,
                                     P(C.c_uint32), P(RbeEntry), C.c_uint32, P(C.c_uint32),
                                     C.c_void_p, C.c_uint64, P(C.c_uint64)]
        L.soa_push_messages.restype = C.c_int
        L.soa_push_messages.argtypes = [C.c_void_p, C.c_uint64, P(C.c_uint64), P(RbeMessage),
                                        P(RbeEntry), C.c_void_p]
        L.soa_get_entries.restype = C.c_int
        L.soa_get_entries.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                      P(RbeEntry)]
        L.soa_faults.restype = C.c_uint32
        L.soa_faults.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
        L.soa_xchg_pack.restype = C.c_int
        L.soa_xchg_pack.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint32)]
        L.soa_xchg_unpack.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                      C.c_uint64, C.c_void_p, C.c_uint64]
        L.soa_snapshot_bytes.restype = C.c_uint64
        L.soa_snapshot_bytes.argtypes = [C.c_void_p, C.c_uint64]
        L.soa_export_bytes.restype = C.c_uint64
        L.soa_export_bytes.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
        L.soa_export_groups.restype = C.c_int
        L.soa_export_groups.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                        C.c_uint64]
        L.soa_import_groups.restype = C.c_int
        L.soa_import_groups.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32]
        u64p, u32p = P(C.c_uint64), P(C.c_uint32)
        L.soa_step_ex.argtypes = [C.c_void_p, C.c_uint32]
        L.soa_xchg_pack_fixed.argtypes = [C.c_void_p, C.c_void_p, P(C.c_uint64)]
        L.soa_xchg_unpack_fixed.argtypes = [C.c_void_p, C.c_void_p, P(C.c_uint64)]
        L.soa_xchg_status.restype = C.c_uint32
        L.soa_xchg_status.argtypes = [C.c_void_p]
        L.soa_get_entry_cmds.restype = C.c_int
        L.soa_get_entry_cmds.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64,
                                         C.c_void_p, C.c_uint64, u64p]
        for name, args in {
                "push_proposals": [C.c_uint64, u64p, u32p, u32p, u32p, P(C.c_uint8)],
                "propose_entries": [C.c_uint64, u64p, u32p, P(RbeEntry), P(C.c_uint8)],
                "push_read_index": [C.c_uint64, u64p, u64p, u64p],
                "request_leader_transfer": [C.c_uint64, u64p, u64p],
                "report_unreachable": [C.c_uint64, u64p, u64p],
                "report_snapshot_status": [C.c_uint64, u64p, u64p, P(C.c_uint8)],
                "notify_applied": [C.c_uint64, u64p, u64p],
                "set_apply_ready": [C.c_uint64, u64p, P(C.c_uint8)],
                "commit": [C.c_uint64, u64p, P(RbeUpdateCommit)],
                "propose_config_change": [C.c_uint64, u64p, u32p, u64p],
                "apply_config_change": [C.c_uint64, u64p, u64p, u32p],
                "reject_config_change": [C.c_uint64, u64p],
                "restore_remotes": [C.c_uint64, u64p, u32p, u64p],
                "set_node_ids": [C.c_uint64, C.c_uint64, u64p],
                "replace_node": [C.c_uint64, u64p, u64p],
                "snapshot_saved": [C.c_uint64, u64p, u64p, u64p, u32p],
                "compact": [C.c_uint64, u64p, u64p],
                "get_update_commits": [C.c_uint64, C.c_uint64, P(RbeUpdateCommit)],
                "get_update_snapshots": [C.c_uint64, C.c_uint64, u64p],
                "launch": [C.c_uint64, u64p, C.c_void_p, C.c_void_p, C.c_void_p]}.items():
            fn = getattr(L, "soa_" + name)
            fn.restype = C.c_int
            fn.argtypes = [C.c_void_p] + args
        _lib = L
    return _lib


class SnapshotError(RuntimeError):
    def __init__(self, rc):
        super().__init__(f"snapshot call failed with rc={rc}")
        self.rc = rc


class SoaCpu(NodeInputs):
    def _input(self, name, *args):
        return getattr(lib(), "soa_" + name)(self.h, *args)

    def __init__(self, full_only=False, staged=0, **kw):
        self.cfg = make_config(**kw)
        self.h = lib().soa_create(C.byref(self.cfg))
        if not self.h:
            raise RuntimeError("soa_create failed")
        ng = C.c_uint64()
        lib().soa_local_groups(self.h, C.byref(ng), None)
        self.n_groups = ng.value
        self.n_rep = self.n_groups * self.cfg.n_replicas
        lib().soa_set_full_only(self.h, int(full_only))
        lib().soa_set_staged(self.h, int(staged))

    def spill_stats(self):
        out = (C.c_uint64 * 5)()
        lib().soa_spill_stats(self.h, out)
        return dict(pool_pages_used=out[0], pool_pages=out[1], spill_peak_bytes=out[2],
                    spill_bytes=out[3], oom=out[4])

    def slow_total(self):
        return lib().soa_slow_total(self.h)

    def sleeping_groups(self):
        return lib().soa_sleeping_groups(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().soa_destroy(self.h)
            self.h = None

    def run(self, rounds=1):
        lib().soa_run(self.h, rounds)

    def update_commits(self, first=0, count=None):
        count = self.n_rep - first if count is None else count
        arr = (RbeUpdateCommit * max(1, count))()
        rc = lib().soa_get_update_commits(self.h, first, count, arr)
        if rc:
            raise RuntimeError(f"soa_get_update_commits rc={rc}")
        return [tuple(getattr(arr[i], f) for f, _ in RbeUpdateCommit._fields_)
                for i in range(count)]

    def update_snapshots(self, first=0, count=None):
        count = self.n_rep - first if count is None else count
        arr = (C.c_uint64 * (4 * max(1, count)))()
        rc = lib().soa_get_update_snapshots(self.h, first, count, arr)
        if rc:
            raise RuntimeError(f"soa_get_update_snapshots rc={rc}")
        return [tuple(arr[4 * i:4 * i + 4]) for i in range(count)]

    def entry_cmds(self, replica, lo, hi):
        return entry_cmds(lib().soa_get_entry_cmds, self.h, replica, lo, hi)

    def entry_records(self, replica, lo, hi):
        """Every raftpb.Entry field of entries [lo, hi] (Engine.entry_records)."""
        arr = (RbeEntry * (hi - lo + 1))()
        rc = lib().soa_get_entries(self.h, replica, lo, hi, arr)
        if rc != 0:
            raise RuntimeError(f"soa_get_entries rc={rc}")
        return [entry_fields(e, c) for e, c in zip(arr, self.entry_cmds(replica, lo, hi))]

    def step(self, tick=True):
        if tick:
            lib().soa_run(self.h, 1)
        else:
            lib().soa_step_ex(self.h, 1)

    # replica-per-GPU exchange, same contract as Engine.xchg_pack / xchg_unpack
    def xchg_pack(self, buf_ptr, caps):
        world = max(1, self.cfg.rep_world)
        cap = (C.c_uint64 * 3)(*caps)
        out = (C.c_uint32 * (3 * world))()
        rc = lib().soa_xchg_pack(self.h, C.c_void_p(buf_ptr), cap, out)
        return rc == 0, list(out)

    def xchg_pack_fixed(self, buf_ptr, caps):
        lib().soa_xchg_pack_fixed(self.h, C.c_void_p(buf_ptr), (C.c_uint64 * 3)(*caps))

    def xchg_unpack_fixed(self, recv_ptr, caps):
        lib().soa_xchg_unpack_fixed(self.h, C.c_void_p(recv_ptr), (C.c_uint64 * 3)(*caps))

    def xchg_status(self):
        return lib().soa_xchg_status(self.h)

    def xchg_unpack(self, cnt_ptr, n_cnt, msg_ptr, n_msg, ent_ptr, n_ent):
        lib().soa_xchg_unpack(self.h, C.c_void_p(cnt_ptr), n_cnt, C.c_void_p(msg_ptr), n_msg,
                              C.c_void_p(ent_ptr), n_ent)

    # transport boundary, same contract as Engine.outbox / Engine.push_messages
    def outbox(self, replica, cap=256, ent_cap=1024, cmd_cap=1 << 20):
        return outbox_call(lib().soa_get_outbox, self.h, replica, cap, ent_cap, cmd_cap)

    def push_messages(self, groups, msgs, ents, cmds=None):
        push_messages_call(lib().soa_push_messages, self.h, groups, msgs, ents, cmds)

    # group-range snapshots, same contract as Engine.export_groups / import_groups
    def export_groups(self, first=0, count=None, cap=None):
        count = self.n_groups - first if count is None else count
        n = lib().soa_export_bytes(self.h, first, count) if cap is None else cap
        buf = C.create_string_buffer(max(1, n))
        rc = lib().soa_export_groups(self.h, first, count, buf, n)
        if rc != 0:
            raise SnapshotError(rc)
        return buf.raw[:n]

    def import_groups(self, snap, resume=False):
        rc = lib().soa_import_groups(self.h, snap, len(snap), 1 if resume else 0)
        if rc != 0:
            raise SnapshotError(rc)

    def views(self):
        arr = (RbeReplicaView * self.n_rep)()
        lib().soa_views(self.h, C.cast(arr, C.c_void_p))
        return arr

    def global_groups(self):
        return global_groups_call(lib().soa_local_groups, self.h, self.n_groups)

    def rate_limited(self):
        return rate_limited_call(lib().soa_rate_limited, self.h, self.n_rep)

    def iso_leaders(self):
        return iso_leaders_call(lib().soa_iso_leaders, self.h, self.cfg.n_groups)

    def set_iso_leaders(self, bits):
        import numpy as np
        b = np.ascontiguousarray(bits, np.uint8)
        lib().soa_set_iso_leaders(self.h, b.ctypes.data)

    def wire_ingest(self, data):
        """Host-build rbe_wire_ingest (Engine.wire_ingest)."""
        return wire_ingest_call(lib().soa_wire_ingest, self.h, data)

    def wire_encode(self, deployment_id=0, bin_ver=0, groups_per_batch=0, source_address=(),
                    dst_rank=-1):
        """Host-build rbe_wire_encode + rbe_wire_fetch: (stream bytes, frames)."""
        addrs = (C.c_char_p * 7)(*[a.encode() for a in source_address])
        n = self.cfg.n_replicas
        gpb = groups_per_batch or self.n_groups
        maxf = n * (n - 1) * ((self.n_groups + gpb - 1) // gpb)
        fr = (RbeWireFrame * max(1, maxf))()
        nf = C.c_uint32()
        # one output buffer per engine, grown when a stream does not fit (-1);
        # only the stream's bytes are copied out
        while True:
            buf = getattr(self, "_wire_buf", None)
            if buf is None:
                buf = self._wire_buf = C.create_string_buffer(1 << 20)
            got = lib().soa_wire_encode(self.h, deployment_id, bin_ver, groups_per_batch, addrs,
                                        buf, len(buf), fr, C.byref(nf), dst_rank)
            if got >= 0:
                break
            assert got == -1, f"soa_wire_encode: {got}"
            self._wire_buf = C.create_string_buffer(4 * len(buf))
        return C.string_at(buf, got), [fr[i] for i in range(nf.value)]

    def snapshot_state(self):
        o = (C.c_uint64 * (8 * self.n_rep))()
        lib().soa_snapshot_state(self.h, o)
        return [tuple(o[8 * r:8 * r + 8]) for r in range(self.n_rep)]

    def counters(self):
        o = (C.c_uint64 * CTR_NUM)()
        lib().soa_counters(self.h, o)
        return {n: o[i] for i, n in enumerate(COUNTER_NAMES)}

    def faults(self):
        n = C.c_uint64()
        o = lib().soa_faults(self.h, C.byref(n))
        return n.value, o
