"""Pin the quiesce manager (quiesce.go) with the reference's own tests
(quiesce_test.go, vectors in tests/golden/quiesce.json).

Three restatements are checked against the same vectors:
  * the oracle's node-side QuiesceManager (oracle/harness.h) — the checker;
  * the device engine's Lane::q_* (rbe_step.h, the full handler table) and
    FastQ (rbe_fast.h, the steady-state fast steps), compiled for the host in
    the test-only tests/soa_cpu build — what k_full_list / k_fast_both run.
"""
import ctypes as C
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "quiesce.json")))
ET = G["election_tick"]
INC, ACT, TRY, QUIESCED, NEW_TO_Q, THRESH, TICK, NAS = 0, 1, 2, 3, 4, 5, 6, 7


class _Q:
    def __init__(self, impl, enabled=True):
        self.impl = impl
        if impl == "oracle":
            L = O.lib()
            L.orc_quiesce_new.restype = C.c_void_p
            L.orc_quiesce_new.argtypes = [C.c_uint64, C.c_int]
            L.orc_quiesce_op.restype = C.c_uint64
            L.orc_quiesce_op.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
            L.orc_quiesce_free.argtypes = [C.c_void_p]
            self.L, self.h = L, L.orc_quiesce_new(ET, int(enabled))
            self._op, self._free = L.orc_quiesce_op, L.orc_quiesce_free
        else:
            from soa_cpu.soa import lib as soa_lib
            L = soa_lib()
            L.soa_quiesce_new.restype = C.c_void_p
            L.soa_quiesce_new.argtypes = [C.c_uint64, C.c_int, C.c_int]
            L.soa_quiesce_op.restype = C.c_uint64
            L.soa_quiesce_op.argtypes = [C.c_void_p, C.c_int, C.c_uint64]
            L.soa_quiesce_free.argtypes = [C.c_void_p]
            self.L, self.h = L, L.soa_quiesce_new(ET, int(enabled), 0 if impl == "lane" else 1)
            self._op, self._free = L.soa_quiesce_op, L.soa_quiesce_free

    def op(self, o, a=0):
        return self._op(self.h, o, a)

    def __del__(self):
        self._free(self.h)

    def increase(self):
        self.op(INC)

    def record(self, t):
        self.op(ACT, t)

    @property
    def quiesced(self):
        return bool(self.op(QUIESCED))

    @property
    def new_to_quiesce(self):
        return bool(self.op(NEW_TO_Q))


IMPLS = ["oracle", "lane", "fastq"]


@pytest.mark.parametrize("impl", IMPLS)
def test_threshold(impl):
    assert _Q(impl).op(THRESH) == ET * 10  # quiesce.go:84-86


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("case", G["increase_tick_can_enter_quiesce"]["cases"])
def test_increase_tick_can_enter_quiesce(impl, case):
    ticks, want = case
    q = _Q(impl)
    for _ in range(ticks):
        q.increase()
    assert q.quiesced == want


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("case", G["quiesce_can_be_disabled"]["cases"])
def test_quiesce_can_be_disabled(impl, case):
    ticks, want = case
    q = _Q(impl, enabled=False)
    for _ in range(ticks):
        q.increase()
    assert q.quiesced == want


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("mtype", G["exit_from_quiesce_when_activity_is_recorded"]["cases"])
def test_exit_from_quiesce_when_activity_is_recorded(impl, mtype):
    q = _Q(impl)
    for _ in range(q.op(THRESH) + 1):
        q.increase()
    assert q.quiesced
    q.record(mtype)
    assert not q.quiesced
    assert q.op(NAS) == q.op(TICK)


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("case", G["heartbeat_will_not_stop_entering_quiesce"]["cases"])
def test_heartbeat_will_not_stop_entering_quiesce(impl, case):
    ticks, want = case
    q = _Q(impl)
    for _ in range(ticks):
        q.increase()
        q.record(17)  # pb.Heartbeat
    assert q.quiesced == want


@pytest.mark.parametrize("impl", IMPLS)
def test_delayed_heartbeat_will_not_exit_quiesce(impl):
    hb = G["delayed_heartbeat_will_not_exit_quiesce"]["heartbeat_type"]
    q = _Q(impl)
    for _ in range(q.op(THRESH) + 1):
        q.increase()
    assert q.quiesced
    assert q.new_to_quiesce
    steps = 0
    while q.new_to_quiesce:
        q.record(hb)
        assert q.quiesced
        q.increase()
        steps += 1
    assert steps == ET  # newToQuiesce lasts electionTick ticks (quiesce.go:88-93)
    q.record(hb)
    assert not q.quiesced
