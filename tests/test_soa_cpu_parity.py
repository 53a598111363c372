"""CPU tier of the parity gate: the device step logic (rbe_step.h — the code
k_triage / k_fast_list / k_full_list run on MI355X), compiled for the host
(tests/soa_cpu, test-only), diffed round by round against the oracle harness.

The -m gpu tests run the same cases through libdragonboat_amd.so on the GPU;
this tier catches protocol regressions where no GPU is available."""
import pytest

import oracle as O
from parity_util import (C1, C2, C3, C3_HOT, C4, C4_DENSE, ENGINE_EXTRA, MIXED, SINGLE,
                         counters_match, run_lockstep)
from soa_cpu.soa import SoaCpu

CASES = {"C1": (C1, 400), "C2": (C2, 300), "C3": (C3, 400), "C3_HOT": (C3_HOT, 400),
         "C4": (C4, 500), "C4_DENSE": (C4_DENSE, 400), "SINGLE": (SINGLE, 150),
         "MIXED": (MIXED, 600)}


@pytest.mark.parametrize("mode", ["pipeline", "full_table", "aux"])
@pytest.mark.parametrize("name", list(CASES))
def test_soa_cpu_lockstep_parity(name, mode):
    """`aux`: the fast steps take their inbound count words from the
    work-list summary word (inbound_aux), as k_fast_both runs them."""
    kw, rounds = CASES[name]
    staged = {"aux": 4}.get(mode, 0)
    eng = SoaCpu(full_only=mode == "full_table", staged=staged, trace=True, **kw,
                 **ENGINE_EXTRA.get(name, {}))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1)
    assert d is None, f"{name}: first divergence {d}"
    n, bits = eng.faults()
    assert n == 0, f"{name}: faults {bits:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"


def test_pipeline_takes_fast_paths():
    """The triage/fast split must actually route steady-state rounds away from
    the full handler table (otherwise the GPU pipeline degenerates)."""
    eng = SoaCpu(trace=True, **C2)
    eng.run(200)
    assert eng.slow_total() < 0.2 * eng.counters()["steps"]


@pytest.mark.parametrize("name", list(CASES))
def test_soa_cpu_untraced_full_table(name):
    """Untraced, every replica-round on the general step: its Replicate sends
    are deferred to the lane's send queue (rbe_step.h SendQ: flushed before a
    ring write, a full queue and the step's end), and every protocol field of
    every replica must still equal the oracle's, round by round."""
    kw, rounds = CASES[name]
    eng = SoaCpu(full_only=True, trace=False, **kw, **ENGINE_EXTRA.get(name, {}))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1, skip=("digest",))
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"


@pytest.mark.parametrize("name", ["C4", "C4_DENSE", "MIXED", "C2", "C3", "C3_HOT"])
def test_soa_cpu_untraced_state_parity(name):
    """Without trace the engine takes the bench paths (lazy quiesced ticks in
    triage, no digest); every protocol field must still match the oracle."""
    kw, rounds = CASES[name]
    eng = SoaCpu(trace=False, **kw, **ENGINE_EXTRA.get(name, {}))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1, skip=("digest",))
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    if name == "C4":  # quiesced groups fall asleep (group sleep, rbe_step.h)
        assert eng.sleeping_groups() > 0


def test_sleeping_groups_wake_on_input():
    """A sleeping group (all replicas lazily quiesced) is woken by host input
    and steps exactly like the oracle; it falls asleep again afterwards."""
    kw = dict(n_groups=8, n_replicas=3, quiesce=True)
    eng = SoaCpu(trace=False, ext_inputs=True, **kw)
    ref = O.Harness(ext_inputs=True, **kw)
    d = run_lockstep(eng, ref, 500, every=1, skip=("digest",))
    assert d is None, f"first divergence {d}"
    assert eng.sleeping_groups() == 8
    v = ref.views()
    leaders = [i for i in range(24) if v[i].role == O.LEADER]
    eng.push_proposals(leaders[:2], [[b"wake"]] * 2)
    for r in leaders[:2]:
        ref.push(O.PUSH_PROPOSE, r, entries=[O.Entry(type=0, cmd=b"wake")])
    d = run_lockstep(eng, ref, 300, every=1, skip=("digest",))
    assert d is None, f"after wake: first divergence {d}"
    assert eng.sleeping_groups() == 8
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"counters differ {bad}"


def test_check_quorum_ticks_stay_on_fast_path():
    """With CheckQuorum, a leader's tick at the election-timeout boundary runs
    leaderHasQuorum (raft.go:378-388); when the quorum holds the fast leader
    step takes it (rbe_fast.h), so a steady C3 group leaves the fast kernels
    only for its first election."""
    kw = dict(C3, iso_period=0)
    eng = SoaCpu(trace=True, **kw)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, 300, every=1) is None
    assert eng.slow_total() < 0.03 * eng.counters()["steps"]
