"""GPU parity: the HIP engine (through the C ABI of libdragonboat_amd.so) against
the oracle harness, on the same seeds, workloads and fault schedules.

Bar: bit-exact.  Every replica's protocol state (term, vote, leader, commit,
lastIndex, processed, savedTo, role, tick counters, quiesce state, readIndex
queue length, vote masks, leader-side remote match/next/state/active) and its
running trace digest (which folds in every emitted message, ReadyToRead,
applied entry and dropped request of every round) must be identical, round by
round.
"""
import pytest

import oracle as O
from parity_util import (C1, C2, C3, C3_HOT, C4, C4_DENSE, ENGINE_EXTRA, MIXED, SINGLE,
                         counters_match, run_lockstep)

pytestmark = pytest.mark.gpu

CASES = {"C1": (C1, 400), "C2": (C2, 300), "C3": (C3, 400), "C3_HOT": (C3_HOT, 400),
         "C4": (C4, 500), "C4_DENSE": (C4_DENSE, 400), "SINGLE": (SINGLE, 150),
         "MIXED": (MIXED, 600)}


def _engine(kw, name):
    from dragonboat_amd.engine import Engine
    return Engine(device=0, trace=True, **kw, **ENGINE_EXTRA.get(name, {}))


@pytest.mark.parametrize("name", list(CASES))
def test_lockstep_parity(gpu_available, name):
    kw, rounds = CASES[name]
    eng = _engine(kw, name)
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1)
    assert d is None, f"{name}: first divergence {d}"
    nf, fo = eng.fault_summary()
    assert nf == 0, f"{name}: {nf} faulted replicas, bits {fo:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    eng.close()


def test_graph_replay_matches_stepwise(gpu_available):
    """rbe_run (graph replay) must equal rbe_step round by round."""
    from dragonboat_amd.engine import Engine
    kw = dict(C4_DENSE)
    a = Engine(device=0, trace=True, **kw)
    b = Engine(device=0, trace=True, **kw)
    a.run(64)
    a.run(64)
    a.run(37)
    for _ in range(165):
        b.step()
    da, db = a.digests(), b.digests()
    assert (da == db).all()
    assert a.counters() == b.counters()


def test_graph_cache_across_round_counts(gpu_available):
    """Graphs captured ahead (rbe_prepare_run) and cached per round count,
    replayed interleaved and past the cache size, equal stepwise rounds."""
    from dragonboat_amd.engine import Engine
    kw = dict(C4_DENSE)
    a = Engine(device=0, trace=True, **kw)
    b = Engine(device=0, trace=True, **kw)
    a.prepare_run(20)
    a.prepare_run(7)
    total = 0
    for k in (20, 7, 20, 5, 3, 11, 7, 20, 2, 9):
        if k == 9:
            assert a.run_timed(k) >= 0.0
        else:
            a.run(k)
        total += k
    for _ in range(total):
        b.step()
    assert (a.digests() == b.digests()).all()
    assert a.counters() == b.counters()


def test_larger_groups_digest_parity(gpu_available):
    """Larger population, compared on digests every 25 rounds."""
    kw = dict(C4, n_groups=2000)
    eng = _engine(kw, "C4")
    ref = O.Harness(**kw, threads=4)
    d = run_lockstep(eng, ref, 300, every=25, full_views=False)
    assert d is None, f"divergence {d}"
    assert eng.fault_summary()[0] == 0


def test_ext_inputs_path(gpu_available):
    """Host-pushed proposals / reads (rbe_push_*) reach the leader and commit."""
    from dragonboat_amd.engine import Engine
    eng = Engine(device=0, n_groups=4, n_replicas=3, ext_inputs=True, trace=True)
    eng.run(40)
    views = eng.views()
    leaders = [i for i, v in enumerate(views) if v.role == 2]
    assert len(leaders) == 4
    c0 = [views[i].committed for i in leaders]
    eng.push_proposals(leaders, [[b"hello-raft-%02d" % i] for i in range(4)])
    eng.run(3)
    views = eng.views()
    for j, i in enumerate(leaders):
        assert views[i].committed == c0[j] + 1
        ents = eng.entries(i, views[i].committed, views[i].committed)
        assert ents[0][3] == b"hello-raft-%02d" % j
    eng.push_read_index(leaders, [(7 << 32 | 1, 99)] * 4)
    eng.step()
    eng.step()
    eng.step()
    assert eng.counters()["reads_confirmed"] == 4


@pytest.mark.parametrize("name", ["C1_10k", "C2", "C3", "C3_HOT", "C4", "C4_DENSE", "SINGLE",
                                  "MIXED"])
def test_engine_reproduces_trace_fixture(gpu_available, name):
    """The HIP engine against the committed round-trace fixtures."""
    from dragonboat_amd.engine import Engine
    from trace_util import check_against_fixture
    eng = check_against_fixture(
        name, lambda kw, extra: Engine(device=0, trace=True, **kw, **extra))
    assert eng.fault_summary()[0] == 0
    eng.close()


@pytest.mark.parametrize("name", ["C4", "C4_DENSE", "MIXED", "C2", "C3"])
def test_engine_untraced_state_parity(gpu_available, name):
    """The bench configuration (trace off: lazy quiesced ticks, no digest) must
    keep every protocol field bit-exact with the oracle, round by round."""
    from dragonboat_amd.engine import Engine
    kw, rounds = CASES[name]
    eng = Engine(device=0, trace=False, **kw, **ENGINE_EXTRA.get(name, {}))
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, rounds, every=1, skip=("digest",))
    assert d is None, f"{name}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    eng.close()


@pytest.mark.parametrize("mode", ["split", "fused", "full"])
@pytest.mark.parametrize("name", ["C2", "C4_DENSE", "MIXED"])
def test_pipeline_modes_parity(gpu_available, monkeypatch, name, mode):
    """Every pipeline (RBE_MODE) is bit-exact with the oracle, not only the
    default one (triage → merged fast launch → full list)."""
    monkeypatch.setenv("RBE_MODE", mode)
    kw, rounds = CASES[name]
    eng = _engine(kw, name)
    ref = O.Harness(**kw)
    d = run_lockstep(eng, ref, min(rounds, 300), every=1)
    assert d is None, f"{name}/{mode}: first divergence {d}"
    assert eng.fault_summary()[0] == 0
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}/{mode}: counters differ {bad}"
    eng.close()
