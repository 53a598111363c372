"""GPU tier of the group-range snapshots (rbe_export_groups / rbe_import_groups).

- checkpoint/resume on the HIP engine: export after an odd number of rounds,
  resume a fresh engine from it, continue bit-exact with the uninterrupted oracle
  (the resumed engine runs its rounds through the captured graph, rbe_run);
- the host build's snapshot bytes are the device layout: a snapshot exported by
  the test-only host build of the step resumes the HIP engine, and the HIP
  engine's export of the same state is byte-identical to it;
- a partial import at the same round overwrites exactly its groups.
"""
import pytest

import oracle as O
from parity_util import C3, C4, ENGINE_EXTRA, MIXED, run_lockstep, view_diff

pytestmark = pytest.mark.gpu

CASES = {"C3": (C3, 141), "C4": (C4, 233), "MIXED": (MIXED, 118)}


def _engine(kw, name, **extra):
    from dragonboat_amd.engine import Engine
    return Engine(device=0, trace=True, **kw, **ENGINE_EXTRA.get(name, {}), **extra)


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_resume_matches_oracle(gpu_available, name):
    kw, at = CASES[name]
    a = _engine(kw, name)
    a.run(at)
    snap = a.export_groups()
    a.close()
    b = _engine(kw, name)
    b.import_groups(snap, resume=True)
    assert b.round == at
    ref = O.Harness(**kw)
    ref.run(at)
    d = run_lockstep(b, ref, 100, every=25)
    assert d is None, f"{name}: first divergence after resume {d}"
    assert b.fault_summary()[0] == 0
    b.close()


@pytest.mark.parametrize("name", ["C3", "C4"])
def test_host_build_snapshot_resumes_gpu_engine(gpu_available, name):
    from soa_cpu.soa import SoaCpu
    kw, at = CASES[name]
    extra = ENGINE_EXTRA.get(name, {})
    h = SoaCpu(trace=True, **kw, **extra)
    h.run(at)
    snap = h.export_groups()
    g = _engine(kw, name)
    g.import_groups(snap, resume=True)
    assert g.export_groups() == snap
    ref = O.Harness(**kw)
    ref.run(at)
    d = run_lockstep(g, ref, 60, every=1)
    assert d is None, f"{name}: first divergence {d}"
    g.close()


def test_gpu_partial_import(gpu_available):
    # one configuration (a snapshot imports only under the behaviour that wrote
    # it); B diverges through host-pushed proposals at every replica
    kw = dict(C3, ext_inputs=True)
    a = _engine(kw, "C3")
    b = _engine(kw, "C3")
    a.run(90)
    b.run(89)
    b.push_proposals(list(range(b.n_rep)), [[b"div-%d" % i] for i in range(b.n_rep)])
    b.run(1)
    before = [v.digest for v in b.views()]
    b.import_groups(a.export_groups(5, 12))
    n = kw["n_replicas"]
    av, bv = a.views(), b.views()
    for i in range(len(bv)):
        if 5 <= i // n < 17:
            assert view_diff(bv[i], av[i]) is None, i
        else:
            assert bv[i].digest == before[i], i
    a.close()
    b.close()
