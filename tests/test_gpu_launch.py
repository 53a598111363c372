"""rbe_launch on the HIP engine: replicas restarted from persisted state
continue bit-exact with the oracle restarting the same nodes through
Peer.Launch over their LogDB (tests/test_launch.py is the CPU twin)."""
import pytest

import oracle as O
from input_util import run_driven
from launch_util import restart
from parity_util import C2, C3, C4, run_lockstep

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,kw,extra", [("C2", C2, {}), ("C3", C3, dict()),
                                           ("C4", C4, {})])
def test_gpu_restart_continues_with_oracle(gpu_available, name, kw, extra):
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=10)
    eng, ref = Engine(device=0, trace=True, **dict(kw, **extra)), O.Harness(**kw)
    assert run_lockstep(eng, ref, 45, every=1) is None
    n = kw["n_replicas"]
    lead = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
    picks = sorted(set([1, lead[0], lead[-1]] + list(range(5 * n, 6 * n))))
    restart(eng, ref, picks, extra.get("ring", 64))
    d = run_lockstep(eng, ref, 60, every=1)
    assert d is None, f"{name}: first divergence after restart {d}"
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_restart_untraced_group_sleep(gpu_available):
    """C4 untraced (group sleep, awake lists): restarting replicas of sleeping
    groups wakes them through a scan round; state stays equal to the oracle."""
    from dragonboat_amd.engine import Engine
    kw = dict(C4, n_groups=40, wl_start_round=10)
    eng, ref = Engine(device=0, trace=False, **kw), O.Harness(**kw)
    assert run_lockstep(eng, ref, 40, every=1, skip=("digest",)) is None
    restart(eng, ref, [0, 1, 2, 30, 61, 100], 64)
    d = run_lockstep(eng, ref, 260, every=1, skip=("digest",))
    assert d is None, f"first divergence after restart {d}"
    eng.close()


def test_gpu_restart_with_lagging_applied(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = dict(C2, n_groups=8, ext_inputs=True, ext_apply=True)
    eng = Engine(device=0, trace=True, **dict(kw))
    ref = O.Harness(**kw)

    def hook(rnd):
        if rnd in (30, 52):
            restart(eng, ref, [0, 4, 8, 9, 10, 11] if rnd == 30 else [1, 2, 7], 256)

    d = run_driven(eng, ref, 80, seed=21, ext_apply=True, before_round=hook)
    assert d is None, f"first divergence after restart {d}"
    assert eng.fault_summary()[0] == 0
    eng.close()
