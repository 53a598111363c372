"""Membership change on the HIP engine (libdragonboat_amd.so, cfg.membership)
against the oracle harness, round by round; the CPU-tier twin is
tests/test_membership.py (its docstring lists the reference paths covered)."""
import random

import pytest

import oracle as O
from input_util import run_driven
from parity_util import C2, C3, MIXED, run_lockstep
from test_membership import CATCHUP, MEMB

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,kw", [("C2", C2), ("C3", C3), ("MIXED", MIXED)])
def test_gpu_membership_schedule_parity(gpu_available, name, kw):
    from dragonboat_amd.engine import Engine
    kw = dict(kw, n_groups=min(kw["n_groups"], 24), **MEMB)
    eng = Engine(device=0, trace=True, **dict(kw, **CATCHUP))
    ref = O.Harness(**kw)
    seen = set()
    for _ in range(8):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"{name}: first divergence {d}"
        seen |= {v.removed for v in ref.views()}
    assert eng.fault_summary()[0] == 0
    assert len(seen) > 2, seen
    eng.close()


def test_gpu_membership_untraced(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = dict(C3, n_groups=16, **MEMB)
    eng = Engine(device=0, trace=False, **dict(kw, **CATCHUP))
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, 300, every=1, skip=("digest",)) is None
    eng.close()


def test_gpu_host_config_changes(gpu_available):
    from dragonboat_amd.engine import Engine
    kw = dict(C2, n_groups=6, ext_inputs=True, ext_apply=True, membership=True)
    eng = Engine(device=0, trace=True, **dict(kw))
    ref = O.Harness(**kw)
    rng = random.Random(3)
    n = kw["n_replicas"]

    def hook(rnd):
        if rnd < 30:
            return
        views = ref.views()
        for r in range(eng.n_rep):
            u = rng.random()
            if u < 0.03:
                t, node = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE)), rng.randrange(1, n + 1)
                eng.propose_config_change([r], [t], [node])
                ref.push(O.PUSH_CC_PROPOSE, r, t, node)
            elif u < 0.06 and views[r].removed != 0b111:
                t, node = rng.choice((O.CC_ADD_NODE, O.CC_REMOVE_NODE)), rng.randrange(0, n + 1)
                eng.apply_config_change([r], [node], [t])
                ref.push(O.PUSH_CC_APPLY, r, node, t)
            elif u < 0.07:
                eng.reject_config_change([r])
                ref.push(O.PUSH_CC_REJECT, r)

    d = run_driven(eng, ref, 200, seed=9, ext_apply=True, before_round=hook, density=0.1)
    assert d is None, f"first divergence {d}"
    eng.close()
