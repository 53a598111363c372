"""Observers and witnesses on the HIP engine against the oracle harness, round
by round; the CPU-tier twin is tests/test_observers_witnesses.py."""
import pytest

import oracle as O
from parity_util import run_lockstep
from test_membership import CATCHUP
from test_observers_witnesses import OW_CASES, SIZES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(OW_CASES))
def test_gpu_observer_witness_schedule(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, rounds = OW_CASES[name]
    eng = Engine(device=0, trace=True, **kw, **SIZES.get(name, CATCHUP))
    ref = O.Harness(**kw)
    wit = 0
    for _ in range(rounds // 50):
        d = run_lockstep(eng, ref, 50, every=1)
        assert d is None, f"{name}: first divergence {d}"
        wit |= max(v.witnesses for v in ref.views())
    assert wit
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_observer_witness_untraced(gpu_available):
    from dragonboat_amd.engine import Engine
    kw, _ = OW_CASES["N6"]
    eng = Engine(device=0, trace=False, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    assert run_lockstep(eng, ref, 300, every=1, skip=("digest",)) is None
    eng.close()


def test_gpu_observer_witness_snapshots(gpu_available):
    from dragonboat_amd.engine import Engine
    from test_membership_snapshot import run_memb_snap
    kw = dict(OW_CASES["N5"][0], snapshot_entries=8, compaction_overhead=2, iso_mod=2)
    eng = Engine(device=0, trace=True, **kw, **CATCHUP)
    ref = O.Harness(**kw)
    run_memb_snap(eng, ref, 400)
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_host_cannot_put_a_node_in_two_sets(gpu_available):
    """rbe_apply_config_change reads the replicas' membership from the device
    and refuses an AddObserver / AddWitness that would put a node in two of
    raft's maps (CPU twin in test_observers_witnesses.py)."""
    from dragonboat_amd.engine import Engine, InputError, RBE_E_INVALID
    from parity_util import C2
    kw = dict(C2, n_groups=2, n_replicas=5, n_voters=3, observer_slots=0b01000,
              witness_slots=0b10000, ext_inputs=True, ext_apply=True, membership=True)
    eng = Engine(device=0, trace=True, **dict(kw))
    eng.run(30)
    eng.apply_config_change([0], [4], [O.CC_ADD_OBSERVER])
    eng.step()
    eng.apply_config_change([0], [5], [O.CC_ADD_WITNESS])
    eng.step()
    for node, t in ((2, O.CC_ADD_OBSERVER), (3, O.CC_ADD_WITNESS), (4, O.CC_ADD_WITNESS),
                    (5, O.CC_ADD_OBSERVER)):
        with pytest.raises(InputError) as ei:
            eng.apply_config_change([0], [node], [t])
        assert ei.value.rc == RBE_E_INVALID, (node, t)
    v = eng.views()[0]
    assert v.observers == 0b01000 and v.witnesses == 0b10000
    assert eng.fault_summary()[0] == 0
    eng.close()
