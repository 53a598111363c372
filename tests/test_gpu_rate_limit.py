"""GPU parity of the rate limiter (cfg.max_inmem_log_size): the HIP engine
against the oracle harness round by round, as tests/test_rate_limit.py runs
the host build: views, trace digests (RateLimit messages and their Hint),
Peer.RateLimited and rl.Get() of every replica (rbe_rate_limited)."""
import pytest

import oracle as O
from parity_util import ENGINE_EXTRA, counters_match
from test_rate_limit import CASES, _lockstep_rl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(CASES))
def test_gpu_rate_limiter_parity(gpu_available, name):
    from dragonboat_amd.engine import Engine
    kw, rounds, limit = CASES[name]
    eng = Engine(device=0, trace=True, max_inmem_log_size=limit, **kw,
                 **ENGINE_EXTRA.get(name.replace("_SNAP", ""), {}))
    ref = O.Harness(max_inmem_log_size=limit, **kw)
    assert _lockstep_rl(eng, ref, rounds) > 0
    nf, fo = eng.fault_summary()
    assert nf == 0, f"{name}: {nf} faulted replicas, bits {fo:#x}"
    bad = counters_match(eng.counters(), ref.counters())
    assert not bad, f"{name}: counters differ {bad}"
    eng.close()


def test_gpu_rate_limiter_untraced(gpu_available):
    """Bench paths (no trace: lazy quiesced ticks in k_triage, group sleep)."""
    from dragonboat_amd.engine import Engine
    kw, rounds, limit = CASES["C4"]
    eng = Engine(device=0, trace=False, max_inmem_log_size=limit, **kw)
    ref = O.Harness(max_inmem_log_size=limit, **kw)
    assert _lockstep_rl(eng, ref, rounds, skip=("digest",)) > 0
    eng.close()


def test_gpu_rate_limiter_after_relaunch(gpu_available):
    """Followers relaunched with commit < last: RateLimit Hints count only the
    in-memory uncommitted entries (logentry.go:180-183, 205-211)."""
    from dragonboat_amd.engine import Engine
    from parity_util import C2
    from test_rate_limit import relaunch_lagging_groups
    kw = dict(C2, n_groups=64)
    eng = Engine(device=0, trace=True, max_inmem_log_size=50, **kw)
    ref = O.Harness(max_inmem_log_size=50, **kw)
    relaunch_lagging_groups(eng, ref)
    assert eng.fault_summary()[0] == 0
    eng.close()


def test_gpu_rate_limiter_ext_commit(gpu_available):
    """appliedLogTo inside the host's rbe_commit (ext_commit), persisted late or partly."""
    from commit_util import run_commit_driven
    from dragonboat_amd.engine import Engine
    from parity_util import C3
    kw = dict(C3, n_groups=12, ext_inputs=True, ext_apply=True, ext_commit=True,
              max_inmem_log_size=400)
    eng = Engine(device=0, trace=True, **kw)
    ref = O.Harness(**kw)
    d, st = run_commit_driven(eng, ref, 160, seed=5)
    assert d is None, f"first divergence {d}"
    el, es = eng.rate_limited()
    rl, rs = ref.rate_limited()
    assert (es == rs).all() and (el == rl).all()
    assert eng.fault_summary()[0] == 0
    eng.close()
