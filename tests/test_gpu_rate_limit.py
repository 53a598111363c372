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
