"""rbe_collect_step_begin / _end (the collection split in two halves so the
node layer's next-round pushes overlap it) return exactly what
rbe_collect_step returns for the same round, in every flag combination; a
round past the mapped buffer's capacities is collected again synchronously;
a step between the halves is refused (RBE_E_STATE)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KW = dict(n_groups=3000, n_replicas=3, quiesce=True, check_quorum=True, wl_enabled=True,
          wl_start_round=20, wl_active_mod=3, wl_read_permille=700, iso_period=40, iso_len=15,
          iso_mod=4)


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and x.shape == y.shape
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


@pytest.mark.parametrize("trace", [False, True])
def test_gpu_collect_async_equals_sync(gpu_available, trace):
    from dragonboat_amd.engine import Engine
    eng = Engine(device=0, trace=trace, **KW)
    eng.run(30)
    seen_msgs = seen_rtr = 0
    for rnd in range(40):
        eng.run(1)
        for remote_only, skip_local in ((False, False), (True, True), (False, True)):
            want = eng.collect_step(remote_only=remote_only, skip_local=skip_local)
            eng.collect_step_begin(remote_only=remote_only, skip_local=skip_local)
            got = eng.collect_step_end()
            _same(got, want)
            seen_msgs += len(want[3])
            seen_rtr += len(want[5])
    assert seen_msgs > 0 and seen_rtr > 0
    # a sub-range
    want = eng.collect_step(first=300, count=900)
    eng.collect_step_begin(first=300, count=900)
    _same(eng.collect_step_end(), want)
    eng.close()


def test_gpu_collect_async_refuses_a_step_between(gpu_available):
    from dragonboat_amd.engine import Engine, EngineError
    eng = Engine(device=0, trace=False, **KW)
    eng.run(30)
    eng.collect_step_begin()
    eng.run(1)
    with pytest.raises(EngineError):
        eng.collect_step_end()
    eng.collect_step_begin()  # the pending call was consumed
    eng.collect_step_end()
    eng.close()
