"""A failed pinned-memory allocation while staging host input is RBE_E_NOMEM at
the C ABI, not std::terminate under ctypes (rbe_engine.hip abi_nomem), and the
refused batch leaves nothing staged: the engine goes on stepping bit-exact.

The limit is injected with RBE_PINNED_LIMIT_BYTES, read once per process at
the first pinned allocation, so the test runs in a child process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys
sys.path[:0] = ["oracle", "tests", "."]  # as tests/conftest.py
import oracle as O
from dragonboat_amd.engine import Engine, InputError, RBE_E_NOMEM
from parity_util import run_lockstep
kw = dict(n_groups=8, n_replicas=3, check_quorum=True, ext_inputs=True)
eng, ref = Engine(device=0, trace=True, **kw), O.Harness(trace=True, **kw)
assert run_lockstep(eng, ref, 40, every=10) is None
leaders = [i for i, v in enumerate(ref.views()) if v.role == O.LEADER]
# 512 entries need 16 KiB of pinned staging, over the 4 KiB limit
try:
    eng.push_proposals([leaders[0]], [[b"x%d" % i for i in range(512)]])
    raise SystemExit("the oversized batch was accepted")
except InputError as e:
    assert e.rc == RBE_E_NOMEM, e.rc
# nothing of it was staged: the engine and the oracle go on equal
assert run_lockstep(eng, ref, 30, every=1) is None
print("ok")
"""


def test_pinned_staging_failure_is_nomem(gpu_available):
    env = dict(os.environ, RBE_PINNED_LIMIT_BYTES="4096")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", CHILD], cwd=root, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout + p.stderr
