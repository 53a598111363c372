"""Compare an engine (oracle harness, host build of the device step, or the
HIP engine) against the committed round-trace fixtures (tests/golden/traces.json)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
TRACES = json.load(open(os.path.join(HERE, "golden", "traces.json")))
from parity_util import ENGINE_EXTRA  # noqa: E402,F401


def check_against_fixture(name, make_engine):
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_traces import digest_checksum, final_state
    fx = TRACES["configs"][name]
    eng = make_engine(fx["kw"], ENGINE_EXTRA.get(name, {}))
    done = 0
    for at, want in fx["checkpoints"]:
        eng.run(at - done)
        done = at
        got = digest_checksum(eng.views())
        assert got == want, f"{name}: trace checksum differs at round {at}"
    assert final_state(eng.views()) == fx["final"], f"{name}: final state differs"
    return eng
