"""Round-trace fixtures (tests/golden/traces.json, made by
tests/golden/make_traces.py): the oracle and the host build of the device
step reproduce them; the -m gpu twin is in test_gpu_parity.py."""
import pytest

import oracle as O
from soa_cpu.soa import SoaCpu
from trace_util import TRACES, check_against_fixture

NAMES = list(TRACES["configs"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name):
    check_against_fixture(name, lambda kw, extra: O.Harness(**kw))


@pytest.mark.parametrize("name", NAMES)
def test_soa_cpu_reproduces_fixture(name):
    check_against_fixture(name, lambda kw, extra: SoaCpu(trace=True, **kw, **extra))


def test_c1_known_answer():
    """BASELINE configs[0]: 1 group x 3, 10k 16-byte proposals.  Every replica
    ends with committed = lastIndex = 3 bootstrap config changes
    (peer.go:396-404) + 1 leader no-op (raft.go:985) + 10,000 proposals, all
    in the first elected term (bootstrap entries are term 1, raft.go campaign
    makes it 2)."""
    fx = TRACES["configs"]["C1_10k"]
    for term, leader, committed, last, role in fx["final"]:
        assert (term, committed, last) == (2, 10004, 10004)
        assert leader == fx["final"][0][1]
    assert sum(1 for x in fx["final"] if x[4] == O.LEADER) == 1
    assert fx["counters"]["proposals"] == 10000
