"""Full-size runs of the HIP engine at the BASELINE configurations the bench
quotes — C4 (1M groups x 3, Quiesce, 90% idle, 9:1 ReadIndex:propose), C3
(100k groups x 5, CheckQuorum, leader isolation) and C2 (10k groups x 3, one
proposal per group per round) — in the bench's untraced
mode, checked through properties that hold at any size plus the oracle on a
seeded sample of groups:

  * no replica faults (no capacity or window overflow, no reference panic);
  * Election Safety: at most one leader per (group, term) (Raft §5.2);
  * commit monotonicity between checkpoints, and processed <= committed <=
    lastIndex on every replica;
  * oracle equality: groups are independent and every input is a function of
    (seed, cluster id, round), so a one-group oracle harness at that group's
    cluster id reproduces it exactly; every protocol field of every replica of
    the sampled groups must match (the digest is off in untraced mode).
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

C4_FULL = dict(n_groups=1_000_000, n_replicas=3, quiesce=True, wl_enabled=True,
               wl_start_round=30, wl_active_mod=10, wl_read_permille=900)
C3_FULL = dict(n_groups=100_000, n_replicas=5, check_quorum=True, wl_enabled=True,
               wl_start_round=40, iso_period=50, iso_len=30, iso_mod=10)
C2_FULL = dict(n_groups=10_000, n_replicas=3, wl_enabled=True, wl_start_round=30)
ENGINE = {"C4": dict(), "C3": dict(), "C2": dict()}
SAMPLE = {"C4": 48, "C3": 48, "C2": 160}
FIELDS = [f for f in O.VIEW_FIELDS if f != "digest"]


def _check_properties(v, n, prev_committed=None):
    G = len(v["role"]) // n
    role = v["role"].reshape(G, n)
    term = v["term"].reshape(G, n)
    lead = role == O.LEADER
    for i in range(n):
        for j in range(i + 1, n):
            both = lead[:, i] & lead[:, j] & (term[:, i] == term[:, j])
            assert not both.any(), f"two leaders in one term, groups {np.nonzero(both)[0][:8]}"
    assert (v["processed"] <= v["committed"]).all()
    assert (v["committed"] <= v["last_index"]).all()
    if prev_committed is not None:
        assert (v["committed"] >= prev_committed).all(), "a commit index moved backwards"
    return v["committed"].copy()


def _fields(eng, chunk=600_000):
    """role/term/committed/processed/last_index of every replica, fetched in
    group-aligned chunks (rbe_get_views)."""
    keep = ["role", "term", "committed", "processed", "last_index"]
    n = eng.n_replicas
    chunk -= chunk % n
    parts = []
    for first in range(0, eng.n_rep, chunk):
        v = eng.views_np(first, min(chunk, eng.n_rep - first))
        parts.append({k: v[k].copy() for k in keep})
    return {k: np.concatenate([p[k] for p in parts]) for k in keep}


def _sampled_oracle(eng, kw, rounds, groups):
    n = kw["n_replicas"]
    for g in groups:
        ref = O.Harness(**dict(kw, n_groups=1, cid_base=1 + int(g)), trace=False)
        ref.run(rounds)
        ev, rv = eng.views(int(g) * n, n), ref.views()
        for k in range(n):
            for f in FIELDS:
                a, b = getattr(ev[k], f), getattr(rv[k], f)
                if hasattr(a, "__len__"):
                    a, b = list(a), list(b)
                assert a == b, f"group {g} replica {k} field {f}: engine {a} oracle {b}"


@pytest.mark.parametrize("name,kw,rounds,check_every",
                         [("C4", C4_FULL, 400, 100), ("C3", C3_FULL, 300, 50),
                          ("C2", C2_FULL, 300, 50)])
def test_fullsize_properties_and_sampled_oracle(gpu_available, name, kw, rounds, check_every):
    from dragonboat_amd.engine import Engine
    eng = Engine(device=0, trace=False, **kw, **ENGINE[name])
    n = kw["n_replicas"]
    prev = None
    done = 0
    while done < rounds:
        eng.run(check_every)
        done += check_every
        nf, fo = eng.fault_summary()
        assert nf == 0, f"{name} round {done}: {nf} faulted replicas, bits {fo:#x}"
        prev = _check_properties(_fields(eng), n, prev)
    c = eng.counters()
    assert c["committed"] > 0
    if name == "C2":  # one proposal per group per round from round 30 on: every group
        v = _fields(eng)  # commits (proposals before its first leader are dropped)
        lead = v["committed"].reshape(-1, n).max(axis=1)
        assert (lead >= (rounds - kw["wl_start_round"]) // 2).all(), int(lead.min())
    rng = np.random.RandomState(0x5EED)
    sample = rng.choice(kw["n_groups"], SAMPLE[name], replace=False)
    _sampled_oracle(eng, kw, rounds, sample)
    eng.close()
