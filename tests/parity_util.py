"""Shared helpers for parity tests: compare an engine (HIP engine or the
test-only host build) with the oracle harness round by round."""
from __future__ import annotations

import oracle as O

FIELDS = list(O.VIEW_FIELDS)

# the paper configs of BASELINE.json, shrunk to sizes the oracle finishes in seconds
C1 = dict(n_groups=1, n_replicas=3, wl_enabled=True, wl_start_round=30)
C2 = dict(n_groups=64, n_replicas=3, wl_enabled=True, wl_start_round=30)
C3 = dict(n_groups=40, n_replicas=5, check_quorum=True, wl_enabled=True, wl_start_round=40,
          iso_period=50, iso_len=30, iso_mod=10)
C3_HOT = dict(C3, iso_mod=2)  # half the groups lose their leader every epoch
C4 = dict(n_groups=80, n_replicas=3, quiesce=True, wl_enabled=True, wl_start_round=30,
          wl_active_mod=10, wl_read_permille=900)
C4_DENSE = dict(C4, wl_active_mod=2)
SINGLE = dict(n_groups=4, n_replicas=1, wl_enabled=True, wl_start_round=20,
              wl_read_permille=400)
MIXED = dict(n_groups=30, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
             wl_start_round=25, wl_active_mod=2, wl_read_permille=500, iso_period=37,
             iso_len=20, iso_mod=2, seed=12345)

# engine-only knobs per config: none.  Every config runs with the engine's
# default capacities (ring 64, rq_cap 8, maxm 12, ecap 32, rtr_cap / dri_cap 8);
# what exceeds them goes to the spill tiers (dragonboat_amd/csrc/rbe_spill.h)
ENGINE_EXTRA = {}


def view_diff(a, b, skip=()):
    for f in FIELDS:
        if f in skip:
            continue
        x, y = getattr(a, f), getattr(b, f)
        if hasattr(x, "__len__"):
            x, y = list(x), list(y)
        if x != y:
            return f, x, y
    return None


def run_lockstep(engine, harness, rounds, every=1, full_views=True, skip=()):
    """Step both for `rounds` rounds; compare every `every` rounds.  Returns
    (round, replica, field, engine_value, oracle_value) of the first
    divergence, or None.  `skip` names view fields not compared (the digest of
    an engine running without trace)."""
    done = 0
    while done < rounds:
        k = min(every, rounds - done)
        engine.run(k)
        harness.run(k)
        done += k
        ev, hv = engine.views(), harness.views()
        for i in range(len(hv)):
            if full_views:
                d = view_diff(ev[i], hv[i], skip)
            else:
                d = None if ev[i].digest == hv[i].digest else ("digest", ev[i].digest,
                                                               hv[i].digest)
            if d is not None:
                return (done, i) + d
    return None


def counters_match(ec, hc):
    bad = {}
    for k, v in hc.items():
        if ec.get(k) != v:
            bad[k] = (ec.get(k), v)
    return bad
