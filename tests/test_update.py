"""Pin the Update helpers (peer.go getUpdateCommit / validateUpdate /
setFastApply) with the reference's peer_test.go tables (tests/golden/update.json):
the oracle's list-form restatement and the engine's range-form restatement
(rbe_step.h update_*, which rbe_get_updates uses for RBE_UF_FAST_APPLY),
compiled for the host in the test-only tests/soa_cpu build."""
import ctypes as C
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "update.json")))
u64p = C.POINTER(C.c_uint64)


def _orc():
    L = O.lib()
    L.orc_update_fn.restype = C.c_int
    L.orc_update_fn.argtypes = [C.c_int, C.c_uint64, u64p, C.c_int, u64p, C.c_int, C.c_uint64,
                                C.c_uint64, u64p]
    return L


def _soa():
    from soa_cpu.soa import lib
    L = lib()
    L.soa_update_fn.restype = C.c_int
    L.soa_update_fn.argtypes = [C.c_int] + [C.c_uint64] * 6 + [u64p]
    return L


def _pairs(first, length, terms=None):
    return [(first + i, (terms or {}).get(first + i, 0)) for i in range(length)]


def _flat(pairs):
    a = (C.c_uint64 * max(1, 2 * len(pairs)))()
    for i, (x, t) in enumerate(pairs):
        a[2 * i], a[2 * i + 1] = x, t
    return a


def _call_orc(fn, commit, cents, sents, snap=0, last_applied=0):
    out = (C.c_uint64 * 6)()
    rc = _orc().orc_update_fn(fn, commit, _flat(cents), len(cents), _flat(sents), len(sents),
                              snap, last_applied, out)
    return rc, list(out)


def _call_soa(fn, commit, first_c, len_c, first_s, len_s, snap=0):
    out = (C.c_uint64 * 3)()
    alo, ahi = (first_c, first_c + len_c - 1) if len_c else (1, 0)
    slo, shi = (first_s, first_s + len_s - 1) if len_s else (1, 0)
    rc = _soa().soa_update_fn(fn, commit, alo, ahi, slo, shi, snap, out)
    return rc, list(out)


def test_get_update_commit():
    v = G["get_update_commit"]
    rc, out = _call_orc(0, 0, v["committed"], v["to_save"], v["snapshot_index"], v["last_applied"])
    assert rc == 0
    e = v["exp"]
    assert out[4] == e["stable_snapshot_to"]
    assert out[0] == e["processed"]
    assert (out[2], out[3]) == (e["stable_log_to"], e["stable_log_term"])
    assert out[1] == e["last_applied"]
    c, s = v["committed"], v["to_save"]
    rc, d = _call_soa(0, 0, c[0][0], len(c), s[0][0], len(s), v["snapshot_index"])
    assert (d[0], d[1], d[2]) == (e["processed"], e["stable_log_to"], e["stable_snapshot_to"])


@pytest.mark.parametrize("case", G["validate_update"]["cases"])
def test_validate_update(case):
    commit, fc, lc, fs, ls, panic = case
    rc, _ = _call_orc(1, commit, _pairs(fc, lc), _pairs(fs, ls))
    assert (rc != 0) == panic
    rc, _ = _call_soa(1, commit, fc, lc, fs, ls)
    assert (rc != 0) == panic


@pytest.mark.parametrize("case", G["set_fast_apply"]["cases"])
def test_set_fast_apply(case):
    snap, fc, lc, fs, ls, fast = case
    rc, out = _call_orc(2, 0, _pairs(fc, lc), _pairs(fs, ls), 1 if snap else 0)
    assert rc == 0 and bool(out[0]) == fast
    rc, out = _call_soa(2, 0, fc, lc, fs, ls, 1 if snap else 0)
    assert rc == 0 and bool(out[0]) == fast
