"""Pin the oracle's in-memory entry window (inmemory.go: merge, entriesToSave,
savedLogTo, restore, appliedLogTo) with the reference's own inmemory_test.go
vectors (tests/golden/inmem.json).  The device engine keeps the same window as
a term/payload ring (rbe_step.h on_replicate, fast_finish); its merge and
savedTo behaviour is pinned against this oracle by the lockstep parity tests."""
import ctypes as C
import json
import os

import pytest

import oracle as O

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "inmem.json")))


def _lib():
    L = O.lib()
    P = C.POINTER
    L.orc_inmem_new.restype = C.c_void_p
    L.orc_inmem_new.argtypes = [C.c_uint64, P(O.OrcEntry), C.c_int, C.c_uint64, C.c_int]
    L.orc_inmem_free.argtypes = [C.c_void_p]
    L.orc_inmem_merge.restype = C.c_int
    L.orc_inmem_merge.argtypes = [C.c_void_p, P(O.OrcEntry), C.c_int]
    L.orc_inmem_op.restype = C.c_int64
    L.orc_inmem_op.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64]
    L.orc_inmem_entries_to_save.restype = C.c_int
    L.orc_inmem_entries_to_save.argtypes = [C.c_void_p, P(O.OrcEntry), C.c_int]
    return L


def _arr(pairs):
    ents = [O.Entry(index=i, term=t) for i, t in pairs]
    return O.entries_array(ents), len(ents)


class InMem:
    def __init__(self, marker, pairs, saved_to=0, shrunk=False):
        self.L = _lib()
        a, n = _arr(pairs)
        self.h = self.L.orc_inmem_new(marker, a, n, saved_to, int(shrunk))

    def __del__(self):
        self.L.orc_inmem_free(self.h)

    def merge(self, pairs):
        a, n = _arr(pairs)
        if self.L.orc_inmem_merge(self.h, a, n) != 0:
            raise O.RaftPanic(self.L.orc_last_error().decode())

    def op(self, o, a=0, b=0):
        v = self.L.orc_inmem_op(self.h, o, a, b)
        assert v != -3, self.L.orc_last_error().decode()
        return v

    last = property(lambda s: s.op(2))
    marker = property(lambda s: s.op(4))
    saved_to = property(lambda s: s.op(5))
    shrunk = property(lambda s: bool(s.op(6)))
    length = property(lambda s: s.op(7))
    first = property(lambda s: s.op(8))

    def term(self, i):
        return self.op(3, i)

    def entries_to_save(self):
        out = (O.OrcEntry * 64)()
        n = self.L.orc_inmem_entries_to_save(self.h, out, 64)
        return [out[i].index for i in range(n)]


@pytest.mark.parametrize("shrunk", G["merge_full_append"]["cases_shrunk"])
def test_merge_full_append(shrunk):
    v = G["merge_full_append"]
    im = InMem(v["marker"], v["entries"], shrunk=shrunk)
    im.merge(v["merge"])
    assert im.shrunk == shrunk
    assert (im.length, im.marker, im.last) == (v["exp_len"], v["exp_marker"], v["exp_last"])


def test_merge_replace():
    v = G["merge_replace"]
    im = InMem(v["marker"], v["entries"], shrunk=v["shrunk"])
    im.merge(v["merge"])
    assert im.shrunk == v["exp_shrunk"]
    assert (im.length, im.marker, im.last) == (v["exp_len"], v["exp_marker"], v["exp_last"])


def test_merge_with_hole_cause_panic():
    v = G["merge_with_hole_cause_panic"]
    im = InMem(v["marker"], v["entries"])
    with pytest.raises(O.RaftPanic):
        im.merge(v["merge"])


def test_merge():
    v = G["merge"]
    im = InMem(v["marker"], v["entries"], shrunk=v["shrunk"])
    im.merge(v["merge"])
    assert im.shrunk == v["exp_shrunk"]
    assert (im.length, im.marker, im.last) == (v["exp_len"], v["exp_marker"], v["exp_last"])
    for i, t in v["exp_terms"]:
        assert im.term(i) == t


@pytest.mark.parametrize("case", G["entries_to_save"]["cases"])
def test_entries_to_save_returns_not_saved_entries(case):
    saved_to, count, first = case
    v = G["entries_to_save"]
    im = InMem(v["marker"], v["entries"], saved_to=saved_to)
    ents = im.entries_to_save()
    assert len(ents) == count
    if first is not None:
        assert ents[0] == first


@pytest.mark.parametrize("case", G["saved_log_to"]["cases"])
def test_saved_log_to_updates_saved_to(case):
    index, term, exp = case
    v = G["saved_log_to"]
    im = InMem(v["marker"], v["entries"], saved_to=v["saved_to"])
    im.op(0, index, term)
    assert im.saved_to == exp


def test_set_saved_to_when_restoring_snapshot():
    v = G["restore_sets_saved_to"]
    im = InMem(v["marker"], v["entries"], saved_to=v["saved_to"])
    im.op(9, *v["snapshot"])
    assert im.saved_to == v["exp_saved_to"]


@pytest.mark.parametrize("case", G["merge_set_saved_to"]["cases"])
def test_merge_set_saved_to(case):
    marker, ents, saved_to, merge, exp = case
    im = InMem(marker, ents, saved_to=saved_to)
    im.merge(merge)
    assert im.saved_to == exp


def test_applied_log_to():
    v = G["applied_log_to"]
    im = InMem(v["marker"], v["entries"], saved_to=v["saved_to"])
    for applied, length, first, shrunk in v["cases"]:
        len1 = im.length
        im.op(1, applied)
        if im.length < len1 and shrunk:
            assert im.shrunk
        assert im.length == length
        assert im.first == first
