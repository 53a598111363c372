"""The C-ABI boundary (include/rbe.h, libdragonboat_amd.so) without a GPU:
the library loads, exports exactly what the header declares, validates
configurations like config.Validate, and fails loudly (no CPU fallback) when
no gfx950 device is present."""
import ctypes as C
import os
import re

import pytest

from dragonboat_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rbe.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*int\s+(rbe_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_binding_surface():
    assert header_functions() == sorted(E.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = E.load_library()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.rbe_abi_version() == E.RBE_ABI_VERSION


def test_library_is_gfx950_code_object():
    blob = open(E.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_footprint_and_validation():
    lib = E.load_library()
    b = C.c_uint64()
    cfg = E.make_config(n_groups=1000, n_replicas=3)
    assert lib.rbe_footprint(C.byref(cfg), C.byref(b)) == 0
    assert b.value > 1000 * 3 * 64
    big = C.c_uint64()
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=2000, n_replicas=3)),
                             C.byref(big)) == 0
    assert big.value > b.value
    # config.Validate (config/config.go:173-208): ElectionRTT > 2 * HeartbeatRTT
    bad = E.make_config(n_groups=10, election_rtt=2, heartbeat_rtt=1)
    assert lib.rbe_footprint(C.byref(bad), C.byref(b)) == -1
    for n in range(1, 8):  # group sizes 1..7
        assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, n_replicas=n)),
                                 C.byref(b)) == 0
    for n in (0, 8):
        assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, n_replicas=n)),
                                 C.byref(b)) == -1
    # spare slots (n_voters < n_replicas) need membership
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, n_replicas=5, n_voters=3)),
                             C.byref(b)) == -1
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, n_replicas=5, n_voters=3,
                                                   membership=True)), C.byref(b)) == 0
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=0)), C.byref(b)) == -1
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, ring=48)), C.byref(b)) == -1
    wrong_abi = E.make_config(n_groups=10)
    wrong_abi.abi_version = 99
    assert lib.rbe_footprint(C.byref(wrong_abi), C.byref(b)) == -1
    # node snapshots: accepted, with their planes in the footprint
    snap = C.c_uint64()
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=1000, snapshot_entries=16,
                                                   compaction_overhead=4)), C.byref(snap)) == 0
    assert snap.value >= b.value + 1000 * 3 * (64 + 3 * 8)
    # host-driven snapshots (ext_apply), also with host-driven commits (ext_commit)
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, snapshot_entries=16, ext_inputs=True,
                                                   ext_apply=True)), C.byref(b)) == 0
    assert lib.rbe_footprint(C.byref(E.make_config(n_groups=10, snapshot_entries=16, ext_inputs=True,
                                                   ext_apply=True, ext_commit=True)),
                             C.byref(b)) == 0


def test_null_handles_are_rejected():
    lib = E.load_library()
    assert lib.rbe_step(None) == -1
    assert lib.rbe_run(None, 3) == -1
    assert lib.rbe_destroy(None) == 0


def test_struct_layouts_match_header():
    # sizes fixed by include/rbe.h (8-byte aligned C structs)
    assert C.sizeof(E.RbeMessage) == 8 + 9 * 8 + 8
    assert C.sizeof(E.RbeEntry) == 40 + 4 * 8  # + Key, ClientID, SeriesID, RespondedTo
    assert C.sizeof(E.RbeReadyToRead) == 24
    assert C.sizeof(E.RbeUpdate) == 8 * 8 + 10 * 4
    # and every binding struct against the library's own sizeof (rbe_abi_sizes)
    lib = E.load_library()
    sz = (C.c_uint64 * 6)()
    assert lib.rbe_abi_sizes(sz, 6) == 6
    assert list(sz) == [C.sizeof(t) for t in (E.RbeConfig, E.RbeReplicaView, E.RbeUpdate,
                                               E.RbeMessage, E.RbeEntry, E.RbeReadyToRead)]


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(E.EngineError):
        E.Engine(n_groups=4, n_replicas=3)


def test_missing_library_raises(tmp_path):
    with pytest.raises(E.EngineError):
        E.load_library(str(tmp_path / "nope.so"))
