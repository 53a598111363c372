"""Session-managed proposals (whole raftpb.Entry values: session fields and
Cmds of any length) on the HIP engine through the C ABI, against the oracle
harness: the scenarios of session_scenarios.py (the CPU tier runs them on the
host build), plus device-side decode of the frames and the decoder's bounds
on hostile input."""
import pytest

import session_scenarios as S
import wire as W
from parity_util import C2, C3

pytestmark = pytest.mark.gpu


def _make(**kw):
    from dragonboat_amd.engine import Engine
    return Engine(device=0, **kw)


@pytest.mark.parametrize("name,kw,ring", [("C2", C2, 64), ("C3", C3, 128)])
def test_gpu_session_proposals_parity(gpu_available, name, kw, ring):
    S.session_proposals_parity(_make, name, kw, ring)


def test_gpu_session_frames_decode(gpu_available):
    S.session_frames_decode(_make, device_decode=True)


@pytest.mark.parametrize("world", [2, 3])
def test_gpu_session_over_transport(gpu_available, world):
    S.session_over_transport(_make, world)


def test_gpu_heap_never_laps_unapplied_entries(gpu_available):
    S.heap_never_laps(_make)


def test_gpu_launch_with_session_entries(gpu_available):
    S.launch_with_session_entries(_make)


def test_gpu_push_forwarded_proposals(gpu_available):
    S.push_forwarded_proposals(_make)


def test_gpu_wire_decode_rejects_oversized_lengths(gpu_available):
    """A length-delimited field whose length is near 2^64 (here inside a
    Message, and as an entry's length) in a frame with valid crc32s is
    ErrInvalidLength in skipRaft / colfer: rbe_wire_decode returns
    RBE_E_CORRUPT instead of wrapping its read position (and never hangs)."""
    from dragonboat_amd.engine import RBE_E_CORRUPT, EngineError
    eng = _make(n_groups=2, n_replicas=3, trace=True)
    eng.step()
    base = W.message_bytes({"type": 17, "to": 2, "from": 1, "cluster_id": 1, "term": 1,
                            "log_term": 0, "log_index": 0, "commit": 0, "reject": 0, "hint": 0,
                            "hint_high": 0}, [])
    huge = bytearray()
    W.put_varint(huge, (1 << 64) - 11)
    bad_msgs = [
        base + b"\x72" + bytes(huge),          # field 14, wire type 2, length 2^64 - 11
        base + b"\x5a" + bytes(huge) + b"\x7f",  # an entry (field 11) of length 2^64 - 11
        base + b"\x61" + b"\x01\x02",           # field 12 wire type 1: 8 bytes past the end
    ]
    for mb in bad_msgs:
        payload = bytearray(b"\x0a")
        W.put_varint(payload, len(mb))
        payload += mb
        with pytest.raises(EngineError) as ei:
            eng.wire_decode(W.frame(bytes(payload)))
        assert getattr(ei.value, "rc", None) == RBE_E_CORRUPT
