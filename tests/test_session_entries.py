"""Session-managed proposals (whole raftpb.Entry values: session fields and
Cmds of any length) on the CPU tier: the device step compiled for the host
(tests/soa_cpu) with the engine's staging code (rbe_host.h), against the
oracle harness.  The scenarios are in session_scenarios.py;
test_gpu_session_entries.py runs them on the HIP engine."""
import pytest

import session_scenarios as S
from parity_util import C2, C3
from soa_cpu.soa import SoaCpu


@pytest.mark.parametrize("name,kw,ring", [("C2", C2, 64), ("C3", C3, 128)])
def test_session_proposals_parity(name, kw, ring):
    S.session_proposals_parity(SoaCpu, name, kw, ring)


def test_session_frames_decode_to_outbox_records():
    S.session_frames_decode(SoaCpu)


@pytest.mark.parametrize("world", [2, 3])
def test_session_proposals_over_transport(world):
    S.session_over_transport(SoaCpu, world)


def test_session_entries_need_a_heap():
    S.session_entries_need_a_heap(SoaCpu)


def test_heap_never_laps_unapplied_entries():
    S.heap_never_laps(SoaCpu)


def test_launch_with_session_entries():
    S.launch_with_session_entries(SoaCpu)


def test_push_messages_carries_forwarded_proposals():
    S.push_forwarded_proposals(SoaCpu)


def test_oracle_decoder_rejects_oversized_lengths():
    """The wire restatement follows skipRaft's bounds (raft.pb.go): a length
    or fixed-width field past the end of its buffer is ErrInvalidLength, not
    a silent truncation (the GPU twin checks rbe_wire_decode on the same
    frames, test_gpu_session_entries.py)."""
    import wire as W
    base = W.message_bytes({"type": 17, "to": 2, "from": 1, "cluster_id": 1, "term": 1,
                            "log_term": 0, "log_index": 0, "commit": 0, "reject": 0, "hint": 0,
                            "hint_high": 0}, [])
    huge = bytearray()
    W.put_varint(huge, (1 << 64) - 11)
    for mb in (base + b"\x72" + bytes(huge), base + b"\x5a" + bytes(huge) + b"\x7f",
               base + b"\x61" + b"\x01\x02"):
        payload = bytearray(b"\x0a")
        W.put_varint(payload, len(mb))
        payload += mb
        with pytest.raises(ValueError):
            W.batch_decode(W.frames_decode(W.frame(bytes(payload)))[0])
