"""Session-managed proposals through the engine boundary: scenarios shared
by the CPU tier (tests/test_session_entries.py, the device step compiled for
the host) and the GPU tier (tests/test_gpu_session_entries.py, the HIP engine
through the C ABI), each against the oracle harness.  `make(**cfg)` builds
the engine under test.

A NodeHost proposal is a whole raftpb.Entry (raft.pb.go:589-598): the client
layer stamps Key, ClientID, SeriesID and RespondedTo on it (requests.go:
994-997) and they travel with the entry through replication and the wire
(raft_optimized.go:214-276).  The engine keeps such an entry as a payload-heap
record, so replication copies a 24-B reference.  Parity here is the whole
path: proposals with session fields (values from 1 to 2^64 - 1, across
colfer's 9-byte form at 2^49) and 0-4 KiB Cmds pushed at leaders AND
followers (a follower forwards them to its leader, raft.go:1841-1853), every
replica field and trace digest round by round (the digest folds each entry's
fingerprint, which covers the session fields), the log windows read back with
every field equal to the oracle's LogDB, and the last round's frames decoded
by oracle/wire.py (and by rbe_wire_decode on the device) equal to the outbox
records."""
import random

import pytest

import oracle as O
from dragonboat_amd.engine import RBE_E_INVALID, RBE_E_NOMEM, InputError, make_entry
from heap_util import mixed_cmd
from input_util import plan_round, run_driven, session_entry, apply_engine, apply_oracle
from parity_util import C2, view_diff
from session_util import check_entry_records, check_outbox_decodes
from transport_util import owner, run_transport

DRIVEN = dict()


def _pair(make, kw, heap_bytes=64 << 20, **eng_more):
    eng = make(trace=True, heap_bytes=heap_bytes, **dict(kw, **DRIVEN, **eng_more))
    return eng, O.Harness(**kw)


def session_proposals_parity(make, name, kw, ring):
    kw = dict(kw, n_groups=8, ext_inputs=True)
    eng, ref = _pair(make, kw, ring=ring)
    pushed = set()

    def keep(ops):
        for kind, _, a in ops:
            if kind == "prop":
                pushed.update(bytes(e.cmd) for e in a)

    d = run_driven(eng, ref, 140, seed=11, cmd=mixed_cmd, on_ops=keep, density=0.25,
                   session=True)
    assert d is None, f"{name}: first divergence {d}"
    assert eng.faults()[0] == 0
    checked, with_session = check_entry_records(eng, ref, kw["n_groups"], kw["n_replicas"], ring,
                                                pushed)
    assert checked > 200 and with_session > 50, (checked, with_session)


def session_frames_decode(make, device_decode=False):
    """Every few rounds of a session-proposal run, the frames rbe_wire_encode
    writes decode (oracle/wire.py) to exactly the outbox records, session
    fields and forwarded Propose entries included."""
    kw = dict(C2, n_groups=8, ext_inputs=True)
    eng, ref = _pair(make, kw)
    rng = random.Random(5)
    views = ref.views()
    seen = ses = props = 0
    for rnd in range(90):
        ops = plan_round(rng, eng.n_rep, 3, rnd, views, False, 0.3, None, mixed_cmd,
                         session=True, props_only=True)
        apply_engine(eng, ops)
        apply_oracle(ref, ops)
        eng.step()
        ref.step()
        views = ref.views()
        if rnd % 3 == 0:
            a, b, c = check_outbox_decodes(eng, kw["n_groups"], 3, gpb=3,
                                           device_decode=device_decode)
            seen, ses, props = seen + a, ses + b, props + c
    ev = eng.views()
    assert all(view_diff(ev[i], views[i]) is None for i in range(eng.n_rep))
    assert seen > 200 and ses > 50 and props > 5, (seen, ses, props)


def session_over_transport(make, world, wire=False):
    """W engines, each stepping the replicas it owns, exchange every message
    (forwarded Proposes and Replicates with session entries and KiB Cmds
    included) through rbe_get_outbox / rbe_push_messages; the receiver stages
    the entries in its own payload heap.  Every owned replica equals the
    oracle's."""
    kw = dict(C2, n_groups=9, ext_inputs=True)
    engs = [make(trace=True, rep_world=world, rep_rank=r, heap_bytes=64 << 20,
                   **dict(kw, **DRIVEN)) for r in range(world)]
    ref = O.Harness(**kw)
    rng = random.Random(world)
    n_rep = kw["n_groups"] * 3

    def inputs(rnd):
        return plan_round(rng, n_rep, 3, rnd, None, False, 0.25, None, mixed_cmd,
                          session=True, props_only=True)

    d, moved = run_transport(engs, ref, 3, 100, every=10, inputs=inputs, wire=wire)
    assert d is None, f"first divergence {d}"
    assert moved > 300
    for e in engs:
        assert e.faults()[0] == 0
    # each engine's log windows hold the oracle's entries, session fields included
    views = ref.views()
    for rank, e in enumerate(engs):
        for r in range(n_rep):
            g, k = divmod(r, 3)
            if owner(g, k, world) != rank:
                continue
            last = views[r].last_index
            lo = max(1, last - 63)
            got = e.entry_records(r, lo, last)
            exp = ref.persisted_entries(r, lo, last)
            for a, x in zip(got, exp):
                assert (a["index"], a["term"], a["key"], a["client_id"], a["series_id"],
                        a["responded_to"], a["cmd"][:64]) == (
                    x.index, x.term, x.key, x.client_id, x.series_id, x.responded_to, x.cmd[:64])


def session_entries_need_a_heap(make):
    """Without a payload heap an entry with session fields (or a Cmd over 16
    bytes) has nowhere to live: the batch is refused whole."""
    eng = make(trace=True, n_groups=2, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError) as ei:
        eng.push_proposals([0], [[O.Entry(cmd=b"x", key=7)]])
    assert ei.value.rc == RBE_E_INVALID
    eng.push_proposals([0], [[O.Entry(cmd=b"x")]])  # no session fields: inline
    eng.step()


def heap_never_laps(make):
    """The state machine stops applying (ext_apply, applied index frozen):
    every record above the groups' low mark stays live, so pushes that would
    lap one get RBE_E_NOMEM, nothing is overwritten, and every entry still
    reads back with the bytes the host proposed (inmemory.go:116-166: an entry
    lives until it is saved and applied).  Once the state machine catches
    up, the heap takes proposals again."""
    kw = dict(C2, n_groups=2, ext_inputs=True, ext_apply=True)
    eng, ref = _pair(make, kw, heap_bytes=96 << 10)
    rng = random.Random(3)
    leaders = []
    pushed, nomem = {}, 0
    rv = ref.views()
    for rnd in range(60):
        ops = []
        if rnd < 25:  # the state machine keeps up (campaigns need committed <= applied)
            ops = [("applied", r, rv[r].processed) for r in range(eng.n_rep)]
            apply_engine(eng, ops)
        else:  # ... then stops applying
            if not leaders:
                leaders = [r for r, v in enumerate(rv) if v.role == O.LEADER]
            for r in leaders:
                e = session_entry(rng, lambda g: g.randbytes(3000))
                try:
                    eng.push_proposals([r], [[e]])
                except InputError as err:
                    assert err.rc == RBE_E_NOMEM
                    nomem += 1
                    continue
                pushed[bytes(e.cmd)] = e
                ops.append(("prop", r, [e]))
        apply_oracle(ref, ops)
        eng.step()
        ref.step()
        ev, rv = eng.views(), ref.views()
        assert all(view_diff(ev[i], rv[i]) is None for i in range(eng.n_rep)), rnd
    assert len(leaders) == 2
    assert nomem > 0, "the heap never filled up"
    # nothing was lapped: every entry of every window reads back intact
    for r in range(eng.n_rep):
        last = rv[r].last_index
        for x in eng.entry_records(r, max(1, last - 255), last):
            if len(x["cmd"]) > 16:
                assert x["cmd"] in pushed and pushed[x["cmd"]].key == x["key"]
    # the state machine catches up: applied = processed, the records die and
    # the heap takes proposals again
    ops = [("applied", r, rv[r].processed) for r in range(eng.n_rep)]
    apply_engine(eng, ops)
    apply_oracle(ref, ops)
    eng.step()
    ref.step()
    e = session_entry(rng, lambda g: g.randbytes(3000))
    eng.push_proposals([leaders[0]], [[e]])


def launch_with_session_entries(make):
    """rbe_launch over a LogDB whose entries carry session fields and long
    Cmds (they go to the payload heap) reads back every field."""
    eng = make(trace=True, n_groups=2, n_replicas=3, ext_inputs=True, heap_bytes=1 << 20)
    ents = [(1, 1, 0, b"a" * 40, 5, 6, 7, 8), (2, 1, 0, b"b", 1 << 60, 0, 3, 0),
            (3, 2, 2, b"", 0, 0, 0, 0)]
    eng.launch([0], [(2, 0, 2, 3)], [ents])
    got = eng.entry_records(0, 1, 3)
    assert [(x["index"], x["term"], x["type"], x["cmd"], x["key"], x["client_id"],
             x["series_id"], x["responded_to"]) for x in got] == ents
    plain = make(trace=True, n_groups=2, n_replicas=3, ext_inputs=True)
    with pytest.raises(InputError):  # session fields need the payload heap
        plain.launch([1], [(2, 0, 1, 1)], [[(1, 1, 0, b"c", 9, 0, 0, 0)]])


def push_forwarded_proposals(make):
    """rbe_push_messages takes a follower's forwarded Propose with its
    entries (raft.go:1841-1853), Cmds over 16 bytes and session fields
    included; a non-Replicate, non-Propose message with entries is refused."""
    from dragonboat_amd.engine import RbeMessage
    kw = dict(n_groups=4, n_replicas=3, wl_enabled=False)
    e = make(trace=True, rep_world=2, rep_rank=0, heap_bytes=1 << 20, ext_inputs=True, **kw)
    e.step()
    # group 0: node 1 owned by rank 0, node 2 by rank 1
    prop = RbeMessage(type=7, to=1, from_=2, n_entries=2)
    ents = [make_entry(cmd=b"q" * 100, key=1 << 50, client_id=9), make_entry(cmd=b"z")]
    e.push_messages([0], [prop], ents, [b"q" * 100, b"z"])
    with pytest.raises(InputError):
        e.push_messages([0], [RbeMessage(type=17, to=1, from_=2, n_entries=1)],
                        [make_entry(cmd=b"x")], [b"x"])
