"""Restart replicas from the oracle's persisted state on an engine (the HIP
engine or the host build) and in the oracle harness, the way a dragonboat node
restarts: Peer.Launch over its LogDB (peer.go:64-86, initial = newNode =
false).  The engine is handed exactly what the node would read back: pb.State
and the tail of the log (its in-memory window)."""


def restart(eng, ref, replicas, ring, snapshots=False):
    """`snapshots`: the LogDB may be compacted; the launch state carries its
    marker and latest snapshot (harness_snapshot_state) and the entries above
    the marker.  `ring` None: the whole LogDB (the engine keeps what is below
    its ring in the cold log), else only its last `ring` entries."""
    states, ents = [], []
    for r in replicas:
        term, vote, commit, last = ref.persisted(r)
        snap = ()
        lo = 1 if ring is None else max(1, last - ring + 1)
        if snapshots:
            marker, mterm, ssi, sst = ref.snapshot_state(r)[:4]
            # the LogDB's membership (its snapshot's; all voters without one)
            snap = (marker, mterm, ssi, sst, ref.snapshot_state(r)[6])
            lo = max(lo, marker + 1)
        es = ref.persisted_entries(r, lo, last) if last >= lo else []
        states.append((term, vote, commit, last) + snap)
        ents.append([(e.index, e.term, e.type, e.cmd) for e in es])
    eng.launch(replicas, states, ents)
    for r in replicas:
        ref.restart(r)
