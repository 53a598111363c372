"""Host transport loop over the Peer.Handle boundary (rbe_get_outbox /
rbe_push_messages): W engines in one process, each stepping the replicas it
owns (replica k of group g on engine (g + k) % W, rep_world = W); after every
round each engine's outbound messages to replicas stepped elsewhere are read
in raftpb form and delivered to the owning engine as its next round's inbound
batch, as dragonboat's transport would carry them between NodeHosts
(node.go:888-905 → nodehost.go:1724 → node.handleReceivedMessages)."""
from parity_util import view_diff


def owner(g, k, world):
    return (g + k) % world


def deliver(engs, n, n_rep):
    """One transport hop: every engine's owned senders → the owners of the
    destinations.  Returns the number of messages moved."""
    world = len(engs)
    batches = [([], [], [], []) for _ in range(world)]
    moved = 0
    for rank, e in enumerate(engs):
        for r in range(n_rep):
            g, k = divmod(r, n)
            if owner(g, k, world) != rank:
                continue
            msgs, ents, cmds = e.outbox(r)
            ei = 0
            for m in msgs:
                ne = m.n_entries
                dst = owner(g, m.to - 1, world)
                if dst != rank:
                    gs, ms, es, cs = batches[dst]
                    gs.append(g)
                    ms.append(m)
                    es.extend(ents[ei:ei + ne])
                    cs.extend(cmds[ei:ei + ne])
                    moved += 1
                ei += ne
            assert ei == len(ents)
    for rank, e in enumerate(engs):
        gs, ms, es, cs = batches[rank]
        e.push_messages(gs, ms, es, cs)
    return moved


def encode_for(e, rank):
    """The wire stream of engine e's last round for the replicas of `rank`
    (rbe_wire_encode with dst_rank + rbe_wire_fetch, or the host build's twin)."""
    if hasattr(e, "wire_fetch"):
        data, _ = e.wire_fetch(e.wire_encode(dst_rank=rank))
    else:
        data, _ = e.wire_encode(dst_rank=rank)
    return data


def deliver_wire(engs):
    """One transport hop as bytes: every engine encodes, per destination
    engine, the MessageBatch frames of its owned senders (rbe_wire_encode),
    and each destination takes the concatenated streams of all its sources in
    one rbe_wire_ingest, on the device.  Returns (messages moved, bytes)."""
    moved = nbytes = 0
    for rank, e in enumerate(engs):
        data = b"".join(encode_for(src, rank) for r2, src in enumerate(engs) if r2 != rank)
        st = e.wire_ingest(data)
        moved += st["messages"] - st["dropped"]
        nbytes += len(data)
    return moved, nbytes


def run_transport(engs, ref, n, rounds, every=25, inputs=None, wire=False):
    """Step W engines and the oracle in lockstep with a transport hop after
    each round (wire=True: as encoded frames through rbe_wire_ingest, else
    through rbe_get_outbox / rbe_push_messages); compare every owned replica
    with the oracle every `every` rounds.  `inputs(rnd)` returns host input ops for the round (input_util
    plan_round form), applied to the owning engine and the oracle.  Returns
    (first divergence or None, messages moved)."""
    from input_util import apply_engine, apply_oracle
    world = len(engs)
    n_rep = len(ref.views())
    moved = 0
    for done in range(1, rounds + 1):
        if inputs:
            ops = inputs(done - 1)
            for rank, e in enumerate(engs):
                apply_engine(e, [op for op in ops if owner(op[1] // n, op[1] % n, world) == rank])
            apply_oracle(ref, ops)
        iso = [e.iso_leaders() for e in engs]  # isolation epochs: the ORed leader bits
        if iso[0] is not None:
            bits = iso[0].copy()
            for b in iso[1:]:
                bits |= b
            for e in engs:
                e.set_iso_leaders(bits)
        for e in engs:
            e.step()
        ref.step()
        moved += deliver_wire(engs)[0] if wire else deliver(engs, n, n_rep)
        if done % every and done != rounds:
            continue
        hv = ref.views()
        evs = [e.views() for e in engs]
        for r in range(n_rep):
            g, k = divmod(r, n)
            d = view_diff(evs[owner(g, k, world)][r], hv[r])
            if d is not None:
                return (done, r) + d, moved
    return None, moved
