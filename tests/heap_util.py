"""Mixed-size Cmds for the payload-heap tests (include/rbe.h cfg.heap_bytes):
inline (0-16 B), small heap entries and 1-4 KiB ones, as a client's
ProposeEntries batches carry them (peer.go:117-123; the reference bounds a Cmd
only by MaxEntrySize / the payload limit, soft.go:226, requests.go:989-991)."""
import random


def mixed_cmd(rng: random.Random) -> bytes:
    u = rng.random()
    if u < 0.3:
        n = rng.randrange(17)
    elif u < 0.6:
        n = rng.randrange(17, 300)
    else:
        n = rng.randrange(1024, 4097)
    return rng.randbytes(n)


def check_logs(eng, n_groups, n, views, ring, pushed):
    """Every replica's window [max(1, last - ring + 1), last] reads back through
    rbe_get_entry_cmds; a Cmd longer than 16 bytes is one the host pushed, and
    replicas of a group agree on the bytes of every index they share."""
    checked = 0
    for g in range(n_groups):
        seen = {}
        for k in range(n):
            r = g * n + k
            last = views[r].last_index
            lo = max(1, last - ring + 1)
            if last < lo:
                continue
            for i, c in zip(range(lo, last + 1), eng.entry_cmds(r, lo, last)):
                if len(c) > 16:
                    assert c in pushed, (r, i, len(c))
                    checked += 1
                if i <= min(views[g * n + j].committed for j in range(n)):
                    assert seen.setdefault(i, c) == c, (g, k, i)
    return checked
