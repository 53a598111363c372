"""C5 at its full per-GPU size, rehearsed on one GPU: W = 2 processes share
cuda:0, each a replica-per-GPU engine (rep_world = 2, compacted planes) of
1M groups x 3 — 500k groups per rank, C5's per-GPU share — stepping the
replicas it owns (replica k of group g on rank (g + k) % 2) and exchanging the
cross-rank records every round through ReplicaExchange: counted rounds first,
then the fixed-capacity exchange with chunks sized from them (to_fixed, as
bench.py --xchg-fixed), gloo staged through host memory (RCCL needs one GPU
per rank; the driver's 8-GPU node runs that).  Untraced (the bench path).

Checked as tests/test_gpu_fullsize.py checks C4/C3 at full size: no faults,
at most one leader per (group, term) over both ranks' replicas, commit
monotonicity and processed <= committed <= lastIndex, and the oracle on a
seeded sample of groups (a one-group harness at the group's cluster id
reproduces it exactly: groups are independent)."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
C5_KW = dict(n_groups=1_000_000, n_replicas=3, wl_enabled=True, wl_start_round=30)
EXTRA = dict(rep_compact=True)
ROUNDS, CHECKS, CAL_AT = 90, (60, 90), 45
KEEP = ["role", "term", "committed", "processed", "last_index"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _views(eng, first, cnt):
    from dragonboat_amd.engine import VIEW_DTYPE
    if hasattr(eng, "views_np"):
        return eng.views_np(first, cnt)
    return np.frombuffer(bytes(eng.views()), VIEW_DTYPE)[first:first + cnt]  # host build


def _owned(eng, rank, world, n, G):
    """global replica ids and KEEP fields of the replicas this rank owns"""
    gmap = eng.global_groups().astype(np.int64)
    ids, cols = [], {k: [] for k in KEEP}
    chunk = 600_000 - 600_000 % n
    for first in range(0, eng.n_rep, chunk):
        cnt = min(chunk, eng.n_rep - first)
        v = _views(eng, first, cnt)
        loc = np.arange(first, first + cnt)
        gl, k = loc // n, loc % n
        gg = gmap[gl]
        own = (gg < G) & ((gg + k) % world == rank)
        ids.append((gg * n + k)[own])
        for f in KEEP:
            cols[f].append(v[f][own].copy())
    return np.concatenate(ids), {f: np.concatenate(c) for f, c in cols.items()}


def _worker(rank, world, port, sample, q, kw=C5_KW, cpu=False):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dragonboat_amd.engine import Engine
        from dragonboat_amd.replica import ReplicaExchange
        n = kw["n_replicas"]
        if cpu:  # the host build (a small dry run of this test's logic)
            from soa_cpu.soa import SoaCpu
            eng = SoaCpu(trace=False, rep_world=world, rep_rank=rank, **kw, **EXTRA)
            xch = ReplicaExchange(eng)
        else:
            eng = Engine(device=0, trace=False, rep_world=world, rep_rank=rank, **kw, **EXTRA)
            xch = ReplicaExchange(eng, buf_device="cuda:0", comm_device="cpu")
        gmap = eng.global_groups().astype(np.int64)
        local_of = {int(g): i for i, g in enumerate(gmap) if g < kw["n_groups"]}
        out = []
        done = 0
        for stop in CHECKS:
            while done < stop:
                if done == CAL_AT - 15:
                    xch.reset_peak()
                if done == CAL_AT:
                    xch.to_fixed()
                xch.step()
                if xch.fixed:
                    xch.exchange_fixed()
                else:
                    xch.exchange()
                done += 1
            xch.check()
            if not cpu:
                eng.sync()
            ids, cols = _owned(eng, rank, world, n, kw["n_groups"])
            samp = {}
            for g in sample:
                lg = local_of[int(g)]
                v = _views(eng, lg * n, n).copy()
                samp[int(g)] = [(k, v[k]) for k in range(n) if (int(g) + k) % world == rank]
            out.append((stop, ids, cols, samp))
        nf = eng.fault_summary()[0] if hasattr(eng, "fault_summary") else eng.faults()[0]
        q.put((rank, out, nf, xch.pad_ratio()))
    except Exception as ex:  # surface worker failures in the parent
        q.put((rank, repr(ex), None, None))
        raise
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_gpu_c5_fullsize_rehearsal(gpu_available):
    run_rehearsal(C5_KW)


def run_rehearsal(kw, cpu=False):
    import torch.multiprocessing as mp
    import oracle as O
    world, n, G = 2, kw["n_replicas"], kw["n_groups"]
    sample = sorted(int(x) for x in np.random.default_rng(5).choice(G, 6, replace=False))
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sample, q, kw, cpu))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=900) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
    for rank, out, nf, pad in res:
        assert not isinstance(out, str), f"rank {rank}: {out}"
        assert nf == 0, f"rank {rank}: {nf} faulty replicas"
        assert pad <= 1.5, f"rank {rank}: fixed chunks {pad:.2f}x the records"
    assert all(p.exitcode == 0 for p in procs)
    prev = None
    fields = [f for f in O.VIEW_FIELDS if f != "digest"]
    for ci, stop in enumerate(CHECKS):
        full = {f: np.zeros(G * n, np.uint64) for f in KEEP}
        seen = np.zeros(G * n, bool)
        for _, out, _, _ in res:
            st, ids, cols, _ = out[ci]
            assert st == stop
            assert not seen[ids].any(), "a replica owned by two ranks"
            seen[ids] = True
            for f in KEEP:
                full[f][ids] = cols[f]
        assert seen.all(), "a replica owned by no rank"
        role, term = full["role"].reshape(G, n), full["term"].reshape(G, n)
        lead = role == O.LEADER
        for i in range(n):
            for j in range(i + 1, n):
                both = lead[:, i] & lead[:, j] & (term[:, i] == term[:, j])
                assert not both.any(), f"two leaders in one term: {np.nonzero(both)[0][:8]}"
        assert (lead.sum(axis=1) >= 1).mean() > 0.99, "groups without a leader"
        assert (full["processed"] <= full["committed"]).all()
        assert (full["committed"] <= full["last_index"]).all()
        if prev is not None:
            assert (full["committed"] >= prev).all(), "a commit index moved backwards"
        prev = full["committed"].copy()
        # the sampled groups against a one-group oracle at their cluster id
        for g in sample:
            ref = O.Harness(**dict(kw, n_groups=1, cid_base=1 + g), trace=False)
            ref.run(stop)
            rv = ref.views()
            got = {}
            for _, out, _, _ in res:
                for k, v in out[ci][3][g]:
                    got[k] = v
            assert sorted(got) == list(range(n))
            for k in range(n):
                for f in fields:
                    a = got[k][f]
                    b = getattr(rv[k], f)
                    a = list(a) if np.ndim(a) else int(a)
                    b = list(b) if hasattr(b, "__len__") else b
                    assert a == b, f"round {stop} group {g} replica {k} {f}: engine {a} oracle {b}"
    assert int(prev.max()) > 30, "nothing committed"
