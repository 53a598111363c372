"""Replica-per-GPU mode (C5) on CPU: W processes (gloo), each stepping the
replicas it owns with the host build of the device step (tests/soa_cpu) and
moving cross-rank messages with dragonboat_amd.replica.ReplicaExchange — the
same record format, pack/clear/scatter functions (rbe_xchg.h) and collective
sequence the GPU path uses.  Every owned replica must equal, field by field
and round by round at the checkpoints, the oracle harness stepping all
replicas in one process; the counters summed over ranks must equal the
oracle's."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {
    # steady replication, 3 replicas over 2 ranks (two replicas share a rank)
    "C2_w2": (dict(n_groups=24, n_replicas=3, wl_enabled=True, wl_start_round=30), 2, 200, {}),
    # quiesce + 9:1 reads, every replica of a group on its own rank
    "C4_w3": (dict(n_groups=30, n_replicas=3, quiesce=True, wl_enabled=True, wl_start_round=30,
                   wl_active_mod=2, wl_read_permille=900), 3, 300, {}),
    # 5 replicas, check-quorum, elections from scratch, over 4 ranks
    "N5_w4": (dict(n_groups=16, n_replicas=5, check_quorum=True, quiesce=True, wl_enabled=True,
                   wl_start_round=25, wl_active_mod=2, wl_read_permille=500, seed=777), 4, 300,
              dict()),
    # C3 with its isolation schedule (leaders cut off for 30 of every 50
    # rounds): each rank knows only its own replicas' roles, so the epoch's
    # leader bits are ORed over ranks before the step (ReplicaExchange.iso_sync)
    "C3_iso_w2": (dict(n_groups=20, n_replicas=5, check_quorum=True, wl_enabled=True,
                       wl_start_round=40, iso_period=50, iso_len=30, iso_mod=3), 2, 300,
                  dict()),
    "C3_iso_w4": (dict(n_groups=20, n_replicas=5, check_quorum=True, wl_enabled=True,
                       wl_start_round=40, iso_period=50, iso_len=30, iso_mod=3), 4, 300,
                  dict()),
    # compacted planes (rep_compact): 3 replicas over 4 ranks, each rank holds
    # the 3/4 of the groups it steps a replica of (W = 8: 3/8); n_groups not a
    # multiple of W leaves padding groups; the second case adds the isolation
    # schedule, whose leader bits are exchanged by global group
    # a group of 7 over 3 ranks: slot 6's count word sits in the sender's own
    # place of the 6-word outbox header (cnt_widx)
    "N7_w3": (dict(n_groups=12, n_replicas=7, check_quorum=True, quiesce=True, wl_enabled=True,
                   wl_start_round=25, wl_active_mod=2, wl_read_permille=500, iso_period=41,
                   iso_len=20, iso_mod=2), 3, 300, dict()),
    "C2_w4c": (dict(n_groups=22, n_replicas=3, wl_enabled=True, wl_start_round=30), 4, 200,
               dict(rep_compact=True)),
    "C3_iso_w4c": (dict(n_groups=22, n_replicas=3, check_quorum=True, wl_enabled=True,
                        wl_start_round=40, iso_period=50, iso_len=30, iso_mod=3), 4, 300,
                   dict(rep_compact=True)),
    # tiny plane capacities (rbe_spill.h): lists past maxm and entries past ecap
    # cross ranks as spill-heap records, each landing at the granule its
    # sender chose in the sender rank's share of the heap (kXSpill)
    "MIXED_tiny_w2": (dict(n_groups=12, n_replicas=5, check_quorum=True, quiesce=True,
                           wl_enabled=True, wl_start_round=25, wl_active_mod=2,
                           wl_read_permille=500, iso_period=37, iso_len=20, iso_mod=2,
                           seed=12345), 2, 300,
                      dict(maxm=1, ecap=1, rtr_cap=1, dri_cap=1, rq_cap=1, ring=8)),
    "MIXED_tiny_w3": (dict(n_groups=12, n_replicas=5, check_quorum=True, quiesce=True,
                           wl_enabled=True, wl_start_round=25, wl_active_mod=2,
                           wl_read_permille=500, iso_period=37, iso_len=20, iso_mod=2,
                           seed=12345), 3, 300,
                      dict(maxm=2, ecap=2, rq_cap=4, ring=8)),
}
CHECK_EVERY = 50


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, gpu, trace, q, fixed=False):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from parity_util import FIELDS
        from dragonboat_amd.replica import ReplicaExchange
        kw, _, rounds, extra = CASES[name]
        # counted exchange: tiny caps exercise grow(); fixed exchange: capacities
        # that never grow (initial_caps), counts travel in the chunk headers;
        # "cal": counted rounds first, then chunks sized from their peak counts
        # (to_fixed, as bench.py --xchg-fixed does)
        # "ovf": fixed chunks of 4 records, so most rounds outgrow them and take
        # the counted second pass (exchange_fixed's repair)
        cal, ovf = fixed == "cal", fixed == "ovf"
        if cal:
            fixed = False
        caps = [4, 4, 4] if ovf else None if (fixed or cal) else [8, 8, 8]
        fixed = bool(fixed)
        if gpu:  # the HIP engine, records staged through host memory for gloo
            from dragonboat_amd.engine import Engine
            eng = Engine(device=0, trace=trace, rep_world=world, rep_rank=rank, **kw, **extra)
            xch = ReplicaExchange(eng, buf_device="cuda:0", comm_device="cpu", caps=caps,
                                  fixed=fixed)
        else:
            from soa_cpu.soa import SoaCpu
            eng = SoaCpu(trace=trace, rep_world=world, rep_rank=rank, **kw, **extra)
            xch = ReplicaExchange(eng, caps=caps, fixed=fixed)
        snaps = []
        n = kw["n_replicas"]
        gmap = eng.global_groups()  # local group -> global group (rep_compact)
        for done in range(CHECK_EVERY, rounds + 1, CHECK_EVERY):
            if cal and done == 2 * CHECK_EVERY:
                xch.reset_peak()
            if cal and done == 3 * CHECK_EVERY:
                xch.to_fixed(1.5)
            xch.run(CHECK_EVERY)
            vs = eng.views()
            own = {}
            for i in range(len(vs)):
                gl, k = divmod(i, n)
                gg = int(gmap[gl])
                if gg >= kw["n_groups"] or (gg + k) % world != rank:
                    continue
                own[gg * n + k] = tuple(tuple(getattr(vs[i], f))
                                        if hasattr(getattr(vs[i], f), "__len__")
                                        else getattr(vs[i], f) for f in FIELDS)
            snaps.append((done, own))
        nf = eng.fault_summary()[0] if gpu else eng.faults()[0]
        if cal:
            assert xch.fixed
        if ovf:
            assert xch.repaired > 0, "no round outgrew its chunks"
        q.put((rank, snaps, eng.counters(), nf,
               [xch.bytes_sent] * 3 if fixed else xch.records_sent))
    except Exception as ex:  # surface worker failures in the parent
        q.put((rank, repr(ex), None, None, None))
        raise
    finally:
        dist.barrier()
        dist.destroy_process_group()


def run_case(name, gpu=False, trace=True, fixed=False):
    import oracle as O
    from parity_util import FIELDS
    kw, world, rounds, _ = CASES[name]
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, gpu, trace, q, fixed))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, snaps, _, _, _ in res:
        assert not isinstance(snaps, str), f"rank {rank}: {snaps}"
    assert all(p.exitcode == 0 for p in procs)

    ref = O.Harness(**kw)
    n_rep = kw["n_groups"] * kw["n_replicas"]
    covered = set()
    for k, done in enumerate(range(CHECK_EVERY, rounds + 1, CHECK_EVERY)):
        ref.run(CHECK_EVERY)
        hv = ref.views()
        for rank, snaps, _, _, _ in res:
            assert snaps[k][0] == done
            for i, got in snaps[k][1].items():
                covered.add(i)
                want = tuple(tuple(getattr(hv[i], f)) if hasattr(getattr(hv[i], f), "__len__")
                             else getattr(hv[i], f) for f in FIELDS)
                bad = [(f, a, b) for f, a, b in zip(FIELDS, got, want)
                       if a != b and (trace or f != "digest")]
                if bad:
                    pytest.fail(f"{name}: round {done} replica {i} (rank {rank}) differs: "
                                f"{bad[:3]}")
    assert covered == set(range(n_rep))
    hc = ref.counters()
    for key, v in hc.items():
        assert sum(r[2][key] for r in res) == v, key
    assert all(r[3] == 0 for r in res), "faults"
    # cross-rank traffic actually flowed: count words, messages and entries
    sent = [sum(r[4][t] for r in res) for t in range(3)]
    assert all(s > 0 for s in sent), sent


@pytest.mark.parametrize("name", list(CASES))
def test_replica_per_rank_matches_oracle(name):
    run_case(name)


def test_replica_per_rank_untraced():
    """Without trace (the bench paths: lazy quiesced ticks, no digest)."""
    run_case("C4_w3", trace=False)


@pytest.mark.parametrize("name", ["C2_w2", "N5_w4"])
def test_replica_fixed_exchange_matches_oracle(name):
    """The fixed-capacity exchange (rbe_xchg_pack_fixed: equal chunks whose
    headers carry the counts, no host-side count read)."""
    run_case(name, fixed=True)


@pytest.mark.parametrize("name", ["C2_w2", "N5_w4", "MIXED_tiny_w2"])
def test_replica_fixed_exchange_overflow_repaired(name):
    """Fixed chunks far too small for the rounds: every round that outgrows
    them is repaired by a counted exchange of the same round (read-and-clear
    rbe_xchg_status), bit-exact with the oracle; an overflow never
    invalidates the run."""
    run_case(name, fixed="ovf")


def test_replica_calibrated_fixed_exchange():
    """Counted rounds, then the fixed exchange with chunks sized from the
    counted rounds' mean counts (ReplicaExchange.to_fixed): still bit-exact
    (rounds above the mean take the counted second pass)."""
    run_case("C2_w2", fixed="cal")
