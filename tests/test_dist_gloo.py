"""The N>1 path on CPU (gloo, world_size 2): group-per-GPU sharding by
cluster id and the statistics reduction bench.py uses.  Each rank steps its
shard with the host build of the device step (tests/soa_cpu) using exactly
the engine configuration bench.py would give that rank; the union of the
shards must equal one unsharded run group by group, and the reduced counters
must equal the unsharded counters."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from dragonboat_amd.shard import cluster_ids, owner_of, reduce_results, shard_params

HERE = os.path.dirname(os.path.abspath(__file__))
KW = dict(n_replicas=3, quiesce=True, wl_enabled=True, wl_start_round=30, wl_active_mod=3,
          wl_read_permille=600)
GROUPS = 24
ROUNDS = 120


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_rule_is_fixed_partitioner():
    world = 4
    seen = set()
    for r in range(world):
        ids = cluster_ids(r, world, 10)
        assert all(owner_of(c, world) == r for c in ids)
        seen.update(ids)
    assert seen == set(range(1, 41))
    assert shard_params(0, 1) == (1, 1)
    with pytest.raises(ValueError):
        shard_params(2, 2)


def _worker(rank, world, port, q):
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from soa_cpu.soa import SoaCpu
    base, stride = shard_params(rank, world)
    eng = SoaCpu(n_groups=GROUPS // world, cid_base=base, cid_stride=stride, trace=True, **KW)
    eng.run(ROUNDS)
    c = eng.counters()
    wall, sums = reduce_results(dist, float(rank + 1), [c["steps"], c["committed"],
                                                      c["reads_confirmed"]])
    digests = [v.digest for v in eng.views()]
    q.put((rank, wall, sums, digests))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_matches_unsharded():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    from soa_cpu.soa import SoaCpu
    full = SoaCpu(n_groups=GROUPS, trace=True, **KW)
    full.run(ROUNDS)
    fc = full.counters()
    fd = np.array([v.digest for v in full.views()], dtype=np.uint64).reshape(GROUPS, 3)
    for rank, wall, sums, digests in res:
        assert wall == float(world)  # max over ranks
        assert sums == [float(fc["steps"]), float(fc["committed"]), float(fc["reads_confirmed"])]
        d = np.array(digests, dtype=np.uint64).reshape(GROUPS // world, 3)
        # engine group g on rank r is cluster 1 + r + g * world = full-run group r + g * world
        for g in range(GROUPS // world):
            assert (d[g] == fd[rank + g * world]).all()
