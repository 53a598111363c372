#!/usr/bin/env python3
"""Benchmark: Raft group-steps/s + committed entries/s on MI355X.

Workload (BASELINE.json `metric`, configs[3] "C4"): per GPU 1M Raft groups x 3
replicas, Quiesce on, 90% of groups idle (quiesced after 200 ticks), 10%
active with a 9:1 ReadIndex:propose mix, 16-byte proposals, ElectionRTT=10,
HeartbeatRTT=1.  A "step" is one lockstep round of every replica of every
group (one k_step launch): inbox → raft protocol → outbox + Update.

Multi-GPU (torchrun, one process per GPU): groups shard by cluster id
(cid % N == rank, dragonboat's FixedPartitioner); no data-path collective;
per-GPU work is fixed (weak scaling).  `value` = group-steps of all ranks ÷
the max-over-ranks timed-region wall time.

Outputs ONE JSON line on rank 0 (see DESIGN.md §Measurement for the byte model).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Raft group-steps/sec + committed entries/sec (1M groups×3), 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# SURVEY.md §8(d) algorithmic bytes per event
BYTES = {
    "active_ticks": 128,     # core state read 64 B + write 64 B per active step
    "quiesced_ticks": 12,    # quiesced tick: 8 B read + 4 B written
    "msg_in": 64, "msg_out": 64,  # fixed message record
    "ent_in": 16, "ent_out": 16,  # payload per carried entry
    "remote_touch": 17,      # match 8 + next 8 + state 1
    "ring_access": 8,        # term-ring access
    "ent_saved": 16,         # payload append
    "rq_touch": 40,          # readIndex queue slot
}

WORKLOADS = {
    # name: (engine kwargs, settle rounds, description)
    "c4": (dict(n_groups=1_000_000, n_replicas=3, quiesce=True, wl_enabled=True,
                wl_start_round=30, wl_active_mod=10, wl_read_permille=900, ring=64),
           260, "C4: 1M groups x 3 replicas per GPU, Quiesce on, 90% idle (quiesced), "
                "10% active with 9:1 ReadIndex:propose, 16 B proposals"),
    "c2": (dict(n_groups=10_000, n_replicas=3, wl_enabled=True, wl_start_round=30, ring=64),
           60, "C2: 10k groups x 3 replicas, 1 proposal per group per round"),
    "c2m": (dict(n_groups=1_000_000, n_replicas=3, wl_enabled=True, wl_start_round=30,
                 ring=64), 60, "C2 at 1M groups x 3: 1 proposal per group per round"),
    "c3": (dict(n_groups=100_000, n_replicas=5, check_quorum=True, wl_enabled=True,
                wl_start_round=40, iso_period=50, iso_len=30, iso_mod=10, ring=128,
                ecap=256),
           100, "C3: 100k groups x 5, CheckQuorum, leader isolation 30/50 rounds for 10%"),
    # node snapshots every 16 applied entries, LogDB compacted to 8 below
    # (config.SnapshotEntries / CompactionOverhead), InstallSnapshot for laggards
    "c2s": (dict(n_groups=1_000_000, n_replicas=3, wl_enabled=True, wl_start_round=30,
                 ring=64, snapshot_entries=16, compaction_overhead=8), 60,
            "C2 at 1M groups x 3 with SnapshotEntries=16, CompactionOverhead=8"),
    "c3s": (dict(n_groups=100_000, n_replicas=5, check_quorum=True, wl_enabled=True,
                 wl_start_round=40, iso_period=150, iso_len=100, iso_mod=10, ring=64,
                 ecap=256, snapshot_entries=20, compaction_overhead=5), 100,
            "C3 with 100-round isolations in a 64-entry window: SnapshotEntries=20, "
            "CompactionOverhead=5, InstallSnapshot brings the isolated replicas back"),
    # groups per GPU; every rank holds the planes of all N x 500k groups and
    # steps the replicas it owns
    # C4 driven from the host through the C ABI, as the node layer would drive
    # it: every round the host stages the ReadIndex / proposal input of the
    # active groups at their leaders (rbe_push_read_index / rbe_push_proposals)
    # and reads back every replica's Update and the round's Messages /
    # ReadyToReads (rbe_get_updates, rbe_collect_outputs); run_host_driven
    "c4h": (dict(n_groups=1_000_000, n_replicas=3, quiesce=True, ext_inputs=True, ring=64,
                 in_cap=200_000), 260,
            "C4 host-driven: 1M groups x 3, Quiesce on, 10% active groups get a ReadIndex "
            "(90%) or a 16 B proposal (10%) per round at their leader through rbe_push_*, "
            "the Updates of the replicas that have one and every output read back through rbe_collect_updates / rbe_collect_outputs"),
    "c5": (dict(n_groups=500_000, n_replicas=3, wl_enabled=True, wl_start_round=30, ring=64),
           60, "C5: 500k groups x 3 per GPU, replica-per-GPU (replica k of group g on rank "
               "(g+k) % N), steady replication, cross-rank messages by all-to-all each round"),
}


# engine capacities (per-replica window and per-round buffers) that the oracle
# does not have: it keeps every entry and message in growable containers
ENGINE_ONLY = ("ring", "ecap", "maxm", "rq_cap", "rtr_cap", "dri_cap")
CAP_DEFAULT = {"ring": 64, "ecap": 32, "maxm": 12, "rq_cap": 8, "rtr_cap": 8, "dri_cap": 8}  # rbe.h

# bounded CPU-baseline samples (groups for the T-thread run, groups for the
# 1-thread run), sized for ~5-15 s of host time each on the GPU box
CPU_SAMPLE = {"c4": (300_000, 30_000), "c2": (10_000, 10_000), "c2m": (100_000, 10_000),
              "c3": (50_000, 5_000), "c5": (100_000, 10_000), "c2s": (100_000, 10_000),
              "c3s": (50_000, 5_000)}


def cfg_overrides(spec):
    """--cfg a=1,b=2: engine capacities (ENGINE_ONLY keys) for A/B runs."""
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=", 1)
        if k not in ENGINE_ONLY:
            raise SystemExit(f"--cfg: {k} is not an engine capacity ({', '.join(ENGINE_ONLY)})")
        out[k] = int(v)
    return out


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Threads the CPU baseline may use: BASELINE.md asks for T = nproc, but on
    the GPU box nproc reports the whole machine while the job is granted a
    share (OMP_NUM_THREADS, 16 per GPU); T is the smaller of the affinity set
    and that share."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, share) if share > 0 else aff), aff


def _oracle_rate(name, groups, settle, rounds, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    kw, _, _ = WORKLOADS[name]
    kw = {k: v for k, v in kw.items() if k not in ENGINE_ONLY}
    kw["n_groups"] = groups
    h = O.Harness(**kw, trace=False, threads=threads)
    h.run(settle)
    c0 = h.counters()
    t0 = time.perf_counter()
    h.run(rounds)
    dt = time.perf_counter() - t0
    c1 = h.counters()
    return ((c1["steps"] - c0["steps"]) / dt, (c1["committed"] - c0["committed"]) / dt,
            (c1["reads_confirmed"] - c0["reads_confirmed"]) / dt, dt)


def _soa_rate(name, groups, settle, rounds, threads):
    """The engine's own SoA step compiled for the host (tests/soa_cpu: the
    device step built with RBE_HD for the CPU, -O2), T engines stepped on T
    threads with the groups partitioned cid % T, as the GPU shards them: the
    same algorithm and layout as the GPU path, on the host's cores."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from soa_cpu.soa import SoaCpu
    kw, _, _ = WORKLOADS[name]
    per = max(1, groups // threads)
    engs = [SoaCpu(trace=False, **dict(kw, n_groups=per, cid_base=1 + t, cid_stride=threads))
            for t in range(threads)]
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda e: e.run(settle), engs))
        c0 = [e.counters() for e in engs]
        t0 = time.perf_counter()
        list(ex.map(lambda e: e.run(rounds), engs))
        dt = time.perf_counter() - t0
    c1 = [e.counters() for e in engs]
    d = {k: sum(b[k] - a[k] for a, b in zip(c0, c1)) for k in ("steps", "committed", "reads_confirmed")}
    return d["steps"] / dt, d["committed"] / dt, d["reads_confirmed"] / dt, dt, per * threads


def cpu_baseline(name, groups, settle, rounds, threads, groups_1t, rounds_1t):
    """The oracle (C++ restatement of internal/raft, test infrastructure) on a
    bounded sample of the same workload, timed on this host's cores: T threads
    with groups partitioned cid % T (FixedPartitioner), plus a 1-thread run
    (CPU baseline plan)."""
    v, ce, rc, dt = _oracle_rate(name, groups, settle, rounds, threads)
    v1, ce1, rc1, dt1 = _oracle_rate(name, groups_1t, settle, rounds_1t, 1)
    _, aff = host_threads()
    kw, _, _ = WORKLOADS[name]
    try:
        srounds = max(rounds, 100)  # the SoA step is ~8x the oracle's speed: more timed rounds
        sv, sce, src, sdt, sg = _soa_rate(name, groups, settle, srounds, threads)
        soa = {"value": sv, "unit": "group-steps/s", "cores": threads,
               "committed_entries_per_s": sce, "read_confirmations_per_s": src, "seconds": sdt,
               "sample": (f"{sg} groups x {kw['n_replicas']} replicas, {srounds} timed rounds "
                          f"after a {settle}-round settle; this engine's SoA step compiled for "
                          f"the host (tests/soa_cpu), {threads} engines on {threads} threads, "
                          f"groups partitioned cid % threads")}
    except Exception as ex:  # a second baseline must not hide the first
        soa = {"error": repr(ex)}
    return {
        "value": v,
        "unit": "group-steps/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": cpu_model(),
        "host_cpus_visible": aff,
        "nproc": os.cpu_count(),
        "sample": (f"{groups} groups x {kw['n_replicas']} replicas of the same workload, "
                   f"{rounds} timed rounds after a {settle}-round settle; C++ restatement "
                   f"of internal/raft (oracle/), not Go; {threads} threads, groups "
                   f"partitioned cid % threads"),
        "committed_entries_per_s": ce,
        "read_confirmations_per_s": rc,
        "seconds": dt,
        "one_thread": {"value": v1, "unit": "group-steps/s", "cores": 1,
                       "committed_entries_per_s": ce1, "read_confirmations_per_s": rc1,
                       "sample": f"{groups_1t} groups, {rounds_1t} timed rounds",
                       "seconds": dt1},
        "soa_host": soa,
    }


def lib_identity():
    """Path and content hash of the engine library this process loaded (RBE_LIB
    can point at an A/B build; the bench line records which one it timed)."""
    import hashlib
    from dragonboat_amd import engine as E
    p = os.environ.get("RBE_LIB") or E.LIB_PATH
    h = hashlib.sha256()
    with open(p, "rb") as f:
        h.update(f.read())
    return {"path": os.path.relpath(p, ROOT), "sha256_16": h.hexdigest()[:16]}


def alg_bytes(c):
    """SURVEY.md §8(d) algorithmic bytes of a counter set."""
    return sum(BYTES[k] * c[k] for k in BYTES)


def load_traffic(name, kernel, lib):
    """Measured HBM bytes per launch of `kernel` from the committed PMC summary
    (profiles/traffic_<workload>.json, written by scripts/pmc_traffic.py), only
    when it was measured on this very library (same content hash); else None."""
    p = os.path.join(ROOT, "profiles", f"traffic_{name}.json")
    if not os.path.exists(p):
        return None, "no PMC summary"
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "unreadable PMC summary"
    if d.get("library_sha256_16") != lib.get("sha256_16"):
        return None, (f"PMC summary measured on library {d.get('library_sha256_16')}, "
                      f"not this one ({lib.get('sha256_16')})")
    x2 = d.get("bytes_per_launch_fetch_x2", {}).get(kernel)
    return d.get("bytes_per_launch", {}).get(kernel), "same library" + (
        f"; with the guide's FETCH_SIZE x 2: {x2:.0f} B" if x2 else "")


def side_line(name, local, steps, prof_rounds):
    """A short line of another BASELINE configuration on the same GPU (one
    rank, untraced, same definitions as the main line): group-steps/s over
    `steps` timed rounds and the per-kernel split of `prof_rounds` more."""
    from dragonboat_amd.engine import Engine, make_config
    kw, settle, desc = WORKLOADS[name]
    eng = Engine(make_config(device=local, trace=False, **dict(kw)))
    eng.run(settle + 10)
    eng.prepare_run(steps)
    eng.sync()
    eng.reset_counters()
    t0 = time.perf_counter()
    ev_ms = eng.run_timed(steps)
    eng.sync()
    wall = time.perf_counter() - t0
    c = eng.counters()
    nf, _ = eng.fault_summary()
    eng.reset_counters()
    kms = eng.profile_rounds(prof_rounds)
    kernels = []
    for ki, kn in enumerate(eng.kernel_names()):
        if not kn:
            continue
        b = alg_bytes(eng.kernel_counters(ki)) / prof_rounds
        us = kms[ki] * 1e3 / prof_rounds
        kernels.append({"kernel": kn, "avg_us": us, "alg_bytes_per_launch": b,
                        "achieved_gbs": (b / (us * 1e-6) / 1e9) if us > 0 else 0.0})
    dom = max(kernels, key=lambda k: k["avg_us"])
    eng.close()
    return {"workload": desc, "value": c["steps"] / wall, "unit": "group-steps/s",
            "ms_per_step": wall * 1e3 / steps, "event_ms_per_round": ev_ms / steps,
            "steps": steps, "faulty_replicas": int(nf),
            "committed_entries_per_s": c["committed"] / wall,
            "dominant": {"kernel": dom["kernel"], "avg_us": dom["avg_us"],
                         "frac": dom["achieved_gbs"] / HBM_PEAK_GBS},
            "kernels": kernels}


def run_replica_mode(args, ws, rank, local, dist, dev, gloo_staged):
    """C5: replica-per-GPU.  Every round = one engine round over the owned
    replicas + one exchange (pack → counts all-to-all → records
    all_to_all_single → unpack, dragonboat_amd/replica.py).  The timed region
    holds both; the exchange share is reported beside it."""
    from dragonboat_amd.engine import Engine, footprint, make_config
    from dragonboat_amd.replica import ReplicaExchange
    from dragonboat_amd.shard import reduce_results

    kw, settle, desc = WORKLOADS["c5"]
    kw = dict(kw)
    per_gpu = args.groups or kw["n_groups"]
    kw["n_groups"] = per_gpu * ws
    # rep_compact: each rank allocates only the groups it steps a replica of
    # (3/8 of them at 8 ranks)
    cfg = make_config(device=0 if gloo_staged else local, trace=False,
                      rep_world=ws if ws > 1 else 0, rep_rank=rank,
                      rep_compact=ws > 1 and not args.no_compact, **kw)
    eng = Engine(cfg)
    xch = None
    if ws > 1:
        # --xchg-fixed: equal chunks with count headers, no host-side count read
        # (rbe_xchg_pack_fixed; with RCCL the collective runs on the engine's
        # stream).  The settle and warmup rounds run the counted exchange; the
        # chunks are then sized from the largest counts of the warmup rounds
        # (ReplicaExchange.to_fixed) and the timed rounds run fixed
        xch = ReplicaExchange(eng, buf_device=dev, comm_device="cpu" if gloo_staged else dev)

    def one_exchange():
        if xch.fixed:
            xch.exchange_fixed()
        else:
            xch.exchange()

    def rounds(k, timed_xchg=None):
        for _ in range(k):
            if xch is not None:
                xch.step()
            else:
                eng.step()
            if xch is not None:
                if timed_xchg is not None:
                    eng.sync()
                    t = time.perf_counter()
                    one_exchange()
                    eng.sync()
                    timed_xchg[0] += time.perf_counter() - t
                else:
                    one_exchange()
        if xch is not None:
            xch.check()

    def barrier():
        if ws > 1:
            dist.barrier()
        eng.sync()

    rounds(settle)
    if xch is not None:
        xch.reset_peak()
    rounds(max(1, args.warmup))
    if xch is not None and args.xchg_fixed:
        xch.to_fixed()
    eng.sync()
    eng.reset_counters()
    b0 = xch.bytes_sent if xch else 0
    barrier()
    t0 = time.perf_counter()
    rounds(args.steps)
    barrier()
    wall = time.perf_counter() - t0
    c = eng.counters()
    nf, fo = eng.fault_summary()
    sent = (xch.bytes_sent - b0) if xch else 0
    # exchange share, on separate rounds (the sync before each exchange would
    # otherwise perturb the timed region)
    xt = [0.0]
    rounds(min(args.steps, 20), timed_xchg=xt)
    xchg_ms = xt[0] * 1e3 / min(args.steps, 20)
    red_dev = None if gloo_staged or ws == 1 else dev
    wall_max, (steps, committed, reads, faulty, sent_all, xms_sum) = reduce_results(
        dist if ws > 1 else None, wall, [c["steps"], c["committed"], c["reads_confirmed"], nf,
                                         sent, xchg_ms], device=red_dev)
    xms_mean = xms_sum / ws
    # kernel split: single profiled rounds, each followed by its exchange
    prof_rounds = max(1, min(args.steps, args.prof_rounds))
    eng.reset_counters()
    kms = [0.0] * 4
    for _ in range(prof_rounds):
        if xch is not None:
            xch.iso_sync()
        for i, v in enumerate(eng.profile_rounds(1)):
            kms[i] += v
        if xch is not None:
            xch.exchange()
    kernels = []
    for ki, name in enumerate(eng.kernel_names()):
        if not name:
            continue
        b = alg_bytes(eng.kernel_counters(ki)) / prof_rounds
        us = kms[ki] * 1e3 / prof_rounds
        kernels.append({"kernel": name, "avg_us": us, "alg_bytes_per_launch": b,
                        "achieved_gbs": (b / (us * 1e-6) / 1e9) if us > 0 else 0.0})
    dom = max(kernels, key=lambda k: k["avg_us"])
    if rank == 0:
        out = {
            "metric": METRIC, "value": steps / wall_max, "unit": "group-steps/s",
            "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": wall_max * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": desc, "groups_per_gpu": per_gpu, "replicas_per_group": 3,
                       "total_groups": kw["n_groups"],
                       "parallelism": f"replica-per-GPU x{ws} ((g+k) % {ws})",
                       "exchange": ("gloo, host-staged (rehearsal)" if gloo_staged else
                                    "RCCL all_to_all_single") if ws > 1 else "none (1 rank)",
                       "election_rtt": 10, "heartbeat_rtt": 1, "settle_rounds": settle,
                       "device_bytes_per_gpu": footprint(cfg)},
            "committed_entries_per_s": committed / wall_max,
            "read_confirmations_per_s": reads / wall_max,
            "faulty_replicas": int(faulty), "fault_bits_rank0": fo,
            "exchange": {"bytes_per_round_all_ranks": sent_all / args.steps,
                         "ms_per_round_mean_rank": xms_mean,
                         "mode": "fixed" if (xch is not None and xch.fixed) else "counted",
                         # one fixed chunk over the mean counted round's
                         # records to one peer (rank 0): the padding
                         "fixed_pad": xch.pad_ratio() if (xch is not None and xch.fixed)
                         else None,
                         # fixed rounds whose records outgrew the chunks, repaired
                         # by a counted second pass (rank 0; never invalid)
                         "repaired_rounds": xch.repaired if xch is not None else 0},
            "roofline": {"bound": "hbm", "achieved": dom["achieved_gbs"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": dom["achieved_gbs"] / HBM_PEAK_GBS,
                         "traffic": None, "kernel": dom["kernel"],
                         "alg_bytes_per_launch": dom["alg_bytes_per_launch"],
                         "avg_launch_us": dom["avg_us"], "profiled_rounds": prof_rounds},
            "round": {"kernels": kernels},
        }
        print(json.dumps(out), flush=True)
    eng.close()


def run_host_driven(args, ws, rank, local, dist):
    """c4h: the C4 round driven through the C ABI as dragonboat's node layer
    drives Peer (node.go:1030-1067 handleEvents, 907-923 getUpdate,
    execengine.go:474-560): each round (1) the ReadIndex / proposal input of
    the active groups is staged at their leaders (rbe_push_read_index,
    rbe_push_proposals with 16 B Cmds; leaders known from the last Updates),
    (2) one rbe_step, (3) the Updates of the replicas that have one
    (rbe_collect_updates, compacted on the device) and the round's Messages /
    ReadyToReads (rbe_collect_outputs) come back to the host.
    The timed region holds all three; the boundary's share (1 + 3) is reported
    beside the device time (HIP events around the step)."""
    import ctypes as C
    import numpy as np
    from dragonboat_amd.engine import (EV_LEADER_UPDATED, RBE_COLLECT_REMOTE_MSGS,
                                       RBE_COLLECT_SKIP_LOCAL, UPDATE_DTYPE, Engine, RbeOutputs,
                                       RbeStepOutputs, RbeUpdateList, _check, footprint,
                                       make_config)
    from dragonboat_amd.shard import reduce_results, shard_params

    kw, settle, desc = WORKLOADS["c4h"]
    kw = dict(kw)
    if args.groups:
        kw["n_groups"] = args.groups
    n_groups, N = int(kw["n_groups"]), int(kw["n_replicas"])
    n_rep = n_groups * N
    cid_base, cid_stride = shard_params(rank, ws)
    cfg = make_config(device=local, cid_base=cid_base, cid_stride=cid_stride, trace=False, **kw)
    eng = Engine(cfg)
    L, h = eng.lib, eng.h
    rng = np.random.default_rng(7 + rank)
    active = np.arange(0, n_groups, 10, dtype=np.uint64)  # 10% of the groups
    ul = RbeUpdateList()
    outs = RbeOutputs()
    so = RbeStepOutputs()
    # --c4h-all-msgs: every Update and every message copied back
    # (rbe_collect_updates + rbe_collect_outputs); default: rbe_collect_step
    # with only the messages for other engines (none here: group-per-GPU, the
    # engine delivers them itself) and only the Updates that hold work for the
    # node besides those messages (RBE_COLLECT_SKIP_LOCAL)
    all_msgs = args.c4h_all_msgs
    cflags = RBE_COLLECT_REMOTE_MSGS | RBE_COLLECT_SKIP_LOCAL
    # default: rbe_collect_step_begin / _end with the next round's pushes in
    # between (requests go to the leaders known through the round before);
    # --c4h-serial: push, step, sync, collect, one after the other
    pipelined = not all_msgs and not args.c4h_serial
    cmd = np.frombuffer(rng.bytes(16 * len(active)), dtype=np.uint8).copy()
    ptr = lambda a, t: a.ctypes.data_as(C.POINTER(t))  # noqa: E731
    stats = {"push": 0.0, "push_abi": 0.0, "step": 0.0, "enqueue": 0.0, "out": 0.0, "reads": 0,
             "props": 0, "msgs": 0, "rtr": 0, "upd": 0, "push_next": 0.0}

    # the node layer learns a group's leader from the listener's LeaderUpdated
    # (event.go:93-95), which the engine reports in Update.events
    ev_leader = np.uint32(EV_LEADER_UPDATED)

    # the replica each active group's requests go to (its leader), kept
    # current from the LeaderUpdated events; NONE while a group has no leader
    NONE = np.uint64(np.iinfo(np.uint64).max)
    active_i = active.astype(np.int64)
    act_of = np.full(n_groups, -1, dtype=np.int64)
    act_of[active_i] = np.arange(len(active))
    lead_rep = np.full(len(active), NONE, dtype=np.uint64)

    def set_leaders(g, lid):
        a = act_of[g]
        on = a >= 0
        lead_rep[a[on]] = np.where(lid[on] != 0, g[on].astype(np.uint64) * np.uint64(N) +
                                   lid[on] - np.uint64(1), NONE)

    def note_leaders(rep, ups):
        chg = (ups["events"] & ev_leader) != 0
        if chg.any():
            lid = ups["leader_id"][chg]
            known = lid != 0
            set_leaders((rep[chg][known] // np.uint64(N)).astype(np.int64), lid[known])

    def read_back():
        if not all_msgs:
            _check(L.rbe_collect_step(h, 0, n_rep, cflags, C.byref(so)), "rbe_collect_step")
            n = so.n
            if n:  # the engine's pinned buffer, read in place
                rep = np.ctypeslib.as_array(so.replica, shape=(n,))
                ups = np.frombuffer((C.c_uint8 * (n * UPDATE_DTYPE.itemsize)).from_address(
                    C.addressof(so.updates.contents)), dtype=UPDATE_DTYPE)
                note_leaders(rep, ups)
            return so.n_messages, so.n_ready_to_reads, n
        _check(L.rbe_collect_updates(h, 0, n_rep, C.byref(ul)), "rbe_collect_updates")
        _check(L.rbe_collect_outputs(h, 0, n_rep, C.byref(outs)), "rbe_collect_outputs")
        n = ul.n
        if n:  # the engine's pinned buffers, read in place
            rep = np.ctypeslib.as_array(ul.replica, shape=(n,))
            ups = np.frombuffer((C.c_uint8 * (n * UPDATE_DTYPE.itemsize)).from_address(
                C.addressof(ul.updates.contents)), dtype=UPDATE_DTYPE)
            note_leaders(rep, ups)
        return outs.n_messages, outs.n_ready_to_reads, n

    # the client workload of every round, drawn before the timed region
    # (synthetic requests, not node-layer work): which active groups get a
    # ReadIndex (90%) and which a proposal
    total_rounds = settle + max(1, args.warmup) + args.steps + 1  # (+1: the pipelined next push)
    read_mask = rng.random((total_rounds, len(active))) < 0.9
    read_at = [np.flatnonzero(m) for m in read_mask]
    prop_at = [np.flatnonzero(~m) for m in read_mask]
    one = np.ones(len(active), dtype=np.uint32)
    zero = np.zeros(len(active), dtype=np.uint32)
    ln = np.full(len(active), 16, dtype=np.uint32)

    def push_round(rnd):
        """The client requests of round rnd, staged at the leaders known so
        far (rbe_push_read_index / rbe_push_proposals); returns (reads,
        proposals, seconds in the ABI calls)."""
        rr, pr = lead_rep[read_at[rnd]], lead_rep[prop_at[rnd]]
        if (len(rr) and rr.max() == NONE) or (len(pr) and pr.max() == NONE):
            rr, pr = rr[rr != NONE], pr[pr != NONE]  # groups without a leader wait
        if len(rr):  # ctx.Low = round << 32 | replica + 1 (never 0), ctx.High = replica
            lo = rr + np.uint64(((rnd + 1) << 32) + 1)
        tc = time.perf_counter()
        if len(rr):
            _check(L.rbe_push_read_index(h, len(rr), ptr(rr, C.c_uint64), ptr(lo, C.c_uint64),
                                         ptr(rr, C.c_uint64)), "rbe_push_read_index")
        if len(pr):
            _check(L.rbe_push_proposals(h, len(pr), ptr(pr, C.c_uint64), ptr(one, C.c_uint32),
                                        ptr(zero, C.c_uint32), ptr(ln, C.c_uint32),
                                        ptr(cmd, C.c_uint8)), "rbe_push_proposals")
        return len(rr), len(pr), time.perf_counter() - tc

    def parse_step_outputs(o):
        n = o.n
        if n:  # the engine's mapped buffer, read in place
            rep = np.ctypeslib.as_array(o.replica, shape=(n,))
            ups = np.frombuffer((C.c_uint8 * (n * UPDATE_DTYPE.itemsize)).from_address(
                C.addressof(o.updates.contents)), dtype=UPDATE_DTYPE)
            note_leaders(rep, ups)
        return o.n_messages, o.n_ready_to_reads, n

    # pipelined: the round whose requests are staged already, and the outputs
    # of the last round (the engine's two mapped buffers, used in turn), read
    # while the device runs the next step
    pending = {"pushed": None, "outs": None}
    so_pair = [RbeStepOutputs(), RbeStepOutputs()]

    def one_round(rnd, timed):
        t0 = time.perf_counter()
        if pending["pushed"] == rnd:
            nrd, npr, tabi = pending["counts"]
        else:
            nrd, npr, tabi = push_round(rnd)
        t1 = time.perf_counter()
        eng.step()
        te = time.perf_counter()
        if pipelined:
            # while the device runs this step: the last round's outputs are
            # read in place; then this round's collection runs on the device
            # while the host stages the next round's requests (at the leaders
            # known through the round before the last)
            nm = nr = nu = 0
            if pending["outs"] is not None:
                nm, nr, nu = parse_step_outputs(pending["outs"])
                pending["outs"] = None
            tp = time.perf_counter()
            _check(L.rbe_collect_step_begin(h, 0, n_rep, cflags), "rbe_collect_step_begin")
            tq = time.perf_counter()
            pending["counts"] = push_round(rnd + 1)
            pending["pushed"] = rnd + 1
            tn = time.perf_counter()
            o = so_pair[rnd & 1]
            _check(L.rbe_collect_step_end(h, C.byref(o)), "rbe_collect_step_end")
            pending["outs"] = o
            t2 = t3 = time.perf_counter()
        else:
            eng.sync()
            t2 = time.perf_counter()
            nm, nr, nu = read_back()
            t3 = time.perf_counter()
        if timed:
            stats["push"] += t1 - t0
            stats["push_abi"] += tabi
            stats["enqueue"] += te - t1
            if pipelined:
                stats["push_next"] += tn - tq  # overlapped with the device
                stats["out"] += tp - te  # the last round's records, read during this step
                # step + collection not hidden by the two
                stats["step"] += t2 - t1 - (tn - tq) - (tp - te)
            else:
                stats["step"] += t2 - t1
                stats["out"] += t3 - t2
            stats["reads"] += nrd
            stats["props"] += npr
            stats["msgs"] += nm
            stats["rtr"] += nr
            stats["upd"] += nu

    for r in range(settle + max(1, args.warmup)):
        if r < settle:
            eng.step()
            if r == settle - 1:  # leaders of every group, quiesced ones included (untimed)
                eng.sync()
                lid = np.frombuffer(bytes(eng.updates()), UPDATE_DTYPE)["leader_id"]
                set_leaders(np.arange(n_groups), lid.reshape(n_groups, N).max(axis=1))
                read_back()
        else:
            one_round(r, False)
    eng.sync()
    eng.reset_counters()
    if dist is not None:
        dist.barrier()
    if pending["outs"] is not None:  # the warmup's last outputs
        parse_step_outputs(pending["outs"])
        pending["outs"] = None
    t0 = time.perf_counter()
    for r in range(args.steps):
        one_round(settle + args.warmup + r, True)
    if pending["outs"] is not None:  # the last timed round's outputs
        tl = time.perf_counter()
        nm, nr, nu = parse_step_outputs(pending["outs"])
        stats["out"] += time.perf_counter() - tl
        stats["msgs"] += nm
        stats["rtr"] += nr
        stats["upd"] += nu
    eng.sync()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    c = eng.counters()
    nf, fo = eng.fault_summary()
    wall_max, (steps, committed, reads) = reduce_results(
        dist, wall, [c["steps"], c["committed"], c["reads_confirmed"]])
    K = args.steps
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": steps / wall_max, "unit": "group-steps/s", "n_gpus": ws,
            "steps": K, "warmup": args.warmup, "ms_per_step": wall_max * 1e3 / K,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": desc, "groups_per_gpu": n_groups, "replicas_per_group": N,
                       "total_groups": n_groups * ws, "parallelism": f"group-per-GPU x{ws}",
                       "election_rtt": 10, "heartbeat_rtt": 1, "settle_rounds": settle,
                       "device_bytes_per_gpu": footprint(cfg)},
            "committed_entries_per_s": committed / wall_max,
            "read_confirmations_per_s": reads / wall_max,
            "faulty_replicas": int(nf), "fault_bits_rank0": fo,
            "boundary": {
                "push_ms_per_round": stats["push"] * 1e3 / K,
                # of which the rbe_push_* calls (the rest: the bench's numpy batch assembly)
                "push_abi_ms_per_round": stats["push_abi"] * 1e3 / K,
                "step_ms_per_round": stats["step"] * 1e3 / K,
                # host part of the step call: input upload staging + launches
                "step_enqueue_ms_per_round": stats["enqueue"] * 1e3 / K,
                "read_back": "rbe_collect_updates + rbe_collect_outputs (every message)"
                if all_msgs else ((("rbe_collect_step_begin / _end, the next round's pushes "
                                    "in between") if pipelined else "rbe_collect_step") +
                                  " (messages for other engines only; RBE_COLLECT_SKIP_LOCAL: "
                                  "Updates with work for the node)"),
                "outputs_ms_per_round": stats["out"] * 1e3 / K,
                "pipelined": pipelined,
                # pipelined: the next round's pushes, made while the device
                # steps and collects this one (inside step_ms when not)
                "push_overlapped_ms_per_round": stats["push_next"] * 1e3 / K,
                "boundary_share": (stats["push"] + stats["push_next"] + stats["out"]) /
                max(1e-12, wall),
                "reads_pushed_per_round": stats["reads"] / K,
                "proposals_pushed_per_round": stats["props"] / K,
                "messages_read_per_round": stats["msgs"] / K,
                "ready_to_reads_per_round": stats["rtr"] / K,
                "updates_read_per_round": stats["upd"] / K,
            },
            "library": lib_identity(),
        }), flush=True)
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--groups", type=int, default=0, help="override groups per GPU")
    ap.add_argument("--cfg", default="",
                    help="engine capacity overrides for A/B runs, e.g. maxm=4,ecap=16 "
                         "(recorded in the line's config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-compact", action="store_true",
                    help="c5: allocate every group's planes on every rank")
    ap.add_argument("--prof-rounds", type=int, default=50,
                    help="rounds profiled per kernel with HIP events after the timed region")
    ap.add_argument("--cpu-groups", type=int, default=0,
                    help="groups in the T-thread CPU sample (0 = per-workload default)")
    ap.add_argument("--cpu-rounds", type=int, default=100)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = host_threads()")
    ap.add_argument("--cpu-groups-1t", type=int, default=0,
                    help="groups in the 1-thread CPU sample (0 = per-workload default)")
    ap.add_argument("--xchg-gloo", action="store_true",
                    help="c5 rehearsal: all ranks on cuda:0, exchange over gloo via host memory")
    ap.add_argument("--also", default="c2,c3",
                    help="other workloads timed briefly in the same run (comma list, '' = none)")
    ap.add_argument("--c4h-all-msgs", action="store_true",
                    help="c4h: read every message back too (rbe_collect_outputs)")
    ap.add_argument("--c4h-serial", action="store_true",
                    help="c4h: push, step, sync and collect one after the other "
                         "(default: rbe_collect_step_begin / _end around the next round's pushes)")
    ap.add_argument("--xchg-fixed", action="store_true",
                    help="c5: fixed-capacity exchange (count headers, no host-side count read)")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    import torch
    import torch.distributed as dist
    use_dist = ws > 1
    gloo_staged = args.workload == "c5" and args.xchg_gloo
    if gloo_staged:
        local = 0
    if use_dist:
        backend = "nccl" if torch.cuda.is_available() and not gloo_staged else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if args.workload == "c4h":
        run_host_driven(args, ws, rank, local, dist if use_dist else None)
        if use_dist:
            dist.destroy_process_group()
        return
    if args.workload == "c5":
        run_replica_mode(args, ws, rank, local, dist, dev, gloo_staged)
        if use_dist:
            dist.destroy_process_group()
        return

    from dragonboat_amd.engine import Engine, footprint, make_config
    from dragonboat_amd.shard import reduce_results, shard_params

    kw, settle, desc = WORKLOADS[args.workload]
    kw = dict(kw)
    if args.groups:
        kw["n_groups"] = args.groups
    kw.update(cfg_overrides(args.cfg))
    # group-per-GPU sharding (dragonboat_amd/shard.py): rank r steps the
    # clusters with (cid - 1) % world == r, dragonboat's FixedPartitioner rule
    cid_base, cid_stride = shard_params(rank, ws)
    cfg = make_config(device=local, cid_base=cid_base, cid_stride=cid_stride, trace=False, **kw)
    eng = Engine(cfg)

    def barrier():
        if use_dist:
            dist.barrier()
        eng.sync()

    # settle to steady state (elections done, idle groups quiesced), then warm up
    eng.run(settle)
    eng.run(max(1, args.warmup))
    # the replay graph of the timed round count is captured and uploaded here,
    # outside the timed region (every timed round still runs all its kernels)
    eng.prepare_run(args.steps)
    eng.sync()
    eng.reset_counters()

    barrier()
    t0 = time.perf_counter()
    ev_ms = eng.run_timed(args.steps)  # HIP events on the engine stream around K launches
    barrier()
    wall = time.perf_counter() - t0

    c = eng.counters()
    nf, fo = eng.fault_summary()
    red_dev = dev if (use_dist and dist.get_backend() == "nccl") else None
    wall_max, (steps, committed, reads, faulty) = reduce_results(
        dist if use_dist else None, wall,
        [c["steps"], c["committed"], c["reads_confirmed"], nf], device=red_dev)

    # whole-round algorithmic bandwidth over the timed region (all kernels)
    round_bytes = alg_bytes(c) / args.steps
    round_gbs = round_bytes / ((ev_ms / 1e3) / args.steps) / 1e9

    # per-kernel split: a further `prof_rounds` rounds, one at a time, each
    # kernel launched with a start / stop HIP event pair its own dispatch
    # stamps (hipExtLaunchKernel, on the engine stream: the kernel's execution
    # as rocprofv3 times it) and each kernel's own counters -> the dominant
    # kernel's roofline
    prof_rounds = max(1, min(args.steps, args.prof_rounds))
    eng.reset_counters()
    kms = eng.profile_rounds(prof_rounds)
    kernels = []
    for ki, name in enumerate(eng.kernel_names()):
        if not name:
            continue
        kc = eng.kernel_counters(ki)
        b = alg_bytes(kc) / prof_rounds
        us = kms[ki] * 1e3 / prof_rounds
        kernels.append({"kernel": name, "avg_us": us, "alg_bytes_per_launch": b,
                        "achieved_gbs": (b / (us * 1e-6) / 1e9) if us > 0 else 0.0})
    dom = max(kernels, key=lambda k: k["avg_us"])
    lib = lib_identity()
    traffic, traffic_src = load_traffic(args.workload, dom["kernel"], lib)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": steps / wall_max,
            "unit": "group-steps/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {
                "workload": desc,
                "groups_per_gpu": int(kw["n_groups"]),
                "replicas_per_group": int(kw["n_replicas"]),
                "total_groups": int(kw["n_groups"]) * ws,
                "parallelism": f"group-per-GPU x{ws} (cid % {ws})",
                "election_rtt": 10, "heartbeat_rtt": 1,
                "settle_rounds": settle,
                "device_bytes_per_gpu": footprint(cfg),
                "capacities": {k: int(getattr(cfg, k)) or CAP_DEFAULT[k] for k in ENGINE_ONLY},
            },
            "committed_entries_per_s": committed / wall_max,
            "read_confirmations_per_s": reads / wall_max,
            "faulty_replicas": int(faulty),
            "fault_bits_rank0": fo,
            "roofline": {
                "bound": "hbm",
                "achieved": dom["achieved_gbs"],
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": dom["achieved_gbs"] / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": dom["kernel"],
                "alg_bytes_per_launch": dom["alg_bytes_per_launch"],
                "avg_launch_us": dom["avg_us"],
                "profiled_rounds": prof_rounds,
            },
            "round": {
                "alg_bytes_per_round": round_bytes,
                "achieved_gbs": round_gbs,
                "frac": round_gbs / HBM_PEAK_GBS,
                "event_ms_per_round": ev_ms / args.steps,
                "kernels": kernels,
            },
        }
        out["library"] = lib
        # the other single-GPU BASELINE configurations, timed in the same run
        # (parity cases elsewhere; here only their rate and kernel split)
        if ws == 1 and args.also:
            out["workloads"] = {}
            for name in [x for x in args.also.split(",") if x and x != args.workload]:
                try:
                    out["workloads"][name] = side_line(name, local, 50, 20)
                except Exception as ex:  # a side line must not hide the main one
                    out["workloads"][name] = {"error": repr(ex)}
        if not args.no_cpu_baseline and ws == 1:
            try:
                ng = int(kw["n_groups"])
                g_t = args.cpu_groups or min(ng, CPU_SAMPLE[args.workload][0])
                g_1 = args.cpu_groups_1t or min(ng, CPU_SAMPLE[args.workload][1])
                threads = args.cpu_threads or host_threads()[0]
                out["cpu_baseline"] = cpu_baseline(args.workload, g_t, settle, args.cpu_rounds,
                                                   threads, g_1, args.cpu_rounds)
            except Exception as ex:  # the baseline must not hide the GPU number
                out["cpu_baseline"] = {"error": repr(ex)}
        print(json.dumps(out), flush=True)
    eng.close()
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
