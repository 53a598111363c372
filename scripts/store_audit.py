"""Store audit of the fast step (k_fast_both) on C4: every global store site of
lead_fast / foll_fast with its stores, bytes and modelled write requests per
launch, against the measured TCP_TCC_WRITE_REQ_sum (profiles/traffic_c4.json).

The counts come from the host build of the same step (tests/soa_cpu built with
-DRBE_STORE_AUDIT: RBE_AUDIT at each store site, rbe_types.h) on C4 at a
reduced group count, scaled to C4's 1M groups (the active set is every 10th
group, so the per-group work is independent of the group count).  Requests
are modelled as the GPU's TCP issues them: one request per store instruction
(a 16-B piece of the record) per distinct 64-B line among the 64 lanes of a
wave, a wave being 64 consecutive items of the round's fast list (leaders
first, ascending replica as triage pushes them).

    python3 scripts/store_audit.py [--groups 100000] [--out profiles/store_audit_c4.json]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "libsoa_audit.so")
SRC = os.path.join(ROOT, "tests", "soa_cpu", "soa_cpu.cpp")
SITES = ["msg", "dropped_ri", "ready_to_read", "snapshot", "update(64 B)", "update chunk 3",
         "count row", "hot", "core chunk", "idle byte", "cold ref", "cold entry", "cold page meta",
         "term ring", "payload ring", "ext input", "remote match/next", "remote state",
         "readIndex queue", "outbox stash"]


MTYPES = {12: "Replicate", 13: "ReplicateResp", 17: "Heartbeat", 18: "HeartbeatResp",
          20: "ReadIndexResp", 21: "Quiesce"}


def build():
    deps = [SRC] + [os.path.join(ROOT, "dragonboat_amd", "csrc", f)
                    for f in os.listdir(os.path.join(ROOT, "dragonboat_amd", "csrc"))]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(d) for d in deps):
        return
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-DRBE_STORE_AUDIT",
                           "-o", LIB, SRC])


def requests(tr):
    """Modelled TCP write requests of a traced round: per (wave, site, k-th
    store of that site in the lane, 16-B piece), the distinct 64-B lines."""
    item, site, addr, nb = tr[:, 0], tr[:, 1], tr[:, 2], tr[:, 3] & 0xFFFFFFFF
    # occurrence index of each record among its (item, site) records
    key = item * 64 + site
    order = np.lexsort((np.arange(len(key)), key))
    ks = key[order]
    first = np.r_[True, ks[1:] != ks[:-1]]
    start = np.maximum.accumulate(np.where(first, np.arange(len(ks)), 0))
    occ = np.empty(len(key), np.int64)
    occ[order] = np.arange(len(ks)) - start
    out = np.zeros(len(SITES))
    pieces = (nb + 15) // 16
    for p in range(int(pieces.max())):
        m = pieces > p
        line = (addr[m] + 16 * p) // 64
        rows = np.stack([item[m] // 64, site[m], occ[m], np.full(m.sum(), p), line], 1)
        u = np.unique(rows, axis=0)
        np.add.at(out, u[:, 1], 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--traced", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "store_audit_c4.json"))
    a = ap.parse_args()
    build()
    os.environ["SOA_LIB"] = LIB
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import bench
    from soa_cpu.soa import SoaCpu, lib
    L = lib()
    L.soa_store_audit.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    L.soa_audit_trace.argtypes = [C.c_int]
    L.soa_audit_trace_get.restype = C.c_uint64
    L.soa_audit_trace_get.argtypes = [C.c_void_p, C.c_uint64]
    kw, settle, _ = bench.WORKLOADS["c4"]
    full_groups = kw["n_groups"]
    e = SoaCpu(trace=False, **dict(kw, n_groups=a.groups))
    e.run(settle)
    buf = (C.c_uint64 * (2 * 20 + 3))()
    L.soa_store_audit(buf, 1)
    e.run(a.rounds)
    L.soa_store_audit(buf, 1)
    v = np.array(buf[:], dtype=np.float64)
    n_sites = len(SITES)
    steps, leads, declined = v[2 * n_sites:2 * n_sites + 3]
    scale = full_groups / a.groups / a.rounds  # per launch at C4's size
    # requests from the address trace of the last rounds
    req = np.zeros(n_sites)
    items = 0
    mtypes = {}
    for _ in range(a.traced):
        L.soa_audit_trace(1)
        e.run(1)
        L.soa_audit_trace(0)
        n = L.soa_audit_trace_get(None, 0)
        arr = np.zeros(n * 4, np.uint64)
        L.soa_audit_trace_get(arr.ctypes.data, n)
        tr = arr.reshape(-1, 4).astype(np.int64)
        req += requests(tr)
        mt = tr[tr[:, 1] == 0, 3] >> 32
        for t, c in zip(*np.unique(mt, return_counts=True)):
            mtypes[int(t)] = mtypes.get(int(t), 0) + int(c)
        items += int(tr[:, 0].max()) + 1 if len(tr) else 0
    req_scale = full_groups / a.groups / a.traced
    rows = []
    for i, name in enumerate(SITES):
        cnt, byt = v[2 * i] * scale, v[2 * i + 1] * scale
        rows.append({"site": name, "stores": cnt, "bytes": byt, "requests": req[i] * req_scale})
    tot = {k: sum(r[k] for r in rows) for k in ("stores", "bytes", "requests")}
    meas = None
    tf = os.path.join(ROOT, "profiles", "traffic_c4.json")
    if os.path.exists(tf):
        t = json.load(open(tf))
        meas = {"tcp_tcc_write_req": (t.get("tcp_tcc_write_req") or {}).get("k_fast_both"),
                "write_bytes": t["write"].get("k_fast_both"),
                "library_sha256_16": t.get("library_sha256_16")}
    res = {"workload": "c4", "groups_run": a.groups, "scaled_to_groups": full_groups,
           "per": "k_fast_both launch", "fast_steps": steps * scale,
           "leader_steps": leads * scale, "declined": declined * scale,
           "messages_by_type": {MTYPES.get(t, str(t)): c * req_scale for t, c in sorted(mtypes.items())},
           "sites": rows, "total": tot, "measured": meas,
           "model": "1 request per 16-B store piece per distinct 64-B line per wave (64 "
                    "consecutive fast-list items); stores = lane stores of the record"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(f"fast steps/launch {steps * scale:,.0f} (leaders {leads * scale:,.0f}, declined "
          f"{declined * scale:,.0f})")
    print(f"{'site':22s} {'stores':>12s} {'bytes':>14s} {'requests':>12s} {'req/step':>9s}")
    for r in sorted(rows, key=lambda r: -r["requests"]):
        if r["stores"] == 0:
            continue
        print(f"{r['site']:22s} {r['stores']:12,.0f} {r['bytes']:14,.0f} {r['requests']:12,.0f}"
              f" {r['requests'] / max(steps * scale, 1):9.2f}")
    print(f"{'total':22s} {tot['stores']:12,.0f} {tot['bytes']:14,.0f} {tot['requests']:12,.0f}"
          f" {tot['requests'] / max(steps * scale, 1):9.2f}")
    print("messages/launch by type:", res["messages_by_type"])
    if meas:
        if meas.get("tcp_tcc_write_req"):
            meas["model_over_measured_requests"] = tot["requests"] / meas["tcp_tcc_write_req"]
            meas["algorithmic_over_write_size"] = tot["bytes"] / meas["write_bytes"]
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        print("measured:", meas)


if __name__ == "__main__":
    main()
