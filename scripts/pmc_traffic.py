"""Fold rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-kernel HBM bytes
per launch (profiles/traffic_<workload>.json, read by bench.py).

Per /opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
streaming reads, and other access widths are to be calibrated on a known byte
count.  The engine's kernels gather 16-B records scattered over the planes, so
the calibration is the group_shape microbenchmark of the same shape
(profiles/r05_calibration/pmc_group_shape.json, kernel k_A: 70.4 MB of known
loads per launch read as FETCH_SIZE 78.7 MB with the active groups adjacent,
98.3 MB with them scattered; doubled that would be 157-197 MB, more than the
kernel can read): for these kernels
FETCH_SIZE counts the bytes fetched, sector over-fetch included, without the
factor 2.  `bytes_per_launch` is therefore FETCH_SIZE + WRITE_SIZE; the guide's
2 x FETCH_SIZE + WRITE_SIZE is kept as `bytes_per_launch_fetch_x2`.  Only the
last LAST dispatches of each kernel are used (the bench's per-kernel profiled
rounds, in steady state).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

LAST = 10
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_key(name):
    if "k_round" in name:
        return "k_round"
    if "k_triage" in name:
        return "k_triage"
    if "k_fast_both" in name:
        return "k_fast_both"
    if "k_fast_list" in name:
        # template args <N, TRACE, MODE>: MODE 1 = LEAD, 2 = FOLL
        mode = name.split("k_fast_list<", 1)[1].split(">", 1)[0].split(",")[-1].strip()
        return "k_fast_list<LEAD>" if mode == "1" else "k_fast_list<FOLL>"
    if "k_full_list" in name:
        return "k_full_list"
    if "k_step" in name:
        return "k_step"
    return None


def per_kernel(d, counter, scale=1024.0):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            k = kernel_key(row.get("Kernel_Name", ""))
            if k:
                vals[k].append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"])))
    out = {}
    for k, v in vals.items():
        v.sort()
        last = [x for _, x in v[-LAST:]]
        out[k] = sum(last) / len(last) * scale  # KiB -> bytes (sizes)
    return out


def main():
    w, fdir, wdir = sys.argv[1:4]
    rdir = sys.argv[4] if len(sys.argv) > 4 else None
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    import hashlib
    lib = os.environ.get("RBE_LIB") or os.path.join(ROOT, "dragonboat_amd", "libdragonboat_amd.so")
    with open(lib, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    # bench.py reports this traffic only for the same library (content hash)
    res = {"workload": w, "unit": "bytes per launch", "dispatches_averaged": LAST,
           "library_sha256_16": sha, "fetch_raw": fetch, "write": write,
           "fetch_calibration": "scattered 16-B gathers: FETCH_SIZE x 1 (profiles/r05_calibration)",
           "bytes_per_launch": {}, "bytes_per_launch_fetch_x2": {}}
    if rdir:  # request counts per launch (not bytes)
        res["tcp_tcc_write_req"] = per_kernel(rdir, "TCP_TCC_WRITE_REQ_sum", 1.0)
        res["tcp_tcc_read_req"] = per_kernel(rdir, "TCP_TCC_READ_REQ_sum", 1.0)
    for k in set(fetch) | set(write):
        res["bytes_per_launch"][k] = fetch.get(k, 0.0) + write.get(k, 0.0)
        res["bytes_per_launch_fetch_x2"][k] = 2.0 * fetch.get(k, 0.0) + write.get(k, 0.0)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    out = os.path.join(ROOT, "gpurun_out", f"traffic_{w}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in sorted(res["bytes_per_launch"].items()):
        print(f"{w} {k:20s} traffic {v / 1e6:9.2f} MB/launch (fetch raw {fetch.get(k, 0) / 1e6:.2f}"
              f" MB, write {write.get(k, 0) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
