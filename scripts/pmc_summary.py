"""Summarise a scripts/profile.sh run into profiles/ (tracked).

  python scripts/pmc_summary.py r01 [--reads 100000000 --contigs 1000]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, as produced),
profiles/<tag>_pmc.json (per-kernel average FETCH_SIZE / WRITE_SIZE) and
profiles/pmc_depth_kernel.json (what bench.py reports as roofline.traffic).
HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE /
WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE counts half the bytes of a
16-byte-per-lane coalesced stream (MI355X_MICROARCH.md §HBM), which is how
depth_kernel and region_seg_kernel load.
"""
import argparse
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import kernel_source_id  # noqa: E402


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--contigs", type=int, default=1000)
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(out, "prof_%s_trace" % a.tag, "run_kernel_stats.csv"),
                os.path.join(prof, "%s_kernel_stats.csv" % a.tag))
    fetch = per_kernel(os.path.join(out, "prof_%s_fetch" % a.tag, "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(out, "prof_%s_write" % a.tag, "run_counter_collection.csv"), "WRITE_SIZE")
    stats = {r["Name"].split("(")[0]: r for r in
             csv.DictReader(open(os.path.join(prof, "%s_kernel_stats.csv" % a.tag)))}
    rows = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith(("mc::", "void mc::")):
            continue
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        hbm = (2 * f + w) * 1024
        st = stats.get(k)
        avg_ns = float(st["AverageNs"]) if st else None
        rows[k] = {"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": hbm,
                   "avg_ns": avg_ns,
                   "hbm_GBps": hbm / avg_ns if avg_ns else None}
    with open(os.path.join(prof, "%s_pmc.json" % a.tag), "w") as fh:
        json.dump(rows, fh, indent=1)
    path = os.path.join(prof, "pmc_depth_kernel.json")
    variants = json.load(open(path)).get("variants", []) if os.path.exists(path) else []
    # the kernels bench.py may report as roofline.traffic: K2 (and K1 in --cigar runs)
    for dk_name in [k for k in rows if "depth_kernel" in k or "cigar_span_kernel" in k]:
        dk = rows[dk_name]
        entry = {"tag": a.tag, "kernel": dk_name, "reads": a.reads, "contigs": a.contigs,
                 "source_id": kernel_source_id(ROOT),
                 "hbm_bytes_per_launch": dk["hbm_bytes_per_launch"],
                 "fetch_kib": dk["FETCH_SIZE_KiB"], "write_kib": dk["WRITE_SIZE_KiB"],
                 "avg_ns": dk["avg_ns"],
                 "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; "
                           "bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB (gfx950 FETCH_SIZE counts 1/2 "
                           "of 16 B/lane streams)"}
        variants = [v for v in variants
                    if (v["kernel"], v.get("reads"), v.get("contigs")) != (dk_name, a.reads, a.contigs)]
        variants.append(entry)
    with open(path, "w") as fh:
        json.dump({"variants": variants}, fh, indent=1)
    for k, v in rows.items():
        print("%-28s %8.3f ms  %7.3f GB  %7.0f GB/s" % (k, (v["avg_ns"] or 0) / 1e6,
                                                      v["hbm_bytes_per_launch"] / 1e9, v["hbm_GBps"] or 0))


if __name__ == "__main__":
    main()
