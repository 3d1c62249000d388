"""SQ counters of the scan kernels (scripts/gpu_scan_sq.sh) -> profiles/sq_scan_kernel.json.

    python scripts/sq_scan_summary.py TAG [NAME]

Per kernel (scan_kernel, kmer_count_kernel) of one bench_scan launch over
the C3-shaped 100 M reads: the SQ instruction counts, wave cycles and busy
cycles, stamped with a fingerprint of csrc/scan.hip; scripts/bench_scan.py
reports its issue roofline from this file when the fingerprint matches.
"""
import collections
import csv
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def scan_source_id(root=ROOT):
    h = hashlib.sha256()
    with open(os.path.join(root, "metacov_amd", "csrc", "scan.hip"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def main():
    tag = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "libmetacov_amd"
    path = os.path.join(ROOT, "gpurun_out", "prof_%s_%s" % (tag, name), "run_counter_collection.csv")
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        for kn in ("scan_kernel", "kmer_count_kernel"):
            if re.search(r"(^|[:\s])%s[<(]" % kn, k):
                agg[kn][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {"source_id": scan_source_id(), "tag": tag, "reads": 100_000_000,
           "kernels": {k: dict(v) for k, v in agg.items()},
           "note": "one launch of each kernel (bench_scan --steps 1 --warmup 0), counters summed over the launch"}
    dst = os.path.join(ROOT, "profiles", "sq_scan_kernel.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
