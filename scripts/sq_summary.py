"""Per-kernel averages of the SQ counter passes of scripts/profile.sh.

    python scripts/sq_summary.py TAG [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "depth_kernel"
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", "prof_%s_sq*" % tag, "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if sub in k:
                agg[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(k)
        for c, v in sorted(cs.items()):
            print("  %-24s %16.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
