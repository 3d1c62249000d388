"""Host time between two direct bench steps from a scripts/api_trace.sh run:
the HIP API calls (with durations) from the end of one step's K3b to the
start of the next step's probe, and the calls inside the step.

    python scripts/api_gaps.py gpurun_out/prof_<TAG>_api [anchor-kernel-substring]

(the anchor is each step's first kernel: probe_kernel on the direct path,
prep_clear_kernel on the full prepare)
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    kern = list(csv.DictReader(open(glob.glob(os.path.join(d, "*kernel_trace.csv"))[0])))
    api = list(csv.DictReader(open(glob.glob(os.path.join(d, "*hip_api_trace.csv"))[0])))
    kern.sort(key=lambda r: int(r["Start_Timestamp"]))
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    anchor = sys.argv[2] if len(sys.argv) > 2 else "probe_kernel"
    probes = [r for r in kern if anchor in r["Kernel_Name"]]
    k3b = [r for r in kern if "region_final_wave_kernel" in r["Kernel_Name"]]
    # one step: probe[i] .. probe[i+1]
    i = len(probes) // 2
    t0, t1 = int(probes[i]["Start_Timestamp"]), int(probes[i + 1]["Start_Timestamp"])
    ks = [r for r in kern if t0 <= int(r["Start_Timestamp"]) < t1]
    print("kernels of one step:")
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("  %8.1f us  +%7.1f  %s" % ((e - s) / 1e3, (s - t0) / 1e3, r["Kernel_Name"][:60]))
    last = [r for r in k3b if t0 <= int(r["Start_Timestamp"]) < t1][-1]
    te = int(last["End_Timestamp"])
    a0 = int(probes[i]["Start_Timestamp"]) - 200_000
    print("API calls from 200 us before the anchor to the next one (relative to the anchor's start):")
    for r in api:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if a0 <= s < t1:
            print("  %+9.1f  %7.1f us  %s" % ((s - t0) / 1e3, (e - s) / 1e3, r["Function"]))
    print("K3b end -> next anchor start: %.1f us" % ((t1 - te) / 1e3))


if __name__ == "__main__":
    main()
