"""A/B of GPU-decode builds (metacov_amd/variants/lib_<name>.so) on one
synthetic BAM in one process: inflate / parse / total ms per variant and a
checksum of the decoded intervals (must agree).

    python scripts/gz_ab.py --reads 10000000 name1 name2 ...
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    from metacov_amd import synth, _lib
    lengths = np.full(1000, 1_000_000, np.int64)
    path = os.path.join(tempfile.mkdtemp(), "ab.bam")
    t0 = time.perf_counter()
    arrs = synth.edge_mix_arrays(lengths, a.reads, seed=1)
    synth.write_bam_fast(path, ["c%d" % i for i in range(1000)], lengths, *arrs, level=6, n_threads=16)
    print("wrote %s (%.2f GB) in %.1f s" % (path, os.path.getsize(path) / 1e9, time.perf_counter() - t0),
          flush=True)
    out = {}
    libs = {name: _lib.load(os.path.join(ROOT, "metacov_amd", "variants", "lib_%s.so" % name))
            for name in a.variants}
    for rep in range(a.reps):             # interleaved: rep-major, every variant per rep
        for name in a.variants:
            lib = libs[name]
            h = ctypes.c_void_p()
            _lib.check(lib.mc_bam_gpu_open(path.encode(), 0, 16, 0x704, a.window, ctypes.byref(h)), lib)
            t = _lib.GpuDecodeTimings()
            _lib.check(lib.mc_bam_gpu_stats(h, ctypes.byref(t)), lib)
            n = ctypes.c_int64()
            ptrs = [ctypes.c_void_p() for _ in range(3)]
            _lib.check(lib.mc_bam_gpu_intervals_device(h, ctypes.byref(n), *[ctypes.byref(p) for p in ptrs]), lib)
            iv = [np.empty(n.value, np.int32) for _ in range(3)]
            _lib.check(lib.mc_bam_gpu_intervals(h, *[_lib.ptr(x) for x in iv]), lib)
            ck = int(sum(int(np.bitwise_xor.reduce(x.view(np.uint32) * np.uint32(2654435761) + np.arange(len(x), dtype=np.uint32)))
                         for x in iv))
            lib.mc_bam_gpu_close(h)
            r = {k: getattr(t, k) for k, _ in t._fields_}
            r["n_kept"] = n.value
            r["checksum"] = ck
            out.setdefault(name, []).append(r)
            print(name, rep, "inflate %.1f ms (kernels %.1f)  parse %.1f ms  read %.1f ms (uploads %.1f)  total %.1f ms  "
                  "resyncs %d  kept %d  ck %d"
                  % (r["inflate_ms"], r.get("kernel_ms", 0), r["parse_ms"], r["read_ms"], r.get("upload_ms", 0),
                     r["total_ms"], r["resyncs"], n.value, ck),
                  flush=True)
    cks = {v[-1]["checksum"] for v in out.values()}
    print(json.dumps({"agree": len(cks) == 1, "runs": out}))
    os.remove(path)


if __name__ == "__main__":
    main()
