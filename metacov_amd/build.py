"""Builds libmetacov_amd.so in-tree with hipcc for gfx950.

    python -m metacov_amd.build

The library is plain C ABI (no torch types): HIP kernels + host engine +
host BAM decoder, linked against the HIP runtime and zlib.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmetacov_amd.so")
SOURCES = ["engine.hip", "ecor.hip", "scan.hip", "bam_decode.cpp", "bam_index.cpp",
           "bam_write.cpp", "exp_reads.cpp", "scan_src.cpp", "depth_cap.cpp", "common.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build(verbose=True, extra_flags=()):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, "kernels.h"), os.path.join(CSRC, "common.h"),
            os.path.join(CSRC, "bgzf.h"),
                   os.path.join(os.path.dirname(HERE), "include", "metacov_amd.h")]
    if os.path.exists(LIB) and not extra_flags and \
            os.path.getmtime(LIB) > max(os.path.getmtime(d) for d in deps):
        return LIB
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", *extra_flags,
           "-o", LIB + ".tmp", *srcs, "-lz", "-lpthread", "-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(extra_flags=tuple(sys.argv[1:]))
