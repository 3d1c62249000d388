"""Builds libmetacov_amd.so in-tree with hipcc for gfx950.

    python -m metacov_amd.build

The library is plain C ABI (no torch types): HIP kernels + host engine +
host BAM decoder, linked against the HIP runtime and zlib.

The build stamps a SHA-256 of its sources, headers and compile flags into the
library (mc_build_id()); it rebuilds whenever the stamp in the existing .so
differs from the tree's, so a library built from other sources is never
reused (the .so is untracked but travels with the tree to the GPU box).
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libmetacov_amd.so")
SOURCES = ["engine.hip", "ecor.hip", "scan.hip", "bam_gpu.hip", "exp_gpu.hip", "bam_decode.cpp", "bam_index.cpp",
           "bam_write.cpp", "exp_reads.cpp", "scan_src.cpp", "depth_cap.cpp", "common.cpp", "runtime.cpp"]
HEADERS = ["kernels.h", "npstd.h", "capmask.h", "exp_gpu.h", "common.h", "bgzf.h", "inflate.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
         "-Wno-unused-function"]
STAMP = b"mc-source-sha256:"


def source_hash(extra_flags=()):
    """SHA-256 over the sources, the headers and the compile flags."""
    h = hashlib.sha256()
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + \
        [os.path.join(os.path.dirname(HERE), "include", "metacov_amd.h")]
    for d in deps:
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + list(extra_flags)).encode())
    return h.hexdigest()


def built_hash(path=LIB):
    """The stamp inside an existing library, or None."""
    try:
        with open(path, "rb") as fh:
            blob = fh.read()
    except OSError:
        return None
    i = blob.find(STAMP)
    return blob[i + len(STAMP):i + len(STAMP) + 64].decode("ascii", "replace") if i >= 0 else None


def build(verbose=True, extra_flags=(), out=LIB):
    digest = source_hash(extra_flags)
    if built_hash(out) == digest:
        return out
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    cmd = [HIPCC, *FLAGS, *extra_flags, '-DMC_SOURCE_HASH="%s"' % digest,
           "-o", out + ".tmp", *srcs, "-lz", "-lpthread", "-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(extra_flags=tuple(sys.argv[1:]))
