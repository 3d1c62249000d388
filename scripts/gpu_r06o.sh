#!/bin/bash
# round 6: the N=8 share (12.5 M reads, 125 contigs): chunk-count floor A/B, in process.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
export PYTHONUNBUFFERED=1
faulted() { if grep -qiE "illegal memory access|memory access fault|hipErrorLaunchFailure|gpu hang" "$@" 2>/dev/null; then echo "GPU fault in $*: stopping"; exit 90; fi; }
V=metacov_amd/variants
L="$V/lib_base.so $V/lib_mc2k.so $V/lib_mc1k.so"
timeout -k 10 400 python scripts/ab_inproc.py --libs $L --mode direct --config c3 --reads 12500000 --contigs 125 --rounds 6 --steps 10 > $O/r06o_ab_direct_shard8.txt 2>&1
s=$?; grep -v amdgpu.ids $O/r06o_ab_direct_shard8.txt | tail -4; faulted $O/r06o_ab_direct_shard8.txt; [ $s -eq 0 ] || exit $s
echo done
