#!/bin/bash
# round 6 (last tree): rocprofv3 trace + FETCH_SIZE + WRITE_SIZE passes of the bench on the
# final kernels, per config (C3, C2, C5, one N=8 share), for scripts/pmc_summary.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=r06last_c3 SQ_PASSES="" bash scripts/profile.sh || exit 1
TAG=r06last_c2 BENCH_ARGS="--config c2" SQ_PASSES="" bash scripts/profile.sh || exit 1
TAG=r06last_c5 BENCH_ARGS="--config c5" SQ_PASSES="" bash scripts/profile.sh || exit 1
TAG=r06last_s8 BENCH_ARGS="--reads 12500000 --contigs 125" SQ_PASSES="" bash scripts/profile.sh || exit 1
echo done
