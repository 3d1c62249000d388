#!/bin/bash
# round 6: C5 K2 SQ breakdown (trace, FETCH/WRITE, SQ sets A and B) on the
# current tree (fill back on the unsorted stores).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=r06i BENCH_ARGS="--config c5" SQ_PASSES="A B" PROF_STEPS=5 bash scripts/profile.sh || exit 1
echo done
