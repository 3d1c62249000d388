#!/bin/bash
# End-to-end CLI-path timing on the GPU box (scripts/e2e.py), one step under its own limit.
set -u
mkdir -p gpurun_out /tmp/e2e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python scripts/e2e.py --reads ${READS:-30000000} --contigs 1000 --length 1000000 --dir /tmp/e2e > gpurun_out/${TAG:-e2e}.json 2> gpurun_out/${TAG:-e2e}.err
s=$?; tail -3 gpurun_out/${TAG:-e2e}.err; cat gpurun_out/${TAG:-e2e}.json; exit $s
