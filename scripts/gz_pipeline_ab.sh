#!/bin/bash
# GPU decode pipeline A/B (scripts/gz_pipeline_ab.py) on the 30 M-record e2e BAM.
set -u
mkdir -p gpurun_out /tmp/e2e
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/gz_pipeline_ab.py --make /tmp/e2e/ab.bam || exit $?
timeout -k 10 600 python scripts/gz_pipeline_ab.py --bam /tmp/e2e/ab.bam --rounds ${ROUNDS:-3} --libs "$@" > gpurun_out/${TAG:-gzab}.txt 2>&1
s=$?; cat gpurun_out/${TAG:-gzab}.txt; exit $s
