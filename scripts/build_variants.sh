#!/bin/bash
# Build tuning variants of libmetacov_amd.so into metacov_amd/variants/.
#   scripts/build_variants.sh name1 "-DMC_X=.." name2 "-DMC_Y=.." ...
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/metacov_amd/variants"
cd "$R/metacov_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags \
      -o "$R/metacov_amd/variants/lib_$name.so" engine.hip ecor.hip scan.hip bam_decode.cpp bam_index.cpp bam_write.cpp exp_reads.cpp scan_src.cpp common.cpp -lz -lpthread -ldl &
done
wait
ls -la "$R/metacov_amd/variants"
