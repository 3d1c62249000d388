#!/bin/bash
# Build tuning variants of libmetacov_amd.so into metacov_amd/variants/.
#   scripts/build_variants.sh name1 "-DMC_X=.." name2 "-DMC_Y=.." ...
# (each through metacov_amd/build.py, so every variant carries its own source
# stamp and the same source list as the product library)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/metacov_amd/variants"
cd "$R"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  python -c "import sys; from metacov_amd import build; build.build(verbose=False, extra_flags=tuple(sys.argv[2:]), out=sys.argv[1])" \
      "$R/metacov_amd/variants/lib_$name.so" $flags &
done
wait
ls -la "$R/metacov_amd/variants"
