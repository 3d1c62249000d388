#!/bin/bash
# Queue a gpurun call: retries only while no GPU slot is free (nothing ran,
# nothing charged); any other outcome, a failure included, ends it.
#   scripts/gpq.sh OUT.log --timeout S -- "command"
out=$1; shift
for i in $(seq 1 40); do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  if grep -qE "are busy|status=transient|no free box|backing off" "$out"; then sleep 60; continue; fi
  break
done
echo "[gpq] done after $i tries" >> "$out"
