#!/bin/bash
# e2e against its copy-only bound, three chunkings
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05zzi_e2e.log
: > $O
for cfg in "--chunks 8 --depth 3" "--chunks 16 --depth 4" "--chunks 32 --depth 4"; do
  echo "== $cfg" >> $O
  timeout -k 10 240 python scripts/e2e.py $cfg >> $O 2>&1 || { echo "e2e $cfg failed"; tail $O; exit 1; }
done
grep -v amdgpu.ids $O
