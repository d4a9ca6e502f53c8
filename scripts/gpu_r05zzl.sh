#!/bin/bash
# e2e: chunks all in flight at once (one stream each) vs the round-5 default
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05zzn_e2e.log
: > $O
for cfg in "--dchunks 8 --ddepth 1" "--dchunks 16 --ddepth 1" "--dchunks 8 --ddepth 2" "--dchunks 4 --ddepth 1"; do
  echo "== $cfg" >> $O
  timeout -k 10 240 python scripts/e2e.py $cfg >> $O 2>&1 || { echo "e2e $cfg failed"; tail $O; exit 1; }
done
grep -v amdgpu.ids $O
