#!/bin/bash
# Round-4 baseline on one box: C2-only bench line, SQ counters of the C2
# launch (pmc_lane3.sh) and the prof build's per-role loop counters.
set -o pipefail
TAG=${TAG:-r04a}
mkdir -p gpurun_out
C2="--no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact"
timeout -k 10 200 python -u bench.py $C2 > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err; rc=$?
echo "bench rc=$rc" >> gpurun_out/${TAG}_c2.err
[ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_c2.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_c2.json
TAG=$TAG bash scripts/pmc_lane3.sh > gpurun_out/${TAG}_sq.txt 2>&1 || { cat gpurun_out/${TAG}_sq.txt; exit 2; }
cat gpurun_out/${TAG}_sq.txt
timeout -k 10 120 python -u scripts/diag_lane3.py > gpurun_out/${TAG}_diag.txt 2>&1 || { tail gpurun_out/${TAG}_diag.txt; exit 3; }
cat gpurun_out/${TAG}_diag.txt
