#!/bin/bash
# Round-4 baseline on one box: C2-only bench line, SQ counters of the C2
# launch (pmc_lane3.sh) and the prof build's per-role loop counters.
set -o pipefail
TAG=${TAG:-r04a}
mkdir -p gpurun_out
C2="--no-cpu-baseline --no-mixed --no-deflate --no-frame --no-exact"
bash scripts/run_bench.sh ${TAG}_c2 200 "d['value'], d['roofline']['kernel_ms'], d['parity_ok']" $C2 || exit 1
TAG=$TAG bash scripts/pmc_lane3.sh > gpurun_out/${TAG}_sq.txt 2>&1 || { cat gpurun_out/${TAG}_sq.txt; exit 2; }
cat gpurun_out/${TAG}_sq.txt
timeout -k 10 120 python -u scripts/diag_lane3.py > gpurun_out/${TAG}_diag.txt 2>&1 || { tail gpurun_out/${TAG}_diag.txt; exit 3; }
cat gpurun_out/${TAG}_diag.txt
