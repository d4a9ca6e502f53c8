#!/bin/bash
# round-5 final evidence, part B: C2 rocprof (kernel trace, FETCH/WRITE, calibration),
# the default bench line, the PCIe-inclusive rate, C2 SQ counters, one 8-way shard's kernels
set -o pipefail
TAG=${TAG:-r05zz}
mkdir -p gpurun_out
TAG=$TAG bash scripts/profile.sh || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG/err.log; exit 3; }
bash scripts/run_bench.sh ${TAG}_bench 900 "d['value'], d['parity_ok']" || exit 4
timeout -k 10 300 python -u scripts/e2e.py > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 5; }
cat gpurun_out/${TAG}_e2e.json
TAG=$TAG BENCH_ARGS="--no-mixed --no-deflate --no-frame" bash scripts/pmc_sq.sh || exit 6
python scripts/sq_summary.py gpurun_out/sq_$TAG > gpurun_out/${TAG}_c2_sq.txt
TAG=$TAG bash scripts/prof_shards.sh > gpurun_out/${TAG}_shards.log 2>&1 || { tail -10 gpurun_out/${TAG}_shards.log; exit 7; }
tail -c 1200 gpurun_out/${TAG}_bench.json
