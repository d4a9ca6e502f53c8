#!/bin/bash
# round-5 evidence, part B: C2 rocprof (kernel trace, FETCH/WRITE, calibration),
# the default bench line, the PCIe-inclusive rate, C2 SQ counters
set -o pipefail
TAG=${TAG:-r05m}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_multi.py > gpurun_out/${TAG}_pytest_multi.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest_multi.log; exit 2; }
tail -2 gpurun_out/${TAG}_pytest_multi.log
TAG=$TAG bash scripts/profile.sh || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG/err.log; exit 3; }
bash scripts/run_bench.sh ${TAG}_bench 900 "d['value'], d['parity_ok']" || exit 4
timeout -k 10 300 python -u scripts/e2e.py > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 5; }
cat gpurun_out/${TAG}_e2e.json
TAG=$TAG BENCH_ARGS="--no-mixed --no-deflate --no-frame" bash scripts/pmc_sq.sh || exit 6
python scripts/sq_summary.py gpurun_out/sq_$TAG > gpurun_out/${TAG}_c2_sq.txt
tail -c 1500 gpurun_out/${TAG}_bench.json
