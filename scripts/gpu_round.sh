#!/bin/bash
# round-end evidence on one box: GPU suite, C1 echo times, C2 rocprof stats +
# PMC passes, the default bench line and the PCIe-inclusive rate; TAG names
# the files under gpurun_out/ (copy the ones to keep into profiles/)
set -o pipefail
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { echo "c1 failed"; tail -20 gpurun_out/${TAG}_c1_echo.log; exit 2; }
grep "C1 echo" gpurun_out/${TAG}_c1_echo.log
TAG=$TAG bash scripts/profile.sh || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG/err.log; exit 3; }
bash scripts/run_bench.sh ${TAG}_bench 600 "d['value'], d['parity_ok']" || exit 4
timeout -k 10 300 python -u scripts/e2e.py > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 5; }
cat gpurun_out/${TAG}_e2e.json; tail -c 600 gpurun_out/${TAG}_bench.json
