#!/bin/bash
# round-end evidence on one box: GPU suite, C2 rocprof stats + PMC passes,
# the default bench line and the PCIe-inclusive e2e rate; TAG names the files
set -o pipefail
TAG=${TAG:-r02c}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
TAG=$TAG bash scripts/profile.sh || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG/err.log; exit 2; }
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
timeout -k 10 300 python -u scripts/e2e.py > gpurun_out/${TAG}_e2e.json 2> gpurun_out/${TAG}_e2e.err || { tail -20 gpurun_out/${TAG}_e2e.err; exit 4; }
cat gpurun_out/${TAG}_e2e.json; tail -c 1500 gpurun_out/${TAG}_bench.json
