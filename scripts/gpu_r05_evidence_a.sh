#!/bin/bash
# round-5 evidence, part A: the whole GPU suite and the C1 echo (TAG names the files)
set -o pipefail
TAG=${TAG:-r05m}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { echo "c1 failed"; tail -20 gpurun_out/${TAG}_c1_echo.log; exit 2; }
grep "C1 echo" gpurun_out/${TAG}_c1_echo.log
