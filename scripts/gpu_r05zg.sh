#!/bin/bash
# deflate parity after the per-history segment floor, C1 wire bytes and facade latency
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zg}
timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_gpu_reference_pins.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_deflate.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_deflate.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_deflate.log
timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_facade_latency.log 2>&1 || { tail -5 gpurun_out/${TAG}_facade_latency.log; exit 2; }
grep facade gpurun_out/${TAG}_facade_latency.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { tail -5 gpurun_out/${TAG}_c1_echo.log; exit 3; }
grep 'C1 echo' gpurun_out/${TAG}_c1_echo.log
