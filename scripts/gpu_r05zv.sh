#!/bin/bash
# stream deflate: one setup launch for a known single message -- parity, latency, C1
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zv}
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_deflate.py tests/test_facade.py tests/test_gpu_reference_pins.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_lat.log 2>&1 || { tail -5 gpurun_out/${TAG}_lat.log; exit 2; }
grep facade gpurun_out/${TAG}_lat.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_c1_echo.log 2>&1 || { tail -5 gpurun_out/${TAG}_c1_echo.log; exit 3; }
grep 'C1 echo' gpurun_out/${TAG}_c1_echo.log
