#!/bin/bash
# block-parallel path check: BP / config parity tests, then the mixed legs.
set -o pipefail
TAG=${TAG:-r04l}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_configs.py tests/test_gpu_inflate.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; }
bash scripts/run_bench.sh ${TAG}_bench 600 "d['value'], d['parity_ok']" --no-cpu-baseline --no-exact --no-frame
