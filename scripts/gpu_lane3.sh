#!/bin/bash
# lane-kernel change check: inflate parity suites, then C2 A/B against VARIANTS
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lane3_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/lane3_pytest.log; [ $rc -eq 0 ] || exit 1
AB_ARGS="--no-deflate --no-mixed --no-frame" bash scripts/ab.sh
