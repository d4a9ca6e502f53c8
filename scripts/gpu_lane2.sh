#!/bin/bash
# lane kernel v2 bring-up: inflate parity (both designs), then A/B timing on C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lane2_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/lane2_pytest.log; [ $rc -eq 0 ] || exit 1
for d in 1 2 3; do
  echo "== BPMD_LANE=$d"
  BPMD_LANE=$d timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-mixed --no-deflate --no-frame 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('inflate', d['value'], d['roofline']['kernel_ms'], d['parity_ok'])" || exit 2
done
