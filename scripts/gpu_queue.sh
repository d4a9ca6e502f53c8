#!/bin/bash
# the work queue under the whole inflate parity suite (grid capped to 1 and 3
# workgroups: every message after the first 64 / 192 goes through the queue),
# then the C4/C5 legs
set -o pipefail
mkdir -p gpurun_out
for w in 1 3; do
  BPMD_QUEUE_WGS=$w timeout -k 10 400 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_takeover.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > gpurun_out/queue_pytest_$w.log 2>&1
  rc=$?; tail -3 gpurun_out/queue_pytest_$w.log; [ $rc -eq 0 ] || exit 1
done
bash scripts/gpu_c4.sh
