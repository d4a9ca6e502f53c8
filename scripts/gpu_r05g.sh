#!/bin/bash
# round 5: per-stream facade latency (pinned staging, one D2H per call, no
# chunk-count read-back) -- per-stream parity and the C1 echo
set -o pipefail
TAG=${TAG:-r05g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_facade.py tests/test_gpu_takeover.py \
  -x -q --timeout 280 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > $OUT/c1_echo.log 2>&1 || { tail -20 $OUT/c1_echo.log; exit 2; }
grep "C1 echo" $OUT/c1_echo.log
