#!/bin/bash
# round 5: per-stream inflater prefetch -- parity, facade latency, C1 echo; single-write test
set -o pipefail
TAG=${TAG:-r05l}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstream.py tests/test_gpu_stream.py tests/test_gpu_deflate.py tests/test_facade.py \
  -x -q --timeout 280 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/facade_latency.py 256 > $OUT/lat.log 2>&1 || { tail $OUT/lat.log; exit 2; }
grep facade $OUT/lat.log
timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > $OUT/c1_echo.log 2>&1 || { tail -20 $OUT/c1_echo.log; exit 3; }
grep "C1 echo" $OUT/c1_echo.log
