#!/bin/bash
# round 5, first box: the changed GPU tests, a C2 bench line, SQ counters of C2
set -o pipefail
TAG=${TAG:-r05a}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_async.py tests/test_gpu_bench_launch.py \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-mixed --no-deflate --no-frame > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || exit 2
cat gpurun_out/${TAG}_c2.json
TAG=$TAG BENCH_ARGS="--no-mixed --no-deflate --no-frame" bash scripts/pmc_sq.sh || exit 3
