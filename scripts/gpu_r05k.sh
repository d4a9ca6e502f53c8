#!/bin/bash
# round 5: single-write chunk-parallel deflate -- deflate parity, A/B vs the stitch
set -o pipefail
TAG=${TAG:-r05k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py \
  tests/test_gpu_stream.py tests/test_gpu_frame.py tests/test_gpu_multi.py tests/test_gpu_batcher.py tests/test_gpu_async.py \
  -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  for v in stitch single; do
    if [ $v = stitch ]; then export BPMD_DEFLATE_STITCH=1; else export BPMD_DEFLATE_STITCH=0; fi
    bash scripts/run_bench.sh ${TAG}_ab_${v}_$r 600 "d['deflate']['deflate_value'], [(k, v.get('deflate_value'), v.get('ratio_rank_local')) for k, v in d['mixed'].items() if isinstance(v, dict)]" \
      --steps 5 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-virtual-shards --no-beast-payloads || exit 2
  done
done
unset BPMD_DEFLATE_STITCH
