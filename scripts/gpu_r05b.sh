#!/bin/bash
# round 5: interleaved per-lane LDS (BPMD3_ILV) -- lane-kernel parity, C2 A/B
# against the contiguous layout (libbeast_pmd_ilv0.so), SQ counters
set -o pipefail
TAG=${TAG:-r05b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_bp.py tests/test_gpu_takeover.py \
  tests/test_gpu_configs.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for r in 1 2 3; do
  for v in ilv0 default; do
    if [ $v = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_ab_${v}_$r 200 "d['value'], d['roofline']['kernel_ms'], d['parity_ok']" \
      --steps 20 --warmup 3 --no-cpu-baseline --no-mixed --no-deflate --no-frame || exit 2
  done
done
TAG=$TAG BENCH_ARGS="--no-mixed --no-deflate --no-frame" bash scripts/pmc_sq.sh || exit 3
python scripts/sq_summary.py gpurun_out/sq_$TAG 2>&1 | tail -30
