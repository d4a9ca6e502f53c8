#!/bin/bash
# round 5: compact canonical search (BPMD3_CKL/CKD) -- lane-kernel parity, C2 A/B
set -o pipefail
TAG=${TAG:-r05j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_bp.py tests/test_gpu_takeover.py \
  tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2 3; do
  for v in ck0 default ck9; do
    if [ $v = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_ab_${v}_$r 200 "d['value'], d['roofline']['kernel_ms'], d['parity_ok']" \
      --steps 20 --warmup 3 --no-cpu-baseline --no-mixed --no-deflate --no-frame || exit 2
  done
done
for st in 1 4; do
  export BPMD_BP_DYN_STRIDE=$st
  for cfg in "c4 6 8" "c5 1 8"; do
    set -- $cfg
    timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 3 > $OUT/stride_${st}_$1.log 2>&1 || exit 3
    echo "dyn stride $st beast $1 | $(tail -1 $OUT/stride_${st}_$1.log | cut -c1-110)"
  done
done
unset BPMD_BP_DYN_STRIDE
bash scripts/gpu_r05i.sh
