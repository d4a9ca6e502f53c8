#!/bin/bash
# round 5: serial resolve step width (BPMD_BP_RSYM 16 / 32 / 64) on shards; BP parity
set -o pipefail
TAG=${TAG:-r05n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in rs16 default rs64; do
    if [ $v = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
    for cfg in "c4 6 8" "c5 1 8"; do
      set -- $cfg
      BPMD_LIB=$L timeout -k 10 200 python -u scripts/diag_own_shard.py $1 $2 $3 3 > $OUT/own_${v}_$1_$r.log 2>&1 || exit 2
      echo "$v own $1 | $(tail -1 $OUT/own_${v}_$1_$r.log | cut -c1-70)"
    done
    BPMD_LIB=$L timeout -k 10 200 python -u scripts/diag_beast_shard.py c4 6 8 3 > $OUT/beast_${v}_c4_$r.log 2>&1 || exit 3
    echo "$v beast c4 | $(tail -1 $OUT/beast_${v}_c4_$r.log | cut -c1-70)"
  done
done
