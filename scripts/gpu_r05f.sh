#!/bin/bash
# round 5: fixed-block skim + BFINAL filter -- BP parity; Beast shards skim on/off
set -o pipefail
TAG=${TAG:-r05f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in "c5 1 8" "c5 6 8" "c4 6 8" "c5 1 1"; do
  set -- $cfg
  for r in on off; do
    if [ $r = off ]; then export BPMD_BP_SKIM=0; else export BPMD_BP_SKIM=1; fi
    timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 3 > $OUT/diag_${r}_$1_$2_$3.log 2>&1 || { tail $OUT/diag_${r}_$1_$2_$3.log; exit 2; }
    echo "skim $r $(sed -n 2p $OUT/diag_${r}_$1_$2_$3.log) | $(tail -1 $OUT/diag_${r}_$1_$2_$3.log)"
  done
done
unset BPMD_BP_SKIM
(cd /tmp && export TMPDIR=/tmp BPMD_BP_SKIM=1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_c5 -o t \
    -- python3 $GRAFT_REPO_ROOT/scripts/diag_beast_shard.py c5 1 8 3 > /dev/null 2>&1) || exit 3
python3 scripts/kernel_summary.py $(find $OUT/prof_c5 -name "t_kernel_trace.csv" | head -1) > $OUT/kernels_c5_1_8.csv || exit 4
head -8 $OUT/kernels_c5_1_8.csv
