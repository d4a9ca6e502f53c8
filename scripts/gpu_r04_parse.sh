#!/bin/bash
# deflate parse A/B (default vs VARIANTS), phase diagnostics, C5 shard BP diag
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deflate.py -x -q --timeout 200 --timeout-method thread > gpurun_out/parse_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/parse_pytest.log; [ $rc -eq 0 ] || exit 1
AB_ARGS="--no-mixed --no-frame --no-exact" VARIANTS="$VARIANTS" bash scripts/ab.sh || exit 2
VARIANTS="$VARIANTS" bash scripts/ab_deflate_mixed.sh || exit 3
for cfg in "json 4096 6 65536" "json 65536 6 4096" "binary 65536 1 4096"; do
  set -- $cfg
  BPMD_LIB=$PWD/beast_amd/libbeast_pmd_prof.so DIAG_KIND=$1 DIAG_SIZE=$2 DIAG_LEVEL=$3 DIAG_MSGS=$4 \
    timeout -k 10 120 python -u scripts/diag_deflate.py > gpurun_out/diag_$1_$2.log 2>&1 || exit 4
  grep "msgs\|parse\|active\|total" gpurun_out/diag_$1_$2.log
done
for v in $BP_VARIANTS; do  # (optional)
  for pr in gpu beast; do
    BPMD_LIB=$PWD/beast_amd/$v timeout -k 10 150 python -u scripts/diag_bp.py case binary 2048 65536 $pr 1 auto 2>&1 | grep -v amdgpu.ids || exit 5
  done
done
echo done
