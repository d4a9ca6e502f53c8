#!/bin/bash
# deflate parse: three candidates per iteration (variant) -- parity, then A/B against two
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05za}
BPMD_LIB=beast_amd/libbeast_pmd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_deflate.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_deflate.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_deflate.log
for round in 1 2; do
for v in default x8; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_${v}_$round 400 \
    "d['deflate']['deflate_value'], d['deflate']['ratio'], {k: (v['deflate_value'], round(v['ratio_rank_local'] / {'c4_l6': 0.2857, 'c5_l1': 0.9856, 'c5_l6': 0.9700}[k], 4), v['roundtrip_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-virtual-shards --no-beast-payloads || exit 2
done
done
