#!/bin/bash
# parse segment floor 32 vs 16 bytes per lane: facade latency, C1 wire bytes, C3/C4 rate and size
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05ze}
for v in default ms16; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L timeout -k 10 300 python -u scripts/facade_latency.py > gpurun_out/${TAG}_${v}_lat.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_lat.log; exit 1; }
  echo "$v $(grep facade gpurun_out/${TAG}_${v}_lat.log)"
  BPMD_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_facade.py -m gpu -k echo -q -s --timeout 280 --timeout-method thread > gpurun_out/${TAG}_${v}_c1.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_c1.log; exit 2; }
  echo "$v $(grep 'C1 echo' gpurun_out/${TAG}_${v}_c1.log)"
  BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_${v} 400 \
    "d['deflate']['deflate_value'], d['deflate']['ratio'], {k: (v['deflate_value'], round(v['ratio_rank_local'] / {'c4_l6': 0.2857, 'c5_l1': 0.9856, 'c5_l6': 0.9700}[k], 4)) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-virtual-shards --no-beast-payloads || exit 3
done
