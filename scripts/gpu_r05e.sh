#!/bin/bash
# round 5: segment-parallel resolve -- BP parity, A/B vs the serial resolve on
# shards (own and Beast payloads), the mixed legs; e2e variants
set -o pipefail
TAG=${TAG:-r05e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_inflate.py tests/test_gpu_configs.py \
  -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in "c4 6 8" "c5 1 8" "c4 6 4"; do
  set -- $cfg
  for r in new serial; do
    if [ $r = serial ]; then export BPMD_BP_RESOLVE=serial; else unset BPMD_BP_RESOLVE; fi
    timeout -k 10 200 python -u scripts/diag_beast_shard.py $1 $2 $3 3 > $OUT/diag_${r}_$1_$2_$3.log 2>&1 || { tail $OUT/diag_${r}_$1_$2_$3.log; exit 2; }
    echo "$r $(tail -1 $OUT/diag_${r}_$1_$2_$3.log)"
  done
done
unset BPMD_BP_RESOLVE
bash scripts/run_bench.sh ${TAG}_mixed 900 "[(k, v.get('inflate_value'), v.get('inflate_beast_value')) for k, v in d['mixed'].items() if isinstance(v, dict)]" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-deflate --no-frame || exit 3
python - <<'PY'
import json
d = json.load(open('gpurun_out/r05e_mixed.json'))
for k, v in d['mixed'].items():
    if not isinstance(v, dict): continue
    for p, s in v.get('virtual_shards', {}).items():
        print(k, p, 'own', s['inflate_projected_speedup'], max(s['inflate_shard_ms']), 'beast', s.get('inflate_beast_projected_speedup'), max(s.get('inflate_beast_shard_ms', [0])), 'deflate', s['deflate_projected_speedup'])
PY
for v in "8 3" "16 4"; do
  set -- $v
  timeout -k 10 200 python -u scripts/e2e.py --chunks $1 --depth $2 > $OUT/e2e_$1_$2.json 2>> $OUT/e2e.err || exit 4
  echo "e2e chunks $1 depth $2: $(cat $OUT/e2e_$1_$2.json)"
done
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u scripts/e2e.py --chunks 8 --depth 3 > $OUT/e2e_nosdma.json 2>> $OUT/e2e.err || exit 5
echo "e2e no-SDMA: $(cat $OUT/e2e_nosdma.json)"
