#!/bin/bash
# round 5: mixed legs with Beast-produced payloads (bench key mixed.*.inflate_beast_*)
set -o pipefail
TAG=${TAG:-r05c}
bash scripts/run_bench.sh ${TAG}_mixed 900 "[(k, v.get('inflate_value'), v.get('inflate_beast_value'), v.get('inflate_beast_ok')) for k, v in d['mixed'].items() if isinstance(v, dict)]" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-deflate --no-frame || exit 1
python - <<'PY'
import json
d = json.load(open('gpurun_out/r05c_mixed.json'))
for k, v in d['mixed'].items():
    if not isinstance(v, dict): continue
    print(k, 'gpu-payload inflate', v['inflate_value'], 'beast-payload inflate', v.get('inflate_beast_value'), v.get('beast_payloads'))
    for p, s in v.get('virtual_shards', {}).items():
        print('  ', p, 'own', s['inflate_projected_speedup'], max(s['inflate_shard_ms']), 'beast', s.get('inflate_beast_projected_speedup'), max(s.get('inflate_beast_shard_ms', [0])))
PY
