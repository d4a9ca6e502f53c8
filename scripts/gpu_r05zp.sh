#!/bin/bash
# pass 2 skips only near a marker: BP parity incl. the one-early-flush foreign payload, C4/C5 shards
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zp}
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate_bp.py tests/test_gpu_inflate.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_bp.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_bp.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_bp.log
bash scripts/run_bench.sh ${TAG}_bench 900 \
  "{k: (v['inflate_value'], v['inflate_beast_value'], {n: (max(y['inflate_shard_ms']), y['inflate_projected_speedup'], max(y['inflate_beast_shard_ms'])) for n, y in v['virtual_shards'].items()}) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate || exit 2
