#!/bin/bash
# marker before a stored chunk 1: deflate + inflate parity, C5 shards
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zo}
timeout -k 10 900 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_stream.py tests/test_gpu_inflate_bp.py tests/test_gpu_reference_pins.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
bash scripts/run_bench.sh ${TAG}_bench 900 \
  "{k: (v['deflate_value'], v['ratio_rank_local'], v['inflate_value'], {n: (max(y['inflate_shard_ms']), y['inflate_projected_speedup']) for n, y in v['virtual_shards'].items()}) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
  --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-beast-payloads || exit 2
