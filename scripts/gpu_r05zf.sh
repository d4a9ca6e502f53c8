#!/bin/bash
# lane decoder: arithmetic fixed-Huffman decode -- parity, then C2 and C4/C5 inflate incl. Beast payloads (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r05zf}
timeout -k 10 900 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_inflate_bp.py tests/test_gpu_configs.py tests/test_gpu_reference_pins.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_inflate.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_inflate.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_inflate.log
for round in 1 2; do
for v in default fx0; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$L bash scripts/run_bench.sh ${TAG}_${v}_$round 600 \
    "d['value'], {k: (v['inflate_value'], v['inflate_beast_value'], v['inflate_beast_ok']) for k, v in d['mixed'].items() if isinstance(v, dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate --no-virtual-shards || exit 2
done
done
