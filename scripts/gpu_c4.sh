#!/bin/bash
# C4/C5 legs: queue parity test, then the mixed legs at 1 Mi and 128 Ki messages
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c4_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/c4_pytest.log; [ $rc -eq 0 ] || exit 1
for c4 in 1048576 131072; do
  bash scripts/run_bench.sh c4_$c4 300 "'C2', d['value'], {k:(v['msgs'], v['deflate_value'], v['inflate_value'], v['roundtrip_ok']) for k,v in d['mixed'].items() if isinstance(v,dict)}" \
    --steps 3 --warmup 1 --no-cpu-baseline --no-deflate --no-frame --c4-msgs $c4 --c5-msgs 16384 || exit 2
done
