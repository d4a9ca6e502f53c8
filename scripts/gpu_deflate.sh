#!/bin/bash
# deflate parity (incl. the host-model byte equality and context takeover),
# then the C3 / C4 / C5 deflate legs, chunk-parallel vs serial chunk walk
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py tests/test_gpu_stream.py tests/test_gpu_batcher.py tests/test_facade.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/deflate_pytest.log 2>&1
rc=$?; tail -5 gpurun_out/deflate_pytest.log; [ $rc -eq 0 ] || exit 1
for ser in 0 1; do
  BPMD_DEFLATE_SERIAL=$ser timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-frame 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('serial=$ser', 'C3', d['deflate']['deflate_value'], d['deflate']['roundtrip_ok'], {k:(v['deflate_value'], v['inflate_value'], v['ratio_rank_local'], v['roundtrip_ok']) for k,v in d['mixed'].items() if isinstance(v,dict)})" || exit 2
done
