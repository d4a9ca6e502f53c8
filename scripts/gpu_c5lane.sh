# C5 (16 Ki x 64 KiB) inflate: automatic kernel choice vs the lane kernel forced
set -o pipefail
mkdir -p gpurun_out/c5lane
for m in auto lane; do
  if [ $m = lane ]; then export BPMD_INFLATE=lane; fi
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact --no-deflate > gpurun_out/c5lane/bench_$m.json 2> gpurun_out/c5lane/bench_$m.err || exit 2
  python -c "import json; d=json.load(open('gpurun_out/c5lane/bench_$m.json')); m=d['mixed']; print('$m C2', d['value'], {k: (v['deflate_value'], v['inflate_value'], v['roundtrip_ok']) for k, v in m.items() if isinstance(v, dict)})"
done
