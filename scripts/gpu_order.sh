# inflate work-queue order A/B on the whole C4/C5 batches (+ the queue parity tests)
set -o pipefail
mkdir -p gpurun_out/order
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/order/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/order/pytest.log; [ $rc -eq 0 ] || exit 1
for o in 0 1; do
  BPMD_INFLATE_ORDER=$o timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-frame --no-exact > gpurun_out/order/bench_$o.json 2> gpurun_out/order/bench_$o.err || exit 2
  python -c "import json; d=json.load(open('gpurun_out/order/bench_$o.json')); m=d['mixed']; print('order=$o C2', d['value'], 'C3', d['deflate']['deflate_value'], {k: (v['deflate_value'], v['inflate_value'], v['roundtrip_ok']) for k, v in m.items() if isinstance(v, dict)})"
done
