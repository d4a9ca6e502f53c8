# Iteration loop for the lane kernel: parity (inflate tests), diag counters, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/it_pytest.log; tail -3 gpurun_out/it_pytest.log
[ $rc -eq 0 ] || exit 1
BPMD_LIB=beast_amd/libbeast_pmd_prof.so timeout -k 10 120 python scripts/diag_lane.py || exit 2
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/it_bench.json 2> gpurun_out/it_bench.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/it_bench.json')); x=d.get('deflate',{}); print('C2 inflate', d['value'], 'GiB/s', d['roofline']['kernel_ms'], 'ms parity', d['parity_ok'], '| deflate', x.get('deflate_value'), 'rt', x.get('roundtrip_ok'), 'reinflate', x.get('inflate_of_gpu_payloads_value'))"
