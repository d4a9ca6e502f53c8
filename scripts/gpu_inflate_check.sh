# lane-kernel change check: inflate parity suites, then an interleaved C2 A/B against the previous library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_inflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py tests/test_gpu_frame.py tests/test_gpu_tables.py -x -q --timeout 200 --timeout-method thread > gpurun_out/inflate_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/inflate_pytest.log; [ $rc -eq 0 ] || exit 1
ROUNDS=${ROUNDS:-3} bash scripts/ab_inflate.sh
