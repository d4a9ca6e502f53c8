# Lane-kernel bring-up: inflate parity on both kernels, then the C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_inflate.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lane_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/lane_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/lane_bench.json 2> gpurun_out/lane_bench.err || exit 3
