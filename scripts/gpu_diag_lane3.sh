set -o pipefail
mkdir -p gpurun_out/diag1
timeout -k 10 200 python -u scripts/diag_lane3.py > gpurun_out/diag1/diag.txt 2>&1 || exit 1
BENCH_ARGS="--no-mixed --no-deflate --no-frame" TAG=diag1 timeout -k 10 500 bash scripts/pmc_sq.sh > gpurun_out/diag1/sq.log 2>&1 || exit 2
python scripts/sq_summary.py gpurun_out/sq_diag1 > gpurun_out/diag1/sq_summary.txt 2>&1
cat gpurun_out/diag1/diag.txt gpurun_out/diag1/sq_summary.txt
