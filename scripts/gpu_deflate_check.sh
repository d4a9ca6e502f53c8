# deflate change check: deflate parity suites (byte-exact vs the host model), then phase counters
set -o pipefail
mkdir -p gpurun_out/dcheck
timeout -k 10 400 python -u -m pytest tests/test_gpu_deflate.py tests/test_gpu_configs.py tests/test_gpu_takeover.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dcheck/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/dcheck/pytest.log; [ $rc -eq 0 ] || exit 1
for k in "json 6 4096 65536" "json 6 65536 4096" "binary 1 65536 4096"; do
  set -- $k
  echo "== $1 L$2 $3 B"
  BPMD_LIB=beast_amd/libbeast_pmd_prof.so DIAG_KIND=$1 DIAG_LEVEL=$2 DIAG_SIZE=$3 DIAG_MSGS=$4 timeout -k 10 120 python -u scripts/diag_deflate.py | grep -v "amdgpu.ids" || exit 2
done
