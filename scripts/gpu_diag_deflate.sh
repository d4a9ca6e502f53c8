# deflate per-phase counters (prof builds): C3 shape at the default cap and at cap 16
set -o pipefail
mkdir -p gpurun_out/ddiag
for v in prof profc16; do
  echo "== $v"
  BPMD_LIB=beast_amd/libbeast_pmd_$v.so DIAG_MSGS=65536 timeout -k 10 120 python -u scripts/diag_deflate.py || exit 1
done
