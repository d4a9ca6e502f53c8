# deflate per-phase counters (prof build) on the chunk-parallel path: 64 KiB JSON (C4's bulk) and binary (C5)
set -o pipefail
for k in "json 6" "binary 1" "binary 6"; do
  set -- $k
  echo "== $1 L$2"
  BPMD_LIB=beast_amd/libbeast_pmd_prof.so DIAG_KIND=$1 DIAG_LEVEL=$2 DIAG_SIZE=65536 DIAG_MSGS=4096 timeout -k 10 120 python -u scripts/diag_deflate.py || exit 1
done
