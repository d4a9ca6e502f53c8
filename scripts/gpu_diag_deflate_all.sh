set -o pipefail
BPMD_LIB=beast_amd/libbeast_pmd_prof.so DIAG_KIND=json DIAG_LEVEL=6 DIAG_SIZE=4096 DIAG_MSGS=65536 timeout -k 10 120 python -u scripts/diag_deflate.py || exit 1
bash scripts/gpu_diag_deflate_big.sh
