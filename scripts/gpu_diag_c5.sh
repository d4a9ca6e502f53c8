# wave-kernel phase counters on the C5 shape (64 KiB binary), prof build
set -o pipefail
mkdir -p gpurun_out/c5diag
BPMD_LIB=beast_amd/libbeast_pmd_prof.so DIAG_KIND=binary DIAG_SIZE=65536 DIAG_MSGS=16384 timeout -k 10 300 python -u scripts/diag_inflate.py
