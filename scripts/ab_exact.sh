#!/bin/bash
# exact-mode C4-shaped rate per library variant (and the host's 32-thread zlib on the same sample)
cd $GRAFT_REPO_ROOT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  BPMD_LIB=$PWD/$L EXACT_C3=0 timeout -k 10 300 python -u scripts/exact_rate.py > gpurun_out/abx_$v.log 2>&1 || { tail -5 gpurun_out/abx_$v.log; exit 1; }
  echo "== $v"; grep "C4-64Ki" gpurun_out/abx_$v.log
done
