#!/bin/bash
# segment-expander A/B: one 8-way shard of C4 and of C5 (inflate), per library variant
cd $GRAFT_REPO_ROOT
for v in default $VARIANTS; do
  if [ "$v" = default ]; then L=beast_amd/libbeast_pmd.so; else L=beast_amd/libbeast_pmd_$v.so; fi
  echo "== $v"
  BPMD_LIB=$PWD/$L timeout -k 10 300 python -u scripts/diag_shards.py --child c4:s8,c5:s8 2>&1 | grep -v amdgpu.ids || exit 1
done
