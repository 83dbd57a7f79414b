#!/bin/bash
# k_upd experiments on the GPU box: stamps-build phase breakdown under env variants
#   bash scripts/upd_variants.sh TAG "ENV=val ..." ...    ("-" = no extra env)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-dev}; shift
OUT=$R/gpurun_out/var_$TAG
mkdir -p $OUT
i=0
for V in "$@"; do
  i=$((i+1))
  [ "$V" = "-" ] && V="PPO_NOTHING=1"
  timeout -k 10 240 env $V python3 -u $R/scripts/diag_stamps.py $OUT/raw_v$i.npy > $OUT/stamps_v$i.txt 2>&1 || { tail -5 $OUT/stamps_v$i.txt; exit 1; }
  echo "== [$V]"; grep -v "amdgpu.ids" $OUT/stamps_v$i.txt
done
