#!/bin/bash
# Is cfg2's k_upd2 layer 1 waiting on its observation gather? Diagnostic build: PPO_UPD2_HOT=1 makes
# every tile gather the rows of the first 8 tiles (L2-resident) instead of random HBM rows.
#   bash scripts/gpu_upd2_hot.sh <tag>
set -o pipefail
TAG=${1:-upd2hot}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so
for HOT in 0 1; do
  PPO_UPD2_HOT=$HOT timeout -k 10 300 python scripts/bench_configs.py --only cfg2 --iters 2 --warmup 1 > $OUT/cfg2_hot$HOT.jsonl 2>&1 || { echo "hot=$HOT failed"; tail -5 $OUT/cfg2_hot$HOT.jsonl; exit 1; }
  echo "hot=$HOT $(tail -1 $OUT/cfg2_hot$HOT.jsonl | cut -c1-400)"
done
