#!/bin/bash
# Is the fused dW bandwidth-bound? Diagnostic build (PPO_DIAG): PPO_DW_HOT=1 makes every stage of
# k_dwf_dma / k_dwf_bx re-read its chunk's first 16 rows (L2-hot) instead of streaming the hand-off.
#   bash scripts/gpu_dw_hot.sh <tag>
set -o pipefail
TAG=${1:-dwhot}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so
for D in f32 bf16x9; do
  for HOT in 0 1; do
    PPO_DW_HOT=$HOT timeout -k 10 120 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --options dw_mfma=$D > $OUT/${D}_hot$HOT.log 2>&1 || { echo "$D hot=$HOT failed"; tail -5 $OUT/${D}_hot$HOT.log; exit 1; }
    echo "$D hot=$HOT $(tail -1 $OUT/${D}_hot$HOT.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernels_ms_per_step"])')"
  done
done
