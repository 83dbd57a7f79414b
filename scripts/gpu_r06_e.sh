#!/bin/bash
# Round 6: is k_dwf_bx (bf16x6) bandwidth-visible? PPO_DW_HOT A/B on the diagnostic build, then the
# k_upd phase stamps of the current default (stamps build).   bash scripts/gpu_r06_e.sh <tag>
set -o pipefail
TAG=${1:-r06e}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so
for rep in 1 2; do
  for HOT in 0 1; do
    PPO_DW_HOT=$HOT timeout -k 10 120 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bx6_hot${HOT}_$rep.log 2>&1 || { echo "hot=$HOT failed"; tail -5 $OUT/bx6_hot${HOT}_$rep.log; exit 1; }
    echo "bf16x6 hot=$HOT rep$rep $(tail -1 $OUT/bx6_hot${HOT}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "dw", k["dw"], "fwdbwd", k["fwdbwd"])')"
  done
done
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "hc stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_hc.txt
