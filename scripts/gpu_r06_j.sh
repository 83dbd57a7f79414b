#!/bin/bash
# Hand-off store coalescing probe (stamps build, timing only): row-major 64 B segments (sched 1) vs
# 16 x 64 blocks written 1 KB per store instruction (bit 14) vs no stores (bits 4-7).
set -o pipefail
TAG=${1:-r06j}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in 1 2; do
for V in 1 16385 241; do
  PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so PPO_UPD_SCHED=$V timeout -k 10 120 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/sched_${V}_$rep.log 2>&1 || { echo "sched $V failed"; tail -5 $OUT/sched_${V}_$rep.log; exit 1; }
  echo "sched=$V $(tail -1 $OUT/sched_${V}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "fwdbwd/launch", round(k["fwdbwd"]/16,4), "dw", k["dw"])')"
done
done
