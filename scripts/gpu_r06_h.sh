#!/bin/bash
# k_upd bound probe (diagnostic stamps build, timing only): a.sched bit 13 = weight units from L1
# (every unit read from the wave's first), bit 12 = no column sums, bits 4-7 = no H1/DZ/Xn stores.
set -o pipefail
TAG=${1:-r06h}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so
for rep in 1 2; do
  for V in 1 8193 4097 241 12529; do
    PPO_UPD_SCHED=$V timeout -k 10 120 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/sched_${V}_$rep.log 2>&1 || { echo "sched $V failed"; tail -5 $OUT/sched_${V}_$rep.log; exit 1; }
    echo "sched=$V rep$rep $(tail -1 $OUT/sched_${V}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "fwdbwd/launch", round(k["fwdbwd"]/16,4))')"
  done
done
PPO_UPD_SCHED=8193 timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_unit0.txt 2>&1 || { echo "stamps failed"; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_unit0.txt
