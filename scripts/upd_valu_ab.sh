#!/bin/bash
# k_upd timing with the column sums skipped (diagnostic stamps build, PPO_UPD_SCHED bit 12; wrong
# gradients, timing only): how much of the tile time the VALU reductions cost.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-valu_ab}
mkdir -p $OUT
cd $R
for sched in 1 4097 1 4097; do
  PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so PPO_UPD_SCHED=$sched timeout -k 10 200 python bench.py --steps 5 --warmup 1 --profile-all --no-cpu-baseline --no-cli > $OUT/sched_$sched.log 2>&1 || { echo "failed $sched"; tail -5 $OUT/sched_$sched.log; exit 1; }
  python - $OUT/sched_$sched.log $sched <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
k = d["kernels_ms_per_step"]
print("sched", sys.argv[2], "ms/step", d["ms_per_step"], "fwdbwd/step", k.get("fwdbwd"), "dw", k.get("dw"))
PY
done
