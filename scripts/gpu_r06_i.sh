#!/bin/bash
# Which hand-off store costs k_upd what (stamps build: a.sched bit 4 H1, 5 DZ2, 6 DZ1, 7 Xn skipped;
# timing only), then plain vs non-temporal hand-off stores (default build, A/B).
set -o pipefail
TAG=${1:-r06i}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for V in 1 17 33 65 129 241; do
  PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_stamps.so PPO_UPD_SCHED=$V timeout -k 10 120 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/sched_$V.log 2>&1 || { echo "sched $V failed"; tail -5 $OUT/sched_$V.log; exit 1; }
  echo "sched=$V $(tail -1 $OUT/sched_$V.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "fwdbwd/launch", round(k["fwdbwd"]/16,4), "dw", k["dw"])')"
done
ARMS="base:-:- nt:ppo.cpp_amd/lib/libppo_hip_nt.so:-" BENCH_ARGS="--no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh $TAG 2
