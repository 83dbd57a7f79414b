#!/bin/bash
# cfg4 shard (Ant, two-phase k_dw_dma): its read-once streams non-temporal (libppo_hip_dwd.so) vs default, 3 reps.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06ee
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for rep in 1 2 3 4; do
  for arm in def nt; do
    if [ $arm = nt ]; then export PPO_HIP_LIB=$GRAFT_REPO_ROOT/ppo.cpp_amd/lib/libppo_hip_dwd.so; else unset PPO_HIP_LIB; fi
    timeout -k 10 200 python scripts/bench_configs.py --only cfg4_shard --iters 3 --warmup 2 > $OUT/cfg4_${arm}_$rep.jsonl 2>&1 || { echo "cfg2 $arm failed"; tail -5 $OUT/cfg4_${arm}_$rep.jsonl; exit 1; }
    grep config $OUT/cfg4_${arm}_$rep.jsonl | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_iteration"]; print("'$arm'", "rep'$rep'", d["ms_per_iteration"], "dw", k["dw"], "fwdbwd", k["fwdbwd"], "colsum", k["colsum"])'
  done
done
