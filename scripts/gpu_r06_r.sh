#!/bin/bash
# dW split-K geometry at the shard sizes: fewer, longer chunks (dw_rows) and output slices (dw_slices)
# write fewer partial rows for k_colsum to read back.   bash scripts/gpu_r06_r.sh <tag>
set -o pipefail
TAG=${1:-r06r}
R=$GRAFT_REPO_ROOT
cd $R
for E in 512 1024; do
  ARMS="def:-:- r256:-:dw_rows=256 r512:-:dw_rows=512 s2:-:dw_slices=2 s2r256:-:dw_slices=2,dw_rows=256" \
    BENCH_ARGS="--num-envs $E --no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh ${TAG}_e$E 2 || exit 1
done
ARMS="def:-:- s2:-:dw_slices=2 r2048:-:dw_rows=2048" BENCH_ARGS="--no-fp32-leg --profile-all" bash scripts/gpu_ab_multi.sh ${TAG}_e4096 2 || exit 1
for f in gpurun_out/${TAG}_e*/bench_*_1.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); k=d["kernels_ms_per_step"]; print(d["ms_per_step"], "dw", k["dw"], "colsum", k["colsum"], "fwdbwd", k["fwdbwd"])')"; done
