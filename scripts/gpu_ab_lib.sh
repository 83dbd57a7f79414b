#!/bin/bash
# A/B of two builds of libppo_hip.so on one box: the default bench line and cfg2, alternating.
#   ALT=ppo.cpp_amd/lib/libppo_hip_<x>.so bash scripts/gpu_ab_lib.sh <tag>
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for L in base alt; do
    if [ $L = alt ]; then export PPO_HIP_LIB=$R/$ALT; else unset PPO_HIP_LIB; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cli ${BENCH_ARGS} > $OUT/bench_${L}_$rep.log 2>&1 || { echo "bench $L failed"; tail -5 $OUT/bench_${L}_$rep.log; exit 1; }
    echo "$L rep$rep $(tail -1 $OUT/bench_${L}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
  done
done
