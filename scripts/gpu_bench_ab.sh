#!/bin/bash
# Metric-config and E = 512 bench lines, twice each, for run-to-run comparison on one box.
#   bash scripts/gpu_bench_ab.sh <tag>
set -o pipefail
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for i in 1 2; do
  for E in 4096 512; do
    timeout -k 10 200 python bench.py --num-envs $E --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli > $OUT/b_${E}_$i.log 2>&1 || { echo "bench E=$E failed"; tail -20 $OUT/b_${E}_$i.log; exit 1; }
    tail -1 $OUT/b_${E}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('E', $E, d['ms_per_step'], d['roofline']['frac'], d['kernels_ms_per_step'])"
  done
done
