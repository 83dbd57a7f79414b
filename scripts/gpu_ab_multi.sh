#!/bin/bash
# A/B of several (library, create options) arms on one box, the default bench line, alternating.
#   ARMS="label:lib_or_-:options ..." bash scripts/gpu_ab_multi.sh <tag> [reps]
#   lib "-" = the in-tree default library; options "-" = none
set -o pipefail
TAG=${1:-abm}
REPS=${2:-2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for rep in $(seq 1 $REPS); do
  for arm in $ARMS; do
    IFS=: read -r label lib opts <<< "$arm"
    if [ "$lib" = "-" ]; then unset PPO_HIP_LIB; else export PPO_HIP_LIB=$R/$lib; fi
    extra=""
    [ "$opts" != "-" ] && extra="--options $opts"
    timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-cli $extra ${BENCH_ARGS} > $OUT/bench_${label}_$rep.log 2>&1 || { echo "bench $label failed"; tail -5 $OUT/bench_${label}_$rep.log; exit 1; }
    echo "$label rep$rep $(tail -1 $OUT/bench_${label}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
  done
done
