#!/bin/bash
# A/B one environment variable on one GPU box: interleaved bench.py runs, one line per run with
# ms per iteration and the dominant kernel's HIP-event launch average.
#   bash scripts/ab_env.sh VAR "v1 v2 ..." [rounds] [extra bench args]
set -o pipefail
VAR=$1
VALS=$2
ROUNDS=${3:-2}
EXTRA=${4:-}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_$VAR
mkdir -p $OUT
cd $R
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    timeout -k 10 120 env $VAR=$v python bench.py --steps 10 --warmup 2 --no-cpu-baseline $EXTRA > $OUT/r${r}_$v.log 2>&1 || { echo "run $VAR=$v failed"; tail -20 $OUT/r${r}_$v.log; exit 1; }
    tail -1 $OUT/r${r}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"
  done
done
