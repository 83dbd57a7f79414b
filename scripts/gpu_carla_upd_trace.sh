#!/bin/bash
# Per-launch durations of one 2 048-row CaRL update (kernel trace).   bash scripts/gpu_carla_upd_trace.sh <tag>
set -o pipefail
TAG=${1:-carlaupd}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
  python3 $R/scripts/bench_carla.py --batch --update-batch 2048 --iters 3 > $OUT/kt.log 2>&1) || { echo "trace failed"; tail -20 $OUT/kt.log; exit 1; }
cd $R
python3 scripts/carla_trace.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) > $OUT/update_launches.txt
cut -d, -f1-4 $(find $OUT/kt -name "*kernel_stats.csv" | head -1) | head -25
tail -3 $OUT/update_launches.txt
