#!/bin/bash
# k_upd phase stamps (diagnostic stamps build) of the metric config and of the cfg4 shard (Ant).
#   bash scripts/gpu_upd_stamps.sh <tag>
set -o pipefail
TAG=${1:-upd_stamps}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 180 python3 scripts/diag_stamps.py --ant > $OUT/kupd_phases_ant.txt 2>&1 || { echo "ant stamps failed"; tail -20 $OUT/kupd_phases_ant.txt; exit 1; }
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "hc stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_ant.txt $OUT/kupd_phases_hc.txt
# CaRL forward at the cfg5 per-GPU rollout batch (32): per-kernel trace
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/carla_kt -o kt -- \
  python3 $R/scripts/bench_carla.py --batch 32 --update-batch --iters 50 > $OUT/carla_kt.log 2>&1 || { echo "carla trace failed"; tail -20 $OUT/carla_kt.log; exit 1; }
grep -v amdgpu.ids $OUT/carla_kt.log
find $OUT/carla_kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-4 {} | head -30
