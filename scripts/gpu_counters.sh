#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc pass each) over a short bench run, for the kernel
# utilisation breakdown in DESIGN.md.   bash scripts/gpu_counters.sh <tag> "<counters pass 1>" ["<pass 2>" ...]
# CTR_CMD overrides the profiled command (default: the metric-config bench), e.g.
#   CTR_CMD="scripts/bench_configs.py --only cfg2 --iters 1 --warmup 1" (a python script + args)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ctr_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT -o p$i -- \
    python3 $R/${CTR_CMD:-bench.py --steps 1 --warmup 1 --no-cpu-baseline} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
cd $R && python3 scripts/ctr_summary.py $OUT
