#!/bin/bash
# Kernel-trace passes of bench.py at E = 512 and E = 4096, then the gaps between consecutive
# kernels (scripts/kernel_gaps.py).   bash scripts/gpu_gaps.sh <tag>
set -o pipefail
TAG=${1:-gaps}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for E in 512 4096; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/e$E -o kt -- \
    python3 $R/bench.py --steps 4 --warmup 1 --num-envs $E --no-cpu-baseline --no-cli > $OUT/bench_e$E.log 2>&1 \
    || { echo "trace pass E=$E failed"; tail -20 $OUT/bench_e$E.log; exit 1; }
  python3 $R/scripts/kernel_gaps.py $OUT/e$E > $OUT/gaps_e$E.txt || exit 1
done
cd $R
