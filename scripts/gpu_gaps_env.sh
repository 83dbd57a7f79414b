#!/bin/bash
# Kernel gaps at E = 512 under kernel-selection switches (read once at ppo_create):
#   bash scripts/gpu_gaps_env.sh <tag> "VAR=VAL ..." ...
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for ENVS in "$@"; do
  i=$((i+1))
  for kv in $ENVS; do export "$kv"; done
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/v$i -o kt -- \
    python3 $R/bench.py --steps 3 --warmup 1 --num-envs 512 --no-cpu-baseline --no-cli > $OUT/bench_v$i.log 2>&1 \
    || { echo "trace pass $ENVS failed"; tail -20 $OUT/bench_v$i.log; exit 1; }
  for kv in $ENVS; do unset "${kv%%=*}"; done
  { echo "# $ENVS"; python3 $R/scripts/kernel_gaps.py $OUT/v$i; } > $OUT/gaps_v$i.txt || exit 1
done
