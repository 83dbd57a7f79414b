#!/bin/bash
# A/B timing of library variants on one box: bash scripts/ab_libs.sh <tag> <lib.so>...  (2 rounds, alternating)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
for round in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    timeout -k 10 200 env PPO_HIP_LIB=$R/$L python bench.py --steps 5 --warmup 1 --profile-all --no-cpu-baseline > $OUT/${n}_$round.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_$round.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$OUT/${n}_$round.log').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$n', $round, d['ms_per_step'], k['fwdbwd'], k.get('rollout'), k.get('values'), k['dw'])"
  done
done
