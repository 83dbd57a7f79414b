#!/bin/bash
# A/B library variants at several env counts (per-kernel HIP-event times): bash scripts/ab_libs_envs.sh "<E list>" <lib.so>...
set -o pipefail
ES=$1; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ab_envs
mkdir -p $OUT
cd $R
for round in 1 2; do
  for e in $ES; do
    for L in "$@"; do
      n=$(basename $L .so)
      timeout -k 10 200 env PPO_HIP_LIB=$R/$L python bench.py --num-envs $e --steps 5 --warmup 1 --profile-all --no-cpu-baseline > $OUT/${n}_${e}_$round.log 2>&1 || { echo "$n failed"; tail -5 $OUT/${n}_${e}_$round.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/${n}_${e}_$round.log').read().strip().splitlines()[-1]); k=d['kernels_ms_per_step']; print('$n', $e, $round, d['ms_per_step'], 'act', k['act'], 'upd', k['fwdbwd'])"
    done
  done
done
