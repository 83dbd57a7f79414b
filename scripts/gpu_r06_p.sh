#!/bin/bash
# k_upd head-weight gradient sums as explicit LDS / global accesses (no flat RMWs) vs HEAD's kernel:
# metric A/B, cfg4 shard (Ant, wide input) A/B, then the update tests on the new default library.
set -o pipefail
TAG=${1:-r06p}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ARMS="base:ppo.cpp_amd/lib/libppo_hip_base.so:- new:-:-" BENCH_ARGS="--no-fp32-leg" bash scripts/gpu_ab_multi.sh $TAG 3 || exit 1
grep -o '"kernels": "[^"]*"' $OUT/bench_new_1.log
for arm in base new; do
  if [ $arm = base ]; then export PPO_HIP_LIB=$R/ppo.cpp_amd/lib/libppo_hip_base.so; else unset PPO_HIP_LIB; fi
  timeout -k 10 200 python scripts/bench_configs.py --only cfg4_shard --iters 4 --warmup 2 > $OUT/cfg4_$arm.jsonl 2>&1 || { echo "cfg4 $arm failed"; tail -5 $OUT/cfg4_$arm.jsonl; exit 1; }
  echo "$arm $(grep config $OUT/cfg4_$arm.jsonl | cut -c1-260)"
done
unset PPO_HIP_LIB
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py tests/test_gpu_e2e_teacher.py tests/test_gpu_parity.py tests/test_gpu_e2e.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
