#!/bin/bash
# Quick GPU check after a rollout / update kernel change: the named -m gpu test files, the rollout
# phase stamps and one config bench.   bash scripts/gpu_quick.sh <tag> "<test files>" [cfg2|cfg4_shard|cfg1|all]
set -o pipefail
TAG=$1; TESTS=$2; CFG=${3:-cfg2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 120 python3 scripts/roll_stamps.py > $OUT/roll_stamps.txt 2>&1 || { echo "roll stamps failed"; tail -20 $OUT/roll_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/roll_stamps.txt
ONLY="--only $CFG"; [ "$CFG" = all ] && ONLY=""
timeout -k 10 300 python3 scripts/bench_configs.py $ONLY > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; tail -20 $OUT/configs.jsonl; exit 1; }
cut -c1-600 $OUT/configs.jsonl
