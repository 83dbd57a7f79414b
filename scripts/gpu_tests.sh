#!/bin/bash
# Run named -m gpu test files (or the whole suite) on the box, then optionally one default bench line.
#   bash scripts/gpu_tests.sh <tag> "<test files or tests/>" [bench]
set -o pipefail
TAG=$1; TESTS=$2; BENCH=${3:-}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -3 $OUT/tests.txt
if [ "$BENCH" = bench ]; then
  timeout -k 10 400 python bench.py --no-cli > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log | cut -c1-1500
fi
