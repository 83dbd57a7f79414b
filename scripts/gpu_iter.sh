#!/bin/bash
# Development loop on the GPU box: parity tests, then per-kernel bench lines (optionally with
# extra env settings to compare kernel variants).   bash scripts/gpu_iter.sh [tag] ["ENV=val ..."]...
set -o pipefail
TAG=${1:-dev}; shift
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/iter_$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" $OUT/pytest.log | head -30; exit 1; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --profile-all --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
i=0
for V in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $V python bench.py --steps 5 --warmup 1 --profile-all --no-cpu-baseline > $OUT/bench_v$i.log 2>&1 || { tail -20 $OUT/bench_v$i.log; exit 1; }
  echo "[$V]"; tail -1 $OUT/bench_v$i.log
done
