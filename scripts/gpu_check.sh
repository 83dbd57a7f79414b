#!/bin/bash
# GPU-box check: parity tests, default bench line (with CPU baseline), rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r01
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log; exit 1; }
echo done
