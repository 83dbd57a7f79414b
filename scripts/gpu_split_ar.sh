#!/bin/bash
# Cost of the split (per-trunk) gradient all-reduce on one GPU: bench.py with and without a one-rank
# RCCL communicator at E = 4 096 / 1 024 / 512, and a kernel trace of the E = 512 communicator run
# (the critic's all-reduce kernel under the actor's dW launch).   bash scripts/gpu_split_ar.sh <tag>
set -o pipefail
TAG=${1:-split}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/comm_tests.log 2>&1 || { echo "comm tests failed"; tail -30 $OUT/comm_tests.log; exit 1; }
tail -2 $OUT/comm_tests.log
for E in 4096 1024 512; do
  for C in "" "--comm-1rank"; do
    timeout -k 10 200 python bench.py --num-envs $E --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli $C > $OUT/bench_e${E}${C}.log 2>&1 || { echo "bench E=$E $C failed"; tail -20 $OUT/bench_e${E}${C}.log; exit 1; }
    echo "E=$E $C: $(tail -1 $OUT/bench_e${E}${C}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("kernels_ms_per_step"))')"
  done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_e512_comm -o kt -- \
  python3 $R/bench.py --num-envs 512 --steps 5 --warmup 2 --no-cpu-baseline --no-cli --comm-1rank > $OUT/trace_e512_comm.log 2>&1) || { echo "trace failed"; exit 1; }
echo split-done
