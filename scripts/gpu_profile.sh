#!/bin/bash
# GPU-box profiling pass for one round: kernel-trace stats of the bench command, then two PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), then the per-kernel HBM
# traffic summary profiles/pmc_traffic.json that bench.py reports as roofline.traffic.
#   bash scripts/gpu_profile.sh r01
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_kt.log 2>&1 || { echo "kernel-trace pass failed"; tail -20 $OUT/bench_kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; tail -20 $OUT/bench_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_write.log 2>&1 || { echo "WRITE_SIZE pass failed"; tail -20 $OUT/bench_write.log; exit 1; }
cd $R
find $OUT -name "*.csv" | sort
python3 scripts/pmc_traffic.py $OUT "E=4096,T=128" > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
