#!/bin/bash
# cfg2 (PPO Humanoid-v4 shape, E=1024, T=2048) on the GPU box: kernel-trace stats and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE: separate passes on gfx950), then the per-launch traffic summary.
#   bash scripts/gpu_profile_cfg2.sh r02
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_cfg2_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- \
  python3 $R/scripts/bench_configs.py --only cfg2 --iters 1 --warmup 1 > $OUT/kt.log 2>&1 || { echo "kernel-trace pass failed"; tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT -o fetch -- \
  python3 $R/scripts/bench_configs.py --only cfg2 --iters 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "FETCH_SIZE pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT -o write -- \
  python3 $R/scripts/bench_configs.py --only cfg2 --iters 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "WRITE_SIZE pass failed"; tail -20 $OUT/write.log; exit 1; }
cd $R
python3 scripts/pmc_traffic.py $OUT "cfg2 E=1024,T=2048" > $OUT/pmc_traffic.json && cat $OUT/pmc_traffic.json
