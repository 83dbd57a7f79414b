#!/bin/bash
# Round-5 evidence on one GPU box: the whole -m gpu suite + smoke (gpu_r03.sh), the default bench
# line (with the CPU baseline and the CLI SPS), the rocprofv3 kernel trace + the two PMC passes of
# the bench command (gpu_profile.sh), the other BASELINE configs, the CaRL benchmark and the N = 8
# shard (E = 512).   bash scripts/gpu_final_r04.sh <tag>
set -o pipefail
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
bash $R/scripts/gpu_r03.sh $TAG || exit 1
cd $R
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-800
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli > $OUT/bench_all.log 2>&1 || { echo "bench profile-all failed"; exit 1; }
bash $R/scripts/gpu_profile.sh $TAG > $OUT/profile.txt 2>&1 || { echo "profile failed"; tail -5 $OUT/profile.txt; exit 1; }
cd $R
timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; exit 1; }
timeout -k 10 300 python scripts/bench_carla.py > $OUT/carla.jsonl 2>&1 || { echo "carla failed"; exit 1; }
timeout -k 10 120 python bench.py --num-envs 512 --steps 30 --warmup 3 --no-cpu-baseline --no-cli > $OUT/bench_e512.log 2>&1 || { echo "e512 failed"; exit 1; }
timeout -k 10 120 python bench.py --num-envs 1024 --steps 30 --warmup 3 --no-cpu-baseline --no-cli > $OUT/bench_e1024.log 2>&1 || { echo "e1024 failed"; exit 1; }
# kernel traces of the N = 8 / N = 4 shards (E = 512 / 1 024) for the strong-scaling projection
export TMPDIR=/tmp
for E in 512 1024; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/scale_e$E -o kt -- \
    python3 $R/bench.py --num-envs $E --steps 10 --warmup 2 --no-cpu-baseline --no-cli > $OUT/scale_e$E.log 2>&1) || { echo "trace E=$E failed"; exit 1; }
done
cut -c1-300 $OUT/configs.jsonl; tail -1 $OUT/bench_e512.log | cut -c1-300
echo final-done
