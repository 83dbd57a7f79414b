#!/bin/bash
# End-of-session evidence on one GPU box: parity suite + smoke + benches (gpu_check.sh), the
# rocprofv3 kernel trace + PMC traffic (gpu_profile.sh), the other BASELINE configs, the CaRL
# benchmark and the N = 8 shard.   bash scripts/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
bash $R/scripts/gpu_check.sh $TAG || exit 1
bash $R/scripts/gpu_profile.sh $TAG > $R/gpurun_out/profile_$TAG.txt 2>&1 || { echo "profile failed"; tail -5 $R/gpurun_out/profile_$TAG.txt; exit 1; }
cd $R
timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; exit 1; }
timeout -k 10 300 python scripts/bench_carla.py > $OUT/carla.jsonl 2>&1 || { echo "carla failed"; exit 1; }
timeout -k 10 120 python bench.py --num-envs 512 --steps 20 --warmup 3 --no-cpu-baseline --no-cli > $OUT/bench_e512.log 2>&1 || { echo "e512 failed"; exit 1; }
grep -h workload $OUT/carla.jsonl; grep -h '"config"' $OUT/configs.jsonl | cut -c1-160; tail -1 $OUT/bench_e512.log | cut -c1-200
echo final-done
