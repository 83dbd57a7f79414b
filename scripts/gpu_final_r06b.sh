#!/bin/bash
# Round-6 evidence, part B: the other BASELINE configs, CaRL, the N = 8 / N = 4 shards (E = 512 / 1 024:
# bench lines without events, per-kernel-class lines, rocprofv3 kernel traces).
#   bash scripts/gpu_final_r06b.sh <tag>   (same tag as part A)
set -o pipefail
TAG=${1:-final_r06}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; tail -5 $OUT/configs.jsonl; exit 1; }
cut -c1-300 $OUT/configs.jsonl
timeout -k 10 300 python scripts/bench_carla.py > $OUT/carla.jsonl 2>&1 || { echo "carla failed"; tail -5 $OUT/carla.jsonl; exit 1; }
for E in 512 1024; do
  timeout -k 10 120 python bench.py --num-envs $E --steps 30 --warmup 3 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_e$E.log 2>&1 || { echo "e$E failed"; exit 1; }
  timeout -k 10 120 python bench.py --num-envs $E --steps 10 --warmup 3 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_all_e$E.log 2>&1 || { echo "e$E all failed"; exit 1; }
  tail -1 $OUT/bench_e$E.log | cut -c1-200
done
export TMPDIR=/tmp
for E in 512 1024; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/scale_e$E -o kt -- \
    python3 $R/bench.py --num-envs $E --steps 10 --warmup 2 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/scale_e$E.log 2>&1) || { echo "trace E=$E failed"; exit 1; }
done
echo final-b-done
