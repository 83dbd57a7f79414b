#!/bin/bash
# Copy a gpu_final_r06.sh (+ gpu_final_r06b.sh) run into profiles/r06/<tag>.   bash scripts/collect_final_r06.sh <tag> [a|b]
set -e
T=$1; PART=${2:-a}; S=gpurun_out/$T; P=gpurun_out/prof_$T; D=profiles/r06/$T
mkdir -p $D/scale
if [ "$PART" = a ]; then
  tail -1 $S/bench_default.log > $D/bench_default.json
  tail -1 $S/bench_all.log > $D/bench_all.json
  grep -E "PASSED|FAILED|passed|failed" $S/gpu_all.log > $D/gpu_tests.txt
  cp $S/smoke.log $D/smoke.log
  cp $P/kt_kernel_stats.csv $D/kernel_stats.csv
  cp $P/pmc_traffic.json $D/pmc_traffic.json
  grep -vE "^\[|^$" $S/sq.txt > $D/sq_counters.txt || true
  grep -vE "^\[|^$" $S/l2.txt > $D/l2_counters.txt || true
  cp $D/pmc_traffic.json profiles/pmc_traffic.json
else
  grep config $S/configs.jsonl > $D/configs.jsonl
  grep workload $S/carla.jsonl > $D/carla.jsonl
  for E in 512 1024; do
    tail -1 $S/bench_e$E.log > $D/scale/bench_e$E.json
    tail -1 $S/bench_all_e$E.log > $D/scale/bench_all_e$E.json
    cp $(find $S/scale_e$E -name "*kernel_stats.csv" | head -1) $D/scale/kernel_stats_e$E.csv
  done
fi
ls -la $D
