#!/bin/bash
# Copy one gpu_final_r0N.sh run (gpurun_out/<tag>, gpurun_out/prof_<tag>) into profiles/<round>/<tag>.
#   ROUND=r04 bash scripts/collect_final.sh <tag>
set -e
T=$1; S=gpurun_out/$T; P=gpurun_out/prof_$T; D=profiles/${ROUND:-r04}/$T
mkdir -p $D/scale
tail -1 $S/bench_default.log > $D/bench_default.json
tail -1 $S/bench_all.log > $D/bench_all.json
grep -E "PASSED|FAILED|passed|failed" $S/gpu_all.log > $D/gpu_tests.txt
cp $S/smoke.log $D/smoke.log
cp $P/kt_kernel_stats.csv $D/kernel_stats.csv
cp $P/pmc_traffic.json $D/pmc_traffic.json
grep config $S/configs.jsonl > $D/configs.jsonl
grep workload $S/carla.jsonl > $D/carla.jsonl
tail -1 $S/bench_e512.log > $D/scale/bench_e512.json
tail -1 $S/bench_e1024.log > $D/scale/bench_e1024.json
for E in 512 1024; do cp $(find $S/scale_e$E -name "*kernel_stats.csv" | head -1) $D/scale/kernel_stats_e$E.csv; done
cp $D/pmc_traffic.json profiles/pmc_traffic.json
