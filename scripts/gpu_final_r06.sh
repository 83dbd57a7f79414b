#!/bin/bash
# Round-6 evidence, part A (one GPU box): the whole -m gpu suite + smoke (gpu_r03.sh), the default bench
# line (fp32-MFMA leg, CLI SPS, CPU baseline), the per-kernel-class line, the rocprofv3 kernel trace + the
# two PMC traffic passes (gpu_profile.sh), SQ counters and an L2 pass over the bench command.
#   bash scripts/gpu_final_r06.sh <tag>
set -o pipefail
TAG=${1:-final_r06}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
bash $R/scripts/gpu_r03.sh $TAG || exit 1
cd $R
timeout -k 10 500 python bench.py > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-600
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_all.log 2>&1 || { echo "bench profile-all failed"; exit 1; }
bash $R/scripts/gpu_profile.sh $TAG > $OUT/profile.txt 2>&1 || { echo "profile failed"; tail -5 $OUT/profile.txt; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg" \
  timeout -k 10 400 bash scripts/gpu_counters.sh ${TAG}_sq "$P1" "$P2" > $OUT/sq.txt 2>&1 || { echo "sq counters failed"; tail -20 $OUT/sq.txt; exit 1; }
grep -E "^(fwdbwd|dw|values) " $OUT/sq.txt | head -40
CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg" \
  timeout -k 10 300 bash scripts/gpu_counters.sh ${TAG}_l2 "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" > $OUT/l2.txt 2>&1 || { echo "l2 counters failed"; tail -20 $OUT/l2.txt; exit 1; }
grep -E "^(fwdbwd|dw|values) " $OUT/l2.txt
echo final-a-done
