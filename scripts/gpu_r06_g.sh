#!/bin/bash
# Round-6 evidence on one box: the default bench line (fp32 leg, CLI, CPU baseline), the kernel
# trace + PMC traffic passes, SQ counters (k_upd, dW, k_vbx) + an L2 pass, the shard lines, the
# other configs and CaRL.   bash scripts/gpu_r06_g.sh <tag>
set -o pipefail
TAG=${1:-r06g}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python bench.py > $OUT/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_all.log 2>&1 || { echo "bench profile-all failed"; exit 1; }
bash $R/scripts/gpu_profile.sh $TAG > $OUT/profile.txt 2>&1 || { echo "profile failed"; tail -5 $OUT/profile.txt; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg" \
  timeout -k 10 400 bash scripts/gpu_counters.sh ${TAG}_sq "$P1" "$P2" > $OUT/sq.txt 2>&1 || { echo "sq counters failed"; tail -20 $OUT/sq.txt; exit 1; }
grep -E "^(fwdbwd|dw|values) " $OUT/sq.txt | head -60
if grep -q "TCP_TCC_READ_REQ_sum" $R/gpurun_out/ctr_${TAG}_sq/counters_list.txt; then
  CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --no-fp32-leg" \
    timeout -k 10 300 bash scripts/gpu_counters.sh ${TAG}_l2 "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" > $OUT/l2.txt 2>&1 || { echo "l2 counters failed"; tail -20 $OUT/l2.txt; exit 1; }
  grep -E "^(fwdbwd|dw|values) " $OUT/l2.txt
fi
timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; exit 1; }
cut -c1-300 $OUT/configs.jsonl
timeout -k 10 300 python scripts/bench_carla.py > $OUT/carla.jsonl 2>&1 || { echo "carla failed"; exit 1; }
for E in 512 1024; do
  timeout -k 10 120 python bench.py --num-envs $E --steps 30 --warmup 3 --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_e$E.log 2>&1 || { echo "e$E failed"; exit 1; }
  timeout -k 10 120 python bench.py --num-envs $E --steps 10 --warmup 3 --profile-all --no-cpu-baseline --no-cli --no-fp32-leg > $OUT/bench_all_e$E.log 2>&1 || { echo "e$E all failed"; exit 1; }
  tail -1 $OUT/bench_all_e$E.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernels_ms_per_step"])'
done
echo g-done
