#!/bin/bash
# Round-5 second half: SQ counters of the split-bf16 k_upd (bx6, the default) and of the fp32 form,
# then the GAE parity tests and cfg2 (GAE time) with the software-pipelined k_gae.
#   bash scripts/gpu_r05_c2.sh <tag>
set -o pipefail
TAG=${1:-r05c2}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ddppo.py -k "gae or ddppo or partial" -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/gae_tests.log 2>&1 || { echo "gae tests failed"; grep -E "FAIL|Error|assert" $OUT/gae_tests.log | head; exit 1; }
grep -cE "PASSED" $OUT/gae_tests.log
timeout -k 10 200 python scripts/bench_configs.py --only cfg2 > $OUT/cfg2.log 2>&1 || { echo "cfg2 failed"; exit 1; }
tail -1 $OUT/cfg2.log | cut -c1-400
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
for V in bx6 16; do
  CTR_CMD="bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-cli --options upd_mfma=$V" \
    timeout -k 10 400 bash scripts/gpu_counters.sh ${TAG}_upd$V "$P1" "$P2" > $OUT/sq_upd$V.txt 2>&1 || { echo "counters $V failed"; tail -20 $OUT/sq_upd$V.txt; exit 1; }
  grep -E "^(fwdbwd|dw) " $OUT/sq_upd$V.txt
done
echo c2-done
