#!/bin/bash
# why k_upd32 is slower: co-residency of the critic / actor workgroups (stamps) and the shader clock
# over each launch (GRBM_GUI_ACTIVE per kernel), k_upd vs k_upd32; the VALU rollout's phases
set -o pipefail
TAG=${1:-upd32diag}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
PPO_OPTS=upd_mfma=32 timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd32_phases_hc.txt 2>&1 || { echo "stamps32 failed"; tail -20 $OUT/kupd32_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_hc.txt | tail -3
grep -v amdgpu.ids $OUT/kupd32_phases_hc.txt | tail -3
timeout -k 10 120 python3 scripts/roll_stamps.py > $OUT/roll_stamps.txt 2>&1 || { echo "roll stamps failed"; tail -20 $OUT/roll_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/roll_stamps.txt
cd /tmp && export TMPDIR=/tmp
for O in upd_mfma=16 upd_mfma=32; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "k_upd" -d $OUT/pmc_$O -o pmc -- python3 $R/bench.py --no-cli --no-cpu-baseline --steps 2 --warmup 1 --options $O > $OUT/pmc_$O.log 2>&1 || { echo "pmc $O failed"; tail -20 $OUT/pmc_$O.log; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_upd" -d $OUT/trace -o tr -- python3 $R/bench.py --no-cli --no-cpu-baseline --steps 2 --warmup 1 --options upd_mfma=32 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
find $OUT -name "*.csv" | head -20
