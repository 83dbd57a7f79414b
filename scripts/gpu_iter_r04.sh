#!/bin/bash
# One round-4 iteration on the box: parity tests of the touched kernels, the default bench line, the
# N = 8 / N = 4 shard lines, the other configs, and the phase stamps.
#   bash scripts/gpu_iter_r04.sh <tag> ["<test files>"]
set -o pipefail
TAG=${1:-iter}
TESTS=${2:-"tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_golden_widths.py tests/test_gpu_update_headline.py"}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for PR in ${PROBES:-}; do
  timeout -k 10 60 scripts/probe/$PR > $OUT/$PR.jsonl 2>&1 || { echo "probe $PR failed"; cat $OUT/$PR.jsonl; exit 1; }
  cat $OUT/$PR.jsonl
done
if [ "$TESTS" != none ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
fi
timeout -k 10 300 python bench.py --no-cli --no-cpu-baseline --profile-all > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
python3 -c "import json;d=json.loads(open('$OUT/bench.log').read().splitlines()[-1]);print('roof',d['roofline']['frac'],d['roofline']['avg_launch_ms']);print(d.get('kernels_ms_per_step'))"
for E in 512 1024; do
timeout -k 10 120 python bench.py --num-envs $E --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli > $OUT/bench_e$E.log 2>&1 || { echo "e$E failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench_e$E.log').read().splitlines()[-1]);print('E=$E',d['ms_per_step'],d.get('kernels_ms_per_step'))"
done
timeout -k 10 300 python scripts/bench_configs.py > $OUT/configs.jsonl 2>&1 || { echo "configs failed"; tail -5 $OUT/configs.jsonl; exit 1; }
cut -c1-400 $OUT/configs.jsonl
timeout -k 10 240 python3 scripts/diag_stamps2.py > $OUT/kupd2_phases.txt 2>&1 || { echo "upd2 stamps failed"; tail -20 $OUT/kupd2_phases.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd2_phases.txt
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "hc stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_hc.txt
timeout -k 10 120 python3 scripts/roll_stamps.py > $OUT/roll_stamps.txt 2>&1 || { echo "roll stamps failed"; tail -20 $OUT/roll_stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/roll_stamps.txt
