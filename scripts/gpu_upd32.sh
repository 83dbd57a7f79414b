#!/bin/bash
# k_upd32 (upd_mfma=32) iteration: its parity tests, then k_upd vs k_upd32 at the metric config and
# the E = 512 / cfg4 shards.   bash scripts/gpu_upd32.sh <tag>
set -o pipefail
TAG=${1:-upd32}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py -k "upd32 or mfma32 or update_vs_golden" \
  > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for O in upd_mfma=16 upd_mfma=32; do
  timeout -k 10 200 python bench.py --no-cli --no-cpu-baseline --profile-all --options $O > $OUT/bench_$O.log 2>&1 || { echo "bench $O failed"; tail -30 $OUT/bench_$O.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_$O.log').read().splitlines()[-1]);print('$O',d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'],d.get('kernels_ms_per_step'))"
  timeout -k 10 120 python bench.py --num-envs 512 --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli --options $O > $OUT/bench_e512_$O.log 2>&1 || { echo "e512 failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_e512_$O.log').read().splitlines()[-1]);print('E=512 $O',d['ms_per_step'],d.get('kernels_ms_per_step'))"
done
for O in upd_mfma=16 upd_mfma=32; do
timeout -k 10 200 python scripts/bench_configs.py --only cfg4_shard --iters 4 --options $O > $OUT/cfg4_$O.jsonl 2>&1 || { echo "configs failed"; tail -5 $OUT/cfg4_$O.jsonl; exit 1; }
grep cfg4 $OUT/cfg4_$O.jsonl | cut -c1-400
done
timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd_phases_hc.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/kupd_phases_hc.txt; exit 1; }
PPO_OPTS=upd_mfma=32 timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupd32_phases_hc.txt 2>&1 || { echo "stamps32 failed"; tail -20 $OUT/kupd32_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupd_phases_hc.txt | head -32
grep -v amdgpu.ids $OUT/kupd32_phases_hc.txt | head -32
