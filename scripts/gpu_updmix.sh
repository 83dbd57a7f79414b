#!/bin/bash
# k_upd vs k_upd32 vs the mixed form (critic 32x32x2, actor 16x16x4): parity tests, then the
# metric-config / E = 512 / cfg4-shard A/B and the stamps of the mixed form.
#   bash scripts/gpu_updmix.sh <tag>
set -o pipefail
TAG=${1:-updmix}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_update_headline.py tests/test_gpu_golden_widths.py > $OUT/tests.txt 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for O in upd_mfma=16 upd_mfma=mix upd_mfma=32; do
  timeout -k 10 200 python bench.py --no-cli --no-cpu-baseline --profile-all --options $O > $OUT/bench_$O.log 2>&1 || { echo "bench $O failed"; tail -30 $OUT/bench_$O.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_$O.log').read().splitlines()[-1]);print('$O',d['ms_per_step'],d['roofline']['frac'],d['roofline']['avg_launch_ms'])"
done
for O in upd_mfma=16 upd_mfma=mix; do
  timeout -k 10 120 python bench.py --num-envs 512 --steps 20 --warmup 3 --profile-all --no-cpu-baseline --no-cli --options $O > $OUT/bench_e512_$O.log 2>&1 || { echo "e512 failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/bench_e512_$O.log').read().splitlines()[-1]);print('E=512 $O',d['ms_per_step'],d.get('kernels_ms_per_step',{}).get('fwdbwd'))"
  timeout -k 10 200 python scripts/bench_configs.py --only cfg4_shard --iters 4 --options $O > $OUT/cfg4_$O.jsonl 2>&1 || { echo "configs failed"; tail -5 $OUT/cfg4_$O.jsonl; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/cfg4_$O.jsonl').read().splitlines()[-1]);print('cfg4 $O',d['ms_per_iteration'],d['kernels_ms_per_iteration']['fwdbwd'])"
done
PPO_OPTS=upd_mfma=mix timeout -k 10 180 python3 scripts/diag_stamps.py > $OUT/kupdmix_phases_hc.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/kupdmix_phases_hc.txt; exit 1; }
grep -v amdgpu.ids $OUT/kupdmix_phases_hc.txt
