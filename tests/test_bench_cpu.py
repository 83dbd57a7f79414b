"""bench.py's launcher logic (no GPU needed): `--gpus N` starts N ranks itself through
torch.distributed.run on 127.0.0.1, and a launcher whose WORLD_SIZE disagrees with --gpus is refused
before anything touches the GPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_cmd_one_process_per_gpu():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "3"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29555" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_import_does_not_load_the_library():
    assert bench.ppo_amd is None


def test_world_size_mismatch_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
