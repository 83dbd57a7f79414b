"""bench.py contract (the driver's JSON line) on one GPU, and its multi-rank path rehearsed with the
host transport (every rank on GPU 0, torch.distributed.run over 127.0.0.1)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline")


def last_json(out):
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def test_bench_single_rank_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-cli", "--no-cpu-baseline", "--num-envs", "512"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, check=True)
    d = last_json(r.stdout)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    roof = d["roofline"]
    assert roof["bound"] == "mfma" and 0 < roof["frac"] < 1 and roof["peak"] == 157.3
    assert abs(d["value"] - 512 * 128 / (d["ms_per_step"] / 1e3)) / d["value"] < 0.01
    assert d["config"]["devices"] == [0] and len(d["config"]["device_pci_bus_ids"]) == 1
    # the precision choice is visible in the line: the fp32-MFMA leg of the same workload beside the
    # headline, and dW's fraction beside k_upd's
    f = d["fp32_mfma"]
    assert f["options"] == "upd_mfma=16,dw_mfma=f32" and f["value"] > 0 and "bx" not in f["kernels"]
    assert 0 < f["fwdbwd"]["frac"] < 1
    assert 0 < roof["dw"]["frac"] < 2 and roof["dw"]["launches"] > 0


def test_bench_one_rank_rccl_reports_its_device():
    """`--comm-1rank`: a one-rank RCCL communicator on the rank's own device; the line names it."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--comm-1rank",
                        "--no-cli", "--no-cpu-baseline", "--num-envs", "512"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, check=True)
    d = last_json(r.stdout)
    assert d["config"]["devices"] == [0]
    assert d["config"]["comm_kind"] == "rccl" and d["config"]["comm_ranks"] == 1


def test_bench_rank_without_its_gpu_fails_loudly():
    """Rank k runs on GPU k (the reference's cudaSetDevice(gpu_ids.at(local_rank)), ac:447-448). A
    rank whose LOCAL_RANK names a GPU the box does not have must fail with a message naming that
    device -- never fall back silently onto GPU 0."""
    import ppo_amd
    n = ppo_amd.device_count()
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK=str(n))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--no-cli",
                        "--no-cpu-baseline", "--num-envs", "512"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=env)
    assert r.returncode != 0
    assert f"device {n} requested but {n} HIP device(s) are visible" in r.stderr, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_two_ranks_host_transport():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--comm", "host", "--num-envs", "1024"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env, check=True)
    d = last_json(r.stdout)
    for k in KEYS:
        assert k in d, k
    assert d["n_gpus"] == 2 and d["config"]["num_envs_per_device"] == 512 and d["config"]["parallelism"] == "dp2"
    assert d["value"] > 0 and "comm" in d["config"]
    assert d["config"]["devices"] == [0, 0] and d["config"]["comm_ranks"] == 2  # the rehearsal: both on GPU 0


def test_bench_gpus_flag_starts_the_ranks_itself():
    """`bench.py --gpus 2` with no external launcher runs two ranks (the driver's SCALE runs may call
    it that way); the communicator itself reports the rank count."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--comm", "host", "--num-envs", "4096", "--no-cli"], capture_output=True, text=True,
                       timeout=300, cwd=ROOT, env=env, check=True)
    d = last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["num_envs_per_device"] == 2048 and d["config"]["parallelism"] == "dp2"
    assert d["config"]["comm_ranks"] == 2 and d["config"]["comm_kind"] == "host"
    assert "cpu_baseline" not in d

