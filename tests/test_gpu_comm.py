"""The product's data-parallel update path (distributed advantage normalisation
ac:830-849, gradient all-reduce before the clip ac:877-885, parameter broadcast ac:551-553) run on
one GPU through the C-ABI:

  * a one-rank RCCL communicator runs the distributed sequence and must give bitwise the same
    parameters, gradient and stats as no communicator (RCCL's one-rank sum / average are exact);
  * the host-transport communicator (ppo_comm_init_host) likewise at world = 1;
  * two ranks (two processes sharing the GPU, all-reduces over torch.distributed gloo) on the two
    halves of the golden ac256 minibatch reproduce the LibTorch two-shard replay (grad_dist2_avg,
    with the distributed advantage statistics dist2_adv_stats) and agree bitwise with each other;
  * a context created with world_size > 1 refuses to update without a communicator.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from golden_inputs import hash_params
from golden_io import load_case

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def filled_agent(seed_data, rank=0, world=1, E=256, T=4, MB=2, EP=2):
    hc = ppo_amd.HipConfig(1, 17, 6, 256, E, T, MB, EP, 0.99, 0.95, 0.1, 0.01, 0.5, 0.5, 1e-5, 1, 1, 1, rank, world)
    ag = ppo_amd.Agent(hc)
    p, x, a, lp, adv, ret, v = seed_data
    ag.load_params(p)
    B = E * T
    ag.buffer(ppo_amd.BUF_OBS, (T, E, 17)).upload(x.reshape(T, E, 17))
    ag.buffer(ppo_amd.BUF_ACTIONS, (T, E, 6)).upload(a.reshape(T, E, 6))
    for buf, arr in ((ppo_amd.BUF_LOGPROBS, lp), (ppo_amd.BUF_ADVANTAGES, adv), (ppo_amd.BUF_RETURNS, ret),
                     (ppo_amd.BUF_VALUES, v)):
        ag.buffer(buf, (T, E)).upload(arr.reshape(T, E))
    assert B == x.shape[0]
    return ag


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(17)
    meta, _ = load_case("ac256_act")
    L = ppo_amd.agent_layout(1, 17, 6, 256)
    p = hash_params(L, meta["hash_base"])
    B = 256 * 4
    x = rng.standard_normal((B, 17)).astype(np.float32)
    a = rng.uniform(-0.95, 0.95, (B, 6)).astype(np.float32)
    lp = (rng.standard_normal(B) * 0.3 - 4.0).astype(np.float32)
    adv = rng.standard_normal(B).astype(np.float32)
    ret = rng.standard_normal(B).astype(np.float32)
    v = rng.standard_normal(B).astype(np.float32)
    return p, x, a, lp, adv, ret, v


def run_two_updates(ag):
    s1 = ag.update(2.5e-4)
    s2 = ag.update(2.0e-4)
    return ag.params(), ag.last_grad(), (s1, s2)


def test_one_rank_rccl_equals_no_communicator_bitwise(data):
    ref = filled_agent(data)
    p_ref, g_ref, s_ref = run_two_updates(ref)
    ref.close()
    ag = filled_agent(data)
    ag.comm_init(ppo_amd.Agent.comm_unique_id(), 0, 1)
    ag.comm_broadcast_params(0)
    np.testing.assert_array_equal(ag.params(), data[0])
    p, g, s = run_two_updates(ag)
    np.testing.assert_array_equal(g, g_ref)
    np.testing.assert_array_equal(p, p_ref)
    assert s == s_ref
    # the communicator's all-reduce entry point itself (average and sum over one rank)
    buf = DeviceArray.from_numpy(np.arange(1000, dtype=np.float32) * 0.37)
    ag.comm_allreduce(buf, average=True)
    np.testing.assert_array_equal(buf.numpy(), np.arange(1000, dtype=np.float32) * np.float32(0.37))
    ag.comm_destroy()
    ag.close()


def test_one_rank_host_transport_equals_no_communicator_bitwise(data):
    ref = filled_agent(data)
    p_ref, g_ref, s_ref = run_two_updates(ref)
    ref.close()
    calls = []
    ag = filled_agent(data)
    ag.comm_init_host(0, 1, lambda buf, avg: calls.append((buf.size, avg)))
    p, g, s = run_two_updates(ag)
    np.testing.assert_array_equal(g, g_ref)
    np.testing.assert_array_equal(p, p_ref)
    assert s == s_ref
    # per update: adv mean (avg) + sum of squares (sum), then one gradient average per minibatch, then stats
    nmb = 2 * 2
    assert calls[0] == (2 * nmb, True) and calls[1] == (nmb, False)
    grads = [(n, avg) for n, avg in calls if n > 100_000]  # the flat (packed) gradient, 146 K floats
    assert len(grads) == 2 * nmb and all(avg for _, avg in grads)  # two updates
    ag.close()


def test_world_size_without_communicator_is_refused(data):
    ag = filled_agent(data, rank=0, world=2)
    with pytest.raises(ppo_amd.PPOError, match="no communicator"):
        ag.update(2.5e-4)
    ag.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_two_ranks_host_transport_vs_golden(tmp_path):
    """Two processes on one GPU, one ac256 half-minibatch each: the averaged gradient equals the
    LibTorch two-shard replay and both ranks end with bitwise identical parameters (rank 1 starts
    from different ones: the broadcast must have replaced them)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_gpu_worker.py"), "ac256", str(tmp_path)],
                              env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(2)]
    outs = []
    for pr in procs:
        try:
            out, _ = pr.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    assert all(pr.returncode == 0 for pr in procs), "\n".join(outs)
    _, d = load_case("ac256_update")
    g0, g1 = np.load(tmp_path / "grad_0.npy"), np.load(tmp_path / "grad_1.npy")
    np.testing.assert_array_equal(g0, g1)
    assert rel(g0, d["grad_dist2_avg"]) < 2e-4, rel(g0, d["grad_dist2_avg"])
    np.testing.assert_array_equal(np.load(tmp_path / "params_0.npy"), np.load(tmp_path / "params_1.npy"))
    np.testing.assert_array_equal(np.load(tmp_path / "stats_0.npy"), np.load(tmp_path / "stats_1.npy"))
