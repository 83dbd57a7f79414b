"""world_size-2 data-parallel CaRL minibatch update over gloo on the CPU — the exchange pattern
ppo_carla_update runs over RCCL when a communicator is attached (ppo.cpp_amd/csrc/ppo_carla.hip,
ppo_carla_comm_init), with the plain PyTorch fp32 reference (tests/carla_torch_ref.py, pinned to
the LibTorch golden in test_carla_oracle) as the per-rank compute:

  * advantage mean all-reduced with averaging, sum of squares about it all-reduced with summing,
    std with Bessel's correction over world * n_local - 1 (ac_ppo_carla.cpp:561-580);
  * every gradient all-reduced with averaging before clip_grad_norm_ + Adam (:608-619).

Checks: both ranks end bit-identical; the rank-averaged gradient, the total norm and the stepped
parameters equal the single-process update of the whole minibatch (the loss is a mean over rows,
so averaging equal-sized shards is the full-batch gradient); fp32 summation order differs, so
gradient rel-L2 < 1e-5 and parameters atol 3e-7 (a first Adam step is ±lr·g/(|g|+eps), so tiny
gradients carry their rounding into it)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import carla_inputs as CI
import carla_torch_ref as TR

N = 4  # whole minibatch; 2 rows per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    rng = np.random.default_rng(11)
    bev = rng.integers(0, 256, size=(N, 15, 192, 192), dtype=np.uint8)
    f = lambda *shape: rng.uniform(-1, 1, shape).astype(np.float32)  # noqa: E731
    return (bev, f(N, 8), f(N, 3), f(N, 2) * 0.95, f(N) * 0.2, rng.standard_normal(N).astype(np.float32),
            rng.standard_normal(N).astype(np.float32), f(N) * 0.1)


def _rank_main(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = CI.layout()
        p = CI.params(L)
        bev, meas, vmeas, act, old_logp, adv, ret, old_v = _batch()
        n = N // world
        sl = slice(rank * n, (rank + 1) * n)
        a = torch.from_numpy(adv[sl].copy())
        mean = a.mean().reshape(1)
        dist.all_reduce(mean)
        mean /= world
        ss = ((a - mean) ** 2).sum().reshape(1)
        dist.all_reduce(ss)
        std = torch.sqrt(ss / float(world * n - 1))

        def avg(grads):
            for g_ in grads:
                dist.all_reduce(g_)
                g_ /= world

        grad, stats, total, newp, _, _ = TR.update(L, p, bev[sl], meas[sl], vmeas[sl], act[sl], old_logp[sl],
                                                   adv[sl], ret[sl], old_v[sl], adv_stats=(mean, std),
                                                   allreduce_grads=avg)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), grad=grad, total=np.float64(total), p1=newp)
    finally:
        dist.destroy_process_group()


def rel(a, b):
    return np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(np.asarray(b, np.float64)), 1e-30)


@pytest.mark.timeout(300)
def test_carla_two_rank_update_gloo(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    for k in ("grad", "total", "p1"):
        np.testing.assert_array_equal(r[0][k], r[1][k])
    L = CI.layout()
    p = CI.params(L)
    grad, _, total, newp, _, _ = TR.update(L, p, *_batch())
    assert rel(r[0]["grad"], grad) < 1e-5
    np.testing.assert_allclose(r[0]["total"], total, rtol=1e-5)
    np.testing.assert_allclose(r[0]["p1"], newp, rtol=0, atol=3e-7)
