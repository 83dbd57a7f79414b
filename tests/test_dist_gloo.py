"""world_size-2 data-parallel update over gloo on the CPU — the exchange pattern ppo_update runs
over RCCL on the GPU (ppo.cpp_amd/csrc/ppo_capi.hip), with the oracle as the per-rank compute:

  * advantage stats: mean all-reduced with averaging, sum of squares all-reduced with summing,
    std with Bessel's correction over world*M_local (ac_ppo_continuous_action.cpp:830-849);
  * gradients all-reduced with averaging before clip_grad_norm_ + Adam (ac:877-885);
  * loss statistics averaged over ranks (ac:896-901).

Checks: the rank-averaged gradient equals the reference's two-shard gradient (golden
grad_dist2_avg) and the single-process gradient; both ranks stay bit-identical after the optimizer
step; the optimizer step matches the reference's single-process step (params_step1)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from golden_io import load_case


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meta, d = load_case("ac_update")
        L = O.layout_init(1, meta["O"], meta["A"], meta["H"])
        cfg = O.LossCfg(meta["clip_coef"], meta["ent_coef"], meta["vf_coef"], meta["clip_vloss"], meta["norm_adv"])
        M = meta["M"]
        Md = M // world
        sl = slice(rank * Md, (rank + 1) * Md)
        adv = d["adv"][sl].astype(np.float32)
        # distributed advantage statistics (ac:833-846), fp32 like the reference tensors
        mean = torch.tensor([adv.mean(dtype=np.float32)], dtype=torch.float32)
        dist.all_reduce(mean)
        mean /= world
        ss = torch.tensor([np.sum(np.square(adv - mean.numpy()[0]), dtype=np.float32)], dtype=torch.float32)
        dist.all_reduce(ss)
        std = float(torch.sqrt(ss / float(world * Md - 1))[0])
        g, stats = O.minibatch_grad(L, d["params"], d["x"][sl], d["action"][sl], d["old_logp"][sl], adv,
                                    d["ret"][sl], d["old_v"][sl], cfg, adv_mean=float(mean[0]), adv_std=std)
        gt = torch.from_numpy(np.ascontiguousarray(g, np.float32))
        dist.all_reduce(gt)
        gt /= world
        st = torch.from_numpy(np.asarray(stats, np.float32).copy())
        dist.all_reduce(st)
        st /= world
        gc, tn = O.clip_grad_norm(L, gt.numpy(), meta["max_grad_norm"])
        p1, _, _ = O.adam_step(L, d["params"], gc, np.zeros(L.P), np.zeros(L.P), 1, meta["lr"], meta["adam_eps"])
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), grad=gt.numpy(), p1=p1, stats=st.numpy(),
                 adv_stats=np.array([float(mean[0]), std], np.float32))
    finally:
        dist.destroy_process_group()


def rel(a, b):
    return np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(np.asarray(b, np.float64)), 1e-30)


@pytest.mark.timeout(300)
def test_two_rank_update_gloo(tmp_path):
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    _, d = load_case("ac_update")
    r = [np.load(tmp_path / f"rank{i}.npz") for i in range(world)]
    np.testing.assert_allclose(r[0]["adv_stats"], d["dist2_adv_stats"], rtol=1e-6)
    assert rel(r[0]["grad"], d["grad_dist2_avg"]) < 2e-5
    assert rel(r[0]["grad"], d["grad_raw"]) < 2e-5
    for k in ("grad", "p1", "stats"):
        np.testing.assert_array_equal(r[0][k], r[1][k])
    np.testing.assert_allclose(r[0]["p1"], d["params_step1"], rtol=0, atol=2e-7)
