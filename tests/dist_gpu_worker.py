"""One rank of tests/test_gpu_comm.py::test_two_ranks_host_transport_vs_golden (run as a child
process, RANK / WORLD_SIZE / MASTER_* in the environment): the product's data-parallel update
(libppo_hip.so ppo_update with a host-transport communicator over torch.distributed gloo) on this
rank's half of a golden minibatch.
  python dist_gpu_worker.py <case> <out_dir>
Writes grad_<rank>.npy (the averaged pre-clip gradient) and params_<rank>.npy (after one Adam step)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "ppo.cpp_amd")):
    sys.path.insert(0, p)

import ppo_amd  # noqa: E402  (imports torch first: one HIP runtime)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from golden_inputs import hash_params  # noqa: E402
from golden_io import load_case  # noqa: E402


def main():
    case, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    meta, _ = load_case(case + "_act")
    mu, d = load_case(case + "_update")
    M = mu["M"]
    Md = M // world
    sl = slice(rank * Md, (rank + 1) * Md)
    O_, A = meta["O"], meta["A"]
    hc = ppo_amd.HipConfig(meta["kind"], O_, A, meta["H"], Md, 1, 1, 1, 0.99, 0.95, mu["clip_coef"], mu["ent_coef"],
                           mu["vf_coef"], mu["max_grad_norm"], mu["adam_eps"], 1, 1, 1, rank, world)
    ppo_amd.set_device(0)
    ag = ppo_amd.Agent(hc)
    L = ag.layout
    p = hash_params(L, meta["hash_base"], meta.get("hi", 1.0), meta.get("lo", -1.0))
    if rank != 0:  # the broadcast (ac:551-553) must replace these
        p = (p * 0.5 + 0.25).astype(np.float32)
    ag.load_params(p)

    def allreduce(buf, average):
        t = torch.from_numpy(buf)  # shares memory with the library's host staging buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if average:
            t /= world
    ag.comm_init_host(rank, world, allreduce)
    ag.comm_broadcast_params(0)
    ag.buffer(ppo_amd.BUF_OBS, (1, Md, O_)).upload(d["x"][sl].reshape(1, Md, O_))
    ag.buffer(ppo_amd.BUF_ACTIONS, (1, Md, A)).upload(d["action"][sl].reshape(1, Md, A))
    for buf, key in ((ppo_amd.BUF_LOGPROBS, "old_logp"), (ppo_amd.BUF_ADVANTAGES, "adv"),
                     (ppo_amd.BUF_RETURNS, "ret"), (ppo_amd.BUF_VALUES, "old_v")):
        ag.buffer(buf, (1, Md)).upload(d[key][sl].reshape(1, Md))
    st = ag.update(mu["lr"], perms=ppo_amd.DeviceArray.from_numpy(np.arange(Md, dtype=np.int32)))
    np.save(os.path.join(out, f"grad_{rank}.npy"), ag.last_grad())
    np.save(os.path.join(out, f"params_{rank}.npy"), ag.params())
    np.save(os.path.join(out, f"stats_{rank}.npy"), np.array([st[k] for k in ("pg_loss", "v_loss", "entropy",
                                                                              "grad_norm")], np.float32))
    ag.comm_destroy()
    ag.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
