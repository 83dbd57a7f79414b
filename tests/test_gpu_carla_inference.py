"""The CaRL inference server (ppo.cpp_amd/bin/ppo_carla_inference, drop-in of
src/carla/ppo_carla_inference.cpp) driven the way eval_agent.py drives it, over ZMTP
from tests/zmtp_peer.py (the Python side of the reference uses pyzmq):

  * hello "Connected to eval_agent.py.", sample type answer, per step an empty keepalive then the
    3-part observation, 4-frame answer [action | value | mu | sigma], a non-empty keepalive ends the
    route (exit 0);
  * the answer is the ensemble mean over every model*.pth in the folder (two here), each model the
    repo's CaRL forward (include/ppo_carla.h) on the same observation: compared with the direct
    ppo_carla_forward calls through the C-ABI — bitwise for mean / roach (deterministic);
  * a folder without a model file exits with status 2, as the reference.
Tolerance: exact (same kernels, same inputs; the mean is a float32 sum over the models / count)."""
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

import carla_inputs as CI
from zmtp_peer import Peer

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(ROOT, "ppo.cpp_amd", "bin", "ppo_carla_inference")


def write_models(folder, L, n_models):
    ps = []
    for i in range(n_models):
        p = CI.params(L).copy()
        if i:  # a second, different model
            rng = np.random.default_rng(i)
            p *= np.float32(1.0) + rng.uniform(-0.2, 0.2, p.shape).astype(np.float32)
            p[L.hi], p[L.lo] = 1.0, -1.0
        ppo_amd.save_carla_pth(ppo_amd.carla_layout(CI.CH, CI.HW, CI.HW, CI.NM, CI.NV, CI.A), p,
                               os.path.join(folder, f"model_{i:04d}.pth"))
        ps.append(p)
    with open(os.path.join(folder, "config.json"), "w") as f:
        json.dump({"seed": 1, "obs_num_channels": CI.CH, "bev_semantics_height": CI.HW, "bev_semantics_width": CI.HW,
                   "obs_num_measurements": CI.NM, "num_value_measurements": CI.NV, "beta_min_a_b_value": CI.BETA_MIN,
                   "image_encoder": "roach", "ports": [5555]}, f)
    return ps


@pytest.mark.parametrize("sample_type", ["mean", "roach"])
def test_inference_server_ensemble(sample_type):
    L = CI.layout()
    bev, meas, vmeas, _ = CI.inputs(3)
    with tempfile.TemporaryDirectory() as models, tempfile.TemporaryDirectory() as ipc:
        ps = write_models(models, L, 2)
        port = 6001
        srv = subprocess.Popen([SERVER, "--path_to_conf_file", models, "--ipc_path", ipc, "--port", str(port)],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        try:
            agent = Peer.connect("PAIR", f"ipc://{ipc}/{port}.lock")
            assert agent.recv() == [b"Connected to eval_agent.py."]
            agent.send([sample_type.encode()])
            answers = []
            for k in range(3):
                agent.send([b""])
                agent.send([bev[k].tobytes(), meas[k].tobytes(), vmeas[k].tobytes()])
                parts = agent.recv()
                assert [len(x) for x in parts] == [4 * CI.A, 4, 4 * CI.A, 4 * CI.A]
                answers.append([np.frombuffer(x, np.float32) for x in parts])
            agent.send([b"done"])
            out, err = srv.communicate(timeout=60)
        finally:
            if srv.poll() is None:
                srv.kill()
        assert srv.returncode == 0, err
        assert "Finished route." in out and f"Deterministic actions: {sample_type}" in out
    # the same forward per model through the C-ABI, then the ensemble mean
    expect = []
    for k in range(3):
        per = []
        for i, p in enumerate(ps):
            ag = ppo_amd.CarlaAgent(1, obs_channels=CI.CH, bev=CI.HW, num_measurements=CI.NM,
                                    num_value_measurements=CI.NV, action_dim=CI.A, beta_min=CI.BETA_MIN, seed=1 + i)
            ag.load_params(p)
            a, _, _, v, al, be = ag.forward(DeviceArray.from_numpy(bev[k:k + 1]), DeviceArray.from_numpy(meas[k:k + 1]),
                                            DeviceArray.from_numpy(vmeas[k:k + 1]), sample_type=sample_type,
                                            step_id=k)
            per.append([a.numpy()[0], v.numpy()[:1], al.numpy()[0], be.numpy()[0]])
            ag.close()
        assert not np.array_equal(per[0][1], per[1][1])  # two different models are averaged
        expect.append([(per[0][j] + per[1][j]) / np.float32(2.0) for j in range(4)])
    for got, want in zip(answers, expect):
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w.astype(np.float32))


def test_inference_server_without_models_exits_2():
    with tempfile.TemporaryDirectory() as models, tempfile.TemporaryDirectory() as ipc:
        with open(os.path.join(models, "config.json"), "w") as f:
            json.dump({"seed": 1}, f)
        srv = subprocess.Popen([SERVER, "--path_to_conf_file", models, "--ipc_path", ipc, "--port", "6002"],
                               stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        try:
            agent = Peer.connect("PAIR", f"ipc://{ipc}/6002.lock")
            assert agent.recv() == [b"Connected to eval_agent.py."]
            agent.send([b"mean"])
            _, err = srv.communicate(timeout=60)
        finally:
            if srv.poll() is None:
                srv.kill()
        assert srv.returncode == 2
        assert "No model file was found in the selected path:" in err
