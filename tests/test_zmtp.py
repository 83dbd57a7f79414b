"""ZMTP transport, DD-PPO store and CaRL env protocol (reference: include/tcp_store.h,
libs/gymcpp/carla/carla_gym.h, src/carla/ac_ppo_carla.cpp:267-412) on the host, no GPU.

The repo's C++ sockets (ppo.cpp_amd/net/zmtp.h, driven by bin/zmtp_tool) talk to an independent
Python ZMTP 3.0 implementation written from RFC 23 (tests/zmtp_peer.py), which plays the reference's
Python side (pyzmq in the CARLA leaderboard gym, store clients on other ranks):
  * greeting and READY bytes equal the RFC 23 grammar built in Python;
  * TCPStoreServer / TCPStoreClient keep the reference protocol: 'i' / 'r' requests, one-byte ' '
    replies, the count published as a raw int; C++ server <-> Python clients, Python server <-> C++
    client, and the in-process multi-thread pattern of ac_ppo_carla.cpp;
  * CarlaEnv + RecordEpisodeStatisticsCarla + SeqVectorEnvCarla against a scripted leaderboard:
    the hello message, 8-part states, float32 actions (clipped to [-1, 1] when clip_actions), the
    next-step autoreset (no action sent, the next episode's first state received), episode infos.
parity: the wire format is pinned by the RFC and by the two implementations agreeing; no libzmq
peer exists in this image (libzmq / pyzmq absent), so interop with libzmq itself is unpinned."""
import os
import random
import struct
import subprocess
import tempfile
import threading
import time

import numpy as np
import pytest

from zmtp_peer import Peer, frame, greeting, ready

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ppo.cpp_amd")
TOOL = os.path.join(PKG, "bin", "zmtp_tool")


@pytest.fixture(scope="module", autouse=True)
def tool():
    subprocess.check_call(["make", "-C", PKG, "-s", "bin/zmtp_tool"])
    return TOOL


def free_port():
    return random.randint(20000, 40000) * 1  # two consecutive ports are used (REP, PUB)


def test_greeting_and_ready_bytes():
    out = subprocess.check_output([TOOL, "greeting"], text=True).split()
    assert bytes.fromhex(out[0]) == greeting()
    for hx, kind in zip(out[1:], ["PAIR", "REQ", "REP", "PUB", "SUB"]):
        assert bytes.fromhex(hx) == ready(kind, b"" if kind == "REQ" else None), kind


def test_store_threads_in_process():
    """ac_ppo_carla.cpp:267-282, :343-345, :399-412: one server, rank 0 resets, every collection
    thread increments once, every thread's get() converges to the count."""
    out = subprocess.check_output([TOOL, "store-selftest", str(free_port()), "8", "10"], text=True, timeout=120)
    assert "ok 10 rounds x 8 threads" in out


def test_cpp_store_server_python_clients():
    port = free_port()
    srv = subprocess.Popen([TOOL, "store-server", "127.0.0.1", str(port), "20"], stdout=subprocess.PIPE, text=True)
    try:
        assert srv.stdout.readline().startswith("Server started")
        sub = Peer.connect("SUB", f"tcp://127.0.0.1:{port + 1}")
        assert sub.peer_props["Socket-Type"] == b"PUB"
        sub.subscribe()
        time.sleep(0.3)  # the server's PUB socket reads the subscription between requests
        req = Peer.connect("REQ", f"tcp://127.0.0.1:{port}")
        assert req.peer_props["Socket-Type"] == b"REP"
        got = []
        for cmd in (b"r", b"i", b"i", b"i", b"r", b"i"):
            req.send([cmd])
            assert req.recv() == [b" "]
            got.append(struct.unpack("<i", sub.recv()[0])[0])
        assert got == [0, 1, 2, 3, 0, 1]
        # a second client sees the shared count
        req2 = Peer.connect("REQ", f"tcp://127.0.0.1:{port}")
        req2.send([b"i"])
        assert req2.recv() == [b" "]
        assert struct.unpack("<i", sub.recv()[0])[0] == 2
    finally:
        srv.kill()
        srv.wait()


def test_store_server_survives_departed_subscriber_and_oversized_frame():
    """A subscriber that disconnects (RST) while the server publishes is dropped, not fatal (libzmq's
    PUB drops a departed subscriber); a client announcing a frame beyond the request socket's maximum
    message size is disconnected (ZMQ_MAXMSGSIZE); the server keeps serving the others."""
    import socket
    port = free_port()
    srv = subprocess.Popen([TOOL, "store-server", "127.0.0.1", str(port), "20"], stdout=subprocess.PIPE, text=True)
    try:
        assert srv.stdout.readline().startswith("Server started")
        keep = Peer.connect("SUB", f"tcp://127.0.0.1:{port + 1}")
        keep.subscribe()
        gone = Peer.connect("SUB", f"tcp://127.0.0.1:{port + 1}")
        gone.subscribe()
        time.sleep(0.3)
        req = Peer.connect("REQ", f"tcp://127.0.0.1:{port}")
        req.send([b"r"])
        assert req.recv() == [b" "]
        assert struct.unpack("<i", keep.recv()[0])[0] == 0
        # abortive close: the next writes to it fail with EPIPE / ECONNRESET
        gone.s.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
        gone.close()
        for k in range(1, 6):
            req.send([b"i"])
            assert req.recv() == [b" "]
            assert struct.unpack("<i", keep.recv()[0])[0] == k
        # a 2**40-byte frame announced to the REP socket: that client is dropped
        bad = Peer.connect("REQ", f"tcp://127.0.0.1:{port}")
        bad.s.sendall(bytes([0x02]) + struct.pack(">Q", 1 << 40) + b"x" * 16)
        time.sleep(0.3)
        with pytest.raises((ConnectionError, OSError)):
            bad.s.settimeout(5)
            bad.send([b"i"])
            bad.recv()
        req.send([b"i"])
        assert req.recv() == [b" "]
        assert struct.unpack("<i", keep.recv()[0])[0] == 6
        assert srv.poll() is None  # still running
    finally:
        srv.kill()
        srv.wait()


def test_python_store_server_cpp_client():
    """the reference protocol served from Python; the C++ client's increment / reset / get."""
    port = free_port()
    lrep = socket_listen(port)
    lpub = socket_listen(port + 1)
    state = {"n": 0}
    subs = []

    def serve():
        pub_conn, _ = lpub.accept()
        subs.append(Peer("PUB", pub_conn))
        sub_msg = subs[0].recv()
        assert sub_msg == [b"\x01"]  # subscribe to everything (ZMTP 3.0 form)
        rep_conn, _ = lrep.accept()
        rep = Peer("REP", rep_conn)
        while True:
            try:
                parts = rep.recv()
            except (ConnectionError, OSError):
                return
            assert parts[0] == b""  # REQ envelope delimiter
            cmd = parts[1]
            state["n"] = state["n"] + 1 if cmd == b"i" else 0
            rep.send([b"", b" "])
            subs[0].send([struct.pack("<i", state["n"])])

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    out = subprocess.check_output([TOOL, "store-client", "127.0.0.1", str(port), "riiiw3iw4rw0"], text=True, timeout=60)
    assert out.split() == ["3", "4", "0"]
    lrep.close()
    lpub.close()


def socket_listen(port):
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.bind(("127.0.0.1", port))
    s.listen(4)
    return s


def fnv(b):
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.parametrize("clip", [1, 0])
def test_carla_env_protocol(clip):
    """zmtp_tool carla-env prints one line per step:
    step t reward R term T trunc U bev H meas H vmeas H info yes|no return length"""
    C, H, W, NM, NV = 3, 8, 6, 8, 3
    steps = 9
    rng = np.random.default_rng(3)
    with tempfile.TemporaryDirectory() as root:
        port = free_port()
        env = subprocess.Popen([TOOL, "carla-env", root, str(port), str(steps), str(C), str(H), str(W), str(NM),
                                str(NV), str(clip)], stdout=subprocess.PIPE, text=True)
        try:
            gym = Peer.connect("PAIR", f"ipc://{root}/comm_files/{port}.lock")
            assert gym.peer_props["Socket-Type"] == b"PAIR"
            gym.send([b"Hello from the leaderboard gym."])

            def state(reward, term, trunc):
                bev = rng.integers(0, 256, C * H * W, dtype=np.uint8).tobytes()
                m = rng.standard_normal(NM).astype(np.float32).tobytes()
                v = rng.standard_normal(NV).astype(np.float32).tobytes()
                gym.send([bev, m, v, struct.pack("<f", reward), bytes([term]), bytes([trunc]), struct.pack("<i", 7),
                          struct.pack("<i", 0)])
                return ["%016x" % fnv(bev), "%016x" % fnv(m), "%016x" % fnv(v)]

            reset_hashes = state(0.0, 0, 0)
            expect = []  # per C++ step: (reward, term, trunc, hashes, info)
            ep_ret, ep_len = np.float32(0.0), 0
            t = 0
            while t < steps:
                a = np.frombuffer(gym.recv()[0], np.float32)
                want = np.array([1.5 * np.sin(np.float32(t)), 1.5 * np.cos(np.float32(t))], np.float32)
                if clip:
                    want = np.clip(want, -1.0, 1.0)
                np.testing.assert_allclose(a, want, rtol=1e-6, atol=1e-7)
                r = np.float32(0.25 * (t + 1))
                term, trunc = int(t == 3), int(t == 6)
                hashes = state(float(r), term, trunc)
                ep_ret, ep_len = np.float32(ep_ret + r), ep_len + 1
                info = (ep_ret, ep_len) if term or trunc else None
                expect.append((r, term, trunc, hashes, info))
                t += 1
                if term or trunc:
                    # SeqVectorEnvCarla's next step is the autoreset: no action, the next episode's first state
                    expect.append((np.float32(0.0), 0, 0, state(0.0, 0, 0), None))
                    ep_ret, ep_len = np.float32(0.0), 0
                    t += 1
            out = env.communicate(timeout=60)[0]
        finally:
            if env.poll() is None:
                env.kill()
        assert env.returncode == 0
        lines = [ln.split() for ln in out.splitlines() if ln.startswith(("reset", "step"))]
        assert lines[0] == ["reset", "bev", reset_hashes[0], "meas", reset_hashes[1], "vmeas", reset_hashes[2]]
        assert len(lines) - 1 == len(expect) == steps
        for k, (f, (r, term, trunc, hashes, info)) in enumerate(zip(lines[1:], expect)):
            assert int(f[1]) == k
            assert np.float32(float(f[3])) == r and int(f[5]) == term and int(f[7]) == trunc, f
            assert [f[9], f[11], f[13]] == hashes, (k, f)
            assert f[15] == ("yes" if info else "no"), f
            if info:
                assert np.float32(float(f[16])) == info[0] and int(f[17]) == info[1], f
