"""A second, independent ZMTP 3.0 implementation (RFC 23, NULL mechanism) for tests: it plays the
Python side of the reference (pyzmq in the CARLA leaderboard gym / eval_agent.py, or store clients)
against the repo's C++ sockets (ppo.cpp_amd/net/zmtp.h). Written from the RFC grammar, not from the
C++ code, so the two check each other's bytes. Test infrastructure only."""
import socket
import struct
import time

SIG = b"\xff" + b"\x00" * 8 + b"\x7f"


def greeting(minor=0):
    """signature, version 3.minor, mechanism "NULL" padded to 20, as-server 0, 31 zero filler"""
    return SIG + bytes([3, minor]) + b"NULL".ljust(20, b"\x00") + b"\x00" + b"\x00" * 31


def frame(body, more=False, command=False):
    flags = (0x01 if more else 0) | (0x04 if command else 0)
    if len(body) > 255:
        return bytes([flags | 0x02]) + struct.pack(">Q", len(body)) + body
    return bytes([flags, len(body)]) + body


def ready(sock_type, identity=None):
    body = b"\x05READY"
    props = [(b"Socket-Type", sock_type.encode())]
    if identity is not None:
        props.append((b"Identity", identity))
    for k, v in props:
        body += bytes([len(k)]) + k + struct.pack(">I", len(v)) + v
    return frame(body, command=True)


class Peer:
    """One ZMTP connection. kind: PAIR, REQ, REP, PUB, SUB (one peer only)."""

    def __init__(self, kind, sock):
        self.kind, self.s, self.buf = kind, sock, b""
        self.s.settimeout(20)
        self.s.sendall(greeting())
        g = self._read(64)
        assert g[:10] == SIG[:1] + g[1:9] + SIG[9:] and g[0] == 0xFF and g[9] == 0x7F, g
        assert g[10] >= 3 and g[12:16] == b"NULL", g
        self.s.sendall(ready(kind, b"" if kind == "REQ" else None))
        flags, body = self._frame()
        assert flags & 0x04 and body[1:1 + body[0]] == b"READY", (flags, body)
        self.peer_props = self._props(body[1 + body[0]:])

    @staticmethod
    def _props(b):
        out, q = {}, 0
        while q < len(b):
            n = b[q]
            k = b[q + 1:q + 1 + n]
            q += 1 + n
            (vn,) = struct.unpack(">I", b[q:q + 4])
            out[k.decode()] = b[q + 4:q + 4 + vn]
            q += 4 + vn
        return out

    @classmethod
    def connect(cls, kind, endpoint, timeout=20):
        t0 = time.time()
        while True:
            try:
                if endpoint.startswith("ipc://"):
                    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                    s.connect(endpoint[6:])
                else:
                    host, port = endpoint[6:].rsplit(":", 1)
                    s = socket.create_connection((host, int(port)))
                return cls(kind, s)
            except (FileNotFoundError, ConnectionRefusedError):
                if time.time() - t0 > timeout:
                    raise
                time.sleep(0.02)

    def _read(self, n):
        while len(self.buf) < n:
            chunk = self.s.recv(65536)
            if not chunk:
                raise ConnectionError("peer closed")
            self.buf += chunk
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def _frame(self):
        flags, = self._read(1)
        if flags & 0x02:
            (n,) = struct.unpack(">Q", self._read(8))
        else:
            n, = self._read(1)
        return flags, self._read(n)

    def send(self, parts):
        if self.kind == "REQ":
            parts = [b""] + list(parts)
        data = b"".join(frame(p, more=i + 1 < len(parts)) for i, p in enumerate(parts))
        self.s.sendall(data)

    def recv(self):
        parts = []
        while True:
            flags, body = self._frame()
            if flags & 0x04:
                continue  # commands (PING etc.)
            parts.append(body)
            if not flags & 0x01:
                break
        if self.kind == "REQ":
            assert parts[0] == b"", parts
            parts = parts[1:]
        return parts

    def subscribe(self, topic=b""):
        self.send([b"\x01" + topic])

    def close(self):
        self.s.close()
