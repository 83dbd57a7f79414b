"""The protobuf-free TensorBoard event writer (ppo.cpp_amd/apps/tensorboard_logger.h, SURVEY
§8(f)-1) against an independent encoder: the tensorflow.Event / Summary / Summary.Value messages are
declared at run time with google.protobuf's descriptor API and serialized by the protobuf runtime
(the reference serializes with libprotobuf, tensorboard_logger.cc:314-335). Records are checked
byte for byte, including the TFRecord framing and its masked CRC32C values."""
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

CASES = [("charts/SPS", 524288, 1.5e7), ("losses/value_loss", 0, 0.0), ("charts/episodic_return", 4096, -12.25),
         ("eval/avg_return", -3, 1e-30), ("losses/clipfrac", 2**31 - 1, 0.3333)]
WALL = 1760000000.0


def event_classes():
    fd = descriptor_pb2.FileDescriptorProto(name="tb_event_test.proto", package="tensorflow", syntax="proto3")
    val = fd.message_type.add(name="Value")
    val.field.add(name="tag", number=1, type=9, label=1)
    val.field.add(name="simple_value", number=2, type=2, label=1, oneof_index=0)
    val.oneof_decl.add(name="value")
    summ = fd.message_type.add(name="Summary")
    summ.field.add(name="value", number=1, type=11, label=3, type_name=".tensorflow.Value")
    ev = fd.message_type.add(name="Event")
    ev.field.add(name="wall_time", number=1, type=1, label=1)
    ev.field.add(name="step", number=2, type=3, label=1)
    ev.field.add(name="summary", number=5, type=11, label=1, type_name=".tensorflow.Summary", oneof_index=0)
    ev.oneof_decl.add(name="what")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tensorflow.Event"))


def crc32c(data):
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ 0x82F63B78 if crc & 1 else crc >> 1
    return crc ^ 0xFFFFFFFF


def masked(data):
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def test_crc32c_known_answer():
    assert crc32c(b"123456789") == 0xE3069283  # CRC-32C check value


def test_event_records_match_protobuf(tmp_path):
    src = tmp_path / "w.cpp"
    lines = [f'  w.write(tb::scalar_event({WALL!r}, {s}, "{t}", (float){v!r}));' for t, s, v in CASES]
    src.write_text('#include "tensorboard_logger.h"\nint main(int, char** argv) {\n'
                   '  TensorBoardLogger w(argv[1]);\n' + "\n".join(lines) + "\n  return 0;\n}\n")
    exe = tmp_path / "w"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "ppo.cpp_amd", "apps"), str(src),
                           "-o", str(exe)])
    out = tmp_path / "tfevents_logs.pb"
    subprocess.check_call([str(exe), str(out)])
    data = out.read_bytes()
    Event = event_classes()
    pos = 0
    for tag, step, value in CASES:
        n, len_crc = struct.unpack_from("<QI", data, pos)
        assert len_crc == masked(data[pos:pos + 8])
        payload = data[pos + 12:pos + 12 + n]
        (data_crc,) = struct.unpack_from("<I", data, pos + 12 + n)
        assert data_crc == masked(payload)
        e = Event()
        e.wall_time = WALL
        e.step = step
        v = e.summary.value.add()
        v.tag = tag
        v.simple_value = value
        assert payload == e.SerializeToString(), tag
        pos += 12 + n + 4
    assert pos == len(data)


def test_basename_must_contain_tfevents(tmp_path):
    src = tmp_path / "b.cpp"
    src.write_text('#include "tensorboard_logger.h"\nint main(int, char** argv) {\n'
                   '  try { TensorBoardLogger w(argv[1]); } catch (const std::runtime_error&) { return 3; }\n'
                   '  return 0;\n}\n')
    exe = tmp_path / "b"
    subprocess.check_call(["g++", "-std=c++17", "-I", os.path.join(ROOT, "ppo.cpp_amd", "apps"), str(src), "-o",
                           str(exe)])
    assert subprocess.call([str(exe), str(tmp_path / "scalars.pb")]) == 3
