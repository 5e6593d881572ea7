"""ROS bag v2.0 input path (include/lego_rosbag.hpp): bags written by the C++
writer and by an independent Python writer (stdlib only, with bz2-compressed chunks) decode back to
the exact sweeps, and malformed bags fail loudly.  CPU only; the GPU replay is in test_cpp_mirror.py."""
import bz2
import os
import struct
import subprocess

import numpy as np
import pytest

from lego_amd import _abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "examples", "bag_tool")


def build():
    from conftest import make_example
    make_example("bag_tool")


def write_scans(path, scans):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(scans)))
        for p in scans:
            p = np.ascontiguousarray(p, dtype=np.float32)
            f.write(struct.pack("<i", p.shape[0]))
            f.write(p.tobytes())


def read_scans(path):
    out = []
    with open(path, "rb") as f:
        (n,) = struct.unpack("<i", f.read(4))
        for _ in range(n):
            (k,) = struct.unpack("<i", f.read(4))
            out.append(np.frombuffer(f.read(16 * k), dtype=np.float32).reshape(k, 4))
    return out


# ---- an independent writer of the bag format (rosbag's record layout) ------------------------
def _field(name, value):
    body = name.encode() + b"=" + value
    return struct.pack("<I", len(body)) + body


def _record(header, data):
    return struct.pack("<I", len(header)) + header + struct.pack("<I", len(data)) + data


def _pc2(seq, sec, nsec, pts, extra_field):
    """sensor_msgs/PointCloud2 with float32 x, y, z (+ an unused uint16 ring field), 22-byte points."""
    fields = [("x", 0, 7), ("y", 4, 7), ("z", 8, 7), ("intensity", 12, 7)]
    step = 16
    if extra_field:
        fields.append(("ring", 16, 4))  # UINT16
        step = 22
    m = struct.pack("<III", seq, sec, nsec) + struct.pack("<I", 8) + b"velodyne"
    m += struct.pack("<II", 1, len(pts)) + struct.pack("<I", len(fields))
    for name, off, dt in fields:
        m += struct.pack("<I", len(name)) + name.encode() + struct.pack("<IBI", off, dt, 1)
    body = bytearray()
    for p in pts:
        body += struct.pack("<4f", *p) + (b"\x07\x00" + b"\x00" * 4 if extra_field else b"")
    m += struct.pack("<B", 0) + struct.pack("<II", step, step * len(pts)) + struct.pack("<I", len(body)) + bytes(body)
    return m + b"\x01"


def py_bag(path, scans, compression, topic="/velodyne_points"):
    conn_hdr = _field("op", b"\x07") + _field("conn", struct.pack("<I", 0)) + _field("topic", topic.encode())
    conn_data = _field("topic", topic.encode()) + _field("type", b"sensor_msgs/PointCloud2") + \
        _field("md5sum", b"1158d486dd51d683ce2f1be655c3c181")
    conn = _record(conn_hdr, conn_data)
    other = _record(_field("op", b"\x07") + _field("conn", struct.pack("<I", 1)) + _field("topic", b"/imu"),
                    _field("type", b"sensor_msgs/Imu"))
    chunk = conn + other
    for i, p in enumerate(scans):
        t = struct.pack("<II", 7 + i // 10, (i % 10) * 100000000)
        chunk += _record(_field("op", b"\x02") + _field("conn", struct.pack("<I", 0)) + _field("time", t),
                         _pc2(i, 7 + i // 10, (i % 10) * 100000000, p, extra_field=(i % 2 == 1)))
        chunk += _record(_field("op", b"\x02") + _field("conn", struct.pack("<I", 1)) + _field("time", t), b"\x00" * 12)
    data = bz2.compress(chunk) if compression == "bz2" else chunk
    ch = _record(_field("op", b"\x05") + _field("compression", compression.encode()) +
                 _field("size", struct.pack("<I", len(chunk))), data)
    hdr = _field("op", b"\x03") + _field("index_pos", struct.pack("<Q", 0)) + \
        _field("conn_count", struct.pack("<I", 2)) + _field("chunk_count", struct.pack("<I", 1))
    bag_header = _record(hdr, b" " * (4096 - 8 - len(hdr)))
    with open(path, "wb") as f:
        f.write(b"#ROSBAG V2.0\n" + bag_header + ch)


def _sweeps(n):
    cfg = A.synth_cfg("vlp16")
    return [A.synth_scan(cfg, 2, k)[:4000] for k in range(n)]


def test_cpp_writer_round_trip(tmp_path):
    build()
    scans = _sweeps(3)
    write_scans(str(tmp_path / "s.bin"), scans)
    r = subprocess.run([TOOL, "write", str(tmp_path / "s.bin"), str(tmp_path / "o.bag")], stdout=subprocess.PIPE,
                       universal_newlines=True)
    assert r.returncode == 0, r.stdout
    info = subprocess.run([TOOL, "info", str(tmp_path / "o.bag")], stdout=subprocess.PIPE, universal_newlines=True)
    assert "topic /velodyne_points type sensor_msgs/PointCloud2 messages 3" in info.stdout
    assert subprocess.call([TOOL, "dump", str(tmp_path / "o.bag"), str(tmp_path / "d.bin")]) == 0
    back = read_scans(str(tmp_path / "d.bin"))
    assert len(back) == 3
    for a, b in zip(scans, back):
        np.testing.assert_array_equal(a[:, :3], b[:, :3])


@pytest.mark.parametrize("compression", ["none", "bz2"])
def test_independent_writer_decodes(tmp_path, compression):
    """Another topic interleaved, a second field layout (22-byte points with a ring field), chunk
    compression none / bz2 (inflated with the system libbz2)."""
    build()
    scans = _sweeps(4)
    py_bag(str(tmp_path / "p.bag"), [s[:500] for s in scans], compression)
    info = subprocess.run([TOOL, "info", str(tmp_path / "p.bag")], stdout=subprocess.PIPE, universal_newlines=True)
    assert info.returncode == 0
    assert "topic /imu type sensor_msgs/Imu messages 4" in info.stdout
    assert "points 500 500 500 500" in info.stdout
    assert subprocess.call([TOOL, "dump", str(tmp_path / "p.bag"), str(tmp_path / "d.bin")]) == 0
    for a, b in zip(scans, read_scans(str(tmp_path / "d.bin"))):
        np.testing.assert_array_equal(a[:500, :3], b[:, :3])


def test_malformed_bags_fail_loudly(tmp_path):
    build()
    (tmp_path / "x.bag").write_bytes(b"#ROSBAG V1.2\n" + b"\x00" * 64)
    assert subprocess.call([TOOL, "info", str(tmp_path / "x.bag")], stderr=subprocess.DEVNULL) == 1
    py_bag(str(tmp_path / "t.bag"), [s[:100] for s in _sweeps(1)], "none")
    raw = (tmp_path / "t.bag").read_bytes()
    (tmp_path / "t2.bag").write_bytes(raw[:-50])  # truncated chunk
    assert subprocess.call([TOOL, "info", str(tmp_path / "t2.bag")], stderr=subprocess.DEVNULL) == 1
