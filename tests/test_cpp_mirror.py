"""The C++ mirror (include/lego_loam_amd.hpp: Channel / ImageProjection / FeatureAssociation over the
C-ABI) builds, refuses to run without a device, and on the GPU reproduces the oracle's odometry
through the reference's two-thread Channel topology (examples/replay_pipeline.cpp)."""
import os
import struct
import subprocess

import numpy as np
import pytest

import helpers as Hs
from conftest import make_example
from lego_amd import _abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "examples", "replay_pipeline")


def build():
    make_example("replay_pipeline")


def write_scans(path, scans):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(scans)))
        for p in scans:
            p = np.ascontiguousarray(p, dtype=np.float32)
            f.write(struct.pack("<i", p.shape[0]))
            f.write(p.tobytes())


def test_mirror_message_helpers(tmp_path):
    """The mirror's helpers between a ROS message and the C-ABI, which ros/lego_nodes.cpp uses as they are
    (xyz_offsets, packed_rows, fill_cloud_info, projection_in, FeatureAssociationCycle): CPU checks."""
    exe = str(tmp_path / "mirror_check")
    lib = os.path.join(REPO, "lego-loam-bor_amd", "lego_amd")
    subprocess.check_call(["g++", "-std=c++14", "-O2", "-Wall", "-Werror", "-I" + os.path.join(REPO, "include"),
                           os.path.join(REPO, "tests", "native", "mirror_check.cpp"), "-o", exe, "-L" + lib,
                           "-llego_frontend", "-Wl,-rpath," + lib, "-pthread"])
    r = subprocess.run([exe], stdout=subprocess.PIPE, universal_newlines=True)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout


def test_mirror_builds_and_fails_loudly_without_device(tmp_path):
    build()
    import lego_amd
    if lego_amd.device_count() > 0:
        pytest.skip("a HIP device is visible")
    f = tmp_path / "s.bin"
    write_scans(str(f), [A.synth_scan(A.synth_cfg("vlp16"), 0, 0)])
    r = subprocess.run([EXE, str(f)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True)
    assert r.returncode == 1 and "rc=-3" in r.stderr


@pytest.mark.gpu
def test_mirror_pipeline_matches_oracle(gpu, tmp_path):
    import oracle as O
    import make_golden as MG
    build()
    cfg = A.synth_cfg("vlp16")
    scans = [A.synth_scan(cfg, 12, k) for k in range(7)]
    f = tmp_path / "s.bin"
    write_scans(str(f), scans)
    r = subprocess.run([EXE, str(f), "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    tok = r.stdout.split()
    cycles = int(tok[1])
    pos = np.array([float(x) for x in tok[5:8]])
    quat = np.array([float(x) for x in tok[9:13]])
    orc = O.Oracle(MG.params_for("vlp16"))
    n_last = n_emit = 0
    frame_count = 1  # publishCloudsLast's skip counter (featureAssociation.cpp:132, :1362-1382)
    for p in scans:
        orc.cloud_handler(p)
        fa = orc.feature_association()
        if fa["status"] & A.ST_INIT:
            continue
        frame_count += 1
        if frame_count >= 2:
            frame_count = 0
            n_last += 1
        n_emit += bool(fa["status"] & A.ST_EMITTED)
    assert cycles == len(scans)
    np.testing.assert_allclose(pos, fa["odom_position"], atol=Hs.TF_TOL, rtol=0)
    np.testing.assert_allclose(quat, fa["odom_orientation"], atol=Hs.TF_TOL, rtol=0)
    # run_feature_association's publication decisions (shared with ros/lego_nodes.cpp)
    assert tok[13] == "last" and int(tok[14]) == n_last and tok[15] == "emitted" and int(tok[16]) == n_emit, tok
    assert n_emit >= 1 and n_last >= 3


@pytest.mark.gpu
def test_rosbag_replay_equals_direct_replay(gpu, tmp_path):
    """The same sweeps replayed from a ROS bag (PointCloud2 decoded zero-copy, lego_rosbag.hpp) and from
    a plain file give the identical odometry line."""
    build()
    make_example("bag_tool")
    cfg = A.synth_cfg("vlp16")
    scans = [A.synth_scan(cfg, 5, k) for k in range(5)]
    f = tmp_path / "s.bin"
    write_scans(str(f), scans)
    bag = tmp_path / "s.bag"
    subprocess.check_call([os.path.join(REPO, "examples", "bag_tool"), "write", str(f), str(bag)],
                          stdout=subprocess.DEVNULL)
    outs = []
    for src in (f, bag):
        r = subprocess.run([EXE, str(src), "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           universal_newlines=True, timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.strip())
    assert outs[0] == outs[1]
    assert outs[0].startswith("cycles 5 ")


S2M_EXE = os.path.join(REPO, "examples", "scan2map")


def _write_problem(path, pr):
    with open(path, "wb") as f:
        for name in ("corner", "surf", "corner_map", "surf_map"):
            a = np.ascontiguousarray(pr[name], dtype=np.float32).reshape(-1, 4)
            f.write(struct.pack("<i", a.shape[0]))
            f.write(a.tobytes())
        f.write(np.asarray(pr["transform"], np.float32).tobytes())


def _problem():
    import oracle as O
    import make_golden as MG
    from lego_amd import mapping as M
    orc = O.Oracle(MG.params_for("vlp16"))
    cfg = A.synth_cfg("vlp16")
    frames = []
    for k in range(5):
        orc.cloud_handler(A.synth_scan(cfg, 13, k))
        frames.append(orc.feature_association())
    return M.build_problem(frames, 4)


def test_scan2map_mirror_fails_loudly_without_device(tmp_path):
    make_example("scan2map")
    import lego_amd
    if lego_amd.device_count() > 0:
        pytest.skip("a HIP device is visible")
    f = tmp_path / "p.bin"
    _write_problem(str(f), _problem())
    r = subprocess.run([S2M_EXE, str(f)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True)
    assert r.returncode == 1 and "rc=-3" in r.stderr


@pytest.mark.gpu
def test_scan2map_mirror_matches_oracle(gpu, tmp_path):
    """ScanToMapOptimization (the C++ mirror of MapOptimization's LM members and scan2MapOptimization)
    reproduces the oracle's optimised transformTobeMapped."""
    import oracle as O
    make_example("scan2map")
    pr = _problem()
    f = tmp_path / "p.bin"
    _write_problem(str(f), pr)
    r = subprocess.run([S2M_EXE, str(f), "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    tok = r.stdout.split()
    t = np.array([float(x) for x in tok[1:7]], np.float32)
    t_ref, dg_ref, info_ref = O.scan2map(pr["corner"], pr["surf"], pr["corner_map"], pr["surf_map"], pr["transform"])
    np.testing.assert_allclose(t, t_ref, atol=Hs.TF_TOL, rtol=0)
    assert int(tok[8]) == dg_ref and int(tok[10]) == info_ref[0] and int(tok[12]) == info_ref[1]


MAP_EXE = os.path.join(REPO, "examples", "mapping")


def _write_cycles(path, assocs):
    with open(path, "wb") as f:
        f.write(struct.pack("<i", len(assocs)))
        for a in assocs:
            for name in ("corner_last", "surf_last", "outlier_last"):
                x = np.ascontiguousarray(a[name], dtype=np.float32).reshape(-1, 4)
                f.write(struct.pack("<i", x.shape[0]))
                f.write(x.tobytes())
            f.write(np.asarray(a["odom_orientation"], np.float64).tobytes())
            f.write(np.asarray(a["odom_position"], np.float64).tobytes())


def test_mapping_mirror_fails_loudly_without_device(tmp_path):
    make_example("mapping")
    import lego_amd
    if lego_amd.device_count() > 0:
        pytest.skip("a HIP device is visible")
    f = tmp_path / "c.bin"
    _write_cycles(str(f), [])
    r = subprocess.run([MAP_EXE, str(f)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True)
    assert r.returncode == 1 and "rc=-3" in r.stderr


@pytest.mark.gpu
def test_mapping_mirror_matches_oracle_loop(gpu, tmp_path):
    """MapOptimization (the C++ mirror of the mapping thread) reproduces the oracle loop's
    transformAftMapped every cycle and its key-frame count."""
    from lego_amd import mapping as M
    from test_gpu_mapping_loop import _emitted, mapping_step_oracle
    make_example("mapping")
    assocs = _emitted(6, 26)
    f = tmp_path / "c.bin"
    _write_cycles(str(f), assocs)
    r = subprocess.run([MAP_EXE, str(f), "0"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, universal_newlines=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == len(assocs) + 1
    import oracle as O
    sq = M.MapSequence(associate=O.associate_to_map, odometry=O.odometry_to_transform)
    for a, line in zip(assocs, lines):
        (_, _, info), = mapping_step_oracle([sq], [a])
        tok = line.split()
        np.testing.assert_allclose(np.array([float(x) for x in tok[1:7]], np.float32), sq.t_aft, atol=1e-4, rtol=0)
        assert int(tok[8]) == int(info[0] == 1) and int(tok[10]) == info[1]
    assert lines[-1] == "keys %d" % len(sq.key_pose6)


@pytest.mark.gpu
def test_pipeline_with_mapping_thread_matches_oracle(gpu, tmp_path):
    """main.cpp's topology with the mapping thread (replay_pipeline --mapping: ImageProjection ->
    FeatureAssociation thread -> blocking Channel<AssociationOut> -> MapOptimization thread) against the
    oracle front end and the oracle mapping loop on the same sweeps: every emitted AssociationOut is
    mapped, the same key frames, and the last /aft_mapped_to_init within 1e-4."""
    import oracle as O
    import make_golden as MG
    from lego_amd import mapping as M
    from test_gpu_mapping_loop import mapping_step_oracle
    build()
    cfg = A.synth_cfg("vlp16")
    scans = [A.synth_scan(cfg, 6, k) for k in range(26)]
    f = tmp_path / "s.bin"
    write_scans(str(f), scans)
    r = subprocess.run([EXE, str(f), "0", "--mapping"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       universal_newlines=True, timeout=300)
    assert r.returncode == 0, r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("mapping ")][0].split()
    orc = O.Oracle(MG.params_for("vlp16"))
    sq = M.MapSequence(associate=O.associate_to_map, odometry=O.odometry_to_transform)
    emitted = 0
    for p in scans:
        orc.cloud_handler(p)
        a = orc.feature_association()
        if a["status"] & 0x080:
            mapping_step_oracle([sq], [a])
            emitted += 1
    assert emitted >= 4 and int(line[2]) == emitted and int(line[4]) == len(sq.key_pose6)
    np.testing.assert_allclose(np.array([float(x) for x in line[6:9]]), sq.t_aft[3:6], atol=1e-4, rtol=0)
