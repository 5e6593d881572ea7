"""CPU tests of the C-ABI library: it loads, exports every declared symbol, and refuses to run
without a device (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import lego_amd as L
from lego_amd import _abi as A

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "lego_frontend.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s+(lego_[a-z0-9_]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ["lego_ctx_create", "lego_ctx_destroy", "lego_cloud_handler", "lego_feature_association",
                     "lego_feature_association_from", "lego_batch_create", "lego_batch_step", "lego_batch_read"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(A.LIB_FRONTEND)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_params_and_validation():
    p = L.params_vlp16()
    assert (p.num_vertical_scans, p.num_horizontal_scans, p.ground_scan_index) == (16, 1800, 7)
    assert p.segment_theta == 60.0 and p.mapping_frequency_divider == 5
    assert L.lib().lego_params_validate(C.byref(p)) == A.LEGO_OK
    p.fp_mode = 1  # double libm overloads (Indigo / Kinetic toolchains)
    assert L.lib().lego_params_validate(C.byref(p)) == A.LEGO_OK
    p.fp_mode = 2
    assert L.lib().lego_params_validate(C.byref(p)) == A.LEGO_EINVAL
    q = L.params_hdl64()
    assert (q.num_vertical_scans, q.num_horizontal_scans, q.ground_scan_index) == (64, 2048, 55)
    q.num_horizontal_scans = 4096
    assert L.lib().lego_params_validate(C.byref(q)) == A.LEGO_EINVAL


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors have the C header's sizes (compiled with the host C compiler)."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "lego_frontend.h"\nint main(void){printf("%zu %zu %zu %zu",'
                   'sizeof(lego_params), sizeof(lego_point), sizeof(lego_projection_out), sizeof(lego_association_out));'
                   'return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I" + os.path.join(REPO, "include"), str(src), "-o", str(exe)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert sizes == [C.sizeof(A.LegoParams), C.sizeof(A.LegoPoint), C.sizeof(A.LegoProjectionOut),
                     C.sizeof(A.LegoAssociationOut)]
    assert sizes[1] == 16  # pcl::PointXYZI payload


def test_no_cpu_fallback_without_device():
    """Creating a context on a machine without a HIP device must fail loudly (LEGO_EDEVICE)."""
    if L.device_count() > 0:
        pytest.skip("a HIP device is visible")
    h = C.c_void_p()
    p = L.params_vlp16()
    assert L.lib().lego_ctx_create(C.byref(p), 0, C.byref(h)) == A.LEGO_EDEVICE
    with pytest.raises(L.LegoError):
        L.Frontend(p)


def test_null_handles_are_rejected():
    """Entry points given no object fail with LEGO_EINVAL before touching a device (so also here)."""
    lib = L.lib()
    ms = C.c_float()
    assert lib.lego_batch_time_hbm_stages(None, 4, None, None, None, None, None, None, C.byref(ms)) == A.LEGO_EINVAL
    assert lib.lego_batch_stage_times(None, C.byref(ms)) == A.LEGO_EINVAL
    assert lib.lego_cloud_handler(None, None, 0, 16, 0, 4, 8, None) == A.LEGO_EINVAL
    assert lib.lego_feature_association(None, None) == A.LEGO_EINVAL


def test_synth_is_deterministic():
    cfg = A.synth_cfg("vlp16")
    a = A.synth_scan(cfg, 3, 5)
    b = A.synth_scan(cfg, 3, 5)
    assert a.shape[0] > 20000 and np.array_equal(a, b)
    pts, cnt = A.synth_batch(cfg, [3, 4], [5, 5], nthreads=2)
    assert cnt[0] == a.shape[0] and np.array_equal(pts[0, :cnt[0]], a)
    assert not np.array_equal(pts[1, :cnt[1]][:100], a[:100])


YAML_VLP16 = """\
lego_loam:
    # a VLP-16, as the reference's config/loam_config.yaml
    laser:
        num_vertical_scans: 16          # rings
        num_horizontal_scans: 1800
        ground_scan_index: 7
        vertical_angle_bottom: -15      # degrees
        vertical_angle_top: 15
        sensor_mount_angle: 0
        scan_period: 0.1
    imageProjection:
        segment_valid_point_num: 5
        segment_valid_line_num: 3
        segment_theta: 60.0
    featureAssociation:
        edge_threshold: 0.1
        surf_threshold: 0.1
        nearest_feature_search_distance: 5
    mapping:
        enable_loop_closure: false
        mapping_frequency_divider: 5
        surrounding_keyframe_search_radius: 50.0
"""


def test_params_from_yaml(tmp_path):
    """lego_params_load_yaml reads the reference's loam_config.yaml layout: the VLP-16 file gives
    lego_params_vlp16 exactly; an HDL-64E-like file and this build's own keys override; malformed
    files and values are rejected without touching the output."""
    f = tmp_path / "loam_config.yaml"
    f.write_text(YAML_VLP16)
    p, q = L.params_from_yaml(str(f)), L.params_vlp16()
    assert bytes(p) == bytes(q)
    f.write_text(YAML_VLP16.replace("num_vertical_scans: 16", "num_vertical_scans: 64")
                 .replace("num_horizontal_scans: 1800", "num_horizontal_scans: 2048")
                 .replace("ground_scan_index: 7", "ground_scan_index: 55")
                 .replace("vertical_angle_bottom: -15", "vertical_angle_bottom: -24.8")
                 .replace("vertical_angle_top: 15", "vertical_angle_top: 2.0")
                 + "    lego_amd:\n        fp_mode: 1\n        voxel_tie_order: 1\n")
    p = L.params_from_yaml(str(f))
    h = L.params_hdl64(fp_mode=1, voxel_tie_order=1)
    assert bytes(p) == bytes(h)
    for bad in (YAML_VLP16.replace("scan_period: 0.1", "scan_period: fast"),        # malformed value
                YAML_VLP16.replace("ground_scan_index: 7", "ground_scan_index: 99"),  # fails validation
                YAML_VLP16 + "  - a sequence item\n"):                               # not the file's YAML
        f.write_text(bad)
        out = L.params_vlp16(segment_theta=1.0)
        rc = L.lib().lego_params_load_yaml(os.fsencode(str(f)), C.byref(out))
        assert rc == A.LEGO_EINVAL and out.segment_theta == 1.0
    assert L.lib().lego_params_load_yaml(b"/nonexistent/loam_config.yaml", C.byref(out)) == A.LEGO_EINVAL
    ref = "/root/reference/LeGO-LOAM/config/loam_config.yaml"
    if os.path.exists(ref):  # the reference's own file (build container only)
        assert bytes(L.params_from_yaml(ref)) == bytes(L.params_vlp16())
