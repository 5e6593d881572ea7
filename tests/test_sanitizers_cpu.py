"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the host code, CPU only:

* the CPU oracle and the synthetic-sweep generator (tests/native/sanitize_oracle.cpp drives them over
  VLP-16 / HDL-64E sequences in both libm models and both VoxelGrid tie orders, edge clouds, the
  VoxelGrid and scan-to-map);
* the ROS bag v2 reader (include/lego_rosbag.hpp, via examples/bag_tool.cpp), which parses untrusted
  bytes: the writer round trip, then a corpus of truncated and byte-garbled bags that must each either
  decode or fail loudly (exit 1), never trip a sanitizer;
* the config loader (lego-loam-bor_amd/csrc/lego_config.cpp) on garbled YAML.

GPU code is never built with sanitizers here (the pool refuses GPU ASan); the product library is
linked unsanitized where a tool needs it.
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1"]
# ASan must not insist on being first in the library list (this harness preloads a library of its own);
# exit codes 86 / 87 tell a sanitizer report from the tools' own failure status.
ENV = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0:exitcode=86:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:exitcode=87:print_stacktrace=1")
LIBDIR = os.path.join(REPO, "lego-loam-bor_amd", "lego_amd")


def _gxx(args, out):
    subprocess.check_call(["g++", "-std=c++14"] + SAN + args + ["-o", out])


def test_oracle_and_synth_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "so")
    _gxx(["-ffp-contract=off", "-fopenmp", os.path.join(REPO, "tests", "native", "sanitize_oracle.cpp"),
          os.path.join(REPO, "oracle", "lego_oracle.cpp"), os.path.join(REPO, "oracle", "s2m_oracle.cpp"),
          os.path.join(REPO, "lego-loam-bor_amd", "csrc", "synth.cpp")], exe)
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True, env=ENV,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "sanitized oracle run: ok" in r.stdout


def _mutants(raw, rng, n):
    """Truncations at spread-out lengths and random byte / length-field corruptions of a valid bag."""
    out = [raw[:k] for k in sorted(set(np.linspace(0, len(raw) - 1, 24).astype(int).tolist()))]
    for _ in range(n):
        b = bytearray(raw)
        for _ in range(int(rng.integers(1, 6))):
            i = int(rng.integers(13, len(b)))  # keep the magic line, so the parser goes past it
            b[i] = int(rng.integers(0, 256)) if rng.random() < 0.7 else 0xFF
        out.append(bytes(b))
    return out


def test_rosbag_reader_under_asan_ubsan(tmp_path):
    import test_rosbag_cpu as RB
    exe = str(tmp_path / "bag_tool")
    _gxx(["-I" + os.path.join(REPO, "include"), os.path.join(REPO, "examples", "bag_tool.cpp"), "-L" + LIBDIR,
          "-llego_frontend", "-Wl,-rpath," + LIBDIR, "-pthread", "-ldl"], exe)
    scans = RB._sweeps(2)
    RB.write_scans(str(tmp_path / "s.bin"), scans)
    assert subprocess.call([exe, "write", str(tmp_path / "s.bin"), str(tmp_path / "o.bag")], env=ENV) == 0
    assert subprocess.call([exe, "dump", str(tmp_path / "o.bag"), str(tmp_path / "d.bin")], env=ENV) == 0
    rng = np.random.default_rng(5)
    corpus = []
    for comp in ("none", "bz2"):
        RB.py_bag(str(tmp_path / ("p_%s.bag" % comp)), [s[:300] for s in scans], comp)
        corpus += _mutants((tmp_path / ("p_%s.bag" % comp)).read_bytes(), rng, 60)
    corpus += _mutants((tmp_path / "o.bag").read_bytes(), rng, 60)
    codes = {}
    for i, data in enumerate(corpus):
        f = tmp_path / ("m%d.bag" % i)
        f.write_bytes(data)
        r = subprocess.run([exe, "dump", str(f), str(tmp_path / "m.bin")], stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, universal_newlines=True, env=ENV, timeout=60)
        assert r.returncode in (0, 1), (i, r.returncode, r.stdout[-3000:])
        codes[r.returncode] = codes.get(r.returncode, 0) + 1
    assert codes.get(1, 0) > len(corpus) // 4  # most mutants are rejected loudly


def test_config_loader_under_asan_ubsan(tmp_path):
    src = tmp_path / "cfg_main.cpp"
    src.write_text('#include <cstdio>\n#include "lego_frontend.h"\n'
                   'extern "C" void lego_params_vlp16(lego_params* p) { *p = lego_params(); p->num_vertical_scans = 16; }\n'
                   'extern "C" int lego_params_validate(const lego_params* p) { return p->num_vertical_scans > 1 ? 0 : -1; }\n'
                   'int main(int c, char** v) { lego_params p = {}; p.num_vertical_scans = 16;\n'
                   '  for (int i = 1; i < c; ++i) printf("%d\\n", lego_params_load_yaml(v[i], &p)); return 0; }\n')
    exe = str(tmp_path / "cfg")
    _gxx(["-I" + os.path.join(REPO, "include"), str(src), os.path.join(REPO, "lego-loam-bor_amd", "csrc", "lego_config.cpp")],
         exe)
    import test_abi_cpu as T
    rng = np.random.default_rng(9)
    base = T.YAML_VLP16.encode()
    files = []
    for i, data in enumerate(_mutants(base, rng, 80) + [b"", b"\t\t:", b"a:" * 3000, b"x" * 9000, b"k: " + b"9" * 400]):
        f = tmp_path / ("c%d.yaml" % i)
        f.write_bytes(data)
        files.append(str(f))
    r = subprocess.run([exe] + files, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True,
                       env=ENV, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
