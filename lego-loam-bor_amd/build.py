"""Build the in-tree native libraries (no JIT cache: the .so files travel with the repo snapshot).

  liblego_frontend.so  product: HIP kernels for gfx950 + C-ABI (include/lego_frontend.h, include/lego_s2m.h)
  liblego_synth.so     synthetic VLP-16 / HDL-64E sweep generator (tests / bench input)

Usage: python lego-loam-bor_amd/build.py [--force]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lego_amd")
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("LEGO_OFFLOAD_ARCH", "gfx950")

FRONTEND_SRC = ["lego_kernels.hip", "lego_frontend.hip", "lego_s2m.hip", "lego_mapper.hip", "lego_config.cpp"]
FRONTEND_DEPS = FRONTEND_SRC + ["lego_device.h", "lego_libm.h", "lego_introsort.h", "lego_wavesort.h", "lego_kdtree.h"]
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=" + ARCH,
             # numerics contract: no FMA contraction, IEEE division/sqrt
             "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-Wno-unused-result", "-Wno-unused-value"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_frontend(force=False, profile=False):
    """One object per translation unit, compiled in parallel (no device code crosses a TU: each kernel is
    launched from the file that defines it), then one shared-library link."""
    target = os.path.join(OUT, "liblego_frontend_prof.so" if profile else "liblego_frontend.so")
    deps = [os.path.join(CSRC, f) for f in FRONTEND_DEPS] + [os.path.join(REPO, "include", h)
                                                          for h in ("lego_frontend.h", "lego_s2m.h")]
    if force or _stale(target, deps):
        import tempfile
        from concurrent.futures import ThreadPoolExecutor
        flags = [f for f in HIP_FLAGS if f != "-shared"] + (["-DLG_PROFILE"] if profile else [])
        with tempfile.TemporaryDirectory() as tmp:
            objs = [os.path.join(tmp, f + ".o") for f in FRONTEND_SRC]

            def compile_one(i):
                cmd = [HIPCC] + flags + ["-c", os.path.join(CSRC, FRONTEND_SRC[i]), "-o", objs[i]]
                print(" ".join(cmd), flush=True)
                subprocess.check_call(cmd)
            with ThreadPoolExecutor(max_workers=len(FRONTEND_SRC)) as ex:
                list(ex.map(compile_one, range(len(FRONTEND_SRC))))
            cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", target]
            print(" ".join(cmd), flush=True)
            subprocess.check_call(cmd)
        print("[build] %s: rebuilt for %s" % (os.path.relpath(target, REPO), ARCH), flush=True)
    else:
        print("[build] %s: up to date (newer than every source and header)" % os.path.relpath(target, REPO), flush=True)
    return target


def build_synth(force=False):
    target = os.path.join(OUT, "liblego_synth.so")
    src = os.path.join(CSRC, "synth.cpp")
    if force or _stale(target, [src]):
        cmd = ["g++", "-std=c++14", "-O3", "-fPIC", "-shared", "-fopenmp", src, "-o", target]
        print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return target


def build_all(force=False):
    """force (or LEGO_FORCE_BUILD=1): recompile even when the libraries are newer than their sources."""
    force = force or os.environ.get("LEGO_FORCE_BUILD") == "1"
    build_synth(force)
    build_frontend(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    if "--profile" in sys.argv:
        build_frontend(force=True, profile=True)
