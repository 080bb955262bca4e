"""Builds libdgs.so (hipcc, gfx950) and the diff_gaussian_sampling._C torch extension in-tree.

    python diff-gaussian-sampling_amd/build.py [--force] [--debug]

Outputs (git-ignored, shipped to the GPU box with the snapshot):
    diff-gaussian-sampling_amd/diff_gaussian_sampling/libdgs.so   HIP kernels + C ABI (include/dgs.h)
    diff-gaussian-sampling_amd/diff_gaussian_sampling/_C.so       pybind surface of ext.cpp:19-32
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
PKG = os.environ.get("DGS_PKG_OUT", os.path.join(HERE, "diff_gaussian_sampling"))  # variants: tools/variant.sh
INCLUDE = os.path.join(REPO, "include")
OBJ = os.environ.get("DGS_OBJ_OUT", os.path.join(HERE, "build"))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("DGS_OFFLOAD_ARCH", "gfx950")
LIB = os.path.join(PKG, "libdgs.so")
EXT = os.path.join(PKG, "_C.so")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError("build step failed: " + os.path.basename(cmd[-1]))
    return r


def build_lib(force=False, debug=False):
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    sources = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    os.makedirs(OBJ, exist_ok=True)
    flags = ["-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
             "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
    flags += ["-O1", "-g"] if debug else ["-O3"]
    flags += os.environ.get("DGS_EXTRA_CFLAGS", "").split()  # experiments / tuning builds
    objs = []
    jobs = []
    for src in sources:
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs.append([os.path.join(ROCM, "bin", "hipcc"), *flags, "-c", src, "-o", obj])
    if jobs:
        with cf.ThreadPoolExecutor(max_workers=min(len(jobs), 8)) as ex:
            list(ex.map(_run, jobs))
    if force or jobs or _newer(LIB, objs):
        _run([os.path.join(ROCM, "bin", "hipcc"), "-shared", f"--offload-arch={ARCH}", "-fPIC",
              *objs, "-o", LIB])
    return LIB


def build_ext(force=False):
    import torch
    import torch.utils.cpp_extension as ce

    src = os.path.join(CSRC, "torch_ext.cpp")
    if not (force or _newer(EXT, [src, LIB] + glob.glob(os.path.join(INCLUDE, "*.h")))):
        return EXT
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["c++", "-O2", "-std=c++17", "-fPIC", "-shared", src, "-o", EXT,
           "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
           "-I", INCLUDE, "-I", os.path.join(ROCM, "include"),
           "-isystem", sysconfig.get_paths()["include"]]
    for p in ce.include_paths():
        cmd += ["-isystem", p]
    cmd += ["-L", tlib, "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
            "-ltorch_hip", "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
            "-L", PKG, "-ldgs", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{tlib}"]
    _run(cmd)
    return EXT


def build(force=False, debug=False):
    build_lib(force=force, debug=debug)
    build_ext(force=force)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    build(force=a.force, debug=a.debug)
    print("built", LIB, EXT)
