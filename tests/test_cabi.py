"""C-ABI checks that need no GPU: libdgs.so loads, exports every function include/dgs.h
declares, and its host-only entry points (version, errors, workspace sizing, argument
validation that fails before any device work) behave as documented."""
import ctypes
import os
import re

import pytest

from conftest import PKG_ROOT, REPO

HEADER = os.path.join(REPO, "include", "dgs.h")
HEADERS = sorted(os.path.join(REPO, "include", f) for f in os.listdir(os.path.join(REPO, "include"))
                 if f.endswith(".h"))
LIB = os.path.join(PKG_ROOT, "diff_gaussian_sampling", "libdgs.so")
DGS_ERR_ARG, DGS_ERR_BUFFER = 1, 4


def declared_functions():
    text = "\n".join(open(h).read() for h in HEADERS)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(dgs_[a-z_0-9]+)\s*\(", text, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail("libdgs.so is not built (python diff-gaussian-sampling_amd/build.py)")
    return ctypes.CDLL(LIB)


def test_header_declares_the_entry_points():
    names = declared_functions()
    for n in ["dgs_last_error", "dgs_version", "dgs_tile_grid", "dgs_preprocess",
              "dgs_sample_workspace_size", "dgs_sample_forward", "dgs_sample_backward",
              "dgs_count_pairs", "dgs_timing_enable", "dgs_timing_read", "dgs_volume_preprocess",
              "dgs_volume_forward", "dgs_volume_backward", "dgs_volume_workspace_size"]:
        assert n in names, n


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_header_compiles_as_c(tmp_path):
    """include/dgs.h is plain C (no C++ or torch types)."""
    src = tmp_path / "t.c"
    src.write_text('#include "dgs.h"\n#include "dgs_volume.h"\n'
                   'int main(void) { return dgs_version() > 0 ? 0 : 1; }\n')
    import subprocess
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.dirname(HEADER),
                        "-c", str(src), "-o", str(tmp_path / "t.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_version_and_error_string(lib):
    lib.dgs_version.restype = ctypes.c_int
    assert lib.dgs_version() >= 1
    lib.dgs_last_error.restype = ctypes.c_char_p
    assert isinstance(lib.dgs_last_error(), bytes)


def test_workspace_sizes_grow_with_problem(lib):
    f = lib.dgs_sample_workspace_size
    f.restype = ctypes.c_size_t
    f.argtypes = [ctypes.c_int] * 6
    small = f(0, 1000, 2, 4000, 1, 0)
    big = f(0, 100000, 2, 400000, 1, 0)
    assert 0 < small < big
    assert f(3, 1000, 2, 4000, 16, 1) > f(0, 1000, 2, 4000, 1, 1)


def test_argument_errors_fail_before_device_work(lib):
    lib.dgs_last_error.restype = ctypes.c_char_p
    fwd = lib.dgs_sample_forward
    fwd.restype = ctypes.c_int
    P = ctypes.c_void_p
    fwd.argtypes = [ctypes.c_int] * 5 + [P] * 5 + [ctypes.c_size_t, P, ctypes.c_size_t, P, P,
                                                   ctypes.c_size_t, P, ctypes.c_int]
    # unknown function
    assert fwd(7, 10, 2, 10, 1, None, None, None, None, None, 0, None, 0, None, None, 0, None, 0) == DGS_ERR_ARG
    assert b"function" in lib.dgs_last_error()
    # D = 3 (the reference leaves it undefined)
    assert fwd(0, 10, 3, 10, 1, None, None, None, None, None, 0, None, 0, None, None, 0, None, 0) == DGS_ERR_ARG
    # missing binning buffers
    assert fwd(0, 10, 2, 10, 1, None, None, None, None, None, 0, None, 0, None, None, 1 << 20, None, 0) == DGS_ERR_BUFFER
    # empty problem: nothing to do
    assert fwd(0, 0, 2, 10, 1, None, None, None, None, None, 0, None, 0, None, None, 0, None, 0) == 0
    pre = lib.dgs_preprocess
    pre.restype = ctypes.c_int
    assert pre(10, 3, 10, None, None, None, None, None, None, None, None, None, None, None, 0) == DGS_ERR_ARG


def test_timing_read_without_records(lib):
    lib.dgs_timing_read.restype = ctypes.c_int
    ms = ctypes.c_double(0)
    assert lib.dgs_timing_read(0, ctypes.byref(ms)) == 0 and ms.value == 0.0
    assert lib.dgs_timing_read(5, ctypes.byref(ms)) < 0


def test_volume_host_validation(lib):
    """dgs_volume_*: workspace sizing and argument errors before any device work."""
    ws = lib.dgs_volume_workspace_size
    ws.restype = ctypes.c_size_t
    ws.argtypes = [ctypes.c_int] * 5
    assert ws(0, 10, 100, 1, 0) == 0
    assert ws(3, 10, 100, 2, 1) == 100 * 10 * 2 * 4  # hs[N][10 unique components][C]
    f = lib.dgs_volume_forward
    f.restype = ctypes.c_int
    assert f(7, 1, 1, 1, None, None, None, None, None, ctypes.c_size_t(0), None, None, 0) == DGS_ERR_ARG
    assert f(0, 1, 1, 1, None, None, None, None, None, ctypes.c_size_t(0), None, None, 0) == DGS_ERR_BUFFER
    p = lib.dgs_volume_preprocess
    p.restype = ctypes.c_int
    assert p(-1, 1, None, None, None, None, None, None, 0) == DGS_ERR_ARG


class BinOptions(ctypes.Structure):
    """dgs_bin_options (include/dgs.h, ABI 12)."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("flags", ctypes.c_uint32), ("present", ctypes.c_void_p),
                ("sample_area", ctypes.c_double), ("capacity_E", ctypes.c_int64), ("capacity_Es", ctypes.c_int64),
                ("capacity_R", ctypes.c_int64), ("num_rendered_device", ctypes.c_void_p),
                ("status_device", ctypes.c_void_p), ("samples_binned", ctypes.c_void_p),
                ("samples_binned_bytes", ctypes.c_size_t)]


def test_bin_options_layout_and_validation(lib, tmp_path):
    """dgs_bin_options as C lays it out, and the option checks of dgs_preprocess_ex /
    dgs_preprocess_auto_ex (ABI 12: samples_binned, DGS_BIN_SAMPLES_FIXED), all before any device
    work: a struct of another size, flags on the auto form, samples_binned with the capturable form
    but without DGS_BIN_SAMPLES_FIXED."""
    import subprocess
    src = tmp_path / "s.c"
    src.write_text('#include <stdio.h>\n#include "dgs.h"\n'
                   'int main(void) { printf("%zu %d %d\\n", sizeof(dgs_bin_options), DGS_ABI_VERSION, '
                   'DGS_BIN_SAMPLES_FIXED); return 0; }\n')
    exe = tmp_path / "s"
    r = subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    size, abi, fixed = map(int, subprocess.run([str(exe)], capture_output=True, text=True).stdout.split())
    assert size == ctypes.sizeof(BinOptions) and fixed == 2
    lib.dgs_version.restype = ctypes.c_int
    assert lib.dgs_version() == abi == 12
    lib.dgs_last_error.restype = ctypes.c_char_p
    alloc_t = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t)
    alloc = alloc_t(lambda ctx, which, nbytes: None)  # (never reached)
    nr = ctypes.c_int64(0)
    grid = (ctypes.c_int * 2)()
    off = (ctypes.c_float * 2)()
    auto = lib.dgs_preprocess_auto_ex
    auto.restype = ctypes.c_int
    P = ctypes.c_void_p
    auto.argtypes = [ctypes.c_int] * 3 + [P] * 4 + [ctypes.POINTER(BinOptions), P, alloc_t, P, P, P, P, P, ctypes.c_int]
    o = BinOptions()
    o.struct_size = ctypes.sizeof(BinOptions) - 8
    args = lambda opts: (10, 2, 10, None, None, None, None, ctypes.byref(opts), None, alloc, None,  # noqa: E731
                         ctypes.byref(nr), grid, off, None, 0)
    assert auto(*args(o)) == DGS_ERR_ARG and b"struct_size" in lib.dgs_last_error()
    o.struct_size = ctypes.sizeof(BinOptions)
    o.flags = 1
    assert auto(*args(o)) == DGS_ERR_ARG and b"flags" in lib.dgs_last_error()
    ex = lib.dgs_preprocess_ex
    ex.restype = ctypes.c_int
    ex.argtypes = [ctypes.c_int] * 3 + [P] * 6 + [ctypes.POINTER(BinOptions), P, alloc_t, P, P, P, ctypes.c_int]
    o.flags = 0
    o.capacity_E, o.capacity_Es, o.capacity_R = 100, 10, 100
    o.samples_binned, o.samples_binned_bytes = 4096, 4096
    assert ex(10, 2, 10, None, None, None, None, grid, off, ctypes.byref(o), None, alloc, None,
              ctypes.byref(nr), None, 0) == DGS_ERR_ARG
    assert b"DGS_BIN_SAMPLES_FIXED" in lib.dgs_last_error()
    o.flags = 4
    assert ex(10, 2, 10, None, None, None, None, grid, off, ctypes.byref(o), None, alloc, None,
              ctypes.byref(nr), None, 0) == DGS_ERR_ARG and b"flags" in lib.dgs_last_error()
    lib.dgs_sample_reuse_count.restype = ctypes.c_int64
    assert lib.dgs_sample_reuse_count() >= 0
