"""The C-ABI library loads and exports every entry point include/sfs2d.h declares (no compute)."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HDR = os.path.join(REPO, "include", "sfs2d.h")


def _declared():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(sfs2d_\w+)\s*\(", src, re.M)))


def _libpath():
    from sfs2d import _lib
    return os.path.abspath(_lib.LIB_PATH)


def test_header_matches_binding_list():
    from sfs2d import _lib
    assert _declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    path = _libpath()
    if not os.path.exists(path):
        subprocess.run(["make", "-C", os.path.dirname(path)], check=True)
    lib = ctypes.CDLL(path)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.sfs2d_abi_version() == 2


def test_no_device_is_reported_not_faked():
    """Without a GPU, creating a context fails loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sfs2d import _lib
    from sfs2d.engine import Engine
    with pytest.raises(_lib.Sfs2dError):
        Engine(0)


def test_window_record_layout():
    from sfs2d import _lib
    src = open(HDR).read()
    body = src[src.index("typedef struct {\n  uint32_t chrom;"):]
    body = body[:body.index("} sfs2d_window;")]
    names = re.findall(r"(\w+)(?:,|;)", body.replace("double t2d, t1d_p1, t1d_p2;", "t2d; t1d_p1; t1d_p2;"))
    assert _lib.WINDOW_DTYPE.itemsize == 64
    assert list(_lib.WINDOW_DTYPE.names)[:3] == ["chrom", "wid", "begin"]
