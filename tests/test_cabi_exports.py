"""The C-ABI library loads and exports every function declared in include/sdrgpu.h
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "sdrgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sdrgpu_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    lib = ctypes.CDLL(os.path.join(ROOT, "sdrpp_amd", "lib", "libsdrgpu.so"))
    names = declared()
    assert len(names) >= 45
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_host_only_entry_points_work_without_gpu():
    from sdrpp_amd import lib
    assert lib.sdrgpu_version() == 100
    assert lib.sdrgpu_taps_estimate_count(912000.0, 61.44e6) == 256
    # bad arguments fail loudly with a message, not silently
    assert lib.sdrgpu_create_window(99, None, 10, 1) < 0
    assert b"create_window" in lib.sdrgpu_last_error()
