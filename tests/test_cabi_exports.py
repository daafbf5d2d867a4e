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


def test_create_without_device_reports_enodev():
    """No CPU fallback: on a host without a GPU (or with a bad device index) every handle
    constructor fails with SDRGPU_ENODEV and a message."""
    import sdrpp_amd
    lib = sdrpp_amd.lib
    h = ctypes.c_void_p()
    bad = lib.sdrgpu_device_count()          # first index past the last device
    assert lib.sdrgpu_rxvfo_create(ctypes.byref(h), bad, 61.44e6, 240e3, 200e3, 0.0) == -5
    assert b"not available" in lib.sdrgpu_last_error()
    assert lib.sdrgpu_fft_create(ctypes.byref(h), bad, 1024, 1024, 6) == -5
    assert lib.sdrgpu_wfm_create(ctypes.byref(h), -1, 100e3, 240e3, 1) == -5
