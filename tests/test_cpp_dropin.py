"""The C++ drop-in blocks (sdrpp_amd/dsp/gpu, reference class names) compile against the
block-API mirror and, on a GPU, reproduce the oracle inside the threaded stream model."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "test_dropin")
FE_BIN = os.path.join(ROOT, "build", "test_iq_frontend")


def _build(pinned=False):
    """pinned: built with SDRGPU_PIN_STREAMS, so every dsp::stream buffer is registered with
    sdrgpu_host_register and the blocks DMA straight from / into the stream buffers."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    binp = BIN + ("_pinned" if pinned else "")
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread"] + (["-DSDRGPU_PIN_STREAMS"] if pinned else []) + [
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "gpu"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime", "dsp", "buffer"),   # resolves "../processor.h"
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
           os.path.join(ROOT, "tests", "cpp", "test_dropin.cpp"),
           "-L", os.path.join(ROOT, "sdrpp_amd", "lib"), "-lsdrgpu",
           "-L", os.path.join(ROOT, "oracle"), "-lsdr_oracle",
           "-Wl,-rpath," + os.path.join(ROOT, "sdrpp_amd", "lib") + ":" + os.path.join(ROOT, "oracle"),
           "-o", binp]
    subprocess.check_call(cmd)
    return binp


@pytest.mark.parametrize("pinned", [False, True])
def test_dropin_compiles(pinned):
    assert os.path.exists(_build(pinned))


@pytest.mark.gpu
@pytest.mark.parametrize("pinned", [False, True])
def test_dropin_runs_on_gpu(pinned):
    b = _build(pinned)
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout


def _build_frontend():
    """The IQFrontEnd drop-in (sdrpp_amd/dsp/gpu/signal_path/iq_frontend.h): its "../dsp/..."
    includes resolve against the block-API mirror through -I runtime/dsp (in the SDR++ tree they
    are the reference's own headers)."""
    os.makedirs(os.path.dirname(FE_BIN), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread",
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "gpu"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime", "dsp"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime", "dsp", "buffer"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
           os.path.join(ROOT, "tests", "cpp", "test_iq_frontend.cpp"),
           "-L", os.path.join(ROOT, "sdrpp_amd", "lib"), "-lsdrgpu",
           "-L", os.path.join(ROOT, "oracle"), "-lsdr_oracle",
           "-Wl,-rpath," + os.path.join(ROOT, "sdrpp_amd", "lib") + ":" + os.path.join(ROOT, "oracle"), "-o", FE_BIN]
    subprocess.check_call(cmd)
    return FE_BIN


def test_iq_frontend_dropin_compiles():
    assert os.path.exists(_build_frontend())


@pytest.mark.gpu
def test_iq_frontend_dropin_runs_on_gpu():
    b = _build_frontend()
    r = subprocess.run([b], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
