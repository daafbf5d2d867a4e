"""The C++ drop-in blocks (sdrpp_amd/dsp/gpu, reference class names) compile against the
block-API mirror and, on a GPU, reproduce the oracle inside the threaded stream model."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "test_dropin")


def _build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-pthread",
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "gpu"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime"),
           "-I", os.path.join(ROOT, "sdrpp_amd", "dsp", "runtime", "dsp", "buffer"),   # resolves "../processor.h"
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
           os.path.join(ROOT, "tests", "cpp", "test_dropin.cpp"),
           "-L", os.path.join(ROOT, "sdrpp_amd", "lib"), "-lsdrgpu",
           "-L", os.path.join(ROOT, "oracle"), "-lsdr_oracle",
           "-Wl,-rpath," + os.path.join(ROOT, "sdrpp_amd", "lib") + ":" + os.path.join(ROOT, "oracle"),
           "-o", BIN]
    subprocess.check_call(cmd)


def test_dropin_compiles():
    _build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_dropin_runs_on_gpu():
    _build()
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
