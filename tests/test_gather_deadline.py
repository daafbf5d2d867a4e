"""The gather's failure path, on the CPU: libsdrgpu's C-ABI gather loads a
stand-in RCCL (tests/stubs/rccl_stub.c, through SDRGPU_RCCL_LIB) whose peer never answers. A rank
must not block forever on it -- the reference never waits forever on a stopped peer either
(core/src/utils/threading.h:53-62, core/src/dsp/stream.h:94-116): communicator init and the gather's
group end each return SDRGPU_ETIMEOUT naming the rank within the deadline (SDRGPU_GATHER_TIMEOUT_S),
after aborting the communicator (ncclCommAbort). Runs in a child process so the stub, not a real
RCCL, is the one the library binds."""
import os
import subprocess
import sys
import textwrap

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

CHILD = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, {root!r})
    import sdrpp_amd
    from sdrpp_amd import dsp
    mode = {mode!r}
    cid = dsp.gather_id()
    t0 = time.perf_counter()
    try:
        g = dsp.SpectraGather(1, 2, cid, device=-1)
        if mode == "group":
            g.gather_dev(0x1000, 16, 0, 0)
        print("NO-ERROR", flush=True)
    except sdrpp_amd.SdrGpuError as e:
        print("ERR %.3f %s" % (time.perf_counter() - t0, e), flush=True)
""")


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    d = tmp_path_factory.mktemp("rccl_stub")
    so = str(d / "librccl_stub.so")
    subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-o", so, os.path.join(HERE, "stubs", "rccl_stub.c")])
    return so


@pytest.mark.parametrize("mode", ["init", "group"])
def test_gather_peer_never_answers_times_out(stub, tmp_path, mode):
    log = tmp_path / "calls.log"
    env = dict(os.environ, SDRGPU_RCCL_LIB=stub, STUB_RCCL_MODE=mode, STUB_RCCL_LOG=str(log),
               SDRGPU_GATHER_TIMEOUT_S="1.5")
    env.pop("SDRGPU_GATHER_BLOCKING", None)
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, mode=mode)], env=env, capture_output=True,
                       text=True, timeout=120)
    out = p.stdout.strip().splitlines()
    assert p.returncode == 0 and out, p.stderr[-2000:]
    assert out[-1].startswith("ERR "), out
    _, secs, msg = out[-1].split(" ", 2)
    # the deadline, not a hang, ended the wait: at least the timeout, well under the test's limit
    assert 1.4 <= float(secs) < 30.0, secs
    assert "sdrgpu error -6" in msg and "rank 1 of 2" in msg and "1.5 s" in msg, msg
    calls = log.read_text().split()
    assert "abort" in calls, calls          # the communicator was aborted, not left hanging
    assert "destroy" not in calls, calls    # (destroy would block on the dead peer's operations)
    if mode == "init":
        assert calls.count("initRankConfig") == 1 and "groupStart" not in calls
    else:
        assert calls.index("groupEnd") < calls.index("abort")


def test_gather_after_abort_refuses(stub, tmp_path):
    """After a timed-out gather the handle accepts only destroy: a later gather fails at once
    (SDRGPU_ESTATE), never touching the aborted communicator."""
    log = tmp_path / "calls.log"
    code = CHILD.format(root=ROOT, mode="group") + textwrap.dedent("""
        t1 = time.perf_counter()
        try:
            g.gather_dev(0x1000, 16, 0, 0)
            print("NO-ERROR-2")
        except sdrpp_amd.SdrGpuError as e:
            print("ERR2 %.3f %s" % (time.perf_counter() - t1, e))
        g.close()
    """)
    env = dict(os.environ, SDRGPU_RCCL_LIB=stub, STUB_RCCL_MODE="group", STUB_RCCL_LOG=str(log),
               SDRGPU_GATHER_TIMEOUT_S="1.0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    out = p.stdout.strip().splitlines()
    assert p.returncode == 0, p.stderr[-2000:]
    assert out[-1].startswith("ERR2 "), out
    _, secs, msg = out[-1].split(" ", 2)
    assert float(secs) < 0.5 and "sdrgpu error -4" in msg and "aborted" in msg, out[-1]
    calls = log.read_text().split()
    assert calls.count("abort") == 1 and calls.count("groupEnd") == 1 and "destroy" not in calls, calls


def test_gather_posts_every_peer_when_ops_in_progress(stub, tmp_path):
    """A non-blocking communicator may answer ncclInProgress for each send/recv: that is
    an accepted operation, so rank 0 of 3 must still post the receive from every peer (ranks 1 and
    2) before the group end, and no abort follows. (The rank-0 self copy after the group needs a
    device; on this CPU host it fails after the group, which is not what is checked here.)"""
    log = tmp_path / "calls.log"
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        import sdrpp_amd
        from sdrpp_amd import dsp
        g = dsp.SpectraGather(0, 3, dsp.gather_id(), device=-1)
        try:
            g.gather_dev(0x1000, 16, 0x2000, 0)
        except sdrpp_amd.SdrGpuError as e:
            print("ERR", e)
    """)
    env = dict(os.environ, SDRGPU_RCCL_LIB=stub, STUB_RCCL_MODE="post", STUB_RCCL_LOG=str(log),
               SDRGPU_GATHER_TIMEOUT_S="2.0")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert "ncclSend/ncclRecv" not in p.stdout, p.stdout
    calls = log.read_text().split()
    g0 = calls.index("groupStart")
    assert calls[g0 + 1:g0 + 4] == ["recv1", "recv2", "groupEnd"], calls
    assert "abort" not in calls, calls
