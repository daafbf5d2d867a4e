"""bench.py's N > 1 control flow at world size 2 on the CPU: the very
`bench.run_config` the 8-GPU run executes -- seeds per rank, warm-up, the double-buffered zoom rows
acquired / published / drained through multistream.GatherPipeline every step, barriers, the
max-over-ranks timing, rank 0's checksum verification of the last gather and the gather report --
with only the device side swapped: bench.CpuRehearsalRuntime (torch CPU tensors, perf_counter
events) and LazyGlooGather (gathers over gloo that execute only when their completion is waited for, so a
buffer overwritten before its gather ran would ship the wrong rows) in place of torch.cuda streams
and libsdrgpu's RCCL gather. The workload is bench.C5Rehearsal, a CPU stand-in for C5 with the same interface
(`zoom` buffers, `zoom_count`, `run(x, s, timed_call, buf)`) whose rows depend on the rank and the
step, so the verification has something to catch."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from sdrpp_amd.multistream import StreamShard
    shard = StreamShard(backend="gloo")
    a = argparse.Namespace(log2_batch=16, steps=5, warmup=2, config="c5")
    B, elapsed, kern_ms, wl = bench.run_config("c5", a, shard, None, "compute", rt=bench.CpuRehearsalRuntime(),
                                               workloads={"c5": bench.C5Rehearsal})
    r = bench.config_result("c5", a, world, B, elapsed, kern_ms, wl)
    # every rank's last published rows, for rank 0's independent check
    last = shard.all_gather_tensor(wl.history[-1])
    if rank == 0:
        q.put((r, [last[i].clone() for i in range(world)], elapsed, kern_ms))
    shard.close()


def test_run_config_world2_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    r, last, elapsed, kern_ms = q.get(timeout=180)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = r["gather"]
    assert g["verified"] is True and g["ranks"] == 2 and g["mismatched_ranks"] == []
    assert g["rows_per_rank"] == 16 * 64 and g["bytes_per_rank_per_step"] == 4 * 16 * 64
    # the value is the whole job (both ranks' samples) over the max-over-ranks time
    assert abs(r["value"] - world * (1 << 16) * 5 / elapsed / 1e6) <= 1e-3 * r["value"]
    assert kern_ms > 0 and elapsed > 0
    # the last step's rows differ per rank (the stream's seed and the rank), as published
    assert not torch.equal(last[0], last[1])
    assert torch.all(last[1] - last[0] > 500)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=240):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    return p, time.monotonic() - t0


REH = ["--runtime", "cpu-rehearsal", "--log2-batch", "16", "--steps", "4", "--warmup", "1"]


def test_bench_cli_gpus2_self_launches_two_ranks():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts two rank processes
    itself (the parent never touches the GPU), and rank 0's line carries n_gpus 2 and a verified
    gather whose received rows match what each rank last published."""
    p, _ = _bench(["--gpus", "2"] + REH)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout   # one JSON line, from rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["runtime"] == "cpu-rehearsal"
    g = r["gather"]
    assert g["verified"] is True and g["ranks"] == 2 and g["mismatched_ranks"] == []
    assert len(r["last_rows_checksums"]) == 2 and r["last_rows_checksums"][0] != r["last_rows_checksums"][1]
    # whole-job value: both ranks' samples over the max-over-ranks time
    assert abs(r["value"] - 2 * r["samples_per_rank_per_step"] * 4 / (r["ms_per_step"] * 4e-3) / 1e6) <= 2e-3 * r["value"]


def test_bench_cli_gpus4_self_launch():
    """The same self-launch at four ranks: rank 0 receives and verifies every rank's rows."""
    p, _ = _bench(["--gpus", "4"] + REH)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 4 and r["gather"]["verified"] is True and r["gather"]["ranks"] == 4
    assert len({tuple(c) for c in r["last_rows_checksums"]}) == 4


def test_bench_cli_gpus1_runs_in_process():
    p, _ = _bench(["--gpus", "1"] + REH)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert r["n_gpus"] == 1 and "gather" not in r


def test_bench_cli_child_death_fails_parent():
    """One rank dying mid-run ends the parent non-zero (with the dead rank's status), within the
    grace period, not after a hang."""
    p, secs = _bench(["--gpus", "2"] + REH, {"SDRGPU_BENCH_REHEARSAL_DIE": "1:2", "SDRGPU_BENCH_GRACE_S": "5",
                                           "SDRGPU_GATHER_TIMEOUT_S": "5"})
    assert p.returncode == 3, (p.returncode, p.stderr[-3000:])
    assert "rank 1 exited with status 3" in p.stderr
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines())
    assert secs < 120


def test_bench_cli_world_size_mismatch_refused():
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"] + REH,
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr, (p.returncode, p.stderr[-2000:])
