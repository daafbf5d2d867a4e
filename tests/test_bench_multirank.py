"""bench.py's N > 1 control flow at world size 2 on the CPU: the very
`bench.run_config` the 8-GPU run executes -- seeds per rank, warm-up, the double-buffered zoom rows
acquired / published / drained through multistream.GatherPipeline every step, barriers, the
max-over-ranks timing, rank 0's checksum verification of the last gather and the gather report --
with only the device side swapped: a CPU runtime (torch CPU tensors, perf_counter events) and
LazyGlooGather (gathers over gloo that execute only when their completion is waited for, so a
buffer overwritten before its gather ran would ship the wrong rows) in place of torch.cuda streams
and libsdrgpu's RCCL gather. The workload is a CPU stand-in for C5 with the same interface
(`zoom` buffers, `zoom_count`, `run(x, s, timed_call, buf)`) whose rows depend on the rank and the
step, so the verification has something to catch."""
import argparse
import os
import socket
import time

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _CpuEvent:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class _CpuRuntime:
    reduce_device = None

    def rand(self, n, seed):
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.rand(n, generator=g) * 2 - 1

    def event(self):
        return _CpuEvent()

    def handle(self, stream):
        return stream

    def synchronize(self):
        pass

    def gather_backend(self, shard, dev):
        from sdrpp_amd.multistream import LazyGlooGather
        return LazyGlooGather()


class _C5Cpu:
    """C5's interface on the CPU: `frames` rows of ZW columns per step, a function of the step's
    input, this rank's stream (seed) and the step number."""
    N, ZW = 4096, 64

    def __init__(self, B, shard, dev):
        self.B = (B // self.N) * self.N
        self.frames = self.B // self.N
        self.zoom = [torch.empty(self.frames * self.ZW) for _ in range(2)]
        self.zoom_count = self.frames * self.ZW
        self.rank = shard.rank
        self.k = 0
        self.bytes_per_sample = 12.0
        self.kernel_bytes = 12.0 * self.B
        self.kernel_name = "cpu stand-in"
        self.history = []

    def run(self, x, s, timed_call, buf=0):
        def body():
            rows = x[:2 * self.B].view(self.frames, -1)[:, :self.ZW] + 1000.0 * self.rank + self.k
            self.zoom[buf].copy_(rows.reshape(-1))
        timed_call(body)
        self.history.append(self.zoom[buf].clone())
        self.k += 1


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    from sdrpp_amd.multistream import StreamShard
    shard = StreamShard(backend="gloo")
    a = argparse.Namespace(log2_batch=16, steps=5, warmup=2, config="c5")
    B, elapsed, kern_ms, wl = bench.run_config("c5", a, shard, None, "compute", rt=_CpuRuntime(),
                                               workloads={"c5": _C5Cpu})
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
