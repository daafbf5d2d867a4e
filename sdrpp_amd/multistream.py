"""Multi-GPU layer of the streaming-DSP path: one independent IQ stream per GPU.

SDR++ has no multi-device code; independent IQ streams (one SDR per
GPU) shard with no per-sample exchange. The only collective is a rank-0 gather of the
spectrum rows for display. On GPUs it is libsdrgpu's C-ABI RCCL gather (sdrgpu_gather_*,
the same call a C++ host makes), its 128-byte communicator id handed from rank 0 to the
other ranks through torch.distributed; on the CPU ("gloo", tests) torch's gather stands in.
Timing is the max over ranks.
"""
import os

import torch
import torch.distributed as dist


class StreamShard:
    """Rank/world bookkeeping for stream-per-GPU sharding."""

    def __init__(self, backend=None):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.backend = backend
        if self.world > 1 and not dist.is_initialized():
            # the process group's collectives (id broadcast, barriers, max over ranks) share the
            # gather's deadline: a rank that never arrives ends the run with an error, not a hang
            import datetime
            tmo = datetime.timedelta(seconds=float(os.environ.get("SDRGPU_GATHER_TIMEOUT_S", "120")) + 60)
            if backend == "nccl":
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), timeout=tmo)
            else:
                dist.init_process_group(backend or "gloo", timeout=tmo)

    # stream parameters of this rank's SDR: a distinct seed and VFO offset per stream
    def seed(self, base=0xACE1):
        return base + self.rank

    def vfo_offset(self, base=2.5e6, step=1e5):
        return base + step * self.rank

    def rccl_gather(self, device):
        """A libsdrgpu SpectraGather for this rank (GPU runs, world > 1): rank 0 makes the RCCL id
        and broadcasts it to the other ranks over the process group."""
        from sdrpp_amd import dsp
        cid = torch.zeros(128, dtype=torch.uint8, device="cuda")
        if self.rank == 0:
            cid.copy_(torch.frombuffer(bytearray(dsp.gather_id()), dtype=torch.uint8))
        dist.broadcast(cid, src=0)
        return dsp.SpectraGather(self.rank, self.world, bytes(cid.cpu().numpy().tobytes()), device=device)

    def gather_spectra(self, local_rows, out_list=None):
        """Gather every rank's latest spectra rows to rank 0 (list indexed by rank there)."""
        if self.world == 1:
            return [local_rows]
        if self.rank == 0 and out_list is None:
            out_list = [torch.empty_like(local_rows) for _ in range(self.world)]
        dist.gather(local_rows, out_list if self.rank == 0 else None, dst=0)
        return out_list if self.rank == 0 else None

    def gather_spectra_async(self, local_rows, out_list=None):
        """Start the rank-0 gather and return (work, out_list); work.wait() before `local_rows`
        or `out_list` are touched again. Over RCCL the collective runs on the process group's
        own stream, so it overlaps the rest of the chain instead of serialising behind it."""
        if self.world == 1:
            return None, [local_rows]
        if self.rank == 0 and out_list is None:
            out_list = [torch.empty_like(local_rows) for _ in range(self.world)]
        work = dist.gather(local_rows, out_list if self.rank == 0 else None, dst=0, async_op=True)
        return work, (out_list if self.rank == 0 else None)

    def all_gather_tensor(self, t):
        """[world, *t.shape] stack of every rank's `t` (same device as t)."""
        if self.world == 1:
            return t.unsqueeze(0)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t)
        return torch.stack(parts)

    def max_over_ranks(self, values, device=None):
        t = torch.tensor(values, dtype=torch.float64, device=device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(v) for v in t]

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def close(self):
        if self.world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def row_checksum(t):
    """Exact, order-sensitive checksum of a float tensor's bits: (sum of the words, sum of word x
    (index mod 65521)), int64 with wrap-around -- the same on every device."""
    w = t.reshape(-1).view(torch.int32).to(torch.int64)
    idx = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521
    return torch.stack([w.sum(), (w * idx).sum()])


class GatherPipeline:
    """Rank-0 gather of a double-buffered batch of rows every step, overlapped with the next
    step (bench.py's C5 at N > 1). Step k's producer writes bufs[acquire()]; publish()
    hands that buffer to the gather stream; a buffer is written again only after the gather that
    last read it has finished (acquire waits for it). verify() proves the last gather delivered:
    rank 0's received slice r must carry rank r's own checksum of the buffer it sent.

    `backend` supplies the device side: CudaGather (torch.cuda streams / events + libsdrgpu's C-ABI
    RCCL gather, GPU runs) or LazyGlooGather (CPU tests: gathers over gloo that run only when their
    completion is waited for, so a buffer overwritten too early is caught)."""

    def __init__(self, shard, count, backend):
        self.shard, self.count, self.be = shard, int(count), backend
        self.bufs = [backend.empty(self.count) for _ in range(2)]
        self.out = backend.empty(shard.world * self.count) if shard.rank == 0 else None
        self.done = [None, None]
        self.steps = 0
        self.last = None
        self.timed = []

    def acquire(self, stream):
        b = self.steps & 1
        if self.done[b] is not None:
            self.be.wait(stream, self.done[b])
        return b

    def publish(self, b, stream, timed=False):
        ready = self.be.record(stream)
        self.be.wait(self.be.gstream, ready)
        t0 = self.be.record(self.be.gstream, timing=True) if timed else None
        self.be.gather(self.bufs[b], self.count, self.out, self.be.gstream, tag=self.steps)
        fin = self.be.record(self.be.gstream, timing=timed)
        if timed:
            self.timed.append((t0, fin))
        self.done[b] = fin
        self.last = b
        self.steps += 1

    def drain(self, stream):
        finish = getattr(self.be, "finish", None)
        if finish is not None:   # the gathers complete (or fail loudly) before anyone waits on them
            finish()
        for e in self.done:
            if e is not None:
                self.be.wait(stream, e)

    def gather_ms(self):
        """Mean duration of the timed gathers on the gather stream (after synchronize)."""
        if not self.timed:
            return None
        return sum(self.be.elapsed_ms(a, b) for a, b in self.timed) / len(self.timed)

    def verify(self):
        """After drain + synchronize, on every rank: (ok, details). ok is rank 0's verdict that each
        received slice equals the sender's own buffer of the last gather (True elsewhere)."""
        own = row_checksum(self.bufs[self.last])
        sent = self.shard.all_gather_tensor(own)
        if self.shard.rank != 0:
            return True, None
        got = torch.stack([row_checksum(self.out[r * self.count:(r + 1) * self.count]) for r in range(self.shard.world)])
        bad = [r for r in range(self.shard.world) if not torch.equal(got[r].cpu(), sent[r].cpu())]
        return not bad, {"ranks": self.shard.world, "rows_per_rank": self.count, "mismatched_ranks": bad}

    def close(self):
        self.be.close()


class CudaGather:
    """GatherPipeline backend for GPU runs: torch.cuda events on a gather stream of its own, and
    libsdrgpu's C-ABI RCCL gather (sdrgpu_gather_rows)."""

    def __init__(self, shard, device):
        self.g = shard.rccl_gather(device)
        self.gstream = torch.cuda.Stream()

    def empty(self, n):
        return torch.empty(n, dtype=torch.float32, device="cuda")

    def record(self, stream, timing=False):
        e = torch.cuda.Event(enable_timing=timing)
        e.record(stream)
        return e

    def wait(self, stream, ev):
        stream.wait_event(ev)

    def gather(self, buf, count, out, stream, tag=None):
        self.g.gather_dev(buf.data_ptr(), count, out.data_ptr() if out is not None else 0, stream.cuda_stream)

    def finish(self):
        """Wait for every enqueued gather against the gather deadline (sdrgpu_gather_wait), so a
        peer that died fails this rank with an error instead of a device synchronise that never
        returns."""
        self.g.wait(self.gstream.cuda_stream)

    def elapsed_ms(self, a, b):
        return a.elapsed_time(b)

    def close(self):
        self.g.close()


class LazyGlooGather:
    """CPU stand-in for CudaGather (tests): 'streams' are labels, a gather is queued and runs over
    gloo only when an event recorded after it is waited for (or at drain) -- like a device gather
    that reads its buffer whenever the GPU gets to it. A pipeline that rewrites a buffer before
    waiting for the gather that reads it therefore ships the wrong rows, and verify() / the history
    show it. history (rank 0): [(tag, [rows of rank r])] in execution order."""

    gstream = "gather"

    def __init__(self):
        self.queue = []       # pending gathers (tag, buf, count, out)
        self.ran = 0          # gathers executed so far (queue position of the next one)
        self.history = []

    def empty(self, n):
        return torch.zeros(n, dtype=torch.float32)

    def record(self, stream, timing=False):
        # compute-stream work runs synchronously on the CPU: its events are complete at once; a
        # gather-stream event completes when every gather queued before it has run
        return self.ran + len(self.queue) if stream == self.gstream else 0

    def wait(self, stream, ev):
        while self.ran < ev:
            tag, buf, count, out = self.queue.pop(0)
            rank0 = out is not None
            parts = [torch.empty(count) for _ in range(dist.get_world_size())] if rank0 else None
            dist.gather(buf, parts, dst=0)
            if rank0:
                for r, p in enumerate(parts):
                    out[r * count:(r + 1) * count] = p
                self.history.append((tag, [p.clone() for p in parts]))
            self.ran += 1

    def gather(self, buf, count, out, stream, tag=None):
        self.queue.append((tag, buf, count, out))

    def elapsed_ms(self, a, b):
        return 0.0

    def close(self):
        self.wait(None, self.ran + len(self.queue))
