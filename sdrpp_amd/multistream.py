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
            if backend == "nccl":
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend or "gloo")

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
