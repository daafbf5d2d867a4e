"""N > 1 path on CPU: world_size-2 gloo run of the stream-sharding + spectra gather + max-time
reduction used by bench.py (the GPU run uses the same code over RCCL)."""
import os
import socket

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
    from sdrpp_amd.multistream import StreamShard
    sh = StreamShard(backend="gloo")
    assert sh.seed() == 0xACE1 + rank and sh.vfo_offset() == 2.5e6 + 1e5 * rank
    rows = torch.full((4, 8), float(rank)) + torch.arange(8, dtype=torch.float32)   # "spectra" of this stream
    got = sh.gather_spectra(rows)
    work, got2 = sh.gather_spectra_async(rows * 2)   # bench.py's overlapped form
    work.wait()
    t = sh.max_over_ranks([1.0 + rank, 5.0 - rank])
    sh.barrier()
    if rank == 0:
        ok = len(got) == world and all(torch.equal(got[r], torch.full((4, 8), float(r)) + torch.arange(8.0))
                                        for r in range(world))
        ok = ok and len(got2) == world and all(torch.equal(got2[r], 2 * got[r]) for r in range(world))
        q.put((ok, t))
    sh.close()


def test_two_rank_gather_and_max():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    ok, t = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok
    assert t == [2.0, 5.0]
