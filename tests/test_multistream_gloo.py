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


def _pipeline_worker(rank, world, port, q, skip_wait):
    """bench.py's N > 1 gather protocol (multistream.GatherPipeline) on gloo with lazily executed
    gathers: step k writes (rank, k) into the buffer it acquired; rank 0 checks every gathered
    slice and the end-of-run checksum verification. skip_wait=True breaks the protocol (the
    producer rewrites a buffer without waiting for its gather) and must be caught."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from sdrpp_amd.multistream import GatherPipeline, LazyGlooGather, StreamShard
    sh = StreamShard(backend="gloo")
    be = LazyGlooGather()
    pipe = GatherPipeline(sh, 64, be)
    steps = 7
    for k in range(steps):
        if skip_wait:
            b = pipe.steps & 1
        else:
            b = pipe.acquire("compute")
        pipe.bufs[b].fill_(1000.0 * rank + k)                 # this step's "waterfall rows"
        pipe.publish(b, "compute", timed=True)
    pipe.drain("compute")
    be.close()
    ok, det = pipe.verify()
    if rank == 0:
        per_step = [all(torch.all(rows[r] == 1000.0 * r + tag).item() for r in range(world)) for tag, rows in be.history]
        q.put((ok, det, [tag for tag, _ in be.history], per_step))
    sh.close()


def _run_pipeline(skip_wait):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_pipeline_worker, args=(r, world, port, q, skip_wait)) for r in range(world)]
    for p in ps:
        p.start()
    res = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


def test_gather_pipeline_protocol():
    ok, det, tags, per_step = _run_pipeline(skip_wait=False)
    assert ok and det["mismatched_ranks"] == [] and det["ranks"] == 2
    assert tags == list(range(7))          # every step gathered once, in order
    assert all(per_step)                    # and each carried that step's rows of every rank


def test_gather_pipeline_catches_early_overwrite():
    ok, det, tags, per_step = _run_pipeline(skip_wait=True)
    assert tags == list(range(7))
    assert not all(per_step)                # a gather shipped rows of a later step
