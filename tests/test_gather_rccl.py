"""The C-ABI spectra gather over RCCL (sdrgpu_gather_*), one rank on the single GPU of
a test box: the communicator is built from an id made by rank 0 and every row arrives at rank 0
(world 1: a send/recv to itself through RCCL). Multi-rank runs need one GPU per rank (RCCL
refuses two ranks on one device), so the world > 1 path is covered by bench.py's N-GPU runs; the
host-side protocol (id distribution, rank-0 buffers, max-over-ranks timing) runs under gloo on
the CPU in test_multistream_gloo.py."""
import numpy as np
import pytest

import sdrpp_amd
from sdrpp_amd import dsp

pytestmark = pytest.mark.gpu


def test_gather_one_rank_rccl():
    import torch
    assert sdrpp_amd.lib.sdrgpu_device_count() > 0
    cid = dsp.gather_id()
    assert len(cid) == 128 and any(cid)
    g = dsp.SpectraGather(0, 1, cid, device=0)
    rows = torch.randn(16 * 2048, device="cuda")
    out = torch.zeros(16 * 2048, device="cuda")
    s = torch.cuda.Stream()
    g.gather_dev(rows.data_ptr(), rows.numel(), out.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(out, rows)
    g.close()


def test_gather_rejects_bad_rank():
    cid = dsp.gather_id()
    with pytest.raises(sdrpp_amd.SdrGpuError):
        dsp.SpectraGather(1, 1, cid, device=0)
