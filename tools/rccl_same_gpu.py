"""Probe: can the C-ABI RCCL gather (sdrgpu_gather_*) run world = 2 with both ranks on ONE GPU? If
RCCL accepts it, the world > 1 branch of sdrgpu_gather_rows (rank 0 receiving from a peer) runs on
the 1-GPU box. The id goes through a file; both ranks time out in 30 s instead of hanging.
  python tools/rccl_same_gpu.py            (parent: starts the two ranks)"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rank_main(rank, idfile):
    import torch
    from sdrpp_amd import dsp
    torch.cuda.set_device(0)
    if rank == 0:
        cid = dsp.gather_id()
        with open(idfile + ".tmp", "wb") as f:
            f.write(cid)
        os.replace(idfile + ".tmp", idfile)
    else:
        t0 = time.time()
        while not os.path.exists(idfile):
            if time.time() - t0 > 30:
                raise SystemExit("no id")
            time.sleep(0.05)
        cid = open(idfile, "rb").read()
    t0 = time.time()
    g = dsp.SpectraGather(rank, 2, cid, device=0, timeout=30)
    n = 1 << 20
    rows = torch.full((n,), float(rank + 1), device="cuda") + torch.arange(n, device="cuda", dtype=torch.float32)
    out = torch.zeros(2 * n, device="cuda") if rank == 0 else None
    s = torch.cuda.current_stream()
    for _ in range(3):
        g.gather_dev(rows.data_ptr(), n, out.data_ptr() if out is not None else 0, s.cuda_stream)
    g.wait(s.cuda_stream)
    torch.cuda.synchronize()
    res = {"rank": rank, "init_and_3_gathers_s": round(time.time() - t0, 3)}
    if rank == 0:
        exp = torch.cat([rows - 1 + 1, rows + 1])   # rank r's rows = r + 1 + arange
        res["verified"] = bool(torch.equal(out, exp))
    g.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        rank_main(int(sys.argv[1]), sys.argv[2])
    else:
        idfile = os.path.join(ROOT, "gpurun_out", "rccl_same_gpu.id")
        if os.path.exists(idfile):
            os.remove(idfile)
        env = dict(os.environ, SDRGPU_GATHER_TIMEOUT_S="30")
        ps = [subprocess.Popen([sys.executable, "-u", __file__, str(r), idfile], env=env) for r in range(2)]
        rc = [p.wait(timeout=120) for p in ps]
        print(json.dumps({"exit_codes": rc}), flush=True)
        sys.exit(max(abs(c) for c in rc))
