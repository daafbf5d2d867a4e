"""C5 at the reference block size (307,200 samples per call) on its own, for a rocprofv3 trace
of the per-call launch sequence: python tools/per_call.py [calls] [single]  (single: only the
one-stream device calls, so per-kernel durations are not stretched by the 16-stream part)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream())
print(json.dumps(bench.per_call_c5(0, torch.cuda.current_stream(), calls=int(sys.argv[1]) if len(sys.argv) > 1 else 300,
                                   single_only=len(sys.argv) > 2 and sys.argv[2] == "single")))
