#!/bin/bash
# The bench's whole per_call object (device, 16 streams, host drop-in pipelined, host sync), 3 times.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; OUT=$R/gpurun_out; TAG=${1:-pcf}; mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 300 python -c "
import json, torch, bench
torch.cuda.set_device(0); torch.cuda.set_stream(torch.cuda.Stream())
print(json.dumps(bench.per_call_c5(0, torch.cuda.current_stream())))" >> $OUT/${TAG}.jsonl 2>>$OUT/${TAG}_err.log || exit $?
done
