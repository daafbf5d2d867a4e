"""The fp64-interior mode's cost against the fp32 kernels (bench.spectrum_f64_cost), one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    import bench
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        print(json.dumps(bench.spectrum_f64_cost(0, s)))


if __name__ == "__main__":
    main()
