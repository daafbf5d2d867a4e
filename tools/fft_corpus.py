"""Spectrum accuracy over the seed-fixed frame corpus (tests/_util.py corpus_ulp_rows: 4096 / 16384 /
65536 points x 7 windows x FRAMES random frames + F1M 1M-point frames), for the library under test
(SDRGPU_LIB_PATH or the in-tree build): fp32 kernels and fp64-interior mode, next to pocketfft single
precision on every frame. Prints one JSON object (aggregates + per-frame rows); the GPU test
test_spectrum_ulp_corpus asserts the bars on the same data."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from _util import corpus_aggregate, corpus_ulp_rows  # noqa: E402

rows = corpus_ulp_rows(int(os.environ.get("FRAMES", "24")), int(os.environ.get("F1M", "6")))
print(json.dumps({"lib": os.environ.get("SDRGPU_LIB_PATH", "in-tree"), "aggregate": corpus_aggregate(rows), "rows": rows}))
