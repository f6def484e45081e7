"""Run bench.py's full-rate band-pass line alone (iteration / rocprofv3)."""
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
os.environ.setdefault("LFDAS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "low-freq-real-time_amd", "lfdas", "liblfdas_diag.so"))  # A/B knobs: diagnostic build only
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    import torch
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000
    print(json.dumps(bench.bench_fullrate(torch.device("cuda:0"), n=n)), flush=True)
