"""Streaming lines of bench.py alone (cfg4 edge latency, cfg5 out-of-core)
for A/B runs and rocprofv3 traces:  python tools/bench_stream.py [cfg4|cfg5|all]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    if which in ("cfg4", "all"):
        out["edge_latency_cfg4"] = bench.bench_edge_cfg4(dev)
        out["edge_latency_cfg4_time_major"] = bench.bench_edge_cfg4(dev, time_major=True)
    if which in ("cfg5", "all"):
        out["out_of_core_cfg5"] = bench.bench_ooc_cfg5(dev)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
