"""profiles/<tag>_kernel_stats.txt from a tools/profile.sh output directory:
per-kernel durations of the lfd kernels in the rocprofv3 kernel trace of the
bench, plus the cfg3-size K1 launches beside the same run's HIP-event K1.
Usage: python tools/trace_summary.py gpurun_out/prof_<tag> profiles/<tag>_kernel_stats.txt"""
import collections
import csv
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv"))))
d = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if "lfd::" not in n:
        continue
    short = n.replace("void lfd::(anonymous namespace)::", "").replace("lfd::(anonymous namespace)::", "").split("(")[0]
    d[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
bench = None
for line in open(os.path.join(src, "bench_traced.log")):
    if line.startswith('{"metric'):
        bench = json.loads(line)
out = ["# rocprofv3 --kernel-trace --stats of: python3 bench.py --steps 5 --warmup 1 --no-cpu --no-rolling --no-stream",
       f"# ({os.path.basename(src)}). kernel, calls, avg ms, min ms, max ms"]
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    out.append(f"{k:60s} {len(v):4d} {sum(v) / len(v):9.3f} {min(v):9.3f} {max(v):9.3f}")
k1key = next((k for k in d if k.startswith("k_block_runs_mfma<")), None)
if k1key and bench:
    # K1 launches grouped by grid size (one group per workload of the bench)
    g = collections.defaultdict(list)
    for r in rows:
        if "k_block_runs_mfma<" in r["Kernel_Name"]:
            g[int(r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    hip = bench["roofline"]["kernel_ms"]
    for grid, v in sorted(g.items()):
        out.append(f"# K1 grid {grid:9d}: n={len(v):2d} avg {sum(v) / len(v):8.3f} ms")
    best = min(g.values(), key=lambda v: abs(sum(v) / len(v) - hip))
    out.append(f"# headline workload's K1 grid: avg {sum(best) / len(best):.3f} ms over {len(best)} launches "
               f"(warm-ups and the off-sample line included); the same run's headline K1 by HIP events: {hip:.3f} ms")
open(dst, "w").write("\n".join(out) + "\n")
print("\n".join(out))
