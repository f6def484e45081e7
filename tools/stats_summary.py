"""Per-kernel rocprofv3 --stats summary of the lfd kernels in one or more
output directories (each holding a <name>_kernel_stats.csv):

    python tools/stats_summary.py gpurun_out/prof_r05f/head gpurun_out/prof_r05f/fr ...
"""
import csv
import glob
import os
import sys


def short(name):
    n = name.replace("void lfd::(anonymous namespace)::", "").replace("lfd::(anonymous namespace)::", "")
    return n.replace("void lfd::", "").replace("lfd::", "").split("(")[0]


def main():
    for d in sys.argv[1:]:
        files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not files:
            print(f"# {d}: no kernel_stats.csv")
            continue
        print(f"# {os.path.relpath(d)}: kernel, calls, avg ms, min ms, max ms")
        for r in sorted(csv.DictReader(open(files[0])), key=lambda r: -float(r["TotalDurationNs"])):
            if "lfd::" not in r["Name"]:
                continue
            print(f"{short(r['Name']):60s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e6:9.3f} "
                  f"{float(r['MinNs']) / 1e6:9.3f} {float(r['MaxNs']) / 1e6:9.3f}")


if __name__ == "__main__":
    main()
