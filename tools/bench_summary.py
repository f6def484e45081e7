"""One-screen summary of a bench.py JSON line: headline, roofline, the
secondary lines' times / fractions, the shard-width projections."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print(f"headline {d['value']:.4g} {d['unit']}  step {d['ms_per_step']:.3f} ms  K1 {r['kernel_ms']:.3f} ms "
      f"frac {r['frac']:.4f}  scan {r['scan_kernel_ms']:.3f} ms  traffic {r.get('traffic')}")
cpu = d.get("cpu_baseline") or {}
if cpu:
    print(f"cpu_baseline {cpu.get('value', 0):.4g} {cpu.get('unit')} cores {cpu.get('cores')} kind {cpu.get('kind')}")
for k, v in d.get("secondary", {}).items():
    if not isinstance(v, dict):
        continue
    if k == "shard_widths_1gpu":
        for n, s in v.items():
            print(f"  {n}: {s['channels']} ch step {s['ms_per_step']:.3f} K1 {s['kernel_ms']:.3f} "
                  f"(frac {s['roofline_frac']:.3f}) scan {s['scan_kernel_ms']:.3f} eff {s['projected_efficiency']:.3f}")
        continue
    rf = v.get("roofline", {})
    ms = v.get("ms", v.get("ms_per_step"))
    extra = ""
    if "kernels_ms" in v:
        extra = " " + ", ".join(f"{a.split(' ')[0]} {b:.3f}" for a, b in v["kernels_ms"].items())
    print(f"  {k}: {ms if ms is None else round(ms, 3)} ms frac {rf.get('frac') if rf.get('frac') is None else round(rf['frac'], 3)}{extra}")
