"""Build tests/golden/gates_measured.json from LFD_GATE_LOG files (JSON lines
{"tag", "rel", "tol"} written by tests/gates.py during a GPU run with
LFD_GATE_MEASURE=1 and a CPU run): the table holds, per check tag, the
largest relRMS measured (tags absent from the logs keep their earlier
value); tests/gates.py gates each check at 10x that.

    python tests/golden/make_gates.py gpurun_out/gates_gpu.jsonl /tmp/gates_cpu.jsonl
"""
import json
import os
import sys


def main(paths):
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gates_measured.json")
    measured, fresh, sources = {}, {}, []
    if os.path.exists(out):  # checks no log re-measured keep their value
        with open(out) as f:
            old = json.load(f)
        measured, sources = old["measured"], list(old.get("source", []))
    for p in paths:
        with open(p) as f:
            for line in f:
                r = json.loads(line)
                fresh[r["tag"]] = max(fresh.get(r["tag"], 0.0), float(r["rel"]))
    measured.update(fresh)
    with open(out, "w") as f:
        sources += [os.path.basename(p) for p in paths if os.path.basename(p) not in sources]
        json.dump({"source": sources, "factor": 10.0,
                   "measured": dict(sorted(measured.items()))}, f, indent=1)
        f.write("\n")
    vals = sorted(measured.values())
    print(f"{len(measured)} checks, measured relRMS {vals[0]:.2e} .. {vals[-1]:.2e} -> {out}")


if __name__ == "__main__":
    main(sys.argv[1:])
