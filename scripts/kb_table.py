"""Tabulate scripts/gpu/kbench.sh logs: one line per (config, variant)."""
import ast
import sys

lab = None
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("=="):
        lab = line.split("build/")[-1].split("/")[0] if "build/" in line else "base"
    elif line.startswith("{"):
        d = ast.literal_eval(line)
        keys = [k for k in d if k not in ("config", "B", "split", "N", "step_us")]
        print(f"{d['config']}:{d['B']:<6d} {lab:7s} step {d['step_us']:8.1f} " + " ".join(f"{k} {d[k]:.1f}" for k in keys))
