#!/usr/bin/env python3
"""Markdown rows of the round-4 results (BASELINE.md / DESIGN.md §4) from profiles/r04/final/."""
import json
import os
import sys

D = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r04", "final")
NAMES = {"2A": "2A: 64×64 MiB, 16 B keys / 256 B values (headline)", "2B": "2B: 64×64 MiB, 37 % superseded",
         "3": "3 scaled: 256×16 MiB, variable keys 8–128 B + 10 % Deletes",
         "3F": "3F: 256×256 MiB (63.4 GB), variable keys + 10 % Deletes",
         "5": "5: 10⁶ × 4 KiB WAL runs, table split", "L0": "L0: 16 buffer runs + 1,024 concatenated L0 runs"}


def load(name):
    p = os.path.join(D, name)
    if not os.path.exists(p):
        return None
    for line in open(p):
        line = line.strip()
        if line.startswith("{"):
            return json.loads(line)
    return None


for c in sys.argv[1:] or ["2A", "2B", "3", "3F", "5", "L0"]:
    b = load(f"bench_{c}.json")
    if b is None:
        continue
    r = b["roofline"]
    io = (b["config"]["input_bytes_per_gpu"] + b["config"]["output_bytes_per_gpu"]) / (b["ms_per_step"] * 1e-3) / 1e12
    h = load(f"host_{c}.json")
    hp = h.get("host_path") if h else None
    cpu = b.get("cpu_baseline", {})
    print(f"| {NAMES.get(c, c)} | {b['value']:.0f} GiB/s ({b['ms_per_step']:.2f} ms) | {io:.2f} | "
          f"{r['kernel']} {r['avg_launch_ms']:.2f} ms, frac {r['frac']:.3f}; pipeline {r['pipeline_frac']:.3f} | "
          f"{'%.1f GiB/s' % hp['value'] if hp else '—'} | {cpu.get('value', '—')} {cpu.get('unit', '')} |")
