#!/usr/bin/env python3
"""One line per bench JSON file: value, step time, kernel times, rooflines, CPU baseline.
usage: python tools/bench_summary.py file [file ...] (the last line of each file is the JSON line)"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except (OSError, ValueError, IndexError) as e:
        print(f, "unreadable:", e)
        continue
    k = {a: (round(b * 1e3, 2) if isinstance(b, float) else b) for a, b in d.get("kernels_ms", {}).items() if a != "note"}
    r = d["roofline"]
    print(f, f"{d['value']:.4g} {d['unit']}, {d['ms_per_step'] * 1e3:.2f} us/step, steps {d['steps']}; kernels us {k}; "
             f"k_scan_w frac {r['frac']:.4f} traffic {r['traffic']}")
    h = d.get("roofline_hbm")
    if h:
        print("   config 3:", {a: round(h[a], 4) for a in ("frac", "ms", "k1_frac", "k1_ms", "pipeline_ms", "windows_per_s")})
    c = d.get("cpu_baseline")
    if c:
        print("   cpu baseline:", round(c["value"], 1), c["unit"])
