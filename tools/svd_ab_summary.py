"""Summarise tools/lib_ab.sh runs of tools/svd_bench.py: C3 ms per mode and library."""
import json
import sys

cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.strip("= \n")
    elif line.startswith("{"):
        d = json.loads(line)
        print(f"{cur:24s} rank16 {d['rank16']['ms']:.3f} ms (acc {d['rank16']['accuracy']['rel_fro_max']:.1e})  "
              f"default {d['default']['ms']:.3f} ms (acc {d['default']['accuracy']['rel_fro_max']:.1e})")
