"""Per-kernel register / LDS / occupancy of one csrc file (hipcc resource-usage remarks).
    python tools/kres.py conv_ae.hip [name-regex]"""
import os
import re
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(R, "spectrogram-enhancement_amd", "csrc", sys.argv[1])
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
       "-I" + os.path.join(R, "include"), "-I" + os.path.dirname(src), "-Xclang", "-target-feature",
       "-Xclang", "-packed-fp32-ops", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
rows = []
for line in err.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|VGPRs Spill|SGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
for r in rows:
    if pat.search(r["name"]):
        print(f"{r['name'][:72]:72s} v{r.get('VGPRs')} a{r.get('AGPRs')} occ{r.get('Occupancy [waves/SIMD]')} "
              f"lds{r.get('LDS Size [bytes/block]')} spill{r.get('VGPRs Spill')}/{r.get('SGPRs Spill')}")
