"""Per-kernel register / spill / LDS summary from hipcc -Rpass-analysis=kernel-resource-usage.

    python tools/resource_usage.py csrc/file.hip [filter]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = os.path.abspath(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
           "-I" + os.path.join(REPO, "include"), "-I" + os.path.dirname(os.path.abspath(src)),
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
           "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
    cur, rows = None, {}
    for line in err.splitlines():
        m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = v
            rows[cur] = {}
        elif cur:
            rows[cur][k.split(" [")[0]] = v
    for name, r in rows.items():
        if filt in name:
            print(f"{name[:90]:90s} v{r.get('VGPRs')} a{r.get('AGPRs')} occ{r.get('Occupancy')} "
                  f"vspill{r.get('VGPRs Spill')} sspill{r.get('SGPRs Spill')} lds{r.get('LDS Size')}")


if __name__ == "__main__":
    main()
