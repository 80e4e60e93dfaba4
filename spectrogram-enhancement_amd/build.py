"""Build libspecenh.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python spectrogram-enhancement_amd/build.py [--force] [--jobs N]

Every csrc/*.hip is compiled to an object (in parallel) and linked into
specenh/libspecenh.so next to the Python package, so the library travels to the
GPU box with the repo snapshot. Incremental: an object is rebuilt only when its
source, a header, or this script is newer.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build", "obj")
LIB = os.path.join(HERE, "specenh", "libspecenh.so")
ARCH = os.environ.get("SPECENH_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -packed-fp32-ops: on CDNA4 a v_pk_*_f32 costs the issue slots of two scalar ops, and
# VOP3P cannot take literal operands, so packed codegen only adds SGPR-held constants
# (spills) and register-pair moves to the FFT kernels.
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + os.path.join(REPO, "include"),
          "-I" + CSRC, "-Wall", "-Wno-unused-function",
          "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def _deps_mtime():
    deps = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(REPO, "include", "*.h"))
    deps.append(os.path.abspath(__file__))
    return max(_mtime(d) for d in deps)


def _compile(src, force):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    if not force and _mtime(obj) > max(_mtime(src), _deps_mtime()):
        return obj, False
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj, True


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    if not srcs:
        raise RuntimeError("no HIP sources found")
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force), srcs))
    objs = [o for o, _ in results]
    rebuilt = any(b for _, b in results)
    if rebuilt or force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        if verbose:
            print(f"[specenh] built {LIB} from {len(objs)} sources")
    elif verbose:
        print(f"[specenh] up to date: {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    args = ap.parse_args()
    try:
        build(args.force, args.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
