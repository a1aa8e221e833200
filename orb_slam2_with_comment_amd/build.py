"""Build liborbmi.so (hand-written HIP kernels for gfx950 + the C ABI) in-tree.

    python -m orb_slam2_with_comment_amd.build

Compiles every csrc/*.hip and csrc/*.cpp with hipcc --offload-arch=gfx950 into
orb_slam2_with_comment_amd/liborbmi.so.  -ffp-contract=off keeps every float expression
one-rounding-per-operation on host and device (pinned semantics P7).
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# ORBMI_LIB / ORBMI_CFLAGS: an alternative library path and extra -D flags, for A/B builds of a
# kernel variant (tools/gpu.sh ab=A,B); the product build uses neither
LIB = os.environ.get("ORBMI_LIB") or os.path.join(PKG, "liborbmi.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("ORBMI_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
         "-Wall", "-Wno-unused-function", f"--offload-arch={ARCH}"]


def sources():
    srcs = sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")))
    srcs += sorted(glob.glob(os.path.join(PKG, "csrc", "*.cpp")))
    return srcs


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    # every file the sources include: headers, the generated csrc/*.inc asm, the C++ mirror
    deps = sources() + glob.glob(os.path.join(PKG, "csrc", "*.h")) + glob.glob(os.path.join(PKG, "csrc", "*.inc"))
    deps += glob.glob(os.path.join(ROOT, "include", "*.h")) + glob.glob(os.path.join(ROOT, "include", "*.hpp"))
    if not force and not _stale(LIB, deps):
        return LIB
    tmp = LIB + ".tmp"
    cmd = [HIPCC, *FLAGS, *os.environ.get("ORBMI_CFLAGS", "").split(), "-o", tmp, *sources()]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
