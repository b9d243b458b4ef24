"""Build libbanjax_gpu.so (gfx950) and the bench/test synthetic-log library in-tree.

hipcc cross-compiles for gfx950 without a GPU; the .so files travel to the GPU
box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
ARCH = os.environ.get("BJX_OFFLOAD_ARCH", "gfx950")
COMMON = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "--offload-arch=%s" % ARCH,
          "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result"]

TARGETS = {
    "libbanjax_gpu.so": ["engine.hip", "regex_compiler.cpp", "tailer.cpp", "node.cpp"],
}


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(HERE, "..", "include", "banjax_gpu.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False):
    os.makedirs(LIBDIR, exist_ok=True)
    for out, srcs in TARGETS.items():
        srcs = [os.path.join(CSRC, s) for s in srcs]
        dst = os.path.join(LIBDIR, out)
        if not force and not _stale(dst, srcs):
            continue
        cmd = ["hipcc"] + COMMON + ["-o", dst] + srcs
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIBDIR


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
