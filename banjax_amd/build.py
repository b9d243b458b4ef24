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
# BJX_PROF=1: also compile the k_lines segment-clock variants (BJX_PROF_LINES)
PROF = ["-DBJX_PROF"] if os.environ.get("BJX_PROF") == "1" else []
# BJX_EXTRA_FLAGS: extra compiler flags (timing experiments only)
PROF += os.environ.get("BJX_EXTRA_FLAGS", "").split()
COMMON = PROF + ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "--offload-arch=%s" % ARCH,
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
    """Each source compiles to its own object (in parallel, only when stale),
    then one link: editing engine.hip does not recompile the host-only sources."""
    os.makedirs(LIBDIR, exist_ok=True)
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    for out, srcs in TARGETS.items():
        srcs = [os.path.join(CSRC, s) for s in srcs]
        dst = os.path.join(LIBDIR, out)
        objs, procs = [], []
        for s in srcs:
            o = os.path.join(objdir, os.path.basename(s) + ".o")
            objs.append(o)
            if force or _stale(o, [s]):
                cmd = ["hipcc"] + [f for f in COMMON if f != "-shared"] + ["-c", "-o", o, s]
                if verbose:
                    print(" ".join(cmd), flush=True)
                procs.append((subprocess.Popen(cmd), cmd))
        for pr, cmd in procs:
            if pr.wait() != 0:
                raise subprocess.CalledProcessError(pr.returncode, cmd)
        if force or procs or _stale(dst, objs):
            cmd = ["hipcc"] + COMMON + ["-o", dst] + objs + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.run(cmd, check=True)
    return LIBDIR

if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
