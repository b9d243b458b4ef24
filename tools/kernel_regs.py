"""Register / LDS / scratch use of the gfx950 kernels in libbanjax_gpu.so.

    python tools/kernel_regs.py [regex]

Extracts the device code object with llvm-objdump --offloading into a temp
dir and reads the AMDHSA metadata notes with llvm-readelf.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "banjax_amd", "lib", "libbanjax_gpu.so")


def main():
    pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else r"k_")
    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "lib.so")
        with open(LIB, "rb") as src, open(lib, "wb") as dst:
            dst.write(src.read())
        subprocess.run([LLVM + "/llvm-objdump", "--offloading", lib], cwd=d, check=True, capture_output=True)
        co = [f for f in os.listdir(d) if "gfx950" in f][0]
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", os.path.join(d, co)], check=True,
                               capture_output=True, text=True).stdout
    cur, rows = {}, []
    for ln in notes.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)", ln)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count":  # first key of each kernel record (keys are sorted)
            if cur.get("name"):
                rows.append(cur)
            cur = {}
        if k == "symbol":
            cur["name"] = v.replace(".kd", "")
        elif k not in cur:
            cur[k] = v
    if cur.get("name"):
        rows.append(cur)
    print("%-60s %5s %5s %5s %6s %7s %6s" % ("kernel", "vgpr", "agpr", "sgpr", "spill", "lds", "priv"))
    for r in rows:
        name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        if not pat.search(name) or "rocprim" in name:
            continue
        short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "")
        print("%-60s %5s %5s %5s %6s %7s %6s" % (short[:60], r.get("vgpr_count"), r.get("agpr_count"), r.get("sgpr_count"),
                                                r.get("vgpr_spill_count"), r.get("group_segment_fixed_size"),
                                                r.get("private_segment_fixed_size")))


if __name__ == "__main__":
    main()
