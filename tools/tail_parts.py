"""Where the tail-inclusive rate goes: the tailer's file reads alone (host
framing mode, no device), one pinned host-to-device copy stream alone, and
both together without the engine.  usage: python tools/tail_parts.py [MiB] [batch_MiB]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from banjax_amd.tailer import LogTailer  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    bm = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bjx_tail_parts.log")
    line = b"1700000000.000 10.0.0.1 GET example.com GET /index.html HTTP/1.1 Mozilla/5.0 xxxxxxxxxxxxxxxxxxxxxxxxxx\n"
    blk = line * ((1 << 20) // len(line))
    with open(path, "wb") as f:
        for _ in range(mib):
            f.write(blk)
    nb = os.path.getsize(path)
    out = {"file_bytes": nb, "batch_MiB": bm}
    for dev, key in ((-1, "read_only_GBps"), (0, "read_and_h2d_GBps")):
        best = 0.0
        for _ in range(2):
            t0 = time.perf_counter()
            got = 0
            with LogTailer(path, device=dev, from_start=True, batch_bytes=bm << 20, poll_ms=1, slots=3) as tl:
                while got < nb:
                    b = tl.next(timeout_ms=1000)
                    if b is None:
                        continue
                    got += b.n_bytes
                    tl.release(b)
            best = max(best, nb / (time.perf_counter() - t0) / 1e9)
        out[key] = round(best, 2)
    h = torch.empty(bm << 20, dtype=torch.uint8).pin_memory()
    d = torch.empty(bm << 20, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_pinned_GBps"] = round(reps * (bm << 20) / (time.perf_counter() - t0) / 1e9, 2)
    print(json.dumps(out), flush=True)
    os.unlink(path)


if __name__ == "__main__":
    main()
