"""Tail-inclusive rate: a log file of synthetic banjax_format
lines is followed from offset 0 by the native tailer (pinned slots, HBM copy
on its own stream) and every batch runs through bjx_process_batch on its HBM
copy.  Prints one JSON line: file bytes, lines, wall time, lines/s, and the
engine-only device time of the same batches (Banner replay not included).
usage: python tools/tail_bench.py [cfg] [lines] [batch_MiB] [dir] [slots]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import workloads as W  # noqa: E402
from banjax_amd import Config, Engine, MockBanner, RegexRateLimiter  # noqa: E402
from banjax_amd.tailer import LogTailer  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
    batch_mib = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    d = sys.argv[4] if len(sys.argv) > 4 else os.environ.get("TMPDIR", "/tmp")
    slots = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    w = W.scaled(getattr(W, cfg.upper()), n)
    t, nb = w.device_lines(0)
    path = os.path.join(d, "bjx_tail_bench.log")
    with open(path, "wb") as f:
        step = 1 << 30
        for o in range(0, nb, step):
            f.write(t[o:min(nb, o + step)].cpu().numpy().tobytes())
    del t
    torch.cuda.empty_cache()
    now = w.now_ns()
    eng = Engine(0)
    lim = RegexRateLimiter(Config.from_yaml(w.rules_yaml), engine=eng, banner=MockBanner())
    # rep 0 warms the engine (binding, workspace, table growth: every IP new);
    # rep 1 is the steady state (the same lines again, every IP known), as in
    # bench.py's timed steps
    res = {}
    for rep in range(2):
        dev_ms = 0.0
        lines = 0
        batches = 0
        t0 = time.perf_counter()
        with LogTailer(path, device=0, from_start=True, batch_bytes=batch_mib << 20, poll_ms=1, slots=slots) as tl:
            got = 0
            while got < nb:
                b = tl.next(timeout_ms=1000)
                if b is None:
                    continue
                # engine only: the Banner replay of the trips is host-side and unchanged
                out = eng.process(lim.ruleset, None, now, device_ptr=b.device_ptr, nbytes=b.n_bytes)
                dev_ms += out.device_ms
                lines += out.n_lines
                got += b.n_bytes
                batches += 1
                tl.release(b)
        wall = time.perf_counter() - t0
        res = {"workload": cfg, "file_bytes": nb, "lines": lines, "batches": batches, "batch_MiB": batch_mib, "slots": slots,
               "wall_s": round(wall, 3), "lines_per_s_tail_inclusive": round(lines / wall, 1),
               "file_to_HBM_GBps": round(nb / wall / 1e9, 2), "engine_device_s": round(dev_ms / 1e3, 3),
               "lines_per_s_engine_only": round(lines / (dev_ms / 1e3), 1), "rep": rep,
               "state": "cold (every IP new)" if rep == 0 else "steady (every IP known)",
               "what": "file (page cache) -> pinned slots -> HBM (the tailer's own stream) -> bjx_process_batch per "
                       "batch, wall clock over the whole file"}
        print(json.dumps(res), flush=True)
    os.unlink(path)
    eng.close()


if __name__ == "__main__":
    main()
