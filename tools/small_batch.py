"""Per-batch cost at tailer-sized batches: K device-resident
batches of B synthetic lines each (the tailer's 256 MiB slots hold about 1.7M
cfg3 lines), run once to warm the tables, then timed again in the steady state.
Prints one JSON line: lines/s by wall clock and by device time, the per-batch
wall and device ms, and the phases of the last batch.
usage: python tools/small_batch.py [cfg] [lines_per_batch] [batches]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import workloads as W  # noqa: E402
from banjax_amd import Config, Engine, Ruleset  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 1_700_000
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    w = W.scaled(getattr(W, cfg.upper()), b * k)
    c = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(c)
    eng = Engine(0)
    eng.set_decision_lists(c.decision_entries)
    bufs = [w.device_lines(0, i * b, b) for i in range(k)]
    now = w.now_ns()
    torch.cuda.synchronize()
    res = None
    for rep in range(2):
        walls, devs = [], []
        for t, nb in bufs:
            t0 = time.perf_counter()
            out = eng.process(rs, None, now, device_ptr=t.data_ptr(), nbytes=nb, compact_trips=True)
            walls.append(time.perf_counter() - t0)
            devs.append(out.device_ms)
        res = {"workload": cfg, "lines_per_batch": b, "batches": k, "bytes_per_batch": bufs[0][1], "rep": rep,
               "wall_ms_per_batch": round(1e3 * sum(walls) / k, 3), "device_ms_per_batch": round(sum(devs) / k, 3),
               "lines_per_s_wall": round(b * k / sum(walls), 1), "lines_per_s_device": round(b * k / (sum(devs) / 1e3), 1),
               "phase_ms_last": eng.phase_ms(), "kernel_ms_last": eng.kernel_ms()}
        print(json.dumps(res), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
