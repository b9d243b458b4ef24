"""Decision emission per step: one workload's batch run
repeatedly into persistent state, each step timed by wall clock with its trip
count, per-IP record count and ban-log bytes, with emission off for the first
`plain` steps and on (full, then records only) afterwards.
usage: python tools/emit_bench.py [cfg] [plain_steps] [emit_steps] [lines]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import workloads as W  # noqa: E402
from banjax_amd import Config, Engine, Ruleset, _lib  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    plain = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    emit = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    w0 = W.ALL[cfg]
    w = W.scaled(w0, n, n_ips=w0.n_ips) if n else w0
    c = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(c)
    eng = Engine(0, ip_arena_bytes=256 << 20)
    eng.set_decision_lists(c.decision_entries)
    eng.set_ban_options(c.expiring_decision_ttl_seconds, [h for h, v in c.disable_logging.items() if v])
    t, nb = w.device_lines(0)
    now = w.now_ns(0, w.n_lines)
    torch.cuda.synchronize()
    modes = ["plain"] * plain + ["full"] * emit + ["records"] * emit
    for k, m in enumerate(modes):
        t0 = time.perf_counter()
        o = eng.process(rs, None, now, device_ptr=t.data_ptr(), nbytes=nb, emit_bans=m != "plain",
                        ban_log=m == "full", compact_trips=True)
        wall = time.perf_counter() - t0
        rec = {"step": k, "mode": m, "wall_ms": round(wall * 1e3, 3), "device_ms": round(o.device_ms, 3),
               "trips": o.n_trips, "phase_ms": eng.phase_ms()}
        if m != "plain":
            bb = _lib.BanBatch()
            if _lib.lib().bjx_batch_bans(eng._h, ctypes.byref(bb)) == 0:
                rec["records"] = int(bb.n_ips)
                rec["log_bytes"] = int(bb.log_bytes)
        print(json.dumps(rec), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
