"""Benchmark: log lines/sec matched + rate-limited on MI355X (BASELINE.json metric).

A step = one pass of the hot path (consumeLine for every line: framing, header
parse, CheckIsAllowed, every applicable rule's regex, RegexRateLimitStates.Apply,
trip compaction + copy of the trips to the host) over one batch of synthetic
nginx lines already resident in HBM.  Workload (default): cfg3 of
BASELINE.json — 1k per-site rules (100 hosts x 10, host-filtered) + 6 globals,
125M lines per GPU (1B lines at 8 GPUs, weak scaling).  Rate-limit state
persists across steps (steady state: every IP already known after warmup).

Prints ONE JSON line on rank 0.  Multi-GPU: launched by torch.distributed.run,
one rank per GPU.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "log lines/sec matched+rate-limited (node) at 1k rules; HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def cpu_baseline(w, sample_lines):
    """Oracle (C restatement of the reference Go path, oracle/) on one host core
    over the first `sample_lines` lines of the same workload."""
    from oracle import oracle as O
    from tests.parity import oracle_config
    from banjax_amd import Config
    data = w.host_lines(0, sample_lines)
    oc = oracle_config(Config.from_yaml(w.rules_yaml))
    st = O.State()
    t0 = time.perf_counter()
    flags, res, consumed = st.consume(oc, data, w.now_ns(0, sample_lines), cap=sample_lines * 8)
    dt = time.perf_counter() - t0
    return {"value": round(sample_lines / dt, 1), "unit": "lines/s", "cores": 1, "kind": "port",
            "sample": "first %d lines of %s (%.1f MB), oracle/bjx_oracle.c single-threaded (the reference path is one "
                      "goroutine, regex_rate_limiter.go:54-77), %.1f s" % (sample_lines, w.name, len(data) / 1e6, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--lines", type=int, default=0, help="lines per GPU (default: workload size)")
    ap.add_argument("--cpu-sample", type=int, default=300_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import workloads as W
    from banjax_amd import Config, Engine, Ruleset

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    w0 = W.ALL[args.config]
    n_lines = args.lines or w0.n_lines
    w = W.scaled(w0, n_lines, n_ips=w0.n_ips) if args.lines else w0
    # weak scaling: rank r owns lines [r*n, (r+1)*n) of the workload's stream
    first = rank * n_lines
    data, nbytes = w.device_lines(local, first, n_lines)
    torch.cuda.synchronize()
    cfg = Config.from_yaml(w.rules_yaml)
    rs = Ruleset(cfg)
    eng = Engine(local, ip_capacity=1 << 22, state_capacity=1 << 26, ip_arena_bytes=256 << 20)
    eng.set_decision_lists(cfg.decision_entries)
    now = w.now_ns(first, n_lines)

    def step():
        return eng.process(rs, None, now, device_ptr=data.data_ptr(), nbytes=nbytes)

    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    match_ms = sum(o.match_kernel_ms for o in outs) / len(outs)
    dev_ms = sum(o.device_ms for o in outs) / len(outs)
    o = outs[-1]
    phases = eng.phase_ms()
    total_lines = n_lines * world
    value = total_lines / (elapsed / args.steps)
    achieved = nbytes / (match_ms / 1000.0) / 1e9
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "lines/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic nginx banjax_format lines (workloads/synth.hip, seeded), resident in HBM",
            "config": {
                "workload": "%s: %s" % (w0.name, w0.description),
                "rules": len(rs),
                "lines_per_gpu": n_lines,
                "bytes_per_gpu": nbytes,
                "distinct_ips": w.n_ips,
                "rule_results_per_step": o.n_results,
                "rate_limit_events_per_step": o.n_events,
                "trips_per_step": o.n_trips,
                "device_ms_per_step": round(dev_ms, 3),
                "phase_ms_last_step": phases,
                "parallelism": "dp%d: chunk-sharded lines" % world,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_parse_match<false> (framing excluded)",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "match_kernel_ms": round(match_ms, 3),
            },
        }
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(w, args.cpu_sample)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
