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
import re
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
    over the first `sample_lines` lines of the same workload, plus the N-core
    IP-sharded variant (oracle/shard_worker.py, one process per core)."""
    from oracle import oracle as O
    from tests.parity import oracle_config
    from banjax_amd import Config
    data = w.host_lines(0, sample_lines)
    oc = oracle_config(Config.from_yaml(w.rules_yaml))
    st = O.State()
    t0 = time.perf_counter()
    flags, res, consumed = st.consume(oc, data, w.now_ns(0, sample_lines), cap=sample_lines * 8)
    dt = time.perf_counter() - t0
    out = {"value": round(sample_lines / dt, 1), "unit": "lines/s", "cores": 1, "kind": "port",
           "sample": "first %d lines of %s (%.1f MB), oracle/bjx_oracle.c single-threaded (the reference path is one "
                     "goroutine, regex_rate_limiter.go:54-77), %.1f s" % (sample_lines, w.name, len(data) / 1e6, dt)}
    try:
        out["n_core"] = cpu_baseline_sharded(w, sample_lines)
    except Exception as e:  # the 1-core figure stands on its own
        out["n_core"] = {"error": str(e)[:200]}
    return out


def cgroup_cpus():
    """CPUs of quota this process's cgroup grants (cgroup v2 cpu.max), or None."""
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if quota == "max" else max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        return None


def cpu_baseline_sharded(w, sample_lines):
    """N worker processes, each running the oracle over its IP-hash shard of
    N x sample_lines / 4 lines; throughput = lines / slowest worker.  N = every
    CPU this process may run on, capped by its cgroup's CPU quota (the GPU box
    shows 256 CPUs but grants 16 of quota: more workers than that only
    time-slice the same 16)."""
    import subprocess
    import tempfile
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    quota = cgroup_cpus()
    n = max(1, min(avail, quota) if quota else avail)
    total = sample_lines * n // 4
    data = w.host_lines(0, total)
    with tempfile.TemporaryDirectory() as d:
        dp, yp = os.path.join(d, "sample.log"), os.path.join(d, "rules.yaml")
        open(dp, "wb").write(data)
        open(yp, "w").write(w.rules_yaml)
        env = dict(os.environ, OMP_NUM_THREADS="1")
        procs = [subprocess.Popen([sys.executable, "-m", "oracle.shard_worker", dp, str(k), str(n),
                                   str(w.now_ns(0, total)), yp], cwd=ROOT, env=env, stdout=subprocess.PIPE)
                 for k in range(n)]
        res = [json.loads(p.communicate()[0].decode().strip().splitlines()[-1]) for p in procs]
    slowest = max(r["seconds"] for r in res)
    return {"value": round(sum(r["lines"] for r in res) / slowest, 1), "unit": "lines/s", "cores": n,
            "host_cpus": os.cpu_count(), "affinity_cpus": avail, "cgroup_cpu_quota": quota, "kind": "port",
            "sample": "first %d lines of %s, IP-hash sharded over %d oracle processes (per-IP order kept), "
                      "slowest shard %.1f s" % (total, w.name, n, slowest)}


def pmc_traffic(kernel):
    """HBM GB per launch of `kernel` from the committed rocprofv3 PMC passes
    over this same command (profiles/pmc_traffic.json, written from the pass
    CSVs under profiles/<round>/ by tools/pmc_traffic.py): FETCH_SIZE x 2
    (gfx950 reports half of a wide streaming read, MI355X_MICROARCH.md "HBM")
    + WRITE_SIZE, both in KB."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    k = d.get("kernels", {}).get(kernel)
    return (k["hbm_gb_per_launch"], d["source"]) if k else (None, None)


KERNELS = {
    "k_scan": "k_scan (framing + line index + literal prefilter over every byte of the batch)",
    "k_lines2": "k_lines2 (one lane per line: header from a %d B window of the line, host, CheckIsAllowed, rule "
                "decisions from the literal hits; undecided pairs emitted as DFA-job windows)",
    "k_lines": "k_lines (the per-line fallback for rulesets past k_lines2's tables: each wave's lines staged in "
               "%d B of LDS, the host's rules walked entry by entry; undecided pairs emitted as DFA jobs)",
    "dfa_jobs": "DFA-job sort + k_dfa / k_nfa (the (line, rule) pairs the literals cannot decide)",
    "k_parse_match": "k_parse_match (scopes past 128 rules: one lane per line parses it and decides the rules its "
                     "literal hits name plus the anchored / ALWAYS ones by their automata, decide_wide)",
}


def kernel_desc(dom, line_kernel):
    if dom != "k_lines":
        return KERNELS[dom]
    name, nb = line_kernel
    t = KERNELS[name or "k_lines2"]
    return t % nb if "%d" in t else t


def roofline(kms, nbytes, args, line_kernel=("k_lines2", 112)):
    """The dominant kernel of the timed steps (HIP events on the engine stream,
    averaged over the timed steps): algorithmic bytes = the batch's log bytes
    (every line read once) / its average time."""
    default = args.config == "cfg3" and not args.lines
    dom = max(kms, key=kms.get)
    ms = kms[dom]
    achieved = nbytes / (ms / 1000.0) / 1e9
    traffic, src = pmc_traffic(dom) if default else (None, None)
    r = {
        "bound": "hbm",
        "kernel": kernel_desc(dom, line_kernel),
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_GB_per_launch": round(nbytes / 1e9, 3),
        "kernel_ms": round(ms, 3),
        "kernels_ms": {k: round(v, 3) for k, v in kms.items()},
        "k_scan": {"ms": round(kms["k_scan"], 3), "achieved": round(nbytes / (kms["k_scan"] / 1000.0) / 1e9, 1),
                   "frac": round(nbytes / (kms["k_scan"] / 1000.0) / 1e9 / HBM_PEAK_GBS, 4)},
    }
    if src:
        r["traffic_source"] = src + ": rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, same command, GB per launch"
    return r


def rank_plan(world, rank, local, node_engines, exchange, n_devices, n_lines, gpus=1):
    """Which engines this rank drives and which lines each engine holds.

    node mode (N>1 with --exchange node, or --node-engines > 1, or a single
    process started as `bench.py --gpus N` with N > 1 and no WORLD_SIZE): rank
    0 drives every engine through one bjx_node, engine k on device k %
    n_devices holding lines [k n_lines, (k + 1) n_lines); the other ranks drive
    nothing and only join the barriers.  Otherwise each rank drives one engine
    on its local GPU over lines [rank n_lines, (rank + 1) n_lines) (weak
    scaling).  A single process asked for more GPUs than it sees fails (the
    line would otherwise report fewer GPUs than were asked for)."""
    if world == 1 and gpus > 1:
        if n_devices < gpus:
            raise SystemExit("bench.py --gpus %d: only %d device(s) visible" % (gpus, n_devices))
        if node_engines and node_engines != gpus:
            raise SystemExit("bench.py: --gpus %d and --node-engines %d disagree" % (gpus, node_engines))
        node_engines = gpus
    node_mode = (world > 1 and exchange == "node") or node_engines > 1
    drives = not node_mode or rank == 0
    n_parts = world if world > 1 else max(1, node_engines)
    devices = [k % n_devices for k in range(n_parts)]
    if node_mode:
        chunks = [(devices[k], k * n_lines, n_lines) for k in range(n_parts)] if drives else []
    else:
        chunks = [(local, rank * n_lines, n_lines)]
    return {"node_mode": node_mode, "drives": drives, "n_parts": n_parts, "devices": devices, "chunks": chunks}


def timed_region(dist, step, sync_all, steps, clock_device):
    """K steps bracketed by a barrier + device sync on both sides; the max over
    ranks of the wall time (every rank calls this the same number of times, a
    rank that drives nothing with a no-op step)."""
    if dist:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    outs = [step() for _ in range(steps)]
    sync_all()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        import torch
        t = torch.tensor([elapsed], device=clock_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, outs


def tail_inclusive(workload):
    """The committed tail-inclusive measurement for this workload (file ->
    pinned -> HBM -> engine, tools/tail_bench.py on the box), reported beside
    the HBM-resident value, never as it."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_tail", "tail_inclusive.json")
    if workload != "cfg3" or not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    st = t["steady"]
    return {"lines_per_s": st["lines_per_s_tail_inclusive"], "file_to_HBM_GBps": st["file_to_HBM_GBps"],
            "lines": st["lines"], "batch_MiB": st["batch_MiB"], "engine_only_lines_per_s": st["lines_per_s_engine_only"],
            "bound": t["parts"]["reading"], "source": "profiles/r06_tail/tail_inclusive.json (%s)" % t["command"],
            "what": "not measured in this run: the committed tools/tail_bench.py result on the same workload"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--lines", type=int, default=0, help="lines per GPU (default: workload size)")
    ap.add_argument("--cpu-sample", type=int, default=600_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--bans", type=int, default=0,
                    help="1: each step also emits the decision updates and ban-log lines of its trips on the device "
                         "(BJX_EMIT_BANS, copied to pinned host memory); 0: trip list only")
    ap.add_argument("--bans-steps", type=int, default=3,
                    help="after the timed region, steps timed again with decision emission on (reported next to value)")
    ap.add_argument("--node-engines", type=int, default=0,
                    help="single process: one bjx_node of this many engines over the visible GPUs (round-robin), "
                         "e.g. to rehearse the N>1 node path on one GPU")
    ap.add_argument("--trips", choices=("compact", "full"), default="compact",
                    help="compact: the trip list crosses PCIe as 8-byte words (line byte offset, rule index: "
                         "BJX_TRIPS_COMPACT; the host has the bytes for the rest); full: 56-byte bjx_trip records")
    ap.add_argument("--exchange", choices=("node", "rccl"), default="node",
                    help="N>1: node = rank 0 drives every local GPU through one bjx_node (the library moves the event "
                         "records over xGMI; the Go host's one-process shape), the other ranks only join the barriers; "
                         "rccl = every rank drives its own engine and the records move by torch.distributed all-to-all")
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
    if world > 1 and args.gpus not in (1, world):
        raise SystemExit("bench.py --gpus %d under %d launched ranks" % (args.gpus, world))
    P = rank_plan(world, rank, local, args.node_engines, args.exchange, torch.cuda.device_count(), n_lines, args.gpus)
    node_mode, drives, n_parts, devices = P["node_mode"], P["drives"], P["n_parts"], P["devices"]
    first = rank * n_lines
    chunks, keep = [], []
    if node_mode and drives:
        for dev, lo, n in P["chunks"]:
            with torch.cuda.device(dev):
                t, nb = w.device_lines(dev, lo, n)
                torch.cuda.synchronize()
            keep.append(t)
            chunks.append((t.data_ptr(), nb))
        data, nbytes = keep[0], chunks[0][1]
    else:
        data, nbytes = w.device_lines(local, first, n_lines)
    torch.cuda.synchronize()
    cfg = Config.from_yaml(w.rules_yaml)
    from banjax_amd import _lib
    _lib.lib()
    tc = time.perf_counter()
    rs = Ruleset(cfg)  # cold: first compile of these patterns in this process (reload = cached patterns only)
    compile_ms = (time.perf_counter() - tc) * 1000.0
    node = None
    disable = [h for h, v in cfg.disable_logging.items() if v]
    if node_mode:
        if drives:
            from banjax_amd import Node
            node = Node(devices, ip_arena_bytes=256 << 20)
            node.set_decision_lists(cfg.decision_entries)
            node.set_ban_options(cfg.expiring_decision_ttl_seconds, disable)
            eng = node.engine(0)
        now = w.now_ns(0, n_lines * n_parts)
    else:
        eng = Engine(local, ip_arena_bytes=256 << 20)  # IP / state tables size themselves to the stream
        eng.set_decision_lists(cfg.decision_entries)
        eng.set_ban_options(cfg.expiring_decision_ttl_seconds, disable)
        now = w.now_ns(first, n_lines)
    bans = bool(args.bans)

    ex = None
    if world > 1 and not node_mode:
        from banjax_amd.distributed import TorchExchange, sharded_batch
        ex = TorchExchange(torch.device("cuda", local))

    compact = args.trips == "compact"

    def step():
        if node_mode:
            return node.process_chunks(rs, chunks, now, emit_bans=bans, compact_trips=compact) if drives else None
        if ex is None:
            return eng.process(rs, None, now, device_ptr=data.data_ptr(), nbytes=nbytes, emit_bans=bans,
                               compact_trips=compact)
        return sharded_batch(eng, rs, now, data.data_ptr(), nbytes, ex, emit_bans=bans)

    def sync_all():
        if node_mode and drives:
            for d in sorted(set(devices)):
                torch.cuda.synchronize(d)
        else:
            torch.cuda.synchronize()

    # the first step goes into empty IP / state tables (every IP and (ip, rule
    # name) state of the batch is new): timed on its own, with its phases
    cold = None
    for wi in range(args.warmup):
        if wi == 0:
            sync_all()
            tc0 = time.perf_counter()
            step()
            sync_all()
            cold = {"ms": round((time.perf_counter() - tc0) * 1000.0, 3)}
            if drives:
                cold["phase_ms"] = eng.phase_ms()
                st0 = node.state_stats() if node else eng.state_stats()
                cold["new_ips"], cold["new_states"] = st0.get("ips"), st0.get("states")
        else:
            step()
    kacc = {"k_scan": 0.0, "k_lines": 0.0, "dfa_jobs": 0.0}

    def timed_step():
        o = step()
        if drives:  # HIP-event times of the step's kernels (host reads only, no sync)
            for k, v in eng.kernel_ms().items():
                kacc[k] += v
        return o

    elapsed, outs = timed_region(dist, timed_step, sync_all, args.steps, "cuda")
    ms_per_step = elapsed * 1000.0 / args.steps
    if not drives:  # node mode, rank > 0: only the barriers and the max-over-ranks clock
        if args.bans_steps > 0 and not bans:
            timed_region(dist, step, sync_all, args.bans_steps, "cuda")
        dist.barrier()
        dist.destroy_process_group()
        return
    match_ms = sum(o.match_kernel_ms for o in outs) / len(outs)
    dev_ms = sum(o.device_ms for o in outs) / len(outs)
    o = outs[-1]
    phases = eng.phase_ms()
    stats = eng.scan_stats()
    state_stats = node.state_stats() if node else eng.state_stats()
    # the same step with the Banner's work on the device too: per-IP decision
    # updates and every LogRegexBan line, copied to pinned host memory
    dec = None
    if args.bans_steps > 0 and not bans:
        bans = True
        # untimed, as many steps as the plain run took: the emission's
        # first-use allocations (pinned host buffers grown to the largest
        # output of the steps' cycle: cfg5's trip count repeats every third
        # step, cfg3 has a trip burst every few dozen)
        for _ in range(max(args.bans_steps, args.warmup + args.steps)):
            step()
        el2, _ = timed_region(dist, step, sync_all, args.bans_steps, "cuda")
        bans = False
        dec = {"value": round(n_lines * n_parts / (el2 / args.bans_steps), 1), "unit": "lines/s",
               "ms_per_step": round(el2 * 1000.0 / args.bans_steps, 3), "steps": args.bans_steps,
               "what": "each step also builds the per-IP DynamicDecisionLists updates and all LogRegexBan JSON lines "
                       "on the device and copies them to pinned host memory (BJX_EMIT_BANS)"}
        if not node_mode and not dist and ex is None:
            # the host's side of the last step: Update per record into an empty
            # decision map, ban-log lines appended to a file (workloads/host_apply.c)
            import ctypes
            import tempfile
            from banjax_amd import _lib as bl
            bb = bl.BanBatch()
            if bl.lib().bjx_batch_bans(eng._h, ctypes.byref(bb)) == 0:
                fd, path = tempfile.mkstemp(prefix="bjx_banlog_", dir="/tmp")
                os.close(fd)
                try:
                    secs, changed = W.host_apply(bb, path)
                finally:
                    os.unlink(path)
                dec["host_apply"] = {
                    "ms": round(secs * 1000.0, 3), "records": int(bb.n_ips), "entries_changed": int(changed),
                    "log_bytes": int(bb.log_bytes),
                    "step_plus_host_lines_per_s": round(n_lines / (el2 / args.bans_steps + secs), 1),
                    "what": "one step's per-IP records applied by a compiled stand-in for the Go host "
                            "(DynamicDecisionLists.Update into an empty open-addressing map keyed by the IP "
                            "bytes, decision.go:404-439) and its LogRegexBan lines appended to a file in /tmp "
                            "(iptables.go:179-228); serial after the step (a pipelined host overlaps it with "
                            "the next batch)"}
    # the decision records alone (BJX_BAN_RECORDS_ONLY: no LogRegexBan lines
    # built or copied), single-engine runs
    rec = None
    if args.bans_steps > 0 and not args.bans and ex is None and not node_mode and not dist:
        for _ in range(args.bans_steps):  # untimed, as above
            eng.process(rs, None, now, device_ptr=data.data_ptr(), nbytes=nbytes, emit_bans=True, ban_log=False)
        sync_all()
        t2 = time.perf_counter()
        for _ in range(args.bans_steps):
            eng.process(rs, None, now, device_ptr=data.data_ptr(), nbytes=nbytes, emit_bans=True, ban_log=False)
        sync_all()
        el3 = time.perf_counter() - t2
        rec = {"value": round(n_lines / (el3 / args.bans_steps), 1), "unit": "lines/s",
               "ms_per_step": round(el3 * 1000.0 / args.bans_steps, 3), "steps": args.bans_steps,
               "what": "each step also builds the per-IP DynamicDecisionLists updates on the device and copies them "
                       "to pinned host memory, without the LogRegexBan lines (BJX_EMIT_BANS | BJX_BAN_RECORDS_ONLY)"}
    # empty tables again, workspace warm: one step that creates every IP and
    # state of the batch (the new-IP path without the engine's first
    # allocations), single-engine runs
    cold_clear = None
    if not node_mode and not dist and ex is None:
        eng.state_clear()
        sync_all()
        tcc = time.perf_counter()
        step()
        sync_all()
        cold_clear = {"ms": round((time.perf_counter() - tcc) * 1000.0, 3), "phase_ms": eng.phase_ms(),
                      "what": "one step right after bjx_state_clear: empty IP / state tables (their capacity kept), "
                              "the per-line workspace already allocated; every IP and state of the batch is created"}
    total_lines = n_lines * n_parts
    value = total_lines / (elapsed / args.steps)
    kms = {k: v / args.steps for k, v in kacc.items()}
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "lines/s",
            "n_gpus": len(set(devices)),
            "engines": n_parts,
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
                "ruleset_compile_ms_cold": round(compile_ms, 1),
                "lines_per_gpu": n_lines,
                "bytes_per_gpu": nbytes,
                "distinct_ips": stats["ips"],
                "ip_pool": w.n_ips,
                "rule_results_per_step_rank0": o.n_results,
                "rate_limit_events_per_step_rank0": o.n_events,
                "trips_per_step_rank0": o.n_trips,
                "trip_records": ("8-byte words (line byte offset << 24 | rule index, BJX_TRIPS_COMPACT)" if compact
                                 else "56-byte bjx_trip records"),
                "decision_emission": ("device: per-IP decision updates + LogRegexBan JSON lines, in the step"
                                      if bans else "off (trip list only)"),
                "device_ms_per_step_rank0": round(dev_ms, 3),
                "pipeline_GBps_rank0": round(nbytes / (ms_per_step / 1000.0) / 1e9, 1),
                "phase_ms_last_step_rank0": phases,
                "scan_stats_last_step_rank0": stats,
                "state_tables": state_stats,
                "parallelism": ("dp%d: chunk-sharded match, IP-hash-sharded rate-limit state, %s" % (
                    n_parts, "one bjx_node (rank 0) of %d engines moving the event records between them with %s" % (
                        n_parts, "one RCCL group of ncclSend/ncclRecv over xGMI" if node is not None and node.exchange == "rccl"
                        else "device copies (engines sharing a GPU)") if node_mode else "RCCL all-to-all of the event records"))
                if n_parts > 1 else "dp1",
            },
            "roofline": roofline(kms, nbytes, args, eng.line_kernel()),
        }
        if cold:
            cold["what"] = ("wall time of the first warm-up step, into empty IP / state tables: every IP and "
                            "(ip, rule name) state of the batch is created (rate_limit.go:45-51); phases of "
                            "engine 0")
            line["cold_first_step"] = cold
        if cold_clear:
            line["cold_step_after_clear"] = cold_clear
        mp_ms = phases["count"] + phases["scan"] + phases["resolve"]
        line["roofline"]["match_pass"] = {
            "kernels": "k_nl_count_wt + k_scan + k_lines + DFA-job sort + k_dfa / k_nfa (phases count+scan+resolve)",
            "ms": round(mp_ms, 3), "achieved": round(nbytes / (mp_ms / 1000.0) / 1e9, 1),
            "frac": round(nbytes / (mp_ms / 1000.0) / 1e9 / HBM_PEAK_GBS, 4)}
        if dec:
            line["with_decision_emission"] = dec
        if rec:
            line["with_decision_records_only"] = rec
        tail = tail_inclusive(w0.name) if n_parts == 1 else None
        if tail:
            line["tail_inclusive"] = tail
        if not args.no_cpu_baseline and n_parts == 1:
            line["cpu_baseline"] = cpu_baseline(w, args.cpu_sample)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
