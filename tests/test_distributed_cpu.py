"""IP-sharded multi-GPU orchestration (banjax_amd/distributed.py) over real
torch.distributed collectives: world_size 2, gloo, CPU tensors, with the CPU
stand-in engine of tests/mock_engine.py.  The sharded run must reproduce the
single-process oracle bit for bit: every RuleResult (seenIp, MatchType,
Exceeded) and every trip, in reference order.  Trips-only batches
(copy_results=False) take the trip-list return path (apply_events_trips /
finish_trips) and must give the same trips."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import workloads as W
from banjax_amd import Config
from banjax_amd.distributed import TorchExchange, sharded_batch
from oracle import oracle as O
from tests.mock_engine import MockEngine
from tests.parity import oracle_config

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _chunks(w, n_chunks, per):
    return [w.host_lines(k * per, per) for k in range(n_chunks)]


def _worker(rank, port, wl, n_chunks, per, q, copy):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    w = W.scaled(W.ALL[wl[0]], per * n_chunks, n_ips=wl[1])
    cfg = Config.from_yaml(w.rules_yaml)
    eng = MockEngine(cfg)
    ex = TorchExchange(torch.device("cpu"))
    chunks = _chunks(w, n_chunks, per)
    got = []
    for step in range(n_chunks // WORLD):
        k = step * WORLD + rank  # rank r holds the r-th chunk of each step: stream order = rank order
        t = torch.frombuffer(bytearray(chunks[k]), dtype=torch.uint8)
        out = sharded_batch(eng, None, w.now_ns(0, per), t.data_ptr(), len(chunks[k]), ex, copy_results=copy)
        got.append((k, [list(r) for r in out.results], [(tr.line_idx, tr.rule_idx) for tr in out.trips]))
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("wl,copy", [(("cfg5", 400), True), (("cfg3", 300), True), (("cfg1", 200), True),
                                     (("cfg3", 300), False), (("cfg5", 400), False)])
def test_sharded_rate_limit_matches_single_process(wl, copy):
    n_chunks, per = 4, 1500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, wl, n_chunks, per, q, copy)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(WORLD))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    by_chunk = {}
    for r in range(WORLD):
        for k, results, trips in res[r]:
            by_chunk[k] = (results, trips)
    # reference: one process, chunks in stream order
    w = W.scaled(W.ALL[wl[0]], per * n_chunks, n_ips=wl[1])
    cfg = Config.from_yaml(w.rules_yaml)
    oc = oracle_config(cfg)
    st = O.State()
    n_trips = 0
    for k, data in enumerate(_chunks(w, n_chunks, per)):
        _, ores, _ = st.consume(oc, data, w.now_ns(0, per), cap=(data.count(b"\n") + 1) * (len(cfg.all_rules()) + 1))
        exp = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, r.seen_ip, r.match_type, r.exceeded] for r in ores]
        results, trips = by_chunk[k]
        if copy:
            assert results == exp, "chunk %d" % k
        assert trips == [(r[0], r[1]) for r in exp if r[6]]
        n_trips += len(trips)
    assert n_trips > 0
