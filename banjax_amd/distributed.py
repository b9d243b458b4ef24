"""Multi-GPU batch: matching sharded by chunk, RegexRateLimitStates by IP.

One engine per GPU.  Rank r holds the r-th contiguous chunk of the log and
runs consumeLine up to Apply on it.  The events of each line go to the engine
that owns the line's IP, (ip_hash >> 32) % world.  The owner applies them with
its HBM state and sends one outcome byte per event back, or, when the batch
wants trips only, the packed indices of the events that tripped.  Exchange volume is
one 32 B record per event line, 4 B per event and the IP bytes; it crosses
xGMI once each way as an RCCL all-to-all.

Owners receive records in source-rank order.  Chunks are in stream order, so
the owner's event order is the reference's (line, then rule position) and
every (ip, rule name) state sees its events in order, as the single
goroutine of the reference does (regex_rate_limiter.go:54-77).

The exchange is pluggable: TorchExchange (torch.distributed all_to_all_single:
RCCL over xGMI, or gloo for CPU tests) and ThreadExchange (ranks as threads of
one process, for single-GPU tests of the sharded path).
"""
from __future__ import annotations

import threading
from typing import List, Sequence, Tuple

import torch

from .config import Ruleset
from .engine import BatchOutput

LINE_REC = 16  # sizeof(bjx_event_line)


def _sync(device: torch.device):
    if device.type == "cuda":
        torch.cuda.current_stream(device).synchronize()


class TorchExchange:
    """all_to_all_single over the default process group (backend "nccl" = RCCL)."""

    def __init__(self, device: torch.device, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def counts(self, send: Sequence[Tuple[int, int, int]]) -> List[Tuple[int, int, int]]:
        t = torch.tensor([c for triple in send for c in triple], dtype=torch.int64, device=self.device)
        r = torch.empty_like(t)
        self.dist.all_to_all_single(r, t, group=self.group)
        v = r.tolist()
        return [(v[3 * k], v[3 * k + 1], v[3 * k + 2]) for k in range(self.world)]

    def exchange(self, send: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
        # every rank calls every collective, even with nothing to move
        recv = torch.empty(max(1, sum(recv_splits)), dtype=torch.uint8, device=self.device)
        self.dist.all_to_all_single(recv[:sum(recv_splits)], send[:sum(send_splits)], output_split_sizes=recv_splits,
                                    input_split_sizes=send_splits, group=self.group)
        _sync(self.device)  # the engine reads it on its own HIP stream
        return recv


class ThreadMesh:
    """Shared rendezvous of `world` ranks running as threads of one process."""

    def __init__(self, world: int):
        self.world = world
        self.barrier = threading.Barrier(world)
        self.slots = [None] * world

    def rank(self, r: int, device: torch.device) -> "ThreadExchange":
        return ThreadExchange(self, r, device)


class ThreadExchange:
    def __init__(self, mesh: ThreadMesh, rank: int, device: torch.device):
        self.mesh, self.rank, self.world, self.device = mesh, rank, mesh.world, device

    def _swap(self, item):
        m = self.mesh
        m.slots[self.rank] = item
        m.barrier.wait()
        got = list(m.slots)
        m.barrier.wait()
        return got

    def counts(self, send):
        got = self._swap(list(send))
        return [got[src][self.rank] for src in range(self.world)]

    def exchange(self, send: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
        offs = [0]
        for s in send_splits:
            offs.append(offs[-1] + s)
        got = self._swap((send, offs))
        parts = []
        for src in range(self.world):
            t, o = got[src]
            parts.append(t[o[self.rank]:o[self.rank + 1]].to(self.device))
        recv = torch.empty(max(1, sum(recv_splits)), dtype=torch.uint8, device=self.device)
        if sum(recv_splits):
            recv[:sum(recv_splits)] = torch.cat(parts)
        _sync(self.device)
        self.mesh.barrier.wait()  # every rank has copied its part before buffers are reused
        return recv


def sharded_batch(engine, rs: Ruleset, now_ns: int, device_ptr: int, nbytes: int, ex,
                  copy_results: bool = False, emit_bans: bool = False) -> BatchOutput:
    """consumeLine over this rank's chunk with IP-sharded rate limiting.
    Every rank of `ex` must call this for the same batch step.  emit_bans: the
    rank's trips also get device decision emission (engine.bans(); merge the
    ranks' records with merge_rank_bans)."""
    world, dev = ex.world, ex.device
    engine.match(rs, now_ns, device_ptr, nbytes, copy_results=copy_results)
    send = engine.events_partition(world)
    recv = ex.counts(send)
    tl, te, tb = (sum(c[i] for c in send) for i in range(3))
    lines = torch.empty(max(1, tl * LINE_REC), dtype=torch.uint8, device=dev)
    events = torch.empty(max(1, te * 4), dtype=torch.uint8, device=dev)
    ipb = torch.empty(max(1, tb), dtype=torch.uint8, device=dev)
    engine.events_pack(lines.data_ptr(), events.data_ptr(), ipb.data_ptr())
    r_lines = ex.exchange(lines, [c[0] * LINE_REC for c in send], [c[0] * LINE_REC for c in recv])
    r_events = ex.exchange(events, [c[1] * 4 for c in send], [c[1] * 4 for c in recv])
    r_ipb = ex.exchange(ipb, [c[2] for c in send], [c[2] for c in recv])
    if not copy_results:
        # trips only: each owner returns the packed indices of the tripping
        # events (4 B per trip instead of 1 B per event)
        offs, acc = [], 0
        for c in send:
            offs.append(acc)
            acc += c[1]
        base = [b[0] for b in ex.counts([(o, 0, 0) for o in offs])]
        tr = torch.empty(max(1, sum(c[1] for c in recv)) * 4, dtype=torch.uint8, device=dev)
        tcnt = engine.apply_events_trips(rs, r_lines.data_ptr(), r_events.data_ptr(), r_ipb.data_ptr(), recv, base,
                                         tr.data_ptr())
        mine = [c[0] for c in ex.counts([(c, 0, 0) for c in tcnt])]
        back = ex.exchange(tr, [c * 4 for c in tcnt], [c * 4 for c in mine])
        if emit_bans:
            return engine.finish_trips(back.data_ptr(), sum(mine), emit_bans=True)
        return engine.finish_trips(back.data_ptr(), sum(mine))
    out = torch.empty(max(1, sum(c[1] for c in recv)), dtype=torch.uint8, device=dev)
    engine.apply_events(rs, r_lines.data_ptr(), r_events.data_ptr(), r_ipb.data_ptr(), recv, out.data_ptr())
    back = ex.exchange(out, [c[1] for c in recv], [c[1] for c in send])
    if emit_bans:
        return engine.finish(back.data_ptr(), copy_results=copy_results, emit_bans=True)
    return engine.finish(back.data_ptr(), copy_results=copy_results)


def merge_rank_bans(parts):
    """One sharded step's decision updates and ban-log lines from every rank's
    bjx_batch_bans.  parts: per rank, in stream order, (BanBatch, trips, chunk
    bytes).  Rank r's trips precede rank r+1's in reference order, so per IP
    the highest decision's first trip is the earliest (rank, trip) reaching
    it, and the log is the ranks' logs concatenated.  Returns (records in
    global trip order, [(kind, line)]); a record is (ip, domain, decision,
    expires_ns, n_trips, iptables)."""
    best = {}
    log = []
    for r, (bans, trips, data) in enumerate(parts):
        for rec in bans.ips:
            t = trips[int(rec["trip_idx"])]
            line = bytes(data[t.line_offset:t.line_offset + t.line_len])
            ip = line[t.ip_off:t.ip_off + t.ip_len]
            host = line[t.host_off:t.host_off + t.host_len]
            key = (r, int(rec["trip_idx"]))
            d = int(rec["decision"])
            cur = best.get(ip)
            if cur is None:
                best[ip] = [key, host, d, int(rec["expires_ns"]), int(rec["n_trips"]), int(rec["iptables"])]
                continue
            if d > cur[2]:
                cur[0], cur[1], cur[2] = key, host, d
            cur[4] += int(rec["n_trips"])
            cur[5] |= int(rec["iptables"])
        log.extend(bans.lines())
    recs = sorted(best.items(), key=lambda kv: kv[1][0])
    return [(ip, v[1], v[2], v[3], v[4], v[5]) for ip, v in recs], log
