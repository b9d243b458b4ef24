"""CPU stand-in for the engine's multi-GPU entry points (test infrastructure).

Implements match / events_partition / events_pack / apply_events / finish (and
the trips-only apply_events_trips / finish_trips) with
the same wire format as include/banjax_gpu.h (bjx_event_line records, u32
rule indices, IP bytes), so banjax_amd.distributed.sharded_batch can run over
real torch.distributed collectives (gloo) on CPU tensors.  Matching comes from
the oracle; Apply is restated here (rate_limit.go:37-78).  Only the
orchestration is under test: ranks, splits, source order, outcome routing.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import struct

from oracle import oracle as O
from tests.parity import oracle_config

REC = struct.Struct("<qIHH")  # bjx_event_line


def ip_hash(ip: bytes) -> int:
    return int.from_bytes(hashlib.blake2b(ip, digest_size=8).digest(), "little") | 1


def go_sub(a, b):
    d = a - b
    return max(min(d, (1 << 63) - 1), -(1 << 63))


class Trip:
    def __init__(self, line_idx, rule_idx):
        self.line_idx, self.rule_idx = line_idx, rule_idx


class Out:
    def __init__(self, n_lines, results, trips):
        self.n_lines, self.results, self.trips, self.n_trips = n_lines, results, trips, len(trips)


class MockEngine:
    def __init__(self, cfg):
        self.cfg = cfg
        self.ocfg = oracle_config(cfg)
        self.rules = cfg.all_rules()  # ruleset index order
        self.state = {}  # ip bytes -> {rule name: [hits, start]}

    # ---- bjx_match_batch
    def match(self, rs, now_ns, device_ptr, nbytes, copy_results=False):
        data = C.string_at(device_ptr, nbytes)
        st = O.State()  # matching only: Apply fields of this fresh state are ignored
        flags, res, consumed = st.consume(self.ocfg, data, now_ns, cap=(data.count(b"\n") + 1) * (len(self.rules) + 1))
        lines = data[:consumed].split(b"\n")[:-1]
        self.n_lines = len(lines)
        self.results = [[r.line_idx, r.rule_id, r.rule_pos, r.skip_host, 0, 0, 0] for r in res]
        self.events = [k for k, r in enumerate(res) if not r.skip_host]  # result index of each event
        self.line_ip, self.line_ts = {}, {}
        for k in self.events:
            j = res[k].line_idx
            if j not in self.line_ip:
                parts = lines[j].split(b" ", 2)
                self.line_ip[j] = parts[1]
                self.line_ts[j] = int(O.parse_float(parts[0])[1] * 1e9)

    # ---- bjx_events_partition
    def events_partition(self, world):
        by_line = {}
        for e, k in enumerate(self.events):
            by_line.setdefault(self.results[k][0], []).append(e)
        self.parts = [[] for _ in range(world)]
        for j in sorted(by_line):
            self.parts[(ip_hash(self.line_ip[j]) >> 32) % world].append((j, by_line[j]))
        return [(len(p), sum(len(ev) for _, ev in p), sum((len(self.line_ip[j]) + 3) & ~3 for j, _ in p))
                for p in self.parts]

    # ---- bjx_events_pack
    def events_pack(self, lines_ptr, events_ptr, bytes_ptr):
        recs, evs, ipb, self.pack_src = bytearray(), bytearray(), bytearray(), []
        for part in self.parts:
            base = len(ipb)
            for j, ev in part:
                ip = self.line_ip[j]
                recs += REC.pack(self.line_ts[j], len(ipb) - base, len(ip), len(ev))
                ipb += ip + b"\0" * (-len(ip) % 4)  # 4-byte aligned IP slots (ABI 5)
                for e in ev:
                    evs += struct.pack("<I", self.results[self.events[e]][1])
                    self.pack_src.append(e)
        C.memmove(lines_ptr, bytes(recs), len(recs))
        C.memmove(events_ptr, bytes(evs), len(evs))
        C.memmove(bytes_ptr, bytes(ipb), len(ipb))

    # ---- bjx_apply_events: Apply (rate_limit.go:37-78) in received (source) order
    def apply_events(self, rs, lines_ptr, events_ptr, bytes_ptr, src_counts, out_ptr):
        nl = sum(c[0] for c in src_counts)
        ne = sum(c[1] for c in src_counts)
        nb = sum(c[2] for c in src_counts)
        recs = C.string_at(lines_ptr, nl * REC.size) if nl else b""
        evs = C.string_at(events_ptr, ne * 4) if ne else b""
        ipb = C.string_at(bytes_ptr, nb) if nb else b""
        out = bytearray()
        i, k, bbase = 0, 0, 0
        for (cl, ce, cb) in src_counts:
            for _ in range(cl):
                ts, off, ln, n_ev = REC.unpack_from(recs, i * REC.size)
                ip = ipb[bbase + off:bbase + off + ln]
                for _ in range(n_ev):
                    rule = self.rules[struct.unpack_from("<I", evs, 4 * k)[0]]
                    states = self.state.get(ip)
                    seen, mt = states is not None, 0
                    if states is None:
                        states = self.state[ip] = {}
                    s = states.get(rule.rule)
                    if s is None:
                        s = states[rule.rule] = [1, ts]
                    elif go_sub(ts, s[1]) > rule.interval:
                        mt, s[0], s[1] = 1, 1, ts
                    else:
                        mt = 2
                        s[0] += 1
                    ex = s[0] > rule.hits_per_interval
                    if ex:
                        s[0] = 0
                    out.append(0x80 | int(seen) | (mt << 1) | (8 if ex else 0))
                    k += 1
                i += 1
            bbase += cb
        C.memmove(out_ptr, bytes(out), len(out))

    # ---- bjx_finish_batch
    def finish(self, outcomes_ptr, copy_results=False):
        o = C.string_at(outcomes_ptr, len(self.pack_src)) if self.pack_src else b""
        per_event = [0] * len(self.events)
        for kk, e in enumerate(self.pack_src):
            per_event[e] = o[kk]
        trips = []
        for e, k in enumerate(self.events):
            v = per_event[e]
            r = self.results[k]
            r[4], r[5], r[6] = v & 1, (v >> 1) & 3, (v >> 3) & 1
            if r[6]:
                trips.append(Trip(r[0], r[1]))
        return Out(self.n_lines, self.results, trips)

    # ---- bjx_apply_events_trips: per source, base + index of its Exceeded events
    def apply_events_trips(self, rs, lines_ptr, events_ptr, bytes_ptr, src_counts, trip_base, trips_ptr):
        ne = sum(c[1] for c in src_counts)
        buf = (C.c_uint8 * max(1, ne))()
        self.apply_events(rs, lines_ptr, events_ptr, bytes_ptr, src_counts, C.addressof(buf))
        out, counts, e0 = [], [], 0
        for k, (_, ce, _) in enumerate(src_counts):
            mine = [trip_base[k] + i for i in range(ce) if buf[e0 + i] & 8]
            out += mine
            counts.append(len(mine))
            e0 += ce
        if out:
            C.memmove(trips_ptr, struct.pack("<%dI" % len(out), *out), 4 * len(out))
        return counts

    # ---- bjx_finish_batch_trips
    def finish_trips(self, trips_ptr, n, emit_bans=False):
        o = bytearray(max(1, len(self.pack_src)))
        for q in (struct.unpack("<%dI" % n, C.string_at(trips_ptr, 4 * n)) if n else ()):
            o[q] = 8
        return self.finish(C.addressof((C.c_uint8 * len(o)).from_buffer(o)))
