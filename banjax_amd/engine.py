"""One MI355X engine (bjx_engine): persistent rate-limit state in HBM plus the
batch pipeline of include/banjax_gpu.h."""
from __future__ import annotations

import ctypes as C
from typing import Iterable, List, Optional, Sequence, Tuple

from . import _lib
from .config import Config, Ruleset


class BatchOutput:
    """Host view of one bjx_process_batch.  The arrays live in engine-owned
    pinned memory valid until the next process(); `trips` / `results` are
    materialized as Python records only when read (trips_array() gives the
    zero-copy numpy view the Banner replay iterates)."""

    def __init__(self, res: _lib.BatchResult, copy_results: bool):
        self.n_lines = res.n_lines
        self.consumed_bytes = res.consumed_bytes
        self.n_results = res.n_results
        self.n_events = res.n_events
        self.n_trips = res.n_trips
        self.device_ms = res.device_ms
        self.match_kernel_ms = res.match_kernel_ms
        self._res = res
        self._trips = None
        self._results = None
        self._copy = copy_results
        self.line_flags = (bytes(C.string_at(res.line_flags, res.n_lines)) if res.n_lines else b"") \
            if copy_results else None

    @property
    def trips(self):
        if self._trips is None:
            self._need_full_trips()
            self._trips = [self._res.trips[i] for i in range(self.n_trips)] if self.n_trips else []
        return self._trips

    def _need_full_trips(self):
        if self.n_trips and not self._res.trips:
            raise ValueError("this batch was run with compact_trips=True: its trips are in trips_compact(), "
                             "not in full bjx_trip records")

    def trips_compact(self):
        """BJX_TRIPS_COMPACT: numpy uint64 words, line byte offset << 24 | rule index (zero-copy)."""
        import numpy as np
        if not self.n_trips or not self._res.trips_compact:
            return np.zeros(0, dtype=np.uint64)
        buf = (C.c_uint64 * self.n_trips).from_address(C.addressof(self._res.trips_compact.contents))
        return np.ctypeslib.as_array(buf)

    def trips_array(self):
        import numpy as np
        if not self.n_trips:
            return np.zeros(0, dtype=np.dtype(_lib.Trip))
        self._need_full_trips()
        buf = (_lib.Trip * self.n_trips).from_address(C.addressof(self._res.trips.contents))
        return np.ctypeslib.as_array(buf)

    @property
    def results(self):
        if not self._copy:
            return None
        if self._results is None:
            self._results = [self._res.results[i] for i in range(self.n_results)] if self.n_results else []
        return self._results


class BanBatch:
    """Host view of bjx_batch_bans: per-IP decision updates (trip order of
    their representative trip) and the LogRegexBan lines of the batch."""

    def __init__(self, bb: _lib.BanBatch):
        import numpy as np
        self.n_ips = bb.n_ips
        self.n_trips = bb.n_trips
        if bb.n_ips:
            arr = (_lib.IpDecision * bb.n_ips).from_address(C.addressof(bb.ips.contents))
            self.ips = np.ctypeslib.as_array(arr).copy()
        else:
            self.ips = np.zeros(0, dtype=np.dtype(_lib.IpDecision))
        self.log = C.string_at(bb.log, bb.log_bytes) if bb.log_bytes else b""
        n = bb.n_trips
        self.log_off = np.ctypeslib.as_array(bb.log_off, shape=(n + 1,)).copy() if n else np.zeros(1, np.uint64)
        self.log_kind = np.ctypeslib.as_array(bb.log_kind, shape=(n,)).copy() if n else np.zeros(0, np.uint8)
        m = bb.n_ips
        self.ip_off = np.ctypeslib.as_array(bb.ip_off, shape=(m + 1,)).copy() if m else np.zeros(1, np.uint64)
        self.ip_bytes = C.string_at(bb.ip_bytes, int(self.ip_off[m])) if m and self.ip_off[m] else b""

    def ip(self, r: int) -> bytes:
        """IP bytes of record r (the Update key)."""
        return self.ip_bytes[int(self.ip_off[r]):int(self.ip_off[r + 1])]

    def lines(self):
        """(kind, line without '\\n') per trip that logs (kind 1 Logger, 2 LoggerTemp)."""
        out = []
        for t in range(self.n_trips):
            k = int(self.log_kind[t])
            if k:
                out.append((k, self.log[int(self.log_off[t]):int(self.log_off[t + 1]) - 1]))
        return out


def _decision_entries(entries):
    entries = list(entries)
    arr = (_lib.DecisionEntry * max(1, len(entries)))()
    keep = []
    for i, (site, dec, ip) in enumerate(entries):
        s = _lib.Str(None, 0) if site is None else _lib.mkstr(site)
        ipb = _lib.mkstr(ip)
        keep.append((s, ipb))
        arr[i] = _lib.DecisionEntry(s, dec, ipb)
    return arr, len(entries), keep


def _ban_options(expiring_ttl_s, disable_logging, tz_offset_s, zone):
    hosts = [h for h in disable_logging]
    arr = (_lib.Str * max(1, len(hosts)))()
    strs = [_lib.mkstr(h) for h in hosts]
    for i, x in enumerate(strs):
        arr[i] = x
    ttl = (int(expiring_ttl_s) * 1_000_000_000) & ((1 << 64) - 1)
    if ttl >= 1 << 63:
        ttl -= 1 << 64
    trans = zone.transitions if zone is not None else []
    off = zone.offset_s if zone is not None else tz_offset_s
    tz = (_lib.TzTransition * max(1, len(trans)))(*[_lib.TzTransition(a, o, 0) for a, o in trans])
    return _lib.BanOptions(ttl, off, 0, arr, len(hosts), tz, len(trans)), (arr, tz, strs)


class Engine:
    def __init__(self, device: int = 0, ip_capacity: int = 0, state_capacity: int = 0, ip_arena_bytes: int = 0):
        L = _lib.lib()
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        opts = _lib.EngineOptions(ip_capacity, state_capacity, ip_arena_bytes)
        rc = L.bjx_engine_create(device, C.byref(opts), C.byref(h), err, 512)
        if rc != _lib.OK:
            raise _lib.BanjaxGpuError(rc, "bjx_engine_create: " + err.value.decode(errors="replace"))
        self._h = h
        self.device = device

    def _check(self, rc, what):
        if rc < 0:
            msg = _lib.lib().bjx_engine_last_error(self._h)
            raise _lib.BanjaxGpuError(rc, "%s: %s" % (what, (msg or b"").decode(errors="replace")))
        return rc

    def set_decision_lists(self, entries: Iterable[Tuple[Optional[str], int, str]]):
        """StaticDecisionLists from config (decision.go:278-374)."""
        arr, n, keep = _decision_entries(entries)
        self._check(_lib.lib().bjx_engine_set_decision_lists(self._h, arr, n), "set_decision_lists")

    def set_ban_options(self, expiring_ttl_s: int, disable_logging: Iterable[str] = (), tz_offset_s: int = 0,
                        zone=None):
        """Banner settings of the device decision emission (bjx_engine_set_ban_options);
        zone: a regex_rate_limiter.Zone (local-zone transitions), else the fixed
        offset tz_offset_s."""
        o, keep = _ban_options(expiring_ttl_s, disable_logging, tz_offset_s, zone)
        self._check(_lib.lib().bjx_engine_set_ban_options(self._h, C.byref(o)), "set_ban_options")

    def bans(self) -> BanBatch:
        """Decision updates and ban-log lines of the last batch (run with emit_bans)."""
        bb = _lib.BanBatch()
        self._check(_lib.lib().bjx_batch_bans(self._h, C.byref(bb)), "batch_bans")
        return BanBatch(bb)

    def process(self, rs: Ruleset, data, now_ns: int, copy_results: bool = False, device_ptr: Optional[int] = None,
                nbytes: Optional[int] = None, emit_bans: bool = False, ban_log: bool = True,
                compact_trips: bool = False) -> BatchOutput:
        """consumeLine over every complete line of `data` (bytes) or of a device
        buffer (device_ptr, nbytes) already resident in HBM.  emit_bans with
        ban_log=False: the per-IP decision records only (BJX_BAN_RECORDS_ONLY).
        compact_trips: trips as 8-byte words (BatchOutput.trips_compact)."""
        res = _lib.BatchResult()
        flags = (_lib.COPY_RESULTS if copy_results else 0) | (_lib.EMIT_BANS if emit_bans else 0) | \
            (_lib.TRIPS_COMPACT if compact_trips else 0)
        if emit_bans and not ban_log:
            flags |= _lib.BAN_RECORDS_ONLY
        if device_ptr is not None:
            rc = _lib.lib().bjx_process_batch(self._h, rs.handle, C.c_void_p(device_ptr), nbytes, now_ns,
                                              flags | _lib.INPUT_DEVICE, C.byref(res))
        else:
            buf = _lib.b(data)
            rc = _lib.lib().bjx_process_batch(self._h, rs.handle, C.c_char_p(buf), len(buf), now_ns, flags,
                                              C.byref(res))
        self._check(rc, "process_batch")
        return BatchOutput(res, copy_results)

    # ---- multi-GPU batch (include/banjax_gpu.h); buffers are device pointers
    def match(self, rs: Ruleset, now_ns: int, device_ptr: int, nbytes: int, copy_results: bool = False):
        """consumeLine up to Apply (bjx_match_batch) over a device buffer."""
        res = _lib.BatchResult()
        flags = (_lib.COPY_RESULTS if copy_results else 0) | _lib.INPUT_DEVICE
        self._check(_lib.lib().bjx_match_batch(self._h, rs.handle, C.c_void_p(device_ptr), nbytes, now_ns, flags,
                                               C.byref(res)), "match_batch")
        return res

    def events_partition(self, n_parts: int) -> List[Tuple[int, int, int]]:
        """Per owner: (event lines, events, IP bytes) this engine sends."""
        arr = (C.c_uint64 * (3 * n_parts))()
        self._check(_lib.lib().bjx_events_partition(self._h, n_parts, arr), "events_partition")
        return [(arr[3 * k], arr[3 * k + 1], arr[3 * k + 2]) for k in range(n_parts)]

    def events_pack(self, lines_ptr: int, events_ptr: int, bytes_ptr: int):
        self._check(_lib.lib().bjx_events_pack(self._h, C.c_void_p(lines_ptr), C.c_void_p(events_ptr),
                                               C.c_void_p(bytes_ptr)), "events_pack")

    def apply_events(self, rs: Ruleset, lines_ptr: int, events_ptr: int, bytes_ptr: int,
                     src_counts: List[Tuple[int, int, int]], out_ptr: int):
        arr = (C.c_uint64 * max(1, 3 * len(src_counts)))()
        for k, (a, b, c) in enumerate(src_counts):
            arr[3 * k], arr[3 * k + 1], arr[3 * k + 2] = a, b, c
        self._check(_lib.lib().bjx_apply_events(self._h, rs.handle, C.c_void_p(lines_ptr), C.c_void_p(events_ptr),
                                                C.c_void_p(bytes_ptr), len(src_counts), arr, C.c_void_p(out_ptr)),
                    "apply_events")

    def apply_events_trips(self, rs: Ruleset, lines_ptr: int, events_ptr: int, bytes_ptr: int,
                           src_counts: List[Tuple[int, int, int]], trip_base: List[int], trips_ptr: int) -> List[int]:
        """Trips-only Apply: per source, its tripping events' packed indices
        (trip_base[k] + index in source k's segment) into trips_ptr, source
        order; returns the per-source counts."""
        n = len(src_counts)
        arr = (C.c_uint64 * max(1, 3 * n))()
        for k, (a, b, c) in enumerate(src_counts):
            arr[3 * k], arr[3 * k + 1], arr[3 * k + 2] = a, b, c
        base = (C.c_uint64 * max(1, n))(*trip_base)
        cnt = (C.c_uint64 * max(1, n))()
        self._check(_lib.lib().bjx_apply_events_trips(self._h, rs.handle, C.c_void_p(lines_ptr), C.c_void_p(events_ptr),
                                                      C.c_void_p(bytes_ptr), n, arr, base, C.c_void_p(trips_ptr), cnt),
                    "apply_events_trips")
        return [cnt[k] for k in range(n)]

    def finish_trips(self, trips_ptr: int, n: int, emit_bans: bool = False) -> BatchOutput:
        res = _lib.BatchResult()
        flags = _lib.EMIT_BANS if emit_bans else 0
        self._check(_lib.lib().bjx_finish_batch_trips(self._h, C.c_void_p(trips_ptr), n, flags, C.byref(res)),
                    "finish_batch_trips")
        return BatchOutput(res, False)

    def finish(self, outcomes_ptr: int, copy_results: bool = False, emit_bans: bool = False) -> BatchOutput:
        res = _lib.BatchResult()
        flags = (_lib.COPY_RESULTS if copy_results else 0) | (_lib.EMIT_BANS if emit_bans else 0)
        self._check(_lib.lib().bjx_finish_batch(self._h, C.c_void_p(outcomes_ptr), flags, C.byref(res)),
                    "finish_batch")
        return BatchOutput(res, copy_results)

    PHASES = ("count", "scan", "resolve", "emit", "capacity", "ip_state_claim", "sort_apply", "trips", "exchange")

    def scan_stats(self):
        out = (C.c_uint64 * 12)()
        _lib.lib().bjx_debug_scan_stats(self._h, out, 12)
        return {"pair_filter_hits": out[0], "literal_hits": out[1], "fallback_lines": out[2], "scan_image_bytes": out[3],
                "dfa_jobs": out[4], "ip_table_slots": out[5], "ips": out[6], "state_table_slots": out[7], "states": out[8],
                "gram_table_hits": out[9], "grouping": out[10], "long_runs": out[11]}

    def state_stats(self):
        """Occupancy of the HBM rate-limit tables (bjx_state_stats_get)."""
        st = _lib.StateStats()
        self._check(_lib.lib().bjx_state_stats_get(self._h, C.byref(st)), "state_stats")
        return {k: getattr(st, k) for k, _ in _lib.StateStats._fields_}

    def phase_ms(self):
        """Device ms of the last batch's phases; "exchange" (a node batch only)
        is the part of "capacity" spent partitioning, packing, moving and
        unpacking the event records."""
        n = len(self.PHASES)
        out = (C.c_double * n)()
        _lib.lib().bjx_debug_phase_ms(self._h, out, n)
        d = {k: round(out[i], 3) for i, k in enumerate(self.PHASES)}
        if not d["exchange"]:
            del d["exchange"]
        return d

    def kernel_ms(self):
        """Device ms of the last batch's k_scan, per-line kernel and DFA-job resolve (HIP events)."""
        out = (C.c_double * 5)()
        _lib.lib().bjx_debug_kernel_ms(self._h, out, 5)
        return {"k_scan": out[0], "k_lines": out[1], "dfa_jobs": out[2]}

    def line_kernel(self):
        """The last batch's per-line kernel: ("k_lines2", window bytes per line), ("k_lines", staging bytes per
        wave), or ("k_parse_match", 0) when every scope is past 128 rules and the per-line fallback took every line."""
        out = (C.c_double * 5)()
        _lib.lib().bjx_debug_kernel_ms(self._h, out, 5)
        names = {1: "k_lines", 2: "k_lines2", 3: "k_parse_match"}
        return names.get(int(out[3])), int(out[4])

    def state_get(self, ip, name):
        hits, start = C.c_int64(), C.c_int64()
        ipb, nb = _lib.b(ip), _lib.b(name)
        rc = self._check(_lib.lib().bjx_state_get(self._h, ipb, len(ipb), nb, len(nb), C.byref(hits), C.byref(start)),
                         "state_get")
        return (hits.value, start.value) if rc == 1 else None

    def state_len(self) -> int:
        return self._check(_lib.lib().bjx_state_len(self._h), "state_len")

    def debug_set_ip_hash_mask(self, mask: int):
        """Test hook: IP hashes become (hash & mask) | 1 (0 = off)."""
        self._check(_lib.lib().bjx_debug_set_ip_hash_mask(self._h, mask), "debug_set_ip_hash_mask")

    def debug_set_claim_budget(self, max_new: int):
        """Test hook: cap the first claim launch per table and batch (0 = off)."""
        self._check(_lib.lib().bjx_debug_set_claim_budget(self._h, max_new), "debug_set_claim_budget")

    def debug_set_slot_cache(self, on: int):
        """Test hook: state-slot cache on (1), off (0), default (-1), from the next batch."""
        self._check(_lib.lib().bjx_debug_set_slot_cache(self._h, on), "debug_set_slot_cache")

    def state_clear(self):
        self._check(_lib.lib().bjx_state_clear(self._h), "state_clear")

    def state_dump(self) -> str:
        n = _lib.lib().bjx_state_dump(self._h, None, 0)
        buf = C.create_string_buffer(n + 1)
        _lib.lib().bjx_state_dump(self._h, buf, n)
        return buf.raw[:n].decode(errors="replace")

    def close(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.bjx_engine_destroy(h)
        self._h = None

    def __del__(self):
        self.close()


class _NodeEngine(Engine):
    """A node's engine: closing it is the node's business."""

    def close(self):
        self._h = None


class Node:
    """The GPUs of one host behind one handle (bjx_node_*): one
    engine per entry of `devices` (repeats allowed), matching sharded by chunk,
    RegexRateLimitStates sharded by IP, the exchange done inside the library.
    Results are in global (reference) order, as one Engine returns them."""

    def __init__(self, devices: Sequence[int], ip_capacity: int = 0, state_capacity: int = 0, ip_arena_bytes: int = 0):
        L = _lib.lib()
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        devs = (C.c_int * len(devices))(*devices)
        opts = _lib.EngineOptions(ip_capacity, state_capacity, ip_arena_bytes)
        rc = L.bjx_node_create(devs, len(devices), C.byref(opts), C.byref(h), err, 512)
        if rc != _lib.OK:
            raise _lib.BanjaxGpuError(rc, "bjx_node_create: " + err.value.decode(errors="replace"))
        self._h = h
        self.devices = list(devices)

    def __len__(self):
        return len(self.devices)

    @property
    def exchange(self) -> str:
        """How the library moves the event records: "rccl" or "copies"."""
        return "rccl" if _lib.lib().bjx_node_exchange_kind(self._h) == 1 else "copies"

    def engine(self, k: int) -> "Engine":
        """Engine k (stats and debug hooks); owned by the node."""
        h = _lib.lib().bjx_node_engine(self._h, k)
        if not h:
            raise IndexError(k)
        e = Engine.__new__(_NodeEngine)
        e._h, e.device, e._node = C.c_void_p(h), self.devices[k], self
        return e

    def _check(self, rc, what):
        if rc < 0:
            msg = _lib.lib().bjx_node_last_error(self._h)
            raise _lib.BanjaxGpuError(rc, "%s: %s" % (what, (msg or b"").decode(errors="replace")))
        return rc

    def set_decision_lists(self, entries: Iterable[Tuple[Optional[str], int, str]]):
        arr, n, keep = _decision_entries(entries)
        self._check(_lib.lib().bjx_node_set_decision_lists(self._h, arr, n), "node_set_decision_lists")

    def set_ban_options(self, expiring_ttl_s: int, disable_logging: Iterable[str] = (), tz_offset_s: int = 0,
                        zone=None):
        o, keep = _ban_options(expiring_ttl_s, disable_logging, tz_offset_s, zone)
        self._check(_lib.lib().bjx_node_set_ban_options(self._h, C.byref(o)), "node_set_ban_options")

    def process(self, rs: Ruleset, data, now_ns: int, copy_results: bool = False, emit_bans: bool = False) -> BatchOutput:
        """consumeLine over the complete lines of a host buffer, split over the engines."""
        res = _lib.BatchResult()
        flags = (_lib.COPY_RESULTS if copy_results else 0) | (_lib.EMIT_BANS if emit_bans else 0)
        buf = _lib.b(data)
        self._check(_lib.lib().bjx_node_process_batch(self._h, rs.handle, C.c_char_p(buf), len(buf), now_ns, flags,
                                                      C.byref(res)), "node_process_batch")
        return BatchOutput(res, copy_results)

    def process_chunks(self, rs: Ruleset, chunks: Sequence[Tuple[int, int]], now_ns: int, copy_results: bool = False,
                       emit_bans: bool = False, compact_trips: bool = False) -> BatchOutput:
        """chunks[k] = (device pointer on engine k's GPU, bytes); all but the last end in '\\n'."""
        res = _lib.BatchResult()
        flags = (_lib.COPY_RESULTS if copy_results else 0) | (_lib.EMIT_BANS if emit_bans else 0) | _lib.INPUT_DEVICE | \
            (_lib.TRIPS_COMPACT if compact_trips else 0)
        ptrs = (C.c_void_p * len(chunks))(*[p for p, _ in chunks])
        lens = (C.c_size_t * len(chunks))(*[n for _, n in chunks])
        self._check(_lib.lib().bjx_node_process_chunks(self._h, rs.handle, ptrs, lens, now_ns, flags, C.byref(res)),
                    "node_process_chunks")
        return BatchOutput(res, copy_results)

    def bans(self) -> BanBatch:
        bb = _lib.BanBatch()
        self._check(_lib.lib().bjx_node_batch_bans(self._h, C.byref(bb)), "node_batch_bans")
        return BanBatch(bb)

    def state_get(self, ip, name):
        hits, start = C.c_int64(), C.c_int64()
        ipb, nb = _lib.b(ip), _lib.b(name)
        rc = self._check(_lib.lib().bjx_node_state_get(self._h, ipb, len(ipb), nb, len(nb), C.byref(hits),
                                                       C.byref(start)), "node_state_get")
        return (hits.value, start.value) if rc == 1 else None

    def state_len(self) -> int:
        return self._check(_lib.lib().bjx_node_state_len(self._h), "node_state_len")

    def state_stats(self):
        st = _lib.StateStats()
        self._check(_lib.lib().bjx_node_state_stats_get(self._h, C.byref(st)), "node_state_stats")
        return {k: getattr(st, k) for k, _ in _lib.StateStats._fields_}

    def state_clear(self):
        self._check(_lib.lib().bjx_node_state_clear(self._h), "node_state_clear")

    def state_dump(self) -> str:
        n = _lib.lib().bjx_node_state_dump(self._h, None, 0)
        buf = C.create_string_buffer(n + 1)
        _lib.lib().bjx_node_state_dump(self._h, buf, n)
        return buf.raw[:n].decode(errors="replace")

    def close(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.bjx_node_destroy(h)
        self._h = None

    def __del__(self):
        self.close()
