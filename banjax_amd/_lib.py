"""ctypes binding of libbanjax_gpu.so (include/banjax_gpu.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, the calls below raise.  Build it with `python -m banjax_amd.build`
(or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# BJX_LIB_PATH: another build of the library (timing experiments only)
LIB_PATH = os.environ.get("BJX_LIB_PATH") or os.path.join(HERE, "lib", "libbanjax_gpu.so")

OK = 0
ERR_REGEX, ERR_ARG, ERR_DEVICE, ERR_NOMEM, ERR_TOO_COMPLEX, ERR_CAPACITY, ERR_DECISION = -1, -2, -3, -4, -5, -6, -7
TAIL_STOPPED, ERR_IO = -8, -9
INPUT_DEVICE, COPY_RESULTS, EMIT_BANS, BAN_RECORDS_ONLY, TRIPS_COMPACT = 1, 2, 4, 8, 16


class Str(C.Structure):
    _fields_ = [("ptr", C.c_char_p), ("len", C.c_size_t)]


class RuleSpec(C.Structure):
    _fields_ = [("name", Str), ("regex", Str), ("interval_ns", C.c_int64), ("hits_per_interval", C.c_int64),
                ("decision", C.c_int32), ("hosts_to_skip", C.POINTER(Str)), ("n_hosts_to_skip", C.c_size_t)]


class SiteRules(C.Structure):
    _fields_ = [("host", Str), ("rules", C.POINTER(RuleSpec)), ("n_rules", C.c_size_t)]


class EngineOptions(C.Structure):
    _fields_ = [("ip_capacity", C.c_uint64), ("state_capacity", C.c_uint64), ("ip_arena_bytes", C.c_uint64)]


class DecisionEntry(C.Structure):
    _fields_ = [("site", Str), ("decision", C.c_int32), ("ip", Str)]


class RuleResult(C.Structure):
    _fields_ = [("line_idx", C.c_uint64), ("rule_idx", C.c_uint32), ("rule_pos", C.c_uint16),
                ("skip_host", C.c_uint8), ("seen_ip", C.c_uint8), ("match_type", C.c_uint8),
                ("exceeded", C.c_uint8), ("_pad", C.c_uint8 * 2)]


class Trip(C.Structure):
    _fields_ = [("line_idx", C.c_uint64), ("line_offset", C.c_uint64), ("line_len", C.c_uint32),
                ("rule_idx", C.c_uint32), ("ts_ns", C.c_int64), ("ip_off", C.c_uint32), ("ip_len", C.c_uint32),
                ("host_off", C.c_uint32), ("host_len", C.c_uint32), ("rest_off", C.c_uint32),
                ("decision", C.c_int32)]


class BatchResult(C.Structure):
    _fields_ = [("n_lines", C.c_uint64), ("consumed_bytes", C.c_uint64), ("n_results", C.c_uint64),
                ("n_events", C.c_uint64), ("n_trips", C.c_uint64), ("line_flags", C.POINTER(C.c_uint8)),
                ("results", C.POINTER(RuleResult)), ("trips", C.POINTER(Trip)), ("device_ms", C.c_double),
                ("match_kernel_ms", C.c_double), ("trips_compact", C.POINTER(C.c_uint64))]


class EventLine(C.Structure):
    """bjx_event_line: one rate-limit record exchanged between GPUs (16 B)."""
    _fields_ = [("ts_ns", C.c_int64), ("ip_off", C.c_uint32), ("ip_len", C.c_uint16), ("n_events", C.c_uint16)]


class TzTransition(C.Structure):
    _fields_ = [("utc_start_s", C.c_int64), ("offset_s", C.c_int32), ("_pad", C.c_int32)]


class BanOptions(C.Structure):
    _fields_ = [("expiring_ttl_ns", C.c_int64), ("tz_offset_s", C.c_int32), ("_pad", C.c_uint32),
                ("disable_logging", C.POINTER(Str)), ("n_disable_logging", C.c_size_t),
                ("tz_transitions", C.POINTER(TzTransition)), ("n_tz_transitions", C.c_size_t)]


class IpDecision(C.Structure):
    _fields_ = [("trip_idx", C.c_uint64), ("n_trips", C.c_uint64), ("expires_ns", C.c_int64),
                ("decision", C.c_int32), ("iptables", C.c_uint32)]


class BanBatch(C.Structure):
    _fields_ = [("n_ips", C.c_uint64), ("ips", C.POINTER(IpDecision)), ("n_trips", C.c_uint64),
                ("log", C.c_void_p), ("log_bytes", C.c_uint64), ("log_off", C.POINTER(C.c_uint64)),
                ("log_kind", C.POINTER(C.c_uint8)), ("ip_bytes", C.c_void_p), ("ip_off", C.POINTER(C.c_uint64))]


class TailerOptions(C.Structure):
    _fields_ = [("device", C.c_int32), ("from_start", C.c_int32), ("slots", C.c_uint32), ("poll_ms", C.c_uint32),
                ("batch_bytes", C.c_uint64)]


class TailBatch(C.Structure):
    _fields_ = [("slot", C.c_uint32), ("reopened", C.c_uint32), ("host_bytes", C.c_void_p),
                ("device_bytes", C.c_void_p), ("n_bytes", C.c_uint64), ("file_offset", C.c_uint64)]


# every symbol include/banjax_gpu.h declares
EXPORTS = [
    "bjx_abi_version", "bjx_ruleset_compile", "bjx_ruleset_release", "bjx_ruleset_num_rules",
    "bjx_ruleset_rule_info", "bjx_engine_create", "bjx_engine_destroy", "bjx_engine_set_decision_lists",
    "bjx_process_batch", "bjx_state_get", "bjx_state_len", "bjx_state_clear", "bjx_state_dump",
    "bjx_engine_last_error", "bjx_match_batch", "bjx_events_partition", "bjx_events_pack", "bjx_apply_events",
    "bjx_finish_batch", "bjx_apply_events_trips", "bjx_finish_batch_trips", "bjx_tailer_open", "bjx_tailer_next", "bjx_tailer_release", "bjx_tailer_stats",
    "bjx_tailer_close", "bjx_engine_set_ban_options", "bjx_batch_bans", "bjx_state_stats_get",
    "bjx_node_create", "bjx_node_destroy", "bjx_node_size", "bjx_node_engine", "bjx_node_last_error", "bjx_node_set_decision_lists",
    "bjx_node_set_ban_options", "bjx_node_process_batch", "bjx_node_process_chunks", "bjx_node_batch_bans",
    "bjx_node_state_get", "bjx_node_state_len", "bjx_node_state_dump", "bjx_node_state_stats_get",
    "bjx_node_state_clear", "bjx_node_exchange_kind",
]


class StateStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("ips", "ip_slots", "states", "state_slots", "arena_bytes", "arena_capacity",
                                            "device_bytes", "rehashes")]

_lib = None


class BanjaxGpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BanjaxGpuError(ERR_DEVICE, "libbanjax_gpu.so not built (run __graft_entry__.build()); "
                                         "there is no CPU fallback")
    # torch wheels bundle their own libamdhip64.so.7 (same soname as
    # /opt/rocm's): load torch first so the process has ONE HIP runtime and
    # device buffers/streams pass freely between torch and the engine.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz = C.c_void_p, C.c_size_t
    L.bjx_abi_version.restype = C.c_int
    L.bjx_ruleset_compile.restype = C.c_int
    L.bjx_ruleset_compile.argtypes = [C.POINTER(RuleSpec), sz, C.POINTER(SiteRules), sz, C.POINTER(vp),
                                      C.POINTER(C.c_int64), C.c_char_p, sz]
    L.bjx_ruleset_release.argtypes = [vp]
    L.bjx_ruleset_num_rules.restype = sz
    L.bjx_ruleset_num_rules.argtypes = [vp]
    L.bjx_ruleset_rule_info.restype = C.c_int
    L.bjx_ruleset_rule_info.argtypes = [vp, sz, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.bjx_engine_create.restype = C.c_int
    L.bjx_engine_create.argtypes = [C.c_int, C.POINTER(EngineOptions), C.POINTER(vp), C.c_char_p, sz]
    L.bjx_engine_destroy.argtypes = [vp]
    L.bjx_engine_set_decision_lists.restype = C.c_int
    L.bjx_engine_set_decision_lists.argtypes = [vp, C.POINTER(DecisionEntry), sz]
    L.bjx_process_batch.restype = C.c_int
    L.bjx_process_batch.argtypes = [vp, vp, vp, sz, C.c_int64, C.c_uint32, C.POINTER(BatchResult)]
    L.bjx_match_batch.restype = C.c_int
    L.bjx_match_batch.argtypes = [vp, vp, vp, sz, C.c_int64, C.c_uint32, C.POINTER(BatchResult)]
    L.bjx_events_partition.restype = C.c_int
    L.bjx_events_partition.argtypes = [vp, C.c_uint32, C.POINTER(C.c_uint64)]
    L.bjx_events_pack.restype = C.c_int
    L.bjx_events_pack.argtypes = [vp, vp, vp, vp]
    L.bjx_apply_events.restype = C.c_int
    L.bjx_apply_events.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.POINTER(C.c_uint64), vp]
    L.bjx_finish_batch.restype = C.c_int
    L.bjx_finish_batch.argtypes = [vp, vp, C.c_uint32, C.POINTER(BatchResult)]
    L.bjx_apply_events_trips.restype = C.c_int
    L.bjx_apply_events_trips.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), vp,
                                         C.POINTER(C.c_uint64)]
    L.bjx_finish_batch_trips.restype = C.c_int
    L.bjx_finish_batch_trips.argtypes = [vp, vp, C.c_uint64, C.c_uint32, C.POINTER(BatchResult)]
    L.bjx_state_get.restype = C.c_int
    L.bjx_state_get.argtypes = [vp, C.c_char_p, sz, C.c_char_p, sz, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.bjx_state_len.restype = C.c_int64
    L.bjx_state_len.argtypes = [vp]
    L.bjx_state_stats_get.restype = C.c_int
    L.bjx_state_stats_get.argtypes = [vp, C.c_void_p]
    L.bjx_state_clear.restype = C.c_int
    L.bjx_state_clear.argtypes = [vp]
    L.bjx_state_dump.restype = sz
    L.bjx_state_dump.argtypes = [vp, C.c_char_p, sz]
    L.bjx_debug_rule_match_host.restype = C.c_int
    L.bjx_debug_rule_match_host.argtypes = [vp, sz, C.c_char_p, sz]
    L.bjx_debug_regex_parse.restype = C.c_int
    L.bjx_debug_regex_parse.argtypes = [C.c_char_p, sz, C.c_char_p, sz]
    L.bjx_debug_rule_lead.restype = C.c_int
    L.bjx_debug_rule_lead.argtypes = [vp, sz]
    L.bjx_debug_rule_literal.restype = sz
    L.bjx_debug_rule_literal.argtypes = [vp, sz, C.c_char_p, sz]
    L.bjx_debug_phase_ms.restype = sz
    L.bjx_debug_phase_ms.argtypes = [vp, C.POINTER(C.c_double), sz]
    L.bjx_debug_kernel_ms.restype = sz
    L.bjx_debug_kernel_ms.argtypes = [vp, C.POINTER(C.c_double), sz]
    L.bjx_debug_scan_stats.restype = sz
    L.bjx_debug_scan_stats.argtypes = [vp, C.POINTER(C.c_uint64), sz]
    L.bjx_debug_set_claim_budget.restype = C.c_int
    L.bjx_debug_set_claim_budget.argtypes = [vp, C.c_uint64]
    L.bjx_debug_set_slot_cache.restype = C.c_int
    L.bjx_debug_set_slot_cache.argtypes = [vp, C.c_int]
    L.bjx_debug_set_ip_hash_mask.restype = C.c_int
    L.bjx_debug_set_ip_hash_mask.argtypes = [vp, C.c_uint64]
    L.bjx_debug_set_dfa_state_cap.restype = C.c_int
    L.bjx_debug_set_dfa_state_cap.argtypes = [C.c_uint32]
    L.bjx_debug_force_wide_nfa.restype = C.c_int
    L.bjx_debug_force_wide_nfa.argtypes = [C.c_int]
    L.bjx_tailer_open.restype = C.c_int
    L.bjx_tailer_open.argtypes = [C.c_char_p, sz, C.POINTER(TailerOptions), C.POINTER(vp), C.c_char_p, sz]
    L.bjx_tailer_next.restype = C.c_int
    L.bjx_tailer_next.argtypes = [vp, C.c_int32, C.POINTER(TailBatch)]
    L.bjx_tailer_release.restype = C.c_int
    L.bjx_tailer_release.argtypes = [vp, C.c_uint32]
    L.bjx_tailer_stats.restype = C.c_int
    L.bjx_tailer_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.bjx_tailer_close.argtypes = [vp]
    L.bjx_engine_set_ban_options.restype = C.c_int
    L.bjx_engine_set_ban_options.argtypes = [vp, C.POINTER(BanOptions)]
    L.bjx_batch_bans.restype = C.c_int
    L.bjx_batch_bans.argtypes = [vp, C.POINTER(BanBatch)]
    L.bjx_engine_last_error.restype = C.c_char_p
    L.bjx_engine_last_error.argtypes = [vp]
    L.bjx_node_create.restype = C.c_int
    L.bjx_node_create.argtypes = [C.POINTER(C.c_int), sz, C.POINTER(EngineOptions), C.POINTER(vp), C.c_char_p, sz]
    L.bjx_node_destroy.argtypes = [vp]
    L.bjx_node_size.restype = sz
    L.bjx_node_size.argtypes = [vp]
    L.bjx_node_engine.restype = vp
    L.bjx_node_engine.argtypes = [vp, sz]
    L.bjx_node_last_error.restype = C.c_char_p
    L.bjx_node_exchange_kind.restype = C.c_int
    L.bjx_node_exchange_kind.argtypes = [vp]
    L.bjx_node_last_error.argtypes = [vp]
    L.bjx_node_set_decision_lists.restype = C.c_int
    L.bjx_node_set_decision_lists.argtypes = [vp, C.POINTER(DecisionEntry), sz]
    L.bjx_node_set_ban_options.restype = C.c_int
    L.bjx_node_set_ban_options.argtypes = [vp, C.POINTER(BanOptions)]
    L.bjx_node_process_batch.restype = C.c_int
    L.bjx_node_process_batch.argtypes = [vp, vp, vp, sz, C.c_int64, C.c_uint32, C.POINTER(BatchResult)]
    L.bjx_node_process_chunks.restype = C.c_int
    L.bjx_node_process_chunks.argtypes = [vp, vp, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int64, C.c_uint32,
                                          C.POINTER(BatchResult)]
    L.bjx_node_batch_bans.restype = C.c_int
    L.bjx_node_batch_bans.argtypes = [vp, C.POINTER(BanBatch)]
    L.bjx_node_state_get.restype = C.c_int
    L.bjx_node_state_get.argtypes = [vp, C.c_char_p, sz, C.c_char_p, sz, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    L.bjx_node_state_len.restype = C.c_int64
    L.bjx_node_state_len.argtypes = [vp]
    L.bjx_node_state_dump.restype = sz
    L.bjx_node_state_dump.argtypes = [vp, C.c_char_p, sz]
    L.bjx_node_state_stats_get.restype = C.c_int
    L.bjx_node_state_stats_get.argtypes = [vp, C.c_void_p]
    L.bjx_node_state_clear.restype = C.c_int
    L.bjx_node_state_clear.argtypes = [vp]
    _lib = L
    return L


def b(x) -> bytes:
    return x if isinstance(x, bytes) else str(x).encode()


def mkstr(x) -> Str:
    bx = b(x)
    return Str(bx, len(bx))
