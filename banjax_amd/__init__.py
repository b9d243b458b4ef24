"""banjax_amd — MI355X engine for deflect-ca/banjax's regex rate-limiting log tailer.

The hot path (consumeLine: header parse, CheckIsAllowed, every rule's regex,
RegexRateLimitStates.Apply) runs as HIP kernels for gfx950 behind the C ABI of
include/banjax_gpu.h; this package is the host surface mirroring the
reference's Go types (config schema, consumeLine, RegexRateLimitStates,
Banner / DynamicDecisionLists).
"""
from .config import (ALLOW, CHALLENGE, IPTABLES_BLOCK, NGINX_BLOCK, Config, ConfigError, RegexWithRate, Ruleset,
                     decision_string, parse_decision)
from .engine import BatchOutput, Engine, Node
from .regex_rate_limiter import (Banner, ConsumeLineResult, DynamicDecisionLists, MockBanner, RateLimitResult,
                                 RegexRateLimiter, RegexRateLimitStates, RuleResult, Zone, consume_line)
from .tailer import LogTailer, TailBatch, TailStopped, run_log_tailer

__all__ = [
    "ALLOW", "CHALLENGE", "NGINX_BLOCK", "IPTABLES_BLOCK", "Config", "ConfigError", "RegexWithRate", "Ruleset",
    "decision_string", "parse_decision", "Engine", "Node", "BatchOutput", "Banner", "MockBanner", "DynamicDecisionLists",
    "ConsumeLineResult", "RuleResult", "RateLimitResult", "RegexRateLimiter", "RegexRateLimitStates", "consume_line", "Zone",
    "LogTailer", "TailBatch", "TailStopped", "run_log_tailer",
]
