"""ORACLE — test / baseline infrastructure only (bench.py's cpu_baseline leg).

One worker of the N-core, IP-sharded CPU baseline: the reference path is one
goroutine (regex_rate_limiter.go:54-77), and RegexRateLimitStates is keyed by
IP (rate_limit.go:45-67), so lines sharded by IP hash keep every IP's
per-rule order and results; N workers model an N-core deployment of the same
algorithm.  usage: python -m oracle.shard_worker <sample file> <k> <n> <now_ns> <rules yaml file>
Prints {"lines": n, "seconds": t} for its shard (filtering excluded from t).
"""
import json
import sys
import time
import zlib


def main():
    path, k, n, now_ns, ypath = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    from oracle import oracle as O
    from tests.parity import oracle_config
    from banjax_amd.config import Config
    data = open(path, "rb").read()
    mine = []
    for ln in data.split(b"\n")[:-1]:
        parts = ln.split(b" ", 2)
        ip = parts[1] if len(parts) > 1 else b""
        if zlib.crc32(ip) % n == k:
            mine.append(ln)
    buf = b"\n".join(mine) + b"\n" if mine else b""
    oc = oracle_config(Config.from_yaml(open(ypath).read()))
    st = O.State()
    t0 = time.perf_counter()
    st.consume(oc, buf, now_ns, cap=max(16, len(mine) * 8))
    dt = time.perf_counter() - t0
    print(json.dumps({"lines": len(mine), "seconds": dt}))


if __name__ == "__main__":
    main()
