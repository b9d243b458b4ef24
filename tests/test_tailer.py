"""Log-tail front end: bjx_tailer_* against hpcloud/tail
v1.0.0's behaviour as RunLogTailer uses it (regex_rate_limiter.go:30-58).

CPU tests run the native tailer in host-framing mode (device -1): start at
EOF, partial lines held until their '\\n', '\\r' kept, truncation re-read from
0, deletion / rename stop, a file that does not exist yet, lines longer than a
slot.  The GPU test follows a file written in random chunks through
run_log_tailer into the engine and compares every batch with the oracle.
"""
import os
import random
import threading
import time

import pytest

from banjax_amd import LogTailer, TailStopped

POLL = 5


def drain(t, until_bytes, timeout_s=10.0):
    """Concatenate batches until `until_bytes` bytes arrived."""
    got = bytearray()
    end = time.time() + timeout_s
    flags = []
    while len(got) < until_bytes and time.time() < end:
        b = t.next(timeout_ms=50)
        if b is None:
            continue
        data = b.bytes()
        assert data.endswith(b"\n")
        flags.append(b.reopened)
        got += data
        t.release(b)
    return bytes(got), flags


def append(path, data):
    with open(path, "ab") as f:
        f.write(data)
        f.flush()


def test_starts_at_eof_and_holds_partial_lines(tmp_path):
    p = str(tmp_path / "access.log")
    append(p, b"old line 1\nold line 2\npartial-before-open")
    with LogTailer(p, device=-1, poll_ms=POLL) as t:
        time.sleep(0.05)
        append(p, b" tail\nline A\r\nline B")  # "partial-before-open" started before EOF: skipped part
        got, _ = drain(t, len(b" tail\nline A\r\n"))
        # Location {0, SeekEnd}: reading starts at the old EOF, mid-line
        assert got == b" tail\nline A\r\n"
        assert t.next(timeout_ms=60) is None  # "line B" waits for its '\n'
        append(p, b" done\n")
        got, _ = drain(t, len(b"line B done\n"))
        assert got == b"line B done\n"
        st = t.stats()
        assert st["read_bytes"] == st["batched_bytes"] == len(b" tail\nline A\r\nline B done\n")


def test_from_start_and_random_chunking(tmp_path):
    p = str(tmp_path / "access.log")
    rng = random.Random(7)
    lines = [("%d 1.2.%d.%d GET h%d GET /%s HTTP/1.1 ua | 200" % (i, i % 256, i % 7, i % 3, "x" * rng.randint(0, 300)))
             .encode() + b"\n" for i in range(3000)]
    blob = b"".join(lines)
    append(p, blob[:1000])
    with LogTailer(p, device=-1, from_start=True, poll_ms=POLL, batch_bytes=8192) as t:
        pos = 1000
        while pos < len(blob):
            k = rng.randint(1, 5000)
            append(p, blob[pos:pos + k])
            pos += k
        got, _ = drain(t, len(blob))
    assert got == blob


def test_long_line_grows_slot(tmp_path):
    p = str(tmp_path / "access.log")
    open(p, "wb").close()
    big = b"1 1.1.1.1 GET h GET /" + b"a" * 50000 + b" HTTP/1.1 | 200\n"
    with LogTailer(p, device=-1, poll_ms=POLL, batch_bytes=4096) as t:
        time.sleep(0.05)
        append(p, b"short\n" + big + b"after\n")
        got, _ = drain(t, len(big) + 12)
    assert got == b"short\n" + big + b"after\n"


def test_truncation_rereads_from_start(tmp_path):
    p = str(tmp_path / "access.log")
    append(p, b"x" * 100 + b"\n")
    with LogTailer(p, device=-1, poll_ms=POLL) as t:
        time.sleep(0.05)
        append(p, b"first\nheld partial")
        got, _ = drain(t, 6)
        assert got == b"first\n"
        with open(p, "wb") as f:  # copytruncate-style rotation
            f.write(b"new1\n")
        got, flags = drain(t, 5)
        assert got == b"new1\n" and flags[0]
        append(p, b"new2\n")
        got, flags = drain(t, 5)
        assert got == b"new2\n" and not flags[0]


@pytest.mark.parametrize("how", ["unlink", "rename"])
def test_deleted_or_moved_file_stops(tmp_path, how):
    p = str(tmp_path / "access.log")
    append(p, b"")
    with LogTailer(p, device=-1, poll_ms=POLL) as t:
        time.sleep(0.05)
        append(p, b"a\n")
        got, _ = drain(t, 2)
        assert got == b"a\n"
        if how == "unlink":
            os.unlink(p)
        else:
            os.rename(p, p + ".1")
        with pytest.raises(TailStopped):
            for _ in range(100):
                t.next(timeout_ms=20)


def test_waits_for_missing_file(tmp_path):
    p = str(tmp_path / "later.log")
    with LogTailer(p, device=-1, poll_ms=POLL) as t:
        assert t.next(timeout_ms=30) is None
        append(p, b"")
        time.sleep(0.1)  # first open: follows from the end of what is there
        append(p, b"l1\nl2\n")
        got, _ = drain(t, 6)
    assert got == b"l1\nl2\n"


@pytest.mark.gpu
def test_gpu_tail_to_engine_parity(tmp_path):
    """Lines written in random chunks -> tailer (pinned slots, HBM copies) ->
    run_log_tailer -> engine, every batch compared with the oracle."""
    import workloads as W
    from banjax_amd import Engine
    from tests.parity import Pair, compare_batch
    from banjax_amd.tailer import run_log_tailer

    w = W.scaled(W.CFG1, 60_000, n_ips=3_000)
    blob = w.host_lines()
    now = w.now_ns()
    eng = Engine(0)
    pair = Pair(w.rules_yaml, eng)
    p = str(tmp_path / "access.log")
    open(p, "wb").close()
    stop = threading.Event()
    seen = []

    def on_batch(b, results, out):
        data = b.bytes()
        oflags, ores, oconsumed = pair.ost.consume(pair.ocfg, data, now,
                                                   cap=(data.count(b"\n") + 1) * (pair.n_rules + 1))
        compare_batch(oflags, ores, oconsumed, out)
        seen.append(len(data))
        if sum(seen) == len(blob):
            stop.set()

    th = threading.Thread(target=run_log_tailer, args=(pair.lim, p, stop),
                          kwargs=dict(now_fn=lambda: now, on_batch=on_batch, batch_bytes=1 << 20, poll_ms=2))
    th.start()
    time.sleep(0.2)
    rng = random.Random(3)
    pos = 0
    while pos < len(blob):
        k = rng.randint(1, 400_000)
        append(p, blob[pos:pos + k])
        pos += k
        time.sleep(0.002)
    th.join(timeout=60)
    stop.set()
    assert sum(seen) == len(blob) and len(seen) > 1
    pair.compare_state()
    eng.close()


def test_large_backlog_parallel_reads(tmp_path):
    """A backlog of 96 MB read from offset 0 in 40 MB slots: each fill is
    split over several pread threads; the batches still concatenate to the
    file's complete lines, in order, and the partial tail waits."""
    p = str(tmp_path / "big.log")
    rnd = random.Random(5)
    lines = [b"%d %s x\n" % (i, b"y" * rnd.randrange(0, 300)) for i in range(400_000)]
    body = b"".join(lines)
    while len(body) < 96 << 20:
        body += body[:len(body) // 2]
        body = body[:body.rindex(b"\n") + 1]
    append(p, body + b"no newline yet")
    with LogTailer(p, device=-1, from_start=True, batch_bytes=40 << 20, poll_ms=POLL) as t:
        got, _ = drain(t, len(body), timeout_s=60)
        assert got == body
        assert t.next(timeout_ms=60) is None
