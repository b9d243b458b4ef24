"""Log-tail front end over bjx_tailer_* (include/banjax_gpu.h).

RunLogTailer (internal/regex_rate_limiter.go:21-78) follows server_log_file
from its end with github.com/hpcloud/tail v1.0.0 and calls consumeLine per
tail.Line.  Here a native reader thread (banjax_amd/csrc/tailer.cpp) bulk-reads
the file into pinned slots, cuts each at its last '\\n' (tail.Line.Text = the
bytes before '\\n', '\\r' kept; a partial last line waits for its '\\n'), and
copies the batch to HBM on its own stream while the engine works on the
previous one.  run_log_tailer() is the loop body: one bjx_process_batch per
batch on the HBM copy, then the Banner replay of the trips in reference order.
"""
from __future__ import annotations

import ctypes as C
import threading
import time
from typing import Callable, Optional

from . import _lib


class TailStopped(RuntimeError):
    """The followed file was deleted or moved away (hpcloud/tail with ReOpen false stops)."""


class TailBatch:
    """A batch of complete lines: pinned host bytes + (device >= 0) their HBM copy."""

    def __init__(self, raw: _lib.TailBatch):
        self.slot = raw.slot
        self.reopened = bool(raw.reopened)
        self.host_ptr = raw.host_bytes
        self.device_ptr = raw.device_bytes
        self.n_bytes = raw.n_bytes
        self.file_offset = raw.file_offset

    def view(self) -> memoryview:
        """The pinned host bytes (valid until release)."""
        return memoryview((C.c_uint8 * self.n_bytes).from_address(self.host_ptr)).cast("B")

    def bytes(self) -> bytes:
        return C.string_at(self.host_ptr, self.n_bytes)


class LogTailer:
    """tail.TailFile(path, Follow, Location {0, io.SeekEnd}) with batched lines."""

    def __init__(self, path: str, device: int = -1, from_start: bool = False, slots: int = 2, poll_ms: int = 20,
                 batch_bytes: int = 0):
        L = _lib.lib()
        opts = _lib.TailerOptions(device, 1 if from_start else 0, slots, poll_ms, batch_bytes)
        h = C.c_void_p()
        err = C.create_string_buffer(512)
        p = _lib.b(path)
        rc = L.bjx_tailer_open(p, len(p), C.byref(opts), C.byref(h), err, 512)
        if rc != _lib.OK:
            raise _lib.BanjaxGpuError(rc, "bjx_tailer_open: " + err.value.decode(errors="replace"))
        self._h = h
        self.device = device

    def next(self, timeout_ms: int = -1) -> Optional[TailBatch]:
        """Next batch (oldest first); None on timeout.  Raises TailStopped."""
        raw = _lib.TailBatch()
        rc = _lib.lib().bjx_tailer_next(self._h, timeout_ms, C.byref(raw))
        if rc == 1:
            return TailBatch(raw)
        if rc == 0:
            return None
        if rc == _lib.TAIL_STOPPED:
            raise TailStopped("tail stopped: file deleted or moved")
        raise _lib.BanjaxGpuError(rc, "bjx_tailer_next")

    def release(self, batch: TailBatch):
        _lib.lib().bjx_tailer_release(self._h, batch.slot)

    def stats(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _lib.lib().bjx_tailer_stats(self._h, C.byref(a), C.byref(b), C.byref(c))
        return {"read_bytes": a.value, "batched_bytes": b.value, "batches": c.value}

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().bjx_tailer_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_log_tailer(limiter, path: str, stop: threading.Event, now_fn: Callable[[], int] = time.time_ns,
                   on_batch: Optional[Callable] = None, from_start: bool = False, batch_bytes: int = 0,
                   poll_ms: int = 20):
    """RunLogTailer (regex_rate_limiter.go:21-78): follow `path` until `stop` is
    set or the file goes away; each batch runs consumeLine for all its lines on
    the GPU under the limiter's current config snapshot (a reload takes effect
    at the next batch).  on_batch(batch, results, out) sees each batch's
    ConsumeLineResults (config.Debug's JSON dump, :68-75) before release."""
    with LogTailer(path, device=limiter.engine.device, from_start=from_start, batch_bytes=batch_bytes,
                   poll_ms=poll_ms) as t:
        while not stop.is_set():
            try:
                b = t.next(timeout_ms=50)
            except TailStopped:
                return
            if b is None:
                continue
            try:
                results, out = limiter.consume_device_batch(b.view(), b.device_ptr, b.n_bytes, now_fn(),
                                                            want_results=on_batch is not None)
                if on_batch is not None:
                    on_batch(b, results, out)
            finally:
                t.release(b)
