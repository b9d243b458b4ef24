// Log-tail front end: follows the nginx access log the way
// RunLogTailer does (internal/regex_rate_limiter.go:21-78 with
// github.com/hpcloud/tail v1.0.0, go.mod:10) and hands the engine batches of
// complete lines that are already on their way to HBM.
//
// hpcloud/tail v1.0.0 behaviour restated (the library is not vendored in the
// reference; its published tail.go is the source):
//   - tailFileSync: with MustExist false the first open waits for the file to
//     exist; Location {0, io.SeekEnd} is applied once, after that first open;
//   - readLine: bufio ReadString('\n'), then TrimRight "\n": Line.Text keeps
//     '\r' and every other byte;
//   - at EOF with a partial line in Follow mode the reader seeks back to the
//     line start and waits; the line is delivered once its '\n' is written;
//   - waitForChanges: Truncated -> reopen and read from offset 0;
//     Deleted (inotify IN_DELETE_SELF / IN_MOVE_SELF) with ReOpen false ->
//     the tail stops and no further lines arrive.
// The equivalents here are a carried partial line, a size check at EOF, and
// an inode / link-count check of the path at EOF.
//
// MI355X side: one reader thread per tailer bulk-reads (pread) into pinned
// slots and issues each slot's host-to-device copy on its own HIP stream, so
// the copy of batch k+1 runs under bjx_process_batch of batch k.  A fill of
// data the file already holds is split over up to 8 pread threads (16 measured no faster: the page-cache reads top out near 23 GB/s on the box).
#include <hip/hip_runtime_api.h>

#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/banjax_gpu.h"

namespace {

struct Slot {
  uint8_t *host = nullptr;  // pinned (device >= 0) or malloc'd
  uint8_t *dev = nullptr;
  uint64_t cap = 0;
  hipEvent_t copied = nullptr;
  uint64_t n = 0, file_offset = 0;
  bool reopened = false;
};

}  // namespace

struct bjx_tailer {
  std::string path;
  bjx_tailer_options o{};
  std::vector<Slot> slots;
  hipStream_t copy_stream = nullptr;

  std::mutex mu;
  std::condition_variable cv_free, cv_ready;
  std::deque<uint32_t> free_q, ready_q;
  bool stop = false;      // close requested
  bool stopped = false;   // reader finished (file gone or error)
  int error = 0;
  std::string error_msg;
  uint64_t read_bytes = 0, batched_bytes = 0, batches = 0;
  uint32_t read_threads = 1;  // pread threads per slot fill
  std::thread reader;
};

namespace {

constexpr uint64_t kParallelReadMin = 16ull << 20;  // bytes per extra read thread

void set_err(char *err, size_t len, const std::string &m) {
  if (err && len) snprintf(err, len, "%s", m.c_str());
}

bool alloc_slot(bjx_tailer *t, Slot &s, uint64_t cap) {
  if (t->o.device >= 0) {
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
    s.host = nullptr;
    s.dev = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&s.host), cap, hipHostMallocDefault) != hipSuccess) return false;
    if (hipMalloc(reinterpret_cast<void **>(&s.dev), cap) != hipSuccess) return false;
  } else {
    free(s.host);
    s.host = static_cast<uint8_t *>(aligned_alloc(64, (cap + 63) & ~63ull));
    if (!s.host) return false;
  }
  s.cap = cap;
  return true;
}

void free_slot(bjx_tailer *t, Slot &s) {
  if (t->o.device >= 0) {
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
    if (s.copied) (void)hipEventDestroy(s.copied);
  } else {
    free(s.host);
  }
  s = Slot{};
}

// The reader's view of the followed file.
struct Follow {
  int fd = -1;
  dev_t dev = 0;
  ino_t ino = 0;
  uint64_t pos = 0;
  bool opened_once = false;
};

enum class Change { None, Truncated, Gone };

Change check_file(const std::string &path, const Follow &f) {
  struct stat a, b;
  if (fstat(f.fd, &a) != 0) return Change::Gone;
  if (a.st_nlink == 0) return Change::Gone;  // unlinked (IN_DELETE_SELF)
  if (stat(path.c_str(), &b) != 0 || b.st_dev != f.dev || b.st_ino != f.ino) return Change::Gone;  // moved away
  if ((uint64_t)a.st_size < f.pos) return Change::Truncated;
  return Change::None;
}

void finish(bjx_tailer *t, int code, const std::string &msg) {
  std::lock_guard<std::mutex> g(t->mu);
  t->stopped = true;
  t->error = code;
  t->error_msg = msg;
  t->cv_ready.notify_all();
}

void reader_main(bjx_tailer *t) {
  if (t->o.device >= 0 && hipSetDevice(t->o.device) != hipSuccess) {
    finish(t, BJX_ERR_DEVICE, "hipSetDevice failed in tailer");
    return;
  }
  Follow f;
  std::vector<uint8_t> carry;   // partial line at the end of the last read
  uint64_t carry_off = 0;       // its file offset
  bool reopened = false;
  const auto poll = std::chrono::milliseconds(t->o.poll_ms);
  auto wait_poll = [&]() {
    std::unique_lock<std::mutex> g(t->mu);
    t->cv_free.wait_for(g, poll, [&] { return t->stop; });
    return !t->stop;
  };

  for (;;) {
    {
      std::lock_guard<std::mutex> g(t->mu);
      if (t->stop) break;
    }
    if (f.fd < 0) {
      const int fd = open(t->path.c_str(), O_RDONLY | O_CLOEXEC);
      if (fd < 0) {
        if (errno != ENOENT) {
          finish(t, BJX_ERR_IO, std::string("open ") + t->path + ": " + strerror(errno));
          return;
        }
        if (!wait_poll()) break;  // not there yet (MustExist false)
        continue;
      }
      struct stat st;
      fstat(fd, &st);
      f.fd = fd;
      f.dev = st.st_dev;
      f.ino = st.st_ino;
      // Location {0, SeekEnd} applies to the first open only
      f.pos = (!f.opened_once && !t->o.from_start) ? (uint64_t)st.st_size : 0;
      f.opened_once = true;
    }
    // a free slot
    uint32_t si;
    {
      std::unique_lock<std::mutex> g(t->mu);
      t->cv_free.wait(g, [&] { return t->stop || !t->free_q.empty(); });
      if (t->stop) break;
      si = t->free_q.front();
      t->free_q.pop_front();
    }
    Slot &s = t->slots[si];
    if (carry.size() >= s.cap / 2 && !alloc_slot(t, s, std::max<uint64_t>(s.cap * 2, carry.size() * 2))) {
      finish(t, BJX_ERR_NOMEM, "tailer slot growth failed");
      return;
    }
    memcpy(s.host, carry.data(), carry.size());
    uint64_t n = carry.size();
    const uint64_t start_off = carry.size() ? carry_off : f.pos;
    bool eof = false;
    uint64_t copied = 0;  // slot bytes whose host-to-device copy is issued
    {
      // what the file already holds past pos is read by several threads at
      // once (each a disjoint range into its own part of the slot): one
      // thread copying from the page cache into pinned memory tops out near
      // 15 GB/s, well under PCIe.  Each thread issues its range's copy to HBM
      // as soon as it has read it, so the slot's copy runs under its read.
      struct stat st;
      const uint64_t room = s.cap - n;
      const uint64_t avail = fstat(f.fd, &st) == 0 && (uint64_t)st.st_size > f.pos ? (uint64_t)st.st_size - f.pos : 0;
      const uint64_t want = std::min(room, avail);
      const uint32_t T = (uint32_t)std::min<uint64_t>(t->read_threads, want / kParallelReadMin);
      if (T > 1) {
        const uint64_t per = (want / T + 4095) & ~4095ull;
        const bool dev = t->o.device >= 0;
        if (dev && n && hipMemcpyAsync(s.dev, s.host, n, hipMemcpyHostToDevice, t->copy_stream) != hipSuccess) {
          finish(t, BJX_ERR_DEVICE, "tailer host-to-device copy failed");
          return;
        }
        std::vector<std::thread> th;
        std::vector<uint64_t> got(T, 0);
        std::vector<int> errs(T, 0), cerr(T, 0);
        for (uint32_t k = 0; k < T; ++k) {
          const uint64_t a = std::min<uint64_t>(want, per * k), b = std::min<uint64_t>(want, per * (k + 1));
          th.emplace_back([&, k, a, b]() {
            uint64_t o = a;
            while (o < b) {
              const ssize_t r = pread(f.fd, s.host + n + o, b - o, (off_t)(f.pos + o));
              if (r < 0 && errno == EINTR) continue;
              if (r < 0) { errs[k] = errno; break; }
              if (r == 0) break;
              o += (uint64_t)r;
            }
            got[k] = o - a;
            if (dev && o > a &&
                (hipSetDevice(t->o.device) != hipSuccess ||
                 hipMemcpyAsync(s.dev + n + a, s.host + n + a, o - a, hipMemcpyHostToDevice, t->copy_stream) != hipSuccess))
              cerr[k] = 1;
          });
        }
        for (auto &x : th) x.join();
        for (uint32_t k = 0; k < T; ++k)
          if (cerr[k]) {
            finish(t, BJX_ERR_DEVICE, "tailer host-to-device copy failed");
            return;
          }
        // keep the contiguous prefix that every range delivered in full
        uint64_t ok = 0;
        for (uint32_t k = 0; k < T; ++k) {
          const uint64_t a = std::min<uint64_t>(want, per * k), b = std::min<uint64_t>(want, per * (k + 1));
          if (errs[k]) {
            finish(t, BJX_ERR_IO, std::string("read ") + t->path + ": " + strerror(errs[k]));
            return;
          }
          ok += got[k];
          if (got[k] != b - a) break;  // the file shrank under the read: stop at the gap
        }
        n += ok;
        f.pos += ok;
        copied = dev ? n : 0;  // ranges past a gap were copied too; the next slot reads them again
        std::lock_guard<std::mutex> g(t->mu);
        t->read_bytes += ok;
      }
    }
    while (n < s.cap) {
      const ssize_t r = pread(f.fd, s.host + n, s.cap - n, (off_t)f.pos);
      if (r < 0) {
        if (errno == EINTR) continue;
        finish(t, BJX_ERR_IO, std::string("read ") + t->path + ": " + strerror(errno));
        return;
      }
      if (r == 0) { eof = true; break; }
      n += (uint64_t)r;
      f.pos += (uint64_t)r;
      std::lock_guard<std::mutex> g(t->mu);
      t->read_bytes += (uint64_t)r;
    }
    const uint8_t *last = n ? static_cast<const uint8_t *>(memrchr(s.host, '\n', n)) : nullptr;
    if (!last) {
      // no complete line: keep the bytes, give the slot back
      carry.assign(s.host, s.host + n);
      carry_off = start_off;
      // the parallel reads may have queued copies out of this slot's pinned
      // bytes: they finish before the slot is refilled or freed
      if (copied && hipStreamSynchronize(t->copy_stream) != hipSuccess) {
        finish(t, BJX_ERR_DEVICE, "tailer host-to-device copy failed");
        return;
      }
      {
        std::lock_guard<std::mutex> g(t->mu);
        t->free_q.push_front(si);
      }
      if (!eof) continue;  // a line longer than the slot: the slot grows next round
    } else {
      const uint64_t nb = (uint64_t)(last - s.host) + 1;
      carry.assign(s.host + nb, s.host + n);
      carry_off = start_off + nb;
      s.n = nb;
      s.file_offset = start_off;
      s.reopened = reopened;
      reopened = false;
      if (t->o.device >= 0) {
        if ((nb > copied &&
             hipMemcpyAsync(s.dev + copied, s.host + copied, nb - copied, hipMemcpyHostToDevice, t->copy_stream) != hipSuccess) ||
            hipEventRecord(s.copied, t->copy_stream) != hipSuccess) {
          finish(t, BJX_ERR_DEVICE, "tailer host-to-device copy failed");
          return;
        }
      }
      {
        std::lock_guard<std::mutex> g(t->mu);
        t->ready_q.push_back(si);
        t->batched_bytes += nb;
        ++t->batches;
        t->cv_ready.notify_all();
      }
      if (!eof) continue;  // more is already there
    }
    // at EOF: the file's fate, then wait for more
    const Change c = check_file(t->path, f);
    if (c == Change::Gone) {
      close(f.fd);
      f.fd = -1;
      finish(t, BJX_TAIL_STOPPED, "file deleted or moved; tail stopped (ReOpen false)");
      return;
    }
    if (c == Change::Truncated) {
      f.pos = 0;  // reopen: read again from the start; the held partial line is gone
      carry.clear();
      reopened = true;
      continue;
    }
    if (!wait_poll()) break;
  }
  if (f.fd >= 0) close(f.fd);
  finish(t, 0, "");
}

}  // namespace

extern "C" int bjx_tailer_open(const char *path, size_t path_len, const bjx_tailer_options *opts, bjx_tailer **out,
                               char *err, size_t err_len) {
  if (!path || !out) return BJX_ERR_ARG;
  *out = nullptr;
  bjx_tailer *t = new (std::nothrow) bjx_tailer;
  if (!t) return BJX_ERR_NOMEM;
  t->path.assign(path, path_len);
  if (opts) t->o = *opts;
  else t->o.device = -1;
  if (!t->o.slots) t->o.slots = 2;
  if (!t->o.poll_ms) t->o.poll_ms = 20;
  if (!t->o.batch_bytes) t->o.batch_bytes = 256ull << 20;
  t->o.batch_bytes = std::max<uint64_t>(t->o.batch_bytes, 4096);
  if (t->o.device >= 0) {
    if (hipSetDevice(t->o.device) != hipSuccess || hipStreamCreateWithFlags(&t->copy_stream, hipStreamNonBlocking) != hipSuccess) {
      set_err(err, err_len, "no HIP device for the tailer");
      delete t;
      return BJX_ERR_DEVICE;
    }
  }
  t->slots.resize(t->o.slots);
  for (uint32_t i = 0; i < t->o.slots; ++i) {
    Slot &s = t->slots[i];
    if (!alloc_slot(t, s, t->o.batch_bytes) ||
        (t->o.device >= 0 && hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) != hipSuccess)) {
      set_err(err, err_len, "tailer buffer allocation failed");
      for (auto &x : t->slots) free_slot(t, x);
      if (t->copy_stream) (void)hipStreamDestroy(t->copy_stream);
      delete t;
      return BJX_ERR_NOMEM;
    }
    t->free_q.push_back(i);
  }
  {
    const unsigned hc = std::thread::hardware_concurrency();
    t->read_threads = std::max(1u, std::min(8u, hc ? hc : 1u));
  }
  t->reader = std::thread(reader_main, t);
  *out = t;
  return BJX_OK;
}

extern "C" int bjx_tailer_next(bjx_tailer *t, int32_t timeout_ms, bjx_tail_batch *out) {
  if (!t || !out) return BJX_ERR_ARG;
  uint32_t si;
  {
    std::unique_lock<std::mutex> g(t->mu);
    auto ready = [&] { return !t->ready_q.empty() || t->stopped; };
    if (timeout_ms < 0) t->cv_ready.wait(g, ready);
    else if (!t->cv_ready.wait_for(g, std::chrono::milliseconds(timeout_ms), ready)) return 0;
    if (t->ready_q.empty()) return t->error ? t->error : 0;
    si = t->ready_q.front();
    t->ready_q.pop_front();
  }
  Slot &s = t->slots[si];
  if (t->o.device >= 0 && hipEventSynchronize(s.copied) != hipSuccess) return BJX_ERR_DEVICE;
  out->slot = si;
  out->reopened = s.reopened;
  out->host_bytes = s.host;
  out->device_bytes = t->o.device >= 0 ? s.dev : nullptr;
  out->n_bytes = s.n;
  out->file_offset = s.file_offset;
  return 1;
}

extern "C" int bjx_tailer_release(bjx_tailer *t, uint32_t slot) {
  if (!t || slot >= t->slots.size()) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(t->mu);
  t->free_q.push_back(slot);
  t->cv_free.notify_all();
  return BJX_OK;
}

extern "C" int bjx_tailer_stats(bjx_tailer *t, uint64_t *read_bytes, uint64_t *batched_bytes, uint64_t *batches) {
  if (!t) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(t->mu);
  if (read_bytes) *read_bytes = t->read_bytes;
  if (batched_bytes) *batched_bytes = t->batched_bytes;
  if (batches) *batches = t->batches;
  return BJX_OK;
}

extern "C" void bjx_tailer_close(bjx_tailer *t) {
  if (!t) return;
  {
    std::lock_guard<std::mutex> g(t->mu);
    t->stop = true;
    t->cv_free.notify_all();
  }
  if (t->reader.joinable()) t->reader.join();
  if (t->copy_stream) (void)hipStreamSynchronize(t->copy_stream);
  for (auto &s : t->slots) free_slot(t, s);
  if (t->copy_stream) (void)hipStreamDestroy(t->copy_stream);
  delete t;
}
