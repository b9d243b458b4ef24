// Node: the GPUs of one host behind one handle (SURVEY.md §8 e).
//
// The reference runs one RegexRateLimitStates (internal/rate_limit.go:19-28,
// created once in banjax.go:80) fed by one consumer goroutine
// (internal/regex_rate_limiter.go:54-77).  A node keeps that shape over n
// engines and hides the sharding:
//   1. engine k runs consumeLine up to Apply on the k-th contiguous chunk
//      (bjx_match_batch);
//   2. each engine sorts its event lines by owner, (ip_hash >> 32) % n, and
//      packs them owner-major (bjx_events_partition / bjx_events_pack);
//   3. the node moves every (source, owner) segment into the owner's receive
//      buffers, concatenated in source order: one RCCL group of
//      ncclSend / ncclRecv pairs over xGMI when the engines sit on distinct
//      GPUs (an all-to-all of variable-size segments, one communicator clique
//      made by ncclCommInitAll), else copies on one stream per GPU
//      (hipMemcpyPeerAsync / hipMemcpyAsync: several engines sharing a GPU,
//      the one-GPU rehearsal; BJX_NODE_EXCHANGE=peer selects it always);
//   4. each owner applies its events (bjx_apply_events): chunks are in stream
//      order, so every (ip, rule name) state sees its events in the
//      reference's order;
//   5. the outcome bytes go back the same way, and each engine selects its
//      trips (bjx_finish_batch); a batch that wants trips only (no
//      BJX_COPY_RESULTS) sends back just the packed indices of the tripping
//      events instead (bjx_apply_events_trips / bjx_finish_batch_trips);
//   6. the node concatenates the engines' trips (global line order) and
//      merges their per-IP decision records (highest decision, first trip).
// Phases 1, 2, 4 and 5 run on one host thread per engine, so the GPUs work
// concurrently; 3 and 5's copies are issued from the calling thread.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/banjax_gpu.h"
#include "../../include/banjax_gpu_debug.h"

namespace {

struct NodeError {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, std::string msg) { throw NodeError{code, std::move(msg)}; }

void hip_ok(hipError_t r, const char *what) {
  if (r != hipSuccess) fail(BJX_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(r));
}

// device buffer on one GPU, grown geometrically
struct DevMem {
  int dev = 0;
  uint8_t *p = nullptr;
  size_t cap = 0;
  uint8_t *ensure(size_t n) {
    if (n <= cap && p) return p;
    hip_ok(hipSetDevice(dev), "hipSetDevice");
    const size_t c = std::max<size_t>(std::max<size_t>(n, 4096), cap + cap / 2);
    if (p) hip_ok(hipFree(p), "hipFree");
    p = nullptr;
    cap = 0;
    hip_ok(hipMalloc(reinterpret_cast<void **>(&p), c), "hipMalloc (node exchange buffer)");
    cap = c;
    return p;
  }
  void release() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
};

constexpr size_t kLineRec = sizeof(bjx_event_line);

struct Part {
  bjx_engine *e = nullptr;
  int dev = 0;
  hipStream_t copy = nullptr;          // exchange copies INTO this engine's buffers
  std::vector<uint64_t> send;          // 3 * n: lines / events / bytes to each owner
  DevMem s_lines, s_ev, s_bytes, s_out;  // packed outgoing records, outcomes coming back
  DevMem r_lines, r_ev, r_bytes, r_out;  // received records, their outcomes
  DevMem r_trips, s_trips;             // trips-only batches: owner's trip lists out, the source's back
  std::vector<uint64_t> tr_counts;     // owner side: trips per source
  bjx_batch_result res{};
};

}  // namespace

struct bjx_node {
  std::vector<Part> parts;
  std::vector<ncclComm_t> comms;  // RCCL clique over the engines' GPUs (empty: peer copies)
  bool force_exchange = false;    // test hook (BJX_NODE_FORCE_EXCHANGE=1): exchange even for one engine
  std::mutex mu;
  std::string last_error;
  // merged results of the last batch
  std::vector<bjx_trip> trips;
  std::vector<uint64_t> trips_c;  // BJX_TRIPS_COMPACT words
  std::vector<bjx_rule_result> results;
  std::vector<uint8_t> line_flags;
  bool bans = false;
  uint64_t ban_trips = 0;
  std::vector<bjx_ip_decision> ips;
  std::vector<uint8_t> ipb;
  std::vector<uint64_t> ipo;
  std::vector<char> log;
  std::vector<uint64_t> log_off;
  std::vector<uint8_t> log_kind;
};

namespace {

// f(k) on one host thread per engine; the first failure (lowest k) is thrown
template <typename F>
void each(bjx_node *n, F f) {
  const size_t N = n->parts.size();
  std::vector<int> rc(N, BJX_OK);
  std::vector<std::string> msg(N);
  auto run = [&](size_t k) {
    try {
      rc[k] = f(k);
      if (rc[k] != BJX_OK) msg[k] = bjx_engine_last_error(n->parts[k].e);
    } catch (const NodeError &x) {
      rc[k] = x.code;
      msg[k] = x.msg;
    } catch (const std::bad_alloc &) {
      rc[k] = BJX_ERR_NOMEM;
      msg[k] = "host out of memory";
    }
  };
  if (N == 1) {
    run(0);
  } else {
    std::vector<std::thread> th;
    th.reserve(N);
    for (size_t k = 0; k < N; ++k) th.emplace_back(run, k);
    for (auto &t : th) t.join();
  }
  for (size_t k = 0; k < N; ++k)
    if (rc[k] != BJX_OK) fail(rc[k], "engine " + std::to_string(k) + ": " + msg[k]);
}

template <typename F>
int guarded(bjx_node *n, F f) {
  if (!n) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(n->mu);
  try {
    return f();
  } catch (const NodeError &x) {
    n->last_error = x.msg;
    return x.code;
  } catch (const std::bad_alloc &) {
    n->last_error = "host out of memory";
    return BJX_ERR_NOMEM;
  }
}

void peer_copy(void *dst, const Part &D, const void *src, const Part &S, size_t bytes);

void nccl_ok(ncclResult_t r, const char *what) {
  if (r != ncclSuccess) fail(BJX_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}

// One all-to-all of variable-size segments: seg(dst_part, src_part) gives the
// destination pointer, source pointer and bytes.  RCCL: a single group of
// ncclSend / ncclRecv over every pair (self pairs included), each GPU's side
// on its copy stream; otherwise a copy per pair on the destination's copy
// stream.  Zero-byte segments move nothing on either side (both sides know
// every size).
template <typename Seg>
void exchange(bjx_node *n, Seg seg) {
  const size_t N = n->parts.size();
  if (n->comms.empty()) {
    for (size_t p = 0; p < N; ++p)
      for (size_t k = 0; k < N; ++k) {
        void *d;
        const void *s;
        size_t b;
        seg(p, k, &d, &s, &b);
        peer_copy(d, n->parts[p], s, n->parts[k], b);
      }
    return;
  }
  nccl_ok(ncclGroupStart(), "ncclGroupStart");
  // the group is always closed on this thread, even when a call inside it
  // fails: the first error is kept and raised after ncclGroupEnd
  ncclResult_t first = ncclSuccess;
  const char *what = "";
  for (size_t p = 0; p < N && first == ncclSuccess; ++p)
    for (size_t k = 0; k < N && first == ncclSuccess; ++k) {
      void *d;
      const void *s;
      size_t b;
      seg(p, k, &d, &s, &b);
      if (!b) continue;
      ncclResult_t r = ncclSend(s, b, ncclUint8, (int)p, n->comms[k], n->parts[k].copy);
      if (r != ncclSuccess) { first = r; what = "ncclSend"; break; }
      r = ncclRecv(d, b, ncclUint8, (int)k, n->comms[p], n->parts[p].copy);
      if (r != ncclSuccess) { first = r; what = "ncclRecv"; break; }
    }
  const ncclResult_t end = ncclGroupEnd();
  nccl_ok(first, what);
  nccl_ok(end, "ncclGroupEnd");
}

void sync_copies(bjx_node *n) {
  for (auto &P : n->parts) {
    hip_ok(hipSetDevice(P.dev), "hipSetDevice");
    hip_ok(hipStreamSynchronize(P.copy), "exchange copy");
  }
}

void peer_copy(void *dst, const Part &D, const void *src, const Part &S, size_t bytes) {
  if (!bytes) return;
  hip_ok(hipSetDevice(D.dev), "hipSetDevice");
  if (D.dev == S.dev)
    hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, D.copy), "hipMemcpyAsync (exchange)");
  else
    hip_ok(hipMemcpyPeerAsync(dst, D.dev, src, S.dev, bytes, D.copy), "hipMemcpyPeerAsync (exchange)");
}

// fn(i) for i in [0, count) over up to `threads` host threads
template <typename F>
void par_for(size_t count, size_t threads, F fn) {
  threads = std::max<size_t>(1, std::min(threads, count));
  if (threads == 1) {
    for (size_t i = 0; i < count; ++i) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::thread> th;
  th.reserve(threads);
  for (size_t t = 0; t < threads; ++t)
    th.emplace_back([&]() {
      for (size_t i; (i = next.fetch_add(1)) < count;) fn(i);
    });
  for (auto &t : th) t.join();
}

size_t host_threads() {
  const unsigned hc = std::thread::hardware_concurrency();
  return std::max<size_t>(1, std::min<size_t>(16, hc ? hc : 1));
}

uint64_t ip_key(const uint8_t *p, size_t n) {  // FNV-1a, finalised
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ull;
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  return h ^ (h >> 33);
}

// Merge the engines' decision records (bjx_batch_bans, each in its own trip
// order) into node trip order.  Engine k's trips precede engine k+1's, so per
// IP the highest decision's first trip is the earliest (k, trip) reaching it
// (the reference's Update sequence over global trip order,
// regex_rate_limiter.go:254-263 into decision.go:404-433).
// Host work, parallel: records are bucketed by a hash of their IP bytes, each
// bucket merged with its own small table (engine order kept inside a bucket),
// and the merged records put back in trip order by a radix sort.
void merge_bans(bjx_node *n, const std::vector<uint64_t> &trip_base) {
  const size_t N = n->parts.size(), T = host_threads();
  std::vector<bjx_ban_batch> bb(N);
  for (size_t k = 0; k < N; ++k) {
    const int rc = bjx_batch_bans(n->parts[k].e, &bb[k]);
    if (rc != BJX_OK) fail(rc, "engine " + std::to_string(k) + ": " + bjx_engine_last_error(n->parts[k].e));
  }
  // ban-log lines: the engines' logs back to back
  std::vector<uint64_t> log_base(N + 1, 0), trip_pos(N + 1, 0);
  for (size_t k = 0; k < N; ++k) {
    log_base[k + 1] = log_base[k] + bb[k].log_bytes;
    trip_pos[k + 1] = trip_pos[k] + bb[k].n_trips;
  }
  n->ban_trips = trip_pos[N];
  n->log.resize(log_base[N]);
  n->log_off.resize(trip_pos[N] + 1);
  n->log_off[0] = 0;
  n->log_kind.resize(trip_pos[N]);
  {
    constexpr uint64_t kPiece = 1ull << 22;  // trips (or log bytes) per task
    std::vector<std::pair<uint32_t, uint64_t>> tasks;  // (engine, first trip / byte), two kinds
    for (size_t k = 0; k < N; ++k)
      for (uint64_t t = 0; t < std::max(bb[k].n_trips, bb[k].log_bytes); t += kPiece) tasks.push_back({(uint32_t)k, t});
    par_for(tasks.size(), T, [&](size_t i) {
      const size_t k = tasks[i].first;
      const uint64_t a = tasks[i].second;
      const bjx_ban_batch &b = bb[k];
      if (a < b.log_bytes) memcpy(&n->log[log_base[k] + a], b.log + a, std::min(kPiece, b.log_bytes - a));
      for (uint64_t t = a; t < std::min(a + kPiece, b.n_trips); ++t) {
        n->log_off[trip_pos[k] + t + 1] = log_base[k] + b.log_off[t + 1];
        n->log_kind[trip_pos[k] + t] = b.log_kind[t];
      }
    });
  }
  // per-IP records
  constexpr size_t kBuckets = 256;
  struct Item {
    uint64_t h;
    uint32_t k, r;
  };
  std::vector<std::vector<uint64_t>> hs(N);
  std::vector<std::vector<uint32_t>> cnt(N, std::vector<uint32_t>(kBuckets, 0));
  par_for(N, T, [&](size_t k) {
    const bjx_ban_batch &b = bb[k];
    hs[k].resize(b.n_ips);
    for (uint64_t r = 0; r < b.n_ips; ++r) {
      hs[k][r] = ip_key(b.ip_bytes + b.ip_off[r], b.ip_off[r + 1] - b.ip_off[r]);
      ++cnt[k][hs[k][r] >> 56];
    }
  });
  std::vector<size_t> boff(kBuckets + 1, 0);
  std::vector<std::vector<size_t>> at(N, std::vector<size_t>(kBuckets));
  for (size_t q = 0; q < kBuckets; ++q) {
    size_t o = boff[q];
    for (size_t k = 0; k < N; ++k) {
      at[k][q] = o;
      o += cnt[k][q];
    }
    boff[q + 1] = o;
  }
  std::vector<Item> items(boff[kBuckets]);
  par_for(N, T, [&](size_t k) {
    std::vector<size_t> &a = at[k];
    for (uint64_t r = 0; r < bb[k].n_ips; ++r) items[a[hs[k][r] >> 56]++] = Item{hs[k][r], (uint32_t)k, (uint32_t)r};
  });
  struct Merged {
    bjx_ip_decision d;
    uint32_t k, r;  // where the IP bytes are
  };
  std::vector<std::vector<Merged>> out(kBuckets);
  par_for(kBuckets, T, [&](size_t q) {
    const size_t b0 = boff[q], b1 = boff[q + 1];
    if (b0 == b1) return;
    size_t cap = 16;
    while (cap < 2 * (b1 - b0)) cap <<= 1;
    std::vector<uint32_t> tab(cap, 0xFFFFFFFFu);
    std::vector<uint64_t> th;
    std::vector<Merged> &o = out[q];
    for (size_t i = b0; i < b1; ++i) {
      const Item &it = items[i];
      const bjx_ban_batch &b = bb[it.k];
      const uint8_t *ip = b.ip_bytes + b.ip_off[it.r];
      const size_t len = b.ip_off[it.r + 1] - b.ip_off[it.r];
      bjx_ip_decision d = b.ips[it.r];
      d.trip_idx += trip_base[it.k];
      size_t s = it.h & (cap - 1);
      for (;; s = (s + 1) & (cap - 1)) {
        const uint32_t m = tab[s];
        if (m == 0xFFFFFFFFu) break;
        if (th[m] != it.h) continue;
        const bjx_ban_batch &c = bb[o[m].k];
        const size_t clen = c.ip_off[o[m].r + 1] - c.ip_off[o[m].r];
        if (clen == len && memcmp(c.ip_bytes + c.ip_off[o[m].r], ip, len) == 0) break;
      }
      if (tab[s] == 0xFFFFFFFFu) {
        tab[s] = (uint32_t)o.size();
        th.push_back(it.h);
        o.push_back(Merged{d, it.k, it.r});
        continue;
      }
      bjx_ip_decision &c = o[tab[s]].d;
      if (d.decision > c.decision) {
        c.decision = d.decision;
        c.trip_idx = d.trip_idx;
      }
      c.n_trips += d.n_trips;
      c.iptables |= d.iptables;
    }
  });
  std::vector<Merged> all;
  {
    size_t m = 0;
    for (auto &v : out) m += v.size();
    all.reserve(m);
    for (auto &v : out) all.insert(all.end(), v.begin(), v.end());
  }
  // trip order: LSD radix sort on trip_idx (16 bits a pass); trip indices of
  // distinct IPs are distinct, so stability is not even needed
  {
    std::vector<Merged> tmp(all.size());
    uint64_t maxt = 0;
    for (auto &x : all) maxt = std::max<uint64_t>(maxt, x.d.trip_idx);
    for (int shift = 0; shift < 64 && (shift == 0 || (maxt >> shift)); shift += 16) {
      std::vector<size_t> c(65537, 0);
      for (auto &x : all) ++c[((x.d.trip_idx >> shift) & 0xFFFF) + 1];
      for (size_t i = 1; i < c.size(); ++i) c[i] += c[i - 1];
      for (auto &x : all) tmp[c[(x.d.trip_idx >> shift) & 0xFFFF]++] = x;
      all.swap(tmp);
    }
  }
  n->ips.resize(all.size());
  n->ipo.resize(all.size() + 1);
  n->ipo[0] = 0;
  for (size_t i = 0; i < all.size(); ++i) {
    const bjx_ban_batch &b = bb[all[i].k];
    n->ips[i] = all[i].d;
    n->ipo[i + 1] = n->ipo[i] + (b.ip_off[all[i].r + 1] - b.ip_off[all[i].r]);
  }
  n->ipb.resize(n->ipo[all.size()]);
  par_for(all.size() ? T : 0, T, [&](size_t t) {
    for (size_t i = t; i < all.size(); i += T) {
      const bjx_ban_batch &b = bb[all[i].k];
      memcpy(n->ipb.data() + n->ipo[i], b.ip_bytes + b.ip_off[all[i].r], n->ipo[i + 1] - n->ipo[i]);
    }
  });
}

void run_batch(bjx_node *n, const bjx_ruleset *rs, const uint8_t *const *chunks, const size_t *lens, int64_t now_ns,
               uint32_t flags, bjx_batch_result *out) {
  const size_t N = n->parts.size();
  const uint32_t match_flags = flags & ~(uint32_t)BJX_EMIT_BANS;
  n->bans = false;
  if (N == 1 && !n->force_exchange) {  // nothing to exchange: the engine's own rate-limit stage
    Part &P = n->parts[0];
    const int rc = bjx_process_batch(P.e, rs, chunks[0], lens[0], now_ns, flags, out);
    if (rc != BJX_OK) fail(rc, std::string("engine 0: ") + bjx_engine_last_error(P.e));
    n->bans = (flags & BJX_EMIT_BANS) != 0;  // bjx_node_batch_bans hands out the engine's own
    return;
  }
  // 1. match each chunk
  each(n, [&](size_t k) { return bjx_match_batch(n->parts[k].e, rs, chunks[k], lens[k], now_ns, match_flags, &n->parts[k].res); });
  for (size_t k = 0; k + 1 < N; ++k)
    if (n->parts[k].res.consumed_bytes != lens[k])
      fail(BJX_ERR_ARG, "chunk " + std::to_string(k) + " does not end in '\\n' (only the last chunk may hold a partial line)");
  // 2. partition by owner
  each(n, [&](size_t k) {
    n->parts[k].send.assign(3 * N, 0);
    return bjx_events_partition(n->parts[k].e, (uint32_t)N, n->parts[k].send.data());
  });
  // segment offsets: send side owner-major, receive side source-major
  std::vector<uint64_t> s_off(3 * N * N), r_off(3 * N * N), recv_counts(3 * N * N);
  std::vector<uint64_t> s_tot(3 * N, 0), r_tot(3 * N, 0);
  for (size_t k = 0; k < N; ++k)
    for (size_t p = 0; p < N; ++p)
      for (int c = 0; c < 3; ++c) {
        const uint64_t v = n->parts[k].send[3 * p + c];
        s_off[(k * N + p) * 3 + c] = s_tot[3 * k + c];
        s_tot[3 * k + c] += v;
        r_off[(p * N + k) * 3 + c] = r_tot[3 * p + c];
        r_tot[3 * p + c] += v;
        recv_counts[(p * N + k) * 3 + c] = v;
      }
  // 3. pack, then move each (source, owner) segment
  each(n, [&](size_t k) {
    Part &P = n->parts[k];
    P.s_lines.ensure(s_tot[3 * k] * kLineRec + 1);
    P.s_ev.ensure(s_tot[3 * k + 1] * 4 + 1);
    P.s_bytes.ensure(s_tot[3 * k + 2] + 1);
    if (flags & BJX_COPY_RESULTS) P.s_out.ensure(s_tot[3 * k + 1] + 1);
    P.r_lines.ensure(r_tot[3 * k] * kLineRec + 1);
    P.r_ev.ensure(r_tot[3 * k + 1] * 4 + 1);
    P.r_bytes.ensure(r_tot[3 * k + 2] + 1);
    if (flags & BJX_COPY_RESULTS) P.r_out.ensure(r_tot[3 * k + 1] + 1);
    return bjx_events_pack(P.e, reinterpret_cast<bjx_event_line *>(P.s_lines.p), reinterpret_cast<uint32_t *>(P.s_ev.p),
                           P.s_bytes.p);
  });
  static const size_t unit[3] = {kLineRec, 4, 1};
  for (int c = 0; c < 3; ++c)
    exchange(n, [&](size_t p, size_t k, void **d, const void **s, size_t *b) {
      DevMem *dst[3] = {&n->parts[p].r_lines, &n->parts[p].r_ev, &n->parts[p].r_bytes};
      const DevMem *src[3] = {&n->parts[k].s_lines, &n->parts[k].s_ev, &n->parts[k].s_bytes};
      *d = dst[c]->p + r_off[(p * N + k) * 3 + c] * unit[c];
      *s = src[c]->p + s_off[(k * N + p) * 3 + c] * unit[c];
      *b = recv_counts[(p * N + k) * 3 + c] * unit[c];
    });
  sync_copies(n);
  if (!(flags & BJX_COPY_RESULTS)) {
    // 4. owners apply their events in source order and list, per source, the
    // packed indices of the events that tripped
    each(n, [&](size_t p) {
      Part &P = n->parts[p];
      std::vector<uint64_t> base(N);
      for (size_t k = 0; k < N; ++k) base[k] = s_off[(k * N + p) * 3 + 1];
      P.tr_counts.assign(N, 0);
      P.r_trips.ensure(r_tot[3 * p + 1] * 4 + 4);
      return bjx_apply_events_trips(P.e, rs, reinterpret_cast<const bjx_event_line *>(P.r_lines.p),
                                    reinterpret_cast<const uint32_t *>(P.r_ev.p), P.r_bytes.p, (uint32_t)N,
                                    &recv_counts[p * N * 3], base.data(), reinterpret_cast<uint32_t *>(P.r_trips.p),
                                    P.tr_counts.data());
    });
    // 5. the trip lists back to their sources (owner order)
    std::vector<uint64_t> o_off(N * N), t_off(N * N), t_tot(N, 0);
    for (size_t p = 0; p < N; ++p) {
      uint64_t o = 0;
      for (size_t k = 0; k < N; ++k) {
        o_off[p * N + k] = o;
        o += n->parts[p].tr_counts[k];
      }
    }
    for (size_t k = 0; k < N; ++k)
      for (size_t p = 0; p < N; ++p) {
        t_off[k * N + p] = t_tot[k];
        t_tot[k] += n->parts[p].tr_counts[k];
      }
    for (size_t k = 0; k < N; ++k) n->parts[k].s_trips.ensure(t_tot[k] * 4 + 4);
    exchange(n, [&](size_t k, size_t p, void **d, const void **s, size_t *b) {
      *d = n->parts[k].s_trips.p + t_off[k * N + p] * 4;
      *s = n->parts[p].r_trips.p + o_off[p * N + k] * 4;
      *b = n->parts[p].tr_counts[k] * 4;
    });
    sync_copies(n);
    each(n, [&](size_t k) {
      return bjx_finish_batch_trips(n->parts[k].e, reinterpret_cast<const uint32_t *>(n->parts[k].s_trips.p), t_tot[k], flags,
                                    &n->parts[k].res);
    });
  } else {
    // 4. owners apply their events in source order
    each(n, [&](size_t p) {
      Part &P = n->parts[p];
      return bjx_apply_events(P.e, rs, reinterpret_cast<const bjx_event_line *>(P.r_lines.p),
                              reinterpret_cast<const uint32_t *>(P.r_ev.p), P.r_bytes.p, (uint32_t)N, &recv_counts[p * N * 3],
                              P.r_out.p);
    });
    // 5. outcomes back to the sources (owner-major, the pack order)
    exchange(n, [&](size_t k, size_t p, void **d, const void **s, size_t *b) {
      *d = n->parts[k].s_out.p + s_off[(k * N + p) * 3 + 1];
      *s = n->parts[p].r_out.p + r_off[(p * N + k) * 3 + 1];
      *b = recv_counts[(p * N + k) * 3 + 1];
    });
    sync_copies(n);
    each(n, [&](size_t k) { return bjx_finish_batch(n->parts[k].e, n->parts[k].s_out.p, flags, &n->parts[k].res); });
  }
  // 6. merge in chunk (= stream) order
  bjx_batch_result r{};
  n->trips.clear(); n->trips_c.clear(); n->results.clear(); n->line_flags.clear();
  std::vector<uint64_t> trip_base(N, 0);
  uint64_t line_base = 0, byte_base = 0;
  for (size_t k = 0; k < N; ++k) {
    const bjx_batch_result &x = n->parts[k].res;
    if (flags & BJX_TRIPS_COMPACT) {
      trip_base[k] = n->trips_c.size();
      for (uint64_t t = 0; t < x.n_trips; ++t) n->trips_c.push_back(x.trips_compact[t] + (byte_base << 24));
    } else {
      trip_base[k] = n->trips.size();
      for (uint64_t t = 0; t < x.n_trips; ++t) {
        bjx_trip tr = x.trips[t];
        tr.line_idx += line_base;
        tr.line_offset += byte_base;
        n->trips.push_back(tr);
      }
    }
    if (flags & BJX_COPY_RESULTS) {
      if (x.n_lines) n->line_flags.insert(n->line_flags.end(), x.line_flags, x.line_flags + x.n_lines);
      const size_t r0 = n->results.size();
      if (x.n_results) n->results.insert(n->results.end(), x.results, x.results + x.n_results);
      for (size_t i = r0; i < n->results.size(); ++i) n->results[i].line_idx += line_base;
    }
    r.n_lines += x.n_lines;
    r.n_results += x.n_results;
    r.n_events += x.n_events;
    r.device_ms = std::max(r.device_ms, x.device_ms);
    r.match_kernel_ms = std::max(r.match_kernel_ms, x.match_kernel_ms);
    line_base += x.n_lines;
    byte_base += lens[k];
  }
  r.consumed_bytes = byte_base - lens[N - 1] + n->parts[N - 1].res.consumed_bytes;
  if (flags & BJX_TRIPS_COMPACT) {
    r.n_trips = n->trips_c.size();
    r.trips_compact = r.n_trips ? n->trips_c.data() : nullptr;
  } else {
    r.n_trips = n->trips.size();
    r.trips = r.n_trips ? n->trips.data() : nullptr;
  }
  if (flags & BJX_COPY_RESULTS) {
    r.line_flags = r.n_lines ? n->line_flags.data() : nullptr;
    r.results = r.n_results ? n->results.data() : nullptr;
  }
  if (flags & BJX_EMIT_BANS) {
    merge_bans(n, trip_base);
    n->bans = true;
  }
  *out = r;
}

}  // namespace

extern "C" int bjx_node_create(const int *devices, size_t n_devices, const bjx_engine_options *opts, bjx_node **out,
                               char *err, size_t err_len) {
  auto say = [&](const std::string &m) {
    if (err && err_len) {
      strncpy(err, m.c_str(), err_len - 1);
      err[err_len - 1] = 0;
    }
  };
  if (!devices || !out || n_devices == 0 || n_devices > 256) {
    say("bjx_node_create: need 1..256 devices and an out pointer");
    return BJX_ERR_ARG;
  }
  *out = nullptr;
  bjx_node *n = new bjx_node();
  n->parts.resize(n_devices);
  int rc = BJX_OK;
  for (size_t k = 0; k < n_devices && rc == BJX_OK; ++k) {
    Part &P = n->parts[k];
    P.dev = devices[k];
    for (DevMem *m : {&P.s_lines, &P.s_ev, &P.s_bytes, &P.s_out, &P.r_lines, &P.r_ev, &P.r_bytes, &P.r_out, &P.r_trips, &P.s_trips})
      m->dev = P.dev;
    char e2[512] = {0};
    rc = bjx_engine_create(P.dev, opts, &P.e, e2, sizeof e2);
    if (rc != BJX_OK) {
      say("engine " + std::to_string(k) + ": " + e2);
      break;
    }
    if (hipSetDevice(P.dev) != hipSuccess || hipStreamCreateWithFlags(&P.copy, hipStreamNonBlocking) != hipSuccess) {
      say("engine " + std::to_string(k) + ": cannot create the exchange stream");
      rc = BJX_ERR_DEVICE;
    }
  }
  if (rc == BJX_OK) {
    // direct xGMI access between every pair of distinct GPUs where the
    // platform offers it (hipMemcpyPeerAsync works either way)
    for (auto &A : n->parts)
      for (auto &B : n->parts) {
        if (A.dev == B.dev) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, A.dev, B.dev) == hipSuccess && can && hipSetDevice(A.dev) == hipSuccess) {
          const hipError_t r = hipDeviceEnablePeerAccess(B.dev, 0);
          if (r != hipSuccess) (void)hipGetLastError();  // already enabled
        }
      }
  }
  if (rc == BJX_OK) {
    // the RCCL clique when every engine has a GPU of its own (an RCCL
    // communicator holds one rank per GPU); peer copies otherwise, on request
    // (BJX_NODE_EXCHANGE=peer), or when RCCL cannot be set up here
    const char *mode = getenv("BJX_NODE_EXCHANGE");
    const char *force = getenv("BJX_NODE_FORCE_EXCHANGE");
    n->force_exchange = force && atoi(force) == 1;
    bool distinct = true;
    for (size_t a = 0; a < n_devices; ++a)
      for (size_t b = a + 1; b < n_devices; ++b) distinct = distinct && devices[a] != devices[b];
    if (distinct && !(mode && strcmp(mode, "peer") == 0) && (n_devices > 1 || n->force_exchange)) {
      n->comms.assign(n_devices, nullptr);
      std::vector<int> dl(devices, devices + n_devices);
      const ncclResult_t r = ncclCommInitAll(n->comms.data(), (int)n_devices, dl.data());
      if (r != ncclSuccess) {
        n->comms.clear();
        if (mode && strcmp(mode, "rccl") == 0) {
          say(std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
          rc = BJX_ERR_DEVICE;
        }
      }
    } else if (mode && strcmp(mode, "rccl") == 0) {
      say("BJX_NODE_EXCHANGE=rccl needs one engine per GPU");
      rc = BJX_ERR_ARG;
    }
  }
  if (rc != BJX_OK) {
    bjx_node_destroy(n);
    return rc;
  }
  *out = n;
  return BJX_OK;
}

extern "C" int bjx_node_exchange_kind(const bjx_node *n) { return !n ? -1 : n->comms.empty() ? 0 : 1; }

extern "C" void bjx_node_destroy(bjx_node *n) {
  if (!n) return;
  for (ncclComm_t c : n->comms)
    if (c) (void)ncclCommDestroy(c);
  for (auto &P : n->parts) {
    for (DevMem *m : {&P.s_lines, &P.s_ev, &P.s_bytes, &P.s_out, &P.r_lines, &P.r_ev, &P.r_bytes, &P.r_out, &P.r_trips,
                      &P.s_trips}) m->release();
    if (P.copy) {
      (void)hipSetDevice(P.dev);
      (void)hipStreamDestroy(P.copy);
    }
    bjx_engine_destroy(P.e);
  }
  delete n;
}

extern "C" size_t bjx_node_size(const bjx_node *n) { return n ? n->parts.size() : 0; }

extern "C" bjx_engine *bjx_node_engine(bjx_node *n, size_t k) { return n && k < n->parts.size() ? n->parts[k].e : nullptr; }

extern "C" const char *bjx_node_last_error(bjx_node *n) { return n ? n->last_error.c_str() : "no node"; }

extern "C" int bjx_node_set_decision_lists(bjx_node *n, const bjx_decision_entry *entries, size_t count) {
  return guarded(n, [&]() -> int {
    each(n, [&](size_t k) { return bjx_engine_set_decision_lists(n->parts[k].e, entries, count); });
    return BJX_OK;
  });
}

extern "C" int bjx_node_set_ban_options(bjx_node *n, const bjx_ban_options *opts) {
  return guarded(n, [&]() -> int {
    each(n, [&](size_t k) { return bjx_engine_set_ban_options(n->parts[k].e, opts); });
    return BJX_OK;
  });
}

extern "C" int bjx_node_process_chunks(bjx_node *n, const bjx_ruleset *rs, const uint8_t *const *chunks, const size_t *lens,
                                       int64_t now_ns, uint32_t flags, bjx_batch_result *out) {
  if (!rs || !out || !chunks || !lens || !(flags & BJX_INPUT_DEVICE)) return BJX_ERR_ARG;
  return guarded(n, [&]() -> int {
    memset(out, 0, sizeof *out);
    run_batch(n, rs, chunks, lens, now_ns, flags, out);
    return BJX_OK;
  });
}

extern "C" int bjx_node_process_batch(bjx_node *n, const bjx_ruleset *rs, const uint8_t *bytes, size_t len, int64_t now_ns,
                                      uint32_t flags, bjx_batch_result *out) {
  if (!rs || !out || (len && !bytes) || (flags & BJX_INPUT_DEVICE)) return BJX_ERR_ARG;
  return guarded(n, [&]() -> int {
    memset(out, 0, sizeof *out);
    const size_t N = n->parts.size();
    // chunk boundaries: just past the first '\n' at or after k * len / N
    std::vector<const uint8_t *> ptr(N);
    std::vector<size_t> lens(N);
    size_t b = 0;
    for (size_t k = 0; k < N; ++k) {
      size_t e = len;
      if (k + 1 < N) {
        e = std::max(b, (size_t)((unsigned __int128)len * (k + 1) / N));
        const void *nl = e < len ? memchr(bytes + e, '\n', len - e) : nullptr;
        e = nl ? (size_t)(static_cast<const uint8_t *>(nl) - bytes) + 1 : len;
        if (!nl) {  // no '\n' left: the remainder is one partial line for the last chunk
          e = b;
        }
      }
      ptr[k] = bytes + b;
      lens[k] = e - b;
      b = e;
    }
    run_batch(n, rs, ptr.data(), lens.data(), now_ns, flags, out);
    return BJX_OK;
  });
}

extern "C" int bjx_node_batch_bans(bjx_node *n, bjx_ban_batch *out) {
  if (!out) return BJX_ERR_ARG;
  return guarded(n, [&]() -> int {
    memset(out, 0, sizeof *out);
    if (!n->bans) fail(BJX_ERR_ARG, "bjx_node_batch_bans: the last batch ran without BJX_EMIT_BANS");
    if (n->parts.size() == 1) {
      const int rc = bjx_batch_bans(n->parts[0].e, out);
      if (rc != BJX_OK) fail(rc, std::string("engine 0: ") + bjx_engine_last_error(n->parts[0].e));
      return BJX_OK;
    }
    out->n_ips = n->ips.size();
    out->ips = out->n_ips ? n->ips.data() : nullptr;
    out->n_trips = n->ban_trips;
    out->log_bytes = n->log.size();
    out->log = out->log_bytes ? n->log.data() : nullptr;
    out->log_off = n->log_off.data();
    out->log_kind = n->ban_trips ? n->log_kind.data() : nullptr;
    out->ip_bytes = n->ipb.empty() ? nullptr : n->ipb.data();
    out->ip_off = n->ipo.data();
    return BJX_OK;
  });
}

// Each IP lives on exactly one shard; the lookups ask every engine rather
// than re-deriving the owner hash on the host.
extern "C" int bjx_node_state_get(bjx_node *n, const char *ip, size_t ip_len, const char *name, size_t name_len,
                                  int64_t *num_hits, int64_t *interval_start_ns) {
  if (!n) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(n->mu);  // not between one batch's shard phases
  for (auto &P : n->parts) {
    const int rc = bjx_state_get(P.e, ip, ip_len, name, name_len, num_hits, interval_start_ns);
    if (rc != 0) return rc;
  }
  return 0;
}

extern "C" int64_t bjx_node_state_len(bjx_node *n) {
  if (!n) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(n->mu);
  int64_t t = 0;
  for (auto &P : n->parts) {
    const int64_t v = bjx_state_len(P.e);
    if (v < 0) return v;
    t += v;
  }
  return t;
}

extern "C" size_t bjx_node_state_dump(bjx_node *n, char *out, size_t cap) {
  if (!n) return 0;
  std::lock_guard<std::mutex> g(n->mu);
  size_t t = 0;
  for (auto &P : n->parts) {
    const size_t room = out && t < cap ? cap - t : 0;
    t += bjx_state_dump(P.e, room ? out + t : nullptr, room);
  }
  return t;
}

extern "C" int bjx_node_state_stats_get(bjx_node *n, bjx_state_stats *out) {
  if (!n || !out) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(n->mu);
  memset(out, 0, sizeof *out);
  for (auto &P : n->parts) {
    bjx_state_stats s{};
    const int rc = bjx_state_stats_get(P.e, &s);
    if (rc != BJX_OK) return rc;
    out->ips += s.ips; out->ip_slots += s.ip_slots; out->states += s.states; out->state_slots += s.state_slots;
    out->arena_bytes += s.arena_bytes; out->arena_capacity += s.arena_capacity; out->device_bytes += s.device_bytes;
    out->rehashes += s.rehashes;
  }
  return BJX_OK;
}

extern "C" int bjx_node_state_clear(bjx_node *n) {
  if (!n) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(n->mu);
  for (auto &P : n->parts) {
    const int rc = bjx_state_clear(P.e);
    if (rc != BJX_OK) return rc;
  }
  return BJX_OK;
}
