/*
 * banjax_gpu.h — C ABI of libbanjax_gpu.so, the MI355X engine behind banjax's
 * regex rate-limiting log tailer.
 *
 * Drop-in boundary: a Go host keeps banjax's surface (YAML schema,
 * consumeLine/RunLogTailer, RegexRateLimitStates, BannerInterface, decision
 * lists) and calls these entry points through cgo (binding: INTEGRATION.md).
 * Plain pointers and sizes only; no GPU or torch types cross the boundary.
 *
 * Reference interfaces replaced (deflect-ca/banjax):
 *   bjx_ruleset_compile     RegexWithRate.UnmarshalYAML        internal/config.go:96-131
 *                           (regexp.Compile per rule, config.go:110; reload: config_holder.go:55-66)
 *   bjx_engine_set_decision_lists  newStaticDecisionListsFromConfig  internal/decision.go:278-374
 *   bjx_process_batch       consumeLine + applyRegexToLog per line
 *                           internal/regex_rate_limiter.go:113-269, fed by RunLogTailer :21-78
 *   bjx_state_get           RegexRateLimitStates.Get           internal/rate_limit.go:81-96
 *   bjx_state_len           RegexRateLimitStates.Len           internal/rate_limit.go:30-35
 *   bjx_state_dump          RegexRateLimitStates.String        internal/rate_limit.go:98-103,204-220
 *   bjx_node_*              the same surface over every GPU of the host (one RegexRateLimitStates,
 *                           banjax.go:80; one consumer goroutine, regex_rate_limiter.go:54-77)
 *   bjx_tailer_*            tail.TailFile(Follow, SeekEnd) + tailer.Lines in RunLogTailer
 *                           internal/regex_rate_limiter.go:21-78 (github.com/hpcloud/tail v1.0.0)
 *
 * Ownership: input buffers are borrowed for the duration of a call.  Result
 * arrays are engine-owned and valid until the next bjx_process_batch on the
 * same engine.  Rulesets are immutable; a reload compiles a new one (state is
 * keyed by rule *name* and survives, as in the reference).
 * Threading: one bjx_process_batch at a time per engine; bjx_state_* may be
 * called from other threads (they serialise on the engine lock, as the
 * reference's mutex does, rate_limit.go:19).
 * Errors: int status (BJX_OK = 0, negative code) + a caller buffer for the
 * message.  Malformed log lines are data (BJX_LINE_ERROR), never API errors.
 */
#ifndef BANJAX_GPU_H
#define BANJAX_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BJX_ABI_VERSION 5  /* 5: IP slots of the exchange byte pool 4-byte aligned; trips-only node return */

enum bjx_status {
  BJX_OK = 0,
  BJX_ERR_REGEX = -1,       /* a rule's regex does not compile (Go error text in err) */
  BJX_ERR_ARG = -2,
  BJX_ERR_DEVICE = -3,      /* HIP runtime failure / no GPU */
  BJX_ERR_NOMEM = -4,
  BJX_ERR_TOO_COMPLEX = -5, /* rule exceeds the engine's automaton limits */
  BJX_ERR_CAPACITY = -6,    /* state tables full (raise bjx_engine_options) */
  BJX_ERR_DECISION = -7,    /* unknown decision string / value */
  BJX_TAIL_STOPPED = -8,    /* bjx_tailer_next: the followed file was deleted or renamed (tail stops) */
  BJX_ERR_IO = -9           /* bjx_tailer: read/open failure other than "not there yet" */
};

/* Decision, reference internal/decision.go:20-28 */
enum bjx_decision { BJX_ALLOW = 1, BJX_CHALLENGE = 2, BJX_NGINX_BLOCK = 3, BJX_IPTABLES_BLOCK = 4 };
/* RateLimitMatchType, reference internal/rate_limit.go:175-181 */
enum bjx_match_type { BJX_FIRST_TIME = 0, BJX_OUTSIDE_INTERVAL = 1, BJX_INSIDE_INTERVAL = 2 };
/* ConsumeLineResult.{Error,OldLine,Exempted}, reference regex_rate_limiter.go:80-85 */
enum bjx_line_flag { BJX_LINE_ERROR = 1, BJX_LINE_OLD = 2, BJX_LINE_EXEMPTED = 4 };

typedef struct bjx_str {
  const char *ptr;
  size_t len;
} bjx_str;

/* One RegexWithRate (config.go:87-94), already decoded from YAML by the host. */
typedef struct bjx_rule_spec {
  bjx_str name;               /* Rule */
  bjx_str regex;              /* RE2 / Go regexp syntax */
  int64_t interval_ns;        /* time.Duration(interval * 1e9), computed by the host (config.go:116) */
  int64_t hits_per_interval;  /* HitsPerInterval (Go int) */
  int32_t decision;           /* enum bjx_decision (ParseDecision, decision.go:30-43) */
  const bjx_str *hosts_to_skip; /* HostsToSkip keys whose value is true */
  size_t n_hosts_to_skip;
} bjx_rule_spec;

/* per_site_regexes_with_rates[host] (config.go:19) */
typedef struct bjx_site_rules {
  bjx_str host;
  const bjx_rule_spec *rules;
  size_t n_rules;
} bjx_site_rules;

typedef struct bjx_ruleset bjx_ruleset;
typedef struct bjx_engine bjx_engine;

/* Compile every rule (regexp.Compile semantics, syntax.Perl flags).  Rule
   indices: global rules 0..n_global-1, then each site's rules in order.  On a
   compile error returns BJX_ERR_REGEX, *err_rule = failing index and the Go
   error text ("error parsing regexp: ...") in err, and no ruleset. */
int bjx_ruleset_compile(const bjx_rule_spec *global_rules, size_t n_global, const bjx_site_rules *per_site,
                        size_t n_sites, bjx_ruleset **out, int64_t *err_rule, char *err, size_t err_len);
void bjx_ruleset_release(bjx_ruleset *rs);
size_t bjx_ruleset_num_rules(const bjx_ruleset *rs);
/* Per-rule automaton statistics (DFA states, rune classes) for diagnostics. */
int bjx_ruleset_rule_info(const bjx_ruleset *rs, size_t rule_idx, uint32_t *dfa_states, uint32_t *classes,
                          uint32_t *flags);

typedef struct bjx_engine_options {
  uint64_t ip_capacity;       /* distinct IPs kept (reference never evicts, rate_limit.go:45-67); 0 = default */
  uint64_t state_capacity;    /* distinct (ip, rule name) states; 0 = default */
  uint64_t ip_arena_bytes;    /* bytes of IP strings; 0 = default */
} bjx_engine_options;

/* One engine per GPU (device index as HIP sees it).  opts may be NULL. */
int bjx_engine_create(int device, const bjx_engine_options *opts, bjx_engine **out, char *err, size_t err_len);
void bjx_engine_destroy(bjx_engine *e);

/* Static decision lists used by CheckIsAllowed (decision.go:185-216): one
   entry per IP/CIDR string of global_decision_lists (site.ptr == NULL) or
   per_site_decision_lists[site], in config order.  Replaces previous lists
   (StaticDecisionLists.UpdateFromConfig on reload, banjax.go:113). */
typedef struct bjx_decision_entry {
  bjx_str site;     /* ptr == NULL: global */
  int32_t decision; /* enum bjx_decision */
  bjx_str ip;       /* IP or CIDR text */
} bjx_decision_entry;
int bjx_engine_set_decision_lists(bjx_engine *e, const bjx_decision_entry *entries, size_t n);

/* RuleResult of one matched (line, rule) pair, reference regex_rate_limiter.go:87-93.
   RegexMatch is implied (only matches are reported, as consumeLine does, :189,208). */
typedef struct bjx_rule_result {
  uint64_t line_idx;
  uint32_t rule_idx;  /* ruleset rule index */
  uint16_t rule_pos;  /* position in the line's evaluation order (per-site rules, then global) */
  uint8_t skip_host;
  uint8_t seen_ip;
  uint8_t match_type; /* enum bjx_match_type */
  uint8_t exceeded;
  uint8_t _pad[2];
} bjx_rule_result;

/* A rate-limit trip (RateLimitResult.Exceeded): the host replays
   Banner.BanOrChallengeIp then Banner.LogRegexBan for it, in the order given
   (regex_rate_limiter.go:254-266).  Offsets are relative to the line start in
   the caller's buffer. */
typedef struct bjx_trip {
  uint64_t line_idx;
  uint64_t line_offset; /* byte offset of the line in the batch */
  uint32_t line_len;    /* without '\n' */
  uint32_t rule_idx;
  int64_t ts_ns;        /* parsed line timestamp (LogRegexBan logTime) */
  uint32_t ip_off, ip_len;
  uint32_t host_off, host_len;
  uint32_t rest_off;    /* timeIpRest[2]: rest runs to line_len */
  int32_t decision;
} bjx_trip;

enum bjx_batch_flags {
  BJX_INPUT_DEVICE = 1,   /* bytes is a device pointer already resident in HBM */
  BJX_COPY_RESULTS = 2,   /* also copy per-line flags and RuleResults to host memory */
  BJX_EMIT_BANS = 4,      /* also build the batch's decision updates and ban-log lines (bjx_batch_bans) */
  BJX_BAN_RECORDS_ONLY = 8, /* with BJX_EMIT_BANS: the per-IP decision records only; no LogRegexBan lines
                              are built or copied (log_bytes 0, every log_kind 0) */
  BJX_TRIPS_COMPACT = 16    /* trips as 8-byte words in trips_compact (trips NULL): what the host cannot
                              re-derive from its own copy of the bytes -- which line, which rule */
};

/* BJX_TRIPS_COMPACT trip word: the line's byte offset in the batch (40 bits)
   and the rule index (24 bits).  Everything else in bjx_trip follows from the
   line's bytes: line_len = up to its '\n', ts / IP / host / rest = the first
   four space-separated fields (as consumeLine splits them), decision =
   the rule's, line_idx = the newlines before it. */
#define BJX_TRIP_OFFSET(w) ((uint64_t)(w) >> 24)
#define BJX_TRIP_RULE(w) ((uint32_t)((w) & 0xFFFFFFu))

typedef struct bjx_batch_result {
  uint64_t n_lines;        /* complete ('\n'-terminated) lines processed */
  uint64_t consumed_bytes; /* offset after the last '\n' (the caller carries the rest) */
  uint64_t n_results;      /* RuleResults (matched rules) */
  uint64_t n_events;       /* RuleResults that reached RegexRateLimitStates.Apply */
  uint64_t n_trips;
  const uint8_t *line_flags;        /* host, n_lines entries, if BJX_COPY_RESULTS */
  const bjx_rule_result *results;   /* host, n_results entries in reference order, if BJX_COPY_RESULTS */
  const bjx_trip *trips;            /* host, n_trips entries in reference order */
  double device_ms;                 /* device time of the batch (HIP events) */
  double match_kernel_ms;           /* device time of the match kernel alone */
  const uint64_t *trips_compact;    /* host, n_trips trip words in reference order, if BJX_TRIPS_COMPACT (ABI 4) */
} bjx_batch_result;

/* consumeLine for every complete line of bytes[0..n) with injected clock
   now_ns (time.Now(), used for OldLine). */
int bjx_process_batch(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns,
                      uint32_t flags, bjx_batch_result *out);

/* ---- Multi-GPU batch.  One engine per GPU; each matches its
   own contiguous chunk of the log, and RegexRateLimitStates shards by IP:
   event lines go to owner (ip_hash >> 32) % n_parts.  Sequence per engine:
     bjx_match_batch                     consumeLine up to Apply (no state touched)
     bjx_events_partition                per-owner sizes of the outgoing records
     bjx_events_pack                     records into caller device buffers, owner-major
     -- caller: all-to-all of the three buffers (RCCL) --
     bjx_apply_events                    Apply for the received records, in source order
     -- caller: all-to-all of the outcome bytes back --
     bjx_finish_batch                    trips / RuleResults of the local lines
   (trips only: bjx_apply_events_trips, the trip lists back, bjx_finish_batch_trips)
   Source order must be stream order (rank r holds the r-th chunk), which makes
   the owner's event order the reference's.  All buffers are device pointers
   allocated by the caller; the engine never retains them. */
typedef struct bjx_event_line {  /* 16 B (ABI 4; the owner hashes the IP bytes itself) */
  int64_t ts_ns;     /* parsed line timestamp */
  uint32_t ip_off;   /* offset of the IP bytes in this owner's part of the byte buffer: each IP
                        starts a 4-byte aligned slot of (ip_len + 3) & ~3 bytes, zero padded (ABI 5) */
  uint16_t ip_len;
  uint16_t n_events; /* events of the line; their rule indices follow in the event buffer */
} bjx_event_line;

int bjx_match_batch(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns, uint32_t flags,
                    bjx_batch_result *out);
/* counts[3*p + 0/1/2] = event lines / events / IP slot bytes going to owner p
   (host array); 1 <= n_parts <= 256.  The byte buffers are 4-byte aligned. */
int bjx_events_partition(bjx_engine *e, uint32_t n_parts, uint64_t *counts);
int bjx_events_pack(bjx_engine *e, bjx_event_line *d_lines, uint32_t *d_events, uint8_t *d_bytes);
/* received records of n_src sources, concatenated in source order; src_counts as
   bjx_events_partition's counts, one triple per source.  d_out: one outcome
   byte per received event (bit0 seenIp, bits1-2 MatchType, bit3 Exceeded). */
int bjx_apply_events(bjx_engine *e, const bjx_ruleset *rs, const bjx_event_line *d_lines, const uint32_t *d_events,
                     const uint8_t *d_bytes, uint32_t n_src, const uint64_t *src_counts, uint8_t *d_out);
/* d_outcomes: one byte per packed event, in bjx_events_pack order */
int bjx_finish_batch(bjx_engine *e, const uint8_t *d_outcomes, uint32_t flags, bjx_batch_result *out);
/* Trips-only round trip (a batch without BJX_COPY_RESULTS needs no per-event
   outcome): the owner hands back, per source, the packed indices of that
   source's events that came out Exceeded.  trip_base[k] is added to each index
   inside source k's received segment (the caller passes that segment's offset
   in source k's bjx_events_pack order); d_trips (device, room for every
   received event) gets the sources' lists concatenated in source order, each
   ascending; trip_counts[k] (host) their lengths.  Replaces the outcome bytes
   + bjx_finish_batch when the batch needs trips (and bans) only. */
int bjx_apply_events_trips(bjx_engine *e, const bjx_ruleset *rs, const bjx_event_line *d_lines, const uint32_t *d_events,
                           const uint8_t *d_bytes, uint32_t n_src, const uint64_t *src_counts, const uint64_t *trip_base,
                           uint32_t *d_trips, uint64_t *trip_counts);
/* d_trips: n packed event indices (bjx_events_pack order) that came out Exceeded,
   in any order; flags without BJX_COPY_RESULTS */
int bjx_finish_batch_trips(bjx_engine *e, const uint32_t *d_trips, uint64_t n, uint32_t flags, bjx_batch_result *out);

/* RegexRateLimitStates.Get(ip)[name]: 1 found (num_hits, start_ns set), 0 not found, <0 error. */
int bjx_state_get(bjx_engine *e, const char *ip, size_t ip_len, const char *name, size_t name_len,
                  int64_t *num_hits, int64_t *interval_start_ns);
/* RegexRateLimitStates.Len(): number of distinct IPs with state. */
int64_t bjx_state_len(bjx_engine *e);
/* Occupancy of the persistent rate-limit state in HBM.  The reference never
   evicts state (rate_limit.go:45-67) and neither does the engine: the tables
   grow (rehashed on the device, 3/4 load factor) until a batch's growth
   cannot be allocated, which returns BJX_ERR_CAPACITY; device_bytes lets the
   host watch that coming (metrics, alongside Len(): config.go:165). */
typedef struct bjx_state_stats {
  uint64_t ips;            /* distinct IP strings (RegexRateLimitStates.Len) */
  uint64_t ip_slots;       /* IP table capacity */
  uint64_t states;         /* (ip, rule name) states */
  uint64_t state_slots;    /* state table capacity */
  uint64_t arena_bytes;    /* IP string bytes stored */
  uint64_t arena_capacity;
  uint64_t device_bytes;   /* HBM held by the state tables and the arena */
  uint64_t rehashes;       /* table growths so far */
} bjx_state_stats;
int bjx_state_stats_get(bjx_engine *e, bjx_state_stats *out);
/* Drop every rate-limit state (a fresh RegexRateLimitStates). */
int bjx_state_clear(bjx_engine *e);
/* RegexRateLimitStates.String(): "ip:\n\trule:\n\t\t{hits start}\n" blocks, IPs in
   first-seen order.  Returns the full length (writes at most cap bytes). */
size_t bjx_state_dump(bjx_engine *e, char *out, size_t cap);

/* ---- Log-tail front end.  Replaces github.com/hpcloud/tail
   v1.0.0 as RunLogTailer uses it (regex_rate_limiter.go:30-58: Follow, start
   at EOF) with bulk reads into pinned buffers and batches of complete lines:
     - a line is the bytes before '\n' ('\r' kept), exactly tail.Line.Text;
     - a trailing partial line is held until its '\n' arrives (tail seeks back
       over it and re-reads, same effect);
     - a missing file is waited for, then followed from its end (MustExist false);
     - a file that shrinks below the read offset was truncated: it is re-read
       from offset 0 and the held partial line is dropped (tail's reopen);
     - a file deleted or renamed away stops the tail (ReOpen false):
       bjx_tailer_next returns BJX_TAIL_STOPPED once every batch is handed out.
   A reader thread fills the next pinned slot and issues its host-to-device
   copy on a copy stream while the caller runs bjx_process_batch on the
   previous slot (double buffering with slots = 2).  Batch = one config
   snapshot for all its lines (the reference reads configHolder.Get() per
   line, :58-59; a reload takes effect at the next batch). */
typedef struct bjx_tailer bjx_tailer;

typedef struct bjx_tailer_options {
  int32_t device;        /* GPU that receives each batch (HBM copy); -1 = host framing only */
  int32_t from_start;    /* 0: first open seeks to EOF (Whence io.SeekEnd, :32-36); 1: offset 0 */
  uint32_t slots;        /* pinned (+ device) buffers in flight; 0 = 2 */
  uint32_t poll_ms;      /* wait at EOF before looking again; 0 = 20 */
  uint64_t batch_bytes;  /* largest batch; 0 = 256 MiB (a longer line grows the slot) */
} bjx_tailer_options;

typedef struct bjx_tail_batch {
  uint32_t slot;               /* give back with bjx_tailer_release */
  uint32_t reopened;           /* the file was truncated and re-read from 0 before this batch */
  const uint8_t *host_bytes;   /* pinned host copy: trips' line offsets index it */
  const uint8_t *device_bytes; /* HBM copy, complete: pass to bjx_process_batch with BJX_INPUT_DEVICE (NULL if device = -1) */
  uint64_t n_bytes;            /* ends with '\n' */
  uint64_t file_offset;        /* file offset of host_bytes[0] */
} bjx_tail_batch;

int bjx_tailer_open(const char *path, size_t path_len, const bjx_tailer_options *opts, bjx_tailer **out, char *err,
                    size_t err_len);
/* Next batch, oldest first.  Waits up to timeout_ms (< 0: forever).  Returns
   1 with *out filled, 0 on timeout, BJX_TAIL_STOPPED, or an error code. */
int bjx_tailer_next(bjx_tailer *t, int32_t timeout_ms, bjx_tail_batch *out);
int bjx_tailer_release(bjx_tailer *t, uint32_t slot);
/* bytes read from the file so far / handed out in batches (held partial line = difference) */
int bjx_tailer_stats(bjx_tailer *t, uint64_t *read_bytes, uint64_t *batched_bytes, uint64_t *batches);
void bjx_tailer_close(bjx_tailer *t);

/* Last error message of an engine call. */
const char *bjx_engine_last_error(bjx_engine *e);
/* ---- Trip -> decision emission.  Replaces the per-trip
   host replay of Banner.BanOrChallengeIp -> DynamicDecisionLists.Update
   (internal/iptables.go:273-294, internal/decision.go:404-439) and
   Banner.LogRegexBan (internal/iptables.go:179-228) that consumeLine runs for
   every trip (internal/regex_rate_limiter.go:254-266).
   Options hold for every later batch run with BJX_EMIT_BANS. */
/* One UTC-offset change of the local time zone LogRegexBan formats its
   timestring in (logTime.Format in time.Local, internal/iptables.go:187). */
typedef struct bjx_tz_transition {
  int64_t utc_start_s; /* first Unix second the offset applies to */
  int32_t offset_s;    /* seconds east of UTC from then on */
  int32_t _pad;
} bjx_tz_transition;

typedef struct bjx_ban_options {
  int64_t expiring_ttl_ns;          /* expiring_decision_ttl_seconds * 1e9 (config.go) */
  int32_t tz_offset_s;              /* UTC offset (seconds east) before the first transition, or always when there are none */
  uint32_t _pad;
  const bjx_str *disable_logging;   /* config.DisableLogging hosts set to true (LoggerTemp lines) */
  size_t n_disable_logging;
  const bjx_tz_transition *tz_transitions; /* the zone's offset changes, ascending by utc_start_s (DST rules
                                              expanded; a Go host walks time.Local with Time.ZoneBounds) */
  size_t n_tz_transitions;
} bjx_ban_options;
int bjx_engine_set_ban_options(bjx_engine *e, const bjx_ban_options *opts);

/* One per distinct IP that tripped in the batch.  Applying
   Update(ip, expires_ns, decision, fromBaskerville=false, domain) once per
   record, with ip / domain (host) taken from trips[trip_idx], leaves the
   decision lists exactly as the per-trip replay does: the entry changes only
   when decision beats the one held, and the first trip with the IP's highest
   decision is the last strict escalation.  iptables: some trip decided
   IptablesBlock (banIp, which the reference calls per such trip). */
typedef struct bjx_ip_decision {
  uint64_t trip_idx;
  uint64_t n_trips;     /* trips of this IP in the batch */
  int64_t expires_ns;   /* now_ns + expiring_ttl_ns (Go wrapping add) */
  int32_t decision;     /* highest decision over the IP's trips */
  uint32_t iptables;
} bjx_ip_decision;

typedef struct bjx_ban_batch {
  uint64_t n_ips;
  const bjx_ip_decision *ips;   /* host, ordered by trip_idx */
  uint64_t n_trips;
  const char *log;              /* host: LogRegexBan lines in trip order, each ending in '\n' */
  uint64_t log_bytes;
  const uint64_t *log_off;      /* host, n_trips + 1: trip t's line is log[log_off[t], log_off[t+1]) (empty: < 6 words) */
  const uint8_t *log_kind;      /* host, n_trips: 0 no line, 1 Logger, 2 LoggerTemp (disable_logging host) */
  const uint8_t *ip_bytes;      /* host: record r's IP (the Update key) is ip_bytes[ip_off[r], ip_off[r+1]) */
  const uint64_t *ip_off;       /* host, n_ips + 1 */
} bjx_ban_batch;
/* The last batch's emission (valid until the next batch; needs BJX_EMIT_BANS). */
int bjx_batch_bans(bjx_engine *e, bjx_ban_batch *out);

/* ---- Node: the GPUs of one host behind one handle.  The Go
   host keeps ONE RegexRateLimitStates (rate_limit.go:19-28, created once in
   banjax.go:80) fed by ONE consumer goroutine (regex_rate_limiter.go:54-77);
   a node keeps that shape over n_devices engines.  Engine k matches the k-th
   contiguous chunk of the batch, the rate-limit state is sharded by IP (owner
   (ip_hash >> 32) % n_devices), and the library moves the event records to
   their owners and the outcome bytes back itself (an RCCL all-to-all of
   ncclSend / ncclRecv pairs over xGMI when every engine has a GPU of its own,
   device-to-device copies when engines share a GPU; no caller collective).
   Results come back in the reference's global order, exactly as one engine
   over the whole batch returns them.  Env: BJX_NODE_EXCHANGE=peer|rccl forces
   the copies / RCCL (rccl: creation fails when it cannot be had). */
typedef struct bjx_node bjx_node;
/* devices: HIP device index of each engine (repeats allowed: engines sharing a GPU). */
int bjx_node_create(const int *devices, size_t n_devices, const bjx_engine_options *opts, bjx_node **out, char *err,
                    size_t err_len);
void bjx_node_destroy(bjx_node *n);
size_t bjx_node_size(const bjx_node *n);
/* Engine k of the node (its own stats and debug hooks); owned by the node. */
bjx_engine *bjx_node_engine(bjx_node *n, size_t k);
/* How the node moves its records: 1 RCCL, 0 device copies, -1 no node. */
int bjx_node_exchange_kind(const bjx_node *n);
const char *bjx_node_last_error(bjx_node *n);
/* bjx_engine_set_decision_lists / bjx_engine_set_ban_options on every engine. */
int bjx_node_set_decision_lists(bjx_node *n, const bjx_decision_entry *entries, size_t count);
int bjx_node_set_ban_options(bjx_node *n, const bjx_ban_options *opts);
/* consumeLine over the complete lines of a host buffer: split at '\n' into
   n_devices chunks of about equal size.  line_offset / line_idx in the result
   are relative to bytes, as bjx_process_batch's. */
int bjx_node_process_batch(bjx_node *n, const bjx_ruleset *rs, const uint8_t *bytes, size_t len, int64_t now_ns,
                           uint32_t flags, bjx_batch_result *out);
/* Same over chunks already resident in HBM: chunks[k] is a device pointer on
   engine k's GPU (flags must include BJX_INPUT_DEVICE) and every chunk but the
   last ends in '\n'.  Offsets are relative to the chunks' concatenation. */
int bjx_node_process_chunks(bjx_node *n, const bjx_ruleset *rs, const uint8_t *const *chunks, const size_t *lens,
                            int64_t now_ns, uint32_t flags, bjx_batch_result *out);
/* The last node batch's decision emission (BJX_EMIT_BANS), merged over the
   engines: one record per IP (highest decision, its first trip), trip_idx
   into the node batch's trips; log lines in node trip order. */
int bjx_node_batch_bans(bjx_node *n, bjx_ban_batch *out);
/* RegexRateLimitStates.Get / Len / String / occupancy over every shard. */
int bjx_node_state_get(bjx_node *n, const char *ip, size_t ip_len, const char *name, size_t name_len, int64_t *num_hits,
                       int64_t *interval_start_ns);
int64_t bjx_node_state_len(bjx_node *n);
size_t bjx_node_state_dump(bjx_node *n, char *out, size_t cap);
int bjx_node_state_stats_get(bjx_node *n, bjx_state_stats *out);
int bjx_node_state_clear(bjx_node *n);

int bjx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BANJAX_GPU_H */
