// Trip -> decision emission on the device.
//
// The reference runs, for every rate-limit trip and in trip order, on the
// tailer goroutine (internal/regex_rate_limiter.go:254-266):
//   Banner.BanOrChallengeIp (internal/iptables.go:273-294)
//     -> DynamicDecisionLists.Update (internal/decision.go:404-439): the entry
//        of the IP is replaced only by a strictly more serious decision, with
//        expires = time.Now() + expiring_decision_ttl_seconds and the trip's host
//        as domain; banIp for IptablesBlock;
//   Banner.LogRegexBan (internal/iptables.go:179-228): one json.Marshal'ed
//     LogJson line when the line's rest has at least 6 space-separated words.
//
// Per batch (one injected clock), a run of Updates for one IP leaves the entry
// that the first trip with the IP's highest decision wrote, whenever that
// decision beats the entry held before the batch (each later strict increase
// overwrites the earlier ones; equal decisions never update).  So the device
// emits one record per distinct IP: {first trip with the max decision, max
// decision, expires, any IptablesBlock trip}, and the host applies it with one
// Update per IP.  The ban-log lines are formatted here byte for byte as Go's
// encoding/json writes them (HTML escaping on, \b \f forms, invalid UTF-8 ->
// �, U+2028/2029 escaped).
#pragma once
#include <stdint.h>

#include "bjx_common.h"

namespace bjx {

struct BanDev {
  const uint8_t *buf;        // batch bytes (device)
  const bjx_trip *trips;     // n_trips, reference order
  uint64_t n_trips;
  const DevRule *rules;
  const uint32_t *name_off;  // per rule-name id: escaped JSON string (with quotes) in name_json
  const uint8_t *name_json;
  const uint64_t *dl_hash;   // disable_logging hosts: sorted hash_bytes
  const uint32_t *dl_off, *dl_len;
  const uint8_t *dl_bytes;
  uint32_t n_dl;
  int32_t tz_offset_s;       // offset before the first transition (fixed zone when n_tz == 0)
  const int64_t *tz_at;      // local zone: UTC second of each offset change, ascending
  const int32_t *tz_off;     // offset from tz_at[i] on
  uint32_t n_tz;
};

template <bool W>
struct JOut {
  uint8_t *p;
  uint64_t n;
  BJX_HD void put(uint8_t c) {
    if (W) p[n] = c;
    ++n;
  }
  BJX_HD void puts(const char *s) {
    while (*s) put((uint8_t)*s++);
  }
  BJX_HD void raw(const uint8_t *s, uint32_t len) {
    for (uint32_t i = 0; i < len; ++i) put(s[i]);
  }
};

__device__ __forceinline__ bool go_is_space(int32_t r) {
  return r == 0x09 || r == 0x0A || r == 0x0B || r == 0x0C || r == 0x0D || r == 0x20 || r == 0x85 || r == 0xA0 ||
         r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 || r == 0x202F || r == 0x205F ||
         r == 0x3000;
}

// strings.TrimSpace on [b, e): unicode.IsSpace runes off both ends
// (DecodeRune forwards, DecodeLastRune backwards; invalid bytes stop it)
__device__ __forceinline__ void go_trim_space(const uint8_t *s, uint32_t &b, uint32_t &e) {
  while (b < e) {
    int w;
    const int32_t r = decode_rune_hd(s + b, e - b, &w);
    if (!go_is_space(r)) break;
    b += (uint32_t)w;
  }
  while (e > b) {
    uint32_t st = e - 1, lim = 0;
    while (st > b && (s[st] & 0xC0) == 0x80 && lim < 3) { --st; ++lim; }
    int w;
    int32_t r = decode_rune_hd(s + st, e - st, &w);
    if ((uint32_t)w != e - st) { r = 0xFFFD; st = e - 1; }
    if (!go_is_space(r)) break;
    e = st;
  }
}

// encoding/json string encoding (encode.go appendString, escapeHTML = true)
template <bool W>
BJX_HDN void json_str(JOut<W> &o, const uint8_t *s, uint32_t n) {
  const char *hex = "0123456789abcdef";
  o.put('"');
  uint32_t i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') o.put(c);
      else if (c == '\\' || c == '"') { o.put('\\'); o.put(c); }
      else if (c == 0x08) { o.put('\\'); o.put('b'); }
      else if (c == 0x0C) { o.put('\\'); o.put('f'); }
      else if (c == 0x0A) { o.put('\\'); o.put('n'); }
      else if (c == 0x0D) { o.put('\\'); o.put('r'); }
      else if (c == 0x09) { o.put('\\'); o.put('t'); }
      else { o.puts("\\u00"); o.put((uint8_t)hex[c >> 4]); o.put((uint8_t)hex[c & 15]); }
      ++i;
      continue;
    }
    int w;
    const int32_t r = decode_rune_hd(s + i, n - i, &w);
    if (r == 0xFFFD && w == 1) o.puts("\\ufffd");
    else if (r == 0x2028) o.puts("\\u2028");
    else if (r == 0x2029) o.puts("\\u2029");
    else o.raw(s + i, (uint32_t)w);
    i += (uint32_t)w;
  }
  o.put('"');
}

template <bool W>
BJX_HD void put_dec(JOut<W> &o, int64_t v, int width) {
  char d[24];
  int k = 0;
  uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
  do { d[k++] = (char)('0' + u % 10); u /= 10; } while (u);
  if (v < 0) o.put('-');
  for (int i = k; i < width; ++i) o.put('0');
  while (k) o.put((uint8_t)d[--k]);
}

// offset of the local zone at Unix second sec (time.Location.lookup: the last
// transition at or before sec)
__device__ __forceinline__ int32_t zone_offset(const BanDev &A, int64_t sec) {
  if (A.n_tz == 0 || sec < A.tz_at[0]) return A.tz_offset_s;
  uint32_t lo = 0, hi = A.n_tz;  // tz_at[lo] <= sec < tz_at[hi]
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (A.tz_at[m] <= sec) lo = m; else hi = m;
  }
  return A.tz_off[lo];
}

// time.Unix(0, ns).In(time.Local).Format("2006-01-02T15:04:05")
template <bool W>
__device__ void put_time(JOut<W> &o, int64_t ns, const BanDev &A) {
  int64_t sec = ns / 1000000000LL;
  if (ns % 1000000000LL < 0) --sec;
  sec += zone_offset(A, sec);
  int64_t days = sec / 86400, sod = sec % 86400;
  if (sod < 0) { sod += 86400; --days; }
  // civil date from days since 1970-01-01 (proleptic Gregorian)
  const int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t d = doy - (153 * mp + 2) / 5 + 1;
  const int64_t m = mp < 10 ? mp + 3 : mp - 9;
  const int64_t y = yoe + era * 400 + (m <= 2 ? 1 : 0);
  put_dec(o, y, 4); o.put('-'); put_dec(o, m, 2); o.put('-'); put_dec(o, d, 2); o.put('T');
  put_dec(o, sod / 3600, 2); o.put(':'); put_dec(o, sod / 60 % 60, 2); o.put(':'); put_dec(o, sod % 60, 2);
}

__device__ __forceinline__ bool dl_contains(const BanDev &A, const uint8_t *h, uint32_t n) {
  if (A.n_dl == 0) return false;
  const uint64_t hh = hash_bytes(h, n);
  uint32_t lo = 0, hi = A.n_dl;
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (A.dl_hash[m] < hh) lo = m + 1; else hi = m;
  }
  for (uint32_t i = lo; i < A.n_dl && A.dl_hash[i] == hh; ++i) {
    if (A.dl_len[i] != n) continue;
    bool eq = true;
    for (uint32_t k = 0; k < n && eq; ++k) eq = A.dl_bytes[A.dl_off[i] + k] == h[k];
    if (eq) return true;
  }
  return false;
}

__device__ __forceinline__ const char *decision_name(int32_t d) {
  // Decision.String (decision.go:45-58)
  return d == 1 ? "Allow" : d == 2 ? "Challenge" : d == 3 ? "NginxBlock" : d == 4 ? "IptablesBlock" : "";
}

// LogRegexBan for trip t: the JSON line plus '\n' (Logger.Println), or nothing
// when the rest has fewer than 6 words.  Returns 1 + disable_logging when a
// line is written, 0 otherwise.
template <bool W>
__device__ uint32_t ban_log_line(const BanDev &A, uint64_t t, JOut<W> &o) {
  const bjx_trip &T = A.trips[t];
  const uint8_t *line = A.buf + T.line_offset;
  const uint8_t *rest = line + T.rest_off;
  const uint32_t rn = T.line_len - T.rest_off;
  // strings.SplitN(logLine, " ", 6)
  uint32_t sp[5], ns = 0;
  for (uint32_t i = 0; i < rn && ns < 5; ++i)
    if (rest[i] == ' ') sp[ns++] = i;
  if (ns < 5) return 0;
  const uint32_t host_b = sp[0] + 1, host_e = sp[1];
  const uint32_t disable = dl_contains(A, rest + host_b, host_e - host_b) ? 1u : 0u;
  // strings.SplitN(words[5], "|", 2)[0], then TrimSpace
  uint32_t ub = sp[4] + 1, ue = ub;
  while (ue < rn && rest[ue] != '|') ++ue;
  go_trim_space(rest, ub, ue);
  const DevRule &R = A.rules[T.rule_idx];
  o.puts("{\"path\":");
  json_str(o, rest + sp[2] + 1, sp[3] - sp[2] - 1);
  o.puts(",\"timestring\":\"");
  put_time(o, T.ts_ns, A);
  o.puts("\",\"trigger\":");
  o.raw(A.name_json + A.name_off[R.name_id], A.name_off[R.name_id + 1] - A.name_off[R.name_id]);
  o.puts(",\"client_ua\":");
  json_str(o, rest + ub, ue - ub);
  o.puts(",\"client_ip\":");
  json_str(o, line + T.ip_off, T.ip_len);
  o.puts(",\"rule_type\":\"regex\",\"client_request_method\":");
  json_str(o, rest, sp[0]);
  o.puts(",\"http_request_scheme\":\"https\",\"client_request_host\":");
  json_str(o, rest + host_b, host_e - host_b);
  o.puts(",\"action\":\"");
  o.puts(decision_name(T.decision));
  o.puts("\",\"number_of_fails\":1,\"disable_logging\":");
  o.put(disable ? '1' : '0');
  o.puts("}\n");
  return 1 + disable;
}

}  // namespace bjx
