// MI355X engine for banjax's regex rate-limiting log tailer.
//
// One bjx_process_batch = the reference's consumeLine applied to every line of
// a '\n'-framed chunk (internal/regex_rate_limiter.go:113-269), with the
// per-(ip, rule-name) fixed-window counters of RegexRateLimitStates.Apply
// (internal/rate_limit.go:37-78) kept resident in HBM across batches.
//
// Pipeline of one batch:
//   k_nl_count_wt + scan       '\n' count per 4 KB wave tile -> each tile's first line
//   k_scan                     line framing (nl[]) and the prefilter literal hits of
//                              every line, from the tile staged in LDS
//   k_lines2 (k_lines)         per line: SplitN header, ParseFloat fast path, host
//                              lookup, CheckIsAllowed, OldLine, rule decisions from
//                              the literal hits; undecided (line, rule) pairs -> jobs
//   job sort + k_dfa / k_nfa   the automaton of every undecided pair
//   k_parse_match<SLOW>        lines whose timestamp needs the general ParseFloat
//   k_emit                     RuleResults and rate-limit events in reference order
//   k_ip_claim / k_st_claim    IP and (ip, rule name) state slots in HBM hash tables
//   radix sort + k_apply       events by state slot (stable), the Apply automaton
//   k_select_trips / k_build_trips   RateLimitResult.Exceeded -> the host's Banner replay
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <tuple>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include "../../include/banjax_gpu.h"
#include "bjx_common.h"
#include "engine_types.h"
#include "regex_compiler.h"
#include "bans.h"

using namespace bjx;

namespace {

struct BjxError : std::runtime_error {
  int code;
  BjxError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

#define HIP_OK(expr)                                                                                   \
  do {                                                                                                 \
    hipError_t e_ = (expr);                                                                            \
    if (e_ != hipSuccess)                                                                              \
      throw BjxError(BJX_ERR_DEVICE, std::string(#expr " failed: ") + hipGetErrorString(e_));          \
  } while (0)

constexpr int kBlock = 256;

// =====================================================================
//                              device code
// =====================================================================

// --------------------------------------------------------------- framing

__device__ __forceinline__ uint32_t nl_mask_word(uint32_t v) {
  // exact per-byte '\n' detector: returns 0x80 in each byte equal to 0x0A
  uint32_t x = v ^ 0x0A0A0A0Au;
  uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return ~t & 0x80808080u;
}

// --------------------------------------------------------------- lookups

__device__ __forceinline__ uint32_t find_space(const uint8_t *p, uint32_t i, uint32_t n) {
  while (i < n && p[i] != ' ') ++i;
  return i;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
  uint32_t k = 0;
  for (; k + 4 <= n; k += 4)
    if (ld4(a + k) != ld4(b + k)) return false;
  for (; k < n; ++k)
    if (a[k] != b[k]) return false;
  return true;
}

// Inline IP key (IpSlot.key16): bytes 0..14 zero padded, byte 15 = min(len, 255).
// Equal keys <=> equal IPs when len <= 15 (every IPv4 text); longer IPs
// compare their bytes in the arena.  Word loads; the caller keeps 3 bytes of
// readable slack past ip + 15 (a log line always continues past its IP).
__device__ __forceinline__ uint4 ip_key16(const uint8_t *ip, uint32_t len) {
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t lo = 4u * k;
    const uint32_t m = len <= lo ? 0u : (len >= lo + 4 ? 0xFFFFFFFFu : (1u << (8 * (len - lo))) - 1u);
    w[k] = m ? ld4(ip + lo) & m : 0u;
  }
  w[3] = (w[3] & 0x00FFFFFFu) | ((len < 255 ? len : 255u) << 24);
  return make_uint4(w[0], w[1], w[2], w[3]);
}
// the same key from bytes that may end at ip + len (exchanged IP pools)
__device__ __forceinline__ uint4 ip_key16_bytes(const uint8_t *ip, uint32_t len) {
  uint32_t w[4] = {0, 0, 0, 0};
  for (uint32_t k = 0; k < len && k < 15; ++k) w[k >> 2] |= (uint32_t)ip[k] << (8 * (k & 3));
  w[3] |= (len < 255 ? len : 255u) << 24;
  return make_uint4(w[0], w[1], w[2], w[3]);
}
constexpr uint32_t kIpWords = 12;  // IPs of < 48 bytes (IPv4 and IPv6 text) are handled as words in registers

// bytes [p, p + n), n <= 4 * NW, as NW zero-padded little-endian words,
// every load issued at once; loads only the aligned words holding at least
// one of the bytes (an exchanged IP pool may end at p + n)
template <uint32_t NW>
__device__ __forceinline__ void ip_words(const uint8_t *p, uint32_t n, uint32_t (&w)[NW]) {
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
  const uint32_t nw = n ? (sh + n + 3) >> 2 : 0u;
  uint32_t r[NW + 1];
#pragma unroll
  for (uint32_t k = 0; k <= NW; ++k) r[k] = k < nw ? a[k] : 0u;
#pragma unroll
  for (uint32_t k = 0; k < NW; ++k) {
    const uint32_t lo = 4u * k;
    const uint32_t m = n <= lo ? 0u : (n >= lo + 4 ? 0xFFFFFFFFu : (1u << (8 * (n - lo))) - 1u);
    w[k] = __builtin_amdgcn_alignbyte(r[k + 1], r[k], sh) & m;
  }
}
// hash_bytes of n < 4 * NW bytes given as ip_words
template <uint32_t NW>
__device__ __forceinline__ uint64_t hash_words(const uint32_t (&w)[NW], uint32_t n) {
  uint32_t a = 0x9E3779B9u ^ n, b = 0x7F4A7C15u + n * 0x85EBCA6Bu;
  const uint32_t full = n >> 2;
  uint32_t t = 0;
#pragma unroll
  for (uint32_t k = 0; k < NW; ++k) {
    if (k < full) {
      a = rotl32(a ^ w[k], 7) * 0x27D4EB2Du;
      b = rotl32(b + w[k], 13) * 0x165667B1u;
    } else if (k == full) {
      t = w[k];
    }
  }
  return hash_finish(a, b, t);
}
// hash_bytes of an IP of n <= 15 bytes from its inline key (ip_key16: the
// bytes zero padded, the length in byte 15)
__device__ __forceinline__ uint64_t key16_hash(const uint4 &k, uint32_t n) {
  const uint32_t w[4] = {k.x, k.y, k.z, k.w & 0x00FFFFFFu};
  return hash_words<4>(w, n);
}
// an IP's inline key and (past 15 bytes) its hash from word loads issued
// together (p + n + 3 readable): no dependent byte loop
__device__ __forceinline__ void ip_key_hash(const uint8_t *p, uint32_t n, uint4 &k16, uint64_t &h) {
  if (n <= 15) {  // the key alone: the hash of so short an IP comes from it where it is needed (key16_hash)
    uint32_t w[4];
    ip_words(p, n, w);
    k16 = make_uint4(w[0], w[1], w[2], w[3] | (n << 24));
    h = 0;
  } else if (n < 4 * kIpWords) {
    uint32_t w[kIpWords];
    ip_words(p, n, w);
    h = hash_words(w, n);
    const uint32_t m3 = n >= 15 ? 0x00FFFFFFu : n <= 12 ? 0u : (1u << (8 * (n - 12))) - 1u;
    k16 = make_uint4(w[0], w[1], w[2], (w[3] & m3) | ((n < 255 ? n : 255u) << 24));
  } else {
    h = hash_bytes(p, n);
    k16 = ip_key16(p, n);
  }
}
__device__ __forceinline__ bool key16_eq(const uint4 &a, const uint4 &b) {
  return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
}
// equal byte strings of length n: below 4 * kIpWords bytes by word loads all
// issued at once (bytes_eq's loop waits for each word pair in turn)
__device__ __forceinline__ bool ip_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
  if (n >= 4 * kIpWords) return bytes_eq(a, b, n);
  uint32_t wa[kIpWords], wb[kIpWords];
  ip_words(a, n, wa);
  ip_words(b, n, wb);
  bool eq = true;
#pragma unroll
  for (uint32_t k = 0; k < kIpWords; ++k) eq = eq && wa[k] == wb[k];
  return eq;
}

// host string -> host id (per_site_regexes_with_rates key / skip host / allow-list site)
__device__ int32_t host_lookup(const Bind &B, const uint8_t *h, uint32_t n) {
  if (B.n_hd == 0) return -1;
  const uint64_t hh = hash_bytes(h, n);
  uint32_t lo = 0, hi = B.n_hd;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (B.hd_hash[m] < hh) lo = m + 1; else hi = m;
  }
  for (; lo < B.n_hd && B.hd_hash[lo] == hh; ++lo)
    if (B.hd_len[lo] == n && bytes_eq(B.hd_bytes + B.hd_off[lo], h, n)) return (int32_t)B.hd_id[lo];
  return -1;
}

__device__ __forceinline__ uint64_t be64(const uint8_t *a) {
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) v = (v << 8) | a[k];
  return v;
}

// IPFilter.Allowed restricted to one scope (decision.go:185-216 with
// github.com/jeremy5189/ipfilter-no-iploc/v2: exact canonical IPs, then subnets).
__device__ __forceinline__ bool scope_allows_addr(const Bind &B, int sc, const uint8_t a[16]) {
  const uint64_t hi = be64(a), lo = be64(a + 8);
  uint32_t b = B.sc_addr_off[sc], e = B.sc_addr_off[sc + 1];
  while (b < e) {
    uint32_t m = (b + e) >> 1;
    uint64_t mh = B.sc_addr[2 * m], ml = B.sc_addr[2 * m + 1];
    if (mh < hi || (mh == hi && ml < lo)) b = m + 1; else e = m;
  }
  if (b < B.sc_addr_off[sc + 1] && B.sc_addr[2 * b] == hi && B.sc_addr[2 * b + 1] == lo) return true;
  const bool v4 = is_v4_mapped(a);
  for (uint32_t k = B.sc_sub_off[sc]; k < B.sc_sub_off[sc + 1]; ++k) {
    const Subnet &s = B.sc_sub[k];
    const uint8_t *ip = v4 ? a + 12 : a;
    const uint32_t l = v4 ? 4 : 16;
    if (l != s.netlen) continue;
    bool ok = true;
    for (uint32_t i = 0; i < l; ++i)
      if ((s.net[i] & s.mask[i]) != (ip[i] & s.mask[i])) { ok = false; break; }
    if (ok) return true;
  }
  return false;
}
// exact-map Allow entries that net.ParseIP refuses (compared byte for byte)
__device__ __forceinline__ bool scope_allows_str(const Bind &B, int sc, uint64_t h, const uint8_t *s, uint32_t n) {
  uint32_t b = B.sc_str_off[sc], e = B.sc_str_off[sc + 1];
  while (b < e) {
    uint32_t m = (b + e) >> 1;
    if (B.sc_str_hash[m] < h) b = m + 1; else e = m;
  }
  for (; b < B.sc_str_off[sc + 1] && B.sc_str_hash[b] == h; ++b)
    if (B.sc_str_len[b] == n && bytes_eq(B.sc_str_bytes + B.sc_str_boff[b], s, n)) return true;
  return false;
}
// StaticDecisionLists.CheckIsAllowed(site, clientIp)
__device__ __forceinline__ bool check_is_allowed(const Bind &B, int32_t host_id, const uint8_t *ip, uint32_t n) {
  const int32_t site_sc = host_id >= 0 ? B.host_scope[host_id] : -1;
  uint8_t a[16];
  bool is4;
  const bool ok = go_parse_addr(ip, n, a, &is4);
  uint64_t h = 0;
  for (int pass = 0; pass < 2; ++pass) {
    const int sc = pass == 0 ? site_sc : 0;
    if (sc < 0) continue;
    if (ok) {
      if (scope_allows_addr(B, sc, a)) return true;
    } else {
      if (!h) h = hash_bytes(ip, n);
      if (scope_allows_str(B, sc, h, ip, n)) return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool is_skip(const Bind &B, uint32_t rule, int32_t host_id) {
  if (host_id < 0 || B.n_skip == 0) return false;
  const uint64_t k = ((uint64_t)rule << 32) | (uint32_t)host_id;
  uint32_t lo = 0, hi = B.n_skip;
  while (lo < hi) {
    uint32_t m = (lo + hi) >> 1;
    if (B.skip_keys[m] < k) lo = m + 1; else hi = m;
  }
  return lo < B.n_skip && B.skip_keys[lo] == k;
}

// --------------------------------------------------------------- regex

// ---- bit-parallel NFA (rules past the DFA state cap; regex_compiler.cpp
// "bit-parallel NFA" gives the algorithm and the table layout).  State sets
// are WT 64-bit words in VGPRs; EXACT: the rule's W equals WT (k_nfa), else W
// <= WT is read from the header (per-line slow path).

template <int WT>
__device__ __forceinline__ bool nfa_bit(const uint64_t (&v)[WT], uint32_t p) {
  uint64_t w = 0;
#pragma unroll
  for (int k = 0; k < WT; ++k) w = (p >> 6) == (uint32_t)k ? v[k] : w;  // selects: no scratch
  return ((w >> (p & 63)) & 1) != 0;
}

// X = D with the assertion closures of context k (ctx * 4 + next category)
template <int WT, bool EXACT>
__device__ __forceinline__ void nfa_cross(const uint64_t *__restrict__ b, const NfaLayout &L, const uint64_t (&D)[WT],
                                          uint64_t (&X)[WT], uint32_t k) {
  const uint32_t W = EXACT ? (uint32_t)WT : L.W;
#pragma unroll
  for (int w = 0; w < WT; ++w) X[w] = D[w];
  if (!(L.flags & kNfaAsserts)) return;
  const uint32_t *apos = reinterpret_cast<const uint32_t *>(b + L.o_apos);
  for (uint32_t a = 0; a < L.nassert; ++a) {
    if (!nfa_bit(D, apos[a])) continue;
    const uint64_t *T = b + L.o_at + (a * 16 + k) * W;
#pragma unroll
    for (int w = 0; w < WT; ++w)
      if (EXACT || (uint32_t)w < W) X[w] |= T[w];
  }
}

// one rune of class c; true = matched (before or after it)
template <int WT, bool EXACT>
__device__ __forceinline__ bool nfa_rune(const uint64_t *__restrict__ b, const NfaLayout &L, uint64_t (&D)[WT], uint32_t c,
                                         uint32_t &ctx) {
  const uint32_t W = EXACT ? (uint32_t)WT : L.W;
  uint64_t X[WT], Y[WT];
  const uint32_t cat = (L.flags & kNfaAsserts) ? reinterpret_cast<const uint8_t *>(b + L.o_cat)[c] : 0u;
  nfa_cross<WT, EXACT>(b, L, D, X, ctx * 4 + cat);
  ctx = cat == 1 ? 1u : (cat == 2 ? 2u : 0u);
  if (L.match != 0xFFFFFFFFu && nfa_bit(X, L.match)) return true;
  const uint64_t *cm = b + L.o_cm + c * W, *sh = b + L.o_sh, *s0 = b + L.o_s0;
#pragma unroll
  for (int w = 0; w < WT; ++w) Y[w] = (EXACT || (uint32_t)w < W) ? X[w] & cm[w] : 0ull;
  uint64_t carry = 0;
#pragma unroll
  for (int w = 0; w < WT; ++w) {
    if (!EXACT && (uint32_t)w >= W) { D[w] = 0; continue; }
    const uint64_t m = Y[w] & sh[w];
    D[w] = (m << 1) | carry | s0[w];
    carry = m >> 63;
  }
  for (uint32_t g = 0; g < L.ngroups; ++g) {
    const uint64_t *gm = b + L.o_gm + g * W, *gt = b + L.o_gt + g * W;
    uint64_t any = 0;
#pragma unroll
    for (int w = 0; w < WT; ++w)
      if (EXACT || (uint32_t)w < W) any |= Y[w] & gm[w];
    if (any) {
#pragma unroll
      for (int w = 0; w < WT; ++w)
        if (EXACT || (uint32_t)w < W) D[w] |= gt[w];
    }
  }
  return L.match != 0xFFFFFFFFu && nfa_bit(D, L.match);
}

template <int WT, bool EXACT>
__device__ __forceinline__ bool nfa_at_s0(const uint64_t *__restrict__ b, const NfaLayout &L, const uint64_t (&D)[WT]) {
  const uint32_t W = EXACT ? (uint32_t)WT : L.W;
  uint64_t d = 0;
#pragma unroll
  for (int w = 0; w < WT; ++w)
    if (EXACT || (uint32_t)w < W) d |= D[w] ^ b[L.o_s0 + w];
  return d == 0;
}

template <int WT, bool EXACT>
__device__ __forceinline__ bool nfa_end(const uint64_t *__restrict__ b, const NfaLayout &L, const uint64_t (&D)[WT], uint32_t ctx) {
  uint64_t X[WT];
  nfa_cross<WT, EXACT>(b, L, D, X, ctx * 4 + 3);
  return L.match != 0xFFFFFFFFu && nfa_bit(X, L.match);
}

__device__ __forceinline__ uint32_t nonascii_class(const Bind &B, const DevRule &R, int32_t rune) {
  const uint32_t *na = B.nonascii + 2 * R.na_off;
  uint32_t lo = 0, hi = R.n_na;  // last interval with start <= rune
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (na[2 * m] <= (uint32_t)rune) lo = m; else hi = m;
  }
  return na[2 * lo + 1];
}

// (*Regexp).Match of a kRuleNfa rule over [t, t + n), tables at b (any
// address space; the per-line slow path reads them from HBM)
__device__ __noinline__ bool nfa_match_generic(const Bind &B, const DevRule &R, const uint8_t *t, uint32_t n) {
  const uint64_t *b = B.nfa + R.nfa_off;
  const NfaLayout L = nfa_layout_of(reinterpret_cast<const uint32_t *>(b));
  const uint16_t *a16 = reinterpret_cast<const uint16_t *>(b + L.o_ascii);
  uint64_t D[16];
#pragma unroll
  for (int w = 0; w < 16; ++w) D[w] = (uint32_t)w < L.W ? b[L.o_s0 + w] : 0ull;
  uint32_t ctx = 3;
  for (uint32_t i = 0; i < n;) {
    uint32_t c;
    if (t[i] < 0x80) { c = a16[t[i]]; ++i; }
    else {
      int w;
      const int32_t rune = decode_rune_hd(t + i, n - i, &w);
      c = nonascii_class(B, R, rune);
      i += (uint32_t)w;
    }
    if (nfa_rune<16, false>(b, L, D, c, ctx)) return true;
    if ((L.flags & kNfaAnchored) && nfa_at_s0<16, false>(b, L, D)) return false;
  }
  return nfa_end<16, false>(b, L, D, ctx);
}

// (*Regexp).Match over rest, via the rule's rune-class DFA (or bit-parallel NFA).
__device__ bool rule_match(const Bind &B, uint32_t r, const uint8_t *t, uint32_t n) {
  const DevRule R = B.rules[r];
  if (R.flags & kRuleAlways) return true;
  if (R.flags & kRuleNever) return false;
  if (R.flags & kRuleNfaWide) return false;  // never asked: the per-line fallback lists wide rules for k_nfa_wide
  if (R.flags & kRuleNfa) return nfa_match_generic(B, R, t, n);
  const uint16_t *tr = B.trans + R.trans_off;
  const uint8_t *ac = B.ascii_cls + (size_t)r * 128;
  const uint32_t ncls = R.ncls;
  uint32_t st = R.start;
  uint32_t i = 0;
  while (i < n) {
    const uint8_t b = t[i];
    uint32_t c;
    if (b < 0x80) {
      c = ac[b];
      ++i;
    } else {
      int w;
      const int32_t rune = decode_rune_hd(t + i, n - i, &w);
      i += (uint32_t)w;
      const uint32_t *na = B.nonascii + 2 * R.na_off;
      uint32_t lo = 0, hi = R.n_na;  // last interval with start <= rune
      while (hi - lo > 1) {
        uint32_t m = (lo + hi) >> 1;
        if (na[2 * m] <= (uint32_t)rune) lo = m; else hi = m;
      }
      c = na[2 * lo + 1];
    }
    st = tr[st * ncls + c];
    if (st <= 1) break;
  }
  return B.accept_end[R.ae_off + st] != 0;
}

// --------------------------------------------------------------- per line

// Wide-NFA jobs of the per-line fallback (k_nfa_wide runs them after it)
struct WideList {
  uint32_t *line, *rule, *pos;
  unsigned long long *count;
  uint64_t cap;
};

__device__ void decide_wide(const Bind &B, const uint8_t *line, uint64_t s, uint32_t n, uint32_t rest_off, int32_t hid, uint64_t j,
                            const Lines &L, const WideList &WL);

__device__ __forceinline__ uint32_t find_spaces(const uint8_t *p, uint32_t n, uint32_t &sp0, uint32_t &sp1,
                                                uint32_t &sp2, uint32_t &sp3);

template <bool SLOW>
__device__ void parse_and_match(const Bind &B, const uint8_t *__restrict__ p, uint64_t s, uint32_t n, uint64_t j, int64_t now_ns,
                                const Lines &L, uint32_t *slow_list, unsigned long long *slow_count, const WideList &WL) {
  uint8_t fl = 0;
  L.counts[j] = 0;
  uint32_t sp1 = 0, sp2 = 0, sp3 = 0, sp4 = 0;  // the first four spaces, 16-B loads (find_spaces)
  if (find_spaces(p, n, sp1, sp2, sp3, sp4) < 4) { L.flags[j] = kLineError; return; }
  const uint32_t ip_off = sp1 + 1, ip_len = sp2 - sp1 - 1;
  const uint32_t rest_off = sp2 + 1, host_off = sp3 + 1, host_len = sp4 - sp3 - 1;
  int32_t hid;
  bool exempt;
  double f;
  hid = host_lookup(B, p + host_off, host_len);
  exempt = B.any_allow && check_is_allowed(B, hid, p + ip_off, ip_len);
  L.ip_len[j] = ip_len;
  L.rest_off[j] = rest_off;
  L.host_id[j] = hid;
  {
    uint4 k16;
    uint64_t h;
    ip_key_hash(p + ip_off, ip_len, k16, h);
    if (ip_len > 15) L.ip_hash[j] = h;
    L.ip16[j] = k16;
  }
  if (!SLOW) {
    if (parse_float_fast(p, sp1, &f) != 0) {
      // rare: exotic timestamp token -> general ParseFloat kernel
      L.flags[j] = kLineSlowTs;
      unsigned long long k = atomicAdd(slow_count, 1ull);
      slow_list[k] = (uint32_t)j;
      return;
    }
  } else if (parse_float_fast(p, sp1, &f) != 0) {
    // the general ParseFloat only for the tokens the fast parser declines (a
    // wide-scope line has an ordinary timestamp and takes the fast one)
    Decimal dec;
    if (go_parse_float(p, sp1, &f, &dec) != 0) { L.flags[j] = kLineError; return; }
  }
  const int64_t ts = ns_from_seconds(f);
  L.ts[j] = ts;
  if (go_sub(now_ns, ts) > 10000000000LL) fl = kLineOld;
  else if (exempt) fl = kLineExempt;
  L.flags[j] = fl;
  if (fl) return;

  // per-site rules first, then global rules, in YAML order (regex_rate_limiter.go:175-211)
  const uint8_t *rest = p + rest_off;
  const uint32_t rest_len = n - rest_off;
  uint64_t word = 0;
  uint32_t pos = 0, wi = 0, nres = 0, nev = 0;
  uint32_t s_begin = 0, s_end = 0;
  if (hid >= 0) { s_begin = B.site_off[hid]; s_end = B.site_off[hid + 1]; }
  const uint32_t napp = (s_end - s_begin) + B.n_global;
  if (SLOW && napp > 128 && B.any_prefilter) {
    // a scope past the line kernels' 128 positions: the rules the line's
    // literal hits name, its anchored / no-literal / ALWAYS rules, not every
    // rule of the scope by its automaton
    decide_wide(B, p, s, n, rest_off, hid, j, L, WL);
    return;
  }
  for (uint32_t k = 0; k < napp; ++k) {
    const uint32_t r = k < s_end - s_begin ? B.site_rules[s_begin + k] : B.global_rules[k - (s_end - s_begin)];
    if (B.any_wide && (B.rules[r].flags & kRuleNfaWide)) {
      const unsigned long long q = atomicAdd(WL.count, 1ull);
      if (q < WL.cap) { WL.line[q] = (uint32_t)j; WL.rule[q] = r; WL.pos[q] = pos; }
    } else if (rule_match(B, r, rest, rest_len)) {
      word |= 1ull << (pos & 63);
      ++nres;
      nev += is_skip(B, r, hid) ? 0u : 1u;
    }
    ++pos;
    if ((pos & 63) == 0) { L.mword(j, wi++) = word; word = 0; }
  }
  if (pos & 63) L.mword(j, wi) = word;
  L.counts[j] = ((uint64_t)nres << 32) | nev;
}

// every line to the per-line fallback (slow count = n; the fallback takes
// line t as line t, no list)
__global__ void k_no_line_pass(unsigned long long *slow_count, unsigned long long n) {
  if (threadIdx.x == 0) *slow_count = n;
}

template <bool SLOW>
__global__ __launch_bounds__(kBlock) void k_parse_match(Bind B, const uint8_t *__restrict__ buf,
                                                        const uint64_t *__restrict__ nl, uint64_t n_lines,
                                                        const uint32_t *__restrict__ list, int64_t now_ns, Lines L,
                                                        uint32_t *slow_list, unsigned long long *slow_count, WideList WL) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_lines) return;
  const uint64_t j = SLOW && list ? list[t] : t;
  const uint64_t s = j ? nl[j - 1] + 1 : 0;
  const uint32_t n = (uint32_t)(nl[j] - s);
  parse_and_match<SLOW>(B, buf + s, s, n, j, now_ns, L, slow_list, slow_count, WL);
}

// =====================================================================
//   match pipeline: wave-tiled scan pass (+ long-line resolve)
// =====================================================================
//
// Every wave owns 4 KB tiles of the batch (64 lanes x 64 B, coalesced 16 B
// loads, next tile prefetched into registers) plus a 512 B halo, staged in a
// wave-private LDS region; no block barrier after the table preload, so a
// wave busy with per-line work never stalls the others.  Per tile:
//   1. '\n' bitmasks -> line positions (nl[]) and the lines that START in the
//      tile (their ends in the tile or the halo),
//   2. 4-byte gram of every position -> LDS bitset -> exact gram table (LDS)
//      -> literal verified against the LDS bytes -> per-line hit slots (LDS);
//      hits on lines that do not fit the window go to global slots,
//   3. one lane per line: header (SplitN x2, ParseFloat fast path), host
//      lookup, CheckIsAllowed, OldLine, then the applicable rules decided from
//      the per-host ALWAYS mask, the anchored / no-literal rules' DFAs and the
//      rules required by the line's verified literals (DFA only when the
//      literal is not sufficient).
// Lines that cannot be decided in the window (longer than the halo, more than
// kLineCap lines in a tile, header past the window, exotic timestamp, more
// than 128 applicable rules) go to k_resolve_long or the per-line fallback.

constexpr uint32_t kWT = 4096;        // bytes per wave tile
constexpr uint32_t kHalo = 512;
constexpr uint32_t kLineCap = 128;    // lines starting in one tile decided from LDS
constexpr uint32_t kHitSlots = 4;     // verified literal hits kept per line
constexpr int kScanWaves = 16;        // waves per block (one block per CU)
constexpr uint32_t kTileLds = kWT + kHalo + 16;
constexpr uint32_t kWaveJobs = 64;   // DFA jobs staged per wave before one global append
constexpr uint32_t kCandList = 128;   // candidate positions verified per round (one per lane)
constexpr uint32_t kBanChunks = 8;                  // ban-log write/copy chunks of a batch (emit_bans)
constexpr uint64_t kBanChunkMin = 64ull << 20;     // logs up to this size go in one chunk
constexpr uint32_t kLongList = 64;   // long-line hits listed per round (k_scan flush_long), one per lane
constexpr uint32_t kWaveLds = kTileLds + kLineCap * (2 + 2) + kCandList * 4 + kLineCap * 4 + kLongList * 8 + 16;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kScanLdsMax = 160 * 1024;  // gfx950 LDS per CU (one scan block per CU)
constexpr uint32_t kLinesImgMax = 16 * 1024;  // k_lines copies the lookup image to LDS up to this size
constexpr uint32_t kLinesHostLdsMax = 6 * 1024;  // k_lines copies the compact host dictionary up to this size
constexpr uint32_t kLinesTabLdsMax = 10 * 1024;  // ... and the plan classes after it, up to this size in all
constexpr uint32_t kLinesBlocksPerCu = 3;       // k_lines' LDS budget: 3 blocks of 4 waves per CU
constexpr uint32_t kSpanBytes = 12 * 1024;    // k_lines: bytes of 64 lines staged per wave

// 16-bit mask of the spaces among 16 bytes
__device__ __forceinline__ uint32_t space_mask16(const uint4 v) {
  const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
  uint32_t m16 = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = wv[k] ^ 0x20202020u;
    const uint32_t hb = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    m16 |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * k);
  }
  return m16;
}

// 4 ASCII digits (first char lowest byte): exact test, and their value
__device__ __forceinline__ bool digits4(uint32_t x) {
  return (x & 0xF0F0F0F0u) == 0x30303030u && (((x & 0x0F0F0F0Fu) + 0x06060606u) & 0xF0F0F0F0u) == 0u;
}
__device__ __forceinline__ uint32_t value4(uint32_t x) {
  x -= 0x30303030u;
  x = x * 10u + (x >> 8);  // byte 0: d0 * 10 + d1, byte 2: d2 * 10 + d3
  return (x & 0xFFu) * 100u + ((x >> 16) & 0xFFu);
}
// parseTimestamp's ParseFloat for the nginx $msec shape "dddddddddd.ddd"
// (14 bytes: 10 integer digits, 3 fraction digits), loop-free from 4 words:
// the same value parse_float_fast computes (the 13-digit mantissa is exact,
// then one correctly rounded division by 1e3).  1: another shape (the caller
// runs parse_float_fast).  Needs 2 readable bytes past the token (a header
// token is followed by the rest of the line).
__device__ __forceinline__ int parse_ts_msec(const uint8_t *p, uint32_t n, double *out) {
  if (n != 14) return 1;
  const uint32_t w0 = ld4(p), w1 = ld4(p + 4), w2 = ld4(p + 8), w3 = ld4(p + 12);
  if (!digits4(w0) || !digits4(w1) || (w2 & 0x00FF0000u) != 0x002E0000u || !digits4((w2 & 0xFF00FFFFu) | 0x00300000u) ||
      !digits4((w3 & 0xFFFFu) | 0x30300000u))
    return 1;
  const uint32_t d8 = w2 & 0xFFu, d9 = (w2 >> 8) & 0xFFu, d11 = w2 >> 24, d12 = w3 & 0xFFu, d13 = (w3 >> 8) & 0xFFu;
  const uint64_t ip = (uint64_t)value4(w0) * 1000000ull + value4(w1) * 100u + (d8 - 48u) * 10u + (d9 - 48u);
  const uint64_t m = ip * 1000ull + (d11 - 48u) * 100u + (d12 - 48u) * 10u + (d13 - 48u);
  *out = (double)m / 1000.0;
  return 0;
}

// first four spaces of the line [p, p + n): 16 B aligned loads, SWAR compare.
// A line of 64 bytes or more (past the alignment skip) has its first 64 loaded
// at once (four independent loads, one wait) and its spaces taken from one
// 64-bit mask; the chunk loop covers the rest.
__device__ __forceinline__ uint32_t find_spaces(const uint8_t *p, uint32_t n, uint32_t &sp0, uint32_t &sp1,
                                                uint32_t &sp2, uint32_t &sp3) {
  const uint32_t skip = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 15);
  const uint4 *base = reinterpret_cast<const uint4 *>(p - skip);  // keeps p's address space
  uint32_t ns = 0, c0 = 0;
  if (n + skip >= 64) {
    const uint4 v0 = base[0], v1 = base[1], v2 = base[2], v3 = base[3];
    uint64_t m = (uint64_t)space_mask16(v0) | ((uint64_t)space_mask16(v1) << 16) | ((uint64_t)space_mask16(v2) << 32) |
                 ((uint64_t)space_mask16(v3) << 48);
    m &= ~((1ull << skip) - 1ull);  // all 64 bytes lie before p + n
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t pos = (uint32_t)__ffsll((unsigned long long)m) - 1 - skip;
      const bool has = m != 0;
      m &= m - 1;
      if (k == 0) sp0 = has ? pos : sp0;
      if (k == 1) sp1 = has ? pos : sp1;
      if (k == 2) sp2 = has ? pos : sp2;
      if (k == 3) sp3 = has ? pos : sp3;
      ns += has ? 1u : 0u;
    }
    c0 = 4;
  }
  for (uint32_t c = c0; c * 16 < n + skip && ns < 4; ++c) {
    const uint4 v = base[c];
    // 16-bit mask of the spaces of this chunk inside [p, p + n)
    uint32_t m16 = 0;
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = wv[k] ^ 0x20202020u;
      const uint32_t hb = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
      m16 |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * k);
    }
    const int32_t lo = (int32_t)skip - (int32_t)(c * 16), hi = lo + (int32_t)n;  // valid chunk bytes [lo, hi)
    if (lo > 0) m16 &= ~((1u << lo) - 1u);
    if (hi < 16) m16 &= hi > 0 ? (1u << hi) - 1u : 0u;
    while (m16 && ns < 4) {  // selects, not an indexed store: no scratch
      const uint32_t pos = c * 16 + (uint32_t)__ffs(m16) - 1 - skip;
      m16 &= m16 - 1;
      sp0 = ns == 0 ? pos : sp0;
      sp1 = ns == 1 ? pos : sp1;
      sp2 = ns == 2 ? pos : sp2;
      sp3 = ns == 3 ? pos : sp3;
      ++ns;
    }
  }
  return ns;
}

struct ScanArgs {
  const uint8_t *buf;
  uint64_t n;
  uint64_t n_tiles;
  uint64_t n_lines;
  const uint64_t *tile_base;  // newlines before each wave tile (pass A)
  uint64_t *nl;
  Lines L;
  unsigned long long *stats;  // [0] bitset hits, [1] recorded literal hits
  uint32_t shared_bytes;      // per-wave LDS regions start here
  uint32_t debug_skip;        // timing experiments only (BJX_DEBUG_SKIP, results invalid): 1 gram phase, 2 candidates,
                              // 4 literal checks of gram table hits, 8 gram table probes
};

// pass A: '\n' count per wave tile
__global__ __launch_bounds__(kBlock) void k_nl_count_wt(const uint8_t *__restrict__ buf, uint64_t n, uint64_t n_tiles,
                                                        uint32_t *__restrict__ counts) {
  const uint64_t t = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (t >= n_tiles) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t base = t * kWT + lane * 64u;
  uint32_t c = 0;
  if (base + 64 <= n) {
    const uint4 *src = reinterpret_cast<const uint4 *>(buf + base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = src[k];
      c += __popc(nl_mask_word(v.x)) + __popc(nl_mask_word(v.y)) + __popc(nl_mask_word(v.z)) + __popc(nl_mask_word(v.w));
    }
  } else {
    for (uint64_t k = base; k < n && k < base + 64; ++k) c += buf[k] == '\n';
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) counts[t] = c;
}

__device__ __forceinline__ void push_list(uint32_t *list, unsigned long long *count, uint64_t j) {
  const unsigned long long k = atomicAdd(count, 1ull);
  list[k] = (uint32_t)j;
}

// lookup image viewed from LDS (scan pass) or HBM (other kernels)
struct Tabs {
  const uint32_t *gt, *ge, *ht;
  const uint64_t *hrec;
  const uint32_t *hid;
  const uint8_t *hbytes;
  const uint32_t *lrec;
  const uint8_t *lbytes;
  const uint8_t *lcim;
  const uint8_t *lchk;
};
__device__ __forceinline__ Tabs make_tabs(const uint8_t *base, const ImgLayout &il) {
  Tabs t;
  t.gt = reinterpret_cast<const uint32_t *>(base + il.gt);
  t.ge = reinterpret_cast<const uint32_t *>(base + il.ge);
  t.ht = reinterpret_cast<const uint32_t *>(base + il.ht);
  t.hrec = reinterpret_cast<const uint64_t *>(base + il.hrec);
  t.hid = reinterpret_cast<const uint32_t *>(base + il.hid);
  t.hbytes = base + il.hbytes;
  t.lrec = reinterpret_cast<const uint32_t *>(base + il.lrec);
  t.lbytes = base + il.lbytes;
  t.lcim = base + il.lcim;
  t.lchk = base + il.lchk;
  return t;
}

// host id from the open-addressing host table
// host id from the inline host slots (per-line pass): each probe step loads
// the whole 64 B slot at once (four 16 B loads, one round trip) and compares
// hosts of up to 48 B from registers, so a lookup costs one dependent global
// access instead of one per 4-byte word
__device__ __forceinline__ int32_t host_lookup_slots(const Bind &B, const uint8_t *h, uint32_t n) {
  if (B.n_hd == 0) return -1;
  const uint64_t hh = hash_bytes(h, n);
  const uint32_t tag = (uint32_t)(hh >> 32) | 1u;
  uint32_t s = (uint32_t)hh & (B.ht_cap - 1);
  for (;;) {
    const uint4 *sp = reinterpret_cast<const uint4 *>(B.hslot + s);
    const uint4 q0 = sp[0], q1 = sp[1], q2 = sp[2], q3 = sp[3];
    if (q0.x == 0) return -1;
    if (q0.x == tag && q0.z == n) {
      if (n > 48) {
        if (bytes_eq(B.hd_bytes + q0.w, h, n)) return (int32_t)q0.y;
      } else {
        const uint32_t iw[12] = {q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
        uint32_t diff = 0;
#pragma unroll
        for (uint32_t k = 0; k < 12; ++k) {
          if (4 * k >= n) break;
          const uint32_t m = n - 4 * k >= 4 ? 0xFFFFFFFFu : (1u << (8 * (n - 4 * k))) - 1u;
          diff |= (ld4(h + 4 * k) ^ iw[k]) & m;
        }
        if (!diff) return (int32_t)q0.y;
      }
    }
    s = (s + 1) & (B.ht_cap - 1);
  }
}

// host id from the LDS copy of Bind::hl (k_lines)
__device__ __forceinline__ int32_t host_lookup_lds(const uint32_t *hl, const uint8_t *h, uint32_t n) {
  const uint32_t cap = hl[0], nh = hl[1];
  const uint2 *slots = reinterpret_cast<const uint2 *>(hl + 2);
  const uint32_t *offs = hl + 2 + 2 * cap;
  const uint8_t *bytes = reinterpret_cast<const uint8_t *>(hl + 2 + 2 * cap + nh);
  // a host of < 32 bytes (every usual one) as words in registers: its loads
  // issued at once, hashed (host_fold: words zero past n, so all eight fold
  // in) and compared from there
  constexpr uint32_t NW = 8;
  uint32_t w[NW];
  const bool short_host = n < 4 * NW;
  uint32_t tag;
  if (short_host) {
    ip_words(h, n, w);
    uint32_t a = 0;
#pragma unroll
    for (uint32_t k = 0; k < NW; ++k) a ^= host_fold_word(w[k], k);
    tag = host_fold_finish(a, n);
  } else {
    tag = host_fold(h, n);
  }
  uint32_t s = tag & (cap - 1);
  for (;;) {
    const uint2 e = slots[s];
    if (e.x == 0) return -1;
    if (e.x == tag && (e.y & 0xFFFFu) == n) {
      const uint32_t hid = e.y >> 16;
      const uint8_t *q = bytes + offs[hid];
      uint32_t diff = 0;
      if (short_host) {
        // dictionary hosts are word aligned and zero padded to a whole word
        const uint32_t *qw = reinterpret_cast<const uint32_t *>(q);
#pragma unroll
        for (uint32_t k = 0; k < NW; ++k)
          if (4 * k < n) diff |= qw[k] ^ w[k];
      } else {
        uint32_t i = 0;
        for (; i + 4 <= n; i += 4) diff |= ld4(h + i) ^ ld4(q + i);
        if (i < n) diff |= (ld4(h + i) ^ ld4(q + i)) & ((1u << (8 * (n - i))) - 1u);
      }
      if (!diff) return (int32_t)hid;
    }
    s = (s + 1) & (cap - 1);
  }
}

__device__ __forceinline__ int32_t host_lookup_ht(const Bind &B, const Tabs &T, const uint8_t *h, uint32_t n) {
  if (B.n_hd == 0) return -1;
  const uint64_t hh = hash_bytes(h, n);
  const uint32_t tag = (uint32_t)(hh >> 32) | 1u;
  uint32_t s = (uint32_t)hh & (B.ht_cap - 1);
  for (;;) {
    const uint32_t k = T.ht[2 * s];
    if (k == 0) return -1;
    if (k == tag) {
      const uint32_t i = T.ht[2 * s + 1];
      const uint64_t rec = T.hrec[i];
      if ((uint32_t)(rec & 0xFFFFFFFFu) == n && bytes_eq(T.hbytes + (rec >> 32), h, n)) return (int32_t)T.hid[i];
    }
    s = (s + 1) & (B.ht_cap - 1);
  }
}

__device__ __forceinline__ uint32_t lit_len_of(const Tabs &T, uint32_t lit) { return T.lrec[lit] & 0xFF; }

// literal `lit` at p: 4 bytes per step, (text | case mask) == literal
// (literals are stored lower-case, 4-byte aligned, zero padded); the literal's
// rarest other window is compared first, so most failing checks cost one step
__device__ __forceinline__ bool literal_at(const Tabs &T, uint32_t lit, const uint8_t *p) {
  const uint32_t rec = T.lrec[lit];
  const uint32_t off = rec >> 8, len = rec & 0xFF;
  const uint8_t *lb = T.lbytes + off, *cm = T.lcim + off;
  const uint32_t c = T.lchk[lit];
  if ((ld4(p + c) | ld4(cm + c)) != ld4(lb + c)) return false;
  uint32_t i = 0;
  for (; i + 4 <= len; i += 4)
    if ((ld4(p + i) | ld4(cm + i)) != ld4(lb + i)) return false;
  if (i < len) {
    const uint32_t m = (1u << (8 * (len - i))) - 1u;
    if (((ld4(p + i) | ld4(cm + i)) ^ ld4(lb + i)) & m) return false;
  }
  return true;
}

// literal_at for the scan pass (text and tables in LDS): a literal of at most
// 16 bytes is compared from five text words, four literal words and four
// case-mask words loaded up front (one LDS round trip, no chain of dependent
// word compares); longer ones go word by word.  The literal tables are padded
// (image slack), and the text is read at most 20 bytes past p - 3, inside the
// wave's tile + halo region for any hit the scan verifies.
__device__ __forceinline__ bool literal_at16(const Tabs &T, uint32_t lit, const uint8_t *p) {
  const uint32_t rec = T.lrec[lit];
  const uint32_t off = rec >> 8, len = rec & 0xFF;
  if (len > 16) return literal_at(T, lit, p);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(p - sh);
  const uint32_t *lw = reinterpret_cast<const uint32_t *>(T.lbytes + off);
  const uint32_t *mw = reinterpret_cast<const uint32_t *>(T.lcim + off);
  uint32_t t[5], l[4], m[4];
#pragma unroll
  for (int k = 0; k < 5; ++k) t[k] = tw[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) { l[k] = lw[k]; m[k] = mw[k]; }
  uint32_t diff = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = __builtin_amdgcn_alignbyte(t[k + 1], t[k], sh);
    const int32_t rest = (int32_t)len - 4 * k;
    const uint32_t valid = rest >= 4 ? ~0u : rest > 0 ? (1u << (8 * rest)) - 1u : 0u;
    diff |= ((x | m[k]) ^ l[k]) & valid;
  }
  return diff == 0;
}

__device__ __forceinline__ void set_pos(uint64_t &m0, uint64_t &m1, uint32_t pos) {
  if (pos < 64) m0 |= 1ull << pos; else m1 |= 1ull << (pos - 64);
}
// home slot of (literal, host) in Bind::lh_tab (cap a power of two)
__host__ __device__ __forceinline__ uint32_t lit_host_slot(uint32_t lit, uint32_t host, uint32_t cap) {
  uint32_t x = lit * 0x9E3779B1u ^ (host + 0x7F4A7C15u) * 0x85EBCA77u;
  x ^= x >> 15;
  x *= 0x2C1B3C6Du;
  x ^= x >> 13;
  return x & (cap - 1);
}
__device__ __forceinline__ bool has_pos(uint64_t m0, uint64_t m1, uint32_t pos) {
  return ((pos < 64 ? m0 >> pos : m1 >> (pos - 64)) & 1) != 0;
}

// DFA work found by the line kernels: staged per wave in LDS, appended to HBM
// with one atomic per wave tile (overflow goes straight to HBM).  A job is
// its line, key (rule | position << 24), slot index (the job sort's value:
// k_dfa finds the line and the window by it) and window record (jrec below).
struct JobSink {
  uint4 *lds;
  uint32_t *cnt;
  uint32_t *jline, *jkey, *jidx;
  uint64_t *jrec;
  unsigned long long *count;
  uint64_t cap;
  uint32_t n_rules;  // a legacy job's key names rule r as n_rules + r: the sort puts them after the windowed ones
};
// Job window records (JobSink::jrec): where k_dfa starts the rule's automaton,
// worked out by the line kernel from the line's hits in registers (k_dfa then
// reads this record and the text, not the line's arrays):
//   bits 0-39 absolute batch offset of the first byte, the text runs to the
//   line's '\n'; kJobSkipState: start in the rule's skip_state (an anchored
//   prefix already matched), else its start state; kJobNoCount: the rule is in
//   the host's hosts_to_skip (a RuleResult, no event).  kJobLegacy: k_dfa
//   derives the window from the line's arrays (kernels other than k_lines2,
//   NFA rules, lead seeks past overflowed hit slots).
constexpr uint64_t kJobOffMask = (1ull << 40) - 1;
constexpr uint64_t kJobSkipState = 1ull << 40;
constexpr uint64_t kJobNoCount = 1ull << 41;
constexpr uint64_t kJobLegacy = 1ull << 63;
constexpr uint32_t kWaveJobBytes = kWaveJobs * 16 + 16;  // per wave: staged jobs + their counter
__device__ __forceinline__ void emit_job(const JobSink &S, uint64_t j, uint32_t r, uint32_t pos, uint64_t rec = kJobLegacy) {
  const uint32_t rk = (rec & kJobLegacy) ? S.n_rules + r : r;
  const uint4 v = make_uint4((uint32_t)j, rk | (pos << 24), (uint32_t)rec, (uint32_t)(rec >> 32));
  const uint32_t c = atomicAdd(S.cnt, 1u);
  if (c < kWaveJobs) { S.lds[c] = v; return; }
  const unsigned long long g = atomicAdd(S.count, 1ull);
  if (g < S.cap) { S.jline[g] = v.x; S.jkey[g] = v.y; S.jidx[g] = (uint32_t)g; S.jrec[g] = rec; }
}

// A wave appends its staged jobs into a chunk of the batch's job array that it
// takes kJobChunk slots at a time: one global atomic per chunk, not one per
// 64 lines (a single counter serialises at ~88 atomics per microsecond:
// MI355X_MICROARCH.md "dequeue").  The chunk's slots left unused at the end
// become null jobs (key null_key, after every rule id in the job sort); the
// wave's real jobs are added to *real once.
constexpr uint32_t kJobChunk = 1024;
struct JobChunk {
  uint64_t base = 0;
  uint32_t left = 0;
  uint64_t real = 0;
};
__device__ __forceinline__ void wave_sync();
__device__ __forceinline__ void flush_jobs(const JobSink &S, JobChunk &C, uint32_t lane) {
  wave_sync();
  const uint32_t cnt = *S.cnt;
  const uint32_t nj = min(cnt, kWaveJobs);
  C.real += cnt;  // the staged ones and those past the staging (emit_job's own slots)
  uint32_t done = 0;
  while (done < nj) {
    if (C.left == 0) {
      unsigned long long b = 0;
      if (lane == 0) b = atomicAdd(S.count, (unsigned long long)kJobChunk);
      C.base = __shfl(b, 0);
      C.left = kJobChunk;
    }
    const uint32_t take = min(C.left, nj - done);
    for (uint32_t i = lane; i < take; i += 64) {
      const uint64_t g = C.base + i;
      const uint4 v = S.lds[done + i];
      if (g < S.cap) {
        S.jline[g] = v.x; S.jkey[g] = v.y; S.jidx[g] = (uint32_t)g;
        S.jrec[g] = ((uint64_t)v.w << 32) | v.z;
      }
    }
    C.base += take;
    C.left -= take;
    done += take;
  }
  wave_sync();
  if (lane == 0) *S.cnt = 0;
  wave_sync();
}
__device__ __forceinline__ void close_jobs(const JobSink &S, JobChunk &C, uint32_t lane, uint32_t null_key,
                                           unsigned long long *real) {
  for (uint32_t i = lane; i < C.left; i += 64) {
    const uint64_t g = C.base + i;
    if (g < S.cap) { S.jline[g] = 0; S.jkey[g] = null_key; S.jidx[g] = (uint32_t)g; S.jrec[g] = kJobLegacy; }
  }
  if (lane == 0 && C.real) atomicAdd(real, (unsigned long long)C.real);
}

// One rule whose decision needs its automaton: an anchored prefix may decide
// it first; otherwise run the DFA here (EMIT = false) or hand it to k_dfa.
template <bool EMIT>
__device__ __forceinline__ void dfa_rule(const Bind &B, const Tabs &T, uint32_t r, uint32_t pos, bool anchored,
                                         const uint8_t *rest, uint32_t rest_len, uint64_t &m0, uint64_t &m1, uint64_t j,
                                         const JobSink &S) {
  if (anchored) {
    const DevRule &R = B.rules[r];
    if (R.anc_len) {
      bool any = false;
      for (uint32_t i = 0; i < R.anc_len && !any; ++i) {
        const uint32_t lit = B.rule_lits[R.anc_off + i];
        any = lit_len_of(T, lit) <= rest_len && literal_at(T, lit, rest);
      }
      if (!any) return;
      if (R.anc_equiv) { set_pos(m0, m1, pos); return; }
    }
  }
  if (EMIT) emit_job(S, j, r, pos);
  else if (rule_match(B, r, rest, rest_len)) set_pos(m0, m1, pos);
}

// Inline test of an anchored rule's single prefix literal (bind record
// dfa_*_q: qa = {len, window offset | exact << 8 | equiv << 9, case mask of
// the 8-byte window}, qb = {window bytes}): 0 = the literal cannot start
// rest (too long, or the window differs), 1 = the whole literal matched
// (len <= 8), 2 = undecided (dfa_rule decides).  The window is the literal's
// tail: per-site literals share their host part with every line of the host.
__device__ __forceinline__ uint32_t anchor_quick(const uint4 qa, const uint4 qb, const uint8_t *rest, uint32_t rest_len) {
  if (qa.x == 0) return 2;
  if (qa.x > rest_len) return 0;
  const uint32_t o = qa.y & 0xFF, nb = qa.x - o < 8 ? qa.x - o : 8;
  const uint32_t m0 = nb >= 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1u;
  const uint32_t m1 = nb >= 8 ? 0xFFFFFFFFu : (nb <= 4 ? 0u : (1u << (8 * (nb - 4))) - 1u);
  const uint32_t t0 = ld4(rest + o), t1 = nb > 4 ? ld4(rest + o + 4) : 0u;
  if ((((t0 | qa.z) ^ qb.x) & m0) | (((t1 | qa.w) ^ qb.y) & m1)) return 0;
  return ((qa.y >> 8) & 1) ? 1u : 2u;
}

// The applicable rules of one line (per-site[host] then global, YAML order;
// regex_rate_limiter.go:175-211) decided from the line's verified literal
// hits.  Writes the match mask (positions < 128) and the result/event counts
// of the rules decided here; rules left to k_dfa add theirs atomically.
// lits: up to 4 literal ids packed 16 bits each.
// The per-host words decide_rules needs, loaded together as soon as the host
// id is known (ahead of the exemption check and the per-line stores, which
// the compiler cannot move these loads across)
struct HostRules {
  uint32_t s_begin, s_end;  // site rules [site_off[hid], site_off[hid + 1])
  uint32_t d_begin, d_end;  // anchored / no-literal site rules (dfa_site_off)
  uint64_t a0, a1, k0, k1;  // ALWAYS and hosts_to_skip position masks of the scope
};
__device__ __forceinline__ HostRules host_rules(const Bind &B, int32_t hid) {
  HostRules H;
  const uint32_t sc = hid >= 0 ? (uint32_t)hid : B.n_hosts;
  H.s_begin = H.s_end = H.d_begin = H.d_end = 0;
  if (hid >= 0) {
    H.s_begin = B.site_off[hid]; H.s_end = B.site_off[hid + 1];
    H.d_begin = B.dfa_site_off[hid]; H.d_end = B.dfa_site_off[hid + 1];
  }
  H.a0 = B.sc_always[2 * sc]; H.a1 = B.sc_always[2 * sc + 1];
  H.k0 = B.sc_skip[2 * sc]; H.k1 = B.sc_skip[2 * sc + 1];
  return H;
}

template <bool EMIT>
__device__ __forceinline__ void decide_rules(const Bind &B, const Tabs &T, const uint8_t *rest, uint32_t rest_len, int32_t hid,
                             const HostRules &H, uint64_t lits, uint64_t lpos, uint32_t nlit, bool ovf, uint64_t j,
                             const Lines &L, const JobSink &S, uint32_t dbg = 0) {
  const uint32_t nsite = H.s_end - H.s_begin;
  uint64_t m0 = H.a0, m1 = H.a1;
  // anchored / no-literal rules: every line
  if (hid >= 0 && !(dbg & 1))
    for (uint32_t i = H.d_begin; i < H.d_end; ++i) {
      const uint2 e = B.dfa_site[i];
      const uint4 qa = B.dfa_site_q[2 * i], qb = B.dfa_site_q[2 * i + 1];
      const uint32_t qk = anchor_quick(qa, qb, rest, rest_len);
      if (qk == 0) continue;
      if (qk == 1 && ((qa.y >> 9) & 1)) { set_pos(m0, m1, e.y); continue; }
      dfa_rule<EMIT>(B, T, e.x, e.y, true, rest, rest_len, m0, m1, j, S);
    }
  for (uint32_t i = 0; i < (dbg & 1 ? 0u : B.n_dfa_glob); ++i) {
    const uint2 e = B.dfa_glob[i];
    const uint4 qa = B.dfa_glob_q[2 * i], qb = B.dfa_glob_q[2 * i + 1];
    const uint32_t qk = anchor_quick(qa, qb, rest, rest_len);
    if (qk == 0) continue;
    if (qk == 1 && ((qa.y >> 9) & 1)) { set_pos(m0, m1, nsite + e.y); continue; }
    dfa_rule<EMIT>(B, T, e.x, nsite + e.y, true, rest, rest_len, m0, m1, j, S);
  }
  if (ovf) {
    // more hits than slots: every literal rule by its DFA (exact, slower)
    if (hid >= 0)
      for (uint32_t i = B.pref_site_off[hid]; i < B.pref_site_off[hid + 1]; ++i) {
        const uint2 e = B.pref_site[i];
        dfa_rule<EMIT>(B, T, e.x, e.y, false, rest, rest_len, m0, m1, j, S);
      }
    for (uint32_t i = 0; i < B.n_pref_glob; ++i) {
      const uint2 e = B.pref_glob[i];
      dfa_rule<EMIT>(B, T, e.x, nsite + e.y, false, rest, rest_len, m0, m1, j, S);
    }
  } else {
    uint64_t t0 = 0, t1 = 0;  // literal rules already decided
    for (uint32_t c = 0; c < nlit; ++c) {
      const uint32_t lit = (uint32_t)(lits >> (16 * c)) & 0xFFFF;
      bool dup = false;
      for (uint32_t d = 0; d < c; ++d) dup = dup || ((uint32_t)(lits >> (16 * d)) & 0xFFFF) == lit;
      const uint32_t b = B.lr_off[lit], g = B.lr_gend[lit], e = B.lr_off[lit + 1];
      // the (literal, host) run's home slot goes out with the literal's bounds:
      // both depend on the literal id alone
      uint32_t sl = hid >= 0 ? lit_host_slot(lit, (uint32_t)hid, B.lh_cap) : 0u;
      uint4 run = hid >= 0 ? B.lh_tab[sl] : make_uint4(0, 0, 0, 0);
      if (dup && g == e) continue;  // site runs are revisited: their full-literal checks are per hit
      for (uint32_t i = dup ? g : b; i < g; ++i) {
        const uint2 x = B.lr_ent[i];
        const uint32_t pos = nsite + x.y;
        if (has_pos(t0, t1, pos)) continue;
        set_pos(t0, t1, pos);
        if (x.x >> 31) set_pos(m0, m1, pos);
        else dfa_rule<EMIT>(B, T, x.x, pos, false, rest, rest_len, m0, m1, j, S);
      }
      if (hid < 0 || g == e) continue;
      // this host's run of the literal's site entries: one (usually) probe
      while (!(run.x == 0 || (run.x == lit + 1 && run.y == (uint32_t)hid))) {
        sl = (sl + 1) & (B.lh_cap - 1);
        run = B.lh_tab[sl];
      }
      if (run.x == 0) continue;
      const uint32_t hp = (uint32_t)(lpos >> (16 * c)) & 0xFFFF;  // hit offset in rest (0xFFFF: unknown)
      for (uint32_t i = run.z; i < run.w; ++i) {
        const uint2 x = B.lr_ent[i];
        if (has_pos(t0, t1, x.y)) continue;
        const uint32_t full = B.lr_full[i];
        if (full != kNone && (x.x >> 31) && hp != 0xFFFF) {
          // host-split literal of an equivalent rule: matched iff the full
          // literal surrounds one of its piece's hits (every hit is recorded:
          // no overflow here); undecided until one does
          const uint32_t fl = full >> 8, off = full & 0xFF;
          if (hp >= off && hp - off + lit_len_of(T, fl) <= rest_len && literal_at(T, fl, rest + (hp - off))) {
            set_pos(t0, t1, x.y);
            set_pos(m0, m1, x.y);
          }
          continue;
        }
        set_pos(t0, t1, x.y);
        if ((x.x >> 31) && full == kNone) set_pos(m0, m1, x.y);
        else dfa_rule<EMIT>(B, T, x.x & 0x7FFFFFFFu, x.y, false, rest, rest_len, m0, m1, j, S);
      }
    }
  }
  L.mword(j, 0) = m0;
  if (B.mask_words > 1) L.mword(j, 1) = m1;
  const uint32_t nres = __popcll(m0) + __popcll(m1);
  const uint32_t nev = __popcll(m0 & ~H.k0) + __popcll(m1 & ~H.k1);
  L.counts[j] = ((uint64_t)nres << 32) | nev;
}

// decide_rules for a scope of more than 128 positions (the per-line fallback,
// k_parse_match<SLOW>): the same literal-driven walk, each rule it names
// decided here by its automaton (or listed for k_nfa_wide), the matches set
// straight in the line's mask words, which hold every position of the scope.
// The reference tries every rule of the scope on every line
// (regex_rate_limiter.go:175-211); a literal rule none of whose prefilter
// literals occurs in the line cannot match, so only the rules of the line's
// hits (all literal rules when the hits overflow the line's slots), its
// anchored / no-literal rules and its ALWAYS rules are looked at.
__device__ __forceinline__ uint32_t lead_start(const Bind &B, const Lines &L, uint64_t j, uint32_t pos, uint64_t rs,
                                               uint32_t rl);

__device__ void decide_wide(const Bind &B, const uint8_t *line, uint64_t s, uint32_t n, uint32_t rest_off, int32_t hid, uint64_t j,
                            const Lines &L, const WideList &WL) {
#ifdef BJX_WIDE_NODECIDE  // timing experiment only (results wrong): the fallback's parse alone
  L.counts[j] = 0;
  return;
#endif
  const Tabs T = make_tabs(B.img, B.il);
  const uint8_t *rest = line + rest_off;
  const uint32_t rest_len = n - rest_off;
  const uint32_t nsite = hid >= 0 ? B.site_off[hid + 1] - B.site_off[hid] : 0u;
  for (uint32_t w = 0; w < B.mask_words; ++w) L.mword(j, w) = 0;
  auto setb = [&](uint32_t pos) { L.mword(j, pos >> 6) |= 1ull << (pos & 63); };
  auto rule_at = [&](uint32_t pos) { return pos < nsite ? B.site_rules[B.site_off[hid] + pos] : pos - nsite; };
  // rule r (its pattern's first rule) at pos by its automaton; wide NFAs to k_nfa_wide
  auto eval = [&](uint32_t r, uint32_t pos) {
#ifdef BJX_WIDE_NOEVAL  // timing experiment only (results wrong): no automaton runs
    return;
#endif
    if (B.any_wide && (B.rules[r].flags & kRuleNfaWide)) {
      const unsigned long long q = atomicAdd(WL.count, 1ull);
      if (q < WL.cap) { WL.line[q] = (uint32_t)j; WL.rule[q] = r; WL.pos[q] = pos; }
    } else if (rule_match(B, r, rest, rest_len)) {
      setb(pos);
    }
  };
  // a rule named by a literal hit: a lead rule's automaton starts at the first
  // hit of its literals (lead_start: every match begins there, as k_dfa's jobs
  // do), not at rest[0]; a lane's run is then a few bytes, not the line
  auto eval_hit = [&](uint32_t r, uint32_t pos) {
#ifdef BJX_WIDE_NOEVAL
    return;
#endif
    if ((B.any_wide && (B.rules[r].flags & kRuleNfaWide)) || !(B.rules[r].lead & 1u)) { eval(r, pos); return; }
    const uint32_t st0 = lead_start(B, L, j, pos, s + rest_off, rest_len);
    if (st0 < rest_len && rule_match(B, r, rest + st0, rest_len - st0)) setb(pos);
  };
  // ALWAYS rules
  if (hid >= 0)
    for (uint32_t i = B.alw_site_off[hid]; i < B.alw_site_off[hid + 1]; ++i) setb(B.alw_site[i]);
  for (uint32_t i = 0; i < B.n_alw_glob; ++i) setb(nsite + B.alw_glob[i]);
  // anchored / no-literal rules: every line (the anchor literal tested first)
  auto anchored = [&](uint32_t r, uint32_t pos, const uint4 qa, const uint4 qb) {
    const uint32_t qk = anchor_quick(qa, qb, rest, rest_len);
    if (qk == 0) return;
    if (qk == 1 && ((qa.y >> 9) & 1)) { setb(pos); return; }
    const DevRule &R = B.rules[r];
    if (R.anc_len) {
      bool any = false;
      for (uint32_t i = 0; i < R.anc_len && !any; ++i) {
        const uint32_t lit = B.rule_lits[R.anc_off + i];
        any = lit_len_of(T, lit) <= rest_len && literal_at(T, lit, rest);
      }
      if (!any) return;
      if (R.anc_equiv) { setb(pos); return; }
    }
    eval(r, pos);
  };
  if (hid >= 0)
    for (uint32_t i = B.dfa_site_off[hid]; i < B.dfa_site_off[hid + 1]; ++i) {
      const uint2 e = B.dfa_site[i];
      anchored(e.x, e.y, B.dfa_site_q[2 * i], B.dfa_site_q[2 * i + 1]);
    }
  for (uint32_t i = 0; i < B.n_dfa_glob; ++i) {
    const uint2 e = B.dfa_glob[i];
    anchored(e.x, nsite + e.y, B.dfa_glob_q[2 * i], B.dfa_glob_q[2 * i + 1]);
  }
  // the line's literal hits inside rest (the scan pass's slots; unverified
  // ones checked here)
  const CandMeta cm =
#ifdef BJX_WIDE_NOHITS  // timing experiment only (results wrong): no literal hits
      CandMeta{};
#else
      L.cand_meta[j];
#endif
  const uint64_t rs = s + rest_off;
  uint32_t lits[kCandSlots], lpos[kCandSlots], nlit = 0;
  const bool ovf = cm.cnt > (uint32_t)kCandSlots;
  for (uint32_t c = 0; c < (uint32_t)kCandSlots && c < cm.cnt && !ovf; ++c) {
    const uint64_t v = L.cand[j * kCandSlots + c];
    const uint32_t lit = (uint32_t)(v & 0x7FFFFF);
    const uint64_t q = v >> 24;
    if (q < rs) continue;
    if (!(v & kCandVerified) && (q + lit_len_of(T, lit) > s + n || !literal_at(T, lit, line + (q - s)))) continue;
    lits[nlit] = lit;
    lpos[nlit++] = q - rs < 0xFFFF ? (uint32_t)(q - rs) : 0xFFFFu;
  }
  if (ovf) {
    // more hits than slots: every literal rule by its automaton (exact, slower)
    if (hid >= 0)
      for (uint32_t i = B.pref_site_off[hid]; i < B.pref_site_off[hid + 1]; ++i) eval(B.pref_site[i].x, B.pref_site[i].y);
    for (uint32_t i = 0; i < B.n_pref_glob; ++i) eval(B.pref_glob[i].x, nsite + B.pref_glob[i].y);
  } else {
    for (uint32_t c = 0; c < nlit; ++c) {
      const uint32_t lit = lits[c];
      bool dup = false;
      for (uint32_t d = 0; d < c; ++d) dup = dup || lits[d] == lit;
      const uint32_t b = B.lr_off[lit], g = B.lr_gend[lit], e = B.lr_off[lit + 1];
      if (!dup)
        for (uint32_t i = b; i < g; ++i) {
          const uint2 x = B.lr_ent[i];
          const uint32_t pos = nsite + x.y;
          if ((L.mword(j, pos >> 6) >> (pos & 63)) & 1) continue;  // matched already
          if (x.x >> 31) setb(pos);
          else eval_hit(x.x, pos);
        }
      if (hid < 0 || g == e) continue;
      // this host's run of the literal's site entries (decide_rules)
      uint32_t sl = lit_host_slot(lit, (uint32_t)hid, B.lh_cap);
      uint4 run = B.lh_tab[sl];
      while (!(run.x == 0 || (run.x == lit + 1 && run.y == (uint32_t)hid))) {
        sl = (sl + 1) & (B.lh_cap - 1);
        run = B.lh_tab[sl];
      }
      if (run.x == 0) continue;
      const uint32_t hp = lpos[c];
      for (uint32_t i = run.z; i < run.w; ++i) {
        const uint2 x = B.lr_ent[i];
        if ((L.mword(j, x.y >> 6) >> (x.y & 63)) & 1) continue;
        const uint32_t full = B.lr_full[i];
        if (full != kNone && (x.x >> 31)) {
          // host-split literal of an equivalent rule: matched iff the full
          // literal surrounds this hit of its piece
          const uint32_t fl = full >> 8, off = full & 0xFF;
          if (hp != 0xFFFF && hp >= off && hp - off + lit_len_of(T, fl) <= rest_len && literal_at(T, fl, rest + (hp - off)))
            setb(x.y);
          else if (hp == 0xFFFF)
            eval_hit(x.x & 0x7FFFFFFFu, x.y);
          continue;
        }
        if ((x.x >> 31) && full == kNone) setb(x.y);
        else eval_hit(x.x & 0x7FFFFFFFu, x.y);
      }
    }
  }
  // RuleResults and events: every set position; no event for a host's hosts_to_skip rules
  uint32_t nres = 0, nev = 0;
  for (uint32_t w = 0; w < B.mask_words; ++w) {
    uint64_t m = L.mword(j, w);
    nres += __popcll(m);
    while (m) {
      const uint32_t pos = 64 * w + (uint32_t)__ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      nev += is_skip(B, rule_at(pos), hid) ? 0u : 1u;
    }
  }
  L.counts[j] = ((uint64_t)nres << 32) | nev;
}

// ---- rule plans (Bind::plan): the same decisions as decide_rules, from one
// 32 B entry per rule of the line's scope.  kinds:
constexpr uint32_t kPlanLit = 0;     // prefilter rule with <= 4 literals: decided by the hits
constexpr uint32_t kPlanLitAny = 1;  // prefilter rule the entry cannot spell out: a DFA job on any hit
constexpr uint32_t kPlanAnchor = 2;  // anchored rule: inline window test, anchor literal, DFA
constexpr uint32_t kPlanScan = 3;    // no literal: a DFA job on every line

// Hits past the line's slots (ovf): which literals occurred (bit = id & 63,
// CandMeta::bits plus the slots' hits)
struct OvfInfo {
  uint64_t bits;
};

template <bool EMIT>
__device__ __forceinline__ void plan_rule(const Bind &B, const Tabs &T, const uint4 a, const uint4 b, uint32_t pos_base,
                                          const uint8_t *rest, uint32_t rest_len, uint64_t lits, uint64_t lpos, uint32_t nlit,
                                          bool ovf, const OvfInfo &ov, uint64_t &m0, uint64_t &m1, uint64_t j,
                                          const JobSink &S) {
  const uint32_t r = a.x & 0xFFFFFu, pos = pos_base + ((a.x >> 20) & 0x7Fu), kind = (a.x >> 27) & 7u;
  const bool eq = ((a.x >> 30) & 1u) != 0;
  if (kind == kPlanScan) {
    dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
  if (kind == kPlanAnchor) {
    const uint4 qa = make_uint4(a.y, a.z, b.x, b.y), qb = make_uint4(b.z, b.w, 0, 0);
    const uint32_t qk = anchor_quick(qa, qb, rest, rest_len);
    if (qk == 0) return;
    if (qk == 1 && ((qa.y >> 9) & 1)) { set_pos(m0, m1, pos); return; }
    if (a.w) {  // the rule's single anchor literal, checked here (dfa_rule's anchored branch)
      if (!((a.w >> 16) <= rest_len && literal_at(T, (a.w & 0xFFFFu) - 1, rest))) return;
      if (eq) { set_pos(m0, m1, pos); return; }
      dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
      return;
    }
    dfa_rule<EMIT>(B, T, r, pos, true, rest, rest_len, m0, m1, j, S);
    return;
  }
  if (ovf) {
    // more hits than slots: a rule none of whose literals occurred cannot
    // match; the others go to their automaton, from the first hit on
    if (kind == kPlanLit) {
      uint64_t need = 0;
      for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t id = ((k < 2 ? a.y : a.z) >> (16 * (k & 1))) & 0xFFFFu;
        if (id != 0xFFFFu) need |= 1ull << (id & 31);
      }
      if (!(ov.bits & need)) return;
    }
    dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
  if (nlit == 0) return;
  if (kind == kPlanLitAny) {
    dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
  for (uint32_t c = 0; c < nlit; ++c) {
    const uint32_t lit = (uint32_t)(lits >> (16 * c)) & 0xFFFFu;
    if (lit != (a.y & 0xFFFFu) && lit != (a.y >> 16) && lit != (a.z & 0xFFFFu) && lit != (a.z >> 16)) continue;
    if (a.w != kNone && eq) {
      // host-split literal of an equivalent rule: matched iff the full literal
      // surrounds one of its piece's hits; undecided until one does
      const uint32_t hp = (uint32_t)(lpos >> (16 * c)) & 0xFFFFu;
      if (hp != 0xFFFFu) {
        const uint32_t fl = a.w >> 8, off = a.w & 0xFFu;
        if (hp >= off && hp - off + b.y <= rest_len && literal_at(T, fl, rest + (hp - off))) set_pos(m0, m1, pos);
        if (has_pos(m0, m1, pos)) return;
        continue;
      }
    }
    if (eq && a.w == kNone) set_pos(m0, m1, pos);
    else dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
}

// decide_rules over the scope's plan entries: the global entries are uniform
// across the wave (scalar loads); a host's site entries are loaded four at a
// time, side by side
template <bool EMIT>
__device__ __forceinline__ void decide_plan(const Bind &B, const Tabs &T, const uint8_t *rest, uint32_t rest_len, int32_t hid,
                                            const HostRules &H, uint64_t lits, uint64_t lpos, uint32_t nlit, bool ovf,
                                            const OvfInfo &ov, uint64_t j, const Lines &L, const JobSink &S, uint32_t dbg = 0) {
  const uint32_t nsite = H.s_end - H.s_begin;
  uint64_t m0 = H.a0, m1 = H.a1;
  if (dbg & 32) nlit = 0;  // timing experiments only (BJX_DEBUG_LINES): 16 no site entries, 32 no literal hits
  if (hid >= 0 && !(dbg & 16)) {
    const uint32_t pb = B.plan_off[hid], pe = B.plan_off[hid + 1];
    for (uint32_t i = pb; i < pe; i += 4) {
      uint4 a[4], b[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool in = i + k < pe;
        a[k] = in ? B.plan[2 * (i + k)] : make_uint4(0, 0, 0, 0);
        b[k] = in ? B.plan[2 * (i + k) + 1] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i + k < pe) plan_rule<EMIT>(B, T, a[k], b[k], 0, rest, rest_len, lits, lpos, nlit, ovf, ov, m0, m1, j, S);
    }
  }
  for (uint32_t i = 0; i < B.n_plan_glob; ++i)
    plan_rule<EMIT>(B, T, B.plan_glob[2 * i], B.plan_glob[2 * i + 1], nsite, rest, rest_len, lits, lpos, nlit, ovf, ov, m0, m1,
                    j, S);
  L.mword(j, 0) = m0;
  if (B.mask_words > 1) L.mword(j, 1) = m1;
  const uint32_t nres = __popcll(m0) + __popcll(m1);
  const uint32_t nev = __popcll(m0 & ~H.k0) + __popcll(m1 & ~H.k1);
  L.counts[j] = ((uint64_t)nres << 32) | nev;
}

// k_lines<.., PROF = true>: wave clock (s_memtime) per loop segment, summed
// over waves: 0 loads + staging, 1 header + timestamp, 2 host lookup, 3 host
// rule words, 4 rule decisions (with decide_plan_lds: the mask stores), 5
// per-line stores, 6 DFA-job flush; in decide_plan_lds 7 hit decoding, 8 site
// class walk, 9 global walk
struct LinesProf {
  uint64_t t = 0;
  uint64_t acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void start() { t = __builtin_amdgcn_s_memtime(); }
  __device__ __forceinline__ void mark(int k) {
    const uint64_t now = __builtin_amdgcn_s_memtime();
    acc[k] += now - t;
    t = now;
  }
};

// ---- plan classes in LDS (k_lines<.., HOST_LDS>, Bind::lt_*).  Hosts whose
// site plans are equal once (a) a host-specific literal F = A + host + C
// becomes a template (A, C) checked around the line's own host field and (b)
// a host-specific rule becomes "the host's rule at this position" share one
// class of entries, so a whole per-site rule set sits in a few hundred bytes of
// LDS next to the host dictionary.
constexpr uint32_t kPlanLitT = 4;     // kPlanLit whose host-split full literal is a template
constexpr uint32_t kPlanAnchorT = 5;  // kPlanAnchor whose single anchor literal is a template
constexpr uint32_t kPlanOwn = 0x80000000u;  // entry word a.x: rule = host's first site rule + position

struct LdsTabs {
  const uint2 *hinfo;   // per host: {class entry offset | entries << 16, first site rule}
  const uint4 *cls;     // class entries (2 x uint4 each, as Bind::plan)
  const uint4 *trec;    // templates: {|A| | |C| << 8 | side << 16, A offset, C offset, 0}
  const uint8_t *pool;  // template bytes (4-byte padded + 4), each followed by its case mask
};

// len bytes at text equal the pool string at p (case mask after the padded bytes)
__device__ __forceinline__ bool pool_eq(const uint8_t *p, uint32_t len, const uint8_t *text) {
  const uint8_t *cm = p + ((len + 3) & ~3u) + 4;
  uint32_t i = 0;
  for (; i + 4 <= len; i += 4)
    if ((ld4(text + i) | ld4(cm + i)) != ld4(p + i)) return false;
  if (i < len) {
    const uint32_t m = (1u << (8 * (len - i))) - 1u;
    if (((ld4(text + i) | ld4(cm + i)) ^ ld4(p + i)) & m) return false;
  }
  return true;
}

// template t = (A, C) occurs in rest at fs as A + host + C, the host being the
// line's own host field (host_rel, host_len: the host lookup matched it exactly)
__device__ __forceinline__ bool tmpl_at(const LdsTabs &LT, uint32_t t, const uint8_t *rest, uint32_t rest_len,
                                        uint32_t host_rel, uint32_t host_len, int32_t fs) {
  const uint4 rec = LT.trec[t];
  const uint32_t la = rec.x & 0xFF, lc = (rec.x >> 8) & 0xFF;
  if (fs < 0) return false;
  const uint32_t hs = (uint32_t)fs + la, he = hs + host_len;
  if (he + lc > rest_len) return false;
  if (!pool_eq(LT.pool + rec.z, lc, rest + he)) return false;
  if (!pool_eq(LT.pool + rec.y, la, rest + fs)) return false;
  if (hs == host_rel) return true;
  // the host spelled somewhere else in rest: compare with the host field
  uint32_t diff = 0, i = 0;
  for (; i + 4 <= host_len; i += 4) diff |= ld4(rest + hs + i) ^ ld4(rest + host_rel + i);
  if (i < host_len) diff |= (ld4(rest + hs + i) ^ ld4(rest + host_rel + i)) & ((1u << (8 * (host_len - i))) - 1u);
  return diff == 0;
}

// one class entry (a, b) of the line's host: template kinds here, the others
// by plan_rule once an own-rule entry names its rule
template <bool EMIT>
__device__ __forceinline__ void plan_rule_lds(const Bind &B, const Tabs &T, const LdsTabs &LT, uint4 a, const uint4 b,
                                              uint32_t first_rule, const uint8_t *rest, uint32_t rest_len, uint32_t host_rel,
                                              uint32_t host_len, uint64_t lits, uint64_t lpos, uint32_t nlit, bool ovf,
                                              const OvfInfo &ov, uint64_t &m0, uint64_t &m1, uint64_t j, const JobSink &S) {
  const uint32_t pos = (a.x >> 20) & 0x7Fu, kind = (a.x >> 27) & 7u;
  if (a.x & kPlanOwn) a.x = (a.x & 0x7FF00000u) | ((first_rule + pos) & 0xFFFFFu);
  const uint32_t r = a.x & 0xFFFFFu;
  const bool eq = ((a.x >> 30) & 1u) != 0;
  if (kind == kPlanAnchorT) {
    if (!tmpl_at(LT, a.w, rest, rest_len, host_rel, host_len, 0)) return;
    if (eq) set_pos(m0, m1, pos);
    else dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
  if (kind != kPlanLitT) {
    plan_rule<EMIT>(B, T, a, b, 0, rest, rest_len, lits, lpos, nlit, ovf, ov, m0, m1, j, S);
    return;
  }
  // the rule requires F = A + host + C; its prefilter literal is the piece A
  // (side 0: F starts at the hit) or C (side 1: the host ends at the hit)
  if (ovf) {
    uint64_t need = 0;
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t id = ((k < 2 ? a.y : a.z) >> (16 * (k & 1))) & 0xFFFFu;
      if (id != 0xFFFFu) need |= 1ull << (id & 31);
    }
    if (!(ov.bits & need)) return;  // the piece never occurred
    dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
  const uint4 rec = LT.trec[a.w];
  const uint32_t la = rec.x & 0xFF;
  const bool side_c = ((rec.x >> 16) & 1u) != 0;
  for (uint32_t c = 0; c < nlit; ++c) {
    const uint32_t lit = (uint32_t)(lits >> (16 * c)) & 0xFFFFu;
    if (lit != (a.y & 0xFFFFu) && lit != (a.y >> 16) && lit != (a.z & 0xFFFFu) && lit != (a.z >> 16)) continue;
    const uint32_t hp = (uint32_t)(lpos >> (16 * c)) & 0xFFFFu;
    if (hp == 0xFFFFu) {  // hit offset unknown: the automaton decides
      dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
      return;
    }
    const int32_t fs = side_c ? (int32_t)hp - (int32_t)host_len - (int32_t)la : (int32_t)hp;
    if (!tmpl_at(LT, a.w, rest, rest_len, host_rel, host_len, fs)) continue;
    if (eq) set_pos(m0, m1, pos);
    else dfa_rule<EMIT>(B, T, r, pos, false, rest, rest_len, m0, m1, j, S);
    return;
  }
}

// decide_plan with the host's site entries from its LDS class
template <bool EMIT>
__device__ __forceinline__ void decide_plan_lds(const Bind &B, const Tabs &T, const LdsTabs &LT, const uint8_t *rest,
                                                uint32_t rest_len, uint32_t host_rel, uint32_t host_len, int32_t hid,
                                                const HostRules &H, uint64_t lits, uint64_t lpos, uint32_t nlit, bool ovf,
                                                const OvfInfo &ov, uint64_t j, const Lines &L, const JobSink &S,
                                                LinesProf *P = nullptr) {
  const uint32_t nsite = H.s_end - H.s_begin;
  uint64_t m0 = H.a0, m1 = H.a1;
  if (P) { __builtin_amdgcn_s_waitcnt(0); P->mark(7); }
  if (hid >= 0) {
    const uint2 hi = LT.hinfo[hid];
    // The wave's lines with a host nearly always share one plan class (hosts
    // whose site rules differ only in their host name share it): its entries
    // are then read with scalar loads from the blob in HBM and each entry's
    // kind is dispatched once for the wave on the scalar unit; otherwise each
    // lane walks its own class from LDS.
    const uint32_t f = (uint32_t)__ffsll((unsigned long long)__ballot(1)) - 1;
    const uint32_t c0 = __builtin_amdgcn_readlane(hi.x, f);
    if (__ballot(hi.x != c0) == 0) {
      typedef const __attribute__((address_space(4))) uint32_t ConstU32;
      ConstU32 *cg = (ConstU32 *)(uintptr_t)(B.hl + B.lt_cls);
      const uint32_t cb = c0 & 0xFFFFu, ce = cb + (c0 >> 16);
      for (uint32_t i = cb; i < ce; ++i) {
        ConstU32 *q = cg + 8 * i;
        plan_rule_lds<EMIT>(B, T, LT, make_uint4(q[0], q[1], q[2], q[3]), make_uint4(q[4], q[5], q[6], q[7]), hi.y, rest, rest_len,
                            host_rel, host_len, lits, lpos, nlit, ovf, ov, m0, m1, j, S);
      }
    } else {
      const uint32_t cb = hi.x & 0xFFFFu, ce = cb + (hi.x >> 16);
      for (uint32_t i = cb; i < ce; ++i)
        plan_rule_lds<EMIT>(B, T, LT, LT.cls[2 * i], LT.cls[2 * i + 1], hi.y, rest, rest_len, host_rel, host_len, lits, lpos,
                            nlit, ovf, ov, m0, m1, j, S);
    }
  }
  if (P) { __builtin_amdgcn_s_waitcnt(0); P->mark(8); }
  for (uint32_t i = 0; i < B.n_plan_glob; ++i)
    plan_rule<EMIT>(B, T, B.plan_glob[2 * i], B.plan_glob[2 * i + 1], nsite, rest, rest_len, lits, lpos, nlit, ovf, ov, m0, m1,
                    j, S);
  if (P) { __builtin_amdgcn_s_waitcnt(0); P->mark(9); }
  L.mword(j, 0) = m0;
  if (B.mask_words > 1) L.mword(j, 1) = m1;
  const uint32_t nres = __popcll(m0) + __popcll(m1);
  const uint32_t nev = __popcll(m0 & ~H.k0) + __popcll(m1 & ~H.k1);
  L.counts[j] = ((uint64_t)nres << 32) | nev;
}

// 16 B per lane global -> LDS without a VGPR round trip (gfx950
// global_load_lds_dwordx4): lane L's bytes land at lds + 16 L (lds wave-uniform)
__device__ __forceinline__ void glds16(const void *g, void *lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                   (__attribute__((address_space(3))) void *)lds, 16, 0, 0);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];

// inclusive wave64 prefix sum on DPP (row_shr within 16-lane rows, then
// row_bcast:15 / row_bcast:31 across rows): no LDS round trips, unlike __shfl_up
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  uint32_t x = v + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xF, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xE, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xC, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}


template <bool IMG_LDS>
__global__ __launch_bounds__(kScanWaves * 64) __attribute__((amdgpu_waves_per_eu(4))) void k_scan(Bind B, ScanArgs A) {
  // ---- block-shared tables (read-only after this barrier): the gram pair
  // table, then the scan's lookup image when it fits
  uint8_t *s_bits = s_dyn;
  uint8_t *s_img = s_dyn + kPairBytes;
  for (uint32_t i = threadIdx.x; i < kPairBytes / 16; i += blockDim.x)
    reinterpret_cast<uint4 *>(s_bits)[i] = reinterpret_cast<const uint4 *>(B.gram_pairs)[i];
  if (IMG_LDS)
    for (uint32_t i = threadIdx.x; i < B.scan_img_bytes / 16; i += blockDim.x)
      reinterpret_cast<uint4 *>(s_img)[i] = reinterpret_cast<const uint4 *>(B.scan_img)[i];
  __syncthreads();
  const Tabs TB = make_tabs(IMG_LDS ? s_img : B.scan_img, B.sil);
  const uint32_t *gt = TB.gt, *ge = TB.ge;

  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t *T = s_dyn + A.shared_bytes + wave * kWaveLds;
  uint16_t *ls = reinterpret_cast<uint16_t *>(T + kTileLds);
  uint16_t *le = ls + kLineCap;
  uint32_t *clist = reinterpret_cast<uint32_t *>(le + kLineCap);
  uint32_t *lcnt = clist + kCandList;
  uint64_t *lh = reinterpret_cast<uint64_t *>(lcnt + kLineCap);  // long-line hits of the round (flush_long)
  uint32_t *lh_n = reinterpret_cast<uint32_t *>(lh + kLongList);
  if (lane == 0) *lh_n = 0;
  const Lines &L = A.L;
  uint32_t n_probe = 0, n_hit = 0, n_gram = 0;

  const uint64_t nw = (uint64_t)gridDim.x * kScanWaves;
  uint64_t t = (uint64_t)blockIdx.x * kScanWaves + wave;
  // Everything a tile needs from HBM is loaded one tile ahead, together: its
  // 64 B per lane, its halo (8 B per lane), and in `qa` the word before the
  // tile (lane 0) and the tile's first line indices tile_base[t] (lanes 1-2)
  // and tile_base[t - 1] (lanes 3-4).  Vector memory operations complete in
  // order (vmcnt), so no load the tile's processing waits for may be issued
  // after the prefetch: the loop body reads only LDS and registers, and the
  // long-line hits that need a slot index from HBM wait at the end of a round
  // (flush_long), when the prefetch has had the whole tile to arrive.
  uint4 q[4];
  uint2 qh;
  uint32_t qa;
  auto load_tile = [&](uint64_t tt) {
    const uint64_t ts = tt * kWT, base = ts + lane * 64u;
    if (base + 64 <= A.n) {
      const uint4 *src = reinterpret_cast<const uint4 *>(A.buf + base);
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = src[k];
    } else {
      // tail tile: bytes past the batch read as 0 (clamped addresses, no branches)
      uint32_t w[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint64_t pos = base + 4 * k + b;
          const uint32_t byte = A.buf[pos < A.n ? pos : A.n - 1];
          v |= (pos < A.n ? byte : 0u) << (8 * b);
        }
        w[k] = v;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    }
    const uint64_t h = ts + kWT + lane * 8u;
    qh = make_uint2(0, 0);
    if (h + 8 <= A.n) qh = *reinterpret_cast<const uint2 *>(A.buf + h);
    else if (h < A.n) {
      uint32_t a = 0, b = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k) {
        const uint64_t pos = h + k;
        const uint32_t byte = pos < A.n ? (uint32_t)A.buf[pos < A.n ? pos : A.n - 1] : 0u;
        if (k < 4) a |= byte << (8 * k); else b |= byte << (8 * (k - 4));
      }
      qh = make_uint2(a, b);
    }
    qa = 0x0A000000u;  // before the batch: as if after a '\n'
    if (lane == 0) {
      if (tt) qa = *reinterpret_cast<const uint32_t *>(A.buf + ts - 4);
    } else if (lane <= 4 && (lane <= 2 || tt)) {
      qa = reinterpret_cast<const uint32_t *>(A.tile_base + tt - (lane <= 2 ? 0 : 1))[(lane - 1) & 1];
    }
  };
  // The long-line hits listed this round (lh): per line one atomicAdd on its
  // hit count gives the slot indices, then the slots or the line summary.
  auto flush_long = [&](uint64_t ts0, uint64_t tb, uint32_t nh) {
    wave_sync();
    const uint32_t nlh = min(*lh_n, kLongList);
    if (nlh == 0) return;
    const bool act = lane < nlh;
    const uint64_t e = act ? lh[lane] : 0;
    const uint32_t lsel = act ? (uint32_t)(e >> 13) & 0x1FFFu : kNone;
    const uint64_t gline = tb + nh + (uint64_t)lsel - 1u;
    uint32_t cc = 0;
    uint64_t pending = __ballot(act);
    while (pending) {
      const uint32_t l0 = (uint32_t)__ffsll((unsigned long long)pending) - 1;
      const uint32_t g = __builtin_amdgcn_readlane(lsel, l0);
      const uint64_t m = __ballot(act && lsel == g);
      uint32_t base = 0;
      if (lane == l0) base = atomicAdd(&L.cand_meta[gline].cnt, (uint32_t)__popcll(m));
      base = __builtin_amdgcn_readlane(base, l0);
      if (act && lsel == g) cc = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      pending &= ~m;
    }
    if (act) {
      const uint32_t rel = (uint32_t)e & 0x1FFFu, lit = (uint32_t)(e >> 32) & 0xFFFFu;
      const uint64_t q0 = ts0 + rel - 256u;
      const uint64_t ver = ((e >> 26) & 1u) ? kCandVerified : 0ull;
      if (cc < (uint32_t)kCandSlots) {
        L.cand[gline * kCandSlots + cc] = (q0 << 24) | ver | lit;
      } else {
        const uint64_t bit = 1ull << (lit & 31);
        atomicOr(reinterpret_cast<unsigned long long *>(&L.cand_meta[gline].bits), ((e >> 27) & 1u) ? bit | (bit << 32) : bit);
        atomicMax(&L.cand_meta[gline].first_inv, ~(uint32_t)(q0 >> 3));
      }
    }
    wave_sync();
    if (lane == 0) *lh_n = 0;
    wave_sync();
  };

  const uint64_t n_iter = (A.n_tiles + nw - 1) / nw;
  if (t < A.n_tiles) load_tile(t);
  for (uint32_t r = 0; r < n_iter; ++r, t += nw) {
    if (t >= A.n_tiles) continue;
    const uint64_t ts0 = t * kWT;
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) { w[4 * k] = q[k].x; w[4 * k + 1] = q[k].y; w[4 * k + 2] = q[k].z; w[4 * k + 3] = q[k].w; }
    const uint2 hv = qh;
    const uint32_t prevb = (uint32_t)__builtin_amdgcn_readlane(qa, 0) >> 24;
    const uint64_t tb = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(qa, 1) | ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(qa, 2) << 32);
    const uint64_t tbm = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(qa, 3) | ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(qa, 4) << 32);
    const uint32_t prev_cnt = t ? (uint32_t)(tb - tbm) : 0u;
    if (t + nw < A.n_tiles) load_tile(t + nw);  // prefetch
    uint4 *dst = reinterpret_cast<uint4 *>(T + lane * 64u);
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    *reinterpret_cast<uint2 *>(T + kWT + lane * 8u) = hv;
    if (lane < 4) reinterpret_cast<uint32_t *>(T + kWT + kHalo)[lane] = 0;

    // ---- '\n' bitmask of my 64 bytes (bytes past the batch end are 0): the
    // 0x80 byte flags of each word (nl_mask_word), 8 bits per two words
    // gathered by v_dot4_u32_u8 (weights 1, 2, 4, 8 on the first word's flags,
    // 16 .. 128 on the second's: the sum is 0x80 x the 8-bit mask)
    uint64_t nlm;
    {
      uint32_t nb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t d = __builtin_amdgcn_udot4(nl_mask_word(w[2 * i]), 0x08040201u, 0u, false);
        nb[i] = __builtin_amdgcn_udot4(nl_mask_word(w[2 * i + 1]), 0x80402010u, d, false) >> 7;
      }
      const uint32_t lo32 = nb[0] | (nb[1] << 8) | (nb[2] << 16) | (nb[3] << 24);
      const uint32_t hi32 = nb[4] | (nb[5] << 8) | (nb[6] << 16) | (nb[7] << 24);
      nlm = ((uint64_t)hi32 << 32) | lo32;
    }
    const uint32_t cnt = __popcll(nlm);
    uint32_t pre = wave_incl_sum(cnt);
    const uint32_t tot = __builtin_amdgcn_readlane(pre, 63);
    pre -= cnt;
    const bool head = prevb == '\n';
    const uint32_t nh = head ? 0u : 1u;
    const bool last_nl = (__shfl((uint32_t)(nlm >> 63), 63) & 1u) != 0;
    const uint32_t n_st = (head ? 1u : 0u) + tot - (last_nl ? 1u : 0u);
    // first '\n' in the tile and in the halo
    const uint64_t any_nl = __ballot(cnt != 0);
    uint32_t p0 = kNone;
    if (any_nl) {
      const uint32_t fl = (uint32_t)__ffsll((unsigned long long)any_nl) - 1;
      const uint64_t fm = __shfl(nlm, fl);
      p0 = fl * 64u + (uint32_t)__ffsll((unsigned long long)fm) - 1;
    }
    uint32_t hmask;
    {
      const uint32_t a = nl_mask_word(hv.x), b = nl_mask_word(hv.y);
      hmask = ((a >> 7) & 1u) | ((a >> 14) & 2u) | ((a >> 21) & 4u) | ((a >> 28) & 8u) |
              (((b >> 7) & 1u) | ((b >> 14) & 2u) | ((b >> 21) & 4u) | ((b >> 28) & 8u)) << 4;
    }
    if (ts0 + kWT + lane * 8u >= A.n) hmask = 0;
    const uint64_t any_h = __ballot(hmask != 0);
    uint32_t hfirst = kNone;
    if (any_h) {
      const uint32_t fl = (uint32_t)__ffsll((unsigned long long)any_h) - 1;
      hfirst = kWT + fl * 8u + (uint32_t)__ffs(__shfl(hmask, fl)) - 1;
    }
    // ---- nl[] and the positions of lines starting in this tile (tile-relative)
    {
      uint64_t x = nlm;
      uint32_t rr = pre;
      while (x) {
        const uint32_t b = (uint32_t)__ffsll((unsigned long long)x) - 1;
        x &= x - 1;
        const uint32_t p = lane * 64u + b;
        if (tb + rr < A.n_lines) A.nl[tb + rr] = ts0 + p;
        const int32_t lk = (int32_t)rr - (int32_t)nh;  // started line this '\n' ends
        if (lk >= 0 && lk < (int32_t)kLineCap) le[lk] = (uint16_t)p;
        if (p + 1 < kWT && lk + 1 < (int32_t)kLineCap) ls[lk + 1] = (uint16_t)(p + 1);
        ++rr;
      }
    }
    if (lane == 0 && head) ls[0] = 0;
    const bool last_in_halo = n_st && !last_nl && hfirst != kNone;
    const bool last_long = n_st && !last_nl && hfirst == kNone;
    if (lane == 0 && last_in_halo && n_st - 1 < kLineCap) le[n_st - 1] = (uint16_t)hfirst;
    wave_sync();
    if (!B.any_prefilter || (A.debug_skip & 1)) continue;
    // bytes of the batch held by the tile + halo in LDS
    const uint64_t win_end = A.n - ts0 < (uint64_t)(kWT + kHalo) ? A.n - ts0 : (uint64_t)(kWT + kHalo);
    // the line open at the tile start is long iff it started before the previous
    // tile (that tile has no '\n') or runs past the previous tile's halo
    const bool open_long = !head && (p0 == kNone || p0 >= kHalo || prev_cnt == 0);
    // window starts in the halo: the last started line's part, before hend
    const uint32_t hend = last_in_halo ? hfirst : kWT;

    // ---- 4-gram prefilter: positions [64 lane, 64 lane + 64) and the last
    // line's halo part.  Positions in pairs (k, k + 1), k even: one 8-byte LDS
    // entry keyed by the 3 bytes the two grams share (gram_pair_index of bytes
    // k + 1 .. k + 3), its low word holding bit (byte k & 31) for the gram at
    // k, its high word bit (byte k + 4 & 31) for the gram at k + 1
    // (engine_types.h gram_pair_*).  Eight entry addresses, then their eight
    // ds_read_b64 in flight together, then the bits: per pair one or two
    // alignbytes, a 24-bit mul, a shift and an and (the address), two bfe (the
    // bfe offsets take the bytes' low 5 bits as they are), a shift, two
    // shift-ors
    {
      const uint32_t nxt = *reinterpret_cast<const uint32_t *>(T + lane * 64u + 64u);
      uint32_t hlo = 0, hhi = 0;
#pragma unroll
      for (int k0 = 0; k0 < 64; k0 += 16) {
        uint2 ent[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k0 + 2 * i;
          const uint32_t lo = w[k >> 2], hi = (k >> 2) < 15 ? w[(k >> 2) + 1] : nxt;
          const uint32_t g1 = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(k & 3) + 1u);  // bytes k + 1 .. k + 4
          ent[i] = *reinterpret_cast<const uint2 *>(s_bits + gram_pair_byte_off(g1));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k0 + 2 * i;
          const uint32_t lo = w[k >> 2], hi = (k >> 2) < 15 ? w[(k >> 2) + 1] : nxt;
          const uint32_t g0 = (k & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(k & 3)) : lo;  // bytes k .. k + 3
          const uint32_t g1 = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(k & 3) + 1u);
          const uint32_t two = __builtin_amdgcn_ubfe(ent[i].x, g0, 1) | (__builtin_amdgcn_ubfe(ent[i].y, g1 >> 24, 1) << 1);
          if (k < 32) hlo |= two << k; else hhi |= two << (k - 32);
        }
      }
      uint64_t hits = ((uint64_t)hhi << 32) | hlo;
      if (ts0 + lane * 64u + 64u > A.n) hits &= (ts0 + lane * 64u >= A.n) ? 0ull : ((1ull << (A.n - ts0 - lane * 64u)) - 1ull);
      // halo positions of the last started line: the lane's 8 halo bytes (hv)
      // and the next lane's first 4, as four pairs with their reads in flight
      uint32_t hh = 0;
      if (lane * 8u + kWT < hend) {
        const uint32_t hw[3] = {hv.x, hv.y, *reinterpret_cast<const uint32_t *>(T + kWT + lane * 8u + 8u)};
        uint2 ent[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 2 * i;
          const uint32_t g1 = __builtin_amdgcn_alignbyte(hw[(k >> 2) + 1], hw[k >> 2], (uint32_t)(k & 3) + 1u);
          ent[i] = *reinterpret_cast<const uint2 *>(s_bits + gram_pair_byte_off(g1));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int k = 2 * i;
          const uint32_t lo = hw[k >> 2], hi = hw[(k >> 2) + 1];
          const uint32_t g0 = (k & 3) ? __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(k & 3)) : lo;
          const uint32_t g1 = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(k & 3) + 1u);
          hh |= (__builtin_amdgcn_ubfe(ent[i].x, g0, 1) | (__builtin_amdgcn_ubfe(ent[i].y, g1 >> 24, 1) << 1)) << k;
        }
        const uint32_t nv = hend - (kWT + lane * 8u);  // halo positions before hend
        if (nv < 8) hh &= (1u << nv) - 1u;
      }
      n_probe += __popcll(hits) + __popc(hh);
      if (A.debug_skip & 2) { hits = 0; hh = 0; }
      // ---- candidates, lane-compacted: every lane appends its surviving
      // positions (with the started-line index they belong to) to a wave list,
      // then the list is verified one candidate per lane
      for (uint32_t i = lane; i < kLineCap; i += 64) lcnt[i] = 0;
      uint64_t rem = hits;
      uint32_t remh = hh;
      for (;;) {
        const uint32_t cn = __popcll(rem) + __popc(remh);
        uint32_t off = wave_incl_sum(cn);
        const uint32_t total = __builtin_amdgcn_readlane(off, 63);
        if (total == 0) break;
        off -= cn;
        // append while the list has room (the rest waits for the next round)
        while ((rem | remh) && off < kCandList) {
          uint32_t pos;
          int32_t lk;
          if (rem) {
            const uint32_t k = (uint32_t)__ffsll((unsigned long long)rem) - 1;
            rem &= rem - 1;
            pos = lane * 64u + k;
            lk = (int32_t)(pre + (uint32_t)__popcll(nlm & ((1ull << k) - 1ull))) - (int32_t)nh;
          } else {
            const uint32_t k = (uint32_t)__ffs(remh) - 1;
            remh &= remh - 1;
            pos = kWT + lane * 8u + k;
            lk = (int32_t)n_st - 1;
          }
          clist[off++] = pos | ((uint32_t)(lk + 1) << 16);
        }
        wave_sync();
        const uint32_t nc = total < kCandList ? total : kCandList;
        for (uint32_t c = lane; c < nc; c += 64) {
          const uint32_t en0 = clist[c];
          const uint32_t s = en0 & 0xFFFF;
          const int32_t lk = (int32_t)(en0 >> 16) - 1;
          const uint32_t g = ld4(T + s);
          if ((g & 0xFF) == '\n' || (A.debug_skip & 8)) continue;
          uint32_t slot = gram_slot(g, B.gt2_cap);
          uint32_t ol;
          for (;;) {
            ol = gt[2 * slot + 1];
            if ((ol & 0xFFFF) == 0 || gt[2 * slot] == g) break;
            slot = (slot + 1) & (B.gt2_cap - 1);
          }
          if ((ol & 0xFFFF) == 0) continue;
          ++n_gram;
          if (A.debug_skip & 4) continue;
          if (lk < 0 && !open_long) continue;  // the previous tile covered it
          const uint64_t gline = tb + nh + (uint64_t)(int64_t)lk;
          if (gline >= A.n_lines) continue;
          // lines whose bytes are all in this window are verified here and
          // counted in LDS (no other tile sees them)
          const bool in_window = lk >= 0 && lk < (int32_t)kLineCap && !(lk == (int32_t)n_st - 1 && last_long);
          for (uint32_t ei = 0; ei < (ol & 0xFFFF); ++ei) {
            const uint32_t en = ge[(ol >> 16) + ei];
            const uint32_t lit = en >> 8, goff = en & 0xFF;
            const int64_t q0 = (int64_t)(ts0 + s) - (int64_t)goff;
            if (q0 < 0) continue;
            const int32_t s0 = (int32_t)s - (int32_t)goff;
            if (in_window) {
              if (s0 < (int32_t)ls[lk] || (uint32_t)s0 + lit_len_of(TB, lit) > le[lk]) continue;
              if (!literal_at16(TB, lit, T + s0)) continue;
              const uint32_t cc = atomicAdd(&lcnt[lk], 1u);
              if (B.cfirst) atomicMin(reinterpret_cast<unsigned long long *>(&L.cand_first[gline * kCandFirstLits + lit]),
                                      (unsigned long long)q0);
              if (cc < (uint32_t)kCandSlots) {
                L.cand[gline * kCandSlots + cc] = ((uint64_t)q0 << 24) | kCandVerified | lit;
              } else {  // past the slots: the line's summary only (CandMeta)
                // a verified hit kCertainGap bytes past the line start lies in
                // rest whenever the header is shorter (k_dfa checks rest_off)
                const bool far = s0 - (int32_t)ls[lk] >= (int32_t)kCertainGap;
                const uint64_t bit = 1ull << (lit & 31);
                atomicOr(reinterpret_cast<unsigned long long *>(&L.cand_meta[gline].bits), far ? bit | (bit << 32) : bit);
                atomicMax(&L.cand_meta[gline].first_inv, ~(uint32_t)((uint64_t)q0 >> 3));
              }
            } else {
              // the line does not fit the window, the literal usually does:
              // checked here when all its bytes are in the tile + halo (literals
              // hold no '\n', so a match cannot cross into another line)
              bool ver = false;
              if (s0 >= 0 && !B.lit_nl && (uint64_t)s0 + lit_len_of(TB, lit) <= win_end) {
                if (!literal_at16(TB, lit, T + s0)) continue;
                ver = true;
              }
              if (B.cfirst) atomicMin(reinterpret_cast<unsigned long long *>(&L.cand_first[gline * kCandFirstLits + lit]),
                                      (unsigned long long)q0);
              // a later line's hit (past the first kLineCap line starts) is
              // never taken as far (an occurrence bit alone is exact)
              const bool far = lk < 0 ? s0 >= (int32_t)kCertainGap
                                      : lk < (int32_t)kLineCap && s0 - (int32_t)ls[lk] >= (int32_t)kCertainGap;
              const uint32_t at = atomicAdd(lh_n, 1u);
              if (at < kLongList && lk + 1 < 0x1FFF) {  // the slot index at the end of the round (flush_long)
                lh[at] = (uint64_t)(uint32_t)(s0 + 256) | ((uint64_t)(uint32_t)(lk + 1) << 13) | ((ver ? 1ull : 0ull) << 26) |
                         ((ver && far ? 1ull : 0ull) << 27) | ((uint64_t)lit << 32);
              } else {  // list full: the slot index right away
                const uint32_t cc = atomicAdd(&L.cand_meta[gline].cnt, 1u);
                if (cc < (uint32_t)kCandSlots) {
                  L.cand[gline * kCandSlots + cc] = ((uint64_t)q0 << 24) | (ver ? kCandVerified : 0ull) | lit;
                } else {
                  const uint64_t bit = 1ull << (lit & 31);
                  atomicOr(reinterpret_cast<unsigned long long *>(&L.cand_meta[gline].bits), ver && far ? bit | (bit << 32) : bit);
                  atomicMax(&L.cand_meta[gline].first_inv, ~(uint32_t)((uint64_t)q0 >> 3));
                }
              }
            }
            ++n_hit;
          }
      }
        flush_long(ts0, tb, nh);
      }
      // hit counts of the lines decided in this window
      const uint32_t n_win = min(n_st, kLineCap) - ((last_long && n_st <= kLineCap) ? 1u : 0u);
      for (uint32_t i = lane; i < n_win; i += 64)
        if (tb + nh + i < A.n_lines) L.cand_meta[tb + nh + i].cnt = lcnt[i];
      wave_sync();
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    n_probe += __shfl_xor(n_probe, o);
    n_hit += __shfl_xor(n_hit, o);
    n_gram += __shfl_xor(n_gram, o);
  }
  if (lane == 0 && (n_probe | n_hit)) {
    atomicAdd(&A.stats[0], (unsigned long long)n_probe);
    atomicAdd(&A.stats[1], (unsigned long long)n_hit);
    atomicAdd(&A.stats[2], (unsigned long long)n_gram);
  }
}

struct LinesArgs {
  uint32_t dbg;  // timing experiments only (BJX_DEBUG_LINES): 1 no anchored checks, 2 no literal hits, 4 unstaged, 8 no host lookup
  uint32_t dbg2; // timing experiments only (BJX_DEBUG_L2, k_lines2; results wrong): 1 no anchored entries, 2 no hit rows, 4 no jobs, 8 no IP fields
  const uint8_t *buf;
  uint64_t n;  // batch bytes
  const uint64_t *nl;
  uint64_t n_lines;
  Lines L;
  int64_t now_ns;
  uint32_t *slow_list;
  unsigned long long *slow_count;
  uint32_t *jline, *jkey, *jidx;
  uint64_t *jrec;
  unsigned long long *job_count;  // job slots taken (chunks)
  unsigned long long *job_real;   // real jobs (the rest are null jobs, key null_key)
  uint32_t null_key;
  uint64_t job_cap;
  uint32_t span_bytes;  // LDS staging per wave (0 = read lines from HBM)
  const uint32_t *list; // non-null: process only these lines (n_list of them), unstaged
  uint64_t n_list;
  unsigned long long *prof;  // BJX_PROF_LINES: shader clocks per k_lines segment (k_lines<.., true>)
};

// consumeLine up to the rule loop for line j (bytes at base + (s - origin)):
// SplitN header, parseTimestamp fast path, host lookup, CheckIsAllowed,
// OldLine, then the rule decisions from the scan pass's literal hits.
// STAGED: base is the wave's LDS span (a distinct instantiation, so the
// compiler cannot merge the two call sites into one generic-pointer copy)
// cc / cv: the line's scan-pass hit count and hit slots, loaded by the caller
// ahead of the staging barrier
template <bool STAGED, bool PROF = false, bool HOST_LDS = false>
__device__ __forceinline__ void line_body(const Bind &B, const Tabs &TB, const LinesArgs &A, const uint8_t *base,
                                          uint64_t origin, uint64_t s, uint32_t n, uint64_t j, const JobSink &S,
                                          const CandMeta &cm, const uint64_t (&cv)[kCandSlots], LinesProf &P,
                                          const uint32_t *hl) {
  const uint32_t cc = cm.cnt;
  const Lines &L = A.L;
  const uint8_t *p = base + (s - origin);
  uint32_t sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0;
  const uint32_t ns = find_spaces(p, n, sp0, sp1, sp2, sp3);
  double f;
  int32_t hid = -1;
  HostRules H;
  bool slow = false;
  if (ns >= 4) {
    slow = parse_ts_msec(p, sp0, &f) != 0 && parse_float_fast(p, sp0, &f) != 0;
    if (PROF) P.mark(1);
    if (!slow) {
      hid = (A.dbg & 8) ? -1
            : HOST_LDS ? host_lookup_lds(hl, p + sp2 + 1, sp3 - sp2 - 1) : host_lookup_slots(B, p + sp2 + 1, sp3 - sp2 - 1);
      if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(2); }
      H = host_rules(B, hid);
      if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(3); }
      slow = (H.s_end - H.s_begin) + B.n_global > 128;
    }
  }
  if (ns < 4) {
    L.flags[j] = kLineError;
    L.counts[j] = 0;
  } else if (slow) {
    // exotic timestamp token or > 128 applicable rules: the per-line fallback
    L.flags[j] = kLineSlowTs;
    L.counts[j] = 0;
    push_list(A.slow_list, A.slow_count, j);
  } else {
    const uint32_t ip_off = sp0 + 1, ip_len = sp1 - sp0 - 1;
    const uint32_t rest_off = sp1 + 1, host_off = sp2 + 1, host_len = sp3 - sp2 - 1;
    const bool exempt = B.any_allow && check_is_allowed(B, hid, p + ip_off, ip_len);
    const int64_t tsn = ns_from_seconds(f);
    uint8_t fl = 0;
    if (go_sub(A.now_ns, tsn) > 10000000000LL) fl = kLineOld;
    else if (exempt) fl = kLineExempt;
    // the per-line stores go out after the rule decisions: on gfx9 stores share
    // vmcnt with loads, so a store issued ahead of decide_rules' dependent
    // table loads would hold up every one of their waits
    if (fl) {
      L.counts[j] = 0;
    } else {
      // literal hits of the scan pass inside rest (unverified ones checked here)
      uint64_t lits = 0, lpos = 0;
      uint32_t nlit = 0;
      const uint64_t rs = s + rest_off;
      OvfInfo ov{0};
#pragma unroll
      for (uint32_t c = 0; c < (uint32_t)kCandSlots; ++c) {
        if (c >= cc) break;
        const uint64_t v = cv[c];
        const uint32_t lit = (uint32_t)(v & 0x7FFFFF);
        const uint64_t q = v >> 24;
        if (q < rs) continue;
        if (!(v & kCandVerified) &&
            (q + lit_len_of(TB, lit) > s + n || !literal_at(TB, lit, base + (q - origin))))
          continue;
        lpos |= (uint64_t)(q - rs < 0xFFFF ? (uint32_t)(q - rs) : 0xFFFFu) << (16 * nlit);
        lits |= (uint64_t)lit << (16 * nlit++);
        ov.bits |= 1ull << (lit & 31);
      }
      if (cc > (uint32_t)kCandSlots) ov.bits |= cm.bits & 0xFFFFFFFFull;  // the hits past the slots
      if (HOST_LDS && B.lt_cls && !(A.dbg & 15)) {
        LdsTabs LT;
        LT.hinfo = reinterpret_cast<const uint2 *>(hl + B.lt_hinfo);
        LT.cls = reinterpret_cast<const uint4 *>(hl + B.lt_cls);
        LT.trec = reinterpret_cast<const uint4 *>(hl + B.lt_trec);
        LT.pool = reinterpret_cast<const uint8_t *>(hl + B.lt_pool);
        decide_plan_lds<true>(B, TB, LT, p + rest_off, n - rest_off, host_off - rest_off, host_len, hid, H, lits, lpos, nlit,
                              cc > (uint32_t)kCandSlots, ov, j, L, S, PROF ? &P : nullptr);
      } else if (B.use_plan && !(A.dbg & 15))
        decide_plan<true>(B, TB, p + rest_off, n - rest_off, hid, H, lits, lpos, nlit, cc > (uint32_t)kCandSlots, ov, j, L, S,
                          A.dbg);
      else
        decide_rules<true>(B, TB, p + rest_off, n - rest_off, hid, H, lits, lpos, (A.dbg & 2) ? 0u : nlit,
                           cc > (uint32_t)kCandSlots, j, L, S, A.dbg);
    }
    if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(4); }
    if (A.dbg & 64) return;  // timing experiment: no per-line stores
    L.ip_len[j] = ip_len;
    L.rest_off[j] = rest_off;
    L.host_id[j] = hid;
    {
      uint4 k16;
      uint64_t h;
      ip_key_hash(p + ip_off, ip_len, k16, h);
      if (ip_len > 15) L.ip_hash[j] = h;
      L.ip16[j] = k16;
    }
    L.ts[j] = tsn;
    L.flags[j] = fl;
    if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(5); }
  }
}

// consumeLine up to the rule loop, one lane per line (regex_rate_limiter.go:113-214):
// SplitN header, parseTimestamp fast path, host lookup, CheckIsAllowed, OldLine,
// then the rule decisions from the scan pass's literal hits (DFA work to k_dfa).
template <bool IMG_LDS, bool PROF = false, bool HOST_LDS = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_lines(Bind B, LinesArgs A) {
  LinesProf P;
  uint8_t *s_img = s_dyn;
  if (IMG_LDS) {
    for (uint32_t i = threadIdx.x; i < B.img_bytes / 16; i += blockDim.x)
      reinterpret_cast<uint4 *>(s_img)[i] = reinterpret_cast<const uint4 *>(B.img)[i];
    __syncthreads();
  }
  const Tabs TB = make_tabs(IMG_LDS ? s_img : B.img, B.il);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the compact host dictionary after the image (host lookups from LDS)
  const uint32_t img_al = (IMG_LDS ? B.img_bytes : 0) + 15u & ~15u, hl_al = HOST_LDS ? B.hl_bytes + 15u & ~15u : 0u;
  uint32_t *s_hl = reinterpret_cast<uint32_t *>(s_dyn + img_al);
  if (HOST_LDS) {
    for (uint32_t i = threadIdx.x; i < B.hl_bytes / 4; i += blockDim.x) s_hl[i] = B.hl[i];
    __syncthreads();
  }
  JobSink S;
  S.lds = reinterpret_cast<uint4 *>(s_dyn + img_al + hl_al + wave * kWaveJobBytes);
  S.cnt = reinterpret_cast<uint32_t *>(S.lds + kWaveJobs);
  S.jline = A.jline;
  S.jkey = A.jkey;
  S.jidx = A.jidx;
  S.jrec = A.jrec;
  S.n_rules = B.n_rules;
  S.count = A.job_count;
  S.cap = A.job_cap;
  if (lane == 0) *S.cnt = 0;
  wave_sync();
  JobChunk JC;
  const Lines &L = A.L;
  // this wave's 64 lines, staged whole in LDS with coalesced 16 B loads when
  // they span at most kSpanBytes (otherwise read from HBM per lane)
  uint8_t *span = s_dyn + img_al + hl_al + (kBlock / 64) * kWaveJobBytes + wave * (A.span_bytes + 32);
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t n_work = A.list ? A.n_list : A.n_lines;
  // span bounds of the wave's next 64 lines, loaded one iteration ahead
  auto span_bounds = [&](uint64_t b, uint64_t &a0, uint64_t &a1) {
    a0 = b ? A.nl[b - 1] + 1 : 0;
    a1 = A.nl[min(b + 63, A.n_lines - 1)];
  };
  uint64_t s0n = 0, s1n = 0;
  const uint64_t base0 = (uint64_t)blockIdx.x * blockDim.x + wave * 64u;
  if (!A.list && base0 < n_work) span_bounds(base0, s0n, s1n);
  for (uint64_t base = base0; base < n_work; base += stride) {
    if (PROF) P.start();
    const uint64_t j = A.list ? (base + lane < n_work ? A.list[base + lane] : A.n_lines) : base + lane;
    const uint64_t s0 = s0n, s1 = s1n;
    if (!A.list && base + stride < n_work) span_bounds(base + stride, s0n, s1n);
    const uint64_t b16 = s0 & ~15ull;
    const bool staged = !A.list && s1 + 16 - b16 <= A.span_bytes && !(A.dbg & 4);  // 16 B of slack for word-wise over-reads
    // per-line loads that do not depend on the staged bytes go out first
    uint64_t s = 0, cv[kCandSlots];
    uint32_t n = 0;
    CandMeta cm{0, 0, 0};
    if (j < A.n_lines) {
      s = j ? A.nl[j - 1] + 1 : 0;
      n = (uint32_t)(A.nl[j] - s);
      if (B.any_prefilter) {
        cm = L.cand_meta[j];
        const ulonglong2 *cp = reinterpret_cast<const ulonglong2 *>(L.cand + j * kCandSlots);
#pragma unroll
        for (int k = 0; k < kCandSlots / 2; ++k) {
          const ulonglong2 w = cp[k];
          cv[2 * k] = w.x; cv[2 * k + 1] = w.y;
        }
      }
    }
    if (staged) {
      const uint32_t n16 = (uint32_t)((s1 + 16 - b16 + 15) >> 4);
      // LDS-DMA: every 1 KB piece of the span in flight at once (the loads
      // write LDS directly: wave-uniform base + lane x 16 B), one wait
      for (uint32_t k = 0; k * 64 < n16; ++k) {
        const uint32_t i = k * 64 + lane;
        const uint64_t a = b16 + 16ull * i;
        if (i < n16 && a + 16 <= A.n)
          glds16(A.buf + a, span + 1024u * k);
      }
      __builtin_amdgcn_s_waitcnt(0);
      // the batch's last bytes (zero past the end): one lane writes the tail piece
      for (uint32_t i = lane; b16 + 16ull * n16 > A.n && i < n16; i += 64) {
        const uint64_t a = b16 + 16ull * i;
        uint4 v;
        if (a + 16 <= A.n) {
          continue;
        } else {
          uint32_t w[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b) {
              const uint64_t q = a + 4 * k + b;
              if (q < A.n) x |= (uint32_t)A.buf[q] << (8 * b);
            }
            w[k] = x;
          }
          v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        reinterpret_cast<uint4 *>(span)[i] = v;
      }
      wave_sync();
    }
    if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(0); }
    if (j < A.n_lines) {
      // two inlined copies: LDS addressing for staged waves, global otherwise
      if (staged) line_body<true, PROF, HOST_LDS>(B, TB, A, span, b16, s, n, j, S, cm, cv, P, s_hl);
      else line_body<false, PROF, HOST_LDS>(B, TB, A, A.buf, 0, s, n, j, S, cm, cv, P, s_hl);
    }
    if (PROF) P.t = __builtin_amdgcn_s_memtime();
    // ---- append this wave's DFA jobs (from its chunk of the job array)
    flush_jobs(S, JC, lane);
    if (PROF) { __builtin_amdgcn_s_waitcnt(0); P.mark(6); }
  }
  close_jobs(S, JC, lane, A.null_key, A.job_real);
  if (PROF && lane == 0)
    for (int k = 0; k < 10; ++k) atomicAdd(&A.prof[k], (unsigned long long)P.acc[k]);
}

#include "lines2.h"


// DFA jobs of the line pass, sorted by rule: one (line, rule) per lane.  A
// block whose jobs share one rule (the common case) stages that rule's
// transition rows and ASCII class map in LDS; every lane reads its text 16 B
// at a time and steps the DFA over the ASCII bytes from registers (a non-ASCII
// byte hands the rest of the text to the rune-decoding loop).  A match sets
// the rule's bit and adds to the line's result / event counts.
// Offset in rest where a DFA job of a lead rule may start (DevRule::lead: the
// pattern's every match begins with one of its literals, and this copy's
// literals are not host-split pieces).  Every occurrence of a literal is one
// of the line's scan candidates (the gram filter misses none): without
// overflow the lowest candidate of the rule's own literals at or past rest
// bounds the first match start (none: no match, start at the end); with
// overflow the lowest candidate of any literal does (CandMeta::first_inv),
// unless one lies before rest.  0 for every other job.
__device__ __forceinline__ uint32_t lead_start(const Bind &B, const Lines &L, uint64_t j, uint32_t pos, uint64_t rs,
                                               uint32_t rl) {
  const int32_t hid = L.host_id[j];
  uint32_t sb = 0, nsite = 0;
  if (hid >= 0) { sb = B.site_off[hid]; nsite = B.site_off[hid + 1] - sb; }
  const uint32_t r = pos < nsite ? B.site_rules[sb + pos] : B.global_rules[pos - nsite];  // the line's own rule
  const uint32_t lead = B.rules[r].lead, lo = B.rules[r].lits_off, ln = B.rules[r].lits_len;
  if ((lead & 3u) != 3u) return 0;
  // a bounded piece may precede the literal (lead_dist; + 3 so a rune cut by
  // the start decodes to errors that end before the match)
  const uint32_t back = B.rules[r].lead_dist ? B.rules[r].lead_dist + 3u : 0u;
  if (B.cfirst) {  // the first candidate of each literal of the line: exact, overflow or not
    uint64_t f = ~0ull;
    for (uint32_t k = 0; k < ln; ++k) {
      const uint64_t q = L.cand_first[j * kCandFirstLits + B.rule_lits[lo + k]];
      f = q < f ? q : f;
    }
    if (f == ~0ull) return rl;  // none of its literals occurs: no match
    // a first candidate in the header still bounds the first one in rest from below
    const uint32_t o = f <= rs ? 0u : (uint32_t)min<uint64_t>(f - rs, rl);
    return o > back ? o - back : 0u;
  }
  const CandMeta cm = L.cand_meta[j];
  const bool ovf = cm.cnt > (uint32_t)kCandSlots;
  uint64_t f = ~0ull;
  const uint32_t ns = min(cm.cnt, (uint32_t)kCandSlots);
  for (uint32_t c = 0; c < ns; ++c) {
    const uint64_t v = L.cand[j * kCandSlots + c];
    const uint64_t q = v >> 24;
    if (q < rs || q >= f) continue;
    bool mine = ovf;
    for (uint32_t k = 0; k < ln && !mine; ++k) mine = B.rule_lits[lo + k] == (uint32_t)(v & 0x7FFFFF);
    if (mine) f = q;
  }
  if (ovf) {
    const uint64_t mf = cm.first_inv ? (uint64_t)(~cm.first_inv) << 3 : ~0ull;
    if (mf < rs) return 0;
    f = mf < f ? mf : f;
  }
  if (f == ~0ull) return rl;
  const uint32_t o = (uint32_t)min<uint64_t>(f - rs, rl);
  return o > back ? o - back : 0u;
}

// First occurrence at or after p (before end) of one of lead rule R's
// literals, or end: the job of a line whose hits overflowed its slots starts
// from the first hit of ANY literal (lead_start), so it skips forward here 16 B
// at a time (first-byte SWAR compare, then the literal's bytes) instead of
// stepping the DFA byte by byte.  Rules with more than 4 literals: p.
constexpr uint32_t kSeekLits = 4;
__device__ __forceinline__ uint64_t lead_seek(const Bind &B, const DevRule &R, const uint8_t *__restrict__ buf, uint64_t n_buf,
                                           uint64_t p, uint64_t end) {
  if (R.lits_len == 0 || R.lits_len > kSeekLits || p >= end) return p;
  const Tabs T = make_tabs(B.img, B.il);
  uint32_t lit[kSeekLits], rep[kSeekLits], cim[kSeekLits];
  const uint32_t nk = R.lits_len;
#pragma unroll
  for (uint32_t k = 0; k < kSeekLits; ++k) {
    lit[k] = k < nk ? B.rule_lits[R.lits_off + k] : 0u;
    const uint32_t off = T.lrec[lit[k]] >> 8;
    rep[k] = k < nk ? (uint32_t)T.lbytes[off] * 0x01010101u : 0u;       // first byte (lower case where ci)
    cim[k] = k < nk ? (uint32_t)T.lcim[off] * 0x01010101u : 0u;         // its case mask
  }
  uint64_t a = p & ~15ull;
  uint32_t skip = (uint32_t)(p - a);
  while (a < end) {
    uint4 v;
    if (a + 16 <= n_buf) v = *reinterpret_cast<const uint4 *>(buf + a);
    else {
      uint32_t w[4];
      for (int k = 0; k < 4; ++k) {
        uint32_t x = 0;
        for (int b = 0; b < 4; ++b) x |= (a + 4 * k + b < n_buf ? (uint32_t)buf[a + 4 * k + b] : 0u) << (8 * b);
        w[k] = x;
      }
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    uint32_t cand = 0;  // bit i: byte a + i equals some literal's first byte
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (uint32_t k = 0; k < kSeekLits; ++k) {
        if (k >= nk) break;
        const uint32_t y = (wv[q] | cim[k]) ^ rep[k];
        const uint32_t hb = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;  // exact zero-byte mask
        cand |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * q);
      }
    }
    cand &= ~((1u << skip) - 1u);
    while (cand) {
      const uint32_t i = (uint32_t)__ffs(cand) - 1;
      cand &= cand - 1;
      const uint64_t q = a + i;
      if (q >= end) return end;
#pragma unroll
      for (uint32_t k = 0; k < kSeekLits; ++k) {
        if (k >= nk) break;
        const uint32_t len = T.lrec[lit[k]] & 0xFF;
        if (q + len <= end && literal_at(T, lit[k], buf + q)) return q;
      }
    }
    skip = 0;
    a += 16;
  }
  return end;
}

// A job of an equivalent literal rule (match <=> one of its literals occurs
// in rest) decided without its automaton when the scan saw one for certain:
// a verified slot hit of the line's own rule's literal at or past rest, or,
// past the slots, a verified hit of it kCertainGap bytes into the line with
// the header shorter than that (CandMeta::bits, exact while the ruleset has
// at most 32 literals).
__device__ __forceinline__ bool eq_certain(const Bind &B, const Lines &L, uint64_t j, uint32_t pos, uint64_t rs) {
  const int32_t hid = L.host_id[j];
  uint32_t sb = 0, nsite = 0;
  if (hid >= 0) { sb = B.site_off[hid]; nsite = B.site_off[hid + 1] - sb; }
  const uint32_t r = pos < nsite ? B.site_rules[sb + pos] : B.global_rules[pos - nsite];
  const DevRule &R = B.rules[r];
  if (!R.equiv || !(R.lead & 2u)) return false;  // equivalent, literals not host-split
  const CandMeta cm = L.cand_meta[j];
  const uint32_t ns = min(cm.cnt, (uint32_t)kCandSlots);
  uint64_t need = 0;
  for (uint32_t k = 0; k < R.lits_len; ++k) need |= 1ull << (B.rule_lits[R.lits_off + k] & 31);
  for (uint32_t c = 0; c < ns; ++c) {
    const uint64_t v = L.cand[j * kCandSlots + c];
    if (!(v & kCandVerified) || (v >> 24) < rs) continue;
    for (uint32_t k = 0; k < R.lits_len; ++k)
      if (B.rule_lits[R.lits_off + k] == (uint32_t)(v & 0x7FFFFF)) return true;
  }
  return cm.cnt > (uint32_t)kCandSlots && B.lits_small && L.rest_off[j] <= kCertainGap && ((cm.bits >> 32) & need) != 0;
}

// lead_start, then, for a line whose hits overflowed its slots (the start is
// then the first hit of any literal), lead_seek to the rule's own literal
__device__ __forceinline__ uint32_t lead_start_seek(const Bind &B, const DevRule &R, const Lines &L, const uint8_t *buf,
                                                    uint64_t n_buf, uint64_t j, uint32_t pos, uint64_t rs, uint32_t rl) {
  const uint32_t st0 = lead_start(B, L, j, pos, rs, rl);
  if ((R.lead & 3u) != 3u || st0 >= rl || B.cfirst || L.cand_meta[j].cnt <= (uint32_t)kCandSlots) return st0;
  const uint32_t back = R.lead_dist ? R.lead_dist + 3u : 0u;
  const uint64_t q = lead_seek(B, R, buf, n_buf, rs + st0 + (st0 ? back : 0u), rs + rl);
  const uint32_t o = (uint32_t)(q - rs);
  return o >= rl ? rl : (o > back && o - back > st0 ? o - back : st0);
}

constexpr uint32_t kDfaLdsEntries = 8192;
constexpr uint32_t kDfaAccelLds = 2048;  // accel words staged per block (8 KB)  // u16 transitions staged per block (16 KB)

// STAGED: tr / ac point into LDS (a distinct instantiation keeps the call
// sites apart, so each keeps its address space instead of generic loads)
// escape mask of 16 text bytes for an accelerated state (Bind::accel word ac):
// bit i set when byte i is one of its n escape bytes or non-ASCII
__device__ __forceinline__ uint32_t accel_mask(const uint4 v, uint32_t ac) {
  const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
  const uint32_t ne = (ac >> 24) & 3u;
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t hb = wv[q] & 0x80808080u;
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      if (k >= ne) break;
      const uint32_t y = wv[q] ^ (((ac >> (8 * k)) & 0xFFu) * 0x01010101u);
      hb |= ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
    }
    m |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * q);
  }
  return m;
}

// STAGED: tr / ac point into LDS (a distinct instantiation keeps the call
// sites apart, so each keeps its address space instead of generic loads).
// acc: the rule's Bind::accel words (nullptr: none): at each 16 B boundary in
// a self-loop state the text up to the next escape byte is skipped, 16 B per
// step, instead of being stepped byte by byte (every skipped byte maps the
// state to itself, so the result is the same)
template <bool STAGED>
__device__ __forceinline__ bool dfa_text(const Bind &B, const DevRule &R, const uint16_t *tr, const uint8_t *ac,
                                         const uint32_t *acc, const uint8_t *__restrict__ buf, uint64_t n_buf, uint64_t t0,
                                         uint32_t len, uint32_t st0) {
  const uint32_t ncls = R.ncls;
  uint32_t st = st0;
  uint64_t a = t0 & ~15ull;
  const uint64_t end = t0 + len;
  uint32_t skip = (uint32_t)(t0 - a);
  auto load16 = [&](uint64_t p) -> uint4 {
    if (p + 16 <= n_buf) return *reinterpret_cast<const uint4 *>(buf + p);
    uint32_t w[4];
    for (int k = 0; k < 4; ++k) {
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b) x |= (p + 4 * k + b < n_buf ? (uint32_t)buf[p + 4 * k + b] : 0u) << (8 * b);
      w[k] = x;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  };
  // software-pipelined: the next 16 B are in flight while the DFA steps over
  // the current ones (each step is a dependent LDS lookup)
  uint4 v = a < end ? load16(a) : make_uint4(0, 0, 0, 0);
  while (a < end) {
    const uint32_t aw = acc ? acc[st] : 0u;
    if (aw >> 31) {
      for (;;) {
        uint32_t m = accel_mask(v, aw) & ~((1u << skip) - 1u);
        if (end - a < 16) m &= (1u << (uint32_t)(end - a)) - 1u;
        if (m) { skip = (uint32_t)__ffs(m) - 1; break; }
        a += 16;
        skip = 0;
        if (a >= end) return B.accept_end[R.ae_off + st] != 0;
        v = load16(a);
      }
    }
    const uint4 vn = a + 16 < end ? load16(a + 16) : make_uint4(0, 0, 0, 0);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    const uint32_t lim = end - a < 16 ? (uint32_t)(end - a) : 16u;
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < skip || k >= lim) continue;
      const uint32_t b = (wv[k >> 2] >> (8 * (k & 3))) & 0xFF;
      if (b >= 0x80) {
        // non-ASCII: decode runes from here on (Go's regexp steps by rune)
        const DevRule *Rp = &R;
        uint64_t i = a + k;
        while (i < end) {
          int w;
          const int32_t rune = decode_rune_hd(buf + i, (uint32_t)(end - i), &w);
          uint32_t c;
          if (rune < 0x80) c = ac[rune];
          else {
            const uint32_t *na = B.nonascii + 2 * Rp->na_off;
            uint32_t lo = 0, hi = Rp->n_na;
            while (hi - lo > 1) {
              const uint32_t m = (lo + hi) >> 1;
              if (na[2 * m] <= (uint32_t)rune) lo = m; else hi = m;
            }
            c = na[2 * lo + 1];
          }
          i += (uint32_t)w;
          st = tr[st * ncls + c];
          if (st <= 1) break;
        }
        return B.accept_end[R.ae_off + st] != 0;
      }
      st = tr[st * ncls + ac[b]];
      if (st <= 1) return st == kAccept;
    }
    skip = 0;
    a += 16;
    v = vn;
  }
  return B.accept_end[R.ae_off + st] != 0;
}

// dfa_text over the text from t0 to the line's '\n' (a job window record,
// kJob*): the end is found in the 16 B loads the automaton steps over anyway
__device__ __forceinline__ uint32_t nl_mask16(const uint4 v) {
  const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t hb = nl_mask_word(wv[q]);
    m |= (((hb >> 7) & 1u) | ((hb >> 14) & 2u) | ((hb >> 21) & 4u) | ((hb >> 28) & 8u)) << (4 * q);
  }
  return m;
}
template <bool STAGED>
__device__ __forceinline__ bool dfa_line(const Bind &B, const DevRule &R, const uint16_t *tr, const uint8_t *ac,
                                         const uint32_t *acc, const uint8_t *__restrict__ buf, uint64_t n_buf, uint64_t t0,
                                         uint32_t st0) {
  const uint32_t ncls = R.ncls;
  uint32_t st = st0;
  uint64_t a = t0 & ~15ull;
  uint32_t skip = (uint32_t)(t0 - a);
  auto load16 = [&](uint64_t p) -> uint4 {
    if (p + 16 <= n_buf) return *reinterpret_cast<const uint4 *>(buf + p);
    uint32_t w[4];
    for (int k = 0; k < 4; ++k) {
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b) x |= (p + 4 * k + b < n_buf ? (uint32_t)buf[p + 4 * k + b] : 0x0Au) << (8 * b);
      w[k] = x;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  };
  uint4 v = load16(a);
  for (;;) {
    uint32_t nlm = nl_mask16(v) & ~((1u << skip) - 1u);
    const uint32_t aw = acc ? acc[st] : 0u;
    if ((aw >> 31) && !nlm) {
      // self-loop state: skip 16 B at a time up to an escape byte or the '\n'
      for (;;) {
        const uint32_t m = accel_mask(v, aw) & ~((1u << skip) - 1u);
        if (m || nlm) {
          const uint32_t f = (uint32_t)__ffs(m | nlm) - 1;
          skip = f;
          break;
        }
        a += 16;
        skip = 0;
        v = load16(a);
        nlm = nl_mask16(v);
      }
    } else if (aw >> 31) {
      const uint32_t m = (accel_mask(v, aw) | nlm) & ~((1u << skip) - 1u);
      skip = (uint32_t)__ffs(m) - 1;  // m != 0: nlm has a bit at or past skip
    }
    const uint32_t lim = nlm ? (uint32_t)__ffs(nlm) - 1 : 16u;  // bytes before the '\n'
    const uint4 vn = lim == 16u ? load16(a + 16) : make_uint4(0, 0, 0, 0);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) {
      if (k < skip || k >= lim) continue;
      const uint32_t b = (wv[k >> 2] >> (8 * (k & 3))) & 0xFF;
      if (b >= 0x80) {
        // non-ASCII: decode runes from here to the '\n' (Go's regexp steps by rune)
        uint64_t i = a + k, end = i;
        while (end < n_buf && buf[end] != '\n') ++end;
        while (i < end) {
          int w;
          const int32_t rune = decode_rune_hd(buf + i, (uint32_t)(end - i), &w);
          uint32_t c;
          if (rune < 0x80) c = ac[rune];
          else {
            const uint32_t *na = B.nonascii + 2 * R.na_off;
            uint32_t lo = 0, hi = R.n_na;
            while (hi - lo > 1) {
              const uint32_t m = (lo + hi) >> 1;
              if (na[2 * m] <= (uint32_t)rune) lo = m; else hi = m;
            }
            c = na[2 * lo + 1];
          }
          i += (uint32_t)w;
          st = tr[st * ncls + c];
          if (st <= 1) break;
        }
        return B.accept_end[R.ae_off + st] != 0;
      }
      st = tr[st * ncls + ac[b]];
      if (st <= 1) return st == kAccept;
    }
    if (lim < 16u) return B.accept_end[R.ae_off + st] != 0;
    skip = 0;
    a += 16;
    v = vn;
  }
}

// The windowed DFA jobs (kJob* records from k_lines2): one lane per job, the
// rule's transition rows staged in LDS when the block's jobs share a rule
// (jobs sorted by key; legacy jobs, keyed n_rules + rule, sort after them and
// are k_dfa_legacy's).  Each job reads its window word and the text from
// there to the line's '\n'; only a match reads the job's line.
__global__ __launch_bounds__(kBlock) void k_dfa(Bind B, const uint8_t *__restrict__ buf, uint64_t n_buf,
                                                const uint32_t *__restrict__ jkey, const uint32_t *__restrict__ jidx,
                                                const uint32_t *__restrict__ jline, const uint64_t *__restrict__ jrec, uint64_t n,
                                                Lines L) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_dfa[];
  uint16_t *s_tr = reinterpret_cast<uint16_t *>(s_dfa);
  uint32_t *s_acc = reinterpret_cast<uint32_t *>(s_dfa + ((B.dfa_tr * 2 + 15) & ~15u));
  uint8_t *s_ac = reinterpret_cast<uint8_t *>(s_acc + B.dfa_acc);
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x;
  if ((jkey[t0] & 0xFFFFFF) >= B.n_rules) return;  // legacy jobs only (they sort last)
  const uint64_t t = t0 + threadIdx.x;
  const uint64_t tl = t0 + blockDim.x - 1 < n ? t0 + blockDim.x - 1 : n - 1;
  const uint32_t r0 = jkey[t0] & 0xFFFFFF;
  const DevRule R0 = B.rules[r0];
  const bool uniform = (jkey[tl] & 0xFFFFFF) == r0;  // the whole block is r0's
  const bool staged = uniform && (uint32_t)R0.ncls * R0.n_states <= B.dfa_tr;
  if (staged) {
    const uint16_t *g = B.trans + R0.trans_off;
    for (uint32_t i = threadIdx.x; i < (uint32_t)R0.ncls * R0.n_states; i += blockDim.x) s_tr[i] = g[i];
    if (threadIdx.x < 128) s_ac[threadIdx.x] = B.ascii_cls[(size_t)r0 * 128 + threadIdx.x];
    if (R0.n_states <= B.dfa_acc)
      for (uint32_t i = threadIdx.x; i < R0.n_states; i += blockDim.x) s_acc[i] = B.accel[R0.ae_off + i];
  }
  __syncthreads();
  if (t >= n) return;
  const uint32_t key = jkey[t];
  const uint32_t r = key & 0xFFFFFF, pos = key >> 24;
  if (r >= B.n_rules) return;  // a legacy job
  const uint32_t slot = jidx[t];
  const uint64_t rec = jrec[slot];
  const uint64_t a = rec & kJobOffMask;
  bool m;
  if (staged) {
    const uint32_t *acc = R0.n_states <= B.dfa_acc ? s_acc : B.accel + R0.ae_off;
    m = dfa_line<true>(B, R0, s_tr, s_ac, acc, buf, n_buf, a, (rec & kJobSkipState) ? R0.skip_state : R0.start);
  } else {
    const DevRule R = B.rules[r];
    m = dfa_line<false>(B, R, B.trans + R.trans_off, B.ascii_cls + (size_t)r * 128, B.accel + R.ae_off, buf, n_buf, a,
                        (rec & kJobSkipState) ? R.skip_state : R.start);
  }
  if (!m) return;
  const uint64_t j = jline[slot];
  atomicOr(reinterpret_cast<unsigned long long *>(&L.mword(j, pos >> 6)), 1ull << (pos & 63));
  atomicAdd(reinterpret_cast<unsigned long long *>(L.counts + j), (1ull << 32) | ((rec & kJobNoCount) ? 0ull : 1ull));
}

// The legacy DFA jobs (keys n_rules + rule: kernels other than k_lines2, and
// k_lines2's NFA rules / seeks past overflowed slots / first-hit tables):
// the start is derived from the line's arrays (eq_certain, skip prefix,
// lead_start_seek), then dfa_text over rest.
__global__ __launch_bounds__(kBlock) void k_dfa_legacy(Bind B, const uint8_t *__restrict__ buf, uint64_t n_buf,
                                                       const uint64_t *__restrict__ nl, const uint32_t *__restrict__ jkey,
                                                       const uint32_t *__restrict__ jidx, const uint32_t *__restrict__ jline,
                                                       uint64_t n, Lines L) {
  __shared__ uint16_t s_tr[kDfaLdsEntries];
  __shared__ uint32_t s_acc[kDfaAccelLds];
  __shared__ uint8_t s_ac[128];
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x;
  const uint64_t t = t0 + threadIdx.x;
  const uint64_t tl = t0 + blockDim.x - 1 < n ? t0 + blockDim.x - 1 : n - 1;
  if ((jkey[tl] & 0xFFFFFF) < B.n_rules) return;  // windowed jobs only
  const uint32_t k0 = jkey[t0] & 0xFFFFFF;
  const uint32_t r0 = k0 >= B.n_rules ? k0 - B.n_rules : k0;
  const DevRule R0 = B.rules[r0];
  const bool uniform = k0 >= B.n_rules && (jkey[tl] & 0xFFFFFF) == k0;  // the whole block is r0's
  if (uniform && (R0.flags & kRuleNfa)) return;                        // k_nfa's
  const bool staged = uniform && (uint32_t)R0.ncls * R0.n_states <= kDfaLdsEntries;
  if (staged) {
    const uint16_t *g = B.trans + R0.trans_off;
    for (uint32_t i = threadIdx.x; i < (uint32_t)R0.ncls * R0.n_states; i += blockDim.x) s_tr[i] = g[i];
    if (threadIdx.x < 128) s_ac[threadIdx.x] = B.ascii_cls[(size_t)r0 * 128 + threadIdx.x];
    if (R0.n_states <= kDfaAccelLds)
      for (uint32_t i = threadIdx.x; i < R0.n_states; i += blockDim.x) s_acc[i] = B.accel[R0.ae_off + i];
  }
  __syncthreads();
  if (t >= n) return;
  const uint32_t key = jkey[t];
  const uint32_t rk = key & 0xFFFFFF, pos = key >> 24;
  if (rk < B.n_rules) return;  // a windowed job
  const uint32_t r = rk - B.n_rules;
  const uint64_t j = jline[jidx[t]];
  const uint64_t s = j ? nl[j - 1] + 1 : 0;
  const uint64_t rs = s + L.rest_off[j];
  const uint32_t rl = (uint32_t)(nl[j] - rs);
  bool m;
  if (!staged && (B.rules[r].flags & kRuleNfa)) return;  // k_nfa's (a mixed block)
  if ((staged ? R0.equiv : B.rules[r].equiv) && eq_certain(B, L, j, pos, rs)) {
    m = true;
  } else if (staged) {
    // anchored prefix literal already matched by k_lines: step in past it;
    // a lead rule's job starts at the first hit of its literals (every match
    // begins at one, regex_compiler.h pref_lead)
    const uint32_t sk = R0.skip_len && R0.skip_len <= rl ? R0.skip_len : 0u;
    const uint32_t st0 = (R0.lead & 1u) ? lead_start_seek(B, R0, L, buf, n_buf, j, pos, rs, rl) : 0u;
    const uint32_t *acc = R0.n_states <= kDfaAccelLds ? s_acc : B.accel + R0.ae_off;
    m = st0 ? dfa_text<true>(B, R0, s_tr, s_ac, acc, buf, n_buf, rs + st0, rl - st0, R0.start)
            : dfa_text<true>(B, R0, s_tr, s_ac, acc, buf, n_buf, rs + sk, rl - sk, sk ? R0.skip_state : R0.start);
  } else {
    const DevRule R = B.rules[r];
    const uint32_t sk = R.skip_len && R.skip_len <= rl ? R.skip_len : 0u;
    const uint32_t st0 = (R.lead & 1u) ? lead_start_seek(B, R, L, buf, n_buf, j, pos, rs, rl) : 0u;
    const uint32_t *acc = B.accel + R.ae_off;
    if (st0) m = dfa_text<false>(B, R, B.trans + R.trans_off, B.ascii_cls + (size_t)r * 128, acc, buf, n_buf, rs + st0,
                                 rl - st0, R.start);
    else m = dfa_text<false>(B, R, B.trans + R.trans_off, B.ascii_cls + (size_t)r * 128, acc, buf, n_buf, rs + sk, rl - sk,
                             sk ? R.skip_state : R.start);
  }
  if (!m) return;
  const int32_t hid = L.host_id[j];
  const uint32_t sc = hid >= 0 ? (uint32_t)hid : B.n_hosts;
  const bool no_count = (B.sc_skip[2 * sc + (pos >> 6)] >> (pos & 63)) & 1;
  atomicOr(reinterpret_cast<unsigned long long *>(&L.mword(j, pos >> 6)), 1ull << (pos & 63));
  atomicAdd(reinterpret_cast<unsigned long long *>(L.counts + j), (1ull << 32) | (no_count ? 0ull : 1ull));
}

// DFA jobs of one kRuleNfa rule (the sorted job range [j0, j1)): one job per
// lane, the rule's tables staged in LDS, WT-word state sets in VGPRs, text
// read 16 B at a time (a non-ASCII byte switches the rest of the text to rune
// decoding, as dfa_text does).
template <int WT>
__global__ __launch_bounds__(kBlock) void k_nfa(Bind B, uint32_t rule, const uint8_t *__restrict__ buf, uint64_t n_buf,
                                                const uint64_t *__restrict__ nl, const uint32_t *__restrict__ jkey,
                                                const uint32_t *__restrict__ jidx, const uint32_t *__restrict__ jline,
                                                uint64_t j0, uint64_t j1, Lines L) {
  uint64_t *s_b = reinterpret_cast<uint64_t *>(s_dyn);
  const DevRule R = B.rules[rule];
  const uint64_t *g = B.nfa + R.nfa_off;
  const uint32_t total = reinterpret_cast<const uint32_t *>(g)[7];
  for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) s_b[i] = g[i];
  __syncthreads();
  const uint64_t t = j0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= j1) return;
  const NfaLayout Ly = nfa_layout_of(reinterpret_cast<const uint32_t *>(s_b));
  const uint16_t *a16 = reinterpret_cast<const uint16_t *>(s_b + Ly.o_ascii);
  const uint32_t key = jkey[t], pos = key >> 24;
  const uint64_t j = jline[jidx ? jidx[t] : t];
  const uint64_t s = j ? nl[j - 1] + 1 : 0;
  const uint64_t end = nl[j];
  uint64_t t0 = s + L.rest_off[j];
  if (R.lead & 1u) t0 += lead_start(B, L, j, pos, t0, (uint32_t)(end - t0));  // from the first hit of its literals
  uint64_t D[WT];
#pragma unroll
  for (int w = 0; w < WT; ++w) D[w] = s_b[Ly.o_s0 + w];
  uint32_t ctx = 3;
  bool m = false, done = false;
  auto load16 = [&](uint64_t p) -> uint4 {
    if (p + 16 <= n_buf) return *reinterpret_cast<const uint4 *>(buf + p);
    uint32_t w4[4];
    for (int k = 0; k < 4; ++k) {
      uint32_t x = 0;
      for (int q = 0; q < 4; ++q) x |= (p + 4 * k + q < n_buf ? (uint32_t)buf[p + 4 * k + q] : 0u) << (8 * q);
      w4[k] = x;
    }
    return make_uint4(w4[0], w4[1], w4[2], w4[3]);
  };
  uint64_t a = t0 & ~15ull;
  uint32_t skip = (uint32_t)(t0 - a);
  uint64_t slow_at = end;  // first non-ASCII byte: runes from here on
  uint4 v = a < end ? load16(a) : make_uint4(0, 0, 0, 0);
  while (a < end && !done) {
    const uint4 vn = a + 16 < end ? load16(a + 16) : make_uint4(0, 0, 0, 0);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
    const uint32_t lim = end - a < 16 ? (uint32_t)(end - a) : 16u;
    for (uint32_t k = skip; k < lim; ++k) {
      const uint32_t by = (wv[k >> 2] >> (8 * (k & 3))) & 0xFF;
      if (by >= 0x80) { slow_at = a + k; done = true; break; }
      if (nfa_rune<WT, true>(s_b, Ly, D, a16[by], ctx)) { m = true; done = true; break; }
      if ((Ly.flags & kNfaAnchored) && nfa_at_s0<WT, true>(s_b, Ly, D)) { done = true; break; }
    }
    skip = 0;
    a += 16;
    v = vn;
  }
  if (!m && slow_at < end) {
    for (uint64_t i = slow_at; i < end;) {
      int w;
      const int32_t rune = decode_rune_hd(buf + i, (uint32_t)(end - i), &w);
      const uint32_t c = rune < 0x80 ? a16[rune] : nonascii_class(B, R, rune);
      i += (uint32_t)w;
      if (nfa_rune<WT, true>(s_b, Ly, D, c, ctx)) { m = true; break; }
      if ((Ly.flags & kNfaAnchored) && nfa_at_s0<WT, true>(s_b, Ly, D)) { slow_at = end; break; }
    }
    if (!m && slow_at != end) m = nfa_end<WT, true>(s_b, Ly, D, ctx);
  } else if (!m && !done) {
    m = nfa_end<WT, true>(s_b, Ly, D, ctx);
  }
  if (!m) return;
  const int32_t hid = L.host_id[j];
  const uint32_t sc = hid >= 0 ? (uint32_t)hid : B.n_hosts;
  const bool skp = (B.sc_skip[2 * sc + (pos >> 6)] >> (pos & 63)) & 1;
  atomicOr(reinterpret_cast<unsigned long long *>(&L.mword(j, pos >> 6)), 1ull << (pos & 63));
  atomicAdd(reinterpret_cast<unsigned long long *>(L.counts + j), (1ull << 32) | (skp ? 0ull : 1ull));
}

// Jobs of kRuleNfaWide rules (regex_compiler.h NfaWideLayout: past the
// per-lane NFA's 1024 positions, e.g. `(?s).*x.{600}y.{600}z`): one block per
// job, the W-word state in LDS (GLB = false) or in a per-block HBM scratch
// (patterns whose state does not fit).  Each thread owns a run of kw words;
// per rune (every thread decodes the same rune): assertion closures of the
// context into A (sparse target lists), the match check, Y = A & CM[c] with
// the groups of Y's positions marked, A = shift(Y & SH) | S0 (the carry from
// the previous thread's last word), then the marked groups' targets into A.
// Same steps as nfa_rune / nfa_wide_match_host.  jpos: RuleResult positions
// of the per-line fallback's jobs (null: position = key >> 24).
template <bool GLB>
__device__ __forceinline__ void wide_sync() {
  if (GLB) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (GLB) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

template <bool GLB>
__global__ __launch_bounds__(kBlock) void k_nfa_wide(Bind B, const uint8_t *__restrict__ buf, uint64_t n_buf,
                                                     const uint64_t *__restrict__ nl, const uint32_t *__restrict__ jkey,
                                                     const uint32_t *__restrict__ jidx, const uint32_t *__restrict__ jline,
                                                     const uint32_t *__restrict__ jpos,
                                                     uint64_t j0, uint64_t j1, Lines L, uint64_t *scratch,
                                                     uint64_t scratch_words) {
  __shared__ uint32_t s_flag;
  const uint32_t tid = threadIdx.x;
  for (uint64_t t = j0 + blockIdx.x; t < j1; t += gridDim.x) {
    const uint32_t key = jkey[t], rk = key & 0xFFFFFFu, r = rk >= B.n_rules ? rk - B.n_rules : rk;
    const uint32_t pos = jpos ? jpos[t] : key >> 24;
    const uint64_t j = jline[jidx ? jidx[t] : t];
    const DevRule R = B.rules[r];
    const uint64_t *b = B.nfa + R.nfa_off;
    const NfaWideLayout Ly = nfa_wide_layout_of(reinterpret_cast<const uint32_t *>(b));
    const uint32_t W = Ly.W, kw = (W + kBlock - 1) / kBlock, w0 = min(W, tid * kw), w1 = min(W, w0 + kw);
    const uint32_t gw = (Ly.ngroups + 31) / 32;
    uint64_t *A = GLB ? scratch + blockIdx.x * scratch_words : reinterpret_cast<uint64_t *>(s_dyn);
    uint64_t *Yb = A + W;
    uint32_t *gmark = reinterpret_cast<uint32_t *>(Yb + W);
    const uint64_t *s0 = b + Ly.o_s0, *sh = b + Ly.o_sh, *gall = b + Ly.o_gall, *am = b + Ly.o_am;
    const uint16_t *a16 = reinterpret_cast<const uint16_t *>(b + Ly.o_ascii);
    const uint8_t *cat = reinterpret_cast<const uint8_t *>(b + Ly.o_cat);
    const uint32_t *aux = reinterpret_cast<const uint32_t *>(b + Ly.o_aux);
    const uint32_t *goff = reinterpret_cast<const uint32_t *>(b + Ly.o_goff), *gtgt = reinterpret_cast<const uint32_t *>(b + Ly.o_gtgt);
    const uint32_t *aoff = reinterpret_cast<const uint32_t *>(b + Ly.o_aoff), *atgt = reinterpret_cast<const uint32_t *>(b + Ly.o_atgt);
    const uint32_t mw = Ly.match >> 6;
    const uint64_t mbit = 1ull << (Ly.match & 63);
    const bool owner = Ly.match != 0xFFFFFFFFu && mw >= w0 && mw < w1;
    for (uint32_t w = w0; w < w1; ++w) A[w] = s0[w];
    for (uint32_t i = tid; i < gw; i += kBlock) gmark[i] = 0;
    if (tid == 0) s_flag = 0;
    wide_sync<GLB>();
    auto cross = [&](uint32_t k) {  // A |= closures (context k) of the assertions in A
      for (uint32_t w = w0; w < w1; ++w)
        for (uint64_t m = A[w] & am[w]; m; m &= m - 1) {
          const uint32_t a = aux[w * 64u + (uint32_t)__builtin_ctzll(m)];
          for (uint32_t i = aoff[a * 16 + k]; i < aoff[a * 16 + k + 1]; ++i)
            atomicOr(reinterpret_cast<unsigned long long *>(&A[atgt[i] >> 6]), 1ull << (atgt[i] & 63));
        }
    };
    const uint64_t s = j ? nl[j - 1] + 1 : 0;
    const uint64_t end = nl[j];
    uint64_t i = s + L.rest_off[j];
    if ((R.lead & 1u) && !jpos) i += lead_start(B, L, j, pos, i, (uint32_t)(end - i));  // from the first hit of its literals
    uint32_t ctx = 3;
    bool m = false;
    while (i < end) {
      uint32_t c;
      const uint8_t by = buf[i];
      if (by < 0x80) { c = a16[by]; ++i; }
      else {
        int wd;
        const int32_t rune = decode_rune_hd(buf + i, (uint32_t)(end - i), &wd);
        c = nonascii_class(B, R, rune);
        i += (uint32_t)wd;
      }
      const uint32_t cc = (Ly.flags & kNfaAsserts) ? cat[c] : 0u;
      if (Ly.flags & kNfaAsserts) {
        cross(ctx * 4 + cc);
        wide_sync<GLB>();
        // matched before c (without assertions A is the D checked after the
        // previous rune); every read of s_flag came before the barrier above
        if (owner && (A[mw] & mbit)) s_flag = 1;
      }
      ctx = cc == 1 ? 1u : (cc == 2 ? 2u : 0u);
      const uint64_t *cm = b + Ly.o_cm + (uint64_t)c * W;
      for (uint32_t w = w0; w < w1; ++w) {
        const uint64_t y = A[w] & cm[w];
        Yb[w] = y;
        for (uint64_t g = y & gall[w]; g; g &= g - 1) {
          const uint32_t gid = aux[w * 64u + (uint32_t)__builtin_ctzll(g)];
          atomicOr(&gmark[gid >> 5], 1u << (gid & 31));
        }
      }
      wide_sync<GLB>();
      if (s_flag) { m = true; break; }
      for (uint32_t w = w0; w < w1; ++w)
        A[w] = ((Yb[w] & sh[w]) << 1) | (w ? (Yb[w - 1] & sh[w - 1]) >> 63 : 0ull) | s0[w];
      wide_sync<GLB>();
      for (uint32_t gi = tid; gi < gw; gi += kBlock) {
        uint32_t mm = gmark[gi];
        if (!mm) continue;
        gmark[gi] = 0;
        for (; mm; mm &= mm - 1) {
          const uint32_t g = gi * 32 + (uint32_t)__ffs(mm) - 1;
          for (uint32_t q = goff[g]; q < goff[g + 1]; ++q)
            atomicOr(reinterpret_cast<unsigned long long *>(&A[gtgt[q] >> 6]), 1ull << (gtgt[q] & 63));
        }
      }
      wide_sync<GLB>();
      if (owner && (A[mw] & mbit)) s_flag = 1;  // matched after c
      wide_sync<GLB>();
      if (s_flag) { m = true; break; }
    }
    if (!m) {  // end of text: the assertions once more with next category "end"
      if (Ly.flags & kNfaAsserts) cross(ctx * 4 + 3);
      wide_sync<GLB>();  // also: every read of s_flag in the loop came before this
      if (owner && (A[mw] & mbit)) s_flag = 1;
      wide_sync<GLB>();
      m = s_flag != 0;
    }
    if (m && tid == 0) {
      const int32_t hid = L.host_id[j];
      atomicOr(reinterpret_cast<unsigned long long *>(&L.mword(j, pos >> 6)), 1ull << (pos & 63));
      atomicAdd(reinterpret_cast<unsigned long long *>(L.counts + j), (1ull << 32) | (is_skip(B, r, hid) ? 0ull : 1ull));
    }
    wide_sync<GLB>();  // the next job reuses A / Yb / gmark / s_flag
  }
}

// first / one-past-last sorted job of every rule that has jobs
__global__ void k_rule_bounds(uint64_t n, const uint32_t *__restrict__ jkey, uint32_t *__restrict__ first,
                              uint32_t *__restrict__ last) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = jkey[i] & 0xFFFFFF;
  if (i == 0 || (jkey[i - 1] & 0xFFFFFF) != r) first[r] = (uint32_t)i;
  if (i + 1 == n || (jkey[i + 1] & 0xFFFFFF) != r) last[r] = (uint32_t)(i + 1);
}

// RuleResults (reference order) and rate-limit events from the per-line masks.
// Events carry their line, rule and result index; bounds[0] += lines with
// events, bounds[1] += their IP bytes (capacity of the IP table / arena),
// reduced per block (grid-stride; one atomic pair per block).
__global__ __launch_bounds__(kBlock) void k_emit(Bind B, uint64_t n_lines, Lines L, const uint64_t *__restrict__ offs,
                                                 uint64_t *__restrict__ res_seq, uint32_t *__restrict__ res_rule,
                                                 uint32_t *__restrict__ ev_el, uint32_t *__restrict__ ev_rule,
                                                 uint32_t *__restrict__ ev_res, unsigned long long *bounds, bool want_res) {
  // want_res: also the RuleResult arrays (res_seq, res_rule, ev_res), read only
  // when the caller copies the RuleResults out (BJX_COPY_RESULTS)
  __shared__ unsigned long long s_acc[2][kBlock / 64];
  unsigned long long has_ev = 0, ipb = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_lines; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t cnt = L.counts[j];
    if (cnt == 0) continue;
    uint64_t ro = offs[j] >> 32, eo = offs[j] & 0xFFFFFFFFull;
    const int32_t hid = L.host_id[j];
    uint32_t s_begin = 0, s_end = 0;
    if (hid >= 0) { s_begin = B.site_off[hid]; s_end = B.site_off[hid + 1]; }
    const uint32_t nsite = s_end - s_begin;
    const uint32_t napp = nsite + B.n_global;
    // HostsToSkip of the line's host by rule position (positions < 128; the
    // per-result binary search only past that)
    const uint32_t sc = hid >= 0 ? (uint32_t)hid : B.n_hosts;
    const uint64_t k0 = B.sc_skip[2 * sc], k1 = B.sc_skip[2 * sc + 1];
    for (uint32_t w = 0; w * 64 < napp; ++w) {
      uint64_t m = L.mword(j, w);
      while (m) {
        const uint32_t b = (uint32_t)__ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const uint32_t pos = w * 64 + b;
        const uint32_t r = pos < nsite ? B.site_rules[s_begin + pos] : B.global_rules[pos - nsite];
        const bool skip = pos < 128 ? (((pos < 64 ? k0 >> pos : k1 >> (pos - 64)) & 1) != 0) : is_skip(B, r, hid);
        if (want_res) {
          res_seq[ro] = (j << 16) | pos;
          res_rule[ro] = r | (skip ? 0x80000000u : 0u);
        }
        if (!skip) {
          ev_el[eo] = (uint32_t)j;
          ev_rule[eo] = r;
          if (want_res) ev_res[eo] = (uint32_t)ro;
          ++eo;
        }
        ++ro;
      }
    }
    if (cnt & 0xFFFFFFFFull) { ++has_ev; ipb += L.ip_len[j]; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    has_ev += __shfl_xor(has_ev, o);
    ipb += __shfl_xor(ipb, o);
  }
  if ((threadIdx.x & 63) == 0) { s_acc[0][threadIdx.x >> 6] = has_ev; s_acc[1][threadIdx.x >> 6] = ipb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a0 = 0, a1 = 0;
    for (int w = 0; w < kBlock / 64; ++w) { a0 += s_acc[0][w]; a1 += s_acc[1][w]; }
    if (a0) { atomicAdd(&bounds[0], a0); atomicAdd(&bounds[1], a1); }
  }
}

// --------------------------------------------------------------- state
//
// RegexRateLimitStates.Apply (rate_limit.go:37-78) for a batch of events, in
// four data-parallel steps (DESIGN.md "Rate limiting"):
//   k_ip_claim    one lane per event line: find the IP's slot (full byte
//                 compare against IPs of earlier batches) or claim a new one
//   k_ip_commit   one lane per event line: the first line of a new IP writes
//                 its bytes; other lines check theirs against it (a 64-bit
//                 hash collision inside the batch -> k_ip_collide, serial)
//   k_st_claim    one lane per event: (ip id, rule name) -> state slot, seenIp
//   radix sort by state slot (stable: reference order inside a slot)
//   k_apply       one lane per state slot run (runs staged in LDS per block
//                 of sorted records): the fixed-window automaton

__device__ __forceinline__ uint64_t line_start(const uint64_t *nl, uint64_t line) { return line ? nl[line - 1] + 1 : 0; }

__device__ __forceinline__ const uint8_t *ev_ip(const EvSrc &E, uint64_t i) {
  return E.bytes + (E.nl ? line_start(E.nl, i) + E.rest_off[i] - E.ip_len[i] - 1 : E.ip_pos[i]);
}
// hash_bytes of event line i's IP: a local line's IP of <= 15 bytes from its
// inline key (no hash is stored for it), else the stored hash
__device__ __forceinline__ uint64_t ev_hash(const EvSrc &E, uint64_t i, const uint4 &k16, uint32_t len) {
  const uint64_t h = E.nl && len <= 15 ? key16_hash(k16, len) : E.ip_hash[i];
  return E.hmask ? (h & E.hmask) | 1ull : h;
}
__device__ __forceinline__ bool ev_has(const EvSrc &E, uint64_t i) {
  return !E.counts || (E.counts[i] & 0xFFFFFFFFull) != 0;
}

constexpr uint32_t kNewIp = 0xFFFFFFFFu;   // el_id: IP created in this batch, id not known to this line
constexpr uint32_t kFirstIp = 0x80000000u; // el_id: this line is the first event line of a new IP

// Claim budgets: a launch may add at most `budget` entries to a table (keeps
// it under its load factor).  Claims are counted per shard of blocks
// (blockIdx % kClaimShards, counters on lines of their own), each shard
// holding budget / kClaimShards; past it the launch raises the overflow flag,
// every lane still running leaves, and the host rolls the claims back, grows
// the table and claims again.  One hot counter would serialise every claim.
constexpr uint32_t kClaimShards = 64;  // = one wave in k_fold_claims
constexpr uint32_t kShardBase = 16;    // counters[kShardBase + 16 * shard + {0: IP claims, 1: state claims}]
constexpr size_t kCounterBytes = (kShardBase + 16 * kClaimShards) * 8;

__device__ __forceinline__ unsigned long long *claim_shard(const State &S, uint32_t which) {
  return (unsigned long long *)&S.counters[kShardBase + 16 * (blockIdx.x % kClaimShards) + which];
}
__device__ __forceinline__ bool flag_set(const State &S, uint32_t f) {
  return __hip_atomic_load(&S.counters[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void raise_flag(const State &S, uint32_t f) {
  if (!flag_set(S, f)) atomicOr((unsigned long long *)&S.counters[f], 1ull);
}
// adds this wave's successful claims to the block's shard; over the shard's
// share -> overflow flag (all lanes of the wave call it)
__device__ __forceinline__ void count_claims(const State &S, uint32_t which, uint32_t ovf_flag, bool claimed, uint64_t shard_budget) {
  const uint64_t won = __ballot(claimed);
  if (won && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)won) - 1))
    if (atomicAdd(claim_shard(S, which), (unsigned long long)__popcll(won)) + __popcll(won) > shard_budget)
      raise_flag(S, ovf_flag);
}

// one event line -> its IP slot; true if this lane claimed a new slot
__device__ __forceinline__ bool ip_claim_line(const EvSrc &E, const State &S, uint32_t epoch, uint64_t i,
                                              uint32_t *__restrict__ el_slot, uint32_t *__restrict__ el_id,
                                              uint64_t shard_budget) {
  const uint32_t len = E.ip_len[i];
  const bool inl = len <= 15;
  // the inline key: the whole IP up to 15 bytes, else its first 15 bytes and
  // length (a slot whose key differs holds another IP; an equal one compares
  // the arena bytes)
  const uint4 k16 = E.ip16 ? E.ip16[i] : ip_key16_bytes(ev_ip(E, i), len);
  const uint64_t h = ev_hash(E, i, k16, len);
  uint64_t s = h & S.ip_mask;
  bool claimed = false;
  for (;;) {
    // the whole 32 B slot in one round trip: hash, id, born, key16.  A slot
    // claimed in this launch may read stale (hash 0 or born 0): the CAS below
    // decides the hash, and born 0 means claimed in this launch.  id and key16
    // of IPs from earlier batches are settled.  (Device-coherent sc1 loads of
    // hash and born, which spare a new IP's later lines their CAS, measured
    // slower: the cold cfg3 claim 46 -> 52 ms, the steady one 4.3 -> 5.5 ms.)
    const uint4 *sp = reinterpret_cast<const uint4 *>(&S.ip[s]);
    const uint4 q0 = sp[0], q1 = sp[1];
    uint64_t cur = ((uint64_t)q0.y << 32) | q0.x;
    if (cur == 0) {
      if (flag_set(S, 5)) return false;  // this launch is rolled back anyway
      if (__hip_atomic_load(claim_shard(S, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= shard_budget) {
        raise_flag(S, 5);
        return false;
      }
      cur = atomicCAS((unsigned long long *)&S.ip[s].hash, 0ull, (unsigned long long)h);
      if (cur == 0) {
        cur = h;
        claimed = true;
        __hip_atomic_store(&S.ip[s].born, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (cur == h) {
      // born: an earlier batch's epoch (stored before this launch, so every
      // lane sees it), or 0 / this epoch for a slot claimed in this launch (its
      // claimer stores the epoch after winning the hash): no atomic per line
      const uint32_t b = claimed ? epoch : q0.w;
      if (b == 0 || b == epoch) {  // created in this batch: identity checked by k_ip_commit
        // a hot new IP has every one of its lines here: read before the atomic,
        // so only lines that can still lower the first index contend for it
        // (a plain load: the index only falls, so a stale value at or below i
        // means the atomic would change nothing)
        if (S.ip_first[s] > (uint32_t)i) atomicMin(&S.ip_first[s], (uint32_t)i);
        el_slot[i] = (uint32_t)s;
        el_id[i] = kNewIp;
        return claimed;
      }
      // created by an earlier batch: short IPs compare inline, long ones in the arena
      const uint32_t id = q0.z;
      if (key16_eq(q1, k16) &&
          (inl || ((len < 255 || S.ip_len[id] == len) && ip_eq(S.arena + S.ip_off[id], ev_ip(E, i), len)))) {
        el_slot[i] = (uint32_t)s;
        el_id[i] = id;
        return claimed;
      }
    }
    s = (s + 1) & S.ip_mask;
  }
}

// exclusive prefix of v over the block and one atomicAdd of the block's total
// on ctr; returns ctr's old value + the prefix (every thread of the block
// calls it).  One atomic per block, not per wave: a single counter address
// takes about 88 atomics per microsecond, which made the per-wave form cost
// 3.5 ms (k_ip_claim's new-line list) and 7 ms (k_ip_commit's two counters)
// on a cold batch of 20M new IPs.
__device__ __forceinline__ uint64_t block_alloc(unsigned long long *ctr, uint64_t v) {
  __shared__ unsigned long long s_w[kBlock / 64 + 1];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  __syncthreads();  // a previous call's readers are done with s_w
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      const unsigned long long t = s_w[w];
      s_w[w] = tot;
      tot += t;
    }
    s_w[kBlock / 64] = tot ? atomicAdd(ctr, tot) : 0ull;
  }
  __syncthreads();
  return s_w[kBlock / 64] + s_w[wave] + (x - v);
}

// counters[4]: the event lines whose IP is new to the table (created in this
// batch), counted per block shard (claim_shard 2) and summed by k_fold_new.
// el_id of a line without events is 0 (k_ip_commit passes over every line).
__global__ __launch_bounds__(kBlock) void k_ip_claim(EvSrc E, State S, uint32_t epoch, uint32_t *__restrict__ el_slot,
                                                     uint32_t *__restrict__ el_id, uint64_t shard_budget) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool claimed = false, isnew = false;
  if (i < E.n && !flag_set(S, 5)) {
    if (ev_has(E, i)) {
      el_id[i] = 0;
      claimed = ip_claim_line(E, S, epoch, i, el_slot, el_id, shard_budget);
      isnew = el_id[i] == kNewIp;
    } else {
      el_id[i] = 0;
    }
  }
  count_claims(S, 0, 5, claimed, shard_budget);
  const uint64_t nn = __ballot(isnew);
  if (nn && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)nn) - 1))
    atomicAdd(claim_shard(S, 2), (unsigned long long)__popcll(nn));
}

// the shards' new-line counts -> counters[4] (one wave: lane = shard)
__global__ void k_fold_new(State S) {
  const uint32_t t = threadIdx.x;
  unsigned long long v = S.counters[kShardBase + 16 * t + 2];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if (t == 0) S.counters[4] = v;
}

// A new IP's first event line (ip_first of its slot) gets its id and arena
// bytes.  Ids and byte offsets come from a scan, not from atomics on one
// counter (a single address takes about 88 atomics per microsecond: a cold
// batch of 125M lines paid about 11 ms for one per block): k_ip_firsts counts
// each block's first lines and their bytes, an exclusive scan over the blocks
// gives each block its base, and k_ip_commit adds the in-block prefix.
__device__ __forceinline__ bool ip_first_line(const EvSrc &E, const State &S, const uint32_t *el_slot, const uint32_t *el_id,
                                              uint64_t i, uint32_t &len) {
  len = 0;
  if (i >= E.n || el_id[i] != kNewIp) return false;
  if (S.ip_first[el_slot[i]] != (uint32_t)i) return false;
  len = E.ip_len[i];
  return true;
}

// block sums of (a, b); valid in thread 0
__device__ __forceinline__ void block_sum2(uint64_t &a, uint64_t &b) {
  __shared__ unsigned long long s_a[kBlock / 64], s_b[kBlock / 64];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) { a += __shfl_xor(a, d); b += __shfl_xor(b, d); }
  if ((threadIdx.x & 63) == 0) { s_a[threadIdx.x >> 6] = a; s_b[threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int w = 1; w < kBlock / 64; ++w) { a += s_a[w]; b += s_b[w]; }
}

__global__ __launch_bounds__(kBlock) void k_ip_firsts(EvSrc E, State S, const uint32_t *__restrict__ el_slot,
                                                      const uint32_t *__restrict__ el_id, uint32_t *__restrict__ blk_n,
                                                      uint64_t *__restrict__ blk_b) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t len;
  const bool first = ip_first_line(E, S, el_slot, el_id, i, len);
  uint64_t a = first ? 1 : 0, b = len;
  block_sum2(a, b);
  if (threadIdx.x == 0) { blk_n[blockIdx.x] = (uint32_t)a; blk_b[blockIdx.x] = b; }
}

// exclusive prefix of v over the block (every thread calls it)
__device__ __forceinline__ uint64_t block_excl(uint64_t v) {
  __shared__ unsigned long long s_w[kBlock / 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  __syncthreads();  // a previous call's readers are done with s_w
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint64_t before = 0;
  for (uint32_t w = 0; w < wave; ++w) before += s_w[w];
  return before + x - v;
}

// every event line whose IP is new in this batch (el_id kNewIp): the first
// line of the IP writes its bytes, id and key; the others check theirs
// against it (a 64-bit hash collision inside the batch -> k_ip_collide, serial)
__global__ __launch_bounds__(kBlock) void k_ip_commit(EvSrc E, State S, const uint32_t *__restrict__ el_slot,
                                                      uint32_t *__restrict__ el_id, const uint32_t *__restrict__ blk_noff,
                                                      const uint64_t *__restrict__ blk_boff, uint32_t *__restrict__ coll) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t len;
  const bool first = ip_first_line(E, S, el_slot, el_id, i, len);
  const uint64_t id_in = block_excl(first ? 1 : 0);
  const uint64_t off_in = block_excl(len);
  const bool act = i < E.n && el_id[i] == kNewIp;
  if (first) {
    const uint32_t s = el_slot[i];
    const uint32_t id = (uint32_t)(S.counters[0] + blk_noff[blockIdx.x] + id_in);
    const uint64_t off = S.counters[1] + blk_boff[blockIdx.x] + off_in;
    const uint8_t *ip = ev_ip(E, i);
    for (uint32_t k = 0; k < len; ++k) S.arena[off + k] = ip[k];
    S.ip_off[id] = off;
    S.ip_len[id] = len;
    S.ip[s].id = id;
    S.ip[s].key16 = E.ip16 ? E.ip16[i] : ip_key16_bytes(ip, len);
    el_id[i] = id | kFirstIp;
  } else if (act) {
    // the same IP as its slot's first line?  IPs of up to 15 bytes by their
    // inline keys (bytes and length: exact), longer ones byte by byte
    const uint32_t f = S.ip_first[el_slot[i]];
    const uint32_t ln = E.ip_len[i], lf = E.ip_len[f];
    const bool same = lf == ln && (ln <= 15 && E.ip16 ? key16_eq(E.ip16[f], E.ip16[i]) : ip_eq(ev_ip(E, f), ev_ip(E, i), ln));
    if (!same) {
      const uint64_t k = atomicAdd((unsigned long long *)&S.counters[3], 1ull);
      coll[k] = (uint32_t)i;
    }
  }
}

// counters[0] / [1] += this batch's new IPs and their bytes (after k_ip_commit)
__global__ void k_ip_commit_total(State S, uint64_t nb, const uint32_t *__restrict__ blk_n, const uint32_t *__restrict__ blk_noff,
                                  const uint64_t *__restrict__ blk_b, const uint64_t *__restrict__ blk_boff) {
  if (blockIdx.x || threadIdx.x) return;
  S.counters[0] += (uint64_t)blk_noff[nb - 1] + blk_n[nb - 1];
  S.counters[1] += blk_boff[nb - 1] + blk_b[nb - 1];
}

// Lines whose IP differs from the first line of its slot (equal 64-bit hash):
// one thread, in line order, with full byte compares; each distinct string
// gets its own slot.  coll[] is sorted ascending.
__global__ void k_ip_collide(EvSrc E, State S, uint32_t epoch, uint32_t *__restrict__ el_slot,
                             uint32_t *__restrict__ el_id, const uint32_t *__restrict__ coll, uint64_t n_coll) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint64_t c = 0; c < n_coll; ++c) {
    const uint32_t i = coll[c];
    const uint32_t len = E.ip_len[i];
    const uint8_t *ip = ev_ip(E, i);
    const uint4 k16 = E.ip16 ? E.ip16[i] : ip_key16_bytes(ip, len);
    const uint64_t h = ev_hash(E, i, k16, len);
    uint64_t s = h & S.ip_mask;
    for (;;) {
      const uint64_t cur = S.ip[s].hash;
      if (cur == 0) {
        const uint32_t id = (uint32_t)S.counters[0]++;
        const uint64_t off = S.counters[1];
        S.counters[1] += len;
        for (uint32_t k = 0; k < len; ++k) S.arena[off + k] = ip[k];
        S.ip_off[id] = off;
        S.ip_len[id] = len;
        S.ip[s].hash = h;
        S.ip[s].id = id;
        S.ip[s].born = epoch;
        S.ip[s].key16 = k16;
        S.ip_first[s] = i;
        el_slot[i] = (uint32_t)s;
        el_id[i] = id | kFirstIp;
        break;
      }
      if (cur == h) {
        const uint32_t id = S.ip[s].id;
        if (S.ip_len[id] == len && bytes_eq(S.arena + S.ip_off[id], ip, len)) {
          el_slot[i] = (uint32_t)s;
          el_id[i] = id;
          break;
        }
      }
      s = (s + 1) & S.ip_mask;
    }
  }
}

// event k -> state slot and its sort record.  seenIp is false only for the
// first event of an IP created in this batch.
// A record whose timestamp the 12-B form cannot hold raises flag 8 (the host
// claims the batch again in the 16-B form).
template <typename R>
__device__ __forceinline__ bool st_claim_event(const EvSrc &E, uint64_t n_ev, uint64_t k, const uint32_t *__restrict__ ev_el,
                                               const uint32_t *__restrict__ ev_rule, const uint32_t *__restrict__ el_slot,
                                               const uint32_t *__restrict__ el_id, const DevRule *__restrict__ rules,
                                               const State &S, uint32_t *__restrict__ ev_st, R *__restrict__ ev_rec,
                                               int64_t base, uint64_t shard_budget) {
  const uint32_t i = ev_el[k];
  const uint32_t r = ev_rule[k];
  uint32_t id = el_id[i];
  const bool first = id != kNewIp && (id & kFirstIp) && (k == 0 || ev_el[k - 1] != i);
  id = id == kNewIp ? S.ip[el_slot[i]].id : (id & ~kFirstIp);
  const uint32_t nm = rules[r].name_id;
  const uint64_t key = ((uint64_t)(id + 1) << 24) | nm;
  const bool hot = nm == S.hot_name && id < S.ip_st_cap;
  const uint32_t c = hot ? S.ip_st[id] : kNone;
  uint64_t q = c;
  bool claimed = false;
  if (c == kNone) {
    q = mix64(key) & S.st_mask;
    for (;;) {
      uint64_t cur = S.st[q].key;
      if (cur == 0) {
        if (flag_set(S, 7)) return false;  // see k_ip_claim
        if (__hip_atomic_load(claim_shard(S, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= shard_budget) {
          raise_flag(S, 7);
          return false;
        }
        cur = atomicCAS((unsigned long long *)&S.st[q].key, 0ull, (unsigned long long)key);
        if (cur == 0) { claimed = true; break; }
      }
      if (cur == key) break;
      q = (q + 1) & S.st_mask;
    }
    if (hot) S.ip_st[id] = (uint32_t)q;
  }
  ev_st[k] = (uint32_t)q;
  const int64_t ts = E.ts[i];
  if (!R::fits(ts, base)) raise_flag(S, 8);
  ev_rec[k] = R::make(ts, r, first, (uint32_t)k, base);
  return claimed;
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_st_claim(EvSrc E, uint64_t n_ev, const uint32_t *__restrict__ ev_el,
                                                     const uint32_t *__restrict__ ev_rule, const uint32_t *__restrict__ el_slot,
                                                     const uint32_t *__restrict__ el_id, const DevRule *__restrict__ rules,
                                                     State S, uint32_t *__restrict__ ev_st, R *__restrict__ ev_rec,
                                                     int64_t base, uint64_t shard_budget) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool claimed = false;
  if (k < n_ev && !flag_set(S, 7)) claimed = st_claim_event(E, n_ev, k, ev_el, ev_rule, el_slot, el_id, rules, S, ev_st, ev_rec,
                                                            base, shard_budget);
  count_claims(S, 1, 7, claimed, shard_budget);
}

// state slots claimed by the last k_st_claim -> table load counters[2]; shards cleared
__global__ void k_fold_claims(State S) {
  const uint32_t t = threadIdx.x;  // one wave: lane = shard
  unsigned long long v = S.counters[kShardBase + 16 * t + 1];
  S.counters[kShardBase + 16 * t] = 0;
  S.counters[kShardBase + 16 * t + 1] = 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if (t == 0) S.counters[2] += v;
}

// The fixed-window automaton of one (ip, rule name) state over its events in
// reference order (records sorted by slot, stable).  A block takes kApplyChunk
// consecutive sorted records, loaded coalesced into LDS with their slots; each
// run that STARTS in the chunk goes to one lane (long runs to the first lanes,
// so short-run waves finish early), which walks it from LDS.  The one run that
// continues past the chunk end is listed for k_long_runs, which applies it
// from its head.  Records before the chunk's first run head belong to the
// previous block's run.  out_sorted[u] = outcome of record u in
// sorted order: bit0 seenIp, bits1-2 MatchType, bit3 Exceeded, bit7 valid.
constexpr uint32_t kApplyChunk = 2048;

template <typename R>
__device__ __forceinline__ uint8_t apply_step(const R &v, int64_t base, const DevRule *__restrict__ rules, uint32_t &pr,
                                              int64_t &interval, int64_t &limit, bool &valid, int64_t &hits, int64_t &start) {
  const uint32_t r = v.rule_id();
  const bool seen = v.seen();
  const int64_t ts = v.time(base);
  if (r != pr) { pr = r; interval = rules[r].interval_ns; limit = rules[r].hits; }  // rules sharing a name share the state
  uint8_t mt;
  if (!valid) { hits = 1; start = ts; mt = BJX_FIRST_TIME; valid = true; }
  else if (go_sub(ts, start) > interval) { mt = BJX_OUTSIDE_INTERVAL; hits = 1; start = ts; }
  else { mt = BJX_INSIDE_INTERVAL; ++hits; }
  const bool ex = hits > limit;
  if (ex) hits = 0;
  return (uint8_t)(0x80 | (seen ? 1 : 0) | (mt << 1) | (ex ? 8 : 0));
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_apply(uint64_t n_ev, const uint32_t *__restrict__ key, const R *__restrict__ rec,
                                                  int64_t tbase, const DevRule *__restrict__ rules, StSlot *__restrict__ st,
                                                  uint8_t *__restrict__ out_sorted, uint64_t *__restrict__ long_heads,
                                                  unsigned long long *__restrict__ n_long, uint32_t *__restrict__ wcnt) {
  constexpr uint32_t kPer = kApplyChunk / kBlock;  // positions per thread for the head scan
  constexpr uint32_t kLongRun = 8;                 // runs at least this long go to the first lanes
  __shared__ R s_rec[kApplyChunk];
  __shared__ uint32_t s_key[kApplyChunk + 1];  // s_key[i + 1] = slot of record i; s_key[0] = slot before the chunk
  __shared__ uint8_t s_out[kApplyChunk];
  __shared__ uint16_t s_head[kApplyChunk];  // run heads in position order
  __shared__ uint16_t s_ord[kApplyChunk];   // run indices: long runs from the front, short ones from the back
  __shared__ uint32_t s_wsum[kBlock / 64], s_front, s_back, s_cont;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t u0 = (uint64_t)blockIdx.x * kApplyChunk;
  const uint32_t n = (uint32_t)min<uint64_t>(kApplyChunk, n_ev - u0);
  for (uint32_t i = tid; i < n; i += kBlock) {
    s_rec[i] = rec[u0 + i];
    s_key[i + 1] = key[u0 + i];
  }
  if (tid == 0) {
    s_key[0] = u0 ? key[u0 - 1] : 0xFFFFFFFFu;
    s_cont = u0 + n < n_ev && key[u0 + n] == key[u0 + n - 1];  // the last run goes on past the chunk
    s_front = 0;
    s_back = 0;
  }
  __syncthreads();
  // run heads, compacted in position order (block scan of per-thread counts)
  uint32_t fl = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = tid * kPer + k;
    if (i < n && s_key[i + 1] != s_key[i]) fl |= 1u << k;
  }
  const uint32_t cnt = __popc(fl);
  uint32_t x = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  uint32_t base = x - cnt, nh = 0;
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    if (w < wave) base += s_wsum[w];
    nh += s_wsum[w];
  }
  for (uint32_t k = 0; fl; ++k, fl >>= 1)
    if (fl & 1) s_head[base++] = (uint16_t)(tid * kPer + k);
  __syncthreads();
  // lanes take runs longest-first (roughly): a wave lasts as long as its longest run
  for (uint32_t h = tid; h < nh; h += kBlock) {
    const uint32_t len = (h + 1 < nh ? s_head[h + 1] : n) - s_head[h];
    if (len >= kLongRun || (h + 1 == nh && s_cont)) s_ord[atomicAdd(&s_front, 1u)] = (uint16_t)h;
    else s_ord[nh - 1 - atomicAdd(&s_back, 1u)] = (uint16_t)h;
  }
  __syncthreads();
  for (uint32_t k = tid; k < nh; k += kBlock) {
    const uint32_t h = s_ord[k];
    const uint32_t b = s_head[h], e = h + 1 < nh ? s_head[h + 1] : n;
    const uint32_t q = s_key[b + 1];
    const StSlot cur = st[q];
    bool valid = cur.valid != 0;
    int64_t hits = cur.hits, start = cur.start, interval = 0, limit = 0;
    uint32_t pr = 0xFFFFFFFFu;
    if (h + 1 == nh && s_cont) {  // continues past the chunk: k_long_runs applies it from its head
      long_heads[atomicAdd(n_long, 1ull)] = u0 + b;
      continue;
    }
    R v = s_rec[b];
    for (uint32_t u = b; u < e; ++u) {
      R nx;
      if (u + 1 < e) nx = s_rec[u + 1];  // next record in flight while this one is applied
      s_out[u] = apply_step(v, tbase, rules, pr, interval, limit, valid, hits, start);
      v = nx;
    }
    st[q].hits = hits;
    st[q].start = start;
    st[q].valid = 1;
  }
  __syncthreads();
  // records before the first head belong to the previous block's run, those
  // of a continuing last run to k_long_*: each outcome has exactly one writer
  const uint32_t s_lo = nh ? s_head[0] : n, s_hi = nh && s_cont ? s_head[nh - 1] : n;
  for (uint32_t i = s_lo + tid; i < s_hi; i += kBlock) {
    out_sorted[u0 + i] = s_out[i];
    if (wcnt) atomicAdd(&wcnt[u0 + i], 1u);
  }
}

// ---- Two-level grouping (round 5).  The global radix sort orders the events
// by the state slot's high kBucketBits bits only (two onesweep passes instead of
// four for a 2^28-slot table); each bucket of 2^L slots then goes to one block
// (k_bucket_apply), which ranks its events by the slot's low L bits in LDS with
// a stable block radix sort and runs Apply over each slot's events as k_apply
// does.  A slot's events never leave its bucket, so no run crosses blocks (no
// k_long_* pass).  Buckets of more than kBucketCap events (hot keys) are listed;
// their events alone go through the full sort + k_apply + k_long_* path.
// out_sorted stays indexed by the position in the (bucket-)sorted array, as
// k_apply's is, so the trip and outcome kernels after it are unchanged.
constexpr int kBucketBits = 16;
constexpr uint32_t kBucketItems = 16;
constexpr uint32_t kBucketCap = kBlock * kBucketItems;  // 4096 events

// bstart[b] = first sorted position whose bucket (key >> L) is >= b, b <= nb
__global__ __launch_bounds__(kBlock) void k_bucket_bounds(uint64_t n_ev, const uint32_t *__restrict__ key, uint32_t L,
                                                          uint32_t nb, uint32_t *__restrict__ bstart) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n_ev) return;
  const uint32_t b = i < n_ev ? key[i] >> L : nb;
  const uint32_t lo = i ? (key[i - 1] >> L) + 1 : 0u;
  for (uint32_t x = lo; x <= b; ++x) bstart[x] = (uint32_t)i;
}

// One bucket per block.  The low key bits are ranked by a stable block radix
// sort of the bucket's (low bits << 12 | position) words on bits [12, 12 + L):
// the position rides in the key's low bits, so the sort moves one word per
// item and no value array; padding ranks take the largest low key and come
// last (they sit after every real record in the sort's input order, which it
// keeps for equal keys).  Run heads are compacted
// in rank order and taken longest first, as in k_apply; a lane walks its run
// through the rank -> position table, loading each record from the bucket's
// few KB of HBM / L2, the next one in flight while the current one is applied.
// (Gathering the records into LDS in rank order first, 16 independent loads
// per thread, measured slower: 6.8 against 6.1 ms per cfg3 batch, at two blocks
// per CU instead of four.)
template <typename R>
__global__ __launch_bounds__(kBlock) void k_bucket_apply(const uint32_t *__restrict__ key, const R *__restrict__ rec,
                                                         const uint32_t *__restrict__ bstart, uint32_t L, int64_t tbase,
                                                         const DevRule *__restrict__ rules, StSlot *__restrict__ st,
                                                         uint8_t *__restrict__ out_sorted, uint32_t *__restrict__ big,
                                                         unsigned long long *__restrict__ n_big, uint32_t *__restrict__ wcnt) {
  using Sort = hipcub::BlockRadixSort<uint32_t, kBlock, kBucketItems>;
  static_assert(kBucketCap <= 4096, "positions ride in 12 key bits");
  constexpr uint32_t kLongRun = 8;
  __shared__ union {
    typename Sort::TempStorage sort;
    uint32_t lk[kBucketCap];  // low key bits in position order (before the sort)
    uint16_t ho[2 * kBucketCap];  // run heads in rank order, run order (after the sort)
  } s_u;
  __shared__ uint16_t s_lk[kBucketCap];    // low key bits in rank order
  __shared__ uint16_t s_perm[kBucketCap];  // rank -> position
  uint16_t *const s_head = s_u.ho;
  uint16_t *const s_ord = s_u.ho + kBucketCap;  // run indices, long runs first
  __shared__ uint8_t s_out[kBucketCap];                     // by position
  __shared__ uint32_t s_wsum[kBlock / 64], s_front, s_back;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t bk = blockIdx.x, u0 = bstart[bk], n = bstart[bk + 1] - u0;
  if (n == 0) return;
  if (n > kBucketCap) {
    if (tid == 0) big[atomicAdd(n_big, 1ull)] = bk;
    return;
  }
  const uint32_t mask = (1u << L) - 1u;
  for (uint32_t i = tid; i < n; i += kBlock) s_u.lk[i] = key[u0 + i] & mask;
  if (tid == 0) { s_front = 0; s_back = 0; }
  __syncthreads();
  uint32_t k[kBucketItems];
#pragma unroll
  for (uint32_t j = 0; j < kBucketItems; ++j) {
    const uint32_t i = tid * kBucketItems + j;  // blocked: the sort is stable in this order
    k[j] = ((i < n ? s_u.lk[i] : mask) << 12) | i;
  }
  __syncthreads();
  Sort(s_u.sort).SortBlockedToStriped(k, 12, 12 + (int)L);
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kBucketItems; ++j) {
    const uint32_t r = j * kBlock + tid;
    s_lk[r] = (uint16_t)(k[j] >> 12);
    s_perm[r] = (uint16_t)(k[j] & 0xFFFu);
  }
  __syncthreads();
  // run heads, compacted in rank order (block scan of per-thread counts)
  uint32_t fl = 0;
#pragma unroll
  for (uint32_t j = 0; j < kBucketItems; ++j) {
    const uint32_t i = tid * kBucketItems + j;
    if (i < n && (i == 0 || s_lk[i] != s_lk[i - 1])) fl |= 1u << j;
  }
  const uint32_t cnt = __popc(fl);
  uint32_t x = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  uint32_t base = x - cnt, nh = 0;
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    if (w < wave) base += s_wsum[w];
    nh += s_wsum[w];
  }
  for (uint32_t j = 0; fl; ++j, fl >>= 1)
    if (fl & 1) s_head[base++] = (uint16_t)(tid * kBucketItems + j);
  __syncthreads();
  for (uint32_t h = tid; h < nh; h += kBlock) {
    const uint32_t len = (h + 1 < nh ? s_head[h + 1] : n) - s_head[h];
    if (len >= kLongRun) s_ord[atomicAdd(&s_front, 1u)] = (uint16_t)h;
    else s_ord[nh - 1 - atomicAdd(&s_back, 1u)] = (uint16_t)h;
  }
  __syncthreads();
  const uint32_t qb = bk << L;
  for (uint32_t t = tid; t < nh; t += kBlock) {
    const uint32_t h = s_ord[t];
    const uint32_t b = s_head[h], e = h + 1 < nh ? s_head[h + 1] : n;
    const uint32_t q = qb | s_lk[b];
    const StSlot cur = st[q];
    bool valid = cur.valid != 0;
    int64_t hits = cur.hits, start = cur.start, interval = 0, limit = 0;
    uint32_t pr = 0xFFFFFFFFu;
    uint32_t p = s_perm[b];
    R rv = rec[u0 + p];
    for (uint32_t u = b; u < e; ++u) {
      R nx;
      uint32_t pn = 0;
      if (u + 1 < e) { pn = s_perm[u + 1]; nx = rec[u0 + pn]; }  // next record in flight while this one is applied
      s_out[p] = apply_step(rv, tbase, rules, pr, interval, limit, valid, hits, start);
      if (wcnt) atomicAdd(&wcnt[u0 + p], 1u);  // BJX_CHECK: writes per sorted position
      rv = nx;
      p = pn;
    }
    st[q].hits = hits;
    st[q].start = start;
    st[q].valid = 1;
  }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kBlock) out_sorted[u0 + i] = s_out[i];
}

// the events of the oversized buckets: keys and sorted positions; one thread
// per event, its segment ({source position, events, destination}) by bisection
__global__ __launch_bounds__(kBlock) void k_big_gather(const uint4 *__restrict__ seg, uint32_t n_seg, uint64_t total,
                                                       const uint32_t *__restrict__ key, uint32_t *__restrict__ ko,
                                                       uint32_t *__restrict__ po) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  uint32_t lo = 0, hi = n_seg - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (seg[mid].z <= i) lo = mid;
    else hi = mid - 1;
  }
  const uint4 s = seg[lo];
  const uint32_t src = s.x + (uint32_t)(i - s.z);
  ko[i] = key[src];
  po[i] = src;
}

template <typename R>
__global__ __launch_bounds__(kBlock) void k_big_recs(uint64_t n, const uint32_t *__restrict__ pos, const R *__restrict__ rec,
                                                     R *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = rec[pos[i]];
}

// (BJX_CHECK: wsrc[i] = writes of o[i] by the full-sort apply, carried to the
// sorted position it lands on, so a position counts exactly once only when its
// outcome was written once there and copied once here)
__global__ __launch_bounds__(kBlock) void k_big_outs(uint64_t n, const uint32_t *__restrict__ pos, const uint8_t *__restrict__ o,
                                                     uint8_t *__restrict__ out_sorted, const uint32_t *__restrict__ wsrc,
                                                     uint32_t *__restrict__ wcnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out_sorted[pos[i]] = o[i];
  if (wcnt) atomicAdd(&wcnt[pos[i]], wsrc[i]);
}

// One (ip, rule name) state whose sorted run crosses a k_apply chunk (hot
// keys: a DDoS IP's run can hold a large share of the batch).
// One block per run, from its head:
//   * the run end and, over the run, whether every event has the same rule
//     interval / limit and timestamps never decrease (block reductions);
//   * if so, the fixed windows of Apply (rate_limit.go:37-78) are found one
//     after another by a block-parallel search (each round samples kBlock
//     timestamps, so a window of w events costs log_kBlock(w) rounds), and
//     every event's outcome follows in closed form: the e-th counted hit of a
//     window that starts with h0 hits is Exceeded iff (h0 + e) % (limit + 1)
//     == 0 (every hit when limit < 0), and the hits after it are that residue;
//   * otherwise (mixed limits, timestamps out of order) thread 0 applies the
//     events one by one, as k_apply's lanes do.
__device__ __forceinline__ uint32_t block_min_u32(uint32_t v, uint32_t *s_red) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t m = s_red[0];
  for (uint32_t w = 1; w < kBlock / 64; ++w) m = min(m, s_red[w]);
  return m;
}

// smallest i in [lo, hi) with pred(i) (pred monotone: false ... true), else hi
template <typename P>
__device__ uint64_t block_first(uint64_t lo, uint64_t hi, P pred, uint32_t *s_red) {
  while (lo < hi) {
    const uint64_t stride = search_stride(lo, hi, kBlock);
    const uint64_t p = lo + (uint64_t)threadIdx.x * stride;
    const bool ok = p < hi && pred(p);
    const uint32_t f = block_min_u32(ok ? threadIdx.x : (uint32_t)kBlock, s_red);
    search_narrow(lo, hi, stride, f, kBlock);  // uniform across the block
  }
  return hi;
}

constexpr uint64_t kLongSerial = 512;  // runs up to this long: thread 0 walks them

// Per crossing run (k_apply's long_heads), k_long_* below keep, in LongRuns:
struct LongRuns {
  const uint64_t *head;  // first sorted record of the run
  uint64_t *end;         // one past its last record
  uint64_t *off;         // exclusive scan of the run lengths (flattened event index)
  int64_t *t0;           // start of the first window (the stored window when the head continues it)
  int64_t *h0;           // hits already in that window
  uint32_t *flags;       // bit0: head continues the stored window; bits1-2: MatchType of the head otherwise;
                         // bit3: serial (mixed limits or decreasing timestamps); bit4: short (serial)
  uint64_t *win;         // window start records, off[r] ... off[r] + nwin[r]
  uint32_t *nwin;
  uint64_t n;
  uint32_t *wcnt;        // BJX_CHECK: writes per sorted outcome (null otherwise)
};

// 1. run end (block-parallel search), the stored state and the first window
template <typename Rec>
__global__ __launch_bounds__(kBlock) void k_long_ends(uint64_t n_ev, const uint32_t *__restrict__ key,
                                                      const Rec *__restrict__ rec, int64_t base, const StSlot *__restrict__ st,
                                                      const DevRule *__restrict__ rules, LongRuns R, uint64_t *__restrict__ len) {
  __shared__ uint32_t s_red[kBlock / 64];
  const uint64_t r = blockIdx.x;
  const uint64_t head = R.head[r];
  const uint32_t q = key[head];
  const uint64_t end = block_first(head + 1, n_ev, [&](uint64_t i) { return key[i] != q; }, s_red);
  if (threadIdx.x != 0) return;
  R.end[r] = end;
  len[r] = end - head;
  const StSlot cur = st[q];
  const int64_t I = rules[rec[head].rule_id()].interval_ns;
  const int64_t ts = rec[head].time(base);
  const bool valid = cur.valid != 0;
  const bool cont = valid && go_sub(ts, cur.start) <= I;
  R.t0[r] = cont ? cur.start : ts;
  R.h0[r] = cont ? cur.hits : 0;
  R.flags[r] = (cont ? 1u : 0u) | ((uint32_t)(valid ? BJX_OUTSIDE_INTERVAL : BJX_FIRST_TIME) << 1) |
               (end - head <= kLongSerial ? 16u : 0u);
}

__device__ __forceinline__ uint64_t long_run_of(const LongRuns &R, uint64_t k) {
  uint64_t lo = 0, hi = R.n;  // last r with off[r] <= k
  while (hi - lo > 1) {
    const uint64_t m = (lo + hi) >> 1;
    if (R.off[m] <= k) lo = m; else hi = m;
  }
  return lo;
}

// 2. every record of every long run, in parallel: same interval / limit as the
// head's rule and timestamps that never decrease, or the run is applied serially
template <typename Rec>
__global__ __launch_bounds__(kBlock) void k_long_check(uint64_t total, const Rec *__restrict__ rec, int64_t base,
                                                       const DevRule *__restrict__ rules, LongRuns R) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= total) return;
  const uint64_t r = long_run_of(R, k);
  const uint64_t head = R.head[r], i = head + (k - R.off[r]);
  if (i == head) return;
  const uint32_t r0 = rec[head].rule_id(), ri = rec[i].rule_id();
  bool bad = rec[i].time(base) < rec[i - 1].time(base);
  if (ri != r0) bad = bad || rules[ri].interval_ns != rules[r0].interval_ns || rules[ri].hits != rules[r0].hits;
  if (bad && !(__hip_atomic_load(&R.flags[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8u)) atomicOr(&R.flags[r], 8u);
}

// 3. per run: the serial walk (short or irregular runs), else the window
// starts one after another (block-parallel search per window) and the final
// state in closed form
template <typename Rec>
__global__ __launch_bounds__(kBlock) void k_long_windows(const uint32_t *__restrict__ key, const Rec *__restrict__ rec,
                                                         int64_t base, const DevRule *__restrict__ rules, StSlot *__restrict__ st,
                                                         uint8_t *__restrict__ out_sorted, LongRuns R) {
  __shared__ uint32_t s_red[kBlock / 64];
  const uint32_t tid = threadIdx.x;
  const uint64_t r = blockIdx.x;
  const uint64_t head = R.head[r], end = R.end[r];
  const uint32_t q = key[head];
  const uint32_t fl = R.flags[r];
  if (fl & 24u) {
    if (tid == 0) {
      const StSlot cur = st[q];
      bool valid = cur.valid != 0;
      int64_t hits = cur.hits, start = cur.start, interval = 0, limit = 0;
      uint32_t pr = 0xFFFFFFFFu;
      for (uint64_t i = head; i < end; ++i) {
        out_sorted[i] = apply_step(rec[i], base, rules, pr, interval, limit, valid, hits, start);
        if (R.wcnt) atomicAdd(&R.wcnt[i], 1u);
      }
      st[q].hits = hits;
      st[q].start = start;
      st[q].valid = 1;
      R.nwin[r] = 0;
    }
    return;
  }
  const uint32_t r0 = rec[head].rule_id();
  const int64_t I = rules[r0].interval_ns, Lim = rules[r0].hits;
  uint64_t *win = R.win + R.off[r];
  uint32_t nw = 0;
  uint64_t a = head;
  int64_t T = R.t0[r], h0 = R.h0[r];
  for (;;) {
    if (tid == 0) win[nw] = a;
    ++nw;
    const int64_t Tw = T;
    const uint64_t b = block_first(a + 1, end, [&](uint64_t i) { return go_sub(rec[i].time(base), Tw) > I; }, s_red);
    if (b >= end) {
      if (tid == 0) {
        const int64_t e = (int64_t)(b - a);
        int64_t hits;
        if (Lim < 0) hits = 0;
        else if (h0 > Lim) hits = (e - 1) % (Lim + 1);
        else hits = (h0 + e) % (Lim + 1);
        st[q].hits = hits;
        st[q].start = Tw;
        st[q].valid = 1;
        R.nwin[r] = nw;
      }
      return;
    }
    a = b;
    T = rec[b].time(base);
    h0 = 0;
  }
}

// 4. every record of the windowed runs, in parallel: its window (binary
// search over the run's window starts) and the closed-form outcome
template <typename Rec>
__global__ __launch_bounds__(kBlock) void k_long_fill(uint64_t total, const Rec *__restrict__ rec,
                                                      const DevRule *__restrict__ rules, uint8_t *__restrict__ out_sorted,
                                                      LongRuns R) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= total) return;
  const uint64_t r = long_run_of(R, k);
  const uint32_t fl = R.flags[r];
  if (fl & 24u) return;  // applied serially
  const uint64_t head = R.head[r], i = head + (k - R.off[r]);
  const uint64_t *win = R.win + R.off[r];
  uint32_t lo = 0, hi = R.nwin[r];  // last window starting at or before i
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (win[m] <= i) lo = m; else hi = m;
  }
  const uint32_t r0 = rec[head].rule_id();
  const int64_t Lim = rules[r0].hits;
  const bool first_win = lo == 0, cont = first_win && (fl & 1u);
  const int64_t h0 = first_win ? R.h0[r] : 0;
  const uint64_t a = win[lo];
  const int64_t e = (int64_t)(i - a) + 1;
  bool ex;
  if (Lim < 0) ex = true;
  else if (h0 > Lim) ex = e == 1 || (e - 1) % (Lim + 1) == 0;
  else ex = (h0 + e) % (Lim + 1) == 0;
  const uint8_t first_mt = first_win ? (uint8_t)((fl >> 1) & 3u) : (uint8_t)BJX_OUTSIDE_INTERVAL;
  const uint8_t mt = (!cont && i == a) ? first_mt : (uint8_t)BJX_INSIDE_INTERVAL;
  const bool seen = rec[i].seen();
  out_sorted[i] = (uint8_t)(0x80 | (seen ? 1 : 0) | (mt << 1) | (ex ? 8 : 0));
  if (R.wcnt) atomicAdd(&R.wcnt[i], 1u);
}

// ---- BJX_CHECK=1 (debugging aid): invariants of the rate-limit stage
__device__ __forceinline__ uint32_t ev_line_id(const State &S, const uint32_t *el_slot, const uint32_t *el_id, uint64_t i) {
  const uint32_t id = el_id[i];
  return id == kNewIp ? S.ip[el_slot[i]].id : (id & ~kFirstIp);
}
// every event line's IP id names the line's IP bytes; every event's state
// slot holds (that id, its rule's name); every sorted outcome was written by
// exactly one writer (wcnt), seenIp false only with FirstTime, and the sorted
// records' event indices form a permutation (pc: k_check_count over EvRec.ev)
__global__ void k_check_rl(EvSrc E, uint64_t n_ev, const uint32_t *__restrict__ ev_el, const uint32_t *__restrict__ ev_rule,
                           const uint32_t *__restrict__ el_slot, const uint32_t *__restrict__ el_id,
                           const DevRule *__restrict__ rules, State S, const uint32_t *__restrict__ ev_st,
                           const uint8_t *__restrict__ out_s, const uint32_t *__restrict__ wcnt,
                           const uint32_t *__restrict__ pc, unsigned long long *__restrict__ chk) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < E.n && ev_has(E, t)) {
    const uint32_t id = ev_line_id(S, el_slot, el_id, t);
    const uint32_t len = E.ip_len[t];
    if (S.ip_len[id] != len || !bytes_eq(S.arena + S.ip_off[id], ev_ip(E, t), len)) {
      if (atomicAdd(&chk[0], 1ull) == 0) { chk[1] = t; chk[2] = id; }
    }
  }
  if (t < n_ev) {
    const uint32_t i = ev_el[t];
    const uint64_t key = ((uint64_t)(ev_line_id(S, el_slot, el_id, i) + 1) << 24) | rules[ev_rule[t]].name_id;
    if (S.st[ev_st[t]].key != key) {
      if (atomicAdd(&chk[3], 1ull) == 0) { chk[4] = t; chk[5] = ev_st[t]; }
    }
    const uint8_t o = out_s[t];
    if (!(o & 0x80)) {
      if (atomicAdd(&chk[6], 1ull) == 0) chk[7] = t;
    }
    if (wcnt[t] != 1) {  // exactly one writer per sorted outcome
      if (atomicAdd(&chk[8], 1ull) == 0) chk[9] = t;
    }
    if (!(o & 1) && ((o >> 1) & 3) != BJX_FIRST_TIME) {  // seenIp false => FirstTime (rate_limit.go:48-51)
      if (atomicAdd(&chk[10], 1ull) == 0) chk[11] = t;
    }
    if (pc[t] != 1) {  // EvRec.ev over the sorted records is a permutation
      if (atomicAdd(&chk[12], 1ull) == 0) chk[13] = t;
    }
  }
}

// BJX_CHECK: each line's RuleResult count (counts >> 32) equals its match
// mask's population (a (line, rule) decided twice shows here)
__global__ void k_check_masks(uint64_t n_lines, Lines L, uint32_t mask_words, unsigned long long *__restrict__ chk) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_lines || mask_words > 2) return;  // past 128 positions the fast path leaves the words it never uses
  uint32_t pc = 0;
  const uint8_t f = L.flags[j];
  if (!(f & (kLineError | kLineOld | kLineExempt)))
    for (uint32_t w = 0; w < mask_words; ++w) pc += __popcll(L.mword(j, w));
  if ((uint32_t)(L.counts[j] >> 32) != pc && atomicAdd(&chk[0], 1ull) == 0) chk[1] = j;
}

// BJX_CHECK: cnt[idx[t * step]] += 1 for t < n (idx < cap, else chk[0]++)
__global__ void k_check_count(uint64_t n, const uint32_t *__restrict__ idx, uint32_t step, uint64_t cap,
                              uint32_t *__restrict__ cnt, unsigned long long *__restrict__ chk) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t v = idx[t * step];
  if (v < cap) atomicAdd(&cnt[v], 1u);
  else atomicAdd(&chk[0], 1ull);
}
// BJX_CHECK: entries of cnt above `most` -> chk[1] (count), chk[2] (first)
__global__ void k_check_most(uint64_t n, const uint32_t *__restrict__ cnt, uint32_t most, unsigned long long *__restrict__ chk) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n && cnt[t] > most && atomicAdd(&chk[1], 1ull) == 0) chk[2] = t;
}

// sorted outcomes -> event order (evw: the sorted records' event index words,
// `stride` words apart: either record form)
__global__ void k_unsort(uint64_t n, const uint32_t *__restrict__ evw, uint32_t stride, const uint8_t *__restrict__ in,
                         uint8_t *__restrict__ out) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) out[evw[u * stride]] = in[u];
}

// event index of each trip found in sorted order
__global__ void k_trip_events(uint64_t n, const uint32_t *__restrict__ pos, const uint32_t *__restrict__ evw, uint32_t stride,
                              uint32_t *__restrict__ ev) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) ev[t] = evw[(uint64_t)pos[t] * stride];
}

struct TripBit {
  __host__ __device__ __forceinline__ bool operator()(uint8_t v) const { return (v & 8) != 0; }
};

// Exceeded outcomes -> their indices, in no particular order (the caller
// sorts them by event): 64 outcomes per lane (four 16 B loads), compacted
// across the block, one atomic per block (a per-wave atomic on one counter
// serialised the kernel)
constexpr uint32_t kSelPer = 64;
__global__ __launch_bounds__(kBlock) void k_select_trips(uint64_t n, const uint8_t *__restrict__ out, uint32_t *__restrict__ idx,
                                                         unsigned long long *__restrict__ cnt) {
  __shared__ uint32_t s_wsum[kBlock / 64];
  __shared__ unsigned long long s_base;
  const uint64_t b = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kSelPer;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t m = 0;
  if (b + kSelPer <= n) {
    const uint4 *src = reinterpret_cast<const uint4 *>(out + b);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = src[q];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = (w[k] >> 3) & 0x01010101u;  // bit 3 (Exceeded) of each byte
        m |= (uint64_t)((x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u)) << (16 * q + 4 * k);
      }
    }
  } else {
    for (uint32_t k = 0; k < kSelPer; ++k)
      if (b + k < n && (out[b + k] & 8)) m |= 1ull << k;
  }
  const uint32_t c = __popcll(m);
  uint32_t x = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (uint32_t w = 0; w < kBlock / 64; ++w) {
    before += w < wave ? s_wsum[w] : 0u;
    tot += s_wsum[w];
  }
  if (threadIdx.x == 0) s_base = tot ? atomicAdd(cnt, (unsigned long long)tot) : 0ull;
  __syncthreads();
  uint64_t o = s_base + before + (x - c);
  while (m) {
    const uint32_t k = (uint32_t)__ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    idx[o++] = (uint32_t)(b + k);
  }
}

__global__ void k_flag_trips(uint64_t n, const uint8_t *__restrict__ ev_out, uint8_t *__restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = (ev_out[i] & 8) ? 1 : 0;
}

// (the host field is found again in the line: the per-line pass stores no
// host offsets, and only about 1 % of lines trip)
__global__ void k_build_trips(uint64_t n_trips, const uint32_t *__restrict__ idx, const uint32_t *__restrict__ ev_el,
                              const uint32_t *__restrict__ ev_rule, const uint8_t *__restrict__ buf,
                              const uint64_t *__restrict__ nl, Lines L, const DevRule *__restrict__ rules,
                              bjx_trip *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_trips) return;
  const uint32_t k = idx[t];
  const uint64_t line = ev_el[k];
  bjx_trip tr;
  tr.line_idx = line;
  tr.line_offset = line_start(nl, line);
  tr.line_len = (uint32_t)(nl[line] - tr.line_offset);
  tr.rule_idx = ev_rule[k];
  tr.ts_ns = L.ts[line];
  tr.ip_len = L.ip_len[line];
  tr.rest_off = L.rest_off[line];
  tr.ip_off = tr.rest_off - tr.ip_len - 1;
  uint32_t sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0;
  find_spaces(buf + tr.line_offset, tr.line_len, sp0, sp1, sp2, sp3);  // an event line has four
  tr.host_off = sp2 + 1;
  tr.host_len = sp3 - sp2 - 1;
  tr.decision = rules[tr.rule_idx].decision;
  out[t] = tr;
}

// ---- trip -> decision emission (bans.h)

// LogRegexBan line length of each trip (entry n_trips: 0, for the exclusive scan)
// BJX_TRIPS_COMPACT: the 8-byte trip words (line offset << 24 | rule index)
__global__ void k_pack_trips(uint64_t n, const bjx_trip *__restrict__ tr, uint64_t *__restrict__ out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = (tr[t].line_offset << 24) | (tr[t].rule_idx & 0xFFFFFFu);
}

__global__ void k_ban_len(BanDev A, uint64_t *__restrict__ len, uint8_t *__restrict__ kind) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > A.n_trips) return;
  if (t == A.n_trips) { len[t] = 0; return; }
  JOut<false> o{nullptr, 0};
  kind[t] = (uint8_t)ban_log_line(A, t, o);
  len[t] = o.n;
}

// trips [t0, t1) of the batch (emit_bans writes the log in chunks)
__global__ void k_ban_write(BanDev A, const uint64_t *__restrict__ off, uint8_t *__restrict__ out, uint64_t t0, uint64_t t1) {
  const uint64_t t = t0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= t1) return;
  JOut<true> o{out + off[t], 0};
  ban_log_line(A, t, o);
}

__device__ __forceinline__ const uint8_t *trip_ip(const BanDev &A, uint64_t t) {
  return A.buf + A.trips[t].line_offset + A.trips[t].ip_off;
}

// per-IP grouping key: hash of the IP bytes (exact grouping below)
__global__ void k_ban_keys(BanDev A, uint64_t mask, uint64_t *__restrict__ key, uint32_t *__restrict__ val) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= A.n_trips) return;
  key[t] = hash_bytes(trip_ip(A, t), A.trips[t].ip_len) & mask;  // mask: collision test hook
  val[t] = (uint32_t)t;
}

__global__ void k_ban_heads(uint64_t n, const uint64_t *__restrict__ ks, uint32_t *__restrict__ head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = (i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}

__device__ __forceinline__ bool same_ip(const BanDev &A, uint64_t a, uint64_t b) {
  const uint32_t n = A.trips[a].ip_len;
  if (A.trips[b].ip_len != n) return false;
  const uint8_t *x = trip_ip(A, a), *y = trip_ip(A, b);
  for (uint32_t k = 0; k < n; ++k)
    if (x[k] != y[k]) return false;
  return true;
}

// (max decision, first trip with it) per hash run: atomicMax of
// decision << 32 | ~trip; a run whose IP bytes differ (64-bit hash collision)
// is flagged and regrouped exactly by k_ban_collide
__global__ void k_ban_reduce(BanDev A, uint64_t n, const uint64_t *__restrict__ ks, const uint32_t *__restrict__ vs,
                             const uint32_t *__restrict__ seg, uint32_t *__restrict__ seg_first,
                             unsigned long long *__restrict__ best, uint32_t *__restrict__ cnt, uint32_t *__restrict__ ipt,
                             uint32_t *__restrict__ coll) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t s = seg[i] - 1, t = vs[i];
  const bool head = i == 0 || ks[i] != ks[i - 1];
  if (head) seg_first[s] = (uint32_t)i;
  else if (!same_ip(A, t, vs[i - 1])) atomicOr(&coll[s], 1u);
  const int32_t d = A.trips[t].decision;
  atomicMax(&best[s], ((unsigned long long)(uint32_t)d << 32) | (0xFFFFFFFFull - t));
  atomicAdd(&cnt[s], 1u);
  if (d == 4) atomicOr(&ipt[s], 1u);
}

__global__ void k_ban_out(uint64_t n_seg, const unsigned long long *__restrict__ best, const uint32_t *__restrict__ cnt,
                          const uint32_t *__restrict__ ipt, const uint32_t *__restrict__ coll, int64_t expires,
                          uint8_t *__restrict__ rep_flag, bjx_ip_decision *__restrict__ rep) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_seg || coll[s]) return;
  const uint32_t t = 0xFFFFFFFFu - (uint32_t)(best[s] & 0xFFFFFFFFull);
  bjx_ip_decision r;
  r.trip_idx = t;
  r.n_trips = cnt[s];
  r.expires_ns = expires;
  r.decision = (int32_t)(best[s] >> 32);
  r.iptables = ipt[s];
  rep[t] = r;
  rep_flag[t] = 1;
}

// hash runs holding more than one IP: one lane per run groups its trips by
// their bytes (trip order within the run, O(run^2); 64-bit collisions only)
__global__ void k_ban_collide(BanDev A, uint64_t n, uint64_t n_seg, const uint32_t *__restrict__ vs,
                              const uint32_t *__restrict__ seg_first, const uint32_t *__restrict__ coll, int64_t expires,
                              uint8_t *__restrict__ rep_flag, bjx_ip_decision *__restrict__ rep) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_seg || !coll[s]) return;
  const uint64_t b = seg_first[s], e = s + 1 < n_seg ? seg_first[s + 1] : n;
  for (uint64_t i = b; i < e; ++i) {
    bool leader = true;
    for (uint64_t k = b; k < i && leader; ++k) leader = !same_ip(A, vs[i], vs[k]);
    if (!leader) continue;
    uint32_t bt = vs[i], nt = 0, ip4 = 0;
    int32_t bd = -1;
    for (uint64_t k = i; k < e; ++k) {
      const uint32_t t = vs[k];
      if (k != i && !same_ip(A, vs[i], t)) continue;
      const int32_t d = A.trips[t].decision;
      if (d > bd || (d == bd && t < bt)) { bd = d; bt = t; }
      ++nt;
      ip4 |= d == 4 ? 1u : 0u;
    }
    bjx_ip_decision r;
    r.trip_idx = bt; r.n_trips = nt; r.expires_ns = expires; r.decision = bd; r.iptables = ip4;
    rep[bt] = r;
    rep_flag[bt] = 1;
  }
}

__global__ void k_scatter_rl(uint64_t n_ev, const uint32_t *__restrict__ ev_res, const uint8_t *__restrict__ ev_out,
                             uint8_t *__restrict__ rl_out) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_ev) rl_out[ev_res[k]] = ev_out[k];
}

__global__ void k_build_results(uint64_t n, const uint64_t *__restrict__ res_seq, const uint32_t *__restrict__ res_rule,
                                const uint8_t *__restrict__ rl_out, bjx_rule_result *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bjx_rule_result r;
  r.line_idx = res_seq[i] >> 16;
  r.rule_pos = (uint16_t)(res_seq[i] & 0xFFFF);
  r.rule_idx = res_rule[i] & 0x7FFFFFFFu;
  r.skip_host = (res_rule[i] >> 31) & 1;
  const uint8_t o = rl_out[i];
  r.seen_ip = o & 1;
  r.match_type = (o >> 1) & 3;
  r.exceeded = (o >> 3) & 1;
  r._pad[0] = r._pad[1] = 0;
  out[i] = r;
}

__global__ void k_final_flags(uint64_t n, uint8_t *__restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] &= (kLineError | kLineOld | kLineExempt);
}

// undo one batch's claims (table overflow): its slots were empty before the
// batch and no earlier key's probe chain runs through them
__global__ void k_ip_rollback(uint64_t cap, State S, uint32_t epoch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const IpSlot v = S.ip[i];
  if (v.hash != 0 && (v.born == epoch || v.born == 0)) {
    S.ip[i] = IpSlot{};
    S.ip_first[i] = 0xFFFFFFFFu;
  }
}
__global__ void k_st_rollback(uint64_t cap, State S) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cap) return;
  const bool live = S.st[i].key != 0 && S.st[i].valid != 0;
  if (S.st[i].key != 0 && !live) S.st[i] = StSlot{};
  const uint64_t m = __ballot(live);
  if (m && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)m) - 1))
    atomicAdd((unsigned long long *)&S.counters[2], (unsigned long long)__popcll(m));
}

// rehash (table growth)
__global__ void k_rehash_ip(uint64_t old_cap, const IpSlot *__restrict__ o, IpSlot *__restrict__ nt, uint64_t nmask) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap || o[i].hash == 0) return;
  uint64_t j = o[i].hash & nmask;
  for (;;) {
    const unsigned long long prev = atomicCAS((unsigned long long *)&nt[j].hash, 0ull, (unsigned long long)o[i].hash);
    if (prev == 0) { nt[j].id = o[i].id; nt[j].born = o[i].born; nt[j].key16 = o[i].key16; return; }
    j = (j + 1) & nmask;
  }
}
__global__ void k_rehash_st(uint64_t old_cap, const StSlot *__restrict__ o, StSlot *__restrict__ nt, uint64_t nmask) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= old_cap || o[i].key == 0) return;
  uint64_t j = mix64(o[i].key) & nmask;
  for (;;) {
    const unsigned long long prev = atomicCAS((unsigned long long *)&nt[j].key, 0ull, (unsigned long long)o[i].key);
    if (prev == 0) { nt[j].hits = o[i].hits; nt[j].start = o[i].start; nt[j].valid = o[i].valid; return; }
    j = (j + 1) & nmask;
  }
}

// --------------------------------------------------------------- multi-GPU exchange
// The partition runs over the lines in tiles of `steps` x kBlock lines (one
// block each, one line per lane per step), in line order: k_part_count sums
// each tile's (event lines, events, IP bytes) per owner; one exclusive scan
// per quantity over [owner][tile] gives every (owner, tile) its first packed
// position, owner-major (the order of a stable sort by owner); k_pack re-reads
// the tile and writes each event line's record, rule indices and IP bytes
// there.  Inside a tile, lanes of one owner are ranked by ballot (one pass per
// distinct owner in the wave) and the four waves by their per-owner totals, so
// a line's place follows line order.  Each IP takes a 4-byte aligned slot of
// the byte pool (its length rounded up), so a lane stores its IP as whole
// words with no neighbour sharing them.
constexpr uint32_t kMaxParts = 256;       // owners of one partition
__host__ __device__ __forceinline__ uint32_t ip_slot_bytes(uint32_t len) { return (len + 3u) & ~3u; }

struct PartLine {
  bool ev;           // an event line
  uint32_t o, ne, len;
};
__device__ __forceinline__ PartLine part_line(uint64_t j, uint64_t n_lines, const Lines &L, uint32_t n_parts) {
  PartLine r{false, 0, 0, 0};
  if (j < n_lines) {
    r.ne = (uint32_t)(L.counts[j] & 0xFFFFFFFFull);
    if (r.ne) {
      r.ev = true;
      r.len = L.ip_len[j];
      // the owner: a function of the IP bytes (hash_bytes), as every source computes it
      r.o = (uint32_t)(((r.len <= 15 ? key16_hash(L.ip16[j], r.len) : L.ip_hash[j]) >> 32) % n_parts);
    }
  }
  return r;
}
// (events | IP slot bytes << 32) of one line; clamped to the 16-bit wire
// fields so a tile's sums stay in 32 bits (a wider line fails the batch: *wide)
__device__ __forceinline__ uint64_t part_eb(const PartLine &x) {
  return (uint64_t)min(x.ne, 0xFFFFu) | ((uint64_t)ip_slot_bytes(min(x.len, 0xFFFFu)) << 32);
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t x = __shfl_up(v, d, 64);
    if (lane >= d) v += x;
  }
  return v;
}

// hist: three arrays of S = n_parts * n_tiles + 1 entries (event lines,
// events, IP bytes), entry o * n_tiles + tile; the last entry of each is left
// zero (the scans then end in the totals).  *wide: a line whose event count or
// IP length does not fit bjx_event_line's 16-bit fields (the batch then fails
// with BJX_ERR_CAPACITY instead of packing a truncated key)
__global__ __launch_bounds__(kBlock) void k_part_count(uint64_t n_lines, uint32_t n_tiles, uint32_t steps, Lines L,
                                                       uint32_t n_parts, uint64_t *__restrict__ hist,
                                                       unsigned long long *__restrict__ wide) {
  __shared__ unsigned long long s_n[kMaxParts], s_eb[kMaxParts];
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t o = threadIdx.x; o < n_parts; o += kBlock) s_n[o] = 0, s_eb[o] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * steps * kBlock;
  bool w = false;
  for (uint32_t s = 0; s < steps; ++s) {
    const PartLine x = part_line(base + s * kBlock + threadIdx.x, n_lines, L, n_parts);
    w |= x.ev && (x.ne > 0xFFFFu || x.len > 0xFFFFu);
    for (uint64_t todo = __ballot(x.ev); todo;) {  // each owner present in the wave once
      const uint32_t lead = (uint32_t)__ffsll((unsigned long long)todo) - 1;
      const uint32_t o = __shfl(x.o, lead, 64);
      const bool mine = x.ev && x.o == o;
      const uint64_t m = __ballot(mine);
      todo &= ~m;
      uint64_t v = mine ? part_eb(x) : 0;
#pragma unroll
      for (uint32_t d = 32; d; d >>= 1) v += __shfl_xor(v, d, 64);
      if (lane == lead) {
        atomicAdd(&s_n[o], (unsigned long long)__popcll(m));
        atomicAdd(&s_eb[o], (unsigned long long)v);
      }
    }
  }
  if (__ballot(w) && lane == 0) atomicOr(wide, 1ull);
  __syncthreads();
  const uint64_t S = (uint64_t)n_parts * n_tiles + 1;
  for (uint32_t o = threadIdx.x; o < n_parts; o += kBlock) {
    const uint64_t i = (uint64_t)o * n_tiles + blockIdx.x;
    hist[i] = s_n[o];
    hist[S + i] = s_eb[o] & 0xFFFFFFFFull;
    hist[2 * S + i] = s_eb[o] >> 32;
  }
}

// per owner: (lines, events, bytes) and the owner's first byte (off: the
// exclusive scans of k_part_count's arrays); one thread
__global__ void k_part_counts(uint32_t n_parts, uint32_t n_tiles, const uint64_t *__restrict__ off,
                              uint64_t *__restrict__ counts, uint64_t *__restrict__ byte_base) {
  if (blockIdx.x || threadIdx.x) return;
  const uint64_t S = (uint64_t)n_parts * n_tiles + 1;
  for (uint32_t k = 0; k < n_parts; ++k) {
    const uint64_t b = (uint64_t)k * n_tiles, e = b + n_tiles;
    for (int c = 0; c < 3; ++c) counts[3 * k + c] = off[c * S + e] - off[c * S + b];
    byte_base[k] = off[2 * S + b];
  }
}

struct PackArgs {
  uint64_t n_lines;
  uint32_t n_tiles, n_parts, steps;
  const uint64_t *off;        // k_part_count's arrays, exclusive-scanned
  const uint64_t *byte_base;  // each owner's first byte
  const uint8_t *buf;
  const uint64_t *nl;
  Lines L;
  const uint64_t *offs;       // line -> first event (low 32 bits)
  const uint32_t *ev_rule;
  bjx_event_line *d_lines;
  uint32_t *d_events;
  uint8_t *d_bytes;
  uint32_t *pack_src;         // packed event -> local event
};

// dynamic LDS: s_run[3][n_parts] (the tile's next positions per owner) and
// s_wt[2][4][n_parts] x 2 words (per step parity and wave: an owner's lines and
// events | bytes << 32)
__host__ __device__ constexpr uint32_t pack_lds_bytes(uint32_t n_parts) {
  return 3 * n_parts * 8 + 2 * (kBlock / 64) * n_parts * 16;
}

__global__ __launch_bounds__(kBlock) void k_pack(PackArgs A) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
  const uint32_t N = A.n_parts, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t *s_run = reinterpret_cast<uint64_t *>(s_dyn);
  uint64_t *s_wt = s_run + 3 * N;  // [parity][wave][owner][2]
  const uint64_t S = (uint64_t)N * A.n_tiles + 1;
  for (uint32_t o = threadIdx.x; o < N; o += kBlock) {
    const uint64_t i = (uint64_t)o * A.n_tiles + blockIdx.x;
    s_run[o] = A.off[i];
    s_run[N + o] = A.off[S + i];
    s_run[2 * N + o] = A.off[2 * S + i];
  }
  const uint64_t base = (uint64_t)blockIdx.x * A.steps * kBlock;
  for (uint32_t s = 0; s < A.steps; ++s) {
    const uint64_t j = base + s * kBlock + threadIdx.x;
    const PartLine x = part_line(j, A.n_lines, A.L, N);
    uint64_t *wt = s_wt + (size_t)(s & 1) * (kBlock / 64) * N * 2;
    uint64_t *mine_wt = wt + (size_t)wv * N * 2;
    // this wave's row: zero, then each present owner's totals
    for (uint32_t o = lane; o < N; o += 64) mine_wt[2 * o] = 0, mine_wt[2 * o + 1] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t rank = 0;
    uint64_t pre = 0;  // events | bytes << 32 of the wave's earlier lanes of this owner
    for (uint64_t todo = __ballot(x.ev); todo;) {
      const uint32_t lead = (uint32_t)__ffsll((unsigned long long)todo) - 1;
      const uint32_t o = __shfl(x.o, lead, 64);
      const bool mine = x.ev && x.o == o;
      const uint64_t m = __ballot(mine);
      todo &= ~m;
      const uint64_t v = mine ? part_eb(x) : 0;
      const uint64_t inc = wave_incl_scan64(v, lane);
      if (mine) {
        rank = (uint32_t)__popcll(m & ((1ull << lane) - 1));
        pre = inc - v;
      }
      const uint64_t tot = __shfl(inc, 63, 64);
      if (lane == lead) mine_wt[2 * o] = (uint64_t)__popcll(m), mine_wt[2 * o + 1] = tot;
    }
    __syncthreads();
    uint64_t pl = 0, pe = 0, pb = 0;
    if (x.ev) {
      uint64_t cl = 0, ceb = 0;
      for (uint32_t w2 = 0; w2 < wv; ++w2) {
        cl += wt[((size_t)w2 * N + x.o) * 2];
        ceb += wt[((size_t)w2 * N + x.o) * 2 + 1];
      }
      pl = s_run[x.o] + cl + rank;
      pe = s_run[N + x.o] + (ceb & 0xFFFFFFFFull) + (pre & 0xFFFFFFFFull);
      pb = s_run[2 * N + x.o] + (ceb >> 32) + (pre >> 32);
    }
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < N; o += kBlock) {  // the tile's positions after this step
      uint64_t cl = 0, ceb = 0;
      for (uint32_t w2 = 0; w2 < kBlock / 64; ++w2) {
        cl += wt[((size_t)w2 * N + o) * 2];
        ceb += wt[((size_t)w2 * N + o) * 2 + 1];
      }
      s_run[o] += cl;
      s_run[N + o] += ceb & 0xFFFFFFFFull;
      s_run[2 * N + o] += ceb >> 32;
    }
    // the line's record and rule indices
    const uint32_t jj = (uint32_t)j;
    if (x.ev) {
      bjx_event_line r;
      r.ts_ns = A.L.ts[jj];
      r.ip_off = (uint32_t)(pb - A.byte_base[x.o]);
      r.ip_len = (uint16_t)x.len;
      r.n_events = (uint16_t)x.ne;
      A.d_lines[pl] = r;
      const uint64_t eo = A.offs[jj] & 0xFFFFFFFFull;
      for (uint32_t t = 0; t < x.ne; ++t) {
        A.d_events[pe + t] = A.ev_rule[eo + t];
        A.pack_src[pe + t] = (uint32_t)(eo + t);
      }
    }
    // the IP bytes as whole words into the line's aligned slot: an IP of <= 15
    // bytes from its inline key, a longer one by aligned word loads from the
    // line, all issued at once (a chain of dependent loads cost a round trip
    // per word), one of 48 bytes or more word by word
    if (x.ev) {
      uint32_t *dst = reinterpret_cast<uint32_t *>(A.d_bytes + pb);
      const uint32_t nw = (x.len + 3) >> 2;
      if (x.len <= 15) {
        const uint4 k16 = A.L.ip16[jj];
        const uint32_t kw[4] = {k16.x, k16.y, k16.z, k16.w & 0x00FFFFFFu};  // byte 15 is the length
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
          if (k < nw) dst[k] = kw[k];
      } else {
        const uint8_t *ip = A.buf + line_start(A.nl, jj) + A.L.rest_off[jj] - x.len - 1;
        if (x.len < 4 * kIpWords) {
          uint32_t iw[kIpWords];
          ip_words(ip, x.len, iw);
#pragma unroll
          for (uint32_t k = 0; k < kIpWords; ++k)
            if (k < nw) dst[k] = iw[k];
        } else {
          for (uint32_t k = 0; k < nw; ++k) {
            const uint32_t w = ld4(ip + 4 * k);
            const uint32_t left = x.len - 4 * k;
            dst[k] = left >= 4 ? w : w & ((1u << (8 * left)) - 1u);
          }
        }
      }
    }
  }
}

// received records of one source -> SoA rate-limit input (absolute IP offsets)
// received event lines -> the rate-limit input arrays, with each IP's inline
// key (IpSlot.key16) built once here from the byte pool (neighbouring lanes
// read neighbouring bytes) instead of in every claim kernel
__global__ void k_unpack_lines(uint64_t n, uint64_t first, uint64_t byte_base, const bjx_event_line *__restrict__ rec,
                               const uint8_t *__restrict__ bytes, int64_t *__restrict__ ts, uint64_t *__restrict__ hash,
                               uint64_t *__restrict__ pos, uint32_t *__restrict__ len, uint64_t *__restrict__ nev,
                               uint4 *__restrict__ ip16, uint64_t dbg_mask) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bjx_event_line r = rec[first + i];
  ts[first + i] = r.ts_ns;
  // the IP's hash (the source's hash_bytes; not on the wire) and inline key,
  // an IP of <= 15 bytes from one set of word loads
  const uint8_t *ip = bytes + byte_base + r.ip_off;
  uint64_t h;
  uint4 k16;
  if (r.ip_len < 4 * kIpWords) {  // IPv4 and IPv6 text: one set of word loads
    uint32_t w[kIpWords];
    ip_words(ip, r.ip_len, w);
    h = hash_words(w, r.ip_len);
    k16 = make_uint4(w[0], w[1], w[2], (r.ip_len <= 15 ? w[3] : w[3] & 0x00FFFFFFu) | (min((uint32_t)r.ip_len, 255u) << 24));
  } else {
    h = hash_bytes(ip, r.ip_len);
    k16 = ip_key16_bytes(ip, r.ip_len);
  }
  hash[first + i] = dbg_mask ? (h & dbg_mask) | 1 : h;
  pos[first + i] = byte_base + r.ip_off;
  len[first + i] = r.ip_len;
  nev[first + i] = r.n_events;
  ip16[first + i] = k16;
}

// event -> its line (events of line i are [off[i], off[i] + nev[i])); flags bad rule ids
__global__ void k_expand_events(uint64_t n, const uint64_t *__restrict__ off, const uint64_t *__restrict__ nev,
                                uint64_t n_ev, const uint32_t *__restrict__ ev_rule, uint32_t n_rules,
                                uint32_t *__restrict__ ev_el, unsigned long long *__restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = off[i], e = b + nev[i];
  if (e > n_ev) { atomicAdd(bad, 1ull); return; }
  for (uint64_t k = b; k < e; ++k) {
    if (ev_rule[k] >= n_rules) atomicAdd(bad, 1ull);
    ev_el[k] = (uint32_t)i;
  }
}

// owner side of bjx_apply_events_trips: the ascending received indices of
// the tripping events -> base[k] + index inside source k's segment (ev_base:
// the segments' first received event, n_src + 1 entries); start[k] = source
// k's first trip (untouched when it has none)
__global__ void k_trip_rebase(uint64_t n, const uint32_t *__restrict__ u, uint32_t n_src, const uint64_t *__restrict__ ev_base,
                              const uint64_t *__restrict__ base, uint32_t *__restrict__ out, uint64_t *__restrict__ start) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint64_t x = u[t];
  uint32_t lo = 0, hi = n_src;  // the last source whose segment starts at or before x
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ev_base[mid] <= x) lo = mid;
    else hi = mid;
  }
  out[t] = (uint32_t)(base[lo] + (x - ev_base[lo]));
  if (t == 0 || u[t - 1] < ev_base[lo]) start[lo] = t;
}

// source side of bjx_finish_batch_trips: packed event index -> local event
// index (out-of-range indices counted in bad)
__global__ void k_map_trips(uint64_t n, const uint32_t *__restrict__ packed, uint64_t n_ev, const uint32_t *__restrict__ src,
                            uint32_t *__restrict__ out, unsigned long long *__restrict__ bad) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t q = packed[t];
  if (q < n_ev) out[t] = src[q];
  else {
    out[t] = 0;
    atomicAdd(bad, 1ull);
  }
}

// sorted event indices: count adjacent equal pairs (a trip list that names one
// event twice)
__global__ void k_count_dups(uint64_t n, const uint32_t *__restrict__ sorted, unsigned long long *__restrict__ dups) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
  if (t < n && sorted[t] == sorted[t - 1]) atomicAdd(dups, 1ull);
}

__global__ void k_scatter_outcomes(uint64_t n, const uint32_t *__restrict__ src, const uint8_t *__restrict__ in,
                                   uint8_t *__restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[src[k]] = in[k];
}

// state query (RegexRateLimitStates.Get for one (ip, name))
__global__ void k_state_get(State S, uint64_t h, const uint8_t *ip, uint32_t len, uint32_t name_id, int64_t *out) {
  out[0] = 0;
  uint64_t i = h & S.ip_mask;
  for (;;) {
    const uint64_t cur = S.ip[i].hash;
    if (cur == 0) return;
    if (cur == h) {
      const uint32_t id = S.ip[i].id;
      if (S.ip_len[id] == len && bytes_eq(S.arena + S.ip_off[id], ip, len)) {
        const uint64_t key = ((uint64_t)(id + 1) << 24) | name_id;
        uint64_t j = mix64(key) & S.st_mask;
        for (;;) {
          const uint64_t k = S.st[j].key;
          if (k == 0) { out[0] = 1; return; }  // ip known, rule state absent
          if (k == key) {
            if (!S.st[j].valid) { out[0] = 1; return; }
            out[0] = 2; out[1] = S.st[j].hits; out[2] = S.st[j].start;
            return;
          }
          j = (j + 1) & S.st_mask;
        }
      }
    }
    i = (i + 1) & S.ip_mask;
  }
}

// =====================================================================
//                               host side
// =====================================================================

template <typename T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  void ensure(size_t want) {
    if (want <= n && p) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t cap = want < 1024 ? 1024 : want + want / 4;
    HIP_OK(hipMalloc(&p, cap * sizeof(T)));
    n = cap;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Pinned host array for batch outputs (D2H at full PCIe rate, no zero-fill).
template <typename T>
struct HostBuf {
  T *p = nullptr;
  size_t n = 0, cap = 0;
  void resize(size_t want) {
    if (want > cap) {
      // geometric growth with headroom: a pinned (re)allocation stalls the
      // batch for ~0.1 ms/MB, and per-batch counts (trips) drift upwards.
      // Past 64 MB the headroom is a quarter (cfg5's 40 GB of ban-log text
      // would otherwise pin 80 GB)
      const size_t big = (64u << 20) / sizeof(T);
      const size_t c = want > big ? std::max<size_t>(want + want / 4, cap + cap / 4)
                                  : std::max<size_t>({want * 2, cap * 2, 1u << 16});
      if (p) (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
      HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&p), c * sizeof(T), hipHostMallocDefault));
      cap = c;
    }
    n = want;
  }
  // capacity of at least `want` elements (contents not kept)
  void reserve(size_t want) {
    if (want <= cap) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&p), want * sizeof(T), hipHostMallocDefault));
    cap = want;
  }
  void clear() { n = 0; }
  bool empty() const { return n == 0; }
  T *data() { return p; }
  size_t size() const { return n; }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = cap = 0;
  }
};

inline unsigned grid_for(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

// ------------------------------------------------------------ ruleset

struct bjx_ruleset {
  struct Rule {
    std::string name, regex;
    int64_t interval_ns = 0, hits = 0;
    int32_t decision = 0;
    std::vector<std::string> skip_hosts;
    CompiledRegex rx;
  };
  std::vector<Rule> rules;
  uint32_t n_global = 0;
  std::vector<std::pair<std::string, std::vector<uint32_t>>> sites;
  uint64_t uid = 0;
};

static std::atomic<uint64_t> g_ruleset_uid{1};

extern "C" int bjx_abi_version(void) { return BJX_ABI_VERSION; }

static void set_err(char *err, size_t len, const std::string &m) {
  if (!err || !len) return;
  size_t k = std::min(len - 1, m.size());
  memcpy(err, m.data(), k);
  err[k] = 0;
}

// Compiled regexes by pattern, process-wide: a reload (ConfigHolder.Reload,
// config_holder.go:55-66) recompiles only the patterns it has not seen
// before.  Entries are immutable once published.
struct RxCacheEntry {
  int rc = 0;
  std::string err;
  CompiledRegex rx;
};
static std::mutex g_rx_mu;
static std::unordered_map<std::string, std::shared_ptr<const RxCacheEntry>> g_rx_cache;
static constexpr size_t kRxCacheMax = 1u << 16;

// compile every pattern not in the cache, on up to 16 host threads
static std::vector<std::shared_ptr<const RxCacheEntry>> compile_patterns(const std::vector<std::string> &pats) {
  std::vector<std::shared_ptr<const RxCacheEntry>> out(pats.size());
  std::vector<size_t> todo;
  {
    std::lock_guard<std::mutex> g(g_rx_mu);
    std::unordered_map<std::string, size_t> first;
    for (size_t i = 0; i < pats.size(); ++i) {
      auto it = g_rx_cache.find(pats[i]);
      if (it != g_rx_cache.end()) out[i] = it->second;
      else if (first.emplace(pats[i], i).second) todo.push_back(i);
    }
  }
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t k; (k = next.fetch_add(1)) < todo.size();) {
      auto e = std::make_shared<RxCacheEntry>();
      e->rc = compile_regex(pats[todo[k]], &e->rx, &e->err);
      out[todo[k]] = std::move(e);
    }
  };
  const size_t nt = std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), (todo.size() + 7) / 8});
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  std::lock_guard<std::mutex> g(g_rx_mu);
  if (g_rx_cache.size() + todo.size() > kRxCacheMax) g_rx_cache.clear();
  for (size_t i : todo) g_rx_cache.emplace(pats[i], out[i]);
  for (size_t i = 0; i < pats.size(); ++i)
    if (!out[i]) out[i] = g_rx_cache.at(pats[i]);
  return out;
}

extern "C" int bjx_ruleset_compile(const bjx_rule_spec *global_rules, size_t n_global, const bjx_site_rules *per_site,
                                   size_t n_sites, bjx_ruleset **out, int64_t *err_rule, char *err, size_t err_len) {
  if (!out) return BJX_ERR_ARG;
  *out = nullptr;
  if (err_rule) *err_rule = -1;
  try {
    auto rs = std::make_unique<bjx_ruleset>();
    // every rule spec in evaluation order: globals, then each site's rules
    std::vector<const bjx_rule_spec *> specs;
    for (size_t i = 0; i < n_global; ++i) specs.push_back(&global_rules[i]);
    for (size_t s = 0; s < n_sites; ++s)
      for (size_t k = 0; k < per_site[s].n_rules; ++k) specs.push_back(&per_site[s].rules[k]);
    std::vector<std::string> pats;
    for (auto *sp : specs) pats.emplace_back(sp->regex.ptr ? sp->regex.ptr : "", sp->regex.len);
    const auto compiled = compile_patterns(pats);
    // the first failing rule in order decides the error, as the sequential
    // UnmarshalYAML -> regexp.Compile does (config.go:110-113)
    size_t si = 0;
    auto add = [&](const bjx_rule_spec &s) -> int {
      const size_t i = si++;
      if (s.decision < BJX_ALLOW || s.decision > BJX_IPTABLES_BLOCK) {
        set_err(err, err_len, "invalid decision value");
        return BJX_ERR_DECISION;
      }
      const RxCacheEntry &ce = *compiled[i];
      if (ce.rc != 0) {
        set_err(err, err_len, ce.err);
        return ce.rc;
      }
      bjx_ruleset::Rule r;
      r.name.assign(s.name.ptr ? s.name.ptr : "", s.name.len);
      r.regex = pats[i];
      r.interval_ns = s.interval_ns;
      r.hits = s.hits_per_interval;
      r.decision = s.decision;
      for (size_t k = 0; k < s.n_hosts_to_skip; ++k) r.skip_hosts.emplace_back(s.hosts_to_skip[k].ptr, s.hosts_to_skip[k].len);
      r.rx = ce.rx;
      rs->rules.push_back(std::move(r));
      return 0;
    };
    for (size_t i = 0; i < n_global; ++i) {
      int rc = add(global_rules[i]);
      if (rc) { if (err_rule) *err_rule = (int64_t)i; return rc; }
    }
    rs->n_global = (uint32_t)n_global;
    size_t max_site = 0;
    for (size_t s = 0; s < n_sites; ++s) {
      std::string host(per_site[s].host.ptr ? per_site[s].host.ptr : "", per_site[s].host.len);
      for (auto &p : rs->sites)
        if (p.first == host) { set_err(err, err_len, "duplicate per-site host: " + host); return BJX_ERR_ARG; }
      std::vector<uint32_t> ids;
      for (size_t k = 0; k < per_site[s].n_rules; ++k) {
        int rc = add(per_site[s].rules[k]);
        if (rc) { if (err_rule) *err_rule = (int64_t)(rs->rules.size()); return rc; }
        ids.push_back((uint32_t)rs->rules.size() - 1);
      }
      max_site = std::max(max_site, ids.size());
      rs->sites.emplace_back(host, std::move(ids));
    }
    if (max_site + n_global >= 65536) { set_err(err, err_len, "more than 65535 rules apply to one host"); return BJX_ERR_TOO_COMPLEX; }
    rs->uid = g_ruleset_uid++;
    *out = rs.release();
    return BJX_OK;
  } catch (const std::exception &e) {
    set_err(err, err_len, e.what());
    return BJX_ERR_NOMEM;
  }
}

extern "C" void bjx_ruleset_release(bjx_ruleset *rs) { delete rs; }
extern "C" size_t bjx_ruleset_num_rules(const bjx_ruleset *rs) { return rs ? rs->rules.size() : 0; }
extern "C" int bjx_ruleset_rule_info(const bjx_ruleset *rs, size_t i, uint32_t *states, uint32_t *classes, uint32_t *flags) {
  if (!rs || i >= rs->rules.size()) return BJX_ERR_ARG;
  const auto &rx = rs->rules[i].rx;
  if (states) *states = rx.nstates;
  if (classes) *classes = rx.ncls;
  if (flags)
    *flags = rx.flags | ((uint32_t)rx.mode << 8) | (rx.pref_equivalent ? 0x10000u : 0u) | (rx.pref_lead ? 0x20000u : 0u) |
             ((uint32_t)rx.pref.size() << 20);
  return BJX_OK;
}

// ------------------------------------------------------------ engine

struct BatchCtx {
  const uint8_t *buf = nullptr;
  uint64_t n_lines = 0, n_res = 0, n_ev = 0;
  uint64_t n_el = 0, el_bytes = 0;  // lines with events, their IP bytes
  uint64_t consumed = 0;
  int64_t now_ns = 0;
  Lines L{};
  bool live = false;
};

struct bjx_engine {
  int device = 0;
  std::mutex mu;
  std::string last_error;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evm0 = nullptr, evm1 = nullptr;
  hipEvent_t evk[4] = {};      // k_lines launch, DFA-job sort + k_dfa / k_nfa (bench: per-kernel roofline)
  double kernel_ms[3] = {};   // last batch: k_scan, k_lines, DFA jobs
  uint32_t last_line_kernel = 0;  // last batch's per-line kernel: 2 = k_lines2, 1 = k_lines, 3 = k_parse_match (every line)
  static constexpr int kPhases = 8;
  hipEvent_t ph[kPhases + 1] = {};
  double phase_ms[kPhases] = {};
  // node batches: from bjx_events_partition to the start of the owner's
  // rate-limit stage (partition, pack, the copies' wait, unpack)
  hipEvent_t xev[2] = {};
  hipStream_t bstream = nullptr;  // the ban log's D2H copies (emit_bans)
  hipEvent_t bev[kBanChunks + 1] = {};
  bool xev_rec = false;
  double exchange_ms = 0;
  bool phase_rec[kPhases + 1] = {};

  // decision lists (config order)
  struct Entry { bool global; std::string site; int32_t decision; std::string ip; };
  std::vector<Entry> decisions;
  uint64_t decisions_version = 1;

  // rule names -> ids (state keys survive reloads)
  std::unordered_map<std::string, uint32_t> name_ids;
  std::vector<std::string> names;

  // binding cache
  uint64_t bound_uid = 0, bound_dec_version = 0;
  DevBuf<uint8_t> bind_blob;
  Bind bind{};
  std::vector<uint4> nfa_rules;  // (rule, state words, table words) of the kRuleNfa patterns (k_nfa launches)
  DevBuf<uint32_t> rb_first, rb_last;
  std::vector<uint32_t> h_first, h_last;
  std::vector<DevRule> host_rules;

  // persistent state
  State S{};
  uint64_t ip_cap = 0, st_cap = 0;
  uint64_t rehashes = 0;
  uint64_t last_new_ips = 0, last_new_states = 0;  // entries the last batch created (capacity prediction)
  uint32_t epoch = 0;  // batch counter (IpSlot.born)
  uint64_t dbg_hash_mask = 0;  // bjx_debug_set_ip_hash_mask
  uint64_t dbg_budget = 0;     // bjx_debug_set_claim_budget (0 = off)
  uint32_t lines2_lds = 0;     // dynamic LDS k_lines2 was last configured for
  uint32_t lines2_w = 0;       // ... and the instance (mask width) it was set on
  int dbg_slot_cache = -1;     // bjx_debug_set_slot_cache: -1 = BJX_SLOT_CACHE / default on, 0 off, 1 on
  uint64_t host_counters[3] = {0, 0, 0};
  // host_counters were read with the match phase's last counts, nothing has
  // touched the tables since (run_batch: match, then straight to the rate limit)
  bool counters_fresh = false, want_counters = false;
  // small device -> host reads (counts, flags) through a pinned ring: a copy
  // into pageable memory makes the host wait for it, so a few in a row cost a
  // round trip (20-30 us) each; queued here they cost one stream sync
  static constexpr uint32_t kPinBytes = 16384, kPinReads = 32;
  uint8_t *pin = nullptr;
  uint32_t pin_used = 0, pin_n = 0;
  struct PinRead { void *dst; const uint8_t *slot; uint32_t n; } pin_q[kPinReads];

  // batch workspace
  DevBuf<uint8_t> staging;
  DevBuf<uint32_t> tile_counts;
  DevBuf<uint64_t> tile_base, nl;
  DevBuf<int64_t> l_ts;
  DevBuf<uint64_t> l_iph, l_counts, l_offs, l_masks;
  DevBuf<uint32_t> l_iplen, l_roff, slow_list;
  DevBuf<int32_t> l_hid;
  DevBuf<uint64_t> l_cand;
  DevBuf<uint4> l_ip16;
  DevBuf<uint32_t> jline, jkey, jidx, jidx2, jkey2;  // jobs by slot (line, key, slot), the sorted keys and slots
  DevBuf<uint64_t> jrec;                           // job window records by slot (kJob*)
  uint64_t last_jobs = 0, last_long_runs = 0;
  DevBuf<uint64_t> long_heads;
  DevBuf<uint64_t> lr_end, lr_len, lr_off, lr_win;
  DevBuf<unsigned long long> chk;
  DevBuf<uint64_t> wide_scratch;             // k_nfa_wide<true>: per-block state sets
  DevBuf<uint32_t> wl_line, wl_rule, wl_pos;  // the per-line fallback's wide-NFA jobs
  uint32_t wide_max_w = 0, wide_max_g = 0, n_wide = 0;
  DevBuf<uint32_t> chk_w;  // BJX_CHECK: per-outcome write counts, event-index counts
  DevBuf<uint32_t> chk_wb;  // BJX_CHECK: write counts of the oversized buckets' full-sort outcomes
  DevBuf<int64_t> lr_t0, lr_h0;
  DevBuf<uint32_t> lr_flags, lr_nwin;
  DevBuf<unsigned long long> long_count;
  // two-level grouping (k_bucket_apply): bucket bounds, oversized buckets, their events
  DevBuf<uint32_t> bk_start, bk_big, bk_key, bk_pos;
  DevBuf<unsigned long long> bk_nbig;
  DevBuf<uint4> bk_seg;
  DevBuf<EvRec> bk_rec;
  DevBuf<uint8_t> bk_out;
  uint64_t last_big_events = 0;
  uint32_t sort2_hold = 0;
  uint64_t last_grouping = 0;  // 0: full sort; else 1 + the events of oversized buckets (bjx_debug_scan_stats[10])  // batches left on the full sort after one with many hot-key events
  uint32_t scan_lds[2] = {0, 0};
  bool lines_attr = false;
  DevBuf<CandMeta> l_ccnt;
  DevBuf<uint64_t> l_cfirst;  // Lines::cand_first
  unsigned long long scan_stats[6] = {0, 0, 0, 0, 0, 0};
  uint64_t last_slow = 0;
  DevBuf<uint8_t> l_flags;
  DevBuf<unsigned long long> scalars;  // [0] slow count, [1..2] bounds, [3] selected
  DevBuf<uint64_t> res_seq;
  bool res_written = false;  // the last match phase wrote the RuleResult arrays
  DevBuf<uint32_t> res_rule, ev_el, ev_rule, ev_res, ev_st, ev_st2, ev_idx, ev_idx2, el_slot, coll, trip_idx;
  DevBuf<EvRec> ev_rec, ev_rec2;  // EvRec12 records when rec12 (the last rate-limit stage's form), from rec_base
  bool rec12 = false;
  int64_t rec_base = 0;
  DevBuf<uint32_t> el_id;
  DevBuf<uint32_t> blk_n;   // k_ip_firsts: first lines per block, then their exclusive scan
  DevBuf<uint64_t> blk_b;   // ... and their IP bytes
  DevBuf<uint8_t> rl_out, ev_out, ev_out_s, trip_flag;
  DevBuf<uint32_t> trip_ev, trip_ev2;
  DevBuf<uint64_t> tr_base;  // bjx_apply_events_trips: segment bases, trip bases, first trips
  DevBuf<bjx_trip> d_trips;
  DevBuf<bjx_rule_result> d_results;
  DevBuf<uint8_t> cub_tmp;
  DevBuf<int64_t> q_out;
  DevBuf<uint8_t> q_ip;

  // the batch between its match phase and its finish (bjx_match_batch / bjx_finish_batch)
  BatchCtx bc;
  // multi-GPU exchange workspace
  DevBuf<uint32_t> pack_src, rx_len, rx_ev_el;
  DevBuf<uint64_t> pk_hist, pk_off, pk_counts, pk_bbase, rx_hash, rx_pos, rx_nev, rx_evoff;
  DevBuf<int64_t> rx_ts;
  DevBuf<uint4> rx_ip16;  // received event lines: IpSlot.key16 of each IP (k_unpack_lines)
  uint32_t pk_parts = 0, pk_tiles = 0, pk_steps = 1;
  uint64_t pk_n_ev = 0;
  bool partitioned = false;

  // trip -> decision emission (bjx_engine_set_ban_options / bjx_batch_bans)
  int64_t ban_ttl_ns = 0;
  int32_t ban_tz = 0;
  DevBuf<int64_t> tz_at; DevBuf<int32_t> tz_off;
  uint32_t n_tz = 0;
  DevBuf<uint64_t> dl_hash; DevBuf<uint32_t> dl_off, dl_len; DevBuf<uint8_t> dl_bytes;
  uint32_t n_dl = 0;
  DevBuf<uint32_t> nm_off; DevBuf<uint8_t> nm_json;
  size_t nm_built = 0;
  DevBuf<uint64_t> bn_key, bn_key2, bn_len, bn_off;
  DevBuf<uint32_t> bn_val, bn_val2, bn_head, bn_seg, bn_first, bn_cnt, bn_ipt, bn_coll;
  DevBuf<unsigned long long> bn_best;
  DevBuf<uint8_t> bn_kind, bn_flag, bn_log;
  DevBuf<bjx_ip_decision> bn_rep, bn_sel;
  DevBuf<uint8_t> bn_ipb;
  bool ban_emitted = false;
  uint64_t ban_n_trips = 0;
  HostBuf<bjx_ip_decision> ban_ips;
  HostBuf<char> ban_log;
  HostBuf<uint64_t> ban_off;
  HostBuf<uint8_t> ban_kind;
  HostBuf<uint8_t> ban_ipb;
  HostBuf<uint64_t> ban_ipo;

  // host copies of the last batch
  HostBuf<bjx_trip> trips;
  HostBuf<uint64_t> trips_c;     // BJX_TRIPS_COMPACT words
  DevBuf<uint64_t> d_trips_c;
  HostBuf<bjx_rule_result> results;
  HostBuf<uint8_t> line_flags;
};

namespace {

uint32_t intern_name(bjx_engine *e, const std::string &n) {
  auto it = e->name_ids.find(n);
  if (it != e->name_ids.end()) return it->second;
  uint32_t id = (uint32_t)e->names.size();
  if (id >= (1u << 24)) throw BjxError(BJX_ERR_CAPACITY, "too many distinct rule names");
  e->names.push_back(n);
  e->name_ids.emplace(n, id);
  return id;
}

uint64_t be64_host(const uint8_t *a) {
  uint64_t v = 0;
  for (int k = 0; k < 8; ++k) v = (v << 8) | a[k];
  return v;
}

struct BlobBuilder {
  std::vector<uint8_t> bytes;
  template <typename T>
  size_t add(const std::vector<T> &v) {
    size_t off = (bytes.size() + 15) & ~size_t(15);
    bytes.resize(off + v.size() * sizeof(T) + 16, 0);
    if (!v.empty()) memcpy(bytes.data() + off, v.data(), v.size() * sizeof(T));
    return off;
  }
};

// net.ParseCIDR + IPNet/To4 handling of ipfilter's ToggleIP (allow entries)
bool parse_allow_entry(const std::string &s, std::vector<std::array<uint8_t, 16>> &addrs, std::vector<Subnet> &subs) {
  auto slash = s.find('/');
  const uint8_t *p = reinterpret_cast<const uint8_t *>(s.data());
  if (slash != std::string::npos) {
    uint8_t a[16];
    bool is4;
    std::string addr = s.substr(0, slash), mask = s.substr(slash + 1);
    if (!go_parse_addr(reinterpret_cast<const uint8_t *>(addr.data()), (uint32_t)addr.size(), a, &is4)) return false;
    if (addr.find('%') != std::string::npos) return false;
    long bits = 0;
    size_t i = 0;
    for (; i < mask.size() && mask[i] >= '0' && mask[i] <= '9'; ++i) {
      bits = bits * 10 + (mask[i] - '0');
      if (bits >= 0xFFFFFF) return false;
    }
    if (i == 0 || i != mask.size()) return false;
    const int bitlen = is4 ? 32 : 128;
    if (bits > bitlen) return false;
    if (bits == bitlen) {  // single address
      std::array<uint8_t, 16> x;
      memcpy(x.data(), a, 16);
      addrs.push_back(x);
      return true;
    }
    Subnet sn;
    memset(&sn, 0, sizeof sn);
    auto mk = [&](int k) -> uint8_t {
      int b = (int)bits - 8 * k;
      return b >= 8 ? 0xFF : (b <= 0 ? 0 : (uint8_t)(0xFF << (8 - b)));
    };
    if (is4) {
      sn.netlen = 4;
      for (int k = 0; k < 4; ++k) { sn.mask[k] = mk(k); sn.net[k] = a[12 + k] & sn.mask[k]; }
    } else {
      uint8_t net[16], m[16];
      for (int k = 0; k < 16; ++k) { m[k] = mk(k); net[k] = a[k] & m[k]; }
      if (is_v4_mapped(net)) { sn.netlen = 4; memcpy(sn.net, net + 12, 4); memcpy(sn.mask, m + 12, 4); }
      else { sn.netlen = 16; memcpy(sn.net, net, 16); memcpy(sn.mask, m, 16); }
    }
    subs.push_back(sn);
    return true;
  }
  uint8_t a[16];
  bool is4;
  if (go_parse_addr(p, (uint32_t)s.size(), a, &is4)) {
    std::array<uint8_t, 16> x;
    memcpy(x.data(), a, 16);
    addrs.push_back(x);
    return true;
  }
  return false;
}

// 4-byte value of literal window [o, o+4) in ASCII-case variant v (bit k set =
// upper-case byte k); false if v flips a case-sensitive byte.
static bool window_variant(const uint8_t *s, const uint8_t *ci, uint32_t v, uint32_t *g) {
  uint32_t x = 0;
  for (int k = 0; k < 4; ++k) {
    uint8_t c = s[k];
    if (ci[k]) c = ((v >> k) & 1) ? (uint8_t)(c & ~0x20) : c;
    else if ((v >> k) & 1) return false;
    x |= (uint32_t)c << (8 * k);
  }
  *g = x;
  return true;
}

// Gram calibration: for each literal pick the 4-byte window (all its ASCII-case
// variants) that occurs least often in a sample of the traffic being bound,
// ties going to the compiler's static choice.  Any window of a literal is a
// necessary condition for it, so the choice changes speed, never results.
// Also picks each literal's check window (the rarest other window, farthest
// from the gram on ties) that verification compares first.
static void calibrate_grams(const std::vector<uint8_t> &lit_bytes, const std::vector<uint8_t> &lit_ci,
                            const std::vector<uint32_t> &lit_off, const std::vector<uint32_t> &lit_len,
                            std::vector<uint32_t> &lit_gram, std::vector<uint8_t> &lit_chk, const uint8_t *sample,
                            size_t n) {
  lit_chk.assign(lit_off.size(), 0);
  for (size_t id = 0; id < lit_off.size(); ++id)
    lit_chk[id] = (uint8_t)(lit_gram[id] >= (lit_len[id] - 4) / 2 ? 0 : lit_len[id] - 4);
  if (n < 4 || lit_off.empty()) return;
  std::unordered_map<uint32_t, uint32_t> cnt;
  std::vector<uint64_t> seen(1u << 14, 0);  // 2^20-bit presence filter
  auto fh = [](uint32_t g) { return (g * 0x9E3779B1u) >> 12; };
  for (size_t id = 0; id < lit_off.size(); ++id)
    for (uint32_t o = 0; o + 4 <= lit_len[id]; ++o)
      for (uint32_t v = 0; v < 16; ++v) {
        uint32_t g;
        if (!window_variant(&lit_bytes[lit_off[id] + o], &lit_ci[lit_off[id] + o], v, &g)) continue;
        cnt.emplace(g, 0);
        seen[fh(g) >> 6] |= 1ull << (fh(g) & 63);
      }
  uint32_t g = 0;
  for (size_t i = 0; i < n; ++i) {
    g = (g >> 8) | ((uint32_t)sample[i] << 24);
    if (i < 3) continue;
    const uint32_t h = fh(g);
    if (!((seen[h >> 6] >> (h & 63)) & 1)) continue;
    auto it = cnt.find(g);
    if (it != cnt.end()) ++it->second;
  }
  // window choice: a gram hit costs one check per literal filed under that
  // gram, so a window costs (sample count + 1) x (literals sharing it).
  // Start from the rarest window of each literal, then a few rounds of
  // re-choosing each literal's window against the others' choices.
  auto variants = [&](size_t id, uint32_t o, uint32_t *out) {
    uint32_t k = 0;
    for (uint32_t v = 0; v < 16; ++v) {
      uint32_t x;
      if (window_variant(&lit_bytes[lit_off[id] + o], &lit_ci[lit_off[id] + o], v, &x)) out[k++] = x;
    }
    return k;
  };
  std::vector<std::vector<uint64_t>> wcs(lit_off.size());
  for (size_t id = 0; id < lit_off.size(); ++id) {
    std::vector<uint64_t> &wc = wcs[id];
    for (uint32_t o = 0; o + 4 <= lit_len[id]; ++o) {
      uint32_t vs[16];
      const uint32_t k = variants(id, o, vs);
      uint64_t c = 0;
      for (uint32_t i = 0; i < k; ++i) c += cnt[vs[i]];
      wc.push_back(c);
    }
    uint64_t best = ~0ull;
    uint32_t best_o = lit_gram[id];
    for (uint32_t o = 0; o < wc.size(); ++o) {
      const uint64_t c = 2 * wc[o] + (o == lit_gram[id] ? 0 : 1);
      if (c < best) { best = c; best_o = o; }
    }
    lit_gram[id] = best_o;
  }
  std::unordered_map<uint32_t, uint32_t> load;  // gram -> literals filed under it
  auto file = [&](size_t id, int d) {
    uint32_t vs[16];
    const uint32_t k = variants(id, lit_gram[id], vs);
    for (uint32_t i = 0; i < k; ++i) load[vs[i]] += d;
  };
  for (size_t id = 0; id < lit_off.size(); ++id) file(id, 1);
  for (int round = 0; round < 3; ++round)
    for (size_t id = 0; id < lit_off.size(); ++id) {
      file(id, -1);
      uint64_t best = ~0ull;
      uint32_t best_o = lit_gram[id];
      for (uint32_t o = 0; o + 4 <= lit_len[id]; ++o) {
        uint32_t vs[16];
        const uint32_t k = variants(id, o, vs);
        uint64_t c = 0;
        for (uint32_t i = 0; i < k; ++i) {
          auto it = load.find(vs[i]);
          c += (cnt[vs[i]] + 1) * (1 + (it == load.end() ? 0 : it->second));
        }
        c = 2 * c + (o == lit_gram[id] ? 0 : 1);  // ties keep the current window
        if (c < best) { best = c; best_o = o; }
      }
      lit_gram[id] = best_o;
      file(id, 1);
    }
  for (size_t id = 0; id < lit_off.size(); ++id) {
    const std::vector<uint64_t> &wc = wcs[id];
    const uint32_t best_o = lit_gram[id];
    uint64_t bc = ~0ull;
    for (uint32_t o = 0; o < wc.size(); ++o) {
      if (o == best_o && wc.size() > 1) continue;
      const uint32_t dist = o > best_o ? o - best_o : best_o - o;
      const uint64_t c = wc[o] * 256 + (255 - std::min<uint32_t>(dist, 255));
      if (c < bc) { bc = c; lit_chk[id] = (uint8_t)o; }
    }
  }
}

// The longest piece (>= 4 bytes) of a prefilter literal left when every
// occurrence of host h is cut out (ASCII-case-insensitive where the literal
// is); *off = its offset in the literal.  Any piece of a required literal is a
// required literal too, so the prefilter stays sound.
static bool split_at_host(const PrefLit &pl, const std::string &h, PrefLit *piece, uint32_t *off) {
  const size_t n = pl.s.size(), m = h.size();
  if (m == 0 || m > n) return false;
  auto at = [&](size_t i) {
    for (size_t k = 0; k < m; ++k) {
      const uint8_t c = (uint8_t)h[k];
      const uint8_t lc = (c >= 'A' && c <= 'Z') ? (uint8_t)(c | 0x20) : c;
      if (pl.ci[i + k] ? (uint8_t)pl.s[i + k] != lc : (uint8_t)pl.s[i + k] != c) return false;
    }
    return true;
  };
  size_t best_b = 0, best_n = 0, b = 0;
  bool cut = false;
  for (size_t i = 0; i + m <= n;) {
    if (at(i)) {
      if (i - b > best_n) { best_b = b; best_n = i - b; }
      b = i + m;
      i = b;
      cut = true;
    } else {
      ++i;
    }
  }
  if (!cut) return false;
  if (n - b > best_n) { best_b = b; best_n = n - b; }
  if (best_n < 4 || best_b > 255) return false;
  piece->s = pl.s.substr(best_b, best_n);
  piece->ci = pl.ci.substr(best_b, best_n);
  piece->gram_off = pl.gram_off >= best_b && pl.gram_off + 4 <= best_b + best_n ? pl.gram_off - (uint32_t)best_b : 0;
  *off = (uint32_t)best_b;
  return true;
}

void bind_ruleset(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *sample, size_t sample_n) {
  if (e->bound_uid == rs->uid && e->bound_dec_version == e->decisions_version) return;
  // DFA job keys: a rule id (windowed jobs r, legacy n_rules + r, null jobs
  // 2 n_rules) in the low 24 bits, the rule's position above them
  if (rs->rules.size() >= (1u << 23))
    throw BjxError(BJX_ERR_TOO_COMPLEX, "ruleset of 2^23 rules or more (DFA job keys hold 2 * n_rules in 24 bits)");
  // host dictionary: per-site hosts, skip hosts, allow-list sites
  std::map<std::string, uint32_t> hosts;
  auto host_id = [&](const std::string &h) {
    auto it = hosts.find(h);
    if (it != hosts.end()) return it->second;
    uint32_t id = (uint32_t)hosts.size();
    hosts.emplace(h, id);
    return id;
  };
  for (auto &s : rs->sites) host_id(s.first);
  for (auto &r : rs->rules)
    for (auto &h : r.skip_hosts) host_id(h);
  // scopes: 0 = global, then one per site that appears in the decision lists
  std::map<std::string, int32_t> scope_of_site;
  for (auto &d : e->decisions)
    if (!d.global && !scope_of_site.count(d.site)) {
      int32_t sc = (int32_t)scope_of_site.size() + 1;
      scope_of_site.emplace(d.site, sc);
      host_id(d.site);
    }
  const uint32_t n_hosts = (uint32_t)hosts.size();
  const uint32_t n_scopes = (uint32_t)scope_of_site.size() + 1;
  std::vector<std::string> host_by_id(n_hosts);
  for (auto &h : hosts) host_by_id[h.second] = h.first;

  // rules
  std::vector<DevRule> drules(rs->rules.size());
  std::vector<uint16_t> trans;
  std::vector<uint8_t> ae, ascii(rs->rules.size() * 128), lits;
  std::vector<uint32_t> nonascii;
  std::map<std::pair<std::string, std::string>, uint32_t> lit_ids;
  std::vector<uint8_t> lit_bytes, lit_ci;
  std::vector<uint32_t> lit_off, lit_len, lit_gram, rule_lits;
  std::vector<uint8_t> lit_pref;
  std::vector<uint64_t> nfa_blob;
  std::vector<uint32_t> accel;  // per DFA state (indexed like accept_end): self-loop acceleration
  std::vector<uint32_t> rule_full;  // per rule_lits entry: (full literal << 8 | piece offset) of a host-split literal
  std::vector<const std::string *> site_host(rs->rules.size(), nullptr);
  for (auto &st : rs->sites)
    for (uint32_t r : st.second) site_host[r] = &st.first;
  bool any_anchored = false;
  for (size_t i = 0; i < rs->rules.size(); ++i) {
    const auto &r = rs->rules[i];
    DevRule &d = drules[i];
    memset(&d, 0, sizeof d);
    d.trans_off = (uint32_t)trans.size();
    trans.insert(trans.end(), r.rx.trans.begin(), r.rx.trans.end());
    d.ae_off = (uint32_t)ae.size();
    ae.insert(ae.end(), r.rx.accept_end.begin(), r.rx.accept_end.end());
    // self-loop acceleration (dfa_text): a state that every ASCII byte but at
    // most 3 maps to itself is left only by those bytes or a non-ASCII one
    for (uint32_t st = 0; st < r.rx.accept_end.size(); ++st) {
      uint32_t a = 0;
      if (st > 1 && !(r.rx.flags & kRuleNfa) && !r.rx.trans.empty()) {
        uint32_t esc[3] = {0, 0, 0}, ne = 0;
        bool ok = true;
        for (uint32_t b = 0; b < 128 && ok; ++b)
          if (r.rx.trans[(size_t)st * r.rx.ncls + r.rx.ascii_cls[b]] != st) {
            if (ne == 3) ok = false;
            else esc[ne++] = b;
          }
        if (ok) a = 0x80000000u | (ne << 24) | (esc[2] << 16) | (esc[1] << 8) | esc[0];
      }
      accel.push_back(a);
    }
    d.na_off = (uint32_t)(nonascii.size() / 2);
    for (auto &p : r.rx.nonascii) { nonascii.push_back(p.first); nonascii.push_back(p.second); }
    d.n_na = (uint16_t)r.rx.nonascii.size();
    d.ncls = (uint16_t)r.rx.ncls;
    d.n_states = r.rx.nstates;
    d.start = r.rx.start;
    d.flags = (uint16_t)r.rx.flags;
    memcpy(&ascii[i * 128], r.rx.ascii_cls, 128);
    d.name_id = intern_name(e, r.name);
    d.decision = r.decision;
    d.mode = (uint8_t)r.rx.mode;
    d.equiv = r.rx.pref_equivalent ? 1 : 0;
    auto intern_lit = [&](const PrefLit &pl, bool pref) {
      auto key = std::make_pair(pl.s, pl.ci);
      auto it = lit_ids.find(key);
      uint32_t id;
      if (it != lit_ids.end()) id = it->second;
      else {
        id = (uint32_t)lit_off.size();
        lit_ids.emplace(key, id);
        lit_off.push_back((uint32_t)lit_bytes.size());
        lit_len.push_back((uint32_t)pl.s.size());
        lit_gram.push_back(pl.gram_off);
        lit_pref.push_back(0);
        lit_bytes.insert(lit_bytes.end(), pl.s.begin(), pl.s.end());
        lit_ci.insert(lit_ci.end(), pl.ci.begin(), pl.ci.end());
      }
      if (pref) { lit_pref[id] = 1; lit_gram[id] = pl.gram_off; }
      return id;
    };
    d.lits_off = (uint32_t)rule_lits.size();
    if (r.rx.mode == kModePrefilter)
      for (auto &pl : r.rx.pref) {
        // a per-site rule's literal that spells its own host (e.g. "GET <host> GET
        // /wp-login.php HTTP/") is filed under its longest host-free piece: the
        // piece is shared by every host's copy of the rule (one gram, one
        // verification), the line's host id picks the rule (lh_tab), and the full
        // literal is checked around the hit in k_lines
        PrefLit piece;
        uint32_t off = 0;
        if (site_host[i] && split_at_host(pl, *site_host[i], &piece, &off)) {
          const uint32_t full = intern_lit(pl, false);
          rule_lits.push_back(intern_lit(piece, true));
          rule_full.push_back((full << 8) | off);
        } else {
          rule_lits.push_back(intern_lit(pl, true));
          rule_full.push_back(kNone);
        }
      }
    d.lits_len = (uint16_t)(rule_lits.size() - d.lits_off);
    d.anc_off = (uint32_t)rule_lits.size();
    if (r.rx.mode == kModeAnchored)
      for (auto &pl : r.rx.anchor) { rule_lits.push_back(intern_lit(pl, false)); rule_full.push_back(kNone); }
    d.anc_len = (uint16_t)(rule_lits.size() - d.anc_off);
    d.anc_equiv = r.rx.anchor_equivalent ? 1 : 0;
    // bit 0: every match of the pattern begins with a literal of pref; bit 1:
    // this copy's literals are those (not host-split pieces): lead_start,
    // eq_certain
    d.lead = 0;
    if (r.rx.mode == kModePrefilter) {
      bool split = false;
      for (uint32_t k = d.lits_off; k < d.lits_off + d.lits_len; ++k) split = split || rule_full[k] != kNone;
      d.lead = (r.rx.pref_lead ? 1 : 0) | (split ? 0 : 2);
    }
    d.lead_dist = r.rx.pref_lead ? r.rx.lead_dist : 0;
    any_anchored = any_anchored || r.rx.mode == kModeAnchored;
    d.interval_ns = r.interval_ns;
    d.hits = r.hits;
    if (r.rx.flags & kRuleNfa) {
      d.nfa_off = (uint32_t)nfa_blob.size();
      d.nfa_words = r.rx.nfa_words;
      nfa_blob.insert(nfa_blob.end(), r.rx.nfa.begin(), r.rx.nfa.end());
    }
    // DFA jobs of an anchored rule exist only once its single prefix literal
    // matched at the start of rest (dfa_rule / plan_rule): when the literal is
    // case-sensitive ASCII, k_dfa starts past it in the state it leads to
    if (r.rx.mode == kModeAnchored && r.rx.anchor.size() == 1 && !(r.rx.flags & (kRuleNfa | kRuleAlways | kRuleNever)) &&
        !getenv("BJX_NO_DFA_SKIP")) {
      const PrefLit &al = r.rx.anchor[0];
      bool ok = !al.s.empty() && al.s.size() < 0x10000;
      uint32_t stt = r.rx.start;
      for (size_t k = 0; ok && k < al.s.size(); ++k) {
        const uint8_t c = (uint8_t)al.s[k];
        if (c >= 0x80 || al.ci[k]) { ok = false; break; }
        stt = r.rx.trans[(size_t)stt * r.rx.ncls + r.rx.ascii_cls[c]];
        if (stt <= 1) ok = false;  // decided inside the literal: no skip
      }
      if (ok) { d.skip_len = (uint16_t)al.s.size(); d.skip_state = (uint16_t)stt; }
    }
  }
  std::vector<uint8_t> lit_chk;
  calibrate_grams(lit_bytes, lit_ci, lit_off, lit_len, lit_gram, lit_chk, sample, sample_n);
  // gram filter: each literal's chosen 4-byte window, every ASCII case variant
  // of its case-insensitive bytes, -> bitset bit + exact table entry
  std::map<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>> gmap;
  for (uint32_t id = 0; id < lit_off.size(); ++id) {
    if (!lit_pref[id]) continue;
    const uint32_t o = lit_off[id] + lit_gram[id];
    for (uint32_t v = 0; v < 16; ++v) {
      uint32_t g;
      if (window_variant(&lit_bytes[o], &lit_ci[o], v, &g)) gmap[g].push_back({id, lit_gram[id]});
    }
  }
  // exact gram table: slot (key, entries offset << 16 | count), entries (lit << 8 | window offset)
  size_t n_gent = 0;
  for (auto &kv : gmap) n_gent += kv.second.size();
  const bool use_pref = n_gent > 0 && n_gent < 65536 && lit_off.size() < 65536;
  std::vector<uint32_t> gram_pairs(2 * kPairEntries, 0);
  const uint32_t gt2_cap = (uint32_t)next_pow2((use_pref ? gmap.size() : 0) * 2 + 16);
  std::vector<uint32_t> gt2(2 * gt2_cap, 0), gt2_ent;
  if (use_pref)
    for (auto &kv : gmap) {
      // both roles of the gram (k_scan tests even positions as the left gram
      // of a pair and odd ones as the right gram)
      const uint32_t g = kv.first;
      gram_pairs[2 * gram_pair_index(g >> 8)] |= 1u << (g & 31u);
      gram_pairs[2 * gram_pair_index(g & 0xFFFFFFu) + 1] |= 1u << ((g >> 24) & 31u);
      uint32_t slot = gram_slot(kv.first, gt2_cap);
      while (gt2[2 * slot + 1] & 0xFFFF) slot = (slot + 1) & (gt2_cap - 1);
      gt2[2 * slot] = kv.first;
      gt2[2 * slot + 1] = ((uint32_t)gt2_ent.size() << 16) | (uint32_t)kv.second.size();
      for (auto &en : kv.second) gt2_ent.push_back((en.first << 8) | en.second);
    }
  if (lit_bytes.empty()) { lit_bytes.push_back(0); lit_ci.push_back(0); }
  std::vector<uint32_t> global_rules(rs->n_global);
  for (uint32_t i = 0; i < rs->n_global; ++i) global_rules[i] = i;
  std::vector<uint32_t> site_off(n_hosts + 1, 0), site_rules;
  std::vector<std::vector<uint32_t>> per_host(n_hosts);
  for (auto &s : rs->sites) per_host[hosts[s.first]] = s.second;
  uint32_t max_app = rs->n_global;
  for (uint32_t h = 0; h < n_hosts; ++h) {
    site_off[h] = (uint32_t)site_rules.size();
    site_rules.insert(site_rules.end(), per_host[h].begin(), per_host[h].end());
    max_app = std::max<uint32_t>(max_app, (uint32_t)per_host[h].size() + rs->n_global);
  }
  site_off[n_hosts] = (uint32_t)site_rules.size();
  // host dict sorted by hash (+ open-addressing table over it for the scan pass)
  std::vector<std::pair<uint64_t, uint32_t>> hd;
  for (uint32_t h = 0; h < n_hosts; ++h)
    hd.push_back({hash_bytes(reinterpret_cast<const uint8_t *>(host_by_id[h].data()), (uint32_t)host_by_id[h].size()), h});
  std::sort(hd.begin(), hd.end());
  std::vector<uint64_t> hd_hash;
  std::vector<uint32_t> hd_id, hd_off, hd_len;
  std::vector<uint8_t> hd_bytes;
  for (auto &p : hd) {
    hd_hash.push_back(p.first);
    hd_id.push_back(p.second);
    hd_off.push_back((uint32_t)hd_bytes.size());
    hd_len.push_back((uint32_t)host_by_id[p.second].size());
    hd_bytes.insert(hd_bytes.end(), host_by_id[p.second].begin(), host_by_id[p.second].end());
  }
  const uint32_t ht_cap = (uint32_t)next_pow2(std::max<size_t>(64, 2 * hd.size()));
  std::vector<uint32_t> ht(2 * ht_cap, 0);
  for (uint32_t i = 0; i < hd.size(); ++i) {
    uint32_t slot = (uint32_t)hd[i].first & (ht_cap - 1);
    while (ht[2 * slot]) slot = (slot + 1) & (ht_cap - 1);
    ht[2 * slot] = (uint32_t)(hd[i].first >> 32) | 1u;
    ht[2 * slot + 1] = i;
  }
  std::vector<HostSlot> hslot(ht_cap);
  memset(hslot.data(), 0, hslot.size() * sizeof(HostSlot));
  for (uint32_t i = 0; i < hd.size(); ++i) {
    uint32_t slot = (uint32_t)hd[i].first & (ht_cap - 1);
    while (hslot[slot].tag) slot = (slot + 1) & (ht_cap - 1);
    HostSlot &hs = hslot[slot];
    hs.tag = (uint32_t)(hd[i].first >> 32) | 1u;
    hs.id = (int32_t)hd[i].second;
    hs.len = hd_len[i];
    hs.off = hd_off[i];
    memcpy(hs.inl, hd_bytes.data() + hd_off[i], std::min<uint32_t>(hd_len[i], 48));
  }
  // compact host dictionary for k_lines' LDS (host_lookup_lds)
  std::vector<uint32_t> hl;
  {
    size_t nbytes = 0;
    bool ok = n_hosts < 0xFFFF;
    for (uint32_t h = 0; h < n_hosts; ++h) {
      ok = ok && host_by_id[h].size() < 0xFFFF;
      nbytes += ((host_by_id[h].size() + 3) & ~size_t(3)) + 4;
    }
    const size_t words = 2 + 2 * (size_t)ht_cap + n_hosts + nbytes / 4;
    // (a ruleset without hosts keeps the empty dictionary: every lookup
    // returns -1, and k_lines2 runs the global rules' decision class)
    if (ok && words * 4 <= kLinesHostLdsMax && !getenv("BJX_NO_HOST_LDS")) {
      hl.assign(words, 0);
      hl[0] = ht_cap;
      hl[1] = n_hosts;
      // slots by host_fold (the per-line pass's cheap dictionary hash)
      for (uint32_t h = 0; h < n_hosts; ++h) {
        const std::string &hs = host_by_id[h];
        const uint32_t tg = host_fold(reinterpret_cast<const uint8_t *>(hs.data()), (uint32_t)hs.size());
        uint32_t sl = tg & (ht_cap - 1);
        while (hl[2 + 2 * sl]) sl = (sl + 1) & (ht_cap - 1);
        hl[2 + 2 * sl] = tg;
        hl[2 + 2 * sl + 1] = (h << 16) | (uint32_t)hs.size();
      }
      uint8_t *by = reinterpret_cast<uint8_t *>(hl.data() + 2 + 2 * ht_cap + n_hosts);
      uint32_t o = 0;
      for (uint32_t h = 0; h < n_hosts; ++h) {
        hl[2 + 2 * ht_cap + h] = o;
        memcpy(by + o, host_by_id[h].data(), host_by_id[h].size());
        o += (uint32_t)(((host_by_id[h].size() + 3) & ~size_t(3)) + 4);
      }
    }
  }
  uint32_t hl_bytes = (uint32_t)(hl.size() * 4);
  if (hl.empty()) hl.push_back(0);
  std::vector<int32_t> host_scope(n_hosts, -1);
  for (auto &s : scope_of_site) host_scope[hosts[s.first]] = s.second;
  std::vector<uint64_t> skip;
  for (size_t i = 0; i < rs->rules.size(); ++i)
    for (auto &h : rs->rules[i].skip_hosts) skip.push_back(((uint64_t)i << 32) | hosts[h]);
  std::sort(skip.begin(), skip.end());
  skip.erase(std::unique(skip.begin(), skip.end()), skip.end());

  // scan-pass rule tables: per scope (host, or n_hosts = none) ALWAYS / skip
  // masks over applicable positions < 128; rules needing a DFA on every line;
  // literal rules; and literal -> rules requiring it
  auto mode_of = [&](uint32_t r) {
    const RuleMode m = rs->rules[r].rx.mode;
    return (m == kModePrefilter && !use_pref) ? kModeScan : m;
  };
  auto equiv_of = [&](uint32_t r) { return rs->rules[r].rx.pref_equivalent ? 0x80000000u : 0u; };
  // rules with the same pattern have the same automaton, anchors and literals:
  // the DFA-side entries below name the first rule of each pattern, so the DFA
  // jobs (sorted by that id) of, e.g., a per-site rule repeated on every host
  // form one run and k_dfa stages its transition table once per block
  std::vector<uint32_t> canon(rs->rules.size());
  {
    std::unordered_map<std::string, uint32_t> first;
    for (uint32_t r = 0; r < (uint32_t)rs->rules.size(); ++r) canon[r] = first.emplace(rs->rules[r].regex, r).first->second;
  }
  std::vector<uint64_t> sc_always(2 * (n_hosts + 1), 0), sc_skipm(2 * (n_hosts + 1), 0);
  for (uint32_t sc = 0; sc <= n_hosts; ++sc) {
    const uint32_t nsite = sc < n_hosts ? (uint32_t)per_host[sc].size() : 0;
    for (uint32_t pos = 0; pos < nsite + rs->n_global && pos < 128; ++pos) {
      const uint32_t r = pos < nsite ? per_host[sc][pos] : pos - nsite;
      if (mode_of(r) == kModeAlways) sc_always[2 * sc + pos / 64] |= 1ull << (pos % 64);
      if (sc < n_hosts && std::binary_search(skip.begin(), skip.end(), ((uint64_t)r << 32) | sc))
        sc_skipm[2 * sc + pos / 64] |= 1ull << (pos % 64);
    }
  }
  std::vector<uint32_t> dfa_site_off(n_hosts + 1, 0), pref_site_off(n_hosts + 1, 0);
  std::vector<uint2> dfa_site, pref_site, dfa_glob, pref_glob;
  for (uint32_t h = 0; h < n_hosts; ++h) {
    dfa_site_off[h] = (uint32_t)dfa_site.size();
    pref_site_off[h] = (uint32_t)pref_site.size();
    for (uint32_t k = 0; k < per_host[h].size(); ++k) {
      const uint32_t r = per_host[h][k];
      const RuleMode m = mode_of(r);
      if (m == kModeAnchored || m == kModeScan) dfa_site.push_back(make_uint2(canon[r], k));
      else if (m == kModePrefilter) pref_site.push_back(make_uint2(canon[r], k));
    }
  }
  dfa_site_off[n_hosts] = (uint32_t)dfa_site.size();
  pref_site_off[n_hosts] = (uint32_t)pref_site.size();
  std::vector<uint32_t> alw_site_off(n_hosts + 1, 0), alw_site, alw_glob;
  for (uint32_t h = 0; h < n_hosts; ++h) {
    alw_site_off[h] = (uint32_t)alw_site.size();
    for (uint32_t k = 0; k < per_host[h].size(); ++k)
      if (mode_of(per_host[h][k]) == kModeAlways) alw_site.push_back(k);
  }
  alw_site_off[n_hosts] = (uint32_t)alw_site.size();
  for (uint32_t g = 0; g < rs->n_global; ++g)
    if (mode_of(g) == kModeAlways) alw_glob.push_back(g);
  for (uint32_t g = 0; g < rs->n_global; ++g) {
    const RuleMode m = mode_of(g);
    if (m == kModeAnchored || m == kModeScan) dfa_glob.push_back(make_uint2(canon[g], g));
    else if (m == kModePrefilter) pref_glob.push_back(make_uint2(canon[g], g));
  }
  // inline anchor tests (anchor_quick) of the dfa_site / dfa_glob entries
  auto anchor_q = [&](const std::vector<uint2> &ents) {
    std::vector<uint4> q;
    for (const uint2 &en : ents) {
      uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
      const DevRule &d = drules[en.x];
      if (mode_of(en.x) == kModeAnchored && d.anc_len == 1) {
        const uint32_t lit = rule_lits[d.anc_off], len = lit_len[lit];
        const uint32_t o = len > 8 ? len - 8 : 0, nb = std::min(8u, len);
        if (len > 0 && o < 256) {
          uint8_t bw[8] = {0}, mw[8] = {0};
          for (uint32_t k = 0; k < nb; ++k) {
            bw[k] = lit_bytes[lit_off[lit] + o + k];
            mw[k] = lit_ci[lit_off[lit] + o + k] ? 0x20 : 0;
          }
          a.x = len;
          a.y = o | ((len <= 8 ? 1u : 0u) << 8) | ((d.anc_equiv ? 1u : 0u) << 9);
          memcpy(&a.z, mw, 4); memcpy(&a.w, mw + 4, 4); memcpy(&b.x, bw, 4); memcpy(&b.y, bw + 4, 4);
        }
      }
      q.push_back(a);
      q.push_back(b);
    }
    return q;
  };
  const std::vector<uint4> dfa_site_q = anchor_q(dfa_site), dfa_glob_q = anchor_q(dfa_glob);
  const uint32_t n_lit = (uint32_t)lit_off.size();
  std::vector<std::vector<uint2>> lr_g(n_lit);
  std::vector<std::vector<std::pair<int32_t, uint3>>> lr_s(n_lit);
  if (use_pref) {
    for (uint32_t g = 0; g < rs->n_global; ++g)
      if (mode_of(g) == kModePrefilter)
        for (uint32_t i = drules[g].lits_off; i < drules[g].lits_off + drules[g].lits_len; ++i)
          lr_g[rule_lits[i]].push_back(make_uint2(canon[g] | equiv_of(g), g));
    for (uint32_t h = 0; h < n_hosts; ++h)
      for (uint32_t k = 0; k < per_host[h].size(); ++k) {
        const uint32_t r = per_host[h][k];
        if (mode_of(r) != kModePrefilter) continue;
        for (uint32_t i = drules[r].lits_off; i < drules[r].lits_off + drules[r].lits_len; ++i)
          lr_s[rule_lits[i]].push_back({(int32_t)h, make_uint3(canon[r] | equiv_of(r), k, rule_full[i])});
      }
  }
  std::vector<uint32_t> lr_off(n_lit + 1, 0), lr_gend(std::max<uint32_t>(1, n_lit), 0);
  std::vector<uint2> lr_ent;
  std::vector<uint32_t> lr_full;
  std::vector<int32_t> lr_host;
  for (uint32_t l = 0; l < n_lit; ++l) {
    lr_off[l] = (uint32_t)lr_ent.size();
    for (auto &x : lr_g[l]) { lr_ent.push_back(x); lr_host.push_back(-1); lr_full.push_back(kNone); }
    lr_gend[l] = (uint32_t)lr_ent.size();
    std::stable_sort(lr_s[l].begin(), lr_s[l].end(),
                     [](const std::pair<int32_t, uint3> &a, const std::pair<int32_t, uint3> &b) { return a.first < b.first; });
    for (auto &x : lr_s[l]) {
      lr_ent.push_back(make_uint2(x.second.x, x.second.y));
      lr_full.push_back(x.second.z);
      lr_host.push_back(x.first);
    }
  }
  lr_off[n_lit] = (uint32_t)lr_ent.size();
  // (literal, host) -> run of that host's site entries (one probe per hit in
  // decide_rules instead of a binary search over lr_host)
  uint32_t lh_n = 0;
  for (uint32_t l = 0; l < n_lit; ++l)
    for (uint32_t i = lr_gend[l]; i < lr_off[l + 1]; ++i) lh_n += (i == lr_gend[l] || lr_host[i] != lr_host[i - 1]);
  uint32_t lh_cap = 16;
  while (lh_cap < 2 * lh_n) lh_cap <<= 1;
  std::vector<uint4> lh_tab(lh_cap, make_uint4(0, 0, 0, 0));
  for (uint32_t l = 0; l < n_lit; ++l)
    for (uint32_t i = lr_gend[l]; i < lr_off[l + 1];) {
      uint32_t k = i;
      while (k < lr_off[l + 1] && lr_host[k] == lr_host[i]) ++k;
      uint32_t s = lit_host_slot(l, (uint32_t)lr_host[i], lh_cap);
      while (lh_tab[s].x) s = (s + 1) & (lh_cap - 1);
      lh_tab[s] = make_uint4(l + 1, (uint32_t)lr_host[i], i, k);
      i = k;
    }

  // rule plans (decide_plan): every non-ALWAYS, non-NEVER rule of a scope at
  // a position < 128, with its decision inputs inline
  const bool use_plan = rs->rules.size() < (1u << 20) && lit_off.size() < 0xFFFF;
  auto plan_entry = [&](uint32_t r, uint32_t pos, std::vector<uint4> &out) {
    const RuleMode m = mode_of(r);
    if (m == kModeAlways || m == kModeNever) return;
    const DevRule &d = drules[r];
    uint4 a = make_uint4(0, 0, 0, 0), b = make_uint4(0, 0, 0, 0);
    uint32_t kind = kPlanScan, eq = 0;
    if (m == kModeAnchored) {
      kind = kPlanAnchor;
      eq = d.anc_equiv ? 1u : 0u;
      const std::vector<uint4> q = anchor_q(std::vector<uint2>{make_uint2(r, 0)});
      a.y = q[0].x; a.z = q[0].y; b.x = q[0].z; b.y = q[0].w; b.z = q[1].x; b.w = q[1].y;
      a.w = d.anc_len == 1 && lit_len[rule_lits[d.anc_off]] < 0x10000u
                ? (rule_lits[d.anc_off] + 1) | (lit_len[rule_lits[d.anc_off]] << 16) : 0u;
    } else if (m == kModePrefilter) {
      eq = rs->rules[r].rx.pref_equivalent ? 1u : 0u;
      const uint32_t nl = d.lits_len;
      bool split = false;
      for (uint32_t i = 0; i < nl; ++i) split = split || rule_full[d.lits_off + i] != kNone;
      if (nl == 0 || nl > 4 || (split && nl > 1)) {
        kind = kPlanLitAny;  // a DFA job on any hit: the automaton decides exactly
      } else {
        kind = kPlanLit;
        uint32_t l[4] = {0xFFFF, 0xFFFF, 0xFFFF, 0xFFFF};
        for (uint32_t i = 0; i < nl; ++i) l[i] = rule_lits[d.lits_off + i];
        a.y = l[0] | (l[1] << 16);
        a.z = l[2] | (l[3] << 16);
        a.w = split ? rule_full[d.lits_off] : kNone;
        b.y = split ? lit_len[rule_full[d.lits_off] >> 8] : 0u;
      }
    }
    a.x = canon[r] | (pos << 20) | (kind << 27) | (eq << 30);
    out.push_back(a);
    out.push_back(b);
  };
  std::vector<uint32_t> plan_off(n_hosts + 1, 0);
  std::vector<uint4> plan, plan_glob;
  if (use_plan) {
    for (uint32_t h = 0; h < n_hosts; ++h) {
      plan_off[h] = (uint32_t)(plan.size() / 2);
      for (uint32_t k = 0; k < per_host[h].size() && k < 128; ++k) plan_entry(per_host[h][k], k, plan);
    }
    plan_off[n_hosts] = (uint32_t)(plan.size() / 2);
    for (uint32_t g = 0; g < rs->n_global && g < 128; ++g) plan_entry(g, g, plan_glob);
  }
  if (plan.empty()) plan.push_back(make_uint4(0, 0, 0, 0));
  if (plan_glob.empty()) plan_glob.push_back(make_uint4(0, 0, 0, 0));

  std::vector<uint8_t> shared_pat(rs->rules.size(), 0);  // some other rule has this rule's pattern
  for (uint32_t r = 0; r < (uint32_t)rs->rules.size(); ++r)
    if (canon[r] != r) shared_pat[canon[r]] = 1;
  // plan classes for k_lines' LDS (decide_plan_lds), appended to the host
  // dictionary blob when both fit kLinesTabLdsMax
  uint32_t lt_hinfo = 0, lt_cls = 0, lt_trec = 0, lt_pool = 0;
  uint32_t l2_hdc = 0, l2_dcls = 0, l2_none = 0, l2_bytes = 0;  // k_lines2 tables (0 bytes: not eligible)
  uint32_t l2_w = 1;  // their mask width in 64-bit words
  if (use_plan && hl_bytes && !getenv("BJX_NO_PLAN_LDS")) {
    std::vector<uint2> hinfo(n_hosts, make_uint2(0, 0));
    std::vector<uint4> cls, trec;
    std::vector<uint8_t> pool;
    std::map<std::vector<uint32_t>, uint32_t> cls_ids;
    std::map<std::tuple<std::string, std::string, std::string, std::string, uint32_t>, uint32_t> tmpl_ids;
    // F = A + host + C with the host spelled exactly once, case-sensitively:
    // its template id (side 1: the prefilter piece is C), or -1
    auto tmpl_of = [&](uint32_t lit, const std::string &h, uint32_t side) -> int32_t {
      const std::string s((const char *)&lit_bytes[lit_off[lit]], lit_len[lit]);
      const std::string ci((const char *)&lit_ci[lit_off[lit]], lit_len[lit]);
      size_t at = std::string::npos, n_at = 0;
      for (size_t i = 0; i + h.size() <= s.size(); ++i) {
        bool eq = true, cs = true;
        for (size_t k = 0; k < h.size() && eq; ++k) {
          const uint8_t c = (uint8_t)h[k], lc = (c >= 'A' && c <= 'Z') ? (uint8_t)(c | 0x20) : c;
          eq = ci[i + k] ? (uint8_t)s[i + k] == lc : (uint8_t)s[i + k] == c;
          cs = cs && !ci[i + k];
        }
        if (!eq) continue;
        ++n_at;
        at = i;
        if (!cs) n_at = 99;
      }
      if (n_at != 1 || h.empty()) return -1;
      const std::string A = s.substr(0, at), Aci = ci.substr(0, at), C = s.substr(at + h.size()),
                        Cci = ci.substr(at + h.size());
      if (A.size() > 255 || C.size() > 255) return -1;
      auto key = std::make_tuple(A, Aci, C, Cci, side);
      auto it = tmpl_ids.find(key);
      if (it != tmpl_ids.end()) return (int32_t)it->second;
      auto put_str = [&](const std::string &b, const std::string &m) {
        const uint32_t off = (uint32_t)pool.size(), pad = (uint32_t)((b.size() + 3) & ~size_t(3)) + 4;
        pool.resize(off + 2 * pad, 0);
        for (size_t k = 0; k < b.size(); ++k) {
          pool[off + k] = (uint8_t)b[k];
          pool[off + pad + k] = m[k] ? 0x20 : 0;
        }
        return off;
      };
      const uint32_t oa = put_str(A, Aci), oc = put_str(C, Cci);
      const uint32_t id = (uint32_t)trec.size();
      trec.push_back(make_uint4((uint32_t)A.size() | ((uint32_t)C.size() << 8) | (side << 16), oa, oc, 0));
      tmpl_ids.emplace(key, id);
      return (int32_t)id;
    };
    for (uint32_t h = 0; h < n_hosts; ++h) {
      std::vector<uint4> ents;
      const std::string &hn = host_by_id[h];
      for (uint32_t k = 0; k < per_host[h].size() && k < 128; ++k) {
        const uint32_t r = per_host[h][k];
        const size_t at = ents.size();
        plan_entry(r, k, ents);
        if (ents.size() == at) continue;
        uint4 &a = ents[at], &b = ents[at + 1];
        const uint32_t kind = (a.x >> 27) & 7u;
        const DevRule &d = drules[r];
        if (kind == kPlanAnchor && d.anc_len == 1) {
          const int32_t t = tmpl_of(rule_lits[d.anc_off], hn, 0);
          if (t >= 0) {
            a = make_uint4((a.x & ~(7u << 27)) | (kPlanAnchorT << 27), 0, 0, (uint32_t)t);
            b = make_uint4(0, 0, 0, 0);
          }
        } else if (kind == kPlanLit && a.w != kNone) {
          const uint32_t full = a.w >> 8, off = a.w & 0xFF, piece = rule_lits[d.lits_off];
          const uint32_t side = off == 0 ? 0u : 1u;
          const int32_t t = tmpl_of(full, hn, side);
          // the piece must be all of A (side 0) or all of C (side 1)
          const bool whole = t >= 0 && (side == 0 ? (trec[t].x & 0xFF) == lit_len[piece]
                                                  : ((trec[t].x >> 8) & 0xFF) == lit_len[piece] &&
                                                        off == (trec[t].x & 0xFF) + hn.size());
          if (whole) {
            a = make_uint4((a.x & ~(7u << 27)) | (kPlanLitT << 27), a.y, a.z, (uint32_t)t);
            b = make_uint4(0, 0, 0, 0);
          }
        }
        // "own" only for a pattern no other rule shares (a shared pattern is
        // named by its first rule on every host alike, so hosts whose rules
        // differ only in their host name keep one class)
        if (canon[r] == r && !shared_pat[r] && r == per_host[h][0] + k) a.x = (a.x & ~0xFFFFFu) | kPlanOwn;
      }
      std::vector<uint32_t> key;
      for (auto &v : ents) { key.push_back(v.x); key.push_back(v.y); key.push_back(v.z); key.push_back(v.w); }
      auto it = cls_ids.find(key);
      uint32_t off;
      if (it != cls_ids.end()) off = it->second;
      else {
        off = (uint32_t)(cls.size() / 2);
        cls.insert(cls.end(), ents.begin(), ents.end());
        cls_ids.emplace(key, off);
      }
      hinfo[h] = make_uint2(off | ((uint32_t)(ents.size() / 2) << 16), per_host[h].empty() ? 0u : per_host[h][0]);
    }
    const uint32_t w0 = ((uint32_t)hl.size() + 3) & ~3u, w_hi = w0, w_cls = (w_hi + 2 * n_hosts + 3) & ~3u,
                   w_tr = w_cls + 4 * (uint32_t)cls.size(), w_pool = w_tr + 4 * (uint32_t)trec.size(),
                   w_end = w_pool + (uint32_t)((pool.size() + 3) / 4);
    if (cls.size() / 2 < 0xFFFF && (size_t)w_end * 4 <= kLinesTabLdsMax) {
      hl.resize(w_end, 0);
      memcpy(hl.data() + w_hi, hinfo.data(), hinfo.size() * 8);
      if (!cls.empty()) memcpy(hl.data() + w_cls, cls.data(), cls.size() * 16);
      if (!trec.empty()) memcpy(hl.data() + w_tr, trec.data(), trec.size() * 16);
      if (!pool.empty()) memcpy(hl.data() + w_pool, pool.data(), pool.size());
      hl_bytes = w_end * 4;
      lt_hinfo = w_hi; lt_cls = w_cls; lt_trec = w_tr; lt_pool = w_pool;
    }
    // k_lines2 decision tables (lines2.h), appended to the blob after what
    // k_lines reads: per decision class (site plan class, site rules, ALWAYS
    // and hosts_to_skip masks) the per-literal rows, their checks, the rule of
    // each position and the anchored / no-literal entries
    // W 64-bit words of position bits cover the ruleset's widest scope (at
    // most 128 positions: the plan entries hold a 7-bit position); one row per
    // prefilter literal id (the literals a hit can carry)
    const uint32_t l2w = max_app <= 64 ? 1u : 2u;
    uint32_t n_lrows = 0;  // rows for literal ids up to the largest prefilter one
    for (uint32_t id = 0; id < lit_pref.size(); ++id)
      if (lit_pref[id]) n_lrows = id + 1;
    if (lt_cls && max_app <= 128 && !getenv("BJX_NO_LINES2")) {
      const uint32_t DW = l2_dcls_words(l2w), RW = l2_row_words(l2w), NP = 64 * l2w;
      using Mask = std::array<uint64_t, 2>;
      struct Dc {
        std::vector<Mask> eq, job, lm;
        std::vector<std::vector<uint4>> chk;
        std::vector<uint32_t> prule;
        std::vector<uint32_t> anc;  // kL2AncWords per entry
        Mask alw{}, skp{}, anyhit{}, anyovf{}, lmbig{};
      };
      std::vector<Dc> dcs;
      std::map<std::tuple<uint32_t, uint32_t, uint64_t, uint64_t, uint64_t, uint64_t>, uint32_t> dc_ids;
      const uint32_t n_glob_ent = (uint32_t)(plan_glob.size() / 2);
      bool ok = true;
      auto set = [](Mask &m, uint32_t p) { m[p >> 6] |= 1ull << (p & 63); };
      auto add_entry = [&](Dc &D, uint4 a, const uint4 b, uint32_t p) {
        const uint32_t kind = (a.x >> 27) & 7u, eq = (a.x >> 30) & 1u;
        if (p >= NP) { ok = false; return; }
        a.x = (a.x & ~(0x7Fu << 20)) | (p << 20);
        D.prule[p] = a.x;
        auto ids = [&](auto fn) {
          const uint32_t l4[4] = {a.y & 0xFFFFu, a.y >> 16, a.z & 0xFFFFu, a.z >> 16};
          for (uint32_t l : l4)
            if (l != 0xFFFFu) {
              if (l >= n_lrows) { ok = false; continue; }
              fn(l);
            }
        };
        if (kind == kPlanLit) {
          ids([&](uint32_t l) {
            set(D.lm[l], p);
            if (l >= 32) set(D.lmbig, p);
            if (a.w == kNone) set(eq ? D.eq[l] : D.job[l], p);
            else if (!eq) set(D.job[l], p);
            else {
              const uint32_t off = a.w & 0xFFu, flen = b.y;
              D.chk[l].push_back(make_uint4(p | (kL2ChkFull << 8) | (1u << 10), a.w, flen, flen > off ? flen - off : 0u));
            }
          });
        } else if (kind == kPlanLitT) {
          const uint4 rec = trec[a.w];
          const uint32_t la = rec.x & 0xFF, lc = (rec.x >> 8) & 0xFF, side = (rec.x >> 16) & 1u;
          ids([&](uint32_t l) {
            set(D.lm[l], p);
            if (l >= 32) set(D.lmbig, p);
            D.chk[l].push_back(make_uint4(p | (kL2ChkTmpl << 8) | (eq << 10) | ((side ? 0u : 1u) << 11), a.w, 0u,
                                          side ? lc : la + lc));
          });
        } else if (kind == kPlanLitAny) {
          set(D.anyhit, p);
          set(D.anyovf, p);
        } else {  // kPlanAnchor, kPlanAnchorT, kPlanScan: the bytes of rest each may read
          uint32_t ext = 0;
          if (kind == kPlanAnchorT) {
            const uint4 rec = trec[a.w];
            ext = ((rec.x & 0xFF) + ((rec.x >> 8) & 0xFF)) | 0x80000000u;
          } else if (kind == kPlanAnchor) {
            ext = std::max<uint32_t>((a.z & 0xFFu) + 8, a.w >> 16);
            const uint32_t r = a.x & 0xFFFFFu;
            for (uint32_t i = 0; i < drules[r].anc_len; ++i) ext = std::max<uint32_t>(ext, lit_len[rule_lits[drules[r].anc_off + i]]);
          }
          if (ext & 0x40000000u) ok = false;
          const uint32_t w[kL2AncWords] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, ext, 0, 0, 0};
          D.anc.insert(D.anc.end(), w, w + kL2AncWords);
        }
      };
      auto dc_of = [&](uint32_t ci, uint32_t n_ent, uint32_t nsite, uint32_t sc) {
        const Mask alw{sc_always[2 * sc], sc_always[2 * sc + 1]}, skp{sc_skipm[2 * sc], sc_skipm[2 * sc + 1]};
        const auto key = std::make_tuple(ci | (n_ent << 16), nsite, alw[0], alw[1], skp[0], skp[1]);
        auto it = dc_ids.find(key);
        if (it != dc_ids.end()) return it->second;
        Dc D;
        D.eq.assign(n_lrows, Mask{}); D.job.assign(n_lrows, Mask{}); D.lm.assign(n_lrows, Mask{});
        D.chk.assign(n_lrows, {});
        D.prule.assign(NP, 0);
        D.alw = alw;
        D.skp = skp;
        for (uint32_t e = 0; e < n_ent; ++e) add_entry(D, cls[2 * (ci + e)], cls[2 * (ci + e) + 1], (cls[2 * (ci + e)].x >> 20) & 0x7Fu);
        for (uint32_t g = 0; g < n_glob_ent; ++g)
          add_entry(D, plan_glob[2 * g], plan_glob[2 * g + 1], nsite + ((plan_glob[2 * g].x >> 20) & 0x7Fu));
        const uint32_t id = (uint32_t)dcs.size();
        dcs.push_back(std::move(D));
        dc_ids.emplace(key, id);
        return id;
      };
      std::vector<uint32_t> hdc(n_hosts, 0);
      for (uint32_t h = 0; h < n_hosts; ++h)
        hdc[h] = dc_of(hinfo[h].x & 0xFFFFu, hinfo[h].x >> 16, (uint32_t)per_host[h].size(), h);
      const uint32_t none = dc_of(0xFFFFu, 0, 0, n_hosts);
      // layout (words, 16 B aligned pieces)
      std::vector<uint32_t> t(((hl.size() + 3) & ~size_t(3)), 0);
      std::copy(hl.begin(), hl.end(), t.begin());
      auto al4 = [&]() { t.resize((t.size() + 3) & ~size_t(3), 0); return (uint32_t)t.size(); };
      auto put = [&](uint32_t at, const Mask &m) {
        for (uint32_t k = 0; k < l2w; ++k) { t[at + 2 * k] = (uint32_t)m[k]; t[at + 2 * k + 1] = (uint32_t)(m[k] >> 32); }
      };
      const uint32_t w_hdc = al4();
      t.insert(t.end(), hdc.begin(), hdc.end());
      const uint32_t w_dc = al4();
      t.resize(t.size() + (size_t)DW * dcs.size(), 0);
      for (uint32_t d = 0; d < dcs.size() && ok; ++d) {
        Dc &D = dcs[d];
        const uint32_t w_rows = al4();
        t.resize(t.size() + (size_t)RW * n_lrows, 0);
        for (uint32_t l = 0; l < n_lrows; ++l) {
          const uint32_t w_ck = al4();
          for (const uint4 &c : D.chk[l]) { t.push_back(c.x); t.push_back(c.y); t.push_back(c.z); t.push_back(c.w); }
          const uint32_t r = w_rows + RW * l;
          put(r, D.eq[l]); put(r + 2 * l2w, D.job[l]); put(r + 4 * l2w, D.lm[l]);
          t[r + 6 * l2w] = w_ck; t[r + 6 * l2w + 1] = (uint32_t)D.chk[l].size();
        }
        const uint32_t w_pr = al4();
        t.insert(t.end(), D.prule.begin(), D.prule.end());
        const uint32_t w_anc = al4();
        t.insert(t.end(), D.anc.begin(), D.anc.end());
        const uint32_t rec = w_dc + DW * d;
        put(rec, D.alw); put(rec + 2 * l2w, D.skp); put(rec + 4 * l2w, D.anyhit); put(rec + 6 * l2w, D.anyovf);
        put(rec + 8 * l2w, D.lmbig);
        t[rec + 10 * l2w] = w_rows; t[rec + 10 * l2w + 1] = w_pr; t[rec + 10 * l2w + 2] = w_anc;
        t[rec + 10 * l2w + 3] = (uint32_t)(D.anc.size() / kL2AncWords);
        if ((size_t)t.size() * 4 > kL2TabMax) ok = false;  // stop laying out tables that cannot be used
      }
      al4();
      // inline DFAs (l2_inline): a position whose rule is anchored at the
      // start of rest (its automaton decides within a few dozen bytes, inside
      // the window; rules that look for a literal anywhere mostly decide past
      // it: at cfg3 inlining those cost k_lines2 2.9 ms and saved 1 % of the
      // jobs) and whose automaton is small (< 256 states, no NFA) gets its
      // next-state table over ASCII bytes
      // (u8 [state][128]) and its accept-at-end flags in the blob, so a job of
      // that rule is run in k_lines2 over the line's window when the window
      // holds the decision; kPlanOwn positions (a different rule per host) and
      // tables past kL2TabMax keep their jobs
      {
        // the inline tables may not cost k_lines2 a block per CU: they fit
        // what two blocks (8 waves and their windows each) leave of the CU's
        // LDS, when the tables before them did
        const size_t two_blocks = kScanLdsMax / 2 - (size_t)(kL2Block / 64) * kL2WaveLds;
        const size_t inl_max = t.size() * 4 <= two_blocks ? std::min<size_t>(kL2TabMax, two_blocks) : (size_t)kL2TabMax;
        std::map<uint32_t, uint32_t> inl_of;  // rule -> entry word offset (0: not inline)
        // The automaton of rule r from its skip state (past its anchored
        // literal prefix) over ASCII, renumbered canonically (dead 0, accept
        // 1, the others in breadth-first order from the skip state, which is
        // 2): rules that differ only in their prefix give equal tables.
        // Empty when r does not qualify or the sub-automaton has 256 states.
        auto suffix_dfa = [&](uint32_t r, std::vector<uint8_t> &tab, std::vector<uint8_t> &ae) {
          tab.clear();
          ae.clear();
          if (r >= drules.size()) return;
          const DevRule &dr = drules[r];
          const CompiledRegex &rx = rs->rules[r].rx;
          if (dr.mode != kModeAnchored || !dr.skip_len || (dr.flags & (kRuleNfa | kRuleNfaWide | kRuleAlways | kRuleNever)) ||
              dr.skip_state <= kAccept || rx.trans.size() < (size_t)dr.n_states * dr.ncls)
            return;
          std::unordered_map<uint32_t, uint32_t> id{{kDead, kDead}, {kAccept, kAccept}};
          std::vector<uint32_t> order{kDead, kAccept, dr.skip_state};
          id[dr.skip_state] = 2;
          for (size_t k = 2; k < order.size(); ++k) {
            if (order.size() > 255) { tab.clear(); ae.clear(); return; }
            const uint32_t st = order[k];
            for (uint32_t b = 0; b < 128; ++b) {
              const uint32_t nx = rx.trans[(size_t)st * dr.ncls + rx.ascii_cls[b]];
              if (!id.count(nx)) { id[nx] = (uint32_t)order.size(); order.push_back(nx); }
            }
          }
          if (order.size() > 255) return;
          tab.assign(order.size() * 128, 0);
          ae.assign(order.size(), 0);
          for (size_t k = 2; k < order.size(); ++k) {
            for (uint32_t b = 0; b < 128; ++b) tab[k * 128 + b] = (uint8_t)id[rx.trans[(size_t)order[k] * dr.ncls + rx.ascii_cls[b]]];
            ae[k] = rx.accept_end[order[k]] ? 1 : 0;
          }
          ae[kAccept] = 1;
        };
        std::map<std::vector<uint8_t>, uint32_t> own_of;  // canonical suffix table (+ flags) -> entry word offset
        auto own_suffix = [&](uint32_t d, uint32_t p) -> uint32_t {
          std::vector<uint8_t> key, tab, ae;
          for (uint32_t h = 0; h < n_hosts; ++h) {
            if (hdc[h] != d) continue;
            suffix_dfa(hinfo[h].y + p, tab, ae);
            if (tab.empty()) return 0;
            std::vector<uint8_t> k2 = tab;
            k2.insert(k2.end(), ae.begin(), ae.end());
            if (key.empty()) key.swap(k2);
            else if (k2 != key) return 0;
          }
          if (key.empty()) return 0;
          auto it = own_of.find(key);
          if (it != own_of.end()) return it->second;
          const uint32_t ns = (uint32_t)(tab.size() / 128);
          const size_t need = 16 + (size_t)ns * 128 + ((ns + 3) & ~3u) + 16;
          uint32_t at = 0;
          if ((t.size() + 4) * 4 + need + 256 <= inl_max) {
            at = al4();
            t.resize(t.size() + 4, 0);
            const uint32_t w_tr = al4();
            t.resize(t.size() + (size_t)ns * 32, 0);
            memcpy(reinterpret_cast<uint8_t *>(t.data() + w_tr), tab.data(), tab.size());
            const uint32_t w_ae = al4();
            t.resize(t.size() + (ns + 3) / 4, 0);
            memcpy(reinterpret_cast<uint8_t *>(t.data() + w_ae), ae.data(), ae.size());
            // no start state: only jobs that begin past the prefix run here
            t[at] = w_tr * 4; t[at + 1] = w_ae * 4; t[at + 2] = kL2NoStart; t[at + 3] = 2;
          }
          own_of.emplace(key, at);
          return at;
        };
        for (uint32_t d = 0; d < dcs.size() && ok; ++d) {
          Dc &D = dcs[d];
          std::vector<uint32_t> pin(NP, 0);
          bool any = false;
          for (uint32_t p = 0; p < NP; ++p) {
            const uint32_t w = D.prule[p];
            if (!w) continue;
            if (w & kPlanOwn) {
              // a different rule per host (its own host spelled in an anchored
              // prefix): inline when every host of the class has the same
              // automaton past its prefix, for the jobs that start there
              const uint32_t e = own_suffix(d, p);
              pin[p] = e;
              any = any || e != 0;
              continue;
            }
            const uint32_t r = w & 0xFFFFFu;
            if (r >= drules.size()) continue;
            auto it = inl_of.find(r);
            if (it == inl_of.end()) {
              const DevRule &dr = drules[r];
              const CompiledRegex &rx = rs->rules[r].rx;
              uint32_t at = 0;
              const size_t need = 16 + (size_t)dr.n_states * 128 + ((dr.n_states + 3) & ~3u) + 16;
              // anchored rules, and lead rules (jobs start at a literal's first
              // hit) whose automaton has no state past the start that waits on
              // most bytes (a .* after the literal: a failing run would walk on)
              auto scans_on = [&]() {
                if (rx.trans.size() < (size_t)dr.n_states * dr.ncls) return true;
                for (uint32_t st = 2; st < dr.n_states; ++st) {
                  if (st == dr.start) continue;
                  uint32_t self = 0;
                  for (uint32_t b = 0; b < 128; ++b) self += rx.trans[(size_t)st * dr.ncls + rx.ascii_cls[b]] == st;
                  if (self >= 64) return true;
                }
                return false;
              };
              if ((dr.mode == kModeAnchored || ((dr.lead & 3u) == 3u && !scans_on())) &&
                  !(dr.flags & (kRuleNfa | kRuleNfaWide | kRuleAlways | kRuleNever)) &&
                  dr.n_states >= 2 && dr.n_states < 256 &&
                  rx.trans.size() >= (size_t)dr.n_states * dr.ncls && (t.size() + 4) * 4 + need + 256 <= inl_max) {
                at = al4();
                t.resize(t.size() + 4, 0);
                const uint32_t w_tr = al4();
                t.resize(t.size() + (size_t)dr.n_states * 32, 0);
                uint8_t *tb = reinterpret_cast<uint8_t *>(t.data() + w_tr);
                for (uint32_t st = 0; st < dr.n_states; ++st)
                  for (uint32_t b = 0; b < 128; ++b) tb[st * 128 + b] = (uint8_t)rx.trans[(size_t)st * dr.ncls + rx.ascii_cls[b]];
                const uint32_t w_ae = al4();
                t.resize(t.size() + (dr.n_states + 3) / 4, 0);
                uint8_t *ab = reinterpret_cast<uint8_t *>(t.data() + w_ae);
                for (uint32_t st = 0; st < dr.n_states; ++st) ab[st] = rx.accept_end[st] ? 1 : 0;
                t[at] = w_tr * 4; t[at + 1] = w_ae * 4; t[at + 2] = dr.start; t[at + 3] = dr.skip_len ? dr.skip_state : dr.start;
              }
              it = inl_of.emplace(r, at).first;
            }
            pin[p] = it->second;
            any = any || it->second != 0;
          }
          if (!any || (t.size() + NP + 4) * 4 > inl_max) continue;
          const uint32_t w_pin = al4();
          t.insert(t.end(), pin.begin(), pin.end());
          t[w_dc + DW * d + 10 * l2w + 4] = w_pin;
        }
        al4();
      }
      if (ok && t.size() * 4 <= kL2TabMax) {
        l2_hdc = w_hdc; l2_dcls = w_dc; l2_none = none;
        l2_bytes = (uint32_t)(t.size() * 4);
        l2_w = l2w;
        hl.swap(t);
      }
      if (getenv("BJX_DEBUG_IMG"))
        fprintf(stderr, "[bjx] k_lines2 tables (%u-word masks): %zu decision classes, %zu B (%s)\n", l2w, dcs.size(),
                (l2_bytes ? hl.size() : t.size()) * 4, l2_bytes ? "on" : "off");
    }
    if (getenv("BJX_DEBUG_IMG"))
      fprintf(stderr, "[bjx] plan classes: %zu entries, %zu templates, pool %zu B, LDS tables %u B (%s)\n", cls.size() / 2,
              trec.size(), pool.size(), w_end * 4, lt_cls ? "in LDS" : "too large");
  }

  // allow scopes (decision.go:278-374): exact maps are last-writer-wins in
  // config order; Allow IPFilters hold every allow entry
  std::vector<std::vector<std::array<uint8_t, 16>>> sc_addrs(n_scopes);
  std::vector<std::vector<Subnet>> sc_subs(n_scopes);
  std::vector<std::map<std::string, int32_t>> sc_exact(n_scopes);
  bool any_allow = false;
  for (auto &d : e->decisions) {
    const int sc = d.global ? 0 : scope_of_site[d.site];
    if (d.ip.find('/') == std::string::npos) sc_exact[sc][d.ip] = d.decision;
    if (d.decision == BJX_ALLOW) {
      any_allow = true;
      parse_allow_entry(d.ip, sc_addrs[sc], sc_subs[sc]);
    }
  }
  std::vector<uint32_t> sc_addr_off(n_scopes + 1, 0), sc_sub_off(n_scopes + 1, 0), sc_str_off(n_scopes + 1, 0);
  std::vector<uint64_t> sc_addr, sc_str_hash;
  std::vector<Subnet> sc_sub;
  std::vector<uint32_t> sc_str_boff, sc_str_len;
  std::vector<uint8_t> sc_str_bytes;
  for (uint32_t sc = 0; sc < n_scopes; ++sc) {
    auto &v = sc_addrs[sc];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    sc_addr_off[sc] = (uint32_t)(sc_addr.size() / 2);
    for (auto &a : v) { sc_addr.push_back(be64_host(a.data())); sc_addr.push_back(be64_host(a.data() + 8)); }
    sc_sub_off[sc] = (uint32_t)sc_sub.size();
    sc_sub.insert(sc_sub.end(), sc_subs[sc].begin(), sc_subs[sc].end());
    sc_str_off[sc] = (uint32_t)sc_str_hash.size();
    std::vector<std::pair<uint64_t, std::string>> strs;
    for (auto &kv : sc_exact[sc]) {
      if (kv.second != BJX_ALLOW) continue;
      uint8_t a[16];
      bool is4;
      if (go_parse_addr(reinterpret_cast<const uint8_t *>(kv.first.data()), (uint32_t)kv.first.size(), a, &is4)) continue;
      strs.push_back({hash_bytes(reinterpret_cast<const uint8_t *>(kv.first.data()), (uint32_t)kv.first.size()), kv.first});
      any_allow = true;
    }
    std::sort(strs.begin(), strs.end());
    for (auto &p : strs) {
      sc_str_hash.push_back(p.first);
      sc_str_boff.push_back((uint32_t)sc_str_bytes.size());
      sc_str_len.push_back((uint32_t)p.second.size());
      sc_str_bytes.insert(sc_str_bytes.end(), p.second.begin(), p.second.end());
    }
  }
  sc_addr_off[n_scopes] = (uint32_t)(sc_addr.size() / 2);
  sc_sub_off[n_scopes] = (uint32_t)sc_sub.size();
  sc_str_off[n_scopes] = (uint32_t)sc_str_hash.size();

  // lookup image (LDS-resident in the scan pass when it fits)
  std::vector<uint8_t> img;
  auto put = [&](const void *p, size_t nbytes) {
    const size_t off = (img.size() + 15) & ~size_t(15);
    img.resize(off + nbytes + 4, 0);
    if (nbytes) memcpy(img.data() + off, p, nbytes);
    return (uint32_t)off;
  };
  std::vector<uint64_t> hrec(hd.size());
  for (size_t i = 0; i < hd.size(); ++i) hrec[i] = ((uint64_t)hd_off[i] << 32) | hd_len[i];
  // literals 4-byte aligned (+4 bytes of slack) with their case masks
  std::vector<uint32_t> lrec(lit_off.size());
  std::vector<uint8_t> lb_al, cm_al;
  for (size_t i = 0; i < lit_off.size(); ++i) {
    const uint32_t off = (uint32_t)lb_al.size();
    lrec[i] = (off << 8) | lit_len[i];
    for (uint32_t k = 0; k < lit_len[i]; ++k) {
      lb_al.push_back(lit_bytes[lit_off[i] + k]);
      cm_al.push_back(lit_ci[lit_off[i] + k] ? 0x20 : 0);
    }
    const size_t padded = ((lb_al.size() + 3) & ~size_t(3)) + 4;
    lb_al.resize(padded, 0);
    cm_al.resize(padded, 0);
  }
  ImgLayout il;
  il.gt = put(gt2.data(), gt2.size() * 4);
  il.ge = put(gt2_ent.data(), gt2_ent.size() * 4);
  il.ht = put(ht.data(), ht.size() * 4);
  il.hrec = put(hrec.data(), hrec.size() * 8);
  il.hid = put(hd_id.data(), hd_id.size() * 4);
  il.hbytes = put(hd_bytes.data(), hd_bytes.size());
  il.lrec = put(lrec.data(), lrec.size() * 4);
  il.lbytes = put(lb_al.data(), lb_al.size());
  il.lcim = put(cm_al.data(), cm_al.size());
  il.lchk = put(lit_chk.data(), lit_chk.size());
  img.resize((img.size() + 15) & ~size_t(15), 0);
  // the scan's own image: only what k_scan reads (gram table, gram entries,
  // the prefilter literals; the gram entries name prefilter literals only),
  // so it fits LDS beside the pair table whatever the ruleset's other literals
  std::vector<uint8_t> simg;
  auto sput = [&](const void *p, size_t nbytes) {
    const size_t off = (simg.size() + 15) & ~size_t(15);
    simg.resize(off + nbytes + 4, 0);
    if (nbytes) memcpy(simg.data() + off, p, nbytes);
    return (uint32_t)off;
  };
  std::vector<uint32_t> slrec(lit_off.size(), 0);
  std::vector<uint8_t> slb, scm;
  for (size_t i = 0; i < lit_off.size(); ++i) {
    if (!lit_pref[i]) continue;
    slrec[i] = ((uint32_t)slb.size() << 8) | lit_len[i];
    for (uint32_t k = 0; k < lit_len[i]; ++k) {
      slb.push_back(lit_bytes[lit_off[i] + k]);
      scm.push_back(lit_ci[lit_off[i] + k] ? 0x20 : 0);
    }
    const size_t padded = ((slb.size() + 3) & ~size_t(3)) + 4;
    slb.resize(padded, 0);
    scm.resize(padded, 0);
  }
  ImgLayout sil{};
  sil.gt = sput(gt2.data(), gt2.size() * 4);
  sil.ge = sput(gt2_ent.data(), gt2_ent.size() * 4);
  sil.lrec = sput(slrec.data(), slrec.size() * 4);
  sil.lbytes = sput(slb.data(), slb.size());
  sil.lcim = sput(scm.data(), scm.size());
  sil.lchk = sput(lit_chk.data(), lit_chk.size());
  simg.resize((simg.size() + 15) & ~size_t(15), 0);
  if (getenv("BJX_DEBUG_IMG"))
    fprintf(stderr, "[bjx] image %zu B: gram table %u, gram entries %u, host table %u, literals %zu (recs %u, bytes %zu x2), "
            "plan %zu entries, lit-rule ents %zu, hosts %zu\n", img.size(), il.ge - il.gt, il.ht - il.ge, il.lrec - il.ht,
            img.size() - il.lrec, il.lbytes - il.lrec, lb_al.size(), plan.size() / 2, lr_ent.size(), hd.size());

  // per rule, what k_lines2 needs to work out a job's window (l2_job_rec):
  // {literal-id mask (ids < 32), flags | lead_dist << 16, skip_len, 0}
  std::vector<uint4> jinfo(drules.size());
  for (size_t r = 0; r < drules.size(); ++r) {
    const DevRule &d = drules[r];
    uint32_t lm = 0, big = 0;
    for (uint32_t k = 0; k < d.lits_len; ++k) {
      const uint32_t id = rule_lits[d.lits_off + k];
      if (id < 32) lm |= 1u << id; else big = 1;
    }
    jinfo[r] = make_uint4(lm, ((d.flags & kRuleNfa) ? kJiNfa : 0u) | (d.equiv ? kJiEquiv : 0u) | ((uint32_t)(d.lead & 3u) << 2) |
                                  (big ? kJiBigLit : 0u) | ((uint32_t)d.lead_dist << 16),
                          d.skip_len, 0u);
  }
  BlobBuilder bb;
  size_t o_jinfo = bb.add(jinfo);
  size_t o_rules = bb.add(drules), o_trans = bb.add(trans), o_ae = bb.add(ae), o_accel = bb.add(accel), o_ascii = bb.add(ascii),
         o_na = bb.add(nonascii), o_lits = bb.add(lits), o_glob = bb.add(global_rules), o_soff = bb.add(site_off),
         o_srules = bb.add(site_rules), o_hdh = bb.add(hd_hash), o_hdid = bb.add(hd_id), o_hdoff = bb.add(hd_off),
         o_hdlen = bb.add(hd_len), o_hdb = bb.add(hd_bytes), o_hsc = bb.add(host_scope), o_skip = bb.add(skip),
         o_sao = bb.add(sc_addr_off), o_sa = bb.add(sc_addr), o_sso = bb.add(sc_sub_off), o_ss = bb.add(sc_sub),
         o_sto = bb.add(sc_str_off), o_sth = bb.add(sc_str_hash), o_stb = bb.add(sc_str_boff), o_stl = bb.add(sc_str_len),
         o_stbytes = bb.add(sc_str_bytes), o_gbits = bb.add(gram_pairs),
         o_rl = bb.add(rule_lits), o_img = bb.add(img), o_simg = bb.add(simg), o_lro = bb.add(lr_off), o_lrg = bb.add(lr_gend),
         o_lre = bb.add(lr_ent), o_lrh = bb.add(lr_host), o_sca = bb.add(sc_always), o_scs = bb.add(sc_skipm),
         o_dso = bb.add(dfa_site_off), o_ds = bb.add(dfa_site), o_dg = bb.add(dfa_glob), o_pso = bb.add(pref_site_off),
         o_dsq = bb.add(dfa_site_q), o_dgq = bb.add(dfa_glob_q),
         o_ps = bb.add(pref_site), o_pg = bb.add(pref_glob), o_hslot = bb.add(hslot), o_lh = bb.add(lh_tab),
         o_aso = bb.add(alw_site_off), o_as = bb.add(alw_site), o_ag = bb.add(alw_glob),
         o_nfa = bb.add(nfa_blob), o_lrf = bb.add(lr_full), o_plan = bb.add(plan), o_plo = bb.add(plan_off),
         o_plg = bb.add(plan_glob), o_hl = bb.add(hl);
  e->bind_blob.ensure(bb.bytes.size());
  HIP_OK(hipMemcpy(e->bind_blob.p, bb.bytes.data(), bb.bytes.size(), hipMemcpyHostToDevice));
  uint8_t *base = e->bind_blob.p;
  Bind &B = e->bind;
  B.rules = reinterpret_cast<const DevRule *>(base + o_rules);
  B.jinfo = reinterpret_cast<const uint4 *>(base + o_jinfo);
  B.trans = reinterpret_cast<const uint16_t *>(base + o_trans);
  B.accept_end = base + o_ae;
  B.accel = reinterpret_cast<const uint32_t *>(base + o_accel);
  B.ascii_cls = base + o_ascii;
  B.nonascii = reinterpret_cast<const uint32_t *>(base + o_na);
  B.lits = base + o_lits;
  B.global_rules = reinterpret_cast<const uint32_t *>(base + o_glob);
  B.site_off = reinterpret_cast<const uint32_t *>(base + o_soff);
  B.site_rules = reinterpret_cast<const uint32_t *>(base + o_srules);
  B.hd_hash = reinterpret_cast<const uint64_t *>(base + o_hdh);
  B.hd_id = reinterpret_cast<const uint32_t *>(base + o_hdid);
  B.hd_off = reinterpret_cast<const uint32_t *>(base + o_hdoff);
  B.hd_len = reinterpret_cast<const uint32_t *>(base + o_hdlen);
  B.hd_bytes = base + o_hdb;
  B.hslot = reinterpret_cast<const HostSlot *>(base + o_hslot);
  B.host_scope = reinterpret_cast<const int32_t *>(base + o_hsc);
  B.skip_keys = reinterpret_cast<const uint64_t *>(base + o_skip);
  B.sc_addr_off = reinterpret_cast<const uint32_t *>(base + o_sao);
  B.sc_addr = reinterpret_cast<const uint64_t *>(base + o_sa);
  B.sc_sub_off = reinterpret_cast<const uint32_t *>(base + o_sso);
  B.sc_sub = reinterpret_cast<const Subnet *>(base + o_ss);
  B.sc_str_off = reinterpret_cast<const uint32_t *>(base + o_sto);
  B.sc_str_hash = reinterpret_cast<const uint64_t *>(base + o_sth);
  B.sc_str_boff = reinterpret_cast<const uint32_t *>(base + o_stb);
  B.sc_str_len = reinterpret_cast<const uint32_t *>(base + o_stl);
  B.sc_str_bytes = base + o_stbytes;
  B.n_rules = (uint32_t)rs->rules.size();
  B.n_global = rs->n_global;
  B.n_hosts = n_hosts;
  B.n_hd = (uint32_t)hd.size();
  B.n_skip = (uint32_t)skip.size();
  B.n_scopes = n_scopes;
  B.any_allow = any_allow ? 1 : 0;
  B.mask_words = std::max<uint32_t>(1, (max_app + 63) / 64);
  B.gram_pairs = reinterpret_cast<const uint2 *>(base + o_gbits);
  B.rule_lits = reinterpret_cast<const uint32_t *>(base + o_rl);
  B.n_lits = n_lit;
  B.any_anchored = any_anchored ? 1 : 0;
  B.any_prefilter = use_pref ? 1 : 0;
  B.lit_nl = std::find(lit_bytes.begin(), lit_bytes.end(), (uint8_t)'\n') != lit_bytes.end() ? 1u : 0u;
  B.lits_small = lit_off.size() <= 32 ? 1u : 0u;
  B.cfirst = lit_off.size() <= kCandFirstLits && use_pref ? 1u : 0u;
  B.img = base + o_img;
  B.img_bytes = (uint32_t)img.size();
  B.il = il;
  B.scan_img = base + o_simg;
  B.scan_img_bytes = (uint32_t)simg.size();
  B.sil = sil;
  B.gt2_cap = gt2_cap;
  B.gt2_nent = (uint32_t)gt2_ent.size();
  B.ht_cap = ht_cap;
  B.max_app = max_app;
  B.lr_off = reinterpret_cast<const uint32_t *>(base + o_lro);
  B.lr_gend = reinterpret_cast<const uint32_t *>(base + o_lrg);
  B.lr_ent = reinterpret_cast<const uint2 *>(base + o_lre);
  B.lr_host = reinterpret_cast<const int32_t *>(base + o_lrh);
  B.lr_full = reinterpret_cast<const uint32_t *>(base + o_lrf);
  B.lh_tab = reinterpret_cast<const uint4 *>(base + o_lh);
  B.lh_cap = lh_cap;
  B.hl = reinterpret_cast<const uint32_t *>(base + o_hl);
  B.hl_bytes = hl_bytes;
  B.lt_hinfo = lt_hinfo; B.lt_cls = lt_cls; B.lt_trec = lt_trec; B.lt_pool = lt_pool;
  B.l2_hdc = l2_hdc; B.l2_dcls = l2_dcls; B.l2_none = l2_none; B.l2_bytes = l2_bytes; B.l2_w = l2_w;
  {
    // k_dfa stages the block's rule in LDS when it fits: size that LDS by the
    // ruleset's largest DFA, not the cap, so smaller rulesets run more blocks
    uint32_t tr = 0, acc = 0;
    for (const DevRule &d : drules) {
      if (d.flags & kRuleNfa) continue;
      const uint32_t ne = (uint32_t)d.ncls * d.n_states;
      if (ne <= kDfaLdsEntries) tr = std::max(tr, ne);
      if (d.n_states <= kDfaAccelLds) acc = std::max(acc, d.n_states);
    }
    B.dfa_tr = tr;
    B.dfa_acc = acc;
    B.dfa_lds = ((tr * 2 + 15) & ~15u) + acc * 4 + 128;
  }
  B.plan = reinterpret_cast<const uint4 *>(base + o_plan);
  B.plan_off = reinterpret_cast<const uint32_t *>(base + o_plo);
  B.plan_glob = reinterpret_cast<const uint4 *>(base + o_plg);
  B.n_plan_glob = use_plan ? (uint32_t)(plan_glob.size() / 2) : 0u;
  B.use_plan = use_plan && !getenv("BJX_NO_PLAN") ? 1u : 0u;
  B.sc_always = reinterpret_cast<const uint64_t *>(base + o_sca);
  B.sc_skip = reinterpret_cast<const uint64_t *>(base + o_scs);
  B.dfa_site_off = reinterpret_cast<const uint32_t *>(base + o_dso);
  B.dfa_site = reinterpret_cast<const uint2 *>(base + o_ds);
  B.dfa_glob = reinterpret_cast<const uint2 *>(base + o_dg);
  B.n_dfa_glob = (uint32_t)dfa_glob.size();
  B.dfa_site_q = reinterpret_cast<const uint4 *>(base + o_dsq);
  B.dfa_glob_q = reinterpret_cast<const uint4 *>(base + o_dgq);
  B.pref_site_off = reinterpret_cast<const uint32_t *>(base + o_pso);
  B.pref_site = reinterpret_cast<const uint2 *>(base + o_ps);
  B.pref_glob = reinterpret_cast<const uint2 *>(base + o_pg);
  B.n_pref_glob = (uint32_t)pref_glob.size();
  B.alw_site_off = reinterpret_cast<const uint32_t *>(base + o_aso);
  B.alw_site = reinterpret_cast<const uint32_t *>(base + o_as);
  B.alw_glob = reinterpret_cast<const uint32_t *>(base + o_ag);
  B.n_alw_glob = (uint32_t)alw_glob.size();
  B.nfa = reinterpret_cast<const uint64_t *>(base + o_nfa);
  B.any_nfa = nfa_blob.empty() ? 0 : 1;
  B.any_wide = 0;
  for (const auto &rr : rs->rules) B.any_wide |= (rr.rx.flags & kRuleNfaWide) ? 1u : 0u;
  // DFA jobs name the first rule of each pattern (canon): those of the NFA rules
  e->nfa_rules.clear();
  e->wide_max_w = e->wide_max_g = e->n_wide = 0;
  for (uint32_t r = 0; r < (uint32_t)rs->rules.size(); ++r)
    if (canon[r] == r && (rs->rules[r].rx.flags & kRuleNfa) && !(rs->rules[r].rx.flags & (kRuleAlways | kRuleNever))) {
      const CompiledRegex &rx = rs->rules[r].rx;
      if (rx.flags & kRuleNfaWide) {
        const uint32_t ng = reinterpret_cast<const uint32_t *>(rx.nfa.data())[3];
        e->nfa_rules.push_back(make_uint4(r, rx.nfa_words, ng, 1));
        e->wide_max_w = std::max(e->wide_max_w, rx.nfa_words);
        e->wide_max_g = std::max(e->wide_max_g, ng);
        ++e->n_wide;
      } else {
        e->nfa_rules.push_back(make_uint4(r, rx.nfa_words, (uint32_t)rx.nfa.size(), 0));
      }
    }
  e->host_rules = drules;
  {
    // the state-slot cache follows the first global rule that matches every line
    uint32_t hot = kNone;
    for (uint32_t g = 0; g < rs->n_global && hot == kNone; ++g)
      if (rs->rules[g].rx.mode == kModeAlways) hot = drules[g].name_id;
    // on by default (-0.9 ms of claim at cfg3; full GPU suite green with it and
    // BJX_CHECK=1, profiles/r03_final2/slot_cache.md); BJX_SLOT_CACHE=0 turns it off
    static const bool slot_cache_env = !(getenv("BJX_SLOT_CACHE") && atoi(getenv("BJX_SLOT_CACHE")) == 0);
    const bool slot_cache = e->dbg_slot_cache < 0 ? slot_cache_env : e->dbg_slot_cache != 0;
    if (!slot_cache || e->st_cap > (1ull << 32)) hot = kNone;
    if (hot != e->S.hot_name && e->S.ip_st) HIP_OK(hipMemsetAsync(e->S.ip_st, 0xFF, e->S.ip_st_cap * 4, e->stream));
    e->S.hot_name = hot;
  }
  e->bound_uid = rs->uid;
  e->bound_dec_version = e->decisions_version;
}

void alloc_state(bjx_engine *e, uint64_t ip_cap, uint64_t st_cap, uint64_t arena_cap) {
  State &S = e->S;
  HIP_OK(hipMalloc(&S.ip, ip_cap * sizeof(IpSlot)));
  HIP_OK(hipMalloc(&S.ip_first, ip_cap * 4));
  HIP_OK(hipMalloc(&S.ip_off, ip_cap * 8));
  HIP_OK(hipMalloc(&S.ip_len, ip_cap * 4));
  HIP_OK(hipMalloc(&S.arena, arena_cap));
  HIP_OK(hipMalloc(&S.st, st_cap * sizeof(StSlot)));
  HIP_OK(hipMalloc(&S.counters, kCounterBytes));
  HIP_OK(hipMemset(S.ip, 0, ip_cap * sizeof(IpSlot)));
  HIP_OK(hipMemset(S.ip_first, 0xFF, ip_cap * 4));
  HIP_OK(hipMemset(S.st, 0, st_cap * sizeof(StSlot)));
  HIP_OK(hipMemset(S.counters, 0, kCounterBytes));
  HIP_OK(hipMalloc(&S.ip_st, ip_cap * 4));
  HIP_OK(hipMemset(S.ip_st, 0xFF, ip_cap * 4));
  S.ip_st_cap = ip_cap;
  S.hot_name = kNone;
  S.ip_mask = ip_cap - 1;
  S.st_mask = st_cap - 1;
  S.arena_cap = arena_cap;
  e->ip_cap = ip_cap;
  e->st_cap = st_cap;
}

void free_state(bjx_engine *e) {
  State &S = e->S;
  for (void *p : {(void *)S.ip, (void *)S.ip_first, (void *)S.ip_off, (void *)S.ip_len, (void *)S.arena, (void *)S.st,
                  (void *)S.counters, (void *)S.ip_st})
    if (p) (void)hipFree(p);
  S = State{};
}

// the sorted records' event index words and their stride, in the form the
// last rate-limit stage used
static const uint32_t *ev_words(const bjx_engine *e) {
  return reinterpret_cast<const uint32_t *>(e->ev_rec2.p) + (e->rec12 ? 2 : 3);
}
static uint32_t rec_stride(const bjx_engine *e) { return e->rec12 ? 3u : 4u; }

// Small device -> host reads: pin_get queues a copy into the engine's pinned
// ring (the value lands in dst at the next pin_sync, which waits for the
// stream once for every read queued)
void pin_sync(bjx_engine *e) {
  HIP_OK(hipStreamSynchronize(e->stream));
  for (uint32_t k = 0; k < e->pin_n; ++k) memcpy(e->pin_q[k].dst, e->pin_q[k].slot, e->pin_q[k].n);
  e->pin_n = 0;
  e->pin_used = 0;
}
void pin_get(bjx_engine *e, void *dst, const void *src, size_t n) {
  if (n > bjx_engine::kPinBytes) throw BjxError(BJX_ERR_DEVICE, "internal: pinned read too large");
  if (e->pin_n == bjx_engine::kPinReads || e->pin_used + n > bjx_engine::kPinBytes) pin_sync(e);
  uint8_t *slot = e->pin + e->pin_used;
  e->pin_used = (uint32_t)((e->pin_used + n + 15) & ~size_t(15));
  HIP_OK(hipMemcpyAsync(slot, src, n, hipMemcpyDeviceToHost, e->stream));
  e->pin_q[e->pin_n++] = {dst, slot, (uint32_t)n};
}

void read_counters(bjx_engine *e) {
  pin_get(e, e->host_counters, e->S.counters, 24);
  pin_sync(e);
}

// rehash the IP table into one that holds `want` IPs under a 3/4 load factor
void grow_ip(bjx_engine *e, uint64_t want) {
  State &S = e->S;
  const uint64_t n_ips = e->host_counters[0];
  const uint64_t cap = next_pow2(want * 4 / 3 + 1024);
  if (cap <= e->ip_cap) return;
  IpSlot *nt; uint32_t *nf; uint64_t *noff; uint32_t *nlen;
  HIP_OK(hipMalloc(&nt, cap * sizeof(IpSlot)));
  HIP_OK(hipMalloc(&nf, cap * 4));
  HIP_OK(hipMalloc(&noff, cap * 8));
  HIP_OK(hipMalloc(&nlen, cap * 4));
  HIP_OK(hipMemsetAsync(nt, 0, cap * sizeof(IpSlot), e->stream));
  HIP_OK(hipMemsetAsync(nf, 0xFF, cap * 4, e->stream));
  HIP_OK(hipMemcpyAsync(noff, S.ip_off, n_ips * 8, hipMemcpyDeviceToDevice, e->stream));
  HIP_OK(hipMemcpyAsync(nlen, S.ip_len, n_ips * 4, hipMemcpyDeviceToDevice, e->stream));
  hipLaunchKernelGGL(k_rehash_ip, dim3(grid_for(e->ip_cap)), dim3(kBlock), 0, e->stream, e->ip_cap, S.ip, nt, cap - 1);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(e->stream));
  (void)hipFree(S.ip); (void)hipFree(S.ip_first); (void)hipFree(S.ip_off); (void)hipFree(S.ip_len);
  S.ip = nt; S.ip_first = nf; S.ip_off = noff; S.ip_len = nlen;
  S.ip_mask = cap - 1;
  (void)hipFree(S.ip_st);
  HIP_OK(hipMalloc(&S.ip_st, cap * 4));
  HIP_OK(hipMemsetAsync(S.ip_st, 0xFF, cap * 4, e->stream));
  S.ip_st_cap = cap;
  e->ip_cap = cap;
  ++e->rehashes;
}

// rehash the state table into one that holds `want` states under a 3/4 load factor
void grow_st(bjx_engine *e, uint64_t want) {
  State &S = e->S;
  const uint64_t cap = next_pow2(want * 4 / 3 + 1024);
  if (cap <= e->st_cap) return;
  StSlot *nt;
  HIP_OK(hipMalloc(&nt, cap * sizeof(StSlot)));
  HIP_OK(hipMemsetAsync(nt, 0, cap * sizeof(StSlot), e->stream));
  hipLaunchKernelGGL(k_rehash_st, dim3(grid_for(e->st_cap)), dim3(kBlock), 0, e->stream, e->st_cap, S.st, nt, cap - 1);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(e->stream));
  (void)hipFree(S.st);
  S.st = nt;
  S.st_mask = cap - 1;
  HIP_OK(hipMemsetAsync(S.ip_st, 0xFF, S.ip_st_cap * 4, e->stream));  // slots moved
  if (cap > (1ull << 32)) S.hot_name = kNone;
  e->st_cap = cap;
  ++e->rehashes;
}

// Tables sized for the steady state, not for every batch's worst case: the
// IP and state tables keep room for `new_ips` / `new_states` more entries
// (claims beyond that roll back and grow, see rate_limit_stage); the arena
// always fits the batch's IP bytes.  Small tables keep the random probes in
// cache and the state-slot sort short.
// (e->host_counters current: the caller has just read them)
void ensure_capacity(bjx_engine *e, uint64_t new_ips, uint64_t new_bytes, uint64_t new_states) {
  State &S = e->S;
  const uint64_t n_ips = e->host_counters[0], used = e->host_counters[1], n_st = e->host_counters[2];
  if ((n_ips + new_ips) * 4 > e->ip_cap * 3) grow_ip(e, 2 * (n_ips + new_ips));
  if (used + new_bytes > S.arena_cap) {
    const uint64_t cap = std::max<uint64_t>(S.arena_cap * 2, used + new_bytes + (1 << 20));
    uint8_t *na;
    HIP_OK(hipMalloc(&na, cap));
    HIP_OK(hipMemcpyAsync(na, S.arena, used, hipMemcpyDeviceToDevice, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    (void)hipFree(S.arena);
    S.arena = na;
    S.arena_cap = cap;
  }
  if ((n_st + new_states) * 4 > e->st_cap * 3) grow_st(e, 2 * (n_st + new_states));
}

template <typename F>
void cub_call(bjx_engine *e, F f) {
  size_t bytes = 0;
  HIP_OK(f((void *)nullptr, bytes));
  e->cub_tmp.ensure(bytes + 16);
  HIP_OK(f((void *)e->cub_tmp.p, bytes));
}

int bit_width(uint64_t x) {
  int b = 0;
  while (x) { ++b; x >>= 1; }
  return b;
}

}  // namespace

extern "C" int bjx_engine_create(int device, const bjx_engine_options *opts, bjx_engine **out, char *err, size_t err_len) {
  if (!out) return BJX_ERR_ARG;
  *out = nullptr;
  auto e = std::make_unique<bjx_engine>();
  try {
    int n = 0;
    HIP_OK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) throw BjxError(BJX_ERR_DEVICE, "no such HIP device");
    e->device = device;
    HIP_OK(hipSetDevice(device));
    HIP_OK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&e->pin), bjx_engine::kPinBytes, hipHostMallocDefault));
    HIP_OK(hipEventCreate(&e->ev0));
    HIP_OK(hipEventCreate(&e->ev1));
    HIP_OK(hipEventCreate(&e->evm0));
    HIP_OK(hipEventCreate(&e->evm1));
    for (auto &x : e->evk) HIP_OK(hipEventCreate(&x));
    for (auto &x : e->ph) HIP_OK(hipEventCreate(&x));
    for (auto &x : e->xev) HIP_OK(hipEventCreate(&x));
    // >= 4M slots: a quarter of the table stays free for the claims in flight
    // when a launch spends its budget (see k_ip_claim)
    uint64_t ipc = std::max<uint64_t>(opts && opts->ip_capacity ? next_pow2(opts->ip_capacity) : 0, 1ull << 22);
    uint64_t stc = std::max<uint64_t>(opts && opts->state_capacity ? next_pow2(opts->state_capacity) : 0, 1ull << 22);
    uint64_t ar = opts && opts->ip_arena_bytes ? opts->ip_arena_bytes : (64ull << 20);
    alloc_state(e.get(), ipc, stc, ar);
    *out = e.release();
    return BJX_OK;
  } catch (const BjxError &x) {
    set_err(err, err_len, x.what());
    return x.code;
  }
}

extern "C" void bjx_engine_destroy(bjx_engine *e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  free_state(e);
  e->trips.release(); e->trips_c.release(); e->d_trips_c.release(); e->results.release(); e->line_flags.release();
  e->ev_out_s.release(); e->trip_ev.release(); e->trip_ev2.release();
  for (auto *b : {&e->staging, &e->l_flags, &e->ev_out, &e->rl_out, &e->trip_flag, &e->bind_blob,
                  &e->cub_tmp, &e->q_ip})
    b->release();
  e->tile_counts.release(); e->tile_base.release(); e->nl.release(); e->l_ts.release(); e->l_iph.release();
  e->l_counts.release(); e->l_offs.release(); e->l_masks.release(); e->l_iplen.release();
  e->l_roff.release(); e->slow_list.release(); e->l_hid.release();
  e->scalars.release(); e->res_seq.release(); e->res_rule.release(); e->ev_el.release(); e->ev_rule.release();

  e->ev_res.release(); e->ev_st.release(); e->ev_st2.release(); e->ev_idx.release(); e->ev_idx2.release();
  e->el_slot.release(); e->coll.release(); e->blk_n.release(); e->blk_b.release(); e->ev_rec.release(); e->ev_rec2.release(); e->el_id.release();

  for (auto *b : {&e->pack_src, &e->rx_len, &e->rx_ev_el}) b->release();
  for (auto *b : {&e->pk_hist, &e->pk_off, &e->pk_counts, &e->pk_bbase, &e->rx_hash, &e->rx_pos, &e->rx_nev, &e->rx_evoff})
    b->release();
  e->rx_ts.release(); e->rx_ip16.release(); e->trip_idx.release(); e->d_trips.release(); e->tr_base.release();
  for (auto *b : {&e->bn_key, &e->bn_key2, &e->bn_len, &e->bn_off, &e->dl_hash}) b->release();
  for (auto *b : {&e->bn_val, &e->bn_val2, &e->bn_head, &e->bn_seg, &e->bn_first, &e->bn_cnt, &e->bn_ipt, &e->bn_coll,
                  &e->dl_off, &e->dl_len, &e->nm_off})
    b->release();
  for (auto *b : {&e->bn_kind, &e->bn_flag, &e->bn_log, &e->dl_bytes, &e->nm_json}) b->release();
  e->bn_best.release(); e->bn_rep.release(); e->bn_sel.release(); e->bn_ipb.release(); e->tz_at.release(); e->tz_off.release();
  e->rb_first.release(); e->rb_last.release(); e->long_heads.release(); e->long_count.release();
  e->lr_end.release(); e->lr_len.release(); e->lr_off.release(); e->lr_win.release(); e->lr_t0.release(); e->lr_h0.release();
  e->lr_flags.release(); e->lr_nwin.release(); e->chk.release(); e->chk_w.release(); e->chk_wb.release();
  for (auto *b : {&e->bk_start, &e->bk_big, &e->bk_key, &e->bk_pos}) b->release();
  e->bk_nbig.release(); e->bk_seg.release(); e->bk_rec.release(); e->bk_out.release();
  e->d_results.release(); e->q_out.release();
  e->ban_ips.release(); e->ban_log.release(); e->ban_off.release(); e->ban_kind.release(); e->ban_ipb.release();
  e->ban_ipo.release();
  e->l_ip16.release(); e->jline.release(); e->jkey.release(); e->jidx.release(); e->jidx2.release(); e->jrec.release(); e->jkey2.release(); e->l_cand.release(); e->l_ccnt.release(); e->l_cfirst.release();
  (void)hipEventDestroy(e->ev0); (void)hipEventDestroy(e->ev1); (void)hipEventDestroy(e->evm0); (void)hipEventDestroy(e->evm1);
  for (auto &x : e->evk) (void)hipEventDestroy(x);
  for (auto &x : e->ph) (void)hipEventDestroy(x);
  for (auto &x : e->xev) (void)hipEventDestroy(x);
  for (auto &x : e->bev) if (x) (void)hipEventDestroy(x);
  if (e->bstream) (void)hipStreamDestroy(e->bstream);
  (void)hipStreamDestroy(e->stream);
  if (e->pin) (void)hipHostFree(e->pin);
  delete e;
}

extern "C" const char *bjx_engine_last_error(bjx_engine *e) { return e ? e->last_error.c_str() : "no engine"; }

extern "C" int bjx_engine_set_decision_lists(bjx_engine *e, const bjx_decision_entry *entries, size_t n) {
  if (!e || (n && !entries)) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  std::vector<bjx_engine::Entry> v;
  for (size_t i = 0; i < n; ++i) {
    if (entries[i].decision < BJX_ALLOW || entries[i].decision > BJX_IPTABLES_BLOCK) return BJX_ERR_DECISION;
    bjx_engine::Entry x;
    x.global = entries[i].site.ptr == nullptr;
    if (!x.global) x.site.assign(entries[i].site.ptr, entries[i].site.len);
    x.decision = entries[i].decision;
    x.ip.assign(entries[i].ip.ptr ? entries[i].ip.ptr : "", entries[i].ip.len);
    v.push_back(std::move(x));
  }
  e->decisions.swap(v);
  e->decisions_version++;
  return BJX_OK;
}

// phase boundaries: 0 start, 1 counted (pass A), 2 scanned (pass B), 3 resolved
// (pass C + fallback), 4 emitted, 5 sorted, 6 segmented, 7 rate-limited, 8 trips
static bool trace_on() {
  static const bool on = getenv("BJX_TRACE") != nullptr;
  return on;
}

static void mark(bjx_engine *e, int k) {
  HIP_OK(hipEventRecord(e->ph[k], e->stream));
  e->phase_rec[k] = true;
  if (trace_on()) {  // debugging aid: drain the stream at every phase boundary
    HIP_OK(hipStreamSynchronize(e->stream));
    fprintf(stderr, "[bjx] phase %d done\n", k);
  }
}

// RegexRateLimitStates.Apply for n_ev events (reference order) whose lines are
// E; writes e->ev_out[k].  n_el / el_bytes bound the new IPs / arena bytes.
// Phases 5 (IP + state slots), 6 (sort), 7 (automaton).
// the event sort (state slot keys, records as values) and the Apply kernels,
// for either record form
// k_apply + k_long_* over n events sorted by their full state slot (key, rec),
// outcomes to out in that order
template <typename Rec>
static uint64_t rl_apply_sorted(bjx_engine *e, const Bind &B, uint64_t n_ev, const uint32_t *key, const Rec *rec2,
                                int64_t base, uint8_t *out, uint32_t *wcnt) {
  hipStream_t st = e->stream;
  const uint64_t n_chunks = (n_ev + kApplyChunk - 1) / kApplyChunk;
  e->long_heads.ensure(n_chunks + 1);
  e->long_count.ensure(1);
  HIP_OK(hipMemsetAsync(e->long_count.p, 0, 8, st));
  hipLaunchKernelGGL(k_apply<Rec>, dim3((unsigned)n_chunks), dim3(kBlock), 0, st, n_ev, key, rec2, base, B.rules, e->S.st,
                     out, e->long_heads.p, e->long_count.p, wcnt);
  HIP_OK(hipGetLastError());
  unsigned long long n_long = 0;
  pin_get(e, &n_long, e->long_count.p, 8);
  pin_sync(e);
  if (n_long) {
    // runs crossing a k_apply chunk (hot keys): ends, a parallel regularity
    // check, the window starts per run, then every record in parallel
    LongRuns R;
    e->lr_end.ensure(n_long); e->lr_len.ensure(n_long + 1); e->lr_off.ensure(n_long + 1); e->lr_t0.ensure(n_long);
    e->lr_h0.ensure(n_long); e->lr_flags.ensure(n_long); e->lr_nwin.ensure(n_long);
    R.head = e->long_heads.p; R.end = e->lr_end.p; R.off = e->lr_off.p; R.t0 = e->lr_t0.p; R.h0 = e->lr_h0.p;
    R.flags = e->lr_flags.p; R.nwin = e->lr_nwin.p; R.n = n_long; R.win = nullptr; R.wcnt = wcnt;
    HIP_OK(hipMemsetAsync(e->lr_len.p + n_long, 0, 8, st));
    hipLaunchKernelGGL(k_long_ends<Rec>, dim3((unsigned)n_long), dim3(kBlock), 0, st, n_ev, key, rec2, base, e->S.st,
                       B.rules, R, e->lr_len.p);
    HIP_OK(hipGetLastError());
    {
      uint64_t *in = e->lr_len.p, *o = e->lr_off.p;
      cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)(n_long + 1), st); });
    }
    uint64_t total = 0;
    pin_get(e, &total, e->lr_off.p + n_long, 8);
    pin_sync(e);
    e->lr_win.ensure(total + 1);
    R.win = e->lr_win.p;
    hipLaunchKernelGGL(k_long_check<Rec>, dim3(grid_for(total)), dim3(kBlock), 0, st, total, rec2, base, B.rules, R);
    hipLaunchKernelGGL(k_long_windows<Rec>, dim3((unsigned)n_long), dim3(kBlock), 0, st, key, rec2, base, B.rules,
                       e->S.st, out, R);
    hipLaunchKernelGGL(k_long_fill<Rec>, dim3(grid_for(total)), dim3(kBlock), 0, st, total, rec2, B.rules, out, R);
    HIP_OK(hipGetLastError());
  }
  return n_long;
}

// RegexRateLimitStates.Apply for n_ev events (reference order) whose lines are
// E; writes e->ev_out[k].  n_el / el_bytes bound the new IPs / arena bytes.
// Phases 5 (IP + state slots), 6 (sort), 7 (automaton).
// the event sort (state slot keys, records as values) and the Apply kernels,
// for either record form
template <typename Rec>
static void rl_sort_apply(bjx_engine *e, const Bind &B, const EvSrc &E, uint64_t n_ev, const uint32_t *ev_el,
                          const uint32_t *ev_rule, int64_t base) {
  hipStream_t st = e->stream;
  const Rec *rec2 = reinterpret_cast<const Rec *>(e->ev_rec2.p);
  const bool check = getenv("BJX_CHECK") != nullptr;
  const int bits = std::max(1, bit_width(e->st_cap - 1));
  const int L = bits - kBucketBits;
  // BJX_SORT2 (test / timing hook, read per batch): 0 the full sort always,
  // 2 two-level whenever the table allows it (no batch-size gate, no hold)
  const char *s2 = getenv("BJX_SORT2");
  const int sort2 = s2 ? atoi(s2) : 1;
  // two-level grouping (k_bucket_apply) unless the buckets would be too full on
  // average (then most of them would take the full path anyway); BJX_CHECK's
  // write accounting covers both paths
  const uint32_t nb = 1u << kBucketBits;
  // a batch whose oversized buckets held more than 1/8 of its events (a hot
  // key) is followed by kSort2Hold batches on the full sort: the events of those
  // buckets pay for a gather and a sort of their own on top of the two passes
  // (cfg5h, 25 %: 16.6 ms against 10.0; the node rehearsal's owners, 8 %: 28.4
  // against 30.6 ms for both engines)
  // (BJX_SORT2_HOLD / BJX_SORT2_MIN: test hooks that shorten the hold and lower
  // the batch-size gate, so test-sized batches exercise the default policy)
  const char *hold_env = getenv("BJX_SORT2_HOLD"), *min_env = getenv("BJX_SORT2_MIN");
  const uint32_t kSort2Hold = hold_env ? (uint32_t)atoi(hold_env) : 32u;
  // small batches (fewer than 512 events per bucket on average) keep the full
  // sort: 2^16 mostly empty blocks cost more than the two passes they save
  // (cfg4, 2M lines: 0.6 -> 1.5 ms)
  const uint64_t per_bucket_min = min_env ? (uint64_t)atoll(min_env) : 512ull;
  bool two = sort2 != 0 && L > 0 && L <= 15 &&
             (sort2 == 2 || (n_ev >= (uint64_t)nb * per_bucket_min && n_ev <= (uint64_t)nb * (kBucketCap * 7 / 8)));
  if (two && sort2 != 2 && e->sort2_hold) {
    --e->sort2_hold;
    two = false;
  }
  {
    uint32_t *ki = e->ev_st.p, *ko = e->ev_st2.p;
    Rec *vi = reinterpret_cast<Rec *>(e->ev_rec.p), *vo = reinterpret_cast<Rec *>(e->ev_rec2.p);
    const int lo = two ? L : 0;
    cub_call(e, [&](void *tmp, size_t &bytes) {
      return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, ki, ko, vi, vo, (int)n_ev, lo, bits, st);
    });
  }
  uint32_t *wcnt = nullptr;
  if (check) {
    HIP_OK(hipMemsetAsync(e->ev_out_s.p, 0, n_ev, st));
    e->chk_w.ensure(2 * n_ev);
    wcnt = e->chk_w.p;
    HIP_OK(hipMemsetAsync(wcnt, 0, 2 * n_ev * 4, st));
  }
  unsigned long long n_long = 0;
  e->last_big_events = 0;
  e->last_grouping = two ? 1 : 0;
  if (!two) {
    n_long = rl_apply_sorted<Rec>(e, B, n_ev, e->ev_st2.p, rec2, base, e->ev_out_s.p, wcnt);
  } else {
    e->bk_start.ensure(nb + 1); e->bk_big.ensure(nb); e->bk_nbig.ensure(1);
    HIP_OK(hipMemsetAsync(e->bk_nbig.p, 0, 8, st));
    hipLaunchKernelGGL(k_bucket_bounds, dim3(grid_for(n_ev + 1)), dim3(kBlock), 0, st, n_ev, e->ev_st2.p, (uint32_t)L, nb,
                       e->bk_start.p);
    hipLaunchKernelGGL(k_bucket_apply<Rec>, dim3(nb), dim3(kBlock), 0, st, e->ev_st2.p, rec2, e->bk_start.p, (uint32_t)L, base,
                       B.rules, e->S.st, e->ev_out_s.p, e->bk_big.p, e->bk_nbig.p, wcnt);
    HIP_OK(hipGetLastError());
    unsigned long long n_big = 0;
    pin_get(e, &n_big, e->bk_nbig.p, 8);
    pin_sync(e);
    if (n_big) {
      // oversized buckets (hot keys): their events, in bucket order, through
      // the full sort and k_apply + k_long_*, outcomes back to their positions
      std::vector<uint32_t> big(n_big), bs(nb + 1);
      HIP_OK(hipMemcpyAsync(big.data(), e->bk_big.p, n_big * 4, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(bs.data(), e->bk_start.p, (nb + 1) * 4ull, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      std::sort(big.begin(), big.end());
      std::vector<uint4> seg(n_big);
      uint64_t total = 0;
      for (size_t k = 0; k < n_big; ++k) {
        const uint32_t b = big[k];
        seg[k] = make_uint4(bs[b], bs[b + 1] - bs[b], (uint32_t)total, 0u);
        total += bs[b + 1] - bs[b];
      }
      e->bk_seg.ensure(n_big); e->bk_key.ensure(2 * total); e->bk_pos.ensure(2 * total);
      e->bk_rec.ensure(total); e->bk_out.ensure(total);
      HIP_OK(hipMemcpyAsync(e->bk_seg.p, seg.data(), n_big * sizeof(uint4), hipMemcpyHostToDevice, st));
      uint32_t *k0 = e->bk_key.p, *k1 = e->bk_key.p + total, *p0 = e->bk_pos.p, *p1 = e->bk_pos.p + total;
      hipLaunchKernelGGL(k_big_gather, dim3(grid_for(total)), dim3(kBlock), 0, st, e->bk_seg.p, (uint32_t)n_big, total,
                         e->ev_st2.p, k0, p0);
      HIP_OK(hipGetLastError());
      cub_call(e, [&](void *tmp, size_t &bytes) {
        return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, k0, k1, p0, p1, (int)total, 0, bits, st);
      });
      Rec *r3 = reinterpret_cast<Rec *>(e->bk_rec.p);
      hipLaunchKernelGGL(k_big_recs<Rec>, dim3(grid_for(total)), dim3(kBlock), 0, st, total, p1, rec2, r3);
      HIP_OK(hipGetLastError());
      uint32_t *wbig = nullptr;
      if (check) {
        e->chk_wb.ensure(total);
        wbig = e->chk_wb.p;
        HIP_OK(hipMemsetAsync(wbig, 0, total * 4, st));
      }
      n_long = rl_apply_sorted<Rec>(e, B, total, k1, r3, base, e->bk_out.p, wbig);
      hipLaunchKernelGGL(k_big_outs, dim3(grid_for(total)), dim3(kBlock), 0, st, total, p1, e->bk_out.p, e->ev_out_s.p, wbig,
                         wcnt);
      HIP_OK(hipGetLastError());
      HIP_OK(hipStreamSynchronize(st));  // seg (host memory) stays alive until its copy is done
      e->last_big_events = total;
      e->last_grouping = 1 + total;
      if (total > n_ev / 8) e->sort2_hold = kSort2Hold;
    }
  }
  e->last_long_runs = n_long;
  if (check) {
    e->chk.ensure(16);
    HIP_OK(hipMemsetAsync(e->chk.p, 0, 128, st));
    uint32_t *pc = wcnt + n_ev;
    hipLaunchKernelGGL(k_check_count, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, n_ev,
                       ev_words(e), rec_stride(e), n_ev, pc, e->chk.p + 14);
    hipLaunchKernelGGL(k_check_rl, dim3(grid_for(std::max<uint64_t>(E.n, n_ev))), dim3(kBlock), 0, st, E, n_ev, ev_el, ev_rule,
                       e->el_slot.p, e->el_id.p, B.rules, e->S, e->ev_st.p, e->ev_out_s.p, wcnt, pc, e->chk.p);
    HIP_OK(hipGetLastError());
    unsigned long long c[16];
    pin_get(e, c, e->chk.p, 128);
    pin_sync(e);
    if (c[0] || c[3] || c[6] || c[8] || c[10] || c[12] || c[14]) {
      char msg[768];
      snprintf(msg, sizeof msg,
               "BJX_CHECK: %llu event lines with a wrong IP id (first line %llu id %llu), %llu events in a wrong state slot "
               "(first %llu slot %llu), %llu unwritten outcomes (first %llu), %llu outcomes not written exactly once (first "
               "%llu), %llu seenIp=false outcomes that are not FirstTime (first %llu), %llu sorted positions whose event "
               "index is not a permutation (first %llu; %llu out of range); epoch %u, %llu long runs, n_ev %llu",
               c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11], c[12], c[13], c[14], e->epoch,
               (unsigned long long)n_long, (unsigned long long)n_ev);
      fprintf(stderr, "%s\n", msg);
      throw BjxError(BJX_ERR_DEVICE, msg);
    }
  }
}

// rec_base (kNoRecBase: none): the events' timestamps are expected within
// 2^43 ns of it either way, so the sort carries 12-B records (EvRec12).
constexpr int64_t kNoRecBase = INT64_MIN;
static void rate_limit_stage(bjx_engine *e, const Bind &B, const EvSrc &E, uint64_t n_el, uint64_t el_bytes, uint64_t n_ev,
                             const uint32_t *ev_el, const uint32_t *ev_rule, int64_t rec_base) {
  hipStream_t st = e->stream;
  const bool force16 = getenv("BJX_REC16") != nullptr;  // test hook: the 16-B records throughout
  bool use12 = rec_base != kNoRecBase && B.n_rules < (1u << EvRec12::kRuleBits) && !force16;
  if (use12) rec_base = (int64_t)((uint64_t)rec_base - (EvRec12::kSpan >> 1));
  else rec_base = 0;
  if (E.n >= 0x7FFFFFFFull || n_ev >= 0xFFFFFFFFull) throw BjxError(BJX_ERR_ARG, "batch too large (2^31 lines / 2^32 events)");
  if (!e->counters_fresh) read_counters(e);
  e->counters_fresh = false;
  // room for the new entries expected: an eighth of the table's entries, or
  // 1.25 x the previous batch's new entries (a stream of new IPs), whichever
  // is more, at most the batch's worst case
  const uint64_t ips0 = e->host_counters[0], st0 = e->host_counters[2];
  ensure_capacity(e, std::min<uint64_t>(n_el, std::max<uint64_t>(std::max<uint64_t>(1u << 18, ips0 / 8), e->last_new_ips * 5 / 4)),
                  el_bytes,
                  std::min<uint64_t>(n_ev, std::max<uint64_t>(std::max<uint64_t>(1u << 20, st0 / 8), e->last_new_states * 5 / 4)));
  if (e->host_counters[0] + n_el >= 0x7FFFFFFFull) throw BjxError(BJX_ERR_CAPACITY, "more than 2^31 distinct IPs");
  if (++e->epoch == 0) ++e->epoch;  // 0 marks a slot being claimed
  const uint32_t epoch = e->epoch;
  e->el_slot.ensure(E.n); e->el_id.ensure(E.n); e->coll.ensure(E.n);
  uint64_t nw_ovf[2] = {0, 0};  // new-IP event lines (k_ip_claim's list), IP table overflow flag
  uint64_t cnt6[6] = {};          // S.counters[0..5] after the IP claims
  e->ev_st.ensure(n_ev); e->ev_st2.ensure(n_ev); e->ev_rec.ensure(n_ev); e->ev_rec2.ensure(n_ev);
  e->ev_out.ensure(n_ev); e->ev_out_s.ensure(n_ev);
  mark(e, 5);
  {
    for (int attempt = 0;; ++attempt) {
      const uint64_t n_ips = e->host_counters[0];
      HIP_OK(hipMemsetAsync(e->S.counters + 3, 0, 3 * 8, st));
      HIP_OK(hipMemsetAsync(e->S.counters + kShardBase, 0, kClaimShards * 128, st));
      uint64_t budget = e->ip_cap * 3 / 4 - n_ips;
      const bool forced = e->dbg_budget && attempt == 0 && e->dbg_budget < budget;  // test hook
      if (forced) budget = e->dbg_budget;
      // a retry after an overflow claims every line again (the rolled-back
      // claims left their lines' el_id set)
      hipLaunchKernelGGL(k_ip_claim, dim3(grid_for(E.n)), dim3(kBlock), 0, st, E, e->S, epoch, e->el_slot.p, e->el_id.p,
                         budget / kClaimShards);
      hipLaunchKernelGGL(k_fold_new, dim3(1), dim3(kClaimShards), 0, st, e->S);
      HIP_OK(hipGetLastError());
      // with the overflow flags, the table counters and the collision count:
      // a batch without new IPs needs no further read before its state claims
      pin_get(e, cnt6, e->S.counters, 48);
      pin_sync(e);
      nw_ovf[0] = cnt6[4];
      nw_ovf[1] = cnt6[5];
      if (!nw_ovf[1]) break;
      // more new IPs than the table had room for: undo, grow, claim again
      hipLaunchKernelGGL(k_ip_rollback, dim3(grid_for(e->ip_cap)), dim3(kBlock), 0, st, e->ip_cap, e->S, epoch);
      HIP_OK(hipGetLastError());
      // straight to the batch's worst case (every event line a new IP): one
      // rollback at most (stepwise growth redid the whole claim pass per step)
      if (!forced) grow_ip(e, n_ips + n_el);
    }
    if (nw_ovf[0]) {
      const uint64_t nb = grid_for(E.n);
      e->blk_n.ensure(2 * nb); e->blk_b.ensure(2 * nb);
      uint32_t *bn = e->blk_n.p, *bno = e->blk_n.p + nb;
      uint64_t *bb = e->blk_b.p, *bbo = e->blk_b.p + nb;
      hipLaunchKernelGGL(k_ip_firsts, dim3(nb), dim3(kBlock), 0, st, E, e->S, e->el_slot.p, e->el_id.p, bn, bb);
      cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, bn, bno, (int)nb, st); });
      cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, bb, bbo, (int)nb, st); });
      hipLaunchKernelGGL(k_ip_commit, dim3(nb), dim3(kBlock), 0, st, E, e->S, e->el_slot.p, e->el_id.p, bno, bbo, e->coll.p);
      hipLaunchKernelGGL(k_ip_commit_total, dim3(1), dim3(64), 0, st, e->S, nb, bn, bno, bb, bbo);
      HIP_OK(hipGetLastError());
    }
    // no new IPs: no commit ran, so the counters read with the flags are final
    const bool cnt_final = nw_ovf[0] == 0;
    uint64_t n_coll = cnt6[3];
    if (!cnt_final) {
      pin_get(e, &n_coll, e->S.counters + 3, 8);
      pin_sync(e);
    }
    if (n_coll) {  // distinct IPs with one 64-bit hash in this batch: resolve exactly, in line order
      if (n_coll > 1) {
        uint32_t *ki = e->coll.p, *ko = e->ev_st2.p;
        cub_call(e, [&](void *tmp, size_t &bytes) {
          return hipcub::DeviceRadixSort::SortKeys(tmp, bytes, ki, ko, (int)n_coll, 0, 32, st);
        });
        HIP_OK(hipMemcpyAsync(e->coll.p, e->ev_st2.p, n_coll * 4, hipMemcpyDeviceToDevice, st));
      }
      hipLaunchKernelGGL(k_ip_collide, dim3(1), dim3(64), 0, st, E, e->S, epoch, e->el_slot.p, e->el_id.p, e->coll.p, n_coll);
      HIP_OK(hipGetLastError());
    }
    for (int attempt = 0;; ++attempt) {
      if (attempt == 0 && cnt_final && n_coll == 0) memcpy(e->host_counters, cnt6, 24);
      else read_counters(e);
      const uint64_t n_st = e->host_counters[2];
      HIP_OK(hipMemsetAsync(e->S.counters + 6, 0, 3 * 8, st));
      HIP_OK(hipMemsetAsync(e->S.counters + kShardBase, 0, kClaimShards * 128, st));
      uint64_t budget = e->st_cap * 3 / 4 - n_st;
      const bool forced = e->dbg_budget && attempt == 0 && e->dbg_budget < budget;  // test hook
      if (forced) budget = e->dbg_budget;
      if (use12)
        hipLaunchKernelGGL(k_st_claim<EvRec12>, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, E, n_ev, ev_el, ev_rule,
                           e->el_slot.p, e->el_id.p, B.rules, e->S, e->ev_st.p, reinterpret_cast<EvRec12 *>(e->ev_rec.p),
                           rec_base, budget / kClaimShards);
      else
        hipLaunchKernelGGL(k_st_claim<EvRec>, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, E, n_ev, ev_el, ev_rule,
                           e->el_slot.p, e->el_id.p, B.rules, e->S, e->ev_st.p, e->ev_rec.p, rec_base, budget / kClaimShards);
      // the shard counts folded into the table count right away (an overflow
      // below rolls the claims back and recounts), read with the flags
      hipLaunchKernelGGL(k_fold_claims, dim3(1), dim3(kClaimShards), 0, st, e->S);
      HIP_OK(hipGetLastError());
      uint64_t ovf[2] = {0, 0};  // state table overflow, a timestamp outside the 12-B records' span
      pin_get(e, ovf, e->S.counters + 7, 16);
      pin_get(e, e->host_counters, e->S.counters, 24);
      pin_sync(e);
      if (!ovf[0]) {
        if (use12 && ovf[1]) {
          // the same claims again (every key is in the table now, so nothing
          // is claimed twice), writing 16-B records
          use12 = false;
          rec_base = 0;
          hipLaunchKernelGGL(k_st_claim<EvRec>, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, E, n_ev, ev_el, ev_rule,
                             e->el_slot.p, e->el_id.p, B.rules, e->S, e->ev_st.p, e->ev_rec.p, rec_base, budget / kClaimShards);
          HIP_OK(hipGetLastError());
        }
        break;
      }
      // more new (ip, rule name) states than the table had room for: undo this
      // batch's claims, recount, grow, claim again
      HIP_OK(hipMemsetAsync(e->S.counters + 2, 0, 8, st));
      hipLaunchKernelGGL(k_st_rollback, dim3(grid_for(e->st_cap)), dim3(kBlock), 0, st, e->st_cap, e->S);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemsetAsync(e->S.ip_st, 0xFF, e->S.ip_st_cap * 4, st));  // may name rolled-back slots
      read_counters(e);
      if (!forced) grow_st(e, e->host_counters[2] + n_ev);  // the batch's worst case, as for the IP table
    }
  }
  mark(e, 6);  // host_counters: read with the last claim pass's flags
  e->last_new_ips = e->host_counters[0] - ips0;
  e->last_new_states = e->host_counters[2] - st0;
  e->rec12 = use12;
  e->rec_base = rec_base;
  if (use12) rl_sort_apply<EvRec12>(e, B, E, n_ev, ev_el, ev_rule, rec_base);
  else rl_sort_apply<EvRec>(e, B, E, n_ev, ev_el, ev_rule, rec_base);
}

// k_nfa_wide over jobs [j0, j1): the state in LDS when it fits 64 KB, else
// in a per-block HBM scratch (grid-stride over the jobs either way)
static void launch_wide(bjx_engine *e, const Bind &B, const uint8_t *buf, uint64_t n, const uint32_t *jkey,
                        const uint32_t *jidx, const uint32_t *jline, const uint32_t *jpos, uint64_t j0, uint64_t j1, const Lines &L, uint32_t W,
                        uint32_t ng) {
  hipStream_t st = e->stream;
  const uint64_t words = 2ull * W + (ng + 63) / 64 + 1;
  static const bool force_glb = getenv("BJX_WIDE_GLB") != nullptr;  // test hook: the HBM-scratch variant
  if (words * 8 <= 64 * 1024 && !force_glb) {
    const unsigned grid = (unsigned)std::min<uint64_t>(j1 - j0, 8192);
    hipLaunchKernelGGL(k_nfa_wide<false>, dim3(grid), dim3(kBlock), (uint32_t)(words * 8), st, B, buf, n, e->nl.p, jkey,
                       jidx, jline, jpos, j0, j1, L, nullptr, (uint64_t)0);
  } else {
    const unsigned grid = (unsigned)std::min<uint64_t>(j1 - j0, 512);
    e->wide_scratch.ensure(grid * words);
    hipLaunchKernelGGL(k_nfa_wide<true>, dim3(grid), dim3(kBlock), 0, st, B, buf, n, e->nl.p, jkey, jidx, jline, jpos, j0, j1, L,
                       e->wide_scratch.p, words);
  }
  HIP_OK(hipGetLastError());
}

// The sorted DFA jobs of the bit-parallel NFA rules: each rule's job range
// (k_rule_bounds), then one k_nfa launch per rule with its state width.
static void run_nfa_jobs(bjx_engine *e, const Bind &B, const uint8_t *buf, uint64_t n, uint64_t n_jobs, const Lines &L) {
  hipStream_t st = e->stream;
  // bounds per job key: rule r's windowed jobs under r, its legacy ones (every
  // NFA job) under n_rules + r
  const uint32_t nk = 2 * B.n_rules;
  e->rb_first.ensure(nk); e->rb_last.ensure(nk);
  HIP_OK(hipMemsetAsync(e->rb_first.p, 0, nk * 4ull, st));
  HIP_OK(hipMemsetAsync(e->rb_last.p, 0, nk * 4ull, st));
  hipLaunchKernelGGL(k_rule_bounds, dim3(grid_for(n_jobs)), dim3(kBlock), 0, st, n_jobs, e->jkey2.p, e->rb_first.p, e->rb_last.p);
  HIP_OK(hipGetLastError());
  e->h_first.resize(nk); e->h_last.resize(nk);
  HIP_OK(hipMemcpyAsync(e->h_first.data(), e->rb_first.p, nk * 4ull, hipMemcpyDeviceToHost, st));
  HIP_OK(hipMemcpyAsync(e->h_last.data(), e->rb_last.p, nk * 4ull, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  for (const uint4 &nr : e->nfa_rules) {
    const uint64_t j0 = e->h_first[B.n_rules + nr.x], j1 = e->h_last[B.n_rules + nr.x];
    if (j1 <= j0) continue;
    if (nr.w) {  // kRuleNfaWide: nr.y = state words, nr.z = groups
      launch_wide(e, B, buf, n, e->jkey2.p, e->jidx2.p, e->jline.p, nullptr, j0, j1, L, nr.y, nr.z);
      continue;
    }
    const unsigned grid = grid_for(j1 - j0);
    const uint32_t lds = nr.z * 8;
    switch (nr.y) {
      case 1: hipLaunchKernelGGL(k_nfa<1>, dim3(grid), dim3(kBlock), lds, st, B, nr.x, buf, n, e->nl.p, e->jkey2.p, e->jidx2.p, e->jline.p, j0, j1, L); break;
      case 2: hipLaunchKernelGGL(k_nfa<2>, dim3(grid), dim3(kBlock), lds, st, B, nr.x, buf, n, e->nl.p, e->jkey2.p, e->jidx2.p, e->jline.p, j0, j1, L); break;
      case 4: hipLaunchKernelGGL(k_nfa<4>, dim3(grid), dim3(kBlock), lds, st, B, nr.x, buf, n, e->nl.p, e->jkey2.p, e->jidx2.p, e->jline.p, j0, j1, L); break;
      case 8: hipLaunchKernelGGL(k_nfa<8>, dim3(grid), dim3(kBlock), lds, st, B, nr.x, buf, n, e->nl.p, e->jkey2.p, e->jidx2.p, e->jline.p, j0, j1, L); break;
      default: hipLaunchKernelGGL(k_nfa<16>, dim3(grid), dim3(kBlock), lds, st, B, nr.x, buf, n, e->nl.p, e->jkey2.p, e->jidx2.p, e->jline.p, j0, j1, L); break;
    }
    HIP_OK(hipGetLastError());
  }
}

// consumeLine up to Apply for every line: framing, header, exemption, rule
// matching, RuleResults and events in reference order (phases 0-4).  Leaves
// the batch context in e->bc; false if the batch has no complete line.
static bool match_phase(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns, uint32_t flags,
                        bjx_batch_result *out) {
  e->bc = BatchCtx{};
  HIP_OK(hipSetDevice(e->device));
  if (e->bound_uid != rs->uid || e->bound_dec_version != e->decisions_version) {
    // (re)binding: calibrate the gram filter on the head of this batch
    const size_t sn = std::min<size_t>(n, 4u << 20);
    std::vector<uint8_t> sample;
    const uint8_t *sp = bytes;
    if (flags & BJX_INPUT_DEVICE) {
      sample.resize(sn);
      if (sn) HIP_OK(hipMemcpy(sample.data(), bytes, sn, hipMemcpyDeviceToHost));
      sp = sample.data();
    }
    bind_ruleset(e, rs, sp, sn);
  }
  const Bind &B = e->bind;
  hipStream_t st = e->stream;
  memset(out, 0, sizeof *out);
  e->trips.clear();
  e->trips_c.clear();
  e->results.clear();
  e->line_flags.clear();
  if (n == 0) return false;

  const uint8_t *buf = bytes;
  if (!(flags & BJX_INPUT_DEVICE) || (reinterpret_cast<uintptr_t>(bytes) & 15)) {
    e->staging.ensure(n + 16);
    HIP_OK(hipMemcpyAsync(e->staging.p, bytes, n, (flags & BJX_INPUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    buf = e->staging.p;
  }
  HIP_OK(hipEventRecord(e->ev0, st));
  for (auto &r : e->phase_rec) r = false;
  mark(e, 0);

  // ---- line framing, two passes: pass A counts the '\n' of each 4 KB wave
  // tile and an exclusive scan gives every tile its first line index
  // (the two in-kernel line-index designs measured slower)
  const uint64_t n_tiles = (n + kWT - 1) / kWT;
  e->tile_counts.ensure(n_tiles);
  e->tile_base.ensure(n_tiles + 1);
  uint64_t n_lines = 0;
  Lines L;
  hipLaunchKernelGGL(k_nl_count_wt, dim3((unsigned)((n_tiles + 3) / 4)), dim3(kBlock), 0, st, buf, (uint64_t)n, n_tiles,
                     e->tile_counts.p);
  HIP_OK(hipGetLastError());
  {
    uint32_t *in = e->tile_counts.p;
    uint64_t *o = e->tile_base.p;
    cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)n_tiles, st); });
  }
  {
    uint64_t last_base = 0;
    uint32_t last_cnt = 0;
    pin_get(e, &last_base, e->tile_base.p + (n_tiles - 1), 8);
    pin_get(e, &last_cnt, e->tile_counts.p + (n_tiles - 1), 4);
    pin_sync(e);
    n_lines = last_base + last_cnt;
  }
  out->n_lines = n_lines;
  if (n_lines == 0) return false;
  const uint64_t cap = n_lines;

  // ---- per-line arrays
  e->nl.ensure(cap);
  e->l_ts.ensure(cap); e->l_iph.ensure(cap); e->l_counts.ensure(cap + 1); e->l_offs.ensure(cap + 1);
  e->l_masks.ensure(cap * B.mask_words);
  e->l_iplen.ensure(cap);
  e->l_roff.ensure(cap); e->l_hid.ensure(cap); e->l_flags.ensure(cap); e->slow_list.ensure(cap);
  e->l_ccnt.ensure(cap); e->l_ip16.ensure(cap);
  e->l_cand.ensure(B.any_prefilter ? cap * kCandSlots : 1);
  e->scalars.ensure(16);
  L.ts = e->l_ts.p; L.ip_hash = e->l_iph.p; L.ip_len = e->l_iplen.p;
  L.rest_off = e->l_roff.p; L.host_id = e->l_hid.p; L.flags = e->l_flags.p;
  L.counts = e->l_counts.p; L.masks = e->l_masks.p; L.mstride = cap;
  L.cand_meta = e->l_ccnt.p; L.cand = e->l_cand.p; L.ip16 = e->l_ip16.p;
  L.cand_first = nullptr;
  if (B.cfirst) {
    e->l_cfirst.ensure(cap * kCandFirstLits);
    L.cand_first = e->l_cfirst.p;
    HIP_OK(hipMemsetAsync(e->l_cfirst.p, 0xFF, cap * kCandFirstLits * 8, st));
  }
  e->jline.ensure(std::max<uint64_t>(e->jline.n, cap + (1u << 20)));
  e->jkey.ensure(e->jline.n); e->jidx.ensure(e->jline.n); e->jrec.ensure(e->jline.n);
  HIP_OK(hipMemsetAsync(e->scalars.p, 0, 16 * sizeof(unsigned long long), st));
  if (B.any_prefilter) HIP_OK(hipMemsetAsync(e->l_ccnt.p, 0, cap * sizeof(CandMeta), st));
  mark(e, 1);

  // ---- the scan kernel: line framing + literal hits; one block (16 waves)
  // per CU, grid-stride over the wave tiles
  {
    int n_cu_scan = 0;
    HIP_OK(hipDeviceGetAttribute(&n_cu_scan, hipDeviceAttributeMultiprocessorCount, e->device));
    const unsigned scan_grid = (unsigned)std::min<uint64_t>((n_tiles + kScanWaves - 1) / kScanWaves, (uint64_t)std::max(1, n_cu_scan));
    ScanArgs A;
    A.buf = buf; A.n = n; A.n_tiles = n_tiles; A.n_lines = cap; A.tile_base = e->tile_base.p; A.nl = e->nl.p;
    A.L = L; A.stats = e->scalars.p + 8;
    A.debug_skip = getenv("BJX_DEBUG_SKIP") ? (uint32_t)atoi(getenv("BJX_DEBUG_SKIP")) : 0u;
    // block-shared LDS: the gram pair table, the scan's lookup image when it fits, then 16 wave regions
    const uint32_t fixed = kPairBytes + kScanWaves * kWaveLds;
    const bool img_lds = fixed + B.scan_img_bytes <= kScanLdsMax;
    A.shared_bytes = kPairBytes + (img_lds ? B.scan_img_bytes : 0);
    const uint32_t lds = A.shared_bytes + kScanWaves * kWaveLds;
    using ScanFn = void (*)(Bind, ScanArgs);
    const ScanFn kfn = img_lds ? k_scan<true> : k_scan<false>;
    if (lds != e->scan_lds[img_lds]) {
      HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      e->scan_lds[img_lds] = lds;
    }
    HIP_OK(hipEventRecord(e->evm0, st));
    hipLaunchKernelGGL(kfn, dim3(scan_grid), dim3(kScanWaves * 64), lds, st, B, A);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(e->evm1, st));
  }
  uint64_t last_nl = 0;
  mark(e, 2);

  // ---- the per-line pass: k_lines2 when the ruleset has its tables, else
  // k_lines (exotic timestamps go to the per-line fallback either way)
  unsigned long long sc4[5] = {0, 0, 0, 0, 0};
  unsigned long long n_jobs = 0;  // real DFA jobs (read with sc4, same sync)
  // BJX_LINES=1 (test hook) keeps the line pass for these rulesets too
  const bool all_wide = B.n_global > 128 && !(getenv("BJX_LINES") && atoi(getenv("BJX_LINES")) == 1);
  int n_cu = 0;
  HIP_OK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, e->device));
  if (!e->lines_attr) {
    for (const void *f : {reinterpret_cast<const void *>(&k_lines<true>), reinterpret_cast<const void *>(&k_lines<false>),
#ifdef BJX_PROF
                          reinterpret_cast<const void *>(&k_lines<true, true>),
                          reinterpret_cast<const void *>(&k_lines<false, true>),
                          reinterpret_cast<const void *>(&k_lines<true, true, true>),
                          reinterpret_cast<const void *>(&k_lines<false, true, true>),
#endif
                          reinterpret_cast<const void *>(&k_lines<true, false, true>),
                          reinterpret_cast<const void *>(&k_lines<false, false, true>)})
      HIP_OK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kScanLdsMax));
    e->lines_attr = true;
  }
  // one resident wave of blocks (grid-stride loops): a grid of several
  // "rounds" leaves the last round partly empty
  auto resident_grid = [&](const void *fn, uint32_t lds, uint64_t work) {
    int per_cu = 0;
    HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds));
    const uint64_t resident = (uint64_t)std::max(1, per_cu) * (uint64_t)std::max(1, n_cu);
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((work + kBlock - 1) / kBlock, resident));
  };
  for (int attempt = 0;; ++attempt) {
    LinesArgs A;
    A.buf = buf; A.n = n; A.nl = e->nl.p; A.n_lines = n_lines; A.L = L; A.now_ns = now_ns;
    A.dbg = getenv("BJX_DEBUG_LINES") ? (uint32_t)atoi(getenv("BJX_DEBUG_LINES")) : 0u;
    A.dbg2 = getenv("BJX_DEBUG_L2") ? (uint32_t)atoi(getenv("BJX_DEBUG_L2")) : 0u;
    A.slow_list = e->slow_list.p; A.slow_count = e->scalars.p;
    A.jline = e->jline.p; A.jkey = e->jkey.p; A.jidx = e->jidx.p; A.jrec = e->jrec.p; A.job_count = e->scalars.p + 11;
    A.job_cap = std::min(std::min(e->jline.n, e->jkey.n), std::min(e->jidx.n, e->jrec.n));
    A.job_real = e->scalars.p + 14;
    A.null_key = 2 * B.n_rules;  // sorts after every job key (windowed r, legacy n_rules + r)
    A.span_bytes = getenv("BJX_SPAN_BYTES") ? (uint32_t)atoi(getenv("BJX_SPAN_BYTES")) & ~15u : kSpanBytes;
    A.list = nullptr; A.n_list = 0; A.prof = nullptr;
    HIP_OK(hipEventRecord(e->evk[0], st));
    // k_lines2 (lines2.h) when the ruleset has its tables; BJX_LINES=1 keeps k_lines
    static const int lines_env = getenv("BJX_LINES") ? atoi(getenv("BJX_LINES")) : 2;
    const bool use_l2 = B.l2_bytes && lines_env != 1 && !getenv("BJX_PROF_LINES") && !A.dbg;
    e->last_line_kernel = all_wide ? 3u : use_l2 ? 2u : 1u;
    if (all_wide) {
      // every scope is past 128 positions (more than 128 global rules): no
      // line-kernel pass, the per-line fallback (decide_wide) takes every line
      // from its own parse
      hipLaunchKernelGGL(k_no_line_pass, dim3(1), dim3(64), 0, st, e->scalars.p, (unsigned long long)n_lines);
      HIP_OK(hipGetLastError());
    } else if (use_l2) {
      const uint32_t lds = B.l2_bytes + (kL2Block / 64) * kL2WaveLds;
      const void *fn = B.l2_w == 2 ? reinterpret_cast<const void *>(&k_lines2<2>) : reinterpret_cast<const void *>(&k_lines2<1>);
      if (lds != e->lines2_lds || B.l2_w != e->lines2_w) {
        HIP_OK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        e->lines2_lds = lds;
        e->lines2_w = B.l2_w;
      }
      int per_cu = 0;
      HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kL2Block, lds));
      const uint64_t resident = (uint64_t)std::max(1, per_cu) * (uint64_t)std::max(1, n_cu);
      const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n_lines + kL2Block - 1) / kL2Block, resident));
      static const bool dbg_img = getenv("BJX_DEBUG_IMG") != nullptr;
      if (dbg_img) fprintf(stderr, "[bjx] k_lines2: %u B LDS per block (tables %u), %d blocks per CU, grid %u\n", lds, B.l2_bytes, per_cu, grid);
#ifdef BJX_PROF_L2
      e->chk.ensure(16);
      HIP_OK(hipMemsetAsync(e->chk.p, 0, 128, st));
      A.prof = e->chk.p;
#endif
      if (B.l2_w == 2) hipLaunchKernelGGL(k_lines2<2>, dim3(grid), dim3(kL2Block), lds, st, B, A);
      else hipLaunchKernelGGL(k_lines2<1>, dim3(grid), dim3(kL2Block), lds, st, B, A);
      HIP_OK(hipGetLastError());
#ifdef BJX_PROF_L2
      {
        unsigned long long c[8];
        pin_get(e, c, e->chk.p, 64);
        pin_sync(e);
        double tot = 0;
        for (int k = 0; k < 8; ++k) tot += (double)c[k];
        fprintf(stderr, "[bjx] k_lines2 segments (%% of wave clocks): loads %.1f header %.1f host+allow %.1f hits %.1f "
                "anchored %.1f jobs %.1f stores %.1f flush %.1f\n", 100 * c[0] / tot, 100 * c[1] / tot, 100 * c[2] / tot,
                100 * c[3] / tot, 100 * c[4] / tot, 100 * c[5] / tot, 100 * c[6] / tot, 100 * c[7] / tot);
      }
#endif
    } else {
      const bool img_lds = B.img_bytes <= kLinesImgMax;
      const bool host_lds = B.hl_bytes != 0;
      const uint32_t fixed = ((img_lds ? B.img_bytes : 0) + 15u & ~15u) + (host_lds ? B.hl_bytes + 15u & ~15u : 0u) +
                             (kBlock / 64) * kWaveJobBytes;
      if (A.span_bytes && !getenv("BJX_SPAN_BYTES")) {
        // spans take what kLinesBlocksPerCu blocks leave of the CU's LDS
        // (LDS goes to blocks in granules: 53 KB blocks fit only twice per CU,
        // measured; stay a 2 KB granule under the share)
        const uint32_t share = (kScanLdsMax / kLinesBlocksPerCu) & ~2047u;
        const uint32_t room = share > fixed ? share - fixed : 0u;
        A.span_bytes = std::min<uint32_t>(kSpanBytes, (room / (kBlock / 64) - 32) & ~15u);
      }
      const uint32_t lds = fixed + (kBlock / 64) * (A.span_bytes ? A.span_bytes + 32 : 0);
      const void *fn = img_lds ? (host_lds ? reinterpret_cast<const void *>(&k_lines<true, false, true>)
                                           : reinterpret_cast<const void *>(&k_lines<true>))
                               : (host_lds ? reinterpret_cast<const void *>(&k_lines<false, false, true>)
                                           : reinterpret_cast<const void *>(&k_lines<false>));
      const unsigned grid = resident_grid(fn, lds, A.list ? A.n_list : n_lines);
      const bool prof = getenv("BJX_PROF_LINES") != nullptr;
      A.prof = nullptr;
      if (prof) {  // debugging aid: clock per k_lines segment, printed to stderr
#ifndef BJX_PROF
        throw BjxError(BJX_ERR_ARG, "BJX_PROF_LINES needs a library built with BJX_PROF=1");
#else
        e->chk.ensure(16);
        HIP_OK(hipMemsetAsync(e->chk.p, 0, 128, st));
        A.prof = e->chk.p;
        if (img_lds && host_lds) hipLaunchKernelGGL((k_lines<true, true, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
        else if (img_lds) hipLaunchKernelGGL((k_lines<true, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
        else if (host_lds) hipLaunchKernelGGL((k_lines<false, true, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
        else hipLaunchKernelGGL((k_lines<false, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
        unsigned long long c[10];
        pin_get(e, c, e->chk.p, 80);
        pin_sync(e);
        double tot = 0;
        for (int k = 0; k < 10; ++k) tot += (double)c[k];
        fprintf(stderr, "[bjx] k_lines segments (%% of wave clocks): loads+staging %.1f header %.1f host %.1f host-rules %.1f "
                "hit-decode %.1f site-walk %.1f global-walk %.1f mask-stores %.1f stores %.1f jobs %.1f\n", 100 * c[0] / tot,
                100 * c[1] / tot, 100 * c[2] / tot, 100 * c[3] / tot, 100 * c[7] / tot, 100 * c[8] / tot, 100 * c[9] / tot,
                100 * c[4] / tot, 100 * c[5] / tot, 100 * c[6] / tot);
#endif
      } else if (img_lds && host_lds) hipLaunchKernelGGL((k_lines<true, false, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
      else if (img_lds) hipLaunchKernelGGL(k_lines<true>, dim3(grid), dim3(kBlock), lds, st, B, A);
      else if (host_lds) hipLaunchKernelGGL((k_lines<false, false, true>), dim3(grid), dim3(kBlock), lds, st, B, A);
      else hipLaunchKernelGGL(k_lines<false>, dim3(grid), dim3(kBlock), lds, st, B, A);
      HIP_OK(hipGetLastError());
    }
    HIP_OK(hipEventRecord(e->evk[1], st));
    pin_get(e, &last_nl, e->nl.p + (n_lines - 1), 8);
    pin_get(e, sc4, e->scalars.p + 8, 32);
    pin_get(e, sc4 + 4, e->scalars.p, 8);
    pin_get(e, &n_jobs, e->scalars.p + 14, 8);
    pin_sync(e);
    if (sc4[3] <= std::min(std::min(e->jline.n, e->jkey.n), std::min(e->jidx.n, e->jrec.n))) break;
    // more DFA jobs than the buffer holds: grow it and redo the (idempotent) line pass
    if (attempt > 0) throw BjxError(BJX_ERR_DEVICE, "internal: DFA job buffer overflow");
    e->jline.ensure(sc4[3] + (1u << 20));
    e->jkey.ensure(sc4[3] + (1u << 20));
    e->jidx.ensure(sc4[3] + (1u << 20));
    e->jrec.ensure(sc4[3] + (1u << 20));
    HIP_OK(hipMemsetAsync(e->scalars.p, 0, 8, st));
    HIP_OK(hipMemsetAsync(e->scalars.p + 11, 0, 16, st));
    HIP_OK(hipMemsetAsync(e->scalars.p + 14, 0, 8, st));
  }
  out->consumed_bytes = last_nl + 1;
  // job slots taken (sc4[3]; the chunks' unused ones hold null jobs) and real jobs (n_jobs)
  const unsigned long long n_slow = sc4[4], n_slots = sc4[3];
  e->last_jobs = n_jobs;
  e->scan_stats[0] = sc4[0]; e->scan_stats[1] = sc4[1]; e->scan_stats[2] = n_slow; e->scan_stats[3] = B.scan_img_bytes;
  e->scan_stats[4] = n_jobs; e->scan_stats[5] = sc4[2];
  HIP_OK(hipEventRecord(e->evk[2], st));
  if (n_jobs) {
    // group the jobs by rule (stable: line order inside a rule), then one lane per job
    e->jidx2.ensure(n_slots); e->jkey2.ensure(n_slots);
    {
      // null jobs (key n_rules) sort after the real ones: k_dfa takes the first n_jobs
      uint32_t *ki = e->jkey.p, *ko = e->jkey2.p, *vi = e->jidx.p, *vo = e->jidx2.p;
      const int bits = std::max(1, bit_width(2 * B.n_rules));
      cub_call(e, [&](void *tmp, size_t &bytes) {
        return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, ki, ko, vi, vo, (int)n_slots, 0, bits, st);
      });
    }
    hipLaunchKernelGGL(k_dfa, dim3(grid_for(n_jobs)), dim3(kBlock), B.dfa_lds, st, B, buf, (uint64_t)n, e->jkey2.p,
                       e->jidx2.p, e->jline.p, e->jrec.p, (uint64_t)n_jobs, L);
    hipLaunchKernelGGL(k_dfa_legacy, dim3(grid_for(n_jobs)), dim3(kBlock), 0, st, B, buf, (uint64_t)n, e->nl.p, e->jkey2.p,
                       e->jidx2.p, e->jline.p, (uint64_t)n_jobs, L);
    HIP_OK(hipGetLastError());
    if (B.any_nfa && !e->nfa_rules.empty()) run_nfa_jobs(e, B, buf, n, n_jobs, L);
    static const bool job_stats = getenv("BJX_JOB_STATS") != nullptr;  // diagnostics: jobs per rule (stderr)
    if (job_stats) {
      const uint32_t nk = 2 * B.n_rules;
      e->rb_first.ensure(nk); e->rb_last.ensure(nk);
      HIP_OK(hipMemsetAsync(e->rb_first.p, 0, nk * 4ull, st));
      HIP_OK(hipMemsetAsync(e->rb_last.p, 0, nk * 4ull, st));
      hipLaunchKernelGGL(k_rule_bounds, dim3(grid_for(n_jobs)), dim3(kBlock), 0, st, (uint64_t)n_jobs, e->jkey2.p, e->rb_first.p,
                         e->rb_last.p);
      std::vector<uint32_t> f(nk), l(nk);
      HIP_OK(hipMemcpyAsync(f.data(), e->rb_first.p, nk * 4ull, hipMemcpyDeviceToHost, st));
      HIP_OK(hipMemcpyAsync(l.data(), e->rb_last.p, nk * 4ull, hipMemcpyDeviceToHost, st));
      HIP_OK(hipStreamSynchronize(st));
      std::map<std::string, uint64_t> by_rx;
      uint64_t n_legacy = 0;
      for (uint32_t k = 0; k < nk; ++k) {
        const uint32_t r = k % B.n_rules;
        if (l[k] <= f[k]) continue;
        by_rx[r < rs->rules.size() ? rs->rules[r].regex.substr(0, 60) : "?"] += l[k] - f[k];
        if (k >= B.n_rules) n_legacy += l[k] - f[k];
      }
      std::vector<std::pair<uint64_t, std::string>> v;
      for (auto &kv : by_rx) v.push_back({kv.second, kv.first});
      std::sort(v.rbegin(), v.rend());
      fprintf(stderr, "BJX_JOB_STATS jobs=%llu (legacy %llu) lines=%llu\n", n_jobs, (unsigned long long)n_legacy,
              (unsigned long long)e->bc.n_lines);
      for (size_t i = 0; i < v.size() && i < 16; ++i) fprintf(stderr, "  %10llu  %s\n", (unsigned long long)v[i].first, v[i].second.c_str());
    }
  }
  HIP_OK(hipEventRecord(e->evk[3], st));
  if (n_slow) {
    WideList WL{nullptr, nullptr, nullptr, e->scalars.p + 13, 0};
    if (B.any_wide) {
      const uint64_t cap = n_slow * (uint64_t)e->n_wide + 1;
      e->wl_line.ensure(cap); e->wl_rule.ensure(cap); e->wl_pos.ensure(cap);
      WL.line = e->wl_line.p; WL.rule = e->wl_rule.p; WL.pos = e->wl_pos.p; WL.cap = cap;
      HIP_OK(hipMemsetAsync(e->scalars.p + 13, 0, 8, st));
    }
    if (all_wide) HIP_OK(hipEventRecord(e->evk[0], st));  // the per-line kernel of this batch (kernel_ms[1])
    hipLaunchKernelGGL(k_parse_match<true>, dim3(grid_for(n_slow)), dim3(kBlock), 0, st, B, buf, e->nl.p, (uint64_t)n_slow,
                       all_wide ? nullptr : e->slow_list.p, now_ns, L, e->slow_list.p, e->scalars.p, WL);
    HIP_OK(hipGetLastError());
    if (B.any_wide) {
      unsigned long long n_wl = 0;
      pin_get(e, &n_wl, e->scalars.p + 13, 8);
      pin_sync(e);
      if (n_wl > WL.cap) throw BjxError(BJX_ERR_DEVICE, "internal: wide-NFA job list overflow");
      if (n_wl) launch_wide(e, B, buf, n, e->wl_rule.p, nullptr, e->wl_line.p, e->wl_pos.p, 0, n_wl, L, e->wide_max_w, e->wide_max_g);
    }
    if (all_wide) HIP_OK(hipEventRecord(e->evk[1], st));
  }
  e->last_slow = n_slow;
  if (getenv("BJX_CHECK")) {
    e->chk.ensure(16);
    HIP_OK(hipMemsetAsync(e->chk.p, 0, 16, st));
    hipLaunchKernelGGL(k_check_masks, dim3(grid_for(n_lines)), dim3(kBlock), 0, st, n_lines, L, B.mask_words, e->chk.p);
    HIP_OK(hipGetLastError());
    unsigned long long c[2];
    pin_get(e, c, e->chk.p, 16);
    pin_sync(e);
    if (c[0]) {
      char msg[160];
      snprintf(msg, sizeof msg, "BJX_CHECK: %llu lines whose RuleResult count differs from their match mask (first %llu)", c[0],
               c[1]);
      throw BjxError(BJX_ERR_DEVICE, msg);
    }
  }
  mark(e, 3);

  // ---- RuleResults + events in reference order
  HIP_OK(hipMemsetAsync(e->l_counts.p + n_lines, 0, 8, st));
  {
    uint64_t *in = e->l_counts.p, *o = e->l_offs.p;
    cub_call(e, [&](void *tmp, size_t &bytes) {
      return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)(n_lines + 1), st);
    });
  }
  uint64_t tot = 0;
  pin_get(e, &tot, e->l_offs.p + n_lines, 8);
  pin_sync(e);
  const uint64_t n_res = tot >> 32, n_ev = tot & 0xFFFFFFFFull;
  out->n_results = n_res;
  out->n_events = n_ev;
  e->res_seq.ensure(n_res + 1); e->res_rule.ensure(n_res + 1); e->rl_out.ensure(n_res + 1);
  e->ev_el.ensure(n_ev + 1); e->ev_rule.ensure(n_ev + 1); e->ev_res.ensure(n_ev + 1);
  HIP_OK(hipMemsetAsync(e->scalars.p + 1, 0, 2 * 8, st));
  e->res_written = false;
  if (n_res) {
    const bool want_res = (flags & BJX_COPY_RESULTS) != 0;
    e->res_written = want_res;
    hipLaunchKernelGGL(k_emit, dim3((unsigned)std::min<uint64_t>(grid_for(n_lines), 4096)), dim3(kBlock), 0, st, B, n_lines, L,
                       e->l_offs.p, e->res_seq.p, e->res_rule.p, e->ev_el.p, e->ev_rule.p, e->ev_res.p, e->scalars.p + 1,
                       e->res_written);
    HIP_OK(hipGetLastError());
    if (e->res_written) HIP_OK(hipMemsetAsync(e->rl_out.p, 0, n_res, st));
  }
  mark(e, 4);
  unsigned long long bnd[2] = {0, 0};
  if (n_ev) {
    pin_get(e, bnd, e->scalars.p + 1, 16);
    if (e->want_counters) pin_get(e, e->host_counters, e->S.counters, 24);
    pin_sync(e);
    e->counters_fresh = e->want_counters;
  }
  BatchCtx &c = e->bc;
  c.buf = buf; c.n_lines = n_lines; c.n_res = n_res; c.n_ev = n_ev; c.L = L; c.n_el = bnd[0]; c.el_bytes = bnd[1];
  c.consumed = out->consumed_bytes;
  c.now_ns = now_ns;
  c.live = true;
  return true;
}

// the local batch's events as rate-limit input
static EvSrc local_evsrc(bjx_engine *e) {
  const BatchCtx &c = e->bc;
  EvSrc E;
  E.bytes = c.buf; E.nl = e->nl.p; E.rest_off = c.L.rest_off; E.ip_pos = nullptr; E.ip_len = c.L.ip_len;
  E.ip_hash = c.L.ip_hash; E.ts = c.L.ts; E.counts = c.L.counts; E.ip16 = c.L.ip16; E.n = c.n_lines;
  E.hmask = e->dbg_hash_mask;
  return E;
}

// escaped JSON of every interned rule name (LogRegexBan "trigger"), rebuilt
// when reloads intern new names
static void ensure_name_json(bjx_engine *e) {
  if (e->nm_built == e->names.size() && e->nm_off.p) return;
  std::vector<uint32_t> off;
  std::vector<uint8_t> js;
  for (const auto &nm : e->names) {
    off.push_back((uint32_t)js.size());
    const uint8_t *b = reinterpret_cast<const uint8_t *>(nm.data());
    JOut<false> c{nullptr, 0};
    json_str(c, b, (uint32_t)nm.size());
    const size_t at = js.size();
    js.resize(at + c.n);
    JOut<true> w{js.data() + at, 0};
    json_str(w, b, (uint32_t)nm.size());
  }
  off.push_back((uint32_t)js.size());
  e->nm_off.ensure(off.size());
  e->nm_json.ensure(js.size() + 16);
  HIP_OK(hipMemcpy(e->nm_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
  if (!js.empty()) HIP_OK(hipMemcpy(e->nm_json.p, js.data(), js.size(), hipMemcpyHostToDevice));
  e->nm_built = e->names.size();
}

// decision updates (one per tripped IP) and LogRegexBan lines of the batch's
// n trips (e->d_trips), copied to pinned host buffers (bans.h)
// IP bytes of each selected record (bjx_ban_batch.ip_bytes): the Update key
// for a host that handed device input, and the node's merge key
__global__ void k_ban_iplen(BanDev A, uint64_t n_ips, const bjx_ip_decision *__restrict__ sel, uint64_t *__restrict__ len) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= n_ips) len[i] = i < n_ips ? A.trips[sel[i].trip_idx].ip_len : 0;
}

__global__ void k_ban_ipcopy(BanDev A, uint64_t n_ips, const bjx_ip_decision *__restrict__ sel,
                             const uint64_t *__restrict__ off, uint8_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ips) return;
  const uint64_t t = sel[i].trip_idx;
  const uint8_t *src = trip_ip(A, t);
  uint8_t *dst = out + off[i];
  for (uint32_t k = 0, n = A.trips[t].ip_len; k < n; ++k) dst[k] = src[k];
}

static void emit_bans(bjx_engine *e, uint64_t n, bool records_only) {
  hipStream_t st = e->stream;
  ensure_name_json(e);
  BanDev A{};
  A.buf = e->bc.buf; A.trips = e->d_trips.p; A.n_trips = n; A.rules = e->bind.rules;
  A.name_off = e->nm_off.p; A.name_json = e->nm_json.p;
  A.dl_hash = e->dl_hash.p; A.dl_off = e->dl_off.p; A.dl_len = e->dl_len.p; A.dl_bytes = e->dl_bytes.p; A.n_dl = e->n_dl;
  A.tz_offset_s = e->ban_tz;
  A.tz_at = e->tz_at.p; A.tz_off = e->tz_off.p; A.n_tz = e->n_tz;
  const int64_t expires = (int64_t)((uint64_t)e->bc.now_ns + (uint64_t)e->ban_ttl_ns);
  // ban-log lines: lengths, offsets, bytes (BJX_BAN_RECORDS_ONLY: none)
  e->ban_off.resize(n + 1);
  e->ban_kind.resize(n);
  if (records_only) {
    memset(e->ban_off.data(), 0, (n + 1) * 8);
    memset(e->ban_kind.data(), 0, n);
  } else {
    e->bn_len.ensure(n + 1); e->bn_off.ensure(n + 1); e->bn_kind.ensure(n);
    hipLaunchKernelGGL(k_ban_len, dim3(grid_for(n + 1)), dim3(kBlock), 0, st, A, e->bn_len.p, e->bn_kind.p);
    HIP_OK(hipGetLastError());
    {
      uint64_t *in = e->bn_len.p, *o = e->bn_off.p;
      cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)(n + 1), st); });
    }
    HIP_OK(hipMemcpyAsync(e->ban_off.data(), e->bn_off.p, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(e->ban_kind.data(), e->bn_kind.p, n, hipMemcpyDeviceToHost, st));
  }
  // per-IP escalation: sort trips by IP hash (stable: trip order within a run)
  e->bn_key.ensure(n); e->bn_key2.ensure(n); e->bn_val.ensure(n); e->bn_val2.ensure(n); e->bn_head.ensure(n);
  e->bn_seg.ensure(n);
  hipLaunchKernelGGL(k_ban_keys, dim3(grid_for(n)), dim3(kBlock), 0, st, A, e->dbg_hash_mask ? e->dbg_hash_mask : ~0ull,
                     e->bn_key.p, e->bn_val.p);
  HIP_OK(hipGetLastError());
  {
    uint64_t *ki = e->bn_key.p, *ko = e->bn_key2.p;
    uint32_t *vi = e->bn_val.p, *vo = e->bn_val2.p;
    cub_call(e, [&](void *tmp, size_t &bytes) {
      return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, ki, ko, vi, vo, (int)n, 0, 64, st);
    });
  }
  hipLaunchKernelGGL(k_ban_heads, dim3(grid_for(n)), dim3(kBlock), 0, st, n, e->bn_key2.p, e->bn_head.p);
  {
    uint32_t *in = e->bn_head.p, *o = e->bn_seg.p;
    cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::InclusiveSum(tmp, bytes, in, o, (int)n, st); });
  }
  uint32_t n_seg = 0;
  pin_get(e, &n_seg, e->bn_seg.p + (n - 1), 4);
  pin_sync(e);
  const uint64_t log_bytes = e->ban_off.data()[n];
  // A trip burst's log can be several times the usual one (cfg3: 0.5 -> 3.4 GB
  // every few dozen batches), and pinning it the first time stalls that batch
  // for ~0.1 ms/MB: the first log buffer already holds half the batch's
  // bytes (at most 16 GB; cfg3's largest bursts: 13M trips, about 5 GB)
  if (log_bytes) e->ban_log.reserve(std::min<uint64_t>(e->bc.consumed / 2, 16ull << 30));
  e->ban_log.resize(log_bytes);
  bool log_copy = false;
  if (log_bytes) {
    // The log leaves on its own stream, in chunks of trips, each chunk as soon
    // as its lines are written: the PCIe copy overlaps the next chunk's writes
    // and the per-IP reduce below; the engine stream joins the copies at the
    // end of emit_bans, so the batch's final sync still covers them.
    e->bn_log.ensure(log_bytes + 16);
    if (!e->bstream) {
      HIP_OK(hipStreamCreateWithFlags(&e->bstream, hipStreamNonBlocking));
      for (auto &x : e->bev) HIP_OK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    }
    const uint64_t nch = log_bytes > kBanChunkMin ? (uint64_t)kBanChunks : 1u;
    const uint64_t *ho = e->ban_off.data();
    for (uint64_t c = 0; c < nch; ++c) {
      const uint64_t a = n * c / nch, b = n * (c + 1) / nch;
      if (a == b) continue;
      hipLaunchKernelGGL(k_ban_write, dim3(grid_for(b - a)), dim3(kBlock), 0, st, A, e->bn_off.p, e->bn_log.p, a, b);
      HIP_OK(hipGetLastError());
      if (ho[b] == ho[a]) continue;
      HIP_OK(hipEventRecord(e->bev[c], st));
      HIP_OK(hipStreamWaitEvent(e->bstream, e->bev[c], 0));
      HIP_OK(hipMemcpyAsync(e->ban_log.data() + ho[a], e->bn_log.p + ho[a], ho[b] - ho[a], hipMemcpyDeviceToHost, e->bstream));
    }
    HIP_OK(hipEventRecord(e->bev[kBanChunks], e->bstream));
    log_copy = true;
  }
  e->bn_first.ensure(n_seg); e->bn_cnt.ensure(n_seg); e->bn_ipt.ensure(n_seg); e->bn_coll.ensure(n_seg);
  e->bn_best.ensure(n_seg); e->bn_flag.ensure(n); e->bn_rep.ensure(n); e->bn_sel.ensure(n);
  HIP_OK(hipMemsetAsync(e->bn_cnt.p, 0, n_seg * 4ull, st));
  HIP_OK(hipMemsetAsync(e->bn_ipt.p, 0, n_seg * 4ull, st));
  HIP_OK(hipMemsetAsync(e->bn_coll.p, 0, n_seg * 4ull, st));
  HIP_OK(hipMemsetAsync(e->bn_best.p, 0, n_seg * 8ull, st));
  HIP_OK(hipMemsetAsync(e->bn_flag.p, 0, n, st));
  hipLaunchKernelGGL(k_ban_reduce, dim3(grid_for(n)), dim3(kBlock), 0, st, A, n, e->bn_key2.p, e->bn_val2.p, e->bn_seg.p,
                     e->bn_first.p, e->bn_best.p, e->bn_cnt.p, e->bn_ipt.p, e->bn_coll.p);
  hipLaunchKernelGGL(k_ban_out, dim3(grid_for(n_seg)), dim3(kBlock), 0, st, (uint64_t)n_seg, e->bn_best.p, e->bn_cnt.p,
                     e->bn_ipt.p, e->bn_coll.p, expires, e->bn_flag.p, e->bn_rep.p);
  hipLaunchKernelGGL(k_ban_collide, dim3(grid_for(n_seg)), dim3(kBlock), 0, st, A, n, (uint64_t)n_seg, e->bn_val2.p,
                     e->bn_first.p, e->bn_coll.p, expires, e->bn_flag.p, e->bn_rep.p);
  HIP_OK(hipGetLastError());
  {
    const bjx_ip_decision *in = e->bn_rep.p;
    const uint8_t *fl = e->bn_flag.p;
    bjx_ip_decision *o = e->bn_sel.p;
    unsigned long long *cnt = e->scalars.p + 5;
    cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceSelect::Flagged(tmp, bytes, in, fl, o, cnt, (int)n, st); });
  }
  unsigned long long n_ips = 0;
  pin_get(e, &n_ips, e->scalars.p + 5, 8);
  pin_sync(e);
  e->ban_ips.resize(n_ips);
  e->ban_ipo.resize(n_ips + 1);
  e->ban_ipo.data()[0] = 0;
  e->ban_ipb.resize(0);
  if (n_ips) {
    HIP_OK(hipMemcpyAsync(e->ban_ips.data(), e->bn_sel.p, n_ips * sizeof(bjx_ip_decision), hipMemcpyDeviceToHost, st));
    // scratch for the IP lengths / offsets (the log offsets are on the host
    // already); sized here, since a records-only batch never sized them
    e->bn_len.ensure(n_ips + 1); e->bn_off.ensure(n_ips + 1);
    uint64_t *len = e->bn_len.p, *off = e->bn_off.p;
    hipLaunchKernelGGL(k_ban_iplen, dim3(grid_for(n_ips + 1)), dim3(kBlock), 0, st, A, (uint64_t)n_ips, e->bn_sel.p, len);
    cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, len, off, (int)(n_ips + 1), st); });
    HIP_OK(hipMemcpyAsync(e->ban_ipo.data(), off, (n_ips + 1) * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    const uint64_t nb = e->ban_ipo.data()[n_ips];
    e->bn_ipb.ensure(nb + 16);
    hipLaunchKernelGGL(k_ban_ipcopy, dim3(grid_for(n_ips)), dim3(kBlock), 0, st, A, (uint64_t)n_ips, e->bn_sel.p, off,
                       e->bn_ipb.p);
    HIP_OK(hipGetLastError());
    e->ban_ipb.resize(nb);
    if (nb) HIP_OK(hipMemcpyAsync(e->ban_ipb.data(), e->bn_ipb.p, nb, hipMemcpyDeviceToHost, st));
  }
  if (log_copy) HIP_OK(hipStreamWaitEvent(st, e->bev[kBanChunks], 0));
  e->ban_n_trips = n;
}

// Where finish_phase finds the trips: Apply outcomes in state-slot order (this
// engine's rate-limit stage), outcomes in event order (a node's
// bjx_finish_batch), or a list of the tripping events (bjx_finish_batch_trips)
enum FinishFrom { kFinSorted, kFinEvents, kFinList };

// Exceeded events -> their event indices, ascending, in e->trip_ev2 (count
// returned).  kFinList: the n_list indices are already in e->trip_idx.
static uint64_t trip_events(bjx_engine *e, uint64_t n_ev, FinishFrom from, uint64_t n_list) {
  hipStream_t st = e->stream;
  uint64_t n_trips = n_list;
  if (from != kFinList) {
    e->trip_idx.ensure(n_ev + 1);
    HIP_OK(hipMemsetAsync(e->scalars.p + 4, 0, 8, st));
    hipLaunchKernelGGL(k_select_trips, dim3(grid_for((n_ev + kSelPer - 1) / kSelPer)), dim3(kBlock), 0, st, n_ev,
                       from == kFinSorted ? e->ev_out_s.p : e->ev_out.p, e->trip_idx.p, e->scalars.p + 4);
    HIP_OK(hipGetLastError());
    unsigned long long nt = 0;
    pin_get(e, &nt, e->scalars.p + 4, 8);
    pin_sync(e);
    n_trips = nt;
  }
  if (!n_trips) return 0;
  e->trip_ev.ensure(n_trips); e->trip_ev2.ensure(n_trips);
  if (from == kFinSorted)
    hipLaunchKernelGGL(k_trip_events, dim3(grid_for(n_trips)), dim3(kBlock), 0, st, n_trips, e->trip_idx.p, ev_words(e),
                       rec_stride(e), e->trip_ev.p);
  uint32_t *ki = from == kFinSorted ? e->trip_ev.p : e->trip_idx.p, *ko = e->trip_ev2.p;
  const int bits = std::max(1, bit_width(n_ev));
  cub_call(e, [&](void *tmp, size_t &bytes) {
    return hipcub::DeviceRadixSort::SortKeys(tmp, bytes, ki, ko, (int)n_trips, 0, bits, st);
  });
  if (from == kFinList && n_trips > 1) {
    // the owners' lists are sets of distinct events: a repeated index would
    // duplicate a trip (and its ban count) silently
    HIP_OK(hipMemsetAsync(e->scalars.p + 6, 0, 8, st));
    hipLaunchKernelGGL(k_count_dups, dim3(grid_for(n_trips)), dim3(kBlock), 0, st, n_trips, ko, e->scalars.p + 6);
    HIP_OK(hipGetLastError());
    unsigned long long dups = 0;
    pin_get(e, &dups, e->scalars.p + 6, 8);
    pin_sync(e);
    if (dups) throw BjxError(BJX_ERR_ARG, "bjx_finish_batch_trips: an event index appears more than once");
  }
  return n_trips;
}

// Trips (reference order) and the optional per-line / RuleResult copies, once
// the local events' Apply outcomes are known (phases 7-8).
static void finish_phase(bjx_engine *e, uint32_t flags, bjx_batch_result *out, FinishFrom from, uint64_t n_list = 0) {
  const Bind &B = e->bind;
  hipStream_t st = e->stream;
  const BatchCtx &c = e->bc;
  const uint64_t n_lines = c.n_lines, n_res = c.n_res, n_ev = c.n_ev;
  const Lines &L = c.L;
  uint64_t n_trips = 0;
  e->ban_emitted = (flags & BJX_EMIT_BANS) != 0;
  e->ban_n_trips = 0;
  e->ban_ips.resize(0); e->ban_log.resize(0); e->ban_off.resize(1); e->ban_off.data()[0] = 0; e->ban_kind.resize(0);
  e->ban_ipb.resize(0); e->ban_ipo.resize(1); e->ban_ipo.data()[0] = 0;
  if (n_ev) {
    mark(e, 7);
    // the trips in reference (event) order
    n_trips = trip_events(e, n_ev, from, n_list);
    if (n_trips) {
      e->d_trips.ensure(n_trips);
      hipLaunchKernelGGL(k_build_trips, dim3(grid_for(n_trips)), dim3(kBlock), 0, st, n_trips, e->trip_ev2.p, e->ev_el.p,
                         e->ev_rule.p, c.buf, e->nl.p, L, B.rules, e->d_trips.p);
      HIP_OK(hipGetLastError());
      if (flags & BJX_TRIPS_COMPACT) {
        e->d_trips_c.ensure(n_trips);
        hipLaunchKernelGGL(k_pack_trips, dim3(grid_for(n_trips)), dim3(kBlock), 0, st, n_trips, e->d_trips.p, e->d_trips_c.p);
        HIP_OK(hipGetLastError());
        e->trips_c.resize(n_trips);
        HIP_OK(hipMemcpyAsync(e->trips_c.data(), e->d_trips_c.p, n_trips * 8, hipMemcpyDeviceToHost, st));
      } else {
        e->trips.resize(n_trips);
        HIP_OK(hipMemcpyAsync(e->trips.data(), e->d_trips.p, n_trips * sizeof(bjx_trip), hipMemcpyDeviceToHost, st));
      }
      if (flags & BJX_EMIT_BANS) emit_bans(e, n_trips, (flags & BJX_BAN_RECORDS_ONLY) != 0);
    }
    if ((flags & BJX_COPY_RESULTS) && !e->res_written) {
      // the match phase ran without BJX_COPY_RESULTS: write the RuleResult
      // arrays now (the per-line masks and offsets are still current)
      HIP_OK(hipMemsetAsync(e->scalars.p + 1, 0, 2 * 8, st));
      hipLaunchKernelGGL(k_emit, dim3((unsigned)std::min<uint64_t>(grid_for(n_lines), 4096)), dim3(kBlock), 0, st, e->bind,
                         n_lines, L, e->l_offs.p, e->res_seq.p, e->res_rule.p, e->ev_el.p, e->ev_rule.p, e->ev_res.p,
                         e->scalars.p + 1, true);
      HIP_OK(hipGetLastError());
      HIP_OK(hipMemsetAsync(e->rl_out.p, 0, n_res, st));
      e->res_written = true;
    }
    if (flags & BJX_COPY_RESULTS) {
      if (from == kFinSorted)
        hipLaunchKernelGGL(k_unsort, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, n_ev, ev_words(e), rec_stride(e), e->ev_out_s.p,
                           e->ev_out.p);
      hipLaunchKernelGGL(k_scatter_rl, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, n_ev, e->ev_res.p, e->ev_out.p, e->rl_out.p);
      HIP_OK(hipGetLastError());
      if (getenv("BJX_CHECK")) {  // every event names its own RuleResult (ev_res injective)
        e->chk_w.ensure(n_res + 1);
        e->chk.ensure(16);
        HIP_OK(hipMemsetAsync(e->chk_w.p, 0, (n_res + 1) * 4, st));
        HIP_OK(hipMemsetAsync(e->chk.p, 0, 32, st));
        hipLaunchKernelGGL(k_check_count, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, n_ev, e->ev_res.p, 1u, n_res, e->chk_w.p,
                           e->chk.p);
        hipLaunchKernelGGL(k_check_most, dim3(grid_for(n_res)), dim3(kBlock), 0, st, n_res, e->chk_w.p, 1u, e->chk.p);
        HIP_OK(hipGetLastError());
        unsigned long long c[3];
        pin_get(e, c, e->chk.p, 24);
        pin_sync(e);
        if (c[0] || c[1]) {
          char msg[256];
          snprintf(msg, sizeof msg, "BJX_CHECK: %llu event result indices out of range, %llu RuleResults named by more than "
                   "one event (first %llu)", c[0], c[1], c[2]);
          throw BjxError(BJX_ERR_DEVICE, msg);
        }
      }
    }
  }
  HIP_OK(hipEventRecord(e->ev1, st));
  mark(e, 8);
  if (flags & BJX_COPY_RESULTS) {
    hipLaunchKernelGGL(k_final_flags, dim3(grid_for(n_lines)), dim3(kBlock), 0, st, n_lines, e->l_flags.p);
    e->line_flags.resize(n_lines);
    HIP_OK(hipMemcpyAsync(e->line_flags.data(), e->l_flags.p, n_lines, hipMemcpyDeviceToHost, st));
    if (n_res) {
      e->d_results.ensure(n_res);
      hipLaunchKernelGGL(k_build_results, dim3(grid_for(n_res)), dim3(kBlock), 0, st, n_res, e->res_seq.p, e->res_rule.p,
                         e->rl_out.p, e->d_results.p);
      e->results.resize(n_res);
      HIP_OK(hipMemcpyAsync(e->results.data(), e->d_results.p, n_res * sizeof(bjx_rule_result), hipMemcpyDeviceToHost, st));
    }
  }
  HIP_OK(hipStreamSynchronize(st));
  float ms = 0, mms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e->ev0, e->ev1));
  HIP_OK(hipEventElapsedTime(&mms, e->evm0, e->evm1));
  {
    float kl = 0, kd = 0;
    HIP_OK(hipEventElapsedTime(&kl, e->evk[0], e->evk[1]));
    HIP_OK(hipEventElapsedTime(&kd, e->evk[2], e->evk[3]));
    e->kernel_ms[0] = mms; e->kernel_ms[1] = kl; e->kernel_ms[2] = kd;
  }
  out->device_ms = ms;
  out->match_kernel_ms = mms;
  for (int k = 0; k < bjx_engine::kPhases; ++k) {
    e->phase_ms[k] = 0;
    if (!e->phase_rec[k]) continue;
    int j = k + 1;
    while (j <= bjx_engine::kPhases && !e->phase_rec[j]) ++j;
    if (j > bjx_engine::kPhases) continue;
    float x = 0;
    HIP_OK(hipEventElapsedTime(&x, e->ph[k], e->ph[j]));
    e->phase_ms[k] = x;
  }
  out->n_trips = n_trips;
  const bool compact = (flags & BJX_TRIPS_COMPACT) != 0;
  out->trips = compact || !n_trips ? nullptr : e->trips.data();
  out->trips_compact = !compact || !n_trips ? nullptr : e->trips_c.data();
  out->results = e->results.empty() ? nullptr : e->results.data();
  out->line_flags = e->line_flags.empty() ? nullptr : e->line_flags.data();
}

static void run_batch(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns, uint32_t flags,
                      bjx_batch_result *out) {
  // a standalone batch has no exchange: no node batch's figure carries over
  e->exchange_ms = 0;
  e->xev_rec = false;
  e->counters_fresh = false;
  e->want_counters = true;
  struct Reset {  // whatever way match_phase leaves
    bjx_engine *e;
    ~Reset() { e->want_counters = false; }
  } reset{e};
  if (!match_phase(e, rs, bytes, n, now_ns, flags, out)) { e->counters_fresh = false; return; }
  e->want_counters = false;
  if (e->bc.n_ev) {
    rate_limit_stage(e, e->bind, local_evsrc(e), e->bc.n_el, e->bc.el_bytes, e->bc.n_ev, e->ev_el.p, e->ev_rule.p,
                     e->bc.now_ns);
  }
  finish_phase(e, flags, out, kFinSorted);
}

extern "C" int bjx_process_batch(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns,
                                 uint32_t flags, bjx_batch_result *out) {
  if (!e || !rs || !out || (n && !bytes)) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    run_batch(e, rs, bytes, n, now_ns, flags, out);
    return BJX_OK;
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  } catch (const std::bad_alloc &) {
    e->last_error = "host out of memory";
    return BJX_ERR_NOMEM;
  }
}

// ------------------------------------------------------------ multi-GPU batch

template <typename F>
static int guarded(bjx_engine *e, F f) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    return f();
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  } catch (const std::bad_alloc &) {
    e->last_error = "host out of memory";
    return BJX_ERR_NOMEM;
  }
}

extern "C" int bjx_match_batch(bjx_engine *e, const bjx_ruleset *rs, const uint8_t *bytes, size_t n, int64_t now_ns,
                               uint32_t flags, bjx_batch_result *out) {
  if (!rs || !out || (n && !bytes)) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    e->partitioned = false;
    e->exchange_ms = 0;  // set by this batch's bjx_events_partition .. apply, if any
    e->xev_rec = false;
    match_phase(e, rs, bytes, n, now_ns, flags, out);
    return BJX_OK;
  });
}

extern "C" int bjx_events_partition(bjx_engine *e, uint32_t n_parts, uint64_t *counts) {
  if (!counts || n_parts == 0 || n_parts > kMaxParts) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    const BatchCtx &c = e->bc;
    memset(counts, 0, sizeof(uint64_t) * 3 * n_parts);
    e->pk_parts = n_parts;
    e->pk_n_ev = 0;
    e->partitioned = true;
    if (!c.live || c.n_ev == 0) return BJX_OK;
    hipStream_t st = e->stream;
    HIP_OK(hipEventRecord(e->xev[0], st));
    e->xev_rec = true;
    const uint64_t nl = c.n_lines;
    // one step per tile (the most blocks in flight) unless the [owner][tile]
    // arrays would pass 4M entries
    const uint64_t rows = (nl + kBlock - 1) / kBlock;
    const uint32_t steps = (uint32_t)std::max<uint64_t>(1, (rows * n_parts + (1u << 22) - 1) >> 22);
    const uint32_t n_tiles = (uint32_t)((rows + steps - 1) / steps);
    const uint64_t S = (uint64_t)n_parts * n_tiles + 1;
    e->pk_hist.ensure(3 * S); e->pk_off.ensure(3 * S);
    e->pk_counts.ensure(3 * n_parts + 1); e->pk_bbase.ensure(n_parts);
    e->pk_tiles = n_tiles;
    e->pk_steps = steps;
    HIP_OK(hipMemsetAsync(e->pk_counts.p + 3 * n_parts, 0, 8, st));
    for (int k = 0; k < 3; ++k) HIP_OK(hipMemsetAsync(e->pk_hist.p + k * S + S - 1, 0, 8, st));
    hipLaunchKernelGGL(k_part_count, dim3(n_tiles), dim3(kBlock), 0, st, nl, n_tiles, steps, c.L, n_parts, e->pk_hist.p,
                       reinterpret_cast<unsigned long long *>(e->pk_counts.p + 3 * n_parts));
    HIP_OK(hipGetLastError());
    for (int k = 0; k < 3; ++k) {
      uint64_t *in = e->pk_hist.p + k * S, *o = e->pk_off.p + k * S;
      cub_call(e, [&](void *tmp, size_t &bytes) { return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)S, st); });
    }
    hipLaunchKernelGGL(k_part_counts, dim3(1), dim3(64), 0, st, n_parts, n_tiles, e->pk_off.p, e->pk_counts.p, e->pk_bbase.p);
    HIP_OK(hipGetLastError());
    uint64_t wide = 0;
    pin_get(e, counts, e->pk_counts.p, 3 * n_parts * 8);
    pin_get(e, &wide, e->pk_counts.p + 3 * n_parts, 8);
    pin_sync(e);
    if (wide) {
      e->partitioned = false;
      throw BjxError(BJX_ERR_CAPACITY, "an event line's IP (or event count) exceeds the exchange record's 16-bit field (65535)");
    }
    uint64_t tl = 0, te = 0;
    for (uint32_t k = 0; k < n_parts; ++k) { tl += counts[3 * k]; te += counts[3 * k + 1]; }
    if (tl != c.n_el || te != c.n_ev) throw BjxError(BJX_ERR_DEVICE, "internal: partition counts disagree with the batch");
    e->pk_n_ev = te;
    return BJX_OK;
  });
}

extern "C" int bjx_events_pack(bjx_engine *e, bjx_event_line *d_lines, uint32_t *d_events, uint8_t *d_bytes) {
  return guarded(e, [&]() -> int {
    const BatchCtx &c = e->bc;
    if (!e->partitioned) throw BjxError(BJX_ERR_ARG, "bjx_events_pack before bjx_events_partition");
    if (!c.live || c.n_ev == 0) return BJX_OK;
    if (!d_lines || !d_events || (c.el_bytes && !d_bytes)) return BJX_ERR_ARG;
    hipStream_t st = e->stream;
    e->pack_src.ensure(c.n_ev);
    PackArgs A;
    A.n_lines = c.n_lines; A.n_tiles = e->pk_tiles; A.n_parts = e->pk_parts; A.steps = e->pk_steps; A.off = e->pk_off.p; A.byte_base = e->pk_bbase.p;
    A.buf = c.buf; A.nl = e->nl.p; A.L = c.L; A.offs = e->l_offs.p; A.ev_rule = e->ev_rule.p;
    A.d_lines = d_lines; A.d_events = d_events; A.d_bytes = d_bytes; A.pack_src = e->pack_src.p;
    const uint32_t lds = pack_lds_bytes(A.n_parts);
    if (lds > 64 * 1024)
      HIP_OK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pack), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_pack, dim3(A.n_tiles), dim3(kBlock), lds, st, A);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(st));
    return BJX_OK;
  });
}

// the received records of n_src sources through the rate-limit stage;
// d_out: each event's outcome byte in received order (nullptr: left in
// state-slot order, e->ev_out_s)
static int apply_received(bjx_engine *e, const bjx_ruleset *rs, const bjx_event_line *d_lines, const uint32_t *d_events,
                          const uint8_t *d_bytes, uint32_t n_src, const uint64_t *src_counts, uint8_t *d_out) {
  uint64_t n_lines = 0, n_ev = 0, n_bytes = 0;
  for (uint32_t k = 0; k < n_src; ++k) {
    n_lines += src_counts[3 * k];
    n_ev += src_counts[3 * k + 1];
    n_bytes += src_counts[3 * k + 2];
  }
  if (n_ev == 0) return BJX_OK;
  if (!d_lines || !d_events || (n_bytes && !d_bytes)) return BJX_ERR_ARG;
  if (e->bound_uid != rs->uid || e->bound_dec_version != e->decisions_version) bind_ruleset(e, rs, nullptr, 0);
  const Bind &B = e->bind;
  hipStream_t st = e->stream;
  e->rx_ts.ensure(n_lines); e->rx_hash.ensure(n_lines); e->rx_pos.ensure(n_lines); e->rx_len.ensure(n_lines);
  e->rx_nev.ensure(n_lines + 1); e->rx_evoff.ensure(n_lines + 1); e->rx_ev_el.ensure(n_ev); e->rx_ip16.ensure(n_lines);
  uint64_t first = 0, bbase = 0;
  for (uint32_t k = 0; k < n_src; ++k) {
    const uint64_t nk = src_counts[3 * k];
    if (nk)
      hipLaunchKernelGGL(k_unpack_lines, dim3(grid_for(nk)), dim3(kBlock), 0, st, nk, first, bbase, d_lines, d_bytes,
                         e->rx_ts.p, e->rx_hash.p, e->rx_pos.p, e->rx_len.p, e->rx_nev.p, e->rx_ip16.p, e->dbg_hash_mask);
    first += nk;
    bbase += src_counts[3 * k + 2];
  }
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemsetAsync(e->rx_nev.p + n_lines, 0, 8, st));
  {
    uint64_t *in = e->rx_nev.p, *o = e->rx_evoff.p;
    cub_call(e, [&](void *tmp, size_t &bytes) {
      return hipcub::DeviceScan::ExclusiveSum(tmp, bytes, in, o, (int)(n_lines + 1), st);
    });
  }
  HIP_OK(hipMemsetAsync(e->scalars.p + 6, 0, 8, st));
  hipLaunchKernelGGL(k_expand_events, dim3(grid_for(n_lines)), dim3(kBlock), 0, st, n_lines, e->rx_evoff.p, e->rx_nev.p,
                     n_ev, d_events, B.n_rules, e->rx_ev_el.p, e->scalars.p + 6);
  HIP_OK(hipGetLastError());
  uint64_t chk[2] = {0, 0};
  pin_get(e, &chk[0], e->rx_evoff.p + n_lines, 8);
  pin_get(e, &chk[1], e->scalars.p + 6, 8);
  pin_sync(e);
  if (chk[0] != n_ev || chk[1]) throw BjxError(BJX_ERR_ARG, "received event records are inconsistent");
  EvSrc E;
  E.bytes = d_bytes; E.nl = nullptr; E.rest_off = nullptr; E.ip_pos = e->rx_pos.p; E.ip_len = e->rx_len.p;
  E.ip_hash = e->rx_hash.p; E.ts = e->rx_ts.p; E.counts = nullptr; E.ip16 = e->rx_ip16.p; E.n = n_lines;
  E.hmask = 0;  // k_unpack_lines applied the test mask
  // the clock of this engine's last match phase (the node's batch) as the
  // 12-B records' base; a stale or foreign one only costs the 16-B re-claim
  const bool timed = e->xev_rec;
  if (timed) HIP_OK(hipEventRecord(e->xev[1], st));
  e->xev_rec = false;
  rate_limit_stage(e, B, E, n_lines, n_bytes, n_ev, e->rx_ev_el.p, d_events, e->bc.now_ns ? e->bc.now_ns : kNoRecBase);
  e->exchange_ms = 0;
  if (timed) {
    float x = 0;
    HIP_OK(hipEventElapsedTime(&x, e->xev[0], e->xev[1]));
    e->exchange_ms = x;
  }
  if (d_out) {
    hipLaunchKernelGGL(k_unsort, dim3(grid_for(n_ev)), dim3(kBlock), 0, st, n_ev, ev_words(e), rec_stride(e), e->ev_out_s.p,
                       d_out);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(st));
  }
  return BJX_OK;
}

extern "C" int bjx_apply_events(bjx_engine *e, const bjx_ruleset *rs, const bjx_event_line *d_lines, const uint32_t *d_events,
                                const uint8_t *d_bytes, uint32_t n_src, const uint64_t *src_counts, uint8_t *d_out) {
  if (!rs || (n_src && !src_counts)) return BJX_ERR_ARG;
  uint64_t n_ev = 0;
  for (uint32_t k = 0; k < n_src; ++k) n_ev += src_counts[3 * k + 1];
  if (n_ev && !d_out) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int { return apply_received(e, rs, d_lines, d_events, d_bytes, n_src, src_counts, d_out); });
}

extern "C" int bjx_finish_batch(bjx_engine *e, const uint8_t *d_outcomes, uint32_t flags, bjx_batch_result *out) {
  if (!out) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    const BatchCtx &c = e->bc;
    memset(out, 0, sizeof *out);
    if (!c.live) return BJX_OK;
    if (c.n_ev) {
      if (!e->partitioned || e->pk_n_ev != c.n_ev || !d_outcomes) throw BjxError(BJX_ERR_ARG, "bjx_finish_batch without a packed batch");
      e->ev_out.ensure(c.n_ev);
      hipLaunchKernelGGL(k_scatter_outcomes, dim3(grid_for(c.n_ev)), dim3(kBlock), 0, e->stream, c.n_ev, e->pack_src.p,
                         d_outcomes, e->ev_out.p);
      HIP_OK(hipGetLastError());
    }
    out->n_lines = c.n_lines;
    out->consumed_bytes = c.consumed;
    out->n_results = c.n_res;
    out->n_events = c.n_ev;
    finish_phase(e, flags, out, kFinEvents);
    e->partitioned = false;
    return BJX_OK;
  });
}

extern "C" int bjx_apply_events_trips(bjx_engine *e, const bjx_ruleset *rs, const bjx_event_line *d_lines,
                                      const uint32_t *d_events, const uint8_t *d_bytes, uint32_t n_src,
                                      const uint64_t *src_counts, const uint64_t *trip_base, uint32_t *d_trips,
                                      uint64_t *trip_counts) {
  if (!rs || (n_src && (!src_counts || !trip_base || !trip_counts)) || n_src > kMaxParts) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    for (uint32_t k = 0; k < n_src; ++k) trip_counts[k] = 0;
    uint64_t n_ev = 0;
    std::vector<uint64_t> host(2 * (size_t)n_src + 1);
    for (uint32_t k = 0; k < n_src; ++k) {
      host[k] = n_ev;
      n_ev += src_counts[3 * k + 1];
    }
    host[n_src] = n_ev;
    if (n_ev == 0) return BJX_OK;
    if (!d_trips) return BJX_ERR_ARG;
    for (uint32_t k = 0; k < n_src; ++k) host[n_src + 1 + k] = trip_base[k];
    // the rate-limit stage on the received records, outcomes left in
    // state-slot order (no event-order copy)
    const int rc = apply_received(e, rs, d_lines, d_events, d_bytes, n_src, src_counts, nullptr);
    if (rc != BJX_OK) return rc;
    hipStream_t st = e->stream;
    const uint64_t n_trips = trip_events(e, n_ev, kFinSorted, 0);
    if (!n_trips) return BJX_OK;
    e->tr_base.ensure(host.size() + n_src);
    uint64_t *ev_base = e->tr_base.p, *base = ev_base + n_src + 1, *start = base + n_src;
    HIP_OK(hipMemcpyAsync(ev_base, host.data(), host.size() * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(start, 0xFF, n_src * 8ull, st));
    hipLaunchKernelGGL(k_trip_rebase, dim3(grid_for(n_trips)), dim3(kBlock), 0, st, n_trips, e->trip_ev2.p, n_src, ev_base, base,
                       d_trips, start);
    HIP_OK(hipGetLastError());
    std::vector<uint64_t> first(n_src);
    HIP_OK(hipMemcpyAsync(first.data(), start, n_src * 8ull, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    uint64_t nxt = n_trips;
    for (int k = (int)n_src - 1; k >= 0; --k) {
      if (first[k] > nxt) first[k] = nxt;  // no trips: empty at the next source's start
      trip_counts[k] = nxt - first[k];
      nxt = first[k];
    }
    return BJX_OK;
  });
}

extern "C" int bjx_finish_batch_trips(bjx_engine *e, const uint32_t *d_trips, uint64_t n, uint32_t flags, bjx_batch_result *out) {
  if (!out || (n && !d_trips)) return BJX_ERR_ARG;
  if (flags & BJX_COPY_RESULTS) return BJX_ERR_ARG;  // per-event outcomes: bjx_finish_batch
  return guarded(e, [&]() -> int {
    const BatchCtx &c = e->bc;
    memset(out, 0, sizeof *out);
    if (!c.live) return BJX_OK;
    if (c.n_ev) {
      if (!e->partitioned || e->pk_n_ev != c.n_ev) throw BjxError(BJX_ERR_ARG, "bjx_finish_batch_trips without a packed batch");
      if (n > c.n_ev) throw BjxError(BJX_ERR_ARG, "bjx_finish_batch_trips: more trips than packed events");
    } else if (n) {
      throw BjxError(BJX_ERR_ARG, "bjx_finish_batch_trips: trips for a batch without events");
    }
    if (n) {
      hipStream_t st = e->stream;
      e->trip_idx.ensure(n + 1);
      HIP_OK(hipMemsetAsync(e->scalars.p + 6, 0, 8, st));
      hipLaunchKernelGGL(k_map_trips, dim3(grid_for(n)), dim3(kBlock), 0, st, n, d_trips, c.n_ev, e->pack_src.p, e->trip_idx.p,
                         e->scalars.p + 6);
      HIP_OK(hipGetLastError());
      unsigned long long bad = 0;
      pin_get(e, &bad, e->scalars.p + 6, 8);
      pin_sync(e);
      if (bad) throw BjxError(BJX_ERR_ARG, "bjx_finish_batch_trips: packed event index out of range");
    }
    out->n_lines = c.n_lines;
    out->consumed_bytes = c.consumed;
    out->n_results = c.n_res;
    out->n_events = c.n_ev;
    finish_phase(e, flags, out, kFinList, n);
    e->partitioned = false;
    return BJX_OK;
  });
}

extern "C" int bjx_engine_set_ban_options(bjx_engine *e, const bjx_ban_options *o) {
  if (!o || (o->n_disable_logging && !o->disable_logging) || (o->n_tz_transitions && !o->tz_transitions) ||
      o->n_tz_transitions >= (1u << 24))
    return BJX_ERR_ARG;
  for (size_t i = 1; i < o->n_tz_transitions; ++i)
    if (o->tz_transitions[i].utc_start_s <= o->tz_transitions[i - 1].utc_start_s) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    e->ban_ttl_ns = o->expiring_ttl_ns;
    e->ban_tz = o->tz_offset_s;
    std::vector<int64_t> tz_at(o->n_tz_transitions);
    std::vector<int32_t> tz_off(o->n_tz_transitions);
    for (size_t i = 0; i < o->n_tz_transitions; ++i) {
      tz_at[i] = o->tz_transitions[i].utc_start_s;
      tz_off[i] = o->tz_transitions[i].offset_s;
    }
    e->n_tz = (uint32_t)tz_at.size();
    e->tz_at.ensure(std::max<size_t>(1, tz_at.size())); e->tz_off.ensure(std::max<size_t>(1, tz_off.size()));
    if (!tz_at.empty()) {
      HIP_OK(hipMemcpy(e->tz_at.p, tz_at.data(), tz_at.size() * 8, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(e->tz_off.p, tz_off.data(), tz_off.size() * 4, hipMemcpyHostToDevice));
    }
    std::vector<std::pair<uint64_t, std::string>> hs;
    for (size_t i = 0; i < o->n_disable_logging; ++i) {
      const bjx_str &h = o->disable_logging[i];
      if (h.len && !h.ptr) return BJX_ERR_ARG;
      std::string x(h.ptr ? h.ptr : "", h.len);
      std::vector<uint8_t> pad(x.begin(), x.end());
      pad.resize(x.size() + 8, 0);
      hs.emplace_back(hash_bytes(pad.data(), (uint32_t)x.size()), x);
    }
    std::sort(hs.begin(), hs.end());
    hs.erase(std::unique(hs.begin(), hs.end()), hs.end());
    std::vector<uint64_t> hh;
    std::vector<uint32_t> off, len;
    std::vector<uint8_t> by;
    for (auto &p : hs) {
      hh.push_back(p.first);
      off.push_back((uint32_t)by.size());
      len.push_back((uint32_t)p.second.size());
      by.insert(by.end(), p.second.begin(), p.second.end());
    }
    e->n_dl = (uint32_t)hs.size();
    e->dl_hash.ensure(hh.size()); e->dl_off.ensure(off.size()); e->dl_len.ensure(len.size()); e->dl_bytes.ensure(by.size() + 16);
    if (!hs.empty()) {
      HIP_OK(hipMemcpy(e->dl_hash.p, hh.data(), hh.size() * 8, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(e->dl_off.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
      HIP_OK(hipMemcpy(e->dl_len.p, len.data(), len.size() * 4, hipMemcpyHostToDevice));
      if (!by.empty()) HIP_OK(hipMemcpy(e->dl_bytes.p, by.data(), by.size(), hipMemcpyHostToDevice));
    }
    return BJX_OK;
  });
}

extern "C" int bjx_batch_bans(bjx_engine *e, bjx_ban_batch *out) {
  if (!out) return BJX_ERR_ARG;
  return guarded(e, [&]() -> int {
    memset(out, 0, sizeof *out);
    if (!e->ban_emitted) throw BjxError(BJX_ERR_ARG, "bjx_batch_bans: the last batch ran without BJX_EMIT_BANS");
    out->n_ips = e->ban_ips.size();
    out->ips = out->n_ips ? e->ban_ips.data() : nullptr;
    out->n_trips = e->ban_n_trips;
    out->log_bytes = e->ban_n_trips ? e->ban_off.data()[e->ban_n_trips] : 0;
    out->log = out->log_bytes ? e->ban_log.data() : nullptr;
    out->log_off = e->ban_off.data();
    out->log_kind = e->ban_n_trips ? e->ban_kind.data() : nullptr;
    out->ip_bytes = e->ban_ipb.size() ? e->ban_ipb.data() : nullptr;
    out->ip_off = e->ban_ipo.data();
    return BJX_OK;
  });
}

extern "C" int bjx_state_get(bjx_engine *e, const char *ip, size_t ip_len, const char *name, size_t name_len,
                             int64_t *num_hits, int64_t *start_ns) {
  if (!e || (ip_len && !ip)) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    auto it = e->name_ids.find(std::string(name ? name : "", name_len));
    if (it == e->name_ids.end()) return 0;
    e->q_ip.ensure(ip_len + 1);
    e->q_out.ensure(4);
    if (ip_len) HIP_OK(hipMemcpyAsync(e->q_ip.p, ip, ip_len, hipMemcpyHostToDevice, e->stream));
    uint64_t h = hash_bytes(reinterpret_cast<const uint8_t *>(ip), (uint32_t)ip_len);
    if (e->dbg_hash_mask) h = (h & e->dbg_hash_mask) | 1;
    hipLaunchKernelGGL(k_state_get, dim3(1), dim3(1), 0, e->stream, e->S, h, e->q_ip.p, (uint32_t)ip_len, it->second, e->q_out.p);
    HIP_OK(hipGetLastError());
    int64_t o[3];
    HIP_OK(hipMemcpyAsync(o, e->q_out.p, 24, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    if (o[0] != 2) return 0;
    if (num_hits) *num_hits = o[1];
    if (start_ns) *start_ns = o[2];
    return 1;
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  }
}

extern "C" int64_t bjx_state_len(bjx_engine *e) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    read_counters(e);
    return (int64_t)e->host_counters[0];
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  }
}

extern "C" int bjx_state_stats_get(bjx_engine *e, bjx_state_stats *out) {
  if (!e || !out) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    read_counters(e);
    out->ips = e->host_counters[0];
    out->ip_slots = e->ip_cap;
    out->states = e->host_counters[2];
    out->state_slots = e->st_cap;
    out->arena_bytes = e->host_counters[1];
    out->arena_capacity = e->S.arena_cap;
    out->device_bytes = e->ip_cap * (sizeof(IpSlot) + 4 + 8 + 4) + e->st_cap * sizeof(StSlot) + e->S.arena_cap;
    out->rehashes = e->rehashes;
    return BJX_OK;
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  }
}

// live keys left in the state / IP tables (bjx_state_clear's check)
__global__ void k_count_live(const StSlot *__restrict__ st, uint64_t st_cap, const IpSlot *__restrict__ ip, uint64_t ip_cap,
                             unsigned long long *__restrict__ cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < st_cap && st[i].key != 0) atomicAdd(&cnt[0], 1ull);
  if (i < ip_cap && ip[i].hash != 0) atomicAdd(&cnt[1], 1ull);
}

extern "C" int bjx_state_clear(bjx_engine *e) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    HIP_OK(hipDeviceSynchronize());  // nothing of an earlier batch may land after the clear
    e->sort2_hold = 0;
    HIP_OK(hipMemsetAsync(e->S.ip, 0, e->ip_cap * sizeof(IpSlot), e->stream));
    HIP_OK(hipMemsetAsync(e->S.ip_first, 0xFF, e->ip_cap * 4, e->stream));
    HIP_OK(hipMemsetAsync(e->S.st, 0, e->st_cap * sizeof(StSlot), e->stream));
    HIP_OK(hipMemsetAsync(e->S.counters, 0, kCounterBytes, e->stream));
    HIP_OK(hipMemsetAsync(e->S.ip_st, 0xFF, e->S.ip_st_cap * 4, e->stream));
    HIP_OK(hipStreamSynchronize(e->stream));
    {
      // the tables must read back empty: IP ids restart at 0, so a state slot
      // that survived would be found again by a new IP's key
      e->chk.ensure(8);
      HIP_OK(hipMemsetAsync(e->chk.p, 0, 16, e->stream));
      const uint64_t n = std::max(e->st_cap, e->ip_cap);
      hipLaunchKernelGGL(k_count_live, dim3(grid_for(n)), dim3(kBlock), 0, e->stream, e->S.st, e->st_cap, e->S.ip, e->ip_cap,
                         e->chk.p);
      HIP_OK(hipGetLastError());
      unsigned long long live[2] = {0, 0};
      HIP_OK(hipMemcpyAsync(live, e->chk.p, 16, hipMemcpyDeviceToHost, e->stream));
      HIP_OK(hipStreamSynchronize(e->stream));
      if (live[0] | live[1]) {
        fprintf(stderr, "[bjx] state_clear: %llu state slots and %llu IP slots survived the clear; clearing again\n", live[0],
                live[1]);
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemset(e->S.st, 0, e->st_cap * sizeof(StSlot)));
        HIP_OK(hipMemset(e->S.ip, 0, e->ip_cap * sizeof(IpSlot)));
        HIP_OK(hipDeviceSynchronize());
      }
    }
    return BJX_OK;
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return x.code;
  }
}

extern "C" size_t bjx_state_dump(bjx_engine *e, char *out, size_t cap) {
  if (!e) return 0;
  std::lock_guard<std::mutex> g(e->mu);
  try {
    HIP_OK(hipSetDevice(e->device));
    read_counters(e);
    const uint64_t n_ips = e->host_counters[0], used = e->host_counters[1];
    std::vector<uint64_t> off(n_ips);
    std::vector<uint32_t> len(n_ips);
    std::vector<StSlot> st(e->st_cap);
    std::vector<uint8_t> arena(used);
    HIP_OK(hipMemcpy(off.data(), e->S.ip_off, n_ips * 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(len.data(), e->S.ip_len, n_ips * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(arena.data(), e->S.arena, used, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(st.data(), e->S.st, e->st_cap * sizeof(StSlot), hipMemcpyDeviceToHost));
    std::vector<std::vector<std::pair<uint32_t, uint64_t>>> per_ip(n_ips);
    for (uint64_t i = 0; i < e->st_cap; ++i)
      if (st[i].key && st[i].valid) per_ip[(st[i].key >> 24) - 1].push_back({(uint32_t)(st[i].key & 0xFFFFFF), i});
    std::string s;
    char buf[96];
    for (uint64_t id = 0; id < n_ips; ++id) {
      s.append(reinterpret_cast<const char *>(arena.data() + off[id]), len[id]);
      s += ":\n";
      std::sort(per_ip[id].begin(), per_ip[id].end(),
                [&](const std::pair<uint32_t, uint64_t> &a, const std::pair<uint32_t, uint64_t> &b) {
                  return e->names[a.first] < e->names[b.first];
                });
      for (auto &p : per_ip[id]) {
        s += "\t" + e->names[p.first] + ":\n";
        snprintf(buf, sizeof buf, "\t\t{%lld %lld}\n", (long long)st[p.second].hits, (long long)st[p.second].start);
        s += buf;
      }
      s += "\n";
    }
    if (out && cap) memcpy(out, s.data(), std::min(cap, s.size()));
    return s.size();
  } catch (const BjxError &x) {
    e->last_error = x.what();
    return 0;
  }
}

// ------------------------------------------------------------ self-test hooks
#include "../../include/banjax_gpu_debug.h"

extern "C" int bjx_debug_rule_match_host(const bjx_ruleset *rs, size_t i, const uint8_t *text, size_t n) {
  if (!rs || i >= rs->rules.size() || (n && !text)) return BJX_ERR_ARG;
  return dfa_match_host(rs->rules[i].rx, text, n) ? 1 : 0;
}
extern "C" int bjx_debug_set_dfa_state_cap(uint32_t cap) {
  set_dfa_state_cap(cap);
  std::lock_guard<std::mutex> g(g_rx_mu);
  g_rx_cache.clear();  // compiled patterns depend on the cap
  return BJX_OK;
}
extern "C" int bjx_debug_force_wide_nfa(int on) {
  set_force_wide_nfa(on != 0);
  std::lock_guard<std::mutex> g(g_rx_mu);
  g_rx_cache.clear();  // compiled patterns depend on it
  return BJX_OK;
}
extern "C" int bjx_debug_set_ip_hash_mask(bjx_engine *e, uint64_t mask) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  e->dbg_hash_mask = mask;
  return BJX_OK;
}
extern "C" int bjx_debug_set_claim_budget(bjx_engine *e, uint64_t max_new) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  e->dbg_budget = max_new;
  return BJX_OK;
}
extern "C" int bjx_debug_set_slot_cache(bjx_engine *e, int on) {
  if (!e) return BJX_ERR_ARG;
  std::lock_guard<std::mutex> g(e->mu);
  e->dbg_slot_cache = on < 0 ? -1 : on != 0;
  e->bound_uid = 0;  // the next batch re-binds and applies it
  return BJX_OK;
}
extern "C" size_t bjx_debug_phase_ms(bjx_engine *e, double *out, size_t cap) {
  if (!e) return 0;
  for (size_t k = 0; k < cap && k < (size_t)bjx_engine::kPhases; ++k) out[k] = e->phase_ms[k];
  if (cap > (size_t)bjx_engine::kPhases) out[bjx_engine::kPhases] = e->exchange_ms;
  return bjx_engine::kPhases + 1;
}
extern "C" size_t bjx_debug_kernel_ms(bjx_engine *e, double *out, size_t cap) {
  if (!e) return 0;
  // [3]: which per-line kernel ran (2 = k_lines2, 1 = k_lines), [4]: its line window / staging bytes
  const double v[5] = {e->kernel_ms[0], e->kernel_ms[1], e->kernel_ms[2], (double)e->last_line_kernel,
                       e->last_line_kernel == 2 ? (double)kL2Win : e->last_line_kernel == 1 ? (double)kSpanBytes : 0.0};
  for (size_t k = 0; k < cap && k < 5; ++k) out[k] = v[k];
  return 5;
}
extern "C" size_t bjx_debug_scan_stats(bjx_engine *e, uint64_t *out, size_t cap) {
  if (!e) return 0;
  std::lock_guard<std::mutex> g(e->mu);
  if (e->S.counters) read_counters(e);
  const uint64_t v[12] = {e->scan_stats[0], e->scan_stats[1], e->scan_stats[2], e->scan_stats[3], e->scan_stats[4],
                          e->ip_cap, e->host_counters[0], e->st_cap, e->host_counters[2], e->scan_stats[5],
                          e->last_grouping, e->last_long_runs};
  for (size_t k = 0; k < 12 && k < cap; ++k) out[k] = v[k];
  return 12;
}
extern "C" int bjx_debug_rule_lead(const bjx_ruleset *rs, size_t i) {
  if (!rs || i >= rs->rules.size()) return BJX_ERR_ARG;
  const auto &rx = rs->rules[i].rx;
  return rx.mode == kModePrefilter && rx.pref_lead ? (int)rx.lead_dist : -1;
}

extern "C" size_t bjx_debug_rule_literal(const bjx_ruleset *rs, size_t i, char *out, size_t cap) {
  if (!rs || i >= rs->rules.size()) return 0;
  // "<mode> <equiv>" then per literal "\n<gram_off> <ci mask as 0/1> <bytes>"
  const CompiledRegex &rx = rs->rules[i].rx;
  std::string l = std::to_string((int)rx.mode) + " " + std::to_string((int)rx.pref_equivalent);
  for (const PrefLit &pl : rx.pref) {
    l += "\n" + std::to_string(pl.gram_off) + " ";
    for (char c : pl.ci) l += c ? '1' : '0';
    l += " " + pl.s;
  }
  for (const PrefLit &pl : rx.anchor) {
    l += std::string("\n^") + (rx.anchor_equivalent ? "=" : "~") + " ";
    for (char c : pl.ci) l += c ? '1' : '0';
    l += " " + pl.s;
  }
  if (out && cap) memcpy(out, l.data(), std::min(cap, l.size()));
  return l.size();
}
