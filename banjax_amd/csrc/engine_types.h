// Device-side data layout of the MI355X engine (see DESIGN.md "Data layout").
#pragma once
#include <stdint.h>

namespace bjx {

// One compiled rule as the kernels see it (rule tables live in one blob).
struct DevRule {
  uint32_t trans_off;   // u16 index into trans[]: row s starts at trans_off + s * ncls
  uint32_t ae_off;      // u8 index into accept_end[]
  uint32_t na_off;      // index into nonascii[] (pairs: lo, class)
  uint16_t n_na;
  uint16_t ncls;
  uint16_t start;
  uint16_t flags;       // kRuleAlways / kRuleNever
  uint32_t name_id;     // engine-wide interned rule name (state key, rate_limit.go:54)
  int32_t decision;
  uint32_t lits_off;     // prefilter literal ids: rule_lits[lits_off .. + lits_len)
  uint16_t lits_len;
  uint8_t mode;          // RuleMode
  uint8_t equiv;         // match <=> one of its literals occurs in rest
  int64_t interval_ns;
  int64_t hits;
};

// Prefilter gram bitset: one bit per hash of a 4-byte window (LDS resident).
constexpr uint32_t kGramLog2 = 18;
constexpr uint32_t kGramWords = (1u << kGramLog2) / 32;
__host__ __device__ inline uint32_t gram_hash(uint32_t g) { return (g * 0x9E3779B1u) >> (32 - kGramLog2); }
constexpr int kCandSlots = 4;

struct Subnet {
  uint8_t net[16];
  uint8_t mask[16];
  uint32_t netlen;  // 4 (IPv4 compare, To4 semantics) or 16
  uint32_t _pad;
};

// Everything the per-line kernels need about the current (ruleset, decision
// lists) pair.  All pointers are device pointers into one blob.
struct Bind {
  const DevRule *rules;
  const uint16_t *trans;
  const uint8_t *accept_end;
  const uint8_t *ascii_cls;    // 128 per rule
  const uint32_t *nonascii;    // (lo, class) pairs
  const uint8_t *lits;
  const uint32_t *global_rules;
  const uint32_t *site_off;    // n_hosts + 1
  const uint32_t *site_rules;
  const uint64_t *hd_hash;     // host dictionary sorted by hash
  const uint32_t *hd_id;
  const uint32_t *hd_off;
  const uint32_t *hd_len;
  const uint8_t *hd_bytes;
  const int32_t *host_scope;   // host id -> allow scope (or -1)
  const uint64_t *skip_keys;   // sorted (rule << 32 | host id)
  const uint32_t *sc_addr_off; // scopes + 1
  const uint64_t *sc_addr;     // 2 words per address, sorted per scope
  const uint32_t *sc_sub_off;
  const Subnet *sc_sub;
  const uint32_t *sc_str_off;
  const uint64_t *sc_str_hash; // sorted per scope
  const uint32_t *sc_str_boff;
  const uint32_t *sc_str_len;
  const uint8_t *sc_str_bytes;
  uint32_t n_rules;
  uint32_t n_global;
  uint32_t n_hosts;
  uint32_t n_hd;
  uint32_t n_skip;
  uint32_t n_scopes;
  uint32_t any_allow;
  uint32_t mask_words;         // ceil(max applicable rules per line / 64)
  // prefilter
  const uint32_t *gram_bits;   // kGramWords
  const uint32_t *gt_key;      // open-addressing gram table (gt_mask + 1 slots)
  const uint32_t *gt_off;      // entries offset (pairs lit, gram offset)
  const uint32_t *gt_len;      // 0 = empty slot
  const uint32_t *gt_entries;
  const uint8_t *lit_bytes;
  const uint8_t *lit_ci;
  const uint32_t *lit_off;
  const uint32_t *lit_len;
  const uint32_t *rule_lits;
  uint32_t gt_mask;
  uint32_t n_lits;
  uint32_t any_anchored;
  uint32_t any_prefilter;
};

// Per-line SoA arrays (batch workspace).
struct Lines {
  int64_t *ts;
  uint64_t *ip_hash;
  uint32_t *ip_off, *ip_len, *host_off, *host_len, *rest_off;
  int32_t *host_id;
  uint8_t *flags;
  uint64_t *counts;    // (n_results << 32) | n_events per line, then scanned in place
  uint64_t *masks;     // mask_words per line
  uint64_t *amask;     // anchored rules decided in the scan pass (positions < 64)
  uint64_t *ares;      // anchored rules left unresolved by the scan pass
  uint32_t *cand_cnt;  // prefilter candidates per line
  uint64_t *cand;      // kCandSlots per line: (start position << 24) | literal id
};

// Persistent rate-limit state (RegexRateLimitStates, rate_limit.go:17-21),
// keyed by IP string and rule name, never evicted (as in the reference).
struct State {
  uint64_t *ip_slot_hash;  // 0 = empty
  uint32_t *ip_slot_id;
  uint64_t *ip_off;        // id -> arena offset
  uint32_t *ip_len;
  uint8_t *arena;
  uint64_t *st_key;        // 0 = empty; key = ((ip_id + 1) << 24) | name_id
  int64_t *st_hits;
  int64_t *st_start;
  uint64_t *counters;      // [0] ips, [1] arena bytes, [2] states
  uint64_t ip_mask;
  uint64_t st_mask;
  uint64_t arena_cap;
};

enum LineFlagBits : uint8_t {
  kLineError = 1, kLineOld = 2, kLineExempt = 4,
  kLineSlowTs = 0x40,     // per-line fallback kernel (timestamp / long header)
  kLineExemptPending = 0x20,
  kLineAnchoredHigh = 0x10, // anchored rules at positions >= 64: resolve in k_resolve
};

}  // namespace bjx
