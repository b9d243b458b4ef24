// Rule compiler: Go regexp (RE2 syntax, syntax.Perl flags) -> per-rule DFA over
// rune classes, for boolean unanchored matching exactly as Go's
// (*Regexp).Match does (reference internal/regex_rate_limiter.go:234; rules
// compiled at config load, internal/config.go:110).
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#if defined(__HIPCC__)
#define BJX_RX_HD __host__ __device__
#else
#define BJX_RX_HD
#endif

namespace bjx {

// DFA state ids: 0 = DEAD (can never match), 1 = ACCEPT (matched; absorbing).
constexpr uint16_t kDead = 0;
constexpr uint16_t kAccept = 1;

enum RuleFlags : uint32_t {
  kRuleAlways = 1,  // matches every input (e.g. ".*", "^"): no scan needed
  kRuleNever = 2,   // matches nothing
  kRuleNfa = 4,     // matched by the bit-parallel NFA (CompiledRegex::nfa), not a DFA
  kRuleNfaWide = 8, // with kRuleNfa: the block-cooperative NFA (no position limit; layout NfaWideLayout)
};

// DFA states before a rule switches to the bit-parallel NFA; NFA limits
constexpr uint32_t kDfaStateCap = 4096;
constexpr uint32_t kNfaMaxPos = 1024;             // positions (16 x 64-bit words per state set)
constexpr size_t kNfaMaxBlobBytes = 48 * 1024;    // tables staged in LDS per block

// Word offsets of the bit-parallel NFA tables in CompiledRegex::nfa (see
// regex_compiler.cpp "bit-parallel NFA"); the header is the first 4 words.
struct NfaLayout {
  uint32_t W, npos, ncls, ngroups, nassert, match, flags, total;
  uint32_t o_ascii, o_cat, o_s0, o_sh, o_cm, o_gm, o_gt, o_apos, o_at;
};
enum NfaFlags : uint32_t { kNfaAsserts = 1, kNfaAnchored = 2 };
BJX_RX_HD inline NfaLayout nfa_layout(uint32_t W, uint32_t npos, uint32_t ncls, uint32_t ng, uint32_t na) {
  NfaLayout L{};
  L.W = W; L.npos = npos; L.ncls = ncls; L.ngroups = ng; L.nassert = na;
  L.o_ascii = 4;
  L.o_cat = L.o_ascii + 32;
  L.o_s0 = L.o_cat + (ncls + 7) / 8;
  L.o_sh = L.o_s0 + W;
  L.o_cm = L.o_sh + W;
  L.o_gm = L.o_cm + ncls * W;
  L.o_gt = L.o_gm + ng * W;
  L.o_apos = L.o_gt + ng * W;
  L.o_at = L.o_apos + (na + 1) / 2;
  L.total = L.o_at + na * 16 * W;
  return L;
}
// layout of a blob from its header words (h = the blob's first 8 u32)
BJX_RX_HD inline NfaLayout nfa_layout_of(const uint32_t *h) {
  NfaLayout L = nfa_layout(h[0], h[1], h[2], h[3], h[4]);
  L.match = h[5];
  L.flags = h[6];
  return L;
}

// The wide NFA (kRuleNfaWide): the same position automaton as the
// bit-parallel NFA, for rules past kNfaMaxPos positions (e.g. `.*x.{600}y`).
// A whole block steps one text: shift edges bit-parallel over the W-word
// state (each thread owns a run of words), the other follow edges as sparse
// target lists of the position groups, assertion closures as sparse target
// lists per (assert position, context).  Limit: Go's own program size
// (regexp/syntax maxSize, 128 MB / 40 B per instruction = 3355443).
constexpr uint32_t kNfaWideMaxPos = 3355443;
struct NfaWideLayout {
  uint32_t W, npos, ncls, ngroups, nassert, match, flags, n_gtgt, n_atgt;
  uint64_t o_ascii, o_cat, o_s0, o_sh, o_gall, o_am, o_cm, o_aux, o_goff, o_gtgt, o_aoff, o_atgt, total;
};
BJX_RX_HD inline NfaWideLayout nfa_wide_layout(uint32_t W, uint32_t npos, uint32_t ncls, uint32_t ng, uint32_t na,
                                               uint32_t n_gtgt, uint32_t n_atgt) {
  NfaWideLayout L{};
  L.W = W; L.npos = npos; L.ncls = ncls; L.ngroups = ng; L.nassert = na; L.n_gtgt = n_gtgt; L.n_atgt = n_atgt;
  L.o_ascii = 8;                                   // header: 16 u32
  L.o_cat = L.o_ascii + 32;                        // u16[128] ascii classes
  L.o_s0 = L.o_cat + (ncls + 7) / 8;               // u8[ncls] class categories
  L.o_sh = L.o_s0 + W;
  L.o_gall = L.o_sh + W;                           // positions with a group
  L.o_am = L.o_gall + W;                           // assert positions
  L.o_cm = L.o_am + W;                             // [ncls][W]
  L.o_aux = L.o_cm + (uint64_t)ncls * W;           // u32[npos]: group id (CHAR) / assert index (ASSERT)
  L.o_goff = L.o_aux + (npos + 1) / 2;             // u32[ng + 1]
  L.o_gtgt = L.o_goff + (ng + 2) / 2;              // u32[n_gtgt]
  L.o_aoff = L.o_gtgt + (n_gtgt + 1) / 2;          // u32[na * 16 + 1]
  L.o_atgt = L.o_aoff + (na * 16 + 2) / 2;         // u32[n_atgt]
  L.total = L.o_atgt + (n_atgt + 1) / 2;
  return L;
}
BJX_RX_HD inline NfaWideLayout nfa_wide_layout_of(const uint32_t *h) {
  NfaWideLayout L = nfa_wide_layout(h[0], h[1], h[2], h[3], h[4], h[8], h[9]);
  L.match = h[5];
  L.flags = h[6];
  return L;
}

// rules compiled after this call switch to the bit-parallel NFA past `cap` DFA
// states (test hook: 1 sends every rule that fits the NFA limits to it)
void set_dfa_state_cap(uint32_t cap);
uint32_t dfa_state_cap();
// test hook: rules compiled after this call go straight to the wide NFA
void set_force_wide_nfa(bool on);

// How the device decides a rule on a line.
enum RuleMode : uint8_t {
  kModeAlways = 0,     // matches every text
  kModeNever = 1,      // matches nothing
  kModeAnchored = 2,   // every match starts at rest[0]: DFA from the start, dies early
  kModePrefilter = 3,  // every match contains one of `pref` literals: candidates from the
                       // byte-parallel gram filter, then literal check (+ DFA unless equivalent)
  kModeScan = 4,       // no usable literal: full DFA scan of rest
};

// A prefilter literal: ASCII bytes; ci[i] = 1 if byte i matches ASCII-case-insensitively
// (only letters whose Go simple-fold orbit is ASCII-only, i.e. not k or s).
struct PrefLit {
  std::string s;
  std::string ci;
  uint32_t gram_off = 0;  // start of the 4-byte window probed by the gram filter
};

struct CompiledRegex {
  uint32_t nstates = 0;  // including DEAD and ACCEPT
  uint32_t ncls = 0;     // rune classes
  uint16_t start = 0;
  uint32_t flags = 0;
  std::vector<uint16_t> trans;      // nstates * ncls, row-major by state
  std::vector<uint8_t> accept_end;  // nstates: matched if the text ends in this state
  uint8_t ascii_cls[128] = {};      // rune < 0x80 -> class
  // rune >= 0x80: sorted (lo, class) interval starts covering [0x80, 0x10FFFF]
  std::vector<std::pair<uint32_t, uint32_t>> nonascii;
  RuleMode mode = kModeScan;
  // every match contains at least one of these (kModePrefilter); each >= 4 bytes
  std::vector<PrefLit> pref;
  bool pref_equivalent = false;  // match <=> text contains one of `pref`
  // every match begins with one of `pref` (the pattern is (.*)* X ... with X's
  // leading assertion-free exact strings = pref): a DFA job may start at the
  // first occurrence of a pref literal instead of rest[0]
  bool pref_lead = false;
  // with pref_lead: every match starts at most lead_dist bytes before the
  // literal it begins with (a pure, bounded piece first, e.g. (?i)s in
  // (?i)scrapy): the job starts lead_dist bytes (and a rune) before the hit
  uint8_t lead_dist = 0;
  // kModeAnchored: every match starts with one of these (exact, ASCII-ci as above)
  std::vector<PrefLit> anchor;
  bool anchor_equivalent = false;  // match <=> text starts with one of `anchor`
  std::string required_literal;  // diagnostics: the first prefilter literal
  // kRuleNfa: bit-parallel NFA tables (layout: regex_compiler.cpp "bit-parallel
  // NFA"); nstates = positions, trans / accept_end empty
  std::vector<uint64_t> nfa;
  uint32_t nfa_words = 0;
};

// Returns 0 on success; otherwise a negative bjx_status with *err set to the
// Go-style message ("error parsing regexp: <code>: `<expr>`").
int parse_regex_only(const std::string &pattern, std::string *err);
int compile_regex(const std::string &pattern, CompiledRegex *out, std::string *err,
                  uint32_t max_dfa_states = 40000);

// Host reference evaluation of compiled tables, DFA or bit-parallel NFA
// (compiler self-test only; the product matches on the GPU).
bool dfa_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n);

}  // namespace bjx
