// Rule compiler: Go regexp (RE2 syntax, syntax.Perl flags) -> per-rule DFA over
// rune classes, for boolean unanchored matching exactly as Go's
// (*Regexp).Match does (reference internal/regex_rate_limiter.go:234; rules
// compiled at config load, internal/config.go:110).
#pragma once
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace bjx {

// DFA state ids: 0 = DEAD (can never match), 1 = ACCEPT (matched; absorbing).
constexpr uint16_t kDead = 0;
constexpr uint16_t kAccept = 1;

enum RuleFlags : uint32_t {
  kRuleAlways = 1,  // matches every input (e.g. ".*", "^"): no scan needed
  kRuleNever = 2,   // matches nothing
};

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
  // kModeAnchored: every match starts with one of these (exact, ASCII-ci as above)
  std::vector<PrefLit> anchor;
  bool anchor_equivalent = false;  // match <=> text starts with one of `anchor`
  std::string required_literal;  // diagnostics: the first prefilter literal
};

// Returns 0 on success; otherwise a negative bjx_status with *err set to the
// Go-style message ("error parsing regexp: <code>: `<expr>`").
int compile_regex(const std::string &pattern, CompiledRegex *out, std::string *err,
                  uint32_t max_dfa_states = 40000);

// Host reference evaluation of compiled tables (compiler self-test only; the
// product matches on the GPU).
bool dfa_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n);

}  // namespace bjx
