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
  // Longest literal every match must contain (byte string, case-sensitive), or
  // empty; used by the device prefilter.  Only set when the literal is pure ASCII.
  std::string required_literal;
  bool literal_equivalent = false;  // match <=> text contains required_literal
};

// Returns 0 on success; otherwise a negative bjx_status with *err set to the
// Go-style message ("error parsing regexp: <code>: `<expr>`").
int compile_regex(const std::string &pattern, CompiledRegex *out, std::string *err,
                  uint32_t max_dfa_states = 40000);

// Host reference evaluation of compiled tables (compiler self-test only; the
// product matches on the GPU).
bool dfa_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n);

}  // namespace bjx
