// Rule compiler for the MI355X engine: Go regexp syntax -> rune-class DFA.
//
// Parsing follows Go 1.25 regexp/syntax (parse.go, published algorithm) with
// the flags regexp.Compile uses (syntax.Perl = ClassNL|OneLine|PerlX|
// UnicodeGroups), so that the set of accepted patterns, their meaning and the
// error texts match the reference's config load (internal/config.go:110-113).
// Matching semantics are those of (*Regexp).Match on []byte (reference
// internal/regex_rate_limiter.go:234): unanchored, boolean, over runes decoded
// with Go's utf8.DecodeRune (an invalid byte is U+FFFD of width 1), with
// empty-width assertions evaluated by syntax.EmptyOpContext.
//
// The automaton built here is a DFA over *rune classes* (a per-rule partition
// of [0, 0x10FFFF]); \b, \B, ^ and $ are handled by carrying the category of
// the previous rune (word / newline / start-of-text) in the DFA state, and the
// unanchored search by re-seeding the NFA start at every rune boundary.
// Accepting is absorbing (boolean match), so the device loop stops at the
// first ACCEPT or DEAD state.
#include "regex_compiler.h"
#include "go_limits.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <strings.h>
#include <map>
#include <memory>
#include <unordered_map>

#include "../../include/banjax_gpu.h"
#include "../../third_party/unicode/fold_orbits.h"
#include "../../third_party/unicode/unicode_tables.h"

namespace bjx {
namespace {

constexpr int32_t kMaxRune = 0x10FFFF;
constexpr int32_t kRuneError = 0xFFFD;

// ---------------------------------------------------------------- runes

int32_t decode_rune(const uint8_t *s, size_t n, int *width) {
  if (n == 0) { *width = 0; return -1; }
  uint8_t b0 = s[0];
  if (b0 < 0x80) { *width = 1; return b0; }
  int need; uint8_t lo = 0x80, hi = 0xBF; int32_t r;
  if (b0 >= 0xC2 && b0 <= 0xDF) { need = 1; r = b0 & 0x1F; }
  else if (b0 == 0xE0) { need = 2; lo = 0xA0; r = b0 & 0x0F; }
  else if ((b0 >= 0xE1 && b0 <= 0xEC) || b0 == 0xEE || b0 == 0xEF) { need = 2; r = b0 & 0x0F; }
  else if (b0 == 0xED) { need = 2; hi = 0x9F; r = b0 & 0x0F; }
  else if (b0 == 0xF0) { need = 3; lo = 0x90; r = b0 & 0x07; }
  else if (b0 >= 0xF1 && b0 <= 0xF3) { need = 3; r = b0 & 0x07; }
  else if (b0 == 0xF4) { need = 3; hi = 0x8F; r = b0 & 0x07; }
  else { *width = 1; return kRuneError; }
  if (n < static_cast<size_t>(need) + 1 || s[1] < lo || s[1] > hi) { *width = 1; return kRuneError; }
  r = (r << 6) | (s[1] & 0x3F);
  for (int k = 2; k <= need; ++k) {
    if (s[k] < 0x80 || s[k] > 0xBF) { *width = 1; return kRuneError; }
    r = (r << 6) | (s[k] & 0x3F);
  }
  *width = need + 1;
  return r;
}

int32_t simple_fold(int32_t r) {
  const uint32_t *b = bjx_fold_from, *e = bjx_fold_from + BJX_FOLD_N;
  const uint32_t *it = std::lower_bound(b, e, static_cast<uint32_t>(r));
  if (it != e && *it == static_cast<uint32_t>(r)) return static_cast<int32_t>(bjx_fold_to[it - b]);
  return r;
}

bool is_word_rune(int32_t r) {
  return r >= 0 && r < 0x80 && ((r >= '0' && r <= '9') || (r >= 'A' && r <= 'Z') || (r >= 'a' && r <= 'z') || r == '_');
}
bool is_alnum(int c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

using Ranges = std::vector<std::pair<int32_t, int32_t>>;

void clean(Ranges &r) {
  std::sort(r.begin(), r.end());
  Ranges o;
  for (auto &p : r) {
    if (!o.empty() && p.first <= o.back().second + 1) o.back().second = std::max(o.back().second, p.second);
    else o.push_back(p);
  }
  r.swap(o);
}
void negate(Ranges &r) {  // r clean
  Ranges o;
  int32_t next = 0;
  for (auto &p : r) {
    if (p.first > next) o.push_back({next, p.first - 1});
    next = p.second + 1;
  }
  if (next <= kMaxRune) o.push_back({next, kMaxRune});
  r.swap(o);
}
void add_folded(Ranges &r, int32_t lo, int32_t hi) {
  const int32_t min_fold = 0x41, max_fold = static_cast<int32_t>(bjx_fold_from[BJX_FOLD_N - 1]);
  if ((lo <= min_fold && hi >= max_fold) || hi < min_fold || lo > max_fold) { r.push_back({lo, hi}); return; }
  if (lo < min_fold) { r.push_back({lo, min_fold - 1}); lo = min_fold; }
  if (hi > max_fold) { r.push_back({max_fold + 1, hi}); hi = max_fold; }
  for (int32_t c = lo; c <= hi; ++c) {
    r.push_back({c, c});
    for (int32_t f = simple_fold(c); f != c; f = simple_fold(f)) r.push_back({f, f});
  }
}

// ------------------------------------------------ Unicode groups (\p{..})
//
// regexp/syntax unicodeTable (Go 1.25): "Any", the general categories of
// package unicode (incl. LC and Cn), its scripts, "Assigned" (= not Cn) and
// "ASCII", then the same names and unicode.CategoryAliases matched loosely
// (canonicalName: case-insensitive, ignoring '_', '-' and ' ').  Tables:
// third_party/unicode/unicode_tables.h (Unicode 15.0.0).

std::string canonical_name(const std::string &n) {
  std::string b;
  bool first = true;
  for (char c : n) {
    if (c == '_' || c == '-' || c == ' ') continue;
    if (first) {
      if (c >= 'a' && c <= 'z') c = static_cast<char>(c - 'a' + 'A');
      first = false;
    } else if (c >= 'A' && c <= 'Z') {
      c = static_cast<char>(c - 'A' + 'a');
    }
    b.push_back(c);
  }
  return b;
}

void table_ranges(const bjx_uni_table &t, Ranges *out) {
  for (uint32_t i = 0; i < t.n; ++i)
    out->push_back({static_cast<int32_t>(bjx_uni_ranges[2 * (t.off + i)]), static_cast<int32_t>(bjx_uni_ranges[2 * (t.off + i) + 1])});
}

const bjx_uni_table *find_table(const std::string &name, bool loose) {
  const std::string c = loose ? canonical_name(name) : name;
  for (size_t i = 0; i < BJX_UNI_NTABLES; ++i)
    if ((loose ? canonical_name(bjx_uni_tables[i].name) : std::string(bjx_uni_tables[i].name)) == c) return &bjx_uni_tables[i];
  return nullptr;
}

// true if name is known: *out = its runes, *sign = -1 when they are to be inverted
bool unicode_table(const std::string &name, Ranges *out, int *sign) {
  *sign = 1;
  out->clear();
  if (name == "Any") { out->push_back({0, kMaxRune}); return true; }
  if (const bjx_uni_table *t = find_table(name, false)) { table_ranges(*t, out); return true; }
  const std::string c = canonical_name(name);
  if (c == "Any") { out->push_back({0, kMaxRune}); return true; }
  if (c == "Assigned") { table_ranges(*find_table("Cn", false), out); *sign = -1; return true; }
  if (c == "Ascii") { out->push_back({0, 0x7F}); return true; }
  if (const bjx_uni_table *t = find_table(name, true)) { table_ranges(*t, out); return true; }
  for (size_t i = 0; i < BJX_UNI_NALIASES; ++i)
    if (canonical_name(bjx_uni_cat_aliases[2 * i]) == c) {
      table_ranges(*find_table(bjx_uni_cat_aliases[2 * i + 1], false), out);
      return true;
    }
  return false;
}

// ------------------------------------------------------------------ AST

enum Op : uint8_t {
  kNoMatch = 1, kEmpty, kLit, kClass, kAnyNotNL, kAnyChar, kBOL, kEOL, kBOT, kEOT, kWB, kNWB,
  kCap, kStar, kPlus, kQuest, kRepeat, kConcat, kAlt,
  kPseudo = 100, kLParen, kVBar
};
enum Flag : uint32_t { kFold = 1, kClassNL = 2, kDotNL = 4, kOneLine = 8, kNonGreedy = 16, kPerlX = 32 };

struct Re {
  Op op;
  uint32_t flags;
  int min = 0, max = 0, cap = 0;
  int32_t rune = 0;
  Ranges cls;
  std::vector<std::unique_ptr<Re>> sub;
  Re(Op o, uint32_t f) : op(o), flags(f) {}
};
using ReP = std::unique_ptr<Re>;

struct ParseError {
  std::string code, expr;
};

const char *kErrInvalidCharRange = "invalid character class range";
const char *kErrInvalidEscape = "invalid escape sequence";
const char *kErrInvalidNamedCapture = "invalid named capture";
const char *kErrInvalidPerlOp = "invalid or unsupported Perl syntax";
const char *kErrInvalidRepeatOp = "invalid nested repetition operator";
const char *kErrInvalidRepeatSize = "invalid repeat count";
const char *kErrInvalidUTF8 = "invalid UTF-8";
const char *kErrMissingBracket = "missing closing ]";
const char *kErrMissingParen = "missing closing )";
const char *kErrMissingRepeatArg = "missing argument to repetition operator";
const char *kErrTrailingBackslash = "trailing backslash at end of expression";
const char *kErrUnexpectedParen = "unexpected )";
const char *kErrNestingDepth = "expression nests too deeply";
const char *kErrLarge = "expression too large";

struct Group { const char *name; int sign; std::vector<int32_t> r; };
const std::vector<Group> &perl_groups() {
  static const std::vector<Group> g = {
    {"\\d", 1, {'0', '9'}}, {"\\D", -1, {'0', '9'}},
    {"\\s", 1, {'\t', '\n', '\f', '\r', ' ', ' '}}, {"\\S", -1, {'\t', '\n', '\f', '\r', ' ', ' '}},
    {"\\w", 1, {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}}, {"\\W", -1, {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}},
  };
  return g;
}
const std::vector<Group> &posix_groups() {
  // built once (thread-safe static init: rulesets compile on worker threads)
  static const std::vector<std::string> names = [] {
    std::vector<std::string> v;
    for (const char *n : {"alnum", "alpha", "ascii", "blank", "cntrl", "digit", "graph", "lower", "print", "punct",
                          "space", "upper", "word", "xdigit"}) {
      v.push_back(std::string("[:") + n + ":]");
      v.push_back(std::string("[:^") + n + ":]");
    }
    return v;
  }();
  static const std::vector<Group> g = [] {
    const std::vector<std::vector<int32_t>> base = {
      {'0', '9', 'A', 'Z', 'a', 'z'}, {'A', 'Z', 'a', 'z'}, {0, 0x7F}, {'\t', '\t', ' ', ' '}, {0, 0x1F, 0x7F, 0x7F},
      {'0', '9'}, {'!', '~'}, {'a', 'z'}, {' ', '~'}, {'!', '/', ':', '@', '[', '`', '{', '~'}, {'\t', '\r', ' ', ' '},
      {'A', 'Z'}, {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'}, {'0', '9', 'A', 'F', 'a', 'f'},
    };
    std::vector<Group> out;
    for (size_t i = 0; i < base.size(); ++i) {
      out.push_back({names[2 * i].c_str(), 1, base[i]});
      out.push_back({names[2 * i + 1].c_str(), -1, base[i]});
    }
    return out;
  }();
  return g;
}

struct SimpleFold {
  int32_t operator()(int32_t r) const { return simple_fold(r); }
};

class Parser {
 public:
  Parser(const std::string &s) : whole_(s), gs_(SimpleFold()) {}

  // Go's size and nesting limits are checked on the way (go_limits.h), at the
  // point of the parse where regexp/syntax would stop
  ReP parse() {
    try {
      return parse_all();
    } catch (const gosh::Limit &l) {
      throw ParseError{l.large ? kErrLarge : kErrNestingDepth, whole_};
    }
  }

 private:
  // Go's parse flags of the current position (FoldCase, NonGreedy)
  uint32_t gf() const { return ((flags_ & kFold) ? gosh::fFold : 0u) | ((flags_ & kNonGreedy) ? gosh::fNonGreedy : 0u); }

  ReP parse_all() {
    const char *t = whole_.data(), *end = whole_.data() + whole_.size();
    const char *last_repeat = nullptr;
    while (t < end) {
      const char *repeat = nullptr;
      switch (*t) {
        case '(':
          if ((flags_ & kPerlX) && end - t >= 2 && t[1] == '?') { t = perl_flags(t, end); break; }
          ++ncap_;
          push_paren(ncap_);
          ++t;
          break;
        case '|':
          gs_.vertical_bar(gf());
          concat();
          if (!swap_vbar()) push(std::make_unique<Re>(kVBar, flags_));
          ++t;
          break;
        case ')': {
          gs_.right_paren(gf());
          concat();
          if (swap_vbar()) stack_.pop_back();
          alternate();
          size_t n = stack_.size();
          if (n < 2) throw ParseError{kErrUnexpectedParen, whole_};
          ReP re1 = std::move(stack_[n - 1]);
          ReP re2 = std::move(stack_[n - 2]);
          stack_.resize(n - 2);
          if (re2->op != kLParen) throw ParseError{kErrUnexpectedParen, whole_};
          flags_ = re2->flags;
          if (re2->cap == 0) push(std::move(re1));
          else { auto c = std::make_unique<Re>(kCap, re1->flags); c->cap = re2->cap; c->sub.push_back(std::move(re1)); push(std::move(c)); }
          ++t;
          break;
        }
        case '^':
          gs_.op((flags_ & kOneLine) ? gosh::gBeginText : gosh::gBeginLine, gf());
          push(std::make_unique<Re>((flags_ & kOneLine) ? kBOT : kBOL, flags_)); ++t; break;
        case '$':
          gs_.op((flags_ & kOneLine) ? gosh::gEndText : gosh::gEndLine, gf() | ((flags_ & kOneLine) ? gosh::fWasDollar : 0u));
          push(std::make_unique<Re>((flags_ & kOneLine) ? kEOT : kEOL, flags_)); ++t; break;
        case '.':
          gs_.op((flags_ & kDotNL) ? gosh::gAnyChar : gosh::gAnyCharNotNL, gf());
          push(std::make_unique<Re>((flags_ & kDotNL) ? kAnyChar : kAnyNotNL, flags_)); ++t; break;
        case '[': t = parse_class(t, end); break;
        case '*': case '+': case '?': {
          Op op = *t == '*' ? kStar : (*t == '+' ? kPlus : kQuest);
          const char *before = t;
          t = apply_repeat(op, 0, 0, before, t + 1, end, last_repeat);
          repeat = before;
          break;
        }
        case '{': {
          const char *before = t, *after;
          int mn, mx;
          if (!parse_repeat(t, end, &mn, &mx, &after)) { literal('{'); ++t; break; }
          if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx))
            throw ParseError{kErrInvalidRepeatSize, std::string(before, after)};
          t = apply_repeat(kRepeat, mn, mx, before, after, end, last_repeat);
          repeat = before;
          break;
        }
        case '\\': t = parse_backslash(t, end); break;
        default: {
          int w;
          int32_t c = next_rune(t, end, &w);
          literal(c);
          t += w;
        }
      }
      last_repeat = repeat;
    }
    gs_.end(gf());
    concat();
    if (swap_vbar()) stack_.pop_back();
    alternate();
    if (stack_.size() != 1) throw ParseError{kErrMissingParen, whole_};
    return std::move(stack_[0]);
  }

  const std::string &whole_;
  uint32_t flags_ = kClassNL | kOneLine | kPerlX;
  int ncap_ = 0;
  std::vector<ReP> stack_;
  gosh::GoShape<SimpleFold> gs_;

  int32_t next_rune(const char *t, const char *end, int *w) {
    int32_t c = decode_rune(reinterpret_cast<const uint8_t *>(t), static_cast<size_t>(end - t), w);
    if (c == kRuneError && *w == 1) throw ParseError{kErrInvalidUTF8, std::string(t, end)};
    return c;
  }

  void push(ReP r) { stack_.push_back(std::move(r)); }
  void push_paren(int cap) {
    gs_.op(gosh::gLeftParen, gf(), cap);
    auto p = std::make_unique<Re>(kLParen, flags_);
    p->cap = cap;
    push(std::move(p));
  }
  void literal(int32_t r) {
    gs_.literal(r, gf());
    auto n = std::make_unique<Re>(kLit, flags_);
    n->rune = r;
    push(std::move(n));
  }
  size_t top_items() const {
    size_t i = stack_.size();
    while (i > 0 && stack_[i - 1]->op < kPseudo) --i;
    return i;
  }
  void concat() {
    size_t i = top_items();
    ReP n;
    if (stack_.size() - i == 0) n = std::make_unique<Re>(kEmpty, flags_);
    else if (stack_.size() - i == 1) n = std::move(stack_[i]);
    else {
      n = std::make_unique<Re>(kConcat, flags_);
      for (size_t k = i; k < stack_.size(); ++k) n->sub.push_back(std::move(stack_[k]));
    }
    stack_.resize(i);
    push(std::move(n));
  }
  void alternate() {
    size_t i = top_items();
    ReP n;
    if (stack_.size() - i == 0) n = std::make_unique<Re>(kNoMatch, flags_);
    else if (stack_.size() - i == 1) n = std::move(stack_[i]);
    else {
      n = std::make_unique<Re>(kAlt, flags_);
      for (size_t k = i; k < stack_.size(); ++k) n->sub.push_back(std::move(stack_[k]));
    }
    stack_.resize(i);
    push(std::move(n));
  }
  // swapVerticalBar: [.. VBAR x] -> [.. x VBAR]
  bool swap_vbar() {
    size_t n = stack_.size();
    if (n >= 2 && stack_[n - 2]->op == kVBar) { std::swap(stack_[n - 1], stack_[n - 2]); return true; }
    return false;
  }

  static bool repeat_valid(const Re *re, int n) {
    if (re->op == kRepeat) {
      int m = re->max;
      if (m == 0) return true;
      if (m < 0) m = re->min;
      if (m > n) return false;
      if (m > 0) n /= m;
    }
    for (auto &s : re->sub)
      if (!repeat_valid(s.get(), n)) return false;
    return true;
  }

  const char *apply_repeat(Op op, int mn, int mx, const char *before, const char *after, const char *end,
                           const char *last_repeat) {
    uint32_t f = flags_;
    if (after < end && *after == '?') { ++after; f ^= kNonGreedy; }
    if (last_repeat) throw ParseError{kErrInvalidRepeatOp, std::string(last_repeat, after)};
    if (stack_.empty() || stack_.back()->op >= kPseudo) throw ParseError{kErrMissingRepeatArg, std::string(before, after)};
    auto n = std::make_unique<Re>(op, f);
    n->min = mn;
    n->max = mx;
    n->sub.push_back(std::move(stack_.back()));
    stack_.back() = std::move(n);
    gs_.repeat(op == kStar ? gosh::gStar : op == kPlus ? gosh::gPlus : op == kQuest ? gosh::gQuest : gosh::gRepeat, mn, mx,
               ((f & kFold) ? gosh::fFold : 0u) | ((f & kNonGreedy) ? gosh::fNonGreedy : 0u));
    if (op == kRepeat && (mn >= 2 || mx >= 2) && !repeat_valid(stack_.back().get(), 1000))
      throw ParseError{kErrInvalidRepeatSize, std::string(before, after)};
    return after;
  }

  static bool parse_int(const char **s, const char *end, int *out) {
    const char *t = *s;
    if (t >= end || *t < '0' || *t > '9') return false;
    if (end - t >= 2 && t[0] == '0' && t[1] >= '0' && t[1] <= '9') return false;
    const char *q = t;
    while (q < end && *q >= '0' && *q <= '9') ++q;
    int n = 0;
    for (const char *c = t; c < q; ++c) {
      if (n >= 100000000) { n = -1; break; }
      n = n * 10 + (*c - '0');
    }
    *out = n;
    *s = q;
    return true;
  }
  static bool parse_repeat(const char *s, const char *end, int *mn, int *mx, const char **rest) {
    if (s >= end || *s != '{') return false;
    ++s;
    if (!parse_int(&s, end, mn)) return false;
    if (s >= end) return false;
    if (*s != ',') *mx = *mn;
    else {
      ++s;
      if (s >= end) return false;
      if (*s == '}') *mx = -1;
      else if (!parse_int(&s, end, mx)) return false;
      else if (*mx < 0) *mn = -1;
    }
    if (s >= end || *s != '}') return false;
    *rest = s + 1;
    return true;
  }

  static int unhex(int32_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  int32_t parse_escape(const char *s, const char *end, const char **rest) {
    const char *t = s + 1;
    if (t >= end) throw ParseError{kErrTrailingBackslash, ""};
    int w;
    int32_t c = next_rune(t, end, &w);
    t += w;
    switch (c) {
      case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (t >= end || *t < '0' || *t > '7') break;
        [[fallthrough]];
      case '0': {
        int32_t r = c - '0';
        for (int i = 1; i < 3; ++i) {
          if (t >= end || *t < '0' || *t > '7') break;
          r = r * 8 + (*t - '0');
          ++t;
        }
        *rest = t;
        return r;
      }
      case 'x': {
        if (t >= end) break;
        c = next_rune(t, end, &w);
        t += w;
        if (c == '{') {
          int nhex = 0;
          int64_t r = 0;
          for (;;) {
            if (t >= end) goto bad;
            c = next_rune(t, end, &w);
            t += w;
            if (c == '}') break;
            int v = unhex(c);
            if (v < 0) goto bad;
            r = r * 16 + v;
            if (r > kMaxRune) goto bad;
            ++nhex;
          }
          if (nhex == 0) goto bad;
          *rest = t;
          return static_cast<int32_t>(r);
        }
        int x = unhex(c), y = -1;
        if (t < end) { c = next_rune(t, end, &w); t += w; y = unhex(c); }
        if (x < 0 || y < 0) break;
        *rest = t;
        return x * 16 + y;
      }
      case 'a': *rest = t; return 7;
      case 'f': *rest = t; return 12;
      case 'n': *rest = t; return 10;
      case 'r': *rest = t; return 13;
      case 't': *rest = t; return 9;
      case 'v': *rest = t; return 11;
      default:
        if (c < 0x80 && !is_alnum(c)) { *rest = t; return c; }
    }
  bad:
    throw ParseError{kErrInvalidEscape, std::string(s, t)};
  }

  void append_group(Ranges &cls, const Group &g) {
    Ranges tmp;
    for (size_t i = 0; i < g.r.size(); i += 2) {
      if (flags_ & kFold) add_folded(tmp, g.r[i], g.r[i + 1]);
      else tmp.push_back({g.r[i], g.r[i + 1]});
    }
    clean(tmp);
    if (g.sign < 0) negate(tmp);
    cls.insert(cls.end(), tmp.begin(), tmp.end());
  }
  const Group *perl_class_escape(const char *s, const char *end) {
    if (!(flags_ & kPerlX) || end - s < 2 || s[0] != '\\') return nullptr;
    for (auto &g : perl_groups())
      if (g.name[1] == s[1]) return &g;
    return nullptr;
  }
  // parseUnicodeClass (UnicodeGroups, part of syntax.Perl): \pN, \p{Name},
  // \PN, \P{Name}, \p{^Name}.  Appends the (folded, negated) table to cls and
  // returns the text after it; nullptr if s is not \p / \P.
  const char *parse_unicode_class(const char *s, const char *end, Ranges &cls) {
    if (end - s < 2 || s[0] != '\\' || (s[1] != 'p' && s[1] != 'P')) return nullptr;
    int sign = s[1] == 'P' ? -1 : 1;
    const char *t = s + 2;
    std::string name, seq;
    if (t >= end || *t != '{') {
      int w = 0;
      if (t < end) next_rune(t, end, &w);
      seq.assign(s, t + w);
      name.assign(t, t + w);
      t += w;
    } else {
      const char *close = static_cast<const char *>(memchr(s, '}', static_cast<size_t>(end - s)));
      if (!close) {
        for (const char *c = s; c < end;) { int w; next_rune(c, end, &w); c += w; }  // checkUTF8
        throw ParseError{kErrInvalidCharRange, std::string(s, end)};
      }
      seq.assign(s, close + 1);
      name.assign(s + 3, close);
      for (const char *c = s + 3; c < close;) { int w; next_rune(c, close, &w); c += w; }
      t = close + 1;
    }
    if (!name.empty() && name[0] == '^') { sign = -sign; name.erase(0, 1); }
    Ranges tab;
    int tsign = 1;
    if (!unicode_table(name, &tab, &tsign)) throw ParseError{kErrInvalidCharRange, seq};
    if (flags_ & kFold) {  // the table plus its fold-equivalent runes (unicode.FoldCategory / FoldScript)
      Ranges f;
      for (auto &p : tab) add_folded(f, p.first, p.second);
      tab.swap(f);
    }
    clean(tab);
    if (sign * tsign < 0) negate(tab);
    cls.insert(cls.end(), tab.begin(), tab.end());
    return t;
  }

  const char *parse_class(const char *s, const char *end) {
    const char *t = s + 1;
    auto re = std::make_unique<Re>(kClass, flags_);
    int sign = 1;
    if (t < end && *t == '^') {
      sign = -1;
      ++t;
      if (!(flags_ & kClassNL)) re->cls.push_back({'\n', '\n'});
    }
    bool first = true;
    while (t >= end || *t != ']' || first) {
      first = false;
      if (end - t > 2 && t[0] == '[' && t[1] == ':') {
        const char *q = nullptr;
        for (const char *c = t + 2; c + 1 < end; ++c)
          if (c[0] == ':' && c[1] == ']') { q = c; break; }
        if (q) {
          std::string name(t, q + 2);
          const Group *g = nullptr;
          for (auto &pg : posix_groups())
            if (name == pg.name) g = &pg;
          if (!g) throw ParseError{kErrInvalidCharRange, name};
          append_group(re->cls, *g);
          t = q + 2;
          continue;
        }
      }
      if (const char *nt = parse_unicode_class(t, end, re->cls)) { t = nt; continue; }
      if (const Group *g = perl_class_escape(t, end)) { append_group(re->cls, *g); t += 2; continue; }
      const char *rng = t;
      int32_t lo, hi;
      if (t >= end) throw ParseError{kErrMissingBracket, std::string(s, end)};
      if (*t == '\\') lo = parse_escape(t, end, &t);
      else { int w; lo = next_rune(t, end, &w); t += w; }
      hi = lo;
      if (end - t >= 2 && t[0] == '-' && t[1] != ']') {
        ++t;
        if (*t == '\\') hi = parse_escape(t, end, &t);
        else { int w; hi = next_rune(t, end, &w); t += w; }
        if (hi < lo) throw ParseError{kErrInvalidCharRange, std::string(rng, t)};
      }
      if (flags_ & kFold) add_folded(re->cls, lo, hi);
      else re->cls.push_back({lo, hi});
    }
    ++t;
    clean(re->cls);
    if (sign < 0) negate(re->cls);
    gs_.char_class(re->cls, gf());
    push(std::move(re));
    return t;
  }

  const char *perl_flags(const char *s, const char *end) {
    const char *t = s;
    size_t off = 0;
    if (end - t > 4 && t[2] == 'P' && t[3] == '<') off = 4;
    else if (end - t > 3 && t[2] == '<') off = 3;
    if (off) {
      const char *gt = static_cast<const char *>(memchr(t, '>', static_cast<size_t>(end - t)));
      if (!gt) {
        for (const char *c = t; c < end;) { int w; next_rune(c, end, &w); c += w; }  // checkUTF8
        throw ParseError{kErrInvalidNamedCapture, std::string(s, end)};
      }
      std::string name(t + off, gt);
      bool ok = !name.empty();
      for (char ch : name)
        if (!(is_alnum(static_cast<unsigned char>(ch)) || ch == '_')) ok = false;
      if (!ok) {
        for (const char *c = t + off; c < gt;) { int w; next_rune(c, gt, &w); c += w; }
        throw ParseError{kErrInvalidNamedCapture, std::string(s, gt + 1)};
      }
      ++ncap_;
      push_paren(ncap_);
      return gt + 1;
    }
    t += 2;
    uint32_t f = flags_;
    int sign = 1;
    bool saw = false;
    while (t < end) {
      int w;
      int32_t c = next_rune(t, end, &w);
      t += w;
      switch (c) {
        case 'i': f |= kFold; saw = true; continue;
        case 'm': f &= ~kOneLine; saw = true; continue;
        case 's': f |= kDotNL; saw = true; continue;
        case 'U': f |= kNonGreedy; saw = true; continue;
        case '-':
          if (sign < 0) goto bad;
          sign = -1;
          f = ~f;
          saw = false;
          continue;
        case ':': case ')':
          if (sign < 0) {
            if (!saw) goto bad;
            f = ~f;
          }
          if (c == ':') push_paren(0);
          flags_ = f;
          return t;
        default:
          goto bad;
      }
    }
  bad:
    throw ParseError{kErrInvalidPerlOp, std::string(s, t)};
  }

  const char *parse_backslash(const char *t, const char *end) {
    if ((flags_ & kPerlX) && end - t >= 2) {
      switch (t[1]) {
        case 'A': gs_.op(gosh::gBeginText, gf()); push(std::make_unique<Re>(kBOT, flags_)); return t + 2;
        case 'b': gs_.op(gosh::gWordBoundary, gf()); push(std::make_unique<Re>(kWB, flags_)); return t + 2;
        case 'B': gs_.op(gosh::gNoWordBoundary, gf()); push(std::make_unique<Re>(kNWB, flags_)); return t + 2;
        case 'C': throw ParseError{kErrInvalidEscape, std::string(t, t + 2)};
        case 'Q': {
          const char *q = t + 2, *e = nullptr;
          for (const char *c = q; c + 1 < end; ++c)
            if (c[0] == '\\' && c[1] == 'E') { e = c; break; }
          const char *lend = e ? e : end;
          while (q < lend) { int w; int32_t c = next_rune(q, lend, &w); literal(c); q += w; }
          return e ? e + 2 : end;
        }
        case 'z': gs_.op(gosh::gEndText, gf()); push(std::make_unique<Re>(kEOT, flags_)); return t + 2;
        default: break;
      }
    }
    gs_.esc_alloc();  // parse's backslash case allocates a class node before it knows
    {
      Ranges u;
      if (const char *nt = parse_unicode_class(t, end, u)) {
        auto re = std::make_unique<Re>(kClass, flags_);
        re->cls.swap(u);
        clean(re->cls);
        gs_.esc_class(re->cls, gf());
        push(std::move(re));
        return nt;
      }
    }
    if (const Group *g = perl_class_escape(t, end)) {
      auto re = std::make_unique<Re>(kClass, flags_);
      append_group(re->cls, *g);
      clean(re->cls);
      gs_.esc_class(re->cls, gf());
      push(std::move(re));
      return t + 2;
    }
    gs_.esc_free();
    const char *rest;
    int32_t c = parse_escape(t, end, &rest);
    literal(c);
    return rest;
  }
};

// ------------------------------------------------------------------ NFA

enum NK : uint8_t { NK_CHAR, NK_EPS, NK_SPLIT, NK_ASSERT, NK_MATCH };
enum Cond : uint8_t { C_BOL = 1, C_EOL = 2, C_BOT = 4, C_EOT = 8, C_WB = 16, C_NWB = 32 };

struct NNode {
  NK k;
  uint8_t cond = 0;
  int32_t out = -1, out1 = -1;
  int32_t set = -1;  // NK_CHAR: index into Nfa::sets
};

struct Nfa {
  std::vector<NNode> nodes;
  std::vector<Ranges> sets;
  std::map<Ranges, int32_t> set_ids;
  int32_t start = -1;
  uint8_t conds = 0;  // union of assertion kinds present
  size_t limit = 8000000;  // past Go's program limit (regexp/syntax maxSize, 3355443 instructions)

  int32_t node(NK k) {
    if (nodes.size() >= limit) throw ParseError{"", ""};
    nodes.push_back(NNode{k});
    return static_cast<int32_t>(nodes.size() - 1);
  }
  int32_t set_id(const Ranges &r) {
    auto it = set_ids.find(r);
    if (it != set_ids.end()) return it->second;
    sets.push_back(r);
    return set_ids[r] = static_cast<int32_t>(sets.size() - 1);
  }
};

struct Frag {
  int32_t start;
  std::vector<int64_t> holes;  // (node << 1) | which
};

class NfaBuilder {
 public:
  explicit NfaBuilder(Nfa &n) : n_(n) {}
  Frag build(const Re *r) {
    switch (r->op) {
      case kNoMatch: { int32_t i = n_.node(NK_CHAR); n_.nodes[i].set = n_.set_id({}); return {i, {}}; }
      case kEmpty: return empty();
      case kLit: {
        Ranges v{{r->rune, r->rune}};
        if (r->flags & kFold)
          for (int32_t f = simple_fold(r->rune); f != r->rune; f = simple_fold(f)) v.push_back({f, f});
        clean(v);
        return chr(v);
      }
      case kClass: return chr(r->cls);
      case kAnyChar: return chr({{0, kMaxRune}});
      case kAnyNotNL: return chr({{0, '\n' - 1}, {'\n' + 1, kMaxRune}});
      case kBOL: return assert_(C_BOL);
      case kEOL: return assert_(C_EOL);
      case kBOT: return assert_(C_BOT);
      case kEOT: return assert_(C_EOT);
      case kWB: return assert_(C_WB);
      case kNWB: return assert_(C_NWB);
      case kCap: return build(r->sub[0].get());
      case kStar: return star(build(r->sub[0].get()));
      case kPlus: {
        Frag b = build(r->sub[0].get());
        int32_t s = n_.node(NK_SPLIT);
        n_.nodes[s].out = b.start;
        patch(b, s);
        return {b.start, {(int64_t(s) << 1) | 1}};
      }
      case kQuest: return quest(build(r->sub[0].get()));
      case kRepeat: {
        const Re *x = r->sub[0].get();
        int mn = r->min, mx = r->max;
        if (mx == 0) return empty();
        Frag acc{-1, {}};
        bool have = false;
        for (int i = 0; i < mn; ++i) {
          Frag c = build(x);
          acc = have ? cat(acc, c) : c;
          have = true;
        }
        if (mx < 0) {
          Frag s = star(build(x));
          return have ? cat(acc, s) : s;
        }
        if (mx > mn) {
          Frag opt = quest(build(x));
          for (int i = mn + 1; i < mx; ++i) opt = quest(cat(build(x), opt));
          return have ? cat(acc, opt) : opt;
        }
        return acc;
      }
      case kConcat: {
        Frag acc = build(r->sub[0].get());
        for (size_t i = 1; i < r->sub.size(); ++i) acc = cat(acc, build(r->sub[i].get()));
        return acc;
      }
      case kAlt: {
        Frag acc = build(r->sub.back().get());
        for (int i = static_cast<int>(r->sub.size()) - 2; i >= 0; --i) {
          Frag a = build(r->sub[i].get());
          int32_t s = n_.node(NK_SPLIT);
          n_.nodes[s].out = a.start;
          n_.nodes[s].out1 = acc.start;
          a.holes.insert(a.holes.end(), acc.holes.begin(), acc.holes.end());
          acc = {s, std::move(a.holes)};
        }
        return acc;
      }
      default: return empty();
    }
  }
  void patch(Frag &f, int32_t target) {
    for (int64_t h : f.holes) {
      NNode &nd = n_.nodes[static_cast<size_t>(h >> 1)];
      if (h & 1) nd.out1 = target; else nd.out = target;
    }
    f.holes.clear();
  }

 private:
  Nfa &n_;
  Frag empty() { int32_t i = n_.node(NK_EPS); return {i, {int64_t(i) << 1}}; }
  Frag chr(const Ranges &r) {
    int32_t i = n_.node(NK_CHAR);
    n_.nodes[i].set = n_.set_id(r);
    return {i, {int64_t(i) << 1}};
  }
  Frag assert_(uint8_t c) {
    int32_t i = n_.node(NK_ASSERT);
    n_.nodes[i].cond = c;
    n_.conds |= c;
    return {i, {int64_t(i) << 1}};
  }
  Frag star(Frag b) {
    int32_t s = n_.node(NK_SPLIT);
    n_.nodes[s].out = b.start;
    patch(b, s);
    return {s, {(int64_t(s) << 1) | 1}};
  }
  Frag quest(Frag b) {
    int32_t s = n_.node(NK_SPLIT);
    n_.nodes[s].out = b.start;
    b.holes.push_back((int64_t(s) << 1) | 1);
    return {s, std::move(b.holes)};
  }
  Frag cat(Frag a, Frag b) {
    patch(a, b.start);
    return {a.start, std::move(b.holes)};
  }
};

// --------------------------------------------------- literal analysis
//
// Prefilter extraction (RE2-style "required literals"): for every node,
// `exact` = the finite set of strings the node can match (when small), and
// `req` = an OR-set such that every match contains one of its strings.  A
// string is ASCII bytes with a per-byte case-insensitivity flag; runes whose
// fold orbit leaves ASCII (k, s, non-ASCII) break strings, so an ASCII
// case-insensitive compare is always a *necessary* condition for a match.

struct LStr {
  std::string s, ci;
};
using LSet = std::vector<LStr>;

struct LInfo {
  bool exact = false;
  LSet ex;
  bool pure = true;  // no empty-width assertions inside
  bool has_req = false;
  LSet req;
};

constexpr size_t kMaxSet = 32, kMaxLen = 96;

bool cross(const LSet &a, const LSet &b, LSet *out) {
  if (a.size() * b.size() > kMaxSet) return false;
  LSet o;
  for (auto &x : a)
    for (auto &y : b) {
      if (x.s.size() + y.s.size() > kMaxLen) return false;
      o.push_back({x.s + y.s, x.ci + y.ci});
    }
  *out = std::move(o);
  return true;
}

bool nonempty_all(const LSet &s) {
  if (s.empty()) return false;
  for (auto &x : s)
    if (x.s.empty()) return false;
  return true;
}

int byte_weight(unsigned char c) {
  static const char *common = "etaoinsrhldcumwfgypbvkxjqz";
  if (c >= 'a' && c <= 'z') {
    const char *p = strchr(common, c);
    return 26 - (int)(p - common);
  }
  if (c >= 'A' && c <= 'Z') return strchr("GETPOSHTML", c) ? 24 : 6;
  if (c >= '0' && c <= '9') return 10;
  switch (c) {
    case ' ': return 30;
    case '/': case '.': return 20;
    case ':': case '|': return 10;
    case '-': case ';': case '(': case ')': case ',': return 8;
    default: return 4;
  }
}

// 4-grams present in nearly every access-log line (method, protocol, common
// host / user-agent tokens): a window equal to one of these is never chosen
// while a rarer one exists.
bool common_log_gram(const char *g) {
  static const char *kCommon[] = {"GET ", "POST", "OST ", "HTTP", "TTP/", "TP/1", "P/1.", "/1.1", "/2.0", "P/2.",
                                  "HEAD", "EAD ", ".com", "www.", "Mozi", "ozil", "zill", "illa", "lla/", "a/5.",
                                  "/5.0", ".php", "html", ".htm", "http", "ttp:", "tp:/", "p://", "://w", "//ww",
                                  "/ww.", "Wind", "indo", "ndow", "dows", "Geck", "ecko", "Appl", "pple", "ebKi"};
  for (const char *c : kCommon)
    if (strncasecmp(c, g, 4) == 0) return true;
  return false;
}

// lower = rarer; windows over case-insensitive bytes cost their variants
int window_score(const LStr &l, size_t o) {
  if (common_log_gram(l.s.data() + o)) return 1000;
  int sc = 0, ci = 0;
  for (size_t i = o; i < o + 4; ++i) {
    unsigned char c = (unsigned char)l.s[i];
    sc += byte_weight(l.ci[i] ? (unsigned char)(c | 0x20) : c);
    ci += l.ci[i] ? 1 : 0;
  }
  return sc + 3 * ci;
}

int string_score(const LStr &l) {
  if (l.s.size() < 4) return 1 << 20;
  int best = 1 << 20;
  for (size_t o = 0; o + 4 <= l.s.size(); ++o) best = std::min(best, window_score(l, o));
  return best;
}

// score of an OR-set: the worst member dominates (every member is probed)
int set_score(const LSet &s) {
  if (!nonempty_all(s)) return 1 << 22;
  int worst = 0;
  for (auto &x : s) worst = std::max(worst, string_score(x));
  return worst + 2 * (int)s.size();
}

void consider(LInfo &o, const LSet &cand) {
  if (!nonempty_all(cand)) return;
  if (!o.has_req || set_score(cand) < set_score(o.req)) {
    o.req = cand;
    o.has_req = true;
  }
}

bool lit_char(const Re *x, LStr *out) {
  auto cs = [&](int32_t r) {
    out->s = std::string(1, (char)r);
    out->ci = std::string(1, '\0');
    return true;
  };
  auto ci_letter = [&](int32_t r) {
    int32_t lo = r | 0x20;
    if (lo == 'k' || lo == 's') return false;  // folds to U+212A / U+017F
    out->s = std::string(1, (char)lo);
    out->ci = std::string(1, '\1');
    return true;
  };
  auto is_letter = [](int32_t r) { return (r >= 'a' && r <= 'z') || (r >= 'A' && r <= 'Z'); };
  if (x->op == kLit) {
    if (x->rune >= 0x80) return false;
    if ((x->flags & kFold) && is_letter(x->rune)) return ci_letter(x->rune);
    return cs(x->rune);
  }
  if (x->op == kClass) {
    const Ranges &c = x->cls;
    if (c.size() == 1 && c[0].first == c[0].second && c[0].first < 0x80) return cs(c[0].first);
    if (c.size() == 2 && c[0].first == c[0].second && c[1].first == c[1].second && c[1].first < 0x80 &&
        is_letter(c[0].first) && (c[0].first | 0x20) == c[1].first && c[1].first - c[0].first == 0x20)
      return ci_letter(c[0].first);
  }
  return false;
}

LInfo analyze(const Re *r) {
  LInfo o;
  LStr ch;
  if (lit_char(r, &ch)) {
    o.exact = true;
    o.ex = {ch};
    o.has_req = true;
    o.req = o.ex;
    return o;
  }
  switch (r->op) {
    case kEmpty:
      o.exact = true;
      o.ex = {LStr{}};
      return o;
    case kBOL: case kEOL: case kBOT: case kEOT: case kWB: case kNWB:
      o.exact = true;
      o.ex = {LStr{}};
      o.pure = false;
      return o;
    case kCap: return analyze(r->sub[0].get());
    case kPlus: {
      LInfo c = analyze(r->sub[0].get());
      if (c.exact && nonempty_all(c.ex)) consider(o, c.ex);
      if (c.has_req) consider(o, c.req);
      o.pure = c.pure;
      return o;
    }
    case kRepeat: {
      LInfo c = analyze(r->sub[0].get());
      o.pure = c.pure;
      if (r->min < 1) return o;
      if (c.exact && nonempty_all(c.ex)) consider(o, c.ex);
      if (c.has_req) consider(o, c.req);
      if (c.exact && r->min == r->max) {
        LSet acc{LStr{}};
        bool ok = true;
        for (int i = 0; i < r->min && ok; ++i) ok = cross(acc, c.ex, &acc);
        if (ok) {
          o.exact = true;
          o.ex = acc;
          consider(o, acc);
        }
      }
      return o;
    }
    case kConcat: {
      LSet run{LStr{}};
      bool all_exact = true, run_ok = true;
      LSet full{LStr{}};
      for (auto &sp : r->sub) {
        LInfo c = analyze(sp.get());
        o.pure = o.pure && c.pure;
        if (c.exact) {
          LSet nr;
          if (run_ok && cross(run, c.ex, &nr)) run = std::move(nr);
          else {
            consider(o, run);
            run = c.ex;
            run_ok = true;
          }
          if (all_exact && !cross(full, c.ex, &full)) all_exact = false;
        } else {
          all_exact = false;
          consider(o, run);
          run = {LStr{}};
          if (c.has_req) consider(o, c.req);
        }
      }
      consider(o, run);
      if (all_exact) {
        o.exact = true;
        o.ex = full;
      }
      return o;
    }
    case kAlt: {
      bool all_exact = true, all_req = true;
      LSet ex, req;
      for (auto &sp : r->sub) {
        LInfo c = analyze(sp.get());
        o.pure = o.pure && c.pure;
        if (c.exact) ex.insert(ex.end(), c.ex.begin(), c.ex.end());
        else all_exact = false;
        const LSet *best = nullptr;
        if (c.exact && nonempty_all(c.ex)) best = &c.ex;
        if (c.has_req && (!best || set_score(c.req) < set_score(*best))) best = &c.req;
        if (best) req.insert(req.end(), best->begin(), best->end());
        else all_req = false;
      }
      if (all_exact && ex.size() <= kMaxSet) {
        o.exact = true;
        o.ex = ex;
      }
      if (all_req && req.size() <= kMaxSet) consider(o, req);
      return o;
    }
    default:
      return o;
  }
}

bool is_dotstar(const Re *r) {
  return r->op == kStar && (r->sub[0]->op == kAnyNotNL || r->sub[0]->op == kAnyChar);
}

// Anchored at rest[0]: the pattern begins with \A / ^ (OneLine).
bool anchored_start(const Re *r) {
  while (r->op == kCap) r = r->sub[0].get();
  if (r->op == kBOT) return true;
  if (r->op == kConcat && !r->sub.empty()) return anchored_start(r->sub[0].get());
  return false;
}

// Anchored rules: the exact strings every match starts with (the longest run
// of exact, assertion-free pieces after \A), and whether the rest of the
// pattern can match anything (only .* left), so that the prefix decides alone.
bool anchored_prefix(const Re *r, LSet *pre, bool *equiv) {
  while (r->op == kCap) r = r->sub[0].get();
  if (r->op != kConcat || r->sub.empty()) return false;
  const Re *first = r->sub[0].get();
  while (first->op == kCap) first = first->sub[0].get();
  if (first->op != kBOT) return false;
  LSet run{LStr{}};
  size_t k = 1;
  for (; k < r->sub.size(); ++k) {
    LInfo c = analyze(r->sub[k].get());
    LSet nr;
    if (!c.exact || !c.pure || !cross(run, c.ex, &nr)) break;
    run = std::move(nr);
  }
  if (!nonempty_all(run)) return false;
  bool rest_any = true;
  for (size_t i = k; i < r->sub.size(); ++i) rest_any = rest_any && is_dotstar(r->sub[i].get());
  *pre = std::move(run);
  *equiv = rest_any;
  return true;
}

// match <=> text contains one of S, when the pattern is (.*)* X (.*)* with X
// pure and exact (S = X's strings), since .* can always match empty.
bool prefilter_equivalent(const Re *r, const LSet &chosen) {
  while (r->op == kCap) r = r->sub[0].get();
  LSet x;
  if (r->op != kConcat) {
    LInfo li = analyze(r);
    if (!li.exact || !li.pure) return false;
    x = li.ex;
  } else {
    size_t i = 0, n = r->sub.size();
    while (i < n && is_dotstar(r->sub[i].get())) ++i;
    size_t j = n;
    while (j > i && is_dotstar(r->sub[j - 1].get())) --j;
    x = {LStr{}};
    for (size_t k = i; k < j; ++k) {
      LInfo li = analyze(r->sub[k].get());
      if (!li.exact || !li.pure || !cross(x, li.ex, &x)) return false;
    }
  }
  if (!nonempty_all(x) || x.size() != chosen.size()) return false;
  auto key = [](const LSet &s) {
    std::vector<std::string> v;
    for (auto &e : s) v.push_back(e.s + '\0' + e.ci);
    std::sort(v.begin(), v.end());
    return v;
  };
  return key(x) == key(chosen);
}

// The strings every match begins with, when the pattern is (.*)* X ... and
// X's leading pieces are exact and assertion-free (text has no '\n', so the
// leading .* never constrains an unanchored match): their cross product.
bool leading_literals(const Re *r, LSet *out) {
  while (r->op == kCap) r = r->sub[0].get();
  LSet run{LStr{}};
  if (r->op != kConcat) {
    LInfo li = analyze(r);
    if (!li.exact || !li.pure) return false;
    run = li.ex;
  } else {
    size_t i = 0;
    const size_t n = r->sub.size();
    while (i < n && is_dotstar(r->sub[i].get())) ++i;
    for (size_t k = i; k < n; ++k) {
      LInfo li = analyze(r->sub[k].get());
      LSet nr;
      if (!li.exact || !li.pure || !cross(run, li.ex, &nr)) break;
      run = std::move(nr);
    }
  }
  if (!nonempty_all(run)) return false;
  *out = std::move(run);
  return true;
}

// Most bytes (UTF-8) a pure node can match; -1 when unbounded or when the node
// holds an empty-width assertion.
int max_match_bytes(const Re *r) {
  auto utf8_len = [](int32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; };
  switch (r->op) {
    case kEmpty: case kNoMatch: return 0;
    case kLit: return (r->flags & kFold) ? 4 : utf8_len(r->rune);  // a fold orbit may leave ASCII
    case kClass: {
      int m = 0;
      for (auto &rg : r->cls) m = std::max(m, utf8_len(rg.second));
      return m;
    }
    case kAnyNotNL: case kAnyChar: return 4;
    case kCap: case kQuest: return max_match_bytes(r->sub[0].get());
    case kRepeat: {
      if (r->max < 0) return -1;
      const int s = max_match_bytes(r->sub[0].get());
      return s < 0 ? -1 : (r->max * s > 4096 ? -1 : r->max * s);
    }
    case kConcat: {
      int t = 0;
      for (auto &s : r->sub) {
        const int m = max_match_bytes(s.get());
        if (m < 0 || t + m > 4096) return -1;
        t += m;
      }
      return t;
    }
    case kAlt: {
      int t = 0;
      for (auto &s : r->sub) {
        const int m = max_match_bytes(s.get());
        if (m < 0) return -1;
        t = std::max(t, m);
      }
      return t;
    }
    default: return -1;  // star, plus, assertions
  }
}

// The strings S every match contains at most *dist bytes after its start,
// when (per branch of a top-level alternation) the pattern is (.*)* P X ...
// with P pure and at most *dist bytes long and X's leading exact,
// assertion-free pieces spelling S (each >= 4 bytes): a DFA job may start
// *dist bytes (plus a rune's worth) before the first hit of S.  dist 0 is
// leading_literals' case.  P being assertion-free keeps the start context of a
// job started inside the text irrelevant.
bool bounded_leading_literals(const Re *r, LSet *out, int *dist) {
  while (r->op == kCap) r = r->sub[0].get();
  if (r->op == kAlt) {
    LSet all;
    int d = 0;
    for (auto &b : r->sub) {
      LSet s;
      int bd = 0;
      if (!bounded_leading_literals(b.get(), &s, &bd)) return false;
      all.insert(all.end(), s.begin(), s.end());
      d = std::max(d, bd);
    }
    if (all.size() > kMaxSet) return false;
    *out = std::move(all);
    *dist = d;
    return true;
  }
  auto long_enough = [](const LSet &s) {
    if (!nonempty_all(s)) return false;
    for (auto &x : s)
      if (x.s.size() < 4) return false;
    return true;
  };
  if (r->op != kConcat) {
    LInfo li = analyze(r);
    if (!li.exact || !li.pure || !long_enough(li.ex)) return false;
    *out = li.ex;
    *dist = 0;
    return true;
  }
  const size_t n = r->sub.size();
  size_t i = 0;
  while (i < n && is_dotstar(r->sub[i].get())) ++i;
  int pre = 0;
  for (size_t k = i; k < n; ++k) {
    LInfo li = analyze(r->sub[k].get());
    if (li.exact && li.pure && nonempty_all(li.ex)) {
      LSet run = li.ex;
      for (size_t q = k + 1; q < n; ++q) {
        LInfo l2 = analyze(r->sub[q].get());
        LSet nr;
        if (!l2.exact || !l2.pure || !cross(run, l2.ex, &nr)) break;
        run = std::move(nr);
      }
      if (long_enough(run)) {
        *out = std::move(run);
        *dist = pre;
        return true;
      }
    }
    const int m = max_match_bytes(r->sub[k].get());
    if (m < 0 || pre + m > 255) return false;
    pre += m;
  }
  return false;
}

constexpr int kLeadScoreMargin = 32;  // window-score units (byte_weight) a leading set may trail the best by

bool same_set(const LSet &a, const LSet &b) {
  auto key = [](const LSet &s) {
    std::vector<std::string> v;
    for (auto &e : s) v.push_back(e.s + '\0' + e.ci);
    std::sort(v.begin(), v.end());
    return v;
  };
  return key(a) == key(b);
}

// ------------------------------------------------------------------ DFA

enum Ctx : uint8_t { X_OTHER = 0, X_WORD = 1, X_NL = 2, X_START = 3 };

uint8_t empty_flags(uint8_t ctx, int nextcat /*0 other,1 word,2 nl,3 end*/) {
  uint8_t op = C_NWB;
  int boundary = 0;
  if (ctx == X_WORD) boundary = 1;
  else if (ctx == X_NL) op |= C_BOL;
  else if (ctx == X_START) op |= C_BOT | C_BOL;
  if (nextcat == 1) boundary ^= 1;
  else if (nextcat == 2) op |= C_EOL;
  else if (nextcat == 3) op |= C_EOT | C_EOL;
  if (boundary) op ^= (C_WB | C_NWB);
  return op;
}

struct KeyHash {
  size_t operator()(const std::string &s) const { return std::hash<std::string>()(s); }
};

// Per-rule partition of [0, 0x10FFFF] into rune classes: runes in one class
// are in exactly the same NFA character sets (and, when \b / ^ / $ occur, of
// the same word / newline category).
struct ClassPart {
  uint32_t ncls = 0;
  std::vector<std::pair<int32_t, uint32_t>> intervals;  // (lo, class) over [0, max]
  std::vector<std::vector<uint8_t>> member;             // set -> class -> in
  std::vector<int> cat;                                 // class -> 0 other / 1 word / 2 nl
};

ClassPart make_classes(const Nfa &n_) {
  ClassPart P;
  std::vector<int32_t> b{0, kMaxRune + 1, 0x80};
  for (auto &s : n_.sets)
    for (auto &p : s) { b.push_back(p.first); b.push_back(p.second + 1); }
  if (n_.conds & (C_WB | C_NWB))
    for (int32_t x : {int32_t('0'), int32_t('9' + 1), int32_t('A'), int32_t('Z' + 1), int32_t('_'), int32_t('_' + 1),
                      int32_t('a'), int32_t('z' + 1)})
      b.push_back(x);
  if (n_.conds & (C_BOL | C_EOL)) { b.push_back('\n'); b.push_back('\n' + 1); }
  std::sort(b.begin(), b.end());
  b.erase(std::unique(b.begin(), b.end()), b.end());
  // signature per elementary interval
  std::map<std::vector<uint8_t>, uint32_t> sig_ids;
  const size_t nsets = n_.sets.size();
  std::vector<std::vector<uint8_t>> cls_sig;
  for (size_t i = 0; i + 1 < b.size(); ++i) {
    int32_t lo = b[i];
    std::vector<uint8_t> sig(nsets + 1, 0);
    for (size_t s = 0; s < nsets; ++s) {
      const Ranges &r = n_.sets[s];
      auto it = std::upper_bound(r.begin(), r.end(), std::make_pair(lo, kMaxRune + 1));
      if (it != r.begin() && std::prev(it)->second >= lo) sig[s] = 1;
    }
    int cat = 0;
    if ((n_.conds & (C_WB | C_NWB)) && is_word_rune(lo)) cat = 1;
    else if ((n_.conds & (C_BOL | C_EOL)) && lo == '\n') cat = 2;
    sig[nsets] = static_cast<uint8_t>(cat);
    auto it = sig_ids.find(sig);
    uint32_t cid;
    if (it == sig_ids.end()) {
      cid = static_cast<uint32_t>(sig_ids.size());
      sig_ids.emplace(sig, cid);
      cls_sig.push_back(sig);
      P.cat.push_back(cat);
    } else cid = it->second;
    P.intervals.push_back({lo, cid});
  }
  P.ncls = static_cast<uint32_t>(sig_ids.size());
  P.member.assign(nsets, std::vector<uint8_t>(P.ncls, 0));
  for (uint32_t c = 0; c < P.ncls; ++c)
    for (size_t s = 0; s < nsets; ++s) P.member[s][c] = cls_sig[c][s];
  return P;
}

// rune -> class tables of a partition: ascii[128], non-ASCII interval starts
void class_tables(const ClassPart &P, uint16_t *ascii, std::vector<std::pair<uint32_t, uint32_t>> *nonascii) {
  const auto &iv = P.intervals;
  for (size_t k = 0; k < iv.size(); ++k) {
    const int32_t lo = iv[k].first;
    if (lo < 0x80) {
      const int32_t hi = k + 1 < iv.size() ? std::min<int32_t>(iv[k + 1].first, 0x80) : 0x80;
      for (int32_t r = lo; r < hi; ++r) ascii[r] = static_cast<uint16_t>(iv[k].second);
    } else if (nonascii->empty() || nonascii->back().second != iv[k].second) {
      nonascii->push_back({static_cast<uint32_t>(lo), iv[k].second});
    }
  }
}

class DfaBuilder {
 public:
  DfaBuilder(const Nfa &nfa, const ClassPart &P, uint32_t max_states)
      : n_(nfa), max_states_(max_states), ncls_(P.ncls), intervals_(P.intervals), member_(P.member), cls_cat_(P.cat) {}

  int build(CompiledRegex *out) {
    if (ncls_ > 255) return BJX_ERR_TOO_COMPLEX;
    track_word_ = (n_.conds & (C_WB | C_NWB)) != 0;
    track_nl_ = (n_.conds & C_BOL) != 0;
    track_start_ = (n_.conds & (C_BOT | C_BOL)) != 0;
    mark_.assign(n_.nodes.size(), 0);
    // state 0 = DEAD placeholder, 1 = ACCEPT
    rows_.assign(2 * ncls_, 0);
    for (uint32_t c = 0; c < ncls_; ++c) { rows_[c] = kDead; rows_[ncls_ + c] = kAccept; }
    acc_end_ = {0, 1};
    std::vector<int32_t> seed{n_.start};
    std::vector<int32_t> s0 = closure0(seed);
    uint32_t start = has_match(s0) ? kAccept : intern(s0, track_start_ ? X_START : X_OTHER);
    while (!work_.empty()) {
      uint32_t sid = work_.back();
      work_.pop_back();
      if (sid >= max_states_) return BJX_ERR_TOO_COMPLEX;
      expand(sid);
    }
    finish(start, out);
    return 0;
  }

 private:
  const Nfa &n_;
  uint32_t max_states_;
  const uint32_t ncls_;
  const std::vector<std::pair<int32_t, uint32_t>> &intervals_;  // (lo, class) over [0, max]
  const std::vector<std::vector<uint8_t>> &member_;             // set -> class -> in
  const std::vector<int> &cls_cat_;                             // class -> 0 other / 1 word / 2 nl
  bool track_word_ = false, track_nl_ = false, track_start_ = false;
  std::unordered_map<std::string, uint32_t, KeyHash> ids_;
  std::vector<std::pair<std::vector<int32_t>, uint8_t>> states_;  // by id (index id-2)
  std::vector<uint32_t> work_;
  std::vector<uint16_t> rows_;
  std::vector<uint8_t> acc_end_;
  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;

  // closure through EPS/SPLIT (not through assertions): CHAR, ASSERT, MATCH nodes
  std::vector<int32_t> closure0(const std::vector<int32_t> &seeds) {
    ++gen_;
    std::vector<int32_t> st(seeds.rbegin(), seeds.rend()), out;
    while (!st.empty()) {
      int32_t i = st.back();
      st.pop_back();
      if (i < 0 || mark_[i] == gen_) continue;
      mark_[i] = gen_;
      const NNode &nd = n_.nodes[i];
      switch (nd.k) {
        case NK_EPS: st.push_back(nd.out); break;
        case NK_SPLIT: st.push_back(nd.out1); st.push_back(nd.out); break;
        default: out.push_back(i);
      }
    }
    std::sort(out.begin(), out.end());
    return out;
  }
  // continue through assertions satisfied by flags; returns CHAR nodes, sets *match
  std::vector<int32_t> closure_flags(const std::vector<int32_t> &seeds, uint8_t flags, bool *match) {
    ++gen_;
    std::vector<int32_t> st(seeds.rbegin(), seeds.rend()), out;
    *match = false;
    while (!st.empty()) {
      int32_t i = st.back();
      st.pop_back();
      if (i < 0 || mark_[i] == gen_) continue;
      mark_[i] = gen_;
      const NNode &nd = n_.nodes[i];
      switch (nd.k) {
        case NK_EPS: st.push_back(nd.out); break;
        case NK_SPLIT: st.push_back(nd.out1); st.push_back(nd.out); break;
        case NK_ASSERT: if ((nd.cond & ~flags) == 0) st.push_back(nd.out); break;
        case NK_MATCH: *match = true; break;
        case NK_CHAR: out.push_back(i); break;
      }
    }
    return out;
  }
  bool has_match(const std::vector<int32_t> &s) const {
    for (int32_t i : s)
      if (n_.nodes[i].k == NK_MATCH) return true;
    return false;
  }
  bool has_assert(const std::vector<int32_t> &s) const {
    for (int32_t i : s)
      if (n_.nodes[i].k == NK_ASSERT) return true;
    return false;
  }
  uint8_t mask_ctx(uint8_t ctx) const {
    if (ctx == X_WORD && !track_word_) return X_OTHER;
    if (ctx == X_NL && !track_nl_) return X_OTHER;
    if (ctx == X_START && !track_start_) return X_OTHER;
    return ctx;
  }
  uint32_t intern(const std::vector<int32_t> &set, uint8_t ctx) {
    if (!has_assert(set)) ctx = X_OTHER;
    ctx = mask_ctx(ctx);
    std::string key(reinterpret_cast<const char *>(set.data()), set.size() * sizeof(int32_t));
    key.push_back(static_cast<char>(ctx));
    auto it = ids_.find(key);
    if (it != ids_.end()) return it->second;
    uint32_t id = static_cast<uint32_t>(states_.size() + 2);
    ids_.emplace(std::move(key), id);
    states_.push_back({set, ctx});
    rows_.resize(static_cast<size_t>(id + 1) * ncls_, 0);
    acc_end_.push_back(0);
    work_.push_back(id);
    return id;
  }
  void expand(uint32_t sid) {
    // copy: states_ may grow during expansion
    std::vector<int32_t> set = states_[sid - 2].first;
    uint8_t ctx = states_[sid - 2].second;
    bool m;
    closure_flags(set, empty_flags(ctx, 3), &m);
    acc_end_[sid] = m ? 1 : 0;
    for (uint32_t c = 0; c < ncls_; ++c) {
      uint8_t f = empty_flags(ctx, cls_cat_[c]);
      std::vector<int32_t> chars = closure_flags(set, f, &m);
      uint32_t next;
      if (m) next = kAccept;
      else {
        std::vector<int32_t> seeds;
        for (int32_t i : chars) {
          const NNode &nd = n_.nodes[i];
          if (member_[nd.set][c]) seeds.push_back(nd.out);
        }
        seeds.push_back(n_.start);
        std::vector<int32_t> nx = closure0(seeds);
        if (has_match(nx)) next = kAccept;
        else {
          uint8_t nctx = cls_cat_[c] == 1 ? X_WORD : (cls_cat_[c] == 2 ? X_NL : X_OTHER);
          next = intern(nx, nctx);
          if (next >= max_states_) { rows_[static_cast<size_t>(sid) * ncls_ + c] = 0; work_.push_back(next); return; }
        }
      }
      rows_[static_cast<size_t>(sid) * ncls_ + c] = static_cast<uint16_t>(next);
    }
  }

  void finish(uint32_t start, CompiledRegex *out) {
    const uint32_t n = static_cast<uint32_t>(states_.size() + 2);
    // live = can reach ACCEPT or an accept_end state
    std::vector<std::vector<uint32_t>> rev(n);
    for (uint32_t s = 2; s < n; ++s)
      for (uint32_t c = 0; c < ncls_; ++c) rev[rows_[static_cast<size_t>(s) * ncls_ + c]].push_back(s);
    std::vector<uint8_t> live(n, 0);
    std::vector<uint32_t> st;
    live[kAccept] = 1;
    st.push_back(kAccept);
    for (uint32_t s = 2; s < n; ++s)
      if (acc_end_[s]) { live[s] = 1; st.push_back(s); }
    while (!st.empty()) {
      uint32_t s = st.back();
      st.pop_back();
      for (uint32_t p : rev[s])
        if (!live[p]) { live[p] = 1; st.push_back(p); }
    }
    // Moore minimisation over live states; dead -> 0
    std::vector<uint32_t> block(n, 0);
    block[kDead] = 0;
    block[kAccept] = 1;
    for (uint32_t s = 2; s < n; ++s) block[s] = live[s] ? (acc_end_[s] ? 2 : 3) : 0;
    uint32_t nblocks = 0;
    for (;;) {
      std::map<std::vector<uint32_t>, uint32_t> sig;
      std::vector<uint32_t> nb(n);
      // keep DEAD = 0 and ACCEPT = 1 fixed
      sig[{0xFFFFFFFFu, 0}] = 0;
      sig[{0xFFFFFFFFu, 1}] = 1;
      nb[kDead] = 0;
      nb[kAccept] = 1;
      for (uint32_t s = 2; s < n; ++s) {
        if (block[s] == 0) { nb[s] = 0; continue; }
        std::vector<uint32_t> k;
        k.reserve(ncls_ + 1);
        k.push_back(block[s]);
        for (uint32_t c = 0; c < ncls_; ++c) k.push_back(block[rows_[static_cast<size_t>(s) * ncls_ + c]]);
        auto it = sig.find(k);
        if (it == sig.end()) it = sig.emplace(k, static_cast<uint32_t>(sig.size())).first;
        nb[s] = it->second;
      }
      uint32_t cnt = static_cast<uint32_t>(sig.size());
      block.swap(nb);
      if (cnt == nblocks) break;
      nblocks = cnt;
    }
    // renumber: BFS from start over blocks
    std::vector<int64_t> newid(nblocks + 2, -1);
    std::vector<uint32_t> rep(nblocks + 2, 0);
    for (uint32_t s = n; s-- > 2;) rep[block[s]] = s;
    newid[0] = kDead;
    newid[1] = kAccept;
    std::vector<uint32_t> order;
    uint32_t next_id = 2;
    uint32_t sb = block[start];
    if (newid[sb] < 0) { newid[sb] = next_id++; order.push_back(sb); }
    for (size_t qi = 0; qi < order.size(); ++qi) {
      uint32_t s = rep[order[qi]];
      for (uint32_t c = 0; c < ncls_; ++c) {
        uint32_t t = block[rows_[static_cast<size_t>(s) * ncls_ + c]];
        if (newid[t] < 0) { newid[t] = next_id++; order.push_back(t); }
      }
    }
    out->nstates = next_id;
    out->ncls = ncls_;
    out->start = static_cast<uint16_t>(newid[sb]);
    out->trans.assign(static_cast<size_t>(next_id) * ncls_, 0);
    out->accept_end.assign(next_id, 0);
    out->accept_end[kAccept] = 1;
    for (uint32_t c = 0; c < ncls_; ++c) { out->trans[c] = kDead; out->trans[ncls_ + c] = kAccept; }
    for (uint32_t b : order) {
      uint32_t s = rep[b];
      uint32_t id = static_cast<uint32_t>(newid[b]);
      out->accept_end[id] = acc_end_[s];
      for (uint32_t c = 0; c < ncls_; ++c)
        out->trans[static_cast<size_t>(id) * ncls_ + c] =
            static_cast<uint16_t>(newid[block[rows_[static_cast<size_t>(s) * ncls_ + c]]]);
    }
    // rune -> class tables
    {
      uint16_t a16[128] = {};
      class_tables(ClassPart{ncls_, intervals_, {}, {}}, a16, &out->nonascii);
      for (int r = 0; r < 128; ++r) out->ascii_cls[r] = static_cast<uint8_t>(a16[r]);
    }
    bool always = out->accept_end[out->start] != 0;
    for (uint32_t c = 0; c < ncls_ && always; ++c)
      if (out->trans[static_cast<size_t>(out->start) * ncls_ + c] != kAccept) always = false;
    if (out->start == kAccept) always = true;
    out->flags = 0;
    if (always) out->flags |= kRuleAlways;
    if (out->start == kDead) out->flags |= kRuleNever;
  }
};


// ------------------------------------------------------- bit-parallel NFA
//
// Rules whose DFA passes kDfaStateCap states (counted repetition after an
// unanchored prefix, e.g. `.*a.{20}`: 2^21 DFA states) or 255 rune classes are
// matched by a bit-parallel simulation of the NFA instead.  A state is a set
// of *positions*: the CHAR, ASSERT and MATCH nodes that closure0 reaches,
// numbered in DFS preorder so that a concatenation steps position p to p + 1.
// One rune of class c, with the assertion context k = (category of the
// previous rune) * 4 + (category of c) (regexp/syntax EmptyOpContext):
//   X  = D | AT[a][k] for each ASSERT position a in D   (assertions crossed)
//   X has MATCH                       -> match before c
//   Y  = X & CM[c]                    (CHAR positions that accept c)
//   D' = ((Y & SH) << 1) | S0 | GT[g] for every group g with Y & GM[g] != 0
//   D' has MATCH                      -> match after c
// SH marks positions whose follow set contains p + 1; every other follow
// target lives in a group (positions with the same remaining follow set share
// one).  S0 = closure0(start) re-seeds the unanchored search at every rune, as
// the DFA construction does.  At the end of the text the assertions are
// crossed once more with next category "end".  Same semantics as DfaBuilder,
// so the two are interchangeable per rule.
//
// Blob layout (u64 words): header (8 x u32: W, npos, ncls, ngroups, nassert,
// match position, flags, total words), ascii classes (u16[128]), class
// categories (u8[ncls]), S0[W], SH[W], CM[ncls][W], GM[G][W], GT[G][W],
// assert positions (u32[nassert]), AT[nassert][16][W].

class BitNfaBuilder {
 public:
  BitNfaBuilder(const Nfa &nfa, const ClassPart &P) : n_(nfa), P_(P) {}

  // DFS preorder numbering over the position graph (false past `limit`)
  bool number(std::vector<int32_t> &s0, uint32_t limit) {
    mark_.assign(n_.nodes.size(), 0);
    pos_.assign(n_.nodes.size(), -1);
    order_.clear();
    kids_.clear();
    s0.clear();
    closure(n_.start, 0, false, s0);
    std::vector<int32_t> st(s0.rbegin(), s0.rend());
    while (!st.empty()) {
      const int32_t i = st.back();
      st.pop_back();
      if (pos_[i] >= 0) continue;
      if (order_.size() >= limit) return false;
      pos_[i] = static_cast<int32_t>(order_.size());
      order_.push_back(i);
      const std::vector<int32_t> &ch = children(i);
      for (auto it = ch.rbegin(); it != ch.rend(); ++it)
        if (pos_[*it] < 0) st.push_back(*it);
    }
    return true;
  }

  int build(CompiledRegex *out) {
    std::vector<int32_t> s0;
    if (!number(s0, kNfaMaxPos)) return BJX_ERR_TOO_COMPLEX;
    const uint32_t npos = static_cast<uint32_t>(order_.size());
    uint32_t W = 1;
    while (64 * W < npos) W *= 2;
    auto setbit = [&](std::vector<uint64_t> &v, size_t base, int32_t node) {
      const uint32_t p = static_cast<uint32_t>(pos_[node]);
      v[base + p / 64] |= 1ull << (p % 64);
    };
    // follow sets, shift bits, groups
    std::vector<uint64_t> s0m(W, 0), sh(W, 0);
    for (int32_t i : s0) setbit(s0m, 0, i);
    std::map<std::vector<int32_t>, uint32_t> group_of;
    std::vector<std::vector<int32_t>> gtarget;
    std::vector<std::vector<uint32_t>> gmembers;
    std::vector<uint32_t> asserts;
    for (uint32_t p = 0; p < npos; ++p) {
      const int32_t node = order_[p];
      const NNode &nd = n_.nodes[node];
      if (nd.k == NK_ASSERT) { asserts.push_back(p); continue; }
      if (nd.k != NK_CHAR) continue;
      std::vector<int32_t> rest;
      for (int32_t f : children(node)) {
        if (static_cast<uint32_t>(pos_[f]) == p + 1) sh[(p) / 64] |= 1ull << (p % 64);
        else rest.push_back(pos_[f]);
      }
      if (rest.empty()) continue;
      std::sort(rest.begin(), rest.end());
      auto it = group_of.find(rest);
      if (it == group_of.end()) {
        it = group_of.emplace(rest, static_cast<uint32_t>(gtarget.size())).first;
        gtarget.push_back(rest);
        gmembers.emplace_back();
      }
      gmembers[it->second].push_back(p);
    }
    const uint32_t ncls = P_.ncls, ng = static_cast<uint32_t>(gtarget.size()), na = static_cast<uint32_t>(asserts.size());
    const NfaLayout L = nfa_layout(W, npos, ncls, ng, na);
    if (static_cast<size_t>(L.total) * 8 > kNfaMaxBlobBytes) return BJX_ERR_TOO_COMPLEX;
    std::vector<uint64_t> b(L.total, 0);
    uint32_t match = 0xFFFFFFFFu, flags = na ? kNfaAsserts : 0u;
    for (uint32_t p = 0; p < npos; ++p)
      if (n_.nodes[order_[p]].k == NK_MATCH) match = p;
    // anchored at the text start: S0 holds only \A / ^ (OneLine) assertions,
    // which never hold again, so a state equal to S0 after the first rune is dead
    bool s0_dead = !s0.empty();
    for (int32_t i : s0)
      if (n_.nodes[i].k != NK_ASSERT || !(n_.nodes[i].cond & C_BOT)) s0_dead = false;
    if (s0_dead) flags |= kNfaAnchored;
    const uint32_t hdr[8] = {W, npos, ncls, ng, na, match, flags, L.total};
    memcpy(b.data(), hdr, sizeof hdr);
    uint16_t a16[128] = {};
    class_tables(P_, a16, &out->nonascii);
    memcpy(&b[L.o_ascii], a16, sizeof a16);
    uint8_t *cat = reinterpret_cast<uint8_t *>(&b[L.o_cat]);
    for (uint32_t c = 0; c < ncls; ++c) cat[c] = static_cast<uint8_t>(P_.cat[c]);
    for (uint32_t w = 0; w < W; ++w) { b[L.o_s0 + w] = s0m[w]; b[L.o_sh + w] = sh[w]; }
    for (uint32_t p = 0; p < npos; ++p) {
      const NNode &nd = n_.nodes[order_[p]];
      if (nd.k != NK_CHAR) continue;
      for (uint32_t c = 0; c < ncls; ++c)
        if (P_.member[nd.set][c]) b[L.o_cm + c * W + p / 64] |= 1ull << (p % 64);
    }
    for (uint32_t g = 0; g < ng; ++g) {
      for (uint32_t p : gmembers[g]) b[L.o_gm + g * W + p / 64] |= 1ull << (p % 64);
      for (int32_t q : gtarget[g]) b[L.o_gt + g * W + q / 64] |= 1ull << (q % 64);
    }
    uint32_t *apos = reinterpret_cast<uint32_t *>(&b[L.o_apos]);
    for (uint32_t a = 0; a < na; ++a) {
      apos[a] = asserts[a];
      const NNode &nd = n_.nodes[order_[asserts[a]]];
      for (uint32_t k = 0; k < 16; ++k) {
        const uint8_t f = empty_flags(static_cast<uint8_t>(k / 4), static_cast<int>(k % 4));
        if ((nd.cond & ~f) != 0) continue;
        std::vector<int32_t> t;
        closure(nd.out, f, true, t);
        for (int32_t i : t) setbit(b, L.o_at + (a * 16 + k) * W, i);
      }
    }
    out->nfa.swap(b);
    out->nfa_words = W;
    out->nstates = npos;
    out->ncls = ncls;
    out->start = 0;
    for (int r = 0; r < 128; ++r) out->ascii_cls[r] = static_cast<uint8_t>(a16[r]);
    out->flags = kRuleNfa;
    if (match != 0xFFFFFFFFu && ((s0m[match / 64] >> (match % 64)) & 1)) out->flags |= kRuleAlways;
    if (match == 0xFFFFFFFFu) out->flags |= kRuleNever;
    return 0;
  }

  // The wide NFA (kRuleNfaWide, regex_compiler.h NfaWideLayout): the same
  // positions, S0 / SH / CM as build(); each group's follow targets and each
  // (assertion, context) closure as a sorted target list instead of a W-word
  // mask, so the tables grow with the pattern, not with groups x positions.
  int build_wide(CompiledRegex *out) {
    std::vector<int32_t> s0;
    if (!number(s0, kNfaWideMaxPos)) return BJX_ERR_TOO_COMPLEX;
    const uint32_t npos = static_cast<uint32_t>(order_.size());
    const uint32_t W = (npos + 63) / 64;
    std::vector<uint64_t> s0m(W, 0), sh(W, 0), gall(W, 0), am(W, 0);
    auto set = [](std::vector<uint64_t> &v, uint32_t p) { v[p / 64] |= 1ull << (p % 64); };
    for (int32_t i : s0) set(s0m, static_cast<uint32_t>(pos_[i]));
    std::vector<uint32_t> aux(npos, 0);
    std::map<std::vector<int32_t>, uint32_t> group_of;
    std::vector<std::vector<int32_t>> gtarget;
    std::vector<uint32_t> asserts;
    uint32_t match = 0xFFFFFFFFu;
    for (uint32_t p = 0; p < npos; ++p) {
      const int32_t node = order_[p];
      const NNode &nd = n_.nodes[node];
      if (nd.k == NK_MATCH) match = p;
      if (nd.k == NK_ASSERT) {
        aux[p] = static_cast<uint32_t>(asserts.size());
        asserts.push_back(p);
        set(am, p);
        continue;
      }
      if (nd.k != NK_CHAR) continue;
      std::vector<int32_t> rest;
      for (int32_t f : children(node)) {
        if (static_cast<uint32_t>(pos_[f]) == p + 1) set(sh, p);
        else rest.push_back(pos_[f]);
      }
      if (rest.empty()) continue;
      std::sort(rest.begin(), rest.end());
      auto it = group_of.find(rest);
      if (it == group_of.end()) {
        it = group_of.emplace(rest, static_cast<uint32_t>(gtarget.size())).first;
        gtarget.push_back(rest);
      }
      aux[p] = it->second;
      set(gall, p);
    }
    const uint32_t ncls = P_.ncls, ng = static_cast<uint32_t>(gtarget.size()), na = static_cast<uint32_t>(asserts.size());
    std::vector<uint32_t> goff{0}, gtgt, aoff{0}, atgt;
    for (auto &t : gtarget) {
      for (int32_t q : t) gtgt.push_back(static_cast<uint32_t>(q));
      goff.push_back(static_cast<uint32_t>(gtgt.size()));
    }
    for (uint32_t a = 0; a < na; ++a) {
      const NNode &nd = n_.nodes[order_[asserts[a]]];
      for (uint32_t k = 0; k < 16; ++k) {
        const uint8_t f = empty_flags(static_cast<uint8_t>(k / 4), static_cast<int>(k % 4));
        if ((nd.cond & ~f) == 0) {
          std::vector<int32_t> t;
          closure(nd.out, f, true, t);
          std::vector<uint32_t> q;
          for (int32_t i : t) q.push_back(static_cast<uint32_t>(pos_[i]));
          std::sort(q.begin(), q.end());
          atgt.insert(atgt.end(), q.begin(), q.end());
        }
        aoff.push_back(static_cast<uint32_t>(atgt.size()));
      }
    }
    const NfaWideLayout L = nfa_wide_layout(W, npos, ncls, ng, na, static_cast<uint32_t>(gtgt.size()),
                                            static_cast<uint32_t>(atgt.size()));
    if (L.total > (1ull << 31)) return BJX_ERR_TOO_COMPLEX;
    std::vector<uint64_t> b(L.total, 0);
    const uint32_t hdr[16] = {W, npos, ncls, ng, na, match, na ? (uint32_t)kNfaAsserts : 0u, static_cast<uint32_t>(L.total),
                              L.n_gtgt, L.n_atgt, 0, 0, 0, 0, 0, 0};
    memcpy(b.data(), hdr, sizeof hdr);
    uint16_t a16[128] = {};
    class_tables(P_, a16, &out->nonascii);
    memcpy(&b[L.o_ascii], a16, sizeof a16);
    uint8_t *cat = reinterpret_cast<uint8_t *>(&b[L.o_cat]);
    for (uint32_t c = 0; c < ncls; ++c) cat[c] = static_cast<uint8_t>(P_.cat[c]);
    for (uint32_t w = 0; w < W; ++w) {
      b[L.o_s0 + w] = s0m[w]; b[L.o_sh + w] = sh[w]; b[L.o_gall + w] = gall[w]; b[L.o_am + w] = am[w];
    }
    for (uint32_t p = 0; p < npos; ++p) {
      const NNode &nd = n_.nodes[order_[p]];
      if (nd.k != NK_CHAR) continue;
      for (uint32_t c = 0; c < ncls; ++c)
        if (P_.member[nd.set][c]) b[L.o_cm + (uint64_t)c * W + p / 64] |= 1ull << (p % 64);
    }
    memcpy(&b[L.o_aux], aux.data(), aux.size() * 4);
    memcpy(&b[L.o_goff], goff.data(), goff.size() * 4);
    if (!gtgt.empty()) memcpy(&b[L.o_gtgt], gtgt.data(), gtgt.size() * 4);
    memcpy(&b[L.o_aoff], aoff.data(), aoff.size() * 4);
    if (!atgt.empty()) memcpy(&b[L.o_atgt], atgt.data(), atgt.size() * 4);
    out->nfa.swap(b);
    out->nfa_words = W;
    out->nstates = npos;
    out->ncls = ncls;
    out->start = 0;
    for (int r = 0; r < 128; ++r) out->ascii_cls[r] = static_cast<uint8_t>(a16[r]);
    out->flags = kRuleNfa | kRuleNfaWide;
    if (match != 0xFFFFFFFFu && ((s0m[match / 64] >> (match % 64)) & 1)) out->flags |= kRuleAlways;
    if (match == 0xFFFFFFFFu) out->flags |= kRuleNever;
    return 0;
  }

 private:
  const Nfa &n_;
  const ClassPart &P_;
  std::vector<uint32_t> mark_;
  uint32_t gen_ = 0;
  std::vector<int32_t> pos_, order_;
  std::map<int32_t, std::vector<int32_t>> kids_;

  // closure in DFS preorder through EPS / SPLIT (and, with through_asserts,
  // the assertions that flags satisfy): CHAR / MATCH nodes, plus the ASSERT
  // nodes where it stops
  void closure(int32_t seed, uint8_t flags, bool through_asserts, std::vector<int32_t> &out) {
    ++gen_;
    std::vector<int32_t> st{seed};
    while (!st.empty()) {
      const int32_t i = st.back();
      st.pop_back();
      if (i < 0 || mark_[i] == gen_) continue;
      mark_[i] = gen_;
      const NNode &nd = n_.nodes[i];
      switch (nd.k) {
        case NK_EPS: st.push_back(nd.out); break;
        case NK_SPLIT: st.push_back(nd.out1); st.push_back(nd.out); break;
        case NK_ASSERT:
          if (!through_asserts) out.push_back(i);
          else if ((nd.cond & ~flags) == 0) st.push_back(nd.out);
          break;
        default: out.push_back(i);
      }
    }
  }
  // successors in the position graph: follow set of a CHAR; every node an
  // ASSERT can lead to under some context
  const std::vector<int32_t> &children(int32_t i) {
    auto it = kids_.find(i);
    if (it != kids_.end()) return it->second;
    std::vector<int32_t> v;
    const NNode &nd = n_.nodes[i];
    if (nd.k == NK_CHAR) {
      closure(nd.out, 0, false, v);
    } else if (nd.k == NK_ASSERT) {
      std::vector<uint8_t> seen(n_.nodes.size(), 0);
      for (uint32_t k = 0; k < 16; ++k) {
        const uint8_t f = empty_flags(static_cast<uint8_t>(k / 4), static_cast<int>(k % 4));
        if ((nd.cond & ~f) != 0) continue;
        std::vector<int32_t> t;
        closure(nd.out, f, true, t);
        for (int32_t x : t)
          if (!seen[x]) { seen[x] = 1; v.push_back(x); }
      }
    }
    return kids_.emplace(i, std::move(v)).first->second;
  }
};

std::atomic<uint32_t> g_dfa_state_cap{kDfaStateCap};

}  // namespace

std::atomic<bool> g_force_wide{false};
void set_force_wide_nfa(bool on) { g_force_wide = on; }
void set_dfa_state_cap(uint32_t cap) { g_dfa_state_cap = cap ? cap : kDfaStateCap; }
uint32_t dfa_state_cap() { return g_dfa_state_cap; }

// syntax.Parse alone: Go's accept / reject decision and error text for a
// pattern, without building its automaton (bjx_debug_regex_parse)
int parse_regex_only(const std::string &pattern, std::string *err) {
  try {
    Parser p(pattern);
    p.parse();
  } catch (const ParseError &e) {
    if (err) *err = "error parsing regexp: " + e.code + ": `" + e.expr + "`";
    return BJX_ERR_REGEX;
  }
  return BJX_OK;
}

int compile_regex(const std::string &pattern, CompiledRegex *out, std::string *err, uint32_t max_dfa_states) {
  ReP root;
  try {
    Parser p(pattern);
    root = p.parse();
  } catch (const ParseError &e) {
    if (err) *err = "error parsing regexp: " + e.code + ": `" + e.expr + "`";
    return BJX_ERR_REGEX;
  }
  Nfa nfa;
  try {
    NfaBuilder b(nfa);
    Frag f = b.build(root.get());
    int32_t m = nfa.node(NK_MATCH);
    b.patch(f, m);
    nfa.start = f.start;
  } catch (const ParseError &) {
    if (err) *err = "rule too complex for the automaton compiler (NFA size)";
    return BJX_ERR_TOO_COMPLEX;
  }
  // DFA up to kDfaStateCap states; past that (or past 255 rune classes) the
  // bit-parallel NFA; a rule with too many NFA positions for that gets a DFA
  // of up to max_dfa_states states
  const ClassPart part = make_classes(nfa);
  *out = CompiledRegex();
  const uint32_t cap = std::min<uint32_t>(max_dfa_states, dfa_state_cap());
  int rc = g_force_wide ? BJX_ERR_TOO_COMPLEX : DfaBuilder(nfa, part, std::max<uint32_t>(cap, 3)).build(out);
  if (g_force_wide) max_dfa_states = cap;  // test hook: no DFA / per-lane NFA on the way
  if (rc != 0 && !g_force_wide) {
    *out = CompiledRegex();
    rc = BitNfaBuilder(nfa, part).build(out);
  }
  if (rc != 0 && max_dfa_states > cap) {
    *out = CompiledRegex();
    rc = DfaBuilder(nfa, part, std::min<uint32_t>(max_dfa_states, 65000)).build(out);
  }
  if (rc != 0) {  // past both: the block-cooperative wide NFA, no position limit short of Go's own
    *out = CompiledRegex();
    rc = BitNfaBuilder(nfa, part).build_wide(out);
  }
  if (rc != 0) {
    if (err) *err = "rule too complex for the automaton engines (more than " + std::to_string(kNfaWideMaxPos) +
                    " NFA positions)";
    return rc;
  }
  if (out->flags & kRuleAlways) out->mode = kModeAlways;
  else if (out->flags & kRuleNever) out->mode = kModeNever;
  else if (anchored_start(root.get())) {
    out->mode = kModeAnchored;
    LSet pre;
    bool eq = false;
    if (anchored_prefix(root.get(), &pre, &eq)) {
      for (auto &x : pre) out->anchor.push_back(PrefLit{x.s, x.ci, 0});
      out->anchor_equivalent = eq;
    }
  }
  else {
    LInfo li = analyze(root.get());
    LSet best;
    bool have = false;
    if (li.exact && nonempty_all(li.ex)) { best = li.ex; have = true; }
    if (li.has_req && (!have || set_score(li.req) < set_score(best))) { best = li.req; have = true; }
    // the strings every match begins with, when nearly as rare as the best
    // required set: a DFA job then starts at their first hit, not at rest[0]
    LSet lead;
    int lead_dist = 0;
    const bool has_lead = leading_literals(root.get(), &lead) || bounded_leading_literals(root.get(), &lead, &lead_dist);
    if (has_lead && set_score(lead) < 1000 && (!have || set_score(lead) <= set_score(best) + kLeadScoreMargin)) {
      best = lead;
      have = true;
    }
    if (have && set_score(best) < (1 << 20)) {
      out->mode = kModePrefilter;
      for (auto &x : best) {
        PrefLit pl{x.s, x.ci, 0};
        int bs = 1 << 30;
        for (size_t o = 0; o + 4 <= x.s.size(); ++o) {
          int sc = window_score(x, o);
          if (sc < bs) { bs = sc; pl.gram_off = (uint32_t)o; }
        }
        out->pref.push_back(pl);
      }
      out->pref_equivalent = prefilter_equivalent(root.get(), best);
      LSet l0;
      out->pref_lead = leading_literals(root.get(), &l0) && same_set(l0, best);
      if (!out->pref_lead && bounded_leading_literals(root.get(), &l0, &lead_dist) && same_set(l0, best)) {
        out->pref_lead = true;
        out->lead_dist = (uint8_t)lead_dist;
      }
      out->required_literal = best[0].s;
    } else {
      out->mode = kModeScan;
    }
  }
  return 0;
}

static bool nfa_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n) {
  const uint64_t *b = rx.nfa.data();
  uint32_t h[8];
  memcpy(h, b, sizeof h);
  const NfaLayout L = nfa_layout_of(h);
  const uint32_t W = L.W, match = L.match, flags = L.flags;
  const uint16_t *a16 = reinterpret_cast<const uint16_t *>(b + L.o_ascii);
  const uint8_t *cat = reinterpret_cast<const uint8_t *>(b + L.o_cat);
  const uint32_t *apos = reinterpret_cast<const uint32_t *>(b + L.o_apos);
  auto has = [&](const std::vector<uint64_t> &v, uint32_t p) { return p != 0xFFFFFFFFu && ((v[p / 64] >> (p % 64)) & 1); };
  std::vector<uint64_t> D(b + L.o_s0, b + L.o_s0 + W), X(W), Y(W);
  uint32_t ctx = 3;  // start of text
  auto cross = [&](uint32_t k) {
    X = D;
    for (uint32_t a = 0; a < L.nassert; ++a)
      if (has(D, apos[a]))
        for (uint32_t w = 0; w < W; ++w) X[w] |= b[L.o_at + (a * 16 + k) * W + w];
  };
  size_t p = 0;
  while (p < n) {
    int w;
    const int32_t r = decode_rune(text + p, n - p, &w);
    uint32_t c;
    if (r < 0x80) c = a16[r];
    else {
      auto it = std::upper_bound(rx.nonascii.begin(), rx.nonascii.end(), std::make_pair(static_cast<uint32_t>(r), 0xFFFFFFFFu));
      c = std::prev(it)->second;
    }
    cross(ctx * 4 + cat[c]);
    if (has(X, match)) return true;
    for (uint32_t k = 0; k < W; ++k) Y[k] = X[k] & b[L.o_cm + c * W + k];
    for (uint32_t k = 0; k < W; ++k)
      D[k] = ((Y[k] & b[L.o_sh + k]) << 1) | (k ? (Y[k - 1] & b[L.o_sh + k - 1]) >> 63 : 0) | b[L.o_s0 + k];
    for (uint32_t g = 0; g < L.ngroups; ++g) {
      uint64_t any = 0;
      for (uint32_t k = 0; k < W; ++k) any |= Y[k] & b[L.o_gm + g * W + k];
      if (any)
        for (uint32_t k = 0; k < W; ++k) D[k] |= b[L.o_gt + g * W + k];
    }
    if (has(D, match)) return true;
    if ((flags & kNfaAnchored) && std::equal(D.begin(), D.end(), b + L.o_s0)) return false;
    ctx = cat[c] == 1 ? 1 : (cat[c] == 2 ? 2 : 0);
    p += static_cast<size_t>(w);
  }
  cross(ctx * 4 + 3);
  return has(X, match);
}

// the wide NFA (build_wide), stepped as k_nfa_wide does: the host copy of
// the device algorithm (compiler self-test and CPU tests)
static bool nfa_wide_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n) {
  const uint64_t *b = rx.nfa.data();
  const NfaWideLayout L = nfa_wide_layout_of(reinterpret_cast<const uint32_t *>(b));
  const uint32_t W = L.W, match = L.match;
  const uint16_t *a16 = reinterpret_cast<const uint16_t *>(b + L.o_ascii);
  const uint8_t *cat = reinterpret_cast<const uint8_t *>(b + L.o_cat);
  const uint32_t *aux = reinterpret_cast<const uint32_t *>(b + L.o_aux);
  const uint32_t *goff = reinterpret_cast<const uint32_t *>(b + L.o_goff), *gtgt = reinterpret_cast<const uint32_t *>(b + L.o_gtgt);
  const uint32_t *aoff = reinterpret_cast<const uint32_t *>(b + L.o_aoff), *atgt = reinterpret_cast<const uint32_t *>(b + L.o_atgt);
  auto has = [&](const std::vector<uint64_t> &v, uint32_t p) { return p != 0xFFFFFFFFu && ((v[p / 64] >> (p % 64)) & 1); };
  std::vector<uint64_t> A(b + L.o_s0, b + L.o_s0 + W), Y(W);
  auto cross = [&](uint32_t k) {  // A |= closures of the assertions A holds (targets hold no assertions)
    for (uint32_t w = 0; w < W; ++w)
      for (uint64_t m = A[w] & b[L.o_am + w]; m; m &= m - 1) {
        const uint32_t a = aux[w * 64 + __builtin_ctzll(m)];
        for (uint32_t i = aoff[a * 16 + k]; i < aoff[a * 16 + k + 1]; ++i) A[atgt[i] / 64] |= 1ull << (atgt[i] % 64);
      }
  };
  std::vector<uint8_t> gmark(L.ngroups, 0);
  uint32_t ctx = 3;
  size_t p = 0;
  while (p < n) {
    int w;
    const int32_t r = decode_rune(text + p, n - p, &w);
    uint32_t c;
    if (r < 0x80) c = a16[r];
    else {
      auto it = std::upper_bound(rx.nonascii.begin(), rx.nonascii.end(), std::make_pair(static_cast<uint32_t>(r), 0xFFFFFFFFu));
      c = std::prev(it)->second;
    }
    cross(ctx * 4 + cat[c]);
    if (has(A, match)) return true;
    for (uint32_t k = 0; k < W; ++k) {
      Y[k] = A[k] & b[L.o_cm + (uint64_t)c * W + k];
      for (uint64_t m = Y[k] & b[L.o_gall + k]; m; m &= m - 1) gmark[aux[k * 64 + __builtin_ctzll(m)]] = 1;
    }
    for (uint32_t k = 0; k < W; ++k)
      A[k] = ((Y[k] & b[L.o_sh + k]) << 1) | (k ? (Y[k - 1] & b[L.o_sh + k - 1]) >> 63 : 0) | b[L.o_s0 + k];
    for (uint32_t g = 0; g < L.ngroups; ++g) {
      if (!gmark[g]) continue;
      gmark[g] = 0;
      for (uint32_t i = goff[g]; i < goff[g + 1]; ++i) A[gtgt[i] / 64] |= 1ull << (gtgt[i] % 64);
    }
    if (has(A, match)) return true;
    ctx = cat[c] == 1 ? 1 : (cat[c] == 2 ? 2 : 0);
    p += static_cast<size_t>(w);
  }
  cross(ctx * 4 + 3);
  return has(A, match);
}

bool dfa_match_host(const CompiledRegex &rx, const uint8_t *text, size_t n) {
  if (rx.flags & kRuleNfaWide) return nfa_wide_match_host(rx, text, n);
  if (rx.flags & kRuleNfa) return nfa_match_host(rx, text, n);
  uint32_t st = rx.start;
  size_t p = 0;
  while (p < n && st > kAccept) {
    int w;
    int32_t r = decode_rune(text + p, n - p, &w);
    uint32_t c;
    if (r < 0x80) c = rx.ascii_cls[r];
    else {
      auto it = std::upper_bound(rx.nonascii.begin(), rx.nonascii.end(), std::make_pair(static_cast<uint32_t>(r), 0xFFFFFFFFu));
      c = std::prev(it)->second;
    }
    st = rx.trans[static_cast<size_t>(st) * rx.ncls + c];
    p += static_cast<size_t>(w);
  }
  return rx.accept_end[st] != 0;
}

}  // namespace bjx

// Test hook (banjax_gpu_debug.h): regexp/syntax's parse decision for one pattern
extern "C" int bjx_debug_regex_parse(const char *pat, size_t len, char *err, size_t err_len) {
  if (!pat && len) return BJX_ERR_ARG;
  std::string e;
  const int rc = bjx::parse_regex_only(std::string(pat ? pat : "", len), &e);
  if (err && err_len) {
    const size_t k = std::min(err_len - 1, e.size());
    memcpy(err, e.data(), k);
    err[k] = 0;
  }
  return rc;
}
