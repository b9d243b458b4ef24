// Go regexp/syntax's parse-size limits (Go 1.25.8, go.mod:3), restated for
// the rule compiler: ErrLarge ("expression too large") and ErrNestingDepth
// ("expression nests too deeply").  A config whose regex Go refuses this way
// fails to load (reference internal/config.go:110-113).
//
// Go checks the limits while it parses (parser.checkLimits after every push
// and repeat, and after factor() rewrites an alternation branch), on its own
// parse-tree shapes: literal runs merged into one node (maybeConcat), one-rune
// classes turned into literals, alternations flattened and factored, freed
// nodes reused from a free list.  Its size check only starts once (regexp
// nodes allocated) x (product of the repeat counts seen) reaches maxSize, and
// its height check once 1000 nodes were allocated; both then use caches of
// per-node results that Go keeps across later rewrites.  GoShape replays
// exactly those steps, driven by the compiler's own parser (regex_compiler.cpp
// Parser) event by event, so a pattern is refused at the same point of the
// parse, before or after the syntax errors Go would report first.
//
// Published algorithm restated: regexp/syntax parse.go (parser.push,
// maybeConcat, literal, op, parseClass's node, the escape node allocated and
// freed in parse, repeat, concat, alternate, collapse, factor,
// leadingString/removeLeadingString, leadingRegexp/removeLeadingRegexp,
// swapVerticalBar, parseRightParen, checkLimits, checkSize/calcSize,
// checkHeight/calcHeight, newRegexp/reuse) and regexp.go's Regexp.Equal,
// mergeCharClass, appendRange, appendFoldedRange, cleanClass, cleanAlt.
#pragma once
#include <algorithm>
#include <cstdint>
#include <memory>
#include <unordered_map>
#include <vector>

namespace gosh {

// Go's Op values: the order matters (swapVerticalBar and factor compare them)
enum GOp : int {
  gNoMatch = 1, gEmptyMatch, gLiteral, gCharClass, gAnyCharNotNL, gAnyChar, gBeginLine, gEndLine, gBeginText, gEndText,
  gWordBoundary, gNoWordBoundary, gCapture, gStar, gPlus, gQuest, gRepeat, gConcat, gAlternate,
  gPseudo = 128, gLeftParen, gVerticalBar
};
constexpr uint32_t fFold = 1, fNonGreedy = 32, fWasDollar = 256;  // Go's Flags bits used here
constexpr int64_t kMaxSize = (int64_t(128) << 20) / 40;  // maxSize: 128 MB of 40-byte Insts
constexpr int64_t kMaxRunes = (int64_t(128) << 20) / 4;  // maxRunes: 128 MB of runes
constexpr int kMaxHeight = 1000;
constexpr int32_t kMinFold = 0x0041, kMaxFold = 0x1e943, kMaxRuneG = 0x10FFFF;

struct GN {
  int op = 0;
  uint32_t flags = 0;
  std::vector<int32_t> r;  // Rune
  std::vector<GN *> sub;
  int min = 0, max = 0, cap = 0;
  GN *free_next = nullptr;
};

struct Limit {  // thrown: which limit
  bool large;
};

template <typename Fold>
class GoShape {
 public:
  explicit GoShape(Fold fold) : fold_(fold) {}

  // ---- events, in the order Go's parse loop would run them; flags = the
  // parser's current Go flags (fFold / fNonGreedy)
  void literal(int32_t c, uint32_t flags) {  // parser.literal
    GN *re = new_re(gLiteral);
    re->flags = flags;
    if (flags & fFold) c = min_fold_rune(c);
    re->r.assign(1, c);
    push(re, flags);
  }
  void op(int o, uint32_t flags, int cap = 0) {  // parser.op
    GN *re = new_re(o);
    re->flags = flags;
    re->cap = cap;
    push(re, flags);
    if (o == gEndText && (flags & fWasDollar)) re->flags |= fWasDollar;
  }
  // a bracketed class (parseClass: its node, the cleaned / negated ranges)
  template <typename R>
  void char_class(const R &ranges, uint32_t flags) {
    GN *re = new_re(gCharClass);
    re->flags = flags;
    for (auto &p : ranges) { re->r.push_back(p.first); re->r.push_back(p.second); }
    push(re, flags);
  }
  // parse's backslash case: a class node is allocated before the escape is
  // known; \p / Perl classes push it, other escapes put it back (reuse)
  void esc_alloc() { esc_ = new_re(gCharClass); }
  template <typename R>
  void esc_class(const R &ranges, uint32_t flags) {
    GN *re = esc_;
    esc_ = nullptr;
    re->flags = flags;
    for (auto &p : ranges) { re->r.push_back(p.first); re->r.push_back(p.second); }
    push(re, flags);
  }
  void esc_free() { reuse(esc_); esc_ = nullptr; }
  void vertical_bar(uint32_t flags) {  // parseVerticalBar
    concat(flags);
    if (!swap_vertical_bar()) op(gVerticalBar, flags);
  }
  // parseRightParen (the parser reports unbalanced parens itself)
  void right_paren(uint32_t flags) {
    concat(flags);
    if (swap_vertical_bar()) stack_.pop_back();
    alternate(flags);
    const size_t n = stack_.size();
    if (n < 2) return;
    GN *re1 = stack_[n - 1], *re2 = stack_[n - 2];
    if (re2->op != gLeftParen) return;
    stack_.resize(n - 2);
    const uint32_t fl = re2->flags;
    if (re2->cap == 0) push(re1, fl);
    else {
      re2->op = gCapture;
      re2->sub.assign(1, re1);
      push(re2, fl);
    }
  }
  // parser.repeat, after its argument checks and before repeatIsValid
  void repeat(int o, int mn, int mx, uint32_t flags) {
    if (stack_.empty()) return;
    GN *sub = stack_.back();
    GN *re = new_re(o);
    re->min = mn;
    re->max = mx;
    re->flags = flags;
    re->sub.assign(1, sub);
    stack_.back() = re;
    check_limits(re);
  }
  void end(uint32_t flags) {  // the end of parse
    concat(flags);
    if (swap_vertical_bar()) stack_.pop_back();
    alternate(flags);
  }

 private:
  Fold fold_;
  std::vector<std::unique_ptr<GN>> pool_;
  std::vector<GN *> stack_;
  GN *free_ = nullptr, *esc_ = nullptr;
  int64_t num_regexp_ = 0, num_runes_ = 0, repeats_ = 0;
  std::unique_ptr<std::unordered_map<GN *, int64_t>> size_;
  std::unique_ptr<std::unordered_map<GN *, int>> height_;

  GN *new_re(int o) {  // newRegexp
    GN *re = free_;
    if (re) {
      free_ = re->free_next;
      *re = GN();
    } else {
      pool_.emplace_back(new GN());
      re = pool_.back().get();
      ++num_regexp_;
    }
    re->op = o;
    return re;
  }
  void reuse(GN *re) {
    if (height_) height_->erase(re);
    re->free_next = free_;
    free_ = re;
  }

  int32_t min_fold_rune(int32_t r) const {
    if (r < kMinFold || r > kMaxFold) return r;
    int32_t m = r;
    const int32_t r0 = r;
    for (r = fold_(r); r != r0; r = fold_(r)) m = std::min(m, r);
    return m;
  }

  GN *push(GN *re, uint32_t flags) {
    num_runes_ += (int64_t)re->r.size();
    if (re->op == gCharClass && re->r.size() == 2 && re->r[0] == re->r[1]) {
      if (maybe_concat(re->r[0], flags & ~fFold)) return nullptr;
      re->op = gLiteral;
      re->r.resize(1);
      re->flags = flags & ~fFold;
    } else if ((re->op == gCharClass && re->r.size() == 4 && re->r[0] == re->r[1] && re->r[2] == re->r[3] &&
                fold_(re->r[0]) == re->r[2] && fold_(re->r[2]) == re->r[0]) ||
               (re->op == gCharClass && re->r.size() == 2 && re->r[0] + 1 == re->r[1] && fold_(re->r[0]) == re->r[1] &&
                fold_(re->r[1]) == re->r[0])) {
      if (maybe_concat(re->r[0], flags | fFold)) return nullptr;
      re->op = gLiteral;
      re->r.resize(1);
      re->flags = flags | fFold;
    } else {
      maybe_concat(-1, 0);
    }
    stack_.push_back(re);
    check_limits(re);
    return re;
  }
  bool maybe_concat(int32_t r, uint32_t flags) {
    const size_t n = stack_.size();
    if (n < 2) return false;
    GN *re1 = stack_[n - 1], *re2 = stack_[n - 2];
    if (re1->op != gLiteral || re2->op != gLiteral || (re1->flags & fFold) != (re2->flags & fFold)) return false;
    re2->r.insert(re2->r.end(), re1->r.begin(), re1->r.end());
    if (r >= 0) {
      re1->r.assign(1, r);
      re1->flags = flags;
      return true;
    }
    stack_.pop_back();
    reuse(re1);
    return false;
  }

  size_t top_items() const {
    size_t i = stack_.size();
    while (i > 0 && stack_[i - 1]->op < gPseudo) --i;
    return i;
  }
  void concat(uint32_t flags) {
    maybe_concat(-1, 0);
    const size_t i = top_items();
    std::vector<GN *> subs(stack_.begin() + i, stack_.end());
    stack_.resize(i);
    if (subs.empty()) {
      GN *re = new_re(gEmptyMatch);
      re->flags = flags;
      push(re, flags);
      return;
    }
    push(collapse(subs, gConcat), flags);
  }
  void alternate(uint32_t flags) {
    const size_t i = top_items();
    std::vector<GN *> subs(stack_.begin() + i, stack_.end());
    stack_.resize(i);
    if (!subs.empty()) clean_alt(subs.back());
    if (subs.empty()) {
      GN *re = new_re(gNoMatch);
      re->flags = flags;
      push(re, flags);
      return;
    }
    push(collapse(subs, gAlternate), flags);
  }
  GN *collapse(std::vector<GN *> subs, int o) {
    if (subs.size() == 1) return subs[0];
    GN *re = new_re(o);
    for (GN *s : subs) {
      if (s->op == o) {
        re->sub.insert(re->sub.end(), s->sub.begin(), s->sub.end());
        reuse(s);
      } else {
        re->sub.push_back(s);
      }
    }
    if (o == gAlternate) {
      re->sub = factor(re->sub);
      if (re->sub.size() == 1) {
        GN *old = re;
        re = re->sub[0];
        reuse(old);
      }
    }
    return re;
  }

  static bool is_char_class(const GN *re) {
    return (re->op == gLiteral && re->r.size() == 1) || re->op == gCharClass || re->op == gAnyCharNotNL ||
           re->op == gAnyChar;
  }
  static bool equal(const GN *x, const GN *y) {  // Regexp.Equal
    if (!x || !y) return x == y;
    if (x->op != y->op) return false;
    switch (x->op) {
      case gEndText:
        return (x->flags & fWasDollar) == (y->flags & fWasDollar);
      case gLiteral: case gCharClass:
        return x->r == y->r;
      case gAlternate: case gConcat:
        if (x->sub.size() != y->sub.size()) return false;
        for (size_t i = 0; i < x->sub.size(); ++i)
          if (!equal(x->sub[i], y->sub[i])) return false;
        return true;
      case gStar: case gPlus: case gQuest:
        return (x->flags & fNonGreedy) == (y->flags & fNonGreedy) && equal(x->sub[0], y->sub[0]);
      case gRepeat:
        return (x->flags & fNonGreedy) == (y->flags & fNonGreedy) && x->min == y->min && x->max == y->max &&
               equal(x->sub[0], y->sub[0]);
      case gCapture:
        return x->cap == y->cap && equal(x->sub[0], y->sub[0]);
      default:
        return true;
    }
  }

  // leadingString / removeLeadingString
  static const GN *lead_node(const GN *re) { return re->op == gConcat && !re->sub.empty() ? re->sub[0] : re; }
  GN *remove_leading_string(GN *re, size_t n) {
    if (re->op == gConcat && !re->sub.empty()) {
      GN *sub = remove_leading_string(re->sub[0], n);
      re->sub[0] = sub;
      if (sub->op == gEmptyMatch) {
        reuse(sub);
        switch (re->sub.size()) {
          case 0: case 1:
            re->op = gEmptyMatch;
            re->sub.clear();
            break;
          case 2: {
            GN *old = re;
            re = re->sub[1];
            reuse(old);
            break;
          }
          default:
            re->sub.erase(re->sub.begin());
        }
      }
      return re;
    }
    if (re->op == gLiteral) {
      re->r.erase(re->r.begin(), re->r.begin() + std::min(n, re->r.size()));
      if (re->r.empty()) re->op = gEmptyMatch;
    }
    return re;
  }
  static GN *leading_regexp(GN *re) {
    if (re->op == gEmptyMatch) return nullptr;
    if (re->op == gConcat && !re->sub.empty()) {
      GN *sub = re->sub[0];
      if (sub->op == gEmptyMatch) return nullptr;
      return sub;
    }
    return re;
  }
  GN *remove_leading_regexp(GN *re, bool reuse_it) {
    if (re->op == gConcat && !re->sub.empty()) {
      if (reuse_it) reuse(re->sub[0]);
      re->sub.erase(re->sub.begin());
      switch (re->sub.size()) {
        case 0:
          re->op = gEmptyMatch;
          re->sub.clear();
          break;
        case 1: {
          GN *old = re;
          re = re->sub[0];
          reuse(old);
          break;
        }
      }
      return re;
    }
    if (reuse_it) reuse(re);
    return new_re(gEmptyMatch);
  }

  std::vector<GN *> factor(std::vector<GN *> sub) {
    if (sub.size() < 2) return sub;
    // Round 1: common literal prefixes
    {
      std::vector<int32_t> str;
      uint32_t strflags = 0;
      size_t start = 0;
      std::vector<GN *> out;
      for (size_t i = 0; i <= sub.size(); ++i) {
        std::vector<int32_t> istr;
        uint32_t iflags = 0;
        if (i < sub.size()) {
          const GN *l = lead_node(sub[i]);
          if (l->op == gLiteral) { istr = l->r; iflags = l->flags & fFold; }
          if (iflags == strflags) {
            size_t same = 0;
            while (same < str.size() && same < istr.size() && str[same] == istr[same]) ++same;
            if (same > 0) {
              str.resize(same);
              continue;
            }
          }
        }
        if (i == start) {
        } else if (i == start + 1) {
          out.push_back(sub[start]);
        } else {
          GN *prefix = new_re(gLiteral);
          prefix->flags = strflags;
          prefix->r = str;
          for (size_t j = start; j < i; ++j) {
            sub[j] = remove_leading_string(sub[j], str.size());
            check_limits(sub[j]);
          }
          GN *suffix = collapse(std::vector<GN *>(sub.begin() + start, sub.begin() + i), gAlternate);
          GN *re = new_re(gConcat);
          re->sub = {prefix, suffix};
          out.push_back(re);
        }
        start = i;
        str = istr;
        strflags = iflags;
      }
      sub = out;
    }
    // Round 2: common leading regexp (a class, or a fixed repeat of one)
    {
      size_t start = 0;
      std::vector<GN *> out;
      GN *first = nullptr;
      for (size_t i = 0; i <= sub.size(); ++i) {
        GN *ifirst = nullptr;
        if (i < sub.size()) {
          ifirst = leading_regexp(sub[i]);
          if (first && equal(first, ifirst) &&
              (is_char_class(first) || (first->op == gRepeat && first->min == first->max && is_char_class(first->sub[0]))))
            continue;
        }
        if (i == start) {
        } else if (i == start + 1) {
          out.push_back(sub[start]);
        } else {
          GN *prefix = first;
          for (size_t j = start; j < i; ++j) {
            sub[j] = remove_leading_regexp(sub[j], j != start);
            check_limits(sub[j]);
          }
          GN *suffix = collapse(std::vector<GN *>(sub.begin() + start, sub.begin() + i), gAlternate);
          GN *re = new_re(gConcat);
          re->sub = {prefix, suffix};
          out.push_back(re);
        }
        start = i;
        first = ifirst;
      }
      sub = out;
    }
    // Round 3: runs of single literals / classes into one class
    {
      size_t start = 0;
      std::vector<GN *> out;
      for (size_t i = 0; i <= sub.size(); ++i) {
        if (i < sub.size() && is_char_class(sub[i])) continue;
        if (i == start) {
        } else if (i == start + 1) {
          out.push_back(sub[start]);
        } else {
          size_t mx = start;
          for (size_t j = start + 1; j < i; ++j)
            if (sub[mx]->op < sub[j]->op || (sub[mx]->op == sub[j]->op && sub[mx]->r.size() < sub[j]->r.size())) mx = j;
          std::swap(sub[start], sub[mx]);
          for (size_t j = start + 1; j < i; ++j) {
            merge_char_class(sub[start], sub[j]);
            reuse(sub[j]);
          }
          clean_alt(sub[start]);
          out.push_back(sub[start]);
        }
        if (i < sub.size()) out.push_back(sub[i]);
        start = i + 1;
      }
      sub = out;
    }
    // Round 4: runs of empty matches
    {
      std::vector<GN *> out;
      for (size_t i = 0; i < sub.size(); ++i) {
        if (i + 1 < sub.size() && sub[i]->op == gEmptyMatch && sub[i + 1]->op == gEmptyMatch) continue;
        out.push_back(sub[i]);
      }
      sub = out;
    }
    return sub;
  }

  bool swap_vertical_bar() {
    const size_t n = stack_.size();
    if (n >= 3 && stack_[n - 2]->op == gVerticalBar && is_char_class(stack_[n - 1]) && is_char_class(stack_[n - 3])) {
      GN *re1 = stack_[n - 1], *re3 = stack_[n - 3];
      if (re1->op > re3->op) {
        std::swap(re1, re3);
        stack_[n - 3] = re3;
      }
      merge_char_class(re3, re1);
      reuse(re1);
      stack_.pop_back();
      return true;
    }
    if (n >= 2) {
      GN *re1 = stack_[n - 1], *re2 = stack_[n - 2];
      if (re2->op == gVerticalBar) {
        if (n >= 3) clean_alt(stack_[n - 3]);
        stack_[n - 2] = re1;
        stack_[n - 1] = re2;
        return true;
      }
    }
    return false;
  }

  // ---- character-class arithmetic on Go's flat rune pairs
  static void append_range(std::vector<int32_t> &r, int32_t lo, int32_t hi) {
    const size_t n = r.size();
    for (size_t i = 2; i <= 4; i += 2) {
      if (n >= i) {
        const int32_t rlo = r[n - i], rhi = r[n - i + 1];
        if (lo <= rhi + 1 && rlo <= hi + 1) {
          if (lo < rlo) r[n - i] = lo;
          if (hi > rhi) r[n - i + 1] = hi;
          return;
        }
      }
    }
    r.push_back(lo);
    r.push_back(hi);
  }
  void append_folded_range(std::vector<int32_t> &r, int32_t lo, int32_t hi) const {
    if ((lo <= kMinFold && hi >= kMaxFold) || hi < kMinFold || lo > kMaxFold) { append_range(r, lo, hi); return; }
    if (lo < kMinFold) { append_range(r, lo, kMinFold - 1); lo = kMinFold; }
    if (hi > kMaxFold) { append_range(r, kMaxFold + 1, hi); hi = kMaxFold; }
    for (int32_t c = lo; c <= hi; ++c) {
      append_range(r, c, c);
      for (int32_t f = fold_(c); f != c; f = fold_(f)) append_range(r, f, f);
    }
  }
  void append_literal(std::vector<int32_t> &r, int32_t x, uint32_t flags) const {
    if (flags & fFold) append_folded_range(r, x, x);
    else append_range(r, x, x);
  }
  static bool match_rune(const GN *re, int32_t c) {
    switch (re->op) {
      case gLiteral: return re->r.size() == 1 && re->r[0] == c;  // (the fold case does not arise for '\n')
      case gCharClass:
        for (size_t i = 0; i + 1 < re->r.size(); i += 2)
          if (re->r[i] <= c && c <= re->r[i + 1]) return true;
        return false;
      case gAnyCharNotNL: return c != '\n';
      case gAnyChar: return true;
    }
    return false;
  }
  void merge_char_class(GN *dst, const GN *src) const {
    switch (dst->op) {
      case gAnyChar: break;
      case gAnyCharNotNL:
        if (match_rune(src, '\n')) dst->op = gAnyChar;
        break;
      case gCharClass:
        if (src->op == gLiteral) append_literal(dst->r, src->r[0], src->flags);
        else
          for (size_t i = 0; i + 1 < src->r.size(); i += 2) append_range(dst->r, src->r[i], src->r[i + 1]);
        break;
      case gLiteral:
        if (src->r[0] == dst->r[0] && src->flags == dst->flags) break;
        {
          const int32_t d0 = dst->r[0];
          dst->op = gCharClass;
          dst->r.clear();
          append_literal(dst->r, d0, dst->flags);
          append_literal(dst->r, src->r[0], src->flags);
        }
        break;
    }
  }
  static void clean_class(std::vector<int32_t> &r) {
    std::vector<std::pair<int32_t, int32_t>> p;
    for (size_t i = 0; i + 1 < r.size(); i += 2) p.push_back({r[i], r[i + 1]});
    std::sort(p.begin(), p.end(), [](const std::pair<int32_t, int32_t> &a, const std::pair<int32_t, int32_t> &b) {
      return a.first != b.first ? a.first < b.first : a.second > b.second;
    });
    r.clear();
    for (auto &q : p) {
      if (!r.empty() && q.first <= r.back() + 1) {
        if (q.second > r.back()) r.back() = q.second;
        continue;
      }
      r.push_back(q.first);
      r.push_back(q.second);
    }
  }
  static void clean_alt(GN *re) {
    if (re->op != gCharClass) return;
    clean_class(re->r);
    if (re->r.size() == 2 && re->r[0] == 0 && re->r[1] == kMaxRuneG) { re->r.clear(); re->op = gAnyChar; return; }
    if (re->r.size() == 4 && re->r[0] == 0 && re->r[1] == '\n' - 1 && re->r[2] == '\n' + 1 && re->r[3] == kMaxRuneG) {
      re->r.clear();
      re->op = gAnyCharNotNL;
    }
  }

  // ---- checkLimits
  void check_limits(GN *re) {
    if (num_runes_ > kMaxRunes) throw Limit{true};
    check_size(re);
    check_height(re);
  }
  void check_size(GN *re) {
    if (!size_) {
      if (repeats_ == 0) repeats_ = 1;
      if (re->op == gRepeat) {
        int64_t n = re->max;
        if (n == -1) n = re->min;
        if (n <= 0) n = 1;
        if (n > kMaxSize / repeats_) repeats_ = kMaxSize;
        else repeats_ *= n;
      }
      if (num_regexp_ < kMaxSize / repeats_) return;
      size_.reset(new std::unordered_map<GN *, int64_t>());
      for (size_t i = 0; i < stack_.size(); ++i) check_size(stack_[i]);
    }
    if (calc_size(re, true) > kMaxSize) throw Limit{true};
  }
  int64_t calc_size(GN *re, bool force) {
    if (!force) {
      auto it = size_->find(re);
      if (it != size_->end()) return it->second;
    }
    int64_t size = 0;
    switch (re->op) {
      case gLiteral: size = (int64_t)re->r.size(); break;
      case gCapture: case gStar: size = 2 + calc_size(re->sub[0], false); break;
      case gPlus: case gQuest: size = 1 + calc_size(re->sub[0], false); break;
      case gConcat:
        for (GN *s : re->sub) size += calc_size(s, false);
        break;
      case gAlternate:
        for (GN *s : re->sub) size += calc_size(s, false);
        if (re->sub.size() > 1) size += (int64_t)re->sub.size() - 1;
        break;
      case gRepeat: {
        const int64_t sub = calc_size(re->sub[0], false);
        if (re->max == -1) {
          size = re->min == 0 ? 2 + sub : 1 + (int64_t)re->min * sub;
          break;
        }
        size = (int64_t)re->max * sub + (int64_t)(re->max - re->min);
        break;
      }
      default: break;
    }
    size = std::max<int64_t>(1, size);
    (*size_)[re] = size;
    return size;
  }
  void check_height(GN *re) {
    if (num_regexp_ < kMaxHeight) return;
    if (!height_) {
      height_.reset(new std::unordered_map<GN *, int>());
      for (size_t i = 0; i < stack_.size(); ++i) check_height(stack_[i]);
    }
    if (calc_height(re, true) > kMaxHeight) throw Limit{false};
  }
  int calc_height(GN *re, bool force) {
    if (!force) {
      auto it = height_->find(re);
      if (it != height_->end()) return it->second;
    }
    int h = 1;
    for (GN *s : re->sub) h = std::max(h, 1 + calc_height(s, false));
    (*height_)[re] = h;
    return h;
  }
};

}  // namespace gosh
