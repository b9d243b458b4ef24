/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into the product library.
 *
 * CPU restatement of Go 1.25 `regexp` (stdlib, not vendored in /root/reference)
 * as used by the banjax hot path:
 *   compile: reference internal/config.go:110  `regexp.Compile(i.Regex)`
 *   match:   reference internal/regex_rate_limiter.go:234 `Regex.Match([]byte(rest))`
 * regexp.Compile parses with syntax.Perl = ClassNL|OneLine|PerlX|UnicodeGroups.
 * The parser below follows the published regexp/syntax algorithm (a stack of
 * regexps with '(' and '|' pseudo-markers, so that accept/reject decisions and
 * error codes come out as Go's do); matching is a rune-level Pike VM using Go's
 * UTF-8 decoding (invalid byte -> U+FFFD, width 1) and EmptyOpContext for the
 * empty-width assertions.  Boolean Match only (no submatches), which is all the
 * hot path asks for.
 *
 * UnicodeGroups (\pL, \p{Greek}, \P{..}, \p{^..}) follow parse.go's
 * parseUnicodeClass / unicodeTable of Go 1.25 over the Unicode 15.0.0 tables of
 * third_party/unicode/unicode_tables.h (tools/gen_unicode_tables.py).
 * Go's ErrLarge / ErrNestingDepth parse limits are replayed on Go's own parse
 * shapes by go_limits.c, event by event as the parser below runs.
 */
#include "go_regexp.h"
#include "go_limits.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../third_party/unicode/fold_orbits.h"
#include "../third_party/unicode/unicode_tables.h"

#define MAX_RUNE 0x10FFFF
#define RUNE_ERROR 0xFFFD

/* ------------------------------------------------------------------ utf-8 */

/* Go unicode/utf8.DecodeRune semantics. */
static int decode_rune(const uint8_t *s, size_t n, int *width) {
  if (n == 0) { *width = 0; return -1; }
  uint8_t b0 = s[0];
  if (b0 < 0x80) { *width = 1; return b0; }
  int need; uint8_t lo = 0x80, hi = 0xBF; int r;
  if (b0 >= 0xC2 && b0 <= 0xDF) { need = 1; r = b0 & 0x1F; }
  else if (b0 == 0xE0) { need = 2; lo = 0xA0; r = b0 & 0x0F; }
  else if ((b0 >= 0xE1 && b0 <= 0xEC) || b0 == 0xEE || b0 == 0xEF) { need = 2; r = b0 & 0x0F; }
  else if (b0 == 0xED) { need = 2; hi = 0x9F; r = b0 & 0x0F; }
  else if (b0 == 0xF0) { need = 3; lo = 0x90; r = b0 & 0x07; }
  else if (b0 >= 0xF1 && b0 <= 0xF3) { need = 3; r = b0 & 0x07; }
  else if (b0 == 0xF4) { need = 3; hi = 0x8F; r = b0 & 0x07; }
  else { *width = 1; return RUNE_ERROR; }
  if (n < (size_t)need + 1) { *width = 1; return RUNE_ERROR; }
  uint8_t b1 = s[1];
  if (b1 < lo || b1 > hi) { *width = 1; return RUNE_ERROR; }
  r = (r << 6) | (b1 & 0x3F);
  for (int k = 2; k <= need; k++) {
    uint8_t b = s[k];
    if (b < 0x80 || b > 0xBF) { *width = 1; return RUNE_ERROR; }
    r = (r << 6) | (b & 0x3F);
  }
  *width = need + 1;
  return r;
}

/* ------------------------------------------------------------ simple fold */

static int simple_fold(int r) {
  int lo = 0, hi = BJX_FOLD_N;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if ((int)bjx_fold_from[m] < r) lo = m + 1; else hi = m;
  }
  if (lo < BJX_FOLD_N && (int)bjx_fold_from[lo] == r) return (int)bjx_fold_to[lo];
  return r;
}

/* ----------------------------------------------------------- rune classes */

typedef struct { int *r; int n, cap; } RV; /* pairs lo,hi */

static void rv_push(RV *v, int lo, int hi) {
  if (v->n + 2 > v->cap) { v->cap = v->cap ? v->cap * 2 : 16; v->r = realloc(v->r, sizeof(int) * v->cap); }
  v->r[v->n++] = lo; v->r[v->n++] = hi;
}
static int cmp_pair(const void *a, const void *b) {
  const int *x = a, *y = b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] < y[1] ? -1 : (x[1] > y[1]);
}
/* sort + merge adjacent/overlapping (Go cleanClass). */
static void rv_clean(RV *v) {
  if (v->n <= 2) return;
  qsort(v->r, v->n / 2, sizeof(int) * 2, cmp_pair);
  int w = 2;
  for (int i = 2; i < v->n; i += 2) {
    int lo = v->r[i], hi = v->r[i + 1];
    if (lo <= v->r[w - 1] + 1) { if (hi > v->r[w - 1]) v->r[w - 1] = hi; continue; }
    v->r[w] = lo; v->r[w + 1] = hi; w += 2;
  }
  v->n = w;
}
static void rv_negate(RV *v) { /* assumes clean */
  RV o = {0};
  int next = 0;
  for (int i = 0; i < v->n; i += 2) {
    if (v->r[i] > next) rv_push(&o, next, v->r[i] - 1);
    next = v->r[i + 1] + 1;
  }
  if (next <= MAX_RUNE) rv_push(&o, next, MAX_RUNE);
  free(v->r); *v = o;
}
#define MIN_FOLD 0x41
static void rv_push_folded(RV *v, int lo, int hi) {
  int max_fold = (int)bjx_fold_from[BJX_FOLD_N - 1];
  if (lo <= MIN_FOLD && hi >= max_fold) { rv_push(v, lo, hi); return; }
  if (hi < MIN_FOLD || lo > max_fold) { rv_push(v, lo, hi); return; }
  if (lo < MIN_FOLD) { rv_push(v, lo, MIN_FOLD - 1); lo = MIN_FOLD; }
  if (hi > max_fold) { rv_push(v, max_fold + 1, hi); hi = max_fold; }
  for (int c = lo; c <= hi; c++) {
    rv_push(v, c, c);
    for (int f = simple_fold(c); f != c; f = simple_fold(f)) rv_push(v, f, f);
  }
}

/* ---------------------------------------------------------------- the AST */

enum {
  OP_NOMATCH = 1, OP_EMPTY, OP_LIT, OP_CLASS, OP_ANYNL, OP_ANY,
  OP_BOL, OP_EOL, OP_BOT, OP_EOT, OP_WB, OP_NWB,
  OP_CAP, OP_STAR, OP_PLUS, OP_QUEST, OP_REPEAT, OP_CONCAT, OP_ALT,
  OP_PSEUDO = 128, OP_LPAREN, OP_VBAR
};
/* parse flags, Go regexp/syntax values are irrelevant; names kept */
enum { F_FOLD = 1, F_CLASSNL = 4, F_DOTNL = 8, F_ONELINE = 16, F_NONGREEDY = 32, F_PERLX = 64 };

typedef struct Node {
  int op, flags, min, max, cap;
  int rune;
  RV cls;
  struct Node **sub; int nsub, capsub;
} Node;

static Node *node_new(int op, int flags) {
  Node *n = calloc(1, sizeof(Node));
  n->op = op; n->flags = flags;
  return n;
}
static void node_add(Node *n, Node *s) {
  if (n->nsub == n->capsub) { n->capsub = n->capsub ? n->capsub * 2 : 4; n->sub = realloc(n->sub, sizeof(Node *) * n->capsub); }
  n->sub[n->nsub++] = s;
}
static void node_free(Node *n) {
  if (!n) return;
  for (int i = 0; i < n->nsub; i++) node_free(n->sub[i]);
  free(n->sub); free(n->cls.r); free(n);
}

/* --------------------------------------------------------------- parser */

typedef struct {
  const char *whole; size_t wlen;
  int flags;
  Node **st; int nst, cst;
  int ncap;
  char *err; size_t errlen;
  int failed;
  GoLim *gl;  /* Go's size / nesting limits (go_limits.c) */
} P;

static const char *E_INVALID_CHAR_CLASS = "invalid character class";
static const char *E_INVALID_CHAR_RANGE = "invalid character class range";
static const char *E_INVALID_ESCAPE = "invalid escape sequence";
static const char *E_INVALID_NAMED_CAPTURE = "invalid named capture";
static const char *E_INVALID_PERL_OP = "invalid or unsupported Perl syntax";
static const char *E_INVALID_REPEAT_OP = "invalid nested repetition operator";
static const char *E_INVALID_REPEAT_SIZE = "invalid repeat count";
static const char *E_INVALID_UTF8 = "invalid UTF-8";
static const char *E_MISSING_BRACKET = "missing closing ]";
static const char *E_MISSING_PAREN = "missing closing )";
static const char *E_MISSING_REPEAT_ARG = "missing argument to repetition operator";
static const char *E_TRAILING_BACKSLASH = "trailing backslash at end of expression";
static const char *E_UNEXPECTED_PAREN = "unexpected )";
static const char *E_NESTING_DEPTH = "expression nests too deeply";
static const char *E_LARGE = "expression too large";

/* Go: "error parsing regexp: " + code + ": `" + expr + "`" */
static void fail(P *p, const char *code, const char *expr, size_t elen) {
  if (p->failed) return;
  p->failed = 1;
  if (p->err && p->errlen) {
    char buf[64];
    size_t show = elen;
    int n = snprintf(p->err, p->errlen, "error parsing regexp: %s: `", code);
    if (n < 0) return;
    size_t room = p->errlen > (size_t)n + 2 ? p->errlen - (size_t)n - 2 : 0;
    if (show > room) show = room;
    memcpy(p->err + n, expr, show);
    p->err[n + show] = 0;
    strncat(p->err, "`", p->errlen - strlen(p->err) - 1);
    (void)buf;
  }
}

/* Go flags of the current position for go_limits.c (FoldCase, NonGreedy) */
static unsigned gfl(const P *p) { return (unsigned)(p->flags & (F_FOLD | F_NONGREEDY)); }
/* a limit crossed at this point of the parse becomes the parse error */
static int lim_check(P *p) {
  const int f = p->gl ? golim_failed(p->gl) : 0;
  if (f && !p->failed) fail(p, f == 1 ? E_LARGE : E_NESTING_DEPTH, p->whole, p->wlen);
  return p->failed;
}

/* nextRune: decode one rune of the pattern; invalid UTF-8 is an error. */
static int next_rune(P *p, const char *t, size_t tl, int *w) {
  int width;
  int c = decode_rune((const uint8_t *)t, tl, &width);
  if (tl == 0) { *w = 0; return RUNE_ERROR; }
  if (c == RUNE_ERROR && width == 1) {
    /* Go returns ErrInvalidUTF8 with Expr = rest of string */
    fail(p, E_INVALID_UTF8, t, tl);
    *w = 1; return -1;
  }
  *w = width; return c;
}

static void push(P *p, Node *n) {
  if (p->nst == p->cst) { p->cst = p->cst ? p->cst * 2 : 16; p->st = realloc(p->st, sizeof(Node *) * p->cst); }
  p->st[p->nst++] = n;
}
static void op_push(P *p, int op) {
  golim_op(p->gl, op, gfl(p), 0);
  push(p, node_new(op, p->flags));
}

static void literal(P *p, int r) {
  golim_literal(p->gl, r, gfl(p));
  Node *n = node_new(OP_LIT, p->flags);
  n->rune = r;
  push(p, n);
}

/* concat: replace the items above the topmost pseudo with their concatenation. */
static void concat(P *p) {
  int i = p->nst;
  while (i > 0 && p->st[i - 1]->op < OP_PSEUDO) i--;
  int cnt = p->nst - i;
  Node *n;
  if (cnt == 0) n = node_new(OP_EMPTY, p->flags);
  else if (cnt == 1) n = p->st[i];
  else { n = node_new(OP_CONCAT, p->flags); for (int k = i; k < p->nst; k++) node_add(n, p->st[k]); }
  p->nst = i;
  push(p, n);
}
static void alternate(P *p) {
  int i = p->nst;
  while (i > 0 && p->st[i - 1]->op < OP_PSEUDO) i--;
  int cnt = p->nst - i;
  Node *n;
  if (cnt == 0) n = node_new(OP_NOMATCH, p->flags);
  else if (cnt == 1) n = p->st[i];
  else { n = node_new(OP_ALT, p->flags); for (int k = i; k < p->nst; k++) node_add(n, p->st[k]); }
  p->nst = i;
  push(p, n);
}
/* swapVerticalBar: [.. VBAR x] -> [.. x VBAR]; everything below the VBAR
   (down to the '(' marker) is a finished alternative.  Returns whether it swapped. */
static int swap_vbar(P *p) {
  int n = p->nst;
  if (n >= 2 && p->st[n - 2]->op == OP_VBAR) {
    Node *tmp = p->st[n - 1];
    p->st[n - 1] = p->st[n - 2];
    p->st[n - 2] = tmp;
    return 1;
  }
  return 0;
}
static void pop_free(P *p) { node_free(p->st[--p->nst]); }

/* repeatIsValid(re, n) from regexp/syntax/parse.go */
static int repeat_valid(Node *re, int n) {
  if (re->op == OP_REPEAT) {
    int m = re->max;
    if (m == 0) return 1;
    if (m < 0) m = re->min;
    if (m > n) return 0;
    if (m > 0) n /= m;
  }
  for (int i = 0; i < re->nsub; i++)
    if (!repeat_valid(re->sub[i], n)) return 0;
  return 1;
}

/* p.repeat: before = text at the operator, after = text following it. */
static const char *do_repeat(P *p, int op, int min, int max, const char *before, const char *after,
                             const char *end, const char *last_repeat) {
  int flags = p->flags;
  if (after < end && *after == '?') { after++; flags ^= F_NONGREEDY; }
  if (last_repeat) { fail(p, E_INVALID_REPEAT_OP, last_repeat, (size_t)(after - last_repeat)); return NULL; }
  if (p->nst == 0 || p->st[p->nst - 1]->op >= OP_PSEUDO) {
    fail(p, E_MISSING_REPEAT_ARG, before, (size_t)(after - before));
    return NULL;
  }
  Node *n = node_new(op, flags);
  n->min = min; n->max = max;
  node_add(n, p->st[p->nst - 1]);
  p->st[p->nst - 1] = n;
  golim_repeat(p->gl, op, min, max, (unsigned)(flags & (F_FOLD | F_NONGREEDY)));
  if (lim_check(p)) return NULL;
  if (op == OP_REPEAT && (min >= 2 || max >= 2) && !repeat_valid(n, 1000)) {
    fail(p, E_INVALID_REPEAT_SIZE, before, (size_t)(after - before));
    return NULL;
  }
  return after;
}

/* parseInt from parse.go: no leading zeros; values >= 1e8 become -1. */
static int parse_int(const char **s, const char *end, int *out) {
  const char *t = *s;
  if (t >= end || *t < '0' || *t > '9') return 0;
  if (end - t >= 2 && t[0] == '0' && t[1] >= '0' && t[1] <= '9') return 0;
  const char *q = t;
  while (q < end && *q >= '0' && *q <= '9') q++;
  int n = 0;
  for (const char *c = t; c < q; c++) {
    if (n >= 100000000) { n = -1; break; }
    n = n * 10 + (*c - '0');
  }
  *out = n; *s = q;
  return 1;
}
static int parse_repeat(const char *s, const char *end, int *min, int *max, const char **rest) {
  if (s >= end || *s != '{') return 0;
  s++;
  if (!parse_int(&s, end, min)) return 0;
  if (s >= end) return 0;
  if (*s != ',') *max = *min;
  else {
    s++;
    if (s >= end) return 0;
    if (*s == '}') *max = -1;
    else if (!parse_int(&s, end, max)) return 0;
    else if (*max < 0) *min = -1;
  }
  if (s >= end || *s != '}') return 0;
  *rest = s + 1;
  return 1;
}

static int is_alnum(int c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
static int unhex(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

/* parseEscape: s points at '\'.  Returns rune, advances *rest. */
static int parse_escape(P *p, const char *s, const char *end, const char **rest) {
  const char *t = s + 1;
  if (t >= end) { fail(p, E_TRAILING_BACKSLASH, "", 0); return -1; }
  int w;
  int c = next_rune(p, t, (size_t)(end - t), &w);
  if (p->failed) return -1;
  t += w;
  switch (c) {
  case '1': case '2': case '3': case '4': case '5': case '6': case '7':
    if (t >= end || *t < '0' || *t > '7') break;
    /* fallthrough */
  case '0': {
    int r = c - '0';
    for (int i = 1; i < 3; i++) {
      if (t >= end || *t < '0' || *t > '7') break;
      r = r * 8 + (*t - '0'); t++;
    }
    *rest = t; return r;
  }
  case 'x': {
    if (t >= end) break;
    c = next_rune(p, t, (size_t)(end - t), &w);
    if (p->failed) return -1;
    t += w;
    if (c == '{') {
      int nhex = 0; long r = 0;
      for (;;) {
        if (t >= end) goto bad;
        c = next_rune(p, t, (size_t)(end - t), &w);
        if (p->failed) return -1;
        t += w;
        if (c == '}') break;
        int v = unhex(c);
        if (v < 0) goto bad;
        r = r * 16 + v;
        if (r > MAX_RUNE) goto bad;
        nhex++;
      }
      if (nhex == 0) goto bad;
      *rest = t; return (int)r;
    }
    int x = unhex(c);
    int y;
    if (t >= end) { y = -1; }
    else {
      c = next_rune(p, t, (size_t)(end - t), &w);
      if (p->failed) return -1;
      t += w; y = unhex(c);
    }
    if (x < 0 || y < 0) break;
    *rest = t; return x * 16 + y;
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
  fail(p, E_INVALID_ESCAPE, s, (size_t)(t - s));
  return -1;
}

/* Perl groups \d \s \w and POSIX classes (ASCII tables of regexp/syntax/perl_groups.go) */
typedef struct { const char *name; int sign; const int *cls; int n; } Group;
static const int cls_d[] = {'0', '9'};
static const int cls_s[] = {'\t', '\n', '\f', '\f', '\r', '\r', ' ', ' '};
static const int cls_w[] = {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'};
static const Group perl_groups[] = {
  {"\\d", 1, cls_d, 2}, {"\\D", -1, cls_d, 2}, {"\\s", 1, cls_s, 8}, {"\\S", -1, cls_s, 8},
  {"\\w", 1, cls_w, 8}, {"\\W", -1, cls_w, 8},
};
static const int c_alnum[] = {'0', '9', 'A', 'Z', 'a', 'z'};
static const int c_alpha[] = {'A', 'Z', 'a', 'z'};
static const int c_ascii[] = {0, 0x7F};
static const int c_blank[] = {'\t', '\t', ' ', ' '};
static const int c_cntrl[] = {0, 0x1F, 0x7F, 0x7F};
static const int c_digit[] = {'0', '9'};
static const int c_graph[] = {'!', '~'};
static const int c_lower[] = {'a', 'z'};
static const int c_print[] = {' ', '~'};
static const int c_punct[] = {'!', '/', ':', '@', '[', '`', '{', '~'};
static const int c_space[] = {'\t', '\r', ' ', ' '};
static const int c_upper[] = {'A', 'Z'};
static const int c_word[] = {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'};
static const int c_xdigit[] = {'0', '9', 'A', 'F', 'a', 'f'};
static const Group posix_groups[] = {
  {"[:alnum:]", 1, c_alnum, 6}, {"[:^alnum:]", -1, c_alnum, 6},
  {"[:alpha:]", 1, c_alpha, 4}, {"[:^alpha:]", -1, c_alpha, 4},
  {"[:ascii:]", 1, c_ascii, 2}, {"[:^ascii:]", -1, c_ascii, 2},
  {"[:blank:]", 1, c_blank, 4}, {"[:^blank:]", -1, c_blank, 4},
  {"[:cntrl:]", 1, c_cntrl, 4}, {"[:^cntrl:]", -1, c_cntrl, 4},
  {"[:digit:]", 1, c_digit, 2}, {"[:^digit:]", -1, c_digit, 2},
  {"[:graph:]", 1, c_graph, 2}, {"[:^graph:]", -1, c_graph, 2},
  {"[:lower:]", 1, c_lower, 2}, {"[:^lower:]", -1, c_lower, 2},
  {"[:print:]", 1, c_print, 2}, {"[:^print:]", -1, c_print, 2},
  {"[:punct:]", 1, c_punct, 8}, {"[:^punct:]", -1, c_punct, 8},
  {"[:space:]", 1, c_space, 4}, {"[:^space:]", -1, c_space, 4},
  {"[:upper:]", 1, c_upper, 2}, {"[:^upper:]", -1, c_upper, 2},
  {"[:word:]", 1, c_word, 8}, {"[:^word:]", -1, c_word, 8},
  {"[:xdigit:]", 1, c_xdigit, 6}, {"[:^xdigit:]", -1, c_xdigit, 6},
};

/* appendGroup: add (possibly folded, possibly negated) group to class. */
static void append_group(P *p, RV *cls, const Group *g) {
  RV tmp = {0};
  for (int i = 0; i < g->n; i += 2) {
    if (p->flags & F_FOLD) rv_push_folded(&tmp, g->cls[i], g->cls[i + 1]);
    else rv_push(&tmp, g->cls[i], g->cls[i + 1]);
  }
  rv_clean(&tmp);
  if (g->sign < 0) rv_negate(&tmp);
  for (int i = 0; i < tmp.n; i += 2) rv_push(cls, tmp.r[i], tmp.r[i + 1]);
  free(tmp.r);
}

static const Group *perl_class_escape(P *p, const char *s, const char *end) {
  if (!(p->flags & F_PERLX) || end - s < 2 || s[0] != '\\') return NULL;
  for (size_t i = 0; i < sizeof(perl_groups) / sizeof(perl_groups[0]); i++)
    if (perl_groups[i].name[1] == s[1]) return &perl_groups[i];
  return NULL;
}

/* unicodeTable (regexp/syntax, Go 1.25): exact names first ("Any", the
   categories incl. LC and Cn, the scripts), then canonicalName matching
   (case-insensitive, '_' '-' ' ' ignored) of "Any", "Assigned" (inverted Cn),
   "ASCII", the table names and unicode.CategoryAliases. */
static void canon(const char *s, size_t n, char *out, size_t cap) {
  size_t k = 0; int first = 1;
  for (size_t i = 0; i < n && k + 1 < cap; i++) {
    char c = s[i];
    if (c == '_' || c == '-' || c == ' ') continue;
    if (first) { if (c >= 'a' && c <= 'z') c = (char)(c - 32); first = 0; }
    else if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
    out[k++] = c;
  }
  out[k] = 0;
}
static int table_by_name(const char *name, size_t n, int loose) {
  char a[128], b[128];
  if (n >= sizeof a) return -1;
  if (loose) canon(name, n, a, sizeof a); else { memcpy(a, name, n); a[n] = 0; }
  for (int i = 0; i < BJX_UNI_NTABLES; i++) {
    const char *t = bjx_uni_tables[i].name;
    if (loose) canon(t, strlen(t), b, sizeof b); else snprintf(b, sizeof b, "%s", t);
    if (strcmp(a, b) == 0) return i;
  }
  return -1;
}
static void push_table(RV *v, int i) {
  const bjx_uni_table *t = &bjx_uni_tables[i];
  for (uint32_t k = 0; k < t->n; k++) rv_push(v, (int)bjx_uni_ranges[2 * (t->off + k)], (int)bjx_uni_ranges[2 * (t->off + k) + 1]);
}
/* 1 if known (runes appended to v, *sign = -1 when to be inverted) */
static int unicode_table(const char *name, size_t n, RV *v, int *sign) {
  char c[128];
  *sign = 1;
  if (n == 3 && memcmp(name, "Any", 3) == 0) { rv_push(v, 0, MAX_RUNE); return 1; }
  int i = table_by_name(name, n, 0);
  if (i >= 0) { push_table(v, i); return 1; }
  if (n >= sizeof c) return 0;
  canon(name, n, c, sizeof c);
  if (strcmp(c, "Any") == 0) { rv_push(v, 0, MAX_RUNE); return 1; }
  if (strcmp(c, "Assigned") == 0) { push_table(v, table_by_name("Cn", 2, 0)); *sign = -1; return 1; }
  if (strcmp(c, "Ascii") == 0) { rv_push(v, 0, 0x7F); return 1; }
  i = table_by_name(name, n, 1);
  if (i >= 0) { push_table(v, i); return 1; }
  for (int k = 0; k < BJX_UNI_NALIASES; k++) {
    char a[128];
    canon(bjx_uni_cat_aliases[2 * k], strlen(bjx_uni_cat_aliases[2 * k]), a, sizeof a);
    if (strcmp(a, c) == 0) {
      const char *tn = bjx_uni_cat_aliases[2 * k + 1];
      push_table(v, table_by_name(tn, strlen(tn), 0));
      return 1;
    }
  }
  return 0;
}

/* parseUnicodeClass: s at "\p" / "\P".  Returns the text after the group with
   its runes appended to cls, s itself if s is not a Unicode group, NULL on error. */
static const char *parse_unicode_class(P *p, const char *s, const char *end, RV *cls) {
  if (end - s < 2 || s[0] != '\\' || (s[1] != 'p' && s[1] != 'P')) return s;
  int sign = s[1] == 'P' ? -1 : 1;
  const char *t = s + 2, *name, *seq_end;
  size_t nlen;
  if (t >= end || *t != '{') {
    int w = 0;
    if (t < end) { next_rune(p, t, (size_t)(end - t), &w); if (p->failed) return NULL; }
    name = t; nlen = (size_t)w; seq_end = t + w;
  } else {
    const char *close = memchr(s, '}', (size_t)(end - s));
    if (!close) {
      for (const char *c = s; c < end;) { int w; next_rune(p, c, (size_t)(end - c), &w); if (p->failed) return NULL; c += w; }
      fail(p, E_INVALID_CHAR_RANGE, s, (size_t)(end - s));
      return NULL;
    }
    for (const char *c = s + 3; c < close;) { int w; next_rune(p, c, (size_t)(close - c), &w); if (p->failed) return NULL; c += w; }
    name = s + 3; nlen = (size_t)(close - name); seq_end = close + 1;
  }
  if (nlen && name[0] == '^') { sign = -sign; name++; nlen--; }
  RV tab = {0};
  int tsign;
  if (!unicode_table(name, nlen, &tab, &tsign)) {
    free(tab.r);
    fail(p, E_INVALID_CHAR_RANGE, s, (size_t)(seq_end - s));
    return NULL;
  }
  if (p->flags & F_FOLD) {  /* the table plus its fold-equivalent runes */
    RV f = {0};
    for (int i = 0; i < tab.n; i += 2) rv_push_folded(&f, tab.r[i], tab.r[i + 1]);
    free(tab.r);
    tab = f;
  }
  rv_clean(&tab);
  if (sign * tsign < 0) rv_negate(&tab);
  for (int i = 0; i < tab.n; i += 2) rv_push(cls, tab.r[i], tab.r[i + 1]);
  free(tab.r);
  return seq_end;
}

/* parseClass: s points at '['. */
static const char *parse_class(P *p, const char *s, const char *end) {
  const char *t = s + 1;
  Node *re = node_new(OP_CLASS, p->flags);
  int sign = 1;
  if (t < end && *t == '^') {
    sign = -1; t++;
    if (!(p->flags & F_CLASSNL)) rv_push(&re->cls, '\n', '\n');
  }
  int first = 1;
  while (t >= end || *t != ']' || first) {
    first = 0;
    if (end - t > 2 && t[0] == '[' && t[1] == ':') {
      const char *q = NULL;
      for (const char *c = t + 2; c + 1 < end; c++) if (c[0] == ':' && c[1] == ']') { q = c; break; }
      if (q) {
        size_t nl = (size_t)(q + 2 - t);
        const Group *g = NULL;
        for (size_t i = 0; i < sizeof(posix_groups) / sizeof(posix_groups[0]); i++)
          if (strlen(posix_groups[i].name) == nl && memcmp(posix_groups[i].name, t, nl) == 0) g = &posix_groups[i];
        if (!g) { fail(p, E_INVALID_CHAR_RANGE, t, nl); node_free(re); return NULL; }
        append_group(p, &re->cls, g);
        t = q + 2;
        continue;
      }
    }
    {
      const char *nt = parse_unicode_class(p, t, end, &re->cls);
      if (!nt) { node_free(re); return NULL; }
      if (nt != t) { t = nt; continue; }
    }
    const Group *g = perl_class_escape(p, t, end);
    if (g) { append_group(p, &re->cls, g); t += 2; continue; }
    const char *rng = t;
    int lo, hi;
    /* parseClassChar */
    if (t >= end) { fail(p, E_MISSING_BRACKET, s, (size_t)(end - s)); node_free(re); return NULL; }
    if (*t == '\\') { lo = parse_escape(p, t, end, &t); }
    else { int w; lo = next_rune(p, t, (size_t)(end - t), &w); t += w; }
    if (p->failed) { node_free(re); return NULL; }
    hi = lo;
    if (end - t >= 2 && t[0] == '-' && t[1] != ']') {
      t++;
      if (t >= end) { fail(p, E_MISSING_BRACKET, s, (size_t)(end - s)); node_free(re); return NULL; }
      if (*t == '\\') { hi = parse_escape(p, t, end, &t); }
      else { int w; hi = next_rune(p, t, (size_t)(end - t), &w); t += w; }
      if (p->failed) { node_free(re); return NULL; }
      if (hi < lo) { fail(p, E_INVALID_CHAR_RANGE, rng, (size_t)(t - rng)); node_free(re); return NULL; }
    }
    if (p->flags & F_FOLD) rv_push_folded(&re->cls, lo, hi);
    else rv_push(&re->cls, lo, hi);
  }
  t++; /* ']' */
  rv_clean(&re->cls);
  if (sign < 0) rv_negate(&re->cls);
  golim_class(p->gl, re->cls.r, re->cls.n / 2, gfl(p));
  push(p, re);
  return t;
}

static int valid_capture_name(const char *s, size_t n) {
  if (n == 0) return 0;
  for (size_t i = 0; i < n; i++)
    if (!(is_alnum((unsigned char)s[i]) || s[i] == '_')) return 0;
  return 1;
}

/* parsePerlFlags: s points at "(?" */
static const char *parse_perl_flags(P *p, const char *s, const char *end) {
  const char *t = s;
  /* named captures (?P<name>re) and (?<name>re) */
  size_t off = 0;
  if (end - t > 4 && t[2] == 'P' && t[3] == '<') off = 4;
  else if (end - t > 3 && t[2] == '<') off = 3;
  if (off) {
    const char *gt = memchr(t + off, '>', (size_t)(end - t - off));
    if (!gt) { fail(p, E_INVALID_NAMED_CAPTURE, s, (size_t)(end - s)); return NULL; }
    const char *name = t + off;
    size_t nlen = (size_t)(gt - name);
    if (!valid_capture_name(name, nlen)) { fail(p, E_INVALID_NAMED_CAPTURE, s, (size_t)(gt + 1 - s)); return NULL; }
    p->ncap++;
    golim_op(p->gl, OP_LPAREN, gfl(p), p->ncap);
    Node *lp = node_new(OP_LPAREN, p->flags);
    lp->cap = p->ncap;
    push(p, lp);
    return gt + 1;
  }
  t += 2;
  int flags = p->flags, sign = 1, saw = 0;
  while (t < end) {
    int w;
    int c = next_rune(p, t, (size_t)(end - t), &w);
    if (p->failed) return NULL;
    t += w;
    switch (c) {
    case 'i': flags |= F_FOLD; saw = 1; continue;
    case 'm': flags &= ~F_ONELINE; saw = 1; continue;
    case 's': flags |= F_DOTNL; saw = 1; continue;
    case 'U': flags |= F_NONGREEDY; saw = 1; continue;
    case '-':
      if (sign < 0) goto bad;
      sign = -1; flags = ~flags; saw = 0; continue;
    case ':': case ')':
      if (sign < 0) { if (!saw) goto bad; flags = ~flags; }
      if (c == ':') { golim_op(p->gl, OP_LPAREN, gfl(p), 0); Node *lp = node_new(OP_LPAREN, p->flags); lp->cap = 0; push(p, lp); }
      p->flags = flags;
      return t;
    default:
      goto bad;
    }
  }
bad:
  fail(p, E_INVALID_PERL_OP, s, (size_t)(t - s));
  return NULL;
}

static int depth(Node *n) {
  int d = 0;
  for (int i = 0; i < n->nsub; i++) { int x = depth(n->sub[i]); if (x > d) d = x; }
  return d + 1;
}

static Node *parse(const char *s, size_t len, char *err, size_t errlen) {
  P p = {0};
  p.whole = s; p.wlen = len; p.err = err; p.errlen = errlen;
  p.flags = F_CLASSNL | F_ONELINE | F_PERLX;
  p.gl = golim_new(simple_fold);
  const char *t = s, *end = s + len;
  const char *last_repeat = NULL;
  while (t < end && !p.failed) {
    const char *repeat = NULL;
    switch (*t) {
    case '(':
      if ((p.flags & F_PERLX) && end - t >= 2 && t[1] == '?') {
        t = parse_perl_flags(&p, t, end);
        break;
      }
      p.ncap++;
      golim_op(p.gl, OP_LPAREN, gfl(&p), p.ncap);
      { Node *lp = node_new(OP_LPAREN, p.flags); lp->cap = p.ncap; push(&p, lp); }
      t++;
      break;
    case '|':
      golim_vertical_bar(p.gl, gfl(&p));
      if (lim_check(&p)) break;
      concat(&p);
      if (!swap_vbar(&p)) op_push(&p, OP_VBAR);
      t++;
      break;
    case ')': {
      golim_right_paren(p.gl, gfl(&p));
      if (lim_check(&p)) break;
      concat(&p);
      if (swap_vbar(&p)) pop_free(&p);
      alternate(&p);
      int n = p.nst;
      if (n < 2) { fail(&p, E_UNEXPECTED_PAREN, p.whole, p.wlen); break; }
      Node *re1 = p.st[n - 1], *re2 = p.st[n - 2];
      if (re2->op != OP_LPAREN) { fail(&p, E_UNEXPECTED_PAREN, p.whole, p.wlen); break; }
      p.nst -= 2;
      p.flags = re2->flags;
      if (re2->cap == 0) { push(&p, re1); node_free(re2); }
      else { re2->op = OP_CAP; node_add(re2, re1); push(&p, re2); }
      t++;
      break;
    }
    case '^':
      op_push(&p, (p.flags & F_ONELINE) ? OP_BOT : OP_BOL); t++; break;
    case '$':
      golim_op(p.gl, (p.flags & F_ONELINE) ? OP_EOT : OP_EOL, gfl(&p) | ((p.flags & F_ONELINE) ? 256u : 0u), 0);
      push(&p, node_new((p.flags & F_ONELINE) ? OP_EOT : OP_EOL, p.flags)); t++; break;
    case '.':
      op_push(&p, (p.flags & F_DOTNL) ? OP_ANY : OP_ANYNL); t++; break;
    case '[':
      t = parse_class(&p, t, end); break;
    case '*': case '+': case '?': {
      const char *before = t;
      int op = *t == '*' ? OP_STAR : (*t == '+' ? OP_PLUS : OP_QUEST);
      const char *after = do_repeat(&p, op, 0, 0, before, t + 1, end, last_repeat);
      if (!after) break;
      repeat = before; t = after;
      break;
    }
    case '{': {
      const char *before = t, *after;
      int min, max;
      if (!parse_repeat(t, end, &min, &max, &after)) { literal(&p, '{'); t++; break; }
      if (min < 0 || min > 1000 || max > 1000 || (max >= 0 && min > max)) {
        fail(&p, E_INVALID_REPEAT_SIZE, before, (size_t)(after - before)); break;
      }
      after = do_repeat(&p, OP_REPEAT, min, max, before, after, end, last_repeat);
      if (!after) break;
      repeat = before; t = after;
      break;
    }
    case '\\': {
      if ((p.flags & F_PERLX) && end - t >= 2) {
        int done = 1;
        switch (t[1]) {
        case 'A': op_push(&p, OP_BOT); t += 2; break;
        case 'b': op_push(&p, OP_WB); t += 2; break;
        case 'B': op_push(&p, OP_NWB); t += 2; break;
        case 'C': fail(&p, E_INVALID_ESCAPE, t, 2); break;
        case 'Q': {
          const char *q = t + 2, *e = NULL;
          for (const char *c = q; c + 1 < end; c++) if (c[0] == '\\' && c[1] == 'E') { e = c; break; }
          const char *lend = e ? e : end;
          while (q < lend) {
            int w; int c = next_rune(&p, q, (size_t)(lend - q), &w);
            if (p.failed) break;
            literal(&p, c); q += w;
          }
          t = e ? e + 2 : end;
          break;
        }
        case 'z': op_push(&p, OP_EOT); t += 2; break;
        default: done = 0;
        }
        if (done) break;
      }
      golim_esc_alloc(p.gl);  /* parse's backslash case allocates a class node first */
      if (end - t >= 2 && (t[1] == 'p' || t[1] == 'P')) {
        Node *re = node_new(OP_CLASS, p.flags);
        const char *nt = parse_unicode_class(&p, t, end, &re->cls);
        if (!nt) { node_free(re); break; }
        rv_clean(&re->cls);
        golim_esc_class(p.gl, re->cls.r, re->cls.n / 2, gfl(&p));
        push(&p, re);
        t = nt;
        break;
      }
      const Group *g = perl_class_escape(&p, t, end);
      if (g) {
        Node *re = node_new(OP_CLASS, p.flags);
        append_group(&p, &re->cls, g);
        rv_clean(&re->cls);
        golim_esc_class(p.gl, re->cls.r, re->cls.n / 2, gfl(&p));
        push(&p, re);
        t += 2;
        break;
      }
      golim_esc_free(p.gl);
      const char *rest;
      int c = parse_escape(&p, t, end, &rest);
      if (p.failed) break;
      literal(&p, c); t = rest;
      break;
    }
    default: {
      int w; int c = next_rune(&p, t, (size_t)(end - t), &w);
      if (p.failed) break;
      literal(&p, c); t += w;
    }
    }
    last_repeat = repeat;
    lim_check(&p);
  }
  Node *root = NULL;
  if (!p.failed) {
    golim_end(p.gl, gfl(&p));
    lim_check(&p);
  }
  if (!p.failed) {
    concat(&p);
    if (swap_vbar(&p)) pop_free(&p);
    alternate(&p);
    if (p.nst != 1) fail(&p, E_MISSING_PAREN, p.whole, p.wlen);
    else {
      root = p.st[0]; p.nst = 0;
    }
  }
  for (int i = 0; i < p.nst; i++) node_free(p.st[i]);
  free(p.st);
  golim_free(p.gl);
  return root;
}

/* ------------------------------------------------------ program (Thompson) */

enum { I_CLASS, I_ANY, I_ANYNL, I_SPLIT, I_JMP, I_EMPTY, I_MATCH };
enum { EMPTY_BOL = 1, EMPTY_EOL = 2, EMPTY_BOT = 4, EMPTY_EOT = 8, EMPTY_WB = 16, EMPTY_NWB = 32 };

typedef struct { int op, x, y, cls, cond; } Inst;

struct gre {
  Inst *in; int nin, cin;
  RV *cls; int ncls, ccls;
  int anchored;          /* program begins with \A-only start */
  uint8_t *prefix; int nprefix;  /* literal prefix for fast skip (optimisation) */
};

static int emit(gre *g, int op) {
  if (g->nin == g->cin) { g->cin = g->cin ? g->cin * 2 : 64; g->in = realloc(g->in, sizeof(Inst) * g->cin); }
  memset(&g->in[g->nin], 0, sizeof(Inst));
  g->in[g->nin].op = op;
  return g->nin++;
}
static int add_class(gre *g, RV *v) {
  if (g->ncls == g->ccls) { g->ccls = g->ccls ? g->ccls * 2 : 16; g->cls = realloc(g->cls, sizeof(RV) * g->ccls); }
  RV c = {0};
  for (int i = 0; i < v->n; i += 2) rv_push(&c, v->r[i], v->r[i + 1]);
  rv_clean(&c);
  g->cls[g->ncls] = c;
  return g->ncls++;
}

/* Fragments are compiled with "patch lists" kept as explicit lists of
   (inst, field) holes. */
typedef struct { int *h; int n, c; } Holes;
static void holes_add(Holes *h, int v) {
  if (h->n == h->c) { h->c = h->c ? h->c * 2 : 8; h->h = realloc(h->h, sizeof(int) * h->c); }
  h->h[h->n++] = v;
}
static void patch(gre *g, Holes *h, int target) {
  for (int i = 0; i < h->n; i++) {
    int v = h->h[i];
    if (v & 1) g->in[v >> 1].y = target; else g->in[v >> 1].x = target;
  }
  h->n = 0;
}
static void holes_cat(Holes *a, Holes *b) { for (int i = 0; i < b->n; i++) holes_add(a, b->h[i]); b->n = 0; }
typedef struct { int start; Holes out; int nullable_dummy; } Frag;

static Frag comp(gre *g, Node *n);

static Frag frag_empty(gre *g) {
  Frag f = {0};
  int i = emit(g, I_JMP);
  f.start = i; holes_add(&f.out, i << 1);
  return f;
}
static Frag frag_star(gre *g, Frag body) {
  Frag f = {0};
  int s = emit(g, I_SPLIT);
  g->in[s].x = body.start;
  patch(g, &body.out, s);
  free(body.out.h);
  f.start = s; holes_add(&f.out, (s << 1) | 1);
  return f;
}
static Frag frag_quest(gre *g, Frag body) {
  Frag f = {0};
  int s = emit(g, I_SPLIT);
  g->in[s].x = body.start;
  f.start = s; f.out = body.out; holes_add(&f.out, (s << 1) | 1);
  return f;
}
static Frag frag_cat(gre *g, Frag a, Frag b) {
  patch(g, &a.out, b.start);
  free(a.out.h);
  Frag f = {0}; f.start = a.start; f.out = b.out;
  return f;
}

static Frag comp(gre *g, Node *n) {
  Frag f = {0};
  switch (n->op) {
  case OP_NOMATCH: {
    /* a class with no ranges never matches */
    RV empty = {0};
    int i = emit(g, I_CLASS);
    g->in[i].cls = add_class(g, &empty);
    f.start = i; /* no out: dead end */
    return f;
  }
  case OP_EMPTY: return frag_empty(g);
  case OP_LIT: {
    RV v = {0};
    if (n->flags & F_FOLD) {
      rv_push(&v, n->rune, n->rune);
      for (int r = simple_fold(n->rune); r != n->rune; r = simple_fold(r)) rv_push(&v, r, r);
    } else rv_push(&v, n->rune, n->rune);
    int i = emit(g, I_CLASS);
    g->in[i].cls = add_class(g, &v);
    free(v.r);
    f.start = i; holes_add(&f.out, i << 1);
    return f;
  }
  case OP_CLASS: {
    int i = emit(g, I_CLASS);
    g->in[i].cls = add_class(g, &n->cls);
    f.start = i; holes_add(&f.out, i << 1);
    return f;
  }
  case OP_ANY: case OP_ANYNL: {
    int i = emit(g, n->op == OP_ANY ? I_ANY : I_ANYNL);
    f.start = i; holes_add(&f.out, i << 1);
    return f;
  }
  case OP_BOL: case OP_EOL: case OP_BOT: case OP_EOT: case OP_WB: case OP_NWB: {
    int i = emit(g, I_EMPTY);
    g->in[i].cond = n->op == OP_BOL ? EMPTY_BOL : n->op == OP_EOL ? EMPTY_EOL : n->op == OP_BOT ? EMPTY_BOT
                  : n->op == OP_EOT ? EMPTY_EOT : n->op == OP_WB ? EMPTY_WB : EMPTY_NWB;
    f.start = i; holes_add(&f.out, i << 1);
    return f;
  }
  case OP_CAP: return comp(g, n->sub[0]);
  case OP_STAR: return frag_star(g, comp(g, n->sub[0]));
  case OP_PLUS: {
    Frag body = comp(g, n->sub[0]);
    int s = emit(g, I_SPLIT);
    g->in[s].x = body.start;
    patch(g, &body.out, s);
    free(body.out.h);
    f.start = body.start; holes_add(&f.out, (s << 1) | 1);
    return f;
  }
  case OP_QUEST: return frag_quest(g, comp(g, n->sub[0]));
  case OP_REPEAT: {
    /* x{min,max}: min copies, then (max-min) nested optionals, or x* if max<0 */
    Node *x = n->sub[0];
    int min = n->min, max = n->max;
    if (max == 0) return frag_empty(g);
    Frag acc = {0}; int have = 0;
    for (int i = 0; i < min; i++) {
      Frag c = comp(g, x);
      if (!have) { acc = c; have = 1; } else acc = frag_cat(g, acc, c);
    }
    if (max < 0) {
      Frag st = frag_star(g, comp(g, x));
      if (!have) return st;
      return frag_cat(g, acc, st);
    }
    if (max > min) {
      /* (x(x(x)?)?)? built inside-out */
      Frag opt = frag_quest(g, comp(g, x));
      for (int i = min + 1; i < max; i++) {
        Frag c = comp(g, x);
        opt = frag_quest(g, frag_cat(g, c, opt));
      }
      if (!have) return opt;
      return frag_cat(g, acc, opt);
    }
    return acc;
  }
  case OP_CONCAT: {
    Frag acc = comp(g, n->sub[0]);
    for (int i = 1; i < n->nsub; i++) acc = frag_cat(g, acc, comp(g, n->sub[i]));
    return acc;
  }
  case OP_ALT: {
    Frag acc = comp(g, n->sub[n->nsub - 1]);
    for (int i = n->nsub - 2; i >= 0; i--) {
      Frag a = comp(g, n->sub[i]);
      int s = emit(g, I_SPLIT);
      g->in[s].x = a.start; g->in[s].y = acc.start;
      Frag r = {0}; r.start = s; r.out = a.out; holes_cat(&r.out, &acc.out);
      free(acc.out.h);
      acc = r;
    }
    return acc;
  }
  }
  return frag_empty(g);
}

/* Literal prefix: leading non-folded literals of a top-level concatenation
   (Go's Prog.Prefix).  Used only to skip ahead; semantics-preserving because
   every match must begin with the prefix. */
static void compute_prefix(gre *g, Node *root) {
  Node *n = root;
  while (n->op == OP_CAP) n = n->sub[0];
  Node **items = &n; int cnt = 1;
  if (n->op == OP_CONCAT) { items = n->sub; cnt = n->nsub; }
  uint8_t buf[256]; int len = 0;
  for (int i = 0; i < cnt; i++) {
    Node *x = items[i];
    if (x->op != OP_LIT || (x->flags & F_FOLD)) break;
    int r = x->rune;
    uint8_t tmp[4]; int k;
    if (r < 0x80) { tmp[0] = (uint8_t)r; k = 1; }
    else if (r < 0x800) { tmp[0] = 0xC0 | (r >> 6); tmp[1] = 0x80 | (r & 0x3F); k = 2; }
    else if (r < 0x10000) {
      if (r >= 0xD800 && r <= 0xDFFF) break;
      tmp[0] = 0xE0 | (r >> 12); tmp[1] = 0x80 | ((r >> 6) & 0x3F); tmp[2] = 0x80 | (r & 0x3F); k = 3;
    } else { tmp[0] = 0xF0 | (r >> 18); tmp[1] = 0x80 | ((r >> 12) & 0x3F); tmp[2] = 0x80 | ((r >> 6) & 0x3F); tmp[3] = 0x80 | (r & 0x3F); k = 4; }
    if (r == RUNE_ERROR) break; /* U+FFFD also matches invalid bytes: no byte prefix */
    if (len + k > (int)sizeof(buf)) break;
    memcpy(buf + len, tmp, (size_t)k); len += k;
  }
  if (len > 0) { g->prefix = malloc((size_t)len); memcpy(g->prefix, buf, (size_t)len); g->nprefix = len; }
}

/* syntax.Parse alone (regexp.Compile's accept / reject decision and its error
   text, without building the program): 0 ok, 1 error (message in err) */
int gre_parse_check(const char *pat, size_t len, char *err, size_t errlen) {
  if (err && errlen) err[0] = 0;
  Node *root = parse(pat, len, err, errlen);
  if (!root) return 1;
  node_free(root);
  return 0;
}

gre *gre_compile(const char *pat, size_t len, char *err, size_t errlen) {
  if (err && errlen) err[0] = 0;
  Node *root = parse(pat, len, err, errlen);
  if (!root) return NULL;
  gre *g = calloc(1, sizeof(gre));
  Frag f = comp(g, root);
  int m = emit(g, I_MATCH);
  patch(g, &f.out, m);
  free(f.out.h);
  /* start instruction index = f.start; store it as inst 0 via a JMP */
  int s = emit(g, I_JMP);
  g->in[s].x = f.start;
  compute_prefix(g, root);
  node_free(root);
  return g;
}

void gre_free(gre *g) {
  if (!g) return;
  for (int i = 0; i < g->ncls; i++) free(g->cls[i].r);
  free(g->cls); free(g->in); free(g->prefix); free(g);
}

/* ------------------------------------------------------------- Pike VM */

static int is_word(int r) { return r >= 0 && r < 0x80 && (is_alnum(r) || r == '_'); }

/* regexp/syntax.EmptyOpContext */
static int empty_ctx(int r1, int r2) {
  int op = EMPTY_NWB, boundary = 0;
  if (is_word(r1)) boundary = 1;
  else if (r1 == '\n') op |= EMPTY_BOL;
  else if (r1 < 0) op |= EMPTY_BOT | EMPTY_BOL;
  if (is_word(r2)) boundary ^= 1;
  else if (r2 == '\n') op |= EMPTY_EOL;
  else if (r2 < 0) op |= EMPTY_EOT | EMPTY_EOL;
  if (boundary) op ^= (EMPTY_WB | EMPTY_NWB);
  return op;
}

static int class_has(const RV *v, int r) {
  int lo = 0, hi = v->n / 2;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (v->r[2 * m + 1] < r) lo = m + 1; else hi = m;
  }
  return lo < v->n / 2 && v->r[2 * lo] <= r;
}

typedef struct { int *dense; int n; unsigned *mark; unsigned gen; } Q;

/* add pc's epsilon closure to q under context cond; returns 1 on Match */
static int addq(const gre *g, Q *q, int pc, int cond, int *stack) {
  int sp = 0;
  stack[sp++] = pc;
  int matched = 0;
  while (sp) {
    int i = stack[--sp];
    if (q->mark[i] == q->gen) continue;
    q->mark[i] = q->gen;
    const Inst *in = &g->in[i];
    switch (in->op) {
    case I_JMP: stack[sp++] = in->x; break;
    case I_SPLIT: stack[sp++] = in->y; stack[sp++] = in->x; break;
    case I_EMPTY: if ((in->cond & ~cond) == 0) stack[sp++] = in->x; break;
    case I_MATCH: matched = 1; break;
    default: q->dense[q->n++] = i; break;
    }
  }
  return matched;
}

static const uint8_t *memmem_(const uint8_t *h, size_t hn, const uint8_t *n, size_t nn) {
  if (nn == 0) return h;
  if (hn < nn) return NULL;
  const uint8_t *end = h + hn - nn;
  for (const uint8_t *p = h; p <= end; ) {
    p = memchr(p, n[0], (size_t)(end - p) + 1);
    if (!p) return NULL;
    if (memcmp(p, n, nn) == 0) return p;
    p++;
  }
  return NULL;
}

int gre_match(const gre *g, const uint8_t *s, size_t n) {
  int start = g->nin - 1;
  Q a, b;
  a.dense = malloc(sizeof(int) * g->nin); b.dense = malloc(sizeof(int) * g->nin);
  a.mark = calloc((size_t)g->nin, sizeof(unsigned)); b.mark = calloc((size_t)g->nin, sizeof(unsigned));
  a.gen = b.gen = 0; a.n = b.n = 0;
  int *stack = malloc(sizeof(int) * (size_t)(g->nin * 2 + 4));
  Q *run = &a, *nxt = &b;
  size_t pos = 0;
  int w, w1 = 0;
  int r = decode_rune(s, n, &w);
  int r1 = -1;
  if (r >= 0) r1 = decode_rune(s + w, n - w, &w1);
  int prev = -1;
  int matched = 0;
  run->gen++;
  for (;;) {
    if (run->n == 0 && g->nprefix > 0) {
      const uint8_t *hit = memmem_(s + pos, n - pos, g->prefix, (size_t)g->nprefix);
      if (!hit) break;
      size_t np = (size_t)(hit - s);
      if (np != pos) {
        /* previous rune for context: decode backwards by byte class (ASCII or not) */
        uint8_t pb = s[np - 1];
        prev = pb < 0x80 ? pb : RUNE_ERROR;
        pos = np;
        r = decode_rune(s + pos, n - pos, &w);
        r1 = r >= 0 ? decode_rune(s + pos + w, n - pos - w, &w1) : -1;
      }
    }
    if (addq(g, run, start, empty_ctx(prev, r), stack)) { matched = 1; break; }
    if (r < 0) break;
    int cond = empty_ctx(r, r1);
    nxt->gen++; nxt->n = 0;
    for (int k = 0; k < run->n; k++) {
      const Inst *in = &g->in[run->dense[k]];
      int ok = 0;
      if (in->op == I_ANY) ok = 1;
      else if (in->op == I_ANYNL) ok = r != '\n';
      else if (in->op == I_CLASS) ok = class_has(&g->cls[in->cls], r);
      if (ok && addq(g, nxt, in->x, cond, stack)) { matched = 1; break; }
    }
    if (matched) break;
    pos += (size_t)w;
    prev = r;
    r = r1; w = w1;
    if (r >= 0) r1 = decode_rune(s + pos + w, n - pos - w, &w1); else r1 = -1;
    Q *tmp = run; run = nxt; nxt = tmp;
  }
  free(a.dense); free(b.dense); free(a.mark); free(b.mark); free(stack);
  return matched;
}
