/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into the product library.
 *
 * Go 1.25 regexp/syntax parse-size limits (not vendored in /root/reference),
 * as the reference's config load meets them (internal/config.go:110-113,
 * `regexp.Compile` -> syntax.Parse):
 *   ErrLarge        "expression too large"         (maxSize = 128 MB / 40 B per
 *                   Inst, maxRunes = 128 MB / 4 B per rune)
 *   ErrNestingDepth "expression nests too deeply"  (maxHeight = 1000)
 * Go checks them while parsing (parser.checkLimits after each push and repeat,
 * and after factor() rewrites an alternation branch) on its own node shapes:
 * merged literal runs (maybeConcat), one-rune classes as literals, flattened
 * and factored alternations, a free list of reused nodes; the size check
 * starts only once (nodes allocated) x (product of repeat counts) reaches
 * maxSize, the height check once 1000 nodes were allocated, and both cache
 * per-node results across later rewrites.  The functions below replay those
 * steps (parse.go: newRegexp, reuse, push, maybeConcat, literal, op, concat,
 * alternate, collapse, factor, leadingString, removeLeadingString,
 * leadingRegexp, removeLeadingRegexp, swapVerticalBar, parseRightParen,
 * repeat, checkLimits, checkSize, calcSize, checkHeight, calcHeight;
 * regexp.go: Equal; parse.go's class helpers mergeCharClass, appendRange,
 * appendFoldedRange, cleanClass, cleanAlt), driven by the oracle parser's
 * events (go_regexp.c).
 */
#include "go_limits.h"

#include <stdlib.h>
#include <string.h>

enum { G_NOMATCH = 1, G_EMPTY, G_LIT, G_CLASS, G_ANYNL, G_ANY, G_BOL, G_EOL, G_BOT, G_EOT, G_WB, G_NWB,
       G_CAP, G_STAR, G_PLUS, G_QUEST, G_REPEAT, G_CONCAT, G_ALT, G_PSEUDO = 128, G_LPAREN, G_VBAR };
#define GF_FOLD 1u
#define GF_NONGREEDY 32u
#define GF_WASDOLLAR 256u
#define MAX_SIZE ((int64_t)(128 << 20) / 40)
#define MAX_RUNES ((int64_t)(128 << 20) / 4)
#define MAX_HEIGHT 1000
#define MIN_FOLD_R 0x0041
#define MAX_FOLD_R 0x1e943

typedef struct GNode {
  int op;
  unsigned flags;
  int *r; int nr, cr;            /* Rune */
  struct GNode **sub; int ns, cs;
  int min, max, cap;
  struct GNode *free_next;
  /* caches (Go's p.size / p.height maps, keyed by node) */
  int64_t size; int has_size;
  int height; int has_height;
  struct GNode *all_next;        /* every node ever allocated (for cleanup) */
} GNode;

struct GoLim {
  int (*fold)(int);
  GNode **st; int nst, cst;
  GNode *free_list, *all, *esc;
  int64_t num_regexp, num_runes, repeats;
  int size_on, height_on;
  int failed;  /* 1 ErrLarge, 2 ErrNestingDepth */
};

static void r_push(GNode *n, int v) {
  if (n->nr == n->cr) { n->cr = n->cr ? 2 * n->cr : 4; n->r = realloc(n->r, sizeof(int) * (size_t)n->cr); }
  n->r[n->nr++] = v;
}
static void s_push(GNode *n, GNode *s) {
  if (n->ns == n->cs) { n->cs = n->cs ? 2 * n->cs : 4; n->sub = realloc(n->sub, sizeof(GNode *) * (size_t)n->cs); }
  n->sub[n->ns++] = s;
}
static void st_push(GoLim *g, GNode *n) {
  if (g->nst == g->cst) { g->cst = g->cst ? 2 * g->cst : 16; g->st = realloc(g->st, sizeof(GNode *) * (size_t)g->cst); }
  g->st[g->nst++] = n;
}

static GNode *new_re(GoLim *g, int op) {
  GNode *re = g->free_list;
  if (re) {
    g->free_list = re->free_next;
    GNode *keep_all = re->all_next;
    int *r = re->r; int cr = re->cr;
    GNode **sub = re->sub; int cs = re->cs;
    int64_t size = re->size; int has_size = re->has_size;  /* Go keeps size-cache entries of reused nodes */
    memset(re, 0, sizeof *re);
    re->all_next = keep_all; re->r = r; re->cr = cr; re->sub = sub; re->cs = cs;
    re->size = size; re->has_size = has_size;
  } else {
    re = calloc(1, sizeof *re);
    re->all_next = g->all;
    g->all = re;
    g->num_regexp++;
  }
  re->op = op;
  return re;
}
static void reuse(GoLim *g, GNode *re) {
  re->has_height = 0;  /* delete(p.height, re) */
  re->free_next = g->free_list;
  g->free_list = re;
}

static int min_fold_rune(GoLim *g, int r) {
  if (r < MIN_FOLD_R || r > MAX_FOLD_R) return r;
  int m = r, r0 = r;
  for (r = g->fold(r); r != r0; r = g->fold(r)) if (r < m) m = r;
  return m;
}

/* ---- limits */
static int64_t calc_size(GNode *re, int force) {
  if (!force && re->has_size) return re->size;
  int64_t size = 0;
  switch (re->op) {
  case G_LIT: size = re->nr; break;
  case G_CAP: case G_STAR: size = 2 + calc_size(re->sub[0], 0); break;
  case G_PLUS: case G_QUEST: size = 1 + calc_size(re->sub[0], 0); break;
  case G_CONCAT: for (int i = 0; i < re->ns; i++) size += calc_size(re->sub[i], 0); break;
  case G_ALT:
    for (int i = 0; i < re->ns; i++) size += calc_size(re->sub[i], 0);
    if (re->ns > 1) size += re->ns - 1;
    break;
  case G_REPEAT: {
    int64_t sub = calc_size(re->sub[0], 0);
    if (re->max == -1) size = re->min == 0 ? 2 + sub : 1 + (int64_t)re->min * sub;
    else size = (int64_t)re->max * sub + (int64_t)(re->max - re->min);
    break;
  }
  default: break;
  }
  if (size < 1) size = 1;
  re->size = size; re->has_size = 1;
  return size;
}
static int calc_height(GNode *re, int force) {
  if (!force && re->has_height) return re->height;
  int h = 1;
  for (int i = 0; i < re->ns; i++) { int x = 1 + calc_height(re->sub[i], 0); if (x > h) h = x; }
  re->height = h; re->has_height = 1;
  return h;
}
static void check_size(GoLim *g, GNode *re) {
  if (g->failed) return;
  if (!g->size_on) {
    if (g->repeats == 0) g->repeats = 1;
    if (re->op == G_REPEAT) {
      int64_t n = re->max;
      if (n == -1) n = re->min;
      if (n <= 0) n = 1;
      if (n > MAX_SIZE / g->repeats) g->repeats = MAX_SIZE;
      else g->repeats *= n;
    }
    if (g->num_regexp < MAX_SIZE / g->repeats) return;
    g->size_on = 1;
    /* a fresh map: every cached size is forgotten */
    for (GNode *a = g->all; a; a = a->all_next) a->has_size = 0;
    for (int i = 0; i < g->nst; i++) check_size(g, g->st[i]);
    if (g->failed) return;
  }
  if (calc_size(re, 1) > MAX_SIZE) g->failed = 1;
}
static void check_height(GoLim *g, GNode *re) {
  if (g->failed) return;
  if (g->num_regexp < MAX_HEIGHT) return;
  if (!g->height_on) {
    g->height_on = 1;
    for (GNode *a = g->all; a; a = a->all_next) a->has_height = 0;
    for (int i = 0; i < g->nst; i++) check_height(g, g->st[i]);
    if (g->failed) return;
  }
  if (calc_height(re, 1) > MAX_HEIGHT) g->failed = 2;
}
static void check_limits(GoLim *g, GNode *re) {
  if (g->failed) return;
  if (g->num_runes > MAX_RUNES) { g->failed = 1; return; }
  check_size(g, re);
  check_height(g, re);
}

/* ---- push / maybeConcat */
static int maybe_concat(GoLim *g, int r, unsigned flags) {
  int n = g->nst;
  if (n < 2) return 0;
  GNode *re1 = g->st[n - 1], *re2 = g->st[n - 2];
  if (re1->op != G_LIT || re2->op != G_LIT || (re1->flags & GF_FOLD) != (re2->flags & GF_FOLD)) return 0;
  for (int i = 0; i < re1->nr; i++) r_push(re2, re1->r[i]);
  if (r >= 0) {
    re1->nr = 0; r_push(re1, r);
    re1->flags = flags;
    return 1;
  }
  g->nst--;
  reuse(g, re1);
  return 0;
}
static GNode *push(GoLim *g, GNode *re, unsigned flags) {
  g->num_runes += re->nr;
  if (re->op == G_CLASS && re->nr == 2 && re->r[0] == re->r[1]) {
    if (maybe_concat(g, re->r[0], flags & ~GF_FOLD)) return NULL;
    re->op = G_LIT; re->nr = 1; re->flags = flags & ~GF_FOLD;
  } else if ((re->op == G_CLASS && re->nr == 4 && re->r[0] == re->r[1] && re->r[2] == re->r[3] &&
              g->fold(re->r[0]) == re->r[2] && g->fold(re->r[2]) == re->r[0]) ||
             (re->op == G_CLASS && re->nr == 2 && re->r[0] + 1 == re->r[1] && g->fold(re->r[0]) == re->r[1] &&
              g->fold(re->r[1]) == re->r[0])) {
    if (maybe_concat(g, re->r[0], flags | GF_FOLD)) return NULL;
    re->op = G_LIT; re->nr = 1; re->flags = flags | GF_FOLD;
  } else {
    maybe_concat(g, -1, 0);
  }
  st_push(g, re);
  check_limits(g, re);
  return re;
}

/* ---- class arithmetic on flat rune pairs */
static void append_range(GNode *n, int lo, int hi) {
  for (int i = 2; i <= 4; i += 2) {
    if (n->nr >= i) {
      int rlo = n->r[n->nr - i], rhi = n->r[n->nr - i + 1];
      if (lo <= rhi + 1 && rlo <= hi + 1) {
        if (lo < rlo) n->r[n->nr - i] = lo;
        if (hi > rhi) n->r[n->nr - i + 1] = hi;
        return;
      }
    }
  }
  r_push(n, lo); r_push(n, hi);
}
static void append_folded_range(GoLim *g, GNode *n, int lo, int hi) {
  if ((lo <= MIN_FOLD_R && hi >= MAX_FOLD_R) || hi < MIN_FOLD_R || lo > MAX_FOLD_R) { append_range(n, lo, hi); return; }
  if (lo < MIN_FOLD_R) { append_range(n, lo, MIN_FOLD_R - 1); lo = MIN_FOLD_R; }
  if (hi > MAX_FOLD_R) { append_range(n, MAX_FOLD_R + 1, hi); hi = MAX_FOLD_R; }
  for (int c = lo; c <= hi; c++) {
    append_range(n, c, c);
    for (int f = g->fold(c); f != c; f = g->fold(f)) append_range(n, f, f);
  }
}
static void append_literal(GoLim *g, GNode *n, int x, unsigned flags) {
  if (flags & GF_FOLD) append_folded_range(g, n, x, x);
  else append_range(n, x, x);
}
static int match_rune(const GNode *re, int c) {
  switch (re->op) {
  case G_LIT: return re->nr == 1 && re->r[0] == c;
  case G_CLASS:
    for (int i = 0; i + 1 < re->nr; i += 2) if (re->r[i] <= c && c <= re->r[i + 1]) return 1;
    return 0;
  case G_ANYNL: return c != '\n';
  case G_ANY: return 1;
  }
  return 0;
}
static void merge_char_class(GoLim *g, GNode *dst, const GNode *src) {
  switch (dst->op) {
  case G_ANY: break;
  case G_ANYNL: if (match_rune(src, '\n')) dst->op = G_ANY; break;
  case G_CLASS:
    if (src->op == G_LIT) append_literal(g, dst, src->r[0], src->flags);
    else for (int i = 0; i + 1 < src->nr; i += 2) append_range(dst, src->r[i], src->r[i + 1]);
    break;
  case G_LIT:
    if (src->r[0] == dst->r[0] && src->flags == dst->flags) break;
    {
      int d0 = dst->r[0];
      dst->op = G_CLASS; dst->nr = 0;
      append_literal(g, dst, d0, dst->flags);
      append_literal(g, dst, src->r[0], src->flags);
    }
    break;
  }
}
static int cmp_pair_go(const void *a, const void *b) {  /* lo increasing, hi decreasing */
  const int *x = a, *y = b;
  if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
  return x[1] > y[1] ? -1 : (x[1] < y[1] ? 1 : 0);
}
static void clean_class(GNode *n) {
  if (n->nr < 2) return;
  qsort(n->r, (size_t)(n->nr / 2), 2 * sizeof(int), cmp_pair_go);
  int w = 2;
  for (int i = 2; i < n->nr; i += 2) {
    int lo = n->r[i], hi = n->r[i + 1];
    if (lo <= n->r[w - 1] + 1) { if (hi > n->r[w - 1]) n->r[w - 1] = hi; continue; }
    n->r[w] = lo; n->r[w + 1] = hi; w += 2;
  }
  n->nr = w;
}
static void clean_alt(GNode *re) {
  if (re->op != G_CLASS) return;
  clean_class(re);
  if (re->nr == 2 && re->r[0] == 0 && re->r[1] == 0x10FFFF) { re->nr = 0; re->op = G_ANY; return; }
  if (re->nr == 4 && re->r[0] == 0 && re->r[1] == '\n' - 1 && re->r[2] == '\n' + 1 && re->r[3] == 0x10FFFF) {
    re->nr = 0; re->op = G_ANYNL;
  }
}
static int is_char_class(const GNode *re) {
  return (re->op == G_LIT && re->nr == 1) || re->op == G_CLASS || re->op == G_ANYNL || re->op == G_ANY;
}
static int equal(const GNode *x, const GNode *y) {
  if (!x || !y) return x == y;
  if (x->op != y->op) return 0;
  switch (x->op) {
  case G_EOT: return (x->flags & GF_WASDOLLAR) == (y->flags & GF_WASDOLLAR);
  case G_LIT: case G_CLASS:
    return x->nr == y->nr && (x->nr == 0 || memcmp(x->r, y->r, sizeof(int) * (size_t)x->nr) == 0);
  case G_ALT: case G_CONCAT:
    if (x->ns != y->ns) return 0;
    for (int i = 0; i < x->ns; i++) if (!equal(x->sub[i], y->sub[i])) return 0;
    return 1;
  case G_STAR: case G_PLUS: case G_QUEST:
    return (x->flags & GF_NONGREEDY) == (y->flags & GF_NONGREEDY) && equal(x->sub[0], y->sub[0]);
  case G_REPEAT:
    return (x->flags & GF_NONGREEDY) == (y->flags & GF_NONGREEDY) && x->min == y->min && x->max == y->max &&
           equal(x->sub[0], y->sub[0]);
  case G_CAP: return x->cap == y->cap && equal(x->sub[0], y->sub[0]);
  }
  return 1;
}

/* ---- collapse / factor */
static GNode *collapse(GoLim *g, GNode **subs, int n, int op);

static GNode *remove_leading_string(GoLim *g, GNode *re, int n) {
  if (re->op == G_CONCAT && re->ns > 0) {
    GNode *sub = remove_leading_string(g, re->sub[0], n);
    re->sub[0] = sub;
    if (sub->op == G_EMPTY) {
      reuse(g, sub);
      if (re->ns <= 1) { re->op = G_EMPTY; re->ns = 0; }
      else if (re->ns == 2) { GNode *old = re; re = re->sub[1]; reuse(g, old); }
      else { memmove(re->sub, re->sub + 1, sizeof(GNode *) * (size_t)(re->ns - 1)); re->ns--; }
    }
    return re;
  }
  if (re->op == G_LIT) {
    int k = n < re->nr ? n : re->nr;
    memmove(re->r, re->r + k, sizeof(int) * (size_t)(re->nr - k));
    re->nr -= k;
    if (re->nr == 0) re->op = G_EMPTY;
  }
  return re;
}
static GNode *leading_regexp(GNode *re) {
  if (re->op == G_EMPTY) return NULL;
  if (re->op == G_CONCAT && re->ns > 0) {
    GNode *sub = re->sub[0];
    if (sub->op == G_EMPTY) return NULL;
    return sub;
  }
  return re;
}
static GNode *remove_leading_regexp(GoLim *g, GNode *re, int reuse_it) {
  if (re->op == G_CONCAT && re->ns > 0) {
    if (reuse_it) reuse(g, re->sub[0]);
    memmove(re->sub, re->sub + 1, sizeof(GNode *) * (size_t)(re->ns - 1));
    re->ns--;
    if (re->ns == 0) { re->op = G_EMPTY; }
    else if (re->ns == 1) { GNode *old = re; re = re->sub[0]; reuse(g, old); }
    return re;
  }
  if (reuse_it) reuse(g, re);
  return new_re(g, G_EMPTY);
}

/* factor(sub) in place; returns the new length */
static int factor(GoLim *g, GNode **sub, int n) {
  if (n < 2) return n;
  GNode **out = malloc(sizeof(GNode *) * (size_t)(n + 1));
  int nout;
  /* Round 1: common literal prefixes */
  {
    int *str = NULL, nstr = 0;
    unsigned strflags = 0;
    int start = 0;
    nout = 0;
    for (int i = 0; i <= n; i++) {
      const int *istr = NULL; int nistr = 0;
      unsigned iflags = 0;
      if (i < n) {
        const GNode *l = (sub[i]->op == G_CONCAT && sub[i]->ns > 0) ? sub[i]->sub[0] : sub[i];
        if (l->op == G_LIT) { istr = l->r; nistr = l->nr; iflags = l->flags & GF_FOLD; }
        if (iflags == strflags) {
          int same = 0;
          while (same < nstr && same < nistr && str[same] == istr[same]) same++;
          if (same > 0) { nstr = same; continue; }
        }
      }
      if (i == start) {
      } else if (i == start + 1) {
        out[nout++] = sub[start];
      } else {
        GNode *prefix = new_re(g, G_LIT);
        prefix->flags = strflags;
        for (int k = 0; k < nstr; k++) r_push(prefix, str[k]);
        for (int j = start; j < i; j++) {
          sub[j] = remove_leading_string(g, sub[j], nstr);
          check_limits(g, sub[j]);
        }
        GNode *suffix = collapse(g, sub + start, i - start, G_ALT);
        GNode *re = new_re(g, G_CONCAT);
        s_push(re, prefix); s_push(re, suffix);
        out[nout++] = re;
      }
      start = i;
      free(str);
      str = NULL; nstr = 0;
      if (nistr) { str = malloc(sizeof(int) * (size_t)nistr); memcpy(str, istr, sizeof(int) * (size_t)nistr); nstr = nistr; }
      strflags = iflags;
    }
    free(str);
    memcpy(sub, out, sizeof(GNode *) * (size_t)nout);
    n = nout;
  }
  /* Round 2: common leading regexp */
  {
    int start = 0;
    GNode *first = NULL;
    nout = 0;
    for (int i = 0; i <= n; i++) {
      GNode *ifirst = NULL;
      if (i < n) {
        ifirst = leading_regexp(sub[i]);
        if (first && equal(first, ifirst) &&
            (is_char_class(first) || (first->op == G_REPEAT && first->min == first->max && is_char_class(first->sub[0]))))
          continue;
      }
      if (i == start) {
      } else if (i == start + 1) {
        out[nout++] = sub[start];
      } else {
        GNode *prefix = first;
        for (int j = start; j < i; j++) {
          sub[j] = remove_leading_regexp(g, sub[j], j != start);
          check_limits(g, sub[j]);
        }
        GNode *suffix = collapse(g, sub + start, i - start, G_ALT);
        GNode *re = new_re(g, G_CONCAT);
        s_push(re, prefix); s_push(re, suffix);
        out[nout++] = re;
      }
      start = i;
      first = ifirst;
    }
    memcpy(sub, out, sizeof(GNode *) * (size_t)nout);
    n = nout;
  }
  /* Round 3: runs of literals / classes into one class */
  {
    int start = 0;
    nout = 0;
    for (int i = 0; i <= n; i++) {
      if (i < n && is_char_class(sub[i])) continue;
      if (i == start) {
      } else if (i == start + 1) {
        out[nout++] = sub[start];
      } else {
        int mx = start;
        for (int j = start + 1; j < i; j++)
          if (sub[mx]->op < sub[j]->op || (sub[mx]->op == sub[j]->op && sub[mx]->nr < sub[j]->nr)) mx = j;
        GNode *t = sub[start]; sub[start] = sub[mx]; sub[mx] = t;
        for (int j = start + 1; j < i; j++) { merge_char_class(g, sub[start], sub[j]); reuse(g, sub[j]); }
        clean_alt(sub[start]);
        out[nout++] = sub[start];
      }
      if (i < n) out[nout++] = sub[i];
      start = i + 1;
    }
    memcpy(sub, out, sizeof(GNode *) * (size_t)nout);
    n = nout;
  }
  /* Round 4: runs of empty matches */
  {
    nout = 0;
    for (int i = 0; i < n; i++) {
      if (i + 1 < n && sub[i]->op == G_EMPTY && sub[i + 1]->op == G_EMPTY) continue;
      out[nout++] = sub[i];
    }
    memcpy(sub, out, sizeof(GNode *) * (size_t)nout);
    n = nout;
  }
  free(out);
  return n;
}

static GNode *collapse(GoLim *g, GNode **subs, int n, int op) {
  if (n == 1) return subs[0];
  GNode *re = new_re(g, op);
  for (int i = 0; i < n; i++) {
    GNode *s = subs[i];
    if (s->op == op) {
      for (int k = 0; k < s->ns; k++) s_push(re, s->sub[k]);
      reuse(g, s);
    } else {
      s_push(re, s);
    }
  }
  if (op == G_ALT) {
    re->ns = factor(g, re->sub, re->ns);
    if (re->ns == 1) { GNode *old = re; re = re->sub[0]; reuse(g, old); }
  }
  return re;
}

static int top_items(GoLim *g) {
  int i = g->nst;
  while (i > 0 && g->st[i - 1]->op < G_PSEUDO) i--;
  return i;
}
static void concat(GoLim *g, unsigned flags) {
  maybe_concat(g, -1, 0);
  int i = top_items(g), n = g->nst - i;
  if (n <= 0) { g->nst = i; push(g, new_re(g, G_EMPTY), flags); return; }
  GNode **subs = malloc(sizeof(GNode *) * (size_t)n);
  memcpy(subs, g->st + i, sizeof(GNode *) * (size_t)n);
  g->nst = i;
  GNode *re = collapse(g, subs, n, G_CONCAT);
  free(subs);
  push(g, re, flags);
}
static void alternate(GoLim *g, unsigned flags) {
  int i = top_items(g), n = g->nst - i;
  if (n > 0) clean_alt(g->st[g->nst - 1]);
  if (n <= 0) { g->nst = i; push(g, new_re(g, G_NOMATCH), flags); return; }
  GNode **subs = malloc(sizeof(GNode *) * (size_t)n);
  memcpy(subs, g->st + i, sizeof(GNode *) * (size_t)n);
  g->nst = i;
  GNode *re = collapse(g, subs, n, G_ALT);
  free(subs);
  push(g, re, flags);
}
static int swap_vertical_bar(GoLim *g) {
  int n = g->nst;
  if (n >= 3 && g->st[n - 2]->op == G_VBAR && is_char_class(g->st[n - 1]) && is_char_class(g->st[n - 3])) {
    GNode *re1 = g->st[n - 1], *re3 = g->st[n - 3];
    if (re1->op > re3->op) { GNode *t = re1; re1 = re3; re3 = t; g->st[n - 3] = re3; }
    merge_char_class(g, re3, re1);
    reuse(g, re1);
    g->nst--;
    return 1;
  }
  if (n >= 2) {
    GNode *re1 = g->st[n - 1], *re2 = g->st[n - 2];
    if (re2->op == G_VBAR) {
      if (n >= 3) clean_alt(g->st[n - 3]);
      g->st[n - 2] = re1;
      g->st[n - 1] = re2;
      return 1;
    }
  }
  return 0;
}

/* ---- events */
GoLim *golim_new(int (*fold)(int)) {
  GoLim *g = calloc(1, sizeof *g);
  g->fold = fold;
  return g;
}
void golim_free(GoLim *g) {
  if (!g) return;
  for (GNode *a = g->all; a;) { GNode *nx = a->all_next; free(a->r); free(a->sub); free(a); a = nx; }
  free(g->st);
  free(g);
}
int golim_failed(const GoLim *g) { return g->failed; }

void golim_literal(GoLim *g, int c, unsigned flags) {
  if (g->failed) return;
  GNode *re = new_re(g, G_LIT);
  re->flags = flags;
  if (flags & GF_FOLD) c = min_fold_rune(g, c);
  r_push(re, c);
  push(g, re, flags);
}
void golim_op(GoLim *g, int op, unsigned flags, int cap) {
  if (g->failed) return;
  GNode *re = new_re(g, op);
  re->flags = flags;
  re->cap = cap;
  push(g, re, flags);
}
void golim_class(GoLim *g, const int *pairs, int n_pairs, unsigned flags) {
  if (g->failed) return;
  GNode *re = new_re(g, G_CLASS);
  re->flags = flags;
  for (int i = 0; i < 2 * n_pairs; i++) r_push(re, pairs[i]);
  push(g, re, flags);
}
void golim_esc_alloc(GoLim *g) {
  if (g->failed) return;
  g->esc = new_re(g, G_CLASS);
}
void golim_esc_class(GoLim *g, const int *pairs, int n_pairs, unsigned flags) {
  if (g->failed) return;
  GNode *re = g->esc;
  g->esc = NULL;
  re->flags = flags;
  for (int i = 0; i < 2 * n_pairs; i++) r_push(re, pairs[i]);
  push(g, re, flags);
}
void golim_esc_free(GoLim *g) {
  if (g->failed || !g->esc) return;
  reuse(g, g->esc);
  g->esc = NULL;
}
void golim_vertical_bar(GoLim *g, unsigned flags) {
  if (g->failed) return;
  concat(g, flags);
  if (g->failed) return;
  if (!swap_vertical_bar(g)) golim_op(g, G_VBAR, flags, 0);
}
void golim_right_paren(GoLim *g, unsigned flags) {
  if (g->failed) return;
  concat(g, flags);
  if (g->failed) return;
  if (swap_vertical_bar(g)) g->nst--;
  alternate(g, flags);
  if (g->failed) return;
  int n = g->nst;
  if (n < 2) return;
  GNode *re1 = g->st[n - 1], *re2 = g->st[n - 2];
  if (re2->op != G_LPAREN) return;
  g->nst -= 2;
  unsigned fl = re2->flags;
  if (re2->cap == 0) push(g, re1, fl);
  else { re2->op = G_CAP; re2->ns = 0; s_push(re2, re1); push(g, re2, fl); }
}
void golim_repeat(GoLim *g, int op, int min, int max, unsigned flags) {
  if (g->failed || g->nst == 0) return;
  GNode *sub = g->st[g->nst - 1];
  GNode *re = new_re(g, op);
  re->min = min; re->max = max; re->flags = flags;
  s_push(re, sub);
  g->st[g->nst - 1] = re;
  check_limits(g, re);
}
void golim_end(GoLim *g, unsigned flags) {
  if (g->failed) return;
  concat(g, flags);
  if (g->failed) return;
  if (swap_vertical_bar(g)) g->nst--;
  alternate(g, flags);
}
