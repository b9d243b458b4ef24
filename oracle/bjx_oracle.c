/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into, or called by, the product library.
 *
 * Plain-C restatement of the banjax regex rate-limiting log tailer
 * (reference: deflect-ca/banjax at /root/reference, Go 1.25.8):
 *   consumeLine            internal/regex_rate_limiter.go:113-214
 *   applyRegexToLog        internal/regex_rate_limiter.go:216-269
 *   parseTimestamp         internal/regex_rate_limiter.go:95-103 (strconv.ParseFloat)
 *   RegexRateLimitStates   internal/rate_limit.go:17-103
 *   CheckIsAllowed         internal/decision.go:185-216, tables 278-374
 *   DynamicDecisionLists   internal/decision.go:377-439 (Update)
 *   Banner                 internal/iptables.go:179-228 (LogRegexBan), 273-294 (BanOrChallengeIp)
 *   MockBanner             internal/regex_rate_limiter_test.go:27-75
 * Third-party algorithms restated from their published behaviour (none is
 * vendored under /root/reference): Go stdlib regexp (go_regexp.c),
 * strconv.ParseFloat, net/netip ParseAddr + net.ParseCIDR/IPNet.Contains,
 * github.com/jeremy5189/ipfilter-no-iploc/v2 v2.0.3 (IPFilter.Allowed),
 * encoding/json string escaping, time.Time.Sub saturation.
 * The injected clock now_ns replaces time.Now().
 */
#include "bjx_oracle.h"

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "go_regexp.h"

/* ------------------------------------------------------------ hash map */

typedef struct { char *k; size_t kl; void *v; uint64_t h; } Slot;
typedef struct { Slot *s; size_t cap, n; } Map;

static uint64_t hbytes(const void *p, size_t n) {
  const uint8_t *b = p;
  uint64_t h = 1469598103934665603ULL;
  for (size_t i = 0; i < n; i++) { h ^= b[i]; h *= 1099511628211ULL; }
  return h ^ (h >> 29);
}
static void map_grow(Map *m);
static Slot *map_find(Map *m, const void *k, size_t kl, int create) {
  if (create && (m->n + 1) * 2 > m->cap) map_grow(m);
  if (!m->cap) return NULL;
  uint64_t h = hbytes(k, kl);
  size_t i = h & (m->cap - 1);
  for (;;) {
    Slot *s = &m->s[i];
    if (!s->k) {
      if (!create) return NULL;
      s->k = malloc(kl ? kl : 1); memcpy(s->k, k, kl); s->kl = kl; s->h = h; s->v = NULL;
      m->n++;
      return s;
    }
    if (s->h == h && s->kl == kl && memcmp(s->k, k, kl) == 0) return s;
    i = (i + 1) & (m->cap - 1);
  }
}
static void map_grow(Map *m) {
  size_t nc = m->cap ? m->cap * 2 : 64;
  Slot *old = m->s; size_t oc = m->cap;
  m->s = calloc(nc, sizeof(Slot)); m->cap = nc;
  for (size_t i = 0; i < oc; i++) {
    if (!old[i].k) continue;
    size_t j = old[i].h & (nc - 1);
    while (m->s[j].k) j = (j + 1) & (nc - 1);
    m->s[j] = old[i];
  }
  free(old);
}
static void map_free(Map *m, void (*fv)(void *)) {
  for (size_t i = 0; i < m->cap; i++)
    if (m->s[i].k) { free(m->s[i].k); if (fv) fv(m->s[i].v); }
  free(m->s); m->s = NULL; m->cap = m->n = 0;
}

/* --------------------------------------------------- strconv.ParseFloat */

static int lower_(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

/* strconv underscoreOK */
static int underscore_ok(const char *s, size_t n) {
  int saw = '^';
  size_t i = 0;
  if (n >= 1 && (s[0] == '-' || s[0] == '+')) { s++; n--; }
  int hex = 0;
  if (n >= 2 && s[0] == '0' && (lower_(s[1]) == 'b' || lower_(s[1]) == 'o' || lower_(s[1]) == 'x')) {
    i = 2; saw = '0'; hex = lower_(s[1]) == 'x';
  }
  for (; i < n; i++) {
    int c = (unsigned char)s[i];
    if ((c >= '0' && c <= '9') || (hex && lower_(c) >= 'a' && lower_(c) <= 'f')) { saw = '0'; continue; }
    if (c == '_') { if (saw != '0') return 0; saw = '_'; continue; }
    if (saw == '_') return 0;
    saw = '!';
  }
  return saw != '_';
}

static size_t common_prefix_ci(const char *s, size_t n, const char *pre) {
  size_t k = strlen(pre), i = 0;
  while (i < n && i < k && lower_((unsigned char)s[i]) == pre[i]) i++;
  return i;
}

int orc_parse_float(const char *s, size_t n, double *out) {
  /* special(): inf / infinity / nan, reference strconv/atof.go */
  if (n > 0) {
    size_t i = 0; int sign = 1; int tried_inf = 0;
    if (s[0] == '+' || s[0] == '-') { if (s[0] == '-') sign = -1; i = 1; tried_inf = 1; }
    if (tried_inf || lower_((unsigned char)s[0]) == 'i') {
      size_t k = common_prefix_ci(s + i, n - i, "infinity");
      if (k > 3 && k < 8) k = 3;
      if (k == 3 || k == 8) {
        if (i + k == n) { *out = sign * INFINITY; return 0; }
        return -1;
      }
    } else if (lower_((unsigned char)s[0]) == 'n') {
      if (common_prefix_ci(s, n, "nan") == 3) {
        if (n == 3) { *out = NAN; return 0; }
        return -1;
      }
    }
  }
  /* readFloat syntax */
  size_t i = 0;
  int underscores = 0, hex = 0;
  if (i >= n) return -1;
  if (s[i] == '+' || s[i] == '-') i++;
  int exp_char = 'e';
  if (i + 2 < n && s[i] == '0' && lower_((unsigned char)s[i + 1]) == 'x') { hex = 1; i += 2; exp_char = 'p'; }
  int sawdot = 0, sawdigits = 0;
  for (; i < n; i++) {
    int c = (unsigned char)s[i];
    if (c == '_') { underscores = 1; continue; }
    if (c == '.') { if (sawdot) break; sawdot = 1; continue; }
    if (c >= '0' && c <= '9') { sawdigits = 1; continue; }
    if (hex && lower_(c) >= 'a' && lower_(c) <= 'f') { sawdigits = 1; continue; }
    break;
  }
  if (!sawdigits) return -1;
  if (i < n && lower_((unsigned char)s[i]) == exp_char) {
    i++;
    if (i >= n) return -1;
    if (s[i] == '+' || s[i] == '-') i++;
    if (i >= n || s[i] < '0' || s[i] > '9') return -1;
    for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); i++)
      if (s[i] == '_') underscores = 1;
  } else if (hex) {
    return -1; /* hex mantissa must have an exponent */
  }
  if (underscores && !underscore_ok(s, i)) return -1;
  if (i != n) return -1; /* ParseFloat: whole string */
  /* value: correctly rounded (Go's ParseFloat is), via glibc strtod on the
     underscore-free text (glibc strtod rounds correctly, hex included). */
  char buf[512];
  char *tmp = n + 1 > sizeof(buf) ? malloc(n + 1) : buf;
  size_t w = 0;
  for (size_t k = 0; k < n; k++) if (s[k] != '_') tmp[w++] = s[k];
  tmp[w] = 0;
  errno = 0;
  char *endp;
  double v = strtod(tmp, &endp);
  if (tmp != buf) free(tmp);
  *out = v;
  if (isinf(v)) return -2; /* overflow -> ErrRange (underflow is not an error in Go) */
  return 0;
}

/* parseTimestamp: ns = int64(f*1e9) with amd64 CVTTSD2SQ semantics for
   out-of-range/NaN (0x8000000000000000).  Returns 0 ok. */
static int parse_ts(const char *s, size_t n, int64_t *ns) {
  double f;
  if (orc_parse_float(s, n, &f) != 0) return -1;
  volatile double x = f * 1e9;
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) *ns = INT64_MIN;
  else *ns = (int64_t)x;
  return 0;
}

/* time.Time.Sub for times built by time.Unix(0, ns): exact difference,
   saturated to [minDuration, maxDuration] (time.go Sub). */
static int64_t go_sub(int64_t t, int64_t u) {
  __int128 d = (__int128)t - (__int128)u;
  if (d > INT64_MAX) return INT64_MAX;
  if (d < INT64_MIN) return INT64_MIN;
  return (int64_t)d;
}

/* ----------------------------------------------------- net/netip parsing */

/* parseIPv4Fields: strict dotted quad, no leading zeros. */
static int parse_v4_fields(const char *s, size_t n, uint8_t f[4]) {
  int val = 0, pos = 0, dig = 0;
  for (size_t i = 0; i < n; i++) {
    int c = (unsigned char)s[i];
    if (c >= '0' && c <= '9') {
      if (dig == 1 && val == 0) return 0;
      val = val * 10 + (c - '0'); dig++;
      if (val > 255) return 0;
    } else if (c == '.') {
      if (i == 0 || i == n - 1 || s[i - 1] == '.') return 0;
      if (pos == 3) return 0;
      f[pos++] = (uint8_t)val; val = 0; dig = 0;
    } else return 0;
  }
  if (pos < 3) return 0;
  f[3] = (uint8_t)val;
  return 1;
}
static int hexv(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
/* netip.parseIPv6; zone => reject (net.ParseIP refuses zones). */
static int parse_v6(const char *in, size_t inlen, uint8_t ip[16]) {
  const char *s = in; size_t n = inlen;
  if (memchr(s, '%', n)) return 0;
  memset(ip, 0, 16);
  int ellipsis = -1;
  if (n >= 2 && s[0] == ':' && s[1] == ':') {
    ellipsis = 0; s += 2; n -= 2;
    if (n == 0) return 1;
  }
  int i = 0;
  while (i < 16) {
    size_t off = 0; uint32_t acc = 0;
    for (; off < n; off++) {
      int v = hexv((unsigned char)s[off]);
      if (v < 0) break;
      acc = (acc << 4) + (uint32_t)v;
      if (off > 3) return 0;
      if (acc > 0xFFFF) return 0;
    }
    if (off == 0) return 0;
    if (off < n && s[off] == '.') {
      if (ellipsis < 0 && i != 12) return 0;
      if (i + 4 > 16) return 0;
      if (!parse_v4_fields(s, n, ip + i)) return 0;
      n = 0; i += 4;
      break;
    }
    ip[i] = (uint8_t)(acc >> 8); ip[i + 1] = (uint8_t)acc; i += 2;
    s += off; n -= off;
    if (n == 0) break;
    if (s[0] != ':') return 0;
    if (n == 1) return 0;
    s++; n--;
    if (s[0] == ':') {
      if (ellipsis >= 0) return 0;
      ellipsis = i; s++; n--;
      if (n == 0) break;
    }
  }
  if (n != 0) return 0;
  if (i < 16) {
    if (ellipsis < 0) return 0;
    int k = 16 - i;
    for (int j = i - 1; j >= ellipsis; j--) ip[j + k] = ip[j];
    for (int j = ellipsis; j < ellipsis + k; j++) ip[j] = 0;
  } else if (ellipsis >= 0) return 0;
  return 1;
}
/* netip.ParseAddr dispatch on the first '.', ':' or '%'.  is4 set for IPv4 text. */
static int parse_addr(const char *s, size_t n, uint8_t out[16], int *is4) {
  for (size_t i = 0; i < n; i++) {
    if (s[i] == '.') {
      uint8_t f[4];
      if (!parse_v4_fields(s, n, f)) return 0;
      memset(out, 0, 10); out[10] = out[11] = 0xFF; memcpy(out + 12, f, 4);
      *is4 = 1; return 1;
    }
    if (s[i] == ':') { *is4 = 0; return parse_v6(s, n, out); }
    if (s[i] == '%') return 0;
  }
  return 0;
}
int orc_parse_ip(const char *s, size_t n, uint8_t out16[16]) {
  int is4;
  return parse_addr(s, n, out16, &is4);
}
static int to4(const uint8_t ip[16]) {
  for (int i = 0; i < 10; i++) if (ip[i]) return 0;
  return ip[10] == 0xFF && ip[11] == 0xFF;
}

/* ipfilter: plain/single IPs by canonical 16 bytes, plus subnets. */
typedef struct { uint8_t net[16]; uint8_t mask[16]; int netlen; /* 4 or 16 */ } Subnet;
typedef struct { Map ips; Subnet *sub; int nsub, csub; } IPFilter;

/* ipfilter ToggleIP(str, true): net.ParseCIDR, else net.ParseIP. */
static void filter_allow(IPFilter *f, const char *s, size_t n) {
  const char *slash = memchr(s, '/', n);
  if (slash) {
    uint8_t a[16]; int is4;
    size_t al = (size_t)(slash - s);
    const char *m = slash + 1; size_t ml = n - al - 1;
    int ok = parse_addr(s, al, a, &is4) && !memchr(s, '%', al);
    /* dtoi */
    size_t i = 0; long bits = 0;
    for (; i < ml && m[i] >= '0' && m[i] <= '9'; i++) { bits = bits * 10 + (m[i] - '0'); if (bits >= 0xFFFFFF) { ok = 0; break; } }
    if (i == 0 || i != ml) ok = 0;
    int bitlen = is4 ? 32 : 128;
    if (ok && bits >= 0 && bits <= bitlen) {
      if (bits == bitlen) { /* single address: f.ips[ip.String()] */
        Slot *sl = map_find(&f->ips, a, 16, 1); sl->v = (void *)1;
        return;
      }
      Subnet sn; memset(&sn, 0, sizeof sn);
      if (is4) {
        sn.netlen = 4;
        for (int k = 0; k < 4; k++) {
          int b = (int)bits - 8 * k; uint8_t mk = b >= 8 ? 0xFF : (b <= 0 ? 0 : (uint8_t)(0xFF << (8 - b)));
          sn.mask[k] = mk; sn.net[k] = a[12 + k] & mk;
        }
      } else {
        uint8_t net[16], mask[16];
        for (int k = 0; k < 16; k++) {
          int b = (int)bits - 8 * k; uint8_t mk = b >= 8 ? 0xFF : (b <= 0 ? 0 : (uint8_t)(0xFF << (8 - b)));
          mask[k] = mk; net[k] = a[k] & mk;
        }
        /* networkNumberAndMask: v4-mapped network => 4-byte compare with mask[12:] */
        if (to4(net)) { sn.netlen = 4; memcpy(sn.net, net + 12, 4); memcpy(sn.mask, mask + 12, 4); }
        else { sn.netlen = 16; memcpy(sn.net, net, 16); memcpy(sn.mask, mask, 16); }
      }
      if (f->nsub == f->csub) { f->csub = f->csub ? f->csub * 2 : 4; f->sub = realloc(f->sub, sizeof(Subnet) * f->csub); }
      f->sub[f->nsub++] = sn;
      return;
    }
    /* fall through to ParseIP of the whole string (fails: contains '/') */
    return;
  }
  uint8_t a[16];
  if (orc_parse_ip(s, n, a)) { Slot *sl = map_find(&f->ips, a, 16, 1); sl->v = (void *)1; }
}
/* IPFilter.Allowed(ipstr) with BlockByDefault=true and allow-only entries. */
static int filter_allowed(IPFilter *f, const char *s, size_t n) {
  uint8_t a[16];
  if (!orc_parse_ip(s, n, a)) return 0;
  if (map_find(&f->ips, a, 16, 0)) return 1;
  int v4 = to4(a);
  for (int i = 0; i < f->nsub; i++) {
    Subnet *sn = &f->sub[i];
    const uint8_t *ip = v4 ? a + 12 : a;
    int l = v4 ? 4 : 16;
    if (l != sn->netlen) continue;
    int ok = 1;
    for (int k = 0; k < l; k++) if ((sn->net[k] & sn->mask[k]) != (ip[k] & sn->mask[k])) { ok = 0; break; }
    if (ok) return 1;
  }
  return 0;
}

/* ------------------------------------------------------------ the config */

typedef struct {
  char *name; size_t name_len;
  gre *re;
  int64_t interval_ns, hits;
  int decision;
  Map skip; /* host -> 1 */
} Rule;

typedef struct { int *ids; int n, c; } IdList;
static void ids_push(IdList *l, int v) {
  if (l->n == l->c) { l->c = l->c ? l->c * 2 : 8; l->ids = realloc(l->ids, sizeof(int) * l->c); }
  l->ids[l->n++] = v;
}

typedef struct { Map exact; IPFilter allow; int has_allow; } Scope; /* decision lists of one scope */

struct orc_cfg {
  Rule *rules; int nrules, crules;
  IdList global;
  Map per_site;   /* site -> IdList* */
  Scope gscope;
  Map site_scope; /* site -> Scope* */
  Map disable_logging;
  int64_t ttl_s;
};

orc_cfg *orc_cfg_new(void) { return calloc(1, sizeof(orc_cfg)); }
static void free_idlist(void *p) { IdList *l = p; if (l) { free(l->ids); free(l); } }
static void free_scope(void *p) {
  Scope *s = p; if (!s) return;
  map_free(&s->exact, NULL); map_free(&s->allow.ips, NULL); free(s->allow.sub);
  if (p) free(s);
}
void orc_cfg_free(orc_cfg *c) {
  for (int i = 0; i < c->nrules; i++) { free(c->rules[i].name); gre_free(c->rules[i].re); map_free(&c->rules[i].skip, NULL); }
  free(c->rules); free(c->global.ids);
  map_free(&c->per_site, free_idlist);
  map_free(&c->gscope.exact, NULL); map_free(&c->gscope.allow.ips, NULL); free(c->gscope.allow.sub);
  map_free(&c->site_scope, free_scope);
  map_free(&c->disable_logging, NULL);
  free(c);
}

int orc_cfg_add_rule(orc_cfg *c, const char *site, size_t site_len, const char *name, size_t name_len,
                     const char *regex, size_t regex_len, int64_t interval_ns, int64_t hits, int decision,
                     char *err, size_t errlen) {
  gre *re = gre_compile(regex, regex_len, err, errlen);
  if (!re) return -1;
  if (c->nrules == c->crules) { c->crules = c->crules ? c->crules * 2 : 16; c->rules = realloc(c->rules, sizeof(Rule) * c->crules); }
  Rule *r = &c->rules[c->nrules];
  memset(r, 0, sizeof *r);
  r->name = malloc(name_len + 1); memcpy(r->name, name, name_len); r->name[name_len] = 0; r->name_len = name_len;
  r->re = re; r->interval_ns = interval_ns; r->hits = hits; r->decision = decision;
  int id = c->nrules++;
  if (!site) ids_push(&c->global, id);
  else {
    Slot *s = map_find(&c->per_site, site, site_len, 1);
    if (!s->v) s->v = calloc(1, sizeof(IdList));
    ids_push((IdList *)s->v, id);
  }
  return id;
}
void orc_cfg_add_skip_host(orc_cfg *c, int id, const char *host, size_t host_len) {
  Slot *s = map_find(&c->rules[id].skip, host, host_len, 1); s->v = (void *)1;
}
void orc_cfg_add_decision_ip(orc_cfg *c, const char *site, size_t site_len, int decision, const char *ip, size_t ip_len) {
  Scope *sc = &c->gscope;
  if (site) {
    Slot *s = map_find(&c->site_scope, site, site_len, 1);
    if (!s->v) s->v = calloc(1, sizeof(Scope));
    sc = s->v;
  }
  if (!memchr(ip, '/', ip_len)) { Slot *s = map_find(&sc->exact, ip, ip_len, 1); s->v = (void *)(intptr_t)decision; }
  if (decision == ORC_ALLOW) { sc->has_allow = 1; filter_allow(&sc->allow, ip, ip_len); }
}
void orc_cfg_set_expiring_ttl(orc_cfg *c, int64_t seconds) { c->ttl_s = seconds; }
void orc_cfg_add_disable_logging(orc_cfg *c, const char *host, size_t host_len) {
  Slot *s = map_find(&c->disable_logging, host, host_len, 1); s->v = (void *)1;
}

/* StaticDecisionLists.CheckIsAllowed(site, clientIp), decision.go:185-216 */
static int check_is_allowed(orc_cfg *c, const char *site, size_t sl, const char *ip, size_t il) {
  Slot *ss = map_find(&c->site_scope, site, sl, 0);
  if (ss) {
    Scope *sc = ss->v;
    Slot *e = map_find(&sc->exact, ip, il, 0);
    if (e && (intptr_t)e->v == ORC_ALLOW) return 1;
    if (sc->has_allow && filter_allowed(&sc->allow, ip, il)) return 1;
  }
  Slot *e = map_find(&c->gscope.exact, ip, il, 0);
  if (e && (intptr_t)e->v == ORC_ALLOW) return 1;
  if (c->gscope.has_allow && filter_allowed(&c->gscope.allow, ip, il)) return 1;
  return 0;
}

/* ------------------------------------------------------------- the state */

typedef struct { int64_t hits, start; } HitState;
typedef struct { int decision; int64_t expires; char *domain; size_t dl; } Expiring;

struct orc_state {
  Map ips;     /* ip -> 1 (ipToRegexStates keys) */
  Map states;  /* u32 iplen | ip | name -> HitState* */
  Map decisions; /* DynamicDecisionLists.expiringDecisionLists: ip -> Expiring* */
  char *banned_ip; size_t banned_len;
  char *log; size_t log_len, log_cap;
};

orc_state *orc_state_new(void) { return calloc(1, sizeof(orc_state)); }
static void free_exp(void *p) { Expiring *e = p; if (e) { free(e->domain); free(e); } }
void orc_state_free(orc_state *s) {
  map_free(&s->ips, NULL); map_free(&s->states, free); map_free(&s->decisions, free_exp);
  free(s->banned_ip); free(s->log); free(s);
}

static Slot *state_slot(orc_state *s, const char *ip, size_t il, const char *name, size_t nl, int create) {
  size_t kl = 4 + il + nl;
  char stackbuf[512];
  char *k = kl <= sizeof(stackbuf) ? stackbuf : malloc(kl);
  uint32_t l32 = (uint32_t)il;
  memcpy(k, &l32, 4); memcpy(k + 4, ip, il); memcpy(k + 4 + il, name, nl);
  Slot *sl = map_find(&s->states, k, kl, create);
  if (k != stackbuf) free(k);
  return sl;
}

/* RegexRateLimitStates.Apply, rate_limit.go:37-78 */
static void apply(orc_state *s, const char *ip, size_t il, const Rule *r, int64_t ts, int *seen_ip, int *mtype, int *exceeded) {
  HitState *st;
  *mtype = ORC_FIRST_TIME;
  Slot *ipslot = map_find(&s->ips, ip, il, 0);
  if (!ipslot) {
    *seen_ip = 0;
    map_find(&s->ips, ip, il, 1)->v = (void *)1;
    st = malloc(sizeof *st); st->hits = 1; st->start = ts;
    state_slot(s, ip, il, r->name, r->name_len, 1)->v = st;
  } else {
    *seen_ip = 1;
    Slot *rs = state_slot(s, ip, il, r->name, r->name_len, 0);
    if (rs) {
      st = rs->v;
      if (go_sub(ts, st->start) > r->interval_ns) { *mtype = ORC_OUTSIDE_INTERVAL; st->hits = 1; st->start = ts; }
      else { *mtype = ORC_INSIDE_INTERVAL; st->hits++; }
    } else {
      st = malloc(sizeof *st); st->hits = 1; st->start = ts;
      state_slot(s, ip, il, r->name, r->name_len, 1)->v = st;
    }
  }
  if (st->hits > r->hits) { st->hits = 0; *exceeded = 1; }
  else *exceeded = 0;
}

/* ---------------------------------------------------------- the Banner */

static void log_append(orc_state *s, const char *p, size_t n) {
  if (s->log_len + n + 1 > s->log_cap) {
    s->log_cap = (s->log_len + n + 1) * 2;
    s->log = realloc(s->log, s->log_cap);
  }
  memcpy(s->log + s->log_len, p, n); s->log_len += n;
}
typedef struct { char *b; size_t n, c; } Buf;
static void bput(Buf *b, const char *p, size_t n) {
  if (b->n + n + 1 > b->c) { b->c = (b->n + n + 1) * 2; b->b = realloc(b->b, b->c); }
  memcpy(b->b + b->n, p, n); b->n += n;
}
static void bputs(Buf *b, const char *s) { bput(b, s, strlen(s)); }

static int dec_rune(const char *s, size_t n, int *w) {
  unsigned char c = (unsigned char)s[0];
  if (c < 0x80) { *w = 1; return c; }
  int need = 0, r = 0; unsigned char lo = 0x80, hi = 0xBF;
  if (c >= 0xC2 && c <= 0xDF) { need = 1; r = c & 0x1F; }
  else if (c == 0xE0) { need = 2; lo = 0xA0; r = c & 0x0F; }
  else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) { need = 2; r = c & 0x0F; }
  else if (c == 0xED) { need = 2; hi = 0x9F; r = c & 0x0F; }
  else if (c == 0xF0) { need = 3; lo = 0x90; r = c & 0x07; }
  else if (c >= 0xF1 && c <= 0xF3) { need = 3; r = c & 0x07; }
  else if (c == 0xF4) { need = 3; hi = 0x8F; r = c & 0x07; }
  else { *w = 1; return 0xFFFD; }
  if ((size_t)need + 1 > n) { *w = 1; return 0xFFFD; }
  unsigned char b1 = (unsigned char)s[1];
  if (b1 < lo || b1 > hi) { *w = 1; return 0xFFFD; }
  r = (r << 6) | (b1 & 0x3F);
  for (int k = 2; k <= need; k++) {
    unsigned char bk = (unsigned char)s[k];
    if (bk < 0x80 || bk > 0xBF) { *w = 1; return 0xFFFD; }
    r = (r << 6) | (bk & 0x3F);
  }
  *w = need + 1; return r;
}
/* encoding/json string encoding with escapeHTML (json.Marshal), Go 1.22+ (\b, \f short forms) */
static void json_str(Buf *b, const char *s, size_t n) {
  static const char hex[] = "0123456789abcdef";
  bput(b, "\"", 1);
  size_t i = 0;
  while (i < n) {
    unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c >= 0x20 && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&') { bput(b, (const char *)&c, 1); i++; continue; }
      switch (c) {
      case '\\': bputs(b, "\\\\"); break;
      case '"': bputs(b, "\\\""); break;
      case '\b': bputs(b, "\\b"); break;
      case '\f': bputs(b, "\\f"); break;
      case '\n': bputs(b, "\\n"); break;
      case '\r': bputs(b, "\\r"); break;
      case '\t': bputs(b, "\\t"); break;
      default: { char u[7] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15], 0}; bputs(b, u); }
      }
      i++; continue;
    }
    /* multi-byte: utf8.DecodeRuneInString; invalid -> \ufffd */
    int need1; int r = dec_rune(s + i, n - i, &need1);
    int ok = !(r == 0xFFFD && need1 == 1);
    int need = need1 - 1;
    if (!ok) { bputs(b, "\\ufffd"); i++; continue; }
    if (r == 0x2028) bputs(b, "\\u2028");
    else if (r == 0x2029) bputs(b, "\\u2029");
    else bput(b, s + i, (size_t)need + 1);
    i += (size_t)need + 1;
  }
  bput(b, "\"", 1);
}

/* strings.TrimSpace (unicode.IsSpace) */
static int is_space_rune(int r) {
  switch (r) {
  case '\t': case '\n': case '\v': case '\f': case '\r': case ' ': case 0x85: case 0xA0:
  case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000: return 1;
  }
  return r >= 0x2000 && r <= 0x200A;
}
static void trim_space(const char **s, size_t *n) {
  while (*n > 0) { int w; int r = dec_rune(*s, *n, &w); if (!is_space_rune(r)) break; *s += w; *n -= (size_t)w; }
  while (*n > 0) {
    /* utf8.DecodeLastRuneInString */
    size_t start = *n - 1;
    int lim = 0;
    while (start > 0 && (((unsigned char)(*s)[start]) & 0xC0) == 0x80 && lim < 3) { start--; lim++; }
    int w; int r = dec_rune(*s + start, *n - start, &w);
    if ((size_t)w != *n - start) { r = 0xFFFD; w = 1; start = *n - 1; }
    if (!is_space_rune(r)) break;
    *n = start;
  }
}

static const char *decision_str(int d) {
  switch (d) { case 1: return "Allow"; case 2: return "Challenge"; case 3: return "NginxBlock"; case 4: return "IptablesBlock"; }
  return "";
}

/* time.Format("2006-01-02T15:04:05") in UTC (the injected TZ). */
static void fmt_time(int64_t ns, char out[64]) {
  int64_t sec = ns / 1000000000; if (ns % 1000000000 < 0) sec--;
  int64_t days = sec / 86400, rem = sec % 86400;
  if (rem < 0) { rem += 86400; days--; }
  /* civil_from_days (H. Hinnant) */
  int64_t z = days + 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  int64_t d = doy - (153 * mp + 2) / 5 + 1;
  int64_t m = mp < 10 ? mp + 3 : mp - 9;
  if (m <= 2) y++;
  snprintf(out, 64, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)m, (long long)d,
           (long long)(rem / 3600), (long long)(rem % 3600 / 60), (long long)(rem % 60));
}

/* Banner.LogRegexBan, iptables.go:179-228 */
static void log_regex_ban(orc_cfg *c, orc_state *s, int64_t ts, const char *ip, size_t il, const Rule *r,
                          const char *rest, size_t rl) {
  /* words := strings.SplitN(logLine, " ", 6) */
  const char *w[6]; size_t wl[6]; int nw = 0;
  const char *p = rest; size_t left = rl;
  while (nw < 5) {
    const char *sp = memchr(p, ' ', left);
    if (!sp) break;
    w[nw] = p; wl[nw] = (size_t)(sp - p); nw++;
    left -= (size_t)(sp - p) + 1; p = sp + 1;
  }
  w[nw] = p; wl[nw] = left; nw++;
  if (nw < 6) return; /* "not enough words" */
  int disable = map_find(&c->disable_logging, w[1], wl[1], 0) != NULL;
  const char *ua = w[5]; size_t ual = wl[5];
  const char *bar = memchr(ua, '|', ual);
  if (bar) ual = (size_t)(bar - ua);
  trim_space(&ua, &ual);
  char tbuf[64]; fmt_time(ts, tbuf);
  Buf b = {0};
  bputs(&b, disable ? "1 " : "0 ");
  bputs(&b, "{\"path\":"); json_str(&b, w[3], wl[3]);
  bputs(&b, ",\"timestring\":"); json_str(&b, tbuf, strlen(tbuf));
  bputs(&b, ",\"trigger\":"); json_str(&b, r->name, r->name_len);
  bputs(&b, ",\"client_ua\":"); json_str(&b, ua, ual);
  bputs(&b, ",\"client_ip\":"); json_str(&b, ip, il);
  bputs(&b, ",\"rule_type\":\"regex\",\"client_request_method\":"); json_str(&b, w[0], wl[0]);
  bputs(&b, ",\"http_request_scheme\":\"https\",\"client_request_host\":"); json_str(&b, w[1], wl[1]);
  bputs(&b, ",\"action\":"); json_str(&b, decision_str(r->decision), strlen(decision_str(r->decision)));
  char tail[64]; snprintf(tail, sizeof tail, ",\"number_of_fails\":1,\"disable_logging\":%d}\n", disable);
  bputs(&b, tail);
  log_append(s, b.b, b.n);
  free(b.b);
}

/* Banner.BanOrChallengeIp (iptables.go:273-294) -> DynamicDecisionLists.Update
   (decision.go:404-439), plus MockBanner's bannedIp bookkeeping. */
static void ban_or_challenge(orc_cfg *c, orc_state *s, const char *ip, size_t il, int decision,
                             const char *domain, size_t dl, int64_t now_ns) {
  free(s->banned_ip); s->banned_ip = malloc(il + 1); memcpy(s->banned_ip, ip, il); s->banned_len = il;
  int64_t expires = (int64_t)((uint64_t)now_ns + (uint64_t)c->ttl_s * 1000000000ULL);
  Slot *sl = map_find(&s->decisions, ip, il, 1);
  Expiring *e = sl->v;
  if (e && decision <= e->decision) return;
  if (!e) { e = calloc(1, sizeof *e); sl->v = e; }
  e->decision = decision; e->expires = expires;
  free(e->domain); e->domain = malloc(dl + 1); memcpy(e->domain, domain, dl); e->dl = dl;
}

/* ------------------------------------------------------------ consumeLine */

typedef struct {
  orc_rule_result *res; size_t cap, n;
} Out;

static void out_push(Out *o, orc_rule_result r) {
  if (o->n < o->cap) o->res[o->n] = r;
  o->n++;
}

/* applyRegexToLog, regex_rate_limiter.go:216-269 */
static void apply_rule(orc_cfg *c, orc_state *s, int id, uint16_t pos, uint64_t line_idx, const char *ip, size_t il,
                       const char *host, size_t hl, const char *rest, size_t rl, int64_t ts, int64_t now_ns, Out *o) {
  const Rule *r = &c->rules[id];
  if (!gre_match(r->re, (const uint8_t *)rest, rl)) return;
  orc_rule_result rr; memset(&rr, 0, sizeof rr);
  rr.line_idx = line_idx; rr.rule_id = (uint32_t)id; rr.rule_pos = pos;
  if (map_find((Map *)&r->skip, host, hl, 0)) { rr.skip_host = 1; out_push(o, rr); return; }
  int seen, mt, ex;
  apply(s, ip, il, r, ts, &seen, &mt, &ex);
  rr.seen_ip = (uint8_t)seen; rr.match_type = (uint8_t)mt; rr.exceeded = (uint8_t)ex;
  out_push(o, rr);
  if (ex) {
    ban_or_challenge(c, s, ip, il, r->decision, host, hl, now_ns);
    log_regex_ban(c, s, ts, ip, il, r, rest, rl);
  }
}

static int consume_line(orc_cfg *c, orc_state *s, const char *line, size_t n, uint64_t line_idx, int64_t now_ns, Out *o) {
  /* timeIpRest := strings.SplitN(line.Text, " ", 3) */
  const char *sp1 = memchr(line, ' ', n);
  if (!sp1) return ORC_LINE_ERROR;
  const char *ipb = sp1 + 1;
  const char *sp2 = memchr(ipb, ' ', (size_t)(line + n - ipb));
  if (!sp2) return ORC_LINE_ERROR;
  size_t il = (size_t)(sp2 - ipb);
  const char *rest = sp2 + 1; size_t rl = (size_t)(line + n - rest);
  int64_t ts;
  if (parse_ts(line, (size_t)(sp1 - line), &ts) != 0) return ORC_LINE_ERROR;
  /* methodUrlRest := strings.SplitN(timeIpRest[2], " ", 3) */
  const char *sp3 = memchr(rest, ' ', rl);
  if (!sp3) return ORC_LINE_ERROR;
  const char *host = sp3 + 1;
  const char *sp4 = memchr(host, ' ', (size_t)(rest + rl - host));
  if (!sp4) return ORC_LINE_ERROR;
  size_t hl = (size_t)(sp4 - host);
  if (go_sub(now_ns, ts) > 10000000000LL) return ORC_LINE_OLD;
  if (check_is_allowed(c, host, hl, ipb, il)) return ORC_LINE_EXEMPTED;
  uint16_t pos = 0;
  Slot *ps = map_find(&c->per_site, host, hl, 0);
  if (ps) {
    IdList *l = ps->v;
    for (int i = 0; i < l->n; i++) apply_rule(c, s, l->ids[i], pos++, line_idx, ipb, il, host, hl, rest, rl, ts, now_ns, o);
  }
  for (int i = 0; i < c->global.n; i++)
    apply_rule(c, s, c->global.ids[i], pos++, line_idx, ipb, il, host, hl, rest, rl, ts, now_ns, o);
  return 0;
}

int64_t orc_consume_batch(orc_cfg *c, orc_state *s, const uint8_t *buf, size_t n, int64_t now_ns, uint8_t *line_flags,
                          orc_rule_result *results, size_t cap, size_t *n_results, size_t *consumed) {
  Out o = {results, cap, 0};
  size_t pos = 0; int64_t li = 0;
  while (pos < n) {
    const uint8_t *nl = memchr(buf + pos, '\n', n - pos);
    if (!nl) break;
    size_t len = (size_t)(nl - (buf + pos));
    int f = consume_line(c, s, (const char *)buf + pos, len, (uint64_t)li, now_ns, &o);
    if (line_flags) line_flags[li] = (uint8_t)f;
    li++;
    pos += len + 1;
  }
  if (n_results) *n_results = o.n;
  if (consumed) *consumed = pos;
  return li;
}

int orc_state_get(orc_state *s, const char *ip, size_t il, const char *name, size_t nl, int64_t *hits, int64_t *start) {
  Slot *sl = state_slot(s, ip, il, name, nl, 0);
  if (!sl) return 0;
  HitState *h = sl->v; *hits = h->hits; *start = h->start;
  return 1;
}
int64_t orc_state_len(orc_state *s) { return (int64_t)s->ips.n; }
int orc_decision_get(orc_state *s, const char *ip, size_t il, int *decision, int64_t *expires, char *domain, size_t cap) {
  Slot *sl = map_find(&s->decisions, ip, il, 0);
  if (!sl) return 0;
  Expiring *e = sl->v;
  *decision = e->decision; *expires = e->expires;
  if (domain && cap) { size_t k = e->dl < cap - 1 ? e->dl : cap - 1; memcpy(domain, e->domain, k); domain[k] = 0; }
  return (int)e->dl + 1;  /* found: domain length + 1 (caller re-asks with a larger buffer) */
}
int64_t orc_decision_len(orc_state *s) { return (int64_t)s->decisions.n; }
/* DynamicDecisionLists.Clear (internal/decision.go:540-546), which the SIGHUP
   handler runs after a successful ConfigHolder.Reload (banjax.go:101-115) */
void orc_decision_clear(orc_state *s) { map_free(&s->decisions, free_exp); }
size_t orc_last_banned_ip(orc_state *s, char *out, size_t cap) {
  size_t k = s->banned_len < cap ? s->banned_len : cap;
  if (s->banned_ip && out) memcpy(out, s->banned_ip, k);
  return s->banned_len;
}
size_t orc_ban_log(orc_state *s, char *out, size_t cap) {
  size_t k = s->log_len < cap ? s->log_len : cap;
  if (out && s->log) memcpy(out, s->log, k);
  return s->log_len;
}
