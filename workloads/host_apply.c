/* Compiled stand-in for the Go host's side of one batch's decisions (bench
 * tooling, not the product; the reference host is Go, absent from the image):
 *   - DynamicDecisionLists.Update once per device-built per-IP record
 *     (reference internal/decision.go:404-439: the entry is replaced only by a
 *     strictly more serious decision), in an open-addressing map keyed by the
 *     IP bytes, the way a Go map[string]ExpiringDecision is;
 *   - the LogRegexBan lines of the batch appended to a log file
 *     (internal/iptables.go:179-228 writes each with Logger.Println).
 * Works on the host arrays bjx_batch_bans returns (include/banjax_gpu.h). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/banjax_gpu.h"

typedef struct {
  uint64_t h;       /* 0 = empty */
  uint64_t key_off; /* IP bytes in keys[] */
  uint32_t key_len;
  int32_t decision;
  int64_t expires_ns;
} Ent;

static Ent *g_tab;
static uint64_t g_cap, g_n;
static char *g_keys;
static uint64_t g_keys_len, g_keys_cap;

static uint64_t fnv(const uint8_t *p, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h | 1;
}

static void grow(void) {
  const uint64_t nc = g_cap ? 2 * g_cap : 1u << 20;
  Ent *nt = (Ent *)calloc(nc, sizeof(Ent));
  for (uint64_t i = 0; i < g_cap; ++i)
    if (g_tab[i].h) {
      uint64_t s = g_tab[i].h & (nc - 1);
      while (nt[s].h) s = (s + 1) & (nc - 1);
      nt[s] = g_tab[i];
    }
  free(g_tab);
  g_tab = nt;
  g_cap = nc;
}

/* Update(ip, expires, decision, false, domain): returns 1 if the entry changed */
static int update(const uint8_t *ip, uint32_t len, int32_t decision, int64_t expires_ns) {
  if (4 * (g_n + 1) > 3 * g_cap) grow();
  const uint64_t h = fnv(ip, len);
  uint64_t s = h & (g_cap - 1);
  for (;;) {
    Ent *e = &g_tab[s];
    if (!e->h) {
      if (g_keys_len + len > g_keys_cap) {
        g_keys_cap = (g_keys_cap + len) * 2;
        g_keys = (char *)realloc(g_keys, g_keys_cap);
      }
      memcpy(g_keys + g_keys_len, ip, len);
      e->h = h; e->key_off = g_keys_len; e->key_len = len; e->decision = decision; e->expires_ns = expires_ns;
      g_keys_len += len;
      ++g_n;
      return 1;
    }
    if (e->h == h && e->key_len == len && memcmp(g_keys + e->key_off, ip, len) == 0) {
      if (decision <= e->decision) return 0;  /* only a more serious decision replaces the entry */
      e->decision = decision;
      e->expires_ns = expires_ns;
      return 1;
    }
    s = (s + 1) & (g_cap - 1);
  }
}

/* Applies one batch; returns wall seconds.  log_path NULL: no log file. */
double bjx_host_apply(const bjx_ban_batch *b, const char *log_path, uint64_t *changed) {
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  uint64_t ch = 0;
  for (uint64_t r = 0; r < b->n_ips; ++r)
    ch += (uint64_t)update(b->ip_bytes + b->ip_off[r], (uint32_t)(b->ip_off[r + 1] - b->ip_off[r]), b->ips[r].decision,
                           b->ips[r].expires_ns);
  if (log_path && b->log_bytes) {
    FILE *f = fopen(log_path, "ab");
    if (f) {
      fwrite(b->log, 1, b->log_bytes, f);
      fclose(f);
    }
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (changed) *changed = ch;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

uint64_t bjx_host_entries(void) { return g_n; }
