/*
 * ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Plain-C restatement of the banjax regex rate-limiting
 * log-tailer path; see bjx_oracle.c for the reference file:line each function
 * follows.  Parity is pinned by the reference's own known-answer tests
 * (tests/test_oracle_reference_kat.py) — see DESIGN.md "Oracle".
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Decision enum, reference internal/decision.go:20-28 */
enum { ORC_ALLOW = 1, ORC_CHALLENGE = 2, ORC_NGINX_BLOCK = 3, ORC_IPTABLES_BLOCK = 4 };
/* RateLimitMatchType, reference internal/rate_limit.go:175-181 */
enum { ORC_FIRST_TIME = 0, ORC_OUTSIDE_INTERVAL = 1, ORC_INSIDE_INTERVAL = 2 };
/* ConsumeLineResult flags, reference internal/regex_rate_limiter.go:80-85 */
enum { ORC_LINE_ERROR = 1, ORC_LINE_OLD = 2, ORC_LINE_EXEMPTED = 4 };

typedef struct orc_cfg orc_cfg;
typedef struct orc_state orc_state;

/* One RuleResult (reference regex_rate_limiter.go:87-93) of one line. */
typedef struct {
  uint64_t line_idx;
  uint32_t rule_id;    /* id returned by orc_cfg_add_rule */
  uint16_t rule_pos;   /* position in the line's evaluation order: per-site rules, then global */
  uint8_t skip_host;
  uint8_t seen_ip;
  uint8_t match_type;
  uint8_t exceeded;
  uint8_t _pad[2];
} orc_rule_result;

orc_cfg *orc_cfg_new(void);
void orc_cfg_free(orc_cfg *c);
/* Append a rule (YAML order). site==NULL: regexes_with_rates; else
   per_site_regexes_with_rates[site].  Returns rule id >= 0, or -1 with a
   Go-style compile error message in err (config.go:110-113). */
int orc_cfg_add_rule(orc_cfg *c, const char *site, size_t site_len, const char *name, size_t name_len,
                     const char *regex, size_t regex_len, int64_t interval_ns, int64_t hits_per_interval,
                     int decision, char *err, size_t errlen);
/* hosts_to_skip[host] = true for rule id (config.go:103, regex_rate_limiter.go:243). */
void orc_cfg_add_skip_host(orc_cfg *c, int rule_id, const char *host, size_t host_len);
/* One entry of global_decision_lists (site==NULL) or per_site_decision_lists[site]
   (decision.go:278-374).  Entries are applied in call order. */
void orc_cfg_add_decision_ip(orc_cfg *c, const char *site, size_t site_len, int decision, const char *ip,
                             size_t ip_len);
void orc_cfg_set_expiring_ttl(orc_cfg *c, int64_t seconds);
void orc_cfg_add_disable_logging(orc_cfg *c, const char *host, size_t host_len);

orc_state *orc_state_new(void);
void orc_state_free(orc_state *s);

/* consumeLine over every '\n'-terminated line of buf (a trailing partial line
   is left unconsumed, as hpcloud/tail does).  now_ns is the injected clock
   (time.Now()).  Writes line_flags[n_lines] (if non-NULL) and RuleResults in
   reference order into results (capacity cap; total count returned in
   *n_results even if it exceeds cap).  Returns the number of lines. */
int64_t orc_consume_batch(orc_cfg *c, orc_state *s, const uint8_t *buf, size_t n, int64_t now_ns,
                          uint8_t *line_flags, orc_rule_result *results, size_t cap, size_t *n_results,
                          size_t *consumed);

/* RegexRateLimitStates.Get(ip)[name] (rate_limit.go:81-96). Returns 1 if found. */
int orc_state_get(orc_state *s, const char *ip, size_t ip_len, const char *name, size_t name_len,
                  int64_t *num_hits, int64_t *start_ns);
/* RegexRateLimitStates.Len() (rate_limit.go:30-35). */
int64_t orc_state_len(orc_state *s);
/* DynamicDecisionLists entry for ip (decision.go:404-439); 1 if present. */
int orc_decision_get(orc_state *s, const char *ip, size_t ip_len, int *decision, int64_t *expires_ns,
                     char *domain, size_t domain_cap);
int64_t orc_decision_len(orc_state *s);
void orc_decision_clear(orc_state *s);
/* MockBanner.bannedIp (regex_rate_limiter_test.go:27-35). */
size_t orc_last_banned_ip(orc_state *s, char *out, size_t cap);
/* Banning-log JSON lines produced by LogRegexBan (iptables.go:179-228), each
   prefixed by "0 " (Logger) or "1 " (LoggerTemp) and ended by '\n'. */
size_t orc_ban_log(orc_state *s, char *out, size_t cap);

/* Go strconv.ParseFloat(s, 64) restated; returns 0 ok, -1 syntax, -2 range. */
int orc_parse_float(const char *s, size_t n, double *out);
/* net.ParseIP restated: returns 1 and 16-byte form if valid. */
int orc_parse_ip(const char *s, size_t n, uint8_t out16[16]);

#ifdef __cplusplus
}
#endif
