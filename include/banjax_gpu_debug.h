/*
 * banjax_gpu_debug.h — self-test hooks of libbanjax_gpu.so (not part of the
 * drop-in boundary; never used by bjx_process_batch).
 *
 * bjx_debug_rule_match_host evaluates one compiled rule's DFA or bit-parallel
 * NFA tables on the host, so the rule compiler can be checked against the oracle on machines
 * without a GPU.  The product matches on the GPU only.
 */
#ifndef BANJAX_GPU_DEBUG_H
#define BANJAX_GPU_DEBUG_H
#include <stddef.h>
#include <stdint.h>
#include "banjax_gpu.h"
#ifdef __cplusplus
extern "C" {
#endif
/* 1 match, 0 no match, <0 error */
int bjx_debug_rule_match_host(const bjx_ruleset *rs, size_t rule_idx, const uint8_t *text, size_t n);
/* required literal the prefilter uses for a rule (bytes written, full length returned) */
size_t bjx_debug_rule_literal(const bjx_ruleset *rs, size_t rule_idx, char *out, size_t cap);
/* a prefilter rule whose every match begins within a bounded distance of its
   literals (its DFA jobs start near the first hit): that distance in bytes;
   -1 for every other rule */
int bjx_debug_rule_lead(const bjx_ruleset *rs, size_t rule_idx);
/* Test hook: regexp/syntax's parse of one pattern alone (accept / refuse and
   Go's error text, e.g. the "expression too large" limits), no automaton. */
int bjx_debug_regex_parse(const char *pattern, size_t len, char *err, size_t err_len);
/* device ms of the last batch's phases: framing count, scan, per-line resolve,
   emit, capacity check, IP/state slot claim, sort + automaton, trips; then the
   node exchange as this engine saw it (bjx_events_partition to the start of
   its owner's rate-limit stage: partition, pack, the wait for the copies,
   unpack; 0 for a batch without one), which the capacity phase of a node
   batch contains (returns 9) */
size_t bjx_debug_phase_ms(bjx_engine *e, double *out, size_t cap);
/* device ms of the last batch's dominant kernels, from HIP events on the
   engine stream: k_scan, the per-line kernel, DFA-job sort + k_dfa / k_nfa;
   then which per-line kernel ran (2 = k_lines2, 1 = k_lines, 3 = the wide
   per-line kernel k_parse_match on every line: rulesets of more than 128
   global rules) and its window bytes per line (k_lines2) or staging bytes per
   wave (k_lines), 0 for k_parse_match (returns 5) */
size_t bjx_debug_kernel_ms(bjx_engine *e, double *out, size_t cap);
/* last batch: gram bitset hits, recorded literal hits, lines sent to the per-line
   fallback, lines decided by the long-line pass, DFA jobs; then the state
   tables: IP slots, IPs, state slots, states; then gram table hits, the
   rate-limit grouping (0: full sort by state slot; else two-level, 1 + the
   events of its oversized buckets), rate-limit runs that crossed a k_apply
   chunk (k_long_runs) (returns the count, 12) */
size_t bjx_debug_scan_stats(bjx_engine *e, uint64_t *out, size_t cap);
/* Test hook: IP hashes become (hash & mask) | 1 (0 = off), so distinct IPs
   share 64-bit hashes and the exact collision path of the IP table runs. */
int bjx_debug_set_ip_hash_mask(bjx_engine *e, uint64_t mask);
/* Test hook: the first claim launch of each table in a batch may add at most
   max_new entries (0 = off), forcing the roll-back / re-claim path. */
int bjx_debug_set_claim_budget(bjx_engine *e, uint64_t max_new);
/* Test hook: the per-IP state-slot cache of k_st_claim on (1), off (0) or as
   BJX_SLOT_CACHE / the default says (-1), from the next batch on. */
int bjx_debug_set_slot_cache(bjx_engine *e, int on);
/* Test hook: rules compiled afterwards use the bit-parallel NFA once their DFA
   passes `cap` states (0 = default 4096; 1 = every rule that fits the NFA),
   process-wide; clears the compiled-pattern cache. */
int bjx_debug_set_dfa_state_cap(uint32_t cap);
/* Test hook: rules compiled afterwards (on != 0) go straight to the wide
   block-cooperative NFA (kRuleNfaWide), process-wide; clears the
   compiled-pattern cache. */
int bjx_debug_force_wide_nfa(int on);
#ifdef __cplusplus
}
#endif
#endif
