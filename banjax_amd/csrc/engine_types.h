// Device-side data layout of the MI355X engine (see DESIGN.md "Data layout").
#pragma once
#include <stdint.h>

namespace bjx {

// One compiled rule as the kernels see it (rule tables live in one blob).
struct DevRule {
  uint32_t trans_off;   // u16 index into trans[]: row s starts at trans_off + s * ncls
  uint32_t ae_off;      // u8 index into accept_end[]
  uint32_t na_off;      // index into nonascii[] (pairs: lo, class)
  uint16_t n_na;
  uint16_t ncls;
  uint16_t start;
  uint16_t flags;       // kRuleAlways / kRuleNever
  uint32_t name_id;     // engine-wide interned rule name (state key, rate_limit.go:54)
  int32_t decision;
  uint32_t lits_off;     // prefilter literal ids: rule_lits[lits_off .. + lits_len)
  uint16_t lits_len;
  uint8_t mode;          // RuleMode
  uint8_t equiv;         // match <=> one of its literals occurs in rest
  uint32_t anc_off;      // anchored rules: prefix literal ids rule_lits[anc_off .. + anc_len)
  uint16_t anc_len;
  uint8_t anc_equiv;     // match <=> rest starts with one of them
  uint8_t lead;          // every match begins with a prefilter literal: a DFA job may start at its first hit
  uint32_t n_states;     // DFA states (rows of trans); NFA positions for kRuleNfa
  int64_t interval_ns;
  int64_t hits;
  uint32_t nfa_off;      // kRuleNfa: u64 index of the rule's tables in Bind::nfa
  uint32_t nfa_words;    // kRuleNfa: 64-bit words per state set (1, 2, 4, 8, 16)
  // anchored rule whose single case-sensitive prefix literal is checked before
  // a DFA job is made: k_dfa starts skip_len bytes in, in state skip_state
  uint16_t skip_len;
  uint16_t skip_state;
  // lead rules (CompiledRegex::lead_dist): a job starts this many bytes (plus
  // a rune's worth) before the first hit of the rule's literals
  uint16_t lead_dist;
};

// Bind::jinfo flags (word y; lead_dist in bits 16-31)
constexpr uint32_t kJiNfa = 1, kJiEquiv = 2, kJiBigLit = 16;  // bits 2-3: lead & 3

// Prefilter gram pair table (k_scan, LDS resident): 2048 entries of 8 B.
// The scan tests byte positions in pairs: positions k (even) and k + 1 share
// the 3 bytes k + 1 .. k + 3, which pick one entry (gram_pair_index); the gram
// at k is bit (its first byte & 31) of the entry's low word, the gram at
// k + 1 bit (its last byte & 31) of the high word.  A registered gram sets its
// bit in both roles (the entry of its last three bytes, low word; the entry of
// its first three bytes, high word), so no occurrence is missed at either
// parity.  gram_mix: the low 32 bits of a 24 x 24-bit product (one full-rate
// v_mul_u32_u24 on the device; only the key's low 24 bits count); its bits
// 13..23 pick the entry.  (Bits 34..44 of the full product spread cfg2's
// similar host literals worse: k_scan 17.5 -> 32 ms, round 4.)
constexpr uint32_t kPairEntries = 2048;
constexpr uint32_t kPairBytes = kPairEntries * 8;
constexpr uint32_t kGramMul = 0x2C1B3Bu;
__host__ __device__ inline uint32_t gram_mix(uint32_t x) {
#ifdef __HIP_DEVICE_COMPILE__
  return __umul24(x, kGramMul);
#else
  return (x & 0xFFFFFFu) * kGramMul;
#endif
}
__host__ __device__ inline uint32_t gram_pair_index(uint32_t key) { return (gram_mix(key) >> 13) & (kPairEntries - 1); }
__host__ __device__ inline uint32_t gram_pair_byte_off(uint32_t key) { return (gram_mix(key) >> 10) & ((kPairEntries - 1) << 3); }
// home slot of a gram in the exact gram table (cap a power of two <= 2^18):
// Fibonacci hashing, high product bits
__host__ __device__ inline uint32_t gram_slot(uint32_t g, uint32_t cap) { return ((g * 0x9E3779B1u) >> 14) & (cap - 1); }
constexpr int kCandSlots = 4;  // literal hits kept per line (more = overflow: every literal rule by DFA)
constexpr uint64_t kCandVerified = 1u << 23;  // hit bytes already checked by the scan pass

struct Subnet {
  uint8_t net[16];
  uint8_t mask[16];
  uint32_t netlen;  // 4 (IPv4 compare, To4 semantics) or 16
  uint32_t _pad;
};

struct ImgLayout {
  uint32_t gt, ge, ht, hrec, hid, hbytes, lrec, lbytes, lcim, lchk;
};

// Host dictionary slot for the per-line pass: one probe reads one 64 B line
// (tag, id and the host bytes inline; longer hosts compare in hd_bytes).
struct HostSlot {
  uint32_t tag;   // (hash >> 32) | 1; 0 = empty
  int32_t id;     // host id
  uint32_t len;
  uint32_t off;   // bytes in hd_bytes (hosts longer than 48 B)
  uint8_t inl[48];
};

// Everything the per-line kernels need about the current (ruleset, decision
// lists) pair.  All pointers are device pointers into one blob.
struct Bind {
  const DevRule *rules;
  const uint4 *jinfo;  // per rule: job-window facts for k_lines2 (engine.hip l2_job_rec; kJi* flags)
  const uint16_t *trans;
  const uint8_t *accept_end;
  // per DFA state (ae_off + state): 0, or 1 << 31 | n << 24 | e2 << 16 | e1 << 8 | e0
  // when every ASCII byte but the n <= 3 escape bytes e0..e2 maps the state to
  // itself (a `.*` loop waiting for a literal): dfa_text skips 16 B at a time
  const uint32_t *accel;
  const uint8_t *ascii_cls;    // 128 per rule
  const uint32_t *nonascii;    // (lo, class) pairs
  const uint8_t *lits;
  const uint32_t *global_rules;
  const uint32_t *site_off;    // n_hosts + 1
  const uint32_t *site_rules;
  const uint64_t *hd_hash;     // host dictionary sorted by hash
  const uint32_t *hd_id;
  const uint32_t *hd_off;
  const uint32_t *hd_len;
  const uint8_t *hd_bytes;
  const HostSlot *hslot;       // open addressing over the host dictionary, ht_cap slots
  const int32_t *host_scope;   // host id -> allow scope (or -1)
  const uint64_t *skip_keys;   // sorted (rule << 32 | host id)
  const uint32_t *sc_addr_off; // scopes + 1
  const uint64_t *sc_addr;     // 2 words per address, sorted per scope
  const uint32_t *sc_sub_off;
  const Subnet *sc_sub;
  const uint32_t *sc_str_off;
  const uint64_t *sc_str_hash; // sorted per scope
  const uint32_t *sc_str_boff;
  const uint32_t *sc_str_len;
  const uint8_t *sc_str_bytes;
  uint32_t n_rules;
  uint32_t n_global;
  uint32_t n_hosts;
  uint32_t n_hd;
  uint32_t n_skip;
  uint32_t n_scopes;
  uint32_t any_allow;
  uint32_t mask_words;         // ceil(max applicable rules per line / 64)
  // prefilter
  const uint2 *gram_pairs;     // kPairEntries: the prefilter's pair table (gram_pair_*)
  const uint32_t *rule_lits;
  uint32_t n_lits;
  uint32_t any_anchored;
  uint32_t any_prefilter;
  uint32_t lits_small;  // at most 32 interned literals: CandMeta bit id & 31 names one literal
  uint32_t lit_nl;  // some literal holds '\n' (k_scan then verifies only lines inside its window)
  uint32_t cfirst;  // ruleset of <= kCandFirstLits literals: Lines::cand_first is kept (stride kCandFirstLits)
  ImgLayout il;
  // Lookup image for the scan pass (one blob, copied whole to LDS when it
  // fits; ImgLayout gives the offsets):
  //   gram table  gt2_cap slots of (key, entries offset << 16 | count),
  //               entries (lit << 8 | window offset)
  //   host table  ht_cap slots of (hash tag, hd index); host records
  //               (bytes offset << 32 | len) and ids; host bytes
  //   literals    (bytes offset << 8 | len); bytes and case masks (0x20 where
  //               ASCII-case-insensitive), 4-byte aligned; check-window offsets
  const uint8_t *img;
  uint32_t img_bytes;
  // k_scan's own image (same layout, the ImgLayout sil): the gram table and
  // entries and the prefilter literals only (host fields unused)
  const uint8_t *scan_img;
  uint32_t scan_img_bytes;
  ImgLayout sil;
  uint32_t gt2_cap, gt2_nent;
  uint32_t ht_cap;
  uint32_t max_app;            // most rules applicable to one line (<= 128 on the scan path)
  // literal -> rules that require it: [lr_off[l], lr_gend[l]) global rules,
  // [lr_gend[l], lr_off[l+1]) site rules sorted by host (lr_host)
  const uint32_t *lr_off;
  const uint32_t *lr_gend;
  const uint2 *lr_ent;         // (rule | equiv << 31, index in its site / global list)
  const uint32_t *lr_full;     // per lr_ent: host-split literal (full literal << 8 | piece offset), or ~0
  const int32_t *lr_host;
  // (literal, host) -> that host's run of site entries of the literal:
  // lh_cap open-addressed slots {lit + 1 (0 = empty), host, begin, end}
  const uint4 *lh_tab;
  uint32_t lh_cap;
  // per scope (host id, or n_hosts = no per-site rules): 2-word masks over the
  // applicable-rule positions of ALWAYS rules and of hosts_to_skip hits
  const uint64_t *sc_always;
  const uint64_t *sc_skip;
  // rules that need a DFA on every line (anchored / no literal), and rules
  // with literals (used when a line overflows its hit slots)
  const uint32_t *dfa_site_off;  // n_hosts + 1
  const uint2 *dfa_site;         // (rule, index)
  const uint2 *dfa_glob;
  uint32_t n_dfa_glob;
  const uint4 *dfa_site_q;       // per dfa_site / dfa_glob entry: 2 x uint4 inline anchor test (anchor_quick)
  const uint4 *dfa_glob_q;
  const uint32_t *pref_site_off;
  const uint2 *pref_site;
  const uint2 *pref_glob;
  uint32_t n_pref_glob;
  // ALWAYS rules by position (the scopes past 128 positions, which sc_always
  // does not cover): site positions of host h [alw_site_off[h],
  // alw_site_off[h + 1]), global indices alw_glob
  const uint32_t *alw_site_off;
  const uint32_t *alw_site;
  const uint32_t *alw_glob;
  uint32_t n_alw_glob;
  // bit-parallel NFA tables of the kRuleNfa rules (DevRule::nfa_off)
  const uint64_t *nfa;
  uint32_t any_nfa;
  uint32_t any_wide;  // some rule is kRuleNfaWide (the per-line fallback lists those for k_nfa_wide)
  // rule plans (decide_plan): per rule of a scope that is neither ALWAYS nor
  // NEVER, one 32 B entry {a, b} holding everything its decision needs (kind,
  // position, literal ids, host-split full literal, inline anchor test), so a
  // line loads its host's entries side by side instead of walking the
  // literal -> rule tables.  Site entries of host h: [plan_off[h],
  // plan_off[h + 1]); global entries (position = nsite + g): plan_glob.
  // compact host dictionary for LDS (k_lines): {cap, n_hosts}, cap x {tag,
  // host id << 16 | len}, n_hosts byte offsets, the host bytes (4-byte padded);
  // hl_bytes = 0 when it does not fit kLinesHostLdsMax.  When lt_cls != 0 the
  // same blob goes on with the plan classes (decide_plan_lds), word offsets:
  // lt_hinfo (uint2 per host), lt_cls (class entries), lt_trec (templates),
  // lt_pool (template bytes)
  const uint32_t *hl;
  uint32_t hl_bytes;
  uint32_t lt_hinfo, lt_cls, lt_trec, lt_pool;
  // k_lines2 decision tables after the plan classes in the same blob (word
  // offsets; lines2.h): per-host decision class, class records, the class of
  // lines without a host; l2_bytes = the blob with them (0: k_lines2 off)
  uint32_t l2_hdc, l2_dcls, l2_none, l2_bytes;
  uint32_t l2_w;  // mask width of k_lines2's tables: 64-bit words of positions (1 or 2; k_lines2<W>)
  // k_dfa's LDS: transition entries / accel words staged per block (the
  // ruleset's largest DFA within kDfaLdsEntries / kDfaAccelLds), dynamic bytes
  uint32_t dfa_tr, dfa_acc, dfa_lds;
  const uint4 *plan;
  const uint32_t *plan_off;  // n_hosts + 1
  const uint4 *plan_glob;
  uint32_t n_plan_glob;
  uint32_t use_plan;
};

// Per-line SoA arrays (batch workspace).
// Per line, the scan pass's literal-hit summary: the first kCandSlots hits go
// to Lines::cand; past them (overflow) only which literals (bit = id & 63)
// and the lowest hit position are kept, which still rules out the literal
// rules whose literals are absent and starts the other DFA jobs at the first hit.
struct CandMeta {
  uint32_t cnt;        // hits recorded (slots hold the first kCandSlots)
  uint32_t first_inv;  // ~(lowest position >> 3) of the hits past the slots (0: none)
  uint64_t bits;       // past the slots: bit (literal id & 31) of every hit; bit 32 + (id & 31) of the
                       // verified ones at least kCertainGap bytes into the line
};
constexpr uint32_t kCertainGap = 256;

// A line's IP is at line start + rest_off - ip_len - 1 (the field before rest);
// its host field is re-derived from the line for the few lines that trip.
struct Lines {
  int64_t *ts;
  uint64_t *ip_hash;   // hash_bytes of the IP, stored only for IPs longer than 15 bytes
                       // (shorter ones: key16_hash of ip16, computed where it is needed)
  uint32_t *ip_len, *rest_off;
  int32_t *host_id;
  uint8_t *flags;
  uint64_t *counts;    // (n_results << 32) | n_events per line, then scanned in place
  uint64_t *masks;     // mask_words per line, word-major: word w of line j at masks[w * mstride + j]
                       // (consecutive lines' words adjacent: coalesced stores / loads for any width)
  uint64_t mstride;    // lines per mask word plane (the batch's line capacity)
  uint4 *ip16;         // key16 of the line's IP (see IpSlot)
  CandMeta *cand_meta;  // literal hits recorded by the scan pass (zeroed before it)
  uint64_t *cand;       // kCandSlots per line: (literal start << 24) | verified | literal id
  // rulesets of at most kCandFirstLits literals (Bind::cfirst): per line and
  // literal id, the lowest candidate position (~0: none), every hit counted
  uint64_t *cand_first;
  __host__ __device__ uint64_t &mword(uint64_t j, uint32_t w) const { return masks[(uint64_t)w * mstride + j]; }
};
constexpr uint32_t kCandFirstLits = 8;

// Persistent rate-limit state (RegexRateLimitStates, rate_limit.go:17-21),
// keyed by IP string and rule name, never evicted (as in the reference).
//   IP table: open addressing on the 64-bit hash of the IP bytes, one 16 B
//   slot per probe; the IP bytes live in the arena (id -> offset, length) and
//   every lookup of an IP created in an earlier batch compares them in full.
//   born = batch epoch that created the slot; first = smallest event-line
//   index of the batch that created it (seenIp of its first event).
struct IpSlot {
  uint64_t hash;  // 0 = empty
  uint32_t id;    // dense IP id (arena index)
  uint32_t born;  // epoch of creation (0 only while being claimed)
  uint4 key16;    // IP bytes 0..14 zero padded, byte 15 = min(len, 255): IPs of <= 15 bytes compare inline
};
//   State table: open addressing on key = ((ip_id + 1) << 24) | name_id,
//   one 32 B slot per probe (NumHitsAndIntervalStart, rate_limit.go:165-168).
struct StSlot {
  uint64_t key;    // 0 = empty
  int64_t hits;    // NumHits (Go int)
  int64_t start;   // IntervalStartTime, ns
  uint64_t valid;  // 0 = claimed this batch, no state yet (Apply's FirstTime branch)
};
struct State {
  IpSlot *ip;
  uint32_t *ip_first;  // per IP slot (meaningful while born == current epoch)
  uint64_t *ip_off;    // id -> arena offset
  uint32_t *ip_len;
  uint8_t *arena;
  StSlot *st;
  uint64_t *counters;  // [0] ips, [1] arena bytes, [2] states; per batch: [3] hash-collision lines,
                       // [5] / [7] IP / state claims over budget; [16 + 16 * shard + 0/1]: claims per
                       // block shard (engine.hip kClaimShards)
  uint64_t ip_mask;
  uint64_t st_mask;
  uint64_t arena_cap;
  // per IP id: state slot of (ip, hot_name) -- the name of the first global
  // rule that matches every line, whose events are one per line -- so
  // k_st_claim finds those slots without probing the state table; all ~0
  // after any rehash / rollback / clear (kNone = not cached, hot_name ~0 = off)
  uint32_t *ip_st;
  uint64_t ip_st_cap;
  uint32_t hot_name;
};

// One rate-limit event as the sort carries it (16 B): line timestamp, rule
// index | (first event of a new IP) << 31, event index (reference order).
// The kernels of the rate-limit stage read it through time / rule_id / seen
// (base: see EvRec12) and are instantiated for both record forms.
struct EvRec {
  int64_t ts;
  uint32_t rule;
  uint32_t ev;
  __host__ __device__ int64_t time(int64_t) const { return ts; }
  __host__ __device__ uint32_t rule_id() const { return rule & 0x7FFFFFFFu; }
  __host__ __device__ bool seen() const { return (rule >> 31) == 0; }
  __host__ __device__ static bool fits(int64_t, int64_t) { return true; }
  __host__ __device__ static EvRec make(int64_t ts, uint32_t r, bool first, uint32_t ev, int64_t) {
    EvRec v;
    v.ts = ts;
    v.rule = r | (first ? 0x80000000u : 0u);
    v.ev = ev;
    return v;
  }
};

// The 12-B form (the default for a local batch): ts - base in 44 bits (4.9 h
// of ns), the rule in 19, the first-event bit, then the event index.  The
// event sort moves 16 B per record instead of 20 per pass.  A batch with an
// event outside [base, base + 2^44) is claimed again in the 16-B form.
struct EvRec12 {
  uint32_t lo, hi, ev;
  static constexpr uint32_t kRuleBits = 19;
  static constexpr uint64_t kSpan = 1ull << 44;
  __host__ __device__ int64_t time(int64_t base) const {
    return (int64_t)((uint64_t)base + ((((uint64_t)hi & 0xFFFu) << 32) | lo));
  }
  __host__ __device__ uint32_t rule_id() const { return (hi >> 12) & ((1u << kRuleBits) - 1); }
  __host__ __device__ bool seen() const { return (hi >> 31) == 0; }
  __host__ __device__ static bool fits(int64_t ts, int64_t base) { return (uint64_t)ts - (uint64_t)base < kSpan; }
  __host__ __device__ static EvRec12 make(int64_t ts, uint32_t r, bool first, uint32_t ev, int64_t base) {
    const uint64_t d = (uint64_t)ts - (uint64_t)base;
    EvRec12 v;
    v.lo = (uint32_t)d;
    v.hi = ((uint32_t)(d >> 32) & 0xFFFu) | (r << 12) | (first ? 0x80000000u : 0u);
    v.ev = ev;
    return v;
  }
};

// Rate-limit input: the lines ("event lines") whose matched rules reach
// RegexRateLimitStates.Apply, and the events themselves in reference order.
// A local batch uses the line arrays directly (nl != nullptr: the IP is at
// line start + rest_off - ip_len - 1, the hash of an IP of <= 15 bytes comes
// from its inline key); records exchanged between GPUs carry explicit IP
// offsets into their own byte pool and every hash (nl == nullptr).
struct EvSrc {
  const uint8_t *bytes;
  const uint64_t *nl;
  const uint32_t *rest_off;
  const uint64_t *ip_pos;
  const uint32_t *ip_len;
  const uint64_t *ip_hash;
  uint64_t hmask;          // test hook (forced 64-bit hash collisions): hashes become (h & hmask) | 1; 0 = off
  const int64_t *ts;
  const uint64_t *counts;  // local batch: low 32 bits = events of line i; nullptr: every record has events
  const uint4 *ip16;       // local batch: per-line key16 of the IP; nullptr: built from the bytes
  uint64_t n;
};

enum LineFlagBits : uint8_t {
  kLineError = 1, kLineOld = 2, kLineExempt = 4,
  kLineTodo = 0x20,       // header not parsed by the scan pass: the per-line kernel (k_lines) does the line
  kLineSlowTs = 0x40,     // per-line fallback kernel (timestamp / long header)
  kLineLong = 0x80,       // line ends past the scan window: rules decided by k_resolve_long
};

}  // namespace bjx
