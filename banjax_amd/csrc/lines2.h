// k_lines2: the per-line pass (consumeLine up to the rule loop,
// internal/regex_rate_limiter.go:113-214) over 112-byte line windows, with the
// rule decisions read from per-(decision class, literal) rows instead of a
// walk over every rule of the line's scope.  Included by engine.hip after
// k_lines, whose helpers it uses; DESIGN.md §4f.
//
// Window: each lane copies the 16 B-aligned 112 bytes that hold its line's
// first bytes into its own LDS window (7 x 16 B loads, 7 ds_write_b128); the
// header, the anchored windows at the start of rest and the template / literal
// checks around hits read it there, anything past it from HBM.  112 B = 28
// dwords per lane (an odd multiple of 4): lanes reading the same window offset
// with ds_read_b128 hit distinct banks.
//
// Decisions.  A decision class is one (site plan class, number of site rules,
// ALWAYS mask, hosts_to_skip mask) of the line's scope; its positions are the
// host's site rules then the global rules, at most 64 W (W = 1 or 2 words of
// position bits, the ruleset's widest scope; k_lines2<W>).  Per class and
// prefilter literal id one row holds:
//   eq   positions a hit of the literal matches outright (equivalent literal
//        rules, literal not host-split),
//   job  positions a hit sends to the automaton (non-equivalent literal rules),
//   lm   positions whose rule requires the literal (the overflow rule: a line
//        with more hits than slots sends a literal rule to its automaton when
//        one of its literals occurred),
//   chk  checks run around the hit: a template A + host + C (kPlanLitT) or a
//        host-split full literal (kPlanLit, equivalent), decided or sent to the
//        automaton per plan_rule / plan_rule_lds.
// Anchored and no-literal entries (kPlanAnchor, kPlanAnchorT, kPlanScan) are
// listed per class and evaluated on every line of the class, as before.  The
// decisions equal decide_plan_lds': the same entries, each decided by the same
// test, a DFA job wherever that test leaves the rule open (k_dfa decides those
// exactly, so a job for a rule also matched here is dropped, J & ~m).

// BJX_PROF_L2 (timing builds only): wave clocks per segment of k_lines2 into
// LinesArgs::prof: 0 window loads, 1 header + timestamp, 2 host lookup +
// CheckIsAllowed, 3 literal hits, 4 anchored entries, 5 jobs + inline automata,
// 6 per-line stores, 7 job flush
#ifdef BJX_PROF_L2
#define L2P(k)                       \
  do {                               \
    __builtin_amdgcn_s_waitcnt(0);   \
    P.mark(k);                       \
  } while (0)
#else
#define L2P(k) \
  do {         \
  } while (0)
#endif

constexpr uint32_t kL2Win = 112;  // bytes of each line's window (odd multiple of 16)
constexpr int kL2Block = 512;     // 8 waves; two blocks per CU
constexpr uint32_t kL2WaveLds = 64 * kL2Win + kWaveJobBytes;
constexpr uint32_t kL2TabMax = 20 * 1024;  // hl blob with the k_lines2 tables (LDS, per block)
constexpr uint32_t kL2ChkTmpl = 1, kL2ChkFull = 2;
constexpr uint32_t kL2AncWords = 12;
constexpr uint32_t kL2InlineSteps = 64;      // bytes an inline automaton steps from its job's start
constexpr uint32_t kL2NoStart = 0xFFFFFFFFu;  // inline entry without a start state (per-host rules: from the skip state only)
// class record (u32 words): ALWAYS, hosts_to_skip, any-hit jobs, overflow
// jobs, overflow jobs of literals with ids >= 32 (W 64-bit words each), then
// the rows, position -> rule, anchored entries (offset, count) and inline-DFA
// offsets; a literal's row: eq, job, lm (W 64-bit words each), checks
// (offset, count)
__host__ __device__ constexpr uint32_t l2_dcls_words(uint32_t w) { return (10 * w + 5 + 3) & ~3u; }
__host__ __device__ constexpr uint32_t l2_row_words(uint32_t w) { return (6 * w + 2 + 3) & ~3u; }

// W-word position masks
template <int W>
struct L2Mask {
  uint64_t w[W];
};
template <int W>
__device__ __forceinline__ L2Mask<W> l2_ld_mask(const uint32_t *hl, uint32_t at) {
  L2Mask<W> m;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    const uint2 v = *reinterpret_cast<const uint2 *>(hl + at + 2 * k);
    m.w[k] = ((uint64_t)v.y << 32) | v.x;
  }
  return m;
}
template <int W>
__device__ __forceinline__ void l2_or(L2Mask<W> &a, const L2Mask<W> &b) {
#pragma unroll
  for (int k = 0; k < W; ++k) a.w[k] |= b.w[k];
}
template <int W>
__device__ __forceinline__ void l2_set(L2Mask<W> &a, uint32_t p) {
#pragma unroll
  for (int k = 0; k < W; ++k)
    if ((p >> 6) == (uint32_t)k) a.w[k] |= 1ull << (p & 63);
}
template <int W>
__device__ __forceinline__ bool l2_has(const L2Mask<W> &a, uint32_t p) {
  bool r = false;
#pragma unroll
  for (int k = 0; k < W; ++k)
    if ((p >> 6) == (uint32_t)k) r = (a.w[k] >> (p & 63)) & 1;
  return r;
}

// up to four spaces of mask m (bit i = line byte base + i) appended to sp0..sp3
__device__ __forceinline__ void l2_take_spaces(uint64_t m, int32_t base, uint32_t &ns, uint32_t &sp0, uint32_t &sp1,
                                               uint32_t &sp2, uint32_t &sp3) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool has = m != 0 && ns < 4;
    const uint32_t pos = (uint32_t)((int32_t)__ffsll((unsigned long long)m) - 1 + base);
    m &= m - 1;
    sp0 = has && ns == 0 ? pos : sp0;
    sp1 = has && ns == 1 ? pos : sp1;
    sp2 = has && ns == 2 ? pos : sp2;
    sp3 = has && ns == 3 ? pos : sp3;
    ns += has ? 1u : 0u;
  }
}

// first four spaces of line bytes [0, n): the window (line byte o at win[sk +
// o]) 64 bytes at a time, then HBM past it (gp = line start)
__device__ __forceinline__ uint32_t l2_spaces(const uint8_t *win, uint32_t sk, const uint8_t *gp, uint32_t n, uint32_t &sp0,
                                              uint32_t &sp1, uint32_t &sp2, uint32_t &sp3) {
  const uint4 *w = reinterpret_cast<const uint4 *>(win);
  uint32_t ns = 0;
  {
    const uint4 v0 = w[0], v1 = w[1], v2 = w[2], v3 = w[3];
    uint64_t m = (uint64_t)space_mask16(v0) | ((uint64_t)space_mask16(v1) << 16) | ((uint64_t)space_mask16(v2) << 32) |
                 ((uint64_t)space_mask16(v3) << 48);
    m &= ~((1ull << sk) - 1ull);
    if (sk + n < 64) m &= (1ull << (sk + n)) - 1ull;
    l2_take_spaces(m, -(int32_t)sk, ns, sp0, sp1, sp2, sp3);
  }
  if (ns < 4 && sk + n > 64) {
    const uint4 v4 = w[4], v5 = w[5], v6 = w[6];
    uint64_t m = (uint64_t)space_mask16(v4) | ((uint64_t)space_mask16(v5) << 16) | ((uint64_t)space_mask16(v6) << 32);
    if (sk + n < kL2Win) m &= (1ull << (sk + n - 64)) - 1ull;
    l2_take_spaces(m, 64 - (int32_t)sk, ns, sp0, sp1, sp2, sp3);
  }
  const uint32_t lim = kL2Win - sk;
  if (ns < 4 && n > lim) {  // a header longer than the window: the rest from HBM
    uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    const uint32_t nq = find_spaces(gp + lim, n - lim, q0, q1, q2, q3);
    const uint32_t q[4] = {q0, q1, q2, q3};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const bool has = k < nq && ns < 4;
      const uint32_t pos = q[k] + lim;
      sp0 = has && ns == 0 ? pos : sp0;
      sp1 = has && ns == 1 ? pos : sp1;
      sp2 = has && ns == 2 ? pos : sp2;
      sp3 = has && ns == 3 ? pos : sp3;
      ns += has ? 1u : 0u;
    }
  }
  return ns;
}

struct L2Line {
  const uint8_t *wp;  // LDS: line byte 0 in the window
  const uint8_t *gp;  // HBM: line byte 0
  uint32_t lim;       // line bytes [0, lim) are in the window
  uint32_t n;         // line length
};
// [o, o + len) plus ld4's slack lies in the window
__device__ __forceinline__ bool l2_in(const L2Line &X, uint32_t o, uint32_t len) { return o + len + 8 <= X.lim; }

// one anchored / no-literal entry (a, b) at position pos of the class
// (plan_rule / plan_rule_lds for kinds kPlanAnchor, kPlanAnchorT, kPlanScan):
// 1 = matched, 2 = DFA job, 0 = no match
template <bool LDS_TEXT>
__device__ __forceinline__ uint32_t l2_anchored(const Bind &B, const Tabs &T, const LdsTabs &LT, const uint4 a, const uint4 b,
                                                uint32_t r, const uint8_t *rest, uint32_t rest_len, uint32_t host_rel,
                                                uint32_t host_len) {
  const uint32_t kind = (a.x >> 27) & 7u;
  const bool eq = ((a.x >> 30) & 1u) != 0;
  if (kind == kPlanScan) return 2;
  if (kind == kPlanAnchorT) {
    if (!tmpl_at(LT, a.w, rest, rest_len, host_rel, host_len, 0)) return 0;
    return eq ? 1u : 2u;
  }
  // kPlanAnchor
  const uint4 qa = make_uint4(a.y, a.z, b.x, b.y), qb = make_uint4(b.z, b.w, 0, 0);
  const uint32_t qk = anchor_quick(qa, qb, rest, rest_len);
  if (qk == 0) return 0;
  if (qk == 1 && ((qa.y >> 9) & 1)) return 1;
  if (a.w) {
    if (!((a.w >> 16) <= rest_len && literal_at(T, (a.w & 0xFFFFu) - 1, rest))) return 0;
    return eq ? 1u : 2u;
  }
  // dfa_rule's anchored branch: the rule's prefix literals
  const DevRule &R = B.rules[r];
  if (R.anc_len) {
    bool any = false;
    for (uint32_t i = 0; i < R.anc_len && !any; ++i) {
      const uint32_t lit = B.rule_lits[R.anc_off + i];
      any = lit_len_of(T, lit) <= rest_len && literal_at(T, lit, rest);
    }
    if (!any) return 0;
    if (R.anc_equiv) return 1;
  }
  return 2;
}

// one check of a literal's row around its hit at rest offset hp: 1 matched,
// 2 job, 0 not here (a later hit of the literal may still decide it)
template <bool LDS_TEXT>
__device__ __forceinline__ uint32_t l2_check(const Tabs &T, const LdsTabs &LT, const uint4 ck, const uint8_t *rest,
                                             uint32_t rest_len, uint32_t host_rel, uint32_t host_len, uint32_t hp) {
  const uint32_t kind = (ck.x >> 8) & 3u;
  const bool eq = ((ck.x >> 10) & 1u) != 0;
  if (kind == kL2ChkTmpl) {
    const uint4 rec = LT.trec[ck.y];
    const uint32_t la = rec.x & 0xFF;
    const bool side_c = ((rec.x >> 16) & 1u) != 0;
    const int32_t fs = side_c ? (int32_t)hp - (int32_t)host_len - (int32_t)la : (int32_t)hp;
    if (!tmpl_at(LT, ck.y, rest, rest_len, host_rel, host_len, fs)) return 0;
    return eq ? 1u : 2u;
  }
  // host-split full literal of an equivalent rule (plan_rule)
  const uint32_t fl = ck.y >> 8, off = ck.y & 0xFFu;
  return hp >= off && hp - off + ck.z <= rest_len && literal_at(T, fl, rest + (hp - off)) ? 1u : 0u;
}

// The window record of a DFA job (engine.hip kJob*), or kJobDecided when the
// pair is decided here: k_dfa's eq_certain, skip and lead_start steps on the
// line's hit slots in registers (or, for rulesets with first-hit tables,
// cfirst, from the line's first candidate of each literal).  Lead seeks past
// overflowed slots, rules with literal ids >= 32 and NFA rules stay with k_dfa
// (kJobLegacy).
constexpr uint64_t kJobDecided = ~0ull;
__device__ __forceinline__ uint64_t l2_job_rec(const Bind &B, uint32_t r, const CandMeta &cm, const uint64_t (&cv)[kCandSlots],
                                               uint64_t rs, uint32_t rl, uint32_t rest_off, const uint64_t *cfirst) {
  // one 16 B load: Bind::jinfo[r] (a class entry naming another rule names one
  // with the same pattern, so its literals and flags are the line's own)
  const uint4 ji = B.jinfo[r];
  const uint32_t lm = ji.x, fl = ji.y, lead = (fl >> 2) & 3u;
  if (fl & (kJiNfa | kJiBigLit)) return kJobLegacy;
  const bool ovf = cm.cnt > (uint32_t)kCandSlots;
  const uint32_t ns = min(cm.cnt, (uint32_t)kCandSlots);
  auto mine = [&](uint64_t v) {
    const uint32_t id = (uint32_t)(v & 0x7FFFFF);
    return id < 32 && ((lm >> id) & 1u);
  };
  if ((fl & kJiEquiv) && (lead & 2u)) {  // eq_certain
#pragma unroll
    for (uint32_t c = 0; c < (uint32_t)kCandSlots; ++c) {
      if (c >= ns) break;
      const uint64_t v = cv[c];
      if ((v & kCandVerified) && (v >> 24) >= rs && mine(v)) return kJobDecided;
    }
    if (ovf && B.lits_small && rest_off <= kCertainGap && ((cm.bits >> 32) & lm) != 0) return kJobDecided;
  }
  const uint32_t skl = ji.z & 0xFFFFu;
  const uint32_t sk = skl && skl <= rl ? skl : 0u;
  uint32_t st0 = 0;
  if (lead == 3u && B.cfirst) {
    // lead_start from the line's first candidate of each of the rule's
    // literals (rulesets of <= kCandFirstLits literals: exact, overflow or not)
    const uint32_t ld = fl >> 16, back = ld ? ld + 3u : 0u;
    uint64_t f = ~0ull;
    for (uint32_t m = lm; m; m &= m - 1) {
      const uint64_t q = cfirst[(uint32_t)__ffs(m) - 1];
      f = q < f ? q : f;
    }
    if (f == ~0ull) st0 = rl;  // none of its literals occurs: no match
    else {
      // a first candidate in the header still bounds the first one in rest from below
      const uint32_t o = f <= rs ? 0u : (uint32_t)min<uint64_t>(f - rs, rl);
      st0 = o > back ? o - back : 0u;
    }
  } else if (lead == 3u) {  // lead_start (lead & 1 gates it, lead & 3 == 3 runs it)
    const uint32_t ld = fl >> 16, back = ld ? ld + 3u : 0u;
    uint64_t f = ~0ull;
#pragma unroll
    for (uint32_t c = 0; c < (uint32_t)kCandSlots; ++c) {
      if (c >= ns) break;
      const uint64_t v = cv[c];
      const uint64_t q = v >> 24;
      if (q < rs || q >= f) continue;
      if (ovf || mine(v)) f = q;
    }
    bool zero = false;
    if (ovf) {
      const uint64_t mf = cm.first_inv ? (uint64_t)(~cm.first_inv) << 3 : ~0ull;
      if (mf < rs) zero = true;
      f = mf < f ? mf : f;
    }
    if (!zero) {
      if (f == ~0ull) st0 = rl;
      else {
        const uint32_t o = (uint32_t)min<uint64_t>(f - rs, rl);
        st0 = o > back ? o - back : 0u;
      }
    }
    // lead_start_seek: past overflowed slots the start is the first hit of ANY
    // literal; k_dfa seeks forward to the rule's own
    if (st0 < rl && ovf) return kJobLegacy;
  }
  if (st0) return rs + st0;
  return (rs + sk) | (sk ? kJobSkipState : 0ull);
}

__device__ __forceinline__ uint4 l2_ld4w(const uint32_t *hl, uint32_t w) { return *reinterpret_cast<const uint4 *>(hl + w); }

// A job's automaton run here, over the line's window, for a rule with an
// inline table (entry word `ent` of the blob: {next-state table byte offset,
// accept-at-end byte offset, start state, skip state}; u8 next states over
// ASCII bytes): 1 matched, 0 no match, 2 undecided (the decision lies past
// the window, or a non-ASCII byte needs rune decoding: the job goes to k_dfa).
// A table shared by per-host rules holds only the automaton past their
// anchored prefix (start kL2NoStart): a job that does not begin there stays a
// job.
// The same steps as dfa_line from the job's start: stop at the dead or accept
// state, or at the line's end with the accept-at-end flag.
__device__ __forceinline__ uint32_t l2_inline(const uint32_t *hl, uint32_t ent, const L2Line &X, uint64_t s, uint64_t rec) {
  const uint4 e = l2_ld4w(hl, ent);
  const uint8_t *tr = reinterpret_cast<const uint8_t *>(hl) + e.x;
  const uint8_t *ae = reinterpret_cast<const uint8_t *>(hl) + e.y;
  if (!(rec & kJobSkipState) && e.z == kL2NoStart) return 2;  // a table from the skip state only
  uint32_t st = (rec & kJobSkipState) ? e.w : e.z;
  uint32_t o = (uint32_t)((rec & kJobOffMask) - s);
  // at most kL2InlineSteps bytes from the job's start: a rule that decides
  // near its literal does so within them; one scanning on (a .* after its
  // literal, no match) stays a job instead of walking the line here
  const uint32_t stop = min(X.n, o + kL2InlineSteps);
  const uint32_t lim = min(stop, X.lim);
  // in the window: four text bytes per LDS word load, so each step waits on
  // its table load only
  while (o + 4 <= lim) {
    const uint32_t w = ld4(X.wp + o);
    if (w & 0x80808080u) break;  // a non-ASCII byte ahead: stepped one by one below
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      st = tr[st * 128u + ((w >> (8 * k)) & 0xFFu)];
      if (st <= 1) return st == kAccept ? 1u : 0u;
    }
    o += 4;
  }
  for (; o < lim; ++o) {
    const uint32_t b = X.wp[o];
    if (b >= 0x80) return 2;
    st = tr[st * 128u + b];
    if (st <= 1) return st == kAccept ? 1u : 0u;
  }
  // past the window (a lead rule's job starts at its literal's first hit,
  // often far into a long line): from HBM, 16 B aligned loads stepped from
  // registers
  const uint32_t end = stop;
  while (o < end) {
    const uint32_t al = (uint32_t)(reinterpret_cast<uintptr_t>(X.gp + o) & 15);
    // the aligned 16 B are read whole only while they end at or before the
    // line's '\n' (every line of a batch has one): no read past the batch
    uint4 v = make_uint4(0, 0, 0, 0);
    if (16 - al <= X.n + 1 - o) v = *reinterpret_cast<const uint4 *>(X.gp + o - al);
    else {
      uint32_t t[4] = {0, 0, 0, 0};
      for (uint32_t k = al; k < 16 && o + (k - al) <= X.n; ++k) t[k >> 2] |= (uint32_t)X.gp[o + (k - al)] << (8 * (k & 3));
      v = make_uint4(t[0], t[1], t[2], t[3]);
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint32_t k = al; k < 16 && o < end; ++k, ++o) {
      const uint32_t b = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      if (b >= 0x80) return 2;
      st = tr[st * 128u + b];
      if (st <= 1) return st == kAccept ? 1u : 0u;
    }
  }
  if (o < X.n) return 2;
  return ae[st] ? 1u : 0u;
}

template <int W>
__global__ __launch_bounds__(kL2Block, 4) void k_lines2(Bind B, LinesArgs A) {
  constexpr uint32_t DW = l2_dcls_words(W), RW = l2_row_words(W);
  uint32_t *s_hl = reinterpret_cast<uint32_t *>(s_dyn);
  for (uint32_t i = threadIdx.x; i < B.l2_bytes / 16; i += blockDim.x)
    reinterpret_cast<uint4 *>(s_hl)[i] = reinterpret_cast<const uint4 *>(B.hl)[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint8_t *wbase = s_dyn + B.l2_bytes + wave * kL2WaveLds;
  uint8_t *win = wbase + lane * kL2Win;
  JobSink S;
  S.lds = reinterpret_cast<uint4 *>(wbase + 64 * kL2Win);
  S.cnt = reinterpret_cast<uint32_t *>(S.lds + kWaveJobs);
  S.jline = A.jline;
  S.jkey = A.jkey;
  S.jidx = A.jidx;
  S.jrec = A.jrec;
  S.n_rules = B.n_rules;
  S.count = A.job_count;
  S.cap = A.job_cap;
  if (lane == 0) *S.cnt = 0;
  wave_sync();
  JobChunk JC;
  const Tabs TB = make_tabs(B.img, B.il);
  LdsTabs LT;
  LT.hinfo = reinterpret_cast<const uint2 *>(s_hl + B.lt_hinfo);
  LT.cls = reinterpret_cast<const uint4 *>(s_hl + B.lt_cls);
  LT.trec = reinterpret_cast<const uint4 *>(s_hl + B.lt_trec);
  LT.pool = reinterpret_cast<const uint8_t *>(s_hl + B.lt_pool);
  const Lines &L = A.L;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
#ifdef BJX_PROF_L2
  LinesProf P;
  P.start();
#endif
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + wave * 64u; base < A.n_lines; base += stride) {
    const uint64_t j = base + lane;
    const bool act = j < A.n_lines;
    uint64_t s = 0;
    uint32_t n = 0;
    CandMeta cm{0, 0, 0};
    uint64_t cv[kCandSlots] = {0, 0, 0, 0};
    if (act) {
      s = j ? A.nl[j - 1] + 1 : 0;
      n = (uint32_t)(A.nl[j] - s);
      if (B.any_prefilter) cm = L.cand_meta[j];  // before the window loads: waited for alone
    }
    // ---- the line's window: 16 B-aligned pieces from its first byte
    const uint64_t a0 = s & ~15ull;
    const uint32_t sk = (uint32_t)(s - a0);
    {
      uint4 v[kL2Win / 16];
#ifdef BJX_L2_TLOAD
      // the wave's 64 windows as 448 pieces of 16 B, piece g = 7 line + k at
      // wbase + 16 g: in step k lane l loads piece 64 k + l, so consecutive
      // lanes read consecutive 16 B of one line (about 9 lines, 18 cache lines
      // per instruction instead of 64) and write one contiguous 1 KB of LDS.
      // A line's window start comes from its lane (offset from lane 0's).
      const uint64_t w0 = __shfl(a0, 0);
      const uint32_t rel = (uint32_t)(a0 - w0);
#pragma unroll
      for (uint32_t k = 0; k < kL2Win / 16; ++k) {
        const uint32_t g = 64u * k + lane;
        const uint32_t ln = (g * 9363u) >> 16;  // g / 7 for g < 448
        const uint64_t a = w0 + __shfl(rel, (int)ln) + 16ull * (g - 7u * ln);
#else
#pragma unroll
      for (uint32_t k = 0; k < kL2Win / 16; ++k) {
        const uint64_t a = a0 + 16ull * k;
#endif
        if (a + 16 <= A.n) v[k] = *reinterpret_cast<const uint4 *>(A.buf + a);
        else {
          uint32_t w4[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t x = 0;
            for (int bb = 0; bb < 4; ++bb) {
              const uint64_t p = a + 4 * q + bb;
              if (p < A.n) x |= (uint32_t)A.buf[p] << (8 * bb);
            }
            w4[q] = x;
          }
          v[k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
      }
      // the hit slots the scan filled (most lines have none or one: 16 B, not 32)
      if (act && B.any_prefilter && cm.cnt) {
        const ulonglong2 *cp = reinterpret_cast<const ulonglong2 *>(L.cand + j * kCandSlots);
        const ulonglong2 w0 = cp[0];
        cv[0] = w0.x;
        cv[1] = w0.y;
        if (cm.cnt > 2) {
          const ulonglong2 w1 = cp[1];
          cv[2] = w1.x;
          cv[3] = w1.y;
        }
      }
#ifdef BJX_L2_TLOAD
#pragma unroll
      for (uint32_t k = 0; k < kL2Win / 16; ++k) reinterpret_cast<uint4 *>(wbase)[64u * k + lane] = v[k];
      wave_sync();  // every lane reads the window its neighbours wrote
#else
#pragma unroll
      for (uint32_t k = 0; k < kL2Win / 16; ++k) reinterpret_cast<uint4 *>(win)[k] = v[k];
#endif
    }
    L2P(0);
    if (act) {
      L2Line X;
      X.wp = win + sk;
      X.gp = A.buf + s;
      X.lim = kL2Win - sk;
      X.n = n;
      uint32_t sp0 = 0, sp1 = 0, sp2 = 0, sp3 = 0;
      const uint32_t ns = l2_spaces(win, sk, X.gp, n, sp0, sp1, sp2, sp3);
      double f = 0.0;
      bool slow = false;
      if (ns >= 4) slow = parse_ts_msec(X.wp, sp0, &f) != 0 && parse_float_fast(X.wp, sp0, &f) != 0;
      L2P(1);
      if (ns < 4) {
        L.flags[j] = kLineError;
        L.counts[j] = 0;
      } else if (slow) {  // exotic timestamp token: the per-line fallback
        L.flags[j] = kLineSlowTs;
        L.counts[j] = 0;
        push_list(A.slow_list, A.slow_count, j);
      } else {
        const uint32_t ip_off = sp0 + 1, ip_len = sp1 - sp0 - 1;
        const uint32_t rest_off = sp1 + 1, host_off = sp2 + 1, host_len = sp3 - sp2 - 1;
        const bool hostw = l2_in(X, host_off, host_len);
        const int32_t hid = hostw ? host_lookup_lds(s_hl, X.wp + host_off, host_len)
                                  : host_lookup_lds(s_hl, X.gp + host_off, host_len);
        const uint32_t dc = hid >= 0 ? s_hl[B.l2_hdc + (uint32_t)hid] : B.l2_none;
        const uint32_t dw = B.l2_dcls + dc * DW;
        const uint32_t rows = s_hl[dw + 10 * W], prule = s_hl[dw + 10 * W + 1], anc = s_hl[dw + 10 * W + 2],
                       n_anc = s_hl[dw + 10 * W + 3];
        const uint32_t first_rule = hid >= 0 ? LT.hinfo[hid].y : 0u;
        const uint32_t pinl = s_hl[dw + 10 * W + 4];  // the class's inline-DFA entries per position (0: none)
        const bool exempt = B.any_allow && check_is_allowed(B, hid, X.gp + ip_off, ip_len);
        L2P(2);
        const int64_t tsn = ns_from_seconds(f);
        uint8_t fl = 0;
        if (go_sub(A.now_ns, tsn) > 10000000000LL) fl = kLineOld;
        else if (exempt) fl = kLineExempt;
        const uint32_t rest_len = n - rest_off, host_rel = host_off - rest_off;
        L2Mask<W> m = l2_ld_mask<W>(s_hl, dw), J;  // ALWAYS
#pragma unroll
        for (int k = 0; k < W; ++k) J.w[k] = 0;
        bool evl = false;  // the line has or may get (through its jobs) a rate-limit event
        if (fl) {
          L.counts[j] = 0;
        } else {
          // literal hits of the scan pass inside rest (unverified ones checked here)
          const uint32_t cc = cm.cnt;
          const bool ovf = cc > (uint32_t)kCandSlots;
          const uint64_t rs = s + rest_off;
          uint32_t ovbits = 0;  // literal ids < 32 among the verified hits
          L2Mask<W> done;
#pragma unroll
          for (int k = 0; k < W; ++k) done.w[k] = 0;
          uint32_t nlit = 0;
#pragma unroll
          for (uint32_t c = 0; c < (uint32_t)kCandSlots; ++c) {
            if (c >= cc || (A.dbg2 & 2)) break;
            const uint64_t v = cv[c];
            const uint32_t lit = (uint32_t)(v & 0x7FFFFF);
            const uint64_t q = v >> 24;
            if (q < rs) continue;
            if (!(v & kCandVerified)) {
              const uint32_t o = (uint32_t)(q - s), ll = lit_len_of(TB, lit);
              if (o + ll > n) continue;
              if (!(l2_in(X, o, ll) ? literal_at(TB, lit, X.wp + o) : literal_at(TB, lit, X.gp + o))) continue;
            }
            if (lit < 32) ovbits |= 1u << lit;
            ++nlit;
            if (ovf) continue;
            const uint32_t hp = q - rs < 0xFFFF ? (uint32_t)(q - rs) : 0xFFFFu;
            const uint32_t rw = rows + lit * RW;
            l2_or(m, l2_ld_mask<W>(s_hl, rw));
            l2_or(J, l2_ld_mask<W>(s_hl, rw + 2 * W));
            const uint32_t ck_off = s_hl[rw + 6 * W], n_ck = s_hl[rw + 6 * W + 1];
            for (uint32_t k = 0; k < n_ck; ++k) {
              const uint4 ck = l2_ld4w(s_hl, ck_off + 4 * k);
              const uint32_t bit = ck.x & 0xFFu;
              if (l2_has(done, bit)) continue;
              uint32_t out;
              if (hp == 0xFFFFu) out = 2;  // hit offset unknown: the automaton decides
              else {
                // in the window: the checked text (ck.w bytes from the hit, plus the
                // host for a template that spells it after the hit) and the host field
                const uint32_t tail = ck.w + (((ck.x >> 11) & 1u) ? host_len : 0u);
                const bool inw = hostw && rest_off + hp + tail + 8 <= X.lim;
                out = inw ? l2_check<true>(TB, LT, ck, X.wp + rest_off, rest_len, host_rel, host_len, hp)
                          : l2_check<false>(TB, LT, ck, X.gp + rest_off, rest_len, host_rel, host_len, hp);
              }
              if (out) {
                l2_set(done, bit);
                if (out == 1) l2_set(m, bit);
                else l2_set(J, bit);
              }
            }
          }
          if (ovf) {
            // more hits than slots: a literal rule none of whose literals occurred
            // cannot match; the others go to their automaton
            // (literal ids >= 32: which occurred is not recorded, so every
            // rule needing one of them goes to its automaton)
            ovbits |= (uint32_t)(cm.bits & 0xFFFFFFFFull);
            uint32_t ob = ovbits;
            while (ob) {
              const uint32_t l = (uint32_t)__ffs(ob) - 1;
              ob &= ob - 1;
              l2_or(J, l2_ld_mask<W>(s_hl, rows + l * RW + 4 * W));
            }
            l2_or(J, l2_ld_mask<W>(s_hl, dw + 6 * W));
            l2_or(J, l2_ld_mask<W>(s_hl, dw + 8 * W));
          } else if (nlit) {
            l2_or(J, l2_ld_mask<W>(s_hl, dw + 4 * W));
          }
          L2P(3);
          // anchored and no-literal entries of the class, each lane its own
          // class's list (a wave-uniform walk per class serialised the classes
          // of a wave's lines; scalar loads of the entries when the whole wave
          // shares one list measured no faster)
          const uint32_t na = (A.dbg2 & 1) ? 0u : n_anc;
          for (uint32_t i = 0; i < na; ++i) {
            const uint32_t ew = anc + kL2AncWords * i;
            const uint4 a = l2_ld4w(s_hl, ew), bq = l2_ld4w(s_hl, ew + 4);
            const uint32_t ext = s_hl[ew + 8];
            const uint32_t pos = (a.x >> 20) & 0x7Fu;
            const uint32_t r = (a.x & kPlanOwn) ? first_rule + pos : (a.x & 0xFFFFFu);
            // in the window: the bytes of rest the entry may read (ext, plus the
            // host for a template) and the host field
            const uint32_t need = (ext & 0x7FFFFFFFu) + ((ext >> 31) ? host_len : 0u);
            const bool inw = hostw && rest_off + need + 8 <= X.lim;
            const uint32_t out = inw ? l2_anchored<true>(B, TB, LT, a, bq, r, X.wp + rest_off, rest_len, host_rel, host_len)
                                     : l2_anchored<false>(B, TB, LT, a, bq, r, X.gp + rest_off, rest_len, host_rel, host_len);
            if (out == 1) l2_set(m, pos);
            else if (out == 2) l2_set(J, pos);
          }
          L2P(4);
          const L2Mask<W> skp = l2_ld_mask<W>(s_hl, dw + 2 * W);
#pragma unroll
          for (int k = 0; k < W; ++k) {
            J.w[k] &= ~m.w[k];
            evl = evl || ((m.w[k] | J.w[k]) & ~skp.w[k]) != 0;
          }
#pragma unroll
          for (int k = 0; k < W; ++k) {
            uint64_t Jk = (A.dbg2 & 4) ? 0ull : J.w[k];
            while (Jk) {
              const uint32_t p = 64u * k + (uint32_t)__ffsll((unsigned long long)Jk) - 1;
              Jk &= Jk - 1;
              const uint32_t w = s_hl[prule + p];
              const uint32_t r = (w & kPlanOwn) ? first_rule + p : (w & 0xFFFFFu);
              const uint64_t rec = l2_job_rec(B, r, cm, cv, rs, rest_len, rest_off,
                                              B.cfirst ? L.cand_first + j * kCandFirstLits : nullptr);
              uint32_t res = 2;
              if (rec == kJobDecided) res = 1;
              else if (pinl && !(rec & kJobLegacy)) {
                const uint32_t ent = s_hl[pinl + p];
                if (ent) res = l2_inline(s_hl, ent, X, s, rec);
              }
              if (res == 1) m.w[k] |= 1ull << (p & 63);
              else if (res == 2) emit_job(S, j, r, p, rec | (((skp.w[k] >> (p & 63)) & 1) ? kJobNoCount : 0ull));
            }
          }
          L2P(5);
          uint32_t n_m = 0, n_ev = 0;
#pragma unroll
          for (int k = 0; k < W; ++k) {
            L.mword(j, k) = m.w[k];
            n_m += __popcll(m.w[k]);
            n_ev += __popcll(m.w[k] & ~skp.w[k]);
          }
          if (W == 1 && B.mask_words > 1) L.mword(j, 1) = 0;
          L.counts[j] = ((uint64_t)n_m << 32) | (uint64_t)n_ev;
        }
        L.rest_off[j] = rest_off;
        L.host_id[j] = hid;
        // the IP is read only for event lines (claims, node exchange, trips,
        // bans): the others get ip_len 0 (the claims skip them).  An event
        // line stores its IP's inline key; the IP's offset follows from
        // rest_off and ip_len, its hash (for <= 15 bytes) from the key, and
        // the host field is found again for the lines that trip
        L.ip_len[j] = evl ? ip_len : 0u;
        if (evl && !(A.dbg2 & 8)) {
          uint4 k16;
          uint64_t h;
          if (l2_in(X, ip_off, ip_len > 16 ? ip_len : 16u)) ip_key_hash(X.wp + ip_off, ip_len, k16, h);
          else ip_key_hash(X.gp + ip_off, ip_len, k16, h);
          if (ip_len > 15) L.ip_hash[j] = h;
          L.ip16[j] = k16;
        }
        L.ts[j] = tsn;
        L.flags[j] = fl;
      }
    }
    L2P(6);
    // ---- append this wave's DFA jobs (from its chunk of the job array)
    flush_jobs(S, JC, lane);
    L2P(7);
  }
  close_jobs(S, JC, lane, A.null_key, A.job_real);
#ifdef BJX_PROF_L2
  if (lane == 0 && A.prof)
    for (int k = 0; k < 8; ++k) atomicAdd(&A.prof[k], (unsigned long long)P.acc[k]);
#endif
}
