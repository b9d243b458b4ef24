// Host/device helpers of the MI355X engine (product code; compiled into
// libbanjax_gpu.so for both the host side and the gfx950 kernels).
//
//  * go_parse_float: strconv.ParseFloat(s, 64) as used by parseTimestamp
//    (reference internal/regex_rate_limiter.go:95-103).  Fast exact path for
//    the nginx $msec shape, plus the exact multi-precision decimal algorithm
//    for every other syntactically valid input (correctly rounded, as Go is).
//  * go_parse_addr: net.ParseIP / netip.ParseAddr (used by the reference's
//    IPFilter in CheckIsAllowed, internal/decision.go:185-216).
//  * decode_rune: unicode/utf8.DecodeRune (Go regexp input stepping).
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define BJX_HD __host__ __device__ __forceinline__
#define BJX_HDN __host__ __device__ inline
#else
#define BJX_HD inline
#define BJX_HDN inline
#endif

namespace bjx {

// ------------------------------------------------------------- utf-8

BJX_HD int32_t decode_rune_hd(const uint8_t *s, uint64_t n, int *width) {
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
  else { *width = 1; return 0xFFFD; }
  if (n < (uint64_t)need + 1 || s[1] < lo || s[1] > hi) { *width = 1; return 0xFFFD; }
  r = (r << 6) | (s[1] & 0x3F);
  for (int k = 2; k <= need; ++k) {
    if (s[k] < 0x80 || s[k] > 0xBF) { *width = 1; return 0xFFFD; }
    r = (r << 6) | (s[k] & 0x3F);
  }
  *width = need + 1;
  return r;
}

// ------------------------------------------------------------- hashing

BJX_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
// 4 little-endian bytes at p, any alignment.  Device: two aligned 32-bit
// loads + v_alignbyte (LDS and HBM alike); the aligned word may extend up to 3
// bytes past p + 3, so callers keep 4 readable bytes of slack (all scan
// buffers and tables are padded).  Host: memcpy.
inline uint32_t ld4(const uint8_t *p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
#ifdef __HIPCC__
__device__ __forceinline__ uint32_t ld4(const uint8_t *p) {
  // align by pointer arithmetic on p itself (no integer round trip), so the
  // compiler keeps p's address space: ds_read for LDS, global_load for HBM
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t *w = reinterpret_cast<const uint32_t *>(p - sh);
  return sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
}
#endif

BJX_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

BJX_HD uint64_t hash_finish(uint32_t a, uint32_t b, uint32_t t);

// 64-bit hash of a byte string (engine-internal: host dictionary, IP state
// keys); 4 bytes per step in two 32-bit lanes, murmur3-style finalizer.
// Never returns 0 or ~0 (table sentinels).
BJX_HD uint64_t hash_bytes(const uint8_t *p, uint32_t n) {
  uint32_t a = 0x9E3779B9u ^ n, b = 0x7F4A7C15u + n * 0x85EBCA6Bu;
  uint32_t i = 0;
  for (; i + 4 <= n; i += 4) {
    const uint32_t w = ld4(p + i);
    a = rotl32(a ^ w, 7) * 0x27D4EB2Du;
    b = rotl32(b + w, 13) * 0x165667B1u;
  }
  uint32_t t = 0;
  for (uint32_t k = 0; i + k < n; ++k) t |= (uint32_t)p[i + k] << (8 * k);
  return hash_finish(a, b, t);
}

// The per-line pass's host dictionary hash (Bind::hl in LDS): word k of the
// host (zero padded, little endian) rotated by 7 k + 3 and folded by xor, then
// the length and a multiply / xorshift mix.  Two operations per word and no
// multiply until the end, independent across words: the dictionary compares
// every candidate in full, so this hash only has to spread the slots.  Never 0
// (the empty-slot tag).
BJX_HD uint32_t host_fold_word(uint32_t w, uint32_t k) {
  const uint32_t r = (7u * k + 3u) & 31u;
  return (w << r) | (w >> ((32u - r) & 31u));
}
BJX_HD uint32_t host_fold_finish(uint32_t a, uint32_t n) {
  a ^= n * 0x9E3779B9u;
  a ^= a >> 15; a *= 0x2C1B3C6Du; a ^= a >> 12; a *= 0x297A2D39u; a ^= a >> 15;
  return a | 1u;
}
BJX_HD uint32_t host_fold(const uint8_t *p, uint32_t n) {
  uint32_t a = 0, k = 0, i = 0;
  for (; i + 4 <= n; i += 4, ++k) a ^= host_fold_word(ld4(p + i), k);
  if (i < n) {
    uint32_t t = 0;
    for (uint32_t b = 0; i + b < n; ++b) t |= (uint32_t)p[i + b] << (8 * b);
    a ^= host_fold_word(t, k);
  }
  return host_fold_finish(a, n);
}

// hash_bytes' last step: the tail word t (the 0-3 bytes after the last full
// word, zero padded) and the finalizer
BJX_HD uint64_t hash_finish(uint32_t a, uint32_t b, uint32_t t) {
  a = rotl32(a ^ t ^ 0xA5A5A5A5u, 7) * 0x27D4EB2Du;
  b = rotl32(b + t, 13) * 0x165667B1u;
  a ^= b >> 16; a *= 0x85EBCA6Bu; a ^= a >> 13; a *= 0xC2B2AE35u; a ^= a >> 16;
  b ^= a >> 15; b *= 0x2C1B3C6Du; b ^= b >> 12; b *= 0x297A2D39u; b ^= b >> 15;
  uint64_t h = ((uint64_t)a << 32) | b;
  if (h == 0 || h == ~0ULL) h = 0x1234567ULL;
  return h;
}

// ------------------------------------------------------------- K-way search

// One narrowing step of a K-way parallel search for the first i in [lo, hi)
// with pred(i) (pred monotone: false ... true).  The K samples are
// lo + t * stride (t < K, stride = ceil((hi - lo) / K)); samples at or past hi
// are not taken.  f = the first sample index whose pred holds, K if none.
// The answer lies in [lo', hi'], so the search ends (answer hi') once
// lo' >= hi'.  With no sample true, the next range starts after the last
// sample taken below hi, which is below lo + (K - 1) * stride when (hi - lo)
// is not a multiple of stride: starting at lo + (K - 1) * stride + 1 would
// skip the positions between them (round-2 hot-key outcome mismatch).
BJX_HD uint64_t search_stride(uint64_t lo, uint64_t hi, uint32_t K) { return (hi - lo + K - 1) / K; }
BJX_HD void search_narrow(uint64_t &lo, uint64_t &hi, uint64_t stride, uint32_t f, uint32_t K) {
  if (f == 0) { hi = lo; return; }
  uint64_t last = f - 1;  // last sample known false
  if (f < K) hi = lo + (uint64_t)f * stride;
  else {
    last = (hi - 1 - lo) / stride;
    if (last > K - 1) last = K - 1;
  }
  lo += last * stride + 1;
}

// ------------------------------------------------------------- time

// time.Time.Sub for time.Unix(0, ns) values: exact difference saturated to
// [minDuration, maxDuration].
BJX_HD int64_t go_sub(int64_t t, int64_t u) {
  int64_t d = (int64_t)((uint64_t)t - (uint64_t)u);
  // overflow iff t and u have different signs and d's sign differs from t's
  if (((t ^ u) & (t ^ d)) < 0) return t < u ? INT64_MIN : INT64_MAX;
  return d;
}

// int64(f * 1e9) with amd64 CVTTSD2SQ semantics (out of range/NaN -> MinInt64).
BJX_HD int64_t ns_from_seconds(double f) {
  double x = f * 1e9;
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}

// ------------------------------------------------------------- ParseFloat

BJX_HD int lower_c(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

// Exact fast path for "[0-9]+(\.[0-9]*)?" with < 2^53 mantissa and <= 22
// fraction digits: one correctly rounded IEEE division (no contraction).
// Returns 0 ok, 1 = needs the general algorithm (not an error).
BJX_HD int parse_float_fast(const uint8_t *s, uint32_t n, double *out) {
  if (n == 0 || n > 40) return 1;
  uint64_t m = 0;
  int frac = -1, digits = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t c = s[i];
    if (c >= '0' && c <= '9') {
      if (m != 0 || c != '0') ++digits;
      if (digits > 16) return 1;
      m = m * 10 + (c - '0');
      if (frac >= 0) ++frac;
    } else if (c == '.' && frac < 0) {
      frac = 0;
    } else {
      return 1;
    }
  }
  if (frac < 0) frac = 0;
  if (s[0] == '.' || (n == 1 && s[0] == '.')) return 1;
  if (m >= (1ULL << 53) || frac > 22) return 1;
  // 10^frac as a product of exact powers of ten: every partial product is a
  // power of ten <= 1e22, exactly representable, so each multiply is exact
  // (no table: an indexed local array would live in scratch on the device)
  double p = 1.0;
  if (frac & 1) p *= 1e1;
  if (frac & 2) p *= 1e2;
  if (frac & 4) p *= 1e4;
  if (frac & 8) p *= 1e8;
  if (frac & 16) p *= 1e16;
  double f = (double)m;
  *out = frac ? f / p : f;
  return 0;
}

// Multi-precision decimal (the classic exact shift algorithm): value =
// 0.d[0..nd) * 10^dp.  Digits are stored as values 0..9.
struct Decimal {
  uint8_t d[800];
  int nd, dp;
  bool neg, trunc;
};

BJX_HDN void dec_trim(Decimal *a) {
  while (a->nd > 0 && a->d[a->nd - 1] == 0) a->nd--;
  if (a->nd == 0) a->dp = 0;
}
// multiply by 2^k, k <= 60 (carry stays < 10 * 2^k < 2^64)
BJX_HDN void dec_lshift(Decimal *a, unsigned k) {
  uint8_t tmp[824];
  int tw = 824;
  uint64_t n = 0;
  for (int r = a->nd - 1; r >= 0; --r) {
    n += (uint64_t)a->d[r] << k;
    uint64_t q = n / 10;
    tmp[--tw] = (uint8_t)(n - 10 * q);
    n = q;
  }
  while (n > 0) {
    uint64_t q = n / 10;
    tmp[--tw] = (uint8_t)(n - 10 * q);
    n = q;
  }
  int newnd = 824 - tw;
  int keep = newnd > 800 ? 800 : newnd;
  for (int i = 0; i < keep; ++i) a->d[i] = tmp[tw + i];
  for (int i = keep; i < newnd; ++i)
    if (tmp[tw + i]) a->trunc = true;
  a->dp += newnd - a->nd;
  a->nd = keep;
  dec_trim(a);
}
// divide by 2^k, k <= 60
BJX_HDN void dec_rshift(Decimal *a, unsigned k) {
  int r = 0, w = 0;
  uint64_t n = 0;
  for (; (n >> k) == 0; ++r) {
    if (r >= a->nd) {
      if (n == 0) { a->nd = 0; return; }
      while ((n >> k) == 0) { n *= 10; ++r; }
      break;
    }
    n = n * 10 + a->d[r];
  }
  a->dp -= r - 1;
  const uint64_t mask = (1ULL << k) - 1;
  for (; r < a->nd; ++r) {
    uint64_t dig = n >> k;
    n &= mask;
    a->d[w++] = (uint8_t)dig;
    n = n * 10 + a->d[r];
  }
  while (n > 0) {
    uint64_t dig = n >> k;
    n &= mask;
    if (w < 800) a->d[w++] = (uint8_t)dig;
    else if (dig > 0) a->trunc = true;
    n = n * 10;
  }
  a->nd = w;
  dec_trim(a);
}
BJX_HDN void dec_shift(Decimal *a, int k) {
  if (a->nd == 0) return;
  if (k > 0) { while (k > 60) { dec_lshift(a, 60); k -= 60; } dec_lshift(a, (unsigned)k); }
  else if (k < 0) { while (k < -60) { dec_rshift(a, 60); k += 60; } dec_rshift(a, (unsigned)-k); }
}
BJX_HDN bool dec_round_up(const Decimal *a, int nd) {
  if (a->d[nd] == 5 && nd + 1 == a->nd) {
    if (a->trunc) return true;
    return nd > 0 && (a->d[nd - 1] % 2) != 0;
  }
  return a->d[nd] >= 5;
}
BJX_HDN uint64_t dec_rounded_integer(const Decimal *a) {
  if (a->dp > 20) return ~0ULL;
  int i = 0;
  uint64_t n = 0;
  for (; i < a->dp && i < a->nd; ++i) n = n * 10 + a->d[i];
  for (; i < a->dp; ++i) n *= 10;
  if (a->dp >= 0 && a->dp < a->nd && dec_round_up(a, a->dp)) ++n;
  return n;
}
// decimal -> float64 bits; *overflow set on +-Inf
BJX_HDN uint64_t dec_float_bits(Decimal *a, bool *overflow) {
  const int mantbits = 52, expbits = 11, bias = -1023;
  const int powtab[9] = {1, 3, 6, 9, 13, 16, 19, 23, 26};
  int exp = 0;
  uint64_t mant = 0;
  *overflow = false;
  if (a->nd == 0) { mant = 0; exp = bias; goto out; }
  if (a->dp > 310) goto ovf;
  if (a->dp < -330) { mant = 0; exp = bias; goto out; }
  while (a->dp > 0) {
    int n = a->dp >= 9 ? 27 : powtab[a->dp];
    dec_shift(a, -n);
    exp += n;
  }
  while (a->dp < 0 || (a->dp == 0 && a->d[0] < 5)) {
    int n = -a->dp >= 9 ? 27 : powtab[-a->dp];
    dec_shift(a, n);
    exp -= n;
  }
  exp--;
  if (exp < bias + 1) {
    int n = bias + 1 - exp;
    dec_shift(a, -n);
    exp += n;
  }
  if (exp - bias >= (1 << expbits) - 1) goto ovf;
  dec_shift(a, 1 + mantbits);
  mant = dec_rounded_integer(a);
  if (mant == (2ULL << mantbits)) {
    mant >>= 1;
    exp++;
    if (exp - bias >= (1 << expbits) - 1) goto ovf;
  }
  if ((mant & (1ULL << mantbits)) == 0) exp = bias;
  goto out;
ovf:
  mant = 0;
  exp = (1 << expbits) - 1 + bias;
  *overflow = true;
out: {
  uint64_t bits = mant & ((1ULL << mantbits) - 1);
  bits |= (uint64_t)((exp - bias) & ((1 << expbits) - 1)) << mantbits;
  if (a->neg) bits |= 1ULL << 63;
  return bits;
}
}

BJX_HD double bits_to_double(uint64_t b) {
  union { uint64_t u; double f; } x;
  x.u = b;
  return x.f;
}

// strconv.ParseFloat(s, 64): 0 ok, -1 syntax error, -2 range error (+-Inf).
// The Decimal scratch (~808 B) is supplied by the caller.
BJX_HDN int go_parse_float(const uint8_t *s, uint32_t n, double *out, Decimal *dec) {
  if (parse_float_fast(s, n, out) == 0) return 0;
  // special(): [+-]inf, [+-]infinity, nan (case-insensitive)
  if (n > 0) {
    uint32_t i = 0; int sign = 1; bool signed_ = false;
    if (s[0] == '+' || s[0] == '-') { sign = s[0] == '-' ? -1 : 1; i = 1; signed_ = true; }
    if (signed_ || lower_c(s[0]) == 'i') {
      const char *inf = "infinity";
      uint32_t k = 0;
      while (i + k < n && k < 8 && lower_c(s[i + k]) == inf[k]) ++k;
      if (k > 3 && k < 8) k = 3;
      if (k == 3 || k == 8) {
        if (i + k != n) return -1;
        *out = sign * bits_to_double(0x7FF0000000000000ULL);
        return 0;
      }
    } else if (lower_c(s[0]) == 'n') {
      if (n >= 3 && lower_c(s[1]) == 'a' && lower_c(s[2]) == 'n') {
        if (n != 3) return -1;
        *out = bits_to_double(0x7FF8000000000001ULL);
        return 0;
      }
    }
  }
  // readFloat
  uint32_t i = 0;
  bool neg = false, underscores = false, hex = false;
  if (n == 0) return -1;
  if (s[i] == '+') ++i;
  else if (s[i] == '-') { neg = true; ++i; }
  int base = 10;
  if (i + 2 < n && s[i] == '0' && lower_c(s[i + 1]) == 'x') { base = 16; hex = true; i += 2; }
  bool sawdot = false, sawdigits = false;
  int nd = 0, ndmant = 0, dp = 0;
  uint64_t mant = 0;
  bool trunc = false;
  const uint32_t digits_begin = i;
  for (; i < n; ++i) {
    uint8_t c = s[i];
    if (c == '_') { underscores = true; continue; }
    if (c == '.') { if (sawdot) break; sawdot = true; dp = nd; continue; }
    if (c >= '0' && c <= '9') {
      sawdigits = true;
      if (c == '0' && nd == 0) { dp--; continue; }
      nd++;
      if (ndmant < (hex ? 16 : 19)) { mant = mant * base + (c - '0'); ndmant++; }
      else if (c != '0') trunc = true;
      continue;
    }
    if (hex && lower_c(c) >= 'a' && lower_c(c) <= 'f') {
      sawdigits = true;
      nd++;
      if (ndmant < 16) { mant = mant * 16 + (lower_c(c) - 'a' + 10); ndmant++; }
      else trunc = true;
      continue;
    }
    break;
  }
  if (!sawdigits) return -1;
  if (!sawdot) dp = nd;
  if (hex) { dp *= 4; ndmant *= 4; }
  const uint32_t mant_end = i;
  int eexp = 0;
  if (i < n && lower_c(s[i]) == (hex ? 'p' : 'e')) {
    ++i;
    if (i >= n) return -1;
    int esign = 1;
    if (s[i] == '+') ++i;
    else if (s[i] == '-') { ++i; esign = -1; }
    if (i >= n || s[i] < '0' || s[i] > '9') return -1;
    int e = 0;
    for (; i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '_'); ++i) {
      if (s[i] == '_') { underscores = true; continue; }
      if (e < 10000) e = e * 10 + (s[i] - '0');
    }
    eexp = e * esign;
    dp += eexp;
  } else if (hex) {
    return -1;
  }
  if (underscores) {
    // underscoreOK(s[:i])
    uint32_t j = 0, m = i;
    int saw = '^';
    if (m >= 1 && (s[0] == '-' || s[0] == '+')) j = 1;
    bool hx = false;
    if (m - j >= 2 && s[j] == '0' && (lower_c(s[j + 1]) == 'b' || lower_c(s[j + 1]) == 'o' || lower_c(s[j + 1]) == 'x')) {
      hx = lower_c(s[j + 1]) == 'x';
      j += 2;
      saw = '0';
    }
    for (; j < m; ++j) {
      int c = s[j];
      if ((c >= '0' && c <= '9') || (hx && lower_c(c) >= 'a' && lower_c(c) <= 'f')) { saw = '0'; continue; }
      if (c == '_') { if (saw != '0') return -1; saw = '_'; continue; }
      if (saw == '_') return -1;
      saw = '!';
    }
    if (saw == '_') return -1;
  }
  if (i != n) return -1;
  if (hex) {
    // atofHex: value = mant * 2^(dp - ndmant), round half even with trunc sticky
    int exp2 = mant != 0 ? dp - ndmant : 0;
    const int mantbits = 52, bias = -1023;
    if (mant == 0) { *out = neg ? bits_to_double(1ULL << 63) : 0.0; return 0; }
    // normalise to 1<<(mantbits+2) .. with 2 extra bits
    exp2 += mantbits;  // mant is an integer; Go: exp += int(flt.mantbits)
    while (mant != 0 && (mant >> (mantbits + 2)) == 0) { mant <<= 1; exp2--; }
    if (trunc) mant |= 1;
    while ((mant >> (1 + mantbits + 2)) != 0) { mant = (mant >> 1) | (mant & 1); exp2++; }
    while (mant > 1 && exp2 < bias + 1 - 2) { mant = (mant >> 1) | (mant & 1); exp2++; }
    uint64_t round = mant & 3;
    mant >>= 2;
    round |= mant & 1;
    exp2 += 2;
    if (round == 3) {
      mant++;
      if (mant == (1ULL << (1 + mantbits))) { mant >>= 1; exp2++; }
    }
    if ((mant >> mantbits) == 0) exp2 = bias;
    int rc = 0;
    if (exp2 > 1023) { mant = 1ULL << mantbits; exp2 = 1023 + 1; rc = -2; }
    uint64_t bits = mant & ((1ULL << mantbits) - 1);
    bits |= (uint64_t)((exp2 - bias) & 0x7FF) << mantbits;
    if (rc == -2) bits = 0x7FF0000000000000ULL;
    if (neg) bits |= 1ULL << 63;
    *out = bits_to_double(bits);
    return rc;
  }
  // decimal: exact multi-precision conversion of the digit string
  dec->nd = 0; dec->dp = 0; dec->neg = neg; dec->trunc = false;
  {
    bool sd = false;
    for (uint32_t k = digits_begin; k < mant_end; ++k) {
      uint8_t c = s[k];
      if (c == '_') continue;
      if (c == '.') { sd = true; dec->dp = dec->nd; continue; }
      if (c == '0' && dec->nd == 0) { dec->dp--; continue; }
      if (dec->nd < 800) dec->d[dec->nd++] = (uint8_t)(c - '0');
      else if (c != '0') dec->trunc = true;
    }
    if (!sd) dec->dp = dec->nd;
    dec->dp += eexp;
    dec_trim(dec);
  }
  bool ovf;
  uint64_t bits = dec_float_bits(dec, &ovf);
  *out = bits_to_double(bits);
  return ovf ? -2 : 0;
}

// ------------------------------------------------------------- netip

BJX_HD int hexv(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
// parseIPv4Fields: strict dotted quad, no leading zeros
BJX_HD bool parse_v4(const uint8_t *s, uint32_t n, uint8_t f[4]) {
  int val = 0, pos = 0, dig = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t c = s[i];
    if (c >= '0' && c <= '9') {
      if (dig == 1 && val == 0) return false;
      val = val * 10 + (c - '0');
      ++dig;
      if (val > 255) return false;
    } else if (c == '.') {
      if (i == 0 || i == n - 1 || s[i - 1] == '.') return false;
      if (pos == 3) return false;
      f[pos++] = (uint8_t)val;
      val = 0;
      dig = 0;
    } else {
      return false;
    }
  }
  if (pos < 3) return false;
  f[3] = (uint8_t)val;
  return true;
}
BJX_HDN bool parse_v6(const uint8_t *s, uint32_t n, uint8_t ip[16]) {
  for (uint32_t k = 0; k < n; ++k)
    if (s[k] == '%') return false;  // zones are refused by net.ParseIP
  for (int k = 0; k < 16; ++k) ip[k] = 0;
  int ellipsis = -1;
  if (n >= 2 && s[0] == ':' && s[1] == ':') {
    ellipsis = 0;
    s += 2; n -= 2;
    if (n == 0) return true;
  }
  int i = 0;
  while (i < 16) {
    uint32_t off = 0, acc = 0;
    for (; off < n; ++off) {
      int v = hexv(s[off]);
      if (v < 0) break;
      acc = (acc << 4) + (uint32_t)v;
      if (off > 3) return false;
      if (acc > 0xFFFF) return false;
    }
    if (off == 0) return false;
    if (off < n && s[off] == '.') {
      if (ellipsis < 0 && i != 12) return false;
      if (i + 4 > 16) return false;
      if (!parse_v4(s, n, ip + i)) return false;
      n = 0;
      i += 4;
      break;
    }
    ip[i] = (uint8_t)(acc >> 8);
    ip[i + 1] = (uint8_t)acc;
    i += 2;
    s += off; n -= off;
    if (n == 0) break;
    if (s[0] != ':') return false;
    if (n == 1) return false;
    ++s; --n;
    if (s[0] == ':') {
      if (ellipsis >= 0) return false;
      ellipsis = i;
      ++s; --n;
      if (n == 0) break;
    }
  }
  if (n != 0) return false;
  if (i < 16) {
    if (ellipsis < 0) return false;
    int k = 16 - i;
    for (int j = i - 1; j >= ellipsis; --j) ip[j + k] = ip[j];
    for (int j = ellipsis; j < ellipsis + k; ++j) ip[j] = 0;
  } else if (ellipsis >= 0) {
    return false;
  }
  return true;
}
// net.ParseIP: 16-byte form (IPv4 as ::ffff:a.b.c.d); *is4 = IPv4 text.
BJX_HDN bool go_parse_addr(const uint8_t *s, uint32_t n, uint8_t out[16], bool *is4) {
  for (uint32_t i = 0; i < n; ++i) {
    if (s[i] == '.') {
      uint8_t f[4];
      if (!parse_v4(s, n, f)) return false;
      for (int k = 0; k < 10; ++k) out[k] = 0;
      out[10] = out[11] = 0xFF;
      out[12] = f[0]; out[13] = f[1]; out[14] = f[2]; out[15] = f[3];
      *is4 = true;
      return true;
    }
    if (s[i] == ':') { *is4 = false; return parse_v6(s, n, out); }
    if (s[i] == '%') return false;
  }
  return false;
}
BJX_HD bool is_v4_mapped(const uint8_t a[16]) {
  for (int i = 0; i < 10; ++i)
    if (a[i]) return false;
  return a[10] == 0xFF && a[11] == 0xFF;
}

}  // namespace bjx
