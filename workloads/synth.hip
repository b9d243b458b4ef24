// Synthetic nginx `banjax_format` access-log generator (bench / test tooling,
// not part of the product).  Format, reference
// supporting-containers/nginx/nginx.conf:40:
//   '$msec $remote_addr $request_method $host $request_method $uri $server_protocol $http_user_agent | $status'
// Line i is a pure function of (cfg, i), computed by the same code on the host
// (CPU baseline samples, golden fixtures) and on the GPU (multi-GB workloads
// written straight into HBM).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstring>

struct SynthCfg {
  uint64_t seed;
  uint64_t first_line;
  uint64_t n_lines;
  int64_t t0_ms;          // timestamp of line 0, milliseconds
  uint32_t us_per_line;   // timestamp step (microseconds)
  uint32_t n_ips;         // IP pool size (uniform draw)
  uint32_t n_hosts;       // site000.example.com .. site{n-1}
  uint32_t other_host_pct;
  uint32_t trigger_permille;
  uint32_t ua_heavy;      // 1: 2-8 KB user agents
  uint32_t ipv6_pct;
  uint32_t ts_decimals;   // 3 = nginx $msec
  uint32_t fixture_hosts; // 1: host 0 = localhost:8081, host 1 = example.com
  uint32_t ip_mode;       // IP pool draw: 0 uniform, 1 Zipf(zipf_milli / 1000), 2 distinct (line i -> pool index i mod n_ips, permuted)
  uint32_t zipf_milli;    // Zipf exponent x 1000 (ip_mode 1)
  uint32_t hot_pct;       // DDoS hot key: this share of lines comes from pool index 0 (any ip_mode)
  uint32_t _pad;
};

#define HD __host__ __device__ __forceinline__

HD uint64_t sm64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

struct Rng {
  uint64_t s;
  HD uint64_t next() { s = sm64(s); return s; }
  HD uint32_t below(uint32_t n) { return (uint32_t)((next() >> 11) % n); }
};

// Writer: counts bytes (dst == nullptr) or writes them.
struct W {
  char *dst;
  uint64_t n;
  HD void c(char ch) { if (dst) dst[n] = ch; ++n; }
  HD void s(const char *p) { while (*p) c(*p++); }
  HD void u(uint64_t v) {
    char b[24]; int k = 0;
    do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k) c(b[--k]);
  }
  HD void u0(uint64_t v, int width) {  // zero padded
    char b[24]; int k = 0;
    do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    while (k < width) b[k++] = '0';
    while (k) c(b[--k]);
  }
  HD void x(uint64_t v, int digits) {
    for (int k = digits - 1; k >= 0; --k) c("0123456789abcdef"[(v >> (4 * k)) & 15]);
  }
};

#define NUA 32
__constant__ const char *kUA_d[NUA] = {
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Safari/537.36",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 10_15_7) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Safari/605.1.15",
  "Mozilla/5.0 (X11; Linux x86_64; rv:125.0) Gecko/20100101 Firefox/125.0",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 10.15; rv:149.0) Gecko/20100101 Firefox/149.0",
  "Mozilla/5.0 (iPhone; CPU iPhone OS 17_4 like Mac OS X) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Mobile/15E148 Safari/604.1",
  "Mozilla/5.0 (Linux; Android 14; Pixel 8) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Mobile Safari/537.36",
  "Mozilla/5.0 (compatible; Googlebot/2.1; +http://www.google.com/bot.html)",
  "Mozilla/5.0 (compatible; bingbot/2.0; +http://www.bing.com/bingbot.htm)",
  "Mozilla/5.0 (compatible; AhrefsBot/7.0; +http://ahrefs.com/robot/)",
  "Mozilla/5.0 (compatible; SemrushBot/7~bl; +http://www.semrush.com/bot.html)",
  "Mozilla/5.0 (compatible; GPTBot/1.0; +https://openai.com/gptbot)",
  "curl/8.5.0",
  "python-requests/2.31.0",
  "Go-http-client/1.1",
  "Scrapy/2.11.2 (+https://scrapy.org)",
  "Python-Mechanize/0.4.9",
  "sqlmap/1.8#stable (https://sqlmap.org)",
  "Wget/1.21.4",
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64; rv:126.0) Gecko/20100101 Firefox/126.0",
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/123.0.0.0 Safari/537.36 Edg/123.0.2420.81",
  "Mozilla/5.0 (X11; Ubuntu; Linux x86_64; rv:124.0) Gecko/20100101 Firefox/124.0",
  "Mozilla/5.0 (Linux; Android 13; SM-S918B) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/122.0.0.0 Mobile Safari/537.36",
  "facebookexternalhit/1.1 (+http://www.facebook.com/externalhit_uatext.php)",
  "Twitterbot/1.0",
  "Mozilla/5.0 (compatible; YandexBot/3.0; +http://yandex.com/bots)",
  "Mozilla/5.0 (iPad; CPU OS 17_4 like Mac OS X) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Mobile/15E148 Safari/604.1",
  "Apache-HttpClient/4.5.14 (Java/17.0.10)",
  "okhttp/4.12.0",
  "Mozilla/5.0 (Windows NT 6.1; WOW64; Trident/7.0; rv:11.0) like Gecko",
  "Mozilla/5.0 (compatible; MJ12bot/v1.4.8; http://mj12bot.com/)",
  "-",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 14_4) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Safari/537.36",
};
static const char *kUA_h[NUA] = {
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Safari/537.36",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 10_15_7) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Safari/605.1.15",
  "Mozilla/5.0 (X11; Linux x86_64; rv:125.0) Gecko/20100101 Firefox/125.0",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 10.15; rv:149.0) Gecko/20100101 Firefox/149.0",
  "Mozilla/5.0 (iPhone; CPU iPhone OS 17_4 like Mac OS X) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Mobile/15E148 Safari/604.1",
  "Mozilla/5.0 (Linux; Android 14; Pixel 8) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Mobile Safari/537.36",
  "Mozilla/5.0 (compatible; Googlebot/2.1; +http://www.google.com/bot.html)",
  "Mozilla/5.0 (compatible; bingbot/2.0; +http://www.bing.com/bingbot.htm)",
  "Mozilla/5.0 (compatible; AhrefsBot/7.0; +http://ahrefs.com/robot/)",
  "Mozilla/5.0 (compatible; SemrushBot/7~bl; +http://www.semrush.com/bot.html)",
  "Mozilla/5.0 (compatible; GPTBot/1.0; +https://openai.com/gptbot)",
  "curl/8.5.0",
  "python-requests/2.31.0",
  "Go-http-client/1.1",
  "Scrapy/2.11.2 (+https://scrapy.org)",
  "Python-Mechanize/0.4.9",
  "sqlmap/1.8#stable (https://sqlmap.org)",
  "Wget/1.21.4",
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64; rv:126.0) Gecko/20100101 Firefox/126.0",
  "Mozilla/5.0 (Windows NT 10.0; Win64; x64) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/123.0.0.0 Safari/537.36 Edg/123.0.2420.81",
  "Mozilla/5.0 (X11; Ubuntu; Linux x86_64; rv:124.0) Gecko/20100101 Firefox/124.0",
  "Mozilla/5.0 (Linux; Android 13; SM-S918B) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/122.0.0.0 Mobile Safari/537.36",
  "facebookexternalhit/1.1 (+http://www.facebook.com/externalhit_uatext.php)",
  "Twitterbot/1.0",
  "Mozilla/5.0 (compatible; YandexBot/3.0; +http://yandex.com/bots)",
  "Mozilla/5.0 (iPad; CPU OS 17_4 like Mac OS X) AppleWebKit/605.1.15 (KHTML, like Gecko) Version/17.4 Mobile/15E148 Safari/604.1",
  "Apache-HttpClient/4.5.14 (Java/17.0.10)",
  "okhttp/4.12.0",
  "Mozilla/5.0 (Windows NT 6.1; WOW64; Trident/7.0; rv:11.0) like Gecko",
  "Mozilla/5.0 (compatible; MJ12bot/v1.4.8; http://mj12bot.com/)",
  "-",
  "Mozilla/5.0 (Macintosh; Intel Mac OS X 14_4) AppleWebKit/537.36 (KHTML, like Gecko) Chrome/124.0.0.0 Safari/537.36",
};

#define NWORD 16
__constant__ const char *kWord_d[NWORD] = {"shoes", "news", "weather", "login", "python", "banjax", "deflect", "cats",
                                           "rust", "hip", "gpu", "music", "maps", "cheap+flights", "recipes", "union"};
static const char *kWord_h[NWORD] = {"shoes", "news", "weather", "login", "python", "banjax", "deflect", "cats",
                                     "rust", "hip", "gpu", "music", "maps", "cheap+flights", "recipes", "union"};

HD const char *ua_of(uint32_t k) {
#ifdef __HIP_DEVICE_COMPILE__
  return kUA_d[k];
#else
  return kUA_h[k];
#endif
}
HD const char *word_of(uint32_t k) {
#ifdef __HIP_DEVICE_COMPILE__
  return kWord_d[k];
#else
  return kWord_h[k];
#endif
}

HD void render(const SynthCfg &cfg, uint64_t i, W &w) {
  Rng r{sm64(cfg.seed * 0x9E3779B97F4A7C15ULL + i)};
  // $msec
  const uint64_t t_us = (uint64_t)cfg.t0_ms * 1000 + i * cfg.us_per_line;
  w.u(t_us / 1000000);
  if (cfg.ts_decimals) {
    w.c('.');
    uint64_t frac = t_us % 1000000;
    int d = (int)cfg.ts_decimals;
    for (int k = d; k < 6; ++k) frac /= 10;
    w.u0(frac, d);
  }
  w.c(' ');
  // $remote_addr: pool index per ip_mode, unique text per pool index
  uint32_t idx;
  const uint64_t rip = r.next();
  if (cfg.hot_pct && (rip >> 40) % 100 < cfg.hot_pct) {
    idx = 0;
  } else if (cfg.ip_mode == 1) {
    // Zipf(s)-shaped rank by the continuous inverse CDF: P(rank <= k) ~ (k^(1-s) - 1) / (N^(1-s) - 1)
    const double s_ = cfg.zipf_milli / 1000.0, e = 1.0 - s_;
    const double u = (double)(rip >> 11) * (1.0 / 9007199254740992.0);
    const double hn = pow((double)cfg.n_ips + 1.0, e) - 1.0;
    double k = pow(1.0 + u * hn, 1.0 / e);
    uint64_t kk = (uint64_t)k;
    if (kk < 1) kk = 1;
    if (kk > cfg.n_ips) kk = cfg.n_ips;
    idx = (uint32_t)(kk - 1);
  } else if (cfg.ip_mode == 2) {
    // every line its own pool index (a bijection of i mod n_ips): n_ips distinct IPs per n_ips lines
    uint64_t x = i % cfg.n_ips;
    uint64_t m = 1;
    while (m < cfg.n_ips) m <<= 1;
    do { x = (x * 0x5DEECE66Dull + 0xBull) & (m - 1); } while (x >= cfg.n_ips);  // cycle-walk a full-period LCG mod 2^k
    idx = (uint32_t)x;
  } else {
    idx = (uint32_t)((rip >> 11) % cfg.n_ips);
  }
  if (r.below(100) < cfg.ipv6_pct) {
    w.s("2001:db8:");
    w.x(idx >> 16, 4); w.c(':'); w.x(idx & 0xFFFF, 4); w.s("::"); w.x((idx * 2654435761u) >> 20, 3);
  } else {
    uint64_t v = idx;
    w.u(1 + v % 223); v /= 223;
    w.c('.'); w.u(v % 256); v /= 256;
    w.c('.'); w.u(v % 256); v /= 256;
    w.c('.'); w.u(v % 256);
  }
  w.c(' ');
  const uint32_t m = r.below(100);
  const char *method = m < 85 ? "GET" : (m < 97 ? "POST" : "HEAD");
  w.s(method);
  w.c(' ');
  // $host
  if (r.below(100) < cfg.other_host_pct || cfg.n_hosts == 0) {
    w.s("cdn"); w.u(r.below(50)); w.s(".other.net");
  } else {
    const uint32_t h = r.below(cfg.n_hosts);
    if (cfg.fixture_hosts && h == 0) w.s("localhost:8081");
    else if (cfg.fixture_hosts && h == 1) w.s("example.com");
    else { w.s("site"); w.u0(h, 3); w.s(".example.com"); }
  }
  w.c(' ');
  w.s(method);
  w.c(' ');
  // $uri
  const uint32_t u = r.below(1000);
  if (r.below(1000) < cfg.trigger_permille) {
    switch (r.below(9)) {
      case 8: w.s("/block_local"); break;
      case 0: w.s("/blockme/"); break;
      case 1: w.s("/?challengeme"); break;
      case 2: w.s("/allowme"); break;
      case 3: w.s("/view.php?f=../../etc/passwd"); break;
      case 4: w.s("/search?q=1+union+select+password+from+users"); break;
      case 5: w.s("/.env"); break;
      case 6: w.s("/banme"); break;
      default: w.s("/wp-admin/admin-ajax.php"); break;
    }
  } else if (u < 250) {
    const char *p[6] = {"/", "/index.html", "/about", "/contact", "/favicon.ico", "/robots.txt"};
    w.s(p[r.below(6)]);
  } else if (u < 450) {
    switch (r.below(3)) {
      case 0: w.s("/static/js/app."); w.x(r.next(), 8); w.s(".js"); break;
      case 1: w.s("/static/css/site."); w.x(r.next(), 8); w.s(".css"); break;
      default: w.s("/img/"); w.u(r.below(100000)); w.s(".png"); break;
    }
  } else if (u < 600) {
    w.s("/api/v1/items/"); w.u(r.below(1000000));
  } else if (u < 700) {
    w.s("/search?q="); w.s(word_of(r.below(NWORD)));
  } else if (u < 760) {
    w.s("/wp-login.php");
  } else if (u < 800) {
    w.s("/xmlrpc.php");
  } else if (u < 850) {
    w.s("/admin/"); w.s(word_of(r.below(NWORD)));
  } else {
    w.s("/blog/"); w.u(2015 + r.below(10)); w.c('/'); w.s(word_of(r.below(NWORD)));
  }
  w.c(' ');
  const uint32_t pr = r.below(100);
  w.s(pr < 90 ? "HTTP/1.1" : (pr < 98 ? "HTTP/2.0" : "HTTP/1.0"));
  w.c(' ');
  // $http_user_agent
  w.s(ua_of(r.below(NUA)));
  if (cfg.ua_heavy) {
    const uint32_t target = 2048 + r.below(6144);  // 2-8 KB
    uint64_t start = w.n;
    while (w.n - start < target) {
      w.s(" ("); w.s(ua_of(r.below(NUA))); w.s(")");
      w.s(" ext/"); w.u(r.below(1000)); w.c('.'); w.u(r.below(100));
    }
  }
  w.s(" | ");
  const uint32_t st = r.below(100);
  w.u(st < 80 ? 200 : (st < 88 ? 301 : (st < 95 ? 404 : (st < 98 ? 403 : 500))));
  w.c('\n');
}

__global__ void k_len(SynthCfg cfg, uint64_t *len) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cfg.n_lines) return;
  W w{nullptr, 0};
  render(cfg, cfg.first_line + t, w);
  len[t] = w.n;
}
__global__ void k_write(SynthCfg cfg, const uint64_t *off, char *out) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= cfg.n_lines) return;
  W w{out + off[t], 0};
  render(cfg, cfg.first_line + t, w);
}

extern "C" {

// Host rendering of lines [first_line, first_line + n_lines): returns the byte
// count; writes to out when out != NULL and it fits in cap.
uint64_t bjx_synth_host(const SynthCfg *cfg, char *out, uint64_t cap) {
  W w{nullptr, 0};
  for (uint64_t i = 0; i < cfg->n_lines; ++i) render(*cfg, cfg->first_line + i, w);
  if (!out || w.n > cap) return w.n;
  W o{out, 0};
  for (uint64_t i = 0; i < cfg->n_lines; ++i) render(*cfg, cfg->first_line + i, o);
  return o.n;
}

// Device rendering into out_dev (capacity cap bytes).  Returns the byte count
// (or the needed size if it does not fit, without writing), or 0 on error.
uint64_t bjx_synth_device(const SynthCfg *cfg, void *out_dev, uint64_t cap, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  const uint64_t n = cfg->n_lines;
  if (n == 0) return 0;
  uint64_t *len = nullptr, *off = nullptr;
  if (hipMalloc(&len, (n + 1) * 8) != hipSuccess) return 0;
  if (hipMalloc(&off, (n + 1) * 8) != hipSuccess) { (void)hipFree(len); return 0; }
  const unsigned grid = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_len, dim3(grid), dim3(256), 0, st, *cfg, len);
  (void)hipMemsetAsync(len + n, 0, 8, st);
  size_t tmp_bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, len, off, (int)(n + 1), st);
  void *tmp = nullptr;
  (void)hipMalloc(&tmp, tmp_bytes + 16);
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, len, off, (int)(n + 1), st);
  uint64_t total = 0;
  (void)hipMemcpyAsync(&total, off + n, 8, hipMemcpyDeviceToHost, st);
  (void)hipStreamSynchronize(st);
  if (total <= cap && out_dev) {
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, st, *cfg, off, (char *)out_dev);
    (void)hipStreamSynchronize(st);
  }
  (void)hipFree(tmp);
  (void)hipFree(len);
  (void)hipFree(off);
  return hipGetLastError() == hipSuccess ? total : 0;
}

}  // extern "C"
