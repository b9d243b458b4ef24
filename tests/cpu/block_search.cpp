// CPU harness for the K-way parallel search step shared with the device
// (bjx::search_narrow in banjax_amd/csrc/bjx_common.h; used by block_first in
// engine.hip for the hot-key run ends and window starts, k_long_*).  The block
// is simulated sequentially: every "lane" t samples lo + t * stride.
#include <stdint.h>
#include "../../banjax_amd/csrc/bjx_common.h"

extern "C" uint64_t bjx_test_block_first(uint64_t lo, uint64_t hi, uint64_t x, uint32_t K) {
  // first i in [lo, hi) with i >= x, else hi
  while (lo < hi) {
    const uint64_t stride = bjx::search_stride(lo, hi, K);
    uint32_t f = K;
    for (uint32_t t = 0; t < K; ++t) {
      const uint64_t p = lo + (uint64_t)t * stride;
      if (p < hi && p >= x) { f = t; break; }
    }
    bjx::search_narrow(lo, hi, stride, f, K);
  }
  return hi;
}
