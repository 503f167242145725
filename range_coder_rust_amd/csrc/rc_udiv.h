// rc_udiv.h — exact u64 / u64 for the one-lane stream bodies (rc_resume.hip): an f64 estimate
// of a quotient below 2^32, then exact integer fix-ups, instead of the compiler's generic 64-bit
// division (~100 instructions on a lane's dependency chain).  range_par_total (range / total,
// range_coder.rs:38-40) has a u32 divisor: the high word goes first, so both parts are
// quotients below 2^32; find_index's (data - low) / r (sample_impl.rs:30) has a divisor of at
// least 2^32 whenever the table is consistent, and the same estimate covers it.
//
// Why the estimate is within one of the quotient q < 2^32: converting x < 2^64 and d to f64 and
// dividing rounds three times, each by a relative 2^-53 at most, so the f64 quotient is off by
// less than q * 2^-51 < 2^-19, and the truncation moves it by less than one more.  The fix-up
// loops are exact whatever the estimate (they compare full products), so the bound only
// decides how often they turn: at most once.
//
// Header-only and compilable for the host, so tests/test_udiv.py checks it against the CPU's
// division.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#define RC_UDIV_FN static __host__ __device__ __forceinline__
#else
#define RC_UDIV_FN static inline
#endif

// the high 64 bits of a * b
RC_UDIV_FN uint64_t rc_mulhi64(uint64_t a, uint64_t b) {
  const uint64_t al = (uint32_t)a, ah = a >> 32, bl = (uint32_t)b, bh = b >> 32;
  const uint64_t ll = al * bl, lh = al * bh, hl = ah * bl, hh = ah * bh;
  const uint64_t mid = (ll >> 32) + (uint32_t)lh + (uint32_t)hl;
  return hh + (lh >> 32) + (hl >> 32) + (mid >> 32);
}

// floor(n / d) for a quotient below 2^32 (n < d * 2^32), d >= 1
RC_UDIV_FN uint64_t rc_udiv_small_q(uint64_t n, uint64_t d) {
  uint64_t q = (uint64_t)((double)n / (double)d);  // <= 2^32
  while (rc_mulhi64(q, d) != 0 || q * d > n) --q;  // q d > n: one too many
  while (n - q * d >= d) ++q;                      // remainder >= d: one too few
  return q;
}

// floor(x / d), d >= 1
RC_UDIV_FN uint64_t rc_udiv64(uint64_t x, uint64_t d) {
  if (d >> 32) return rc_udiv_small_q(x, d);  // x < 2^64 <= d * 2^32
  const uint32_t d32 = (uint32_t)d, xh = (uint32_t)(x >> 32);
  const uint32_t qh = xh / d32;
  const uint64_t n = ((uint64_t)(xh - qh * d32) << 32) | (uint32_t)x;  // < d * 2^32
  return ((uint64_t)qh << 32) + rc_udiv_small_q(n, d);
}
