// Host check of rc_udiv.h against the CPU's u64 division (tests/test_udiv.py builds and runs it):
// edge values around every power of two and the ranges the stream bodies divide (a coder range
// by a u32 total, a range difference by range / total), then seeded random pairs at every
// divisor width.  Prints the count checked, or the first mismatch and exits 1.
#include <stdio.h>
#include <stdlib.h>

#include "../../range_coder_rust_amd/csrc/rc_udiv.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  s ^= s << 13, s ^= s >> 7, s ^= s << 17;
  return s;
}
static unsigned long long checked = 0;
static void check(uint64_t x, uint64_t d) {
  if (d == 0) return;
  ++checked;
  const uint64_t q = rc_udiv64(x, d);
  if (q != x / d) {
    printf("mismatch: %llu / %llu = %llu, got %llu\n", (unsigned long long)x,
           (unsigned long long)d, (unsigned long long)(x / d), (unsigned long long)q);
    exit(1);
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  uint64_t edge[200];
  int ne = 0;
  for (int b = 0; b < 64; ++b) {
    const uint64_t p = 1ull << b;
    edge[ne++] = p;
    edge[ne++] = p - 1;
    edge[ne++] = p + 1;
  }
  edge[ne++] = ~0ull;
  edge[ne++] = ~0ull - 1;
  for (int i = 0; i < ne; ++i)
    for (int j = 0; j < ne; ++j) check(edge[i], edge[j]);
  for (long i = 0; i < n; ++i) {
    const int bx = 1 + (int)(rnd() % 64), bd = 1 + (int)(rnd() % 64);
    const uint64_t x = bx == 64 ? rnd() : rnd() >> (64 - bx);
    const uint64_t d = bd == 64 ? rnd() : rnd() >> (64 - bd);
    check(x, d);
    check(x, d | 1);
    // range / total and (data - low) / (range / total), as the bodies divide them
    const uint64_t range = (1ull << 48) + (rnd() >> 16) + (rnd() >> 8);
    const uint32_t total = 1 + (uint32_t)(rnd() >> 40);
    const uint64_t r = range / total;
    check(range, total);
    check(rnd() % range, r);
    check(range - 1, r);
  }
  printf("%llu\n", checked);
  return 0;
}
