// A caller-side adaptive PModel through the C++ host API, the way a user of the reference
// writes one: the model borrowed by Encoder::encode / Decoder::decode is updated by the caller
// after every symbol (encoder.rs:24-31, decoder.rs:38-50 read it on every call).  Prints the
// stream as hex (checked against oracle/ref_literal.py by tests/test_gpu_stream.py).
// Usage: adaptive_impl <n_symbols> <seed>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "range_coder.hpp"

// FreqTable (examples/sample_impl.rs) plus the update rule of the build's adaptive order-0 model
class AdaptiveTable : public rc::PModel {
 public:
  AdaptiveTable(size_t n, uint32_t inc, uint32_t limit, uint32_t period)
      : c_(n, 1), cum_(n), inc_(inc), limit_(limit), period_(period) {
    calc_cum();
  }
  size_t alphabet_count() const override { return c_.size(); }
  uint32_t c_freq(size_t i) const override { return c_.at(i); }
  uint32_t cum_freq(size_t i) const override { return cum_.at(i); }
  uint32_t total_freq() const override { return total_; }
  void update(size_t s, uint64_t i) {
    c_[s] += inc_;
    calc_cum();
    if ((i + 1) % period_ == 0 && total_ > limit_) {
      for (auto& x : c_) x = (x + 1) >> 1;
      calc_cum();
    }
  }

 private:
  void calc_cum() {
    uint32_t t = 0;
    for (size_t i = 0; i < c_.size(); ++i) {
      cum_[i] = t;
      t += c_[i];
    }
    total_ = t;
  }
  std::vector<uint32_t> c_, cum_;
  uint32_t total_ = 0, inc_, limit_, period_;
};

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1000;
  uint64_t x = argc > 2 ? strtoull(argv[2], nullptr, 0) : 1;
  std::vector<size_t> syms(n);
  for (auto& s : syms) {  // skewed symbols (xorshift64)
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const uint64_t r = x % 1000;
    s = r < 500 ? r % 4 : (r < 800 ? r % 32 : r % 256);
  }
  AdaptiveTable em(256, 32, 4000, 64);
  rc::Encoder enc;
  uint64_t settled = 0;
  for (uint64_t i = 0; i < n; ++i) {
    settled += enc.encode(em, syms[i]);
    em.update(syms[i], i);
  }
  const std::vector<uint8_t> code = enc.finish();
  AdaptiveTable dm(256, 32, 4000, 64);
  rc::Decoder dec(code);
  for (uint64_t i = 0; i < n; ++i) {
    const size_t s = dec.decode(dm);
    if (s != syms[i]) {
      std::printf("round trip FAILED at %llu\n", (unsigned long long)i);
      return 1;
    }
    dm.update(s, i);
  }
  if (settled + 8 != code.size()) {
    std::printf("byte counts FAILED\n");
    return 1;
  }
  for (uint8_t b : code) std::printf("%02x", b);
  std::printf("\n");
  return 0;
}
