// PModel::find_index (pmodel.rs:12) and the reference's errors (error.rs:3-13) through the C++
// host API, on the GPU:
//  - a FreqTable whose find_index is overridden by a linear scan is called once per decoded
//    symbol (decoder.rs:40) and decodes the sample data (examples/sample_impl.rs:72-128);
//  - a model whose cum_freq makes lower_bound + r * cum overflow raises LowerBoundOverflow with
//    the reference's payload {lower_bound, add_val, range}.
// Built by __graft_entry__.build(); run by tests/test_gpu_stream.py::test_cpp_find_index.
#include <cstdio>
#include <vector>

#include "range_coder.hpp"

struct LinearTable : rc::FreqTable {
  explicit LinearTable(size_t n) : rc::FreqTable(n) {}
  mutable size_t calls = 0;
  size_t find_index(const rc::Decoder& d) const override {
    ++calls;
    const rc::RangeCoder r = d.range_coder();
    const uint64_t rfreq = (d.data() - r.lower_bound()) / (r.range() / total_freq());
    size_t i = 0;
    while (i + 1 < alphabet_count() && cum_freq(i + 1) <= rfreq) ++i;
    return i;
  }
};

struct Overflowing : rc::PModel {
  bool bad = false;
  size_t alphabet_count() const override { return 2; }
  uint32_t c_freq(size_t) const override { return 1; }
  uint32_t cum_freq(size_t i) const override { return bad ? 0xFFFFFFFFu : (uint32_t)i; }
  uint32_t total_freq() const override { return 2; }
};

int main() {
  const std::vector<size_t> test_data = {2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5};
  LinearTable sd(10);
  for (size_t i : test_data) sd.add_alphabet_freq(i);
  sd.calc_cum();
  rc::Encoder encoder;
  for (size_t i : test_data) encoder.encode(sd, i);
  const std::vector<uint8_t> code = encoder.finish();
  rc::Decoder decoder(code);
  std::vector<size_t> out;
  for (size_t k = 0; k < test_data.size(); ++k) out.push_back(decoder.decode(sd));
  if (out != test_data || sd.calls != test_data.size()) {
    std::printf("find_index FAILED (calls %zu)\n", sd.calls);
    return 1;
  }
  std::printf("find_index called %zu times, round trip ok\n", sd.calls);

  Overflowing m;
  rc::Encoder e2;
  for (size_t i : {1, 1, 0, 1}) e2.encode(m, i);
  const rc::RangeCoder before = e2.range_coder();
  m.bad = true;
  e2.encode(m, 1);
  try {
    e2.peek_code();
    std::printf("no error FAILED\n");
    return 1;
  } catch (const rc::RangeCoderError& e) {
    const uint64_t r = before.range() / 2, add = r * 0xFFFFFFFFull;
    if (e.kind != rc::RangeCoderError::LOWER_BOUND_OVERFLOW ||
        e.lower_bound != before.lower_bound() || e.add_val != add || e.range != r) {
      std::printf("payload FAILED: %s\n", e.what());
      return 1;
    }
    std::printf("LowerBoundOverflow {lower_bound: %llu, add_val: %llu, range: %llu}\n",
                (unsigned long long)e.lower_bound, (unsigned long long)e.add_val,
                (unsigned long long)e.range);
  }
  std::printf("test passed\n");
  return 0;
}
