// The reference's examples/sample_impl.rs (:72-128) through the C++ host API: build a FreqTable
// from the test data, encode it, decode it and check the round trip — on the GPU.
// Built by __graft_entry__.build(); run by tests/test_gpu_parity.py::test_cpp_sample_impl.
#include <cstdio>
#include <vector>

#include "range_coder.hpp"

int main() {
  const std::vector<size_t> test_data = {2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5};
  rc::FreqTable sd(10);
  for (size_t i : test_data) sd.add_alphabet_freq(i);
  sd.calc_cum();
  std::printf("FREQ TABLE\n");
  for (size_t i = 0; i < sd.alphabet_count(); ++i)
    std::printf("index:%zu, c:%u, cum:%u\n", i, sd.c_freq(i), sd.cum_freq(i));

  rc::Encoder encoder;
  uint32_t settled = 0;  // sum of encode()'s return values (encoder.rs:36)
  for (size_t i : test_data) settled += encoder.encode(sd, i);
  const std::vector<uint8_t> code = encoder.finish();
  std::printf("output : 0x");
  for (uint8_t b : code) std::printf("%02x", b);
  std::printf("\nlength : %zubyte\n", code.size());
  if (settled + 8 != code.size()) {
    std::printf("byte counts FAILED\n");
    return 1;
  }

  rc::Decoder decoder(code);  // Decoder::new(code): the count stays out-of-band
  std::vector<size_t> decodeds;
  for (size_t k = 0; k < test_data.size(); ++k) decodeds.push_back(decoder.decode(sd));
  if (decodeds != test_data) {
    std::printf("round trip FAILED\n");
    return 1;
  }
  std::printf("test passed\n");
  return 0;
}
