// Per-call cost of the C++ host mirror (include/range_coder.hpp) with a caller-adaptive model:
// the table changes after every symbol, so every Decoder::decode is one rc_stream_decode_host
// call (decoder.rs:38-54 reads the model at each call).  The model update is timed on its own
// and subtracted.  Prints one JSON line.  RC_STREAM_SERVICE=0 measures the launch path.
//   hipcc -O2 -std=c++17 -Iinclude tools/percall_native.cpp -o tools/percall_native \
//     -Lrange_coder_rust_amd -lrc_amd -Wl,-rpath,'$ORIGIN/../range_coder_rust_amd'
//   tools/percall_native [n_symbols]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "range_coder.hpp"

// librc_amd's internal service timings (rc_resume.hip), not part of the public header
extern "C" rc_status rc_svc_probe_(rc_ctx* ctx, uint64_t* out);

class AdaptiveTable : public rc::PModel {  // examples/adaptive_impl.cpp's model
 public:
  AdaptiveTable() : c_(256, 1), cum_(256) { calc_cum(); }
  size_t alphabet_count() const override { return c_.size(); }
  uint32_t c_freq(size_t i) const override { return c_[i]; }
  uint32_t cum_freq(size_t i) const override { return cum_[i]; }
  uint32_t total_freq() const override { return total_; }
  void update(size_t s, uint64_t i) {
    c_[s] += 32;
    calc_cum();
    if ((i + 1) % 256 == 0 && total_ > 57343) {
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
  uint32_t total_ = 0;
};

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : 5000;
  std::vector<size_t> syms(n);
  uint64_t x = 7;
  for (auto& s : syms) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    const uint64_t r = x % 1000;
    s = r < 500 ? r % 4 : (r < 800 ? r % 32 : r % 256);
  }
  {  // warm-up: context, staging, the service wave, and the launch path at this size (the
     // first launch of a kernel loads its code object)
    AdaptiveTable m;
    rc::Encoder e;
    for (uint64_t i = 0; i < n; ++i) {
      e.encode(m, syms[i]);
      m.update(syms[i], i);
    }
    const auto code = e.finish();
    AdaptiveTable dm;
    rc::Decoder d(code);
    for (uint64_t i = 0; i < 200; ++i) dm.update(d.decode(dm), i);
  }
  AdaptiveTable um;
  double t0 = now_us();
  for (uint64_t i = 0; i < n; ++i) um.update(syms[i], i);
  const double upd = (now_us() - t0) / n;

  AdaptiveTable em;
  rc::Encoder enc;
  t0 = now_us();
  for (uint64_t i = 0; i < n; ++i) {
    enc.encode(em, syms[i]);
    em.update(syms[i], i);
  }
  const std::vector<uint8_t> code = enc.finish();
  const double enc_us = (now_us() - t0) / n - upd;

  uint64_t pr[5];
  rc_svc_probe_(rc::Context::default_context().get(), pr);  // (reset)
  AdaptiveTable dm;
  rc::Decoder dec(code);
  t0 = now_us();
  for (uint64_t i = 0; i < n; ++i) {
    const size_t s = dec.decode(dm);
    if (s != syms[i]) {
      std::printf("{\"error\": \"round trip failed at %llu\"}\n", (unsigned long long)i);
      return 1;
    }
    dm.update(s, i);
  }
  const double dec_us = (now_us() - t0) / n - upd;
  rc_svc_probe_(rc::Context::default_context().get(), pr);
  const double pc = pr[0] ? (double)pr[0] : 1.0;
  // encode() with its return value read at every call (encoder.rs:34-36): one flush, so one
  // GPU call, per symbol
  AdaptiveTable cm;
  rc::Encoder cenc;
  uint64_t nb_sum = 0;
  t0 = now_us();
  for (uint64_t i = 0; i < n; ++i) {
    nb_sum += (uint32_t)cenc.encode(cm, syms[i]);
    cm.update(syms[i], i);
  }
  const double cnt_us = (now_us() - t0) / n - upd;
  if (cenc.finish().size() != code.size() || nb_sum + 8 != code.size()) {
    std::printf("{\"error\": \"per-symbol encode differs\"}\n");
    return 1;
  }
  const char* sv = getenv("RC_STREAM_SERVICE");
  std::printf("{\"n\": %llu, \"service\": %s, \"model_update_us\": %.3f, "
              "\"adaptive_encode_us\": %.3f, \"adaptive_encode_count_us\": %.3f, "
              "\"adaptive_decode_us\": %.3f, \"decode_service_calls\": %llu, "
              "\"wave_to_lds_us\": %.3f, \"wave_to_body_done_us\": %.3f, "
              "\"wave_to_written_us\": %.3f, \"host_wait_us\": %.3f}\n",
              (unsigned long long)n, (sv && sv[0] == '0') ? "false" : "true", upd, enc_us,
              cnt_us, dec_us, (unsigned long long)pr[0], pr[1] / pc / 100.0, pr[2] / pc / 100.0,
              pr[3] / pc / 100.0, pr[4] / pc / 1000.0);
  return 0;
}
