// range_coder.hpp — C++ host API over the C ABI (include/range_coder.h), mirroring the public
// surface of diegodox/range_coder_rust (src/lib.rs:1-13) for host programs.
//
//   trait PModel            (src/pmodel.rs:4-41)         -> rc::PModel (abstract class)
//   FreqTable example model (examples/sample_impl.rs)    -> rc::FreqTable
//   Encoder::new/encode/finish (src/encoder.rs:14-46)    -> rc::Encoder (one stream, staged;
//                                                           finish() encodes on the GPU)
//   Decoder::new/decode       (src/decoder.rs:14-54)     -> rc::Decoder (count out-of-band)
//   error::RangeCoderError     (src/error.rs:3-13)       -> rc::RangeCoderError (exception)
//   (new) batch API                                      -> rc::encode_chunks / decode_chunks
//
// Header-only; link with librc_amd.so.  Everything runs on the GPU through the C ABI: there is
// no CPU implementation of the coder in the product.
#ifndef RANGE_CODER_AMD_HPP
#define RANGE_CODER_AMD_HPP

#include <cmath>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "range_coder.h"

namespace rc {

class RangeCoderError : public std::runtime_error {
 public:
  RangeCoderError(const std::string& what, int status = 0, uint32_t flags = 0)
      : std::runtime_error(what), status(status), flags(flags) {}
  int status;      // rc_status of the failing call
  uint32_t flags;  // RC_F_* of the failing chunk (0 if not chunk-specific)
};

inline void check(rc_status s, const char* what) {
  if (s != RC_OK) {
    std::string msg = std::string(what) + ": " + rc_status_string(s);
    if (s == RC_E_DEVICE) msg += std::string(" (") + rc_last_error() + ")";
    throw RangeCoderError(msg, s);
  }
}

inline std::string flag_string(uint32_t f) {
  std::string s;
  if (f & RC_F_ZERO_FREQ) s += "ZERO_FREQ|";
  if (f & RC_F_BAD_SYMBOL) s += "BAD_SYMBOL|";
  if (f & RC_F_CAPACITY) s += "CAPACITY|";
  if (f & RC_F_TRUNCATED) s += "TRUNCATED|";
  if (f & RC_F_CORRUPT) s += "CORRUPT|";
  if (!s.empty()) s.pop_back();
  return s;
}

class Decoder;

// trait PModel (src/pmodel.rs:4-41)
class PModel {
 public:
  virtual ~PModel() = default;
  virtual uint32_t c_freq(size_t index) const = 0;    // pmodel.rs:6
  virtual uint32_t cum_freq(size_t index) const = 0;  // pmodel.rs:8
  virtual uint32_t total_freq() const = 0;            // pmodel.rs:10
  // pmodel.rs:12.  The GPU decoder evaluates the canonical inverse cum[s] <= rfreq < cum[s+1]
  // itself (FreqTable::find_index, sample_impl.rs:27-45); this hook is not called.
  virtual size_t find_index(const Decoder&) const {
    throw RangeCoderError("find_index runs inside the GPU decode kernel");
  }
  // pmodel.rs:14-40
  virtual double ideal_code_length(size_t index) const {
    const double p = (double)c_freq(index);
    if (p == 0.0) throw RangeCoderError("code length is undefind when probability is zero");
    return (std::log((double)total_freq()) - std::log(p)) / std::log(2.0);
  }
  // Alphabet size: not a trait method in the reference (FreqTable::alphabet_count,
  // sample_impl.rs:55-57) but needed to snapshot the table for the GPU.
  virtual size_t alphabet_count() const = 0;
};

// examples/sample_impl.rs:4-70
class FreqTable : public PModel {
 public:
  explicit FreqTable(size_t alphabet_count) : c_(alphabet_count, 0), cum_(alphabet_count, 0) {}
  size_t alphabet_count() const override { return c_.size(); }
  void add_alphabet_freq(size_t index) { c_.at(index) += 1; }  // :58-60
  void calc_cum() {                                             // :61-69
    uint32_t t = 0;
    for (size_t i = 0; i < c_.size(); ++i) {
      cum_[i] = t;
      t += c_[i];
    }
    total_ = t;
  }
  uint32_t c_freq(size_t i) const override { return c_.at(i); }
  uint32_t cum_freq(size_t i) const override { return cum_.at(i); }
  uint32_t total_freq() const override { return total_; }

 private:
  std::vector<uint32_t> c_, cum_;
  uint32_t total_ = 0;
};

// One device (rc_ctx)
class Context {
 public:
  explicit Context(int device = 0) { check(rc_ctx_create(device, &ctx_), "rc_ctx_create"); }
  ~Context() {
    if (ctx_) rc_ctx_destroy(ctx_);
  }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  rc_ctx* get() const { return ctx_; }
  static Context& default_context() {
    static Context c(0);
    return c;
  }

 private:
  rc_ctx* ctx_ = nullptr;
};

// Device snapshot of a PModel's (c_freq, cum_freq, total_freq) table (rc_model)
class Model {
 public:
  Model(Context& ctx, const PModel& pm) : Model(ctx, snapshot_c(pm), snapshot_cum(pm), pm.total_freq()) {}
  Model(Context& ctx, const std::vector<uint32_t>& c, const std::vector<uint32_t>& cum,
        uint32_t total)
      : ctx_(&ctx), c_(c) {
    check(rc_model_create_static(ctx.get(), (uint32_t)c.size(), c.data(), cum.data(), total, &m_),
          "rc_model_create_static");
    total_ = total;
  }
  ~Model() {
    if (m_) rc_model_destroy(m_);
  }
  Model(const Model&) = delete;
  Model& operator=(const Model&) = delete;
  rc_model* get() const { return m_; }
  Context& ctx() const { return *ctx_; }
  // a slot large enough for n symbols in nearly every case (CAPACITY chunks are retried)
  uint64_t slot_capacity(uint64_t n) const {
    uint32_t cmin = 0xFFFFFFFFu;
    for (uint32_t x : c_)
      if (x && x < cmin) cmin = x;
    const double bits = std::log2((double)total_ / (double)cmin);
    return ((uint64_t)std::ceil(n * bits / 8.0 * 1.02 + 64.0) + 15) & ~(uint64_t)15;
  }

 private:
  static std::vector<uint32_t> snapshot_c(const PModel& pm) {
    std::vector<uint32_t> v(pm.alphabet_count());
    for (size_t i = 0; i < v.size(); ++i) v[i] = pm.c_freq(i);
    return v;
  }
  static std::vector<uint32_t> snapshot_cum(const PModel& pm) {
    std::vector<uint32_t> v(pm.alphabet_count());
    for (size_t i = 0; i < v.size(); ++i) v[i] = pm.cum_freq(i);
    return v;
  }
  Context* ctx_;
  rc_model* m_ = nullptr;
  std::vector<uint32_t> c_;
  uint32_t total_ = 0;
};

// Encode many independent chunks (one reference Encoder each) in one launch.
inline std::vector<std::vector<uint8_t>> encode_chunks(
    const Model& m, const std::vector<std::vector<uint8_t>>& chunks) {
  const uint32_t n = (uint32_t)chunks.size();
  std::vector<uint64_t> sym_off(n + 1, 0), cap(n), out_off(n + 1, 0), out_len(n);
  std::vector<uint32_t> flags(n);
  for (uint32_t k = 0; k < n; ++k) {
    sym_off[k + 1] = sym_off[k] + chunks[k].size();
    cap[k] = m.slot_capacity(chunks[k].size());
  }
  std::vector<uint8_t> syms(sym_off[n] ? sym_off[n] : 1);
  for (uint32_t k = 0; k < n; ++k)
    std::copy(chunks[k].begin(), chunks[k].end(), syms.begin() + sym_off[k]);
  std::vector<uint8_t> out;
  for (int attempt = 0; attempt < 2; ++attempt) {
    for (uint32_t k = 0; k < n; ++k) out_off[k + 1] = out_off[k] + cap[k];
    out.assign(out_off[n] ? out_off[n] : 1, 0);
    rc_status s = rc_encode_host(m.ctx().get(), m.get(), syms.data(), sym_off.data(), n,
                                 out.data(), out_off.data(), out_len.data(), flags.data());
    if (s != RC_OK && s != RC_E_CHUNK) check(s, "rc_encode_host");
    bool retry = false;
    for (uint32_t k = 0; k < n; ++k)
      if (flags[k] == RC_F_CAPACITY) {  // exact length is known: retry with it
        cap[k] = (out_len[k] + 15) & ~(uint64_t)15;
        retry = true;
      }
    if (!retry) break;
  }
  std::vector<std::vector<uint8_t>> res(n);
  for (uint32_t k = 0; k < n; ++k) {
    if (flags[k])
      throw RangeCoderError("chunk " + std::to_string(k) + ": " + flag_string(flags[k]),
                            RC_E_CHUNK, flags[k]);
    res[k].assign(out.begin() + out_off[k], out.begin() + out_off[k] + out_len[k]);
  }
  return res;
}

// Decode many independent streams; counts[k] symbols each (out-of-band, sample_impl.rs:113-120)
inline std::vector<std::vector<uint8_t>> decode_chunks(
    const Model& m, const std::vector<std::vector<uint8_t>>& codes,
    const std::vector<uint64_t>& counts) {
  const uint32_t n = (uint32_t)codes.size();
  std::vector<uint64_t> code_off(n), code_len(n), sym_off(n + 1, 0);
  std::vector<uint32_t> flags(n);
  uint64_t tot = 0;
  for (uint32_t k = 0; k < n; ++k) {
    code_off[k] = tot;
    code_len[k] = codes[k].size();
    tot += codes[k].size();
    sym_off[k + 1] = sym_off[k] + counts.at(k);
  }
  std::vector<uint8_t> code(tot + 16, 0), syms(sym_off[n] ? sym_off[n] : 1);
  for (uint32_t k = 0; k < n; ++k)
    std::copy(codes[k].begin(), codes[k].end(), code.begin() + code_off[k]);
  rc_status s = rc_decode_host(m.ctx().get(), m.get(), code.data(), code_off.data(),
                               code_len.data(), syms.data(), sym_off.data(), n, flags.data());
  if (s != RC_OK && s != RC_E_CHUNK) check(s, "rc_decode_host");
  std::vector<std::vector<uint8_t>> res(n);
  for (uint32_t k = 0; k < n; ++k) {
    if (flags[k])
      throw RangeCoderError("chunk " + std::to_string(k) + ": " + flag_string(flags[k]),
                            RC_E_CHUNK, flags[k]);
    res[k].assign(syms.begin() + sym_off[k], syms.begin() + sym_off[k + 1]);
  }
  return res;
}

// Encoder (src/encoder.rs:7-55) for one stream: encode() stages the symbol (it cannot return
// the per-symbol byte count of encoder.rs:36 because nothing is coded before finish()).
class Encoder {
 public:
  Encoder() = default;
  static Encoder new_() { return Encoder(); }
  void encode(const PModel& pm, size_t index) {
    if (pm_ && pm_ != &pm) throw RangeCoderError("one static model per staged stream");
    pm_ = &pm;
    if (index >= pm.alphabet_count() || index > 255)
      throw RangeCoderError("symbol index outside the alphabet", RC_E_CHUNK, RC_F_BAD_SYMBOL);
    syms_.push_back((uint8_t)index);
  }
  // Encoder::finish (encoder.rs:40-46): the stream, 8 + sum of per-symbol bytes long
  std::vector<uint8_t> finish(Context& ctx = Context::default_context()) {
    if (!pm_) return std::vector<uint8_t>(8, 0);  // lower_bound == 0, 8 bytes
    Model m(ctx, *pm_);
    return encode_chunks(m, {syms_})[0];
  }

 private:
  const PModel* pm_ = nullptr;
  std::vector<uint8_t> syms_;
};

// Decoder (src/decoder.rs:6-55) for one stream of n_symbols symbols.
class Decoder {
 public:
  Decoder(std::vector<uint8_t> code, uint64_t n_symbols) : code_(std::move(code)), n_(n_symbols) {
    if (code_.size() < 8)  // Decoder::new panics (decoder.rs:21, :33)
      throw RangeCoderError("code shorter than 8 bytes", RC_E_CHUNK, RC_F_TRUNCATED);
  }
  size_t decode(const PModel& pm, Context& ctx = Context::default_context()) {
    if (!decoded_) {
      Model m(ctx, pm);
      out_ = decode_chunks(m, {code_}, {n_})[0];
      decoded_ = true;
    }
    if (pos_ >= out_.size()) throw RangeCoderError("more decode() calls than n_symbols");
    return out_[pos_++];
  }

 private:
  std::vector<uint8_t> code_, out_;
  uint64_t n_;
  size_t pos_ = 0;
  bool decoded_ = false;
};

}  // namespace rc

#endif  // RANGE_CODER_AMD_HPP
