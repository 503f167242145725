// range_coder.hpp — C++ host API over the C ABI (include/range_coder.h), mirroring the public
// surface of diegodox/range_coder_rust (src/lib.rs:1-13) for host programs.
//
//   trait PModel            (src/pmodel.rs:4-41)         -> rc::PModel (abstract class)
//   FreqTable example model (examples/sample_impl.rs)    -> rc::FreqTable
//   RangeCoder accessors      (src/range_coder.rs:26-146) -> rc::RangeCoder (a state snapshot)
//   Encoder::new/encode/peek_code/finish, pub range_coder
//                             (src/encoder.rs:7-55)       -> rc::Encoder (model read per call;
//                                                           encode() returns a ByteCount)
//   Decoder::new/decode/range_coder/data
//                             (src/decoder.rs:6-55)       -> rc::Decoder (model read per call)
//   error::RangeCoderError     (src/error.rs:3-13)       -> rc::RangeCoderError (exception)
//   (new) batch API                                      -> rc::encode_chunks / decode_chunks
//
// Header-only; link with librc_amd.so.  Everything runs on the GPU through the C ABI: there is
// no CPU implementation of the coder in the product.
#ifndef RANGE_CODER_AMD_HPP
#define RANGE_CODER_AMD_HPP

#include <algorithm>
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
  // error.rs:3-13: which reference error a BAD_MODEL flag stands for, with its payload
  enum Kind { OTHER = 0, LOWER_BOUND_OVERFLOW, UPPER_BOUND_OVERFLOW, DIVIDE_BY_ZERO };
  RangeCoderError(const std::string& what, int status = 0, uint32_t flags = 0)
      : std::runtime_error(what), status(status), flags(flags) {}
  int status;      // rc_status of the failing call
  uint32_t flags;  // RC_F_* of the failing chunk (0 if not chunk-specific)
  Kind kind = OTHER;
  // LowerBoundOverflow {lower_bound, add_val, range} / UpperBoundOverflow {lower_bound, range}
  uint64_t lower_bound = 0, add_val = 0, range = 0;
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
  if (f & RC_F_TOO_LONG) s += "TOO_LONG|";
  if (f & RC_F_BAD_MODEL) s += "BAD_MODEL|";
  if (f & RC_F_FINISHED) s += "FINISHED|";
  if (!s.empty()) s.pop_back();
  return s;
}

class Decoder;

// trait PModel (src/pmodel.rs:4-41)
class PModel {
 public:
  static constexpr size_t kCanonical = ~(size_t)0;
  virtual ~PModel() = default;
  virtual uint32_t c_freq(size_t index) const = 0;    // pmodel.rs:6
  virtual uint32_t cum_freq(size_t index) const = 0;  // pmodel.rs:8
  virtual uint32_t total_freq() const = 0;            // pmodel.rs:10
  // pmodel.rs:12.  Not overridden (returns kCanonical): the GPU decoder evaluates
  // FreqTable::find_index (sample_impl.rs:27-45) itself and decodes ahead.  Overridden:
  // Decoder::decode calls it at every symbol with the decoder (range_coder(), data() give the
  // exact state), as decoder.rs:40 does, and param_update uses the index it returns.
  virtual size_t find_index(const Decoder&) const { return kCanonical; }
  // An override that keeps FreqTable's binary-search semantics may return true here to keep
  // the decode-ahead path (its find_index is then not called).
  virtual bool canonical_find_index() const { return false; }
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

// RangeCoder (src/range_coder.rs:7-146): the public accessors of a coder state (a snapshot: a
// stream's state lives with its GPU calls, rc_stream_state)
class RangeCoder {
 public:
  static constexpr uint64_t TOP8 = 1ull << 56;   // range_coder.rs:23
  static constexpr uint64_t TOP16 = 1ull << 48;  // range_coder.rs:24
  RangeCoder() = default;                         // Default (:13-20)
  RangeCoder(uint64_t lower_bound, uint64_t range) : low_(lower_bound), range_(range) {}
  static RangeCoder new_() { return RangeCoder(); }
  uint64_t lower_bound() const { return low_; }  // :30-32
  uint64_t range() const { return range_; }      // :33-35
  uint64_t range_par_total(uint32_t total_freq) const {  // :38-40
    if (total_freq == 0) throw RangeCoderError("range_par_total: attempt to divide by zero");
    return range_ / total_freq;
  }
  uint64_t upper_bound() const {  // :138-146
    const uint64_t u = low_ + range_;
    if (u < low_) throw RangeCoderError("UpperBoundOverflow");
    return u;
  }
  bool operator==(const RangeCoder& o) const { return low_ == o.low_ && range_ == o.range_; }

 private:
  uint64_t low_ = 0, range_ = ~0ull;
};

inline void throw_flags(uint32_t f, const std::string& where) {
  if (f) throw RangeCoderError(where + ": " + flag_string(f), RC_E_CHUNK, f);
}

// The reference's error for a BAD_MODEL symbol coded from state (low, range) with (c, cum,
// total): param_update's own arithmetic (range_coder.rs:53-81, :138-146; u64 products wrap).
[[noreturn]] inline void throw_bad_model(uint64_t low, uint64_t range, uint32_t c, uint32_t cum,
                                         uint32_t total, const std::string& where) {
  RangeCoderError e(where + ": BAD_MODEL", RC_E_CHUNK, RC_F_BAD_MODEL);
  if (total == 0) {
    e = RangeCoderError(where + ": range_par_total: attempt to divide by zero", RC_E_CHUNK,
                        RC_F_BAD_MODEL);
    e.kind = RangeCoderError::DIVIDE_BY_ZERO;
    throw e;
  }
  const uint64_t r = range / total, nr = r * c, add = r * cum;
  if (low + add < add) {
    e = RangeCoderError(where + ": LowerBoundOverflow", RC_E_CHUNK, RC_F_BAD_MODEL);
    e.kind = RangeCoderError::LOWER_BOUND_OVERFLOW;
    e.lower_bound = low, e.add_val = add, e.range = nr;
  } else if (low + add + nr < nr) {
    e = RangeCoderError(where + ": UpperBoundOverflow", RC_E_CHUNK, RC_F_BAD_MODEL);
    e.kind = RangeCoderError::UPPER_BOUND_OVERFLOW;
    e.lower_bound = low + add, e.range = nr;
  }
  throw e;
}

class Encoder;

// Encoder::encode's return value (encoder.rs:34-36: the bytes that symbol settled).  Symbols
// are staged and coded on the GPU in batches; converting to uint32_t flushes them if needed.
// Valid while its Encoder lives.
class ByteCount {
 public:
  ByteCount(Encoder* e, uint64_t i) : e_(e), i_(i) {}
  operator uint32_t() const;

 private:
  Encoder* e_;
  uint64_t i_;
};

// Encoder (src/encoder.rs:7-55) for one stream, with the reference's per-call semantics:
// encode() reads (c_freq(index), cum_freq(index), total_freq()) at that call
// (encoder.rs:24-31), so a PModel the caller changes between calls is coded exactly as the
// reference codes it.  The staged triples are coded by the resumable stream kernel
// (rc_stream_encode_host) when a result is needed: peek_code(), range_coder(), finish(), a
// ByteCount's value, or every 2^20 symbols.  No length limit.
class Encoder {
 public:
  static constexpr size_t FLUSH_AT = 1u << 20;
  explicit Encoder(Context& ctx = Context::default_context()) : ctx_(&ctx) {}
  Encoder(const Encoder&) = delete;
  Encoder& operator=(const Encoder&) = delete;
  static Encoder new_() { return Encoder(); }  // encoder.rs:14-16

  ByteCount encode(const PModel& pm, size_t index) {  // encoder.rs:24-37
    if (finished_) throw RangeCoderError("encode after finish", RC_E_CHUNK, RC_F_FINISHED);
    if (index >= pm.alphabet_count())  // sample_impl.rs:19: get(index).unwrap() panics
      throw RangeCoderError("symbol index outside the alphabet", RC_E_CHUNK, RC_F_BAD_SYMBOL);
    const uint32_t c = pm.c_freq(index), cum = pm.cum_freq(index), total = pm.total_freq();
    if (c == 0)  // range_coder.rs:83-85 would never terminate
      throw RangeCoderError("encode: c_freq == 0", RC_E_CHUNK, RC_F_ZERO_FREQ);
    if (total == 0)  // range_coder.rs:38-40 divides by zero
      throw RangeCoderError("encode: total_freq == 0", RC_E_CHUNK, RC_F_BAD_MODEL);
    trip_.insert(trip_.end(), {c, cum, total});
    const uint64_t i = staged0_ + trip_.size() / 3 - 1;
    if (trip_.size() >= 3 * FLUSH_AT) flush(false);
    return ByteCount(this, i);
  }
  const std::vector<uint8_t>& peek_code() {  // encoder.rs:18-20
    flush(false);
    return code_;
  }
  RangeCoder range_coder() {  // the pub field of encoder.rs:8 (a snapshot)
    flush(false);
    return RangeCoder(st_.lower_bound, st_.range);
  }
  std::vector<uint8_t> finish() {  // encoder.rs:40-46
    if (finished_) throw RangeCoderError("finish twice", RC_E_CHUNK, RC_F_FINISHED);
    flush(true);
    finished_ = true;
    return code_;
  }
  uint32_t count(uint64_t i) {
    if (i >= staged0_) flush(false);
    if (i >= counts_.size()) throw RangeCoderError("symbol not coded (an earlier one failed)");
    return counts_[i];
  }

 private:
  void flush(bool finish) {
    const uint64_t n = trip_.size() / 3;
    if (n == 0 && !finish) return;
    throw_flags(st_.flags, "encode");
    const uint64_t cap = RC_STREAM_MAX_BYTES(n, finish);
    std::vector<uint8_t> out(cap ? cap : 1), nb(n ? n : 1);
    uint64_t len = 0;
    uint32_t fl = 0;
    const uint64_t n0 = st_.n;
    const rc_status s = rc_stream_encode_host(ctx_->get(), &st_, trip_.data(), n, out.data(), cap,
                                              &len, nb.data(), finish ? 1u : 0u, &fl);
    if (s != RC_OK && s != RC_E_CHUNK) check(s, "rc_stream_encode_host");
    code_.insert(code_.end(), out.begin(), out.begin() + len);
    const uint64_t done = st_.n - n0;
    counts_.insert(counts_.end(), nb.begin(), nb.begin() + done);
    staged0_ += n;
    const std::string where = "encode (symbol " + std::to_string(st_.n) + ")";
    if ((fl & RC_F_BAD_MODEL) && done < n) {
      const uint32_t* t = trip_.data() + 3 * done;
      const uint32_t c = t[0], cum = t[1], total = t[2];
      trip_.clear();
      throw_bad_model(st_.lower_bound, st_.range, c, cum, total, where);
    }
    trip_.clear();
    throw_flags(fl, where);
  }
  Context* ctx_;
  rc_stream_state st_ = RC_STREAM_STATE_INIT;
  std::vector<uint8_t> code_, counts_;
  std::vector<uint32_t> trip_;
  uint64_t staged0_ = 0;
  bool finished_ = false;
};

inline ByteCount::operator uint32_t() const { return e_->count(i_); }

// Decoder (src/decoder.rs:6-55) for one stream, with the reference's per-call semantics:
// decode() reads the model's table at that call and decodes with FreqTable::find_index's
// binary search and param_update (sample_impl.rs:27-45, decoder.rs:38-54) on the GPU
// (rc_stream_decode_host).  Symbols are decoded ahead in blocks that double while the table
// stays the same; when the caller's table changes the state at that symbol is re-derived, so
// every symbol is decoded with the table held at its call.  A PModel that overrides find_index
// gets it called per symbol and its index decoded (one GPU step per symbol, launch-bound).
class Decoder {
 public:
  static constexpr uint64_t MAX_BLOCK = 1u << 20;
  // Decoder::new (decoder.rs:14-23): a code shorter than 8 bytes panics there
  explicit Decoder(std::vector<uint8_t> code, Context& ctx = Context::default_context())
      : Decoder(std::move(code), ~0ull, ctx) {}
  // n_symbols: the out-of-band count (sample_impl.rs:113-120); only bounds the decode-ahead
  Decoder(std::vector<uint8_t> code, uint64_t n_symbols, Context& ctx = Context::default_context())
      : ctx_(&ctx), code_(std::move(code)), limit_(n_symbols) {
    if (code_.size() < 8)
      throw RangeCoderError("code shorter than 8 bytes", RC_E_CHUNK, RC_F_TRUNCATED);
    Table t{{1}, {0}, 1};
    run(start_, t, 0, nullptr);  // prime the data window
    end_ = start_;
  }
  static Decoder new_(std::vector<uint8_t> code) { return Decoder(std::move(code)); }

  size_t decode(const PModel& pm) {  // decoder.rs:38-54
    if (!pm.canonical_find_index()) {
      const size_t idx = pm.find_index(*this);  // reads range_coder() / data() at this symbol
      if (idx != PModel::kCanonical) return decode_index(pm, idx);
    }
    table_of(pm, tmp_);  // (into reused vectors: no allocation per call)
    Table& t = tmp_;
    const bool same = have_ && t == sig_;
    if (same && bpos_ < buf_.size()) {
      ++taken_;
      return buf_[bpos_++];
    }
    if (same && err_) decode_error(end_, t, err_);
    block_ = (same && bpos_ == buf_.size()) ? std::min<uint64_t>(2 * block_, MAX_BLOCK) : 1;
    rc_stream_state st = here();
    uint64_t n = block_;
    if (limit_ != ~0ull) n = std::max<uint64_t>(1, std::min<uint64_t>(n, limit_ - taken_));
    const rc_stream_state start = st;
    std::vector<uint8_t>& out = spare_;  // (reused: swapped with buf_ below)
    out.resize(n);
    const uint32_t fl = run(st, t, n, out.data());
    out.resize(st.n - start.n);
    start_ = start;
    end_ = st;
    buf_.swap(out);
    bpos_ = 0;
    std::swap(sig_, t);  // (member-wise: the vectors swap their storage)
    have_ = true;
    err_ = fl;
    if (buf_.empty()) decode_error(start, sig_, fl);
    ++taken_;
    return buf_[bpos_++];
  }
  RangeCoder range_coder() const {  // decoder.rs:24-26 (a snapshot)
    const rc_stream_state st = here();
    return RangeCoder(st.lower_bound, st.range);
  }
  uint64_t data() const { return here().data; }  // decoder.rs:27-29

 private:
  struct Table {
    std::vector<uint32_t> c, cum;
    uint32_t total;
    bool operator==(const Table& o) const { return total == o.total && c == o.c && cum == o.cum; }
  };
  // decoder.rs:38-54 with the caller's find_index: param_update and shift_left_buffer for the
  // index it returned, on the GPU (a one-entry table, so the kernel's search has no choice)
  size_t decode_index(const PModel& pm, size_t idx) {
    const rc_stream_state st = here();
    Table t{{pm.c_freq(idx)}, {pm.cum_freq(idx)}, pm.total_freq()};
    rc_stream_state nxt = st;
    uint8_t sym = 0;
    const uint32_t fl = run(nxt, t, 1, &sym);
    const std::string where = "decode (symbol " + std::to_string(taken_) + ")";
    if (nxt.n == st.n) {
      if (fl & RC_F_BAD_MODEL) throw_bad_model(st.lower_bound, st.range, t.c[0], t.cum[0], t.total, where);
      throw_flags(fl, where);
    }
    start_ = end_ = nxt;
    buf_.clear();
    bpos_ = 0;
    have_ = false;
    err_ = 0;
    ++taken_;
    return idx;
  }
  // the reference's error for a decode that stopped at state st under table t
  [[noreturn]] void decode_error(const rc_stream_state& st, const Table& t, uint32_t fl) const {
    const std::string where = "decode (symbol " + std::to_string(taken_) + ")";
    if ((fl & RC_F_BAD_MODEL) && t.total && !t.c.empty()) {
      // the index FreqTable::find_index chose (sample_impl.rs:29-44), for the error's payload
      const uint64_t rf = (st.data - st.lower_bound) / (st.range / t.total);
      size_t left = 0, right = t.c.size() - 1;
      while (left < right) {
        const size_t mid = (left + right) / 2;
        if ((uint64_t)t.cum[mid + 1] <= rf) left = mid + 1;
        else right = mid;
      }
      throw_bad_model(st.lower_bound, st.range, t.c[left], t.cum[left], t.total, where);
    }
    if (fl & RC_F_BAD_MODEL) throw_bad_model(st.lower_bound, st.range, 0, 0, t.total, where);
    throw_flags(fl ? fl : RC_F_CORRUPT, where);
    throw RangeCoderError(where);
  }
  static void table_of(const PModel& pm, Table& t) {
    const size_t n = pm.alphabet_count();
    t.c.resize(n);
    t.cum.resize(n);
    for (size_t i = 0; i < n; ++i) {
      t.c[i] = pm.c_freq(i);
      t.cum[i] = pm.cum_freq(i);
    }
    t.total = pm.total_freq();
  }
  uint32_t run(rc_stream_state& st, const Table& t, uint64_t n, uint8_t* out) const {
    uint32_t fl = 0;
    uint8_t dummy = 0;
    const rc_status s = rc_stream_decode_host(ctx_->get(), t.c.data(), t.cum.data(),
                                              (uint32_t)t.c.size(), t.total, &st, code_.data(),
                                              code_.size(), out ? out : &dummy, n, &fl);
    if (s != RC_OK && s != RC_E_CHUNK) check(s, "rc_stream_decode_host");
    return fl;
  }
  // the state at the current symbol (re-derived inside a block, which then starts here)
  rc_stream_state here() const {
    if (bpos_ == 0) return start_;
    if (bpos_ == buf_.size()) {
      rc_stream_state st = end_;
      st.flags = 0;
      return st;
    }
    rc_stream_state st = start_;
    std::vector<uint8_t> tmp(bpos_);
    run(st, sig_, bpos_, tmp.data());
    start_ = st;
    buf_.erase(buf_.begin(), buf_.begin() + bpos_);
    bpos_ = 0;
    return st;
  }
  // (the decode-ahead block is a cache of the stream: range_coder() / data() re-derive into it)
  Context* ctx_;
  std::vector<uint8_t> code_;
  mutable std::vector<uint8_t> buf_;
  uint64_t limit_;
  mutable rc_stream_state start_ = RC_STREAM_STATE_INIT;
  rc_stream_state end_ = RC_STREAM_STATE_INIT;
  mutable size_t bpos_ = 0;
  Table sig_, tmp_;                // the table of the decoded-ahead block; the caller's, read now
  std::vector<uint8_t> spare_;     // the next block's symbols before they replace buf_
  bool have_ = false;
  uint32_t err_ = 0;
  uint64_t block_ = 1, taken_ = 0;
};

}  // namespace rc

#endif  // RANGE_CODER_AMD_HPP
