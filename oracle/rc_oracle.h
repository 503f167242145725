/*
 * rc_oracle.h — CPU restatement of diegodox/range_coder_rust (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity oracle, not product code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / the timed CPU baseline.
 * The product path (range_coder_rust_amd/, librc_amd.so) never links or calls it.
 *
 * Parity status: the reference is Rust and no Rust toolchain exists in this image, so the
 * reference cannot be compiled or run here.  The oracle is pinned by
 *   (1) the reference's only test, the examples/sample_impl.rs:72-128 round trip
 *       (decode(encode(x)) == x on its 10-symbol table, incl. a zero-frequency bin);
 *   (2) known-answer vectors K1-K3 from SURVEY.md §8c, derived independently of this file;
 *   (3) oracle/ref_literal.py, a line-by-line pure-Python restatement of the Rust source.
 * Byte-stream parity against an executed reference binary is UNPINNED (no rustc/cargo).
 */
#ifndef RC_ORACLE_H
#define RC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-chunk flags: identical bit values to include/range_coder.h RC_F_* */
#define ORC_F_ZERO_FREQ  1u  /* encode of a c==0 symbol: reference loops forever (range_coder.rs:83-85) */
#define ORC_F_BAD_SYMBOL 2u  /* symbol index >= alphabet: reference panics (sample_impl.rs:19 unwrap) */
#define ORC_F_CAPACITY   4u  /* encoded stream longer than its output slot */
#define ORC_F_TRUNCATED  8u  /* decoder ran out of code bytes: reference panics (decoder.rs:33) */
#define ORC_F_CORRUPT   16u  /* decoder selected a c==0 symbol: reference loops forever */
#define ORC_F_BAD_MODEL 64u  /* (c, cum, total) on which the reference panics: total == 0
                                (division by zero, range_coder.rs:38-40), LowerBoundOverflow
                                (:68-81) or UpperBoundOverflow (:138-146) */
#define ORC_F_FINISHED 128u  /* encode after Encoder::finish (which consumes it, encoder.rs:40) */

typedef struct orc_range_coder {
    uint64_t lower_bound; /* range_coder.rs:9  */
    uint64_t range;       /* range_coder.rs:11 */
} orc_range_coder;

/* RangeCoder::default (range_coder.rs:13-20) */
void orc_rc_init(orc_range_coder* rc);
/* RangeCoder::param_update (range_coder.rs:53-92).  Writes the settled bytes to out (<= 16),
 * returns their count, or -1 when c_freq makes the reference's renormalisation loop diverge. */
int orc_param_update(orc_range_coder* rc, uint32_t c_freq, uint32_t cum_freq, uint32_t total_freq,
                     uint8_t out[16]);

/* Encoder::new + n x Encoder::encode + Encoder::finish (encoder.rs:14-46) on one stream.
 * Writes min(len, cap) bytes; *out_len = exact stream length.  Returns ORC_F_* flags. */
uint32_t orc_encode(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                    const uint8_t* syms, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len);

/* Decoder::new + n x Decoder::decode (decoder.rs:14-54) with the sample FreqTable::find_index
 * (sample_impl.rs:27-45).  Returns ORC_F_* flags. */
uint32_t orc_decode(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                    const uint8_t* code, uint64_t code_len, uint64_t n, uint8_t* syms_out);

/* Batch drivers over independent chunks on `threads` host threads (chunk = one Encoder). */
void orc_encode_batch(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                      const uint8_t* syms, const uint64_t* sym_off, uint32_t n_chunks,
                      uint8_t* out, const uint64_t* out_off, uint64_t* out_len, uint32_t* flags,
                      int threads);
void orc_decode_batch(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                      const uint8_t* code, const uint64_t* code_off, const uint64_t* code_len,
                      uint8_t* syms_out, const uint64_t* sym_off, uint32_t n_chunks,
                      uint32_t* flags, int threads);

/* Build-defined adaptive order-0 model (not in the reference), per chunk:
 * c[i] = 1 for i < n_alpha; after coding the i-th symbol s (0-based): c[s] += inc, and if
 * (i + 1) % period == 0 and the total exceeds limit, every c = (c + 1) >> 1.
 * The coder sees (c[s], cum[s], total) of the model BEFORE the update, through the reference's
 * PModel interface (pmodel.rs:4-12); the decoder's index search is FreqTable::find_index's. */
uint32_t orc_encode_adaptive(uint32_t n_alpha, uint32_t inc, uint32_t limit, uint32_t period,
                             const uint8_t* syms, uint64_t n, uint8_t* out, uint64_t cap,
                             uint64_t* out_len);
uint32_t orc_decode_adaptive(uint32_t n_alpha, uint32_t inc, uint32_t limit, uint32_t period,
                             const uint8_t* code, uint64_t code_len, uint64_t n, uint8_t* syms_out);

/* Resumable single streams (the rc_stream_* entry points of include/range_coder.h): the state of
 * one reference Encoder or Decoder between calls.  stage: 0 fresh (a decoder has not yet run
 * Decoder::new), 1 running, 2 finished (encoder).  flags: sticky first error. */
typedef struct orc_stream {
    uint64_t lower_bound, range; /* RangeCoder (range_coder.rs:7-12) */
    uint64_t data;               /* Decoder::data (decoder.rs:8) */
    uint64_t pos;                /* encoder: bytes emitted; decoder: bytes consumed */
    uint64_t n;                  /* symbols coded */
    uint32_t flags, stage;
} orc_stream;

void orc_stream_init(orc_stream* st);
/* n x Encoder::encode with the (c_freq, cum_freq, total_freq) triple read per call
 * (encoder.rs:24-37), then Encoder::finish if `finish` (encoder.rs:40-46).  New bytes go to
 * out[0..); *out_len = their count; nbytes[i] = the return value of the i-th encode().  The
 * state advances over the symbols coded before an error.  cap < 12 n (+ 8 with finish):
 * ORC_F_CAPACITY, nothing done.  Returns the flags. */
uint32_t orc_stream_encode(orc_stream* st, const uint32_t* triples, uint64_t n, uint8_t* out,
                           uint64_t cap, uint64_t* out_len, uint8_t* nbytes, int finish);
/* Decoder::new (if fresh) + n x Decoder::decode (decoder.rs:14-54) with the sample
 * FreqTable::find_index (sample_impl.rs:27-45) over an arbitrary (c, cum) table: code[0..code_len)
 * is the whole stream (st->pos indexes it).  Stops before the first symbol that errs; *n_done
 * symbols were written to syms.  Returns the flags. */
uint32_t orc_stream_decode(orc_stream* st, const uint32_t* c, const uint32_t* cum,
                           uint32_t n_alpha, uint32_t total, const uint8_t* code,
                           uint64_t code_len, uint8_t* syms, uint64_t n, uint64_t* n_done);

/* FNV-1a 64 of a byte string (used by the known-answer tests). */
uint64_t orc_fnv1a64(const uint8_t* p, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
