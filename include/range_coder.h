/*
 * range_coder.h — C ABI of the MI355X-native batched range coder (librc_amd.so).
 *
 * Drop-in boundary for the encode/decode hot path of diegodox/range_coder_rust.  The reference
 * exposes a per-stream, per-symbol Rust API (src/lib.rs:1-13):
 *     Encoder::new / encode<T: PModel>(&T, usize) -> u32 / finish() -> VecDeque<u8>
 *         (src/encoder.rs:14-46)
 *     Decoder::new(code) / decode<T: PModel>(&T) -> usize      (src/decoder.rs:14-54)
 *     trait PModel { c_freq, cum_freq, total_freq, find_index } (src/pmodel.rs:4-12)
 * Each of these entry points replaces the reference's per-symbol loops over many independent
 * streams ("chunks", one fresh Encoder/Decoder each) with one kernel launch.  The emitted bytes
 * of every chunk are bit-identical to Encoder::encode* + Encoder::finish on the same symbols.
 *
 * Conventions
 *  - Plain pointers and sizes only.  "dev" pointers are HIP device (or managed) memory; "host"
 *    pointers are ordinary host memory.  No exceptions or panics cross this boundary.
 *  - Every function returns an rc_status (RC_OK == 0).  Data-dependent problems of a single
 *    chunk are reported per chunk in a uint32 flags array (RC_F_*), never by aborting.
 *  - Batch calls are asynchronous and stream-ordered on the context's stream.
 *  - Offsets: chunk k's symbols are sym[sym_off[k] .. sym_off[k+1]) (n_chunks+1 entries,
 *    non-decreasing, any alignment).  Encoder output slot k is out[out_off[k] .. out_off[k+1]).
 */
#ifndef RANGE_CODER_AMD_H
#define RANGE_CODER_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (function results) ---- */
typedef int rc_status;
#define RC_OK 0
#define RC_E_ARG (-1)       /* null handle/pointer, n_chunks too large, bad parameter */
#define RC_E_BAD_MODEL (-2) /* frequency table rejected (see rc_model_create_static) */
#define RC_E_DEVICE (-3)    /* HIP runtime error (launch, allocation, copy) */
#define RC_E_NO_DEVICE (-4) /* no gfx950 device visible / device index out of range */
#define RC_E_CHUNK (-5)     /* synchronous helpers only: at least one chunk has a flag set */
#define RC_E_BAD_CONTAINER (-6) /* container header / index malformed or inconsistent */
#define RC_E_CAPACITY (-7)  /* destination buffer too small (the needed size is reported) */

/* ---- per-chunk flags (bitwise; the first error of a chunk wins) ----
 * Where the reference panics or never terminates, the kernels flag the chunk instead.      */
#define RC_F_ZERO_FREQ 1u  /* encode of a symbol with c_freq == 0: the reference loops forever
                              in no_carry_expansion (range_coder.rs:83-85, 110-116)          */
#define RC_F_BAD_SYMBOL 2u /* symbol index >= n_symbols: the reference panics
                              (examples/sample_impl.rs:19, Vec::get().unwrap())              */
#define RC_F_CAPACITY 4u   /* encoded chunk longer than its output slot; out_len[k] still holds
                              the exact length so the caller can retry with a larger slot   */
#define RC_F_TRUNCATED 8u  /* decoder needed a byte past code_len: the reference panics
                              (decoder.rs:33, pop_front().unwrap())                         */
#define RC_F_CORRUPT 16u   /* decoder selected a c_freq == 0 symbol (only possible on corrupt
                              input): the reference loops forever                            */
#define RC_F_BAD_MODEL 64u /* stream API: a (c, cum, total) on which the reference panics — total
                              0 (u64 division by zero, range_coder.rs:38-40), LowerBoundOverflow
                              (:68-81) or UpperBoundOverflow (upper_bound().unwrap(), :138-146) */
#define RC_F_FINISHED 128u /* stream API: encode after Encoder::finish, which consumes the
                              encoder (encoder.rs:40)                                        */
#define RC_F_TOO_LONG 32u  /* chunk of more than RC_MAX_CHUNK_SYMBOLS symbols: the batch kernels
                              keep 32-bit in-chunk stream positions, so such a chunk is neither
                              read nor written (out_len 0).  The reference has no limit
                              (VecDeque, encoder.rs:7-11): code a longer stream with the
                              resumable stream entry points (rc_stream_*), which have none    */

/* Longest chunk of the batch entry points.  A symbol settles at most 12 code bytes (5 in
 * no_carry_expansion, range_coder.rs:110-116, and 7 in range_reduction_expansion, :126-135;
 * DESIGN.md §3), so 2^25 symbols stay below 2^29 code bytes = 2^32 bits. */
#define RC_MAX_CHUNK_SYMBOLS (1ull << 25)

/* Maximum chunks per batch call (grid limit) */
#define RC_MAX_CHUNKS (1u << 28)

typedef struct rc_ctx rc_ctx;     /* one device + one stream; use one per host thread */

/* Environment.  rc_ctx_create reads these switches once and the context keeps them; nothing
 * reads the environment per launch or per call (changing a variable affects contexts created
 * after the change only).  Unset is the default.
 *   RC_PRIO=off             wave priorities off (every launch oldest-first)
 *   RC_DEC_PAIR=512|1024    decode 2^15 < total <= 2^16 static models with the pair-bucket
 *                           decoder in workgroups of that size (measurements; slower)
 *   RC_STREAM_SERVICE=0     per-call stream entry points launch a kernel per call instead of
 *                           using the stream-service wave
 *   RC_STREAM_DMA=1         host pipeline (rc_*_host): every transfer by DMA engine copies
 *   RC_STREAM_DIRECT=0      host pipeline: stage outputs in HBM instead of writing them into
 *                           mapped host memory from the kernel
 *   RC_STREAM_BATCH_BYTES=n host pipeline batch size in input bytes (default 2 GiB)
 *   RC_HIST_HOT=0           rc_histogram without its ballot-counted most frequent symbol */
typedef struct rc_model rc_model; /* device-resident snapshot of a PModel */

/* ---- context ---- */
rc_status rc_ctx_create(int device, rc_ctx** out);
rc_status rc_ctx_destroy(rc_ctx* ctx);
/* Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL is the HIP null (legacy default) stream.  rc_ctx_reset_stream returns to the
 * context's own non-blocking stream. */
rc_status rc_ctx_set_stream(rc_ctx* ctx, void* hip_stream);
rc_status rc_ctx_reset_stream(rc_ctx* ctx);
rc_status rc_ctx_synchronize(rc_ctx* ctx);
const char* rc_status_string(rc_status s);
/* Text of the last HIP runtime error seen by this thread ("" if none) */
const char* rc_last_error(void);
/* Library / device info: writes a short NUL-terminated description (arch, CUs) */
rc_status rc_device_info(int device, char* buf, size_t buf_len);

/* ---- models (the PModel plug-in point, pmodel.rs:4-12) ----
 * Static model: a snapshot of PModel::c_freq(i), cum_freq(i) (i < n_symbols) and total_freq().
 * Accepted when 1 <= n_symbols <= 256, total_freq >= 1, cum_freq[0] == 0,
 * cum_freq[i+1] == cum_freq[i] + c_freq[i] and cum_freq[n-1] + c_freq[n-1] == total_freq
 * (the tables FreqTable::calc_cum builds, sample_impl.rs:61-69).  The decoder then uses the
 * canonical inverse cum[s] <= rfreq < cum[s+1] — exactly FreqTable::find_index
 * (sample_impl.rs:27-45), including its choice of n_symbols-1 when rfreq >= total.
 * Zero-frequency symbols are allowed in the table (they are just never encodable).       */
rc_status rc_model_create_static(rc_ctx* ctx, uint32_t n_symbols, const uint32_t* c_freq_host,
                                 const uint32_t* cum_freq_host, uint32_t total_freq,
                                 rc_model** out);
/* Adaptive order-0 model (build-defined; the reference ships none).
 * Per chunk, c[i] = 1 for i < n_symbols.  After coding the i-th symbol s (0-based):
 * c[s] += increment, and if (i + 1) % period == 0 and the total exceeds limit, every
 * c[i] = (c[i] + 1) >> 1.  The coder sees (c[s], cum[s], total) before the update.
 * Accepted when 1 <= n_symbols <= 256, increment >= 1, period is a power of two <= 65536 and
 * n_symbols + increment*period <= limit <= 65535 - increment*period (so the total, and every
 * count, stays below 2^16 for all inputs).  Default (config C4): increment 32, limit 57343,
 * period 256.                                                                               */
rc_status rc_model_create_adaptive(rc_ctx* ctx, uint32_t n_symbols, uint32_t increment,
                                   uint32_t limit, uint32_t period, rc_model** out);
rc_status rc_model_destroy(rc_model* m);

/* ---- batch encode (replaces n_chunks x {Encoder::new; encode...; finish}) ----
 * syms_dev      symbol bytes (index < n_symbols), chunk k = [sym_off[k], sym_off[k+1])
 * sym_off_dev   n_chunks+1 offsets into syms_dev
 * out_dev       output arena; chunk k's stream is written at out_off[k], capacity
 *               out_off[k+1]-out_off[k] bytes (any alignment; 16-B aligned is fastest)
 * out_len_dev   n_chunks: exact stream length (== 8 + sum of encode() return values);
 *               slot bytes past out_len are unspecified, nothing outside the slot is written
 * flags_dev     n_chunks: RC_F_* (0 == success)                                         */
rc_status rc_encode_batch(rc_ctx* ctx, const rc_model* m, const uint8_t* syms_dev,
                          const uint64_t* sym_off_dev, uint32_t n_chunks, uint8_t* out_dev,
                          const uint64_t* out_off_dev, uint64_t* out_len_dev,
                          uint32_t* flags_dev);

/* ---- batch decode (replaces n_chunks x {Decoder::new(code); n x decode}) ----
 * code_dev      code arena; chunk k's stream = code[code_off[k] .. code_off[k]+code_len[k])
 * code_off_dev, code_len_dev   n_chunks entries each
 * syms_out_dev  decoded symbols; chunk k gets sym_off[k+1]-sym_off[k] symbols (the count is
 *               out-of-band, as in the reference: sample_impl.rs:113-120)
 * flags_dev     n_chunks: RC_F_* (0 == success)                                         */
rc_status rc_decode_batch(rc_ctx* ctx, const rc_model* m, const uint8_t* code_dev,
                          const uint64_t* code_off_dev, const uint64_t* code_len_dev,
                          uint8_t* syms_out_dev, const uint64_t* sym_off_dev, uint32_t n_chunks,
                          uint32_t* flags_dev);

/* ---- synchronous host-memory helpers (stage through device memory, wait for completion;
 *      returns RC_E_CHUNK when any chunk is flagged — flags are still filled in).  Their
 *      staging buffers (4 x ~2 batches of ~1 GiB, on the context's device) stay allocated
 *      with the context between calls and are freed by rc_ctx_destroy. ---- */
rc_status rc_encode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* syms,
                         const uint64_t* sym_off, uint32_t n_chunks, uint8_t* out,
                         const uint64_t* out_off, uint64_t* out_len, uint32_t* flags);
rc_status rc_decode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                         const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                         const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags);

/* ---- several devices of one node from one host thread (the rc_*_multi entry points) ----
 * rc_encode_host / rc_decode_host over a list of contexts (one per device; two contexts on one
 * device also work): the chunks are cut into n_ctx contiguous ranges of about equal input
 * bytes, coded concurrently (one host thread per context).  Chunks are independent streams
 * (a fresh Encoder each, encoder.rs:48-55), so there is no data-path exchange between devices:
 * every device reads its range of the caller's buffers and writes its chunks' results in place.
 * models[i] is the model as created on ctxs[i]'s device (identical tables).  Returns the first
 * failing status, RC_E_CHUNK when a chunk is flagged, else RC_OK.                             */
rc_status rc_encode_host_multi(rc_ctx* const* ctxs, const rc_model* const* models, uint32_t n_ctx,
                               const uint8_t* syms, const uint64_t* sym_off, uint32_t n_chunks,
                               uint8_t* out, const uint64_t* out_off, uint64_t* out_len,
                               uint32_t* flags);
rc_status rc_decode_host_multi(rc_ctx* const* ctxs, const rc_model* const* models, uint32_t n_ctx,
                               const uint8_t* code, const uint64_t* code_off,
                               const uint64_t* code_len, uint8_t* syms_out,
                               const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags);

/* ---- resumable streams: the reference's per-call Encoder / Decoder (any PModel) ----
 * The batch entry points code whole chunks against one table.  The reference instead reads the
 * model on EVERY call — Encoder::encode takes (c_freq(i), cum_freq(i), total_freq()) of the
 * caller's PModel at that moment (encoder.rs:24-31), Decoder::decode runs find_index and reads
 * the table again (decoder.rs:38-50) — so a caller may change its model between calls
 * (adaptive models).  These entry points keep a stream's state between calls instead:
 *   encode: the caller passes the (c, cum, total) triple it read for each symbol;
 *   decode: the caller passes the table to use for the next n symbols (FreqTable::find_index's
 *           binary search over cum, sample_impl.rs:27-45, and param_update over (c, cum, total),
 *           evaluated as given: no consistency requirement on the table).
 * State positions are 64-bit: a stream has no length limit.  Per-symbol arithmetic follows
 * range_coder.rs:53-135 exactly; where the reference panics or never terminates the stream is
 * flagged (sticky) and stops before that symbol. */
typedef struct rc_stream_state {
  uint64_t lower_bound, range; /* RangeCoder (range_coder.rs:7-12): Encoder::range_coder, or
                                  Decoder::range_coder() (decoder.rs:24-26)                   */
  uint64_t data;               /* decoder: Decoder::data() (decoder.rs:27-29)                */
  uint64_t pos;                /* encoder: code bytes emitted (peek_code().len(), encoder.rs:18);
                                  decoder: code bytes consumed, incl. the 8 of Decoder::new   */
  uint64_t n;                  /* symbols coded so far                                       */
  uint32_t flags;              /* sticky RC_F_* (ZERO_FREQ, BAD_MODEL, TRUNCATED, CORRUPT,
                                  FINISHED)                                                  */
  uint32_t stage;              /* 0 fresh (a decoder runs Decoder::new on its first call),
                                  1 running, 2 finished (encoder)                            */
} rc_stream_state;
/* RangeCoder::default / Encoder::new / a decoder before Decoder::new */
#define RC_STREAM_STATE_INIT {0u, ~(uint64_t)0, 0u, 0u, 0u, 0u, 0u}
/* bytes one call may emit: a symbol settles at most 12 bytes, finish 8 */
#define RC_STREAM_MAX_BYTES(n, finish) (12ull * (uint64_t)(n) + ((finish) ? 8ull : 0ull))

/* Encoder::encode x n (+ Encoder::finish if `finish`) for n_streams independent streams.
 * states_dev     n_streams rc_stream_state, updated in place
 * triples_dev    per symbol {c_freq, cum_freq, total_freq} (3 x uint32); stream k's symbols are
 *                triples [sym_off[k], sym_off[k+1])
 * out_dev        this call's NEW bytes of stream k go to out[out_off[k] ..); the slot must hold
 *                RC_STREAM_MAX_BYTES(symbols, finish) or the stream is flagged RC_F_CAPACITY
 *                (not sticky) and left unchanged
 * out_len_dev    n_streams: new bytes written
 * nbytes_dev     NULL or one uint8 per symbol (same indexing as the triples): encode()'s return
 *                value, the bytes that symbol settled (encoder.rs:34-36)
 * flags_dev      n_streams: RC_F_* of this call (the sticky ones are also in the state)      */
rc_status rc_stream_encode(rc_ctx* ctx, rc_stream_state* states_dev, const uint32_t* triples_dev,
                           const uint64_t* sym_off_dev, uint32_t n_streams, uint8_t* out_dev,
                           const uint64_t* out_off_dev, uint64_t* out_len_dev,
                           uint8_t* nbytes_dev, uint32_t finish, uint32_t* flags_dev);
/* Decoder::decode x (sym_off[k+1] - sym_off[k]) for n_streams streams against one table
 * (c_dev, cum_dev: n_symbols uint32 each; total_freq).  Stream k's whole code is
 * code[code_off[k] .. + code_len[k]) and the state's pos indexes it.  Symbols go to
 * syms_dev[sym_off[k] ..).  A stream stops before its first failing symbol; state.n counts the
 * symbols decoded.                                                                           */
rc_status rc_stream_decode(rc_ctx* ctx, const uint32_t* c_dev, const uint32_t* cum_dev,
                           uint32_t n_symbols, uint32_t total_freq, rc_stream_state* states_dev,
                           const uint8_t* code_dev, const uint64_t* code_off_dev,
                           const uint64_t* code_len_dev, uint8_t* syms_dev,
                           const uint64_t* sym_off_dev, uint32_t n_streams, uint32_t* flags_dev);
/* One stream in host memory, synchronous (the host mirrors' Encoder / Decoder).  Only the bytes a
 * call can touch cross PCIe: the encoder's new bytes, the decoder's window
 * [pos, pos + RC_STREAM_MAX_BYTES(n, 0) + 8).  Return RC_E_CHUNK when a flag is set (in
 * *flags_out, and sticky ones in the state).
 * Small calls (request and result within 64 KiB) go to the context's stream-service wave: one
 * workgroup of one wave, launched by the first such call on a stream of its own, holding 64.4 KiB
 * of one CU's LDS, which polls a mailbox in pinned host memory and leaves 0.25 ms after its last
 * request, 1 ms after its launch at most, or as soon as a batch entry point of the library
 * launches a kernel (the next call launches another wave).  While it runs it occupies that CU
 * slot and its hardware queue like any resident kernel: a kernel of another library on a
 * stream that shares that queue can wait up to 1 ms behind it.  A call waits for the
 * wave WITHOUT a time limit while the wave has not started (a wave waiting for a CU behind
 * long-running kernels is waited for, exactly as a launch would be); once the wave runs, a
 * call that sees no answer within 10 s returns RC_E_DEVICE and the context's service is off
 * from then on (later calls take the launch path).  RC_STREAM_SERVICE=0 (below) sends every
 * call down the launch path.                                                                 */
rc_status rc_stream_encode_host(rc_ctx* ctx, rc_stream_state* state, const uint32_t* triples,
                                uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                uint8_t* nbytes, uint32_t finish, uint32_t* flags_out);
rc_status rc_stream_decode_host(rc_ctx* ctx, const uint32_t* c, const uint32_t* cum,
                                uint32_t n_symbols, uint32_t total_freq, rc_stream_state* state,
                                const uint8_t* code, uint64_t code_len, uint8_t* syms,
                                uint64_t n, uint32_t* flags_out);

/* ---- synthetic workload generator (bench/test inputs, generated in HBM) ----
 * Fills n_chunks chunks of chunk_len symbols at syms_dev (chunk k at k*chunk_len).  Symbol i of
 * chunk k = inv_cdf[u16] where u16 = bits [16(i%4), 16(i%4)+16) of
 * mix64(seed + 0x9E3779B97F4A7C15 * ((k << 32) + i/4 + 1)) (splitmix64 finaliser).
 * inv_cdf_host: 65536 symbol bytes (an inverse CDF quantised to 2^16).                      */
rc_status rc_synth_fill(rc_ctx* ctx, uint64_t seed, const uint8_t* inv_cdf_host,
                        uint8_t* syms_dev, uint64_t chunk_len, uint32_t n_chunks);

/* ---- model construction: the step before encode ----
 * The reference builds a FreqTable by counting symbols (FreqTable::new + add_alphabet_freq per
 * symbol, examples/sample_impl.rs:49-60) and then scanning (calc_cum, :61-69).              */

/* Symbol histogram of n_chunks chunks (device pointers; stream-ordered).
 * chunk_hist_dev  NULL or n_chunks*256 uint32: row k = counts of chunk k (overwritten)
 * hist_dev        NULL or 256 uint64: batch counts ADDED into it (zero it first)          */
rc_status rc_histogram(rc_ctx* ctx, const uint8_t* syms_dev, const uint64_t* sym_off_dev,
                       uint32_t n_chunks, uint32_t* chunk_hist_dev, uint64_t* hist_dev);

/* Counts -> (c, cum, total) table (host only, no device needed).
 * target_total == 0: calc_cum's exact table, c = counts (total must stay < 2^32; with
 * RC_Q_ALL_SYMBOLS absent symbols get c = 1);
 * otherwise c_i = max(1, round(counts_i * T / sum)) for modelled symbols, the difference to T
 * folded into the largest entry (deficit; lowest index on ties) or taken from the largest
 * entries first, never below 1 (excess).  Modelled symbols: counts_i > 0, or every symbol
 * with RC_Q_ALL_SYMBOLS (so symbols absent from the sample stay encodable).
 * Returns RC_E_BAD_MODEL when no table exists (T below the number of modelled symbols, an
 * empty sample without RC_Q_ALL_SYMBOLS, a total >= 2^32).                                  */
#define RC_Q_ALL_SYMBOLS 1u
rc_status rc_quantize_counts(const uint64_t* counts_host, uint32_t n_symbols,
                             uint64_t target_total, uint32_t qflags, uint32_t* c_out_host,
                             uint32_t* cum_out_host, uint32_t* total_out_host);

/* Batched PModel::ideal_code_length (pmodel.rs:14-40): bits_dev[k] = sum over symbols s of
 * chunk k of log2(total / c[s]) = sum_i hist[k][i] * (ln total - ln c_i) / ln 2, in f64,
 * from rc_histogram's chunk rows.  A symbol with c == 0 (no code length in the reference)
 * makes its chunk's sum +inf.  Synchronous with respect to the host table.                 */
rc_status rc_ideal_bits(rc_ctx* ctx, const uint32_t* c_freq_host, uint32_t n_symbols,
                        uint32_t total_freq, const uint32_t* chunk_hist_dev, uint32_t n_chunks,
                        double* bits_dev);

/* ---- chunked container "RCB1"  ----
 * The reference's stream carries neither its symbol count (sample_impl.rs:113-120) nor its
 * model (decoder.rs:38).  The container frames a batch of chunk streams with both:
 *   offset 0          header, RC_CONTAINER_HEADER_BYTES, little-endian:
 *                       0 "RCB1"  4 u32 version 1 | header bytes << 16  8 u32 kind (0 static,
 *                       1 adaptive)  12 u32 n_symbols  16 u32 total_freq (static)
 *                       20/24/28 u32 increment/limit/period (adaptive)  32 u64 n_chunks
 *                       40 u64 symbols in all chunks  48 u64 payload bytes  56 reserved (0)
 *   table_off = 64    static: n_symbols x u32 c_freq (cum rebuilt by calc_cum), zero padded
 *                     to 16 B; adaptive: empty
 *   index_off         n_chunks x {u64 symbol count, u64 code length}
 *   payload_off       = index_off + 16 n_chunks; chunk k's code stream starts at payload_off +
 *                     sum_{j<k} pad16(code length j), zero padded to 16 B
 * A container is produced from encode_batch's slots and read back for decode_batch.        */
#define RC_CONTAINER_HEADER_BYTES 64
typedef struct rc_container_info {
  uint32_t version, kind, n_symbols, total_freq, increment, limit, period, reserved;
  uint64_t n_chunks, n_syms, payload_bytes;
  uint64_t table_off, index_off, payload_off, container_bytes;
} rc_container_info;

/* Pack encoded slots (rc_encode_batch's out/out_off/out_len, chunk sizes from sym_off) and
 * the model into a container at dst_dev.  Synchronous.  *dst_len_host receives the container
 * size; RC_E_CAPACITY (nothing written) when it exceeds dst_cap or dst_dev is NULL.        */
rc_status rc_container_pack(rc_ctx* ctx, const rc_model* m, const uint8_t* slots_dev,
                            const uint64_t* slot_off_dev, const uint64_t* code_len_dev,
                            const uint64_t* sym_off_dev, uint32_t n_chunks, uint8_t* dst_dev,
                            uint64_t dst_cap, uint64_t* dst_len_host);
/* Parse the header (head_host: the first >= RC_CONTAINER_HEADER_BYTES bytes). */
rc_status rc_container_info_parse(const uint8_t* head_host, uint64_t head_len,
                                  rc_container_info* info);
/* Decode arguments from a device-resident container: code_off/code_len (n_chunks each, into
 * the container), sym_off (n_chunks + 1).  Synchronous; RC_E_BAD_CONTAINER when the index does
 * not add up to the header's payload and symbol totals.                                    */
rc_status rc_container_offsets(rc_ctx* ctx, const uint8_t* container_dev,
                               const rc_container_info* info, uint64_t* code_off_dev,
                               uint64_t* code_len_dev, uint64_t* sym_off_dev);

#ifdef __cplusplus
}
#endif
#endif /* RANGE_CODER_AMD_H */
