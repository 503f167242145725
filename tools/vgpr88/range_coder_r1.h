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

/* Maximum chunks per batch call (grid limit) */
#define RC_MAX_CHUNKS (1u << 28)

typedef struct rc_ctx rc_ctx;     /* one device + one stream; use one per host thread */
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
/* Adaptive order-0 model (build-defined; the reference ships none):
 * per chunk, c[i] = 1 for i < n_symbols; after coding symbol s: c[s] += increment, and when the
 * total exceeds limit every c[i] = (c[i] + 1) >> 1.  Requires limit + increment < 2^31.     */
rc_status rc_model_create_adaptive(rc_ctx* ctx, uint32_t n_symbols, uint32_t increment,
                                   uint32_t limit, rc_model** out);
rc_status rc_model_destroy(rc_model* m);

/* ---- batch encode (replaces n_chunks x {Encoder::new; encode...; finish}) ----
 * syms_dev      symbol bytes (index < n_symbols), chunk k = [sym_off[k], sym_off[k+1])
 * sym_off_dev   n_chunks+1 offsets into syms_dev
 * out_dev       output arena; chunk k's stream is written at out_off[k], capacity
 *               out_off[k+1]-out_off[k] bytes (any alignment; 16-B aligned is fastest)
 * out_len_dev   n_chunks: exact stream length (== 8 + sum of encode() return values)
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
 *      returns RC_E_CHUNK when any chunk is flagged — flags are still filled in) ---- */
rc_status rc_encode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* syms,
                         const uint64_t* sym_off, uint32_t n_chunks, uint8_t* out,
                         const uint64_t* out_off, uint64_t* out_len, uint32_t* flags);
rc_status rc_decode_host(rc_ctx* ctx, const rc_model* m, const uint8_t* code,
                         const uint64_t* code_off, const uint64_t* code_len, uint8_t* syms_out,
                         const uint64_t* sym_off, uint32_t n_chunks, uint32_t* flags);

/* ---- synthetic workload generator (bench/test inputs, generated in HBM) ----
 * Fills n_chunks chunks of chunk_len symbols at syms_dev (chunk k at k*chunk_len).  Symbol i of
 * chunk k = inv_cdf[u16] where u16 = bits [16(i%4), 16(i%4)+16) of
 * mix64(seed + 0x9E3779B97F4A7C15 * ((k << 32) + i/4 + 1)) (splitmix64 finaliser).
 * inv_cdf_host: 65536 symbol bytes (an inverse CDF quantised to 2^16).                      */
rc_status rc_synth_fill(rc_ctx* ctx, uint64_t seed, const uint8_t* inv_cdf_host,
                        uint8_t* syms_dev, uint64_t chunk_len, uint32_t n_chunks);

#ifdef __cplusplus
}
#endif
#endif /* RANGE_CODER_AMD_H */
