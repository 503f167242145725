// A CPU stand-in for the two one-stream entry points of include/range_coder.h that the C++ host
// mirror (include/range_coder.hpp) calls, rc_stream_encode_host / rc_stream_decode_host, backed
// by the C oracle's resumable coder (oracle/rc_oracle.c), plus the context calls around them.
// It lets tests/test_mirror_host.py build and run the C++ examples (examples/*.cpp) on a machine
// without a GPU, so what they check is the mirror's own logic (staging, decode-ahead blocks,
// mid-block state, find_index overrides, error mapping).  Test infrastructure only.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/range_coder.h"
#include "../../oracle/rc_oracle.h"

static_assert(sizeof(rc_stream_state) == sizeof(orc_stream), "stream state layouts");

extern "C" {

rc_status rc_ctx_create(int, rc_ctx** out) {
  static int token;
  *out = reinterpret_cast<rc_ctx*>(&token);
  return RC_OK;
}
rc_status rc_ctx_destroy(rc_ctx*) { return RC_OK; }
const char* rc_status_string(rc_status) { return "status"; }
const char* rc_last_error(void) { return ""; }

rc_status rc_stream_encode_host(rc_ctx*, rc_stream_state* state, const uint32_t* triples,
                                uint64_t n, uint8_t* out, uint64_t out_cap, uint64_t* out_len,
                                uint8_t* nbytes, uint32_t finish, uint32_t* flags_out) {
  orc_stream st;
  memcpy(&st, state, sizeof st);
  std::vector<uint8_t> nb_tmp(nbytes ? 0 : (n ? n : 1));
  const uint32_t f = orc_stream_encode(&st, triples, n, out, out_cap, out_len,
                                       nbytes ? nbytes : nb_tmp.data(), finish ? 1 : 0);
  memcpy(state, &st, sizeof st);
  if (flags_out) *flags_out = f;
  return f ? RC_E_CHUNK : RC_OK;
}

rc_status rc_stream_decode_host(rc_ctx*, const uint32_t* c, const uint32_t* cum,
                                uint32_t n_symbols, uint32_t total_freq, rc_stream_state* state,
                                const uint8_t* code, uint64_t code_len, uint8_t* syms, uint64_t n,
                                uint32_t* flags_out) {
  orc_stream st;
  memcpy(&st, state, sizeof st);
  uint64_t done = 0;
  const uint32_t f =
      orc_stream_decode(&st, c, cum, n_symbols, total_freq, code, code_len, syms, n, &done);
  memcpy(state, &st, sizeof st);
  if (flags_out) *flags_out = f;
  return f ? RC_E_CHUNK : RC_OK;
}

rc_status rc_svc_probe_(rc_ctx*, uint64_t* out) {
  for (int i = 0; i < 5; ++i) out[i] = 0;
  return RC_OK;
}

}  // extern "C"
