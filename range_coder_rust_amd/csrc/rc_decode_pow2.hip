// rc_decode_pow2.hip — k_decode_static variants for power-of-two totals (range >> log2 total).
#define RC_DEC_DIV 0
#include "rc_decode.inc"
