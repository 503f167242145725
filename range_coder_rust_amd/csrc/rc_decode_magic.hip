// rc_decode_magic.hip — k_decode_static variants for other totals (exact reciprocal multiply).
#define RC_DEC_DIV 1
#include "rc_decode.inc"
