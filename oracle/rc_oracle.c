/*
 * rc_oracle.c — CPU restatement of diegodox/range_coder_rust (TEST INFRASTRUCTURE ONLY).
 * See rc_oracle.h for the parity status.  Every function cites the reference line it follows.
 * Rust release-build integer semantics are used (u64 wrap-around), except where the reference
 * checks explicitly (overflowing_add -> Err, which is unreachable for valid tables).
 */
#include "rc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define TOP8 (1ull << 56)  /* range_coder.rs:23 */
#define TOP16 (1ull << 48) /* range_coder.rs:24 */

void orc_rc_init(orc_range_coder* rc) { /* range_coder.rs:13-20 */
    rc->lower_bound = 0;
    rc->range = UINT64_MAX;
}

/* range_coder.rs:95-100 */
static uint8_t left_shift(orc_range_coder* rc) {
    uint8_t b = (uint8_t)(rc->lower_bound >> 56);
    rc->range <<= 8;
    rc->lower_bound <<= 8;
    return b;
}

int orc_param_update(orc_range_coder* rc, uint32_t c_freq, uint32_t cum_freq, uint32_t total_freq,
                     uint8_t out[16]) {
    int n = 0;
    uint64_t r = rc->range / (uint64_t)total_freq; /* range_par_total, range_coder.rs:38-40 */
    rc->range = r * (uint64_t)c_freq;             /* range_coder.rs:65 */
    uint64_t add = r * (uint64_t)cum_freq;        /* range_coder.rs:68-81 (overflow unreachable) */
    rc->lower_bound += add;
    if (rc->range == 0) return -1; /* c_freq == 0: the loop at :83-85 never terminates */
    for (;;) {                     /* no_carry_expansion, range_coder.rs:83-85, 110-116 */
        uint64_t upper = rc->lower_bound + rc->range; /* upper_bound, :138-146 */
        if ((rc->lower_bound ^ upper) < TOP8)
            out[n++] = left_shift(rc);
        else
            break;
    }
    while (rc->range < TOP16) { /* range_reduction_expansion, range_coder.rs:87-89, 126-135 */
        rc->range = ~rc->lower_bound & (TOP16 - 1);
        out[n++] = left_shift(rc);
    }
    return n;
}

uint32_t orc_encode(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                    const uint8_t* syms, uint64_t n, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    orc_range_coder rc;
    uint8_t tmp[16];
    uint64_t len = 0;
    orc_rc_init(&rc); /* Encoder::default, encoder.rs:48-55 */
    for (uint64_t i = 0; i < n; ++i) { /* Encoder::encode, encoder.rs:24-37 */
        uint32_t s = syms[i];
        if (s >= n_alpha) { *out_len = len; return ORC_F_BAD_SYMBOL; }
        int k = orc_param_update(&rc, c[s], cum[s], total, tmp);
        if (k < 0) { *out_len = len; return ORC_F_ZERO_FREQ; }
        for (int j = 0; j < k; ++j, ++len)
            if (len < cap) out[len] = tmp[j];
    }
    for (int j = 0; j < 8; ++j, ++len) { /* Encoder::finish, encoder.rs:40-46 */
        uint8_t b = left_shift(&rc);
        if (len < cap) out[len] = b;
    }
    *out_len = len;
    return len > cap ? ORC_F_CAPACITY : 0u;
}

/* FreqTable::find_index, sample_impl.rs:27-45 */
static uint32_t find_index(const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                           const orc_range_coder* rc, uint64_t data) {
    uint64_t rfreq = (data - rc->lower_bound) / (rc->range / (uint64_t)total);
    uint32_t left = 0, right = n_alpha - 1;
    while (left < right) {
        uint32_t mid = (left + right) / 2;
        if ((uint64_t)cum[mid + 1] <= rfreq)
            left = mid + 1;
        else
            right = mid;
    }
    return left;
}

uint32_t orc_decode(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                    const uint8_t* code, uint64_t code_len, uint64_t n, uint8_t* syms_out) {
    orc_range_coder rc;
    uint8_t tmp[16];
    uint64_t data = 0, pos = 0;
    orc_rc_init(&rc);
    if (code_len < 8) return ORC_F_TRUNCATED; /* Decoder::new, decoder.rs:14-23 (pop_front panic) */
    for (; pos < 8; ++pos) data = (data << 8) | code[pos];
    for (uint64_t i = 0; i < n; ++i) { /* Decoder::decode, decoder.rs:38-54 */
        uint32_t s = find_index(cum, n_alpha, total, &rc, data);
        int k = orc_param_update(&rc, c[s], cum[s], total, tmp);
        if (k < 0) return ORC_F_CORRUPT;
        if (pos + (uint64_t)k > code_len) return ORC_F_TRUNCATED; /* shift_left_buffer, :31-35 */
        for (int j = 0; j < k; ++j) data = (data << 8) | code[pos++];
        syms_out[i] = (uint8_t)s;
    }
    return 0;
}

/* ---------------- adaptive order-0 model (build-defined) ---------------- */
typedef struct {
    uint32_t c[256], cum[257], total, n;
} adapt_model;

static void adapt_init(adapt_model* m, uint32_t n) {
    m->n = n;
    for (uint32_t i = 0; i < n; ++i) m->c[i] = 1;
    m->cum[0] = 0;
    for (uint32_t i = 0; i < n; ++i) m->cum[i + 1] = m->cum[i] + m->c[i];
    m->total = m->cum[n];
}

/* after coding symbol number i (0-based) of the chunk: c[s] += inc; then, every period-th
 * symbol, halve all counts (rounding up) if the total exceeds limit */
static void adapt_update(adapt_model* m, uint32_t s, uint32_t inc, uint32_t limit,
                         uint32_t period, uint64_t i) {
    m->c[s] += inc;
    m->total += inc;
    if ((i + 1) % period == 0 && m->total > limit)
        for (uint32_t j = 0; j < m->n; ++j) m->c[j] = (m->c[j] + 1) >> 1;
    m->cum[0] = 0;
    for (uint32_t i = 0; i < m->n; ++i) m->cum[i + 1] = m->cum[i] + m->c[i];
    m->total = m->cum[m->n];
}

uint32_t orc_encode_adaptive(uint32_t n_alpha, uint32_t inc, uint32_t limit, uint32_t period,
                             const uint8_t* syms, uint64_t n, uint8_t* out, uint64_t cap,
                             uint64_t* out_len) {
    adapt_model m;
    orc_range_coder rc;
    uint8_t tmp[16];
    uint64_t len = 0;
    adapt_init(&m, n_alpha);
    orc_rc_init(&rc);
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t s = syms[i];
        if (s >= n_alpha) { *out_len = len; return ORC_F_BAD_SYMBOL; }
        int k = orc_param_update(&rc, m.c[s], m.cum[s], m.total, tmp);
        for (int j = 0; j < k; ++j, ++len)
            if (len < cap) out[len] = tmp[j];
        adapt_update(&m, s, inc, limit, period, i);
    }
    for (int j = 0; j < 8; ++j, ++len) {
        uint8_t b = left_shift(&rc);
        if (len < cap) out[len] = b;
    }
    *out_len = len;
    return len > cap ? ORC_F_CAPACITY : 0u;
}

uint32_t orc_decode_adaptive(uint32_t n_alpha, uint32_t inc, uint32_t limit, uint32_t period,
                             const uint8_t* code, uint64_t code_len, uint64_t n, uint8_t* syms_out) {
    adapt_model m;
    orc_range_coder rc;
    uint8_t tmp[16];
    uint64_t data = 0, pos = 0;
    adapt_init(&m, n_alpha);
    orc_rc_init(&rc);
    if (code_len < 8) return ORC_F_TRUNCATED;
    for (; pos < 8; ++pos) data = (data << 8) | code[pos];
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t s = find_index(m.cum, m.n, m.total, &rc, data);
        int k = orc_param_update(&rc, m.c[s], m.cum[s], m.total, tmp);
        if (k < 0) return ORC_F_CORRUPT;
        if (pos + (uint64_t)k > code_len) return ORC_F_TRUNCATED;
        for (int j = 0; j < k; ++j) data = (data << 8) | code[pos++];
        syms_out[i] = (uint8_t)s;
        adapt_update(&m, s, inc, limit, period, i);
    }
    return 0;
}

uint64_t orc_fnv1a64(const uint8_t* p, uint64_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint64_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

/* ---------------- threaded batch drivers ---------------- */
typedef struct {
    int enc;
    const uint32_t *c, *cum;
    uint32_t n_alpha, total;
    const uint8_t* in;
    const uint64_t *in_off, *in_len; /* encode: in_off = sym_off (n+1); decode: code_off, code_len */
    uint8_t* out;
    const uint64_t* out_off; /* encode: slot offsets (n+1); decode: sym_off (n+1) */
    uint64_t* out_len;
    uint32_t* flags;
    uint32_t n_chunks;
    int tid, nthreads;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    for (uint32_t k = (uint32_t)j->tid; k < j->n_chunks; k += (uint32_t)j->nthreads) {
        if (j->enc) {
            j->flags[k] = orc_encode(j->c, j->cum, j->n_alpha, j->total, j->in + j->in_off[k],
                                     j->in_off[k + 1] - j->in_off[k], j->out + j->out_off[k],
                                     j->out_off[k + 1] - j->out_off[k], &j->out_len[k]);
        } else {
            j->flags[k] = orc_decode(j->c, j->cum, j->n_alpha, j->total, j->in + j->in_off[k],
                                     j->in_len[k], j->out_off[k + 1] - j->out_off[k],
                                     j->out + j->out_off[k]);
        }
    }
    return NULL;
}

static void run_batch(batch_job* proto, int threads) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    batch_job* jobs = (batch_job*)malloc(sizeof(batch_job) * (size_t)threads);
    for (int t = 0; t < threads; ++t) {
        jobs[t] = *proto;
        jobs[t].tid = t;
        jobs[t].nthreads = threads;
        if (threads == 1)
            batch_worker(&jobs[t]);
        else
            pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
}

void orc_encode_batch(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                      const uint8_t* syms, const uint64_t* sym_off, uint32_t n_chunks,
                      uint8_t* out, const uint64_t* out_off, uint64_t* out_len, uint32_t* flags,
                      int threads) {
    batch_job j;
    memset(&j, 0, sizeof j);
    j.enc = 1; j.c = c; j.cum = cum; j.n_alpha = n_alpha; j.total = total;
    j.in = syms; j.in_off = sym_off; j.out = out; j.out_off = out_off; j.out_len = out_len;
    j.flags = flags; j.n_chunks = n_chunks;
    run_batch(&j, threads);
}

void orc_decode_batch(const uint32_t* c, const uint32_t* cum, uint32_t n_alpha, uint32_t total,
                      const uint8_t* code, const uint64_t* code_off, const uint64_t* code_len,
                      uint8_t* syms_out, const uint64_t* sym_off, uint32_t n_chunks,
                      uint32_t* flags, int threads) {
    batch_job j;
    memset(&j, 0, sizeof j);
    j.enc = 0; j.c = c; j.cum = cum; j.n_alpha = n_alpha; j.total = total;
    j.in = code; j.in_off = code_off; j.in_len = code_len; j.out = syms_out; j.out_off = sym_off;
    j.flags = flags; j.n_chunks = n_chunks;
    run_batch(&j, threads);
}

/* ---------------- resumable single streams (rc_stream_* restated) ---------------- */
void orc_stream_init(orc_stream* st) {
    memset(st, 0, sizeof *st);
    st->range = UINT64_MAX; /* RangeCoder::default, range_coder.rs:13-20 */
}

/* RangeCoder::param_update (range_coder.rs:53-92) with the reference's panics as flags:
 * returns the settled byte count, or -(flag) */
static int param_update_checked(orc_range_coder* rc, uint32_t c_freq, uint32_t cum_freq,
                                uint32_t total_freq, uint8_t out[16], uint32_t zero_flag) {
    if (total_freq == 0) return -(int)ORC_F_BAD_MODEL;   /* u64 / 0 panics (:38-40) */
    uint64_t r = rc->range / (uint64_t)total_freq;
    uint64_t range = r * (uint64_t)c_freq;                /* :65 (release: wraps) */
    uint64_t add = r * (uint64_t)cum_freq;
    if (rc->lower_bound + add < add) return -(int)ORC_F_BAD_MODEL; /* overflowing_add, :68-81 */
    uint64_t low = rc->lower_bound + add;
    if (range == 0) return -(int)zero_flag;               /* :83-85 never terminates */
    if (low + range < range) return -(int)ORC_F_BAD_MODEL; /* upper_bound().unwrap(), :138-146 */
    rc->range = range;
    rc->lower_bound = low;
    int n = 0;
    for (;;) { /* no_carry_expansion, :110-116 (upper_bound cannot overflow from here on) */
        if ((rc->lower_bound ^ (rc->lower_bound + rc->range)) < TOP8)
            out[n++] = left_shift(rc);
        else
            break;
    }
    while (rc->range < TOP16) { /* range_reduction_expansion, :126-135 */
        rc->range = ~rc->lower_bound & (TOP16 - 1);
        out[n++] = left_shift(rc);
    }
    return n;
}

uint32_t orc_stream_encode(orc_stream* st, const uint32_t* triples, uint64_t n, uint8_t* out,
                           uint64_t cap, uint64_t* out_len, uint8_t* nbytes, int finish) {
    uint64_t len = 0;
    *out_len = 0;
    if (st->flags) return st->flags;
    if (st->stage == 2) return st->flags = ORC_F_FINISHED; /* finish() consumed the encoder */
    if (cap < 12 * n + (finish ? 8 : 0)) return ORC_F_CAPACITY; /* not sticky, no change */
    orc_range_coder rc = {st->lower_bound, st->range};
    uint8_t tmp[16];
    for (uint64_t i = 0; i < n; ++i) { /* Encoder::encode, encoder.rs:24-37 */
        const uint32_t* t = triples + 3 * i;
        orc_range_coder save = rc;
        int k = param_update_checked(&rc, t[0], t[1], t[2], tmp, ORC_F_ZERO_FREQ);
        if (k < 0) {
            rc = save;
            st->flags = (uint32_t)(-k);
            break;
        }
        for (int j = 0; j < k; ++j) out[len++] = tmp[j];
        if (nbytes) nbytes[i] = (uint8_t)k;
        st->n++;
    }
    if (finish && !st->flags) { /* Encoder::finish, encoder.rs:40-46 */
        for (int j = 0; j < 8; ++j) out[len++] = left_shift(&rc);
        st->stage = 2;
    } else if (st->stage == 0) {
        st->stage = 1;
    }
    st->lower_bound = rc.lower_bound;
    st->range = rc.range;
    st->pos += len;
    *out_len = len;
    return st->flags;
}

uint32_t orc_stream_decode(orc_stream* st, const uint32_t* c, const uint32_t* cum,
                           uint32_t n_alpha, uint32_t total, const uint8_t* code,
                           uint64_t code_len, uint8_t* syms, uint64_t n, uint64_t* n_done) {
    *n_done = 0;
    if (st->flags) return st->flags;
    if (st->stage == 0) { /* Decoder::new, decoder.rs:14-23 */
        if (code_len < 8) return st->flags = ORC_F_TRUNCATED;
        st->data = 0;
        for (st->pos = 0; st->pos < 8; ++st->pos) st->data = (st->data << 8) | code[st->pos];
        st->stage = 1;
    }
    orc_range_coder rc = {st->lower_bound, st->range};
    uint8_t tmp[16];
    for (uint64_t i = 0; i < n; ++i) { /* Decoder::decode, decoder.rs:38-54 */
        if (total == 0) { st->flags = ORC_F_BAD_MODEL; break; } /* find_index's division */
        uint32_t s = find_index(cum, n_alpha, total, &rc, st->data);
        orc_range_coder save = rc;
        int k = param_update_checked(&rc, c[s], cum[s], total, tmp, ORC_F_CORRUPT);
        if (k < 0) {
            rc = save;
            st->flags = (uint32_t)(-k);
            break;
        }
        if (st->pos + (uint64_t)k > code_len) { /* shift_left_buffer panics, :31-35 */
            rc = save;
            st->flags = ORC_F_TRUNCATED;
            break;
        }
        for (int j = 0; j < k; ++j) st->data = (st->data << 8) | code[st->pos++];
        syms[i] = (uint8_t)s;
        st->n++;
        *n_done = i + 1;
    }
    st->lower_bound = rc.lower_bound;
    st->range = rc.range;
    return st->flags;
}
