/*
 * b64_stages.c -- the base64 encoder and decoder bytestream_1 stages
 * (include/base64encoder.h, include/base64decoder.h), computed on the GPU
 * through the b64x C ABI (include/b64x.h).
 *
 * Reference: src/base64encoder.c and src/base64decoder.c.  The reference
 * transforms in place inside the caller's buffer, one byte per loop trip
 * (encoder :101-142, decoder :52-80).  Here each stage pulls a large block
 * from its upstream into pinned staging, runs one GPU round trip
 * (b64x_session_*), and serves reads from the staged result:
 *
 *  - encoder: whole 3-byte groups are encoded; the 0-2 leftover bytes are
 *    carried to the next pull, and encoded with the final padding once
 *    upstream reports EOF (the reference's finalize(), :61-99);
 *  - decoder: whole 4-character groups are decoded (B64X_DEC_HOLD_TAIL);
 *    the 0-3 leftover sextets are carried (re-spelled as alphabet
 *    characters) to the next pull, and flushed at EOF with the
 *    reference's truncation rule (floor(6V/8) bytes overall).
 *
 * The character/byte stream each stage produces is the reference's, byte
 * for byte.  Per-call return counts may differ (a stage returns what it
 * has staged; it never returns 0 before EOF), errno from upstream (EAGAIN
 * included) is passed through with all state kept, and count == 0
 * returns 0 (ref :103-104, :54-55).  The reference's assert at
 * src/base64encoder.c:140 (read counts not divisible by 4) has no
 * counterpart: any count works.
 *
 * Tuning (environment, read when a stage is created):
 *   ASYNC_B64_STAGE_CAPACITY  staging bytes per stage (default 1 MiB)
 *   ASYNC_B64_MIN_PULL        smallest upstream request (default 64 KiB)
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "b64x.h"
#include "base64decoder.h"
#include "base64encoder.h"

enum stage_state { STAGE_OPEN, STAGE_DONE, STAGE_FAILED };

typedef struct {
    b64x_session *sess;
    int err;            /* errno to report when sess is NULL / failed */
    size_t min_pull;
    const uint8_t *out; /* staged output, inside the session's host_out */
    size_t out_pos, out_len;
    enum stage_state state;
} stage_common;

static size_t env_size(const char *name, size_t dflt, size_t lo)
{
    const char *v = getenv(name);
    if (!v || !*v)
        return dflt;
    char *end = NULL;
    unsigned long long x = strtoull(v, &end, 0);
    if (!end || *end || x < lo)
        return dflt;
    return (size_t) x;
}

static void stage_init(stage_common *c)
{
    size_t cap = env_size("ASYNC_B64_STAGE_CAPACITY", (size_t) 1 << 20, 64);
    c->min_pull = env_size("ASYNC_B64_MIN_PULL", (size_t) 64 << 10, 1);
    c->sess = b64x_session_open(cap);
    c->err = c->sess ? 0 : (errno ? errno : ENODEV);
    c->state = c->sess ? STAGE_OPEN : STAGE_FAILED;
}

static ssize_t stage_fail(stage_common *c, int negerr)
{
    c->state = STAGE_FAILED;
    c->err = negerr < 0 ? -negerr : EIO;
    errno = c->err;
    return -1;
}

/* Serve from the staged result; -2 when nothing is staged. */
static ssize_t stage_serve(stage_common *c, void *buf, size_t count)
{
    size_t avail = c->out_len - c->out_pos;
    if (!avail)
        return -2;
    size_t n = avail < count ? avail : count;
    memcpy(buf, c->out + c->out_pos, n);
    c->out_pos += n;
    return (ssize_t) n;
}

static size_t pull_size(const stage_common *c, size_t want, size_t held)
{
    size_t cap = b64x_session_capacity(c->sess) - held;
    if (want < c->min_pull)
        want = c->min_pull;
    return want < cap ? want : cap;
}

/* ================================================================ encoder */

struct base64encoder {
    async_t *async;
    bytestream_1 stream;
    b64x_alphabet abc;
    stage_common c;
    uint8_t carry[2];
    size_t ncarry;
};

base64encoder_t *base64_encode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63, bool pad, char padchar)
{
    base64encoder_t *e = calloc(1, sizeof *e);
    if (!e)
        abort();
    e->async = async;
    e->stream = stream;
    e->abc.pos62 = pos62;
    e->abc.pos63 = pos63;
    e->abc.padchar = padchar;
    e->abc.pad = pad;
    stage_init(&e->c);
    return e;
}

ssize_t base64encoder_read(base64encoder_t *e, void *buf, size_t count)
{
    if (!count)
        return 0;
    for (;;) {
        ssize_t n = stage_serve(&e->c, buf, count);
        if (n != -2)
            return n;
        if (e->c.state == STAGE_DONE)
            return 0;
        if (e->c.state == STAGE_FAILED) {
            errno = e->c.err;
            return -1;
        }
        uint8_t *in = b64x_session_host_in(e->c.sess);
        memcpy(in, e->carry, e->ncarry);
        /* The reference asks upstream for ceil(6*count/8)-ish bytes
         * (src/base64encoder.c:124); ask for at least min_pull. */
        size_t want = pull_size(&e->c, (count * 6 + 7) / 8, e->ncarry);
        ssize_t got = bytestream_1_read(e->stream, in + e->ncarry, want);
        if (got < 0)
            return -1; /* errno from upstream; carry kept */
        size_t total = e->ncarry + (size_t) got;
        uint64_t m = 0;
        int rc;
        if (got == 0) {
            e->c.state = STAGE_DONE;
            e->ncarry = 0;
            if (total == 0)
                return 0;
            rc = b64x_session_encode(e->c.sess, total, &e->abc, &m);
            if (rc)
                return stage_fail(&e->c, rc);
        } else {
            size_t whole = total - total % 3;
            size_t rest = total - whole;
            uint8_t keep[2];
            memcpy(keep, in + whole, rest);
            if (whole) {
                rc = b64x_session_encode(e->c.sess, whole, &e->abc, &m);
                if (rc)
                    return stage_fail(&e->c, rc);
            }
            memcpy(e->carry, keep, rest);
            e->ncarry = rest;
        }
        e->c.out = b64x_session_host_out(e->c.sess);
        e->c.out_pos = 0;
        e->c.out_len = (size_t) m;
    }
}

void base64encoder_close(base64encoder_t *e)
{
    bytestream_1_close(e->stream);
    b64x_session_close(e->c.sess);
    e->c.sess = NULL;
    async_wound(e->async, e);
    e->async = NULL;
}

void base64encoder_register_callback(base64encoder_t *e, action_1 action)
{
    bytestream_1_register_callback(e->stream, action);
}

void base64encoder_unregister_callback(base64encoder_t *e)
{
    bytestream_1_unregister_callback(e->stream);
}

static ssize_t enc_read_vt(void *o, void *buf, size_t count)
{
    return base64encoder_read(o, buf, count);
}
static void enc_close_vt(void *o)
{
    base64encoder_close(o);
}
static void enc_reg_vt(void *o, action_1 a)
{
    base64encoder_register_callback(o, a);
}
static void enc_unreg_vt(void *o)
{
    base64encoder_unregister_callback(o);
}

static const struct bytestream_1_vt encoder_vt = {
    enc_read_vt, enc_close_vt, enc_reg_vt, enc_unreg_vt
};

bytestream_1 base64encoder_as_bytestream_1(base64encoder_t *e)
{
    return (bytestream_1) { e, &encoder_vt };
}

/* ================================================================ decoder */

struct base64decoder {
    async_t *async;
    bytestream_1 stream;
    b64x_alphabet abc;
    stage_common c;
    uint8_t carry[4]; /* alphabet characters of the incomplete group */
    size_t ncarry;
};

base64decoder_t *base64_decode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63)
{
    base64decoder_t *d = calloc(1, sizeof *d);
    if (!d)
        abort();
    d->async = async;
    d->stream = stream;
    d->abc.pos62 = pos62;
    d->abc.pos63 = pos63;
    d->abc.padchar = (char) -1;
    d->abc.pad = false;
    stage_init(&d->c);
    return d;
}

/* A character that decodes to sextet v under this alphabet.  Only values
 * the device actually produced are asked for, so 62/63 always have a
 * matching pos62/pos63 (ref map(), src/base64decoder.c:38-48). */
static uint8_t spell_sextet(const b64x_alphabet *abc, unsigned v)
{
    if (v < 26)
        return (uint8_t) ('A' + v);
    if (v < 52)
        return (uint8_t) ('a' + v - 26);
    if (v < 62)
        return (uint8_t) ('0' + v - 52);
    char p = v == 62 ? abc->pos62 : abc->pos63;
    if (p == (char) -1)
        p = v == 62 ? '+' : '/';
    return (uint8_t) p;
}

ssize_t base64decoder_read(base64decoder_t *d, void *buf, size_t count)
{
    if (!count)
        return 0;
    for (;;) {
        ssize_t n = stage_serve(&d->c, buf, count);
        if (n != -2)
            return n;
        if (d->c.state == STAGE_DONE)
            return 0;
        if (d->c.state == STAGE_FAILED) {
            errno = d->c.err;
            return -1;
        }
        uint8_t *in = b64x_session_host_in(d->c.sess);
        memcpy(in, d->carry, d->ncarry);
        size_t want = pull_size(&d->c, count, d->ncarry);
        ssize_t got = bytestream_1_read(d->stream, in + d->ncarry, want);
        if (got < 0)
            return -1; /* errno from upstream; carry kept */
        size_t total = d->ncarry + (size_t) got;
        b64x_dec_result res;
        memset(&res, 0, sizeof res);
        int rc;
        if (got == 0) {
            d->c.state = STAGE_DONE;
            d->ncarry = 0;
            if (total == 0)
                return 0;
            rc = b64x_session_decode(d->c.sess, total, &d->abc, 0, &res);
            if (rc)
                return stage_fail(&d->c, rc);
        } else {
            rc = b64x_session_decode(d->c.sess, total, &d->abc,
                                     B64X_DEC_HOLD_TAIL, &res);
            if (rc)
                return stage_fail(&d->c, rc);
            d->ncarry = res.tail_n;
            for (unsigned i = 0; i < res.tail_n; i++)
                d->carry[i] = spell_sextet(&d->abc, res.tail[i]);
        }
        d->c.out = b64x_session_host_out(d->c.sess);
        d->c.out_pos = 0;
        d->c.out_len = (size_t) res.out_len;
    }
}

void base64decoder_close(base64decoder_t *d)
{
    bytestream_1_close(d->stream);
    b64x_session_close(d->c.sess);
    d->c.sess = NULL;
    async_wound(d->async, d);
    d->async = NULL;
}

void base64decoder_register_callback(base64decoder_t *d, action_1 action)
{
    bytestream_1_register_callback(d->stream, action);
}

void base64decoder_unregister_callback(base64decoder_t *d)
{
    bytestream_1_unregister_callback(d->stream);
}

static ssize_t dec_read_vt(void *o, void *buf, size_t count)
{
    return base64decoder_read(o, buf, count);
}
static void dec_close_vt(void *o)
{
    base64decoder_close(o);
}
static void dec_reg_vt(void *o, action_1 a)
{
    base64decoder_register_callback(o, a);
}
static void dec_unreg_vt(void *o)
{
    base64decoder_unregister_callback(o);
}

static const struct bytestream_1_vt decoder_vt = {
    dec_read_vt, dec_close_vt, dec_reg_vt, dec_unreg_vt
};

bytestream_1 base64decoder_as_bytestream_1(base64decoder_t *d)
{
    return (bytestream_1) { d, &decoder_vt };
}
