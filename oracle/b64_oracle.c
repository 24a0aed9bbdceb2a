/*
 * b64_oracle.c -- TEST INFRASTRUCTURE ONLY (see b64_oracle.h).
 *
 * A line-by-line *behavioural* restatement of the reference's two stages,
 * kept deliberately scalar (one byte per loop trip, like the reference)
 * so that its speed is also the honest CPU baseline:
 *
 *   enc_map()       <- src/base64encoder.c:26-27, 49-59
 *   enc_finalize()  <- src/base64encoder.c:61-99
 *   enc_read()      <- src/base64encoder.c:101-142 (do_read)
 *   dec_map()       <- src/base64decoder.c:38-48, with fsdyn's
 *                      base64_bitfield_decoding[] restated as a table
 *                      "A-Z a-z 0-9 -> 0..61, everything else -1"
 *                      (the table is an un-vendored dependency; see
 *                      oracle/README.md for what pins it)
 *   dec_read()      <- src/base64decoder.c:52-80 (decoder_read)
 *   nice_read()     <- src/nicestream.c:34-51
 *   queue_read()    <- src/queuestream.c:150-191 over blobstream elements
 *                      (src/blobstream.c:30-41), queue terminated
 *   chunk_read()    <- src/chunkencoder.c:31-77 (framing), :167-191
 *                      (max_chunk_size clamp)
 *   the reftest     <- test/asynctest-base64encoder.c:11-151
 *
 * Differences from the reference are limited to plumbing: no event loop
 * (EAGAIN is retried immediately, which is what the loop callback does),
 * no tracing, and the encoder's out-of-bounds write at :140 is detected
 * and reported instead of corrupting memory/aborting.
 */
#include "b64_oracle.h"

#include <errno.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ streams -- */

typedef struct ostream ostream;
struct ostream {
    ssize_t (*read)(ostream *s, void *buf, size_t count);
};

typedef struct {
    ostream base;
    const uint8_t *data;
    size_t size, pos, chunk;
} mem_source;

static ssize_t mem_read(ostream *s, void *buf, size_t count)
{
    mem_source *m = (mem_source *) s;
    size_t n = m->size - m->pos;
    if (n > count)
        n = count;
    if (m->chunk && n > m->chunk)
        n = m->chunk;
    memcpy(buf, m->data + m->pos, n);
    m->pos += n;
    return (ssize_t) n;
}

typedef struct {
    ostream base;
    size_t size, cursor;
} counting_source; /* test/asynctest-base64encoder.c:25-35 */

static ssize_t counting_read(ostream *s, void *buf, size_t count)
{
    counting_source *c = (counting_source *) s;
    size_t remaining = c->size - c->cursor;
    if (remaining < count)
        count = remaining;
    uint8_t *p = buf;
    for (size_t i = 0; i < count; i++)
        *p++ = (uint8_t) c->cursor++;
    return (ssize_t) count;
}

typedef struct {
    ostream base;
    ostream *up;
    size_t this_burst, max_burst;
} nice_stream; /* src/nicestream.c:34-51 */

static ssize_t nice_read(ostream *s, void *buf, size_t count)
{
    nice_stream *n = (nice_stream *) s;
    if (n->this_burst > n->max_burst) {
        n->this_burst = 0;
        errno = EAGAIN;
        return -1;
    }
    ssize_t got = n->up->read(n->up, buf, count);
    if (got < 0)
        n->this_burst = 0;
    else
        n->this_burst += (size_t) got;
    return got;
}

static void nice_init(nice_stream *n, ostream *up, size_t burst)
{
    n->base.read = nice_read;
    n->up = up;
    n->this_burst = 0;
    n->max_burst = burst;
}

/* ------------------------------------------------------------ encoder -- */

enum { ENC_PAD = -1, ENC_PAD2 = -2, ENC_EOF = -3 };

static const char ALNUM62[] =
    "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

typedef struct {
    ostream base;
    ostream *up;
    char pos62, pos63, padchar;
    bool pad;
    long bit_count; /* 0, 2, 4, or ENC_PAD / ENC_PAD2 / ENC_EOF */
    unsigned bits;
    size_t overflow_reads;
} enc_stream;

static char enc_map(const enc_stream *e, unsigned v)
{
    if (v == 62)
        return e->pos62;
    if (v == 63)
        return e->pos63;
    return ALNUM62[v];
}

static ssize_t enc_finalize(enc_stream *e, size_t count, char *q)
{
    if (e->bit_count == 2) {
        *q++ = enc_map(e, (e->bits << 4) & 0x3f);
        if (!e->pad) {
            e->bit_count = ENC_EOF;
            return 1;
        }
        if (count > 1) {
            *q++ = e->padchar;
            if (count > 2) {
                *q = e->padchar;
                e->bit_count = ENC_EOF;
                return 3;
            }
            e->bit_count = ENC_PAD;
            return 2;
        }
        e->bit_count = ENC_PAD2;
        return 1;
    }
    if (e->bit_count == 4) {
        *q++ = enc_map(e, (e->bits << 2) & 0x3f);
        if (!e->pad) {
            e->bit_count = ENC_EOF;
            return 1;
        }
        if (count > 1) {
            *q = e->padchar;
            e->bit_count = ENC_EOF;
            return 2;
        }
        e->bit_count = ENC_PAD;
        return 1;
    }
    e->bit_count = ENC_EOF;
    return 0;
}

/* `buf` must have room for count + 2 bytes: the reference can write up to
 * two characters past `count` when its assert would fire; that is detected
 * here rather than reproduced. */
static ssize_t enc_read(ostream *s, void *buf, size_t count)
{
    enc_stream *e = (enc_stream *) s;
    if (!count)
        return 0;
    char *q = buf;
    switch (e->bit_count) {
    case ENC_PAD2:
        *q++ = e->padchar;
        if (count > 1) {
            *q = e->padchar;
            e->bit_count = ENC_EOF;
            return 2;
        }
        e->bit_count = ENC_PAD;
        return 1;
    case ENC_PAD:
        *q = e->padchar;
        e->bit_count = ENC_EOF;
        return 1;
    case ENC_EOF:
        return 0;
    default:
        break;
    }
    size_t need = (count * 6 + 7 - (size_t) e->bit_count) / 8;
    uint8_t *p = (uint8_t *) buf + count - need;
    ssize_t n = e->up->read(e->up, p, need);
    if (n < 0)
        return -1;
    if (n == 0)
        return enc_finalize(e, count, q);
    while (n--) {
        e->bits = e->bits << 8 | *p++;
        e->bit_count += 8;
        while (e->bit_count >= 6) {
            e->bit_count -= 6;
            *q++ = enc_map(e, (e->bits >> e->bit_count) & 0x3f);
        }
    }
    if ((size_t) (q - (char *) buf) > count)
        e->overflow_reads++;
    return q - (char *) buf;
}

static void enc_init(enc_stream *e, ostream *up, char pos62, char pos63,
                     bool pad, char padchar)
{
    e->base.read = enc_read;
    e->up = up;
    e->pos62 = pos62 == (char) -1 ? '+' : pos62;
    e->pos63 = pos63 == (char) -1 ? '/' : pos63;
    e->pad = pad;
    e->padchar = padchar == (char) -1 ? '=' : padchar;
    e->bit_count = 0;
    e->bits = 0;
    e->overflow_reads = 0;
}

/* ------------------------------------------------------------ decoder -- */

/* fsdyn's base64_bitfield_decoding[256] (included by the reference at
 * src/base64decoder.c:5, looked up at :40), restated: A-Z a-z 0-9 -> 0..61,
 * every other byte -1.  A table, as in the reference, so that the per-char
 * cost -- one load, a predictable compare -- and hence the CPU baseline's
 * speed are the reference's (0.23-0.28 GiB/s per core). */
static const int8_t bitfield_decoding[256] = {
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    52, 53, 54, 55, 56, 57, 58, 59, 60, 61, -1, -1, -1, -1, -1, -1,
    -1,  0,  1,  2,  3,  4,  5,  6,  7,  8,  9, 10, 11, 12, 13, 14,
    15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, -1, -1, -1, -1, -1,
    -1, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40,
    41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
};

typedef struct {
    ostream base;
    ostream *up;
    char pos62, pos63;
    size_t bit_count; /* (size_t) -1 after EOF */
    unsigned bits;
} dec_stream;

static int8_t dec_map(const dec_stream *d, uint8_t c)
{
    int8_t v = bitfield_decoding[c];
    if (v != -1)
        return v;
    /* uint8_t compared with (signed, on x86-64) char: a pos62/pos63 of
     * 0x80 or above never matches, exactly like the reference. */
    if (c == d->pos62)
        return 62;
    if (c == d->pos63)
        return 63;
    return -1;
}

static ssize_t dec_read(ostream *s, void *buf, size_t count)
{
    dec_stream *d = (dec_stream *) s;
    if (!count || d->bit_count == (size_t) -1)
        return 0;
    uint8_t *q = buf;
    do {
        ssize_t n = d->up->read(d->up, buf, count);
        if (n < 0)
            return -1;
        if (n == 0) {
            d->bit_count = (size_t) -1;
            break;
        }
        uint8_t *p = buf;
        while (n--) {
            int v = dec_map(d, *p++);
            if (v < 0)
                continue;
            d->bits = d->bits << 6 | (unsigned) v;
            d->bit_count += 6;
            if (d->bit_count >= 8) {
                d->bit_count -= 8;
                *q++ = (uint8_t) (d->bits >> d->bit_count);
            }
        }
    } while (q == (uint8_t *) buf);
    return q - (uint8_t *) buf;
}

static void dec_init(dec_stream *d, ostream *up, char pos62, char pos63)
{
    d->base.read = dec_read;
    d->up = up;
    d->pos62 = pos62 == (char) -1 ? '+' : pos62;
    d->pos63 = pos63 == (char) -1 ? '/' : pos63;
    d->bit_count = 0;
    d->bits = 0;
}

/* ------------------------------------------------------------ drivers -- */

/* Drain `s` with reads of `read_size` into a scratch buffer of
 * read_size + 2 bytes (the +2 only catches the encoder's overrun),
 * retrying on EAGAIN like the reference test's verify_read does. */
static ssize_t drain(ostream *s, size_t read_size, uint8_t *out, size_t cap)
{
    uint8_t *scratch = malloc(read_size + 2);
    if (!scratch)
        return -1;
    size_t total = 0;
    for (;;) {
        /* straight into the destination while there is room for a whole
         * read (and the 2 bytes an overrunning read may write), like the
         * harness's consumer of the GPU stages */
        const bool direct = cap - total >= read_size + 2;
        uint8_t *dst = direct ? out + total : scratch;
        ssize_t n = s->read(s, dst, read_size);
        if (n < 0) {
            if (errno == EAGAIN)
                continue;
            free(scratch);
            return -1;
        }
        if (n == 0)
            break;
        size_t take = (size_t) n > read_size ? read_size : (size_t) n;
        if (total + take > cap) {
            free(scratch);
            errno = ENOSPC;
            return -1;
        }
        if (!direct)
            memcpy(out + total, scratch, take);
        total += take;
    }
    free(scratch);
    return (ssize_t) total;
}

void orc_decode_table(char pos62, char pos63, int8_t out[256])
{
    dec_stream d;
    dec_init(&d, NULL, pos62, pos63);
    for (int c = 0; c < 256; c++)
        out[c] = (int8_t) dec_map(&d, (uint8_t) c);
}

static ostream *source_chain(mem_source *src, nice_stream *nice,
                             const uint8_t *in, size_t n, size_t src_chunk,
                             size_t burst)
{
    src->base.read = mem_read;
    src->data = in;
    src->size = n;
    src->pos = 0;
    src->chunk = src_chunk;
    if (!burst)
        return &src->base;
    nice_init(nice, &src->base, burst);
    return &nice->base;
}

ssize_t orc_encode_stream(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, int pad, char padchar, uint8_t *out,
                          size_t out_cap, size_t *overflow_reads)
{
    mem_source src;
    nice_stream nice;
    enc_stream enc;
    ostream *up = source_chain(&src, &nice, in, n, src_chunk, burst);
    enc_init(&enc, up, pos62, pos63, pad != 0, padchar);
    ssize_t r = drain(&enc.base, read_size, out, out_cap);
    if (overflow_reads)
        *overflow_reads = enc.overflow_reads;
    return enc.overflow_reads ? -1 : r;
}

ssize_t orc_decode_stream(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, uint8_t *out, size_t out_cap)
{
    mem_source src;
    nice_stream nice;
    dec_stream dec;
    ostream *up = source_chain(&src, &nice, in, n, src_chunk, burst);
    dec_init(&dec, up, pos62, pos63);
    return drain(&dec.base, read_size, out, out_cap);
}

size_t orc_encode(const uint8_t *in, size_t n, char pos62, char pos63, int pad,
                  char padchar, uint8_t *out)
{
    size_t cap = (n + 2) / 3 * 4;
    size_t rs = 1 << 20; /* a multiple of 4: outside the assert domain */
    ssize_t r = orc_encode_stream(in, n, 0, 0, rs, pos62, pos63, pad, padchar,
                                  out, cap, NULL);
    return r < 0 ? 0 : (size_t) r;
}

size_t orc_decode(const uint8_t *in, size_t n, char pos62, char pos63,
                  uint8_t *out)
{
    size_t cap = (n + 3) / 4 * 3;
    /* decoder_read reads up to `count` characters into the caller's
     * buffer, so the drain buffer must hold a whole read of input. */
    ssize_t r = orc_decode_stream(in, n, 0, 0, 1 << 20, pos62, pos63, out,
                                  cap ? cap : 1);
    return r < 0 ? 0 : (size_t) r;
}

/* A pass-through that copies the bytes it forwards (tap between the
 * encoder and nice(91) in the reference topology). */
typedef struct {
    ostream base;
    ostream *up;
    uint8_t *copy;
    size_t cap, len;
    bool overflow;
} tee_stream;

static ssize_t tee_read(ostream *s, void *buf, size_t count)
{
    tee_stream *t = (tee_stream *) s;
    ssize_t n = t->up->read(t->up, buf, count);
    if (n > 0) {
        if (t->len + (size_t) n <= t->cap)
            memcpy(t->copy + t->len, buf, (size_t) n);
        else
            t->overflow = true;
        t->len += (size_t) n;
    }
    return n;
}

ssize_t orc_reftest(size_t length, uint8_t *enc_out, size_t enc_cap,
                    size_t *enc_len, uint8_t *dec_out, size_t dec_cap)
{
    counting_source src = { { counting_read }, length, 0 };
    nice_stream nice1, nice2, nice3;
    enc_stream enc;
    dec_stream dec;
    tee_stream tee;
    nice_init(&nice1, &src.base, 113);
    enc_init(&enc, &nice1.base, '.', '_', true, '-');
    tee.base.read = tee_read;
    tee.up = &enc.base;
    tee.copy = enc_out;
    tee.cap = enc_cap;
    tee.len = 0;
    tee.overflow = false;
    nice_init(&nice2, &tee.base, 91);
    dec_init(&dec, &nice2.base, '.', '_');
    nice_init(&nice3, &dec.base, 97);
    ssize_t r = drain(&nice3.base, 200, dec_out, dec_cap);
    if (enc_len)
        *enc_len = tee.len;
    if (tee.overflow || enc.overflow_reads)
        return -1;
    return r;
}

/* ------------------------------------------------- config-5 egress stack -- */

typedef struct {
    ostream base;
    const uint8_t *data;
    const size_t *lens;
    size_t npieces, piece, off, base_off;
} queue_source;

/* queuestream do_read with every element a blobstream and the queue
 * terminated: fill `count` across elements, dropping each at its EOF. */
static ssize_t queue_read(ostream *s, void *buf, size_t count)
{
    queue_source *q = (queue_source *) s;
    uint8_t *dst = buf;
    size_t got = 0;
    while (got < count && q->piece < q->npieces) {
        size_t left = q->lens[q->piece] - q->off;
        if (!left) { /* blobstream EOF: close and unlink the element */
            q->base_off += q->lens[q->piece];
            q->piece++;
            q->off = 0;
            continue;
        }
        size_t n = left < count - got ? left : count - got;
        memcpy(dst + got, q->data + q->base_off + q->off, n);
        q->off += n;
        got += n;
    }
    return (ssize_t) got; /* 0 = terminated and empty */
}

enum { ORC_CHUNK_HEAD = 11, ORC_CHUNK_MAX = 16 * 1024 * 1024 };

typedef struct {
    ostream base;
    ostream *up;
    size_t max_chunk;
    int termination;
    uint8_t *buf;
    size_t next, eoc, chunk_count;
    bool eof_pending;
} chunk_stream;

static ssize_t chunk_read(ostream *s, void *buf, size_t count)
{
    chunk_stream *c = (chunk_stream *) s;
    if (!count)
        return 0;
    if (c->next >= c->eoc) {
        if (c->eof_pending)
            return 0;
        ssize_t n = c->up->read(c->up, c->buf + ORC_CHUNK_HEAD, c->max_chunk);
        if (n < 0)
            return n;
        if (n == 0) {
            c->eof_pending = true;
            c->eoc = ORC_CHUNK_HEAD;
            if (c->termination == 0) {
                c->buf[c->eoc++] = '\r';
                c->buf[c->eoc++] = '\n';
            } else if (c->termination == 2) {
                c->eoc -= 2;
            }
        } else {
            c->eoc = ORC_CHUNK_HEAD + (size_t) n;
        }
        c->next = ORC_CHUNK_HEAD - 2;
        size_t v = (size_t) n;
        do {
            c->buf[--c->next] = (uint8_t) "0123456789abcdef"[v % 16];
            v /= 16;
        } while (v);
        if (c->chunk_count++ > 0) {
            c->buf[--c->next] = '\n';
            c->buf[--c->next] = '\r';
        }
    }
    size_t n = c->eoc - c->next;
    if (n > count)
        n = count;
    memcpy(buf, c->buf + c->next, n);
    c->next += n;
    return (ssize_t) n;
}

ssize_t orc_chunked_encode(const uint8_t *in, const size_t *piece_len,
                           size_t npieces, size_t max_chunk, int termination,
                           size_t read_size, char pos62, char pos63, int pad,
                           char padchar, uint8_t *out, size_t out_cap)
{
    queue_source q = { { queue_read }, in, piece_len, npieces, 0, 0, 0 };
    enc_stream enc;
    enc_init(&enc, &q.base, pos62, pos63, pad != 0, padchar);
    chunk_stream c;
    memset(&c, 0, sizeof c);
    c.base.read = chunk_read;
    c.up = &enc.base;
    c.max_chunk = max_chunk < 2 ? 2 : max_chunk > ORC_CHUNK_MAX ? ORC_CHUNK_MAX : max_chunk;
    c.termination = termination;
    /* +2: the encoder's overrun (assert :140) is caught, not corrupting */
    c.buf = malloc(ORC_CHUNK_HEAD + c.max_chunk + 2);
    if (!c.buf)
        return -1;
    c.buf[ORC_CHUNK_HEAD - 2] = '\r';
    c.buf[ORC_CHUNK_HEAD - 1] = '\n';
    ssize_t r = drain(&c.base, read_size, out, out_cap);
    free(c.buf);
    return enc.overflow_reads ? -1 : r;
}

typedef struct {
    ostream base;
    ostream *up;
    ssize_t *log;
    size_t cap, n;
} count_tap;

static ssize_t count_tap_read(ostream *s, void *buf, size_t count)
{
    count_tap *t = (count_tap *) s;
    ssize_t n = t->up->read(t->up, buf, count);
    if (n > 0) {
        if (t->n < t->cap)
            t->log[t->n] = n;
        t->n++;
    }
    return n;
}

ssize_t orc_encode_counts(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, int pad, char padchar, ssize_t *counts,
                          size_t max_counts)
{
    mem_source src;
    nice_stream nice;
    enc_stream enc;
    ostream *up = source_chain(&src, &nice, in, n, src_chunk, burst);
    enc_init(&enc, up, pos62, pos63, pad != 0, padchar);
    count_tap t = { { count_tap_read }, &enc.base, counts, max_counts, 0 };
    size_t cap = (n + 2) / 3 * 4 + 8;
    uint8_t *out = malloc(cap);
    if (!out)
        return -1;
    ssize_t r = drain(&t.base, read_size, out, cap);
    free(out);
    if (r < 0 || enc.overflow_reads)
        return -1;
    return (ssize_t) t.n;
}

/* Row batches (bench.py's all-core CPU baseline: one call per thread over
 * its slice of independent buffers, one reference stage per buffer, read
 * with one read the size of the buffer's output -- a multiple of 4, so
 * outside the reference's assert domain, base64encoder.c:124,140). */
size_t orc_encode_rows(const uint8_t *in, size_t len, size_t nbuf, uint8_t *out,
                       size_t out_stride)
{
    const size_t cap = (len + 2) / 3 * 4;
    size_t tot = 0;
    for (size_t i = 0; i < nbuf; i++) {
        ssize_t r = orc_encode_stream(in + i * len, len, 0, 0, cap ? cap : 4, (char) -1,
                                      (char) -1, 1, (char) -1, out + i * out_stride, cap, NULL);
        tot += r < 0 ? 0 : (size_t) r;
    }
    return tot;
}

size_t orc_decode_rows(const uint8_t *in, size_t len, size_t nbuf, uint8_t *out,
                       size_t out_stride)
{
    const size_t cap = (len + 3) / 4 * 3;
    size_t tot = 0;
    for (size_t i = 0; i < nbuf; i++) {
        ssize_t r = orc_decode_stream(in + i * len, len, 0, 0, len > 4 ? len : 4, (char) -1,
                                      (char) -1, out + i * out_stride, cap ? cap : 1);
        tot += r < 0 ? 0 : (size_t) r;
    }
    return tot;
}
