/*
 * b64_stages.c -- the base64 encoder and decoder bytestream_1 stages
 * (include/base64encoder.h, include/base64decoder.h), computed on the GPU
 * through the b64x C ABI (include/b64x.h).
 *
 * Reference: src/base64encoder.c and src/base64decoder.c.  The reference
 * transforms in place inside the caller's buffer, one byte per loop trip
 * (encoder :101-142, decoder :52-80), synchronously inside read().  Here a
 * stage is a small pipeline of two slots, each a b64x session (pinned host
 * staging + device buffers + a HIP stream):
 *
 *   read() --> serve the oldest finished slot
 *          --> top up: pull upstream into an idle slot's pinned buffer and
 *              queue H2D + kernels + D2H on its stream (read-ahead: both
 *              slots can be in flight while the consumer drains a third
 *              block's worth of output)
 *          --> nothing finished yet: -1 / EAGAIN.
 *
 *   GPU completion: a HIP host function marks the slot finished and writes
 *   the stage's eventfd; the eventfd is registered with async_register(),
 *   so the loop calls the stage, which calls the consumer's registered
 *   callback -- the same "EAGAIN now, callback later" contract every
 *   bytestream_1 in the reference follows.
 *
 * Group carries:
 *  - encoder: whole 3-byte groups are encoded; the 0-2 leftover bytes are
 *    carried on the host into the next block, and encoded with the final
 *    padding once upstream reports EOF (the reference's finalize(),
 *    :61-99);
 *  - decoder: blocks are decoded with B64X_DEC_HOLD_TAIL; the 0-3 sextets
 *    a block leaves over are device-determined, so the next block is
 *    chained on the device (b64x_session_decode_async(carry_from)) instead
 *    of waiting for the result on the host; at EOF the last block (or an
 *    empty flush) is decoded without HOLD_TAIL, giving the reference's
 *    floor(6V/8) bytes overall.
 *
 * The byte stream each stage produces is the reference's, byte for byte.
 * Per-call counts differ: a stage returns what it has finished, and
 * returns -1/EAGAIN while the GPU is busy (a consumer written for the
 * reference already handles EAGAIN from any stream).  Upstream errors are
 * passed through with all state kept when nothing is in flight; count ==
 * 0 returns 0 (ref :103-104, :54-55).  The reference's assert at
 * src/base64encoder.c:140 (counts not divisible by 4) has no counterpart.
 * With no usable GPU the first read fails with ENODEV: there is no CPU
 * path.
 *
 * Tuning (environment, read when a stage is created):
 *   ASYNC_B64_STAGE_CAPACITY  staging bytes per slot (default 1 MiB)
 *   ASYNC_B64_MIN_PULL        gather at least this much from upstream
 *                             before launching, unless it runs dry
 *                             (default 64 KiB)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include "async.h"
#include "b64x.h"
#include "base64decoder.h"
#include "base64encoder.h"

enum { NSLOTS = 2 };

typedef struct stage stage;

typedef struct {
    stage *owner;
    b64x_session *sess;
    atomic_int done;  /* set by the HIP host function */
    size_t out_pos, out_len;
} slot;

typedef enum { DIR_ENCODE, DIR_DECODE } direction;

struct stage {
    async_t *async;
    bytestream_1 up;
    action_1 cb;        /* the consumer's callback, or NULL_ACTION_1 */
    direction dir;
    b64x_alphabet abc;
    size_t cap, min_pull;
    int efd;            /* GPU completion -> loop */
    bool started;       /* sessions + eventfd exist */
    int err;            /* sticky failure errno, 0 while healthy */
    slot slots[NSLOTS];
    unsigned head;      /* oldest busy slot */
    unsigned nbusy;     /* launched, output not fully served */
    bool final_queued;  /* the last block (or nothing) has been launched */
    bool launched_any;
    uint8_t carry[2];   /* encoder: bytes of the incomplete group */
    size_t ncarry;
};

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

static void stage_init(stage *st, async_t *async, bytestream_1 up,
                       direction dir, b64x_alphabet abc)
{
    memset(st, 0, sizeof *st);
    st->async = async;
    st->up = up;
    st->cb = NULL_ACTION_1;
    st->dir = dir;
    st->abc = abc;
    st->cap = env_size("ASYNC_B64_STAGE_CAPACITY", (size_t) 1 << 20, 64);
    st->min_pull = env_size("ASYNC_B64_MIN_PULL", (size_t) 64 << 10, 1);
    st->efd = -1;
    for (int i = 0; i < NSLOTS; i++)
        st->slots[i].owner = st;
}

static ssize_t stage_fail(stage *st, int negerr)
{
    st->err = negerr < 0 ? -negerr : EIO;
    errno = st->err;
    return -1;
}

/* Loop side of the completion eventfd. */
static void stage_wake(stage *st)
{
    uint64_t v;
    while (read(st->efd, &v, sizeof v) == (ssize_t) sizeof v)
        ;
    action_1_perf(st->cb);
}

/* HIP runtime thread: publish, then signal. */
static void slot_done(void *arg)
{
    slot *sl = arg;
    atomic_store_explicit(&sl->done, 1, memory_order_release);
    uint64_t one = 1;
    ssize_t rc = write(sl->owner->efd, &one, sizeof one);
    (void) rc; /* EAGAIN only when the counter is saturated: still readable */
}

static int stage_start(stage *st)
{
    if (st->started)
        return 0;
    st->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (st->efd < 0)
        return -errno;
    if (async_register(st->async, st->efd,
                       (action_1) { st, (act_1) stage_wake }) < 0) {
        int e = errno ? errno : EIO;
        close(st->efd);
        st->efd = -1;
        return -e;
    }
    for (int i = 0; i < NSLOTS; i++) {
        st->slots[i].sess = b64x_session_open(st->cap);
        if (!st->slots[i].sess)
            return -(errno ? errno : ENODEV);
    }
    st->started = true;
    return 0;
}

static void stage_stop(stage *st)
{
    for (int i = 0; i < NSLOTS; i++) {
        if (st->slots[i].sess) {
            (void) b64x_session_wait(st->slots[i].sess);
            b64x_session_close(st->slots[i].sess);
            st->slots[i].sess = NULL;
        }
    }
    if (st->efd >= 0) {
        (void) async_unregister(st->async, st->efd);
        close(st->efd);
        st->efd = -1;
    }
    st->started = false;
}

/* Pull from upstream into dst until `want` bytes, EOF, EAGAIN or an
 * error.  Returns bytes gathered; *eof / *err report why it stopped. */
static size_t gather(stage *st, uint8_t *dst, size_t room, bool *eof,
                     int *err)
{
    size_t got = 0;
    size_t want = st->min_pull < room ? st->min_pull : room;
    *eof = false;
    *err = 0;
    while (got < want) {
        ssize_t n = bytestream_1_read(st->up, dst + got, room - got);
        if (n < 0) {
            *err = errno ? errno : EIO;
            break;
        }
        if (n == 0) {
            *eof = true;
            break;
        }
        got += (size_t) n;
    }
    return got;
}

static slot *next_launch_slot(stage *st)
{
    if (st->nbusy >= NSLOTS || st->final_queued)
        return NULL;
    return &st->slots[(st->head + st->nbusy) % NSLOTS];
}

static void slot_arm(stage *st, slot *sl)
{
    atomic_store_explicit(&sl->done, 0, memory_order_relaxed);
    sl->out_pos = sl->out_len = 0;
    st->nbusy++;
}

/* Launch as many blocks as slots and upstream allow.  Returns 0, or a
 * positive errno from upstream (EAGAIN included) that stopped it, or a
 * negative errno from the GPU side. */
static int top_up_encoder(stage *st)
{
    slot *sl;
    while ((sl = next_launch_slot(st))) {
        uint8_t *in = b64x_session_host_in(sl->sess);
        memcpy(in, st->carry, st->ncarry);
        bool eof;
        int uerr;
        size_t got = gather(st, in + st->ncarry, st->cap - st->ncarry, &eof,
                            &uerr);
        size_t total = st->ncarry + got;
        size_t n;
        if (eof) {
            st->final_queued = true;
            st->ncarry = 0;
            if (total == 0)
                return 0;
            n = total; /* finalize(): partial group + padding */
        } else {
            n = total - total % 3;
            st->ncarry = total - n;
            memcpy(st->carry, in + n, st->ncarry);
            if (n == 0)
                return uerr ? uerr : EAGAIN;
        }
        slot_arm(st, sl);
        int rc = b64x_session_encode_async(sl->sess, n, &st->abc, slot_done,
                                           sl);
        if (rc)
            return rc;
        sl->out_len = (size_t) b64x_encoded_len(n, eof && st->abc.pad);
        /* Non-final blocks are whole groups: no padding either way. */
        if (uerr)
            return uerr;
    }
    return 0;
}

static int top_up_decoder(stage *st)
{
    slot *sl;
    while ((sl = next_launch_slot(st))) {
        slot *prev = st->launched_any
                         ? &st->slots[(st->head + st->nbusy + NSLOTS - 1) %
                                      NSLOTS]
                         : NULL;
        bool eof;
        int uerr;
        size_t got = gather(st, b64x_session_host_in(sl->sess), st->cap, &eof,
                            &uerr);
        unsigned flags = B64X_DEC_HOLD_TAIL;
        if (eof) {
            st->final_queued = true;
            if (!st->launched_any && got == 0)
                return 0;
            flags = 0; /* last block, or a flush of the carried sextets */
        } else if (got == 0) {
            return uerr ? uerr : EAGAIN;
        }
        slot_arm(st, sl);
        int rc = b64x_session_decode_async(sl->sess, got, &st->abc, flags,
                                           prev ? prev->sess : NULL, slot_done,
                                           sl);
        if (rc)
            return rc;
        st->launched_any = true;
        if (uerr)
            return uerr;
    }
    return 0;
}

static ssize_t stage_read(stage *st, void *buf, size_t count)
{
    if (!count)
        return 0;
    if (st->err) {
        errno = st->err;
        return -1;
    }
    int rc = stage_start(st);
    if (rc)
        return stage_fail(st, rc);
    for (;;) {
        slot *h = &st->slots[st->head];
        if (st->nbusy &&
            atomic_load_explicit(&h->done, memory_order_acquire)) {
            if (st->dir == DIR_DECODE && h->out_len == 0 && h->out_pos == 0)
                h->out_len = (size_t) b64x_session_result(h->sess)->out_len;
            size_t avail = h->out_len - h->out_pos;
            size_t n = avail < count ? avail : count;
            if (n) {
                memcpy(buf, b64x_session_host_out(h->sess) + h->out_pos, n);
                h->out_pos += n;
            }
            if (h->out_pos == h->out_len) {
                st->nbusy--;
                st->head = (st->head + 1) % NSLOTS;
            }
            if (n) {
                /* Keep the GPU busy while the consumer works. */
                rc = st->dir == DIR_ENCODE ? top_up_encoder(st)
                                           : top_up_decoder(st);
                if (rc < 0)
                    return stage_fail(st, rc);
                return (ssize_t) n;
            }
            continue; /* an empty block: look at the next one */
        }
        rc = st->dir == DIR_ENCODE ? top_up_encoder(st) : top_up_decoder(st);
        if (rc < 0)
            return stage_fail(st, rc);
        if (st->nbusy) {
            if (atomic_load_explicit(&st->slots[st->head].done,
                                     memory_order_acquire))
                continue;
            errno = EAGAIN; /* the eventfd brings the consumer back */
            return -1;
        }
        if (st->final_queued)
            return 0;
        errno = rc ? rc : EAGAIN;
        return -1;
    }
}

static void stage_close(stage *st)
{
    stage_stop(st);
    bytestream_1_close(st->up);
    async_wound(st->async, st);
    st->async = NULL;
}

static void stage_register(stage *st, action_1 action)
{
    st->cb = action;
    bytestream_1_register_callback(st->up, action);
}

static void stage_unregister(stage *st)
{
    st->cb = NULL_ACTION_1;
    bytestream_1_unregister_callback(st->up);
}

/* ================================================================ encoder */

struct base64encoder {
    stage st; /* first member: the object pointer is the stage */
};

base64encoder_t *base64_encode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63, bool pad, char padchar)
{
    base64encoder_t *e = malloc(sizeof *e);
    if (!e)
        abort();
    b64x_alphabet abc = { pos62, pos63, padchar, pad };
    stage_init(&e->st, async, stream, DIR_ENCODE, abc);
    return e;
}

ssize_t base64encoder_read(base64encoder_t *e, void *buf, size_t count)
{
    return stage_read(&e->st, buf, count);
}

void base64encoder_close(base64encoder_t *e)
{
    stage_close(&e->st);
}

void base64encoder_register_callback(base64encoder_t *e, action_1 action)
{
    stage_register(&e->st, action);
}

void base64encoder_unregister_callback(base64encoder_t *e)
{
    stage_unregister(&e->st);
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
    stage st;
};

base64decoder_t *base64_decode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63)
{
    base64decoder_t *d = malloc(sizeof *d);
    if (!d)
        abort();
    b64x_alphabet abc = { pos62, pos63, (char) -1, false };
    stage_init(&d->st, async, stream, DIR_DECODE, abc);
    return d;
}

ssize_t base64decoder_read(base64decoder_t *d, void *buf, size_t count)
{
    return stage_read(&d->st, buf, count);
}

void base64decoder_close(base64decoder_t *d)
{
    stage_close(&d->st);
}

void base64decoder_register_callback(base64decoder_t *d, action_1 action)
{
    stage_register(&d->st, action);
}

void base64decoder_unregister_callback(base64decoder_t *d)
{
    stage_unregister(&d->st);
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
