/*
 * framing.c -- queuestream (include/queuestream.h) and chunkencoder
 * (include/chunkencoder.h): the producer and the consumer around the base64
 * encoder stage in the HTTP-style egress stack of SURVEY.md §3 CS-2 /
 * §8(d) config 5 (rows f2/f3 of §8(f)):
 *
 *   queuestream (messages) -> base64_encode (GPU stage) -> chunk_encode
 *
 * Written from the behaviour the headers restate (ref src/queuestream.c,
 * src/chunkencoder.c); objects come from fsalloc() and are freed through
 * async_wound() like the reference's (include/fsalloc.h), so callbacks
 * arriving after close() find valid memory.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <limits.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "b64_lend.h"
#include "b64_pin.h"
#include "blobstream.h"
#include "chunkencoder.h"
#include "fsalloc.h"
#include "queuestream.h"

static void *xmalloc(size_t size)
{
    return fsalloc(size);
}

/* ================================================================ queue */

static const struct bytestream_1_vt queue_vt;

typedef struct qnode {
    bytestream_1 stream;
    struct qnode *next;
} qnode;

struct queuestream {
    async_t *async;
    qnode *first, *last;
    int deferred_errno;      /* a failure to report on the next read */
    bool terminated, closed, released;
    bool callback_owed;      /* we answered EAGAIN: notify on progress */
    action_1 callback;
};

queuestream_t *make_relaxed_queuestream(async_t *async)
{
    queuestream_t *q = xmalloc(sizeof *q);
    memset(q, 0, sizeof *q);
    q->async = async;
    q->callback = NULL_ACTION_1;
    return q;
}

queuestream_t *make_queuestream(async_t *async)
{
    queuestream_t *q = make_relaxed_queuestream(async);
    queuestream_release(q);
    return q;
}

bool queuestream_closed(queuestream_t *q)
{
    return q->closed;
}

void queuestream_release(queuestream_t *q)
{
    q->released = true;
    if (q->closed)
        async_wound(q->async, q);
}

/* Progress on the queue: wake the reader if it is waiting. */
static void queue_progress(queuestream_t *q)
{
    if (!q->callback_owed)
        return;
    q->callback_owed = false;
    action_1_perf(q->callback);
}

static void queue_adopt(queuestream_t *q, bytestream_1 s, bool at_front)
{
    if (q->closed) {
        bytestream_1_close_relaxed(q->async, s);
        return;
    }
    qnode *n = xmalloc(sizeof *n);
    n->stream = s;
    n->next = NULL;
    if (at_front) {
        n->next = q->first;
        q->first = n;
        if (!q->last)
            q->last = n;
    } else {
        if (q->last)
            q->last->next = n;
        else
            q->first = n;
        q->last = n;
    }
    action_1 wake = { q, (act_1) queue_progress };
    bytestream_1_register_callback(s, wake);
    async_execute(q->async, wake);
}

void queuestream_enqueue(queuestream_t *q, bytestream_1 s)
{
    queue_adopt(q, s, false);
}

void queuestream_push(queuestream_t *q, bytestream_1 s)
{
    queue_adopt(q, s, true);
}

/* The copy (ref src/queuestream.c:117-131) goes into pinned memory
 * (streams.c b64_pinned_blobstream), so that a GPU encoder stage reading
 * this queue can take the bytes from there (b64_src_peek). */
void queuestream_enqueue_bytes(queuestream_t *q, const void *blob, size_t count)
{
    queue_adopt(q, blobstream_as_bytestream_1(b64_pinned_blobstream(q->async, blob, count)),
                false);
}

void queuestream_push_bytes(queuestream_t *q, const void *blob, size_t count)
{
    queue_adopt(q, blobstream_as_bytestream_1(b64_pinned_blobstream(q->async, blob, count)),
                true);
}

void queuestream_terminate(queuestream_t *q)
{
    if (q->closed)
        return;
    q->terminated = true;
    async_execute(q->async, (action_1) { q, (act_1) queue_progress });
}

static void queue_drop_first(queuestream_t *q)
{
    qnode *n = q->first;
    q->first = n->next;
    if (!q->first)
        q->last = NULL;
    bytestream_1_close(n->stream);
    fsfree(n);
}

ssize_t queuestream_read(queuestream_t *q, void *buf, size_t count)
{
    if (q->deferred_errno) {
        errno = q->deferred_errno;
        q->deferred_errno = 0;
        return -1;
    }
    if (!count)
        return 0;
    if (count > SSIZE_MAX)
        count = SSIZE_MAX;
    uint8_t *dst = buf;
    size_t got = 0;
    while (got < count && q->first) {
        ssize_t n = bytestream_1_read(q->first->stream, dst + got, count - got);
        if (n > 0) {
            got += (size_t) n;
            continue;
        }
        if (n == 0) {
            queue_drop_first(q);
            continue;
        }
        if (got == 0) {
            if (errno == EAGAIN)
                q->callback_owed = true;
            return -1;
        }
        if (errno != EAGAIN)
            q->deferred_errno = errno;
        break;
    }
    if (got)
        return (ssize_t) got;
    if (q->terminated)
        return 0;
    q->callback_owed = true;
    errno = EAGAIN;
    return -1;
}

bool b64_src_peek(bytestream_1 s, const uint8_t **p, size_t *n, b64_pin_slab **slab)
{
    if (s.vt != &queue_vt)
        return false;
    queuestream_t *q = s.obj;
    if (q->deferred_errno)
        return false;
    while (q->first) {
        if (!b64_blob_lend_peek(q->first->stream, p, n, slab) || !*slab)
            return false;
        if (*n)
            break;
        queue_drop_first(q); /* as queuestream_read() would */
    }
    return q->first != NULL;
}

void b64_src_take(bytestream_1 s, size_t n)
{
    queuestream_t *q = s.obj;
    b64_blob_lend_take(q->first->stream, n);
}

size_t b64_src_plain(bytestream_1 s, size_t lend_min, size_t limit)
{
    if (s.vt != &queue_vt)
        return limit;
    queuestream_t *q = s.obj;
    size_t plain = 0;
    for (qnode *e = q->first; e && plain < limit; e = e->next) {
        const uint8_t *p;
        size_t n;
        b64_pin_slab *slab;
        if (!b64_blob_lend_peek(e->stream, &p, &n, &slab))
            return limit; /* another kind of stream: no telling */
        if (slab && n >= lend_min)
            return plain < limit ? plain : limit;
        plain += n;
    }
    return limit;
}

void queuestream_close(queuestream_t *q)
{
    while (q->first)
        queue_drop_first(q);
    q->closed = true;
    if (q->released)
        async_wound(q->async, q);
}

void queuestream_register_callback(queuestream_t *q, action_1 action)
{
    q->callback = action;
}

void queuestream_unregister_callback(queuestream_t *q)
{
    q->callback = NULL_ACTION_1;
}

static ssize_t q_read_vt(void *o, void *buf, size_t count)
{
    return queuestream_read(o, buf, count);
}
static void q_close_vt(void *o)
{
    queuestream_close(o);
}
static void q_reg_vt(void *o, action_1 a)
{
    queuestream_register_callback(o, a);
}
static void q_unreg_vt(void *o)
{
    queuestream_unregister_callback(o);
}

static const struct bytestream_1_vt queue_vt = { q_read_vt, q_close_vt, q_reg_vt,
                                                 q_unreg_vt };

bytestream_1 queuestream_as_bytestream_1(queuestream_t *q)
{
    return (bytestream_1) { q, &queue_vt };
}

/* ========================================================= chunk framing */

static const struct bytestream_1_vt chunk_vt;

enum {
    CHUNK_MIN = 2,
    CHUNK_MAX = 16 * 1024 * 1024,
    /* room in front of a chunk's data: "\r\n" + up to 7 hex digits (16 MiB
     * is 0x1000000) + "\r\n" */
    CHUNK_HEAD = 2 + 7 + 2,
};

struct chunkencoder {
    async_t *async;
    bytestream_1 up;
    size_t max_chunk;
    chunkencoder_termination_t termination;
    uint8_t *frame;    /* CHUNK_HEAD + max_chunk (+2 for the final CRLF) */
    const uint8_t *data; /* the chunk's data lent by a GPU encoder stage
                            (b64_lend.h), or NULL: it is in frame */
    bool lend;         /* upstream lends every chunk: frame is header-only */
    size_t pos, end;   /* unserved part of the current frame */
    size_t chunks;     /* frames started */
    bool last_framed;  /* the zero-length chunk has been built */
};

chunkencoder_t *chunk_encode_2(async_t *async, bytestream_1 stream,
                               size_t max_chunk_size,
                               chunkencoder_termination_t termination)
{
    chunkencoder_t *c = xmalloc(sizeof *c);
    memset(c, 0, sizeof *c);
    c->async = async;
    c->up = stream;
    c->max_chunk = max_chunk_size < CHUNK_MIN   ? CHUNK_MIN
                   : max_chunk_size > CHUNK_MAX ? CHUNK_MAX
                                                : max_chunk_size;
    c->termination = termination;
    /* over the GPU encoder the chunk's data is lent (b64_lend.h): the frame
     * holds only the header and the final CRLF, not max_chunk bytes */
    c->lend = b64_lend_capable(stream);
    c->frame = xmalloc(CHUNK_HEAD + (c->lend ? 2 : c->max_chunk));
    return c;
}

chunkencoder_t *chunk_encode(async_t *async, bytestream_1 stream,
                             size_t max_chunk_size)
{
    return chunk_encode_2(async, stream, max_chunk_size, CHUNKENCODER_SIMPLE);
}

/* Write "[\r\n]<hex n>\r\n" so that it ends right before the data at
 * frame + CHUNK_HEAD; returns where the header starts. */
static size_t chunk_header(chunkencoder_t *c, size_t n)
{
    static const char hex[] = "0123456789abcdef";
    size_t p = CHUNK_HEAD;
    c->frame[--p] = '\n';
    c->frame[--p] = '\r';
    do {
        c->frame[--p] = (uint8_t) hex[n & 15];
        n >>= 4;
    } while (n);
    if (c->chunks++) {
        c->frame[--p] = '\n';
        c->frame[--p] = '\r';
    }
    return p;
}

/* The current frame is served: build the next one (1), or 0 after the
 * terminating frame, -1 with errno from upstream. */
static int chunk_refill(chunkencoder_t *c)
{
    if (c->data) { /* the lent chunk has been served */
        b64_lend_return(c->up);
        c->data = NULL;
    }
    if (c->last_framed)
        return 0;
    /* same count as a read into the frame; from the GPU encoder the
     * data usually stays where the stage has it (one copy fewer) */
    ssize_t n = b64_lend_read(c->up, c->lend ? NULL : c->frame + CHUNK_HEAD, c->max_chunk,
                              &c->data);
    if (n < 0)
        return -1;
    c->pos = chunk_header(c, (size_t) n);
    c->end = CHUNK_HEAD + (size_t) n;
    if (n == 0) {
        c->last_framed = true;
        switch (c->termination) {
            case CHUNKENCODER_SIMPLE: /* "0\r\n" + empty trailer "\r\n" */
                c->frame[c->end++] = '\r';
                c->frame[c->end++] = '\n';
                break;
            case CHUNKENCODER_STOP_AT_TRAILER: /* "0\r\n" */
                break;
            case CHUNKENCODER_STOP_AT_FINAL_EXTENSIONS: /* "0" */
                c->end -= 2;
                break;
            default:
                abort();
        }
    }
    return 1;
}

/* The next contiguous run of the frame, at most `count` bytes: the header
 * (and closing CRLF) from the frame, the data from the frame or from where
 * the GPU encoder stage lent it. */
static size_t chunk_run(chunkencoder_t *c, size_t count, const uint8_t **p)
{
    size_t n = c->end - c->pos;
    if (n > count)
        n = count;
    if (c->data && c->pos < CHUNK_HEAD) {
        if (n > CHUNK_HEAD - c->pos)
            n = CHUNK_HEAD - c->pos;
        *p = c->frame + c->pos;
    } else {
        *p = (c->data ? c->data - CHUNK_HEAD : c->frame) + c->pos;
    }
    c->pos += n;
    return n;
}

ssize_t chunkencoder_read(chunkencoder_t *c, void *buf, size_t count)
{
    if (!count)
        return 0;
    if (c->pos == c->end) {
        int r = chunk_refill(c);
        if (r <= 0)
            return r;
    }
    /* as many bytes as the frame has, in up to two runs */
    size_t done = 0, want = c->end - c->pos < count ? c->end - c->pos : count;
    while (done < want) {
        const uint8_t *p;
        size_t n = chunk_run(c, want - done, &p);
        memcpy((uint8_t *) buf + done, p, n);
        done += n;
    }
    return (ssize_t) done;
}

bool b64_chunk_lendable(bytestream_1 s)
{
    return s.vt == &chunk_vt;
}

ssize_t b64_chunk_lend(bytestream_1 s, size_t count, const uint8_t **p)
{
    chunkencoder_t *c = s.obj;
    if (!count)
        return 0;
    if (c->pos == c->end) {
        int r = chunk_refill(c);
        if (r <= 0)
            return r;
    }
    return (ssize_t) chunk_run(c, count, p);
}

void chunkencoder_close(chunkencoder_t *c)
{
    c->data = NULL; /* the stage's close ends the loan */
    bytestream_1_close(c->up);
    fsfree(c->frame);
    c->frame = NULL;
    async_wound(c->async, c);
    c->async = NULL;
}

void chunkencoder_register_callback(chunkencoder_t *c, action_1 action)
{
    bytestream_1_register_callback(c->up, action);
}

void chunkencoder_unregister_callback(chunkencoder_t *c)
{
    bytestream_1_unregister_callback(c->up);
}

static ssize_t c_read_vt(void *o, void *buf, size_t count)
{
    return chunkencoder_read(o, buf, count);
}
static void c_close_vt(void *o)
{
    chunkencoder_close(o);
}
static void c_reg_vt(void *o, action_1 a)
{
    chunkencoder_register_callback(o, a);
}
static void c_unreg_vt(void *o)
{
    chunkencoder_unregister_callback(o);
}

static const struct bytestream_1_vt chunk_vt = { c_read_vt, c_close_vt, c_reg_vt,
                                                 c_unreg_vt };

bytestream_1 chunkencoder_as_bytestream_1(chunkencoder_t *c)
{
    return (bytestream_1) { c, &chunk_vt };
}
