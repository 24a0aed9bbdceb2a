/*
 * streams.c -- the small bytestream_1 sources and wrappers the base64
 * path is fed and tested through:
 *
 *   NULL_ACTION_1, bytestream_1_close_relaxed   ref src/action_1.c,
 *                                               src/bytestream_1.c:13-18
 *   blobstream (memory source)                  ref src/blobstream.c
 *   nicestream (periodic EAGAIN injector)       ref src/nicestream.c:34-51
 *
 * Written from the interface contracts in the include/ headers; objects come
 * from fsalloc() and are freed through async_wound() like the reference's
 * (include/fsalloc.h), so a callback arriving after close() still finds
 * valid memory and a counting allocator sees every object go.
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "b64_lend.h"
#include "b64_pin.h"
#include "blobstream.h"
#include "bytestream_1.h"
#include "fsalloc.h"
#include "nicestream.h"

static void do_nothing(void *obj)
{
    (void) obj;
}

action_1 NULL_ACTION_1 = { NULL, do_nothing };

static void *xcalloc(size_t size)
{
    return fscalloc(1, size);
}

/* ---- bytestream_1_close_relaxed ----------------------------------- */

struct relaxed_close {
    bytestream_1 stream;
};

static void relaxed_close_now(struct relaxed_close *rc)
{
    bytestream_1 s = rc->stream;
    fsfree(rc);
    bytestream_1_close(s);
}

void bytestream_1_close_relaxed(async_t *async, bytestream_1 stream)
{
    struct relaxed_close *rc = xcalloc(sizeof *rc);
    rc->stream = stream;
    async_execute(async, (action_1) { rc, (act_1) relaxed_close_now });
}

/* ---- blobstream ------------------------------------------------------- */

struct blobstream {
    async_t *async;
    const uint8_t *data;
    size_t size, pos;
    void *owned;
    b64_pin_slab *slab; /* data is a pinned piece of this slab (b64_pin.h) */
    action_1 on_close;
};

static blobstream_t *new_blob(async_t *async, const void *blob, size_t count,
                              void *owned, action_1 on_close)
{
    blobstream_t *b = xcalloc(sizeof *b);
    b->async = async;
    b->data = blob;
    b->size = count;
    b->owned = owned;
    b->on_close = on_close;
    return b;
}

blobstream_t *open_blobstream(async_t *async, const void *blob, size_t count)
{
    return new_blob(async, blob, count, NULL, NULL_ACTION_1);
}

blobstream_t *copy_blobstream(async_t *async, const void *blob, size_t count)
{
    void *copy = fsalloc(count ? count : 1);
    if (count)
        memcpy(copy, blob, count);
    return new_blob(async, copy, count, copy, NULL_ACTION_1);
}

blobstream_t *adopt_blobstream(async_t *async, const void *blob, size_t count,
                               action_1 close_action)
{
    return new_blob(async, blob, count, NULL, close_action);
}

size_t blobstream_remaining(blobstream_t *b)
{
    return b->size - b->pos;
}

ssize_t blobstream_read(blobstream_t *b, void *buf, size_t count)
{
    size_t n = blobstream_remaining(b);
    if (n > count)
        n = count;
    if (n)
        memcpy(buf, b->data + b->pos, n);
    b->pos += n;
    return (ssize_t) n;
}

/* copy_blobstream() into pinned memory the GPU can read (b64_pin.h), so
 * that an encoder stage can take the bytes without copying them; an
 * ordinary copy when the pool is off or has no room. */
blobstream_t *b64_pinned_blobstream(async_t *async, const void *blob, size_t count)
{
    b64_pin_slab *slab = NULL;
    uint8_t *copy = count ? b64_pin_alloc(count, &slab) : NULL;
    if (!copy)
        return copy_blobstream(async, blob, count);
    memcpy(copy, blob, count);
    blobstream_t *b = new_blob(async, copy, count, NULL, NULL_ACTION_1);
    b->slab = slab;
    return b;
}

void blobstream_close(blobstream_t *b)
{
    action_1_perf(b->on_close);
    fsfree(b->owned);
    b->owned = NULL;
    if (b->slab) {
        b64_pin_unref(b->slab);
        b->slab = NULL;
    }
    async_wound(b->async, b);
    b->async = NULL;
}

void blobstream_register_callback(blobstream_t *b, action_1 action)
{
    (void) b;
    (void) action; /* never returns EAGAIN, so never calls back */
}

void blobstream_unregister_callback(blobstream_t *b)
{
    (void) b;
}

static ssize_t blob_read_vt(void *o, void *buf, size_t count)
{
    return blobstream_read(o, buf, count);
}
static void blob_close_vt(void *o)
{
    blobstream_close(o);
}
static void blob_reg_vt(void *o, action_1 a)
{
    blobstream_register_callback(o, a);
}
static void blob_unreg_vt(void *o)
{
    blobstream_unregister_callback(o);
}

static const struct bytestream_1_vt blob_vt = {
    blob_read_vt, blob_close_vt, blob_reg_vt, blob_unreg_vt
};

bytestream_1 blobstream_as_bytestream_1(blobstream_t *b)
{
    return (bytestream_1) { b, &blob_vt };
}

/* b64_lend.h, upstream side: a pinned blob's unread bytes. */
bool b64_blob_lend_peek(bytestream_1 s, const uint8_t **p, size_t *n, b64_pin_slab **slab)
{
    if (s.vt != &blob_vt)
        return false;
    blobstream_t *b = s.obj;
    *p = b->data + b->pos;
    *n = b->size - b->pos;
    *slab = b->slab;
    return true;
}

void b64_blob_lend_take(bytestream_1 s, size_t n)
{
    blobstream_t *b = s.obj;
    b->pos += n;
}


/* ---- nicestream ------------------------------------------------------- */

struct nicestream {
    async_t *async;
    bytestream_1 upstream;
    size_t burst, max_burst;
    action_1 callback;
};

nicestream_t *make_nice(async_t *async, bytestream_1 stream, size_t max_burst)
{
    nicestream_t *n = xcalloc(sizeof *n);
    n->async = async;
    n->upstream = stream;
    n->max_burst = max_burst;
    n->callback = NULL_ACTION_1;
    return n;
}

static void nice_retry(nicestream_t *n)
{
    if (n->async) /* not after close */
        action_1_perf(n->callback);
}

ssize_t nicestream_read(nicestream_t *n, void *buf, size_t count)
{
    if (n->burst > n->max_burst) {
        /* Back off once, and promise the caller a callback. */
        n->burst = 0;
        async_execute(n->async, (action_1) { n, (act_1) nice_retry });
        errno = EAGAIN;
        return -1;
    }
    ssize_t got = bytestream_1_read(n->upstream, buf, count);
    n->burst = got < 0 ? 0 : n->burst + (size_t) got;
    return got;
}

void nicestream_close(nicestream_t *n)
{
    bytestream_1_close(n->upstream);
    async_wound(n->async, n);
    n->async = NULL;
}

void nicestream_register_callback(nicestream_t *n, action_1 action)
{
    n->callback = action;
    bytestream_1_register_callback(n->upstream, action);
}

void nicestream_unregister_callback(nicestream_t *n)
{
    n->callback = NULL_ACTION_1;
    bytestream_1_unregister_callback(n->upstream);
}

static ssize_t nice_read_vt(void *o, void *buf, size_t count)
{
    return nicestream_read(o, buf, count);
}
static void nice_close_vt(void *o)
{
    nicestream_close(o);
}
static void nice_reg_vt(void *o, action_1 a)
{
    nicestream_register_callback(o, a);
}
static void nice_unreg_vt(void *o)
{
    nicestream_unregister_callback(o);
}

static const struct bytestream_1_vt nice_vt = {
    nice_read_vt, nice_close_vt, nice_reg_vt, nice_unreg_vt
};

bytestream_1 nicestream_as_bytestream_1(nicestream_t *n)
{
    return (bytestream_1) { n, &nice_vt };
}
