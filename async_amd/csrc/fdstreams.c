/*
 * fdstreams.c -- the file-descriptor ends of the base64 path (SURVEY.md
 * §8(f) row f1): where real traffic enters and leaves the event loop.
 *
 *   pipestream   an fd read as a non-blocking bytestream_1
 *                (include/pipestream.h; ref src/pipestream.c:23-109)
 *   fdsink       a bytestream_1 drained into an fd, 10,240 bytes per pull
 *                (include/fdsink.h; the egress loop of ref
 *                src/tcp_connection.c:451-484, 669-727, with write(2))
 *
 * Both register their fd with async_register(), the loop's edge-triggered
 * watch (include/async.h), and allocate through fsalloc()/async_wound()
 * like every other object of the library.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <string.h>
#include <unistd.h>

#include "b64_lend.h"
#include "b64_trace.h"
#include "fdsink.h"
#include "fsalloc.h"
#include "pipestream.h"

/* ---- pipestream --------------------------------------------------------- */

struct pipestream {
    async_t *async;
    uint64_t uid;    /* the reference's trace uid */
    int fd;          /* owned; -1 once closed */
    action_1 cb;     /* the consumer's callback */
};

FSTRACE_DECL(ASYNC_PIPESTREAM_CREATE, "UID=%64u PTR=%p ASYNC=%p FD=%d");
FSTRACE_DECL(ASYNC_PIPESTREAM_READ, "UID=%64u WANT=%z GOT=%z ERRNO=%e");
FSTRACE_DECL(ASYNC_PIPESTREAM_CLOSE, "UID=%64u");

/* An edge on the fd (or the registration's possible spurious call): the
 * consumer may read again. */
static void pipe_edge(pipestream_t *p)
{
    if (p->async)
        action_1_perf(p->cb);
}

pipestream_t *open_pipestream(async_t *async, int fd)
{
    pipestream_t *p = fscalloc(1, sizeof *p);
    p->async = async;
    p->uid = b64_trace_unique_id();
    p->fd = fd;
    p->cb = NULL_ACTION_1;
    FSTRACE(ASYNC_PIPESTREAM_CREATE, p->uid, p, async, fd);
    /* non-blocking, edge-triggered; a failure shows at the first read
     * (EBADF and the like) rather than here, as in the reference */
    (void) async_register(async, fd, (action_1) { p, (act_1) pipe_edge });
    return p;
}

ssize_t pipestream_read(pipestream_t *p, void *buf, size_t count)
{
    ssize_t n = read(p->fd, buf, count);
    FSTRACE(ASYNC_PIPESTREAM_READ, p->uid, count, n);
    return n;
}

void pipestream_close(pipestream_t *p)
{
    FSTRACE(ASYNC_PIPESTREAM_CLOSE, p->uid);
    if (p->fd >= 0) {
        (void) async_unregister(p->async, p->fd);
        close(p->fd);
        p->fd = -1;
    }
    p->cb = NULL_ACTION_1;
    async_wound(p->async, p);
    p->async = NULL;
}

void pipestream_register_callback(pipestream_t *p, action_1 action)
{
    p->cb = action;
}

void pipestream_unregister_callback(pipestream_t *p)
{
    p->cb = NULL_ACTION_1;
}

static ssize_t pipe_read_vt(void *o, void *buf, size_t count)
{
    return pipestream_read(o, buf, count);
}
static void pipe_close_vt(void *o)
{
    pipestream_close(o);
}
static void pipe_reg_vt(void *o, action_1 a)
{
    pipestream_register_callback(o, a);
}
static void pipe_unreg_vt(void *o)
{
    pipestream_unregister_callback(o);
}

static const struct bytestream_1_vt pipe_vt = {
    pipe_read_vt, pipe_close_vt, pipe_reg_vt, pipe_unreg_vt
};

bytestream_1 pipestream_as_bytestream_1(pipestream_t *p)
{
    return (bytestream_1) { p, &pipe_vt };
}

/* ---- fdsink ------------------------------------------------------------- */

enum {
    SINK_BURST = 256, /* pulls per turn before yielding to other tasks */
};

struct fdsink {
    async_t *async;
    uint64_t uid;
    bytestream_1 source;  /* owned */
    int fd;               /* owned; -1 once closed */
    size_t cursor, count; /* unsent bytes: out[cursor, count) */
    const uint8_t *out;   /* outbuf, or the run the chunkencoder lent */
    bool lend;            /* the source is this library's chunkencoder */
    bool done, closed, probe_queued;
    int err;
    uint64_t bytes;
    action_1 cb;          /* performed once when done */
    uint8_t outbuf[FDSINK_PULL_SIZE];
};

FSTRACE_DECL(ASYNC_FDSINK_CREATE, "UID=%64u PTR=%p ASYNC=%p FD=%d");
FSTRACE_DECL(ASYNC_FDSINK_REPLENISH, "UID=%64u GOT=%z ERRNO=%e");
FSTRACE_DECL(ASYNC_FDSINK_WRITE, "UID=%64u WANT=%z GOT=%z ERRNO=%e");

static void sink_probe(fdsink_t *s);

static void sink_finish(fdsink_t *s, int err)
{
    s->done = true;
    s->err = err;
    if (s->fd >= 0) { /* EOF for the reader (ref: shutdown(SHUT_WR), :474) */
        (void) async_unregister(s->async, s->fd);
        close(s->fd);
        s->fd = -1;
    }
    action_1_perf(s->cb);
}

static void sink_requeue(fdsink_t *s)
{
    s->probe_queued = false;
    sink_probe(s);
}

/* The fd could not be watched (open_fdsink): done with that error, reported
 * from the loop like any other completion, so a callback registered after
 * open_fdsink() returned is performed too. */
static void sink_report(fdsink_t *s)
{
    s->probe_queued = false;
    if (s->closed || s->done)
        return;
    s->done = true;
    action_1_perf(s->cb);
}

/* ref push_output() :669-727: send what the outbuf holds, refill it with
 * one read of the source when it is empty (replenish_outbuf() :451-484);
 * EAGAIN from either side ends the turn (an fd edge or the source's
 * callback brings the sink back). */
static void sink_probe(fdsink_t *s)
{
    if (s->closed || s->done || s->fd < 0)
        return;
    for (int burst = 0; burst < SINK_BURST; burst++) {
        if (s->cursor == s->count) {
            /* over this library's chunkencoder the pull lends the frame's
             * bytes where they are (the header, the encoder's staged
             * characters): the same bytes and counts, one copy fewer */
            const uint8_t *lent = NULL;
            ssize_t n = s->lend ? b64_chunk_lend(s->source, sizeof s->outbuf, &lent)
                                : bytestream_1_read(s->source, s->outbuf, sizeof s->outbuf);
            s->out = lent ? lent : s->outbuf;
            FSTRACE(ASYNC_FDSINK_REPLENISH, s->uid, n);
            if (n < 0) {
                if (errno != EAGAIN)
                    sink_finish(s, errno ? errno : EIO);
                return;
            }
            if (n == 0) {
                sink_finish(s, 0);
                return;
            }
            s->cursor = 0;
            s->count = (size_t) n;
        }
        ssize_t w = write(s->fd, s->out + s->cursor, s->count - s->cursor);
        FSTRACE(ASYNC_FDSINK_WRITE, s->uid, s->count - s->cursor, w);
        if (w < 0) {
            if (errno == EAGAIN)
                return; /* the fd's next edge */
            if (errno == EINTR)
                continue;
            sink_finish(s, errno);
            return;
        }
        s->cursor += (size_t) w;
        s->bytes += (uint64_t) w;
    }
    if (!s->probe_queued) { /* let the loop's other tasks run */
        s->probe_queued = true;
        async_execute(s->async, (action_1) { s, (act_1) sink_requeue });
    }
}

fdsink_t *open_fdsink(async_t *async, bytestream_1 source, int fd)
{
    fdsink_t *s = fscalloc(1, sizeof *s);
    s->async = async;
    s->uid = b64_trace_unique_id();
    s->source = source;
    s->fd = fd;
    s->out = s->outbuf;
    s->lend = b64_chunk_lendable(source);
    s->cb = NULL_ACTION_1;
    FSTRACE(ASYNC_FDSINK_CREATE, s->uid, s, async, fd);
    action_1 probe = { s, (act_1) sink_probe };
    bytestream_1_register_callback(source, probe);
    if (async_register(async, fd, probe) < 0) {
        s->err = errno ? errno : EBADF;
        if (fd >= 0)
            close(fd);
        s->fd = -1;
        s->probe_queued = true;
        async_execute(async, (action_1) { s, (act_1) sink_report });
        return s;
    }
    s->probe_queued = true;
    async_execute(async, (action_1) { s, (act_1) sink_requeue });
    return s;
}

void fdsink_register_callback(fdsink_t *s, action_1 action)
{
    s->cb = action;
}

void fdsink_unregister_callback(fdsink_t *s)
{
    s->cb = NULL_ACTION_1;
}

bool fdsink_done(fdsink_t *s)
{
    return s->done;
}

int fdsink_error(fdsink_t *s)
{
    return s->err;
}

uint64_t fdsink_bytes(fdsink_t *s)
{
    return s->bytes;
}

void fdsink_close(fdsink_t *s)
{
    s->closed = true;
    s->cb = NULL_ACTION_1;
    bytestream_1_unregister_callback(s->source);
    bytestream_1_close(s->source);
    if (s->fd >= 0) {
        (void) async_unregister(s->async, s->fd);
        close(s->fd);
        s->fd = -1;
    }
    async_wound(s->async, s);
    s->async = NULL;
}
