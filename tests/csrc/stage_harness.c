/*
 * stage_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives the product's bytestream_1 stages (libasync_b64.so) on the
 * product's own event loop, the way the reference's test does
 * (test/asynctest-base64encoder.c:86-151): a verify action reads from the
 * outermost stream, re-schedules itself with async_execute() after data,
 * waits for the registered callback after EAGAIN and quits at EOF.
 * Python calls these through ctypes (tests/test_stages_gpu.py).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <pthread.h>
#include <unistd.h>

#include "async.h"
#include "base64decoder.h"
#include "base64encoder.h"
#include "blobstream.h"
#include "chunkencoder.h"
#include "fdsink.h"
#include "fsalloc.h"
#include "nicestream.h"
#include "pipestream.h"
#include "queuestream.h"

/* ---- the reference runner's leak check: test/asynctest.c:108-147 ------ */

/* Wired like the reference's main() (test/asynctest.c:276-278): every
 * fsalloc()/fsfree() of the library (loop, streams, stages, hub) goes
 * through test_realloc, which counts live objects and fills fresh ones with
 * 0xa5; h_count_end() returns what is still outstanding (the reference's
 * posttest_check fails a test on anything but 0). */
static int outstanding_object_count;
static fs_realloc_t reallocator;

static void *test_realloc(void *ptr, size_t size)
{
    void *obj = reallocator(ptr, size);
    if (ptr)
        outstanding_object_count--;
    if (obj) {
        if (!ptr)
            memset(obj, 0xa5, size);
        outstanding_object_count++;
    }
    return obj;
}

static void test_reallocator_counter(int count)
{
    outstanding_object_count += count;
}

void h_count_begin(void)
{
    outstanding_object_count = 0;
    reallocator = fs_get_reallocator();
    fs_set_reallocator(test_realloc);
    fs_set_reallocator_counter(test_reallocator_counter);
}

int h_count_end(void)
{
    fs_set_reallocator(reallocator);
    fs_set_reallocator_counter(NULL);
    return outstanding_object_count;
}

/* ---- counting source: test/asynctest-base64encoder.c:11-78 ------------ */

typedef struct {
    async_t *async;
    size_t size, cursor;
} counting_source;

static ssize_t cs_read(void *obj, void *buf, size_t count)
{
    counting_source *s = obj;
    size_t remaining = s->size - s->cursor;
    if (remaining < count)
        count = remaining;
    uint8_t *p = buf;
    for (size_t i = 0; i < count; i++)
        *p++ = (uint8_t) s->cursor++;
    return (ssize_t) count;
}

static void cs_close(void *obj)
{
    counting_source *s = obj;
    async_wound(s->async, s);
    s->async = NULL;
}

static void cs_reg(void *obj, action_1 a)
{
    (void) obj;
    (void) a;
}

static void cs_unreg(void *obj)
{
    (void) obj;
}

static const struct bytestream_1_vt cs_vt = { cs_read, cs_close, cs_reg,
                                              cs_unreg };

/* ---- failing source: data, then a hard error -------------------------- */

/* Serves in[0..n) at most `chunk` bytes per read (chunk 0: every read
 * full, a read that the rest cannot fill fails), then fails every read with
 * errno `fail` (a socket reset, a disk error): the upstream ADVICE r04
 * describes, whose error the stage must not turn into EAGAIN. */
typedef struct {
    async_t *async;
    const uint8_t *in;
    size_t n, cursor, chunk;
    int fail;
} failing_source;

static ssize_t fs_src_read(void *obj, void *buf, size_t count)
{
    failing_source *s = obj;
    if (s->cursor == s->n || (!s->chunk && s->n - s->cursor < count)) {
        s->cursor = s->n;
        errno = s->fail;
        return -1;
    }
    if (s->chunk && count > s->chunk)
        count = s->chunk;
    if (count > s->n - s->cursor)
        count = s->n - s->cursor;
    memcpy(buf, s->in + s->cursor, count);
    s->cursor += count;
    return (ssize_t) count;
}

static void fs_src_close(void *obj)
{
    failing_source *s = obj;
    async_wound(s->async, s);
    s->async = NULL;
}

static const struct bytestream_1_vt fs_src_vt = { fs_src_read, fs_src_close, cs_reg,
                                                  cs_unreg };

/* ---- tap: copies what flows between two stages ------------------------ */

typedef struct {
    async_t *async;
    bytestream_1 up;
    uint8_t *copy;
    size_t cap, len;
    size_t *len_out; /* outlives the stream, which the loop frees */
    int overflow;
} tap_stream;

static ssize_t tap_read(void *obj, void *buf, size_t count)
{
    tap_stream *t = obj;
    ssize_t n = bytestream_1_read(t->up, buf, count);
    if (n > 0) {
        if (t->copy && t->len + (size_t) n <= t->cap)
            memcpy(t->copy + t->len, buf, (size_t) n);
        else if (t->copy)
            t->overflow = 1;
        t->len += (size_t) n;
        if (t->len_out)
            *t->len_out = t->len;
    }
    return n;
}

static void tap_close(void *obj)
{
    tap_stream *t = obj;
    bytestream_1_close(t->up);
    async_wound(t->async, t);
    t->async = NULL;
}

static void tap_reg(void *obj, action_1 a)
{
    tap_stream *t = obj;
    bytestream_1_register_callback(t->up, a);
}

static void tap_unreg(void *obj)
{
    tap_stream *t = obj;
    bytestream_1_unregister_callback(t->up);
}

static const struct bytestream_1_vt tap_vt = { tap_read, tap_close, tap_reg,
                                               tap_unreg };

/* ---- the consumer ----------------------------------------------------- */

typedef struct {
    async_t *async;
    bytestream_1 material;
    size_t read_size;
    uint8_t *out;
    size_t cap, len;
    int err;      /* errno of a failed read, 0 otherwise */
    int done;
    size_t eagains, reads;
    ssize_t *counts; /* optional log of positive read returns */
    size_t max_counts, ncounts;
    size_t *live;    /* optional: consumers still running; quit at 0 */
    int timed_out;   /* the watchdog ended the run */
} consumer;

static void watchdog(consumer *c)
{
    c->timed_out = 1;
    async_quit_loop(c->async);
}

/* ASYNC_B64_HUB_TRACE=1: the consumers' read time on this thread (the
 * reads include what they trigger: upstream gathers, launches, framing,
 * the copy out), for the config-5 phase breakdown (scripts/cfg5_profile.py). */
static double now_s(void);
static __thread double tl_read_s;
static __thread unsigned long tl_reads;

static int read_tracing(void)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("ASYNC_B64_HUB_TRACE");
        on = e && *e && *e != '0';
    }
    return on;
}

double h_take_read_seconds(unsigned long *reads)
{
    double s = tl_read_s;
    if (reads)
        *reads = tl_reads;
    tl_read_s = 0;
    tl_reads = 0;
    return s;
}

static void consumer_finish(consumer *c)
{
    c->done = 1;
    bytestream_1_close(c->material);
    if (!c->live || --*c->live == 0)
        async_quit_loop(c->async);
}

/* Reads `read_size` at a time straight into the destination (the way a
 * socket writer reads into the buffer it sends from); a scratch buffer
 * only when fewer than read_size bytes of room are left, so that an
 * overlong stream is still detected. */
static void consume(consumer *c)
{
    if (c->done)
        return;
    uint8_t *scratch = NULL, *buf = c->out + c->len;
    if (c->cap - c->len < c->read_size) {
        scratch = malloc(c->read_size);
        if (!scratch)
            abort();
        buf = scratch;
    }
    double t0 = read_tracing() ? now_s() : 0;
    ssize_t n = bytestream_1_read(c->material, buf, c->read_size);
    if (t0) {
        tl_read_s += now_s() - t0;
        tl_reads++;
    }
    c->reads++;
    if (n < 0) {
        free(scratch);
        if (errno == EAGAIN) {
            c->eagains++;
            return; /* the registered callback brings us back */
        }
        c->err = errno;
        consumer_finish(c);
        return;
    }
    if (n == 0) {
        free(scratch);
        consumer_finish(c);
        return;
    }
    if (c->len + (size_t) n > c->cap) {
        free(scratch);
        c->err = ENOSPC;
        consumer_finish(c);
        return;
    }
    if (scratch) {
        memcpy(c->out + c->len, scratch, (size_t) n);
        free(scratch);
    }
    c->len += (size_t) n;
    if (c->counts && c->ncounts < c->max_counts)
        c->counts[c->ncounts] = n;
    c->ncounts++;
    async_execute(c->async, (action_1) { c, (act_1) consume });
}

static ssize_t run(async_t *async, bytestream_1 material, size_t read_size,
                   uint8_t *out, size_t cap, int *err_out, size_t *eagains)
{
    consumer c;
    memset(&c, 0, sizeof c);
    c.async = async;
    c.material = material;
    c.read_size = read_size;
    c.out = out;
    c.cap = cap;
    action_1 cb = { &c, (act_1) consume };
    bytestream_1_register_callback(material, cb);
    async_execute(async, cb);
    int rc = async_loop(async);
    if (err_out)
        *err_out = rc < 0 ? errno : c.err;
    if (eagains)
        *eagains = c.eagains;
    /* Let wounded objects be freed. */
    destroy_async(async);
    if (rc < 0 || c.err)
        return -1;
    return (ssize_t) c.len;
}

/* The reference topology, with the product's stages in the middle. */
ssize_t h_reftest(size_t length, uint8_t *enc_out, size_t enc_cap,
                  size_t *enc_len, uint8_t *dec_out, size_t dec_cap,
                  int *err_out, size_t *eagains)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    counting_source *src = fscalloc(1, sizeof *src);
    src->async = async;
    src->size = length;
    nicestream_t *n1 = make_nice(async, (bytestream_1) { src, &cs_vt }, 113);
    base64encoder_t *enc = base64_encode(async, nicestream_as_bytestream_1(n1),
                                         '.', '_', true, '-');
    tap_stream *tap = fscalloc(1, sizeof *tap);
    tap->async = async;
    tap->up = base64encoder_as_bytestream_1(enc);
    tap->copy = enc_out;
    tap->cap = enc_cap;
    if (enc_len)
        *enc_len = 0;
    tap->len_out = enc_len;
    nicestream_t *n2 = make_nice(async, (bytestream_1) { tap, &tap_vt }, 91);
    base64decoder_t *dec =
        base64_decode(async, nicestream_as_bytestream_1(n2), '.', '_');
    nicestream_t *n3 = make_nice(async, base64decoder_as_bytestream_1(dec), 97);
    return run(async, nicestream_as_bytestream_1(n3), 200, dec_out, dec_cap,
               err_out, eagains);
}

static bytestream_1 blob_chain(async_t *async, const uint8_t *in, size_t n,
                               size_t burst)
{
    bytestream_1 s = blobstream_as_bytestream_1(open_blobstream(async, in, n));
    if (burst)
        s = nicestream_as_bytestream_1(make_nice(async, s, burst));
    return s;
}

ssize_t h_encode_stream(const uint8_t *in, size_t n, size_t burst,
                        size_t read_size, char pos62, char pos63, int pad,
                        char padchar, uint8_t *out, size_t cap, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    base64encoder_t *enc = base64_encode(async, blob_chain(async, in, n, burst),
                                         pos62, pos63, pad != 0, padchar);
    return run(async, base64encoder_as_bytestream_1(enc), read_size, out, cap,
               err_out, NULL);
}

ssize_t h_decode_stream(const uint8_t *in, size_t n, size_t burst,
                        size_t read_size, char pos62, char pos63, uint8_t *out,
                        size_t cap, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    base64decoder_t *dec =
        base64_decode(async, blob_chain(async, in, n, burst), pos62, pos63);
    return run(async, base64decoder_as_bytestream_1(dec), read_size, out, cap,
               err_out, NULL);
}

/* failing source (n bytes in reads of `chunk`, then errno `fail`) ->
 * encoder (decode == 0) or decoder -> consumer reading `read_size`.  The
 * output before the failure goes to out; returns its length (also when the
 * run ends in the error), *err_out the errno the consumer saw (0 at EOF). */
ssize_t h_stage_upstream_error(int decode, const uint8_t *in, size_t n, size_t chunk, int fail,
                               size_t read_size, uint8_t *out, size_t cap, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    failing_source *src = fscalloc(1, sizeof *src);
    src->async = async;
    src->in = in;
    src->n = n;
    src->chunk = chunk;
    src->fail = fail;
    bytestream_1 up = { src, &fs_src_vt };
    bytestream_1 st = decode ? base64decoder_as_bytestream_1(base64_decode(async, up, -1, -1))
                             : base64encoder_as_bytestream_1(base64_encode(async, up, -1, -1,
                                                                           true, -1));
    consumer c;
    memset(&c, 0, sizeof c);
    c.async = async;
    c.material = st;
    c.read_size = read_size;
    c.out = out;
    c.cap = cap;
    action_1 cb = { &c, (act_1) consume };
    bytestream_1_register_callback(st, cb);
    async_execute(async, cb);
    /* the reference runner's watchdog (test/asynctest.c:60-69): a consumer
     * left waiting for a callback that never comes ends as ETIMEDOUT */
    async_timer_t *dog = async_timer_start(async, async_now(async) + 5 * (uint64_t) ASYNC_S,
                                           (action_1) { &c, (act_1) watchdog });
    int rc = async_loop(async);
    if (!c.timed_out)
        async_timer_cancel(async, dog);
    destroy_async(async);
    if (err_out)
        *err_out = rc < 0 ? errno : c.timed_out ? ETIMEDOUT : c.err;
    return rc < 0 ? -1 : (ssize_t) c.len;
}

/* Loop + streams only (no GPU): blob -> nice(burst) -> consumer. */
ssize_t h_copy_stream(const uint8_t *in, size_t n, size_t burst,
                      size_t read_size, uint8_t *out, size_t cap, int *err_out,
                      size_t *eagains)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    return run(async, blob_chain(async, in, n, burst), read_size, out, cap,
               err_out, eagains);
}

/* The GPU encoder stage's positive read returns, for comparison with the
 * reference's (oracle orc_encode_counts).  Returns how many, or -1. */
ssize_t h_encode_counts(const uint8_t *in, size_t n, size_t src_chunk,
                        size_t burst, size_t read_size, char pos62, char pos63,
                        int pad, char padchar, ssize_t *counts,
                        size_t max_counts, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    (void) src_chunk;
    base64encoder_t *enc = base64_encode(async, blob_chain(async, in, n, burst),
                                         pos62, pos63, pad != 0, padchar);
    size_t cap = (n + 2) / 3 * 4 + 16;
    uint8_t *out = malloc(cap);
    consumer c;
    memset(&c, 0, sizeof c);
    c.async = async;
    c.material = base64encoder_as_bytestream_1(enc);
    c.read_size = read_size;
    c.out = out;
    c.cap = cap;
    c.counts = counts;
    c.max_counts = max_counts;
    action_1 cb = { &c, (act_1) consume };
    bytestream_1_register_callback(c.material, cb);
    async_execute(async, cb);
    int rc = async_loop(async);
    destroy_async(async);
    free(out);
    if (err_out)
        *err_out = rc < 0 ? errno : c.err;
    return rc < 0 || c.err ? -1 : (ssize_t) c.ncounts;
}

/* chunkencoder over blob -> nice(burst), no GPU (the reference's
 * test/asynctest-chunkencoder.c reads 100 at a time, MAX_CHUNK 30). */
ssize_t h_chunk_stream(const uint8_t *in, size_t n, size_t burst,
                       size_t max_chunk, int termination, size_t read_size,
                       uint8_t *out, size_t cap, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    chunkencoder_t *ch = chunk_encode_2(async, blob_chain(async, in, n, burst),
                                        max_chunk,
                                        (chunkencoder_termination_t) termination);
    return run(async, chunkencoder_as_bytestream_1(ch), read_size, out, cap,
               err_out, NULL);
}

/* queuestream of `npieces` blobs (enqueued, or pushed in reverse order when
 * `push`), each behind nice(burst); terminated only after the first read
 * has answered EAGAIN, so the notify path is exercised.  No GPU. */
typedef struct {
    queuestream_t *q;
    int fired;
} late_terminate;

static void do_terminate(late_terminate *t)
{
    if (!t->fired) {
        t->fired = 1;
        queuestream_terminate(t->q);
    }
}

ssize_t h_queue_stream(const uint8_t *in, const size_t *lens, size_t npieces,
                       int push, size_t burst, size_t read_size, uint8_t *out,
                       size_t cap, int *err_out, size_t *eagains)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    queuestream_t *q = make_queuestream(async);
    size_t off = 0;
    const uint8_t **starts = malloc((npieces ? npieces : 1) * sizeof *starts);
    for (size_t i = 0; i < npieces; i++) {
        starts[i] = in + off;
        off += lens[i];
    }
    for (size_t k = 0; k < npieces; k++) {
        size_t i = push ? npieces - 1 - k : k;
        bytestream_1 s = blob_chain(async, starts[i], lens[i], burst);
        if (push)
            queuestream_push(q, s);
        else
            queuestream_enqueue(q, s);
    }
    free(starts);
    late_terminate *t = calloc(1, sizeof *t);
    t->q = q;
    async_timer_start(async, async_now(async) + 2000000, /* 2 ms */
                      (action_1) { t, (act_1) do_terminate });
    ssize_t r = run(async, queuestream_as_bytestream_1(q), read_size, out, cap,
                    err_out, eagains);
    free(t);
    return r;
}

/* `nmsg` independent egress stacks
 * queuestream(message) -> base64_encode (GPU) -> chunk_encode(max_chunk),
 * all on one loop, each drained `read_size` at a time into
 * out + out_off[i] (capacity out_off[i+1] - out_off[i]); out_len[i]
 * receives each framed length.  Returns 0, or -1 with *err_out. */
static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

int h_egress_stacks(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                    size_t max_chunk, size_t read_size, char pos62, char pos63,
                    int pad, char padchar, uint8_t *out, const uint64_t *out_off,
                    uint64_t *out_len, int *err_out, double *times)
{
    double t0 = now_s();
    async_t *async = make_async();
    if (!async)
        return -1;
    consumer *cs = calloc(nmsg ? nmsg : 1, sizeof *cs);
    size_t live = nmsg;
    for (size_t i = 0; i < nmsg; i++) {
        queuestream_t *q = make_queuestream(async);
        queuestream_enqueue_bytes(q, in + in_off[i], in_off[i + 1] - in_off[i]);
        queuestream_terminate(q);
        base64encoder_t *e = base64_encode(async, queuestream_as_bytestream_1(q),
                                           pos62, pos63, pad != 0, padchar);
        chunkencoder_t *ch = chunk_encode(async, base64encoder_as_bytestream_1(e),
                                          max_chunk);
        consumer *c = &cs[i];
        c->async = async;
        c->material = chunkencoder_as_bytestream_1(ch);
        c->read_size = read_size;
        c->out = out + out_off[i];
        c->cap = out_off[i + 1] - out_off[i];
        c->live = &live;
        action_1 cb = { c, (act_1) consume };
        bytestream_1_register_callback(c->material, cb);
        async_execute(async, cb);
    }
    double t1 = now_s();
    int rc = nmsg ? async_loop(async) : 0;
    int err = rc < 0 ? errno : 0;
    double t2 = now_s();
    if (times) {
        times[0] = t1 - t0; /* stack creation (queuestream copies) */
        times[1] = t2 - t1; /* the loop: pulls, GPU batches, framing, reads */
    }
    for (size_t i = 0; i < nmsg; i++) {
        out_len[i] = cs[i].len;
        if (!err && cs[i].err)
            err = cs[i].err;
        if (!cs[i].done && !err)
            err = EPIPE;
    }
    destroy_async(async);
    free(cs);
    if (err_out)
        *err_out = err;
    return err ? -1 : 0;
}

/* One egress stack over a queue of `npieces` messages copied in by
 * queuestream_enqueue_bytes() (or _push_bytes() in reverse order when
 * `push`: the same queue) -> base64_encode (GPU stage) -> chunk_encode.  With
 * `late`, the queue is terminated only after the first read has answered
 * EAGAIN (a timer, 2 ms), else at once.  Large messages are lent to the
 * encoder from their pinned copies (b64_pin.h); the framed stream equals
 * the oracle's for the concatenation whatever the mix. */
ssize_t h_egress_pieces(const uint8_t *in, const size_t *lens, size_t npieces, int push,
                        int late, size_t max_chunk, size_t read_size, uint8_t *out, size_t cap,
                        int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    queuestream_t *q = make_queuestream(async);
    size_t off = 0;
    const uint8_t **starts = malloc((npieces ? npieces : 1) * sizeof *starts);
    for (size_t i = 0; i < npieces; i++) {
        starts[i] = in + off;
        off += lens[i];
    }
    for (size_t k = 0; k < npieces; k++) {
        size_t i = push ? npieces - 1 - k : k;
        if (push)
            queuestream_push_bytes(q, starts[i], lens[i]);
        else
            queuestream_enqueue_bytes(q, starts[i], lens[i]);
    }
    free(starts);
    late_terminate *t = calloc(1, sizeof *t);
    t->q = q;
    if (late)
        async_timer_start(async, async_now(async) + 2000000, /* 2 ms */
                          (action_1) { t, (act_1) do_terminate });
    else
        queuestream_terminate(q);
    base64encoder_t *e = base64_encode(async, queuestream_as_bytestream_1(q), -1, -1, true, -1);
    chunkencoder_t *ch = chunk_encode(async, base64encoder_as_bytestream_1(e), max_chunk);
    ssize_t r = run(async, chunkencoder_as_bytestream_1(ch), read_size, out, cap, err_out, NULL);
    free(t);
    return r;
}

/* The ingress mirror of config 5: `nmsg` decoder stacks
 * queuestream(encoded message) -> base64_decode (GPU) on one loop, each
 * drained `read_size` at a time into out + out_off[i].  Short streams are
 * decoded as jobs of shared hub batches. */
int h_ingress_stacks(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                     size_t read_size, char pos62, char pos63, uint8_t *out,
                     const uint64_t *out_off, uint64_t *out_len, int *err_out,
                     double *times)
{
    double t0 = now_s();
    async_t *async = make_async();
    if (!async)
        return -1;
    consumer *cs = calloc(nmsg ? nmsg : 1, sizeof *cs);
    size_t live = nmsg;
    for (size_t i = 0; i < nmsg; i++) {
        queuestream_t *q = make_queuestream(async);
        queuestream_enqueue_bytes(q, in + in_off[i], in_off[i + 1] - in_off[i]);
        queuestream_terminate(q);
        base64decoder_t *d =
            base64_decode(async, queuestream_as_bytestream_1(q), pos62, pos63);
        consumer *c = &cs[i];
        c->async = async;
        c->material = base64decoder_as_bytestream_1(d);
        c->read_size = read_size;
        c->out = out + out_off[i];
        c->cap = out_off[i + 1] - out_off[i];
        c->live = &live;
        action_1 cb = { c, (act_1) consume };
        bytestream_1_register_callback(c->material, cb);
        async_execute(async, cb);
    }
    double t1 = now_s();
    int rc = nmsg ? async_loop(async) : 0;
    int err = rc < 0 ? errno : 0;
    double t2 = now_s();
    if (times) {
        times[0] = t1 - t0;
        times[1] = t2 - t1;
    }
    for (size_t i = 0; i < nmsg; i++) {
        out_len[i] = cs[i].len;
        if (!err && cs[i].err)
            err = cs[i].err;
        if (!cs[i].done && !err)
            err = EPIPE;
    }
    destroy_async(async);
    free(cs);
    if (err_out)
        *err_out = err;
    return err ? -1 : 0;
}

/* Config 5 over `nthreads` event loops (one per thread, each with its own
 * hub): messages are split into contiguous ranges of about equal bytes.
 * times[0] = slowest thread's setup, times[1] = wall time of the loops. */
typedef struct {
    const uint8_t *in;
    const uint64_t *in_off;
    size_t first, count, max_chunk, read_size;
    char pos62, pos63, padchar;
    int pad;
    uint8_t *out;
    const uint64_t *out_off;
    uint64_t *out_len;
    int err;
    double times[2];
    int device;  /* -1: the calling thread's current device */
} egress_share;

/* HIP runtime entry points (C linkage; hipError_t is an int-sized enum):
 * the threaded driver can put each event loop on its own GPU. */
extern int hipSetDevice(int device);
extern int hipGetDeviceCount(int *count);

int h_device_count(void)
{
    int n = 0;
    return hipGetDeviceCount(&n) == 0 ? n : 0;
}

static void *egress_thread(void *arg)
{
    egress_share *e = arg;
    size_t f = e->first;
    if (e->device >= 0 && hipSetDevice(e->device) != 0) {
        e->err = ENODEV;
        return NULL;
    }
    /* out pointers are absolute; shift offsets to this share */
    e->err = 0;
    if (h_egress_stacks(e->in, e->in_off + f, e->count, e->max_chunk, e->read_size,
                        e->pos62, e->pos63, e->pad, e->padchar, e->out,
                        e->out_off + f, e->out_len + f, &e->err, e->times) < 0 &&
        !e->err)
        e->err = EIO;
    return NULL;
}

#include <pthread.h>

/* Config 5 over `nthreads` event loops; with ndevices > 1 loop t runs on
 * GPU t mod ndevices (every stage of a loop uses its loop's GPU). */
int h_egress_stacks_mt_dev(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                           size_t max_chunk, size_t read_size, char pos62, char pos63,
                           int pad, char padchar, uint8_t *out, const uint64_t *out_off,
                           uint64_t *out_len, int *err_out, double *times,
                           size_t nthreads, int ndevices);

int h_egress_stacks_mt(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                       size_t max_chunk, size_t read_size, char pos62, char pos63,
                       int pad, char padchar, uint8_t *out, const uint64_t *out_off,
                       uint64_t *out_len, int *err_out, double *times,
                       size_t nthreads)
{
    return h_egress_stacks_mt_dev(in, in_off, nmsg, max_chunk, read_size, pos62, pos63, pad,
                                  padchar, out, out_off, out_len, err_out, times, nthreads, 1);
}

static int egress_mt(const uint8_t *in, const uint64_t *in_off, size_t nmsg, size_t max_chunk,
                     size_t read_size, char pos62, char pos63, int pad, char padchar,
                     uint8_t *out, const uint64_t *out_off, uint64_t *out_len, int *err_out,
                     double *times, size_t nthreads, int ndevices, int device);

int h_egress_stacks_mt_dev(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                           size_t max_chunk, size_t read_size, char pos62, char pos63,
                           int pad, char padchar, uint8_t *out, const uint64_t *out_off,
                           uint64_t *out_len, int *err_out, double *times,
                           size_t nthreads, int ndevices)
{
    return egress_mt(in, in_off, nmsg, max_chunk, read_size, pos62, pos63, pad, padchar, out,
                     out_off, out_len, err_out, times, nthreads, ndevices, -1);
}

/* Every loop on GPU `device` (a rank of a multi-GPU run: threads start on
 * device 0, whatever the process's main thread selected). */
int h_egress_stacks_mt_on(const uint8_t *in, const uint64_t *in_off, size_t nmsg,
                          size_t max_chunk, size_t read_size, char pos62, char pos63,
                          int pad, char padchar, uint8_t *out, const uint64_t *out_off,
                          uint64_t *out_len, int *err_out, double *times, size_t nthreads,
                          int device)
{
    return egress_mt(in, in_off, nmsg, max_chunk, read_size, pos62, pos63, pad, padchar, out,
                     out_off, out_len, err_out, times, nthreads, 1, device);
}

static int egress_mt(const uint8_t *in, const uint64_t *in_off, size_t nmsg, size_t max_chunk,
                     size_t read_size, char pos62, char pos63, int pad, char padchar,
                     uint8_t *out, const uint64_t *out_off, uint64_t *out_len, int *err_out,
                     double *times, size_t nthreads, int ndevices, int device)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > nmsg)
        nthreads = nmsg ? nmsg : 1;
    egress_share *sh = calloc(nthreads, sizeof *sh);
    pthread_t *th = calloc(nthreads, sizeof *th);
    uint64_t total = in_off[nmsg];
    size_t first = 0;
    for (size_t t = 0; t < nthreads; t++) {
        uint64_t goal = total / nthreads * (t + 1);
        size_t last = first;
        if (t + 1 == nthreads)
            last = nmsg;
        else
            while (last < nmsg && in_off[last] < goal)
                last++;
        sh[t] = (egress_share) { in, in_off, first, last - first, max_chunk, read_size,
                                 pos62, pos63, padchar, pad, out, out_off, out_len, 0,
                                 { 0, 0 }, -1 };
        if (ndevices > 1) {  /* loop t on GPU t mod ndevices (mod what exists) */
            const int have = h_device_count();
            sh[t].device = have > 0 ? (int) (t % (size_t) ndevices) % have : 0;
        } else if (device >= 0) {
            sh[t].device = device;
        }
        first = last;
    }
    double t0 = now_s();
    for (size_t t = 0; t < nthreads; t++)
        pthread_create(&th[t], NULL, egress_thread, &sh[t]);
    int err = 0;
    double setup = 0;
    for (size_t t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (!err && sh[t].err)
            err = sh[t].err;
        if (sh[t].times[0] > setup)
            setup = sh[t].times[0];
    }
    double t1 = now_s();
    if (times) {
        times[0] = setup;
        times[1] = t1 - t0 - setup;
    }
    free(sh);
    free(th);
    if (err_out)
        *err_out = err;
    return err ? -1 : 0;
}

/* ---- the fd ends of the path: pipe/socket -> decoder, encoder -> pipe ---
 * (bench.py `host_fd`, tests/test_fd_*.py).  A
 * writer (ingress) or reader (egress) thread sits on the other end of a
 * pipe or an AF_UNIX socketpair, doing blocking write(2)/read(2), as a
 * peer process would; the product's loop does the rest. */
#include <fcntl.h>
#include <sys/socket.h>

static int make_channel(int fds[2], int sock)
{
    if (sock) {
        if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, fds) < 0)
            return -1;
        int sz = 4 << 20;
        (void) setsockopt(fds[0], SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
        (void) setsockopt(fds[1], SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
        return 0;
    }
    if (pipe2(fds, O_CLOEXEC) < 0)
        return -1;
    (void) fcntl(fds[1], F_SETPIPE_SZ, 1 << 20); /* the default pipe-max-size */
    return 0;
}

typedef struct {
    int fd;
    const uint8_t *data;
    size_t n, chunk;
    uint8_t *out;
    size_t cap, got;
    int err;
    double t_end;
} peer;

static void *peer_writer(void *arg)
{
    peer *p = arg;
    size_t off = 0;
    while (off < p->n) {
        size_t k = p->n - off < p->chunk ? p->n - off : p->chunk;
        ssize_t w = write(p->fd, p->data + off, k);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            p->err = errno;
            break;
        }
        off += (size_t) w;
    }
    close(p->fd);
    return NULL;
}

static void *peer_reader(void *arg)
{
    peer *p = arg;
    for (;;) {
        size_t room = p->cap - p->got;
        if (!room) { /* overlong: drain and flag */
            uint8_t sink[4096];
            ssize_t r = read(p->fd, sink, sizeof sink);
            if (r > 0) {
                p->err = ENOSPC;
                continue;
            }
            break;
        }
        ssize_t r = read(p->fd, p->out + p->got, room);
        if (r < 0) {
            if (errno == EINTR)
                continue;
            p->err = errno;
            break;
        }
        if (r == 0)
            break;
        p->got += (size_t) r;
    }
    p->t_end = now_s();
    close(p->fd);
    return NULL;
}

/* Ingress: `chars` written into a pipe (or socketpair) by a peer thread in
 * `write_chunk` pieces -> pipestream -> base64_decode (GPU stage) ->
 * consumer reading `read_size` at a time into out.  times[0] = wall time
 * from the first byte written to the consumer's EOF.  Returns the decoded
 * length or -1 + *err_out. */
ssize_t h_fd_decode(const uint8_t *chars, size_t n, size_t write_chunk, size_t read_size,
                    char pos62, char pos63, uint8_t *out, size_t cap, int sock,
                    int *err_out, double *times)
{
    int fds[2];
    if (make_channel(fds, sock) < 0) {
        if (err_out)
            *err_out = errno;
        return -1;
    }
    async_t *async = make_async();
    if (!async) {
        close(fds[0]);
        close(fds[1]);
        return -1;
    }
    pipestream_t *ps = open_pipestream(async, fds[0]);
    base64decoder_t *dec = base64_decode(async, pipestream_as_bytestream_1(ps), pos62, pos63);
    peer w = { fds[1], chars, n, write_chunk ? write_chunk : (1 << 20), NULL, 0, 0, 0, 0 };
    pthread_t th;
    double t0 = now_s();
    pthread_create(&th, NULL, peer_writer, &w);
    ssize_t r = run(async, base64decoder_as_bytestream_1(dec), read_size, out, cap, err_out,
                    NULL);
    double t1 = now_s();
    pthread_join(th, NULL);
    if (times)
        times[0] = t1 - t0;
    if (r >= 0 && w.err) {
        if (err_out)
            *err_out = w.err;
        return -1;
    }
    return r;
}

/* The channel alone (calibration for h_fd_decode): the same peer writer,
 * and this thread reading the bytes with blocking read(2)s of read_size
 * straight into out -- the least any consumer of the fd does. */
ssize_t h_fd_raw(const uint8_t *data, size_t n, size_t write_chunk, size_t read_size,
                 uint8_t *out, size_t cap, int sock, int *err_out, double *times)
{
    int fds[2];
    if (make_channel(fds, sock) < 0) {
        if (err_out)
            *err_out = errno;
        return -1;
    }
    peer w = { fds[1], data, n, write_chunk ? write_chunk : (1 << 20), NULL, 0, 0, 0, 0 };
    pthread_t th;
    double t0 = now_s();
    pthread_create(&th, NULL, peer_writer, &w);
    size_t got = 0;
    int err = 0;
    for (;;) {
        size_t k = cap - got < read_size ? cap - got : read_size;
        if (!k) {
            err = ENOSPC;
            break;
        }
        ssize_t r = read(fds[0], out + got, k);
        if (r < 0) {
            if (errno == EINTR)
                continue;
            err = errno;
            break;
        }
        if (r == 0)
            break;
        got += (size_t) r;
    }
    double t1 = now_s();
    close(fds[0]);
    pthread_join(th, NULL);
    if (times)
        times[0] = t1 - t0;
    if (!err)
        err = w.err;
    if (err_out)
        *err_out = err;
    return err ? -1 : (ssize_t) got;
}

typedef struct {
    async_t *async;
    fdsink_t *sink;
} sink_watch;

static void sink_finished(sink_watch *sw)
{
    async_quit_loop(sw->async);
}

/* Egress: the `npieces` pieces of `in` (lens[i] bytes each) as blobstreams
 * on one terminated queuestream -> base64_encode (GPU stage) ->
 * chunk_encode(max_chunk) -> fdsink (10,240-byte pulls, write(2)) into a
 * pipe (or socketpair) that a peer thread reads into out.  max_chunk 0:
 * no framing, the sink reads the encoder itself (its copying path).  times[0] = wall
 * time from the loop's start to the peer's EOF.  Returns the framed length
 * or -1 + *err_out. */
ssize_t h_fd_encode(const uint8_t *in, const size_t *lens, size_t npieces, size_t max_chunk,
                    char pos62, char pos63, int pad, char padchar, uint8_t *out, size_t cap,
                    int sock, int *err_out, double *times)
{
    int fds[2];
    if (make_channel(fds, sock) < 0) {
        if (err_out)
            *err_out = errno;
        return -1;
    }
    async_t *async = make_async();
    if (!async) {
        close(fds[0]);
        close(fds[1]);
        return -1;
    }
    queuestream_t *q = make_queuestream(async);
    size_t off = 0;
    for (size_t i = 0; i < npieces; i++) {
        queuestream_enqueue(q, blobstream_as_bytestream_1(open_blobstream(async, in + off,
                                                                          lens[i])));
        off += lens[i];
    }
    queuestream_terminate(q);
    base64encoder_t *e = base64_encode(async, queuestream_as_bytestream_1(q), pos62, pos63,
                                       pad != 0, padchar);
    bytestream_1 src = base64encoder_as_bytestream_1(e);
    if (max_chunk)
        src = chunkencoder_as_bytestream_1(chunk_encode(async, src, max_chunk));
    peer rd = { fds[0], NULL, 0, 0, out, cap, 0, 0, 0 };
    pthread_t th;
    double t0 = now_s();
    pthread_create(&th, NULL, peer_reader, &rd);
    sink_watch sw = { async, NULL };
    sw.sink = open_fdsink(async, src, fds[1]);
    fdsink_register_callback(sw.sink, (action_1) { &sw, (act_1) sink_finished });
    int rc = fdsink_done(sw.sink) ? 0 : async_loop(async);
    int err = rc < 0 ? errno : fdsink_error(sw.sink);
    uint64_t written = fdsink_bytes(sw.sink);
    fdsink_close(sw.sink);
    pthread_join(th, NULL);
    if (times)
        times[0] = rd.t_end - t0;
    destroy_async(async);
    if (!err && rd.err)
        err = rd.err;
    if (!err && written != rd.got)
        err = EPIPE;
    if (err_out)
        *err_out = err;
    return err ? -1 : (ssize_t) rd.got;
}

/* fdsink over a descriptor the loop cannot watch (-1, a regular file):
 * the sink ends with the error and a callback registered after
 * open_fdsink() returned is still performed.  Returns 1 if the
 * callback ran (0 if the watchdog ended the loop); *err_out the sink's
 * errno. */
typedef struct {
    async_t *async;
    int fired;
} sink_flag;

static void sink_flag_fire(sink_flag *f)
{
    f->fired = 1;
    async_quit_loop(f->async);
}

static void sink_flag_dog(sink_flag *f)
{
    async_quit_loop(f->async);
}

int h_fdsink_unwatchable(int fd, int *err_out)
{
    async_t *async = make_async();
    if (!async)
        return -1;
    static const uint8_t msg[] = "aGVsbG8=";
    bytestream_1 src = blobstream_as_bytestream_1(open_blobstream(async, msg, sizeof msg - 1));
    sink_flag f = { async, 0 };
    fdsink_t *sink = open_fdsink(async, src, fd);
    fdsink_register_callback(sink, (action_1) { &f, (act_1) sink_flag_fire });
    async_timer_t *dog = async_timer_start(async, async_now(async) + 5 * (uint64_t) ASYNC_S,
                                           (action_1) { &f, (act_1) sink_flag_dog });
    (void) async_loop(async);
    if (f.fired)
        async_timer_cancel(async, dog);
    if (err_out)
        *err_out = fdsink_error(sink);
    fdsink_close(sink);
    destroy_async(async);
    return f.fired;
}

/* ---- a crash report: the faulting thread's native stack ------------------
 * (Python's faulthandler shows Python frames only.)  Printed to stderr,
 * then the previous handler runs. */
#include <execinfo.h>
#include <signal.h>

static struct sigaction prev_segv;

static void segv_report(int sig, siginfo_t *si, void *uc)
{
    void *frames[64];
    int n = backtrace(frames, 64);
    static const char msg[] = "\nstage_harness: native stack of the faulting thread:\n";
    ssize_t w = write(2, msg, sizeof msg - 1);
    char line[96];
    int len = snprintf(line, sizeof line, "fault address %p, frames %d\n", si->si_addr, n);
    w = write(2, line, (size_t) len);
    (void) w;
    backtrace_symbols_fd(frames, n, 2);
    sigaction(SIGSEGV, &prev_segv, NULL);
    if (prev_segv.sa_flags & SA_SIGINFO) {
        if (prev_segv.sa_sigaction)
            prev_segv.sa_sigaction(sig, si, uc);
    } else if (prev_segv.sa_handler != SIG_DFL && prev_segv.sa_handler != SIG_IGN) {
        prev_segv.sa_handler(sig);
    }
    raise(sig);
}

void h_segv_install(void);
__attribute__((constructor)) void h_segv_install(void)
{
    /* an alternate stack (this thread's): a stack overflow still reports */
    static char altstack[1 << 16];
    stack_t ss = { .ss_sp = altstack, .ss_size = sizeof altstack, .ss_flags = 0 };
    sigaltstack(&ss, NULL);
    struct sigaction cur;
    sigaction(SIGSEGV, NULL, &cur);
    if ((cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == segv_report)
        return; /* ours already */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = segv_report;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &prev_segv);
}

/* ---- a small sampling profiler (SIGPROF, process CPU time) ---------------
 * h_prof_start(hz) / h_prof_stop(path): a histogram of interrupted program
 * counters, resolved with dladdr to "object symbol+offset", written as
 * "count symbol" lines (test infrastructure: host-side profiles of the loop
 * without perf, which the GPU image lacks). */
#include <dlfcn.h>
#include <signal.h>
#include <stdatomic.h>
#include <sys/time.h>
#include <ucontext.h>

enum { PROF_MAX = 1 << 20 };
static uintptr_t *prof_pc;
static atomic_size_t prof_n;

static void prof_handler(int sig, siginfo_t *si, void *uc_)
{
    (void) sig;
    (void) si;
    ucontext_t *uc = uc_;
    size_t i = atomic_fetch_add_explicit(&prof_n, 1, memory_order_relaxed);
    if (i < PROF_MAX)
        prof_pc[i] = (uintptr_t) uc->uc_mcontext.gregs[REG_RIP];
}

int h_prof_start(int hz)
{
    if (!prof_pc && !(prof_pc = malloc(PROF_MAX * sizeof *prof_pc)))
        return -1;
    atomic_store(&prof_n, 0);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = prof_handler;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGPROF, &sa, NULL) < 0)
        return -1;
    struct itimerval it = { { 0, 1000000 / hz }, { 0, 1000000 / hz } };
    return setitimer(ITIMER_PROF, &it, NULL);
}

static int cmp_uptr(const void *a, const void *b)
{
    uintptr_t x = *(const uintptr_t *) a, y = *(const uintptr_t *) b;
    return x < y ? -1 : x > y;
}

int h_prof_stop(const char *path)
{
    struct itimerval it;
    memset(&it, 0, sizeof it);
    setitimer(ITIMER_PROF, &it, NULL);
    signal(SIGPROF, SIG_IGN);
    size_t n = atomic_load(&prof_n);
    if (n > PROF_MAX)
        n = PROF_MAX;
    /* map each pc to its symbol start, then count per symbol */
    for (size_t i = 0; i < n; i++) {
        Dl_info d;
        if (dladdr((void *) prof_pc[i], &d) && d.dli_saddr && d.dli_sname)
            prof_pc[i] = (uintptr_t) d.dli_saddr;
    }
    qsort(prof_pc, n, sizeof *prof_pc, cmp_uptr);
    FILE *f = fopen(path, "w");
    if (!f)
        return -1;
    fprintf(f, "%zu samples\n", n);
    for (size_t i = 0; i < n;) {
        size_t j = i;
        while (j < n && prof_pc[j] == prof_pc[i])
            j++;
        Dl_info d;
        const char *sym = "?", *obj = "?";
        uintptr_t off = prof_pc[i];
        if (dladdr((void *) prof_pc[i], &d)) {
            if (d.dli_sname)
                sym = d.dli_sname;
            if (d.dli_fname)
                obj = d.dli_fname;
            off -= (uintptr_t) d.dli_fbase;
        }
        /* object-relative offset: scripts/prof_resolve.py names the
         * static functions with nm */
        fprintf(f, "%zu %s %s %#lx\n", j - i, obj, sym, (unsigned long) off);
        i = j;
    }
    fclose(f);
    return 0;
}
