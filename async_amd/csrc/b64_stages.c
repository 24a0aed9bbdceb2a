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
 *   GPU completion: a HIP host function marks the slot finished and posts
 *   the stage on the loop's hub, whose one eventfd is registered with
 *   async_register(), so the loop calls the stage, which calls the
 *   consumer's registered
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
 * The byte stream each stage produces is the reference's, byte for byte,
 * and the encoder's per-read counts are too whenever upstream keeps up
 * (see stage_read()); while blocks are on the GPU a read returns -1/EAGAIN
 * (a consumer written for the reference already handles EAGAIN from any
 * stream).  Upstream errors are passed through with all state kept when
 * nothing is in flight; count == 0 returns 0 (ref :103-104, :54-55).  The
 * reference's assert at src/base64encoder.c:140 (counts not divisible by
 * 4) has no counterpart.  With no usable GPU the first read fails with
 * ENODEV: there is no CPU path.
 *
 * Tuning (environment, read when a stage is created):
 *   ASYNC_B64_STAGE_CAPACITY  staging bytes per slot (default 1 MiB; the
 *                             encoder grows it to hold its first read's
 *                             count, up to ASYNC_B64_STAGE_MAX_CAPACITY,
 *                             default 64 MiB)
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
#include <unistd.h>

#include "async.h"
#include "b64_hub.h"
#include "b64_lend.h"
#include "b64x.h"
#include "base64decoder.h"
#include "base64encoder.h"

enum { NSLOTS = 4 }; /* blocks in flight or staged per stage (read-ahead) */

typedef struct stage stage;

typedef struct {
    stage *owner;
    b64x_session *sess; /* decoder: this slot's session */
    b64_ticket ticket;  /* encoder, and a short decoder stream: this slot's
                           job in a hub batch */
    bool hubbed;        /* decoder: the slot's block went through the hub */
    atomic_int done;    /* decoder: set by the HIP host function */
    bool resolved;    /* out_len/body_end valid (decoder: after done) */
    size_t out_pos;
    size_t body_end;  /* encoder: end of the full sextets; the finalize
                         characters after it are served on their own */
    size_t out_len;
} slot;

typedef enum { DIR_ENCODE, DIR_DECODE } direction;

struct stage {
    async_t *async;
    bytestream_1 up;
    action_1 cb;        /* the consumer's callback, or NULL_ACTION_1 */
    direction dir;
    b64x_alphabet abc;
    size_t cap, min_pull, max_cap;
    b64_hub *hub;       /* the loop's batching hub */
    bool hub_first;     /* decoder: the first block may go through the hub
                           (a stream that ends inside it is one job) */
    atomic_bool wake_posted; /* decoder: a session completion is queued
                                on the hub for this stage */
    unsigned hub_waits; /* entries on the hub's waiter list (room for a block) */
    bool started;       /* the hub (and any sessions) are held */
    int err;            /* sticky failure errno, 0 while healthy */
    slot slots[NSLOTS];
    unsigned head;      /* oldest busy slot */
    unsigned nbusy;     /* launched, output not fully served */
    bool final_queued;  /* the last block (or nothing) has been launched */
    bool launched_any;
    bool short_seen;    /* an upstream read came up short (not EAGAIN)
                           since the staged output last ran out */
    uint8_t carry[2];   /* encoder: bytes of the incomplete group */
    size_t ncarry;
    bool lend_want;     /* this read may lend instead of copy (b64_lend.h) */
    uint8_t *spill;     /* lent copy of reads that span blocks (no fallback) */
    size_t spill_cap;
    const uint8_t *lent;/* what the last read lent, until returned */
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
    st->max_cap = env_size("ASYNC_B64_STAGE_MAX_CAPACITY", (size_t) 64 << 20, 64);
    for (int i = 0; i < NSLOTS; i++)
        st->slots[i].owner = st;
}

static ssize_t stage_fail(stage *st, int negerr)
{
    st->err = negerr < 0 ? -negerr : EIO;
    errno = st->err;
    return -1;
}

/* The hub has room again: this stage is off its waiter list. */
static void stage_kicked(stage *st)
{
    if (st->hub_waits)
        st->hub_waits--;
    action_1_perf(st->cb);
}

/* Loop side of a session completion (posted through the loop's hub: one
 * eventfd per loop, not one per stage -- thousands of decoder streams
 * would otherwise hold a descriptor each). */
static void stage_posted(stage *st)
{
    atomic_store_explicit(&st->wake_posted, false, memory_order_relaxed);
    action_1_perf(st->cb);
}

/* HIP runtime thread: publish, then signal (once until the loop runs it). */
static void slot_done(void *arg)
{
    slot *sl = arg;
    stage *st = sl->owner;
    atomic_store_explicit(&sl->done, 1, memory_order_release);
    if (!atomic_exchange_explicit(&st->wake_posted, true, memory_order_acq_rel))
        b64_hub_post(st->hub, (action_1) { st, (act_1) stage_posted });
}

/* Hub completion of one of this stage's blocks (on the loop). */
static void stage_notify(stage *st)
{
    action_1_perf(st->cb);
}

static int stage_start(stage *st, size_t count)
{
    if (st->started)
        return 0;
    if (st->dir == DIR_ENCODE) {
        /* A fresh block must be able to hold a full read (see
         * stage_read()); blocks go to the loop's hub. */
        size_t need = (count + 3) / 4 * 3 + 3;
        if (need > st->max_cap)
            need = st->max_cap;
        if (need > st->cap)
            st->cap = need;
        int rc = b64x_device_check(); /* fail loudly: no CPU path */
        if (rc)
            return rc;
        st->hub = b64_hub_acquire(st->async);
        if (!st->hub)
            return -(errno ? errno : ENODEV);
        st->started = true;
        return 0;
    }
    /* A stream that ends inside its first block is decoded as one job of
     * a hub batch (many short streams, one launch); longer streams take
     * sessions, from the process-wide pool as slots are first used, whose
     * completions come back through the hub's eventfd too (a descriptor
     * per stage would cap a loop at ~1,000 decoder streams and cost
     * fd-table expansions). */
    int rc = b64x_device_check(); /* fail loudly: no CPU path */
    if (rc)
        return rc;
    st->hub = b64_hub_acquire(st->async);
    if (!st->hub)
        return -(errno ? errno : ENODEV);
    st->hub_first = true;
    st->started = true;
    return 0;
}

static void stage_stop(stage *st)
{
    /* sessions first: a release waits for the session's work, so no
     * completion can be posted for this stage after the forget below */
    for (int i = 0; i < NSLOTS; i++) {
        if (st->slots[i].sess) {
            b64x_session_release(st->slots[i].sess); /* waits, then pools */
            st->slots[i].sess = NULL;
        }
    }
    if (st->hub) {
        b64_hub_forget(st->hub, st, st->hub_waits > 0);
        for (int i = 0; i < NSLOTS; i++)
            b64_ticket_release(&st->slots[i].ticket);
        b64_hub_release(st->hub);
        st->hub = NULL;
    }
    st->started = false;
}

/* Pull from upstream into dst until at least min_pull bytes have come
 * in, or EOF, EAGAIN or an error; after a short read it asks once more,
 * so the EOF of a finite upstream lands in the same block.  Returns bytes
 * gathered; *eof / *err report why it stopped. */
static size_t gather(stage *st, uint8_t *dst, size_t room, bool *eof,
                     int *err)
{
    size_t got = 0;
    size_t want = st->min_pull < room ? st->min_pull : room;
    *eof = false;
    *err = 0;
    while (got < room) {
        size_t ask = room - got;
        ssize_t n = bytestream_1_read(st->up, dst + got, ask);
        if (n < 0) {
            *err = errno ? errno : EIO;
            break;
        }
        if (n == 0) {
            *eof = true;
            break;
        }
        got += (size_t) n;
        if ((size_t) n < ask)
            st->short_seen = true;
        else if (got >= want)
            break;
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
    sl->resolved = false;
    sl->out_pos = sl->body_end = sl->out_len = 0;
    st->nbusy++;
}

/* Characters finalize() emits for a last block of n bytes: the partial
 * sextet plus padding (ref base64encoder.c:61-99). */
static size_t finalize_len(size_t n, bool pad)
{
    switch (n % 3) {
        case 1:
            return pad ? 3 : 1;
        case 2:
            return pad ? 2 : 1;
        default:
            return 0;
    }
}

/* Launch as many blocks as slots and upstream allow.  Returns 0, or a
 * positive errno from upstream (EAGAIN included) that stopped it, or a
 * negative errno from the GPU side. */
static int top_up_encoder(stage *st)
{
    slot *sl;
    while ((sl = next_launch_slot(st))) {
        /* Room in the hub's open arena: up to a full slot, but a few KiB
         * will do (the next block gets a fresh arena and a full slot, so
         * two slots always cover a full read). */
        size_t room;
        /* Backpressure: a stage may be made to wait for an arena unless
         * it holds finished output that cannot be served without more
         * input (it must make progress, or arenas could stay pinned by
         * partially read jobs forever). */
        bool must_progress = st->nbusy > 0;
        for (unsigned i = 0; i < st->nbusy && must_progress; i++)
            if (!atomic_load_explicit(&st->slots[(st->head + i) % NSLOTS].ticket.done,
                                      memory_order_acquire))
                must_progress = false; /* a completion will wake us */
        action_1 waiter = { NULL, NULL };
        if (!must_progress)
            waiter = (action_1) { st, (act_1) stage_kicked };
        uint8_t *in = b64_hub_reserve(st->hub, B64_HUB_ENCODE, &st->abc, st->cap,
                                      st->ncarry + 4096, &room, waiter);
        if (!in) {
            if (errno == EAGAIN && waiter.act)
                st->hub_waits++;
            return errno == EAGAIN ? EAGAIN : -(errno ? errno : ENOMEM);
        }
        memcpy(in, st->carry, st->ncarry);
        bool eof;
        int uerr;
        size_t got = gather(st, in + st->ncarry, room - st->ncarry, &eof,
                            &uerr);
        size_t total = st->ncarry + got;
        /* The block encodes all `total` bytes.  Its full sextets,
         * floor(8*total/6) characters, are served now -- the reference
         * emits them in the read that brought the bytes in
         * (base64encoder.c:132-139).  The 0-2 bytes of a trailing partial
         * group are carried: the next block re-encodes them and skips the
         * characters (one per carried byte) already served from this one. */
        size_t skip = st->ncarry;
        if (eof) {
            st->final_queued = true;
            st->ncarry = 0;
            if (total == 0) {
                b64_hub_cancel(st->hub);
                return 0;
            }
        } else {
            if (got == 0) {
                b64_hub_cancel(st->hub);
                return uerr ? uerr : EAGAIN;
            }
            st->ncarry = total % 3;
            memcpy(st->carry, in + total - st->ncarry, st->ncarry);
        }
        slot_arm(st, sl);
        sl->out_len = (size_t) b64x_encoded_len(total, st->abc.pad);
        b64_hub_commit(st->hub, &sl->ticket, total, sl->out_len,
                       (action_1) { st, (act_1) stage_notify });
        sl->out_pos = skip;
        sl->body_end = total * 8 / 6;
        if (eof) /* finalize(): the partial sextet and the pads */
            sl->body_end = sl->out_len - finalize_len(total, st->abc.pad);
        else
            sl->out_len = sl->body_end; /* the rest is re-encoded later */
        sl->resolved = true;
        if (uerr)
            return uerr;
    }
    return 0;
}

/* The first block of a decoder stream through the hub: a stream that
 * ends inside it is one job (its final partial group emitted, like the
 * reference at EOF); one that does not moves what was gathered into a
 * session and continues on sessions.  Returns as top_up does, or 1 when
 * the caller should launch `*moved` bytes already in sl's session. */
static int decoder_first_via_hub(stage *st, slot *sl, size_t *moved)
{
    *moved = 0;
    action_1 waiter = { st, (act_1) stage_kicked };
    size_t room;
    uint8_t *in = b64_hub_reserve(st->hub, B64_HUB_DECODE, &st->abc, st->cap, 4096, &room,
                                  waiter);
    if (!in) {
        if (errno == EAGAIN)
            st->hub_waits++;
        return errno == EAGAIN ? EAGAIN : -(errno ? errno : ENOMEM);
    }
    bool eof;
    int uerr;
    size_t got = gather(st, in, room, &eof, &uerr);
    if (eof) {
        st->final_queued = true;
        st->hub_first = false;
        if (got == 0) {
            b64_hub_cancel(st->hub);
            return 0;
        }
        slot_arm(st, sl);
        sl->hubbed = true;
        b64_hub_commit(st->hub, &sl->ticket, got, (got + 3) / 4 * 3,
                       (action_1) { st, (act_1) stage_notify });
        st->launched_any = true;
        return 0;
    }
    if (got == 0) {
        b64_hub_cancel(st->hub);
        return uerr ? uerr : EAGAIN;
    }
    /* more than a block, or upstream paused: the session path from here */
    st->hub_first = false;
    if (!sl->sess && !(sl->sess = b64x_session_acquire(st->cap))) {
        b64_hub_cancel(st->hub);
        return -(errno ? errno : ENOMEM);
    }
    memcpy(b64x_session_host_in(sl->sess), in, got);
    b64_hub_cancel(st->hub);
    *moved = got;
    return 1;
}

static int top_up_decoder(stage *st)
{
    slot *sl;
    while ((sl = next_launch_slot(st))) {
        size_t moved = 0;
        if (st->hub_first && !st->launched_any) {
            int rc = decoder_first_via_hub(st, sl, &moved);
            if (rc != 1) {
                if (rc)
                    return rc;
                continue;
            }
        }
        slot *prev = st->launched_any
                         ? &st->slots[(st->head + st->nbusy + NSLOTS - 1) %
                                      NSLOTS]
                         : NULL;
        if (!sl->sess) {
            sl->sess = b64x_session_acquire(st->cap);
            if (!sl->sess)
                return -(errno ? errno : ENOMEM);
        }
        bool eof = false;
        int uerr = 0;
        size_t got = moved;
        if (!moved)
            got = gather(st, b64x_session_host_in(sl->sess), st->cap, &eof, &uerr);
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
        sl->hubbed = false;
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

static int top_up(stage *st)
{
    return st->dir == DIR_ENCODE ? top_up_encoder(st) : top_up_decoder(st);
}

/* A finished slot's lengths (the decoder's are device-determined). */
static bool slot_ready(slot *sl)
{
    if (sl->owner->dir == DIR_ENCODE)
        return atomic_load_explicit(&sl->ticket.done, memory_order_acquire);
    if (sl->hubbed) {
        if (!atomic_load_explicit(&sl->ticket.done, memory_order_acquire))
            return false;
        if (!sl->resolved) {
            sl->out_len = sl->ticket.out_len;
            sl->body_end = sl->out_len;
            sl->resolved = true;
        }
        return true;
    }
    if (!atomic_load_explicit(&sl->done, memory_order_acquire))
        return false;
    if (!sl->resolved) {
        sl->out_len = (size_t) b64x_session_result(sl->sess)->out_len;
        sl->body_end = sl->out_len;
        sl->resolved = true;
    }
    return true;
}

static const uint8_t *slot_out(slot *sl)
{
    return sl->owner->dir == DIR_ENCODE || sl->hubbed ? sl->ticket.out
                                                      : b64x_session_host_out(sl->sess);
}

static void retire_head(stage *st)
{
    b64_ticket_release(&st->slots[st->head].ticket);
    st->nbusy--;
    st->head = (st->head + 1) % NSLOTS;
}

/* Finished body characters from the head on, in order; *blocked is set
 * when a slot still in flight ends the run. */
static size_t staged_body(stage *st, bool *blocked)
{
    size_t total = 0;
    *blocked = false;
    for (unsigned i = 0; i < st->nbusy; i++) {
        slot *sl = &st->slots[(st->head + i) % NSLOTS];
        if (!slot_ready(sl)) {
            *blocked = true;
            break;
        }
        total += sl->body_end - sl->out_pos;
        if (sl->body_end < sl->out_len)
            break; /* finalize characters: a read of their own */
    }
    return total;
}

static size_t serve_body(stage *st, uint8_t *dst, size_t n)
{
    slot *h = &st->slots[st->head];
    if (st->lend_want && st->nbusy && h->body_end - h->out_pos >= n) {
        /* all n in the head block: lend them; the slot stays busy (and its
         * arena held) until the bytes are returned */
        st->lent = slot_out(h) + h->out_pos;
        h->out_pos += n;
        return n;
    }
    uint8_t *spill = NULL;
    if (!dst) { /* a lending read without a fallback: the stage's own buffer */
        if (st->spill_cap < n) {
            free(st->spill);
            st->spill = malloc(n);
            if (!st->spill)
                abort(); /* like fsalloc: allocation failure is fatal */
            st->spill_cap = n;
        }
        dst = spill = st->spill;
    }
    size_t done = 0;
    while (done < n && st->nbusy) {
        slot *sl = &st->slots[st->head];
        size_t take = sl->body_end - sl->out_pos;
        if (take > n - done)
            take = n - done;
        memcpy(dst + done, slot_out(sl) + sl->out_pos, take);
        sl->out_pos += take;
        done += take;
        if (sl->out_pos == sl->out_len)
            retire_head(st);
        else if (sl->out_pos == sl->body_end)
            break;
    }
    if (spill)
        st->lent = spill;
    return done;
}

/*
 * Read semantics: the reference encoder returns
 * exactly `count` characters whenever its upstream fills the request
 * (base64encoder.c:124-141), a short count only when upstream came up
 * short, and the finalize() characters in a read of their own
 * (:127-128 -> :61-99).  The encoder stage does the same -- full count or
 * EAGAIN while blocks are in flight, a short count only when upstream has
 * run dry (EAGAIN/EOF) and nothing is left on the GPU -- so wrappers that
 * frame on read counts (chunkencoder) frame identically.  The decoder
 * returns whatever is finished, up to `count` (the reference's decoder
 * counts depend on where junk falls inside each read; no framing wrapper
 * consumes them).
 */
/* The lent bytes are no longer used: a head block they finished retires. */
static void stage_return(stage *st)
{
    if (!st->lent)
        return;
    st->lent = NULL;
    slot *h = &st->slots[st->head];
    if (st->nbusy && h->out_pos == h->out_len)
        retire_head(st);
}

static ssize_t stage_read(stage *st, void *buf, size_t count)
{
    stage_return(st); /* a new read ends any loan */
    if (!count)
        return 0;
    if (st->err) {
        errno = st->err;
        return -1;
    }
    int rc = stage_start(st, count);
    if (rc)
        return stage_fail(st, rc);
    rc = top_up(st);
    if (rc < 0)
        return stage_fail(st, rc);
    for (;;) {
        slot *h = &st->slots[st->head];
        if (st->nbusy && slot_ready(h) && h->ticket.err)
            return stage_fail(st, h->ticket.err);
        if (st->nbusy && slot_ready(h) && h->out_pos == h->body_end &&
            h->out_pos < h->out_len) {
            /* finalize(): partial sextet and pads, `count` at a time */
            size_t n = h->out_len - h->out_pos;
            if (n > count)
                n = count;
            if (st->lend_want) {
                st->lent = slot_out(h) + h->out_pos;
                h->out_pos += n;
                return (ssize_t) n;
            }
            memcpy(buf, slot_out(h) + h->out_pos, n);
            h->out_pos += n;
            if (h->out_pos == h->out_len)
                retire_head(st);
            return (ssize_t) n;
        }
        bool blocked;
        size_t staged = staged_body(st, &blocked);
        /* A short count only where the reference would return one: at
         * EOF, or after upstream itself came up short (a full-or-EAGAIN
         * upstream such as nicestream never does); or when no slot is
         * free to pull more (a read larger than both slots). */
        bool serve = staged >= count || (staged && st->dir == DIR_DECODE) ||
                     (staged && !blocked &&
                      (st->final_queued || st->short_seen || !next_launch_slot(st)));
        if (serve) {
            size_t n = serve_body(st, buf, staged < count ? staged : count);
            if (n == staged)
                st->short_seen = false;
            rc = top_up(st); /* keep the GPU busy while the consumer works */
            if (rc < 0)
                return stage_fail(st, rc);
            return (ssize_t) n;
        }
        if (blocked) {
            errno = EAGAIN; /* the completion brings the consumer back */
            return -1;
        }
        if (st->nbusy) { /* finished slots with nothing left to serve */
            retire_head(st);
            rc = top_up(st);
            if (rc < 0)
                return stage_fail(st, rc);
            continue;
        }
        if (st->final_queued)
            return 0;
        errno = rc > 0 ? rc : EAGAIN;
        return -1;
    }
}

static void stage_close(stage *st)
{
    st->lent = NULL;
    free(st->spill);
    st->spill = NULL;
    st->spill_cap = 0;
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

/* b64_lend.h: zero-copy reads for wrappers in this library. */
ssize_t b64_lend_read(bytestream_1 s, void *fallback, size_t count, const uint8_t **data)
{
    *data = NULL;
    if (s.vt != &encoder_vt)
        return bytestream_1_read(s, fallback, count);
    stage *st = &((base64encoder_t *) s.obj)->st;
    st->lend_want = true;
    ssize_t n = stage_read(st, fallback, count);
    st->lend_want = false;
    if (n > 0)
        *data = st->lent; /* NULL: copied into fallback */
    return n;
}

bool b64_lend_capable(bytestream_1 s)
{
    return s.vt == &encoder_vt;
}

void b64_lend_return(bytestream_1 s)
{
    if (s.vt == &encoder_vt)
        stage_return(&((base64encoder_t *) s.obj)->st);
}

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
