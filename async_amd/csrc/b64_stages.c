/*
 * b64_stages.c -- the base64 encoder and decoder bytestream_1 stages
 * (include/base64encoder.h, include/base64decoder.h), computed on the GPU
 * through the b64x C ABI (include/b64x.h).
 *
 * Reference: src/base64encoder.c and src/base64decoder.c.  The reference
 * transforms in place inside the caller's buffer, one byte per loop trip
 * (encoder :101-142, decoder :52-80), synchronously inside read().  Here a
 * stage is a small pipeline of up to NSLOTS blocks, each a job of a batch
 * of the loop's hub (b64_hub.h), which packs the blocks of every stage on
 * the loop into one ragged GPU launch:
 *
 *   read() --> serve the oldest finished block
 *          --> top up: pull upstream straight into the hub's pinned arena
 *              and commit the block as a job
 *          --> nothing finished yet: -1 / EAGAIN.
 *
 *   GPU completion: a HIP host function writes the hub's eventfd, which is
 *   registered with async_register(); the loop checks the batch, marks its
 *   jobs done and calls each stage, which calls the consumer's registered
 *   callback -- the same "EAGAIN now, callback later" contract every
 *   bytestream_1 in the reference follows.  A
 *   stage holds no HIP stream, event or session of its own.
 *
 * Group carries:
 *  - encoder: whole 3-byte groups are encoded; the 0-2 leftover bytes are
 *    carried on the host into the next block, and encoded with the final
 *    padding once upstream reports EOF (the reference's finalize(),
 *    :61-99);
 *  - decoder: blocks are decoded with B64X_DEC_HOLD_TAIL; the device
 *    reports the 0-3 sextets a block leaves over (its result record), and
 *    they are spelled as alphabet characters in a 4-byte head in front of
 *    the stream's next block (the reference keeps those bits in
 *    decoder->bits across reads, :64-76) -- by the host when the block
 *    before has finished, by the device (a chained job, b64_hub.h) while
 *    it is still in flight, so a decoder stream keeps up to NSLOTS blocks
 *    on the GPU.  At EOF the last block (or a head alone) is decoded
 *    without HOLD_TAIL, giving the reference's floor(6V/8) bytes overall.
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
 * Round 1 ran decoder blocks past the first on per-stage chained sessions
 * (a HIP stream, pinned buffers and a device carry chain each); under load
 * (600 streams on one loop) a block's result record copied back from the
 * device was read before it held the launch's values, and the block was
 * served as empty.  Every block now goes through the hub,
 * whose kernels write outputs and records into host memory themselves and
 * whose batches are checked before they are read.
 *
 * Tuning (environment, read when a stage is created):
 *   ASYNC_B64_STAGE_CAPACITY  bytes per block (default 1 MiB; the encoder
 *                             grows it to hold its first read's count, up
 *                             to ASYNC_B64_STAGE_MAX_CAPACITY, default
 *                             64 MiB)
 *   ASYNC_B64_MIN_PULL        gather at least this much from upstream
 *                             before launching, unless it runs dry
 *                             (default 64 KiB)
 *   ASYNC_B64_LEND_MIN        encoder: a queued message of at least this
 *                             many unread bytes (copied into pinned memory
 *                             by queuestream_enqueue_bytes, b64_pin.h) is
 *                             taken without copying (default 4 KiB; shorter
 *                             ones are gathered into a block together)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "async.h"
#include "b64_hub.h"
#include "b64_lend.h"
#include "b64_pin.h"
#include "b64_trace.h"
#include "b64x.h"
#include "base64decoder.h"
#include "base64encoder.h"
#include "fsalloc.h"

enum {
    NSLOTS = 4,   /* blocks in flight or staged per stage (read-ahead) */
    DEC_HEAD = 4, /* decoder: characters in front of a block for the carry */
};

typedef struct stage stage;

typedef struct {
    stage *owner;
    b64_ticket ticket;  /* this slot's job in a hub batch */
    bool hold;          /* decoder: more of the stream follows this block */
    bool carry_out;     /* decoder: the next block took this one's held-back
                           sextets on the device (b64_hub_chainable) */
    bool resolved;      /* out_len/body_end valid (decoder: after done) */
    size_t out_pos;
    size_t body_end;    /* encoder: end of the full sextets; the finalize
                           characters after it are served on their own */
    size_t out_len;
} slot;

typedef enum { DIR_ENCODE, DIR_DECODE } direction;

struct stage {
    async_t *async;
    uint64_t uid;       /* the reference's trace uid (b64_trace.h) */
    bytestream_1 up;
    action_1 cb;        /* the consumer's callback, or NULL_ACTION_1 */
    direction dir;
    b64x_alphabet abc;
    size_t cap, min_pull, max_cap;
    size_t grow_max;    /* a stream whose blocks fill grows its blocks to this */
    size_t lend_min;    /* encoder: pinned messages this long are lent */
    b64_hub *hub;       /* the loop's batching hub */
    unsigned hub_waits; /* entries on the hub's waiter list (room for a block) */
    bool started;       /* the hub is held */
    int err;            /* sticky failure errno, 0 while healthy */
    slot slots[NSLOTS];
    unsigned head;      /* oldest busy slot */
    unsigned nbusy;     /* launched, output not fully served */
    bool final_queued;  /* the last block (or nothing) has been launched */
    bool short_seen;    /* an upstream read came up short (not EAGAIN)
                           since the staged output last ran out */
    int up_err;         /* an upstream read failed (errno other than EAGAIN)
                           after the bytes before it were committed: the
                           staged output is served first, then one read
                           returns -1 with it (ref base64encoder.c:127-129,
                           base64decoder.c:58-61 return upstream's errno) */
    uint8_t carry[3];   /* encoder: bytes of the incomplete group;
                           decoder: sextets the last block held back */
    size_t ncarry;
    uint8_t skip;       /* decoder: a character its alphabet skips */
    bool lend_want;     /* this read may lend instead of copy (b64_lend.h) */
    uint8_t *spill;     /* lent copy of reads that span blocks (no fallback) */
    size_t spill_cap;
    const uint8_t *lent;/* what the last read lent, until returned */
    uint8_t tail[2];    /* encoder: the last two bytes of the block being gathered */
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

/* The decoder alphabet's effective positions 62/63 ((char) -1 = the
 * reference's defaults, base64decoder.c:31-32). */
static char dec_pos62(const b64x_alphabet *abc)
{
    return abc->pos62 == (char) -1 ? '+' : abc->pos62;
}

static char dec_pos63(const b64x_alphabet *abc)
{
    return abc->pos63 == (char) -1 ? '/' : abc->pos63;
}

/* A byte the decoder skips (ref map(), base64decoder.c:38-48: not
 * alphanumeric and not pos62/pos63). */
static uint8_t skip_char(const b64x_alphabet *abc)
{
    const char cand[3] = { '\n', '\r', ' ' };
    for (int i = 0; i < 3; i++)
        if (cand[i] != dec_pos62(abc) && cand[i] != dec_pos63(abc))
            return (uint8_t) cand[i];
    return '\n'; /* unreachable: two characters cannot shadow three */
}

/* A sextet as a character that decodes back to it.  62 and 63 only reach
 * a carry when the decoder recognised them, i.e. through pos62/pos63. */
static uint8_t spell_sextet(const b64x_alphabet *abc, uint8_t v)
{
    if (v < 26)
        return (uint8_t) ('A' + v);
    if (v < 52)
        return (uint8_t) ('a' + (v - 26));
    if (v < 62)
        return (uint8_t) ('0' + (v - 52));
    return (uint8_t) (v == 62 ? dec_pos62(abc) : dec_pos63(abc));
}

static void stage_init(stage *st, async_t *async, bytestream_1 up,
                       direction dir, b64x_alphabet abc)
{
    memset(st, 0, sizeof *st);
    st->async = async;
    st->uid = b64_trace_unique_id();
    st->up = up;
    st->cb = NULL_ACTION_1;
    st->dir = dir;
    st->abc = abc;
    st->cap = env_size("ASYNC_B64_STAGE_CAPACITY", (size_t) 1 << 20, 64);
    st->min_pull = env_size("ASYNC_B64_MIN_PULL", (size_t) 64 << 10, 1);
    st->lend_min = env_size("ASYNC_B64_LEND_MIN", 4096, 1);
    st->max_cap = env_size("ASYNC_B64_STAGE_MAX_CAPACITY", (size_t) 64 << 20, 64);
    /* an explicit block size stays fixed unless growth is asked for too */
    st->grow_max = env_size("ASYNC_B64_STAGE_GROW_MAX",
                            getenv("ASYNC_B64_STAGE_CAPACITY") ? st->cap : (size_t) 8 << 20, 64);
    if (st->grow_max < st->cap)
        st->grow_max = st->cap;
    st->skip = skip_char(&abc);
    b64_pin_activate(); /* queued messages are pinned for GPU stages from now on */
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
         * stage_read()). */
        size_t need = (count + 3) / 4 * 3 + 3;
        if (need > st->max_cap)
            need = st->max_cap;
        if (need > st->cap)
            st->cap = need;
    }
    int rc = b64x_device_check(); /* fail loudly: no CPU path */
    if (rc)
        return rc;
    st->hub = b64_hub_acquire(st->async);
    if (!st->hub)
        return -(errno ? errno : ENODEV);
    st->started = true;
    return 0;
}

static void stage_stop(stage *st)
{
    if (st->hub) {
        b64_hub_forget(st->hub, st, st->hub_waits > 0);
        for (int i = 0; i < NSLOTS; i++)
            b64_ticket_release(&st->slots[i].ticket);
        b64_hub_release(st->hub);
        st->hub = NULL;
    }
    st->started = false;
}

/* Lending from the queue (b64_lend.h, upstream side) needs this library's
 * own queuestream (framing.c, the standalone library).  The stages-only
 * library (INTEGRATION.md Option A) runs over the reference's queuestream,
 * which it cannot see into: there these weak stand-ins take over and every
 * block is gathered by reading, as before. */
__attribute__((weak)) bool b64_src_peek(bytestream_1 s, const uint8_t **p, size_t *n,
                                        struct b64_pin_slab **slab)
{
    (void) s, (void) p, (void) n, (void) slab;
    return false;
}

__attribute__((weak)) void b64_src_take(bytestream_1 s, size_t n)
{
    (void) s, (void) n;
}

__attribute__((weak)) size_t b64_src_plain(bytestream_1 s, size_t lend_min, size_t limit)
{
    (void) s, (void) lend_min;
    return limit;
}

/* Pull from upstream into the reservation `in` from offset `at` on, until
 * at least min_pull bytes have come in, or EOF, EAGAIN or an error; after
 * a short read it asks once more, so the EOF of a finite upstream lands in
 * the same block.  Returns bytes gathered; *eof / *err report why it
 * stopped.  Encoder: a queued message with at least lend_min unread bytes
 * in pinned memory (queuestream_enqueue_bytes, b64_pin.h) is not copied --
 * its bytes become a segment of the block that the GPU reads from where
 * they are (b64_hub_lend) -- when the hub has room for the segment; and
 * st->tail gets the block's last two bytes wherever they came from. */
FSTRACE_DECL(ASYNC_BASE64DECODER_READ_INPUT_DUMP, "UID=%64u DATA=%A");

static size_t gather(stage *st, uint8_t *in, size_t at, size_t room, bool *eof, int *err)
{
    uint8_t *dst = in + at;
    size_t got = 0;
    size_t want = st->min_pull < room ? st->min_pull : room;
    *eof = false;
    *err = 0;
    struct timespec t0 = { 0, 0 };
    const bool tr = b64_hub_tracing(st->hub);
    if (tr)
        clock_gettime(CLOCK_MONOTONIC, &t0);
    if (st->dir == DIR_ENCODE) /* the block so far: the carry */
        for (size_t i = 0; i < at; i++)
            st->tail[0] = st->tail[1], st->tail[1] = in[i];
    /* the last step took fewer bytes than one copying read of the room
     * would have (a lent message, or a read stopped where one begins): a
     * split of what the queue's own read would have returned in one call */
    bool split = false;
    while (got < room) {
        size_t ask = room - got;
        const uint8_t *lp;
        size_t ln;
        struct b64_pin_slab *ls;
        if (st->dir == DIR_ENCODE && b64_src_peek(st->up, &lp, &ln, &ls) && ln >= st->lend_min) {
            size_t n = ln < ask ? ln : ask;
            if (b64_hub_lend(st->hub, at + got, lp, n, ls)) {
                b64_src_take(st->up, n);
                if (n >= 2) {
                    st->tail[0] = lp[n - 2];
                    st->tail[1] = lp[n - 1];
                } else {
                    st->tail[0] = st->tail[1];
                    st->tail[1] = lp[0];
                }
                got += n;
                split = true;
                /* no min_pull stop here: a copying read of `ask` would have
                 * gone on into the next elements, so the block fills its
                 * room as that read would (block sizes decide the read
                 * counts the encoder can serve, and so the framing) */
                continue;
            }
        }
        bool limited = false;
        if (st->dir == DIR_ENCODE) {
            ask = b64_src_plain(st->up, st->lend_min, ask);
            if (!ask) /* a lendable message comes next, but the hub is full */
                ask = room - got;
            limited = ask < room - got;
        }
        ssize_t n = bytestream_1_read(st->up, dst + got, ask);
        if (st->dir == DIR_DECODE)
            FSTRACE(ASYNC_BASE64DECODER_READ_INPUT_DUMP, st->uid, dst + got, n);
        if (n < 0) {
            *err = errno ? errno : EIO;
            /* after a split, the queue's own read would have returned the
             * bytes before it as a short count (ref src/queuestream.c read
             * loop) */
            if (split && *err == EAGAIN)
                st->short_seen = true;
            break;
        }
        if (n == 0) {
            *eof = true;
            break;
        }
        split = limited && (size_t) n == ask;
        if (n >= 2) {
            st->tail[0] = dst[got + (size_t) n - 2];
            st->tail[1] = dst[got + (size_t) n - 1];
        } else {
            st->tail[0] = st->tail[1];
            st->tail[1] = dst[got];
        }
        got += (size_t) n;
        if ((size_t) n < ask)
            st->short_seen = true;
        else if (got >= want && !split)
            break;
    }
    if (tr) {
        struct timespec t1;
        clock_gettime(CLOCK_MONOTONIC, &t1);
        b64_hub_trace_gather(st->hub, (double) (t1.tv_sec - t0.tv_sec) +
                                          1e-9 * (double) (t1.tv_nsec - t0.tv_nsec), got);
    }
    return got;
}

/* A block that took all the room it asked for (upstream kept up) doubles
 * the next one, up to grow_max: one long stream then moves in a few large
 * blocks instead of many 1 MiB ones.  A stream's blocks are chained on one
 * lane (its carry), so each block is a serial round trip -- H2D, the
 * decode's kernels, the completion -- of 140 us or so at 1 MiB, and one
 * stream through the stages was bound by that, not by the copies: 1 GiB of
 * characters from memory 5.1 GiB/s with 1 MiB blocks, 8.5 with 4 MiB, 9.1
 * with 8 MiB; through an AF_UNIX socket 5.0 / 7.4 / 8.4
 * (profiles/r05_host_fd_stage_cap_*).  Messages that do not fill a block
 * (config 5's, a short read) never grow it. */
static void grow_block(stage *st, size_t granted, size_t asked, bool filled)
{
    if (filled && granted == asked && st->cap < st->grow_max) {
        size_t c = 2 * st->cap;
        st->cap = c < st->grow_max ? c : st->grow_max;
    }
}

static slot *next_launch_slot(stage *st)
{
    if (st->nbusy >= NSLOTS || st->final_queued)
        return NULL;
    return &st->slots[(st->head + st->nbusy) % NSLOTS];
}

static void slot_arm(stage *st, slot *sl)
{
    sl->resolved = false;
    sl->hold = false;
    sl->carry_out = false;
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

/* Backpressure: a stage may be made to wait for an arena unless it holds
 * finished output that cannot be served without more input (it must make
 * progress, or arenas could stay pinned by partially read jobs forever). */
static action_1 hub_waiter(stage *st)
{
    bool must_progress = st->nbusy > 0;
    for (unsigned i = 0; i < st->nbusy && must_progress; i++)
        if (!atomic_load_explicit(&st->slots[(st->head + i) % NSLOTS].ticket.done,
                                  memory_order_acquire))
            must_progress = false; /* a completion will wake us */
    if (must_progress)
        return (action_1) { NULL, NULL };
    return (action_1) { st, (act_1) stage_kicked };
}

static int reserve_failed(stage *st, action_1 waiter)
{
    if (errno == EAGAIN && waiter.act)
        st->hub_waits++;
    return errno == EAGAIN ? EAGAIN : -(errno ? errno : ENOMEM);
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
        action_1 waiter = hub_waiter(st);
        uint8_t *in = b64_hub_reserve(st->hub, B64_HUB_ENCODE, &st->abc, st->cap,
                                      st->ncarry + 4096, &room, waiter);
        if (!in)
            return reserve_failed(st, waiter);
        memcpy(in, st->carry, st->ncarry);
        bool eof;
        int uerr;
        const size_t asked = st->cap;
        size_t got = gather(st, in, st->ncarry, room - st->ncarry, &eof, &uerr);
        size_t total = st->ncarry + got;
        grow_block(st, room, asked, !eof && !uerr && total == room);
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
            /* the block's last bytes (lent ones are not in the arena) */
            memcpy(st->carry, st->tail + 2 - st->ncarry, st->ncarry);
        }
        slot_arm(st, sl);
        sl->out_len = (size_t) b64x_encoded_len(total, st->abc.pad);
        b64_hub_commit(st->hub, &sl->ticket, total, sl->out_len, 0, NULL,
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

static bool slot_ready(slot *sl);

/* Decoder blocks: each one a hub job of DEC_HEAD + n characters whose head
 * carries the 0-3 sextets the previous block held back (the reference keeps
 * them in decoder->bits across reads, base64decoder.c:64-76).  When the
 * previous block has finished, the host spells them into the head.  While
 * it is still queued or on the GPU, the block is chained to it
 * (b64_hub_chainable): the device spells them between the two decodes, in
 * stream order on one lane, so a stream keeps up to NSLOTS blocks in
 * flight.  A block that cannot be chained (its predecessor is filling at
 * another nesting level, or the arena follows another batch) waits for the
 * predecessor's completion. */
static int top_up_decoder(stage *st)
{
    slot *sl;
    while ((sl = next_launch_slot(st))) {
        slot *last = st->nbusy ? &st->slots[(st->head + st->nbusy - 1) % NSLOTS] : NULL;
        const bool pending = last && !slot_ready(last); /* its carry is not known here */
        size_t room;
        action_1 waiter = hub_waiter(st);
        size_t want = DEC_HEAD + st->cap;
        uint8_t *in = b64_hub_reserve(st->hub, B64_HUB_DECODE, &st->abc, want,
                                      DEC_HEAD + (st->cap < 4096 ? st->cap : 4096), &room,
                                      waiter);
        if (!in)
            return reserve_failed(st, waiter);
        if (pending && !b64_hub_chainable(st->hub, &last->ticket)) {
            b64_hub_cancel(st->hub);
            return 0; /* its completion brings us back */
        }
        bool eof;
        int uerr;
        size_t got = gather(st, in, DEC_HEAD, room - DEC_HEAD, &eof, &uerr);
        grow_block(st, room, want, !eof && !uerr && got == room - DEC_HEAD);
        if (eof) {
            st->final_queued = true;
            if (got == 0 && !pending && st->ncarry == 0) { /* nothing held back: done */
                b64_hub_cancel(st->hub);
                return 0;
            }
        } else if (got == 0) {
            b64_hub_cancel(st->hub);
            return uerr ? uerr : EAGAIN;
        }
        memset(in, st->skip, DEC_HEAD);
        for (size_t k = 0; k < st->ncarry; k++)
            in[DEC_HEAD - st->ncarry + k] = spell_sextet(&st->abc, st->carry[k]);
        st->ncarry = 0;
        slot_arm(st, sl);
        sl->hold = !eof;
        if (pending)
            last->carry_out = true;
        b64_hub_commit(st->hub, &sl->ticket, DEC_HEAD + got,
                       (size_t) b64x_decoded_cap(DEC_HEAD + got),
                       eof ? 0u : B64X_DEC_HOLD_TAIL, pending ? &last->ticket : NULL,
                       (action_1) { st, (act_1) stage_notify });
        if (uerr)
            return uerr;
    }
    return 0;
}

static int top_up(stage *st)
{
    return st->dir == DIR_ENCODE ? top_up_encoder(st) : top_up_decoder(st);
}

/* A finished slot's lengths (the decoder's come from its checked record,
 * whose held-back sextets become the next block's carry). */
static bool slot_ready(slot *sl)
{
    if (!atomic_load_explicit(&sl->ticket.done, memory_order_acquire))
        return false;
    if (!sl->resolved) { /* decoder */
        stage *st = sl->owner;
        sl->out_len = sl->ticket.err ? 0 : sl->ticket.out_len;
        sl->body_end = sl->out_len;
        sl->resolved = true;
        if (sl->hold && !sl->carry_out && !sl->ticket.err) {
            st->ncarry = sl->ticket.res.tail_n < 4 ? sl->ticket.res.tail_n : 0;
            memcpy(st->carry, sl->ticket.res.tail, st->ncarry);
        }
    }
    return true;
}

static int slot_err(slot *sl)
{
    return sl->ticket.err;
}

static const uint8_t *slot_out(slot *sl)
{
    return sl->ticket.out;
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
            fsfree(st->spill);
            st->spill = fsalloc(n);
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

/* top_up(), except that an upstream failure other than EAGAIN is kept in
 * up_err (its bytes before it are committed and get served first) and no
 * upstream read is made while one is pending. */
static int stage_top_up(stage *st)
{
    if (st->up_err)
        return 0;
    int rc = top_up(st);
    if (rc > 0 && rc != EAGAIN) {
        st->up_err = rc;
        return 0;
    }
    return rc;
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
    rc = stage_top_up(st);
    if (rc < 0)
        return stage_fail(st, rc);
    for (;;) {
        slot *h = &st->slots[st->head];
        if (st->nbusy && slot_ready(h) && slot_err(h))
            return stage_fail(st, slot_err(h));
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
                      (st->final_queued || st->short_seen || st->up_err ||
                       !next_launch_slot(st)));
        if (serve) {
            size_t n = serve_body(st, buf, staged < count ? staged : count);
            if (n == staged)
                st->short_seen = false;
            rc = stage_top_up(st); /* keep the GPU busy while the consumer works */
            if (rc < 0)
                return stage_fail(st, rc);
            return (ssize_t) n;
        }
        if (blocked) {
            errno = EAGAIN; /* the completion brings the consumer back */
            return -1;
        }
        if (!st->up_err && st->nbusy &&
            st->slots[st->head].out_pos < st->slots[st->head].out_len) {
            /* staged output short of `count` while upstream answered
             * EAGAIN: upstream's callback brings the consumer back (a
             * full-or-EAGAIN upstream makes the reference return EAGAIN
             * here too, never a short count) */
            errno = EAGAIN;
            return -1;
        }
        if (st->nbusy) { /* finished slots with nothing left to serve */
            retire_head(st);
            rc = stage_top_up(st);
            if (rc < 0)
                return stage_fail(st, rc);
            continue;
        }
        if (st->final_queued)
            return 0;
        if (st->up_err) { /* everything before the failure has been served */
            errno = st->up_err;
            st->up_err = 0;
            return -1;
        }
        errno = rc > 0 ? rc : EAGAIN;
        return -1;
    }
}

/* Ownership: the object came from fsalloc() and goes back
 * through async_wound() -> fsfree() on a later loop turn, so posthumous
 * callbacks (a hub wake already collected for this stage) find it valid;
 * everything else the stage holds is given back here. */
static void stage_close(stage *st)
{
    st->lent = NULL;
    fsfree(st->spill);
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

FSTRACE_DECL(ASYNC_BASE64ENCODER_CREATE, "UID=%64u PTR=%p ASYNC=%p SOURCE=%p");
FSTRACE_DECL(ASYNC_BASE64ENCODER_READ, "UID=%64u WANT=%z GOT=%z ERRNO=%e");
FSTRACE_DECL(ASYNC_BASE64ENCODER_READ_DUMP, "UID=%64u DATA=%A");
FSTRACE_DECL(ASYNC_BASE64ENCODER_CLOSE, "UID=%64u");
FSTRACE_DECL(ASYNC_BASE64ENCODER_REGISTER, "UID=%64u OBJ=%p ACT=%p");
FSTRACE_DECL(ASYNC_BASE64ENCODER_UNREGISTER, "UID=%64u");

struct base64encoder {
    stage st; /* first member: the object pointer is the stage */
};

base64encoder_t *base64_encode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63, bool pad, char padchar)
{
    base64encoder_t *e = fsalloc(sizeof *e); /* ref base64encoder.c:33 */
    b64x_alphabet abc = { pos62, pos63, padchar, pad };
    stage_init(&e->st, async, stream, DIR_ENCODE, abc);
    FSTRACE(ASYNC_BASE64ENCODER_CREATE, e->st.uid, e, async, stream.obj);
    return e;
}

ssize_t base64encoder_read(base64encoder_t *e, void *buf, size_t count)
{
    ssize_t n = stage_read(&e->st, buf, count);
    FSTRACE(ASYNC_BASE64ENCODER_READ, e->st.uid, count, n);
    FSTRACE(ASYNC_BASE64ENCODER_READ_DUMP, e->st.uid, buf, n);
    return n;
}

void base64encoder_close(base64encoder_t *e)
{
    FSTRACE(ASYNC_BASE64ENCODER_CLOSE, e->st.uid);
    stage_close(&e->st);
}

void base64encoder_register_callback(base64encoder_t *e, action_1 action)
{
    FSTRACE(ASYNC_BASE64ENCODER_REGISTER, e->st.uid, action.obj, action.act);
    stage_register(&e->st, action);
}

void base64encoder_unregister_callback(base64encoder_t *e)
{
    FSTRACE(ASYNC_BASE64ENCODER_UNREGISTER, e->st.uid);
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

FSTRACE_DECL(ASYNC_BASE64DECODER_CREATE, "UID=%64u PTR=%p ASYNC=%p SOURCE=%p");
FSTRACE_DECL(ASYNC_BASE64DECODER_READ, "UID=%64u WANT=%z GOT=%z ERRNO=%e");
FSTRACE_DECL(ASYNC_BASE64DECODER_READ_DUMP, "UID=%64u DATA=%A");
FSTRACE_DECL(ASYNC_BASE64DECODER_CLOSE, "UID=%64u");
FSTRACE_DECL(ASYNC_BASE64DECODER_REGISTER, "UID=%64u OBJ=%p ACT=%p");
FSTRACE_DECL(ASYNC_BASE64DECODER_UNREGISTER, "UID=%64u");

struct base64decoder {
    stage st;
};

base64decoder_t *base64_decode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63)
{
    base64decoder_t *d = fsalloc(sizeof *d); /* ref base64decoder.c:25 */
    b64x_alphabet abc = { pos62, pos63, (char) -1, false };
    stage_init(&d->st, async, stream, DIR_DECODE, abc);
    FSTRACE(ASYNC_BASE64DECODER_CREATE, d->st.uid, d, async, stream.obj);
    return d;
}

ssize_t base64decoder_read(base64decoder_t *d, void *buf, size_t count)
{
    ssize_t n = stage_read(&d->st, buf, count);
    FSTRACE(ASYNC_BASE64DECODER_READ, d->st.uid, count, n);
    FSTRACE(ASYNC_BASE64DECODER_READ_DUMP, d->st.uid, buf, n);
    return n;
}

void base64decoder_close(base64decoder_t *d)
{
    FSTRACE(ASYNC_BASE64DECODER_CLOSE, d->st.uid);
    stage_close(&d->st);
}

void base64decoder_register_callback(base64decoder_t *d, action_1 action)
{
    FSTRACE(ASYNC_BASE64DECODER_REGISTER, d->st.uid, action.obj, action.act);
    stage_register(&d->st, action);
}

void base64decoder_unregister_callback(base64decoder_t *d)
{
    FSTRACE(ASYNC_BASE64DECODER_UNREGISTER, d->st.uid);
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
