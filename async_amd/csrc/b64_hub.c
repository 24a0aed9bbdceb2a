/*
 * b64_hub.c -- cross-stream batching of encoder blocks and short decoder
 * streams (see b64_hub.h).
 *
 * Life of an arena ("batch"):
 *
 *   FREE --reserve--> FILLING --full / end of loop turn--> READY
 *        --lane free--> INFLIGHT --HIP host fn + eventfd--> DONE
 *        --every job's ticket released--> FREE (kept for reuse)
 *
 * All of it runs on the loop's thread except batch_done(), which only
 * publishes the flag and writes the eventfd.  The registry that maps an
 * async_t to its hub is the only state shared between threads (loops on
 * different threads each get their own hub) and is mutex-protected.
 *
 * Life of a hub: the first stage of a loop that starts work acquires it;
 * when the last one releases it, it is torn down at once (lanes waited
 * for, arenas back to the pool, eventfd unregistered) unless the loop is
 * inside one of its actions, which then tears it down on the way out.  Its
 * memory comes from fsalloc() and goes through async_wound(): a flush or
 * kick task already queued on the loop still finds it (and sees it dead),
 * and a loop destroyed before those tasks run frees it all the same
 * (destroy_async() frees wounded objects, ref src/async.c:140-162).
 */
#define _GNU_SOURCE
#include "b64_hub.h"
#include "b64_pin.h"
#include "fsalloc.h"

#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/eventfd.h>
#include <time.h>
#include <unistd.h>

enum {
    HUB_LANES = 4,          /* batches in flight per loop */
    HUB_MAX_LIVE = HUB_LANES + 4, /* arenas a hub holds before idle
                                     stages are made to wait */
    POOL_MAX = 256,         /* default of ASYNC_B64_POOL_MAX: idle arenas kept
                               process-wide for reuse (~41 MB pinned each at
                               the default ASYNC_B64_BATCH_BYTES).  Every arena
                               freed and allocated again costs milliseconds of
                               pinned-memory calls that stall the other loops:
                               config 5 on 16 loops holds more than 128 at its
                               peak (a hub exceeds HUB_MAX_LIVE for stages that
                               must progress), and with 128 kept each pass
                               allocated 1-18 arenas again and ran 10.8-14.1
                               GiB/s against 16.2-16.5 without
                               (profiles/r05_cfg5_t16_pool128.jsonl).  The pool
                               never holds more than the process's peak. */
    HUB_JOBS = 1 << 16,     /* jobs per arena */
    HUB_DEPTH = 8,          /* reservations open at once (stages reading
                               through stages, see b64_hub_reserve) */
    HUB_SEGS = 1 << 14,     /* lent segments per arena (more are copied) */
    LANE_QUEUE = 4,         /* decode batches queued on one lane: a batch
                               whose chained jobs continue streams of a batch
                               in flight on that lane waits behind it there */
};

typedef enum { B_FREE, B_FILLING, B_READY, B_INFLIGHT, B_DONE } batch_state;

struct b64_batch {
    b64_hub *hub;
    b64_batch *next;             /* ready / free list */
    uint8_t *h_in, *h_out;       /* pinned arenas */
    uint64_t *h_in_off, *h_out_off; /* pinned, HUB_JOBS + 1 each */
    uint8_t *h_flags;            /* pinned, HUB_JOBS: decode jobs' flags */
    b64x_dec_result *h_res;      /* pinned, HUB_JOBS: decode jobs' records */
    b64x_dec_result *h_spell;    /* pinned, HUB_JOBS: chained jobs' spell logs */
    const b64x_dec_result **h_prev; /* HUB_JOBS: chained jobs' predecessor records */
    b64x_seg *h_seg;             /* pinned, HUB_SEGS: encode input lent from pinned
                                    messages (b64_hub_lend), by device offset */
    b64_pin_slab **pins;         /* HUB_SEGS: the slab each segment holds */
    uint32_t nseg;
    b64_batch *after;            /* a batch in flight (or ready) whose records
                                    chained jobs of this one read: this one
                                    runs behind it on its lane */
    unsigned after_refs;         /* references this batch holds on `after` */
    b64_batch *lane_next;        /* the lane's queue of batches in flight */
    int lane;                    /* lane it runs on, -1 before launch */
    uint32_t seq;                /* decode batches: the lane's sequence number */
    b64_hub_kind kind;
    b64_ticket **jobs;
    size_t in_cap, out_cap;
    size_t in_used, out_used;
    uint32_t njobs;
    unsigned refs;               /* tickets still holding a job */
    b64x_alphabet abc;
    batch_state state;
    atomic_int done;
    int err;
};

struct b64_hub {
    async_t *async;
    b64_hub *next_hub;           /* registry */
    unsigned users;
    int efd;
    b64x_lane *lanes[HUB_LANES];
    b64_batch *lane_head[HUB_LANES], *lane_tail[HUB_LANES]; /* in flight, in order */
    unsigned lane_depth[HUB_LANES];
    b64_batch *filling[HUB_DEPTH]; /* the open arena of each nesting level */
    unsigned depth;              /* reservations open (gathers in progress) */
    b64_batch *ready, *ready_tail;
    unsigned inflight;
    unsigned live;               /* arenas taken from the pool */
    size_t batch_bytes;
    bool flush_scheduled, kick_scheduled; /* a task of ours is queued */
    bool in_wake, in_kick;       /* inside hub_wake() / hub_kick() */
    bool doomed;                 /* no users: torn down when not inside */
    bool dead;                   /* torn down; memory awaits async_wound() */
    action_1 *wakes;             /* scratch for hub_wake() */
    size_t nwakes, wakes_cap;
    action_1 *waiters;           /* idle stages waiting for an arena */
    size_t nwaiters, waiters_cap;
    action_1 *kicking;           /* the list hub_kick() is working through */
    size_t nkicking;
    struct {                     /* ASYNC_B64_HUB_TRACE=1: printed at teardown */
        bool on;
        unsigned long batches, jobs, allocs, wake_calls, max_ready, max_live;
        unsigned long long in_bytes, out_bytes, gather_bytes;
        unsigned long reserves, lent_jobs;
        unsigned long long lent_bytes;
        double wake_s, launch_s, t_first, t_last;
        double gather_s, reserve_s; /* the stages' upstream reads; arena reservations */
    } tr;
};

static double mono_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static pthread_mutex_t registry_lock = PTHREAD_MUTEX_INITIALIZER;
static b64_hub *registry;
static atomic_uint nhubs; /* hubs in the registry (loops with GPU stages) */

/* Idle arenas, shared by all hubs of the process (pinned allocation costs
 * milliseconds; a hub's life may be one message). */
static pthread_mutex_t pool_lock = PTHREAD_MUTEX_INITIALIZER;
static b64_batch *pool;
static unsigned npool;
static unsigned pool_max = POOL_MAX;
static pthread_once_t pool_once = PTHREAD_ONCE_INIT;

static size_t env_bytes(const char *name, size_t dflt, size_t lo)
{
    const char *v = getenv(name);
    if (!v || !*v)
        return dflt;
    char *end = NULL;
    unsigned long long x = strtoull(v, &end, 0);
    return (!end || *end || x < lo) ? dflt : (size_t) x;
}

static void pool_init(void)
{
    pool_max = (unsigned) env_bytes("ASYNC_B64_POOL_MAX", POOL_MAX, 0);
}

/* ---------------------------------------------------------------- batches */

static atomic_uint arenas_total; /* arenas in existence, pooled or not */
static atomic_bool stocking;      /* a thread is stocking the pool */

static void batch_free(b64_batch *b)
{
    atomic_fetch_sub_explicit(&arenas_total, 1, memory_order_relaxed);
    b64x_host_free(b->h_in);
    b64x_host_free(b->h_out);
    b64x_host_free(b->h_in_off);
    b64x_host_free(b->h_out_off);
    b64x_host_free(b->h_flags);
    b64x_host_free(b->h_res);
    b64x_host_free(b->h_spell);
    b64x_host_free(b->h_seg);
    free(b->pins);
    free(b->h_prev);
    free(b->jobs);
    free(b);
}

static b64_batch *batch_new(b64_hub *h, size_t in_cap)
{
    b64_batch *b = calloc(1, sizeof *b);
    if (!b)
        return NULL;
    b->hub = h;
    b->in_cap = in_cap;
    /* per job at most 4 characters beyond 4n/3 */
    b->out_cap = (in_cap + 2) / 3 * 4 + 4 * (size_t) HUB_JOBS;
    b->h_in = b64x_host_alloc(in_cap);
    b->h_out = b64x_host_alloc(b->out_cap);
    b->h_in_off = b64x_host_alloc((HUB_JOBS + 1) * sizeof(uint64_t));
    b->h_out_off = b64x_host_alloc((HUB_JOBS + 1) * sizeof(uint64_t));
    b->h_flags = b64x_host_alloc(HUB_JOBS);
    b->h_res = b64x_host_alloc(HUB_JOBS * sizeof(b64x_dec_result));
    b->h_spell = b64x_host_alloc(HUB_JOBS * sizeof(b64x_dec_result));
    b->h_prev = calloc(HUB_JOBS, sizeof *b->h_prev);
    b->h_seg = b64x_host_alloc(HUB_SEGS * sizeof *b->h_seg);
    b->pins = calloc(HUB_SEGS, sizeof *b->pins);
    b->jobs = malloc(HUB_JOBS * sizeof *b->jobs);
    b->lane = -1;
    atomic_fetch_add_explicit(&arenas_total, 1, memory_order_relaxed);
    if (!b->h_in || !b->h_out || !b->h_in_off || !b->h_out_off || !b->h_flags || !b->h_res ||
        !b->h_spell || !b->h_prev || !b->h_seg || !b->pins || !b->jobs) {
        batch_free(b);
        errno = ENOMEM;
        return NULL;
    }
    return b;
}

static void schedule_kick(b64_hub *h);

/* Back to the process pool (or freed); wakes stages waiting for room. */
static void batch_put(b64_batch *b)
{
    for (uint32_t i = 0; i < b->nseg; i++) /* the GPU has read them (or never will) */
        b64_pin_unref(b->pins[i]);
    b->nseg = 0;
    b->state = B_FREE;
    b->in_used = b->out_used = 0;
    b->njobs = 0;
    b->err = 0;
    b->hub = NULL;
    b->after = NULL;
    b->after_refs = 0;
    b->lane_next = NULL;
    b->lane = -1;
    atomic_store_explicit(&b->done, 0, memory_order_relaxed);
    pthread_once(&pool_once, pool_init);
    pthread_mutex_lock(&pool_lock);
    if (npool < pool_max) {
        b->next = pool;
        pool = b;
        npool++;
        b = NULL;
    }
    pthread_mutex_unlock(&pool_lock);
    if (b)
        batch_free(b);
}

static void batch_recycle(b64_hub *h, b64_batch *b)
{
    batch_put(b);
    h->live--;
    if (h->nwaiters)
        schedule_kick(h);
}

/* This batch no longer reads its `after` batch's records. */
static void batch_drop_after(b64_hub *h, b64_batch *b)
{
    b64_batch *a = b->after;
    if (!a)
        return;
    unsigned n = b->after_refs;
    b->after = NULL;
    b->after_refs = 0;
    a->refs -= n;
    if (a->refs == 0 && a->state == B_DONE)
        batch_recycle(h, a);
}

/* The pool ran dry: stock it, by one thread at a time and within the
 * pool's cap.  Demand grows a little at a time -- config 5 on 16 loops took
 * one more arena than ever before in a pass now and then -- and every arena
 * allocated on demand is a pinned-memory call that stalls every loop for
 * milliseconds: with the pool filled only on demand, passes that allocated
 * ran 10.8-14.1 GiB/s against 16.2-16.5 for those that did not
 * (profiles/r05_cfg5_t16_pool128.jsonl, r05_cfg5_t16_stocked.jsonl).
 *  - Several loops with GPU stages (nhubs > 1): up to the arenas the live
 *    hubs hold under their normal limit (HUB_MAX_LIVE each).
 *  - Otherwise, and past that: a quarter of the arenas in existence.  A
 *    process with one loop that decodes one message allocates its one arena
 *    and no more (round 5 stocked HUB_MAX_LIVE at once: ~330 MB pinned for
 *    one message); one that keeps 4+ arenas busy grows by a
 *    quarter each time the pool runs dry.
 * The pool never holds more than ASYNC_B64_POOL_MAX idle arenas (256 by
 * default, ~41 MB pinned each at the default ASYNC_B64_BATCH_BYTES: a
 * ceiling of ~10.5 GB of idle pinned memory, reached only by a process whose
 * peak held that many). */
static void stock_pool(b64_hub *h)
{
    bool idle = false;
    if (!atomic_compare_exchange_strong(&stocking, &idle, true))
        return;
    const unsigned total = atomic_load_explicit(&arenas_total, memory_order_relaxed);
    const unsigned hubs = atomic_load_explicit(&nhubs, memory_order_relaxed);
    const unsigned cover = hubs > 1 ? hubs * HUB_MAX_LIVE : 0;
    const unsigned want = cover > total ? cover - total : total / 4;
    pthread_once(&pool_once, pool_init);
    for (unsigned i = 0; i < want; i++) {
        pthread_mutex_lock(&pool_lock);
        const bool room = npool < pool_max;
        pthread_mutex_unlock(&pool_lock);
        if (!room)
            break;
        b64_batch *x = batch_new(h, h->batch_bytes);
        if (!x)
            break;
        h->tr.allocs++;
        batch_put(x);
    }
    atomic_store(&stocking, false);
}

static b64_batch *batch_get(b64_hub *h, size_t need)
{
    b64_batch *b = NULL;
    pthread_mutex_lock(&pool_lock);
    for (b64_batch **p = &pool; *p; p = &(*p)->next) {
        if ((*p)->in_cap >= need) {
            b = *p;
            *p = b->next;
            npool--;
            break;
        }
    }
    pthread_mutex_unlock(&pool_lock);
    if (!b) {
        h->tr.allocs++;
        b = batch_new(h, need > h->batch_bytes ? need : h->batch_bytes);
        if (!b)
            return NULL;
        if (need <= h->batch_bytes)
            stock_pool(h);
    }
    b->hub = h;
    h->live++;
    if (h->live > h->tr.max_live)
        h->tr.max_live = h->live;
    return b;
}

/* HIP runtime thread. */
static void batch_done(void *arg)
{
    b64_batch *b = arg;
    atomic_store_explicit(&b->done, 1, memory_order_release);
    uint64_t one = 1;
    ssize_t rc = write(b->hub->efd, &one, sizeof one);
    (void) rc;
}

/* ------------------------------------------------------------ scheduling */

static void seal(b64_hub *h, unsigned level)
{
    b64_batch *b = h->filling[level];
    if (!b)
        return;
    h->filling[level] = NULL;
    b->state = B_READY;
    b->next = NULL;
    if (h->ready_tail)
        h->ready_tail->next = b;
    else
        h->ready = b;
    h->ready_tail = b;
    if (h->tr.on) {
        unsigned long depth = 0;
        for (b64_batch *r = h->ready; r; r = r->next)
            depth++;
        if (depth > h->tr.max_ready)
            h->tr.max_ready = depth;
    }
}

/* The lane a ready batch goes to: behind the batch its chained jobs read
 * from while that one is in flight (its lane's queue has room), else an
 * idle lane; -1 when it has to wait. */
static int pick_lane(b64_hub *h, const b64_batch *b)
{
    if (b->after && b->after->state == B_INFLIGHT) {
        int i = b->after->lane;
        return h->lane_depth[i] < LANE_QUEUE ? i : -1;
    }
    for (int i = 0; i < HUB_LANES; i++)
        if (!h->lane_depth[i])
            return i;
    return -1;
}

static void launch_ready(b64_hub *h)
{
    double t0 = h->tr.on ? mono_s() : 0;
    /* in order: a batch that must wait keeps every later one waiting (a
     * batch's `after` is always ahead of it) */
    while (h->ready) {
        b64_batch *b = h->ready;
        int i = pick_lane(h, b);
        if (i < 0)
            break;
        h->ready = b->next;
        if (!h->ready)
            h->ready_tail = NULL;
        b->state = B_INFLIGHT;
        b->lane = i;
        b->lane_next = NULL;
        if (h->lane_tail[i])
            h->lane_tail[i]->lane_next = b;
        else
            h->lane_head[i] = b;
        h->lane_tail[i] = b;
        h->lane_depth[i]++;
        h->inflight++;
        int rc = 0;
        if (!h->lanes[i] && !(h->lanes[i] = b64x_lane_acquire()))
            rc = -(errno ? errno : ENODEV);
        if (!rc)
            rc = b->kind == B64_HUB_DECODE
                     ? b64x_lane_decode_async(h->lanes[i], b->h_in, b->njobs, b->h_in_off,
                                              b->h_out, b->h_out_off, b->h_flags, b->h_res,
                                              b->h_prev, b->h_spell, &b->abc, batch_done, b,
                                              &b->seq)
                     : b64x_lane_encode_async(h->lanes[i], b->h_in, b->njobs, b->h_in_off,
                                              b->h_out, b->h_out_off, b->h_seg, b->nseg,
                                              &b->abc, batch_done, b);
        if (rc) { /* report through the normal completion path */
            /* work queued before the failure may still write into the
             * arena: wait for it, so the arena is idle when it is recycled */
            if (h->lanes[i])
                (void) b64x_lane_wait(h->lanes[i]);
            b->err = rc;
            batch_done(b);
        }
        if (h->tr.on) {
            h->tr.batches++;
            h->tr.jobs += b->njobs;
            h->tr.in_bytes += b->in_used;
            h->tr.out_bytes += b->out_used;
            if (!h->tr.t_first)
                h->tr.t_first = t0;
        }
    }
    if (h->tr.on)
        h->tr.launch_s += mono_s() - t0;
}

static void hub_teardown(b64_hub *h);

/* A doomed hub is torn down as soon as none of its actions is running. */
static void hub_maybe_teardown(b64_hub *h)
{
    if (h->doomed && !h->dead && !h->in_wake && !h->in_kick)
        hub_teardown(h);
}

static void hub_flush(b64_hub *h)
{
    h->flush_scheduled = false;
    if (h->dead || h->doomed)
        return;
    for (unsigned l = 0; l < HUB_DEPTH; l++)
        if (h->filling[l] && h->filling[l]->njobs && l >= h->depth)
            seal(h, l);
    launch_ready(h);
}

static void schedule_flush(b64_hub *h)
{
    if (h->flush_scheduled || h->dead)
        return;
    h->flush_scheduled = true;
    async_execute(h->async, (action_1) { h, (act_1) hub_flush });
}

/* Room freed up: let every waiting stage retry (deferred, so no stage is
 * re-entered from inside another stage's read()). */
static void hub_kick(b64_hub *h)
{
    h->kick_scheduled = false;
    if (h->dead || h->doomed)
        return;
    /* Oldest first, and only until one of them still finds no room (it
     * re-queues itself): waking thousands of stages for one free arena
     * would cost a retry each. */
    size_t n = h->nwaiters;
    action_1 *w = h->waiters;
    h->waiters = NULL;
    h->nwaiters = h->waiters_cap = 0;
    h->kicking = w;
    h->nkicking = n;
    h->in_kick = true;
    size_t i = 0;
    while (i < n && !h->doomed) {
        action_1 a = w[i++];
        if (!a.act)
            continue; /* forgotten: its stage closed meanwhile */
        action_1_perf(a);
        if (h->nwaiters)
            break;
    }
    h->kicking = NULL;
    h->nkicking = 0;
    h->in_kick = false;
    for (; i < n && !h->doomed; i++) { /* the rest keep their place */
        if (!w[i].act)
            continue;
        if (h->nwaiters == h->waiters_cap) {
            size_t cap = h->waiters_cap ? 2 * h->waiters_cap : 64;
            action_1 *nw = realloc(h->waiters, cap * sizeof *nw);
            if (!nw)
                abort();
            h->waiters = nw;
            h->waiters_cap = cap;
        }
        h->waiters[h->nwaiters++] = w[i];
    }
    free(w);
    hub_maybe_teardown(h);
}

static void schedule_kick(b64_hub *h)
{
    if (h->kick_scheduled || h->doomed || h->dead)
        return;
    h->kick_scheduled = true;
    async_execute(h->async, (action_1) { h, (act_1) hub_kick });
}

static void push_wake(b64_hub *h, action_1 a)
{
    if (h->nwakes == h->wakes_cap) {
        size_t cap = h->wakes_cap ? 2 * h->wakes_cap : 64;
        action_1 *w = realloc(h->wakes, cap * sizeof *w);
        if (!w)
            abort();
        h->wakes = w;
        h->wakes_cap = cap;
    }
    h->wakes[h->nwakes++] = a;
}

/* A finished batch: publish every live job's output. */
static void complete(b64_hub *h, b64_batch *b, bool collect)
{
    for (uint32_t j = 0; j < b->njobs; j++) {
        b64_ticket *t = b->jobs[j];
        if (!t)
            continue;
        t->out = b->h_out + b->h_out_off[j];
        if (b->kind == B64_HUB_DECODE && !b->err) {
            t->res = b->h_res[j];
            t->out_len = (size_t) t->res.out_len;
        }
        t->err = b->err;
        atomic_store_explicit(&t->done, 1, memory_order_release);
        if (collect)
            push_wake(h, t->wake);
    }
    b->state = B_DONE;
    batch_drop_after(h, b);
    if (b->refs == 0)
        batch_recycle(h, b);
}

static void hub_wake(b64_hub *h)
{
    /* Drain to EAGAIN first: async_register() is edge-triggered (the
     * reference's contract, include/async.h), so the next completion's
     * write is a fresh edge; batch_done() publishes `done` before it
     * writes, so every batch whose write this read consumed is seen done
     * below. */
    if (h->dead)
        return;
    uint64_t v;
    while (read(h->efd, &v, sizeof v) == (ssize_t) sizeof v)
        ;
    double t0 = h->tr.on ? mono_s() : 0;
    h->in_wake = true;
    h->nwakes = 0;
    for (int i = 0; i < HUB_LANES; i++) {
        /* a lane's batches finish in the order they were queued */
        b64_batch *b;
        while ((b = h->lane_head[i]) && atomic_load_explicit(&b->done, memory_order_acquire)) {
            h->lane_head[i] = b->lane_next;
            if (!h->lane_head[i])
                h->lane_tail[i] = NULL;
            h->lane_depth[i]--;
            h->inflight--;
            /* the batch's records or completion stamp, checked (and
             * waited for, should the callback have come early) before
             * anything of it is read */
            if (!b->err)
                b->err = b->kind == B64_HUB_DECODE
                             ? b64x_lane_decode_check(h->lanes[i], b->seq, b->h_in_off,
                                                      b->h_flags, b->h_res, b->h_prev,
                                                      b->h_spell, b->njobs)
                             : b64x_lane_encode_check(h->lanes[i]);
            if (b->err && b->kind == B64_HUB_DECODE) /* chained successors read its records */
                for (b64_batch *q = h->lane_head[i]; q; q = q->lane_next)
                    if (q->after == b && !q->err)
                        q->err = b->err;
            complete(h, b, true);
        }
    }
    launch_ready(h);
    /* Callbacks may close stages (and release tickets) or read again
     * (and reserve): the wake list is the hub's own scratch, so copy out
     * nothing but run them in order; no batch pointer is used below. */
    size_t n = h->nwakes;
    for (size_t i = 0; i < n; i++)
        action_1_perf(h->wakes[i]);
    h->in_wake = false;
    if (h->tr.on) {
        h->tr.wake_calls++;
        h->tr.t_last = mono_s();
        h->tr.wake_s += h->tr.t_last - t0;
    }
    hub_maybe_teardown(h);
}

/* ------------------------------------------------------------- lifecycle */

b64_hub *b64_hub_acquire(async_t *async)
{
    pthread_mutex_lock(&registry_lock);
    for (b64_hub *h = registry; h; h = h->next_hub) {
        if (h->async == async && !h->doomed) {
            h->users++;
            pthread_mutex_unlock(&registry_lock);
            return h;
        }
    }
    b64_hub *h = fscalloc(1, sizeof *h);
    h->async = async;
    h->batch_bytes = env_bytes("ASYNC_B64_BATCH_BYTES", (size_t) 16 << 20, 4096);
    h->tr.on = env_bytes("ASYNC_B64_HUB_TRACE", 0, 0) != 0;
    h->efd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (h->efd < 0 ||
        async_register(async, h->efd, (action_1) { h, (act_1) hub_wake }) < 0) {
        int e = errno ? errno : EIO;
        if (h->efd >= 0)
            close(h->efd);
        fsfree(h);
        pthread_mutex_unlock(&registry_lock);
        errno = e;
        return NULL;
    }
    /* the loop's thread onto the GPU's NUMA node (b64x_bind_thread): its
     * copies into pinned arenas and out of them are the loop's work */
    if (env_bytes("ASYNC_B64_BIND", 1, 0) != 0)
        (void) b64x_bind_thread(-1);
    h->users = 1;
    h->next_hub = registry;
    registry = h;
    atomic_fetch_add_explicit(&nhubs, 1, memory_order_relaxed);
    pthread_mutex_unlock(&registry_lock);
    return h;
}

/* Teardown's batches: every one the hub still holds, collected before any
 * goes back to the process pool (a pooled batch may be taken by another
 * loop's hub at once, so none is read after its batch_put). */
typedef struct {
    b64_batch **v;
    size_t n, cap;
} batch_set;

static void set_add(batch_set *s, b64_batch *b)
{
    for (size_t i = 0; i < s->n; i++)
        if (s->v[i] == b)
            return;
    if (s->n == s->cap) {
        size_t cap = s->cap ? 2 * s->cap : 16;
        b64_batch **v = realloc(s->v, cap * sizeof *v);
        if (!v)
            abort(); /* a few pointers; fsalloc() aborts likewise */
        s->v = v;
        s->cap = cap;
    }
    s->v[s->n++] = b;
}

static void hub_teardown(b64_hub *h)
{
    h->dead = true;
    if (h->tr.on)
        fprintf(stderr,
                "b64_hub: batches %lu jobs %lu in %llu out %llu allocs %lu "
                "max_ready %lu max_live %lu wakes %lu wake_s %.4f launch_s %.4f span_s %.4f "
                "first %.6f last %.6f gather_s %.4f gather_bytes %llu reserve_s %.4f "
                "reserves %lu lent_segs %lu lent_bytes %llu\n",
                h->tr.batches, h->tr.jobs, h->tr.in_bytes, h->tr.out_bytes,
                h->tr.allocs, h->tr.max_ready, h->tr.max_live, h->tr.wake_calls, h->tr.wake_s,
                h->tr.launch_s, h->tr.t_last - h->tr.t_first, h->tr.t_first, h->tr.t_last,
                h->tr.gather_s, h->tr.gather_bytes, h->tr.reserve_s, h->tr.reserves,
                h->tr.lent_jobs, h->tr.lent_bytes);
    pthread_mutex_lock(&registry_lock);
    for (b64_hub **p = &registry; *p; p = &(*p)->next_hub) {
        if (*p == h) {
            *p = h->next_hub;
            atomic_fetch_sub_explicit(&nhubs, 1, memory_order_relaxed);
            break;
        }
    }
    pthread_mutex_unlock(&registry_lock);
    batch_set all = { NULL, 0, 0 };
    for (int i = 0; i < HUB_LANES; i++) {
        if (h->lane_head[i]) /* teardown: wait, do not wake anyone */
            (void) b64x_lane_wait(h->lanes[i]);
        while (h->lane_head[i]) {
            b64_batch *b = h->lane_head[i];
            h->lane_head[i] = b->lane_next;
            set_add(&all, b);
        }
        h->lane_tail[i] = NULL;
        h->lane_depth[i] = 0;
        b64x_lane_release(h->lanes[i]);
    }
    for (unsigned l = 0; l < HUB_DEPTH; l++)
        if (h->filling[l])
            set_add(&all, h->filling[l]);
    while (h->ready) {
        b64_batch *b = h->ready;
        h->ready = b->next;
        set_add(&all, b);
    }
    /* the finished batches they still read records of (held only by those
     * references: every stage is gone), then every link dropped, then each
     * batch back to the pool exactly once */
    for (size_t i = 0; i < all.n; i++) {
        b64_batch *a = all.v[i]->after;
        all.v[i]->after = NULL;
        all.v[i]->after_refs = 0;
        if (a && a->state == B_DONE)
            set_add(&all, a);
    }
    for (size_t i = 0; i < all.n; i++)
        batch_put(all.v[i]);
    free(all.v);
    (void) async_unregister(h->async, h->efd);
    close(h->efd);
    h->efd = -1;
    free(h->wakes);
    free(h->waiters);
    h->wakes = h->waiters = NULL;
    h->nwakes = h->nwaiters = h->wakes_cap = h->waiters_cap = 0;
    async_wound(h->async, h);
}

void b64_hub_release(b64_hub *h)
{
    if (!h || --h->users)
        return;
    pthread_mutex_lock(&registry_lock);
    h->doomed = true; /* no new stage may pick it up */
    pthread_mutex_unlock(&registry_lock);
    hub_maybe_teardown(h);
}

void b64_hub_forget(b64_hub *h, void *obj, bool waiting)
{
    if (!waiting)
        return;
    for (size_t i = 0; i < h->nkicking; i++)
        if (h->kicking[i].obj == obj)
            h->kicking[i].act = NULL;
    size_t k = 0;
    for (size_t i = 0; i < h->nwaiters; i++)
        if (h->waiters[i].obj != obj)
            h->waiters[k++] = h->waiters[i];
    h->nwaiters = k;
}

/* -------------------------------------------------------------- the API */

/*
 * Reservations nest: a stage gathers its block from upstream while holding
 * its reservation, and that upstream may itself be a base64 stage on the
 * same loop reserving its own block (the reference test's decoder reads
 * through nice(91) from the encoder, test/asynctest-base64encoder.c:
 * 123-151).  Each open reservation has its own arena (filling[depth]), so
 * an inner reservation never moves, seals or recycles an outer one.
 */
static uint8_t *reserve(b64_hub *h, b64_hub_kind kind, const b64x_alphabet *abc,
                        size_t room, size_t min_room, size_t *granted, action_1 waiter)
{
    if (h->depth == HUB_DEPTH) {
        errno = ELOOP; /* stages nested deeper than HUB_DEPTH */
        return NULL;
    }
    const unsigned lv = h->depth;
    if (min_room > room)
        min_room = room;
    b64_batch *b = h->filling[lv];
    if (b && (b->kind != kind || memcmp(&b->abc, abc, sizeof *abc) || b->njobs == HUB_JOBS ||
              b->in_cap - b->in_used < (min_room ? min_room : 1))) {
        if (b->njobs) {
            seal(h, lv);
            launch_ready(h);
        }
        b = h->filling[lv]; /* NULL after seal; kept if it was empty */
        if (b && (b->in_cap < room || b->kind != kind || memcmp(&b->abc, abc, sizeof *abc))) {
            h->filling[lv] = NULL;
            batch_put(b);
            h->live--;
            b = NULL;
        }
    }
    if (!b) {
        if (waiter.act && h->live >= HUB_MAX_LIVE) {
            if (h->nwaiters == h->waiters_cap) {
                size_t cap = h->waiters_cap ? 2 * h->waiters_cap : 64;
                action_1 *w = realloc(h->waiters, cap * sizeof *w);
                if (!w)
                    abort();
                h->waiters = w;
                h->waiters_cap = cap;
            }
            h->waiters[h->nwaiters++] = waiter;
            errno = EAGAIN;
            return NULL;
        }
        b = batch_get(h, room);
        if (!b)
            return NULL;
        b->state = B_FILLING;
        b->abc = *abc;
        b->kind = kind;
        h->filling[lv] = b;
    }
    size_t avail = b->in_cap - b->in_used;
    *granted = room < avail ? room : avail;
    h->depth++;
    return b->h_in + b->in_used;
}

uint8_t *b64_hub_reserve(b64_hub *h, b64_hub_kind kind, const b64x_alphabet *abc,
                         size_t room, size_t min_room, size_t *granted, action_1 waiter)
{
    if (!h->tr.on)
        return reserve(h, kind, abc, room, min_room, granted, waiter);
    double t0 = mono_s(); /* includes the launches of the batches it seals */
    uint8_t *p = reserve(h, kind, abc, room, min_room, granted, waiter);
    h->tr.reserve_s += mono_s() - t0;
    h->tr.reserves++;
    return p;
}

bool b64_hub_tracing(const b64_hub *h)
{
    return h->tr.on;
}

void b64_hub_trace_gather(b64_hub *h, double secs, size_t bytes)
{
    h->tr.gather_s += secs;
    h->tr.gather_bytes += bytes;
}

bool b64_hub_chainable(b64_hub *h, const b64_ticket *prev)
{
    const b64_batch *p = prev->batch;
    if (!h->depth || !p || atomic_load_explicit(&prev->done, memory_order_acquire))
        return false;
    const b64_batch *b = h->filling[h->depth - 1];
    if (p == b)
        return true; /* earlier job of the same batch */
    if (p->state != B_READY && p->state != B_INFLIGHT)
        return false; /* filling at another nesting level */
    return !b->after || b->after == p;
}

void b64_hub_commit(b64_hub *h, b64_ticket *t, size_t n, size_t out_len,
                    unsigned flags, const b64_ticket *prev, action_1 wake)
{
    b64_batch *b = h->filling[--h->depth];
    uint32_t j = b->njobs++;
    b->h_flags[j] = (uint8_t) flags;
    b->h_prev[j] = NULL;
    if (prev) { /* b64_hub_chainable() said yes */
        b64_batch *p = prev->batch;
        b->h_flags[j] |= B64X_LANE_CHAINED;
        b->h_prev[j] = p->h_res + prev->index;
        if (p != b) { /* p's records must outlive b's kernels */
            b->after = p;
            b->after_refs++;
            p->refs++;
        }
    }
    b->h_in_off[j] = b->in_used;
    b->in_used += n;
    b->h_in_off[j + 1] = b->in_used;
    b->h_out_off[j] = b->out_used;
    b->out_used += out_len;
    b->h_out_off[j + 1] = b->out_used;
    b->jobs[j] = t;
    b->refs++;
    t->batch = b;
    t->index = j;
    t->err = 0;
    t->out = NULL;
    t->out_len = 0;
    t->wake = wake;
    atomic_store_explicit(&t->done, 0, memory_order_relaxed);
    schedule_flush(h);
}

static atomic_ulong lent_total; /* segments lent, process-wide (tests) */

unsigned long b64_hub_pooled(void)
{
    pthread_mutex_lock(&pool_lock);
    unsigned long n = npool;
    pthread_mutex_unlock(&pool_lock);
    return n;
}

unsigned long b64_hub_lent_total(void)
{
    return atomic_load_explicit(&lent_total, memory_order_relaxed);
}

bool b64_hub_lend(b64_hub *h, size_t pos, const uint8_t *src, size_t n, b64_pin_slab *slab)
{
    b64_batch *b = h->depth ? h->filling[h->depth - 1] : NULL;
    if (!b || b->kind != B64_HUB_ENCODE || b->nseg == HUB_SEGS || !n)
        return false;
    const uint64_t off = b->in_used + pos;
    if (b->nseg && b->h_seg[b->nseg - 1].off + b->h_seg[b->nseg - 1].len > off)
        return false; /* out of order: never, for one gather */
    b->h_seg[b->nseg] = (b64x_seg) { off, n, src };
    b->pins[b->nseg++] = slab;
    b64_pin_ref(slab);
    atomic_fetch_add_explicit(&lent_total, 1, memory_order_relaxed);
    if (h->tr.on) {
        h->tr.lent_jobs++;
        h->tr.lent_bytes += n;
    }
    return true;
}

void b64_hub_cancel(b64_hub *h)
{
    b64_batch *b = h->filling[--h->depth];
    /* segments lent into the cancelled reservation (none in practice: a
     * block that took bytes is committed) */
    while (b && b->nseg && b->h_seg[b->nseg - 1].off >= b->in_used)
        b64_pin_unref(b->pins[--b->nseg]);
}

void b64_ticket_release(b64_ticket *t)
{
    b64_batch *b = t->batch;
    if (!b)
        return;
    t->batch = NULL;
    b->jobs[t->index] = NULL;
    if (--b->refs == 0 && b->state == B_DONE)
        batch_recycle(b->hub, b);
}
