/*
 * fake_b64x.c -- TEST INFRASTRUCTURE ONLY (never part of the product).
 *
 * A CPU stand-in for the GPU side of the b64x C ABI (include/b64x.h): the
 * sessions and lanes the bytestream_1 stages (async_amd/csrc/b64_stages.c)
 * and the batching hub (b64_hub.c) drive.  Linked with the product's own
 * host C (loop, streams, framing, hub, stages) and the test harness into
 * tests/csrc/libstage_fake.so, it makes the stages' slot accounting and
 * completion handling testable on a machine without a GPU, with the
 * interleavings chosen by a seeded generator instead of by the hardware:
 *
 *  - work is computed when it is queued (the oracle's decode table and
 *    encoder), but *published* -- output bytes copied to the host buffers,
 *    the result record / per-job counts written, then the completion
 *    callback run -- by worker threads that pick, at random, any queued
 *    job that is first on its session or lane (each keeps its own order;
 *    different ones complete in any order);
 *  - "early" jobs (probability fake_configure(..., early_pct)) run their
 *    callback first and leave publication until someone waits for their
 *    session or lane (b64x_session_wait / b64x_lane_wait), or the owner's
 *    next job is launched or starts to run, or the owner is released: the
 *    failure of round 1, where a decode's result record did not hold the
 *    launch's values when its completion callback ran;
 *  - raw mode stands for the round-1 stage: b64x_session_decode_result and
 *    b64x_lane_decode_check return what is there without checking (and
 *    nothing is poisoned), so an early job's block is read as the previous
 *    call's record;
 *  - "zero" mode: an early job publishes an all-zero record before its
 *    callback (what round 1's stage once served: a well-formed "nothing
 *    decoded" record, profiles/r02_diag_notes.md), and the real one later;
 *  - "torn" mode: an early job publishes its record's every field but the
 *    held-back sextets tail[] before its callback (a record
 *    whose tail_n landed before its tail bytes).
 *
 * b64x_session_decode_result / b64x_lane_decode_check otherwise run the
 * library's own check (async_amd/csrc/b64x_result_check.h).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include "b64_oracle.h"
#include "b64x.h"
#include "b64x_result_check.h"

/* ------------------------------------------------------------ the "device" */

typedef struct fjob fjob;
struct fjob {
    fjob *next;
    void *owner;             /* session or lane: completes in its own order */
    bool early;              /* callback before publication */
    bool called;             /* callback has run (early jobs) */
    uint8_t *out_dst;        /* publish: out bytes -> out_dst */
    uint8_t *out_src;
    size_t out_n;
    b64x_dec_result *res_dst;/* publish: the result record */
    b64x_dec_result res;
    b64x_dec_result *recs_dst; /* publish: per-job records */
    b64x_dec_result *recs;
    b64x_dec_result *spells_dst; /* publish: chained jobs' spell logs */
    b64x_dec_result *spells;
    uint32_t njobs;
    uint64_t *stamp_dst;     /* publish: a lane's completion stamp */
    uint64_t stamp;
    b64x_done_fn done;
    void *arg;
    /* lane encode batches run when a worker takes them (reading their
     * inputs then, as the device would): */
    const uint8_t *enc_in;
    uint64_t *enc_in_off, *enc_out_off; /* copies */
    b64x_seg *enc_seg;                  /* copy, or NULL */
    uint32_t enc_jobs, enc_nseg;
    b64x_alphabet enc_abc;
};

/* The device copy of the batch: the arena with the lent segments laid
 * over it (read now, as the gather kernel would when the batch runs). */
static void run_encode(fjob *j)
{
    const uint64_t total = j->enc_in_off[j->enc_jobs];
    uint8_t *dev = malloc(total + 1);
    memcpy(dev, j->enc_in, total);
    for (uint32_t i = 0; i < j->enc_nseg; i++)
        memcpy(dev + j->enc_seg[i].off, j->enc_seg[i].src, j->enc_seg[i].len);
    for (uint32_t k = 0; k < j->enc_jobs; k++) {
        size_t n = j->enc_in_off[k + 1] - j->enc_in_off[k];
        (void) orc_encode(dev + j->enc_in_off[k], n, j->enc_abc.pos62, j->enc_abc.pos63,
                          j->enc_abc.pad, j->enc_abc.padchar, j->out_src + j->enc_out_off[k]);
    }
    free(dev);
}

static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t cv = PTHREAD_COND_INITIALIZER;
static fjob *queue_head;     /* queued, not yet taken by a worker */
static fjob *parked;         /* early jobs: called back, not yet published */
static unsigned busy;        /* jobs a worker is processing */
static void *busy_owner[64];
static pthread_t workers[8];
static unsigned nworkers;
static bool stopping;
static uint64_t rng_state = 1;
static unsigned early_pct;
static bool raw_mode;
enum { MODE_CHECKED = 0, MODE_RAW = 1, MODE_ZERO = 2, MODE_TORN = 3 };
static int fake_mode;
static atomic_uint g_seq;

static uint32_t next_seq(void)
{
    uint32_t v;
    do
        v = atomic_fetch_add(&g_seq, 1) + 1;
    while (v == 0);
    return v;
}
static atomic_ulong n_early, n_jobs, n_chained;

static uint64_t rnd(void) /* splitmix64, under mu */
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* What an early job shows before its callback in zero / torn mode. */
static void publish_early_record(b64x_dec_result *dst, const b64x_dec_result *r)
{
    if (fake_mode == MODE_ZERO) {
        memset(dst, 0, sizeof *dst);
    } else if (fake_mode == MODE_TORN) {
        volatile b64x_dec_result *v = dst;
        v->out_len = r->out_len;
        v->valid = r->valid;
        v->tail_n = r->tail_n;
        v->nchars = r->nchars;
        v->seq = r->seq;
        v->flags = r->flags; /* tail[] left as it was */
    }
}

static void publish_early(fjob *j)
{
    if (j->res_dst)
        publish_early_record(j->res_dst, &j->res);
    for (uint32_t k = 0; j->recs_dst && k < j->njobs; k++)
        publish_early_record(j->recs_dst + k, j->recs + k);
}

static void publish(fjob *j)
{
    if (j->out_n)
        memcpy(j->out_dst, j->out_src, j->out_n);
    if (j->res_dst)
        *j->res_dst = j->res;
    if (j->recs_dst)
        memcpy(j->recs_dst, j->recs, (size_t) j->njobs * sizeof *j->recs);
    if (j->spells_dst)
        memcpy(j->spells_dst, j->spells, (size_t) j->njobs * sizeof *j->spells);
    if (j->stamp_dst)
        *(volatile uint64_t *) j->stamp_dst = j->stamp;
}

static void job_free(fjob *j)
{
    free(j->enc_in_off);
    free(j->enc_out_off);
    free(j->enc_seg);
    free(j->out_src);
    free(j->recs);
    free(j->spells);
    free(j);
}

static bool owner_busy(void *owner)
{
    for (unsigned i = 0; i < 64; i++)
        if (busy_owner[i] == owner)
            return true;
    return false;
}

static void flush_parked(void *owner);

static void *worker(void *unused)
{
    (void) unused;
    pthread_mutex_lock(&mu);
    for (;;) {
        /* candidates: first queued job of an owner no worker is running */
        fjob *cand[64];
        unsigned nc = 0;
        for (fjob *j = queue_head; j && nc < 64; j = j->next) {
            bool first = !owner_busy(j->owner);
            for (fjob *k = queue_head; k != j && first; k = k->next)
                if (k->owner == j->owner)
                    first = false;
            if (first)
                cand[nc++] = j;
        }
        if (!nc) {
            if (stopping)
                break;
            pthread_cond_wait(&cv, &mu);
            continue;
        }
        fjob *j = cand[rnd() % nc];
        for (fjob **p = &queue_head; *p; p = &(*p)->next)
            if (*p == j) {
                *p = j->next;
                break;
            }
        flush_parked(j->owner); /* the owner's previous job lands before this one runs */
        unsigned slot = 0;
        while (busy_owner[slot])
            slot++;
        busy_owner[slot] = j->owner;
        busy++;
        bool early = j->early;
        unsigned spin = (unsigned) (rnd() % 50);
        pthread_mutex_unlock(&mu);
        for (volatile unsigned i = 0; i < spin * 100; i++)
            ;
        if (j->enc_jobs)
            run_encode(j);
        if (early) {
            atomic_fetch_add(&n_early, 1);
            j->called = true;
            publish_early(j);
            if (j->done)
                j->done(j->arg); /* callback first: the round-1 hazard */
            pthread_mutex_lock(&mu);
            j->next = parked;
            parked = j;
        } else {
            publish(j);
            if (j->done)
                j->done(j->arg);
            pthread_mutex_lock(&mu);
            job_free(j);
        }
        busy_owner[slot] = NULL;
        busy--;
        pthread_cond_broadcast(&cv);
    }
    pthread_mutex_unlock(&mu);
    return NULL;
}

static void start_workers(void)
{
    if (nworkers)
        return;
    stopping = false;
    for (unsigned i = 0; i < 2; i++)
        pthread_create(&workers[nworkers++], NULL, worker, NULL);
}

/* Publish `owner`'s parked jobs (under mu). */
static void flush_parked(void *owner)
{
    for (fjob **p = &parked; *p;) {
        fjob *j = *p;
        if (j->owner == owner) {
            *p = j->next;
            publish(j);
            job_free(j);
        } else {
            p = &j->next;
        }
    }
}

static void owner_wait(void *owner)
{
    pthread_mutex_lock(&mu);
    for (;;) {
        bool pending = owner_busy(owner);
        for (fjob *j = queue_head; j && !pending; j = j->next)
            pending = j->owner == owner;
        if (!pending)
            break;
        pthread_cond_wait(&cv, &mu);
    }
    flush_parked(owner);
    pthread_mutex_unlock(&mu);
}

static void submit(fjob *j)
{
    pthread_mutex_lock(&mu);
    start_workers();
    flush_parked(j->owner); /* a new launch: the previous one has landed */
    j->early = early_pct && rnd() % 100 < early_pct;
    j->next = NULL;
    fjob **p = &queue_head;
    while (*p)
        p = &(*p)->next;
    *p = j;
    atomic_fetch_add(&n_jobs, 1);
    pthread_cond_broadcast(&cv);
    pthread_mutex_unlock(&mu);
}

/* Test control: seed, % of early jobs, mode (0 checked, 1 raw round-1
 * reads, 2 zero records, 3 torn tails).  Waits for the device to go idle
 * first. */
void fake_configure(uint64_t seed, unsigned pct, int mode)
{
    pthread_mutex_lock(&mu);
    while (queue_head || busy)
        pthread_cond_wait(&cv, &mu);
    while (parked) {
        fjob *j = parked;
        parked = j->next;
        publish(j);
        job_free(j);
    }
    rng_state = seed ? seed : 1;
    early_pct = pct;
    raw_mode = mode == MODE_RAW;
    fake_mode = mode;
    pthread_mutex_unlock(&mu);
}

/* chained lane jobs (heads spelled "on the device") since load */
uint64_t fake_chained(void)
{
    return atomic_load(&n_chained);
}

/* jobs queued and early ones since load */
void fake_stats(uint64_t out[2])
{
    out[0] = atomic_load(&n_jobs);
    out[1] = atomic_load(&n_early);
}

/* ------------------------------------------------------------- the b64x ABI */

static atomic_ulong g_early_session, g_early_lane;

uint64_t b64x_encoded_len(uint64_t n, bool pad)
{
    return pad ? (n + 2) / 3 * 4 : (n * 4 + 2) / 3;
}

uint64_t b64x_decoded_cap(uint64_t nchars)
{
    return (nchars + 3) / 4 * 3;
}

int b64x_device_check(void)
{
    return 0;
}

/* No device, no node: the hub's binding leaves the thread as it is. */
int b64x_bind_thread(int device)
{
    (void) device;
    return -ENOENT;
}

/* Pinned buffers stand-in: the allocation ends (64-byte aligned) right
 * before an inaccessible page, so that a write past a buffer's end faults
 * here as it does against the real pinned mappings (calloc'd buffers let
 * an arena overrun go unnoticed). */
static atomic_ullong g_host_bytes, g_host_allocs; /* live "pinned" bytes; allocations */

void *b64x_host_alloc(uint64_t bytes)
{
    const size_t pg = 4096, need = ((bytes ? bytes : 1) + 63) / 64 * 64;
    const size_t data = (need + 16 + pg - 1) / pg * pg, total = data + pg;
    uint8_t *base = mmap(NULL, total, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED)
        return NULL;
    if (mprotect(base + data, pg, PROT_NONE) != 0) {
        munmap(base, total);
        return NULL;
    }
    uint8_t *p = base + data - need;
    ((size_t *) p)[-2] = (size_t) base;
    ((size_t *) p)[-1] = total;
    atomic_fetch_add(&g_host_bytes, total);
    atomic_fetch_add(&g_host_allocs, 1);
    return p;
}

void b64x_host_free(void *p)
{
    if (!p)
        return;
    atomic_fetch_sub(&g_host_bytes, ((size_t *) p)[-1]);
    munmap((void *) ((size_t *) p)[-2], ((size_t *) p)[-1]);
}

/* Tests: pinned-stand-in bytes live now, and allocations ever made. */
void fake_host_stats(uint64_t out[2])
{
    out[0] = atomic_load(&g_host_bytes);
    out[1] = atomic_load(&g_host_allocs);
}

void b64x_diag_counters(uint64_t out[2])
{
    out[0] = atomic_load(&g_early_session);
    out[1] = atomic_load(&g_early_lane);
}

/* The decoder's character map for an alphabet (ref map(),
 * src/base64decoder.c:38-48, via the oracle's table). */
static void dec_table(const b64x_alphabet *abc, int8_t t[256])
{
    orc_decode_table(abc->pos62, abc->pos63, t);
}

static const char *kStd = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";

/* Decode `pre` sextets then chars[0..n): whole groups (hold) or
 * floor(6V/8) bytes; returns the record. */
static b64x_dec_result decode_bits(const uint8_t *chars, size_t n, const b64x_alphabet *abc,
                                   bool hold, uint32_t seq, uint8_t *out)
{
    int8_t t[256];
    dec_table(abc, t);
    b64x_dec_result r;
    memset(&r, 0, sizeof r);
    uint64_t V = 0, bits = 0, nb = 0, olen = 0;
    uint8_t last[4] = {0, 0, 0, 0};
    for (size_t i = 0; i < n; i++) {
        int v = t[chars[i]];
        if (v < 0)
            continue;
        last[V & 3] = (uint8_t) v;
        V++;
        bits = (bits << 6) | (uint64_t) v;
        nb += 6;
        if (nb >= 8) {
            nb -= 8;
            out[olen++] = (uint8_t) (bits >> nb);
        }
    }
    r.valid = V;
    r.tail_n = (uint32_t) (V & 3);
    r.out_len = hold ? V / 4 * 3 : V * 6 / 8;
    for (uint32_t k = 0; k < r.tail_n; k++)
        r.tail[k] = last[(V - r.tail_n + k) & 3];
    r.nchars = n;
    r.seq = seq;
    r.flags = hold ? 1u : 0u;
    (void) olen; /* the first out_len bytes are the stream's; the rest is scratch */
    return r;
}

struct b64x_session {
    uint64_t cap;
    uint8_t *h_in, *h_out;
    b64x_dec_result h_res;   /* the host-visible record */
    uint64_t res_len;
    unsigned res_flags;
    uint32_t res_seq;
};

static b64x_session *spool[64];
static int nspool;
static pthread_mutex_t spool_mu = PTHREAD_MUTEX_INITIALIZER;

b64x_session *b64x_session_open(uint64_t capacity)
{
    b64x_session *s = calloc(1, sizeof *s);
    s->cap = capacity;
    s->h_in = calloc(1, capacity + 64);
    s->h_out = calloc(1, (capacity + 16 + 3) / 4 * 3 + 64);
    return s;
}

void b64x_session_close(b64x_session *s)
{
    if (!s)
        return;
    owner_wait(s);
    free(s->h_in);
    free(s->h_out);
    free(s);
}

b64x_session *b64x_session_acquire(uint64_t capacity)
{
    pthread_mutex_lock(&spool_mu);
    for (int i = nspool - 1; i >= 0; i--) {
        if (spool[i]->cap == capacity) {
            b64x_session *s = spool[i];
            spool[i] = spool[--nspool];
            pthread_mutex_unlock(&spool_mu);
            return s; /* keeps its last record: a stale one, as pooled GPU sessions do */
        }
    }
    pthread_mutex_unlock(&spool_mu);
    return b64x_session_open(capacity);
}

void b64x_session_release(b64x_session *s)
{
    if (!s)
        return;
    owner_wait(s);
    pthread_mutex_lock(&spool_mu);
    if (nspool < 64) {
        spool[nspool++] = s;
        s = NULL;
    }
    pthread_mutex_unlock(&spool_mu);
    if (s)
        b64x_session_close(s);
}

uint8_t *b64x_session_host_in(b64x_session *s)
{
    return s->h_in;
}

uint8_t *b64x_session_host_out(b64x_session *s)
{
    return s->h_out;
}

int b64x_session_wait(b64x_session *s)
{
    owner_wait(s);
    return 0;
}

int b64x_session_decode_async(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                              unsigned flags, b64x_done_fn done, void *arg)
{
    if (!s || n > s->cap)
        return -EINVAL;
    fjob *j = calloc(1, sizeof *j);
    j->owner = s;
    j->out_src = malloc(b64x_decoded_cap(n + 4) + 16);
    s->res_seq = next_seq();
    j->res = decode_bits(s->h_in, n, abc, flags & B64X_DEC_HOLD_TAIL, s->res_seq, j->out_src);
    j->out_n = j->res.out_len;
    j->out_dst = s->h_out;
    j->res_dst = &s->h_res;
    j->done = done;
    j->arg = arg;
    s->res_len = n;
    s->res_flags = flags;
    pthread_mutex_lock(&mu);
    flush_parked(s); /* the previous launch lands before the poison */
    pthread_mutex_unlock(&mu);
    if (!raw_mode)
        b64x_poison_result(&s->h_res);
    submit(j);
    return 0;
}

int b64x_session_encode_async(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                              b64x_done_fn done, void *arg)
{
    (void) s;
    (void) n;
    (void) abc;
    (void) done;
    (void) arg;
    return -ENOSYS; /* the stages encode through the hub */
}

const b64x_dec_result *b64x_session_result(const b64x_session *s)
{
    return &s->h_res;
}

int b64x_session_decode_result(b64x_session *s, b64x_dec_result *res)
{
    if (raw_mode) { /* round 1: whatever the record holds */
        *res = *(volatile b64x_dec_result *) &s->h_res;
        return 0;
    }
    if (b64x_result_ok(&s->h_res, s->res_len, s->res_flags, s->res_seq, res))
        return 0;
    atomic_fetch_add(&g_early_session, 1);
    owner_wait(s);
    return b64x_result_ok(&s->h_res, s->res_len, s->res_flags, s->res_seq, res) ? 0 : -EIO;
}

struct b64x_lane {
    uint64_t stamp; /* the "host memory" stamp, published with a batch */
    uint64_t seq;   /* the last encode batch queued */
};

b64x_lane *b64x_lane_acquire(void)
{
    return calloc(1, sizeof(b64x_lane));
}

void b64x_lane_release(b64x_lane *l)
{
    if (!l)
        return;
    owner_wait(l);
    free(l);
}

int b64x_lane_wait(b64x_lane *l)
{
    owner_wait(l);
    return 0;
}

int b64x_lane_encode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const b64x_seg *h_seg, uint32_t nseg,
                           const b64x_alphabet *abc, b64x_done_fn done, void *arg)
{
    fjob *j = calloc(1, sizeof *j);
    j->owner = l;
    size_t total = njobs ? h_out_off[njobs] : 0;
    j->out_src = malloc(total + 16);
    if (njobs) {
        j->enc_in = h_in;
        j->enc_jobs = njobs;
        j->enc_abc = *abc;
        j->enc_in_off = malloc((njobs + 1) * sizeof *j->enc_in_off);
        j->enc_out_off = malloc((njobs + 1) * sizeof *j->enc_out_off);
        memcpy(j->enc_in_off, h_in_off, (njobs + 1) * sizeof *h_in_off);
        memcpy(j->enc_out_off, h_out_off, (njobs + 1) * sizeof *h_out_off);
        for (uint32_t i = 0; i < nseg; i++)
            if (h_seg[i].off + h_seg[i].len > h_in_off[njobs] ||
                (i && h_seg[i].off < h_seg[i - 1].off + h_seg[i - 1].len))
                abort(); /* the hub's segments are sorted, inside the batch */
        if (nseg) {
            j->enc_seg = malloc(nseg * sizeof *j->enc_seg);
            memcpy(j->enc_seg, h_seg, nseg * sizeof *h_seg);
            j->enc_nseg = nseg;
        }
    }
    j->out_dst = h_out;
    j->out_n = total;
    j->stamp_dst = &l->stamp;
    j->stamp = ++l->seq;
    j->done = done;
    j->arg = arg;
    submit(j);
    return 0;
}

int b64x_lane_encode_check(b64x_lane *l)
{
    if (raw_mode || *(volatile uint64_t *) &l->stamp == l->seq)
        return 0;
    atomic_fetch_add(&g_early_lane, 1);
    owner_wait(l);
    return *(volatile uint64_t *) &l->stamp == l->seq ? 0 : -EIO;
}

/* The records the device has computed, by the host address they will be
 * published to: a chained job reads its predecessor's record on the
 * device after that one has been decoded, whether or not the host has it
 * yet (ordered on the lane).  Open addressing, overwritten on reuse. */
enum { REG_SIZE = 1 << 18 };
static struct {
    const b64x_dec_result *addr;
    b64x_dec_result rec;
} reg[REG_SIZE];
static pthread_mutex_t reg_mu = PTHREAD_MUTEX_INITIALIZER;

static size_t reg_slot(const b64x_dec_result *addr)
{
    size_t i = ((uintptr_t) addr >> 3) * 0x9E3779B97F4A7C15ull >> 46;
    while (reg[i].addr && reg[i].addr != addr)
        i = (i + 1) & (REG_SIZE - 1);
    return i;
}

static void reg_put(const b64x_dec_result *addr, const b64x_dec_result *r)
{
    pthread_mutex_lock(&reg_mu);
    size_t i = reg_slot(addr);
    reg[i].addr = addr;
    reg[i].rec = *r;
    pthread_mutex_unlock(&reg_mu);
}

static bool reg_get(const b64x_dec_result *addr, b64x_dec_result *r)
{
    pthread_mutex_lock(&reg_mu);
    size_t i = reg_slot(addr);
    bool ok = reg[i].addr == addr;
    if (ok)
        *r = reg[i].rec;
    pthread_mutex_unlock(&reg_mu);
    return ok;
}

int b64x_lane_decode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const uint8_t *h_flags,
                           b64x_dec_result *h_res, const b64x_dec_result *const *h_prev,
                           b64x_dec_result *h_spell, const b64x_alphabet *abc,
                           b64x_done_fn done, void *arg, uint32_t *seq)
{
    fjob *j = calloc(1, sizeof *j);
    j->owner = l;
    size_t total = njobs ? h_out_off[njobs] : 0;
    j->out_src = malloc(total + 16);
    j->recs = calloc(njobs ? njobs : 1, sizeof *j->recs);
    j->spells = calloc(njobs ? njobs : 1, sizeof *j->spells);
    *seq = next_seq();
    bool chained_any = false;
    for (uint32_t k = 0; k < njobs; k++) {
        size_t n = h_in_off[k + 1] - h_in_off[k];
        const uint8_t *src = h_in + h_in_off[k];
        uint8_t *tmp = NULL;
        if (h_flags[k] & B64X_LANE_CHAINED) {
            /* the device spells the predecessor's held-back sextets into
             * the head (k_spell_head) after that one's decode */
            chained_any = true;
            atomic_fetch_add(&n_chained, 1);
            b64x_dec_result p;
            if (!h_prev || !h_prev[k] || n < 4 || !reg_get(h_prev[k], &p))
                return -EINVAL;
            j->spells[k] = p;
            tmp = malloc(n);
            memcpy(tmp, src, n);
            const char *p62 = abc->pos62 == (char) -1 ? "+" : &abc->pos62;
            const char *p63 = abc->pos63 == (char) -1 ? "/" : &abc->pos63;
            for (uint32_t i = 0; i < p.tail_n && i < 4; i++) {
                uint8_t v = p.tail[i];
                tmp[4 - p.tail_n + i] = v < 62 ? (uint8_t) kStd[v] : (uint8_t) (v == 62 ? *p62 : *p63);
            }
            src = tmp;
        }
        j->recs[k] = decode_bits(src, n, abc, h_flags[k] & B64X_DEC_HOLD_TAIL, *seq,
                                 j->out_src + h_out_off[k]);
        reg_put(h_res + k, &j->recs[k]);
        free(tmp);
    }
    j->out_dst = h_out;
    j->out_n = total;
    j->recs_dst = h_res;
    j->spells_dst = chained_any ? h_spell : NULL;
    j->njobs = njobs;
    j->done = done;
    j->arg = arg;
    if (!raw_mode)
        for (uint32_t k = 0; k < njobs; k++)
            b64x_poison_result(h_res + k);
    submit(j);
    return 0;
}

static bool jobs_ok(uint32_t seq, const uint64_t *h_in_off, const uint8_t *h_flags,
                    const b64x_dec_result *h_res, const b64x_dec_result *const *h_prev,
                    const b64x_dec_result *h_spell, uint32_t njobs)
{
    for (uint32_t k = 0; k < njobs; k++) {
        if (!b64x_result_ok(h_res + k, h_in_off[k + 1] - h_in_off[k], h_flags[k], seq, NULL))
            return false;
        if ((h_flags[k] & B64X_LANE_CHAINED) && !b64x_spell_ok(h_spell + k, h_prev[k]))
            return false;
    }
    return true;
}

int b64x_lane_decode_check(b64x_lane *l, uint32_t seq, const uint64_t *h_in_off,
                           const uint8_t *h_flags, const b64x_dec_result *h_res,
                           const b64x_dec_result *const *h_prev,
                           const b64x_dec_result *h_spell, uint32_t njobs)
{
    if (raw_mode || jobs_ok(seq, h_in_off, h_flags, h_res, h_prev, h_spell, njobs))
        return 0;
    atomic_fetch_add(&g_early_lane, 1);
    owner_wait(l);
    return jobs_ok(seq, h_in_off, h_flags, h_res, h_prev, h_spell, njobs) ? 0 : -EIO;
}

/* The product's record check on a caller's record (tests/test_stage_fake.py
 * checks what it accepts and rejects). */
int fake_result_ok(const b64x_dec_result *r, uint64_t len, unsigned flags, uint32_t seq)
{
    return b64x_result_ok(r, len, flags, seq, NULL);
}

void fake_poison(b64x_dec_result *r)
{
    b64x_poison_result(r);
}

/* The harness's multi-GPU driver asks the HIP runtime for devices. */
int hipSetDevice(int device)
{
    return device == 0 ? 0 : 1;
}

int hipGetDeviceCount(int *count)
{
    *count = 1;
    return 0;
}

/* unused by the stages; keeps the alphabet string referenced */
const char *fake_b64x_alphabet(void)
{
    return kStd;
}
