/*
 * b64_copy.c -- the stages' large host copies, split across helper threads
 * (see b64_copy.h).
 */
#define _GNU_SOURCE
#include "b64_copy.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum {
    COPY_MAX_HELPERS = 8,
    COPY_SPIN = 1 << 14, /* polls of a helper before it sleeps */
};

typedef struct {
    pthread_t th;
    pthread_mutex_t mu;
    pthread_cond_t cv;
    uint8_t *dst;
    const uint8_t *src;
    size_t n;
    atomic_uint seq;  /* bumped by the caller when a part is posted */
    atomic_uint done; /* = seq once the helper has copied it */
    atomic_bool sleeping;
} helper;

static pthread_once_t copy_once = PTHREAD_ONCE_INIT;
static pthread_mutex_t copy_lock = PTHREAD_MUTEX_INITIALIZER; /* one split copy at a time */
static helper helpers[COPY_MAX_HELPERS];
static unsigned nhelpers;
static size_t split_min = (size_t) 128 << 10;

static size_t env_size(const char *name, size_t dflt)
{
    const char *v = getenv(name);
    if (!v || !*v)
        return dflt;
    char *end = NULL;
    unsigned long long x = strtoull(v, &end, 0);
    return (!end || *end) ? dflt : (size_t) x;
}

static void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

static void *helper_main(void *arg)
{
    helper *h = arg;
    unsigned seen = 0;
    for (;;) {
        unsigned s;
        int spins = 0;
        while ((s = atomic_load_explicit(&h->seq, memory_order_acquire)) == seen) {
            if (++spins < COPY_SPIN) {
                cpu_relax();
                continue;
            }
            pthread_mutex_lock(&h->mu);
            atomic_store(&h->sleeping, true);
            while ((s = atomic_load(&h->seq)) == seen)
                pthread_cond_wait(&h->cv, &h->mu);
            atomic_store(&h->sleeping, false);
            pthread_mutex_unlock(&h->mu);
            break;
        }
        memcpy(h->dst, h->src, h->n);
        seen = s;
        atomic_store_explicit(&h->done, s, memory_order_release);
    }
    return NULL;
}

static void copy_init(void)
{
    unsigned want = (unsigned) env_size("ASYNC_B64_COPY_THREADS", 2);
    if (want > COPY_MAX_HELPERS)
        want = COPY_MAX_HELPERS;
    split_min = env_size("ASYNC_B64_COPY_SPLIT", split_min);
    if (split_min < 16384)
        split_min = 16384;
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    pthread_attr_setstacksize(&attr, 64 << 10);
    for (unsigned i = 0; i < want; i++) {
        helper *h = &helpers[i];
        pthread_mutex_init(&h->mu, NULL);
        pthread_cond_init(&h->cv, NULL);
        atomic_init(&h->seq, 0);
        atomic_init(&h->done, 0);
        atomic_init(&h->sleeping, false);
        if (pthread_create(&h->th, &attr, helper_main, h) != 0)
            break;
        pthread_detach(h->th);
        nhelpers++;
    }
    pthread_attr_destroy(&attr);
}

void b64_copy(void *dst, const void *src, size_t n)
{
    if (n < split_min || pthread_once(&copy_once, copy_init) != 0 || !nhelpers ||
        pthread_mutex_trylock(&copy_lock) != 0) {
        memcpy(dst, src, n);
        return;
    }
    /* parts on cache-line boundaries: the caller takes the first */
    const unsigned k = nhelpers + 1;
    const size_t part = ((n + k - 1) / k + 63) & ~(size_t) 63;  /* k parts cover n */
    uint8_t *d = dst;
    const uint8_t *s = src;
    size_t off = part < n ? part : n;
    unsigned posted = 0;
    for (unsigned i = 0; i < nhelpers && off < n; i++) {
        helper *h = &helpers[i];
        const size_t len = n - off < part ? n - off : part;
        h->dst = d + off;
        h->src = s + off;
        h->n = len;
        const unsigned seq = atomic_load_explicit(&h->seq, memory_order_relaxed) + 1;
        /* seq_cst with the helper's store of `sleeping` and load of `seq`:
         * one of the two sides sees the other's store, so a helper going to
         * sleep is either signalled or finds the part */
        atomic_store(&h->seq, seq);
        if (atomic_load(&h->sleeping)) {
            pthread_mutex_lock(&h->mu);
            pthread_cond_signal(&h->cv);
            pthread_mutex_unlock(&h->mu);
        }
        off += len;
        posted++;
    }
    memcpy(d, s, part < n ? part : n);
    for (unsigned i = 0; i < posted; i++) {
        helper *h = &helpers[i];
        const unsigned seq = atomic_load_explicit(&h->seq, memory_order_relaxed);
        while (atomic_load_explicit(&h->done, memory_order_acquire) != seq)
            cpu_relax();
    }
    pthread_mutex_unlock(&copy_lock);
}
