/*
 * b64_pin.c -- the pinned message pool (see b64_pin.h).
 */
#define _GNU_SOURCE
#include "b64_pin.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>

#include "b64x.h"

enum {
    PIN_SLAB = 32 << 20, /* default slab bytes */
    PIN_ALIGN = 64,      /* pieces start on a cache line */
};
#define PIN_IDLE_BYTES ((size_t) 2 << 30) /* default idle bytes kept */

struct b64_pin_slab {
    uint8_t *base;
    size_t size, used;
    atomic_long refs; /* live pieces, + 1 while a thread's current slab */
    b64_pin_slab *next;
};

static pthread_once_t pin_once = PTHREAD_ONCE_INIT;
static pthread_key_t pin_key;
static pthread_mutex_t pin_lock = PTHREAD_MUTEX_INITIALIZER;
static b64_pin_slab *pin_free; /* idle standard slabs, refs == 0 */
static size_t pin_idle;        /* their bytes */
static size_t pin_slab = PIN_SLAB;
static size_t pin_idle_max = PIN_IDLE_BYTES;
static bool pin_on = true;
static atomic_bool pin_active; /* a GPU stage exists (b64_pin_activate) */
static atomic_long pin_refs; /* references held on pieces (not the threads') */

static size_t env_size(const char *name, size_t dflt)
{
    const char *v = getenv(name);
    if (!v || !*v)
        return dflt;
    char *end = NULL;
    unsigned long long x = strtoull(v, &end, 0);
    return (!end || *end) ? dflt : (size_t) x;
}

/* Back to the idle list while the idle bytes stay within the cap; an
 * oversize slab (a piece of its own) is never kept. */
static void slab_release(b64_pin_slab *s)
{
    s->used = 0;
    pthread_mutex_lock(&pin_lock);
    if (s->size == pin_slab && pin_idle + s->size <= pin_idle_max) {
        s->next = pin_free;
        pin_free = s;
        pin_idle += s->size;
        s = NULL;
    }
    pthread_mutex_unlock(&pin_lock);
    if (s) {
        b64x_host_free(s->base);
        free(s);
    }
}

static void slab_unref(b64_pin_slab *s)
{
    if (atomic_fetch_sub_explicit(&s->refs, 1, memory_order_acq_rel) == 1)
        slab_release(s);
}

void b64_pin_ref(b64_pin_slab *s)
{
    atomic_fetch_add_explicit(&s->refs, 1, memory_order_relaxed);
    atomic_fetch_add_explicit(&pin_refs, 1, memory_order_relaxed);
}

void b64_pin_unref(b64_pin_slab *s)
{
    atomic_fetch_sub_explicit(&pin_refs, 1, memory_order_relaxed);
    slab_unref(s);
}

/* A thread ends: its current slab loses the thread's reference. */
static void thread_done(void *cur)
{
    if (cur)
        slab_unref(cur);
}

static void pin_init(void)
{
    pin_on = env_size("ASYNC_B64_PIN", 1) != 0;
    pin_slab = env_size("ASYNC_B64_PIN_SLAB", PIN_SLAB);
    if (pin_slab < (1u << 20))
        pin_slab = 1u << 20;
    pin_idle_max = env_size("ASYNC_B64_PIN_IDLE_BYTES", PIN_IDLE_BYTES);
    (void) pthread_key_create(&pin_key, thread_done);
}

bool b64_pin_enabled(void)
{
    pthread_once(&pin_once, pin_init);
    return pin_on;
}

void b64_pin_activate(void)
{
    atomic_store_explicit(&pin_active, true, memory_order_relaxed);
}

size_t b64_pin_idle_bytes(void)
{
    pthread_mutex_lock(&pin_lock);
    size_t n = pin_idle;
    pthread_mutex_unlock(&pin_lock);
    return n;
}

long b64_pin_live_refs(void)
{
    return atomic_load_explicit(&pin_refs, memory_order_relaxed);
}

/* An idle standard slab (size == pin_slab), or a new one; refs = 0. */
static b64_pin_slab *slab_get(size_t size)
{
    b64_pin_slab *s = NULL;
    if (size == pin_slab) {
        pthread_mutex_lock(&pin_lock);
        if ((s = pin_free)) {
            pin_free = s->next;
            pin_idle -= s->size;
        }
        pthread_mutex_unlock(&pin_lock);
    }
    if (!s) {
        s = calloc(1, sizeof *s);
        if (!s)
            return NULL;
        s->base = b64x_host_alloc(size);
        if (!s->base) {
            free(s);
            return NULL;
        }
        s->size = size;
    }
    s->used = 0;
    s->next = NULL;
    atomic_store_explicit(&s->refs, 0, memory_order_relaxed);
    return s;
}

void *b64_pin_alloc(size_t n, b64_pin_slab **slab)
{
    if (!b64_pin_enabled() || !atomic_load_explicit(&pin_active, memory_order_relaxed))
        return NULL;
    const size_t need = (n + PIN_ALIGN - 1) / PIN_ALIGN * PIN_ALIGN;
    if (need > pin_slab / 4) { /* a slab of its own */
        b64_pin_slab *s = slab_get(need);
        if (!s)
            return NULL;
        s->used = need;
        b64_pin_ref(s);
        *slab = s;
        return s->base;
    }
    b64_pin_slab *cur = pthread_getspecific(pin_key);
    if (!cur || cur->size - cur->used < need) {
        b64_pin_slab *s = slab_get(pin_slab);
        if (!s)
            return NULL;
        atomic_store_explicit(&s->refs, 1, memory_order_relaxed); /* the thread's */
        if (cur)
            slab_unref(cur);
        cur = s;
        (void) pthread_setspecific(pin_key, cur);
    }
    void *p = cur->base + cur->used;
    cur->used += need;
    b64_pin_ref(cur);
    *slab = cur;
    return p;
}
