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
    PIN_POOL = 64,       /* default idle slabs kept */
    PIN_ALIGN = 64,      /* pieces start on a cache line */
};

struct b64_pin_slab {
    uint8_t *base;
    size_t size, used;
    atomic_long refs; /* live pieces, + 1 while a thread's current slab */
    b64_pin_slab *next;
};

static pthread_once_t pin_once = PTHREAD_ONCE_INIT;
static pthread_key_t pin_key;
static pthread_mutex_t pin_lock = PTHREAD_MUTEX_INITIALIZER;
static b64_pin_slab *pin_free; /* idle slabs, refs == 0 */
static unsigned pin_nfree;
static size_t pin_slab = PIN_SLAB;
static unsigned pin_pool = PIN_POOL;
static bool pin_on = true;
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

static void slab_release(b64_pin_slab *s)
{
    s->used = 0;
    pthread_mutex_lock(&pin_lock);
    if (pin_nfree < pin_pool) {
        s->next = pin_free;
        pin_free = s;
        pin_nfree++;
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
    pin_pool = (unsigned) env_size("ASYNC_B64_PIN_POOL", PIN_POOL);
    (void) pthread_key_create(&pin_key, thread_done);
}

bool b64_pin_enabled(void)
{
    pthread_once(&pin_once, pin_init);
    return pin_on;
}

long b64_pin_live_refs(void)
{
    return atomic_load_explicit(&pin_refs, memory_order_relaxed);
}

/* An idle slab of at least `size` bytes, or a new one; refs = 0. */
static b64_pin_slab *slab_get(size_t size)
{
    b64_pin_slab *s = NULL;
    pthread_mutex_lock(&pin_lock);
    for (b64_pin_slab **p = &pin_free; *p; p = &(*p)->next) {
        if ((*p)->size >= size) {
            s = *p;
            *p = s->next;
            pin_nfree--;
            break;
        }
    }
    pthread_mutex_unlock(&pin_lock);
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
    if (!b64_pin_enabled())
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
