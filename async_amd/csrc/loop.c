/*
 * loop.c -- minimal single-threaded event loop (include/async.h).
 *
 * Scope: only what the base64 stages and their test/bench topologies need
 * (SURVEY.md §8(f) row f4).  The reference's loop (src/async.c) is an
 * epoll/kqueue multiplexer with timers, immediate tasks, deferred frees
 * and cross-thread notification; here:
 *
 *  - timers sit in a binary min-heap ordered by (expiry, sequence
 *    number); immediate tasks (async_execute(), ref src/async.c:376-383)
 *    in a FIFO list that runs before any due timer -- the order of a
 *    single heap in which they expire at 0, without its O(log n) cost
 *    when tens of thousands of streams share a loop; task records are
 *    recycled through a free list;
 *  - async_wound() queues the object and schedules a task that frees the
 *    oldest wounded object with fsfree(), so a free happens only after
 *    every task that was already scheduled (ref src/async.c:386-392);
 *    destroy_async() frees the ones still queued (ref :140-162).  Every
 *    object of the loop itself comes from fsalloc() (include/fsalloc.h),
 *    so a counting allocator sees the loop's objects come and go;
 *  - at most kBurst due tasks run before the loop polls file descriptors
 *    (ref take_immediate_action, src/async.c:564-590, uses 20);
 *  - async_register() has the reference's contract (include/async.h,
 *    src/async.c:733-760): the descriptor is made non-blocking and watched
 *    edge-triggered for EPOLLIN | EPOLLOUT, so the action runs when the
 *    descriptor's state changes and is guaranteed only after a read or
 *    write on it has returned EAGAIN (a registration itself may bring one
 *    spurious call).  The GPU completion eventfd of the stages goes through
 *    it; its action drains the eventfd to EAGAIN (b64_hub.c hub_wake), as
 *    the reference's notification probe drains its pipe
 *    (src/notification.c:24-43).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <time.h>
#include <unistd.h>

#include "async.h"
#include "fsalloc.h"

enum { kBurst = 20, kMaxEvents = 16 };

struct async_timer {
    uint64_t expires;
    uint64_t seq;
    action_1 action;
    size_t slot; /* index in the heap; kInFifo: an immediate task */
    struct async_timer *prev, *next; /* FIFO links; next: free list */
};

#define kInFifo ((size_t) -1)
enum { kFreeMax = 4096 };

struct wounded {
    void *object;
    struct wounded *next;
};

struct fd_watch {
    int fd;
    bool pending; /* an edge arrived after the loop was told to quit */
    action_1 action;
    struct fd_watch *next;
};

struct async {
    int epfd;
    async_timer_t **heap;
    size_t nheap, capheap;
    async_timer_t *fifo_head, *fifo_tail; /* immediate tasks */
    async_timer_t *free_list;
    size_t nfree;
    uint64_t seq;
    bool quit;
    bool pending_scheduled; /* deliver_pending() is queued */
    struct wounded *wound_head, *wound_tail;
    struct fd_watch *watches;
};

uint64_t async_now(async_t *async)
{
    (void) async;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t) ts.tv_sec * 1000000000ull + (uint64_t) ts.tv_nsec;
}

static bool earlier(const async_timer_t *a, const async_timer_t *b)
{
    return a->expires < b->expires ||
           (a->expires == b->expires && a->seq < b->seq);
}

static void heap_place(async_t *async, size_t i, async_timer_t *t)
{
    async->heap[i] = t;
    t->slot = i;
}

static void sift_up(async_t *async, size_t i)
{
    async_timer_t *t = async->heap[i];
    while (i > 0) {
        size_t parent = (i - 1) / 2;
        if (!earlier(t, async->heap[parent]))
            break;
        heap_place(async, i, async->heap[parent]);
        i = parent;
    }
    heap_place(async, i, t);
}

static void sift_down(async_t *async, size_t i)
{
    async_timer_t *t = async->heap[i];
    for (;;) {
        size_t c = 2 * i + 1;
        if (c >= async->nheap)
            break;
        if (c + 1 < async->nheap && earlier(async->heap[c + 1], async->heap[c]))
            c++;
        if (!earlier(async->heap[c], t))
            break;
        heap_place(async, i, async->heap[c]);
        i = c;
    }
    heap_place(async, i, t);
}

static void heap_remove(async_t *async, size_t i)
{
    async_timer_t *last = async->heap[--async->nheap];
    if (i == async->nheap)
        return;
    heap_place(async, i, last);
    if (i > 0 && earlier(last, async->heap[(i - 1) / 2]))
        sift_up(async, i);
    else
        sift_down(async, i);
}

async_t *make_async(void)
{
    async_t *async = fscalloc(1, sizeof *async);
    async->epfd = epoll_create1(EPOLL_CLOEXEC);
    if (async->epfd < 0) {
        int e = errno;
        fsfree(async);
        errno = e;
        return NULL;
    }
    return async;
}

static void run_wound_task(async_t *async)
{
    struct wounded *w = async->wound_head;
    if (!w)
        return;
    async->wound_head = w->next;
    if (!async->wound_head)
        async->wound_tail = NULL;
    fsfree(w->object);
    fsfree(w);
}

void destroy_async(async_t *async)
{
    if (!async)
        return;
    for (size_t i = 0; i < async->nheap; i++)
        fsfree(async->heap[i]);
    fsfree(async->heap);
    while (async->fifo_head) {
        async_timer_t *t = async->fifo_head;
        async->fifo_head = t->next;
        fsfree(t);
    }
    while (async->free_list) {
        async_timer_t *t = async->free_list;
        async->free_list = t->next;
        fsfree(t);
    }
    while (async->wound_head)
        run_wound_task(async);
    while (async->watches) {
        struct fd_watch *w = async->watches;
        async->watches = w->next;
        fsfree(w);
    }
    close(async->epfd);
    fsfree(async);
}

static async_timer_t *task_new(async_t *async)
{
    async_timer_t *t = async->free_list;
    if (t) {
        async->free_list = t->next;
        async->nfree--;
        return t;
    }
    return fsalloc(sizeof *t);
}

static void task_free(async_t *async, async_timer_t *t)
{
    if (async->nfree < kFreeMax) {
        t->next = async->free_list;
        async->free_list = t;
        async->nfree++;
    } else {
        fsfree(t);
    }
}

static void fifo_unlink(async_t *async, async_timer_t *t)
{
    if (t->prev)
        t->prev->next = t->next;
    else
        async->fifo_head = t->next;
    if (t->next)
        t->next->prev = t->prev;
    else
        async->fifo_tail = t->prev;
}

async_timer_t *async_timer_start(async_t *async, uint64_t expires,
                                 action_1 action)
{
    if (async->nheap == async->capheap) {
        size_t cap = async->capheap ? 2 * async->capheap : 64;
        async_timer_t **h = fsalloc(cap * sizeof *h);
        if (async->nheap)
            memcpy(h, async->heap, async->nheap * sizeof *h);
        fsfree(async->heap);
        async->heap = h;
        async->capheap = cap;
    }
    async_timer_t *t = task_new(async);
    t->expires = expires;
    t->seq = async->seq++;
    t->action = action;
    heap_place(async, async->nheap++, t);
    sift_up(async, async->nheap - 1);
    return t;
}

void async_timer_cancel(async_t *async, async_timer_t *timer)
{
    if (timer->slot == kInFifo)
        fifo_unlink(async, timer);
    else
        heap_remove(async, timer->slot);
    task_free(async, timer);
}

async_timer_t *async_execute(async_t *async, action_1 action)
{
    async_timer_t *t = task_new(async);
    t->expires = 0;
    t->seq = async->seq++;
    t->action = action;
    t->slot = kInFifo;
    t->next = NULL;
    t->prev = async->fifo_tail;
    if (async->fifo_tail)
        async->fifo_tail->next = t;
    else
        async->fifo_head = t;
    async->fifo_tail = t;
    return t;
}

void async_wound(async_t *async, void *object)
{
    struct wounded *w = fsalloc(sizeof *w);
    w->object = object;
    w->next = NULL;
    if (async->wound_tail)
        async->wound_tail->next = w;
    else
        async->wound_head = w;
    async->wound_tail = w;
    async_execute(async, (action_1) { async, (act_1) run_wound_task });
}

void async_quit_loop(async_t *async)
{
    async->quit = true;
}

static struct fd_watch *find_watch(async_t *async, int fd)
{
    for (struct fd_watch *w = async->watches; w; w = w->next)
        if (w->fd == fd)
            return w;
    return NULL;
}

int async_register(async_t *async, int fd, action_1 action)
{
    int fl = fcntl(fd, F_GETFL, 0);
    if (fl < 0 || (!(fl & O_NONBLOCK) && fcntl(fd, F_SETFL, fl | O_NONBLOCK) < 0))
        return -1;
    struct fd_watch *w = find_watch(async, fd);
    if (w) {
        w->action = action;
        return 0;
    }
    struct epoll_event ev;
    memset(&ev, 0, sizeof ev);
    ev.events = EPOLLIN | EPOLLOUT | EPOLLET;
    ev.data.fd = fd;
    if (epoll_ctl(async->epfd, EPOLL_CTL_ADD, fd, &ev) < 0)
        return -1;
    w = fsalloc(sizeof *w);
    w->fd = fd;
    w->pending = false;
    w->action = action;
    w->next = async->watches;
    async->watches = w;
    return 0;
}

int async_unregister(async_t *async, int fd)
{
    for (struct fd_watch **p = &async->watches; *p; p = &(*p)->next) {
        if ((*p)->fd == fd) {
            struct fd_watch *w = *p;
            *p = w->next;
            fsfree(w);
            return epoll_ctl(async->epfd, EPOLL_CTL_DEL, fd, NULL);
        }
    }
    errno = ENOENT;
    return -1;
}

/* Edges that came in while the loop was quitting, one at a time (an
 * action may unregister any watch, so the list is searched afresh). */
static void deliver_pending(async_t *async)
{
    async->pending_scheduled = false;
    for (;;) {
        struct fd_watch *w = async->watches;
        while (w && !w->pending)
            w = w->next;
        if (!w)
            return;
        if (async->quit) { /* an action quit again: next time round */
            async->pending_scheduled = true;
            async_execute(async, (action_1) { async, (act_1) deliver_pending });
            return;
        }
        w->pending = false;
        action_1_perf(w->action);
    }
}

int async_loop(async_t *async)
{
    async->quit = false;
    while (!async->quit) {
        uint64_t now = async_now(async);
        for (int i = 0; i < kBurst && !async->quit; i++) {
            async_timer_t *t = async->fifo_head;
            if (t) {
                fifo_unlink(async, t);
            } else {
                if (!async->nheap || async->heap[0]->expires > now)
                    break;
                t = async->heap[0];
                heap_remove(async, 0);
            }
            action_1 a = t->action;
            task_free(async, t);
            action_1_perf(a);
        }
        if (async->quit)
            break;
        int timeout_ms = -1;
        if (async->fifo_head) {
            timeout_ms = 0;
        } else if (async->nheap) {
            uint64_t exp = async->heap[0]->expires;
            now = async_now(async);
            timeout_ms = exp <= now ? 0 : (int) ((exp - now + 999999) / 1000000);
        } else if (!async->watches) {
            /* Nothing can ever happen again. */
            errno = EDEADLK;
            return -1;
        }
        struct epoll_event evs[kMaxEvents];
        int n = epoll_wait(async->epfd, evs, kMaxEvents, timeout_ms);
        if (n < 0) {
            if (errno == EINTR)
                continue;
            return -1;
        }
        /* Every returned event is acted on: the registration is
         * edge-triggered, so an edge dropped here would not be reported
         * again.  Events that arrive after an action quit the loop are
         * marked on their watch and delivered by a task when the loop runs
         * again, unless the descriptor is unregistered first (the reference
         * triggers each event as an immediate task and never drops one,
         * src/async.c:300-330; an unregistered event is a zombie, :349-363). */
        for (int i = 0; i < n; i++) {
            struct fd_watch *w = find_watch(async, evs[i].data.fd);
            if (!w)
                continue;
            if (!async->quit) {
                action_1_perf(w->action);
                continue;
            }
            w->pending = true;
            if (!async->pending_scheduled) {
                async->pending_scheduled = true;
                async_execute(async, (action_1) { async, (act_1) deliver_pending });
            }
        }
    }
    return 0;
}
