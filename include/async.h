/*
 * async.h -- the minimal single-threaded event loop that the base64
 * byte-stream stages and their test topology need.
 *
 * The reference's loop (src/async.c, 883 lines: epoll/kqueue, timers,
 * immediate tasks, deferred free) is plumbing and out of scope (SURVEY.md
 * §2 row 4).  This is a from-scratch subset with the same names and
 * semantics for the calls the hot path touches:
 *
 *   make_async / destroy_async      ref include/async.h:52,57
 *   async_now                       ref include/async.h:65
 *   async_timer_start / _cancel     ref include/async.h:80-91
 *   async_execute                   ref include/async.h:117 (src/async.c:376)
 *   async_wound                     ref include/async.h:129 (src/async.c:386)
 *   async_loop / async_quit_loop    ref include/async.h:191,223 (src/async.c:620)
 *   async_register / _unregister    ref include/async.h:249,277 (src/async.c:766)
 *
 * async_register() has the reference's edge-triggered contract (below): it
 * is used for the eventfd through which GPU completions re-enter the loop
 * ("Where a GPU would enter").
 *
 * Objects: everything this loop allocates, and every object handed to
 * async_wound(), comes from fsalloc() (include/fsalloc.h), as in the
 * reference.
 */
#ifndef ASYNC_AMD_ASYNC_H
#define ASYNC_AMD_ASYNC_H

#include <stdint.h>

#include "action_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct async async_t;
typedef struct async_timer async_timer_t;

#define ASYNC_NS ((int64_t) 1)
#define ASYNC_US (1000 * ASYNC_NS)
#define ASYNC_MS (1000 * ASYNC_US)
#define ASYNC_S (1000 * ASYNC_MS)

/* NULL + errno on failure. */
async_t *make_async(void);
void destroy_async(async_t *async);

/* Monotonic nanoseconds. */
uint64_t async_now(async_t *async);

/* Run `action` once async_now() >= expires. */
async_timer_t *async_timer_start(async_t *async, uint64_t expires,
                                 action_1 action);
void async_timer_cancel(async_t *async, async_timer_t *timer);

/* Run `action` from the loop at the first opportunity. */
async_timer_t *async_execute(async_t *async, action_1 action);

/* fsfree() `object` (allocated with fsalloc()) from the loop at the first
 * opportunity, after every task already scheduled has run; destroy_async()
 * frees those still waiting. */
void async_wound(async_t *async, void *object);

/* Run until async_quit_loop(); 0 on quit, -1 + errno on error. */
int async_loop(async_t *async);
void async_quit_loop(async_t *async);

/* Watch `fd` edge-triggered (ref include/async.h:236-249): the descriptor
 * is made non-blocking, and `action` is called when its state changes --
 * it is guaranteed a call only after a read or write on `fd` has returned
 * EAGAIN, so the action should drain it.  A registration may bring one
 * spurious call.  An edge that arrives while the loop is quitting is kept
 * and delivered when the loop runs again (unless `fd` is unregistered
 * first). */
int async_register(async_t *async, int fd, action_1 action);
int async_unregister(async_t *async, int fd);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_ASYNC_H */
