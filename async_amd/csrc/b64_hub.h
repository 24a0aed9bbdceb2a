/*
 * b64_hub.h -- internal: cross-stream batching of encoder and decoder
 * blocks for one event loop.
 *
 * Every base64 stage on an async_t shares one hub.  A stage reserves room
 * in the hub's open pinned arena, reads its upstream straight into it, and
 * commits the block as a job; the hub launches the arena as one ragged
 * batch (b64x_lane_encode_async / _decode_async: one H2D, the kernels
 * writing their outputs straight into the pinned arena) when the arena
 * fills or at the end of the current loop turn, on up to 4 concurrent HIP
 * streams ("lanes").  Completion comes back through one eventfd registered
 * with async_register(); the hub checks the batch (b64x_lane_*_check),
 * marks each job's ticket done and calls the stage's wake action.
 *
 * Many small messages (config 5: Zipf 64 B - 1 MiB) thus cost one launch
 * and one copy per arena instead of per message, and a loop's thousands of
 * streams hold no HIP stream of their own.
 */
#ifndef ASYNC_AMD_B64_HUB_H
#define ASYNC_AMD_B64_HUB_H

#include <stdatomic.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "action_1.h"
#include "async.h"
#include "b64x.h"

typedef struct b64_hub b64_hub;
typedef struct b64_batch b64_batch;
struct b64_pin_slab;

/* One committed block, owned by the stage. */
typedef struct {
    b64_batch *batch;      /* NULL when idle */
    uint32_t index;        /* job index in the batch */
    atomic_int done;       /* output ready (or err set) */
    int err;               /* negative errno if the batch failed */
    const uint8_t *out;    /* the block's output, valid once done */
    size_t out_len;        /* decode jobs: the bytes decoded (device count) */
    b64x_dec_result res;   /* decode jobs: the job's checked result record */
    action_1 wake;         /* performed on the loop when done */
} b64_ticket;

/* What a batch does with its jobs. */
typedef enum { B64_HUB_ENCODE = 0, B64_HUB_DECODE = 1 } b64_hub_kind;

/* The hub for `async` (created on first use); NULL + errno on failure. */
b64_hub *b64_hub_acquire(async_t *async);
/* A stage is gone; the last release tears the hub down (waiting for its
 * batches still in flight). */
void b64_hub_release(b64_hub *h);

/* Room for one block of at most `room` bytes, at least `min_room`, encoded
 * with `abc`; returns where to write it, or NULL + errno.  *granted gets
 * the room actually given.  Must be followed by commit or cancel before
 * control returns to the loop.  Reservations nest (the caller may read
 * upstream through other stages of the same hub while holding one, up to 8
 * deep, ELOOP beyond): each open reservation has its own arena.
 * Backpressure: when the hub already holds
 * its share of arenas and a new one is needed, a caller passing a
 * `waiter` (a stage with nothing staged or in flight) gets NULL/EAGAIN and
 * the waiter is performed once an arena is recycled; NULL_ACTION_1-like
 * {.act = NULL} callers (stages holding data, which must make progress)
 * are always served. */
uint8_t *b64_hub_reserve(b64_hub *h, b64_hub_kind kind, const b64x_alphabet *abc,
                         size_t room, size_t min_room, size_t *granted, action_1 waiter);
/* When `waiting` (the stage may be on the waiter list): drop any waiter
 * whose object is `obj` (its stage is closing).  The waiter lists can hold
 * thousands of stages: scanning them on every close would be quadratic. */
void b64_hub_forget(b64_hub *h, void *obj, bool waiting);
/* Turn the reservation into a job of n bytes -> out_len characters
 * (`prev`: NULL, or as b64_hub_chainable() allowed)
 * (encode) or of n characters -> at most out_len bytes (decode; `flags`
 * B64X_DEC_HOLD_TAIL when more of the stream follows: whole groups only,
 * the last V mod 4 sextets reported; 0 ends the stream: its final partial
 * group emitted).  A decode job's record lands in ticket->res, its byte
 * count in ticket->out_len. */
void b64_hub_commit(b64_hub *h, b64_ticket *t, size_t n, size_t out_len,
                    unsigned flags, const b64_ticket *prev, action_1 wake);
/* Decoder streams in blocks (the stage's carry): while
 * a reservation is open, may the job about to be committed take its 0-3
 * carried sextets on the device from `prev`, a job of the same stream whose
 * record the host has not seen yet?  Yes when `prev` is an earlier job of
 * the arena being filled, or of a batch that is ready or in flight (this
 * arena's batch then runs behind it on its lane; it can follow one such
 * batch only).  The job is then committed with `prev` (a 4-character head
 * of non-alphabet characters first): the device spells prev's held-back
 * sextets into the head between prev's decode and its own. */
bool b64_hub_chainable(b64_hub *h, const b64_ticket *prev);
/* While a reservation of an encode block is open: its bytes [pos, pos+n)
 * are not written into the arena but lent -- they are at `src`, in a pinned
 * message of `slab` (b64_pin.h).  The batch holds a reference on the slab
 * until it has finished, and its lane reads the bytes straight from there
 * (b64x_lane_encode_async, h_seg).  False (nothing recorded: copy them
 * instead) when the arena's segment table is full. */
bool b64_hub_lend(b64_hub *h, size_t pos, const uint8_t *src, size_t n,
                  struct b64_pin_slab *slab);
/* Segments lent so far in this process (tests). */
unsigned long b64_hub_lent_total(void);
/* Idle arenas in the process-wide pool (tests, traces). */
unsigned long b64_hub_pooled(void);
void b64_hub_cancel(b64_hub *h);
/* ASYNC_B64_HUB_TRACE=1: the stages add the time of their upstream reads
 * (the copies into the arenas) to the hub's trace line. */
bool b64_hub_tracing(const b64_hub *h);
void b64_hub_trace_gather(b64_hub *h, double secs, size_t bytes);
/* The stage is done with the ticket (consumed, or closing before the
 * batch finished: its output is then discarded). */
void b64_ticket_release(b64_ticket *t);

#endif /* ASYNC_AMD_B64_HUB_H */
