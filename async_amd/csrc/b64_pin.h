/*
 * b64_pin.h -- internal: pinned, GPU-readable copies of queued messages.
 *
 * queuestream_enqueue_bytes() copies its message (as the reference's does,
 * src/queuestream.c:117-122 -> copy_blobstream()).  Made into pinned host
 * memory from this pool, the copy is one the GPU can read directly: the
 * encoder stage then lends the message's bytes from the queue (b64_lend.h,
 * upstream side) and commits them as a job of the hub's batch without
 * copying them into the batch's arena; the lane's gather kernel reads them
 * over the host link (b64x_lane_encode_async, h_src).  That is one host copy
 * of every byte fewer on the loop's thread.
 *
 * Slabs of ASYNC_B64_PIN_SLAB bytes (default 32 MiB) are carved by a bump
 * pointer per thread; a slab counts its live pieces plus one while it is a
 * thread's current slab, and goes back to a process-wide free list when the
 * count drops to zero, while the idle slabs stay within
 * ASYNC_B64_PIN_IDLE_BYTES (default 2 GiB; beyond it a released slab is
 * freed).  Pieces larger than a quarter slab get a slab of their own, which
 * is freed when released, never kept idle.  Every reference is taken and
 * dropped with atomics: the hub drops the ones its batches hold when they
 * complete, possibly on another loop's thread.
 *
 * The pool starts only once a GPU stage exists in the process
 * (b64_pin_activate(), from base64_encode()/base64_decode()): until then a
 * message is copied into ordinary memory, so a process that uses the queue
 * without the GPU stages never allocates pinned memory or starts the HIP
 * runtime.  ASYNC_B64_PIN=0 turns the pool off (messages are copied into
 * ordinary memory and every encoder block is gathered into the arena).
 */
#ifndef ASYNC_AMD_B64_PIN_H
#define ASYNC_AMD_B64_PIN_H

#include <stdbool.h>
#include <stddef.h>

typedef struct b64_pin_slab b64_pin_slab;

/* Pinned room for n bytes (16-byte aligned); *slab gets the slab, which
 * holds one reference for the piece.  NULL when the pool is off or pinned
 * memory is not to be had. */
void *b64_pin_alloc(size_t n, b64_pin_slab **slab);
void b64_pin_ref(b64_pin_slab *s);
void b64_pin_unref(b64_pin_slab *s);
bool b64_pin_enabled(void);
/* A GPU stage exists: queued messages are pinned from now on. */
void b64_pin_activate(void);
/* References held on pieces: by their blobstreams and by the batches that
 * read them (tests: zero once every stream is closed and every batch done). */
long b64_pin_live_refs(void);
/* Bytes of the idle slabs the pool keeps (tests). */
size_t b64_pin_idle_bytes(void);

#endif
