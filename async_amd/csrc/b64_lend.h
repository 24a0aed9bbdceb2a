/*
 * b64_lend.h -- internal: zero-copy reads from the GPU encoder stage for
 * wrappers built into the same library (framing.c's chunkencoder), and
 * zero-copy input to it from the queuestream (below).
 *
 * b64_lend_read() returns exactly what bytestream_1_read(s, fallback,
 * count) would (same count, same -1/errno), but when those bytes lie in
 * one staged block it does not copy them: *data points at them inside the
 * stage's pinned output, lent until b64_lend_return() (or the stage's next
 * read or close).  *data is NULL when the bytes were copied to `fallback`.
 * For any other stream it is a plain read into `fallback`.
 *
 * From a stream for which b64_lend_capable() holds, `fallback` may be
 * NULL: bytes that span blocks are then gathered into the stage's own
 * buffer and lent from there, so *data is never NULL when the result is
 * positive (a wrapper needs no max-size buffer of its own).
 */
#ifndef ASYNC_AMD_B64_LEND_H
#define ASYNC_AMD_B64_LEND_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#include "blobstream.h"
#include "bytestream_1.h"

ssize_t b64_lend_read(bytestream_1 s, void *fallback, size_t count, const uint8_t **data);
void b64_lend_return(bytestream_1 s);
bool b64_lend_capable(bytestream_1 s);

/*
 * Upstream side: the GPU encoder stage takes its input without copying it
 * when its upstream is a queuestream whose head element is a message
 * queuestream_enqueue_bytes() / _push_bytes() copied into pinned memory
 * (b64_pin.h).
 *
 * b64_src_peek(): true when upstream is such a queue whose head holds
 * unread pinned bytes: *p, *n = them, *slab = their slab.  Exhausted head
 * elements are dropped first, as a read would.  b64_src_take(): n of those
 * bytes (n <= *n) are consumed, exactly as a read of n bytes would have.
 */
struct b64_pin_slab;
bool b64_src_peek(bytestream_1 s, const uint8_t **p, size_t *n, struct b64_pin_slab **slab);
void b64_src_take(bytestream_1 s, size_t n);
/* How much of a read of up to `limit` bytes from upstream can be taken
 * before it would enter a queued pinned message with at least lend_min
 * unread bytes (limit when there is none, or upstream is another kind of
 * stream): a block gathered by reading stops there, so that the message
 * is lent rather than copied. */
size_t b64_src_plain(bytestream_1 s, size_t lend_min, size_t limit);
/* streams.c: the same for one blobstream (slab NULL: not pinned). */
bool b64_blob_lend_peek(bytestream_1 s, const uint8_t **p, size_t *n,
                        struct b64_pin_slab **slab);
void b64_blob_lend_take(bytestream_1 s, size_t n);
/* Downstream of the chunkencoder (fdstreams.c's fdsink): b64_chunk_lend()
 * serves exactly the bytes chunkencoder_read(s, buf, count) would, but lends
 * them instead of copying: *p points at the next contiguous run of the
 * frame (the header, or the data where the encoder stage lent it), at most
 * `count` bytes, valid until the next call or close.  -1/errno and 0 as a
 * read. */
bool b64_chunk_lendable(bytestream_1 s);
ssize_t b64_chunk_lend(bytestream_1 s, size_t count, const uint8_t **p);
/* copy_blobstream() into the pinned pool (an ordinary copy without it). */
blobstream_t *b64_pinned_blobstream(async_t *async, const void *blob, size_t count);

#endif
