/*
 * b64_lend.h -- internal: zero-copy reads from the GPU encoder stage for
 * wrappers built into the same library (framing.c's chunkencoder).
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

#include "bytestream_1.h"

ssize_t b64_lend_read(bytestream_1 s, void *fallback, size_t count, const uint8_t **data);
void b64_lend_return(bytestream_1 s);
bool b64_lend_capable(bytestream_1 s);

#endif
