/*
 * b64_copy.h -- internal: the stages' large host copies.
 *
 * A stage's read() copies its finished output into the caller's buffer, as
 * the bytestream_1 contract requires (ref src/base64decoder.c:58: the
 * reference decodes into the caller's buffer in place).  One stream through
 * one loop thread is then bound by that copy plus the upstream read(2): about
 * 2.3 bytes copied per payload byte on ingress.  A copy of at
 * least ASYNC_B64_COPY_SPLIT bytes (default 128 KiB) is split across
 * ASYNC_B64_COPY_THREADS helper threads (default 2) and the caller, which
 * waits for all parts: the same bytes in the same buffer when read()
 * returns, in a fraction of the time.  One split copy runs at a time; a
 * copy that finds the helpers busy (another loop's) is an ordinary memcpy.
 * ASYNC_B64_COPY_THREADS=0 turns the helpers off.
 */
#ifndef ASYNC_AMD_B64_COPY_H
#define ASYNC_AMD_B64_COPY_H

#include <stddef.h>

void b64_copy(void *dst, const void *src, size_t n);

#endif
