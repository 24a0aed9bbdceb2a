/*
 * b64_trace.h -- the reference's fstrace points for the base64 stages, kept
 * as compile-time no-ops (the external fstrace library is out
 * of scope; the IDs stay so a build with real tracing can map them 1:1).
 *
 * Reference: FSTRACE_DECL / FSTRACE in src/base64encoder.c:29,144-145,155,
 * 166,174 and src/base64decoder.c:20,50,82-83,93,104,112.  Each stage also
 * carries the reference's per-object `uid` (fstrace_get_unique_id()).
 */
#ifndef ASYNC_AMD_B64_TRACE_H
#define ASYNC_AMD_B64_TRACE_H

#include <stdatomic.h>
#include <stdint.h>

#define FSTRACE_DECL(id, fmt) enum { id##_TRACE_ID = 0 }
#define FSTRACE(id, ...) ((void) id##_TRACE_ID)

static inline uint64_t b64_trace_unique_id(void)
{
    static _Atomic uint64_t next = 1;
    return atomic_fetch_add_explicit(&next, 1, memory_order_relaxed);
}

#endif
