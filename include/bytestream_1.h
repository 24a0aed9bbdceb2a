/*
 * bytestream_1 -- the pull-model, non-blocking byte-stream ABI that the
 * base64 stages implement and consume.
 *
 * Drop-in boundary: the fat pointer {obj, vt} and the vtable member order
 * (read, close, register_callback, unregister_callback) are the
 * reference's, /root/reference/include/bytestream_1.h:15-57, so objects
 * built against either header interoperate.
 *
 * Contract (restated from the reference's comments, same file :21-56):
 *  - read() behaves like read(2): >0 bytes produced, 0 = end of stream
 *    (sticky), -1 + errno on error; EAGAIN means a callback will follow.
 *    It never blocks on I/O and must not be called after close().
 *  - close() never fails; resources may be released later from the loop.
 *  - register_callback() replaces the callback that is invoked when read()
 *    should be retried; callbacks may arrive after close().
 */
#ifndef ASYNC_AMD_BYTESTREAM_1_H
#define ASYNC_AMD_BYTESTREAM_1_H

#include <sys/types.h>

#include "action_1.h"
#include "async.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    void *obj;
    const struct bytestream_1_vt *vt;
} bytestream_1;

struct bytestream_1_vt {
    ssize_t (*read)(void *obj, void *buf, size_t count);
    void (*close)(void *obj);
    void (*register_callback)(void *obj, action_1 action);
    void (*unregister_callback)(void *obj);
};

static inline ssize_t bytestream_1_read(bytestream_1 stream, void *buf,
                                        size_t count)
{
    return stream.vt->read(stream.obj, buf, count);
}

static inline void bytestream_1_close(bytestream_1 stream)
{
    stream.vt->close(stream.obj);
}

static inline void bytestream_1_register_callback(bytestream_1 stream,
                                                  action_1 action)
{
    stream.vt->register_callback(stream.obj, action);
}

static inline void bytestream_1_unregister_callback(bytestream_1 stream)
{
    stream.vt->unregister_callback(stream.obj);
}

/* Close `stream` from the loop at the first opportunity.
 * (ref: src/bytestream_1.c:13-18) */
void bytestream_1_close_relaxed(async_t *async, bytestream_1 stream);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_BYTESTREAM_1_H */
