/*
 * nicestream.h -- a pass-through bytestream_1 that answers EAGAIN (and
 * schedules a retry callback) once more than `max_burst` bytes went
 * through since the last back-off.  The reference's base64 test chains
 * three of them (test/asynctest-base64encoder.c:126-138) to exercise the
 * stages' EAGAIN paths.  Same API as /root/reference/include/nicestream.h;
 * implementation in async_amd/csrc/streams.c.
 */
#ifndef ASYNC_AMD_NICESTREAM_H
#define ASYNC_AMD_NICESTREAM_H

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nicestream nicestream_t;

nicestream_t *make_nice(async_t *async, bytestream_1 stream, size_t max_burst);
bytestream_1 nicestream_as_bytestream_1(nicestream_t *nice);
ssize_t nicestream_read(nicestream_t *nice, void *buf, size_t count);
void nicestream_close(nicestream_t *nice);
void nicestream_register_callback(nicestream_t *nice, action_1 action);
void nicestream_unregister_callback(nicestream_t *nice);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_NICESTREAM_H */
