/*
 * queuestream.h -- a bytestream_1 that concatenates a dynamic queue of
 * streams (the producer of SURVEY.md §8(d) config 5: messages are enqueued
 * as blobs, the queue is terminated, a base64 encoder pulls from it).
 * Same API as /root/reference/include/queuestream.h; implementation in
 * async_amd/csrc/framing.c.
 *
 * Behaviour restated from the reference (src/queuestream.c):
 *  - read() fills `count` from successive queued streams, closing each at
 *    its EOF (:150-191); it returns the bytes gathered so far when a queued
 *    stream answers EAGAIN or fails (a failure other than EAGAIN is then
 *    reported by the next read, :171-176);
 *  - with the queue empty it returns 0 once terminated, else -1/EAGAIN
 *    and calls the registered callback when a stream is enqueued/pushed,
 *    the queue is terminated, or a queued stream calls back (:64-69);
 *  - make_queuestream() objects are freed at close(); a "relaxed" one
 *    stays valid after close() until queuestream_release() (:28-59).
 */
#ifndef ASYNC_AMD_QUEUESTREAM_H
#define ASYNC_AMD_QUEUESTREAM_H

#include <stdbool.h>

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct queuestream queuestream_t;

queuestream_t *make_queuestream(async_t *async);
queuestream_t *make_relaxed_queuestream(async_t *async);
bool queuestream_closed(queuestream_t *qstr);
void queuestream_release(queuestream_t *qstr);
/* Append (enqueue) or prepend (push) a stream; after close() the stream is
 * closed instead. */
void queuestream_enqueue(queuestream_t *qstr, bytestream_1 stream);
void queuestream_push(queuestream_t *qstr, bytestream_1 stream);
/* Same, over a private copy of `count` bytes at `blob`. */
void queuestream_enqueue_bytes(queuestream_t *qstr, const void *blob,
                               size_t count);
void queuestream_push_bytes(queuestream_t *qstr, const void *blob,
                            size_t count);
/* No more streams will be added: EOF after the queued ones. */
void queuestream_terminate(queuestream_t *qstr);
bytestream_1 queuestream_as_bytestream_1(queuestream_t *qstr);
ssize_t queuestream_read(queuestream_t *qstr, void *buf, size_t count);
void queuestream_close(queuestream_t *qstr);
void queuestream_register_callback(queuestream_t *qstr, action_1 action);
void queuestream_unregister_callback(queuestream_t *qstr);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_QUEUESTREAM_H */
