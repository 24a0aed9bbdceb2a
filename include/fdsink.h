/*
 * fdsink.h -- the egress end of the base64 path: drain a bytestream_1 into
 * a file descriptor (pipe or socket) from the event loop (SURVEY.md §8(f)
 * row f1, §3 CS-2).
 *
 * The reference's egress is its TCP connection's output side
 * (/root/reference/src/tcp_connection.c): push_output() (:669-727)
 * refills a 10,240-byte outbuf (OUTBUF_SIZE, :22) with one read of the
 * output stream (replenish_outbuf(), :451-484) and hands it to send(2),
 * waiting for the socket's edge on EAGAIN from send and for the stream's
 * callback on EAGAIN from the read; at the stream's EOF it shuts the
 * socket's write side.  The TCP layer itself is out of scope (SURVEY.md §2
 * row 10); this is that loop for any fd, with write(2):
 *
 *   open_fdsink(async, source, fd)   starts draining (from the loop);
 *   the sink owns `source` and `fd`: at the source's EOF, once every byte
 *   is written, the fd is closed (a pipe's reader sees EOF); on an error
 *   the fd is closed too and fdsink_error() reports the errno.
 *   fdsink_register_callback(action)  performed once the sink is finished
 *   (EOF written out, or an error);
 *   fdsink_close()                    closes the source (and the fd if
 *   still open) and frees the sink through async_wound().
 *
 * Implementation in async_amd/csrc/fdstreams.c.
 */
#ifndef ASYNC_AMD_FDSINK_H
#define ASYNC_AMD_FDSINK_H

#include <stdbool.h>
#include <stdint.h>

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fdsink fdsink_t;

/* The reference's OUTBUF_SIZE (tcp_connection.c:22): bytes per pull. */
#define FDSINK_PULL_SIZE 10240

fdsink_t *open_fdsink(async_t *async, bytestream_1 source, int fd);
void fdsink_register_callback(fdsink_t *sink, action_1 action);
void fdsink_unregister_callback(fdsink_t *sink);
/* Finished: the source's EOF was reached and every byte written, or an
 * error ended the sink. */
bool fdsink_done(fdsink_t *sink);
/* 0, or the errno that ended the sink (from the source's read or from
 * write(2)). */
int fdsink_error(fdsink_t *sink);
/* Bytes written to the fd so far. */
uint64_t fdsink_bytes(fdsink_t *sink);
void fdsink_close(fdsink_t *sink);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_FDSINK_H */
