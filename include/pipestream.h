/*
 * pipestream.h -- an open file descriptor (pipe, socket, any pipe-like fd)
 * read as a non-blocking bytestream_1: the host ingress of the base64 path
 * (the event loop's read() from a socket
 * or pipe, feeding base64_decode()).
 *
 * Same API as /root/reference/include/pipestream.h:17-23 (behaviour
 * /root/reference/src/pipestream.c:23-109); implementation in
 * async_amd/csrc/fdstreams.c.
 *
 *  - read() is read(2) on the fd: bytes, 0 at EOF, -1 + errno (EAGAIN when
 *    the fd has nothing yet -- the registered callback follows).
 *  - open_pipestream() registers the fd with async_register() (which makes
 *    it non-blocking and watches it edge-triggered); each edge calls the
 *    registered callback.
 *  - The stream owns the fd: close() unregisters and closes it.
 */
#ifndef ASYNC_AMD_PIPESTREAM_H
#define ASYNC_AMD_PIPESTREAM_H

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pipestream pipestream_t;

pipestream_t *open_pipestream(async_t *async, int fd);

bytestream_1 pipestream_as_bytestream_1(pipestream_t *pipestr);
ssize_t pipestream_read(pipestream_t *pipestr, void *buf, size_t count);
void pipestream_close(pipestream_t *pipestr);
void pipestream_register_callback(pipestream_t *pipestr, action_1 action);
void pipestream_unregister_callback(pipestream_t *pipestr);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_PIPESTREAM_H */
