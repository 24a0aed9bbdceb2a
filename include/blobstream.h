/*
 * blobstream.h -- a bytestream_1 over a memory blob (the feed of the
 * reference's base64 test topology).
 * Same API as /root/reference/include/blobstream.h; implementation in
 * async_amd/csrc/streams.c.
 */
#ifndef ASYNC_AMD_BLOBSTREAM_H
#define ASYNC_AMD_BLOBSTREAM_H

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct blobstream blobstream_t;

/* Stream `count` bytes at `blob`; the blob must outlive the stream. */
blobstream_t *open_blobstream(async_t *async, const void *blob, size_t count);
/* Same, over a private copy of the blob. */
blobstream_t *copy_blobstream(async_t *async, const void *blob, size_t count);
/* Same as open_blobstream(); `close_action` runs when the stream closes. */
blobstream_t *adopt_blobstream(async_t *async, const void *blob, size_t count,
                               action_1 close_action);

bytestream_1 blobstream_as_bytestream_1(blobstream_t *blobstr);
size_t blobstream_remaining(blobstream_t *blobstr);
ssize_t blobstream_read(blobstream_t *blobstr, void *buf, size_t count);
void blobstream_close(blobstream_t *blobstr);
void blobstream_register_callback(blobstream_t *blobstr, action_1 action);
void blobstream_unregister_callback(blobstream_t *blobstr);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_BLOBSTREAM_H */
