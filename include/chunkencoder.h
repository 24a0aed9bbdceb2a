/*
 * chunkencoder.h -- HTTP/1.1 chunked transfer framing over a bytestream_1
 * (the consumer of the base64 encoder in SURVEY.md §8(d) config 5).
 * Same API as /root/reference/include/chunkencoder.h; implementation in
 * async_amd/csrc/framing.c.
 *
 * Framing restated from the reference (src/chunkencoder.c:31-77): each
 * upstream read of up to max_chunk_size bytes (clamped to [2, 16 MiB],
 * :23-26, :178-183) becomes one chunk "<hex length>\r\n<data>", chunks
 * after the first are preceded by "\r\n", and upstream EOF becomes the
 * zero-length chunk, terminated per chunkencoder_termination_t.  A chunk's
 * header and data are served from one contiguous frame, so a read may
 * return both.  Chunk boundaries therefore follow the upstream's read
 * counts exactly -- the reason the GPU base64 encoder stage returns the
 * same counts as the reference encoder (async_amd/csrc/b64_stages.c).
 */
#ifndef ASYNC_AMD_CHUNKENCODER_H
#define ASYNC_AMD_CHUNKENCODER_H

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct chunkencoder chunkencoder_t;

chunkencoder_t *chunk_encode(async_t *async, bytestream_1 stream,
                             size_t max_chunk_size);

typedef enum {
    CHUNKENCODER_SIMPLE,                  /* terminate with "0\r\n\r\n" */
    CHUNKENCODER_STOP_AT_TRAILER,         /* terminate with "0\r\n"     */
    CHUNKENCODER_STOP_AT_FINAL_EXTENSIONS /* terminate with "0"         */
} chunkencoder_termination_t;

chunkencoder_t *chunk_encode_2(async_t *async, bytestream_1 stream,
                               size_t max_chunk_size,
                               chunkencoder_termination_t termination);
bytestream_1 chunkencoder_as_bytestream_1(chunkencoder_t *encoder);
ssize_t chunkencoder_read(chunkencoder_t *encoder, void *buf, size_t count);
void chunkencoder_close(chunkencoder_t *encoder);
void chunkencoder_register_callback(chunkencoder_t *encoder, action_1 action);
void chunkencoder_unregister_callback(chunkencoder_t *encoder);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_CHUNKENCODER_H */
