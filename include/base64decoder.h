/*
 * base64decoder.h -- drop-in replacement for the reference's lenient
 * base64 decoding byte-stream stage, computed on an MI355X (gfx950)
 * through the b64x C ABI (include/b64x.h).
 *
 * Every declaration below replaces the same-named one of
 * /root/reference/include/base64decoder.h:11-23 with an identical C
 * signature:
 *
 *   base64_decode                     ref include/base64decoder.h:15-16
 *                                     (src/base64decoder.c:22-36)
 *   base64decoder_as_bytestream_1     ref :18 (src/base64decoder.c:147-150)
 *   base64decoder_read                ref :19 (src/base64decoder.c:52-91)
 *   base64decoder_close               ref :20 (src/base64decoder.c:95-102)
 *   base64decoder_register_callback   ref :22 (src/base64decoder.c:106-110)
 *   base64decoder_unregister_callback ref :23 (src/base64decoder.c:114-118)
 *
 * Semantics (the reference's, src/base64decoder.c:52-80): every byte that
 * is not in the alphabet -- '=', CR/LF, anything -- is skipped without an
 * error; the output is the first floor(6V/8) bytes of the big-endian
 * packing of the V alphabet characters of the whole stream.
 */
#ifndef ASYNC_AMD_BASE64DECODER_H
#define ASYNC_AMD_BASE64DECODER_H

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct base64decoder base64decoder_t;

/* Take ownership of `stream` and present its base64 decoding.  A value of
 * (char) -1 for pos62 or pos63 selects '+' or '/'. */
base64decoder_t *base64_decode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63);

bytestream_1 base64decoder_as_bytestream_1(base64decoder_t *decoder);
ssize_t base64decoder_read(base64decoder_t *decoder, void *buf, size_t count);
void base64decoder_close(base64decoder_t *decoder);
void base64decoder_register_callback(base64decoder_t *decoder, action_1 action);
void base64decoder_unregister_callback(base64decoder_t *decoder);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_BASE64DECODER_H */
