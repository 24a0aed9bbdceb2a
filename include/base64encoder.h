/*
 * base64encoder.h -- drop-in replacement for the reference's base64
 * encoding byte-stream stage, computed on an MI355X (gfx950) through the
 * b64x C ABI (include/b64x.h).
 *
 * Every declaration below replaces the same-named one of
 * /root/reference/include/base64encoder.h:13-27 with an identical C
 * signature, so code written against the reference relinks unchanged:
 *
 *   base64_encode                     ref include/base64encoder.h:19-20
 *                                     (src/base64encoder.c:31-47)
 *   base64encoder_as_bytestream_1     ref :22 (src/base64encoder.c:209-212)
 *   base64encoder_read                ref :23 (src/base64encoder.c:101-153)
 *   base64encoder_close               ref :24 (src/base64encoder.c:157-164)
 *   base64encoder_register_callback   ref :26 (src/base64encoder.c:168-172)
 *   base64encoder_unregister_callback ref :27 (src/base64encoder.c:176-180)
 *
 * Semantics: the produced character stream is the reference's, byte for
 * byte (standard base64, chars 62/63 = pos62/pos63, optional padding with
 * padchar, no line breaks; (char) -1 selects '+', '/', '=').  So are the
 * read counts: `count` whenever upstream keeps up, the full
 * sextets of a partial group in the same read, finalize()'s characters in
 * a read of their own -- except that a read answers -1/EAGAIN while its
 * block is still on the GPU (a callback follows).  The reference's assert
 * at src/base64encoder.c:140 for read counts not divisible by 4 is not
 * reproduced: every count works here.
 */
#ifndef ASYNC_AMD_BASE64ENCODER_H
#define ASYNC_AMD_BASE64ENCODER_H

#include <stdbool.h>

#include "async.h"
#include "bytestream_1.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct base64encoder base64encoder_t;

/* Take ownership of `stream` and present its base64 encoding.  A value of
 * (char) -1 for pos62, pos63 or padchar selects '+', '/' or '='. */
base64encoder_t *base64_encode(async_t *async, bytestream_1 stream, char pos62,
                               char pos63, bool pad, char padchar);

bytestream_1 base64encoder_as_bytestream_1(base64encoder_t *encoder);
ssize_t base64encoder_read(base64encoder_t *encoder, void *buf, size_t count);
void base64encoder_close(base64encoder_t *encoder);
void base64encoder_register_callback(base64encoder_t *encoder, action_1 action);
void base64encoder_unregister_callback(base64encoder_t *encoder);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_BASE64ENCODER_H */
