/*
 * b64_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's base64 byte-stream stages
 * (/root/reference/src/base64encoder.c, src/base64decoder.c), used as the
 * parity checker by tests/, by __graft_entry__.smoke() and as the
 * cpu_baseline leg of bench.py.  Nothing in the product (async_amd/)
 * links, loads or calls it.  See oracle/README.md for how it is pinned.
 */
#ifndef B64_ORACLE_H
#define B64_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The effective 256-entry decode map (-1 = skipped byte). */
void orc_decode_table(char pos62, char pos63, int8_t out[256]);

/* Whole-buffer encode/decode through the streaming state machines with a
 * single large read (never in the reference's assert domain).  Return the
 * number of bytes written to `out`; `out` must hold 4*ceil(n/3) (encode)
 * or 3*ceil(n/4) (decode) bytes. */
size_t orc_encode(const uint8_t *in, size_t n, char pos62, char pos63, int pad,
                  char padchar, uint8_t *out);
size_t orc_decode(const uint8_t *in, size_t n, char pos62, char pos63,
                  uint8_t *out);

/* nbuf independent rows of `len` bytes/characters at in + i*len, each
 * encoded (default alphabet, padding) or decoded to out + i*out_stride;
 * return the total bytes written. */
size_t orc_encode_rows(const uint8_t *in, size_t len, size_t nbuf, uint8_t *out,
                       size_t out_stride);
size_t orc_decode_rows(const uint8_t *in, size_t len, size_t nbuf, uint8_t *out,
                       size_t out_stride);

/* Pull-model simulations with the reference's read pattern:
 *  - the source hands out at most `src_chunk` bytes per read (0 = no
 *    limit);
 *  - if `burst` > 0 a nicestream-style wrapper sits between source and
 *    stage and answers EAGAIN once more than `burst` bytes have gone
 *    through since its last back-off (ref src/nicestream.c:34-51); the
 *    consumer retries, like the loop callback would;
 *  - the consumer drains the stage with reads of `read_size` bytes into a
 *    buffer of exactly `read_size` bytes.
 * Return the output length, or -1 if a read would have tripped the
 * reference's assert at src/base64encoder.c:140 (the write overran the
 * caller's buffer); *overflow_reads counts such reads. */
ssize_t orc_encode_stream(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, int pad, char padchar, uint8_t *out,
                          size_t out_cap, size_t *overflow_reads);
ssize_t orc_decode_stream(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, uint8_t *out, size_t out_cap);

/* The reference's own base64 test topology
 * (test/asynctest-base64encoder.c:123-151): counting bytes (i & 0xff),
 * `length` of them -> nice(113) -> encode('.', '_', pad '-') -> nice(91)
 * -> decode('.', '_') -> nice(97), drained 200 bytes at a time.  The
 * character stream between encoder and nice(91) is copied to enc_out
 * (*enc_len = its length).  Returns the number of decoded bytes, which
 * must equal `length` and reproduce the counting pattern. */
ssize_t orc_reftest(size_t length, uint8_t *enc_out, size_t enc_cap,
                    size_t *enc_len, uint8_t *dec_out, size_t dec_cap);

/* The config-5 egress stack: a terminated queuestream
 * of `npieces` blobs (piece_len[i] bytes each, concatenated at `in`) ->
 * encoder -> chunkencoder(max_chunk, termination 0/1/2 = SIMPLE /
 * STOP_AT_TRAILER / STOP_AT_FINAL_EXTENSIONS), drained `read_size` at a
 * time.  Returns the framed length, or -1 (assert domain / no memory). */
ssize_t orc_chunked_encode(const uint8_t *in, const size_t *piece_len,
                           size_t npieces, size_t max_chunk, int termination,
                           size_t read_size, char pos62, char pos63, int pad,
                           char padchar, uint8_t *out, size_t out_cap);

/* Like orc_encode_stream(), logging the encoder's positive read returns
 * (the first max_counts of them) -- what a counting wrapper such as the
 * chunkencoder sees.  Returns the number of positive reads, -1 on error. */
ssize_t orc_encode_counts(const uint8_t *in, size_t n, size_t src_chunk,
                          size_t burst, size_t read_size, char pos62,
                          char pos63, int pad, char padchar, ssize_t *counts,
                          size_t max_counts);

#ifdef __cplusplus
}
#endif

#endif
