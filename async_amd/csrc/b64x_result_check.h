/*
 * b64x_result_check.h -- internal: the host-side check of completion
 * records, shared by the library (b64x_kernels.hip) and the CPU test
 * backend (tests/csrc/fake_b64x.c), so the deterministic stage tests run the
 * product's own check.
 *
 * A decode's result record (b64x_dec_result: a session's, or each job's of
 * a lane batch) is poisoned on the host before the launch; the kernels
 * overwrite it in host memory, echoing the call's character count, flags
 * and sequence number.  When the completion callback has run, a record
 * that still holds poison, names another call or whose fields contradict
 * each other was read too early: the caller waits for the stream and
 * checks again (b64x.h, b64x_session_decode_result /
 * b64x_lane_decode_check).
 */
#ifndef ASYNC_AMD_B64X_RESULT_CHECK_H
#define ASYNC_AMD_B64X_RESULT_CHECK_H

#include <stdbool.h>
#include <stdint.h>

#include "b64x.h"

#define B64X_RES_POISON (~(uint64_t) 0)
#define B64X_TAIL_POISON (~(uint32_t) 0)

/* Every field gets a value no finished record can hold (seq 0 is never
 * drawn; a tail byte is a sextet or 0). */
static inline void b64x_poison_result(b64x_dec_result *r)
{
    volatile b64x_dec_result *v = r;
    v->out_len = B64X_RES_POISON;
    v->valid = B64X_RES_POISON;
    v->tail_n = B64X_TAIL_POISON;
    for (int j = 0; j < 4; j++)
        v->tail[j] = 0xFF;
    v->nchars = B64X_RES_POISON;
    v->seq = 0;
    v->flags = B64X_TAIL_POISON;
}

/* A landed record of *this* call -- the decode of `len` characters with
 * `flags` that was given sequence number `seq` -- and self-consistent;
 * *copy receives what was read (each field once).  A record of an earlier
 * call (stale), a zero-filled one and a partly written one all fail. */
static inline bool b64x_result_ok(const b64x_dec_result *r, uint64_t len, unsigned flags,
                                  uint32_t seq, b64x_dec_result *copy)
{
    const volatile b64x_dec_result *v = r;
    b64x_dec_result c;
    c.out_len = v->out_len;
    c.valid = v->valid;
    c.tail_n = v->tail_n;
    for (int j = 0; j < 4; j++)
        c.tail[j] = v->tail[j];
    c.nchars = v->nchars;
    c.seq = v->seq;
    c.flags = v->flags;
    if (copy)
        *copy = c;
    const unsigned hold = flags & B64X_DEC_HOLD_TAIL;
    if (c.seq != seq || seq == 0 || c.nchars != len || c.flags != hold)
        return false;
    if (c.valid > len || c.tail_n != (uint32_t) (c.valid & 3))
        return false;
    for (uint32_t j = 0; j < 4; j++)
        if (j < c.tail_n ? c.tail[j] >= 64 : c.tail[j] != 0)
            return false;
    return c.out_len == (hold ? c.valid / 4 * 3 : c.valid * 6 / 8);
}

/* A chained lane job's spell log (what the device spelled its head from)
 * against the predecessor's record as checked on the host: the same call
 * (seq, nchars, flags) and the same held-back sextets.  A log taken from a
 * record that had not landed yet (poison, or an older call's) fails. */
static inline bool b64x_spell_ok(const b64x_dec_result *log, const b64x_dec_result *prev)
{
    const volatile b64x_dec_result *v = log;
    if (v->seq != prev->seq || v->nchars != prev->nchars || v->flags != prev->flags ||
        v->tail_n != prev->tail_n || v->valid != prev->valid)
        return false;
    for (int j = 0; j < 4; j++)
        if (v->tail[j] != prev->tail[j])
            return false;
    return true;
}

#endif /* ASYNC_AMD_B64X_RESULT_CHECK_H */
