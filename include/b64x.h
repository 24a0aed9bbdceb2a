/*
 * b64x.h -- C ABI of the MI355X (gfx950) base64 engine.
 *
 * This is the thin shim between host code (the bytestream_1 stages in
 * include/base64encoder.h / base64decoder.h, Python via ctypes, any FFI)
 * and the hand-written HIP kernels in async_amd/csrc/b64x_kernels.hip.
 * Only plain pointers, sizes and PODs cross it; no HIP or torch types.
 *
 * What each entry point replaces in the reference (all C, CPU only):
 *
 *   b64x_encode_dev / _strided / _batch
 *       the per-byte bit-accumulator loop of do_read() + finalize(),
 *       /root/reference/src/base64encoder.c:61-142, applied to a whole
 *       device-resident buffer (or a batch of independent buffers -- one
 *       encoder object per buffer in the reference).
 *   b64x_decode_dev / _strided / _batch
 *       the per-character loop of decoder_read() with map(),
 *       /root/reference/src/base64decoder.c:38-80, including its
 *       leniency (non-alphabet bytes skipped, bits carried across '=',
 *       trailing partial bits dropped).
 *   b64x_session_*
 *       the host-memory leg of the bytestream_1 stages: pinned staging,
 *       H2D, kernel, D2H.
 *
 * Error convention: 0 on success or a negative errno value (-EINVAL bad
 * argument, -ENOMEM allocation, -ENODEV no usable GPU, -EIO any other
 * HIP failure).  Nothing here aborts.
 *
 * All device pointers are HIP device (or host-pinned-mapped) pointers.
 * `stream` is a hipStream_t passed as void * (NULL = the null stream).
 * Device-side launches are asynchronous and capture-safe (no allocation
 * or synchronisation inside) unless the comment says otherwise.  A call
 * being captured into a graph does not reuse a line model held from earlier
 * calls (it captures the probe or prep too); the junk hint's pick of path is
 * replayed as made at capture -- exact either way, only the speed differs.
 */
/*
 * Process-wide state a decode call reads and writes.  None of it decides a
 * byte of output: every path below is exact for any input, and the state only
 * picks which path runs (b64x_diag_paths counts the picks).
 *
 *   library workspaces   at most 8, one per (device, stream), for calls with
 *                        d_workspace NULL and for b64x_decode_strided's rows
 *                        with room.  Read and written by those calls: scratch
 *                        (left zeroed), the probe's line model with the length
 *                        it was made for, a row batch's model and the shape it
 *                        was made for.  Guarded by a mutex; an entry is pinned
 *                        while a call enqueues on it.
 *   held models          64 entries keyed by a hash of the workspace address:
 *                        {workspace, length of its last probe}, plus a pinned
 *                        "probe again" flag each.  Read by every automatic
 *                        b64x_decode_dev of <= 2^31 characters (not
 *                        EXPECT_JUNK): a call of the same length on the same
 *                        workspace with the flag down skips the probe.
 *                        Written by every probe launch (host) and by
 *                        k_decode_suffix, which raises the flag whenever it
 *                        finds anything to decode past the line pass.  Any
 *                        model is exact (k_decode_lines checks every slot and
 *                        the model's length); a wrong one only costs speed.
 *   probe hints          64 pinned entries keyed by a hash of (workspace,
 *                        input address, length): "the last probe of this key
 *                        cut the model near the start".  Read (without a
 *                        sync) by every automatic decode, which then takes the
 *                        probe + single exact pass; written by every probe on
 *                        the device.  A stale or torn hint only picks the
 *                        slower path; new content at the same address and
 *                        length is decoded exactly either way.
 *   row-model staleness  one pinned flag per library workspace, raised by
 *                        k_rows_finish when a batch's first row failed its
 *                        model; read by the next b64x_decode_strided of the
 *                        same shape on that workspace, which then probes.
 *   sequence numbers     one counter, drawn by every decode call and batch
 *                        (b64x_dec_result.seq).
 *
 * A call being captured into a graph reads no held model or row model (it
 * captures the probe or prep), and never allocates or takes over a library
 * workspace.  The hint's pick is recorded in the capture as made.
 */

#ifndef ASYNC_AMD_B64X_H
#define ASYNC_AMD_B64X_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B64X_ABI_VERSION 4

/* Alphabet descriptor.  (char) -1 selects the reference's defaults,
 * exactly like base64_encode()/base64_decode() (ref
 * src/base64encoder.c:40-43, src/base64decoder.c:31-32).  `pad` and
 * `padchar` are ignored by the decoder, which has no pad parameter. */
typedef struct b64x_alphabet {
    char pos62;
    char pos63;
    char padchar;
    bool pad;
} b64x_alphabet;

/* Per-call decode result, written by the device.  A record names the call
 * that wrote it: `nchars` and `flags` echo the call's arguments and `seq` is
 * a nonzero number the library draws for every decode call (or batch), so
 * a record left over from an earlier call, or a zero-filled one, is never
 * taken for this call's (b64x_session_decode_result, b64x_lane_decode_check). */
typedef struct b64x_dec_result {
    uint64_t out_len;  /* bytes written to the output */
    uint64_t valid;    /* alphabet characters seen (V) */
    uint32_t tail_n;   /* V mod 4 */
    uint8_t tail[4];   /* the last tail_n sextet values (0..63); the rest 0 */
    uint64_t nchars;   /* characters this decode covered */
    uint32_t seq;      /* the call's sequence number, never 0 */
    uint32_t flags;    /* the call's B64X_DEC_HOLD_TAIL bit */
} b64x_dec_result;

/* Decode flags. */
#define B64X_DEC_HOLD_TAIL 1u /* emit only whole 4-char groups (3 bytes
                                 each); the V mod 4 trailing sextets are
                                 reported in b64x_dec_result.tail and
                                 produce no output.  Used by the streaming
                                 stage, which carries them to its next
                                 call. */
#define B64X_DEC_EXPECT_JUNK 2u /* a hint that the input holds non-alphabet
                                   bytes throughout (MIME line breaks):
                                   decode in one pass (counts, look-back,
                                   exact decode) instead of the optimistic
                                   pass that clean input takes.  Same
                                   result either way. */

/* ---- sizes ------------------------------------------------------------ */

/* Characters produced for n input bytes: 4*ceil(n/3) with pad,
 * ceil(4n/3) without. */
uint64_t b64x_encoded_len(uint64_t n, bool pad);
/* Output capacity the decoder needs for n input characters:
 * 3*ceil(n/4).  Bytes beyond b64x_dec_result.out_len are unspecified
 * (the reference likewise treats the caller's whole buffer as scratch,
 * src/base64decoder.c:58). */
uint64_t b64x_decoded_cap(uint64_t nchars);
/* Device workspace bytes b64x_decode_dev() needs for nchars. */
uint64_t b64x_decode_workspace_size(uint64_t nchars);

/* ---- one device-resident buffer ----------------------------------------- */

/* Encode n bytes at d_in into b64x_encoded_len(n, abc->pad) characters at
 * d_out.  Any alignment is accepted; 4-byte aligned d_in and 16-byte
 * aligned d_out take the fast path. */
int b64x_encode_dev(const void *d_in, uint64_t n, void *d_out,
                    const b64x_alphabet *abc, void *stream);

/* Decode nchars characters at d_in into d_out (capacity
 * b64x_decoded_cap(nchars)); *d_res (device memory) receives the result.
 * d_workspace: b64x_decode_workspace_size(nchars) bytes of device memory,
 * zero-filled before its first use (each call leaves it ready for the
 * next, holding the line model of its last probe: a call of the same length
 * may reuse it and skip the probe; one workspace per stream), or NULL to use
 * a library-owned one
 * per (device, stream).  The library keeps at most 8 such workspaces
 * (about 14 MiB of HBM each), allocated on first need and never freed: a
 * call on a stream without one takes an idle one (its stream made to wait
 * on the device for the workspace's last use), or -EBUSY if all eight are
 * in use by calls being enqueued right then.  A stream being captured into
 * a graph that holds no library workspace yet also gets -EBUSY (allocating
 * or rebinding one cannot be captured): decode on it once outside the
 * capture, or pass d_workspace.  A workspace stays with its stream until
 * b64x_release_stream() or until another stream takes it over; no event is
 * recorded per call. */
int b64x_decode_dev(const void *d_in, uint64_t nchars, void *d_out,
                    b64x_dec_result *d_res, const b64x_alphabet *abc,
                    unsigned flags, void *d_workspace, void *stream);
/* b64x_decode_dev, also returning in *seq (may be NULL) the sequence number
 * the call drew: the `seq` its record holds once it has landed.  A caller
 * that copies the record back (from any stream) checks it with
 * b64x_result_check() and so never takes a stale, zero-filled or partly
 * written record for this call's. */
int b64x_decode_dev_seq(const void *d_in, uint64_t nchars, void *d_out,
                        b64x_dec_result *d_res, const b64x_alphabet *abc,
                        unsigned flags, void *d_workspace, void *stream, uint32_t *seq);
/* 0 if *res (host memory) is the landed, self-consistent record of the
 * decode of `nchars` characters with `flags` that drew `seq` (the rules of
 * b64x_session_decode_result), -EAGAIN if it is not (yet). */
int b64x_result_check(const b64x_dec_result *res, uint64_t nchars, unsigned flags,
                      uint32_t seq);
/* Unbind the library-owned decode workspace of `stream` on the current
 * device, if it has one, so another stream can take it.  REQUIRED before
 * destroying a stream that decoded with d_workspace == NULL: the workspace
 * stays bound to the stream's handle, and a later call on another stream
 * that takes it over records an event on that handle (and asks whether it
 * is being captured) -- on a destroyed stream that is a dangling handle.
 * Released here, the event is recorded while the stream is still alive.
 * The NULL stream may hold a workspace like any other. */
void b64x_release_stream(void *stream);

/* ---- batches of independent buffers ----------------------------------- */

/* nbuf buffers of `len` bytes at d_in + i*in_stride; buffer i's
 * b64x_encoded_len(len, pad) characters go to d_out + i*out_stride. */
int b64x_encode_strided(const void *d_in, uint64_t in_stride, uint64_t len,
                        uint32_t nbuf, void *d_out, uint64_t out_stride,
                        const b64x_alphabet *abc, void *stream);

/* nbuf buffers of `len` characters at d_in + i*in_stride, decoded to
 * d_out + i*out_stride (capacity b64x_decoded_cap(len) each);
 * d_outlen[i] (device) receives buffer i's byte count.  Rows with room
 * (out_stride >= 12*ceil(len/16)) use the stream's library workspace (as
 * b64x_decode_dev with d_workspace NULL) to hold the batch's line model;
 * when none can be had (all pinned, or a capture on a stream holding none)
 * the batch takes the general path, same bytes. */
int b64x_decode_strided(const void *d_in, uint64_t in_stride, uint64_t len,
                        uint32_t nbuf, void *d_out, uint64_t out_stride,
                        uint64_t *d_outlen, const b64x_alphabet *abc,
                        void *stream);

/* Ragged batch: buffer i is d_in[d_in_off[i] .. d_in_off[i+1]) (nbuf+1
 * monotone offsets, device memory) and goes to d_out + d_out_off[i]. */
int b64x_encode_batch(const void *d_in, const uint64_t *d_in_off,
                      uint32_t nbuf, void *d_out, const uint64_t *d_out_off,
                      const b64x_alphabet *abc, void *stream);
int b64x_decode_batch(const void *d_in, const uint64_t *d_in_off,
                      uint32_t nbuf, void *d_out, const uint64_t *d_out_off,
                      uint64_t *d_outlen, const b64x_alphabet *abc,
                      void *stream);

/* ---- host-memory sessions (used by the bytestream_1 stages) ----------- */

typedef struct b64x_session b64x_session;

/* A session owns a HIP stream, pinned host staging of `capacity` input
 * bytes/characters and matching device buffers.  NULL + errno on
 * failure (ENODEV when no GPU is usable). */
b64x_session *b64x_session_open(uint64_t capacity);
void b64x_session_close(b64x_session *s);
uint64_t b64x_session_capacity(const b64x_session *s);
/* Pooled form: acquire takes an idle session of this capacity on the
 * current device from a process-wide pool (opening one if there is none);
 * release waits for the session's queued work and returns it to the pool
 * (closing it when the pool is full).  Opening a session costs pinned
 * allocations and a HIP stream -- milliseconds -- so stages that come and
 * go per message reuse them. */
b64x_session *b64x_session_acquire(uint64_t capacity);
void b64x_session_release(b64x_session *s);
/* Pinned host staging areas: fill host_in, read results from host_out. */
uint8_t *b64x_session_host_in(b64x_session *s);
uint8_t *b64x_session_host_out(b64x_session *s);

/* Synchronous round trips host_in[0..n) -> GPU -> host_out.  The encoder
 * leg encodes all n bytes (padding the final group iff `final` and
 * abc->pad); the caller passes whole 3-byte groups unless `final`.  The
 * decoder leg honours `flags` as b64x_decode_dev(). */
int b64x_session_encode(b64x_session *s, uint64_t n,
                        const b64x_alphabet *abc, uint64_t *out_len);
int b64x_session_decode(b64x_session *s, uint64_t n,
                        const b64x_alphabet *abc, unsigned flags,
                        b64x_dec_result *res);

/* Completion callback of the asynchronous session calls.  It runs on a HIP
 * runtime thread and must not call HIP; it should only signal (set a flag,
 * write an eventfd). */
typedef void (*b64x_done_fn)(void *arg);

/* Asynchronous forms of b64x_session_encode/_decode: enqueue H2D, kernels
 * and D2H on the session's stream and return at once.  `done(arg)` (may be
 * NULL) runs once the call's work has finished; for decode, read the
 * result with b64x_session_decode_result().  One call in flight per
 * session. */
int b64x_session_encode_async(b64x_session *s, uint64_t n,
                              const b64x_alphabet *abc, b64x_done_fn done,
                              void *arg);
/* A caller that decodes one stream in several blocks uses
 * B64X_DEC_HOLD_TAIL and spells the record's held-back sextets in front of
 * its next block itself (ABI version 1's device-side chaining of sessions,
 * `carry_from`, is gone: DESIGN.md §8, "Round 1's decoder-ingress block
 * loss"). */
int b64x_session_decode_async(b64x_session *s, uint64_t n,
                              const b64x_alphabet *abc, unsigned flags,
                              b64x_done_fn done, void *arg);
/* The decode result of the last completed call (host memory; the kernels
 * write it there themselves).  Raw view: prefer the checked form below. */
const b64x_dec_result *b64x_session_result(const b64x_session *s);
/* Checked copy of the last decode's result, to be called once its `done`
 * has run (or after b64x_session_wait).  The record is poisoned before each
 * launch; one that is still poisoned, names another call (seq, nchars or
 * flags differ) or is inconsistent (valid > characters, tail_n != valid
 * mod 4, a held-back sextet >= 64 or a nonzero unused tail byte, out_len
 * not the flags' function of valid) is counted (b64x_diag_counters), the
 * session's stream is waited for and the record is checked again.  0, or
 * -EIO if it is still wrong. */
int b64x_session_decode_result(b64x_session *s, b64x_dec_result *res);
/* Wait for everything queued on the session. */
int b64x_session_wait(b64x_session *s);

/* ---- batch lanes (cross-stream batching of host blocks) --------------- */

/* Pinned host memory for batch arenas (hipHostMalloc, fine-grained); NULL
 * on failure. */
void *b64x_host_alloc(uint64_t bytes);
void b64x_host_free(void *p);

/* A lane: one HIP stream plus device buffers that grow on demand.  It
 * runs ragged batches out of caller-owned pinned arenas; the bytestream_1
 * stages pack many streams' blocks into one batch so that a launch (and
 * its one H2D copy) is amortised over them (ref
 * src/queuestream.c:150-191 being the per-message feed).  The kernels
 * write every output -- characters, bytes, result records -- straight into
 * the pinned host buffers: there is no D2H copy to trust.  After a batch's
 * `done(arg)` has run, the caller checks it with b64x_lane_encode_check /
 * b64x_lane_decode_check before reading anything. */
typedef struct b64x_lane b64x_lane;

b64x_lane *b64x_lane_open(void);
void b64x_lane_close(b64x_lane *l);
/* Pooled form (see b64x_session_acquire): an idle lane of the current
 * device from the process-wide pool, or a new one; release waits for the
 * lane's queued work and pools it. */
b64x_lane *b64x_lane_acquire(void);
void b64x_lane_release(b64x_lane *l);
/* Encode njobs buffers: buffer i is h_in[h_in_off[i] .. h_in_off[i+1])
 * and its b64x_encoded_len(len, abc->pad) characters go to
 * h_out + h_out_off[i] (both offset arrays hold njobs+1 monotone entries
 * starting at 0).  All four host buffers must be pinned (b64x_host_alloc)
 * and stay untouched until `done(arg)` has run.  Asynchronous; the lane's
 * device buffers are grown (synchronously) when a batch needs more.  One
 * batch in flight per lane.
 *
 * h_seg[0 .. nseg) (pinned; nseg may be 0): parts of the batch's input
 * that are not in h_in but elsewhere in pinned host memory -- the input's
 * bytes [off, off+len) are at src (h_in's bytes there are not read) --
 * sorted by off, not overlapping.  A batch with segments is gathered into
 * the device by one kernel that reads h_in and the segments straight from
 * host memory (no DMA of h_in). */
typedef struct {
    uint64_t off, len;
    const uint8_t *src;
} b64x_seg;
int b64x_lane_encode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const b64x_seg *h_seg, uint32_t nseg,
                           const b64x_alphabet *abc, b64x_done_fn done, void *arg);
/* The encode batch whose `done` has run really finished: its completion
 * stamp (written by a kernel queued behind the encode) is there; if not,
 * counted (b64x_diag_counters), waited for and checked again.  0 or -EIO. */
int b64x_lane_encode_check(b64x_lane *l);
/* Lane decode job flag (h_flags): the job is chained -- h_prev[i] names the
 * record whose held-back sextets complete its 4-byte head (below). */
#define B64X_LANE_CHAINED 4u

/* Decode njobs character buffers: job i is h_in[h_in_off[i] ..
 * h_in_off[i+1]), its bytes go to h_out + h_out_off[i] (capacity
 * >= b64x_decoded_cap(len)) and its result record to h_res[i].  h_flags[i]
 * & B64X_DEC_HOLD_TAIL: more of the job's stream follows, so only whole
 * groups are emitted and the last V mod 4 sextets are reported in the
 * record (b64x_decode_dev's HOLD_TAIL); otherwise the job ends its stream
 * and its final partial group is emitted.  Pinned host buffers, as for
 * b64x_lane_encode_async; the records are poisoned here.  *seq receives
 * the batch's sequence number (its records' `seq`; pass it to
 * b64x_lane_decode_check).
 *
 * Chained jobs (one stream decoded in blocks without waiting for each
 * block's record on the host): h_flags[i] & B64X_LANE_CHAINED and h_prev[i]
 * (h_prev may be NULL when no job is chained) points at the pinned host
 * record of an earlier HOLD_TAIL job of the same stream -- in this batch or
 * in a batch queued before it on this lane.  Job i's first 4 characters are
 * a head of characters outside the alphabet; on the device, after that
 * record has been written and before job i is decoded, its last tail_n
 * head bytes are replaced by the record's held-back sextets spelled as
 * alphabet characters, and what was spelled from is logged to h_spell[i]
 * (pinned), which b64x_lane_decode_check compares with the record.
 * Chained jobs and jobs of 128 KiB or more are decoded one after another
 * in job order; the rest in one batch launch before them.
 *
 * Several decode batches may be queued on one lane; they run in order.
 * Encode batches only go to an idle lane. */
int b64x_lane_decode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const uint8_t *h_flags,
                           b64x_dec_result *h_res, const b64x_dec_result *const *h_prev,
                           b64x_dec_result *h_spell, const b64x_alphabet *abc,
                           b64x_done_fn done, void *arg, uint32_t *seq);
/* Checks a finished decode batch's records (see b64x_session_decode_result
 * for what is checked) and, for chained jobs, that the head was spelled
 * from the finished predecessor record: one still poisoned or inconsistent
 * is counted, the lane is waited for and the records are checked again.  0
 * or -EIO. */
int b64x_lane_decode_check(b64x_lane *l, uint32_t seq, const uint64_t *h_in_off,
                           const uint8_t *h_flags, const b64x_dec_result *h_res,
                           const b64x_dec_result *const *h_prev,
                           const b64x_dec_result *h_spell, uint32_t njobs);
/* Wait for everything queued on the lane. */
int b64x_lane_wait(b64x_lane *l);

/* Completion results found unfinished when their `done` had already run:
 * out[0] session decode records, out[1] lane batches (process-wide totals,
 * for tests and diagnostics). */
void b64x_diag_counters(uint64_t out[2]);
/* Paths the automatic decodes took (process-wide totals, for tests and
 * diagnostics): out[0] probes launched, out[1] probes skipped on a held
 * model, out[2] hinted single passes, out[3] row-batch preps launched,
 * out[4] row-batch preps skipped (the workspace's row model reused). */
void b64x_diag_paths(uint64_t out[5]);

/* ---- utilities ----------------------------------------------------------- */

/* Fill n bytes with the splitmix64 stream used by every synthetic
 * workload: 8 little-endian bytes per step,
 * state = seed + k*0x9E3779B97F4A7C15 for k = 1, 2, ... */
int b64x_fill_splitmix64(void *d_out, uint64_t n, uint64_t seed,
                         void *stream);

/* 0 if a gfx950 device is usable, -ENODEV otherwise. */
int b64x_device_check(void);

/* ---- host placement ------------------------------------------------------ */

/* The NUMA node the GPU `device` (-1: the current device) hangs off, from
 * sysfs; -ENOENT when unknown (no NUMA, a virtual device).  */
int b64x_device_numa_node(int device);
/* Bind the calling thread to the CPUs of `device`'s NUMA node (-1: the
 * current device) that its affinity mask allows, and prefer that node for
 * the pages it faults in.  Event loops that feed a GPU spend their time
 * copying messages into pinned arenas and reading frames back: one loop ran
 * config 5 at 6.1-6.2 GiB/s on the GPU's node and 4.4-4.5 on the other
 * socket of the same box (profiles/r06_numa_probe.jsonl).  A thread whose
 * mask already lies inside one node (the application placed it) is left as
 * it is.  Returns the node the thread runs on afterwards, or a negative errno
 * (-ENOENT: the node or its CPUs are unknown; the thread is unchanged).  The
 * batching hub calls it on a loop's thread when the loop gets its first GPU
 * stage, unless ASYNC_B64_BIND=0. */
int b64x_bind_thread(int device);
/* Static description of the compiled kernels (for logs). */
const char *b64x_build_info(void);
const char *b64x_strerror(int err);

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_B64X_H */
