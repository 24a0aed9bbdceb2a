// b64x_kernels.hip -- hand-written gfx950 (CDNA4) kernels for the base64
// byte-stream stage, plus the extern "C" shim declared in include/b64x.h.
//
// What the reference does (all CPU, one byte per loop trip):
//   encode: src/base64encoder.c:132-139 shifts each input byte into a bit
//           accumulator and emits a character per 6 bits through map()
//           (:49-59); finalize() (:61-99) emits the last 1-2 characters
//           and the padding.
//   decode: src/base64decoder.c:67-77 maps each character through a
//           256-entry table plus the pos62/pos63 checks (:38-48), skips
//           non-alphabet bytes and emits a byte per 8 accumulated bits.
//
// How it runs here (DESIGN.md §5 has the byte budget and the rooflines):
//   * encode is stateless per 3-byte group.  One lane turns 12 input bytes
//     (one dwordx3 load) into 16 characters (one dwordx4 store), one quad
//     per lane; the 64-entry alphabet sits in LDS and is read with
//     ds_read_u8 (k_encode_flat and the batch kernels).  Byte
//     regrouping is v_perm_b32, not shifts (k_encode_flat; batches:
//     k_encode_tight2, k_encode_strided, k_encode_ragged).
//   * decode is stateful only through the number of alphabet characters
//     seen so far.  For inputs up to 2^31 characters: k_decode_probe reads
//     the stream's first 256 bytes for a line model -- lines of L alphabet
//     characters and s separator bytes, L = 0 for clean input -- under which
//     every character's output place is known in closed form, and checks
//     256 samples further in against it (junk there cuts the model's slots);
//     k_decode_lines is output-indexed (lane slot t = sextets [16t, 16t+16)
//     = output bytes [12t, 12t+12)), loads each slot's span, drops the
//     separator with funnel shifts, checks it and stores 12 bytes, and
//     publishes the first slot that does not fit the model;
//     k_decode_suffix_held decodes exactly whatever follows that slot
//     (nothing, on clean and MIME-formatted text): persistent tiles of 16
//     ranges of 2,048 characters, each decoded once and held in VGPRs until
//     the tile's prefix (group sums) is known, and the range body
//     that ORs each lane's compacted sextet fields into a wave's LDS window
//     (v_perm compaction, v_dot4 fields, ds_or) -- the window's bytes are
//     the output bytes.  Larger inputs: pass 1 (input-indexed fast paths),
//     a scan, pass 2 with the same range body.
//   * batches: the row kernel (k_decode_rows_lines, rows with room) takes
//     clean rows lane by lane and MIME-formatted rows by the same line
//     model (k_rows_prep probes row 0), and marks rows with junk once per
//     wave; the fix-up (k_decode_batch_fix2) decodes the marked rows with
//     the bit-stream range body, one wave per row.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <type_traits>
#include <utility>

#include "b64x.h"
#include "b64x_result_check.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kThreads = 256;  // 4 waves of 64
constexpr int kWavesPerBlock = kThreads / 64;
constexpr int kChunk = 1024;            // characters per wave step
constexpr uint32_t kMaxRanges = 1u << 20; // decode ranges (waves) per call
constexpr uint64_t kRangeChunks = 2;    // default decode range: 2 KiB
constexpr int kEncUnroll = 4;           // quads in flight per lane

typedef uint32_t u32x3a4 __attribute__((ext_vector_type(3), aligned(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

struct EncAlpha {
    uint32_t p62, p63, padc, pad;
};

// Effective decode alphabet: p62/p63 are the reference's `char` values
// after defaulting, sign-extended like the comparison at
// src/base64decoder.c:43-46 (uint8_t vs char on x86-64), so a negative
// value never matches any byte.
struct DecAlpha {
    int p62, p63;
};

// ---------------------------------------------------------------- tables --

// src/base64encoder.c:26-27 (62-char map) + :49-59 (62 -> pos62, 63 -> pos63)
DEV uint32_t enc_char(uint32_t v, const EncAlpha &a)
{
    return v < 26 ? 'A' + v
         : v < 52 ? 'a' + (v - 26)
         : v < 62 ? '0' + (v - 52)
         : v == 62 ? a.p62 : a.p63;
}

// fsdyn's base64_bitfield_decoding (62 alphanumerics -> 0..61, assumption
// recorded in DESIGN.md) followed by the pos62/pos63 fallbacks of
// src/base64decoder.c:38-48.  0xFF marks "not in the alphabet".
DEV uint32_t dec_value(uint32_t c, const DecAlpha &a)
{
    if (c - 'A' < 26u) return c - 'A';
    if (c - 'a' < 26u) return c - 'a' + 26;
    if (c - '0' < 10u) return c - '0' + 52;
    if ((int) c == a.p62) return 62;
    if ((int) c == a.p63) return 63;
    return 0xFF;
}

DEV void build_enc_table(uint8_t *tab, const EncAlpha &a)
{
    if (threadIdx.x < 64) tab[threadIdx.x] = (uint8_t) enc_char(threadIdx.x, a);
}

DEV void build_dec_table(uint8_t *tab, const DecAlpha &a)
{
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x)
        tab[c] = (uint8_t) dec_value(c, a);
}

// The bit-stream decode's form (k_decode_suffix_held): sextet v as 4 v, 0xFF
// for "not in the alphabet" -- the flag in bit 0, so a dword's four flags
// are one AND, and the sextets still pack by v_dot4 (weights 64, 1).
DEV void build_dec_table_lo(uint8_t *tab, const DecAlpha &a)
{
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) {
        const uint32_t v = dec_value(c, a);
        tab[c] = (uint8_t) (v < 64 ? v << 2 : 0xFFu);
    }
}

// ------------------------------------------------------- memory helpers --

typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x4a16 __attribute__((ext_vector_type(4), aligned(16)));

// Store the first `nbytes` (0..12) bytes of {o0, o1, o2}: whole dwords when
// `p` is dword aligned, then at most 3 single bytes.
// The first nbytes (<= 12) bytes of o0:o1:o2 one at a time, in a loop the
// compiler keeps rolled: for the rare tail blocks of a hot kernel, whose
// unrolled byte tests (store_bytes12) the compiler hoists out of the
// kernel's slot loop as SGPR masks that then spill.
DEV void store_bytes12_rolled(uint8_t *p, uint32_t o0, uint32_t o1, uint32_t o2, uint32_t nbytes)
{
#pragma unroll 1
    for (uint32_t k = 0; k < nbytes; k++) {
        const uint32_t w = k < 4 ? o0 : k < 8 ? o1 : o2;
        p[k] = (uint8_t) (w >> (8 * (k & 3)));
    }
}

DEV void store_bytes12(uint8_t *p, uint32_t o0, uint32_t o1, uint32_t o2,
                       uint32_t nbytes)
{
    if ((((uintptr_t) p) & 3) == 0) {
        const uint32_t nd = nbytes >> 2;
        if (nd == 3) {
            *(u32x3a4 *) p = u32x3a4{o0, o1, o2};
            return;
        }
        if (nd == 2) *(u32x2a4 *) p = u32x2a4{o0, o1};
        else if (nd == 1) *(uint32_t *) p = o0;
        const uint32_t rem = nbytes & 3;
        if (rem) {
            const uint32_t w = nd == 0 ? o0 : nd == 1 ? o1 : o2;
            uint8_t *q = p + 4 * nd;
            q[0] = (uint8_t) w;
            if (rem > 1) q[1] = (uint8_t) (w >> 8);
            if (rem > 2) q[2] = (uint8_t) (w >> 16);
        }
        return;
    }
    uint32_t w[3] = {o0, o1, o2};
#pragma unroll
    for (uint32_t i = 0; i < 12; i++)
        if (i < nbytes) p[i] = (uint8_t) (w[i >> 2] >> (8 * (i & 3)));
}

// Same for up to 16 bytes.
DEV void store_bytes16(uint8_t *p, const uint32_t w[4], uint32_t nbytes)
{
    if (nbytes == 16 && (((uintptr_t) p) & 3) == 0) {
        *(u32x4a4 *) p = u32x4a4{w[0], w[1], w[2], w[3]};
        return;
    }
    if (nbytes > 12) {
        store_bytes12(p, w[0], w[1], w[2], 12);
        store_bytes12(p + 12, w[3], 0, 0, nbytes - 12);
    } else {
        store_bytes12(p, w[0], w[1], w[2], nbytes);
    }
}

// True when the 16 bytes at p lie in one 4 KiB page.  A load of them is
// then safe as soon as one of them belongs to a live buffer: memory is
// mapped page-wise, so a window that shares a page with an in-range byte
// cannot fault.  The extra bytes are never used (callers mask by count).
DEV bool same_page16(const uint8_t *p)
{
    return (((uintptr_t) p) & 4095) <= 4096 - 16;
}

// Up to 16 characters at `p`, `nin` (>= 1) of which are inside the range;
// the others are unspecified (callers mask them out by position).
DEV uint4 load_chars(const uint8_t *p, uint32_t nin)
{
    if ((((uintptr_t) p) & 3) == 0 && (nin == 16 || same_page16(p))) {
        u32x4a4 v = *(const u32x4a4 *) p;
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        if (i < nin) w[i >> 2] |= (uint32_t) p[i] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// __syncthreads() with every LDS access of this wave done first.  hipcc's
// barrier for a workgroup-scope release did not always wait for them: in
// k_decode_suffix_held's loop the barrier at the top of an iteration had no
// lgkmcnt(0) behind thread 0's write of the next tile's ticket at the end of
// the last one, and now and then another wave read the old ticket after the
// barrier (profiles/r05_sfx_held_stress*.jsonl: one 1 GiB decode in 5 wrong
// at 3 ranges per wave, the waves' tickets seen differing; none with this).
DEV void block_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
}

// ----------------------------------------------------------- encode core --

// 3 bytes (big-endian in bits 23..0) -> 4 characters, little-endian dword.
DEV uint32_t enc_group(const uint8_t *tab, uint32_t g)
{
    uint32_t c0 = tab[g >> 18];
    uint32_t c1 = tab[(g >> 12) & 63];
    uint32_t c2 = tab[(g >> 6) & 63];
    uint32_t c3 = tab[g & 63];
    return c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
}

// 12 input bytes in dwords a, b, c -> 16 characters.
DEV uint4 enc_quad(const uint8_t *tab, uint32_t a, uint32_t b, uint32_t c)
{
    // v_perm_b32 selectors: byte i of the result picks byte sel[i] of
    // {S0:S1} (0-3 = S1, 4-7 = S0, 0x0c = zero).
    uint32_t g0 = __builtin_amdgcn_perm(0u, a, 0x0c000102u);  // in0 in1 in2
    uint32_t g1 = __builtin_amdgcn_perm(b, a, 0x0c030405u);   // in3 in4 in5
    uint32_t g2 = __builtin_amdgcn_perm(c, b, 0x0c020304u);   // in6 in7 in8
    uint32_t g3 = __builtin_amdgcn_perm(0u, c, 0x0c010203u);  // in9 in10 in11
    uint4 o;
    o.x = enc_group(tab, g0);
    o.y = enc_group(tab, g1);
    o.z = enc_group(tab, g2);
    o.w = enc_group(tab, g3);
    return o;
}

// Encode r (1..12) bytes at `src` byte by byte; `last` = these are the
// final bytes of the stream (finalize(), src/base64encoder.c:61-99:
// a trailing 1 or 2 bytes give 2 or 3 characters, then padding).
// Returns the number of characters written.
DEV uint32_t enc_bytes(const uint8_t *tab, const uint8_t *src, uint32_t r,
                       uint8_t *dst, bool last, const EncAlpha &a)
{
    uint32_t o = 0, k = 0;
    for (; k + 3 <= r; k += 3) {
        uint32_t g = ((uint32_t) src[k] << 16) | ((uint32_t) src[k + 1] << 8) | src[k + 2];
        dst[o++] = tab[g >> 18];
        dst[o++] = tab[(g >> 12) & 63];
        dst[o++] = tab[(g >> 6) & 63];
        dst[o++] = tab[g & 63];
    }
    uint32_t rem = r - k;
    if (rem) {
        uint32_t g = (uint32_t) src[k] << 16;
        if (rem == 2) g |= (uint32_t) src[k + 1] << 8;
        dst[o++] = tab[g >> 18];
        dst[o++] = tab[(g >> 12) & 63];
        if (rem == 2) dst[o++] = tab[(g >> 6) & 63];
        if (last && a.pad) {
            dst[o++] = (uint8_t) a.padc;
            if (rem == 1) dst[o++] = (uint8_t) a.padc;
        }
    }
    return o;
}

// The final r (1..11) bytes of a buffer at a dword-aligned `src`: loaded as
// one 12-byte window when it stays in the page of its first byte (else
// bytewise), encoded like a quad with the missing bytes zeroed, the partial
// group's padding (finalize(), src/base64encoder.c:61-99) merged in, and
// stored as whole dwords plus at most 3 bytes.
DEV void enc_tail(const uint8_t *tab, const uint8_t *src, uint32_t r, uint8_t *dst,
                  const EncAlpha &a)
{
    uint32_t x, y, z;
    if ((((uintptr_t) src) & 4095) <= 4096 - 12) {
        u32x3a4 v = *(const u32x3a4 *) src;
        x = v.x;
        y = v.y;
        z = v.z;
    } else {
        uint32_t w[3] = {0, 0, 0};
        for (uint32_t i = 0; i < r; i++) w[i >> 2] |= (uint32_t) src[i] << (8 * (i & 3));
        x = w[0];
        y = w[1];
        z = w[2];
    }
    // zero the bytes at and past r
    x &= r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1;
    y &= r >= 8 ? 0xFFFFFFFFu : r <= 4 ? 0u : (1u << (8 * (r - 4))) - 1;
    z &= r <= 8 ? 0u : (1u << (8 * (r - 8))) - 1;
    const uint4 o = enc_quad(tab, x, y, z);
    uint32_t dw[4] = {o.x, o.y, o.z, o.w};
    const uint32_t ng = r / 3, rem = r % 3;
    uint32_t m = 4 * ng;
    if (rem) {
        const uint32_t keep = rem + 1;  // characters of the partial group
        if (a.pad) {
            const uint32_t mask = keep == 2 ? 0xFFFFu : 0xFFFFFFu;
            const uint32_t pads = a.padc * 0x01010101u;
#pragma unroll
            for (uint32_t g = 0; g < 4; g++)
                if (g == ng) dw[g] = (dw[g] & mask) | (pads & ~mask);
            m += 4;
        } else {
            m += keep;
        }
    }
    store_bytes16(dst, dw, m);
}

// Encode one quad slot: full 12-byte quads with dword-aligned source and
// destination go through dwordx3 load / dwordx4 store; everything else
// (buffer tail, misaligned buffers) bytewise.
DEV void enc_slot(const uint8_t *tab, const uint8_t *src, uint64_t avail,
                  uint8_t *dst, const EncAlpha &a)
{
    if (avail >= 12 && ((((uintptr_t) src) | ((uintptr_t) dst)) & 3) == 0) {
        u32x3a4 v = *(const u32x3a4 *) src;
        uint4 o = enc_quad(tab, v.x, v.y, v.z);
        *(u32x4a4 *) dst = u32x4a4{o.x, o.y, o.z, o.w};
    } else {
        uint32_t r = avail < 12 ? (uint32_t) avail : 12;
        enc_bytes(tab, src, r, dst, avail <= 12, a);
    }
}

// Single buffer (nbuf == 1) or uniform-stride batch.  Lane slot t covers
// quad q of buffer b; slots are dealt so that one wave instruction touches
// 64 consecutive quads (768 B in, 1 KiB out).
__global__ __launch_bounds__(kThreads) void k_encode(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint64_t len,
    uint32_t nbuf, uint8_t *__restrict__ out, uint64_t out_stride,
    uint64_t quads_per_buf, uint64_t total_slots, EncAlpha a)
{
    __shared__ uint8_t tab[64];
    build_enc_table(tab, a);
    block_sync();

    const uint64_t step = (uint64_t) gridDim.x * kThreads * kEncUnroll;
    for (uint64_t base = (uint64_t) blockIdx.x * kThreads * kEncUnroll;
         base < total_slots; base += step) {
        // Issue every load of this step before any compute (memory-level
        // parallelism: kEncUnroll x 768 B per wave in flight).
        uint32_t va[kEncUnroll], vb[kEncUnroll], vc[kEncUnroll];
        const uint8_t *srcs[kEncUnroll];
        uint8_t *dsts[kEncUnroll];
        uint64_t avails[kEncUnroll];
        bool fast[kEncUnroll];
#pragma unroll
        for (int u = 0; u < kEncUnroll; u++) {
            uint64_t t = base + (uint64_t) u * kThreads + threadIdx.x;
            fast[u] = false;
            avails[u] = 0;
            srcs[u] = in;
            dsts[u] = out;
            if (t < total_slots) {
                uint64_t b, q;
                if (nbuf == 1) {
                    b = 0;
                    q = t;
                } else {
                    uint32_t t32 = (uint32_t) t, qp = (uint32_t) quads_per_buf;
                    uint32_t b32 = t32 / qp;
                    b = b32;
                    q = t32 - b32 * qp;
                }
                const uint8_t *src = in + b * in_stride + q * 12;
                uint8_t *dst = out + b * out_stride + q * 16;
                uint64_t avail = len - q * 12;
                srcs[u] = src;
                dsts[u] = dst;
                avails[u] = avail;
                fast[u] = avail >= 12 && ((((uintptr_t) src) | ((uintptr_t) dst)) & 3) == 0;
                if (fast[u]) {
                    u32x3a4 v = *(const u32x3a4 *) src;
                    va[u] = v.x;
                    vb[u] = v.y;
                    vc[u] = v.z;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kEncUnroll; u++) {
            if (fast[u]) {
                uint4 o = enc_quad(tab, va[u], vb[u], vc[u]);
                *(u32x4a4 *) dsts[u] = u32x4a4{o.x, o.y, o.z, o.w};
            } else if (avails[u]) {
                uint32_t r = avails[u] < 12 ? (uint32_t) avails[u] : 12;
                enc_bytes(tab, srcs[u], r, dsts[u], avails[u] <= 12, a);
            }
        }
    }
}

template <bool NT>
DEV void store16(uint8_t *p, uint4 o)
{
    if (NT) {
        __builtin_nontemporal_store(u32x4a4{o.x, o.y, o.z, o.w}, (u32x4a4 *) p);
    } else {
        *(u32x4a4 *) p = u32x4a4{o.x, o.y, o.z, o.w};
    }
}

template <bool NT>
DEV u32x3a4 ld12(const uint8_t *p)
{
    if (NT) return __builtin_nontemporal_load((const u32x3a4 *) p);
    return *(const u32x3a4 *) p;
}

// One dword-aligned device buffer (the BASELINE config-2 hot path): one
// quad (12 bytes in, 16 characters out) per lane, the n/12 full quads in
// tiles of one 256-lane block each; a block takes whole tiles with no
// per-lane guards, so loads and stores are never exec-masked and the
// compiler can wait on loads with counted vmcnt instead of draining the
// stores (vmcnt counts both).  Loads and stores are non-temporal, the
// 64-character alphabet an LDS table.  Launched with one block per tile (a
// non-persistent grid streams fastest here: tests/tools/copy_sweep.hip; the
// loop only matters past 2^31 tiles).  The last, partial tile and the final
// n mod 12 bytes (with padding) are done by the last block.  Measured forms
// (DESIGN.md §5): one quad per lane with the LDS table 397 us per 1 GiB
// (profiles/r03_ab_enc*.jsonl); the alphabet read across lanes by
// ds_bpermute 445 us; two quads per lane 405; 512- and 1,024-lane blocks
// +20 / +120 us; software pipelining and cached loads slower (r01_v6_*).
constexpr uint32_t kEncTH = 256;


__global__ __launch_bounds__(kEncTH) void k_encode_flat(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, uint64_t full, uint64_t n,
    EncAlpha a)
{
    // `full` (the whole tiles) comes from the host, so a wave issues its
    // load without a 64-bit division by 12 first.
    __shared__ uint8_t tab[64];
    const uint32_t tid = threadIdx.x;
    build_enc_table(tab, a);
    block_sync();
    for (uint64_t t = blockIdx.x; t < full; t += gridDim.x) {
        const uint64_t q = t * kEncTH + tid;
        const u32x3a4 v = ld12<true>(in + q * 12);
        store16<true>(out + q * 16, enc_quad(tab, v.x, v.y, v.z));
    }
    if (blockIdx.x == gridDim.x - 1) {
        const uint64_t nq = n / 12;
        for (uint64_t q = full * kEncTH + tid; q < nq; q += kEncTH) {
            const u32x3a4 v = *(const u32x3a4 *) (in + q * 12);
            store16<true>(out + q * 16, enc_quad(tab, v.x, v.y, v.z));
        }
        if (tid == 0 && n % 12)
            enc_bytes(tab, in + nq * 12, (uint32_t) (n % 12), out + nq * 16, true, a);
    }
}

// Uniform-stride batch encode: slot t = (buffer t / Q, quad t mod Q), Q =
// quads per buffer; one tile of U slots per lane per block (non-persistent
// grid), non-temporal loads and stores on whole, dword-aligned quads, the
// buffer tails (and misaligned buffers) bytewise.
template <int U, bool NTL>
__global__ __launch_bounds__(kThreads) void k_encode_strided(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint64_t len,
    uint32_t nbuf, uint8_t *__restrict__ out, uint64_t out_stride,
    uint32_t qpb, uint32_t total_slots, EncAlpha a)
{
    __shared__ uint8_t tab[64];
    build_enc_table(tab, a);
    block_sync();
    u32x3a4 v[U];
    const uint8_t *srcs[U];
    uint8_t *dsts[U];
    uint64_t avails[U];
    bool fast[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t t = (blockIdx.x * U + u) * kThreads + threadIdx.x;
        fast[u] = false;
        avails[u] = 0;
        srcs[u] = in;
        dsts[u] = out;
        if (t < total_slots) {
            const uint32_t b = t / qpb, q = t - b * qpb;
            srcs[u] = in + (uint64_t) b * in_stride + (uint64_t) q * 12;
            dsts[u] = out + (uint64_t) b * out_stride + (uint64_t) q * 16;
            avails[u] = len - (uint64_t) q * 12;
            fast[u] = avails[u] >= 12 && ((((uintptr_t) srcs[u]) | ((uintptr_t) dsts[u])) & 3) == 0;
            if (fast[u]) v[u] = ld12<NTL>(srcs[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (fast[u]) {
            store16<true>(dsts[u], enc_quad(tab, v[u].x, v[u].y, v[u].z));
        } else if (avails[u]) {
            const uint32_t r = avails[u] < 12 ? (uint32_t) avails[u] : 12;
            if (avails[u] < 12 && (((uintptr_t) srcs[u]) & 3) == 0)
                enc_tail(tab, srcs[u], r, dsts[u], a);
            else
                enc_bytes(tab, srcs[u], r, dsts[u], avails[u] <= 12, a);
        }
    }
}

// The seam lane of k_encode_tight2: x, y, z are the 12 input bytes from
// the lane's first group on, q the normal encoding of them, p the lane's
// character offset in its buffer (p + 16 >= E, r = len % 3 != 0).  Groups
// before the partial group gs are q's; the partial group keeps q's first
// r characters, gets the character of the zero-extended last byte and the
// padding (finalize(), src/base64encoder.c:61-99); groups after it start
// the next buffer, whose bytes sit 3 - r earlier than a full group would
// put them -- i.e. the 9 bytes from offset r, encoded one group later.
DEV uint4 enc_seam2(const uint8_t *tab, uint32_t x, uint32_t y, uint32_t z, uint4 q,
                    uint32_t p, uint32_t E, uint32_t r, const EncAlpha &a)
{
    const uint32_t gs = ((E - p) >> 2) - 1;  // 0..3
    // groups of the next buffer: bytes r .. r+8 of x:y:z
    const uint32_t x2 = __builtin_amdgcn_alignbyte(y, x, r);
    const uint32_t y2 = __builtin_amdgcn_alignbyte(z, y, r);
    const uint32_t z2 = __builtin_amdgcn_alignbyte(0u, z, r);
    const uint32_t n0 = enc_group(tab, __builtin_amdgcn_perm(0u, x2, 0x0c000102u));
    const uint32_t n1 = enc_group(tab, __builtin_amdgcn_perm(y2, x2, 0x0c030405u));
    const uint32_t n2 = enc_group(tab, __builtin_amdgcn_perm(z2, y2, 0x0c020304u));
    // the partial group: last real byte is byte 3*gs + r - 1 of x:y:z
    const uint32_t bi = 3 * gs + r - 1;
    const uint32_t wd = bi < 4 ? x : bi < 8 ? y : z;
    const uint32_t lb = (wd >> (8 * (bi & 3))) & 0xFFu;
    const uint32_t qg = gs == 0 ? q.x : gs == 1 ? q.y : gs == 2 ? q.z : q.w;
    const uint32_t pads = a.padc * 0x01010101u;
    const uint32_t pg = r == 1
        ? (qg & 0xFFu) | ((uint32_t) tab[(lb & 3u) << 4] << 8) | (pads & 0xFFFF0000u)
        : (qg & 0xFFFFu) | ((uint32_t) tab[(lb & 15u) << 2] << 16) | (pads & 0xFF000000u);
    uint4 o;
    o.x = gs == 0 ? pg : q.x;
    o.y = gs == 1 ? pg : gs == 0 ? n0 : q.y;
    o.z = gs == 2 ? pg : gs < 2 ? n1 : q.z;
    o.w = gs == 3 ? pg : n2;
    return o;
}

// Tight-layout batch encode, second form: the block's first output slot
// gives its buffer b0 and offset p0 once (scalar), each lane's slot is a
// 32-bit offset from there, split with a 32-bit multiply-high (magic =
// ceil(2^32/E), exact below 2^32/E -- the launcher checks).  Seam lanes
// (one per buffer) take enc_seam2.  Blocks that touch the last two buffers
// or the end of the output ("tail" blocks, block-uniform) guard their
// loads and stores, so one launch covers the whole batch.
template <int U>
__global__ __launch_bounds__(kThreads) void k_encode_tight2(
    const uint8_t *__restrict__ in, uint64_t len, uint32_t E, uint32_t r, uint32_t magic,
    uint64_t m64, uint8_t *__restrict__ out, uint64_t nslots, uint64_t total_in,
    uint64_t total_out, uint64_t tail_slot, EncAlpha a)
{
    __shared__ uint8_t tab[64];
    build_enc_table(tab, a);
    block_sync();
    const uint64_t s0 = (uint64_t) blockIdx.x * U * kThreads;
    const uint64_t b0 = __umul64hi(16 * s0, m64);
    const uint32_t p0 = (uint32_t) (16 * s0 - b0 * E);
    const uint8_t *ib = in + b0 * len;
    uint32_t pp[U];
    uint64_t pos[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t rel = p0 + 16u * (u * kThreads + threadIdx.x);
        const uint32_t bl = __umulhi(rel, magic);
        pp[u] = rel - bl * E;
        pos[u] = (uint64_t) bl * len + 3 * (pp[u] >> 2);
    }
    if (s0 + U * kThreads > tail_slot) {
        // tail block: guarded loads (the last buffer's windows may run past
        // the input) and stores (the output may end inside a slot)
        for (int u = 0; u < U; u++) {
            const uint64_t t = s0 + (u * kThreads + threadIdx.x);
            if (t >= nslots) continue;
            const uint8_t *src = ib + (pos[u] & ~3ull);
            const uint64_t gofs = (uint64_t) (src - in);
            const uint32_t nin = total_in - gofs >= 16 ? 16u : (uint32_t) (total_in - gofs);
            const uint4 w = load_chars(src, nin);
            const uint32_t s = (uint32_t) (pos[u] & 3);
            const uint32_t x = __builtin_amdgcn_alignbyte(w.y, w.x, s);
            const uint32_t y = __builtin_amdgcn_alignbyte(w.z, w.y, s);
            const uint32_t z = __builtin_amdgcn_alignbyte(w.w, w.z, s);
            uint4 c = enc_quad(tab, x, y, z);
            if (r != 0 && pp[u] + 16 >= E) c = enc_seam2(tab, x, y, z, c, pp[u], E, r, a);
            const uint32_t dw[4] = {c.x, c.y, c.z, c.w};
            const uint64_t left = total_out - 16 * t;
            store_bytes16(out + 16 * t, dw, left >= 16 ? 16u : (uint32_t) left);
        }
        return;
    }
    u32x4a4 w[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        w[u] = __builtin_nontemporal_load((const u32x4a4 *) (ib + (pos[u] & ~3ull)));
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t s = (uint32_t) (pos[u] & 3);
        const uint32_t x = __builtin_amdgcn_alignbyte(w[u].y, w[u].x, s);
        const uint32_t y = __builtin_amdgcn_alignbyte(w[u].z, w[u].y, s);
        const uint32_t z = __builtin_amdgcn_alignbyte(w[u].w, w[u].z, s);
        uint4 c = enc_quad(tab, x, y, z);
        if (r != 0 && pp[u] + 16 >= E) c = enc_seam2(tab, x, y, z, c, pp[u], E, r, a);
        store16<true>(out + 16 * (s0 + (u * kThreads + threadIdx.x)), c);
    }
}

// Ragged batch: one block per buffer.
__global__ __launch_bounds__(kThreads) void k_encode_ragged(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
    uint32_t nbuf, uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off,
    EncAlpha a)
{
    __shared__ uint8_t tab[64];
    build_enc_table(tab, a);
    block_sync();
    for (uint32_t b = blockIdx.x; b < nbuf; b += gridDim.x) {
        const uint64_t beg = in_off[b], len = in_off[b + 1] - beg;
        const uint8_t *src = in + beg;
        uint8_t *dst = out + out_off[b];
        const uint64_t quads = (len + 11) / 12;
        for (uint64_t q = threadIdx.x; q < quads; q += kThreads)
            enc_slot(tab, src + q * 12, len - q * 12, dst + q * 16, a);
    }
}

// ----------------------------------------------------------- decode core --

DEV uint32_t lane_id() { return threadIdx.x & 63; }

// Keep the compiler from moving LDS accesses across this point.  Within
// one wave the LDS executes DS instructions in issue order, so program
// order is all that cross-lane hand-offs in the wave's scratch need.
DEV void wave_lds_order()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// Four groups -> 12 output bytes as three little-endian dwords.
DEV void groups_to_bytes(uint32_t G0, uint32_t G1, uint32_t G2, uint32_t G3,
                         uint32_t &o0, uint32_t &o1, uint32_t &o2)
{
    o0 = __builtin_amdgcn_perm(G1, G0, 0x06000102u);  // G0.b2 G0.b1 G0.b0 G1.b2
    o1 = __builtin_amdgcn_perm(G2, G1, 0x05060001u);  // G1.b1 G1.b0 G2.b2 G2.b1
    o2 = __builtin_amdgcn_perm(G3, G2, 0x04050600u);  // G2.b0 G3.b2 G3.b1 G3.b0
}

// Hot-path mapping: 16 table lookups folded straight into the four 24-bit
// groups of the lane (3 v_lshl_or per group) plus an OR accumulator;
// `bad` is nonzero unless all 16 characters are present and in the
// alphabet (then G is exact).
DEV void map_fast(const uint8_t *tab, uint4 w, uint32_t nin, uint32_t G[4], uint32_t &bad)
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t acc = nin < 16 ? 0x80u : 0u;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint32_t t0 = tab[dw[g] & 0xFFu];
        uint32_t t1 = tab[(dw[g] >> 8) & 0xFFu];
        uint32_t t2 = tab[(dw[g] >> 16) & 0xFFu];
        uint32_t t3 = tab[dw[g] >> 24];
        G[g] = (t0 << 18) | (t1 << 12) | (t2 << 6) | t3;
        acc |= t0 | t1 | t2 | t3;
    }
    bad = acc & ~63u;
}

// map_fast keeping the OR of each dword's four table values (A[g] < 64:
// dword g is all alphabet), for callers that judge dwords separately.
DEV void map_fast_acc(const uint8_t *tab, uint4 w, uint32_t G[4], uint32_t A[4])
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint32_t t0 = tab[dw[g] & 0xFFu];
        uint32_t t1 = tab[(dw[g] >> 8) & 0xFFu];
        uint32_t t2 = tab[(dw[g] >> 16) & 0xFFu];
        uint32_t t3 = tab[dw[g] >> 24];
        G[g] = (t0 << 18) | (t1 << 12) | (t2 << 6) | t3;
        A[g] = t0 | t1 | t2 | t3;
    }
}

// Slow-path view of a lane's 16 characters: groups with every absent or
// non-alphabet character's sextet zeroed, and the alphabet bit mask.
DEV uint4 load16_a4(const uint8_t *p)
{
    u32x4a4 v = *(const u32x4a4 *) p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct LaneChunk {
    uint32_t G[4];
    uint32_t vmask;  // bit k: character k present and in the alphabet
};

DEV void map_chunk(const uint8_t *tab_, uint4 w, uint32_t nin, LaneChunk &lc)
{
    // Re-read the table (volatile): sharing the hot path's lookups would keep
    // all 16 per-character values of every in-flight chunk alive.
    const volatile uint8_t *tab = tab_;
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = 4 * g + j;
            uint32_t t = tab[(dw[g] >> (8 * j)) & 0xFFu];
            bool ok = t < 64u && (uint32_t) k < nin;
            v |= (ok ? t : 0u) << (18 - 6 * j);
            m |= (ok ? 1u : 0u) << k;
        }
        lc.G[g] = v;
    }
    lc.vmask = m;
}

// map_chunk without the volatile re-read, for kernels whose table pointer
// the compiler can see is LDS (a volatile access defeats address-space
// inference and becomes a FLAT load, counted against VMEM).
DEV void map_chunk_lds(const uint8_t *tab, uint4 w, uint32_t nin, LaneChunk &lc)
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int k = 4 * g + j;
            uint32_t t = tab[(dw[g] >> (8 * j)) & 0xFFu];
            bool ok = t < 64u && (uint32_t) k < nin;
            v |= (ok ? t : 0u) << (18 - 6 * j);
            m |= (ok ? 1u : 0u) << k;
        }
        lc.G[g] = v;
    }
    lc.vmask = m;
}

// A row slot's 16 characters for the line-structured row kernel: G the four
// groups with each non-alphabet character's sextet replaced by 0x3F, *im bit
// i set when character i is not in the alphabet.  In a slot that passes, the
// replaced sextets all sit after its alphabet prefix (j characters), so they
// only reach output bits past its floor(6j/8) counted bytes.  Per dword: the
// four table values packed, the group by two v_dot4 of their low 6 bits, the
// bit-7s gathered by a third (no 32-bit multiply: those issue at a quarter
// of the VALU rate, and the first form's two per dword made the MIME rows VALU-bound).
DEV void map_row_slot(const uint8_t *tab, uint4 w, uint32_t G[4], uint32_t &im)
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const uint32_t P = (uint32_t) tab[dw[g] & 0xFFu] | ((uint32_t) tab[(dw[g] >> 8) & 0xFFu] << 8) |
                           ((uint32_t) tab[(dw[g] >> 16) & 0xFFu] << 16) |
                           ((uint32_t) tab[dw[g] >> 24] << 24);
        const uint32_t Pz = P & 0x3F3F3F3Fu;
        const uint32_t hi = __builtin_amdgcn_udot4(Pz, 0x00000140u, 0u, false);  // s0*64 + s1
        const uint32_t lo = __builtin_amdgcn_udot4(Pz, 0x01400000u, 0u, false);  // s2*64 + s3
        G[g] = (hi << 12) | lo;
        // 128 x (the dword's 4-bit non-alphabet mask)
        m |= __builtin_amdgcn_udot4(P & 0x80808080u, 0x08040201u, 0u, false) << (4 * g);
    }
    im = m >> 7;
}

// Fast path (a): a lane's 16 alphabet characters, as 4 groups, to 12 bytes.
DEV void emit_full(const uint32_t G[4], uint8_t *out)
{
    uint32_t o0, o1, o2;
    groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
    store_bytes12(out + 12 * lane_id(), o0, o1, o2, 12);
}

// Hot-path form: `out` is known dword aligned (checked once, uniformly, by
// the caller), so the store is one unmasked dwordx3.
template <bool NT>
DEV void emit_full_a4(const uint32_t G[4], uint8_t *out)
{
    uint32_t o0, o1, o2;
    groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
    u32x3a4 *p = (u32x3a4 *) (out + 12 * lane_id());
    if (NT)
        __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, p);
    else
        *p = u32x3a4{o0, o1, o2};
}

// emit_full_a4 at out + off, off a 32-bit byte offset (a uniform base plus a
// 32-bit vector offset: no 64-bit address arithmetic per store)
template <bool NT>
DEV void emit_full_off(const uint32_t G[4], uint8_t *out, uint32_t off)
{
    uint32_t o0, o1, o2;
    groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
    u32x3a4 *p = (u32x3a4 *) (out + off);
    if (NT)
        __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, p);
    else
        *p = u32x3a4{o0, o1, o2};
}

// Fast path (b), for the stream's final chunk when it starts on a group
// boundary: if its alphabet characters form a prefix -- lanes 0..f-1 full,
// lane f a prefix of its 16, no alphabet character after that (the shape
// of every padded or unaligned stream end) -- emit them, lane f including
// the final partial group (floor(6r/8) bytes, src/base64decoder.c:71-76)
// unless `hold`.  Returns the characters consumed, or -1 if the shape does
// not apply.  Wave-uniform.
DEV int fast_prefix(const LaneChunk &lc, bool hold, uint8_t *out)
{
    const uint32_t lane = lane_id();
    const uint32_t m = lc.vmask;
    if (!__all((m & (m + 1)) == 0)) return -1;
    const uint64_t F = __ballot(m == 0xFFFFu);
    const uint64_t NZ = __ballot(m != 0);
    const uint32_t f = __popcll(F);
    if (f == 64) {
        emit_full(lc.G, out);
        return kChunk;
    }
    if (F != ((1ull << f) - 1)) return -1;
    if (f < 63 && (NZ >> (f + 1))) return -1;
    const uint32_t k = __popc(m);
    const uint32_t nbytes = 3 * (k >> 2) + (hold ? 0u : (6 * (k & 3)) >> 3);
    if (nbytes) {
        uint32_t o0, o1, o2;
        groups_to_bytes(lc.G[0], lc.G[1], lc.G[2], lc.G[3], o0, o1, o2);
        store_bytes12(out + 12 * lane, o0, o1, o2, nbytes);
    }
    return (int) (16 * f + __shfl(k, (int) f, 64));
}

// Decode workspace: b64x_decode_workspace_size() bytes, zero-filled before
// its first use; every call leaves it re-armed for the next.
//   fd      ~((range << 32) | offset) of the first chunk pass 1 could not
//           take on a fast path, combined with atomicMax over the waves that
//           hit one; 0 = none.  The scan moves it to fd_cur and zeroes it.
//   ticket  the scan's tile ticket (blocks take tiles in the order they
//           start; zero between calls)
//   counts  alphabet characters per range (pass 1, every range)
//   bases   exclusive prefix of counts (scan, dirty calls only)
//   status  per scan tile: flag (bits 63..62: 1 aggregate, 2 inclusive
//           prefix; 0 = not yet) | value, for the scan's decoupled
//           look-back; zero between calls (the scan's last tile clears it)
//   lfail   kFailWords words, kFailStride apart (one per 128-byte line):
//           ~(first failing slot) of k_decode_lines, published by each wave
//           into word (block mod kFailWords) so that failing waves do not all
//           read one line; 0 = none (cleared by k_decode_suffix_held)
//   fail_any  nonzero when any failure word was published (set by the probe
//           and by the first publisher into a word, which sees it zero;
//           cleared by k_decode_suffix_held): the idle suffix kernel's one
//           scalar load instead of a wave reading all 64 words per block
//   model   the line model k_decode_probe found, for k_decode_lines and
//           k_decode_suffix_held; model_n the length of the stream it was made for:
//           a call of the same length may reuse it without a probe
//           (decode_dev_ws), and k_decode_lines checks that it does
//   fticket, fstatus, fsuper, wdone  k_decode_suffix_held's tile ticket, tile
//           counts, group sums and count of blocks that have left
//   sfx_start  where the last call's k_decode_suffix_held<false> started (its
//           first failing slot's span), ~0 when it had nothing to do; read
//           by the tests only (clean and MIME input must never need it)
// The regions that must be zero between calls (status, fstatus, fsuper, lfail,
// wdone) sit at fixed offsets after the header, sized for the largest plan,
// so calls of different sizes on one workspace never find another call's scratch
// (counts, bases) where they expect zeros.
// The line model of k_decode_lines (see there): lines of L alphabet
// characters, each followed by s separator bytes; L = 0: no separators.
struct LineModel {
    uint32_t L, s;  // L = 0: no separators
    uint32_t P;     // L + s
    uint32_t T;     // the stream's interior slots (k_decode_lines)
    uint32_t m, k;  // i / L == (i * m) >> (31 + k) for every i < 2^31
    uint32_t rcp;   // ceil(2^20 / L): i / L == (i * rcp) >> 20 for i < 4,096
    uint32_t skip;  // 1: k_decode_probe already published slot T as failing (no tail)
};
static_assert(sizeof(LineModel) == 32, "the workspace header holds 32 bytes of model");

struct DecodeWs {
    uint64_t *lfail;     // kFailWords words, kFailStride apart
    uint64_t *fail_any;  // nonzero: some failure word was published (own line)
    uint32_t *wdone;     // k_decode_suffix_held: blocks that have left (own line; zero between calls)
    LineModel *model;    // k_decode_lines' model, for k_decode_suffix_held
    uint64_t *model_n;   // the stream length the model was probed for (0: none yet)
    uint64_t *fd;
    uint64_t *fd_cur;
    uint32_t *ticket;
    uint32_t *fticket;   // the single-pass decode's tile ticket (zero between calls)
    uint64_t *sfx_start; // where k_decode_suffix_held<false> started, ~0 = nothing to do
    uint32_t *counts;
    uint64_t *bases;
    uint64_t *status;
    uint64_t *fstatus;   // the single-pass decode's tile status words (zero between calls)
    uint64_t *fsuper;    // k_decode_suffix_held's group sums: tiles counted << 56 | sum (zero between calls)
};

constexpr uint32_t kScanTile = 1024;  // ranges per scan tile: 256 threads x 4
// k_decode_suffix_held: ranges per wave of a tile (held in VGPRs; 4 at 5
// waves per SIMD: 2, 3, 5-8 per wave and 4 or 6 waves per SIMD all measured
// slower, profiles/r05_ab_sfx_held*.jsonl)
constexpr uint32_t kHeldPer = 4;
constexpr uint32_t kHeldWaves = 5;  // waves per SIMD (96 VGPRs: two tiles held)
constexpr uint32_t kHeldTile = kHeldPer * kWavesPerBlock;
// Inputs up to kLinesMaxChars characters (8 Gi: 6 GiB of payload) take the
// probe / lines / held-suffix decode with 2,048-character ranges -- up to
// kLinesMaxRanges of them, whose tile words the workspace's fixed regions
// hold; larger ones pass 1, the scan and pass 2 (kMaxRanges longer ranges).
constexpr uint64_t kLinesMaxChars = 1ull << 33;
constexpr uint32_t kLinesMaxRanges = (uint32_t) (kLinesMaxChars / (2 * kChunk));
constexpr uint32_t kFailWords = 64, kFailStride = 16;
constexpr uint64_t kWsModelN = 64;                                        // the model's stream length
constexpr uint64_t kWsStatus = 128;                                       // scan tile status
constexpr uint64_t kWsFStatus = kWsStatus + kMaxRanges / kScanTile * 8;   // suffix tile status
constexpr uint32_t kSfxGroup = 64;  // k_decode_suffix_held: tiles per group sum
constexpr uint64_t kGroupFull = (uint64_t) kSfxGroup << 56;
constexpr uint64_t kWsFSuper = kWsFStatus + (kLinesMaxRanges / kHeldTile + 1) * 8;   // suffix group sums
constexpr uint64_t kWsFail = kWsFSuper + (kLinesMaxRanges / kHeldTile / kSfxGroup + 16) * 8;  // lines failures
// failure words, fail_any, wdone: one 128-byte line each
constexpr uint64_t kWsScratch = kWsFail + (kFailWords + 2) * kFailStride * 8;  // counts, bases

// Workspace bytes for plans of up to nr ranges: the fixed regions, then
// counts + bases (at least 64 bytes).
constexpr uint64_t ws_bytes_for(uint64_t nr)
{
    return kWsScratch + ((nr * 4 + 7) / 8 * 8 + nr * 8 > 64 ? (nr * 4 + 7) / 8 * 8 + nr * 8 : 64);
}

// Layout: 64-byte header (fd, fd_cur, ticket, fticket, sfx_start, model), the
// model's stream length (its own 64 bytes), the zero-between-calls regions at
// fixed offsets, then the scratch counts and bases of `nranges` ranges.
DEV DecodeWs ws_view(void *ws, uint32_t nranges)
{
    DecodeWs w;
    uint8_t *p = (uint8_t *) ws;
    w.fd = (uint64_t *) p;
    w.fd_cur = (uint64_t *) (p + 8);
    w.ticket = (uint32_t *) (p + 16);
    w.fticket = (uint32_t *) (p + 20);
    w.sfx_start = (uint64_t *) (p + 24);
    w.model = (LineModel *) (p + 32);
    w.model_n = (uint64_t *) (p + kWsModelN);
    w.status = (uint64_t *) (p + kWsStatus);
    w.fstatus = (uint64_t *) (p + kWsFStatus);
    w.fsuper = (uint64_t *) (p + kWsFSuper);
    w.lfail = (uint64_t *) (p + kWsFail);
    w.fail_any = w.lfail + kFailWords * kFailStride;
    w.wdone = (uint32_t *) (w.fail_any + kFailStride);
    w.counts = (uint32_t *) (p + kWsScratch);
    w.bases = (uint64_t *) (p + kWsScratch + ((uint64_t) nranges * 4 + 7) / 8 * 8);
    return w;
}

DEV uint32_t wave_sum(uint32_t x)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

DEV uint64_t wave_sum64(uint64_t x)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

template <bool NT>
DEV uint4 ld16(const uint8_t *p)
{
    if (NT) {
        u32x4a4 v = __builtin_nontemporal_load((const u32x4a4 *) p);
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return load16_a4(p);
}

constexpr uint32_t kNoDirty = 0xFFFFFFFFu;

// Alphabet characters among a lane's first `nin` characters: the table
// values packed 4 per dword, non-alphabet ones have bit 7 set.
DEV uint32_t count_valid(const uint8_t *tab, uint4 w, uint32_t nin)
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t bad = 0;
#pragma unroll
    for (uint32_t g = 0; g < 4; g++) {
        uint32_t P = tab[dw[g] & 0xFFu] | ((uint32_t) tab[(dw[g] >> 8) & 0xFFu] << 8) |
                     ((uint32_t) tab[(dw[g] >> 16) & 0xFFu] << 16) |
                     ((uint32_t) tab[dw[g] >> 24] << 24);
        const uint32_t in_g = nin > 4 * g ? nin - 4 * g : 0u;
        P |= in_g >= 4 ? 0u : ~0u << (8 * in_g);
        bad += __popc(P & 0x80808080u);
    }
    return 16u - bad;
}

// Pass 1's step for one chunk at stream position `pos` of range [rb, re):
// while the range is still clean, the fast paths (an all-alphabet chunk;
// the stream's final chunk in the prefix shape); the first chunk that fits
// neither becomes the range's dirty offset; from then on the range only
// counts.
DEV void p1_chunk(const uint8_t *tab, uint4 w, uint32_t nin, uint64_t pos, uint64_t rb,
                  uint64_t re, bool last, uint32_t hold, uint8_t *o, uint32_t &dirty,
                  uint32_t &cnt)
{
    if (dirty != kNoDirty) {
        cnt += count_valid(tab, w, nin);
        return;
    }
    uint32_t G[4], bad;
    map_fast(tab, w, nin, G, bad);
    if (__all(bad == 0)) {
        cnt += 16;
        emit_full(G, o + (pos - rb) / 4 * 3);
        return;
    }
    const bool final = last && pos + kChunk >= re;
    if (!final) {
        cnt += count_valid(tab, w, nin);
        dirty = (uint32_t) (pos - rb);
        return;
    }
    LaneChunk lc;
    map_chunk_lds(tab, w, nin, lc);
    cnt += __popc(lc.vmask);
    if (fast_prefix(lc, hold != 0, o + (pos - rb) / 4 * 3) < 0) dirty = (uint32_t) (pos - rb);
}

// Pass 1 (fast paths only), one wave per range; each range assumes every
// earlier range was all alphabet.  The hot loop takes groups of U full
// chunks while every chunk is all alphabet (no per-lane guards, scalar loop
// control; NT = non-temporal loads and stores, the policy that lets a plain
// stream reach ~6.3 TB/s on this part).  The first exception drops to a
// one-chunk loop that still emits fast-path chunks until one does not fit;
// that chunk is published (atomicMax of the complemented (range, offset))
// and the range only counts from then on.
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(7)))
void k_decode_pass1(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out,
    uint64_t R, uint32_t nranges, DecAlpha a, void *ws, uint32_t hold)
{
    __shared__ uint8_t tab[256];
    build_dec_table(tab, a);
    block_sync();
    const uint32_t lane = lane_id();
    // wave-uniform, and provably so (scalar loop control, no exec masking)
    const uint32_t r = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (r >= nranges) return;
    const uint64_t rb = (uint64_t) r * R;
    const uint64_t re = rb + R < n ? rb + R : n;
    const bool last = r + 1 == nranges;
    uint8_t *o = out + rb / 4 * 3;
    uint32_t cnt = 0;  // per lane; summed over the wave at the end
    uint32_t dirty = kNoDirty;
    uint64_t pos = rb;
    const uint64_t hot_end = re - (re - rb) % ((uint64_t) kChunk * U);
    if (((((uintptr_t) in) | ((uintptr_t) o)) & 3) == 0 && pos < hot_end) {
        uint4 cur[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            cur[u] = ld16<NT>(in + pos + (uint64_t) u * kChunk + 16 * lane);
        for (;;) {
            const uint64_t np = pos + (uint64_t) kChunk * U;
            int u = 0;
#pragma unroll
            for (; u < U; u++) {
                uint32_t G[4], bad;
                map_fast(tab, cur[u], 16, G, bad);
                if (!__all(bad == 0)) break;
                emit_full_a4<NT>(G, o + (pos + (uint64_t) u * kChunk - rb) / 4 * 3);
            }
            cnt += 16 * u;
            if (u < U) {
                const uint64_t cpos = pos + (uint64_t) u * kChunk;
                if (!(last && cpos + kChunk >= re)) {
                    // chunk u is the range's first dirty one: count it and
                    // the rest of the tile from the registers they are in
                    dirty = (uint32_t) (cpos - rb);
#pragma unroll
                    for (int v = 0; v < U; v++)
                        if (v >= u) cnt += count_valid(tab, cur[v], 16);
                    pos = np;
                } else {
                    pos = cpos;  // the stream's final chunk: prefix rule below
                }
                break;
            }
            pos = np;
            if (pos >= hot_end) break;
#pragma unroll
            for (int v = 0; v < U; v++)
                cur[v] = ld16<NT>(in + pos + (uint64_t) v * kChunk + 16 * lane);
        }
    }
    for (; pos < re; pos += 2 * (uint64_t) kChunk) {
        // two chunks' loads in flight, then each chunk in order
        uint4 w[2];
        uint32_t nin[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint64_t p = pos + (uint64_t) h * kChunk + 16 * lane;
            nin[h] = p >= re ? 0u : (re - p >= 16 ? 16u : (uint32_t) (re - p));
            w[h] = nin[h] ? load_chars(in + p, nin[h]) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int h = 0; h < 2; h++)
            if (pos + (uint64_t) h * kChunk < re)
                p1_chunk(tab, w[h], nin[h], pos + (uint64_t) h * kChunk, rb, re, last, hold, o,
                         dirty, cnt);
    }
    cnt = wave_sum(cnt);
    if (lane == 0) {
        DecodeWs v = ws_view(ws, nranges);
        v.counts[r] = cnt;
        if (dirty != kNoDirty) {
            // Only an improvement is published: on input that is dirty
            // everywhere (CRLF every 76 characters) every range would
            // otherwise hit this one word with an atomic, serialised at
            // its L2 channel.  The device-scope load sees what earlier
            // ranges published.
            const unsigned long long key = ~(((uint64_t) r << 32) | dirty);
            const unsigned long long cur = __hip_atomic_load(
                (unsigned long long *) v.fd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (key > cur) atomicMax((unsigned long long *) v.fd, key);
        }
    }
}

// The stream's last V mod 4 alphabet characters (as sextets) into
// res->tail, scanning backwards from the end; one wave.
template <bool LO = false>  // LO: a build_dec_table_lo table
DEV void find_tail_sextets(const uint8_t *tab, const uint8_t *in, uint64_t n, uint64_t V,
                           b64x_dec_result *res, b64x_dec_result *hres)
{
    const uint32_t lane = lane_id();
    int need = (int) (V & 3);
    uint8_t got[4] = {0, 0, 0, 0};
    uint64_t end = n;
    while (need > 0 && end > 0) {
        uint64_t beg = end >= 64 ? end - 64 : 0;
        uint64_t p = beg + lane;
        uint32_t t = p < end ? tab[in[p]] : 0xFFu;
        if (LO) t = t & 3u ? 0xFFu : t >> 2;
        uint64_t bm = __ballot(t < 64u);
        while (need > 0 && bm) {
            int hi = 63 - __clzll(bm);
            got[--need] = (uint8_t) __shfl(t, hi, 64);
            bm &= ~(1ull << hi);
        }
        end = beg;
    }
    if (lane == 0) {
        for (int j = 0; j < 4; j++) res->tail[j] = got[j];
        if (hres) {
            for (int j = 0; j < 4; j++) hres->tail[j] = got[j];
            hres->tail_n = (uint32_t) (V & 3);
        }
    }
}

// The result record: `res` in device memory, and, when `hres` is set, the
// same record in fine-grained host memory, written by this kernel instead
// of a D2H copy queued behind it (see b64x_session_decode_async).  The
// record names its call -- `n` characters, the hold flag and the call's
// sequence number `seq` (drawn by the host, never 0) -- so the host's check
// (b64x_result_check.h) rejects a record of an earlier call or a zeroed one
// as well as poison; it checks every field, so the order of these stores
// does not matter.
DEV void write_result(b64x_dec_result *res, b64x_dec_result *hres, uint64_t V, uint32_t hold,
                      uint64_t n, uint32_t seq)
{
    const uint64_t out_len = hold ? V / 4 * 3 : V * 6 / 8;
    res->valid = V;
    res->tail_n = (uint32_t) (V & 3);
    res->out_len = out_len;
    res->nchars = n;
    res->seq = seq;
    res->flags = hold ? 1u : 0u;
    if (hres) {
        hres->valid = V;
        hres->out_len = out_len;
        hres->nchars = n;
        hres->seq = seq;
        hres->flags = hold ? 1u : 0u;
    }
}

// Block-wide exclusive scan of one u64 per thread (256 threads); returns
// the exclusive prefix, `total` the block sum.
DEV uint64_t block_excl_scan256(uint64_t x, uint64_t *wtot, uint64_t &total)
{
    const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
    uint64_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(v, d, 64);
        if (lane >= (uint32_t) d) v += y;
    }
    if (lane == 63) wtot[wave] = v;
    block_sync();
    uint64_t before = 0;
    total = 0;
#pragma unroll
    for (uint32_t i = 0; i < kWavesPerBlock; i++) {
        if (i < wave) before += wtot[i];
        total += wtot[i];
    }
    return before + v - x;
}

constexpr uint64_t kStAgg = 1ull << 62, kStIncl = 2ull << 62;
constexpr uint64_t kStVal = (1ull << 62) - 1;

// Tile status words are written and read with relaxed device-scope atomics
// (one 64-bit word carries flag and value, so no fence orders a value
// against its flag: a release here would write back the whole L2).
DEV void st_store(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

DEV uint64_t st_load(uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Scan, device-wide (it replaced a one-block scan: 2.3 ms dirty), one block per
// tile of 1024 ranges.  Clean call (no first-dirty record): block 0 alone
// computes V from the last range's count and the result record; every
// other block returns at once.  Dirty call: a single-pass scan of
// counts[r0 ..] with decoupled look-back.  Blocks take tiles from a ticket
// in the order they start, so a tile's predecessors are always running or
// done and the look-back cannot wait on a block that is not yet dispatched,
// whatever else shares the GPU (6 us more on 1 GiB than tiles by block
// index, which relies on in-order dispatch across the XCDs).  Each tile publishes its aggregate, looks back over its
// predecessors 64 at a time (one wave) until an inclusive prefix,
// publishes its own and writes the bases of its ranges.  The last tile
// writes the result record and the tail sextets, waits until every tile
// has published its inclusive prefix (so no look-back is still reading)
// and every block has its ticket, then clears the status words and the
// ticket and re-arms the workspace (fd -> fd_cur).
__global__ __launch_bounds__(kThreads) void k_decode_scan2(
    const uint8_t *__restrict__ in, uint64_t n, uint64_t R, uint32_t nranges,
    DecAlpha a, void *ws, b64x_dec_result *res, b64x_dec_result *hres, uint32_t hold,
    uint32_t seq)
{
    __shared__ uint8_t tab[256];
    __shared__ uint64_t wtot[kWavesPerBlock];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_tile;
    DecodeWs w = ws_view(ws, nranges);
    const uint64_t packed = *(volatile uint64_t *) w.fd;
    if (packed == 0) {
        if (blockIdx.x != 0) return;
        build_dec_table(tab, a);
        block_sync();
        const uint64_t V = (uint64_t) (nranges - 1) * R + w.counts[nranges - 1];
        if (threadIdx.x == 0) {
            *w.fd_cur = 0;
            write_result(res, hres, V, hold, n, seq);
        }
        if (threadIdx.x < 64) find_tail_sextets(tab, in, n, V, res, hres);
        return;
    }
    const uint32_t r0 = (uint32_t) (~packed >> 32);
    const uint32_t ntiles = (nranges - r0 + kScanTile - 1) / kScanTile;
    if (threadIdx.x == 0) s_tile = atomicAdd(w.ticket, 1u);
    block_sync();
    const uint32_t t = s_tile;
    if (t >= ntiles) return;
    build_dec_table(tab, a);
    const uint32_t base = r0 + t * kScanTile + 4 * threadIdx.x;
    uint32_t c[4];
    uint64_t mine = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        c[j] = base + j < nranges ? w.counts[base + j] : 0u;
        mine += c[j];
    }
    uint64_t agg;
    const uint64_t ex = block_excl_scan256(mine, wtot, agg);
    const uint32_t lane = lane_id();
    if (threadIdx.x < 64) {
        uint64_t excl = (uint64_t) r0 * R;
        if (t > 0) {
            if (lane == 0) st_store(&w.status[t], kStAgg | agg);
            excl = 0;
            int64_t p = (int64_t) t - 1;
            for (;;) {
                const int64_t q = p - lane;
                const uint64_t v = q >= 0 ? st_load(&w.status[q]) : kStIncl;  // before tile 0: 0
                const uint32_t f = (uint32_t) (v >> 62);
                const uint64_t inc = __ballot(f == 2);
                const uint32_t k = inc ? (uint32_t) __ffsll((unsigned long long) inc) - 1 : 63u;
                if (!__all(lane > k || f != 0)) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                uint64_t part = lane <= k ? (v & kStVal) : 0;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) part += __shfl_xor(part, d, 64);
                excl += part;
                if (inc) break;
                p -= 64;
            }
        }
        if (lane == 0) {
            st_store(&w.status[t], kStIncl | (excl + agg));
            s_excl = excl;
        }
    }
    block_sync();
    uint64_t run = s_excl + ex;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (base + j < nranges) w.bases[base + j] = run;
        run += c[j];
    }
    if (t == ntiles - 1 && threadIdx.x < 64) {
        const uint64_t V = s_excl + agg;
        if (lane == 0) write_result(res, hres, V, hold, n, seq);
        find_tail_sextets(tab, in, n, V, res, hres);
        for (;;) {  // every tile inclusive -> every look-back is over
            bool all = true;
            for (uint32_t i = lane; i < ntiles; i += 64)
                all = all && (st_load(&w.status[i]) >> 62) == 2;
            if (__all(all)) break;
            __builtin_amdgcn_s_sleep(1);
        }
        for (uint32_t i = lane; i < ntiles; i += 64) st_store(&w.status[i], 0);
        if (lane == 0) {
            // every block has its ticket -> re-arm the counter
            while (__hip_atomic_load(w.ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                   gridDim.x)
                __builtin_amdgcn_s_sleep(1);
            __hip_atomic_store(w.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *w.fd_cur = packed;
            *w.fd = 0;
        }
    }
}

// ---- pass 2: shared pieces ----------------------------------------------
//
// Ranges of kP2Range characters; pass 2 issues all of a range's loads at
// once (its base, both chunks, 64 lookahead bytes) and, for the middle
// ranges, the next range's before processing this one.
constexpr uint32_t kP2Range = 2048;

// A wave-uniform 64-bit load through the scalar cache (s_load, counted by
// lgkmcnt): a vector load of a per-range base that is then made scalar
// forces an s_waitcnt vmcnt that also drains every store the wave issued
// before it, once per range.  Only for data written by an earlier kernel.
DEV uint64_t scalar_load_u64(const uint64_t *p)
{
    return *(const __attribute__((address_space(4))) uint64_t *) p;
}

DEV void lane_values(const uint8_t *tab, uint4 w, uint32_t nin, uint32_t P[4])
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (uint32_t g = 0; g < 4; g++) {
        const uint32_t t0 = tab[dw[g] & 0xFFu];
        const uint32_t t1 = tab[(dw[g] >> 8) & 0xFFu];
        const uint32_t t2 = tab[(dw[g] >> 16) & 0xFFu];
        const uint32_t t3 = tab[dw[g] >> 24];
        // two byte pairs and an OR (written as shifts, the compiler made it
        // three shifts and a three-way OR)
        P[g] = __builtin_amdgcn_perm(t1, t0, 0x0C0C0400u) | __builtin_amdgcn_perm(t3, t2, 0x04000C0Cu);
    }
    if (nin < 16) {
#pragma unroll
        for (uint32_t g = 0; g < 4; g++) {
            const uint32_t in_g = nin > 4 * g ? nin - 4 * g : 0u;
            P[g] |= in_g >= 4 ? 0u : ~0u << (8 * in_g);
        }
    }
}


// One wave copies 64 x 16 bytes from gsrc (per lane) to LDS at lds_dst +
// 16 x lane, straight into LDS (global_load_lds_dwordx4: no VGPR holds the
// data).  Issued as inline asm so that the compiler does not track the copy:
// it cannot tell the copy's destination from the decode's other LDS traffic
// (the window's atomic ORs go through a pointer) and waited for every copy
// in flight (vmcnt(0)) at the first of them, right after the copy was
// issued.  The reader waits itself (vm_wait_all) before it reads the copy.
// The source is a wave-uniform base (SGPRs) plus 16 x lane: with a per-lane
// 64-bit address the compiler hoisted `in + 16 lane` out of the tile loop
// and spilled it, and its reload before each copy waited (vmcnt(0)) for the
// stores of the tile before.
DEV void lds_dma16(const uint8_t *gbase, void *lds_dst)
{
    const uint32_t l = (uint32_t) (uintptr_t) (__attribute__((address_space(3))) void *) lds_dst;
    const uint32_t voff = 16u * lane_id();
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(gbase), "s"(l) : "memory");
}

DEV void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// ---- pass 2, bit-stream form ----------------------------------------------
//
// The range's output is built in LDS directly as the decoded BIT stream (a
// per-character scatter of sextets into LDS, read back and converted group
// by group, cost ~520 VALU per range -- round 1's pass 2c): each lane compacts every dword of its table
// values (v_perm, selector by the dword's invalid mask), turns the 0-4
// surviving sextets into one left-aligned 24-bit field (two v_dot4), and
// ORs that field into the wave's zeroed LDS buffer at bit 6 x (its sextet
// index) -- the bytes of that buffer ARE the output bytes.  The buffer is
// laid out so that LDS byte 4 + (ob & 3) is output byte ob: its dwords map
// onto aligned output dwords, and the store is a straight copy with byte
// stores only for the first and last partial dwords.
// head, skew (decode_range aligns its window to 16 output bytes), out, slack
constexpr uint32_t kP2dBytes = 16 + 15 + kP2Range / 4 * 3 + 16;
constexpr uint32_t kP2dBlocks = (kP2dBytes + 15) / 16;                  // uint4 per wave

struct __attribute__((aligned(16))) P2dSmem {
    uint8_t tab[256];
    uint32_t sel[16];
    uint4 bits[kWavesPerBlock][kP2dBlocks];
};

// sel[m]: the v_perm selector that packs a dword's bytes whose bit j of m
// is clear (the alphabet ones) into its low bytes, zeros above.
// KEEP_SET: indexed by the alphabet bytes' mask instead (bit j set: keep).
template <bool KEEP_SET = false>
DEV void build_compact_sel(uint32_t *sel)
{
    if (threadIdx.x < 16) {
        uint32_t v = 0x0C0C0C0Cu, k = 0;
        for (uint32_t j = 0; j < 4; j++)
            if (((threadIdx.x >> j) & 1u) == (KEEP_SET ? 1u : 0u)) {
                v = (v & ~(0xFFu << (8 * k))) | (j << (8 * k));
                k++;
            }
        sel[threadIdx.x] = v;
    }
}

DEV uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x00010203u); }

// OR a field left-aligned in G (bits 31..32-w; the rest zero) into the
// big-endian bit stream held in `bits` (dwords), its first bit at stream
// bit p.  BE: the dwords hold the stream big-endian (the reader swaps each
// dword once when it stores: decode_range's 16-byte blocks), else
// little-endian per byte, the output bytes as they are (decode_buf_bits).
// The two dwords are G >> o and the bits shifted out of it (v_lshrrev,
// v_alignbit: both take the shift's low 5 bits, so p goes in as it is), the
// dword index one v_bfe (round 5: a 64-bit shift of a zero-extended 24-bit
// field by 40 - o, and a shift, mask and add for the address).
template <bool BE = false>
DEV void or_field(uint32_t *bits, uint32_t p, uint32_t G)
{
    const uint32_t o = p & 31u;
    const uint32_t hi = G >> o, lo = __builtin_amdgcn_alignbit(G, 0u, o);
    uint32_t *q = bits + __builtin_amdgcn_ubfe(p, 5, 27);
    __hip_atomic_fetch_or(q, BE ? hi : bswap32(hi), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    __hip_atomic_fetch_or(q + 1, BE ? lo : bswap32(lo), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// Sextets in bytes 0..3 of D (stream order; absent ones zero; LO: as 4 s)
// -> the group s0 s1 s2 s3 left-aligned in 32 bits (bits 31..8).
template <bool LO = false>
DEV uint32_t group_dot(uint32_t D)
{
    const uint32_t x = __builtin_amdgcn_udot4(D, 0x00000140u, 0u, false);  // s0*64 + s1
    const uint32_t y = __builtin_amdgcn_udot4(D, 0x01400000u, 0u, false);  // s2*64 + s3
    return LO ? (x << 18) | (y << 6) : (x << 20) | (y << 8);
}

// Copy LDS bytes [lo, hi) of `b` (a wave's buffer) to dst0 + [lo, hi),
// where dst0 = the output address of LDS byte 0 (dword aligned; bytes
// below lo are never written).
DEV void store_bits(const uint32_t *b, uint32_t lo, uint32_t hi, uint8_t *dst0)
{
    const uint32_t lane = lane_id();
    const uint32_t klo = (lo + 3) >> 2, khi = hi >> 2;  // whole dwords [klo, khi)
    if (klo < khi) {
        for (uint32_t k0 = klo + 4 * lane; k0 < khi; k0 += 256) {
            const uint32_t d0 = b[k0], d1 = b[k0 + 1], d2 = b[k0 + 2], d3 = b[k0 + 3];
            uint32_t *q = (uint32_t *) (dst0 + 4 * (uint64_t) k0);
            if (k0 + 4 <= khi) {
                *(u32x4a4 *) q = u32x4a4{d0, d1, d2, d3};
            } else {
                q[0] = d0;
                if (k0 + 1 < khi) q[1] = d1;
                if (k0 + 2 < khi) q[2] = d2;
            }
        }
    }
    // partial dwords: the head bytes [lo, 4 klo) by lane 0, the tail bytes
    // [4 khi, hi) by lane 1 (when the range lies inside one dword, lane 0)
    const uint8_t *bb = (const uint8_t *) b;
    uint32_t from = 0, to = 0;
    if (lane == 0) {
        from = lo;
        to = 4 * klo < hi ? 4 * klo : hi;
    } else if (lane == 1 && klo <= khi) {
        from = 4 * khi > lo ? 4 * khi : lo;
        to = hi;
    }
#pragma unroll
    for (uint32_t i = 0; i < 3; i++)  // at most 3 bytes each
        if (from + i < to) dst0[from + i] = bb[from + i];
}

// Copy stream bytes [lo, hi) of a wave's big-endian window `b` (or_field<true>)
// to dst0 + [lo, hi), where
// dst0 = the output address of LDS byte 0, 16-byte aligned: the whole
// 16-byte blocks as aligned ds_read_b128 / dwordx4 non-temporal pairs (lane
// k takes block klo + k, conflict-free), the head and tail bytes of the
// partial blocks (at most 15 each) as one byte store of up to 30 lanes.
DEV void store_bits16(const uint4 *b, uint32_t lo, uint32_t hi, uint8_t *dst0)
{
    const uint32_t lane = lane_id();
    const uint32_t klo = (lo + 15) >> 4, khi = hi >> 4;  // whole blocks [klo, khi)
    for (uint32_t k = klo + lane; k < khi; k += 64) {
        const uint4 v = b[k];  // big-endian dwords (or_field<true>)
        __builtin_nontemporal_store(u32x4a16{bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w)},
                                    (u32x4a16 *) (dst0 + 16 * (uint64_t) k));
    }
    const uint32_t hend = 16 * klo < hi ? 16 * klo : hi;  // head bytes [lo, hend)
    uint32_t i = 0;
    bool act = false;
    if (lane < 16) {
        i = lo + lane;
        act = i < hend;
    } else if (lane < 32) {
        i = 16 * khi + (lane - 16);  // tail bytes [max(16 khi, hend), hi)
        act = i < hi && i >= hend;
    }
    if (act) dst0[i] = ((const uint8_t *) b)[i ^ 3u];
}

// Inclusive prefix sum over the wave with DPP (row shifts, then the two
// row broadcasts of gfx9): six full-rate adds instead of a ballot per bit
// plane; x may pack independent 16-bit counts.
DEV uint32_t wave_incl_scan_dpp(uint32_t x)
{
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// One 2,048-character step of the bit-stream decode: lanes' chunks c[h]
// (nin[h] characters each) are looked up, compacted per dword, and their
// sextet fields OR-ed into `bits` from window bit `bit0` on (bit0 may sit
// up to 18 bits past the window's byte 4: skipped sextets land in its
// head).  Returns the step's alphabet characters.
template <bool BE = false, class SM = P2dSmem, bool LO = false>  // LO: build_dec_table_lo
DEV uint32_t bits_step(const SM &sm, uint32_t *bits, const uint4 c[2],
                       const uint32_t nin[2], int bit0)
{
    // per dword: table values, the v_perm compaction selector (by the
    // invalid-byte pattern, via v_dot4 of the bit-7s) and 6 x the count of
    // non-alphabet bytes; the scan runs over the lanes' BIT counts (both
    // chunks packed in one DPP scan), so positions need no multiply
    // acc[h][g]: -6 x the non-alphabet bytes of chunk h before group g, a
    // running signed v_dot4 (group g's field sits 24 g + acc[h][g] bits into
    // the lane's share of the chunk).  LO: the alphabet bytes' flags (one
    // v_bitop3 of the table values), the selectors indexed by them
    // (build_compact_sel<true>), and acc[h][g] the bits before group g, a
    // running unsigned v_dot4 (its own destination: the signed one
    // accumulates in place, a v_mov per group to keep each sum)
    uint32_t P[2][4], sel[2][4], cnt = 0;
    uint32_t acc[2][5];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        lane_values(sm.tab, c[h], nin[h], P[h]);
        acc[h][0] = 0;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t iv = LO ? ~P[h][g] & 0x01010101u : (P[h][g] >> 7) & 0x01010101u;
            const uint32_t off = __builtin_amdgcn_udot4(iv, 0x20100804u, 0u, false);
            sel[h][g] = *(const uint32_t *) ((const uint8_t *) sm.sel + off);
            acc[h][g + 1] = LO ? __builtin_amdgcn_udot4(iv, 0x06060606u, acc[h][g], false)
                               : (uint32_t) __builtin_amdgcn_sdot4((int) iv, (int) 0xFAFAFAFAu,
                                                                  (int) acc[h][g], false);
        }
        cnt |= (LO ? acc[h][4] : 96u + acc[h][4]) << (16 * h);  // the lane's output bits in chunk h (<= 96)
    }
    const uint32_t incl = wave_incl_scan_dpp(cnt);  // halves <= 6,144
    const uint32_t ex = incl - cnt;
    const uint32_t tot = (uint32_t) __builtin_amdgcn_readlane((int) incl, 63);
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint32_t before = h ? tot & 0xFFFFu : 0u;
        const uint32_t p = (uint32_t) bit0 + before + ((ex >> (16 * h)) & 0xFFFFu);
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t D = __builtin_amdgcn_perm(0u, P[h][g], sel[h][g]);
            // absent sextets are zero bytes
            or_field<BE>(bits, p + (LO ? 0u : 24u * g) + acc[h][g], group_dot<LO>(D));
        }
    }
    return ((tot & 0xFFFFu) + (tot >> 16)) / 6u;  // alphabet characters (scalar)
}

// ---- line-structured single-pass decode ------------------------------------
//
// MIME-formatted base64 (RFC 2045: 76-character lines and CRLF; PEM: 64 and
// LF) is clean text with separators at fixed positions.  Under a model of
// the stream -- lines of L alphabet characters, each followed by s bytes
// outside the alphabet, from position 0 on; L = 0 for no separators (clean
// input) -- sextet i sits at position pos(i) = (i / L)(L + s) + i % L, so
// every character's output place is known in closed form and no scan is
// needed.  k_decode_lines is output-indexed: lane slot t owns sextets
// [16t, 16t + 16), i.e. output bytes [12t, 12t + 12), and its span of input
// [pos(16t), pos(16t + 16)) -- 16 characters plus, when a line ends inside
// the slot, that line's s separator bytes.  It loads the span (one
// dword-aligned 24-byte window), drops the separator with two funnel shifts
// and a byte select, checks that the 16 characters are alphabet and the
// separator bytes are not, and stores 12 bytes.  Slots whose spans lie in
// the input ("interior", t < T) partition [0, pos(16T)), so when all pass,
// that prefix holds exactly 16T alphabet characters in model order and the
// stored bytes are the reference's; the < 16 + s bytes left after it are
// decoded exactly by the one wave that owns slot T, which also writes the
// result record.  The first failing slot t_f (any other structure, junk,
// '=' inside the stream) is published; everything before pos(16 t_f) is
// final, and k_decode_suffix_held<false> decodes [pos(16 t_f), n) exactly.  The
// model is probed from the first 256 bytes by one wave per block; the
// decode never depends on it being right, only its speed does.
//
// Reference: the per-character loop of decoder_read(), src/base64decoder.c:
// 52-80 (skip non-alphabet bytes, 8 bits out per 4 characters' 24).
// slots per lane (2: +1-3 %, 8: +7 %; with one ballot per wave, round 5: 2 +1 %,
// 6 +4 % clean, profiles/r05_ab_lines_u.jsonl)
constexpr uint32_t kLinesU = 4;
constexpr uint32_t kLinesSlots = 64 * kLinesU;      // per wave
constexpr uint32_t kLinesMaxL = 252, kLinesMaxS = 4;

DEV uint64_t line_pos(const LineModel &m, uint64_t i)  // position of sextet i
{
    if (m.L == 0) return i;
    return i / m.L * m.P + i % m.L;
}

DEV uint32_t line_div(const LineModel &m, uint32_t i)  // i / L, i < 2^31
{
    return (uint32_t) (((uint64_t) i * m.m) >> (31 + m.k));
}

// One wave: the model from the first 256 bytes -- L = the first byte
// outside the alphabet, s = the run of such bytes after it.  Anything that
// does not look like lines (L < 16 or > kLinesMaxL, s > kLinesMaxS, no
// alphabet after the first run) gives the clean model.
DEV LineModel probe_lines(const uint8_t *tab, const uint8_t *in, uint64_t n,
                          uint32_t *first_junk = nullptr)
{
    const uint32_t lane = lane_id();
    const uint32_t p = 4 * lane;
    uint32_t alpha = 0, pres = 0;
    // the lane's 4 bytes with their loads issued together (a guarded load and
    // lookup per byte compiled to four dependent memory round trips, most of
    // the probe kernel's 4-5 us)
    uint32_t c[4];
    if (p + 4 <= n) {
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) c[j] = in[p + j];
    } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) c[j] = p + j < n ? in[p + j] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const bool here = p + j < n;
        pres |= (here ? 1u : 0u) << j;
        alpha |= (here && tab[c[j]] < 64u ? 1u : 0u) << j;
    }
    LineModel m{};
    const uint32_t junk = pres & ~alpha;
    const uint64_t bj = __ballot(junk != 0);
    if (!bj) return m;
    const uint32_t lj = (uint32_t) __ffsll((unsigned long long) bj) - 1;
    const uint32_t L = 4 * lj + (uint32_t) __builtin_ctz(
                                    (uint32_t) __builtin_amdgcn_readlane((int) junk, (int) lj));
    if (first_junk) *first_junk = L;
    // the first alphabet byte after L
    const uint32_t gt = p > L ? 0xFu : (p + 4 <= L + 1 ? 0u : (0xFu << (L + 1 - p)) & 0xFu);
    const uint32_t am = alpha & gt;
    const uint64_t ba = __ballot(am != 0);
    if (!ba) return m;
    const uint32_t la = (uint32_t) __ffsll((unsigned long long) ba) - 1;
    const uint32_t P = 4 * la + (uint32_t) __builtin_ctz(
                                    (uint32_t) __builtin_amdgcn_readlane((int) am, (int) la));
    const uint32_t s = P - L;
    if (L < 16 || L > kLinesMaxL || s > kLinesMaxS) return m;
    // the whole window must follow the model (unstructured junk whose first
    // byte happens to look like a line end does not)
    uint32_t expect = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if ((p + j) % P < L) expect |= 1u << j;
    if (__ballot((expect & pres) != alpha)) return m;
    m.L = L;
    m.s = s;
    return m;
}

// 16 bytes from a dword-aligned p; bytes at or past `end` are unspecified
// (never faulting: a partial window is read bytewise).
DEV uint4 load_win16(const uint8_t *p, const uint8_t *end)
{
    const int64_t left = end - p;
    if (left >= 16) return load16_a4(p);
    if (left <= 0) return make_uint4(0, 0, 0, 0);
    return load_chars(p, (uint32_t) left);
}

DEV uint2 load_win8(const uint8_t *p, const uint8_t *end)
{
    const int64_t left = end - p;
    if (left >= 8) {
        const u32x2a4 v = *(const u32x2a4 *) p;
        return make_uint2(v.x, v.y);
    }
    uint32_t w[2] = {0, 0};
    for (int64_t i = 0; i < left; i++) w[i >> 2] |= (uint32_t) p[i] << (8 * (i & 3));
    return make_uint2(w[0], w[1]);
}

// byte-select: bytes of x where mask has 0xFF, else bytes of y
DEV uint32_t bsel(uint32_t mask, uint32_t x, uint32_t y) { return (x & mask) | (y & ~mask); }

// The 16 characters of a slot whose span starts at window byte o of w[0..5]
// (24 bytes from a dword boundary), c of them before a line end followed by
// s separator bytes (c = 16 when no line ends inside or right after the
// slot); *sep receives the separator bytes (low s bytes).
DEV uint4 slot_chars(const uint32_t w[6], uint32_t o, uint32_t c, uint32_t s, uint32_t *sep)
{
    uint32_t A[6];
#pragma unroll
    for (int j = 0; j < 5; j++) A[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], o);
    A[5] = __builtin_amdgcn_alignbyte(0u, w[5], o);
    uint32_t D[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        // the bytes after the separator: A shifted by s (1..4, wave-uniform)
        const uint32_t Bj = s >= 4 ? A[j + 1] : __builtin_amdgcn_alignbyte(A[j + 1], A[j], s);
        const int keep = (int) c - 4 * j;  // bytes of dword j before the line end
        const uint32_t mask = keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
        D[j] = bsel(mask, A[j], Bj);
    }
    // separator bytes at A[c .. c + s)
    const uint32_t q = c >> 2, r = c & 3u;
    // A[q] and A[q + 1], q = 0..4, as levels of selects on q's bits
    const bool b0 = q & 1u, b1 = q & 2u, b2 = q & 4u;
    const uint32_t a01 = b0 ? A[1] : A[0], a23 = b0 ? A[3] : A[2], a45 = b0 ? A[5] : A[4];
    const uint32_t a12 = b0 ? A[2] : A[1], a34 = b0 ? A[4] : A[3];
    const uint32_t lo = b2 ? a45 : b1 ? a23 : a01;
    const uint32_t hi = b2 ? A[5] : b1 ? a34 : a12;
    *sep = __builtin_amdgcn_alignbyte(hi, lo, r);
    return make_uint4(D[0], D[1], D[2], D[3]);
}

// slot_chars for L % 4 == 0 (RFC 2045's 76, PEM's 64): a line end can only
// fall on a dword boundary of the 16 characters (c = 4 c4), so the merge is
// a dword select and the separator the c4-th funnel-shifted dword.
DEV uint4 slot_chars4(const uint32_t w[6], uint32_t o, uint32_t c4, uint32_t s, uint32_t *sep)
{
    uint32_t A[5];
#pragma unroll
    for (int j = 0; j < 5; j++) A[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], o);
    uint32_t D[4];
    D[0] = A[0];  // c4 >= 1
#pragma unroll
    for (int j = 1; j < 4; j++) {
        const uint32_t Bj = s >= 4 ? A[j + 1] : __builtin_amdgcn_alignbyte(A[j + 1], A[j], s);
        D[j] = (uint32_t) j < c4 ? A[j] : Bj;
    }
    // A[c4], c4 = 1..4, as two levels of selects (an equality chain here
    // compiled to exec-mask branches per slot)
    const uint32_t x = c4 - 1;
    const uint32_t lo = (x & 1u) ? A[2] : A[1];
    const uint32_t hi = (x & 1u) ? A[4] : A[3];
    *sep = (x & 2u) ? hi : lo;
    return make_uint4(D[0], D[1], D[2], D[3]);
}

// Bit 8k set when byte k of `sep` is outside the alphabet (table value
// 0xFF), for all four bytes: four lookups, no wait between them.
DEV uint32_t sep_nonalpha(const uint8_t *tab, uint32_t sep)
{
    const uint32_t v = (uint32_t) tab[sep & 0xFFu] | ((uint32_t) tab[(sep >> 8) & 0xFFu] << 8) |
                       ((uint32_t) tab[(sep >> 16) & 0xFFu] << 16) | ((uint32_t) tab[sep >> 24] << 24);
    return (v >> 7) & 0x01010101u;
}

// The sep_nonalpha bits of the first n (0..4) separator bytes.
DEV uint32_t sep_need(uint32_t n)
{
    return n >= 4 ? 0x01010101u : 0x01010101u & ((1u << (8 * n)) - 1u);
}

// The table values of x's four bytes, packed (byte k: the value of byte k),
// with two v_perm pairs and one merge instead of three shifts and ors.
DEV uint32_t tab_pack4(const uint8_t *tab, uint32_t x)
{
    const uint32_t t0 = tab[x & 0xFFu], t1 = tab[(x >> 8) & 0xFFu];
    const uint32_t t2 = tab[(x >> 16) & 0xFFu], t3 = tab[x >> 24];
    const uint32_t lo = __builtin_amdgcn_perm(t1, t0, 0x0c0c0400u);  // t0 t1 0 0
    const uint32_t hi = __builtin_amdgcn_perm(t3, t2, 0x0c0c0400u);  // t2 t3 0 0
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);                // t0 t1 t2 t3
}

// The model, the stream's interior slot count T and the division constants
// into the workspace, for k_decode_lines (every block reads them with one
// scalar load instead of probing -- 175 K probes of the same 256 bytes cost
// 7 % of a 1 GiB decode -- and of computing T and L's reciprocals: hundreds
// of scalar instructions per wave) and k_decode_suffix_held.  n <= 2^33 (the
// launcher's bound, kLinesMaxChars): positions are 64-bit, slot indices
// (< 2^29) 32-bit; the division constants m, k serve sextet indices below
// 2^31, and k_decode_lines divides larger ones in 64 bits.
//
// Wave 0 probes the model from the first 256 bytes.  Every thread also
// checks 64 bytes sampled further in (half of them over the stream's first
// sixteenth, half over all of it, spaced quadratically), against the model: where a sample breaks it, every slot
// from there on is left to k_decode_suffix_held (T is cut there), so that junk
// the first window did not show -- sparse junk, one character in a thousand
// -- is not decoded twice, once by k_decode_lines until its slots fail and
// again by k_decode_suffix_held from the first failure.  Where T falls never
// matters for the result (k_decode_lines takes slots [0, T) exactly or
// publishes their failure; k_decode_suffix_held takes the rest), only for speed.
constexpr uint32_t kProbeThreads = 256;

// What the probe of the last call on a (workspace, input, length) saw, for
// the next call on the same three (pinned host memory the probe writes, the
// host reads without a sync: a stale or torn hint only picks the slower
// path).  junky: the probe cut the line model within the stream's first
// sixteenth, so k_decode_lines would take almost nothing and the single
// pass (k_decode_suffix_held<true>) is the faster exact decode.
struct DecodeHint {
    uint32_t key, junky;
};
constexpr uint32_t kDecodeHints = 64;
constexpr uint64_t kProbeSampleMin = 1u << 18;  // shorter streams: the first window only
constexpr uint32_t kProbeNS = 256;              // sampling threads
constexpr uint64_t kProbeTailKeep = 4096;       // samples avoid the stream's end (padding, a short last line)

struct ProbeSmem {
    uint8_t tab[256];
    LineModel m;
    unsigned long long first;
};

// The probe, run by one block of kProbeThreads threads (all of them call
// it).  publish: also publish a cut model's slot T as failing (lfail,
// fail_any) for the k_decode_lines and k_decode_suffix_held<false> launches
// that follow it.  The hinted single pass runs it itself, in the first
// block that finds no tile left, with publish 0: it then only renews the
// hint and the model for the next call, and a call that reuses that model
// has k_decode_lines publish the cut itself.
DEV void probe_stream(ProbeSmem &ps, const uint8_t *__restrict__ in, uint64_t n, DecAlpha a,
                      void *ws, uint32_t nranges, DecodeHint *hint, uint32_t key, uint32_t publish)
{
    uint8_t *const tab = ps.tab;
    LineModel &s_m = ps.m;
    unsigned long long &s_first = ps.first;
    // the samples' loads are issued first: they overlap the table build and
    // the window probe
    const bool sample = n >= kProbeSampleMin && threadIdx.x < kProbeNS;
    uint32_t sw[16];
    uint64_t q = 0;
    if (sample) {
        // half the samples over the first 1/16 of the stream, half over all
        // of it, each half at quadratically growing distances
        const uint64_t W = n - kProbeTailKeep - 64 - 256;
        const uint64_t span = threadIdx.x < kProbeNS / 2 ? W / 16 : W;
        const uint64_t i = threadIdx.x % (kProbeNS / 2) + 1;
        const uint64_t raw = 256 + span * i * i / ((uint64_t) kProbeNS * kProbeNS / 4);
        const uint8_t *pa = (const uint8_t *) ((uintptr_t) (in + raw) & ~(uintptr_t) 15);
        q = (uint64_t) (pa - in);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint4 x = *(const uint4 *) (pa + 16 * k);
            sw[4 * k] = x.x;
            sw[4 * k + 1] = x.y;
            sw[4 * k + 2] = x.z;
            sw[4 * k + 3] = x.w;
        }
    }
    build_dec_table(tab, a);
    if (threadIdx.x == 0) s_first = ~0ull;
    block_sync();
    if (threadIdx.x < 64) {
        uint32_t pj = 0xFFFFFFFFu;
        LineModel m = probe_lines(tab, in, n, &pj);
        if (threadIdx.x == 0) {
            if (m.L == 0 && pj != 0xFFFFFFFFu) {
                // junk in the window that no line model explains (unstructured
                // junk, a short first line): under the clean model the slot
                // holding it fails, so k_decode_lines takes only the slots
                // before it, and k_decode_suffix_held everything from there
                m.T = pj / 16;
                m.skip = 1;
            } else if (m.L == 0) {
                m.T = (uint32_t) (n / 16);
            } else {
                m.P = m.L + m.s;
                // T: the slots whose spans lie wholly inside the input -- those
                // whose 16 characters are model positions below n, less the
                // last one if a line ends right after it and its separator is
                // cut off
                const uint64_t F = n / m.P * m.L + (n % m.P < m.L ? n % m.P : m.L);
                m.T = (uint32_t) (F / 16);
                const uint64_t i = 16ull * m.T;
                if (m.T && i % m.L == 0 && i / m.L * m.P > n) m.T--;
                m.k = 32 - __builtin_clz(m.L - 1);  // ceil(log2 L)
                m.m = (uint32_t) ((((uint64_t) 1 << (31 + m.k)) + m.L - 1) / m.L);
                m.rcp = ((1u << 20) + m.L - 1) / m.L;
            }
            s_m = m;
        }
    }
    block_sync();
    const LineModel m = s_m;
    if (sample && !m.skip) {
        // the first sampled byte the model gets wrong: outside the alphabet
        // where a line character belongs, or inside it where a separator does
        uint32_t r = m.L ? (uint32_t) (q % m.P) : 0u;
        uint64_t first = ~0ull;
#pragma unroll
        for (uint32_t j = 0; j < 64; j++) {
            const bool al = tab[(sw[j >> 2] >> (8 * (j & 3))) & 0xFFu] < 64u;
            const bool want = m.L == 0 || r < m.L;
            if (al != want && first == ~0ull) first = q + j;
            if (m.L && ++r == m.P) r = 0;
        }
        if (first != ~0ull) atomicMin(&s_first, (unsigned long long) first);
    }
    block_sync();
    if (threadIdx.x != 0) return;
    LineModel mo = m;
    const uint64_t pf = s_first;
    if (!mo.skip && pf != ~0ull) {
        // the slot holding model position F(pf): every slot from there on is
        // k_decode_suffix_held's
        const uint64_t F = mo.L ? pf / mo.P * mo.L + (pf % mo.P < mo.L ? pf % mo.P : mo.L) : pf;
        if (F / 16 < mo.T) {
            mo.T = (uint32_t) (F / 16);
            mo.skip = 1;
        }
    }
    if (mo.skip && publish) {
        *ws_view(ws, nranges).lfail = ~(uint64_t) mo.T;
        *ws_view(ws, nranges).fail_any = 1;
    }
    *ws_view(ws, nranges).model = mo;
    *ws_view(ws, nranges).model_n = n;
    if (hint) {
        volatile DecodeHint *h = hint;
        h->junky = mo.skip && 256 * (uint64_t) mo.T < n ? 1u : 0u;  // 16 T < n / 16
        h->key = key;
    }
}

__global__ void __launch_bounds__(kProbeThreads) k_decode_probe(const uint8_t *__restrict__ in, uint64_t n,
                                                                DecAlpha a, void *ws, uint32_t nranges,
                                                                DecodeHint *hint, uint32_t key)
{
    __shared__ ProbeSmem ps;
    probe_stream(ps, in, n, a, ws, nranges, hint, key, 1u);
}

// At least 6 waves per SIMD (80 VGPRs): unconstrained, the rarely taken
// generic and tail paths pushed the kernel to 81 VGPRs and 5 waves, which
// cost the clean path 5 us per 1 GiB; 8 waves (64 VGPRs) spill.  256-lane
// blocks with one block-wide table (per-wave tables without the barrier:
// neutral, profiles/r03_ab_probe_wtab.jsonl).
constexpr uint32_t kLinesTH = 256, kLinesWaves = kLinesTH / 64;

// The wave's first failing slot from each lane's failed-slot bits (bit u:
// slot u): one ballot on the hot paths, the per-slot ones only when
// something failed (a ballot and a scalar branch per slot: clean 1 GiB
// 412.9 -> 408.6 us, CRLF-76 447.3 -> 445.0 with the separator check made
// branch-free, profiles/r05_ab_lines_defer.jsonl).
DEV void lines_first_fail(uint32_t badm, uint32_t &fail_u, uint32_t &fail_lane)
{
    if (__ballot(badm != 0) == 0) return;
#pragma unroll
    for (uint32_t u = 0; u < kLinesU; u++) {
        const uint64_t fb = __ballot((badm >> u) & 1u);
        if (fb) {
            fail_u = u;
            fail_lane = (uint32_t) __ffsll((unsigned long long) fb) - 1;
            return;
        }
    }
}

// k_decode_lines' hot path for line-structured text (a full wave, aligned
// buffers, every window inside the input): lane slot t0 + 64 u + lane for u
// < kLinesU; returns the lane's failed-slot bits.  inw: the input at the
// dword below the wave's first line start, pos0 (0..3) that line start's
// offset from it (BIG; else inw = in and pos0 the line start's position);
// the output of slot t0 is outw + obase (BIG: obase 0, outw 64-bit; else
// outw = out), so lane offsets stay 32-bit at any stream length.  A4: L % 4 == 0 (RFC
// 2045's 76, PEM's 64), where a line end falls on a dword of the slot.
template <bool A4>
DEV uint32_t lines_hot(const uint8_t *tab, const uint8_t *__restrict__ inw, uint32_t pos0,
                       uint8_t *__restrict__ outw, uint32_t obase, const LineModel &m,
                       uint32_t col0, uint32_t lane)
{
    const uint32_t L = m.L, s = m.s, P = m.P;
    uint4 win[kLinesU];
    uint2 wx[kLinesU];
    uint32_t oo[kLinesU], cc[kLinesU];
    bool hs[kLinesU];
#pragma unroll
    for (uint32_t u = 0; u < kLinesU; u++) {
        // rel < L + 4,096 and rcp < 2^16: 24-bit products (full rate;
        // a 32-bit multiply issues at a quarter of it), exact
        const uint32_t rel = col0 + 16 * (u * 64 + lane);
        const uint32_t dl = __umul24(rel, m.rcp) >> 20;
        const uint32_t col = rel - __umul24(dl, L);
        const uint32_t pos = pos0 + __umul24(dl, P) + col;
        hs[u] = L - col <= 16;  // a line ends in (or right after) the slot
        cc[u] = hs[u] ? L - col : 16u;
        oo[u] = pos & 3u;
        const uint8_t *ab = inw + (pos & ~3u);
        // (non-temporal: neutral, r02_ab_lines_ntl.jsonl; with the 8-byte
        // load too, 443 -> 476 us, r06_e_ab.jsonl)
        win[u] = ld16<false>(ab);
        const u32x2a4 v = *(const u32x2a4 *) (ab + 16);
        wx[u] = make_uint2(v.x, v.y);
    }
    const uint32_t need = sep_need(s);
    uint32_t badm = 0;  // bit u: this lane's slot u failed
#pragma unroll
    for (uint32_t u = 0; u < kLinesU; u++) {
        const uint32_t w6[6] = {win[u].x, win[u].y, win[u].z, win[u].w, wx[u].x, wx[u].y};
        uint32_t sep, G[4], bad;
        const uint4 d = A4 ? slot_chars4(w6, oo[u], cc[u] >> 2, s, &sep)
                           : slot_chars(w6, oo[u], cc[u], s, &sep);
        map_fast(tab, d, 16, G, bad);
        // the separator bytes of a line that ends here must all be
        // outside the alphabet (looked up by every lane, kept by those)
        // (no branch: the bytes required are zero where no line ends)
        const uint32_t nd = hs[u] ? need : 0u;
        if ((sep_nonalpha(tab, sep) & nd) != nd) bad |= 0x100u;
        badm |= bad ? 1u << u : 0u;
        emit_full_off<true>(G, outw, obase + 12 * (u * 64 + lane));
    }
    return badm;
}

// BIG: n > 2^31 (up to kLinesMaxChars): sextet indices and positions of a
// wave's first slot are 64-bit, divided by L in 64 bits, and the wave's loads
// and stores go through 64-bit wave bases; below, the 32-bit forms of rounds
// 2-5 (the 64-bit bases cost the clean decode 1.5 %, r06_h_ab.jsonl).
template <bool BIG>
__global__ __launch_bounds__(kLinesTH) __attribute__((amdgpu_waves_per_eu(6)))
void k_decode_lines(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out, uint32_t nranges,
    DecAlpha a, void *ws, uint32_t hold, b64x_dec_result *res, uint32_t seq)
{
    __shared__ uint8_t tab[256];
    __shared__ uint8_t s_tail[64];
    // the scalar loads of the model overlap the table build
    const uint64_t *mp = (const uint64_t *) ws_view(ws, nranges).model;
    const uint64_t mw0 = scalar_load_u64(mp), mw1 = scalar_load_u64(mp + 1),
                   mw2 = scalar_load_u64(mp + 2), mw3 = scalar_load_u64(mp + 3);
    const uint64_t mn = scalar_load_u64(ws_view(ws, nranges).model_n);
    build_dec_table(tab, a);
    // A model made for another length (a workspace whose last probe was not
    // for this length, or a fresh one at a reused address): the clean model
    // of this length instead (L = 0, every slot, no cut) -- exact like any
    // model; clean input keeps the fast path and anything else fails a slot
    // and goes to k_decode_suffix_held (which then asks for a probe).
    const bool mok = mn == n;
    const uint32_t T = mok ? (uint32_t) (mw1 >> 32) : (uint32_t) (n / 16);
    // a block wholly past slot T (the probe cut the model's slots at junk)
    // leaves before the barrier: on junk-laden input nearly every block of
    // this launch does.  (Tested before the table build, the model's load
    // no longer overlapped the build: MIME text +2 %.)
    if (blockIdx.x * kLinesWaves * kLinesSlots > T) return;
    block_sync();
    LineModel m;
    m.L = mok ? (uint32_t) mw0 : 0u;
    m.s = (uint32_t) (mw0 >> 32);
    m.P = (uint32_t) mw1;
    m.T = T;
    m.m = (uint32_t) mw2;
    m.k = (uint32_t) (mw2 >> 32);
    m.rcp = (uint32_t) mw3;
    m.skip = mok ? (uint32_t) (mw3 >> 32) : 0u;
    const uint32_t lane = lane_id();
    const uint32_t L = m.L, s = m.s, P = m.P;
    // the wave's first slot, made visibly wave-uniform: its line coordinates
    // and output address are then scalar (a vector t0 cost a 64-bit
    // multiply-add per slot store and a 32-bit multiply per wave)
    const uint32_t wv = (uint32_t) __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6));
    const uint32_t t0 = (blockIdx.x * kLinesWaves + wv) * kLinesSlots;
    if (t0 > T) return;
    const uint32_t ns = T - t0 >= kLinesSlots ? kLinesSlots : T - t0;  // interior slots here
    const bool full = ns == kLinesSlots;
    const bool oal = (((uintptr_t) out) & 3) == 0;
    const bool ial = (((uintptr_t) in) & 3) == 0;
    uint32_t fail_u = kLinesU, fail_lane = 0;  // the wave's first failing slot
    // line coordinates of the wave's first sextet (scalar; BIG: a 64-bit
    // division, once per wave)
    const uint64_t i0 = 16ull * t0;
    const uint32_t line0 = !L ? 0u : !BIG ? line_div(m, (uint32_t) i0) : (uint32_t) (i0 / L);
    const uint32_t col0 = (uint32_t) (i0 - (uint64_t) line0 * L);
    // the wave's windows all end inside the input (24 bytes from a dword at
    // or below each span's start)
    const uint64_t ie = i0 + 16 * ns;
    const uint32_t le = !L ? 0u : !BIG ? line_div(m, (uint32_t) ie) : (uint32_t) (ie / L);
    const bool safe = (L ? (uint64_t) le * P + (ie - (uint64_t) le * L) : ie) + 24 <= n;
    // the wave's first line start and its output: BIG, 64-bit bases and
    // 32-bit offsets from them; else 32-bit offsets from in and out
    const uint64_t pos0 = (uint64_t) line0 * P;
    uint8_t *const outw = BIG ? out + 12ull * t0 : out;
    const uint32_t obase = BIG ? 0u : 12 * t0;
    if (ns && L == 0 && full && oal && ial) {
        // The hot path (clean input, a full wave, aligned buffers): lane t's
        // 16 characters are one non-temporal dwordx4 at 16t, its 12 bytes one
        // non-temporal dwordx3 at 12t -- pass 1's fast path, output-indexed.
        // Kept apart from the general paths below so that no load or store
        // here is exec-masked (a masked form also lost the nt bit and waited
        // on every load at once: 7 % slower).
        uint4 c[kLinesU];
        const uint8_t *const inw = BIG ? in + 16ull * t0 : in;
        const uint32_t ibase = BIG ? 0u : 16 * t0;
#pragma unroll
        for (uint32_t u = 0; u < kLinesU; u++) c[u] = ld16<true>(inw + (ibase + 16 * (u * 64 + lane)));
        uint32_t badm = 0;  // bit u: this lane's slot u failed
#pragma unroll
        for (uint32_t u = 0; u < kLinesU; u++) {
            uint32_t G[4], bad;
            map_fast(tab, c[u], 16, G, bad);
            badm |= bad ? 1u << u : 0u;
            emit_full_off<true>(G, outw, obase + 12 * (u * 64 + lane));
        }
        lines_first_fail(badm, fail_u, fail_lane);
    } else if (ns && L != 0 && full && oal && ial && safe) {
        // The hot path of line-structured text: 32-bit offsets from the
        // wave's bases, unguarded window loads, non-temporal stores.  Two
        // instances, one per line-length class, behind a wave-uniform branch:
        // written as `a4 ? slot_chars4(..) : slot_chars(..)` the compiler
        // computed both forms for every slot and selected (692 VALU for a
        // wave's 4 slots in the listing, ~250 of them the general form that
        // CRLF-76 never uses).
        const uint8_t *const inw = BIG ? in + (pos0 & ~3ull) : in;
        const uint32_t p0 = (uint32_t) (BIG ? pos0 & 3u : pos0);
        const uint32_t badm = (L & 3) == 0
            ? lines_hot<true>(tab, inw, p0, outw, obase, m, col0, lane)
            : lines_hot<false>(tab, inw, p0, outw, obase, m, col0, lane);
        lines_first_fail(badm, fail_u, fail_lane);
    } else if (ns) {
        // Everything else (a partial wave, the input's end, misaligned
        // buffers): guarded window loads through 64-bit addresses.
        uint32_t G[kLinesU][4], bad[kLinesU];
        const uint8_t *end = in + n;
        uint4 win[kLinesU];
        uint2 wx[kLinesU];
        uint32_t oo[kLinesU], cc[kLinesU];
        bool hs[kLinesU];
#pragma unroll
        for (uint32_t u = 0; u < kLinesU; u++) {
            const uint32_t rel = col0 + 16 * (u * 64 + lane);
            const uint32_t dl = L ? (rel * m.rcp) >> 20 : 0;
            const uint32_t col = rel - dl * L;
            const uint64_t pos = L ? (uint64_t) (line0 + dl) * P + col : i0 + 16 * (u * 64 + lane);
            hs[u] = L && L - col <= 16;
            cc[u] = hs[u] ? L - col : 16u;
            const uint8_t *ap = in + pos;
            const uint8_t *ab = (const uint8_t *) ((uintptr_t) ap & ~(uintptr_t) 3);
            oo[u] = (uint32_t) (ap - ab);
            const bool live = u * 64 + lane < ns;
            win[u] = live ? load_win16(ab, end) : make_uint4(0, 0, 0, 0);
            wx[u] = live ? load_win8(ab + 16, end) : make_uint2(0, 0);
        }
#pragma unroll
        for (uint32_t u = 0; u < kLinesU; u++) {
            const uint32_t w6[6] = {win[u].x, win[u].y, win[u].z, win[u].w, wx[u].x, wx[u].y};
            uint32_t sep;
            const uint4 d = slot_chars(w6, oo[u], cc[u], s, &sep);
            map_fast(tab, d, 16, G[u], bad[u]);
            const uint32_t need = sep_need(s);
            if (hs[u] && (sep_nonalpha(tab, sep) & need) != need) bad[u] |= 0x100u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kLinesU; u++) {
            const bool live = u * 64 + lane < ns;
            const uint64_t fb = __ballot(live && bad[u] != 0);
            if (fb && fail_u == kLinesU) {
                fail_u = u;
                fail_lane = (uint32_t) __ffsll((unsigned long long) fb) - 1;
            }
            if (live) {
                uint32_t o0, o1, o2;
                groups_to_bytes(G[u][0], G[u][1], G[u][2], G[u][3], o0, o1, o2);
                store_bytes12(out + 12 * (uint64_t) (t0 + u * 64 + lane), o0, o1, o2, 12);
            }
        }
    }
    // Under a cut model (skip) the wave that owns slot T publishes it as
    // failing unless one of its slots failed first: the probe has done so
    // when it ran, and a call that reused the model has no probe.
    const bool cut = m.skip && T < t0 + kLinesSlots;
    if ((fail_u < kLinesU || cut) && lane == 0) {
        // publish the first failing slot; only an improvement (the
        // device-scope load sees what earlier waves published)
        const unsigned long long key =
            ~(unsigned long long) (fail_u < kLinesU ? t0 + fail_u * 64 + fail_lane : T);
        unsigned long long *lf = (unsigned long long *) ws_view(ws, nranges).lfail +
                                 (blockIdx.x % kFailWords) * kFailStride;
        const unsigned long long cur =
            __hip_atomic_load(lf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (key > cur) atomicMax(lf, key);
        // the first publisher into a word sees it zero (at most a few racing
        // ones do): they raise the summary the idle suffix kernel reads
        if (cur == 0) *ws_view(ws, nranges).fail_any = 1;
    }
    if (T >= t0 + kLinesSlots || m.skip) return;
    // This wave owns slot T: the < 16 + s bytes after the last interior
    // span, decoded exactly, and the result record (replaced by
    // k_decode_suffix_held when a slot failed).
    const uint64_t Q = line_pos(m, 16 * (uint64_t) T);
    const uint32_t tl = (uint32_t) (n - Q);  // < 16 + s <= 20
    const bool here = lane < tl;
    const uint32_t tv = here ? tab[in[Q + lane]] : 0xFFu;
    const bool al = tv < 64u;
    const uint64_t mb = __ballot(al);
    const uint32_t Vt = (uint32_t) __popcll(mb);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (mb >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t) mb, 0u));
    if (al) s_tail[rank] = (uint8_t) tv;
    wave_lds_order();
    const uint32_t ng = Vt >> 2, rem = Vt & 3u;
    uint8_t *ot = out + 12 * (uint64_t) T;
    if (lane < ng) {
        const uint32_t G = ((uint32_t) s_tail[4 * lane] << 18) | ((uint32_t) s_tail[4 * lane + 1] << 12) |
                           ((uint32_t) s_tail[4 * lane + 2] << 6) | s_tail[4 * lane + 3];
        ot[3 * lane] = (uint8_t) (G >> 16);
        ot[3 * lane + 1] = (uint8_t) (G >> 8);
        ot[3 * lane + 2] = (uint8_t) G;
    } else if (lane == ng && !hold && rem >= 2) {
        // the final partial group: floor(6r/8) bytes (src/base64decoder.c:71-76)
        const uint32_t G = ((uint32_t) s_tail[4 * ng] << 18) | ((uint32_t) s_tail[4 * ng + 1] << 12) |
                           (rem > 2 ? (uint32_t) s_tail[4 * ng + 2] << 6 : 0u);
        ot[3 * ng] = (uint8_t) (G >> 16);
        if (rem > 2) ot[3 * ng + 1] = (uint8_t) (G >> 8);
    }
    if (lane == 0) {
        const uint64_t V = 16 * (uint64_t) T + Vt;
        b64x_dec_result r;
        r.out_len = hold ? V / 4 * 3 : V * 6 / 8;
        r.valid = V;
        r.tail_n = rem;
        for (uint32_t j = 0; j < 4; j++) r.tail[j] = j < rem ? s_tail[4 * ng + j] : 0;
        r.nchars = n;
        r.seq = seq;
        r.flags = hold ? 1u : 0u;
        *res = r;  // provisional: k_decode_suffix_held mirrors it to the host or replaces it
    }
}

// One range of the exact decode: characters [start, re) (re = the range's
// end, the stream's when `last`), whose first 2,048 characters' chunks are
// c[] (nin[] characters of each lane in range).  T0 = 0 when the range
// starts on a group boundary, else minus the 0-3 sextets the previous range
// owns (they land in the window's head); ob = the output address of the
// range's first owned group; la (valid if la_ok) = the lookahead byte after
// re.  A range longer than 2,048 characters (inputs past 2 GiB: the range
// count is capped) is taken 2,048 at a time, the window's whole dwords
// flushed between steps and its partial dword carried to the front (as
// decode_buf_bits does); the bytes flushed early are final and never reach
// the next range's output.
DEV void decode_range(const P2dSmem &sm, uint4 *bq, const uint8_t *__restrict__ in, uint64_t n,
                      uint64_t start, uint64_t re, int T0, uint8_t *ob, const uint4 c[2],
                      const uint32_t nin[2], uint32_t la, bool la_ok, bool last, uint32_t hold,
                      const uint8_t *la_lds = nullptr, bool la_late = false)
{
    const uint32_t lane = lane_id();
    uint32_t *bits = (uint32_t *) bq;
    int T = T0;
    // the window is aligned to 16 output bytes: LDS byte 16 + (ob & 15) is
    // output byte ob, so whole blocks copy as aligned 16-byte pairs
    const uint32_t skew = (uint32_t) ((uintptr_t) ob & 15);
    uint32_t lo = 16 + skew;      // LDS byte of output byte `done`
    int pb0 = 8 * (int) lo;       // window bit of relative sextet 0
    uint32_t done = 0;            // bytes flushed by earlier steps
    static_assert(kP2dBlocks > 64 && kP2dBlocks <= 128, "two zeroing stores per lane");
    bq[lane] = make_uint4(0, 0, 0, 0);
    if (lane + 64 < kP2dBlocks) bq[lane + 64] = make_uint4(0, 0, 0, 0);
    wave_lds_order();
    // the first step from the chunks given (its own code: joined with the
    // loads of the later steps, the compiler waited for every load in
    // flight before the step, ranges read ahead included)
    T += (int) bits_step<true>(sm, bits, c, nin, pb0 + 6 * T);
    for (uint64_t pos = start + 2 * kChunk; pos < re; pos += 2 * kChunk) {
        // more of this range: flush the window's whole blocks and carry the
        // partial one to the front
        wave_lds_order();
        const int bit_end = pb0 + 6 * T;
        const uint32_t kcut = bit_end > 0 ? ((uint32_t) bit_end >> 3) & ~15u : 0u;
        if (kcut > lo) {
            store_bits16(bq, lo, kcut, ob + done - lo);
            done += kcut - lo;
            const uint4 keep = bq[kcut >> 4];
            wave_lds_order();
            bq[lane] = make_uint4(0, 0, 0, 0);
            if (lane + 64 < kP2dBlocks) bq[lane + 64] = make_uint4(0, 0, 0, 0);
            wave_lds_order();
            if (lane == 0) bq[1] = keep;
            wave_lds_order();
            pb0 -= 8 * (int) (kcut - 16);
            lo = 16;
        }
        uint4 ch[2];
        uint32_t nh[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint64_t q = pos + (uint64_t) h * kChunk + 16 * lane;
            nh[h] = q >= re ? 0u : (re - q >= 16 ? 16u : (uint32_t) (re - q));
            ch[h] = nh[h] ? load_chars(in + q, nh[h]) : make_uint4(0, 0, 0, 0);
        }
        T += (int) bits_step<true>(sm, bits, ch, nh, pb0 + 6 * T);
    }
    bool at_end = last;
    if (!last && T > 0 && (T & 3)) {
        // complete the range's last group from the characters after it:
        // given (la, la_ok), in LDS at la_lds (the next range, whole, copied
        // there by k_decode_suffix_held while this range decoded: waited for
        // now), or read from `in` only now (la_late)
        bool ok = la_ok;
        if (la_lds) {
            vm_wait_all();
            ok = true;
            la = la_lds[lane];
        } else if (la_late) {
            ok = re + lane < n;
            la = ok ? in[re + lane] : 0u;
        }
        for (uint64_t q = re;;) {
            const uint32_t t = ok ? sm.tab[la] : 0xFFu;
            const bool v = t < 64u;
            const uint64_t m = __ballot(v);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
            const int need = 4 - (T & 3);
            if (v && (int) rank < need)
                or_field<true>(bits, (uint32_t) (pb0 + 6 * (T + (int) rank)), t << 26);
            const int got = __popcll(m);
            if (got >= need) {
                T += need;
                break;
            }
            T += got;
            q += 64;
            if (q >= n) {
                at_end = true;  // the stream's final, incomplete group
                break;
            }
            ok = q + lane < n;
            la = ok ? in[q + lane] : 0u;
        }
    }
    wave_lds_order();
    if (T > 0) {
        const uint32_t ng = (uint32_t) T >> 2, rem = (uint32_t) T & 3u;
        // the final partial group: 2 sextets -> 1 byte, 3 -> 2 (floor(6r/8),
        // src/base64decoder.c:59-62,71-76)
        const uint32_t tail = at_end && !hold && rem >= 2 ? rem - 1 : 0u;
        const uint32_t total = 3 * ng + tail;
        if (total > done) store_bits16(bq, lo, lo + (total - done), ob + done - lo);
    }
    wave_lds_order();  // the next range re-zeroes the buffer
}

// The first step's chunks of the range [rb, re) from `start` on, and its
// lookahead byte.
DEV void load_range(const uint8_t *__restrict__ in, uint64_t n, uint64_t start, uint64_t re,
                    bool last, uint4 c[2], uint32_t nin[2], uint32_t &la, bool &la_ok)
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint64_t p = start + (uint64_t) h * kChunk + 16 * lane;
        nin[h] = p >= re ? 0u : (re - p >= 16 ? 16u : (uint32_t) (re - p));
        c[h] = nin[h] ? load_chars(in + p, nin[h]) : make_uint4(0, 0, 0, 0);
    }
    la_ok = !last && re + lane < n;
    la = la_ok ? in[re + lane] : 0u;
}

DEV int range_skip(uint64_t B) { return -(int) ((4 - (B & 3)) & 3); }

// Pass 2 (exact), after pass 1 and the scan: grid-stride over the ranges
// from the first dirty chunk on, with exactly the resident blocks.  The
// first dirty range resumes at its dirty chunk (everything before it was
// alphabet and is final); later ranges re-run with their true base.  For
// the middle ranges the next range's loads (both chunks, the lookahead
// bytes, its base) are issued before this range is processed.
__global__ __launch_bounds__(kThreads) void k_decode_pass2d(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out,
    uint64_t R, uint32_t nranges, DecAlpha a, void *ws, uint32_t hold)
{
    DecodeWs w = ws_view(ws, nranges);
    const uint64_t packed = *w.fd_cur;
    if (packed == 0) return;
    const uint32_t r0 = (uint32_t) (~packed >> 32);
    const uint32_t off0 = (uint32_t) ~packed;
    __shared__ P2dSmem sm;
    build_dec_table(sm.tab, a);
    build_compact_sel(sm.sel);
    block_sync();
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 *bq = sm.bits[wv];
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    auto generic = [&](uint32_t r) {
        const uint64_t rb = (uint64_t) r * R;
        const uint64_t re = rb + R < n ? rb + R : n;
        const bool last = r + 1 == nranges, first = r == r0;
        const uint64_t B = scalar_load_u64(w.bases + r);
        const uint64_t start = first ? rb + off0 : rb;
        uint4 c[2];
        uint32_t nin[2], la;
        bool la_ok;
        load_range(in, n, start, re, last, c, nin, la, la_ok);
        decode_range(sm, bq, in, n, start, re, first ? 0 : range_skip(B),
                     out + (first ? (B + off0) / 4 * 3 : (B + 3) / 4 * 3), c, nin, la, la_ok,
                     last, hold);
    };
    uint32_t r = r0 + blockIdx.x * kWavesPerBlock + wv;
    if (r == r0 && r < nranges) {
        generic(r);
        r += nw;
    }
    const uint32_t mid_end = nranges - 1;
    if (R == 2 * kChunk && r < mid_end && (((uintptr_t) in) & 3) == 0) {
        const uint32_t full[2] = {16u, 16u};
        auto ld_la = [&](uint32_t rr) {
            const uint64_t q = (uint64_t) (rr + 1) * R + lane;
            return (uint32_t) in[q < n ? q : n - 1];
        };
        uint4 c[2];
        c[0] = load16_a4(in + (uint64_t) r * R + 16 * lane);
        c[1] = load16_a4(in + (uint64_t) r * R + kChunk + 16 * lane);
        uint32_t la = ld_la(r);
        uint64_t B = scalar_load_u64(w.bases + r);
        while (r < mid_end) {
            const uint32_t rn = r + nw < mid_end ? r + nw : r;  // unconditional prefetch
            uint4 cn[2];
            cn[0] = load16_a4(in + (uint64_t) rn * R + 16 * lane);
            cn[1] = load16_a4(in + (uint64_t) rn * R + kChunk + 16 * lane);
            const uint32_t lan = ld_la(rn);
            const uint64_t Bn = scalar_load_u64(w.bases + rn);
            const uint64_t rb = (uint64_t) r * R;
            decode_range(sm, bq, in, n, rb, rb + R, range_skip(B), out + (B + 3) / 4 * 3, c, full,
                         la, (uint64_t) (r + 1) * R + lane < n, false, hold);
            r += nw;
            c[0] = cn[0];
            c[1] = cn[1];
            la = lan;
            B = Bn;
        }
    }
    for (; r < nranges; r += nw) generic(r);
}

// ---- single-pass exact decode of a suffix ---------------------------------
//
// k_decode_suffix_held decodes characters [S, n) into out + O, S being a
// group boundary of the whole stream (Vb = the alphabet characters before S,
// a multiple of 4, O = 3 Vb / 4), and writes the result record for the whole
// stream.  WHOLE: S = 0 (B64X_DEC_EXPECT_JUNK, and the hinted single pass);
// else S, O, Vb come from the first failing slot k_decode_lines published,
// and the kernel exits at once when there is none (the common case: every
// block reads one word and returns).
//
// Ranges are the pass-1 ranges of R = 2,048 characters, aligned to the
// stream; the first one, r0 = S / R, starts at S.  Persistent blocks take
// tiles of kHeldTile ranges (kHeldPer per wave) from a ticket in the order
// they start, so a tile's predecessors are running or done whatever else
// shares the GPU.  A tile's prefix is not a chained look-back: it is the
// counts of the tiles before it in its group of 64 tiles (one status word
// per lane) plus the sums of the earlier groups (every tile adds its count
// into its group's word), loaded at once.  (Round 2's chained look-back --
// back over predecessors' aggregates 64 at a time to the first inclusive
// prefix, three waves idle at a barrier -- cost 157 of 945 us on 1 GiB at
// junk density 0.05, profiles/r03_ab_sfx_breakdown.jsonl.)  Every block
// counts itself out in `wdone` when it leaves; the block that decodes the
// last tile writes the record, waits until every block has left (so no
// prefix read is in flight), then clears the status and group words, the
// ticket, `wdone` and the failure words.  Rounds 3-5 shipped a form that
// counted each tile one tile ahead and re-read it to decode (FETCH 2.01x the
// input); it was removed in round 6 (DESIGN.md §5 keeps its measurements).
// hint (the hinted single pass only; else null): the block that draws
// ticket ntiles -- the first with no tile left -- runs the probe
// (probe_stream, publish 0) for the next call while the others finish.

// The idle test of k_decode_suffix_held<false>: false when k_decode_lines took
// everything (its record is then mirrored to the host and the call is
// done); else S, Vb of the first failing slot, and *reprobe (pinned, the
// launcher's: the next call of this length on the workspace probes again
// instead of reusing the model) is set.  Every block.
DEV bool suffix_start(DecodeWs w, uint64_t n, b64x_dec_result *res, b64x_dec_result *hres,
                      uint64_t &S, uint64_t &Vb, uint32_t *reprobe)
{
    __shared__ uint64_t s_key;
    uint64_t key = 0;
    if (scalar_load_u64(w.fail_any) != 0) {
        // the first failing slot: the largest key over the failure words
        if (threadIdx.x < 64) {
            key = __hip_atomic_load((unsigned long long *) w.lfail + (threadIdx.x % kFailWords) *
                                    kFailStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                const uint64_t o = __shfl_xor(key, d, 64);
                key = o > key ? o : key;
            }
        }
        if (threadIdx.x == 0) s_key = key;
        block_sync();
        key = s_key;
    }
    if (key == 0) {
        // nothing failed: k_decode_lines' record is final.  The host mirror
        // is written only now, so a completion never finds a consistent but
        // provisional record there.
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (hres) {
                const b64x_dec_result r = *res;
                *hres = r;
            }
            *w.sfx_start = ~0ull;
        }
        return false;
    }
    Vb = 16 * ~key;  // the first failing slot of k_decode_lines
    // under the model k_decode_lines used: the workspace's, or the clean
    // model when the workspace's was made for another length
    S = scalar_load_u64(w.model_n) == n ? line_pos(*w.model, Vb) : Vb;
    if (reprobe && blockIdx.x == 0 && threadIdx.x == 0) *(volatile uint32_t *) reprobe = 1u;
    return true;
}

// ---- each range read and looked up once -----------------------------------
//
// A range is decoded once, at relative bit 0 of the wave's window (its
// prefix is not known yet), and the window -- the range's output bit stream,
// at most 1,536 bytes -- is held in VGPRs (6 dwords per lane) while the tile
// is published and the next tile is decoded; the range's count comes out of
// the decode.  A tile is stored one iteration later, when its prefix is
// known (its predecessors have had a whole tile's time to publish): the held
// dwords go back into the window, the range's last partial group is
// completed from the characters after it (their raw bytes loaded when the
// range was decoded), and the window is copied to the output shifted by the
// range's skip (0-3 sextets the range before it completed) and the output's
// alignment.  Each input byte is read from HBM once and looked up once.  On
// 1 GiB at junk density 0.05 (profiles/r05_pmc_sfx_held.txt,
// r05_ab_sfx_held*.jsonl): FETCH 1.02x the input against the count-ahead
// form's 2.01x, VALU -10 %, SALU -27 %, LDS instructions -20 %, and the same
// time: the kernel is bound by latency at 5 waves per SIMD (96 VGPRs, two
// tiles held while the next decodes), not by its bytes.  Tried and slower: a
// tile's ticket drawn one iteration ahead (940 us), storing range j of A
// right after decoding range j of B (2.2-2.8 ms, tiles waiting on their
// predecessors), 3 or 2 ranges per wave (815 / 1,153 against 725), 5-8
// ranges per wave at 3-4 waves per SIMD (807-1,031), 4 waves per SIMD
// without spills (835 us).  The prefix loads only the groups completed since
// the block's last tile (746.5 against 778.2 us,
// profiles/r05_ab_sfx_prefix_incremental.jsonl).
//
// Its first form's barriers were hipcc's __syncthreads(), and the one at the
// top of an iteration did not wait for thread 0's write of the next ticket:
// now and then a wave decoded another tile than its block (one repeated
// 1 GiB decode in five came out shifted).  The ISA shows why
// (profiles/r06_isa_barrier_evidence.txt): the fence of __syncthreads()
// leaves a soft s_waitcnt lgkmcnt(0) before the s_barrier, and gfx950's
// back-off barrier needs no wait of its own, so SIInsertWaitcnts may drop
// the soft one -- and at this loop's header it did (present in the MIR
// before the pass, gone after), although the back edge carries thread 0's
// ds_write of the ticket.  block_sync()'s wait is inline asm, which the pass
// cannot drop; tests/tools/isa_check.py walks the control-flow graph of
// every kernel in the shipped code object and finds no barrier reached with
// an LDS write in flight (test_abi.py::test_code_object_barriers_drain_lds).

// The window dword a range's held dwords go back to, so that
// store_window_bits reads aligned 16-byte groups: the range's bits start at
// bit s (its skip) and its output at dst.
DEV uint32_t window_delta(uint32_t s, const uint8_t *dst)
{
    const uint32_t a = (uint32_t) ((uintptr_t) dst & 15);
    const uint32_t i0 = (s + (a ? 128u : 0u) - 8 * a) >> 5;
    return (4u - (i0 & 3u)) & 3u;
}

// Output bytes [0, nb) at dst are window bits [s, s + 8 nb) (big-endian
// dwords, or_field<true>; s placed by window_delta): aligned 16-byte
// blocks of dst, each four window dwords read as one aligned 16-byte LDS
// read (consecutive lanes, consecutive 16-byte groups: no bank conflicts)
// plus, when the shift is not 0, the next group's first dword (a
// ds_read_b32 four ways conflicted; taking it from the next lane by DPP
// cost more VALU than the conflicts), funnel-shifted by the same
// amount for every block; the partial blocks at both ends one byte per lane.
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const v4u32 lds_v4u32;

DEV void store_window_bits(const uint32_t *win, uint32_t s, uint32_t nb, uint8_t *dst)
{
    const uint32_t lane = lane_id();
    // wave-uniform arguments, made visibly so (read back from LDS counts, the
    // compiler kept them and everything derived from them in VGPRs: the
    // shift's test an exec-mask branch, the block loop's bounds vector)
    s = (uint32_t) __builtin_amdgcn_readfirstlane((int) s);
    nb = (uint32_t) __builtin_amdgcn_readfirstlane((int) nb);
    const uint32_t a = (uint32_t) ((uintptr_t) dst & 15);
    // block m of the aligned grid covers bytes [16 m - a, 16 m - a + 16)
    const uint32_t m0 = a ? 1u : 0u, mend = (nb + a) >> 4;
    const uint32_t b0 = s + 128 * m0 - 8 * a;
    const uint32_t i0 = b0 >> 5, sh = b0 & 31;  // block m0's first window dword (a multiple of 4)
    const uint32_t nblk = mend > m0 ? mend - m0 : 0u;
    uint8_t *const base = dst - a + 16 * m0;     // 16-byte aligned, wave-uniform
    constexpr uint32_t kLast = kP2dBlocks * 4 - 8;  // the last group read in full
    // The partial blocks' bytes (head [0, hend), tail [tb, nb); at most 15
    // each, one per lane of lanes 0-31): their two window dwords are read
    // first, so that one wait covers them and the first groups.
    const uint32_t hend = a ? (16 - a < nb ? 16 - a : nb) : 0u;
    const uint32_t tb = mend > m0 ? 16 * mend - a : hend;
    // (lane + a scalar: written as lane - 16 + ..., the loop-invariant
    // lane - 16 was hoisted out of the tile loop and spilled, and its reload
    // in every range waited for the previous range's stores)
    const uint32_t bi = lane + (lane < 16 ? 0u : (tb > hend ? tb : hend) - 16u);
    const bool act = lane < 16 ? bi < hend : lane < 32 && bi < nb;
    const uint32_t X = s + 8 * bi, xi = (X >> 5) < kLast ? X >> 5 : kLast;
    const uint32_t x0 = win[xi], x1 = win[xi + 1];
    // Every lane reads its group and the next dword (no shuffle, no masked
    // read: an index clamped inside the window for lanes past the end), the
    // funnel shift is one v_alignbit per dword (sh = 0, wave-uniform: none),
    // and only the store is masked (round 5: a masked read, a shuffle and a
    // masked read of the next dword, each waited for, and 64-bit shifts).
    for (uint32_t k0 = 0; k0 < nblk; k0 += 64) {
        const uint32_t k = k0 + lane;
        const uint32_t ik = i0 + 4 * k;
        const uint32_t i = ik < kLast ? ik : kLast;
        // one ds_read_b128 (a plain uint4 read was split into five reads
        // of overlapping dword pairs, each waited for: the non-temporal form
        // keeps it whole; LDS has no temporal hint to take)
        const v4u32 g4 = __builtin_nontemporal_load((const lds_v4u32 *) (win + i));
        const uint4 g = make_uint4(g4.x, g4.y, g4.z, g4.w);
        const uint32_t w4 = win[i + 4];
        uint32_t o0 = g.x, o1 = g.y, o2 = g.z, o3 = g.w;
        if (sh) {
            const uint32_t r = 32u - sh;
            o0 = __builtin_amdgcn_alignbit(g.x, g.y, r);
            o1 = __builtin_amdgcn_alignbit(g.y, g.z, r);
            o2 = __builtin_amdgcn_alignbit(g.z, g.w, r);
            o3 = __builtin_amdgcn_alignbit(g.w, w4, r);
        }
        if (k < nblk)
            __builtin_nontemporal_store(u32x4a16{bswap32(o0), bswap32(o1), bswap32(o2), bswap32(o3)},
                                        (u32x4a16 *) (base + 16 * k));
    }
    if (act) dst[bi] = (uint8_t) ((((uint64_t) x0 << 32) | x1) >> (56 - (X & 31)));
}

// BIG: n > 2^31 (up to kLinesMaxChars): a tile's prefix -- alphabet
// characters of the suffix before it -- in 64 bits (in 32 below: the 64-bit
// sums cost 7 % at junk density 0.05, r06_h_ab.jsonl).
template <bool WHOLE, bool BIG>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kHeldWaves)))
void k_decode_suffix_held(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out, uint32_t nranges,
    DecAlpha a, void *ws, uint32_t hold, b64x_dec_result *res, b64x_dec_result *hres,
    uint32_t seq, uint32_t *reprobe, DecodeHint *hint, uint32_t key)
{
    constexpr uint64_t R = 2 * kChunk;
    constexpr uint32_t HP = kHeldPer, TILE = kHeldTile;
    DecodeWs w = ws_view(ws, nranges);
    uint64_t S = 0, Vb = 0;
    if (!WHOLE && !suffix_start(w, n, res, hres, S, Vb, reprobe)) return;
    uint8_t *base_out = out + Vb / 4 * 3;
    const uint32_t r0 = (uint32_t) (S / R);
    const uint32_t ntiles = (nranges - r0 + TILE - 1) / TILE;
    if (!WHOLE && blockIdx.x == 0 && threadIdx.x == 0) *w.sfx_start = S;
    const bool dma = (((uintptr_t) in) & 15) == 0;
    __shared__ P2dSmem sm;
    __shared__ uint4 s_rng[kWavesPerBlock][2][128];
    __shared__ uint32_t s_tile[2];
    using Cnt = typename std::conditional<BIG, uint64_t, uint32_t>::type;
    __shared__ uint32_t s_cnt[2][TILE];
    __shared__ Cnt s_excl;
    build_dec_table_lo(sm.tab, a);  // the bit-stream form: sextets as 4 v, flag in bit 0
    build_compact_sel<true>(sm.sel);  // indexed by the alphabet bytes (bits_step<..., true>)
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 *bq = sm.bits[wv];
    uint32_t *bits = (uint32_t *) bq;

    auto publish = [&](uint32_t t, uint32_t b) {
        uint32_t agg = 0;
        for (uint32_t i = 0; i < TILE; i++) agg += s_cnt[b][i];
        st_store(&w.fstatus[t], kStAgg | agg);
        __hip_atomic_fetch_add(&w.fsuper[t / kSfxGroup], (1ull << 56) | agg, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    // The groups before kdone are complete and sum to sdone (wave 0's, from
    // its earlier prefixes): a prefix loads its own group's statuses and the
    // groups since -- about 20 for a block's next tile, one word per lane,
    // one round trip.  (Loading every earlier group, 64 per lane-pass, took
    // one round trip per pass, each waited for before the next: 6 on average
    // on 1 GiB.)
    // (64-bit sums: a suffix of a stream past 2^32 characters, up to
    // kLinesMaxChars)
    uint32_t kdone = 0;
    Cnt sdone = 0;
    auto prefix = [&](uint32_t t) -> Cnt {
        const uint32_t k = t / kSfxGroup, own = t - k * kSfxGroup;
        for (;;) {
            const uint64_t v = lane < own ? st_load(&w.fstatus[k * kSfxGroup + lane]) : kStAgg;
            bool ok = (v & kStAgg) != 0;
            uint32_t sg = 0;
            for (uint32_t j0 = kdone; j0 < k; j0 += 64) {
                const uint32_t j = j0 + lane;
                const uint64_t g = j < k ? st_load(&w.fsuper[j]) : kGroupFull;
                ok = ok && (g >> 56) == kSfxGroup;
                sg += j < k ? (uint32_t) g : 0u;
            }
            if (__all(ok)) {
                sdone += BIG ? (Cnt) wave_sum64(sg) : (Cnt) wave_sum(sg);
                kdone = k;
                return sdone + wave_sum((uint32_t) v);
            }
            __builtin_amdgcn_s_sleep(2);
        }
    };
    auto whole = [&](uint32_t r) {
        return dma && r < nranges && r != r0 && (uint64_t) (r + 1) * R <= n;
    };
    auto fetch = [&](uint32_t r, uint32_t buf) {
        const uint8_t *src = in + (uint64_t) r * R;  // wave-uniform
        lds_dma16(src, &s_rng[wv][buf][0]);
        lds_dma16(src + kChunk, &s_rng[wv][buf][64]);
    };

    // Decode range j of tile t (this wave's) into the window; hold its
    // dwords [6 lane, 6 lane + 6) in Hn and, in lan, the table value of the
    // byte at lane offset after its end (the completion's first look, looked
    // up here: the load has landed by the range's wait); count into s_cnt[b].
    auto la_load = [&](uint32_t r) -> uint32_t {
        if (r >= nranges) return 0u;
        const uint64_t re = (uint64_t) r * R + R < n ? (uint64_t) r * R + R : n;
        return re + lane < n ? (uint32_t) in[re + lane] : 0u;
    };
    auto decode_one = [&](uint32_t rw, uint32_t j, uint32_t b, uint32_t Hn[6], uint32_t &lan,
                          uint32_t &lan_next) {
        const uint32_t r = rw + j;
        uint32_t T = 0;
#pragma unroll
        for (int i = 0; i < 6; i++) Hn[i] = 0;
        // this range's copy (issued by the range before, or for the tile's
        // first) has landed: waited for on every path, so that no path of
        // the listing reaches a barrier with a copy in flight
        // (tests/tools/isa_check.py; under `if (whole(r))` the checker saw
        // the infeasible path that skips it)
        vm_wait_all();
        if (r < nranges) {
            const uint64_t rb = (uint64_t) r * R;
            const uint64_t re = rb + R < n ? rb + R : n;
            const uint64_t start = r == r0 ? S : rb;
            const bool next_dma = j + 1 < HP && whole(r + 1);
            uint4 *buf = s_rng[wv][j & 1];
            uint32_t nin[2] = {16u, 16u};
            if (!whole(r)) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const uint64_t p = start + (uint64_t) h * kChunk + 16 * lane;
                    nin[h] = p >= re ? 0u : (re - p >= 16 ? 16u : (uint32_t) (re - p));
                    buf[64 * h + lane] = nin[h] ? load_chars(in + p, nin[h]) : make_uint4(0, 0, 0, 0);
                }
            }
            uint4 c[2];
            c[0] = buf[lane];
            c[1] = buf[64 + lane];
            if (next_dma) fetch(r + 1, (j + 1) & 1);
            if (j + 1 < HP) lan_next = la_load(r + 1);
            wave_lds_order();
            bq[lane] = make_uint4(0, 0, 0, 0);
            if (lane + 64 < kP2dBlocks) bq[lane + 64] = make_uint4(0, 0, 0, 0);
            wave_lds_order();
            // the wave's window as bits past sm.bits[0]: the ORs' addresses
            // are then a constant plus (p >> 3) & ~3, no per-wave base added
            T = bits_step<true, P2dSmem, true>(sm, (uint32_t *) sm.bits[0], c, nin, (int) (wv * kP2dBlocks * 128));
            wave_lds_order();
#pragma unroll
            for (int i = 0; i < 6; i++) Hn[i] = bits[lane + 64 * i];  // consecutive lanes
            lan = re + lane < n ? (uint32_t) sm.tab[lan] : 0xFFu;
            wave_lds_order();
        } else {
            lan = 0;
        }
        if (lane == 0) s_cnt[b][wv * HP + j] = T;
    };
    // Store range j of tile A (this wave's) from its held dwords: Bp = the
    // suffix's alphabet characters before it, T its own.
    // the window holds dwords dl + [0, 384) (dl <= 3) and the 8 zeroed after
    static_assert(kP2dBlocks * 4 >= 3 + 384 + 8, "held window fits the wave's LDS window");
    auto store_one = [&](uint32_t r, Cnt Bp, uint32_t T, const uint32_t Hj[6], uint32_t la) {
        const uint64_t rb = (uint64_t) r * R;
        const uint64_t re = rb + R < n ? rb + R : n;
        const bool last = r + 1 == nranges;
        const uint32_t k = (4u - ((uint32_t) Bp & 3u)) & 3u;  // sextets the range before took
        uint8_t *dst = base_out + (uint64_t) (Bp + k) / 4 * 3;
        const uint32_t dl = window_delta(6 * k, dst);  // the held dwords go to dl..
#pragma unroll
        for (int i = 0; i < 6; i++) bits[dl + lane + 64 * i] = Hj[i];
        if (lane < 8) bits[dl + 384 + lane] = 0;  // past 1,536 bytes: the completion's
        wave_lds_order();
        uint32_t Tc = T;
        bool at_end = last;
        if (!last && (((uint32_t) Bp + T) & 3u)) {
            // complete the range's last group from the characters after it
            bool ok = re + lane < n;
            for (uint64_t q = re;;) {
                const uint32_t t = ok ? la : 0xFFu;  // a table value (4 v, or 0xFF)
                const bool v = (t & 3u) == 0;
                const uint64_t m = __ballot(v);
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t) (m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
                const uint32_t need = 4u - (((uint32_t) Bp + Tc) & 3u);
                if (v && rank < need) or_field<true>(bits, 32 * dl + 6 * (Tc + rank), t << 24);
                const uint32_t got = (uint32_t) __popcll(m);
                if (got >= need) {
                    Tc += need;
                    break;
                }
                Tc += got;
                q += 64;
                if (q >= n) {
                    at_end = true;
                    break;
                }
                ok = q + lane < n;
                la = ok ? sm.tab[in[q + lane]] : 0xFFu;
            }
            wave_lds_order();
        }
        if (Tc > k) {
            const uint32_t Tk = Tc - k;
            const uint32_t rem = Tk & 3u;
            const uint32_t tail = at_end && !hold && rem >= 2 ? rem - 1 : 0u;
            store_window_bits(bits, 32 * dl + 6 * k, 3 * (Tk >> 2) + tail, dst);
        }
        wave_lds_order();
    };

    // Tile A (decoded, published, held: HA, LA, counts in s_cnt[bA]) is
    // stored after tile B is drawn, decoded and published, so that A's
    // predecessors have had a whole tile's time to publish.
    // (LA: the bytes after each held range, byte j for range j)
    uint32_t HA[HP][6];
    uint32_t LA = 0;
    static_assert(HP <= 4, "one byte per held range in LA");
#pragma unroll
    for (uint32_t j = 0; j < HP; j++) {
#pragma unroll
        for (int i = 0; i < 6; i++) HA[j][i] = 0;
    }
    block_sync();  // the tables
    bool haveA = false, owner = false;
    uint32_t tA = 0, bA = 1, bB = 0;
    Cnt Vs = 0;
    if (threadIdx.x == 0) s_tile[0] = atomicAdd(w.fticket, 1u);
    for (;;) {
        block_sync();  // the ticket; s_cnt[bB] (two tiles back) consumed
        const uint32_t tB = s_tile[bB];
        const bool haveB = tB < ntiles;
        if (!haveA && !haveB) break;
        uint32_t HB[HP][6];
        uint32_t LB = 0;
        if (haveB) {
            const uint32_t rwB = r0 + tB * TILE + wv * HP;
            if (whole(rwB)) fetch(rwB, 0);
            uint32_t lan = la_load(rwB);
#pragma unroll
            for (uint32_t j = 0; j < HP; j++) {
                uint32_t lan_next = 0;
                decode_one(rwB, j, bB, HB[j], lan, lan_next);
                LB |= lan << (8 * j);
                lan = lan_next;
            }
        }
        block_sync();  // s_cnt[bB] complete
        if (haveB && threadIdx.x == 0) publish(tB, bB);
        if (haveA) {
            // (every wave taking the prefix itself, no barrier: 841 against
            // 780 us, profiles/r05_ab_sfx_held_wavepfx.jsonl)
            if (wv == 0) {
                const Cnt ex = tA ? prefix(tA) : (Cnt) 0;
                if (lane == 0) s_excl = ex;
            }
            block_sync();
            const Cnt exw = s_excl;
            Cnt Bp = exw;
            for (uint32_t i = 0; i < wv * HP; i++) Bp += s_cnt[bA][i];
            const uint32_t rwA = r0 + tA * TILE + wv * HP;
#pragma unroll
            for (uint32_t j = 0; j < HP; j++) {
                if (rwA + j < nranges) {
                    const uint32_t T = s_cnt[bA][wv * HP + j];
                    store_one(rwA + j, Bp, T, HA[j], (uint32_t) (LA >> (8 * j)) & 0xFFu);
                    Bp += T;
                }
            }
            if (tA == ntiles - 1) {
                owner = true;
                Vs = exw;
                for (uint32_t i = 0; i < TILE; i++) Vs += s_cnt[bA][i];
            }
        }
        if (!haveB) break;
        LA = LB;
#pragma unroll
        for (uint32_t j = 0; j < HP; j++) {
#pragma unroll
            for (int i = 0; i < 6; i++) HA[j][i] = HB[j][i];
        }
        haveA = true;
        tA = tB;
        bA = bB;
        bB ^= 1u;
        // (drawn right after the publish instead, its round trip under the
        // stores: 762 against 730 us, profiles/r05_ab_sfx_early_draw.jsonl --
        // the tile then starts later and its successors wait)
        if (threadIdx.x == 0) s_tile[bB] = atomicAdd(w.fticket, 1u);
    }
    // (s_tile[bB]: the block's last ticket, read at the loop's last pass)
    if (WHOLE && hint && s_tile[bB] == ntiles) {
        // the hinted single pass's probe, in the first block that drew no
        // tile (ticket ntiles: exactly one block), while the others finish
        // theirs -- not a launch of its own after the decode (3.7 us and a
        // kernel boundary on every hinted call)
        __shared__ ProbeSmem ps;
        probe_stream(ps, in, n, a, ws, nranges, hint, key, 0u);
    }
    block_sync();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(w.wdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!owner || wv != 0) return;
    const uint64_t V = Vb + Vs;
    if (lane == 0) write_result(res, hres, V, hold, n, seq);
    find_tail_sextets<true>(sm.tab, in, n, V, res, hres);
    if (lane == 0) {
        while (__hip_atomic_load(w.wdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gridDim.x)
            __builtin_amdgcn_s_sleep(1);
    }
    for (uint32_t i = lane; i < ntiles; i += 64) st_store(&w.fstatus[i], 0);
    for (uint32_t i = lane; i < (ntiles + kSfxGroup - 1) / kSfxGroup; i += 64) st_store(&w.fsuper[i], 0);
    if (lane == 0) {
        __hip_atomic_store(w.fticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w.wdone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t i = 0; i < kFailWords; i++) w.lfail[i * kFailStride] = 0;
        *w.fail_any = 0;
    }
}

// Batches: buffer b is in[ioff(b) .. +len(b)) -> out + ooff(b).
struct BatchLayout {
    const uint64_t *in_off;   // nbuf+1 offsets, or null for a uniform stride
    const uint64_t *out_off;  // nbuf offsets, or null
    uint64_t in_stride, out_stride, len;
    uint64_t big;             // ragged: jobs of >= big characters are skipped (0: none)
    const uint8_t *flags;     // ragged: jobs flagged B64X_LANE_CHAINED are skipped too
};

DEV void batch_buf(const BatchLayout &L, uint32_t b, uint64_t &beg, uint64_t &len,
                   uint64_t &obeg)
{
    if (L.in_off) {
        beg = L.in_off[b];
        len = L.in_off[b + 1] - beg;
        obeg = L.out_off[b];
        // decoded by the single-buffer pipeline: big and chained jobs
        if ((L.big && len >= L.big) || (L.flags && (L.flags[b] & B64X_LANE_CHAINED))) len = 0;
    } else {
        beg = (uint64_t) b * L.in_stride;
        len = L.len;
        obeg = (uint64_t) b * L.out_stride;
    }
}

constexpr uint64_t kNeedsExact = ~0ull;

// Up to 16 characters of a lane from src[p..] within [0, len): one
// dwordx4 (non-temporal) when the lane's 16 are present and dword aligned.
DEV uint4 load_lane(const uint8_t *src, uint64_t p, uint64_t len, bool aligned, uint32_t &nin)
{
    nin = p >= len ? 0u : (len - p >= 16 ? 16u : (uint32_t) (len - p));
    if (nin == 16 && aligned) return ld16<true>(src + p);
    return nin ? load_chars(src + p, nin) : make_uint4(0, 0, 0, 0);
}

// Batch decode, fast paths only.  Persistent waves walk buffers b, b+W,
// ... two chunks ("a pair") at a time; the loads of the next pair -- of
// this buffer, or the first pair of the next one -- are issued before the
// current pair is decoded, so small buffers do not each pay a full memory
// latency.  A buffer any of whose chunks needs the exact path is marked in
// outlen[] for the fix-up.  RV: outlen[] receives the alphabet count V
// instead of floor(6V/8) bytes (the hub's jobs, k_batch_finish).
template <bool RV>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1)))
void k_decode_batch_fast(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, BatchLayout L,
    uint32_t nbuf, uint64_t *__restrict__ outlen, DecAlpha a)
{
    __shared__ uint8_t tab[256];
    build_dec_table(tab, a);
    block_sync();
    const uint32_t lane = lane_id();
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    uint32_t b = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (b >= nbuf) return;
    uint64_t beg, len, obeg;
    batch_buf(L, b, beg, len, obeg);
    bool aligned = ((((uintptr_t) (in + beg)) | ((uintptr_t) (out + obeg))) & 3) == 0;
    uint32_t nin[2];
    uint4 w[2];
    w[0] = load_lane(in + beg, 16 * lane, len, aligned, nin[0]);
    w[1] = load_lane(in + beg, kChunk + 16 * lane, len, aligned, nin[1]);
    uint64_t pos = 0, V = 0;
    bool ok = true;
    for (;;) {
        // issue the next pair's loads
        const bool more_here = pos + 2 * kChunk < len;
        const uint32_t bn = b + nw;
        uint64_t nbeg = beg, nlen = len, nobeg = obeg, npos = pos + 2 * kChunk;
        if (!more_here && bn < nbuf) {
            batch_buf(L, bn, nbeg, nlen, nobeg);
            npos = 0;
        }
        const bool naligned = ((((uintptr_t) (in + nbeg)) | ((uintptr_t) (out + nobeg))) & 3) == 0;
        uint32_t nnin[2] = {0, 0};
        uint4 nw4[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
        if (more_here || bn < nbuf) {
            nw4[0] = load_lane(in + nbeg, npos + 16 * lane, nlen, naligned, nnin[0]);
            nw4[1] = load_lane(in + nbeg, npos + kChunk + 16 * lane, nlen, naligned, nnin[1]);
        }
        // decode the current pair of buffer b
        uint8_t *dst = out + obeg;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint64_t cpos = pos + (uint64_t) u * kChunk;
            if (!ok || cpos >= len) break;
            uint32_t G[4], bad;
            map_fast(tab, w[u], nin[u], G, bad);
            if (__all(bad == 0)) {
                if (aligned) emit_full_a4<true>(G, dst + cpos / 4 * 3);
                else emit_full(G, dst + cpos / 4 * 3);
                V += kChunk;
                continue;
            }
            LaneChunk lc;
            map_chunk(tab, w[u], nin[u], lc);
            int got = cpos + kChunk >= len ? fast_prefix(lc, false, dst + cpos / 4 * 3) : -1;
            if (got < 0) ok = false;
            else V += (uint32_t) got;
        }
        if (more_here && ok) {
            pos = npos;
        } else {
            if (lane == 0) outlen[b] = ok ? (RV ? V : V * 6 / 8) : kNeedsExact;
            if (bn >= nbuf) break;
            bool fresh_aligned = naligned;
            if (more_here) {
                // buffer b was abandoned early (marked): what was loaded is
                // its next pair, not the next buffer's first pair
                batch_buf(L, bn, nbeg, nlen, nobeg);
                fresh_aligned = ((((uintptr_t) (in + nbeg)) | ((uintptr_t) (out + nobeg))) & 3) == 0;
                nw4[0] = load_lane(in + nbeg, 16 * lane, nlen, fresh_aligned, nnin[0]);
                nw4[1] = load_lane(in + nbeg, kChunk + 16 * lane, nlen, fresh_aligned, nnin[1]);
            }
            b = bn;
            beg = nbeg;
            len = nlen;
            obeg = nobeg;
            aligned = fresh_aligned;
            pos = 0;
            V = 0;
            ok = true;
        }
        w[0] = nw4[0];
        w[1] = nw4[1];
        nin[0] = nnin[0];
        nin[1] = nnin[1];
    }
}

// Uniform-stride batch decode, flattened: lane slot t = (buffer t / S,
// 16-character slot t mod S), S = slots per buffer.  Interior slots must
// be all alphabet (12 bytes out); the last slot of a buffer takes the
// prefix shape of a padded or unaligned end (fast_prefix's rule, per lane)
// and publishes the buffer's length.  Any other slot marks the buffer.
// Both go through atomicMax on outlen[] (zeroed by the launcher), so a mark
// always wins; the fix-up then decodes marked buffers exactly.
template <int U>
__global__ __launch_bounds__(kThreads) void k_decode_slots(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint64_t len,
    uint8_t *__restrict__ out, uint64_t out_stride,
    unsigned long long *__restrict__ outlen, uint32_t S, uint32_t total_slots, DecAlpha a)
{
    __shared__ uint8_t tab[256];
    build_dec_table(tab, a);
    block_sync();
    uint4 w[U];
    uint32_t nin[U], bq[U][2];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t t = (blockIdx.x * U + u) * kThreads + threadIdx.x;
        nin[u] = 0;
        bq[u][0] = bq[u][1] = 0;
        w[u] = make_uint4(0, 0, 0, 0);
        if (t < total_slots) {
            const uint32_t b = t / S, q = t - b * S;
            bq[u][0] = b;
            bq[u][1] = q;
            const uint8_t *src = in + (uint64_t) b * in_stride + (uint64_t) q * 16;
            const uint64_t avail = len - (uint64_t) q * 16;
            nin[u] = avail >= 16 ? 16u : (uint32_t) avail;
            if (nin[u] == 16 && (((uintptr_t) src) & 3) == 0) w[u] = ld16<true>(src);
            else w[u] = load_chars(src, nin[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (!nin[u]) continue;
        const uint32_t b = bq[u][0], q = bq[u][1];
        uint8_t *dst = out + (uint64_t) b * out_stride + (uint64_t) q * 12;
        uint32_t G[4], bad;
        map_fast(tab, w[u], nin[u], G, bad);
        uint32_t nbytes = 12, k = 16;
        bool ok = bad == 0;
        if (!ok && q == S - 1) {
            LaneChunk lc;
            map_chunk(tab, w[u], nin[u], lc);
            const uint32_t m = lc.vmask;
            ok = (m & (m + 1)) == 0;  // alphabet characters form a prefix
            k = __popc(m);
            nbytes = 3 * (k >> 2) + ((6 * (k & 3)) >> 3);
#pragma unroll
            for (int g = 0; g < 4; g++) G[g] = lc.G[g];
        }
        if (ok) {
            uint32_t o0, o1, o2;
            groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
            if (nbytes == 12 && (((uintptr_t) dst) & 3) == 0) {
                __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, (u32x3a4 *) dst);
            } else if (nbytes) {
                store_bytes12(dst, o0, o1, o2, nbytes);
            }
            if (q == S - 1)
                atomicMax(&outlen[b], (unsigned long long) ((16ull * q + k) * 6 / 8));
        } else {
            atomicMax(&outlen[b], (unsigned long long) kNeedsExact);
        }
    }
}

// The last slot of a row (its nlast = 1..16 characters in range) under
// the prefix rule of a padded or unaligned end: on return G holds the
// groups with out-of-prefix characters zeroed, k the prefix length, and
// the result says whether the shape applies.  Common shape first: every
// dword before d (the dword holding the last in-range character, uniform)
// all alphabet (A[g] < 64) and d's in-range characters an alphabet prefix
// -- 4 lookups; anything else takes the general per-character rule.
DEV bool row_last_slot(const uint8_t *tab, uint4 w, const uint32_t A[4], uint32_t G[4],
                       uint32_t nlast, uint32_t &k)
{
    const uint32_t d = (nlast - 1) >> 2;
    bool pre = true;
#pragma unroll
    for (uint32_t g = 0; g < 3; g++)
        if (g < d) pre = pre && A[g] < 64u;
    const uint32_t wd = d == 0 ? w.x : d == 1 ? w.y : d == 2 ? w.z : w.w;
    uint32_t v = 0, Gd = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t t = tab[(wd >> (8 * j)) & 0xFFu];
        const bool okj = 4 * d + j < nlast && t < 64u;
        v |= (okj ? 1u : 0u) << j;
        Gd |= (okj ? t : 0u) << (18 - 6 * j);
    }
    if (pre && (v & (v + 1)) == 0) {
        k = 4 * d + __popc(v);
#pragma unroll
        for (uint32_t g = 0; g < 4; g++)
            if (g == d) G[g] = Gd;
        return true;
    }
    LaneChunk lc;
    map_chunk_lds(tab, w, nlast, lc);
    const uint32_t m = lc.vmask;
    k = __popc(m);
#pragma unroll
    for (int g = 0; g < 4; g++) G[g] = lc.G[g];
    return (m & (m + 1)) == 0;  // alphabet characters form a prefix
}

// ---- line-structured rows ---------------------------------------------------
//
// Uniform-stride batch decode of rows with room (out_stride >= 12 S), with
// k_decode_lines' line model (MIME-formatted batches:
// every row in 76-character lines with CRLF).  The model is probed from the
// batch's first row by k_rows_prep (which also zeroes the failure bitmap)
// and applies to every row; a row that does not follow it fails a
// check and is marked for the fix-up, which decodes it exactly.  Row slot q
// owns the row's sextets [16q, 16q + 16) and their span; slots before the
// row's last are checked strictly (16 alphabet characters, separator bytes
// outside the alphabet), the last one by the prefix rule of a padded or
// unaligned end (its model positions: alphabet characters, then only
// others; any trailing separator bytes outside the alphabet).
struct RowModel {
    uint32_t L, s, P, rcp;  // the line model; L = 0: clean rows (k_decode_rows2's path)
    uint32_t S;             // slots per row under the model
    uint32_t magic;         // ceil(2^32 / S), exact for the kernel's offsets
    uint64_t m64;           // ceil(2^64 / S)
    uint32_t F;             // model positions per row
    uint32_t m, k;          // i / L == (i * m) >> (31 + k)
    uint32_t mL;            // ceil(2^32 / L): i / L == umulhi(i, mL) for i < 2^24
    uint32_t j0;            // alphabet characters in a passing row's last slot (row 0's);
                            // kNoRowShape: no row passes (every row is decoded exactly)
    uint32_t rcpS;          // ceil(2^20 / S) when rel / S == umul24(rel, rcpS) >> 20 for every
                            // slot offset of a block (and, for line-structured rows,
                            // 16 S <= 4,096: the 20-bit line division), else 0
    uint64_t len0;          // output bytes of a passing row: floor(6 (16 (S - 1) + j0) / 8)
    uint32_t Sx;            // slots per row of the line-structured hot path: S, or
                            // out_stride / 12 when that is whole (slots from S on store
                            // only filler, so consecutive rows' writes are contiguous)
    uint32_t pad;
    uint64_t m64x;          // ceil(2^64 / Sx)
    // Row-group mapping of the line-structured hot path (k_decode_rows_lines):
    // a lane keeps one row slot q for all its U slots, which
    // lie in rows Ru apart; NB blocks of kThreads lanes cover Ru rows' Sx
    // slots (NB kThreads = Ru Sx = lcm(kThreads, Sx)), so the line position
    // of q is computed once per lane, not once per slot.
    uint32_t nb, ru;        // blocks per row band, rows per band
    uint32_t mx;            // ceil(2^32 / Sx): exact for slot offsets below NB kThreads
    uint32_t rg;            // 1: the mapping applies
};
static_assert(sizeof(RowModel) == 96, "RowModel layout");
constexpr uint32_t kNoRowShape = 0xFFFFFFFFu;

// The library workspace of the stream holds the rows' failure bitmap in the
// region pass 1 uses for its per-range counts (scratch between calls; bit b
// set when row b must be decoded exactly), and the model past the end of the
// decode workspace proper, where no other kernel writes: the model of the
// stream's last row batch stays there for the next one of the same shape.
DEV unsigned long long *row_fail(void *ws)
{
    return (unsigned long long *) ((uint8_t *) ws + kWsScratch + sizeof(RowModel));
}

constexpr uint32_t kRowsU = 4;  // slots per lane of the row kernels


// The groups and the invalid mask (x 128, bits 7..22) of 16 characters by
// packed table values: groups by v_dot4 of their low 6 bits (a non-alphabet
// character contributes 63 inside its own field), the mask by v_dot4 of the
// bit 7s.
DEV void map_row_dot4(const uint8_t *tab, uint4 d, uint32_t G[4], uint32_t &m128)
{
    const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
    m128 = 0;
#pragma unroll
    for (int g = 0; g < 4; g++) {
        const uint32_t P = tab_pack4(tab, dw[g]);
        const uint32_t Pz = P & 0x3F3F3F3Fu;
        G[g] = (__builtin_amdgcn_udot4(Pz, 0x00000140u, 0u, false) << 12) |
               __builtin_amdgcn_udot4(Pz, 0x01400000u, 0u, false);
        const uint32_t w = (g & 1) ? 0x80402010u : 0x08040201u;
        const uint32_t part = __builtin_amdgcn_udot4(P & 0x80808080u, w, 0u, false);
        m128 += (g & 2) ? part << 8 : part;
    }
}

// One slot of a line-structured row: its 16 model characters from the
// window at its span, checked strictly (interior) or by the prefix rule
// (the row's last slot, k model positions, nspan bytes of span); returns
// whether it passes, G the groups (out-of-prefix characters zeroed), *j the
// alphabet characters taken.
DEV bool row_lines_slot(const uint8_t *tab, const RowModel &rm, const uint32_t w6[6], uint32_t o,
                        uint32_t col, bool last, uint32_t k, uint32_t nspan, uint32_t G[4],
                        uint32_t *j)
{
    const uint32_t L = rm.L, s = rm.s;
    const bool hs = L - col <= 16;
    const uint32_t c = hs ? L - col : 16u;
    uint32_t sep;
    const uint4 d = (L & 3) == 0 ? slot_chars4(w6, o, c >> 2, s, &sep)
                                 : slot_chars(w6, o, c, s, &sep);
    // separator bytes inside the span that must be outside the alphabet
    const uint32_t nsep = !hs ? 0u : !last ? s : c > k ? 0u : (nspan - c < s ? nspan - c : s);
    const uint32_t need = sep_need(nsep);
    const bool sep_alpha = (sep_nonalpha(tab, sep) & need) != need;
    // interior slots: all 16 alphabet; the last: the alphabet characters of
    // its k model positions form a prefix (one rule, no branch: k = 16 for
    // interior slots makes it "all 16")
    uint32_t im;
    map_row_slot(tab, d, G, im);
    const uint32_t kk = last ? k : 16u;
    const uint32_t mk = ~im & (kk >= 16 ? 0xFFFFu : (1u << kk) - 1u);
    *j = __popc(mk);
    const bool shape = last ? (mk & (mk + 1)) == 0 : im == 0;
    return shape && !sep_alpha;
}

// Rows with room (out_stride >= 12 S), one pass over the row slots, the
// lengths written afterwards (k_rows_finish):
//   k_rows_prep   zeroes the failure bitmap and, in one wave, probes the line
//                 model from row 0 and decodes row 0's last slot: its
//                 alphabet count j0 is the shape every passing row's last slot
//                 must have, so a passing row's length is known in advance
//                 (skipped when the workspace holds the model of a batch of
//                 the same shape: b64x_decode_strided);
//   k_decode_rows_lines  checks and decodes every slot, marking a row that
//                 does not pass (one atomicOr of its bit, by the first failing
//                 lane of the row in the wave; no per-row atomics otherwise);
//   k_rows_finish writes every row's length with coalesced stores and decodes
//                 the marked rows exactly.
// (Round 2 zeroed outlen[] and took every row's length by an atomicMax from
// the lane of its last slot: 1 M scattered 8-byte atomics per batch of 1 M
// rows, 1.09x the output's write traffic, profiles/r02_pmc_rows32_crlf76.json.)
__global__ __launch_bounds__(kThreads) void k_rows_prep(
    uint32_t nbuf, const uint8_t *__restrict__ in, uint32_t len, uint64_t in_stride, uint32_t S,
    uint64_t out_stride, DecAlpha a, void *ws, RowModel *rmodel)
{
    unsigned long long *bm = row_fail(ws);
    const uint32_t nw = (nbuf + 63) / 64;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < nw; i += gridDim.x * kThreads)
        bm[i] = 0;
    if (blockIdx.x != 0) return;
    __shared__ uint8_t tab[256];
    build_dec_table(tab, a);
    block_sync();
    if (threadIdx.x >= 64) return;
    const LineModel lm = probe_lines(tab, in, len);
    RowModel r{};
    const uint32_t L = lm.L, s = lm.s, P = L + s;
    if (L) {
        const uint32_t F = len / P * L + (len % P < L ? len % P : L);
        const uint32_t Sm = (F + 15) / 16;
        const uint32_t magic = (uint32_t) ((0xFFFFFFFFull + Sm) / Sm);
        const uint64_t e = (uint64_t) magic * Sm - (1ull << 32);
        const uint64_t relmax = Sm + (uint64_t) kRowsU * kThreads;
        // (rows of at least 32 bytes: a window never reads more than 24
        // bytes past a row start beyond the next row's)
        if (Sm >= 2 && len >= 32 && relmax * e < (1ull << 32) &&
            (relmax / Sm + 1) * in_stride < (1ull << 40)) {
            r.L = L;
            r.s = s;
            r.P = P;
            r.rcp = ((1u << 20) + L - 1) / L;
            r.S = Sm;
            r.magic = magic;
            r.m64 = ~0ull / Sm + 1;
            r.F = F;
            r.k = 32 - __builtin_clz(L - 1);
            r.m = (uint32_t) ((((uint64_t) 1 << (31 + r.k)) + L - 1) / L);
            // exact for i < 16 S <= 2^24: i (mL L - 2^32) < 2^24 * 252 < 2^32
            r.mL = (uint32_t) ((0xFFFFFFFFull + L) / L);
        }
    }
    // row 0's last slot: the shape of every passing row's
    uint32_t j0 = kNoRowShape;
    const uint32_t Sr = r.L ? r.S : S;
    if (r.L) {
        const uint32_t i = 16 * (Sr - 1), k = r.F - i;
        const uint32_t dl = i / L, col = i - dl * L, pos = dl * P + col;
        const uint8_t *ab = in + (pos & ~3u);
        const uint8_t *end = in + len;
        const uint4 w = load_win16(ab, end);
        const uint2 x = load_win8(ab + 16, end);
        const uint32_t w6[6] = {w.x, w.y, w.z, w.w, x.x, x.y};
        uint32_t G[4], j;
        if (row_lines_slot(tab, r, w6, pos & 3u, col, true, k, len - pos, G, &j)) j0 = j;
    } else {
        const uint32_t nlast = len - 16 * (Sr - 1);
        const uint4 w = load_chars(in + 16 * (Sr - 1), nlast);
        uint32_t G[4], A[4], k = 16;
        map_fast_acc(tab, w, G, A);
        if (row_last_slot(tab, w, A, G, nlast, k)) j0 = k;
    }
    r.j0 = j0;
    r.len0 = j0 == kNoRowShape ? 0 : (16ull * (Sr - 1) + j0) * 6 / 8;
    // Line-structured rows use fewer slots per row (the model's S) than the
    // characters would (the launcher's S); when the output stride is whole
    // slots, the hot path takes that many per row (at most the launcher's)
    // and fills the slack, so no row leaves a hole between its bytes and the
    // next row's (a hole makes every row's last line a partial write).
    r.Sx = r.L && out_stride % 12 == 0
               ? (out_stride / 12 < S ? (uint32_t) (out_stride / 12) : S) : Sr;
    const uint32_t Sq = r.L ? r.Sx : Sr;
    r.m64x = ~0ull / r.Sx + 1;
    // the 24-bit slot mapping: rel < Sq + U x 256 for every lane slot of a
    // block; rel / Sq exact as (rel * rcpS) >> 20 iff rel (rcpS Sq - 2^20) < 2^20
    const uint32_t rS = ((1u << 20) + Sq - 1) / Sq;
    const uint64_t relmax = Sq + (uint64_t) kRowsU * kThreads;
    if ((!r.L || 16ull * Sr <= 4096) && relmax * ((uint64_t) rS * Sq - (1u << 20)) < (1u << 20))
        r.rcpS = rS;
    if (r.L && r.Sx < 4096) {
        const uint32_t g = (r.Sx & (0u - r.Sx)) < kThreads ? (r.Sx & (0u - r.Sx)) : kThreads;
        r.nb = r.Sx / g;          // Sx / gcd(Sx, kThreads)
        r.ru = kThreads / g;      // kThreads / gcd(Sx, kThreads)
        r.mx = (uint32_t) ((0xFFFFFFFFull + r.Sx) / r.Sx);
        // 32-bit lane offsets within a band (rin < ru rows), 24-bit products
        r.rg = (uint64_t) kRowsU * r.ru * in_stride + len + 32 < (1ull << 31) &&
               (uint64_t) kRowsU * r.ru * out_stride < (1ull << 31) && in_stride < (1u << 24) &&
               out_stride < (1u << 24);
    }
    if (threadIdx.x == 0) *rmodel = r;
}

// The row kernel.  Clean rows (the model's L = 0): the block's first slot
// gives its row b0 and slot q0 once, each lane's slot is a 32-bit offset
// from there split with a 32-bit multiply-high (magic = ceil(2^32/S), exact
// in range -- the launcher checks); lane slots load 16 characters and store
// 12 bytes unconditionally (the last slot of a row over-writes past its
// length inside its own row).  Line-structured rows: the same shape with the
// model's S and each slot's span (row_lines_slot); when the model allows
// (rcpS), the slot mapping and the line division are 24-bit products, as in
// k_decode_lines (a 32-bit multiply issues at a quarter of the VALU rate).
// A slot passes when it is all alphabet (interior) or when its alphabet
// characters are a prefix as long as row 0's last slot's (the last; j0, the
// prep's) -- then the row's length is the prep's len0.  The first failing
// lane of a row in the wave sets the row's bit for the exact decode
// (k_rows_finish); nothing else is written per row.  Blocks that touch the
// last row ("tail", block-uniform) read page-safely and store only decoded
// bytes, so one launch covers the batch.

// Mark the rows of this u-step's failing lanes: the first failing lane of
// each row among the wave's lanes (rows are contiguous runs of lanes: lane
// l's slot q = l - (its row's first lane)).  Wave-uniform call.
DEV void mark_failed_rows(unsigned long long *bm, uint64_t junk, uint32_t q, uint64_t row)
{
    const uint32_t ln = lane_id();
    const uint32_t rs = q < ln ? ln - q : 0u;
    const uint64_t row_junk = junk & (~0ull << rs);
    if ((junk >> ln) & 1 && (uint32_t) __ffsll((unsigned long long) row_junk) - 1 == ln)
        atomicOr(bm + (row >> 6), 1ull << (row & 63));
}

template <int U, bool O32>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1)))
void k_decode_rows_lines(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint32_t len,
    uint8_t *__restrict__ out, uint64_t out_stride, uint32_t S, uint32_t magic, uint64_t m64,
    uint64_t nslots, uint64_t tail_slot, DecAlpha a, uint32_t nbuf, void *ws,
    const RowModel *rmodel)
{
    __shared__ uint8_t tab[256];
    const uint64_t *rmw = (const uint64_t *) rmodel;
    const uint64_t r0 = scalar_load_u64(rmw), r6 = scalar_load_u64(rmw + 6);
    unsigned long long *bm = row_fail(ws);
    // (the row bands' spare blocks leave after the table build: tested
    // before it, the model's loads no longer overlapped the build and MIME
    // rows ran 481.6 -> 499.2 us, profiles/r04_ab_rows_early_exit.jsonl)
    build_dec_table(tab, a);
    block_sync();
    const uint32_t j0 = (uint32_t) r6, rcpS = (uint32_t) (r6 >> 32);
    if ((uint32_t) r0 != 0) {
        RowModel rm;
        const uint64_t r1 = scalar_load_u64(rmw + 1), r2 = scalar_load_u64(rmw + 2),
                       r3 = scalar_load_u64(rmw + 3), r4 = scalar_load_u64(rmw + 4),
                       r5 = scalar_load_u64(rmw + 5);
        rm.L = (uint32_t) r0;
        rm.s = (uint32_t) (r0 >> 32);
        rm.P = (uint32_t) r1;
        rm.rcp = (uint32_t) (r1 >> 32);
        rm.S = (uint32_t) r2;
        rm.magic = (uint32_t) (r2 >> 32);
        rm.m64 = r3;
        rm.F = (uint32_t) r4;
        rm.m = (uint32_t) (r4 >> 32);
        rm.k = (uint32_t) r5;
        rm.mL = (uint32_t) (r5 >> 32);
        const uint32_t Sm = rm.S;
        const uint64_t s0 = (uint64_t) blockIdx.x * U * kThreads;
        const uint32_t Sx = (uint32_t) scalar_load_u64(rmw + 8);
        const uint64_t r10 = scalar_load_u64(rmw + 10), r11 = scalar_load_u64(rmw + 11);
        if (O32 && rcpS && (rm.L & 3) == 0 && (uint32_t) (r11 >> 32)) {
            const uint32_t NB = (uint32_t) r10, Ru = (uint32_t) (r10 >> 32), mx = (uint32_t) r11;
            const uint32_t st = blockIdx.x / NB, bi = blockIdx.x - st * NB;  // scalar
            const uint64_t row_st = (uint64_t) st * (U * Ru);  // the block's first row
            if (row_st >= nbuf) return;
            // blocks with rows at or past the last: page-safe loads, decoded
            // bytes only (as below)
            const bool tail = row_st + U * Ru > nbuf - 1;
            const uint8_t *end = in + (uint64_t) (nbuf - 1) * in_stride + len;
            const uint32_t nb_last = j0 == kNoRowShape ? 0u : 3 * (j0 >> 2) + ((6 * (j0 & 3)) >> 3);
            const uint32_t kq = rm.F - 16 * (Sm - 1);
            const uint32_t iL = 16 * (Sm - 1), dL = iL / rm.L, colL = iL - dL * rm.L;
            const uint32_t cL = rm.L - colL < 16 ? rm.L - colL : 16u;
            const uint32_t spanL = len - (dL * rm.P + colL);
            const uint32_t nsepL = rm.L - colL > 16 || cL > kq ? 0u
                                 : (spanL - cL < rm.s ? spanL - cL : rm.s);
            const uint32_t need_L = sep_need(nsepL);
            const uint32_t kmask = 128u * (kq >= 16 ? 0xFFFFu : (1u << kq) - 1u);
            const uint32_t expm = j0 == kNoRowShape ? 1u : kmask & ~(128u * ((1u << j0) - 1u));
            // the lane's slot q and row in the band, once for its U slots
            const uint32_t F = bi * kThreads + threadIdx.x;  // < NB kThreads = Ru Sx
            const uint32_t rin = __umulhi(F, mx);
            const uint32_t q = F - __umul24(rin, Sx);
            const uint32_t i = 16 * (q < Sm ? q : Sm - 1);
            const uint32_t dl = __umul24(i, rm.rcp) >> 20;
            const uint32_t col = i - __umul24(dl, rm.L);
            const uint32_t pos = __umul24(dl, rm.P) + col;
            const uint32_t oo = pos & 3u;
            const bool last = q == Sm - 1;
            const bool hs = rm.L - col <= 16;
            const uint32_t c = hs ? rm.L - col : 16u;
            const uint32_t ioff = __umul24(rin, (uint32_t) in_stride) + (pos & ~3u);
            const uint32_t ooff = __umul24(rin, (uint32_t) out_stride) + __umul24(q, 12u);
            // one 64-bit base per block; every lane offset is 32-bit (the
            // prep checks U bands of rows span under 2^31 bytes), so the
            // loads and stores take a scalar base and a VGPR offset and the
            // per-band bases cost no SGPR pairs (they spilled to VGPR lanes)
            const uint8_t *ib = in + row_st * in_stride;
            uint8_t *ob = out + row_st * out_stride;
            const uint32_t ui = Ru * (uint32_t) in_stride, uo = Ru * (uint32_t) out_stride;
            // the separator bytes a slot must find outside the alphabet: the
            // line's s when a line ends in (or right after) the slot, the
            // last slot's own count -- lane-constant (every u-step has the
            // same q), so the check below is four lookups and a mask test,
            // no branch
            const uint32_t need_s = sep_need(rm.s);
            const uint32_t nd = last ? need_L : hs ? need_s : 0u;
            // Tail bands (rows at or past the last: page-safe loads, decoded
            // bytes only) apart from the hot path, as in the clean rows: joined,
            // the compiler merged the two per u-step and spilled SGPRs
            // (VERDICT r04 item 4).
            if (tail) {
                for (int u = 0; u < U; u++) {
                    const uint64_t row = row_st + u * Ru + rin;
                    const bool live = row < nbuf;
                    const uint8_t *ab = ib + (ioff + u * ui);
                    const uint4 wn = live ? load_win16(ab, end) : make_uint4(0, 0, 0, 0);
                    const uint2 wy = live ? load_win8(ab + 16, end) : make_uint2(0, 0);
                    const uint32_t w6[6] = {wn.x, wn.y, wn.z, wn.w, wy.x, wy.y};
                    uint32_t sep, G[4], m128;
                    const uint4 d = slot_chars4(w6, oo, c >> 2, rm.s, &sep);
                    map_row_dot4(tab, d, G, m128);
                    uint32_t bad = last ? (m128 & kmask) ^ expm : m128;
                    if ((sep_nonalpha(tab, sep) & nd) != nd) bad |= 1u;
                    if (q >= Sm || !live) bad = 0;  // slack filler: the bytes are scratch
                    uint32_t o0, o1, o2;
                    groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
                    if (live && q < Sm && bad == 0)
                        store_bytes12_rolled(ob + (ooff + u * uo), o0, o1, o2, last ? nb_last : 12u);
                    const uint64_t junk = __ballot(bad != 0);
                    if (junk) mark_failed_rows(bm, junk, q, row);
                }
                return;
            }
            uint4 win[U];
            uint2 wx[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint8_t *ab = ib + (ioff + u * ui);
                win[u] = load16_a4(ab);
                const u32x2a4 v = *(const u32x2a4 *) (ab + 16);
                wx[u] = make_uint2(v.x, v.y);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t w6[6] = {win[u].x, win[u].y, win[u].z, win[u].w, wx[u].x, wx[u].y};
                uint32_t sep, G[4], m128;
                const uint4 d = slot_chars4(w6, oo, c >> 2, rm.s, &sep);
                map_row_dot4(tab, d, G, m128);
                uint32_t bad = last ? (m128 & kmask) ^ expm : m128;
                if ((sep_nonalpha(tab, sep) & nd) != nd) bad |= 1u;
                if (q >= Sm) bad = 0;  // slack filler: the bytes are scratch
                uint32_t o0, o1, o2;
                groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
                __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, (u32x3a4 *) (ob + (ooff + u * uo)));
                // (one ballot per wave instead, as k_decode_lines: neutral
                // here, profiles/r05_ab_rows_defer.jsonl)
                const uint64_t junk = __ballot(bad != 0);
                if (junk) mark_failed_rows(bm, junk, q, row_st + u * Ru + rin);
            }
            return;
        }
        // (Round 2's slot-by-slot hot path for these rows, the fallback when
        // the row bands do not apply, was removed in round 3: with the bands
        // only oversized strides reached it, so every such batch now takes
        // the general path below.)
        const uint64_t ns_m = (uint64_t) Sm * nbuf;
        const uint64_t tail_m = (uint64_t) Sm * (nbuf - 1);
        if (s0 >= ns_m) return;
        const uint64_t b0 = __umul64hi(s0, rm.m64);
        const uint32_t q0 = (uint32_t) (s0 - b0 * Sm);
        const uint8_t *ib = in + b0 * in_stride;
        uint8_t *ob = out + b0 * out_stride;
        const bool tail = s0 + U * kThreads > tail_m;
        const uint8_t *end = in + (uint64_t) (nbuf - 1) * in_stride + len;
        uint32_t bl[U], qq[U], oo[U], cl[U], pp[U];
        uint4 win[U];
        uint2 wx[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t rel = q0 + u * kThreads + threadIdx.x;
            bl[u] = __umulhi(rel, rm.magic);
            qq[u] = rel - bl[u] * Sm;
            const uint32_t i = 16 * qq[u];
            const uint32_t dl = __umulhi(i, rm.mL);
            cl[u] = i - dl * rm.L;
            const uint32_t pos = dl * rm.P + cl[u];
            pp[u] = pos;
            oo[u] = pos & 3u;
            // O32: the block's rows lie within 2^31 bytes of its first and
            // the strides below 2^24 (the launcher checks), so offsets are
            // 32-bit from a uniform base and the products full-rate 24-bit
            const uint8_t *ab = O32 ? ib + (__umul24(bl[u], (uint32_t) in_stride) + (pos & ~3u))
                                    : ib + (uint64_t) bl[u] * in_stride + (pos & ~3u);
            if (!tail) {
                win[u] = load16_a4(ab);
                const u32x2a4 v = *(const u32x2a4 *) (ab + 16);
                wx[u] = make_uint2(v.x, v.y);
            } else {
                const bool live = s0 + u * kThreads + threadIdx.x < ns_m;
                win[u] = live ? load_win16(ab, end) : make_uint4(0, 0, 0, 0);
                wx[u] = live ? load_win8(ab + 16, end) : make_uint2(0, 0);
            }
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t q = qq[u];
            const bool last = q == Sm - 1;
            const uint32_t i = 16 * q;
            const uint32_t k = last ? rm.F - i : 16u;
            const uint32_t pos = pp[u];
            const uint32_t w6[6] = {win[u].x, win[u].y, win[u].z, win[u].w, wx[u].x, wx[u].y};
            uint32_t G[4], j;
            bool ok = row_lines_slot(tab, rm, w6, oo[u], cl[u], last, k, len - pos, G, &j);
            ok = ok && (!last || j == j0);
            uint32_t o0, o1, o2;
            groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
            uint8_t *dst = O32 ? ob + (__umul24(bl[u], (uint32_t) out_stride) + __umul24(q, 12u))
                               : ob + (uint64_t) bl[u] * out_stride + 12 * q;
            const bool live = !tail || s0 + u * kThreads + threadIdx.x < ns_m;
            if (!tail) {
                __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, (u32x3a4 *) dst);
            } else if (live && ok) {
                store_bytes12(dst, o0, o1, o2, last ? 3 * (j >> 2) + ((6 * (j & 3)) >> 3) : 12u);
            }
            const uint64_t junk = __ballot(live && !ok);
            if (junk) mark_failed_rows(bm, junk, q, b0 + bl[u]);
        }
        return;
    }
    // clean rows: k_decode_rows2's body
    const uint64_t s0 = (uint64_t) blockIdx.x * U * kThreads;
    const uint64_t b0 = __umul64hi(s0, m64);
    const uint32_t q0 = (uint32_t) (s0 - b0 * S);
    const uint8_t *ib = in + b0 * in_stride;
    uint8_t *ob = out + b0 * out_stride;
    const uint32_t nlast = len - 16 * (S - 1);  // characters in a row's last slot
    uint32_t bl[U], qq[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t rel = q0 + (u * kThreads + threadIdx.x);
        if (rcpS) {
            bl[u] = __umul24(rel, rcpS) >> 20;
            qq[u] = rel - __umul24(bl[u], S);
        } else {
            bl[u] = __umulhi(rel, magic);
            qq[u] = rel - bl[u] * S;
        }
    }
    if (s0 + U * kThreads > tail_slot) {
        // tail block: page-safe loads, decoded bytes only
        for (int u = 0; u < U; u++) {
            const uint64_t t = s0 + (u * kThreads + threadIdx.x);
            const uint32_t q = qq[u];
            const bool live = t < nslots;
            const bool last = q == S - 1;
            bool ok = true;
            uint32_t G[4], A[4], k = 16;
            if (live) {
                const uint4 wv = load_chars(ib + (uint64_t) bl[u] * in_stride + 16 * q,
                                            last ? nlast : 16u);
                map_fast_acc(tab, wv, G, A);
                ok = ((A[0] | A[1] | A[2] | A[3]) & ~63u) == 0;
                if (last) ok = row_last_slot(tab, wv, A, G, nlast, k) && k == j0;
                if (ok) {
                    uint32_t o0, o1, o2;
                    groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
                    store_bytes12(ob + (uint64_t) bl[u] * out_stride + 12 * q, o0, o1, o2,
                                  3 * (k >> 2) + ((6 * (k & 3)) >> 3));
                }
            }
            const uint64_t junk = __ballot(live && !ok);
            if (junk) mark_failed_rows(bm, junk, q, b0 + bl[u]);
        }
        return;
    }
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; u++)
        w[u] = ld16<true>(O32 ? ib + (__umul24(bl[u], (uint32_t) in_stride) + 16 * qq[u])
                              : ib + (uint64_t) bl[u] * in_stride + 16 * qq[u]);
    // the last slot's rule as a mask test (the band path's): bits 7.. of
    // the invalid mask over its nlast characters must be exactly those past
    // row 0's j0
    const uint32_t ckm = 128u * (nlast >= 16 ? 0xFFFFu : (1u << nlast) - 1u);
    const uint32_t cexp = j0 == kNoRowShape ? 1u : ckm & ~(128u * ((1u << j0) - 1u));
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint32_t q = qq[u];
        const bool last = q == S - 1;
        // packed table values: groups by v_dot4 of their low 6 bits (a
        // non-alphabet character contributes 63 inside its own field, past
        // a passing last slot's bytes), the invalid mask by v_dot4 of the
        // bit 7s; the row's last slot by a mask test, no branch (the
        // per-lane row_last_slot branch cost 6 us per config-4 batch,
        // profiles/r05_ab_rows_last.jsonl)
        const uint32_t dw[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
        uint32_t G[4], m128 = 0;
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t P = tab_pack4(tab, dw[g]);
            const uint32_t Pz = P & 0x3F3F3F3Fu;
            G[g] = (__builtin_amdgcn_udot4(Pz, 0x00000140u, 0u, false) << 12) |
                   __builtin_amdgcn_udot4(Pz, 0x01400000u, 0u, false);
            const uint32_t wt = (g & 1) ? 0x80402010u : 0x08040201u;
            const uint32_t part = __builtin_amdgcn_udot4(P & 0x80808080u, wt, 0u, false);
            m128 += (g & 2) ? part << 8 : part;
        }
        const bool ok = (last ? (m128 & ckm) ^ cexp : m128) == 0;
        uint32_t o0, o1, o2;
        groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
        uint8_t *dst = O32 ? ob + (__umul24(bl[u], (uint32_t) out_stride) + __umul24(q, 12u))
                           : ob + (uint64_t) bl[u] * out_stride + 12 * q;
        __builtin_nontemporal_store(u32x3a4{o0, o1, o2}, (u32x3a4 *) dst);
        const uint64_t junk = __ballot(!ok);
        if (junk) mark_failed_rows(bm, junk, q, b0 + bl[u]);
    }
}

// Batch fix-up, bit-stream form (k_decode_pass2d's machinery, one wave per
// marked buffer, no cross-wave prefix): the buffer's characters are taken
// 2,048 at a time; their sextets are OR-ed into the wave's LDS window as a
// bit stream; whole dwords are flushed to the output and the partial last
// dword moves to the window front.  A buffer of V alphabet characters
// yields floor(6V/8) bytes -- the reference's final partial group rule
// falls out of the bit count.
// First-step characters of a buffer (chunks 0 and 1 of lane `lane`).
DEV void buf_first_chunks(const uint8_t *src, uint64_t len, uint4 c[2])
{
    const uint32_t lane = lane_id();
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint64_t q = (uint64_t) h * kChunk + 16 * lane;
        const uint32_t nin = q >= len ? 0u : (len - q >= 16 ? 16u : (uint32_t) (len - q));
        c[h] = nin ? load_chars(src + q, nin) : make_uint4(0, 0, 0, 0);
    }
}

DEV uint64_t decode_buf_bits(const P2dSmem &sm, uint4 *bq, const uint8_t *src, uint64_t len,
                             uint8_t *dst, const uint4 first[2])
{
    const uint32_t lane = lane_id();
    uint32_t *bits = (uint32_t *) bq;
    const uint32_t skew = (uint32_t) ((uintptr_t) dst & 3);
    uint32_t lo = 4 + skew;   // LDS byte of output byte `done`
    uint32_t pb = 8 * lo;     // next free bit of the window
    uint64_t done = 0, V = 0;
    bq[lane] = make_uint4(0, 0, 0, 0);
    if (lane + 64 < kP2dBlocks) bq[lane + 64] = make_uint4(0, 0, 0, 0);
    wave_lds_order();
    for (uint64_t p = 0;; p += 2 * kChunk) {
        uint4 ch[2];
        uint32_t nh[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const uint64_t q = p + (uint64_t) h * kChunk + 16 * lane;
            nh[h] = q >= len ? 0u : (len - q >= 16 ? 16u : (uint32_t) (len - q));
            ch[h] = p == 0 ? first[h]
                  : nh[h] ? load_chars(src + q, nh[h]) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t got = bits_step(sm, bits, ch, nh, (int) pb);
        pb += 6u * got;
        V += got;
        wave_lds_order();
        const bool last = p + 2 * kChunk >= len;
        if (last) {
            store_bits(bits, lo, pb >> 3, dst + done - lo);
            break;
        }
        // flush the whole dwords; the partial one becomes dword 1
        const uint32_t kcut = (pb >> 3) & ~3u;
        store_bits(bits, lo, kcut, dst + done - lo);
        done += kcut - lo;
        const uint32_t keep = bits[kcut >> 2];
        wave_lds_order();
        bq[lane] = make_uint4(0, 0, 0, 0);
        if (lane + 64 < kP2dBlocks) bq[lane + 64] = make_uint4(0, 0, 0, 0);
        wave_lds_order();
        if (lane == 0) bits[1] = keep;
        wave_lds_order();
        pb -= 8 * (kcut - 4);
        lo = 4;
    }
    wave_lds_order();  // the next buffer re-zeroes the window
    return V;
}

template <bool RV>
__global__ __launch_bounds__(kThreads) void k_decode_batch_fix2(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, BatchLayout L,
    uint32_t nbuf, uint64_t *__restrict__ outlen, DecAlpha a)
{
    __shared__ P2dSmem sm;
    build_dec_table(sm.tab, a);
    build_compact_sel(sm.sel);
    block_sync();
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t) gridDim.x * kWavesPerBlock;
    for (uint64_t base = ((uint64_t) blockIdx.x * kWavesPerBlock + wv) * 64; base < nbuf;
         base += nw * 64) {
        const uint64_t bl = base + lane;
        uint64_t m = __ballot(bl < nbuf && outlen[bl] == kNeedsExact);
        while (m) {
            const uint32_t b = (uint32_t) (base + __ffsll((unsigned long long) m) - 1);
            m &= m - 1;
            uint64_t beg, len, obeg;
            batch_buf(L, b, beg, len, obeg);
            uint4 c[2];
            buf_first_chunks(in + beg, len, c);
            const uint64_t V = decode_buf_bits(sm, sm.bits[wv], in + beg, len, out + obeg, c);
            if (lane == 0) outlen[b] = RV ? V : V * 6 / 8;
        }
    }
}

// Row lengths after k_decode_rows_lines: one wave per 64 rows (one bitmap
// word, read through the scalar cache and cleared for the next batch), every
// unmarked row's length (the model's len0) by one coalesced store per lane,
// then the marked rows decoded exactly one after another with pass 2d's
// bit-stream machinery (as k_decode_batch_fix2 does).  Row 0 marked: the
// model does not fit this batch's first row, so *stale (pinned, the
// launcher's) asks for a fresh probe next time.
__global__ __launch_bounds__(kThreads) void k_rows_finish(
    const uint8_t *__restrict__ in, uint8_t *__restrict__ out, BatchLayout L,
    uint32_t nbuf, uint64_t *__restrict__ outlen, DecAlpha a, void *ws,
    const RowModel *rmodel, uint32_t *stale)
{
    __shared__ P2dSmem sm;
    const uint64_t len0 = scalar_load_u64((const uint64_t *) rmodel + 7);
    const unsigned long long *bm = row_fail(ws);
    build_dec_table(sm.tab, a);
    build_compact_sel(sm.sel);
    block_sync();
    const uint32_t lane = lane_id();
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t) gridDim.x * kWavesPerBlock;
    for (uint64_t g = (uint64_t) blockIdx.x * kWavesPerBlock + wv; g * 64 < nbuf; g += nw) {
        const uint64_t base = g * 64;
        uint64_t m = scalar_load_u64((const uint64_t *) bm + g);
        const uint64_t b = base + lane;
        if (b < nbuf && !((m >> lane) & 1)) outlen[b] = len0;
        if (m && lane == 0) {
            ((unsigned long long *) bm)[g] = 0;
            if (g == 0 && (m & 1) && stale) *stale = 1u;
        }
        while (m) {
            const uint32_t r = (uint32_t) (base + __ffsll((unsigned long long) m) - 1);
            m &= m - 1;
            uint64_t beg, len, obeg;
            batch_buf(L, r, beg, len, obeg);
            uint4 c[2];
            buf_first_chunks(in + beg, len, c);
            const uint64_t V = decode_buf_bits(sm, sm.bits[wv], in + beg, len, out + obeg, c);
            if (lane == 0) outlen[r] = V * 6 / 8;
        }
    }
}

// The hub's decode jobs, after k_decode_batch_fast/fix2<true> left each
// job's alphabet count V in vcount[]: one wave per job writes the job's
// result record straight into host memory (hres[j]; no D2H copy to trust).
// A job with flags[j] & 1 (HOLD: more of its stream follows) emits only
// whole groups, V/4*3 bytes, and reports its last V mod 4 sextets, which
// the stage spells in front of the stream's next job (the reference keeps
// those bits in decoder->bits across reads, base64decoder.c:64-76); a final
// job emits floor(6V/8) (the trailing partial bits dropped, :71-76).
__global__ __launch_bounds__(kThreads) void k_batch_finish(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
    const uint8_t *__restrict__ flags, const uint64_t *__restrict__ vcount, uint32_t njobs,
    uint64_t big, DecAlpha a, b64x_dec_result *__restrict__ hres, uint32_t seq)
{
    __shared__ uint8_t tab[256];
    build_dec_table(tab, a);
    block_sync();
    const uint32_t lane = lane_id();
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t j = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
         j < njobs; j += nw) {
        const uint64_t beg = in_off[j], n = in_off[j + 1] - beg, V = vcount[j];
        if ((big && n >= big) || (flags[j] & B64X_LANE_CHAINED))
            continue;  // its pipeline wrote the record
        const bool hold = flags[j] & 1;
        int need = hold ? (int) (V & 3) : 0;
        uint8_t got[4] = {0, 0, 0, 0};
        uint64_t end = n;
        while (need > 0 && end > 0) {  // the last V mod 4 alphabet characters
            const uint64_t b0 = end >= 64 ? end - 64 : 0;
            const uint64_t p = b0 + lane;
            const uint32_t t = p < end ? tab[in[beg + p]] : 0xFFu;
            uint64_t bm = __ballot(t < 64u);
            while (need > 0 && bm) {
                const int hi = 63 - __clzll(bm);
                got[--need] = (uint8_t) __shfl(t, hi, 64);
                bm &= ~(1ull << hi);
            }
            end = b0;
        }
        if (lane == 0) {
            b64x_dec_result *r = hres + j;
            for (int k = 0; k < 4; k++) r->tail[k] = got[k];
            r->valid = V;
            r->out_len = hold ? V / 4 * 3 : V * 6 / 8;
            r->tail_n = (uint32_t) (V & 3);
            r->nchars = n;
            r->seq = seq;
            r->flags = hold ? 1u : 0u;
        }
    }
}

// Completion stamp of a lane's encode batch: written into host memory by a
// kernel queued behind the batch's encode (b64x_lane_encode_check).
__global__ void __launch_bounds__(64) k_stamp(uint64_t *h_stamp, uint64_t v)
{
    if (threadIdx.x == 0) *(volatile uint64_t *) h_stamp = v;
}

// A chained lane job's head (the reference keeps these
// bits in decoder->bits across reads, src/base64decoder.c:64-76): the
// held-back sextets of the stream's previous block, read from its record
// (host memory, written by an earlier kernel of this stream), spelled as
// alphabet characters into the last tail_n of the 4 head bytes (the rest
// stay outside the alphabet).  What it read is logged, for the host to
// compare with the record it checked (b64x_spell_ok).
__global__ void __launch_bounds__(64) k_spell_head(uint8_t *head, const b64x_dec_result *prev,
                                                   b64x_dec_result *log, DecAlpha a)
{
    if (threadIdx.x != 0) return;
    const volatile b64x_dec_result *v = prev;
    b64x_dec_result r;
    r.out_len = v->out_len;
    r.valid = v->valid;
    r.tail_n = v->tail_n;
    for (int k = 0; k < 4; k++) r.tail[k] = v->tail[k];
    r.nchars = v->nchars;
    r.seq = v->seq;
    r.flags = v->flags;
    volatile b64x_dec_result *w = log;
    w->out_len = r.out_len;
    w->valid = r.valid;
    w->tail_n = r.tail_n;
    for (int k = 0; k < 4; k++) w->tail[k] = r.tail[k];
    w->nchars = r.nchars;
    w->seq = r.seq;
    w->flags = r.flags;
    const uint32_t n = r.tail_n <= 3 ? r.tail_n : 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t s = r.tail[k];
        if (s < 64) head[4 - n + k] = (uint8_t) (s < 62 ? enc_char(s, EncAlpha{}) : s == 62 ? a.p62 : a.p63);
    }
}

// ------------------------------------------------------------ utilities --

__global__ __launch_bounds__(kThreads) void k_fill_splitmix64(
    uint8_t *__restrict__ out, uint64_t n, uint64_t seed)
{
    const uint64_t words = (n + 7) / 8;
    for (uint64_t i = (uint64_t) blockIdx.x * kThreads + threadIdx.x; i < words;
         i += (uint64_t) gridDim.x * kThreads) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        if (i * 8 + 8 <= n) {
            if ((((uintptr_t) out) & 7) == 0) {
                *(uint64_t *) (out + i * 8) = z;
            } else {
                for (int k = 0; k < 8; k++) out[i * 8 + k] = (uint8_t) (z >> (8 * k));
            }
        } else {
            for (uint64_t k = 0; i * 8 + k < n; k++) out[i * 8 + k] = (uint8_t) (z >> (8 * k));
        }
    }
}

// ------------------------------------------------------------- host side --

struct DeviceInfo {
    bool ok = false;
    int cus = 256;
    int enc_blocks_per_cu = 8;
    int dec_blocks_per_cu = 8;
};

DeviceInfo query_device()
{
    DeviceInfo d;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return d;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return d;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return d;
    d.cus = prop.multiProcessorCount;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_encode, kThreads, 0) == hipSuccess && nb > 0)
        d.enc_blocks_per_cu = nb;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_decode_batch_fast<false>, kThreads, 0) == hipSuccess && nb > 0)
        d.dec_blocks_per_cu = nb;
    d.ok = true;
    return d;
}

// Per-device cache (one process per GPU is the deployment model, but
// tests may switch devices).
constexpr int kMaxDevices = 64;
std::mutex g_mu;
DeviceInfo g_info[kMaxDevices];
bool g_info_done[kMaxDevices];
// Library-owned decode workspaces, one per (device, stream): a workspace
// carries state from one kernel of a decode to the next, so streams must
// not share one at the same time.  At most kWsCache of them exist (about
// 12.7 MiB of HBM each), allocated on first need and then kept: a stream
// that needs one takes a free slot, or rebinds the least recently used
// idle workspace of its device, and never frees memory on the way.
//  - A call pins its entry from the lookup until its kernels are enqueued
//    (`pins`), so no other thread can rebind a workspace between handing it
//    out and enqueuing on it; when all kWsCache entries are pinned the call
//    gets -EBUSY.
//  - Rebinding makes the new stream wait on the device for the workspace's
//    last use (hipStreamWaitEvent): no host wait, no device-wide
//    synchronisation, no hipFree, and no lock held across a HIP call that
//    waits, so a host callback on any stream that calls back into the
//    library cannot deadlock on it.  (Round 3 freed the LRU workspace after
//    a hipDeviceSynchronize under the library's lock; a first fix that freed
//    it with hipFree outside the lock hung a 12-thread test on the MI355X:
//    hipFree waits for the whole device.)
//  - The event that marks the last use is recorded when the workspace leaves
//    its stream, not after every call: on the old stream when another stream
//    takes it over (everything enqueued there so far includes every use),
//    or on the stream being released (b64x_release_stream, which the caller
//    runs before destroying it).  Round 4 recorded it behind every call; an
//    event between two kernels leaves the GPU idle for several microseconds,
//    which showed as +5 us per config-3 batch decode.
//  - Each call leaves the workspace zeroed for the next (re-armed by the
//    kernels), so a rebound workspace needs no clearing.
// A library workspace: the decode workspace for the largest plan, then the
// row batches' model (row_model_of).
constexpr uint64_t kLibRowsOff = (ws_bytes_for(kMaxRanges) + 255) & ~255ull;
constexpr uint64_t kLibWsBytes = kLibRowsOff + 256;
static RowModel *row_model_of(void *ws) { return (RowModel *) ((uint8_t *) ws + kLibRowsOff); }

// The shape a row batch's model was made for (nbuf 0: no model held).
struct RowsShape {
    uint64_t len, in_stride, out_stride;
    uint32_t nbuf;
    int p62, p63;
    bool operator==(const RowsShape &o) const
    {
        return len == o.len && in_stride == o.in_stride && out_stride == o.out_stride &&
               nbuf == o.nbuf && p62 == o.p62 && p63 == o.p63;
    }
};

struct WsEntry {
    int dev;
    bool bound;         // held by `stream` (which may be the NULL stream); else idle
    void *stream;       // the stream it is bound to (meaningful only when bound)
    void *ws;           // nullptr: slot not allocated yet
    hipEvent_t last;    // recorded behind the last use when it left a stream
    bool recorded;      // `last` guards a use on a stream it has left
    uint64_t used;      // last use (g_ws_tick)
    int pins;           // calls between lookup and their event record
    bool release;       // b64x_release_stream while pinned: unbind at unpin
    RowsShape rows;     // the row batch shape whose model the workspace holds
};
constexpr int kWsCache = 8;
std::mutex g_ws_mu;     // g_ws, g_ws_tick (held across hipEventRecord, which only
                        // enqueues, never across a HIP call that waits)
WsEntry g_ws[kWsCache];
uint64_t g_ws_tick;

const DeviceInfo *device_info()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_info_done[dev]) {
        g_info[dev] = query_device();
        g_info_done[dev] = true;
    }
    return g_info[dev].ok ? &g_info[dev] : nullptr;
}

EncAlpha enc_alpha(const b64x_alphabet *abc)
{
    EncAlpha a;
    const char p62 = abc ? abc->pos62 : (char) -1;
    const char p63 = abc ? abc->pos63 : (char) -1;
    const char pc = abc ? abc->padchar : (char) -1;
    a.p62 = (uint8_t) (p62 == (char) -1 ? '+' : p62);
    a.p63 = (uint8_t) (p63 == (char) -1 ? '/' : p63);
    a.padc = (uint8_t) (pc == (char) -1 ? '=' : pc);
    a.pad = abc ? (abc->pad ? 1 : 0) : 1;
    return a;
}

DecAlpha dec_alpha(const b64x_alphabet *abc)
{
    DecAlpha a;
    const char p62 = abc ? abc->pos62 : (char) -1;
    const char p63 = abc ? abc->pos63 : (char) -1;
    a.p62 = (int) (signed char) (p62 == (char) -1 ? '+' : p62);
    a.p63 = (int) (signed char) (p63 == (char) -1 ? '/' : p63);
    return a;
}

int hip_err(hipError_t e)
{
    if (e == hipSuccess) return 0;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return -ENODEV;
    if (e == hipErrorOutOfMemory) return -ENOMEM;
    return -EIO;
}

int launch_status() { return hip_err(hipGetLastError()); }

uint32_t cap_grid(uint64_t want, uint64_t cap)
{
    if (want < 1) want = 1;
    return (uint32_t) (want < cap ? want : cap);
}

struct RangePlan {
    uint64_t R;
    uint32_t nranges;
};

#ifdef B64X_TEST_HOOKS
// Test builds only (tests/csrc/libb64x_hooks.so): a decode range length in
// chunks, so ranges longer than one pass-2 step can be tested at small
// sizes.  The product library has no such knob.
uint64_t g_test_range_chunks = 0;
#endif

// Ranges of kRangeChunks chunks, at most kMaxRanges of them: many short
// ranges, one wave each, launched as a non-persistent grid -- the shape
// that streams fastest -- and enough parallelism for the exact pass 2 on
// dirty input.
RangePlan plan_ranges(uint64_t n)
{
    uint64_t chunks = kRangeChunks;
#ifdef B64X_TEST_HOOKS
    if (g_test_range_chunks) chunks = g_test_range_chunks;
#endif
    uint64_t R = chunks * kChunk;
    // up to kLinesMaxChars: 2,048-character ranges for the lines path, past
    // kMaxRanges too (its kernels use no per-range scratch)
    if ((n + R - 1) / R > kMaxRanges && !(chunks == kRangeChunks && n <= kLinesMaxChars)) {
        R = (n + kMaxRanges - 1) / kMaxRanges;
        R = (R + kChunk - 1) / kChunk * kChunk;
    }
    RangePlan p;
    p.R = R;
    p.nranges = (uint32_t) ((n + R - 1) / R);
    if (p.nranges == 0) p.nranges = 1;
    return p;
}

template <typename K>
int occupancy_of(K kernel)
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, kThreads, 0) != hipSuccess || nb < 1)
        nb = 1;
    return nb;
}

// Pass 1's shipped form: two chunks per lane in flight, non-temporal loads
// and stores (round 1's A/B of 1-8 chunks, pipelining and cached loads,
// profiles/r01_v6_*).
constexpr auto k_pass1 = k_decode_pass1<2, true>;

}  // namespace

// ================================================================ C ABI ==

extern "C" {

uint64_t b64x_encoded_len(uint64_t n, bool pad)
{
    return pad ? (n + 2) / 3 * 4 : (n * 4 + 2) / 3;
}

uint64_t b64x_decoded_cap(uint64_t nchars) { return (nchars + 3) / 4 * 3; }

uint64_t b64x_decode_workspace_size(uint64_t nchars)
{
    // the fixed regions, then counts + bases for as many ranges as any
    // plan can use for nchars (ranges are at least one chunk; 0 = the
    // largest input); at least room for a RowModel in the scratch
    uint64_t nr = nchars ? (nchars + kChunk - 1) / kChunk : kMaxRanges;
    if (nr > kMaxRanges) nr = kMaxRanges;
    return ws_bytes_for(nr);
}

int b64x_device_check(void) { return device_info() ? 0 : -ENODEV; }

// ---- host placement (sysfs; no libnuma in the image) ----------------------

static bool read_small(const char *path, char *buf, size_t cap)
{
    FILE *f = fopen(path, "r");
    if (!f) return false;
    const size_t n = fread(buf, 1, cap - 1, f);
    fclose(f);
    buf[n] = 0;
    return n > 0;
}

int b64x_device_numa_node(int device)
{
    if (device < 0 && hipGetDevice(&device) != hipSuccess) return -ENODEV;
    char bus[64];
    if (hipDeviceGetPCIBusId(bus, (int) sizeof bus, device) != hipSuccess) return -ENODEV;
    for (char *c = bus; *c; c++)
        if (*c >= 'A' && *c <= 'F') *c = (char) (*c - 'A' + 'a');
    char path[160], v[32];
    snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
    if (!read_small(path, v, sizeof v)) return -ENOENT;
    const int node = atoi(v);
    return node >= 0 ? node : -ENOENT;
}

// "0-63,128-191" -> set
static bool parse_cpulist(const char *s, cpu_set_t *set)
{
    CPU_ZERO(set);
    bool any = false;
    while (*s) {
        char *e = nullptr;
        long a = strtol(s, &e, 10);
        if (e == s) break;
        long b = a;
        s = e;
        if (*s == '-') {
            b = strtol(s + 1, &e, 10);
            s = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++) {
            CPU_SET((int) c, set);
            any = true;
        }
        while (*s == ',' || *s == '\n' || *s == ' ') s++;
    }
    return any;
}

int b64x_bind_thread(int device)
{
    const int node = b64x_device_numa_node(device);
    if (node < 0) return node;
    char path[96], list[4096];
    snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
    cpu_set_t on_node, mine, both;
    if (!read_small(path, list, sizeof list) || !parse_cpulist(list, &on_node)) return -ENOENT;
    if (sched_getaffinity(0, sizeof mine, &mine) != 0) return -errno;
    CPU_AND(&both, &on_node, &mine);
    if (CPU_COUNT(&both) == 0) return -ENOENT;  // the thread may not run there
    if (CPU_EQUAL(&both, &mine)) return node;   // already inside the node
    // a mask inside another single node: the application placed the thread
    bool one_node = true;
    int first = -1;
    for (int c = 0; c < CPU_SETSIZE && one_node; c++) {
        if (!CPU_ISSET(c, &mine)) continue;
        char np[96];
        int n = -1;
        for (int k = 0; k < 64 && n < 0; k++) {
            snprintf(np, sizeof np, "/sys/devices/system/cpu/cpu%d/node%d", c, k);
            if (access(np, F_OK) == 0) n = k;
        }
        if (first < 0) first = n;
        else if (n != first) one_node = false;
    }
    if (one_node) return first;
    if (sched_setaffinity(0, sizeof both, &both) != 0) return -errno;
    // prefer the node for the pages this thread faults in from now on
    unsigned long mask[16] = {0};
    if (node < 64 * 16) {
        mask[node / 64] = 1ul << (node % 64);
        (void) syscall(SYS_set_mempolicy, 1 /* MPOL_PREFERRED */, mask, (unsigned long) 64 * 16);
    }
    return node;
}

int b64x_encode_dev(const void *d_in, uint64_t n, void *d_out,
                    const b64x_alphabet *abc, void *stream)
{
    if (n == 0) return 0;
    if (!d_in || !d_out) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    if (((((uintptr_t) d_in) | ((uintptr_t) d_out)) & 3) == 0) {
        const uint64_t tiles = n / 12 / kEncTH;
        hipLaunchKernelGGL(k_encode_flat, dim3(cap_grid(tiles, (uint64_t) 1 << 31)),
                           dim3(kEncTH), 0, (hipStream_t) stream, (const uint8_t *) d_in,
                           (uint8_t *) d_out, tiles, n, enc_alpha(abc));
        return launch_status();
    }
    // Misaligned buffers: the generic slot kernel (bytewise where needed).
    const uint64_t slots = (n + 11) / 12;
    const uint64_t per_block = (uint64_t) kThreads * kEncUnroll;
    uint32_t grid = cap_grid((slots + per_block - 1) / per_block,
                             (uint64_t) d->cus * d->enc_blocks_per_cu);
    hipLaunchKernelGGL(k_encode, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (const uint8_t *) d_in, (uint64_t) 0, n, 1u, (uint8_t *) d_out,
                       (uint64_t) 0, slots, slots, enc_alpha(abc));
    return launch_status();
}

int b64x_encode_strided(const void *d_in, uint64_t in_stride, uint64_t len,
                        uint32_t nbuf, void *d_out, uint64_t out_stride,
                        const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0 || len == 0) return 0;
    if (!d_in || !d_out) return -EINVAL;
    if (nbuf == 1) return b64x_encode_dev(d_in, len, d_out, abc, stream);
    if (in_stride < len || out_stride < b64x_encoded_len(len, enc_alpha(abc).pad))
        return -EINVAL;
    const uint64_t qpb = (len + 11) / 12;
    const uint64_t slots = qpb * nbuf;
    if (slots > 0xFFFFFFFFull - 4096) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    // output slots per lane of k_encode_tight2 (1: +9 %, 4: +5 % on config
    // 4, profiles/r05_ab_tight_shapes.jsonl)
    constexpr int U = 2;
    const EncAlpha ea = enc_alpha(abc);
    const uint64_t E = b64x_encoded_len(len, ea.pad);
    const uint32_t r = (uint32_t) (len % 3);
    // Tight layout, one launch (k_encode_tight2).
    const bool tight = in_stride == len && out_stride == E && len >= 16 && (ea.pad || r == 0) &&
                       (((uintptr_t) d_in) & 3) == 0 && (((uintptr_t) d_out) & 15) == 0;
    if (tight && E < (1u << 20)) {
        const uint32_t magic = (uint32_t) ((0xFFFFFFFFull + E) / E);
        const uint64_t e = (uint64_t) magic * E - (1ull << 32);
        if ((E + 16ull * U * kThreads) * e < (1ull << 32)) {
            const uint64_t total_out = (uint64_t) nbuf * E;
            const uint64_t nslots = (total_out + 15) / 16;
            const uint64_t tail_slot = (nbuf - 1) * E / 16 ? (nbuf - 1) * E / 16 - 1 : 0;
            const uint64_t m64 = ~0ull / E + 1;
            const uint64_t per = (uint64_t) U * kThreads;
            const dim3 g((uint32_t) ((nslots + per - 1) / per));
            hipLaunchKernelGGL(k_encode_tight2<U>, g, dim3(kThreads), 0, (hipStream_t) stream,
                               (const uint8_t *) d_in, len, (uint32_t) E, r, magic, m64,
                               (uint8_t *) d_out, nslots, (uint64_t) nbuf * len, total_out,
                               tail_slot, ea);
            return launch_status();
        }
    }
    // Any other layout: one lane per (buffer, quad).
    constexpr int US = 2;
    const uint64_t per_block = (uint64_t) kThreads * US;
    hipLaunchKernelGGL((k_encode_strided<US, true>), dim3((uint32_t) ((slots + per_block - 1) / per_block)),
                       dim3(kThreads), 0, (hipStream_t) stream, (const uint8_t *) d_in,
                       in_stride, len, nbuf, (uint8_t *) d_out, out_stride, (uint32_t) qpb,
                       (uint32_t) slots, enc_alpha(abc));
    return launch_status();
}

int b64x_encode_batch(const void *d_in, const uint64_t *d_in_off, uint32_t nbuf,
                      void *d_out, const uint64_t *d_out_off,
                      const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0) return 0;
    if (!d_in || !d_in_off || !d_out || !d_out_off) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    uint32_t grid = cap_grid(nbuf, (uint64_t) 1 << 30);
    hipLaunchKernelGGL(k_encode_ragged, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (const uint8_t *) d_in, d_in_off, nbuf, (uint8_t *) d_out,
                       d_out_off, enc_alpha(abc));
    return launch_status();
}

// A stream being captured into a graph: its calls never reuse what earlier
// calls left (a held model) -- the graph replays later, after other calls
// may have replaced it, so the capture records the probe or prep as well --
// and never allocate or take over a library workspace.
static bool capturing(void *stream)
{
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing((hipStream_t) stream, &st) == hipSuccess &&
           st != hipStreamCaptureStatusNone;
}

// The workspace of (current device, stream), pinned; *slot receives its
// entry for ws_unpin().  A stream that holds none and is being captured
// gets nullptr with *err = -EBUSY: allocating or rebinding one (a hipMalloc,
// or a wait on an event recorded outside the capture) has no place in a
// graph, so such a stream decodes once outside the capture first, or passes
// a workspace of its own.
static void *library_workspace(void *stream, int *slot, int *err, RowsShape *rows = nullptr)
{
    if (rows) *rows = RowsShape{};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        *err = -ENODEV;
        return nullptr;
    }
    int v = -1;
    bool fresh = false, wait = false;
    hipEvent_t after = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        for (int i = 0; i < kWsCache; i++) {
            WsEntry &e = g_ws[i];
            if (e.ws && e.dev == dev && e.bound && e.stream == stream && !e.release) {
                e.used = ++g_ws_tick;
                e.pins++;
                *slot = i;
                *err = 0;
                if (rows) *rows = e.rows;
                return e.ws;
            }
        }
        if (capturing(stream)) {
            *err = -EBUSY;
            return nullptr;
        }
        // the least recently used idle workspace of this device (released,
        // or bound to a stream that is not being captured), else a slot
        // never allocated
        unsigned skip = 0;
        for (;;) {
            v = -1;
            for (int i = 0; i < kWsCache; i++) {
                const WsEntry &e = g_ws[i];
                if (e.ws && e.dev == dev && !e.pins && !((skip >> i) & 1) &&
                    (v < 0 || e.used < g_ws[v].used))
                    v = i;
            }
            if (v < 0 || !g_ws[v].bound || !capturing(g_ws[v].stream)) break;
            skip |= 1u << v;
        }
        if (v < 0)
            for (int i = 0; i < kWsCache && v < 0; i++)
                if (!g_ws[i].ws && !g_ws[i].pins) v = i;
        if (v < 0) {
            *err = -EBUSY;  // every workspace is in use by a call, or on another device
            return nullptr;
        }
        WsEntry &e = g_ws[v];
        fresh = !e.ws;
        if (!fresh && e.bound) {
            // taken from a stream that still holds it: mark the end of
            // everything enqueued there so far, its last use included (an
            // enqueue, no wait; under the lock, so the owner cannot release
            // and destroy the stream in between)
            if (hipEventRecord(e.last, (hipStream_t) e.stream) != hipSuccess) {
                *err = -EBUSY;
                return nullptr;
            }
            e.recorded = true;
        }
        wait = !fresh && e.recorded;
        after = e.last;
        if (fresh) e = WsEntry{};
        e.dev = dev;
        e.bound = true;
        e.stream = stream;
        e.used = ++g_ws_tick;
        e.pins = 1;  // reserved: nobody else takes this slot
        e.release = false;
        e.rows = RowsShape{};  // the old stream's row model is not this stream's
    }
    int rc = 0;
    if (fresh) {
        void *p = nullptr;
        hipEvent_t ev = nullptr;
        const uint64_t wsz = kLibWsBytes;
        hipError_t he = hipMalloc(&p, wsz);
        if (he == hipSuccess) he = hipMemsetAsync(p, 0, wsz, (hipStream_t) stream);
        if (he == hipSuccess) he = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        std::lock_guard<std::mutex> lk(g_ws_mu);
        if (he != hipSuccess) {
            if (p) (void) hipFree(p);
            if (ev) (void) hipEventDestroy(ev);
            g_ws[v] = WsEntry{};
            *err = hip_err(he);
            return nullptr;
        }
        g_ws[v].ws = p;
        g_ws[v].last = ev;
    } else if (wait) {
        // the previous stream's last use of it finishes first, on the device
        rc = hip_err(hipStreamWaitEvent((hipStream_t) stream, after, 0));
    }
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if (rc) {
        g_ws[v].bound = false;  // idle again, its event still guards it
        g_ws[v].stream = nullptr;
        g_ws[v].pins = 0;
        *err = rc;
        return nullptr;
    }
    *slot = v;
    *err = 0;
    if (rows) *rows = g_ws[v].rows;
    return g_ws[v].ws;
}

// Unbind entry e from its stream, marking the stream's position (the end of
// the workspace's last use) with the entry's event.  Under g_ws_mu.
static void ws_leave(WsEntry &e)
{
    if (e.bound && hipEventRecord(e.last, (hipStream_t) e.stream) == hipSuccess)
        e.recorded = true;
    else if (e.bound)
        e.recorded = false;  // nothing to wait on; the caller owns the ordering
    e.bound = false;
    e.stream = nullptr;
    e.release = false;
}

// The call that pinned entry `slot` has enqueued its kernels on `stream`:
// unpin it.  rows: the shape of the row batch whose model and cleared bitmap
// the call leaves in the workspace; none for any other call (its kernels use
// the scratch).  No event here: the workspace stays with its stream, whose
// own order protects the next call (see g_ws).
static void ws_unpin(int slot, void *stream, RowsShape rows = RowsShape{})
{
    (void) stream;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    WsEntry &e = g_ws[slot];
    e.rows = rows;
    if (--e.pins == 0 && e.release) ws_leave(e);
}

void b64x_release_stream(void *stream)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (int i = 0; i < kWsCache; i++) {
        WsEntry &e = g_ws[i];
        if (!e.ws || e.dev != dev || !e.bound || e.stream != stream) continue;
        if (e.pins)
            e.release = true;  // the last unpin unbinds it
        else
            ws_leave(e);  // idle: the next stream waits on its event
    }
}

__global__ void __launch_bounds__(64) k_result_zero(b64x_dec_result *res, b64x_dec_result *hres,
                                                    uint32_t hold, uint32_t seq)
{
    if (threadIdx.x != 0) return;
    b64x_dec_result r{};
    r.seq = seq;
    r.flags = hold ? 1u : 0u;
    *res = r;
    if (hres) *hres = r;
}

// Sequence numbers of decode calls and batches: nonzero, process-wide.
static uint32_t next_seq()
{
    static std::atomic<uint32_t> g_seq{0};
    uint32_t v;
    do {
        v = g_seq.fetch_add(1, std::memory_order_relaxed) + 1;
    } while (v == 0);
    return v;
}

// The probes' hints (k_decode_probe), pinned, one per hash of (workspace,
// input, length); allocated on first use.
static DecodeHint *decode_hints()
{
    static DecodeHint *h = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        void *p = nullptr;
        if (hipHostMalloc(&p, kDecodeHints * sizeof(DecodeHint), hipHostMallocCoherent) == hipSuccess) {
            memset(p, 0, kDecodeHints * sizeof(DecodeHint));
            h = (DecodeHint *) p;
        }
    });
    return h;
}

// Per library workspace: set by k_rows_finish when the batch's first row
// failed the model it was decoded with (pinned, coherent); allocated on
// first use, nullptr if that fails (then every row batch probes).
static uint32_t *rows_stale(int slot)
{
    static uint32_t *h = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        void *p = nullptr;
        if (hipHostMalloc(&p, kWsCache * 64, hipHostMallocCoherent) == hipSuccess) {
            memset(p, 0, kWsCache * 64);
            h = (uint32_t *) p;
        }
    });
    return h ? h + 16 * slot : nullptr;  // one 64-byte line each
}

// Workspaces whose line model (k_decode_probe's, kept in the workspace with
// the length it was made for) a call of the same length may reuse without a
// probe: one entry per hash of the workspace, and a pinned flag beside it
// that k_decode_suffix_held<false> raises when a call found anything to decode
// past k_decode_lines (junk, another format, a cut model), so that the next
// call probes again.  A wrong entry or a late flag only costs speed: any
// model gives exact output, and k_decode_lines checks the model's length.
struct HeldModel {
    const void *ws;
    uint64_t n;
};
constexpr int kHeldModels = 64;
std::mutex g_held_mu;
HeldModel g_held[kHeldModels];

static uint32_t *held_reprobe(int slot)
{
    static uint32_t *h = nullptr;
    static std::once_flag once;
    std::call_once(once, [] {
        void *p = nullptr;
        if (hipHostMalloc(&p, kHeldModels * 64, hipHostMallocCoherent) == hipSuccess) {
            memset(p, 0, kHeldModels * 64);
            h = (uint32_t *) p;
        }
    });
    return h ? h + 16 * slot : nullptr;  // one 64-byte line each
}

static int held_slot(const void *ws)
{
    const uint64_t x = (uintptr_t) ws * 0x9E3779B97F4A7C15ull;
    return (int) (x >> 58);  // 64 entries
}

// Which path each automatic decode and row batch took (b64x_diag_paths):
// probes launched, probes skipped (held model), hinted single passes, row
// preps launched, row preps skipped (row model reused).
enum { kPathProbe, kPathHeld, kPathHinted, kPathRowsPrep, kPathRowsReuse, kPaths };
static std::atomic<uint64_t> g_paths[kPaths];

static void path_taken(int k) { g_paths[k].fetch_add(1, std::memory_order_relaxed); }

void b64x_diag_paths(uint64_t out[5])
{
    for (int k = 0; k < kPaths; k++) out[k] = g_paths[k].load(std::memory_order_relaxed);
}

static uint32_t hint_key(const void *ws, const void *in, uint64_t n)
{
    uint64_t x = (uintptr_t) ws * 0x9E3779B97F4A7C15ull ^ (uintptr_t) in * 0xC2B2AE3D27D4EB4Full ^
                 n * 0x165667B19E3779F9ull;
    x ^= x >> 31;
    return (uint32_t) (x >> 32) | 1u;  // never 0, the unused slot's key
}

// decode_dev_impl's launches on a given workspace.

static int decode_dev_ws(const void *d_in, uint64_t nchars, void *d_out,
                         b64x_dec_result *d_res, b64x_dec_result *h_res,
                         const b64x_alphabet *abc, unsigned flags, void *ws, void *stream,
                         uint32_t seq, const DeviceInfo *d)
{
    hipStream_t s = (hipStream_t) stream;
    int err = 0;
    const RangePlan p = plan_ranges(nchars);
    const uint32_t blocks = (p.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const DecAlpha a = dec_alpha(abc);
    const uint32_t hold = flags & B64X_DEC_HOLD_TAIL;
    if (p.R == 2 * kChunk) {
        // Inputs up to 2^31 characters: the line-structured single pass
        // (clean input is its L = 0 case), then the exact single-pass decode
        // of whatever suffix it could not take -- nothing, on clean and
        // MIME-formatted text: each block of that launch reads one word and
        // returns.  EXPECT_JUNK skips the first.
        // BIG instances past 2^31 characters (64-bit positions and prefixes)
        const bool big = nchars > (1ull << 31);
        static const int occ_small = occupancy_of(k_decode_suffix_held<false, false>);
        static const int occ_big = occupancy_of(k_decode_suffix_held<false, true>);
        const int occ_sfx = big ? occ_big : occ_small;
        auto *const k_whole = big ? k_decode_suffix_held<true, true> : k_decode_suffix_held<true, false>;
        auto *const k_sfx = big ? k_decode_suffix_held<false, true> : k_decode_suffix_held<false, false>;
        auto *const k_lines = big ? k_decode_lines<true> : k_decode_lines<false>;
        const uint32_t sfx_grid = (uint32_t) d->cus * occ_sfx;
        if (flags & B64X_DEC_EXPECT_JUNK) {
            hipLaunchKernelGGL(k_whole, dim3(sfx_grid), dim3(kThreads), 0, s,
                               (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.nranges, a, ws,
                               hold, d_res, h_res, seq, nullptr, nullptr, 0u);
            return launch_status();
        }
        // The probe of the last call on the same workspace, input and length
        // cut the line model near the start (junk throughout): this call
        // takes the single pass, which runs the probe itself (renewing the
        // hint and the model for the next call) in its first block to run
        // out of tiles, while the others finish theirs, and skips
        // k_decode_lines' launch of blocks that would all leave at once.
        // Same bytes either way; only the path differs.
        DecodeHint *hints = decode_hints();
        const uint32_t key = hint_key(ws, d_in, nchars);
        DecodeHint *hint = hints ? hints + (key % kDecodeHints) : nullptr;
        const bool junky = hint && ((volatile DecodeHint *) hint)->key == key &&
                           ((volatile DecodeHint *) hint)->junky;
        // The workspace holds the model its last probe made for a stream of
        // this length, and no call since found anything past
        // k_decode_lines: the probe is skipped (HeldModel).
        const int hs = held_slot(ws);
        uint32_t *reprobe = held_reprobe(hs);
        bool reuse = false;
        if (!junky && reprobe && !capturing(stream)) {
            std::lock_guard<std::mutex> lk(g_held_mu);
            reuse = g_held[hs].ws == ws && g_held[hs].n == nchars &&
                    !*(volatile uint32_t *) reprobe;
        }
        if (junky) {
            path_taken(kPathHinted);
            if (reprobe) *(volatile uint32_t *) reprobe = 0;
            hipLaunchKernelGGL(k_whole, dim3(sfx_grid), dim3(kThreads), 0, s,
                               (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.nranges, a, ws,
                               hold, d_res, h_res, seq, nullptr, hint, key);
            if ((err = launch_status())) return err;
            path_taken(kPathProbe);
            std::lock_guard<std::mutex> lk(g_held_mu);
            g_held[hs] = HeldModel{ws, nchars};
            return 0;
        }
        if (!reuse) {
            if (reprobe) *(volatile uint32_t *) reprobe = 0;
            hipLaunchKernelGGL(k_decode_probe, dim3(1), dim3(kProbeThreads), 0, s,
                               (const uint8_t *) d_in, nchars, a, ws, p.nranges, hint, key);
            if ((err = launch_status())) return err;
            path_taken(kPathProbe);
            std::lock_guard<std::mutex> lk(g_held_mu);
            g_held[hs] = HeldModel{ws, nchars};
        } else {
            path_taken(kPathHeld);
        }
        const uint64_t waves = (nchars / 16 + 1 + kLinesSlots - 1) / kLinesSlots;
        hipLaunchKernelGGL(k_lines, dim3((uint32_t) ((waves + kLinesWaves - 1) / kLinesWaves)),
                           dim3(kLinesTH), 0, s, (const uint8_t *) d_in, nchars, (uint8_t *) d_out,
                           p.nranges, a, ws, hold, d_res, seq);
        if ((err = launch_status())) return err;
        hipLaunchKernelGGL(k_sfx, dim3(sfx_grid), dim3(kThreads), 0, s,
                           (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.nranges, a, ws,
                           hold, d_res, h_res, seq, reprobe, nullptr, 0u);
        return launch_status();
    }
    // Larger inputs (ranges longer than 2,048 characters): pass 1, the scan,
    // pass 2.
    hipLaunchKernelGGL(k_pass1, dim3(blocks), dim3(kThreads), 0, s, (const uint8_t *) d_in,
                       nchars, (uint8_t *) d_out, p.R, p.nranges, a, ws, hold);
    if ((err = launch_status())) return err;
    hipLaunchKernelGGL(k_decode_scan2, dim3((p.nranges + kScanTile - 1) / kScanTile),
                       dim3(kThreads), 0, s, (const uint8_t *) d_in, nchars, p.R, p.nranges, a,
                       ws, d_res, h_res, hold, seq);
    if ((err = launch_status())) return err;
    // grid-stride over the ranges with exactly the resident blocks (a second
    // partial round of blocks would trail the rest)
    static const int occ2d = occupancy_of(k_decode_pass2d);
    const uint32_t b2 = cap_grid(blocks, (uint64_t) d->cus * occ2d);
    hipLaunchKernelGGL(k_decode_pass2d, dim3(b2), dim3(kThreads), 0, s,
                       (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.R, p.nranges,
                       a, ws, hold);
    return launch_status();
}

// b64x_decode_dev, plus an optional host mirror of the result record that
// the kernels write themselves (sessions; see write_result).
static int decode_dev_impl(const void *d_in, uint64_t nchars, void *d_out,
                           b64x_dec_result *d_res, b64x_dec_result *h_res,
                           const b64x_alphabet *abc, unsigned flags, void *d_workspace,
                           void *stream, uint32_t seq)
{
    if (!d_res) return -EINVAL;
    if (flags & ~(unsigned) (B64X_DEC_HOLD_TAIL | B64X_DEC_EXPECT_JUNK)) return -EINVAL;
    if (nchars && (!d_in || !d_out)) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    hipStream_t s = (hipStream_t) stream;
    if (nchars == 0) {
        hipLaunchKernelGGL(k_result_zero, dim3(1), dim3(64), 0, s, d_res, h_res,
                           flags & B64X_DEC_HOLD_TAIL, seq);
        return launch_status();
    }
    if (d_workspace)
        return decode_dev_ws(d_in, nchars, d_out, d_res, h_res, abc, flags, d_workspace, stream,
                             seq, d);
    int err = 0, slot = -1;
    void *ws = library_workspace(stream, &slot, &err);
    if (!ws) return err;
    err = decode_dev_ws(d_in, nchars, d_out, d_res, h_res, abc, flags, ws, stream, seq, d);
    ws_unpin(slot, stream);
    return err;
}

int b64x_decode_dev(const void *d_in, uint64_t nchars, void *d_out,
                    b64x_dec_result *d_res, const b64x_alphabet *abc,
                    unsigned flags, void *d_workspace, void *stream)
{
    return decode_dev_impl(d_in, nchars, d_out, d_res, nullptr, abc, flags, d_workspace,
                           stream, next_seq());
}

int b64x_decode_dev_seq(const void *d_in, uint64_t nchars, void *d_out,
                        b64x_dec_result *d_res, const b64x_alphabet *abc,
                        unsigned flags, void *d_workspace, void *stream, uint32_t *seq)
{
    const uint32_t q = next_seq();
    if (seq) *seq = q;
    return decode_dev_impl(d_in, nchars, d_out, d_res, nullptr, abc, flags, d_workspace,
                           stream, q);
}

int b64x_result_check(const b64x_dec_result *res, uint64_t nchars, unsigned flags,
                      uint32_t seq)
{
    if (!res) return -EINVAL;
    return b64x_result_ok(res, nchars, flags, seq, nullptr) ? 0 : -EAGAIN;
}

// rv: d_outlen receives alphabet counts V (the hub's jobs) instead of bytes.
static int launch_batch_decode(const void *d_in, const BatchLayout &L, uint32_t nbuf,
                               void *d_out, uint64_t *d_outlen,
                               const b64x_alphabet *abc, void *stream, bool rv = false)
{
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    hipStream_t s = (hipStream_t) stream;
    const DecAlpha a = dec_alpha(abc);
    static const int occ = occupancy_of(k_decode_batch_fast<false>);
    uint32_t grid = cap_grid((nbuf + kWavesPerBlock - 1) / kWavesPerBlock,
                             (uint64_t) d->cus * occ);
    hipLaunchKernelGGL(rv ? k_decode_batch_fast<true> : k_decode_batch_fast<false>, dim3(grid),
                       dim3(kThreads), 0, s, (const uint8_t *) d_in, (uint8_t *) d_out, L, nbuf,
                       d_outlen, a);
    int err = launch_status();
    if (err) return err;
    // The fix-up scans outlen[] 64 words per wave; on clean input that is
    // all it does.
    uint32_t fgrid = cap_grid(((uint64_t) nbuf + 64 * kWavesPerBlock - 1) / (64 * kWavesPerBlock),
                              (uint64_t) d->cus * 8);
    hipLaunchKernelGGL(rv ? k_decode_batch_fix2<true> : k_decode_batch_fix2<false>, dim3(fgrid),
                       dim3(kThreads), 0, s, (const uint8_t *) d_in, (uint8_t *) d_out, L, nbuf,
                       d_outlen, a);
    return launch_status();
}

int b64x_decode_strided(const void *d_in, uint64_t in_stride, uint64_t len,
                        uint32_t nbuf, void *d_out, uint64_t out_stride,
                        uint64_t *d_outlen, const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0) return 0;
    if (!d_in || !d_out || !d_outlen) return -EINVAL;
    if (nbuf > 1 && (in_stride < len || out_stride < b64x_decoded_cap(len))) return -EINVAL;
    const uint64_t S = (len + 15) / 16;
    const uint64_t slots = S * nbuf;
    BatchLayout L{nullptr, nullptr, in_stride, out_stride, len, 0, nullptr};
    if (slots > 0xFFFFFFFFull - 4096 || len > 0xFFFFFFFFull)
        return launch_batch_decode(d_in, L, nbuf, d_out, d_outlen, abc, stream);
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    hipStream_t s = (hipStream_t) stream;
    const DecAlpha a = dec_alpha(abc);
    const bool rows = nbuf >= 2 && S >= 2 && out_stride >= 12 * S && (in_stride & 3) == 0 &&
                      (out_stride & 3) == 0 && (((uintptr_t) d_in) & 3) == 0 &&
                      (((uintptr_t) d_out) & 3) == 0;
    bool done = false;
    int err = 0;
    if (rows && S < (1u << 20)) {
        // rows with room: k_rows_prep (the failure bitmap, the line model
        // and the shape of row 0's last slot), k_decode_rows_lines (clean
        // rows by k_decode_rows2's path, MIME-formatted rows by the model),
        // k_rows_finish (every row's length; the marked rows exactly)
        constexpr uint32_t U = kRowsU;
        const uint32_t magic = (uint32_t) ((0xFFFFFFFFull + S) / S);
        const uint64_t e = (uint64_t) magic * S - (1ull << 32);
        const uint64_t relmax = S + (uint64_t) U * kThreads;
        void *ws = nullptr;
        int slot = -1;
        RowsShape held{};
        const uint64_t bitmap = ((uint64_t) nbuf + 63) / 64 * 8 + sizeof(RowModel);
        if (relmax * e < (1ull << 32) && (relmax / S + 1) * in_stride < (1ull << 40) &&
            bitmap <= b64x_decode_workspace_size(0) - kWsScratch &&
            (ws = library_workspace(stream, &slot, &err, &held))) {
            const uint64_t m64 = ~0ull / S + 1;
            const uint64_t per = (uint64_t) U * kThreads;
            const uint64_t tail_slot = (uint64_t) S * (nbuf - 1);
            const uint64_t nwords = ((uint64_t) nbuf + 63) / 64;
            RowModel *rm = row_model_of(ws);
            // The workspace's last call was a row batch of this shape and its
            // first row fit the model: the model is still there and the bitmap
            // cleared, so the probe is skipped.  Any model is exact (a row
            // passes only by its own checks); a stale one only sends rows to
            // the fix-up, and its first row marked renews it next time.
            uint32_t *stale = rows_stale(slot);
            const RowsShape key{len, in_stride, out_stride, nbuf, a.p62, a.p63};
            if (!(held == key) || !stale || *(volatile uint32_t *) stale || capturing(stream)) {
                if (stale) *(volatile uint32_t *) stale = 0;
                hipLaunchKernelGGL(k_rows_prep, dim3(cap_grid((nwords + kThreads - 1) / kThreads,
                                                              (uint64_t) d->cus)),
                                   dim3(kThreads), 0, s, nbuf, (const uint8_t *) d_in,
                                   (uint32_t) len, in_stride, (uint32_t) S, out_stride, a, ws, rm);
                if ((err = launch_status())) {
                    ws_unpin(slot, stream);
                    return err;
                }
                path_taken(kPathRowsPrep);
            } else {
                path_taken(kPathRowsReuse);
            }
            // + S blocks: the row-group mapping rounds the rows up to whole
            // bands of U Ru rows (NB <= S blocks each); spare blocks return
            const dim3 g((uint32_t) ((slots + per - 1) / per + S));
            // 32-bit offsets within a block's rows (relmax / S + 1 rows at most)
            const uint64_t brows = relmax / S + 1;
            const bool o32 = in_stride < (1u << 24) && out_stride < (1u << 24) &&
                             brows * in_stride < (1ull << 31) && brows * out_stride < (1ull << 31);
            hipLaunchKernelGGL((o32 ? k_decode_rows_lines<U, true> : k_decode_rows_lines<U, false>),
                               g, dim3(kThreads), 0, s,
                               (const uint8_t *) d_in, in_stride, (uint32_t) len, (uint8_t *) d_out,
                               out_stride, (uint32_t) S, magic, m64, slots, tail_slot, a, nbuf, ws,
                               (const RowModel *) rm);
            if ((err = launch_status())) {
                ws_unpin(slot, stream);
                return err;
            }
            const uint32_t fg = cap_grid(((uint64_t) nbuf + 64 * kWavesPerBlock - 1) /
                                         (64 * kWavesPerBlock), (uint64_t) d->cus * 8);
            hipLaunchKernelGGL(k_rows_finish, dim3(fg), dim3(kThreads), 0, s,
                               (const uint8_t *) d_in, (uint8_t *) d_out, L, nbuf, d_outlen, a, ws,
                               (const RowModel *) rm, stale);
            err = launch_status();
            ws_unpin(slot, stream, err ? RowsShape{} : key);
            return err;
        } else if (err && err != -EBUSY) {
            return err;
        }
        // -EBUSY (every library workspace pinned by calls being enqueued, or
        // a capture on a stream that holds none): the general path below
        // needs no workspace
        err = 0;
    }
    if (!done && (err = hip_err(hipMemsetAsync(d_outlen, 0, (size_t) nbuf * 8, s)))) return err;
    if (!done && slots) {
        // any other layout: one lane per (buffer, 16-character slot)
        constexpr int U = 2;
        const uint64_t per_block = (uint64_t) kThreads * U;
        const dim3 g((uint32_t) ((slots + per_block - 1) / per_block));
        hipLaunchKernelGGL(k_decode_slots<U>, g, dim3(kThreads), 0, s, (const uint8_t *) d_in,
                           in_stride, len, (uint8_t *) d_out, out_stride,
                           (unsigned long long *) d_outlen, (uint32_t) S, (uint32_t) slots, a);
        if ((err = launch_status())) return err;
    }
    uint32_t fgrid = cap_grid(((uint64_t) nbuf + 64 * kWavesPerBlock - 1) / (64 * kWavesPerBlock),
                              (uint64_t) d->cus * 8);
    hipLaunchKernelGGL(k_decode_batch_fix2<false>, dim3(fgrid), dim3(kThreads), 0, s,
                       (const uint8_t *) d_in, (uint8_t *) d_out, L, nbuf, d_outlen, a);
    return launch_status();
}

int b64x_decode_batch(const void *d_in, const uint64_t *d_in_off, uint32_t nbuf,
                      void *d_out, const uint64_t *d_out_off, uint64_t *d_outlen,
                      const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0) return 0;
    if (!d_in || !d_in_off || !d_out || !d_out_off || !d_outlen) return -EINVAL;
    BatchLayout L{d_in_off, d_out_off, 0, 0, 0, 0, nullptr};
    return launch_batch_decode(d_in, L, nbuf, d_out, d_outlen, abc, stream);
}

int b64x_fill_splitmix64(void *d_out, uint64_t n, uint64_t seed, void *stream)
{
    if (n == 0) return 0;
    if (!d_out) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    uint64_t words = (n + 7) / 8;
    uint32_t grid = cap_grid((words + kThreads - 1) / kThreads, (uint64_t) d->cus * 8);
    hipLaunchKernelGGL(k_fill_splitmix64, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (uint8_t *) d_out, n, seed);
    return launch_status();
}

// ------------------------------------------------------------- sessions --

struct b64x_session {
    int device;
    hipStream_t stream;
    uint64_t cap;
    uint8_t *h_in, *h_out;
    uint8_t *h_base;     // h_in - kSessionHead (pinned, for in-place decodes)
    uint8_t *d_base;     // d_in - kSessionHead
    uint64_t last_len;   // characters of the last decode (0: none yet)
    bool dec_staged;     // the last decode found junk throughout: stage the next
    uint64_t res_len;    // characters, flags and sequence number of the last
    unsigned res_flags;  // decode, for the result check
    uint32_t res_seq;    // (b64x_session_decode_result)
    uint8_t *d_in, *d_out;
    void *d_ws;
    b64x_dec_result *d_res, *h_res;
};

// ---- completion results: written by the kernels, checked by the host ----
//
// A session decode's result record is written by the kernel that computes
// it straight into the fine-grained host mirror (no D2H copy behind the
// kernels), the host poisons the mirror before every launch, and
// b64x_session_decode_result() checks every field: a record that is still
// poisoned or inconsistent is counted, the session's stream is waited for,
// and the record is checked again (-EIO if it is still wrong: loud, never a
// silently short stream).  The hub's lanes do the same for their batches
// (b64x_lane_*_check).  Round 1 read records that D2H copies had filled, and
// under load (600 decoder streams on one loop on per-stage sessions) a block
// was now and then served as empty from a well-formed "nothing decoded"
// record (profiles/r02_diag_notes.md).  The check itself is
// b64x_result_check.h, shared with the CPU stage tests.
static std::atomic<uint64_t> g_early_session{0}, g_early_lane{0};

// Device headroom in front of d_in (kept for the decode kernels' vector
// loads, which may start below an unaligned input).
constexpr uint64_t kSessionHead = 256;
// Pinned slack after host_in: the decode kernels' last vector loads may
// reach past the input, harmless in a page-rounded hipMalloc, not assumed
// of host memory read in place.
constexpr uint64_t kSessionTail = 64;

static uint64_t session_out_cap(uint64_t cap)
{
    uint64_t e = b64x_encoded_len(cap, true), dcap = b64x_decoded_cap(cap);
    return e > dcap ? e : dcap;
}

// A session's pinned buffers are fine-grained (hipHostMallocCoherent).
// host_in/host_out are read and written in place by the kernels (zero-copy),
// and host_res is the target of the last small D2H copy before the
// completion callback once the output copy is gone; fine-grained memory is
// never held in an XCD's L2, so no fence scope can leave the host a stale
// line.  Defensive: the rates are unchanged (resident decode blocks 28.1 ->
// 27.8, encode 31.0 -> 30.9 GiB/s).  It did NOT cure the intermittent
// missing-block bug of the 600-stream decoder ingress (known
// issues; tests/tools/stress_ingress.py).
constexpr unsigned kSessionHostFlags = hipHostMallocCoherent;

b64x_session *b64x_session_open(uint64_t capacity)
{
    if (capacity == 0) {
        errno = EINVAL;
        return nullptr;
    }
    if (!device_info()) {
        errno = ENODEV;
        return nullptr;
    }
    b64x_session *s = (b64x_session *) calloc(1, sizeof(*s));
    if (!s) return nullptr;
    s->cap = capacity;
    (void) hipGetDevice(&s->device);
    const uint64_t ocap = session_out_cap(capacity);
    const uint64_t wsz = b64x_decode_workspace_size(capacity);
    bool ok = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
              hipHostMalloc((void **) &s->h_base, kSessionHead + capacity + kSessionTail,
                            kSessionHostFlags) == hipSuccess &&
              hipHostMalloc((void **) &s->h_out, ocap, kSessionHostFlags) == hipSuccess &&
              hipHostMalloc((void **) &s->h_res, sizeof(b64x_dec_result), kSessionHostFlags) == hipSuccess &&
              hipMalloc((void **) &s->d_base, kSessionHead + capacity) == hipSuccess &&
              hipMalloc((void **) &s->d_out, ocap) == hipSuccess &&
              hipMalloc((void **) &s->d_res, sizeof(b64x_dec_result)) == hipSuccess &&
              hipMalloc(&s->d_ws, wsz) == hipSuccess &&
              hipMemset(s->d_ws, 0, wsz) == hipSuccess;
    if (!ok) {
        b64x_session_close(s);
        errno = ENOMEM;
        return nullptr;
    }
    s->d_in = s->d_base + kSessionHead;
    s->h_in = s->h_base + kSessionHead;
    return s;
}

void b64x_session_close(b64x_session *s)
{
    if (!s) return;
    int prev = 0;
    (void) hipGetDevice(&prev);
    (void) hipSetDevice(s->device);
    if (s->stream) (void) hipStreamSynchronize(s->stream);
    if (s->h_base) (void) hipHostFree(s->h_base);
    if (s->h_out) (void) hipHostFree(s->h_out);
    if (s->h_res) (void) hipHostFree(s->h_res);
    if (s->d_base) (void) hipFree(s->d_base);
    if (s->d_out) (void) hipFree(s->d_out);
    if (s->d_res) (void) hipFree(s->d_res);
    if (s->d_ws) (void) hipFree(s->d_ws);
    if (s->stream) (void) hipStreamDestroy(s->stream);
    (void) hipSetDevice(prev);
    free(s);
}

uint64_t b64x_session_capacity(const b64x_session *s) { return s ? s->cap : 0; }

// Idle sessions, any device / capacity; at most kPoolMax kept.
static std::mutex g_pool_mu;
static b64x_session *g_pool[64];
static int g_npool;
constexpr int kPoolMax = 64;

static bool pool_enabled()
{
    static const bool on = [] {
        const char *v = getenv("ASYNC_B64_SESSION_POOL");
        return !(v && v[0] == '0');
    }();
    return on;
}

b64x_session *b64x_session_acquire(uint64_t capacity)
{
    int dev = 0;
    if (pool_enabled() && hipGetDevice(&dev) == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (int i = g_npool - 1; i >= 0; i--) {
            b64x_session *s = g_pool[i];
            if (s->device == dev && s->cap == capacity) {
                g_pool[i] = g_pool[--g_npool];
                return s;
            }
        }
    }
    return b64x_session_open(capacity);
}

void b64x_session_release(b64x_session *s)
{
    if (!s) return;
    if (pool_enabled() && b64x_session_wait(s) == 0) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_npool < kPoolMax) {
            g_pool[g_npool++] = s;
            return;
        }
    }
    b64x_session_close(s);
}
uint8_t *b64x_session_host_in(b64x_session *s) { return s ? s->h_in : nullptr; }
uint8_t *b64x_session_host_out(b64x_session *s) { return s ? s->h_out : nullptr; }

int b64x_session_encode(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                        uint64_t *out_len)
{
    if (!s || n > s->cap || !out_len) return -EINVAL;
    *out_len = 0;
    int err;
    if ((err = b64x_session_encode_async(s, n, abc, nullptr, nullptr))) return err;
    if ((err = b64x_session_wait(s))) return err;
    *out_len = n ? b64x_encoded_len(n, enc_alpha(abc).pad) : 0;
    return 0;
}

int b64x_session_decode(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                        unsigned flags, b64x_dec_result *res)
{
    if (!s || n > s->cap || !res) return -EINVAL;
    memset(res, 0, sizeof(*res));
    int err;
    if ((err = b64x_session_decode_async(s, n, abc, flags, nullptr, nullptr))) return err;
    if ((err = b64x_session_wait(s))) return err;
    return b64x_session_decode_result(s, res);
}

// A session's encode reads and writes its pinned host buffers in place over
// PCIe (zero-copy) instead of H2D, kernel, D2H: each byte crosses PCIe once
// either way, but one kernel's reads and writes overlap (duplex) and nothing
// is staged through HBM -- 30 GiB/s of payload against 22 staged for 32 MiB
// blocks (bench_host_pipeline resident_encode; scripts/bench_zero_copy.py).
// Not for the hub's ragged batches: one block per job is PCIe-latency-bound
// in place (a single 1 MiB stream ran at half the staged rate).
// ASYNC_B64_ZERO_COPY=0 stages sessions too.
static bool zero_copy_sessions()
{
    static const bool on = [] {
        const char *v = getenv("ASYNC_B64_ZERO_COPY");
        return !(v && v[0] == '0');
    }();
    return on;
}

int b64x_session_encode_async(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                              b64x_done_fn done, void *arg)
{
    if (!s || n > s->cap) return -EINVAL;
    int err;
    if ((err = hip_err(hipSetDevice(s->device)))) return err;
    if (n && zero_copy_sessions()) {
        if ((err = b64x_encode_dev(s->h_in, n, s->h_out, abc, s->stream))) return err;
    } else if (n) {
        const uint64_t m = b64x_encoded_len(n, enc_alpha(abc).pad);
        if ((err = hip_err(hipMemcpyAsync(s->d_in, s->h_in, n, hipMemcpyHostToDevice, s->stream)))) return err;
        if ((err = b64x_encode_dev(s->d_in, n, s->d_out, abc, s->stream))) return err;
        if ((err = hip_err(hipMemcpyAsync(s->h_out, s->d_out, m, hipMemcpyDeviceToHost, s->stream)))) return err;
    }
    if (done) return hip_err(hipLaunchHostFunc(s->stream, done, arg));
    return 0;
}

// A session's decode reads host_in and writes host_out in place over PCIe
// too, unless its last decode found junk throughout (MIME line breaks):
// pass 2 re-reads the input and pass-1 output where junk is, which in place
// means a second PCIe crossing.  Clean 256 MiB blocks 22.6 -> 34.5 GiB/s,
// CRLF-76 ones 21.6 staged against 17.7 in place (scripts/bench_zero_copy.py).
// The result of the last decode is consulted only once the session's stream
// has drained, so the policy never waits and never reads a result in flight.
// ASYNC_B64_ZERO_COPY=0 stages every decode as well.
constexpr uint64_t kZeroCopyJunk = 80;  // skipped characters that make the next decode staged

static bool decode_in_place(b64x_session *s)
{
    if (!zero_copy_sessions()) return false;
    b64x_dec_result r;
    if (s->last_len && hipStreamQuery(s->stream) == hipSuccess &&
        b64x_result_ok(s->h_res, s->res_len, s->res_flags, s->res_seq, &r)) {
        const uint64_t junk = s->last_len - (r.valid < s->last_len ? r.valid : s->last_len);
        s->dec_staged = junk > kZeroCopyJunk;
        s->last_len = 0;
    }
    return !s->dec_staged;
}

// Round 1 chained a stream's blocks over sessions on the device (a carry
// spelled by a kernel on the previous session's stream, a cross-stream
// event, the record copied D2H behind the kernels), and a block was once in
// a while served as empty from a well-formed "nothing decoded" record.  That
// chaining is gone: a session decode is H2D (or in place),
// the kernels and the completion, all on the session's own stream, and the
// record the kernels write into host memory names this call (n, flags and
// a fresh sequence number), so no earlier or zero-filled record passes the
// check.
int b64x_session_decode_async(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                              unsigned flags, b64x_done_fn done, void *arg)
{
    if (!s || n > s->cap) return -EINVAL;
    int err;
    if ((err = hip_err(hipSetDevice(s->device)))) return err;
    const bool in_place = decode_in_place(s);
    uint8_t *in = in_place ? s->h_in : s->d_in;
    uint8_t *out = in_place ? s->h_out : s->d_out;
    if (n && !in_place &&
        (err = hip_err(hipMemcpyAsync(s->d_in, s->h_in, n, hipMemcpyHostToDevice, s->stream))))
        return err;
    b64x_poison_result(s->h_res);
    s->res_len = n;
    s->res_flags = flags;
    s->res_seq = next_seq();
    if ((err = decode_dev_impl(in, n, out, s->d_res, s->h_res, abc, flags, s->d_ws, s->stream,
                               s->res_seq)))
        return err;
    s->last_len = n;
    // The output length is device-determined: copy the capacity bound.
    if (n && !in_place &&
        (err = hip_err(hipMemcpyAsync(s->h_out, s->d_out, b64x_decoded_cap(n),
                                      hipMemcpyDeviceToHost, s->stream))))
        return err;
    if (done) return hip_err(hipLaunchHostFunc(s->stream, done, arg));
    return 0;
}

const b64x_dec_result *b64x_session_result(const b64x_session *s)
{
    return s ? s->h_res : nullptr;
}

int b64x_session_decode_result(b64x_session *s, b64x_dec_result *res)
{
    if (!s || !res) return -EINVAL;
    if (b64x_result_ok(s->h_res, s->res_len, s->res_flags, s->res_seq, res)) return 0;
    g_early_session.fetch_add(1, std::memory_order_relaxed);
    int err = b64x_session_wait(s);
    if (err) return err;
    const bool ok = b64x_result_ok(s->h_res, s->res_len, s->res_flags, s->res_seq, res);
    return ok ? 0 : -EIO;
}

void b64x_diag_counters(uint64_t out[2])
{
    out[0] = g_early_session.load(std::memory_order_relaxed);
    out[1] = g_early_lane.load(std::memory_order_relaxed);
}

int b64x_session_wait(b64x_session *s)
{
    if (!s) return -EINVAL;
    return hip_err(hipStreamSynchronize(s->stream));
}

// ------------------------------------------------------------ batch lanes --

void *b64x_host_alloc(uint64_t bytes)
{
    void *p = nullptr;
    if (!device_info()) return nullptr;
    // Fine-grained, like a session's buffers: a lane's decode batch ends on a
    // small D2H copy of the output lengths right before its host callback
    // (see kSessionHostFlags).
    if (hipHostMalloc(&p, bytes ? bytes : 1, kSessionHostFlags) != hipSuccess) return nullptr;
    return p;
}

void b64x_host_free(void *p)
{
    if (p) (void) hipHostFree(p);
}

// A lane's batches read their input from device memory (one H2D copy of the
// arena) and write their outputs -- characters, bytes and the decode jobs'
// result records -- straight into the pinned host arena: no D2H copy.  The
// host checks every batch once its completion callback has run: decode
// records were poisoned before the launch (b64x_lane_decode_check), and an
// encode batch ends with a kernel that stamps the lane's sequence number
// into host memory (b64x_lane_encode_check).  Round 1's D2H copies of
// results are what lost blocks under load.
struct b64x_lane {
    int device;
    hipStream_t stream;
    uint8_t *d_in;
    uint64_t *d_offs;     // in_off | out_off | vcount (decode) words
    uint8_t *d_flags;
    uint64_t *h_stamp;    // fine-grained pinned: the last finished encode batch
    uint64_t seq;         // the last encode batch queued
    uint64_t in_cap, offs_cap, flags_cap;  // bytes allocated
    b64x_seg *d_seg;      // an encode batch's lent segments (k_gather_host)
    uint64_t seg_cap;
    b64x_dec_result *d_res;  // big decode jobs: the pipeline's record ...
    void *d_ws;              // ... and workspace (allocated at the first)
};

b64x_lane *b64x_lane_open(void)
{
    if (!device_info()) {
        errno = ENODEV;
        return nullptr;
    }
    b64x_lane *l = (b64x_lane *) calloc(1, sizeof(*l));
    if (!l) return nullptr;
    (void) hipGetDevice(&l->device);
    if (hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking) != hipSuccess) {
        free(l);
        errno = EIO;
        return nullptr;
    }
    if (hipHostMalloc((void **) &l->h_stamp, sizeof(uint64_t), kSessionHostFlags) != hipSuccess) {
        (void) hipStreamDestroy(l->stream);
        free(l);
        errno = ENOMEM;
        return nullptr;
    }
    *l->h_stamp = 0;
    return l;
}

void b64x_lane_close(b64x_lane *l)
{
    if (!l) return;
    (void) hipSetDevice(l->device);
    (void) hipStreamSynchronize(l->stream);
    if (l->d_in) (void) hipFree(l->d_in);
    if (l->d_offs) (void) hipFree(l->d_offs);
    if (l->d_flags) (void) hipFree(l->d_flags);
    if (l->d_seg) (void) hipFree(l->d_seg);
    if (l->d_res) (void) hipFree(l->d_res);
    if (l->d_ws) (void) hipFree(l->d_ws);
    if (l->h_stamp) (void) hipHostFree(l->h_stamp);
    (void) hipStreamDestroy(l->stream);
    free(l);
}

static b64x_lane *g_lane_pool[64];
static int g_nlane_pool;

b64x_lane *b64x_lane_acquire(void)
{
    int dev = 0;
    if (pool_enabled() && hipGetDevice(&dev) == hipSuccess) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (int i = g_nlane_pool - 1; i >= 0; i--) {
            b64x_lane *l = g_lane_pool[i];
            if (l->device == dev) {
                g_lane_pool[i] = g_lane_pool[--g_nlane_pool];
                return l;
            }
        }
    }
    return b64x_lane_open();
}

void b64x_lane_release(b64x_lane *l)
{
    if (!l) return;
    if (pool_enabled() && b64x_lane_wait(l) == 0) {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_nlane_pool < kPoolMax) {
            g_lane_pool[g_nlane_pool++] = l;
            return;
        }
    }
    b64x_lane_close(l);
}

// Grow a device buffer to at least `need`, and on first use at least to
// `floor`: the size the hub's default batches need (16 MiB arenas, 2^16 jobs,
// 2^14 lent segments), so that a lane taken from the pool by another loop
// does not grow under load.  Growing synchronises the lane's stream and
// frees the old buffer (hipFree waits for the whole device); under config 5
// on 16 loops the lanes' growth and the arenas' allocation made passes
// 10-20 % slower now and then.
constexpr uint64_t kLaneInFloor = (16u << 20) + (1u << 20);
constexpr uint64_t kLaneOffsFloor = 3ull * ((1u << 16) + 1) * 8;
constexpr uint64_t kLaneFlagsFloor = (1u << 16) + 64;
constexpr uint64_t kLaneSegFloor = (1u << 14) * sizeof(b64x_seg);
static int lane_grow(b64x_lane *l, void **buf, uint64_t *cap, uint64_t need, uint64_t floor)
{
    if (need <= *cap) return 0;
    uint64_t want = need + need / 4 + (1u << 20);
    if (want < floor) want = floor;
    int err;
    if ((err = hip_err(hipStreamSynchronize(l->stream)))) return err;
    if (*buf) (void) hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    if (hipMalloc(buf, want) != hipSuccess) return -ENOMEM;
    *cap = want;
    return 0;
}

// Offsets (and, for decode, the per-job counts) and the input on the device
// (h_in NULL: the offsets only).
static int lane_stage_in(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                         const uint64_t *h_in_off, const uint64_t *h_out_off, uint64_t words_extra)
{
    const uint64_t in_bytes = h_in_off[njobs];
    const uint64_t words = (uint64_t) njobs + 1;
    int err;
    if ((err = lane_grow(l, (void **) &l->d_in, &l->in_cap, in_bytes + 64, kLaneInFloor))) return err;
    if ((err = lane_grow(l, (void **) &l->d_offs, &l->offs_cap, (2 * words + words_extra) * 8,
                          kLaneOffsFloor)))
        return err;
    if ((err = hip_err(hipMemcpyAsync(l->d_offs, h_in_off, words * 8, hipMemcpyHostToDevice,
                                      l->stream))) ||
        (err = hip_err(hipMemcpyAsync(l->d_offs + words, h_out_off, words * 8,
                                      hipMemcpyHostToDevice, l->stream))))
        return err;
    if (h_in && in_bytes && (err = hip_err(hipMemcpyAsync(l->d_in, h_in, in_bytes,
                                                          hipMemcpyHostToDevice, l->stream))))
        return err;
    return 0;
}

// Copy host bytes [sa, se) to device bytes from d on (any alignments):
// aligned 16-byte loads of the host range (host memory is not cached: each
// byte crosses the link once), byte stores (device memory; a few store
// instructions per 16 bytes -- the link, not the stores, bounds this).
// Block-wide.
DEV void copy_from_host(const uint8_t *sa, const uint8_t *se, uint8_t *d)
{
    const uintptr_t u0 = (uintptr_t) sa & ~(uintptr_t) 15;
    uint8_t *dd = d - (uintptr_t) sa;  // dd[(uintptr_t) p]: the device byte of host p
    for (uintptr_t u = u0 + 16 * threadIdx.x; u < (uintptr_t) se; u += 16 * kThreads) {
        const uint4 v = *(const uint4 *) u;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
            const uintptr_t p = u + k;
            if (p >= (uintptr_t) sa && p < (uintptr_t) se) dd[p] = (uint8_t) (w[k >> 2] >> (8 * (k & 3)));
        }
    }
}

// A batch with lent segments into the device: block b covers device bytes
// [b T, (b+1) T) of the batch, finds the first segment ending past its
// start by a binary search over the segment table (copied to the device
// first: a search over host memory would pay the link's latency per step),
// and copies its bytes from the segments' sources or, between segments,
// from the arena h_in -- both read straight from pinned host memory.
constexpr uint32_t kGatherTile = 64u << 10;
__global__ __launch_bounds__(kThreads) void k_gather_host(
    uint8_t *__restrict__ d_in, const uint8_t *__restrict__ h_in, uint64_t total,
    const b64x_seg *__restrict__ seg, uint32_t nseg)
{
    __shared__ uint32_t s_i0;
    const uint64_t lo = (uint64_t) blockIdx.x * kGatherTile;
    const uint64_t hi = lo + kGatherTile < total ? lo + kGatherTile : total;
    if (threadIdx.x == 0) {  // the first segment ending past lo (nseg if none)
        uint32_t a = 0, b = nseg;
        while (a < b) {
            const uint32_t m = (a + b) / 2;
            if (seg[m].off + seg[m].len > lo) b = m;
            else a = m + 1;
        }
        s_i0 = a;
    }
    block_sync();
    uint64_t p = lo;
    for (uint32_t i = s_i0; p < hi; i++) {
        const uint64_t so = i < nseg ? seg[i].off : hi, se = i < nseg ? seg[i].off + seg[i].len : hi;
        const uint64_t gap_end = so < hi ? so : hi;  // arena bytes before the segment
        if (p < gap_end) {
            copy_from_host(h_in + p, h_in + gap_end, d_in + p);
            p = gap_end;
        }
        if (p >= hi) break;
        const uint64_t e = se < hi ? se : hi;
        copy_from_host(seg[i].src + (p - so), seg[i].src + (e - so), d_in + p);
        p = e;
    }
}

int b64x_lane_encode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const b64x_seg *h_seg, uint32_t nseg,
                           const b64x_alphabet *abc, b64x_done_fn done, void *arg)
{
    if (!l || (njobs && (!h_in || !h_in_off || !h_out || !h_out_off)) || (nseg && !h_seg))
        return -EINVAL;
    int err;
    if ((err = hip_err(hipSetDevice(l->device)))) return err;
    if (njobs) {
        const uint64_t words = (uint64_t) njobs + 1;
        const uint64_t in_bytes = h_in_off[njobs];
        for (uint32_t i = 0; i < nseg; i++)  // sorted, inside the batch
            if (h_seg[i].off + h_seg[i].len > in_bytes || (i && h_seg[i].off < h_seg[i - 1].off + h_seg[i - 1].len))
                return -EINVAL;
        if ((err = lane_stage_in(l, nseg ? nullptr : h_in, njobs, h_in_off, h_out_off, 0)))
            return err;
        if (nseg && in_bytes) {
            if ((err = lane_grow(l, (void **) &l->d_seg, &l->seg_cap, (uint64_t) nseg * sizeof(b64x_seg),
                               kLaneSegFloor)) ||
                (err = hip_err(hipMemcpyAsync(l->d_seg, h_seg, (size_t) nseg * sizeof(b64x_seg),
                                              hipMemcpyHostToDevice, l->stream))))
                return err;
            hipLaunchKernelGGL(k_gather_host, dim3((uint32_t) ((in_bytes + kGatherTile - 1) / kGatherTile)),
                               dim3(kThreads), 0, l->stream, l->d_in, h_in, in_bytes,
                               (const b64x_seg *) l->d_seg, nseg);
            if ((err = launch_status())) return err;
        }
        if ((err = b64x_encode_batch(l->d_in, l->d_offs, njobs, h_out, l->d_offs + words, abc,
                                     l->stream)))
            return err;
    }
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, l->stream, l->h_stamp, ++l->seq);
    if ((err = launch_status())) return err;
    if (done) return hip_err(hipLaunchHostFunc(l->stream, done, arg));
    return 0;
}

int b64x_lane_encode_check(b64x_lane *l)
{
    if (!l) return -EINVAL;
    if (*(volatile uint64_t *) l->h_stamp == l->seq) return 0;
    g_early_lane.fetch_add(1, std::memory_order_relaxed);
    int err = b64x_lane_wait(l);
    if (err) return err;
    return *(volatile uint64_t *) l->h_stamp == l->seq ? 0 : -EIO;
}

// Hub decode jobs this long go through the single-buffer pipeline.
static constexpr uint64_t kBigJob = 128u << 10;

int b64x_lane_decode_async(b64x_lane *l, const uint8_t *h_in, uint32_t njobs,
                           const uint64_t *h_in_off, uint8_t *h_out,
                           const uint64_t *h_out_off, const uint8_t *h_flags,
                           b64x_dec_result *h_res, const b64x_dec_result *const *h_prev,
                           b64x_dec_result *h_spell, const b64x_alphabet *abc,
                           b64x_done_fn done, void *arg, uint32_t *seq)
{
    if (!l || !seq || (njobs && (!h_in || !h_in_off || !h_out || !h_out_off || !h_flags || !h_res)))
        return -EINVAL;
    for (uint32_t j = 0; j < njobs; j++)
        if ((h_flags[j] & B64X_LANE_CHAINED) &&
            (!h_prev || !h_prev[j] || !h_spell || h_in_off[j + 1] - h_in_off[j] < 4))
            return -EINVAL;
    int err;
    if ((err = hip_err(hipSetDevice(l->device)))) return err;
    *seq = next_seq();
    if (njobs) {
        const uint64_t words = (uint64_t) njobs + 1;
        for (uint32_t j = 0; j < njobs; j++) b64x_poison_result(h_res + j);
        if ((err = lane_stage_in(l, h_in, njobs, h_in_off, h_out_off, words))) return err;
        if ((err = lane_grow(l, (void **) &l->d_flags, &l->flags_cap, njobs, kLaneFlagsFloor))) return err;
        if ((err = hip_err(hipMemcpyAsync(l->d_flags, h_flags, njobs, hipMemcpyHostToDevice,
                                          l->stream))))
            return err;
        uint64_t *d_in_off = l->d_offs, *d_out_off = l->d_offs + words,
                 *d_vcount = l->d_offs + 2 * words;
        // Jobs of kBigJob characters or more (whole stage blocks) would each
        // keep one wave of the batch kernel busy for hundreds of us: they
        // take the single-buffer pipeline instead, in job order on the lane's
        // stream, which writes their records itself; so do chained jobs,
        // whose heads are spelled between their predecessor's decode and
        // their own.  The batch kernels skip both.
        uint32_t npiped = 0;
        for (uint32_t j = 0; j < njobs; j++)
            npiped += h_in_off[j + 1] - h_in_off[j] >= kBigJob || (h_flags[j] & B64X_LANE_CHAINED);
        const BatchLayout L{d_in_off, d_out_off, 0, 0, 0, kBigJob, (const uint8_t *) l->d_flags};
        const uint8_t *src = h_in_off[njobs] ? l->d_in : (const uint8_t *) l->d_offs;
        const DecAlpha da = dec_alpha(abc);
        if (npiped < njobs) {
            if ((err = launch_batch_decode(src, L, njobs, h_out, d_vcount, abc, l->stream, true)))
                return err;
            const DeviceInfo *d = device_info();
            const uint32_t grid = cap_grid((njobs + kWavesPerBlock - 1) / kWavesPerBlock,
                                           (uint64_t) d->cus * 8);
            hipLaunchKernelGGL(k_batch_finish, dim3(grid), dim3(kThreads), 0, l->stream, src,
                               d_in_off, (const uint8_t *) l->d_flags,
                               (const uint64_t *) d_vcount, njobs, kBigJob, da, h_res, *seq);
            if ((err = launch_status())) return err;
        }
        if (npiped && !l->d_ws) {
            const uint64_t wsz = b64x_decode_workspace_size(0);
            if (!l->d_res && hipMalloc(&l->d_res, sizeof *l->d_res) != hipSuccess) {
                l->d_res = nullptr;
                return -ENOMEM;
            }
            if (hipMalloc(&l->d_ws, wsz) != hipSuccess) {
                l->d_ws = nullptr;
                return -ENOMEM;
            }
            if ((err = hip_err(hipMemsetAsync(l->d_ws, 0, wsz, l->stream)))) return err;
        }
        for (uint32_t j = 0; npiped && j < njobs; j++) {
            const uint64_t n = h_in_off[j + 1] - h_in_off[j];
            const bool chained = h_flags[j] & B64X_LANE_CHAINED;
            if (n < kBigJob && !chained) continue;
            if (chained) {
                hipLaunchKernelGGL(k_spell_head, dim3(1), dim3(64), 0, l->stream,
                                   l->d_in + h_in_off[j], h_prev[j], h_spell + j, da);
                if ((err = launch_status())) return err;
            }
            if ((err = decode_dev_impl(l->d_in + h_in_off[j], n, h_out + h_out_off[j], l->d_res,
                                       h_res + j, abc, h_flags[j] & 1 ? B64X_DEC_HOLD_TAIL : 0,
                                       l->d_ws, l->stream, *seq)))
                return err;
        }
    }
    if (done) return hip_err(hipLaunchHostFunc(l->stream, done, arg));
    return 0;
}

int b64x_lane_wait(b64x_lane *l)
{
    if (!l) return -EINVAL;
    return hip_err(hipStreamSynchronize(l->stream));
}

// Every record is this batch's and consistent; every chained job's head was
// spelled from its predecessor's finished record (checked before it: the
// predecessor is an earlier job of this batch or of a batch before it).
static bool jobs_ok(const uint64_t *h_in_off, const uint8_t *h_flags,
                    const b64x_dec_result *h_res, const b64x_dec_result *const *h_prev,
                    const b64x_dec_result *h_spell, uint32_t njobs, uint32_t seq)
{
    for (uint32_t j = 0; j < njobs; j++) {
        if (!b64x_result_ok(h_res + j, h_in_off[j + 1] - h_in_off[j], h_flags[j] & 1, seq,
                            nullptr))
            return false;
        if ((h_flags[j] & B64X_LANE_CHAINED) && !b64x_spell_ok(h_spell + j, h_prev[j]))
            return false;
    }
    return true;
}

int b64x_lane_decode_check(b64x_lane *l, uint32_t seq, const uint64_t *h_in_off,
                           const uint8_t *h_flags, const b64x_dec_result *h_res,
                           const b64x_dec_result *const *h_prev,
                           const b64x_dec_result *h_spell, uint32_t njobs)
{
    if (!l || (njobs && (!h_in_off || !h_flags || !h_res))) return -EINVAL;
    if (jobs_ok(h_in_off, h_flags, h_res, h_prev, h_spell, njobs, seq)) return 0;
    g_early_lane.fetch_add(1, std::memory_order_relaxed);
    int err = b64x_lane_wait(l);
    if (err) return err;
    return jobs_ok(h_in_off, h_flags, h_res, h_prev, h_spell, njobs, seq) ? 0 : -EIO;
}

#ifdef B64X_TEST_HOOKS
// Test builds only: the copy ceiling bench.py reads the roofline against
// (SURVEY.md 8(d)): 16-byte loads and stores, U per lane in flight, a
// non-persistent grid of TH-thread blocks -- the kernels' own access shape
// with no arithmetic (mode 0: U = 4, TH = 256, non-temporal; the other modes
// are the shapes b64x__test_copy_mode sweeps).  n a multiple of
// 16 * TH * U, buffers 16-byte aligned.
extern "C++" {
template <int U, int TH, bool NT>
__global__ __launch_bounds__(TH) void k_test_copy(const uint8_t *__restrict__ in,
                                                  uint8_t *__restrict__ out)
{
    const uint64_t base = (uint64_t) blockIdx.x * TH * U * 16 + 16 * threadIdx.x;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld16<NT>(in + base + (uint64_t) u * TH * 16);
#pragma unroll
    for (int u = 0; u < U; u++) store16<NT>(out + base + (uint64_t) u * TH * 16, v[u]);
}

template <int U, int TH, bool NT>
static int test_copy(const void *src, void *dst, uint64_t n, void *stream)
{
    const uint64_t per = (uint64_t) TH * U * 16;
    if (n % per || ((((uintptr_t) src) | ((uintptr_t) dst)) & 15)) return -EINVAL;
    hipLaunchKernelGGL((k_test_copy<U, TH, NT>), dim3((uint32_t) (n / per)), dim3(TH), 0,
                       (hipStream_t) stream, (const uint8_t *) src, (uint8_t *) dst);
    return launch_status();
}
}  // extern "C++"

int b64x__test_copy_mode(const void *src, void *dst, uint64_t n, void *stream, int mode)
{
    switch (mode) {
    case 0: return test_copy<4, 256, true>(src, dst, n, stream);
    case 1: return test_copy<1, 256, true>(src, dst, n, stream);
    case 2: return test_copy<2, 256, true>(src, dst, n, stream);
    case 3: return test_copy<8, 256, true>(src, dst, n, stream);
    case 4: return test_copy<4, 512, true>(src, dst, n, stream);
    case 5: return test_copy<4, 1024, true>(src, dst, n, stream);
    case 6: return test_copy<4, 256, false>(src, dst, n, stream);
    case 7: return test_copy<2, 1024, true>(src, dst, n, stream);
    case 8: return test_copy<1, 1024, true>(src, dst, n, stream);
    default: return -EINVAL;
    }
}

int b64x__test_copy(const void *src, void *dst, uint64_t n, void *stream)
{
    return b64x__test_copy_mode(src, dst, n, stream, 0);
}

// Test builds only: copies with a kernel's own read/write mix, for the copy
// ceiling of each leg (bench.py): every lane loads IN bytes (dwordx3 or
// dwordx4, non-temporal) and stores OUT bytes, U of them in flight --
// encode's 12 -> 16 (3 : 4) and decode's 16 -> 12 (4 : 3), no arithmetic
// beyond one XOR that makes the stored dwords depend on the loaded ones.
// `units` lane-steps; one block of TH lanes takes TH * U of them.
extern "C++" {
template <int U, int TH, int IN, int OUT>
__global__ __launch_bounds__(TH) void k_test_mix(const uint8_t *__restrict__ in,
                                                 uint8_t *__restrict__ out)
{
    const uint64_t u0 = (uint64_t) blockIdx.x * TH * U + threadIdx.x;
    uint32_t v[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint8_t *p = in + (u0 + (uint64_t) u * TH) * (IN == 1612 ? 12 : IN);
        if (IN == 1612) {  // 16 bytes at a 12-byte stride (k_encode_tight2's loads)
            const u32x4a4 w = __builtin_nontemporal_load((const u32x4a4 *) p);
            v[u][0] = w.x, v[u][1] = w.y ^ w.w, v[u][2] = w.z, v[u][3] = w.x ^ w.z;
        } else if (IN == 16) {
            const uint4 w = ld16<true>(p);
            v[u][0] = w.x, v[u][1] = w.y, v[u][2] = w.z, v[u][3] = w.w;
        } else {
            const u32x3a4 w = ld12<true>(p);
            v[u][0] = w.x, v[u][1] = w.y, v[u][2] = w.z, v[u][3] = w.x ^ w.z;
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        uint8_t *q = out + (u0 + (uint64_t) u * TH) * OUT;
        if (OUT == 16)
            store16<true>(q, uint4{v[u][0], v[u][1], v[u][2], v[u][3]});
        else
            __builtin_nontemporal_store(u32x3a4{v[u][0], v[u][1] ^ v[u][3], v[u][2]},
                                        (u32x3a4 *) q);
    }
}

template <int U, int TH, int IN, int OUT>
static int test_mix(const void *src, void *dst, uint64_t units, void *stream)
{
    const uint64_t per = (uint64_t) TH * U;
    if (units % per || ((((uintptr_t) src) | ((uintptr_t) dst)) & 15)) return -EINVAL;
    hipLaunchKernelGGL((k_test_mix<U, TH, IN, OUT>), dim3((uint32_t) (units / per)), dim3(TH),
                       0, (hipStream_t) stream, (const uint8_t *) src, (uint8_t *) dst);
    return launch_status();
}
}  // extern "C++"

// mix 0: encode's 12 -> 16, mix 1: decode's 16 -> 12, mix 2: 16-byte loads
// at a 12-byte stride -> 16 (k_encode_tight2's shape); shape 0..2: U = 1, 2,
// 4 (TH = 256).  `units` must be a multiple of 256 * U.
int b64x__test_copy_mix(const void *src, void *dst, uint64_t units, void *stream, int mix,
                        int shape)
{
    switch (mix * 3 + shape) {
    case 0: return test_mix<1, 256, 12, 16>(src, dst, units, stream);
    case 1: return test_mix<2, 256, 12, 16>(src, dst, units, stream);
    case 2: return test_mix<4, 256, 12, 16>(src, dst, units, stream);
    case 3: return test_mix<1, 256, 16, 12>(src, dst, units, stream);
    case 4: return test_mix<2, 256, 16, 12>(src, dst, units, stream);
    case 5: return test_mix<4, 256, 16, 12>(src, dst, units, stream);
    case 6: return test_mix<1, 256, 1612, 16>(src, dst, units, stream);
    case 7: return test_mix<2, 256, 1612, 16>(src, dst, units, stream);
    case 8: return test_mix<4, 256, 1612, 16>(src, dst, units, stream);
    default: return -EINVAL;
    }
}

// Test builds only: decode ranges of `chunks` chunks (0 = the default);
// returns the previous setting.
uint64_t b64x__test_range_chunks(uint64_t chunks)
{
    const uint64_t old = g_test_range_chunks;
    g_test_range_chunks = chunks;
    return old;
}
#endif

const char *b64x_build_info(void)
{
#define B64X_STR2(x) #x
#define B64X_STR(x) B64X_STR2(x)
    return "b64x abi=" B64X_STR(B64X_ABI_VERSION) " arch=gfx950 enc:quad12->16 lds-alphabet "
           "1 quad/lane; dec:probe+line-model single pass (4 slots/lane) + exact suffix "
           "(decoded once, held until its prefix, group sums, LDS read-ahead); rows:line model in row "
           "bands; lanes:chained decoder blocks";
}

const char *b64x_strerror(int err)
{
    switch (err) {
    case 0: return "success";
    case -EINVAL: return "invalid argument";
    case -ENOMEM: return "out of memory";
    case -ENODEV: return "no usable gfx950 device";
    case -EIO: return "HIP runtime error";
    default: return "unknown error";
    }
}

}  // extern "C"
