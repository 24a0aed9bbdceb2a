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
// How it runs here (DESIGN.md §Kernels has the byte budget):
//   * encode is stateless per 3-byte group.  One lane turns 12 input bytes
//     (one dwordx3 load) into 16 characters (one dwordx4 store); the
//     64-entry alphabet sits in LDS and is read with ds_read_u8 (the whole
//     table is 16 dwords, so no two lanes ever hit one bank with different
//     dwords).  Byte regrouping is v_perm_b32, not shifts.
//   * decode is stateful only through the number of alphabet characters
//     seen so far.  A wave owns a contiguous range of the input and walks
//     it in 1024-character chunks (16 per lane, one dwordx4 load).  The
//     fast path -- chunk entirely alphabet, wave aligned to a 4-character
//     group -- maps through the 256-entry inverse table in LDS and stores
//     12 bytes per lane (dwordx3).  Anything else (junk, '=', CR/LF, a
//     partial chunk) takes the exact path: a wave-wide prefix sum of valid
//     counts compacts the sextets into the wave's LDS scratch, whole
//     4-sextet groups are emitted and 0-3 sextets carry to the next chunk.
//   * a single large buffer is split into one range per resident wave.
//     Pass 1 assumes every earlier range was all-alphabet (true for clean
//     input) and records each range's valid count; a one-block scan finds
//     the first range where that assumption broke and the true prefix;
//     pass 2 re-runs only the ranges after it.  Padding at the end of
//     clean input never triggers pass 2 (the last range is allowed to be
//     dirty).
//   * batches: encode flattens (buffer, 12-byte quad) onto lanes; decode
//     runs one wave per buffer.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "b64x.h"

#define DEV __device__ __forceinline__

namespace {

constexpr int kThreads = 256;  // 4 waves of 64
constexpr int kWavesPerBlock = kThreads / 64;
constexpr int kChunk = 1024;            // characters per wave step
constexpr int kSxBytes = 1088;          // per-wave sextet scratch in LDS
constexpr uint32_t kMaxRanges = 8192;   // decode ranges (waves) per call
constexpr uint64_t kMinRange = 4096;    // characters per range, at least
constexpr int kEncUnroll = 4;           // quads in flight per lane
constexpr int kDecUnroll = 4;           // chunks in flight per wave

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
    __syncthreads();

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

// Ragged batch: one block per buffer.
__global__ __launch_bounds__(kThreads) void k_encode_ragged(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
    uint32_t nbuf, uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off,
    EncAlpha a)
{
    __shared__ uint8_t tab[64];
    build_enc_table(tab, a);
    __syncthreads();
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

struct __attribute__((aligned(16))) DecSmem {
    uint8_t tab[256];
    uint8_t sx[kWavesPerBlock][kSxBytes];
};

DEV uint32_t lane_id() { return threadIdx.x & 63; }

DEV uint32_t wave_excl_scan(uint32_t x, uint32_t *total)
{
    const uint32_t lane = lane_id();
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(v, d, 64);
        if (lane >= (uint32_t) d) v += y;
    }
    *total = __shfl(v, 63, 64);
    return v - x;
}

// Keep the compiler from moving LDS accesses across this point.  Within
// one wave the LDS executes DS instructions in issue order, so program
// order is all that cross-lane hand-offs in the wave's scratch need.
DEV void wave_lds_order()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Four sextets (bits 23..0 of a group) from dword `d` holding them as
// bytes 0..3 in stream order.
DEV uint32_t group_of_bytes(uint32_t d)
{
    return ((d & 0xFFu) << 18) | (((d >> 8) & 0xFFu) << 12) |
           (((d >> 16) & 0xFFu) << 6) | (d >> 24);
}

// Four groups -> 12 output bytes as three little-endian dwords.
DEV void groups_to_bytes(uint32_t G0, uint32_t G1, uint32_t G2, uint32_t G3,
                         uint32_t &o0, uint32_t &o1, uint32_t &o2)
{
    o0 = __builtin_amdgcn_perm(G1, G0, 0x06000102u);  // G0.b2 G0.b1 G0.b0 G1.b2
    o1 = __builtin_amdgcn_perm(G2, G1, 0x05060001u);  // G1.b1 G1.b0 G2.b2 G2.b1
    o2 = __builtin_amdgcn_perm(G3, G2, 0x04050600u);  // G2.b0 G3.b2 G3.b1 G3.b0
}

DEV void store_bytes12(uint8_t *p, uint32_t o0, uint32_t o1, uint32_t o2,
                       uint32_t nbytes)
{
    if (nbytes == 12 && (((uintptr_t) p) & 3) == 0) {
        *(u32x3a4 *) p = u32x3a4{o0, o1, o2};
        return;
    }
    uint32_t w[3] = {o0, o1, o2};
#pragma unroll
    for (uint32_t i = 0; i < 12; i++)
        if (i < nbytes) p[i] = (uint8_t) (w[i >> 2] >> (8 * (i & 3)));
}

// Up to 16 characters at `p`, `nin` of which are inside the range.
// Missing characters read as 0, which is never in the alphabet; callers
// mask them out by position anyway.
DEV uint4 load_chars(const uint8_t *p, uint32_t nin)
{
    if (nin == 16) {
        if ((((uintptr_t) p) & 15) == 0) return *(const uint4 *) p;
        if ((((uintptr_t) p) & 3) == 0) {
            u32x4a4 v = *(const u32x4a4 *) p;
            return make_uint4(v.x, v.y, v.z, v.w);
        }
    }
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        if (i < nin) w[i >> 2] |= (uint32_t) p[i] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

struct LaneChunk {
    uint32_t t[16];  // table values (0..63, or 0xFF)
    uint32_t vmask;  // bit k: character k present and in the alphabet
};

DEV void map_chunk(const uint8_t *tab, uint4 w, uint32_t nin, LaneChunk &lc)
{
    const uint32_t dw[4] = {w.x, w.y, w.z, w.w};
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint32_t c = (dw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        lc.t[k] = tab[c];
        m |= (lc.t[k] < 64u ? 1u : 0u) << k;
    }
    lc.vmask = m & (nin >= 16 ? 0xFFFFu : ((1u << nin) - 1u));
}

struct RangeState {
    int carry;        // sextets waiting in sx[0..carry); < 0: still to skip
    uint64_t groups;  // whole groups emitted (3 bytes each) from `out`
    uint64_t valid;   // alphabet characters seen in the range
};

// Exact path for one chunk: compact, emit whole groups, keep the rest.
DEV void exact_chunk(uint8_t *sx, uint8_t *out, const LaneChunk &lc, RangeState &st)
{
    const uint32_t lane = lane_id();
    uint32_t cnt = __popc(lc.vmask), total;
    uint32_t excl = wave_excl_scan(cnt, &total);
    int idx = st.carry + (int) excl;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if ((lc.vmask >> k) & 1u) {
            if (idx >= 0) sx[idx] = (uint8_t) lc.t[k];
            idx++;
        }
    }
    wave_lds_order();
    st.valid += total;
    int T = st.carry + (int) total;
    if (T >= 4) {
        uint32_t ng = (uint32_t) T >> 2;
        uint32_t nlanes = (ng + 3) >> 2;
        if (lane < nlanes) {
            uint4 sv = *(const uint4 *) (sx + 16 * lane);
            uint32_t o0, o1, o2;
            groups_to_bytes(group_of_bytes(sv.x), group_of_bytes(sv.y),
                            group_of_bytes(sv.z), group_of_bytes(sv.w), o0, o1, o2);
            uint32_t gl = ng - 4 * lane;
            store_bytes12(out + 3 * st.groups + 12 * lane, o0, o1, o2,
                          3 * (gl < 4 ? gl : 4));
        }
        wave_lds_order();
        int nc = T - 4 * (int) ng;
        if (lane == 0)
            for (int j = 0; j < nc; j++) sx[j] = sx[4 * ng + j];
        wave_lds_order();
        st.groups += ng;
        st.carry = nc;
    } else {
        st.carry = T;  // sextets (if any) already sit at sx[0..T)
    }
}

// Emit the final, incomplete group (1..3 sextets at sx[0..r)):
// floor(6r/8) bytes, exactly what the reference's accumulator has produced
// when its upstream reaches EOF (src/base64decoder.c:59-62,71-76).
DEV void emit_partial(uint8_t *sx, uint8_t *dst, int r)
{
    if (lane_id() == 0 && r >= 2) {
        uint32_t G = ((uint32_t) sx[0] << 18) | ((uint32_t) sx[1] << 12) |
                     (r > 2 ? (uint32_t) sx[2] << 6 : 0u);
        dst[0] = (uint8_t) (G >> 16);
        if (r > 2) dst[1] = (uint8_t) (G >> 8);
    }
}

// Decode characters [rb, re) of the stream in[0..n).  The first `skip`
// (0..3) alphabet characters complete a group owned by the previous range
// and are not emitted here.  `out` receives this range's first owned
// group.  If the range is not the last, the final group is completed with
// up to 3 alphabet characters read past `re` (lookahead).  With `hold`
// the stream's final incomplete group is not emitted.
// Returns the number of alphabet characters in [rb, re).
DEV uint64_t decode_range(const uint8_t *tab, uint8_t *sx, const uint8_t *in,
                          uint64_t n, uint64_t rb, uint64_t re, int skip,
                          uint8_t *out, bool is_last, bool hold)
{
    const uint32_t lane = lane_id();
    RangeState st{-skip, 0, 0};
    for (uint64_t pos = rb; pos < re; pos += (uint64_t) kChunk * kDecUnroll) {
        uint4 w[kDecUnroll];
        uint32_t nin[kDecUnroll];
#pragma unroll
        for (int u = 0; u < kDecUnroll; u++) {
            uint64_t p = pos + (uint64_t) u * kChunk + 16 * lane;
            nin[u] = p >= re ? 0u : (re - p >= 16 ? 16u : (uint32_t) (re - p));
            w[u] = nin[u] ? load_chars(in + p, nin[u]) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kDecUnroll; u++) {
            const uint64_t cpos = pos + (uint64_t) u * kChunk;
            if (cpos >= re) break;
            LaneChunk lc;
            map_chunk(tab, w[u], nin[u], lc);
            if (st.carry == 0 && __all(lc.vmask == 0xFFFFu)) {
                // Fast path: 1024 alphabet characters, group aligned.
                uint32_t G[4];
#pragma unroll
                for (int g = 0; g < 4; g++)
                    G[g] = (lc.t[4 * g] << 18) | (lc.t[4 * g + 1] << 12) |
                           (lc.t[4 * g + 2] << 6) | lc.t[4 * g + 3];
                uint32_t o0, o1, o2;
                groups_to_bytes(G[0], G[1], G[2], G[3], o0, o1, o2);
                store_bytes12(out + 3 * st.groups + 12 * lane, o0, o1, o2, 12);
                st.groups += kChunk / 4;
                st.valid += kChunk;
            } else {
                exact_chunk(sx, out, lc, st);
            }
        }
    }
    int r = st.carry;
    if (!is_last && r > 0) {
        // Complete the last group from the characters that follow.
        for (uint64_t q = re; r < 4 && q < n; q += 64) {
            uint64_t p = q + lane;
            uint32_t t = p < n ? tab[in[p]] : 0xFFu;
            bool v = t < 64u;
            uint64_t m = __ballot(v);
            uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t) (m >> 32),
                            __builtin_amdgcn_mbcnt_lo((uint32_t) m, 0u));
            if (v && (int) rank < 4 - r) sx[r + rank] = (uint8_t) t;
            int got = __popcll(m);
            r = r + got > 4 ? 4 : r + got;
        }
        wave_lds_order();
        if (r == 4) {
            if (lane == 0) {
                uint32_t G = ((uint32_t) sx[0] << 18) | ((uint32_t) sx[1] << 12) |
                             ((uint32_t) sx[2] << 6) | sx[3];
                uint8_t *d = out + 3 * st.groups;
                d[0] = (uint8_t) (G >> 16);
                d[1] = (uint8_t) (G >> 8);
                d[2] = (uint8_t) G;
            }
            return st.valid;
        }
        // Ran into the end of the stream: this is the final group.
    }
    if (r > 0 && !hold) emit_partial(sx, out + 3 * st.groups, r);
    return st.valid;
}

struct DecodeWs {
    uint32_t *counts;  // [kMaxRanges] valid characters per range
    uint64_t *bases;   // [kMaxRanges] exclusive prefix of counts
    uint32_t *first_dirty;
};

DEV DecodeWs ws_view(void *ws)
{
    DecodeWs w;
    w.counts = (uint32_t *) ws;
    w.bases = (uint64_t *) ((uint8_t *) ws + kMaxRanges * sizeof(uint32_t));
    w.first_dirty = (uint32_t *) ((uint8_t *) ws + kMaxRanges * 12);
    return w;
}

// Pass 1: every range assumes all earlier ranges were all-alphabet.
__global__ __launch_bounds__(kThreads) void k_decode_pass1(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out,
    uint64_t R, uint32_t nranges, DecAlpha a, void *ws, uint32_t hold)
{
    __shared__ DecSmem sm;
    build_dec_table(sm.tab, a);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t r = blockIdx.x * kWavesPerBlock + wv;
    if (r >= nranges) return;
    const uint64_t rb = (uint64_t) r * R;
    const uint64_t re = rb + R < n ? rb + R : n;
    uint64_t v = decode_range(sm.tab, sm.sx[wv], in, n, rb, re, 0,
                              out + rb / 4 * 3, r + 1 == nranges, hold != 0);
    if (lane_id() == 0) ws_view(ws).counts[r] = (uint32_t) v;
}

// One block: find the first range whose valid count fell short of its
// length, prefix-sum the counts, fill the result, and collect the stream's
// last V mod 4 sextets (for B64X_DEC_HOLD_TAIL callers).
__global__ __launch_bounds__(1024) void k_decode_scan(
    const uint8_t *__restrict__ in, uint64_t n, uint64_t R, uint32_t nranges,
    DecAlpha a, void *ws, b64x_dec_result *res, uint32_t hold)
{
    __shared__ uint8_t tab[256];
    __shared__ uint64_t part[1024];
    __shared__ uint32_t first_dirty;
    build_dec_table(tab, a);
    if (threadIdx.x == 0) first_dirty = nranges;
    __syncthreads();
    DecodeWs w = ws_view(ws);
    const uint32_t per = (nranges + 1023) / 1024;
    const uint32_t r0 = threadIdx.x * per;
    uint64_t sum = 0;
    uint32_t fd = nranges;
    for (uint32_t i = 0; i < per; i++) {
        uint32_t r = r0 + i;
        if (r >= nranges) break;
        uint64_t rb = (uint64_t) r * R, re = rb + R < n ? rb + R : n;
        uint32_t c = w.counts[r];
        if (c != re - rb && fd == nranges) fd = r;
        sum += c;
    }
    if (fd != nranges) atomicMin(&first_dirty, fd);
    part[threadIdx.x] = sum;
    __syncthreads();
    // Hillis-Steele inclusive scan over the 1024 partial sums.
    for (int d = 1; d < 1024; d <<= 1) {
        uint64_t y = threadIdx.x >= (uint32_t) d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += y;
        __syncthreads();
    }
    uint64_t run = part[threadIdx.x] - sum;
    for (uint32_t i = 0; i < per; i++) {
        uint32_t r = r0 + i;
        if (r >= nranges) break;
        w.bases[r] = run;
        run += w.counts[r];
    }
    const uint64_t V = part[1023];
    if (threadIdx.x == 0) {
        *w.first_dirty = first_dirty;
        res->valid = V;
        res->tail_n = (uint32_t) (V & 3);
        res->out_len = hold ? V / 4 * 3 : V * 6 / 8;
    }
    // Last V mod 4 alphabet characters, scanning backwards (wave 0).
    if (threadIdx.x < 64) {
        int need = (int) (V & 3);
        uint8_t got[4] = {0, 0, 0, 0};
        uint64_t end = n;
        while (need > 0 && end > 0) {
            uint64_t beg = end >= 64 ? end - 64 : 0;
            uint64_t p = beg + threadIdx.x;
            uint32_t t = p < end ? tab[in[p]] : 0xFFu;
            uint64_t m = __ballot(t < 64u);
            while (need > 0 && m) {
                int hi = 63 - __clzll(m);
                got[--need] = (uint8_t) __shfl(t, hi, 64);
                m &= ~(1ull << hi);
            }
            end = beg;
        }
        if (threadIdx.x == 0)
            for (int j = 0; j < 4; j++) res->tail[j] = got[j];
    }
}

// Pass 2: re-run the ranges after the first dirty one with true bases.
__global__ __launch_bounds__(kThreads) void k_decode_pass2(
    const uint8_t *__restrict__ in, uint64_t n, uint8_t *__restrict__ out,
    uint64_t R, uint32_t nranges, DecAlpha a, void *ws, uint32_t hold)
{
    DecodeWs w = ws_view(ws);
    const uint32_t fd = *w.first_dirty;
    if (blockIdx.x * kWavesPerBlock + kWavesPerBlock - 1 <= fd) return;
    __shared__ DecSmem sm;
    build_dec_table(sm.tab, a);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t r = blockIdx.x * kWavesPerBlock + wv;
    if (r >= nranges || r <= fd) return;
    const uint64_t rb = (uint64_t) r * R;
    const uint64_t re = rb + R < n ? rb + R : n;
    const uint64_t B = w.bases[r];
    const int skip = (int) ((4 - (B & 3)) & 3);
    decode_range(sm.tab, sm.sx[wv], in, n, rb, re, skip, out + (B + 3) / 4 * 3,
                 r + 1 == nranges, hold != 0);
}

// Uniform-stride batch decode: one wave per buffer.
__global__ __launch_bounds__(kThreads) void k_decode_strided(
    const uint8_t *__restrict__ in, uint64_t in_stride, uint64_t len,
    uint32_t nbuf, uint8_t *__restrict__ out, uint64_t out_stride,
    uint64_t *__restrict__ outlen, DecAlpha a)
{
    __shared__ DecSmem sm;
    build_dec_table(sm.tab, a);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t b = blockIdx.x * kWavesPerBlock + wv; b < nbuf; b += nw) {
        const uint8_t *src = in + (uint64_t) b * in_stride;
        uint64_t v = decode_range(sm.tab, sm.sx[wv], src, len, 0, len, 0,
                                  out + (uint64_t) b * out_stride, true, false);
        if (lane_id() == 0) outlen[b] = v * 6 / 8;
    }
}

// Ragged batch decode: one wave per buffer.
__global__ __launch_bounds__(kThreads) void k_decode_ragged(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
    uint32_t nbuf, uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off,
    uint64_t *__restrict__ outlen, DecAlpha a)
{
    __shared__ DecSmem sm;
    build_dec_table(sm.tab, a);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t nw = gridDim.x * kWavesPerBlock;
    for (uint32_t b = blockIdx.x * kWavesPerBlock + wv; b < nbuf; b += nw) {
        const uint64_t beg = in_off[b], len = in_off[b + 1] - beg;
        uint64_t v = decode_range(sm.tab, sm.sx[wv], in + beg, len, 0, len, 0,
                                  out + out_off[b], true, false);
        if (lane_id() == 0) outlen[b] = v * 6 / 8;
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
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_decode_pass1, kThreads, 0) == hipSuccess && nb > 0)
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
void *g_ws[kMaxDevices];

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

RangePlan plan_ranges(uint64_t n, const DeviceInfo &d)
{
    uint64_t resident = (uint64_t) d.cus * d.dec_blocks_per_cu * kWavesPerBlock;
    if (resident > kMaxRanges) resident = kMaxRanges;
    uint64_t want = (n + kMinRange - 1) / kMinRange;
    if (want > resident) want = resident;
    if (want < 1) want = 1;
    uint64_t R = (n + want - 1) / want;
    R = (R + kChunk - 1) / kChunk * kChunk;
    RangePlan p;
    p.R = R;
    p.nranges = (uint32_t) ((n + R - 1) / R);
    if (p.nranges == 0) p.nranges = 1;
    return p;
}

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
    (void) nchars;
    return (uint64_t) kMaxRanges * 12 + 64;
}

int b64x_device_check(void) { return device_info() ? 0 : -ENODEV; }

int b64x_encode_dev(const void *d_in, uint64_t n, void *d_out,
                    const b64x_alphabet *abc, void *stream)
{
    if (n == 0) return 0;
    if (!d_in || !d_out) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
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
    if (nbuf > 1 && (in_stride < len || out_stride < b64x_encoded_len(len, enc_alpha(abc).pad)))
        return -EINVAL;
    const uint64_t qpb = (len + 11) / 12;
    const uint64_t slots = qpb * nbuf;
    if (nbuf > 1 && slots > 0xFFFFFFFFull) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    const uint64_t per_block = (uint64_t) kThreads * kEncUnroll;
    uint32_t grid = cap_grid((slots + per_block - 1) / per_block,
                             (uint64_t) d->cus * d->enc_blocks_per_cu);
    hipLaunchKernelGGL(k_encode, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (const uint8_t *) d_in, in_stride, len, nbuf, (uint8_t *) d_out,
                       out_stride, qpb, slots, enc_alpha(abc));
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

static void *library_workspace(int *err)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) {
        *err = -ENODEV;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ws[dev]) {
        void *p = nullptr;
        hipError_t e = hipMalloc(&p, b64x_decode_workspace_size(0));
        if (e != hipSuccess) {
            *err = hip_err(e);
            return nullptr;
        }
        g_ws[dev] = p;
    }
    *err = 0;
    return g_ws[dev];
}

int b64x_decode_dev(const void *d_in, uint64_t nchars, void *d_out,
                    b64x_dec_result *d_res, const b64x_alphabet *abc,
                    unsigned flags, void *d_workspace, void *stream)
{
    if (!d_res) return -EINVAL;
    if (flags & ~(unsigned) B64X_DEC_HOLD_TAIL) return -EINVAL;
    if (nchars && (!d_in || !d_out)) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    hipStream_t s = (hipStream_t) stream;
    if (nchars == 0)
        return hip_err(hipMemsetAsync(d_res, 0, sizeof(b64x_dec_result), s));
    int err = 0;
    void *ws = d_workspace ? d_workspace : library_workspace(&err);
    if (!ws) return err;
    const RangePlan p = plan_ranges(nchars, *d);
    const uint32_t blocks = (p.nranges + kWavesPerBlock - 1) / kWavesPerBlock;
    const DecAlpha a = dec_alpha(abc);
    const uint32_t hold = flags & B64X_DEC_HOLD_TAIL;
    hipLaunchKernelGGL(k_decode_pass1, dim3(blocks), dim3(kThreads), 0, s,
                       (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.R,
                       p.nranges, a, ws, hold);
    if ((err = launch_status())) return err;
    hipLaunchKernelGGL(k_decode_scan, dim3(1), dim3(1024), 0, s, (const uint8_t *) d_in,
                       nchars, p.R, p.nranges, a, ws, d_res, hold);
    if ((err = launch_status())) return err;
    if (p.nranges > 1) {
        hipLaunchKernelGGL(k_decode_pass2, dim3(blocks), dim3(kThreads), 0, s,
                           (const uint8_t *) d_in, nchars, (uint8_t *) d_out, p.R,
                           p.nranges, a, ws, hold);
        if ((err = launch_status())) return err;
    }
    return 0;
}

int b64x_decode_strided(const void *d_in, uint64_t in_stride, uint64_t len,
                        uint32_t nbuf, void *d_out, uint64_t out_stride,
                        uint64_t *d_outlen, const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0) return 0;
    if (!d_in || !d_out || !d_outlen) return -EINVAL;
    if (nbuf > 1 && (in_stride < len || out_stride < b64x_decoded_cap(len))) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    uint32_t grid = cap_grid((nbuf + kWavesPerBlock - 1) / kWavesPerBlock,
                             (uint64_t) d->cus * d->dec_blocks_per_cu * 16);
    hipLaunchKernelGGL(k_decode_strided, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (const uint8_t *) d_in, in_stride, len, nbuf, (uint8_t *) d_out,
                       out_stride, d_outlen, dec_alpha(abc));
    return launch_status();
}

int b64x_decode_batch(const void *d_in, const uint64_t *d_in_off, uint32_t nbuf,
                      void *d_out, const uint64_t *d_out_off, uint64_t *d_outlen,
                      const b64x_alphabet *abc, void *stream)
{
    if (nbuf == 0) return 0;
    if (!d_in || !d_in_off || !d_out || !d_out_off || !d_outlen) return -EINVAL;
    const DeviceInfo *d = device_info();
    if (!d) return -ENODEV;
    uint32_t grid = cap_grid((nbuf + kWavesPerBlock - 1) / kWavesPerBlock,
                             (uint64_t) d->cus * d->dec_blocks_per_cu * 16);
    hipLaunchKernelGGL(k_decode_ragged, dim3(grid), dim3(kThreads), 0, (hipStream_t) stream,
                       (const uint8_t *) d_in, d_in_off, nbuf, (uint8_t *) d_out,
                       d_out_off, d_outlen, dec_alpha(abc));
    return launch_status();
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
    uint8_t *d_in, *d_out;
    void *d_ws;
    b64x_dec_result *d_res, *h_res;
};

static uint64_t session_out_cap(uint64_t cap)
{
    uint64_t e = b64x_encoded_len(cap, true), dcap = b64x_decoded_cap(cap);
    return e > dcap ? e : dcap;
}

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
    bool ok = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
              hipHostMalloc((void **) &s->h_in, capacity, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void **) &s->h_out, ocap, hipHostMallocDefault) == hipSuccess &&
              hipHostMalloc((void **) &s->h_res, sizeof(b64x_dec_result), hipHostMallocDefault) == hipSuccess &&
              hipMalloc((void **) &s->d_in, capacity) == hipSuccess &&
              hipMalloc((void **) &s->d_out, ocap) == hipSuccess &&
              hipMalloc((void **) &s->d_res, sizeof(b64x_dec_result)) == hipSuccess &&
              hipMalloc(&s->d_ws, b64x_decode_workspace_size(capacity)) == hipSuccess;
    if (!ok) {
        b64x_session_close(s);
        errno = ENOMEM;
        return nullptr;
    }
    return s;
}

void b64x_session_close(b64x_session *s)
{
    if (!s) return;
    int prev = 0;
    (void) hipGetDevice(&prev);
    (void) hipSetDevice(s->device);
    if (s->stream) (void) hipStreamSynchronize(s->stream);
    if (s->h_in) (void) hipHostFree(s->h_in);
    if (s->h_out) (void) hipHostFree(s->h_out);
    if (s->h_res) (void) hipHostFree(s->h_res);
    if (s->d_in) (void) hipFree(s->d_in);
    if (s->d_out) (void) hipFree(s->d_out);
    if (s->d_res) (void) hipFree(s->d_res);
    if (s->d_ws) (void) hipFree(s->d_ws);
    if (s->stream) (void) hipStreamDestroy(s->stream);
    (void) hipSetDevice(prev);
    free(s);
}

uint64_t b64x_session_capacity(const b64x_session *s) { return s ? s->cap : 0; }
uint8_t *b64x_session_host_in(b64x_session *s) { return s ? s->h_in : nullptr; }
uint8_t *b64x_session_host_out(b64x_session *s) { return s ? s->h_out : nullptr; }

int b64x_session_encode(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                        uint64_t *out_len)
{
    if (!s || n > s->cap || !out_len) return -EINVAL;
    *out_len = 0;
    if (n == 0) return 0;
    int err;
    const uint64_t m = b64x_encoded_len(n, enc_alpha(abc).pad);
    if ((err = hip_err(hipSetDevice(s->device)))) return err;
    if ((err = hip_err(hipMemcpyAsync(s->d_in, s->h_in, n, hipMemcpyHostToDevice, s->stream)))) return err;
    if ((err = b64x_encode_dev(s->d_in, n, s->d_out, abc, s->stream))) return err;
    if ((err = hip_err(hipMemcpyAsync(s->h_out, s->d_out, m, hipMemcpyDeviceToHost, s->stream)))) return err;
    if ((err = hip_err(hipStreamSynchronize(s->stream)))) return err;
    *out_len = m;
    return 0;
}

int b64x_session_decode(b64x_session *s, uint64_t n, const b64x_alphabet *abc,
                        unsigned flags, b64x_dec_result *res)
{
    if (!s || n > s->cap || !res) return -EINVAL;
    memset(res, 0, sizeof(*res));
    if (n == 0) return 0;
    int err;
    if ((err = hip_err(hipSetDevice(s->device)))) return err;
    if ((err = hip_err(hipMemcpyAsync(s->d_in, s->h_in, n, hipMemcpyHostToDevice, s->stream)))) return err;
    if ((err = b64x_decode_dev(s->d_in, n, s->d_out, s->d_res, abc, flags, s->d_ws, s->stream))) return err;
    if ((err = hip_err(hipMemcpyAsync(s->h_res, s->d_res, sizeof(b64x_dec_result),
                                      hipMemcpyDeviceToHost, s->stream)))) return err;
    if ((err = hip_err(hipMemcpyAsync(s->h_out, s->d_out, b64x_decoded_cap(n),
                                      hipMemcpyDeviceToHost, s->stream)))) return err;
    if ((err = hip_err(hipStreamSynchronize(s->stream)))) return err;
    *res = *s->h_res;
    return 0;
}

const char *b64x_build_info(void)
{
    return "b64x abi=1 arch=gfx950 enc:quad12->16 lds-alphabet unroll=4; "
           "dec:wave-range chunk=1024 lds-inverse-table 2-pass-fixup";
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
