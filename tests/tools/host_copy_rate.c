/*
 * host_copy_rate.c -- TEST TOOL: one thread's copy rate on this host for the
 * loop thread's copies (a decoder stage serving its pinned output into a
 * consumer's buffer): glibc memcpy against an AVX2 non-temporal-store copy,
 * in chunks of 64 KiB .. 1 MiB over 1 GiB, from ordinary and from pinned
 * (hipHostMalloc, fine-grained) memory.  Prints one JSON line per case.
 *   cc -O2 -mavx2 tests/tools/host_copy_rate.c -o tests/tools/host_copy_rate \
 *      -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -L/opt/rocm/lib -lamdhip64
 */
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

extern int hipHostMalloc(void **p, size_t n, unsigned flags);
extern int hipHostFree(void *p);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void copy_nt(uint8_t *d, const uint8_t *s, size_t n)
{
    size_t i = 0;
    while (i < n && ((uintptr_t) (d + i) & 31)) {
        d[i] = s[i];
        i++;
    }
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *) (s + i));
        __m256i b = _mm256_loadu_si256((const __m256i *) (s + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *) (s + i + 64));
        __m256i e = _mm256_loadu_si256((const __m256i *) (s + i + 96));
        _mm256_stream_si256((__m256i *) (d + i), a);
        _mm256_stream_si256((__m256i *) (d + i + 32), b);
        _mm256_stream_si256((__m256i *) (d + i + 64), c);
        _mm256_stream_si256((__m256i *) (d + i + 96), e);
    }
    for (; i < n; i++)
        d[i] = s[i];
    _mm_sfence();
}

int main(void)
{
    const size_t N = (size_t) 1 << 30;
    uint8_t *dst = malloc(N), *src = malloc(N), *pin = NULL;
    memset(dst, 1, N);
    memset(src, 2, N);
    if (hipHostMalloc((void **) &pin, N, 0x4 /* coherent */) != 0)
        pin = NULL;
    else
        memset(pin, 3, N);
    const size_t chunks[] = { 64 << 10, 256 << 10, 1 << 20 };
    for (int from_pin = 0; from_pin < 2; from_pin++) {
        const uint8_t *s = from_pin ? pin : src;
        if (!s)
            continue;
        for (int c = 0; c < 3; c++) {
            for (int nt = 0; nt < 2; nt++) {
                double best = 1e9;
                for (int rep = 0; rep < 3; rep++) {
                    double t0 = now();
                    for (size_t o = 0; o < N; o += chunks[c]) {
                        if (nt)
                            copy_nt(dst + o, s + o, chunks[c]);
                        else
                            memcpy(dst + o, s + o, chunks[c]);
                    }
                    double dt = now() - t0;
                    if (dt < best)
                        best = dt;
                }
                printf("{\"src\": \"%s\", \"chunk\": %zu, \"copy\": \"%s\", \"GB_s\": %.2f}\n",
                       from_pin ? "pinned" : "malloc", chunks[c], nt ? "avx2_nt" : "memcpy",
                       N / best / 1e9);
                fflush(stdout);
            }
        }
    }
    return 0;
}
