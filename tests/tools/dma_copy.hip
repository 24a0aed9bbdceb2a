// dma_copy.hip -- calibration only (not product, not shipped): does a copy
// whose reads go global -> LDS directly (global_load_lds_dwordx4) stream
// faster than the plain register copy that bench.py's copy ceiling uses?
// Build: hipcc --offload-arch=gfx950 -O3 -o dma_copy dma_copy.hip ; run on
// the GPU box.  Prints GB/s of read + written bytes per shape.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// plain: one 16-byte non-temporal load and store per lane (the ceiling's
// fastest shape), U per lane, 256-lane blocks
template <int U>
__global__ __launch_bounds__(256) void plain(const v4u *__restrict__ in, v4u *__restrict__ out)
{
    const uint64_t b = (uint64_t) blockIdx.x * 256 * U + threadIdx.x;
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(in + b + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(v[u], out + b + u * 256);
}

// plain with a dword-aligned (not 16-byte aligned) source
template <int U>
__global__ __launch_bounds__(256) void plain_mis(const uint8_t *__restrict__ in, v4u *__restrict__ out)
{
    typedef uint32_t v4a4 __attribute__((ext_vector_type(4), aligned(4)));
    const uint64_t b = (uint64_t) blockIdx.x * 256 * U + threadIdx.x;
    v4a4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load((const v4a4 *) in + b + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(v4u{v[u].x, v[u].y, v[u].z, v[u].w}, out + b + u * 256);
}

// the wave's 1 KiB per step read straight into its LDS slice (M0 = the
// slice, each lane's 16 bytes at lane * 16), then read back and stored
template <int U, int NT>
__global__ __launch_bounds__(256) void dma(const uint8_t *__restrict__ in, v4u *__restrict__ out)
{
    __shared__ v4u buf[4][U][64];
    const uint32_t w = (uint32_t) __builtin_amdgcn_readfirstlane((int) (threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const uint64_t base = ((uint64_t) blockIdx.x * 4 + w) * U * 1024;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint8_t *src = in + base + u * 1024 + 16 * lane;
        const uint32_t l = (uint32_t) (uintptr_t) (__attribute__((address_space(3))) void *) &buf[w][u][0];
        uint32_t keep;
        if (NT)
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(l) : "memory");
        else
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                         "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(src), "s"(l) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++)
        __builtin_nontemporal_store(buf[w][u][lane], out + (base + u * 1024) / 16 + lane);
}

template <typename F>
float timeit(F launch)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    launch();
    float best = 1e9;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(a);
        for (int i = 0; i < 20; i++) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms / 20 < best) best = ms / 20;
    }
    return best;
}

int main()
{
    const uint64_t half = (2505397592ull / 2) / (1 << 16) * (1 << 16);  // bench.py's copy
    uint8_t *in, *out;
    if (hipMalloc(&in, half) || hipMalloc(&out, half)) return 1;
    hipMemset(in, 7, half);
    hipMemset(out, 0, half);
    const double gb = 2.0 * half / 1e9;
    for (int round = 0; round < 2; round++) {
        float ms;
        ms = timeit([&] { plain<1><<<half / 4096, 256>>>((const v4u *) in, (v4u *) out); });
        printf("plain U1      %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { plain<2><<<half / 8192, 256>>>((const v4u *) in, (v4u *) out); });
        printf("plain U2      %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        // the same copy reading from 8 bytes past a 16-byte boundary (every
        // 16-byte load straddles two 16-byte blocks: config 4's odd rows)
        ms = timeit([&] { plain_mis<1><<<half / 4096 - 1, 256>>>(in + 8, (v4u *) out); });
        printf("plain U1 +8   %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { plain_mis<1><<<half / 4096 - 1, 256>>>(in + 4, (v4u *) out); });
        printf("plain U1 +4   %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { dma<1, 0><<<half / 4096, 256>>>(in, (v4u *) out); });
        printf("dma U1        %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { dma<1, 1><<<half / 4096, 256>>>(in, (v4u *) out); });
        printf("dma U1 nt     %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { dma<2, 0><<<half / 8192, 256>>>(in, (v4u *) out); });
        printf("dma U2        %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { dma<2, 1><<<half / 8192, 256>>>(in, (v4u *) out); });
        printf("dma U2 nt     %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
        ms = timeit([&] { dma<4, 1><<<half / 16384, 256>>>(in, (v4u *) out); });
        printf("dma U4 nt     %.4f ms %.0f GB/s\n", ms, gb / ms * 1e3);
    }
    // check the last copy moved the bytes
    uint8_t h[4096];
    hipMemcpy(h, out + half - 4096, 4096, hipMemcpyDeviceToHost);
    for (int i = 0; i < 4096; i++)
        if (h[i] != 7) {
            printf("MISMATCH at %d\n", i);
            return 2;
        }
    printf("ok\n");
    return 0;
}
