// copy_sweep.hip -- calibration only (not product, not shipped): how fast
// can a plain HBM stream go on this part, by unroll depth, grid size and
// load/store cache policy?  Build: hipcc --offload-arch=gfx950 -O3 -o
// copy_sweep copy_sweep.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int U, int LNT, int SNT>
__global__ __launch_bounds__(256) void copyk(const v4u *__restrict__ in, v4u *__restrict__ out,
                                              uint64_t n16)
{
    const uint64_t tile = 256ull * U, full = n16 / tile;
    for (uint64_t t = blockIdx.x; t < full; t += gridDim.x) {
        const uint64_t b = t * tile + threadIdx.x;
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = LNT ? __builtin_nontemporal_load(in + b + u * 256) : in[b + u * 256];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (SNT) __builtin_nontemporal_store(v[u], out + b + u * 256);
            else out[b + u * 256] = v[u];
        }
    }
}

template <int U, int LNT, int SNT>
float run(const v4u *in, v4u *out, uint64_t n16, int grid)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    copyk<U, LNT, SNT><<<grid, 256>>>(in, out, n16);
    hipEventRecord(a);
    for (int i = 0; i < 20; i++) copyk<U, LNT, SNT><<<grid, 256>>>(in, out, n16);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 20;
}

#define RUN(U, L, S)                                                                          \
    for (int g : grids) {                                                                     \
        float ms = run<U, L, S>(in, out, n16, g);                                             \
        printf("U=%2d ldnt=%d stnt=%d grid=%6d  %.4f ms  %.0f GB/s\n", U, L, S, g, ms,         \
               2.0 * n16 * 16 / ms / 1e6);                                                    \
    }

int main()
{
    const uint64_t bytes = 1ull << 30, n16 = bytes / 16;
    v4u *in, *out;
    if (hipMalloc(&in, bytes) || hipMalloc(&out, bytes)) return 1;
    hipMemset(in, 1, bytes);
    hipMemset(out, 0, bytes);
    int grids[] = {1024, 2048, 4096, 8192, 32768};
    RUN(1, 0, 0) RUN(4, 0, 0) RUN(4, 0, 1) RUN(4, 1, 1) RUN(8, 0, 1) RUN(8, 1, 1) RUN(16, 0, 1)
    return 0;
}
