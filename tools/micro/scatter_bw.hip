// scatter_bw.hip -- HBM write-locality microbenchmark for the radix scatter.
// Copies N bytes with 16-B-per-lane loads (sequential) and stores whose
// B-byte blocks land at multiplicatively permuted block positions, i.e. the
// store stream is a random permutation of B-byte blocks.  B = 0: identity.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/scatter_bw.hip -o /tmp/scatter_bw && /tmp/scatter_bw
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

typedef long long i64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(1024) void copy_perm(const i64x2 *__restrict__ src, i64x2 *__restrict__ dst,
                                                  uint64_t n16, int blk16_log2, uint64_t nblk_mask,
                                                  uint64_t mul, int per) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024 * per;
#pragma unroll 4
    for (int k = 0; k < per; k++) {
        const uint64_t i = base + (uint64_t)k * 1024 + threadIdx.x;
        if (i >= n16) break;
        const i64x2 v = src[i];
        uint64_t o = i;
        if (blk16_log2 >= 0) {
            const uint64_t b = i >> blk16_log2;
            const uint64_t pb = (b * mul) & nblk_mask;
            o = (pb << blk16_log2) | (i & ((1ull << blk16_log2) - 1));
        }
        dst[o] = v;
    }
}

int main() {
    const uint64_t bytes = 1ull << 31;  // 2 GiB (power of two: the block map is a bijection)
    const uint64_t n16 = bytes / 16;
    i64x2 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int per = 8;
    const unsigned grid = (unsigned)((n16 + 1024 * per - 1) / (1024 * per));
    const int blocks[] = {-1, 16, 32, 64, 128, 256, 512, 1024, 4096, 65536};
    for (int bi = 0; bi < (int)(sizeof(blocks) / sizeof(blocks[0])); bi++) {
        const int B = blocks[bi];
        int lg = -1;
        if (B > 0) { lg = 0; while ((16 << lg) < B) lg++; }
        const uint64_t nblk = B > 0 ? bytes / B : 1;
        for (int rep = 0; rep < 2; rep++)
            hipLaunchKernelGGL(copy_perm, dim3(grid), dim3(1024), 0, 0, a, b, n16, lg, nblk - 1,
                               0x9E3779B97F4A7C15ull | 1ull, per);
        CK(hipEventRecord(e0));
        const int reps = 5;
        for (int rep = 0; rep < reps; rep++)
            hipLaunchKernelGGL(copy_perm, dim3(grid), dim3(1024), 0, 0, a, b, n16, lg, nblk - 1,
                               0x9E3779B97F4A7C15ull | 1ull, per);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("block %6d B: %.3f ms  copy %.2f TB/s (read+write)\n", B, ms, 2.0 * bytes / (ms * 1e-3) / 1e12);
    }
    return 0;
}
