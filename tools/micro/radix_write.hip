// radix_write.hip -- write-pattern cost of one stable radix/bucket scatter pass
// with perfect LDS staging, as a function of the digit width D and tile size.
//
// Setup (untimed): rows get a uniform random D-bit digit; every tile of T rows
// is pre-permuted into digit order (what the LDS staging of a scatter kernel
// produces) and every staged row gets its global destination: digit start +
// rows of that digit in earlier tiles + rank in the tile (a stable counting
// sort's layout).  Timed: read the staged rows (16 B) and their u32
// destinations sequentially, store every row to its destination.  D = 0 is
// the identity (a copy carrying the same index read).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/radix_write.hip -o tools/micro/radix_write
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef long long i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((x ^ (x >> 31)) >> 32);
}

// tile histograms: cnt[t][d]
__global__ void k_hist(uint32_t *cnt, int64_t n, int T, int D) {
    extern __shared__ uint32_t h[];
    const int R = 1 << D;
    for (int i = threadIdx.x; i < R; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const int64_t t = blockIdx.x;
    for (int j = threadIdx.x; j < T; j += blockDim.x) {
        const int64_t i = t * T + j;
        if (i < n) atomicAdd(&h[D ? mix(i) >> (32 - D) : 0], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += blockDim.x) cnt[t * R + i] = h[i];
}

// per digit: exclusive offsets over (digit, tile) order, in place
__global__ void k_scan(uint32_t *cnt, int64_t ntiles, int R, const uint32_t *dstart) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= R) return;
    uint32_t off = dstart[d];
    for (int64_t t = 0; t < ntiles; t++) {
        const uint32_t c = cnt[t * R + d];
        cnt[t * R + d] = off;
        off += c;
    }
}

__global__ void k_totals(const uint32_t *cnt, int64_t ntiles, int R, uint32_t *tot) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= R) return;
    uint32_t s = 0;
    for (int64_t t = 0; t < ntiles; t++) s += cnt[t * R + d];
    tot[d] = s;
}

// stage each tile in digit order: src row of staged slot, its destination
__global__ void k_stage(const uint32_t *offs, int64_t n, int T, int D, i64x2 *staged, uint32_t *dst) {
    extern __shared__ uint32_t h[];  // [R] counts -> local starts, [R] cursors
    const int R = 1 << D;
    uint32_t *cur = h + R;
    for (int i = threadIdx.x; i < R; i += blockDim.x) { h[i] = 0; cur[i] = 0; }
    __syncthreads();
    const int64_t t = blockIdx.x;
    for (int j = threadIdx.x; j < T; j += blockDim.x) {
        const int64_t i = t * T + j;
        if (i < n) atomicAdd(&h[D ? mix(i) >> (32 - D) : 0], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int d = 0; d < R; d++) { const uint32_t c = h[d]; h[d] = s; s += c; }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < T; j += blockDim.x) {
        const int64_t i = t * T + j;
        if (i >= n) continue;
        const uint32_t d = D ? mix(i) >> (32 - D) : 0;
        const uint32_t r = atomicAdd(&cur[d], 1u);
        const int64_t slot = t * T + h[d] + r;
        staged[slot] = i64x2{(long long)i, (long long)d};
        dst[slot] = D ? offs[t * R + d] + r : (uint32_t)i;
    }
}

template <int PER>
__global__ __launch_bounds__(256) void k_scatter(const i64x2 *__restrict__ src, const uint32_t *__restrict__ dst,
                                                 i64x2 *__restrict__ out, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * PER + threadIdx.x;
    i64x2 v[PER];
    uint32_t o[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const int64_t i = min(base + k * 256, n - 1);
        v[k] = src[i];
        o[k] = dst[i];
    }
#pragma unroll
    for (int k = 0; k < PER; k++) out[o[k]] = v[k];
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    i64x2 *staged, *out;
    uint32_t *dst, *cnt, *dstart;
    CK(hipMalloc(&staged, n * 16));
    CK(hipMalloc(&out, n * 16));
    CK(hipMalloc(&dst, n * 4));
    CK(hipMalloc(&dstart, 65536 * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int Ds[] = {0, 6, 8, 10, 11, 12, 13, 14};
    const int Ts[] = {4096, 8192, 16384, 32768};
    for (int ti = 0; ti < 4; ti++) {
        const int T = Ts[ti];
        const int64_t ntiles = (n + T - 1) / T;
        for (int di = 0; di < 8; di++) {
            const int D = Ds[di], R = 1 << D;
            if (D == 0 && ti > 0) continue;
            CK(hipMalloc(&cnt, ntiles * R * 4));
            hipLaunchKernelGGL(k_hist, dim3(ntiles), dim3(1024), 2 * R * 4, 0, cnt, n, T, D);
            hipLaunchKernelGGL(k_totals, dim3((R + 255) / 256), dim3(256), 0, 0, cnt, ntiles, R, dstart);
            // exclusive scan of the totals on the host (tiny)
            uint32_t *ht = (uint32_t *)malloc(R * 4);
            CK(hipMemcpy(ht, dstart, R * 4, hipMemcpyDeviceToHost));
            uint32_t s = 0;
            for (int d = 0; d < R; d++) { const uint32_t c = ht[d]; ht[d] = s; s += c; }
            CK(hipMemcpy(dstart, ht, R * 4, hipMemcpyHostToDevice));
            free(ht);
            hipLaunchKernelGGL(k_scan, dim3((R + 255) / 256), dim3(256), 0, 0, cnt, ntiles, R, dstart);
            hipLaunchKernelGGL(k_stage, dim3(ntiles), dim3(1024), 2 * R * 4, 0, cnt, n, T, D, staged, dst);
            CK(hipDeviceSynchronize());
            CK(hipFree(cnt));
            constexpr int PER = 8;
            const unsigned grid = (unsigned)((n + 256 * PER - 1) / (256 * PER));
            for (int rep = 0; rep < 2; rep++)
                hipLaunchKernelGGL(k_scatter<PER>, dim3(grid), dim3(256), 0, 0, staged, dst, out, n);
            CK(hipEventRecord(e0));
            const int reps = 5;
            for (int rep = 0; rep < reps; rep++)
                hipLaunchKernelGGL(k_scatter<PER>, dim3(grid), dim3(256), 0, 0, staged, dst, out, n);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= reps;
            printf("T %5d D %2d (avg run %7.2f rows): %.3f ms  rows r+w %.2f TB/s  (incl. idx %.2f TB/s)\n", T, D,
                   (double)T / R, ms, 32.0 * n / (ms * 1e-3) / 1e12, 36.0 * n / (ms * 1e-3) / 1e12);
            fflush(stdout);
        }
    }
    return 0;
}
