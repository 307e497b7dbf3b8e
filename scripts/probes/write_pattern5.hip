// Store-bandwidth ceiling, part 5: which property of a flat store stream sets its rate.
// write_pattern3 measured 6.5 TB/s for a grid-stride stream with one 256-thread block per CU
// (1 MB written per grid step) and 5.5 / 4.7 / 4.2 TB/s with 2 / 4 / 16 blocks per CU.  The
// variants below separate the width of the grid step ("window") from the bytes a wave writes
// contiguously and from the waves per CU.
//   chunk<N>   1 block/CU, each wave writes N KB contiguous per grid step (window N MB)
//   x2         1 block/CU, 8-byte stores (512 B per wave-instruction, window 512 KB)
//   x2b2       2 blocks/CU, 8-byte stores (window 1 MB)
//   w8         1 block/CU of 512 threads (8 waves, window 2 MB)
//   split4     1 block/CU, the 4 waves of a block write 4 regions a quarter-buffer apart
//   step<N>    1 block/CU, stream nt, but a wave issues N stores then N x 32 fp64 FMAs
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern5.hip -o scripts/probes/_write_pattern5
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

// each wave writes CH x 1 KB contiguous per grid step
template <int CH>
__global__ void __launch_bounds__(512) k_chunk(dbl2 *out, size_t n16) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const size_t step = (size_t)gridDim.x * nw * 64 * CH;  // dbl2 per grid step
    dbl2 v = {1.0 * lane, 2.0};
    for (size_t base = ((size_t)blockIdx.x * nw + wave) * 64 * CH; base < n16; base += step) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const size_t i = base + c * 64 + lane;
            if (i < n16) __builtin_nontemporal_store(v, out + i);
        }
    }
}

__global__ void __launch_bounds__(256) k_x2(double *out, size_t n8) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const double v = threadIdx.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride)
        __builtin_nontemporal_store(v, out + i);
}

// the 4 waves of a block write 4 separate quarters of the buffer
__global__ void __launch_bounds__(256) k_split4(dbl2 *out, size_t n16) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t q = n16 / 4;
    dbl2 v = {1.0 * lane, 2.0};
    for (size_t i = (size_t)blockIdx.x * 64 + lane; i < q; i += (size_t)gridDim.x * 64)
        __builtin_nontemporal_store(v, out + wave * q + i);
}

template <int N>
__global__ void __launch_bounds__(256) k_step(dbl2 *out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    double a = threadIdx.x, b = 1.0;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    while (i < n16) {
#pragma unroll
        for (int k = 0; k < N; ++k, i += stride)
            if (i < n16) __builtin_nontemporal_store(dbl2{a, b}, out + i);
#pragma unroll
        for (int k = 0; k < 32 * N; ++k) a = fma(a, 1.0000001, b);
    }
}

static double bytes_g;

template <class F>
void timeit(const char *name, F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i) launch();
    const int reps = 50;
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-26s %.4f ms  %6.0f GB/s\n", name, ms, bytes_g / ms / 1e6);
    fflush(stdout);
}

int main() {
    const size_t bytes = (size_t)49 * 1563 * 4 * 256 * 8;  // k_prune's cfg2 KEEP CLV bytes
    bytes_g = (double)bytes;
    void *buf;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    dbl2 *o16 = (dbl2 *)buf;
    const size_t n16 = bytes / 16;
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(buf, 0, bytes, 0); });
        timeit("chunk1 (1 KB)", [&] {
            hipLaunchKernelGGL(k_chunk<1>, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("chunk2 (2 KB)", [&] {
            hipLaunchKernelGGL(k_chunk<2>, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("chunk4 (4 KB)", [&] {
            hipLaunchKernelGGL(k_chunk<4>, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("chunk1 half grid", [&] {
            hipLaunchKernelGGL(k_chunk<1>, dim3(n_cu / 2), dim3(256), 0, 0, o16, n16);
        });
        timeit("x2", [&] {
            hipLaunchKernelGGL(k_x2, dim3(n_cu), dim3(256), 0, 0, (double *)buf, bytes / 8);
        });
        timeit("x2b2", [&] {
            hipLaunchKernelGGL(k_x2, dim3(2 * n_cu), dim3(256), 0, 0, (double *)buf, bytes / 8);
        });
        timeit("w8 (512 threads)", [&] {
            hipLaunchKernelGGL(k_chunk<1>, dim3(n_cu), dim3(512), 0, 0, o16, n16);
        });
        timeit("split4", [&] {
            hipLaunchKernelGGL(k_split4, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("step1", [&] {
            hipLaunchKernelGGL(k_step<1>, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("step2", [&] {
            hipLaunchKernelGGL(k_step<2>, dim3(n_cu), dim3(256), 0, 0, o16, n16);
        });
        timeit("step2 2blk", [&] {
            hipLaunchKernelGGL(k_step<2>, dim3(2 * n_cu), dim3(256), 0, 0, o16, n16);
        });
    }
    (void)hipFree(buf);
    return 0;
}
