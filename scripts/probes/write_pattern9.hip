// Store-bandwidth ceiling for k_prune's KEEP write stream, part 9 (r03, late): the cache-policy
// bits of the stores.  write_pattern3 compared nt with plain stores only; k_prune went from
// 0.137 to 0.123 ms when its streamed stores became `sc1 nt` (written through the L2).  Same
// bytes as part 3 (49 slots x 1563 tiles x 4 categories x 2 KB = 627 MB per launch).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern9.hip -o scripts/probes/_write_pattern9
//   scripts/probes/_write_pattern9 [n_slots=49] [n_tiles=1563] [C=4]
//
//   stream  P W : flat grid-stride fill, 16 B per lane per instruction, W blocks/CU
//   slotmaj P   : k_prune's shape -- one wave per (tile, category), 2 KB per op, a few
//                 dependent fp64 FMAs between ops, slot-major [slot][cat][tile][4][64]
//   occN        : slotmaj with dynamic LDS limiting a CU to N workgroups
// P: policy 0 plain, 1 nt, 2 sc1, 3 sc1 nt, 4 sc0 sc1 nt
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int P>
__device__ __forceinline__ void st(dbl2 v, dbl2 *p) {
    if constexpr (P == 0)
        asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 1)
        asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 2)
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (P == 3)
        asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}

template <int P>
__global__ void __launch_bounds__(256) k_stream(dbl2 *out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    dbl2 v = {1.0 * threadIdx.x, 2.0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        st<P>(v, out + i);
}

template <int P>
__global__ void __launch_bounds__(256) k_ops(double *clv, int n_slots, int n_tiles, int C) {
    extern __shared__ double lds_pad[];
    const int lane = threadIdx.x & 63;
    const int wt = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tile = wt / C, cat = wt - tile * C;
    if (tile >= n_tiles) return;
    if (n_slots < 0) lds_pad[threadIdx.x] = 0.0;  // keeps the LDS allocation
    double v0 = lane, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3;
    for (int p = 0; p < n_slots; ++p) {
        for (int w = 0; w < 8; ++w) {  // some dependent fp64 work per op, as in k_prune
            v0 = fma(v0, 1.0000001, v1);
            v1 = fma(v1, 0.9999999, v2);
            v2 = fma(v2, 1.0000001, v3);
            v3 = fma(v3, 0.9999999, v0);
        }
        const size_t row = ((size_t)p * C + cat) * n_tiles + tile;
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * 256) + lane;
        dbl2 a = {v0, v1}, b = {v2, v3};
        st<P>(a, q);
        st<P>(b, q + 64);
    }
}

static double bytes_g;

template <class F>
void timeit(const char *name, F launch) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i) launch();
    const int reps = 50;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("%-28s %.4f ms  %6.0f GB/s\n", name, ms, bytes_g / ms / 1e6);
    fflush(stdout);
}

template <int P>
void run_policy(double *clv, int n_cu, size_t bytes, int n_slots, int n_tiles, int C) {
    const int grid = (n_tiles * C + 3) / 4;
    char nm[64];
    for (int w : {1, 2, 4, 8}) {
        snprintf(nm, sizeof nm, "stream P%d %d blk/CU", P, w);
        timeit(nm, [&] {
            hipLaunchKernelGGL(k_stream<P>, dim3(n_cu * w), dim3(256), 0, 0, (dbl2 *)clv,
                               bytes / 16);
        });
    }
    snprintf(nm, sizeof nm, "slotmaj P%d", P);
    timeit(nm, [&] {
        hipLaunchKernelGGL(k_ops<P>, dim3(grid), dim3(256), 0, 0, clv, n_slots, n_tiles, C);
    });
    for (int occ : {2, 4, 6}) {
        const size_t lds = (160 * 1024) / (occ + 1) + 512;
        snprintf(nm, sizeof nm, "slotmaj P%d occ%d", P, occ);
        timeit(nm, [&] {
            hipLaunchKernelGGL(k_ops<P>, dim3(grid), dim3(256), lds, 0, clv, n_slots, n_tiles,
                               C);
        });
    }
}

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = argc > 3 ? atoi(argv[3]) : 4;
    const size_t bytes = (size_t)n_slots * n_tiles * C * 256 * 8;
    bytes_g = (double)bytes;
    double *clv;
    if (hipMalloc(&clv, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("bytes per launch %.1f MB, %d CUs\n", bytes / 1e6, n_cu);
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(clv, 0, bytes, 0); });
        run_policy<1>(clv, n_cu, bytes, n_slots, n_tiles, C);
        run_policy<3>(clv, n_cu, bytes, n_slots, n_tiles, C);
        run_policy<4>(clv, n_cu, bytes, n_slots, n_tiles, C);
        run_policy<2>(clv, n_cu, bytes, n_slots, n_tiles, C);
        run_policy<0>(clv, n_cu, bytes, n_slots, n_tiles, C);
    }
    hipFree(clv);
    return 0;
}
