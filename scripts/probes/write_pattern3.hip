// Store-bandwidth ceiling for k_prune's KEEP write stream (49 CLV slots x 1563 tiles x 4
// categories x 64 lanes x 4 doubles = 627 MB per launch), part 3: what the chip's write path
// gives this byte count, by store flavour, waves per CU and address order.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern3.hip -o scripts/probes/_write_pattern3
//   scripts/probes/_write_pattern3 [n_slots=49] [n_tiles=1563] [C=4]
//
// Every kernel writes the same bytes once per launch; times are hipEvent averages over 50
// back-to-back launches after 20 warm-ups.
//   stream   : flat grid-stride fill, 16 B per lane per instruction, W blocks/CU persistent
//   slotmaj  : k_prune's shape -- one wave per (tile, category), one 2 KB block per op
//              (two 1-KB dwordx4 instructions), slot-major [slot][cat][tile][4][64]
//   wavemaj  : the same waves, each writing its own contiguous 98 KB run [cat][tile][slot]
//   slotmajP : slotmaj with plain (not nt) stores
//   occ<N>   : slotmaj with dynamic LDS limiting the CU to N workgroups (4N waves)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void st(dbl2 v, dbl2 *p) {
    if (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template <bool NT>
__global__ void __launch_bounds__(256) k_stream(dbl2 *out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    dbl2 v = {1.0 * threadIdx.x, 2.0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        st<NT>(v, out + i);
}

// L: 0 slot-major, 1 wave-major
template <int L, bool NT>
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
        size_t row;
        if (L == 0)
            row = ((size_t)p * C + cat) * n_tiles + tile;
        else
            row = ((size_t)cat * n_tiles + tile) * n_slots + p;
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * 256) + lane;
        dbl2 a = {v0, v1}, b = {v2, v3};
        st<NT>(a, q);
        st<NT>(b, q + 64);
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
    printf("%-26s %.4f ms  %6.0f GB/s\n", name, ms, bytes_g / ms / 1e6);
    fflush(stdout);
}

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = argc > 3 ? atoi(argv[3]) : 4;
    const size_t rows = (size_t)n_slots * n_tiles * C;
    const size_t bytes = rows * 256 * 8;
    bytes_g = (double)bytes;
    double *clv;
    if (hipMalloc(&clv, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("bytes per launch %.1f MB, %d CUs\n", bytes / 1e6, n_cu);
    const int grid = (n_tiles * C + 3) / 4;
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(clv, 0, bytes, 0); });
        for (int w : {1, 2, 4, 8, 16}) {
            char nm[64];
            snprintf(nm, sizeof nm, "stream nt  %2d blk/CU", w);
            timeit(nm, [&] {
                hipLaunchKernelGGL(k_stream<true>, dim3(n_cu * w), dim3(256), 0, 0, (dbl2 *)clv,
                                   bytes / 16);
            });
            snprintf(nm, sizeof nm, "stream pl  %2d blk/CU", w);
            timeit(nm, [&] {
                hipLaunchKernelGGL(k_stream<false>, dim3(n_cu * w), dim3(256), 0, 0,
                                   (dbl2 *)clv, bytes / 16);
            });
        }
        timeit("slotmaj nt", [&] {
            hipLaunchKernelGGL((k_ops<0, true>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                               n_tiles, C);
        });
        timeit("slotmaj plain", [&] {
            hipLaunchKernelGGL((k_ops<0, false>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                               n_tiles, C);
        });
        timeit("wavemaj nt", [&] {
            hipLaunchKernelGGL((k_ops<1, true>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                               n_tiles, C);
        });
        timeit("wavemaj plain", [&] {
            hipLaunchKernelGGL((k_ops<1, false>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                               n_tiles, C);
        });
        for (int occ : {2, 3, 4, 5, 6, 7, 8}) {
            // LDS per workgroup so that only `occ` workgroups fit a CU's 160 KB
            const size_t lds = (160 * 1024) / (occ + 1) + 512;
            char nm[64];
            snprintf(nm, sizeof nm, "slotmaj nt occ%d (%zuB)", occ, lds);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_ops<0, true>), dim3(grid), dim3(256), lds, 0, clv, n_slots,
                                   n_tiles, C);
            });
        }
    }
    hipFree(clv);
    return 0;
}
