// Store-bandwidth ceiling for k_prune's KEEP write stream, part 10 (r04): the CLV LAYOUT under
// the write-through streamed stores (`sc1 nt`) at the 4-workgroups-per-CU operating point.  The
// r02 layout probes (parts 3-7) used `nt` stores only; r03 / r04 found that write-through
// stores change which occupancy wins, so the layout question is asked again.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern10.hip -o scripts/probes/_write_pattern10
//   scripts/probes/_write_pattern10 [n_slots=49] [n_tiles=1563] [C=4]
//
// One wave per (tile, category), 2 KB per op (two dwordx4 per lane), a few dependent fp64 FMAs
// between ops, as k_prune; the layouts of the [slot][cat][tile] blocks of 2 KB:
//   L0 slot-major  [slot][cat][tile]   (k_prune's)      a slot's tiles are contiguous
//   L1 tile-major  [tile][slot][cat]   a workgroup writes 8 KB contiguous per op, sequentially
//   L2 wave-major  [tile][cat][slot]   a wave streams its own contiguous region op after op
// occ k: dynamic LDS limits a CU to k workgroups (4: k_prune's KEEP plans since r04)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void st(dbl2 v, dbl2 *p) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}

template <int L>
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
        size_t blk;
        if constexpr (L == 0)
            blk = ((size_t)p * C + cat) * n_tiles + tile;
        else if constexpr (L == 1)
            blk = ((size_t)tile * n_slots + p) * C + cat;
        else
            blk = ((size_t)tile * C + cat) * n_slots + p;
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + blk * 256) + lane;
        dbl2 a = {v0, v1}, b = {v2, v3};
        st(a, q);
        st(b, q + 64);
    }
}

__global__ void __launch_bounds__(256) k_stream(dbl2 *out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    dbl2 v = {1.0 * threadIdx.x, 2.0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        st(v, out + i);
}

static double bytes_g;

template <class F>
void timeit(const char *name, F launch, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) launch();
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

template <int L>
void run_layout(double *clv, int n_slots, int n_tiles, int C, int reps) {
    const int grid = (n_tiles * C + 3) / 4;
    char nm[64];
    for (int occ : {4, 6}) {
        const size_t lds = (size_t)(163839 / occ) / 512 * 512;
        snprintf(nm, sizeof nm, "L%d occ%d", L, occ);
        timeit(nm, [&] {
            hipLaunchKernelGGL(k_ops<L>, dim3(grid), dim3(256), lds, 0, clv, n_slots, n_tiles, C);
        }, reps);
    }
}

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = argc > 3 ? atoi(argv[3]) : 4;
    const size_t bytes = (size_t)n_slots * n_tiles * C * 256 * 8;
    bytes_g = (double)bytes;
    const int reps = bytes > (size_t)4e9 ? 5 : 50;
    double *clv;
    if (hipMalloc(&clv, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("bytes per launch %.1f MB, %d CUs, slots %d tiles %d C %d\n", bytes / 1e6, n_cu,
           n_slots, n_tiles, C);
    for (int r = 0; r < 2; ++r) {
        timeit("stream 1 blk/CU", [&] {
            hipLaunchKernelGGL(k_stream, dim3(n_cu), dim3(256), 0, 0, (dbl2 *)clv, bytes / 16);
        }, reps);
        run_layout<0>(clv, n_slots, n_tiles, C, reps);
        run_layout<1>(clv, n_slots, n_tiles, C, reps);
        run_layout<2>(clv, n_slots, n_tiles, C, reps);
    }
    hipFree(clv);
    return 0;
}
