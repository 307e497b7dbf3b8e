// Store-bandwidth microbenchmark for the traversal's CLV write pattern (KEEP mode).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/write_pattern.hip -o /tmp/write_pattern
//   /tmp/write_pattern [n_slots=49] [n_tiles=1563] [C=4]
//
// Every wave (one (tile, category)) writes n_slots CLV blocks of 64 lanes x (K=4 doubles +
// 1 scaler), one block per "op", like k_prune does.  Layouts:
//   slot-major  [slot][cat][tile][...]   (the current tiled layout)
//   tile-major  [tile][cat][slot][...]   (each wave streams into its own contiguous range)
// Reported: GB/s of CLV + scaler bytes, nt (streaming) and normal stores.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <bool TILE_MAJOR, bool NT, int WORK>
__global__ void __launch_bounds__(256) k_write(double *clv, double *scale, int n_slots,
                                               int n_tiles, int C) {
    const int lane = threadIdx.x & 63;
    const int wt = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tile = wt / C, cat = wt - tile * C;
    if (tile >= n_tiles) return;
    double v0 = lane, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3, s = 0.5;
    for (int p = 0; p < n_slots; ++p) {
        // some dependent fp64 work per op, like the 32 FMAs of a pruning update
        for (int w = 0; w < WORK; ++w) {
            v0 = fma(v0, 1.0000001, v1);
            v1 = fma(v1, 0.9999999, v2);
            v2 = fma(v2, 1.0000001, v3);
            v3 = fma(v3, 0.9999999, v0);
        }
        size_t row = TILE_MAJOR ? (((size_t)tile * C + cat) * n_slots + p)
                                : (((size_t)p * C + cat) * n_tiles + tile);
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * 256) + lane;
        dbl2 a = {v0, v1}, b = {v2, v3};
        double *sc = scale + row * 64 + lane;
        if (NT) {
            __builtin_nontemporal_store(a, q);
            __builtin_nontemporal_store(b, q + 64);
            __builtin_nontemporal_store(s, sc);
        } else {
            q[0] = a;
            q[64] = b;
            *sc = s;
        }
    }
}

template <bool TM, bool NT, int WORK>
void run(const char *name, double *clv, double *scale, int n_slots, int n_tiles, int C) {
    const int grid = (n_tiles * C + 3) / 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL((k_write<TM, NT, WORK>), dim3(grid), dim3(256), 0, 0, clv, scale,
                           n_slots, n_tiles, C);
    const int reps = 50;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((k_write<TM, NT, WORK>), dim3(grid), dim3(256), 0, 0, clv, scale,
                           n_slots, n_tiles, C);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double bytes = (double)n_slots * n_tiles * C * 64 * 5 * 8;
    printf("%-28s work=%2d  %.4f ms  %.0f GB/s\n", name, WORK, ms, bytes / ms / 1e6);
}

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = argc > 3 ? atoi(argv[3]) : 4;
    const size_t rows = (size_t)n_slots * n_tiles * C;
    double *clv, *scale;
    if (hipMalloc(&clv, rows * 256 * 8) != hipSuccess ||
        hipMalloc(&scale, rows * 64 * 8) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    // warm the clocks
    for (int i = 0; i < 200; ++i)
        hipLaunchKernelGGL((k_write<false, true, 0>), dim3((n_tiles * C + 3) / 4), dim3(256), 0,
                           0, clv, scale, n_slots, n_tiles, C);
    hipDeviceSynchronize();
    run<false, true, 0>("slot-major nt", clv, scale, n_slots, n_tiles, C);
    run<false, false, 0>("slot-major cached", clv, scale, n_slots, n_tiles, C);
    run<true, true, 0>("tile-major nt", clv, scale, n_slots, n_tiles, C);
    run<true, false, 0>("tile-major cached", clv, scale, n_slots, n_tiles, C);
    run<false, true, 8>("slot-major nt", clv, scale, n_slots, n_tiles, C);
    run<true, true, 8>("tile-major nt", clv, scale, n_slots, n_tiles, C);
    run<false, true, 32>("slot-major nt", clv, scale, n_slots, n_tiles, C);
    run<true, true, 32>("tile-major nt", clv, scale, n_slots, n_tiles, C);
    hipFree(clv);
    hipFree(scale);
    return 0;
}
