// Store-bandwidth microbenchmark, part 2: which CLV layout writes fastest (KEEP mode).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/write_pattern2.hip -o scripts/_write_pattern2
//   scripts/_write_pattern2 [n_slots=49] [n_tiles=1563] [C=4]
//
// Every wave (one (tile, category)) writes n_slots blocks of 64 lanes x K=4 doubles (+ one
// scaler per lane when SC), one block per "op", as k_prune does, streamed (nt).  Layouts:
//   0 slot-major  [slot][cat][tile][4][64], scalers [slot][cat][tile][64] (k_prune today)
//   2 wg-major    [slot][tile][cat][4][64]: a workgroup's 4 category waves write 8 KB
//   3 fused       [slot][cat][tile][5][64]: CLV and scaler adjacent (2.5 KB per wave)
//   4 wg-fused    [slot][tile][cat][5][64]: 10 KB per workgroup
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int L, bool SC>
__global__ void __launch_bounds__(256) k_write(double *clv, double *scale, int n_slots,
                                               int n_tiles, int C) {
    const int lane = threadIdx.x & 63;
    const int wt = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tile = wt / C, cat = wt - tile * C;
    if (tile >= n_tiles) return;
    double v0 = lane, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3, s = 0.5;
    for (int p = 0; p < n_slots; ++p) {
        for (int w = 0; w < 8; ++w) {  // some dependent fp64 work per op
            v0 = fma(v0, 1.0000001, v1);
            v1 = fma(v1, 0.9999999, v2);
            v2 = fma(v2, 1.0000001, v3);
            v3 = fma(v3, 0.9999999, v0);
        }
        size_t row;
        if (L == 0 || L == 3)
            row = ((size_t)p * C + cat) * n_tiles + tile;
        else
            row = ((size_t)p * n_tiles + tile) * C + cat;
        const size_t stride = (L >= 3) ? 320 : 256;  // doubles per (row)
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * stride) + lane;
        double *sc = (L >= 3) ? clv + row * stride + 256 + lane : scale + row * 64 + lane;
        dbl2 a = {v0, v1}, b = {v2, v3};
        __builtin_nontemporal_store(a, q);
        __builtin_nontemporal_store(b, q + 64);
        if (SC) __builtin_nontemporal_store(s, sc);
    }
}

template <int L, bool SC>
void run(const char *name, double *clv, double *scale, int n_slots, int n_tiles, int C) {
    const int grid = (n_tiles * C + 3) / 4;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL((k_write<L, SC>), dim3(grid), dim3(256), 0, 0, clv, scale, n_slots,
                           n_tiles, C);
    const int reps = 50;
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((k_write<L, SC>), dim3(grid), dim3(256), 0, 0, clv, scale, n_slots,
                           n_tiles, C);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double bytes = (double)n_slots * n_tiles * C * 64 * (SC ? 5 : 4) * 8;
    printf("%-22s scaler=%d  %.4f ms  %.0f GB/s\n", name, SC ? 1 : 0, ms, bytes / ms / 1e6);
}

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = argc > 3 ? atoi(argv[3]) : 4;
    const size_t rows = (size_t)n_slots * n_tiles * C;
    double *clv, *scale;
    if (hipMalloc(&clv, rows * 320 * 8) != hipSuccess ||
        hipMalloc(&scale, rows * 64 * 8) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    for (int i = 0; i < 200; ++i)
        hipLaunchKernelGGL((k_write<0, true>), dim3((n_tiles * C + 3) / 4), dim3(256), 0, 0,
                           clv, scale, n_slots, n_tiles, C);
    hipDeviceSynchronize();
    for (int r = 0; r < 2; ++r) {
        run<0, true>("slot-major", clv, scale, n_slots, n_tiles, C);
        run<0, false>("slot-major", clv, scale, n_slots, n_tiles, C);
        run<2, true>("wg-major", clv, scale, n_slots, n_tiles, C);
        run<2, false>("wg-major", clv, scale, n_slots, n_tiles, C);
        run<3, true>("fused", clv, scale, n_slots, n_tiles, C);
        run<4, true>("wg-fused", clv, scale, n_slots, n_tiles, C);
    }
    hipFree(clv);
    hipFree(scale);
    return 0;
}
