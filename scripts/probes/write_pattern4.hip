// Store-bandwidth ceiling, part 4 (after write_pattern3: a flat stream reaches 6.5 TB/s with
// ONE 256-thread block per CU and falls to 4.2-4.7 TB/s with 4-16 blocks per CU, i.e. the
// width of the concurrently written address window matters).  Here k_prune's shape -- one wave
// per (tile, category), 49 ops, one 2 KB block per op, some fp64 work per op -- is run as a
// persistent grid: B workgroups per CU walk the tiles in rounds, so at any moment only
// n_cu * B adjacent tiles are being written.
//   pers-slot B  : slot-major layout [slot][cat][tile][4][64] (today's)
//   pers-group B : [round][slot][cat][tile-in-round][4][64]: the tiles of one round write one
//                  contiguous n_cu*B*8 KB window per op
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern4.hip -o scripts/probes/_write_pattern4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int L, int WORK>
__global__ void __launch_bounds__(256) k_pers(double *clv, int n_slots, int n_tiles, int C) {
    const int lane = threadIdx.x & 63;
    const int cat = threadIdx.x >> 6;  // C == 4: one workgroup = one tile
    const int grid = gridDim.x;
    for (int tile = blockIdx.x; tile < n_tiles; tile += grid) {
        const int round = tile / grid, tin = tile - round * grid;
        double v0 = lane + tile, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3;
        for (int p = 0; p < n_slots; ++p) {
#pragma unroll
            for (int w = 0; w < WORK; ++w) {
                v0 = fma(v0, 1.0000001, v1);
                v1 = fma(v1, 0.9999999, v2);
                v2 = fma(v2, 1.0000001, v3);
                v3 = fma(v3, 0.9999999, v0);
            }
            size_t row;
            if (L == 0) {
                row = ((size_t)p * C + cat) * n_tiles + tile;
            } else {
                const size_t r0 = (size_t)round * grid * C * n_slots;  // rows before this round
                const int in_round = min(grid, n_tiles - round * grid);
                row = r0 + ((size_t)p * C + cat) * in_round + tin;
            }
            dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * 256) + lane;
            dbl2 a = {v0, v1}, b = {v2, v3};
            __builtin_nontemporal_store(a, q);
            __builtin_nontemporal_store(b, q + 64);
        }
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

int main(int argc, char **argv) {
    const int n_slots = argc > 1 ? atoi(argv[1]) : 49;
    const int n_tiles = argc > 2 ? atoi(argv[2]) : 1563;
    const int C = 4;
    const size_t rows = (size_t)n_slots * n_tiles * C;
    const size_t bytes = rows * 256 * 8;
    bytes_g = (double)bytes;
    double *clv;
    if (hipMalloc(&clv, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("bytes per launch %.1f MB, %d CUs\n", bytes / 1e6, n_cu);
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(clv, 0, bytes, 0); });
        for (int B : {1, 2, 3, 4, 6, 7}) {
            const int grid = std::min(n_cu * B, n_tiles);
            char nm[64];
            snprintf(nm, sizeof nm, "pers-slot  B=%d w8", B);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_pers<0, 8>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                                   n_tiles, C);
            });
            snprintf(nm, sizeof nm, "pers-group B=%d w8", B);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_pers<1, 8>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                                   n_tiles, C);
            });
            snprintf(nm, sizeof nm, "pers-group B=%d w0", B);
            timeit(nm, [&] {
                hipLaunchKernelGGL((k_pers<1, 0>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                                   n_tiles, C);
            });
        }
    }
    (void)hipFree(clv);
    return 0;
}
