// Store-bandwidth ceiling, part 7: does splitting a wave's 2 KB per op into two 1 KB pieces in
// separate regions (chunk1-like, write_pattern5: 6.5 TB/s) beat k_prune's adjacent pair
// (5.4-5.7 TB/s)?  k_prune's shape (one wave per (tile, category), 49 ops, 8 dependent fp64
// FMA chains per op), layouts of the 4-double CLV of a (slot, category, tile):
//   L0 [slot][cat][tile][2][64 x 16 B]            today's: the two halves adjacent (2 KB)
//   L1 [slot][half][cat][tile][64 x 16 B]          halves in two regions of the slot
//   L2 [half][slot][cat][tile][64 x 16 B]          halves in two regions of the buffer
//   L3 [slot][half][tile][cat][64 x 16 B]          as L1, a workgroup's 4 waves adjacent
// each on the default grid (1563 workgroups) and on a persistent grid of B blocks per CU.
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern7.hip -o scripts/probes/_write_pattern7
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int L>
__device__ __forceinline__ size_t piece(int p, int h, int cat, int tile, int n_slots, int C,
                                        int n_tiles) {
    // index of a 1 KB piece (64 x 16 B)
    if (L == 0) return (((size_t)p * C + cat) * n_tiles + tile) * 2 + h;
    if (L == 1) return (((size_t)p * 2 + h) * C + cat) * n_tiles + tile;
    if (L == 2) return (((size_t)h * n_slots + p) * C + cat) * n_tiles + tile;
    return (((size_t)p * 2 + h) * n_tiles + tile) * C + cat;
}

template <int L>
__global__ void __launch_bounds__(256) k_ops(dbl2 *out, int n_slots, int n_tiles, int C) {
    const int lane = threadIdx.x & 63, cat = threadIdx.x >> 6;  // C == 4
    for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        double v0 = lane + tile, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3;
        for (int p = 0; p < n_slots; ++p) {
#pragma unroll
            for (int w = 0; w < 8; ++w) {
                v0 = fma(v0, 1.0000001, v1);
                v1 = fma(v1, 0.9999999, v2);
                v2 = fma(v2, 1.0000001, v3);
                v3 = fma(v3, 0.9999999, v0);
            }
            __builtin_nontemporal_store(
                dbl2{v0, v1}, out + piece<L>(p, 0, cat, tile, n_slots, C, n_tiles) * 64 + lane);
            __builtin_nontemporal_store(
                dbl2{v2, v3}, out + piece<L>(p, 1, cat, tile, n_slots, C, n_tiles) * 64 + lane);
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
    printf("%-30s %.4f ms  %6.0f GB/s\n", name, ms, bytes_g / ms / 1e6);
    fflush(stdout);
}

int main() {
    const int n_slots = 49, n_tiles = 1563, C = 4;
    const size_t bytes = (size_t)n_slots * n_tiles * C * 256 * 8;
    bytes_g = (double)bytes;
    dbl2 *buf;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(buf, 0, bytes, 0); });
        for (int B : {0, 1, 2, 6}) {
            const int grid = B == 0 ? n_tiles : n_cu * B;
            char nm[64];
#define RUN(LL)                                                                        \
    snprintf(nm, sizeof nm, "L%d grid %s%d", LL, B ? "B=" : "", B ? B : grid);         \
    timeit(nm, [&] {                                                                   \
        hipLaunchKernelGGL((k_ops<LL>), dim3(grid), dim3(256), 0, 0, buf, n_slots,     \
                           n_tiles, C);                                                \
    });
            RUN(0) RUN(1) RUN(2) RUN(3)
        }
    }
    (void)hipFree(buf);
    return 0;
}
