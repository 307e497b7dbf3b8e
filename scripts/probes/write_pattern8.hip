// Store-bandwidth probe, part 8: does arithmetic between the stores slow a k_prune-shaped
// store stream because it is VALU work?  Same stream as write_pattern6 (one wave per (tile,
// category), 49 ops x 2 KB, 627 MB), with per op either no arithmetic, W dependent
// v_fma_f64 chains (VALU), or the same flop count as v_mfma_f64_4x4x4_4b (matrix core), or
// W independent VALU FMAs (throughput, not latency).
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern8.hip -o scripts/probes/_write_pattern8
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double dbl2 __attribute__((ext_vector_type(2)));

// MODE 0: none; 1: dependent VALU fma chains; 2: MFMA 4x4x4_4b; 3: independent VALU fmas
template <int MODE, int W>
__global__ void __launch_bounds__(256) k_ops(double *clv, int n_slots, int n_tiles, int C) {
    const int lane = threadIdx.x & 63;
    const int wt = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tile = wt / C, cat = wt - tile * C;
    if (tile >= n_tiles) return;
    double v0 = lane, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3;
    for (int p = 0; p < n_slots; ++p) {
        if constexpr (MODE == 1) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                v0 = fma(v0, 1.0000001, v1);
                v1 = fma(v1, 0.9999999, v2);
                v2 = fma(v2, 1.0000001, v3);
                v3 = fma(v3, 0.9999999, v0);
            }
        } else if constexpr (MODE == 2) {
            // one 4x4x4_4b = 256 MACs per wave = 4 per lane: W / 2 x 2 of them = 4 W MACs per
            // lane, the VALU variant's 4 W fmas per lane (W = 8: the 8 MFMAs a DNA op needs)
#pragma unroll
            for (int w = 0; w < W / 2; ++w) {
                v0 = __builtin_amdgcn_mfma_f64_4x4x4f64(v1, v2, v0, 0, 0, 0);
                v3 = __builtin_amdgcn_mfma_f64_4x4x4f64(v2, v1, v3, 0, 0, 0);
            }
        } else if constexpr (MODE == 3) {
            double a[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] = v0 + i;
#pragma unroll
            for (int w = 0; w < W / 2; ++w)
#pragma unroll
                for (int i = 0; i < 8; ++i) a[i] = fma(a[i], 1.0000001, v1);
            v0 = a[0] + a[1] + a[2] + a[3];
            v2 = a[4] + a[5] + a[6] + a[7];
        }
        const size_t row = ((size_t)p * C + cat) * n_tiles + tile;
        dbl2 *q = reinterpret_cast<dbl2 *>(clv + row * 256) + lane;
        __builtin_nontemporal_store(dbl2{v0, v1}, q);
        __builtin_nontemporal_store(dbl2{v2, v3}, q + 64);
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
    printf("%-34s %.4f ms  %6.0f GB/s\n", name, ms, bytes_g / ms / 1e6);
    fflush(stdout);
}

int main() {
    const int n_slots = 49, n_tiles = 1563, C = 4;
    const size_t bytes = (size_t)n_slots * n_tiles * C * 256 * 8;
    bytes_g = (double)bytes;
    double *clv;
    if (hipMalloc(&clv, bytes) != hipSuccess) return 1;
    const int grid = (n_tiles * C + 3) / 4;
#define RUN(M, W, NAME)                                                                        \
    timeit(NAME, [&] {                                                                         \
        hipLaunchKernelGGL((k_ops<M, W>), dim3(grid), dim3(256), 0, 0, clv, n_slots, n_tiles, \
                           C);                                                                 \
    });
    for (int r = 0; r < 2; ++r) {
        RUN(0, 0, "no arithmetic")
        RUN(1, 8, "VALU dependent 32 fma")
        RUN(3, 8, "VALU independent 32 fma")
        RUN(2, 8, "MFMA 4x4x4_4b x8")
        RUN(1, 16, "VALU dependent 64 fma")
        RUN(3, 16, "VALU independent 64 fma")
        RUN(2, 16, "MFMA 4x4x4_4b x16")
    }
    (void)hipFree(clv);
    return 0;
}
