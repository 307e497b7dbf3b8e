// Store-bandwidth ceiling, part 6: staggered starts.  write_pattern3/5 showed that a store
// stream runs at 6.5 TB/s when the addresses written at any moment form a small window that
// moves monotonically (one 256-thread block per CU, 1 KB per wave per grid step) and at
// 4.2-5.5 TB/s when they are spread over several MB in random order.  k_prune's waves all
// start together and write op t's slot (12.8 MB) at about the same time, in no particular
// tile order.  Here each workgroup first waits (blockIdx / grid) * D microseconds, so that
// within one op period the tiles write their blocks in tile order: a write front that sweeps
// each slot sequentially.
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/write_pattern6.hip -o scripts/probes/_write_pattern6
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

// L 0: [slot][cat][tile][4][64] (k_prune's), 1: [slot][tile][cat][4][64]
template <int L>
__global__ void __launch_bounds__(256) k_ops(double *clv, int n_slots, int n_tiles, int C,
                                             int delay_ticks, int work) {
    const int lane = threadIdx.x & 63;
    const int wt = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tile = wt / C, cat = wt - tile * C;
    if (tile >= n_tiles) return;
    if (delay_ticks > 0) {  // 100 MHz real-time counter
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long until =
            t0 + (unsigned long long)delay_ticks * blockIdx.x / gridDim.x;
        while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(2);
    }
    double v0 = lane, v1 = lane + 1, v2 = lane + 2, v3 = lane + 3;
    for (int p = 0; p < n_slots; ++p) {
        for (int w = 0; w < work; ++w) {
            v0 = fma(v0, 1.0000001, v1);
            v1 = fma(v1, 0.9999999, v2);
            v2 = fma(v2, 1.0000001, v3);
            v3 = fma(v3, 0.9999999, v0);
        }
        size_t row;
        if (L == 0)
            row = ((size_t)p * C + cat) * n_tiles + tile;
        else
            row = ((size_t)p * n_tiles + tile) * C + cat;
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
    if (hipMalloc(&clv, bytes) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    const int grid = (n_tiles * C + 3) / 4;
    for (int r = 0; r < 2; ++r) {
        timeit("memsetAsync", [&] { (void)hipMemsetAsync(clv, 0, bytes, 0); });
        for (int work : {8, 32}) {
            for (int d : {0, 100, 200, 300, 500, 1000}) {  // ticks of 10 ns
                char nm[64];
                snprintf(nm, sizeof nm, "slot-cat-tile w%d delay %dus", work, d / 100);
                if (d % 100) snprintf(nm, sizeof nm, "slot-cat-tile w%d delay %d0ns", work, d);
                timeit(nm, [&] {
                    hipLaunchKernelGGL((k_ops<0>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                                       n_tiles, C, d, work);
                });
                snprintf(nm, sizeof nm, "slot-tile-cat w%d delay %d0ns", work, d);
                timeit(nm, [&] {
                    hipLaunchKernelGGL((k_ops<1>), dim3(grid), dim3(256), 0, 0, clv, n_slots,
                                       n_tiles, C, d, work);
                });
            }
        }
    }
    (void)hipFree(clv);
    return 0;
}
