// Throughput of k_prune_mfma's MFMA mix with no memory traffic: per "op", 5 k-steps of
// v_mfma_f64_16x16x4 + v_mfma_f64_4x4x4_4b per child (10 + 10 MFMAs for two children),
// accumulating chains as the kernel does.  Variants:
//   both : the two children's chains interleaved per k-step (x0, y0, x4, y4: k_prune_mfma)
//   one  : one child's 5 steps, then the other's (k_prune_mfma_pipe's order)
//   only16: the 16x16x4 MFMAs alone (no 4x4x4_4b)
// Waves per SIMD W = 1, 2, 3, 4 (grid = 256 CUs x 4 SIMDs x W waves, 64-thread blocks).
// Reports cycles per op per SIMD at the measured clock (s_memtime over the kernel) and the
// fraction of the 800-cycle / op busy figure (64 per 16x16x4, 16 per 4x4x4_4b).
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_mix_probe.hip -o scripts/_mfma_mix_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int V>
__global__ void __launch_bounds__(64) k_mix(double *out, int n_ops) {
    const int lane = threadIdx.x;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    d4 x0 = {0, 0, 0, 0}, y0 = {0, 0, 0, 0};
    double x4 = 0, y4 = 0;
    for (int t = 0; t < n_ops; ++t) {
        if (V == 0) {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, x0, 0, 0, 0);
                y0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, y0, 0, 0, 0);
                x4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, x4, 0, 0, 0);
                y4 = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, y4, 0, 0, 0);
            }
        } else if (V == 1) {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, x0, 0, 0, 0);
                x4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, x4, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                y0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, y0, 0, 0, 0);
                y4 = __builtin_amdgcn_mfma_f64_4x4x4f64(b, a, y4, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, x0, 0, 0, 0);
                y0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, y0, 0, 0, 0);
            }
        }
        // a dependency on the results each op, as the epilogue has
        a = a * 0.999999 + x0[0] * 1e-30 + x4 * 1e-30;
        b = b * 1.000001 + y0[1] * 1e-30 + y4 * 1e-30;
    }
    out[blockIdx.x * 64 + lane] = x0[0] + x0[1] + x0[2] + x0[3] + y0[0] + x4 + y4;
}

int main() {
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    (void)hipMalloc(&out, (size_t)n_cu * 4 * 8 * 64 * 8);
    const int n_ops = 2000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[3] = {"both interleaved", "one side then other", "16x16x4 only"};
    const double busy[3] = {800, 800, 640};
    for (int v = 0; v < 3; ++v)
        for (int W : {1, 2, 3, 4}) {
            const int grid = n_cu * 4 * W;
            auto launch = [&] {
                if (v == 0) hipLaunchKernelGGL(k_mix<0>, dim3(grid), dim3(64), 0, 0, out, n_ops);
                if (v == 1) hipLaunchKernelGGL(k_mix<1>, dim3(grid), dim3(64), 0, 0, out, n_ops);
                if (v == 2) hipLaunchKernelGGL(k_mix<2>, dim3(grid), dim3(64), 0, 0, out, n_ops);
            };
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            // cycles per op per SIMD at 2.4 GHz: W waves x n_ops ops each
            const double cyc = ms * 1e-3 * 2.4e9 / ((double)W * n_ops);
            printf("%-22s W=%d  %.3f ms  %6.0f cycles/op/SIMD  busy frac %.2f\n", names[v], W, ms,
                   cyc, busy[v] / cyc);
            fflush(stdout);
        }
    return 0;
}
