// FP64 matrix cores on this part: rates of v_mfma_f64_16x16x4_f64 (2048 FLOP) and
// v_mfma_f64_4x4x4_4b_f64 (4 blocks of 4x4x4: 512 FLOP), and the 4x4x4_4b operand layout.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/mfma_f64_probe.hip -o scripts/_mfma_f64_probe
//   scripts/_mfma_f64_probe
//
// throughput: every SIMD of every CU runs W waves, each issuing MFMAs over CH independent
//             accumulators (TFLOP/s over the chip; s_memtime ticks per wave)
// latency:    one chain per wave
// layout:     B one-hot at lane L: D lanes that become non-zero, and the A lane each copies
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH, bool SMALL>
__global__ void __launch_bounds__(256) k_tp(double *out, int n, long long *cyc) {
    const int l = threadIdx.x & 63;
    double a = 1.0 + l * 1e-9, b = 1.0 - l * 1e-9;
    d4 acc[CH];
    double sacc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        acc[c] = d4{0.0, 0.0, 0.0, 0.0};
        sacc[c] = 0.0;
    }
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if constexpr (SMALL)
                sacc[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, sacc[c], 0, 0, 0);
            else
                acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3] + sacc[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}

template <int CH, bool SMALL>
void run(const char *name, int blocks, int n, double *out, long long *cyc) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL((k_tp<CH, SMALL>), dim3(blocks), dim3(256), 0, 0, out, n, cyc);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_tp<CH, SMALL>), dim3(blocks), dim3(256), 0, 0, out, n, cyc);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double mfmas = (double)blocks * 4 * n * CH;
    const double flop = SMALL ? 512.0 : 2048.0;
    printf("%-10s %-30s blocks %5d  %8.3f ms  %6.1f TFLOP/s  %6.1f ticks per MFMA per wave\n",
           SMALL ? "4x4x4_4b" : "16x16x4", name, blocks, ms, mfmas * flop / ms / 1e9,
           (double)c / (n * CH));
}

// D = A B with A = lane + 1 at every lane and B one-hot at lane L; CBSZ = 2 broadcasts
// block ABID's A to all 4 blocks
template <int CBSZ, int ABID>
__global__ void k_layout(double *out) {
    const int l = threadIdx.x;
    for (int L = 0; L < 64; ++L) {
        const double a = l + 1, b = (l == L) ? 1.0 : 0.0;
        const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, CBSZ, ABID, 0);
        out[L * 64 + l] = d;
    }
}

template <int CBSZ, int ABID>
void layout() {
    double *out;
    (void)hipMalloc(&out, 64 * 64 * sizeof(double));
    hipLaunchKernelGGL((k_layout<CBSZ, ABID>), dim3(1), dim3(64), 0, 0, out);
    static double h[64 * 64];
    (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
    printf("4x4x4_4b layout, CBSZ %d ABID %d: B one-hot lane -> [D lane = A lane ...]\n", CBSZ,
           ABID);
    for (int L = 0; L < 64; ++L) {
        if (CBSZ && L % 4) continue;
        printf("B%02d:", L);
        for (int l = 0; l < 64; ++l)
            if (h[L * 64 + l] != 0.0) printf(" D%02d=A%02d", l, (int)h[L * 64 + l] - 1);
        printf("\n");
    }
    (void)hipFree(out);
}

int main() {
    double *out;
    long long *cyc;
    (void)hipMalloc(&out, 256 * 4096 * sizeof(double));
    (void)hipMalloc(&cyc, 8);
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("%s: %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);

    layout<0, 0>();
    layout<2, 1>();
    layout<2, 3>();

    const int n = 20000;
    run<4, false>("4 chains, 1 wave/SIMD", cus, n, out, cyc);
    run<1, false>("1 chain, 1 wave/SIMD", cus, 4 * n, out, cyc);
    run<2, false>("2 chains, 3 waves/SIMD", 3 * cus, 2 * n, out, cyc);
    run<4, true>("4 chains, 1 wave/SIMD", cus, 4 * n, out, cyc);
    run<8, true>("8 chains, 1 wave/SIMD", cus, 2 * n, out, cyc);
    run<1, true>("1 chain, 1 wave/SIMD", cus, 16 * n, out, cyc);
    run<2, true>("2 chains, 3 waves/SIMD", 3 * cus, 8 * n, out, cyc);
    run<4, true>("4 chains, 3 waves/SIMD", 3 * cus, 4 * n, out, cyc);
    run<2, false>("2 chains, 3 waves/SIMD", 3 * cus, 2 * n, out, cyc);
    (void)hipFree(out);
    (void)hipFree(cyc);
    return 0;
}
