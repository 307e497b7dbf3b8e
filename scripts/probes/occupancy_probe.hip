// How many 256-thread workgroups with a given dynamic LDS size run concurrently per CU?
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/occupancy_probe.hip -o scripts/_occupancy_probe
//   scripts/_occupancy_probe <regs variant 0-4> 20000 22000 22656 23552 24576 ...
//
// Each workgroup holds its CU for ~50 us and records (start, end) in s_memrealtime ticks;
// with far more workgroups than fit, peak concurrency = workgroups resident at once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int REGS>
__global__ void __launch_bounds__(256) k_probe(unsigned long long *t, int spin) {
    extern __shared__ double lds[];
    // raise the kernel's VGPR / SGPR high-water marks to those of the traversal kernel
    if constexpr (REGS == 1) asm volatile("" ::: "v64", "s99");
    if constexpr (REGS == 2) asm volatile("" ::: "v71", "s99");
    if constexpr (REGS == 3) asm volatile("" ::: "v63", "s99");
    if constexpr (REGS == 4) asm volatile("" ::: "v64", "s90");
    if constexpr (REGS == 5) asm volatile("" ::: "v63");
    if constexpr (REGS == 6) asm volatile("" ::: "v56");
    if constexpr (REGS == 7) asm volatile("" ::: "s99");
    if constexpr (REGS == 8) asm volatile("" ::: "s80");
    if constexpr (REGS == 9) asm volatile("" ::: "v47");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    unsigned long long now = t0;
    while (now - t0 < (unsigned long long)spin) {
        __builtin_amdgcn_s_sleep(8);
        now = __builtin_amdgcn_s_memrealtime();
    }
    if (threadIdx.x == 0) {
        t[2 * blockIdx.x] = t0;
        t[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() + (lds[5] > 1e30 ? 1 : 0);
    }
}

int main(int argc, char **argv) {
    const int n = 256 * 16;
    unsigned long long *d;
    if (hipMalloc(&d, 2 * n * sizeof(unsigned long long)) != hipSuccess) return 1;
    std::vector<unsigned long long> h(2 * n);
    for (int i = 1; i < argc; ++i) {
        const int lds = atoi(argv[i]);
        const int regs = i == 1 ? 0 : atoi(argv[1]);
        if (i == 1) continue;  // argv[1]: register variant
        switch (regs) {  // 50 us @ 100 MHz
            case 1: hipLaunchKernelGGL(k_probe<1>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 2: hipLaunchKernelGGL(k_probe<2>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 3: hipLaunchKernelGGL(k_probe<3>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 4: hipLaunchKernelGGL(k_probe<4>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 5: hipLaunchKernelGGL(k_probe<5>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 6: hipLaunchKernelGGL(k_probe<6>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 7: hipLaunchKernelGGL(k_probe<7>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 8: hipLaunchKernelGGL(k_probe<8>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            case 9: hipLaunchKernelGGL(k_probe<9>, dim3(n), dim3(256), lds, 0, d, 5000); break;
            default: hipLaunchKernelGGL(k_probe<0>, dim3(n), dim3(256), lds, 0, d, 5000);
        }
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("lds %d: launch failed\n", lds);
            continue;
        }
        if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        // peak number of overlapping [start, end) intervals
        std::vector<std::pair<unsigned long long, int>> ev;
        for (int b = 0; b < n; ++b) {
            ev.push_back({h[2 * b], 1});
            ev.push_back({h[2 * b + 1], -1});
        }
        std::sort(ev.begin(), ev.end());
        int cur = 0, peak = 0;
        for (auto &e : ev) peak = std::max(peak, cur += e.second);
        printf("regs %d lds %6d B: peak %5d resident workgroups = %.2f per CU (256 CUs)\n", regs, lds, peak,
               peak / 256.0);
    }
    hipFree(d);
    return 0;
}
