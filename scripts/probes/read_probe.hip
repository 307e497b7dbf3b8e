// Read-floor probe for k_edge's shape: how long does a short single-round kernel take to read
// two CLV slots (2 x 12.8 MB) and their scaler rows (2 x 3.2 MB) of a 634 MB buffer, one
// 64-site tile per wave (cfg2: 1563 tiles x 4 categories), with no arithmetic beyond a sum?
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/read_probe.hip -o scripts/_read_probe
// Variants: W waves per workgroup (4 = one tile's categories per workgroup, k_edge's form;
// the per-wave form = one tile's 4 categories per wave), and a pure streaming read of the same
// bytes as one contiguous range.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int kTiles = 1563, kC = 4, kK = 4;
constexpr size_t kSlot = (size_t)kTiles * kC * kK * 64;  // doubles per CLV slot
constexpr size_t kSrow = (size_t)kTiles * kC * 64;       // doubles per scaler slot

// one wave = (tile, category): k_edge's workgroup form
__global__ void __launch_bounds__(256) k_wave_cat(const double *clv, const double *scale,
                                                  int sa, int sb, double *out) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int tile = blockIdx.x, cat = w;
    const size_t row = (size_t)cat * kTiles + tile;
    const dbl2 *a = reinterpret_cast<const dbl2 *>(clv + sa * kSlot + row * kK * 64) + lane;
    const dbl2 *b = reinterpret_cast<const dbl2 *>(clv + sb * kSlot + row * kK * 64) + lane;
    const dbl2 a0 = a[0], a1 = a[64], b0 = b[0], b1 = b[64];
    const double s = scale[sa * kSrow + row * 64 + lane] + scale[sb * kSrow + row * 64 + lane];
    double v = a0.x * b0.x + a0.y * b0.y + a1.x * b1.x + a1.y * b1.y + s;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) out[blockIdx.x * 4 + w] = v;
}

// one wave = one tile with all categories (the per-wave form)
__global__ void __launch_bounds__(256) k_wave_tile(const double *clv, const double *scale,
                                                   int sa, int sb, double *out) {
    const int lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= kTiles) return;
    double v = 0.0;
#pragma unroll
    for (int cat = 0; cat < kC; ++cat) {
        const size_t row = (size_t)cat * kTiles + tile;
        const dbl2 *a = reinterpret_cast<const dbl2 *>(clv + sa * kSlot + row * kK * 64) + lane;
        const dbl2 *b = reinterpret_cast<const dbl2 *>(clv + sb * kSlot + row * kK * 64) + lane;
        const dbl2 a0 = a[0], a1 = a[64], b0 = b[0], b1 = b[64];
        v += a0.x * b0.x + a0.y * b0.y + a1.x * b1.x + a1.y * b1.y +
             scale[sa * kSrow + row * 64 + lane] + scale[sb * kSrow + row * 64 + lane];
    }
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) out[tile] = v;
}

// the same number of bytes as one contiguous grid-stride stream
__global__ void __launch_bounds__(256) k_stream(const dbl2 *p, size_t n, double *out) {
    double v = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const dbl2 t = p[i];
        v += t.x + t.y;
    }
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = v;
}

__global__ void k_empty(double *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1.0;
}

template <class F>
void timeit(const char *name, double bytes, F launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 20; ++i) launch();
    const int reps = 200;
    float total = 0.f;
    for (int r = 0; r < reps; ++r) {  // one launch per event pair, like the edge bench
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        total += ms;
    }
    const double ms = total / reps;
    printf("%-40s %.4f ms  %6.0f GB/s\n", name, ms, bytes / ms / 1e6);
    fflush(stdout);
}

int main() {
    const int n_slots = 49;
    const size_t n = kSlot * n_slots;
    double *clv, *scale, *out;
    if (hipMalloc(&clv, n * 8) != hipSuccess || hipMalloc(&scale, kSrow * n_slots * 8) ||
        hipMalloc(&out, (size_t)kTiles * 4 * 8 * 4))
        return 1;
    (void)hipMemset(clv, 0, n * 8);
    (void)hipMemset(scale, 0, kSrow * n_slots * 8);
    const double bytes = 2.0 * (kSlot + kSrow) * 8;
    const int sa = 17, sb = 40;
    for (int r = 0; r < 2; ++r) {
        timeit("empty kernel (1563 x 256)", bytes, [&] {
            hipLaunchKernelGGL(k_empty, dim3(kTiles), dim3(256), 0, 0, out);
        });
        timeit("wave = (tile, cat), 1563 WG x 4 waves", bytes, [&] {
            hipLaunchKernelGGL(k_wave_cat, dim3(kTiles), dim3(256), 0, 0, clv, scale, sa, sb, out);
        });
        timeit("wave = tile, 391 WG x 4 waves", bytes, [&] {
            hipLaunchKernelGGL(k_wave_tile, dim3((kTiles + 3) / 4), dim3(256), 0, 0, clv, scale,
                               sa, sb, out);
        });
        timeit("contiguous stream, 1024 WG", bytes, [&] {
            hipLaunchKernelGGL(k_stream, dim3(1024), dim3(256), 0, 0,
                               reinterpret_cast<const dbl2 *>(clv + 5 * kSlot),
                               (size_t)(bytes / 16), out);
        });
    }
    return 0;
}
