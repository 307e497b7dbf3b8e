// r05 probe: where do k_pmatrix_aa's ~9-10 us per launch go (cfg3: 1592 = 398 sides x 4
// categories of 20 x 20 P)?  Variants of the library kernel's body, timed back-to-back with
// hipEvents:  MODE 0 full, 1 P only, 2 A operands only, 3 no stores (kept live), 4 no exp,
// 5 empty body (launch + dispatch floor), 6 one wave per matrix with full stores, 7 the r05
// per-side kernel, 8 an empty grid of its shape.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/pmat_probe scripts/probes/pmat_aa_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int K = 20, KK = K * K, kBlock = 256;

template <int MODE>
__global__ void __launch_bounds__(kBlock) k_var(int C, const double *evecs, const double *evals,
                                                const double *ivecs, const double *brlens,
                                                const double *rates, double *P, double *Pa) {
    if constexpr (MODE == 5) return;
    __shared__ double evx[KK], iv[KK], ex[K];
    const int sd = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
    const bool hi = tid + kBlock < KK;
    const double e0 = evecs[tid], e1 = hi ? evecs[tid + kBlock] : 0.0;
    iv[tid] = ivecs[tid];
    if (hi) iv[tid + kBlock] = ivecs[tid + kBlock];
    if (tid < K) {
        const double x = evals[tid] * (brlens[sd] * rates[c]);
        ex[tid] = MODE == 4 ? x : exp(x);
    }
    __syncthreads();
    evx[tid] = e0 * ex[tid % K];
    if (hi) evx[tid + kBlock] = e1 * ex[(tid + kBlock) % K];
    __syncthreads();
    const size_t m = (size_t)sd * C + c;
    double *out = P + m * KK;
    double *pa = Pa + m * 5 * 128;
    auto put = [&](int i, int j, double v) {
        if (MODE == 3) {
            if (v == 12345.678) out[0] = v;
            return;
        }
        if (MODE != 2) out[i * K + j] = v;
        if (MODE == 1) return;
        double *o = pa + (j >> 2) * 128 + 2 * (16 * (j & 3));
        if (i < 16) {
            o[2 * i] = v;
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b) o[2 * (4 * b + i - 16) + 1] = v;
        }
    };
    if (tid < 12 * K) {
        const int r = tid / K, j = tid - r * K;
        const bool two = r + 12 < K;
        double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double b = iv[k * K + j];
            acc0 = fma(evx[r * K + k], b, acc0);
            if (two) acc1 = fma(evx[(r + 12) * K + k], b, acc1);
        }
        put(r, j, acc0);
        if (two) put(r + 12, j, acc1);
    }
}

// one wave per (side, category)
__global__ void __launch_bounds__(64) k_wave(int C, const double *evecs, const double *evals,
                                             const double *ivecs, const double *brlens,
                                             const double *rates, double *P, double *Pa) {
    __shared__ double evx[KK], iv[KK], ex[K];
    const int sd = blockIdx.x, c = blockIdx.y, l = threadIdx.x;
    if (l < K) ex[l] = exp(evals[l] * (brlens[sd] * rates[c]));
    double e[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int idx = l + 64 * q;
        e[q] = idx < KK ? evecs[idx] : 0.0;
        if (idx < KK) iv[idx] = ivecs[idx];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 7; ++q) {
        const int idx = l + 64 * q;
        if (idx < KK) evx[idx] = e[q] * ex[idx % K];
    }
    __syncthreads();
    const size_t m = (size_t)sd * C + c;
    double *out = P + m * KK;
    double *pa = Pa + m * 5 * 128;
    // lane (g, j), g < 3: rows g, g + 3, ...
    if (l >= 60) return;
    const int g = l / K, j = l - g * K;
    double acc[7];
#pragma unroll
    for (int r = 0; r < 7; ++r) acc[r] = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double b = iv[k * K + j];
#pragma unroll
        for (int r = 0; r < 7; ++r)
            if (g + 3 * r < K) acc[r] = fma(evx[(g + 3 * r) * K + k], b, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        const int i = g + 3 * r;
        if (i >= K) continue;
        out[i * K + j] = acc[r];
        double *o = pa + (j >> 2) * 128 + 2 * (16 * (j & 3));
        if (i < 16) o[2 * i] = acc[r];
        else
            for (int b = 0; b < 4; ++b) o[2 * (4 * b + i - 16) + 1] = acc[r];
    }
}

// r05 library form: one workgroup per side and up to 4 categories, P via LDS, contiguous stores
__global__ void __launch_bounds__(kBlock) k_side(int C, const double *evecs, const double *evals,
                                                 const double *ivecs, const double *brlens,
                                                 const double *rates, double *P, double *Pa) {
    constexpr int NA = 5 * 128, CP = 4;
    __shared__ double ev[KK], iv[KK], ex[CP][K], pm[CP * KK];
    const int sd = blockIdx.x, c0 = blockIdx.y * CP, tid = threadIdx.x;
    const int nc = min(CP, C - c0);
    for (int e = tid; e < KK; e += kBlock) {
        ev[e] = evecs[e];
        iv[e] = ivecs[e];
    }
    if (tid < nc * K) {
        const int c = tid / K, k = tid - c * K;
        ex[c][k] = exp(evals[k] * (brlens[sd] * rates[c0 + c]));
    }
    __syncthreads();
    if (tid < nc * K * 3) {
        constexpr int G = 3, R = (K + G - 1) / G;
        const int c = tid / (G * K), r = tid - c * G * K, j = r / G, g = r - j * G;
        double acc[R];
#pragma unroll
        for (int m = 0; m < R; ++m) acc[m] = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double b = iv[k * K + j], x = ex[c][k];
#pragma unroll
            for (int m = 0; m < R; ++m)
                if (g + G * m < K) acc[m] = fma(ev[(g + G * m) * K + k] * x, b, acc[m]);
        }
#pragma unroll
        for (int m = 0; m < R; ++m)
            if (g + G * m < K) pm[c * KK + (g + G * m) * K + j] = acc[m];
    }
    __syncthreads();
    double *Po = P + ((size_t)sd * C + c0) * KK;
    for (int o = tid; o < nc * KK; o += kBlock) Po[o] = pm[o];
    double *Pao = Pa + ((size_t)sd * C + c0) * NA;
    for (int o = tid; o < nc * NA; o += kBlock) {
        const int c = o / NA, r = o - c * NA, q = r >> 7, lane = (r & 127) >> 1, h = r & 1;
        const int col = 4 * q + (lane >> 4), row = h ? 16 + (lane & 3) : (lane & 15);
        Pao[o] = pm[c * KK + row * K + col];
    }
}

// per (side, category) as the r04 kernel, P staged in LDS, only the A operands stored, as
// contiguous runs (P itself rebuilt from them on demand)
__global__ void __launch_bounds__(kBlock) k_cat_pa(int C, const double *evecs, const double *evals,
                                                   const double *ivecs, const double *brlens,
                                                   const double *rates, double *P, double *Pa) {
    constexpr int NA = 5 * 128;
    __shared__ double evx[KK], iv[KK], ex[K], pm[KK];
    const int sd = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
    const bool hi = tid + kBlock < KK;
    const double e0 = evecs[tid], e1 = hi ? evecs[tid + kBlock] : 0.0;
    iv[tid] = ivecs[tid];
    if (hi) iv[tid + kBlock] = ivecs[tid + kBlock];
    if (tid < K) ex[tid] = exp(evals[tid] * (brlens[sd] * rates[c]));
    __syncthreads();
    evx[tid] = e0 * ex[tid % K];
    if (hi) evx[tid + kBlock] = e1 * ex[(tid + kBlock) % K];
    __syncthreads();
    if (tid < 12 * K) {
        const int r = tid / K, j = tid - r * K;
        const bool two = r + 12 < K;
        double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double b = iv[k * K + j];
            acc0 = fma(evx[r * K + k], b, acc0);
            if (two) acc1 = fma(evx[(r + 12) * K + k], b, acc1);
        }
        pm[r * K + j] = acc0;
        if (two) pm[(r + 12) * K + j] = acc1;
    }
    __syncthreads();
    double *Pao = Pa + ((size_t)sd * C + c) * NA;
    for (int o = tid; o < NA; o += kBlock) {
        const int q = o >> 7, lane = (o & 127) >> 1, h = o & 1;
        const int col = 4 * q + (lane >> 4), row = h ? 16 + (lane & 3) : (lane & 15);
        Pao[o] = pm[row * K + col];
    }
}

int main() {
    const int sides = 398, C = 4;
    std::vector<double> h(KK * 2 + K + sides + C);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01 * ((i * 37) % 101) - 0.3;
    double *d, *P, *Pa;
    CK(hipMalloc(&d, h.size() * 8));
    CK(hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&P, (size_t)sides * C * KK * 8));
    CK(hipMalloc(&Pa, (size_t)sides * C * 640 * 8));
    const double *ev = d, *iv = d + KK, *el = d + 2 * KK, *bl = el + K, *rt = bl + sides;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"full", "P only", "Pa only", "no stores", "no exp", "empty", "one wave", "r05 side", "side empty", "cat Pa lds"};
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 10; ++mode) {
            auto launch = [&]() {
                dim3 g(sides, C);
                switch (mode) {
                case 0: hipLaunchKernelGGL(k_var<0>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 1: hipLaunchKernelGGL(k_var<1>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 2: hipLaunchKernelGGL(k_var<2>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 3: hipLaunchKernelGGL(k_var<3>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 4: hipLaunchKernelGGL(k_var<4>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 5: hipLaunchKernelGGL(k_var<5>, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 6: hipLaunchKernelGGL(k_wave, g, dim3(64), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 7: hipLaunchKernelGGL(k_side, dim3(sides, 1), dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 8: hipLaunchKernelGGL(k_var<5>, dim3(sides, 1), dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                case 9: hipLaunchKernelGGL(k_cat_pa, g, dim3(kBlock), 0, 0, C, ev, el, iv, bl, rt, P, Pa); break;
                }
            };
            for (int i = 0; i < 20; ++i) launch();
            CK(hipDeviceSynchronize());
            // single launches, each timed alone (the library's case: one per step)
            float best = 1e9, sum = 0;
            for (int i = 0; i < 50; ++i) {
                CK(hipEventRecord(e0, 0));
                launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                sum += ms;
            }
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < 200; ++i) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-10s single min %.2f us mean %.2f us | back-to-back %.2f us\n", names[mode],
                   best * 1e3, sum / 50 * 1e3, ms / 200 * 1e3);
        }
    return 0;
}
