// Launch-floor probe: how long does a small kernel take on the GPU timeline?
//   k_empty       15 blocks, no memory access
//   k_touch       15 blocks, one dependent load + store per thread (buffer written by the
//                 previous launch: the k_stitch -> k_stitch_sum pattern)
//   k_chain4      15 blocks, four dependent loads per thread
//   k_bigcode     15 blocks, ~16 KB of straight-line code (8 independent FMA chains, ~2k
//                 instructions): separates instruction-fetch cost from memory latency
// Run under rocprofv3 --kernel-trace --stats; the program also prints HIP-event times.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int *o) {
    if (threadIdx.x == 1000) o[0] = 1;  // never true: keeps the kernel non-trivial to the compiler
}
__global__ void k_touch(const double *in, double *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    out[i] = in[i] + 1.0;
}
__global__ void k_chain4(const int *idx, const double *in, double *out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    int j = idx[i];
    j = idx[j];
    j = idx[j];
    out[i] = in[j] + 1.0;
}

__global__ void k_bigcode(float *o, float a) {
    float x[8];
#pragma unroll
    for (int c = 0; c < 8; c++) x[c] = (float)(threadIdx.x + c);
#pragma unroll
    for (int i = 0; i < 128; i++)
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = fmaf(x[c], a, (float)(i * 8 + c) * 0.37f + 1.0f);
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) s += x[c];
    o[blockIdx.x * 256 + threadIdx.x] = s;
}

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main() {
    const int nb = 15, n = nb * 256;
    double *a, *b;
    int *idx, *o;
    CK(hipMalloc(&a, n * sizeof(double)));
    CK(hipMalloc(&b, n * sizeof(double)));
    CK(hipMalloc(&idx, n * sizeof(int)));
    CK(hipMalloc(&o, sizeof(int)));
    int h_idx[15 * 256];
    for (int i = 0; i < n; i++) h_idx[i] = (i * 97 + 13) % n;
    CK(hipMemcpy(idx, h_idx, sizeof(h_idx), hipMemcpyHostToDevice));
    CK(hipMemset(a, 0, n * sizeof(double)));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[5] = {"k_empty", "k_touch", "k_chain4", "k_bigcode", "k_bigcode+k_empty pair"};
    for (int which = 0; which < 5; which++) {
        for (int rep = 0; rep < 2; rep++) {  // rep 0 warms up
            const int iters = 200;
            CK(hipEventRecord(e0, s));
            for (int it = 0; it < iters; it++) {
                if (which == 0) k_empty<<<nb, 256, 0, s>>>(o);
                else if (which == 1) k_touch<<<nb, 256, 0, s>>>(it & 1 ? b : a, it & 1 ? a : b);
                else if (which == 2) k_chain4<<<nb, 256, 0, s>>>(idx, it & 1 ? b : a, it & 1 ? a : b);
                else if (which == 3) k_bigcode<<<nb, 256, 0, s>>>(reinterpret_cast<float *>(b), 0.999f);
                else {  // alternating kernels: the big kernel's code is not the last one run
                    k_bigcode<<<nb, 256, 0, s>>>(reinterpret_cast<float *>(b), 0.999f);
                    k_empty<<<nb, 256, 0, s>>>(o);
                }
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) std::printf("%s: %.2f us per launch (back to back, %d launches)\n", names[which], 1e3 * ms / iters, iters);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
