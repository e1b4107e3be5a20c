// Calibration probe for k_linearize's access pattern: what an MI355X sustains, and
// what rocprofv3 FETCH_SIZE reports, when 128-B lines of an HBM-resident buffer are read
//   stream     float4 per lane, consecutive (the guide's calibrated case)
//   full_rand  whole lines (8 lanes x 16 B) in random line order
//   one_rand   one dword per line, random line order
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/gather_probe tools/gather_probe.hip
// Run:   tools/gather_probe [MiB]   (prints ms and line-GB/s per kernel, 5 launches each)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void k_stream(const float4 *__restrict__ a, long long n4, float *out) {
    float acc = 0.f;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[0] = acc;
}

__global__ void k_full_rand(const float4 *__restrict__ a, const int *__restrict__ perm, int nlines, float *out) {
    const int g = (blockIdx.x * blockDim.x + threadIdx.x) >> 3, sl = threadIdx.x & 7;
    if (g >= nlines) return;
    const float4 v = a[(long long)perm[g] * 8 + sl];
    const float s = v.x + v.y + v.z + v.w;
    if (s == 12345.f) out[0] = s;
}

__global__ void k_one_rand(const float *__restrict__ a, const int *__restrict__ perm, int nlines, float *out) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nlines) return;
    const float s = a[(long long)perm[g] * 32 + (g & 31)];
    if (s == 12345.f) out[0] = s;
}

int main(int argc, char **argv) {
    const long long mib = argc > 1 ? atoll(argv[1]) : 1024;
    const long long bytes = mib << 20;
    const int nlines = (int)(bytes / 128);
    float *a, *out;
    int *perm;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&perm, (size_t)nlines * 4));
    CK(hipMemset(a, 0, bytes));
    std::vector<int> p(nlines);
    std::iota(p.begin(), p.end(), 0);
    std::mt19937 rng(1);
    std::shuffle(p.begin(), p.end(), rng);
    CK(hipMemcpy(perm, p.data(), (size_t)nlines * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        printf("%-10s %8.3f ms  %7.0f GB/s of lines (%lld MiB)\n", name, best, bytes / (best * 1e-3) / 1e9, mib);
    };
    run("stream", [&] { k_stream<<<256 * 16, 256>>>((const float4 *)a, bytes / 16, out); });
    run("full_rand", [&] { k_full_rand<<<(nlines * 8 + 255) / 256, 256>>>((const float4 *)a, perm, nlines, out); });
    run("one_rand", [&] { k_one_rand<<<(nlines + 255) / 256, 256>>>(a, perm, nlines, out); });
    CK(hipFree(a));
    CK(hipFree(out));
    CK(hipFree(perm));
    return 0;
}
