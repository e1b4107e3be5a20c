// Does a 2-D tile order help k_linearize's image reads?  Each wave gathers the footprints of 8
// "residuals" (random centres in one random 640x480 frame of 448, 550 MB > the 256-MiB Infinity
// Cache): the 8x8-pixel box [x-3, x+4] x [y-3, y+4] as the 128-B lines (8x4-pixel intensity tiles)
// it straddles, one 16-B piece per line and lane, as k_linearize's band-column loads do.  Three
// orders of the tiles in memory, the same lines touched:
//   0 row-major tiles (the library's layout: band after band, 80 tiles per band)
//   1 4 KB super-tiles of 4 x 8 tiles (32 x 32 pixels), row-major inside
//   2 4 KB super-tiles of 8 x 4 tiles (64 x 16 pixels)
// A 2-D order keeps a footprint's lines in one 4 KB block (DRAM row / channel locality); if that
// raised the random-line rate, the library's band_offset would change.  Prints GB/s of lines.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/footprint_probe tools/footprint_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int kW = 640, kH = 480, kTpr = kW / 8, kBands = kH / 4;
constexpr int kLinesPerFrame = kTpr * kBands;  // 9600 lines = 1.2 MB

__device__ __forceinline__ unsigned line_of(int order, int tx, int b) {
    if (order == 0) return (unsigned)(b * kTpr + tx);
    if (order == 1) {  // 4 x 8 tiles per 4 KB block
        const int st = (b >> 3) * (kTpr / 4) + (tx >> 2);
        return (unsigned)(st * 32 + (b & 7) * 4 + (tx & 3));
    }
    const int st = (b >> 2) * (kTpr / 8) + (tx >> 3);  // 8 x 4 tiles per 4 KB block
    return (unsigned)(st * 32 + (b & 3) * 8 + (tx & 7));
}

__global__ void k_footprints(const float4 *__restrict__ img, const int4 *__restrict__ res, int n_res, int order,
                             float *out) {
    const int lane = threadIdx.x & 63, g = lane >> 3, sl = lane & 7;
    const int r = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 8 + g;
    if (r >= n_res) return;
    const int4 q = res[r];  // frame, x, y
    const int x0 = q.y - 3, y0 = q.z - 3;
    const int tx0 = x0 >> 3, tx1 = (x0 + 7) >> 3, b0 = y0 >> 2, b1 = (y0 + 7) >> 2;
    const int ntx = tx1 - tx0 + 1;
    const int n = ntx * (b1 - b0 + 1);  // <= 6 lines
    float s = 0.f;
    if (sl < n) {
        const int tx = tx0 + sl % ntx, b = b0 + sl / ntx;
        const size_t line = (size_t)q.x * kLinesPerFrame + line_of(order, tx, b);
        const float4 v = img[line * 8 + (sl & 7)];
        s = v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

int main(int argc, char **argv) {
    const int frames = 448, n_res = argc > 1 ? atoi(argv[1]) : 768000;
    const size_t bytes = (size_t)frames * kLinesPerFrame * 128;
    float4 *img;
    int4 *res;
    float *out;
    CK(hipMalloc(&img, bytes));
    CK(hipMemset(img, 0, bytes));
    CK(hipMalloc(&res, (size_t)n_res * sizeof(int4)));
    CK(hipMalloc(&out, 64));
    std::vector<int4> h(n_res);
    srand(7);
    for (int i = 0; i < n_res; i += 64) {  // 64 residuals of one frame per chunk, as a k_linearize wave
        const int f = rand() % frames;
        for (int k = i; k < i + 64 && k < n_res; k++) h[k] = make_int4(f, 4 + rand() % (kW - 12), 4 + rand() % (kH - 12), 0);
    }
    CK(hipMemcpy(res, h.data(), h.size() * sizeof(int4), hipMemcpyHostToDevice));
    // lines touched per launch (the same for every order)
    long long lines = 0;
    for (const int4 &q : h) {
        const int x0 = q.y - 3, y0 = q.z - 3;
        lines += (long long)(((x0 + 7) >> 3) - (x0 >> 3) + 1) * (((y0 + 7) >> 2) - (y0 >> 2) + 1);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int threads = 256, blocks = (int)(((long long)n_res * 8 + threads - 1) / threads);
    printf("residuals %d, lines per launch %lld (%.1f per residual, %.1f MB)\n", n_res, lines, (double)lines / n_res,
           lines * 128e-6);
    for (int rep = 0; rep < 3; rep++)
        for (int order = 0; order < 3; order++) {
            k_footprints<<<blocks, threads>>>(img, res, n_res, order, out);
            CK(hipDeviceSynchronize());
            float best = 1e30f;
            for (int it = 0; it < 10; it++) {
                CK(hipEventRecord(e0));
                k_footprints<<<blocks, threads>>>(img, res, n_res, order, out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            printf("order %d  %8.2f us  %7.0f GB/s of lines\n", order, best * 1e3, lines * 128.0 / (best * 1e-3) / 1e9);
        }
    CK(hipFree(img));
    CK(hipFree(res));
    CK(hipFree(out));
    return 0;
}
