// FETCH_SIZE calibration for k_linearize's read pattern: 16-B pieces
// (buffer_load_dwordx4, one piece per lane) of 128-B lines in random line order, 1, 2, 4 or 8
// contiguous pieces per line (8 = whole lines, the probe of tools/gather_probe.hip).  Every line of
// a 1-GiB buffer (> the 256-MiB Infinity Cache) is touched exactly once per launch, so the bytes
// the HBM must deliver are known: at least the requested pieces, at most the whole lines.
// rocprofv3 --pmc FETCH_SIZE (separate pass) per kernel is then compared with
//   lines x 128 B, lines x 16 B x pieces, and half of each (the gfx950 x2 rule for streams).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/gather_probe_pieces tools/gather_probe_pieces.hip
// Run:   tools/gather_probe_pieces [MiB]   (ms, GB/s of requested and of whole-line bytes)
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

// kP pieces of line perm[g] per group of kP lanes, starting at slot 3g mod 8 (wrapping inside
// the line), through a buffer resource as k_linearize loads its band columns
template <int kP>
__global__ void k_pieces(const float *__restrict__ a, long long bytes, const int *__restrict__ perm, int nlines,
                         float *out) {
    const long long tid = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    const int g = (int)(tid / kP), sl = (int)(tid % kP);
    if (g >= nlines) return;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a), (short)0, (int)(bytes > 0x7FFFFFFF ? 0x7FFFFFFF : bytes), 0x00020000);
    const unsigned slot = (unsigned)((3 * g + sl) & 7);
    const long long off = (long long)perm[g] * 128 + slot * 16;
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    // lines beyond 2 GiB - 1 are out of the resource's range: the probe uses <= 1 GiB
    const i32x4 v = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    const float s = __int_as_float(v.x) + __int_as_float(v.y) + __int_as_float(v.z) + __int_as_float(v.w);
    if (s == 12345.f) out[0] = s;
}

int main(int argc, char **argv) {
    const long long mib = argc > 1 ? atoll(argv[1]) : 1024;
    if (mib > 1024) {
        fprintf(stderr, "at most 1024 MiB (buffer resource range)\n");
        return 1;
    }
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
    printf("lines per launch %d (%lld MiB), perm array %lld KiB read once per launch\n", nlines, mib,
           (long long)nlines * 4 / 1024);
    auto run = [&](const char *name, int pieces, auto launch) {
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
        const double req = (double)nlines * 16 * pieces, whole = (double)nlines * 128;
        printf("%-9s pieces %d  %8.3f ms  requested %7.0f GB/s  whole lines %7.0f GB/s  (requested %.0f KiB, lines %.0f KiB)\n",
               name, pieces, best, req / (best * 1e-3) / 1e9, whole / (best * 1e-3) / 1e9, req / 1024, whole / 1024);
    };
    const int tb = 256;
    run("k_pieces1", 1, [&] { k_pieces<1><<<(int)(((long long)nlines * 1 + tb - 1) / tb), tb>>>(a, bytes, perm, nlines, out); });
    run("k_pieces2", 2, [&] { k_pieces<2><<<(int)(((long long)nlines * 2 + tb - 1) / tb), tb>>>(a, bytes, perm, nlines, out); });
    run("k_pieces4", 4, [&] { k_pieces<4><<<(int)(((long long)nlines * 4 + tb - 1) / tb), tb>>>(a, bytes, perm, nlines, out); });
    run("k_pieces8", 8, [&] { k_pieces<8><<<(int)(((long long)nlines * 8 + tb - 1) / tb), tb>>>(a, bytes, perm, nlines, out); });
    CK(hipFree(a));
    CK(hipFree(out));
    CK(hipFree(perm));
    return 0;
}
