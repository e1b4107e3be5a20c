// Dependent-chain latencies of the instructions k_solve_reg's serial chain is made of, one
// wave, s_memtime around 256 dependent repetitions (cycles per repetition printed).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double readlane_f64(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ double dpp_max(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    const int olo = __builtin_amdgcn_update_dpp(lo, lo, 0x111, 0xF, 0xF, false);
    const int ohi = __builtin_amdgcn_update_dpp(hi, hi, 0x111, 0xF, 0xF, false);
    return fmax(x, __hiloint2double(ohi, olo));
}
__device__ __forceinline__ unsigned dpp_maxu(unsigned x) {
    const unsigned o = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
    return o > x ? o : x;
}
constexpr int R = 256;
// straight-line code run twice: the first pass pays the instruction fetches
__global__ void probe_ifetch(float *out, unsigned long long *cyc, float a) {
    float x0 = a + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    unsigned long long t[3];
#pragma unroll 1
    for (int rep = 0; rep < 2; rep++) {
        t[rep] = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int i = 0; i < 512; i++) {
            x0 = x0 * 1.0001f + x3;
            x1 = x1 * 0.9999f + x0;
            x2 = x2 * 1.0002f + x1;
            x3 = x3 * 0.9998f + x2;
        }
    }
    t[2] = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x0 + x1 + x2 + x3;
    if (threadIdx.x == 0) {
        cyc[9] = t[1] - t[0];
        cyc[10] = t[2] - t[1];
    }
}
__global__ void probe(double *out, unsigned long long *cyc, double a, double b, int sel) {
    const int lane = threadIdx.x;
    double x = a + lane * 1e-3, y = b;
    unsigned u = lane;
    __shared__ double sh[256];
    sh[lane] = x;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (sel) {
    case 0:  // f64 fma chain
        for (int i = 0; i < R; i++) x = fma(x, y, 1e-9);
        break;
    case 1:  // f64 mul chain
        for (int i = 0; i < R; i++) x = x * y;
        break;
    case 2:  // readlane -> fma chain
        for (int i = 0; i < R; i++) x = fma(readlane_f64(x, i & 63), y, x);
        break;
    case 3:  // f64 DPP max stage
        for (int i = 0; i < R; i++) x = dpp_max(x) * y;
        break;
    case 4:  // u32 DPP max stage
        for (int i = 0; i < R; i++) u = dpp_maxu(u) + 1;
        break;
    case 5:  // f64 division chain
        for (int i = 0; i < R; i++) x = 1.0 / x;
        break;
    case 6:  // LDS read -> use chain
        for (int i = 0; i < R; i++) x = sh[((int)x + lane) & 255] + 1.0;
        break;
    case 7:  // independent f64 fma throughput (4 chains)
    {
        double x1 = x + 1, x2 = x + 2, x3 = x + 3;
        for (int i = 0; i < R; i++) {
            x = fma(x, y, 1e-9);
            x1 = fma(x1, y, 1e-9);
            x2 = fma(x2, y, 1e-9);
            x3 = fma(x3, y, 1e-9);
        }
        x += x1 + x2 + x3;
        break;
    }
    case 8:  // ballot + ctz + readlane chain (pivot tail)
        for (int i = 0; i < R; i++) {
            const unsigned long long m = __ballot(x > y);
            const int l = __builtin_ctzll(m | (1ull << 63));
            x = readlane_f64(x, l) + x;
        }
        break;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = x + u;
    if (lane == 0) cyc[sel] = t1 - t0;
}
// one block gathers 2 x 1830 doubles (the solve's assembly pattern) from a buffer another
// kernel wrote: cycles from the first load to the last value in registers
__global__ void writer(double *buf, int n) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) buf[i] = i * 1e-3;
}
__global__ void __launch_bounds__(320) gather(const double *buf, double *out, unsigned long long *cyc, int pl) {
    const int tid = threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double a[6], b[6];
#pragma unroll
    for (int u = 0; u < 6; u++) {
        const int f = min(tid + 320 * u, pl - 1);
        a[u] = buf[f];
        b[u] = buf[pl + f];
    }
    double s = 0;
#pragma unroll
    for (int u = 0; u < 6; u++) s += a[u] * b[u];
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[tid] = s;
    if (tid == 0) cyc[11] = t1 - t0;
}
// the shader clock while one wave spins: s_memtime ticks per s_memrealtime tick (100 MHz)
__global__ void clock_probe(unsigned long long *cyc, int iters) {
    const unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    float x = threadIdx.x;
    for (int i = 0; i < iters; i++) x = x * 1.0000001f + 1e-7f;
    const unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        cyc[12] = m1 - m0;
        cyc[13] = r1 - r0;
        cyc[14] = (unsigned long long)x;
    }
}
int main() {
    double *out;
    unsigned long long *cyc, h[16];
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, 16 * sizeof(unsigned long long));
    const char *names[] = {"fma_f64 chain", "mul_f64 chain", "readlane->fma", "dpp max f64 stage (+mul)",
                           "dpp max u32 stage (+add)", "div f64", "lds read->use", "4 indep fma_f64 (per iter)",
                           "ballot/ctz/readlane"};
    for (int rep = 0; rep < 3; rep++)
        for (int s = 0; s < 9; s++) probe<<<1, 64>>>(out, cyc, 1.0000001, 0.9999999, s);
    probe_ifetch<<<1, 64>>>((float *)out, cyc, 1.0f);
    double *big, *o2;
    hipMalloc(&big, 64 << 20);
    hipMalloc(&o2, 4096);
    for (int r = 0; r < 5; r++) {
        writer<<<64, 256>>>(big, 4096);
        gather<<<1, 320>>>(big, o2, cyc, 1830);
        hipDeviceSynchronize();
        unsigned long long c;
        hipMemcpy(&c, cyc + 11, 8, hipMemcpyDeviceToHost);
        printf("gather 2x1830 doubles after a writer kernel: %llu cycles\n", c);
    }
    for (int iters : {1000, 100000, 1000000}) {
        clock_probe<<<1, 64>>>(cyc, iters);
        hipDeviceSynchronize();
        unsigned long long c[2];
        hipMemcpy(c, cyc + 12, 16, hipMemcpyDeviceToHost);
        printf("clock probe %d iters: %llu memtime ticks over %llu realtime ticks = %.3f GHz\n", iters, c[0], c[1],
               c[1] ? (double)c[0] / c[1] * 0.1 : 0.0);
    }
    for (int r = 0; r < 3; r++) {
        gather<<<1, 320>>>(big, o2, cyc, 1830);
        hipDeviceSynchronize();
        unsigned long long c;
        hipMemcpy(&c, cyc + 11, 8, hipMemcpyDeviceToHost);
        printf("gather again (no writer): %llu cycles\n", c);
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("2048 dependent-ish fma_f32 straight line: first pass %llu cycles, second pass %llu\n", h[9], h[10]);
    for (int s = 0; s < 9; s++) printf("%-30s %.1f cycles/rep\n", names[s], (double)h[s] / R);
    return 0;
}
