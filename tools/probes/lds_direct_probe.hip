// Checks where buffer_load_dwordx4 ... lds (gfx950) puts each lane's 16 bytes: lane l loads
// source dwords 4 (63 - l) .. +3; prints the LDS slot layout.  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float *src, float *out, int n) {
    __shared__ __attribute__((aligned(16))) float box[64 * 4 * 2];
    const int lane = threadIdx.x & 63;
    for (int i = lane; i < 512; i += 64) box[i] = -1.f;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(src), (short)0, n * 4, 0x00020000);
    if (lane % 3 != 1)  // exec-masked lanes: their slots stay -1
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void *)(box + 256), 16,
                                                 (63 - lane) * 16, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = lane; i < 512; i += 64) out[i] = box[i];
}
int main() {
    float *s, *o, h[512];
    hipMalloc(&s, 1024 * 4);
    hipMalloc(&o, 512 * 4);
    float hs[1024];
    for (int i = 0; i < 1024; i++) hs[i] = (float)i;
    hipMemcpy(s, hs, sizeof(hs), hipMemcpyHostToDevice);
    k<<<1, 64>>>(s, o, 1024);
    hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 4; j++) {
            const float want = (l % 3 != 1) ? (float)((63 - l) * 4 + j) : -1.f;
            if (h[256 + l * 4 + j] != want) bad++;
        }
    for (int i = 0; i < 256; i++) bad += h[i] != -1.f;
    printf("lds_direct layout: %s (%d mismatches); slot 0: %g %g %g %g, slot 1: %g\n", bad ? "NOT lane-major" : "lane-major, exec-masked lanes untouched",
           bad, h[256], h[257], h[258], h[259], h[260]);
    return bad ? 1 : 0;
}
