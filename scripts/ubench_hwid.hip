// ubench_hwid.hip -- where the waves of a 1024-thread workgroup run: HW_ID
// (SIMD, CU, SE) of every wave of a 256-workgroup launch with 128 KiB LDS per
// workgroup (the prove PRF launch's shape).  Experiment code, not shipped.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <map>
__global__ __launch_bounds__(1024) void k_id(unsigned *out) {
    __shared__ unsigned lds[32768];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const unsigned id = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        out[blockIdx.x * 16 + threadIdx.x / 64] = id ^ (lds[(threadIdx.x + 64) & 1023] & 0);
    }
}
int main() {
    unsigned *d;
    const int G = 256;
    hipMalloc(&d, G * 16 * 4);
    hipLaunchKernelGGL(k_id, dim3(G), dim3(1024), 0, 0, d);
    unsigned h[256 * 16];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int simd_is_w4 = 0, total = 0;
    std::map<unsigned, int> cus;
    for (int g = 0; g < G; ++g) {
        for (int w = 0; w < 16; ++w) {
            const unsigned id = h[g * 16 + w];
            const unsigned simd = (id >> 4) & 3, cu = (id >> 8) & 15, sh = (id >> 12) & 1, se = (id >> 13) & 7;
            if (g < 2) printf("wg %d wave %2d: wave_id %u simd %u cu %u sh %u se %u xcc-bits %08x\n", g, w, id & 15, simd, cu, sh, se, id);
            simd_is_w4 += simd == (unsigned)(w & 3);
            total++;
            if (w == 0) cus[(se << 8) | (sh << 4) | cu]++;
        }
    }
    printf("waves with simd == w %% 4: %d of %d; distinct (se,sh,cu) of wave 0 among %d WGs: %zu\n", simd_is_w4, total, G, cus.size());
    return 0;
}
