// Issue-rate microbenchmark of gfx950 integer multiply forms (one wave per
// SIMD and 8 waves per SIMD, 8 independent chains per lane).  Build:
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_int.hip -o /tmp/ubench_int
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_ITER 32768
template <int OP>
__global__ void k(uint32_t *out, uint32_t seed) {
    uint32_t a[8], b = seed * 2654435761u + threadIdx.x;
    uint64_t acc[8];
    for (int i = 0; i < 8; ++i) { a[i] = seed + i * 7 + threadIdx.x; acc[i] = a[i]; }
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) {  // v_mad_u64_u32
                asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a[i]), "v"(b) : "vcc");
            } else if (OP == 1) {  // v_mul_lo_u32
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 2) {  // v_mul_hi_u32
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 3) {  // v_mad_u32_u24
                asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
            } else if (OP == 4) {  // v_add_u32
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 5) {  // v_fma_f64
                double d = (double)acc[i];
                asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d) : "v"((double)b));
                acc[i] = (uint64_t)d;
            } else if (OP == 6) {  // v_mul_hi_u32_u24
                asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 7) {  // v_perm_b32
                asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(0x0c0c0401u));
            } else if (OP == 8) {  // v_bitop3_b32 (xor3)
                asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(a[i]) : "v"(b));
            } else if (OP == 9) {  // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %1, 8" : "+v"(a[i]) : "v"(b));
            } else if (OP == 10) {  // v_add3_u32
                asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b));
            } else if (OP == 11) {  // v_xor_b32
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 12) {  // v_pk_add_u16 (packed)
                asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 14) {  // v_mov_b32_sdwa, byte 1 of dst <- byte 2 of src, rest preserved
                asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
            } else if (OP == 15) {  // v_lshl_or_b32
                asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 16) {  // v_and_or_b32
                asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
            } else if (OP == 17) {  // v_bfe_u32
                asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[i]));
            } else if (OP == 13) {  // v_lshl_add_u64
                asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(acc[i]) : "v"(acc[(i + 1) & 7]));
            }
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    const char *names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_add_u32",
                           "v_fma_f64", "v_mul_hi_u32_u24", "v_perm_b32", "v_bitop3_b32", "v_alignbit_b32",
                           "v_add3_u32", "v_xor_b32", "v_pk_add_u16", "v_lshl_add_u64", "v_mov_b32_sdwa",
                           "v_lshl_or_b32", "v_and_or_b32", "v_bfe_u32"};
    uint32_t *out;
    (void)hipMalloc(&out, 256 * 1024 * 4 * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 256;
    for (int wps = 4; wps <= 4; wps *= 2) {
        for (int op = 0; op < 18; ++op) {
            dim3 g(cus * (wps > 4 ? wps / 4 : 1)), b(256 * (wps > 4 ? 4 : wps));
            for (int rep = 0; rep < 2; ++rep) {
                (void)hipEventRecord(e0);
                switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, g, b, 0, 0, out, 1); break;
                case 1: hipLaunchKernelGGL(k<1>, g, b, 0, 0, out, 1); break;
                case 2: hipLaunchKernelGGL(k<2>, g, b, 0, 0, out, 1); break;
                case 3: hipLaunchKernelGGL(k<3>, g, b, 0, 0, out, 1); break;
                case 4: hipLaunchKernelGGL(k<4>, g, b, 0, 0, out, 1); break;
                case 5: hipLaunchKernelGGL(k<5>, g, b, 0, 0, out, 1); break;
                case 6: hipLaunchKernelGGL(k<6>, g, b, 0, 0, out, 1); break;
                case 7: hipLaunchKernelGGL(k<7>, g, b, 0, 0, out, 1); break;
                case 8: hipLaunchKernelGGL(k<8>, g, b, 0, 0, out, 1); break;
                case 9: hipLaunchKernelGGL(k<9>, g, b, 0, 0, out, 1); break;
                case 10: hipLaunchKernelGGL(k<10>, g, b, 0, 0, out, 1); break;
                case 11: hipLaunchKernelGGL(k<11>, g, b, 0, 0, out, 1); break;
                case 12: hipLaunchKernelGGL(k<12>, g, b, 0, 0, out, 1); break;
                case 13: hipLaunchKernelGGL(k<13>, g, b, 0, 0, out, 1); break;
                case 14: hipLaunchKernelGGL(k<14>, g, b, 0, 0, out, 1); break;
                case 15: hipLaunchKernelGGL(k<15>, g, b, 0, 0, out, 1); break;
                case 16: hipLaunchKernelGGL(k<16>, g, b, 0, 0, out, 1); break;
                case 17: hipLaunchKernelGGL(k<17>, g, b, 0, 0, out, 1); break;
                }
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (rep == 1) {
                    double waves = (double)cus * 4 * wps;   // waves on the chip
                    double instr_per_wave = 8.0 * N_ITER;
                    // cycles per wave-instruction per SIMD at 2.4 GHz
                    double simd_cycles = ms * 1e-3 * 2.4e9 / (instr_per_wave * wps);
                    printf("%-18s waves/SIMD=%d  %.3f ms  ~%.2f SIMD-cycles per wave-instruction (at 2.4 GHz)\n",
                           names[op], wps, ms, simd_cycles);
                }
            }
        }
    }
    return 0;
}
