// Throughput of single VALU instructions on gfx950 (8 independent chains per lane,
// 32 waves per CU): the cost model behind the SSS tile kernel's arithmetic choices.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITER 4096
template <int OP>
__global__ void k(uint32_t* out, uint32_t s) {
    uint32_t a[8];
    for (int j = 0; j < 8; j++) a[j] = threadIdx.x * 7 + j + s;
    uint64_t d[8];
    for (int j = 0; j < 8; j++) d[j] = a[j];
    double f[8];
    for (int j = 0; j < 8; j++) f[j] = a[j];
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 2) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(d[j]) : "v"(a[j]), "v"(s));
            if (OP == 3) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 4) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 6) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(f[j]) : "v"((double)s));
            if (OP == 7) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[j]) : "v"(s));
            if (OP == 8) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(d[j]) : "v"((uint64_t)s));
            if (OP == 9) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 10) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[j]) : "v"(s));
            if (OP == 11) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[j]));
            if (OP == 12) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(a[j]) : "v"(s));
            if (OP == 14) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 15) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 16) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(a[j]));
            if (OP == 17) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 18) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(s));
            if (OP == 19) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 20) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 21) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 22) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(a[(j+1)&7]));
            if (OP == 23) asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(a[j]));
            if (OP == 24) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 25) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 26) asm volatile("v_cmp_lt_u32 vcc, %0, %1" : : "v"(a[j]), "v"(s));
            if (OP == 27) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 28) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 29) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 30) asm volatile("v_min3_u32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 31) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 32) asm volatile("v_sad_u32 %0, %0, %1, %0" : "+v"(a[j]) : "v"(s));
            if (OP == 33) asm volatile("v_med3_u32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 34) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 35) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(a[j]) : "v"(s));
            if (OP == 13) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(d[j]) : "v"((uint64_t)s));
        }
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; j++) r += a[j] + (uint32_t)d[j] + (uint32_t)f[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int OP>
void run(const char* name, uint32_t* d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8 * 4, th = 256;
    k<OP><<<blocks, th>>>(d, 3);
    hipEventRecord(e0);
    k<OP><<<blocks, th>>>(d, 3);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double waveinstr = (double)blocks * th / 64 * ITER * 8;
    printf("%-22s %8.3f ms  %7.3f T wave-instr/s  (%.2f per CU-cycle @2.4GHz)\n", name, ms, waveinstr / ms / 1e9,
           waveinstr / (ms * 1e-3) / 256 / 2.4e9);
}
int main() {
    uint32_t* d; hipMalloc(&d, 256 * 8 * 4 * 256 * 4);
    run<5>("v_add_u32", d); run<0>("v_mul_lo_u32", d); run<1>("v_mul_hi_u32", d); run<2>("v_mad_u64_u32", d);
    run<3>("v_mul_u32_u24", d); run<4>("v_mul_hi_u32_u24", d); run<10>("v_mad_u32_u24", d); run<6>("v_fma_f64", d);
    run<7>("v_alignbit_b32", d); run<8>("v_lshl_add_u64", d); run<9>("v_min_u32", d); run<11>("v_cvt_f32_u32", d);
    run<12>("v_fma_f32", d); run<13>("v_pk_fma_f32", d);
    run<14>("v_and_b32", d); run<15>("v_xor_b32", d); run<16>("v_lshlrev_b32", d); run<17>("v_sub_u32", d); run<18>("v_cndmask_b32", d); run<19>("v_min_f32", d); run<20>("v_max_u32", d); run<21>("v_add_co_u32", d); run<22>("v_mov_b32", d); run<23>("v_bfe_u32", d); run<24>("v_lshl_add_u32", d); run<25>("v_add3_u32", d); run<26>("v_cmp_lt_u32", d); run<27>("v_mul_f32", d); run<28>("v_add_f32", d); run<29>("v_pk_add_u16", d); run<30>("v_min3_u32", d); run<31>("v_perm_b32", d); run<32>("v_sad_u32", d); run<33>("v_med3_u32", d); run<34>("v_pk_min_u16", d); run<35>("v_max3_f32", d);
    return 0;
}
