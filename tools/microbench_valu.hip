// microbench_valu.hip -- measured issue cost (SIMD cycles per wave64
// instruction) of the VALU instruction classes the SGM kernels use, at
// 1, 2 and 4 waves per SIMD.  Each wave runs REPS x 32 independent
// instructions of one class (8 independent registers, no dependency stalls)
// and reads s_memtime around the loop.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o build/mb && build/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define REPS 2000

#define BODY8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define BODY32(I) BODY8(I) BODY8(I) BODY8(I) BODY8(I)

template <int KIND>
__global__ void bench(unsigned* out, unsigned seed) {
    unsigned r0 = seed + threadIdx.x, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11,
             r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19, s = seed | 1;
    float f0 = r0, f1 = r1, f2 = r2, f3 = r3, f4 = r4, f5 = r5, f6 = r6, f7 = r7;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < REPS; it++) {
#define R(i) r##i
#define F(i) f##i
        if constexpr (KIND == 0) {
#define I(i) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(F(i)) : "v"(f0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 1) {
#define I(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 2) {
#define I(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 3) {
#define I(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 4) {
#define I(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 5) {
#define I(i) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 6) {
#define I(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 7) {
#define I(i) asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 8) {
#define I(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 9) {
#define I(i) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 10) {
#define I(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 11) {
#define I(i) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 12) {
#define I(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 13) {
#define I(i) asm volatile("v_min_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 14) {
#define I(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(*(double*)&R(i)) : "v"(*(double*)&r0));
            (void)s;
#undef I
        } else if constexpr (KIND == 15) {
#define I(i) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(R(i)) : "v"(r0), "v"(r1));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 16) {
#define I(i) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 17) {
#define I(i) asm volatile("v_pk_min_u16 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        }
#undef R
#undef F
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned acc = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ (unsigned)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    if ((threadIdx.x & 63) == 0) {
        out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = (unsigned)(t1 - t0);
        out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = acc;
    }
}

static const char* NAMES[] = {"v_fma_f32", "v_add_u32", "v_pk_min_u16", "v_pk_add_u16",
                              "v_perm_b32", "v_alignbit_b32", "v_add3_u32",
                              "s_nop1+v_min_u32_dpp", "v_min_u32", "v_pk_add_f16", "v_min3_u32",
                              "v_bcnt_u32_b32", "v_xor_b32", "v_min_u16", "v_pk_fma_f32(skip)",
                              "v_sad_u8", "v_mov_b32_dpp", "v_pk_min_u16 op_sel"};

template <int K>
void run(unsigned* d, int cus) {
    for (int wps : {1, 2, 4}) {
        // one 256-thread block = 4 waves = one per SIMD; wps blocks per CU
        int blocks = cus * wps;
        hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(256), 0, 0, d, 7u);
        hipDeviceSynchronize();
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(256), 0, 0, d, 9u);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        std::vector<unsigned> h(2 * blocks * 4);
        hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
        double cyc = 0;
        for (int i = 0; i < blocks * 4; i++) cyc += h[2 * i];
        cyc /= blocks * 4;
        const double n = (double)REPS * 32;
        // per-wave cycles per instruction; SIMD cycles per instruction = that / wps
        printf("%-22s waves/SIMD=%d  wave cyc/instr=%6.2f  SIMD cyc/instr=%5.2f  kernel %.3f ms\n",
               NAMES[K], wps, cyc / n, cyc / n / wps, ms);
    }
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    unsigned* d;
    hipMalloc(&d, 1 << 24);
    int cus = p.multiProcessorCount;
    printf("device %s CUs %d\n", p.gcnArchName, cus);
    run<0>(d, cus); run<1>(d, cus); run<2>(d, cus); run<3>(d, cus); run<4>(d, cus);
    run<5>(d, cus); run<6>(d, cus); run<7>(d, cus); run<8>(d, cus); run<9>(d, cus);
    run<10>(d, cus); run<11>(d, cus); run<12>(d, cus); run<13>(d, cus); run<15>(d, cus);
    run<16>(d, cus); run<17>(d, cus);
    return 0;
}
