// microbench_valu.hip -- measured issue cost (SIMD cycles per wave64
// instruction) of the VALU instruction classes the SGM and Mode R kernels
// use, at 1, 2, 4 and 8 waves per SIMD, and the chip-wide issue rate in
// wave-instructions per second from the kernel's own hipEvent time (clock
// independent: this is the figure bench.py's VALU rooflines divide by).
// Each wave runs REPS x 32 independent instructions of one class (8
// independent registers, each written 8 instructions before it is read
// again: no dependency or DPP hazard stalls) and reads s_memtime around the
// loop.  Kinds 18 and 19 are MIXES in the static proportions of the hot code
// (tools/isa_mix.py): the wta_hv_kernel<8,3,false> body and the
// ref_plane3_kernel<20> per-plane body.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench_valu.hip -o build/mb && build/mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define REPS 8000

#define BODY8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define BODY32(I) BODY8(I) BODY8(I) BODY8(I) BODY8(I)

template <int KIND>
__global__ __launch_bounds__(256, 8) void bench(unsigned* out, unsigned seed) {
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
        } else if constexpr (KIND == 18) {
            // wta_hv_kernel<8,3,false> static mix (1,781 VALU): perm 23 %, add3 13 %,
            // pk_minimum3 9 %, pk_min 9 %, min_u32 dpp 9 %, pk_add 7 %, alignbit 4 %,
            // mov dpp 4 %, the rest single ops -- per 32 instructions:
#define PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
#define ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
#define MIN3H(i) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
#define PKMIN(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define MINDPP(i) asm volatile("v_min_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)));
#define PKADD(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define ALIGN(i) asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(R(i)) : "v"(r0));
#define MOVDPP(i) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)) : "v"(r0));
#define MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(R(i)) : "v"(r0));
#define ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define SUB(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define MIN16(i) asm volatile("v_min_u16 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define MUL24(i) asm volatile("v_mul_i32_i24 %0, 0xfffeffff, %0" : "+v"(R(i)));
#define MIN3(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
            PERM(0) ADD3(1) MIN3H(2) PKMIN(3) MINDPP(4) PKADD(5) PERM(6) ALIGN(7)
            PERM(0) ADD3(1) MIN3H(2) PKMIN(3) MINDPP(4) PKADD(5) PERM(6) MOVDPP(7)
            PERM(0) ADD3(1) MIN3H(2) PKMIN(3) MINDPP(4) MOV(5) PERM(6) ADD(7)
            PERM(0) ADD3(1) SUB(2) MIN16(3) MUL24(4) MIN3(5) PERM(6) ALIGN(7)
        } else if constexpr (KIND == 19) {
            // ref_plane3_kernel<20> per-plane body (the blocks with the
            // ds_bpermute): add dpp 15 %, cndmask 11 %, cmp_eq 9 %, sub 8 %,
            // sad_u8 8 %, add 6 %, cmp_ne 5 %, alignbyte 4 %, perm 4 %,
            // readlane 4 %, the rest single ops -- per 32 instructions:
#define ADDDPP(i) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)));
#define CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(R(i)) : "v"(r0) : "vcc");
#define CMPEQ(i) asm volatile("v_cmp_eq_u32 vcc, %0, %1" :: "v"(R(i)), "v"(r0) : "vcc");
#define CMPNE(i) asm volatile("v_cmp_ne_u32 vcc, %0, %1" :: "v"(R(i)), "v"(r0) : "vcc");
#define CMPLT(i) asm volatile("v_cmp_lt_u32 vcc, %0, %1" :: "v"(R(i)), "v"(r0) : "vcc");
#define SAD(i) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(R(i)) : "v"(r0), "v"(r1));
#define ALIGNB(i) asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(R(i)) : "v"(r0));
#define RDL(i) asm volatile("v_readlane_b32 %0, %1, 63" : "=s"(s) : "v"(R(i)));
#define AND(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define MINI(i) asm volatile("v_min_i32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define MAXI(i) asm volatile("v_max_i32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
#define SUBREV(i) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(R(i)) : "v"(r0));
            ADDDPP(0) CND(1) CMPEQ(2) SUB(3) SAD(4) ADD(5) ALIGNB(6) PERM(7)
            ADDDPP(0) CND(1) CMPEQ(2) SUB(3) SAD(4) CMPNE(5) RDL(6) SUBREV(7)
            ADDDPP(0) CND(1) CMPEQ(2) ADD(3) SAD(4) AND(5) ALIGNB(6) PERM(7)
            ADDDPP(0) ADDDPP(1) MINI(2) MAXI(3) MOV(4) ADD3(5) CMPLT(6) MIN3(7)
#undef PERM
#undef ADD3
#undef MIN3H
#undef PKMIN
#undef MINDPP
#undef PKADD
#undef ALIGN
#undef MOVDPP
#undef MOV
#undef ADD
#undef SUB
#undef MIN16
#undef MUL24
#undef MIN3
#undef ADDDPP
#undef CND
#undef CMPEQ
#undef CMPNE
#undef CMPLT
#undef SAD
#undef ALIGNB
#undef RDL
#undef AND
#undef MINI
#undef MAXI
#undef SUBREV
        } else if constexpr (KIND == 20) {
#define I(i) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(R(i)) : "v"(r0), "v"(r1));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 21) {
#define I(i) asm volatile("v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(R(i)));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 22) {
#define I(i) asm volatile("v_alignbyte_b32 %0, %0, %1, 2" : "+v"(R(i)) : "v"(r0));
            BODY32(I)
#undef I
        } else if constexpr (KIND == 23) {
#define I(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(R(i)) : "v"(r0) : "vcc");
            BODY32(I)
#undef I
        }
#undef R
#undef F
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned acc = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7 ^ s ^ (unsigned)(f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7);
    if ((threadIdx.x & 63) == 0) {
        out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = (unsigned)(t1 - t0);
        out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = acc;
    }
}

static const char* NAMES[] = {"v_fma_f32", "v_add_u32", "v_pk_min_u16", "v_pk_add_u16",
                              "v_perm_b32", "v_alignbit_b32", "v_add3_u32",
                              "s_nop1+v_min_u32_dpp", "v_min_u32", "v_pk_add_f16", "v_min3_u32",
                              "v_bcnt_u32_b32", "v_xor_b32", "v_min_u16", "v_pk_fma_f32(skip)",
                              "v_sad_u8", "v_mov_b32_dpp", "v_pk_min_u16 op_sel",
                              "MIX wta_hv<8,3>", "MIX ref_plane3<20>", "v_pk_minimum3_f16",
                              "v_add_u32_dpp", "v_alignbyte_b32", "v_cndmask_b32"};

template <int K>
void run(unsigned* d, int cus) {
    for (int wps : {1, 2, 4, 8}) {
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
        // per-wave cycles per instruction; SIMD cycles per instruction = that / wps.
        // Chip rate from the event time: every SIMD issued wps * n wave-instructions
        // (clock-independent; 1,024 SIMDs x 2.4 GHz / 2 cycles = 1.229e12/s is the
        // SIMD-32 issue peak of MI355X_MICROARCH.md)
        const double rate = (double)cus * 4 * wps * n / (ms * 1e-3);
        printf("%-22s waves/SIMD=%d  wave cyc/instr=%6.2f  SIMD cyc/instr=%5.2f  kernel %.3f ms"
               "  chip %.3e wave-instr/s (%.3f of 1.229e12)  memtime clock %.2f GHz\n",
               NAMES[K], wps, cyc / n, cyc / n / wps, ms, rate, rate / 1.2288e12,
               cyc / (ms * 1e-3) * 1e-9);
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
    run<16>(d, cus); run<17>(d, cus); run<18>(d, cus); run<19>(d, cus); run<20>(d, cus);
    run<21>(d, cus); run<22>(d, cus); run<23>(d, cus);
    return 0;
}
