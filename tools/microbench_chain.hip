// microbench_chain.hip -- DEPENDENT-chain latency (cycles per instruction)
// of the cross-lane operations a path-recurrence step is built from, one
// wave alone on its SIMD (why one line per wave lost).
// Each kind runs REPS x 8 instructions, each consuming the previous one's
// result; timed by hipEvents around the one-wave launch (s_memtime as a
// cross-check).
//   hipcc --offload-arch=gfx950 -O3 -I include -I stereovisionarray_amd/csrc \
//         tools/microbench_chain.hip -o build/mbc && build/mbc
#include <hip/hip_runtime.h>

#include <cstdio>

#include "sgm_common.h"

#define REPS 200000
#define X8(I) I I I I I I I I

template <int KIND>
__global__ void chain(unsigned* out, unsigned seed) {
    unsigned v = seed + threadIdx.x, w = seed * 3 + threadIdx.x;
    unsigned A[2] = {v & 0x00ff00ffu, w & 0x00ff00ffu}, m = 0;
    unsigned c[2] = {0x00030004u, 0x00050006u};
    unsigned ow[1];
    sva::sgm::Edges e;
    unsigned s = seed;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < REPS; it++) {
        if constexpr (KIND == 0) {           // plain dependent VALU
            X8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(v) : "v"(w));)
        } else if constexpr (KIND == 1) {    // row DPP (quad_perm), s_nop 1 for the hazard
            X8(asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v));)
        } else if constexpr (KIND == 2) {    // row_bcast:15
            X8(asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(v));)
        } else if constexpr (KIND == 3) {    // wave_shr:1
            X8(asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v));)
        } else if constexpr (KIND == 4) {    // row_shr:1 (the 16-lane layout's shift)
            X8(asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v));)
        } else if constexpr (KIND == 5) {    // VALU -> SGPR -> SALU -> VALU round trip (s_mul: no SCC write,
                                             // which would clobber the loop branch)
            X8(asm volatile("v_readlane_b32 %1, %0, 63\n\ts_mul_i32 %1, %1, 3\n\tv_add_u32 %0, %1, %0" : "+v"(v), "+s"(s));)
        } else if constexpr (KIND == 6) {    // v_pk_minimum3_f16 chain
            X8(asm volatile("v_pk_minimum3_f16 %0, %0, %1, %1" : "+v"(v) : "v"(w));)
        } else if constexpr (KIND == 7) {    // the 16-lane step at DPL = 4 (D = 64)
            X8(sva::sgm::sgm_step_c<4>(c, A, m, ow, 10u, 120u, e); asm volatile("" : "+v"(A[0]), "+v"(A[1]));)
        } else if constexpr (KIND == 8) {    // v_readfirstlane round trip
            X8(asm volatile("v_readfirstlane_b32 %1, %0\n\ts_mul_i32 %1, %1, 3\n\tv_add_u32 %0, %1, %0" : "+v"(v), "+s"(s));)
        } else if constexpr (KIND == 10) {   // one-line-per-wave step at D = 64 (sgm_paths_wide.hip)
            X8({
                const unsigned X = __builtin_amdgcn_update_dpp(0x7fff, (int)v, 0x138, 0xf, 0xf, false);
                const unsigned Y = __builtin_amdgcn_update_dpp(0x7fff, (int)v, 0x130, 0xf, 0xf, false);
                unsigned t = (X < Y ? X : Y) + 10u;
                t = t < v ? t : v;
                t = t < m + 120u ? t : m + 120u;
                v = t + (w & 63u) - m;
                unsigned r = sva::row_min_u32<false>(v);
                unsigned q = __builtin_amdgcn_update_dpp((int)r, (int)r, 0x142, 0xa, 0xf, false);
                r = r < q ? r : q;
                q = __builtin_amdgcn_update_dpp((int)r, (int)r, 0x143, 0xc, 0xf, false);
                r = r < q ? r : q;
                m = (unsigned)__builtin_amdgcn_readlane((int)r, 63);
            })
        } else if constexpr (KIND == 9) {    // permlane32_swap + min (cross-half min)
            X8(asm volatile("v_mov_b32 %1, %0\n\ts_nop 1\n\tv_permlane32_swap_b32 %1, %0\n\tv_min_u32 %0, %0, %1" : "+v"(v), "+v"(w));)
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = (unsigned)(t1 - t0);
    out[1 + threadIdx.x] = v + A[0] + A[1] + m + s + w;
}

// ns per chained instruction from hipEvents around the launch (one wave),
// and the s_memtime delta per instruction as a cross-check
template <int K>
static double run(unsigned* d, double* memtime_per_op) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, d, 7u);
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(chain<K>, dim3(1), dim3(64), 0, 0, d, 7u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    unsigned t = 0;
    hipMemcpy(&t, d, 4, hipMemcpyDeviceToHost);
    *memtime_per_op = (double)t / (REPS * 8.0);
    return ms * 1e6 / (REPS * 8.0);
}

int main() {
    unsigned* d;
    hipMalloc(&d, 4096);
    const char* names[] = {"v_add_u32 chain", "quad_perm dpp min (+s_nop 1)", "row_bcast15 dpp min (+s_nop 1)",
                           "wave_shr:1 dpp mov (+s_nop 1)", "row_shr:1 dpp mov (+s_nop 1)",
                           "readlane->s_mul->v_add", "v_pk_minimum3_f16 chain",
                           "16-lane step DPL=4 (per step)", "readfirstlane->s_mul->v_add",
                           "mov+permlane32_swap+min", "one-line-per-wave step DPL=1 (per step)"};
    double mt[11];
    double r[11] = {run<0>(d, &mt[0]), run<1>(d, &mt[1]), run<2>(d, &mt[2]), run<3>(d, &mt[3]),
                    run<4>(d, &mt[4]), run<5>(d, &mt[5]), run<6>(d, &mt[6]), run<7>(d, &mt[7]),
                    run<8>(d, &mt[8]), run<9>(d, &mt[9]), run<10>(d, &mt[10])};
    for (int i = 0; i < 11; i++)
        printf("{\"kind\": \"%s\", \"ns_per_op\": %.3f, \"memtime_ticks_per_op\": %.3f}\n", names[i],
               r[i], mt[i]);
    hipFree(d);
    return 0;
}
