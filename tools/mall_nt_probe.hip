// mall_nt_probe.hip -- does a streamed store pollute the Infinity Cache?
//
// Re-reads a table of T MB after writing a stream of S MB (non-temporal or
// default stores) and reports the table read's time: near the cache-hit rate
// if the table stayed resident, near the HBM rate if the stream evicted it.
// Informs the banded path-kernel idea in DESIGN.md §4.3.  Standalone:
//   hipcc --offload-arch=gfx950 -O3 tools/mall_nt_probe.hip -o build/mall_nt_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void read_kernel(const v4u* __restrict__ t, size_t n, unsigned* __restrict__ sink) {
    v4u acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        acc ^= t[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;   // keep the loads
}

__global__ void write_kernel(v4u* __restrict__ x, size_t n, int nt) {
    const v4u v = {1u, 2u, 3u, (unsigned)n};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        if (nt) __builtin_nontemporal_store(v, x + i);
        else x[i] = v;
    }
}

#define CK(e)                                                                    \
    do {                                                                         \
        hipError_t r_ = (e);                                                     \
        if (r_ != hipSuccess) {                                                  \
            std::printf("HIP error %s at %d\n", hipGetErrorString(r_), __LINE__); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

int main() {
    const size_t MB = 1 << 20;
    const int tables[] = {64, 160};
    const int streams[] = {0, 64, 128, 256, 512, 1024};
    v4u *t, *x;
    unsigned* sink;
    CK(hipMalloc(&t, 2048 * MB));
    CK(hipMalloc(&x, 1024 * MB));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(t, 1, 2048 * MB));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 grid(256 * 8), block(256);
    // reference: a 2 GB table cannot be resident -> HBM read rate
    {
        const size_t n = 2048 * MB / 16;
        read_kernel<<<grid, block>>>(t, n, sink);
        CK(hipDeviceSynchronize());
        float tot = 0;
        for (int r = 0; r < 5; r++) {
            CK(hipEventRecord(e0));
            read_kernel<<<grid, block>>>(t, n, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        std::printf("{\"table_MB\": 2048, \"stream_MB\": 0, \"nt\": 0, \"read_TBps\": %.2f}\n",
                    2048.0 * MB / (tot / 5 * 1e-3) / 1e12);
    }
    // store-only rate: 256 MB and 1 GB streams, default and nt stores
    for (int S : {256, 1024})
        for (int nt = 0; nt < 2; nt++) {
            const size_t m = (size_t)S * MB / 16;
            write_kernel<<<grid, block>>>(x, m, nt);
            CK(hipDeviceSynchronize());
            float tot = 0;
            for (int r = 0; r < 10; r++) {
                CK(hipEventRecord(e0));
                write_kernel<<<grid, block>>>(x, m, nt);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                tot += ms;
            }
            std::printf("{\"store_MB\": %d, \"nt\": %d, \"store_us\": %.2f, \"store_TBps\": %.2f}\n",
                        S, nt, tot / 10 * 1e3, (double)S * MB / (tot / 10 * 1e-3) / 1e12);
        }
    for (int T : tables)
        for (int nt = 0; nt < 2; nt++)
            for (int S : streams) {
                const size_t n = (size_t)T * MB / 16, m = (size_t)S * MB / 16;
                read_kernel<<<grid, block>>>(t, n, sink);   // warm the table
                CK(hipDeviceSynchronize());
                float tot = 0;
                const int reps = 10;
                for (int r = 0; r < reps; r++) {
                    if (m) write_kernel<<<grid, block>>>(x, m, nt);
                    CK(hipEventRecord(e0));
                    read_kernel<<<grid, block>>>(t, n, sink);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    tot += ms;
                }
                const double ms = tot / reps;
                std::printf("{\"table_MB\": %d, \"stream_MB\": %d, \"nt\": %d, \"read_us\": %.2f, "
                            "\"read_TBps\": %.2f}\n",
                            T, S, nt, ms * 1e3, (double)T * MB / (ms * 1e-3) / 1e12);
            }
    return 0;
}
