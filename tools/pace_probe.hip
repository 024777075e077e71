// pace_probe.hip -- does an agent-scope atomic counter reach every XCD?
// Each of NB workgroups (one wave each, spread over the 8 XCDs) adds 1 per
// epoch and then polls (bounded) until all NB arrived; reports polls and
// give-ups for hipMalloc, fine-grained and uncached counter memory.
//   hipcc --offload-arch=gfx950 -O3 tools/pace_probe.hip -o build/pace_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void probe(unsigned* cnt, int nb, int epochs, int maxpolls, unsigned* stats) {
    unsigned giveups = 0, polls = 0;
    for (int e = 1; e <= epochs; e++) {
        if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (unsigned)(e * nb);
        int i = 0;
        for (; i < maxpolls; i++) {
            const unsigned v = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if ((int)(v - target) >= 0) break;
            __builtin_amdgcn_s_sleep(1);
        }
        polls += i;
        if (i == maxpolls) giveups++;
    }
    if (threadIdx.x == 0) {
        atomicAdd(stats + 0, polls);
        atomicAdd(stats + 1, giveups);
    }
}

int main() {
    const int nb = 2048, epochs = 20, maxpolls = 20000;
    const char* names[3] = {"hipMalloc", "fine-grained", "uncached"};
    unsigned flags[3] = {0, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    for (int m = 0; m < 3; m++) {
        unsigned* cnt = nullptr;
        unsigned* st = nullptr;
        hipError_t e = m == 0 ? hipMalloc(&cnt, 256) : hipExtMallocWithFlags((void**)&cnt, 256, flags[m]);
        if (e != hipSuccess) { printf("%s: alloc failed %s\n", names[m], hipGetErrorString(e)); continue; }
        (void)hipMalloc(&st, 8);
        (void)hipMemset(cnt, 0, 256);
        (void)hipMemset(st, 0, 8);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, 0, cnt, nb, epochs, maxpolls, st);
        (void)hipEventRecord(b, 0);
        (void)hipDeviceSynchronize();
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        unsigned h[2], c = 0;
        (void)hipMemcpy(h, st, 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&c, cnt, 4, hipMemcpyDeviceToHost);
        printf("%-13s count %u (expect %u)  polls/epoch/wave %.1f  give-ups %u  %.3f ms (%.2f us/epoch)\n",
               names[m], c, (unsigned)(nb * epochs), (double)h[0] / nb / epochs, h[1], ms,
               ms * 1e3 / epochs);
        (void)hipFree(cnt);
        (void)hipFree(st);
    }
    return 0;
}
