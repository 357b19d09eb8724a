// randbench.hip -- random 16-B probe rate vs table size (development aid).
// Decides whether partitioning hash inserts/lookups into cache-sized regions can
// pay: one 16-B load per lane at a hashed slot, over tables from 16 MiB to 8 GiB,
// and the same restricted to a window of W bytes that slides through the table
// (what a region-ordered pass would see).
//   hipcc -O3 --offload-arch=gfx950 tools/randbench.hip -o /tmp/randbench && /tmp/randbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

// n probes; probe i reads slot (window base of i) + hash(i) % wslots
__global__ void probe_kernel(const u64x2 *t, uint64_t slots, uint64_t wslots, uint64_t n, uint64_t *out) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t win = (i * (slots / wslots)) / n;   // windows in order as i advances
        const uint64_t s = win * wslots + (mix(i) & (wslots - 1));
        acc += t[s][0];
    }
    if (acc == 42) *out = acc;
}

__global__ void cas_kernel(u64x2 *t, uint64_t slots, uint64_t wslots, uint64_t n, uint64_t *out) {
    uint64_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t win = (i * (slots / wslots)) / n;
        const uint64_t s = win * wslots + (mix(i) & (wslots - 1));
        acc += atomicCAS((unsigned long long *)(t + s), 0ull, (unsigned long long)i + 1);
    }
    if (acc == 42) *out = acc;
}

int main() {
    const uint64_t maxb = 8ull << 30;
    u64x2 *t;
    uint64_t *o;
    if (hipMalloc(&t, maxb) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) { printf("alloc failed\n"); return 1; }
    (void)hipMemset(t, 0, maxb);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint64_t n = 1ull << 30;
    const uint64_t tsz[] = {16ull << 20, 64ull << 20, 128ull << 20, 256ull << 20, 1ull << 30, 8ull << 30};
    for (int kind = 0; kind < 2; kind++)
        for (uint64_t tb : tsz)
            for (uint64_t wb : {tb, (uint64_t)4 << 20, (uint64_t)32 << 20, (uint64_t)128 << 20}) {
                if (wb > tb) continue;
                if (wb != tb && tb != (8ull << 30)) continue;
                const uint64_t slots = tb / 16, ws = wb / 16;
                for (int rep = 0; rep < 2; rep++) {
                    (void)hipEventRecord(a);
                    if (kind == 0) hipLaunchKernelGGL(probe_kernel, dim3(8192), dim3(256), 0, 0, t, slots, ws, n, o);
                    else hipLaunchKernelGGL(cas_kernel, dim3(8192), dim3(256), 0, 0, t, slots, ws, n, o);
                    (void)hipEventRecord(b);
                    (void)hipEventSynchronize(b);
                    float ms;
                    (void)hipEventElapsedTime(&ms, a, b);
                    if (rep) printf("%s table %6llu MiB window %6llu MiB: %.2f G probes/s\n", kind ? "cas  " : "load ",
                                    (unsigned long long)(tb >> 20), (unsigned long long)(wb >> 20), n / ms / 1e6);
                }
            }
    return 0;
}
