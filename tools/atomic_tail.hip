// atomic_tail.hip -- what a per-wave counter atomic at the end of a grid-stride kernel costs
// (development aid, round 6).  The sparse kernels end with wave_add(): every wave adds its
// count to ONE counter.  Kernel: n items, each thread reads one u64 and sums it; then
//   mode 0  no counter
//   mode 1  one atomicAdd per wave (wave_add)
//   mode 2  one atomicAdd per workgroup (the waves' sums meet in LDS)
// for grids of 256-thread workgroups up to 8192 (grid_for's cap).  Times by hipEvent, best of 20.
//
//   hipcc -O3 --offload-arch=gfx950 tools/atomic_tail.hip -o /tmp/atomic_tail && /tmp/atomic_tail
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

template <int MODE>
__global__ __launch_bounds__(256) void tail_kernel(const uint64_t *__restrict__ in, uint64_t n,
                                                   unsigned long long *cnt) {
    uint64_t v = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) v += in[i] & 1ull;
    v += 1;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if constexpr (MODE == 1) {
        if ((threadIdx.x & 63) == 0) atomicAdd(cnt, (unsigned long long)v);
    } else if constexpr (MODE == 2) {
        __shared__ unsigned long long part[4];
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd(cnt, part[0] + part[1] + part[2] + part[3]);
    } else {
        if (v == 0x123456789ull) cnt[1] = v;   // keep the sum live
    }
}

template <int MODE>
static float time_it(const uint64_t *in, uint64_t n, unsigned grid, unsigned long long *cnt) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int r = 0; r < 20; r++) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(tail_kernel<MODE>, dim3(grid), dim3(256), 0, 0, in, n, cnt);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return best * 1e3f;
}

int main() {
    const uint64_t maxn = 1ull << 26;
    uint64_t *in;
    unsigned long long *cnt;
    CK(hipMalloc(&in, maxn * 8));
    CK(hipMemset(in, 0, maxn * 8));
    CK(hipMalloc(&cnt, 16));
    printf("%10s %6s %12s %12s %12s   (us, best of 20)\n", "items", "grid", "no counter", "per wave", "per group");
    for (uint64_t n : {1ull << 16, 1ull << 20, 1ull << 22, 1ull << 24, 1ull << 26}) {
        for (unsigned grid : {256u, 1024u, 2048u, 4096u, 8192u}) {
            if ((uint64_t)grid * 256 > n * 4) continue;
            const float t0 = time_it<0>(in, n, grid, cnt), t1 = time_it<1>(in, n, grid, cnt),
                        t2 = time_it<2>(in, n, grid, cnt);
            printf("%10llu %6u %12.1f %12.1f %12.1f\n", (unsigned long long)n, grid, t0, t1, t2);
        }
    }
    CK(hipFree(in));
    CK(hipFree(cnt));
    return 0;
}
