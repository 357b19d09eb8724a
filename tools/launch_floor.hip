// Launch floor on gfx950 (development aid): 41 dependent launches of a
// one-wave kernel captured in one hipGraph and replayed, per kernel body:
//   0 empty; 1 one 16-B load and one 16-B store per lane (sc1 store, like a box row);
//   2 the load, a dependent chain of 2,000 VALU, the store.
// Prints the replay's mean time per launch (HIP events, 200 replays).
//   hipcc -O3 --offload-arch=gfx950 tools/launch_floor.hip -o /tmp/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(64) void floor_kernel(u32x4 *buf, unsigned n) {
    if constexpr (MODE == 0) return;
    const unsigned i = (blockIdx.x * 64u + threadIdx.x) % n;
    u32x4 v = __builtin_nontemporal_load(buf + i);
    if constexpr (MODE == 2) {
#pragma unroll 1
        for (int k = 0; k < 500; k++) {
            v.x = v.x * 3u + v.y;
            v.y = v.y ^ (v.x >> 3);
            v.z = v.z + v.x;
            v.w = v.w * 5u + v.z;
        }
    }
    __builtin_amdgcn_raw_buffer_store_b128(v, __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0xFFFFFFFFu, 0x00020000),
                                          16u * ((i + 64u) % n), 0, 16);
}

template <int MODE>
static float run(hipStream_t s, u32x4 *buf, unsigned n, int grid) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int t = 0; t < 41; t++) hipLaunchKernelGGL(floor_kernel<MODE>, dim3(grid), dim3(64), 0, s, buf, n);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int r = 0; r < 20; r++) hipGraphLaunch(ge, s);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    for (int r = 0; r < 200; r++) hipGraphLaunch(ge, s);
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1000.0f / (200 * 41);
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    const unsigned n = 1u << 24;
    u32x4 *buf;
    if (hipMalloc(&buf, (size_t)n * 16) != hipSuccess) return 1;
    hipMemset(buf, 1, (size_t)n * 16);
    for (int grid : {1, 8, 256, 2048}) {
        printf("grid %5d: empty %.2f us, load+store %.2f us, load+2000 VALU+store %.2f us per launch\n", grid,
               run<0>(s, buf, n, grid), run<1>(s, buf, n, grid), run<2>(s, buf, n, grid));
    }
    hipFree(buf);
    return 0;
}
