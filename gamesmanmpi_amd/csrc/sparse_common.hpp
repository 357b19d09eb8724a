// sparse_common.hpp -- small helpers of the sparse engines (sparse_tables.hpp has
// the tables themselves).
#pragma once
#include "gm_internal.hpp"

#include <algorithm>

namespace gm {

namespace {

// wave-level sum then one atomic per wave
__device__ __forceinline__ void wave_add(unsigned long long *dst, uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

// The count a kernel adds to one device counter at its end (a frontier count, an edge count):
// the waves' sums meet in LDS and the workgroup makes ONE atomic.  Atomics on one address
// serialise at ~12 ns each on MI355X (tools/atomic_tail.hip, profiles/r06/r06r_atomic_tail.txt):
// one per wave of an 8,192-workgroup grid adds ~0.39 ms to a launch, one per workgroup of a
// 2,048-workgroup grid (grid_counted) ~0.03 ms.  Every thread of the workgroup (at most 1,024)
// must call it, equally often.
__device__ __forceinline__ void block_add(unsigned long long *dst, uint64_t v) {
    __shared__ unsigned long long part[16];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    __syncthreads();   // the previous call's reads of part are done
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (unsigned w = 0; w < (blockDim.x + 63) / 64; w++) s += part[w];
        if (s) atomicAdd(dst, s);
    }
}

__global__ void fill_empty_kernel(uint64_t *keys, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        keys[i] = EMPTY_KEY;
}

}  // namespace

inline unsigned grid_for(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, 8192));
}

// grid of a streaming 256-thread kernel that ends in block_add (classify, digest, bucket): at
// most 2,048 workgroups (eight per CU on the 256 CUs, one generation), so its counter sees
// <= 2,048 atomics.  The random-access insert kernels keep grid_for's 8,192: their workgroups
// finish unevenly and later generations fill the gaps (Toot 6x4 expand with 2,048: +23 %).
inline unsigned grid_counted(uint64_t n) { return std::min(grid_for(n), 2048u); }

inline uint64_t pow2_at_least(uint64_t n) {
    uint64_t c = 1024;
    while (c < n) c <<= 1;
    return c;
}

// Owner rank of a key in the hash-sharded engines: the high half of mix64, so it is
// independent of the slot index (low bits).  Mirrors GameState.get_hash
// (src/game_state.py:23-31): any function of the key works, only balance matters.
GM_HD uint32_t owner_rank(uint64_t key, uint32_t G) { return (uint32_t)((mix64(key) >> 32) % G); }
GM_HD uint32_t owner_rank(const K128 &key, uint32_t G) { return (uint32_t)((mix_key(key) >> 32) % G); }

}  // namespace gm
