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
