// sparse_common.hpp -- open-addressing tier tables shared by the single-GPU and
// sharded sparse engines (the HBM replacement of CacheDict, src/cache_dict.py).
#pragma once
#include "gm_internal.hpp"

#include <algorithm>

namespace gm {

struct Table {
    uint64_t *keys = nullptr;
    uint16_t *score = nullptr;
    uint64_t cap = 0;      // power of two (0 = not allocated)
    uint64_t count = 0;    // distinct keys held (host mirror)
};

struct TableRef {
    uint64_t *keys;
    uint16_t *score;
    uint64_t mask;
    unsigned long long *count;
};

namespace {

__device__ __forceinline__ bool table_insert(const TableRef &t, uint64_t key, uint32_t *err) {
    uint64_t h = mix64(key) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        uint64_t cur = t.keys[h];
        if (cur == key) return false;
        if (cur == EMPTY_KEY) {
            unsigned long long prev = atomicCAS((unsigned long long *)&t.keys[h],
                                                (unsigned long long)EMPTY_KEY, (unsigned long long)key);
            if (prev == EMPTY_KEY) return true;
            if (prev == key) return false;
        }
        h = (h + 1) & t.mask;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    return false;
}

__device__ __forceinline__ int64_t table_find(const TableRef &t, uint64_t key) {
    if (!t.keys) return -1;
    uint64_t h = mix64(key) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        uint64_t cur = t.keys[h];
        if (cur == key) return (int64_t)h;
        if (cur == EMPTY_KEY) return -1;
        h = (h + 1) & t.mask;
    }
    return -1;
}

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

__global__ void rehash_kernel(const uint64_t *__restrict__ okeys, const uint16_t *__restrict__ oscore,
                              uint64_t ocap, TableRef dst, uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = okeys[i];
        if (k == EMPTY_KEY) continue;
        uint64_t h = mix64(k) & dst.mask;
        bool placed = false;
        for (uint64_t probe = 0; probe <= dst.mask; probe++) {
            unsigned long long prev = atomicCAS((unsigned long long *)&dst.keys[h],
                                                (unsigned long long)EMPTY_KEY, (unsigned long long)k);
            if (prev == EMPTY_KEY) { dst.score[h] = oscore[i]; placed = true; break; }
            h = (h + 1) & dst.mask;
        }
        if (!placed) atomicOr(err, DEV_ERR_TABLE_FULL);
    }
}

__global__ void digest_kernel(const uint64_t *__restrict__ keys, const uint16_t *__restrict__ score,
                              uint64_t cap, unsigned long long *acc) {
    uint64_t sum = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k != EMPTY_KEY) sum += digest_term(k, record_of_score(score[i]));
    }
    wave_add(acc, sum);
}

__global__ void gather_kernel(const uint64_t *__restrict__ keys, const uint16_t *__restrict__ score,
                              uint64_t cap, uint64_t *okeys, uint16_t *orec, unsigned long long *cursor) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k == EMPTY_KEY) continue;
        unsigned long long at = atomicAdd(cursor, 1ull);
        okeys[at] = k;
        orec[at] = record_of_score(score[i]);
    }
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

// Allocate an empty table of `cap` slots.
inline int alloc_table(hipStream_t s, Table &T, uint64_t cap) {
    T.cap = cap;
    if (hipMalloc(&T.keys, cap * 8) != hipSuccess || hipMalloc(&T.score, cap * 2) != hipSuccess) {
        set_error("out of device memory for a %llu-slot tier table", (unsigned long long)cap);
        return GM_E_NOMEM;
    }
    hipLaunchKernelGGL(fill_empty_kernel, dim3(grid_for(cap)), dim3(256), 0, s, T.keys, cap);
    GM_HIP(hipMemsetAsync(T.score, 0, cap * 2, s));
    return GM_OK;
}

// Re-home a table into `cap` slots (grow, or shrink to load <= 1/2).
inline int resize_table(hipStream_t s, Table &T, uint64_t cap, uint32_t *d_err) {
    Table N;
    GM_TRY(alloc_table(s, N, cap));
    if (T.cap) {
        TableRef dst{N.keys, N.score, cap - 1, nullptr};
        hipLaunchKernelGGL(rehash_kernel, dim3(grid_for(T.cap)), dim3(256), 0, s, T.keys, T.score, T.cap, dst,
                           d_err);
        GM_HIP(hipStreamSynchronize(s));
        (void)hipFree(T.keys);
        (void)hipFree(T.score);
    }
    N.count = T.count;
    T = N;
    return GM_OK;
}

inline void free_table(Table &T) {
    if (T.keys) (void)hipFree(T.keys);
    if (T.score) (void)hipFree(T.score);
    T = Table{};
}

// Owner rank of a key in the hash-sharded engines: the high half of mix64, so it is
// independent of the slot index (low bits).  Mirrors GameState.get_hash
// (src/game_state.py:23-31): any function of the key works, only balance matters.
GM_HD uint32_t owner_rank(uint64_t key, uint32_t G) { return (uint32_t)((mix64(key) >> 32) % G); }

}  // namespace gm
