// sparse_tables.hpp -- per-tier tables and the kernels shared by the single-GPU
// sparse engine (sparse.hip) and its hash-sharded twin (dist_sparse.hip).
//
//   frontier table  u64 keys, open addressing on mix64, atomicCAS insert (dedup);
//   resolved table  16-byte slots {key, score}, load <= 1/2, one 16-B load a probe;
//   interior list   dense (key, resolved slot) of a tier's undecided positions.
// These replace the reference's CacheDict tables (src/cache_dict.py:7-82) and
// the per-edge LOOK_UP / primitive test of Process.lookup (src/new_process.py:102-133).
#pragma once
#include "sparse_common.hpp"

namespace gm {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

struct alignas(16) RSlot {
    uint64_t key;
    uint64_t score;   // u16 preference score in the low bits
};

struct FrontRef {
    uint64_t *keys;
    uint64_t mask;
    unsigned long long *count;
};
struct ResRef {
    RSlot *s;
    uint64_t mask;
};
template <int S>
struct Fronts {
    FrontRef t[S];
};
template <int S>
struct Ress {
    ResRef t[S];
};

struct SpTier {
    uint64_t *fkeys = nullptr;   // frontier table (transient: freed once the tier is classified)
    uint64_t fcap = 0, fcount = 0;
    RSlot *res = nullptr;        // resolved table
    uint64_t rcap = 0, count = 0;
    uint64_t *ikeys = nullptr;   // interior (undecided) positions and their resolved slots
    uint32_t *islot = nullptr;
    uint64_t ni = 0;
};


namespace {


__device__ __forceinline__ bool front_insert(const FrontRef &t, uint64_t key, uint32_t *err) {
    uint64_t h = mix64(key) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        uint64_t cur = t.keys[h];
        if (cur == key) return false;
        if (cur == EMPTY_KEY) {
            unsigned long long prev = atomicCAS((unsigned long long *)&t.keys[h], (unsigned long long)EMPTY_KEY,
                                                (unsigned long long)key);
            if (prev == EMPTY_KEY) return true;
            if (prev == key) return false;
        }
        h = (h + 1) & t.mask;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    return false;
}

// file a key that is known to be new (keys arrive deduplicated)
__device__ __forceinline__ uint32_t res_insert(const ResRef &t, uint64_t key, uint16_t score, uint32_t *err) {
    uint64_t h = mix64(key) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        unsigned long long prev = atomicCAS((unsigned long long *)&t.s[h].key, (unsigned long long)EMPTY_KEY,
                                            (unsigned long long)key);
        if (prev == EMPTY_KEY) {
            t.s[h].score = score;
            return (uint32_t)h;
        }
        h = (h + 1) & t.mask;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    return 0;
}

// score of key, or -1 when absent; each probe is one 16-byte load
__device__ __forceinline__ int res_find(const ResRef &t, uint64_t key) {
    if (!t.s) return -1;
    uint64_t h = mix64(key) & t.mask;
    for (uint64_t probe = 0; probe <= t.mask; probe++) {
        const u64x2 v = *(const u64x2 *)&t.s[h];
        if (v[0] == key) return (int)(v[1] & 0xFFFFu);
        if (v[0] == EMPTY_KEY) return -1;
        h = (h + 1) & t.mask;
    }
    return -1;
}


__global__ void res_fill_kernel(RSlot *s, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        *(u64x2 *)&s[i] = u64x2{EMPTY_KEY, 0};
}

__global__ void front_rehash_kernel(const uint64_t *__restrict__ okeys, uint64_t ocap, FrontRef dst, uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = okeys[i];
        if (k != EMPTY_KEY) front_insert(dst, k, err);
    }
}

__global__ void front_insert_one_kernel(FrontRef t, uint64_t key, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && front_insert(t, key, err)) atomicAdd(t.count, 1ull);
}

// Stream compaction of a frontier table into a dense key list.  A workgroup
// takes CROWS rows of 256 slots, ranks its valid keys through LDS and reserves
// its output range with ONE atomic (a per-wave atomic on one counter serialises
// at ~90 per microsecond and dominated this pass).
constexpr int CROWS = 16;
__global__ __launch_bounds__(256) void compact_kernel(const uint64_t *__restrict__ keys, uint64_t cap,
                                                      uint64_t *__restrict__ out, unsigned long long *cursor) {
    __shared__ uint32_t woff[CROWS * 4];
    __shared__ unsigned long long sbase;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint64_t chunk = blockIdx.x * (256ull * CROWS); chunk < cap; chunk += (uint64_t)gridDim.x * 256ull * CROWS) {
        uint64_t k[CROWS], m[CROWS];
#pragma unroll
        for (int r = 0; r < CROWS; r++) {
            const uint64_t i = chunk + 256ull * r + threadIdx.x;
            k[r] = i < cap ? keys[i] : EMPTY_KEY;
        }
#pragma unroll
        for (int r = 0; r < CROWS; r++) {
            m[r] = __ballot(k[r] != EMPTY_KEY);
            if (lane == 0) woff[r * 4 + w] = (uint32_t)__popcll(m[r]);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int j = 0; j < CROWS * 4; j++) {
                const uint32_t c = woff[j];
                woff[j] = acc;
                acc += c;
            }
            sbase = acc ? atomicAdd(cursor, (unsigned long long)acc) : 0ull;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < CROWS; r++)
            if (k[r] != EMPTY_KEY) out[sbase + woff[r * 4 + w] + __popcll(m[r] & below)] = k[r];
        __syncthreads();
    }
}

// one atomic per workgroup step: rank of this lane's item among the block's items
__device__ __forceinline__ uint64_t block_reserve(bool v, unsigned long long *cursor, uint32_t *woff,
                                                  unsigned long long *sbase) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t m = __ballot(v);
    if (lane == 0) woff[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t a = woff[0], b = woff[1], c = woff[2], d = woff[3], tot = a + b + c + d;
        woff[0] = 0; woff[1] = a; woff[2] = a + b; woff[3] = a + b + c;
        *sbase = tot ? atomicAdd(cursor, (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    const uint64_t at = *sbase + woff[w] + __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();
    return at;
}

// primitive() once per position; file it; list the undecided; count their edges per tier step
template <class D>
__global__ __launch_bounds__(256) void classify_kernel(D d, const uint64_t *__restrict__ dense, uint64_t n,
                                                       ResRef rt, uint64_t *__restrict__ ikeys,
                                                       uint32_t *__restrict__ islot, unsigned long long *icount,
                                                       unsigned long long *edges, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    __shared__ uint32_t woff[4];
    __shared__ unsigned long long sbase;
    uint64_t cnt[S];
#pragma unroll
    for (int s = 0; s < S; s++) cnt[s] = 0;
    for (uint64_t base = blockIdx.x * 256ull; base < n; base += (uint64_t)gridDim.x * 256ull) {
        const uint64_t i = base + threadIdx.x;
        bool interior = false;
        uint32_t slot = 0;
        uint64_t k = 0;
        if (i < n) {
            k = dense[i];
            const int p = d.primitive(k);
            if (p == DRAW) atomicOr(err, DEV_ERR_DRAW);
            interior = p == UNDECIDED;
            slot = res_insert(rt, k, interior ? 0 : score_of_primitive(p), err);
            if (interior) {
                const int64_t tk = d.tier(k);
                int nk = 0;
                d.visit(k, [&](uint64_t c) {
                    const int64_t dt = d.tier(c) - tk;
                    nk++;
                    if (dt < 1 || dt > S) atomicOr(err, DEV_ERR_TIER);
#pragma unroll
                    for (int s = 0; s < S; s++) cnt[s] += dt == s + 1;
                    return true;
                });
                if (!nk) atomicOr(err, DEV_ERR_NOMOVES);
            }
        }
        const uint64_t at = block_reserve(interior, icount, woff, &sbase);
        if (interior) {
            ikeys[at] = k;
            islot[at] = slot;
        }
    }
#pragma unroll
    for (int s = 0; s < S; s++) wave_add(edges + s, cnt[s]);
}

template <class D>
__global__ void query_kernel(D d, int64_t t_root, const ResRef *tabs, int ntabs, const uint64_t *__restrict__ keys,
                             uint16_t *__restrict__ out, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = keys[i];
    int64_t t = d.valid(k) ? d.tier(k) - t_root : -1;
    uint16_t r = REC_UNSOLVED;
    if (t >= 0 && t < ntabs) {
        int s = res_find(tabs[t], k);
        if (s >= 0) r = record_of_score((uint16_t)s);
    }
    out[i] = r;
}

__global__ void res_digest_kernel(const RSlot *__restrict__ s, uint64_t cap, unsigned long long *acc) {
    uint64_t sum = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const u64x2 v = *(const u64x2 *)&s[i];
        if (v[0] != EMPTY_KEY) sum += digest_term(v[0], record_of_score((uint16_t)v[1]));
    }
    wave_add(acc, sum);
}

__global__ void res_gather_kernel(const RSlot *__restrict__ s, uint64_t cap, uint64_t *okeys, uint16_t *orec,
                                  unsigned long long *cursor) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const u64x2 v = *(const u64x2 *)&s[i];
        if (v[0] == EMPTY_KEY) continue;
        unsigned long long at = atomicAdd(cursor, 1ull);
        okeys[at] = v[0];
        orec[at] = record_of_score((uint16_t)v[1]);
    }
}

}  // namespace

inline int front_alloc(Ctx *c, uint64_t **keys, uint64_t cap) {
    GM_TRY(dev_alloc(c, (void **)keys, cap * 8));
    hipLaunchKernelGGL(fill_empty_kernel, dim3(grid_for(cap)), dim3(256), 0, c->stream, *keys, cap);
    return GM_OK;
}

// grow a frontier table to `cap` slots, re-inserting what it holds
inline int front_grow(Ctx *c, SpTier &T, uint64_t cap, uint32_t *d_err) {
    uint64_t *nk;
    GM_TRY(front_alloc(c, &nk, cap));
    if (T.fcap) {
        FrontRef dst{nk, cap - 1, nullptr};
        hipLaunchKernelGGL(front_rehash_kernel, dim3(grid_for(T.fcap)), dim3(256), 0, c->stream, T.fkeys, T.fcap, dst,
                           d_err);
        dev_free(c, T.fkeys);
    }
    T.fkeys = nk;
    T.fcap = cap;
    return GM_OK;
}

inline ResRef res_ref_of(const SpTier &T) { return ResRef{T.res, T.rcap ? T.rcap - 1 : 0}; }

inline void free_tier(Ctx *c, SpTier &T) {
    for (void *p : {(void *)T.fkeys, (void *)T.res, (void *)T.ikeys, (void *)T.islot}) dev_free(c, p);
    T = SpTier{};
}

}  // namespace gm
