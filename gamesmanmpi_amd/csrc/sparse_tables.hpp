// sparse_tables.hpp -- per-tier tables and the kernels shared by the single-GPU
// sparse engine (sparse.hip) and its hash-sharded twin (dist_sparse.hip).
//
//   tier table     16-byte slots {u64 key, u64 score}, linear probing from
//                  home = mixed key * cap >> 64 (any capacity, no power-of-two
//                  rounding).  Sized for load <= 0.7 from the edges into the
//                  tier times a predicted distinct fraction (sparse.hip); an
//                  insert that probes past MAX_PROBE slots flags the table full
//                  and the insert pass is re-run into a larger table (inserts are
//                  idempotent).  The tiers above atomicCAS-insert their
//                  children's keys (deduplication); classify_kernel then streams
//                  it once, scoring every position in place; retrograde lookups
//                  read key and score with one 16-byte load.
//   interior list  dense (key, slot) of the tier's undecided positions.
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

// loc: the table's home function (home_slot): 0 = a hash of the whole key; else
// gshift | wlog << 8 = the key's group (key >> gshift) picks a base slot and a hash of the
// key one of the 2^wlog slots from it (GM_SPARSE_HOME_W, sparse.hip)
struct FrontRef {           // inserting into a tier table
    RSlot *s;
    uint64_t cap;
    unsigned long long *count;
    uint32_t loc = 0;
};
struct ResRef {             // looking up in a tier table
    RSlot *s;
    uint64_t cap;
    uint32_t loc = 0;
};
// the home function a table of `cap` slots uses: a locality home only when the table
// holds at least two windows (the same rule for inserts, lookups and rehashes)
inline GM_HD uint32_t eff_loc(uint32_t loc, uint64_t cap) {
    return (loc >> 8) && cap >= (2ull << (loc >> 8)) ? loc : 0u;
}

// 128-bit keys (gm_common.hpp K128): 32-byte slots.  An insert claims a slot by atomicCAS of
// hi from EMPTY_HI to the key's hi without its publish bit, stores lo, then publishes hi
// (coherent stores, ordered by a wait: front_insert below); a probe that meets a claimed but
// unpublished slot with its own hi re-reads that slot (the claiming lane publishes in the same iteration of the probe loop, so lanes of
// one wave never wait on each other across iterations).  Lookups run after the tier is
// complete and read (hi, lo) with one 16-byte load.
struct alignas(32) WSlot {
    uint64_t hi, lo;
    uint64_t score;   // u16 preference score in the low bits
    uint64_t pad;
};
struct WFrontRef {
    WSlot *s;
    uint64_t cap;
    unsigned long long *count;
    uint32_t loc = 0;
};
struct WResRef {
    WSlot *s;
    uint64_t cap;
    uint32_t loc = 0;
};

// the table types of a key type
template <class K>
struct KT;
template <>
struct KT<uint64_t> {
    using Slot = RSlot;
    using Front = FrontRef;
    using Res = ResRef;
};
template <>
struct KT<K128> {
    using Slot = WSlot;
    using Front = WFrontRef;
    using Res = WResRef;
};

constexpr uint64_t MAX_PROBE = 2048;   // an insert probing further marks the table full
constexpr double TABLE_LOAD = 0.7;     // planned load of a tier table
template <int S>
struct Fronts {
    FrontRef t[S];
};
template <int S>
struct Ress {
    ResRef t[S];
};

template <class K>
struct SpTierT {
    typename KT<K>::Slot *slots = nullptr;
    uint64_t cap = 0;
    uint64_t fcount = 0;         // keys inserted so far (host mirror of the device counter)
    uint64_t count = 0;          // positions of the tier once classified (stored representatives)
    uint64_t count_all = 0;      // positions they stand for (orbits expanded, games.hpp NoSym)
    K *ikeys = nullptr;          // interior (undecided) positions and their slots
    uint32_t *islot = nullptr;
    uint8_t *iwon = nullptr;     // per interior position: 1 = has a LOSS-in-0 child (set by expand)
    uint64_t ni = 0;
    // single-GPU engine, large tiers: the interior list sorted by the key's top bits
    // (sparse.hip, batch kernels); expand, retro and iwon then follow this order
    K *skeys = nullptr;
    uint32_t *sslot = nullptr;
    int64_t tier = 0;            // the descriptor tier of the positions (root tier + index)
    uint32_t loc = 0;            // home function (FrontRef::loc) requested for this tier's table
    // GM_SPARSE_CSR (sparse.hip, one-step games on the plain kernels): per interior position
    // in the order expand / retro walk it, its undecided children's slots in the next tier's
    // table (cslot[coff .. coff + ccnt)) and the best score of its primitive children
    uint32_t *coff = nullptr, *cslot = nullptr;
    uint8_t *ccnt = nullptr;
    uint16_t *pbest = nullptr;
};
using SpTier = SpTierT<uint64_t>;

namespace {

// home slot: the low half of mix64 scaled to cap (the high half picks the owner
// rank in the sharded engine, so the two stay independent).  With a locality home
// (loc != 0) the keys of one group -- one value of the key's top bits, which the sorted
// interior lists walk together -- share a window of 2^wlog slots at a hashed base.
__device__ __forceinline__ uint64_t home_slot(uint64_t key, uint64_t cap, uint32_t loc) {
    const uint64_t m = mix64(key);
    if (!loc) return __umul64hi((m << 32) | (m >> 32), cap);
    const uint64_t g = mix64((key >> (loc & 63u)) ^ 0x5851F42D4C957F2Dull);
    const uint64_t h = __umul64hi(g, cap) + (m & ((1ull << (loc >> 8)) - 1ull));
    return h >= cap ? h - cap : h;
}

__device__ __forceinline__ bool front_insert(const FrontRef &t, uint64_t key, uint32_t *err) {
    uint64_t h = home_slot(key, t.cap, t.loc);
    const uint64_t lim = t.cap < MAX_PROBE ? t.cap : MAX_PROBE;
    for (uint64_t probe = 0; probe < lim; probe++) {
        const uint64_t cur = t.s[h].key;
        if (cur == key) return false;
        if (cur == EMPTY_KEY) {
            const unsigned long long prev = atomicCAS((unsigned long long *)&t.s[h].key,
                                                      (unsigned long long)EMPTY_KEY, (unsigned long long)key);
            if (prev == EMPTY_KEY) return true;
            if (prev == key) return false;
        }
        h = h + 1 == t.cap ? 0 : h + 1;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    return false;
}

// as front_insert, and the key's slot (new or found) in *slot (~0u when the table is full)
__device__ __forceinline__ bool front_insert_slot(const FrontRef &t, uint64_t key, uint32_t *err, uint32_t *slot) {
    uint64_t h = home_slot(key, t.cap, t.loc);
    const uint64_t lim = t.cap < MAX_PROBE ? t.cap : MAX_PROBE;
    for (uint64_t probe = 0; probe < lim; probe++) {
        const uint64_t cur = t.s[h].key;
        if (cur == key) { *slot = (uint32_t)h; return false; }
        if (cur == EMPTY_KEY) {
            const unsigned long long prev = atomicCAS((unsigned long long *)&t.s[h].key,
                                                      (unsigned long long)EMPTY_KEY, (unsigned long long)key);
            if (prev == EMPTY_KEY || prev == key) { *slot = (uint32_t)h; return prev == EMPTY_KEY; }
        }
        h = h + 1 == t.cap ? 0 : h + 1;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    *slot = ~0u;
    return false;
}

// score of key, or -1 when absent; each probe is one 16-byte load
__device__ __forceinline__ int res_find(const ResRef &t, uint64_t key) {
    if (!t.s) return -1;
    uint64_t h = home_slot(key, t.cap, t.loc);
    for (uint64_t probe = 0; probe < t.cap; probe++) {
        const u64x2 v = *(const u64x2 *)&t.s[h];
        if (v[0] == key) return (int)(v[1] & 0xFFFFu);
        if (v[0] == EMPTY_KEY) return -1;
        h = h + 1 == t.cap ? 0 : h + 1;
    }
    return -1;
}

__device__ __forceinline__ uint64_t home_slot(const K128 &key, uint64_t cap, uint32_t) {
    const uint64_t m = mix_key(key);
    return __umul64hi((m << 32) | (m >> 32), cap);
}

__device__ __forceinline__ bool front_insert(const WFrontRef &t, const K128 &key, uint32_t *err) {
    // No acquire / release here: on this chip an agent-scope acquire invalidates the XCD's L2
    // (buffer_inv sc1) and a release writes it back (buffer_wbl2 sc1) -- per probe, that made
    // the 8x8 forward pass ~10x slower.  Instead lo is stored with a coherent (sc1) atomic
    // store that the wave waits for before it publishes hi with another; a reader that sees
    // the published hi reads lo with a coherent load.  The first read of a slot is a plain
    // load: a stale view can only show the slot emptier than it is (EMPTY for claimed, claimed
    // for published -- the CAS, or a coherent re-read, settles it), never another key.
    const uint64_t claim = key.hi & ~K128_PUB;
    uint64_t h = home_slot(key, t.cap, t.loc);
    const uint64_t lim = t.cap < MAX_PROBE ? t.cap : MAX_PROBE;
    uint32_t spins = 0;
    bool coherent = false;   // this slot was seen claimed but unpublished: re-read it coherently
    for (uint64_t probe = 0; probe < lim;) {
        uint64_t cur = coherent ? __hip_atomic_load(&t.s[h].hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : t.s[h].hi;
        if (cur == EMPTY_HI) {
            const unsigned long long prev =
                atomicCAS((unsigned long long *)&t.s[h].hi, (unsigned long long)EMPTY_HI, (unsigned long long)claim);
            if (prev == EMPTY_HI) {
                __hip_atomic_store(&t.s[h].lo, key.lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // lo has reached the coherent level
                __hip_atomic_store(&t.s[h].hi, key.hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return true;
            }
            cur = prev;
        }
        if ((cur | K128_PUB) == key.hi) {
            if (!(cur & K128_PUB)) {   // claimed with this hi, lo not published yet: read the slot again
                if (++spins > (1u << 24)) {
                    atomicOr(err, DEV_ERR_TABLE_FULL);
                    return false;
                }
                coherent = true;
                continue;
            }
            if (__hip_atomic_load(&t.s[h].lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == key.lo) return false;
        }
        coherent = false;
        h = h + 1 == t.cap ? 0 : h + 1;
        probe++;
    }
    atomicOr(err, DEV_ERR_TABLE_FULL);
    return false;
}

__device__ __forceinline__ int res_find(const WResRef &t, const K128 &key) {
    if (!t.s) return -1;
    uint64_t h = home_slot(key, t.cap, t.loc);
    for (uint64_t probe = 0; probe < t.cap; probe++) {
        const u64x2 v = *(const u64x2 *)&t.s[h];
        if (v[0] == key.hi && v[1] == key.lo) return (int)(t.s[h].score & 0xFFFFu);
        if (v[0] == EMPTY_HI) return -1;
        h = h + 1 == t.cap ? 0 : h + 1;
    }
    return -1;
}

// slot access shared by the two slot types
__device__ __forceinline__ void slot_clear_key(uint64_t &k) { k = EMPTY_KEY; }
__device__ __forceinline__ void slot_clear_key(K128 &k) { k = K128{0, EMPTY_HI}; }
__device__ __forceinline__ uint64_t slot_key(const RSlot &s) { return s.key; }
__device__ __forceinline__ K128 slot_key(const WSlot &s) {
    const u64x2 v = *(const u64x2 *)&s;
    return K128{v[1], v[0]};
}
__device__ __forceinline__ uint64_t slot_score(const RSlot &s) { return s.score; }
__device__ __forceinline__ uint64_t slot_score(const WSlot &s) { return s.score; }
__device__ __forceinline__ void slot_set(RSlot &s, uint64_t k, uint64_t score) { *(u64x2 *)&s = u64x2{k, score}; }
__device__ __forceinline__ void slot_set(WSlot &s, const K128 &, uint64_t score) { s.score = score; }
__device__ __forceinline__ void slot_clear(RSlot &s) { *(u64x2 *)&s = u64x2{EMPTY_KEY, 0}; }
__device__ __forceinline__ void slot_clear(WSlot &s) {
    *(u64x2 *)&s = u64x2{EMPTY_HI, 0};
    *((u64x2 *)&s + 1) = u64x2{0, 0};
}

template <class Slot>
__global__ void slot_fill_kernel(Slot *s, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        slot_clear(s[i]);
}

// every table of a replay in one launch: blockIdx.y = table, x strides inside it
__global__ void slot_fill_many_kernel(const ResRef *__restrict__ t) {
    const ResRef r = t[blockIdx.y];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < r.cap; i += (uint64_t)gridDim.x * blockDim.x)
        *(u64x2 *)&r.s[i] = u64x2{EMPTY_KEY, 0};
}

template <class K>
__global__ void front_rehash_kernel(const typename KT<K>::Slot *__restrict__ old, uint64_t ocap,
                                    typename KT<K>::Front dst, uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ocap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const K k = slot_key(old[i]);
        if (!key_empty(k)) front_insert(dst, k, err);
    }
}

// the record of one key of a resolved table (0 = not found) -> *out
__global__ void res_lookup_one_kernel(ResRef t, uint64_t key, unsigned long long *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int s = res_find(t, key);
        *out = s < 0 ? 0ull : (unsigned long long)record_of_score((uint16_t)s) | (1ull << 32);
    }
}

__global__ void front_insert_one_kernel(FrontRef t, uint64_t key, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && front_insert(t, key, err)) atomicAdd(t.count, 1ull);
}
__global__ void front_insert_one_wkernel(WFrontRef t, K128 key, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && front_insert(t, key, err)) atomicAdd(t.count, 1ull);
}

// One streaming pass over a finished tier table: primitive() once per position,
// its score stored in place (whole 16-B slots, coalesced), the undecided ones
// appended to the interior list with their edge counts per tier step.  A
// workgroup takes CROWS rows of 256 slots and reserves its part of the interior
// list with ONE atomic (a per-wave atomic on one counter serialises at ~90 per
// microsecond).  seen = positions found (a check against the insert count);
// seen[1] = the positions they stand for (each representative's orbit, games.hpp).
// Tables below CLASSIFY_ROWS_MIN slots take one row per workgroup: with CROWS rows a
// small tier ran on one or two workgroups whose threads each walked 16 positions in
// turn (Othello 4x4: classify 0.1-0.4 ms per tier, most of the solve).
constexpr int CROWS = 16;
constexpr uint64_t CLASSIFY_ROWS_MIN = 1ull << 22;
template <class D, int ROWS, bool COUNT = true, bool EDGES = COUNT>
__global__ __launch_bounds__(256) void classify_kernel(D d, typename KT<key_t<D>>::Slot *__restrict__ slots, uint64_t cap,
                                                       key_t<D> *__restrict__ ikeys, uint32_t *__restrict__ islot,
                                                       unsigned long long *icount, unsigned long long *edges,
                                                       unsigned long long *seen, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    __shared__ uint32_t woff[ROWS * 4];
    __shared__ unsigned long long sbase;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1ull;
    uint64_t cnt[S];
#pragma unroll
    for (int s = 0; s < S; s++) cnt[s] = 0;
    uint64_t nseen = 0, nall = 0;
    for (uint64_t chunk = blockIdx.x * (256ull * ROWS); chunk < cap; chunk += (uint64_t)gridDim.x * 256ull * ROWS) {
        using K = key_t<D>;
        K k[ROWS];
        uint64_t m[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            const uint64_t i = chunk + 256ull * r + threadIdx.x;
            if (i < cap) k[r] = slot_key(slots[i]);
            else slot_clear_key(k[r]);
        }
#pragma unroll
        for (int r = 0; r < ROWS; r++) {
            bool interior = false;
            if (!key_empty(k[r])) {
                nseen++;
                if (COUNT) d.orbit(k[r], [&](const K &) { nall++; });   // a replay knows its orbit counts
                const uint64_t i = chunk + 256ull * r + threadIdx.x;
                const int p = d.primitive(k[r]);
                if (p == DRAW) atomicOr(err, DEV_ERR_DRAW);
                interior = p == UNDECIDED;
                if (!interior) {
                    slot_set(slots[i], k[r], (uint64_t)score_of_primitive(p));
                } else if (EDGES) {   // a replay knows its sizes, the sharded path counts bins: no edge counts
                    if constexpr (step_count_t<D>::value) {
                        int dt = 0;
                        const int nk = d.count_children(k[r], &dt);
                        if (dt < 1 || dt > S) atomicOr(err, DEV_ERR_TIER);
#pragma unroll
                        for (int s = 0; s < S; s++) cnt[s] += dt == s + 1 ? (uint64_t)nk : 0ull;
                    } else {
                        const int64_t tk = d.tier(k[r]);
                        int nk = 0;
                        unreduced(d).visit(k[r], [&](const K &c) {   // tiers only: no canonical children
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
            }
            m[r] = __ballot(interior);
            if (lane == 0) woff[r * 4 + w] = (uint32_t)__popcll(m[r]);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (int j = 0; j < ROWS * 4; j++) {
                const uint32_t c = woff[j];
                woff[j] = acc;
                acc += c;
            }
            sbase = acc ? atomicAdd(icount, (unsigned long long)acc) : 0ull;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < ROWS; r++)
            if ((m[r] >> lane) & 1ull) {
                const uint64_t at = sbase + woff[r * 4 + w] + __popcll(m[r] & below);
                ikeys[at] = k[r];
                islot[at] = (uint32_t)(chunk + 256ull * r + threadIdx.x);
            }
        __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < S; s++) block_add(edges + s, cnt[s]);
    block_add(seen, nseen);
    block_add(seen + 1, nall);
}

template <class D>
__global__ void query_kernel(D d, int64_t t_root, const typename KT<key_t<D>>::Res *tabs, int ntabs,
                             const key_t<D> *__restrict__ keys, uint16_t *__restrict__ out, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const key_t<D> k = keys[i];
    int64_t t = d.valid(k) ? d.tier(k) - t_root : -1;
    uint16_t r = REC_UNSOLVED;
    if (t >= 0 && t < ntabs) {
        int s = res_find(tabs[t], d.canon(k));
        if (s >= 0) r = record_of_score((uint16_t)s);
    }
    out[i] = r;
}

// digest and export expand every stored representative's orbit (games.hpp)
template <class D>
__global__ void res_digest_kernel(D d, const typename KT<key_t<D>>::Slot *__restrict__ s, uint64_t cap,
                                  unsigned long long *acc) {
    using K = key_t<D>;
    uint64_t sum = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const K key = slot_key(s[i]);
        if (!key_empty(key)) {
            const uint16_t rec = record_of_score((uint16_t)slot_score(s[i]));
            d.orbit(key, [&](const K &k) { sum += digest_term(k, rec); });
        }
    }
    block_add(acc, sum);
}

template <class D>
__global__ void res_gather_kernel(D d, const typename KT<key_t<D>>::Slot *__restrict__ s, uint64_t cap,
                                  key_t<D> *okeys, uint16_t *orec, unsigned long long *cursor) {
    using K = key_t<D>;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const K key = slot_key(s[i]);
        if (key_empty(key)) continue;
        const uint16_t rec = record_of_score((uint16_t)slot_score(s[i]));
        d.orbit(key, [&](const K &k) {
            const unsigned long long at = atomicAdd(cursor, 1ull);
            okeys[at] = k;
            orec[at] = rec;
        });
    }
}

}  // namespace

template <class Slot>
inline int tier_alloc(Ctx *c, Slot **slots, uint64_t cap) {
    GM_TRY(dev_alloc(c, (void **)slots, cap * sizeof(Slot)));
    hipLaunchKernelGGL(slot_fill_kernel<Slot>, dim3(grid_for(cap)), dim3(256), 0, c->stream, *slots, cap);
    return GM_OK;
}

// grow a tier table to `cap` slots, re-inserting the keys it holds
template <class K>
inline int tier_grow(Ctx *c, SpTierT<K> &T, uint64_t cap, uint32_t *d_err) {
    typename KT<K>::Slot *ns;
    GM_TRY(tier_alloc(c, &ns, cap));
    if (T.cap) {
        typename KT<K>::Front dst{ns, cap, nullptr, eff_loc(T.loc, cap)};
        hipLaunchKernelGGL(front_rehash_kernel<K>, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.slots, T.cap, dst,
                           d_err);
        dev_free(c, T.slots);
    }
    T.slots = ns;
    T.cap = cap;
    return GM_OK;
}

template <class K>
inline typename KT<K>::Res res_ref_of(const SpTierT<K> &T) {
    return typename KT<K>::Res{T.slots, T.cap, eff_loc(T.loc, T.cap)};
}

// capacity for `n` keys at the planned load (multiple of 1024)
inline uint64_t table_cap_for(uint64_t n) {
    const uint64_t c = (uint64_t)((double)n / TABLE_LOAD) + 1;
    return std::max<uint64_t>(1024, (c + 1023) & ~1023ull);
}

// Distinct fraction of a tier's incoming edges, predicted from the last insert
// pass (fresh keys / keys offered) with a margin; 1 (the exact upper bound)
// until a pass of some size has been seen.  GM_TEST_DEDUP_RATIO pins the
// ratio (tests use a tiny one to drive the full-table re-run path).
struct DedupEstimate {
    double ratio = 1.0;
    bool pinned = false;
    DedupEstimate() {
        if (const char *e = getenv("GM_TEST_DEDUP_RATIO")) {
            ratio = atof(e);
            pinned = true;
        }
    }
    void observe(uint64_t fresh, uint64_t offered) {
        if (pinned || offered < (1u << 20)) return;
        ratio = std::min(1.0, 1.25 * (double)fresh / (double)offered + 0.05);
    }
    void missed() {
        if (!pinned) ratio = 1.0;
    }
    uint64_t distinct(uint64_t offered) const { return (uint64_t)(ratio * (double)offered) + 1; }
};

// classify a finished tier table: scores in place, interior list, edge counts
// (scr[0, S) edges by step, scr[9] interior count, scr[10] positions seen)
// scr: [0, S) edges per tier step, [9] interior count, [10] positions, [11] positions with orbits
template <class D, bool COUNT = true, bool EDGES = COUNT>
inline void launch_classify(hipStream_t st, const D &d, typename KT<key_t<D>>::Slot *slots, uint64_t cap,
                            key_t<D> *ikeys, uint32_t *islot, unsigned long long *scr, uint32_t *err) {
    // a replay's classify (no edge or orbit counts) does less per row: 32 rows
    // per thread there (Toot 6x4 replay: 8.8 vs 9.5 ms; rows 8 / 4: 12.6 / 19.6 ms -- each
    // chunk's barriers and reservation atomic are paid fewer times)
    constexpr int rows = COUNT ? CROWS : 32;
    if (cap >= CLASSIFY_ROWS_MIN)
        hipLaunchKernelGGL((classify_kernel<D, rows, COUNT, EDGES>), dim3(grid_counted(cap / rows + 1)), dim3(256), 0,
                           st, d, slots, cap, ikeys, islot, scr + 9, scr, scr + 10, err);
    else
        hipLaunchKernelGGL((classify_kernel<D, 1, COUNT, EDGES>), dim3(grid_counted(cap)), dim3(256), 0, st, d, slots,
                           cap, ikeys, islot, scr + 9, scr, scr + 10, err);
}

// edges = false (the sharded path, whose bucket pass counts the children per bin): no edge counts
template <class D>
inline int classify_tier_table(Ctx *c, const D &d, SpTierT<key_t<D>> &T, unsigned long long *scr, uint32_t *d_err,
                               bool edges = true) {
    const uint64_t n = T.fcount;
    GM_TRY(dev_alloc(c, (void **)&T.ikeys, std::max<uint64_t>(n, 1) * sizeof(key_t<D>)));
    GM_TRY(dev_alloc(c, (void **)&T.islot, std::max<uint64_t>(n, 1) * 4));
    GM_TRY(dev_alloc(c, (void **)&T.iwon, std::max<uint64_t>(n, 1)));
    GM_HIP(hipMemsetAsync(scr, 0, 16 * sizeof(unsigned long long), c->stream));
    if (edges)
        launch_classify(c->stream, d, T.slots, T.cap, T.ikeys, T.islot, scr, d_err);
    else
        launch_classify<D, true, false>(c->stream, d, T.slots, T.cap, T.ikeys, T.islot, scr, d_err);
    GM_HIP(hipGetLastError());
    return GM_OK;
}

template <class K>
inline void free_tier(Ctx *c, SpTierT<K> &T) {
    for (void *p : {(void *)T.slots, (void *)T.ikeys, (void *)T.islot, (void *)T.iwon, (void *)T.skeys, (void *)T.sslot,
                    (void *)T.coff, (void *)T.cslot, (void *)T.ccnt, (void *)T.pbest})
        dev_free(c, p);
    T = SpTierT<K>{};
}

}  // namespace gm
