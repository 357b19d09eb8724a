// sparse.hip -- level-synchronous frontier expansion + tiered retrograde for
// games without a dense index (Four-To-One, Toot-and-Otto, Othello; any
// descriptor).
//
// Replaces the reference's asynchronous job loop and its tables:
//   LOOK_UP / DISTRIBUTE (src/new_process.py:102-162)  -> per tier: the tier
//       table (16-byte slots {key, score}, open addressing; children of the
//       tiers above are atomicCAS-inserted into it, which deduplicates them)
//       is streamed once by classify_kernel, which evaluates primitive() once
//       per position, writes the score in place and appends the undecided ones
//       to the tier's interior list; expand_kernel generates the interior
//       positions' children into the tables of tiers t+1..t+MAX_SKIP
//   CacheDict resolved/remote (src/cache_dict.py)      -> the same tier
//       tables: a lookup reads key and score with one 16-byte load
//   RESOLVE / _res_red (src/new_process.py:223-265)    -> retro_kernel, tiers
//       deepest first, over the interior list: regenerate children; a primitive
//       child is scored from primitive() with no memory access (a LOSS-in-0
//       child ends the search: nothing beats it); the others are looked up in
//       their tier's resolved table; u16 max over preference scores, parent
//       score (gm_common.hpp), written into the parent's slot
// Every kernel walks a dense list, so no lane idles on an empty hash slot.  The
// reference expands a position once per path that reaches it (tree search,
// SURVEY §0.2); here each distinct position is expanded once.
#include "sparse_tables.hpp"

#include <hipcub/hipcub.hpp>

namespace gm {

struct Sparse {
    std::vector<SpTier> tiers;
    unsigned long long *d_counts = nullptr;   // per-tier frontier counts (device)
    uint64_t counts_cap = 0;
    unsigned long long *d_scratch = nullptr;  // [0,S) edges, [9] interior count, [10] seen, [12] export cursor
    uint32_t *d_err = nullptr;
    int64_t t_root = 0;
    uint64_t edges = 0;
    // replay (GM_SPARSE_REPLAY, default on): a solve of the same game, parameters and
    // root as the synced solve that built these tables re-runs them with no host
    // round trip -- every table size and list length is known -- as one hipGraph
    bool plan_ok = false;
    int64_t plan_key[7] = {0, 0, 0, 0, 0, 0, 0};   // game, params[0..3], root, symmetry
    unsigned long long *d_replay = nullptr;     // replay results: counts | 16 classify counters per tier | err | root
    unsigned long long *h_replay = nullptr;     // pinned host copy
    ResRef *d_tabs = nullptr;                   // the tier tables, for the one-launch refill
    uint64_t replay_words = 0;
    hipGraphExec_t graph = nullptr;
    void *sort_tmp = nullptr;                   // radix-sort scratch of the batch path (largest tier)
    size_t sort_tmp_bytes = 0;
    gm_stats_t rec_stats{};                     // the recorded solve's counts, restored by a replay
    uint64_t rec_n_positions = 0;               // ... and its position count and per-tier counts: another
    std::vector<uint64_t> rec_tier_counts;      // engine may have solved on this context in between
};

// Abandon a capture that failed half-way: the stream must leave capture mode (the
// caller falls back to a synced solve on it) and the partial graph is dropped.
static int abort_capture(Ctx *c, int rc) {
    hipGraph_t partial = nullptr;
    (void)hipStreamEndCapture(c->stream, &partial);
    if (partial) (void)hipGraphDestroy(partial);
    (void)hipGetLastError();
    return rc;
}

// ----------------------------------------------------------------- kernels
// Also marks the parents with a LOSS-in-0 child (a move that wins at once): their
// value is final here (WIN in 1), so the retrograde pass skips their lookups.
template <class D>
__global__ __launch_bounds__(256) void expand_kernel(D d, const uint64_t *__restrict__ ikeys, uint64_t n,
                                                     Fronts<D::MAX_SKIP> next, uint8_t *__restrict__ iwon,
                                                     uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    uint64_t fresh[S];
#pragma unroll
    for (int s = 0; s < S; s++) fresh[s] = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (*(volatile uint32_t *)err & DEV_ERR_TABLE_FULL) break;   // the pass is re-run into larger tables
        const uint64_t k = ikeys[i];
        const int64_t tk = d.tier(k);
        bool won = false;
        d.visit(k, [&](uint64_t c) {
            const int64_t dt = d.tier(c) - tk;
#pragma unroll
            for (int s = 0; s < S; s++)
                if (dt == s + 1 && front_insert(next.t[s], c, err)) fresh[s]++;
            if (!won) won = d.primitive(c) == LOSS;
            return true;
        });
        iwon[i] = won ? 1 : 0;
    }
#pragma unroll
    for (int s = 0; s < S; s++) block_add(next.t[s].count, fresh[s]);
}

template <class D>
__global__ __launch_bounds__(256) void retro_kernel(D d, const uint64_t *__restrict__ ikeys,
                                                    const uint32_t *__restrict__ islot,
                                                    const uint8_t *__restrict__ iwon, uint64_t n, ResRef self,
                                                    Ress<D::MAX_SKIP> next, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (iwon[i]) {   // a LOSS-in-0 child: nothing beats it, no lookup needed
            self.s[islot[i]].score = parent_score(0xFFFFu);
            continue;
        }
        const uint64_t k = ikeys[i];
        const int64_t tk = d.tier(k);
        uint32_t best = 0;
        // children as the moves make them; only one that needs a lookup is brought to its
        // stored (canonical) form -- primitive() and tier() are symmetric (games.hpp)
        unreduced(d).visit(k, [&](uint64_t c) {
            const int p = d.primitive(c);
            uint32_t sc;
            if (p != UNDECIDED) {
                sc = score_of_primitive(p);
            } else {
                const int64_t dt = d.tier(c) - tk;
                c = d.canon(c);
                int f = -1;
#pragma unroll
                for (int s = 0; s < S; s++)
                    if (dt == s + 1) f = res_find(next.t[s], c);
                if (f < 0) { atomicOr(err, DEV_ERR_MISSING_CHILD); f = 0; }
                sc = (uint32_t)f;
            }
            best = max(best, sc);
            return best != 0xFFFFu;   // a LOSS-in-0 child: nothing can beat it
        });
        if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
        self.s[islot[i]].score = parent_score(best);
    }
}

// Small tiers (fewer than SPLIT_MAX interior positions): latency, not throughput,
// bounds a tier, and with one lane per parent a lane walks its children's inserts
// (or lookups) one after the other.  The split kernels give each parent G = 16
// lanes of one DPP row; lane j handles the parent's children j, j + G, ...  (every
// lane runs the descriptor's move generator, which is arithmetic only), so the
// memory round trips of one parent overlap.  The won flag (expand) is a ballot over
// the row, the best child score (retro) a max over the row.
constexpr uint64_t SPLIT_MAX_DEFAULT = 1ull << 16;
// GM_SPARSE_SPLIT_MAX (test aid) moves the threshold, e.g. to drive small games through the
// batch kernels below
static uint64_t split_max() {
    static const uint64_t v = getenv("GM_SPARSE_SPLIT_MAX") ? strtoull(getenv("GM_SPARSE_SPLIT_MAX"), nullptr, 10)
                                                             : SPLIT_MAX_DEFAULT;
    return v;
}
constexpr int SPLIT_G = 16;

template <class D>
__global__ __launch_bounds__(256) void expand_split_kernel(D d, const uint64_t *__restrict__ ikeys, uint64_t n,
                                                           Fronts<D::MAX_SKIP> next, uint8_t *__restrict__ iwon,
                                                           uint32_t *err) {
    constexpr int S = D::MAX_SKIP, G = SPLIT_G;
    uint64_t fresh[S];
#pragma unroll
    for (int s = 0; s < S; s++) fresh[s] = 0;
    const int sub = threadIdx.x % G, row = (threadIdx.x & 63) & ~(G - 1);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x / G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; i < n; i += stride) {
        const uint64_t k = ikeys[i];
        const int64_t tk = d.tier(k);
        bool won = false;
        auto child = [&](uint64_t c) {
            const int64_t dt = d.tier(c) - tk;
#pragma unroll
            for (int s = 0; s < S; s++)
                if (dt == s + 1 && front_insert(next.t[s], c, err)) fresh[s]++;
            if (!won) won = d.primitive(c) == LOSS;
            return true;
        };
        if constexpr (part_visit_t<D>::value) {
            const int nm = d.visit_part(k, sub, G, child);
            if (!((__ballot(nm > 0) >> row) & ((1ull << G) - 1)) && sub == 0) child(d.pass_child(k));
        } else {
            int idx = 0;
            d.visit(k, [&](uint64_t c) { return idx++ % G != sub ? true : child(c); });
        }
        const uint64_t m = (__ballot(won) >> row) & ((1ull << G) - 1);
        if (sub == 0) iwon[i] = m ? 1 : 0;
    }
#pragma unroll
    for (int s = 0; s < S; s++) block_add(next.t[s].count, fresh[s]);
}

template <class D>
__global__ __launch_bounds__(256) void retro_split_kernel(D d, const uint64_t *__restrict__ ikeys,
                                                          const uint32_t *__restrict__ islot,
                                                          const uint8_t *__restrict__ iwon, uint64_t n, ResRef self,
                                                          Ress<D::MAX_SKIP> next, uint32_t *err) {
    constexpr int S = D::MAX_SKIP, G = SPLIT_G;
    const int sub = threadIdx.x % G, row = (threadIdx.x & 63) & ~(G - 1);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x / G;
    for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G; i < n; i += stride) {
        uint32_t best = 0;
        const bool won = iwon[i];   // a LOSS-in-0 child: nothing beats it, no lookup needed
        if (won) best = 0xFFFFu;
        const uint64_t k = ikeys[i];
        const int64_t tk = d.tier(k);
        auto child = [&](uint64_t c) {
                const int p = d.primitive(c);
                uint32_t sc;
                if (p != UNDECIDED) {
                    sc = score_of_primitive(p);
                } else {
                    const int64_t dt = d.tier(c) - tk;
                    int f = -1;
#pragma unroll
                    for (int s = 0; s < S; s++)
                        if (dt == s + 1) f = res_find(next.t[s], c);
                    if (f < 0) { atomicOr(err, DEV_ERR_MISSING_CHILD); f = 0; }
                    sc = (uint32_t)f;
                }
                best = max(best, sc);
                return best != 0xFFFFu;
        };
        if constexpr (part_visit_t<D>::value) {
            // every lane of the row takes part in the ballot, won or not
            const int nm = won ? 1 : d.visit_part(k, sub, G, child);
            if (!((__ballot(nm > 0) >> row) & ((1ull << G) - 1)) && sub == 0) child(d.pass_child(k));
        } else if (!won) {
            int idx = 0;
            d.visit(k, [&](uint64_t c) { return idx++ % G != sub ? true : child(c); });
        }
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, o, G));
        if (sub == 0) {
            if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
            self.s[islot[i]].score = parent_score(best);
        }
    }
}

// GM_SPARSE_CSR=1 (round 6; games whose moves go one tier deeper): expand
// also records, per interior position in the order it walks them, the slots its undecided
// children occupy in the next tier's table (a CSR: coff / ccnt / cslot) and the best score of
// its primitive children (pbest); retro then reads those slots and makes one direct load per
// child, with no move generation, probe chain or key compare.  A lane stages its slots in LDS
// (a dynamically indexed register array would go to scratch), and a wave reserves one
// contiguous run for its 64 positions with one atomic.
template <class D>
__global__ __launch_bounds__(256) void expand_csr_kernel(D d, const uint64_t *__restrict__ ikeys, uint64_t n,
                                                         FrontRef next, uint8_t *__restrict__ iwon,
                                                         uint32_t *__restrict__ coff, uint8_t *__restrict__ ccnt,
                                                         uint16_t *__restrict__ pbest, uint32_t *__restrict__ cslot,
                                                         unsigned long long *cursor, uint32_t *err) {
    constexpr int C = D::MAXC;
    __shared__ uint32_t stage[256 * C];
    uint32_t *my = stage + threadIdx.x * C;
    const int lane = threadIdx.x & 63;
    uint64_t fresh = 0;
    // every lane of a wave runs every iteration (the wave's prefix sum below)
    for (uint64_t base = blockIdx.x * (uint64_t)blockDim.x; base < n; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = base + threadIdx.x;
        const bool live = i < n && !(*(volatile uint32_t *)err & DEV_ERR_TABLE_FULL);
        uint32_t m = 0, pb = 0;
        bool won = false;
        if (live)
            d.visit(ikeys[i], [&](uint64_t c) {
                uint32_t sl;
                if (front_insert_slot(next, c, err, &sl)) fresh++;
                const int p = d.primitive(c);
                if (p != UNDECIDED) {
                    pb = max(pb, (uint32_t)score_of_primitive(p));
                    won = won || p == LOSS;
                } else if (m < (uint32_t)C) {
                    my[m++] = sl;
                }
                return true;
            });
        uint32_t incl = m;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const uint32_t total = __shfl(incl, 63);
        uint32_t wb = 0;
        if (lane == 63 && total) wb = (uint32_t)atomicAdd(cursor, (unsigned long long)total);
        wb = __shfl(wb, 63);
        if (live) {
            const uint32_t at = wb + incl - m;
            iwon[i] = won ? 1 : 0;
            coff[i] = at;
            ccnt[i] = (uint8_t)m;
            pbest[i] = (uint16_t)pb;
            for (uint32_t j = 0; j < m; j++) cslot[at + j] = my[j];
        }
    }
    block_add(next.count, fresh);
}

template <class D>
__global__ __launch_bounds__(256) void retro_csr_kernel(const uint32_t *__restrict__ islot,
                                                        const uint8_t *__restrict__ iwon,
                                                        const uint32_t *__restrict__ coff,
                                                        const uint8_t *__restrict__ ccnt,
                                                        const uint16_t *__restrict__ pbest,
                                                        const uint32_t *__restrict__ cslot, uint64_t n, ResRef self,
                                                        ResRef next, uint32_t *err) {
    constexpr int C = D::MAXC;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t best = 0xFFFFu;
        if (!iwon[i]) {   // (a LOSS-in-0 child: nothing beats it)
            best = pbest[i];
            const uint32_t o = coff[i], m = ccnt[i];
            uint32_t sl[C];
#pragma unroll
            for (int j = 0; j < C; j++) sl[j] = (uint32_t)j < m ? cslot[o + j] : ~0u;
#pragma unroll
            for (int j = 0; j < C; j++)   // independent loads: every child's in flight at once
                if (sl[j] != ~0u) best = max(best, (uint32_t)(next.s[sl[j]].score & 0xFFFFu));
        }
        if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
        self.s[islot[i]].score = parent_score(best);
    }
}

static bool csr_enabled() {
    static const bool on = getenv("GM_SPARSE_CSR") && atoi(getenv("GM_SPARSE_CSR")) == 1;
    return on;
}

// Large tiers (round 4): the interior list sorted by the key's top BATCH_SORT_BITS bits
// (hipcub radix sort of (key, slot) pairs, a few ms per solve).  Positions that agree on
// the top cells of the T and O planes then sit together and share many children (69 % of
// the inserts are duplicates; tools/expand_dup_model.cpp), so the plain expand / retro
// kernels, walking the sorted list, meet a duplicate child while its line is still in L2
// instead of as one more random 64-B HBM access (the inserts and the lookups are the
// roofline of this engine).  Default (GM_SPARSE_BATCH 1).

constexpr int BATCH_SORT_BITS = 24;       // Toot 6x4 per solve: 8 bits 133.3 ms, 16 132.3, 24 129.5, 32 133.9, 48 137.5

// development check (GM_SPARSE_BATCH=3): the sorted list holds the same (key, slot) pairs
__global__ void batch_verify_kernel(const uint64_t *__restrict__ skeys, const uint32_t *__restrict__ sslot,
                                    uint64_t n, const RSlot *__restrict__ slots, uint64_t cap,
                                    unsigned long long *bad) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (sslot[i] >= cap || slots[sslot[i]].key != skeys[i]) atomicAdd(bad, 1ull);
}

// GM_SPARSE_BATCH: 1 (default) large tiers' interior lists sorted by the key's top bits;
// 0 unsorted (round 3); 3 as 1 with a check of every sorted pair (debug).  (2, the LDS
// batch kernels of round 4, measured slower and was removed: DESIGN.md §4.2.)
static int batch_mode() {
    static const int m = getenv("GM_SPARSE_BATCH") ? atoi(getenv("GM_SPARSE_BATCH")) : 1;
    return m;
}
static bool batch_enabled() { return batch_mode() != 0; }
static int sort_bits() {   // GM_SPARSE_SORT_BITS (development): key bits the lists are sorted by
    static const int b = getenv("GM_SPARSE_SORT_BITS") ? atoi(getenv("GM_SPARSE_SORT_BITS")) : BATCH_SORT_BITS;
    return b;
}

// expand / retro of one tier: the split kernels below SPLIT_MAX interior positions, else
// the plain kernels over the sorted interior list (or the unsorted one, GM_SPARSE_BATCH 0)
template <class D>
static void launch_expand(hipStream_t st, const D &d, const SpTier &T, const Fronts<D::MAX_SKIP> &nx, uint32_t *err,
                          unsigned long long *csr_cursor = nullptr) {
    if constexpr (D::MAX_SKIP == 1) {
        if (T.cslot && csr_cursor && T.ni >= split_max()) {
            (void)hipMemsetAsync(csr_cursor, 0, 8, st);
            hipLaunchKernelGGL(expand_csr_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, st, d,
                               T.skeys ? T.skeys : T.ikeys, T.ni, nx.t[0], T.iwon, T.coff, T.ccnt, T.pbest, T.cslot,
                               csr_cursor, err);
            return;
        }
    }
    if (T.ni < split_max())
        hipLaunchKernelGGL(expand_split_kernel<D>, dim3(grid_counted(T.ni * SPLIT_G)), dim3(256), 0, st, d, T.ikeys, T.ni,
                           nx, T.iwon, err);
    else
        hipLaunchKernelGGL(expand_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, st, d, T.skeys ? T.skeys : T.ikeys,
                           T.ni, nx, T.iwon, err);
}

template <class D>
static void launch_retro(hipStream_t st, const D &d, const SpTier &T, const ResRef &self,
                         const Ress<D::MAX_SKIP> &nx, uint32_t *err) {
    if constexpr (D::MAX_SKIP == 1) {
        if (T.cslot && T.ni >= split_max()) {
            hipLaunchKernelGGL(retro_csr_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, st,
                               T.skeys ? T.sslot : T.islot, T.iwon, T.coff, T.ccnt, T.pbest, T.cslot, T.ni, self,
                               nx.t[0], err);
            return;
        }
    }
    if (T.ni < split_max())
        hipLaunchKernelGGL(retro_split_kernel<D>, dim3(grid_for(T.ni * SPLIT_G)), dim3(256), 0, st, d, T.ikeys,
                           T.islot, T.iwon, T.ni, self, nx, err);
    else
        hipLaunchKernelGGL(retro_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, st, d, T.skeys ? T.skeys : T.ikeys,
                           T.skeys ? T.sslot : T.islot, T.iwon, T.ni, self, nx, err);
}

// ----------------------------------------------------------------- host side
// bits of the descriptor keys (the batch path sorts the interior list by the top ones)
static int key_bits(const Ctx *c) {
    switch (c->game) {
    case GM_GAME_TOOT: return 2 * c->toot.A + 16;
    case GM_GAME_OTHELLO: return 2 * c->oth.A + 16;
    case GM_GAME_TTT: return 15;
    case GM_GAME_SUBTRACT: return 4 * c->sub.heaps;
    }
    return 64;
}

// GM_SPARSE_HOME_W = w > 0 (development): the tier tables' locality home -- a key's group
// is its top sort_bits() bits (the bits the interior lists are sorted by), each group's keys
// hashed into 2^w slots from a hashed base (sparse_tables.hpp home_slot); 0 = hash of the key
static uint32_t home_loc(const Ctx *c) {
    static const int w = getenv("GM_SPARSE_HOME_W") ? atoi(getenv("GM_SPARSE_HOME_W")) : 0;
    if (w <= 0 || w > 30) return 0;
    const int kb = std::min(key_bits(c), 63), b0 = std::max(0, kb - sort_bits());
    return (uint32_t)b0 | (uint32_t)w << 8;
}

// Sort a large tier's interior list by the key's top BATCH_SORT_BITS bits into
// (skeys, sslot) for the batch kernels; the scratch is kept for the replay's sorts.
static int batch_sort(Ctx *c, Sparse *sp, SpTier &T, bool alloc) {
    // end bit at most 63: ROCm 7's radix sort with end_bit 64 on u64 keys broke the
    // (key, value) pairing of about half the pairs (Toot 6x4, whose keys use bit 63:
    // GM_SPARSE_BATCH=3 counted 67,851 of 132,912 pairs wrong, profiles/r04d_*), so the
    // top key bit is left out of the grouping (the locality only needs the cells below it)
    const int kb = std::min(key_bits(c), 63), b0 = std::max(0, kb - sort_bits());
    size_t need = 0;
    GM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, need, T.ikeys, T.skeys, T.islot, T.sslot, (int)T.ni, b0, kb,
                                             c->stream));
    if (alloc) {
        GM_TRY(dev_alloc(c, (void **)&T.skeys, T.ni * 8));
        GM_TRY(dev_alloc(c, (void **)&T.sslot, T.ni * 4));
        if (need > sp->sort_tmp_bytes) {
            if (sp->sort_tmp) dev_free(c, sp->sort_tmp);
            GM_TRY(dev_alloc(c, &sp->sort_tmp, need));
            sp->sort_tmp_bytes = need;
        }
    }
    size_t have = sp->sort_tmp_bytes;
    if (have < need) { set_error("batch sort: scratch of %zu bytes, need %zu", have, need); return GM_E_STATE; }
    GM_HIP(hipcub::DeviceRadixSort::SortPairs(sp->sort_tmp, have, T.ikeys, T.skeys, T.islot, T.sslot, (int)T.ni, b0,
                                             kb, c->stream));
    if (batch_mode() == 3 && alloc) {
        GM_HIP(hipMemsetAsync(sp->d_scratch + 13, 0, 8, c->stream));
        hipLaunchKernelGGL(batch_verify_kernel, dim3(grid_for(T.ni)), dim3(256), 0, c->stream, T.skeys, T.sslot, T.ni,
                           T.slots, T.cap, sp->d_scratch + 13);
        unsigned long long bad = 0;
        GM_HIP(hipMemcpyAsync(&bad, sp->d_scratch + 13, 8, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        fprintf(stderr, "[gm] batch sort of tier %lld: %llu interior, %llu pairs differ, scratch %zu of %zu bytes\n",
                (long long)T.tier, (unsigned long long)T.ni, bad, need, have);
        if (bad) { set_error("batch sort of tier %lld: %llu pairs differ", (long long)T.tier, bad); return GM_E_STATE; }
    }
    return GM_OK;
}

static int ensure_counts(Sparse *sp, size_t n) {
    if (n <= sp->counts_cap) return GM_OK;
    uint64_t cap = std::max<uint64_t>(64, pow2_at_least(n));
    unsigned long long *p;
    GM_HIP(hipMalloc(&p, cap * sizeof(unsigned long long)));
    GM_HIP(hipMemset(p, 0, cap * sizeof(unsigned long long)));
    if (sp->d_counts) {
        GM_HIP(hipMemcpy(p, sp->d_counts, sp->counts_cap * sizeof(unsigned long long), hipMemcpyDeviceToDevice));
        GM_HIP(hipFree(sp->d_counts));
    }
    sp->d_counts = p;
    sp->counts_cap = cap;
    return GM_OK;
}

static FrontRef front_ref(Sparse *sp, size_t t) {
    SpTier &T = sp->tiers[t];
    return FrontRef{T.slots, T.cap, sp->d_counts + t, eff_loc(T.loc, T.cap)};
}

static ResRef res_ref(Sparse *sp, size_t t) { return res_ref_of(sp->tiers[t]); }

static int tier_grow(Ctx *c, Sparse *sp, size_t t, uint64_t cap) { return tier_grow(c, sp->tiers[t], cap, sp->d_err); }

static int read_err(Ctx *c, Sparse *sp) {
    uint32_t e;
    GM_HIP(hipMemcpyAsync(&e, sp->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    return e ? dev_error_to_gm(e) : GM_OK;
}

static bool replay_enabled() {
    const char *e = getenv("GM_SPARSE_REPLAY");
    return !e || atoi(e) != 0;
}

static void plan_key_of(const Ctx *c, uint64_t root, int64_t (&key)[7]) {
    const int64_t k[7] = {c->game, c->params[0], c->params[1], c->params[2], c->params[3], (int64_t)root,
                          c->game == GM_GAME_TOOT ? (int64_t)c->toot.sym
                          : c->game == GM_GAME_OTHELLO ? (int64_t)c->oth.sym : 0};
    std::copy(k, k + 7, key);
}

static bool plan_matches(const Ctx *c, const Sparse *sp, uint64_t root) {
    int64_t key[7];
    plan_key_of(c, root, key);
    return sp && sp->plan_ok && std::equal(key, key + 7, sp->plan_key);
}

// Re-run the previous solve's tier sequence on its own tables (see Sparse::graph):
// refill, re-insert the root, classify + expand every tier, retrograde, all
// enqueued (and captured once) with the recorded sizes; one read-back at the end
// checks every tier's insert count, positions seen and interior count against
// the record.  Any difference (or device error) drops the record: the caller
// then runs the synced solve.
template <class D>
static int replay_with(Ctx *c, const D &d, uint64_t root) {
    constexpr int S = D::MAX_SKIP;
    Sparse *sp = c->sp;
    const size_t T = sp->tiers.size(), NC = T + S + 1;
    const double t0 = now_ms();
    if (!sp->graph) {
        // one buffer for everything read back: insert counts [0, NC), classify counters
        // [NC, NC + 16 T), the device error word, the root record (kept from an
        // earlier attempt whose capture failed)
        sp->replay_words = NC + 16 * T + 2;
        if (!sp->d_replay) GM_HIP(hipMalloc(&sp->d_replay, sp->replay_words * 8));
        if (!sp->h_replay) GM_HIP(hipHostMalloc(&sp->h_replay, sp->replay_words * 8, hipHostMallocDefault));
        unsigned long long *cnt = sp->d_replay, *tscr = sp->d_replay + NC, *rootw = sp->d_replay + NC + 16 * T + 1;
        uint32_t *err = (uint32_t *)(sp->d_replay + NC + 16 * T);
        auto fref = [&](size_t u) { return FrontRef{u < T ? sp->tiers[u].slots : nullptr, u < T ? sp->tiers[u].cap : 0,
                                                    cnt + u, u < T ? eff_loc(sp->tiers[u].loc, sp->tiers[u].cap) : 0u}; };
        std::vector<ResRef> tabs(T);
        uint64_t maxcap = 1;
        for (size_t t = 0; t < T; t++) {
            tabs[t] = res_ref(sp, t);
            maxcap = std::max(maxcap, sp->tiers[t].cap);
        }
        if (!sp->d_tabs) GM_HIP(hipMalloc(&sp->d_tabs, T * sizeof(ResRef)));
        GM_HIP(hipMemcpy(sp->d_tabs, tabs.data(), T * sizeof(ResRef), hipMemcpyHostToDevice));
        hipGraph_t g;
        GM_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        if (hipMemsetAsync(sp->d_replay, 0, sp->replay_words * 8, c->stream) != hipSuccess)
            return abort_capture(c, GM_E_HIP);
        hipLaunchKernelGGL(slot_fill_many_kernel, dim3(grid_for(maxcap), (unsigned)T), dim3(256), 0, c->stream,
                           sp->d_tabs);   // refill every tier table with one launch
        hipLaunchKernelGGL(front_insert_one_kernel, dim3(1), dim3(64), 0, c->stream, fref(0), root, err);
        for (size_t t = 0; t < T; t++) {
            SpTier &Tt = sp->tiers[t];
            if (!Tt.count) continue;
            unsigned long long *scr = tscr + 16 * t;
            launch_classify<D, false>(c->stream, d, Tt.slots, Tt.cap, Tt.ikeys, Tt.islot, scr, err);
            if (!Tt.ni) continue;
            if (Tt.skeys && batch_sort(c, sp, Tt, false) != GM_OK) return abort_capture(c, GM_E_HIP);
            Fronts<S> nx;   // a tier past the last one received nothing: no table (cap 0)
            for (int s = 0; s < S; s++) nx.t[s] = fref(t + 1 + s);
            launch_expand(c->stream, d, Tt, nx, err, sp->d_scratch + 40);
        }
        for (size_t tt = T; tt-- > 0;) {
            SpTier &Tt = sp->tiers[tt];
            if (!Tt.ni) continue;
            Ress<S> nx;
            for (int s = 0; s < S; s++) {
                const size_t u = tt + 1 + s;
                nx.t[s] = u < T ? res_ref(sp, u) : ResRef{nullptr, 0};
            }
            launch_retro(c->stream, d, Tt, res_ref(sp, tt), nx, err);
        }
        hipLaunchKernelGGL(res_lookup_one_kernel, dim3(1), dim3(64), 0, c->stream, res_ref(sp, 0), d.canon(root),
                           rootw);
        if (hipMemcpyAsync(sp->h_replay, sp->d_replay, sp->replay_words * 8, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess)
            return abort_capture(c, GM_E_HIP);
        g = nullptr;
        const hipError_t e = hipStreamEndCapture(c->stream, &g);
        if (e != hipSuccess) {
            if (g) (void)hipGraphDestroy(g);
            set_error("sparse replay capture failed: %s", hipGetErrorString(e));
            return GM_E_HIP;
        }
        const hipError_t ie = hipGraphInstantiate(&sp->graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ie != hipSuccess) {
            sp->graph = nullptr;
            set_error("sparse replay instantiate failed: %s", hipGetErrorString(ie));
            return GM_E_HIP;
        }
    }
    GM_HIP(hipGraphLaunch(sp->graph, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    const unsigned long long *h = sp->h_replay, *scr = h + NC;
    const uint32_t err = (uint32_t)h[NC + 16 * T];
    const unsigned long long rootw = h[NC + 16 * T + 1];
    bool ok = !err && (rootw >> 32);
    for (size_t t = 0; t < T && ok; t++) {
        const SpTier &Tt = sp->tiers[t];
        // (the replay's classify counts no orbit members: with the same positions, the
        // record's are theirs)
        ok = h[t] == Tt.count && (!Tt.count || (scr[16 * t + 10] == Tt.count && scr[16 * t + 9] == Tt.ni));
    }
    if (!ok) {
        if (trace_on()) fprintf(stderr, "[gm] sparse replay differs from its record (err %#x): full solve\n", err);
        sp->plan_ok = false;
        return GM_E_STATE;
    }
    const double t1 = now_ms();
    c->root_record = (uint16_t)(rootw & 0xFFFF);
    c->n_positions = sp->rec_n_positions;
    c->tier_counts = sp->rec_tier_counts;
    const gm_stats_t keep = c->stats;
    c->stats = sp->rec_stats;
    c->stats.kernel_launches = keep.kernel_launches;
    c->stats.world = keep.world;
    c->stats.forward_ms = 0;
    c->stats.backward_ms = t1 - t0;
    c->stats.solve_ms = t1 - t0;
    return GM_OK;   // positions, tiers, edges, bytes: unchanged from the recorded solve
}

// GM_SPARSE_PROBE_STATS (development): per tier table, the mean number of probes a lookup
// of a stored key takes (its slot's distance from its home + 1) and the longest, on stderr
__global__ void probe_stats_kernel(const RSlot *__restrict__ s, uint64_t cap, uint32_t loc,
                                   unsigned long long *acc) {
    uint64_t sum = 0, cnt = 0, mx = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = s[i].key;
        if (k == EMPTY_KEY) continue;
        const uint64_t h = home_slot(k, cap, loc);
        const uint64_t dist = i >= h ? i - h : i + cap - h;
        sum += dist + 1;
        cnt++;
        mx = dist + 1 > mx ? dist + 1 : mx;
    }
    wave_add(acc, sum);
    wave_add(acc + 1, cnt);
    atomicMax(acc + 2, (unsigned long long)mx);
}

static int probe_stats(Ctx *c, Sparse *sp) {
    unsigned long long *acc = sp->d_scratch + 32, h[3];
    uint64_t tsum = 0, tcnt = 0;
    for (size_t t = 0; t < sp->tiers.size(); t++) {
        const SpTier &T = sp->tiers[t];
        if (!T.cap) continue;
        GM_HIP(hipMemsetAsync(acc, 0, 24, c->stream));
        hipLaunchKernelGGL(probe_stats_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.slots, T.cap,
                           eff_loc(T.loc, T.cap), acc);
        GM_HIP(hipMemcpyAsync(h, acc, 24, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        tsum += h[0];
        tcnt += h[1];
        fprintf(stderr, "[gm] probe stats tier %zu: %llu keys in %llu slots, mean probes %.3f, longest %llu\n", t,
                h[1], (unsigned long long)T.cap, h[1] ? (double)h[0] / h[1] : 0.0, h[2]);
    }
    fprintf(stderr, "[gm] probe stats all tiers: %llu keys, mean probes %.3f (loc %#x)\n", (unsigned long long)tcnt,
            tcnt ? (double)tsum / tcnt : 0.0, sp->tiers.empty() ? 0u : sp->tiers[0].loc);
    return GM_OK;
}

template <class D>
static int solve_with(Ctx *c, const D &d, uint64_t root) {
    constexpr int S = D::MAX_SKIP;
    if (replay_enabled() && plan_matches(c, c->sp, root) && replay_with(c, d, root) == GM_OK) return GM_OK;
    sparse_free(c);
    Sparse *sp = c->sp = new Sparse();
    sp->t_root = d.tier(root);
    GM_HIP(hipMalloc(&sp->d_scratch, 64 * sizeof(unsigned long long)));
    GM_HIP(hipMalloc(&sp->d_err, 4));
    GM_HIP(hipMemsetAsync(sp->d_err, 0, 4, c->stream));
    GM_TRY(ensure_counts(sp, 64));
    double t0 = now_ms();

    sp->tiers.resize(1);
    sp->tiers[0].loc = home_loc(c);
    GM_TRY(tier_alloc(c, &sp->tiers[0].slots, 1024));
    sp->tiers[0].cap = 1024;
    hipLaunchKernelGGL(front_insert_one_kernel, dim3(1), dim3(64), 0, c->stream, front_ref(sp, 0), root, sp->d_err);
    sp->tiers[0].fcount = 1;
    DedupEstimate est;

    // ---------------- forward: tier by tier
    for (size_t t = 0; t < sp->tiers.size(); t++) {
        const uint64_t n = sp->tiers[t].fcount;
        if (!n) continue;
        // 1. the tier is complete: score it in place, list its undecided positions
        GM_TRY(classify_tier_table(c, d, sp->tiers[t], sp->d_scratch, sp->d_err));
        unsigned long long sc[12];
        GM_HIP(hipMemcpyAsync(sc, sp->d_scratch, sizeof sc, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(read_err(c, sp));
        if (sc[10] != n) {
            set_error("tier %zu: found %llu positions, inserted %llu", t, sc[10], (unsigned long long)n);
            return GM_E_STATE;
        }
        sp->tiers[t].count = n;
        sp->tiers[t].count_all = sc[11];
        sp->tiers[t].ni = sc[9];
        sp->tiers[t].tier = sp->t_root + (int64_t)t;
        if (!sp->tiers[t].ni) continue;
        if (sp->tiers[t].ni >= split_max() && batch_enabled()) GM_TRY(batch_sort(c, sp, sp->tiers[t], true));
        // 2. size the tables of the tiers the children land in: load <= 0.7 for the
        //    predicted distinct children; a misprediction costs one re-run
        if (sp->tiers.size() < t + S + 1) {
            sp->tiers.resize(t + S + 1);
            for (auto &U : sp->tiers) U.loc = home_loc(c);
        }
        GM_TRY(ensure_counts(sp, sp->tiers.size()));
        uint64_t offered = 0, before = 0;
        for (int s = 0; s < S; s++) {
            const size_t u = t + 1 + s;
            sp->edges += sc[s];
            offered += sc[s];
            before += sp->tiers[u].fcount;
            const uint64_t need = table_cap_for(sp->tiers[u].fcount + est.distinct(sc[s]));
            if (sc[s] && sp->tiers[u].cap < need) GM_TRY(tier_grow(c, sp, u, need));
        }
        // GM_SPARSE_CSR: the expand records its children's slots for retro (one-step games,
        // the plain kernels; slots and offsets in 32 bits)
        if (S == 1 && csr_enabled() && sp->tiers[t].ni >= split_max() && sp->tiers[t + 1].cap < (1ull << 32) &&
            sc[0] < (1ull << 32)) {
            SpTier &Tt = sp->tiers[t];
            const uint64_t ni = Tt.ni;
            GM_TRY(dev_alloc(c, (void **)&Tt.coff, ni * 4));
            GM_TRY(dev_alloc(c, (void **)&Tt.ccnt, ni));
            GM_TRY(dev_alloc(c, (void **)&Tt.pbest, ni * 2));
            GM_TRY(dev_alloc(c, (void **)&Tt.cslot, std::max<uint64_t>(sc[0], 1) * 4));
        }
        // 3. expand the interior positions
        for (int attempt = 0;; attempt++) {
            Fronts<S> nx;
            for (int s = 0; s < S; s++) nx.t[s] = front_ref(sp, t + 1 + s);
            launch_expand(c->stream, d, sp->tiers[t], nx, sp->d_err, sp->d_scratch + 40);
            GM_HIP(hipGetLastError());
            uint32_t e;
            GM_HIP(hipMemcpyAsync(&e, sp->d_err, 4, hipMemcpyDeviceToHost, c->stream));
            GM_HIP(hipStreamSynchronize(c->stream));
            if (e != DEV_ERR_TABLE_FULL || attempt) break;
            // mispredicted: grow to the exact upper bound (every edge distinct) and re-run
            if (trace_on()) fprintf(stderr, "[gm] tier %zu: tables full at ratio %.3f, re-running\n", t, est.ratio);
            GM_HIP(hipMemsetAsync(sp->d_err, 0, 4, c->stream));
            for (int s = 0; s < S; s++) {
                const size_t u = t + 1 + s;
                const uint64_t need = table_cap_for(sp->tiers[u].fcount + sc[s]);
                if (sc[s] && sp->tiers[u].cap < need) GM_TRY(tier_grow(c, sp, u, need));
            }
            est.missed();
        }
        std::vector<unsigned long long> cnt(sp->tiers.size());
        GM_HIP(hipMemcpyAsync(cnt.data(), sp->d_counts, cnt.size() * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(read_err(c, sp));
        uint64_t after = 0;
        for (size_t u = t + 1; u < cnt.size(); u++) sp->tiers[u].fcount = cnt[u];
        for (int s = 0; s < S; s++) after += sp->tiers[t + 1 + s].fcount;
        est.observe(after - before, offered);
        if (trace_on())
            fprintf(stderr, "[gm] tier %zu: %llu positions, %llu interior, %llu edges, at %.1f ms\n", t,
                    (unsigned long long)n, (unsigned long long)sp->tiers[t].ni, (unsigned long long)sc[0],
                    now_ms() - t0);
    }
    while (!sp->tiers.empty() && !sp->tiers.back().count) sp->tiers.pop_back();
    double t1 = now_ms();

    // ---------------- backward: deepest tier first
    for (size_t tt = sp->tiers.size(); tt-- > 0;) {
        SpTier &T = sp->tiers[tt];
        if (!T.ni) continue;
        Ress<S> nx;
        for (int s = 0; s < S; s++) {
            const size_t u = tt + 1 + s;
            nx.t[s] = u < sp->tiers.size() ? res_ref(sp, u) : ResRef{nullptr, 0};
        }
        launch_retro(c->stream, d, T, res_ref(sp, tt), nx, sp->d_err);
    }
    GM_HIP(hipGetLastError());
    GM_TRY(read_err(c, sp));
    double t2 = now_ms();

    {
        uint64_t rk[1] = {root};
        uint16_t rr[1];
        GM_TRY(sparse_query(c, rk, rr, 1));
        c->root_record = rr[0];
    }
    uint64_t n = 0, tb = 0, stored = 0;
    c->tier_counts.clear();
    for (auto &T : sp->tiers) {
        stored += T.count;
        n += T.count_all;
        c->tier_counts.push_back(T.count_all);
        tb += T.cap * sizeof(RSlot) + T.ni * 13;
    }
    if (getenv("GM_SPARSE_PROBE_STATS")) GM_TRY(probe_stats(c, sp));
    c->n_positions = n;
    c->stats.n_positions = n;
    c->stats.n_stored = stored;
    c->stats.n_tiers = (int32_t)sp->tiers.size();
    c->stats.forward_ms = t1 - t0;
    c->stats.backward_ms = t2 - t1;
    c->stats.solve_ms = t2 - t0;
    c->stats.n_edges = sp->edges;
    // SURVEY §8d sparse model: 8 (parent key) + 8 d (child keys) + 8 d (dedup) + 2 (1 + d) per position
    c->stats.algo_bytes = 10 * n + 18 * sp->edges;
    c->stats.table_bytes = tb;
    // record for replay: the tables, lists and counts above belong to (game, params, root)
    plan_key_of(c, root, sp->plan_key);
    sp->rec_stats = c->stats;
    sp->rec_n_positions = c->n_positions;
    sp->rec_tier_counts = c->tier_counts;
    sp->plan_ok = true;
    return GM_OK;
}

// call f with the context's game descriptor
template <class F>
static int with_desc(Ctx *c, F &&f) {
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: return f(c->f2o);
    case GM_GAME_TTT: return f(c->ttt);
    case GM_GAME_TOOT: return f(c->toot);
    case GM_GAME_OTHELLO: return f(c->oth);
    case GM_GAME_SUBTRACT: return f(c->sub);
    }
    set_error("sparse engine: unknown game");
    return GM_E_GAME;
}

int sparse_solve(Ctx *c, uint64_t root) {
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: return solve_with(c, c->f2o, root);
    case GM_GAME_TTT: return solve_with(c, c->ttt, root);
    case GM_GAME_TOOT: return solve_with(c, c->toot, root);
    case GM_GAME_OTHELLO: return solve_with(c, c->oth, root);
    case GM_GAME_SUBTRACT: return solve_with(c, c->sub, root);
    }
    set_error("sparse engine: unknown game");
    return GM_E_GAME;
}

template <class D>
static void launch_query(Ctx *c, const D &d, Sparse *sp, ResRef *tabs, const uint64_t *dk, uint16_t *dr,
                         uint64_t n) {
    hipLaunchKernelGGL(query_kernel<D>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, d, sp->t_root,
                       tabs, (int)sp->tiers.size(), dk, dr, n);
}

int sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    Sparse *sp = c->sp;
    if (!n) return GM_OK;
    std::vector<ResRef> h(sp->tiers.size());
    for (size_t t = 0; t < h.size(); t++) h[t] = res_ref(sp, t);
    ResRef *tabs;
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&tabs, std::max<size_t>(1, h.size()) * sizeof(ResRef)));
    GM_HIP(hipMalloc(&dk, n * 8));
    GM_HIP(hipMalloc(&dr, n * 2));
    if (!h.empty()) GM_HIP(hipMemcpyAsync(tabs, h.data(), h.size() * sizeof(ResRef), hipMemcpyHostToDevice, c->stream));
    GM_HIP(hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: launch_query(c, c->f2o, sp, tabs, dk, dr, n); break;
    case GM_GAME_TTT: launch_query(c, c->ttt, sp, tabs, dk, dr, n); break;
    case GM_GAME_TOOT: launch_query(c, c->toot, sp, tabs, dk, dr, n); break;
    case GM_GAME_OTHELLO: launch_query(c, c->oth, sp, tabs, dk, dr, n); break;
    case GM_GAME_SUBTRACT: launch_query(c, c->sub, sp, tabs, dk, dr, n); break;
    }
    GM_HIP(hipMemcpyAsync(recs, dr, n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    (void)hipFree(tabs);
    return GM_OK;
}

int sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    Sparse *sp = c->sp;
    uint64_t total = 0;
    for (auto &T : sp->tiers) total += T.count_all;
    *n = total;
    if (!keys) return GM_OK;
    if (cap < total) {
        set_error("export buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)total);
        return GM_E_CAP;
    }
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, std::max<uint64_t>(1, total) * 8));
    GM_HIP(hipMalloc(&dr, std::max<uint64_t>(1, total) * 2));
    GM_HIP(hipMemsetAsync(sp->d_scratch + 12, 0, 8, c->stream));
    GM_TRY(with_desc(c, [&](const auto &d) {
        for (auto &T : sp->tiers)
            if (T.count)
                hipLaunchKernelGGL(res_gather_kernel<std::decay_t<decltype(d)>>, dim3(grid_for(T.cap)), dim3(256), 0,
                                   c->stream, d, T.slots, T.cap, dk, dr, sp->d_scratch + 12);
        return GM_OK;
    }));
    std::vector<uint64_t> hk(total);
    std::vector<uint16_t> hr(total);
    GM_HIP(hipMemcpyAsync(hk.data(), dk, total * 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipMemcpyAsync(hr.data(), dr, total * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    std::vector<uint64_t> idx(total);
    for (uint64_t i = 0; i < total; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return hk[a] < hk[b]; });
    for (uint64_t i = 0; i < total; i++) {
        keys[i] = hk[idx[i]];
        recs[i] = hr[idx[i]];
    }
    return GM_OK;
}

int sparse_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    Sparse *sp = c->sp;
    GM_HIP(hipMemsetAsync(sp->d_scratch + 12, 0, 8, c->stream));
    uint64_t total = 0;
    for (auto &T : sp->tiers) total += T.count_all;
    GM_TRY(with_desc(c, [&](const auto &d) {
        for (auto &T : sp->tiers)
            if (T.count)
                hipLaunchKernelGGL(res_digest_kernel<std::decay_t<decltype(d)>>, dim3(grid_counted(T.cap)), dim3(256), 0,
                                   c->stream, d, T.slots, T.cap, sp->d_scratch + 12);
        return GM_OK;
    }));
    unsigned long long h;
    GM_HIP(hipMemcpyAsync(&h, sp->d_scratch + 12, 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = h;
    *n = total;
    return GM_OK;
}

void sparse_free(Ctx *c) {
    Sparse *sp = c->sp;
    if (!sp) return;
    for (auto &T : sp->tiers) free_tier(c, T);
    (void)hipStreamSynchronize(c->stream);
    if (sp->graph) (void)hipGraphExecDestroy(sp->graph);
    for (void *p : {(void *)sp->d_counts, (void *)sp->d_scratch, (void *)sp->d_err, (void *)sp->d_replay,
                    (void *)sp->d_tabs})
        if (p) (void)hipFree(p);
    dev_free(c, sp->sort_tmp);
    if (sp->h_replay) (void)hipHostFree(sp->h_replay);
    delete sp;
    c->sp = nullptr;
}

}  // namespace gm
