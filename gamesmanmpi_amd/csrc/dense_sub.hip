// dense_sub.hip -- dense tiered retrograde for the synthetic subtraction game.
//
// Replaces, for config 5, the reference's per-edge job loop (Process.lookup /
// distribute / resolve, src/new_process.py:102-265) and its shelve tables
// (src/cache_dict.py): every one of the 16^heaps positions gets a 2-byte slot
// in one HBM array indexed by the key itself.
//
// Decomposition.  A key is `heaps` nibbles.  The low LOW nibbles index a
// position inside a *block* of 16^LOW slots (8 KiB at LOW = 3) that one
// workgroup solves in LDS; the high HIGH = heaps - LOW nibbles name the block.
// A move lowers exactly one nibble, so a position's children are either in its
// own block (low move) or at the same offset of a block whose high part is
// 1 or 2 smaller in one nibble (high move).  Blocks are therefore processed in
// tiers of their high-nibble sum, one launch per tier:
//
//   pass A  fold the high children: for every valid child block, stream its
//           16^LOW scores with 16-B loads and keep the running u16 max
//           (v_pk_max_u16) -- fully coalesced whole-block reads;
//   pass B  walk the block's own low tiers (low-nibble sum 0..15*LOW) in LDS:
//           each position folds its <= 2*LOW in-block children and turns the
//           best score into its own (gm_common.hpp), one barrier per low tier;
//   pass C  write the block back with 16-B stores.
//
// HBM traffic per position: 2 B written + 2 B per high child (1.8125 per high
// nibble on average); the SURVEY's algorithmic figure (31 B/position) counts
// every child edge as a 2-B read.
#include "gm_internal.hpp"

#include <algorithm>
#include <chrono>

namespace gm {

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));

struct DenseSub {
    int heaps = 0, low = 0, high = 0;
    uint16_t *table = nullptr;          // 16^heaps scores
    bool owned = false;
    uint64_t slots = 0;
    uint16_t *zero = nullptr;           // one block of zeros (padding source)
    uint32_t *d_blocks = nullptr;       // high parts sorted by (tier, value)
    std::vector<uint32_t> tier_off;     // block offsets per high tier
    uint64_t *d_acc = nullptr;          // digest / counters
    hipGraphExec_t graph = nullptr;
    hipStream_t graph_stream = nullptr;
    std::vector<hipEvent_t> ev;         // per-launch timing events
};

// ---------------------------------------------------------------------------
template <int LOW, int HIGH>
__global__ __launch_bounds__(256) void sub_tier_kernel(uint16_t *__restrict__ table,
                                                       const uint32_t *__restrict__ blocks,
                                                       uint32_t nblk,
                                                       const uint16_t *__restrict__ zero) {
    constexpr int NPOS = 1 << (4 * LOW);
    constexpr int NCH = NPOS >= 8 ? NPOS / 8 : 1;      // 16-B chunks per block
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;   // child blocks, padded
    __shared__ __attribute__((aligned(16))) uint16_t s[NPOS < 8 ? 8 : NPOS];
    const int tid = threadIdx.x;

    // XCD-aware order: blocks b and b+8 share an XCD (MI355X_MICROARCH.md
    // "Workgroup dispatch"), so give each XCD a contiguous run of the tier list;
    // neighbouring high parts share child blocks in that XCD's L2.
    const uint32_t b = blockIdx.x, q = nblk >> 3, r = nblk & 7u, x = b & 7u, i = b >> 3;
    const uint32_t logical = x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
    const uint32_t hp = blocks[logical];
    uint16_t *const out = table + ((uint64_t)hp << (4 * LOW));

    // ---- pass A: high children -------------------------------------------
    // Slot k = 2j + s is the child "take s+1 from high nibble j".  A missing
    // child (nibble too small) re-reads the first existing child block (max is
    // idempotent and the repeat is an L2 hit) or, with no child at all, the
    // zero block.  Every index is a compile-time constant after unrolling, so
    // the pointers stay in (scalar) registers.
    const uint16_t *src[NMAX];
    {
        const uint16_t *first = zero;
#pragma unroll
        for (int j = HIGH - 1; j >= 0; j--) {
            const uint32_t h = (hp >> (4 * j)) & 15u;
            if (h >= 1) first = table + ((uint64_t)(hp - (1u << (4 * j))) << (4 * LOW));
        }
#pragma unroll
        for (int j = 0; j < HIGH; j++) {
            const uint32_t h = (hp >> (4 * j)) & 15u;
            src[2 * j] = h >= 1 ? table + ((uint64_t)(hp - (1u << (4 * j))) << (4 * LOW)) : first;
            src[2 * j + 1] = h >= 2 ? table + ((uint64_t)(hp - (2u << (4 * j))) << (4 * LOW)) : first;
        }
        if constexpr (HIGH == 0) src[0] = zero;
    }
    if constexpr (NPOS >= 8) {
        for (int c = tid; c < NCH; c += 256) {
            u16x8 v[NMAX];
#pragma unroll
            for (int k = 0; k < NMAX; k++) v[k] = *(const u16x8 *)(src[k] + 8 * c);
            u16x8 acc = v[0];
#pragma unroll
            for (int k = 1; k < NMAX; k++) acc = __builtin_elementwise_max(acc, v[k]);
            *(u16x8 *)(s + 8 * c) = acc;
        }
    } else {
        if (tid < NPOS) {
            uint16_t acc = 0;
#pragma unroll
            for (int k = 0; k < NMAX; k++) acc = acc > src[k][tid] ? acc : src[k][tid];
            s[tid] = acc;
        }
    }
    __syncthreads();

    // ---- pass B: low tiers in LDS -----------------------------------------
    const int a0 = tid & 15, a1 = (tid >> 4) & 15;
    auto solve_one = [&](int L) {
        uint32_t best = s[L];
#pragma unroll
        for (int j = 0; j < LOW; j++) {
            const int h = (L >> (4 * j)) & 15;
            if (h >= 1) best = max(best, (uint32_t)s[L - (1 << (4 * j))]);
            if (h >= 2) best = max(best, (uint32_t)s[L - (2 << (4 * j))]);
        }
        s[L] = (hp == 0 && L == 0) ? (uint16_t)0xFFFF : parent_score(best);
    };
    if constexpr (LOW == 3) {
        // thread = low two nibbles; the third nibble is fixed by the tier
        const int s0 = a0 + a1;
        for (int tau = 0; tau <= 45; tau++) {
            const int c = tau - s0;
            if (c >= 0 && c <= 15) solve_one(tid + 256 * c);
            __syncthreads();
        }
    } else {
        const int L = tid;
        int sum = 0;
#pragma unroll
        for (int j = 0; j < LOW; j++) sum += (L >> (4 * j)) & 15;
        for (int tau = 0; tau <= 15 * LOW; tau++) {
            if (L < NPOS && sum == tau) solve_one(L);
            __syncthreads();
        }
    }

    // ---- pass C: write back -------------------------------------------------
    if constexpr (NPOS >= 8) {
        for (int c = tid; c < NCH; c += 256) *(u16x8 *)(out + 8 * c) = *(const u16x8 *)(s + 8 * c);
    } else {
        if (tid < NPOS) out[tid] = s[tid];
    }
}

typedef void (*tier_kernel_t)(uint16_t *, const uint32_t *, uint32_t, const uint16_t *);

template <int LOW>
static tier_kernel_t pick_high(int high) {
    switch (high) {
    case 0: return sub_tier_kernel<LOW, 0>;
    case 1: return sub_tier_kernel<LOW, 1>;
    case 2: return sub_tier_kernel<LOW, 2>;
    case 3: return sub_tier_kernel<LOW, 3>;
    case 4: return sub_tier_kernel<LOW, 4>;
    case 5: return sub_tier_kernel<LOW, 5>;
    case 6: return LOW <= 2 ? sub_tier_kernel<LOW, 6> : nullptr;
    case 7: return LOW <= 1 ? sub_tier_kernel<LOW, 7> : nullptr;
    }
    return nullptr;
}

static tier_kernel_t pick_kernel(int low, int high) {
    switch (low) {
    case 1: return pick_high<1>(high);
    case 2: return pick_high<2>(high);
    case 3: return pick_high<3>(high);
    }
    return nullptr;
}

bool sub_kernel_exists(int low, int high) { return pick_kernel(low, high) != nullptr; }

void launch_sub_tier(int low, int high, uint32_t nblocks, uint16_t *table, const uint32_t *list,
                     const uint16_t *zero, hipStream_t s) {
    if (!nblocks) return;
    hipLaunchKernelGGL(pick_kernel(low, high), dim3(nblocks), dim3(256), 0, s, table, list, nblocks, zero);
}

// ---------------------------------------------------------------------------
__global__ void sub_digest_kernel(const uint16_t *__restrict__ table, uint64_t slots, int heaps,
                                  uint64_t root, unsigned long long *acc) {
    uint64_t sum = 0, cnt = 0;
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < slots;
         k += (uint64_t)gridDim.x * blockDim.x) {
        bool in = true;
        for (int j = 0; j < heaps; j++) in &= ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
        if (!in) continue;
        sum += digest_term(k, record_of_score(table[k]));
        cnt++;
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        cnt += __shfl_xor(cnt, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(acc, (unsigned long long)sum);
        atomicAdd(acc + 1, (unsigned long long)cnt);
    }
}

__global__ void sub_query_kernel(const uint16_t *__restrict__ table, uint64_t slots,
                                 const uint64_t *__restrict__ keys, uint16_t *__restrict__ out,
                                 uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = keys[i] < slots ? record_of_score(table[keys[i]]) : REC_UNSOLVED;
}

// ---------------------------------------------------------------------------
static int prepare(Ctx *c, DenseSub *d) {
    int heaps = c->sub.heaps;
    int low = std::min(c->sub_low, heaps);
    if (low < 1) low = 1;
    if (low > 3) low = 3;
    int high = heaps - low;
    if (!pick_kernel(low, high)) {
        set_error("no dense kernel for %d heaps at %d low heaps", heaps, low);
        return GM_E_GAME;
    }
    d->heaps = heaps; d->low = low; d->high = high;
    d->slots = 1ull << (4 * heaps);
    uint64_t nhigh = 1ull << (4 * high);
    // counting sort of high parts by nibble sum (tier)
    std::vector<uint32_t> cnt(15 * high + 2, 0), order(nhigh);
    auto tsum = [&](uint64_t v) { int s = 0; for (int j = 0; j < high; j++) s += (v >> (4 * j)) & 15; return s; };
    for (uint64_t v = 0; v < nhigh; v++) cnt[tsum(v) + 1]++;
    for (size_t t = 1; t < cnt.size(); t++) cnt[t] += cnt[t - 1];
    d->tier_off.assign(cnt.begin(), cnt.end());
    std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
    for (uint64_t v = 0; v < nhigh; v++) order[pos[tsum(v)]++] = (uint32_t)v;
    GM_HIP(hipMalloc(&d->d_blocks, nhigh * sizeof(uint32_t)));
    GM_HIP(hipMemcpy(d->d_blocks, order.data(), nhigh * sizeof(uint32_t), hipMemcpyHostToDevice));
    size_t zbytes = std::max<size_t>(16, (size_t)2 << (4 * low));
    GM_HIP(hipMalloc(&d->zero, zbytes));
    GM_HIP(hipMemset(d->zero, 0, zbytes));
    GM_HIP(hipMalloc(&d->d_acc, 2 * sizeof(uint64_t)));
    uint64_t bytes = d->slots * 2;
    if (c->adopted_dense) {
        if (c->adopted_dense_bytes < bytes) {
            set_error("adopted dense table holds %llu bytes, need %llu",
                      (unsigned long long)c->adopted_dense_bytes, (unsigned long long)bytes);
            return GM_E_CAP;
        }
        d->table = (uint16_t *)c->adopted_dense;
        d->owned = false;
    } else {
        if (hipMalloc(&d->table, bytes) != hipSuccess) {
            set_error("hipMalloc of %llu-byte dense table failed", (unsigned long long)bytes);
            return GM_E_NOMEM;
        }
        d->owned = true;
    }
    return GM_OK;
}

static int ensure_events(DenseSub *d) {
    int ntiers = (int)d->tier_off.size() - 1;
    for (int i = (int)d->ev.size(); i < 2 * ntiers; i++) {
        hipEvent_t e;
        GM_HIP(hipEventCreate(&e));
        d->ev.push_back(e);
    }
    return GM_OK;
}

static int launch_tiers(Ctx *c, DenseSub *d, bool timed) {
    tier_kernel_t k = pick_kernel(d->low, d->high);
    int ntiers = (int)d->tier_off.size() - 1;
    for (int t = 0; t < ntiers; t++) {
        uint32_t nb = d->tier_off[t + 1] - d->tier_off[t];
        if (!nb) continue;
        if (timed) GM_HIP(hipEventRecord(d->ev[2 * t], c->stream));
        hipLaunchKernelGGL(k, dim3(nb), dim3(256), 0, c->stream, d->table,
                           d->d_blocks + d->tier_off[t], nb, d->zero);
        if (timed) GM_HIP(hipEventRecord(d->ev[2 * t + 1], c->stream));
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

int dense_sub_solve(Ctx *c, uint64_t root) {
    DenseSub *d = c->dsub;
    if (!d || d->heaps != c->sub.heaps || d->low != std::min(std::max(c->sub_low, 1), std::min(3, c->sub.heaps)) ||
        (c->adopted_dense && d->table != c->adopted_dense)) {
        dense_sub_free(c);
        d = c->dsub = new DenseSub();
        GM_TRY(prepare(c, d));
    }
    double t0 = now_ms();
    bool timed = c->timing;
    if (timed) GM_TRY(ensure_events(d));
    if (c->use_graph) {
        // Replay the per-tier launches as one hipGraph.  Timing brackets the
        // whole replay with one event pair (event-record nodes captured into a
        // graph do not update the host-visible events), so the per-launch time
        // it yields includes the graph's inter-kernel gaps.
        if (!d->graph || d->graph_stream != c->stream) {
            if (d->graph) { hipGraphExecDestroy(d->graph); d->graph = nullptr; }
            hipGraph_t g;
            GM_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
            int rc = launch_tiers(c, d, false);
            hipError_t e = hipStreamEndCapture(c->stream, &g);
            if (rc != GM_OK) return rc;
            if (e != hipSuccess) { set_error("graph capture failed: %s", hipGetErrorString(e)); return GM_E_HIP; }
            GM_HIP(hipGraphInstantiate(&d->graph, g, nullptr, nullptr, 0));
            GM_HIP(hipGraphDestroy(g));
            d->graph_stream = c->stream;
        }
        if (timed) GM_HIP(hipEventRecord(d->ev[0], c->stream));
        GM_HIP(hipGraphLaunch(d->graph, c->stream));
        if (timed) GM_HIP(hipEventRecord(d->ev[1], c->stream));
    } else {
        GM_TRY(launch_tiers(c, d, timed));
    }
    uint16_t rs;
    GM_HIP(hipMemcpyAsync(&rs, d->table + root, 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    double t1 = now_ms();

    c->root_record = record_of_score(rs);
    uint64_t n = 1;
    for (int j = 0; j < d->heaps; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    int ntiers = (int)d->tier_off.size() - 1;
    c->tier_counts.assign(15 * d->heaps + 1, 0);
    // positions per global tier (heap sum) of the full table
    {
        std::vector<uint64_t> one(16, 1), acc(1, 1);
        for (int j = 0; j < d->heaps; j++) {
            std::vector<uint64_t> nx(acc.size() + 15, 0);
            for (size_t s = 0; s < acc.size(); s++)
                for (int h = 0; h < 16; h++) nx[s + h] += acc[s];
            acc.swap(nx);
        }
        for (size_t s = 0; s < acc.size() && s < c->tier_counts.size(); s++) c->tier_counts[s] = acc[s];
    }
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = ntiers;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.forward_ms = 0;
    // 2 B written + 2 B per child edge = 2 * (1 + 1.8125 * heaps) per slot
    double dbar = 1.8125 * d->heaps;
    c->stats.algo_bytes = (uint64_t)((double)d->slots * 2.0 * (1.0 + dbar));
    c->stats.table_bytes = d->slots * 2;
    if (timed) {
        float total = 0;
        int launches = 0;
        for (int t = 0; t < ntiers; t++) {
            if (d->tier_off[t + 1] == d->tier_off[t]) continue;
            launches++;
            if (c->use_graph) continue;
            float ms = 0;
            GM_HIP(hipEventElapsedTime(&ms, d->ev[2 * t], d->ev[2 * t + 1]));
            total += ms;
        }
        if (c->use_graph) GM_HIP(hipEventElapsedTime(&total, d->ev[0], d->ev[1]));
        c->stats.kernel_ms = total;
        c->stats.kernel_launches = launches;
    }
    return GM_OK;
}

int dense_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DenseSub *d = c->dsub;
    *n = c->n_positions;
    if (!keys) return GM_OK;
    if (cap < c->n_positions) { set_error("export buffer holds %llu, need %llu",
                                          (unsigned long long)cap, (unsigned long long)c->n_positions);
                                return GM_E_CAP; }
    std::vector<uint16_t> h(d->slots);
    GM_HIP(hipMemcpy(h.data(), d->table, d->slots * 2, hipMemcpyDeviceToHost));
    uint64_t j = 0;
    for (uint64_t k = 0; k < d->slots; k++) {
        bool in = true;
        for (int i = 0; i < d->heaps && in; i++) in = ((k >> (4 * i)) & 15u) <= ((c->root >> (4 * i)) & 15u);
        if (!in) continue;
        keys[j] = k;
        recs[j] = record_of_score(h[k]);
        j++;
    }
    return GM_OK;
}

int dense_sub_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    DenseSub *d = c->dsub;
    if (!n) return GM_OK;
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, n * 8));
    GM_HIP(hipMalloc(&dr, n * 2));
    GM_HIP(hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(sub_query_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream,
                       d->table, d->slots, dk, dr, n);
    GM_HIP(hipMemcpyAsync(recs, dr, n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    hipFree(dk);
    hipFree(dr);
    return GM_OK;
}

int dense_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DenseSub *d = c->dsub;
    GM_HIP(hipMemsetAsync(d->d_acc, 0, 16, c->stream));
    hipLaunchKernelGGL(sub_digest_kernel, dim3(2048), dim3(256), 0, c->stream, d->table, d->slots,
                       d->heaps, c->root, (unsigned long long *)d->d_acc);
    uint64_t h[2];
    GM_HIP(hipMemcpyAsync(h, d->d_acc, 16, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = h[0];
    *n = h[1];
    return GM_OK;
}

int dense_sub_table(Ctx *c, void **p, uint64_t *bytes) {
    DenseSub *d = c->dsub;
    *p = d->table;
    *bytes = d->slots * 2;
    return GM_OK;
}

void dense_sub_free(Ctx *c) {
    DenseSub *d = c->dsub;
    if (!d) return;
    if (d->graph) hipGraphExecDestroy(d->graph);
    for (auto e : d->ev) hipEventDestroy(e);
    if (d->owned && d->table) hipFree(d->table);
    if (d->zero) hipFree(d->zero);
    if (d->d_blocks) hipFree(d->d_blocks);
    if (d->d_acc) hipFree(d->d_acc);
    delete d;
    c->dsub = nullptr;
}

}  // namespace gm
