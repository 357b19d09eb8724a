// graph.hip -- retrograde over an explicit position graph (GM_GAME_GRAPH).
//
// For plugins that no device descriptor reproduces: the host
// walks the plugin itself (initial_position / gen_moves / do_move / primitive,
// reference README.md:28-88) and hands over the graph in CSR form -- position i's
// primitive() code and the indices of its children; the device resolves it with
// the same canonical reduction as every other engine (Appendix A,
// gm_common.hpp preference scores).
//
// Rounds: every unresolved position whose children are all resolved takes
// parent_score(max child score); a round that resolves nothing while positions
// remain means a cycle (the reference would never terminate either) and fails.
// Rounds = the height of the graph; a position is written once, when final, so
// reading a child in the round it is written is benign.
#include "gm_internal.hpp"

#include <algorithm>

namespace gm {

struct Graph {
    uint64_t n = 0;
    uint8_t *prim = nullptr;
    uint64_t *off = nullptr;
    uint32_t *kid = nullptr;
    uint16_t *score = nullptr;
    unsigned long long *d_count = nullptr;
    uint32_t *d_err = nullptr;
};

__global__ __launch_bounds__(256) void graph_init_kernel(const uint8_t *__restrict__ prim, uint64_t n,
                                                         uint16_t *__restrict__ score, uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int p = prim[i];
        if (p > UNDECIDED) atomicOr(err, DEV_ERR_TIER);   // not a primitive() code
        if (p == DRAW) atomicOr(err, DEV_ERR_DRAW);
        score[i] = p == UNDECIDED ? 0 : score_of_primitive(p);
    }
}

__global__ __launch_bounds__(256) void graph_round_kernel(const uint64_t *__restrict__ off,
                                                          const uint32_t *__restrict__ kid, uint64_t n,
                                                          uint16_t *score, unsigned long long *resolved,
                                                          uint32_t *err) {
    uint64_t done = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        if (score[i]) continue;
        const uint64_t a = off[i], b = off[i + 1];
        if (a == b) { atomicOr(err, DEV_ERR_NOMOVES); continue; }
        uint32_t best = 0;
        bool ready = true;
        for (uint64_t e = a; e < b; e++) {
            const uint32_t s = ((const volatile uint16_t *)score)[kid[e]];
            if (!s) { ready = false; break; }
            best = max(best, s);
        }
        if (!ready) continue;
        if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
        ((volatile uint16_t *)score)[i] = parent_score(best);
        done++;
    }
    for (int o = 32; o > 0; o >>= 1) done += __shfl_xor(done, o);
    if ((threadIdx.x & 63) == 0 && done) atomicAdd(resolved, (unsigned long long)done);
}

__global__ void graph_records_kernel(const uint16_t *__restrict__ score, const uint64_t *__restrict__ idx,
                                     uint16_t *__restrict__ out, uint64_t n, uint64_t total) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = idx ? idx[i] : i;
    out[i] = k < total ? record_of_score(score[k]) : REC_UNSOLVED;
}

__global__ void graph_digest_kernel(const uint16_t *__restrict__ score, uint64_t n, unsigned long long *acc) {
    uint64_t sum = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        sum += digest_term(i, record_of_score(score[i]));
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, (unsigned long long)sum);
}

static unsigned grid_of(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192)); }

int graph_solve(Ctx *c, uint64_t n, const uint8_t *prim, const uint64_t *off, const uint32_t *kid) {
    graph_free(c);
    if (!n) { set_error("empty graph"); return GM_E_ARG; }
    Graph *g = c->graph = new Graph();
    g->n = n;
    const uint64_t m = off[n];
    for (uint64_t i = 0; i < m; i++)
        if (kid[i] >= n) { set_error("child index %u out of range", kid[i]); return GM_E_ARG; }
    double t0 = now_ms();
    GM_TRY(dev_alloc(c, (void **)&g->prim, n));
    GM_TRY(dev_alloc(c, (void **)&g->off, (n + 1) * 8));
    GM_TRY(dev_alloc(c, (void **)&g->kid, std::max<uint64_t>(m, 1) * 4));
    GM_TRY(dev_alloc(c, (void **)&g->score, n * 2));
    GM_TRY(dev_alloc(c, (void **)&g->d_count, 8));
    GM_TRY(dev_alloc(c, (void **)&g->d_err, 4));
    GM_HIP(hipMemcpyAsync(g->prim, prim, n, hipMemcpyHostToDevice, c->stream));
    GM_HIP(hipMemcpyAsync(g->off, off, (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    if (m) GM_HIP(hipMemcpyAsync(g->kid, kid, m * 4, hipMemcpyHostToDevice, c->stream));
    GM_HIP(hipMemsetAsync(g->d_err, 0, 4, c->stream));
    hipLaunchKernelGGL(graph_init_kernel, dim3(grid_of(n)), dim3(256), 0, c->stream, g->prim, n, g->score, g->d_err);
    uint64_t interior = 0;
    for (uint64_t i = 0; i < n; i++) interior += prim[i] == UNDECIDED;
    uint64_t left = interior;
    int rounds = 0;
    while (left) {
        GM_HIP(hipMemsetAsync(g->d_count, 0, 8, c->stream));
        hipLaunchKernelGGL(graph_round_kernel, dim3(grid_of(n)), dim3(256), 0, c->stream, g->off, g->kid, n, g->score,
                           g->d_count, g->d_err);
        unsigned long long got = 0;
        uint32_t e = 0;
        GM_HIP(hipMemcpyAsync(&got, g->d_count, 8, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipMemcpyAsync(&e, g->d_err, 4, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        if (e) return dev_error_to_gm(e);
        rounds++;
        if (!got) {
            set_error("%llu positions never resolve: the graph has a cycle", (unsigned long long)left);
            return GM_E_STATE;
        }
        left -= got;
    }
    uint32_t e = 0;
    GM_HIP(hipMemcpyAsync(&e, g->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    uint16_t rs;
    GM_HIP(hipMemcpyAsync(&rs, g->score, 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    if (e) return dev_error_to_gm(e);
    double t1 = now_ms();
    c->root = 0;
    c->root_record = record_of_score(rs);
    c->n_positions = n;
    c->stats.n_positions = n;
    c->stats.n_primitive = n - interior;
    c->stats.n_tiers = rounds;
    c->stats.n_edges = m;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.table_bytes = n * 11 + m * 4;
    c->tier_counts.clear();
    return GM_OK;
}

int graph_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    Graph *g = c->graph;
    *n = g->n;
    if (!keys) return GM_OK;
    if (cap < g->n) { set_error("export buffer too small"); return GM_E_CAP; }
    uint16_t *dr;
    GM_HIP(hipMalloc(&dr, g->n * 2));
    hipLaunchKernelGGL(graph_records_kernel, dim3((unsigned)((g->n + 255) / 256)), dim3(256), 0, c->stream, g->score,
                       (const uint64_t *)nullptr, dr, g->n, g->n);
    GM_HIP(hipMemcpyAsync(recs, dr, g->n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dr);
    for (uint64_t i = 0; i < g->n; i++) keys[i] = i;
    return GM_OK;
}

int graph_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    Graph *g = c->graph;
    if (!n) return GM_OK;
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, n * 8));
    GM_HIP(hipMalloc(&dr, n * 2));
    GM_HIP(hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(graph_records_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, g->score, dk,
                       dr, n, g->n);
    GM_HIP(hipMemcpyAsync(recs, dr, n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

int graph_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    Graph *g = c->graph;
    GM_HIP(hipMemsetAsync(g->d_count, 0, 8, c->stream));
    hipLaunchKernelGGL(graph_digest_kernel, dim3(grid_of(g->n)), dim3(256), 0, c->stream, g->score, g->n, g->d_count);
    unsigned long long h;
    GM_HIP(hipMemcpyAsync(&h, g->d_count, 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = h;
    *n = g->n;
    return GM_OK;
}

void graph_free(Ctx *c) {
    Graph *g = c->graph;
    if (!g) return;
    for (void *p : {(void *)g->prim, (void *)g->off, (void *)g->kid, (void *)g->score, (void *)g->d_count,
                    (void *)g->d_err})
        dev_free(c, p);
    (void)hipStreamSynchronize(c->stream);
    delete g;
    c->graph = nullptr;
}

}  // namespace gm
