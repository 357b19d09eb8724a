// sparse.hip -- level-synchronous frontier expansion + tiered retrograde over
// per-tier open-addressing tables in HBM (Four-To-One, Toot-and-Otto, Othello;
// any descriptor).
//
// Replaces the reference's asynchronous job loop and its tables:
//   LOOK_UP / DISTRIBUTE (src/new_process.py:102-162)  -> expand kernel: one lane
//       per position of tier t evaluates primitive() and, if undecided,
//       generates its children and inserts them (atomicCAS on u64 keys) into the
//       tables of tiers t+1..t+MAX_SKIP; the table IS the deduplicated frontier
//   CacheDict resolved/remote (src/cache_dict.py)      -> per-tier tables:
//       u64 key[cap] (2^63 = empty) + u16 score[cap], linear probing on mix64(key)
//   RESOLVE / _res_red (src/new_process.py:223-265)    -> retro kernel, tiers
//       deepest first: regenerate children, look each up in its tier's table,
//       u16 max over preference scores, parent score (gm_common.hpp)
// The reference expands a position once per path that reaches it (tree
// search); here each distinct position is expanded once.
#include "sparse_common.hpp"

namespace gm {

template <int S>
struct NextTables {
    TableRef t[S];
};

struct Sparse {
    std::vector<Table> tiers;
    unsigned long long *d_counts = nullptr;   // per-tier distinct counts (device)
    uint64_t counts_cap = 0;
    unsigned long long *d_scratch = nullptr;  // edge counts / digest / export cursor
    uint32_t *d_err = nullptr;
    int64_t t_root = 0;
    int max_skip = 1;
};

// ----------------------------------------------------------------- kernels
template <class D>
__global__ __launch_bounds__(256) void count_edges_kernel(D d, const uint64_t *__restrict__ keys,
                                                          uint64_t cap, unsigned long long *edges,
                                                          uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    uint64_t cnt[S];
#pragma unroll
    for (int s = 0; s < S; s++) cnt[s] = 0;
    uint64_t kids[D::MAXC];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k == EMPTY_KEY) continue;
        int p = d.primitive(k);
        if (p != UNDECIDED) {
            if (p == DRAW) atomicOr(err, DEV_ERR_DRAW);
            continue;
        }
        int n = d.children(k, kids);
        if (!n) atomicOr(err, DEV_ERR_NOMOVES);
        int64_t tk = d.tier(k);
        for (int c = 0; c < n; c++) {
            int64_t dt = d.tier(kids[c]) - tk;
            if (dt < 1 || dt > S) { atomicOr(err, DEV_ERR_TIER); continue; }
#pragma unroll
            for (int s = 0; s < S; s++) cnt[s] += dt == s + 1;
        }
    }
#pragma unroll
    for (int s = 0; s < S; s++) wave_add(edges + s, cnt[s]);
}

template <class D>
__global__ __launch_bounds__(256) void expand_kernel(D d, const uint64_t *__restrict__ keys,
                                                     uint16_t *__restrict__ score, uint64_t cap,
                                                     NextTables<D::MAX_SKIP> next, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    uint64_t fresh[S];
#pragma unroll
    for (int s = 0; s < S; s++) fresh[s] = 0;
    uint64_t kids[D::MAXC];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k == EMPTY_KEY) continue;
        int p = d.primitive(k);
        if (p != UNDECIDED) {
            score[i] = score_of_primitive(p);
            continue;
        }
        score[i] = 0;
        int n = d.children(k, kids);
        int64_t tk = d.tier(k);
        for (int c = 0; c < n; c++) {
            int64_t dt = d.tier(kids[c]) - tk;
#pragma unroll
            for (int s = 0; s < S; s++)
                if (dt == s + 1 && table_insert(next.t[s], kids[c], err)) fresh[s]++;
        }
    }
#pragma unroll
    for (int s = 0; s < S; s++) wave_add(next.t[s].count, fresh[s]);
}

template <class D>
__global__ __launch_bounds__(256) void retro_kernel(D d, const uint64_t *__restrict__ keys,
                                                    uint16_t *__restrict__ score, uint64_t cap,
                                                    NextTables<D::MAX_SKIP> next, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    uint64_t kids[D::MAXC];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k == EMPTY_KEY || score[i]) continue;   // empty slot or primitive
        int n = d.children(k, kids);
        int64_t tk = d.tier(k);
        uint32_t best = 0;
        for (int c = 0; c < n; c++) {
            int64_t dt = d.tier(kids[c]) - tk;
            uint32_t sc = 0;
#pragma unroll
            for (int s = 0; s < S; s++)
                if (dt == s + 1) {
                    int64_t slot = table_find(next.t[s], kids[c]);
                    if (slot < 0) atomicOr(err, DEV_ERR_MISSING_CHILD);
                    else sc = next.t[s].score[slot];
                }
            best = max(best, sc);
        }
        if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
        score[i] = parent_score(best);
    }
}

__global__ void insert_one_kernel(TableRef t, uint64_t key, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && table_insert(t, key, err)) atomicAdd(t.count, 1ull);
}

template <class D>
__global__ void query_kernel(D d, int64_t t_root, const TableRef *tabs, int ntabs,
                             const uint64_t *__restrict__ keys, uint16_t *__restrict__ out, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t k = keys[i];
    int64_t t = d.valid(k) ? d.tier(k) - t_root : -1;
    uint16_t r = REC_UNSOLVED;
    if (t >= 0 && t < ntabs && tabs[t].mask) {
        int64_t s = table_find(tabs[t], k);
        if (s >= 0) r = record_of_score(tabs[t].score[s]);
    }
    out[i] = r;
}

// ----------------------------------------------------------------- host side
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

static TableRef ref_of(Sparse *sp, size_t t) {
    Table &T = sp->tiers[t];
    TableRef r;
    r.keys = T.keys;
    r.score = T.score;
    r.mask = T.cap ? T.cap - 1 : 0;
    r.count = sp->d_counts + t;
    return r;
}

static int resize_tier(Ctx *c, Sparse *sp, size_t t, uint64_t cap) {
    return resize_table(c->stream, sp->tiers[t], cap, sp->d_err);
}

static int read_err(Ctx *c, Sparse *sp) {
    uint32_t e;
    GM_HIP(hipMemcpyAsync(&e, sp->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    return e ? dev_error_to_gm(e) : GM_OK;
}

template <class D>
static int solve_with(Ctx *c, const D &d, uint64_t root) {
    constexpr int S = D::MAX_SKIP;
    sparse_free(c);
    Sparse *sp = c->sp = new Sparse();
    sp->max_skip = S;
    sp->t_root = d.tier(root);
    GM_HIP(hipMalloc(&sp->d_scratch, 64 * sizeof(unsigned long long)));
    GM_HIP(hipMalloc(&sp->d_err, 4));
    GM_HIP(hipMemsetAsync(sp->d_err, 0, 4, c->stream));
    GM_TRY(ensure_counts(sp, 64));
    double t0 = now_ms();

    sp->tiers.resize(1);
    GM_TRY(alloc_table(c->stream, sp->tiers[0], 1024));
    hipLaunchKernelGGL(insert_one_kernel, dim3(1), dim3(64), 0, c->stream, ref_of(sp, 0), root, sp->d_err);
    sp->tiers[0].count = 1;

    // ---------------- forward: tier by tier
    for (size_t t = 0; t < sp->tiers.size(); t++) {
        if (!sp->tiers[t].count) continue;
        Table &T = sp->tiers[t];
        // final now: shrink to load <= 1/2 (improves retro probing and memory)
        uint64_t want = pow2_at_least(2 * T.count);
        if (T.cap > 2 * want) GM_TRY(resize_tier(c, sp, t, want));
        GM_HIP(hipMemsetAsync(sp->d_scratch, 0, S * sizeof(unsigned long long), c->stream));
        hipLaunchKernelGGL(count_edges_kernel<D>, dim3(grid_for(sp->tiers[t].cap)), dim3(256), 0, c->stream, d,
                           sp->tiers[t].keys, sp->tiers[t].cap, sp->d_scratch, sp->d_err);
        unsigned long long edges[S];
        GM_HIP(hipMemcpyAsync(edges, sp->d_scratch, S * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                              c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(read_err(c, sp));
        if (sp->tiers.size() < t + S + 1) sp->tiers.resize(t + S + 1);
        GM_TRY(ensure_counts(sp, sp->tiers.size()));
        for (int s = 0; s < S; s++) {
            size_t u = t + 1 + s;
            uint64_t need = pow2_at_least((sp->tiers[u].count + edges[s]) * 5 / 4 + 1);
            if (edges[s] && sp->tiers[u].cap < need) GM_TRY(resize_tier(c, sp, u, need));
        }
        NextTables<S> nx;
        for (int s = 0; s < S; s++) nx.t[s] = ref_of(sp, t + 1 + s);
        hipLaunchKernelGGL(expand_kernel<D>, dim3(grid_for(sp->tiers[t].cap)), dim3(256), 0, c->stream, d,
                           sp->tiers[t].keys, sp->tiers[t].score, sp->tiers[t].cap, nx, sp->d_err);
        GM_HIP(hipGetLastError());
        std::vector<unsigned long long> cnt(sp->tiers.size());
        GM_HIP(hipMemcpyAsync(cnt.data(), sp->d_counts, cnt.size() * sizeof(unsigned long long),
                              hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(read_err(c, sp));
        for (size_t u = 0; u < cnt.size(); u++) sp->tiers[u].count = cnt[u];
    }
    while (!sp->tiers.empty() && !sp->tiers.back().count) sp->tiers.pop_back();
    double t1 = now_ms();

    // ---------------- backward: deepest tier first
    for (size_t tt = sp->tiers.size(); tt-- > 0;) {
        Table &T = sp->tiers[tt];
        if (!T.count) continue;
        NextTables<S> nx;
        for (int s = 0; s < S; s++) {
            size_t u = tt + 1 + s;
            nx.t[s] = u < sp->tiers.size() ? ref_of(sp, u) : TableRef{nullptr, nullptr, 0, nullptr};
        }
        hipLaunchKernelGGL(retro_kernel<D>, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, d, T.keys, T.score,
                           T.cap, nx, sp->d_err);
    }
    GM_HIP(hipGetLastError());
    GM_TRY(read_err(c, sp));
    double t2 = now_ms();

    // root record
    {
        uint64_t rk[1] = {root};
        uint16_t rr[1];
        GM_TRY(sparse_query(c, rk, rr, 1));
        c->root_record = rr[0];
    }
    uint64_t n = 0;
    c->tier_counts.clear();
    for (auto &T : sp->tiers) {
        n += T.count;
        c->tier_counts.push_back(T.count);
    }
    c->n_positions = n;
    c->stats.n_positions = n;
    c->stats.n_tiers = (int32_t)sp->tiers.size();
    c->stats.forward_ms = t1 - t0;
    c->stats.backward_ms = t2 - t1;
    c->stats.solve_ms = t2 - t0;
    uint64_t tb = 0;
    for (auto &T : sp->tiers) tb += T.cap * 10;
    c->stats.table_bytes = tb;
    return GM_OK;
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

static int sparse_query_refs(Ctx *c, Sparse *sp, TableRef **d_tabs) {
    std::vector<TableRef> h(sp->tiers.size());
    for (size_t t = 0; t < h.size(); t++) h[t] = ref_of(sp, t);
    GM_HIP(hipMalloc(d_tabs, std::max<size_t>(1, h.size()) * sizeof(TableRef)));
    GM_HIP(hipMemcpy(*d_tabs, h.data(), h.size() * sizeof(TableRef), hipMemcpyHostToDevice));
    return GM_OK;
}

template <class D>
static void launch_query(Ctx *c, const D &d, Sparse *sp, TableRef *tabs, const uint64_t *dk, uint16_t *dr,
                         uint64_t n) {
    hipLaunchKernelGGL(query_kernel<D>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, d,
                       sp->t_root, tabs, (int)sp->tiers.size(), dk, dr, n);
}

int sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    Sparse *sp = c->sp;
    if (!n) return GM_OK;
    TableRef *tabs;
    GM_TRY(sparse_query_refs(c, sp, &tabs));
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, n * 8));
    GM_HIP(hipMalloc(&dr, n * 2));
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
    hipFree(dk);
    hipFree(dr);
    hipFree(tabs);
    return GM_OK;
}

int sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    Sparse *sp = c->sp;
    uint64_t total = 0;
    for (auto &T : sp->tiers) total += T.count;
    *n = total;
    if (!keys) return GM_OK;
    if (cap < total) { set_error("export buffer holds %llu, need %llu", (unsigned long long)cap,
                                 (unsigned long long)total); return GM_E_CAP; }
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, std::max<uint64_t>(1, total) * 8));
    GM_HIP(hipMalloc(&dr, std::max<uint64_t>(1, total) * 2));
    GM_HIP(hipMemsetAsync(sp->d_scratch, 0, 8, c->stream));
    for (auto &T : sp->tiers)
        if (T.count)
            hipLaunchKernelGGL(gather_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.keys, T.score,
                               T.cap, dk, dr, sp->d_scratch);
    std::vector<uint64_t> hk(total);
    std::vector<uint16_t> hr(total);
    GM_HIP(hipMemcpyAsync(hk.data(), dk, total * 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipMemcpyAsync(hr.data(), dr, total * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    hipFree(dk);
    hipFree(dr);
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
    GM_HIP(hipMemsetAsync(sp->d_scratch, 0, 8, c->stream));
    uint64_t total = 0;
    for (auto &T : sp->tiers) {
        total += T.count;
        if (T.count)
            hipLaunchKernelGGL(digest_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.keys, T.score,
                               T.cap, sp->d_scratch);
    }
    unsigned long long h;
    GM_HIP(hipMemcpyAsync(&h, sp->d_scratch, 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = h;
    *n = total;
    return GM_OK;
}

void sparse_free(Ctx *c) {
    Sparse *sp = c->sp;
    if (!sp) return;
    for (auto &T : sp->tiers) free_table(T);
    if (sp->d_counts) hipFree(sp->d_counts);
    if (sp->d_scratch) hipFree(sp->d_scratch);
    if (sp->d_err) hipFree(sp->d_err);
    delete sp;
    c->sp = nullptr;
}

}  // namespace gm
