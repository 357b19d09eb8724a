// dist_sparse.hip -- the sparse engine hash-sharded over G ranks (Othello, Toot, ...).
//
// Every position has one owner, owner_rank(key) = (mix64(key) >> 32) % G
// (the role of GameState.get_hash, reference src/game_state.py:23-31).  The
// reference sends one pickled Job per edge: LOOK_UP to the child's owner
// (src/new_process.py:159) and RESOLVE back to the parent's rank (:186).  Here
// both are batched per tier into bulk-synchronous exchanges:
//
// forward, tier t:   each rank expands its own tier-t positions; children are
//                    bucketed by (owner, tier offset) with an LDS histogram per
//                    workgroup; counts are all-gathered; keys move with one
//                    ncclGroup of send/recv per peer; owners insert them into their
//                    tier tables (deduplicating on insert).
// backward, tier t:  each rank regenerates its own positions' children and sends
//                    the keys to their owners (LOOK_UP); owners answer with the
//                    children's u16 scores in the same order (RESOLVE); the
//                    parent folds them with atomicMax and turns the best score into
//                    its own (gm_common.hpp).
//
// Exchanges use RCCL point-to-point (one process per GPU) or, with
// GM_OPT_VIRTUAL_RANKS, device copies between G virtual ranks in one context.
#include "sparse_common.hpp"

namespace gm {

struct SpRank {
    int rank = 0;
    std::vector<Table> tiers;
    uint32_t *d_err = nullptr;
    unsigned long long *d_hist = nullptr;    // G*S counters
    unsigned long long *d_cursor = nullptr;  // G*S cursors
    unsigned long long *d_seg = nullptr;     // G*S segment bases
    unsigned long long *d_acc = nullptr;
    // per-tier scratch (grown on demand)
    uint64_t *sendk = nullptr, *recvk = nullptr;
    uint64_t *sendp = nullptr;               // parent slot of each outgoing request
    uint16_t *reply_out = nullptr, *reply_in = nullptr;
    uint32_t *best = nullptr;
    uint64_t send_cap = 0, recv_cap = 0, best_cap = 0;
};

struct DistSparse {
    int G = 1, S = 1;
    bool loopback = false;
    int64_t t_root = 0;
    std::vector<SpRank> ranks;
    std::vector<uint64_t> global_tier_counts;
    unsigned long long *d_mat = nullptr;     // all-gathered G*G*S counts (RCCL mode)
    uint32_t *d_root = nullptr;
    uint64_t sent_bytes = 0;
};

// ------------------------------------------------------------------ kernels
// Pass 1 (count) and pass 2 (scatter) share the edge enumeration: for every
// occupied slot of the tier, primitive positions get their score, others emit
// (child, owner, dt).  LDS histogram over the G*S bins, one global atomic per
// bin per workgroup; pass 2 reserves a range per bin per workgroup and writes.
template <class D, bool SCATTER>
__global__ __launch_bounds__(256) void edge_kernel(D d, const uint64_t *__restrict__ keys,
                                                   uint16_t *__restrict__ score, uint64_t cap, int G,
                                                   unsigned long long *hist,
                                                   const unsigned long long *__restrict__ seg,
                                                   unsigned long long *cursor, uint64_t *out_keys,
                                                   uint64_t *out_parent, int set_scores, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    constexpr int MAXBINS = 64 * 3;
    __shared__ unsigned int lh[MAXBINS];
    __shared__ unsigned long long lbase[MAXBINS];
    const int nb = G * S;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    uint64_t kids[D::MAXC];
    uint16_t bins[D::MAXC];
    int n = 0;
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t k = i < cap ? keys[i] : EMPTY_KEY;
    if (k != EMPTY_KEY) {
        int p = d.primitive(k);
        if (p != UNDECIDED) {
            if (p == DRAW) atomicOr(err, DEV_ERR_DRAW);
            if (set_scores) score[i] = score_of_primitive(p);
        } else {
            if (set_scores) score[i] = 0;
            n = d.children(k, kids);
            if (!n) atomicOr(err, DEV_ERR_NOMOVES);
            int64_t tk = d.tier(k);
            for (int c = 0; c < n; c++) {
                int64_t dt = d.tier(kids[c]) - tk;
                if (dt < 1 || dt > S) { atomicOr(err, DEV_ERR_TIER); dt = 1; }
                bins[c] = (uint16_t)(owner_rank(kids[c], (uint32_t)G) * S + (dt - 1));
            }
        }
    }
    // local positions inside each bin
    uint32_t local[D::MAXC];
    for (int c = 0; c < n; c++) local[c] = atomicAdd(&lh[bins[c]], 1u);
    __syncthreads();
    if (!SCATTER) {
        for (int b = threadIdx.x; b < nb; b += blockDim.x)
            if (lh[b]) atomicAdd(&hist[b], (unsigned long long)lh[b]);
        return;
    }
    for (int b = threadIdx.x; b < nb; b += blockDim.x)
        lbase[b] = lh[b] ? seg[b] + atomicAdd(&cursor[b], (unsigned long long)lh[b]) : 0;
    __syncthreads();
    for (int c = 0; c < n; c++) {
        unsigned long long at = lbase[bins[c]] + local[c];
        out_keys[at] = kids[c];
        if (out_parent) out_parent[at] = i;
    }
}

__global__ void insert_keys_kernel(const uint64_t *__restrict__ in, uint64_t n, TableRef t, uint32_t *err) {
    uint64_t fresh = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        if (table_insert(t, in[i], err)) fresh++;
    wave_add(t.count, fresh);
}

__global__ void lookup_kernel(const uint64_t *__restrict__ in, uint64_t n, TableRef t, uint16_t *out,
                              uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        int64_t s = table_find(t, in[i]);
        if (s < 0) { atomicOr(err, DEV_ERR_MISSING_CHILD); out[i] = 0; }
        else out[i] = t.score[s];
    }
}

__global__ void fold_kernel(const uint16_t *__restrict__ reply, const uint64_t *__restrict__ parent, uint64_t n,
                            uint32_t *best) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
        atomicMax(&best[parent[i]], (uint32_t)reply[i]);
}

__global__ void finalize_kernel(const uint64_t *__restrict__ keys, uint16_t *score, const uint32_t *best,
                                uint64_t cap, uint32_t *err) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (keys[i] == EMPTY_KEY || score[i]) continue;
        uint32_t b = best[i];
        if (!b) atomicOr(err, DEV_ERR_MISSING_CHILD);
        if (score_overflows(b)) atomicOr(err, DEV_ERR_OVERFLOW);
        score[i] = parent_score(b);
    }
}

__global__ void insert_root_kernel(TableRef t, uint64_t key, uint32_t *err) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && table_insert(t, key, err)) atomicAdd(t.count, 1ull);
}

// ------------------------------------------------------------------ host helpers
static int grow(uint64_t **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap) return GM_OK;
    if (*p) (void)hipFree(*p);
    uint64_t c = std::max<uint64_t>(need + need / 4, 1 << 16);
    GM_HIP(hipMalloc(p, c * 8));
    *cap = c;
    return GM_OK;
}

static int grow16(uint16_t **p, uint64_t cap) {
    if (*p) (void)hipFree(*p);
    GM_HIP(hipMalloc(p, std::max<uint64_t>(cap, 1) * 2));
    return GM_OK;
}

static TableRef ref(Table &T, unsigned long long *count) {
    return TableRef{T.keys, T.score, T.cap ? T.cap - 1 : 0, count};
}

// Cross-rank exchange of G*S-segmented arrays.
struct Xch {
    Ctx *c;
    DistSparse *d;
    // RCCL: send to every peer its (dest) region, receive from every peer into (src) regions
    int sendrecv(SpRank &R, const void *send, const uint64_t *send_off, void *recv, const uint64_t *recv_off,
                 size_t elem) {
        if (d->loopback) return GM_OK;   // loopback copies are done by the caller
        GM_NCCL(ncclGroupStart());
        for (int p = 0; p < d->G; p++) {
            uint64_t sn = send_off[p + 1] - send_off[p], rn = recv_off[p + 1] - recv_off[p];
            if (sn) GM_NCCL(ncclSend((const char *)send + send_off[p] * elem, sn * elem, ncclUint8, p, c->comm, c->stream));
            if (rn) GM_NCCL(ncclRecv((char *)recv + recv_off[p] * elem, rn * elem, ncclUint8, p, c->comm, c->stream));
            d->sent_bytes += sn * elem;
        }
        GM_NCCL(ncclGroupEnd());
        return GM_OK;
    }
};

template <class D>
static int run_edges(Ctx *c, DistSparse *d, const D &desc, SpRank &R, Table &T, bool scatter, bool set_scores,
                     uint64_t *out_parent) {
    const int nb = d->G * d->S;
    unsigned grid = (unsigned)std::max<uint64_t>(1, (T.cap + 255) / 256);
    if (!scatter) {
        GM_HIP(hipMemsetAsync(R.d_hist, 0, nb * 8, c->stream));
        hipLaunchKernelGGL((edge_kernel<D, false>), dim3(grid), dim3(256), 0, c->stream, desc, T.keys, T.score, T.cap,
                           d->G, R.d_hist, nullptr, nullptr, nullptr, nullptr, set_scores, R.d_err);
    } else {
        GM_HIP(hipMemsetAsync(R.d_cursor, 0, nb * 8, c->stream));
        hipLaunchKernelGGL((edge_kernel<D, true>), dim3(grid), dim3(256), 0, c->stream, desc, T.keys, T.score, T.cap,
                           d->G, nullptr, R.d_seg, R.d_cursor, R.sendk, out_parent, 0, R.d_err);
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

// counts[r][dest*S+dt] for all ranks -> host matrix (G x G*S)
static int gather_counts(Ctx *c, DistSparse *d, std::vector<uint64_t> &mat) {
    const int nb = d->G * d->S;
    mat.assign((size_t)d->G * nb, 0);
    if (d->loopback) {
        for (auto &R : d->ranks)
            GM_HIP(hipMemcpyAsync(&mat[(size_t)R.rank * nb], R.d_hist, nb * 8, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        return GM_OK;
    }
    SpRank &R = d->ranks[0];
    GM_NCCL(ncclAllGather(R.d_hist, d->d_mat, nb, ncclUint64, c->comm, c->stream));
    GM_HIP(hipMemcpyAsync(mat.data(), d->d_mat, mat.size() * 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    return GM_OK;
}

static int check_err(Ctx *c, DistSparse *d) {
    for (auto &R : d->ranks) {
        uint32_t e;
        GM_HIP(hipMemcpyAsync(&e, R.d_err, 4, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        if (e) return dev_error_to_gm(e);
    }
    return GM_OK;
}

// One exchange step of keys (and optionally the way back of u16 replies).
// mat: G x (G*S) counts, row = source rank, column = dest*S + dt.
struct Layout {
    std::vector<uint64_t> seg;        // send segment bases per bin (dest-major), size G*S
    std::vector<uint64_t> send_off;   // per dest, size G+1
    std::vector<uint64_t> recv_off;   // per source, size G+1 (all dts of that source)
    std::vector<uint64_t> recv_seg;   // per (source, dt) base in the recv buffer, size G*S
    uint64_t nsend = 0, nrecv = 0;
};

static Layout layout_for(DistSparse *d, const std::vector<uint64_t> &mat, int r) {
    const int G = d->G, S = d->S, nb = G * S;
    Layout L;
    L.seg.resize(nb);
    L.send_off.assign(G + 1, 0);
    uint64_t acc = 0;
    for (int p = 0; p < G; p++) {
        L.send_off[p] = acc;
        for (int s = 0; s < S; s++) { L.seg[p * S + s] = acc; acc += mat[(size_t)r * nb + p * S + s]; }
    }
    L.send_off[G] = acc;
    L.nsend = acc;
    L.recv_off.assign(G + 1, 0);
    L.recv_seg.resize(nb);
    acc = 0;
    for (int q = 0; q < G; q++) {
        L.recv_off[q] = acc;
        for (int s = 0; s < S; s++) { L.recv_seg[q * S + s] = acc; acc += mat[(size_t)q * nb + r * S + s]; }
    }
    L.recv_off[G] = acc;
    L.nrecv = acc;
    return L;
}

template <class D>
static int solve_sharded(Ctx *c, const D &desc, uint64_t root) {
    dist_sparse_free(c);
    DistSparse *d = c->dist_sp = new DistSparse();
    d->loopback = c->virtual_ranks > 1;
    d->G = d->loopback ? c->virtual_ranks : c->world;
    d->S = D::MAX_SKIP;
    d->t_root = desc.tier(root);
    const int G = d->G, S = d->S, nb = G * S;
    if (nb > 64 * 3) { set_error("too many ranks for the sharded sparse engine"); return GM_E_ARG; }
    d->ranks.resize(d->loopback ? G : 1);
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SpRank &R = d->ranks[i];
        R.rank = d->loopback ? (int)i : c->rank;
        GM_HIP(hipMalloc(&R.d_err, 4));
        GM_HIP(hipMemset(R.d_err, 0, 4));
        GM_HIP(hipMalloc(&R.d_hist, nb * 8));
        GM_HIP(hipMalloc(&R.d_cursor, nb * 8));
        GM_HIP(hipMalloc(&R.d_seg, nb * 8));
        GM_HIP(hipMalloc(&R.d_acc, 64));
        R.tiers.resize(1);
        GM_TRY(alloc_table(c->stream, R.tiers[0], 1024));
    }
    GM_HIP(hipMalloc(&d->d_mat, (size_t)G * nb * 8));
    GM_HIP(hipMalloc(&d->d_root, 4));
    // per-rank device counters for table counts: one array per rank, indexed by tier
    std::vector<unsigned long long *> dcnt(d->ranks.size(), nullptr);
    size_t cnt_cap = 0;
    auto ensure_cnt = [&](size_t ntiers) -> int {
        if (ntiers <= cnt_cap) return GM_OK;
        size_t nc = std::max<size_t>(64, ntiers * 2);
        for (size_t i = 0; i < d->ranks.size(); i++) {
            unsigned long long *p;
            GM_HIP(hipMalloc(&p, nc * 8));
            GM_HIP(hipMemset(p, 0, nc * 8));
            if (dcnt[i]) { GM_HIP(hipMemcpy(p, dcnt[i], cnt_cap * 8, hipMemcpyDeviceToDevice)); (void)hipFree(dcnt[i]); }
            dcnt[i] = p;
        }
        cnt_cap = nc;
        return GM_OK;
    };
    GM_TRY(ensure_cnt(64));
    // the root lives on its owner
    for (size_t i = 0; i < d->ranks.size(); i++)
        if ((int)owner_rank(root, G) == d->ranks[i].rank)
            hipLaunchKernelGGL(insert_root_kernel, dim3(1), dim3(64), 0, c->stream,
                               ref(d->ranks[i].tiers[0], dcnt[i] + 0), root, d->ranks[i].d_err);
    d->global_tier_counts.assign(1, 1);
    double t0 = now_ms();

    std::vector<uint64_t> mat;
    // ---------------- forward
    for (size_t t = 0; t < d->global_tier_counts.size(); t++) {
        if (!d->global_tier_counts[t]) continue;
        size_t need = t + S + 1;
        if (d->global_tier_counts.size() < need) d->global_tier_counts.resize(need, 0);
        GM_TRY(ensure_cnt(need));
        for (auto &R : d->ranks) {
            if (R.tiers.size() < need) R.tiers.resize(need);
            Table &T = R.tiers[t];
            if (!T.cap) GM_TRY(alloc_table(c->stream, T, 1024));
            uint64_t want = pow2_at_least(2 * T.count);
            if (T.cap > 2 * want) GM_TRY(resize_table(c->stream, T, want, R.d_err));
            GM_TRY(run_edges(c, d, desc, R, T, false, true, nullptr));
        }
        GM_TRY(gather_counts(c, d, mat));
        GM_TRY(check_err(c, d));
        std::vector<Layout> lay(d->ranks.size());
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRank &R = d->ranks[i];
            lay[i] = layout_for(d, mat, R.rank);
            GM_TRY(grow(&R.sendk, &R.send_cap, lay[i].nsend));
            GM_TRY(grow(&R.recvk, &R.recv_cap, lay[i].nrecv));
            GM_HIP(hipMemcpyAsync(R.d_seg, lay[i].seg.data(), nb * 8, hipMemcpyHostToDevice, c->stream));
            GM_TRY(run_edges(c, d, desc, R, R.tiers[t], true, false, nullptr));
        }
        // exchange child keys
        if (d->loopback) {
            for (size_t i = 0; i < d->ranks.size(); i++)          // dest i
                for (size_t j = 0; j < d->ranks.size(); j++) {    // source j
                    uint64_t n = lay[i].recv_off[j + 1] - lay[i].recv_off[j];
                    if (n) GM_HIP(hipMemcpyAsync(d->ranks[i].recvk + lay[i].recv_off[j],
                                                 d->ranks[j].sendk + lay[j].send_off[i], n * 8,
                                                 hipMemcpyDeviceToDevice, c->stream));
                }
        } else {
            Xch x{c, d};
            GM_TRY(x.sendrecv(d->ranks[0], d->ranks[0].sendk, lay[0].send_off.data(), d->ranks[0].recvk,
                              lay[0].recv_off.data(), 8));
        }
        // owners insert: grow each destination table to hold all it may receive
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRank &R = d->ranks[i];
            for (int s = 0; s < S; s++) {
                uint64_t in = 0;
                for (int q = 0; q < G; q++) in += mat[(size_t)q * nb + R.rank * S + s];
                if (!in) continue;
                Table &U = R.tiers[t + 1 + s];
                uint64_t needc = pow2_at_least((U.count + in) * 5 / 4 + 1);
                if (U.cap < needc) GM_TRY(resize_table(c->stream, U, needc, R.d_err));
                for (int q = 0; q < G; q++) {
                    uint64_t n = mat[(size_t)q * nb + R.rank * S + s];
                    if (n)
                        hipLaunchKernelGGL(insert_keys_kernel, dim3(grid_for(n)), dim3(256), 0, c->stream,
                                           R.recvk + lay[i].recv_seg[q * S + s], n, ref(U, dcnt[i] + t + 1 + s),
                                           R.d_err);
                }
            }
        }
        GM_TRY(check_err(c, d));
        // global tier counts (sum over ranks of each rank's table counts)
        std::vector<uint64_t> local(need, 0), hc(need);
        for (size_t i = 0; i < d->ranks.size(); i++) {
            GM_HIP(hipMemcpyAsync(hc.data(), dcnt[i], need * 8, hipMemcpyDeviceToHost, c->stream));
            GM_HIP(hipStreamSynchronize(c->stream));
            for (size_t u = 0; u < need; u++) {
                d->ranks[i].tiers[u].count = hc[u];
                local[u] += hc[u];
            }
        }
        if (!d->loopback) {
            GM_HIP(hipMemcpyAsync(d->d_mat, local.data(), need * 8, hipMemcpyHostToDevice, c->stream));
            GM_NCCL(ncclAllReduce(d->d_mat, d->d_mat, need, ncclUint64, ncclSum, c->comm, c->stream));
            GM_HIP(hipMemcpyAsync(local.data(), d->d_mat, need * 8, hipMemcpyDeviceToHost, c->stream));
            GM_HIP(hipStreamSynchronize(c->stream));
        }
        for (size_t u = 0; u < need; u++) d->global_tier_counts[u] = local[u];
    }
    while (!d->global_tier_counts.empty() && !d->global_tier_counts.back()) d->global_tier_counts.pop_back();
    double t1 = now_ms();

    // ---------------- backward
    for (size_t t = d->global_tier_counts.size(); t-- > 0;) {
        if (!d->global_tier_counts[t]) continue;
        for (auto &R : d->ranks) GM_TRY(run_edges(c, d, desc, R, R.tiers[t], false, false, nullptr));
        GM_TRY(gather_counts(c, d, mat));
        std::vector<Layout> lay(d->ranks.size());
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRank &R = d->ranks[i];
            lay[i] = layout_for(d, mat, R.rank);
            uint64_t pc = R.send_cap;
            GM_TRY(grow(&R.sendk, &R.send_cap, lay[i].nsend));
            if (R.send_cap != pc || !R.sendp) {
                if (R.sendp) (void)hipFree(R.sendp);
                GM_HIP(hipMalloc(&R.sendp, R.send_cap * 8));
                GM_TRY(grow16(&R.reply_in, R.send_cap));
            }
            uint64_t rc = R.recv_cap;
            GM_TRY(grow(&R.recvk, &R.recv_cap, lay[i].nrecv));
            if (R.recv_cap != rc || !R.reply_out) GM_TRY(grow16(&R.reply_out, R.recv_cap));
            GM_HIP(hipMemcpyAsync(R.d_seg, lay[i].seg.data(), nb * 8, hipMemcpyHostToDevice, c->stream));
            GM_TRY(run_edges(c, d, desc, R, R.tiers[t], true, false, R.sendp));
        }
        // LOOK_UP: keys to owners
        if (d->loopback) {
            for (size_t i = 0; i < d->ranks.size(); i++)
                for (size_t j = 0; j < d->ranks.size(); j++) {
                    uint64_t n = lay[i].recv_off[j + 1] - lay[i].recv_off[j];
                    if (n) GM_HIP(hipMemcpyAsync(d->ranks[i].recvk + lay[i].recv_off[j],
                                                 d->ranks[j].sendk + lay[j].send_off[i], n * 8,
                                                 hipMemcpyDeviceToDevice, c->stream));
                }
        } else {
            Xch x{c, d};
            GM_TRY(x.sendrecv(d->ranks[0], d->ranks[0].sendk, lay[0].send_off.data(), d->ranks[0].recvk,
                              lay[0].recv_off.data(), 8));
        }
        // owners look up the scores
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRank &R = d->ranks[i];
            for (int q = 0; q < G; q++)
                for (int s = 0; s < S; s++) {
                    uint64_t n = mat[(size_t)q * nb + R.rank * S + s];
                    if (!n) continue;
                    Table &U = R.tiers[t + 1 + s];
                    hipLaunchKernelGGL(lookup_kernel, dim3(grid_for(n)), dim3(256), 0, c->stream,
                                       R.recvk + lay[i].recv_seg[q * S + s], n, ref(U, nullptr),
                                       R.reply_out + lay[i].recv_seg[q * S + s], R.d_err);
                }
        }
        // RESOLVE: scores back to the requesters (the reverse exchange)
        if (d->loopback) {
            for (size_t i = 0; i < d->ranks.size(); i++)          // requester i
                for (size_t j = 0; j < d->ranks.size(); j++) {    // owner j
                    uint64_t n = lay[i].send_off[j + 1] - lay[i].send_off[j];
                    if (n) GM_HIP(hipMemcpyAsync(d->ranks[i].reply_in + lay[i].send_off[j],
                                                 d->ranks[j].reply_out + lay[j].recv_off[i], n * 2,
                                                 hipMemcpyDeviceToDevice, c->stream));
                }
        } else {
            Xch x{c, d};
            GM_TRY(x.sendrecv(d->ranks[0], d->ranks[0].reply_out, lay[0].recv_off.data(), d->ranks[0].reply_in,
                              lay[0].send_off.data(), 2));
        }
        // fold and finalise
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRank &R = d->ranks[i];
            Table &T = R.tiers[t];
            if (T.cap > R.best_cap) {
                if (R.best) (void)hipFree(R.best);
                GM_HIP(hipMalloc(&R.best, T.cap * 4));
                R.best_cap = T.cap;
            }
            GM_HIP(hipMemsetAsync(R.best, 0, T.cap * 4, c->stream));
            if (lay[i].nsend)
                hipLaunchKernelGGL(fold_kernel, dim3(grid_for(lay[i].nsend)), dim3(256), 0, c->stream, R.reply_in,
                                   R.sendp, lay[i].nsend, R.best);
            hipLaunchKernelGGL(finalize_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.keys, T.score,
                               R.best, T.cap, R.d_err);
        }
        GM_TRY(check_err(c, d));
    }
    double t2 = now_ms();
    for (auto p : dcnt) (void)hipFree(p);

    // root record: owner's score, max-reduced
    uint32_t rs = 0;
    for (auto &R : d->ranks) {
        if ((int)owner_rank(root, G) != R.rank) continue;
        TableRef tr = ref(R.tiers[0], nullptr);
        uint64_t *dk;
        uint16_t *dv;
        GM_HIP(hipMalloc(&dk, 8));
        GM_HIP(hipMalloc(&dv, 2));
        GM_HIP(hipMemcpyAsync(dk, &root, 8, hipMemcpyHostToDevice, c->stream));
        hipLaunchKernelGGL(lookup_kernel, dim3(1), dim3(64), 0, c->stream, dk, 1, tr, dv, R.d_err);
        uint16_t v;
        GM_HIP(hipMemcpyAsync(&v, dv, 2, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(dk);
        (void)hipFree(dv);
        rs = v;
    }
    if (!d->loopback) {
        GM_HIP(hipMemcpyAsync(d->d_root, &rs, 4, hipMemcpyHostToDevice, c->stream));
        GM_NCCL(ncclAllReduce(d->d_root, d->d_root, 1, ncclUint32, ncclMax, c->comm, c->stream));
        GM_HIP(hipMemcpyAsync(&rs, d->d_root, 4, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
    }
    c->root_record = record_of_score((uint16_t)rs);
    uint64_t n = 0;
    for (auto v : d->global_tier_counts) n += v;
    c->n_positions = n;
    c->tier_counts = d->global_tier_counts;
    c->stats.n_positions = n;
    c->stats.n_tiers = (int32_t)d->global_tier_counts.size();
    c->stats.world = G;
    c->stats.forward_ms = t1 - t0;
    c->stats.backward_ms = t2 - t1;
    c->stats.solve_ms = t2 - t0;
    c->stats.exchanged_bytes = d->sent_bytes;
    uint64_t tb = 0;
    for (auto &R : d->ranks)
        for (auto &T : R.tiers) tb += T.cap * 10;
    c->stats.table_bytes = tb;
    return GM_OK;
}

int dist_sparse_solve(Ctx *c, uint64_t root) {
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: return solve_sharded(c, c->f2o, root);
    case GM_GAME_TTT: return solve_sharded(c, c->ttt, root);
    case GM_GAME_TOOT: return solve_sharded(c, c->toot, root);
    case GM_GAME_OTHELLO: return solve_sharded(c, c->oth, root);
    case GM_GAME_SUBTRACT: return solve_sharded(c, c->sub, root);
    }
    set_error("unknown game");
    return GM_E_GAME;
}

int dist_sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DistSparse *d = c->dist_sp;
    uint64_t total = 0;
    for (auto &R : d->ranks)
        for (auto &T : R.tiers) total += T.count;
    *n = total;
    if (!keys) return GM_OK;
    if (cap < total) { set_error("export buffer too small"); return GM_E_CAP; }
    uint64_t *dk;
    uint16_t *dr;
    unsigned long long *cur;
    GM_HIP(hipMalloc(&dk, std::max<uint64_t>(1, total) * 8));
    GM_HIP(hipMalloc(&dr, std::max<uint64_t>(1, total) * 2));
    GM_HIP(hipMalloc(&cur, 8));
    GM_HIP(hipMemsetAsync(cur, 0, 8, c->stream));
    for (auto &R : d->ranks)
        for (auto &T : R.tiers)
            if (T.count)
                hipLaunchKernelGGL(gather_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.keys, T.score,
                                   T.cap, dk, dr, cur);
    std::vector<uint64_t> hk(total);
    std::vector<uint16_t> hr(total);
    GM_HIP(hipMemcpyAsync(hk.data(), dk, total * 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipMemcpyAsync(hr.data(), dr, total * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    (void)hipFree(cur);
    std::vector<uint64_t> idx(total);
    for (uint64_t i = 0; i < total; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) { return hk[a] < hk[b]; });
    for (uint64_t i = 0; i < total; i++) { keys[i] = hk[idx[i]]; recs[i] = hr[idx[i]]; }
    return GM_OK;
}

int dist_sparse_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DistSparse *d = c->dist_sp;
    unsigned long long *acc;
    GM_HIP(hipMalloc(&acc, 8));
    GM_HIP(hipMemsetAsync(acc, 0, 8, c->stream));
    uint64_t total = 0;
    for (auto &R : d->ranks)
        for (auto &T : R.tiers) {
            total += T.count;
            if (T.count)
                hipLaunchKernelGGL(digest_kernel, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, T.keys, T.score,
                                   T.cap, acc);
        }
    unsigned long long h;
    GM_HIP(hipMemcpyAsync(&h, acc, 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(acc);
    *digest = h;
    *n = total;
    return GM_OK;
}

int dist_sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    // host-side probe of the owner's tier tables (tests and the CLI's single lookups)
    DistSparse *d = c->dist_sp;
    for (uint64_t i = 0; i < n; i++) {
        recs[i] = REC_UNSOLVED;
        uint32_t own = owner_rank(keys[i], d->G);
        for (auto &R : d->ranks) {
            if ((uint32_t)R.rank != own) continue;
            for (auto &T : R.tiers) {
                if (!T.cap) continue;
                uint64_t h = mix64(keys[i]) & (T.cap - 1);
                for (uint64_t p = 0; p < T.cap; p++) {
                    uint64_t k;
                    GM_HIP(hipMemcpy(&k, T.keys + h, 8, hipMemcpyDeviceToHost));
                    if (k == EMPTY_KEY) break;
                    if (k == keys[i]) {
                        uint16_t s;
                        GM_HIP(hipMemcpy(&s, T.score + h, 2, hipMemcpyDeviceToHost));
                        recs[i] = record_of_score(s);
                        break;
                    }
                    h = (h + 1) & (T.cap - 1);
                }
            }
        }
    }
    return GM_OK;
}

void dist_sparse_free(Ctx *c) {
    DistSparse *d = c->dist_sp;
    if (!d) return;
    for (auto &R : d->ranks) {
        for (auto &T : R.tiers) free_table(T);
        for (void *p : {(void *)R.d_err, (void *)R.d_hist, (void *)R.d_cursor, (void *)R.d_seg, (void *)R.d_acc,
                        (void *)R.sendk, (void *)R.recvk, (void *)R.sendp, (void *)R.reply_out,
                        (void *)R.reply_in, (void *)R.best})
            if (p) (void)hipFree(p);
    }
    if (d->d_mat) (void)hipFree(d->d_mat);
    if (d->d_root) (void)hipFree(d->d_root);
    delete d;
    c->dist_sp = nullptr;
}

}  // namespace gm
