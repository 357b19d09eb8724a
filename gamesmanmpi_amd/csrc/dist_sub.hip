// dist_sub.hip -- the dense subtraction solve partitioned over G = 2, 4 or 8 ranks.
//
// Ownership ("block owner"): with LOW heaps inside a block, the g =
// log2 G top heaps are split in halves; rank bit a says whether heap (heaps-1-a)
// of the rank's blocks is >= 8.  The reference hashes every position to an
// owner (GameState.get_hash, src/game_state.py:23-31) and sends one message per
// edge (src/new_process.py:159,186); here a move changes one heap by 1 or 2, so a
// block's children live on its own rank except across a split heap, where the
// upper rank needs the two layers h = 6, 7 of its lower neighbour: a halo of
// <= 25 % of a rank per split heap, exchanged once per tier.
//
// Per tier t, on every rank:
//   exchange  lower neighbours' tier-(t-1) boundary blocks arrive (ncclRecv) while
//             this rank's tier-(t-1) boundary blocks leave (ncclSend), on a comm
//             stream, one ncclGroup per tier (point-to-point over xGMI);
//   compute A the blocks of tier t that need nothing from tier t-1 across a split
//             (overlaps the exchange);
//   unpack    the received halo into the table (global key layout on every rank);
//   compute B the blocks whose split heap is 8 (they read the fresh halo);
//   pack      this rank's tier-t boundary blocks for the next exchange.
// Ranks never synchronise globally inside a solve: each waits only for its
// neighbours' halo, so a rank whose blocks sit in later tiers trails its lower
// neighbours by a tier instead of idling at a barrier.
//
// Transports: RCCL (one process per GPU, gm_set_comm) or loopback (G virtual
// ranks inside one context on one GPU, halos moved by device copies) -- the same
// partition, lists, kernels and order of operations, so the loopback mode makes
// the sharded path parity-testable on a single GPU.
#include "gm_internal.hpp"

#include <algorithm>

namespace gm {

struct SubRank {
    int rank = 0;
    uint16_t *table = nullptr;
    bool owned = false;
    std::vector<uint32_t> offA, offB;          // per-tier offsets into listA / listB
    uint32_t *dA = nullptr, *dB = nullptr;
    std::vector<uint32_t> send_off[3], recv_off[3];
    uint32_t *dsend[3] = {nullptr, nullptr, nullptr}, *drecv[3] = {nullptr, nullptr, nullptr};
    uint16_t *sendbuf[3][2] = {}, *recvbuf[3][2] = {};
    uint64_t own_blocks = 0;
};

struct DistSub {
    int heaps = 0, low = 0, high = 0, g = 0, G = 1, ntiers = 0;
    bool loopback = false;
    std::vector<SubRank> ranks;
    uint16_t *zero = nullptr;
    uint64_t *d_acc = nullptr;
    uint32_t *d_root = nullptr;
    hipEvent_t ev_packed[2] = {}, ev_recv[2] = {};
    std::vector<hipEvent_t> ev;                // timing
};

static inline int nib(uint64_t v, int k) { return (int)((v >> (4 * k)) & 15u); }

// rank owning high part H (axis a = high nibble high-1-a)
static inline int owner_of(const DistSub *d, uint64_t H) {
    int r = 0;
    for (int a = 0; a < d->g; a++)
        if (nib(H, d->high - 1 - a) >= 8) r |= 1 << a;
    return r;
}

__global__ void block_copy_kernel(const uint16_t *__restrict__ src, const uint32_t *__restrict__ list,
                                  uint16_t *__restrict__ dst, int low, int pack) {
    typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
    const uint64_t bsz = 1ull << (4 * low);
    const uint64_t blk = (uint64_t)list[blockIdx.x] << (4 * low);
    const uint64_t stg = (uint64_t)blockIdx.x * bsz;
    for (uint64_t c = threadIdx.x; c < bsz / 8; c += blockDim.x) {
        if (pack)
            *(u16x8 *)(dst + stg + 8 * c) = *(const u16x8 *)(src + blk + 8 * c);
        else
            *(u16x8 *)(dst + blk + 8 * c) = *(const u16x8 *)(src + stg + 8 * c);
    }
}

static int upload(const std::vector<uint32_t> &v, uint32_t **d) {
    GM_HIP(hipMalloc(d, std::max<size_t>(1, v.size()) * 4));
    if (!v.empty()) GM_HIP(hipMemcpy(*d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    return GM_OK;
}

// Build rank r's block lists (identical enumeration on every rank).
static int build_rank(Ctx *c, DistSub *d, SubRank &R) {
    const int T = d->ntiers;
    const uint64_t nhigh = 1ull << (4 * d->high);
    auto tsum = [&](uint64_t H) { int s = 0; for (int k = 0; k < d->high; k++) s += nib(H, k); return s; };
    std::vector<std::vector<uint32_t>> A(T), B(T), S[3], Rv[3];
    for (int a = 0; a < 3; a++) { S[a].resize(T); Rv[a].resize(T); }
    for (uint64_t H = 0; H < nhigh; H++) {
        int own = owner_of(d, H), t = tsum(H);
        if (own == R.rank) {
            bool needs = false;
            for (int a = 0; a < d->g; a++)
                if (((R.rank >> a) & 1) && nib(H, d->high - 1 - a) == 8) needs = true;
            (needs ? B : A)[t].push_back((uint32_t)H);
            R.own_blocks++;
            for (int a = 0; a < d->g; a++) {
                int h = nib(H, d->high - 1 - a);
                if (!((R.rank >> a) & 1) && (h == 6 || h == 7)) S[a][t].push_back((uint32_t)H);
            }
        } else {
            for (int a = 0; a < d->g; a++) {
                int h = nib(H, d->high - 1 - a);
                if (((R.rank >> a) & 1) && own == (R.rank ^ (1 << a)) && (h == 6 || h == 7))
                    Rv[a][t].push_back((uint32_t)H);
            }
        }
    }
    auto flatten = [&](std::vector<std::vector<uint32_t>> &L, std::vector<uint32_t> &off, uint32_t **dptr,
                       size_t *maxn) -> int {
        std::vector<uint32_t> flat;
        off.assign(T + 1, 0);
        size_t mx = 0;
        for (int t = 0; t < T; t++) {
            off[t] = (uint32_t)flat.size();
            flat.insert(flat.end(), L[t].begin(), L[t].end());
            mx = std::max(mx, L[t].size());
        }
        off[T] = (uint32_t)flat.size();
        if (maxn) *maxn = mx;
        return upload(flat, dptr);
    };
    GM_TRY(flatten(A, R.offA, &R.dA, nullptr));
    GM_TRY(flatten(B, R.offB, &R.dB, nullptr));
    const uint64_t bbytes = 2ull << (4 * d->low);
    for (int a = 0; a < d->g; a++) {
        size_t ms = 0, mr = 0;
        GM_TRY(flatten(S[a], R.send_off[a], &R.dsend[a], &ms));
        GM_TRY(flatten(Rv[a], R.recv_off[a], &R.drecv[a], &mr));
        for (int p = 0; p < 2; p++) {
            if (ms) GM_HIP(hipMalloc(&R.sendbuf[a][p], ms * bbytes));
            if (mr) GM_HIP(hipMalloc(&R.recvbuf[a][p], mr * bbytes));
        }
    }
    const uint64_t bytes = 2ull << (4 * d->heaps);
    if (!d->loopback && c->adopted_dense) {
        if (c->adopted_dense_bytes < bytes) { set_error("adopted dense table too small"); return GM_E_CAP; }
        R.table = (uint16_t *)c->adopted_dense;
    } else {
        if (hipMalloc(&R.table, bytes) != hipSuccess) {
            set_error("hipMalloc of a %llu-byte rank table failed", (unsigned long long)bytes);
            return GM_E_NOMEM;
        }
        R.owned = true;
    }
    return GM_OK;
}

static int prepare(Ctx *c, DistSub *d, int G, bool loopback) {
    d->heaps = c->sub.heaps;
    d->low = std::min(3, d->heaps);
    d->high = d->heaps - d->low;
    d->G = G;
    d->g = G == 2 ? 1 : G == 4 ? 2 : G == 8 ? 3 : -1;
    d->loopback = loopback;
    if (d->g < 0) { set_error("world size %d: the dense path shards over 2, 4 or 8 ranks", G); return GM_E_ARG; }
    if (d->g > d->high) {
        set_error("%d heaps leave %d block heaps; cannot split %d ways", d->heaps, d->high, G);
        return GM_E_ARG;
    }
    if (!sub_kernel_exists(d->low, d->high)) { set_error("no dense kernel"); return GM_E_GAME; }
    d->ntiers = 15 * d->high + 1;
    size_t zb = 2ull << (4 * d->low);
    GM_HIP(hipMalloc(&d->zero, zb));
    GM_HIP(hipMemset(d->zero, 0, zb));
    GM_HIP(hipMalloc(&d->d_acc, 16));
    GM_HIP(hipMalloc(&d->d_root, 4));
    if (loopback) {
        d->ranks.resize(G);
        for (int r = 0; r < G; r++) { d->ranks[r].rank = r; GM_TRY(build_rank(c, d, d->ranks[r])); }
    } else {
        d->ranks.resize(1);
        d->ranks[0].rank = c->rank;
        GM_TRY(build_rank(c, d, d->ranks[0]));
        for (int p = 0; p < 2; p++) {
            GM_HIP(hipEventCreateWithFlags(&d->ev_packed[p], hipEventDisableTiming));
            GM_HIP(hipEventCreateWithFlags(&d->ev_recv[p], hipEventDisableTiming));
        }
        if (!c->comm_stream) GM_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    }
    return GM_OK;
}

static void copy_blocks(DistSub *d, const uint16_t *src, const uint32_t *list, uint32_t n, uint16_t *dst,
                        bool pack, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(block_copy_kernel, dim3(n), dim3(256), 0, s, src, list, dst, d->low, pack ? 1 : 0);
}

static uint32_t cnt(const std::vector<uint32_t> &off, int t) { return off[t + 1] - off[t]; }

int dist_sub_solve(Ctx *c, uint64_t root) {
    const bool loopback = c->virtual_ranks > 1;
    const int G = loopback ? c->virtual_ranks : c->world;
    DistSub *d = c->dist_sub;
    if (!d || d->heaps != c->sub.heaps || d->G != G || d->loopback != loopback) {
        dist_sub_free(c);
        d = c->dist_sub = new DistSub();
        GM_TRY(prepare(c, d, G, loopback));
    }
    const int T = d->ntiers;
    const uint64_t bbytes = 2ull << (4 * d->low);
    hipStream_t S = c->stream;
    double t0 = now_ms();
    uint64_t sent = 0;
    if (loopback) {
        for (int t = 0; t < T; t++) {
            if (t > 0)   // exchange tier t-1 boundaries: lower neighbour's sendbuf -> my recvbuf
                for (auto &R : d->ranks)
                    for (int a = 0; a < d->g; a++) {
                        if (!((R.rank >> a) & 1)) continue;
                        SubRank &L = d->ranks[R.rank ^ (1 << a)];
                        uint32_t n = cnt(R.recv_off[a], t - 1);
                        if (n != cnt(L.send_off[a], t - 1)) { set_error("halo lists disagree"); return GM_E_STATE; }
                        if (n) GM_HIP(hipMemcpyAsync(R.recvbuf[a][(t - 1) & 1], L.sendbuf[a][(t - 1) & 1],
                                                     n * bbytes, hipMemcpyDeviceToDevice, S));
                        sent += n * bbytes;
                    }
            for (auto &R : d->ranks) {
                launch_sub_tier(d->low, d->high, cnt(R.offA, t), R.table, R.dA + R.offA[t], d->zero, S);
                if (t > 0)
                    for (int a = 0; a < d->g; a++)
                        if ((R.rank >> a) & 1)
                            copy_blocks(d, R.recvbuf[a][(t - 1) & 1], R.drecv[a] + R.recv_off[a][t - 1],
                                        cnt(R.recv_off[a], t - 1), R.table, false, S);
                launch_sub_tier(d->low, d->high, cnt(R.offB, t), R.table, R.dB + R.offB[t], d->zero, S);
                for (int a = 0; a < d->g; a++)
                    if (!((R.rank >> a) & 1))
                        copy_blocks(d, R.table, R.dsend[a] + R.send_off[a][t], cnt(R.send_off[a], t),
                                    R.sendbuf[a][t & 1], true, S);
            }
        }
        GM_HIP(hipGetLastError());
        // root record from its owner
        SubRank &O = d->ranks[owner_of(d, root >> (4 * d->low))];
        uint16_t rs;
        GM_HIP(hipMemcpyAsync(&rs, O.table + root, 2, hipMemcpyDeviceToHost, S));
        GM_HIP(hipStreamSynchronize(S));
        c->root_record = record_of_score(rs);
    } else {
        SubRank &R = d->ranks[0];
        hipStream_t C = c->comm_stream;
        for (int t = 0; t < T; t++) {
            int u = t - 1;   // tier whose boundary is exchanged at this step
            bool any = false;
            if (t > 0) {
                for (int a = 0; a < d->g; a++)
                    any |= ((R.rank >> a) & 1) ? cnt(R.recv_off[a], u) > 0 : cnt(R.send_off[a], u) > 0;
            }
            if (any) {
                GM_HIP(hipStreamWaitEvent(C, d->ev_packed[u & 1], 0));
                GM_NCCL(ncclGroupStart());
                for (int a = 0; a < d->g; a++) {
                    int peer = R.rank ^ (1 << a);
                    if ((R.rank >> a) & 1) {
                        uint32_t n = cnt(R.recv_off[a], u);
                        if (n) GM_NCCL(ncclRecv(R.recvbuf[a][u & 1], n * bbytes, ncclUint8, peer, c->comm, C));
                    } else {
                        uint32_t n = cnt(R.send_off[a], u);
                        if (n) GM_NCCL(ncclSend(R.sendbuf[a][u & 1], n * bbytes, ncclUint8, peer, c->comm, C));
                        sent += n * bbytes;
                    }
                }
                GM_NCCL(ncclGroupEnd());
                GM_HIP(hipEventRecord(d->ev_recv[u & 1], C));
            }
            launch_sub_tier(d->low, d->high, cnt(R.offA, t), R.table, R.dA + R.offA[t], d->zero, S);
            if (any) {
                GM_HIP(hipStreamWaitEvent(S, d->ev_recv[u & 1], 0));
                for (int a = 0; a < d->g; a++)
                    if ((R.rank >> a) & 1)
                        copy_blocks(d, R.recvbuf[a][u & 1], R.drecv[a] + R.recv_off[a][u], cnt(R.recv_off[a], u),
                                    R.table, false, S);
            }
            launch_sub_tier(d->low, d->high, cnt(R.offB, t), R.table, R.dB + R.offB[t], d->zero, S);
            for (int a = 0; a < d->g; a++)
                if (!((R.rank >> a) & 1))
                    copy_blocks(d, R.table, R.dsend[a] + R.send_off[a][t], cnt(R.send_off[a], t),
                                R.sendbuf[a][t & 1], true, S);
            GM_HIP(hipEventRecord(d->ev_packed[t & 1], S));
        }
        GM_HIP(hipGetLastError());
        // root record: max-allreduce of the owner's score (others contribute 0)
        int own = owner_of(d, root >> (4 * d->low)) == R.rank;
        GM_HIP(hipMemsetAsync(d->d_root, 0, 4, S));
        if (own) GM_HIP(hipMemcpyAsync(d->d_root, R.table + root, 2, hipMemcpyDeviceToDevice, S));
        GM_NCCL(ncclAllReduce(d->d_root, d->d_root, 1, ncclUint32, ncclMax, c->comm, S));
        uint32_t rs;
        GM_HIP(hipMemcpyAsync(&rs, d->d_root, 4, hipMemcpyDeviceToHost, S));
        GM_HIP(hipStreamSynchronize(S));
        c->root_record = record_of_score((uint16_t)rs);
    }
    double t1 = now_ms();
    uint64_t n = 1;
    for (int j = 0; j < d->heaps; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = T;
    c->stats.world = G;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.exchanged_bytes = sent;
    uint64_t ownb = 0;
    for (auto &R : d->ranks) ownb += R.own_blocks;
    c->stats.algo_bytes = (uint64_t)((double)(ownb << (4 * d->low)) * 2.0 * (1.0 + 1.8125 * d->heaps));
    c->stats.table_bytes = (2ull << (4 * d->heaps)) * d->ranks.size();
    c->tier_counts.clear();
    return GM_OK;
}

// host copy of the blocks this context owns (one rank, or every virtual rank)
template <class F>
static int for_owned_blocks(Ctx *c, F f) {
    DistSub *d = c->dist_sub;
    const uint64_t bsz = 1ull << (4 * d->low);
    std::vector<uint16_t> buf(bsz);
    const uint64_t nhigh = 1ull << (4 * d->high);
    for (uint64_t H = 0; H < nhigh; H++) {
        int own = owner_of(d, H);
        SubRank *R = nullptr;
        for (auto &x : d->ranks)
            if (x.rank == own) R = &x;
        if (!R) continue;
        GM_HIP(hipMemcpy(buf.data(), R->table + (H << (4 * d->low)), bsz * 2, hipMemcpyDeviceToHost));
        f(H << (4 * d->low), buf.data(), bsz);
    }
    return GM_OK;
}

static bool in_box(uint64_t k, uint64_t root, int heaps) {
    for (int i = 0; i < heaps; i++)
        if (((k >> (4 * i)) & 15u) > ((root >> (4 * i)) & 15u)) return false;
    return true;
}

int dist_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DistSub *d = c->dist_sub;
    uint64_t cntv = 0;
    std::vector<std::pair<uint64_t, uint16_t>> out;
    GM_TRY(for_owned_blocks(c, [&](uint64_t base, const uint16_t *s, uint64_t len) {
        for (uint64_t i = 0; i < len; i++)
            if (in_box(base + i, c->root, d->heaps)) {
                if (keys) out.emplace_back(base + i, record_of_score(s[i]));
                cntv++;
            }
    }));
    *n = cntv;
    if (!keys) return GM_OK;
    if (cap < cntv) { set_error("export buffer too small"); return GM_E_CAP; }
    std::sort(out.begin(), out.end());
    for (uint64_t i = 0; i < cntv; i++) { keys[i] = out[i].first; recs[i] = out[i].second; }
    return GM_OK;
}

int dist_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DistSub *d = c->dist_sub;
    uint64_t s = 0, k = 0;
    GM_TRY(for_owned_blocks(c, [&](uint64_t base, const uint16_t *v, uint64_t len) {
        for (uint64_t i = 0; i < len; i++)
            if (in_box(base + i, c->root, d->heaps)) { s += digest_term(base + i, record_of_score(v[i])); k++; }
    }));
    *digest = s;
    *n = k;
    return GM_OK;
}

int dist_sub_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    DistSub *d = c->dist_sub;
    for (uint64_t i = 0; i < n; i++) {
        recs[i] = REC_UNSOLVED;
        if (keys[i] >> (4 * d->heaps)) continue;
        int own = owner_of(d, keys[i] >> (4 * d->low));
        for (auto &R : d->ranks)
            if (R.rank == own) {
                uint16_t s;
                GM_HIP(hipMemcpy(&s, R.table + keys[i], 2, hipMemcpyDeviceToHost));
                recs[i] = record_of_score(s);
            }
    }
    return GM_OK;
}

void dist_sub_free(Ctx *c) {
    DistSub *d = c->dist_sub;
    if (!d) return;
    for (auto &R : d->ranks) {
        if (R.owned && R.table) hipFree(R.table);
        if (R.dA) hipFree(R.dA);
        if (R.dB) hipFree(R.dB);
        for (int a = 0; a < 3; a++) {
            if (R.dsend[a]) hipFree(R.dsend[a]);
            if (R.drecv[a]) hipFree(R.drecv[a]);
            for (int p = 0; p < 2; p++) {
                if (R.sendbuf[a][p]) hipFree(R.sendbuf[a][p]);
                if (R.recvbuf[a][p]) hipFree(R.recvbuf[a][p]);
            }
        }
    }
    for (int p = 0; p < 2; p++) {
        if (d->ev_packed[p]) hipEventDestroy(d->ev_packed[p]);
        if (d->ev_recv[p]) hipEventDestroy(d->ev_recv[p]);
    }
    if (d->zero) hipFree(d->zero);
    if (d->d_acc) hipFree(d->d_acc);
    if (d->d_root) hipFree(d->d_root);
    delete d;
    c->dist_sub = nullptr;
}

}  // namespace gm
