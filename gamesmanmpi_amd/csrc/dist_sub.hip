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
// Per tier t, on every rank (S = compute stream, C = exchange stream):
//   C  exchange  tier t-1 boundary blocks: ncclRecv from lower neighbours,
//                ncclSend to upper neighbours, one ncclGroup per tier;
//   S  compute A the blocks of tier t that need nothing from tier t-1 across a
//                split (runs while the exchange is in flight);
//   S  unpack    (after the exchange event) the halo into the table;
//   S  compute B the blocks whose split heap is 8 (they read the fresh halo);
//   S  pack      this rank's tier-t boundary blocks into a K-deep ring of send
//                slots (a lower rank can run up to K-1 tiers ahead of its upper
//                neighbours; it waits only when a slot is still being sent).
// There is no global barrier inside a solve: a rank waits only for the halos it
// reads.  Launches are eager (see run_solve).
//
// Transports: RCCL (one process per GPU, gm_set_comm) or loopback (G virtual
// ranks inside one context on one GPU, each with its own S and C streams; the
// receiver's C stream copies from the sender's send slot after the sender's
// pack event).  Same partition, lists, kernels, streams and events; only the
// byte movement differs -- so the loopback mode tests the sharded path on one GPU.
#include "gm_internal.hpp"

#include <algorithm>

namespace gm {

constexpr int KSLOTS = 4;

struct SubRank {
    int rank = 0;
    uint8_t *table = nullptr;           // 1-byte codes (gm_common.hpp)
    bool owned = false;
    std::vector<uint32_t> offA, offB;          // per-tier offsets into listA / listB
    uint32_t *dA = nullptr, *dB = nullptr;
    std::vector<uint32_t> send_off[3], recv_off[3];
    uint32_t *dsend[3] = {nullptr, nullptr, nullptr}, *drecv[3] = {nullptr, nullptr, nullptr};
    uint8_t *sendbuf[3][KSLOTS] = {}, *recvbuf[3][KSLOTS] = {};
    uint64_t own_blocks = 0;
    hipStream_t S = nullptr, C = nullptr;      // loopback: own streams; RCCL: the context's
    bool own_streams = false;
    hipEvent_t ev_packed[KSLOTS] = {}, ev_xch[KSLOTS] = {};
};

struct DistSub {
    int heaps = 0, low = 0, high = 0, g = 0, G = 1, ntiers = 0, nt = 256;
    int want_threads = 0, want_x4 = 0;
    bool loopback = false;
    std::vector<SubRank> ranks;
    uint8_t *zero = nullptr;
    unsigned long long *d_acc = nullptr;
    uint32_t *d_root = nullptr;
    hipEvent_t ev_fork = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
};

static inline int nib(uint64_t v, int k) { return (int)((v >> (4 * k)) & 15u); }

// rank owning high part H (axis a = high nibble high-1-a)
static inline int owner_of(const DistSub *d, uint64_t H) {
    int r = 0;
    for (int a = 0; a < d->g; a++)
        if (nib(H, d->high - 1 - a) >= 8) r |= 1 << a;
    return r;
}

__global__ void block_copy_kernel(const uint8_t *__restrict__ src, const uint32_t *__restrict__ list,
                                  uint8_t *__restrict__ dst, int low, int pack) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t bsz = 1ull << (4 * low);
    const uint64_t blk = (uint64_t)list[blockIdx.x] << (4 * low);
    const uint64_t stg = (uint64_t)blockIdx.x * bsz;
    if (bsz >= 16) {
        for (uint64_t c = threadIdx.x; c < bsz / 16; c += blockDim.x) {
            if (pack)
                *(u32x4 *)(dst + stg + 16 * c) = *(const u32x4 *)(src + blk + 16 * c);
            else
                *(u32x4 *)(dst + blk + 16 * c) = *(const u32x4 *)(src + stg + 16 * c);
        }
    } else {
        for (uint64_t c = threadIdx.x; c < bsz; c += blockDim.x) {
            if (pack) dst[stg + c] = src[blk + c];
            else dst[blk + c] = src[stg + c];
        }
    }
}

// digest over a list of whole blocks, restricted to the root's box
__global__ void block_digest_kernel(const uint8_t *__restrict__ table, const uint32_t *__restrict__ list,
                                    uint64_t nblocks, int low, int heaps, uint64_t root,
                                    unsigned long long *acc) {
    const uint64_t bsz = 1ull << (4 * low);
    uint64_t s = 0, k = 0;
    for (uint64_t b = blockIdx.x; b < nblocks; b += gridDim.x) {
        const uint64_t base = (uint64_t)list[b] << (4 * low);
        for (uint64_t i = threadIdx.x; i < bsz; i += blockDim.x) {
            uint64_t key = base + i;
            bool in = true;
            for (int j = 0; j < heaps; j++) in &= ((key >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
            if (!in) continue;
            s += digest_term(key, record_of_code(table[key]));
            k++;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        k += __shfl_xor(k, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(acc, (unsigned long long)s);
        atomicAdd(acc + 1, (unsigned long long)k);
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
    std::vector<std::vector<uint32_t>> A(T), B(T), Sd[3], Rv[3];
    for (int a = 0; a < 3; a++) { Sd[a].resize(T); Rv[a].resize(T); }
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
                if (!((R.rank >> a) & 1) && (h == 6 || h == 7)) Sd[a][t].push_back((uint32_t)H);
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
    const uint64_t bbytes = 1ull << (4 * d->low);
    for (int a = 0; a < d->g; a++) {
        size_t ms = 0, mr = 0;
        GM_TRY(flatten(Sd[a], R.send_off[a], &R.dsend[a], &ms));
        GM_TRY(flatten(Rv[a], R.recv_off[a], &R.drecv[a], &mr));
        for (int p = 0; p < KSLOTS; p++) {
            if (ms) GM_HIP(hipMalloc(&R.sendbuf[a][p], ms * bbytes));
            if (mr) GM_HIP(hipMalloc(&R.recvbuf[a][p], mr * bbytes));
        }
    }
    for (int p = 0; p < KSLOTS; p++) {
        GM_HIP(hipEventCreateWithFlags(&R.ev_packed[p], hipEventDisableTiming));
        GM_HIP(hipEventCreateWithFlags(&R.ev_xch[p], hipEventDisableTiming));
    }
    const uint64_t bytes = 1ull << (4 * d->heaps);
    if (!d->loopback && c->adopted_dense) {
        if (c->adopted_dense_bytes < bytes) { set_error("adopted dense table too small"); return GM_E_CAP; }
        R.table = (uint8_t *)c->adopted_dense;
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
    d->nt = sub_kernel_threads(c, d->low);
    d->want_threads = c->sub_threads;
    d->want_x4 = c->sub_interleave;
    if (!sub_kernel_exists(d->low, d->high, d->nt)) { set_error("no dense kernel"); return GM_E_GAME; }
    d->ntiers = 15 * d->high + 1;
    size_t zb = std::max<size_t>(16, 1ull << (4 * d->low));
    GM_HIP(hipMalloc(&d->zero, zb));
    GM_HIP(hipMemset(d->zero, 0, zb));
    GM_HIP(hipMalloc(&d->d_acc, 16));
    GM_HIP(hipMalloc(&d->d_root, 4));
    GM_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    GM_HIP(hipEventCreate(&d->ev_t0));
    GM_HIP(hipEventCreate(&d->ev_t1));
    if (!loopback && !c->comm_stream) GM_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    d->ranks.resize(loopback ? G : 1);
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SubRank &R = d->ranks[i];
        R.rank = loopback ? (int)i : c->rank;
        GM_TRY(build_rank(c, d, R));
        if (loopback) {
            GM_HIP(hipStreamCreateWithFlags(&R.S, hipStreamNonBlocking));
            GM_HIP(hipStreamCreateWithFlags(&R.C, hipStreamNonBlocking));
            R.own_streams = true;
        }
    }
    return GM_OK;
}

static void copy_blocks(DistSub *d, const uint8_t *src, const uint32_t *list, uint32_t n, uint8_t *dst,
                        bool pack, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(block_copy_kernel, dim3(n), dim3(256), 0, s, src, list, dst, d->low, pack ? 1 : 0);
}

static uint32_t cnt(const std::vector<uint32_t> &off, int t) {
    return (t < 0 || t + 1 >= (int)off.size()) ? 0 : off[t + 1] - off[t];
}
static bool is_upper(const SubRank &R, int a) { return (R.rank >> a) & 1; }

// Enqueue one whole solve on the ranks' streams (eager or under capture).
// S/C of every rank must already be joined to the capture when capturing.
static int enqueue_solve(Ctx *c, DistSub *d, uint64_t *sent) {
    const int T = d->ntiers, K = KSLOTS;
    const uint64_t bbytes = 1ull << (4 * d->low);
    *sent = 0;
    for (int t = 0; t < T; t++) {
        const int u = t - 1;   // tier whose boundary is exchanged at this step
        // ---- C: exchange tier u
        for (auto &R : d->ranks) {
            bool any = false;
            for (int a = 0; a < d->g; a++) any |= cnt(is_upper(R, a) ? R.recv_off[a] : R.send_off[a], u) > 0;
            if (!any) continue;
            GM_HIP(hipStreamWaitEvent(R.C, R.ev_packed[u % K], 0));   // my step u done (send data, recv slot)
            if (d->loopback) {
                for (int a = 0; a < d->g; a++) {
                    if (!is_upper(R, a)) continue;
                    uint32_t n = cnt(R.recv_off[a], u);
                    if (!n) continue;
                    SubRank &L = d->ranks[R.rank ^ (1 << a)];
                    if (n != cnt(L.send_off[a], u)) { set_error("halo lists disagree"); return GM_E_STATE; }
                    GM_HIP(hipStreamWaitEvent(R.C, L.ev_packed[u % K], 0));
                    GM_HIP(hipMemcpyAsync(R.recvbuf[a][u % K], L.sendbuf[a][u % K], n * bbytes,
                                          hipMemcpyDeviceToDevice, R.C));
                    *sent += n * bbytes;
                }
            } else {
                GM_NCCL(ncclGroupStart());
                for (int a = 0; a < d->g; a++) {
                    int peer = R.rank ^ (1 << a);
                    if (is_upper(R, a)) {
                        uint32_t n = cnt(R.recv_off[a], u);
                        if (n) GM_NCCL(ncclRecv(R.recvbuf[a][u % K], n * bbytes, ncclUint8, peer, c->comm, R.C));
                    } else {
                        uint32_t n = cnt(R.send_off[a], u);
                        if (n) GM_NCCL(ncclSend(R.sendbuf[a][u % K], n * bbytes, ncclUint8, peer, c->comm, R.C));
                        *sent += n * bbytes;
                    }
                }
                GM_NCCL(ncclGroupEnd());
            }
            GM_HIP(hipEventRecord(R.ev_xch[u % K], R.C));
        }
        // ---- S: compute, unpack, compute, pack
        for (auto &R : d->ranks) {
            launch_sub_tier(d->low, d->high, d->nt, cnt(R.offA, t), R.table, R.dA + R.offA[t], d->zero, R.S);
            bool recv = false;
            for (int a = 0; a < d->g; a++) recv |= is_upper(R, a) && cnt(R.recv_off[a], u) > 0;
            if (recv) {
                GM_HIP(hipStreamWaitEvent(R.S, R.ev_xch[u % K], 0));
                for (int a = 0; a < d->g; a++)
                    if (is_upper(R, a))
                        copy_blocks(d, R.recvbuf[a][u % K], R.drecv[a] + R.recv_off[a][u], cnt(R.recv_off[a], u),
                                    R.table, false, R.S);
            }
            launch_sub_tier(d->low, d->high, d->nt, cnt(R.offB, t), R.table, R.dB + R.offB[t], d->zero, R.S);
            // slot t % K last carried tier t-K, exchanged at step t-K+1: wait until it has left
            for (int a = 0; a < d->g; a++) {
                if (is_upper(R, a) || !cnt(R.send_off[a], t)) continue;
                if (cnt(R.send_off[a], t - K) > 0) {
                    if (d->loopback)
                        GM_HIP(hipStreamWaitEvent(R.S, d->ranks[R.rank ^ (1 << a)].ev_xch[(t - K) % K], 0));
                    else
                        GM_HIP(hipStreamWaitEvent(R.S, R.ev_xch[(t - K) % K], 0));
                }
                copy_blocks(d, R.table, R.dsend[a] + R.send_off[a][t], cnt(R.send_off[a], t), R.sendbuf[a][t % K],
                            true, R.S);
            }
            GM_HIP(hipEventRecord(R.ev_packed[t % K], R.S));
        }
    }
    // join every exchange stream back into its compute stream
    for (auto &R : d->ranks) {
        GM_HIP(hipEventRecord(R.ev_xch[0], R.C));
        GM_HIP(hipStreamWaitEvent(R.S, R.ev_xch[0], 0));
    }
    return GM_OK;
}

// Run one solve: fork every rank's streams off the caller's stream, enqueue, join.
// Launches are eager: HIP 7.2's stream capture crashes on this multi-stream event
// pattern (tools/diag_dist.py), and in RCCL mode a capture refused half-way would
// leave the ranks' point-to-point sequence numbers out of step.
static int run_solve(Ctx *c, DistSub *d, uint64_t *sent) {
    hipStream_t H = c->stream;
    if (!d->loopback) { d->ranks[0].S = c->stream; d->ranks[0].C = c->comm_stream; }
    // eager
    GM_HIP(hipEventRecord(d->ev_fork, H));
    for (auto &R : d->ranks) {
        if (R.S != H) GM_HIP(hipStreamWaitEvent(R.S, d->ev_fork, 0));
        GM_HIP(hipStreamWaitEvent(R.C, d->ev_fork, 0));
    }
    GM_TRY(enqueue_solve(c, d, sent));
    for (auto &R : d->ranks)
        if (R.S != H) {
            GM_HIP(hipEventRecord(R.ev_packed[0], R.S));
            GM_HIP(hipStreamWaitEvent(H, R.ev_packed[0], 0));
        }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

int dist_sub_solve(Ctx *c, uint64_t root) {
    const bool loopback = c->virtual_ranks > 1;
    const int G = loopback ? c->virtual_ranks : c->world;
    DistSub *d = c->dist_sub;
    if (!d || d->heaps != c->sub.heaps || d->G != G || d->loopback != loopback || d->want_threads != c->sub_threads || d->want_x4 != c->sub_interleave ||
        (!loopback && c->adopted_dense && d->ranks[0].table != c->adopted_dense)) {
        dist_sub_free(c);
        d = c->dist_sub = new DistSub();
        GM_TRY(prepare(c, d, G, loopback));
    }
    hipStream_t H = c->stream;
    double t0 = now_ms();
    uint64_t sent = 0;
    GM_HIP(hipEventRecord(d->ev_t0, H));
    GM_TRY(run_solve(c, d, &sent));
    GM_HIP(hipEventRecord(d->ev_t1, H));
    // root record: max over ranks of the owner's code (the others contribute 0)
    GM_HIP(hipMemsetAsync(d->d_root, 0, 4, H));
    for (auto &R : d->ranks)
        if (owner_of(d, root >> (4 * d->low)) == R.rank)
            GM_HIP(hipMemcpyAsync(d->d_root, R.table + root, 1, hipMemcpyDeviceToDevice, H));
    if (!loopback) GM_NCCL(ncclAllReduce(d->d_root, d->d_root, 1, ncclUint32, ncclMax, c->comm, H));
    uint32_t rs = 0;
    GM_HIP(hipMemcpyAsync(&rs, d->d_root, 4, hipMemcpyDeviceToHost, H));
    GM_HIP(hipStreamSynchronize(H));
    double t1 = now_ms();
    c->root_record = record_of_code((uint8_t)rs);
    uint64_t n = 1;
    for (int j = 0; j < d->heaps; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = d->ntiers;
    c->stats.world = G;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.exchanged_bytes = sent;
    if (c->timing) {
        float ms = 0;
        GM_HIP(hipEventElapsedTime(&ms, d->ev_t0, d->ev_t1));
        c->stats.kernel_ms = ms;
        uint32_t launches = 0;
        for (auto &R : d->ranks)
            for (int t = 0; t < d->ntiers; t++) launches += (cnt(R.offA, t) > 0) + (cnt(R.offB, t) > 0);
        c->stats.kernel_launches = (int32_t)launches;
    }
    uint64_t ownb = 0;
    for (auto &R : d->ranks) ownb += R.own_blocks;
    c->stats.algo_bytes = (uint64_t)((double)(ownb << (4 * d->low)) * (1.0 + 1.8125 * d->heaps));
    c->stats.table_bytes = (1ull << (4 * d->heaps)) * d->ranks.size();
    c->tier_counts.clear();
    return GM_OK;
}

// ---------------------------------------------------------------- results
static bool in_box(uint64_t k, uint64_t root, int heaps) {
    for (int i = 0; i < heaps; i++)
        if (((k >> (4 * i)) & 15u) > ((root >> (4 * i)) & 15u)) return false;
    return true;
}

int dist_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DistSub *d = c->dist_sub;
    hipStream_t H = c->stream;
    GM_HIP(hipMemsetAsync(d->d_acc, 0, 16, H));
    for (auto &R : d->ranks) {
        uint32_t na = R.offA.back(), nb = R.offB.back();
        if (na) hipLaunchKernelGGL(block_digest_kernel, dim3(std::min<uint32_t>(na, 8192)), dim3(256), 0, H, R.table,
                                   R.dA, (uint64_t)na, d->low, d->heaps, c->root, d->d_acc);
        if (nb) hipLaunchKernelGGL(block_digest_kernel, dim3(std::min<uint32_t>(nb, 8192)), dim3(256), 0, H, R.table,
                                   R.dB, (uint64_t)nb, d->low, d->heaps, c->root, d->d_acc);
    }
    unsigned long long h[2];
    GM_HIP(hipMemcpyAsync(h, d->d_acc, 16, hipMemcpyDeviceToHost, H));
    GM_HIP(hipStreamSynchronize(H));
    *digest = h[0];
    *n = h[1];
    return GM_OK;
}

int dist_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DistSub *d = c->dist_sub;
    hipStream_t H = c->stream;
    const uint64_t bsz = 1ull << (4 * d->low);
    std::vector<std::pair<uint64_t, uint16_t>> out;
    uint64_t total = 0;
    for (auto &R : d->ranks) {
        for (int which = 0; which < 2; which++) {
            uint32_t nb = which ? R.offB.back() : R.offA.back();
            const uint32_t *lst = which ? R.dB : R.dA;
            if (!nb) continue;
            uint8_t *stg;
            GM_HIP(hipMalloc(&stg, (uint64_t)nb * bsz));
            copy_blocks(d, R.table, lst, nb, stg, true, H);
            std::vector<uint8_t> hs((uint64_t)nb * bsz);
            std::vector<uint32_t> hl(nb);
            GM_HIP(hipMemcpyAsync(hs.data(), stg, hs.size(), hipMemcpyDeviceToHost, H));
            GM_HIP(hipMemcpyAsync(hl.data(), lst, nb * 4, hipMemcpyDeviceToHost, H));
            GM_HIP(hipStreamSynchronize(H));
            (void)hipFree(stg);
            for (uint32_t b = 0; b < nb; b++)
                for (uint64_t i = 0; i < bsz; i++) {
                    uint64_t key = ((uint64_t)hl[b] << (4 * d->low)) + i;
                    if (!in_box(key, c->root, d->heaps)) continue;
                    total++;
                    if (keys) out.emplace_back(key, record_of_code(hs[(uint64_t)b * bsz + i]));
                }
        }
    }
    *n = total;
    if (!keys) return GM_OK;
    if (cap < total) { set_error("export buffer too small"); return GM_E_CAP; }
    std::sort(out.begin(), out.end());
    for (uint64_t i = 0; i < total; i++) { keys[i] = out[i].first; recs[i] = out[i].second; }
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
                uint8_t s;
                GM_HIP(hipMemcpy(&s, R.table + keys[i], 1, hipMemcpyDeviceToHost));
                recs[i] = record_of_code(s);
            }
    }
    return GM_OK;
}

void dist_sub_free(Ctx *c) {
    DistSub *d = c->dist_sub;
    if (!d) return;
    for (auto &R : d->ranks) {
        if (R.owned && R.table) (void)hipFree(R.table);
        if (R.dA) (void)hipFree(R.dA);
        if (R.dB) (void)hipFree(R.dB);
        for (int a = 0; a < 3; a++) {
            if (R.dsend[a]) (void)hipFree(R.dsend[a]);
            if (R.drecv[a]) (void)hipFree(R.drecv[a]);
            for (int p = 0; p < KSLOTS; p++) {
                if (R.sendbuf[a][p]) (void)hipFree(R.sendbuf[a][p]);
                if (R.recvbuf[a][p]) (void)hipFree(R.recvbuf[a][p]);
            }
        }
        for (int p = 0; p < KSLOTS; p++) {
            if (R.ev_packed[p]) (void)hipEventDestroy(R.ev_packed[p]);
            if (R.ev_xch[p]) (void)hipEventDestroy(R.ev_xch[p]);
        }
        if (R.own_streams) {
            (void)hipStreamDestroy(R.S);
            (void)hipStreamDestroy(R.C);
        }
    }
    for (hipEvent_t e : {d->ev_fork, d->ev_t0, d->ev_t1})
        if (e) (void)hipEventDestroy(e);
    if (d->zero) (void)hipFree(d->zero);
    if (d->d_acc) (void)hipFree(d->d_acc);
    if (d->d_root) (void)hipFree(d->d_root);
    delete d;
    c->dist_sub = nullptr;
}

}  // namespace gm
