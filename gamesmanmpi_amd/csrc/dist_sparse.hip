// dist_sparse.hip -- the sparse engine hash-sharded over G ranks (Othello, Toot, ...).
//
// Every position has one owner, owner_rank(key) = (mix64(key) >> 32) % G
// (the role of GameState.get_hash, reference src/game_state.py:23-31).  The
// reference sends one pickled Job per edge: LOOK_UP to the child's owner
// (src/new_process.py:159) and RESOLVE back to the parent's rank (:186).  Here
// both are batched per tier into bulk-synchronous exchanges over the same
// per-tier tables as the single-GPU engine (sparse_tables.hpp):
//
// forward, tier t:   each rank classifies its tier-t table (one primitive()
//                    per position, scored in place; interior list), and generates its interior positions' children,
//                    bucketed by (owner, tier step) through an LDS histogram;
//                    counts are all-gathered; keys move with one ncclGroup of
//                    send/recv per peer; owners insert them into their tier
//                    tables (deduplicating on insert).
// backward, tier t:  the owners look up again the keys they received in the
//                    forward exchange of tier t (kept per tier, as each sender
//                    keeps the parent of every key it sent) and answer with the
//                    u16 scores in the same order (RESOLVE); per chunk of 256
//                    parents the scores meet in LDS (max) and each best becomes
//                    its parent's score (gm_common.hpp).  So the backward pass
//                    makes no move and sends no key: the LOOK_UP of a child
//                    happened once, forward.
//
// Exchanges use one of three transports:
//   RCCL (GM_OPT_SPARSE_TRANSPORT 0, one process per GPU): counts all-gathered, keys and
//     replies as one ncclGroup of send/recv per peer, totals all-reduced;
//   IPC (GM_OPT_SPARSE_TRANSPORT 1, one process per rank on one node, ranks may share a GPU):
//     each rank publishes the HIP IPC handle of one fixed exchange window in a POSIX
//     shared-memory segment; per round the senders copy the next part of their send buffers
//     into their windows, a host barrier, each receiver PULLS its pieces out of the peers'
//     windows (a copy kernel reading the mapping), a second barrier frees the windows.  Counts,
//     totals and the root record are all-gathered through the same segment (SpIpc below);
//   loopback (GM_OPT_VIRTUAL_RANKS): device copies between G virtual ranks in one context.
// The three share the layout (layout_for): rank r's send segment for p starts at
// lay(r).send_off[p], p's receive segment from r at lay(p).recv_off[r].
#include "sparse_tables.hpp"

#include <array>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace gm {

// ------------------------------------------------------------------ IPC transport
// One segment per solve, /gmsp-<unique id>-<solve number> (identical on every rank: solves are
// collective).  Slot r is written only by rank r.  A barrier is a monotone epoch: rank r
// stores its epoch in slot r, then waits until every slot holds at least it.  The all-gather
// payload is double-buffered by epoch parity: a rank writes buffer k & 1 before barrier k and
// reads it after; it writes that buffer again only after barrier k + 1, which no rank passes
// before every rank has finished reading it.
constexpr int SP_IPC_WORDS = 512;
constexpr double SP_IPC_WAIT_MS = 120e3;
struct SpIpcSlot {
    hipIpcMemHandle_t h[2];          // 0 = the rank's exchange window (exchange_ipc); 1 unused
    uint64_t off[2], gen[2];         // the buffer's offset in its allocation; bumped per new buffer
    uint64_t arrive;                 // barrier epoch reached
    uint64_t failed;                 // the rank left the solve with an error
    uint64_t val[2][SP_IPC_WORDS];   // all-gather payload, by epoch parity
};

struct SpIpc {
    SpIpcSlot *slot = nullptr;
    size_t bytes = 0;
    int G = 0, me = 0;
    uint64_t epoch = 0;
    char name[96] = {};
    void *pub[2] = {};               // what this rank published
    uint64_t gen[2] = {};
    std::vector<uint64_t> pgen[2];   // per peer: the generation mapped
    std::vector<void *> pbase[2];    // per peer: the mapping of that generation's allocation
    // per peer, every allocation mapped in this solve (a peer's buffer can come back from its
    // allocation cache as another kind: one mapping per allocation, closed at the end)
    std::vector<std::vector<std::pair<hipIpcMemHandle_t, void *>>> maps;
};

static int sp_ipc_barrier(SpIpc &X) {
    X.epoch++;
    __atomic_store_n(&X.slot[X.me].arrive, X.epoch, __ATOMIC_RELEASE);
    const double t0 = now_ms();
    for (int r = 0; r < X.G; r++)
        for (unsigned spin = 0; __atomic_load_n(&X.slot[r].arrive, __ATOMIC_ACQUIRE) < X.epoch; spin++) {
            for (int q = 0; q < X.G; q++)
                if (__atomic_load_n(&X.slot[q].failed, __ATOMIC_ACQUIRE)) {
                    set_error("sparse IPC transport: rank %d failed (segment %s)", q, X.name);
                    return GM_E_COMM;
                }
            if (now_ms() - t0 > SP_IPC_WAIT_MS) {
                set_error("sparse IPC transport: rank %d did not reach barrier %llu within %.0f s (segment %s)", r,
                          (unsigned long long)X.epoch, SP_IPC_WAIT_MS / 1e3, X.name);
                return GM_E_COMM;
            }
            if (spin > 64) usleep(spin > 4096 ? 200 : 10);
        }
    return GM_OK;
}

// all[r * n + i] = rank r's mine[i]
static int sp_ipc_allgather(SpIpc &X, const uint64_t *mine, size_t n, uint64_t *all) {
    size_t o = 0;
    do {   // chunks of SP_IPC_WORDS, one barrier each (at least one, so every rank calls alike)
        const size_t k = std::min<size_t>(SP_IPC_WORDS, n - o);
        const int buf = (int)((X.epoch + 1) & 1);
        std::memcpy(X.slot[X.me].val[buf], mine + o, k * 8);
        GM_TRY(sp_ipc_barrier(X));
        for (int r = 0; r < X.G; r++) std::memcpy(all + (size_t)r * n + o, X.slot[r].val[buf], k * 8);
        o += k;
    } while (o < n);
    return GM_OK;
}

static int sp_ipc_open(Ctx *c, SpIpc &X, int G) {
    uint64_t k0, k1;
    std::memcpy(&k0, c->uid, 8);
    std::memcpy(&k1, c->uid + 8, 8);
    snprintf(X.name, sizeof X.name, "/gmsp-%016llx%016llx-%d", (unsigned long long)k0, (unsigned long long)k1,
             c->sparse_solves++);
    X.G = G;
    X.me = c->rank;
    X.bytes = sizeof(SpIpcSlot) * (size_t)G;
    const int fd = shm_open(X.name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) { set_error("shm_open(%s) failed", X.name); return GM_E_COMM; }
    if (ftruncate(fd, (off_t)X.bytes) != 0) {
        close(fd);
        set_error("ftruncate of %s failed", X.name);
        return GM_E_COMM;
    }
    void *m = mmap(nullptr, X.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) { set_error("mmap of %s failed", X.name); return GM_E_COMM; }
    X.slot = (SpIpcSlot *)m;
    for (int k = 0; k < 2; k++) {
        X.pgen[k].assign(G, 0);
        X.pbase[k].assign(G, nullptr);
    }
    X.maps.assign(G, {});
    // every rank has the segment open once this barrier passes: its name can go
    const int rc = sp_ipc_barrier(X);
    if (rc == GM_OK && X.me == 0) shm_unlink(X.name);
    return rc;
}

static void sp_ipc_fail(SpIpc &X) {
    if (X.slot) __atomic_store_n(&X.slot[X.me].failed, 1, __ATOMIC_RELEASE);
}

static void sp_ipc_close(SpIpc &X) {
    for (auto &m : X.maps)
        for (auto &e : m) (void)hipIpcCloseMemHandle(e.second);
    X.maps.clear();
    if (X.slot) munmap(X.slot, X.bytes);
    X.slot = nullptr;
}

// publish this rank's send buffer of kind k (0 keys, 1 replies); the next barrier orders it
static int sp_ipc_publish(SpIpc &X, int k, void *p) {
    if (p == X.pub[k]) return GM_OK;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess ||
        hipIpcGetMemHandle(&X.slot[X.me].h[k], (void *)base) != hipSuccess) {
        (void)hipGetLastError();
        set_error("hipIpcGetMemHandle of rank %d's send buffer failed", X.me);
        return GM_E_COMM;
    }
    X.slot[X.me].off[k] = (uint64_t)((char *)p - (char *)base);
    X.slot[X.me].gen[k] = ++X.gen[k];
    X.pub[k] = p;
    return GM_OK;
}

// rank r's send buffer of kind k, mapped into this process (after the barrier that follows its publish)
static int sp_ipc_peer(SpIpc &X, int r, int k, char **out) {
    const uint64_t g = X.slot[r].gen[k];
    if (!g) { set_error("rank %d published no send buffer", r); return GM_E_COMM; }
    if (X.pgen[k][r] != g) {
        const hipIpcMemHandle_t &h = X.slot[r].h[k];
        void *b = nullptr;
        for (auto &e : X.maps[r])
            if (!std::memcmp(&e.first, &h, sizeof h)) b = e.second;
        if (!b) {
            if (trace_on()) fprintf(stderr, "[gm] ipc rank %d opens rank %d's buffer gen %llu\n", X.me, r,
                                    (unsigned long long)g);
            if (hipIpcOpenMemHandle(&b, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
                (void)hipGetLastError();
                set_error("hipIpcOpenMemHandle of rank %d's send buffer failed", r);
                return GM_E_COMM;
            }
            X.maps[r].emplace_back(h, b);
        }
        X.pbase[k][r] = b;
        X.pgen[k][r] = g;
    }
    *out = (char *)X.pbase[k][r] + X.slot[r].off[k];
    return GM_OK;
}

// Layout of one exchange: mat is G x (G*S), row = source rank, column = dest*S + dt.
struct Layout {
    std::vector<uint64_t> seg;        // send segment bases per bin (dest-major), size G*S
    std::vector<uint64_t> send_off;   // per dest, size G+1
    std::vector<uint64_t> recv_off;   // per source, size G+1 (all dts of that source)
    std::vector<uint64_t> recv_seg;   // per (source, dt) base in the recv buffer, size G*S
    uint64_t nsend = 0, nrecv = 0;
};

template <class K>
struct SpRankT {
    int rank = 0;
    std::vector<SpTierT<K>> tiers;
    unsigned long long *d_cnt = nullptr;     // per-tier frontier counts
    uint32_t *d_err = nullptr;
    unsigned long long *d_hist = nullptr;    // G*S bins
    unsigned long long *d_cursor = nullptr;  // G*S bins
    unsigned long long *d_seg = nullptr;     // G*S bins
    unsigned long long *d_scr = nullptr;     // [0,8) edges by step, [9] interior count, [10] seen, [12] cursor
    K *sendk = nullptr, *recvk = nullptr;    // recvk: the current tier's (kept[t].recvk)
    uint64_t send_cap = 0, rout_cap = 0, rin_cap = 0;
    uint16_t *reply_out = nullptr, *reply_in = nullptr;
    // per tier, from the forward exchange to the backward one
    struct Kept {
        K *recvk = nullptr;          // the keys this rank received as their owner (one rank, one context: sent)
        uint8_t *lp = nullptr;       // per key sent: its parent's index within its chunk of 256 parents
        uint64_t *cbase = nullptr;   // per (chunk, bin): where the chunk's keys for the bin start, send order
        uint32_t *ccnt = nullptr;    // ... and how many there are
        uint64_t *rb = nullptr;      // the receive segments' bounds (insert_bins / lookup_bins)
    };
    std::vector<Kept> kept;
};

// the key-independent part of a sharded solve (c->dist_sp); DistSparseK<K> adds the ranks
struct DistSparse {
    virtual ~DistSparse() = default;
    int G = 1, S = 1;
    bool loopback = false;
    bool ipc = false;                        // GM_OPT_SPARSE_TRANSPORT 1
    bool wide = false;                       // 128-bit keys (DistSparseK<K128>)
    SpIpc X;
    int64_t t_root = 0;
    std::vector<uint64_t> gcount;            // global positions per tier
    size_t cnt_cap = 0;
    unsigned long long *d_mat = nullptr;     // all-gathered G*G*S counts (RCCL mode)
    unsigned long long *d_tot = nullptr;     // per-tier totals, all-reduced (RCCL mode)
    size_t tot_cap = 0;
    uint32_t *d_root = nullptr;
    uint64_t sent_bytes = 0, edges = 0;
    DedupEstimate est;
    char *win = nullptr;                     // IPC: this rank's exchange window (SP_IPC_WIN bytes)
};
template <class K>
struct DistSparseK : DistSparse {
    std::vector<SpRankT<K>> ranks;
    std::vector<std::vector<Layout>> t_lay;      // per tier: every local rank's exchange layout
    std::vector<std::vector<uint64_t>> t_mat;    // per tier: the all-gathered count matrix
};

// ------------------------------------------------------------------ kernels
constexpr int MAXBINS = 64 * 3;

// Children of the interior positions of a tier, bucketed by bin = owner * S + (step - 1).
// COUNT: an LDS histogram over all of the workgroup's chunks, added to hist once at the end
// (atomics on one line serialise: block_add).  SCATTER: per chunk of 256 parents the workgroup
// reserves a range per bin, and a second visit writes the keys; kept for the backward fold are
// each key's parent within its chunk (out_lp, one byte) and each (chunk, bin) range.
template <class D, bool SCATTER>
__global__ __launch_bounds__(256) void bucket_kernel(D d, const key_t<D> *__restrict__ ikeys, uint64_t n, int G,
                                                     unsigned long long *hist,
                                                     const unsigned long long *__restrict__ seg,
                                                     unsigned long long *cursor, key_t<D> *out_keys,
                                                     uint8_t *out_lp, uint64_t *cbase, uint32_t *ccnt,
                                                     uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    using K = key_t<D>;
    __shared__ unsigned int lh[MAXBINS], lh2[MAXBINS];
    __shared__ unsigned long long lbase[MAXBINS];
    const int nb = G * S;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = lh2[b] = 0;
    for (uint64_t base = blockIdx.x * 256ull; base < n; base += (uint64_t)gridDim.x * 256ull) {
        if (SCATTER)
            for (int b = threadIdx.x; b < nb; b += blockDim.x) lh[b] = lh2[b] = 0;
        __syncthreads();
        const uint64_t i = base + threadIdx.x;
        const bool live = i < n;
        K k{};
        if (live) k = ikeys[i];
        const int64_t tk = live ? d.tier(k) : 0;
        // one pass over the children, `emit(c, bin)` for each
        auto walk = [&](auto emit) {
            if (!live) return;
            d.visit(k, [&](const K &c) {
                int64_t dt = d.tier(c) - tk;
                if (dt < 1 || dt > S) { atomicOr(err, DEV_ERR_TIER); dt = 1; }
                emit(c, (int)(owner_rank(c, (uint32_t)G) * S + (dt - 1)));
                return true;
            });
        };
        walk([&](const K &, int bin) { atomicAdd(&lh[bin], 1u); });
        __syncthreads();
        if (SCATTER) {
            const uint64_t k = base / 256;
            for (int b = threadIdx.x; b < nb; b += blockDim.x) {
                lbase[b] = lh[b] ? seg[b] + atomicAdd(&cursor[b], (unsigned long long)lh[b]) : 0ull;
                cbase[k * nb + b] = lbase[b];
                ccnt[k * nb + b] = lh[b];
            }
            __syncthreads();
            walk([&](const K &c, int bin) {
                const unsigned long long at = lbase[bin] + atomicAdd(&lh2[bin], 1u);
                out_keys[at] = c;
                out_lp[at] = (uint8_t)threadIdx.x;
            });
        }
        __syncthreads();
    }
    if (!SCATTER)
        for (int b = threadIdx.x; b < nb; b += blockDim.x)
            if (lh[b]) atomicAdd(&hist[b], (unsigned long long)lh[b]);
}

// Backward fold and finalize of a tier in one pass, one workgroup per chunk of 256 parents: the
// scores that came back for the chunk's keys (contiguous per bin, in send order) meet in LDS,
// and each parent's best child score becomes its own (gm_common.hpp parent_score).
template <class R>
__global__ __launch_bounds__(256) void fold_finalize_kernel(const uint16_t *__restrict__ reply,
                                                            const uint8_t *__restrict__ lp,
                                                            const uint64_t *__restrict__ cbase,
                                                            const uint32_t *__restrict__ ccnt, int nb,
                                                            const uint32_t *__restrict__ islot, uint64_t n, R self,
                                                            uint32_t *err) {
    __shared__ uint32_t best[256];
    const uint64_t nchunks = (n + 255) / 256;
    for (uint64_t k = blockIdx.x; k < nchunks; k += gridDim.x) {
        best[threadIdx.x] = 0;
        __syncthreads();
        for (int b = 0; b < nb; b++) {
            const uint64_t base = cbase[k * nb + b];
            const uint32_t cnt = ccnt[k * nb + b];
            for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x)
                atomicMax(&best[lp[base + j]], (uint32_t)reply[base + j]);
        }
        __syncthreads();
        const uint64_t i = k * 256 + threadIdx.x;
        if (i < n) {
            const uint32_t v = best[threadIdx.x];
            if (!v) atomicOr(err, DEV_ERR_MISSING_CHILD);
            if (score_overflows(v)) atomicOr(err, DEV_ERR_OVERFLOW);
            self.s[islot[i]].score = parent_score(v);
        }
        __syncthreads();
    }
}

template <class K>
__global__ void root_lookup_kernel(typename KT<K>::Res t, K key, uint32_t *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const int s = res_find(t, key);
        *out = s < 0 ? 0u : (uint32_t)s;
    }
}

// One rank in one context (self_only below: a 128-bit-key game on one GPU) exchanges nothing,
// so the bucket / insert / lookup / fold kernels above collapse into two: the lane that
// generates a child inserts it into its tier's table (forward) or looks it up there (backward),
// as the single-GPU engine's expand / retro do (sparse.hip).  One move generation per pass
// instead of the bucket kernels' three, and no key, parent or reply lists.
template <class K, int S>
struct FrontsK {
    typename KT<K>::Front t[S];
};
template <class K, int S>
struct RessK {
    typename KT<K>::Res t[S];
};

template <class D>
__global__ __launch_bounds__(256) void self_expand_kernel(D d, const key_t<D> *__restrict__ ikeys, uint64_t n,
                                                          FrontsK<key_t<D>, D::MAX_SKIP> next,
                                                          uint8_t *__restrict__ iwon, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    using K = key_t<D>;
    uint64_t fresh[S];
#pragma unroll
    for (int s = 0; s < S; s++) fresh[s] = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (*(volatile uint32_t *)err & DEV_ERR_TABLE_FULL) break;   // re-run into larger tables
        const K k = ikeys[i];
        const int64_t tk = d.tier(k);
        bool won = false;
        d.visit(k, [&](const K &c) {
            const int64_t dt = d.tier(c) - tk;
            if (dt < 1 || dt > S) atomicOr(err, DEV_ERR_TIER);
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
__global__ __launch_bounds__(256) void self_retro_kernel(D d, const key_t<D> *__restrict__ ikeys,
                                                         const uint32_t *__restrict__ islot,
                                                         const uint8_t *__restrict__ iwon, uint64_t n,
                                                         typename KT<key_t<D>>::Res self,
                                                         RessK<key_t<D>, D::MAX_SKIP> next, uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    using K = key_t<D>;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t best = 0xFFFFu;   // a LOSS-in-0 child (iwon): nothing beats it, no lookup needed
        if (!iwon[i]) {
            best = 0;
            const K k = ikeys[i];
            const int64_t tk = d.tier(k);
            d.visit(k, [&](const K &c) {
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
            });
        }
        if (!best) atomicOr(err, DEV_ERR_MISSING_CHILD);
        if (score_overflows(best)) atomicOr(err, DEV_ERR_OVERFLOW);
        self.s[islot[i]].score = parent_score(best);
    }
}

// A rank's whole receive buffer of a tier in ONE launch: segment (q, s) -- source q, tier step
// s + 1 -- starts at bounds[q S + s] (the exchange layout's recv_seg; bounds[G S] = the total),
// and each key finds its step by a binary search over the G S + 1 bounds.  One launch per rank
// and tier instead of one per segment: the launch tails and the counter atomics are paid once.
template <int S>
__device__ __forceinline__ int bin_step(const uint64_t *__restrict__ bounds, int nbins, uint64_t j) {
    if constexpr (S == 1) {
        return 0;
    } else {
        int lo = 0, hi = nbins;   // bounds[lo] <= j < bounds[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (bounds[mid] <= j) lo = mid;
            else hi = mid;
        }
        return lo % S;
    }
}

template <class K, int S>
__global__ __launch_bounds__(256) void insert_bins_kernel(const K *__restrict__ in, uint64_t n,
                                                          const uint64_t *__restrict__ bounds, int nbins,
                                                          FrontsK<K, S> t, uint32_t *err) {
    uint64_t fresh[S];
#pragma unroll
    for (int s = 0; s < S; s++) fresh[s] = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        if (*(volatile uint32_t *)err & DEV_ERR_TABLE_FULL) break;   // re-run into larger tables
        const int st = bin_step<S>(bounds, nbins, i);
        const K k = in[i];
#pragma unroll
        for (int s = 0; s < S; s++)
            if (s == st && front_insert(t.t[s], k, err)) fresh[s]++;
    }
#pragma unroll
    for (int s = 0; s < S; s++) block_add(t.t[s].count, fresh[s]);
}

// (a primitive key is answered from primitive(), as classify scored it, with no table access)
template <class D>
__global__ __launch_bounds__(256) void lookup_bins_kernel(D d, const key_t<D> *__restrict__ in, uint64_t n,
                                                          const uint64_t *__restrict__ bounds, int nbins,
                                                          RessK<key_t<D>, D::MAX_SKIP> t, uint16_t *out,
                                                          uint32_t *err) {
    constexpr int S = D::MAX_SKIP;
    using K = key_t<D>;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const K k = in[i];
        const int p = d.primitive(k);
        int f;
        if (p != UNDECIDED) {
            f = score_of_primitive(p);
        } else {
            const int st = bin_step<S>(bounds, nbins, i);
            f = -1;
#pragma unroll
            for (int s = 0; s < S; s++)
                if (s == st) f = res_find(t.t[s], k);
            if (f < 0) atomicOr(err, DEV_ERR_MISSING_CHILD);
        }
        out[i] = f < 0 ? 0 : (uint16_t)f;
    }
}

// ------------------------------------------------------------------ host helpers
// element-wise sum (or max) over ranks of a host vector, through the IPC segment
static int sp_ipc_reduce(SpIpc &X, std::vector<uint64_t> &v, bool max) {
    std::vector<uint64_t> all((size_t)X.G * v.size());
    GM_TRY(sp_ipc_allgather(X, v.data(), v.size(), all.data()));
    for (size_t i = 0; i < v.size(); i++) {
        uint64_t a = 0;
        for (int r = 0; r < X.G; r++) a = max ? std::max(a, all[(size_t)r * v.size() + i]) : a + all[(size_t)r * v.size() + i];
        v[i] = a;
    }
    return GM_OK;
}

template <class K>
static int grow_keys(Ctx *c, K **p, uint64_t *cap, uint64_t need) {
    if (need <= *cap && *p) return GM_OK;
    dev_free(c, *p);
    const uint64_t nc = std::max<uint64_t>(need + need / 4, 1 << 16);
    GM_TRY(dev_alloc(c, (void **)p, nc * sizeof(K)));
    *cap = nc;
    return GM_OK;
}

template <class T>
static int grow_to(Ctx *c, T **p, uint64_t n) {   // paired with a grow_keys'd buffer of n entries
    dev_free(c, *p);
    return dev_alloc(c, (void **)p, std::max<uint64_t>(n, 1) * sizeof(T));
}

template <class K>
static typename KT<K>::Front fref(SpRankT<K> &R, size_t t) {
    SpTierT<K> &T = R.tiers[t];
    return typename KT<K>::Front{T.slots, T.cap, R.d_cnt + t};
}

// Cross-rank exchange of G-segmented arrays (RCCL mode; loopback copies are done by the caller).
static int sendrecv(Ctx *c, DistSparse *d, const void *send, const uint64_t *send_off, void *recv,
                    const uint64_t *recv_off, size_t elem) {
    // messages go in pieces of <= 1 GiB (the k-th piece to a peer matches its k-th receive)
    constexpr uint64_t PIECE = 1ull << 30;
    GM_NCCL(ncclGroupStart());
    for (int p = 0; p < d->G; p++) {
        const uint64_t sb = (send_off[p + 1] - send_off[p]) * elem, rb = (recv_off[p + 1] - recv_off[p]) * elem;
        const char *sp = (const char *)send + send_off[p] * elem;
        char *rp = (char *)recv + recv_off[p] * elem;
        for (uint64_t o = 0; o < sb; o += PIECE)
            GM_NCCL(ncclSend(sp + o, std::min(PIECE, sb - o), ncclUint8, p, c->comm, c->stream));
        for (uint64_t o = 0; o < rb; o += PIECE)
            GM_NCCL(ncclRecv(rp + o, std::min(PIECE, rb - o), ncclUint8, p, c->comm, c->stream));
        if (p != c->rank) d->sent_bytes += sb;
    }
    GM_NCCL(ncclGroupEnd());
    return GM_OK;
}

template <class D, bool SCATTER>
static void run_bucket(Ctx *c, DistSparse *d, const D &desc, SpRankT<key_t<D>> &R, size_t t) {
    SpTierT<key_t<D>> &T = R.tiers[t];
    if (!T.ni) return;
    typename SpRankT<key_t<D>>::Kept none{};
    const auto &kp = SCATTER ? R.kept[t] : none;
    hipLaunchKernelGGL((bucket_kernel<D, SCATTER>), dim3(grid_counted(T.ni)), dim3(256), 0, c->stream, desc, T.ikeys,
                       T.ni, d->G, R.d_hist, R.d_seg, R.d_cursor, R.sendk, kp.lp, kp.cbase, kp.ccnt, R.d_err);
}

// every local rank's device error word: enqueue the reads (read_errs), then after the stream
// synchronises turn the first set one into a status (errs_rc) -- one sync for all the ranks
template <class K>
static int read_errs(Ctx *c, DistSparseK<K> *d, std::vector<uint32_t> &errs) {
    errs.assign(d->ranks.size(), 0);
    for (size_t i = 0; i < d->ranks.size(); i++)
        GM_HIP(hipMemcpyAsync(&errs[i], d->ranks[i].d_err, 4, hipMemcpyDeviceToHost, c->stream));
    return GM_OK;
}
static int errs_rc(const std::vector<uint32_t> &errs) {
    for (uint32_t e : errs)
        if (e) return dev_error_to_gm(e);
    return GM_OK;
}
// counts[r][dest*S+dt] for all ranks -> host matrix (G x G*S)
// (the local ranks' device errors are read in the same synchronisation)
template <class K>
static int gather_counts(Ctx *c, DistSparseK<K> *d, std::vector<uint64_t> &mat) {
    const int nb = d->G * d->S;
    mat.assign((size_t)d->G * nb, 0);
    std::vector<uint32_t> errs;
    if (d->loopback) {
        for (auto &R : d->ranks)
            GM_HIP(hipMemcpyAsync(&mat[(size_t)R.rank * nb], R.d_hist, nb * 8, hipMemcpyDeviceToHost, c->stream));
        GM_TRY(read_errs(c, d, errs));
        GM_HIP(hipStreamSynchronize(c->stream));
        return errs_rc(errs);
    }
    if (d->ipc) {
        std::vector<uint64_t> row(nb);
        GM_HIP(hipMemcpyAsync(row.data(), d->ranks[0].d_hist, nb * 8, hipMemcpyDeviceToHost, c->stream));
        GM_TRY(read_errs(c, d, errs));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(errs_rc(errs));
        return sp_ipc_allgather(d->X, row.data(), nb, mat.data());
    }
    GM_NCCL(ncclAllGather(d->ranks[0].d_hist, d->d_mat, nb, ncclUint64, c->comm, c->stream));
    GM_HIP(hipMemcpyAsync(mat.data(), d->d_mat, mat.size() * 8, hipMemcpyDeviceToHost, c->stream));
    GM_TRY(read_errs(c, d, errs));
    GM_HIP(hipStreamSynchronize(c->stream));
    return errs_rc(errs);
}

template <class K>
static int check_err(Ctx *c, DistSparseK<K> *d) {
    std::vector<uint32_t> errs;
    GM_TRY(read_errs(c, d, errs));
    GM_HIP(hipStreamSynchronize(c->stream));
    return errs_rc(errs);
}


static Layout layout_for(int G, int S, const uint64_t *mat, int r) {
    const int nb = G * S;
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

static Layout layout_for(DistSparse *d, const std::vector<uint64_t> &mat, int r) {
    return layout_for(d->G, d->S, mat.data(), r);
}

// Host only (gm_sparse_layout): the layout every transport uses, for the CPU tests that replay
// the RCCL op list over gloo
int dist_sparse_layout(int G, int S, const uint64_t *mat, int r, uint64_t *seg, uint64_t *send_off,
                       uint64_t *recv_off, uint64_t *recv_seg) {
    if (G < 1 || S < 1 || G * S > MAXBINS || r < 0 || r >= G || !mat) {
        set_error("bad sparse layout arguments");
        return GM_E_ARG;
    }
    const Layout L = layout_for(G, S, mat, r);
    if (seg) std::copy(L.seg.begin(), L.seg.end(), seg);
    if (send_off) std::copy(L.send_off.begin(), L.send_off.end(), send_off);
    if (recv_off) std::copy(L.recv_off.begin(), L.recv_off.end(), recv_off);
    if (recv_seg) std::copy(L.recv_seg.begin(), L.recv_seg.end(), recv_seg);
    return GM_OK;
}

// A pull out of a peer's IPC-mapped window: hipMemcpyAsync takes the runtime's copy path for
// such memory (tools/ipc_big_probe.hip: 26-54 GB/s for 1 GiB on one GPU); a kernel reading the
// mapping directly streams like any device copy.  8-byte words (key segments) or 2-byte ones
// (reply segments).
template <class W>
__global__ __launch_bounds__(256) void ipc_pull_kernel(W *__restrict__ dst, const W *__restrict__ src, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
static int ipc_pull(Ctx *c, char *dst, const char *src, uint64_t bytes) {
    if (!bytes) return GM_OK;
    const uintptr_t a = (uintptr_t)dst | (uintptr_t)src | bytes;
    if (!(a & 7u))
        hipLaunchKernelGGL(ipc_pull_kernel<uint64_t>, dim3(grid_for(bytes / 8)), dim3(256), 0, c->stream,
                           (uint64_t *)dst, (const uint64_t *)src, bytes / 8);
    else if (!(a & 1u))
        hipLaunchKernelGGL(ipc_pull_kernel<uint16_t>, dim3(grid_for(bytes / 2)), dim3(256), 0, c->stream,
                           (uint16_t *)dst, (const uint16_t *)src, bytes / 2);
    else
        GM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    GM_HIP(hipGetLastError());
    return GM_OK;
}

// move every rank's segmented send buffer to the owners (or, reverse = true, the replies back).
// IPC: through one fixed window per rank, exported and mapped once per solve (SP_IPC_WIN bytes).
// Mapping each grown send buffer afresh stalled: Toot 6x4 without the symmetry reduction, the
// import of a 2.6 GB send buffer never returned (profiles/r06/r06ae_*, r06ak_*).  An exchange
// runs in rounds: the sender copies the next window-sized part of its send buffer into its
// window, a barrier, every receiver pulls the pieces of its segments that lie in that part out
// of the peers' windows, a barrier.  Every rank knows every rank's layout, so all take the same
// number of rounds.
constexpr uint64_t SP_IPC_WIN = 1ull << 30;
template <class K>
static int exchange_ipc(Ctx *c, DistSparseK<K> *d, const Layout &me, const std::vector<uint64_t> &mat, bool reply) {
    SpRankT<K> &R = d->ranks[0];
    SpIpc &X = d->X;
    const int G = d->G;
    const size_t elem = reply ? 2 : sizeof(K);
    char *mine = reply ? (char *)R.reply_out : (char *)R.sendk;
    char *dst = reply ? (char *)R.reply_in : (char *)R.recvk;
    if (!d->win) {   // once per solve: publish the window, then map the peers' one rank at a time
        // (two processes opening each other's IPC handles at once can block each other)
        GM_TRY(dev_alloc(c, (void **)&d->win, SP_IPC_WIN));
        GM_TRY(sp_ipc_publish(X, 0, d->win));
        GM_TRY(sp_ipc_barrier(X));
        for (int turn = 0; turn < G; turn++) {
            if (turn == X.me)
                for (int p = 0; p < G; p++) {
                    char *unused;
                    if (p != X.me) GM_TRY(sp_ipc_peer(X, p, 0, &unused));
                }
            GM_TRY(sp_ipc_barrier(X));
        }
    }
    std::vector<Layout> L(G);
    uint64_t rounds = 1;
    for (int p = 0; p < G; p++) {
        L[p] = layout_for(d, mat, p);
        const uint64_t tb = (reply ? L[p].nrecv : L[p].nsend) * elem;   // p's send buffer, bytes
        rounds = std::max<uint64_t>(rounds, (tb + SP_IPC_WIN - 1) / SP_IPC_WIN);
    }
    const uint64_t tme = (reply ? me.nrecv : me.nsend) * elem;
    GM_HIP(hipStreamSynchronize(c->stream));   // the send buffer is complete
    {   // this rank's own segment: a local copy
        const uint64_t n = reply ? me.send_off[X.me + 1] - me.send_off[X.me] : me.recv_off[X.me + 1] - me.recv_off[X.me];
        const uint64_t so = reply ? me.recv_off[X.me] : me.send_off[X.me];
        const uint64_t dof = reply ? me.send_off[X.me] : me.recv_off[X.me];
        GM_TRY(ipc_pull(c, dst + dof * elem, mine + so * elem, n * elem));
    }
    for (uint64_t j = 0; j < rounds; j++) {
        const uint64_t lo = j * SP_IPC_WIN, hi = lo + SP_IPC_WIN;
        if (lo < tme) GM_TRY(ipc_pull(c, d->win, mine + lo, std::min(hi, tme) - lo));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(sp_ipc_barrier(X));
        for (int p = 0; p < G; p++) {
            if (p == X.me) continue;
            // p's bytes for this rank, in p's send order: keys its send segment, replies its
            // answers to this rank's requests (p's receive segment from this rank)
            const uint64_t a = (reply ? L[p].recv_off[X.me] : L[p].send_off[X.me]) * elem;
            const uint64_t b = (reply ? L[p].recv_off[X.me + 1] : L[p].send_off[X.me + 1]) * elem;
            const uint64_t s0 = std::max(a, lo), e0 = std::min(b, hi);
            if (s0 >= e0) continue;
            char *pw;
            GM_TRY(sp_ipc_peer(X, p, 0, &pw));
            const uint64_t dof = (reply ? me.send_off[p] : me.recv_off[p]) * elem + (s0 - a);
            if (trace_on())
                fprintf(stderr, "[gm] ipc rank %d round %llu pulls %llu B from rank %d\n", X.me,
                        (unsigned long long)j, (unsigned long long)(e0 - s0), p);
            GM_TRY(ipc_pull(c, dst + dof, pw + (s0 - lo), e0 - s0));
        }
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_TRY(sp_ipc_barrier(X));   // the windows may be refilled
    }
    for (int p = 0; p < G; p++)   // what this rank sent: its segments other ranks pulled
        if (p != X.me)
            d->sent_bytes += (reply ? me.recv_off[p + 1] - me.recv_off[p] : me.send_off[p + 1] - me.send_off[p]) * elem;
    return GM_OK;
}

// One rank in one context (a 128-bit-key game on one GPU): its send order IS its receive
// order (one destination, one source), so the receive side reads the send buffers in place
// and the exchange copies nothing.
static bool self_only(const DistSparse *d) { return d->loopback && d->G == 1; }
// ... and then the fused kernels run (GM_SPARSE_SELF_FUSED=0, development: the bucket path)
static bool self_fused(const DistSparse *d) {
    static const bool on = !getenv("GM_SPARSE_SELF_FUSED") || atoi(getenv("GM_SPARSE_SELF_FUSED")) != 0;
    return on && self_only(d);
}
template <class K>
static K *recv_keys(const DistSparse *d, SpRankT<K> &R) { return self_only(d) ? R.sendk : R.recvk; }
template <class K>
static uint16_t *recv_replies(const DistSparse *d, SpRankT<K> &R) { return self_only(d) ? R.reply_out : R.reply_in; }

template <class K>
static int exchange(Ctx *c, DistSparseK<K> *d, const std::vector<Layout> &lay, const std::vector<uint64_t> &mat,
                    bool reply) {
    constexpr uint64_t KB = sizeof(K);
    if (self_only(d)) return GM_OK;
    if (c->poison)   // test hook: a segment that never lands reads as 0xFF, not as an earlier tier's data
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRankT<K> &R = d->ranks[i];
            const uint64_t n = reply ? lay[i].nsend : lay[i].nrecv;
            if (n) GM_HIP(hipMemsetAsync(reply ? (void *)R.reply_in : (void *)R.recvk, 0xFF, n * (reply ? 2 : KB), c->stream));
        }
    if (d->loopback) {
        for (size_t i = 0; i < d->ranks.size(); i++)
            for (size_t j = 0; j < d->ranks.size(); j++) {
                if (!reply) {   // keys: source j's segment for dest i -> i's recv segment from j
                    const uint64_t n = lay[i].recv_off[j + 1] - lay[i].recv_off[j];
                    if (n) GM_HIP(hipMemcpyAsync(d->ranks[i].recvk + lay[i].recv_off[j],
                                                 d->ranks[j].sendk + lay[j].send_off[i], n * KB,
                                                 hipMemcpyDeviceToDevice, c->stream));
                    if (i != j) d->sent_bytes += n * KB;
                } else {        // replies: owner j's answers to requester i
                    const uint64_t n = lay[i].send_off[j + 1] - lay[i].send_off[j];
                    if (n) GM_HIP(hipMemcpyAsync(d->ranks[i].reply_in + lay[i].send_off[j],
                                                 d->ranks[j].reply_out + lay[j].recv_off[i], n * 2,
                                                 hipMemcpyDeviceToDevice, c->stream));
                    if (i != j) d->sent_bytes += n * 2;
                }
            }
        return GM_OK;
    }
    SpRankT<K> &R = d->ranks[0];
    if (d->ipc) return exchange_ipc(c, d, lay[0], mat, reply);
    return reply ? sendrecv(c, d, R.reply_out, lay[0].recv_off.data(), R.reply_in, lay[0].send_off.data(), 2)
                 : sendrecv(c, d, R.sendk, lay[0].send_off.data(), R.recvk, lay[0].recv_off.data(), KB);
}

template <class K>
static int ensure_cnt(Ctx *c, DistSparseK<K> *d, size_t ntiers) {
    if (ntiers <= d->cnt_cap) return GM_OK;
    const size_t nc = std::max<size_t>(64, ntiers * 2);
    for (auto &R : d->ranks) {
        unsigned long long *p;
        GM_TRY(dev_alloc(c, (void **)&p, nc * 8));
        GM_HIP(hipMemsetAsync(p, 0, nc * 8, c->stream));
        if (R.d_cnt) {
            GM_HIP(hipMemcpyAsync(p, R.d_cnt, d->cnt_cap * 8, hipMemcpyDeviceToDevice, c->stream));
            dev_free(c, R.d_cnt);
        }
        R.d_cnt = p;
    }
    d->cnt_cap = nc;
    return GM_OK;
}

// classify tier t of every rank (scores in place + interior list)
// (every rank's classify enqueued, then one synchronisation reads the counters and the errors)
template <class D>
static int classify_tier(Ctx *c, DistSparseK<key_t<D>> *d, const D &desc, size_t t) {
    std::vector<std::array<unsigned long long, 12>> sc(d->ranks.size());
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SpRankT<key_t<D>> &R = d->ranks[i];
        if (!R.tiers[t].fcount) continue;
        GM_TRY(classify_tier_table(c, desc, R.tiers[t], R.d_scr, R.d_err, self_fused(d)));
        GM_HIP(hipMemcpyAsync(sc[i].data(), R.d_scr, sizeof sc[i], hipMemcpyDeviceToHost, c->stream));
    }
    std::vector<uint32_t> errs;
    GM_TRY(read_errs(c, d, errs));
    GM_HIP(hipStreamSynchronize(c->stream));
    GM_TRY(errs_rc(errs));
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SpRankT<key_t<D>> &R = d->ranks[i];
        SpTierT<key_t<D>> &T = R.tiers[t];
        const uint64_t n = T.fcount;
        if (!n) continue;
        if (sc[i][10] != n) {
            set_error("rank %d tier %zu: found %llu of %llu keys", R.rank, t, sc[i][10], (unsigned long long)n);
            return GM_E_STATE;
        }
        T.count = n;
        T.count_all = sc[i][11];
        T.ni = sc[i][9];
    }
    return GM_OK;
}

// forward step of tier t on one rank in one context (self_fused): classify's edge counts per
// tier step size the next tiers' tables; the expand inserts the children itself
template <class D>
static int self_expand(Ctx *c, DistSparseK<key_t<D>> *d, const D &desc, size_t t, uint64_t &offered,
                       uint64_t &before) {
    using K = key_t<D>;
    constexpr int S = D::MAX_SKIP;
    SpRankT<K> &R = d->ranks[0];
    SpTierT<K> &T = R.tiers[t];
    unsigned long long sc[S];
    GM_HIP(hipMemcpyAsync(sc, R.d_scr, sizeof sc, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    for (int s = 0; s < S; s++) {
        offered += sc[s];
        before += R.tiers[t + 1 + s].fcount;
        d->edges += sc[s];
    }
    if (!T.ni) return GM_OK;
    for (int attempt = 0; attempt < 2; attempt++) {
        FrontsK<K, S> nx;
        for (int s = 0; s < S; s++) {
            SpTierT<K> &U = R.tiers[t + 1 + s];
            const uint64_t need = table_cap_for(U.fcount + (attempt ? sc[s] : d->est.distinct(sc[s])));
            if (sc[s] && U.cap < need) GM_TRY(tier_grow(c, U, need, R.d_err));
            nx.t[s] = fref(R, t + 1 + s);
        }
        hipLaunchKernelGGL(self_expand_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, c->stream, desc, T.ikeys, T.ni,
                           nx, T.iwon, R.d_err);
        GM_HIP(hipGetLastError());
        uint32_t e;
        GM_HIP(hipMemcpyAsync(&e, R.d_err, 4, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        if (e != DEV_ERR_TABLE_FULL || attempt) break;
        if (trace_on()) fprintf(stderr, "[gm] tier %zu: tables full at ratio %.3f, re-running\n", t, d->est.ratio);
        GM_HIP(hipMemsetAsync(R.d_err, 0, 4, c->stream));
        d->est.missed();
    }
    return GM_OK;
}

template <class D>
static int solve_sharded(Ctx *c, const D &desc, const key_t<D> &root) {
    using K = key_t<D>;
    dist_sparse_free(c);
    DistSparseK<K> *d = new DistSparseK<K>();
    c->dist_sp = d;
    d->wide = sizeof(K) > 8;
    // one context, one GPU and no communicator (a 128-bit-key game's only engine): loopback, G = 1
    d->loopback = c->virtual_ranks > 1 || (c->world <= 1 && !c->have_uid);
    d->ipc = !d->loopback && c->sparse_transport == 1;
    d->G = d->loopback ? std::max(1, c->virtual_ranks) : c->world;
    d->S = D::MAX_SKIP;
    d->t_root = desc.tier(root);
    const int G = d->G, S = d->S, nb = G * S;
    if (!d->loopback && !d->ipc && !c->comm) {
        set_error("the sharded sparse engine needs a communicator (gm_set_comm) or virtual ranks");
        return GM_E_ARG;
    }
    if (nb > MAXBINS) { set_error("too many ranks for the sharded sparse engine"); return GM_E_ARG; }
    if (d->ipc) GM_TRY(sp_ipc_open(c, d->X, G));
    d->ranks.resize(d->loopback ? G : 1);
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SpRankT<K> &R = d->ranks[i];
        R.rank = d->loopback ? (int)i : c->rank;
        GM_TRY(dev_alloc(c, (void **)&R.d_err, 4));
        GM_HIP(hipMemsetAsync(R.d_err, 0, 4, c->stream));
        GM_TRY(dev_alloc(c, (void **)&R.d_hist, nb * 8));
        GM_TRY(dev_alloc(c, (void **)&R.d_cursor, nb * 8));
        GM_TRY(dev_alloc(c, (void **)&R.d_seg, nb * 8));
        GM_TRY(dev_alloc(c, (void **)&R.d_scr, 16 * 8));
        R.tiers.resize(1);
    }
    GM_TRY(dev_alloc(c, (void **)&d->d_mat, (size_t)G * nb * 8));
    GM_TRY(dev_alloc(c, (void **)&d->d_root, 4));
    GM_TRY(ensure_cnt(c, d, 64));
    // the root lives on its owner
    for (auto &R : d->ranks)
        if ((int)owner_rank(root, G) == R.rank) {
            GM_TRY(tier_alloc(c, &R.tiers[0].slots, 1024));
            R.tiers[0].cap = 1024;
            if constexpr (sizeof(K) > 8)
                hipLaunchKernelGGL(front_insert_one_wkernel, dim3(1), dim3(64), 0, c->stream, fref(R, 0), root, R.d_err);
            else
                hipLaunchKernelGGL(front_insert_one_kernel, dim3(1), dim3(64), 0, c->stream, fref(R, 0), root, R.d_err);
            R.tiers[0].fcount = 1;
        }
    d->gcount.assign(1, 1);
    const double t0 = now_ms();

    std::vector<uint64_t> mat;
    // ---------------- forward
    for (size_t t = 0; t < d->gcount.size(); t++) {
        if (!d->gcount[t]) continue;
        const size_t need = t + S + 1;
        if (d->gcount.size() < need) d->gcount.resize(need, 0);
        GM_TRY(ensure_cnt(c, d, need));
        for (auto &R : d->ranks)
            if (R.tiers.size() < need) R.tiers.resize(need);
        GM_TRY(classify_tier(c, d, desc, t));
        uint64_t offered = 0, before = 0;
        std::vector<std::vector<uint64_t>> hcs(d->ranks.size(), std::vector<uint64_t>(need, 0));
        bool counted = false;   // hcs read already (the bucket path reads them with its errors)
        if (self_fused(d)) {
            GM_TRY(self_expand(c, d, desc, t, offered, before));
        } else {
            // children -> owners
            for (auto &R : d->ranks) {
                GM_HIP(hipMemsetAsync(R.d_hist, 0, nb * 8, c->stream));
                run_bucket<D, false>(c, d, desc, R, t);
            }
            GM_TRY(gather_counts(c, d, mat));
            if (d->t_lay.size() < need) {
                d->t_lay.resize(need);
                d->t_mat.resize(need);
            }
            std::vector<Layout> &lay = d->t_lay[t];
            lay.assign(d->ranks.size(), Layout{});
            d->t_mat[t] = mat;
            for (size_t i = 0; i < d->ranks.size(); i++) {
                SpRankT<K> &R = d->ranks[i];
                lay[i] = layout_for(d, mat, R.rank);
                d->edges += lay[i].nsend;
                if (R.kept.size() < need) R.kept.resize(need);
                auto &kp = R.kept[t];
                const uint64_t nch = std::max<uint64_t>((R.tiers[t].ni + 255) / 256, 1);
                GM_TRY(dev_alloc(c, (void **)&kp.lp, std::max<uint64_t>(lay[i].nsend, 1)));
                GM_TRY(dev_alloc(c, (void **)&kp.cbase, nch * nb * 8));
                GM_TRY(dev_alloc(c, (void **)&kp.ccnt, nch * nb * 4));
                if (self_only(d)) {   // one rank, one context: what it sends is what it receives, kept
                    GM_TRY(dev_alloc(c, (void **)&kp.recvk, std::max<uint64_t>(lay[i].nsend, 1) * sizeof(K)));
                    R.sendk = kp.recvk;
                } else {
                    GM_TRY(grow_keys(c, &R.sendk, &R.send_cap, lay[i].nsend));
                    GM_TRY(dev_alloc(c, (void **)&kp.recvk, std::max<uint64_t>(lay[i].nrecv, 1) * sizeof(K)));
                    R.recvk = kp.recvk;
                }
                GM_HIP(hipMemcpyAsync(R.d_seg, lay[i].seg.data(), nb * 8, hipMemcpyHostToDevice, c->stream));
                GM_HIP(hipMemsetAsync(R.d_cursor, 0, nb * 8, c->stream));
                run_bucket<D, true>(c, d, desc, R, t);
            }
            GM_TRY(exchange(c, d, lay, mat, false));
            // owners insert into their tier tables, sized for load <= 0.7 of the predicted
            // distinct keys; a misprediction re-runs the (idempotent) inserts once.  Every rank's
            // inserts are enqueued, then one synchronisation reads the errors and the frontier
            // counts of all of them.
            const size_t NR = d->ranks.size();
            std::vector<std::vector<uint64_t>> in(NR, std::vector<uint64_t>(S, 0)), rbs(NR);
            for (size_t i = 0; i < NR; i++) {
                SpRankT<K> &R = d->ranks[i];
                for (int s = 0; s < S; s++) {
                    for (int q = 0; q < G; q++) in[i][s] += mat[(size_t)q * nb + R.rank * S + s];
                    offered += in[i][s];
                    before += R.tiers[t + 1 + s].fcount;
                }
                rbs[i] = lay[i].recv_seg;
                rbs[i].push_back(lay[i].nrecv);
                GM_TRY(dev_alloc(c, (void **)&R.kept[t].rb, (nb + 1) * 8));
                GM_HIP(hipMemcpyAsync(R.kept[t].rb, rbs[i].data(), (nb + 1) * 8, hipMemcpyHostToDevice, c->stream));
            }
            std::vector<char> todo(NR, 1);
            for (int attempt = 0; attempt < 2; attempt++) {
                for (size_t i = 0; i < NR; i++) {
                    if (!todo[i]) continue;
                    SpRankT<K> &R = d->ranks[i];
                    constexpr int SS = D::MAX_SKIP;
                    FrontsK<K, SS> nx;
                    for (int s = 0; s < S; s++) {
                        const size_t u = t + 1 + s;
                        SpTierT<K> &U = R.tiers[u];
                        const uint64_t nd = attempt ? in[i][s] : d->est.distinct(in[i][s]);
                        const uint64_t needc = table_cap_for(U.fcount + nd);
                        if (in[i][s] && U.cap < needc) GM_TRY(tier_grow(c, U, needc, R.d_err));
                        nx.t[s] = fref(R, u);
                    }
                    if (lay[i].nrecv)
                        hipLaunchKernelGGL((insert_bins_kernel<K, SS>), dim3(grid_for(lay[i].nrecv)), dim3(256), 0,
                                           c->stream, R.kept[t].recvk, lay[i].nrecv, R.kept[t].rb, nb, nx, R.d_err);
                    GM_HIP(hipGetLastError());
                }
                std::vector<uint32_t> errs;
                GM_TRY(read_errs(c, d, errs));
                for (size_t i = 0; i < NR; i++)
                    GM_HIP(hipMemcpyAsync(hcs[i].data(), d->ranks[i].d_cnt, need * 8, hipMemcpyDeviceToHost,
                                          c->stream));
                GM_HIP(hipStreamSynchronize(c->stream));
                bool again = false;
                for (size_t i = 0; i < NR; i++) {
                    if (!todo[i]) continue;
                    todo[i] = 0;
                    if (errs[i] == DEV_ERR_TABLE_FULL && !attempt) {
                        if (trace_on())
                            fprintf(stderr, "[gm] rank %d tier %zu: tables full at ratio %.3f, re-running\n",
                                    d->ranks[i].rank, t, d->est.ratio);
                        GM_HIP(hipMemsetAsync(d->ranks[i].d_err, 0, 4, c->stream));
                        d->est.missed();
                        todo[i] = 1;
                        again = true;
                    }
                }
                if (!again) {
                    GM_TRY(errs_rc(errs));
                    break;
                }
            }
            for (auto &R : d->ranks) {   // the tier's buffers now belong to kept[t]
                R.recvk = nullptr;
                if (self_only(d)) R.sendk = nullptr;
            }
            counted = true;
        }
        if (!counted) {   // (the fused path)
            GM_TRY(check_err(c, d));
            for (size_t i = 0; i < d->ranks.size(); i++)
                GM_HIP(hipMemcpyAsync(hcs[i].data(), d->ranks[i].d_cnt, need * 8, hipMemcpyDeviceToHost, c->stream));
            GM_HIP(hipStreamSynchronize(c->stream));
        }
        // global tier counts (sum over ranks of each rank's frontier counts)
        std::vector<uint64_t> local(need, 0);
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRankT<K> &R = d->ranks[i];
            for (size_t u = t + 1; u < need; u++) {
                R.tiers[u].fcount = hcs[i][u];
                local[u] += hcs[i][u];
            }
        }
        if (d->ipc) {
            GM_TRY(sp_ipc_reduce(d->X, local, false));
        } else if (!d->loopback) {
            if (need > d->tot_cap) {   // the tier count grows past the G*G*S count matrix
                if (d->d_tot) dev_free(c, d->d_tot);
                d->tot_cap = std::max<size_t>(64, 2 * need);
                GM_TRY(dev_alloc(c, (void **)&d->d_tot, d->tot_cap * 8));
            }
            GM_HIP(hipMemcpyAsync(d->d_tot, local.data(), need * 8, hipMemcpyHostToDevice, c->stream));
            GM_NCCL(ncclAllReduce(d->d_tot, d->d_tot, need, ncclUint64, ncclSum, c->comm, c->stream));
            GM_HIP(hipMemcpyAsync(local.data(), d->d_tot, need * 8, hipMemcpyDeviceToHost, c->stream));
            GM_HIP(hipStreamSynchronize(c->stream));
        }
        for (size_t u = t + 1; u < need; u++) d->gcount[u] = local[u];
        uint64_t after = 0;
        for (auto &R : d->ranks)
            for (int s = 0; s < S; s++) after += R.tiers[t + 1 + s].fcount;
        d->est.observe(after - before, offered);
        if (trace_on())
            fprintf(stderr, "[gm] sharded rank %d forward tier %zu: %llu positions (all ranks), at %.1f ms\n",
                    d->ranks[0].rank, t, (unsigned long long)d->gcount[t], now_ms() - t0);
    }
    while (!d->gcount.empty() && !d->gcount.back()) d->gcount.pop_back();
    const double t1 = now_ms();

    // ---------------- backward
    for (size_t t = d->gcount.size(); t-- > 0;) {
        if (!d->gcount[t]) continue;
        if (trace_on())
            fprintf(stderr, "[gm] sharded rank %d backward tier %zu at %.1f ms\n", d->ranks[0].rank, t, now_ms() - t0);
        if (self_fused(d)) {
            SpRankT<K> &R = d->ranks[0];
            SpTierT<K> &T = R.tiers[t];
            if (T.ni) {
                constexpr int SS = D::MAX_SKIP;
                RessK<K, SS> nx;
                for (int s = 0; s < SS; s++) {
                    const size_t u = t + 1 + s;
                    nx.t[s] = u < R.tiers.size() ? res_ref_of(R.tiers[u]) : typename KT<K>::Res{nullptr, 0};
                }
                hipLaunchKernelGGL(self_retro_kernel<D>, dim3(grid_for(T.ni)), dim3(256), 0, c->stream, desc, T.ikeys,
                                   T.islot, T.iwon, T.ni, res_ref_of(T), nx, R.d_err);
                GM_HIP(hipGetLastError());
            }
            GM_TRY(check_err(c, d));
            continue;
        }
        // RESOLVE: each owner looks up again the keys it received for tier t, the scores go back
        // in the same layout, and each sender folds them into the parents it recorded
        const std::vector<Layout> &lay = d->t_lay[t];
        const std::vector<uint64_t> &tmat = d->t_mat[t];
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRankT<K> &R = d->ranks[i];
            const uint64_t nrecv = self_only(d) ? lay[i].nsend : lay[i].nrecv;
            if (nrecv > R.rout_cap || !R.reply_out) {
                R.rout_cap = std::max<uint64_t>(nrecv + nrecv / 4, 1 << 16);
                GM_TRY(grow_to(c, &R.reply_out, R.rout_cap));
            }
            if (!self_only(d) && (lay[i].nsend > R.rin_cap || !R.reply_in)) {
                R.rin_cap = std::max<uint64_t>(lay[i].nsend + lay[i].nsend / 4, 1 << 16);
                GM_TRY(grow_to(c, &R.reply_in, R.rin_cap));
            }
            if (!nrecv) continue;
            constexpr int SS = D::MAX_SKIP;
            RessK<K, SS> nx;
            for (int s = 0; s < S; s++) {
                const size_t u = t + 1 + s;
                nx.t[s] = u < R.tiers.size() ? res_ref_of(R.tiers[u]) : typename KT<K>::Res{nullptr, 0};
            }
            hipLaunchKernelGGL(lookup_bins_kernel<D>, dim3(grid_for(nrecv)), dim3(256), 0, c->stream, desc,
                               R.kept[t].recvk, nrecv, R.kept[t].rb, nb, nx, R.reply_out, R.d_err);
        }
        GM_TRY(exchange(c, d, lay, tmat, true));                  // RESOLVE: scores back
        for (size_t i = 0; i < d->ranks.size(); i++) {
            SpRankT<K> &R = d->ranks[i];
            SpTierT<K> &T = R.tiers[t];
            const auto &kp = R.kept[t];
            if (T.ni)
                hipLaunchKernelGGL(fold_finalize_kernel<typename KT<K>::Res>, dim3(grid_for(T.ni)), dim3(256), 0,
                                   c->stream, recv_replies(d, R), kp.lp, kp.cbase, kp.ccnt, nb, T.islot, T.ni,
                                   res_ref_of(T), R.d_err);
        }
        // (no synchronisation per tier: the device errors are sticky and read after the pass; the
        // buffers below are stream-ordered, so the allocator may hand them out again at once)
        for (auto &R : d->ranks) {   // tier t is resolved: what the forward kept for it can go
            auto &kp = R.kept[t];
            for (void *p : {(void *)kp.recvk, (void *)kp.lp, (void *)kp.cbase, (void *)kp.ccnt, (void *)kp.rb})
                dev_free(c, p);
            kp = typename SpRankT<K>::Kept{};
        }
    }
    GM_TRY(check_err(c, d));
    const double t2 = now_ms();

    // root record: the owner's score, max-reduced over ranks
    GM_HIP(hipMemsetAsync(d->d_root, 0, 4, c->stream));
    for (auto &R : d->ranks)
        if ((int)owner_rank(root, G) == R.rank && !R.tiers.empty())
            hipLaunchKernelGGL(root_lookup_kernel<K>, dim3(1), dim3(64), 0, c->stream, res_ref_of(R.tiers[0]), root,
                               d->d_root);
    if (!d->loopback && !d->ipc) GM_NCCL(ncclAllReduce(d->d_root, d->d_root, 1, ncclUint32, ncclMax, c->comm, c->stream));
    uint32_t rs = 0;
    GM_HIP(hipMemcpyAsync(&rs, d->d_root, 4, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    if (d->ipc) {
        std::vector<uint64_t> v{rs};
        GM_TRY(sp_ipc_reduce(d->X, v, true));
        rs = (uint32_t)v[0];
    }
    c->root_record = record_of_score((uint16_t)rs);
    // positions per tier: the stored representatives' orbits (games.hpp), summed over ranks
    // (the last word: the stored representatives, summed over ranks too)
    std::vector<uint64_t> gall(d->gcount.size() + 1, 0);
    for (auto &R : d->ranks)
        for (size_t t = 0; t < d->gcount.size() && t < R.tiers.size(); t++) {
            gall[t] += R.tiers[t].count_all;
            gall.back() += R.tiers[t].count;
        }
    if (d->ipc) {
        GM_TRY(sp_ipc_reduce(d->X, gall, false));
    } else if (!d->loopback && !gall.empty()) {
        if (gall.size() > d->tot_cap) {
            if (d->d_tot) dev_free(c, d->d_tot);
            d->tot_cap = std::max<size_t>(64, 2 * gall.size());
            GM_TRY(dev_alloc(c, (void **)&d->d_tot, d->tot_cap * 8));
        }
        GM_HIP(hipMemcpyAsync(d->d_tot, gall.data(), gall.size() * 8, hipMemcpyHostToDevice, c->stream));
        GM_NCCL(ncclAllReduce(d->d_tot, d->d_tot, gall.size(), ncclUint64, ncclSum, c->comm, c->stream));
        GM_HIP(hipMemcpyAsync(gall.data(), d->d_tot, gall.size() * 8, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
    }
    const uint64_t stored = gall.back();
    gall.pop_back();
    uint64_t n = 0, tb = 0;
    for (auto v : gall) n += v;
    for (auto &R : d->ranks)
        for (auto &T : R.tiers) tb += T.cap * sizeof(typename KT<K>::Slot) + T.ni * (sizeof(K) + 5);
    c->n_positions = n;
    c->tier_counts = gall;
    c->stats.n_positions = n;
    c->stats.n_stored = stored;
    c->stats.n_tiers = (int32_t)d->gcount.size();
    c->stats.world = G;
    c->stats.forward_ms = t1 - t0;
    c->stats.backward_ms = t2 - t1;
    c->stats.solve_ms = t2 - t0;
    c->stats.exchanged_bytes = d->sent_bytes;
    c->stats.n_edges = d->edges;
    c->stats.table_bytes = tb;
    return GM_OK;
}

// the context's descriptor: the 64-bit-key games (with_game) or Othello 8x8 (K128 keys)
template <class F>
static int with_game(Ctx *c, F &&f) {
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: return f(c->f2o);
    case GM_GAME_TTT: return f(c->ttt);
    case GM_GAME_TOOT: return f(c->toot);
    case GM_GAME_OTHELLO: return f(c->oth);
    case GM_GAME_SUBTRACT: return f(c->sub);
    }
    set_error("unknown game");
    return GM_E_GAME;
}
template <class F>
static int with_any_game(Ctx *c, F &&f) {
    if (c->wide) return f(c->oth8);
    return with_game(c, f);
}

static int finish_solve(Ctx *c, int rc) {
    // IPC: a rank that leaves with an error marks the segment, so its peers' next barrier fails
    // at once instead of waiting out the limit
    if (rc != GM_OK && c->dist_sp) sp_ipc_fail(c->dist_sp->X);
    return rc;
}

int dist_sparse_solve(Ctx *c, uint64_t root) {
    if (c->wide) { set_error("this game's keys are 128-bit: gm_solve_key"); return GM_E_ARG; }
    return finish_solve(c, with_game(c, [&](const auto &desc) { return solve_sharded(c, desc, root); }));
}

int dist_sparse_solve_wide(Ctx *c, const K128 &root) {
    if (!c->wide) { set_error("not a 128-bit-key game"); return GM_E_ARG; }
    return finish_solve(c, solve_sharded(c, c->oth8, root));
}

// every rank's positions (each representative's orbit expanded), sorted by key
template <class D>
static int export_ranks(Ctx *c, const D &desc, key_t<D> *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    using K = key_t<D>;
    auto *d = static_cast<DistSparseK<K> *>(c->dist_sp);
    uint64_t total = 0;
    for (auto &R : d->ranks)
        for (auto &T : R.tiers) total += T.count_all;
    *n = total;
    if (!keys) return GM_OK;
    if (cap < total) { set_error("export buffer too small"); return GM_E_CAP; }
    K *dk;
    uint16_t *dr;
    unsigned long long *cur;
    GM_HIP(hipMalloc(&dk, std::max<uint64_t>(1, total) * sizeof(K)));
    GM_HIP(hipMalloc(&dr, std::max<uint64_t>(1, total) * 2));
    GM_HIP(hipMalloc(&cur, 8));
    GM_HIP(hipMemsetAsync(cur, 0, 8, c->stream));
    for (auto &R : d->ranks)
        for (auto &T : R.tiers)
            if (T.count)
                hipLaunchKernelGGL(res_gather_kernel<D>, dim3(grid_for(T.cap)), dim3(256), 0, c->stream, desc, T.slots,
                                   T.cap, dk, dr, cur);
    std::vector<K> hk(total);
    std::vector<uint16_t> hr(total);
    GM_HIP(hipMemcpyAsync(hk.data(), dk, total * sizeof(K), hipMemcpyDeviceToHost, c->stream));
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

int dist_sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    if (c->wide) { set_error("this game's keys are 128-bit: gm_export_key"); return GM_E_ARG; }
    return with_game(c, [&](const auto &desc) { return export_ranks(c, desc, keys, recs, cap, n); });
}

int dist_sparse_export_wide(Ctx *c, K128 *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    if (!c->wide) { set_error("not a 128-bit-key game"); return GM_E_ARG; }
    return export_ranks(c, c->oth8, keys, recs, cap, n);
}

int dist_sparse_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    unsigned long long *acc;
    GM_HIP(hipMalloc(&acc, 8));
    GM_HIP(hipMemsetAsync(acc, 0, 8, c->stream));
    uint64_t total = 0;
    GM_TRY(with_any_game(c, [&](const auto &desc) {
        using D = std::decay_t<decltype(desc)>;
        auto *d = static_cast<DistSparseK<key_t<D>> *>(c->dist_sp);
        for (auto &R : d->ranks)
            for (auto &T : R.tiers) {
                total += T.count_all;
                if (T.count)
                    hipLaunchKernelGGL(res_digest_kernel<D>, dim3(grid_counted(T.cap)), dim3(256), 0, c->stream, desc,
                                       T.slots, T.cap, acc);
            }
        return GM_OK;
    }));
    unsigned long long h;
    GM_HIP(hipMemcpyAsync(&h, acc, 8, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(acc);
    *digest = h;
    *n = total;
    return GM_OK;
}

template <class D>
static int query_ranks(Ctx *c, const D &desc, const key_t<D> *keys, uint16_t *recs, uint64_t n) {
    using K = key_t<D>;
    using Res = typename KT<K>::Res;
    auto *d = static_cast<DistSparseK<K> *>(c->dist_sp);
    K *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, n * sizeof(K)));
    GM_HIP(hipMalloc(&dr, n * 2));
    GM_HIP(hipMemcpyAsync(dk, keys, n * sizeof(K), hipMemcpyHostToDevice, c->stream));
    std::vector<uint16_t> part(n);
    for (uint64_t i = 0; i < n; i++) recs[i] = REC_UNSOLVED;
    for (auto &R : d->ranks) {
        std::vector<Res> h(R.tiers.size());
        for (size_t t = 0; t < h.size(); t++) h[t] = res_ref_of(R.tiers[t]);
        Res *tabs;
        GM_HIP(hipMalloc(&tabs, std::max<size_t>(1, h.size()) * sizeof(Res)));
        if (!h.empty()) GM_HIP(hipMemcpyAsync(tabs, h.data(), h.size() * sizeof(Res), hipMemcpyHostToDevice, c->stream));
        hipLaunchKernelGGL(query_kernel<D>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, desc,
                           d->t_root, tabs, (int)h.size(), dk, dr, n);
        GM_HIP(hipMemcpyAsync(part.data(), dr, n * 2, hipMemcpyDeviceToHost, c->stream));
        GM_HIP(hipStreamSynchronize(c->stream));
        (void)hipFree(tabs);
        for (uint64_t i = 0; i < n; i++)
            if (part[i] != REC_UNSOLVED) recs[i] = part[i];
    }
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

int dist_sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    if (!n) return GM_OK;
    if (c->wide) { set_error("this game's keys are 128-bit: gm_query_key"); return GM_E_ARG; }
    return with_game(c, [&](const auto &desc) { return query_ranks(c, desc, keys, recs, n); });
}

int dist_sparse_query_wide(Ctx *c, const K128 *keys, uint16_t *recs, uint64_t n) {
    if (!n) return GM_OK;
    if (!c->wide) { set_error("not a 128-bit-key game"); return GM_E_ARG; }
    return query_ranks(c, c->oth8, keys, recs, n);
}

template <class K>
static void free_ranks(Ctx *c, DistSparseK<K> *d) {
    for (auto &R : d->ranks) {
        for (auto &T : R.tiers) free_tier(c, T);
        // every buffer once: after a failed solve recvk / sendk may still alias a tier's
        std::vector<void *> ps = {(void *)R.d_cnt, (void *)R.d_err, (void *)R.d_hist, (void *)R.d_cursor,
                                  (void *)R.d_seg, (void *)R.d_scr, (void *)R.sendk, (void *)R.recvk,
                                  (void *)R.reply_out, (void *)R.reply_in};
        for (auto &kp : R.kept)
            for (void *p : {(void *)kp.recvk, (void *)kp.lp, (void *)kp.cbase, (void *)kp.ccnt, (void *)kp.rb})
                ps.push_back(p);
        std::sort(ps.begin(), ps.end());
        ps.erase(std::unique(ps.begin(), ps.end()), ps.end());
        for (void *p : ps) dev_free(c, p);
    }
}

void dist_sparse_free(Ctx *c) {
    DistSparse *d = c->dist_sp;
    if (!d) return;
    if (d->wide) free_ranks(c, static_cast<DistSparseK<K128> *>(d));
    else free_ranks(c, static_cast<DistSparseK<uint64_t> *>(d));
    dev_free(c, d->d_mat);
    if (d->d_tot) dev_free(c, d->d_tot);
    dev_free(c, d->d_root);
    dev_free(c, d->win);   // (to the allocation cache: a peer may not have closed its mapping yet)
    (void)hipStreamSynchronize(c->stream);
    sp_ipc_close(d->X);
    delete d;
    c->dist_sp = nullptr;
}

}  // namespace gm
