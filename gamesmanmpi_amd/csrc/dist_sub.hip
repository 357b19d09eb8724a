// dist_sub.hip -- the dense subtraction solve partitioned over G = 2, 4 or 8 ranks.
//
// Ownership ("block owner"): with LOW heaps inside a block, the g =
// log2 G top heaps are split in halves; rank bit a says whether heap (heaps-1-a)
// of the rank's blocks is >= 8.  The reference hashes every position to an
// owner (GameState.get_hash, src/game_state.py:23-31) and sends one message per
// edge (src/new_process.py:159,186); here a move changes one heap by 1 or 2, so a
// block's children live on its own rank except across a split heap, where the
// upper rank reads the two layers h = 6, 7 of its lower neighbour (tier t reads
// the neighbour's tiers t-1 and t-2): a halo of <= 25 % of a rank per split heap.
//
// Symmetric fill (GM_OPT_DIST_SYMMETRY, default on).  The game is symmetric under
// any permutation of heaps (DescSub: the same moves on every heap, one primitive
// position), so a position's code equals that of any heap permutation of it.  A
// halo block whose split nibble (6 or 7) can be swapped with an unsplit high
// nibble >= 8 is that permutation of a block the upper rank owns, of the SAME
// tier (a swap keeps the high sum), which the upper rank has just computed: it
// copies it locally after that tier's launch instead of receiving it.  Only
// halo blocks whose unsplit high nibbles are all <= 7 cross the link: 1/16, 1/8,
// 1/4 of the halo at G = 2, 4, 8 (5 high nibbles).  Every position is still
// computed by its owner; only the transfer is avoided.
//
// Tier-balanced owner (GM_OPT_DIST_OWNER 1).  Owner 0 staggers the ranks: rank r's
// blocks start at tier 8*popcount(r), so at a given tier one rank holds far more
// than 1/G of it and the job spans the whole 76-tier chain.  Owner 1 makes rank
// bits compare two heaps, [h_x < h_y]; a heap swap maps the two classes onto each
// other and keeps the tier, so every rank holds a share of every tier.  A child
// crossing into the other class is a permutation of a block its own rank owns
// (filled locally, any high-nibble permutation is searched), except the ties
// h_x == h_y, which only the [h_x < h_y] side needs: one direction per axis, as
// with owner 0, so the same lower/upper schedule carries them.
//
// Schedule.  Tiers (high-nibble sums) are grouped in batches of B (GM_OPT_DIST_BATCH);
// batch j is tiers [jB, jB+B).  Before batch j an upper rank needs its lower
// neighbour's halo of tiers [jB-1, jB+B-2] -- message X_j, which the lower rank
// packs and sends right after computing tier jB+B-2.  So a rank makes one launch
// per tier and one exchange per batch and split heap; an upper rank trails its
// lower neighbour by about one batch, which the partition's own stagger absorbs
// (rank r's blocks start at tier 8*popcount(r)).
//
// Streams and communicators (RCCL mode, one process per GPU): the compute stream
// S, plus one exchange stream X[a] and one communicator per split heap a
// (ncclCommSplit of the world communicator).  On axis a a rank is either the
// lower side (it only sends) or the upper side (it only receives), so an exchange
// stream never holds both a send and a receive, and a lower rank waits for an
// upper one only when its ring of K send buffers (GM_OPT_DIST_SLOTS) is full.
//
// Every rank's work is a precomputed list of ops (tier launch, unpack, send,
// receive, event record / wait).  The compute stream S carries only the tier
// launches and event waits/records: the tier kernel itself (sub_tier_kernel_b4x)
// writes each block, from the registers that hold it, also to the block's extra
// destinations -- its symmetric-fill images in the table and its slot in the
// halo message of every split heap it is sent on -- so no fill or pack kernel
// sits between two tiers, and the unpack of a received halo runs on X[a].  A
// tier that writes into a ring slot first waits until the slot's previous
// message has left.  RCCL mode runs its list in order.  The
// loopback mode (GM_OPT_VIRTUAL_RANKS: G ranks inside one context on one GPU,
// for testing the partition without a second GPU) runs the same lists on per-rank
// streams, a receive being a device copy from the sender's ring slot after the
// sender's pack event; a host-side scheduler interleaves the lists so that every
// cross-rank wait is enqueued after the record it waits for.
#include "gm_internal.hpp"

#include <mutex>

#include <algorithm>

namespace gm {

constexpr int MAX_AXES = 3;

enum EvKind { EV_PACKED = 0, EV_XCH = 1, EV_UNPACKED = 2, EV_KINDS = 3 };
enum OpKind { OP_TIER, OP_PACK, OP_UNPACK, OP_SEND, OP_RECV, OP_RECORD, OP_WAIT, OP_FILL };

struct Op {
    uint8_t kind, axis, ev, on_x;   // on_x: runs on X[axis], else on S
    int32_t arg;                    // tier (OP_TIER) or batch
    int32_t peer;                   // rank owning the event (OP_WAIT) / the other side (OP_SEND, OP_RECV)
};

struct SubRank {
    int rank = 0;
    uint8_t *table = nullptr;           // 1-byte codes (gm_common.hpp)
    bool owned = false;
    std::vector<uint32_t> off;          // per-tier offsets into dlist (owned blocks)
    uint32_t *dlist = nullptr;
    std::vector<uint32_t> fill_off;     // per-tier offsets into the fill pairs (symmetric fill; plan only)
    std::vector<uint32_t> xoff;         // per own block (dlist order): its extra destinations in xd
    std::vector<uint32_t> xd;           // (kind, value) pairs: XD_TABLE high part | XD_SEND + axis, (batch, index)
    uint32_t *dxoff = nullptr;
    uint64_t *dxdst = nullptr;          // xd resolved to device addresses (table / ring slots)
    std::vector<uint32_t> send_off[MAX_AXES], recv_off[MAX_AXES];   // per-batch offsets
    uint32_t *drecv[MAX_AXES] = {};
    uint8_t *sendbuf[MAX_AXES] = {}, *recvbuf[MAX_AXES] = {};       // rings of nslots slots
    uint64_t send_slot[MAX_AXES] = {}, recv_slot[MAX_AXES] = {};    // bytes per slot
    std::vector<hipEvent_t> ev[EV_KINDS][MAX_AXES];                 // nslots each
    hipEvent_t ev_join[MAX_AXES] = {};
    uint64_t own_blocks = 0;
    hipStream_t S = nullptr;
    hipStream_t X[MAX_AXES] = {};
    bool own_S = false;
    std::vector<Op> ops;
    size_t pc = 0;
    int recorded[EV_KINDS][MAX_AXES] = {};   // batches whose event is enqueued (host order)
};

struct DistSub {
    int heaps = 0, low = 0, high = 0, g = 0, G = 1, ntiers = 0, nt = 256;
    int batch = 4, nbatch = 0, nslots = 0;
    int want_threads = 0, want_x4 = 0, want_order = 0, want_batch = 0, want_slots = 0, want_sym = 0;
    int owner = 0, npair = 0;           // owner function (GM_OPT_DIST_OWNER); axes 0..npair-1 compare two heaps
    bool loopback = false;
    std::vector<SubRank> ranks;
    std::vector<int> lo, hi;            // per batch: tier range of X_j (empty if lo > hi)
    uint8_t *zero = nullptr;
    unsigned long long *d_acc = nullptr;
    uint32_t *d_root = nullptr;
    hipEvent_t ev_fork = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    ncclComm_t comm[MAX_AXES] = {};     // comm[0] = the context's; the others split from it
    bool own_comm[MAX_AXES] = {};
    uint64_t sent = 0;
};

static inline int nib(uint64_t v, int k) { return (int)((v >> (4 * k)) & 15u); }

// rank owning high part H.  Owner 0: rank bit a = [nibble high-1-a >= 8].  Owner 1
// (tier-balanced): for a < npair, bit a = [nibble high-1-2a < nibble high-2-2a];
// the remaining axes take [nibble >= 8] on the next unused nibbles.  A move lowers
// one nibble, so a child's owner differs from its parent's in at most one bit.
static inline int owner_of(const DistSub *d, uint64_t H) {
    int r = 0;
    if (d->owner == 0) {
        for (int a = 0; a < d->g; a++)
            if (nib(H, d->high - 1 - a) >= 8) r |= 1 << a;
        return r;
    }
    for (int a = 0; a < d->npair; a++)
        if (nib(H, d->high - 1 - 2 * a) < nib(H, d->high - 2 - 2 * a)) r |= 1 << a;
    for (int a = d->npair; a < d->g; a++)
        if (nib(H, d->high - 1 - d->npair - a) >= 8) r |= 1 << a;
    return r;
}

// Some block of rank q has H as a child block (H + 1 or + 2 on one nibble is q's).
static bool needed_by(const DistSub *d, uint64_t H, int q) {
    for (int k = 0; k < d->high; k++)
        for (uint64_t s = 1; s <= 2; s++)
            if ((uint64_t)nib(H, k) + s <= 15 && owner_of(d, H + (s << (4 * k))) == q) return true;
    return false;
}

// Owner 1: the first high-nibble permutation of H (lexicographic) that rank q owns.
static bool perm_source(const DistSub *d, uint64_t H, int q, uint64_t *src) {
    int idx[8];
    for (int k = 0; k < d->high; k++) idx[k] = k;
    while (std::next_permutation(idx, idx + d->high)) {
        uint64_t P = 0;
        for (int k = 0; k < d->high; k++) P |= (uint64_t)nib(H, idx[k]) << (4 * k);
        if (owner_of(d, P) == q) { *src = P; return true; }
    }
    return false;
}

static inline bool is_upper(int rank, int a) { return (rank >> a) & 1; }

// extra destinations of an own block (written by the tier kernel from the same registers)
enum XdKind { XD_TABLE = 0, XD_SEND = 1 };   // XD_SEND + axis; value = batch << 16 | index in the message

// Halo block H of axis a as a heap permutation of a block of the receiving (upper)
// rank: swap the split nibble (6 or 7) with the first unsplit high nibble >= 8.
// Returns false when every unsplit high nibble is <= 7 (the block is sent).
static bool sym_source(const DistSub *d, uint64_t H, int a, uint64_t *src) {
    const int ka = d->high - 1 - a;
    for (int j = 0; j < d->high - d->g; j++) {
        const uint64_t v = (uint64_t)nib(H, j);
        if (v < 8) continue;
        const uint64_t hv = (uint64_t)nib(H, ka);
        *src = H - (v << (4 * j)) + (hv << (4 * j)) - (hv << (4 * ka)) + (v << (4 * ka));
        return true;
    }
    return false;
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

static uint32_t cnt(const std::vector<uint32_t> &off, int i) {
    return (i < 0 || i + 1 >= (int)off.size()) ? 0 : off[i + 1] - off[i];
}

// Rank `rank`'s block lists, host only: own blocks per tier, symmetric-fill
// (dst, src) pairs per tier, halo blocks sent / received per batch and split heap.
struct Plan {
    std::vector<uint32_t> off, own, fill_off, fill, xoff, xd;
    std::vector<uint32_t> send_off[MAX_AXES], send[MAX_AXES], recv_off[MAX_AXES], recv[MAX_AXES];
    uint64_t own_blocks = 0;
};

// Identical enumeration on every rank, so a sender's halo list and its
// receiver's list agree block for block.
static int plan_lists(const Ctx *c, const DistSub *d, int rank, Plan &P) {
    const int T = d->ntiers, NB = d->nbatch;
    const uint64_t nhigh = 1ull << (4 * d->high);
    auto tsum = [&](uint64_t H) { int s = 0; for (int k = 0; k < d->high; k++) s += nib(H, k); return s; };
    std::vector<int> xb(T, -1);   // halo message carrying tier t
    for (int j = 0; j < NB; j++)
        for (int t = d->lo[j]; t <= d->hi[j]; t++) xb[t] = j;
    std::vector<std::vector<uint32_t>> own(T), Sd[MAX_AXES], Rv[MAX_AXES], fill(T);
    for (int a = 0; a < MAX_AXES; a++) { Sd[a].resize(NB); Rv[a].resize(NB); }
    for (uint64_t H = 0; H < nhigh; H++) {
        const int o = owner_of(d, H), t = tsum(H);
        for (int a = 0; a < d->g; a++) {
            if (xb[t] < 0) continue;
            const int q = o ^ (1 << a);   // the rank across axis a
            uint64_t src = 0;
            bool sym;
            if (d->owner == 0) {
                const int h = nib(H, d->high - 1 - a);
                if (h != 6 && h != 7) continue;
                sym = c->dist_symmetry && sym_source(d, H, a, &src);
            } else {
                if ((q != rank && o != rank) || !needed_by(d, H, q)) continue;
                sym = perm_source(d, H, q, &src);
                if (!is_upper(q, a)) {
                    // a lower rank needing an upper rank's block: always a permutation of its own
                    if (!sym) {
                        set_error("tier-balanced owner: block %llx would cross axis %d downwards",
                                  (unsigned long long)H, a);
                        return GM_E_STATE;
                    }
                    if (q == rank) {
                        // same guard as the upward branch: the fill source must be an own
                        // block of the same tier, computed by this rank's tier-t launch
                        if (owner_of(d, src) != rank || tsum(src) != t) {
                            set_error("symmetric fill source of block %llx is not an own block of its tier",
                                      (unsigned long long)H);
                            return GM_E_STATE;
                        }
                        fill[t].push_back((uint32_t)H);
                        fill[t].push_back((uint32_t)src);
                    }
                    continue;
                }
            }
            if (o == rank && !is_upper(rank, a) && !sym) Sd[a][xb[t]].push_back((uint32_t)H);
            if (is_upper(rank, a) && o == (rank ^ (1 << a))) {
                if (!sym) {
                    Rv[a][xb[t]].push_back((uint32_t)H);
                } else {
                    if (owner_of(d, src) != rank || tsum(src) != t) {
                        set_error("symmetric halo source of block %llx is not an own block of its tier",
                                  (unsigned long long)H);
                        return GM_E_STATE;
                    }
                    fill[t].push_back((uint32_t)H);
                    fill[t].push_back((uint32_t)src);
                }
            }
        }
        if (o == rank) {
            own[t].push_back((uint32_t)H);
            P.own_blocks++;
        }
    }
    auto flatten = [&](std::vector<std::vector<uint32_t>> &L, std::vector<uint32_t> &off,
                       std::vector<uint32_t> &flat) {
        off.assign(L.size() + 1, 0);
        for (size_t i = 0; i < L.size(); i++) {
            off[i] = (uint32_t)flat.size();
            flat.insert(flat.end(), L[i].begin(), L[i].end());
        }
        off[L.size()] = (uint32_t)flat.size();
    };
    flatten(own, P.off, P.own);
    if (c->sub_order >= 1) sort_tiers_morton(P.own, P.off, d->high, c->sub_order);
    flatten(fill, P.fill_off, P.fill);
    for (int a = 0; a < d->g; a++) {
        flatten(Sd[a], P.send_off[a], P.send[a]);
        flatten(Rv[a], P.recv_off[a], P.recv[a]);
    }
    // each own block's extra destinations, in the own list's (possibly Morton) order
    std::vector<std::vector<uint32_t>> ex(nhigh);
    for (size_t i = 0; i + 1 < P.fill.size(); i += 2) {
        ex[P.fill[i + 1]].push_back(XD_TABLE);
        ex[P.fill[i + 1]].push_back(P.fill[i]);
    }
    for (int a = 0; a < d->g; a++)
        for (int j = 0; j < NB; j++)
            for (int k = 0; k < (int)Sd[a][j].size(); k++) {
                if (k >= (1 << 16) || j >= (1 << 16)) { set_error("halo message too large"); return GM_E_STATE; }
                ex[Sd[a][j][k]].push_back(XD_SEND + a);
                ex[Sd[a][j][k]].push_back((uint32_t)j << 16 | (uint32_t)k);
            }
    P.xoff.assign(P.own.size() + 1, 0);
    for (size_t i = 0; i < P.own.size(); i++) {
        P.xoff[i] = (uint32_t)(P.xd.size() / 2);
        P.xd.insert(P.xd.end(), ex[P.own[i]].begin(), ex[P.own[i]].end());
    }
    P.xoff[P.own.size()] = (uint32_t)(P.xd.size() / 2);
    return GM_OK;
}

// Plan rank R's lists and put them on the device with its exchange buffers and events.
static int build_lists(Ctx *c, DistSub *d, SubRank &R) {
    const int NB = d->nbatch;
    Plan P;
    GM_TRY(plan_lists(c, d, R.rank, P));
    R.own_blocks = P.own_blocks;
    R.off = P.off;
    R.fill_off = P.fill_off;
    R.xoff = P.xoff;
    R.xd = P.xd;
    GM_TRY(upload(P.own, &R.dlist));
    GM_TRY(upload(P.xoff, &R.dxoff));
    const uint64_t bb = 1ull << (4 * d->low);
    for (int a = 0; a < d->g; a++) {
        R.send_off[a] = P.send_off[a];
        R.recv_off[a] = P.recv_off[a];
        GM_TRY(upload(P.recv[a], &R.drecv[a]));
        uint64_t ms = 0, mr = 0;
        for (int j = 0; j < NB; j++) {
            ms = std::max<uint64_t>(ms, cnt(R.send_off[a], j));
            mr = std::max<uint64_t>(mr, cnt(R.recv_off[a], j));
        }
        R.send_slot[a] = ms * bb;
        R.recv_slot[a] = mr * bb;
        if (ms) GM_HIP(hipMalloc(&R.sendbuf[a], ms * bb * d->nslots));
        if (mr) GM_HIP(hipMalloc(&R.recvbuf[a], mr * bb * d->nslots));
        for (int k = 0; k < EV_KINDS; k++) {
            R.ev[k][a].resize(d->nslots);
            for (auto &e : R.ev[k][a]) GM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        GM_HIP(hipEventCreateWithFlags(&R.ev_join[a], hipEventDisableTiming));
    }
    return GM_OK;
}

static uint8_t *send_ptr(const DistSub *d, const SubRank &R, int a, int j) {
    return R.sendbuf[a] + (uint64_t)(j % d->nslots) * R.send_slot[a];
}
static uint8_t *recv_ptr(const DistSub *d, const SubRank &R, int a, int j) {
    return R.recvbuf[a] + (uint64_t)(j % d->nslots) * R.recv_slot[a];
}

// R.xd -> device addresses, once the table and the send rings exist
static int upload_xdst(DistSub *d, SubRank &R) {
    const uint64_t bb = 1ull << (4 * d->low);
    std::vector<uint64_t> a64(std::max<size_t>(1, R.xd.size() / 2), 0);
    for (size_t i = 0; i < R.xd.size() / 2; i++) {
        const uint32_t kind = R.xd[2 * i], v = R.xd[2 * i + 1];
        if (kind == XD_TABLE) {
            a64[i] = (uint64_t)(uintptr_t)(R.table + ((uint64_t)v << (4 * d->low)));
        } else {
            const int a = (int)kind - XD_SEND, j = (int)(v >> 16), k = (int)(v & 0xFFFFu);
            a64[i] = (uint64_t)(uintptr_t)(send_ptr(d, R, a, j) + (uint64_t)k * bb);
        }
    }
    GM_HIP(hipMalloc(&R.dxdst, a64.size() * 8));
    GM_HIP(hipMemcpy(R.dxdst, a64.data(), a64.size() * 8, hipMemcpyHostToDevice));
    return GM_OK;
}

// The op list of rank R for one solve (see the file comment).
static void build_ops(DistSub *d, SubRank &R) {
    const int T = d->ntiers, NB = d->nbatch, B = d->batch, NS = d->nslots;
    auto op = [&](int kind, int axis, int ev, bool on_x, int arg, int peer) {
        R.ops.push_back(Op{(uint8_t)kind, (uint8_t)axis, (uint8_t)ev, (uint8_t)on_x, arg, peer});
    };
    std::vector<std::vector<int>> send_after(T), send_from(T);   // halo messages ending / starting at tier t
    for (int j = 0; j < NB; j++)
        if (d->lo[j] <= d->hi[j]) {
            send_after[d->hi[j]].push_back(j);
            send_from[d->lo[j]].push_back(j);
        }
    R.ops.clear();
    for (int j = 0; j < NB; j++) {
        // receive X_j on every axis where this rank is the upper side; X[a] unpacks it
        // (the previous message in its ring slot was unpacked earlier on the same stream)
        for (int a = 0; a < d->g; a++) {
            if (!is_upper(R.rank, a) || !cnt(R.recv_off[a], j)) continue;
            const int lower = R.rank ^ (1 << a);
            if (d->loopback) op(OP_WAIT, a, EV_PACKED, true, j, lower);
            op(OP_RECV, a, 0, true, j, lower);
            op(OP_RECORD, a, EV_XCH, true, j, R.rank);
            op(OP_UNPACK, a, 0, true, j, R.rank);
            op(OP_RECORD, a, EV_UNPACKED, true, j, R.rank);
            op(OP_WAIT, a, EV_UNPACKED, false, j, R.rank);
        }
        for (int t = j * B; t < std::min(T, j * B + B); t++) {
            // the tier kernel writes the halo blocks of messages starting here into their
            // ring slots: the slot's previous message (jj - NS) must have left
            for (int jj : send_from[t])
                for (int a = 0; a < d->g; a++) {
                    if (is_upper(R.rank, a) || !cnt(R.send_off[a], jj)) continue;
                    // the slot's last non-empty message (empty ones record nothing; with
                    // owner 1 a batch's message can be empty between two that are not)
                    int jp = jj - NS;
                    while (jp >= 0 && !cnt(R.send_off[a], jp)) jp -= NS;
                    if (jp >= 0) op(OP_WAIT, a, EV_XCH, false, jp, d->loopback ? (R.rank ^ (1 << a)) : R.rank);
                }
            op(OP_TIER, 0, 0, false, t, R.rank);
            for (int jj : send_after[t])
                for (int a = 0; a < d->g; a++) {
                    if (is_upper(R.rank, a) || !cnt(R.send_off[a], jj)) continue;
                    op(OP_RECORD, a, EV_PACKED, false, jj, R.rank);
                    if (!d->loopback) {
                        op(OP_WAIT, a, EV_PACKED, true, jj, R.rank);
                        op(OP_SEND, a, 0, true, jj, R.rank ^ (1 << a));
                        op(OP_RECORD, a, EV_XCH, true, jj, R.rank);
                    }
                }
        }
    }
}

// The partition's shape (block split, tiers, batches, ring depth), host only.
static int plan_shape(const Ctx *c, DistSub *d, int G, bool loopback) {
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
    d->nt = -2;   // ranks always run the byte-image tier kernel (its extra-destination variant)
    d->want_threads = c->sub_threads;
    d->want_x4 = c->sub_interleave;
    d->want_order = c->sub_order;
    d->want_batch = c->dist_batch;
    d->want_slots = c->dist_slots;
    d->want_sym = c->dist_symmetry;
    d->owner = c->dist_owner;
    if (d->owner == 1) {
        // as many two-heap comparisons as leave a nibble for every remaining axis
        d->npair = std::max(0, std::min(d->g, d->high - d->g));
        if (!c->dist_symmetry) {
            set_error("the tier-balanced owner needs GM_OPT_DIST_SYMMETRY 1 (its downward halo is all fills)");
            return GM_E_ARG;
        }
    }
    if (d->low != 3 || !sub_kernel_x_exists(d->high)) { set_error("no sharded dense kernel"); return GM_E_GAME; }
    d->ntiers = 15 * d->high + 1;
    d->batch = std::max(1, std::min(c->dist_batch, d->ntiers));
    d->nbatch = (d->ntiers + d->batch - 1) / d->batch;
    d->nslots = std::max(1, std::min(c->dist_slots, d->nbatch));
    d->lo.resize(d->nbatch);
    d->hi.resize(d->nbatch);
    for (int j = 0; j < d->nbatch; j++) {
        d->lo[j] = std::max(0, j * d->batch - 1);
        d->hi[j] = std::min(d->ntiers - 2, j * d->batch + d->batch - 2);
    }
    return GM_OK;
}

static int prepare(Ctx *c, DistSub *d, int G, bool loopback) {
    GM_TRY(plan_shape(c, d, G, loopback));
    size_t zb = std::max<size_t>(16, 1ull << (4 * d->low));
    GM_HIP(hipMalloc(&d->zero, zb));
    GM_HIP(hipMemset(d->zero, 0, zb));
    GM_HIP(hipMalloc(&d->d_acc, 16));
    GM_HIP(hipMalloc(&d->d_root, 4));
    GM_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    GM_HIP(hipEventCreate(&d->ev_t0));
    GM_HIP(hipEventCreate(&d->ev_t1));
    if (!loopback) {
        // one communicator per split heap; every rank makes the same calls in the same order
        d->comm[0] = c->comm;
        for (int a = 1; a < d->g; a++) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 1;
            GM_NCCL(ncclCommSplit(c->comm, 0, c->rank, &d->comm[a], &cfg));
            d->own_comm[a] = true;
        }
    }
    d->ranks.resize(loopback ? G : 1);
    for (size_t i = 0; i < d->ranks.size(); i++) {
        SubRank &R = d->ranks[i];
        R.rank = loopback ? (int)i : c->rank;
        GM_TRY(build_lists(c, d, R));
        const uint64_t bytes = 1ull << (4 * d->heaps);
        if (!loopback && c->adopted_dense) {
            if (c->adopted_dense_bytes < bytes) { set_error("adopted dense table too small"); return GM_E_CAP; }
            R.table = (uint8_t *)c->adopted_dense;
        } else {
            if (hipMalloc(&R.table, bytes) != hipSuccess) {
                set_error("hipMalloc of a %llu-byte rank table failed", (unsigned long long)bytes);
                return GM_E_NOMEM;
            }
            R.owned = true;
        }
        if (loopback) {
            GM_HIP(hipStreamCreateWithFlags(&R.S, hipStreamNonBlocking));
            R.own_S = true;
        }
        for (int a = 0; a < d->g; a++) GM_HIP(hipStreamCreateWithFlags(&R.X[a], hipStreamNonBlocking));
        GM_TRY(upload_xdst(d, R));
        build_ops(d, R);
    }
    return GM_OK;
}

static void copy_blocks(DistSub *d, const uint8_t *src, const uint32_t *list, uint32_t n, uint8_t *dst,
                        bool pack, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(block_copy_kernel, dim3(n), dim3(256), 0, s, src, list, dst, d->low, pack ? 1 : 0);
}

static int exec_op(DistSub *d, SubRank &R, const Op &o) {
    const int a = o.axis, j = o.arg;
    const uint64_t bb = 1ull << (4 * d->low);
    hipStream_t st = o.on_x ? R.X[a] : R.S;
    switch (o.kind) {
    case OP_TIER:
        launch_sub_tier_x(d->high, cnt(R.off, j), R.table, R.dlist + R.off[j], d->zero, R.dxoff + R.off[j], R.dxdst,
                          st, d->want_x4);
        break;
    case OP_FILL:
    case OP_PACK:   // folded into OP_TIER (extra destinations); not in the lists
        set_error("unexpected op %d", (int)o.kind);
        return GM_E_STATE;
    case OP_UNPACK:
        copy_blocks(d, recv_ptr(d, R, a, j), R.drecv[a] + R.recv_off[a][j], cnt(R.recv_off[a], j), R.table, false,
                    st);
        break;
    case OP_SEND:
        GM_NCCL(ncclSend(send_ptr(d, R, a, j), cnt(R.send_off[a], j) * bb, ncclUint8, o.peer, d->comm[a], st));
        break;
    case OP_RECV: {
        const uint64_t n = cnt(R.recv_off[a], j) * bb;
        if (d->loopback) {
            const SubRank &L = d->ranks[o.peer];
            if (cnt(L.send_off[a], j) * bb != n) { set_error("halo lists disagree"); return GM_E_STATE; }
            GM_HIP(hipMemcpyAsync(recv_ptr(d, R, a, j), send_ptr(d, L, a, j), n, hipMemcpyDeviceToDevice, st));
        } else {
            GM_NCCL(ncclRecv(recv_ptr(d, R, a, j), n, ncclUint8, o.peer, d->comm[a], st));
        }
        break;
    }
    case OP_RECORD:
        if (o.ev == EV_PACKED) d->sent += cnt(R.send_off[a], j) * bb;   // message j complete in its slot
        GM_HIP(hipEventRecord(R.ev[o.ev][a][j % d->nslots], st));
        R.recorded[o.ev][a] = j + 1;
        break;
    case OP_WAIT: {
        const SubRank &P = d->loopback ? d->ranks[o.peer] : R;
        GM_HIP(hipStreamWaitEvent(st, P.ev[o.ev][a][j % d->nslots], 0));
        break;
    }
    }
    return GM_OK;
}

// Enqueue one whole solve.  RCCL mode: the single rank's list in order.
// Loopback: round-robin over the ranks, each running until its next op waits on
// an event another rank has not enqueued yet.
static int enqueue_solve(DistSub *d, int solo) {
    if (solo > 0) {   // diagnostic: one rank's tier launches back to back (results invalid)
        if (!d->loopback || solo > (int)d->ranks.size()) { set_error("dist_solo needs loopback ranks"); return GM_E_ARG; }
        SubRank &R = d->ranks[solo - 1];
        for (const Op &o : R.ops)
            if (o.kind == OP_TIER) GM_TRY(exec_op(d, R, o));
        GM_HIP(hipGetLastError());
        return GM_OK;
    }
    for (auto &R : d->ranks) {
        R.pc = 0;
        for (auto &k : R.recorded)
            for (int &x : k) x = 0;
    }
    d->sent = 0;
    for (;;) {
        bool done = true, progress = false;
        for (auto &R : d->ranks) {
            while (R.pc < R.ops.size()) {
                const Op &o = R.ops[R.pc];
                if (d->loopback && o.kind == OP_WAIT && o.peer != R.rank &&
                    d->ranks[o.peer].recorded[o.ev][o.axis] <= o.arg)
                    break;
                GM_TRY(exec_op(d, R, o));
                R.pc++;
                progress = true;
            }
            done &= R.pc == R.ops.size();
        }
        if (done) break;
        if (!progress) { set_error("sharded schedule cannot make progress"); return GM_E_STATE; }
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

// Run one solve: fork every rank's streams off the caller's stream, enqueue, join.
// Launches are eager: in RCCL mode a stream capture refused half-way would
// leave the ranks' point-to-point sequence numbers out of step.
static int run_solve(Ctx *c, DistSub *d) {
    hipStream_t H = c->stream;
    if (!d->loopback) d->ranks[0].S = c->stream;
    GM_HIP(hipEventRecord(d->ev_fork, H));
    for (auto &R : d->ranks) {
        if (R.S != H) GM_HIP(hipStreamWaitEvent(R.S, d->ev_fork, 0));
        for (int a = 0; a < d->g; a++) GM_HIP(hipStreamWaitEvent(R.X[a], d->ev_fork, 0));
    }
    GM_TRY(enqueue_solve(d, c->dist_solo));
    for (auto &R : d->ranks) {
        for (int a = 0; a < d->g; a++) {
            GM_HIP(hipEventRecord(R.ev_join[a], R.X[a]));
            GM_HIP(hipStreamWaitEvent(R.S, R.ev_join[a], 0));
        }
        if (R.S != H) {
            GM_HIP(hipEventRecord(R.ev_join[0], R.S));
            GM_HIP(hipStreamWaitEvent(H, R.ev_join[0], 0));
        }
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

int dist_sub_solve(Ctx *c, uint64_t root) {
    const bool loopback = c->virtual_ranks > 1;
    const int G = loopback ? c->virtual_ranks : c->world;
    DistSub *d = c->dist_sub;
    if (!d || d->heaps != c->sub.heaps || d->G != G || d->loopback != loopback ||
        d->want_threads != c->sub_threads || d->want_x4 != c->sub_interleave || d->want_order != c->sub_order ||
        d->want_batch != c->dist_batch || d->want_slots != c->dist_slots || d->want_sym != c->dist_symmetry ||
        d->owner != c->dist_owner ||
        (!loopback && c->adopted_dense && d->ranks[0].table != c->adopted_dense)) {
        dist_sub_free(c);
        d = c->dist_sub = new DistSub();
        GM_TRY(prepare(c, d, G, loopback));
    }
    hipStream_t H = c->stream;
    double t0 = now_ms();
    GM_HIP(hipEventRecord(d->ev_t0, H));
    GM_TRY(run_solve(c, d));
    GM_HIP(hipEventRecord(d->ev_t1, H));
    double t_enq = now_ms();
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
    c->stats.forward_ms = t_enq - t0;   // host time spent enqueueing the solve
    c->stats.exchanged_bytes = d->sent;
    if (c->timing) {
        float ms = 0;
        GM_HIP(hipEventElapsedTime(&ms, d->ev_t0, d->ev_t1));
        c->stats.kernel_ms = ms;
        uint32_t launches = 0;
        for (auto &R : d->ranks)
            for (int t = 0; t < d->ntiers; t++) launches += cnt(R.off, t) > 0;
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
        uint32_t nb = R.off.back();
        if (nb) hipLaunchKernelGGL(block_digest_kernel, dim3(std::min<uint32_t>(nb, 8192)), dim3(256), 0, H, R.table,
                                   R.dlist, (uint64_t)nb, d->low, d->heaps, c->root, d->d_acc);
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
        uint32_t nb = R.off.back();
        if (!nb) continue;
        uint8_t *stg;
        GM_HIP(hipMalloc(&stg, (uint64_t)nb * bsz));
        copy_blocks(d, R.table, R.dlist, nb, stg, true, H);
        std::vector<uint8_t> hs((uint64_t)nb * bsz);
        std::vector<uint32_t> hl(nb);
        GM_HIP(hipMemcpyAsync(hs.data(), stg, hs.size(), hipMemcpyDeviceToHost, H));
        GM_HIP(hipMemcpyAsync(hl.data(), R.dlist, nb * 4, hipMemcpyDeviceToHost, H));
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
        bool in = true;   // outside the root's region: unsolved (include/gmsolve.h gm_query)
        for (int j = 0; j < d->heaps && in; j++) in = ((keys[i] >> (4 * j)) & 15u) <= ((c->root >> (4 * j)) & 15u);
        if (!in) continue;
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
    (void)hipDeviceSynchronize();
    for (auto &R : d->ranks) {
        if (R.owned && R.table) (void)hipFree(R.table);
        if (R.dlist) (void)hipFree(R.dlist);
        if (R.dxoff) (void)hipFree(R.dxoff);
        if (R.dxdst) (void)hipFree(R.dxdst);
        for (int a = 0; a < MAX_AXES; a++) {
            if (R.drecv[a]) (void)hipFree(R.drecv[a]);
            if (R.sendbuf[a]) (void)hipFree(R.sendbuf[a]);
            if (R.recvbuf[a]) (void)hipFree(R.recvbuf[a]);
            for (int k = 0; k < EV_KINDS; k++)
                for (auto e : R.ev[k][a]) (void)hipEventDestroy(e);
            if (R.ev_join[a]) (void)hipEventDestroy(R.ev_join[a]);
            if (R.X[a]) (void)hipStreamDestroy(R.X[a]);
        }
        if (R.own_S) (void)hipStreamDestroy(R.S);
    }
    for (hipEvent_t e : {d->ev_fork, d->ev_t0, d->ev_t1})
        if (e) (void)hipEventDestroy(e);
    for (int a = 0; a < MAX_AXES; a++)
        if (d->own_comm[a] && d->comm[a]) (void)ncclCommDestroy(d->comm[a]);
    if (d->zero) (void)hipFree(d->zero);
    if (d->d_acc) (void)hipFree(d->d_acc);
    if (d->d_root) (void)hipFree(d->d_root);
    delete d;
    c->dist_sub = nullptr;
}

// gm_dist_plan: the plan one rank of an RCCL-mode solve executes, built by the
// same host code as dist_sub_solve (plan_shape, plan_lists, build_ops) but with
// no device or communicator call.
int dist_sub_plan(int heaps, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *off,
                  uint64_t off_cap, uint64_t *n_off, uint32_t *data, uint64_t data_cap, uint64_t *n_data) {
    if (heaps < 1 || heaps > 8 || rank < 0 || rank >= world || !n_off || !n_data) {
        set_error("gm_dist_plan: bad heaps / rank / world");
        return GM_E_ARG;
    }
    Ctx c;
    c.game = GM_GAME_SUBTRACT;
    c.sub.heaps = heaps;
    if (opts) {
        c.dist_batch = std::max(1, (int)opts[0]);
        c.dist_slots = std::max(1, (int)opts[1]);
        c.dist_symmetry = opts[2] & 1;
        c.dist_owner = (opts[2] >> 1) & 1;
    }
    DistSub d;
    GM_TRY(plan_shape(&c, &d, world, false));
    if (axis < 0 || axis >= std::max(1, d.g)) { set_error("gm_dist_plan: axis out of range"); return GM_E_ARG; }
    std::vector<uint32_t> O, D;
    if (what == GM_PLAN_SHAPE) {
        D = {(uint32_t)d.low, (uint32_t)d.high, (uint32_t)d.ntiers, (uint32_t)d.batch, (uint32_t)d.nbatch,
             (uint32_t)d.nslots, (uint32_t)d.g};
        for (int j = 0; j < d.nbatch; j++) { O.push_back((uint32_t)d.lo[j]); O.push_back((uint32_t)d.hi[j]); }
    } else {
        // the last plan is kept (a caller reads one rank's lists with several calls),
        // behind a lock: this context-free entry point may be called from any thread
        static std::mutex mu;
        static std::vector<int> last_key;
        static Plan last;
        std::lock_guard<std::mutex> lock(mu);
        const std::vector<int> key = {heaps, world, rank, d.batch, d.nslots, c.dist_symmetry, c.dist_owner};
        if (key != last_key) {
            last_key.clear();
            last = Plan();
            GM_TRY(plan_lists(&c, &d, rank, last));
            last_key = key;
        }
        const Plan &P = last;
        switch (what) {
        case GM_PLAN_OWN: O = P.off; D = P.own; break;
        case GM_PLAN_FILL: O = P.fill_off; D = P.fill; break;
        case GM_PLAN_SEND: O = P.send_off[axis]; D = P.send[axis]; break;
        case GM_PLAN_RECV: O = P.recv_off[axis]; D = P.recv[axis]; break;
        case GM_PLAN_XDEST: O = P.xoff; D = P.xd; break;
        case GM_PLAN_OPS: {
            SubRank R;
            R.rank = rank;
            R.off = P.off;
            R.fill_off = P.fill_off;
            for (int a = 0; a < d.g; a++) { R.send_off[a] = P.send_off[a]; R.recv_off[a] = P.recv_off[a]; }
            build_ops(&d, R);
            for (const Op &o : R.ops) {
                D.push_back(o.kind);
                D.push_back(o.axis);
                D.push_back(o.ev);
                D.push_back(o.on_x);
                D.push_back((uint32_t)o.arg);
                D.push_back((uint32_t)o.peer);
            }
            break;
        }
        default: set_error("gm_dist_plan: unknown `what` %d", what); return GM_E_ARG;
        }
    }
    *n_off = O.size();
    *n_data = D.size();
    if (off) {
        if (off_cap < O.size()) { set_error("gm_dist_plan: off buffer too small"); return GM_E_CAP; }
        std::copy(O.begin(), O.end(), off);
    }
    if (data) {
        if (data_cap < D.size()) { set_error("gm_dist_plan: data buffer too small"); return GM_E_CAP; }
        std::copy(D.begin(), D.end(), data);
    }
    return GM_OK;
}

}  // namespace gm
