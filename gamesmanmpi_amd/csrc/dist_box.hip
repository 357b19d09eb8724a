// dist_box.hip -- the 8-heap synthetic game (config 5) on the box engine, split over G ranks:
// every box computed by exactly ONE rank, cross-rank child boxes handed over per batch of
// box-tiers.
//
// The reference shards positions by an owner hash, md5(str(pos)) % world
// (src/game_state.py:23-31), sends every child to its owner (src/new_process.py:156-160) and
// every result back to the parent's rank (:179-187).  Here the owner of a box is a function
// of its box coordinates (box_common.hpp) with one bit per split AXIS:
//   HALF(d)       bit = [c_d >= thr_d], thr_d = (lim_d + 2) / 2 (2 of 0..3 for an A heap, 4 of
//                 0..7 for a B heap at the full root);
//   CMP(x, y, F)  bit = [c_x < c_y], a tie c_x = c_y = k going to the 1 side only when k is odd
//                 and some heap p of the free set F has c_p != k (tier-balanced: the swap of
//                 x and y maps one side onto the other inside every box-tier).
// A move lowers one heap, so a child box differs from its parent in one coordinate and crosses
// at most one axis.  Children that cross are needed only by the 1 side of the axis (checked
// for every box by the plan; the CMP tie rule is what makes that hold), so each axis carries
// data one way, lower rank -> upper rank (upper = lower | 1 << axis), and ranks can run ahead
// of the ranks they feed.
//
// Symmetric fill (GM_OPT_DIST_SYMMETRY, default on).  Every heap plays by the same rules, so a
// transposition of two A heaps or two B heaps maps a box to a box of equal values in the same
// box-tier (box_common.hpp).  A crossing child C whose image s(C) under some such s is a box
// of the receiving rank -- computed by it in the box-tier before -- is read through s
// (box_tier_kernel<true>, 4 bits per child direction) instead of crossing the link.  Every box
// is still computed by exactly one rank; only the transfer is avoided.
//
// Schedule.  Box-tiers are grouped in batches of B (GM_OPT_DIST_BATCH): batch j = tiers
// [jB, jB+B).  The lower rank's crossing boxes of tiers [jB-1, jB+B-2] (an A-heap crossing: the
// child box's two top layers along that heap, 2 KiB; else the whole 4 KiB box) reach the upper
// rank before its batch j.  The tier kernel writes each such box a second time, from the
// registers that hold it:
//   RCCL transport (GM_OPT_BOX_TRANSPORT 0, any number of nodes): into its slot of the batch's
//     message; after tier jB+B-2 the axis's exchange stream X[a] ncclSends it on the axis's
//     communicator, and the upper rank ncclRecvs and unpacks the batch's messages on its compute
//     stream right before its batch j.  Launched eagerly.
//   IPC transport (1, one node) and virtual ranks (GM_OPT_VIRTUAL_RANKS, testing): straight into
//     the upper rank's table (mapped through hipIpcOpenMemHandle, or the other virtual rank's),
//     the slot the box has there; after the tier one signal per batch -- a one-lane flag kernel
//     (IPC) or an event record (virtual ranks) -- and the upper rank's compute stream waits for
//     it before its batch.  A solve's launches are captured once and replayed as one hipGraph.
// Every rank's work is a precomputed op list (tier launch, unpack, send, receive, event record /
// wait; gm_box_plan shows it on the host); virtual ranks run theirs on per-rank streams and
// tables, enqueued by a host scheduler that interleaves the lists so that every cross-rank wait
// comes after the record it waits for.
#include "gm_internal.hpp"
#include "gm_common.hpp"
#include "box_common.hpp"

#include <algorithm>
#include <mutex>

#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

namespace gm {

enum { BXA_NULL = 0, BXA_HALF = 1, BXA_CMP = 2 };
struct BxAxis {
    int kind = BXA_NULL;
    int d = 0, thr = 0;        // HALF
    int x = 0, y = 0;          // CMP
    uint32_t freemask = 0;     // CMP: heaps of the free set F (bit per heap)
};

struct BxShape {
    int G = 1, g = 0, split = 0, batch = 2, nbatch = 0, ntiers = 0;
    bool fill = true;
    uint32_t root_hi = 0;
    int lim[8] = {};
    BxAxis ax[3];
    std::vector<int> lo, hi;   // per batch: tier range of its message
};

static int bx_axis_bit(const BxAxis &A, uint32_t b) {
    switch (A.kind) {
    case BXA_HALF: return box_coord(b, A.d) >= A.thr;
    case BXA_CMP: {
        const int cx = box_coord(b, A.x), cy = box_coord(b, A.y);
        if (cx != cy) return cx < cy;
        if (!(cx & 1)) return 0;
        for (int p = 0; p < 8; p++)
            if (((A.freemask >> p) & 1u) && box_coord(b, p) != cx) return 1;
        return 0;
    }
    }
    return 0;
}
static int bx_owner(const BxShape &S, uint32_t b) {
    int r = 0;
    for (int a = 0; a < S.g; a++) r |= bx_axis_bit(S.ax[a], b) << a;
    return r;
}
static bool bx_in_region(const BxShape &S, uint32_t b) {
    for (int i = 0; i < 8; i++)
        if (box_coord(b, i) > S.lim[i]) return false;
    return true;
}

// The partition's shape: axes, batches.  Host only, identical on every rank.
static int bx_shape(uint32_t root_hi, int world, int batch, int fill, int split, BxShape *S) {
    if (world < 1) { set_error("bad world %d", world); return GM_E_ARG; }
    if (split < 0 || split > 1) { set_error("box split must be 0 (halves) or 1 (comparisons)"); return GM_E_ARG; }
    S->G = world;
    S->g = 0;
    while (S->g < 3 && (2 << S->g) <= world) S->g++;
    S->split = split;
    S->fill = fill != 0;
    S->root_hi = root_hi;
    S->ntiers = 1;
    for (int i = 0; i < 8; i++) {
        S->lim[i] = box_coord(root_hi, i);
        S->ntiers += S->lim[i];
    }
    bool used[8] = {};
    auto half = [&](int d) {
        BxAxis A;
        A.kind = BXA_HALF;
        A.d = d;
        A.thr = (S->lim[d] + 2) / 2;
        used[d] = true;
        return A;
    };
    // a comparison axis needs a region the swap of x and y maps onto itself, and its free
    // heaps the same range
    auto cmp = [&](int x, int y, std::initializer_list<int> F, BxAxis *out) {
        if (used[x] || used[y] || S->lim[x] != S->lim[y] || S->lim[x] < 1) return false;
        BxAxis A;
        A.kind = BXA_CMP;
        A.x = x;
        A.y = y;
        for (int p : F)
            if (!used[p] && S->lim[p] == S->lim[x]) A.freemask |= 1u << p;
        used[x] = used[y] = true;
        for (int p : F) used[p] = used[p] || ((A.freemask >> p) & 1u);
        *out = A;
        return true;
    };
    int n = 0;
    if (split == 1) {
        // two comparisons with their free heaps, a half split on top at G = 8 (its heap taken
        // from the first comparison's free set): tools/box_split_model.py
        BxAxis A;
        if (S->g >= 2 && cmp(0, 1, S->g >= 3 ? std::initializer_list<int>{2} : std::initializer_list<int>{2, 3}, &A))
            S->ax[n++] = A;
        if (n < S->g && cmp(4, 5, {6, 7}, &A)) S->ax[n++] = A;
    }
    static const int pref[3][3] = {{3, -1, -1}, {3, 7, -1}, {2, 3, 7}};
    static const int order[8] = {3, 7, 2, 6, 1, 5, 0, 4};
    // GM_BOX_SPLIT_HEAPS (development): the half-split heaps, e.g. "1,2,3"
    int envh[3] = {-1, -1, -1};
    if (const char *e = getenv("GM_BOX_SPLIT_HEAPS"))
        for (int k = 0; k < 3 && *e; k++) {
            envh[k] = atoi(e);
            while (*e && *e != ',') e++;
            if (*e == ',') e++;
        }
    if (S->g > 0)
        for (int k = 0; k < 3 && n < S->g; k++) {
            const int d = envh[0] >= 0 ? envh[k] : pref[S->g - 1][k];
            if (d >= 0 && d < 8 && !used[d] && S->lim[d] >= 1) S->ax[n++] = half(d);
        }
    for (int k = 0; k < 8 && n < S->g; k++)
        if (!used[order[k]] && S->lim[order[k]] >= 1) S->ax[n++] = half(order[k]);
    for (; n < S->g; n++) S->ax[n] = BxAxis();   // not splittable: ranks with this bit own nothing
    S->batch = std::max(1, std::min(batch, S->ntiers));
    S->nbatch = (S->ntiers + S->batch - 1) / S->batch;
    S->lo.resize(S->nbatch);
    S->hi.resize(S->nbatch);
    for (int j = 0; j < S->nbatch; j++) {
        S->lo[j] = std::max(0, j * S->batch - 1);
        S->hi[j] = std::min(S->ntiers - 2, j * S->batch + S->batch - 2);
    }
    return GM_OK;
}

// Rank r's part of the plan.  Entries of a message: box | code << 20, code 0 = the whole box,
// 1 + i = the two top layers along A heap i (rows with a_i in {2, 3}).
struct BxPlan {
    std::vector<uint32_t> boxes, fills, tier_off;   // computed boxes by box-tier (Hilbert order), fill words
    std::vector<uint32_t> srcs;                     // per box, 8 per child direction: the box read
    std::vector<uint32_t> dsts;                     // per box, 3: its halo message slots (dense_box.hip BxGroup)
    std::vector<uint32_t> dsts_direct;              // the same slots as kind << 28 | axis << 26 (direct writes)
    std::vector<uint32_t> send_off[3], send[3], recv_off[3], recv[3];   // per axis: per-batch offsets, entries
    uint64_t filled = 0, received = 0;              // child reads through a transposition / from a message
};

static uint32_t bx_entry_bytes(uint32_t e) { return (e >> 20) ? 2048u : 4096u; }

// The boxes rank r computes, by box-tier, and its receive lists (entries per axis and batch).
static int bx_rank_boxes(const BxShape &S, int r, std::vector<uint32_t> &boxes, std::vector<uint32_t> &tier_off) {
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> tiers(S.ntiers);
    for (uint32_t b = 0; b < (1u << 20); b++)
        if (bx_in_region(S, b) && bx_owner(S, b) == r) tiers[box_tier(b)].push_back({box_hilbert(b), b});
    boxes.clear();
    tier_off.assign(1, 0);
    for (auto &tv : tiers) {
        std::sort(tv.begin(), tv.end());
        for (auto &e : tv) boxes.push_back(e.second);
        tier_off.push_back((uint32_t)boxes.size());
    }
    return GM_OK;
}

// Fill words of rank r's boxes and the messages it receives.  Fails if a crossing child
// would have to travel against its axis (the partition's one-way property).
// The kernel's fill word (dense_box.hip BxGroup): per direction 4 bits, an A transposition as
// its digit pair q << 2 | p, a B transposition as 1 + its pair of B heaps.
static int bx_rank_reads(const BxShape &S, int r, const std::vector<uint32_t> &boxes, std::vector<uint32_t> *fills,
                         std::vector<uint32_t> *srcs, std::vector<uint32_t> (&roff)[3], std::vector<uint32_t> (&rent)[3],
                         uint64_t *nfill, uint64_t *nrecv) {
    // per axis and batch: crossing box -> direction mask
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> need(3 * S.nbatch);
    if (fills) fills->assign(boxes.size(), 0);
    if (srcs) srcs->assign(8 * boxes.size(), 0);
    uint64_t nf = 0, nr = 0;
    for (size_t i = 0; i < boxes.size(); i++) {
        const uint32_t P = boxes[i];
        uint32_t f = 0;
        for (int d = 0; d < 8; d++) {
            if (box_coord(P, d) < 1) continue;
            const uint32_t C = P - box_unit(d);
            if (srcs) (*srcs)[8 * i + d] = C;
            const int oc = bx_owner(S, C);
            if (oc == r) continue;
            uint32_t code = 0;
            // the kernel reads an A child through two A heaps, a B child through two B heaps
            if (S.fill)
                for (uint32_t s = d < 4 ? 1u : 7u; s < (d < 4 ? 7u : (uint32_t)BX_NSWAP) && !code; s++) {
                    const uint32_t X = bx_swap_box(s, C);
                    if (X != C && bx_in_region(S, X) && bx_owner(S, X) == r) code = s;
                }
            if (code) {
                const uint32_t kc = d < 4 ? (bx_pair_q(code - 1) << 2 | bx_pair_p(code - 1)) : code - 6;
                f |= kc << (4 * d);
                if (srcs) (*srcs)[8 * i + d] = bx_swap_box(code, C);
                nf++;
                continue;
            }
            const int diff = oc ^ r;
            int a = 0;
            while (a < 3 && diff != (1 << a)) a++;
            if (a >= S.g || !((r >> a) & 1)) {
                set_error("box split: child box %#x of box %#x (rank %d) lies on rank %d, against the axis order",
                          C, P, r, oc);
                return GM_E_STATE;
            }
            const int j = box_tier(P) / S.batch;
            need[3 * j + a].push_back({C, 1u << d});
            nr++;
        }
        if (fills) (*fills)[i] = f;
    }
    for (int a = 0; a < 3; a++) {
        roff[a].assign(1, 0);
        rent[a].clear();
    }
    for (int a = 0; a < S.g; a++) {
        for (int j = 0; j < S.nbatch; j++) {
            auto &v = need[3 * j + a];
            std::sort(v.begin(), v.end());
            for (size_t k = 0; k < v.size();) {
                uint32_t mask = 0;
                const uint32_t C = v[k].first;
                for (; k < v.size() && v[k].first == C; k++) mask |= v[k].second;
                uint32_t code = 0;
                for (int i = 0; i < 4; i++)
                    if (mask == (1u << i)) code = 1 + (uint32_t)i;
                rent[a].push_back(C | code << 20);
            }
            roff[a].push_back((uint32_t)rent[a].size());
        }
    }
    if (nfill) *nfill = nf;
    if (nrecv) *nrecv = nr;
    return GM_OK;
}

// Byte layout of a rank's send (or receive) buffer: axes one after the other, each axis's
// messages in batch order, entries in list order.  eoff[a][k]: entry k's offset; moff[a][j]:
// message j's (moff[a][nbatch] = the axis's end).
static void bx_layout(const BxShape &S, const std::vector<uint32_t> (&off)[3], const std::vector<uint32_t> (&ent)[3],
                      std::vector<uint64_t> (&eoff)[3], std::vector<uint64_t> (&moff)[3], uint64_t *total) {
    uint64_t o = 0;
    for (int a = 0; a < 3; a++) {
        eoff[a].assign(ent[a].size(), 0);
        moff[a].assign(S.nbatch + 1, o);
        if (a >= S.g) continue;
        for (int j = 0; j < S.nbatch; j++) {
            moff[a][j] = o;
            for (uint32_t k = off[a][j]; k < off[a][j + 1]; k++) {
                eoff[a][k] = o;
                o += bx_entry_bytes(ent[a][k]);
            }
        }
        moff[a][S.nbatch] = o;
    }
    *total = o;
}

static int bx_plan(const BxShape &S, int r, BxPlan &P) {
    if (r < 0 || r >= S.G) { set_error("bad rank %d of %d", r, S.G); return GM_E_ARG; }
    GM_TRY(bx_rank_boxes(S, r, P.boxes, P.tier_off));
    GM_TRY(bx_rank_reads(S, r, P.boxes, &P.fills, &P.srcs, P.recv_off, P.recv, &P.filled, &P.received));
    for (int a = 0; a < 3; a++) {
        P.send_off[a].assign(1, 0);
        P.send[a].clear();
    }
    // what this rank sends on an axis where it is the lower side: its upper neighbour's
    // receive list, computed by the same code the neighbour runs
    for (int a = 0; a < S.g; a++) {
        if ((r >> a) & 1) continue;
        const int U = r | (1 << a);
        if (U >= S.G) {
            P.send_off[a].assign(S.nbatch + 1, 0);
            continue;
        }
        std::vector<uint32_t> ub, uoff, roff[3], rent[3];
        GM_TRY(bx_rank_boxes(S, U, ub, uoff));
        GM_TRY(bx_rank_reads(S, U, ub, nullptr, nullptr, roff, rent, nullptr, nullptr));
        P.send_off[a] = roff[a];
        P.send[a] = rent[a];
        for (uint32_t e : P.send[a])
            if (bx_owner(S, e & 0xFFFFFu) != r) { set_error("box split: send list holds a box of another rank"); return GM_E_STATE; }
    }
    for (int a = 0; a < 3; a++) {
        if (P.recv_off[a].size() != (size_t)S.nbatch + 1) P.recv_off[a].assign(S.nbatch + 1, 0);
        if (P.send_off[a].size() != (size_t)S.nbatch + 1) P.send_off[a].assign(S.nbatch + 1, 0);
    }
    // the tier kernel writes each sent box, from its registers, to its message slots: up to
    // one per axis (a box's tier lies in one message's range)
    std::vector<uint64_t> eoff[3], moff[3];
    uint64_t total;
    bx_layout(S, P.send_off, P.send, eoff, moff, &total);
    std::vector<uint32_t> idx(1u << 20, ~0u);
    for (size_t i = 0; i < P.boxes.size(); i++) idx[P.boxes[i]] = (uint32_t)i;
    P.dsts.assign(3 * P.boxes.size(), 0);
    P.dsts_direct.assign(3 * P.boxes.size(), 0);
    for (int a = 0; a < S.g; a++)
        for (size_t k = 0; k < P.send[a].size(); k++) {
            const uint32_t e = P.send[a][k], i = idx[e & 0xFFFFFu], code = e >> 20;
            uint32_t *d = &P.dsts[3 * (size_t)i];
            int slot = 0;
            while (slot < 3 && d[slot]) slot++;
            if (i == ~0u || slot >= 3 || (eoff[a][k] >> 11) >= (1u << 28)) {
                set_error("box split: no destination slot for box %#x", e & 0xFFFFFu);
                return GM_E_STATE;
            }
            d[slot] = (code ? code : 5u) << 28 | (uint32_t)(eoff[a][k] >> 11);
            P.dsts_direct[3 * (size_t)i + slot] = (code ? code : 5u) << 28 | (uint32_t)a << 26;
        }
    return GM_OK;
}

// ---------------------------------------------------------------------------- op lists
enum { BOP_TIER = 0, BOP_PACK = 1, BOP_UNPACK = 2, BOP_SEND = 3, BOP_RECV = 4, BOP_RECORD = 5, BOP_WAIT = 6 };
enum { BEV_DONE = 0, BEV_PACKED = 1, BEV_KINDS = 2 };
struct BxOp {
    uint8_t kind, axis, ev, on_x;   // on_x: runs on X[axis], else on S
    int32_t arg;                    // tier (BOP_TIER) or batch
    int32_t peer;                   // rank whose event (BOP_WAIT) / the other side (BOP_SEND, BOP_RECV)
};

static uint32_t bx_cnt(const std::vector<uint32_t> &off, int j) {
    return (j < 0 || j + 1 >= (int)off.size()) ? 0u : off[j + 1] - off[j];
}

// Rank r's ops, per batch j: its messages' receives on the compute stream S and ONE unpack of
// all of them (the tiers need them, and a cross-stream event wait per batch cost more than
// the ops: profiles/r05b_*), then its tiers; after the tier that ends message jj's range, on
// each axis where it is the lower side, the exchange stream X[a] waits for that tier and sends
// (the tier kernel wrote the message itself: no pack op).
static void bx_build_ops(const BxShape &S, int r, const BxPlan &P, bool loopback, bool direct, std::vector<BxOp> &ops) {
    (void)loopback;
    auto op = [&](int kind, int axis, int ev, bool on_x, int arg, int peer) {
        ops.push_back(BxOp{(uint8_t)kind, (uint8_t)axis, (uint8_t)ev, (uint8_t)on_x, arg, peer});
    };
    ops.clear();
    const int T = S.ntiers, B = S.batch;
    for (int j = 0; j < S.nbatch; j++) {
        bool any = false;
        for (int a = 0; a < S.g; a++) {
            if (!((r >> a) & 1) || !bx_cnt(P.recv_off[a], j)) continue;
            op(BOP_RECV, a, 0, false, j, r ^ (1 << a));
            any = true;
        }
        if (any && !direct) op(BOP_UNPACK, 0, 0, false, j, r);   // direct: the sender wrote the table
        for (int t = j * B; t < std::min(T, j * B + B); t++) {
            op(BOP_TIER, 0, 0, false, t, r);
            for (int jj = 0; jj < S.nbatch; jj++) {
                if (S.hi[jj] != t || S.lo[jj] > S.hi[jj]) continue;
                bool recorded = false;
                for (int a = 0; a < S.g; a++) {
                    if (((r >> a) & 1) || !bx_cnt(P.send_off[a], jj)) continue;
                    if (direct) {   // the boxes are in the receiver's table: signal it, from S
                        op(BOP_SEND, a, 0, false, jj, r | (1 << a));
                        continue;
                    }
                    if (!recorded) op(BOP_RECORD, 0, BEV_DONE, false, jj, r);   // one event per tier
                    recorded = true;
                    op(BOP_WAIT, a, BEV_DONE, true, jj, r);
                    op(BOP_SEND, a, 0, true, jj, r | (1 << a));
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------- kernels
// Unpack: one workgroup of 256 lanes per entry of a batch's messages; a lane moves one 16-B
// row from the receive buffer to the box's slot in the table (a half entry's 128 rows are
// those with a_i in {2, 3}, message row t -> the row whose other digits are t's and whose
// a_i is 2 + bit 2i of t, as the tier kernel wrote them).
__global__ __launch_bounds__(256) void box_unpack_kernel(uint8_t *__restrict__ table, const uint32_t *__restrict__ ent,
                                                         const uint32_t *__restrict__ eoff, const uint8_t *__restrict__ msg) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t e = ent[blockIdx.x], code = e >> 20, t = threadIdx.x;
    uint8_t *b = table + ((uint64_t)(e & 0xFFFFFu) << 12);
    const uint8_t *m = msg + ((uint64_t)eoff[blockIdx.x] << 11);
    uint32_t row = t;
    if (code) {
        if (t >= 128) return;
        const uint32_t i2 = 2u * (code - 1u);
        row = (t & ((1u << i2) - 1u)) | ((2u | ((t >> i2) & 1u)) << i2) | ((t >> (i2 + 1u)) << (i2 + 2u));
    }
    *(u32x4 *)(b + 16u * row) = *(const u32x4 *)(m + 16u * t);
}

// Solo timing (GM_OPT_DIST_SOLO): holds the stream for `ticks` of the 100 MHz realtime clock
// while the host enqueues the rank's list behind it; one wave, ends on time.
__global__ void bx_hold_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// IPC transport (GM_OPT_BOX_TRANSPORT 1): completion flags in device memory, monotone per
// solve (the solve's sequence number), set by one lane with a system-scope release after the
// stream's earlier work, and polled by one lane with system-scope acquire loads.  A wait that
// outlasts its limit (s_memrealtime, 100 MHz) sets *err and ends, so a peer that never
// delivers ends the solve with GM_E_COMM instead of holding the stream.  The sequence number
// lives in device memory (*seqp, advanced by bx_seq_kernel at the start of every solve), so
// a solve replays as one captured graph.
__global__ void bx_seq_kernel(uint64_t *seqp) {
    if (!threadIdx.x) *seqp += 1;
}

// GM_OPT_POISON (test hook): every box this rank receives reads 0xFF until its sender stores it
// again; one workgroup per box, 16 B a lane
__global__ void bx_poison_kernel(uint8_t *table, const uint32_t *boxes) {
    uint4 *b = (uint4 *)(table + ((uint64_t)boxes[blockIdx.x] << 12));
    b[threadIdx.x] = make_uint4(~0u, ~0u, ~0u, ~0u);
}

// GM_OPT_POISON 2 / 3 (test hook): from solve `from` on, hold this stream for `ticks` (a sender
// made late)
__global__ void bx_hold_from_kernel(const uint64_t *seqp, uint64_t from, uint64_t ticks) {
    if (threadIdx.x || *seqp < from) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// waits until *flag >= (*seqp + add) << shift
__global__ void bx_flag_wait_kernel(const uint64_t *flag, const uint64_t *seqp, int add, uint32_t shift, uint64_t ticks,
                                    uint32_t *err) {
    if (threadIdx.x) return;
    // a wait of this solve already timed out: the rest return at once (one 30 s wait per solve
    // at most, not one per batch)
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const int64_t w = (int64_t)*seqp + add;
    const uint64_t want = w > 0 ? (uint64_t)w << shift : 0u;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
            atomicOr(err, 1u);
            return;
        }
        __builtin_amdgcn_s_sleep(4);
    }
}

// the receives of one batch on every axis in one launch: waits until each given flag holds the
// solve's number
// (skip_from > 0, GM_OPT_POISON 2 / 3 test hook: from solve skip_from on, return at once -- a
// receiver that reads its halo as if the flag had been set early)
__global__ void bx_flags_wait_kernel(const uint64_t *f0, const uint64_t *f1, const uint64_t *f2, const uint64_t *seqp,
                                     int add, uint64_t ticks, uint32_t *err, uint64_t skip_from = 0) {
    if (threadIdx.x) return;
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;   // as bx_flag_wait_kernel
    if (skip_from && *seqp >= skip_from) return;
    const int64_t w = (int64_t)*seqp + add;
    const uint64_t want = w > 0 ? (uint64_t)w : 0u;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (const uint64_t *f : {f0, f1, f2}) {
        if (!f) continue;
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                atomicOr(err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(4);
        }
    }
}

__global__ void bx_flags_set_kernel(uint64_t *f0, uint64_t *f1, uint64_t *f2, const uint64_t *seqp) {
    if (threadIdx.x) return;
    const uint64_t v = *seqp;
    __threadfence_system();
    if (f0) __hip_atomic_store(f0, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (f1) __hip_atomic_store(f1, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (f2) __hip_atomic_store(f2, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void bx_mark_kernel(uint32_t *flag, const uint32_t *boxes, uint32_t n, uint32_t ep) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[boxes[i]] = ep;
}

// the root's code, tagged with the solve's sequence number, into every rank's flag block
__global__ void bx_root_post_kernel(const uint8_t *slot, uint64_t *const *words, int n, const uint64_t *seqp) {
    if (threadIdx.x) return;
    const uint64_t v = *seqp << 8 | *slot;
    __threadfence_system();
    for (int i = 0; i < n; i++) __hip_atomic_store(words[i], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint64_t BX_IPC_WAIT_TICKS = 30ull * 100000000ull;   // 30 s

// ---------------------------------------------------------------------------- context
struct BxRank {
    int rank = 0;
    uint8_t *table = nullptr;
    bool owned = false;
    std::vector<uint32_t> tier_off;
    std::vector<uint8_t> tier_fill;       // per tier: some box reads a child through a transposition
    std::vector<uint32_t> boxes;          // host copy
    uint32_t *d_boxes = nullptr, *d_fills = nullptr, *d_srcs = nullptr, *d_dsts = nullptr;
    // one send and one receive buffer; per axis the byte offset of each batch's message
    uint8_t *sbuf = nullptr, *rbuf = nullptr;
    uint64_t sbytes = 0, rbytes = 0;
    std::vector<uint64_t> smoff[3], rmoff[3];
    std::vector<uint32_t> send_off[3], recv_off[3];
    // per batch, the entries of every message it receives, with their offsets / 2 KiB in rbuf
    std::vector<uint32_t> unp_off;
    uint32_t *d_unp_ent = nullptr, *d_unp_eoff = nullptr;
    std::vector<hipEvent_t> ev[BEV_KINDS][3];
    hipEvent_t ev_join[4] = {};
    hipStream_t S = nullptr, X[3] = {};
    bool own_S = false;
    std::vector<BxOp> ops;
    size_t pc = 0;
    int recorded[BEV_KINDS][3] = {};      // batches whose event is enqueued (host order, loopback)
    uint64_t filled = 0, received = 0, sent_bytes = 0;
    // GM_OPT_TIMING 2: an event pair around every op (per-op GPU ms, gm_rank_op_ms)
    std::vector<hipEvent_t> tev;
    std::vector<double> op_ms;
    float span_ms = 0;
    // IPC transport: own flag block {arrived[3][nbatch], consumed[3], root}, error word, and the
    // mapped flag blocks of the ranks this one sends to (their tables: peer_table)
    uint64_t *flags = nullptr;
    uint32_t *d_err = nullptr;
    uint64_t *peer_flags[3] = {};
    uint8_t *peer_table[3] = {};          // direct writes: the table of the rank this one sends to, per axis
    // GM_OPT_BOX_FLOW 1 (split dataflow): group queues, per-box flags (own and received boxes),
    // the receivers' flag arrays, the boxes it receives (solo timing marks them stored)
    uint32_t *d_groups = nullptr, *boxflag = nullptr, *d_recv_boxes = nullptr;
    uint32_t qbase[8] = {}, qlen[8] = {};
    uint32_t *peer_boxflag[3] = {};
    uint32_t n_recv_boxes = 0;
    uint32_t *d_poison_boxes = nullptr;   // GM_OPT_POISON: every box this rank receives
    uint32_t n_poison_boxes = 0;
    int sig_done = 0;                     // direct: batches signalled so far in this solve (+1)
    int rcv_done = 0;                     // IPC: batches whose receives are waited for (+1)
};

struct DistBox {
    BxShape S;
    bool loopback = false;
    int want_batch = 0, want_sym = 0, want_split = 0, want_poison = 0;
    std::vector<BxRank> ranks;            // the ranks this context runs
    int grid_cap = 2048;
    unsigned long long *d_acc = nullptr;
    uint32_t *d_root = nullptr;
    uint8_t *d_owner = nullptr;           // per box id: index into d_tables of its holder (0xFF: none)
    const uint8_t **d_tables = nullptr;
    hipEvent_t ev_fork = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    ncclComm_t comm[3] = {};
    bool own_comm[3] = {};
    uint64_t sent = 0;
    // IPC transport
    bool ipc = false;
    bool direct = false;                  // halo boxes written straight into the receiver's table (loopback, IPC)
    bool flow = false;                    // GM_OPT_BOX_FLOW 1: each rank's chain one dataflow launch
    BxSplitFlowDesc *d_desc = nullptr;    // per rank (index = position in `ranks`)
    uint32_t *d_flow_err = nullptr;
    int flow_grid = 0;
    uint64_t flow_ticks = 0;
    bool flow_sys = false;                // a peer on another GPU: system-scope flag polls and stores
    uint64_t seq = 0;                     // solves run on this context (the flags' values)
    uint64_t *d_seq = nullptr;            // IPC: the same count in device memory (the kernels read it)
    // GM_BOX_SIGNAL_KERNELS=1 (development, virtual ranks): each signal and each receive also
    // launches the IPC transport's one-lane flag kernel (on a scratch flag), so a solo span
    // carries the launches an IPC rank's list holds
    uint64_t *d_scratch = nullptr;
    // virtual ranks and the IPC transport: a solve's launches captured once and replayed as one
    // graph (the op lists are fixed per plan); key = the solo rank it was captured for
    hipGraphExec_t gexec = nullptr;
    hipStream_t graph_stream = nullptr;
    int graph_key = -1;
    bool graph_bad = false;               // capture refused: launch eagerly from then on
    uint64_t graph_sent = 0;
    std::vector<uint64_t> graph_rank_sent;
    std::vector<void *> opened;           // peer mappings (hipIpcCloseMemHandle on free)
    uint64_t **d_root_words = nullptr;    // every rank's root word (the root's owner posts to all)
    int n_root_words = 0;
};

// flag block layout: arrived[a][j] at a * nbatch + j, consumed[a] at 3 * nbatch + a, root word after
static size_t bx_flag_words(const BxShape &S) { return 3 * (size_t)S.nbatch + 4; }
static size_t bx_flag_consumed(const BxShape &S, int a) { return 3 * (size_t)S.nbatch + a; }
static size_t bx_flag_root(const BxShape &S) { return 3 * (size_t)S.nbatch + 3; }

// Rendezvous of the IPC transport: every rank publishes handles of its table (the allocation
// holding it and the table's offset there: an adopted torch tensor may sit inside a larger
// block) and its flag block in a POSIX shared-memory segment named by the unique id and this context's prepare
// count (identical on every rank: prepares are collective), maps the handles of the ranks it
// needs, and rank 0 unlinks the segment once every rank has mapped.
struct BxShmSlot {
    hipIpcMemHandle_t table, flags, boxflag;
    uint64_t table_off, has_table, has_boxflag, pci, ready, mapped;
};

static int bx_ipc_rendezvous(Ctx *c, DistBox *d, BxRank &R) {
    const BxShape &S = d->S;
    char name[96];
    uint64_t k0, k1;
    std::memcpy(&k0, c->uid, 8);
    std::memcpy(&k1, c->uid + 8, 8);
    snprintf(name, sizeof name, "/gmbx-%016llx%016llx-%d", (unsigned long long)k0, (unsigned long long)k1,
             c->box_prepares);
    const size_t bytes = sizeof(BxShmSlot) * (size_t)S.G;
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) { set_error("shm_open(%s) failed", name); return GM_E_COMM; }
    if (ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        set_error("ftruncate of %s failed", name);
        return GM_E_COMM;
    }
    void *m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) { set_error("mmap of %s failed", name); return GM_E_COMM; }
    BxShmSlot *slot = (BxShmSlot *)m;
    int rc = GM_OK;
    auto wait_all = [&](uint64_t BxShmSlot::*field) {
        const double t0 = now_ms();
        for (int r = 0; r < S.G; r++)
            while (__atomic_load_n(&(slot[r].*field), __ATOMIC_ACQUIRE) == 0) {
                if (now_ms() - t0 > 120e3) return false;
                usleep(200);
            }
        return true;
    };
    slot[R.rank].has_table = R.table ? 1 : 0;
    if (R.table) {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)R.table) != hipSuccess ||
            hipIpcGetMemHandle(&slot[R.rank].table, (void *)base) != hipSuccess) {
            (void)hipGetLastError();
            set_error("hipIpcGetMemHandle of rank %d's table failed", R.rank);
            rc = GM_E_COMM;
        }
        slot[R.rank].table_off = (uint64_t)((uint8_t *)R.table - (uint8_t *)base);
    }
    if (rc == GM_OK && hipIpcGetMemHandle(&slot[R.rank].flags, R.flags) != hipSuccess) {
        (void)hipGetLastError();
        set_error("hipIpcGetMemHandle of rank %d's flags failed", R.rank);
        rc = GM_E_COMM;
    }
    slot[R.rank].has_boxflag = R.boxflag ? 1 : 0;
    if (rc == GM_OK && R.boxflag && hipIpcGetMemHandle(&slot[R.rank].boxflag, R.boxflag) != hipSuccess) {
        (void)hipGetLastError();
        set_error("hipIpcGetMemHandle of rank %d's box flags failed", R.rank);
        rc = GM_E_COMM;
    }
    {
        int bus = 0, dev = 0, dom = 0;
        (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->device);
        (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, c->device);
        (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->device);
        slot[R.rank].pci = (uint64_t)(uint32_t)dom << 32 | (uint64_t)(uint32_t)bus << 8 | (uint64_t)(uint32_t)dev;
    }
    __atomic_store_n(&slot[R.rank].ready, rc == GM_OK ? 1 : 2, __ATOMIC_RELEASE);
    if (rc == GM_OK && !wait_all(&BxShmSlot::ready)) {
        set_error("IPC rendezvous %s: not every rank published its handles within 120 s", name);
        rc = GM_E_COMM;
    }
    for (int r = 0; r < S.G && rc == GM_OK; r++)
        if (__atomic_load_n(&slot[r].ready, __ATOMIC_ACQUIRE) != 1) {
            set_error("IPC rendezvous %s: rank %d failed to publish", name, r);
            rc = GM_E_COMM;
        }
    auto open = [&](const hipIpcMemHandle_t &h, void **p) {
        if (hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        d->opened.push_back(*p);
        return true;
    };
    std::vector<uint64_t *> words(S.G, nullptr);
    for (int r = 0; r < S.G && rc == GM_OK; r++) {
        if (r == R.rank) {
            words[r] = R.flags + bx_flag_root(S);
            continue;
        }
        void *f = nullptr;
        if (!open(slot[r].flags, &f)) {
            set_error("hipIpcOpenMemHandle of rank %d's flags failed", r);
            rc = GM_E_COMM;
            break;
        }
        words[r] = (uint64_t *)f + bx_flag_root(S);
        for (int a = 0; a < S.g; a++)
            if (!((R.rank >> a) & 1) && r == (R.rank | (1 << a))) {
                R.peer_flags[a] = (uint64_t *)f;
                if (!slot[r].has_table) continue;   // a rank without boxes receives nothing
                void *b = nullptr;
                if (!open(slot[r].table, &b)) {
                    set_error("hipIpcOpenMemHandle of rank %d's table failed", r);
                    rc = GM_E_COMM;
                    break;
                }
                R.peer_table[a] = (uint8_t *)b + slot[r].table_off;
                if (slot[r].has_boxflag) {
                    void *bf = nullptr;
                    if (!open(slot[r].boxflag, &bf)) {
                        set_error("hipIpcOpenMemHandle of rank %d's box flags failed", r);
                        rc = GM_E_COMM;
                        break;
                    }
                    R.peer_boxflag[a] = (uint32_t *)bf;
                }
            }
    }
    if (rc == GM_OK && d->flow) {   // ranks sharing this GPU run their dataflow launches side by side
        int share = 0;
        for (int r = 0; r < S.G; r++) {
            share += slot[r].pci == slot[R.rank].pci;
            d->flow_sys = d->flow_sys || slot[r].pci != slot[R.rank].pci;
        }
        d->flow_grid = std::max(8, (d->flow_grid / std::max(1, share)) & ~7);
    }
    if (rc == GM_OK) {
        if (hipMalloc(&d->d_root_words, S.G * sizeof(uint64_t *)) != hipSuccess ||
            hipMemcpy(d->d_root_words, words.data(), S.G * sizeof(uint64_t *), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            set_error("root word table");
            rc = GM_E_HIP;
        }
        d->n_root_words = S.G;
    }
    __atomic_store_n(&slot[R.rank].mapped, 1, __ATOMIC_RELEASE);
    if (R.rank == 0) {
        (void)wait_all(&BxShmSlot::mapped);
        shm_unlink(name);
    }
    munmap(m, bytes);
    return rc;
}

static int bx_upload(const std::vector<uint32_t> &v, uint32_t **d) {
    GM_HIP(hipMalloc(d, std::max<size_t>(1, v.size()) * 4));
    if (!v.empty()) GM_HIP(hipMemcpy(*d, v.data(), v.size() * 4, hipMemcpyHostToDevice));
    return GM_OK;
}

void dist_box_free(Ctx *c);

static int bx_prepare(Ctx *c, DistBox *d, uint64_t root, int G, bool loopback) {
    d->loopback = loopback;
    d->want_batch = c->dist_batch;
    d->want_sym = c->dist_symmetry;
    d->want_split = c->box_split;
    d->want_poison = c->poison;
    GM_TRY(bx_shape(box_index_of_key((uint32_t)root) >> 12, G, c->dist_batch, c->dist_symmetry, c->box_split, &d->S));
    const BxShape &S = d->S;
    d->grid_cap = box_grid_cap(c->device);
    d->ipc = !loopback && c->box_transport == 1;
    d->direct = loopback || d->ipc;
    d->flow = d->direct && c->box_flow == 1;
    if (d->flow) {
        d->flow_grid = box_split_flow_resident(c->device) & ~7;
        if (d->flow_grid < 8) { set_error("split dataflow kernel: no resident workgroups"); return GM_E_HIP; }
        // 200 ms of s_memrealtime (100 MHz) for virtual ranks, which start together; 30 s across
        // processes, which reach their launches at their own pace
        d->flow_ticks = d->ipc ? BX_IPC_WAIT_TICKS : (uint64_t)(200.0 * 1e5);
        if (const char *tm = getenv("GM_BOX_FLOW_TIMEOUT_MS")) d->flow_ticks = (uint64_t)(std::max(0.001, atof(tm)) * 1e5);
        GM_HIP(hipMalloc(&d->d_flow_err, 4));
        GM_HIP(hipMemset(d->d_flow_err, 0, 4));
    }
    c->box_prepares++;
    if (d->ipc || (loopback && getenv("GM_BOX_SIGNAL_KERNELS") && atoi(getenv("GM_BOX_SIGNAL_KERNELS")) == 1)) {
        GM_HIP(hipMalloc(&d->d_seq, 8));
        GM_HIP(hipMemset(d->d_seq, 0, 8));
        if (!d->ipc) {
            GM_HIP(hipMalloc(&d->d_scratch, 16));   // flag, error word
            GM_HIP(hipMemset(d->d_scratch, 0, 16));
        }
    }
    GM_HIP(hipMalloc(&d->d_acc, 16));
    GM_HIP(hipMalloc(&d->d_root, 4));
    GM_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    GM_HIP(hipEventCreate(&d->ev_t0));
    GM_HIP(hipEventCreate(&d->ev_t1));
    if (!loopback && !d->ipc) {
        // one communicator per axis; every rank makes the same calls in the same order
        d->comm[0] = c->comm;
        for (int a = 1; a < S.g; a++) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 1;
            GM_NCCL(ncclCommSplit(c->comm, 0, c->rank, &d->comm[a], &cfg));
            d->own_comm[a] = true;
        }
    }
    d->ranks.resize(loopback ? G : 1);
    std::vector<uint8_t> owner(1u << 20, 0xFF);
    std::vector<const uint8_t *> tabs;
    for (size_t i = 0; i < d->ranks.size(); i++) {
        BxRank &R = d->ranks[i];
        R.rank = loopback ? (int)i : c->rank;
        BxPlan P;
        GM_TRY(bx_plan(S, R.rank, P));
        R.tier_off = P.tier_off;
        R.tier_fill.assign(P.tier_off.size(), 0);
        for (size_t t = 0; t + 1 < P.tier_off.size(); t++)
            for (uint32_t k = P.tier_off[t]; k < P.tier_off[t + 1] && !R.tier_fill[t]; k++) R.tier_fill[t] = P.fills[k] != 0;
        R.boxes = P.boxes;
        R.filled = P.filled;
        R.received = P.received;
        GM_TRY(bx_upload(P.boxes, &R.d_boxes));
        GM_TRY(bx_upload(P.fills, &R.d_fills));
        GM_TRY(bx_upload(P.srcs, &R.d_srcs));
        GM_TRY(bx_upload(d->direct ? P.dsts_direct : P.dsts, &R.d_dsts));
        std::vector<uint64_t> seoff[3], reoff[3];
        bx_layout(S, P.send_off, P.send, seoff, R.smoff, &R.sbytes);
        bx_layout(S, P.recv_off, P.recv, reoff, R.rmoff, &R.rbytes);
        for (uint64_t bytes : {R.sbytes, R.rbytes})
            if ((bytes >> 11) >= (1u << 28)) { set_error("halo buffer of %llu bytes", (unsigned long long)bytes); return GM_E_STATE; }
        if (!d->direct) {   // messages: a send buffer the tier kernel fills, a receive buffer to unpack
            GM_HIP(hipMalloc(&R.sbuf, std::max<uint64_t>(16, R.sbytes)));
            GM_HIP(hipMalloc(&R.rbuf, std::max<uint64_t>(16, R.rbytes)));
            std::vector<uint32_t> ue, uo;
            R.unp_off.assign(1, 0);
            for (int j = 0; j < S.nbatch; j++) {
                for (int a = 0; a < S.g; a++)
                    for (uint32_t k = P.recv_off[a][j]; k < P.recv_off[a][j + 1]; k++) {
                        ue.push_back(P.recv[a][k]);
                        uo.push_back((uint32_t)(reoff[a][k] >> 11));
                    }
                R.unp_off.push_back((uint32_t)ue.size());
            }
            GM_TRY(bx_upload(ue, &R.d_unp_ent));
            GM_TRY(bx_upload(uo, &R.d_unp_eoff));
        }
        for (int a = 0; a < 3; a++) {
            R.send_off[a] = P.send_off[a];
            R.recv_off[a] = P.recv_off[a];
        }
        if (c->poison) {
            std::vector<uint32_t> pb;
            for (int a = 0; a < S.g; a++)
                for (uint32_t e : P.recv[a]) pb.push_back(e & 0xFFFFFu);
            std::sort(pb.begin(), pb.end());
            pb.erase(std::unique(pb.begin(), pb.end()), pb.end());
            R.n_poison_boxes = (uint32_t)pb.size();
            if (!pb.empty()) GM_TRY(bx_upload(pb, &R.d_poison_boxes));
        }
        if (d->ipc) {
            GM_HIP(hipMalloc(&R.flags, bx_flag_words(S) * 8));
            GM_HIP(hipMemset(R.flags, 0, bx_flag_words(S) * 8));
            GM_HIP(hipMalloc(&R.d_err, 4));
            GM_HIP(hipMemset(R.d_err, 0, 4));
        }
        // one completion event per batch the rank sends (slot 0: all axes share it)
        R.ev[BEV_DONE][0].assign(S.nbatch, nullptr);
        for (int j = 0; j < S.nbatch; j++) {
            bool any = false;
            for (int a = 0; a < S.g; a++) any |= bx_cnt(P.send_off[a], j) != 0;
            if (any) GM_HIP(hipEventCreateWithFlags(&R.ev[BEV_DONE][0][j], hipEventDisableTiming));
        }
        bx_build_ops(S, R.rank, P, loopback, d->direct, R.ops);
        if (d->flow) {   // queues as the one-GPU dataflow launch's: per XCD run x, tier after tier
            std::vector<uint32_t> q[8];
            for (size_t t = 0; t + 1 < R.tier_off.size(); t++) {
                const uint32_t o0 = R.tier_off[t], nb = R.tier_off[t + 1] - o0, ng = (nb + 1) / 2;
                const uint32_t qq = ng >> 3, rr = ng & 7u;
                for (uint32_t x = 0; x < 8; x++) {
                    const uint32_t g0 = x * qq + std::min(x, rr), g1 = g0 + qq + (x < rr ? 1u : 0u);
                    for (uint32_t g = g0; g < g1; g++)
                        q[x].push_back((o0 + 2 * g) | ((2 * g + 1 < nb) ? 1u << 31 : 0u));
                }
            }
            std::vector<uint32_t> all;
            for (int x = 0; x < 8; x++) {
                R.qbase[x] = (uint32_t)all.size();
                R.qlen[x] = (uint32_t)q[x].size();
                all.insert(all.end(), q[x].begin(), q[x].end());
            }
            GM_TRY(bx_upload(all, &R.d_groups));
            GM_HIP(hipMalloc(&R.boxflag, (1u << 20) * 4));
            GM_HIP(hipMemset(R.boxflag, 0, (1u << 20) * 4));
            std::vector<uint32_t> rb;
            for (int a = 0; a < S.g; a++)
                for (uint32_t e : P.recv[a]) rb.push_back(e & 0xFFFFFu);
            R.n_recv_boxes = (uint32_t)rb.size();
            GM_TRY(bx_upload(rb, &R.d_recv_boxes));
        }
        for (auto &e : R.ev_join) GM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // the table: a rank without boxes holds none
        if (!loopback && c->adopted_dense) {
            if (c->adopted_dense_bytes < (1ull << 32)) { set_error("adopted dense table too small"); return GM_E_CAP; }
            R.table = (uint8_t *)c->adopted_dense;
        } else if (!P.boxes.empty()) {
            if (hipMalloc(&R.table, 1ull << 32) != hipSuccess) {
                (void)hipGetLastError();
                set_error("hipMalloc of a 4 GiB rank table failed (rank %d)", R.rank);
                return GM_E_NOMEM;
            }
            R.owned = true;
        }
        // every rank's table starts as 0xFF (LOSS in 0, the largest code): a read of a box the
        // rank neither computed nor received changes its results instead of reading leftover
        // bytes (a fresh allocation or an adopted buffer); once per prepare, before the IPC
        // rendezvous lets a peer store into it
        if (R.table) GM_HIP(hipMemset(R.table, 0xFF, 1ull << 32));
        if (R.table) {
            for (uint32_t b : P.boxes) owner[b] = (uint8_t)tabs.size();
            tabs.push_back(R.table);
        }
        if (loopback) {
            GM_HIP(hipStreamCreateWithFlags(&R.S, hipStreamNonBlocking));
            R.own_S = true;
        }
        for (int a = 0; a < S.g; a++) GM_HIP(hipStreamCreateWithFlags(&R.X[a], hipStreamNonBlocking));
    }
    if (loopback)   // direct writes: a lower rank's tier kernel stores its halo boxes into the upper's table
        for (auto &R : d->ranks)
            for (int a = 0; a < S.g; a++)
                if (!((R.rank >> a) & 1) && (R.rank | (1 << a)) < G) {
                    R.peer_table[a] = d->ranks[R.rank | (1 << a)].table;
                    R.peer_boxflag[a] = d->ranks[R.rank | (1 << a)].boxflag;
                }
    if (d->ipc) {
        GM_HIP(hipDeviceSynchronize());   // buffers zeroed before any peer can write into them
        GM_TRY(bx_ipc_rendezvous(c, d, d->ranks[0]));
    }
    if (d->flow) {
        std::vector<BxSplitFlowDesc> desc(d->ranks.size());
        for (size_t i = 0; i < d->ranks.size(); i++) {
            const BxRank &R = d->ranks[i];
            BxSplitFlowDesc &D = desc[i];
            D.table = R.table;
            D.boxes = R.d_boxes;
            D.fills = R.d_fills;
            D.srcs = R.d_srcs;
            D.dsts = R.d_dsts;
            D.groups = R.d_groups;
            for (int x = 0; x < 8; x++) {
                D.qbase[x] = R.qbase[x];
                D.qlen[x] = R.qlen[x];
            }
            D.flag = R.boxflag;
            for (int a = 0; a < 3; a++) {
                D.ptab[a] = R.peer_table[a];
                D.pflag[a] = R.peer_boxflag[a];
            }
        }
        GM_HIP(hipMalloc(&d->d_desc, desc.size() * sizeof(BxSplitFlowDesc)));
        GM_HIP(hipMemcpy(d->d_desc, desc.data(), desc.size() * sizeof(BxSplitFlowDesc), hipMemcpyHostToDevice));
    }
    GM_HIP(hipMalloc(&d->d_owner, 1u << 20));
    GM_HIP(hipMemcpy(d->d_owner, owner.data(), 1u << 20, hipMemcpyHostToDevice));
    GM_HIP(hipMalloc(&d->d_tables, std::max<size_t>(1, tabs.size()) * sizeof(uint8_t *)));
    if (!tabs.empty())
        GM_HIP(hipMemcpy(d->d_tables, tabs.data(), tabs.size() * sizeof(uint8_t *), hipMemcpyHostToDevice));
    return GM_OK;
}

static int bx_exec(Ctx *c, DistBox *d, BxRank &R, size_t i, bool solo, bool op_events) {
    const BxOp &o = R.ops[i];
    const int a = o.axis, j = o.arg;
    hipStream_t st = o.on_x ? R.X[a] : R.S;
    const bool timed = op_events && o.kind != BOP_RECORD && o.kind != BOP_WAIT;
    if (timed) GM_HIP(hipEventRecord(R.tev[2 * i], st));
    switch (o.kind) {
    case BOP_TIER: {
        const uint32_t nb = R.tier_off[j + 1] - R.tier_off[j];
        if (nb) {
            const uint32_t ng = (nb + 1) / 2;
            const uint32_t grid = std::max<uint32_t>(8u, std::min<uint32_t>(ng, (uint32_t)d->grid_cap));
            const size_t o0 = R.tier_off[j];
            box_launch_tier_split(grid, R.table, R.d_boxes + o0, R.d_fills + o0, R.d_srcs + 8 * o0, R.d_dsts + 3 * o0,
                                  R.sbuf, d->direct ? R.peer_table : nullptr, nb, R.tier_fill[j] != 0, st);
        }
        break;
    }
    case BOP_UNPACK: {
        const uint32_t n = bx_cnt(R.unp_off, j);
        if (n)
            hipLaunchKernelGGL(box_unpack_kernel, dim3(n), dim3(256), 0, st, R.table, R.d_unp_ent + R.unp_off[j],
                               R.d_unp_eoff + R.unp_off[j], R.rbuf);
        break;
    }
    case BOP_PACK:   // fused into the tier kernel
        set_error("unexpected op %d", (int)o.kind);
        return GM_E_STATE;
    case BOP_SEND: {
        const uint64_t o0 = R.smoff[a][j], n = R.smoff[a][j + 1] - o0;
        if (d->direct) {   // the tier kernels wrote the boxes into the receiver's table: tell it
            if (R.sig_done != j + 1) {   // one signal per batch for every axis (bx_advance groups them)
                R.sig_done = j + 1;
                if (d->ipc) {
                    uint64_t *f[3] = {nullptr, nullptr, nullptr};
                    for (size_t k = i; k < R.ops.size() && R.ops[k].kind == BOP_SEND && R.ops[k].arg == j; k++)
                        f[R.ops[k].axis] = R.peer_flags[R.ops[k].axis] + (size_t)R.ops[k].axis * d->S.nbatch + j;
                    hipLaunchKernelGGL(bx_flags_set_kernel, dim3(1), dim3(64), 0, st, f[0], f[1], f[2],
                                       (const uint64_t *)d->d_seq);
                } else {
                    if (d->d_scratch)
                        hipLaunchKernelGGL(bx_flags_set_kernel, dim3(1), dim3(64), 0, st, d->d_scratch, (uint64_t *)nullptr,
                                           (uint64_t *)nullptr, (const uint64_t *)d->d_seq);
                    GM_HIP(hipEventRecord(R.ev[BEV_DONE][0][j], st));
                    R.recorded[BEV_DONE][0] = j + 1;
                }
            }
        } else {
            // pieces of <= 1 GiB (one ncclSend above 2 GiB arrived corrupted, csrc/dist_sparse.hip)
            for (uint64_t p = 0; p < n; p += 1ull << 30)
                GM_NCCL(ncclSend(R.sbuf + o0 + p, std::min<uint64_t>(n - p, 1ull << 30), ncclUint8, o.peer, d->comm[a],
                                 st));
        }
        R.sent_bytes += n;
        if (!d->loopback) d->sent += n;   // loopback counts each message once, at its receive
        break;
    }
    case BOP_RECV: {
        const uint64_t o0 = R.rmoff[a][j], n = R.rmoff[a][j + 1] - o0;
        if (d->loopback) {   // direct writes: the boxes are in place once the sender's tier passed
            const BxRank &L = d->ranks[o.peer];
            if (L.smoff[a][j + 1] - L.smoff[a][j] != n || bx_cnt(L.send_off[a], j) != bx_cnt(R.recv_off[a], j)) {
                set_error("box split: rank %d's message %d on axis %d disagrees with rank %d's", o.peer, j, a, R.rank);
                return GM_E_STATE;
            }
            // solo timing: the other ranks' boxes are taken as written (the previous full solve's)
            if (!solo) GM_HIP(hipStreamWaitEvent(st, L.ev[BEV_DONE][0][j], 0));
            if (d->d_scratch && R.rcv_done != j + 1) {   // one wait per batch, as IPC (the flag holds 0: at once)
                R.rcv_done = j + 1;
                hipLaunchKernelGGL(bx_flag_wait_kernel, dim3(1), dim3(64), 0, st, (const uint64_t *)d->d_scratch,
                                   (const uint64_t *)d->d_seq, -(1 << 30), 0u, BX_IPC_WAIT_TICKS, (uint32_t *)(d->d_scratch + 1));
            }
            d->sent += n;
        } else if (d->ipc) {   // the sender's tier kernels stored the boxes here; wait for its flags
            if (R.rcv_done != j + 1) {   // one wait for the batch's receives on every axis
                R.rcv_done = j + 1;
                const uint64_t *f[3] = {nullptr, nullptr, nullptr};
                for (size_t k = i; k < R.ops.size() && R.ops[k].kind == BOP_RECV && R.ops[k].arg == j; k++)
                    f[R.ops[k].axis] = R.flags + (size_t)R.ops[k].axis * d->S.nbatch + j;
                hipLaunchKernelGGL(bx_flags_wait_kernel, dim3(1), dim3(64), 0, st, f[0], f[1], f[2],
                                   (const uint64_t *)d->d_seq, 0, BX_IPC_WAIT_TICKS, R.d_err,
                                   (uint64_t)(c->poison >= 2 ? 2 : 0));
            }
        } else {
            for (uint64_t p = 0; p < n; p += 1ull << 30)
                GM_NCCL(ncclRecv(R.rbuf + o0 + p, std::min<uint64_t>(n - p, 1ull << 30), ncclUint8, o.peer, d->comm[a], st));
        }
        break;
    }
    case BOP_RECORD:   // a tier's completion (one event per rank and batch: slot 0)
        GM_HIP(hipEventRecord(R.ev[BEV_DONE][0][j], st));
        break;
    case BOP_WAIT:
        GM_HIP(hipStreamWaitEvent(st, R.ev[BEV_DONE][0][j], 0));
        break;
    }
    if (timed) GM_HIP(hipEventRecord(R.tev[2 * i + 1], st));
    return GM_OK;
}

// Run a rank's ops from R.pc while they do not wait for another rank's unrecorded event.
// (RCCL mode: one receive per axis and batch, issued one after another on S -- no ncclGroup
// across the axes' communicators; the chain of waits runs from higher rank bits to lower ones
// and rank 0 receives nothing, so no cycle can form.)
static int bx_advance(Ctx *c, DistBox *d, BxRank &R, bool solo, bool op_events, bool *progress) {
    while (R.pc < R.ops.size()) {
        const BxOp &o = R.ops[R.pc];
        if (d->loopback && !solo && o.kind == BOP_RECV && d->ranks[o.peer].recorded[BEV_DONE][0] <= o.arg) break;
        GM_TRY(bx_exec(c, d, R, R.pc, solo, op_events));
        R.pc++;
        *progress = true;
    }
    return GM_OK;
}

// Enqueue one whole solve.  RCCL mode: the single rank's list in order.  Loopback: round-robin
// over the ranks, each running until its next op waits on an event another rank has not
// enqueued yet.  solo > 0 (GM_OPT_DIST_SOLO, loopback): rank solo - 1's list alone, its
// cross-rank waits dropped -- its own GPU critical path; the other ranks' messages of the
// previous full solve stand in for its inputs.
static int bx_enqueue(Ctx *c, DistBox *d, int solo, bool op_events) {
    for (auto &R : d->ranks) {
        R.pc = 0;
        R.sig_done = 0;
        R.rcv_done = 0;
        for (auto &k : R.recorded)
            for (int &x : k) x = 0;
        if (op_events && R.tev.size() != 2 * R.ops.size()) {
            for (auto e : R.tev) (void)hipEventDestroy(e);
            R.tev.assign(2 * R.ops.size(), nullptr);
            for (auto &e : R.tev) GM_HIP(hipEventCreate(&e));
        }
    }
    d->sent = 0;
    for (auto &R : d->ranks) R.sent_bytes = 0;
    bool progress = false;
    if (solo > 0) {
        if (!d->loopback || solo > (int)d->ranks.size()) { set_error("dist_solo needs loopback ranks"); return GM_E_ARG; }
        GM_TRY(bx_advance(c, d, d->ranks[solo - 1], true, op_events, &progress));
        GM_HIP(hipGetLastError());
        return GM_OK;
    }
    for (;;) {
        bool done = true;
        progress = false;
        for (auto &R : d->ranks) {
            GM_TRY(bx_advance(c, d, R, false, op_events, &progress));
            done &= R.pc == R.ops.size();
        }
        if (done) break;
        if (!progress) { set_error("box split schedule cannot make progress"); return GM_E_STATE; }
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

// One solve: fork every rank's streams off the caller's stream, enqueue, join.  Launches are
// eager: in RCCL mode a stream capture refused half-way would leave the ranks' point-to-point
// sequence numbers out of step.
static int bx_run(Ctx *c, DistBox *d, bool op_events) {
    hipStream_t H = c->stream;
    if (!d->loopback) d->ranks[0].S = c->stream;
    GM_HIP(hipEventRecord(d->ev_fork, H));
    for (auto &R : d->ranks) {
        if (R.S != H) GM_HIP(hipStreamWaitEvent(R.S, d->ev_fork, 0));
        for (int a = 0; a < d->S.g; a++) GM_HIP(hipStreamWaitEvent(R.X[a], d->ev_fork, 0));
    }
    if (d->ipc) {
        hipLaunchKernelGGL(bx_seq_kernel, dim3(1), dim3(64), 0, d->ranks[0].S, d->d_seq);   // this solve's number
        // the ranks this one writes into finished reading the previous solve's halos (one launch)
        for (auto &R : d->ranks) {
            const uint64_t *f[3] = {nullptr, nullptr, nullptr};
            bool any = false;
            for (int a = 0; a < d->S.g; a++)
                if (R.peer_flags[a]) {
                    f[a] = R.peer_flags[a] + bx_flag_consumed(d->S, a);
                    any = true;
                }
            if (any)
                hipLaunchKernelGGL(bx_flags_wait_kernel, dim3(1), dim3(64), 0, R.S, f[0], f[1], f[2],
                                   (const uint64_t *)d->d_seq, -1, BX_IPC_WAIT_TICKS, R.d_err, (uint64_t)0);
            if (c->poison >= 2 && R.rank == 0)   // test hook: rank 0 (it only sends) late from solve 2 on
                hipLaunchKernelGGL(bx_hold_from_kernel, dim3(1), dim3(64), 0, R.S, (const uint64_t *)d->d_seq,
                                   (uint64_t)2, (uint64_t)(50 * 100000));
        }
    }
    if (d->flow) {
        // one launch: every virtual rank together (co-resident), a solo rank alone (its received
        // boxes marked stored: the previous full solve's stand in), or this process's rank
        const uint32_t ep = (uint32_t)d->seq;
        if (d->loopback && c->dist_solo > 0) {
            const int r = c->dist_solo - 1;
            if (r >= (int)d->ranks.size()) { set_error("dist_solo out of range"); return GM_E_ARG; }
            BxRank &R = d->ranks[r];
            if (R.n_recv_boxes)
                hipLaunchKernelGGL(bx_mark_kernel, dim3((R.n_recv_boxes + 255) / 256), dim3(256), 0, R.S, R.boxflag,
                                   (const uint32_t *)R.d_recv_boxes, R.n_recv_boxes, ep);
            box_launch_split_flow((uint32_t)d->flow_grid, d->d_desc + r, 1, ep, d->d_flow_err, d->flow_ticks, false, R.S);
        } else if (d->loopback) {
            const uint32_t n = (uint32_t)d->ranks.size();
            box_launch_split_flow(std::max<uint32_t>(8 * n, (uint32_t)d->flow_grid / n * n), d->d_desc, n, ep,
                                  d->d_flow_err, d->flow_ticks, false, d->ranks[0].S);
        } else {
            box_launch_split_flow((uint32_t)d->flow_grid, d->d_desc, 1, ep, d->d_flow_err, d->flow_ticks, d->flow_sys,
                                  d->ranks[0].S);
        }
        for (auto &R : d->ranks) R.sent_bytes = 0;
        d->sent = 0;
        for (auto &R : d->ranks)
            for (int a = 0; a < d->S.g; a++)
                for (int j = 0; j < d->S.nbatch; j++)
                    if (!d->loopback || !c->dist_solo) d->sent += R.smoff[a][j + 1] - R.smoff[a][j];
    } else {
        GM_TRY(bx_enqueue(c, d, c->dist_solo, op_events));
    }
    if (c->poison == 1 || c->poison == 2)   // test hook: the halo boxes just read go back to 0xFF before the senders may store the next solve's
        for (auto &R : d->ranks)
            if (R.n_poison_boxes)
                hipLaunchKernelGGL(bx_poison_kernel, dim3(R.n_poison_boxes), dim3(256), 0, R.S, R.table,
                                   (const uint32_t *)R.d_poison_boxes);
    if (d->ipc)   // this solve's halos are read: the senders may write the next solve's (one launch)
        for (auto &R : d->ranks) {
            uint64_t *f[3] = {nullptr, nullptr, nullptr};
            bool any = false;
            for (int a = 0; a < d->S.g; a++)
                if ((R.rank >> a) & 1) {
                    f[a] = R.flags + bx_flag_consumed(d->S, a);
                    any = true;
                }
            if (any)
                hipLaunchKernelGGL(bx_flags_set_kernel, dim3(1), dim3(64), 0, R.S, f[0], f[1], f[2],
                                   (const uint64_t *)d->d_seq);
        }
    for (auto &R : d->ranks) {
        for (int a = 0; a < d->S.g; a++) {
            GM_HIP(hipEventRecord(R.ev_join[a], R.X[a]));
            GM_HIP(hipStreamWaitEvent(R.S, R.ev_join[a], 0));
        }
        if (R.S != H) {
            GM_HIP(hipEventRecord(R.ev_join[3], R.S));
            GM_HIP(hipStreamWaitEvent(H, R.ev_join[3], 0));
        }
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

// A solve's launches.  Virtual ranks and the IPC transport (every op a kernel launch, an event
// record / wait or a flag kernel reading the device-side sequence number) capture them once
// per plan and solo rank and replay the graph: the tier launches then follow each other with
// no per-launch gap.  RCCL mode launches eagerly (a capture refused half-way would leave the
// ranks' point-to-point sequence numbers out of step); so do per-op timing (GM_OPT_TIMING 2)
// and the dataflow launch, and GM_OPT_GRAPH 0.
static int bx_launch(Ctx *c, DistBox *d, bool op_events) {
    hipStream_t H = c->stream;
    if (!c->use_graph || op_events || d->flow || !(d->loopback || d->ipc) || d->graph_bad) return bx_run(c, d, op_events);
    const int key = d->loopback ? c->dist_solo : 0;
    if (!d->gexec || d->graph_key != key || d->graph_stream != H) {
        if (d->gexec) {
            (void)hipGraphExecDestroy(d->gexec);
            d->gexec = nullptr;
        }
        hipGraph_t g = nullptr;
        if (hipStreamBeginCapture(H, hipStreamCaptureModeThreadLocal) != hipSuccess) {   // e.g. a legacy stream
            (void)hipGetLastError();
            d->graph_bad = true;
            return bx_run(c, d, false);
        }
        const int rc = bx_run(c, d, false);
        const hipError_t e = hipStreamEndCapture(H, &g);
        if (rc != GM_OK) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        if (e != hipSuccess || !g || hipGraphInstantiate(&d->gexec, g, nullptr, nullptr, 0) != hipSuccess) {
            (void)hipGetLastError();
            if (g) (void)hipGraphDestroy(g);
            d->gexec = nullptr;
            d->graph_bad = true;   // nothing of the capture ran: launch the same ops eagerly
            return bx_run(c, d, false);
        }
        (void)hipGraphDestroy(g);
        d->graph_key = key;
        d->graph_stream = H;
        d->graph_sent = d->sent;
        d->graph_rank_sent.clear();
        for (auto &R : d->ranks) d->graph_rank_sent.push_back(R.sent_bytes);
    }
    d->sent = d->graph_sent;   // the host counts of the captured enqueue
    for (size_t i = 0; i < d->ranks.size(); i++) d->ranks[i].sent_bytes = d->graph_rank_sent[i];
    GM_HIP(hipGraphLaunch(d->gexec, H));
    return GM_OK;
}

int dist_box_solve(Ctx *c, uint64_t root) {
    const bool loopback = c->world <= 1 && c->virtual_ranks > 1;
    const int G = loopback ? c->virtual_ranks : c->world;
    const bool ipc = !loopback && c->box_transport == 1;
    if (!loopback && !ipc && !c->comm) {
        set_error("a %d-rank solve needs an RCCL communicator (gm_set_comm with a unique id)", G);
        return GM_E_COMM;
    }
    if (ipc && !c->have_uid) {
        set_error("the IPC transport needs gm_set_comm with a unique id (it names the rendezvous)");
        return GM_E_COMM;
    }
    DistBox *d = c->dist_box;
    const uint32_t rh = box_index_of_key((uint32_t)root) >> 12;
    if (!d || d->S.G != G || d->loopback != loopback || d->S.root_hi != rh || d->want_batch != c->dist_batch ||
        d->want_sym != c->dist_symmetry || d->want_split != c->box_split || d->want_poison != c->poison ||
        (!loopback && c->adopted_dense && d->ranks[0].table != c->adopted_dense) ||
        (!loopback && d->ranks[0].rank != c->rank) || d->ipc != ipc || d->flow != ((loopback || ipc) && c->box_flow == 1)) {
        dist_box_free(c);
        d = c->dist_box = new DistBox();
        const int rc = bx_prepare(c, d, root, G, loopback);
        if (rc != GM_OK) {
            dist_box_free(c);
            return rc;
        }
    }
    hipStream_t H = c->stream;
    const double t0 = now_ms();
    // GM_OPT_DIST_SOLO with GM_OPT_TIMING: the solo list is enqueued behind a timed hold on the
    // caller's stream (bx_hold_kernel), so every op is queued before the GPU reaches it and the
    // rank's span and per-op times hold no host enqueue gaps
    const bool solo = loopback && c->dist_solo > 0;
    const bool op_events = c->timing >= 2 && !(d->flow);   // a dataflow solve is one op
    if (solo && c->timing) hipLaunchKernelGGL(bx_hold_kernel, dim3(1), dim3(64), 0, H, (uint64_t)(20000 * 100));
    if (ipc || d->flow) d->seq++;   // the flags' value of this solve (IPC transport, dataflow epochs)
    GM_HIP(hipEventRecord(d->ev_t0, H));
    GM_TRY(bx_launch(c, d, op_events));
    GM_HIP(hipEventRecord(d->ev_t1, H));
    const double t_enq = now_ms();
    // root record: the max over ranks of the owner's code (the others contribute 0); with the
    // IPC transport the owner posts it, tagged with the solve's number, to every rank
    const int ro = bx_owner(d->S, rh);
    uint32_t rs = 0;
    if (ipc) {
        BxRank &R = d->ranks[0];
        if (R.rank == ro)
            hipLaunchKernelGGL(bx_root_post_kernel, dim3(1), dim3(64), 0, H, R.table + box_index_of_key((uint32_t)root),
                               d->d_root_words, d->n_root_words, (const uint64_t *)d->d_seq);
        hipLaunchKernelGGL(bx_flag_wait_kernel, dim3(1), dim3(64), 0, H, R.flags + bx_flag_root(d->S),
                           (const uint64_t *)d->d_seq, 0, 8u, BX_IPC_WAIT_TICKS, R.d_err);
        uint64_t w = 0;
        uint32_t err = 0;
        GM_HIP(hipMemcpyAsync(&w, R.flags + bx_flag_root(d->S), 8, hipMemcpyDeviceToHost, H));
        GM_HIP(hipMemcpyAsync(&err, R.d_err, 4, hipMemcpyDeviceToHost, H));
        GM_HIP(hipStreamSynchronize(H));
        if (err) {
            GM_HIP(hipMemset(R.d_err, 0, 4));
            set_error("IPC transport: a peer rank did not deliver within %llu s (solve %llu)",
                      (unsigned long long)(BX_IPC_WAIT_TICKS / 100000000ull), (unsigned long long)d->seq);
            return GM_E_COMM;
        }
        rs = (uint32_t)(w & 0xFF);
    } else {
        GM_HIP(hipMemsetAsync(d->d_root, 0, 4, H));
        for (auto &R : d->ranks)
            if (R.rank == ro && R.table)
                GM_HIP(hipMemcpyAsync(d->d_root, R.table + box_index_of_key((uint32_t)root), 1, hipMemcpyDeviceToDevice,
                                      H));
        if (!loopback) GM_NCCL(ncclAllReduce(d->d_root, d->d_root, 1, ncclUint32, ncclMax, c->comm, H));
        GM_HIP(hipMemcpyAsync(&rs, d->d_root, 4, hipMemcpyDeviceToHost, H));
        GM_HIP(hipStreamSynchronize(H));
    }
    if (d->flow) {
        uint32_t ferr = 0;
        GM_HIP(hipMemcpy(&ferr, d->d_flow_err, 4, hipMemcpyDeviceToHost));
        if (ferr) {
            GM_HIP(hipMemset(d->d_flow_err, 0, 4));
            set_error("split dataflow: a box waited longer than %.0f ms for its child boxes (solve %llu)",
                      d->flow_ticks / 1e5, (unsigned long long)d->seq);
            return GM_E_STATE;
        }
    }
    const double t1 = now_ms();
    c->root_record = record_of_code((uint8_t)rs);
    uint64_t n = 1;
    for (int j = 0; j < 8; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    box_tier_counts(root, c->tier_counts);
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = d->S.ntiers;
    c->stats.world = G;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.forward_ms = t_enq - t0;   // host time spent enqueueing the solve
    c->stats.exchanged_bytes = d->sent;
    c->stats.flow_fallbacks = c->box_flow_fallbacks;
    uint64_t boxes = 0, tables = 0;
    for (auto &R : d->ranks) {
        boxes += R.boxes.size();
        tables += R.owned || (!loopback && R.table) ? 1 : 0;
    }
    c->stats.algo_bytes = (uint64_t)((double)(boxes << 12) * (1.0 + 1.8125 * 8));
    c->stats.table_bytes = tables << 32;
    if (c->timing) {
        float ms = 0;
        GM_HIP(hipEventElapsedTime(&ms, d->ev_t0, d->ev_t1));
        c->stats.kernel_ms = ms;
        int launches = 0;
        for (auto &R : d->ranks) {
            R.op_ms.assign(R.ops.size(), 0.0);
            const bool ran = !c->dist_solo || &R == &d->ranks[c->dist_solo - 1];
            if (!op_events) {   // GM_OPT_TIMING 1: the whole solve (a solo rank's own list) only
                R.span_ms = ran ? ms : 0.0f;
                for (const BxOp &o : R.ops)
                    launches += ran && o.kind == BOP_TIER && R.tier_off[o.arg + 1] > R.tier_off[o.arg];
                continue;
            }
            for (size_t i = 0; i < R.ops.size() && ran; i++) {
                const BxOp &o = R.ops[i];
                if (o.kind == BOP_RECORD || o.kind == BOP_WAIT) continue;
                float m = 0;
                GM_HIP(hipEventElapsedTime(&m, R.tev[2 * i], R.tev[2 * i + 1]));
                R.op_ms[i] = m;
                launches += o.kind == BOP_TIER && R.tier_off[o.arg + 1] > R.tier_off[o.arg];
            }
            // the rank's span: its first op's start to the last op's end on its compute stream
            R.span_ms = 0;
            size_t first = R.ops.size(), last = 0;
            for (size_t i = 0; i < R.ops.size(); i++)
                if (R.ops[i].kind == BOP_TIER) {
                    first = std::min(first, i);
                    last = i;
                }
            if (ran && first < R.ops.size()) GM_HIP(hipEventElapsedTime(&R.span_ms, R.tev[2 * first], R.tev[2 * last + 1]));
        }
        c->stats.kernel_launches = d->flow ? 1 : launches;
    }
    return GM_OK;
}

// ---------------------------------------------------------------------------- results
int dist_box_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    DistBox *d = c->dist_box;
    if (!n) return GM_OK;
    uint64_t *dk;
    uint16_t *dr;
    const uint64_t chunk = std::min<uint64_t>(n, 1ull << 26);
    GM_HIP(hipMalloc(&dk, chunk * 8));
    GM_HIP(hipMalloc(&dr, chunk * 2));
    for (uint64_t o = 0; o < n; o += chunk) {
        const uint64_t m = std::min(chunk, n - o);
        GM_HIP(hipMemcpyAsync(dk, keys + o, m * 8, hipMemcpyHostToDevice, c->stream));
        box_launch_query(d->d_tables, d->d_owner, c->root, dk, dr, m, c->stream);
        GM_HIP(hipMemcpyAsync(recs + o, dr, m * 2, hipMemcpyDeviceToHost, c->stream));
    }
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

// Export: every virtual rank together = the root's region; a rank of a multi-process solve:
// the positions of the boxes it computed, ascending.
int dist_box_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DistBox *d = c->dist_box;
    if (d->loopback) {
        *n = c->n_positions;
        if (!keys) return GM_OK;
        if (cap < c->n_positions) {
            set_error("export buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)c->n_positions);
            return GM_E_CAP;
        }
        box_region_keys(c->root, keys, c->n_positions);
        return dist_box_query(c, keys, recs, c->n_positions);
    }
    std::vector<uint64_t> ks;
    for (uint32_t b : d->ranks[0].boxes)
        for (uint32_t o = 0; o < 4096; o++) {
            const uint32_t k = box_key_of_index((b << 12) | o);
            bool in = true;
            for (int i = 0; i < 8 && in; i++) in = ((k >> (4 * i)) & 15u) <= ((c->root >> (4 * i)) & 15u);
            if (in) ks.push_back(k);
        }
    *n = ks.size();
    if (!keys) return GM_OK;
    if (cap < ks.size()) {
        set_error("export buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)ks.size());
        return GM_E_CAP;
    }
    std::sort(ks.begin(), ks.end());
    std::copy(ks.begin(), ks.end(), keys);
    return dist_box_query(c, keys, recs, ks.size());
}

// Digest of the boxes this context's ranks computed: the whole region over all virtual ranks,
// this rank's part in a multi-process solve (the parts sum to the whole).
int dist_box_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DistBox *d = c->dist_box;
    GM_HIP(hipMemsetAsync(d->d_acc, 0, 16, c->stream));
    for (auto &R : d->ranks)
        if (R.table) box_launch_digest(R.table, R.d_boxes, R.boxes.size(), c->root, d->d_acc, c->stream);
    GM_HIP(hipGetLastError());
    unsigned long long h[2];
    GM_HIP(hipMemcpyAsync(h, d->d_acc, 16, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = h[0];
    *n = h[1];
    return GM_OK;
}

int dist_box_table(Ctx *c, void **p, uint64_t *bytes) {
    DistBox *d = c->dist_box;
    *p = d->ranks[0].table;
    *bytes = d->ranks[0].table ? 1ull << 32 : 0;
    return GM_OK;
}

int dist_box_rank_stats(Ctx *c, double *kernel_ms, uint64_t *boxes, uint64_t *recv_bytes, int cap, int *n) {
    DistBox *d = c->dist_box;
    *n = (int)d->ranks.size();
    if (!kernel_ms && !boxes && !recv_bytes) return GM_OK;
    if (cap < *n) { set_error("rank stats buffer holds %d, need %d", cap, *n); return GM_E_CAP; }
    for (int i = 0; i < *n; i++) {
        if (kernel_ms) kernel_ms[i] = d->ranks[i].span_ms;
        if (boxes) boxes[i] = d->ranks[i].boxes.size();
        if (recv_bytes) recv_bytes[i] = d->ranks[i].rbytes;
    }
    return GM_OK;
}

int dist_box_op_ms(Ctx *c, int rank, double *ms, int cap, int *n) {
    DistBox *d = c->dist_box;
    const BxRank *R = nullptr;
    for (auto &x : d->ranks)
        if (x.rank == rank) R = &x;
    if (!R) { set_error("rank %d is not run by this context", rank); return GM_E_ARG; }
    *n = (int)R->ops.size();
    if (!ms) return GM_OK;
    if (cap < *n) { set_error("op buffer holds %d, need %d", cap, *n); return GM_E_CAP; }
    for (int i = 0; i < *n; i++) ms[i] = i < (int)R->op_ms.size() ? R->op_ms[i] : 0.0;
    return GM_OK;
}

void dist_box_free(Ctx *c) {
    DistBox *d = c->dist_box;
    if (!d) return;
    (void)hipDeviceSynchronize();
    if (d->gexec) (void)hipGraphExecDestroy(d->gexec);
    for (auto &R : d->ranks) {
        if (R.owned && R.table) (void)hipFree(R.table);
        for (void *q : {(void *)R.d_boxes, (void *)R.d_fills, (void *)R.d_srcs, (void *)R.d_dsts, (void *)R.sbuf,
                        (void *)R.rbuf, (void *)R.d_unp_ent, (void *)R.d_unp_eoff})
            if (q) (void)hipFree(q);
        for (int a = 0; a < 3; a++) {
            for (int k = 0; k < BEV_KINDS; k++)
                for (auto e : R.ev[k][a])
                    if (e) (void)hipEventDestroy(e);
            if (R.X[a]) (void)hipStreamDestroy(R.X[a]);
        }
        for (auto e : R.ev_join)
            if (e) (void)hipEventDestroy(e);
        for (auto e : R.tev)
            if (e) (void)hipEventDestroy(e);
        if (R.own_S) (void)hipStreamDestroy(R.S);
    }
    for (hipEvent_t e : {d->ev_fork, d->ev_t0, d->ev_t1})
        if (e) (void)hipEventDestroy(e);
    for (void *q : d->opened) (void)hipIpcCloseMemHandle(q);
    for (auto &R : d->ranks)
        for (void *q : {(void *)R.flags, (void *)R.d_err})
            if (q) (void)hipFree(q);
    if (d->d_root_words) (void)hipFree(d->d_root_words);
    for (auto &R : d->ranks)
        for (void *q : {(void *)R.d_groups, (void *)R.boxflag, (void *)R.d_recv_boxes, (void *)R.d_poison_boxes})
            if (q) (void)hipFree(q);
    for (void *q : {(void *)d->d_desc, (void *)d->d_flow_err})
        if (q) (void)hipFree(q);
    for (int a = 0; a < 3; a++)
        if (d->own_comm[a] && d->comm[a]) (void)ncclCommDestroy(d->comm[a]);
    for (void *q : {(void *)d->d_acc, (void *)d->d_root, (void *)d->d_owner, (void *)d->d_tables, (void *)d->d_seq,
                    (void *)d->d_scratch})
        if (q) (void)hipFree(q);
    delete d;
    c->dist_box = nullptr;
}

// ---------------------------------------------------------------------------- gm_box_plan
// The plan rank `rank` of a `world`-rank split solve executes, built by the same host code as
// dist_box_solve (bx_shape, bx_plan, bx_build_ops) with no device or communicator call.
int dist_box_plan(uint64_t root, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *out,
                  uint64_t cap, uint64_t *n) {
    if (root >> 32) { set_error("root must be a 32-bit key (8 heaps)"); return GM_E_KEY; }
    if (!n) return GM_E_ARG;
    Ctx dflt;
    const int batch = opts ? (int)opts[0] : dflt.dist_batch;
    const int fill = opts ? (int)opts[1] : dflt.dist_symmetry;
    const int split = opts ? (int)opts[2] : dflt.box_split;
    const int loopback = opts ? (int)opts[3] : 0;
    const int transport = opts ? (int)opts[4] : 0;
    BxShape S;
    GM_TRY(bx_shape(box_index_of_key((uint32_t)root) >> 12, world, batch, fill, split, &S));
    if (rank < 0 || rank >= world) { set_error("bad rank %d of %d", rank, world); return GM_E_ARG; }
    if (axis < 0 || axis >= 3) { set_error("axis out of range"); return GM_E_ARG; }
    std::vector<uint32_t> v;
    if (what == GM_BOXPLAN_SHAPE) {
        v = {(uint32_t)S.G, (uint32_t)S.g, (uint32_t)S.ntiers, (uint32_t)S.batch, (uint32_t)S.nbatch, (uint32_t)S.split,
             (uint32_t)S.fill};
        for (int a = 0; a < 3; a++) {
            const BxAxis &A = S.ax[a];
            v.push_back((uint32_t)A.kind);
            v.push_back((uint32_t)(A.kind == BXA_CMP ? A.x : A.d));
            v.push_back((uint32_t)(A.kind == BXA_CMP ? A.y : A.thr));
            v.push_back(A.freemask);
        }
    } else if (what == GM_BOXPLAN_HALO) {
        for (int j = 0; j < S.nbatch; j++) {
            v.push_back((uint32_t)S.lo[j]);
            v.push_back((uint32_t)S.hi[j]);
        }
    } else {
        // the last plan is kept (a caller reads one rank's lists with several calls), behind a
        // lock: this context-free entry point may be called from any thread
        static std::mutex mu;
        static std::vector<uint64_t> last_key;
        static BxPlan last;
        std::lock_guard<std::mutex> lock(mu);
        const std::vector<uint64_t> key = {root, (uint64_t)world, (uint64_t)rank, (uint64_t)S.batch, (uint64_t)S.fill,
                                           (uint64_t)S.split};
        if (key != last_key) {
            last_key.clear();
            last = BxPlan();
            GM_TRY(bx_plan(S, rank, last));
            last_key = key;
        }
        const BxPlan &P = last;
        switch (what) {
        case GM_BOXPLAN_BOXES: v = P.boxes; break;
        case GM_BOXPLAN_FILLS: v = P.fills; break;
        case GM_BOXPLAN_SRCS: v = P.srcs; break;
        case GM_BOXPLAN_DSTS: v = P.dsts; break;
        case GM_BOXPLAN_TIER_OFF: v = P.tier_off; break;
        case GM_BOXPLAN_OWN: v = P.boxes; std::sort(v.begin(), v.end()); break;
        case GM_BOXPLAN_SEND: v = P.send[axis]; break;
        case GM_BOXPLAN_SEND_OFF: v = P.send_off[axis]; break;
        case GM_BOXPLAN_RECV: v = P.recv[axis]; break;
        case GM_BOXPLAN_RECV_OFF: v = P.recv_off[axis]; break;
        case GM_BOXPLAN_OPS: {
            std::vector<BxOp> ops;
            bx_build_ops(S, rank, P, loopback != 0, loopback != 0 || transport == 1, ops);
            for (const BxOp &o : ops) {
                v.push_back(o.kind);
                v.push_back(o.axis);
                v.push_back(o.ev);
                v.push_back(o.on_x);
                v.push_back((uint32_t)o.arg);
                v.push_back((uint32_t)o.peer);
            }
            break;
        }
        case GM_BOXPLAN_COUNTS: v = {(uint32_t)P.boxes.size(), (uint32_t)P.filled, (uint32_t)P.received}; break;
        default: set_error("unknown box plan item %d", what); return GM_E_ARG;
        }
    }
    *n = v.size();
    if (!out) return GM_OK;
    if (cap < v.size()) {
        set_error("box plan buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)v.size());
        return GM_E_CAP;
    }
    std::copy(v.begin(), v.end(), out);
    return GM_OK;
}

}  // namespace gm
