// dense_box.hip -- box-tiled dense retrograde for the 8-heap synthetic subtraction game
// (config 5, GM_OPT_SUB_INTERLEAVE 20).
//
// Replaces, like dense_sub.hip, the reference's per-edge job loop (Process.lookup /
// distribute / resolve, src/new_process.py:102-265) and its shelve tables
// (src/cache_dict.py) for the 2^32-position game: every position gets a 1-byte code
// (gm_common.hpp: WIN R -> R+1, LOSS R -> 255-R), exported as u16 records.
//
// Decomposition.  dense_sub.hip's blocks are the 16^3 positions sharing the high five
// nibbles, so half of a position's 16 children live in 10 other blocks spread over TWO
// block tiers, and every block is read by ten parents in two launches.  Here the
// 16^8 lattice is cut into BOXES of 4 x 4 x 4 x 4 x 2 x 2 x 2 x 2 positions (heaps
// 0-3 in quarters "A", heaps 4-7 in halves "B"): 4,096 positions, 2^20 boxes.  A move
// takes 1 or 2 from one heap, so every child outside a box lies in the box ONE step
// below it along that heap, in that box's top two layers of the heap (half of it
// along an A heap, all of it along a B heap).  Boxes are solved in box-tiers (sum of
// the eight box coordinates, 0..40, one launch each); a launch reads only the tier
// before it, each box once per parent, 5 B of child rows per position instead of 10
// (tools/l2sim_box.cpp: 1.9 B/position of L2 misses modelled, against 3.8 for the
// block order the block engine uses).
//
// Table layout: index = box << 12 | A << 4 | B, with A = a0 + 4 a1 + 16 a2 + 64 a3
// (a_i = heap i mod 4) and B = b0 + 2 b1 + 4 b2 + 8 b3 (b_j = heap 4+j mod 2); the box
// id packs the coordinates h_i >> 2 (2 bits each, bits 0-7) and h_{4+j} >> 1 (3 bits
// each, bits 8-19).  A bit permutation of the key: export, query and digest map it.
//
// One workgroup = ONE wave, solving two boxes at a time (their codes share each LDS
// dword as a u16 pair: low half box 0, high half box 1), persistent over its share of
// the tier:
//   fold   the child rows: per target row (16 positions, one A), the four B-children
//          rows (whole 16-B rows, shifted by one B step where b_j = 0) and, for the rows
//          a3 = 0, 1 this lane owns, heap 3's two top layers of the box below; then per
//          A heap 0-2 those layers merged into the rows a_i = 0, 1 of the image;
//   walk   lane (a0 = lane & 3, b = lane >> 2) walks p = 0..63 (A = a0 + 4 p) starting
//          d = b0 + b1 + 2 (b2 + b3) + a0 steps late, so each child made inside the box
//          is old enough to fetch: the a0 - 1 / a0 - 2 / b0 / b1 children by DPP row_shr
//          1/2/4/8 from the lanes below, the b2 / b3 children from the image in LDS (a
//          zero slot where there is none), (a1, a2) from this lane's own last 1/2/4/8
//          codes (masked at their digit boundaries) and (a3) from its codes 16 and 32
//          steps ago (zero before its start); 73 steps, no barrier;
//   store  16-B rows of both boxes (write-through).
// The max of up to 13 inputs uses v_pk_maximum3_f16: a code 0..255 in the low byte of
// an f16 is a subnormal, ordered like the integer (the kernel keeps f16 denormals,
// .amdhsa_float_denorm_mode_16_64 3).
#include "gm_internal.hpp"
#include "gm_common.hpp"
#include "box_common.hpp"

#include <algorithm>
#include <utility>

namespace gm {

typedef uint32_t bx_u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 bx_h2 __attribute__((ext_vector_type(2)));
typedef uint16_t bx_u16x2 __attribute__((ext_vector_type(2)));

#ifndef GM_BOX_MAX3
#define GM_BOX_MAX3 1          // 1: v_pk_maximum3_f16 on subnormal codes; 0: v_pk_max_u16
#endif
#ifndef GM_BOX_STORE_CPOL
#define GM_BOX_STORE_CPOL 16   // sc1 write-through: a stored box is next read a launch later
#endif
#ifndef GM_BOX_TIER_STORE_CPOL
#define GM_BOX_TIER_STORE_CPOL GM_BOX_STORE_CPOL   // the tier launches' own (the dataflow kernels keep sc1)
#endif
#ifndef GM_BOX_WAVES
#define GM_BOX_WAVES 2         // waves per SIMD the register budget must allow
#endif
#ifndef GM_BOX_SPLIT_PLAIN
#define GM_BOX_SPLIT_PLAIN 1   // split tier kernel: a group without fills issues its loads as at N = 1
#endif
// development ablations (results invalid): bit 1 no walk, 2 no child loads, 4 no stores, 8 no fold;
// split solve: 16 children read as at N = 1 (no fills: exact for rank 0), 32 no halo stores
#ifndef GM_BOX_EXP
#define GM_BOX_EXP 0
#endif
// wave priority per phase (s_setprio): the load issue first (48 instructions), then the
// walk's dependent chain, then the fold, the store last.  The two waves of a SIMD
// otherwise share its issue slots by age: 3.57 ms with none, 3.31 with the walk raised,
// 3.28 with walk 2 / fold 1, ~2 % less again with the load issue at 3.
#ifndef GM_BOX_PRIO_W
#define GM_BOX_PRIO_W 2
#endif
#ifndef GM_BOX_PRIO_F
#define GM_BOX_PRIO_F 1
#endif
#ifndef GM_BOX_PRIO_S
#define GM_BOX_PRIO_S 0
#endif
#ifndef GM_BOX_PRIO_I
#define GM_BOX_PRIO_I 3        // issuing the next group's child loads
#endif

// ---------------------------------------------------------------------------
// device helpers
__device__ __forceinline__ uint32_t bx_max2(uint32_t a, uint32_t b) {
#if GM_BOX_MAX3
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_bit_cast(bx_h2, a),
                                                                     __builtin_bit_cast(bx_h2, b)));
#else
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(bx_u16x2, a),
                                                                 __builtin_bit_cast(bx_u16x2, b)));
#endif
}
__device__ __forceinline__ uint32_t bx_max3(uint32_t a, uint32_t b, uint32_t c) { return bx_max2(bx_max2(a, b), c); }
// parent code of a pair of best-child codes (gm_common.hpp parent_code, per u16 half)
__device__ __forceinline__ uint32_t bx_code(uint32_t m) { return (m ^ 0x00FF00FFu) + ((m >> 6) & 0x00020002u); }
template <int CTRL>
__device__ __forceinline__ uint32_t bx_dpp_shr(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
// x & sext(byte N of m): one masked child per instruction (SDWA), the masks held as bytes
template <int N>
__device__ __forceinline__ uint32_t bx_and_byte(uint32_t x, uint32_t m) {
    uint32_t r;
    if constexpr (N == 0)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
            : "=v"(r) : "v"(x), "v"(m));
    else if constexpr (N == 1)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
            : "=v"(r) : "v"(x), "v"(m));
    else if constexpr (N == 2)
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
            : "=v"(r) : "v"(x), "v"(m));
    else
        asm("v_and_b32_sdwa %0, %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
            : "=v"(r) : "v"(x), "v"(m));
    return r;
}
// LDS ops of one wave complete in order; this keeps the compiler from moving them
#define BX_LDS_ORDER() asm volatile("" ::: "memory")

// 16 codes of box 0 (x0) and box 1 (x1), one 16-B row each -> 16 u16 pairs (b0 | b1 << 16)
__device__ __forceinline__ void bx_pairs(const bx_u32x4 &x0, const bx_u32x4 &x1, uint32_t (&p)[16]) {
#pragma unroll
    for (int b = 0; b < 16; b++) {
        const uint32_t r = (uint32_t)(b & 3);
        p[b] = __builtin_amdgcn_perm(x1[b >> 2], x0[b >> 2], r | 0x0c00u | ((4u + r) << 16) | 0x0c000000u);
    }
}

// Image: position (A, B), A = a0 + 4 p, at dword PITCH p + ASTRIDE a0 + B; dword ZSLOT of
// every p-row is used by no position and kept zero (the walk's slot for a missing b2 / b3
// neighbour).  The walk reads at per-lane offsets + PITCH T (immediates), so the layout must
// stay affine in p; among those layouts the LDS bank model (tools/lds_bank_model.py, the
// CDNA4 rules of MI355X_MICROARCH.md) puts pitch 76 / a0-stride 20 at 15 % fewer LDS cycles
// than round 3's 68 / 16 (walk 921 vs 1079, fold + store 848 vs 1000 per group).
#ifndef GM_BOX_PITCH
#define GM_BOX_PITCH 76
#endif
#ifndef GM_BOX_ASTRIDE
#define GM_BOX_ASTRIDE 20
#endif
#ifndef GM_BOX_ZSLOT
#define GM_BOX_ZSLOT 19
#endif
constexpr int BX_PITCH = GM_BOX_PITCH, BX_AS = GM_BOX_ASTRIDE, BX_Z = GM_BOX_ZSLOT;
// rows stay 16-B aligned for ds_read/write_b128 (pitch 74, 8-B aligned rows: 5.3 ms, not 3.3)
static_assert(BX_PITCH % 4 == 0 && BX_AS % 4 == 0, "16-B aligned image rows");
static_assert(BX_AS >= 16 && 3 * BX_AS + 16 <= BX_PITCH, "a0 sub-rows inside a p-row, disjoint");
static_assert(BX_Z >= 0 && BX_Z < BX_PITCH && !(BX_Z < 16) && !(BX_Z >= BX_AS && BX_Z < BX_AS + 16) &&
                  !(BX_Z >= 2 * BX_AS && BX_Z < 2 * BX_AS + 16) && !(BX_Z >= 3 * BX_AS && BX_Z < 3 * BX_AS + 16),
              "the zero slot is used by no position");
constexpr int BX_IMG = 64 * BX_PITCH;     // dwords
constexpr int BX_PAD = 32;                // guard in front: the walk's (a0-1, a0-2) reads of row 0 at p = 0
constexpr int BX_LDS = BX_PAD + BX_IMG + 64;   // + one dummy dword per lane for idle walk steps
__device__ __forceinline__ uint32_t bx_row(uint32_t A) { return (A >> 2) * BX_PITCH + (uint32_t)BX_AS * (A & 3u); }
constexpr int BX_NLOAD = 48;              // 16-B child rows per lane per group

struct BxGroup {
    uint32_t box[2];
    uint32_t fill[2];   // split solve (dist_box.hip): per child direction d, 4 bits at 4 d: for an A
                        // heap the digit pair (q << 2 | p) of the A transposition the child is read
                        // through (q = p: none), for a B heap 1 + the pair of B heaps (0: none)
    uint32_t srcv;      // split solve: lane 8 k + d holds the box read for box k's child along heap
                        // d (the child box C, or its image under that transposition, which this
                        // rank computed); one VGPR, read with readlane when the loads are issued
    uint32_t dstv;      // split solve: lane 4 k + e (e < 3) holds box k's e-th halo destination: bits
                        // 28-31 kind (0 none, 1-4 the two top layers along A heap kind - 1, 5 the
                        // whole box), bits 0-27 its offset in the send buffer / 2 KiB
    bool valid[2];
};

template <bool SHARD, bool FILL = true>
__device__ __forceinline__ BxGroup bx_group(const uint32_t *__restrict__ boxes, const uint32_t *__restrict__ fills,
                                            const uint32_t *__restrict__ srcs, const uint32_t *__restrict__ dsts,
                                            uint32_t nbox, uint32_t g, uint32_t lane) {
    BxGroup G;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t i = 2 * g + k;
        G.valid[k] = i < nbox;
        G.box[k] = G.valid[k] ? boxes[i] : 0u;
        G.fill[k] = (SHARD && FILL && G.valid[k]) ? fills[i] : 0u;
    }
    G.srcv = G.dstv = 0;
    if constexpr (SHARD) {
        const uint32_t i = 2 * g + (lane >> 3);
        if (FILL && lane < 16 && i < nbox) G.srcv = srcs[8 * i + (lane & 7u)];
        const uint32_t i2 = 2 * g + (lane >> 2);
        if (lane < 8 && (lane & 3u) < 3u && i2 < nbox) G.dstv = dsts[3 * i2 + (lane & 3u)];
    }
    return G;
}
template <bool SHARD>
__device__ __forceinline__ uint32_t bx_src(const BxGroup &G, int k, int d) {
    return (uint32_t)__builtin_amdgcn_readlane((int)G.srcv, 8 * k + d);
}

// Byte B of a child row read through the B transposition of heaps 4 + Q, 4 + P is byte
// swap(B) of the loaded row (bits Q, P of B exchanged): each output dword takes its four
// bytes from at most two loaded dwords, one v_perm_b32.
constexpr int bx_swb(int b, int q, int p) { return b ^ ((((b >> q) ^ (b >> p)) & 1) * ((1 << q) | (1 << p))); }
constexpr int bx_src_lo(int w, int q, int p) {
    int m = 3;
    for (int e = 0; e < 4; e++) m = bx_swb(4 * w + e, q, p) / 4 < m ? bx_swb(4 * w + e, q, p) / 4 : m;
    return m;
}
constexpr int bx_src_hi(int w, int q, int p) {
    int m = 0;
    for (int e = 0; e < 4; e++) m = bx_swb(4 * w + e, q, p) / 4 > m ? bx_swb(4 * w + e, q, p) / 4 : m;
    return m;
}
constexpr uint32_t bx_bsel(int w, int q, int p) {
    uint32_t sel = 0;
    for (int e = 0; e < 4; e++) {
        const int s = bx_swb(4 * w + e, q, p);
        sel |= (uint32_t)((s / 4 == bx_src_lo(w, q, p) ? 0 : 4) + (s & 3)) << (8 * e);
    }
    return sel;
}
template <int Q, int P, int W>
__device__ __forceinline__ uint32_t bx_bsw_dw(const bx_u32x4 &x) {
    constexpr int lo = bx_src_lo(W, Q, P), hi = bx_src_hi(W, Q, P);
    constexpr uint32_t sel = bx_bsel(W, Q, P);
    if constexpr (sel == 0x03020100u) return x[lo];
    return __builtin_amdgcn_perm(x[hi], x[lo], sel);
}
template <int Q, int P>
__device__ __forceinline__ bx_u32x4 bx_bsw(const bx_u32x4 &x) {
    return bx_u32x4{bx_bsw_dw<Q, P, 0>(x), bx_bsw_dw<Q, P, 1>(x), bx_bsw_dw<Q, P, 2>(x), bx_bsw_dw<Q, P, 3>(x)};
}
// a loaded row back to the child's byte order; `code` (1 + pair of B heaps) is uniform
__device__ __forceinline__ bx_u32x4 bx_bswap_row(const bx_u32x4 &x, uint32_t code) {
    switch (code) {
    case 1: return bx_bsw<0, 1>(x);
    case 2: return bx_bsw<0, 2>(x);
    case 3: return bx_bsw<0, 3>(x);
    case 4: return bx_bsw<1, 2>(x);
    case 5: return bx_bsw<1, 3>(x);
    case 6: return bx_bsw<2, 3>(x);
    }
    return x;
}
__device__ __forceinline__ uint32_t bx_fcode(const BxGroup &G, int k, int dir) { return (G.fill[k] >> (4 * dir)) & 15u; }

// Every child row of a group, in flight at once: R[0..31] the B children of target rows
// m = lane + 64 i (R[8 i + 4 k + j]: box k, heap 4 + j), R[32..47] the A children's top
// layers (R[32 + 4 i + 2 k + v]: heap i, box k, layer 3 - v) of the rows a_i in {2, 3}
// whose other coordinates are the lane.
//
// Split solve (SHARD, dist_box.hip): a child box C that this rank neither computes nor
// received is read from its image S = s(C) under a transposition s of two heaps of the child's
// own kind (an A child through two A heaps, a B child through two B heaps); this rank computed
// S in the box-tier before (a transposition keeps the box-tier).  The plan gives per box the
// eight boxes read (scalar loads; computing the swaps here overflowed the SGPRs) and the fill
// word: an A transposition moves rows (row A of C is row swap(A) of S, digits q and p: a
// per-lane address change here), a B transposition permutes the bytes of a row (bx_fold).
template <bool SHARD_, int CPOL = 0, bool PLAIN = false>
__device__ __forceinline__ void bx_issue(const uint8_t *table, const BxGroup &G, uint32_t lane,
                                         bx_u32x4 (&R)[BX_NLOAD]) {
    constexpr bool SHARD = SHARD_ && !(GM_BOX_EXP & 16);
    if constexpr (SHARD && PLAIN)   // a group without fills reads every child where it lies (uniform)
        if (!(G.fill[0] | G.fill[1])) {
            bx_issue<false, CPOL>(table, G, lane, R);
            return;
        }
    const __amdgpu_buffer_rsrc_t rt =
        __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, (GM_BOX_EXP & 2) ? 0u : 0xFFFFFFFFu, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, 0u, 0x00020000);
    // one (descriptor, offset) per child box, used by consecutive loads; a B child read through
    // a B transposition is the same rows of the image box (bytes permuted in bx_fold)
    {
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const bool ok = G.valid[k] && box_coord(G.box[k], 4 + j) >= 1;
                uint32_t src = G.box[k] - box_unit(4 + j);
                if constexpr (SHARD) src = bx_src<SHARD>(G, k, 4 + j);
                const uint32_t soff = ok ? src << 12 : 0u;
                const __amdgpu_buffer_rsrc_t r = ok ? rt : rz;
#pragma unroll
                for (int i = 0; i < 4; i++)
                    R[8 * i + 4 * k + j] = __builtin_bit_cast(
                        bx_u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 16u * (lane + 64u * i), soff, CPOL));
            }
    }
    // an A child read through an A transposition (digits q, p): row A of C is row swap(A) of
    // the image box -- branch-free, shifts of 0 for no transposition
    {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t lo = lane & ((1u << (2 * i)) - 1u), hi = (lane >> (2 * i)) << (2 * i + 2);
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const bool ok = G.valid[k] && box_coord(G.box[k], i) >= 1;
                uint32_t src = G.box[k] - box_unit(i), sq = 0, sp = 0;
                if constexpr (SHARD) {
                    const uint32_t code = bx_fcode(G, k, i);
                    src = bx_src<SHARD>(G, k, i);
                    sq = 2u * (code >> 2);
                    sp = 2u * (code & 3u);
                }
                const uint32_t soff = ok ? src << 12 : 0u;
                const __amdgpu_buffer_rsrc_t r = ok ? rt : rz;
                uint32_t A[2];
#pragma unroll
                for (int v = 0; v < 2; v++) A[v] = lo | ((3u - v) << (2 * i)) | hi;
                if constexpr (SHARD) {   // branch-free: shifts of 0 for no transposition
#pragma unroll
                    for (int v = 0; v < 2; v++) {
                        const uint32_t t = ((A[v] >> sq) ^ (A[v] >> sp)) & 3u;
                        A[v] ^= (t << sq) | (t << sp);
                    }
                }
#pragma unroll
                for (int v = 0; v < 2; v++)
                    R[32 + 4 * i + 2 * k + v] =
                        __builtin_bit_cast(bx_u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 16u * A[v], soff, CPOL));
            }
        }
    }
}

// fold: the image's slot of every position gets the max of its children outside the box
template <bool SHARD_>
__device__ __forceinline__ void bx_fold(uint32_t *s, const BxGroup &G, uint32_t lane, bx_u32x4 (&R)[BX_NLOAD]) {
    constexpr bool SHARD = SHARD_ && !(GM_BOX_EXP & 16);
    if constexpr (SHARD) {   // B children read through a B transposition: back to C's byte order (uniform branches)
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t code = bx_fcode(G, k, 4 + j);
                if (code)
#pragma unroll
                    for (int i = 0; i < 4; i++) R[8 * i + 4 * k + j] = bx_bswap_row(R[8 * i + 4 * k + j], code);
            }
    }
    // B children: row m of the child box below along heap 4 + j; a position with b_j = 0
    // also takes b | e_j of that row (its child two below)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t m = lane + 64u * i;
        // two heaps at a time into F: each position's inputs are its row's code in the four
        // child boxes, and the code one B step up where b_j = 0 (48 maxes per row)
        uint32_t F[16];
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
            uint32_t P[16], Q[16];
            bx_pairs(R[8 * i + jp], R[8 * i + 4 + jp], P);
            bx_pairs(R[8 * i + jp + 1], R[8 * i + 4 + jp + 1], Q);
#pragma unroll
            for (int b = 0; b < 16; b++) {
                uint32_t in[5];
                int n = 0;
                if (jp) in[n++] = F[b];
                in[n++] = P[b];
                in[n++] = Q[b];
                if (!((b >> jp) & 1)) in[n++] = P[b | (1 << jp)];
                if (!((b >> (jp + 1)) & 1)) in[n++] = Q[b | (2 << jp)];
                uint32_t f = n >= 3 ? bx_max3(in[0], in[1], in[2]) : bx_max2(in[0], in[1]);
                if (n == 4) f = bx_max2(f, in[3]);
                if (n == 5) f = bx_max3(f, in[3], in[4]);
                F[b] = f;
            }
        }
        // heap 3's children: rows m = lane + 64 i have a3 = i, so the top layers of the
        // box below along heap 3 that this lane loaded (rows lane + 64 (3 - v)) are its own
        // rows' (a3 = 0 takes layers 3 and 2, a3 = 1 layer 3)
        if (i < 2) {
            uint32_t L3[16], L2[16];
            bx_pairs(R[32 + 12 + 0], R[32 + 12 + 2], L3);
            if (i == 0) bx_pairs(R[32 + 12 + 1], R[32 + 12 + 3], L2);
#pragma unroll
            for (int b = 0; b < 16; b++) F[b] = i == 0 ? bx_max3(F[b], L3[b], L2[b]) : bx_max2(F[b], L3[b]);
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
            *(bx_u32x4 *)(s + bx_row(m) + 4u * q) = bx_u32x4{F[4 * q], F[4 * q + 1], F[4 * q + 2], F[4 * q + 3]};
    }
    BX_LDS_ORDER();
    // A children of heaps 0-2: layers 3 and 2 of the box below along heap i go to the rows
    // a_i = 0 (both) and a_i = 1 (layer 3); one heap after the other (a row can take from
    // several)
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (!((G.valid[0] && box_coord(G.box[0], i) >= 1) || (G.valid[1] && box_coord(G.box[1], i) >= 1))) continue;
        const uint32_t lo = lane & ((1u << (2 * i)) - 1u), hi = (lane >> (2 * i)) << (2 * i + 2);
        uint32_t L3[16], L2[16];
        bx_pairs(R[32 + 4 * i + 0], R[32 + 4 * i + 2], L3);
        bx_pairs(R[32 + 4 * i + 1], R[32 + 4 * i + 3], L2);
        uint32_t *t0 = s + bx_row(lo | hi), *t1 = s + bx_row(lo | (1u << (2 * i)) | hi);
        bx_u32x4 T0[4], T1[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            T0[q] = *(const bx_u32x4 *)(t0 + 4 * q);
            T1[q] = *(const bx_u32x4 *)(t1 + 4 * q);
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int e = 0; e < 4; e++) {
                T0[q][e] = bx_max3(T0[q][e], L3[4 * q + e], L2[4 * q + e]);
                T1[q][e] = bx_max2(T1[q][e], L3[4 * q + e]);
            }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            *(bx_u32x4 *)(t0 + 4 * q) = T0[q];
            *(bx_u32x4 *)(t1 + 4 * q) = T1[q];
        }
        BX_LDS_ORDER();
    }
}

// walk: see the file comment.  The image holds the fold of every position; each code
// overwrites its slot as it is made.
template <int T>
struct BxT { static constexpr int v = T; };
template <class F, int... I>
__device__ __forceinline__ void bx_unroll(F &f, std::integer_sequence<int, I...>) { (f(BxT<I>{}), ...); }

// Lane (a0 = lane bits 0-1, b = lane bits 2-5) starts at step d = (b0 + b1) + 2 (b2 + b3)
// + a0: a step after the lanes one a0 / b0 / b1 step below it, whose codes of the step
// before it takes by DPP (row_shr 1, 2, 4, 8 inside a 16-lane row), and two steps after
// the lanes one b2 / b3 step below (the rows 16 and 32 lanes down), whose codes it reads
// from the image, fetched two steps ahead.
#ifndef GM_BOX_WALK_B01
#define GM_BOX_WALK_B01 0   // 1: the b0 / b1 neighbours from the image too (no DPP; d = S2 popc(b) + a0)
#endif
constexpr int BX_S2 = 2;
constexpr int BX_DMAX = GM_BOX_WALK_B01 ? 4 * BX_S2 + 3 : 2 + 2 * BX_S2 + 3;   // latest start
constexpr int BX_STEPS = 64 + BX_DMAX;
#ifndef GM_BOX_FAHEAD
#define GM_BOX_FAHEAD 4   // the fold value of a step is read from LDS this many steps ahead
#endif
constexpr int BX_FA = GM_BOX_FAHEAD;
// parent codes of a pair (gm_common.hpp parent_code per u16 half), two dependent ops deep
__device__ __forceinline__ uint32_t bx_code2(uint32_t m) {
    // (m >> 7) * 2 + (m ^ 255) per half; written out so the compiler keeps the packed
    // multiply-add (it otherwise shifts, masks and adds: one op and one level more)
    uint32_t g, t, x;
    asm("v_pk_lshrrev_b16 %1, 7, %3 op_sel_hi:[0,1]\n\t"
        "v_xor_b32 %2, 0xff00ff, %3\n\t"
        "v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]"
        : "=v"(g), "=&v"(t), "=&v"(x) : "v"(m));
    return g;
}
// per-lane constants of the walk, computed once per workgroup
struct BxLaneC {
    int d;                                   // start step
    uint32_t m01, m02, mb0;                  // a0 - 1 / a0 - 2 / b0 neighbour validity
    uint32_t v11, v12, v21[4], v22[4];       // (a1, a2) child validity bytes by step phase
};
__device__ __forceinline__ BxLaneC bx_lane_consts(uint32_t lane, int dadd = 0) {
    BxLaneC L;
    const uint32_t a0 = lane & 3u, b = (lane >> 2) & 15u;
    const int d = dadd + (GM_BOX_WALK_B01 ? BX_S2 * (int)__popc(b) + (int)a0
                                          : (int)__popc(b & 3u) + BX_S2 * (int)__popc(b & 12u) + (int)a0);
    L.d = d;
    L.m01 = a0 >= 1 ? ~0u : 0u;
    L.m02 = a0 >= 2 ? ~0u : 0u;
    L.mb0 = (b & 1u) ? ~0u : 0u;   // b1 needs none: row_shr 8 gives 0 to the lanes it leaves
    // opaque, so they stay VGPR masks (one v_and_b32_dpp per neighbour, not a DPP move
    // and a select on a lane-mask SGPR pair)
    asm volatile("" : "+v"(L.m01), "+v"(L.m02), "+v"(L.mb0));
    // validity of this lane's own earlier codes as (a1, a2) children at step t (p = t - d,
    // a1 = p & 3, a2 = (p >> 2) & 3), one byte (0 or 0xFF) per step phase: t & 3 for a1,
    // t & 15 for a2 (byte t & 3 of word (t >> 2) & 3)
    L.v11 = L.v12 = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) L.v21[q] = L.v22[q] = 0;
#pragma unroll
    for (int t = 0; t < 16; t++) {
        const uint32_t q = (uint32_t)(t - d) & 15u;
        if (t < 4) {
            L.v11 |= ((q & 3u) >= 1 ? 0xFFu : 0u) << (8 * t);
            L.v12 |= ((q & 3u) >= 2 ? 0xFFu : 0u) << (8 * t);
        }
        L.v21[t >> 2] |= ((q >> 2) >= 1 ? 0xFFu : 0u) << (8 * (t & 3));
        L.v22[t >> 2] |= ((q >> 2) >= 2 ? 0xFFu : 0u) << (8 * (t & 3));
    }
    return L;
}
__device__ __forceinline__ void bx_walk(uint32_t *s, uint32_t ln, const BxLaneC &L) {
    const int d = L.d;
    const uint32_t m01 = L.m01, m02 = L.m02, mb0 = L.mb0;
    const uint32_t v11 = L.v11, v12 = L.v12;
    const uint32_t v21[4] = {L.v21[0], L.v21[1], L.v21[2], L.v21[3]};
    const uint32_t v22[4] = {L.v22[0], L.v22[1], L.v22[2], L.v22[3]};
    // position (A = a0 + 4 p, B = b) of step t = p + d at dword base + PITCH t; the
    // neighbour one b2 (b3) step below is 4 (8) dwords lower; a lane without one reads
    // the row's zero slot (dword ZSLOT).  (From the opaque lane, per group:
    // registers held across the group loop would spill in the fold.)
    const uint32_t a0 = ln & 3u, b = (ln >> 2) & 15u;
    const int base = (int)((uint32_t)BX_AS * a0 + b) - BX_PITCH * d, zb = BX_Z - BX_PITCH * d;
    const int base2 = (b & 4u) ? base - 4 : zb, base3 = (b & 8u) ? base - 8 : zb;
    const int base0 = (b & 1u) ? base - 1 : zb, base1 = (b & 2u) ? base - 2 : zb;
    const int dummy = BX_IMG + (int)ln;   // idle steps (before d, after d + 63) use a slot of their own
    // this lane's codes as (a1 - 1, a1 - 2, a2 - 1, a2 - 2) children of the positions 1, 2,
    // 4 and 8 steps later, masked when they are made (0 where the digit wraps): rings by step
    uint32_t g1 = 0, g2[2] = {0, 0}, g4[4] = {0, 0, 0, 0}, g8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // this lane's codes of the last 32 steps: (a3 - 1, a3 - 2) children and the DPP source
    uint32_t hk[32];
#pragma unroll
    for (int q = 0; q < 32; q++) hk[q] = 0;
    auto slot = [&](auto TT, int bs) {
        constexpr int T = decltype(TT)::v;
        int idx = bs + BX_PITCH * T;
        if constexpr (T < BX_DMAX || T >= 64) idx = (uint32_t)(T - d) < 64u ? idx : dummy;
        return idx;
    };
    // LDS inputs: the fold (nothing in the walk writes it before its step), FA steps
    // ahead; the b2 / b3 neighbours' codes, made S2 steps before they are needed
#if GM_BOX_WALK_B01
    struct In { uint32_t C2, C3, C0, C1; };
    auto fetchc = [&](auto TT) { return In{s[slot(TT, base2)], s[slot(TT, base3)], s[slot(TT, base0)], s[slot(TT, base1)]}; };
#else
    struct In { uint32_t C2, C3; };
    auto fetchc = [&](auto TT) { return In{s[slot(TT, base2)], s[slot(TT, base3)]}; };
    (void)base0;
    (void)base1;
#endif
    auto fetchf = [&](auto TT) { return s[slot(TT, base)]; };
    uint32_t pff[BX_FA];
    In pfc[BX_S2];
    auto firstf = [&](auto TT) { pff[decltype(TT)::v] = fetchf(TT); };
    bx_unroll(firstf, std::make_integer_sequence<int, BX_FA>{});
    auto firstc = [&](auto TT) { pfc[decltype(TT)::v] = fetchc(TT); };
    bx_unroll(firstc, std::make_integer_sequence<int, BX_S2>{});
    // the max of a step's inputs that exist a step before it (the fold, the a0 - 2
    // neighbour, this lane's a1 - 2, a2 and a3 children), formed in that step, off the
    // step-to-step chain
    uint32_t pre = pff[0];
    auto step = [&](auto TT) {
        constexpr int T = decltype(TT)::v;
        constexpr bool peel = T < BX_DMAX || T >= 64;
        // the step-to-step chain: the a0 - 1, b0 and b1 neighbours' codes of the step
        // before (DPP), this lane's own (the a1 - 1 child), the b2 / b3 neighbours (LDS)
        const uint32_t hb = hk[(T + 31) & 31];
        const uint32_t y1 = bx_dpp_shr<0x111>(hb) & m01;
        const In cn = pfc[T % BX_S2];
#if GM_BOX_WALK_B01
        const uint32_t m = bx_max3(bx_max3(bx_max3(pre, cn.C2, cn.C3), y1, cn.C0), cn.C1, g1);
        (void)mb0;
#else
        const uint32_t c0 = bx_dpp_shr<0x114>(hb) & mb0, c1 = bx_dpp_shr<0x118>(hb);
        const uint32_t m = bx_max3(bx_max3(bx_max3(pre, cn.C2, cn.C3), y1, c0), c1, g1);
#endif
        if constexpr (T + 1 < BX_STEPS) {
            constexpr int U = T + 1;
            const uint32_t y2 = bx_dpp_shr<0x112>(hb) & m02;   // the a0 - 2 neighbour of step U: its code of step U - 2
            uint32_t q = bx_max3(pff[U % BX_FA], g2[U & 1], g4[U & 3]);
            if constexpr (U >= 32) q = bx_max3(q, hk[(U + 16) & 31], hk[U & 31]);
            else if constexpr (U >= 16) q = bx_max2(q, hk[(U + 16) & 31]);
            pre = bx_max3(q, g8[U & 7], y2);
        }
        uint32_t c = bx_code2(m);
        if constexpr (peel) c = (uint32_t)(T - d) < 64u ? c : 0u;
        // the masks of the steps that will read c: byte (T + k) & 3 of the phase words
        hk[T & 31] = c;
        g1 = bx_and_byte<(T + 1) & 3>(c, v11);
        g2[T & 1] = bx_and_byte<(T + 2) & 3>(c, v12);
        g4[T & 3] = bx_and_byte<(T + 4) & 3>(c, v21[((T + 4) >> 2) & 3]);
        g8[T & 7] = bx_and_byte<(T + 8) & 3>(c, v22[((T + 8) >> 2) & 3]);
        s[slot(TT, base)] = c;
        BX_LDS_ORDER();
        // the b2 / b3 neighbours of step T + S2 made their codes in this step's write
        if constexpr (T + BX_FA < BX_STEPS) pff[T % BX_FA] = fetchf(BxT<T + BX_FA>{});
        if constexpr (T + BX_S2 < BX_STEPS) pfc[T % BX_S2] = fetchc(BxT<T + BX_S2>{});
        __builtin_amdgcn_sched_barrier(0);   // no instruction crosses a step (a hoisted use would wait on a prefetch)
    };
    bx_unroll(step, std::make_integer_sequence<int, BX_STEPS>{});
}

// store: rows m = lane + 64 i of both boxes, bytes regrouped per box.  Split solve: a box another
// rank needs is also written, from the same registers, to its slot in the halo message (the
// whole box, or only its two top layers along an A heap, rows compacted as box_pack_kernel
// packs them), so no pack launch sits between the tier launches.
// DIRECT (loopback and IPC transports): the box goes straight to its slot in the receiving
// rank's own table (peer p0..p2 by axis, slot kind << 28 | axis << 26), rows where they lie,
// so the receiver needs no unpack.
// (NI rows per lane from row set i0: the one-wave kernel stores all four, a wave of the
// four-wave kernel its own.)
template <bool SHARD_, bool DIRECT = false, int CP = GM_BOX_STORE_CPOL, int NI = 4>
__device__ __forceinline__ void bx_store(uint8_t *table, uint8_t *msg, uint8_t *p0, uint8_t *p1, uint8_t *p2,
                                         const BxGroup &G, const uint32_t *s, uint32_t lane, uint32_t i0 = 0) {
    constexpr bool SHARD = SHARD_ && !(GM_BOX_EXP & 32);
    __amdgpu_buffer_rsrc_t w[2];
#pragma unroll
    for (int k = 0; k < 2; k++)
        w[k] = __builtin_amdgcn_make_buffer_rsrc(table + ((uint64_t)G.box[k] << 12), 0,
                                                 (G.valid[k] && !(GM_BOX_EXP & 4)) ? 4096u : 0u, 0x00020000);
    uint32_t dst[2][3] = {{0, 0, 0}, {0, 0, 0}};
    __amdgpu_buffer_rsrc_t wm;
    if constexpr (SHARD) {
        wm = __builtin_amdgcn_make_buffer_rsrc((void *)msg, 0, 0xFFFFFFFFu, 0x00020000);
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int e = 0; e < 3; e++) dst[k][e] = (uint32_t)__builtin_amdgcn_readlane((int)G.dstv, 4 * k + e);
    }
#pragma unroll
    for (int ii = 0; ii < NI; ii++) {
        const uint32_t m = lane + 64u * (i0 + (uint32_t)ii);
        bx_u32x4 o[2];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const bx_u32x4 x = *(const bx_u32x4 *)(s + bx_row(m) + 4u * q);
            const uint32_t t01 = __builtin_amdgcn_perm(x[1], x[0], 0x06020400u);
            const uint32_t t23 = __builtin_amdgcn_perm(x[3], x[2], 0x06020400u);
            o[0][q] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
            o[1][q] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
        }
        __builtin_amdgcn_raw_buffer_store_b128(o[0], w[0], 16u * m, 0, CP);
        __builtin_amdgcn_raw_buffer_store_b128(o[1], w[1], 16u * m, 0, CP);
        if constexpr (SHARD && DIRECT) {
#pragma unroll
            for (int k = 0; k < 2; k++)
#pragma unroll
                for (int e = 0; e < 3; e++) {
                    const uint32_t d = dst[k][e], kind = d >> 28, ax = (d >> 26) & 3u;
                    if (!kind) continue;   // uniform
                    uint8_t *pb = ax == 0 ? p0 : (ax == 1 ? p1 : p2);
                    const __amdgpu_buffer_rsrc_t wp =
                        __builtin_amdgcn_make_buffer_rsrc(pb + ((uint64_t)G.box[k] << 12), 0, 4096u, 0x00020000);
                    const uint32_t a = (m >> (2u * ((kind - 1u) & 3u))) & 3u;
                    if (kind == 5 || a >= 2u)
                        __builtin_amdgcn_raw_buffer_store_b128(o[k], wp, 16u * m, 0, CP);
                }
        } else if constexpr (SHARD) {
#pragma unroll
            for (int k = 0; k < 2; k++)
#pragma unroll
                for (int e = 0; e < 3; e++) {
                    const uint32_t d = dst[k][e], kind = d >> 28;
                    if (!kind) continue;   // uniform
                    const uint32_t base = (d & 0x0FFFFFFFu) << 11;
                    if (kind == 5) {
                        __builtin_amdgcn_raw_buffer_store_b128(o[k], wm, 16u * m, base, 0);
                    } else {
                        const uint32_t hh = 2u * (kind - 1u), a = (m >> hh) & 3u;
                        const uint32_t t = (m & ((1u << hh) - 1u)) | ((a & 1u) << hh) | ((m >> (hh + 2u)) << (hh + 1u));
                        if (a >= 2u) __builtin_amdgcn_raw_buffer_store_b128(o[k], wm, 16u * t, base, 0);
                    }
                }
        }
    }
}

#ifndef GM_BOX_TRACE
#define GM_BOX_TRACE 0         // development: per-phase shader-clock sums, printed after a solve
#endif
#if GM_BOX_TRACE
__device__ unsigned long long bx_trace_acc[8];
#define BX_STAMP(v)                                                                         \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");          \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#endif

// One launch per box-tier.  Workgroup w runs on XCD w % 8 and takes groups (box pairs)
// of that XCD's contiguous run of the tier list (boxes sorted along a Hilbert walk), the
// workgroups of an XCD side by side, so neighbouring groups share child boxes in its L2.
// SHARD: one rank of the sharded solve: its own box list, with a fill code
// per box saying where each child box is read from.
// FILL (split solve): some box of the launch reads a child through a transposition; a launch
// without (every tier of rank 0, most of the others' first tiers) reads its children as at N = 1.
template <bool SHARD, bool DIRECT = false, bool FILL = true>
__global__ __launch_bounds__(64, GM_BOX_WAVES) void box_tier_kernel(uint8_t *__restrict__ table,
                                                                     const uint32_t *__restrict__ boxes,
                                                                     const uint32_t *__restrict__ fills,
                                                                     const uint32_t *__restrict__ srcs,
                                                                     const uint32_t *__restrict__ dsts,
                                                                     uint8_t *__restrict__ msg, uint8_t *p0, uint8_t *p1,
                                                                     uint8_t *p2, uint32_t nbox) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[BX_LDS];
    uint32_t *s = lds + BX_PAD;
    const uint32_t lane = threadIdx.x;
    const uint32_t ng = (nbox + 1) / 2, nw = gridDim.x, w = blockIdx.x;
    const uint32_t x = w & 7u, kx = w >> 3, Kx = (nw - x + 7u) >> 3;
    const uint32_t q = ng >> 3, r = ng & 7u;
    const uint32_t g0 = x * q + (x < r ? x : r), g1 = g0 + q + (x < r ? 1u : 0u);
    uint32_t g = g0 + kx;
    if (g >= g1) return;
    const BxLaneC L = bx_lane_consts(lane);
    // the zero slot of each p-row (no position uses it): the walk's slot for a missing
    // b2 / b3 neighbour
    s[BX_PITCH * lane + BX_Z] = 0;
    bx_u32x4 R[BX_NLOAD];
    constexpr bool SF = SHARD && FILL;
    BxGroup G = bx_group<SHARD, FILL>(boxes, fills, srcs, dsts, nbox, g, lane);
    bx_issue<SF, 0, GM_BOX_SPLIT_PLAIN>(table, G, lane, R);
#if GM_BOX_TRACE
    unsigned long long tt[5], acc[4] = {0, 0, 0, 0}, ngr = 0, tbeg, rbeg;
    BX_STAMP(tbeg);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rbeg)::"memory");
#endif
    // (issuing the next group's loads earlier -- during the walk or before the store --
    // measured slower: the 192 registers they hold spill, or they queue behind the store)
    for (;;) {
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));   // lane-derived addresses are recomputed per group, not held in registers
#if GM_BOX_TRACE
        BX_STAMP(tt[0]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        BX_STAMP(tt[1]);
#endif
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_F);
        if (!(GM_BOX_EXP & 8)) bx_fold<SF>(s, G, ln, R);
        else   // keep the loads live: one xor per row into the image
            for (int q = 0; q < BX_NLOAD; q++) s[ln + 64 * (q & 7)] ^= R[q][0] ^ R[q][3];
        const uint32_t gn = g + Kx;
        const bool more = gn < g1;
        BxGroup Gn = G;
        if (more) Gn = bx_group<SHARD, FILL>(boxes, fills, srcs, dsts, nbox, gn, lane);
        BX_LDS_ORDER();
#if GM_BOX_TRACE
        BX_STAMP(tt[2]);
#endif
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_W);
        if (!(GM_BOX_EXP & 1)) bx_walk(s, ln, L);
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_S);
#if GM_BOX_TRACE
        BX_STAMP(tt[3]);
#endif
        bx_store<SHARD, DIRECT, GM_BOX_TIER_STORE_CPOL>(table, msg, p0, p1, p2, G, s, ln);
        BX_LDS_ORDER();
#if GM_BOX_TRACE
        BX_STAMP(tt[4]);
        for (int k = 0; k < 4; k++) acc[k] += tt[k + 1] - tt[k];
        ngr++;
#endif
        if (!more) break;
        g = gn;
        G = Gn;
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_I);   // the next group's loads out first
        bx_issue<SF, 0, GM_BOX_SPLIT_PLAIN>(table, G, lane, R);
    }
#if GM_BOX_TRACE
    unsigned long long tend, rend;
    BX_STAMP(tend);
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rend)::"memory");
    if (lane == 0) {
        for (int k = 0; k < 4; k++) atomicAdd(&bx_trace_acc[k], acc[k]);
        atomicAdd(&bx_trace_acc[4], ngr);
        atomicAdd(&bx_trace_acc[5], tend - tbeg);
        atomicAdd(&bx_trace_acc[6], 1ull);
        atomicAdd(&bx_trace_acc[7], rend - rbeg);
    }
#endif
}


// ---------------------------------------------------------------------------
// Thin box-tiers (round 5): one group per workgroup of FOUR waves.  A lone group of the
// one-wave kernel is a latency chain of ~8.5 µs (48 child loads, the fold of all 256 rows,
// 73 walk steps, the store), and a box-tier with fewer groups than the chip has SIMDs pays
// it whole (§9.1: 12 of the 41 box-tiers at N = 1, 14 of a rank's 33 at G = 8).  Here wave w
// owns the rows with a3 = w (A = lane + 64 w): it loads only its rows' children (8 B-child
// rows, the top layers of the boxes below along heaps 0-2 -- a row takes them by its own
// digit, the others are zeroed in the pairing -- and along heap 3 when w < 2), folds them,
// walks p' = 0..15 of its quarter (p = 16 w + p') and stores it.  Its a3 - 1 / a3 - 2
// children are the codes waves w - 1 / w - 2 made BX4_L / 2 BX4_L steps before: the waves run
// BX4_L steps apart and a workgroup barrier ends every step, so a step's codes are visible
// to the other waves' prefetches that follow it (read from the image like the b2 / b3
// neighbours).  31 walk steps instead of 73.
#ifndef GM_BOX4_K
#define GM_BOX4_K 1   // a workgroup barrier every K steps
#endif
constexpr int BX4_K = GM_BOX4_K;
constexpr int BX4_L = BX_S2 + BX4_K - 1;   // lag between consecutive waves: a prefetch sees the code
constexpr int BX4_STEPS = 16 + BX_DMAX + 3 * BX4_L;
constexpr int BX4_NLOAD = 24;

// 16 u16 pairs of two rows, or zeros where the lane does not take them (per-lane selectors)
__device__ __forceinline__ void bx_pairs_if(const bx_u32x4 &x0, const bx_u32x4 &x1, bool take, uint32_t (&p)[16]) {
    uint32_t sel[4];
#pragma unroll
    for (int r = 0; r < 4; r++)
        sel[r] = take ? ((uint32_t)r | 0x0c00u | ((4u + (uint32_t)r) << 16) | 0x0c000000u) : 0x0c0c0c0cu;
#pragma unroll
    for (int b = 0; b < 16; b++) p[b] = __builtin_amdgcn_perm(x1[b >> 2], x0[b >> 2], sel[b & 3]);
}

// R[4 k + j]: row m of box k's child along heap 4 + j; R[8 + 4 i + 2 k + v]: row m with digit i
// set to 3 - v of box k's child along heap i (i < 3); R[20 + 2 k + v]: heap 3's (w < 2)
template <bool SHARD>
__device__ __forceinline__ void bx4_issue(const uint8_t *table, const BxGroup &G, uint32_t lane, uint32_t w,
                                          bx_u32x4 (&R)[BX4_NLOAD]) {
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, 0xFFFFFFFFu, 0x00020000);
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void *)table, 0, 0u, 0x00020000);
    const uint32_t m = lane + 64u * w;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const bool ok = G.valid[k] && box_coord(G.box[k], 4 + j) >= 1;
            uint32_t src = G.box[k] - box_unit(4 + j);
            if constexpr (SHARD) src = bx_src<SHARD>(G, k, 4 + j);
            R[4 * k + j] = __builtin_bit_cast(bx_u32x4, __builtin_amdgcn_raw_buffer_load_b128(ok ? rt : rz, 16u * m,
                                                                                              ok ? src << 12 : 0u, 0));
        }
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < 2; k++) {
            // heap 3: only the rows a3 = 0 (layers 3, 2) and a3 = 1 (layer 3) take children (uniform)
            const bool ok = G.valid[k] && box_coord(G.box[k], i) >= 1 && (i < 3 || w < 2u);
            uint32_t src = G.box[k] - box_unit(i), sq = 0, sp = 0;
            if constexpr (SHARD) {
                const uint32_t code = bx_fcode(G, k, i);
                src = bx_src<SHARD>(G, k, i);
                sq = 2u * (code >> 2);
                sp = 2u * (code & 3u);
            }
#pragma unroll
            for (int v = 0; v < 2; v++) {
                uint32_t A = (m & ~(3u << (2 * i))) | ((3u - v) << (2 * i));
                if constexpr (SHARD) {
                    const uint32_t t = ((A >> sq) ^ (A >> sp)) & 3u;
                    A ^= (t << sq) | (t << sp);
                }
                R[8 + 4 * i + 2 * k + v] = __builtin_bit_cast(
                    bx_u32x4, __builtin_amdgcn_raw_buffer_load_b128(ok ? rt : rz, 16u * A, ok ? src << 12 : 0u, 0));
            }
        }
}

template <bool SHARD>
__device__ __forceinline__ void bx4_fold(uint32_t *s, const BxGroup &G, uint32_t lane, uint32_t w,
                                         bx_u32x4 (&R)[BX4_NLOAD]) {
    if constexpr (SHARD) {   // B children read through a B transposition: back to C's byte order
#pragma unroll
        for (int k = 0; k < 2; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t code = bx_fcode(G, k, 4 + j);
                if (code) R[4 * k + j] = bx_bswap_row(R[4 * k + j], code);
            }
    }
    uint32_t F[16];
#pragma unroll
    for (int jp = 0; jp < 4; jp += 2) {   // as bx_fold: two B heaps at a time
        uint32_t P[16], Q[16];
        bx_pairs(R[jp], R[4 + jp], P);
        bx_pairs(R[jp + 1], R[4 + jp + 1], Q);
#pragma unroll
        for (int b = 0; b < 16; b++) {
            uint32_t in[5];
            int n = 0;
            if (jp) in[n++] = F[b];
            in[n++] = P[b];
            in[n++] = Q[b];
            if (!((b >> jp) & 1)) in[n++] = P[b | (1 << jp)];
            if (!((b >> (jp + 1)) & 1)) in[n++] = Q[b | (2 << jp)];
            uint32_t f = n >= 3 ? bx_max3(in[0], in[1], in[2]) : bx_max2(in[0], in[1]);
            if (n == 4) f = bx_max2(f, in[3]);
            if (n == 5) f = bx_max3(f, in[3], in[4]);
            F[b] = f;
        }
    }
    const uint32_t m = lane + 64u * w;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        // the row's digit a_i: 0 takes layers 3 and 2 of the box below, 1 layer 3, else none
        const uint32_t a = (m >> (2 * i)) & 3u;
        uint32_t L3[16], L2[16];
        bx_pairs_if(R[8 + 4 * i + 0], R[8 + 4 * i + 2], a <= 1u, L3);
        bx_pairs_if(R[8 + 4 * i + 1], R[8 + 4 * i + 3], a == 0u, L2);
#pragma unroll
        for (int b = 0; b < 16; b++) F[b] = bx_max3(F[b], L3[b], L2[b]);
    }
#pragma unroll
    for (int q = 0; q < 4; q++)
        *(bx_u32x4 *)(s + bx_row(m) + 4u * q) = bx_u32x4{F[4 * q], F[4 * q + 1], F[4 * q + 2], F[4 * q + 3]};
}

// bx_walk for wave w's quarter (p' = 0..15, p = 16 w + p'), a barrier per step
__device__ __forceinline__ void bx4_walk(uint32_t *s, uint32_t ln, uint32_t w, const BxLaneC &L) {
    const int d = L.d;   // this lane's start, BX4_L w later than in wave 0
    const uint32_t m01 = L.m01, m02 = L.m02, mb0 = L.mb0;
    const uint32_t v11 = L.v11, v12 = L.v12;
    const uint32_t v21[4] = {L.v21[0], L.v21[1], L.v21[2], L.v21[3]};
    const uint32_t v22[4] = {L.v22[0], L.v22[1], L.v22[2], L.v22[3]};
    const uint32_t a0 = ln & 3u, b = (ln >> 2) & 15u;
    // position (A = a0 + 4 p, B = b), p = 16 w + T - d, at dword base + PITCH T
    const int base = (int)((uint32_t)BX_AS * a0 + b) + BX_PITCH * (16 * (int)w - d);
    const int zb = BX_Z + BX_PITCH * (16 * (int)w - d);
    const int base2 = (b & 4u) ? base - 4 : zb, base3 = (b & 8u) ? base - 8 : zb;
    const int base31 = w >= 1u ? base - 16 * BX_PITCH : zb, base32 = w >= 2u ? base - 32 * BX_PITCH : zb;
    const int dummy = BX_IMG + (int)ln;
    uint32_t g1 = 0, g2[2] = {0, 0}, g4[4] = {0, 0, 0, 0}, g8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t hb = 0;   // this lane's code of the step before (the DPP source)
    auto slot = [&](auto TT, int bs) {
        constexpr int T = decltype(TT)::v;
        const int idx = bs + BX_PITCH * T;
        return (uint32_t)(T - d) < 16u ? idx : dummy;
    };
    struct In { uint32_t C2, C3, A1, A2; };
    auto fetchc = [&](auto TT) {
        return In{s[slot(TT, base2)], s[slot(TT, base3)], s[slot(TT, base31)], s[slot(TT, base32)]};
    };
    auto fetchf = [&](auto TT) { return s[slot(TT, base)]; };
    uint32_t pff[BX_FA];
    In pfc[BX_S2];
    auto firstf = [&](auto TT) { pff[decltype(TT)::v] = fetchf(TT); };
    bx_unroll(firstf, std::make_integer_sequence<int, BX_FA>{});
    auto firstc = [&](auto TT) { pfc[decltype(TT)::v] = fetchc(TT); };
    bx_unroll(firstc, std::make_integer_sequence<int, BX_S2>{});
    uint32_t pre = bx_max3(pff[0], pfc[0].A1, pfc[0].A2);
    auto step = [&](auto TT) {
        constexpr int T = decltype(TT)::v;
        const uint32_t y1 = bx_dpp_shr<0x111>(hb) & m01, c0 = bx_dpp_shr<0x114>(hb) & mb0, c1 = bx_dpp_shr<0x118>(hb);
        const In cn = pfc[T % BX_S2];
        const uint32_t mx = bx_max3(bx_max3(bx_max3(pre, cn.C2, cn.C3), y1, c0), c1, g1);
        if constexpr (T + 1 < BX4_STEPS) {
            constexpr int U = T + 1;
            const uint32_t y2 = bx_dpp_shr<0x112>(hb) & m02;
            const In cu = pfc[U % BX_S2];
            const uint32_t q = bx_max3(pff[U % BX_FA], g2[U & 1], g4[U & 3]);
            pre = bx_max3(bx_max3(q, g8[U & 7], y2), cu.A1, cu.A2);
        }
        uint32_t c = bx_code2(mx);
        c = (uint32_t)(T - d) < 16u ? c : 0u;
        hb = c;
        g1 = bx_and_byte<(T + 1) & 3>(c, v11);
        g2[T & 1] = bx_and_byte<(T + 2) & 3>(c, v12);
        g4[T & 3] = bx_and_byte<(T + 4) & 3>(c, v21[((T + 4) >> 2) & 3]);
        g8[T & 7] = bx_and_byte<(T + 8) & 3>(c, v22[((T + 8) >> 2) & 3]);
        s[slot(TT, base)] = c;
        if constexpr ((T + 1) % BX4_K == 0)
            __syncthreads();   // the codes so far, for the other waves' prefetches below
        else
            BX_LDS_ORDER();
        if constexpr (T + BX_FA < BX4_STEPS) pff[T % BX_FA] = fetchf(BxT<T + BX_FA>{});
        if constexpr (T + BX_S2 < BX4_STEPS) pfc[T % BX_S2] = fetchc(BxT<T + BX_S2>{});
        __builtin_amdgcn_sched_barrier(0);
    };
    bx_unroll(step, std::make_integer_sequence<int, BX4_STEPS>{});
}

template <bool SHARD, bool DIRECT = false, bool FILL = true>
__global__ __launch_bounds__(256) void box_tier4_kernel(uint8_t *__restrict__ table, const uint32_t *__restrict__ boxes,
                                                        const uint32_t *__restrict__ fills,
                                                        const uint32_t *__restrict__ srcs,
                                                        const uint32_t *__restrict__ dsts, uint8_t *__restrict__ msg,
                                                        uint8_t *p0, uint8_t *p1, uint8_t *p2, uint32_t nbox) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[BX_LDS];
    uint32_t *s = lds + BX_PAD;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t ng = (nbox + 1) / 2;
    constexpr bool SF = SHARD && FILL;
    const BxLaneC L = bx_lane_consts(lane, BX4_L * (int)w);
    if (lane < 16u) s[BX_PITCH * (16u * w + lane) + BX_Z] = 0;   // this wave's rows' zero slots
    for (uint32_t g = blockIdx.x; g < ng; g += gridDim.x) {
        const BxGroup G = bx_group<SHARD, FILL>(boxes, fills, srcs, dsts, nbox, g, lane);
        bx_u32x4 R[BX4_NLOAD];
        bx4_issue<SF>(table, G, lane, w, R);
        bx4_fold<SF>(s, G, lane, w, R);
        BX_LDS_ORDER();
        bx4_walk(s, lane, w, L);
        bx_store<SHARD, DIRECT, GM_BOX_TIER_STORE_CPOL, 1>(table, msg, p0, p1, p2, G, s, lane, w);
        BX_LDS_ORDER();
    }
}

// ---------------------------------------------------------------------------
// One-launch (dataflow) solve, GM_BOX_FLOW: the box-tier launches' groups, tier after
// tier, go into 8 queues (workgroup w takes from queue w % 8, which hold the same XCD
// runs as the tiered launches; workgroup k of a queue takes its groups k, k + K, ...), and
// a group starts as soon as its child boxes are stored
// instead of when the whole box-tier before it is: the partial last round of each
// launch fills with the next tier's groups.  Hand-off per box (MI355X_MICROARCH.md,
// the first row of the sc1 hand-off table): the group's stores are sc1, the wave waits for
// them, then one lane stores the box's flag (the solve's epoch) sc1; a consumer polls
// its child boxes' flags with sc1 loads and then reads them with sc1 loads.  A workgroup
// takes its groups in tier order, so the workgroup whose current group has the lowest tier
// has all its children stored and never waits (no deadlock while every workgroup is
// resident: the grid is at most the resident capacity); a wait that outlasts
// 200 ms (GM_BOX_FLOW_TIMEOUT_MS) flags an error that every wave sees and leaves by, and the host then
// re-solves with the tiered launches.
#ifndef GM_BOX_FLOW_SLEEP
#define GM_BOX_FLOW_SLEEP 2        // s_sleep between two polls of a child's flag (64 clocks a unit)
#endif
#ifndef GM_BOX_FLOW_LOAD_CPOL
#define GM_BOX_FLOW_LOAD_CPOL 16   // child rows read sc1 (the hand-off table's consumer loads)
#endif
// the hand-off needs the producer's rows written through to the coherent level before its flag
static_assert(GM_BOX_STORE_CPOL & 16, "box_flow_kernel publishes flags after sc1 stores: keep GM_BOX_STORE_CPOL sc1");
struct BxFlow {
    const uint32_t *groups;   // queue q: groups[qbase[q] + j], j < qlen[q]: box-list index | second box << 31
    uint32_t qbase[8], qlen[8];
    uint32_t *ctr;            // [8] error; zeroed before each solve
    uint32_t *flag;           // per box id: the epoch of the solve that stored it
    const uint32_t *epoch;    // this solve's epoch
    uint64_t timeout;         // s_memrealtime ticks (100 MHz) a wait may last (GM_BOX_FLOW_TIMEOUT_MS)
    uint32_t dev;             // development: 1 = no waits (wrong results; times the rest); test: 8 = wait
                              // for an epoch no flag holds (every wait times out: the fallback path)
};

template <bool SHARD>
__device__ __forceinline__ BxGroup bx_group_rec(const uint32_t *__restrict__ boxes, const uint32_t *__restrict__ fills,
                                                const uint32_t *__restrict__ srcs, uint32_t rec, uint32_t lane) {
    BxGroup G;
    const uint32_t i = rec & 0x7FFFFFFFu;
    const bool two = rec >> 31;
    G.valid[0] = true;
    G.box[0] = boxes[i];
    G.valid[1] = two;
    G.box[1] = two ? boxes[i + 1] : 0u;
    G.fill[0] = SHARD ? fills[i] : 0u;
    G.fill[1] = (SHARD && two) ? fills[i + 1] : 0u;
    G.srcv = G.dstv = 0;
    if constexpr (SHARD)
        if (lane < 16 && (lane < 8 || two)) G.srcv = srcs[8 * (i + (lane >> 3)) + (lane & 7u)];
    return G;
}

// the box the group's box k reads for its child along heap dir (bx_issue's choice), ~0 if none;
// lane 8 k + dir asks for its own
template <bool SHARD>
__device__ __forceinline__ uint32_t bx_child_src(const BxGroup &G, uint32_t k, uint32_t dir) {
    const uint32_t box = k ? G.box[1] : G.box[0];
    if (!(k ? G.valid[1] : G.valid[0]) || box_coord(box, (int)dir) < 1) return ~0u;
    if constexpr (SHARD) return G.srcv;
    return box - box_unit((int)dir);
}

// lanes 0-15 each wait for one child box of G (k = lane >> 3, heap lane & 7): src, and the
// flag value `seen` loaded earlier (~0 = none); false when an error (a timeout, here or
// in another wave) ends the solve
__device__ __forceinline__ uint32_t bx_flag_src_load(const BxFlow &F, uint32_t src) {
    return src == ~0u ? 0u : __hip_atomic_load(&F.flag[src], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool bx_wait(const BxFlow &F, uint32_t src, uint32_t seen, uint32_t lane, uint32_t ep) {
    if (F.dev & 8u) ep += 1u;
    if (__all(src == ~0u || seen == ep)) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__all(src == ~0u || bx_flag_src_load(F, src) == ep)) return true;
        if (__hip_atomic_load(&F.ctr[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (__builtin_amdgcn_s_memrealtime() - t0 > F.timeout) {
            if (lane == 0) atomicOr(&F.ctr[8], 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(GM_BOX_FLOW_SLEEP);
    }
}

#ifndef GM_BOX_FLOW_TRACE
#define GM_BOX_FLOW_TRACE 0   // development: per-group realtime stamps (tools/flow_trace.py)
#endif
#if GM_BOX_FLOW_TRACE
constexpr uint32_t BX_FT_WORDS = 6;   // picked, children ready, folded, walked, flagged, box | workgroup << 32
constexpr uint32_t BX_FT_GROUPS = (1u << 19) + 4096u;   // 2^20 boxes in pairs, plus an odd box per tier run
__device__ unsigned long long bx_ftrace[BX_FT_WORDS * BX_FT_GROUPS];
#define BX_RT(v)                                                                        \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");  \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)
#endif

template <bool SHARD>
__global__ __launch_bounds__(64, GM_BOX_WAVES) void box_flow_kernel(uint8_t *__restrict__ table,
                                                                     const uint32_t *__restrict__ boxes,
                                                                     const uint32_t *__restrict__ fills,
                                                                     const uint32_t *__restrict__ srcs, BxFlow F) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[BX_LDS];
    uint32_t *s = lds + BX_PAD;
    const uint32_t lane = threadIdx.x, q = blockIdx.x & 7u, qn = F.qlen[q];
    const uint32_t *gq = F.groups + F.qbase[q];
    const uint32_t ep = __builtin_amdgcn_readfirstlane(*F.epoch);
    // workgroup k of queue q takes its groups k, k + K, k + 2 K, ... (K workgroups per
    // queue): static, like the tier launches, so no atomic per group
    const uint32_t K = (gridDim.x - q + 7u) >> 3;
    uint32_t j = blockIdx.x >> 3;
    if (j >= qn) return;
    const BxLaneC L = bx_lane_consts(lane);
    s[BX_PITCH * lane + BX_Z] = 0;
    bx_u32x4 R[BX_NLOAD];
    for (;;) {
#if GM_BOX_FLOW_TRACE
        unsigned long long ft[5];
        BX_RT(ft[0]);
#endif
        const BxGroup G = bx_group_rec<SHARD>(boxes, fills, srcs, gq[j], lane);
        const uint32_t src = lane < 16u ? bx_child_src<SHARD>(G, lane >> 3, lane & 7u) : ~0u;
        const uint32_t seen = bx_flag_src_load(F, src);
        if (!(F.dev & 1u) && !bx_wait(F, src, seen, lane, ep)) return;
#if GM_BOX_FLOW_TRACE
        BX_RT(ft[1]);
#endif
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_I);
        bx_issue<SHARD, GM_BOX_FLOW_LOAD_CPOL>(table, G, lane, R);
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_F);
        bx_fold<SHARD>(s, G, ln, R);
        BX_LDS_ORDER();
#if GM_BOX_FLOW_TRACE
        BX_RT(ft[2]);
#endif
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_W);
        bx_walk(s, ln, L);
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_S);
#if GM_BOX_FLOW_TRACE
        BX_RT(ft[3]);
#endif
        bx_store<false>(table, nullptr, nullptr, nullptr, nullptr, G, s, ln);
        BX_LDS_ORDER();
        // publish: the wave's sc1 stores done, then one lane stores each box's flag sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
            __hip_atomic_store(&F.flag[G.box[0]], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (G.valid[1]) __hip_atomic_store(&F.flag[G.box[1]], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#if GM_BOX_FLOW_TRACE
        BX_RT(ft[4]);
        if (lane == 0 && F.qbase[q] + j < BX_FT_GROUPS) {
            unsigned long long *o = bx_ftrace + BX_FT_WORDS * (F.qbase[q] + j);
            for (int k = 0; k < 5; k++) o[k] = ft[k];
            o[5] = G.box[0] | ((unsigned long long)blockIdx.x << 32);
        }
#endif
        j += K;
        if (j >= qn) break;
    }
}

// ---------------------------------------------------------------------------
// Split solve as dataflow (dist_box.hip, GM_OPT_BOX_FLOW 1 with virtual ranks or the IPC
// transport): each rank's whole box-tier chain in one launch, as box_flow_kernel, and the
// exchange folded into the same hand-off -- a group stores its halo boxes straight into the
// receiving rank's table (bx_store DIRECT), drains, and then stores those boxes' flags in the
// RECEIVER's flag array with a system-scope release; the receiver's groups wait on their child
// boxes' flags in their own array whoever stored them.  So a box starts when its own children
// are in, across ranks as within one.  One launch may carry several ranks (virtual ranks on
// one GPU: workgroup w runs rank w % n, all of them resident together, which the waits need);
// every rank's epoch is the solve's sequence number.
// per rank (gm_internal.hpp BxSplitFlowDesc): table, box list, fill words, sources, halo
// slots, group queues (as BxFlow::groups), its flag array (per box id: the epoch of the solve
// that stored it -- own boxes and the halo boxes other ranks store into its table), and per
// axis the receiving rank's table and flag array (null where this rank sends nothing)
typedef BxSplitFlowDesc BxSplitFlow;

// SYS: some rank stores into this one's flags from another GPU (IPC transport across devices):
// system-scope polls, which bypass the L2; else agent scope, as box_flow_kernel
template <bool SYS>
__device__ __forceinline__ bool bx_split_wait(const uint32_t *flag, uint32_t src, uint32_t ep, uint32_t *err,
                                              uint64_t timeout, uint32_t lane) {
    auto ld = [&](uint32_t b) {
        if (b == ~0u) return ep;
        return SYS ? __hip_atomic_load(&flag[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                   : __hip_atomic_load(&flag[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    if (__all(ld(src) == ep)) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__all(ld(src) == ep)) return true;
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
            if (lane == 0) atomicOr(err, 1u);
            return false;
        }
        __builtin_amdgcn_s_sleep(GM_BOX_FLOW_SLEEP);
    }
}

template <bool SYS>
__global__ __launch_bounds__(64, GM_BOX_WAVES) void box_split_flow_kernel(const BxSplitFlow *__restrict__ ranks,
                                                                           uint32_t nranks, uint32_t ep, uint32_t *err,
                                                                           uint64_t timeout) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[BX_LDS];
    uint32_t *s = lds + BX_PAD;
    const uint32_t lane = threadIdx.x;
    const uint32_t r = blockIdx.x % nranks, k = blockIdx.x / nranks;
    const uint32_t nk = (gridDim.x - r + nranks - 1u) / nranks;   // workgroups of rank r
    const uint32_t q = k & 7u, K = (nk - q + 7u) >> 3;
    // the descriptor is re-read (scalar loads) where each field is used instead of held in
    // SGPRs across the group: held, its pointers overflow the SGPR budget of the fold and walk
    auto fd = [&]() {
        const BxSplitFlow *p = ranks + r;
        asm volatile("" : "+s"(p));
        return p;
    };
    const uint32_t qn = fd()->qlen[q];
    uint32_t j = k >> 3;
    if (j >= qn) return;
    const BxLaneC L = bx_lane_consts(lane);
    s[BX_PITCH * lane + BX_Z] = 0;
    bx_u32x4 R[BX_NLOAD];
    for (;;) {
        BxGroup G;
        uint32_t rec;
        {
            const BxSplitFlow *F = fd();
            rec = F->groups[F->qbase[q] + j];
            G = bx_group_rec<true>(F->boxes, F->fills, F->srcs, rec, lane);
            const uint32_t src = lane < 16u ? bx_child_src<true>(G, lane >> 3, lane & 7u) : ~0u;
            if (!bx_split_wait<SYS>(F->flag, src, ep, err, timeout, lane)) return;
        }
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_I);
        bx_issue<true, GM_BOX_FLOW_LOAD_CPOL>(fd()->table, G, lane, R);
        uint32_t ln = lane;
        asm volatile("" : "+v"(ln));
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_F);
        bx_fold<true>(s, G, ln, R);
        BX_LDS_ORDER();
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_W);
        bx_walk(s, ln, L);
        __builtin_amdgcn_s_setprio(GM_BOX_PRIO_S);
        {
            const BxSplitFlow *F = fd();
            const uint32_t i = (rec & 0x7FFFFFFFu) + (lane >> 2);   // the halo slots, needed from here on
            if (lane < 8 && (lane & 3u) < 3u && (lane < 4 || (rec >> 31))) G.dstv = F->dsts[3 * i + (lane & 3u)];
            bx_store<true, true>(F->table, nullptr, F->ptab[0], F->ptab[1], F->ptab[2], G, s, ln);
        }
        BX_LDS_ORDER();
        // publish (the hand-off of box_flow_kernel): the wave's stores are written through
        // (GM_BOX_STORE_CPOL, own and halo rows alike) and done, then the flags -- own boxes in
        // this rank's array, halo boxes also in the receiver's.  No release fence: on this chip
        // it would write back the XCD's whole L2 per group (measured: 4x slower solves)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        {
            const BxSplitFlow *F = fd();
            if (lane == 0) {
                __hip_atomic_store(&F->flag[G.box[0]], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (G.valid[1]) __hip_atomic_store(&F->flag[G.box[1]], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (lane < 8 && (lane & 3u) < 3u && (G.dstv >> 28)) {
                const uint32_t ax = (G.dstv >> 26) & 3u, b = (lane >> 2) ? G.box[1] : G.box[0];
                uint32_t *pf = ax == 0 ? F->pflag[0] : (ax == 1 ? F->pflag[1] : F->pflag[2]);
                if (SYS) __hip_atomic_store(&pf[b], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else __hip_atomic_store(&pf[b], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        j += K;
        if (j >= qn) break;
    }
}

__global__ void box_epoch_kernel(uint32_t *epoch) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *epoch += 1u;
}

// digest of the positions of a box list that lie in the root's region
__global__ void box_digest_kernel(const uint8_t *__restrict__ table, const uint32_t *__restrict__ boxes, uint64_t nbox,
                                  uint64_t root, unsigned long long *acc) {
    uint64_t sum = 0, cnt = 0;
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < (nbox << 12);
         x += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t idx = (boxes[x >> 12] << 12) | (uint32_t)(x & 4095u);
        const uint32_t k = box_key_of_index(idx);
        bool in = true;
        for (int j = 0; j < 8; j++) in &= ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
        if (!in) continue;
        sum += digest_term(k, record_of_code(table[idx]));
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

// Records of keys: REC_UNSOLVED outside the root's region (a key with a nibble above the
// root's, whose slot the solve never wrote).  Split solve with virtual ranks (dist_box.hip):
// `owner` gives per box id the rank whose table holds it (0xFF: none), `tables` per rank.
__global__ void box_query_kernel(const uint8_t *const *__restrict__ tables, const uint8_t *__restrict__ owner,
                                 uint64_t root, const uint64_t *__restrict__ keys, uint16_t *__restrict__ out, uint64_t n) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    bool in = k < (1ull << 32);
    for (int j = 0; j < 8 && in; j++) in = ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
    if (!in) { out[i] = REC_UNSOLVED; return; }
    const uint32_t idx = box_index_of_key((uint32_t)k);
    const uint32_t r = owner ? owner[idx >> 12] : 0u;
    out[i] = r == 0xFFu ? REC_UNSOLVED : record_of_code(tables[r][idx]);
}

// ---------------------------------------------------------------------------
// host

// Hilbert index (Skilling's transpose form) of the first 7 box coordinates, 3 bits each
uint64_t box_hilbert(uint32_t box) {
    const int n = 7;
    uint32_t xv[8];
    for (int i = 0; i < n; i++) xv[i] = (uint32_t)box_coord(box, i);
    for (uint32_t qq = 4; qq > 1; qq >>= 1) {
        const uint32_t p = qq - 1;
        for (int i = 0; i < n; i++) {
            if (xv[i] & qq) xv[0] ^= p;
            else { const uint32_t t = (xv[0] ^ xv[i]) & p; xv[0] ^= t; xv[i] ^= t; }
        }
    }
    for (int i = 1; i < n; i++) xv[i] ^= xv[i - 1];
    uint32_t t = 0;
    for (uint32_t qq = 4; qq > 1; qq >>= 1) if (xv[n - 1] & qq) t ^= qq - 1;
    for (int i = 0; i < n; i++) xv[i] ^= t;
    uint64_t hv = 0;
    for (int bit = 2; bit >= 0; bit--)
        for (int i = 0; i < n; i++) hv = (hv << 1) | ((xv[i] >> bit) & 1u);
    return hv;
}

// Resident one-wave workgroups of a box kernel on this device (dynamic LDS `dyn` bytes):
// the tier launches' grid cap, and the dataflow launch's grid, which must be resident
// whole for its waits to make progress (asked of the runtime, not
// assumed).
static int box_resident(const void *kernel, int device, size_t dyn) {
    int cus = 256, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 64, dyn) != hipSuccess || per < 1) {
        (void)hipGetLastError();
        per = 4 * GM_BOX_WAVES;
    }
    return cus * per;
}
int box_grid_cap(int device) { return box_resident((const void *)box_tier_kernel<true>, device, 0); }

// Box-tiers of at most this many groups run the four-wave kernel (GM_BOX_THIN_GROUPS, development;
// default 0 = never: measured no faster -- a thin launch's ~9 µs is not its walk, §9.1)
uint32_t box_thin_groups() {   // (read per launch: the launches are enqueued once per captured graph)
    const char *e = getenv("GM_BOX_THIN_GROUPS");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 0u;
}

void box_launch_tier_split(uint32_t grid, uint8_t *table, const uint32_t *boxes, const uint32_t *fills,
                           const uint32_t *srcs, const uint32_t *dsts, uint8_t *msg, uint8_t *const *peers,
                           uint32_t nbox, bool fill, hipStream_t s) {
    const uint32_t ng = (nbox + 1) / 2;
    if (ng <= box_thin_groups()) {   // a thin box-tier: the four-wave kernel, one group per workgroup
        uint8_t *q0 = peers ? peers[0] : nullptr, *q1 = peers ? peers[1] : nullptr, *q2 = peers ? peers[2] : nullptr;
        if (peers && fill)
            hipLaunchKernelGGL((box_tier4_kernel<true, true, true>), dim3(ng), dim3(256), 0, s, table, boxes, fills, srcs,
                               dsts, nullptr, q0, q1, q2, nbox);
        else if (peers)
            hipLaunchKernelGGL((box_tier4_kernel<true, true, false>), dim3(ng), dim3(256), 0, s, table, boxes, fills, srcs,
                               dsts, nullptr, q0, q1, q2, nbox);
        else if (fill)
            hipLaunchKernelGGL((box_tier4_kernel<true, false, true>), dim3(ng), dim3(256), 0, s, table, boxes, fills, srcs,
                               dsts, msg, nullptr, nullptr, nullptr, nbox);
        else
            hipLaunchKernelGGL((box_tier4_kernel<true, false, false>), dim3(ng), dim3(256), 0, s, table, boxes, fills, srcs,
                               dsts, msg, nullptr, nullptr, nullptr, nbox);
        return;
    }
    if (peers && fill)
        hipLaunchKernelGGL((box_tier_kernel<true, true, true>), dim3(grid), dim3(64), 0, s, table, boxes, fills, srcs,
                           dsts, nullptr, peers[0], peers[1], peers[2], nbox);
    else if (peers)
        hipLaunchKernelGGL((box_tier_kernel<true, true, false>), dim3(grid), dim3(64), 0, s, table, boxes, fills, srcs,
                           dsts, nullptr, peers[0], peers[1], peers[2], nbox);
    else if (fill)
        hipLaunchKernelGGL((box_tier_kernel<true, false, true>), dim3(grid), dim3(64), 0, s, table, boxes, fills, srcs,
                           dsts, msg, nullptr, nullptr, nullptr, nbox);
    else
        hipLaunchKernelGGL((box_tier_kernel<true, false, false>), dim3(grid), dim3(64), 0, s, table, boxes, fills, srcs,
                           dsts, msg, nullptr, nullptr, nullptr, nbox);
}
void box_launch_split_flow(uint32_t grid, const void *ranks, uint32_t nranks, uint32_t ep, uint32_t *err,
                           uint64_t timeout_ticks, bool sys, hipStream_t s) {
    if (sys)
        hipLaunchKernelGGL(box_split_flow_kernel<true>, dim3(grid), dim3(64), 0, s, (const BxSplitFlow *)ranks, nranks,
                           ep, err, timeout_ticks);
    else
        hipLaunchKernelGGL(box_split_flow_kernel<false>, dim3(grid), dim3(64), 0, s, (const BxSplitFlow *)ranks, nranks,
                           ep, err, timeout_ticks);
}
int box_split_flow_resident(int device) {
    return std::min(box_resident((const void *)box_split_flow_kernel<true>, device, 0),
                    box_resident((const void *)box_split_flow_kernel<false>, device, 0));
}
void box_launch_digest(const uint8_t *table, const uint32_t *boxes, uint64_t nbox, uint64_t root,
                       unsigned long long *acc, hipStream_t s) {
    if (nbox) hipLaunchKernelGGL(box_digest_kernel, dim3(4096), dim3(256), 0, s, table, boxes, nbox, root, acc);
}
void box_launch_query(const uint8_t *const *tables, const uint8_t *owner, uint64_t root, const uint64_t *keys,
                      uint16_t *out, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(box_query_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tables, owner, root, keys,
                              out, n);
}

struct DenseBox {
    uint32_t root_hi = 0;
    uint8_t *table = nullptr;
    bool owned = false;
    uint32_t *d_boxes = nullptr;
    std::vector<uint32_t> tier_off;
    std::vector<uint32_t> boxes;      // host copy (digest list = every box of the region)
    hipGraphExec_t graph = nullptr;
    hipStream_t graph_stream = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    int grid_cap = 2048;
    uint64_t *d_acc = nullptr;
    const uint8_t **d_tables = nullptr;   // [1] = table (box_query_kernel's table array)
    bool flow = false;                // one-launch (dataflow) solve (GM_OPT_BOX_FLOW)
    int flow_grid = 0;                // the dataflow launch's grid: its resident capacity
    size_t flow_dyn = 0;              // dynamic LDS of the dataflow launch (GM_BOX_FLOW_EXTRA_LDS, tests)
    uint32_t *d_flow = nullptr;       // [0, 9) error word at [8], [16] epoch, [64, 64 + 2^20) box flags
    uint32_t *d_groups = nullptr;     // the 8 group queues (BxFlow)
    uint32_t qbase[8] = {}, qlen[8] = {};
    uint32_t *h_res = nullptr;        // pinned: [0] the root's code (low byte), [1] the dataflow error word
};

// GM_BOX_FLOW (development, overrides GM_OPT_BOX_FLOW): 0 tier launches, 1 dataflow, 2 dataflow
// without its waits (wrong results: times everything else)
static int box_flow_env() {
    static const int v = getenv("GM_BOX_FLOW") ? atoi(getenv("GM_BOX_FLOW")) : -1;
    return v;
}
static bool box_flow_wanted(const Ctx *c) {
    const int e = box_flow_env();
    if (e >= 0) return e != 0;
    return c->box_flow == 1 && !c->box_flow_failed;
}

// The tier launches' groups in 8 queues: queue x = every tier's XCD run x, tier after
// tier.  Inside a run the groups are ordered by when their child boxes are stored: a
// group's key is the latest normalised position (0..1 along its queue's run) of its
// children in the tier before, and the run is sorted by key (stable: Hilbert order among
// equals), so the first rounds of a tier take the groups whose children the first rounds
// of the tier before made (GM_BOX_FLOW_ORDER 0: Hilbert order only).
static void box_flow_queues(DenseBox &R, std::vector<uint32_t> &out) {
    static const int order = getenv("GM_BOX_FLOW_ORDER") ? atoi(getenv("GM_BOX_FLOW_ORDER")) : 1;
    const std::vector<uint32_t> &boxes = R.boxes;
    std::vector<uint32_t> q[8];
    std::vector<float> when(1u << 20, 0.0f);   // per box id: normalised position of its group
    for (size_t t = 0; t + 1 < R.tier_off.size(); t++) {
        const uint32_t o = R.tier_off[t], nb = R.tier_off[t + 1] - o, ng = (nb + 1) / 2;
        const uint32_t qq = ng >> 3, r = ng & 7u;
        for (uint32_t x = 0; x < 8; x++) {
            const uint32_t g0 = x * qq + (x < r ? x : r), g1 = g0 + qq + (x < r ? 1u : 0u);
            std::vector<std::pair<float, uint32_t>> run;
            for (uint32_t g = g0; g < g1; g++) {
                const uint32_t i = o + 2 * g;
                const bool two = i + 1 < o + nb;
                float key = 0.0f;
                if (order)
                    for (uint32_t k = 0; k < (two ? 2u : 1u); k++)
                        for (int dir = 0; dir < 8; dir++)
                            if (box_coord(boxes[i + k], dir) >= 1)
                                key = std::max(key, when[boxes[i + k] - box_unit(dir)]);
                run.push_back({key, i | (two ? 0x80000000u : 0u)});
            }
            std::stable_sort(run.begin(), run.end(),
                             [](const std::pair<float, uint32_t> &a, const std::pair<float, uint32_t> &b) {
                                 return a.first < b.first;
                             });
            for (size_t n = 0; n < run.size(); n++) {
                const uint32_t rec = run[n].second, i = rec & 0x7FFFFFFFu;
                const float w = (float)(n + 1) / (float)run.size();
                when[boxes[i]] = w;
                if (rec >> 31) when[boxes[i + 1]] = w;
                q[x].push_back(rec);
            }
        }
    }
    out.clear();
    for (int x = 0; x < 8; x++) {
        R.qbase[x] = (uint32_t)out.size();
        R.qlen[x] = (uint32_t)q[x].size();
        out.insert(out.end(), q[x].begin(), q[x].end());
    }
}

// every box of the root's region by box-tier, Hilbert order inside a tier
static void box_region_tiers(uint32_t root_hi, std::vector<uint32_t> &boxes, std::vector<uint32_t> &tier_off) {
    int lim[8], tmax = 0;
    for (int i = 0; i < 8; i++) { lim[i] = box_coord(root_hi, i); tmax += lim[i]; }
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> tiers(tmax + 1);
    for (uint32_t b = 0; b < (1u << 20); b++) {
        bool in = true;
        for (int i = 0; i < 8 && in; i++) in = box_coord(b, i) <= lim[i];
        if (in) tiers[box_tier(b)].push_back({box_hilbert(b), b});
    }
    boxes.clear();
    tier_off.assign(1, 0);
    for (auto &tv : tiers) {
        std::sort(tv.begin(), tv.end());
        for (auto &e : tv) boxes.push_back(e.second);
        tier_off.push_back((uint32_t)boxes.size());
    }
}

void dense_box_free(Ctx *c);

// A half-built context is never kept: every failure path frees it.
static int box_prepare(Ctx *c, DenseBox *d, uint64_t root) {
    d->root_hi = box_index_of_key((uint32_t)root) >> 12;
    GM_HIP(hipMalloc(&d->d_acc, 2 * sizeof(uint64_t)));
    d->grid_cap = box_resident((const void *)box_tier_kernel<false>, c->device, 0);
    const uint64_t bytes = 1ull << 32;
    if (c->adopted_dense && c->adopted_dense_bytes < bytes) {
        set_error("adopted dense table holds %llu bytes, need %llu", (unsigned long long)c->adopted_dense_bytes,
                  (unsigned long long)bytes);
        return GM_E_CAP;
    }
    box_region_tiers(d->root_hi, d->boxes, d->tier_off);
    GM_HIP(hipMalloc(&d->d_boxes, std::max<size_t>(1, d->boxes.size()) * 4));
    GM_HIP(hipMemcpy(d->d_boxes, d->boxes.data(), d->boxes.size() * 4, hipMemcpyHostToDevice));
    d->flow = box_flow_wanted(c);
    if (d->flow) {
        const size_t words = 64 + (1u << 20);
        GM_HIP(hipMalloc(&d->d_flow, words * 4));
        GM_HIP(hipMemset(d->d_flow, 0, words * 4));
        std::vector<uint32_t> qs;
        box_flow_queues(*d, qs);
        GM_HIP(hipMalloc(&d->d_groups, std::max<size_t>(1, qs.size()) * 4));
        GM_HIP(hipMemcpy(d->d_groups, qs.data(), qs.size() * 4, hipMemcpyHostToDevice));
        const char *xl = getenv("GM_BOX_FLOW_EXTRA_LDS");   // tests: fewer resident workgroups
        d->flow_dyn = xl ? (size_t)std::max(0, atoi(xl)) : 0;
        d->flow_grid = box_resident((const void *)box_flow_kernel<false>, c->device, d->flow_dyn) & ~7;
        if (d->flow_grid < 8) { set_error("box dataflow kernel: no resident workgroups"); return GM_E_HIP; }
    }
    if (c->adopted_dense) {
        d->table = (uint8_t *)c->adopted_dense;
    } else {
        if (hipMalloc(&d->table, bytes) != hipSuccess) {
            (void)hipGetLastError();
            set_error("hipMalloc of a 4 GiB dense table failed");
            return GM_E_NOMEM;
        }
        d->owned = true;
    }
    GM_HIP(hipMalloc(&d->d_tables, sizeof(uint8_t *)));
    GM_HIP(hipMemcpy(d->d_tables, &d->table, sizeof(uint8_t *), hipMemcpyHostToDevice));
    return GM_OK;
}

static int box_launch_flow(Ctx *c, DenseBox *d) {
    BxFlow F;
    F.groups = d->d_groups;
    for (int x = 0; x < 8; x++) {
        F.qbase[x] = d->qbase[x];
        F.qlen[x] = d->qlen[x];
    }
    F.ctr = d->d_flow;
    F.epoch = d->d_flow + 16;
    F.flag = d->d_flow + 64;
    F.dev = box_flow_env() == 2 ? 1u : 0u;
    if (getenv("GM_BOX_FLOW_TEST_STALL") && atoi(getenv("GM_BOX_FLOW_TEST_STALL"))) F.dev |= 8u;
    // milliseconds, fractions kept (0.5 used to truncate to 0 ticks); <= 0 is refused
    const char *tm = getenv("GM_BOX_FLOW_TIMEOUT_MS");
    const double ms = tm ? atof(tm) : 200.0;
    if (!(ms > 0.0)) { set_error("GM_BOX_FLOW_TIMEOUT_MS must be > 0 (got %s)", tm); return GM_E_ARG; }
    F.timeout = (uint64_t)(ms * 100000.0);
    GM_HIP(hipMemsetAsync(d->d_flow, 0, 9 * 4, c->stream));
    hipLaunchKernelGGL(box_epoch_kernel, dim3(1), dim3(64), 0, c->stream, d->d_flow + 16);
    hipLaunchKernelGGL(box_flow_kernel<false>, dim3((uint32_t)d->flow_grid), dim3(64), d->flow_dyn, c->stream, d->table,
                       d->d_boxes, (const uint32_t *)nullptr, (const uint32_t *)nullptr, F);
    GM_HIP(hipGetLastError());
    return GM_OK;
}

static int box_launch_tiers(Ctx *c, DenseBox *d) {
    if (d->flow) return box_launch_flow(c, d);
    for (size_t t = 0; t + 1 < d->tier_off.size(); t++) {
        const uint32_t nb = d->tier_off[t + 1] - d->tier_off[t];
        if (!nb) continue;
        const uint32_t ng = (nb + 1) / 2;
        if (ng <= box_thin_groups()) {   // a thin box-tier: the four-wave kernel, one group per workgroup
            hipLaunchKernelGGL(box_tier4_kernel<false>, dim3(ng), dim3(256), 0, c->stream, d->table,
                               d->d_boxes + d->tier_off[t], (const uint32_t *)nullptr, (const uint32_t *)nullptr,
                               (const uint32_t *)nullptr, (uint8_t *)nullptr, (uint8_t *)nullptr, (uint8_t *)nullptr,
                               (uint8_t *)nullptr, nb);
            continue;
        }
        // at least 8 workgroups (one per XCD run), at most the resident capacity
        const uint32_t grid = std::max<uint32_t>(8u, std::min<uint32_t>(ng, (uint32_t)d->grid_cap));
        hipLaunchKernelGGL(box_tier_kernel<false>, dim3(grid), dim3(64), 0, c->stream, d->table,
                           d->d_boxes + d->tier_off[t], (const uint32_t *)nullptr, (const uint32_t *)nullptr,
                           (const uint32_t *)nullptr, (uint8_t *)nullptr, (uint8_t *)nullptr, (uint8_t *)nullptr,
                           (uint8_t *)nullptr, nb);
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

static int box_launches(const DenseBox *d) {
    if (d->flow) return 1;
    int n = 0;
    for (size_t t = 0; t + 1 < d->tier_off.size(); t++) n += d->tier_off[t + 1] > d->tier_off[t];
    return n;
}

// per-position tier counts of the root's region (positions of heap sum t)
void box_tier_counts(uint64_t root, std::vector<uint64_t> &acc) {
    acc.assign(1, 1);
    for (int j = 0; j < 8; j++) {
        const int lim = (int)((root >> (4 * j)) & 15u);
        std::vector<uint64_t> nx(acc.size() + lim, 0);
        for (size_t s = 0; s < acc.size(); s++)
            for (int hh = 0; hh <= lim; hh++) nx[s + hh] += acc[s];
        acc.swap(nx);
    }
}

int dense_box_solve(Ctx *c, uint64_t root) {
    if (c->world > 1 || c->virtual_ranks > 1) {   // the split solve (dist_box.hip)
        dense_box_free(c);
        return dist_box_solve(c, root);
    }
    dist_box_free(c);
    DenseBox *d = c->dbox;
    const uint32_t rh = box_index_of_key((uint32_t)root) >> 12;
    if (!d || (c->adopted_dense && d->table != c->adopted_dense) || d->root_hi != rh || d->flow != box_flow_wanted(c)) {
        dense_box_free(c);
        d = c->dbox = new DenseBox();
        const int rc = box_prepare(c, d, root);
        if (rc != GM_OK) {
            dense_box_free(c);
            return rc;
        }
    }
    const double t0 = now_ms();
    if (c->timing && !d->ev[0]) {
        GM_HIP(hipEventCreate(&d->ev[0]));
        GM_HIP(hipEventCreate(&d->ev[1]));
    }
    if (c->use_graph) {
        if (!d->graph || d->graph_stream != c->stream) {
            if (d->graph) { (void)hipGraphExecDestroy(d->graph); d->graph = nullptr; }
            hipGraph_t g;
            GM_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
            const int rc = box_launch_tiers(c, d);
            const hipError_t e = hipStreamEndCapture(c->stream, &g);
            if (rc != GM_OK) return rc;
            if (e != hipSuccess) { set_error("graph capture failed: %s", hipGetErrorString(e)); return GM_E_HIP; }
            GM_HIP(hipGraphInstantiate(&d->graph, g, nullptr, nullptr, 0));
            GM_HIP(hipGraphDestroy(g));
            d->graph_stream = c->stream;
        }
        if (c->timing) GM_HIP(hipEventRecord(d->ev[0], c->stream));
        GM_HIP(hipGraphLaunch(d->graph, c->stream));
        if (c->timing) GM_HIP(hipEventRecord(d->ev[1], c->stream));
    } else {
        if (c->timing) GM_HIP(hipEventRecord(d->ev[0], c->stream));
        GM_TRY(box_launch_tiers(c, d));
        if (c->timing) GM_HIP(hipEventRecord(d->ev[1], c->stream));
    }
#if GM_BOX_FLOW_TRACE
    if (d->flow && getenv("GM_BOX_FLOW_TRACE_OUT")) {
        uint64_t ng = 0;
        for (int x = 0; x < 8; x++) ng += d->qlen[x];
        std::vector<unsigned long long> h(BX_FT_WORDS * std::min<uint64_t>(ng, BX_FT_GROUPS));
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_HIP(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(bx_ftrace), h.size() * 8));
        if (FILE *f = fopen(getenv("GM_BOX_FLOW_TRACE_OUT"), "wb")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
#endif
#if GM_BOX_TRACE
    {
        unsigned long long h[8];
        GM_HIP(hipStreamSynchronize(c->stream));
        GM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(bx_trace_acc), sizeof(h)));
        const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        GM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(bx_trace_acc), z, sizeof(z)));
        const double n = (double)(h[4] ? h[4] : 1);
        fprintf(stderr, "box trace: %llu groups %llu waves | per group cycles: load-wait %.0f fold %.0f walk %.0f store+issue %.0f | per wave total %.0f ticks = %.2f us at 100 MHz realtime (%.2f GHz)\n",
                h[4], h[6], h[0] / n, h[1] / n, h[2] / n, h[3] / n, h[5] / (double)(h[6] ? h[6] : 1),
                h[7] / (double)(h[6] ? h[6] : 1) / 100.0, h[5] / (double)(h[7] ? h[7] : 1) / 10.0);
    }
#endif
    // the root's code and the dataflow error word in one pinned buffer: one wait per solve
    if (!d->h_res) GM_HIP(hipHostMalloc((void **)&d->h_res, 8, hipHostMallocDefault));
    d->h_res[0] = d->h_res[1] = 0;
    GM_HIP(hipMemcpyAsync(d->h_res, d->table + box_index_of_key((uint32_t)root), 1, hipMemcpyDeviceToHost, c->stream));
    if (d->flow) GM_HIP(hipMemcpyAsync(d->h_res + 1, d->d_flow + 8, 4, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    const uint8_t rs = (uint8_t)(d->h_res[0] & 0xFFu);
    if (d->flow && d->h_res[1]) {
        // A wait timed out: solve again with the tier launches.  The context keeps tier
        // launches from then on (box_flow_failed, cleared by gm_set_option GM_OPT_BOX_FLOW);
        // every solve that fell back counts in gm_stats_t.flow_fallbacks.
        fprintf(stderr, "gmsolve: the one-launch box solve timed out waiting for a child box; "
                        "re-solving with tier launches\n");
        c->box_flow_failed = true;
        c->box_flow_fallbacks++;
        const int fb = c->box_flow_fallbacks;
        const int rc = dense_box_solve(c, root);
        c->stats.flow_fallbacks = fb;
        return rc;
    }
    const double t1 = now_ms();
    c->root_record = record_of_code(rs);
    uint64_t n = 1;
    for (int j = 0; j < 8; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    box_tier_counts(root, c->tier_counts);
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = (int)d->tier_off.size() - 1;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.forward_ms = 0;
    c->stats.exchanged_bytes = 0;
    c->stats.flow_fallbacks = c->box_flow_fallbacks;
    c->stats.algo_bytes = (uint64_t)((double)(1ull << 32) * (1.0 + 1.8125 * 8));
    c->stats.table_bytes = 1ull << 32;
    if (c->timing) {
        float ms = 0;
        GM_HIP(hipEventElapsedTime(&ms, d->ev[0], d->ev[1]));
        c->stats.kernel_ms = ms;
        c->stats.kernel_launches = box_launches(d);
    }
    return GM_OK;
}

int dense_box_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    if (c->dist_box) return dist_box_query(c, keys, recs, n);
    DenseBox *d = c->dbox;
    if (!n) return GM_OK;
    uint64_t *dk;
    uint16_t *dr;
    const uint64_t chunk = std::min<uint64_t>(n, 1ull << 26);
    GM_HIP(hipMalloc(&dk, chunk * 8));
    GM_HIP(hipMalloc(&dr, chunk * 2));
    for (uint64_t o = 0; o < n; o += chunk) {
        const uint64_t m = std::min(chunk, n - o);
        GM_HIP(hipMemcpyAsync(dk, keys + o, m * 8, hipMemcpyHostToDevice, c->stream));
        box_launch_query(d->d_tables, nullptr, c->root, dk, dr, m, c->stream);
        GM_HIP(hipMemcpyAsync(recs + o, dr, m * 2, hipMemcpyDeviceToHost, c->stream));
    }
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

// keys of the root's region in ascending order (heap 0 fastest)
void box_region_keys(uint64_t root, uint64_t *keys, uint64_t n) {
    uint32_t lim[8], h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 8; i++) lim[i] = (uint32_t)((root >> (4 * i)) & 15u);
    for (uint64_t j = 0; j < n; j++) {
        uint32_t k = 0;
        for (int i = 0; i < 8; i++) k |= h[i] << (4 * i);
        keys[j] = k;
        for (int i = 0; i < 8; i++) {
            if (h[i] < lim[i]) { h[i]++; break; }
            h[i] = 0;
        }
    }
}

// Export: the root's region in ascending key order.
int dense_box_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    if (c->dist_box) return dist_box_export(c, keys, recs, cap, n);
    DenseBox *d = c->dbox;
    *n = c->n_positions;
    if (!keys) return GM_OK;
    if (cap < c->n_positions) {
        set_error("export buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)c->n_positions);
        return GM_E_CAP;
    }
    box_region_keys(c->root, keys, c->n_positions);
    if (c->n_positions <= (1ull << 26)) return dense_box_query(c, keys, recs, c->n_positions);
    // large regions: one copy of the table, decoded on the host
    std::vector<uint8_t> tab(1ull << 32);
    GM_HIP(hipMemcpy(tab.data(), d->table, tab.size(), hipMemcpyDeviceToHost));
    for (uint64_t j = 0; j < c->n_positions; j++) recs[j] = record_of_code(tab[box_index_of_key((uint32_t)keys[j])]);
    return GM_OK;
}

int dense_box_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    if (c->dist_box) return dist_box_digest(c, digest, n);
    DenseBox *d = c->dbox;
    GM_HIP(hipMemsetAsync(d->d_acc, 0, 16, c->stream));
    box_launch_digest(d->table, d->d_boxes, d->boxes.size(), c->root, (unsigned long long *)d->d_acc, c->stream);
    GM_HIP(hipGetLastError());
    uint64_t hst[2];
    GM_HIP(hipMemcpyAsync(hst, d->d_acc, 16, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    *digest = hst[0];
    *n = hst[1];
    return GM_OK;
}

int dense_box_table(Ctx *c, void **p, uint64_t *bytes) {
    if (c->dist_box) return dist_box_table(c, p, bytes);
    *p = c->dbox->table;
    *bytes = 1ull << 32;
    return GM_OK;
}

void dense_box_free(Ctx *c) {
    DenseBox *d = c->dbox;
    if (!d) return;
    if (d->graph) (void)hipGraphExecDestroy(d->graph);
    for (auto e : d->ev)
        if (e) (void)hipEventDestroy(e);
    if (d->owned && d->table) (void)hipFree(d->table);
    for (void *q : {(void *)d->d_boxes, (void *)d->d_groups, (void *)d->d_acc, (void *)d->d_flow, (void *)d->d_tables})
        if (q) (void)hipFree(q);
    if (d->h_res) (void)hipHostFree(d->h_res);
    delete d;
    c->dbox = nullptr;
}

}  // namespace gm
