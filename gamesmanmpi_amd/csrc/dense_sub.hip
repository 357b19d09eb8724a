// dense_sub.hip -- dense tiered retrograde for the synthetic subtraction game.
//
// Replaces, for config 5, the reference's per-edge job loop (Process.lookup /
// distribute / resolve, src/new_process.py:102-265) and its shelve tables
// (src/cache_dict.py): every one of the 16^heaps positions gets a 1-byte slot
// in one HBM array indexed by the key itself (the order-preserving codes of
// gm_common.hpp: WIN R -> R+1, LOSS R -> 255-R; exported as u16 records).
//
// Decomposition.  A key is `heaps` nibbles.  The low LOW nibbles index a
// position inside a *block* of 16^LOW slots (4 KiB at LOW = 3) that a workgroup
// solves in LDS; the high HIGH = heaps - LOW nibbles name the block.  A move
// lowers exactly one nibble, so a position's children are either in its own
// block (low move) or at the same offset of a block whose high part is 1 or 2
// smaller in one nibble (high move).  Blocks are processed in tiers of their
// high-nibble sum, one launch per tier:
//
//   pass A  fold the high children: for every valid child block, stream its
//           codes with 16-B buffer loads and keep the running max -- fully
//           coalesced whole-block reads, one scalar buffer descriptor per child;
//   pass B  walk the block's low tiers (low-nibble sum 0..15*LOW) in LDS: each
//           position folds its <= 2*LOW in-block children and turns the best
//           code into its own (parent_code), one barrier per low tier;
//   pass C  write the block back with 16-B stores.
//
// The default kernel (sub_tier_kernel_x4) solves FOUR blocks per workgroup with
// their LDS images interleaved (slot 4L+k), so every address, branch and LDS
// access of pass B serves four positions and the arithmetic is packed u16.
//
// HBM bytes per position: 1 written + 1 per high child (1.8125 per high nibble
// on average).  The SURVEY §8d edge model charges 1 B per record and per child
// edge: 1 + 14.5 = 15.5 B per position at 8 heaps (31 B with u16 records).
#include "gm_internal.hpp"

#include <algorithm>
#include <type_traits>
#include <chrono>

namespace gm {

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

struct DenseSub {
    int heaps = 0, low = 0, high = 0, nt = 128;   // nt 0 = interleaved x4 kernel
    int want_threads = 0, want_x4 = 0, want_order = 0;
    uint8_t *table = nullptr;           // 16^heaps codes
    bool owned = false;
    uint64_t slots = 0;
    uint8_t *zero = nullptr;            // one block of zeros (padding source)
    uint32_t *d_blocks = nullptr;       // high parts sorted by (tier, value)
    std::vector<uint32_t> tier_off;     // block offsets per high tier
    uint64_t *d_acc = nullptr;          // digest / counters
    hipGraphExec_t graph = nullptr;
    hipStream_t graph_stream = nullptr;
    // dataflow kernel (nt == -3): per-XCD item lists, heads, per-block flags
    void *flow_items = nullptr;
    uint32_t *flow_list_off = nullptr, *flow_heads = nullptr, *flow_flags = nullptr, *flow_abort = nullptr;
    unsigned flow_grid = 0;
    std::vector<hipEvent_t> ev;         // timing events
};

// one scalar buffer descriptor per block (num_records = block bytes; 0 drops stores)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t block_rsrc(const uint8_t *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, bytes, 0x00020000);
}

__device__ __forceinline__ u32x4v load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// Byte codes have no packed max on CDNA4, so 16 codes (one u32x4 load) are
// split into u16 pairs -- even bytes (positions 4j, 4j+2) with one v_and, odd
// bytes (4j+1, 4j+3) with one v_perm -- and folded with v_pk_max_u16.
struct Fold16 {
    uint32_t e[4], o[4];
};
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a),
                                                                  __builtin_bit_cast(u16x2, b)));
}
__device__ __forceinline__ uint32_t even_bytes(uint32_t x) { return x & 0x00FF00FFu; }
__device__ __forceinline__ uint32_t odd_bytes(uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c01u); }
template <int N>
__device__ __forceinline__ Fold16 fold16(const u32x4v (&v)[N]) {
    Fold16 f;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        f.e[j] = even_bytes(v[0][j]);
        f.o[j] = odd_bytes(v[0][j]);
#pragma unroll
        for (int m = 1; m < N; m++) {
            f.e[j] = pk_max(f.e[j], even_bytes(v[m][j]));
            f.o[j] = pk_max(f.o[j], odd_bytes(v[m][j]));
        }
    }
    return f;
}
// parent_code on a pair of u16 codes (each <= 255, so no borrow crosses the halves)
__device__ __forceinline__ uint32_t code_x2(uint32_t b) {
    return (0x00FF00FFu - b) + ((b >> 6) & 0x00020002u);
}
// four u16 codes (positions 4j..4j+3 as pairs (p0,p1), (p2,p3)) -> one dword of bytes
__device__ __forceinline__ uint32_t pack_bytes(uint32_t p01, uint32_t p23) {
    return __builtin_amdgcn_perm(p23, p01, 0x06040200u);
}

// pointers of the 2*HIGH child blocks of high part hp (slot 2j+s = "take s+1
// from high nibble j"); a missing child re-reads the first existing one (max
// is idempotent, the repeat is an L2 hit) or, with none, the zero block
template <int LOW, int HIGH, int NMAX>
__device__ __forceinline__ void child_blocks(const uint8_t *table, const uint8_t *zero, uint32_t hp, bool valid,
                                             const uint8_t *(&src)[NMAX]) {
    const uint8_t *first = zero;
#if defined(GM_EXP) && (GM_EXP & 2)
    valid = false;   // experiment: no child-block traffic
#endif
#pragma unroll
    for (int j = HIGH - 1; j >= 0; j--) {
        const uint32_t h = (hp >> (4 * j)) & 15u;
        if (valid && h >= 1) first = table + ((uint64_t)(hp - (1u << (4 * j))) << (4 * LOW));
    }
#pragma unroll
    for (int j = 0; j < HIGH; j++) {
        const uint32_t h = (hp >> (4 * j)) & 15u;
        src[2 * j] = (valid && h >= 1) ? table + ((uint64_t)(hp - (1u << (4 * j))) << (4 * LOW)) : first;
        src[2 * j + 1] = (valid && h >= 2) ? table + ((uint64_t)(hp - (2u << (4 * j))) << (4 * LOW)) : first;
    }
    if constexpr (HIGH == 0) src[0] = zero;
}

__device__ __forceinline__ uint32_t xcd_order(uint32_t b, uint32_t n) {
    // blocks b and b+8 share an XCD (MI355X_MICROARCH.md "Workgroup dispatch"):
    // give each XCD a contiguous run of the tier list, whose neighbouring high
    // parts share child blocks in that XCD's L2
    const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}
// the same runs, each walked from its end (serpentine order on alternate tiers: the
// groups an XCD starts a tier with are next to the ones it ended the previous tier with)
__device__ __forceinline__ uint32_t xcd_order_rev(uint32_t b, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, i = b >> 3;
    const uint32_t len = q + (x < r ? 1u : 0u);
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (len - 1u - i);
}

// ---------------------------------------------------------------------------
// One block per workgroup of NT threads (any LOW).
template <int LOW, int HIGH, int NT>
__global__ __launch_bounds__(NT) void sub_tier_kernel(uint8_t *__restrict__ table,
                                                      const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                      const uint8_t *__restrict__ zero) {
    constexpr int NPOS = 1 << (4 * LOW);
    constexpr int NCH = NPOS / 16;                      // 16-position chunks
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    __shared__ __attribute__((aligned(16))) uint16_t s[NPOS];
    const int tid = threadIdx.x;
    const uint32_t hp = blocks[xcd_order(blockIdx.x, nblk)];

    const uint8_t *src[NMAX];
    child_blocks<LOW, HIGH, NMAX>(table, zero, hp, true, src);
    __amdgpu_buffer_rsrc_t rs[NMAX];
#pragma unroll
    for (int k = 0; k < NMAX; k++) rs[k] = block_rsrc(src[k], NPOS);
    for (uint32_t c = tid; c < (uint32_t)NCH; c += NT) {
        u32x4v v[NMAX];
#pragma unroll
        for (int k = 0; k < NMAX; k++) v[k] = load16(rs[k], 16u * c);
        const Fold16 f = fold16(v);
        u32x4v lo, hi;   // positions 16c..16c+7, 16c+8..16c+15 as u16 pairs
        lo[0] = __builtin_amdgcn_perm(f.o[0], f.e[0], 0x05040100u);
        lo[1] = __builtin_amdgcn_perm(f.o[0], f.e[0], 0x07060302u);
        lo[2] = __builtin_amdgcn_perm(f.o[1], f.e[1], 0x05040100u);
        lo[3] = __builtin_amdgcn_perm(f.o[1], f.e[1], 0x07060302u);
        hi[0] = __builtin_amdgcn_perm(f.o[2], f.e[2], 0x05040100u);
        hi[1] = __builtin_amdgcn_perm(f.o[2], f.e[2], 0x07060302u);
        hi[2] = __builtin_amdgcn_perm(f.o[3], f.e[3], 0x05040100u);
        hi[3] = __builtin_amdgcn_perm(f.o[3], f.e[3], 0x07060302u);
        *(u32x4v *)(s + 16 * c) = lo;
        *(u32x4v *)(s + 16 * c + 8) = hi;
    }
    __syncthreads();

    auto best_of = [&](int L) -> uint32_t {
        uint32_t best = s[L];
#pragma unroll
        for (int j = 0; j < LOW; j++) {
            const int h = (L >> (4 * j)) & 15;
            if (h >= 1) best = max(best, (uint32_t)s[L - (1 << (4 * j))]);
            if (h >= 2) best = max(best, (uint32_t)s[L - (2 << (4 * j))]);
        }
        return (hp == 0 && L == 0) ? 255u : parent_code(best);
    };
    if constexpr (LOW == 3) {
        // (heap0, heap1) pairs spread over the threads; heap2 is fixed by the tier.
        // A step's positions are independent: all reads before any write.
        constexpr int PER = 256 / NT;
        int sum[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const int p = tid + NT * k;
            sum[k] = (p & 15) + (p >> 4);
        }
        for (int tau = 0; tau <= 45; tau++) {
            uint32_t res[PER];
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int c = tau - sum[k];
                res[k] = (c >= 0 && c <= 15) ? best_of(tid + NT * k + 256 * c) : 0u;
            }
#pragma unroll
            for (int k = 0; k < PER; k++) {
                const int c = tau - sum[k];
                if (c >= 0 && c <= 15) s[tid + NT * k + 256 * c] = (uint16_t)res[k];
            }
            __syncthreads();
        }
    } else {
        for (int tau = 0; tau <= 15 * LOW; tau++) {
            for (int L = tid; L < NPOS; L += NT) {
                int sum = 0;
#pragma unroll
                for (int j = 0; j < LOW; j++) sum += (L >> (4 * j)) & 15;
                if (sum == tau) s[L] = (uint16_t)best_of(L);
            }
            __syncthreads();
        }
    }

    const __amdgpu_buffer_rsrc_t wr = block_rsrc(table + ((uint64_t)hp << (4 * LOW)), NPOS);
    for (uint32_t c = tid; c < (uint32_t)NCH; c += NT) {
        const u32x4v lo = *(const u32x4v *)(s + 16 * c), hi = *(const u32x4v *)(s + 16 * c + 8);
        u32x4v o;
        o[0] = pack_bytes(lo[0], lo[1]);
        o[1] = pack_bytes(lo[2], lo[3]);
        o[2] = pack_bytes(hi[0], hi[1]);
        o[3] = pack_bytes(hi[2], hi[3]);
        __builtin_amdgcn_raw_buffer_store_b128(o, wr, 16u * c, 0, 0);
    }
}

// ---------------------------------------------------------------------------
// Anti-diagonal order of the 256 (a0, a1) pairs of a 16 x 16 plane: sorted by
// s = a0 + a1, then by a1.  diag_base(s) = pairs with a smaller sum.
__device__ __forceinline__ int diag_base(int s) {
    return s <= 16 ? (s * (s + 1)) >> 1 : 136 + (((47 - s) * (s - 16)) >> 1);
}
__device__ __forceinline__ int diag_index(int a0, int a1) {
    const int s = a0 + a1;
    return diag_base(s) + (s <= 15 ? a1 : a1 - (s - 15));
}

// ---------------------------------------------------------------------------
// Four blocks per workgroup (LOW = 3), LDS images interleaved: position L of the
// group's k-th block is the u16 at 4L + k.  Pass B handles the four copies of a
// position with one address, one validity test and one ds_read_b64 per child,
// in packed u16 arithmetic.  Pass A folds each block's children separately and
// transposes 4 x 8 codes at a time with v_perm_b32; pass C transposes back.

// DIAG: pass B gives thread t the t-th (a0, a1) pair in anti-diagonal order
// instead of a0 = t & 15, a1 = t >> 4.  A thread's position at low tier tau is
// (a0, a1, tau - a0 - a1), valid for a0 + a1 in [tau - 15, tau]; with diagonals
// packed into waves, a wave whose diagonals are all out of range skips the step
// (~94 wave-steps per workgroup instead of 4 x 46, most lanes masked).
template <int HIGH, bool DIAG>
__global__ __launch_bounds__(256) void sub_tier_kernel_x4(uint8_t *__restrict__ table,
                                                          const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                          const uint8_t *__restrict__ zero) {
    constexpr int NPOS = 4096, NCH = 256, NT = 256, K = 4;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    __shared__ __attribute__((aligned(16))) uint16_t s[NPOS * K];   // 32 KiB
    const int tid = threadIdx.x;
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + K - 1) / K);
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = grp * K + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? blocks[idx] : 0u;
    }

    // ---- pass A -------------------------------------------------------------
    // NCH == NT: one 16-position chunk per thread.  The blocks are folded one
    // after the other (sched_barrier) so that only one block's descriptors and
    // loads are live at a time: 2*HIGH loads of 16 B in flight per thread.
    static_assert(NCH == NT, "one chunk per thread");
    {
        const uint32_t c = tid;
        Fold16 f[K];   // f[k].e[j] = positions (4j, 4j+2), .o[j] = (4j+1, 4j+3) of chunk c, block k
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint8_t *src[NMAX];
            child_blocks<3, HIGH, NMAX>(table, zero, hp[k], valid[k], src);
            u32x4v v[NMAX];
#pragma unroll
            for (int m = 0; m < NMAX; m++) v[m] = load16(block_rsrc(src[m], NPOS), 16u * c);
            f[k] = fold16(v);
            __builtin_amdgcn_sched_barrier(0);
        }
        // transpose to the interleaved image: position p -> 4 u16 (blocks 0..3)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            u32x4v o0, o1;
            o0[0] = __builtin_amdgcn_perm(f[1].e[j], f[0].e[j], 0x05040100u);   // pos 4j,   blocks 0,1
            o0[1] = __builtin_amdgcn_perm(f[3].e[j], f[2].e[j], 0x05040100u);   // pos 4j,   blocks 2,3
            o0[2] = __builtin_amdgcn_perm(f[1].o[j], f[0].o[j], 0x05040100u);   // pos 4j+1
            o0[3] = __builtin_amdgcn_perm(f[3].o[j], f[2].o[j], 0x05040100u);
            o1[0] = __builtin_amdgcn_perm(f[1].e[j], f[0].e[j], 0x07060302u);   // pos 4j+2
            o1[1] = __builtin_amdgcn_perm(f[3].e[j], f[2].e[j], 0x07060302u);
            o1[2] = __builtin_amdgcn_perm(f[1].o[j], f[0].o[j], 0x07060302u);   // pos 4j+3
            o1[3] = __builtin_amdgcn_perm(f[3].o[j], f[2].o[j], 0x07060302u);
            *(u32x4v *)((char *)s + 128u * c + 32u * j) = o0;
            *(u32x4v *)((char *)s + 128u * c + 32u * j + 16u) = o1;
        }
    }
    __syncthreads();

    // ---- pass B -------------------------------------------------------------
    // Thread (a0, a1) owns the column c = 0..15 and solves (a0, a1, c) at low tier
    // tau = a0 + a1 + c.  An invalid in-block child reads the position itself (max is
    // idempotent), so the seven ds_read_b64 of a step issue back to back with one
    // wait and no branches; position 0 (tau = 0) is peeled so the root override
    // stays out of the loop.
    int a0 = tid & 15, a1 = tid >> 4;
    if constexpr (DIAG) {
        int sd = 0;
        while (diag_base(sd + 1) <= tid) sd++;
        a1 = sd <= 15 ? tid - diag_base(sd) : tid - diag_base(sd) + sd - 15;
        a0 = sd - a1;
    }
    const int s0 = a0 + a1;
    const uint32_t me = 8u * (uint32_t)(a0 + 16 * a1);
    const uint32_t d01 = a0 >= 1 ? 8u : 0u, d02 = a0 >= 2 ? 16u : 0u;
    const uint32_t d11 = a1 >= 1 ? 128u : 0u, d12 = a1 >= 2 ? 256u : 0u;
    char *const sb = (char *)s;
    auto ld = [&](uint32_t off) -> u32x2v { return *(const u32x2v *)(sb + off); };
#if defined(GM_EXP) && (GM_EXP & 1)
    constexpr int TAU_END = 0;   // experiment: no pass B
#else
    constexpr int TAU_END = 45;
#endif
    if (tid == 0) {
        u32x2v r = ld(0);
        r[0] = code_x2(r[0]);
        r[1] = code_x2(r[1]);
        if (valid[0] && hp[0] == 0) r[0] = (r[0] & 0xFFFF0000u) | 255u;   // all heaps empty: LOSS in 0
        *(u32x2v *)sb = r;
    }
    __syncthreads();
    for (int tau = 1; tau <= TAU_END; tau++) {
        const int c = tau - s0;
        if (c >= 0 && c <= 15) {
            const uint32_t o = me + 2048u * (uint32_t)c;
            const uint32_t dc1 = c >= 1 ? 2048u : 0u, dc2 = c >= 2 ? 4096u : 0u;
            const u32x2v v0 = ld(o), v1 = ld(o - d01), v2 = ld(o - d02), v3 = ld(o - d11), v4 = ld(o - d12),
                         v5 = ld(o - dc1), v6 = ld(o - dc2);
            u32x2v r;
#pragma unroll
            for (int h = 0; h < 2; h++)
                r[h] = code_x2(pk_max(pk_max(pk_max(v0[h], v1[h]), pk_max(v2[h], v3[h])),
                                      pk_max(pk_max(v4[h], v5[h]), v6[h])));
            *(u32x2v *)(sb + o) = r;
        }
        __syncthreads();
    }

    // ---- pass C -------------------------------------------------------------
    __amdgpu_buffer_rsrc_t wr[K];
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0);
#if defined(GM_EXP) && (GM_EXP & 4)
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table, 0);   // experiment: stores dropped (out of range)
#endif
    {
        const uint32_t c = tid;
        u32x4v out[K];   // 16 codes of chunk c per block
#pragma unroll
        for (int j = 0; j < 4; j++) {   // positions 4j..4j+3: 8 B each (blocks 0,1 | 2,3)
            const u32x4v q0 = *(const u32x4v *)((const char *)s + 128u * c + 32u * j);
            const u32x4v q1 = *(const u32x4v *)((const char *)s + 128u * c + 32u * j + 16u);
            // [p0.k, p1.k, p0.k+1, p1.k+1] and [p2.k, p3.k, p2.k+1, p3.k+1] for k = 0 (A) and 2 (B)
            const uint32_t xa = __builtin_amdgcn_perm(q0[2], q0[0], 0x06020400u);
            const uint32_t ya = __builtin_amdgcn_perm(q1[2], q1[0], 0x06020400u);
            const uint32_t xb = __builtin_amdgcn_perm(q0[3], q0[1], 0x06020400u);
            const uint32_t yb = __builtin_amdgcn_perm(q1[3], q1[1], 0x06020400u);
            out[0][j] = __builtin_amdgcn_perm(ya, xa, 0x05040100u);
            out[1][j] = __builtin_amdgcn_perm(ya, xa, 0x07060302u);
            out[2][j] = __builtin_amdgcn_perm(yb, xb, 0x05040100u);
            out[3][j] = __builtin_amdgcn_perm(yb, xb, 0x07060302u);
        }
#pragma unroll
        for (int k = 0; k < K; k++)   // num_records 0 drops the store of an unused slot
            __builtin_amdgcn_raw_buffer_store_b128(out[k], wr[k], 16u * c, 0, 0);
    }
}

// ---------------------------------------------------------------------------
// Byte-image variant (GM_OPT_SUB_INTERLEAVE 6): the four blocks' codes of a
// position share one dword of LDS (byte k = block k), so a workgroup's image is
// 16 KiB instead of 32 and twice as many workgroups can be resident per CU to
// hide pass B's barrier chain and pass A's load latency.  Pass B reads seven
// dwords per position and takes the bytewise max as two u16-pair maxima
// (even / odd bytes).
__device__ __forceinline__ uint32_t code_x4(uint32_t b) {   // parent_code on four bytes
    return ~b + ((b >> 6) & 0x02020202u);
}
// parent codes of split halves: E holds codes in the low byte of each u16, O in the high byte
__device__ __forceinline__ uint32_t code_lo2(uint32_t e) { return (0x00FF00FFu - e) + ((e >> 6) & 0x00020002u); }
__device__ __forceinline__ uint32_t code_hi2(uint32_t o) { return (0xFF00FF00u - o) + ((o >> 6) & 0x02000200u); }

#ifndef GM_PASSB_PRIO
#define GM_PASSB_PRIO 0   // s_setprio of pass B (0 = off)
#endif
#ifndef GM_PASSB_REG
#define GM_PASSB_REG 2   // pass B children (a0-1, a0-2) by DPP and (c-1, c-2) from registers, codes split (2)
#endif
#ifndef GM_B4_WAVES
#define GM_B4_WAVES 1
#endif
#ifndef GM_B4_LAT_WAVES
#define GM_B4_LAT_WAVES 1   // min waves per SIMD for the latency form (1: the compiler's choice, 126 VGPRs)
#endif
#ifndef GM_B4_STORE_CPOL
#define GM_B4_STORE_CPOL 16   // sc1: write-through, the stored block does not stay in L2 (0 = plain)
#endif
template <int NMAX>
__device__ __forceinline__ void p4_fold(const u32x4v (&v)[NMAX], uint32_t (&e)[4], uint32_t (&o)[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        uint32_t ev = v[0][j] & 0x00FF00FFu, ov = v[0][j];   // ov: odd bytes valid in the high byte of each u16
#pragma unroll
        for (int m = 1; m < NMAX; m++) {
            ev = pk_max(ev, v[m][j] & 0x00FF00FFu);
            ov = pk_max(ov, v[m][j]);
        }
        e[j] = ev;
        o[j] = ov;
    }
}
// four blocks' folds of chunk c -> the byte image (position p: byte k = block k)
__device__ __forceinline__ void p4_write_image(uint32_t *s, uint32_t c, const uint32_t (&e)[4][4],
                                               const uint32_t (&o)[4][4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t xe = __builtin_amdgcn_perm(e[1][j], e[0][j], 0x06020400u);
        const uint32_t ye = __builtin_amdgcn_perm(e[3][j], e[2][j], 0x06020400u);
        const uint32_t xo = __builtin_amdgcn_perm(o[1][j], o[0][j], 0x07030501u);
        const uint32_t yo = __builtin_amdgcn_perm(o[3][j], o[2][j], 0x07030501u);
        u32x4v q;
        q[0] = __builtin_amdgcn_perm(ye, xe, 0x05040100u);   // 4j
        q[1] = __builtin_amdgcn_perm(yo, xo, 0x05040100u);   // 4j+1
        q[2] = __builtin_amdgcn_perm(ye, xe, 0x07060302u);   // 4j+2
        q[3] = __builtin_amdgcn_perm(yo, xo, 0x07060302u);   // 4j+3
        *(u32x4v *)(s + 16 * c + 4 * j) = q;
    }
}
// the 2*HIGH child blocks of block hp: one whole-table descriptor, each child a
// scalar offset (a missing child re-reads the first existing one; a block with
// none, only high part 0, reads through a zero-size descriptor: all 0)
// the folds of blocks 2 pr and 2 pr + 1 -> bytes 2 pr, 2 pr + 1 of the image's dwords (u16 stores)
__device__ __forceinline__ void p4_write_pair(uint32_t *s, uint32_t c, int pr, const uint32_t (&e)[2][4],
                                              const uint32_t (&o)[2][4]) {
    char *const b = (char *)s;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t xe = __builtin_amdgcn_perm(e[1][j], e[0][j], 0x06020400u);   // positions 4j | 4j+2
        const uint32_t xo = __builtin_amdgcn_perm(o[1][j], o[0][j], 0x07030501u);   // positions 4j+1 | 4j+3
        const uint32_t a = 4u * (16u * c + 4u * j) + 2u * (uint32_t)pr;
        *(uint16_t *)(b + a) = (uint16_t)xe;
        *(uint16_t *)(b + a + 4) = (uint16_t)xo;
        *(uint16_t *)(b + a + 8) = (uint16_t)(xe >> 16);
        *(uint16_t *)(b + a + 12) = (uint16_t)(xo >> 16);
    }
}
#ifndef GM_SKIP_MISSING
#define GM_SKIP_MISSING 1
#endif
template <int HIGH, int LCPOL = 0>
__device__ __forceinline__ void p4_issue(uint8_t *table, uint32_t hp, bool valid, uint32_t c,
                                         u32x4v (&v)[2 * HIGH > 0 ? 2 * HIGH : 1]) {
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    uint32_t soff[NMAX];
    uint32_t first = 0;
    bool any = false;
#if defined(GM_EXP) && (GM_EXP & 2)
    valid = false;   // experiment: no child-block traffic (out-of-range loads return 0)
#endif
#pragma unroll
    for (int j = HIGH - 1; j >= 0; j--)
        if (valid && ((hp >> (4 * j)) & 15u) >= 1) { first = (hp - (1u << (4 * j))) << 12; any = true; }
#pragma unroll
    for (int j = 0; j < HIGH; j++) {
        const uint32_t h = (hp >> (4 * j)) & 15u;
        soff[2 * j] = (valid && h >= 1) ? (hp - (1u << (4 * j))) << 12 : first;
        soff[2 * j + 1] = (valid && h >= 2) ? (hp - (2u << (4 * j))) << 12 : first;
    }
    if constexpr (HIGH == 0) soff[0] = 0;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(table, 0, any ? 0xFFFFFFFFu : 0u, 0x00020000);
#if GM_SKIP_MISSING
    // a missing child (heap nibble < 1 or < 2) reads through a zero-size descriptor: the
    // load returns 0 (max ignores it) without touching L1/L2 -- 9.06 child blocks per
    // block on average instead of 10 loads
    const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(table, 0, 0u, 0x00020000);
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const uint32_t h = HIGH > 0 ? (hp >> (4 * (m >> 1))) & 15u : 0u;
        const bool ok = HIGH > 0 && valid && h >= (uint32_t)(m & 1) + 1u;
        v[m] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(ok ? r : rz, 16u * c, soff[m], LCPOL));
    }
#else
#pragma unroll
    for (int m = 0; m < NMAX; m++)
        v[m] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, 16u * c, soff[m], LCPOL));
#endif
}

// One workgroup solves the four blocks hp[0..3] (valid[k] false: slot unused).
// CPOL = cache policy of the child loads and the stores (0 plain; CPOL_SC1 in the
// dataflow kernel, whose consumers may sit on another XCD: write-through stores,
// L1-bypassing loads -- MI355X_MICROARCH.md, inter-workgroup visibility).
constexpr int CPOL_SC1 = 16;
// XD (sharded solve): block k also goes to the extra destinations xdst[xoff[idx0 + k] ..
// xoff[idx0 + k + 1]) -- symmetric-fill images in the table and halo ring slots --
// from the same registers, so no separate fill / pack launch follows the tier.
// LAT (small tiers, latency-bound): all four blocks' child loads are issued before
// any is folded -- one memory round trip instead of four -- at the price of the
// VGPRs that limit the default kernel to 7 workgroups per CU.
template <int HIGH, int CPOL, int LCPOL = CPOL, bool XD = false, bool LAT = false>
__device__ __forceinline__ void b4_solve(uint8_t *__restrict__ table, const uint8_t *__restrict__ zero,
                                         const uint32_t (&hp)[4], const bool (&valid)[4], uint32_t *s,
                                         const uint32_t *__restrict__ xoff = nullptr,
                                         const uint64_t *__restrict__ xdst = nullptr, uint32_t idx0 = 0) {
    constexpr int NPOS = 4096, NCH = 256, NT = 256, K = 4;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    const int tid = threadIdx.x;
    static_assert(NCH == NT, "one chunk per thread");

    // ---- pass A: chunk tid = positions 16 tid .. 16 tid + 15
    if constexpr (LAT) {
        const uint32_t c = tid;
        u32x4v v[K][NMAX];
#pragma unroll
        for (int k = 0; k < K; k++) p4_issue<HIGH, LCPOL>(table, hp[k], valid[k], c, v[k]);
#if GM_B4_LAT_BARRIER
        __builtin_amdgcn_sched_barrier(0);   // keep every load ahead of the first fold
#endif
        uint32_t e[2][4], o[2][4];
#pragma unroll
        for (int k = 0; k < K; k += 2) {
            p4_fold<NMAX>(v[k], e[0], o[0]);
            p4_fold<NMAX>(v[k + 1], e[1], o[1]);
            p4_write_pair(s, c, k >> 1, e, o);
        }
    } else {
        const uint32_t c = tid;
        Fold16 f[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint8_t *src[NMAX];
            child_blocks<3, HIGH, NMAX>(table, zero, hp[k], valid[k], src);
            u32x4v v[NMAX];
#pragma unroll
            for (int m = 0; m < NMAX; m++)
                v[m] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(block_rsrc(src[m], NPOS), 16u * c, 0, LCPOL));
            f[k] = fold16(v);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {   // positions 4j .. 4j+3 -> one dword each (bytes = blocks 0..3)
            const uint32_t xe = __builtin_amdgcn_perm(f[1].e[j], f[0].e[j], 0x06020400u);
            const uint32_t ye = __builtin_amdgcn_perm(f[3].e[j], f[2].e[j], 0x06020400u);
            const uint32_t xo = __builtin_amdgcn_perm(f[1].o[j], f[0].o[j], 0x06020400u);
            const uint32_t yo = __builtin_amdgcn_perm(f[3].o[j], f[2].o[j], 0x06020400u);
            u32x4v q;
            q[0] = __builtin_amdgcn_perm(ye, xe, 0x05040100u);   // 4j
            q[1] = __builtin_amdgcn_perm(yo, xo, 0x05040100u);   // 4j+1
            q[2] = __builtin_amdgcn_perm(ye, xe, 0x07060302u);   // 4j+2
            q[3] = __builtin_amdgcn_perm(yo, xo, 0x07060302u);   // 4j+3
            *(u32x4v *)(s + 16 * c + 4 * j) = q;
        }
    }
    __syncthreads();

    // ---- pass B (see sub_tier_kernel_x4): thread (a0, a1), position c = tau - a0 - a1
#if GM_PASSB_PRIO
    __builtin_amdgcn_s_setprio(GM_PASSB_PRIO);   // the barrier chain before other workgroups' folds
#endif
    const int a0 = tid & 15, a1 = tid >> 4, s0 = a0 + a1;
    const uint32_t d01 = a0 >= 1 ? 1u : 0u, d02 = a0 >= 2 ? 2u : 0u;
    const uint32_t d11 = a1 >= 1 ? 16u : 0u, d12 = a1 >= 2 ? 32u : 0u;
#if defined(GM_EXP) && (GM_EXP & 1)
    constexpr int TAU_END = 0;   // experiment: no pass B
#else
    constexpr int TAU_END = 45;
#endif
#if GM_PASSB_REG == 2
    // As below, with the codes split while they live in registers (w1_solve): E =
    // bytes 0, 2 in the low byte of each u16 half, O = bytes 1, 3 in the high byte;
    // an inactive lane records 0, so (c-1, c-2) need no validity select.
    uint32_t pe1 = 0, po1 = 0, pe2 = 0, po2 = 0;
    if (tid == 0) {
        const uint32_t v = s[0];
        uint32_t re = code_lo2(v & 0x00FF00FFu), ro = code_hi2(v & 0xFF00FF00u);
        if (valid[0] && hp[0] == 0) re = (re & 0xFFFFFF00u) | 255u;   // all heaps empty: LOSS in 0
        s[0] = re | ro;
        pe1 = re;
        po1 = ro;
    }
    __syncthreads();
    for (int tau = 1; tau <= TAU_END; tau++) {
        const uint32_t n1e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe1, 0x111, 0xF, 0xF, true);
        const uint32_t n1o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po1, 0x111, 0xF, 0xF, true);
        const uint32_t n2e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe2, 0x112, 0xF, 0xF, true);
        const uint32_t n2o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po2, 0x112, 0xF, 0xF, true);
        const int c = tau - s0;
        uint32_t re = 0, ro = 0;
        if (c >= 0 && c <= 15) {
            const uint32_t o = (uint32_t)(tid + 256 * c);
            const uint32_t v0 = s[o], v3 = s[o - d11], v4 = s[o - d12];
            const uint32_t me = pk_max(pk_max(pk_max(v0 & 0x00FF00FFu, v3 & 0x00FF00FFu), pk_max(v4 & 0x00FF00FFu, n1e)),
                                       pk_max(pk_max(n2e, pe1), pe2));
            const uint32_t mo = pk_max(pk_max(pk_max(v0, v3), pk_max(v4, n1o)), pk_max(pk_max(n2o, po1), po2));
            re = code_lo2(me);
            ro = code_hi2(mo & 0xFF00FF00u);
            s[o] = re | ro;
        }
        pe2 = pe1;
        po2 = po1;
        pe1 = re;
        po1 = ro;
        __syncthreads();
    }
#else
    uint32_t p1 = 0, p2 = 0;   // this thread's codes of the last two steps: (a0, a1, c-1), (a0, a1, c-2)
    if (tid == 0) {
        uint32_t r = code_x4(s[0]);
        if (valid[0] && hp[0] == 0) r = (r & 0xFFFFFF00u) | 255u;   // all heaps empty: LOSS in 0
        s[0] = r;
        p1 = r;
    }
    __syncthreads();
#endif
#if GM_PASSB_REG == 2
#elif GM_PASSB_REG
    // Children inside the block, by where they live: (a0-1 | a0-2, a1, c) are the codes
    // lanes tid-1 / tid-2 (same 16-lane DPP row) produced one / two steps ago, moved
    // with row_shr (an invalid child reads 0, which max ignores: every position but
    // the primitive has a child); (a0, a1, c-1 | c-2) are this thread's own last two
    // codes; only (a0, a1-1 | a1-2, c), written by other waves, and the child-block
    // fold s[o] come from LDS.  So a step issues 3 LDS reads instead of 7.
    for (int tau = 1; tau <= TAU_END; tau++) {
        const uint32_t n1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p1, 0x111, 0xF, 0xF, true);   // row_shr:1
        const uint32_t n2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p2, 0x112, 0xF, 0xF, true);   // row_shr:2
        const int c = tau - s0;
        uint32_t r = 0;
        if (c >= 0 && c <= 15) {
            const uint32_t o = (uint32_t)(tid + 256 * c);
            const uint32_t v0 = s[o], v3 = s[o - d11], v4 = s[o - d12];
            const uint32_t q1 = c >= 1 ? p1 : 0u, q2 = c >= 2 ? p2 : 0u;
            const uint32_t e = pk_max(pk_max(pk_max(even_bytes(v0), even_bytes(v3)), pk_max(even_bytes(v4), even_bytes(n1))),
                                      pk_max(pk_max(even_bytes(n2), even_bytes(q1)), even_bytes(q2)));
            const uint32_t od = pk_max(pk_max(pk_max(odd_bytes(v0), odd_bytes(v3)), pk_max(odd_bytes(v4), odd_bytes(n1))),
                                       pk_max(pk_max(odd_bytes(n2), odd_bytes(q1)), odd_bytes(q2)));
            r = code_x4(__builtin_amdgcn_perm(od, e, 0x06020400u));
            s[o] = r;
        }
        p2 = p1;
        p1 = r;
        __syncthreads();
    }
#else
    for (int tau = 1; tau <= TAU_END; tau++) {
        const int c = tau - s0;
        if (c >= 0 && c <= 15) {
            const uint32_t o = (uint32_t)(tid + 256 * c);
            const uint32_t dc1 = c >= 1 ? 256u : 0u, dc2 = c >= 2 ? 512u : 0u;
            const uint32_t v0 = s[o], v1 = s[o - d01], v2 = s[o - d02], v3 = s[o - d11], v4 = s[o - d12],
                           v5 = s[o - dc1], v6 = s[o - dc2];
            const uint32_t e = pk_max(pk_max(pk_max(even_bytes(v0), even_bytes(v1)), pk_max(even_bytes(v2), even_bytes(v3))),
                                      pk_max(pk_max(even_bytes(v4), even_bytes(v5)), even_bytes(v6)));
            const uint32_t od = pk_max(pk_max(pk_max(odd_bytes(v0), odd_bytes(v1)), pk_max(odd_bytes(v2), odd_bytes(v3))),
                                       pk_max(pk_max(odd_bytes(v4), odd_bytes(v5)), odd_bytes(v6)));
            s[o] = code_x4(__builtin_amdgcn_perm(od, e, 0x06020400u));
        }
        __syncthreads();
    }
#endif

    // ---- pass C: back to four 16-byte rows per chunk
#if GM_PASSB_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    __amdgpu_buffer_rsrc_t wr[K];
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0);
#if defined(GM_EXP) && (GM_EXP & 4)
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table, 0);   // experiment: stores dropped (out of range)
#endif
    {
        const uint32_t c = tid;
        u32x4v out[K];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32x4v q = *(const u32x4v *)(s + 16 * c + 4 * j);
            const uint32_t t01 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
            const uint32_t t23 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
            const uint32_t u01 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
            const uint32_t u23 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
            out[0][j] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
            out[1][j] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
            out[2][j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
            out[3][j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
        }
#pragma unroll
        for (int k = 0; k < K; k++) __builtin_amdgcn_raw_buffer_store_b128(out[k], wr[k], 16u * c, 0, CPOL);
        if constexpr (XD) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!valid[k]) continue;
                const uint32_t m1 = xoff[idx0 + k + 1];
                for (uint32_t m = xoff[idx0 + k]; m < m1; m++)
                    __builtin_amdgcn_raw_buffer_store_b128(out[k], block_rsrc((uint8_t *)xdst[m], NPOS), 16u * c, 0, 0);
            }
        }
    }
}

template <int HIGH, bool LAT = false>
__global__ __launch_bounds__(256, LAT ? GM_B4_LAT_WAVES : GM_B4_WAVES) void sub_tier_kernel_b4(uint8_t *__restrict__ table,
                                                          const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                          const uint8_t *__restrict__ zero) {
    constexpr int K = 4;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + K - 1) / K);
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = grp * K + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? blocks[idx] : 0u;
    }
    b4_solve<HIGH, GM_B4_STORE_CPOL, 0, false, LAT>(table, zero, hp, valid, s);
}

// The sharded solve's tier kernel (csrc/dist_sub.hip): as above, plus each block's
// extra destinations (xoff / xdst indexed like `blocks`).
template <int HIGH, bool LAT = false>
__global__ __launch_bounds__(256, GM_B4_WAVES) void sub_tier_kernel_b4x(uint8_t *__restrict__ table,
                                                           const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                           const uint8_t *__restrict__ zero,
                                                           const uint32_t *__restrict__ xoff,
                                                           const uint64_t *__restrict__ xdst) {
    constexpr int K = 4;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + K - 1) / K);
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = grp * K + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? blocks[idx] : 0u;
    }
    b4_solve<HIGH, 0, 0, true, LAT>(table, zero, hp, valid, s, xoff, xdst, grp * K);
}

// ---------------------------------------------------------------------------
// Walker form of the 4-block kernel (GM_OPT_SUB_INTERLEAVE 10 and 11).
//
// Pass B of b4_solve maps thread (a0, a1) to the column c = tau - a0 - a1: 256
// threads walk the block's 46 low tiers with one barrier each, and a thread has a
// position in only 16 of them, so two thirds of pass B's issue slots -- measured:
// pass B alone 2.4 ms of the 4.9 ms 2^32 solve -- are spent on idle lanes and
// barriers.  Here ONE wave walks the whole block after pass A: lane (z = c,
// yb) of the 64 takes the rows y = 4 yb .. 4 yb + 3 (y = a1) of column z and walks
// p = 4 x + (y - 4 yb) (x = a0) in order, lane (z, yb) p steps after its start
// z + 4 yb.  Every child of a position was made at least one step earlier:
//   (z-1 | z-2)  lanes z-1 / z-2 of the same 16-lane row, one / two steps ago:
//                DPP row_shr of their last two codes (z = 0, 1: bound_ctrl zero);
//   (x-1 | x-2)  this lane, 4 / 8 steps ago: a ring of the last 8 codes in
//                registers (x = 0, 1: the ring's initial zeros);
//   (y-1 | y-2)  the image in LDS, where every code is stored as it is made:
//                this lane one / two steps ago, or the row below (lane - 16) one
//                or two steps ago -- one wave's LDS operations complete in
//                order, so no barrier is needed; y = 0, 1 read two zero rows
//                in front of every z slice.
// 91 steps with 64 of 64 lanes busy in most of them, against 4 waves x 46 steps:
// about half the VALU issue of pass B and no barrier.
//
// Option 10 (sub_tier_kernel_wk): 256 threads load (pass A), then one wave walks and
// writes the blocks (pass C); the other three leave.  A per-workgroup trace
// (GM_WK_TRACE build, tools/wk_trace.py) showed what that buys: an exited wave's
// slot is not reused while its workgroup lives, so a CU holds 4 such workgroups
// (128 VGPRs) and at any time ~2 of them walk while ~2 load -- the walk (9.9 us per
// group) and the loads (9 us) alternate instead of overlapping.
//
// Option 11 (sub_tier_kernel_wkp, the default): persistent workgroups of 5 waves and two
// images.  Four waves load and fold group i+1 into one image while the fifth walks
// and writes group i from the other; one barrier per group.  A CU holds 3 of them
// (15 waves of 128 VGPRs), each walking all the time while its loads are in flight.
#ifndef GM_WK_ROT
#define GM_WK_ROT 1   // the walking wave rotates with the workgroup index (spread over the SIMDs)
#endif
#ifndef GM_WK_UNMASK
#define GM_WK_UNMASK 1   // no activity masking in the walk's all-active middle steps
#endif
#ifndef GM_WK_SERP
#define GM_WK_SERP 0   // serpentine XCD runs (alternate tiers walked backwards)
#endif
#ifndef GM_WK_PAIRS
#define GM_WK_PAIRS 0   // pass A in two rounds of two blocks' loads (development option)
#endif
#ifndef GM_WK_WAVES
#define GM_WK_WAVES (GM_WK_PAIRS ? 5 : 4)   // waves per SIMD the register budget must allow
#endif
#ifndef GM_WKP_PER_CU
#define GM_WKP_PER_CU 3   // persistent 320-thread workgroups per CU (5 waves x 128 VGPRs: 15 of 16 slots)
#endif
constexpr int WK_ZS = 292;   // dwords per z slice of the image: 18 rows of 16 + 4 (bank spread for the walk)
constexpr int WK_IMG = WK_ZS * 16;   // dwords per image (18.25 KiB)
__device__ __forceinline__ uint32_t wk_chunk(uint32_t c) {   // image dword of position (0, c & 15, c >> 4)
    return 16u * (c & 15u) + 32u + WK_ZS * (c >> 4);
}
__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shr2(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
}
// parent codes of the split halves (gm_common.hpp parent_code: (255 - b) + 2 (b >> 7)),
// E: codes in the low byte of each u16 (high bytes zero); O: codes in the high byte
__device__ __forceinline__ uint32_t wk_code_e(uint32_t e) { return (e ^ 0x00FF00FFu) + ((e >> 6) & 0x00020002u); }
__device__ __forceinline__ uint32_t wk_code_o(uint32_t o) { return (~o & 0xFF00FF00u) + ((o >> 6) & 0x02000200u); }

#ifdef GM_WK_TRACE
// diagnostic build only (-DGM_WK_TRACE): per-workgroup phase timestamps (s_memrealtime,
// 100 MHz) and hardware ids, written by the walking wave's lane 0 with vector stores
__device__ uint64_t *gm_trace_buf;
__device__ uint32_t *gm_trace_cnt;
__device__ __forceinline__ void wk_trace(uint64_t t0, uint64_t t1, uint64_t t2, uint32_t hp0, uint64_t tl, uint64_t tf) {
    if (gm_trace_buf) {
        const uint64_t t3 = __builtin_amdgcn_s_memrealtime();
        const uint32_t slot = atomicAdd(gm_trace_cnt, 1u);
        if (slot < (1u << 20)) {
            uint64_t *e = gm_trace_buf + 8ull * slot;
            e[0] = t0; e[1] = t1; e[2] = t2; e[3] = t3;
            e[4] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                   ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);   // HW_ID, XCC_ID
            e[5] = (uint64_t)blockIdx.x | ((uint64_t)hp0 << 32);
            e[6] = tl;   // the walking wave's loads all back
            e[7] = tf;   // its folds written
        }
    }
}
#endif

// pass A by 256 loader threads (lt = 0..255: chunk lt of all four blocks, every child
// load in flight at once): the folds into image s; zero = also clear its zero rows
template <int HIGH>
__device__ __forceinline__ void wk_load(uint8_t *__restrict__ table, const uint32_t (&hp)[4], const bool (&valid)[4],
                                        uint32_t *s, uint32_t lt, bool zero, uint64_t *tl = nullptr) {
    constexpr int K = 4;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    const uint32_t c = lt;
    // the zero rows y = -2, -1 of every z slice: 16 x 32 dwords
    if (zero) *(u32x2v *)(s + WK_ZS * (lt >> 4) + 2u * (lt & 15u)) = u32x2v{0u, 0u};
#if GM_WK_PAIRS
    // two rounds of 2 blocks' loads (fewer registers, more workgroups per CU)
    char *const b = (char *)s;
    const uint32_t base = wk_chunk(c);
#pragma unroll
    for (int k = 0; k < K; k += 2) {
        u32x4v v[2][NMAX];
        p4_issue<HIGH>(table, hp[k], valid[k], c, v[0]);
        p4_issue<HIGH>(table, hp[k + 1], valid[k + 1], c, v[1]);
        uint32_t e[2][4], o[2][4];
        p4_fold<NMAX>(v[0], e[0], o[0]);
        p4_fold<NMAX>(v[1], e[1], o[1]);
#else
    u32x4v v[K][NMAX];
#pragma unroll
    for (int k = 0; k < K; k++) p4_issue<HIGH>(table, hp[k], valid[k], c, v[k]);
#ifdef GM_WK_TRACE
    __builtin_amdgcn_s_waitcnt(0);   // diagnostic: every load back before the first fold
    if (tl) *tl = __builtin_amdgcn_s_memrealtime();
#endif
    char *const b = (char *)s;
    const uint32_t base = wk_chunk(c);
#pragma unroll
    for (int k = 0; k < K; k += 2) {
        uint32_t e[2][4], o[2][4];
        p4_fold<NMAX>(v[k], e[0], o[0]);
        p4_fold<NMAX>(v[k + 1], e[1], o[1]);
#endif
#pragma unroll
        for (int j = 0; j < 4; j++) {   // bytes k, k+1 of positions 4j .. 4j+3 (see p4_write_pair)
            const uint32_t xe = __builtin_amdgcn_perm(e[1][j], e[0][j], 0x06020400u);
            const uint32_t xo = __builtin_amdgcn_perm(o[1][j], o[0][j], 0x07030501u);
            const uint32_t a = 4u * (base + 4u * j) + 2u * (uint32_t)(k >> 1);
            *(uint16_t *)(b + a) = (uint16_t)xe;
            *(uint16_t *)(b + a + 4) = (uint16_t)xo;
            *(uint16_t *)(b + a + 8) = (uint16_t)(xe >> 16);
            *(uint16_t *)(b + a + 12) = (uint16_t)(xo >> 16);
        }
    }
}

// pass B: one wave (lane 0..63) walks image s in place (folds in, codes out)
__device__ __forceinline__ void wk_walk(uint32_t *s, uint32_t lane) {
    const uint32_t z = lane & 15, yb = lane >> 4;
    const int s0 = (int)(z + 4u * yb);
    const uint32_t lbase = 16u * (4u * yb + 2u) + WK_ZS * z;   // image dword of (0, 4 yb, z)
    uint32_t re[8], ro[8];   // this lane's codes of the last 8 steps (split halves), ring by step
#pragma unroll
    for (int j = 0; j < 8; j++) re[j] = ro[j] = 0;
#if defined(GM_EXP) && (GM_EXP & 1)
    constexpr int TAU_END = 0;   // experiment: no pass B
#elif defined(GM_EXP) && (GM_EXP & 8)
    constexpr int TAU_END = 48;  // experiment: half the walk (results invalid; timing only)
#else
    constexpr int TAU_END = 91;  // p = tau - s0 in [0, 64), s0 <= 15 + 12
#endif
    // Only (y-1) -- the code this wave stored one step ago -- is on the step-to-step
    // chain; the fold F and (y-2) of the next step are read a step ahead.
    // Addresses: p = t0 + j - s0 with t0 a multiple of 8, so (p >> 2, p & 3) =
    // (t0 / 4 + ((j - s0) >> 2), (j - s0) & 3) and the image dword is
    // lbase + t0 / 4 + cj[j]: one add per step.  An idle lane (p outside [0, 64))
    // reads some dword of the image (unused), writes a dword of its own in the
    // slice's spare tail, and records 0.
    int cj[9];
#pragma unroll
    for (int j = 0; j < 9; j++) cj[j] = ((j - s0) >> 2) + 16 * ((j - s0) & 3);
    const uint32_t dummy = WK_ZS * z + 288u + yb;
    uint32_t Fv, Y2v;
    {
        const uint32_t o = lbase + cj[0];
        Fv = s[o];
        Y2v = s[o - 32];
    }
    auto step = [&](int t0, auto J, auto MASK) {
        constexpr int j = decltype(J)::value;
        constexpr bool masked = decltype(MASK)::value;
        // one base per position (its (y-2) dword): (y-1) and the position itself are at
        // +16 and +32 dwords, immediate offsets of the same LDS address
        const uint32_t b0 = lbase - 32u + (uint32_t)(t0 >> 2);
        const uint32_t o2 = b0 + cj[j], o = o2 + 32u;
        const uint32_t Y1 = s[o2 + 16];   // stored one step ago (this lane or the row below)
        const uint32_t on2 = b0 + cj[j + 1];   // cj[8] = cj[0] + 2: the next t0's first step
        const uint32_t Fn = s[on2 + 32], Y2n = s[on2];
        const uint32_t n1e = dpp_shr1(re[(j + 7) & 7]), n1o = dpp_shr1(ro[(j + 7) & 7]);
        const uint32_t n2e = dpp_shr2(re[(j + 6) & 7]), n2o = dpp_shr2(ro[(j + 6) & 7]);
        // all-ones on an active lane; opaque, so the compiler keeps this straight-line
        // (a branch would sink the (y-1) read behind the prefetch)
        uint32_t act = ~0u;
        if constexpr (masked) {
            act = (uint32_t)(t0 + j - s0) < 64u ? ~0u : 0u;
            asm volatile("" : "+v"(act));
        }
        const uint32_t pe = pk_max(pk_max(Fv & 0x00FF00FFu, Y2v & 0x00FF00FFu),
                                   pk_max(pk_max(n2e, re[(j + 4) & 7]), re[j]));
        const uint32_t po = pk_max(pk_max(Fv, Y2v), pk_max(pk_max(n2o, ro[(j + 4) & 7]), ro[j]));
        const uint32_t me = pk_max(pk_max(pe, n1e), Y1 & 0x00FF00FFu);
        const uint32_t mo = pk_max(pk_max(po, n1o), Y1);
        if constexpr (masked) {
            re[j] = wk_code_e(me) & act;
            ro[j] = wk_code_o(mo) & act;
            s[dummy + ((o - dummy) & act)] = re[j] | ro[j];
        } else {
            re[j] = wk_code_e(me);
            ro[j] = wk_code_o(mo);
            s[o] = re[j] | ro[j];
        }
        Fv = Fn;
        Y2v = Y2n;
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;
    using I6 = std::integral_constant<int, 6>;
    using I7 = std::integral_constant<int, 7>;
    // 88 steps in blocks of 8 (the ring's period), then the last three (tau 88..90);
    // in tau 32..63 every lane has a position (s0 <= 27, p < 64): no masking there
    using M1 = std::true_type;
    using M0 = std::false_type;
    constexpr int MAIN = TAU_END >= 88 ? 88 : TAU_END;
    for (int t0 = 0; t0 < MAIN; t0 += 8) {
        if (GM_WK_UNMASK && t0 >= 32 && t0 < 64) {
            step(t0, I0{}, M0{}); step(t0, I1{}, M0{}); step(t0, I2{}, M0{}); step(t0, I3{}, M0{});
            step(t0, I4{}, M0{}); step(t0, I5{}, M0{}); step(t0, I6{}, M0{}); step(t0, I7{}, M0{});
        } else {
            step(t0, I0{}, M1{}); step(t0, I1{}, M1{}); step(t0, I2{}, M1{}); step(t0, I3{}, M1{});
            step(t0, I4{}, M1{}); step(t0, I5{}, M1{}); step(t0, I6{}, M1{}); step(t0, I7{}, M1{});
        }
    }
    if constexpr (TAU_END > 88) {
        step(88, I0{}, M1{}); step(88, I1{}, M1{}); step(88, I2{}, M1{});
    }
}

// pass C: one wave writes the four blocks from image s (chunks lane + 64 i), and in the
// sharded solve (XD) each block also to its extra destinations
template <int CPOL, bool XD, int NW = 1>
__device__ __forceinline__ void wk_store(uint8_t *__restrict__ table, const uint32_t (&hp)[4], const bool (&valid)[4],
                                         const uint32_t *s, uint32_t lane, const uint32_t *__restrict__ xoff,
                                         const uint64_t *__restrict__ xdst, uint32_t idx0) {
    constexpr int NPOS = 4096, K = 4;
    __amdgpu_buffer_rsrc_t wr[K];
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0);
#if defined(GM_EXP) && (GM_EXP & 4)
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table, 0);   // experiment: stores dropped (out of range)
#endif
#pragma unroll
    for (int i = 0; i < 4 / NW; i++) {   // lane = 0 .. 64 NW - 1 over the NW storing waves
        const uint32_t c = lane + 64u * NW * i;
        const uint32_t base = wk_chunk(c);
        u32x4v out[K];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32x4v q = *(const u32x4v *)(s + base + 4 * j);
            const uint32_t t01 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
            const uint32_t t23 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
            const uint32_t u01 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
            const uint32_t u23 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
            out[0][j] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
            out[1][j] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
            out[2][j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
            out[3][j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
        }
#pragma unroll
        for (int k = 0; k < K; k++) __builtin_amdgcn_raw_buffer_store_b128(out[k], wr[k], 16u * c, 0, CPOL);
        if constexpr (XD) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!valid[k]) continue;
                const uint32_t m1 = xoff[idx0 + k + 1];
                for (uint32_t m = xoff[idx0 + k]; m < m1; m++)
                    __builtin_amdgcn_raw_buffer_store_b128(out[k], block_rsrc((uint8_t *)xdst[m], NPOS), 16u * c, 0, 0);
            }
        }
    }
}

__device__ __forceinline__ void wk_group(const uint32_t *__restrict__ blocks, uint32_t nblk, uint32_t g, uint32_t (&hp)[4],
                                         bool (&valid)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t idx = g * 4 + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? blocks[idx] : 0u;
    }
}

// option 10: one group per workgroup of 256 threads
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wk_solve(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks, uint32_t nblk,
                                         uint32_t *s, const uint32_t *__restrict__ xoff = nullptr,
                                         const uint64_t *__restrict__ xdst = nullptr) {
#if GM_WK_SERP
    uint32_t t0 = 0;   // the tier's parity from its first block's high-nibble sum
    {
        const uint32_t h = blocks[0];
#pragma unroll
        for (int j = 0; j < 8; j++) t0 += (h >> (4 * j)) & 15u;
    }
    const uint32_t grp = (t0 & 1u) ? xcd_order_rev(blockIdx.x, (nblk + 3) / 4) : xcd_order(blockIdx.x, (nblk + 3) / 4);
#else
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + 3) / 4);
#endif
    uint32_t hp[4];
    bool valid[4];
    wk_group(blocks, nblk, grp, hp, valid);
    const uint32_t tid = threadIdx.x;
#ifdef GM_WK_TRACE
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    uint64_t trl = 0;
    wk_load<HIGH>(table, hp, valid, s, tid, true, &trl);
    const uint64_t trf = __builtin_amdgcn_s_memrealtime();
#else
    wk_load<HIGH>(table, hp, valid, s, tid, true);
#endif
    __syncthreads();
#if GM_WK_ROT
    if ((tid >> 6) != (blockIdx.x & 3u)) return;   // one wave walks and stores
#else
    if (tid >= 64) return;
#endif
    const uint32_t lane = tid & 63;
#ifdef GM_WK_TRACE
    const uint64_t tr1 = __builtin_amdgcn_s_memrealtime();
#endif
    wk_walk(s, lane);
#ifdef GM_WK_TRACE
    const uint64_t tr2 = __builtin_amdgcn_s_memrealtime();
#endif
    wk_store<CPOL, XD>(table, hp, valid, s, lane, xoff, xdst, grp * 4);
#ifdef GM_WK_TRACE
    if (lane == 0) wk_trace(tr0, tr1, tr2, hp[0], trl, trf);
#endif
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                          uint32_t nblk, const uint8_t *__restrict__ zero) {
    __shared__ __attribute__((aligned(16))) uint32_t s[WK_IMG];   // 18.25 KiB
    wk_solve<HIGH, GM_B4_STORE_CPOL, false>(table, blocks, nblk, s);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wkx(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                           uint32_t nblk, const uint8_t *__restrict__ zero,
                                                           const uint32_t *__restrict__ xoff,
                                                           const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t s[WK_IMG];
    wk_solve<HIGH, 0, true>(table, blocks, nblk, s, xoff, xdst);
}

// pass B by TWO waves (option 14): wave h walks the rows y = 8h .. 8h + 7, lane (z, yb) the
// rows y = 8h + 2 yb + {0, 1} of column z in the order p = 2x + (y - 8h - 2 yb), starting
// z + 2 yb + 16 h steps late: 69 steps instead of 91.  Every dependency is as in wk_walk
// ((x-1 | x-2) now 2 / 4 steps back in the ring), except rows y = 8, 9 of wave 1, whose
// (y-1 | y-2) wave 0 made 9-10 steps earlier: both waves pass a barrier every 8 steps, so
// those LDS writes are visible.  An idle lane writes out of the LDS allocation (dropped).
__device__ __forceinline__ void wk_walk2(uint32_t *s, uint32_t lane, uint32_t h) {
    const uint32_t z = lane & 15, yb = lane >> 4;
    const int s0 = (int)(z + 2u * yb + 16u * h);
    const uint32_t lbase = 16u * (8u * h + 2u * yb + 2u) + WK_ZS * z;   // image dword of (0, 8h + 2yb, z)
    uint32_t re[8], ro[8];
#pragma unroll
    for (int j = 0; j < 8; j++) re[j] = ro[j] = 0;
    int cj[9];
#pragma unroll
    for (int j = 0; j < 9; j++) cj[j] = ((j - s0) >> 1) + 16 * ((j - s0) & 1);
    constexpr uint32_t DUMMY = 0x3FFFFFC0u;   // an idle lane's write: beyond the allocation, dropped
    uint32_t Fv, Y2v;
    {
        const uint32_t o2 = lbase - 32u + cj[0];
        Fv = s[o2 + 32];
        Y2v = s[o2];
    }
    auto step = [&](int t0, auto J) {
        constexpr int j = decltype(J)::value;
        const uint32_t b0 = lbase - 32u + (uint32_t)(t0 >> 1);
        const uint32_t o2 = b0 + cj[j], o = o2 + 32u;
        const uint32_t Y1 = s[o2 + 16];
        const uint32_t on2 = b0 + cj[j + 1];   // cj[8] = cj[0] + 4
        const uint32_t Fn = s[on2 + 32], Y2n = s[on2];
        const uint32_t n1e = dpp_shr1(re[(j + 7) & 7]), n1o = dpp_shr1(ro[(j + 7) & 7]);
        const uint32_t n2e = dpp_shr2(re[(j + 6) & 7]), n2o = dpp_shr2(ro[(j + 6) & 7]);
        uint32_t act = (uint32_t)(t0 + j - s0) < 32u ? ~0u : 0u;
        asm volatile("" : "+v"(act));
        const uint32_t pe = pk_max(pk_max(Fv & 0x00FF00FFu, Y2v & 0x00FF00FFu),
                                   pk_max(pk_max(n2e, re[(j + 6) & 7]), re[(j + 4) & 7]));
        const uint32_t po = pk_max(pk_max(Fv, Y2v), pk_max(pk_max(n2o, ro[(j + 6) & 7]), ro[(j + 4) & 7]));
        const uint32_t me = pk_max(pk_max(pe, n1e), Y1 & 0x00FF00FFu);
        const uint32_t mo = pk_max(pk_max(po, n1o), Y1);
        re[j] = wk_code_e(me) & act;
        ro[j] = wk_code_o(mo) & act;
        s[DUMMY + ((o - DUMMY) & act)] = re[j] | ro[j];
        Fv = Fn;
        Y2v = Y2n;
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    using I5 = std::integral_constant<int, 5>;
    using I6 = std::integral_constant<int, 6>;
    using I7 = std::integral_constant<int, 7>;
    // steps 0 .. 71 (69 needed: the last three are idle for both waves), a barrier
    // after every 8 (the other wave's (y-1 | y-2) writes of >= 9 steps ago are visible)
    for (int t0 = 0; t0 < 72; t0 += 8) {
        step(t0, I0{}); step(t0, I1{}); step(t0, I2{}); step(t0, I3{});
        step(t0, I4{}); step(t0, I5{}); step(t0, I6{}); step(t0, I7{});
        __syncthreads();
    }
}

// option 14: pass A by 256 threads, pass B by two waves, pass C by each wave for its half
// of the rows (chunks with y in its range)
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wk2w_solve(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                           uint32_t nblk, uint32_t *s, const uint32_t *__restrict__ xoff = nullptr,
                                           const uint64_t *__restrict__ xdst = nullptr) {
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + 3) / 4);
    uint32_t hp[4];
    bool valid[4];
    wk_group(blocks, nblk, grp, hp, valid);
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    wk_load<HIGH>(table, hp, valid, s, tid, true);
    __syncthreads();
    const uint32_t w0 = (blockIdx.x & 1u) * 2u;   // waves (0, 1) or (2, 3): two SIMDs either way
    if (wave != w0 && wave != w0 + 1) return;
    wk_walk2(s, lane, wave - w0);
    __syncthreads();   // both halves walked
    wk_store<CPOL, XD, 2>(table, hp, valid, s, lane + 64u * (wave - w0), xoff, xdst, grp * 4);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2w(uint8_t *__restrict__ table,
                                                            const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                            const uint8_t *__restrict__ zero) {
    __shared__ __attribute__((aligned(16))) uint32_t s[WK_IMG];
    wk2w_solve<HIGH, GM_B4_STORE_CPOL, false>(table, blocks, nblk, s);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2wx(uint8_t *__restrict__ table,
                                                             const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                             const uint8_t *__restrict__ zero,
                                                             const uint32_t *__restrict__ xoff,
                                                             const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t s[WK_IMG];
    wk2w_solve<HIGH, 0, true>(table, blocks, nblk, s, xoff, xdst);
}

// option 15: two groups per workgroup, the second one's loads overlapped with the first's
// walk.  The per-workgroup trace of option 10 showed the walk as the limiter: a CU keeps
// ~2 walkers busy (the rest of its slots are loading), each walk 10 us.  Here pass A of
// group A runs on all four waves; then the walking wave walks and writes A while the
// other three load and fold group B into the second image (192 loader threads: chunks
// 0-191 in one round, 192-255 by the first loader wave in a second); then the walker
// walks and writes B.  The walker is busy for ~2/3 of the workgroup's life instead of
// ~1/2.
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wk2p_solve(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                           uint32_t nblk, uint32_t *img, const uint32_t *__restrict__ xoff = nullptr,
                                           const uint64_t *__restrict__ xdst = nullptr) {
    const uint32_t ng = (nblk + 3) / 4;
    const uint32_t pair = xcd_order(blockIdx.x, (ng + 1) / 2);
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const bool two = 2 * pair + 1 < ng;   // uniform
    uint32_t hp[4];
    bool valid[4];
    wk_group(blocks, nblk, 2 * pair, hp, valid);
    *(u32x2v *)(img + WK_IMG + WK_ZS * (tid >> 4) + 2u * (tid & 15u)) = u32x2v{0u, 0u};   // image 1's zero rows
    wk_load<HIGH>(table, hp, valid, img, tid, true);
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
#if GM_WK_ROT
    const uint32_t w0 = blockIdx.x & 3u;
#else
    const uint32_t w0 = 0;
#endif
    if (wave == w0) {
        wk_walk(img, lane);
        wk_store<CPOL, XD>(table, hp, valid, img, lane, xoff, xdst, 2 * pair * 4);
    } else if (two) {
        const uint32_t li = (wave + 3u - w0) & 3u, lt = li * 64u + lane;   // loader thread 0 .. 191
        wk_group(blocks, nblk, 2 * pair + 1, hp, valid);
        wk_load<HIGH>(table, hp, valid, img + WK_IMG, lt, false);
        __builtin_amdgcn_sched_barrier(0);   // the second round reuses the first's registers
        if (li == 0) wk_load<HIGH>(table, hp, valid, img + WK_IMG, 192u + lt, false);
    }
    __syncthreads();
    if (wave != w0 || !two) return;
    wk_group(blocks, nblk, 2 * pair + 1, hp, valid);
    wk_walk(img + WK_IMG, lane);
    wk_store<CPOL, XD>(table, hp, valid, img + WK_IMG, lane, xoff, xdst, (2 * pair + 1) * 4);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2p(uint8_t *__restrict__ table,
                                                            const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                            const uint8_t *__restrict__ zero) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];   // 36.5 KiB
    wk2p_solve<HIGH, GM_B4_STORE_CPOL, false>(table, blocks, nblk, img);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2px(uint8_t *__restrict__ table,
                                                             const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                             const uint8_t *__restrict__ zero,
                                                             const uint32_t *__restrict__ xoff,
                                                             const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];
    wk2p_solve<HIGH, 0, true>(table, blocks, nblk, img, xoff, xdst);
}

// option 12: two groups per workgroup of 256 threads, two images.  Pass A loads and
// folds them one after the other (the same registers), then two waves walk them at
// once, one group each.  Per group a CU's wave slots are held for ~13 us instead of
// ~21 us (option 10: the three waves that leave after pass A keep their slots until
// the walker is done).
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wk2_solve(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks, uint32_t nblk,
                                          uint32_t *img, const uint32_t *__restrict__ xoff = nullptr,
                                          const uint64_t *__restrict__ xdst = nullptr) {
    const uint32_t ng = (nblk + 3) / 4;
    const uint32_t pair = xcd_order(blockIdx.x, (ng + 1) / 2);
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    uint32_t hp[4];
    bool valid[4];
    const bool two = 2 * pair + 1 < ng;   // uniform
    wk_group(blocks, nblk, 2 * pair, hp, valid);
    wk_load<HIGH>(table, hp, valid, img, tid, true);
    __builtin_amdgcn_sched_barrier(0);   // the second group's loads reuse the first's registers
    if (two) {
        wk_group(blocks, nblk, 2 * pair + 1, hp, valid);
        wk_load<HIGH>(table, hp, valid, img + WK_IMG, tid, true);
    }
    __syncthreads();
#if GM_WK_ROT
    const uint32_t w0 = (blockIdx.x & 1u) * 2u;   // waves (0, 1) or (2, 3): two different SIMDs either way
#else
    const uint32_t w0 = 0;
#endif
    if (wave != w0 && !(two && wave == w0 + 1)) return;
    const uint32_t g = 2 * pair + (wave - w0);
    uint32_t *s = img + (wave - w0) * WK_IMG;
    wk_group(blocks, nblk, g, hp, valid);
    wk_walk(s, lane);
    wk_store<CPOL, XD>(table, hp, valid, s, lane, xoff, xdst, g * 4);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                           uint32_t nblk, const uint8_t *__restrict__ zero) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];   // 36.5 KiB
    wk2_solve<HIGH, GM_B4_STORE_CPOL, false>(table, blocks, nblk, img);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_WK_WAVES) void sub_tier_kernel_wk2x(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                            uint32_t nblk, const uint8_t *__restrict__ zero,
                                                            const uint32_t *__restrict__ xoff,
                                                            const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];
    wk2_solve<HIGH, 0, true>(table, blocks, nblk, img, xoff, xdst);
}

// option 11: persistent, 320 threads, two images.  XCD x (= blockIdx & 7 under the
// round-robin dispatch) owns the contiguous run of the tier's groups that xcd_order
// gives it; its workgroups take the run's groups in turn (i0, i0 + nx, ...).
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wkp_run(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks, uint32_t nblk,
                                        uint32_t *img, const uint32_t *__restrict__ xoff = nullptr,
                                        const uint64_t *__restrict__ xdst = nullptr) {
    const uint32_t ng = (nblk + 3) / 4, G = gridDim.x, x = blockIdx.x & 7u, i0 = blockIdx.x >> 3;
    const uint32_t q = ng >> 3, r = ng & 7u;
    const uint32_t start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = q + (x < r ? 1u : 0u);
    const uint32_t nx = (G + 7u - x) >> 3;   // workgroups on XCD x
    if (i0 >= len) return;   // the whole workgroup
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#if GM_WK_ROT
    const uint32_t walker = (blockIdx.x >> 3) % 5u;   // spread the walkers of a CU's workgroups over its SIMDs
#else
    const uint32_t walker = 0;
#endif
    const uint32_t end = start + len;
    uint32_t hp[4];
    bool valid[4];
    // the two roles run separate loops with the same barrier count (one per group)
    if (wave == walker) {
        __syncthreads();
        for (uint32_t g = start + i0, it = 0;; g += nx, it++) {
            uint32_t *cur = img + (it & 1u) * WK_IMG;
            wk_group(blocks, nblk, g, hp, valid);
            wk_walk(cur, lane);
            wk_store<CPOL, XD>(table, hp, valid, cur, lane, xoff, xdst, g * 4);
            __syncthreads();
            if (g + nx >= end) break;
        }
    } else {
        const uint32_t lt = ((wave + 4u - walker) % 5u) * 64u + lane;   // loader thread 0..255
        wk_group(blocks, nblk, start + i0, hp, valid);
        wk_load<HIGH>(table, hp, valid, img, lt, true);
        *(u32x2v *)(img + WK_IMG + WK_ZS * (lt >> 4) + 2u * (lt & 15u)) = u32x2v{0u, 0u};   // image 1's zero rows
        __syncthreads();
        for (uint32_t g = start + i0, it = 0;; g += nx, it++) {
            const uint32_t gn = g + nx;
            if (gn < end) {
                wk_group(blocks, nblk, gn, hp, valid);
                wk_load<HIGH>(table, hp, valid, img + ((it + 1u) & 1u) * WK_IMG, lt, false);
            }
            __syncthreads();
            if (gn >= end) break;
        }
    }
}

template <int HIGH>
__global__ __launch_bounds__(320, GM_WK_WAVES) void sub_tier_kernel_wkp(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                           uint32_t nblk, const uint8_t *__restrict__ zero) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];   // 36.5 KiB
    wkp_run<HIGH, GM_B4_STORE_CPOL, false>(table, blocks, nblk, img);
}

template <int HIGH>
__global__ __launch_bounds__(320, GM_WK_WAVES) void sub_tier_kernel_wkpx(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks,
                                                            uint32_t nblk, const uint8_t *__restrict__ zero,
                                                            const uint32_t *__restrict__ xoff,
                                                            const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t img[2 * WK_IMG];
    wkp_run<HIGH, 0, true>(table, blocks, nblk, img, xoff, xdst);
}

// grid of the persistent walker kernel: at most GM_WKP_PER_CU workgroups per CU
static uint32_t wkp_grid(uint32_t nblocks) {
    static int cus = 0;
    if (!cus) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    }
    static const int per = getenv("GM_WKP_PER_CU") ? atoi(getenv("GM_WKP_PER_CU")) : GM_WKP_PER_CU;   // dev aid
    const uint32_t ng = (nblocks + 3) / 4, cap = (uint32_t)(per * cus);
    return ng < cap ? ng : cap;
}

// ---------------------------------------------------------------------------
// Pipelined persistent variant (GM_OPT_SUB_INTERLEAVE 9).  Measured on the b4
// kernel: its loads and stores alone (pass B skipped) take 4.0 ms of the 5.1 ms
// solve, and while a workgroup walks pass B's barrier chain it has no load in
// flight.  Here a workgroup keeps two byte images (32 KiB) and works through a
// run of 4-block groups: while pass B walks group g's 46 low tiers in image
// g & 1, the child blocks of group g+1 are loaded and folded into the other image
// -- one block's 2*HIGH loads issued every 11 pass-B steps and folded 11 steps
// later -- so the memory pipe stays busy during the chain.  The grid is 4
// workgroups per CU (118 VGPRs; 5 would fit the LDS); XCD x works through a contiguous run of
// the tier's groups (the runs of xcd_order), its workgroups striding by their
// count, so at any time an XCD covers a window of neighbouring groups.
#ifndef GM_P4_WAVES
#define GM_P4_WAVES 4   // waves per SIMD = workgroups of 4 waves per CU (5 fit the LDS but spill at 96 VGPRs)
#endif
constexpr int P4_PER_CU = GM_P4_WAVES;
constexpr uint32_t B4_LAT_MAX_BLOCKS = 0xFFFFFFFFu;   // every tier (measured: faster at all sizes)
#ifndef GM_B4_LAT_BARRIER
#define GM_B4_LAT_BARRIER 0
#endif

template <int HIGH>
__global__ __launch_bounds__(256, GM_P4_WAVES) void sub_tier_kernel_p4(uint8_t *__restrict__ table,
                                                         const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                         const uint8_t *__restrict__ zero) {
    constexpr int K = 4, NPOS = 4096;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    __shared__ __attribute__((aligned(16))) uint32_t img[2][4096];   // 2 x 16 KiB
    const int tid = threadIdx.x;
    const uint32_t c = tid;   // pass A / C chunk: positions 16c .. 16c+15
    const uint32_t ng = (nblk + K - 1) / K;
    uint32_t g, stride, gend;
    if (ng <= gridDim.x) {   // one group per workgroup
        g = xcd_order(blockIdx.x, ng);
        stride = 1;
        gend = g + 1;
    } else {                 // gridDim.x = 8 W: XCD x's W workgroups stride through its run
        const uint32_t x = blockIdx.x & 7u, i = blockIdx.x >> 3, W = gridDim.x >> 3;
        const uint32_t q = ng >> 3, r = ng & 7u;
        const uint32_t start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = x < r ? q + 1 : q;
        g = start + i;
        stride = W;
        gend = start + len;
    }
    if (g >= gend) return;
    auto group = [&](uint32_t grp, uint32_t (&hp)[K], bool (&valid)[K]) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const uint32_t idx = grp * K + k;
            valid[k] = idx < nblk;
            hp[k] = valid[k] ? blocks[idx] : 0u;
        }
    };
    uint32_t hp[K];
    bool valid[K];
    group(g, hp, valid);

    // pass A of the first group, on its own
#pragma unroll
    for (int k = 0; k < K; k += 2) {
        uint32_t e[2][4], o[2][4];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            u32x4v v[NMAX];
            p4_issue<HIGH>(table, hp[k + h], valid[k + h], c, v);
            p4_fold<NMAX>(v, e[h], o[h]);
            __builtin_amdgcn_sched_barrier(0);
        }
        p4_write_pair(img[0], c, k >> 1, e, o);
    }
    __syncthreads();

    const int a0 = tid & 15, a1 = tid >> 4, s0 = a0 + a1;
    const uint32_t d11 = a1 >= 1 ? 16u : 0u, d12 = a1 >= 2 ? 32u : 0u;
    int cur = 0;
    for (;;) {
        const uint32_t gn = g + stride;
        const bool more = gn < gend;
        uint32_t hq[K];
        bool vq[K];
        group(more ? gn : g, hq, vq);
        if (!more)
#pragma unroll
            for (int k = 0; k < K; k++) vq[k] = false;
        uint32_t *s = img[cur];

        // ---- pass B on image cur (split registers, as GM_PASSB_REG 2), with pass A
        //      of group gn into image cur ^ 1 between its steps
        uint32_t pe1 = 0, po1 = 0, pe2 = 0, po2 = 0;
        if (tid == 0) {
            const uint32_t v = s[0];
            uint32_t re = code_lo2(v & 0x00FF00FFu), ro = code_hi2(v & 0xFF00FF00u);
            if (valid[0] && hp[0] == 0) re = (re & 0xFFFFFF00u) | 255u;   // all heaps empty: LOSS in 0
            s[0] = re | ro;
            pe1 = re;
            po1 = ro;
        }
        __syncthreads();
        auto step = [&](int tau) {
            const uint32_t n1e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe1, 0x111, 0xF, 0xF, true);
            const uint32_t n1o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po1, 0x111, 0xF, 0xF, true);
            const uint32_t n2e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe2, 0x112, 0xF, 0xF, true);
            const uint32_t n2o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po2, 0x112, 0xF, 0xF, true);
            const int cc = tau - s0;
            uint32_t re = 0, ro = 0;
            if (cc >= 0 && cc <= 15) {
                const uint32_t o = (uint32_t)(tid + 256 * cc);
                const uint32_t v0 = s[o], v3 = s[o - d11], v4 = s[o - d12];
                const uint32_t me = pk_max(pk_max(pk_max(v0 & 0x00FF00FFu, v3 & 0x00FF00FFu),
                                                  pk_max(v4 & 0x00FF00FFu, n1e)),
                                           pk_max(pk_max(n2e, pe1), pe2));
                const uint32_t mo = pk_max(pk_max(pk_max(v0, v3), pk_max(v4, n1o)), pk_max(pk_max(n2o, po1), po2));
                re = code_lo2(me);
                ro = code_hi2(mo & 0xFF00FF00u);
                s[o] = re | ro;
            }
            pe2 = pe1;
            po2 = po1;
            pe1 = re;
            po1 = ro;
            __syncthreads();
        };
        // block k's fold is held until block k ^ 1's is done, then the pair goes to
        // the other image as u16 halves (bytes k & 2, (k & 2) + 1 of each dword)
        uint32_t e[2][4], o[2][4];
#pragma unroll
        for (int k = 0; k < K; k++) {
            u32x4v v[NMAX];
            if (more) p4_issue<HIGH>(table, hq[k], vq[k], c, v);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
            for (int t = 1; t <= 11; t++) step(11 * k + t);   // kept rolled: unrolled, the compiler hoists
                                                              // every step's addresses out of the group loop
            __builtin_amdgcn_sched_barrier(0);
            if (more) {
                p4_fold<NMAX>(v, e[k & 1], o[k & 1]);
                if (k & 1) p4_write_pair(img[cur ^ 1], c, k >> 1, e, o);
            }
        }
        step(45);

        // ---- pass C of group g
        __amdgpu_buffer_rsrc_t wr[K];
#pragma unroll
        for (int k = 0; k < K; k++) wr[k] = block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0);
        {
            u32x4v out[K];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const u32x4v q = *(const u32x4v *)(s + 16 * c + 4 * j);
                const uint32_t t01 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
                const uint32_t t23 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
                const uint32_t u01 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
                const uint32_t u23 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
                out[0][j] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
                out[1][j] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
                out[2][j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
                out[3][j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
            }
#pragma unroll
            for (int k = 0; k < K; k++) __builtin_amdgcn_raw_buffer_store_b128(out[k], wr[k], 16u * c, 0, GM_B4_STORE_CPOL);
        }
        if (!more) break;
        __syncthreads();   // image cur is read by pass C above and written by the next pass A
        cur ^= 1;
        g = gn;
#pragma unroll
        for (int k = 0; k < K; k++) { hp[k] = hq[k]; valid[k] = vq[k]; }
    }
}

// ---------------------------------------------------------------------------
// One-wave variant (GM_OPT_SUB_INTERLEAVE 8): a 64-lane workgroup solves four
// blocks in the byte image of the b4 kernel (16 KiB of LDS) with NO workgroup
// barrier.  Measured on the b4 kernel (tools/gpu_call_ablation.sh): its pass B
// alone took 3.2 ms of the 5.4 ms solve, a chain of 46 barrier-separated steps
// in which the four waves wait for the slowest; pass A + C alone took 4.2 ms.
// Here one wave owns the whole 4-block group:
//   * pass A: lane l folds chunks l, l+64, l+128, l+192 (16 positions each) of
//     the four blocks' <= 2*HIGH child blocks -- one buffer descriptor over the
//     whole table, each child a scalar offset;
//   * pass B: the 16 x 16 (a0, a1) columns are four "slots" of four 16-lane DPP
//     rows (a1 = 4j .. 4j+3); at low tier tau slot j works iff tau in
//     [4j, 4j+33], every slot's children are from tiers tau-1 and tau-2, so the
//     slots of one step are independent and the step needs no barrier: LDS ops
//     of one wave execute in order (a wavefront-scope fence keeps the compiler
//     from reordering them across steps);
//   * codes stay split while they live in registers: E = bytes 0 and 2 (blocks
//     0, 2) in the low byte of each u16 half, O = bytes 1 and 3 in the high
//     byte, so a bytewise max is one v_pk_max_u16 per half-set and the packed
//     code for LDS is E | O.  An inactive lane records 0, so a column's
//     (c-1, c-2) children and the DPP neighbours need no validity select.
// 10 workgroups per CU (LDS-bound), each independent.
#ifndef GM_W1_WAVES
#define GM_W1_WAVES 3
#endif
#ifndef GM_W1_STORE_CPOL
#define GM_W1_STORE_CPOL 0
#endif
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int HIGH, bool XD>
__device__ __forceinline__ void w1_solve(uint8_t *__restrict__ table, const uint32_t (&hp)[4], const bool (&valid)[4],
                                         uint32_t *s, const uint32_t *__restrict__ xoff,
                                         const uint64_t *__restrict__ xdst, uint32_t idx0) {
    constexpr int NPOS = 4096, K = 4;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    const uint32_t lane = threadIdx.x;

    // ---- pass A
    {
        // whole-table descriptor (offsets < 2^32; the last table byte is never a
        // child), and a zero-size one for a block without high children (reads 0)
        const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(table, 0, 0xFFFFFFFFu, 0x00020000);
        const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc(table, 0, 0, 0x00020000);
        uint32_t soff[K][NMAX];
        bool has[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            uint32_t first = 0;
            bool any = false;
#pragma unroll
            for (int j = HIGH - 1; j >= 0; j--)
                if (valid[k] && ((hp[k] >> (4 * j)) & 15u) >= 1) { first = (hp[k] - (1u << (4 * j))) << 12; any = true; }
#pragma unroll
            for (int j = 0; j < HIGH; j++) {
                const uint32_t h = (hp[k] >> (4 * j)) & 15u;
                soff[k][2 * j] = (valid[k] && h >= 1) ? (hp[k] - (1u << (4 * j))) << 12 : first;
                soff[k][2 * j + 1] = (valid[k] && h >= 2) ? (hp[k] - (2u << (4 * j))) << 12 : first;
            }
            if constexpr (HIGH == 0) soff[k][0] = 0;
            has[k] = any;
        }
        // 16 rounds (chunk i, block k) of NMAX loads; round n+1's loads are issued
        // before round n is folded, so two rounds are in flight per lane
        u32x4v vb[2][NMAX];
        auto issue = [&](int n, u32x4v (&v)[NMAX]) {
            const int i = n >> 2, k = n & 3;
            const __amdgpu_buffer_rsrc_t r = has[k] ? rt : rz;
#pragma unroll
            for (int m = 0; m < NMAX; m++)
                v[m] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, 16u * (lane + 64u * i),
                                                                                         soff[k][m], 0));
        };
        issue(0, vb[0]);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t c = lane + 64u * i;   // chunk: positions 16c .. 16c+15
            uint32_t e[K][4], o[K][4];
#pragma unroll
            for (int k = 0; k < K; k++) {
                const int n = 4 * i + k;
                if (n + 1 < 16) issue(n + 1, vb[(n + 1) & 1]);
                const u32x4v(&v)[NMAX] = vb[n & 1];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    uint32_t ev = v[0][j] & 0x00FF00FFu, ov = v[0][j];   // ov: odd bytes valid in the high byte
#pragma unroll
                    for (int m = 1; m < NMAX; m++) {
                        ev = pk_max(ev, v[m][j] & 0x00FF00FFu);
                        ov = pk_max(ov, v[m][j]);
                    }
                    e[k][j] = ev;
                    o[k][j] = ov;
                }
            }
#pragma unroll
            for (int j = 0; j < 4; j++) {   // positions 4j .. 4j+3 -> one dword each (bytes = blocks 0..3)
                const uint32_t xe = __builtin_amdgcn_perm(e[1][j], e[0][j], 0x06020400u);
                const uint32_t ye = __builtin_amdgcn_perm(e[3][j], e[2][j], 0x06020400u);
                const uint32_t xo = __builtin_amdgcn_perm(o[1][j], o[0][j], 0x07030501u);
                const uint32_t yo = __builtin_amdgcn_perm(o[3][j], o[2][j], 0x07030501u);
                u32x4v q;
                q[0] = __builtin_amdgcn_perm(ye, xe, 0x05040100u);   // 4j
                q[1] = __builtin_amdgcn_perm(yo, xo, 0x05040100u);   // 4j+1
                q[2] = __builtin_amdgcn_perm(ye, xe, 0x07060302u);   // 4j+2
                q[3] = __builtin_amdgcn_perm(yo, xo, 0x07060302u);   // 4j+3
                *(u32x4v *)(s + 16 * c + 4 * j) = q;
            }
        }
    }
    wave_fence();

    // ---- pass B: lane = a0 + 16 r; slot j holds a1 = 4j + r
    const int a0 = (int)(lane & 15u), r0 = (int)(lane >> 4);
#if defined(GM_EXP) && (GM_EXP & 1)
    constexpr int TAU_END = 0;
#else
    constexpr int TAU_END = 45;
#endif
    uint32_t pe1[4] = {0, 0, 0, 0}, po1[4] = {0, 0, 0, 0}, pe2[4] = {0, 0, 0, 0}, po2[4] = {0, 0, 0, 0};
    if (lane == 0) {   // position 0 (tau 0) of slot 0
        const uint32_t v = s[0];
        uint32_t re = code_lo2(v & 0x00FF00FFu), ro = code_hi2(v & 0xFF00FF00u);
        if (valid[0] && hp[0] == 0) re = (re & 0xFFFFFF00u) | 255u;   // all heaps empty: LOSS in 0
        s[0] = re | ro;
        pe1[0] = re;
        po1[0] = ro;
    }
    wave_fence();
    for (int tau = 1; tau <= TAU_END; tau++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (tau < 4 * j || tau > 4 * j + 33) continue;   // wave-uniform: no column of the slot is on this tier
            const int a1 = 4 * j + r0, cc = tau - a0 - a1;
            // (a0-1 | a0-2, a1, c): lanes -1 / -2 of the row one / two steps ago (0 past the row start)
            const uint32_t n1e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe1[j], 0x111, 0xF, 0xF, true);
            const uint32_t n1o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po1[j], 0x111, 0xF, 0xF, true);
            const uint32_t n2e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe2[j], 0x112, 0xF, 0xF, true);
            const uint32_t n2o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po2[j], 0x112, 0xF, 0xF, true);
            uint32_t re = 0, ro = 0;
            if (cc >= 0 && cc <= 15) {
                const uint32_t o = lane + 64u * (uint32_t)j + 256u * (uint32_t)cc;   // = a0 + 16 a1 + 256 c
                const uint32_t d1 = a1 >= 1 ? 16u : 0u, d2 = a1 >= 2 ? 32u : 0u;
                const uint32_t v0 = s[o], v3 = s[o - d1], v4 = s[o - d2];
                const uint32_t me = pk_max(pk_max(pk_max(v0 & 0x00FF00FFu, v3 & 0x00FF00FFu),
                                                  pk_max(v4 & 0x00FF00FFu, n1e)),
                                           pk_max(pk_max(n2e, pe1[j]), pe2[j]));
                const uint32_t mo = pk_max(pk_max(pk_max(v0, v3), pk_max(v4, n1o)), pk_max(pk_max(n2o, po1[j]), po2[j]));
                re = code_lo2(me);
                ro = code_hi2(mo & 0xFF00FF00u);
                s[o] = re | ro;
            }
            pe2[j] = pe1[j];
            po2[j] = po1[j];
            pe1[j] = re;
            po1[j] = ro;
        }
        wave_fence();
    }

    // ---- pass C
    __amdgpu_buffer_rsrc_t wr[K];
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0);
#if defined(GM_EXP) && (GM_EXP & 4)
#pragma unroll
    for (int k = 0; k < K; k++) wr[k] = block_rsrc(table, 0);   // experiment: stores dropped (out of range)
#endif
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t c = lane + 64u * i;
        u32x4v out[K];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const u32x4v q = *(const u32x4v *)(s + 16 * c + 4 * j);
            const uint32_t t01 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
            const uint32_t t23 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
            const uint32_t u01 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
            const uint32_t u23 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
            out[0][j] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
            out[1][j] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
            out[2][j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
            out[3][j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
        }
#pragma unroll
        for (int k = 0; k < K; k++)
            __builtin_amdgcn_raw_buffer_store_b128(out[k], wr[k], 16u * c, 0, GM_W1_STORE_CPOL);
        if constexpr (XD) {
#pragma unroll
            for (int k = 0; k < K; k++) {
                if (!valid[k]) continue;
                const uint32_t m1 = xoff[idx0 + k + 1];
                for (uint32_t m = xoff[idx0 + k]; m < m1; m++)
                    __builtin_amdgcn_raw_buffer_store_b128(out[k], block_rsrc((uint8_t *)xdst[m], NPOS), 16u * c, 0, 0);
            }
        }
    }
}

template <int HIGH>
__global__ __launch_bounds__(64, GM_W1_WAVES) void sub_tier_kernel_w1(uint8_t *__restrict__ table,
                                                        const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                        const uint8_t *__restrict__ zero) {
    constexpr int K = 4;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + K - 1) / K);
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = grp * K + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? __builtin_amdgcn_readfirstlane(blocks[idx]) : 0u;
    }
    w1_solve<HIGH, false>(table, hp, valid, s, nullptr, nullptr, 0);
}

template <int HIGH>
__global__ __launch_bounds__(64, GM_W1_WAVES) void sub_tier_kernel_w1x(uint8_t *__restrict__ table,
                                                         const uint32_t *__restrict__ blocks, uint32_t nblk,
                                                         const uint8_t *__restrict__ zero,
                                                         const uint32_t *__restrict__ xoff,
                                                         const uint64_t *__restrict__ xdst) {
    constexpr int K = 4;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + K - 1) / K);
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t idx = grp * K + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? __builtin_amdgcn_readfirstlane(blocks[idx]) : 0u;
    }
    w1_solve<HIGH, true>(table, hp, valid, s, xoff, xdst, grp * K);
}

// ---------------------------------------------------------------------------
// Dataflow variant: the whole solve in ONE launch (GM_OPT_SUB_INTERLEAVE 7).
// The tiered launches pay a fill/drain of ~12-16 us each (76 per solve): a tier's
// last workgroups run on an almost idle chip.  Here every block still waits for
// exactly its <= 10 child blocks, not for a whole tier:
//   * items = groups of 4 blocks of one tier, in tier order, split into one list
//     per XCD (the same contiguous Morton runs the tiered launch gives each XCD);
//     a workgroup reads its XCD id and dequeues from that list with one atomic,
//     then from the other lists once its own is empty;
//   * before pass A one lane per child block polls the child's flag (sc1 loads);
//     after pass C every wave drains its sc1 stores (s_waitcnt vmcnt(0)), the
//     workgroup joins a barrier and lane k sets flag[hp[k]] (sc1 store).
// No deadlock: lists are dequeued in tier order and a block only waits on lower
// tiers, so along any chain of waits the tiers strictly decrease; a workgroup
// waits only after it has dequeued, i.e. while running.  Waits are bounded in
// time (GM_FLOW_WAIT_TICKS of the 100 MHz clock): a timeout raises `abort`,
// every later wait is skipped, and the solve reports an error instead of hanging.
constexpr uint64_t GM_FLOW_WAIT_TICKS = 5000000;   // 50 ms
struct FlowItem {
    uint32_t off;   // first block in the tier-sorted block list
    uint32_t n;     // blocks in the group (1..4)
};

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7u;
}

#ifndef GM_FLOW_LAT
#define GM_FLOW_LAT 0   // 1: the latency form of pass A (measured 7.5 ms against 5.4)
#endif
#ifndef GM_FLOW_WAVES
#define GM_FLOW_WAVES 1
#endif
#ifndef GM_FLOW_LOAD_CPOL
#define GM_FLOW_LOAD_CPOL CPOL_SC1
#endif
template <int HIGH>
__global__ __launch_bounds__(256, GM_FLOW_WAVES) void sub_flow_kernel_b4(uint8_t *__restrict__ table,
                                                          const uint32_t *__restrict__ blocks,
                                                          const FlowItem *__restrict__ items,
                                                          const uint32_t *__restrict__ list_off,
                                                          uint32_t *heads, uint32_t *flags, uint32_t *abort_flag,
                                                          const uint8_t *__restrict__ zero) {
    constexpr int K = 4;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    __shared__ int item_sh;
    const int tid = threadIdx.x;
    const uint32_t home = xcc_id();
    int list = (int)home, tries = 0;
    for (;;) {
        if (tid == 0) {
            int got = -1;
            while (tries < 8) {
                const uint32_t len = list_off[list + 1] - list_off[list];
                const uint32_t i = atomicAdd(&heads[list], 1u);
                if (i < len) { got = (int)(list_off[list] + i); break; }
                list = (list + 1) & 7;
                tries++;
            }
            item_sh = got;
        }
        __syncthreads();
        const int it = item_sh;
        if (it < 0) break;
        const FlowItem item = items[it];
        uint32_t hp[K];
        bool valid[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            valid[k] = (uint32_t)k < item.n;
            hp[k] = valid[k] ? blocks[item.off + k] : 0u;
        }
        // wait for the child blocks: lane 10k + m of wave 0 polls child m of block k
        if (tid < 64) {
            const int k = tid / 10, m = tid % 10, j = m >> 1, sub = (m & 1) + 1;
            bool need = false;
            uint32_t child = 0;
            if (k < K && j < HIGH) {
                const uint32_t h = (hp[k] >> (4 * j)) & 15u;
                need = valid[k] && h >= (uint32_t)sub;
                child = hp[k] - ((uint32_t)sub << (4 * j));
            }
            if (need && __hip_atomic_load(&flags[child], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    __builtin_amdgcn_s_sleep(2);
                    if (__hip_atomic_load(&flags[child], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
                    if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > GM_FLOW_WAIT_TICKS) {
                        __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                }
            }
        }
        __syncthreads();
        b4_solve<HIGH, CPOL_SC1, GM_FLOW_LOAD_CPOL, false, GM_FLOW_LAT>(table, zero, hp, valid, s);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid < K && valid[tid]) __hip_atomic_store(&flags[hp[tid]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// Row-granular dataflow (GM_OPT_SUB_INTERLEAVE 13, development option): the whole solve as
// ONE launch of every tier's 4-block groups in tier order, no tier barrier.  Position
// (a0, a1, c) of a block needs (a0, a1, c) of its child blocks, which pass B makes at the
// same step tau = a0 + a1 + c, so the 16-B row (a1, c) of a child -- one of pass A's
// loads -- is final once the child has passed step a1 + c + 15.  Each block publishes
// `progress` (the last step whose completed rows are globally visible): at checkpoints
// every few steps the workgroup stores the rows completed since the previous one
// (write-through `sc1` stores, so pass C disappears), waits for its previous
// checkpoint's stores, and one lane publishes that checkpoint (MI355X_MICROARCH.md
// hand-off row 1: `sc1` payload, every storing wave's vmcnt(0), barrier, `sc1` flag;
// `sc1` loads on the consumer).  A pass-A thread (one row) waits until every child block
// has published the row's step.  Workgroups are launched in tier order, so a waiting
// workgroup only waits on earlier ones (dispatched before it); a wait longer than
// GM_FLOW_WAIT_TICKS raises `abort` and the solve fails loudly.
constexpr uint32_t RF_DONE = 46;   // progress of a finished block
#ifndef GM_RF_CK
#define GM_RF_CK 4   // steps between checkpoints (the last one at step 45)
#endif
#ifndef GM_RF_LCPOL
#define GM_RF_LCPOL CPOL_SC1   // child loads: sc1 (L1-bypassing) for the cross-workgroup hand-off
#endif
__device__ __forceinline__ uint32_t rf_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_B4_LAT_WAVES) void sub_rowflow_kernel(uint8_t *__restrict__ table,
                                                                         const uint32_t *__restrict__ blocks,
                                                                         const FlowItem *__restrict__ items,
                                                                         uint32_t *progress, uint32_t *abort_flag) {
    constexpr int K = 4, NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1, NPOS = 4096;
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    __shared__ uint32_t prog_sh[4 * NMAX];
    const FlowItem item = items[blockIdx.x];
    if (item.n == 0) return;   // padding of a tier's workgroup count to a multiple of 8
    const int tid = threadIdx.x;
#ifdef GM_WK_TRACE
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t hp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        valid[k] = (uint32_t)k < item.n;
        hp[k] = valid[k] ? blocks[item.off + k] : 0u;
    }
    // ---- wait for the rows this thread loads: row (y, z) = chunk tid, final at step y + z + 15
    auto child_of = [&](int j, uint32_t &ch) {   // child j = 2 * nibble + (s - 1) of block j / NMAX
        const int k = j / NMAX, m = j % NMAX, nb = m >> 1, sub = (m & 1) + 1;
        if (HIGH == 0 || !valid[k]) return false;
        const uint32_t h = (hp[k] >> (4 * nb)) & 15u;
        if (h < (uint32_t)sub) return false;
        ch = hp[k] - ((uint32_t)sub << (4 * nb));
        return true;
    };
    if (tid < 4 * NMAX) {
        uint32_t ch = 0;
        prog_sh[tid] = child_of(tid, ch) ? rf_load(progress + ch) : RF_DONE;
    }
    __syncthreads();
    {
        const uint32_t need = (uint32_t)(tid & 15) + (uint32_t)(tid >> 4) + 15u;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
        for (int j = 0; j < 4 * NMAX; j++) {
            if (prog_sh[j] >= need) continue;
            uint32_t ch = 0;
            child_of(j, ch);
            while (rf_load(progress + ch) < need) {
                __builtin_amdgcn_s_sleep(2);
                if (rf_load(abort_flag) != 0u) return;
                if (__builtin_amdgcn_s_memrealtime() - t0 > GM_FLOW_WAIT_TICKS) {
                    __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    return;
                }
            }
        }
    }
#ifdef GM_WK_TRACE
    __syncthreads();
    const uint64_t trw = __builtin_amdgcn_s_memrealtime();   // every row's children ready
#endif
    // ---- pass A: every child load in flight at once (L1-bypassing sc1 loads: hand-off bytes)
    {
        const uint32_t c = tid;
        u32x4v v[K][NMAX];
#pragma unroll
        for (int k = 0; k < K; k++) p4_issue<HIGH, GM_RF_LCPOL>(table, hp[k], valid[k], c, v[k]);
        uint32_t e[2][4], o[2][4];
#pragma unroll
        for (int k = 0; k < K; k += 2) {
            p4_fold<NMAX>(v[k], e[0], o[0]);
            p4_fold<NMAX>(v[k + 1], e[1], o[1]);
            p4_write_pair(s, c, k >> 1, e, o);
        }
    }
    // a thread that returned above (abort) leaves the barrier count short only when the
    // whole solve is abandoned anyway; every thread of a live workgroup arrives here
    __syncthreads();

#ifdef GM_WK_TRACE
    const uint64_t tra = __builtin_amdgcn_s_memrealtime();
#endif
    // ---- pass B as in b4_solve (split-register form), with row stores at checkpoints
    const uint32_t row_done = (uint32_t)(tid & 15) + (uint32_t)(tid >> 4) + 15u;   // chunk tid's final step
    uint32_t last_ck = 0;
    auto checkpoint = [&](uint32_t tau) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's rows of the previous checkpoint
        __syncthreads();
        if (last_ck && tid < K && valid[tid])
            __hip_atomic_store(progress + hp[tid], last_ck, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (row_done > last_ck && row_done <= tau) {   // store row tid of the four blocks
            u32x4v out[K];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const u32x4v q = *(const u32x4v *)(s + 16 * tid + 4 * j);
                const uint32_t t01 = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
                const uint32_t t23 = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
                const uint32_t u01 = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
                const uint32_t u23 = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
                out[0][j] = __builtin_amdgcn_perm(t23, t01, 0x05040100u);
                out[1][j] = __builtin_amdgcn_perm(t23, t01, 0x07060302u);
                out[2][j] = __builtin_amdgcn_perm(u23, u01, 0x05040100u);
                out[3][j] = __builtin_amdgcn_perm(u23, u01, 0x07060302u);
            }
#pragma unroll
            for (int k = 0; k < K; k++)
                __builtin_amdgcn_raw_buffer_store_b128(out[k], block_rsrc(table + ((uint64_t)hp[k] << 12), valid[k] ? NPOS : 0),
                                                       16u * tid, 0, CPOL_SC1);
        }
        last_ck = tau;
    };
    const int a0 = tid & 15, a1 = tid >> 4, s0 = a0 + a1;
    uint32_t pe1 = 0, po1 = 0, pe2 = 0, po2 = 0;
    const uint32_t d11 = a1 >= 1 ? 16u : 0u, d12 = a1 >= 2 ? 32u : 0u;
    if (tid == 0) {
        const uint32_t v = s[0];
        uint32_t re = code_lo2(v & 0x00FF00FFu), ro = code_hi2(v & 0xFF00FF00u);
        if (valid[0] && hp[0] == 0) re = (re & 0xFFFFFF00u) | 255u;   // all heaps empty: LOSS in 0
        s[0] = re | ro;
        pe1 = re;
        po1 = ro;
    }
    __syncthreads();
    for (int tau = 1; tau <= 45; tau++) {
        const uint32_t n1e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe1, 0x111, 0xF, 0xF, true);
        const uint32_t n1o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po1, 0x111, 0xF, 0xF, true);
        const uint32_t n2e = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pe2, 0x112, 0xF, 0xF, true);
        const uint32_t n2o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)po2, 0x112, 0xF, 0xF, true);
        const int c = tau - s0;
        uint32_t re = 0, ro = 0;
        if (c >= 0 && c <= 15) {
            const uint32_t o = (uint32_t)(tid + 256 * c);
            const uint32_t v0 = s[o], v3 = s[o - d11], v4 = s[o - d12];
            const uint32_t me = pk_max(pk_max(pk_max(v0 & 0x00FF00FFu, v3 & 0x00FF00FFu), pk_max(v4 & 0x00FF00FFu, n1e)),
                                       pk_max(pk_max(n2e, pe1), pe2));
            const uint32_t mo = pk_max(pk_max(pk_max(v0, v3), pk_max(v4, n1o)), pk_max(pk_max(n2o, po1), po2));
            re = code_lo2(me);
            ro = code_hi2(mo & 0xFF00FF00u);
            s[o] = re | ro;
        }
        pe2 = pe1;
        po2 = po1;
        pe1 = re;
        po1 = ro;
        __syncthreads();
        if (tau >= 45 - GM_RF_CK * ((45 - 15) / GM_RF_CK) && (45 - tau) % GM_RF_CK == 0) checkpoint((uint32_t)tau);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < K && valid[tid]) __hip_atomic_store(progress + hp[tid], RF_DONE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef GM_WK_TRACE
    if (tid == 0) wk_trace(tr0, tra, trw, hp[0], trw, tra);
#endif
}

typedef void (*rowflow_kernel_t)(uint8_t *, const uint32_t *, const FlowItem *, uint32_t *, uint32_t *);
static rowflow_kernel_t pick_rowflow(int high) {
    switch (high) {
    case 0: return sub_rowflow_kernel<0>;
    case 1: return sub_rowflow_kernel<1>;
    case 2: return sub_rowflow_kernel<2>;
    case 3: return sub_rowflow_kernel<3>;
    case 4: return sub_rowflow_kernel<4>;
    case 5: return sub_rowflow_kernel<5>;
    }
    return nullptr;
}

typedef void (*tier_kernel_t)(uint8_t *, const uint32_t *, uint32_t, const uint8_t *);
typedef void (*flow_kernel_t)(uint8_t *, const uint32_t *, const FlowItem *, const uint32_t *, uint32_t *, uint32_t *,
                              uint32_t *, const uint8_t *);

static flow_kernel_t pick_flow(int high) {
    switch (high) {
    case 0: return sub_flow_kernel_b4<0>;
    case 1: return sub_flow_kernel_b4<1>;
    case 2: return sub_flow_kernel_b4<2>;
    case 3: return sub_flow_kernel_b4<3>;
    case 4: return sub_flow_kernel_b4<4>;
    case 5: return sub_flow_kernel_b4<5>;
    }
    return nullptr;
}

template <bool LAT>
static tier_kernel_t pick_b4(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_b4<0, LAT>;
    case 1: return sub_tier_kernel_b4<1, LAT>;
    case 2: return sub_tier_kernel_b4<2, LAT>;
    case 3: return sub_tier_kernel_b4<3, LAT>;
    case 4: return sub_tier_kernel_b4<4, LAT>;
    case 5: return sub_tier_kernel_b4<5, LAT>;
    }
    return nullptr;
}
static tier_kernel_t pick_b4(int high) { return pick_b4<false>(high); }

// Tiers of at most this many blocks (GM_B4_LAT overrides, development aid) run the
// latency variant of the b4 kernel: every child load issued up front.
static uint32_t b4_lat_max() {
    static const uint32_t v = getenv("GM_B4_LAT") ? (uint32_t)atoi(getenv("GM_B4_LAT")) : B4_LAT_MAX_BLOCKS;
    return v;
}

// Tiers of fewer blocks than this run the b4 kernel instead of the walker: a lone
// workgroup's walk (91 dependent steps, ~8 us) is longer than b4's 46-step barrier
// chain, so below a few rounds of workgroups per CU the b4 kernel's latency wins
// (GM_WK_MIN overrides, development aid).
#ifndef GM_WK_MIN_BLOCKS
#define GM_WK_MIN_BLOCKS 4096
#endif
static uint32_t wk_min_blocks() {
    static const uint32_t v = getenv("GM_WK_MIN") ? (uint32_t)atoi(getenv("GM_WK_MIN")) : GM_WK_MIN_BLOCKS;
    return v;
}

// development aid: GM_PAD_LDS=<bytes> of unused dynamic LDS per workgroup (fewer workgroups per CU)
static unsigned pad_lds() {
    static const unsigned v = getenv("GM_PAD_LDS") ? (unsigned)atoi(getenv("GM_PAD_LDS")) : 0u;
    return v;
}

static tier_kernel_t pick_w1(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_w1<0>;
    case 1: return sub_tier_kernel_w1<1>;
    case 2: return sub_tier_kernel_w1<2>;
    case 3: return sub_tier_kernel_w1<3>;
    case 4: return sub_tier_kernel_w1<4>;
    case 5: return sub_tier_kernel_w1<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_wkp(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_wkp<0>;
    case 1: return sub_tier_kernel_wkp<1>;
    case 2: return sub_tier_kernel_wkp<2>;
    case 3: return sub_tier_kernel_wkp<3>;
    case 4: return sub_tier_kernel_wkp<4>;
    case 5: return sub_tier_kernel_wkp<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_wk2w(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_wk2w<0>;
    case 1: return sub_tier_kernel_wk2w<1>;
    case 2: return sub_tier_kernel_wk2w<2>;
    case 3: return sub_tier_kernel_wk2w<3>;
    case 4: return sub_tier_kernel_wk2w<4>;
    case 5: return sub_tier_kernel_wk2w<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_wk2p(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_wk2p<0>;
    case 1: return sub_tier_kernel_wk2p<1>;
    case 2: return sub_tier_kernel_wk2p<2>;
    case 3: return sub_tier_kernel_wk2p<3>;
    case 4: return sub_tier_kernel_wk2p<4>;
    case 5: return sub_tier_kernel_wk2p<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_wk2(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_wk2<0>;
    case 1: return sub_tier_kernel_wk2<1>;
    case 2: return sub_tier_kernel_wk2<2>;
    case 3: return sub_tier_kernel_wk2<3>;
    case 4: return sub_tier_kernel_wk2<4>;
    case 5: return sub_tier_kernel_wk2<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_wk(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_wk<0>;
    case 1: return sub_tier_kernel_wk<1>;
    case 2: return sub_tier_kernel_wk<2>;
    case 3: return sub_tier_kernel_wk<3>;
    case 4: return sub_tier_kernel_wk<4>;
    case 5: return sub_tier_kernel_wk<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_p4(int high) {
    switch (high) {
    case 0: return sub_tier_kernel_p4<0>;
    case 1: return sub_tier_kernel_p4<1>;
    case 2: return sub_tier_kernel_p4<2>;
    case 3: return sub_tier_kernel_p4<3>;
    case 4: return sub_tier_kernel_p4<4>;
    case 5: return sub_tier_kernel_p4<5>;
    }
    return nullptr;
}

static tier_kernel_t pick_x4(int high, bool diag) {
    switch (high) {
    case 0: return diag ? sub_tier_kernel_x4<0, true> : sub_tier_kernel_x4<0, false>;
    case 1: return diag ? sub_tier_kernel_x4<1, true> : sub_tier_kernel_x4<1, false>;
    case 2: return diag ? sub_tier_kernel_x4<2, true> : sub_tier_kernel_x4<2, false>;
    case 3: return diag ? sub_tier_kernel_x4<3, true> : sub_tier_kernel_x4<3, false>;
    case 4: return diag ? sub_tier_kernel_x4<4, true> : sub_tier_kernel_x4<4, false>;
    case 5: return diag ? sub_tier_kernel_x4<5, true> : sub_tier_kernel_x4<5, false>;
    }
    return nullptr;
}

template <int LOW, int NT>
static tier_kernel_t pick_high(int high) {
    switch (high) {
    case 0: return sub_tier_kernel<LOW, 0, NT>;
    case 1: return sub_tier_kernel<LOW, 1, NT>;
    case 2: return sub_tier_kernel<LOW, 2, NT>;
    case 3: return sub_tier_kernel<LOW, 3, NT>;
    case 4: return sub_tier_kernel<LOW, 4, NT>;
    case 5: return sub_tier_kernel<LOW, 5, NT>;
    case 6: if constexpr (LOW <= 2) return sub_tier_kernel<LOW, 6, NT>; else return nullptr;
    case 7: if constexpr (LOW <= 1) return sub_tier_kernel<LOW, 7, NT>; else return nullptr;
    }
    return nullptr;
}

template <int NT>
static tier_kernel_t pick_low(int low, int high) {
    switch (low) {
    case 1: return pick_high<1, NT>(high);
    case 2: return pick_high<2, NT>(high);
    case 3: return pick_high<3, NT>(high);
    }
    return nullptr;
}

static tier_kernel_t pick_kernel(int low, int high, int nt) {
    switch (nt) {
    case 64: return pick_low<64>(low, high);
    case 128: return pick_low<128>(low, high);
    case 256: return pick_low<256>(low, high);
    }
    return nullptr;
}

// nt == 0 / -1 / -2 select the 4-block interleaved kernels (LOW = 3, 256 threads):
// u16 image with row-major / anti-diagonal pass B, byte image; nt == -4 the
// one-wave byte-image kernel (64 threads).
static tier_kernel_t pick_interleaved(int high, int nt) {
    if (nt == -4) return pick_w1(high);
    if (nt == -5) return pick_p4(high);
    if (nt == -6) return pick_wk(high);
    if (nt == -7) return pick_wkp(high);
    if (nt == -8) return pick_wk2(high);
    if (nt == -10) return pick_wk2w(high);
    if (nt == -11) return pick_wk2p(high);
    return nt == -2 ? pick_b4(high) : pick_x4(high, nt == -1);
}

bool sub_kernel_exists(int low, int high, int nt) {
    if (nt == -3) return low == 3 && pick_flow(high) != nullptr;
    if (nt == -9) return low == 3 && pick_rowflow(high) != nullptr;
    return nt <= 0 ? (low == 3 && pick_interleaved(high, nt) != nullptr) : pick_kernel(low, high, nt) != nullptr;
}

void launch_sub_tier(int low, int high, int nt, uint32_t nblocks, uint8_t *table, const uint32_t *list,
                     const uint8_t *zero, hipStream_t s) {
    if (!nblocks) return;
    if (nt == -5) {   // persistent: at most P4_PER_CU workgroups per CU (a multiple of 8)
        static int cus = 0;
        if (!cus) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
        }
        const uint32_t ng = (nblocks + 3) / 4, cap = (uint32_t)(P4_PER_CU * cus) & ~7u;
        hipLaunchKernelGGL(pick_p4(high), dim3(ng <= cap ? ng : cap), dim3(256), 0, s, table, list, nblocks, zero);
    } else if (nt == -2 && nblocks <= b4_lat_max()) {
        hipLaunchKernelGGL(pick_b4<true>(high), dim3((nblocks + 3) / 4), dim3(256), pad_lds(), s, table, list, nblocks,
                           zero);
    } else if (nt == -11 && nblocks >= wk_min_blocks()) {
        hipLaunchKernelGGL(pick_wk2p(high), dim3(((nblocks + 3) / 4 + 1) / 2), dim3(256), 0, s, table, list, nblocks,
                           zero);
    } else if (nt == -10 && nblocks >= wk_min_blocks()) {
        hipLaunchKernelGGL(pick_wk2w(high), dim3((nblocks + 3) / 4), dim3(256), 0, s, table, list, nblocks, zero);
    } else if ((nt == -6 || nt == -10 || nt == -11) && nblocks < wk_min_blocks()) {   // small tier: one workgroup's latency decides
        hipLaunchKernelGGL(pick_b4<true>(high), dim3((nblocks + 3) / 4), dim3(256), 0, s, table, list, nblocks, zero);
    } else if (nt == -6) {
        hipLaunchKernelGGL(pick_wk(high), dim3((nblocks + 3) / 4), dim3(256), pad_lds(), s, table, list, nblocks, zero);
    } else if (nt == -8) {
        hipLaunchKernelGGL(pick_wk2(high), dim3(((nblocks + 3) / 4 + 1) / 2), dim3(256), pad_lds(), s, table, list,
                           nblocks, zero);
    } else if (nt == -7) {
        hipLaunchKernelGGL(pick_wkp(high), dim3(wkp_grid(nblocks)), dim3(320), pad_lds(), s, table, list, nblocks, zero);
    } else if (nt <= 0)
        hipLaunchKernelGGL(pick_interleaved(high, nt), dim3((nblocks + 3) / 4), dim3(nt == -4 ? 64 : 256), 0, s, table,
                           list, nblocks, zero);
    else
        hipLaunchKernelGGL(pick_kernel(low, high, nt), dim3(nblocks), dim3(nt), 0, s, table, list, nblocks, zero);
}

typedef void (*tier_kernel_x_t)(uint8_t *, const uint32_t *, uint32_t, const uint8_t *, const uint32_t *,
                                const uint64_t *);
template <bool LAT>
static tier_kernel_x_t pick_b4x(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_b4x<1, LAT>;
    case 2: return sub_tier_kernel_b4x<2, LAT>;
    case 3: return sub_tier_kernel_b4x<3, LAT>;
    case 4: return sub_tier_kernel_b4x<4, LAT>;
    case 5: return sub_tier_kernel_b4x<5, LAT>;
    }
    return nullptr;
}
static tier_kernel_x_t pick_b4x(int high) { return pick_b4x<false>(high); }

static tier_kernel_x_t pick_wkpx(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_wkpx<1>;
    case 2: return sub_tier_kernel_wkpx<2>;
    case 3: return sub_tier_kernel_wkpx<3>;
    case 4: return sub_tier_kernel_wkpx<4>;
    case 5: return sub_tier_kernel_wkpx<5>;
    }
    return nullptr;
}

static tier_kernel_x_t pick_wk2wx(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_wk2wx<1>;
    case 2: return sub_tier_kernel_wk2wx<2>;
    case 3: return sub_tier_kernel_wk2wx<3>;
    case 4: return sub_tier_kernel_wk2wx<4>;
    case 5: return sub_tier_kernel_wk2wx<5>;
    }
    return nullptr;
}

static tier_kernel_x_t pick_wk2px(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_wk2px<1>;
    case 2: return sub_tier_kernel_wk2px<2>;
    case 3: return sub_tier_kernel_wk2px<3>;
    case 4: return sub_tier_kernel_wk2px<4>;
    case 5: return sub_tier_kernel_wk2px<5>;
    }
    return nullptr;
}

static tier_kernel_x_t pick_wk2x(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_wk2x<1>;
    case 2: return sub_tier_kernel_wk2x<2>;
    case 3: return sub_tier_kernel_wk2x<3>;
    case 4: return sub_tier_kernel_wk2x<4>;
    case 5: return sub_tier_kernel_wk2x<5>;
    }
    return nullptr;
}

static tier_kernel_x_t pick_wkx(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_wkx<1>;
    case 2: return sub_tier_kernel_wkx<2>;
    case 3: return sub_tier_kernel_wkx<3>;
    case 4: return sub_tier_kernel_wkx<4>;
    case 5: return sub_tier_kernel_wkx<5>;
    }
    return nullptr;
}

static tier_kernel_x_t pick_w1x(int high) {
    switch (high) {
    case 1: return sub_tier_kernel_w1x<1>;
    case 2: return sub_tier_kernel_w1x<2>;
    case 3: return sub_tier_kernel_w1x<3>;
    case 4: return sub_tier_kernel_w1x<4>;
    case 5: return sub_tier_kernel_w1x<5>;
    }
    return nullptr;
}

bool sub_kernel_x_exists(int high) {
    return pick_b4x(high) != nullptr && pick_w1x(high) != nullptr && pick_wkx(high) != nullptr &&
           pick_wkpx(high) != nullptr && pick_wk2x(high) != nullptr && pick_wk2wx(high) != nullptr &&
           pick_wk2px(high) != nullptr;
}

// kind: the sub_interleave option (8 one-wave kernel, 10 walker, otherwise the b4 kernel)
void launch_sub_tier_x(int high, uint32_t nblocks, uint8_t *table, const uint32_t *list, const uint8_t *zero,
                       const uint32_t *xoff, const uint64_t *xdst, hipStream_t s, int kind) {
    if (!nblocks) return;
    if (kind == 15 && nblocks >= wk_min_blocks()) {
        hipLaunchKernelGGL(pick_wk2px(high), dim3(((nblocks + 3) / 4 + 1) / 2), dim3(256), 0, s, table, list, nblocks,
                           zero, xoff, xdst);
        return;
    }
    if (kind == 12) {
        hipLaunchKernelGGL(pick_wk2x(high), dim3(((nblocks + 3) / 4 + 1) / 2), dim3(256), 0, s, table, list, nblocks,
                           zero, xoff, xdst);
        return;
    }
    if (kind == 11) {
        hipLaunchKernelGGL(pick_wkpx(high), dim3(wkp_grid(nblocks)), dim3(320), 0, s, table, list, nblocks, zero, xoff,
                           xdst);
        return;
    }
    const bool wave = kind == 8;
    hipLaunchKernelGGL(wave ? pick_w1x(high) : kind == 10 && nblocks >= wk_min_blocks() ? pick_wkx(high)
                       : kind == 14 && nblocks >= wk_min_blocks() ? pick_wk2wx(high)
                       : nblocks <= b4_lat_max() ? pick_b4x<true>(high) : pick_b4x<false>(high),
                       dim3((nblocks + 3) / 4), dim3(wave ? 64 : 256), 0, s,
                       table, list, nblocks, zero, xoff, xdst);
}

int sub_kernel_threads(const Ctx *c, int low) {
    if (low == 3 && c->sub_interleave == 4) return 0;
    if (low == 3 && c->sub_interleave == 5) return -1;
    if (low == 3 && c->sub_interleave == 6) return -2;
    if (low == 3 && c->sub_interleave == 7) return -3;
    if (low == 3 && c->sub_interleave == 8) return -4;
    if (low == 3 && c->sub_interleave == 9) return -5;
    if (low == 3 && c->sub_interleave == 10) return -6;
    if (low == 3 && c->sub_interleave == 11) return -7;
    if (low == 3 && c->sub_interleave == 12) return -8;
    if (low == 3 && c->sub_interleave == 13) return -9;
    if (low == 3 && c->sub_interleave == 14) return -10;
    if (low == 3 && c->sub_interleave == 15) return -11;
    return c->sub_threads;
}

// ---------------------------------------------------------------------------
__global__ void sub_digest_kernel(const uint8_t *__restrict__ table, uint64_t slots, int heaps,
                                  uint64_t root, unsigned long long *acc) {
    uint64_t sum = 0, cnt = 0;
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < slots;
         k += (uint64_t)gridDim.x * blockDim.x) {
        bool in = true;
        for (int j = 0; j < heaps; j++) in &= ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
        if (!in) continue;
        sum += digest_term(k, record_of_code(table[k]));
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

__global__ void sub_query_kernel(const uint8_t *__restrict__ table, uint64_t slots,
                                 const uint64_t *__restrict__ keys, uint16_t *__restrict__ out, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) out[i] = keys[i] < slots ? record_of_code(table[keys[i]]) : REC_UNSOLVED;
}

// ---------------------------------------------------------------------------
// Morton (bit-interleaved) code of a high part's nibbles.  Sorting each tier by it
// keeps the five same-tier parents of a child block (one high nibble +1 each) close
// in the launch order, hence on the same XCD at about the same time: their shared
// child blocks are read from HBM once and then hit that XCD's L2.
static uint32_t morton_of(uint32_t v, int high) {
    uint32_t m = 0;
    for (int b = 0; b < 4; b++)
        for (int j = 0; j < high; j++) m |= ((v >> (4 * j + b)) & 1u) << (b * high + j);
    return m;
}

// Hilbert index (Skilling's transpose form) of the first n = high - 1 nibbles: a
// tier's blocks have high - 1 free coordinates (the last nibble is fixed by the
// sum), and a Hilbert walk of them keeps consecutive blocks adjacent (order 2).
static uint64_t hilbert_of(uint32_t v, int high) {
    const int n = std::max(1, high - 1);
    uint32_t x[8];
    for (int i = 0; i < n; i++) x[i] = (v >> (4 * i)) & 15u;
    for (uint32_t q = 8; q > 1; q >>= 1) {
        const uint32_t p = q - 1;
        for (int i = 0; i < n; i++) {
            if (x[i] & q) x[0] ^= p;
            else { const uint32_t t = (x[0] ^ x[i]) & p; x[0] ^= t; x[i] ^= t; }
        }
    }
    for (int i = 1; i < n; i++) x[i] ^= x[i - 1];
    uint32_t t = 0;
    for (uint32_t q = 8; q > 1; q >>= 1) if (x[n - 1] & q) t ^= q - 1;
    for (int i = 0; i < n; i++) x[i] ^= t;
    uint64_t h = 0;
    for (int b = 3; b >= 0; b--)
        for (int i = 0; i < n; i++) h = (h << 1) | ((x[i] >> b) & 1u);
    return h;
}

// Order 3: the Hilbert order's eight XCD runs (xcd_order) keep their blocks, but
// each run is walked layer by layer in one high nibble (GM_ORDER_LAYER, default 3),
// a 3-D Hilbert walk of the other free nibbles inside a layer, alternate layers
// reversed: a child block's same-tier parents (+1 in one nibble) are then at most
// about one layer apart in the run, inside the window the XCD's L2 still holds,
// where the 4-D walk puts some of them half a run away.
static int order_layer_nibble(int high) {
    const char *s = getenv("GM_ORDER_LAYER");
    const int j = s ? atoi(s) : 3;
    return j >= 0 && j < high ? j : high - 1;
}

// sorts order[b0, b1) by key(v); every key is unique inside a tier (its free nibbles
// name the block), so the keys are computed once and the pairs sorted
template <class K>
static void sort_by_key(std::vector<uint32_t> &order, size_t b0, size_t b1, K key) {
    std::vector<std::pair<uint64_t, uint32_t>> kv(b1 - b0);
    for (size_t i = b0; i < b1; i++) kv[i - b0] = {key(order[i]), order[i]};
    std::sort(kv.begin(), kv.end());
    for (size_t i = b0; i < b1; i++) order[i] = kv[i - b0].second;
}

static void layer_runs(std::vector<uint32_t> &order, uint32_t b0, uint32_t b1, int high) {
    if (high < 3) return;
    const int L = order_layer_nibble(high);
    sort_by_key(order, b0, b1, [&](uint32_t v) {
        uint32_t rest = 0;
        for (int j = 0, k = 0; j < high - 1 && k < 3; j++)
            if (j != L) rest |= ((v >> (4 * j)) & 15u) << (4 * k++);
        const uint32_t layer = (v >> (4 * L)) & 15u;
        const uint64_t h = hilbert_of(rest, std::min(high, 4));
        return ((uint64_t)layer << 32) | (layer & 1u ? ~h & 0xFFFFFFFFull : h);
    });
}

void sort_tiers_morton(std::vector<uint32_t> &order, const std::vector<uint32_t> &off, int high, int mode) {
    for (size_t t = 0; t + 1 < off.size(); t++) {
        if (mode >= 2) sort_by_key(order, off[t], off[t + 1], [high](uint32_t v) { return hilbert_of(v, high); });
        else sort_by_key(order, off[t], off[t + 1], [high](uint32_t v) { return (uint64_t)morton_of(v, high); });
        if (mode == 3) {
            const uint32_t nb = off[t + 1] - off[t], ng = (nb + 3) / 4, q = ng >> 3, r = ng & 7;
            for (uint32_t x = 0; x < 8; x++) {
                const uint32_t g0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = x < r ? q + 1 : q;
                if (len) layer_runs(order, off[t] + 4 * g0, off[t] + std::min(nb, 4 * (g0 + len)), high);
            }
        }
    }
}

static int prepare(Ctx *c, DenseSub *d) {
    int heaps = c->sub.heaps;
    int low = std::min(c->sub_low, heaps);
    if (low < 1) low = 1;
    if (low > 3) low = 3;
    int high = heaps - low;
    int nt = sub_kernel_threads(c, low);
    if (!sub_kernel_exists(low, high, nt)) {
        set_error("no dense kernel for %d heaps at %d low heaps", heaps, low);
        return GM_E_GAME;
    }
    d->heaps = heaps; d->low = low; d->high = high; d->nt = nt;
    d->want_threads = c->sub_threads; d->want_x4 = c->sub_interleave; d->want_order = c->sub_order;
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
    if (c->sub_order >= 1) sort_tiers_morton(order, d->tier_off, high, c->sub_order);
    GM_HIP(hipMalloc(&d->d_blocks, nhigh * sizeof(uint32_t)));
    GM_HIP(hipMemcpy(d->d_blocks, order.data(), nhigh * sizeof(uint32_t), hipMemcpyHostToDevice));
    size_t zbytes = std::max<size_t>(16, (size_t)1 << (4 * low));
    GM_HIP(hipMalloc(&d->zero, zbytes));
    GM_HIP(hipMemset(d->zero, 0, zbytes));
    GM_HIP(hipMalloc(&d->d_acc, 2 * sizeof(uint64_t)));
    if (nt == -9) {
        // one workgroup per group, tiers in order, each tier's workgroups padded to a
        // multiple of 8 so workgroup b runs on XCD b % 8 with the run xcd_order gives it
        std::vector<FlowItem> all;
        for (size_t t = 0; t + 1 < d->tier_off.size(); t++) {
            const uint32_t nb = d->tier_off[t + 1] - d->tier_off[t], ng = (nb + 3) / 4, q = ng >> 3, r = ng & 7;
            const uint32_t ng8 = (ng + 7) & ~7u;
            for (uint32_t b = 0; b < ng8; b++) {
                const uint32_t x = b & 7u, i = b >> 3, len = x < r ? q + 1 : q;
                const uint32_t g = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
                all.push_back(i < len ? FlowItem{d->tier_off[t] + 4 * g, std::min(4u, nb - 4 * g)} : FlowItem{0, 0});
            }
        }
        GM_HIP(hipMalloc(&d->flow_items, all.size() * sizeof(FlowItem)));
        GM_HIP(hipMemcpy(d->flow_items, all.data(), all.size() * sizeof(FlowItem), hipMemcpyHostToDevice));
        GM_HIP(hipMalloc(&d->flow_abort, 4));
        GM_HIP(hipMalloc(&d->flow_flags, nhigh * 4));
        d->flow_grid = (unsigned)all.size();
    }
    if (nt == -3) {
        // per-XCD item lists: each tier's 4-block groups split into the same 8
        // contiguous runs that xcd_order gives the tiered launch
        std::vector<FlowItem> lists[8];
        for (size_t t = 0; t + 1 < d->tier_off.size(); t++) {
            const uint32_t nb = d->tier_off[t + 1] - d->tier_off[t], ng = (nb + 3) / 4, q = ng >> 3, r = ng & 7;
            for (uint32_t x = 0; x < 8; x++) {
                const uint32_t g0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = x < r ? q + 1 : q;
                for (uint32_t g = g0; g < g0 + len; g++)
                    lists[x].push_back(FlowItem{d->tier_off[t] + 4 * g, std::min(4u, nb - 4 * g)});
            }
        }
        std::vector<FlowItem> all;
        std::vector<uint32_t> off(9, 0);
        for (int x = 0; x < 8; x++) {
            off[x] = (uint32_t)all.size();
            all.insert(all.end(), lists[x].begin(), lists[x].end());
        }
        off[8] = (uint32_t)all.size();
        GM_HIP(hipMalloc(&d->flow_items, all.size() * sizeof(FlowItem)));
        GM_HIP(hipMemcpy(d->flow_items, all.data(), all.size() * sizeof(FlowItem), hipMemcpyHostToDevice));
        GM_HIP(hipMalloc(&d->flow_list_off, 9 * 4));
        GM_HIP(hipMemcpy(d->flow_list_off, off.data(), 9 * 4, hipMemcpyHostToDevice));
        GM_HIP(hipMalloc(&d->flow_heads, 8 * 4));
        GM_HIP(hipMalloc(&d->flow_abort, 4));
        GM_HIP(hipMalloc(&d->flow_flags, nhigh * 4));
        int per_cu = 0, dev = 0;
        GM_HIP(hipGetDevice(&dev));
        hipDeviceProp_t prop;
        GM_HIP(hipGetDeviceProperties(&prop, dev));
        GM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(pick_flow(high)),
                                                            256, 0));
        d->flow_grid = (unsigned)std::max(1, per_cu) * (unsigned)prop.multiProcessorCount;
        d->flow_grid = std::min<unsigned>(d->flow_grid, (unsigned)all.size());
    }
    uint64_t bytes = d->slots;
    if (c->adopted_dense) {
        if (c->adopted_dense_bytes < bytes) {
            set_error("adopted dense table holds %llu bytes, need %llu",
                      (unsigned long long)c->adopted_dense_bytes, (unsigned long long)bytes);
            return GM_E_CAP;
        }
        d->table = (uint8_t *)c->adopted_dense;
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
    int ntiers = (int)d->tier_off.size() - 1;
    if (d->nt == -9) {
        const uint64_t nhigh = 1ull << (4 * d->high);
        if (timed) GM_HIP(hipEventRecord(d->ev[0], c->stream));
        GM_HIP(hipMemsetAsync(d->flow_abort, 0, 4, c->stream));
        GM_HIP(hipMemsetAsync(d->flow_flags, 0, nhigh * 4, c->stream));
        hipLaunchKernelGGL(pick_rowflow(d->high), dim3(d->flow_grid), dim3(256), 0, c->stream, d->table, d->d_blocks,
                           (const FlowItem *)d->flow_items, d->flow_flags, d->flow_abort);
        if (timed) GM_HIP(hipEventRecord(d->ev[1], c->stream));
        GM_HIP(hipGetLastError());
        return GM_OK;
    }
    if (d->nt == -3) {
        const uint64_t nhigh = 1ull << (4 * d->high);
        if (timed) GM_HIP(hipEventRecord(d->ev[0], c->stream));
        GM_HIP(hipMemsetAsync(d->flow_heads, 0, 8 * 4, c->stream));
        GM_HIP(hipMemsetAsync(d->flow_abort, 0, 4, c->stream));
        GM_HIP(hipMemsetAsync(d->flow_flags, 0, nhigh * 4, c->stream));
        hipLaunchKernelGGL(pick_flow(d->high), dim3(d->flow_grid), dim3(256), 0, c->stream, d->table, d->d_blocks,
                           (const FlowItem *)d->flow_items, d->flow_list_off, d->flow_heads, d->flow_flags,
                           d->flow_abort, d->zero);
        if (timed) GM_HIP(hipEventRecord(d->ev[1], c->stream));
        GM_HIP(hipGetLastError());
        return GM_OK;
    }
    for (int t = 0; t < ntiers; t++) {
        uint32_t nb = d->tier_off[t + 1] - d->tier_off[t];
        if (!nb) continue;
        if (timed) GM_HIP(hipEventRecord(d->ev[2 * t], c->stream));
        launch_sub_tier(d->low, d->high, d->nt, nb, d->table, d->d_blocks + d->tier_off[t], d->zero, c->stream);
        if (timed) GM_HIP(hipEventRecord(d->ev[2 * t + 1], c->stream));
    }
    GM_HIP(hipGetLastError());
    return GM_OK;
}

int dense_sub_solve(Ctx *c, uint64_t root) {
    DenseSub *d = c->dsub;
    if (!d || d->heaps != c->sub.heaps || d->want_threads != c->sub_threads || d->want_x4 != c->sub_interleave ||
        d->want_order != c->sub_order || d->low != std::min(std::max(c->sub_low, 1), std::min(3, c->sub.heaps)) ||
        (c->adopted_dense && d->table != c->adopted_dense)) {
        dense_sub_free(c);
        d = c->dsub = new DenseSub();
        GM_TRY(prepare(c, d));
    }
#ifdef GM_WK_TRACE
    static uint64_t *tbuf = nullptr;
    static uint32_t *tcnt = nullptr;
    const char *tpath = getenv("GM_TRACE_OUT");
    if (tpath && !tbuf) {
        GM_HIP(hipMalloc(&tbuf, 64ull << 20));
        GM_HIP(hipMalloc(&tcnt, 4));
        GM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(gm_trace_buf), &tbuf, sizeof(tbuf)));
        GM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(gm_trace_cnt), &tcnt, sizeof(tcnt)));
        GM_HIP(hipMemset(tcnt, 0, 4));
        GM_HIP(hipDeviceSynchronize());
    }
#endif
    double t0 = now_ms();
    bool timed = c->timing;
    if (timed) GM_TRY(ensure_events(d));
    if (c->use_graph) {
        // Replay the per-tier launches as one hipGraph; timing brackets the whole
        // replay with one event pair (event nodes captured into a graph do not
        // update host-visible events), so the per-launch time includes the
        // graph's inter-kernel gaps.
        if (!d->graph || d->graph_stream != c->stream) {
            if (d->graph) { (void)hipGraphExecDestroy(d->graph); d->graph = nullptr; }
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
    uint8_t rs;
    uint32_t aborted = 0;
    GM_HIP(hipMemcpyAsync(&rs, d->table + root, 1, hipMemcpyDeviceToHost, c->stream));
    if (d->nt == -3 || d->nt == -9) GM_HIP(hipMemcpyAsync(&aborted, d->flow_abort, 4, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    double t1 = now_ms();
    if (aborted) {
        set_error("dataflow solve: a wait for a child block timed out");
        return GM_E_STATE;
    }

#ifdef GM_WK_TRACE
    if (tpath && tbuf) {   // the entries of this solve, then reset for the next
        uint32_t cnt = 0;
        GM_HIP(hipMemcpy(&cnt, tcnt, 4, hipMemcpyDeviceToHost));
        cnt = std::min(cnt, 1u << 20);
        std::vector<uint64_t> h(8ull * cnt);
        GM_HIP(hipMemcpy(h.data(), tbuf, h.size() * 8, hipMemcpyDeviceToHost));
        if (FILE *f = fopen(tpath, "wb")) { fwrite(h.data(), 8, h.size(), f); fclose(f); }
        GM_HIP(hipMemset(tcnt, 0, 4));
    }
#endif
    c->root_record = record_of_code(rs);
    uint64_t n = 1;
    for (int j = 0; j < d->heaps; j++) n *= ((root >> (4 * j)) & 15u) + 1;
    c->n_positions = n;
    int ntiers = (int)d->tier_off.size() - 1;
    // positions per global tier (heap sum) of the full table
    {
        std::vector<uint64_t> acc(1, 1);
        for (int j = 0; j < d->heaps; j++) {
            std::vector<uint64_t> nx(acc.size() + 15, 0);
            for (size_t s = 0; s < acc.size(); s++)
                for (int h = 0; h < 16; h++) nx[s + h] += acc[s];
            acc.swap(nx);
        }
        c->tier_counts = acc;
    }
    c->stats.n_positions = n;
    c->stats.n_primitive = 1;
    c->stats.n_tiers = ntiers;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.forward_ms = 0;
    // SURVEY §8d edge model with 1-byte records: 1 B written + 1 B per child edge
    c->stats.algo_bytes = (uint64_t)((double)d->slots * (1.0 + 1.8125 * d->heaps));
    c->stats.table_bytes = d->slots;
    if (timed) {
        float total = 0;
        int launches = 0;
        for (int t = 0; t < ntiers && d->nt != -3 && d->nt != -9; t++) {
            if (d->tier_off[t + 1] == d->tier_off[t]) continue;
            launches++;
            if (c->use_graph) continue;
            float ms = 0;
            GM_HIP(hipEventElapsedTime(&ms, d->ev[2 * t], d->ev[2 * t + 1]));
            total += ms;
        }
        if (d->nt == -3 || d->nt == -9) launches = 1;
        if (c->use_graph || d->nt == -3 || d->nt == -9) GM_HIP(hipEventElapsedTime(&total, d->ev[0], d->ev[1]));
        c->stats.kernel_ms = total;
        c->stats.kernel_launches = launches;
    }
    return GM_OK;
}

int dense_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    DenseSub *d = c->dsub;
    *n = c->n_positions;
    if (!keys) return GM_OK;
    if (cap < c->n_positions) {
        set_error("export buffer holds %llu, need %llu", (unsigned long long)cap, (unsigned long long)c->n_positions);
        return GM_E_CAP;
    }
    std::vector<uint8_t> h(d->slots);
    GM_HIP(hipMemcpy(h.data(), d->table, d->slots, hipMemcpyDeviceToHost));
    uint64_t j = 0;
    for (uint64_t k = 0; k < d->slots; k++) {
        bool in = true;
        for (int i = 0; i < d->heaps && in; i++) in = ((k >> (4 * i)) & 15u) <= ((c->root >> (4 * i)) & 15u);
        if (!in) continue;
        keys[j] = k;
        recs[j] = record_of_code(h[k]);
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
    hipLaunchKernelGGL(sub_query_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, d->table,
                       d->slots, dk, dr, n);
    GM_HIP(hipMemcpyAsync(recs, dr, n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

int dense_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    DenseSub *d = c->dsub;
    GM_HIP(hipMemsetAsync(d->d_acc, 0, 16, c->stream));
    hipLaunchKernelGGL(sub_digest_kernel, dim3(2048), dim3(256), 0, c->stream, d->table, d->slots, d->heaps, c->root,
                       (unsigned long long *)d->d_acc);
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
    *bytes = d->slots;
    return GM_OK;
}

void dense_sub_free(Ctx *c) {
    DenseSub *d = c->dsub;
    if (!d) return;
    if (d->graph) (void)hipGraphExecDestroy(d->graph);
    for (auto e : d->ev) (void)hipEventDestroy(e);
    if (d->owned && d->table) (void)hipFree(d->table);
    if (d->zero) (void)hipFree(d->zero);
    if (d->d_blocks) (void)hipFree(d->d_blocks);
    if (d->d_acc) (void)hipFree(d->d_acc);
    for (void *p : {(void *)d->flow_items, (void *)d->flow_list_off, (void *)d->flow_heads, (void *)d->flow_flags,
                    (void *)d->flow_abort})
        if (p) (void)hipFree(p);
    delete d;
    c->dsub = nullptr;
}

}  // namespace gm
