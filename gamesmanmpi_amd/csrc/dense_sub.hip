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
// Kernels (LOW = 3): sub_tier_kernel_wk (the walker, default on tiers of >= 4,096
// blocks) and sub_tier_kernel_b4 (smaller tiers) solve FOUR blocks per workgroup with
// their codes interleaved bytewise in one LDS image, so one LDS access of pass B
// serves four positions; sub_tier_kernel (one block per workgroup, any LOW) serves
// games of fewer than 3 heaps and GM_OPT_SUB_INTERLEAVE 1.  The *_x forms add the
// sharded solve's extra destinations (csrc/dist_sub.hip).
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
    int heaps = 0, low = 0, high = 0, nt = 128;   // nt > 0: one block per workgroup; NT_* below: LOW = 3 kernels
    int want_threads = 0, want_x4 = 0, want_order = 0;
    uint8_t *table = nullptr;           // 16^heaps codes
    bool owned = false;
    uint64_t slots = 0;
    uint8_t *zero = nullptr;            // one block of zeros (padding source)
    uint32_t *d_blocks = nullptr;       // high parts of the root box, sorted by (tier, order)
    uint32_t box = 0;                   // the root's high part: blocks with every nibble <= its
    std::vector<uint32_t> tier_off;     // block offsets per high tier
    uint64_t *d_acc = nullptr;          // digest / counters
    hipGraphExec_t graph = nullptr;
    hipStream_t graph_stream = nullptr;
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
// Four blocks per workgroup (LOW = 3, GM_OPT_SUB_INTERLEAVE 6; the small tiers of the
// default option 10): the four blocks' codes of a position share one dword of LDS
// (byte k = block k), a 16 KiB image, so one address, one validity test and one LDS
// access of pass B serve four positions.
//   pass A  all four blocks' 2*HIGH child loads are issued before the first fold
//           (one memory round trip per workgroup -- measured faster than folding
//           block by block at every tier size), the codes folded as even / odd u16
//           pairs with v_pk_max_u16 and transposed into the byte image;
//   pass B  thread (a0, a1) solves (a0, a1, tau - a0 - a1) at low tier tau, one
//           barrier per tier;
//   pass C  transpose back and write each block with 16-B buffer stores.
// parent codes of split halves: E holds codes in the low byte of each u16, O in the high byte
__device__ __forceinline__ uint32_t code_lo2(uint32_t e) { return (0x00FF00FFu - e) + ((e >> 6) & 0x00020002u); }
__device__ __forceinline__ uint32_t code_hi2(uint32_t o) { return (0xFF00FF00u - o) + ((o >> 6) & 0x02000200u); }

#ifndef GM_B4_WAVES
#define GM_B4_WAVES 1   // min waves per SIMD (1: the compiler's choice, 126 VGPRs)
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
// the 2*HIGH child blocks of block hp, chunk c: one whole-table descriptor, each child a
// scalar offset (a block with no child at all, only high part 0, reads through a
// zero-size descriptor).  Written so that the compiler keeps every load of the four
// blocks in flight before the first fold (126-128 VGPRs); an equivalent form that chose
// the offset per load let it drain after each block's loads (64-89 VGPRs: 4.71 ms per
// 2^32 solve against 4.63-4.66, profiles/r03a_bench_subtract8.log).
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
}

// Cache policy of stores / loads: 0 plain; CPOL_SC1 write-through stores and
// L1-bypassing loads (MI355X_MICROARCH.md, inter-workgroup visibility).
constexpr int CPOL_SC1 = 16;
// One workgroup solves the four blocks hp[0..3] (valid[k] false: slot unused).
// XD (sharded solve): block k also goes to the extra destinations xdst[xoff[idx0 + k] ..
// xoff[idx0 + k + 1]) -- symmetric-fill images in the table and halo ring slots --
// from the same registers, so no separate fill / pack launch follows the tier.
template <int HIGH, int CPOL, bool XD = false>
__device__ __forceinline__ void b4_solve(uint8_t *__restrict__ table, const uint32_t (&hp)[4],
                                         const bool (&valid)[4], uint32_t *s,
                                         const uint32_t *__restrict__ xoff = nullptr,
                                         const uint64_t *__restrict__ xdst = nullptr, uint32_t idx0 = 0) {
    constexpr int NPOS = 4096, NCH = 256, NT = 256, K = 4;
    constexpr int NMAX = 2 * HIGH > 0 ? 2 * HIGH : 1;
    const int tid = threadIdx.x;
    static_assert(NCH == NT, "one chunk per thread");

    // ---- pass A: chunk tid = positions 16 tid .. 16 tid + 15
    {
        const uint32_t c = tid;
        u32x4v v[K][NMAX];
#pragma unroll
        for (int k = 0; k < K; k++) p4_issue<HIGH>(table, hp[k], valid[k], c, v[k]);
        uint32_t e[2][4], o[2][4];
#pragma unroll
        for (int k = 0; k < K; k += 2) {
            p4_fold<NMAX>(v[k], e[0], o[0]);
            p4_fold<NMAX>(v[k + 1], e[1], o[1]);
            p4_write_pair(s, c, k >> 1, e, o);
        }
    }
    __syncthreads();

    // ---- pass B: thread (a0, a1), position c = tau - a0 - a1.  Children inside the
    // block, by where they live: (a0-1 | a0-2, a1, c) are the codes lanes tid-1 / tid-2
    // (same 16-lane DPP row) made one / two steps ago, moved with row_shr (an invalid
    // child arrives as 0, which max ignores); (a0, a1, c-1 | c-2) are this thread's own
    // last two codes; only (a0, a1-1 | a1-2, c), written by other waves, and the
    // child-block fold s[o] come from LDS: 3 LDS reads per step.  Codes stay split while
    // they live in registers: E = bytes 0, 2 in the low byte of each u16 half, O = bytes
    // 1, 3 in the high byte; an inactive lane records 0, so (c-1, c-2) need no select.
    const int a0 = tid & 15, a1 = tid >> 4, s0 = a0 + a1;
    const uint32_t d11 = a1 >= 1 ? 16u : 0u, d12 = a1 >= 2 ? 32u : 0u;
    (void)a0;
#if defined(GM_EXP) && (GM_EXP & 1)
    constexpr int TAU_END = 0;   // experiment: no pass B
#else
    constexpr int TAU_END = 45;
#endif
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

    // ---- pass C: back to four 16-byte rows per chunk
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

__device__ __forceinline__ void group_of(const uint32_t *__restrict__ blocks, uint32_t nblk, uint32_t g,
                                         uint32_t (&hp)[4], bool (&valid)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t idx = g * 4 + k;
        valid[k] = idx < nblk;
        hp[k] = valid[k] ? blocks[idx] : 0u;
    }
}

template <int HIGH>
__global__ __launch_bounds__(256, GM_B4_WAVES) void sub_tier_kernel_b4(uint8_t *__restrict__ table,
                                                                       const uint32_t *__restrict__ blocks,
                                                                       uint32_t nblk, const uint8_t *__restrict__) {
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + 3) / 4);
    uint32_t hp[4];
    bool valid[4];
    group_of(blocks, nblk, grp, hp, valid);
    b4_solve<HIGH, GM_B4_STORE_CPOL>(table, hp, valid, s);
}

// The sharded solve's tier kernel (csrc/dist_sub.hip): as above, plus each block's
// extra destinations (xoff / xdst indexed like `blocks`).
template <int HIGH>
__global__ __launch_bounds__(256, GM_B4_WAVES) void sub_tier_kernel_b4x(uint8_t *__restrict__ table,
                                                                        const uint32_t *__restrict__ blocks,
                                                                        uint32_t nblk, const uint8_t *__restrict__,
                                                                        const uint32_t *__restrict__ xoff,
                                                                        const uint64_t *__restrict__ xdst) {
    __shared__ __attribute__((aligned(16))) uint32_t s[4096];   // 16 KiB
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + 3) / 4);
    uint32_t hp[4];
    bool valid[4];
    group_of(blocks, nblk, grp, hp, valid);
    b4_solve<HIGH, 0, true>(table, hp, valid, s, xoff, xdst, grp * 4);
}

// ---------------------------------------------------------------------------
// Walker form of the 4-block kernel (GM_OPT_SUB_INTERLEAVE 10, the default).
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
// sub_tier_kernel_wk: 256 threads load (pass A), then one wave walks and writes the
// blocks (pass C); the other three leave.  A per-workgroup trace (GM_WK_TRACE build,
// tools/wk_trace.py) showed what that buys: an exited wave's slot is not reused while
// its workgroup lives, so a CU holds 4 such workgroups (128 VGPRs) and at any time ~2
// of them walk while ~2 load -- the walk (9.9 us per group) and the loads (9 us)
// alternate instead of overlapping.  The variants that tried to overlap them
// (persistent double-buffered, two groups per workgroup, two walking waves) were
// bit-exact and slower; DESIGN.md §4.1 keeps their measurements.
#ifndef GM_WK_ROT
#define GM_WK_ROT 1   // the walking wave rotates with the workgroup index (spread over the SIMDs)
#endif
#ifndef GM_WK_UNMASK
#define GM_WK_UNMASK 1   // no activity masking in the walk's all-active middle steps
#endif
#ifndef GM_WK_WAVES
#define GM_WK_WAVES 4   // waves per SIMD the register budget must allow
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

// one group per workgroup of 256 threads
template <int HIGH, int CPOL, bool XD>
__device__ __forceinline__ void wk_solve(uint8_t *__restrict__ table, const uint32_t *__restrict__ blocks, uint32_t nblk,
                                         uint32_t *s, const uint32_t *__restrict__ xoff = nullptr,
                                         const uint64_t *__restrict__ xdst = nullptr) {
    const uint32_t grp = xcd_order(blockIdx.x, (nblk + 3) / 4);
    uint32_t hp[4];
    bool valid[4];
    group_of(blocks, nblk, grp, hp, valid);
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

typedef void (*tier_kernel_t)(uint8_t *, const uint32_t *, uint32_t, const uint8_t *);
typedef void (*tier_kernel_x_t)(uint8_t *, const uint32_t *, uint32_t, const uint8_t *, const uint32_t *,
                                const uint64_t *);

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

#define GM_PICK_HIGH(K, ...)                      \
    switch (high) {                               \
    case 0: return K<0 __VA_ARGS__>;              \
    case 1: return K<1 __VA_ARGS__>;              \
    case 2: return K<2 __VA_ARGS__>;              \
    case 3: return K<3 __VA_ARGS__>;              \
    case 4: return K<4 __VA_ARGS__>;              \
    case 5: return K<5 __VA_ARGS__>;              \
    }                                             \
    return nullptr;

static tier_kernel_t pick_b4(int high) { GM_PICK_HIGH(sub_tier_kernel_b4) }
static tier_kernel_t pick_wk(int high) { GM_PICK_HIGH(sub_tier_kernel_wk) }
static tier_kernel_x_t pick_b4x(int high) { if (high < 1) return nullptr; GM_PICK_HIGH(sub_tier_kernel_b4x) }
static tier_kernel_x_t pick_wkx(int high) { if (high < 1) return nullptr; GM_PICK_HIGH(sub_tier_kernel_wkx) }

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

// nt > 0: one block per workgroup of nt threads (any LOW); LOW = 3 only:
// NT_B4 the four-block kernel on every tier, NT_WALK the walker on tiers of at least
// wk_min_blocks() blocks (b4 below)
enum { NT_B4 = -2, NT_WALK = -6 };

bool sub_kernel_exists(int low, int high, int nt) {
    if (nt == NT_B4 || nt == NT_WALK) return low == 3 && pick_b4(high) != nullptr;
    return nt > 0 && pick_kernel(low, high, nt) != nullptr;
}

void launch_sub_tier(int low, int high, int nt, uint32_t nblocks, uint8_t *table, const uint32_t *list,
                     const uint8_t *zero, hipStream_t s) {
    if (!nblocks) return;
    if (nt == NT_WALK && nblocks >= wk_min_blocks())
        hipLaunchKernelGGL(pick_wk(high), dim3((nblocks + 3) / 4), dim3(256), 0, s, table, list, nblocks, zero);
    else if (nt == NT_B4 || nt == NT_WALK)
        hipLaunchKernelGGL(pick_b4(high), dim3((nblocks + 3) / 4), dim3(256), 0, s, table, list, nblocks, zero);
    else
        hipLaunchKernelGGL(pick_kernel(low, high, nt), dim3(nblocks), dim3(nt), 0, s, table, list, nblocks, zero);
}

bool sub_kernel_x_exists(int high) { return pick_b4x(high) != nullptr && pick_wkx(high) != nullptr; }

// kind: the sub_interleave option (10 walker on the large tiers, otherwise the b4 kernel)
void launch_sub_tier_x(int high, uint32_t nblocks, uint8_t *table, const uint32_t *list, const uint8_t *zero,
                       const uint32_t *xoff, const uint64_t *xdst, hipStream_t s, int kind) {
    if (!nblocks) return;
    hipLaunchKernelGGL((kind == 10 || kind == 20) && nblocks >= wk_min_blocks() ? pick_wkx(high) : pick_b4x(high),
                       dim3((nblocks + 3) / 4), dim3(256), 0, s, table, list, nblocks, zero, xoff, xdst);
}

int sub_kernel_threads(const Ctx *c, int low) {
    if (low == 3 && c->sub_interleave == 6) return NT_B4;
    if (low == 3 && (c->sub_interleave == 10 || c->sub_interleave == 20)) return NT_WALK;   // 20: box engine at 8 heaps
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

// a key outside the root's region (a heap above the root's) answers REC_UNSOLVED: the slot
// may hold an earlier solve's code (include/gmsolve.h gm_query)
__global__ void sub_query_kernel(const uint8_t *__restrict__ table, uint64_t slots, uint64_t root, int heaps,
                                 const uint64_t *__restrict__ keys, uint16_t *__restrict__ out, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    bool in = k < slots;
    for (int j = 0; j < heaps && in; j++) in = ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
    out[i] = in ? record_of_code(table[k]) : REC_UNSOLVED;
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

// sorts order[b0, b1) by key(v); every key is unique inside a tier (its free nibbles
// name the block), so the keys are computed once and the pairs sorted
template <class K>
static void sort_by_key(std::vector<uint32_t> &order, size_t b0, size_t b1, K key) {
    std::vector<std::pair<uint64_t, uint32_t>> kv(b1 - b0);
    for (size_t i = b0; i < b1; i++) kv[i - b0] = {key(order[i]), order[i]};
    std::sort(kv.begin(), kv.end());
    for (size_t i = b0; i < b1; i++) order[i] = kv[i - b0].second;
}

void sort_tiers_morton(std::vector<uint32_t> &order, const std::vector<uint32_t> &off, int high, int mode) {
    for (size_t t = 0; t + 1 < off.size(); t++) {
        if (mode >= 2) sort_by_key(order, off[t], off[t + 1], [high](uint32_t v) { return hilbert_of(v, high); });
        else sort_by_key(order, off[t], off[t + 1], [high](uint32_t v) { return (uint64_t)morton_of(v, high); });
    }
}

// The high part of the root bounds the blocks a solve needs: a move lowers one nibble,
// so every position reachable from the root has each high nibble <= the root's
// (positions of a needed block beyond the root's low nibbles are solved too: they
// are exact, only not counted or exported).
static uint32_t root_box(const DenseSub *d, uint64_t root) { return (uint32_t)(root >> (4 * d->low)); }
static bool in_box(uint32_t v, uint32_t box, int high) {
    for (int j = 0; j < high; j++)
        if (((v >> (4 * j)) & 15u) > ((box >> (4 * j)) & 15u)) return false;
    return true;
}

static int prepare(Ctx *c, DenseSub *d, uint64_t root) {
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
    const uint64_t nhigh = 1ull << (4 * high);
    d->box = root_box(d, root);
    // counting sort of the root box's high parts by nibble sum (tier)
    std::vector<uint32_t> cnt(15 * high + 2, 0), order;
    auto tsum = [&](uint64_t v) { int s = 0; for (int j = 0; j < high; j++) s += (v >> (4 * j)) & 15; return s; };
    for (uint64_t v = 0; v < nhigh; v++)
        if (in_box((uint32_t)v, d->box, high)) cnt[tsum(v) + 1]++;
    for (size_t t = 1; t < cnt.size(); t++) cnt[t] += cnt[t - 1];
    d->tier_off.assign(cnt.begin(), cnt.end());
    order.resize(cnt.back());
    std::vector<uint32_t> pos(cnt.begin(), cnt.end() - 1);
    for (uint64_t v = 0; v < nhigh; v++)
        if (in_box((uint32_t)v, d->box, high)) order[pos[tsum(v)]++] = (uint32_t)v;
    if (c->sub_order >= 1) sort_tiers_morton(order, d->tier_off, high, c->sub_order);
    GM_HIP(hipMalloc(&d->d_blocks, std::max<size_t>(1, order.size()) * sizeof(uint32_t)));
    GM_HIP(hipMemcpy(d->d_blocks, order.data(), order.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    size_t zbytes = std::max<size_t>(16, (size_t)1 << (4 * low));
    GM_HIP(hipMalloc(&d->zero, zbytes));
    GM_HIP(hipMemset(d->zero, 0, zbytes));
    GM_HIP(hipMalloc(&d->d_acc, 2 * sizeof(uint64_t)));
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
    if (c->sub.heaps == 8 && c->sub_interleave == 20) {   // the box engine (dense_box.hip)
        dense_sub_free(c);
        c->dbox_active = true;
        return dense_box_solve(c, root);
    }
    dense_box_free(c);
    dist_box_free(c);
    c->dbox_active = false;
    DenseSub *d = c->dsub;
    if (!d || d->heaps != c->sub.heaps || d->want_threads != c->sub_threads || d->want_x4 != c->sub_interleave ||
        d->want_order != c->sub_order || d->low != std::min(std::max(c->sub_low, 1), std::min(3, c->sub.heaps)) ||
        (c->adopted_dense && d->table != c->adopted_dense) || root_box(d, root) != d->box) {
        dense_sub_free(c);
        d = c->dsub = new DenseSub();
        GM_TRY(prepare(c, d, root));
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
    GM_HIP(hipMemcpyAsync(&rs, d->table + root, 1, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    double t1 = now_ms();

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
        for (int t = 0; t < ntiers; t++) {
            if (d->tier_off[t + 1] == d->tier_off[t]) continue;
            launches++;
            if (c->use_graph) continue;
            float ms = 0;
            GM_HIP(hipEventElapsedTime(&ms, d->ev[2 * t], d->ev[2 * t + 1]));
            total += ms;
        }
        if (c->use_graph) GM_HIP(hipEventElapsedTime(&total, d->ev[0], d->ev[1]));
        c->stats.kernel_ms = total;
        c->stats.kernel_launches = launches;
    }
    return GM_OK;
}

int dense_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    if (c->dbox_active) return dense_box_export(c, keys, recs, cap, n);
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
    if (c->dbox_active) return dense_box_query(c, keys, recs, n);
    DenseSub *d = c->dsub;
    if (!n) return GM_OK;
    uint64_t *dk;
    uint16_t *dr;
    GM_HIP(hipMalloc(&dk, n * 8));
    GM_HIP(hipMalloc(&dr, n * 2));
    GM_HIP(hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(sub_query_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, d->table,
                       d->slots, c->root, c->sub.heaps, dk, dr, n);
    GM_HIP(hipMemcpyAsync(recs, dr, n * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dk);
    (void)hipFree(dr);
    return GM_OK;
}

int dense_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    if (c->dbox_active) return dense_box_digest(c, digest, n);
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
    if (c->dbox_active) return dense_box_table(c, p, bytes);
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
    delete d;
    c->dsub = nullptr;
}

}  // namespace gm