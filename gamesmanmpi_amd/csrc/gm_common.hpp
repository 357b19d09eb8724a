// gm_common.hpp -- shared host/device definitions of libgmsolve.
//
// Records and preference scores
// -----------------------------
// The ABI record (include/gmsolve.h) is (value << 14) | remoteness.  Inside the
// solver every table slot instead holds a *preference score*: a monotone
// re-encoding chosen so that a parent's choice of best child
// (GameState.compare_gamestates, reference src/game_state.py:105-125, with the
// argmin/argmax of src/utils.py:90-105) is a plain unsigned max:
//
//     WIN  child, remoteness R  ->  0x4000 | R            (prefer the LONGEST win)
//     TIE  child, remoteness R  ->  0x8000 | (0x3FFF - R) (prefer the SHORTEST tie)
//     LOSS child, remoteness R  ->  0xC000 | (0x3FFF - R) (prefer the SHORTEST loss)
//     nothing / unsolved        ->  0
//
// and the parent's own score follows from the best child's score b
// (Process._res_red src/new_process.py:189-198; remoteness + 1 at :250):
//
//     b is LOSS -> parent WIN,  R = R_b + 1 -> 0x8000 - (b & 0x3FFF)
//     b is TIE  -> parent TIE,  R = R_b + 1 -> b - 1
//     b is WIN  -> parent LOSS, R = R_b + 1 -> 0xFFFE - (b & 0x3FFF)
//
// so the retrograde inner loop is u16 max (v_pk_max_u16 on packed pairs) and a
// three-way select per position, never per edge.
#pragma once
#include <stdint.h>

#ifndef GM_HD
#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD inline
#endif
#endif

namespace gm {

enum { WIN = 0, LOSS = 1, TIE = 2, DRAW = 3, UNDECIDED = 4 };

constexpr uint16_t REC_UNSOLVED = 0xFFFF;
constexpr uint64_t EMPTY_KEY = 0x8000000000000000ull;  // no game produces key 2^63
constexpr int MAX_CHILDREN = 16;
constexpr int MAX_REMOTENESS = 0x3FFE;

GM_HD uint16_t score_of_primitive(int v) {
    // remoteness 0 (PRIMITIVE_REMOTENESS, src/utils.py:7)
    return v == WIN ? 0x4000 : (v == LOSS ? 0xFFFF : 0xBFFF);
}

GM_HD uint16_t parent_score(uint32_t b) {
    uint32_t low = b & 0x3FFFu;
    uint32_t cls = b >> 14;
    uint32_t s = cls == 3 ? 0x8000u - low : (cls == 2 ? b - 1u : 0xFFFEu - low);
    return (uint16_t)s;
}

GM_HD uint16_t record_of_score(uint16_t s) {
    uint32_t cls = s >> 14, low = s & 0x3FFFu;
    if (cls == 1) return (uint16_t)low;                                   // WIN, R
    if (cls == 2) return (uint16_t)(0x8000u | (0x3FFFu - low));           // TIE
    if (cls == 3) return (uint16_t)(0x4000u | (0x3FFFu - low));           // LOSS
    return REC_UNSOLVED;
}

GM_HD uint16_t score_of_record(uint16_t r) {
    if (r == REC_UNSOLVED) return 0;
    uint32_t v = r >> 14, R = r & 0x3FFFu;
    if (v == WIN) return (uint16_t)(0x4000u | R);
    if (v == TIE) return (uint16_t)(0x8000u | (0x3FFFu - R));
    return (uint16_t)(0xC000u | (0x3FFFu - R));
}

// Remoteness overflow guard: a parent score would wrap when the child is at the
// end of its class range.
GM_HD bool score_overflows(uint32_t b) {
    uint32_t cls = b >> 14, low = b & 0x3FFFu;
    return (cls == 3 && low == 0) || (cls == 2 && low == 0) || (cls == 1 && low >= 0x3FFE);
}

// 1-byte codes of the dense subtraction path.  That game has a single primitive
// (all heaps empty: LOSS in 0), so only WIN and LOSS classes exist, and its
// remoteness is at most the heap total (<= 120 for 8 heaps of 4 bits):
//     WIN R -> R + 1 (1..127)      LOSS R -> 255 - R (129..255)      none -> 0
// The order matches the u16 scores above, so the best child is still a max, and
//     parent_code(b) = (255 - b) + 2 * (b >> 7)
// (best child LOSS R -> WIN R+1; best child WIN R -> LOSS R+1).
GM_HD uint32_t parent_code(uint32_t b) { return (255u - b) + ((b >> 7) << 1); }

GM_HD uint16_t record_of_code(uint8_t b) {
    if (b == 0) return REC_UNSOLVED;
    if (b >= 128) return (uint16_t)((1u << 14) | (255u - b));   // LOSS
    return (uint16_t)(b - 1u);                                   // WIN
}

GM_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

GM_HD uint64_t digest_term(uint64_t key, uint16_t rec) {
    return mix64(key * 0x9E3779B97F4A7C15ull + rec);
}

// 128-bit keys (boards whose position string exceeds 64 bits: Othello 8x8, games.hpp
// DescOthello8).  hi is the word a table insert claims with atomicCAS (sparse_tables.hpp): it
// never holds EMPTY_HI in a real key, and its bit PUB is set once the slot's lo word is
// written (1 in every complete key).
struct K128 {
    uint64_t lo, hi;
};
constexpr uint64_t EMPTY_HI = ~0ull;
constexpr uint64_t K128_PUB = 1ull << 36;   // hi's publish bit (every K128 descriptor keeps it set in its keys)
GM_HD bool operator==(const K128 &a, const K128 &b) { return a.lo == b.lo && a.hi == b.hi; }
GM_HD bool operator!=(const K128 &a, const K128 &b) { return !(a == b); }
GM_HD bool operator<(const K128 &a, const K128 &b) { return a.hi != b.hi ? a.hi < b.hi : a.lo < b.lo; }
GM_HD uint64_t mix_key(uint64_t k) { return mix64(k); }
GM_HD uint64_t mix_key(const K128 &k) { return mix64(k.lo ^ mix64(k.hi ^ 0x2545F4914F6CDD1Dull)); }
GM_HD bool key_empty(uint64_t k) { return k == EMPTY_KEY; }
GM_HD bool key_empty(const K128 &k) { return k.hi == EMPTY_HI; }
// the digest of a 128-bit key folds it to one word first (include/gmsolve.h gm_digest)
GM_HD uint64_t digest_term(const K128 &k, uint16_t rec) { return digest_term(mix_key(k), rec); }

GM_HD int popc64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __popcll(x);
#else
    return __builtin_popcountll(x);
#endif
}

}  // namespace gm
