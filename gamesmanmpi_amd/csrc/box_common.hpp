// box_common.hpp -- box geometry of the 8-heap synthetic game, shared by the one-GPU box engine
// (dense_box.hip) and its split over ranks (dist_box.hip).
//
// The 16^8 lattice is cut into BOXES of 4 x 4 x 4 x 4 x 2 x 2 x 2 x 2 positions: heaps 0-3
// in quarters ("A" heaps, box coordinate c_i = h_i >> 2, 0..3), heaps 4-7 in halves ("B" heaps,
// c_j = h_j >> 1, 0..7).  Table index = box << 12 | A << 4 | B, A = sum over heaps 0-3 of
// (h_i & 3) << 2i, B = sum over heaps 4-7 of (h_j & 1) << (j - 4); the box id packs c_i at
// bits 2i (i < 4) and c_j at bits 8 + 3 (j - 4) (j >= 4).
//
// Heap transpositions.  Every heap plays by the same rules and the only primitive position
// has all heaps empty, so swapping two heaps maps a position to one of equal value and
// remoteness.  Swapping two A heaps or two B heaps maps boxes to boxes and keeps the box-tier
// (the sum of the box coordinates).  Code of a transposition: 0 = none, 1..6 = the A heaps of
// pair code - 1, 7..12 = the B heaps 4 + q, 4 + p of pair code - 7, pairs in the order
// (0,1) (0,2) (0,3) (1,2) (1,3) (2,3).  On a box it swaps two coordinate fields; on a row of
// 16 codes (one A, B = 0..15) an A transposition moves the row (A's digits q, p swap: row A
// of box C is row swap(A) of box swap(C)), a B transposition permutes its bytes (byte B of a
// row of C is byte swap(B) of the same row of swap(C)).
#pragma once
#include <stdint.h>

#ifndef GM_HD
#define GM_HD __host__ __device__ __forceinline__
#endif

namespace gm {

GM_HD uint32_t box_index_of_key(uint32_t k) {
    uint32_t off = 0, box = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t h = (k >> (4 * i)) & 15u;
        off |= (h & 3u) << (4 + 2 * i);
        box |= (h >> 2) << (2 * i);
    }
    for (int j = 0; j < 4; j++) {
        const uint32_t h = (k >> (16 + 4 * j)) & 15u;
        off |= (h & 1u) << j;
        box |= (h >> 1) << (8 + 3 * j);
    }
    return (box << 12) | off;
}
GM_HD uint32_t box_key_of_index(uint32_t x) {
    const uint32_t off = x & 4095u, box = x >> 12;
    uint32_t k = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t h = (((box >> (2 * i)) & 3u) << 2) | ((off >> (4 + 2 * i)) & 3u);
        k |= h << (4 * i);
    }
    for (int j = 0; j < 4; j++) {
        const uint32_t h = (((box >> (8 + 3 * j)) & 7u) << 1) | ((off >> j) & 1u);
        k |= h << (16 + 4 * j);
    }
    return k;
}
GM_HD int box_coord(uint32_t box, int dim) {
    return dim < 4 ? (int)((box >> (2 * dim)) & 3u) : (int)((box >> (8 + 3 * (dim - 4))) & 7u);
}
GM_HD uint32_t box_unit(int dim) { return dim < 4 ? 1u << (2 * dim) : 1u << (8 + 3 * (dim - 4)); }
GM_HD int box_tier(uint32_t box) {
    int t = 0;
    for (int i = 0; i < 8; i++) t += box_coord(box, i);
    return t;
}

// transposition codes (see the file comment)
constexpr int BX_NSWAP = 13;
GM_HD uint32_t bx_pair_q(uint32_t pc) { return pc < 3 ? 0u : pc < 5 ? 1u : 2u; }
GM_HD uint32_t bx_pair_p(uint32_t pc) { return pc < 3 ? pc + 1 : pc < 5 ? pc - 1 : 3u; }
GM_HD bool bx_swap_is_a(uint32_t code) { return code >= 1 && code <= 6; }
GM_HD bool bx_swap_is_b(uint32_t code) { return code >= 7; }
// the transposition's two heaps (0..7)
GM_HD void bx_swap_heaps(uint32_t code, int *q, int *p) {
    const uint32_t pc = bx_swap_is_a(code) ? code - 1 : code - 7, o = bx_swap_is_a(code) ? 0u : 4u;
    *q = (int)(o + bx_pair_q(pc));
    *p = (int)(o + bx_pair_p(pc));
}
GM_HD uint32_t bx_swap_box(uint32_t code, uint32_t b) {
    if (!code) return b;
    if (bx_swap_is_a(code)) {
        const uint32_t q = 2u * bx_pair_q(code - 1), p = 2u * bx_pair_p(code - 1);
        const uint32_t t = ((b >> q) ^ (b >> p)) & 3u;
        return b ^ (t << q) ^ (t << p);
    }
    const uint32_t q = 8u + 3u * bx_pair_q(code - 7), p = 8u + 3u * bx_pair_p(code - 7);
    const uint32_t t = ((b >> q) ^ (b >> p)) & 7u;
    return b ^ (t << q) ^ (t << p);
}
// row index A (0..255) of the box read through an A transposition (identity for the others)
GM_HD uint32_t bx_swap_row(uint32_t code, uint32_t A) {
    if (!bx_swap_is_a(code)) return A;
    const uint32_t q = 2u * bx_pair_q(code - 1), p = 2u * bx_pair_p(code - 1);
    const uint32_t t = ((A >> q) ^ (A >> p)) & 3u;
    return A ^ (t << q) ^ (t << p);
}
// a key through a transposition (heap i at bits 4 i)
GM_HD uint32_t bx_swap_key(uint32_t code, uint32_t k) {
    if (!code) return k;
    int q, p;
    bx_swap_heaps(code, &q, &p);
    const uint32_t t = ((k >> (4 * q)) ^ (k >> (4 * p))) & 15u;
    return k ^ (t << (4 * q)) ^ (t << (4 * p));
}

}  // namespace gm
