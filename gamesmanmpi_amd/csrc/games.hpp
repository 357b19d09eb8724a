// games.hpp -- bit-packed game descriptors (host + device).
//
// Each descriptor restates one reference plugin over a u64 key:
//   primitive(k)          -> WIN/LOSS/TIE/DRAW/UNDECIDED     (plugin primitive())
//   visit(k, f)           -> calls f(child) for each child in gen_moves order until f
//                            returns false (gen_moves + do_move, i.e. GameState.expand,
//                            reference src/game_state.py:33-41); children(k, out)
//                            collects them into an array
//   tier(k)               -> a potential that strictly increases along every move;
//                            children land 1..MAX_SKIP tiers deeper
//   valid(k)              -> whether k is a position the plugin can represent
//
// Board games work on the key's planes directly.  A key stores cell (x, y) of an
// L x H board at plane bit c' = A-1-(L*y + x) (the reference string is MSB-first,
// App. B), i.e. the board rotated by 180 degrees: x' = L-1-x, y' = H-1-y and
// c' = L*y' + x'.  Word/line/flip rules are invariant under that rotation, so
// the descriptors use ordinary shift arithmetic in (x', y').
#pragma once
#include "gm_common.hpp"

namespace gm {

// children(k, out) of every descriptor: its visit() order (the plugin's gen_moves
// order) into an array.  Device kernels call visit() directly, so no child array
// has to live in (scratch) memory.
template <class D>
GM_HD int collect(const D &d, uint64_t k, uint64_t *out) {
    int n = 0;
    d.visit(k, [&](uint64_t c) {
        out[n++] = c;
        return true;
    });
    return n;
}

// Symmetry hooks (the reference's own hook is othello_bit_new.py:224-235,
// symmetry_functions, unused by its engines).  canon(k) is the representative the
// tables store; orbit(k, f) calls f once per distinct position the representative
// stands for.  A descriptor whose visit() returns canonical children solves one
// representative per orbit; counts, digests and exports expand every orbit, so the
// results are those of the unreduced game.  Games without a symmetry in use:
// descriptors with a visit_part() (the split kernels' per-lane share of visit())
template <class D, class = void>
struct part_visit_t {
    static constexpr bool value = false;
};
template <class D>
struct part_visit_t<D, std::void_t<decltype(D::PART_VISIT)>> {
    static constexpr bool value = D::PART_VISIT;
};

// descriptors with a count_children(k, &dt) (classify's edge counts by tier step without
// making the children: every child of k lands dt tiers deeper)
template <class D, class = void>
struct step_count_t {
    static constexpr bool value = false;
};
template <class D>
struct step_count_t<D, std::void_t<decltype(D::STEP_COUNT)>> {
    static constexpr bool value = D::STEP_COUNT;
};

// The key type of a descriptor: D::Key when it declares one (DescOthello8: K128), else u64.
template <class D, class = void>
struct key_of {
    using type = uint64_t;
};
template <class D>
struct key_of<D, std::void_t<typename D::Key>> {
    using type = typename D::Key;
};
template <class D>
using key_t = typename key_of<D>::type;

struct NoSym {
    GM_HD uint64_t canon(uint64_t k) const { return k; }
    template <class F>
    GM_HD void orbit(uint64_t k, F &&f) const { f(k); }
};

// ---------------------------------------------------------------- Four-To-One
// reference test_games/four_to_one.py:8-31 (moves are always -1, -2: the
// `x == 1` test at :15 compares a str with an int and never fires).
struct DescF2O : NoSym {
    static constexpr int MAX_SKIP = 2;
    static constexpr int MAXC = 2;
    GM_HD int primitive(uint64_t k) const { return (int64_t)k <= 0 ? LOSS : UNDECIDED; }
    template <class F>
    GM_HD void visit(uint64_t k, F &&f) const {
        if (f(k - 1)) f(k - 2);
    }
    GM_HD int children(uint64_t k, uint64_t *out) const { return collect(*this, k, out); }
    GM_HD int64_t tier(uint64_t k) const { return -(int64_t)k; }
    GM_HD bool valid(uint64_t k) const {
        int64_t x = (int64_t)k;
        return x > -((int64_t)1 << 60) && x < ((int64_t)1 << 60);
    }
};

// ---------------------------------------------------------------- Tic-tac-toe
// reference test_games/mttt.py:11-127 and tic_tac_toe_np.py:7-61.
// key = sum c_i 3^i, i = x + 3y, c: 0 blank, 1 X (player 1), 2 O (player 2).
struct DescTTT : NoSym {
    static constexpr int MAX_SKIP = 1;
    static constexpr int MAXC = 9;
    static constexpr uint32_t SLOTS = 19683;
    GM_HD static uint32_t pow3(int i) {
        uint32_t p = 1;
        for (int j = 0; j < i; j++) p *= 3;
        return p;
    }
    GM_HD static void decode(uint64_t k, int c[9]) {
        uint32_t v = (uint32_t)k;
        for (int i = 0; i < 9; i++) { c[i] = (int)(v % 3u); v /= 3u; }
    }
    GM_HD int primitive(uint64_t k) const {
        int c[9];
        decode(k, c);
        // rows, columns, diagonals: the lines checked from each piece in
        // directions (1,0), (0,1), (1,1), (-1,1) by mttt.py:69-83
        const int L[8][3] = {{0, 1, 2}, {3, 4, 5}, {6, 7, 8}, {0, 3, 6},
                             {1, 4, 7}, {2, 5, 8}, {0, 4, 8}, {2, 4, 6}};
        for (int l = 0; l < 8; l++) {
            int a = c[L[l][0]];
            if (a && a == c[L[l][1]] && a == c[L[l][2]]) return LOSS;
        }
        for (int i = 0; i < 9; i++)
            if (!c[i]) return UNDECIDED;
        return TIE;
    }
    template <class F>
    GM_HD void visit(uint64_t k, F &&f) const {
        int c[9], nx = 0, no = 0;
        decode(k, c);
        for (int i = 0; i < 9; i++) { nx += c[i] == 1; no += c[i] == 2; }
        uint64_t mover = no >= nx ? 1 : 2;   // mttt.py:39-43
        uint64_t p = 1;
        for (int i = 0; i < 9; i++, p *= 3)
            if (!c[i] && !f(k + mover * p)) return;
    }
    GM_HD int children(uint64_t k, uint64_t *out) const { return collect(*this, k, out); }
    GM_HD int64_t tier(uint64_t k) const {
        int c[9], n = 0;
        decode(k, c);
        for (int i = 0; i < 9; i++) n += c[i] != 0;
        return n;
    }
    GM_HD bool valid(uint64_t k) const { return k < SLOTS; }
};

// ---------------------------------------------------------------- Toot-and-Otto
// reference test_games/toot_and_otto_bitstring.py.  Key = first 2A+16 string
// bits: T plane at key bits [A+16, 2A+16), O plane at [16, A+16), then the hand
// nibbles P1-T (bits 12..15), P1-O (8..11), P2-T (4..7), P2-O (0..3).  The turn
// bit of the string equals the piece count mod 2 (player 2 moves first).
struct DescToot {
    static constexpr int MAX_SKIP = 1;
    static constexpr int MAXC = 16;
    int L, H, A;
    uint32_t amask;
    uint32_t start_h, start_v, start_d, start_a;   // segment starts per direction
    uint32_t colmask;                              // cells of column x' = 0
    // left-right mirror symmetry (set per solve, gm_api.hip: only when the root is its
    // own mirror image): the rules are mirror-invariant -- TOOT and OTTO are
    // palindromes, and the mirror swaps the two diagonal directions -- so a position
    // and its mirror image share value and remoteness, and with sym set visit()
    // returns min(child, mirror(child)).  Hands (bits 0..15) are unchanged.
    uint32_t sym = 0;
    GM_HD uint32_t mirror_plane(uint32_t p) const {
        uint32_t m = 0;
        for (int y = 0; y < H; y++) {
            const uint32_t row = (p >> (L * y)) & ((1u << L) - 1u);
            m |= (__builtin_bitreverse32(row) >> (32 - L)) << (L * y);
        }
        return m;
    }
    GM_HD uint64_t mirror(uint64_t k) const {
        return (k & 0xFFFFull) | ((uint64_t)mirror_plane(oplane(k)) << 16) |
               ((uint64_t)mirror_plane(tplane(k)) << (A + 16));
    }
    GM_HD uint64_t canon(uint64_t k) const {
        if (!sym) return k;
        const uint64_t m = mirror(k);
        return m < k ? m : k;
    }
    template <class F>
    GM_HD void orbit(uint64_t k, F &&f) const {
        f(k);
        if (sym) {
            const uint64_t m = mirror(k);
            if (m != k) f(m);
        }
    }

    static bool make(int L_, int H_, DescToot *d) {
        if (L_ < 1 || H_ < 1 || L_ > 8 || 2 * L_ * H_ + 16 > 64) return false;
        d->L = L_; d->H = H_; d->A = L_ * H_;
        d->amask = d->A == 32 ? 0xFFFFFFFFu : ((1u << d->A) - 1u);
        d->start_h = d->start_v = d->start_d = d->start_a = 0;
        d->colmask = 0;
        for (int y = 0; y < H_; y++) {
            d->colmask |= 1u << (L_ * y);
            for (int x = 0; x < L_; x++) {
                uint32_t b = 1u << (L_ * y + x);
                if (x + 3 < L_) d->start_h |= b;
                if (y + 3 < H_) d->start_v |= b;
                if (x + 3 < L_ && y + 3 < H_) d->start_d |= b;
                if (x - 3 >= 0 && y + 3 < H_) d->start_a |= b;
            }
        }
        return true;
    }
    GM_HD uint32_t tplane(uint64_t k) const { return (uint32_t)(k >> (A + 16)) & amask; }
    GM_HD uint32_t oplane(uint64_t k) const { return (uint32_t)(k >> 16) & amask; }
    GM_HD static int words(uint32_t a, uint32_t b, int d, uint32_t start) {
        // segments a b b a along step d (TOOT with a = T plane, OTTO with a = O plane)
        return popc64(a & (b >> d) & (b >> (2 * d)) & (a >> (3 * d)) & start);
    }
    GM_HD int primitive(uint64_t k) const {
        uint32_t t = tplane(k), o = oplane(k);
        int toot = words(t, o, 1, start_h) + words(t, o, L, start_v) +
                   words(t, o, L + 1, start_d) + words(t, o, L - 1, start_a);
        int otto = words(o, t, 1, start_h) + words(o, t, L, start_v) +
                   words(o, t, L + 1, start_d) + words(o, t, L - 1, start_a);
        int pieces = popc64(t | o);
        if (toot == otto) return pieces == A ? TIE : UNDECIDED;
        bool p1 = pieces & 1;                         // is_player1_turn (:218-219)
        return ((toot > otto) != p1) ? LOSS : WIN;    // :82-85
    }
    template <class F>
    GM_HD void visit(uint64_t k, F &&f) const {
        uint32_t occ = tplane(k) | oplane(k);
        bool p1 = popc64(occ) & 1;
        int tsh = p1 ? 12 : 4, osh = p1 ? 8 : 0;     // get_hand_count (:202-207)
        uint32_t th = (uint32_t)(k >> tsh) & 15u, oh = (uint32_t)(k >> osh) & 15u;
        bool have_t = th >= 1 && th <= 7, have_o = oh >= 1 && oh <= 7;  // signed nibble > 0
        for (int x = 0; x < L; x++) {                 // gen_moves order (:94-99)
            int xr = L - 1 - x;
            if (occ & (1u << xr)) continue;           // top cell (x, H-1) taken
            int filled = popc64(occ & (colmask << xr));
            int bit = L * (H - 1 - filled) + xr;      // lowest empty y (:112-115)
            if (have_t && !f(canon(k - (1ull << tsh) + (1ull << (A + 16 + bit))))) return;
            if (have_o && !f(canon(k - (1ull << osh) + (1ull << (16 + bit))))) return;
        }
    }
    GM_HD int children(uint64_t k, uint64_t *out) const { return collect(*this, k, out); }
    GM_HD int64_t tier(uint64_t k) const { return popc64(tplane(k) | oplane(k)); }
    GM_HD bool valid(uint64_t k) const {
        uint32_t t = tplane(k), o = oplane(k);
        if (t & o) return false;
        if (2 * A + 16 < 64 && (k >> (2 * A + 16))) return false;
        uint32_t occ = t | o;
        for (int xr = 0; xr < L; xr++) {              // pieces stacked from the bottom
            int filled = popc64(occ & (colmask << xr));
            for (int yr = 0; yr < H; yr++) {
                bool want = yr >= H - filled;
                if (((occ >> (L * yr + xr)) & 1u) != (uint32_t)want) return false;
            }
        }
        return true;
    }
};

// the descriptor with its symmetry reduction off: where only a child's tier matters
// (classify's edge counts), canonicalising every child is wasted work
template <class D>
GM_HD D unreduced(const D &d) { return d; }
GM_HD DescToot unreduced(const DescToot &d) {
    DescToot r = d;
    r.sym = 0;
    return r;
}


// ---------------------------------------------------------------- Othello
// reference test_games/othello_bit_new.py (square boards).  Key = all 2A+16
// string bits: WHITE plane at [A+16, 2A+16), BLACK plane at [16, A+16), the
// signed turn byte (1 BLACK, 2 WHITE) at bits 8..15, the pass byte at 0..7.
struct DescOthello {
    static constexpr int MAX_SKIP = 3;
    static constexpr int MAXC = 24;
    int L, A;
    uint32_t amask;
    // Board symmetries (set per solve, gm_api.hip): bit g of `sym` = element g of the
    // square's dihedral group D4 (0 identity, 1-3 rotations by 90/180/270 degrees, 4
    // transpose, 5 anti-transpose, 6/7 mirrors in x/y) that maps the ROOT to itself.
    // The rules -- flips along all 8 directions, the pass rule, the piece count -- are
    // invariant under D4 with colours kept, so positions in one orbit share value and
    // remoteness, and the positions reachable from a root that the subgroup fixes are
    // closed under it: visit() returns canonical children (min over the orbit) and
    // every count / export / digest expands the orbit.  From the standard start the
    // subgroup is {identity, rotation by 180, transpose, anti-transpose}.  The
    // reference's own declared symmetry, player_flip (othello_bit_new.py:224-235:
    // colours swapped and the turn advanced), fixes no reachable position set: a
    // reachable position's turn is fixed by its piece count (a pass keeps the mover,
    // who then passes again and ends the game), and player_flip keeps the pieces but
    // swaps the turn -- it maps every reachable position to an unreachable one, so it
    // merges nothing.
    uint32_t sym = 0;
    // 4x4 planes (the one Othello board above 2x2 a 64-bit key holds): bit permutations
    // by masks and shifts instead of the cell loop below (the canonical form is taken
    // for every child, in the latency-bound small-tier kernels)
    GM_HD static uint32_t mirror_x4(uint32_t p) {   // (x, y) -> (3 - x, y)
        return ((p & 0x1111u) << 3) | ((p & 0x8888u) >> 3) | ((p & 0x2222u) << 1) | ((p & 0x4444u) >> 1);
    }
    GM_HD static uint32_t mirror_y4(uint32_t p) {   // (x, y) -> (x, 3 - y)
        return ((p & 0x000Fu) << 12) | ((p & 0x00F0u) << 4) | ((p & 0x0F00u) >> 4) | ((p & 0xF000u) >> 12);
    }
    GM_HD static uint32_t transpose4(uint32_t p) {   // (x, y) -> (y, x)
        uint32_t t = (p ^ (p >> 3)) & 0x0A0Au;
        p ^= t ^ (t << 3);
        t = (p ^ (p >> 6)) & 0x00CCu;
        return p ^ t ^ (t << 6);
    }
    GM_HD static uint32_t xform_plane4(uint32_t p, int g) {
        switch (g) {
        case 1: return mirror_x4(transpose4(p));
        case 2: return mirror_x4(mirror_y4(p));
        case 3: return transpose4(mirror_x4(p));
        case 4: return transpose4(p);
        case 5: return mirror_x4(mirror_y4(transpose4(p)));
        case 6: return mirror_x4(p);
        case 7: return mirror_y4(p);
        }
        return p;
    }
    GM_HD uint32_t xform_plane(uint32_t p, int g) const {
        if (L == 4) return xform_plane4(p, g);
        return xform_plane_cells(p, g);
    }
    GM_HD uint32_t xform_plane_cells(uint32_t p, int g) const {
        uint32_t out = 0;
        for (int y = 0; y < L; y++)
            for (int x = 0; x < L; x++) {
                if (!((p >> (L * y + x)) & 1u)) continue;
                int nx = x, ny = y;
                switch (g) {
                case 1: nx = L - 1 - y; ny = x; break;
                case 2: nx = L - 1 - x; ny = L - 1 - y; break;
                case 3: nx = y; ny = L - 1 - x; break;
                case 4: nx = y; ny = x; break;
                case 5: nx = L - 1 - y; ny = L - 1 - x; break;
                case 6: nx = L - 1 - x; break;
                case 7: ny = L - 1 - y; break;
                }
                out |= 1u << (L * ny + nx);
            }
        return out;
    }
    GM_HD uint64_t xform(uint64_t k, int g) const {
        return ((uint64_t)xform_plane(wplane(k), g) << (A + 16)) | ((uint64_t)xform_plane(bplane(k), g) << 16) |
               (k & 0xFFFFull);
    }
    GM_HD uint64_t canon(uint64_t k) const {
        uint64_t m = k;
        for (int g = 1; g < 8; g++)
            if ((sym >> g) & 1u) {
                const uint64_t t = xform(k, g);
                m = t < m ? t : m;
            }
        return m;
    }
    template <class F>
    GM_HD void orbit(uint64_t k, F &&f) const {
        uint64_t seen[8];
        int n = 0;
        for (int g = 0; g < 8; g++) {
            if (g && !((sym >> g) & 1u)) continue;
            const uint64_t t = g ? xform(k, g) : k;
            bool dup = false;
            for (int i = 0; i < n; i++) dup |= seen[i] == t;
            if (!dup) { seen[n++] = t; f(t); }
        }
    }
    // the elements of D4 that fix k (bit 0 always set)
    GM_HD uint32_t stabilizer(uint64_t k) const {
        uint32_t s = 1u;
        for (int g = 1; g < 8; g++)
            if (xform(k, g) == k) s |= 1u << g;
        return s;
    }

    static bool make(int L_, int H_, DescOthello *d) {
        if (L_ != H_ || L_ < 2 || (L_ & 1) || 2 * L_ * H_ + 16 > 64) return false;
        d->L = L_; d->A = L_ * H_;
        d->amask = (1u << d->A) - 1u;
        return true;
    }
    GM_HD uint32_t wplane(uint64_t k) const { return (uint32_t)(k >> (A + 16)) & amask; }
    GM_HD uint32_t bplane(uint64_t k) const { return (uint32_t)(k >> 16) & amask; }
    GM_HD static int sbyte(uint64_t k, int sh) { return (int)(int8_t)(uint8_t)(k >> sh); }
    GM_HD int primitive(uint64_t k) const {
        uint32_t w = wplane(k), b = bplane(k);
        int pass = sbyte(k, 0), turn = sbyte(k, 8);
        if (popc64(w | b) != A && pass < 2) return UNDECIDED;   // :311-320
        int nb = popc64(b), nw = popc64(w);
        if (nb == nw) return TIE;
        return ((nb > nw) != (turn == 1)) ? LOSS : WIN;         // :305-309
    }
    // Pieces of `opp` flipped by `me` playing at (x, y) (rotated coordinates).
    GM_HD uint32_t flips(uint32_t me, uint32_t opp, int x, int y) const {
        uint32_t all = 0;
        for (int dx = -1; dx <= 1; dx++)
            for (int dy = -1; dy <= 1; dy++) {
                if (!dx && !dy) continue;
                uint32_t run = 0;
                int cx = x + dx, cy = y + dy;
                while (cx >= 0 && cy >= 0 && cx < L && cy < L) {
                    uint32_t b = 1u << (L * cy + cx);
                    if (opp & b) { run |= b; }
                    else { if (me & b) all |= run; break; }
                    cx += dx; cy += dy;
                }
            }
        return all;
    }
    template <class F>
    GM_HD void visit(uint64_t k, F &&fn) const {
        uint32_t w = wplane(k), b = bplane(k);
        int turn = sbyte(k, 8);
        bool black = turn == 1;
        uint32_t me = black ? b : w, opp = black ? w : b;
        uint64_t low = ((uint64_t)(uint8_t)(3 - turn)) << 8;     // incr_turn, pass reset
        int n = 0;
        for (int y = 0; y < L; y++)
            for (int x = 0; x < L; x++) {
                uint32_t cell = 1u << (L * y + x);
                if ((w | b) & cell) continue;
                uint32_t f = flips(me, opp, x, y);
                if (!f) continue;                                 // legit_move (:370-382)
                uint32_t nme = me | cell | f, nopp = opp & ~f;
                uint32_t nw = black ? nopp : nme, nb = black ? nme : nopp;
                n++;
                if (!fn(canon(((uint64_t)nw << (A + 16)) | ((uint64_t)nb << 16) | low))) return;
            }
        if (!n) fn(canon(k + 1));                                 // [None]: pass + 1 (:122-124)
    }
    GM_HD int children(uint64_t k, uint64_t *out) const { return collect(*this, k, out); }
    // The split kernels' per-lane share of visit(): the children from the empty squares
    // part, part + nparts, ... only (a 16-lane row of the 4x4 board: one square per
    // lane instead of every lane scanning all 16).  Returns how many legal moves they
    // gave; the caller emits pass_child(k) when no lane of the row found one.
    static constexpr bool PART_VISIT = true;
    template <class F>
    GM_HD int visit_part(uint64_t k, int part, int nparts, F &&fn) const {
        uint32_t w = wplane(k), b = bplane(k);
        int turn = sbyte(k, 8);
        bool black = turn == 1;
        uint32_t me = black ? b : w, opp = black ? w : b;
        uint64_t low = ((uint64_t)(uint8_t)(3 - turn)) << 8;
        int n = 0;
        for (int sq = part; sq < A; sq += nparts) {
            uint32_t cell = 1u << sq;
            if ((w | b) & cell) continue;
            uint32_t f = flips(me, opp, sq % L, sq / L);
            if (!f) continue;
            uint32_t nme = me | cell | f, nopp = opp & ~f;
            uint32_t nw = black ? nopp : nme, nb = black ? nme : nopp;
            n++;
            if (!fn(canon(((uint64_t)nw << (A + 16)) | ((uint64_t)nb << 16) | low))) return n;
        }
        return n;
    }
    GM_HD uint64_t pass_child(uint64_t k) const { return canon(k + 1); }
    GM_HD int64_t tier(uint64_t k) const {
        return 3 * popc64(wplane(k) | bplane(k)) + sbyte(k, 0);
    }
    GM_HD bool valid(uint64_t k) const {
        if (wplane(k) & bplane(k)) return false;
        if (2 * A + 16 < 64 && (k >> (2 * A + 16))) return false;
        int turn = sbyte(k, 8), pass = sbyte(k, 0);
        return (turn == 1 || turn == 2) && pass >= 0 && pass <= 2;
    }
};

GM_HD DescOthello unreduced(const DescOthello &d) {
    DescOthello r = d;
    r.sym = 0;
    return r;
}

// ---------------------------------------------------------------- Othello 8x8 (128-bit keys)
// The reference plugin at its default board, reference test_games/othello_bit_new.py:8 (8x8):
// its position string is 2A + 16 = 144 bits (white plane, black plane, turn byte, pass byte,
// :36-55), so the key is a K128 (gm_common.hpp) and the tables are 32-byte slots
// (sparse_tables.hpp).  Planes are read big-endian from the string, so string bit j = 8y + x
// is plane bit 63 - j: the board rotated by 180 degrees, which the rules do not see.
//   lo = the white plane
//   hi = the occupied plane (white | black) with its four centre bits -- squares that are
//        occupied in every position (the start's four discs are never removed) -- reused:
//        bit 27 = white to move (turn byte 2), bits 28 / 35 = pass count bits 0 / 1, bit 36 =
//        the insert's publish bit (set in every key; never all-ones: pass 3 does not occur)
// The ABI key (include/gmsolve.h, gm_key_words = 3) is the position string as one integer, in
// little-endian u64 words (to_words / from_words).  Rules as DescOthello (pass keeps the mover,
// :122-124; the game ends on a full board or a second pass, :82-84).  No symmetry reduction.
struct DescOthello8 {
    using Key = K128;
    static constexpr int MAX_SKIP = 3;
    static constexpr int MAXC = 64;
    static constexpr uint64_t CENTRE = (1ull << 27) | (1ull << 28) | (1ull << 35) | (1ull << 36);
    static constexpr uint64_t TURN_W = 1ull << 27, PASS0 = 1ull << 28, PASS1 = 1ull << 35, PUB = K128_PUB;
    GM_HD K128 canon(const K128 &k) const { return k; }
    template <class F>
    GM_HD void orbit(const K128 &k, F &&f) const { f(k); }
    GM_HD static uint64_t occ(const K128 &k) { return k.hi | CENTRE; }
    GM_HD static int turn(const K128 &k) { return (k.hi & TURN_W) ? 2 : 1; }
    GM_HD static int pass(const K128 &k) { return (int)((k.hi >> 28) & 1u) | (int)(((k.hi >> 35) & 1u) << 1); }
    GM_HD static K128 pack(uint64_t w, uint64_t b, int turn, int pass) {
        K128 k;
        k.lo = w;
        k.hi = ((w | b) & ~CENTRE) | (turn == 2 ? TURN_W : 0) | ((pass & 1) ? PASS0 : 0) | ((pass & 2) ? PASS1 : 0) | PUB;
        return k;
    }
    GM_HD int primitive(const K128 &k) const {
        const uint64_t o = occ(k), w = k.lo, b = o & ~w;
        if (o != ~0ull && pass(k) < 2) return UNDECIDED;          // :75-84
        const int nb = popc64(b), nw = popc64(w);
        if (nb == nw) return TIE;
        return ((nb > nw) != (turn(k) == 1)) ? LOSS : WIN;         // :59-73
    }
    // Bitboard move generation (round 6; round 5 walked the squares, a loop per direction --
    // gm_expand_host_key's tests pin the children to the plugin's either way).  step<DIR> moves every
    // disc of a plane one square in direction DIR (E W S N SE SW NE NW on bit 8y + x), clearing
    // the column a shift wraps into; run<DIR>(from, opp) is the opp discs in an unbroken line
    // from the squares next to `from` (at most 6 on an 8-wide board).  Every lane runs the same
    // instructions, where the square walk's loops diverged with each lane's position.
    template <int DIR>
    GM_HD static uint64_t step(uint64_t b) {
        constexpr uint64_t notA = 0xFEFEFEFEFEFEFEFEull, notH = 0x7F7F7F7F7F7F7F7Full;
        if constexpr (DIR == 0) return (b << 1) & notA;
        else if constexpr (DIR == 1) return (b >> 1) & notH;
        else if constexpr (DIR == 2) return b << 8;
        else if constexpr (DIR == 3) return b >> 8;
        else if constexpr (DIR == 4) return (b << 9) & notA;
        else if constexpr (DIR == 5) return (b << 7) & notH;
        else if constexpr (DIR == 6) return (b >> 7) & notA;
        else return (b >> 9) & notH;
    }
    template <int DIR>
    GM_HD static uint64_t run(uint64_t from, uint64_t opp) {
        uint64_t t = step<DIR>(from) & opp;
#pragma unroll
        for (int i = 0; i < 5; i++) t |= step<DIR>(t) & opp;
        return t;
    }
    // the squares `me` can play: empty, at the end of a run of opp discs that starts next to a me disc
    template <int DIR = 0>
    GM_HD static uint64_t legal(uint64_t me, uint64_t opp) {
        const uint64_t m = step<DIR>(run<DIR>(me, opp)) & ~(me | opp);
        if constexpr (DIR < 7) return m | legal<DIR + 1>(me, opp);
        else return m;
    }
    // the opp discs `me` flips by playing the square `bit` (flip_helper, :100-118): each
    // direction's run, when a me disc ends it
    template <int DIR = 0>
    GM_HD static uint64_t flips_at(uint64_t me, uint64_t opp, uint64_t bit) {
        const uint64_t t = run<DIR>(bit, opp);
        const uint64_t f = (step<DIR>(t) & me) ? t : 0ull;
        if constexpr (DIR < 7) return f | flips_at<DIR + 1>(me, opp, bit);
        else return f;
    }
    // classify's edge counts without making the children: every move lands 3 - pass tiers
    // deeper (one more disc, the pass count reset), the pass child 1 (sparse_tables.hpp)
    static constexpr bool STEP_COUNT = true;
    GM_HD int count_children(const K128 &k, int *dt) const {
        const uint64_t o = occ(k), w = k.lo, b = o & ~w;
        const bool black = turn(k) == 1;
        const int n = popc64(legal(black ? b : w, black ? w : b));
        *dt = n ? 3 - pass(k) : 1;
        return n ? n : 1;
    }
    template <class F>
    GM_HD void visit(const K128 &k, F &&fn) const {
        const uint64_t o = occ(k), w = k.lo, b = o & ~w;
        const int t = turn(k);
        const bool black = t == 1;
        const uint64_t me = black ? b : w, opp = black ? w : b;
        uint64_t mv = legal(me, opp);   // legit moves (:134-146), in square order
        if (!mv) {
            fn(pack(w, b, t, pass(k) + 1));                         // [None]: incr_pass only (:122-124)
            return;
        }
        for (; mv; mv &= mv - 1) {
            const uint64_t bit = mv & (~mv + 1);
            const uint64_t f = flips_at(me, opp, bit);
            const uint64_t nme = me | bit | f, nopp = opp & ~f;
            if (!fn(pack(black ? nopp : nme, black ? nme : nopp, 3 - t, 0))) return;   // incr_turn, reset_pass
        }
    }
    GM_HD int children(const K128 &k, K128 *out) const {
        int n = 0;
        visit(k, [&](const K128 &c) {
            out[n++] = c;
            return true;
        });
        return n;
    }
    GM_HD int64_t tier(const K128 &k) const { return 3 * popc64(occ(k)) + pass(k); }
    GM_HD bool valid(const K128 &k) const {
        if (!(k.hi & PUB) || k.hi == EMPTY_HI) return false;
        if (k.lo & ~occ(k)) return false;
        return pass(k) <= 2;
    }
    // ABI words (the 144-bit string integer I = W << 80 | B << 16 | turn << 8 | pass)
    static void to_words(const K128 &k, uint64_t *wd) {
        const uint64_t w = k.lo, b = occ(k) & ~w;
        wd[0] = (b << 16) | ((uint64_t)turn(k) << 8) | (uint64_t)pass(k);
        wd[1] = (b >> 48) | (w << 16);
        wd[2] = w >> 48;
    }
    // false when the words are no position of this descriptor (a centre square empty, the
    // planes overlapping, turn / pass out of range, bits above 144)
    static bool from_words(const uint64_t *wd, K128 *k) {
        if (wd[2] >> 16) return false;
        const uint64_t w = (wd[1] >> 16) | (wd[2] << 48), b = (wd[0] >> 16) | (wd[1] << 48);
        const int t = (int)((wd[0] >> 8) & 0xFF), ps = (int)(wd[0] & 0xFF);
        if ((w & b) || ((w | b) & CENTRE) != CENTRE || (t != 1 && t != 2) || ps > 2) return false;
        *k = pack(w, b, t, ps);
        return true;
    }
};

// ---------------------------------------------------------------- Subtract
// The build's synthetic game: `heaps` heaps of 4 bits; a move
// takes 1 or 2 from one non-empty heap, floor 0 (duplicate children dropped);
// all heaps empty is a LOSS.  One heap = Four-To-One for piles >= 0.
struct DescSub : NoSym {
    static constexpr int MAX_SKIP = 2;
    static constexpr int MAXC = 16;
    int heaps;
    GM_HD int primitive(uint64_t k) const { return k == 0 ? LOSS : UNDECIDED; }
    template <class F>
    GM_HD void visit(uint64_t k, F &&f) const {
        for (int i = 0; i < heaps; i++) {
            uint64_t h = (k >> (4 * i)) & 15u;
            if (h >= 1 && !f(k - (1ull << (4 * i)))) return;
            if (h >= 2 && !f(k - (2ull << (4 * i)))) return;
        }
    }
    GM_HD int children(uint64_t k, uint64_t *out) const { return collect(*this, k, out); }
    GM_HD int64_t tier(uint64_t k) const {
        int64_t s = 0;
        for (int i = 0; i < heaps; i++) s += (k >> (4 * i)) & 15u;
        return -s;
    }
    GM_HD bool valid(uint64_t k) const { return heaps >= 16 || (k >> (4 * heaps)) == 0; }
};

}  // namespace gm
