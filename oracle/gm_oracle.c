/*
 * gm_oracle.c -- CPU oracle (plain C restatement of the reference's algorithm).
 *
 * TEST INFRASTRUCTURE ONLY.  Built into oracle/_build/liboracle.so and loaded
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
 * checker.  The solver product (libgmsolve.so, gamesmanmpi_amd/) never links,
 * loads or calls it.
 *
 * Semantics: SURVEY Appendix A (canonical fixed point):
 *   - closure of the root under the plugin's moves; primitives are not expanded
 *     (reference src/new_process.py:102-133);
 *   - primitive -> (primitive value, remoteness 0)  (src/utils.py:7, src/new_process.py:122);
 *   - otherwise: any LOSS child -> WIN, 1 + min R over LOSS children; else any TIE
 *     child -> TIE, 1 + min R over TIE children; else LOSS, 1 + max R
 *     (GameState.compare_gamestates src/game_state.py:105-125, argmin/argmax
 *     src/utils.py:90-105, Process._res_red src/new_process.py:189-198, R+1 at :250).
 *   - DRAW primitives and non-primitive positions without moves are errors.
 *
 * The game rules below are deliberately written cell-by-cell, the way the
 * reference plugins are (board_get / word_test / flip_helper), not with the
 * bit tricks of the device descriptors, so the two implementations are
 * independent.  Keys follow SURVEY Appendix B.
 *
 * Pinned by: the tests/golden npz tables (canonical tables over the reference's own
 * plugin modules) and roots.json (the reference's game_tests expectations).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define WIN 0
#define LOSS 1
#define TIE 2
#define DRAW 3
#define UNDECIDED 4

#define G_F2O 1
#define G_TTT 2
#define G_TOOT 3
#define G_OTHELLO 4
#define G_SUBTRACT 5

#define MAXKIDS 64

typedef struct {
    int game;
    int L, H;     /* board dims (toot / othello); heaps (subtract) in L */
} game_t;

static char g_err[256];
const char *oracle_last_error(void) { return g_err; }

/* ------------------------------------------------------------------ F2O */
/* reference test_games/four_to_one.py:8-31; the x == 1 branch (:15) is dead. */
static int f2o_prim(int64_t x) { return x <= 0 ? LOSS : UNDECIDED; }
static int f2o_kids(int64_t x, uint64_t *out) {
    out[0] = (uint64_t)(x - 1);
    out[1] = (uint64_t)(x - 2);
    return 2;
}

/* ------------------------------------------------------------------ TTT */
/* reference test_games/mttt.py:11-127 (cell (x,y) = x + 3y, X to move iff #O >= #X). */
static void ttt_decode(uint64_t key, int c[9]) {
    for (int i = 0; i < 9; i++) { c[i] = (int)(key % 3); key /= 3; }
}
static uint64_t ttt_encode(const int c[9]) {
    uint64_t k = 0;
    for (int i = 8; i >= 0; i--) k = k * 3 + (uint64_t)c[i];
    return k;
}
static int ttt_piece(const int c[9], int x, int y) {
    if (x < 0 || x > 2 || y < 0 || y > 2) return -1;  /* 'B' border */
    return c[x + 3 * y];
}
static int ttt_prim(uint64_t key) {
    int c[9];
    ttt_decode(key, c);
    int blank = 0;
    for (int i = 0; i < 9; i++) {
        if (c[i] == 0) { blank = 1; continue; }
        int x = i % 3, y = i / 3, p = c[i];
        if ((ttt_piece(c, x + 1, y) == p && ttt_piece(c, x + 2, y) == p) ||
            (ttt_piece(c, x, y + 1) == p && ttt_piece(c, x, y + 2) == p) ||
            (ttt_piece(c, x + 1, y + 1) == p && ttt_piece(c, x + 2, y + 2) == p) ||
            (ttt_piece(c, x - 1, y + 1) == p && ttt_piece(c, x - 2, y + 2) == p))
            return LOSS;
    }
    return blank ? UNDECIDED : TIE;
}
static int ttt_kids(uint64_t key, uint64_t *out) {
    int c[9], nx = 0, no = 0, n = 0;
    ttt_decode(key, c);
    for (int i = 0; i < 9; i++) { nx += c[i] == 1; no += c[i] == 2; }
    int mover = no >= nx ? 1 : 2;
    for (int i = 0; i < 9; i++) {
        if (c[i]) continue;
        c[i] = mover;
        out[n++] = ttt_encode(c);
        c[i] = 0;
    }
    return n;
}

/* ------------------------------------------------------------------ Toot */
/* reference test_games/toot_and_otto_bitstring.py.  The key is the first 2A+16
 * bits of the position string (MSB-first): bit j of the string is key bit
 * (2A+15-j).  Cells: T plane j = L*y+x, O plane j = A+L*y+x; hands at
 * j = 2A + 8(p-1) + (0 T | 4 O), 4 bits each.  The turn bit (last string bit)
 * equals the number of pieces mod 2 (it starts 0 and toggles every move). */
typedef struct { int cell[64]; int hand[2][2]; int pieces; } toot_t;   /* hand[p-1][0=T,1=O] */
#define T_ 1
#define O_ (-1)

static int keybit(uint64_t key, int nkey, int j) { return (int)((key >> (nkey - 1 - j)) & 1u); }

static void toot_decode(const game_t *g, uint64_t key, toot_t *s) {
    int L = g->L, H = g->H, A = L * H, nk = 2 * A + 16;
    s->pieces = 0;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < L; x++) {
            int j = L * y + x, v = 0;
            if (keybit(key, nk, j)) v = T_;
            else if (keybit(key, nk, A + j)) v = O_;
            s->cell[j] = v;
            s->pieces += v != 0;
        }
    for (int p = 0; p < 2; p++)
        for (int l = 0; l < 2; l++) {
            int start = 2 * A + 8 * p + 4 * l, v = 0;
            for (int b = 0; b < 4; b++) v = (v << 1) | keybit(key, nk, start + b);
            s->hand[p][l] = v >= 8 ? v - 16 : v;   /* BitArray.int is signed */
        }
}
static uint64_t toot_encode(const game_t *g, const toot_t *s) {
    int L = g->L, H = g->H, A = L * H, nk = 2 * A + 16;
    uint64_t key = 0;
    for (int j = 0; j < A; j++) {
        if (s->cell[j] == T_) key |= 1ull << (nk - 1 - j);
        if (s->cell[j] == O_) key |= 1ull << (nk - 1 - (A + j));
    }
    for (int p = 0; p < 2; p++)
        for (int l = 0; l < 2; l++) {
            int start = 2 * A + 8 * p + 4 * l;
            uint64_t v = (uint64_t)(s->hand[p][l] & 15);
            key |= v << (nk - start - 4);
        }
    (void)H;
    return key;
}
static int toot_get(const game_t *g, const toot_t *s, int x, int y) { return s->cell[g->L * y + x]; }
/* word_test, toot_and_otto_bitstring.py:70-77 */
static int toot_word(const game_t *g, const toot_t *s, int x, int y, const char *w, int dx, int dy, int pos) {
    if (pos >= 4) return 1;
    if (x < 0 || y < 0 || x >= g->L || y >= g->H) return 0;
    int c = toot_get(g, s, x, y);
    char ch = c == T_ ? 'T' : (c == O_ ? 'O' : '-');
    if (ch != w[pos]) return 0;
    return toot_word(g, s, x + dx, y + dy, w, dx, dy, pos + 1);
}
static int toot_prim(const game_t *g, uint64_t key) {
    toot_t s;
    toot_decode(g, key, &s);
    int toot = 0, otto = 0, full = 1;
    for (int x = 0; x < g->L; x++)
        for (int y = 0; y < g->H; y++) {
            int c = toot_get(g, &s, x, y);
            if (!c) { full = 0; continue; }
            const char *w = c == T_ ? "TOOT" : "OTTO";
            int *sc = c == T_ ? &toot : &otto;
            *sc += toot_word(g, &s, x + 1, y, w, 1, 0, 1);
            *sc += toot_word(g, &s, x, y + 1, w, 0, 1, 1);
            *sc += toot_word(g, &s, x + 1, y + 1, w, 1, 1, 1);
            *sc += toot_word(g, &s, x + 1, y - 1, w, 1, -1, 1);
        }
    if (toot == otto) return full ? TIE : UNDECIDED;
    int p1 = s.pieces & 1;
    return ((toot > otto) ^ p1) ? LOSS : WIN;
}
static int toot_kids(const game_t *g, uint64_t key, uint64_t *out) {
    toot_t s;
    toot_decode(g, key, &s);
    int p = (s.pieces & 1) ? 0 : 1;   /* player 1 iff the turn bit is set */
    int n = 0;
    for (int x = 0; x < g->L; x++) {
        if (toot_get(g, &s, x, g->H - 1)) continue;
        for (int l = 0; l < 2; l++) {
            if (s.hand[p][l] <= 0) continue;
            toot_t c = s;
            c.hand[p][l] -= 1;
            for (int y = 0; y < g->H; y++)
                if (!toot_get(g, &c, x, y)) { c.cell[g->L * y + x] = l == 0 ? T_ : O_; break; }
            out[n++] = toot_encode(g, &c);
        }
    }
    return n;
}

/* ------------------------------------------------------------------ Othello */
/* reference test_games/othello_bit_new.py.  Key = all 2A+16 bits of the string:
 * WHITE plane j = L*y+x, BLACK plane A+j, 8-bit signed turn (1 BLACK, 2 WHITE),
 * 8-bit pass count. */
#define OW 2
#define OB 1
typedef struct { int cell[64]; int turn; int pass; } oth_t;
static void oth_decode(const game_t *g, uint64_t key, oth_t *s) {
    int A = g->L * g->H, nk = 2 * A + 16;
    for (int j = 0; j < A; j++)
        s->cell[j] = keybit(key, nk, j) ? OW : (keybit(key, nk, A + j) ? OB : 0);
    int t = (int)((key >> 8) & 0xFF), p = (int)(key & 0xFF);
    s->turn = t >= 128 ? t - 256 : t;
    s->pass = p >= 128 ? p - 256 : p;
}
static uint64_t oth_encode(const game_t *g, const oth_t *s) {
    int A = g->L * g->H, nk = 2 * A + 16;
    uint64_t key = 0;
    for (int j = 0; j < A; j++) {
        if (s->cell[j] == OW) key |= 1ull << (nk - 1 - j);
        if (s->cell[j] == OB) key |= 1ull << (nk - 1 - (A + j));
    }
    key |= (uint64_t)(s->turn & 0xFF) << 8;
    key |= (uint64_t)(s->pass & 0xFF);
    return key;
}
static int oth_get(const game_t *g, const oth_t *s, int x, int y) { return s->cell[g->L * y + x]; }
static int oth_mover(const oth_t *s) { return s->turn == 1 ? OB : OW; }
static int oth_prim(const game_t *g, uint64_t key) {
    oth_t s;
    oth_decode(g, key, &s);
    int filled = 0, black = 0, white = 0;
    for (int x = 0; x < g->L; x++)
        for (int y = 0; y < g->H; y++) {
            int c = oth_get(g, &s, x, y);
            filled += c != 0;
            black += c == OB;
            white += c == OW;
        }
    if (filled != g->L * g->H && s.pass < 2) return UNDECIDED;
    if (black == white) return TIE;
    return ((black > white) ^ (s.turn == 1)) ? LOSS : WIN;
}
/* legit_helper, othello_bit_new.py:384-396 */
static int oth_legit(const game_t *g, const oth_t *s, int x, int y, int dx, int dy, int first) {
    if (x >= g->L || y >= g->H || x < 0 || y < 0) return 0;
    int me = oth_mover(s), opp = me == OB ? OW : OB, c = oth_get(g, s, x, y);
    if (first) return c == opp ? oth_legit(g, s, x + dx, y + dy, dx, dy, 0) : 0;
    if (c == me) return 1;
    if (c == opp) return oth_legit(g, s, x + dx, y + dy, dx, dy, 0);
    return 0;
}
static void oth_flip_dir(const game_t *g, oth_t *s, int x, int y, int dx, int dy, int me) {
    /* flip_helper / flip_helper2, othello_bit_new.py:336-354 (x bound by height, y by length) */
    int opp = me == OB ? OW : OB, run[64][2], n = 0;
    if (x >= g->H || y >= g->L || x < 0 || y < 0) return;
    if (oth_get(g, s, x, y) != opp) return;
    run[n][0] = x; run[n][1] = y; n++;
    for (;;) {
        x += dx; y += dy;
        if (x >= g->H || y >= g->L || x < 0 || y < 0) return;
        int c = oth_get(g, s, x, y);
        if (c == me) {
            for (int i = 0; i < n; i++) s->cell[g->L * run[i][1] + run[i][0]] = me;
            return;
        }
        if (c != opp) return;
        run[n][0] = x; run[n][1] = y; n++;
    }
}
static int oth_kids(const game_t *g, uint64_t key, uint64_t *out) {
    oth_t s;
    oth_decode(g, key, &s);
    int n = 0;
    for (int x = 0; x < g->L; x++)
        for (int y = 0; y < g->H; y++) {
            if (oth_get(g, &s, x, y)) continue;
            int ok = 0;
            for (int dx = -1; dx <= 1 && !ok; dx++)
                for (int dy = -1; dy <= 1 && !ok; dy++)
                    if ((dx || dy) && oth_legit(g, &s, x + dx, y + dy, dx, dy, 1)) ok = 1;
            if (!ok) continue;
            oth_t c = s;
            int me = oth_mover(&s);
            c.pass = 0;
            c.cell[g->L * y + x] = me;
            for (int dx = -1; dx <= 1; dx++)
                for (int dy = -1; dy <= 1; dy++)
                    if (dx || dy) oth_flip_dir(g, &c, x + dx, y + dy, dx, dy, me);
            c.turn = c.turn % 2 + 1;
            out[n++] = oth_encode(g, &c);
        }
    if (n == 0) {   /* the [None] move: pass count + 1, turn unchanged (:122-124) */
        oth_t c = s;
        c.pass += 1;
        out[n++] = oth_encode(g, &c);
    }
    return n;
}

/* ------------------------------------------------------------------ Subtract */
/* The build's synthetic game: heaps of 4 bits; take 1 or 2, floor 0. */
static int sub_prim(uint64_t key) { return key == 0 ? LOSS : UNDECIDED; }
static int sub_kids(const game_t *g, uint64_t key, uint64_t *out) {
    int n = 0;
    for (int i = 0; i < g->L; i++) {
        uint64_t h = (key >> (4 * i)) & 15;
        if (h >= 1) out[n++] = key - (1ull << (4 * i));
        if (h >= 2) out[n++] = key - (2ull << (4 * i));
    }
    return n;
}

/* ------------------------------------------------------------------ dispatch */
static int g_prim(const game_t *g, uint64_t k) {
    switch (g->game) {
    case G_F2O: return f2o_prim((int64_t)k);
    case G_TTT: return ttt_prim(k);
    case G_TOOT: return toot_prim(g, k);
    case G_OTHELLO: return oth_prim(g, k);
    case G_SUBTRACT: return sub_prim(k);
    }
    return -1;
}
static int g_kids(const game_t *g, uint64_t k, uint64_t *out) {
    switch (g->game) {
    case G_F2O: return f2o_kids((int64_t)k, out);
    case G_TTT: return ttt_kids(k, out);
    case G_TOOT: return toot_kids(g, k, out);
    case G_OTHELLO: return oth_kids(g, k, out);
    case G_SUBTRACT: return sub_kids(g, k, out);
    }
    return -1;
}
/* A potential strictly increasing along every move (children may skip levels). */
static int64_t g_tier(const game_t *g, uint64_t k) {
    switch (g->game) {
    case G_F2O: return -(int64_t)k;
    case G_TTT: { int c[9], n = 0; ttt_decode(k, c); for (int i = 0; i < 9; i++) n += c[i] != 0; return n; }
    case G_TOOT: { toot_t s; toot_decode(g, k, &s); return s.pieces; }
    case G_OTHELLO: {
        oth_t s; oth_decode(g, k, &s); int n = 0;
        for (int j = 0; j < g->L * g->H; j++) n += s.cell[j] != 0;
        return 3 * n + s.pass;
    }
    case G_SUBTRACT: { int64_t t = 0; for (int i = 0; i < g->L; i++) t += (k >> (4 * i)) & 15; return -t; }
    }
    return 0;
}

static int g_make(game_t *g, int game, const int32_t *params, int nparams) {
    memset(g, 0, sizeof *g);
    g->game = game;
    switch (game) {
    case G_F2O: case G_TTT: return 0;
    case G_TOOT: case G_OTHELLO:
        g->L = nparams > 0 ? params[0] : (game == G_TOOT ? 6 : 4);
        g->H = nparams > 1 ? params[1] : (game == G_TOOT ? 4 : 4);
        if (g->L < 1 || g->H < 1 || 2 * g->L * g->H + 16 > 64) {
            snprintf(g_err, sizeof g_err, "board %dx%d does not fit a 64-bit key", g->L, g->H);
            return -1;
        }
        return 0;
    case G_SUBTRACT:
        g->L = nparams > 0 ? params[0] : 8;
        if (g->L < 1 || g->L > 8) { snprintf(g_err, sizeof g_err, "heaps must be 1..8"); return -1; }
        return 0;
    }
    snprintf(g_err, sizeof g_err, "unknown game %d", game);
    return -1;
}

int oracle_initial(int game, const int32_t *params, int nparams, uint64_t *root) {
    game_t g;
    if (g_make(&g, game, params, nparams)) return -1;
    switch (game) {
    case G_F2O: *root = 4; return 0;
    case G_TTT: *root = 0; return 0;
    case G_TOOT: {
        toot_t s; memset(&s, 0, sizeof s);
        for (int p = 0; p < 2; p++) s.hand[p][0] = s.hand[p][1] = 6;
        *root = toot_encode(&g, &s);
        return 0;
    }
    case G_OTHELLO: {
        /* othello_bit_new.py:36-55: centre cells, turn 0 -> 1 -> 2 (WHITE). */
        oth_t s; memset(&s, 0, sizeof s);
        int L = g.L, H = g.H;
        s.cell[L * (H / 2 - 1) + (L / 2 - 1)] = OW;
        s.cell[L * (H / 2) + (L / 2 - 1)] = OB;
        s.cell[L * (H / 2 - 1) + (L / 2)] = OB;
        s.cell[L * (H / 2) + (L / 2)] = OW;
        s.turn = 2;
        *root = oth_encode(&g, &s);
        return 0;
    }
    case G_SUBTRACT: *root = (1ull << (4 * g.L)) - 1; return 0;
    }
    return -1;
}

int oracle_expand(int game, const int32_t *params, int nparams, uint64_t key,
                  uint64_t *children, int *nchildren, int *prim, int64_t *tier) {
    game_t g;
    if (g_make(&g, game, params, nparams)) return -1;
    *prim = g_prim(&g, key);
    *tier = g_tier(&g, key);
    *nchildren = *prim == UNDECIDED ? g_kids(&g, key, children) : 0;
    return 0;
}

/* ---------------------------------------------- open-addressing key -> record map */
typedef struct { uint64_t *keys; uint16_t *rec; uint64_t cap, n; } map_t;
/* 2^63 is no valid key: F2O keys are piles >= -1, TTT < 3^9, Othello < 2^48,
 * subtract < 2^32, and a Toot key with only the first T cell set would need all
 * hands empty.  (-1 = all ones IS a F2O key, so it cannot be the sentinel.) */
#define EMPTY_KEY 0x8000000000000000ull
static uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
static int map_init(map_t *m, uint64_t cap) {
    uint64_t c = 1024;
    while (c < cap) c <<= 1;
    m->cap = c; m->n = 0;
    m->keys = (uint64_t *)malloc(c * sizeof(uint64_t));
    m->rec = (uint16_t *)malloc(c * sizeof(uint16_t));
    if (!m->keys || !m->rec) return -1;
    for (uint64_t i = 0; i < c; i++) m->keys[i] = EMPTY_KEY;
    return 0;
}
static uint64_t map_find(const map_t *m, uint64_t k) {
    uint64_t i = mix(k) & (m->cap - 1);
    while (m->keys[i] != k) {
        if (m->keys[i] == EMPTY_KEY) return EMPTY_KEY;
        i = (i + 1) & (m->cap - 1);
    }
    return i;
}
static int map_grow(map_t *m);
static int map_insert(map_t *m, uint64_t k, int *fresh) {
    if ((m->n + 1) * 2 > m->cap && map_grow(m)) return -1;
    uint64_t i = mix(k) & (m->cap - 1);
    while (m->keys[i] != k) {
        if (m->keys[i] == EMPTY_KEY) { m->keys[i] = k; m->rec[i] = 0xFFFF; m->n++; *fresh = 1; return 0; }
        i = (i + 1) & (m->cap - 1);
    }
    *fresh = 0;
    return 0;
}
static int map_grow(map_t *m) {
    map_t nm;
    if (map_init(&nm, m->cap * 2)) return -1;
    for (uint64_t i = 0; i < m->cap; i++) {
        if (m->keys[i] == EMPTY_KEY) continue;
        uint64_t j = mix(m->keys[i]) & (nm.cap - 1);
        while (nm.keys[j] != EMPTY_KEY) j = (j + 1) & (nm.cap - 1);
        nm.keys[j] = m->keys[i]; nm.rec[j] = m->rec[i]; nm.n++;
    }
    free(m->keys); free(m->rec);
    *m = nm;
    return 0;
}

typedef struct { uint64_t *v; uint64_t n, cap; } vec_t;
static int vec_push(vec_t *a, uint64_t x) {
    if (a->n == a->cap) {
        uint64_t c = a->cap ? a->cap * 2 : 64;
        uint64_t *p = (uint64_t *)realloc(a->v, c * sizeof(uint64_t));
        if (!p) return -1;
        a->v = p; a->cap = c;
    }
    a->v[a->n++] = x;
    return 0;
}

/* Appendix A fold as a max over a preference score (see file header). */
static uint32_t pref(uint16_t rec) {
    uint32_t v = rec >> 14, r = rec & 0x3FFF;
    if (v == LOSS) return 0x30000u | (0x3FFFu - r);
    if (v == TIE) return 0x20000u | (0x3FFFu - r);
    return 0x10000u | r;  /* WIN */
}
static uint16_t from_pref(uint32_t best) {
    uint32_t cls = best >> 16, low = best & 0xFFFF;
    if (cls == 3) return (uint16_t)((WIN << 14) | (0x3FFFu - low + 1));
    if (cls == 2) return (uint16_t)((TIE << 14) | (0x3FFFu - low + 1));
    return (uint16_t)((LOSS << 14) | (low + 1));
}

static int cmp_pair(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* Strong solve from root; returns the number of positions (or -1) and hands out
 * malloc'd, key-sorted arrays (free with oracle_free). */
int64_t oracle_solve(int game, const int32_t *params, int nparams, uint64_t root,
                     uint64_t **keys_out, uint16_t **recs_out) {
    game_t g;
    if (g_make(&g, game, params, nparams)) return -1;
    map_t m;
    if (map_init(&m, 1 << 16)) { snprintf(g_err, sizeof g_err, "out of memory"); return -1; }
    int64_t t0 = g_tier(&g, root);
    vec_t *tiers = NULL;
    int64_t ntiers = 0, maxt = 0;
    uint64_t kids[MAXKIDS];
    int fresh;
    /* forward: tier by tier */
#define ENSURE_TIER(t) do { \
        if ((t) >= ntiers) { int64_t nt = ntiers ? ntiers : 16; while (nt <= (t)) nt *= 2; \
            vec_t *p = (vec_t *)realloc(tiers, nt * sizeof(vec_t)); if (!p) goto oom; \
            memset(p + ntiers, 0, (nt - ntiers) * sizeof(vec_t)); tiers = p; ntiers = nt; } } while (0)
    ENSURE_TIER(0);
    map_insert(&m, root, &fresh);
    if (vec_push(&tiers[0], root)) goto oom;
    for (int64_t t = 0; t <= maxt; t++) {
        for (uint64_t i = 0; i < tiers[t].n; i++) {
            uint64_t k = tiers[t].v[i];
            int p = g_prim(&g, k);
            if (p == DRAW) { snprintf(g_err, sizeof g_err, "DRAW primitive"); goto fail; }
            if (p != UNDECIDED) continue;
            int n = g_kids(&g, k, kids);
            if (n <= 0) { snprintf(g_err, sizeof g_err, "non-primitive position without moves"); goto fail; }
            for (int c = 0; c < n; c++) {
                int64_t tc = g_tier(&g, kids[c]) - t0;
                if (tc <= t) { snprintf(g_err, sizeof g_err, "tier not increasing along a move"); goto fail; }
                if (map_insert(&m, kids[c], &fresh)) goto oom;
                if (fresh) {
                    ENSURE_TIER(tc);
                    if (vec_push(&tiers[tc], kids[c])) goto oom;
                    if (tc > maxt) maxt = tc;
                }
            }
        }
    }
    /* backward: deepest tier first */
    for (int64_t t = maxt; t >= 0; t--) {
        for (uint64_t i = 0; i < tiers[t].n; i++) {
            uint64_t k = tiers[t].v[i];
            uint64_t slot = map_find(&m, k);
            int p = g_prim(&g, k);
            if (p != UNDECIDED) { m.rec[slot] = (uint16_t)(p << 14); continue; }
            int n = g_kids(&g, k, kids);
            uint32_t best = 0;
            for (int c = 0; c < n; c++) {
                uint16_t r = m.rec[map_find(&m, kids[c])];
                uint32_t s = pref(r);
                if (s > best) best = s;
            }
            m.rec[slot] = from_pref(best);
        }
    }
    {
        uint64_t n = m.n;
        uint64_t *pairs = (uint64_t *)malloc(n * 2 * sizeof(uint64_t));
        if (!pairs) goto oom;
        uint64_t j = 0;
        for (uint64_t i = 0; i < m.cap; i++)
            if (m.keys[i] != EMPTY_KEY) { pairs[2 * j] = m.keys[i]; pairs[2 * j + 1] = m.rec[i]; j++; }
        qsort(pairs, n, 2 * sizeof(uint64_t), cmp_pair);
        uint64_t *ko = (uint64_t *)malloc(n * sizeof(uint64_t));
        uint16_t *ro = (uint16_t *)malloc(n * sizeof(uint16_t));
        if (!ko || !ro) { free(pairs); free(ko); free(ro); goto oom; }
        for (uint64_t i = 0; i < n; i++) { ko[i] = pairs[2 * i]; ro[i] = (uint16_t)pairs[2 * i + 1]; }
        free(pairs);
        *keys_out = ko; *recs_out = ro;
        for (int64_t t = 0; t < ntiers; t++) free(tiers[t].v);
        free(tiers); free(m.keys); free(m.rec);
        return (int64_t)n;
    }
oom:
    snprintf(g_err, sizeof g_err, "out of memory");
fail:
    for (int64_t t = 0; t < ntiers; t++) free(tiers[t].v);
    free(tiers); free(m.keys); free(m.rec);
    return -1;
#undef ENSURE_TIER
}

void oracle_free(void *p) { free(p); }

/* Dense synthetic solver: every key in [0, 16^heaps) in ascending key order.
 * All children of a key are smaller keys, so one sequential sweep is a valid
 * retrograde order.  Scalar, single thread (the bench's cpu_baseline). */
int oracle_subtract_dense(int heaps, uint16_t *rec) {
    if (heaps < 1 || heaps > 8) { snprintf(g_err, sizeof g_err, "heaps must be 1..8"); return -1; }
    uint64_t n = 1ull << (4 * heaps);
    rec[0] = (uint16_t)(LOSS << 14);
    for (uint64_t k = 1; k < n; k++) {
        uint32_t best = 0;
        for (int i = 0; i < heaps; i++) {
            uint64_t h = (k >> (4 * i)) & 15;
            if (h >= 1) { uint32_t s = pref(rec[k - (1ull << (4 * i))]); if (s > best) best = s; }
            if (h >= 2) { uint32_t s = pref(rec[k - (2ull << (4 * i))]); if (s > best) best = s; }
        }
        rec[k] = from_pref(best);
    }
    return 0;
}

/* The same dense solve on `threads` OpenMP threads (<= 0: all), in the GPU's
 * decomposition: blocks of 16^low keys sharing their high nibbles, blocks grouped
 * by the sum of the high nibbles (a child block has a smaller sum), the blocks of
 * one group in parallel, each block swept in ascending key order.  The bench's
 * multi-core cpu_baseline. */
int oracle_subtract_dense_mt(int heaps, uint16_t *rec, int threads) {
    if (heaps < 1 || heaps > 8) { snprintf(g_err, sizeof g_err, "heaps must be 1..8"); return -1; }
    const int low = heaps < 3 ? heaps : 3, high = heaps - low;
    const uint64_t bsz = 1ull << (4 * low), nhigh = 1ull << (4 * high);
    uint32_t *order = (uint32_t *)malloc(nhigh * sizeof(uint32_t));
    uint64_t *off = (uint64_t *)calloc(15 * high + 2, sizeof(uint64_t));
    if (!order || !off) { free(order); free(off); snprintf(g_err, sizeof g_err, "out of memory"); return -1; }
    for (uint64_t v = 0; v < nhigh; v++) {
        int s = 0;
        for (int j = 0; j < high; j++) s += (int)((v >> (4 * j)) & 15);
        off[s + 1]++;
    }
    for (int t = 1; t < 15 * high + 2; t++) off[t] += off[t - 1];
    {
        uint64_t *pos = (uint64_t *)malloc((15 * high + 1) * sizeof(uint64_t));
        if (!pos) { free(order); free(off); snprintf(g_err, sizeof g_err, "out of memory"); return -1; }
        memcpy(pos, off, (15 * high + 1) * sizeof(uint64_t));
        for (uint64_t v = 0; v < nhigh; v++) {
            int s = 0;
            for (int j = 0; j < high; j++) s += (int)((v >> (4 * j)) & 15);
            order[pos[s]++] = (uint32_t)v;
        }
        free(pos);
    }
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    for (int t = 0; t <= 15 * high; t++) {
        const long long b0 = (long long)off[t], b1 = (long long)off[t + 1];
#pragma omp parallel for schedule(dynamic, 4)
        for (long long b = b0; b < b1; b++) {
            const uint64_t base = (uint64_t)order[b] << (4 * low);
            for (uint64_t i = 0; i < bsz; i++) {
                const uint64_t k = base + i;
                if (k == 0) { rec[0] = (uint16_t)(LOSS << 14); continue; }
                uint32_t best = 0;
                for (int j = 0; j < heaps; j++) {
                    uint64_t h = (k >> (4 * j)) & 15;
                    if (h >= 1) { uint32_t s = pref(rec[k - (1ull << (4 * j))]); if (s > best) best = s; }
                    if (h >= 2) { uint32_t s = pref(rec[k - (2ull << (4 * j))]); if (s > best) best = s; }
                }
                rec[k] = from_pref(best);
            }
        }
    }
    free(order);
    free(off);
    return 0;
}

int oracle_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static uint64_t digest_term(uint64_t key, uint16_t rec) {
    return mix(key * 0x9E3779B97F4A7C15ull + rec);   /* the gm_digest formula, include/gmsolve.h */
}

/* Digest of a dense table rec[0..n) (key = index), OpenMP.  With the dense
 * solvers above it pins the device's full 2^32 table: gm_digest of the GPU
 * solve must equal oracle_dense_digest(oracle_subtract_dense_mt(8)). */
int oracle_dense_digest(const uint16_t *rec, uint64_t n, int threads, uint64_t *digest) {
    uint64_t sum = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for reduction(+ : sum) schedule(static)
    for (long long k = 0; k < (long long)n; k++) sum += digest_term((uint64_t)k, rec[k]);
    *digest = sum;
    return 0;
}

/* The same digest restricted to whole blocks: positions hp << 4*low .. + 16^low - 1 of
 * every listed high part hp that lie inside the root's box (every nibble <= the
 * root's).  A sharded solve's rank digests its own blocks (gm_digest at N > 1), so
 * this names the rank whose part of the table differs. */
int oracle_dense_digest_blocks(const uint16_t *rec, int heaps, int low, uint64_t root, const uint32_t *blocks,
                               uint64_t nblocks, int threads, uint64_t *digest, uint64_t *count) {
    uint64_t sum = 0, cnt = 0;
    const uint64_t bsz = 1ull << (4 * low);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for reduction(+ : sum, cnt) schedule(dynamic, 64)
    for (long long b = 0; b < (long long)nblocks; b++) {
        const uint64_t base = (uint64_t)blocks[b] << (4 * low);
        for (uint64_t i = 0; i < bsz; i++) {
            const uint64_t k = base + i;
            int in = 1;
            for (int j = 0; j < heaps && in; j++) in = ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
            if (!in) continue;
            sum += digest_term(k, rec[k]);
            cnt++;
        }
    }
    *digest = sum;
    *count = cnt;
    return 0;
}

/* The same digest over the 8-heap game's BOXES (the sharded box solve's unit of
 * ownership, include/gmsolve.h gm_box_plan): box id bits 2i..2i+1 = heap i >> 2 for
 * heaps 0-3, bits 8+3j..10+3j = heap 4+j >> 1; a box holds the 4096 keys whose heaps
 * 0-3 have those high two bits and heaps 4-7 those high three bits.  Restated here from
 * that definition (not from the product's code) so a wrong rank of a sharded solve is
 * named.  Positions outside the root's region are skipped, as above. */
int oracle_dense_digest_boxes(const uint16_t *rec, uint64_t root, const uint32_t *boxes, uint64_t nboxes,
                              int threads, uint64_t *digest, uint64_t *count) {
    uint64_t sum = 0, cnt = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for reduction(+ : sum, cnt) schedule(dynamic, 64)
    for (long long b = 0; b < (long long)nboxes; b++) {
        const uint32_t id = boxes[b];
        uint64_t base = 0;
        for (int i = 0; i < 4; i++) base |= (uint64_t)(((id >> (2 * i)) & 3u) << 2) << (4 * i);
        for (int j = 0; j < 4; j++) base |= (uint64_t)(((id >> (8 + 3 * j)) & 7u) << 1) << (16 + 4 * j);
        for (uint32_t o = 0; o < 4096; o++) {
            uint64_t k = base;
            for (int i = 0; i < 4; i++) k |= (uint64_t)((o >> (2 * i)) & 3u) << (4 * i);
            for (int j = 0; j < 4; j++) k |= (uint64_t)((o >> (8 + j)) & 1u) << (16 + 4 * j);
            int in = 1;
            for (int j = 0; j < 8 && in; j++) in = ((k >> (4 * j)) & 15u) <= ((root >> (4 * j)) & 15u);
            if (!in) continue;
            sum += digest_term(k, rec[k]);
            cnt++;
        }
    }
    *digest = sum;
    *count = cnt;
    return 0;
}

/* ------------------------------------------------ layered solver (OpenMP) */
/* The same Appendix-A fixed point as oracle_solve, on a different data
 * structure so the two check each other: per tier a SORTED array of distinct
 * keys (parallel LSD radix sort + unique) instead of one hash map, children
 * found by binary search in their tier's array.  Memory ~ 10 B per position plus
 * the duplicate child keys of one tier, so Toot-and-Otto 6x4 (1.19 G positions,
 * SURVEY App. D) fits a 64 GB host: it is the full-size oracle of config 3.
 * Also the host-core CPU baseline of configs 3 and 4 in bench.py. */
#define LAYER_MAXSKIP 16

static int nthreads_now(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
static int thread_id(void) {
#ifdef _OPENMP
    return omp_get_thread_num();
#else
    return 0;
#endif
}

/* stable parallel LSD radix sort of a[0..n) on its varying bits, 11-bit digits;
 * returns the array holding the result (a or tmp) */
static uint64_t *radix_sort(uint64_t *a, uint64_t *tmp, uint64_t n) {
    if (n < 2) return a;
    uint64_t vary = 0;
    for (uint64_t i = 1; i < n; i++) vary |= a[i] ^ a[0];
    if (!vary) return a;
    int lo = __builtin_ctzll(vary), hi = 63 - __builtin_clzll(vary);
    const int T = nthreads_now(), DB = 11, NB = 1 << DB;
    uint64_t *hist = (uint64_t *)malloc((size_t)T * NB * sizeof(uint64_t));
    if (!hist) return NULL;
    for (int shift = lo; shift <= hi; shift += DB) {
        memset(hist, 0, (size_t)T * NB * sizeof(uint64_t));
#pragma omp parallel num_threads(T)
        {
            const int t = thread_id();
            const uint64_t b0 = n * (uint64_t)t / T, b1 = n * (uint64_t)(t + 1) / T;
            uint64_t *h = hist + (size_t)t * NB;
            for (uint64_t i = b0; i < b1; i++) h[(a[i] >> shift) & (NB - 1)]++;
#pragma omp barrier
#pragma omp single
            {
                uint64_t run = 0;
                for (int d = 0; d < NB; d++)
                    for (int u = 0; u < T; u++) {
                        uint64_t c = hist[(size_t)u * NB + d];
                        hist[(size_t)u * NB + d] = run;
                        run += c;
                    }
            }
            for (uint64_t i = b0; i < b1; i++) tmp[h[(a[i] >> shift) & (NB - 1)]++] = a[i];
        }
        uint64_t *s = a; a = tmp; tmp = s;
    }
    free(hist);
    return a;
}

typedef struct {
    uint64_t *keys;     /* sorted distinct keys of the tier */
    uint16_t *rec;
    uint64_t n;
    uint64_t *idx;      /* idx[p] = first key whose top bits (key - kmin) >> ishift >= p */
    int ishift;
    uint64_t kmin, np;
} layer_t;

static void layer_index(layer_t *L) {
    L->idx = NULL;
    if (L->n < 64) return;
    uint64_t span = L->keys[L->n - 1] - L->keys[0];
    int bits = 1;
    while (((uint64_t)1 << bits) < L->n / 4 && bits < 26) bits++;
    int top = 64 - __builtin_clzll(span | 1);
    L->ishift = top > bits ? top - bits : 0;
    L->kmin = L->keys[0];
    uint64_t np = (span >> L->ishift) + 2;
    L->np = np;
    L->idx = (uint64_t *)malloc(np * sizeof(uint64_t));
    if (!L->idx) return;
    uint64_t j = 0;
    for (uint64_t p = 0; p < np; p++) {
        while (j < L->n && ((L->keys[j] - L->kmin) >> L->ishift) < p) j++;
        L->idx[p] = j;
    }
}

static int64_t layer_find(const layer_t *L, uint64_t k) {
    uint64_t lo = 0, hi = L->n;
    if (L->idx) {
        if (k < L->kmin) return -1;
        uint64_t p = (k - L->kmin) >> L->ishift;
        if (p + 1 >= L->np) return -1;
        lo = L->idx[p];
        hi = L->idx[p + 1];
    }
    while (lo < hi) {
        uint64_t m = (lo + hi) >> 1;
        if (L->keys[m] < k) lo = m + 1; else hi = m;
    }
    return (lo < L->n && L->keys[lo] == k) ? (int64_t)lo : -1;
}

/* Strong solve from root on `threads` OpenMP threads (<= 0: all).  Outputs the
 * number of positions, the digest of the full table, the root's record and the
 * positions per tier (tier = descriptor potential - root's; for Toot the ply).
 * Returns 0, or -1 with oracle_last_error(). */
int oracle_solve_layered(int game, const int32_t *params, int nparams, uint64_t root, int threads,
                         uint64_t *n_positions, uint64_t *digest, uint16_t *root_record,
                         uint64_t *per_tier, int per_tier_cap, int *n_tiers) {
    game_t g;
    if (g_make(&g, game, params, nparams)) return -1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
    const int T = nthreads_now();
    const int64_t t0 = g_tier(&g, root);
    int64_t cap = 64, maxt = 0;
    layer_t *lay = (layer_t *)calloc(cap, sizeof(layer_t));
    vec_t *pend = (vec_t *)calloc(cap, sizeof(vec_t));   /* children (with duplicates) waiting per tier */
    vec_t *loc = (vec_t *)calloc((size_t)T * (LAYER_MAXSKIP + 1), sizeof(vec_t));
    int err = 0;
    if (!lay || !pend || !loc) { err = 1; goto done; }
    if (vec_push(&pend[0], root)) { err = 1; goto done; }
    /* forward: tier t's pending children -> sorted distinct keys -> their children */
    for (int64_t t = 0; t <= maxt && !err; t++) {
        vec_t *pv = &pend[t];
        uint64_t *tmp = (uint64_t *)malloc((pv->n ? pv->n : 1) * sizeof(uint64_t));
        if (!tmp) { err = 1; break; }
        uint64_t *s = pv->n ? radix_sort(pv->v, tmp, pv->n) : tmp;
        if (!s) { free(tmp); err = 1; break; }
        uint64_t m = 0;
        for (uint64_t i = 0; i < pv->n; i++)
            if (i == 0 || s[i] != s[i - 1]) s[m++] = s[i];
        /* keep the sorted buffer, free the other */
        if (s == pv->v) free(tmp); else free(pv->v);
        lay[t].keys = (uint64_t *)realloc(s, (m ? m : 1) * sizeof(uint64_t));
        lay[t].n = m;
        pv->v = NULL; pv->n = pv->cap = 0;
        lay[t].rec = (uint16_t *)malloc((m ? m : 1) * sizeof(uint16_t));
        if (!lay[t].keys || !lay[t].rec) { err = 1; break; }
        int64_t dmax = 0;
#pragma omp parallel num_threads(T) reduction(max : dmax)
        {
            const int th = thread_id();
            uint64_t kids[MAXKIDS];
            vec_t *mine = loc + (size_t)th * (LAYER_MAXSKIP + 1);
#pragma omp for schedule(dynamic, 4096)
            for (long long i = 0; i < (long long)m; i++) {
                const uint64_t k = lay[t].keys[i];
                const int p = g_prim(&g, k);
                if (p == DRAW) { dmax = 1000000; continue; }
                if (p != UNDECIDED) continue;
                const int nk = g_kids(&g, k, kids);
                if (nk <= 0) { dmax = 2000000; continue; }
                for (int c = 0; c < nk; c++) {
                    const int64_t d = g_tier(&g, kids[c]) - t0 - t;
                    if (d < 1 || d > LAYER_MAXSKIP) { dmax = 3000000; continue; }
                    if (d > dmax) dmax = d;
                    if (vec_push(&mine[d], kids[c])) dmax = 4000000;
                }
            }
        }
        if (dmax >= 1000000) {
            snprintf(g_err, sizeof g_err, "%s", dmax == 1000000 ? "DRAW primitive" : dmax == 2000000 ?
                     "non-primitive position without moves" : dmax == 3000000 ?
                     "tier not increasing along a move (or skip > 16)" : "out of memory");
            err = 2;
            break;
        }
        if (t + dmax >= cap) {
            int64_t nc = cap;
            while (t + dmax >= nc) nc *= 2;
            layer_t *nl = (layer_t *)realloc(lay, nc * sizeof(layer_t));
            if (nl) lay = nl;
            vec_t *np = (vec_t *)realloc(pend, nc * sizeof(vec_t));
            if (np) pend = np;
            if (!nl || !np) { err = 1; break; }
            memset(lay + cap, 0, (nc - cap) * sizeof(layer_t));
            memset(pend + cap, 0, (nc - cap) * sizeof(vec_t));
            cap = nc;
        }
        for (int64_t d = 1; d <= dmax; d++) {
            uint64_t add = 0;
            for (int th = 0; th < T; th++) add += loc[(size_t)th * (LAYER_MAXSKIP + 1) + d].n;
            if (!add) continue;
            vec_t *q = &pend[t + d];
            uint64_t *nv = (uint64_t *)realloc(q->v, (q->n + add) * sizeof(uint64_t));
            if (!nv) { err = 1; break; }
            q->v = nv;
            q->cap = q->n + add;
            for (int th = 0; th < T; th++) {
                vec_t *src = &loc[(size_t)th * (LAYER_MAXSKIP + 1) + d];
                memcpy(q->v + q->n, src->v, src->n * sizeof(uint64_t));
                q->n += src->n;
                src->n = 0;
            }
            if (t + d > maxt) maxt = t + d;
        }
    }
    if (err) goto done;
    for (int64_t t = 0; t <= maxt; t++) layer_index(&lay[t]);
    /* backward: deepest tier first */
    for (int64_t t = maxt; t >= 0 && !err; t--) {
        int bad = 0;
#pragma omp parallel for num_threads(T) schedule(dynamic, 4096) reduction(| : bad)
        for (long long i = 0; i < (long long)lay[t].n; i++) {
            uint64_t kids[MAXKIDS];
            const uint64_t k = lay[t].keys[i];
            const int p = g_prim(&g, k);
            if (p != UNDECIDED) { lay[t].rec[i] = (uint16_t)(p << 14); continue; }
            const int nk = g_kids(&g, k, kids);
            uint32_t best = 0;
            for (int c = 0; c < nk; c++) {
                const int64_t tc = g_tier(&g, kids[c]) - t0;
                const int64_t j = layer_find(&lay[tc], kids[c]);
                if (j < 0) { bad = 1; continue; }
                const uint32_t sc = pref(lay[tc].rec[j]);
                if (sc > best) best = sc;
            }
            lay[t].rec[i] = from_pref(best);
        }
        if (bad) { snprintf(g_err, sizeof g_err, "child missing from its tier"); err = 2; }
    }
    if (err) goto done;
    {
        uint64_t n = 0, dsum = 0;
        for (int64_t t = 0; t <= maxt; t++) {
            uint64_t s = 0;
#pragma omp parallel for num_threads(T) reduction(+ : s) schedule(static)
            for (long long i = 0; i < (long long)lay[t].n; i++) s += digest_term(lay[t].keys[i], lay[t].rec[i]);
            dsum += s;
            n += lay[t].n;
            if (per_tier && t < per_tier_cap) per_tier[t] = lay[t].n;
        }
        *n_positions = n;
        *digest = dsum;
        *root_record = lay[0].rec[0];
        if (n_tiers) *n_tiers = (int)(maxt + 1);
    }
done:
    if (err == 1) snprintf(g_err, sizeof g_err, "out of memory");
    if (lay)
        for (int64_t t = 0; t < cap; t++) { free(lay[t].keys); free(lay[t].rec); free(lay[t].idx); }
    if (pend)
        for (int64_t t = 0; t < cap; t++) free(pend[t].v);
    if (loc)
        for (int i = 0; i < T * (LAYER_MAXSKIP + 1); i++) free(loc[i].v);
    free(lay); free(pend); free(loc);
    return err ? -1 : 0;
}
