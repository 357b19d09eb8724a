// gm_api.hip -- the C ABI (include/gmsolve.h): contexts, dispatch, errors.
#include "gm_internal.hpp"

#include <chrono>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace gm {

static thread_local char g_err[512];

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

int dev_error_to_gm(uint32_t f) {
    if (f & DEV_ERR_DRAW) { set_error("a DRAW primitive was reached (unsupported)"); return GM_E_DRAW; }
    if (f & DEV_ERR_NOMOVES) { set_error("a non-primitive position has no moves"); return GM_E_NOMOVES; }
    if (f & DEV_ERR_TIER) { set_error("descriptor tier does not increase by 1..MAX_SKIP along a move"); return GM_E_GAME; }
    if (f & DEV_ERR_TABLE_FULL) { set_error("tier table overflow"); return GM_E_NOMEM; }
    if (f & DEV_ERR_MISSING_CHILD) { set_error("retrograde found a child missing from its tier table"); return GM_E_STATE; }
    if (f & DEV_ERR_OVERFLOW) { set_error("remoteness exceeds 14 bits"); return GM_E_CAP; }
    set_error("device error flags 0x%x", f);
    return GM_E_STATE;
}

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

bool trace_on() {
    static const bool on = getenv("GM_TRACE") && atoi(getenv("GM_TRACE"));
    return on;
}

// The communicator is made when a solve first needs it -- every rank's first sharded solve,
// so the call is collective as RCCL requires -- and not at all for a transport that needs none
// (the split box engine's IPC peer copies, which also run when the ranks share one GPU, where
// RCCL refuses to make a communicator).
int ensure_comm(Ctx *c) {
    if (c->comm) return GM_OK;
    if (!c->have_uid) {
        set_error("a %d-rank solve needs gm_set_comm with a unique id", c->world);
        return GM_E_COMM;
    }
    ncclUniqueId id;
    memcpy(&id, c->uid, sizeof id);
    GM_HIP(hipSetDevice(c->device));
    GM_NCCL(ncclCommInitRank(&c->comm, c->world, id, c->rank));
    return GM_OK;
}

// Best fit from the context's cache of released buffers (no more than 2x the
// request), else hipMalloc; if that fails, release the cache and retry once.
int dev_alloc(Ctx *c, void **p, uint64_t bytes) {
    bytes = std::max<uint64_t>(bytes, 256);
    size_t best = c->buf_cache.size();
    for (size_t i = 0; i < c->buf_cache.size(); i++) {
        const uint64_t sz = c->buf_cache[i].second;
        if (sz >= bytes && sz <= 2 * bytes && (best == c->buf_cache.size() || sz < c->buf_cache[best].second))
            best = i;
    }
    if (best < c->buf_cache.size()) {
        *p = c->buf_cache[best].first;
        c->buf_live.push_back(c->buf_cache[best]);
        c->buf_cache.erase(c->buf_cache.begin() + best);
        return GM_OK;
    }
    const double t0 = trace_on() ? now_ms() : 0;
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(c->stream);
        for (auto &b : c->buf_cache) (void)hipFree(b.first);
        c->buf_cache.clear();
        e = hipMalloc(p, bytes);
    }
    if (trace_on()) fprintf(stderr, "[gm] hipMalloc %.3f GB in %.2f ms\n", bytes / 1e9, now_ms() - t0);
    if (e != hipSuccess) {
        *p = nullptr;
        set_error("out of device memory (%llu bytes): %s", (unsigned long long)bytes, hipGetErrorString(e));
        return GM_E_NOMEM;
    }
    c->buf_live.emplace_back(*p, bytes);
    return GM_OK;
}

// Return a buffer to the cache: a fresh multi-GB hipMalloc after a hipFree can
// stall for seconds (measured: 8.6 GB in 4.9 s on the second Toot 6x4 solve),
// so repeated solves reuse the previous solve's buffers instead.
void dev_free(Ctx *c, void *p) {
    if (!p) return;
    for (size_t i = 0; i < c->buf_live.size(); i++)
        if (c->buf_live[i].first == p) {
            c->buf_cache.push_back(c->buf_live[i]);
            c->buf_live.erase(c->buf_live.begin() + i);
            return;
        }
    (void)hipFree(p);   // not ours: plain free
}

static int engine_for(const Ctx *c) {
    if (c->engine_opt == GM_ENGINE_SPARSE) return GM_ENGINE_SPARSE;
    if (c->engine_opt == GM_ENGINE_DENSE) {
        if (c->game == GM_GAME_SUBTRACT || c->game == GM_GAME_TTT) return GM_ENGINE_DENSE;
        return GM_ENGINE_SPARSE;
    }
    return (c->game == GM_GAME_SUBTRACT || c->game == GM_GAME_TTT) ? GM_ENGINE_DENSE : GM_ENGINE_SPARSE;
}

static bool key_valid(const Ctx *c, uint64_t k) {
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: return c->f2o.valid(k);
    case GM_GAME_TTT: return c->ttt.valid(k);
    case GM_GAME_TOOT: return c->toot.valid(k);
    case GM_GAME_OTHELLO: return c->oth.valid(k);
    case GM_GAME_SUBTRACT: return c->sub.valid(k);
    }
    return false;
}

static void free_engines(Ctx *c) {
    graph_free(c);
    dense_sub_free(c);
    dense_box_free(c);
    small_dense_free(c);
    sparse_free(c);
    dist_sub_free(c);
    dist_box_free(c);
    dist_sparse_free(c);
}

}  // namespace gm

using namespace gm;

extern "C" {

static int need_solved(gm_ctx *h);

int gm_version(void) { return GM_ABI_VERSION; }

const char *gm_last_error(void) { return g_err; }

int gm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int gm_open(int game, const int32_t *params, int nparams, int device, gm_ctx **out) {
    if (!out) { set_error("out is NULL"); return GM_E_ARG; }
    *out = nullptr;
    if (nparams < 0 || nparams > 4 || (nparams && !params)) { set_error("bad params"); return GM_E_ARG; }
    gm_ctx *h = new gm_ctx();
    Ctx *c = &h->c;
    c->game = game;
    for (int i = 0; i < nparams; i++) c->params[i] = params[i];
    bool ok = true;
    switch (game) {
    case GM_GAME_FOUR_TO_ONE: case GM_GAME_TTT: case GM_GAME_GRAPH: break;
    case GM_GAME_TOOT:
        ok = DescToot::make(nparams > 0 ? params[0] : 6, nparams > 1 ? params[1] : 4, &c->toot);
        break;
    case GM_GAME_OTHELLO:
        // 8x8 (the reference plugin's default board, othello_bit_new.py:8): 128-bit keys
        c->wide = nparams > 1 && params[0] == 8 && params[1] == 8;
        ok = c->wide || DescOthello::make(nparams > 0 ? params[0] : 4, nparams > 1 ? params[1] : 4, &c->oth);
        break;
    case GM_GAME_SUBTRACT:
        c->sub.heaps = nparams > 0 ? params[0] : 8;
        ok = c->sub.heaps >= 1 && c->sub.heaps <= 8;
        break;
    default:
        ok = false;
    }
    if (!ok) {
        set_error("game %d with these parameters is not supported", game);
        delete h;
        return GM_E_GAME;
    }
    int ndev = gm_device_count();
    if (ndev <= 0) {
        // Contexts can still be used for gm_pack_initial / gm_expand_host.
        c->device = -1;
        *out = h;
        return GM_OK;
    }
    if (device < 0) {
        if (hipGetDevice(&c->device) != hipSuccess) c->device = 0;
    } else {
        if (device >= ndev) { set_error("device %d out of range (%d visible)", device, ndev); delete h; return GM_E_ARG; }
        c->device = device;
    }
    if (hipSetDevice(c->device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("cannot initialise HIP device %d", c->device);
        delete h;
        return GM_E_HIP;
    }
    c->stream = c->own_stream;
    *out = h;
    return GM_OK;
}

int gm_set_stream(gm_ctx *h, void *s) {
    if (!h) return GM_E_ARG;
    h->c.stream = s ? (hipStream_t)s : h->c.own_stream;
    return GM_OK;
}

int gm_set_option(gm_ctx *h, int opt, int64_t v) {
    if (!h) return GM_E_ARG;
    Ctx *c = &h->c;
    switch (opt) {
    case GM_OPT_ENGINE:
        if (v < GM_ENGINE_AUTO || (v > GM_ENGINE_SPARSE && v != GM_ENGINE_DIST_SPARSE)) {
            set_error("bad engine");
            return GM_E_ARG;
        }
        c->engine_opt = (int)v;
        return GM_OK;
    case GM_OPT_SUB_LOW:
        if (v < 1 || v > 3) { set_error("sub_low must be 1..3"); return GM_E_ARG; }
        c->sub_low = (int)v;
        return GM_OK;
    case GM_OPT_GRAPH: c->use_graph = v != 0; return GM_OK;
    case GM_OPT_TIMING:
        if (v < 0 || v > 2) { set_error("timing must be 0, 1 or 2"); return GM_E_ARG; }
        c->timing = (int)v;
        return GM_OK;
    case GM_OPT_SUB_THREADS:
        if (v != 64 && v != 128 && v != 256) { set_error("sub_threads must be 64, 128 or 256"); return GM_E_ARG; }
        c->sub_threads = (int)v;
        return GM_OK;
    case GM_OPT_SUB_INTERLEAVE:
        if (v != 1 && v != 6 && v != 10 && v != 20) {
            set_error("sub_interleave must be 1 (one block per workgroup), 6 (four-block kernel), 10 (walker) "
                      "or 20 (box engine, 8 heaps)");
            return GM_E_ARG;
        }
        c->sub_interleave = (int)v;
        return GM_OK;
    case GM_OPT_SUB_ORDER:
        if (v < 0 || v > 2) { set_error("sub_order must be 0, 1 or 2"); return GM_E_ARG; }
        c->sub_order = (int)v;
        return GM_OK;
    case GM_OPT_DIST_BATCH:
        if (v < 1 || v > 128) { set_error("dist_batch must be 1..128"); return GM_E_ARG; }
        c->dist_batch = (int)v;
        return GM_OK;
    case GM_OPT_DIST_SLOTS:
        if (v < 1 || v > 128) { set_error("dist_slots must be 1..128"); return GM_E_ARG; }
        c->dist_slots = (int)v;
        return GM_OK;
    case GM_OPT_DIST_SYMMETRY:
        if (v < 0 || v > 1) { set_error("dist_symmetry must be 0 or 1"); return GM_E_ARG; }
        c->dist_symmetry = (int)v;
        return GM_OK;
    case GM_OPT_DIST_OWNER:
        if (v < 0 || v > 1) { set_error("dist_owner must be 0 or 1"); return GM_E_ARG; }
        c->dist_owner = (int)v;
        return GM_OK;
    case GM_OPT_DIST_SOLO:
        if (v < 0 || v > 64) { set_error("dist_solo must be 0..64"); return GM_E_ARG; }
        c->dist_solo = (int)v;
        return GM_OK;
    case GM_OPT_BOX_FLOW:
        if (v < -1 || v > 1) { set_error("box flow must be -1, 0 or 1"); return GM_E_ARG; }
        c->box_flow = (int)v;
        c->box_flow_failed = false;   // setting it again retries the dataflow launch
        return GM_OK;
    case GM_OPT_BOX_TRANSPORT:
        if (v < 0 || v > 1) { set_error("GM_OPT_BOX_TRANSPORT must be 0 (RCCL) or 1 (IPC peer copies)"); return GM_E_ARG; }
        c->box_transport = (int)v;
        return GM_OK;
    case GM_OPT_SPARSE_TRANSPORT:
        if (v < 0 || v > 1) { set_error("GM_OPT_SPARSE_TRANSPORT must be 0 (RCCL) or 1 (IPC pulls)"); return GM_E_ARG; }
        c->sparse_transport = (int)v;
        return GM_OK;
    case GM_OPT_POISON:
        if (v < 0 || v > 3) { set_error("GM_OPT_POISON must be 0..3"); return GM_E_ARG; }
        c->poison = (int)v;
        return GM_OK;
    case GM_OPT_BOX_SPLIT:
        if (v < 0 || v > 1) { set_error("box split must be 0 (halves) or 1 (comparisons)"); return GM_E_ARG; }
        c->box_split = (int)v;
        return GM_OK;
    case GM_OPT_SYMMETRY:
        if (v < 0 || v > 1) { set_error("symmetry must be 0 or 1"); return GM_E_ARG; }
        c->symmetry = (int)v;
        return GM_OK;
    case GM_OPT_VIRTUAL_RANKS:
        if (v < 1 || v > 64) { set_error("virtual ranks must be 1..64"); return GM_E_ARG; }
        c->virtual_ranks = (int)v;
        return GM_OK;
    }
    set_error("unknown option %d", opt);
    return GM_E_ARG;
}

int gm_pack_initial(gm_ctx *h, uint64_t *key) {
    if (!h || !key) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->wide) { set_error("this game's keys have %d words: gm_pack_initial_key", gm_key_words(h)); return GM_E_ARG; }
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: *key = 4; return GM_OK;   // four_to_one.py:8-10
    case GM_GAME_TTT: *key = 0; return GM_OK;           // empty board
    case GM_GAME_TOOT: *key = 0x6666; return GM_OK;     // empty planes, hands 6/6/6/6 (:36-44)
    case GM_GAME_OTHELLO: {                              // othello_bit_new.py:36-55
        const DescOthello &o = c->oth;
        int L = o.L, A = o.A;
        auto bit = [&](int x, int y) { return 1u << (A - 1 - (L * y + x)); };   // rotated plane bit
        uint32_t w = bit(L / 2 - 1, L / 2 - 1) | bit(L / 2, L / 2);
        uint32_t b = bit(L / 2 - 1, L / 2) | bit(L / 2, L / 2 - 1);
        *key = ((uint64_t)w << (A + 16)) | ((uint64_t)b << 16) | (2ull << 8);
        return GM_OK;
    }
    case GM_GAME_SUBTRACT: *key = (1ull << (4 * c->sub.heaps)) - 1; return GM_OK;
    }
    return GM_E_GAME;
}

int gm_expand_host(gm_ctx *h, uint64_t key, uint64_t *children, int cap, int *n, int *prim, int64_t *tier) {
    if (!h || !n || !prim || !tier) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->wide) { set_error("this game's keys have %d words: gm_expand_host_key", gm_key_words(h)); return GM_E_ARG; }
    uint64_t kids[32];
    int p = UNDECIDED, k = 0;
    int64_t t = 0;
    if (!key_valid(c, key)) { set_error("key is not a valid position"); return GM_E_KEY; }
    switch (c->game) {
    case GM_GAME_FOUR_TO_ONE: p = c->f2o.primitive(key); t = c->f2o.tier(key); if (p == UNDECIDED) k = c->f2o.children(key, kids); break;
    case GM_GAME_TTT: p = c->ttt.primitive(key); t = c->ttt.tier(key); if (p == UNDECIDED) k = c->ttt.children(key, kids); break;
    case GM_GAME_TOOT: {   // the plugin's own moves: no symmetry reduction
        DescToot d = c->toot;
        d.sym = 0;
        p = d.primitive(key); t = d.tier(key); if (p == UNDECIDED) k = d.children(key, kids);
        break;
    }
    case GM_GAME_OTHELLO: {   // the plugin's own moves: no symmetry reduction
        DescOthello d = c->oth;
        d.sym = 0;
        p = d.primitive(key); t = d.tier(key); if (p == UNDECIDED) k = d.children(key, kids);
        break;
    }
    case GM_GAME_SUBTRACT: p = c->sub.primitive(key); t = c->sub.tier(key); if (p == UNDECIDED) k = c->sub.children(key, kids); break;
    default: return GM_E_GAME;
    }
    *prim = p;
    *tier = t;
    *n = k;
    if (k > cap) { set_error("children buffer holds %d, need %d", cap, k); return GM_E_CAP; }
    if (children)
        for (int i = 0; i < k; i++) children[i] = kids[i];
    return GM_OK;
}

int gm_comm_unique_id(void *uid, int bytes) {
    if (!uid || bytes < (int)sizeof(ncclUniqueId)) { set_error("uid buffer must hold %d bytes", (int)sizeof(ncclUniqueId)); return GM_E_ARG; }
    ncclUniqueId id;
    GM_NCCL(ncclGetUniqueId(&id));
    memcpy(uid, &id, sizeof id);
    return GM_OK;
}

int gm_set_comm(gm_ctx *h, int rank, int world, const void *uid, int bytes) {
    if (!h || world < 1 || rank < 0 || rank >= world) { set_error("bad rank/world"); return GM_E_ARG; }
    Ctx *c = &h->c;
    // the sharded engines' transports (per-axis communicators split from c->comm, IPC
    // mappings) belong to the previous communicator: torn down first (dist_box_free
    // synchronises the device and destroys the split communicators), then the parent
    if (c->dist_box) dist_box_free(c);
    if (c->dist_sub) dist_sub_free(c);
    if (c->dist_sp) dist_sparse_free(c);
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    c->rank = rank;
    c->world = world;
    c->have_uid = false;
    // no uid: rank and world only; the sharded engines refuse to solve without one (gm_solve)
    if (!uid || bytes <= 0) return GM_OK;
    if (bytes < (int)sizeof(ncclUniqueId)) { set_error("uid must hold %d bytes", (int)sizeof(ncclUniqueId)); return GM_E_ARG; }
    if (c->device < 0) { set_error("no HIP device"); return GM_E_HIP; }
    static_assert(sizeof(ncclUniqueId) <= sizeof(c->uid), "unique id size");
    memcpy(c->uid, uid, sizeof(ncclUniqueId));
    c->have_uid = true;
    return GM_OK;
}

int gm_solve(gm_ctx *h, uint64_t root, uint64_t *n_positions, uint16_t *root_record) {
    if (!h) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->wide) { set_error("this game's keys have %d words: gm_solve_key", gm_key_words(h)); return GM_E_ARG; }
    if (c->game == GM_GAME_GRAPH) { set_error("a GM_GAME_GRAPH context is solved with gm_solve_graph"); return GM_E_GAME; }
    if (c->device < 0) { set_error("no HIP device is visible: the solver needs an MI355X (gfx950)"); return GM_E_HIP; }
    if (!key_valid(c, root)) { set_error("root key 0x%llx is not a valid position", (unsigned long long)root); return GM_E_KEY; }
    GM_HIP(hipSetDevice(c->device));
    c->solved = false;
    int32_t launches = c->stats.kernel_launches;
    c->stats = gm_stats_t{};
    c->stats.kernel_launches = c->timing ? launches : 0;
    c->stats.world = c->world;
    c->root = root;
    // symmetry reduction (games.hpp): Toot-and-Otto's mirror, when the root is its own mirror image;
    if (c->game == GM_GAME_TOOT) c->toot.sym = (c->symmetry && c->toot.mirror(root) == root) ? 1u : 0u;
    // Othello: the board symmetries that fix the root (games.hpp DescOthello::sym)
    if (c->game == GM_GAME_OTHELLO) c->oth.sym = c->symmetry ? c->oth.stabilizer(root) : 0u;
    int eng = engine_for(c);
    // GM_ENGINE_DIST_SPARSE forces the hash-sharded engine, e.g. over a one-rank communicator
    const bool force_dist_sparse = c->engine_opt == GM_ENGINE_DIST_SPARSE;
    bool sharded = c->world > 1 || c->virtual_ranks > 1 || force_dist_sparse;
    if (sharded && c->world > 1 && c->virtual_ranks > 1) {
        set_error("virtual ranks and a multi-process communicator are exclusive");
        return GM_E_ARG;
    }
    // the 8-heap game on the box engine splits inside dense_box.hip (dist_box.hip); other
    // heap counts and GM_OPT_SUB_INTERLEAVE != 20 keep the block engine's sharded path
    const bool box = !force_dist_sparse && eng == GM_ENGINE_DENSE && c->game == GM_GAME_SUBTRACT &&
                     c->sub.heaps == 8 && c->sub_interleave == 20;
    // transports that need no communicator: the split box engine's IPC stores and the sparse
    // engine's IPC pulls (both also run with the ranks sharing one GPU, where RCCL refuses)
    const bool dense_sharded = !force_dist_sparse && eng == GM_ENGINE_DENSE && c->game == GM_GAME_SUBTRACT;
    const bool no_comm = box ? c->box_transport == 1 : (!dense_sharded && c->sparse_transport == 1);
    if (sharded && c->virtual_ranks <= 1 && (c->world > 1 || force_dist_sparse) && no_comm && !c->have_uid) {
        set_error("the IPC transport needs gm_set_comm with a unique id (it names the rendezvous)");
        return GM_E_COMM;
    }
    if (sharded && c->virtual_ranks <= 1 && (c->world > 1 || force_dist_sparse) && !no_comm) {
        if (!c->have_uid) {
            set_error("a %d-rank solve of this game needs an RCCL communicator (gm_set_comm with a unique id)", c->world);
            return GM_E_COMM;
        }
        GM_TRY(ensure_comm(c));
    }
    if (sharded && !box) eng = dense_sharded ? GM_ENGINE_DIST_DENSE : GM_ENGINE_DIST_SPARSE;
    int rc;
    switch (eng) {
    case GM_ENGINE_DENSE:
        rc = c->game == GM_GAME_SUBTRACT ? dense_sub_solve(c, root) : small_dense_solve(c, root);
        break;
    case GM_ENGINE_DIST_DENSE: rc = dist_sub_solve(c, root); break;
    case GM_ENGINE_DIST_SPARSE: rc = dist_sparse_solve(c, root); break;
    default: rc = sparse_solve(c, root);
    }
    if (rc != GM_OK) return rc;
    if (!c->stats.n_stored) c->stats.n_stored = c->stats.n_positions;   // engines without a symmetry reduction
    c->engine = eng;
    c->stats.engine = (box && sharded) ? GM_ENGINE_DIST_DENSE : eng;
    c->stats.world = sharded ? (c->world > 1 ? c->world : c->virtual_ranks) : 1;
    c->solved = true;
    if (n_positions) *n_positions = c->n_positions;
    if (root_record) *root_record = c->root_record;
    return GM_OK;
}

// ---------------------------------------------------------------- multi-word keys
static constexpr int WIDE_WORDS = 3;   // Othello 8x8: the 144-bit position string (games.hpp DescOthello8)

int gm_key_words(gm_ctx *h) {
    if (!h) return GM_E_ARG;
    return h->c.wide ? WIDE_WORDS : 1;
}

int gm_pack_initial_key(gm_ctx *h, uint64_t *words) {
    if (!h || !words) return GM_E_ARG;
    if (!h->c.wide) return gm_pack_initial(h, words);
    // othello_bit_new.py:36-55: white (3,3) (4,4), black (3,4) (4,3), turn 2, no pass
    auto bit = [](int x, int y) { return 1ull << (63 - (8 * y + x)); };
    const uint64_t w = bit(3, 3) | bit(4, 4), b = bit(3, 4) | bit(4, 3);
    DescOthello8::to_words(DescOthello8::pack(w, b, 2, 0), words);
    return GM_OK;
}

int gm_expand_host_key(gm_ctx *h, const uint64_t *words, uint64_t *children, int cap, int *n, int *prim,
                       int64_t *tier) {
    if (!h || !words || !n || !prim || !tier) return GM_E_ARG;
    Ctx *c = &h->c;
    if (!c->wide) return gm_expand_host(h, words[0], children, cap, n, prim, tier);
    K128 k;
    if (!DescOthello8::from_words(words, &k)) { set_error("key is not a valid position"); return GM_E_KEY; }
    K128 kids[64];
    const DescOthello8 &d = c->oth8;
    *prim = d.primitive(k);
    *tier = d.tier(k);
    *n = *prim == UNDECIDED ? d.children(k, kids) : 0;
    if (*n > cap) { set_error("children buffer holds %d, need %d", cap, *n); return GM_E_CAP; }
    if (children)
        for (int i = 0; i < *n; i++) DescOthello8::to_words(kids[i], children + (size_t)WIDE_WORDS * i);
    return GM_OK;
}

int gm_solve_key(gm_ctx *h, const uint64_t *words, uint64_t *n_positions, uint16_t *root_record) {
    if (!h || !words) return GM_E_ARG;
    Ctx *c = &h->c;
    if (!c->wide) return gm_solve(h, words[0], n_positions, root_record);
    if (c->device < 0) { set_error("no HIP device is visible: the solver needs an MI355X (gfx950)"); return GM_E_HIP; }
    K128 root;
    if (!DescOthello8::from_words(words, &root)) {
        set_error("root key is not a valid position (an 8x8 Othello position keeps its four centre squares)");
        return GM_E_KEY;
    }
    GM_HIP(hipSetDevice(c->device));
    c->solved = false;
    c->stats = gm_stats_t{};
    if (c->world > 1 && c->virtual_ranks > 1) {
        set_error("virtual ranks and a multi-process communicator are exclusive");
        return GM_E_ARG;
    }
    // the hash-sharded sparse engine is this game's engine: one GPU (G = 1), virtual ranks, or
    // one process per rank over RCCL / the IPC transport
    if (c->virtual_ranks <= 1 && (c->world > 1 || c->have_uid)) {
        if (!c->have_uid) { set_error("a %d-rank solve needs gm_set_comm with a unique id", c->world); return GM_E_COMM; }
        if (c->sparse_transport != 1) GM_TRY(ensure_comm(c));
    }
    GM_TRY(dist_sparse_solve_wide(c, root));
    if (!c->stats.n_stored) c->stats.n_stored = c->stats.n_positions;
    c->engine = GM_ENGINE_DIST_SPARSE;
    c->stats.engine = GM_ENGINE_DIST_SPARSE;
    c->stats.world = c->world > 1 ? c->world : std::max(1, c->virtual_ranks);
    c->solved = true;
    if (n_positions) *n_positions = c->n_positions;
    if (root_record) *root_record = c->root_record;
    return GM_OK;
}

int gm_export_key(gm_ctx *h, uint64_t *words, uint16_t *recs, uint64_t cap, uint64_t *n) {
    GM_TRY(need_solved(h));
    if (!n || (words && !recs)) return GM_E_ARG;
    Ctx *c = &h->c;
    if (!c->wide) return gm_export(h, words, recs, cap, n);
    GM_HIP(hipSetDevice(c->device));
    GM_TRY(dist_sparse_export_wide(c, nullptr, nullptr, 0, n));
    if (!words) return GM_OK;
    if (cap < *n) { set_error("export buffer too small"); return GM_E_CAP; }
    std::vector<K128> k(*n);
    std::vector<uint16_t> r(*n);
    GM_TRY(dist_sparse_export_wide(c, k.data(), r.data(), *n, n));
    std::vector<uint64_t> w((size_t)WIDE_WORDS * *n);
    for (uint64_t i = 0; i < *n; i++) DescOthello8::to_words(k[i], &w[(size_t)WIDE_WORDS * i]);
    // sorted by the key's integer value (most significant word first)
    std::vector<uint64_t> idx(*n);
    for (uint64_t i = 0; i < *n; i++) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](uint64_t a, uint64_t b) {
        for (int j = WIDE_WORDS - 1; j >= 0; j--) {
            const uint64_t x = w[(size_t)WIDE_WORDS * a + j], y = w[(size_t)WIDE_WORDS * b + j];
            if (x != y) return x < y;
        }
        return false;
    });
    for (uint64_t i = 0; i < *n; i++) {
        for (int j = 0; j < WIDE_WORDS; j++) words[(size_t)WIDE_WORDS * i + j] = w[(size_t)WIDE_WORDS * idx[i] + j];
        recs[i] = r[idx[i]];
    }
    return GM_OK;
}

int gm_query_key(gm_ctx *h, const uint64_t *words, uint16_t *recs, uint64_t n) {
    GM_TRY(need_solved(h));
    if (n && (!words || !recs)) return GM_E_ARG;
    Ctx *c = &h->c;
    if (!c->wide) return gm_query(h, words, recs, n);
    GM_HIP(hipSetDevice(c->device));
    std::vector<K128> k(n);
    std::vector<uint8_t> ok(n);
    for (uint64_t i = 0; i < n; i++) {
        ok[i] = DescOthello8::from_words(words + (size_t)WIDE_WORDS * i, &k[i]);
        if (!ok[i]) k[i] = K128{0, 0};   // no valid key: answers 0xFFFF below
    }
    GM_TRY(dist_sparse_query_wide(c, k.data(), recs, n));
    for (uint64_t i = 0; i < n; i++)
        if (!ok[i]) recs[i] = REC_UNSOLVED;
    return GM_OK;
}

int gm_solve_graph(gm_ctx *h, uint64_t n, const uint8_t *prim, const uint64_t *off, const uint32_t *kid,
                   uint16_t *root_record) {
    if (!h || !prim || !off || (off[n] && !kid)) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->game != GM_GAME_GRAPH) { set_error("gm_solve_graph needs a GM_GAME_GRAPH context"); return GM_E_GAME; }
    if (c->device < 0) { set_error("no HIP device is visible: the solver needs an MI355X (gfx950)"); return GM_E_HIP; }
    if (n >= (1ull << 32)) { set_error("graphs are limited to 2^32 - 1 positions"); return GM_E_ARG; }
    for (uint64_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) { set_error("child_off is not monotone at %llu", (unsigned long long)i); return GM_E_ARG; }
    GM_HIP(hipSetDevice(c->device));
    c->solved = false;
    c->stats = gm_stats_t{};
    c->stats.world = 1;
    GM_TRY(graph_solve(c, n, prim, off, kid));
    c->engine = GM_ENGINE_GRAPH;
    c->stats.engine = GM_ENGINE_GRAPH;
    c->solved = true;
    if (root_record) *root_record = c->root_record;
    return GM_OK;
}

static int need_solved(gm_ctx *h) {
    if (!h) return GM_E_ARG;
    if (!h->c.solved) { set_error("call gm_solve first"); return GM_E_STATE; }
    return GM_OK;
}

int gm_export(gm_ctx *h, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    GM_TRY(need_solved(h));
    if (!n || (keys && !recs)) return GM_E_ARG;
    Ctx *c = &h->c;
    GM_HIP(hipSetDevice(c->device));
    if (c->engine == GM_ENGINE_GRAPH) return graph_export(c, keys, recs, cap, n);
    if (c->engine == GM_ENGINE_DENSE)
        return c->game == GM_GAME_SUBTRACT ? dense_sub_export(c, keys, recs, cap, n)
                                           : small_dense_export(c, keys, recs, cap, n);
    if (c->engine == GM_ENGINE_DIST_DENSE) return dist_sub_export(c, keys, recs, cap, n);
    if (c->engine == GM_ENGINE_DIST_SPARSE) return dist_sparse_export(c, keys, recs, cap, n);
    return sparse_export(c, keys, recs, cap, n);
}

int gm_query(gm_ctx *h, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    GM_TRY(need_solved(h));
    if (n && (!keys || !recs)) return GM_E_ARG;
    Ctx *c = &h->c;
    GM_HIP(hipSetDevice(c->device));
    if (c->engine == GM_ENGINE_GRAPH) return graph_query(c, keys, recs, n);
    if (c->engine == GM_ENGINE_DENSE)
        return c->game == GM_GAME_SUBTRACT ? dense_sub_query(c, keys, recs, n) : small_dense_query(c, keys, recs, n);
    if (c->engine == GM_ENGINE_DIST_DENSE) return dist_sub_query(c, keys, recs, n);
    if (c->engine == GM_ENGINE_DIST_SPARSE) return dist_sparse_query(c, keys, recs, n);
    return sparse_query(c, keys, recs, n);
}

int gm_digest(gm_ctx *h, uint64_t *digest, uint64_t *n) {
    GM_TRY(need_solved(h));
    if (!digest || !n) return GM_E_ARG;
    Ctx *c = &h->c;
    GM_HIP(hipSetDevice(c->device));
    if (c->engine == GM_ENGINE_GRAPH) return graph_digest(c, digest, n);
    if (c->engine == GM_ENGINE_DENSE)
        return c->game == GM_GAME_SUBTRACT ? dense_sub_digest(c, digest, n) : small_dense_digest(c, digest, n);
    if (c->engine == GM_ENGINE_DIST_DENSE) return dist_sub_digest(c, digest, n);
    if (c->engine == GM_ENGINE_DIST_SPARSE) return dist_sparse_digest(c, digest, n);
    return sparse_digest(c, digest, n);
}

int gm_stats(gm_ctx *h, gm_stats_t *out) {
    if (!h || !out) return GM_E_ARG;
    *out = h->c.stats;
    return GM_OK;
}

int gm_tier_counts(gm_ctx *h, uint64_t *counts, int cap, int *n) {
    GM_TRY(need_solved(h));
    if (!n) return GM_E_ARG;
    Ctx *c = &h->c;
    *n = (int)c->tier_counts.size();
    if (!counts) return GM_OK;
    if (cap < *n) { set_error("tier buffer too small"); return GM_E_CAP; }
    for (int i = 0; i < *n; i++) counts[i] = c->tier_counts[i];
    return GM_OK;
}

int gm_adopt_buffer(gm_ctx *h, int role, void *p, uint64_t bytes) {
    if (!h || !p) return GM_E_ARG;
    if (role != GM_BUF_DENSE_TABLE) { set_error("unknown buffer role %d", role); return GM_E_ARG; }
    h->c.adopted_dense = p;
    h->c.adopted_dense_bytes = bytes;
    return GM_OK;
}

int gm_dense_table(gm_ctx *h, void **p, uint64_t *bytes) {
    GM_TRY(need_solved(h));
    if (!p || !bytes) return GM_E_ARG;
    if (h->c.engine != GM_ENGINE_DENSE || h->c.game != GM_GAME_SUBTRACT) {
        set_error("only the SUBTRACT dense path has a dense table");
        return GM_E_STATE;
    }
    return dense_sub_table(&h->c, p, bytes);
}

int gm_dist_plan(int heaps, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *off,
                 uint64_t off_cap, uint64_t *n_off, uint32_t *data, uint64_t data_cap, uint64_t *n_data) {
    return dist_sub_plan(heaps, world, rank, opts, what, axis, off, off_cap, n_off, data, data_cap, n_data);
}

int gm_box_plan(uint64_t root, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *out,
                uint64_t cap, uint64_t *n) {
    if (!n) return GM_E_ARG;
    return dist_box_plan(root, world, rank, opts, what, axis, out, cap, n);
}

int gm_sparse_layout(int world, int steps, const uint64_t *counts, int rank, uint64_t *seg, uint64_t *send_off,
                     uint64_t *recv_off, uint64_t *recv_seg) {
    return dist_sparse_layout(world, steps, counts, rank, seg, send_off, recv_off, recv_seg);
}

int gm_rank_stats(gm_ctx *h, double *kernel_ms, uint64_t *boxes, uint64_t *recv_bytes, int cap, int *n) {
    GM_TRY(need_solved(h));
    if (!n) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->engine != GM_ENGINE_DENSE || !c->dbox_active || !c->dist_box) { *n = 0; return GM_OK; }
    return dist_box_rank_stats(c, kernel_ms, boxes, recv_bytes, cap, n);
}

int gm_rank_op_ms(gm_ctx *h, int rank, double *ms, int cap, int *n) {
    GM_TRY(need_solved(h));
    if (!n) return GM_E_ARG;
    Ctx *c = &h->c;
    if (c->engine != GM_ENGINE_DENSE || !c->dbox_active || !c->dist_box) { *n = 0; return GM_OK; }
    return dist_box_op_ms(c, rank, ms, cap, n);
}

void gm_close(gm_ctx *h) {
    if (!h) return;
    Ctx *c = &h->c;
    if (c->device >= 0) hipSetDevice(c->device);
    free_engines(c);
    if (c->device >= 0) (void)hipDeviceSynchronize();
    for (auto &b : c->buf_cache) (void)hipFree(b.first);
    for (auto &b : c->buf_live) (void)hipFree(b.first);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->own_stream) hipStreamDestroy(c->own_stream);
    if (c->comm_stream) hipStreamDestroy(c->comm_stream);
    delete h;
}

}  // extern "C"
