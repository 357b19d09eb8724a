// gm_internal.hpp -- context and helpers shared by the libgmsolve translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdarg.h>
#include <stdio.h>
#include <string>
#include <vector>

#include "../../include/gmsolve.h"
#include "games.hpp"

namespace gm {

void set_error(const char *fmt, ...);

#define GM_HIP(expr)                                                              \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess) {                                                   \
            ::gm::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                            __FILE__, __LINE__);                                  \
            return GM_E_HIP;                                                      \
        }                                                                         \
    } while (0)

#define GM_TRY(expr)            \
    do {                        \
        int r_ = (expr);        \
        if (r_ != GM_OK) return r_; \
    } while (0)

#define GM_NCCL(expr)                                                              \
    do {                                                                           \
        ncclResult_t r_ = (expr);                                                  \
        if (r_ != ncclSuccess) {                                                   \
            ::gm::set_error("%s failed: %s", #expr, ncclGetErrorString(r_));       \
            return GM_E_COMM;                                                      \
        }                                                                          \
    } while (0)

// Device error flags written by kernels (bitwise OR).
enum : uint32_t {
    DEV_ERR_DRAW = 1,
    DEV_ERR_NOMOVES = 2,
    DEV_ERR_TABLE_FULL = 4,
    DEV_ERR_MISSING_CHILD = 8,
    DEV_ERR_OVERFLOW = 16,
    DEV_ERR_TIER = 32
};

int dev_error_to_gm(uint32_t flags);

struct DenseSub;
struct DenseBox;
struct SmallDense;
struct Sparse;
struct DistSub;
struct DistBox;
struct DistSparse;
struct Graph;

struct Ctx {
    int game = 0;
    int device = 0;
    int32_t params[4] = {0, 0, 0, 0};
    DescF2O f2o;
    DescTTT ttt;
    DescToot toot;
    DescOthello oth;
    DescSub sub;
    DescOthello8 oth8;       // GM_GAME_OTHELLO at 8x8: 128-bit keys (wide)
    bool wide = false;       // keys of more than 64 bits: gm_*_key entry points, the sharded sparse engine

    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    int engine_opt = GM_ENGINE_AUTO;
    int sub_low = 3;
    int sub_threads = 128;
    int sub_interleave = 20;     // 20 box engine at 8 heaps, else the walker (default); 10 walker, 6 four-block, 13 row dataflow, 1 one block
    int sub_order = 2;   // block order inside a tier: 0 key, 1 Morton, 2 Hilbert (default)
    bool use_graph = true;
    int timing = 0;          // 1: event pair around the dominant kernel's launches; 2 (split box engine) also per op

    // multi-GPU
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;   // made on first use from uid (ensure_comm): a transport that needs none never makes it
    bool have_uid = false;
    unsigned char uid[128] = {};
    int box_transport = 0;       // split box engine across processes: 0 RCCL, 1 peer copies over IPC (GM_OPT_BOX_TRANSPORT)
    int box_prepares = 0;        // split box contexts built so far (names the IPC rendezvous of each)
    int sparse_transport = 0;    // hash-sharded sparse engine across processes: 0 RCCL, 1 IPC pulls (GM_OPT_SPARSE_TRANSPORT)
    int sparse_solves = 0;       // sharded sparse solves run with the IPC transport (names each one's segment)
    int poison = 0;              // test hook (GM_OPT_POISON): received data pre-filled with 0xFF; 2 = early flag
    int virtual_ranks = 1;   // >1: run that many ranks inside this context (loopback transport)
    hipStream_t comm_stream = nullptr;
    int dist_batch = 4;      // sharded dense path: tiers per halo exchange
    int dist_slots = 4;      // sharded dense path: ring of exchange buffers, in batches
    int dist_solo = 0;       // diagnostic (loopback): enqueue only rank dist_solo-1's tier launches
    int dist_symmetry = 1;   // sharded dense path: halo blocks derivable by a heap swap are filled locally
    int dist_owner = 0;      // sharded dense path: 0 = split heaps in halves, 1 = tier-balanced comparisons
    int box_flow = -1;       // box engine, one GPU: -1 / 0 tier launches, 1 dataflow (GM_OPT_BOX_FLOW)
    bool box_flow_failed = false;   // a dataflow solve timed out: tier launches until GM_OPT_BOX_FLOW is set again
    int box_flow_fallbacks = 0;     // dataflow solves of this context that fell back to tier launches
    int box_split = 0;       // split box engine (N > 1): 0 halves, 1 comparisons (GM_OPT_BOX_SPLIT)
    int symmetry = 1;        // sparse engines: store one representative per symmetry orbit (games.hpp)

    // results
    bool solved = false;
    int engine = 0;          // engine used by the last solve
    uint64_t root = 0;
    uint64_t n_positions = 0;
    uint16_t root_record = REC_UNSOLVED;
    gm_stats_t stats{};
    std::vector<uint64_t> tier_counts;

    // device buffer cache (dev_alloc / dev_free)
    std::vector<std::pair<void *, uint64_t>> buf_live, buf_cache;

    // adopted buffers
    void *adopted_dense = nullptr;
    uint64_t adopted_dense_bytes = 0;

    DenseSub *dsub = nullptr;
    DenseBox *dbox = nullptr;   // the box engine (GM_OPT_SUB_INTERLEAVE 20, 8 heaps)
    bool dbox_active = false;   // the last dense SUBTRACT solve used dbox
    SmallDense *sd = nullptr;
    Sparse *sp = nullptr;
    DistSub *dist_sub = nullptr;
    DistBox *dist_box = nullptr;  // the box engine split over ranks (dist_box.hip), reached through dense_box_*
    DistSparse *dist_sp = nullptr;
    Graph *graph = nullptr;
};

// engines (each returns GM_OK or a GM_E_* code)
int dense_sub_solve(Ctx *c, uint64_t root);
int dense_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dense_sub_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int dense_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void dense_sub_free(Ctx *c);
int dense_sub_table(Ctx *c, void **p, uint64_t *bytes);
// the box-tiled engine for 8 heaps (dense_box.hip), reached through dense_sub_*
int dense_box_solve(Ctx *c, uint64_t root);
int dense_box_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dense_box_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int dense_box_digest(Ctx *c, uint64_t *digest, uint64_t *n);
int dense_box_table(Ctx *c, void **p, uint64_t *bytes);
void dense_box_free(Ctx *c);
// shared with the split box engine (dist_box.hip)
uint64_t box_hilbert(uint32_t box);
int box_grid_cap(int device);
void box_launch_split_flow(uint32_t grid, const void *ranks, uint32_t nranks, uint32_t ep, uint32_t *err,
                           uint64_t timeout_ticks, bool sys, hipStream_t s);
int box_split_flow_resident(int device);
// the split dataflow launch's per-rank descriptor (dense_box.hip BxSplitFlow), filled by dist_box.hip
struct BxSplitFlowDesc {
    uint8_t *table;
    const uint32_t *boxes, *fills, *srcs, *dsts, *groups;
    uint32_t qbase[8], qlen[8];
    uint32_t *flag;
    uint8_t *ptab[3];
    uint32_t *pflag[3];
};
void box_launch_tier_split(uint32_t grid, uint8_t *table, const uint32_t *boxes, const uint32_t *fills,
                           const uint32_t *srcs, const uint32_t *dsts, uint8_t *msg, uint8_t *const *peers,
                           uint32_t nbox, bool fill, hipStream_t s);
void box_launch_digest(const uint8_t *table, const uint32_t *boxes, uint64_t nbox, uint64_t root,
                       unsigned long long *acc, hipStream_t s);
void box_launch_query(const uint8_t *const *tables, const uint8_t *owner, uint64_t root, const uint64_t *keys,
                      uint16_t *out, uint64_t n, hipStream_t s);
void box_tier_counts(uint64_t root, std::vector<uint64_t> &acc);
void box_region_keys(uint64_t root, uint64_t *keys, uint64_t n);
// the box engine split over G ranks (dist_box.hip)
int dist_box_solve(Ctx *c, uint64_t root);
int dist_box_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dist_box_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int dist_box_digest(Ctx *c, uint64_t *digest, uint64_t *n);
int dist_box_table(Ctx *c, void **p, uint64_t *bytes);
int dist_box_rank_stats(Ctx *c, double *kernel_ms, uint64_t *boxes, uint64_t *recv_bytes, int cap, int *n);
int dist_box_op_ms(Ctx *c, int rank, double *ms, int cap, int *n);
void dist_box_free(Ctx *c);
int dist_box_plan(uint64_t root, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *out,
                  uint64_t cap, uint64_t *n);

// the dense tier kernel, shared with the partitioned (multi-GPU) driver
bool sub_kernel_exists(int low, int high, int nt);
void launch_sub_tier(int low, int high, int nt, uint32_t nblocks, uint8_t *table, const uint32_t *list,
                     const uint8_t *zero, hipStream_t s);
// the sharded solve's byte-image tier kernel with per-block extra destinations (LOW = 3)
bool sub_kernel_x_exists(int high);
void launch_sub_tier_x(int high, uint32_t nblocks, uint8_t *table, const uint32_t *list, const uint8_t *zero,
                       const uint32_t *xoff, const uint64_t *xdst, hipStream_t s, int kind);
int sub_kernel_threads(const Ctx *c, int low);   // 0 = the 4-block interleaved kernel
void sort_tiers_morton(std::vector<uint32_t> &order, const std::vector<uint32_t> &tier_off, int high, int mode);

// partitioned dense solve: `world` ranks, real (RCCL, one per process) or virtual (loopback)
int dist_sub_solve(Ctx *c, uint64_t root);
int dist_sub_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dist_sub_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int dist_sub_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void dist_sub_free(Ctx *c);
int dist_sub_plan(int heaps, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *off,
                  uint64_t off_cap, uint64_t *n_off, uint32_t *data, uint64_t data_cap, uint64_t *n_data);

int dist_sparse_solve(Ctx *c, uint64_t root);
int dist_sparse_solve_wide(Ctx *c, const K128 &root);
int dist_sparse_layout(int G, int S, const uint64_t *mat, int r, uint64_t *seg, uint64_t *send_off,
                       uint64_t *recv_off, uint64_t *recv_seg);
int dist_sparse_export_wide(Ctx *c, K128 *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dist_sparse_query_wide(Ctx *c, const K128 *keys, uint16_t *recs, uint64_t n);
int dist_sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int dist_sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int dist_sparse_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void dist_sparse_free(Ctx *c);

int small_dense_solve(Ctx *c, uint64_t root);
int small_dense_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int small_dense_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int small_dense_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void small_dense_free(Ctx *c);

int graph_solve(Ctx *c, uint64_t n, const uint8_t *prim, const uint64_t *off, const uint32_t *kid);
int graph_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int graph_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int graph_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void graph_free(Ctx *c);

int sparse_solve(Ctx *c, uint64_t root);
int sparse_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n);
int sparse_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n);
int sparse_digest(Ctx *c, uint64_t *digest, uint64_t *n);
void sparse_free(Ctx *c);

double now_ms();

// Device buffers of the per-solve tables, cached per context and reused by the
// next solve (dev_free keeps the buffer; gm_close releases them).  Buffers are
// only used on the context's stream, so reuse is stream-ordered.  GM_TRACE=1
// logs every hipMalloc with its host time.
int dev_alloc(Ctx *c, void **p, uint64_t bytes);
void dev_free(Ctx *c, void *p);
bool trace_on();
int ensure_comm(Ctx *c);   // the RCCL communicator of gm_set_comm's unique id (collective on first use)

}  // namespace gm

struct gm_ctx {
    gm::Ctx c;
};
