/*
 * gmsolve.h -- C ABI of libgmsolve.so, the MI355X strong solver.
 *
 * This is the drop-in boundary for the reference's solve path.  In the reference
 * a solve is the mpi4py job loop of src/new_process.py (Process.run :37-60,
 * lookup :102-133, distribute :145-162, resolve :223-265) over the shelve tables
 * of src/cache_dict.py, started by solver_launcher.py:132-164.  Here a solve is
 * one call, gm_solve(), over HBM-resident tables; the Python host
 * (gamesmanmpi_amd/, solver_launcher.py, solve_local.py) binds these symbols with
 * ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - every function returns GM_OK (0) or a negative GM_E_* code and never aborts;
 *     gm_last_error() describes the last failure on the calling thread;
 *   - host arrays are owned by the caller; device tables are owned by the context
 *     (or adopted from the caller with gm_adopt_buffer) and die with gm_close();
 *   - a gm_ctx is not thread-safe; use one per host thread;
 *   - no torch types: plain pointers and sizes only.
 *
 * Records (u16): bits 15..14 = value (0 WIN, 1 LOSS, 2 TIE; the codes of
 * reference src/utils.py:4), bits 13..0 = remoteness.  0xFFFF = not reached.
 */
#ifndef GMSOLVE_H
#define GMSOLVE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_ABI_VERSION 2   /* 2: gm_box_plan opts/axis, gm_rank_stats recv_bytes, gm_stats_t.flow_fallbacks,
                               GM_OPT_SPARSE_TRANSPORT, GM_OPT_POISON */

/* Game descriptors.  Params per game:
 *   GM_GAME_FOUR_TO_ONE  none                  (reference test_games/four_to_one.py)
 *   GM_GAME_TTT          none                  (test_games/mttt.py, tic_tac_toe_np.py)
 *   GM_GAME_TOOT         {length, height}      (test_games/toot_and_otto_bitstring.py), 2*L*H+16 <= 64
 *   GM_GAME_OTHELLO      {length, height}      (test_games/othello_bit_new.py), square, 2*L*H+16 <= 64,
 *                                              or {8, 8} with 3-word keys (gm_key_words)
 *   GM_GAME_SUBTRACT     {heaps}               (the build's synthetic game, 1..8 heaps of 4 bits)
 *   GM_GAME_GRAPH        none                  (any plugin: an explicit graph from gm_solve_graph)
 */
enum {
    GM_GAME_FOUR_TO_ONE = 1,
    GM_GAME_TTT = 2,
    GM_GAME_TOOT = 3,
    GM_GAME_OTHELLO = 4,
    GM_GAME_SUBTRACT = 5,
    GM_GAME_GRAPH = 6
};

enum {
    GM_OK = 0,
    GM_E_ARG = -1,          /* bad argument */
    GM_E_GAME = -2,         /* unknown game or unsupported parameters */
    GM_E_HIP = -3,          /* HIP runtime error (no device, launch failure, ...) */
    GM_E_NOMEM = -4,        /* device or host allocation failed */
    GM_E_STATE = -5,        /* call out of order (e.g. export before solve) */
    GM_E_DRAW = -6,         /* a DRAW primitive was reached (unsupported) */
    GM_E_NOMOVES = -7,      /* non-primitive position without moves (the reference hangs) */
    GM_E_CAP = -8,          /* caller buffer too small / remoteness overflow */
    GM_E_COMM = -9,         /* RCCL failure */
    GM_E_KEY = -10          /* root key is not a valid position of the game */
};

/* Internal engine selection (gm_set_option GM_OPT_ENGINE). */
enum {
    GM_ENGINE_AUTO = 0,     /* dense for SUBTRACT / TTT, sparse otherwise */
    GM_ENGINE_DENSE = 1,
    GM_ENGINE_SPARSE = 2,
    GM_ENGINE_DIST_DENSE = 3,   /* reported in gm_stats_t.engine: sharded dense path */
    GM_ENGINE_DIST_SPARSE = 4,  /* reported in gm_stats_t.engine: sharded sparse path; as GM_OPT_ENGINE it
                                   forces that path (needs gm_set_comm or GM_OPT_VIRTUAL_RANKS) */
    GM_ENGINE_GRAPH = 5         /* reported in gm_stats_t.engine: explicit graph (gm_solve_graph) */
};

enum {
    GM_OPT_ENGINE = 1,      /* GM_ENGINE_* */
    GM_OPT_SUB_LOW = 2,     /* SUBTRACT dense path: heaps solved per workgroup in LDS (1..4) */
    GM_OPT_GRAPH = 3,       /* SUBTRACT dense path: replay the tier launches as a hipGraph (0/1, default
                               1); the split box engine with virtual ranks or GM_OPT_BOX_TRANSPORT 1
                               captures each solve's launches once and replays them too (RCCL
                               transport: always eager) */
    GM_OPT_TIMING = 4,      /* record HIP events around every launch of the dominant kernel (0/1); 2 = on
                               the split box engine also an event pair around every op (gm_rank_op_ms) */
    GM_OPT_VIRTUAL_RANKS = 5, /* >1: run the sharded algorithm with that many ranks inside this one
                                context on one GPU (loopback transport instead of RCCL); for testing
                                the multi-GPU partition on a single device */
    GM_OPT_SUB_THREADS = 6, /* SUBTRACT dense path: threads per block workgroup (64, 128, 256) */
    GM_OPT_SUB_INTERLEAVE = 7, /* SUBTRACT dense path: 20 (default) = the box engine at 8 heaps
                                  (dense_box.hip: 4x4x4x4x2x2x2x2 boxes, 41 launches; split at N > 1, every
                                  box on one rank, halo boxes over RCCL, gm_box_plan); other heap counts
                                  use 10; 10 = the block
                                  engine's walker kernel on tiers of >= 4096 blocks, the four-block kernel
                                  below (sharded at N > 1 with halo exchanges, gm_dist_plan); 6 = the
                                  four-block kernel (byte LDS image, 256-thread barrier walk) on every tier;
                                  1 = one block per workgroup of GM_OPT_SUB_THREADS */
    GM_OPT_SUB_ORDER = 8,   /* SUBTRACT dense path: block order inside a tier, 0 = key order, 1 = Morton,
                               2 = Hilbert walk of the tier's free high nibbles (default) */
    GM_OPT_DIST_BATCH = 9,  /* sharded SUBTRACT path: tiers (box engine: box-tiers) per halo exchange
                               (default 4) */
    GM_OPT_DIST_SLOTS = 10, /* sharded SUBTRACT path: exchange buffers per split heap, in batches (default 4) */
    GM_OPT_DIST_SOLO = 12,  /* diagnostic, loopback sharded SUBTRACT path: r + 1 = enqueue only rank r's
                               tier launches (no exchange, no waits), to time one rank's compute
                               critical path; the results are NOT valid.  0 (default) = off. */
    GM_OPT_DIST_SYMMETRY = 11, /* sharded SUBTRACT path: 1 (default) = fill halo blocks that are a heap
                                 permutation of an own block locally (box engine: read a crossing child
                                 box through a heap transposition of a box this rank computed), 0 =
                                 receive every halo block */
    GM_OPT_DIST_OWNER = 13, /* sharded SUBTRACT path, block owner: 0 = split the top heaps in halves
                               (rank bit a = [heap >= 8]); 1 = tier-balanced: rank bits compare two
                               heaps ([h_x < h_y]) while enough heaps remain, [heap >= 8] after, so
                               every rank holds a share of every tier (needs GM_OPT_DIST_SYMMETRY 1) */
    GM_OPT_SYMMETRY = 14,   /* sparse engines, symmetry reduction (the reference's unused
                               hook othello_bit_new.py:224-235): 1 (default) = TOOT stores one position
                               per left-right mirror pair when the root is its own mirror image; every
                               count, export, query and digest still covers both positions.  0 = off */
    GM_OPT_BOX_FLOW = 15,   /* box engine (SUBTRACT, 8 heaps), one GPU: -1 (default) / 0 = one launch per
                               box-tier; 1 = one dataflow launch (box_flow_kernel: a box group starts
                               when its child boxes are stored; its grid is the kernel's resident
                               capacity from the occupancy API).  A dataflow solve whose waits time out
                               is redone with tier launches, and the context keeps tier launches until
                               this option is set again; gm_stats_t.flow_fallbacks counts them.
                               Split solve (virtual ranks or GM_OPT_BOX_TRANSPORT 1): 1 = each rank's
                               chain one launch, halo boxes and their flags stored into the receiving
                               rank's table and flag array (box_split_flow_kernel); a wait past 200 ms
                               (30 s across processes) fails the solve with GM_E_STATE. */
    GM_OPT_BOX_SPLIT = 16,  /* box engine at N > 1 (gm_box_plan): 0 (default) = split heaps in halves
                               (rank bit a = [box coordinate >= half]); 1 = tier-balanced comparisons
                               (rank bit = [c_x < c_y], ties by a rule that keeps every axis one-way) */
    GM_OPT_BOX_TRANSPORT = 17, /* box engine at N > 1, one process per rank: how a halo message
                               travels.  0 (default) = ncclSend / ncclRecv on per-axis communicators;
                               1 = the sender's tier kernel stores its halo boxes straight into the
                               receiver's table, mapped through HIP IPC (hipIpcGetMemHandle, exchanged
                               through a POSIX shared-memory segment named by the unique id), with
                               completion flags in device memory that stream-ordered kernels set and
                               poll (30 s limit, then GM_E_COMM).  1
                               also runs when the ranks share one GPU, where RCCL refuses; all the
                               ranks of one node.  Set on every rank before the first solve. */
    GM_OPT_SPARSE_TRANSPORT = 18, /* hash-sharded sparse engine (GM_ENGINE_DIST_SPARSE; Toot, Othello, ...) at
                               N > 1, one process per rank: how the per-tier LOOK_UP keys and RESOLVE
                               scores travel (reference src/new_process.py:156-160, :179-187).  0 (default)
                               = ncclSend / ncclRecv groups, counts all-gathered and totals all-reduced
                               over RCCL; 1 = IPC: every rank publishes its send buffers' HIP IPC handles
                               in a POSIX shared-memory segment named by the unique id, each receiver
                               pulls its segments from the senders' buffers (hipMemcpyAsync from the
                               mapping), and counts, totals and the root record are all-gathered through
                               the same segment, ordered by host barriers (120 s limit, then GM_E_COMM;
                               a rank that fails marks the segment and its peers fail at once).  1 runs
                               when the ranks share one GPU (RCCL refuses that); all the ranks of one
                               node.  Set on every rank before the solve. */
    GM_OPT_POISON = 19      /* test hook, multi-process sharded solves: 1 = fill what a rank receives
                               with 0xFF before it arrives -- the split box engine's table (IPC / RCCL
                               transports) before every solve, the sparse engine's receive buffers
                               before every exchange -- so a halo or reply that never lands, or lands
                               late, changes the results instead of reading a previous solve's bytes.
                               0 (default) = off.  Fault hook (box engine, IPC transport, tests only):
                               2 = 1 plus, from the second solve on, every receiver reads its halo boxes
                               without waiting for their arrival flags (as if they were set early) while
                               rank 0 is held 50 ms -- solve 2 then differs from the oracle; 3 = the
                               same fault without the poisoning, which no digest can see (solve 2 reads
                               solve 1's identical bytes; tests/test_gpu_multiproc.py) */
};

/* Buffer roles for gm_adopt_buffer. */
enum {
    GM_BUF_DENSE_TABLE = 1  /* SUBTRACT dense table: 1 byte per slot, 16^heaps slots */
};

typedef struct gm_ctx gm_ctx;

typedef struct {
    uint64_t n_positions;   /* reachable positions with a final record (all ranks) */
    uint64_t n_primitive;   /* of which primitive (this rank; dense path: all) */
    int32_t n_tiers;        /* tiers walked */
    int32_t world;          /* ranks in the solve */
    double solve_ms;        /* wall time of the last gm_solve (host clock, device-synchronised) */
    double forward_ms;      /* sparse path: forward expansion part */
    double backward_ms;     /* retrograde part */
    double exchange_ms;     /* multi-GPU: time inside RCCL calls (host-observed) */
    uint64_t algo_bytes;    /* algorithmic HBM bytes of the solve (SURVEY §8d edge model) */
    uint64_t table_bytes;   /* device bytes held by the tables */
    uint64_t exchanged_bytes; /* multi-GPU: bytes sent over RCCL by this rank */
    double kernel_ms;       /* GM_OPT_TIMING: summed event time of the dominant kernel's launches */
    int32_t kernel_launches;/* GM_OPT_TIMING: number of those launches */
    int32_t engine;         /* GM_ENGINE_DENSE or GM_ENGINE_SPARSE */
    uint64_t n_edges;       /* sparse path: parent->child edges expanded (this rank) */
    int32_t flow_fallbacks; /* box engine: dataflow solves of this context redone with tier launches */
    uint64_t n_stored;      /* positions the solve expanded and resolved (all ranks): with a symmetry
                               reduction (GM_OPT_SYMMETRY) one representative per orbit, so <= n_positions,
                               which counts every position the representatives stand for; = n_positions
                               for the other engines */
} gm_stats_t;

/* Library version (GM_ABI_VERSION). */
int gm_version(void);

/* Last error message of the calling thread ("" if none). */
const char *gm_last_error(void);

/* Number of visible HIP devices (0 when none). */
int gm_device_count(void);

/* Create a context for one game on one HIP device (device < 0: the current one).
 * Replaces the per-rank Process construction (reference src/new_process.py:62-94). */
int gm_open(int game_id, const int32_t *params, int nparams, int device, gm_ctx **out);

/* Run subsequent work on the caller's HIP stream (hipStream_t), e.g. torch's
 * current stream; NULL restores the context's own stream. */
int gm_set_stream(gm_ctx *ctx, void *hip_stream);

/* Tunables (GM_OPT_*). */
int gm_set_option(gm_ctx *ctx, int option, int64_t value);

/* Key of the game's initial position (reference GameState.INITIAL_POS,
 * src/game_state.py:15, i.e. initial_position() of the plugin). */
int gm_pack_initial(gm_ctx *ctx, uint64_t *key);

/* Host twin of the device descriptor for ONE position: its primitive value
 * (0..4, src/utils.py:4), its tier, and (if not primitive) its children keys in
 * the plugin's gen_moves order.  Used to match a plugin module to a descriptor
 * and by tests; not on the solve path (reference GameState.expand /
 * GameState.primitive, src/game_state.py:33-41, :59-85). */
int gm_expand_host(gm_ctx *ctx, uint64_t key, uint64_t *children, int cap,
                   int *n_children, int *primitive, int64_t *tier);

/* Multi-GPU: join a solve of `world` ranks (one process per GPU).  `uid` is a
 * 128-byte ncclUniqueId produced by gm_comm_unique_id on rank 0 and shared by
 * the caller (e.g. over torch.distributed).  Replaces the mpi4py COMM_WORLD the
 * reference passes to Process (solver_launcher.py:47-52, :132-140).  With
 * world = 1 and a uid, a one-rank communicator is created: with GM_OPT_ENGINE =
 * GM_ENGINE_DIST_SPARSE the hash-sharded engine then runs its RCCL transport on
 * one GPU (self send/recv, all-gather, all-reduce), which tests use.
 * The communicator itself is made by the first solve that needs one (collective: every rank's
 * first sharded solve), not by this call, so ranks whose transport needs none -- the split box
 * engine with GM_OPT_BOX_TRANSPORT 1, possibly several ranks on one GPU -- never make it.
 * uid NULL sets rank and world only, with no communicator; every sharded engine then refuses to
 * solve (GM_E_COMM).  gm_solve checks the root key and the options before it makes the
 * communicator, so a call that every rank makes with the same arguments fails on every rank
 * before the first collective; a sharded solve's first call must be made by all ranks. */
int gm_comm_unique_id(void *uid, int bytes);
int gm_set_comm(gm_ctx *ctx, int rank, int world, const void *uid, int bytes);

/* Strong-solve every position reachable from root_key (collective when a
 * communicator is set: every rank calls it with the same root).  Returns the
 * global number of reachable positions and the root's record (on every rank).
 * Replaces Process.run/lookup/distribute/check_for_updates/send_back/resolve
 * (src/new_process.py:37-265) and the root line of :42-53. */
int gm_solve(gm_ctx *ctx, uint64_t root_key, uint64_t *n_positions, uint16_t *root_record);

/* Keys of more than 64 bits.  A board whose position string exceeds 64 bits -- GM_GAME_OTHELLO
 * with params {8, 8}, the reference plugin's default (test_games/othello_bit_new.py:8: 2A + 16 =
 * 144 bits) -- has keys of gm_key_words() u64 words: the position string read as one big-endian
 * integer, stored least significant word first (the one-word games' keys are that integer too).
 * Such a context is solved by the hash-sharded sparse engine with 128-bit device keys (one GPU,
 * virtual ranks, or one process per rank) and uses the *_key calls below; the one-word calls
 * return GM_E_ARG for it.  For one-word games the *_key calls equal their one-word forms.
 * gm_digest folds each key to one word first (mix64(lo ^ mix64(hi ^ c)) of the device key), so
 * digests compare across ranks and world sizes, not with one-word games. */
int gm_key_words(gm_ctx *ctx);
int gm_pack_initial_key(gm_ctx *ctx, uint64_t *key_words);
int gm_expand_host_key(gm_ctx *ctx, const uint64_t *key_words, uint64_t *children_words, int cap,
                       int *n_children, int *primitive, int64_t *tier);
int gm_solve_key(gm_ctx *ctx, const uint64_t *root_words, uint64_t *n_positions, uint16_t *root_record);
int gm_export_key(gm_ctx *ctx, uint64_t *key_words, uint16_t *records, uint64_t cap, uint64_t *n);
int gm_query_key(gm_ctx *ctx, const uint64_t *key_words, uint16_t *records, uint64_t n);

/* Strong-solve an explicit position graph (context opened with GM_GAME_GRAPH):
 * for plugins no device descriptor reproduces, the host enumerates positions
 * 0..n-1 with the plugin's own functions (position 0 = the root) and passes
 * primitive[i] (the plugin's primitive() code, src/utils.py:4) and the children of
 * i as child_idx[child_off[i] .. child_off[i+1]) (CSR, child_off has n+1 entries).
 * The device resolves every position (Appendix A); keys of gm_export / gm_query /
 * gm_digest are then the position indices.  A cycle, a DRAW primitive or an
 * undecided position without children is an error (the reference would hang).
 * Replaces the reference's per-position job loop for arbitrary plugins
 * (src/new_process.py:37-265, GameState.expand src/game_state.py:33-41). */
int gm_solve_graph(gm_ctx *ctx, uint64_t n, const uint8_t *primitive, const uint64_t *child_off,
                   const uint32_t *child_idx, uint16_t *root_record);

/* Copy this rank's solved table to host arrays, sorted by key.  With keys ==
 * NULL only *n is set (the count).  Replaces reading the resolved/remote shelve
 * tables (src/cache_dict.py:38-79, src/new_process.py:76-78). */
int gm_export(gm_ctx *ctx, uint64_t *keys, uint16_t *records, uint64_t cap, uint64_t *n);

/* Records of n keys (0xFFFF for keys this rank does not hold: in a multi-process solve a rank
 * holds the keys it computed -- box engine: the boxes of gm_box_plan GM_BOXPLAN_BOXES, sparse
 * engine: its hash share; with virtual ranks, or on one GPU, every key of the root's region;
 * 0xFFFF outside it).  Replaces
 * `pos in self.resolved` / `self.resolved[pos]` lookups (src/new_process.py:111-117). */
int gm_query(gm_ctx *ctx, const uint64_t *keys, uint16_t *records, uint64_t n);

/* Order-independent digest of this rank's table:
 * sum over positions of mix64(key * 0x9E3779B97F4A7C15 + record) (mod 2^64),
 * computed on the device; sums of the ranks' digests compare across world sizes. */
int gm_digest(gm_ctx *ctx, uint64_t *digest, uint64_t *n);

/* Solve statistics of the last gm_solve. */
int gm_stats(gm_ctx *ctx, gm_stats_t *out);

/* Positions per tier of the last solve (this rank); *n = number of tiers. */
int gm_tier_counts(gm_ctx *ctx, uint64_t *counts, int cap, int *n);

/* Back a table with caller-owned device memory (e.g. a torch tensor's storage).
 * The caller keeps it alive until gm_close. */
int gm_adopt_buffer(gm_ctx *ctx, int role, void *dev_ptr, uint64_t bytes);

/* Device pointer and size of the dense table (GM_BUF_DENSE_TABLE) after a solve;
 * its slots hold 1-byte order-preserving codes ("HBM layout"), not records.
 * The slot of a key depends on the engine:
 *   - block engine (heaps != 8, or GM_OPT_SUB_INTERLEAVE != 20): slot = key;
 *   - box engine (8 heaps, the default): slot = box << 12 | A << 4 | B, with box = the box
 *     id of gm_box_plan (heap i >> 2 at bits 2i for heaps 0-3, heap j >> 1 at bits
 *     8 + 3 (j - 4) for heaps 4-7), A = sum over heaps 0-3 of (heap i & 3) << 2i and
 *     B = sum over heaps 4-7 of (heap j & 1) << (j - 4).  At N > 1 a rank's table holds
 *     the boxes it computed (gm_box_plan GM_BOXPLAN_BOXES) and the halo boxes it received.
 * Read records through gm_query / gm_export unless the layout is handled. */
int gm_dense_table(gm_ctx *ctx, void **dev_ptr, uint64_t *bytes);

/* Host only -- makes no HIP or RCCL call, so it runs without a GPU: the plan
 * that rank `rank` of a `world`-rank sharded SUBTRACT solve executes, built by
 * the same code gm_solve uses (block-owner partition, halo lists, op list;
 * DESIGN.md §5).  For tests and tooling that check the multi-GPU schedule on the
 * CPU.  The reference has no counterpart: its schedule is the dynamic mpi4py job
 * queue (src/new_process.py:37-60, :145-187).  `opts` = {GM_OPT_DIST_BATCH,
 * GM_OPT_DIST_SLOTS, GM_OPT_DIST_SYMMETRY | GM_OPT_DIST_OWNER << 1} values, NULL = defaults.
 *   GM_PLAN_SHAPE  data = {low, high, ntiers, batch, nbatch, nslots, g};
 *                  off = (lo, hi) tier range of each batch's halo message
 *   GM_PLAN_OWN    data = high parts this rank computes; off[t]..off[t+1] = tier t
 *   GM_PLAN_FILL   data = (dst, src) pairs of tier t filled locally (off in u32 entries)
 *   GM_PLAN_SEND   data = halo high parts sent on split heap `axis`; off per batch
 *   GM_PLAN_RECV   data = halo high parts received on split heap `axis`; off per batch
 *   GM_PLAN_OPS    data = 6 u32 per op {kind, axis, event, on_exchange_stream, tier|batch, peer},
 *                  kind: 0 tier launch (also writes every block's extra destinations:
 *                  its symmetric-fill images and its halo ring slots), 2 unpack, 3 send,
 *                  4 recv, 5 event record, 6 event wait (kinds 1 pack and 7 fill are
 *                  folded into 0); event: 0 message complete in its slot, 1 exchanged,
 *                  2 unpacked
 *   GM_PLAN_XDEST  per own block (GM_PLAN_OWN order) its extra destinations:
 *                  off[i]..off[i+1] index (kind, value) u32 pairs of data; kind 0 =
 *                  table block (value = high part), 1 + axis = halo message slot
 *                  (value = batch << 16 | index in the message)
 * With off / data NULL only *n_off / *n_data are set. */
enum { GM_PLAN_SHAPE = 0, GM_PLAN_OWN = 1, GM_PLAN_FILL = 2, GM_PLAN_SEND = 3, GM_PLAN_RECV = 4, GM_PLAN_OPS = 5,
       GM_PLAN_XDEST = 6 };
int gm_dist_plan(int heaps, int world, int rank, const int32_t *opts, int what, int axis,
                 uint32_t *off, uint64_t off_cap, uint64_t *n_off,
                 uint32_t *data, uint64_t data_cap, uint64_t *n_data);

/* Host only (no HIP call): the plan of rank `rank` of a `world`-rank split solve of the 8-heap
 * SUBTRACT game on the box engine (the default at 8 heaps), built by the same
 * code gm_solve runs.  The reference's counterpart is its owner hash, md5(str(pos)) % world
 * (src/game_state.py:23-31), with every child sent to its owner and every result sent back
 * (src/new_process.py:156-160, :179-187).  Here each box has ONE owner, a function of its box
 * coordinates with one bit per split axis (world rounded down to 1, 2, 4 or 8 ranks with work);
 * a child box another rank owns is read through a heap transposition of a box this rank
 * computed, or received from that rank in the batch's halo message.  Box ids pack the box
 * coordinates (heap i >> 2 for heaps 0-3 at bits 2i, heap j >> 1 for heaps 4-7 at bits
 * 8 + 3 (j - 4)).  `opts` = {GM_OPT_DIST_BATCH, GM_OPT_DIST_SYMMETRY, GM_OPT_BOX_SPLIT, loopback op
 * list 0/1, GM_OPT_BOX_TRANSPORT} values (5 int32), NULL = defaults.  `axis` selects the axis of SEND / RECV items.
 *   GM_BOXPLAN_SHAPE     {world, axes, box-tiers, batch, batches, split, fill} then per axis a = 0..2
 *                        {kind (0 none, 1 half, 2 comparison), heap d | x, threshold | y, free-heap mask}
 *   GM_BOXPLAN_BOXES     the boxes this rank computes, by box-tier (GM_BOXPLAN_TIER_OFF)
 *   GM_BOXPLAN_FILLS     per computed box (the kernel's fill word): 4 bits per child direction d at
 *                        bit 4 d; A heap d: q << 2 | p, the child read through the transposition of
 *                        A heaps q and p (q = p: the child box itself); B heap d: 0 = the child box
 *                        itself, 1..6 = through the transposition of B heaps 4 + pair, pairs (0,1)
 *                        (0,2) (0,3) (1,2) (1,3) (2,3)
 *   GM_BOXPLAN_SRCS      per computed box 8 words: the box read for the child along heap d (the
 *                        child box, or its image under that transposition; 0 where there is no child)
 *   GM_BOXPLAN_DSTS      per computed box 3 words: the halo message slots the tier kernel also
 *                        writes it to (bits 28-31: 0 none, 1..4 the two top layers along A heap
 *                        kind - 1, 5 the whole box; bits 0-27: byte offset in the rank's send
 *                        buffer / 2 KiB; the buffer holds axis 0's messages, then axis 1's, ...)
 *   GM_BOXPLAN_TIER_OFF  offsets of the box-tiers in GM_BOXPLAN_BOXES
 *   GM_BOXPLAN_OWN       GM_BOXPLAN_BOXES ascending (digest, export); the ranks' lists partition
 *                        the root's region
 *   GM_BOXPLAN_SEND / _RECV          halo entries sent / received on `axis`: box | code << 20,
 *                        code 0 = the whole box, 1 + i = its two top layers along A heap i
 *   GM_BOXPLAN_SEND_OFF / _RECV_OFF  their offsets per batch
 *   GM_BOXPLAN_HALO      (lo, hi) box-tier range of each batch's message
 *   GM_BOXPLAN_OPS       6 u32 per op {kind, axis, event, on_exchange_stream, tier | batch, peer};
 *                        kind 0 tier launch (which also writes its boxes' halo slots), 2 unpack (every
 *                        message of the batch, `axis` unused), 3 send, 4 receive, 5 event record,
 *                        6 event wait (1 pack is fused into 0); event 0 tier done, 1 message
 *                        complete (loopback lists)
 *   GM_BOXPLAN_COUNTS    {boxes computed, child reads through a transposition, child reads from a message}
 * With out NULL only *n is set. */
enum { GM_BOXPLAN_SHAPE = 0, GM_BOXPLAN_BOXES = 1, GM_BOXPLAN_FILLS = 2, GM_BOXPLAN_TIER_OFF = 3, GM_BOXPLAN_OWN = 4,
       GM_BOXPLAN_SEND = 5, GM_BOXPLAN_SEND_OFF = 6, GM_BOXPLAN_RECV = 7, GM_BOXPLAN_RECV_OFF = 8,
       GM_BOXPLAN_HALO = 9, GM_BOXPLAN_OPS = 10, GM_BOXPLAN_COUNTS = 11, GM_BOXPLAN_SRCS = 12,
       GM_BOXPLAN_DSTS = 13 };
int gm_box_plan(uint64_t root_key, int world, int rank, const int32_t *opts, int what, int axis, uint32_t *out,
                uint64_t cap, uint64_t *n);

/* Host only (no HIP or RCCL call): the layout of one exchange of the hash-sharded sparse engine
 * (csrc/dist_sparse.hip), the same for its RCCL, IPC and loopback transports.  counts is the
 * world x (world * steps) matrix of one exchange: row q = source rank, column p * steps + s =
 * children of q's parents owned by rank p that lie s + 1 tiers deeper.  For rank `rank`:
 *   seg[p * steps + s]       where that bin starts in rank's send buffer (destination-major)
 *   send_off[p], p <= world  rank's send segment for destination p (all steps)
 *   recv_off[q], q <= world  rank's receive segment from source q (all steps)
 *   recv_seg[q * steps + s]  where source q's keys of step s start in rank's receive buffer
 * LOOK_UP keys go send_off -> recv_off; RESOLVE scores come back recv_off -> send_off
 * (reference src/new_process.py:156-160, :179-187).  Any array may be NULL. */
int gm_sparse_layout(int world, int steps, const uint64_t *counts, int rank, uint64_t *seg, uint64_t *send_off,
                     uint64_t *recv_off, uint64_t *recv_seg);

/* Per rank this context ran in its last solve on the split box engine (all virtual ranks, or its
 * own rank of a multi-process solve): with GM_OPT_TIMING the GPU time from the start of the rank's
 * first tier launch to the end of its last, the boxes it computed, and the halo bytes it receives
 * per solve.  With GM_OPT_DIST_SOLO r + 1 (virtual ranks) rank r's list runs alone, its cross-rank
 * waits dropped -- its own critical path -- enqueued whole behind a 20 ms hold of the stream, so
 * the time has no host enqueue gaps.  *n = 0 for every other engine. */
int gm_rank_stats(gm_ctx *ctx, double *kernel_ms, uint64_t *boxes, uint64_t *recv_bytes, int cap, int *n);

/* With GM_OPT_TIMING, the GPU ms of every op of `rank`'s op list (GM_BOXPLAN_OPS order; 0 for
 * event records and waits) in the last solve of the split box engine, with GM_OPT_TIMING 2 (an event
 * pair around each op; 1 times only the whole solve and each rank's span). */
int gm_rank_op_ms(gm_ctx *ctx, int rank, double *ms, int cap, int *n);

/* Release everything. */
void gm_close(gm_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* GMSOLVE_H */
