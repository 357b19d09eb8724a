// small_dense.hip -- one-workgroup, all-in-LDS solver for games with a small
// dense key space (tic-tac-toe: 3^9 = 19,683 slots).
//
// The whole solve is ONE launch: forward reachability by tier (the
// level-synchronous replacement of Process.distribute / LOOK_UP,
// reference src/new_process.py:145-162), then the retrograde by tier from the
// deepest (Process.resolve, :223-265), both over LDS arrays, with one barrier
// per tier.  A launch-bound config: the table is 58 KB, far below any roofline.
#include "gm_internal.hpp"

namespace gm {

struct SmallDense {
    uint16_t *d_rec = nullptr;     // SLOTS records (0xFFFF = unreachable)
    uint32_t *d_info = nullptr;    // [0] error flags, [1] reachable count, [2] primitive count
    uint32_t slots = 0;
    std::vector<uint16_t> h_rec;   // host copy after solve
};

template <class D>
__global__ __launch_bounds__(1024) void small_dense_kernel(D d, uint64_t root, int max_tier,
                                                           uint16_t *__restrict__ out,
                                                           uint32_t *__restrict__ info) {
    constexpr uint32_t SLOTS = D::SLOTS;
    __shared__ uint16_t score[SLOTS];
    __shared__ uint8_t reach[SLOTS];
    __shared__ uint8_t tier[SLOTS];
    __shared__ uint32_t s_err, s_cnt, s_prim;
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < SLOTS; i += blockDim.x) {
        score[i] = 0;
        reach[i] = 0;
        tier[i] = (uint8_t)d.tier(i);
    }
    if (tid == 0) { s_err = 0; s_cnt = 0; s_prim = 0; }
    __syncthreads();
    if (tid == 0) reach[root] = 1;
    __syncthreads();
    const int t0 = (int)d.tier(root);
    uint64_t kids[D::MAXC];
    // forward: mark children of every reachable non-primitive position, tier by tier
    for (int t = t0; t <= max_tier; t++) {
        for (uint32_t i = tid; i < SLOTS; i += blockDim.x) {
            if (!reach[i] || tier[i] != t) continue;
            int p = d.primitive(i);
            if (p != UNDECIDED) {
                if (p == DRAW) atomicOr(&s_err, DEV_ERR_DRAW);
                score[i] = score_of_primitive(p);
                continue;
            }
            int n = d.children(i, kids);
            if (!n) atomicOr(&s_err, DEV_ERR_NOMOVES);
            for (int c = 0; c < n; c++) reach[(uint32_t)kids[c]] = 1;
        }
        __syncthreads();
    }
    // backward: deepest tier first
    for (int t = max_tier; t >= t0; t--) {
        for (uint32_t i = tid; i < SLOTS; i += blockDim.x) {
            if (!reach[i] || tier[i] != t || score[i]) continue;
            int n = d.children(i, kids);
            uint32_t best = 0;
            for (int c = 0; c < n; c++) best = max(best, (uint32_t)score[(uint32_t)kids[c]]);
            if (!best) atomicOr(&s_err, DEV_ERR_MISSING_CHILD);
            score[i] = parent_score(best);
        }
        __syncthreads();
    }
    uint32_t cnt = 0, prim = 0;
    for (uint32_t i = tid; i < SLOTS; i += blockDim.x) {
        out[i] = reach[i] ? record_of_score(score[i]) : REC_UNSOLVED;
        if (reach[i]) { cnt++; prim += d.primitive(i) != UNDECIDED; }
    }
    atomicAdd(&s_cnt, cnt);
    atomicAdd(&s_prim, prim);
    __syncthreads();
    if (tid == 0) { info[0] = s_err; info[1] = s_cnt; info[2] = s_prim; }
}

int small_dense_solve(Ctx *c, uint64_t root) {
    if (c->game != GM_GAME_TTT) { set_error("small dense engine supports tic-tac-toe only"); return GM_E_GAME; }
    SmallDense *s = c->sd;
    if (!s) {
        s = c->sd = new SmallDense();
        s->slots = DescTTT::SLOTS;
        GM_HIP(hipMalloc(&s->d_rec, s->slots * 2));
        GM_HIP(hipMalloc(&s->d_info, 16));
    }
    double t0 = now_ms();
    hipLaunchKernelGGL(small_dense_kernel<DescTTT>, dim3(1), dim3(1024), 0, c->stream, c->ttt, root, 9,
                       s->d_rec, s->d_info);
    GM_HIP(hipGetLastError());
    uint32_t info[4];
    s->h_rec.resize(s->slots);
    GM_HIP(hipMemcpyAsync(info, s->d_info, 12, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipMemcpyAsync(s->h_rec.data(), s->d_rec, s->slots * 2, hipMemcpyDeviceToHost, c->stream));
    GM_HIP(hipStreamSynchronize(c->stream));
    double t1 = now_ms();
    if (info[0]) return dev_error_to_gm(info[0]);
    c->n_positions = info[1];
    c->root_record = s->h_rec[root];
    c->tier_counts.assign(10, 0);
    for (uint32_t i = 0; i < s->slots; i++)
        if (s->h_rec[i] != REC_UNSOLVED) c->tier_counts[c->ttt.tier(i)]++;
    c->stats.n_positions = info[1];
    c->stats.n_primitive = info[2];
    c->stats.n_tiers = 10;
    c->stats.solve_ms = t1 - t0;
    c->stats.backward_ms = t1 - t0;
    c->stats.table_bytes = s->slots * 2;
    c->stats.algo_bytes = 0;
    return GM_OK;
}

int small_dense_export(Ctx *c, uint64_t *keys, uint16_t *recs, uint64_t cap, uint64_t *n) {
    SmallDense *s = c->sd;
    *n = c->n_positions;
    if (!keys) return GM_OK;
    if (cap < c->n_positions) { set_error("export buffer too small"); return GM_E_CAP; }
    uint64_t j = 0;
    for (uint32_t i = 0; i < s->slots; i++)
        if (s->h_rec[i] != REC_UNSOLVED) { keys[j] = i; recs[j] = s->h_rec[i]; j++; }
    return GM_OK;
}

int small_dense_query(Ctx *c, const uint64_t *keys, uint16_t *recs, uint64_t n) {
    SmallDense *s = c->sd;
    for (uint64_t i = 0; i < n; i++) recs[i] = keys[i] < s->slots ? s->h_rec[keys[i]] : REC_UNSOLVED;
    return GM_OK;
}

int small_dense_digest(Ctx *c, uint64_t *digest, uint64_t *n) {
    SmallDense *s = c->sd;
    uint64_t d = 0, k = 0;
    for (uint32_t i = 0; i < s->slots; i++)
        if (s->h_rec[i] != REC_UNSOLVED) { d += digest_term(i, s->h_rec[i]); k++; }
    *digest = d;
    *n = k;
    return GM_OK;
}

void small_dense_free(Ctx *c) {
    SmallDense *s = c->sd;
    if (!s) return;
    if (s->d_rec) hipFree(s->d_rec);
    if (s->d_info) hipFree(s->d_info);
    delete s;
    c->sd = nullptr;
}

}  // namespace gm
