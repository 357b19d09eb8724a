// l2sim.cpp -- CPU model of the dense tier kernel's L2 / Infinity-Cache traffic
// (development aid, not part of the product).  For the 2^32 game (LOW = 3, HIGH = 5)
// it replays, tier by tier, the child-block reads and block writes of every
// workgroup in dispatch order (workgroup b on XCD b % 8, group index from
// xcd_order), through one LRU per XCD (the 4 MiB L2, in 4 KiB blocks) and one LRU
// shared by all XCDs (the 256 MiB Infinity Cache).  Prints L2-miss bytes (the
// FETCH_SIZE analogue) and Infinity-Cache-miss bytes per position for each
// block order.
//
//   g++ -O2 -o /tmp/l2sim tools/l2sim.cpp && /tmp/l2sim [l2_blocks] [mall_blocks]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <list>
#include <unordered_map>
#include <vector>

struct LRU {
    size_t cap;
    std::list<uint32_t> q;
    std::unordered_map<uint32_t, std::list<uint32_t>::iterator> m;
    explicit LRU(size_t c) : cap(c) { m.reserve(c * 2); }
    bool touch(uint32_t k) {   // true = hit
        auto it = m.find(k);
        if (it != m.end()) {
            q.splice(q.begin(), q, it->second);
            return true;
        }
        q.push_front(k);
        m[k] = q.begin();
        if (q.size() > cap) {
            m.erase(q.back());
            q.pop_back();
        }
        return false;
    }
};

static const int HIGH = 5;
static int nib(uint32_t v, int j) { return (v >> (4 * j)) & 15; }
static int tsum(uint32_t v) { int s = 0; for (int j = 0; j < HIGH; j++) s += nib(v, j); return s; }
static uint32_t morton(uint32_t v, const int *dims, int nd) {
    uint32_t m = 0;
    for (int b = 0; b < 4; b++)
        for (int j = 0; j < nd; j++) m |= ((v >> (4 * dims[j] + b)) & 1u) << (b * nd + j);
    return m;
}
static uint32_t xcd_order(uint32_t b, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

struct Result { double l2_miss, mall_miss; };

// order: sort key per block within a tier; groups of K blocks; xcd: whether runs per XCD
static bool g_write_alloc = true;
static bool g_flush = false;   // empty every L2 at each launch boundary
static int g_layer = -1;       // >= 0: each XCD run re-walked layer by layer in this nibble (order 3)
static uint64_t hilbert(const uint32_t *xin, int n, int b);
static uint64_t layer_key(uint32_t v) {
    uint32_t x[3];
    for (int j = 0, k = 0; j < 4 && k < 3; j++) if (j != g_layer) x[k++] = nib(v, j);
    const uint32_t layer = nib(v, g_layer);
    const uint64_t h = hilbert(x, 3, 4);
    return ((uint64_t)layer << 32) | (layer & 1u ? ~h & 0xFFFFFFFFull : h);
}
// Skilling's transpose form of the n-dimensional Hilbert index (b bits per axis)
static uint64_t hilbert(const uint32_t *xin, int n, int b) {
    uint32_t x[8];
    for (int i = 0; i < n; i++) x[i] = xin[i];
    const uint32_t M = 1u << (b - 1);
    for (uint32_t Q = M; Q > 1; Q >>= 1) {
        const uint32_t P = Q - 1;
        for (int i = 0; i < n; i++) {
            if (x[i] & Q) x[0] ^= P;
            else { uint32_t t = (x[0] ^ x[i]) & P; x[0] ^= t; x[i] ^= t; }
        }
    }
    for (int i = 1; i < n; i++) x[i] ^= x[i - 1];
    uint32_t t = 0;
    for (uint32_t Q = M; Q > 1; Q >>= 1) if (x[n - 1] & Q) t ^= Q - 1;
    for (int i = 0; i < n; i++) x[i] ^= t;
    uint64_t h = 0;
    for (int bit = b - 1; bit >= 0; bit--)
        for (int i = 0; i < n; i++) h = (h << 1) | ((x[i] >> bit) & 1u);
    return h;
}
static Result run(std::function<uint64_t(uint32_t)> key, size_t l2cap, size_t mallcap, int K = 4,
                  std::function<uint32_t(uint32_t, uint32_t)> place = nullptr, int window = 1) {
    const uint32_t nh = 1u << (4 * HIGH);
    std::vector<std::vector<uint32_t>> tiers(15 * HIGH + 1);
    for (uint32_t v = 0; v < nh; v++) tiers[tsum(v)].push_back(v);
    std::vector<LRU> l2(8, LRU(l2cap));
    LRU mall(mallcap);
    uint64_t l2m = 0, mm = 0;
    for (auto &t : tiers) {
        if (g_flush)
            for (auto &l : l2) { l.q.clear(); l.m.clear(); }
        std::stable_sort(t.begin(), t.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
        const uint32_t ng = (t.size() + K - 1) / K;
        if (g_layer >= 0) {
            const uint32_t q = ng >> 3, r = ng & 7;
            for (uint32_t x = 0; x < 8; x++) {
                const uint32_t g0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = x < r ? q + 1 : q;
                if (!len) continue;
                const size_t b0 = (size_t)K * g0, b1 = std::min(t.size(), (size_t)K * (g0 + len));
                std::stable_sort(t.begin() + b0, t.begin() + b1, [](uint32_t a, uint32_t b) { return layer_key(a) < layer_key(b); });
            }
        }
        // per XCD, the groups in dispatch order
        std::vector<std::vector<uint32_t>> per(8);
        for (uint32_t b = 0; b < ng; b++) {
            uint32_t g = place ? place(b, ng) : xcd_order(b, ng);
            per[b & 7].push_back(g);
        }
        // interleave XCDs in time (round-robin), each XCD sequential
        size_t mx = 0;
        for (auto &p : per) mx = std::max(mx, p.size());
        for (size_t i = 0; i < mx; i++)
            for (int x = 0; x < 8; x++) {
                if (i >= per[x].size()) continue;
                const uint32_t g = per[x][i];
                for (int k = 0; k < K; k++) {
                    const uint32_t idx = g * K + k;
                    if (idx >= t.size()) continue;
                    const uint32_t hp = t[idx];
                    for (int j = 0; j < HIGH; j++)
                        for (int s = 1; s <= 2; s++) {
                            if (nib(hp, j) < s) continue;
                            const uint32_t ch = hp - ((uint32_t)s << (4 * j));
                            if (!l2[x].touch(ch)) {
                                l2m++;
                                if (!mall.touch(ch)) mm++;
                            }
                        }
                }
                for (int k = 0; k < K; k++) {
                    const uint32_t idx = g * K + k;
                    if (idx >= t.size()) continue;
                    if (g_write_alloc) l2[x].touch(t[idx]);
                    mall.touch(t[idx]);
                }
            }
    }
    const double pos = (double)nh * 4096.0;
    return Result{(double)l2m * 4096.0 / pos, (double)mm * 4096.0 / pos};
}

// XCD chosen per block by `region`, each XCD's blocks in `key` order, groups of K
static Result run_regions(std::function<int(uint32_t)> region, std::function<uint64_t(uint32_t)> key, size_t l2cap,
                          size_t mallcap, double *imbalance, int K = 4) {
    const uint32_t nh = 1u << (4 * HIGH);
    std::vector<std::vector<uint32_t>> tiers(15 * HIGH + 1);
    for (uint32_t v = 0; v < nh; v++) tiers[tsum(v)].push_back(v);
    std::vector<LRU> l2(8, LRU(l2cap));
    LRU mall(mallcap);
    uint64_t l2m = 0, mm = 0;
    double wsum = 0, wmax = 0;
    for (auto &t : tiers) {
        std::vector<std::vector<uint32_t>> per(8);
        for (uint32_t v : t) per[region(v)].push_back(v);
        size_t mx = 0;
        for (auto &p : per) {
            std::stable_sort(p.begin(), p.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
            mx = std::max(mx, p.size());
        }
        wsum += (double)t.size() / 8;
        wmax += (double)mx;
        for (size_t i = 0; i < mx; i += K)
            for (int x = 0; x < 8; x++) {
                for (size_t k = i; k < std::min(i + K, per[x].size()); k++) {
                    const uint32_t hp = per[x][k];
                    for (int j = 0; j < HIGH; j++)
                        for (int s = 1; s <= 2; s++) {
                            if (nib(hp, j) < s) continue;
                            const uint32_t ch = hp - ((uint32_t)s << (4 * j));
                            if (!l2[x].touch(ch)) {
                                l2m++;
                                if (!mall.touch(ch)) mm++;
                            }
                        }
                }
                for (size_t k = i; k < std::min(i + K, per[x].size()); k++) {
                    l2[x].touch(per[x][k]);
                    mall.touch(per[x][k]);
                }
            }
    }
    *imbalance = wmax / wsum;
    const double pos = (double)nh * 4096.0;
    return Result{(double)l2m * 4096.0 / pos, (double)mm * 4096.0 / pos};
}

int main(int argc, char **argv) {
    size_t l2cap = argc > 1 ? atoi(argv[1]) : 1024, mallcap = argc > 2 ? atoi(argv[2]) : 65536;
    const int all5[5] = {0, 1, 2, 3, 4};
    auto show = [&](const char *name, Result r) {
        printf("%-44s L2-miss %.2f B/pos  MALL-miss %.2f B/pos\n", name, r.l2_miss, r.mall_miss);
        fflush(stdout);
    };
    double imb = 0;
    if (argc > 3 && argv[3][0] == 'K') {   // blocks per workgroup sharing child loads
        auto hil4 = [&](uint32_t v) { uint32_t x[4] = {(uint32_t)nib(v, 0), (uint32_t)nib(v, 1), (uint32_t)nib(v, 2), (uint32_t)nib(v, 3)}; return hilbert(x, 4, 4); };
        for (int K : {4, 8, 16, 32}) {
            char nm[64];
            snprintf(nm, sizeof nm, "hilbert 4D, %d blocks per workgroup", K);
            show(nm, run(hil4, l2cap, mallcap, K));
        }
        return 0;
    }
    if (argc > 3 && argv[3][0] == 'L') {   // the order-3 comparison only
        auto hil4 = [&](uint32_t v) { uint32_t x[4] = {(uint32_t)nib(v, 0), (uint32_t)nib(v, 1), (uint32_t)nib(v, 2), (uint32_t)nib(v, 3)}; return hilbert(x, 4, 4); };
        show("hilbert 4D (h0..h3)", run(hil4, l2cap, mallcap));
        for (g_layer = 0; g_layer < 5; g_layer++) {
            char nm[64];
            snprintf(nm, sizeof nm, "hilbert 4D runs, layered in h%d", g_layer);
            show(nm, run(hil4, l2cap, mallcap));
        }
        return 0;
    }
    auto lt = [](uint32_t v, int a, int b) { return nib(v, a) < nib(v, b) || (nib(v, a) == nib(v, b) && (nib(v, 0) + nib(v, 1) + nib(v, 2) + nib(v, 3) + nib(v, 4)) % 2); };
    auto reg_cmp = [&](uint32_t v) {
        int s12 = nib(v, 0) + nib(v, 1), s34 = nib(v, 2) + nib(v, 3);
        return (int)lt(v, 0, 1) | ((int)lt(v, 2, 3) << 1) | ((int)(s12 < s34 || (s12 == s34 && nib(v, 4) % 2)) << 2);
    };
    Result r = run_regions(reg_cmp, [&](uint32_t v) { return (uint64_t)morton(v, all5, 5); }, l2cap, mallcap, &imb);
    printf("regions cmp(h0<h1, h2<h3, h0+h1<h2+h3), morton: L2-miss %.2f MALL-miss %.2f imbalance %.3f\n", r.l2_miss, r.mall_miss, imb);
    auto reg_split = [&](uint32_t v) { return (nib(v, 0) >> 3) | ((nib(v, 1) >> 3) << 1) | ((nib(v, 2) >> 3) << 2); };
    r = run_regions(reg_split, [&](uint32_t v) { return (uint64_t)morton(v, all5, 5); }, l2cap, mallcap, &imb);
    printf("regions split h0,h1,h2 halves, morton:       L2-miss %.2f MALL-miss %.2f imbalance %.3f\n", r.l2_miss, r.mall_miss, imb);
    if (argc > 3) {
        show("morton (current)", run([&](uint32_t v) { return (uint64_t)morton(v, all5, 5); }, l2cap, mallcap));
        auto hil4 = [&](uint32_t v) { uint32_t x[4] = {(uint32_t)nib(v, 0), (uint32_t)nib(v, 1), (uint32_t)nib(v, 2), (uint32_t)nib(v, 3)}; return hilbert(x, 4, 4); };
        show("hilbert 4D (h0..h3)", run(hil4, l2cap, mallcap));
        for (g_layer = 0; g_layer < 5; g_layer++) {
            char nm[64];
            snprintf(nm, sizeof nm, "hilbert 4D runs, layered in h%d", g_layer);
            show(nm, run(hil4, l2cap, mallcap));
        }
        g_layer = -1;
        auto hil5 = [&](uint32_t v) { uint32_t x[5]; for (int j = 0; j < 5; j++) x[j] = nib(v, j); return hilbert(x, 5, 4); };
        show("hilbert 5D", run(hil5, l2cap, mallcap));
        auto mor4 = [&](uint32_t v) { const int d4[4] = {0, 1, 2, 3}; return (uint64_t)morton(v, d4, 4); };
        show("morton 4D (h0..h3)", run(mor4, l2cap, mallcap));
        g_flush = true;
        show("hilbert 4D, L2 flushed per launch", run(hil4, l2cap, mallcap));
        g_flush = false;
        g_write_alloc = false;
        show("morton, stores not allocating in L2", run([&](uint32_t v) { return (uint64_t)morton(v, all5, 5); }, l2cap, mallcap));
        show("hilbert 4D, stores not allocating", run(hil4, l2cap, mallcap));
        return 0;
    }
    show("key order", run([](uint32_t v) { return (uint64_t)v; }, l2cap, mallcap));
    show("morton (current)", run([&](uint32_t v) { return (uint64_t)morton(v, all5, 5); }, l2cap, mallcap));
    for (int major = 0; major < 5; major += 4) {
        int rest[4], n = 0;
        for (int j = 0; j < 5; j++) if (j != major) rest[n++] = j;
        char nm[64];
        snprintf(nm, sizeof nm, "h%d-major, morton rest", major);
        show(nm, run([&](uint32_t v) { return ((uint64_t)nib(v, major) << 32) | morton(v, rest, 4); }, l2cap, mallcap));
    }
    return 0;
}
