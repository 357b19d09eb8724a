// l2sim_box.cpp -- CPU model of the L2 / Infinity-Cache traffic of a BOX-tiled dense
// solve (development aid, not part of the product).  The 8 nibble heaps are cut into
// boxes of sides s_i in {2, 4, 8} positions (so a child two below a position is at most
// one box below it); a box's children outside it lie in the 8 boxes one step below,
// whose top two layers in that dimension are read.  Boxes of one box-tier (sum of box
// indices) are independent, so a launch per box-tier reads only the previous one.
// Box layout: the hi bits of every dimension above the lo bits, so a halo slab of a
// side-4 dimension is a set of whole 256-B chunks; the model counts 256-B chunks.
//
//   g++ -O2 -o /tmp/l2sim_box tools/l2sim_box.cpp && /tmp/l2sim_box 44442222 [K] [order]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <unordered_map>
#include <vector>

struct LRU {
    size_t cap;
    std::list<uint64_t> q;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> m;
    explicit LRU(size_t c) : cap(c) { m.reserve(c * 2); }
    bool touch(uint64_t k) {
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

int main(int argc, char **argv) {
    const char *sides_s = argc > 1 ? argv[1] : "44442222";
    const int K = argc > 2 ? atoi(argv[2]) : 1;
    const int order = argc > 3 ? atoi(argv[3]) : 0;
    const size_t l2_bytes = argc > 4 ? atoll(argv[4]) : (4u << 20);
    int s[8], nb[8], lb[8];
    int box_pos = 1;
    for (int i = 0; i < 8; i++) {
        s[i] = sides_s[i] - '0';
        nb[i] = 16 / s[i];
        lb[i] = s[i] == 2 ? 1 : s[i] == 4 ? 2 : 3;
        box_pos *= s[i];
    }
    const int chunk = 256, nchunks = box_pos / chunk;
    // hi-bit mask of the box offset per dimension, in chunk-index bits: the offset's
    // low 8 bits are the lo bits; for a side-4 dimension the hi bit is one chunk bit,
    // for side 8 two hi bits (of which the top is a chunk bit: top two layers = 6,7 =
    // hi bits 11b -> a quarter), side 2 has no hi bit (whole box).
    // Build per dimension the list of chunks of the child box that a parent above reads.
    std::vector<std::vector<int>> halo(8);
    {
        // assign offset bits: first every dim's lowest bit, then second bits, then third
        std::vector<std::pair<int, int>> bits;   // (dim, bit index within dim)
        for (int lvl = 0; lvl < 3; lvl++)
            for (int i = 0; i < 8; i++)
                if (lb[i] > lvl) bits.push_back({i, lvl});
        // offset bit position of each (dim, lvl)
        int pos[8][3];
        for (size_t k = 0; k < bits.size(); k++) pos[bits[k].first][bits[k].second] = (int)k;
        for (int i = 0; i < 8; i++) {
            std::vector<char> need(nchunks, 0);
            for (int off = 0; off < box_pos; off++) {
                int c = 0;
                for (int l = 0; l < lb[i]; l++) c |= ((off >> pos[i][l]) & 1) << l;
                if (c >= s[i] - 2) need[off / chunk] = 1;
            }
            for (int q = 0; q < nchunks; q++) if (need[q]) halo[i].push_back(q);
        }
    }
    uint64_t nbox = 1;
    for (int i = 0; i < 8; i++) nbox *= nb[i];
    int maxt = 0;
    for (int i = 0; i < 8; i++) maxt += nb[i] - 1;
    std::vector<std::vector<uint32_t>> tiers(maxt + 1);
    auto coords = [&](uint32_t b, int *c) { for (int i = 0; i < 8; i++) { c[i] = b % nb[i]; b /= nb[i]; } };
    auto index = [&](const int *c) { uint32_t b = 0; for (int i = 7; i >= 0; i--) b = b * nb[i] + c[i]; return b; };
    for (uint32_t b = 0; b < nbox; b++) {
        int c[8], t = 0;
        coords(b, c);
        for (int i = 0; i < 8; i++) t += c[i];
        tiers[t].push_back(b);
    }
    auto key = [&](uint32_t b) -> uint64_t {
        int c[8];
        coords(b, c);
        if (order == 0) return b;
        uint32_t x[8];
        for (int i = 0; i < 8; i++) x[i] = c[i];
        if (order == 1) return hilbert(x, 8, 3);
        // order 2: Hilbert over the 7 dims other than the last (the last is fixed by the sum)
        return hilbert(x, 7, 3);
    };
    std::vector<LRU> l2(8, LRU(l2_bytes / chunk));
    LRU mall((256u << 20) / chunk);
    uint64_t l2m = 0, mm = 0, raw = 0, peak_t = 0;
    for (auto &t : tiers) {
        peak_t = std::max<uint64_t>(peak_t, t.size());
        std::stable_sort(t.begin(), t.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
        const uint32_t ng = (t.size() + K - 1) / K;
        std::vector<std::vector<uint32_t>> per(8);
        const uint32_t q = ng >> 3, r = ng & 7;
        for (uint32_t x = 0; x < 8; x++) {
            const uint32_t g0 = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q, len = x < r ? q + 1 : q;
            for (uint32_t g = g0; g < g0 + len; g++) per[x].push_back(g);
        }
        size_t mx = 0;
        for (auto &p : per) mx = std::max(mx, p.size());
        for (size_t i = 0; i < mx; i++)
            for (int x = 0; x < 8; x++) {
                if (i >= per[x].size()) continue;
                const uint32_t g = per[x][i];
                for (int k = 0; k < K; k++) {
                    const size_t idx = (size_t)g * K + k;
                    if (idx >= t.size()) continue;
                    int c[8];
                    coords(t[idx], c);
                    for (int d = 0; d < 8; d++) {
                        if (c[d] == 0) continue;
                        c[d]--;
                        const uint64_t cb = index(c);
                        c[d]++;
                        for (int qd : halo[d]) {
                            raw++;
                            const uint64_t line = cb * nchunks + qd;
                            if (!l2[x].touch(line)) {
                                l2m++;
                                if (!mall.touch(line)) mm++;
                            }
                        }
                    }
                }
                for (int k = 0; k < K; k++) {
                    const size_t idx = (size_t)g * K + k;
                    if (idx >= t.size()) continue;
                    for (int qd = 0; qd < nchunks; qd++) {
                        const uint64_t line = (uint64_t)t[idx] * nchunks + qd;
                        mall.touch(line);
                    }
                }
            }
    }
    const double pos = 4294967296.0;
    printf("sides %s K=%d order=%d L2=%zu KiB: box %d pos, %llu boxes, %d box-tiers (peak %llu boxes), "
           "in-box sub-tiers %d | halo reads %.2f B/pos, L2-miss %.2f B/pos, MALL-miss %.2f B/pos\n",
           sides_s, K, order, l2_bytes >> 10, box_pos, (unsigned long long)nbox, maxt + 1,
           (unsigned long long)peak_t, [&] { int st = 1; for (int i = 0; i < 8; i++) st += s[i] - 1; return st; }(),
           raw * (double)chunk / pos, l2m * (double)chunk / pos, mm * (double)chunk / pos);
    return 0;
}
