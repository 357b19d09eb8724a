// expand_dup_model.cpp -- how many of the sparse engine's child inserts would a
// workgroup-local (LDS) dedup remove?  Development aid for VERDICT r03 item 5.
//
//   /opt/rocm/lib/llvm/bin/clang++ -O2 -std=c++17 -include type_traits -I gamesmanmpi_amd/csrc \
//       tools/expand_dup_model.cpp -o tools/_bin/expand_dup_model
//   tools/_bin/expand_dup_model L H
//
// Enumerates Toot-and-Otto LxH ply by ply with the device descriptor's host twin
// (csrc/games.hpp, mirror reduction on as in the engine), and for each ply's interior
// positions, in the order expand_kernel sees them (the tier table's slot order: home
// slot = the hash of the key) and in two locality orders (ascending key; ascending key
// with the cells renumbered top row first, so positions that differ only in their top
// cells sit together), counts per batch of B consecutive parents the child inserts and
// the distinct children among them.  1 - distinct / inserts is the fraction an LDS hash
// over a B-parent batch would keep away from HBM (the engine's inserts are all random
// 64-B probes of a multi-GB table: DESIGN.md §4.2).
#include "games.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <unordered_set>
#include <vector>

using namespace gm;

int main(int argc, char **argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 5, H = argc > 2 ? atoi(argv[2]) : 4;
    DescToot d;
    if (!DescToot::make(L, H, &d)) { fprintf(stderr, "bad dims\n"); return 1; }
    d.sym = 1;   // the empty board is its own mirror image: the engine reduces
    const int A = L * H;
    // key with cells renumbered top row first (rows H-1 .. 0), planes and hands kept
    auto topfirst = [&](uint64_t k) {
        uint64_t r = k & 0xFFFFull;
        for (int plane = 0; plane < 2; plane++) {
            const uint32_t p = (uint32_t)(k >> (16 + plane * A)) & d.amask;
            uint32_t q = 0;
            for (int y = 0; y < H; y++) q |= ((p >> (L * y)) & ((1u << L) - 1u)) << (L * (H - 1 - y));
            r |= (uint64_t)q << (16 + plane * A);
        }
        return r;
    };
    const int B[] = {256, 1024, 4096, 65536};
    // bucketed orders: ascending key >> shift, hash order inside a bucket (one counting-sort
    // pass over the top bits instead of a full sort)
    const int shifts[] = {2 * A + 16 - 8, 2 * A + 16 - 12, 2 * A + 16 - 16, A + 16};
    constexpr int NO = 3 + 4;
    std::vector<uint64_t> ply = {0x6666ull};
    double tot_ins = 0, tot_dist = 0;
    double saved[NO][4] = {};
    for (int t = 0; !ply.empty(); t++) {
        std::vector<uint64_t> interior;
        for (uint64_t k : ply)
            if (d.primitive(k) == UNDECIDED) interior.push_back(k);
        std::vector<uint64_t> next;
        for (uint64_t k : interior) d.visit(k, [&](uint64_t c) { next.push_back(c); return true; });
        const double ins = (double)next.size();
        std::sort(next.begin(), next.end());
        next.erase(std::unique(next.begin(), next.end()), next.end());
        tot_ins += ins;
        tot_dist += (double)next.size();
        printf("ply %2d: %10zu positions, %10zu interior, %11.0f inserts, %10zu distinct (%.3f)", t, ply.size(),
               interior.size(), ins, next.size(), ins ? next.size() / ins : 0.0);
        for (int o = 0; o < NO; o++) {
            std::vector<uint64_t> ord = interior;
            auto hsh = [](uint64_t a) { const uint64_t m = mix64(a); return (m << 32) | (m >> 32); };
            if (o == 0)
                std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return hsh(a) < hsh(b); });
            else if (o == 2)
                std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return topfirst(a) < topfirst(b); });
            else if (o >= 3) {
                const int sh = shifts[o - 3];
                std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
                    return (a >> sh) != (b >> sh) ? (a >> sh) < (b >> sh) : hsh(a) < hsh(b);
                });
            }
            for (int bi = 0; bi < 4; bi++) {
                double dist = 0;
                std::unordered_set<uint64_t> seen;
                for (size_t i = 0; i < ord.size(); i += B[bi]) {
                    seen.clear();
                    for (size_t j = i; j < std::min(ord.size(), i + (size_t)B[bi]); j++)
                        d.visit(ord[j], [&](uint64_t c) { seen.insert(c); return true; });
                    dist += (double)seen.size();
                }
                saved[o][bi] += ins - dist;
            }
        }
        printf("\n");
        fflush(stdout);
        ply.swap(next);
    }
    printf("total inserts %.0f, distinct children %.0f (%.3f): duplicates %.3f of the inserts\n", tot_ins, tot_dist,
           tot_dist / tot_ins, 1 - tot_dist / tot_ins);
    const char *name[3] = {"slot (hash) order", "key order", "top-row-first key order"};
    for (int o = 0; o < NO; o++) {
        if (o < 3) printf("%-24s", name[o]);
        else printf("key >> %-2d, hash inside    ", shifts[o - 3]);
        for (int bi = 0; bi < 4; bi++) printf("  B=%-6d removes %.4f", B[bi], saved[o][bi] / tot_ins);
        printf("\n");
    }
    return 0;
}
