// child_at_check.cpp -- DescToot::child_at(k, j) against visit(k) on every position of a
// Toot-and-Otto board, with and without the mirror reduction (csrc/games.hpp; the
// sparse engine's MLP kernels make children with child_at, the others with visit).
//
//   /opt/rocm/lib/llvm/bin/clang++ -O2 -std=c++17 -include type_traits -I gamesmanmpi_amd/csrc \
//       tools/child_at_check.cpp -o tools/_bin/child_at_check
//   tools/_bin/child_at_check L H      -> "ok <positions> <edges>" or the first mismatch
#include "games.hpp"

#include <cstdio>
#include <cstdlib>
#include <unordered_set>
#include <vector>

using namespace gm;

int main(int argc, char **argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 4, H = argc > 2 ? atoi(argv[2]) : 3;
    DescToot d;
    if (!DescToot::make(L, H, &d)) { fprintf(stderr, "bad dims\n"); return 2; }
    uint64_t positions = 0, edges = 0;
    for (int sym = 0; sym < 2; sym++) {
        d.sym = sym;
        std::vector<uint64_t> ply = {0x6666ull};
        std::unordered_set<uint64_t> seen(ply.begin(), ply.end());
        while (!ply.empty()) {
            std::vector<uint64_t> next;
            for (uint64_t k : ply) {
                positions++;
                if (d.primitive(k) != UNDECIDED) continue;
                std::vector<uint64_t> a, b;
                d.visit(k, [&](uint64_t c) { a.push_back(c); return true; });
                for (int j = 0; j < DescToot::MAXC; j++) {
                    uint64_t c;
                    if (d.child_at(k, j, c)) b.push_back(c);
                }
                if (a != b) {
                    printf("mismatch at key %#llx (sym %d): visit %zu children, child_at %zu\n",
                           (unsigned long long)k, sym, a.size(), b.size());
                    return 1;
                }
                edges += a.size();
                for (uint64_t c : a)
                    if (seen.insert(c).second) next.push_back(c);
            }
            ply.swap(next);
        }
    }
    printf("ok %llu %llu\n", (unsigned long long)positions, (unsigned long long)edges);
    return 0;
}
