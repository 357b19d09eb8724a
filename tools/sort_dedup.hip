// sort_dedup.hip -- the streaming alternative to the sparse engine's hash dedup
// (SURVEY §7.5 "dedup by sort+unique"), measured on
// Toot-and-Otto 6x4 with the same descriptor (csrc/games.hpp, mirror reduction on).
//
// Forward pass, per ply p, on sorted distinct keys K_p:
//   classify   primitive() per key; interior keys compacted (hipcub DeviceSelect::Flagged)
//   count      children per interior key -> exclusive scan -> offsets
//   expand     every child (canonical) written to C at its offset: 8 B per edge, streaming
//   sort       hipcub DeviceRadixSort::SortKeys on the 64-bit keys of C
//   unique     hipcub DeviceSelect::Unique -> K_{p+1}
// Checked: per-ply counts with every mirror orbit expanded = SURVEY Appendix D.  The
// time of these phases is compared with the hash engine's forward half (classify_kernel
// + expand_kernel, csrc/sparse.hip): the retrograde half of a sort-based engine would
// add a second sort (children by key with their parent's index) or random gathers on
// top, so if the forward half alone is slower the design loses.
//
//   hipcc -O3 --offload-arch=gfx950 -I include -I gamesmanmpi_amd/csrc tools/sort_dedup.hip -o tools/_bin/sort_dedup
//   tools/_bin/sort_dedup [L H]
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "games.hpp"

using namespace gm;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static const uint64_t APPENDIX_D_6x4[] = {1, 12, 114, 748, 4266, 19692, 81140, 285708, 928196, 2665424, 7098172,
                                          17010952, 37792450, 64636776, 100084356, 136321692, 169785424, 180777508,
                                          172831136, 135153280, 91440950, 45953432, 19196602, 4537828, 606968};

__global__ void classify_k(DescToot d, const uint64_t *__restrict__ keys, uint64_t n, uint8_t *__restrict__ interior,
                           uint32_t *__restrict__ nkids, unsigned long long *orbits) {
    uint64_t orb = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        d.orbit(k, [&](uint64_t) { orb++; });
        const bool in = d.primitive(k) == UNDECIDED;
        interior[i] = in;
        uint32_t c = 0;
        if (in) d.visit(k, [&](uint64_t) { c++; return true; });
        nkids[i] = c;
    }
    for (int o = 32; o > 0; o >>= 1) orb += __shfl_xor(orb, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(orbits, (unsigned long long)orb);
}

__global__ void expand_k(DescToot d, const uint64_t *__restrict__ keys, uint64_t n, const uint32_t *__restrict__ off,
                         uint64_t *__restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        if (d.primitive(k) != UNDECIDED) continue;
        uint64_t at = off[i];
        d.visit(k, [&](uint64_t c) { out[at++] = c; return true; });
    }
}

static unsigned grid(uint64_t n) { return (unsigned)std::min<uint64_t>((n + 255) / 256, 1u << 20); }

int main(int argc, char **argv) {
    const int L = argc > 2 ? atoi(argv[1]) : 6, H = argc > 2 ? atoi(argv[2]) : 4;
    DescToot d;
    if (!DescToot::make(L, H, &d)) { fprintf(stderr, "bad board\n"); return 1; }
    d.sym = 1;   // the root (empty board) is its own mirror image
    const uint64_t root = 0x6666;
    uint64_t cap = 64ull << 20;                 // grown as needed
    uint64_t *keys, *kids, *kids2, *next;
    uint8_t *interior;
    uint32_t *nkids, *off;
    unsigned long long *d_cnt;
    CK(hipMalloc(&d_cnt, 64));
    auto alloc_all = [&](uint64_t c) {
        CK(hipMalloc(&keys, c * 8)); CK(hipMalloc(&next, c * 8)); CK(hipMalloc(&interior, c));
        CK(hipMalloc(&nkids, c * 4)); CK(hipMalloc(&off, c * 4));
    };
    alloc_all(cap);
    uint64_t kcap = 64ull << 20;
    CK(hipMalloc(&kids, kcap * 8)); CK(hipMalloc(&kids2, kcap * 8));
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    auto ensure_tmp = [&](size_t b) {
        if (b <= tmp_bytes) return;
        if (tmp) CK(hipFree(tmp));
        CK(hipMalloc(&tmp, b));
        tmp_bytes = b;
    };
    hipEvent_t ev[8];
    for (auto &e : ev) CK(hipEventCreate(&e));
    double t_cls = 0, t_exp = 0, t_sort = 0, t_uniq = 0, t_scan = 0;
    uint64_t n = 1, edges = 0, total = 0;
    CK(hipMemcpy(keys, &root, 8, hipMemcpyHostToDevice));
    bool ok = true;
    for (int ply = 0; n; ply++) {
        CK(hipMemset(d_cnt, 0, 64));
        CK(hipEventRecord(ev[0]));
        hipLaunchKernelGGL(classify_k, dim3(grid(n)), dim3(256), 0, 0, d, keys, n, interior, nkids, d_cnt);
        CK(hipEventRecord(ev[1]));
        // offsets of every key's children (primitive keys have 0)
        size_t b = 0;
        CK(hipcub::DeviceScan::ExclusiveSum(nullptr, b, nkids, off, (int)n));
        ensure_tmp(b);
        CK(hipcub::DeviceScan::ExclusiveSum(tmp, b, nkids, off, (int)n));
        uint32_t last_off, last_n;
        CK(hipMemcpy(&last_off, off + n - 1, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&last_n, nkids + n - 1, 4, hipMemcpyDeviceToHost));
        unsigned long long orb;
        CK(hipMemcpy(&orb, d_cnt, 8, hipMemcpyDeviceToHost));
        CK(hipEventRecord(ev[2]));
        const uint64_t m = (uint64_t)last_off + last_n;
        if (ply < 25) {
            const bool good = orb == APPENDIX_D_6x4[ply] || !(L == 6 && H == 4);
            ok &= good;
            printf("ply %2d: %10llu keys (%10llu with mirror images%s), %10llu children\n", ply, (unsigned long long)n,
                   orb, good ? "" : " MISMATCH", (unsigned long long)m);
        }
        total += orb;
        edges += m;
        if (!m) break;
        if (m > kcap) {
            CK(hipFree(kids)); CK(hipFree(kids2));
            kcap = m + m / 4;
            CK(hipMalloc(&kids, kcap * 8)); CK(hipMalloc(&kids2, kcap * 8));
        }
        CK(hipEventRecord(ev[3]));
        hipLaunchKernelGGL(expand_k, dim3(grid(n)), dim3(256), 0, 0, d, keys, n, off, kids);
        CK(hipEventRecord(ev[4]));
        b = 0;
        CK(hipcub::DeviceRadixSort::SortKeys(nullptr, b, kids, kids2, (int)m, 0, 2 * d.A + 16));
        ensure_tmp(b);
        CK(hipcub::DeviceRadixSort::SortKeys(tmp, b, kids, kids2, (int)m, 0, 2 * d.A + 16));
        CK(hipEventRecord(ev[5]));
        if (m > cap) {
            for (void *p : {(void *)keys, (void *)next, (void *)interior, (void *)nkids, (void *)off}) CK(hipFree(p));
            cap = m + m / 4;
            alloc_all(cap);
        }
        b = 0;
        CK(hipcub::DeviceSelect::Unique(nullptr, b, kids2, next, d_cnt + 1, (int)m));
        ensure_tmp(b);
        CK(hipcub::DeviceSelect::Unique(tmp, b, kids2, next, d_cnt + 1, (int)m));
        CK(hipEventRecord(ev[6]));
        CK(hipEventSynchronize(ev[6]));
        unsigned long long nn;
        CK(hipMemcpy(&nn, d_cnt + 1, 8, hipMemcpyDeviceToHost));
        float a, bb, c, e, f;
        CK(hipEventElapsedTime(&a, ev[0], ev[1]));
        CK(hipEventElapsedTime(&bb, ev[1], ev[2]));
        CK(hipEventElapsedTime(&c, ev[3], ev[4]));
        CK(hipEventElapsedTime(&e, ev[4], ev[5]));
        CK(hipEventElapsedTime(&f, ev[5], ev[6]));
        t_cls += a; t_scan += bb; t_exp += c; t_sort += e; t_uniq += f;
        std::swap(keys, next);
        n = nn;
    }
    printf("positions %llu (Appendix D total 1187212827 for 6x4): %s\n", (unsigned long long)total,
           ok ? "per-ply counts match" : "MISMATCH");
    printf("edges %llu\n", (unsigned long long)edges);
    printf("forward ms: classify %.1f, scan %.1f, expand %.1f, radix sort %.1f, unique %.1f; total %.1f\n", t_cls,
           t_scan, t_exp, t_sort, t_uniq, t_cls + t_scan + t_exp + t_sort + t_uniq);
    printf("per edge: sort %.2f ns, expand %.2f ns\n", t_sort * 1e6 / edges, t_exp * 1e6 / edges);
    return ok ? 0 : 2;
}
