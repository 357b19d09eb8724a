// valu_issue_bench.hip -- issue cost of the box kernel's VALU instruction forms on gfx950
// (development aid): one wave (or two per SIMD) runs 8 independent streams of one
// instruction form, 256 x 8 instructions, timed with s_memtime; cycles per instruction.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/vib tools/valu_issue_bench.hip && /tmp/vib
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ void bench(unsigned long long *out, unsigned seed) {
    unsigned v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, v5 = v0 * 13,
             v6 = v0 * 17, v7 = v0 * 19, m = 0x00FF00FFu ^ threadIdx.x;
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int it = 0; it < 256; it++) {
#define V(i) v##i
        if constexpr (K == 0) {
#define OP(i) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %1" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 1) {
#define OP(i) asm volatile("v_and_b32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 2) {
#define OP(i) asm volatile("v_and_b32_sdwa %0, %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 3) {
#define OP(i) asm volatile("v_pk_mad_u16 %0, %0, 2, %1 op_sel_hi:[1,0,1]" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 4) {
#define OP(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 5) {
#define OP(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(V(i)) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 6) {
#define OP(i) asm volatile("v_pk_lshrrev_b16 %0, 7, %0 op_sel_hi:[0,1]" : "+v"(V(i)));
            REP8(OP)
#undef OP
        } else if constexpr (K == 7) {
#define OP(i) asm volatile("v_mov_b32_dpp %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(V(i)));
            REP8(OP)
#undef OP
        } else if constexpr (K == 8) {   // a dependent chain of v_pk_maximum3_f16 (latency)
#define OP(i) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %1" : "+v"(v0) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 9) {   // a dependent chain of v_and_b32_dpp (latency)
#define OP(i) asm volatile("v_and_b32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v0) : "v"(m));
            REP8(OP)
#undef OP
        } else if constexpr (K == 10) {  // a dependent chain of v_xor_b32 (latency)
#define OP(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v0) : "v"(m));
            REP8(OP)
#undef OP
        }
#undef V
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
    if ((v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7) == 0x12345679u) out[1023] = 1;   // keep the streams live
}

template <int K>
static void run(const char *name, unsigned long long *d, int blocks) {
    hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(64), 0, 0, d, 1u);
    hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(64), 0, 0, d, 2u);
    unsigned long long h[1024];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-34s blocks %5d: %.2f cycles per instruction per wave\n", name, blocks, h[0] / (256.0 * 8));
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 1024 * sizeof(unsigned long long));
    for (int blocks : {1, 1024, 2048}) {   // one wave; one and two waves per SIMD chip-wide
        run<0>("v_pk_maximum3_f16 (independent)", d, blocks);
        run<1>("v_and_b32_dpp (independent)", d, blocks);
        run<2>("v_and_b32_sdwa (independent)", d, blocks);
        run<3>("v_pk_mad_u16 (independent)", d, blocks);
        run<4>("v_perm_b32 (independent)", d, blocks);
        run<5>("v_xor_b32 (independent)", d, blocks);
        run<6>("v_pk_lshrrev_b16 (independent)", d, blocks);
        run<7>("v_mov_b32_dpp (independent)", d, blocks);
        run<8>("v_pk_maximum3_f16 (chain)", d, blocks);
        run<9>("v_and_b32_dpp (chain)", d, blocks);
        run<10>("v_xor_b32 (chain)", d, blocks);
    }
    hipFree(d);
    return 0;
}
