// Issue cost and dependent latency of the instructions a single-wave serial
// replay is built from (wg_lanes_serial.hip), one wave on an idle chip: for
// each instruction a stream of 16 independent copies (issue cost) and a chain
// of dependent ones (latency), 1024 times, timed with s_memtime.  Prints one
// JSON line: cycles per instruction.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

template <int K>
__global__ void __launch_bounds__(64) k_chain(unsigned long long *out, uint32_t seed) {
    uint32_t v0 = threadIdx.x + seed, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
    uint32_t s0 = __builtin_amdgcn_readfirstlane(seed), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    uint64_t q0 = ((uint64_t)s0 << 32) | s1, q1 = q0 + 5, q2 = q0 + 9, q3 = q0 + 17;
    const unsigned long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 1024; i++) {
        if (K == 0) asm volatile(R16("s_nop 0\n\t") ::: "scc");
        // SALU add: independent (4 registers round robin) / dependent
        if (K == 1) asm volatile(R4("s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\ts_add_u32 %3, %3, 1\n\t") : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) :: "scc");
        if (K == 2) asm volatile(R16("s_add_u32 %0, %0, 1\n\t") : "+s"(s0) :: "scc");
        // 64-bit bit ops: s_bitset0_b64 dependent on s_ff1_i32_b64 (the allocation pair)
        if (K == 3) asm volatile(R16("s_ff1_i32_b64 %1, %0\n\ts_bitset0_b64 %0, %1\n\t") : "+s"(q0), "+s"(s0) :: "scc");
        if (K == 4) asm volatile(R4("s_bitset1_b64 %0, 3\n\ts_bitset1_b64 %1, 5\n\ts_bitset1_b64 %2, 7\n\ts_bitset1_b64 %3, 9\n\t") : "+s"(q0), "+s"(q1), "+s"(q2), "+s"(q3) :: "scc");
        // VALU add: independent / dependent
        if (K == 5) asm volatile(R4("v_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\t") : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
        if (K == 6) asm volatile(R16("v_add_u32 %0, 1, %0\n\t") : "+v"(v0));
        // v_readlane (constant lane) independent
        if (K == 7) asm volatile(R4("v_readlane_b32 %0, %4, 1\n\tv_readlane_b32 %1, %4, 2\n\tv_readlane_b32 %2, %4, 3\n\tv_readlane_b32 %3, %4, 4\n\t") : "=s"(s0), "=s"(s1), "=s"(s2), "=s"(s3) : "v"(v0) : "scc");
        // v_writelane (M0 lane select, set once) independent destinations
        if (K == 8) asm volatile("s_mov_b32 m0, 5\n\t" R4("v_writelane_b32 %0, %4, m0\n\tv_writelane_b32 %1, %4, m0\n\tv_writelane_b32 %2, %4, m0\n\tv_writelane_b32 %3, %4, m0\n\t") : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3) : "s"(s0) : "m0", "scc");
        // v_cmp to an SGPR pair, independent
        if (K == 9) asm volatile(R4("v_cmp_gt_u32_e64 %0, %4, %5\n\tv_cmp_gt_u32_e64 %1, %4, %5\n\tv_cmp_gt_u32_e64 %2, %4, %5\n\tv_cmp_gt_u32_e64 %3, %4, %5\n\t") : "=s"(q0), "=s"(q1), "=s"(q2), "=s"(q3) : "s"(s0), "v"(v0) : "scc");
        // VALU -> SALU -> VALU: v_cmp -> s_ff1 (M0) -> v_writelane of the compared register
        if (K == 10) asm volatile(R16("v_cmp_gt_u32_e64 %1, %2, %0\n\ts_ff1_i32_b64 m0, %1\n\tv_writelane_b32 %0, %2, m0\n\t") : "+v"(v0), "=&s"(q0) : "s"(s0) : "m0", "scc");
        // the same with the subtract in front (the unpipelined serial step)
        if (K == 11) asm volatile(R16("v_subrev_u32 %3, %2, %0\n\tv_cmp_gt_u32_e64 %1, %2, %3\n\ts_ff1_i32_b64 m0, %1\n\tv_writelane_b32 %0, %2, m0\n\t") : "+v"(v0), "=&s"(q0), "+s"(s0), "=&v"(v1) :: "m0", "scc");
        // SALU -> VALU: s_ff1 into M0, v_writelane; chain through the SGPR pair the next ff1 reads
        if (K == 12) asm volatile(R16("s_ff1_i32_b64 m0, %1\n\ts_bitset0_b64 %1, m0\n\tv_writelane_b32 %0, %2, m0\n\t") : "+v"(v0), "+s"(q0) : "s"(s0) : "m0", "scc");
        // v_readfirstlane dependent on a VALU write (the VALU -> SALU turnaround)
        if (K == 13) asm volatile(R16("v_add_u32 %0, %1, %0\n\ts_nop 0\n\tv_readfirstlane_b32 %1, %0\n\t") : "+v"(v0), "+s"(s0) :: "scc");
    }
    const unsigned long long t1 = clock64();
    if (threadIdx.x == 0) out[K] = t1 - t0;
    if (threadIdx.x == 0) out[32 + K] = v0 + v1 + v2 + v3 + s0 + s1 + s2 + s3 + (uint32_t)(q0 ^ q1 ^ q2 ^ q3);
}

template <int K>
static void run(unsigned long long *d) {
    hipLaunchKernelGGL(k_chain<K>, dim3(1), dim3(64), 0, 0, d, 7u);
    hipLaunchKernelGGL(k_chain<K>, dim3(1), dim3(64), 0, 0, d, 7u);
}

int main() {
    unsigned long long *d, h[64];
    if (hipMalloc(&d, 64 * 8) != hipSuccess) return 1;
    run<0>(d); run<1>(d); run<2>(d); run<3>(d); run<4>(d); run<5>(d); run<6>(d); run<7>(d);
    run<8>(d); run<9>(d); run<10>(d); run<11>(d); run<12>(d); run<13>(d);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    // instructions per repetition of each kernel's body
    const double per[14] = {16, 16, 16, 32, 16, 16, 16, 16, 16, 16, 48, 64, 48, 48};
    const char *names[14] = {"s_nop", "salu_indep", "salu_dep", "ff1_bitset0_dep(pair)", "bitset1_b64_indep", "valu_indep",
                             "valu_dep", "readlane_indep", "writelane_m0_indep", "vcmp_sgpr_indep",
                             "cmp_ff1_writelane_dep(triple)", "sub_cmp_ff1_writelane_dep(quad)", "ff1_bitset0_writelane(triple)",
                             "vadd_nop_readfirstlane(triple)"};
    printf("{\"unit\": \"cycles per instruction (chains: per instruction of the chain)\"");
    for (int k = 0; k < 14; k++) printf(", \"%s\": %.2f", names[k], (double)h[k] / (1024.0 * per[k]));
    printf("}\n");
    return 0;
}
