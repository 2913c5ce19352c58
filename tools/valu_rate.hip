// VALU issue-rate probe for the instruction mix of the fused decoder's check pass.
// Each lane runs NITER rounds of 8 independent chains (no memory traffic in the loop); the
// rate is wave-instructions per SIMD-cycle, computed from the measured time and the clock
// reported by hipDeviceProp.  Build: hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NITER = 65536;

template <int MIX>
__global__ void __launch_bounds__(256) k_mix(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
    uint32_t a[8], b[8], c[8];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = seed * (threadIdx.x + 1) + j;
        b[j] = a[j] ^ 0x5a5a5a5a;
        c[j] = a[j] * 3u;
    }
    for (int it = 0; it < NITER; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (MIX == 0) {            // plain v_add_u32
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 1) {     // v_med3_u32 (VOP3)
                asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            } else if (MIX == 2) {     // SDWA subtract, word/byte selects
                asm volatile("v_sub_u32_sdwa %0, sext(%0), sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_2"
                             : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 3) {     // v_perm_b32
                asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            } else if (MIX == 4) {     // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 5) {     // the pass-1 edge sequence: sdwa sub, neg, max, lshl_or, alignbit, min, med3
                uint32_t d, n, k;
                asm volatile("v_sub_u32_sdwa %0, sext(%1), sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_1"
                             : "=v"(d) : "v"(a[j]), "v"(b[j]));
                asm volatile("v_sub_u32 %0, 0, %1" : "=v"(n) : "v"(d));
                asm volatile("v_max_i32 %0, %1, %2" : "=v"(n) : "v"(d), "v"(n));
                asm volatile("v_lshl_or_b32 %0, %1, 8, 5" : "=v"(k) : "v"(n));
                asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(c[j]) : "v"(d));
                asm volatile("v_min_u32 %0, %0, %1" : "+v"(b[j]) : "v"(k));
                asm volatile("v_med3_u32 %0, %1, %0, %2" : "+v"(a[j]) : "v"(b[j]), "v"(k));
            } else if (MIX == 6) {     // dependent chain of v_add (one chain per lane)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[0]) : "v"(b[j]));
            } else if (MIX == 7) {     // VOP3 encoding of the same add
                asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 8) {     // VOP2 with a 32-bit literal (8-byte instruction)
                asm volatile("v_add_u32 %0, 0x12345, %0" : "+v"(a[j]));
            } else if (MIX == 9) {     // packed 16-bit (VOP3P)
                asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 10) {    // VOP2 with an SGPR operand
                asm volatile("v_and_b32 %0, %1, %0" : "+v"(a[j]) : "s"(seed));
            } else if (MIX == 11) {    // v_lshrrev (VOP2) + v_and (VOP2, SGPR): the unpack pair
                asm volatile("v_lshrrev_b32 %0, 16, %0" : "+v"(a[j]));
            } else if (MIX == 12) {    // VOP1 move
                asm volatile("v_not_b32 %0, %0" : "+v"(a[j]));
            } else if (MIX == 13) {    // v_min_u32 VOP2 / v_max_i32 mix
                asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 14) {    // v_pk_min_u16 (VOP3P)
                asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 15) {    // v_cndmask (VOP2, vcc)
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 16) {    // v_add3 (VOP3, 3 operands)
                asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            } else if (MIX == 17) {    // DPP row_shr (VOP2 + DPP word)
                asm volatile("v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 18) {    // 32 x 32 -> 64 multiply-add (Philox round product)
                uint64_t x = ((uint64_t)b[j] << 32) | a[j];
                uint64_t cy;
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(cy) : "v"(b[j]), "v"(c[j]));
                a[j] = (uint32_t)x ^ (uint32_t)(x >> 32);
            } else if (MIX == 19) {    // v_mul_hi_u32
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 20) {    // v_mul_lo_u32
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 21) {    // v_bitop3_b32 (VOP3, any 3-input boolean function)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            } else if (MIX == 22) {    // v_log_f32 (transcendental)
                asm volatile("v_log_f32 %0, %0" : "+v"(a[j]));
            } else if (MIX == 23) {    // v_bitop3_b32 with one SGPR operand
                asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x6c" : "+v"(a[j]) : "s"(seed), "v"(c[j]));
            } else if (MIX == 24) {    // v_mov_b32 from an SGPR (VOP1)
                asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "s"(seed + j));
            } else if (MIX == 25) {    // v_xor_b32 VGPR, VGPR (VOP2)
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 26) {    // v_and_b32 with an inline constant
                asm volatile("v_and_b32 %0, 0x7fff, %0" : "+v"(a[j]));
            } else if (MIX == 28) {    // DPP move, quad_perm, bound_ctrl (the lane-group merges)
                asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a[j]) : "v"(b[j]));
            } else if (MIX == 29) {    // VOP2 xor with a DPP quad_perm source (a folded DPP move)
                asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a[j]) : "v"(b[j]));
            } else if (MIX == 30) {    // v_mov_b32 of an inline constant (VOP1)
                asm volatile("v_mov_b32 %0, 0" : "=v"(a[j]));
            } else if (MIX == 31) {    // 1 DPP move + 3 v_bitop3 (the merge mix)
                asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(c[j]) : "v"(b[j]));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(b[j]) : "v"(a[j]), "v"(c[j]));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            } else if (MIX == 32) {    // a v_bitop3 and a dependent VOP2 xor
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(b[j]) : "v"(a[j]));
            } else if (MIX == 27) {    // ds_read_b128 broadcast (all lanes, same LDS address) + 2 bitop3
                // (LDS traffic in the VALU loop: the table-leaf alternative)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6c" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= a[j] ^ b[j] ^ c[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) atomicMax(cyc, t1 - t0);     // longest wave, shader clocks
}

template <int MIX>
void run(const char* name, int ops_per_j, int waves_per_simd, int ncu, double clk_ghz, uint32_t* d) {
    const int block = 256;                                  // 4 waves = 1 per SIMD
    const int grid = ncu * waves_per_simd;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    unsigned long long* cyc = reinterpret_cast<unsigned long long*>(d + (size_t)ncu * 8 * 256 * 2);
    hipLaunchKernelGGL(k_mix<MIX>, dim3(grid), dim3(block), 0, 0, d, 7u, cyc);
    hipMemset(cyc, 0, 8);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mix<MIX>, dim3(grid), dim3(block), 0, 0, d, 9u, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime counts shader-clock cycles: per SIMD, waves_per_simd waves shared the cycles
    const double per_simd_instr = (double)waves_per_simd * NITER * 8.0 * ops_per_j;
    printf("%-28s waves/SIMD %d  %8.3f ms  %6.2f shader cycles per wave-instr  (clock %.2f GHz)\n",
           name, waves_per_simd, ms, (double)c / per_simd_instr, (double)c / (ms * 1e6));
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    const double clk = p.clockRate / 1e6;                   // kHz -> GHz
    printf("%s  CUs %d  clock %.3f GHz (device max; the measured rate uses it)\n", p.name, ncu, clk);
    uint32_t* d;
    hipMalloc(&d, (size_t)ncu * 8 * 256 * 4 * 4);
    for (int w : {2, 6, 8}) {
        run<0>("v_add_u32", 1, w, ncu, clk, d);
        run<1>("v_med3_u32", 1, w, ncu, clk, d);
        run<2>("v_sub_u32_sdwa", 1, w, ncu, clk, d);
        run<3>("v_perm_b32", 1, w, ncu, clk, d);
        run<4>("v_alignbit_b32", 1, w, ncu, clk, d);
        run<5>("pass-1 edge (7 ops)", 7, w, ncu, clk, d);
        run<6>("dependent v_add chain", 1, w, ncu, clk, d);
        run<7>("v_add_u32_e64 (VOP3)", 1, w, ncu, clk, d);
        run<8>("v_add_u32 literal", 1, w, ncu, clk, d);
        run<9>("v_pk_add_u16", 1, w, ncu, clk, d);
        run<10>("v_and_b32 sgpr", 1, w, ncu, clk, d);
        run<11>("v_lshrrev_b32 imm", 1, w, ncu, clk, d);
        run<12>("v_not_b32 (VOP1)", 1, w, ncu, clk, d);
        run<13>("v_min_u32", 1, w, ncu, clk, d);
        run<14>("v_pk_min_u16", 1, w, ncu, clk, d);
        run<15>("v_cndmask_b32 vcc", 1, w, ncu, clk, d);
        run<16>("v_add3_u32", 1, w, ncu, clk, d);
        run<17>("v_add_u32_dpp", 1, w, ncu, clk, d);
        run<18>("v_mad_u64_u32 (+1 xor)", 2, w, ncu, clk, d);
        run<19>("v_mul_hi_u32", 1, w, ncu, clk, d);
        run<20>("v_mul_lo_u32", 1, w, ncu, clk, d);
        run<21>("v_bitop3_b32", 1, w, ncu, clk, d);
        run<22>("v_log_f32", 1, w, ncu, clk, d);
        run<23>("v_bitop3_b32 1 sgpr", 1, w, ncu, clk, d);
        run<24>("v_mov_b32 from sgpr", 1, w, ncu, clk, d);
        run<25>("v_xor_b32 vv", 1, w, ncu, clk, d);
        run<26>("v_and_b32 inline const", 1, w, ncu, clk, d);
        run<28>("v_mov_b32_dpp quad_perm", 1, w, ncu, clk, d);
        run<29>("v_xor_b32_dpp quad_perm", 1, w, ncu, clk, d);
        run<30>("v_mov_b32 0", 1, w, ncu, clk, d);
        run<31>("dpp mov + 3 bitop3", 4, w, ncu, clk, d);
        run<32>("bitop3 + v_xor (dependent)", 2, w, ncu, clk, d);
    }
    hipFree(d);
    return 0;
}
