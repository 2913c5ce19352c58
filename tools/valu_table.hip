// VALU issue cost per instruction on gfx950: each lane runs NITER rounds of 8 independent
// chains of one instruction (no memory traffic).  Prints shader cycles per wave-instruction per
// SIMD at 2 and 6 waves/SIMD.  Build: hipcc --offload-arch=gfx950 -O3 tools/valu_table.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NITER = 16384;

template <int MIX>
__global__ void __launch_bounds__(256) k_mix(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
    extern __shared__ uint32_t lds_dummy[];
    (void)lds_dummy;
    uint32_t a[8], b[8], c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = seed * (threadIdx.x + 1) + j;
        b[j] = (a[j] ^ 0x5a5a5a5a) & 0x1f;
        c[j] = a[j] * 3u;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NITER; ++it) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (false) {}
        else if (MIX == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 1) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 2) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 3) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 4) asm volatile("v_or_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 5) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 6) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 7) asm volatile("v_max_i32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 8) asm volatile("v_min_i32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 9) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 10) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 11) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 12) asm volatile("v_lshlrev_b32 %0, 8, %0" : "+v"(a[j]));
        else if (MIX == 13) asm volatile("v_ashrrev_i32 %0, 24, %0" : "+v"(a[j]));
        else if (MIX == 14) asm volatile("v_and_b32 %0, 0xff, %0" : "+v"(a[j]));
        else if (MIX == 15) asm volatile("v_and_b32 %0, 63, %0" : "+v"(a[j]));
        else if (MIX == 16) asm volatile("v_add_u32 %0, 5, %0" : "+v"(a[j]));
        else if (MIX == 17) asm volatile("v_min_u32 %0, 5, %0" : "+v"(a[j]));
        else if (MIX == 18) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 19) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 20) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(a[j]));
        else if (MIX == 21) asm volatile("v_bfe_i32 %0, %0, 8, 8" : "+v"(a[j]));
        else if (MIX == 22) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 23) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 24) asm volatile("v_add_lshl_u32 %0, %0, %1, 1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 25) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 26) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 27) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 28) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 29) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 30) asm volatile("v_sad_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 31) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 33) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 34) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 35) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 36) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(a[j]));
        else if (MIX == 37) asm volatile("v_rndne_f32 %0, %0" : "+v"(a[j]));
        else if (MIX == 38) asm volatile("v_mov_b32 %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 39) { uint64_t t = ((uint64_t)a[j] << 32) | b[j]; asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(t) : "v"(((uint64_t)c[j]<<32)|b[j])); a[j] ^= (uint32_t)t; }
        else if (MIX == 40) asm volatile("v_add_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 41) asm volatile("v_max_i16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 42) asm volatile("v_sub_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 43) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 44) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 45) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 46) asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 47) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 48) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 49) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 50) asm volatile("v_min_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 51) asm volatile("v_max_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 52) asm volatile("v_min_i16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 53) asm volatile("v_sub_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 54) asm volatile("v_subrev_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 55) asm volatile("v_lshlrev_b16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 56) asm volatile("v_lshrrev_b16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 57) asm volatile("v_ashrrev_i16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 58) asm volatile("v_mul_lo_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 59) asm volatile("v_max_u32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 60) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 61) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 62) asm volatile("v_cmp_gt_u32 vcc, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 63) asm volatile("v_fmac_f32 %0, %1, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 64) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 65) asm volatile("v_sub_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 66) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 67) asm volatile("v_add_f16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 68) asm volatile("v_max_f16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 69) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a[j]));
        else if (MIX == 70) asm volatile("v_not_b32 %0, %0" : "+v"(a[j]));
        else if (MIX == 71) asm volatile("v_ffbh_u32 %0, %0" : "+v"(a[j]));
        else if (MIX == 72) asm volatile("v_bfrev_b32 %0, %0" : "+v"(a[j]));
        else if (MIX == 73) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 74) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 75) asm volatile("v_sub_u32_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 76) asm volatile("v_min_u32_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 77) asm volatile("v_max_i16_e64 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 78) asm volatile("v_pk_sub_u16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 79) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 80) asm volatile("v_pk_mad_u16 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 81) asm volatile("v_pk_lshlrev_b16 %0, %1, %0" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 82) asm volatile("v_lshl_or_b32 %0, %0, 8, %1" : "+v"(a[j]) : "v"(b[j]) : "vcc");
        else if (MIX == 83) asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(8)" : "+v"(a[j]) : "v"(b[j] * 4u + (threadIdx.x & 63u) * 64u));
        else if (MIX == 84) asm volatile("ds_read_u16_d16_hi %0, %1\n s_waitcnt lgkmcnt(8)" : "+v"(a[j]) : "v"(b[j] * 4u + (threadIdx.x & 63u) * 64u));
        else if (MIX == 85) asm volatile("ds_add_u32 %1, %0\n s_waitcnt lgkmcnt(8)" : "+v"(a[j]) : "v"(b[j] * 4u + (threadIdx.x & 63u) * 64u));
        else if (MIX == 86) asm volatile("v_sad_u16 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 87) asm volatile("v_med3_u16 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 88) asm volatile("v_sad_u8 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 89) asm volatile("v_sad_u16 %0, %0, %1, 17" : "+v"(a[j]) : "v"(b[j]));
        else if (MIX == 90) asm volatile("v_max3_u32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 91) asm volatile("v_med3_i16 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        else if (MIX == 92) asm volatile("v_sub_u32_sdwa %0, sext(%0), sext(%1) dst_sel:BYTE_1 dst_unused:UNUSED_SEXT src0_sel:WORD_1 src1_sel:BYTE_2" : "+v"(a[j]) : "v"(b[j]));
        else if (MIX == 93) asm volatile("v_msad_u8 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b[j]), "v"(c[j]));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) r ^= a[j] ^ b[j] ^ c[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) atomicMax(cyc, t1 - t0);
}

template <int MIX>
void run(const char* name, int ncu, uint32_t* d) {
    printf("%-26s", name);
    for (int w : {1, 2, 6}) {
        unsigned long long* cyc = reinterpret_cast<unsigned long long*>(d + (size_t)ncu * 8 * 256 * 2);
        hipLaunchKernelGGL(k_mix<MIX>, dim3(ncu * w), dim3(256), 8192, 0, d, 7u, cyc);
        hipMemset(cyc, 0, 8);
        hipLaunchKernelGGL(k_mix<MIX>, dim3(ncu * w), dim3(256), 8192, 0, d, 9u, cyc);
        hipDeviceSynchronize();
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("  w%d %6.2f", w, (double)c / ((double)w * NITER * 8.0));
    }
    printf("\n");
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    uint32_t* d;
    hipMalloc(&d, (size_t)ncu * 8 * 256 * 4 * 4);
    printf("shader cycles per wave-instruction per SIMD (w = waves/SIMD)\n");
    run<0>("v_add_u32 vv", ncu, d);
    run<1>("v_sub_u32 vv", ncu, d);
    run<2>("v_subrev_u32 vv", ncu, d);
    run<3>("v_and_b32 vv", ncu, d);
    run<4>("v_or_b32 vv", ncu, d);
    run<5>("v_xor_b32 vv", ncu, d);
    run<6>("v_min_u32 vv", ncu, d);
    run<7>("v_max_i32 vv", ncu, d);
    run<8>("v_min_i32 vv", ncu, d);
    run<9>("v_lshlrev_b32 vv", ncu, d);
    run<10>("v_lshrrev_b32 vv", ncu, d);
    run<11>("v_ashrrev_i32 vv", ncu, d);
    run<12>("v_lshlrev_b32 imm", ncu, d);
    run<13>("v_ashrrev_i32 imm", ncu, d);
    run<14>("v_and_b32 imm", ncu, d);
    run<15>("v_and_b32 inl", ncu, d);
    run<16>("v_add_u32 inl", ncu, d);
    run<17>("v_min_u32 inl", ncu, d);
    run<18>("v_mul_u32_u24", ncu, d);
    run<19>("v_mul_lo_u32", ncu, d);
    run<20>("v_bfe_u32", ncu, d);
    run<21>("v_bfe_i32", ncu, d);
    run<22>("v_lshl_or_b32", ncu, d);
    run<23>("v_lshl_add_u32", ncu, d);
    run<24>("v_add_lshl_u32", ncu, d);
    run<25>("v_and_or_b32", ncu, d);
    run<26>("v_or3_b32", ncu, d);
    run<27>("v_max3_i32", ncu, d);
    run<28>("v_min3_u32", ncu, d);
    run<29>("v_mad_u32_u24", ncu, d);
    run<30>("v_sad_u32", ncu, d);
    run<31>("v_bcnt_u32_b32", ncu, d);
    run<32>("v_add_f32", ncu, d);
    run<33>("v_fma_f32", ncu, d);
    run<34>("v_max_f32", ncu, d);
    run<35>("v_med3_f32", ncu, d);
    run<36>("v_cvt_f32_i32", ncu, d);
    run<37>("v_rndne_f32", ncu, d);
    run<38>("v_mov_b32", ncu, d);
    run<39>("v_pk_add_f32", ncu, d);
    run<40>("v_add_u16", ncu, d);
    run<41>("v_max_i16", ncu, d);
    run<42>("v_sub_u16_sdwa", ncu, d);
    run<43>("v_cmp_gt_u32 + cndmask", ncu, d);
    run<44>("v_cndmask_b32 vcc only", ncu, d);
    run<45>("v_perm_b32", ncu, d);
    run<46>("v_alignbit_b32", ncu, d);
    run<47>("v_alignbyte_b32", ncu, d);
    run<48>("v_med3_u32", ncu, d);
    run<49>("v_med3_i32", ncu, d);
    run<50>("v_min_u16", ncu, d);
    run<51>("v_max_u16", ncu, d);
    run<52>("v_min_i16", ncu, d);
    run<53>("v_sub_u16", ncu, d);
    run<54>("v_subrev_u16", ncu, d);
    run<55>("v_lshlrev_b16", ncu, d);
    run<56>("v_lshrrev_b16", ncu, d);
    run<57>("v_ashrrev_i16", ncu, d);
    run<58>("v_mul_lo_u16", ncu, d);
    run<59>("v_max_u32", ncu, d);
    run<60>("v_add_co_u32 (vcc)", ncu, d);
    run<61>("v_addc_co_u32", ncu, d);
    run<62>("v_cmp_gt_u32 only", ncu, d);
    run<63>("v_fmac_f32", ncu, d);
    run<64>("v_mul_f32", ncu, d);
    run<65>("v_sub_f32", ncu, d);
    run<66>("v_min_f32", ncu, d);
    run<67>("v_add_f16", ncu, d);
    run<68>("v_max_f16", ncu, d);
    run<69>("v_cvt_i32_f32", ncu, d);
    run<70>("v_not_b32", ncu, d);
    run<71>("v_ffbh_u32", ncu, d);
    run<72>("v_bfrev_b32", ncu, d);
    run<73>("v_mov_b32_dpp quad", ncu, d);
    run<74>("v_add_u32_e64 vv", ncu, d);
    run<75>("v_sub_u32_e64 vv", ncu, d);
    run<76>("v_min_u32_e64 vv", ncu, d);
    run<77>("v_max_i16_e64 vv", ncu, d);
    run<78>("v_pk_sub_u16", ncu, d);
    run<79>("v_pk_max_i16", ncu, d);
    run<80>("v_pk_mad_u16", ncu, d);
    run<81>("v_pk_lshlrev_b16", ncu, d);
    run<82>("v_lshl_or_b32 2x", ncu, d);
    run<83>("ds_read_b32", ncu, d);
    run<84>("ds_read_u16_d16_hi", ncu, d);
    run<85>("ds_add_u32", ncu, d);
    run<86>("v_sad_u16", ncu, d);
    run<87>("v_med3_u16", ncu, d);
    run<88>("v_sad_u8", ncu, d);
    run<89>("v_sad_u16 inl", ncu, d);
    run<90>("v_max3_u32", ncu, d);
    run<91>("v_med3_i16", ncu, d);
    run<92>("v_sub_u32_sdwa byte", ncu, d);
    run<93>("v_msad_u8", ncu, d);
    hipFree(d);
    return 0;
}
