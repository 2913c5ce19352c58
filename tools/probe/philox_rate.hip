// Philox4x32-10 issue cost on gfx950 by multiply form (probe for the in-prologue channel):
//   0: the compiler's form (v_mad_u64_u32, multiplier in an SGPR)
//   1: v_mad_u64_u32 with the multiplier in a VGPR
//   2: v_mul_hi_u32 + v_mul_lo_u32, multiplier in a VGPR
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/philox_rate.hip -o tools/bin/philox_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int NITER = 4096;

template <int V>
__device__ __forceinline__ void round(uint32_t (&c)[4], uint32_t k0, uint32_t k1, uint32_t m0, uint32_t m1) {
    uint32_t hi0, lo0, hi1, lo1;
    if (V == 0) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0; hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
    } else if (V == 1) {
        uint64_t p0, p1;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p0) : "v"(m0), "v"(c[0]) : "vcc");
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p1) : "v"(m1), "v"(c[2]) : "vcc");
        hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0; hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
    } else {
        asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(hi0) : "v"(m0), "v"(c[0]));
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(lo0) : "v"(m0), "v"(c[0]));
        asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(hi1) : "v"(m1), "v"(c[2]));
        asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(lo1) : "v"(m1), "v"(c[2]));
    }
    c[0] = __builtin_amdgcn_bitop3_b32(hi1, c[1], k0, 0x96);
    c[1] = lo1;
    c[2] = __builtin_amdgcn_bitop3_b32(hi0, c[3], k1, 0x96);
    c[3] = lo0;
}

template <int V>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed, unsigned long long* cyc) {
    uint32_t m0 = 0xD2511F53u, m1 = 0xCD9E8D57u;
    asm volatile("" : "+v"(m0), "+v"(m1));
    uint32_t acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NITER; ++it) {
        // two independent calls per iteration (as a lane generating several quads)
        uint32_t a[4] = {(uint32_t)it, threadIdx.x, seed, 0x4C445134u};
        uint32_t b[4] = {(uint32_t)it, threadIdx.x + 1, seed, 0x4C445134u};
        uint32_t k0 = seed, k1 = seed ^ 0x1234u;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            round<V>(a, k0, k1, m0, m1);
            round<V>(b, k0, k1, m0, m1);
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        acc ^= a[0] ^ a[1] ^ a[2] ^ a[3] ^ b[0] ^ b[1] ^ b[2] ^ b[3];
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if ((threadIdx.x & 63) == 0) atomicMax(cyc, t1 - t0);
}

template <int V>
void run(const char* name, int wps, int ncu, uint32_t* d) {
    unsigned long long* cyc = reinterpret_cast<unsigned long long*>(d + (size_t)ncu * 8 * 256);
    hipLaunchKernelGGL(k<V>, dim3(ncu * wps), dim3(256), 0, 0, d, 7u, cyc);
    hipMemset(cyc, 0, 8);
    hipLaunchKernelGGL(k<V>, dim3(ncu * wps), dim3(256), 0, 0, d, 9u, cyc);
    hipDeviceSynchronize();
    unsigned long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // per SIMD: wps waves x NITER x 2 calls
    printf("%-34s waves/SIMD %d  %7.1f shader cycles per Philox4x32-10 call per wave\n", name, wps,
           (double)c / ((double)wps * NITER * 2));
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    uint32_t* d;
    hipMalloc(&d, (size_t)ncu * 8 * 256 * 4 + 64);
    for (int w : {2, 6, 8}) {
        run<0>("compiler (mad_u64, SGPR multiplier)", w, ncu, d);
        run<1>("mad_u64, VGPR multiplier", w, ncu, d);
        run<2>("mul_hi + mul_lo, VGPR multiplier", w, ncu, d);
    }
    return 0;
}
