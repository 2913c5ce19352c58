// ldpc_channel.hip — on-GPU AWGN channel / LLR generator (SURVEY.md §8 f, rank 1).
//
// Same channel model as create_mix_epoch (Print_Functions.py:29-72) for the all-zero word:
//   y = sigma * n - 1 (BPSK 0 -> -1),  LLR = 2 y / sigma^2 (log p1/p0), computed in double;
//   QMS: Cal_MSA_Q (round half to even + clip, in double); punctured bits -> 0 (0.001 for
//   sum-product); shortened bits -> -clip_LLR (after quantization).
// The noise comes from a counter-based Philox4x32-10 stream keyed by `seed`, indexed by the
// GLOBAL codeword index (offset + b) and element, so a batch split over ranks by codeword
// offset draws exactly the numbers a single GPU would.  Box-Muller with a 53-bit uniform
// under the logarithm (|n| up to ~8.5 sigma) keeps the tails that matter for FER ~1e-9.
// It is NOT the numpy RandomState stream: host-generated LLRs remain the seed-parity path.
#include <cmath>

#include "ldpc_internal.h"

namespace ldpc {

struct Philox {
    static __device__ __forceinline__ void round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c[0] = hi1 ^ c[1] ^ k[0];
        c[1] = lo1;
        c[2] = hi0 ^ c[3] ^ k[1];
        c[3] = lo0;
    }
    static __device__ __forceinline__ void gen(uint32_t (&c)[4], uint32_t k0, uint32_t k1) {
        uint32_t k[2] = {k0, k1};
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            round(c, k);
            k[0] += 0x9E3779B9u;
            k[1] += 0xBB67AE85u;
        }
    }
};

__device__ __forceinline__ double quant_host(double x, int q_bit) {
    switch (q_bit) {
        case 6: return fmin(fmax(rint(x), -15.5), 15.5);
        case 5: return fmin(fmax(rint(x * 2.0) / 2.0, -7.5), 7.5);
        case -5: return fmin(fmax(rint(x), -15.0), 15.0);
        case 4: return fmin(fmax(rint(x), -7.0), 7.0);
        default: return fmin(fmax(rint(x / 2.0) * 2.0, -6.0), 6.0);
    }
}

__global__ void __launch_bounds__(256) k_awgn(float* __restrict__ out, int64_t B, int n_vars,
                                              double sigma, uint32_t k0, uint32_t k1,
                                              int64_t offset, int decoding_type, int q_bit,
                                              int ps, int pe, int ss, int se, float clip) {
    const int npairs = (n_vars + 1) / 2;
    const int64_t total = B * npairs;
    const double inv = 2.0 / (sigma * sigma);
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = id / npairs;
        const int pr = (int)(id - b * npairs);
        const uint64_t gcw = (uint64_t)(offset + b);
        uint32_t c[4] = {(uint32_t)pr, (uint32_t)gcw, (uint32_t)(gcw >> 32), 0x4C445043u};
        Philox::gen(c, k0, k1);
        const uint64_t m53 = ((uint64_t)c[0] << 21) ^ (uint64_t)(c[1] >> 11);
        const double u1 = ((double)(m53 & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;   // (0,1)
        const double u2 = ((double)c[2] + 0.5) * 0x1.0p-32;
        const double r = sqrt(-2.0 * log(u1));
        double sn, cs;
        sincospi(2.0 * u2, &sn, &cs);
        const double nz[2] = {r * cs, r * sn};
        for (int h = 0; h < 2; ++h) {
            const int v = 2 * pr + h;
            if (v >= n_vars) break;
            double llr = (nz[h] * sigma - 1.0) * inv;
            if (decoding_type == LDPC_DEC_QMS) llr = quant_host(llr, q_bit);
            const int bit = v + 1;                          // 1-based like the reference
            if (ps > 0 && bit >= ps && bit <= pe) llr = (decoding_type == 0) ? 0.001 : 0.0;
            if (ss > 0 && bit >= ss && bit <= se) llr = -(double)clip;
            out[b * n_vars + v] = (float)llr;
        }
    }
}

}  // namespace ldpc

extern "C" int ldpc_channel_awgn(float* llr_dev, int64_t B, int32_t n_vars, double sigma,
                                 uint64_t seed, int64_t offset, int32_t decoding_type,
                                 int32_t q_bit, int32_t punct_start, int32_t punct_end,
                                 int32_t short_start, int32_t short_end, float clip_llr,
                                 void* stream) {
    if (!llr_dev || B <= 0 || n_vars <= 0 || !(sigma > 0.0) || offset < 0) return LDPC_ERR_ARG;
    if (decoding_type == LDPC_DEC_QMS && ldpc::mode_of(decoding_type, q_bit) < 0) return LDPC_ERR_ARG;
    const int64_t total = B * ((n_vars + 1) / 2);
    const unsigned grid = (unsigned)std::min<int64_t>(8192, (total + 255) / 256);
    hipLaunchKernelGGL(ldpc::k_awgn, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       llr_dev, B, (int)n_vars, sigma, (uint32_t)seed, (uint32_t)(seed >> 32), offset,
                       (int)decoding_type, (int)q_bit, (int)punct_start, (int)punct_end,
                       (int)short_start, (int)short_end, clip_llr);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
