// ldpc_awgn.h — the on-GPU AWGN LLR generator shared by ldpc_channel_awgn (ldpc_channel.hip)
// and the fused decoder's in-prologue channel (ldpc_fused5.hip), so that generating inside the
// decoder is bit-identical to generating into HBM and decoding.
//
// Channel model of create_mix_epoch (Print_Functions.py:29-72) for the all-zero word:
//   y = sigma * n - 1 (BPSK 0 -> -1),  LLR = 2 y / sigma^2 (log p1/p0);  QMS: Cal_MSA_Q
//   (round half to even + clip); punctured bits -> 0 (0.001 for sum-product); shortened bits
//   -> -clip_LLR (after quantization).
// Noise: counter-based Philox4x32-10 keyed by the 64-bit seed, counter = (pair index, global
// codeword index, tag), so any shard generated with its global codeword offset draws exactly
// the numbers one GPU would.  Box-Muller on (u1, u2): u1 takes 53 random bits and is converted
// to fp32 only at the logarithm — fp32's exponent range reaches 2^-54, so |n| goes to ~8.6
// sigma and the tails that matter at FER ~1e-9 are kept — everything else is fp32.
// It is NOT the numpy RandomState stream: host-generated LLRs remain the seed-parity path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldpc_nms.h"

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

struct AwgnParams {
    uint32_t k0, k1;        // Philox key (seed low / high word)
    int64_t offset;         // global index of the batch's first codeword
    float sigma, inv;       // inv = 2 / sigma^2
    float clip;
    int decoding_type, q_bit;
    int ps, pe, ss, se;     // 1-based inclusive puncture / shorten ranges (0: none)
};

// host: parameters from the C-ABI arguments (ldpc_channel.hip)
AwgnParams make_awgn(double sigma, uint64_t seed, int64_t offset, int decoding_type, int q_bit,
                     int ps, int pe, int ss, int se, float clip);

__device__ __forceinline__ float awgn_quant(float x, int q_bit) {
    switch (q_bit) {
        case 6: return fminf(fmaxf(rintf(x), -15.5f), 15.5f);
        case 5: return fminf(fmaxf(rintf(x * 2.0f) * 0.5f, -7.5f), 7.5f);
        case -5: return fminf(fmaxf(rintf(x), -15.0f), 15.0f);
        case 4: return fminf(fmaxf(rintf(x), -7.0f), 7.0f);
        default: return fminf(fmaxf(rintf(x * 0.5f) * 2.0f, -6.0f), 6.0f);
    }
}

// LLRs of elements 2*pr and 2*pr+1 of codeword `b` (batch-relative) into l[0], l[1].
// QB: the quantizer, fixed at compile time (0 = none, i.e. a float mode; else the q_bit), or
// AWGN_QRT to take decoding_type / q_bit from `a` at run time (the runtime switch compiles to
// all five quantizers and selects)
constexpr int AWGN_QRT = 99;
template <int QB = AWGN_QRT>
__device__ __forceinline__ void awgn_pair(const AwgnParams& a, int64_t b, int pr, float (&l)[2]) {
    const uint64_t gcw = (uint64_t)(a.offset + b);
    uint32_t c[4] = {(uint32_t)pr, (uint32_t)gcw, (uint32_t)(gcw >> 32), 0x4C445043u};
    Philox::gen(c, a.k0, a.k1);
    const uint64_t m53 = (((uint64_t)c[0] << 21) ^ (uint64_t)(c[1] >> 11)) & ((1ull << 53) - 1);
    const float u1 = ((float)m53 + 0.5f) * 0x1.0p-53f;                  // (0, 1]
    const float u2 = ((float)c[2] + 0.5f) * 0x1.0p-32f;
    const float r = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincospif(2.0f * u2, &sn, &cs);
    const float nz[2] = {r * cs, r * sn};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int bit = 2 * pr + h + 1;                                  // 1-based like the reference
        float llr = (nz[h] * a.sigma - 1.0f) * a.inv;
        if constexpr (QB == AWGN_QRT) {
            if (a.decoding_type == LDPC_DEC_QMS) llr = awgn_quant(llr, a.q_bit);
        } else if constexpr (QB != 0) {
            llr = awgn_quant(llr, QB);
        }
        if (a.ps > 0 && bit >= a.ps && bit <= a.pe) llr = (a.decoding_type == 0) ? 0.001f : 0.0f;
        if (a.ss > 0 && bit >= a.ss && bit <= a.se) llr = -a.clip;
        l[h] = llr;
    }
}

}  // namespace ldpc
