// ldpc_channel.hip — on-GPU AWGN channel / LLR generator (SURVEY.md §8 f, rank 1) into HBM.
// The generator itself (model, Philox stream, precision) is ldpc_awgn.h, shared with the
// fused decoder's in-prologue channel.
#include <algorithm>
#include <type_traits>

#include "ldpc_awgn.h"
#include "ldpc_internal.h"

namespace ldpc {

// one (codeword, element pair) per thread, grid-strided.  The index -> (codeword, pair) split is
// a 32-bit division whenever the batch has fewer than 2^32 pairs (a 64-bit one is a long
// emulated sequence), and an even row length stores the pair as one 8-byte write.
template <bool WIDE, int QB>
__global__ void __launch_bounds__(256) k_awgn(float* __restrict__ out, int64_t B, int n_vars,
                                              AwgnParams a, int pairs8) {
    const int npairs = (n_vars + 1) / 2;
    const int64_t total = B * npairs;
    const bool even = pairs8 != 0;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        int64_t b;
        int pr;
        if (WIDE) {
            b = id / npairs;
            pr = (int)(id - b * npairs);
        } else {
            const uint32_t q = (uint32_t)id / (uint32_t)npairs;
            b = q;
            pr = (int)((uint32_t)id - q * (uint32_t)npairs);
        }
        float l[2];
        awgn_pair<QB>(a, b, pr, l);
        float* row = out + b * n_vars;
        if (even) {
            *reinterpret_cast<float2*>(row + 2 * pr) = make_float2(l[0], l[1]);
        } else {
            row[2 * pr] = l[0];
            if (2 * pr + 1 < n_vars) row[2 * pr + 1] = l[1];
        }
    }
}

AwgnParams make_awgn(double sigma, uint64_t seed, int64_t offset, int decoding_type, int q_bit,
                     int ps, int pe, int ss, int se, float clip) {
    AwgnParams a{};
    a.k0 = (uint32_t)seed;
    a.k1 = (uint32_t)(seed >> 32);
    a.offset = offset;
    a.sigma = (float)sigma;
    a.inv = (float)(2.0 / (sigma * sigma));
    a.clip = clip;
    a.decoding_type = decoding_type;
    a.q_bit = q_bit;
    a.ps = ps;
    a.pe = pe;
    a.ss = ss;
    a.se = se;
    return a;
}

}  // namespace ldpc

extern "C" int ldpc_channel_awgn(float* llr_dev, int64_t B, int32_t n_vars, double sigma,
                                 uint64_t seed, int64_t offset, int32_t decoding_type,
                                 int32_t q_bit, int32_t punct_start, int32_t punct_end,
                                 int32_t short_start, int32_t short_end, float clip_llr,
                                 void* stream) {
    if (!llr_dev) return LDPC_ERR_ARG;
    const int chk = ldpc::host::check_channel(B, n_vars, sigma, offset, decoding_type, q_bit,
                                              punct_start, punct_end, short_start, short_end,
                                              clip_llr);
    if (chk != LDPC_OK) return chk;
    const int64_t total = B * ((n_vars + 1) / 2);
    const unsigned grid = (unsigned)std::min<int64_t>(8192, (total + 255) / 256);
    const ldpc::AwgnParams a = ldpc::make_awgn(sigma, seed, offset, decoding_type, q_bit,
                                               punct_start, punct_end, short_start, short_end,
                                               clip_llr);
    // 8-byte pair stores: even rows in an 8-byte aligned buffer
    const int pairs8 = ((n_vars & 1) == 0 && (reinterpret_cast<uintptr_t>(llr_dev) & 7) == 0) ? 1 : 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool wide = total + (int64_t)grid * 256 >= ((int64_t)1 << 32);
    const int qb = decoding_type == LDPC_DEC_QMS ? q_bit : 0;
    auto go = [&](auto qc) {
        constexpr int Q = decltype(qc)::value;
        if (wide) hipLaunchKernelGGL((ldpc::k_awgn<true, Q>), dim3(grid), dim3(256), 0, s, llr_dev, B, (int)n_vars, a, pairs8);
        else hipLaunchKernelGGL((ldpc::k_awgn<false, Q>), dim3(grid), dim3(256), 0, s, llr_dev, B, (int)n_vars, a, pairs8);
    };
    switch (qb) {       // one build per quantizer (check_channel has validated q_bit)
        case 6: go(std::integral_constant<int, 6>{}); break;
        case 5: go(std::integral_constant<int, 5>{}); break;
        case -5: go(std::integral_constant<int, -5>{}); break;
        case 4: go(std::integral_constant<int, 4>{}); break;
        case 3: go(std::integral_constant<int, 3>{}); break;
        default: go(std::integral_constant<int, 0>{}); break;
    }
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
