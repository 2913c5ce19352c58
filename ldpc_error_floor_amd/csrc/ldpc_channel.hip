// ldpc_channel.hip — on-GPU AWGN channel / LLR generator (SURVEY.md §8 f, rank 1) into HBM.
// The generator itself (model, Philox stream, precision) is ldpc_awgn.h, shared with the
// fused decoder's in-prologue channel.
#include <algorithm>

#include "ldpc_awgn.h"
#include "ldpc_internal.h"

namespace ldpc {

// float modes: one (codeword, element pair) per thread, grid-strided.  The index -> (codeword, pair) split is
// a 32-bit division whenever the batch has fewer than 2^32 pairs (a 64-bit one is a long
// emulated sequence), and an even row length stores the pair as one 8-byte write.
template <bool WIDE>
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
        awgn_pair(a, b, pr, l);
        float* row = out + b * n_vars;
        if (even) {
            *reinterpret_cast<float2*>(row + 2 * pr) = make_float2(l[0], l[1]);
        } else {
            row[2 * pr] = l[0];
            if (2 * pr + 1 < n_vars) row[2 * pr + 1] = l[1];
        }
    }
}

// QMS: Box-Muller's replacement.  One thread per (global codeword quad, variable); variable
// fastest, so each of the four row stores is coalesced across the wave.  The bucket table and
// thresholds are built in LDS by each workgroup (awgn_bucket_fill2, 8 KB).  A thread's (quad,
// variable) advances by the grid stride without a division per item: the stride's quotient and
// remainder by n_vars are fixed.
__global__ void __launch_bounds__(256) k_awgn_qf(float* __restrict__ out, int64_t B, int n_vars,
                                                 AwgnParams a) {
    __shared__ uint2 bucket[1 << AWGN_KB];
    __shared__ uint32_t thi[AWGN_NB_MAX], tlo[AWGN_NB_MAX];
    __shared__ float val[AWGN_NB_MAX + 1];
    awgn_bucket_fill2(a, bucket, thi, tlo, threadIdx.x, blockDim.x);
    if (threadIdx.x <= (unsigned)a.nb) val[threadIdx.x] = a.val[threadIdx.x];
    __syncthreads();
    const uint64_t g0 = (uint64_t)a.offset;
    const uint64_t q0 = g0 >> 2;
    const int64_t nq = (int64_t)(((g0 + (uint64_t)B - 1) >> 2) - q0 + 1);
    const int64_t id0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t S = (int64_t)gridDim.x * blockDim.x;
    int64_t m = id0 / n_vars;
    int v = (int)(id0 - m * n_vars);
    const int64_t dm = S / n_vars;
    const int dv = (int)(S - dm * n_vars);
    for (; m < nq; m += dm) {
        const uint64_t gq = q0 + (uint64_t)m;
        const int64_t bq = (int64_t)(gq * 4 - g0);          // batch index of the quad's word 0
        const int fx = awgn_fixed(a, v + 1);
        float l[4];
        if (fx == 0) {
            int lv[4];
            awgn_levels4b(a, bucket, thi, tlo, (uint32_t)v, gq, lv);
#pragma unroll
            for (int j = 0; j < 4; ++j) l[j] = val[lv[j]];
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) l[j] = fx == 1 ? 0.0f : -a.clip;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (bq + j >= 0 && bq + j < B) out[(bq + j) * n_vars + v] = l[j];
        v += dv;
        if (v >= n_vars) {
            v -= n_vars;
            ++m;
        }
    }
}

// the rows of an index list: rows[r] = the LLR row ldpc_channel_awgn writes for batch codeword
// idx[r] (global index a.offset + idx[r]), one thread per element; for the few frames an
// uncorrected-word sweep collects after a decode whose channel never left the kernel
// (QMS: awgn_qms_elem, the level sampler's stream by a linear threshold scan)
__global__ void __launch_bounds__(256) k_awgn_rows(float* __restrict__ out, const int64_t* __restrict__ idx,
                                                   int64_t n, int n_vars, AwgnParams a) {
    const bool qms = a.decoding_type == LDPC_DEC_QMS;
    const int per = qms ? n_vars : (n_vars + 1) / 2;
    const int64_t total = n * per;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = id / per;
        const int k = (int)(id - r * per);
        const int64_t b = idx[r];
        float* row = out + r * n_vars;
        if (qms) {
            row[k] = awgn_qms_elem(a, (uint64_t)(a.offset + b), k);
        } else {
            float l[2];
            awgn_pair(a, b, k, l);
            row[2 * k] = l[0];
            if (2 * k + 1 < n_vars) row[2 * k + 1] = l[1];
        }
    }
}

void awgn_gen_table(const AwgnParams& a, uint32_t* out) {
    constexpr int NB = 1 << AWGN_KB;
    for (int b = 0; b < NB; ++b) {
        uint32_t base = 0u, cnt = 0u, first = 0u;
        for (int i = 0; i < a.nb; ++i) {
            const uint32_t tb = a.thr_hi[i] >> (32 - AWGN_KB);
            if (tb < (uint32_t)b) ++base;
            if (tb == (uint32_t)b) {
                if (cnt == 0u) first = a.thr_hi[i];
                ++cnt;
            }
        }
        out[2 * b] = base | cnt << 8;
        out[2 * b + 1] = cnt ? first : ~0u;     // (awgn_bucket_fill2's entries)
    }
    for (int i = 0; i < AWGN_NB_MAX; ++i) {
        out[2 * NB + i] = i < a.nb ? a.thr_hi[i] : 0u;
        out[2 * NB + AWGN_NB_MAX + i] = i < a.nb ? a.thr_lo[i] : 0u;
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
    if (decoding_type == LDPC_DEC_QMS) host::awgn_qms_levels(sigma, q_bit, &a.nb, &a.kmin, a.thr_hi, a.thr_lo, a.val);
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
    const ldpc::AwgnParams a = ldpc::make_awgn(sigma, seed, offset, decoding_type, q_bit,
                                               punct_start, punct_end, short_start, short_end,
                                               clip_llr);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (decoding_type == LDPC_DEC_QMS) {
        // the level sampler (ldpc_awgn.h): one thread per (codeword quad, variable)
        const int64_t nq = (int64_t)((((uint64_t)offset + (uint64_t)B - 1) >> 2) - ((uint64_t)offset >> 2) + 1);
        const int64_t total = nq * n_vars;
        const unsigned grid = (unsigned)std::min<int64_t>(8192, (total + 255) / 256);
        hipLaunchKernelGGL(ldpc::k_awgn_qf, dim3(grid), dim3(256), 0, s, llr_dev, B, (int)n_vars, a);
        return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
    }
    // float modes: Box-Muller per element pair
    const int64_t total = B * ((n_vars + 1) / 2);
    const unsigned grid = (unsigned)std::min<int64_t>(8192, (total + 255) / 256);
    // 8-byte pair stores: even rows in an 8-byte aligned buffer
    const int pairs8 = ((n_vars & 1) == 0 && (reinterpret_cast<uintptr_t>(llr_dev) & 7) == 0) ? 1 : 0;
    const bool wide = total + (int64_t)grid * 256 >= ((int64_t)1 << 32);
    if (wide) hipLaunchKernelGGL(ldpc::k_awgn<true>, dim3(grid), dim3(256), 0, s, llr_dev, B, (int)n_vars, a, pairs8);
    else hipLaunchKernelGGL(ldpc::k_awgn<false>, dim3(grid), dim3(256), 0, s, llr_dev, B, (int)n_vars, a, pairs8);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}


extern "C" int ldpc_channel_awgn_rows(float* rows_dev, const int64_t* idx_dev, int64_t n, int32_t n_vars,
                                      double sigma, uint64_t seed, int64_t offset, int32_t decoding_type,
                                      int32_t q_bit, int32_t punct_start, int32_t punct_end,
                                      int32_t short_start, int32_t short_end, float clip_llr,
                                      void* stream) {
    if (n < 0 || (n > 0 && (!rows_dev || !idx_dev))) return LDPC_ERR_ARG;
    const int chk = ldpc::host::check_channel(1, n_vars, sigma, offset, decoding_type, q_bit,
                                              punct_start, punct_end, short_start, short_end,
                                              clip_llr);
    if (chk != LDPC_OK) return chk;
    if (n == 0) return LDPC_OK;
    const ldpc::AwgnParams a = ldpc::make_awgn(sigma, seed, offset, decoding_type, q_bit,
                                               punct_start, punct_end, short_start, short_end,
                                               clip_llr);
    const int64_t per = decoding_type == LDPC_DEC_QMS ? n_vars : (n_vars + 1) / 2;
    const unsigned grid = (unsigned)std::min<int64_t>(8192, (n * per + 255) / 256);
    hipLaunchKernelGGL(ldpc::k_awgn_rows, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       rows_dev, idx_dev, n, (int)n_vars, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
