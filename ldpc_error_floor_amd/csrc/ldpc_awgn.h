// ldpc_awgn.h — the on-GPU AWGN LLR generator shared by ldpc_channel_awgn (ldpc_channel.hip),
// the bit-sliced kernels' in-prologue channel (ldpc_bs_kernel.h gen_bytes) and the fused v5
// decoder's (ldpc_fused5.hip), so that generating inside the decoder is bit-identical to
// generating into HBM and decoding.
//
// Channel model of create_mix_epoch (Print_Functions.py:29-72) for the all-zero word:
//   y = sigma * n - 1 (BPSK 0 -> -1),  LLR = 2 y / sigma^2 (log p1/p0);  QMS: Cal_MSA_Q
//   (round half to even + clip); punctured bits -> 0 (0.001 for sum-product); shortened bits
//   -> -clip_LLR (after quantization).
// Noise: counter-based Philox4x32-10 keyed by the 64-bit seed, so any shard generated with its
// global codeword offset draws exactly the numbers one GPU would.  Two samplers:
//  * float modes (SP, MS): Box-Muller per (codeword, element pair), counter = (pair index,
//    global codeword index, tag).  u1 takes 53 random bits and is converted to fp32 only at the
//    logarithm — fp32's exponent range reaches 2^-54, so |n| goes to ~8.6 sigma — everything
//    else is fp32.
//  * QMS (every q_bit): the quantized LLR is one of at most 33 levels, and level j is taken
//    with probability Phi(n_j) - Phi(n_{j-1}), n_j the noise value of the j-th rounding
//    boundary of Cal_MSA_Q (computed on the host in float64 from erfc, as a 64-bit fixed-point
//    CDF threshold T_j = P(level <= j) 2^64).  Element (b, v) compares a 64-bit uniform U with
//    the thresholds: level = #{j : U >= T_j}.  U's high word is word (b mod 4) of
//    Philox(v, b / 4, tag 'LDQ4') — one Philox call serves four codewords of one variable, and
//    punctured / shortened variables draw nothing — and its low word (word b mod 4 of
//    Philox(v, b / 4, tag 'LDQR')) is drawn only when the high word equals a threshold's (about
//    once per 2^27 elements).  This is the reference's distribution to the precision of the
//    thresholds: float64 erfc (about 2^-53 relative per level) rounded down to a multiple of
//    2^-64; a level whose upper tail is below 2^-64 gets probability 2^-64 (threshold 2^64 - 1)
//    -- against fp32 Box-Muller's ulp-level boundary errors and its ~8.6 sigma tail cut -- with
//    no logarithm, square root or sine: about a third of the Box-Muller VALU per element.
// It is NOT the numpy RandomState stream: host-generated LLRs remain the seed-parity path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ldpc_nms.h"

namespace ldpc {

// Philox products as separate high / low multiplies (A/B switch; off: the v_mad_u64_u32 form
// is faster in the prologue channel despite valu_rate's per-instruction figures -- C2 sweep step
// 4.652 against 4.733 ms, C4 10.960 against 11.130, profiles/r6/session_r6aa.log)
#ifndef AWGN_MULHL
#define AWGN_MULHL 0
#endif

struct Philox {
    static __device__ __forceinline__ void round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
#if AWGN_MULHL
        // (v_mul_hi_u32 + v_mul_lo_u32 instead of the one v_mad_u64_u32 of the 64-bit product)
        const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
#else
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#endif
        // (three-input xors as one v_bitop3 each)
        c[0] = __builtin_amdgcn_bitop3_b32(hi1, c[1], k[0], 0x96);
        c[1] = lo1;
        c[2] = __builtin_amdgcn_bitop3_b32(hi0, c[3], k[1], 0x96);
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

constexpr int AWGN_NB_MAX = 32;        // rounding boundaries of the widest quantizer (q = 6)
constexpr uint32_t AWGN_TAG_Q = 0x4C445134u;   // 'LDQ4': high words of the QMS uniforms
constexpr uint32_t AWGN_TAG_R = 0x4C445152u;   // 'LDQR': their low words (rarely drawn)

struct AwgnParams {
    uint32_t k0, k1;        // Philox key (seed low / high word)
    int64_t offset;         // global index of the batch's first codeword
    float sigma, inv;       // inv = 2 / sigma^2
    float clip;
    int decoding_type, q_bit;
    int ps, pe, ss, se;     // 1-based inclusive puncture / shorten ranges (0: none)
    // QMS level sampler (make_awgn fills it when decoding_type is QMS)
    int nb;                 // boundaries; levels 0 .. nb
    int kmin;               // grid index of level 0 (value / grid step), for the byte output
    uint32_t thr_hi[AWGN_NB_MAX], thr_lo[AWGN_NB_MAX];   // T_j, ascending
    float val[AWGN_NB_MAX + 1];                           // LLR value of level j
};

// host: parameters from the C-ABI arguments, with the QMS level thresholds (ldpc_channel.hip)
AwgnParams make_awgn(double sigma, uint64_t seed, int64_t offset, int decoding_type, int q_bit,
                     int ps, int pe, int ss, int se, float clip);
// the QMS level sampler's lookup tables in one block, built on the host (the same entries as
// awgn_bucket_fill2): words [0, 2 NB) the bucket entries {base | count << 8, first threshold},
// then thr_hi[AWGN_NB_MAX], thr_lo[AWGN_NB_MAX] -- the bit-sliced kernels' in-prologue channel
// copies it into LDS
constexpr int AWGN_TAB_W = 2 * (1 << 10) + 2 * 32;
void awgn_gen_table(const AwgnParams& a, uint32_t* out /*[AWGN_TAB_W]*/);

// float modes (SP, MS): LLRs of elements 2*pr and 2*pr+1 of codeword `b` (batch-relative)
// into l[0], l[1] by Box-Muller (QMS uses the level sampler below)
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
        if (a.ps > 0 && bit >= a.ps && bit <= a.pe) llr = (a.decoding_type == 0) ? 0.001f : 0.0f;
        if (a.ss > 0 && bit >= a.ss && bit <= a.se) llr = -a.clip;
        l[h] = llr;
    }
}

// ---- QMS level sampler -------------------------------------------------------------------------
// Level of a codeword from the high word u of its uniform.  bucket / thi: the bucket table
// (awgn_bucket_fill) and thresholds, in LDS or global memory.  A bucket holds base | count << 8:
// U's top AWGN_KB bits fix every threshold but the `count` ones starting at `base`, compared one
// by one.  A tie of the high words (u == thi[lv], P ~ nb 2^-32) stops the scan with `tie` set:
// the low word decides (awgn_tie_scan), drawn only then -- kept out of this loop so that the
// compiler cannot hoist the second Philox in front of it.
constexpr int AWGN_KB = 10;                 // bucket bits (1024 buckets, 2 KB of LDS)
#ifndef AWGN_FAST
#define AWGN_FAST 1     // awgn_levels4b's branch-free common case (A/B switch)
#endif
static_assert(AWGN_TAB_W == 2 * (1 << AWGN_KB) + 2 * AWGN_NB_MAX, "awgn_gen_table layout");
template <typename P16, typename P32>
__device__ __forceinline__ int awgn_level_hi(P16 bucket, P32 thi, uint32_t u, bool& tie) {
    const uint32_t e = bucket[u >> (32 - AWGN_KB)];
    int lv = (int)(e & 0xFFu);
    const int cnt = (int)(e >> 8);
    for (int i = 0; i < cnt; ++i) {
        const uint32_t th = thi[lv];
        if (u <= th) {                           // thresholds ascend: the rest are above U too
            tie = u == th;
            break;
        }
        ++lv;
    }
    return lv;
}

// the scan from a tie at level lv on: full 64-bit comparisons (hi word u, low word lo)
template <typename P32>
__device__ __forceinline__ int awgn_tie_scan(int nb, P32 thi, P32 tlo, uint32_t u, uint32_t lo, int lv) {
    for (; lv < nb; ++lv) {
        const uint32_t th = thi[lv];
        if (u < th || (u == th && lo < tlo[lv])) break;
    }
    return lv;
}

// the bucket table of a's thresholds, built by the threads of a workgroup (tid < n) into LDS:
// each pass over the (uniform) thresholds counts for four buckets per lane, b = tid + k n
// (one pass from 256 threads on)
__device__ __forceinline__ void awgn_bucket_fill(const AwgnParams& a, uint16_t* bucket, uint32_t* thi,
                                                 uint32_t* tlo, int tid, int n) {
    for (int i = tid; i < a.nb; i += n) {
        thi[i] = a.thr_hi[i];
        tlo[i] = a.thr_lo[i];
    }
    constexpr int NB = 1 << AWGN_KB;
    for (int b0 = tid; b0 < NB; b0 += 4 * n) {
        uint32_t base[4] = {0u, 0u, 0u, 0u}, cnt[4] = {0u, 0u, 0u, 0u};
        for (int i = 0; i < a.nb; ++i) {
            // (readfirstlane returns an int: shifted as unsigned, or the thresholds above 2^31
            // would sign-extend out of every bucket)
            const uint32_t tb = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.thr_hi[i]) >> (32 - AWGN_KB);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t b = (uint32_t)(b0 + k * n);
                base[k] += tb < b ? 1u : 0u;
                cnt[k] += tb == b ? 1u : 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (b0 + k * n < NB) bucket[b0 + k * n] = (uint16_t)(base[k] | cnt[k] << 8);
    }
}

// the levels of codewords 4 gq .. 4 gq + 3 at variable v (0-based; punctured / shortened
// variables are the caller's): level indices 0 .. a.nb
template <typename P16, typename P32>
__device__ __forceinline__ void awgn_levels4(const AwgnParams& a, P16 bucket, P32 thi, P32 tlo,
                                             uint32_t v, uint64_t gq, int (&lv)[4]) {
    uint32_t c[4] = {v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_Q};
    Philox::gen(c, a.k0, a.k1);
    bool tie[4] = {false, false, false, false};
#pragma unroll
    for (int j = 0; j < 4; ++j) lv[j] = awgn_level_hi(bucket, thi, c[j], tie[j]);
    if (tie[0] | tie[1] | tie[2] | tie[3]) {
        uint32_t r[4] = {v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_R};
        Philox::gen(r, a.k0, a.k1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (tie[j]) lv[j] = awgn_tie_scan(a.nb, thi, tlo, c[j], r[j], lv[j]);
    }
}

// ---- the channel kernels' form: each bucket carries its first threshold -----------------------
// (ldpc_channel.hip: 8 KB of LDS per workgroup).  A bucket entry is {base | count << 8, the high
// word of threshold `base` (2^32 - 1 if count = 0)}: one ds_read_b64 decides U's level whenever its
// bucket holds at most one threshold (all but the few buckets where the CDF climbs by more than
// one level within 2^-10: the far tails); the others scan on from there.  Same levels as
// awgn_levels4.
__device__ __forceinline__ void awgn_bucket_fill2(const AwgnParams& a, uint2* bucket, uint32_t* thi,
                                                  uint32_t* tlo, int tid, int n) {
    for (int i = tid; i < a.nb; i += n) {
        thi[i] = a.thr_hi[i];
        tlo[i] = a.thr_lo[i];
    }
    constexpr int NB = 1 << AWGN_KB;
    for (int b0 = tid; b0 < NB; b0 += 4 * n) {
        uint32_t base[4] = {0u, 0u, 0u, 0u}, cnt[4] = {0u, 0u, 0u, 0u}, first[4] = {0u, 0u, 0u, 0u};
        for (int i = 0; i < a.nb; ++i) {
            const uint32_t th = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.thr_hi[i]);
            const uint32_t tb = th >> (32 - AWGN_KB);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t b = (uint32_t)(b0 + k * n);
                base[k] += tb < b ? 1u : 0u;
                if (tb == b) {
                    if (cnt[k] == 0u) first[k] = th;
                    ++cnt[k];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)     // (an empty bucket's first: 2^32 - 1, above every U's high word but one)
            if (b0 + k * n < NB) bucket[b0 + k * n] = make_uint2(base[k] | cnt[k] << 8, cnt[k] ? first[k] : ~0u);
    }
}

// the levels of codewords 4 gq .. 4 gq + 3 at variable v from the inline-threshold table: the
// four bucket reads issued together, the level from the entry alone (U against the bucket's
// first threshold), and only then the rare scans: buckets holding more thresholds, high-word ties
// (A: anything with the key k0, k1 and the boundary count nb: AwgnParams, or the bit-sliced
// kernels' in-prologue generator; PB / P32: the tables in LDS or global memory)
// (awgn_levels4b_c: the levels from the high words c = Philox(v, gq, 'LDQ4') already drawn)
template <typename A, typename PB, typename P32>
__device__ __forceinline__ void awgn_levels4b_c(const A& a, PB bucket, P32 thi, P32 tlo, uint32_t v,
                                                uint64_t gq, const uint32_t (&c)[4], int (&lv)[4]) {
    uint2 e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const auto ej = bucket[c[j] >> (32 - AWGN_KB)];
        e[j] = make_uint2(ej.x, ej.y);
    }
#if AWGN_FAST
    // the common case, branch-free: level = base + [U > first] (an empty bucket's first is
    // 2^32 - 1, so nothing exceeds it).  A bucket holding two or more thresholds (count field
    // >= 2: the far tails) or a high word equal to a bucket's first threshold (a tie, or U = 2^32
    // - 1 in an empty bucket) sends the quad through the exact path below, which gives the same
    // levels in every other case
    {
        const uint32_t ex = e[0].x | e[1].x | e[2].x | e[3].x;
        const uint32_t dm = min(min(c[0] ^ e[0].y, c[1] ^ e[1].y), min(c[2] ^ e[2].y, c[3] ^ e[3].y));
#pragma unroll
        for (int j = 0; j < 4; ++j) lv[j] = (int)(e[j].x & 0xFFu) + (c[j] > e[j].y ? 1 : 0);
        if (ex < 2u << 8 && dm != 0u) return;
    }
#endif
    uint32_t ties = 0u, more = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t cnt = e[j].x >> 8;
        const bool in = cnt != 0u;
        const bool gt = in && c[j] > e[j].y;
        lv[j] = (int)(e[j].x & 0xFFu) + (gt ? 1 : 0);
        ties |= (in && c[j] == e[j].y) ? 1u << j : 0u;
        more |= (cnt > 1u && gt) ? 1u << j : 0u;
    }
    if (more) {                         // (rare) more thresholds inside U's bucket
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (!((more >> j) & 1u)) continue;
            const uint32_t cnt = e[j].x >> 8;
            for (uint32_t i = 1; i < cnt; ++i) {
                const uint32_t th = thi[lv[j]];
                if (c[j] <= th) {
                    if (c[j] == th) ties |= 1u << j;
                    break;
                }
                ++lv[j];
            }
        }
    }
    if (ties) {
        uint32_t r[4] = {v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_R};
        Philox::gen(r, a.k0, a.k1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((ties >> j) & 1u) lv[j] = awgn_tie_scan(a.nb, thi, tlo, c[j], r[j], lv[j]);
    }
}
template <typename A, typename PB, typename P32>
__device__ __forceinline__ void awgn_levels4b(const A& a, PB bucket, P32 thi, P32 tlo,
                                              uint32_t v, uint64_t gq, int (&lv)[4]) {
    uint32_t c[4] = {v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_Q};
    Philox::gen(c, a.k0, a.k1);
    awgn_levels4b_c(a, bucket, thi, tlo, v, gq, c, lv);
}

// what a QMS element at 1-based bit `bit` is: 0 random, 1 punctured (LLR 0), 2 shortened (-clip)
__device__ __forceinline__ int awgn_fixed(const AwgnParams& a, int bit) {
    if (a.ss > 0 && bit >= a.ss && bit <= a.se) return 2;
    if (a.ps > 0 && bit >= a.ps && bit <= a.pe) return 1;
    return 0;
}

// one QMS element (codeword at global index gb, variable v) by a linear threshold scan over a's
// own tables: the fused v5 kernel's in-prologue channel for batches whose offset is not a
// multiple of 4 (same stream as awgn_levels4)
__device__ __forceinline__ float awgn_qms_elem(const AwgnParams& a, uint64_t gb, int v) {
    const int fx = awgn_fixed(a, v + 1);
    if (fx == 1) return 0.0f;
    if (fx == 2) return -a.clip;
    const uint64_t gq = gb >> 2;
    const int j = (int)(gb & 3);
    uint32_t c[4] = {(uint32_t)v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_Q};
    Philox::gen(c, a.k0, a.k1);
    const uint32_t u = c[j];
    int lv = 0;
    while (lv < a.nb && u > a.thr_hi[lv]) ++lv;
    if (lv < a.nb && u == a.thr_hi[lv]) {        // a tie of the high words: draw the low word
        uint32_t r[4] = {(uint32_t)v, (uint32_t)gq, (uint32_t)(gq >> 32), AWGN_TAG_R};
        Philox::gen(r, a.k0, a.k1);
        lv = awgn_tie_scan(a.nb, a.thr_hi, a.thr_lo, u, r[j], lv);
    }
    return a.val[lv];
}

}  // namespace ldpc
