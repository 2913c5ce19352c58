// ldpc_fused4.hip — fused QMS decoder, v4: two codewords per lane (packed 16-bit SWAR).
//
// Same semantics as v3 (ldpc_fused3.hip) / oracle/nms_oracle.py.  In QMS every check-side
// quantity is a small integer in grid units, so two codewords share one 32-bit lane value and
// the check-node arithmetic runs as v_pk_* 16-bit ops: one address, one LDS read, one
// min-tracking step for both codewords.  Requirements: z > 1, check degree <= 16 (per-edge
// bit masks live in 16-bit halves), per-row (not per-edge) CN weights.
//
// Lanes: lane = slot * CWP + p; a lane holds codewords p and p + CWP of the workgroup's
// CW = 2*CWP; the SLOTS = 64/CWP slots of a wave work on consecutive checks h = hg*SLOTS + s
// of one proto row.
//
// LDS  TW[v][p] u32 = Tv of codeword p (low 16) | Tv of codeword p+CWP (high 16)
//                     (with UCN: Tv in bits 14..0 of each half, previous hard decision in bit 15)
//      SW[v][p] u32 = S of both codewords, accumulated by ds_add of (c + BIAS) per half so no
//                     carry crosses halves; S = half - BIAS * deg(v)
//      CH[v][c] f32 (c < CW);  BT[T][N] = {beta, BIAS*deg(column)};  RED[8]
#include <cstdio>
#include <cstdlib>

#include "ldpc_fused.h"

namespace ldpc {

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t U(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t U(i16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 AU(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ i16x2 AI(uint32_t x) { return __builtin_bit_cast(i16x2, x); }
__device__ __forceinline__ uint32_t pack2(int lo, int hi) {
    return ((uint32_t)lo & 0xFFFFu) | ((uint32_t)hi << 16);
}

constexpr int F4_BIG_KEY = 0xFFFF;            // (1023 << 6) | 63: "no other edge"
constexpr int F4_BIG_U = 1023;
constexpr size_t F4_LDS_MAX = 160 * 1024;

struct F4Args {
    const float* llr;
    const float* beta;
    float* app_out;
    uint64_t* hd_out;
    int64_t* counters;
    uint8_t* flags;
    const int32_t* row_ptr;
    const int32_t* pe_col;
    const int32_t* pe_shift;
    const int32_t* col_ptr;
    int64_t B;
    int ntiles, T, target_bits, clip_u, qmax, bias;
    float inv, step;
    int n_vars, N, E, z;
    int hstep, ngroups, nent;
    uint32_t zmagic;
};

__device__ __forceinline__ int q_units4(float x, float inv, int qmax) {
    const float r = fminf(fmaxf(rintf(x * inv), -(float)qmax), (float)qmax);
    return (int)r;
}

__device__ __forceinline__ int q_mag4(int m, float w, float step, float inv, int qmax) {
    const float mv = (m >= F4_BIG_U) ? 10000.0f : (float)m * step;
    float x = mv * w;                          // fl32(|o| * w)
    x = (x > 0.f) ? x : 0.f;                   // x * [x > 0]
    return q_units4(x, inv, qmax);
}

// C->V messages of edge k for both codewords: +-(k == idx ? mB : mA)
__device__ __forceinline__ uint32_t msg4(int k, uint32_t PA, uint32_t PB, uint32_t OH, uint32_t NS) {
    const uint32_t eqm = U(AI(U(AU(OH) << (unsigned short)(15 - k))) >> (short)15);
    const uint32_t m = (eqm & PB) | (~eqm & PA);
    const uint32_t sm = U(AI(U(AU(NS) << (unsigned short)(15 - k))) >> (short)15);
    return U(AI(m ^ sm) - AI(sm));
}

template <int CWP, int MAXG, int MAXDEG, bool UCN>
__global__ void __launch_bounds__(1024, 1)
k_fused4(F4Args a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn) {
    static_assert(MAXDEG <= 16, "16-bit edge masks");
    constexpr int SLOTS = 64 / CWP;
    constexpr int CW = 2 * CWP;
    constexpr int LOGP = (CWP == 32) ? 5 : (CWP == 16) ? 4 : (CWP == 8) ? 3 : (CWP == 4) ? 2 : 1;
    constexpr int NPK = (MAXDEG + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nv = a.n_vars;
    const int npe = nv * CWP;                                  // pair entries
    uint32_t* TW = reinterpret_cast<uint32_t*>(smem);
    uint32_t* SW = TW + npe;
    float* CH = reinterpret_cast<float*>(smem + ((size_t)2 * npe + CW) * 4);   // [nv][CW]
    float2* BT = reinterpret_cast<float2*>(smem + ((((size_t)2 * npe + CW) * 4 + (size_t)nv * CW * 4 + 7) & ~(size_t)7));
    unsigned long long* RED = reinterpret_cast<unsigned long long*>(BT + (size_t)a.T * a.N);
    const uint32_t sw_off = (uint32_t)npe * 4u;

    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int NWV = NT >> 6;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slot = lane >> LOGP;
    const int p = lane & (CWP - 1);
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int64_t nvalid = (b0 + CW <= a.B) ? CW : (a.B - b0);
    const unsigned long long pmask = (1ull << CWP) - 1;
    const unsigned long long valid_cw = (nvalid >= 64) ? ~0ull : ((1ull << nvalid) - 1);
    const int qmax = a.qmax;
    const float inv = a.inv, step = a.step;
    const int z = a.z;
    const uint32_t BB = pack2(a.bias, a.bias);
    const uint32_t QQ = pack2(qmax, qmax);

    // ---- prologue ----------------------------------------------------------------------------
    {
        float* scr = reinterpret_cast<float*>(TW);              // [CW][nv+1] over TW|SW|pad
        const int rl = nv + 1;
        for (int f = tid; f < CW * nv; f += NT) {
            const int r = f / nv, v = f - r * nv;
            scr[r * rl + v] = (r < nvalid) ? a.llr[(b0 + r) * nv + v] : 0.f;
        }
        for (int f = tid; f < a.T * a.N; f += NT) {
            const int j = f % a.N;
            BT[f] = make_float2(a.beta[f], __int_as_float(a.bias * (a.col_ptr[j + 1] - a.col_ptr[j])));
        }
        if (tid < 8) RED[tid] = (tid == 1) ? ~0ull : 0ull;
        __syncthreads();
        for (int e = tid; e < nv * CW; e += NT) {
            const int v = e / CW, c = e - v * CW;
            CH[e] = scr[c * rl + v];
        }
        __syncthreads();
        for (int e = tid; e < npe; e += NT) {
            const uint32_t v = (uint32_t)e >> LOGP;
            const int pp = e & (CWP - 1);
            const float bt = BT[__umulhi(v, a.zmagic)].x;
            const int ta = q_units4(CH[v * CW + pp] * bt, inv, qmax);            // lw_0
            const int tb = q_units4(CH[v * CW + pp + CWP] * bt, inv, qmax);
            if (UCN)
                TW[e] = pack2((ta & 0x7FFF) | ((ta >= 0) << 15), (tb & 0x7FFF) | ((tb >= 0) << 15));
            else
                TW[e] = pack2(ta, tb);
            SW[e] = 0;
        }
    }

    // ---- per-group edge addresses (bytes of TW; SW = +sw_off), row info, validity ------------
    uint32_t gad[MAXG][NPK];
    uint32_t grow[MAXG];
    bool gval[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) {
        grow[gi] = 0;
        gval[gi] = false;
#pragma unroll
        for (int q = 0; q < NPK; ++q) gad[gi][q] = 0;
        const int grp = wave + gi * NWV;
        if (grp < a.ngroups) {
            const int i = grp / a.hstep;
            const int hg = grp - i * a.hstep;
            const int r0 = a.row_ptr[i];
            const int deg = a.row_ptr[i + 1] - r0;
            const int h = hg * SLOTS + slot;
            gval[gi] = h < z;
            const int hl = (h < z) ? h : hg * SLOTS;
            grow[gi] = (uint32_t)r0 | ((uint32_t)deg << 16);
#pragma unroll
            for (int k = 0; k < MAXDEG; ++k) {
                const int pe = r0 + ((k < deg) ? k : deg - 1);
                int hs = hl + a.pe_shift[pe];
                hs = (hs >= z) ? hs - z : hs;
                const uint32_t byte = (uint32_t)(((a.pe_col[pe] * z + hs) << LOGP) + p) * 4u;
                gad[gi][k >> 1] |= (k & 1) ? (byte << 16) : byte;
            }
        }
    }
    __syncthreads();

    // packed check state per group: magnitudes (quantized), one-hot argmin, negative-sign mask
    uint32_t PA[MAXG], PB[MAXG], OH[MAXG], NS[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) { PA[gi] = 0; PB[gi] = 0; OH[gi] = 0; NS[gi] = 0; }

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {
            RED[1] &= RED[0];
            RED[0] = 0;
        }
        const float* at = alpha + (size_t)t * a.E;
        const float* au = UCN ? alpha_ucn + (size_t)t * a.E : nullptr;
        // ======== check nodes, pass 1: V->C, two minima, sign masks (reads only) ==============
        uint32_t K1[MAXG], K2[MAXG], NEG[MAXG], SYN[MAXG];
#pragma unroll
        for (int gi = 0; gi < MAXG; ++gi) {
            K1[gi] = pack2(F4_BIG_KEY, F4_BIG_KEY);
            K2[gi] = K1[gi];
            NEG[gi] = 0;
            SYN[gi] = 0;
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) break;
            const int deg = (int)(__builtin_amdgcn_readfirstlane(grow[gi]) >> 16);
#pragma unroll
            for (int c8 = 0; c8 < MAXDEG; c8 += 8) {
                if (c8 < deg) {
                    uint32_t wv[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = c8 + j;
                        if (k < MAXDEG) {
                            const uint32_t pk = gad[gi][k >> 1];
                            const uint32_t addr = (k & 1) ? (pk >> 16) : (pk & 0xFFFFu);
                            wv[j] = *reinterpret_cast<const uint32_t*>(smem + addr);
                        }
                    }
                    uint32_t kk[8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = c8 + j;
                        kk[j] = pack2(F4_BIG_KEY, F4_BIG_KEY);
                        if (k < MAXDEG && k < deg) {
                            uint32_t tv = wv[j];
                            if (UCN) {
                                SYN[gi] ^= (tv >> 15) & 0x10001u;
                                tv = U(AI(U(AU(tv) << (unsigned short)1)) >> (short)1);
                            }
                            const uint32_t c = msg4(k, PA[gi], PB[gi], OH[gi], NS[gi]);
                            const i16x2 x = AI(tv) - AI(c);
                            const i16x2 ax = __builtin_elementwise_max(x, -x);
                            const u16x2 mag = __builtin_elementwise_min(AU(U(ax)), AU(QQ));
                            kk[j] = U(mag * (unsigned short)64 + AU(pack2(k, k)));
                            const uint32_t km = 0x10001u << k;
                            NEG[gi] = (km & (U(x) >> (15 - k))) | (~km & NEG[gi]);
                        }
                    }
                    u16x2 lo[4], hi[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        lo[j] = __builtin_elementwise_min(AU(kk[2 * j]), AU(kk[2 * j + 1]));
                        hi[j] = __builtin_elementwise_max(AU(kk[2 * j]), AU(kk[2 * j + 1]));
                    }
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const u16x2 a1 = lo[2 * j], a2 = hi[2 * j], b1 = lo[2 * j + 1], b2 = hi[2 * j + 1];
                        lo[j] = __builtin_elementwise_min(a1, b1);
                        hi[j] = __builtin_elementwise_min(__builtin_elementwise_max(a1, b1),
                                                          __builtin_elementwise_min(a2, b2));
                    }
                    const u16x2 c1 = __builtin_elementwise_min(lo[0], lo[1]);
                    const u16x2 c2 = __builtin_elementwise_min(__builtin_elementwise_max(lo[0], lo[1]),
                                                               __builtin_elementwise_min(hi[0], hi[1]));
                    const u16x2 o1 = AU(K1[gi]), o2 = AU(K2[gi]);
                    K1[gi] = U(__builtin_elementwise_min(o1, c1));
                    K2[gi] = U(__builtin_elementwise_min(__builtin_elementwise_max(o1, c1),
                                                         __builtin_elementwise_min(o2, c2)));
                }
            }
        }
        // ======== new state, pass 2: S scatter ================================================
#pragma unroll
        for (int gi = 0; gi < MAXG; ++gi) {
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) break;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(grow[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)(ri >> 16);
            const uint32_t dm = (1u << deg) - 1u;
            const uint32_t pos = ~NEG[gi] & (dm | (dm << 16));
            const uint32_t par_a = __popc(pos & 0xFFFFu) & 1u, par_b = __popc(pos >> 16) & 1u;
            const uint32_t parm = (par_a ? 0xFFFFu : 0u) | (par_b ? 0xFFFF0000u : 0u);
            NS[gi] = ~(pos ^ parm);                      // 1 = message negative (even count)
            const uint32_t k1 = K1[gi], k2 = K2[gi];
            OH[gi] = (1u << (k1 & 63u)) | (1u << (16 + ((k1 >> 16) & 63u)));
            const float wA = at[r0], wU = UCN ? au[r0] : 0.f;
            const float wa = (UCN && (SYN[gi] & 1u)) ? wU : wA;
            const float wb = (UCN && (SYN[gi] >> 16)) ? wU : wA;
            const int a1 = q_mag4((int)((k1 & 0xFFFFu) >> 6), wa, step, inv, qmax);
            const int b1 = q_mag4((int)(k1 >> 22), wb, step, inv, qmax);
            const int a2 = q_mag4((int)((k2 & 0xFFFFu) >> 6), wa, step, inv, qmax);
            const int b2 = q_mag4((int)(k2 >> 22), wb, step, inv, qmax);
            PA[gi] = gval[gi] ? pack2(a1, b1) : 0u;
            PB[gi] = gval[gi] ? pack2(a2, b2) : 0u;
#pragma unroll
            for (int c8 = 0; c8 < MAXDEG; c8 += 8) {
                if (c8 < deg) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int k = c8 + j;
                        if (k < MAXDEG && k < deg) {
                            const uint32_t pk = gad[gi][k >> 1];
                            const uint32_t addr = ((k & 1) ? (pk >> 16) : (pk & 0xFFFFu)) + sw_off;
                            const uint32_t c = msg4(k, PA[gi], PB[gi], OH[gi], NS[gi]);
                            if (gval[gi])
                                atomicAdd(reinterpret_cast<uint32_t*>(smem + addr), U(AU(c) + AU(BB)));
                        }
                    }
                }
            }
        }
        __syncthreads();
        // ======== variable nodes ===========================================================
        const bool last = (t == a.T - 1);
        const float2* btn = BT + (size_t)(last ? t : t + 1) * a.N;
        uint32_t any_hd = 0, any_pos = 0, nbits = 0;       // bit0: codeword p, bit1: p+CWP
        for (int r = 0; r < a.nent; ++r) {
            const int e = tid + r * NT;
            if (e < npe) {
                const uint32_t v = (uint32_t)e >> LOGP;
                const float2 bt = btn[__umulhi(v, a.zmagic)];
                const int bdeg = __float_as_int(bt.y);
                const uint32_t sw = SW[e];
                const int Sa = (int)(sw & 0xFFFFu) - bdeg;
                const int Sb = (int)(sw >> 16) - bdeg;
                const float cha = CH[v * CW + p], chb = CH[v * CW + p + CWP];
                int appa = q_units4(cha, inv, qmax) + Sa;
                int appb = q_units4(chb, inv, qmax) + Sb;
                appa = min(max(appa, -a.clip_u), a.clip_u);
                appb = min(max(appb, -a.clip_u), a.clip_u);
                if (!last) {
                    const int ta = q_units4(cha * bt.x, inv, qmax) + Sa;
                    const int tb = q_units4(chb * bt.x, inv, qmax) + Sb;
                    if (UCN)
                        TW[e] = pack2((ta & 0x7FFF) | ((appa >= 0) << 15), (tb & 0x7FFF) | ((appb >= 0) << 15));
                    else
                        TW[e] = pack2(ta, tb);
                    SW[e] = 0;
                }
                if ((int)v < a.target_bits) {
                    any_hd |= (uint32_t)(appa >= 0) | ((uint32_t)(appb >= 0) << 1);
                    if (last) {
                        any_pos |= (uint32_t)(appa > 0) | ((uint32_t)(appb > 0) << 1);
                        nbits += (uint32_t)(appa >= 0 && p < nvalid) + (uint32_t)(appb >= 0 && p + CWP < nvalid);
                    }
                    if (a.app_out) {
                        if (p < nvalid)
                            a.app_out[((size_t)t * a.B + b0 + p) * a.target_bits + v] = (float)appa * step;
                        if (p + CWP < nvalid)
                            a.app_out[((size_t)t * a.B + b0 + p + CWP) * a.target_bits + v] = (float)appb * step;
                    }
                }
                if (a.hd_out) {
#pragma unroll
                    for (int h2 = 0; h2 < 2; ++h2) {
                        const int c = p + h2 * CWP;
                        if ((h2 ? appb : appa) >= 0 && c < nvalid) {
                            const int64_t b = b0 + c;
                            const int64_t tile = b / TILE;
                            const int bl = (int)(b - tile * TILE);
                            const size_t idx = ((((size_t)(t + 1) * a.ntiles + tile) * nv + v) * 4) + (bl & 3);
                            atomicOr(reinterpret_cast<unsigned long long*>(a.hd_out + idx), 1ull << (bl >> 2));
                        }
                    }
                }
            }
        }
        {
            const unsigned long long ba = __ballot(any_hd & 1u), bb = __ballot(any_hd & 2u);
            unsigned long long ma = 0, mb = 0;
#pragma unroll
            for (int s2 = 0; s2 < SLOTS; ++s2) { ma |= (ba >> (s2 * CWP)) & pmask; mb |= (bb >> (s2 * CWP)) & pmask; }
            const unsigned long long m = ma | (mb << CWP);
            if (lane == 0 && m) atomicOr(&RED[0], m);
        }
        if (last) {
            const unsigned long long ba = __ballot(any_pos & 1u), bb = __ballot(any_pos & 2u);
            unsigned long long ma = 0, mb = 0;
#pragma unroll
            for (int s2 = 0; s2 < SLOTS; ++s2) { ma |= (ba >> (s2 * CWP)) & pmask; mb |= (bb >> (s2 * CWP)) & pmask; }
            const unsigned long long m = ma | (mb << CWP);
            if (lane == 0 && m) atomicOr(&RED[2], m);
            uint32_t nb = nbits;
            for (int off = 32; off > 0; off >>= 1) nb += __shfl_xor(nb, off);
            if (lane == 0 && nb) atomicAdd(&RED[3], (unsigned long long)nb);
        }
        __syncthreads();
    }
    if (tid == 0) {
        const unsigned long long wl = RED[0] & valid_cw;
        const unsigned long long all = RED[1] & RED[0] & valid_cw;
        const unsigned long long ap = RED[2] & valid_cw;
        if (a.counters) {
            const unsigned long long c0 = RED[3];
            const unsigned long long c1 = __popcll(wl);
            const unsigned long long c2 = __popcll(all);
            const unsigned long long c3 = 2ull * __popcll(ap) + __popcll(wl & ~ap);
            unsigned long long* cc = reinterpret_cast<unsigned long long*>(a.counters);
            if (c0) atomicAdd(cc + 0, c0);
            if (c1) atomicAdd(cc + 1, c1);
            if (c2) atomicAdd(cc + 2, c2);
            if (c3) atomicAdd(cc + 3, c3);
        }
        RED[5] = all;
        RED[6] = wl;
    }
    if (a.flags) {
        __syncthreads();
        if (tid < nvalid)
            a.flags[b0 + tid] = (uint8_t)(((RED[5] >> tid) & 1) | (((RED[6] >> tid) & 1) << 1));
    }
}

struct Shape4 {
    int cwp, maxg, maxdeg;
};
constexpr Shape4 kShapes4[] = {
    {8, 2, 16},    // z=24 (wman): 18 groups of 8 checks, 9 waves
    {8, 3, 16},    // 6 waves
    {4, 3, 16},    // z=64 (5G BG2): 16 checks per group
};

size_t f4_lds(int nv, int cwp, int T, int N) {
    const int cw = 2 * cwp;
    return ((((size_t)2 * nv * cwp + cw) * 4 + (size_t)nv * cw * 4 + 7) & ~(size_t)7) +
           (size_t)T * N * 8 + 8 * 8;
}

struct Plan4 {
    int shape = -1, nw = 0, hstep = 0, ngroups = 0;
    size_t lds = 0;
};

Plan4 plan4(const DevGraph& g, int T) {
    Plan4 best;
    double best_score = 0;
    if (g.z == 1 || g.max_cdeg > 16) return best;
    int forced = -1;
    if (const char* e = getenv("LDPC_F4_SHAPE")) forced = atoi(e);
    for (int si = 0; si < (int)(sizeof(kShapes4) / sizeof(kShapes4[0])); ++si) {
        if (forced >= 0 && si != forced) continue;
        const Shape4& sh = kShapes4[si];
        const int slots = 64 / sh.cwp;
        const int hstep = (g.z + slots - 1) / slots;
        const int ngroups = g.M * hstep;
        const int nw = (ngroups + sh.maxg - 1) / sh.maxg;
        if (nw > 16 || nw < 1) continue;
        const size_t lds = f4_lds(g.n_vars, sh.cwp, T, g.N);
        if (lds > F4_LDS_MAX) continue;
        if ((size_t)g.n_vars * sh.cwp * 4 * 2 >= 65536) continue;      // 16-bit byte addresses
        const int wgs = std::max(1, std::min((int)(F4_LDS_MAX / lds), 32 / nw));
        const double fill = (double)g.z / (double)(hstep * slots);     // valid slot fraction
        const double score = (double)(wgs * nw) * fill;
        if (score > best_score) {
            best_score = score;
            best.shape = si;
            best.nw = nw;
            best.hstep = hstep;
            best.ngroups = ngroups;
            best.lds = lds;
        }
    }
    return best;
}

template <int CWP, int MAXG, int MAXDEG, bool UCN>
int launch4k(const F4Args& a, int nblocks, int nw, size_t lds, const float* alpha,
             const float* alpha_ucn, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused4<CWP, MAXG, MAXDEG, UCN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)F4_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_fused4<CWP, MAXG, MAXDEG, UCN>), dim3(nblocks), dim3(64 * nw), lds, s, a,
                       alpha, alpha_ucn);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

template <int CWP, int MAXG, int MAXDEG>
int launch4s(const F4Args& a, int nblocks, int nw, size_t lds, const float* alpha,
             const float* alpha_ucn, hipStream_t s) {
    return alpha_ucn ? launch4k<CWP, MAXG, MAXDEG, true>(a, nblocks, nw, lds, alpha, alpha_ucn, s)
                     : launch4k<CWP, MAXG, MAXDEG, false>(a, nblocks, nw, lds, alpha, nullptr, s);
}

}  // namespace

bool fused4_supported(const DevGraph& g, int T, int qmax, bool per_edge_w) {
    if (per_edge_w) return false;
    if (qmax + 1 > 64) return false;
    return plan4(g, T).shape >= 0;
}

const char* fused4_shape_name(const DevGraph& g, int T) {
    static thread_local char buf[64];
    const Plan4 p = plan4(g, T);
    if (p.shape < 0) return "";
    const Shape4& sh = kShapes4[p.shape];
    snprintf(buf, sizeof(buf), "fused4[cwp%d,g%d,d%d,w%d]", sh.cwp, sh.maxg, sh.maxdeg, p.nw);
    return buf;
}

int fused4_decode(const DevGraph& g, const Bufs& b, const float* llr, int qmax, float step,
                  int clip_u, uint64_t* hd_out, int64_t* counters, uint8_t* flags, hipStream_t s) {
    const Plan4 p = plan4(g, b.T);
    if (p.shape < 0) return LDPC_ERR_UNSUPPORTED;
    const Shape4& sh = kShapes4[p.shape];
    F4Args a{};
    a.llr = llr;
    a.beta = b.beta;
    a.app_out = b.app_out;
    a.hd_out = hd_out;
    a.counters = counters;
    a.flags = flags;
    a.row_ptr = g.row_ptr;
    a.pe_col = g.pe_col;
    a.pe_shift = g.pe_shift;
    a.col_ptr = g.col_ptr;
    a.B = b.B;
    a.ntiles = b.ntiles;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.clip_u = clip_u;
    a.qmax = qmax;
    a.bias = qmax + 1;
    a.step = step;
    a.inv = 1.0f / step;
    a.n_vars = g.n_vars;
    a.N = g.N;
    a.E = g.E;
    a.z = g.z;
    a.hstep = p.hstep;
    a.ngroups = p.ngroups;
    a.nent = (g.n_vars * sh.cwp + 64 * p.nw - 1) / (64 * p.nw);
    a.zmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.z - 1) / (uint64_t)g.z);
    const int cw = 2 * sh.cwp;
    const int nblocks = (int)((b.B + cw - 1) / cw);
    switch (p.shape) {
        case 0: return launch4s<8, 2, 16>(a, nblocks, p.nw, p.lds, b.alpha, b.alpha_ucn, s);
        case 1: return launch4s<8, 3, 16>(a, nblocks, p.nw, p.lds, b.alpha, b.alpha_ucn, s);
        case 2: return launch4s<4, 3, 16>(a, nblocks, p.nw, p.lds, b.alpha, b.alpha_ucn, s);
        default: return LDPC_ERR_UNSUPPORTED;
    }
}

}  // namespace ldpc
