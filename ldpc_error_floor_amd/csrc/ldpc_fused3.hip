// ldpc_fused3.hip — fused QMS decoder, v3 (shape-specialised, occupancy-oriented).
//
// Same semantics as ldpc_fused.hip (v2) and oracle/nms_oracle.py; differences are in how the
// work maps onto a CU:
//  * the per-lane LDS byte address of every edge of every check group a wave owns is
//    computed once at kernel start and kept in VGPRs (two 16-bit addresses per register),
//    so an edge costs one VALU op of addressing instead of the cyclic-shift arithmetic;
//  * edge loops are fully unrolled up to MAXDEG (a compile-time bucket) and the LDS reads of
//    a check are issued 8 at a time before any of them is consumed;
//  * the previous iteration's hard decision is bit 15 of the Tv half of W (no HD array);
//  * the wave count per workgroup is chosen so the check groups split evenly, and the LDS
//    footprint (CW = 16 codewords for z > 1) leaves room for 2 workgroups per CU, so one
//    workgroup's barrier waits overlap the other's arithmetic.
//
//   LDS W[v][cw]  u32 = S_{t+1} (bits 31..16, ds_add) | hd_t (bit 15) | Tv (bits 14..0, signed)
//       CH[v][cw] f32 channel LLR;  BETA[T][N];  RED[8] frame-flag masks / counters
#include <cstdio>
#include <cstdlib>

#include "ldpc_fused.h"

namespace ldpc {

namespace {

constexpr int F3_BIG_U = 1023;               // "no other edge": value 10000 (Main_Functions.py:248)
constexpr size_t F3_LDS_MAX = 160 * 1024;

struct F3Args {
    const float* llr;
    const float* beta;
    float* app_out;
    uint64_t* hd_out;
    int64_t* counters;
    uint8_t* flags;
    const int32_t* row_ptr;
    const int32_t* pe_col;
    const int32_t* pe_shift;
    int64_t B;
    int ntiles, T, target_bits, clip_u, qmax;
    float inv, step;
    int n_vars, N, E, z;
    int hstep, ngroups, nent;
    uint32_t zmagic;
    int ablate;        // diagnostic only (LDPC_DIAG_ABLATE): 1 skip CN pass 1, 2 skip pass 2, 4 skip VN
};

__device__ __forceinline__ int q_units(float x, float inv, int qmax) {
    const float r = __builtin_amdgcn_fmed3f(rintf(x * inv), -(float)qmax, (float)qmax);
    return (int)r;
}
// Q(x) in grid units when x is already scaled by the (power-of-two) inverse step
__device__ __forceinline__ int q_scaled(float xs, float qm) {
    return (int)__builtin_amdgcn_fmed3f(rintf(xs), -qm, qm);
}

__device__ __forceinline__ int q_mag(int m, float w, float step, float inv, int qmax) {
    const float mv = (m >= F3_BIG_U) ? 10000.0f : (float)m * step;
    float x = mv * w;                          // fl32(|o| * w)
    x = (x > 0.f) ? x : 0.f;                   // x * [x > 0]
    return q_units(x, inv, qmax);
}

struct St3 {
    int mA, mB;        // quantized magnitudes (raw minima with per-edge weights)
    uint32_t oh;       // one-hot argmin edge
    uint32_t ns;       // bit k: message of edge k is negative (even count of other positives)
    int ucn;           // syndrome of the previous hard decision (per-edge weights only)
};

// -1 if bit k of x is set, else 0 (v_bfe_i32)

__device__ __forceinline__ int bfe1(uint32_t x, int k) {           // -1 if bit k set, else 0
    int r;
    asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(r) : "v"(x), "s"(k));
    return r;
}
__device__ __forceinline__ int bfi(int mask, int a, int b) {         // mask ? a : b (bitwise)
    int r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
    return r;
}

template <bool PEW>
__device__ __forceinline__ int msg3(const St3& s, int k, float w, float wu, float step, float inv,
                                    int qmax) {
    int m = bfi(bfe1(s.oh, k), s.mB, s.mA);                 // argmin edge ? mB : mA
    if constexpr (PEW) m = q_mag(m, s.ucn ? wu : w, step, inv, qmax);
    const int sg = bfe1(s.ns, k);
    return (m ^ sg) - sg;                                   // sg ? -m : m
}

__device__ __forceinline__ int med3i(int x, int lo, int hi) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "s"(hi));
    return r;
}

template <int CW, int MAXG, int MAXDEG, bool UCN, bool PEW>
__global__ void __launch_bounds__(1024)
k_fused3(F3Args a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn) {
    constexpr int SLOTS = 64 / CW;
    constexpr int LOGCW = (CW == 64) ? 6 : (CW == 32) ? 5 : (CW == 16) ? 4 : 3;
    constexpr int NPK = (MAXDEG + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nv = a.n_vars;
    const int total = nv * CW;
    uint32_t* W = reinterpret_cast<uint32_t*>(smem);                              // [nv*CW + CW]
    float* CH = reinterpret_cast<float*>(smem + ((size_t)total + CW) * 4);        // [nv*CW]
    float* BETA = CH + total;                                                     // [T*N]
    unsigned long long* RED = reinterpret_cast<unsigned long long*>(
        smem + ((((size_t)total + CW) * 4 + (size_t)total * 4 + (size_t)a.T * a.N * 4 + 15) & ~(size_t)15));

    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int NWV = NT >> 6;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slot = lane >> LOGCW;
    const int cw = lane & (CW - 1);
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int64_t nvalid = (b0 + CW <= a.B) ? CW : (a.B - b0);
    const unsigned long long cwmask = (CW == 64) ? ~0ull : ((1ull << CW) - 1);
    const unsigned long long valid_cw = (nvalid >= 64) ? ~0ull : ((1ull << nvalid) - 1);
    const int qmax = a.qmax;
    const float inv = a.inv, step = a.step;
    const int z = a.z;

    // ---- prologue: coalesced LLR block -> padded scratch -> CH[v][cw]; beta; W = Tv_0 | hd ----
    {
        float* scr = reinterpret_cast<float*>(W);            // [CW][nv+1]
        const int rl = nv + 1;
        for (int v0 = 0; v0 < nv; v0 += NT) {
            const int v = v0 + tid;
            float x[CW];
#pragma unroll
            for (int r = 0; r < CW; ++r)
                x[r] = (v < nv && r < nvalid) ? a.llr[(b0 + r) * nv + v] : 0.f;
#pragma unroll
            for (int r = 0; r < CW; ++r)
                if (v < nv) scr[r * rl + v] = x[r];
        }
        // beta pre-multiplied by 1/step (a power of two): fl32(ch*beta)/step == fl32(ch*(beta/step))
        for (int f = tid; f < a.T * a.N; f += NT) BETA[f] = a.beta[f] * inv;
        if (tid < 8) RED[tid] = (tid == 1) ? ~0ull : 0ull;
        __syncthreads();
        for (int e = tid; e < total; e += NT) CH[e] = scr[(e & (CW - 1)) * rl + (e >> LOGCW)];
        __syncthreads();
        for (int e = tid; e < total; e += NT) {
            const uint32_t v = (uint32_t)e >> LOGCW;
            const int t0 = q_scaled(CH[e] * BETA[__umulhi(v, a.zmagic)], (float)qmax);   // lw_0
            W[e] = ((uint32_t)t0 & 0x7FFFu) | ((uint32_t)(t0 >= 0) << 15);           // hd_{-1}
        }
    }

    // ---- per-group edge addresses (bytes, 16-bit packed), row info, lane validity ----------
    uint32_t gad[MAXG][NPK];
    uint32_t grow[MAXG];
    bool gval[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) {
        grow[gi] = 0;
        gval[gi] = false;
#pragma unroll
        for (int p = 0; p < NPK; ++p) gad[gi][p] = 0;
        const int grp = wave + gi * NWV;
        if (grp < a.ngroups) {
            const int i = grp / a.hstep;
            const int hg = grp - i * a.hstep;
            const int r0 = a.row_ptr[i];
            const int deg = a.row_ptr[i + 1] - r0;
            // consecutive checks on consecutive slots: their variable rows are adjacent, so
            // the two slots sharing a ds_read lane group hit disjoint bank halves
            const int h = hg * SLOTS + slot;
            gval[gi] = h < z;
            const int hl = (h < z) ? h : hg * SLOTS;
            grow[gi] = (uint32_t)r0 | ((uint32_t)deg << 16);
#pragma unroll
            for (int k = 0; k < MAXDEG; ++k) {
                const int pe = r0 + ((k < deg) ? k : deg - 1);
                int hs = hl + a.pe_shift[pe];
                hs = (hs >= z) ? hs - z : hs;
                const uint32_t byte = (uint32_t)(((a.pe_col[pe] * z + hs) << LOGCW) + cw) * 4u;
                gad[gi][k >> 1] |= (k & 1) ? (byte << 16) : byte;
            }
        }
    }
    __syncthreads();

    St3 st[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) { st[gi].mA = 0; st[gi].mB = 0; st[gi].oh = 0; st[gi].ns = 0; st[gi].ucn = 0; }

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {        // fold iteration t-1's frame flags (its VN phase is done)
            RED[1] &= RED[0];
            RED[0] = 0;
        }
        const float* at = alpha + (size_t)t * a.E;
        const float* au = UCN ? alpha_ucn + (size_t)t * a.E : nullptr;
        const float* atp = alpha + (size_t)(t > 0 ? t - 1 : 0) * a.E;
        const float* aup = UCN ? alpha_ucn + (size_t)(t > 0 ? t - 1 : 0) * a.E : nullptr;
        // ======== check nodes ================================================================
        // pass 1 for every group first (reads only), then pass 2 (S scatter): the groups'
        // dependency chains are independent, so the compiler can interleave them.
        uint32_t K1[MAXG], K2[MAXG], NEG[MAXG], SYN[MAXG];
#pragma unroll
        for (int gi = 0; gi < MAXG; ++gi) {
            K1[gi] = ((uint32_t)F3_BIG_U << 6) | 63u;
            K2[gi] = K1[gi];
            NEG[gi] = 0;
            SYN[gi] = 0;
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) break;
            if (a.ablate & 1) continue;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(grow[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)(ri >> 16);
            const St3& s = st[gi];
            uint32_t c1 = ((uint32_t)F3_BIG_U << 6) | 63u, c2 = c1;
            // one chunk of 8 edges; `full` is a literal at each call site, so full chunks carry
            // no masks, and in the last (partial) chunk slots k >= deg read a duplicate address
            // and are neutralised with wave-uniform masks — no per-edge branches either way.
            auto chunk = [&](const int c8, const bool full) __attribute__((always_inline)) {
                uint32_t wv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = c8 + j;
                    const uint32_t pk = gad[gi][k >> 1];
                    const uint32_t addr = (k & 1) ? (pk >> 16) : (pk & 0xFFFFu);
                    wv[j] = *reinterpret_cast<const uint32_t*>(smem + addr);
                }
                uint32_t kk[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = c8 + j;
                    const bool in = full || k < deg;
                    const int tv = ((int)(wv[j] << 17)) >> 17;                 // bits 14..0
                    const int kw = in ? k : 0;
                    const float w = PEW ? atp[r0 + kw] : 0.f;
                    const float wu = (PEW && UCN) ? aup[r0 + kw] : 0.f;
                    const int cold = msg3<PEW>(s, k, w, wu, step, inv, qmax);
                    const int d = tv - cold;                                   // V->C before Q
                    const uint32_t mag = (uint32_t)min(max(d, -d), qmax);      // |Q(v2c)|, 0 == +1e-4
                    kk[j] = (mag << 6) | (uint32_t)k;
                    if (!full) kk[j] |= in ? 0u : 0xFFFFFFFFu;
                    NEG[gi] |= ((uint32_t)d >> 31) << k;                      // Q keeps the sign
                    if (UCN) SYN[gi] ^= (wv[j] >> 15) & (in ? 1u : 0u);
                }
                uint32_t lo[4], hi[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) { lo[j] = min(kk[2 * j], kk[2 * j + 1]); hi[j] = max(kk[2 * j], kk[2 * j + 1]); }
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t a1 = lo[2 * j], a2 = hi[2 * j], b1 = lo[2 * j + 1], b2 = hi[2 * j + 1];
                    lo[j] = min(a1, b1);
                    hi[j] = min(max(a1, b1), min(a2, b2));
                }
                const uint32_t d1 = min(lo[0], lo[1]);
                const uint32_t d2 = min(max(lo[0], lo[1]), min(hi[0], hi[1]));
                const uint32_t o1 = c1, o2 = c2;
                c1 = min(o1, d1);
                c2 = min(max(o1, d1), min(o2, d2));
            };
#pragma unroll
            for (int c8 = 0; c8 < MAXDEG; c8 += 8) {
                if (c8 + 8 <= deg) chunk(c8, true);
                else if (c8 < deg) chunk(c8, false);
            }
            uint32_t lo[1] = {c1}, hi[1] = {c2};
            K1[gi] = lo[0];
            K2[gi] = hi[0];
        }
#pragma unroll
        for (int gi = 0; gi < MAXG; ++gi) {
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) break;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(grow[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)(ri >> 16);
            St3& s = st[gi];
            const uint32_t dmask = (deg >= 32) ? 0xFFFFFFFFu : ((1u << deg) - 1u);
            const uint32_t pos = ~NEG[gi] & dmask;
            const uint32_t par = __popc(pos) & 1u;
            const uint32_t syn = SYN[gi];
            s.ns = ~(pos ^ (par ? 0xFFFFFFFFu : 0u));      // negative: even count of other positives
            s.oh = 1u << (K1[gi] & 63u);
            s.ucn = (int)syn;
            const int m1 = (int)(K1[gi] >> 6), m2 = (int)(K2[gi] >> 6);
            if (PEW) {
                s.mA = m1;
                s.mB = m2;
            } else {
                const float w = (UCN && syn) ? au[r0] : at[r0];
                s.mA = q_mag(m1, w, step, inv, qmax);
                s.mB = q_mag(m2, w, step, inv, qmax);
            }
            if (!gval[gi]) { s.mA = 0; s.mB = 0; }    // duplicate stand-in check: no messages
            if (a.ablate & 2) continue;
            auto scatter = [&](const int c8, const bool full) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int k = c8 + j;
                    const bool in = full || k < deg;
                    const uint32_t pk = gad[gi][k >> 1];
                    const uint32_t addr = (k & 1) ? (pk >> 16) : (pk & 0xFFFFu);
                    const int kw = in ? k : 0;
                    const float w = PEW ? at[r0 + kw] : 0.f;
                    const float wu = (PEW && UCN) ? au[r0 + kw] : 0.f;
                    const int c = msg3<PEW>(s, k, w, wu, step, inv, qmax);
                    uint32_t v = (uint32_t)c << 16;
                    if (!full) v &= in ? 0xFFFFFFFFu : 0u;                    // padding slot adds 0
                    atomicAdd(reinterpret_cast<uint32_t*>(smem + addr), v);
                }
            };
#pragma unroll
            for (int c8 = 0; c8 < MAXDEG; c8 += 8) {
                if (c8 + 8 <= deg) scatter(c8, true);
                else if (c8 < deg) scatter(c8, false);
            }
        }
        __syncthreads();
        // ======== variable nodes ===========================================================
        const bool last = (t == a.T - 1);
        const float* bnext = BETA + (size_t)(last ? t : t + 1) * a.N;
        uint32_t any_hd = 0, any_pos = 0, nbits = 0;
        const float qmf = (float)qmax;
        const bool full_target = a.target_bits >= nv;
        if (a.app_out == nullptr && a.hd_out == nullptr) {
            // fast path: 4 entries' LDS reads in flight before any is consumed
            for (int r0 = 0; r0 < ((a.ablate & 4) ? 0 : a.nent); r0 += 4) {
                uint32_t wv[4], vv[4];
                float chv[4], bv[4];
                bool in[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int e = tid + (r0 + j) * NT;
                    in[j] = e < total;
                    const int ee = in[j] ? e : tid;
                    vv[j] = (uint32_t)ee >> LOGCW;
                    wv[j] = W[ee];
                    chv[j] = CH[ee];
                    bv[j] = bnext[__umulhi(vv[j], a.zmagic)];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int e = tid + (r0 + j) * NT;
                    const int S = (int)wv[j] >> 16;
                    int app = q_scaled(chv[j] * inv, qmf) + S;                // Q(xa) + sum C2V
                    app = med3i(app, -a.clip_u, a.clip_u);                   // clip +-clip_LLR
                    if (in[j]) {
                        if (!last) {
                            const int tn = q_scaled(chv[j] * bv[j], qmf) + S;
                            W[e] = UCN ? (((uint32_t)tn & 0x7FFFu) | (((uint32_t)~app >> 16) & 0x8000u))
                                       : ((uint32_t)tn & 0xFFFFu);
                        }
                        const bool tgt = full_target || (int)vv[j] < a.target_bits;
                        const uint32_t hdb = (uint32_t)(app >= 0) & (uint32_t)tgt;
                        any_hd |= hdb;
                        if (last) { any_pos |= (uint32_t)(app > 0) & (uint32_t)tgt; nbits += hdb; }
                    }
                }
            }
        } else {
        for (int r = 0; r < ((a.ablate & 4) ? 0 : a.nent); ++r) {
            const int e = tid + r * NT;
            if (e < total) {
                const uint32_t v = (uint32_t)e >> LOGCW;
                const uint32_t wv = W[e];
                const int S = (int)wv >> 16;
                const float ch = CH[e];
                int app = q_units(ch, inv, qmax) + S;                    // Q(xa) + sum C2V
                app = min(max(app, -a.clip_u), a.clip_u);                // clip +-clip_LLR
                if (!last) {
                    const int tn = q_scaled(ch * bnext[__umulhi(v, a.zmagic)], (float)qmax) + S;
                    W[e] = ((uint32_t)tn & 0x7FFFu) | ((uint32_t)(app >= 0) << 15);
                }
                if ((int)v < a.target_bits) {
                    any_hd |= (uint32_t)(app >= 0);
                    if (last) { any_pos |= (uint32_t)(app > 0); nbits += (uint32_t)(app >= 0); }
                    if (a.app_out && cw < nvalid)
                        a.app_out[((size_t)t * a.B + b0 + cw) * a.target_bits + v] = (float)app * step;
                }
                if (a.hd_out && app >= 0 && cw < nvalid) {
                    const int64_t b = b0 + cw;
                    const int64_t tile = b / TILE;
                    const int bl = (int)(b - tile * TILE);
                    const size_t idx = ((((size_t)(t + 1) * a.ntiles + tile) * nv + v) * 4) + (bl & 3);
                    atomicOr(reinterpret_cast<unsigned long long*>(a.hd_out + idx), 1ull << (bl >> 2));
                }
            }
        }
        }
        unsigned long long bw = __ballot(any_hd);
        unsigned long long m = 0;
#pragma unroll
        for (int s2 = 0; s2 < SLOTS; ++s2) m |= (bw >> (s2 * CW)) & cwmask;
        if (lane == 0 && m) atomicOr(&RED[0], m);
        if (last) {
            bw = __ballot(any_pos);
            m = 0;
#pragma unroll
            for (int s2 = 0; s2 < SLOTS; ++s2) m |= (bw >> (s2 * CW)) & cwmask;
            if (lane == 0 && m) atomicOr(&RED[2], m);
            uint32_t nb = (cw < nvalid) ? nbits : 0u;
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

// ---- shapes ------------------------------------------------------------------------------
struct Shape3 {
    int cw, maxg, maxdeg;
};
constexpr Shape3 kShapes[] = {
    {16, 3, 16},   // wman-like (z=24, deg 14-15)
    {16, 3, 24},   // 802.11n-like (deg 22)
    {8, 5, 16},    // 5G BG2-like (z=64, deg <= 10)
    {64, 3, 8},    // z=1 sparse (MacKay)
    {64, 2, 32},   // z=1 dense rows (BCH)
};

size_t f3_lds(int nv, int cw, int T, int N) {
    return ((((size_t)nv * cw + cw) * 4 + (size_t)nv * cw * 4 + (size_t)T * N * 4 + 15) & ~(size_t)15) + 8 * 8;
}

struct Plan3 {
    int shape = -1, nw = 0, hstep = 0, ngroups = 0;
    size_t lds = 0;
};

Plan3 plan3(const DevGraph& g, int T) {
    Plan3 best;
    double best_score = 0;
    for (int si = 0; si < (int)(sizeof(kShapes) / sizeof(kShapes[0])); ++si) {
        const Shape3& sh = kShapes[si];
        if ((g.z == 1) != (sh.cw == 64)) continue;
        if (g.max_cdeg > sh.maxdeg) continue;
        const int slots = 64 / sh.cw;
        const int hstep = (g.z + slots - 1) / slots;
        const int ngroups = g.M * hstep;
        const int nw = (ngroups + sh.maxg - 1) / sh.maxg;
        if (nw > 16 || nw < 1) continue;
        const size_t lds = f3_lds(g.n_vars, sh.cw, T, g.N);
        if (lds > F3_LDS_MAX) continue;
        if ((size_t)g.n_vars * sh.cw * 4 + sh.cw * 4 >= 65536) continue;    // 16-bit addresses
        const int wg_lds = (int)(F3_LDS_MAX / lds);
        const int wg_waves = 32 / nw;
        const int wgs = std::max(1, std::min(wg_lds, wg_waves));
        // occupancy (waves per CU) x edge-slot efficiency (deg / MAXDEG rounded to chunks)
        const double eff = (double)g.max_cdeg / (double)(((g.max_cdeg + 7) / 8) * 8);
        const double score = (double)(wgs * nw) * eff + 1e-3 * sh.cw;
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

template <int CW, int MAXG, int MAXDEG, bool UCN, bool PEW>
int launch3k(const F3Args& a, int nblocks, int nw, size_t lds, const float* alpha,
             const float* alpha_ucn, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused3<CW, MAXG, MAXDEG, UCN, PEW>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)F3_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_fused3<CW, MAXG, MAXDEG, UCN, PEW>), dim3(nblocks), dim3(64 * nw), lds, s,
                       a, alpha, alpha_ucn);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

template <int CW, int MAXG, int MAXDEG>
int launch3s(const F3Args& a, int nblocks, int nw, size_t lds, const float* alpha,
             const float* alpha_ucn, bool pew, hipStream_t s) {
    if (alpha_ucn)
        return pew ? launch3k<CW, MAXG, MAXDEG, true, true>(a, nblocks, nw, lds, alpha, alpha_ucn, s)
                   : launch3k<CW, MAXG, MAXDEG, true, false>(a, nblocks, nw, lds, alpha, alpha_ucn, s);
    return pew ? launch3k<CW, MAXG, MAXDEG, false, true>(a, nblocks, nw, lds, alpha, nullptr, s)
               : launch3k<CW, MAXG, MAXDEG, false, false>(a, nblocks, nw, lds, alpha, nullptr, s);
}

}  // namespace

bool fused3_supported(const DevGraph& g, int T) { return plan3(g, T).shape >= 0; }

const char* fused3_shape_name(const DevGraph& g, int T) {
    static thread_local char buf[64];
    const Plan3 p = plan3(g, T);
    if (p.shape < 0) return "";
    const Shape3& sh = kShapes[p.shape];
    snprintf(buf, sizeof(buf), "fused3[cw%d,g%d,d%d,w%d]", sh.cw, sh.maxg, sh.maxdeg, p.nw);
    return buf;
}

int fused3_decode(const DevGraph& g, const Bufs& b, const float* llr, int qmax, float step,
                  int clip_u, bool per_edge_w, uint64_t* hd_out, int64_t* counters,
                  uint8_t* flags, hipStream_t s) {
    const Plan3 p = plan3(g, b.T);
    if (p.shape < 0) return LDPC_ERR_UNSUPPORTED;
    const Shape3& sh = kShapes[p.shape];
    F3Args a{};
    a.llr = llr;
    a.beta = b.beta;
    a.app_out = b.app_out;
    a.hd_out = hd_out;
    a.counters = counters;
    a.flags = flags;
    a.row_ptr = g.row_ptr;
    a.pe_col = g.pe_col;
    a.pe_shift = g.pe_shift;
    a.B = b.B;
    a.ntiles = b.ntiles;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.clip_u = clip_u;
    a.qmax = qmax;
    a.step = step;
    a.inv = 1.0f / step;
    a.n_vars = g.n_vars;
    a.N = g.N;
    a.E = g.E;
    a.z = g.z;
    a.hstep = p.hstep;
    a.ngroups = p.ngroups;
    a.nent = (g.n_vars * sh.cw + 64 * p.nw - 1) / (64 * p.nw);
    a.zmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.z - 1) / (uint64_t)g.z);
    if (const char* e = getenv("LDPC_DIAG_ABLATE")) a.ablate = atoi(e);   // timing only
    const int nblocks = (int)((b.B + sh.cw - 1) / sh.cw);
    const float* au = b.alpha_ucn;
    switch (p.shape) {
        case 0: return launch3s<16, 3, 16>(a, nblocks, p.nw, p.lds, b.alpha, au, per_edge_w, s);
        case 1: return launch3s<16, 3, 24>(a, nblocks, p.nw, p.lds, b.alpha, au, per_edge_w, s);
        case 2: return launch3s<8, 5, 16>(a, nblocks, p.nw, p.lds, b.alpha, au, per_edge_w, s);
        case 3: return launch3s<64, 3, 8>(a, nblocks, p.nw, p.lds, b.alpha, au, per_edge_w, s);
        case 4: return launch3s<64, 2, 32>(a, nblocks, p.nw, p.lds, b.alpha, au, per_edge_w, s);
        default: return LDPC_ERR_UNSUPPORTED;
    }
}

}  // namespace ldpc
