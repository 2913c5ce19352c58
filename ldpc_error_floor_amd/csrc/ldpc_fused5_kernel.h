#pragma once
// ldpc_fused5_kernel.h — fused QMS decoder, v5: byte-packed check state, 2-op message decode.
// (kernel template; shared by ldpc_fused5.hip (planning, tables, dispatch) and the per-shape
// translation units built from ldpc_fused5_shape.hip)
//
// Same semantics and work mapping as v3 (ldpc_fused3.hip: one workgroup owns CW codewords for
// all T iterations, lane = slot*CW + cw, a wave's slots take consecutive checks of one proto
// row, per-edge LDS addresses precomputed and packed 2x16 bit).  What changes is how a check's
// compressed min-sum state is held and decoded, which sets the VALU count per edge:
//
//  * P   — one VGPR holding the check's four possible output messages as signed bytes
//          [-mA, +mA, -mB, +mB] (mA: min over all edges, mB: second minimum, both already
//          weighted and quantized, in grid units);
//  * SEL — one selector byte per edge, four edges per VGPR: byte = 2*is_argmin + (v2c >= 0),
//          the index of the edge's message inside P.  v_perm_b32(P, P, SEL[w]) yields four
//          edges' messages, and pass 1 subtracts a message straight from its byte with an
//          SDWA sign-extended source: a quarter op per edge to decode (v3: 5 ops);
//  * pass 2 (scatter) of a group runs right after its state update (F5_P2_MODE).
//  * pass 1 folds V->C magnitudes with one v_min + one v_med3 per edge (running first/second
//    minimum of key = |v2c| << 8 | edge code, |v2c| from the offset-binary difference with one
//    v_sad_u16), and the V->C signs with one v_perm per edge, which appends the offset-binary
//    byte (bit 7: "v2c >= 0") to a SEL-shaped word;
//    the quantizer clamp moves after the minimum (clamp is monotonic);
//  * W[v][cw] = hd (bit 31) | Tv + 128 (bits 30..16) | S + 2^14 (bits 15..0): pass 1 reads Tv
//    with an SDWA word select, pass 2 adds the message without a shift;
//  * an edge slot past a check's degree points at a per-lane dummy word whose Tv is -96: its
//    |v2c| never wins a minimum, its sign is negative (not counted), its hd bit is 0, and pass 2
//    adds into it harmlessly (the VN phase resets it), so partial chunks need no masks.
//
// Per-edge weights (sharing types with one weight per edge) keep raw minima in P (16 bit
// each) and quantize per edge at decode; this path is correct but not tuned.
#include <algorithm>
#include <climits>
#include <type_traits>
#include <vector>
#include <cstdio>
#include <cstdlib>

#include "ldpc_awgn.h"
#include "ldpc_fused.h"

namespace ldpc {

namespace f5 {

// pass-2 placement: 0 = every group's pass 1 + state, then every group's scatter; 1 = each
// group's scatter right after its state update (pass-1 reads of Tv are unaffected by the
// scatter's adds into the biased S field, so the order is free)
#ifndef F5_P2_MODE
#define F5_P2_MODE 1
#endif
constexpr int F5_BIG_U = 1023;               // "no other edge": value 10000 (Main_Functions.py:248)
constexpr size_t F5_LDS_MAX = 160 * 1024;
constexpr uint32_t F5_SBIAS = 16384;         // S field bias (bits 14..0)
// W's Tv field holds Tv + F5_TVB: pass 1's byte subtract then yields V->C + 128 in offset
// binary, whose distance from 128 (one v_sad_u16) is |V->C| and whose top bit is "V->C >= 0"
constexpr int F5_TVB = 128;
// padding edges read this word: Tv = -96 gives a V->C value in [-127, -65] for any message
// (|m| <= 31): negative (absent from the count of positive signs), never below qmax and inside
// the 8-bit range pass 1 works in
constexpr uint32_t F5_DUMMY_W = ((uint32_t)(F5_TVB - 96) << 16) | F5_SBIAS;
// one dummy word per lane (after W): padding slots of different lanes never add into the same
// LDS word, so their pass-2 atomics do not serialise
constexpr int F5_NDUMMY = 64;
constexpr float F5_MAGIC = 12582912.0f;                 // 1.5 * 2^23
constexpr int F5_MAGIC_BITS = 0x4B400000;              // bit pattern of F5_MAGIC
constexpr int F5_APP0 = F5_MAGIC_BITS + (int)F5_SBIAS;  // APP == 0 in the VN's biased domain
// (Tv + F5_APP0) * 2^16 + F5_WBIAS == ((Tv + F5_TVB) << 16) | F5_SBIAS  (mod 2^32)
constexpr uint32_t F5_WBIAS = F5_SBIAS + (uint32_t)F5_TVB * 65536u - (uint32_t)F5_APP0 * 65536u;
// APP path magic: 1.5 * 2^23 + 2^22 - S bias, same binade, so Q(y) + APP bits land at
// F5_APPH + APP with F5_APPH = 0x4B800000: APP >= 0 exactly when bit 23 is set (an OR over
// entries then answers "any hard decision 1")
constexpr float F5_MAGIC_A = 16760832.0f;
// counters-only VN without UCN: bits 0x4B7F4000, so the low 16 bits of its Q(y) bits plus the W
// word's low half (S + 2^14) are APP + 0x8000, whose bit 15 is [APP >= 0]
constexpr float F5_MAGIC_H = 16728064.0f;
static_assert(16728064 == 8388608 + 0x7F4000, "F5_MAGIC_H bits 0x4B7F4000");
constexpr int F5_APPH = 0x4B800000;
static_assert(12582912 + 4194304 - (int)F5_SBIAS == 16760832, "APP magic");

struct F5Args {
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
    int ngroups, nent;
    int nfull, cpw;    // VN: full 64-entry chunks, chunks per wave
    int Mp;            // proto rows
    const float* betas;        // [T][N] beta (the kernel keeps ch / step)
    const uint16_t* qtab;      // [T][qslice] weight tables (setup kernel), LUT builds only
    int qslice;                // halfwords per iteration: [alpha | alpha_ucn][Mp][qrow], even
    int qrow;                  // halfwords per table row: 3 qmax + 2
    int qucn;                  // halfword offset of the alpha_ucn table inside a slice
    const uint32_t* gad;       // [ngroups][NPK][64] packed edge byte addresses (k_f5_gad)
    const uint4* grow;         // [ngroups] {r0 | deg << 16 | row << 24, lane-valid mask lo, hi, 0}
    unsigned long long* stamps;   // diagnostic (LDPC_DIAG_STAMPS): [block][8] s_memtime marks
    int gen;                   // 1: LLRs from the in-kernel AWGN channel (awgn), llr unused
    AwgnParams awgn;
    uint32_t zmagic;
    int ablate;        // diagnostic only (LDPC_DIAG_ABLATE): 1 skip CN pass 1, 2 skip pass 2, 4 skip VN
    const uint32_t* only;  // null, or [packs of 32 codewords]: decode only blocks of flagged packs
    uint32_t* iter_wrong;  // [T][ceil(B/32)] per-iteration frame-error words (zeroed), or null
};

__device__ __forceinline__ int q_units5(float x, float inv, int qmax) {
    return (int)__builtin_amdgcn_fmed3f(rintf(x * inv), -(float)qmax, (float)qmax);
}
// Q(x) in grid units when x is already scaled by the (power-of-two) inverse step
__device__ __forceinline__ int q_scaled5(float xs, float qm) {
    return (int)__builtin_amdgcn_fmed3f(rintf(xs), -qm, qm);
}
// quantized C->V magnitude: Q(relu(|o| * w)), |o| in grid units (>= F5_BIG_U: the 10000 rule)
__device__ __forceinline__ int q_mag5(int m, float w, float step, float inv, int qmax) {
    const float mv = (m >= F5_BIG_U) ? 10000.0f : (float)m * step;
    float x = mv * w;                          // fl32(|o| * w)
    x = (x > 0.f) ? x : 0.f;                   // x * [x > 0]
    return q_units5(x, inv, qmax);
}

// 16-bit VOP2 forms: full issue rate on gfx950 where the 32-bit min / max / shift-left and
// every SDWA / VOP3 form take twice the cycles (tools/valu_table.hip); the high half of the
// result is zeroed.
__device__ __forceinline__ uint32_t min_u16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// LDS word at a byte address (the decoder's dynamic LDS starts at 0: k_fused5 checks)
typedef __attribute__((address_space(3))) uint32_t LdsU32;
// the low / high 16-bit byte address of a packed pair
__device__ __forceinline__ uint32_t lo16(uint32_t x) {
    uint32_t r;
    asm("v_and_b32 %0, 0xffff, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t hi16(uint32_t x) {
    uint32_t r;
    asm("v_lshrrev_b32 %0, 16, %1" : "=v"(r) : "v"(x));
    return r;
}
// d256 = (Tv + 128 - m mod 256) << 8, bits 31..16 zero: V->C in offset binary in byte 1, whose
// bit 7 (bit 15) is "Tv - m >= 0"; the high half of the W word holds Tv + F5_TVB, m = signed
// byte POS of r.  Exact while |Tv - m| <= 127 (Tv is kept within +-2 qmax, |m| <= qmax <= 31).
template <int POS>
__device__ __forceinline__ uint32_t sub_d256(uint32_t w, uint32_t r) {
    uint32_t d;
    if constexpr (POS == 0)
        asm("v_sub_u32_sdwa %0, sext(%1), sext(%2) dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_0"
            : "=v"(d) : "v"(w), "v"(r));
    else if constexpr (POS == 1)
        asm("v_sub_u32_sdwa %0, sext(%1), sext(%2) dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_1"
            : "=v"(d) : "v"(w), "v"(r));
    else if constexpr (POS == 2)
        asm("v_sub_u32_sdwa %0, sext(%1), sext(%2) dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_2"
            : "=v"(d) : "v"(w), "v"(r));
    else
        asm("v_sub_u32_sdwa %0, sext(%1), sext(%2) dst_sel:BYTE_1 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_3"
            : "=v"(d) : "v"(w), "v"(r));
    return d;
}

// min(max(a, lo), hi) on the low 16 bits, bounds uniform (SGPR)
__device__ __forceinline__ uint32_t clamp_i16(uint32_t a, uint32_t lo, uint32_t hi) {
    uint32_t r;
    asm("v_max_i16 %0, %1, %2" : "=v"(r) : "s"(lo), "v"(a));
    asm("v_min_i16 %0, %1, %2" : "=v"(r) : "s"(hi), "v"(r));
    return r;
}
// key = |V->C| << 8 | code = |d256 - 0x8000| + code.  (v_sad_u16 sums the absolute differences
// of BOTH 16-bit halves, tools/probe/sad_probe.hip: d256's high half is zero, and so is ksad's.)
__device__ __forceinline__ uint32_t key_sad(uint32_t d256, uint32_t ksad, uint32_t code) {
    return __builtin_amdgcn_sad_u16(d256, ksad, code);
}
// NG << 8 | byte 1 of d: appends an edge's offset-binary V->C byte to a selector-shaped word
__device__ __forceinline__ uint32_t append_b1(uint32_t ng, uint32_t d) {
    return __builtin_amdgcn_perm(ng, d, 0x06050401u);
}

// the lane index, recomputed where it is used (2 VALU): volatile, so the compiler can neither
// hoist it nor keep values derived from it live across the check phase, where the register
// budget of the shape is exhausted and such values were spilled to scratch (one scratch store
// per wave and block: the kernel's only HBM writes besides the counters)
__device__ __forceinline__ uint32_t lane_fresh() {
    uint32_t r;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
    return r;
}

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---- SEL layout: edge k -> byte of word k/4, counted from the last inserted edge ------------
// A selector byte is 2*is_argmin + (V->C >= 0): the index of the edge's message inside P, so
// v_perm_b32(P, P, SEL[w]) yields the messages of four edges at once.
template <int MAXDEG>
struct Sel {
    static constexpr int NSEL = (MAXDEG + 3) / 4;
    static constexpr int nins(int w) { return (MAXDEG - 4 * w) < 4 ? (MAXDEG - 4 * w) : 4; }
    static constexpr int pos(int k) { return nins(k / 4) - 1 - (k % 4); }
    static constexpr uint32_t code(int k) { return ((uint32_t)(k / 4) << 5) | (uint32_t)(8 * pos(k) + 1); }
    static constexpr uint32_t bmask(int w) {
        uint32_t m = 0;
        for (int i = 0; i < nins(w); ++i) m |= 1u << (8 * i);
        return m;
    }
    // number of edges of word w inside chunk [c8, c8+8)
    static constexpr int in_chunk(int w, int c8) {
        int n = 0;
        for (int k = c8; k < c8 + 8 && k < MAXDEG; ++k) n += (k / 4 == w);
        return n;
    }
};

// diagnostic phase marks: wave 0 lane 0 of each workgroup records s_memrealtime (100 MHz)
#define F5_STAMP(i)                                                                         \
    do {                                                                                    \
        if (a.stamps && tid == 0) a.stamps[(size_t)bx * 32 + (i)] = __builtin_amdgcn_s_memrealtime();       \
    } while (0)

// per-slot degree bound: a wave's first HG group slots take rows of degree <= MAXDEG, the
// others rows of degree <= LDEG (shapes for graphs whose rows differ widely in degree: the
// state of a light slot needs fewer registers).  HG == MAXG: one bound for every slot.
template <int MAXDEG, int HG, int LDEG>
struct GDeg {
    static constexpr int deg(int gi) { return gi < HG ? MAXDEG : LDEG; }
    static constexpr int nsel(int gi) { return (deg(gi) + 3) / 4; }
    static constexpr int npk(int gi) { return (deg(gi) + 1) / 2; }
};
constexpr int f5_logcw(int cw) { return cw == 64 ? 6 : cw == 32 ? 5 : cw == 16 ? 4 : cw == 8 ? 3 : 2; }

// WPE: the shape's occupancy target (waves per SIMD): the VGPR budget that lets the planned
// number of workgroups share a CU (Shape5::wpe; plan5 assumes the same figure)
template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE, bool UCN, bool PEW, bool OUT, bool LUT>
__device__ __forceinline__ void
f5_block(const F5Args& a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn, const int64_t bx) {
    using SL = Sel<MAXDEG>;                 // selector layout of every slot (light ones use a prefix)
    using GD = GDeg<MAXDEG, HG, LDEG>;
    constexpr int NSEL = SL::NSEL;
    constexpr int SLOTS = 64 / CW;
    constexpr int LOGCW = f5_logcw(CW);
    constexpr int NPK = (MAXDEG + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nv = a.n_vars;
    const int total = nv * CW;
    uint32_t* W = reinterpret_cast<uint32_t*>(smem);                              // [nv*CW + CW]
    float* CH = reinterpret_cast<float*>(smem + ((size_t)total + F5_NDUMMY) * 4); // [nv*CW]
    // CH holds ch / step (exact: step is a power of two), so Q(ch) is a clamp and rounding of
    // CH, and Q(fl32(ch * beta)) in grid units is that of fl32(CH * beta)
    float* BETA = CH + total;                     // [2][N]: beta_t in slot t & 1
    unsigned long long* RED = reinterpret_cast<unsigned long long*>(
        smem + ((((size_t)total + F5_NDUMMY) * 4 + (size_t)total * 4 + (size_t)2 * a.N * 4 + 15) & ~(size_t)15));
    uint16_t* QT = reinterpret_cast<uint16_t*>(RED + 8);                          // [2][qslice]

    if ((uint32_t)(uintptr_t)smem != 0u) __builtin_trap();   // edge addresses are LDS-absolute
    if (a.only && a.only[(bx * CW) >> 5] == 0u) return;   // bit-sliced fixup
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int NWV = NT >> 6;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cw = lane & (CW - 1);
    const int64_t b0 = bx * CW;
    const int64_t nvalid = (b0 + CW <= a.B) ? CW : (a.B - b0);
    const unsigned long long cwmask = (CW == 64) ? ~0ull : ((1ull << CW) - 1);
    const unsigned long long valid_cw = (nvalid >= 64) ? ~0ull : ((1ull << nvalid) - 1);
    const int qmax = a.qmax;
    const float inv = a.inv, step = a.step;
    const int z = a.z;

    if (a.only && a.hd_out) {
        // bit-sliced fixup with a hard-bit export: nobody zeroed the tile buffer (the host
        // skips that memset for bit-sliced decodes), so clear this block's codeword bits of the
        // iterations the export reads (slots t + 1, t < T) before the VN phases OR them in.
        // Other blocks of the same tile own other bits of the same words: atomicAnd only.
        const int64_t tile = b0 / TILE;
        const int bl0 = (int)(b0 - tile * TILE);          // CW divides TILE: one tile per block
        const int n = a.T * nv * 4;
        for (int i = tid; i < n; i += NT) {
            const int w = i & 3;
            const int v = (i >> 2) % nv;
            const int t = (i >> 2) / nv;
            const int kmin = (bl0 - w + 3) >> 2, kmax = (bl0 + (int)nvalid - 1 - w) >> 2;
            if (kmax < kmin) continue;
            const unsigned long long m = ((kmax - kmin == 63) ? ~0ull : ((2ull << (kmax - kmin)) - 1)) << kmin;
            atomicAnd(reinterpret_cast<unsigned long long*>(
                          a.hd_out + ((((size_t)(t + 1) * a.ntiles + tile) * nv + v) * 4) + w), ~m);
        }
        __syncthreads();
    }

    F5_STAMP(0);
    // ---- prologue: coalesced LLR block -> padded scratch -> CH[v][cw]; beta; W = Tv_0 | hd ----
    {
        float* scr = reinterpret_cast<float*>(W);            // [CW][nv+1]
        const int rl = nv + 1;
        if (a.gen) {
            // in-kernel channel: the same QMS level sampler as ldpc_channel_awgn (ldpc_awgn.h),
            // its bucket table in the CH region (written only after the scratch is consumed)
            const AwgnParams& g = a.awgn;
            const uint64_t g0 = (uint64_t)g.offset + (uint64_t)b0;    // global index of row 0
            if ((size_t)total * 4 >= (2u << AWGN_KB) + (3 * AWGN_NB_MAX + 1) * 4) {
                uint16_t* bk = reinterpret_cast<uint16_t*>(CH);
                uint32_t* th = reinterpret_cast<uint32_t*>(CH) + (1 << AWGN_KB) / 2;
                uint32_t* tl = th + AWGN_NB_MAX;
                float* vl = reinterpret_cast<float*>(tl + AWGN_NB_MAX);
                awgn_bucket_fill(g, bk, th, tl, tid, NT);
                if (tid <= g.nb) vl[tid] = g.val[tid];
                __syncthreads();
                const int sh = (int)(g0 & 3);
                const int nq = (CW + sh + 3) >> 2;                     // quads covering the rows
                for (int i = tid; i < nq * nv; i += NT) {
                    const int m = i / nv, v = i - m * nv;
                    const int fx = awgn_fixed(g, v + 1);
                    int lv[4] = {0, 0, 0, 0};
                    if (fx == 0) awgn_levels4(g, bk, th, tl, (uint32_t)v, (g0 >> 2) + (uint64_t)m, lv);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 4 * m + j - sh;
                        if (r < 0 || r >= CW) continue;
                        scr[r * rl + v] = r >= nvalid ? 0.f : fx == 0 ? vl[lv[j]] : fx == 1 ? 0.f : -g.clip;
                    }
                }
            } else {                   // tiny graphs: a threshold scan per element
                for (int i = tid; i < CW * nv; i += NT) {
                    const int r = i / nv, v = i - r * nv;
                    scr[r * rl + v] = r < nvalid ? awgn_qms_elem(g, g0 + (uint64_t)r, v) : 0.f;
                }
            }
        } else
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
        // beta / step and the weight table come precomputed (k_f5_tables): plain copies
        // beta_0 and beta_1; slice t+1 (t >= 1) is copied during iteration t's check phase
        for (int f = tid; f < min(a.T, 2) * a.N; f += NT) BETA[f] = a.betas[f];
        if (tid < 8) RED[tid] = (tid == 1) ? ~0ull : 0ull;
        if constexpr (LUT) {       // iteration 0's slice; slice t+1 is copied during VN t
            const int nw32 = a.qslice >> 1;
            for (int f = tid; f < nw32; f += NT)
                reinterpret_cast<uint32_t*>(QT)[f] = reinterpret_cast<const uint32_t*>(a.qtab)[f];
        }
        __syncthreads();
        for (int e = tid; e < total; e += NT) CH[e] = scr[(e & (CW - 1)) * rl + (e >> LOGCW)] * inv;
        __syncthreads();
        for (int e = tid; e < total; e += NT) {
            const uint32_t v = (uint32_t)e >> LOGCW;
            const int t0 = q_scaled5(CH[e] * BETA[__umulhi(v, a.zmagic)], (float)qmax);  // lw_0
            W[e] = ((uint32_t)(t0 + F5_TVB) << 16) | ((uint32_t)(UCN && t0 >= 0) << 31) | F5_SBIAS;   // hd_{-1}
        }
        if (tid < F5_NDUMMY) W[total + tid] = F5_DUMMY_W;
    }

    F5_STAMP(1);
    // ---- per-group edge addresses (bytes, 16-bit packed) and row info ----------------------
    // (built once per decode by k_f5_gad; one coalesced load per packed word)
    uint32_t gad[MAXG][NPK];
    uint32_t grow[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) {
        grow[gi] = 0;
#pragma unroll
        for (int p = 0; p < NPK; ++p) gad[gi][p] = 0;
        const int grp = wave + gi * NWV;
        if (grp < a.ngroups) {
            const uint32_t* gt = a.gad + (size_t)grp * NPK * 64 + lane;
#pragma unroll
            for (int p = 0; p < NPK; ++p)
                if (p < GD::npk(gi)) gad[gi][p] = gt[p * 64];
            grow[gi] = __builtin_amdgcn_readfirstlane(a.grow[grp].x);   // wave-uniform: an SGPR
        }
    }
    __syncthreads();

    F5_STAMP(2);
    // v_sad_u16's second operand (VOP3 takes no literal; one opaque VGPR, not rematerialised)
    uint32_t ksad;
    asm volatile("v_mov_b32 %0, 0x8000" : "=v"(ksad));
    // check state: P (messages / raw minima), SEL (per-edge fields), ucn (syndrome, PEW only)
    uint32_t P[MAXG], SEL[MAXG][NSEL];
    int UC[MAXG];
#pragma unroll
    for (int gi = 0; gi < MAXG; ++gi) {
        P[gi] = 0;
        UC[gi] = 0;
#pragma unroll
        for (int w = 0; w < NSEL; ++w)
            if (w < GD::nsel(gi)) SEL[gi][w] = 0;
    }

    // C->V message of edge k, given R = v_perm(P, P, SEL[k/4]) (the word's four messages)
    auto msg = [&](const int gi, const int k, const uint32_t R, const float* wt, const float* wtu,
                   const int r0) __attribute__((always_inline)) -> int {
        if constexpr (!PEW) {
            return (int)(signed char)(R >> (8 * SL::pos(k)));
        } else {
            const int m = (int)((R >> (8 * SL::pos(k))) & 0xFFu);        // 255: no other edge
            const float w = (UCN && UC[gi]) ? wtu[r0 + k] : wt[r0 + k];
            const int mq = q_mag5(m == 255 ? F5_BIG_U : m, w, step, inv, qmax);
            return ((SEL[gi][k / 4] >> (8 * SL::pos(k))) & 1u) ? -mq : mq;
        }
    };
    auto perm_word = [&](const int gi, const int w) __attribute__((always_inline)) -> uint32_t {
        return (w < GD::nsel(gi)) ? __builtin_amdgcn_perm(P[gi], P[gi], SEL[gi][w < NSEL ? w : 0]) : 0u;
    };

    for (int t = 0; t < a.T; ++t) {
        if (t < 22) F5_STAMP(8 + t);
        if (tid == 0 && t > 0) {        // fold iteration t-1's frame flags (its VN phase is done)
            if (a.iter_wrong) put_iter_wrong(a.iter_wrong, a.B, t - 1, b0, CW, RED[0] & valid_cw);
            RED[1] &= RED[0];
            RED[0] = 0;
        }
        const float* at = alpha + (size_t)t * a.E;
        const float* au = UCN ? alpha_ucn + (size_t)t * a.E : nullptr;
        // the next iteration's weight-table slice, loaded now, stored to LDS in the VN phase
        // (double buffer: slice t+1 goes where slice t-1 was, which pass 1 of t no longer reads)
        uint32_t qnext = 0;
        if constexpr (LUT) {
            if (t + 1 < a.T && tid < (a.qslice >> 1))
                qnext = reinterpret_cast<const uint32_t*>(a.qtab + (size_t)(t + 1) * a.qslice)[tid];
        }
        // beta_{t+1} for this iteration's VN phase, stored to LDS before the pass-2 barrier
        // (its slot last held beta_{t-1}, read by the VN phase of iteration t-2)
        const bool bcopy = t >= 1 && t + 1 < a.T && tid < a.N;
        float bload = 0.f;
        if (bcopy) bload = a.betas[(size_t)(t + 1) * a.N + tid];
        const float* atp = alpha + (size_t)(t > 0 ? t - 1 : 0) * a.E;
        const float* aup = UCN ? alpha_ucn + (size_t)(t > 0 ? t - 1 : 0) * a.E : nullptr;
        // ======== check nodes: pass 2 (scatter C->V into S), one group ======================
        auto pass2g = [&](const int gi) __attribute__((always_inline)) {
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) return;
            if (a.ablate & 2) return;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(grow[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)((ri >> 16) & 0xFFu);
            // whole 8-edge chunks, padding slots adding into the lane's dummy word (exact 6- and
            // 7-edge chunks measured 2.5% slower on wman (CW 16) and 4% slower on 5G BG2 (CW 8));
            // CW 4 (5G BG1, degrees 3..19, a third of the slots would be padding): exact chunks
            auto chunk2 = [&](const int c8, auto ne) __attribute__((always_inline)) {
                constexpr int NE = decltype(ne)::value;
                const uint32_t R0 = perm_word(gi, c8 / 4);
                const uint32_t R1 = (NE > 4) ? perm_word(gi, c8 / 4 + 1) : 0u;
#pragma unroll
                for (int j = 0; j < NE; ++j) {
                    const int k = c8 + j;
                    if (k < GD::deg(gi)) {
                        const uint32_t pk = gad[gi][k >> 1];
                        const uint32_t addr = (k & 1) ? hi16(pk) : lo16(pk);
                        const int c = msg(gi, k, j < 4 ? R0 : R1, at, au, r0);
                        __atomic_fetch_add(reinterpret_cast<LdsU32*>(addr), (uint32_t)c, __ATOMIC_RELAXED);
                    }
                }
            };
            using N8 = std::integral_constant<int, 8>;
#pragma unroll
            for (int c8 = 0; c8 < GD::deg(gi); c8 += 8) {
                const int n = deg - c8;
                if (CW > 4 || n >= 8) { if (n > 0) chunk2(c8, N8{}); }
                else if (n == 7) chunk2(c8, std::integral_constant<int, 7>{});
                else if (n == 6) chunk2(c8, std::integral_constant<int, 6>{});
                else if (n == 5) chunk2(c8, std::integral_constant<int, 5>{});
                else if (n == 4) chunk2(c8, std::integral_constant<int, 4>{});
                else if (n == 3) chunk2(c8, std::integral_constant<int, 3>{});
                else if (n == 2) chunk2(c8, std::integral_constant<int, 2>{});
                else if (n == 1) chunk2(c8, std::integral_constant<int, 1>{});
            }
        };
        // ======== check nodes: pass 1 (read Tv, fold minima and signs) + new state ==========
#pragma unroll
        for (int gi = 0; gi < MAXG; ++gi) {
            const int grp = wave + gi * NWV;
            if (grp >= a.ngroups) break;
            if (a.ablate & 1) continue;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(grow[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)((ri >> 16) & 0xFFu);
            uint32_t c1 = 0xFFFFFFFFu, c2 = 0xFFFFFFFFu;
            uint32_t NG[NSEL];
#pragma unroll
            for (int w = 0; w < NSEL; ++w) NG[w] = 0;
            uint32_t syn = 0;     // UCN: XOR of the edges' W words (bit 31: previous hard decisions)
            // this row's weights as scalar loads issued ahead of the chunks (a per-lane choice
            // between two global addresses would be a vector load waited on in the state update)
            float wa = 0.f, wu = 0.f;
            if constexpr (!PEW && !LUT) {
                wa = at[r0];
                if constexpr (UCN) wu = au[r0];
            }
            // one chunk of up to 8 edges, straight-line.  NE = edges present (compile time):
            // 6 and 7 cover rows ending inside the chunk; other short chunks run as 8 and their
            // padding slots (k >= deg) read the dummy word (|v2c| never below qmax, positive
            // sign).  Skipping slots behind scalar branches was measured slower: the branches
            // split the chunk's schedule.
            auto chunk1 = [&](const int c8, auto ne) __attribute__((always_inline)) {
                constexpr int NE = decltype(ne)::value;
                uint32_t wv[8];
#pragma unroll
                for (int j = 0; j < NE; ++j) {
                    const int k = c8 + j;
                    if (k < GD::deg(gi)) {
                        const uint32_t pk = gad[gi][k >> 1];
                        const uint32_t addr = (k & 1) ? hi16(pk) : lo16(pk);
                        wv[j] = *reinterpret_cast<const LdsU32*>(addr);
                    }
                }
                const uint32_t R0 = perm_word(gi, c8 / 4);
                const uint32_t R1 = (NE > 4) ? perm_word(gi, c8 / 4 + 1) : 0u;
                // V->C before Q, times 256: d256 = (Tv - m) << 8, sign-extended.  All of them
                // first: an SDWA result with a sub-dword dst_sel read by the very next
                // instruction costs a wait state.
                uint32_t dd[8];
#pragma unroll
                for (int j = 0; j < NE; ++j) {
                    const int k = c8 + j;
                    if (k < GD::deg(gi)) {
                        if constexpr (PEW) {
                            const int cold = msg(gi, k, j < 4 ? R0 : R1, atp, aup, r0);
                            dd[j] = sub_d256<0>(wv[j], (uint32_t)cold);
                        } else {
                            const uint32_t R = j < 4 ? R0 : R1;
                            switch (SL::pos(k)) {
                                case 0: dd[j] = sub_d256<0>(wv[j], R); break;
                                case 1: dd[j] = sub_d256<1>(wv[j], R); break;
                                case 2: dd[j] = sub_d256<2>(wv[j], R); break;
                                default: dd[j] = sub_d256<3>(wv[j], R); break;
                            }
                        }
                        if (UCN) syn ^= wv[j];
                    }
                }
#pragma unroll
                for (int j = 0; j < NE; ++j) {
                    const int k = c8 + j;
                    if (k < GD::deg(gi)) {
                        const uint32_t d256 = dd[j];
                        // key = |d| << 8 | code, all in the low 16 bits
                        const uint32_t key = key_sad(d256, ksad, SL::code(k));
                        // append the offset-binary V->C byte (bit 7: d >= 0) to the selector word
                        NG[k / 4] = append_b1(NG[k / 4], d256);
                        const uint32_t o1 = c1;
                        c1 = min_u16(o1, key);
                        c2 = med3u(o1, c2, key);
                    }
                }
                // absent slots of the chunk enter as zero bytes (not counted as positive)
#pragma unroll
                for (int w = 0; w < NSEL; ++w) {
                    int n = 0;
#pragma unroll
                    for (int j = NE; j < 8; ++j) n += (c8 + j < MAXDEG && (c8 + j) / 4 == w);
                    if (n > 0) NG[w] = (n >= 4) ? 0u : (NG[w] << (8 * n));
                }
            };
#pragma unroll
            for (int c8 = 0; c8 < GD::deg(gi); c8 += 8) {
                const int n = deg - c8;
                // a row ending inside the chunk runs the shape with exactly its edges (shapes
                // below 6 only where a shape's rows are that short: 5G-like graphs)
                if (n >= 8) chunk1(c8, std::integral_constant<int, 8>{});
                else if (n == 7) chunk1(c8, std::integral_constant<int, 7>{});
                else if (n == 6) chunk1(c8, std::integral_constant<int, 6>{});
                else if (CW <= 8 && n == 5) chunk1(c8, std::integral_constant<int, 5>{});
                else if (CW <= 8 && n == 4) chunk1(c8, std::integral_constant<int, 4>{});
                else if (CW <= 8 && n == 3) chunk1(c8, std::integral_constant<int, 3>{});
                else if (CW <= 8 && n == 2) chunk1(c8, std::integral_constant<int, 2>{});
                else if (CW <= 8 && n == 1) chunk1(c8, std::integral_constant<int, 1>{});
                else if (n > 0) chunk1(c8, std::integral_constant<int, 8>{});
                else {
                    // chunk skipped (deg <= c8): its edges enter as zero bytes
#pragma unroll
                    for (int w = 0; w < NSEL; ++w) {
                        const int nn = SL::in_chunk(w, c8);
                        if (nn > 0) NG[w] = (nn >= 4) ? 0u : (NG[w] << (8 * nn));
                    }
                }
            }
            // ---- new state: quantized minima, selector bytes, argmin bit ----
            uint32_t px = 0;                           // parity of the V->C >= 0 flags
#pragma unroll
            for (int w = 0; w < NSEL; ++w) {
                NG[w] = (NG[w] >> 7) & SL::bmask(w);   // bit 0 of each byte: V->C >= 0
                px ^= NG[w];
            }
            // message sign = V->C sign XOR (count of positives odd): applied to P as a byte
            // swap inside each half; for PEW (P holds magnitudes) to the selector bytes, whose
            // bit 0 then means "negative message" (V->C >= 0 XOR count even)
            if constexpr (UCN) syn = syn >> 31;
            const bool podd = (uint32_t)__popc(px) & 1u;
            // argmin bit: the edge code is 8 * b + 1 for selector byte b (word b / 4), so one
            // 64-bit shift places it inside the word pair b / 8
            const uint32_t code = c1 & 255u;
            const uint64_t onepair = 1ull << (code & 63u);
            const uint32_t pairsel = code >> 6;
            const uint32_t pm = (PEW && !podd) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int w = 0; w < NSEL; ++w)
                if (w < GD::nsel(gi)) {
                    const uint32_t ob = (w & 1) ? (uint32_t)(onepair >> 32) : (uint32_t)onepair;
                    SEL[gi][w] = (NG[w] ^ (pm & SL::bmask(w))) | ((pairsel == (uint32_t)(w >> 1)) ? ob : 0u);
                }
            const int m1 = min((int)(c1 >> 8), qmax);
            if constexpr (PEW) {
                const uint32_t m2 = (deg < 2) ? 255u : (uint32_t)min((int)(c2 >> 8), qmax);
                UC[gi] = (int)syn;
                P[gi] = (uint32_t)m1 * 0x0101u | (m2 * 0x0101u) << 16;
            } else {
                uint32_t p;
                if constexpr (LUT) {
                    // [+m, -m] byte pairs of Q(relu(m*w)) for this iteration and proto row,
                    // indexed by the unclamped |V->C| (the table repeats Q(qmax) up to 3 qmax,
                    // |Tv - m|'s bound); entry nq - 1 stands for "no other edge"
                    const int row = (int)((ri >> 24) & 0xFFu);
                    const unsigned char* qt = reinterpret_cast<const unsigned char*>(
                        QT + (t & 1) * a.qslice + ((UCN && syn) ? a.qucn : 0) + row * a.qrow);
                    // byte offsets 2 |d| = key >> 7 (the code byte stays below 128 up to 16 edges)
                    const uint32_t o1 = (MAXDEG <= 16) ? (c1 >> 7) : ((c1 >> 7) & ~1u);
                    const uint32_t o2 = (deg < 2) ? 2u * (uint32_t)(a.qrow - 1)
                                                  : ((MAXDEG <= 16) ? (c2 >> 7) : ((c2 >> 7) & 0x1FEu));
                    const uint32_t qa = *reinterpret_cast<const uint16_t*>(qt + o1);
                    const uint32_t qb = *reinterpret_cast<const uint16_t*>(qt + o2);
                    // [-mA, +mA, -mB, +mB] (index 2 is_argmin + (V->C >= 0)), halves swapped
                    // when the count of positives is odd
                    p = __builtin_amdgcn_perm(qb, qa, podd ? 0x05040100u : 0x04050001u);
                } else {
                    const int m2 = (deg < 2) ? F5_BIG_U : min((int)(c2 >> 8), qmax);
                    const float w = (UCN && syn) ? wu : wa;
                    const int mA = q_mag5(m1, w, step, inv, qmax);
                    const int mB = q_mag5(m2, w, step, inv, qmax);
                    const uint32_t pa = ((uint32_t)mA & 0xFFu) | (((uint32_t)(-mA) & 0xFFu) << 8);
                    const uint32_t pb = ((uint32_t)mB & 0xFFu) | (((uint32_t)(-mB) & 0xFFu) << 8);
                    p = pa | (pb << 16);
                    p = __builtin_amdgcn_perm(p, p, podd ? 0x03020100u : 0x02030001u);
                }
                // (a lane past its run's last check has every edge on its own dummy word, so
                // its messages land there: no validity mask needed)
                P[gi] = p;
            }
            if constexpr (F5_P2_MODE == 1) pass2g(gi);     // this group's scatter right away
        }
        if (t == 0) F5_STAMP(5);
        if constexpr (F5_P2_MODE == 0) {
#pragma unroll
            for (int gi = 0; gi < MAXG; ++gi) pass2g(gi);
        }
        if (bcopy) BETA[((t + 1) & 1) * a.N + tid] = bload;
        __syncthreads();
        if (t == 0) F5_STAMP(6);
        // ======== variable nodes ===========================================================
        const bool last = (t == a.T - 1);
        if constexpr (LUT) {
            if (!last && tid < (a.qslice >> 1))
                reinterpret_cast<uint32_t*>(QT + ((t + 1) & 1) * a.qslice)[tid] = qnext;
        }
        const float* bnext = BETA + (size_t)((t + 1) & 1) * a.N;     // unused when last
        uint32_t any_hd = 0, any_pos = 0, nbits = 0;
        const float qmf = (float)qmax;
        const int sb = -(int)F5_SBIAS;
        if (tid < F5_NDUMMY) W[total + tid] = F5_DUMMY_W;    // pass-2 adds of padding edges
        if constexpr (!OUT) {
            // counters only.  A wave owns the contiguous 64-entry chunks [c_beg, c_end); with
            // SLOTS | z a chunk lies in one proto column, so beta is wave-uniform.  Only the
            // hard-decision sign matters here, and clipping never changes a sign.
            int amax = INT_MIN;                       // max APP over the target entries (last)
            uint32_t aor = 0;                         // OR of F5_APPH-biased APPs (bit 23)
            const int c_beg = wave * a.cpw;
            const int c_end = min(c_beg + a.cpw, a.nfull);
            const bool zuni = (z % SLOTS) == 0;
            const uint32_t cvalid = (cw < nvalid) ? 1u : 0u;
            const int tb = a.target_bits;
            // Tv clamp bounds as the low 16 bits of Tv + F5_APP0 (= 16384 + Tv)
            const uint32_t tlo = (uint32_t)(F5_APP0 - 2 * qmax) & 0xFFFFu;
            const uint32_t thi = (uint32_t)(F5_APP0 + 2 * qmax) & 0xFFFFu;
            // one loop body per (last iteration, whole word is target) pair; 4 chunks per trip
            // with the reads issued first.  Reads past c_end stay inside LDS and are unused.
            auto vn_loop = [&](auto lastc, auto fullc, auto zunic) __attribute__((always_inline)) {
                constexpr bool LAST = decltype(lastc)::value;
                constexpr bool FULLT = decltype(fullc)::value;
                constexpr bool ZUNI = decltype(zunic)::value;
                const int vl = (int)lane_fresh();
                const uint32_t* Wr = W + c_beg * 64 + vl;
                const float* Cr = CH + c_beg * 64 + vl;
                for (int c = c_beg; c < c_end; c += 4, Wr += 256, Cr += 256) {
                    uint32_t wv[4];
                    float chv[4], bv[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        wv[j] = Wr[j * 64];
                        chv[j] = Cr[j * 64];
                        if (!LAST) {
                            if (ZUNI) {
                                const uint32_t col = __umulhi((uint32_t)((c + j) * SLOTS), a.zmagic);
                                bv[j] = bnext[__builtin_amdgcn_readfirstlane(col)];
                            } else {
                                const uint32_t v = (uint32_t)((c + j) * 64 + vl) >> LOGCW;
                                bv[j] = bnext[__umulhi(v, a.zmagic)];
                            }
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (j == 0 || c + j < c_end) {
                            // Q(y) for y already scaled to grid units: clamp to +-qmax, then
                            // add 1.5*2^23 so the float add rounds half to even (as rintf) and
                            // the integer sits in the low mantissa bits: bits - F5_MAGIC_BITS
                            if (!LAST) {
                                // W's low half is exactly S + bias (the hd bit is bit 31) and only
                                // low halves matter: add the whole word, no mask.
                                // Low 16 bits of qh + W = APP + 0x8000: bit 15 = [APP >= 0]
                                const uint32_t wraw = wv[j];
                                const float yc = __builtin_amdgcn_fmed3f(chv[j], -qmf, qmf);
                                const uint32_t apph = (uint32_t)__float_as_int(yc + F5_MAGIC_H) + wraw;
                                if (FULLT) {
                                    aor |= apph;
                                } else {
                                    const int v = ((c + j) * 64 + vl) >> LOGCW;
                                    aor |= (v < tb) ? apph : 0u;
                                }
                                const float yb = __builtin_amdgcn_fmed3f(chv[j] * bv[j], -qmf, qmf);
                                const uint32_t tb2 = clamp_i16((uint32_t)__float_as_int(yb + F5_MAGIC) + wraw,
                                                               tlo, thi);
                                uint32_t wn = tb2 * 65536u + F5_WBIAS;
                                if (UCN) wn |= (apph << 16) & 0x80000000u;       // hd for the syndrome
                                const_cast<uint32_t*>(Wr)[j * 64] = wn;
                                continue;
                            }
                            // last iteration: counters only (no W update)
                            const int s = (int)(wv[j] & 0x7FFFu);                     // S + bias
                            const float yc = __builtin_amdgcn_fmed3f(chv[j], -qmf, qmf);
                            const int qc = __float_as_int(yc + F5_MAGIC_A);
                            // APP + F5_APPH: bit 23 set iff APP >= 0
                            const int appb = qc + s;
                            int appt = appb;
                            if (!FULLT) {
                                const int v = ((c + j) * 64 + vl) >> LOGCW;
                                appt = (v < tb) ? appb : INT_MIN;
                            }
                            amax = max(amax, appt);
                            nbits += (uint32_t)(appt >= F5_APPH) & cvalid;
                        }
                    }
                }
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            if (!(a.ablate & 4)) {
                const bool fullt = tb >= nv;
                if (last) {                       // no W update: beta unused
                    if (fullt) vn_loop(T_{}, T_{}, T_{}); else vn_loop(T_{}, F_{}, T_{});
                } else if (zuni) {
                    if (fullt) vn_loop(F_{}, T_{}, T_{}); else vn_loop(F_{}, F_{}, T_{});
                } else {
                    if (fullt) vn_loop(F_{}, T_{}, F_{}); else vn_loop(F_{}, F_{}, F_{});
                }
            }
            // the partial last chunk (n_vars*CW not a multiple of 64), per-lane checks
            if (a.nfull * 64 < total && wave == (a.nfull / max(a.cpw, 1)) % NWV && !(a.ablate & 4)) {
                const int e = a.nfull * 64 + (int)lane_fresh();
                if (e < total) {
                    const uint32_t v = (uint32_t)e >> LOGCW;
                    const int s = (int)(W[e] & 0x7FFFu);
                    const float ch = CH[e];
                    const int app = q_scaled5(ch, qmf) + s + sb;
                    const int appt = ((int)v < a.target_bits) ? app : INT_MIN;
                    amax = max(amax, appt == INT_MIN ? INT_MIN : appt + F5_APPH);
                    aor |= (appt != INT_MIN && appt >= 0) ? 0x8000u : 0u;
                    if (!last) {
                        const int tn = min(max(q_scaled5(ch * bnext[__umulhi(v, a.zmagic)], qmf) + s + sb,
                                               -2 * qmax), 2 * qmax);
                        W[e] = ((uint32_t)(tn + F5_TVB) << 16) | ((uint32_t)~app & 0x80000000u) | F5_SBIAS;
                    } else {
                        nbits += (uint32_t)(appt >= 0 && appt != INT_MIN) & (uint32_t)cvalid;
                    }
                }
            }
            any_hd = last ? (amax >= F5_APPH) : ((aor >> 15) & 1u);     // bit 15: some APP >= 0
            any_pos = amax > F5_APPH;
        } else {
        for (int r = 0; r < ((a.ablate & 4) ? 0 : a.nent); ++r) {
            const int e = tid + r * NT;
            if (e < total) {
                const uint32_t v = (uint32_t)e >> LOGCW;
                const uint32_t wv = W[e];
                const int S = (int)(wv & 0x7FFFu) + sb;
                const float ch = CH[e];
                int app = q_scaled5(ch, (float)qmax) + S;                // Q(xa) + sum C2V
                app = min(max(app, -a.clip_u), a.clip_u);                // clip +-clip_LLR
                if (!last) {
                    const int tn = min(max(q_scaled5(ch * bnext[__umulhi(v, a.zmagic)], (float)qmax) + S,
                                           -2 * qmax), 2 * qmax);
                    W[e] = ((uint32_t)(tn + F5_TVB) << 16) | ((uint32_t)(app >= 0) << 31) | F5_SBIAS;
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
        if (last) nbits = (cw < nvalid) ? nbits : 0u;
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
            uint32_t nb = nbits;
            for (int off = 32; off > 0; off >>= 1) nb += __shfl_xor(nb, off);
            if (lane == 0 && nb) atomicAdd(&RED[3], (unsigned long long)nb);
        }
        __syncthreads();
    }
    F5_STAMP(30);
    if (a.stamps && tid == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.stamps[(size_t)bx * 32 + 31] = ((unsigned long long)xcc << 32) | hw;
    }
    if (tid == 0) {
        const unsigned long long wl = RED[0] & valid_cw;
        const unsigned long long all = RED[1] & RED[0] & valid_cw;
        const unsigned long long ap = RED[2] & valid_cw;
        if (a.iter_wrong) put_iter_wrong(a.iter_wrong, a.B, a.T - 1, b0, CW, wl);
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

template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE, bool UCN, bool PEW, bool OUT, bool LUT>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE)))
k_fused5(F5Args a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn) {
    f5_block<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>(a, alpha, alpha_ucn, (int64_t)blockIdx.x);
}

// The bit-sliced kernels' fixup (a.only set): a grid of at most a few workgroups per CU walks the
// blocks and decodes those of flagged packs.  One workgroup per block (k_fused5 with a.only)
// launched the full 2^20 / CW grid, whose workgroups almost all exit at once: 59 us per C2
// decode (1 % of it) for the dispatch alone.
template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE, bool UCN, bool PEW, bool OUT, bool LUT>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE)))
k_fused5_fix(F5Args a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn, int64_t nblk) {
    // the flags of 64 of the workgroup's blocks per round, one per lane, loaded at once (every
    // wave takes the same ballot, so the list is uniform without LDS); walking the blocks one
    // flag load at a time cost 66 us per C2 decode in load latency alone
    const int lane = threadIdx.x & 63;
    for (int64_t base = blockIdx.x; base < nblk; base += 64 * (int64_t)gridDim.x) {
        const int64_t cand = base + (int64_t)lane * gridDim.x;
        const bool flagged = cand < nblk && a.only[(cand * CW) >> 5] != 0u;
        unsigned long long m = __ballot(flagged);
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            f5_block<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>(a, alpha, alpha_ucn,
                                                                        base + (int64_t)l * gridDim.x);
            __syncthreads();
        }
    }
}

// ---- shapes ------------------------------------------------------------------------------
struct Shape5 {
    int cw, maxg, maxdeg;
    int wpe;       // occupancy target, waves per SIMD (1: no VGPR cap).  VALU issue saturates near 6
    bool autosel;  // considered by plan5 (else only via LDPC_F5_SHAPE=<index>)
    bool bal;      // deal groups to waves by row degree (k_f5_gad); LDPC_F5_BALANCE=0/1 overrides
    int hg = 0, ldeg = 0;   // hg < maxg: slots gi >= hg take rows of degree <= ldeg (GDeg; the
                            // degree-ranked dealing puts the heaviest groups in slots gi < hg)
};
constexpr Shape5 kShapes5[] = {
    {16, 3, 16, 6, true, false},    // wman-like (z=24, deg 14-15)
    {16, 3, 24, 1, true, false},    // 802.11n-like (deg 22)
    {8, 5, 16, 1, true, false},     // 5G BG2-like (z=64, deg <= 10)
    {64, 3, 8, 1, true, false},     // z=1 sparse (MacKay)
    {64, 2, 32, 1, true, false},    // z=1 dense rows (BCH)
    {4, 3, 12, 7, true, false},     // 5G BG2-like at two workgroups per CU (z=64: 16 slots, 4 codewords)
    {8, 2, 22, 6, true, false},     // 802.11n-like (deg <= 22: no all-padding address word) at three WGs per CU
    {4, 4, 20, 4, true, false},     // 5G BG1-like (n = 2304 variables, deg 3-19, z = 72), one WG per CU
    {4, 7, 20, 4, true, true, 3, 10},   // 5G BG1-like, 3 heavy + 4 light slots, 8 waves: two WGs per CU
    {4, 5, 10, 6, true, true, 2, 6},    // 5G BG2-like (deg 8-10 / 4-6), 8 waves: three WGs per CU
    // measured and dropped: {8, 2, 16} at 8 waves/SIMD (64 VGPRs) ran 28.3 ms vs 21.3 ms for
    // {16, 3, 16} on wman -- twice the per-workgroup fixed cost per codeword; {4, 5, 20, 2/10} at
    // 10 waves and 80 VGPRs spilled ~50 registers; {8, 3, 16} (wman, 6 waves, four WGs per CU)
    // 23.1 ms vs 18.7 ms; {4, 2, 24} (802.11n, 4 waves, seven WGs per CU) within 0.3% of {8, 2, 24}
};

constexpr int F5_FIX_GRID = 512;      // fixup grid (k_fused5_fix): two workgroups per CU

template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE, bool UCN, bool PEW, bool OUT, bool LUT>
int launch5o(const F5Args& a, int nblocks, int nw, size_t lds, const float* alpha,
             const float* alpha_ucn, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused5<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)F5_LDS_MAX);
        attr = true;
    }
    if constexpr (!PEW) {               // (the bit-sliced kernels serve row-uniform weights only;
                                        // OUT: their hard-decision export build)
        if (a.only) {
            static bool attr_fix = false;
            if (!attr_fix) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused5_fix<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)F5_LDS_MAX);
                attr_fix = true;
            }
            const int grid = nblocks < F5_FIX_GRID ? nblocks : F5_FIX_GRID;
            hipLaunchKernelGGL((k_fused5_fix<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>), dim3(grid), dim3(64 * nw), lds, s,
                               a, alpha, alpha_ucn, (int64_t)nblocks);
            return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
        }
    }
    hipLaunchKernelGGL((k_fused5<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, OUT, LUT>), dim3(nblocks), dim3(64 * nw), lds, s,
                       a, alpha, alpha_ucn);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

// the weight table is used when every row shares one weight and there is no UCN weight set
template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE, bool UCN, bool PEW>
int launch5k(const F5Args& a, int nblocks, int nw, size_t lds, bool lut, const float* alpha,
             const float* alpha_ucn, hipStream_t s) {
    constexpr bool CANLUT = !PEW;
    const bool out = a.app_out || a.hd_out;
    if (CANLUT && lut)
        return out ? launch5o<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, true, CANLUT>(a, nblocks, nw, lds, alpha, alpha_ucn, s)
                   : launch5o<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, false, CANLUT>(a, nblocks, nw, lds, alpha, alpha_ucn, s);
    return out ? launch5o<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, true, false>(a, nblocks, nw, lds, alpha, alpha_ucn, s)
               : launch5o<CW, MAXG, MAXDEG, HG, LDEG, WPE, UCN, PEW, false, false>(a, nblocks, nw, lds, alpha, alpha_ucn, s);
}

template <int CW, int MAXG, int MAXDEG, int HG, int LDEG, int WPE>
int launch5s(const F5Args& a, int nblocks, int nw, size_t lds, bool lut, const float* alpha,
             const float* alpha_ucn, bool pew, hipStream_t s) {
    if (alpha_ucn)
        return pew ? launch5k<CW, MAXG, MAXDEG, HG, LDEG, WPE, true, true>(a, nblocks, nw, lds, lut, alpha, alpha_ucn, s)
                   : launch5k<CW, MAXG, MAXDEG, HG, LDEG, WPE, true, false>(a, nblocks, nw, lds, lut, alpha, alpha_ucn, s);
    return pew ? launch5k<CW, MAXG, MAXDEG, HG, LDEG, WPE, false, true>(a, nblocks, nw, lds, lut, alpha, nullptr, s)
               : launch5k<CW, MAXG, MAXDEG, HG, LDEG, WPE, false, false>(a, nblocks, nw, lds, lut, alpha, nullptr, s);
}

// the launcher of shape S (kShapes5[S]); defined in the translation unit built from
// ldpc_fused5_shape.hip with -DF5_SHAPE=S
template <int S>
int f5_launch(const F5Args& a, int nblocks, int nw, size_t lds, bool lut, const float* alpha,
              const float* alpha_ucn, bool pew, hipStream_t s);

}  // namespace f5
}  // namespace ldpc
