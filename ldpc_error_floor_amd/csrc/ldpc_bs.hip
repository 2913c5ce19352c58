// ldpc_bs.hip — bit-sliced fused QMS decoder ("bs"): 32 codewords per 32-bit word.
//
// Same semantics as the v5 kernel (ldpc_fused5_kernel.h) and the reference graph
// (Main_Functions.py:157-335): all T flooding iterations of a block in one launch, integer
// arithmetic in units of the q-bit grid (q = 5 / -5: qmax = 15).  What changes is the data
// layout: a workgroup decodes one PACK of 32 codewords and every quantity is held as bit
// planes (plane word p of a value holds bit p of that value for the 32 codewords, bit r =
// codeword b0 + r).  The min-sum arithmetic — V->C subtraction, |.| with saturation, the
// two-minimum search, the sign parity, the weighted quantization (a 16-entry table per
// iteration, evaluated as a mux tree) and the variable-node sums — is boolean algebra on whole
// words, which gfx950 issues as v_bitop3_b32 (any function of three words in one VALU op).
// One lane does the work of 32 codeword-lanes of v5.
//
// LDS holds one 5-word SLOT per lifted edge (slot s = proto edge * z + check index within the
// row, so lanes on consecutive checks or variables touch consecutive slots):
//   between the variable and the check phase: V->C = clamp(Tv - C->V, +-15), as a negative flag
//     and 4 magnitude planes (the nudged zero is positive, Main_Functions.py:229-230);
//   between the check and the variable phase: C->V, as a negative flag and 4 magnitude planes.
// Each slot is read and then rewritten by exactly one lane per phase, so the two share it.
// Check phase: one lane per check (up to D edges, padding edges read the all-ones PAD slot:
// negative, magnitude 15, so they change neither minimum nor parity).  Variable phase: one lane
// per variable (variables ordered by degree so a wave's loop bound is tight; padding edges read
// the all-zero ZERO slot); the channel stays in the lane's registers for the whole decode.
// Packs with an LLR off the quantizer grid are flagged in `bad` and decoded by the v5 kernel
// instead, so the result is exact for any input.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldpc_fused.h"
#include "ldpc_fused5_kernel.h"

namespace ldpc {
namespace bs {

constexpr int PACK = 32;                 // codewords per workgroup
constexpr int SLOT_W = 5;                // words per edge slot: negative flag, magnitude 0..3
constexpr int SLOT_B = SLOT_W * 4;
constexpr int LUT_W = 64;                // words per 16-entry table: [bit j][pair p] {X, Y}
constexpr int QMAX = 15;
constexpr size_t BS_LDS_MAX = 160 * 1024;

struct BsArgs {
    const float* llr;
    int64_t B;
    int n_vars, n_checks, T, target_bits, cn_lanes, cn_dmin;
    float inv;
    const int32_t* row_ptr;      // [M + 1] proto edges of each row (the check degrees)
    const int32_t* row_lay;      // [M][2] slot layout of each proto row: first slot, j-block stride
    int z;
    const uint32_t* vn_tab;      // [64 nw][VNW]: slot byte addresses (2 per word), variable (-1 idle)
    const int32_t* vn_wdeg;      // [nw][2] most and fewest edges of a variable of each wave
    const uint32_t* alut;        // [T][arows][LUT_W]: Q(relu(alpha m step)) for m = 0..15
    const uint32_t* blut;        // [T][bcols][LUT_W]: |Q(beta m)| for m = 0..15 (grid units)
    int arows, bcols;
    int64_t* counters;
    uint8_t* flags;
    uint32_t* bad;               // [packs] 1: decoded by the v5 fixup instead
    uint32_t off_pad, off_zero, off_red, off_alut, off_blut;   // LDS byte offsets
    int ablate;   // timing diagnostics, builds with -DBS_DIAG only (LDPC_DIAG_ABLATE, wrong
                  // results): 1 no check phase, 2 no beta table, 4 no V->C pass, 8 no frame
                  // flags, 16 no iterations, 32 no LLR loads.  (Compiled in, the uniform
                  // tests alone cost 4 %.)
};

// ---- bit-plane arithmetic ---------------------------------------------------------------------
// Every 3-input function is one v_bitop3_b32 with an explicit truth table (the compiler's own
// boolean synthesis often emits two or three ops for one such function); 2-input functions are
// left to the compiler, which emits the 2-cycle VOP2 forms (v_and / v_or / v_xor / v_xnor).
// Truth table of f: f(0xF0, 0xCC, 0xAA) for operands (a, b, c).
#define B3(F, a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), (F))
constexpr unsigned TA = 0xF0, TB = 0xCC, TC = 0xAA;
constexpr unsigned T_XOR3 = (TA ^ TB ^ TC) & 0xFF;                       // a ^ b ^ c
constexpr unsigned T_XNOR3 = ~(TA ^ TB ^ TC) & 0xFF;                     // ~(a ^ b ^ c)
constexpr unsigned T_MAJ = ((TA & TB) | (TA & TC) | (TB & TC)) & 0xFF;   // maj(a, b, c)
constexpr unsigned T_MAJNB = ((TA & ~TB) | (TA & TC) | (~TB & TC)) & 0xFF;   // maj(a, ~b, c)
constexpr unsigned T_MUX = ((TA & TB) | (~TA & TC)) & 0xFF;              // a ? b : c
constexpr unsigned T_LT = ((~TA & TB) | (~(TA ^ TB) & TC)) & 0xFF;       // a < b at this bit, else c
constexpr unsigned T_ANDN = (~TA & TB) & 0xFF;                           // ~a & b
constexpr unsigned T_LEAF = ((TA & TB) ^ TC) & 0xFF;                     // (a & b) ^ c
constexpr unsigned T_AND3 = (TA & TB & TC) & 0xFF;                       // a & b & c
constexpr unsigned T_SAT = ((TA & ~TB) | (~TA & TC)) & 0xFF;             // a ? ~b : c
constexpr unsigned T_XAND = (TA ^ (TB & TC)) & 0xFF;                     // a ^ (b & c)
constexpr unsigned T_ANDNA = (TA & ~TB) & 0xFF;                          // a & ~b
constexpr unsigned T_ORXOR = (TA | (TB ^ TC)) & 0xFF;                    // a | (b ^ c)
__device__ __forceinline__ uint32_t mux(uint32_t s, uint32_t a, uint32_t b) { return B3(T_MUX, s, a, b); }

// S += m for m = (negative flag n, b) with b_i = M_i ^ n (M the 4 magnitude planes): the
// two's complement of m is b sign-extended with n, plus n
template <int SB>
__device__ __forceinline__ void add_b(uint32_t (&S)[SB], const uint32_t (&b)[4], uint32_t n) {
    uint32_t c = n;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        const uint32_t bi = (i < 4) ? b[i] : n;
        const uint32_t s = B3(T_XOR3, S[i], bi, c);
        if (i + 1 < SB) c = B3(T_MAJ, S[i], bi, c);
        S[i] = s;
    }
}
// S = m (same operand form), S previously zero
template <int SB>
__device__ __forceinline__ void set_b(uint32_t (&S)[SB], const uint32_t (&b)[4], uint32_t n) {
    uint32_t c = n;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        const uint32_t bi = (i < 4) ? b[i] : n;
        S[i] = bi ^ c;
        c = bi & c;
    }
}

// x = Tv - m (7 planes, two's complement; Tv in [-32, 31], |m| <= 15) with m = (n, b) as above:
// -m is ~b sign-extended with ~n, plus ~n
__device__ __forceinline__ void sub_tv(uint32_t (&x)[7], const uint32_t (&T)[6], const uint32_t (&b)[4],
                                       uint32_t n) {
    uint32_t c = ~n;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const uint32_t t = T[i < 6 ? i : 5];
        const uint32_t bi = (i < 4) ? b[i] : n;
        x[i] = B3(T_XNOR3, t, bi, c);
        if (i < 6) c = B3(T_MAJNB, t, bi, c);
    }
}

// min(|x|, 15) (4 planes) of a 7-plane two's complement x in [-64, 63]; the sign is x[6].
// For x < 0 the low bits of -x are x_i ^ OR(x_j, j < i); |x| >= 16 is x5 | x4 for x >= 0 and
// "not (x5 & x4 & low 4 bits nonzero)" for x < 0.
__device__ __forceinline__ void abs_sat(uint32_t (&X)[4], const uint32_t (&x)[7]) {
    const uint32_t neg = x[6];
    const uint32_t o2 = x[0] | x[1], o3 = o2 | x[2], o4 = o3 | x[3];
    const uint32_t sat = B3(T_SAT, neg, B3(T_AND3, x[5], x[4], o4), x[5] | x[4]);
    X[0] = x[0] | sat;
    X[1] = B3(T_XAND, x[1], neg, x[0]) | sat;
    X[2] = B3(T_XAND, x[2], neg, o2) | sat;
    X[3] = B3(T_XAND, x[3], neg, o3) | sat;
}

// a < b for 4-plane unsigned values
__device__ __forceinline__ uint32_t lt4(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
    uint32_t l = B3(T_ANDN, a[0], b[0], 0u);
#pragma unroll
    for (int i = 1; i < 4; ++i) l = B3(T_LT, a[i], b[i], l);
    return l;
}

// SB-plane two's complement -> 6 planes, saturated to [-32, 31]
template <int SB>
__device__ __forceinline__ void clamp6(uint32_t (&T)[6], const uint32_t (&v)[SB]) {
    uint32_t ovf = 0;
#pragma unroll
    for (int i = 5; i < SB - 1; ++i) ovf |= v[i] ^ v[i + 1];
    const uint32_t s = v[SB - 1];
#pragma unroll
    for (int i = 0; i < 5; ++i) T[i] = B3(T_SAT, ovf, s, v[i]);
    T[5] = mux(ovf, s, v[5]);
}

// LDS accesses by byte address (all slots and tables are LDS-absolute: the kernel's dynamic
// LDS starts at 0, checked at entry)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t LdsW;
typedef __attribute__((address_space(3))) v4u LdsQ;

__device__ __forceinline__ uint32_t lds_w(uint32_t addr) { return *reinterpret_cast<const LdsW*>(addr); }
__device__ __forceinline__ v4u lds_q(uint32_t addr) { return *reinterpret_cast<const LdsQ*>(addr); }

__device__ __forceinline__ void read_slot(uint32_t& n, uint32_t (&M)[4], uint32_t addr) {
    const LdsW* p = reinterpret_cast<const LdsW*>(addr);
    n = p[0];
    M[0] = p[1];
    M[1] = p[2];
    M[2] = p[3];
    M[3] = p[4];
}
__device__ __forceinline__ void write_slot(uint32_t addr, uint32_t n, const uint32_t (&M)[4]) {
    LdsW* p = reinterpret_cast<LdsW*>(addr);
    p[0] = n;
    p[1] = M[0];
    p[2] = M[1];
    p[3] = M[2];
    p[4] = M[3];
}

// 16-entry table g(m) (4 -> 4 bits) at LDS byte address `tab`: level 1 of the mux tree is
// (m0 & X) ^ Y per pair of entries, levels 2-4 select by m1, m2, m3
template <int NI>
__device__ __forceinline__ void lut(uint32_t (&o)[NI][4], const uint32_t (&in)[NI][4], uint32_t tab) {
    uint32_t tj = tab;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // one output bit at a time (the next bit's table loads wait for this bit's result), so
        // that the scheduler cannot hoist all 16 table loads into 64 registers
        if (j > 0) asm volatile("" : "+v"(tj) : "v"(o[0][j - 1]));
        uint32_t g[NI][4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u w = lds_q(tj + (uint32_t)(j * 64 + q * 16));      // pairs 2q, 2q + 1
#pragma unroll
            for (int u = 0; u < NI; ++u) {
                const uint32_t l0 = B3(T_LEAF, in[u][0], w.x, w.y), l1 = B3(T_LEAF, in[u][0], w.z, w.w);
                g[u][q] = mux(in[u][1], l1, l0);
            }
        }
#pragma unroll
        for (int u = 0; u < NI; ++u)
            o[u][j] = mux(in[u][3], mux(in[u][2], g[u][3], g[u][2]), mux(in[u][2], g[u][1], g[u][0]));
    }
}

// the same 16-entry table when it is one table for the whole workgroup (uniform weights): its
// 64 leaf words come by scalar loads (constant address space) into SGPRs, so the evaluation
// costs no LDS traffic; a leaf is a v_and + v_xor with SGPR operands (the 2-cycle VOP2 forms,
// one SGPR per instruction) in place of one v_bitop3 — the same issue cycles
typedef __attribute__((address_space(4))) const uint32_t ConstW;
__device__ __forceinline__ void lut_s(uint32_t (&o)[4], const uint32_t (&a)[4], const ConstW* tab) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t l0 = (a[0] & tab[j * 16 + 4 * q]) ^ tab[j * 16 + 4 * q + 1];
            const uint32_t l1 = (a[0] & tab[j * 16 + 4 * q + 2]) ^ tab[j * 16 + 4 * q + 3];
            g[q] = mux(a[1], l1, l0);
        }
        o[j] = mux(a[3], mux(a[2], g[3], g[2]), mux(a[2], g[1], g[0]));
    }
}

// bit j of the table output for NI inputs (4 b128 loads of the table's bit-j leaves at tab_j)
template <int NI>
__device__ __forceinline__ void lut_bit(uint32_t (&o)[NI], const uint32_t (&in)[NI][4], uint32_t tab_j) {
    uint32_t g[NI][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const v4u w = lds_q(tab_j + (uint32_t)(q * 16));      // pairs 2q, 2q + 1
#pragma unroll
        for (int u = 0; u < NI; ++u) {
            const uint32_t l0 = B3(T_LEAF, in[u][0], w.x, w.y), l1 = B3(T_LEAF, in[u][0], w.z, w.w);
            g[u][q] = mux(in[u][1], l1, l0);
        }
    }
#pragma unroll
    for (int u = 0; u < NI; ++u)
        o[u] = mux(in[u][3], mux(in[u][2], g[u][3], g[u][2]), mux(in[u][2], g[u][1], g[u][0]));
}

// lane permutation inside each group of 4 lanes (DPP quad_perm, a VALU move)
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
constexpr int QP_X1 = 0xB1;          // [1, 0, 3, 2]
constexpr int QP_X2 = 0x4E;          // [2, 3, 0, 1]

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
// OR / sum over the wave (wave-uniform result): butterflies inside each row of 16 lanes by DPP
// (quad_perm, row_half_mirror, row_mirror), then the four row results by readlane
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    x |= dpp<QP_X1>(x);
    x |= dpp<QP_X2>(x);
    x |= dpp<0x141>(x);
    x |= dpp<0x140>(x);
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 15) | __builtin_amdgcn_readlane((int)x, 31) |
                      __builtin_amdgcn_readlane((int)x, 47) | __builtin_amdgcn_readlane((int)x, 63));
}
__device__ __forceinline__ uint32_t wave_add(uint32_t x) {
    x += dpp<QP_X1>(x);
    x += dpp<QP_X2>(x);
    x += dpp<0x141>(x);
    x += dpp<0x140>(x);
    return (uint32_t)(__builtin_amdgcn_readlane((int)x, 15) + __builtin_amdgcn_readlane((int)x, 31) +
                      __builtin_amdgcn_readlane((int)x, 47) + __builtin_amdgcn_readlane((int)x, 63));
}

// two smallest of {m1 <= m2} and {b1 <= b2} into m1 <= m2 (4-plane magnitudes)
__device__ __forceinline__ void merge2(uint32_t (&m1)[4], uint32_t (&m2)[4], const uint32_t (&b1)[4],
                                       const uint32_t (&b2)[4]) {
    const uint32_t l = lt4(b1, m1);
    uint32_t x[4], y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[i] = mux(l, b2[i], m2[i]);      // the winner's second
        y[i] = mux(l, m1[i], b1[i]);      // the loser's first
        m1[i] = mux(l, b1[i], m1[i]);
    }
    const uint32_t l2 = lt4(x, y);
#pragma unroll
    for (int i = 0; i < 4; ++i) m2[i] = mux(l2, x[i], y[i]);
}
template <int CTRL>
__device__ __forceinline__ void merge_lanes(uint32_t (&m1)[4], uint32_t (&m2)[4]) {
    uint32_t b1[4], b2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        b1[i] = qperm<CTRL>(m1[i]);
        b2[i] = qperm<CTRL>(m2[i]);
    }
    merge2(m1, m2, b1, b2);
}

// 8 waves per SIMD (64 VGPRs): three 9-wave workgroups per CU.  At a 72-register budget only
// two were resident (the waves of a workgroup are not spread evenly over the SIMDs): measured
// 7.56 ms (72 VGPRs) -> 6.51 ms (64) per 2^20-codeword C2 decode (tools/bs_variant.sh A/B).
#ifdef BS_DIAG
#define ABL(bit) (a.ablate & (bit))
#else
#define ABL(bit) 0
#endif
#ifndef BS_WPE
#define BS_WPE 8
#endif
#ifndef BS_KEEP
#define BS_KEEP 0
#endif
template <int D, int DV, int LPC>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(BS_WPE)))
k_bs(BsArgs a) {
    static_assert(LPC == 2 || LPC == 4, "lanes per check");
    constexpr int SB = (DV * QMAX + QMAX <= 127) ? 8 : 9;     // planes of S and of lw + S
    constexpr int EPL = (D + LPC - 1) / LPC;                     // edge slots per check lane
    constexpr int OB = 4 / LPC;                                  // alpha-table output bits per lane
    constexpr int VNW = (DV + 1) / 2 + 1;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if ((uint32_t)(uintptr_t)smem != 0u) __builtin_trap();          // slots are LDS-absolute
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nv = a.n_vars;
    const int64_t b0 = (int64_t)blockIdx.x * PACK;
    const int nvalid = (int)min<int64_t>(PACK, a.B - b0);
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);   // [0] wrong_t, [1] all t, [2] APP > 0, [3] bits
    const int AL = a.arows * LUT_W, BL = a.bcols * LUT_W;
    uint32_t* ALUT = reinterpret_cast<uint32_t*>(smem + a.off_alut);   // [2][arows][LUT_W]
    uint32_t* BLUT = reinterpret_cast<uint32_t*>(smem + a.off_blut);   // [2][bcols][LUT_W]

    // ---- per-lane tables -----------------------------------------------------------------------
    // (the slot addresses are reloaded from the L2-resident tables in each phase rather than
    // held in registers through the whole decode)
    const uint32_t* vt = a.vn_tab + (size_t)tid * VNW;
    uint32_t va[VNW - 1];                                 // slot byte addresses, two per word
#pragma unroll
    for (int p = 0; p < VNW - 1; ++p) va[p] = vt[p];
    const int v = (int)vt[VNW - 1];                       // -1: no variable
    int dw = __builtin_amdgcn_readfirstlane(a.vn_wdeg[2 * wave]);
    int dwmin = __builtin_amdgcn_readfirstlane(a.vn_wdeg[2 * wave + 1]);
    int cn_dmin = a.cn_dmin;
    const bool counted = v >= 0 && v < a.target_bits;
    const uint32_t tab_b = (a.bcols > 1 && v >= 0) ? (uint32_t)((v / (nv / a.bcols)) * LUT_W * 4) : 0u;
    const bool is_cn = tid < a.cn_lanes;

    // ---- channel planes: the lane's variable for the 32 codewords of the pack --------------------
    // (no __syncthreads_or: it allocates static LDS, which would move the dynamic LDS base
    // away from 0; the flag word lives in RED)
    if (tid == 0) RED[7] = 0u;
    __syncthreads();
    uint32_t cs = 0u, cm[4] = {0u, 0u, 0u, 0u};
    int off = 0;
    if (v >= 0 && !ABL(32)) {
        const float* src = a.llr + b0 * nv + v;
        // all 32 loads issued before any use: one HBM round trip per workgroup prologue (with
        // batches of 8 the LLR fetch cost 0.75 ms of a 6.5 ms C2 decode, with this 0.44 ms:
        // the workgroups stay in step, so every pack boundary is a chip-wide HBM burst; a
        // persistent grid prefetching the next pack during the check phases needed 6 more
        // loop-carried registers and spilled: 7.56 ms)
        float xv[PACK];
#pragma unroll
        for (int r = 0; r < PACK; ++r) xv[r] = src[(int64_t)min(r, nvalid - 1) * nv];
#pragma unroll
        for (int r = 0; r < PACK; ++r) {
            const float x = xv[r] * a.inv;
            const float xr = rintf(x);
            off |= (xr != x || fabsf(xr) > (float)QMAX) ? 1 : 0;
            const int xi = (r < nvalid) ? (int)xr : 0;
            const uint32_t m = (uint32_t)(xi < 0 ? -xi : xi);
            cs |= (xi < 0 ? 1u : 0u) << r;
#pragma unroll
            for (int p = 0; p < 4; ++p) cm[p] |= ((m >> p) & 1u) << r;
        }
    }
    if (off) atomicOr(&RED[7], 1u);
    __syncthreads();
    if (RED[7]) {                              // off the grid: the v5 fixup decodes this pack
        if (tid == 0) a.bad[blockIdx.x] = 1u;
        return;
    }
    if (tid == 0) a.bad[blockIdx.x] = 0u;
    // PAD slot (all ones: V->C negative, magnitude 15), ZERO slot (a zero C->V), counters,
    // iteration 0's tables
    if (tid < SLOT_W) {
        reinterpret_cast<uint32_t*>(smem + a.off_pad)[tid] = 0xFFFFFFFFu;
        reinterpret_cast<uint32_t*>(smem + a.off_zero)[tid] = 0u;
    }
    if (tid < 8) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
    for (int w = tid; w < AL; w += NT) ALUT[w] = a.alut[w];
    for (int w = tid; w < BL; w += NT) BLUT[w] = a.blut[w];
    __syncthreads();

    // ---- variable phase -------------------------------------------------------------------------
    //   first: lw_0 as every edge's V->C (no C->V yet);
    //   else:  S = sum of the C->V, APP_t = Q(ch) + S (hard decision, counters); unless last,
    //          Tv = clamp(Q(beta_{t+1} ch) + S) and V->C_e = clamp(Tv - C->V_e, +-15) per edge
    auto vn_phase = [&](const bool first, const bool last, const uint32_t btab, const int tb)
                        __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < VNW - 1; ++p) asm volatile("" : "+v"(va[p]));   // unpacked per use
        auto vaddr = [&](int f) __attribute__((always_inline)) -> uint32_t {
            return (f & 1) ? (va[f >> 1] >> 16) : (va[f >> 1] & 0xFFFFu);
        };
        uint32_t lw[1][4];                   // |Q(beta_{t+1} ch)| (before the C->V: fewer live registers)
        if (!last) {
            if (ABL(2)) {
#pragma unroll
                for (int i = 0; i < 4; ++i) lw[0][i] = cm[i];
            } else if (a.bcols == 1) {          // one beta per iteration: table in SGPRs
                lut_s(lw[0], cm, (const ConstW*)(a.blut) + (size_t)tb * LUT_W);
            } else {
                const uint32_t cmi[1][4] = {{cm[0], cm[1], cm[2], cm[3]}};
                lut<1>(lw, cmi, btab);
            }
        }
        // C->V of the first KEEP edges stay in registers for the V->C pass, the others are read
        // again (the register budget of three 9-wave workgroups per CU)
        constexpr int KEEP = BS_KEEP < DV ? BS_KEEP : DV;
        uint32_t mn[KEEP > 0 ? KEEP : 1], mb[KEEP > 0 ? KEEP : 1][4];
        uint32_t S[SB];
#pragma unroll
        for (int i = 0; i < SB; ++i) S[i] = 0u;
        if (!first) {
#pragma unroll
            for (int f = 0; f < DV; ++f) {
                if (f < dw) {
                    uint32_t M[4], n, b[4];
                    read_slot(n, M, vaddr(f));
#pragma unroll
                    for (int i = 0; i < 4; ++i) b[i] = M[i] ^ n;
                    if (f == 0) set_b<SB>(S, b, n);
                    else add_b<SB>(S, b, n);
                    if (f < KEEP) {
                        mn[f < KEEP ? f : 0] = n;
#pragma unroll
                        for (int i = 0; i < 4; ++i) mb[f < KEEP ? f : 0][i] = b[i];
                    }
                }
            }
            // APP_t = Q(ch) + S: the sign (hard decision) from the carry chain alone, the full
            // sum only in the last iteration (APP > 0 for the loss counter)
            uint32_t hd, nz = 0u;
            if (last) {
                uint32_t A[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) A[i] = S[i];
                const uint32_t cb[4] = {cm[0] ^ cs, cm[1] ^ cs, cm[2] ^ cs, cm[3] ^ cs};
                add_b<SB>(A, cb, cs);
                hd = ~A[SB - 1];
#pragma unroll
                for (int i = 0; i < SB; ++i) nz |= A[i];
            } else {
                uint32_t c = cs;
#pragma unroll
                for (int i = 0; i < SB - 1; ++i) c = B3(T_MAJ, S[i], i < 4 ? (cm[i] ^ cs) : cs, c);
                hd = B3(T_XNOR3, S[SB - 1], cs, c);
            }
            hd &= valid;                                     // APP >= 0 -> hard decision 1
            if (ABL(8)) hd = 0u;
            uint32_t wr = counted ? hd : 0u, apos = 0u, nb = 0u;
            if (last && counted) {
                apos = hd & nz;
                nb = (uint32_t)__popc(hd);
            }
            if (!ABL(8)) wr = wave_or(wr);
            if (last) {
                apos = wave_or(apos);
                nb = wave_add(nb);
            }
            if (lane == 0) {
                if (wr) atomicOr(&RED[0], wr);
                if (last) {
                    if (apos) atomicOr(&RED[2], apos);
                    if (nb) atomicAdd(&RED[3], nb);
                }
            }
        }
        if (last) return;
        // Tv = clamp(Q(beta ch) + S): the table gives |Q(beta ch)|, the channel the sign
        uint32_t lb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) lb[i] = lw[0][i] ^ cs;
        add_b<SB>(S, lb, cs);
        uint32_t Tv[6];
        clamp6<SB>(Tv, S);
        if (first) {
            uint32_t x[7], X[4];
#pragma unroll
            for (int i = 0; i < 7; ++i) x[i] = Tv[i < 6 ? i : 5];
            abs_sat(X, x);
#pragma unroll
            for (int f = 0; f < DV; ++f)
                if (f < dw && (f < dwmin || vaddr(f) != a.off_zero)) write_slot(vaddr(f), x[6], X);
        } else {
#pragma unroll
            for (int f = 0; f < DV; ++f) {
                if (f < dw) {
                    if (ABL(4)) continue;
                    uint32_t x[7], X[4], n, b[4];
                    if (f < KEEP) {
                        n = mn[f < KEEP ? f : 0];
#pragma unroll
                        for (int i = 0; i < 4; ++i) b[i] = mb[f < KEEP ? f : 0][i];
                    } else {
                        uint32_t M[4];
                        read_slot(n, M, vaddr(f));
#pragma unroll
                        for (int i = 0; i < 4; ++i) b[i] = M[i] ^ n;
                    }
                    sub_tv(x, Tv, b, n);
                    abs_sat(X, x);
                    if (f < dwmin || vaddr(f) != a.off_zero) write_slot(vaddr(f), x[6], X);
                }
            }
        }
    };

    vn_phase(true, false, a.off_blut + tab_b, 0);
    // check lanes: lane LPC c + j (check c = row i, index h) takes edges k = LPC m + j, at slots
    // first_i + j A_i + m z + h (a.row_lay); edges past the degree read the all-ones PAD slot
    // and are not written; idle lanes (c >= n_checks) read PAD only
    const int cc = tid / LPC, cj = tid % LPC;
    const int ci = min(cc / a.z, a.n_checks / a.z - 1);
    const int cdeg = (cc < a.n_checks) ? a.row_ptr[ci + 1] - a.row_ptr[ci] : 0;
    uint32_t cbase = (uint32_t)((a.row_lay[2 * ci] + cj * a.row_lay[2 * ci + 1] + (cc - ci * a.z)) * SLOT_B);
    const uint32_t cstride = (uint32_t)(a.z * SLOT_B);
    // (lane j of a check's group evaluates output bits OB j .. OB j + OB - 1 of the alpha table:
    // 16 words per bit, at 64 B per bit)
    const uint32_t tab_a = a.off_alut + (uint32_t)((a.arows > 1 ? ci : 0) * LUT_W * 4) + (uint32_t)(cj * OB * 64);
    __syncthreads();

    for (int t = 0; t < (ABL(16) ? 0 : a.T); ++t) {
        if (tid == 0 && t > 0) {            // fold iteration t-1's frame flags
            RED[1] &= RED[0];
            RED[0] = 0u;
        }
        const int nx = (t + 1) & 1;
        asm volatile("" : "+s"(dw), "+s"(dwmin), "+s"(cn_dmin));   // compared per use, not hoisted as masks
        // next iteration's tables (their slots were last read two phases ago)
        if (t + 1 < a.T) {
            for (int w = tid; w < AL; w += NT) ALUT[nx * AL + w] = a.alut[(size_t)(t + 1) * AL + w];
            if (a.bcols > 1)
                for (int w = tid; w < BL; w += NT) BLUT[nx * BL + w] = a.blut[(size_t)(t + 1) * BL + w];
        }
        // ======== check nodes ===================================================================
        if (is_cn && !ABL(1)) {
            asm volatile("" : "+v"(cbase));
            // slot m of the lane: always a real edge while LPC m + LPC - 1 < cn_dmin
            auto real = [&](int m) __attribute__((always_inline)) -> bool {
                return LPC * m + LPC - 1 < cn_dmin || LPC * m + cj < cdeg;
            };
            auto caddr = [&](int m) __attribute__((always_inline)) -> uint32_t {
                return real(m) ? cbase + m * cstride : a.off_pad;
            };
            // pass 1: two minima of |V->C| and the parity of [V->C >= 0] over the lane's edges
            // (padding edges: negative, magnitude 15), then merged across the lane group
            // (the lane's EPL slots are read once, all loads issued before any use, and kept
            // in registers for pass 2)
            uint32_t Xs[EPL][4], ns[EPL];
#pragma unroll
            for (int m = 0; m < EPL; ++m) read_slot(ns[m], Xs[m], caddr(m));
            uint32_t m1[4] = {Xs[0][0], Xs[0][1], Xs[0][2], Xs[0][3]}, m2[4] = {~0u, ~0u, ~0u, ~0u};
            uint32_t par = ns[0];
#pragma unroll
            for (int m = 1; m < EPL; ++m) {
                const uint32_t(&X)[4] = Xs[m];
                const uint32_t l1 = lt4(X, m1), l2 = lt4(X, m2);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    m2[i] = mux(l1, m1[i], mux(l2, X[i], m2[i]));
                    m1[i] = mux(l1, X[i], m1[i]);
                }
                par ^= ns[m];
            }
            par ^= qperm<QP_X1>(par);
            merge_lanes<QP_X1>(m1, m2);
            if (LPC == 4) {
                par ^= qperm<QP_X2>(par);
                merge_lanes<QP_X2>(m1, m2);
            }
            // message k is negative iff an even number of the OTHER edges have V->C >= 0
            // (Main_Functions.py:251-254): par ^ n_k, par the parity of [V->C >= 0] over the
            // LPC EPL slots (an even count, padding included)
            // weighted, quantized minima: each lane evaluates OB output bits, the group shares them
            uint32_t q1[4], q2[4];
            {
                const uint32_t mm[2][4] = {{m1[0], m1[1], m1[2], m1[3]}, {m2[0], m2[1], m2[2], m2[3]}};
                const uint32_t tab = tab_a + (uint32_t)((t & 1) * AL * 4);
                uint32_t qb[OB][2];
#pragma unroll
                for (int b = 0; b < OB; ++b) {
                    uint32_t o[2];
                    lut_bit<2>(o, mm, tab + (uint32_t)(b * 64));
                    qb[b][0] = o[0];
                    qb[b][1] = o[1];
                }
                if (LPC == 4) {
                    q1[0] = qperm<0x00>(qb[0][0]); q1[1] = qperm<0x55>(qb[0][0]);
                    q1[2] = qperm<0xAA>(qb[0][0]); q1[3] = qperm<0xFF>(qb[0][0]);
                    q2[0] = qperm<0x00>(qb[0][1]); q2[1] = qperm<0x55>(qb[0][1]);
                    q2[2] = qperm<0xAA>(qb[0][1]); q2[3] = qperm<0xFF>(qb[0][1]);
                } else {                // lane 0 of a pair holds bits 0, 1; lane 1 bits 2, 3
                    q1[0] = qperm<0xA0>(qb[0][0]); q1[1] = qperm<0xA0>(qb[OB - 1][0]);
                    q1[2] = qperm<0xF5>(qb[0][0]); q1[3] = qperm<0xF5>(qb[OB - 1][0]);
                    q2[0] = qperm<0xA0>(qb[0][1]); q2[1] = qperm<0xA0>(qb[OB - 1][1]);
                    q2[2] = qperm<0xF5>(qb[0][1]); q2[3] = qperm<0xF5>(qb[OB - 1][1]);
                }
            }
            // pass 2: an edge whose |V->C| equals the minimum gets the weighted second minimum
            // (if it is not the only one, the two minima are equal), the others the minimum
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                if (real(m)) {
                    const uint32_t addr = cbase + m * cstride;
                    const uint32_t(&X)[4] = Xs[m];
                    const uint32_t n = ns[m];
                    uint32_t Mg[4];
                    uint32_t ne = X[0] ^ m1[0];
#pragma unroll
                    for (int i = 1; i < 4; ++i) ne = B3(T_ORXOR, ne, X[i], m1[i]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) Mg[i] = mux(ne, q1[i], q2[i]);
                    write_slot(addr, par ^ n, Mg);
                }
            }
        }
        __syncthreads();
        // ======== variable nodes ================================================================
        const uint32_t btab = a.off_blut + (uint32_t)(nx * BL * 4) + tab_b;
        if (t == a.T - 1) vn_phase(false, true, btab, t + 1);
        else vn_phase(false, false, btab, t + 1);
        __syncthreads();
    }
    if (tid == 0) {
        const uint32_t wl = RED[0] & valid;
        const uint32_t all = RED[1] & RED[0] & valid;
        const uint32_t ap = RED[2] & valid;
        if (a.counters) {
            unsigned long long* cc = reinterpret_cast<unsigned long long*>(a.counters);
            const unsigned long long c0 = RED[3], c1 = __popc(wl), c2 = __popc(all),
                                     c3 = 2ull * __popc(ap) + __popc(wl & ~ap);
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

// per-decode tables: 16-entry g(m) tables as mux-tree leaves, [t][table][bit j][pair p] {X, Y}
// with Y = bit j of g(2p) (as a 0 / ~0 word) and X = Y ^ (bit j of g(2p + 1)):
// level 1 of the tree is (m0 & X) ^ Y.
//   alpha: g(m) = Q(relu(fl32(m step * alpha_{t,row}))) (Main_Functions.py:266-316), m = min(|V->C|)
//   beta:  g(m) = Q(fl32(m * beta_{t,col})) in grid units (lw = Q(beta ch), :164-177; beta >= 0)
__global__ void k_bs_tables(const float* __restrict__ alpha, const float* __restrict__ beta,
                            const int32_t* __restrict__ row_ptr, int T, int E, int N, int arows,
                            int bcols, float step, float inv, uint32_t* alut, uint32_t* blut) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;    // one table per thread
    const int na = T * arows, nbt = T * bcols;
    if (f >= na + nbt) return;
    int g[16];
    uint32_t* out;
    if (f < na) {
        const int t = f / arows, row = f - t * arows;
        const float w = alpha[(size_t)t * E + row_ptr[row]];
        for (int m = 0; m < 16; ++m) g[m] = f5::q_mag5(m, w, step, inv, QMAX);
        out = alut + (size_t)f * LUT_W;
    } else {
        const int f2 = f - na;
        const int t = f2 / bcols, col = f2 - t * bcols;
        const float b = beta[(size_t)t * N + col];
        for (int m = 0; m < 16; ++m) {
            const int q = (int)__builtin_amdgcn_fmed3f(rintf((float)m * b), -(float)QMAX, (float)QMAX);
            g[m] = q < 0 ? -q : q;       // beta >= 0 (checked on the host)
        }
        out = blut + (size_t)f2 * LUT_W;
    }
    for (int j = 0; j < 4; ++j)
        for (int p = 0; p < 8; ++p) {
            const uint32_t y = ((g[2 * p] >> j) & 1) ? ~0u : 0u;
            const uint32_t x = y ^ (((g[2 * p + 1] >> j) & 1) ? ~0u : 0u);
            out[j * 16 + 2 * p] = x;
            out[j * 16 + 2 * p + 1] = y;
        }
}

// ---- host: planning, graph tables, launch -------------------------------------------------
// kernel instances (D = check-degree bound, DV = variable-degree bound)
// (LPC = lanes per check: 4 measured 6.31 ms against 2's 6.73 ms per C2 decode, same box)
struct BsInst { int D, DV, LPC; };
constexpr BsInst kInst[] = {{15, 6, 4}, {16, 8, 4}, {15, 6, 2}};

struct BsPlan {
    bool ok = false;
    int inst = -1, nw = 0, cn_lanes = 0, arows = 1, bcols = 1;
    uint32_t off_pad = 0, off_zero = 0, off_red = 0, off_alut = 0, off_blut = 0;
    int cn_dmin = 0;
    size_t lds = 0;
    std::vector<int32_t> lay;      // [M][2] first slot of proto row i, stride A_i of its j-blocks
};

// Slot layout: edge k of check (row i, index h) is slot first_i + (k mod LPC) A_i +
// (k div LPC) z + h.  LDS banking (MI355X_MICROARCH.md, LDS): ds_read_b32 / ds_read2_b32 /
// ds_write_b32 serve a wave in two 32-lane groups, bank = dword address mod 32; a slot's words
// are 5 s + p, so a group is conflict-free when its 32 slot numbers are distinct mod 32.  The
// 32 / LPC consecutive checks of a group read, for one m, slots first + j A + h: with
// first_i = first_{i-1} + z (mod 32) the checks stay consecutive mod 32 across a row boundary,
// and A_i is the smallest stride >= the j = 0 block whose multiples j A_i (j < LPC) are at
// least 32 / LPC apart mod 32.
static std::vector<int32_t> slot_layout(const host::GraphTables& h, int LPC, size_t* nslot) {
    std::vector<int32_t> lay((size_t)2 * h.M, 0);
    const int sep = 32 / LPC;
    auto ok = [&](int A) {
        for (int d = 1; d < LPC; ++d) {
            const int r = (d * A) % 32;
            if (std::min(r, 32 - r) < sep) return false;
        }
        return true;
    };
    size_t cur = 0;
    for (int i = 0; i < h.M; ++i) {
        const int deg = h.row_ptr[i + 1] - h.row_ptr[i];
        size_t first = cur;
        if (i > 0) first += (size_t)((((int64_t)lay[2 * (i - 1)] + h.z - (int64_t)cur) % 32 + 32) % 32);
        int A = ((deg + LPC - 1) / LPC) * h.z;
        while (!ok(A)) ++A;
        const int last_rows = (deg - (LPC - 1) + LPC - 1) / LPC;   // block j = LPC - 1
        cur = first + (size_t)(LPC - 1) * A + (size_t)std::max(last_rows, 0) * h.z;
        lay[2 * i] = (int32_t)first;
        lay[2 * i + 1] = A;
    }
    *nslot = cur;
    return lay;
}

BsPlan bs_plan(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    BsPlan p;
    const char* e = getenv("LDPC_BS");
    if (e && atoi(e) == 0) return p;
    const char* el = getenv("LDPC_BS_LPC");          // A/B: force 2 or 4 lanes per check
    const int want_lpc = el ? atoi(el) : 0;
    if (mode != MODE_Q5 && mode != MODE_QM5) return p;           // qmax 15: 4 magnitude planes
    if (ucn || per_edge_w || !g.host || !g.w_beta_nonneg) return p;
    const host::GraphTables& h = *g.host;
    int min_cdeg = 1 << 30;
    for (int i = 0; i < h.M; ++i) min_cdeg = std::min(min_cdeg, h.row_ptr[i + 1] - h.row_ptr[i]);
    if (min_cdeg < 2) return p;                                   // ("no other edge" rule unneeded)
    for (int i = 0; i < (int)(sizeof(kInst) / sizeof(kInst[0])); ++i)
        if (h.max_cdeg <= kInst[i].D && h.max_vdeg <= kInst[i].DV &&
            (want_lpc == 0 || want_lpc == kInst[i].LPC)) { p.inst = i; break; }
    if (p.inst < 0) return p;
    const int LPC = kInst[p.inst].LPC;
    const int nv = g.n_vars, nc = g.n_checks;
    p.cn_lanes = 64 * ((LPC * nc + 63) / 64);
    p.nw = std::max((nv + 63) / 64, p.cn_lanes / 64);
    if (p.nw > 16) return p;                                      // one variable per lane
    p.arows = g.w_alpha_uniform ? 1 : h.M;
    p.bcols = g.w_beta_uniform ? 1 : h.N;
    // idle check lanes: every slot is decided per lane
    p.cn_dmin = (p.cn_lanes == LPC * nc) ? min_cdeg : 0;
    size_t nslot = 0;
    p.lay = slot_layout(h, LPC, &nslot);
    p.off_pad = (uint32_t)(nslot * SLOT_B);
    p.off_zero = p.off_pad + SLOT_B;
    const size_t slot_end = (size_t)p.off_zero + SLOT_B;
    if (slot_end > 65535) return p;                               // 16-bit slot addresses
    size_t o = (slot_end + 15) & ~(size_t)15;
    p.off_red = (uint32_t)o;
    o += 64;
    p.off_alut = (uint32_t)o;
    o += (size_t)2 * p.arows * LUT_W * 4;
    p.off_blut = (uint32_t)o;
    o += (size_t)2 * p.bcols * LUT_W * 4;
    p.lds = (o + 15) & ~(size_t)15;
    if (p.lds > BS_LDS_MAX) return p;
    p.ok = true;
    return p;
}

}  // namespace bs

using namespace bs;

bool bs_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    return bs_plan(g, mode, ucn, per_edge_w).ok;
}

const char* bs_kernel_name(const DevGraph& g) {
    static thread_local char buf[48];
    const BsPlan p = bs_plan(g, MODE_Q5, false, false);
    snprintf(buf, sizeof(buf), "bsl[p32,w%d,d%d,v%d,l%d]", p.nw, p.inst >= 0 ? kInst[p.inst].D : 0,
             p.inst >= 0 ? kInst[p.inst].DV : 0, p.inst >= 0 ? kInst[p.inst].LPC : 0);
    return buf;
}

// graph tables, built once per context on the host (ws.bs_graph)
static int bs_graph_tables(const DevGraph& g, const BsPlan& p, FusedWorkspace& ws, hipStream_t s) {
    if (ws.bs_graph) return LDPC_OK;
    const host::GraphTables& h = *g.host;
    const int nv = g.n_vars, nc = g.n_checks, z = h.z;
    const int DV = kInst[p.inst].DV;
    const int VNW = (DV + 1) / 2 + 1;
    const int nl = 64 * p.nw;
    std::vector<uint32_t> vn((size_t)nl * VNW, 0u);
    std::vector<int32_t> wdeg(2 * p.nw, 0);
    auto put16 = [](uint32_t* w, int k, uint32_t addr) { w[k >> 1] |= addr << (16 * (k & 1)); };
    auto slot_addr = [&](int i, int k, int hc) {
        const int LPC = kInst[p.inst].LPC;
        return (uint32_t)(((size_t)p.lay[2 * i] + (size_t)(k % LPC) * p.lay[2 * i + 1] +
                           (size_t)(k / LPC) * z + hc) * SLOT_B);
    };
    // variable lanes: variables by descending degree in chunks of 64; the chunks are dealt to
    // waves so that the SIMDs (wave w on SIMD w mod 4) get similar work (a chunk costs about
    // 3 + dw units, dw its largest degree); edge f of variable (col j, index hh) through proto
    // edge pe (row i, position k) is slot (i, k, (hh - shift) mod z)
    std::vector<int> order(nv);
    for (int v = 0; v < nv; ++v) order[v] = v;
    auto vdeg = [&](int v) { const int j = v / z; return h.col_ptr[j + 1] - h.col_ptr[j]; };
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return vdeg(x) > vdeg(y); });
    const int nch = (nv + 63) / 64;
    std::vector<int> wave_of(nch, -1), simd_load(4, 0);
    std::vector<char> used(p.nw, 0);
    for (int ch = 0; ch < nch; ++ch) {                 // chunks come in descending cost order
        const int cost = 3 + vdeg(order[64 * ch]);
        int best = -1;
        for (int sm = 0; sm < 4; ++sm) {
            bool free_slot = false;
            for (int w = sm; w < p.nw; w += 4) free_slot |= !used[w];
            if (free_slot && (best < 0 || simd_load[sm] < simd_load[best])) best = sm;
        }
        int w = best;
        while (used[w]) w += 4;
        used[w] = 1;
        wave_of[ch] = w;
        simd_load[best] += cost;
    }
    for (int w = 0; w < p.nw; ++w) {
        wdeg[2 * w] = 0;
        wdeg[2 * w + 1] = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t* q = &vn[(size_t)(64 * w + l) * VNW];
            for (int f = 0; f < DV; ++f) put16(q, f, p.off_zero);
            q[VNW - 1] = 0xFFFFFFFFu;
        }
    }
    for (int ch = 0; ch < nch; ++ch) {
        const int w = wave_of[ch];
        int dmax = 0, dmin = 1 << 30;
        for (int l = 0; l < 64; ++l) {
            uint32_t* q = &vn[(size_t)(64 * w + l) * VNW];
            const int o = 64 * ch + l;
            if (o >= nv) { dmin = 0; continue; }
            const int v = order[o], j = v / z, hh = v - j * z;
            const int c0 = h.col_ptr[j], dv = h.col_ptr[j + 1] - c0;
            q[0] = 0u;
            for (int pw = 1; pw < VNW - 1; ++pw) q[pw] = 0u;
            for (int f = 0; f < DV; ++f) {
                uint32_t addr = p.off_zero;
                if (f < dv) {
                    const int pe = h.col_pe[c0 + f], i = h.pe_row[pe];
                    int hc = hh - h.pe_shift[pe];
                    hc = hc < 0 ? hc + z : hc;
                    addr = slot_addr(i, pe - h.row_ptr[i], hc);
                }
                put16(q, f, addr);
            }
            q[VNW - 1] = (uint32_t)v;
            dmax = std::max(dmax, dv);
            dmin = std::min(dmin, dv);
        }
        wdeg[2 * w] = dmax;
        wdeg[2 * w + 1] = dmin;
    }
    const size_t bytes = (vn.size() + wdeg.size() + p.lay.size()) * 4;
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
    uint32_t* dp = reinterpret_cast<uint32_t*>(d);
    if (hipMemcpyAsync(dp, vn.data(), vn.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dp + vn.size(), wdeg.data(), wdeg.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dp + vn.size() + wdeg.size(), p.lay.data(), p.lay.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(d);
        return LDPC_ERR_HIP;
    }
    ws.bs_graph = d;
    ws.bs_graph_inst = p.inst;
    return LDPC_OK;
}

template <int D, int DV, int LPC>
static int launch_bs(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bs<D, DV, LPC>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)BS_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_bs<D, DV, LPC>), dim3(nblocks), dim3(64 * nw), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

int bs_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
              int64_t* counters, uint8_t* flags, uint32_t* bad, hipStream_t s) {
    const BsPlan p = bs_plan(g, mode, false, false);
    if (!p.ok) return LDPC_ERR_UNSUPPORTED;
    if (ws.bs_graph && ws.bs_graph_inst != p.inst) {
        (void)hipFree(ws.bs_graph);
        ws.bs_graph = nullptr;
    }
    int st = bs_graph_tables(g, p, ws, s);
    if (st != LDPC_OK) return st;
    const float step = (mode == MODE_Q5) ? 0.5f : 1.0f;
    const size_t na = (size_t)b.T * p.arows * LUT_W, nb = (size_t)b.T * p.bcols * LUT_W;
    const size_t bytes = (na + nb) * 4;
    if (bytes > ws.bs_lut_bytes) {
        if (ws.bs_lut) (void)hipFree(ws.bs_lut);
        ws.bs_lut = nullptr;
        ws.bs_lut_bytes = 0;
        if (hipMalloc(&ws.bs_lut, bytes) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
        ws.bs_lut_bytes = bytes;
    }
    uint32_t* alut = reinterpret_cast<uint32_t*>(ws.bs_lut);
    uint32_t* blut = alut + na;
    const int ntab = b.T * (p.arows + p.bcols);
    hipLaunchKernelGGL(k_bs_tables, dim3((unsigned)((ntab + 127) / 128)), dim3(128), 0, s, b.alpha,
                       b.beta, g.row_ptr, b.T, g.E, g.N, p.arows, p.bcols, step, 1.0f / step,
                       alut, blut);
    if (hipGetLastError() != hipSuccess) return LDPC_ERR_HIP;
    const int D = kInst[p.inst].D, DV = kInst[p.inst].DV;
    const int VNW = (DV + 1) / 2 + 1;
    (void)D;
    const uint32_t* gt = reinterpret_cast<const uint32_t*>(ws.bs_graph);
    BsArgs a{};
    a.llr = llr;
    a.B = b.B;
    a.n_vars = g.n_vars;
    a.n_checks = g.n_checks;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.cn_lanes = p.cn_lanes;
    a.cn_dmin = p.cn_dmin;
    a.inv = 1.0f / step;
    a.row_ptr = g.row_ptr;
    a.z = g.z;
    a.vn_tab = gt;
    a.vn_wdeg = reinterpret_cast<const int32_t*>(a.vn_tab + (size_t)64 * p.nw * VNW);
    a.row_lay = a.vn_wdeg + 2 * p.nw;
    a.alut = alut;
    a.blut = blut;
    a.arows = p.arows;
    a.bcols = p.bcols;
    a.counters = counters;
    a.flags = flags;
    a.bad = bad;
    a.off_pad = p.off_pad;
    a.off_zero = p.off_zero;
    a.off_red = p.off_red;
    a.off_alut = p.off_alut;
    a.off_blut = p.off_blut;
    if (const char* e = getenv("LDPC_DIAG_ABLATE")) a.ablate = atoi(e);   // -DBS_DIAG builds
    const int nblocks = (int)((b.B + PACK - 1) / PACK);
    switch (p.inst) {
        case 0: return launch_bs<15, 6, 4>(a, nblocks, p.nw, p.lds, s);
        case 1: return launch_bs<16, 8, 4>(a, nblocks, p.nw, p.lds, s);
        default: return launch_bs<15, 6, 2>(a, nblocks, p.nw, p.lds, s);
    }
}

}  // namespace ldpc
