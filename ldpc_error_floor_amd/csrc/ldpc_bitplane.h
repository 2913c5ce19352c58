// ldpc_bitplane.h — the bit-sliced kernels' plane arithmetic (bsl, bsc): every quantity of a
// 32-codeword pack is a set of bit planes, and each 3-input boolean function one v_bitop3_b32.
// Kept free of HIP so that tests/native/bitplane_check.cpp can run every function on the host
// over all operand values (LDPC_BP_FN / LDPC_BITOP3 defined there as host code).
#pragma once
#include <cstdint>

#ifndef LDPC_BP_FN
#define LDPC_BP_FN __device__ __forceinline__
#endif
#ifndef LDPC_BITOP3
#define LDPC_BITOP3(a, b, c, F) __builtin_amdgcn_bitop3_b32((a), (b), (c), (F))
#endif

namespace ldpc {
namespace bs {

// ---- bit-plane arithmetic ---------------------------------------------------------------------
// fewer ops in the variable phase's plane arithmetic (set_b's sign planes, sub_tv's carry-in,
// abs_sat's conditional negation; A/B switch)
#ifndef BS_SETB
#define BS_SETB 1
#endif
// abs_sat in 12 ops (A/B switch)
#ifndef BS_ABS12
#define BS_ABS12 1
#endif
// set_b's sign planes as copies of plane 4 (A/B switch, off: the compiler turned the copies into
// v_mov and the C2 build spilled 3 VGPRs, for no fewer instructions in the sum)
#ifndef BS_SETB_SIGN
#define BS_SETB_SIGN 0
#endif
// Every 3-input function is one v_bitop3_b32 with an explicit truth table (the compiler's own
// boolean synthesis often emits two or three ops for one such function); 2-input functions are
// left to the compiler, which emits the 2-cycle VOP2 forms (v_and / v_or / v_xor / v_xnor).
// Truth table of f: f(0xF0, 0xCC, 0xAA) for operands (a, b, c).
#define B3(F, a, b, c) LDPC_BITOP3((a), (b), (c), (F))
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
constexpr unsigned T_ORXOR = (TA | (TB ^ TC)) & 0xFF;                    // a | (b ^ c)
LDPC_BP_FN uint32_t mux(uint32_t s, uint32_t a, uint32_t b) { return B3(T_MUX, s, a, b); }

// S += m for m = (negative flag n, b) with b_i = M_i ^ n (M the 4 magnitude planes): the
// two's complement of m is b sign-extended with n, plus n
template <int SB>
LDPC_BP_FN void add_b(uint32_t (&S)[SB], const uint32_t (&b)[4], uint32_t n) {
    // (the carry first: S[i]'s last use is then the instruction that redefines it, so the sum
    // stays in S's registers; summed under a wave-uniform "edge f exists" branch, the other order
    // left a copy of every plane at the branch's merge, 7 v_mov per edge)
    uint32_t c = n;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        const uint32_t bi = (i < 4) ? b[i] : n;
        const uint32_t cn = (i + 1 < SB) ? B3(T_MAJ, S[i], bi, c) : 0u;
        S[i] = B3(T_XOR3, S[i], bi, c);
        c = cn;
    }
}
// S = m (same operand form), S previously zero.  Above the magnitude planes every plane is the
// same word: the carry into plane 4 is n & b0 & .. & b3, a subset of n, so S_i = n ^ c4 for
// i >= 4 (BS_SETB_SIGN: the SB - 5 planes above plane 4 as its copies)
template <int SB>
LDPC_BP_FN void set_b(uint32_t (&S)[SB], const uint32_t (&b)[4], uint32_t n) {
    uint32_t c = n;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        if (BS_SETB_SIGN && i > 4) {
            S[i] = S[4];
            continue;
        }
        const uint32_t bi = (i < 4) ? b[i] : n;
        S[i] = bi ^ c;
        c = bi & c;
    }
}

// x = Tv - m (7 planes, two's complement; Tv in [-32, 31], |m| <= 15) with m = (n, b) as above:
// -m is ~b sign-extended with ~n, plus ~n
LDPC_BP_FN void sub_tv(uint32_t (&x)[7], const uint32_t (&T)[6], const uint32_t (&b)[4],
                                       uint32_t n) {
    // (plane 0 takes the carry-in ~n inside its truth tables: no v_not of n, BS_SETB)
    constexpr unsigned T_MAJNN = ((TA & ~TB) | (TA & ~TC) | (~TB & ~TC)) & 0xFF;   // maj(a, ~b, ~c)
    uint32_t c;
    if (BS_SETB) {
        x[0] = B3(T_XOR3, T[0], b[0], n);
        c = B3(T_MAJNN, T[0], b[0], n);
    } else {
        c = ~n;
        x[0] = B3(T_XNOR3, T[0], b[0], c);
        c = B3(T_MAJNB, T[0], b[0], c);
    }
#pragma unroll
    for (int i = 1; i < 7; ++i) {
        const uint32_t t = T[i < 6 ? i : 5];
        const uint32_t bi = (i < 4) ? b[i] : n;
        x[i] = B3(T_XNOR3, t, bi, c);
        if (i < 6) c = B3(T_MAJNB, t, bi, c);
    }
}

// min(|x|, 15) (4 planes) of a 7-plane two's complement x in [-64, 63]; the sign is x[6].
// For x < 0 the low bits of -x are x_i ^ OR(x_j, j < i); |x| >= 16 is x5 | x4 for x >= 0 and
// "not (x5 & x4 & low 4 bits nonzero)" for x < 0.
LDPC_BP_FN void abs_sat(uint32_t (&X)[4], const uint32_t (&x)[7]) {
    const uint32_t neg = x[6];
    if (BS_ABS12) {
        // p_i = neg & (x_0 | .. | x_{i-1}), then X_i = (x_i ^ p_i) | sat in one op each (12 ops
        // against 13)
        constexpr unsigned T_ANDOR = (TA & (TB | TC)) & 0xFF;      // a & (b | c)
        constexpr unsigned T_ORAND = (TA | (TB & TC)) & 0xFF;      // a | (b & c)
        constexpr unsigned T_XOROR = ((TA ^ TB) | TC) & 0xFF;      // (a ^ b) | c
        constexpr unsigned T_OR3 = (TA | TB | TC) & 0xFF;
        const uint32_t p1 = neg & x[0];
        const uint32_t p2 = B3(T_ANDOR, neg, x[0], x[1]);
        const uint32_t p3 = B3(T_ORAND, p2, neg, x[2]);
        const uint32_t o4 = B3(T_OR3, x[0] | x[1], x[2], x[3]);
        const uint32_t sat = B3(T_SAT, neg, B3(T_AND3, x[5], x[4], o4), x[5] | x[4]);
        X[0] = x[0] | sat;
        X[1] = B3(T_XOROR, x[1], p1, sat);
        X[2] = B3(T_XOROR, x[2], p2, sat);
        X[3] = B3(T_XOROR, x[3], p3, sat);
        return;
    }
    const uint32_t o2 = x[0] | x[1], o3 = o2 | x[2], o4 = o3 | x[3];
    const uint32_t sat = B3(T_SAT, neg, B3(T_AND3, x[5], x[4], o4), x[5] | x[4]);
    X[0] = x[0] | sat;
    X[1] = B3(T_XAND, x[1], neg, x[0]) | sat;
    X[2] = B3(T_XAND, x[2], neg, o2) | sat;
    X[3] = B3(T_XAND, x[3], neg, o3) | sat;
}

// a < b for 4-plane unsigned values
LDPC_BP_FN uint32_t lt4(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
    uint32_t l = B3(T_ANDN, a[0], b[0], 0u);
#pragma unroll
    for (int i = 1; i < 4; ++i) l = B3(T_LT, a[i], b[i], l);
    return l;
}

// SB-plane two's complement -> 6 planes, saturated to [-32, 31]
template <int SB>
LDPC_BP_FN void clamp6(uint32_t (&T)[6], const uint32_t (&v)[SB]) {
    uint32_t ovf = 0;
#pragma unroll
    for (int i = 5; i < SB - 1; ++i) ovf |= v[i] ^ v[i + 1];
    const uint32_t s = v[SB - 1];
#pragma unroll
    for (int i = 0; i < 5; ++i) T[i] = B3(T_SAT, ovf, s, v[i]);
    T[5] = mux(ovf, s, v[5]);
}

}  // namespace bs
}  // namespace ldpc
