// Host check of the bit-sliced kernels' plane arithmetic (csrc/ldpc_bitplane.h), exhaustive over
// the operand ranges the kernels use: every function runs on the host with v_bitop3_b32 emulated
// bit by bit from its truth table, and 32 different operands ride in the 32 bit positions of each
// plane word, as 32 codewords of a pack do.  Built and run by tests/test_bitplane.py (g++, with
// and without -DBS_SETB=0).  Prints "ok <cases>" or the first mismatches; exit status 1 on any.
#include <cstdint>
#include <cstdio>
#include <vector>

static inline uint32_t bitop3_host(uint32_t a, uint32_t b, uint32_t c, unsigned F) {
    uint32_t r = 0;
    for (int k = 0; k < 32; ++k) {
        const unsigned idx = (((a >> k) & 1u) << 2) | (((b >> k) & 1u) << 1) | ((c >> k) & 1u);
        r |= ((F >> idx) & 1u) << k;
    }
    return r;
}
#define LDPC_BP_FN inline
#define LDPC_BITOP3(a, b, c, F) bitop3_host((a), (b), (c), (F))
#include "ldpc_bitplane.h"

using namespace ldpc::bs;

static long g_bad = 0, g_cases = 0;
static void fail(const char* what, int a, int b, int got, int want) {
    if (g_bad++ < 8) std::printf("%s(%d, %d): got %d, want %d\n", what, a, b, got, want);
}

// lane k of a plane set -> signed value of NP planes (two's complement)
template <int NP>
static int lane_val(const uint32_t (&P)[NP], int k) {
    int v = 0;
    for (int i = 0; i < NP; ++i) v |= (int)((P[i] >> k) & 1u) << i;
    return (v & (1 << (NP - 1))) ? v - (1 << NP) : v;
}
// 32 signed messages in [-15, 15] -> (n, b = M ^ n) operand form
static void msg_planes(const int* m, uint32_t& n, uint32_t (&b)[4]) {
    n = 0;
    for (int i = 0; i < 4; ++i) b[i] = 0;
    for (int k = 0; k < 32; ++k) {
        const int M = m[k] < 0 ? -m[k] : m[k];
        const uint32_t nk = m[k] < 0 ? 1u : 0u;
        n |= nk << k;
        for (int i = 0; i < 4; ++i) b[i] |= ((((uint32_t)M >> i) & 1u) ^ nk) << k;
    }
}

template <int SB>
static void check_sums() {
    // S = m0 (set_b), then + m1 + m2 (add_b): every (m0, m1) pair, m2 cycling
    std::vector<int> all;
    for (int m = -15; m <= 15; ++m) all.push_back(m);
    for (size_t i0 = 0; i0 < all.size(); ++i0)
        for (size_t j = 0; j < all.size(); j += 1) {
            int m0[32], m1[32], m2[32];
            for (int k = 0; k < 32; ++k) {
                m0[k] = all[i0];
                m1[k] = all[(j + (size_t)k) % all.size()];
                m2[k] = all[(i0 * 7 + j * 3 + (size_t)k * 5) % all.size()];
            }
            uint32_t S[SB] = {}, n, b[4];
            msg_planes(m0, n, b);
            set_b<SB>(S, b, n);
            for (int k = 0; k < 32; ++k)
                if (lane_val<SB>(S, k) != m0[k]) fail("set_b", m0[k], 0, lane_val<SB>(S, k), m0[k]);
            msg_planes(m1, n, b);
            add_b<SB>(S, b, n);
            msg_planes(m2, n, b);
            add_b<SB>(S, b, n);
            for (int k = 0; k < 32; ++k) {
                const int want = m0[k] + m1[k] + m2[k];
                if (lane_val<SB>(S, k) != want) fail("add_b", m0[k], m1[k], lane_val<SB>(S, k), want);
                ++g_cases;
            }
            // clamp6: S + a large offset, saturated to [-32, 31]
            if (SB >= 8) {
                int off[32];
                for (int k = 0; k < 32; ++k) off[k] = (k % 2 ? 15 : -15);
                for (int r = 0; r < 2; ++r) {
                    msg_planes(off, n, b);
                    add_b<SB>(S, b, n);
                }
                uint32_t T[6];
                clamp6<SB>(T, S);
                for (int k = 0; k < 32; ++k) {
                    int v = lane_val<SB>(S, k);
                    v = v > 31 ? 31 : (v < -32 ? -32 : v);
                    if (lane_val<6>(T, k) != v) fail("clamp6", lane_val<SB>(S, k), 0, lane_val<6>(T, k), v);
                }
            }
        }
}

int main() {
    check_sums<7>();
    check_sums<8>();
    check_sums<9>();
    // V->C = clamp(Tv - m, +-15) as sign / magnitude: sub_tv + abs_sat, every Tv in [-32, 31]
    // and m in [-15, 15] (a zero is positive, Main_Functions.py:229-230)
    for (int Tv0 = -32; Tv0 <= 31; ++Tv0)
        for (int m0 = -15; m0 <= 15; ++m0) {
            int Tvk[32], mk[32];
            for (int k = 0; k < 32; ++k) {
                Tvk[k] = ((Tv0 + 32 + k) % 64) - 32;
                mk[k] = ((m0 + 15 + 3 * k) % 31) - 15;
            }
            uint32_t T[6] = {}, n, b[4], x[7], X[4];
            for (int k = 0; k < 32; ++k)
                for (int i = 0; i < 6; ++i) T[i] |= (((uint32_t)Tvk[k] >> i) & 1u) << k;
            msg_planes(mk, n, b);
            sub_tv(x, T, b, n);
            abs_sat(X, x);
            for (int k = 0; k < 32; ++k) {
                int v = Tvk[k] - mk[k];
                if (lane_val<7>(x, k) != v) fail("sub_tv", Tvk[k], mk[k], lane_val<7>(x, k), v);
                v = v > 15 ? 15 : (v < -15 ? -15 : v);
                const int want_neg = v < 0, want_mag = v < 0 ? -v : v;
                int mag = 0;
                for (int i = 0; i < 4; ++i) mag |= (int)((X[i] >> k) & 1u) << i;
                if (mag != want_mag) fail("abs_sat magnitude", Tvk[k], mk[k], mag, want_mag);
                if ((int)((x[6] >> k) & 1u) != want_neg) fail("abs_sat sign", Tvk[k], mk[k], (x[6] >> k) & 1u, want_neg);
                ++g_cases;
            }
        }
    // lt4: every (a, b) of 4-bit magnitudes
    for (int a0 = 0; a0 < 16; ++a0) {
        uint32_t A[4] = {}, B[4] = {};
        for (int k = 0; k < 32; ++k) {
            const int bk = k % 16, ak = (k < 16) ? a0 : 15 - a0;
            for (int i = 0; i < 4; ++i) {
                A[i] |= (((uint32_t)ak >> i) & 1u) << k;
                B[i] |= (((uint32_t)bk >> i) & 1u) << k;
            }
        }
        const uint32_t l = lt4(A, B);
        for (int k = 0; k < 32; ++k) {
            const int ak = (k < 16) ? a0 : 15 - a0, bk = k % 16;
            if ((int)((l >> k) & 1u) != (ak < bk ? 1 : 0)) fail("lt4", ak, bk, (l >> k) & 1u, ak < bk);
            ++g_cases;
        }
    }
    if (g_bad) {
        std::printf("FAILED %ld of %ld\n", g_bad, g_cases);
        return 1;
    }
    std::printf("ok %ld\n", g_cases);
    return 0;
}
