// ldpc_bs.hip — bit-sliced fused QMS decoder ("bs"): 32 codewords per 32-bit word.
//
// Same semantics as the v5 kernel (ldpc_fused5_kernel.h) and the reference graph
// (Main_Functions.py:157-335): all T flooding iterations of a block in one launch, integer
// arithmetic in units of the q-bit grid (q = 5 / -5: qmax = 15).  What changes is the data
// layout.  A workgroup decodes one PACK of 32 codewords and every quantity is held as bit
// planes: plane word p of a value holds bit p of that value for the 32 codewords (bit r =
// codeword b0 + r).  The min-sum arithmetic — the V->C subtraction, |.| with saturation, the
// two-minimum / argmin search, the sign parity, the weighted quantization (a 16-entry table
// per iteration and proto row, evaluated as a mux tree) and the variable-node sums — becomes
// boolean algebra on whole words, which gfx950 executes as v_bitop3_b32 (any function of three
// words in one VALU op).  One lane does the work of 32 codeword-lanes of v5: per edge and
// codeword the check side costs ~2 lane-ops instead of ~6 wave-ops/64, and LDS traffic falls
// by the same factor.
//
// Representation (grid units):
//   channel c = Q(ch) on the grid, |c| <= qmax: sign plane + 4 magnitude planes (the LLRs must
//     be on the grid, which they are for the QMS channel; a pack with an off-grid or
//     out-of-range value is flagged in `bad` and decoded by the v5 kernel instead: exact for
//     any input)
//   C->V message: negative flag + 4 magnitude planes, derived from the check record
//     {q1, q2 (weighted quantized minima), idx (argmin edge), ns[k] (message k negative)}
//   Tv = clamp(Q(beta_{t+1} ch) + S, [-32, 31]): 6 planes, two's complement (any bound >= 2 qmax
//     gives the reference's V->C = clamp(Tv - C->V, +-qmax))
//   S = sum of C->V over the variable's edges: SB planes, two's complement
// A variable record in LDS is 16 words: Tv planes 0..5, channel sign 8, magnitude 9..12.
// A check record is 12 + DMAX words: q1 0..3, q2 4..7, idx 8..11, ns 12..12+DMAX-1.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldpc_fused.h"
#include "ldpc_fused5_kernel.h"

namespace ldpc {
namespace bs {

constexpr int PACK = 32;                 // codewords per workgroup
constexpr int VREC_W = 16;               // words per variable record
constexpr int VREC_B = VREC_W * 4;
constexpr int LUT_W = 64;                // words per 16-entry table: [bit j][pair p] {X, Y}
constexpr int QMAX = 15;
constexpr size_t BS_LDS_MAX = 160 * 1024;

struct BsArgs {
    const float* llr;
    int64_t B;
    int n_vars, n_checks, N, M, T, target_bits;
    float inv;
    const uint32_t* cn_addr;     // [n_checks][DMAX/2] VREC byte addresses, two per word
    const uint32_t* cn_row;      // [n_checks] proto row
    const uint32_t* vn_edges;    // [n_vars][dvmax] CREC byte address | k << 16 (zero record if unused)
    int dvmax;
    const uint32_t* alut;        // [T][M][LUT_W] alpha tables, Q(relu(alpha m step)) for m = 0..15
    const uint32_t* blut;        // [T][N][LUT_W] beta tables, Q(beta m) for m = 0..15 (grid units)
    int64_t* counters;
    uint8_t* flags;
    uint32_t* bad;               // [blocks] 1: decoded by the v5 fixup instead
    uint32_t off_crec, off_alut, off_blut, off_red, off_stage;   // LDS byte offsets
    int crec_w;                  // words per check record
    int arows, bcols;            // tables per iteration: 1 (one weight for all rows / columns) or M / N
};

// ---- bit-plane arithmetic (the compiler maps these 3-input functions to v_bitop3_b32) ---------
__device__ __forceinline__ uint32_t maj3(uint32_t a, uint32_t b, uint32_t c) { return (a & b) | (a & c) | (b & c); }
__device__ __forceinline__ uint32_t mux(uint32_t s, uint32_t a, uint32_t b) { return (s & a) | (~s & b); }  // s ? a : b

// S + m for m given as (negative flag n, 4 magnitude planes M): two's complement, SB planes
template <int SB>
__device__ __forceinline__ void add_sm(uint32_t (&S)[SB], const uint32_t (&M)[4], uint32_t n) {
    uint32_t c = n;
#pragma unroll
    for (int i = 0; i < SB; ++i) {
        const uint32_t b = (i < 4) ? (M[i] ^ n) : n;
        const uint32_t s = S[i] ^ b ^ c;
        if (i + 1 < SB) c = maj3(S[i], b, c);
        S[i] = s;
    }
}

// V->C before the clamp: x = Tv - m (7 planes, two's complement; Tv in [-32, 31], |m| <= 15)
__device__ __forceinline__ void sub_tv(uint32_t (&x)[7], const uint32_t (&T)[6], const uint32_t (&M)[4],
                                       uint32_t n) {
    const uint32_t p = ~n;          // m >= 0: add ~M + 1 (subtract); m < 0: add M
    uint32_t c = p;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
        const uint32_t t = T[i < 6 ? i : 5];
        const uint32_t b = (i < 4) ? (M[i] ^ p) : p;
        x[i] = t ^ b ^ c;
        if (i < 6) c = maj3(t, b, c);
    }
}

// |x| saturated at 15 (4 planes) for x in 7-plane two's complement; sign = x[6]
__device__ __forceinline__ void abs_sat(uint32_t (&X)[4], const uint32_t (&x)[7]) {
    const uint32_t neg = x[6];
    uint32_t c = neg, r[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const uint32_t y = x[i] ^ neg;
        r[i] = y ^ c;
        if (i < 5) c = y & c;
    }
    const uint32_t hi = r[4] | r[5];
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = r[i] | hi;
}

// a < b for 4-plane unsigned values
__device__ __forceinline__ uint32_t lt4(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
    uint32_t l = ~a[0] & b[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) l = (~a[i] & b[i]) | (~(a[i] ^ b[i]) & l);
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
    for (int i = 0; i < 5; ++i) T[i] = mux(ovf, ~s, v[i]);
    T[5] = mux(ovf, s, v[5]);
}

// LDS accesses by byte address (all records and tables are LDS-absolute: the kernel's dynamic
// LDS starts at 0, checked at entry)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint32_t LdsW;
typedef __attribute__((address_space(3))) v4u LdsQ;
typedef __attribute__((address_space(3))) v2u LdsD;

__device__ __forceinline__ uint32_t lds_w(uint32_t addr) { return *reinterpret_cast<const LdsW*>(addr); }
__device__ __forceinline__ v4u lds_q(uint32_t addr) { return *reinterpret_cast<const LdsQ*>(addr); }
__device__ __forceinline__ void st_q(uint32_t addr, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    v4u v = {x, y, z, w};
    *reinterpret_cast<LdsQ*>(addr) = v;
}
__device__ __forceinline__ void st_d(uint32_t addr, uint32_t x, uint32_t y) {
    v2u v = {x, y};
    *reinterpret_cast<LdsD*>(addr) = v;
}

// the Tv planes of the variable record at `addr`
__device__ __forceinline__ void read_tv(uint32_t (&T)[6], uint32_t addr) {
    const v4u a = lds_q(addr);
    const v2u b = *reinterpret_cast<const LdsD*>(addr + 16);
    T[0] = a.x; T[1] = a.y; T[2] = a.z; T[3] = a.w; T[4] = b.x; T[5] = b.y;
}

// 16-entry table g(m) (4 -> 4 bits) at LDS byte address `tab`, for two inputs at once
__device__ __forceinline__ void lut2(uint32_t (&oa)[4], uint32_t (&ob)[4], const uint32_t (&a)[4],
                                     const uint32_t (&b)[4], uint32_t tab) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t xy[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u w = lds_q(tab + (uint32_t)(j * 64 + q * 16));
            xy[4 * q] = w.x; xy[4 * q + 1] = w.y; xy[4 * q + 2] = w.z; xy[4 * q + 3] = w.w;
        }
        uint32_t ga[8], gb[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            ga[p] = (a[0] & xy[2 * p]) ^ xy[2 * p + 1];
            gb[p] = (b[0] & xy[2 * p]) ^ xy[2 * p + 1];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ga[q] = mux(a[1], ga[2 * q + 1], ga[2 * q]);
            gb[q] = mux(b[1], gb[2 * q + 1], gb[2 * q]);
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            ga[r] = mux(a[2], ga[2 * r + 1], ga[2 * r]);
            gb[r] = mux(b[2], gb[2 * r + 1], gb[2 * r]);
        }
        oa[j] = mux(a[3], ga[1], ga[0]);
        ob[j] = mux(b[3], gb[1], gb[0]);
    }
}

__device__ __forceinline__ void lut1(uint32_t (&oa)[4], const uint32_t (&a)[4], uint32_t tab) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t xy[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const v4u w = lds_q(tab + (uint32_t)(j * 64 + q * 16));
            xy[4 * q] = w.x; xy[4 * q + 1] = w.y; xy[4 * q + 2] = w.z; xy[4 * q + 3] = w.w;
        }
        uint32_t g[8];
#pragma unroll
        for (int p = 0; p < 8; ++p) g[p] = (a[0] & xy[2 * p]) ^ xy[2 * p + 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = mux(a[1], g[2 * q + 1], g[2 * q]);
#pragma unroll
        for (int r = 0; r < 2; ++r) g[r] = mux(a[2], g[2 * r + 1], g[2 * r]);
        oa[j] = mux(a[3], g[1], g[0]);
    }
}



#ifndef BS_WPE
#define BS_WPE 4
#endif
template <int DMAX, int SB>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(BS_WPE)))
k_bs(BsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if ((uint32_t)(uintptr_t)smem != 0u) __builtin_trap();          // records are LDS-absolute
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int nwv = NT >> 6;
    const int nv = a.n_vars;
    const int z = nv / a.N;
    const int64_t b0 = (int64_t)blockIdx.x * PACK;
    const int nvalid = (int)min<int64_t>(PACK, a.B - b0);
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);   // [0] wrong_t, [1] all t, [2] APP > 0, [3] bits
    const uint32_t crec = a.off_crec;
    const int CW = a.crec_w;
    const int AL = a.arows * LUT_W, BL = a.bcols * LUT_W;
    LdsW* ALUT = reinterpret_cast<LdsW*>(a.off_alut);   // [2][arows][LUT_W]
    LdsW* BLUT = reinterpret_cast<LdsW*>(a.off_blut);   // [2][bcols][LUT_W]

    // ---- prologue: LLRs -> grid integers (int8 staging, coalesced along each codeword) -------
    signed char* STG = reinterpret_cast<signed char*>(smem + a.off_stage);   // [32][nv]
    if (tid == 0) RED[7] = 0u;             // "some LLR of the pack is off the grid" (RED is past STG)
    __syncthreads();
    int off = 0;
    for (int e = tid; e < PACK * nv; e += NT) {
        const int r = e / nv, v = e - r * nv;
        int xi = 0;
        if (r < nvalid) {
            const float x = a.llr[(b0 + r) * nv + v] * a.inv;
            const float xr = rintf(x);
            off |= (xr != x || fabsf(xr) > (float)QMAX) ? 1 : 0;
            xi = (int)xr;
        }
        STG[e] = (signed char)xi;
    }
    if (off) atomicOr(&RED[7], 1u);
    __syncthreads();
    if (RED[7]) {                             // off the grid: the v5 fixup decodes this pack
        if (tid == 0) a.bad[blockIdx.x] = 1u;
        return;
    }
    if (tid == 0) a.bad[blockIdx.x] = 0u;
    // channel planes by ballot: lanes 0..31 = codewords of variable v, 32..63 of v + 1
    {
        const int r = lane & 31, half = lane >> 5;
        for (int base = 2 * wave; base < nv; base += 2 * nwv) {
            const int v = base + half;
            const int x = (v < nv) ? (int)STG[r * nv + v] : 0;
            const int m = x < 0 ? -x : x;
            const uint64_t bs = __ballot(x < 0);
            const uint64_t c0 = __ballot(m & 1), c1 = __ballot(m & 2), c2 = __ballot(m & 4),
                           c3 = __ballot(m & 8);
            if (r == 0 && v < nv) {
                const int sh = 32 * half;
                const uint32_t rec = (uint32_t)(v * VREC_B);
                st_q(rec + 32, (uint32_t)(bs >> sh), (uint32_t)(c0 >> sh), (uint32_t)(c1 >> sh),
                               (uint32_t)(c2 >> sh));
                reinterpret_cast<LdsW*>(rec + 48)[0] = (uint32_t)(c3 >> sh);
            }
        }
    }
    __syncthreads();
    // zero check records (+ the zero record at n_checks), dummy variable record Tv = -32,
    // counters, iteration 0's tables
    for (int w = tid; w < (a.n_checks + 1) * CW; w += NT) reinterpret_cast<LdsW*>(crec)[w] = 0u;
    if (tid < 16) reinterpret_cast<LdsW*>((uint32_t)(nv * VREC_B))[tid] = (tid == 5) ? 0xFFFFFFFFu : 0u;
    if (tid < 7) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
    for (int w = tid; w < AL; w += NT) ALUT[w] = a.alut[w];
    for (int w = tid; w < BL; w += NT) BLUT[w] = a.blut[w];
    __syncthreads();
    // Tv_0 = Q(beta_0 ch): the table gives the magnitude, the channel sign the sign
    for (int v = tid; v < nv; v += NT) {
        const uint32_t rec = (uint32_t)(v * VREC_B);
        const v4u cq = lds_q(rec + 32);
        const uint32_t cm[4] = {cq.y, cq.z, cq.w, lds_w(rec + 48)};
        uint32_t lw[4];
        lut1(lw, cm, a.off_blut + (uint32_t)((a.bcols > 1 ? v / z : 0) * LUT_W * 4));
        uint32_t S[SB];
#pragma unroll
        for (int i = 0; i < SB; ++i) S[i] = 0u;
        add_sm<SB>(S, lw, cq.x);
        uint32_t T[6];
        clamp6<SB>(T, S);
        st_q(rec, T[0], T[1], T[2], T[3]);
        st_d(rec + 16, T[4], T[5]);
    }
    // per-lane graph tables (one check per lane: checked on the host)
    uint32_t pk[DMAX / 2];
    uint32_t tab_a = a.off_alut;
    const bool is_check = tid < a.n_checks;
    if (is_check) {
#pragma unroll
        for (int p = 0; p < DMAX / 2; ++p) pk[p] = a.cn_addr[(size_t)tid * (DMAX / 2) + p];
        if (a.arows > 1) tab_a += a.cn_row[tid] * (LUT_W * 4);
    }
    __syncthreads();

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {            // fold iteration t-1's frame flags
            RED[1] &= RED[0];
            RED[0] = 0u;
        }
        const int nx = (t + 1) & 1;
        // beta_{t+1} for this iteration's variable phase (its slot was last read two phases ago)
        if (t + 1 < a.T)
            for (int w = tid; w < BL; w += NT) BLUT[nx * BL + w] = a.blut[(size_t)(t + 1) * BL + w];
        // ======== check nodes ===================================================================
        if (is_check) {
            const uint32_t rec = crec + (uint32_t)(tid * CW * 4);
            const v4u q1v = lds_q(rec), q2v = lds_q(rec + 16), ixv = lds_q(rec + 32);
            const uint32_t q1[4] = {q1v.x, q1v.y, q1v.z, q1v.w};
            const uint32_t q2[4] = {q2v.x, q2v.y, q2v.z, q2v.w};
            const uint32_t ix[4] = {ixv.x, ixv.y, ixv.z, ixv.w};
            uint32_t m1[4] = {~0u, ~0u, ~0u, ~0u}, m2[4] = {~0u, ~0u, ~0u, ~0u};
            uint32_t id[4] = {0u, 0u, 0u, 0u};
            uint32_t pos[DMAX];
#pragma unroll
            for (int k = 0; k < DMAX; ++k) {
                const uint32_t addr = (k & 1) ? (pk[k >> 1] >> 16) : (pk[k >> 1] & 0xFFFFu);
                uint32_t T[6];
                read_tv(T, addr);
                // old message of edge k: magnitude q2 at the argmin edge, else q1
                uint32_t am = ~0u;
#pragma unroll
                for (int i = 0; i < 4; ++i) am &= ((k >> i) & 1) ? ix[i] : ~ix[i];
                const uint32_t ns = lds_w(rec + 48 + 4 * k);
                uint32_t Mg[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) Mg[i] = mux(am, q2[i], q1[i]);
                uint32_t x[7], X[4];
                sub_tv(x, T, Mg, ns);
                abs_sat(X, x);
                pos[k] = ~x[6];                                 // V->C >= 0 (the nudged zero too)
                const uint32_t l1 = lt4(X, m1), l2 = lt4(X, m2);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    m2[i] = mux(l1, m1[i], mux(l2, X[i], m2[i]));
                    m1[i] = mux(l1, X[i], m1[i]);
                    id[i] = ((k >> i) & 1) ? (id[i] | l1) : (id[i] & ~l1);
                }
            }
            uint32_t par = 0u;
#pragma unroll
            for (int k = 0; k < DMAX; ++k) par ^= pos[k];
            uint32_t q1n[4], q2n[4];
            lut2(q1n, q2n, m1, m2, tab_a + (uint32_t)((t & 1) * AL * 4));
            st_q(rec, q1n[0], q1n[1], q1n[2], q1n[3]);
            st_q(rec + 16, q2n[0], q2n[1], q2n[2], q2n[3]);
            st_q(rec + 32, id[0], id[1], id[2], id[3]);
            // message k negative iff an even number of the OTHER edges have V->C >= 0
            // (Main_Functions.py:251-254: sgn = -prod(1 - 2 [v2c < 0]) ... o = m * sign(sgn))
#pragma unroll
            for (int k = 0; k < DMAX; k += 4)
                st_q(rec + 48 + 4 * k, ~(par ^ pos[k]), ~(par ^ pos[k + 1]), ~(par ^ pos[k + 2]),
                               ~(par ^ pos[k + 3]));
        }
        __syncthreads();
        const bool last = (t == a.T - 1);
        // alpha_{t+1} for the next check phase (slot last read by the check phase of t - 1)
        if (t + 1 < a.T)
            for (int w = tid; w < AL; w += NT) ALUT[nx * AL + w] = a.alut[(size_t)(t + 1) * AL + w];
        // ======== variable nodes ================================================================
        uint32_t wr = 0u, apos = 0u, nb = 0u;
        for (int v = tid; v < nv; v += NT) {
            const uint32_t vrec = (uint32_t)(v * VREC_B);
            uint32_t S[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) S[i] = 0u;
            for (int e = 0; e < a.dvmax; ++e) {
                const uint32_t ed = a.vn_edges[(size_t)v * a.dvmax + e];
                const uint32_t r = crec + (ed & 0xFFFFu);
                const uint32_t k = ed >> 16;
                const v4u q1v = lds_q(r), q2v = lds_q(r + 16), ixv = lds_q(r + 32);
                const uint32_t ns = lds_w(r + 48 + 4 * k);
                const uint32_t k0 = 0u - (k & 1u), k1 = 0u - ((k >> 1) & 1u), k2 = 0u - ((k >> 2) & 1u),
                               k3 = 0u - ((k >> 3) & 1u);
                const uint32_t am = ~((ixv.x ^ k0) | (ixv.y ^ k1) | (ixv.z ^ k2) | (ixv.w ^ k3));
                const uint32_t Mg[4] = {mux(am, q2v.x, q1v.x), mux(am, q2v.y, q1v.y),
                                        mux(am, q2v.z, q1v.z), mux(am, q2v.w, q1v.w)};
                add_sm<SB>(S, Mg, ns);
            }
            const v4u cq = lds_q(vrec + 32);
            const uint32_t cs = cq.x;
            const uint32_t cm[4] = {cq.y, cq.z, cq.w, lds_w(vrec + 48)};
            // APP_t = clip(Q(ch) + S, +-clip_LLR): its sign and zero-ness are all the counters need
            uint32_t A[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) A[i] = S[i];
            add_sm<SB>(A, cm, cs);
            const uint32_t hd = ~A[SB - 1] & valid;          // APP >= 0 -> hard decision 1
            if (v < a.target_bits) {
                wr |= hd;
                if (last) {
                    uint32_t nz = 0u;
#pragma unroll
                    for (int i = 0; i < SB; ++i) nz |= A[i];
                    apos |= hd & nz;
                    nb += (uint32_t)__popc(hd);
                }
            }
            if (!last) {          // Tv_{t+1} = clamp(Q(beta_{t+1} ch) + S_{t+1})
                uint32_t lw[4];
                lut1(lw, cm, a.off_blut + (uint32_t)((nx * BL + (a.bcols > 1 ? v / z : 0) * LUT_W) * 4));
                add_sm<SB>(S, lw, cs);
                uint32_t T[6];
                clamp6<SB>(T, S);
                st_q(vrec, T[0], T[1], T[2], T[3]);
                st_d(vrec + 16, T[4], T[5]);
            }
        }
        // reductions over the block
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            wr |= __shfl_xor(wr, o);
            if (last) {
                apos |= __shfl_xor(apos, o);
                nb += __shfl_xor(nb, o);
            }
        }
        if (lane == 0) {
            if (wr) atomicOr(&RED[0], wr);
            if (last) {
                if (apos) atomicOr(&RED[2], apos);
                if (nb) atomicAdd(&RED[3], nb);
            }
        }
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
//   beta:  g(m) = Q(fl32(m * beta_{t,col})) in grid units (lw = Q(beta ch), :164-177)
__global__ void k_bs_tables(const float* __restrict__ alpha, const float* __restrict__ beta,
                            const int32_t* __restrict__ row_ptr, int T, int E, int N, int z,
                            int arows, int bcols, float step, float inv, uint32_t* alut,
                            uint32_t* blut) {
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
            g[m] = q < 0 ? -q : q;       // beta >= 0 in practice; the sign comes from the channel
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
struct BsPlan {
    bool ok = false;
    int nw = 0, dmax = 16, sb = 8, dvmax = 0, crec_w = 0, arows = 1, bcols = 1;
    uint32_t off_crec = 0, off_alut = 0, off_blut = 0, off_red = 0, off_stage = 0;
    size_t lds = 0;
};

static int bits_for(int maxabs) {        // two's complement planes holding [-maxabs, maxabs]
    int b = 1;
    while ((1 << (b - 1)) - 1 < maxabs) ++b;
    return b;
}

BsPlan bs_plan(const DevGraph& g, int mode, bool ucn, bool per_edge_w, bool arow_uniform,
               bool bcol_uniform) {
    BsPlan p;
    const char* e = getenv("LDPC_BS");
    if (e && atoi(e) == 0) return p;
    if (mode != MODE_Q5 && mode != MODE_QM5) return p;           // qmax 15: 4 magnitude planes
    if (ucn || per_edge_w || !g.host) return p;
    const host::GraphTables& h = *g.host;
    int min_cdeg = 1 << 30;
    for (int i = 0; i < h.M; ++i) min_cdeg = std::min(min_cdeg, h.row_ptr[i + 1] - h.row_ptr[i]);
    if (h.max_cdeg > 16 || min_cdeg < 2) return p;               // ("no other edge" rule unneeded)
    const int nv = g.n_vars, nc = g.n_checks;
    p.nw = std::min(16, (std::max(nv, nc) + 63) / 64);
    if (nc > 64 * p.nw) return p;                                 // one check per lane
    if ((size_t)(nv + 1) * VREC_B > 65535) return p;              // 16-bit record addresses
    p.sb = bits_for(h.max_vdeg * QMAX + QMAX);
    if (p.sb != 8 && p.sb != 10) p.sb = (p.sb < 8) ? 8 : (p.sb <= 10 ? 10 : 0);
    if (p.sb == 0) return p;
    p.dvmax = h.max_vdeg;
    p.crec_w = 12 + p.dmax;
    p.arows = arow_uniform ? 1 : h.M;
    p.bcols = bcol_uniform ? 1 : h.N;
    size_t o = (size_t)(nv + 1) * VREC_B;
    p.off_crec = (uint32_t)o;
    o += (size_t)(nc + 1) * p.crec_w * 4;
    if (o > 65535) return p;                                      // 16-bit check record addresses
    p.off_alut = (uint32_t)o;
    o += (size_t)2 * p.arows * LUT_W * 4;
    p.off_blut = (uint32_t)o;
    o += (size_t)2 * p.bcols * LUT_W * 4;
    // int8 staging of the LLR block: over the check records and tables (used before them);
    // the counters (RED) after both, since the prologue uses RED[7] while staging
    p.off_stage = p.off_crec;
    o = std::max(o, (size_t)p.off_stage + (size_t)PACK * nv);
    o = (o + 15) & ~(size_t)15;
    p.off_red = (uint32_t)o;
    o += 64;
    p.lds = (o + 15) & ~(size_t)15;
    if (p.lds > BS_LDS_MAX) return p;
    p.ok = true;
    return p;
}

}  // namespace bs

using namespace bs;

bool bs_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    return bs_plan(g, mode, ucn, per_edge_w, true, true).ok;
}

const char* bs_kernel_name(const DevGraph& g) {
    static thread_local char buf[48];
    const BsPlan p = bs_plan(g, MODE_Q5, false, false, true, true);
    snprintf(buf, sizeof(buf), "bsl[p32,w%d,s%d]", p.nw, p.sb);
    return buf;
}

// graph tables, built once per context on the host (ws.bs_graph)
static int bs_graph_tables(const DevGraph& g, const BsPlan& p, FusedWorkspace& ws, hipStream_t s) {
    if (ws.bs_graph) return LDPC_OK;
    const host::GraphTables& h = *g.host;
    const int nv = g.n_vars, nc = g.n_checks, z = g.z;
    const int npk = p.dmax / 2;
    std::vector<uint32_t> tab;
    tab.reserve((size_t)nc * npk + nc + (size_t)nv * p.dvmax);
    // cn_addr: VREC byte address of each edge's variable, the dummy record past the degree
    std::vector<int> kpos((size_t)nv * p.dvmax, -1);
    std::vector<int> kchk((size_t)nv * p.dvmax, -1);
    std::vector<int> nfill(nv, 0);
    for (int c = 0; c < nc; ++c) {
        const int i = c / z, hh = c - i * z, r0 = h.row_ptr[i], deg = h.row_ptr[i + 1] - r0;
        for (int q = 0; q < npk; ++q) {
            uint32_t w = 0;
            for (int j = 0; j < 2; ++j) {
                const int k = 2 * q + j;
                uint32_t addr = (uint32_t)(nv * VREC_B);
                if (k < deg) {
                    int sh = hh + h.pe_shift[r0 + k];
                    sh = sh >= z ? sh - z : sh;
                    const int v = h.pe_col[r0 + k] * z + sh;
                    addr = (uint32_t)(v * VREC_B);
                    const int f = nfill[v]++;
                    kpos[(size_t)v * p.dvmax + f] = k;
                    kchk[(size_t)v * p.dvmax + f] = c;
                }
                w |= addr << (16 * j);
            }
            tab.push_back(w);
        }
    }
    for (int c = 0; c < nc; ++c) tab.push_back((uint32_t)(c / z));
    // vn_edges: check record offset (from the CREC base) | position k << 16; unused slots read the
    // zero record at n_checks (a zero message)
    for (int v = 0; v < nv; ++v)
        for (int f = 0; f < p.dvmax; ++f) {
            const int c = kchk[(size_t)v * p.dvmax + f];
            const uint32_t rec = (uint32_t)((c >= 0 ? c : nc) * p.crec_w * 4);
            tab.push_back(rec | ((uint32_t)(c >= 0 ? kpos[(size_t)v * p.dvmax + f] : 0) << 16));
        }
    void* d = nullptr;
    if (hipMalloc(&d, tab.size() * 4) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
    if (hipMemcpyAsync(d, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(d);
        return LDPC_ERR_HIP;
    }
    ws.bs_graph = d;
    return LDPC_OK;
}

template <int DMAX, int SB>
static int launch_bs(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_bs<DMAX, SB>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)BS_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_bs<DMAX, SB>), dim3(nblocks), dim3(64 * nw), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

int bs_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
              bool arow_uniform, bool bcol_uniform, int64_t* counters, uint8_t* flags,
              uint32_t* bad, hipStream_t s) {
    const BsPlan p = bs_plan(g, mode, false, false, arow_uniform, bcol_uniform);
    if (!p.ok) return LDPC_ERR_UNSUPPORTED;
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
                       b.beta, g.row_ptr, b.T, g.E, g.N, g.z, p.arows, p.bcols, step, 1.0f / step,
                       alut, blut);
    if (hipGetLastError() != hipSuccess) return LDPC_ERR_HIP;
    const uint32_t* gt = reinterpret_cast<const uint32_t*>(ws.bs_graph);
    BsArgs a{};
    a.llr = llr;
    a.B = b.B;
    a.n_vars = g.n_vars;
    a.n_checks = g.n_checks;
    a.N = g.N;
    a.M = g.M;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.inv = 1.0f / step;
    a.cn_addr = gt;
    a.cn_row = gt + (size_t)g.n_checks * (p.dmax / 2);
    a.vn_edges = a.cn_row + g.n_checks;
    a.dvmax = p.dvmax;
    a.alut = alut;
    a.blut = blut;
    a.counters = counters;
    a.flags = flags;
    a.bad = bad;
    a.off_crec = p.off_crec;
    a.off_alut = p.off_alut;
    a.off_blut = p.off_blut;
    a.off_red = p.off_red;
    a.off_stage = p.off_stage;
    a.crec_w = p.crec_w;
    a.arows = p.arows;
    a.bcols = p.bcols;
    const int nblocks = (int)((b.B + PACK - 1) / PACK);
    if (p.sb == 8) return launch_bs<16, 8>(a, nblocks, p.nw, p.lds, s);
    return launch_bs<16, 10>(a, nblocks, p.nw, p.lds, s);
}

}  // namespace ldpc
