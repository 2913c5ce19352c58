// ldpc_bsc.hip — bit-sliced fused QMS decoder with COMPRESSED check messages ("bsc"), for the
// graphs whose one-slot-per-edge state (ldpc_bs_kernel.h: 20 B per lifted edge and pack) does
// not fit the 160 KB of LDS — 5G NR BG1 n2112 (C5: 8,784 edges = 176 KB).
//
// Same arithmetic and semantics as the bsl kernel (32 codewords per 32-bit word, one pack per
// workgroup, Main_Functions.py:157-335 in units of the q-bit grid) with a different state
// split (LDS per pack, BG1: 151 KB):
//   TV[v][6]      Tv = clamp(Q(beta ch) + S, [-32, 31]) per variable (6 two's-complement planes)
//   REC[c][8]     the check's two possible C->V magnitudes: q1 (every edge whose |V->C| is not
//                 the minimum) and q2 (those that are), 4 planes each
//   SGN[e], ARG[e] per edge: the C->V sign (parity ^ own V->C sign) and [|V->C| == minimum]
// so the check phase recomputes V->C = clamp(Tv - C->V_old, +-15) from Tv and its own previous
// message (instead of the variable phase writing it per edge), and the variable phase reads
// each edge's C->V as (SGN, ARG ? q2 : q1) from the check's record.  The check side keeps the
// bsl structure (LPC lanes per check, quad DPP merges, alpha table by mux tree); the variable
// side needs no per-edge write-back.  Variable lanes hold several variables (VPL) and check
// lanes several 64-lane chunks (CPL), one 16-wave workgroup per CU.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "ldpc_bs_kernel.h"

// the variable places' edge words not made opaque per use (bsl's BS_VAO; A/B switch, off: the C5
// build then spills 16-17 VGPRs instead of 7)
#ifndef BSC_TOPO
#define BSC_TOPO 0     // the loop-top copies' bounds opaque per iteration (A/B switch: C5 46.37
                       // against 46.34 ms, profiles/r6/session_r6y.log; off)
#endif
#ifndef BSC_VAO
#define BSC_VAO 0
#endif

namespace ldpc {
namespace bs {

// the variable phase at the fewest planes of S for each place's largest degree (bsl's BS_SBV;
// A/B switch)
#ifndef BSC_SBV
#define BSC_SBV 1
#endif
#ifndef BSC_SBV_SET
#define BSC_SBV_SET 3   // the lower plane counts that get a copy: 1 seven, 2 eight (A/B)
#endif

// instances: D = check-degree bound, DVH / DVL = variable-degree bound of a lane's first /
// other variables, LPC lanes per check, VPL variables and CPL check chunks per lane
// (a wman-sized instance — one variable and one check chunk per lane, 64 VGPRs — was measured
// against bsl on C2: 61 spills, and the BG1 instance there ran 68 M cw/s against bsl's 176 M)
// MIX: rows of degree <= LPC / 2 * EPL take LPC / 2 lanes per check (their own 64-lane chunks,
// after the LPC-lane ones): one lane merge and one more table bit per lane instead of two
// merges and twice the lanes, for the low-degree rows
struct BscInst { int D, DVH, DVL, LPC, VPL, CPL; int WPE; int NW = 16; bool MIX = false; };
constexpr BscInst kBscInst[] = {
    {20, 10, 5, 4, 3, 3, 4},          // 5G BG1 (C5): degree 19 rows, degree 10 / 8 columns, 16 waves
    {20, 10, 5, 2, 3, 2, 4},          // the same with 2 lanes per check (LDPC_BS_LPC A/B)
    // 12 waves: 36 variable chunks on 36 places, 45 check chunks on 48, up to 168 VGPRs (the
    // 16-wave build spills 25 VGPRs at 128): LDPC_BSC_INST=2 A/B
    {20, 10, 5, 4, 3, 4, 3, 12},
    // mixed lanes per check (5G BG1: four degree-19 rows at 4 lanes, six of degree 3-10 at 2)
    {20, 10, 5, 4, 3, 3, 4, 16, true},
    {20, 10, 5, 4, 3, 2, 4, 16, true},
};

struct BscArgs {
    const float* llr;            // (Q8 builds: unused, the channel is generated, as bsl's)
    int64_t B;
    int n_vars, n_checks, T, target_bits, cn_dmin, z;
    float inv, cu;
    int qmax;                    // the grid's largest magnitude in grid units (15, 7 or 3)
    int beta_id;                 // every beta is 1: Q(beta ch) = ch, no table
    const int32_t* row_ptr;
    const int32_t* row_lay;      // [M][2] slot layout (as bsl): first slot, j-block stride
    const uint32_t* vn_tab;      // [VPL][64 nw][DVH + 1]: per edge slot | (record offset / 16) << 16, variable
    const int32_t* vn_wdeg;      // [VPL][nw][2]
    const int32_t* cn_chunk;     // [nw][CPL]
    const uint32_t* cn_var;      // [chunks * 64][CVW] variables of the lane's edges (16-bit packed)
    const int32_t* cn_lane;      // MIX: [chunks * 64] check | lane << 16 | lanes per check << 20, -1 idle
    const uint32_t* alut;        // [T][arows][LUT_W]
    const uint32_t* blut;        // [T][bcols][BLUT_W]
    int arows, bcols;
    const int32_t* atid;         // one alpha per iteration (arows 1): [T] kBetaTab index of its
                                 // table (-1: not in the set), or null
    int64_t* counters;
    uint8_t* flags;
    uint32_t* bad;
    uint32_t* iter_wrong;        // [T][packs] per-iteration frame-error words, or null
    int stagger, stagger_n;      // start offsets of workgroups 0 .. stagger_n - 1 (the first
                                 // generation, one per CU), spread over 0 .. stagger x 512 clocks
    uint32_t* hdx;               // XP builds: [T][packs][n_vars] hard decisions (as bsl's)
    uint32_t off_a, off_rec, off_tv, off_red, off_alut, off_blut;   // SGN at LDS byte 0
                                 // (RED: 16 words, then T words: iteration t's frame-error word)
    BsGen gen;                   // Q8 builds: the in-prologue channel (bsl's; tables at SGN)
};

typedef unsigned int v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void lds_qput(uint32_t addr, const uint32_t (&x)[4]) {
    v4u v;
    v.x = x[0];
    v.y = x[1];
    v.z = x[2];
    v.w = x[3];
    *reinterpret_cast<LdsQ*>(addr) = v;
}
// the fixed-table check weighting for one alpha per iteration (A/B switch, off: C5 62.7 ms with
// it against 59.6 without, same box (r3i), and 62.8 with it compiled in but turned off at run
// time (LDPC_BS_NOAFIX=1) — its 18 live operands raise the register pressure of the whole check
// phase, which costs more than the 30 table operations and 8 LDS reads it saves)
#ifndef BSC_AFIX
#define BSC_AFIX 0
#endif
// the bit-serial two minima of bsl (min2_bits) in place of the tournament and lane-group merges
// (A/B switch)
#ifndef BSC_BSMIN
#define BSC_BSMIN 1
#endif

// Check records in blocks of 16: the q1 words of records 16 b .. 16 b + 15 (256 B), then their q2
// words (256 B), so q2 is q1 + 256 (an instruction offset) and a ds_read_b128 group of 16 lanes
// on consecutive records covers 64 distinct banks (with 32-B records side by side it covered 32,
// two-way).  Byte offset of record r inside REC:
__host__ __device__ constexpr uint32_t rec_off(uint32_t r) { return ((r >> 4) << 9) + ((r & 15u) << 4); }
constexpr uint32_t REC_Q2 = 256;
typedef __attribute__((address_space(3))) v2u LdsD;
__device__ __forceinline__ v2u lds_d(uint32_t addr) { return *reinterpret_cast<const LdsD*>(addr); }
__device__ __forceinline__ void lds_dput(uint32_t addr, uint32_t x, uint32_t y) {
    v2u v;
    v.x = x;
    v.y = y;
    *reinterpret_cast<LdsD*>(addr) = v;
}

// B1: every beta is 1 and one column table (a.beta_id, bcols 1: C5's flat weights), so the
// channel term is Q(ch) itself and neither the beta table's operands nor the shortened-bit
// planes are live (C5's instance: 124 VGPRs, no spills, against 128 and 10 spilled)
template <int D, int DVH, int DVL, int LPC, int VPL, int CPL, int WPE, bool XP, int LB, bool MIX, bool B1, bool Q8>
__global__ void __launch_bounds__(LB) __attribute__((amdgpu_waves_per_eu(WPE)))
k_bsc(BscArgs a) {
    constexpr int SB = (DVH * QMAX + QMAX <= 127) ? 8 : 9;
    constexpr int EPL = (D + LPC - 1) / LPC;
    constexpr int VNW = DVH + 1;
    constexpr int CVW = (EPL + 1) / 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if ((uint32_t)(uintptr_t)smem != 0u) __builtin_trap();          // LDS-absolute addresses
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwv = NT >> 6;
    const int nv = a.n_vars;
    const int64_t b0 = (int64_t)blockIdx.x * PACK;
    const int nvalid = (int)min<int64_t>(PACK, a.B - b0);
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);
    const int flor = 16 + ((a.T + 3) & ~3);                         // (BS_FLOR) the 32 OR words
    const int AL = a.arows * LUT_W, BL = a.bcols * BLUT_W;
    uint32_t* ALUT = reinterpret_cast<uint32_t*>(smem + a.off_alut);
    uint32_t* BLUT = reinterpret_cast<uint32_t*>(smem + a.off_blut);

    // ---- per-lane variables ------------------------------------------------------------------
    uint32_t va[VPL][DVH];
    int vv[VPL], dw[VPL], dwmin[VPL];
    uint32_t tab_b[VPL];
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const int dvu = u == 0 ? DVH : DVL;
        const uint32_t* vt = a.vn_tab + ((size_t)u * NT + tid) * VNW;
#pragma unroll
        for (int p = 0; p < DVH; ++p) va[u][p] = (p < dvu) ? vt[p] : 0u;
        vv[u] = (int)vt[DVH];                                // v | Tv index << 16, or -1
        dw[u] = __builtin_amdgcn_readfirstlane(a.vn_wdeg[2 * (u * nwv + wave)]);
        dwmin[u] = __builtin_amdgcn_readfirstlane(a.vn_wdeg[2 * (u * nwv + wave) + 1]);
        tab_b[u] = (!B1 && a.bcols > 1 && vv[u] >= 0) ? (uint32_t)(((vv[u] & 0xFFFF) / (nv / a.bcols)) * BLUT_W * 4) : 0u;
    }
    (void)dwmin;

    // ---- channel planes (as bsl: shortened bits = +-cu decoded here, other off-grid packs
    // flagged for the v5 fixup) --------------------------------------------------------------
    // one workgroup per CU: the first generation starts in lockstep, and with every pack taking
    // the same time, each later generation again fetches its LLR blocks in one chip-wide burst
    // while HBM idles the rest of the pack.  Spreading the first starts over a pack's duration
    // keeps the fetches apart for the whole grid (later workgroups inherit the offsets).
    if (a.stagger > 0 && (int)blockIdx.x < a.stagger_n) {
        const int n = (int)(((uint32_t)blockIdx.x * 97u % (uint32_t)a.stagger_n) * (uint32_t)a.stagger /
                            (uint32_t)a.stagger_n);
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(8);
    }
    if (tid == 0) RED[7] = 0u;
    if constexpr (Q8) gen_tables(a.gen, tid, NT);
    __syncthreads();
    uint32_t cs[VPL], cm[VPL][4], bg[VPL];
    int off = 0;
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        cs[u] = 0u;
        bg[u] = 0u;
#pragma unroll
        for (int p = 0; p < 4; ++p) cm[u][p] = 0u;
        const int v = vv[u] < 0 ? -1 : (vv[u] & 0xFFFF);
        if (Q8 && v >= 0) {                        // generated channel (ldpc_decode_awgn), a build of its own
            uint32_t Dq[8];
            gen_bytes(a.gen, blockIdx.x, v, a.qmax, Dq);
            pack_bytes<true>(Dq, valid, cs[u], cm[u], bg[u]);
        } else if (v >= 0) {
            // (buffer loads: a wave-uniform descriptor over the pack's rows, the lane's 4 v in
            // voffset, the row's 4 r nv in soffset: no 64-bit VGPR address per load, as bsl)
            const __amdgpu_buffer_rsrc_t llr_rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(a.llr + b0 * nv), 0, nvalid * nv * 4, 0x00020000);
            float xv[PACK];
#pragma unroll
            for (int r = 0; r < PACK; ++r)
                xv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(llr_rs, 4 * v, 4 * r * nv, BS_LLR_CPOL));
            if (BS_PACKT) {
                off |= pack_channel<true>(xv, a.inv, a.qmax, a.cu, valid, cs[u], cm[u], bg[u]);
                continue;
            }
#pragma unroll
            for (int r = 0; r < PACK; ++r) {
                const float x = xv[r] * a.inv;
                const float xr = rintf(x);
                const bool big = fabsf(x) == a.cu;
                off |= ((xr != x || fabsf(xr) > (float)a.qmax) && !big) ? 1 : 0;
                const int xi = (r < nvalid) ? (big ? (x < 0.f ? -a.qmax : a.qmax) : (int)xr) : 0;
                const uint32_t m = (uint32_t)(xi < 0 ? -xi : xi);
                cs[u] |= (xi < 0 ? 1u : 0u) << r;
                bg[u] |= (big && r < nvalid ? 1u : 0u) << r;
#pragma unroll
                for (int p = 0; p < 4; ++p) cm[u][p] |= ((m >> p) & 1u) << r;
            }
        }
    }
    if (off) atomicOr(&RED[7], 1u);
    __syncthreads();
    if (RED[7]) {
        if (tid == 0) a.bad[blockIdx.x] = 1u;
        return;
    }
    if (tid == 0) a.bad[blockIdx.x] = 0u;
    // the zero edge / zero record (padding edges of the variable lanes), counters, tables
    if (tid < 8)
        reinterpret_cast<uint32_t*>(smem + a.off_rec + rec_off((uint32_t)a.n_checks) + (tid >> 2) * REC_Q2)[tid & 3] = 0u;
    if (tid < 8) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
    if (BS_FLOR && tid < BS_FLORW) RED[flor + tid] = 0u;
    for (int w = tid; w < AL; w += NT) ALUT[w] = a.alut[w];
    for (int w = tid; w < BL; w += NT) BLUT[w] = a.blut[w];
    __syncthreads();

    // ---- variable phase --------------------------------------------------------------------
    //   S = sum of the C->V (SGN, ARG ? q2 : q1), APP_t = Q(ch) + S (hard decision, counters);
    //   unless last, TV[v] = clamp(Q(beta_{t+1} ch) + S)
    auto vn_phase = [&](const bool first, const bool last, const uint32_t bslice, const int tb)
                        __attribute__((always_inline)) {
        uint32_t wr = 0u, apos = 0u, nb = 0u;
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            const int dvu = u == 0 ? DVH : DVL;
            if (BS_VSKIP && dw[u] < 0) continue;   // no variable chunk at this (wave, u) place
#pragma unroll
            for (int p = 0; p < DVH; ++p)
                if (p < dvu && !BSC_VAO) asm volatile("" : "+v"(va[u][p]));   // (as bsl's BS_VAO)
            const int v = vv[u] < 0 ? -1 : (vv[u] & 0xFFFF);
            const bool counted = v >= 0 && v < a.target_bits;
            uint32_t lw[1][4];
            if (!last) {
                if (B1 || a.beta_id) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) lw[0][i] = cm[u][i];
                } else if (a.bcols == 1) {
                    const ConstW* tg = (const ConstW*)(a.blut) + (size_t)tb * BLUT_W;
                    lut_s(lw[0], cm[u], tg);
#pragma unroll
                    for (int i = 0; i < 4; ++i) lw[0][i] = mux(bg[u], tg[LUT_W + i], lw[0][i]);
                } else {
                    const uint32_t btab = bslice + tab_b[u];
                    const uint32_t cmi[1][4] = {{cm[u][0], cm[u][1], cm[u][2], cm[u][3]}};
                    lut<1>(lw, cmi, btab);
                    const v4u gb = lds_q(btab + LUT_W * 4);
                    lw[0][0] = mux(bg[u], gb.x, lw[0][0]);
                    lw[0][1] = mux(bg[u], gb.y, lw[0][1]);
                    lw[0][2] = mux(bg[u], gb.z, lw[0][2]);
                    lw[0][3] = mux(bg[u], gb.w, lw[0][3]);
                }
            }
            const int dwu = dw[u];
            // the rest at SBX planes of S: the fewest that hold 15 dw + 15 for the place's largest
            // degree (bsl's BS_SBV; the places past the first hold at most DVL edges)
            auto vbody = [&](auto sbc) __attribute__((always_inline)) {
                constexpr int SB = decltype(sbc)::value;
                uint32_t S[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) S[i] = 0u;
                if (!first) {
#pragma unroll
                    for (int f = 0; f < DVH; ++f) {
                        if (f < dvu && f < dwu) {
                            const uint32_t wd = va[u][f];
                            const uint32_t sa = (wd & 0xFFFFu) << 2;
                            const uint32_t ra = a.off_rec + ((wd >> 16) << 4);
                            const uint32_t n = lds_w(sa), am = lds_w(sa + a.off_a);
                            const v4u q1 = lds_q(ra), q2 = lds_q(ra + REC_Q2);
                            uint32_t b[4];
                            b[0] = mux(am, q2.x, q1.x) ^ n;
                            b[1] = mux(am, q2.y, q1.y) ^ n;
                            b[2] = mux(am, q2.z, q1.z) ^ n;
                            b[3] = mux(am, q2.w, q1.w) ^ n;
                            if (f == 0) set_b<SB>(S, b, n);
                            else add_b<SB>(S, b, n);
                        }
                    }
                    uint32_t hd, nz = 0u;
                    const uint32_t c_s = cs[u];
                    if (last) {
                        uint32_t A[SB];
#pragma unroll
                        for (int i = 0; i < SB; ++i) A[i] = S[i];
                        const uint32_t cb[4] = {cm[u][0] ^ c_s, cm[u][1] ^ c_s, cm[u][2] ^ c_s, cm[u][3] ^ c_s};
                        add_b<SB>(A, cb, c_s);
                        hd = ~A[SB - 1];
#pragma unroll
                        for (int i = 0; i < SB; ++i) nz |= A[i];
                    } else {
                        uint32_t c = c_s;
#pragma unroll
                        for (int i = 0; i < SB - 1; ++i) c = B3(T_MAJ, S[i], i < 4 ? (cm[u][i] ^ c_s) : c_s, c);
                        hd = B3(T_XNOR3, S[SB - 1], c_s, c);
                    }
                    hd &= valid;
                    if constexpr (XP) {                              // iteration tb - 1's hard decisions
                        if (v >= 0) a.hdx[((size_t)(tb - 1) * (size_t)((a.B + 31) >> 5) + blockIdx.x) * nv + v] = hd;
                    }
                    if (counted) {
                        wr |= hd;
                        if (last) {
                            apos |= hd & nz;
                            nb += (uint32_t)__popc(hd);
                        }
                    }
                }
                if (last || v < 0) return;
                uint32_t lb[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) lb[i] = lw[0][i] ^ cs[u];
                add_b<SB>(S, lb, cs[u]);
                uint32_t Tv[6];
                clamp6<SB>(Tv, S);
                const uint32_t ta = a.off_tv + 24u * ((uint32_t)vv[u] >> 16);     // the Tv index
                lds_dput(ta, Tv[0], Tv[1]);
                lds_dput(ta + 8, Tv[2], Tv[3]);
                lds_dput(ta + 16, Tv[4], Tv[5]);
            };
            if constexpr (BSC_SBV) {
                auto dispatch = [&](auto smax) __attribute__((always_inline)) {
                    constexpr int SM = decltype(smax)::value;
                    if ((BSC_SBV_SET & 1) && dwu * QMAX + QMAX <= 63) vbody(std::integral_constant<int, 7>{});
                    else if ((BSC_SBV_SET & 2) && SM == 9 && dwu * QMAX + QMAX <= 127)
                        vbody(std::integral_constant<int, (SM == 9 ? 8 : SM)>{});
                    else vbody(std::integral_constant<int, SM>{});
                };
                constexpr int SBL = (DVL * QMAX + QMAX <= 127) ? 8 : 9;    // places past the first
                if (u == 0) dispatch(std::integral_constant<int, SB>{});
                else dispatch(std::integral_constant<int, SBL>{});
            } else {
                vbody(std::integral_constant<int, SB>{});
            }
        }
        if (!first && BS_FLOR && !last) {    // (bsl's BS_FLOR: one ds_or per lane into 32 words)
            const uint32_t la = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 31u;
            __hip_atomic_fetch_or(RED + flor + la, wr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (!first) {
            wr = wave_or(wr);
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
    };

    vn_phase(true, false, a.off_blut, 0);
    // check groups (as bsl): lane LPC c + j of a chunk takes edges k = LPC m + j of check c
    // (MIX: each chunk's lanes per check from its lane map; lane 0 of a chunk always holds a check)
    int gchunk[CPL], gdeg[CPL], gm[CPL], gl4[CPL];
    uint32_t gslot[CPL], grec[CPL], gtab[CPL], gvar[CPL][CVW];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        gchunk[c] = __builtin_amdgcn_readfirstlane(a.cn_chunk[wave * CPL + c]);
        const int ql = max(gchunk[c], 0) * 64 + lane;
        int cc, cjc, Lc = LPC;
        gl4[c] = 1;
        if constexpr (MIX) {
            const int32_t d = gchunk[c] >= 0 ? a.cn_lane[ql] : -1;
            cc = d < 0 ? a.n_checks : (d & 0xFFFF);
            cjc = d < 0 ? 0 : ((d >> 16) & 15);
            gl4[c] = __builtin_amdgcn_readfirstlane(d < 0 ? LPC : ((d >> 20) & 15)) == LPC ? 1 : 0;
            Lc = gl4[c] ? LPC : LPC / 2;
        } else {
            cc = ql / LPC;
            cjc = lane % LPC;
        }
        const int ci = min(cc / a.z, a.n_checks / a.z - 1);
        gdeg[c] = (cc < a.n_checks) ? a.row_ptr[ci + 1] - a.row_ptr[ci] : 0;
        // edge positions m holding a real edge for some lane of the chunk (wave-uniform): the
        // positions past them are padding for every lane and skipped (LPC, an even count, lanes
        // of each group skip together, so the group's [V->C >= 0] parity is unchanged)
        gm[c] = __popc(wave_or((1u << ((gdeg[c] + Lc - 1) / Lc)) - 1u));
        (void)nwv;
        gslot[c] = (uint32_t)(4 * (a.row_lay[2 * ci] + cjc * a.row_lay[2 * ci + 1] + (cc - ci * a.z)));
        grec[c] = a.off_rec + rec_off((uint32_t)min(cc, a.n_checks - 1));
        gtab[c] = a.off_alut + (uint32_t)((a.arows > 1 ? ci : 0) * LUT_W * 4) + (uint32_t)(cjc * (4 / Lc) * 64);
#pragma unroll
        for (int p = 0; p < CVW; ++p) gvar[c][p] = gchunk[c] >= 0 ? a.cn_var[(size_t)ql * CVW + p] : 0u;
    }
    const uint32_t sstride = (uint32_t)(4 * a.z);
    // the lane's real edge positions, one word for all its chunks: bit RB c + m = position m of
    // chunk c holds an edge of the lane's check, bit RB c + EPL = the lane holds a check.  Read
    // through an opaque copy per iteration, so [L m + j < degree] is not hoisted out of the T
    // loop as CPL x EPL x 2 64-bit lane masks, whose SGPR pairs the loop spilled and reloaded by
    // v_readlane (C5: 166 reloads in the loop body)
    constexpr int RB = EPL + 1;                  // bits per chunk
    static_assert(CPL * RB <= 32, "real-position word");
    uint32_t rpk = 0u;
    {
        const int cn_dmin = a.cn_dmin;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int L = (!MIX || gl4[c]) ? LPC : LPC / 2;
            const int cjl = lane & (L - 1);
#pragma unroll
            for (int m = 0; m < EPL; ++m)
                if (L * m + L - 1 < cn_dmin || L * m + cjl < gdeg[c]) rpk |= 1u << (RB * c + m);
            if (gdeg[c] > 0) rpk |= 1u << (RB * c + EPL);
        }
    }
    __syncthreads();

    for (int t = 0; t < a.T; ++t) {
        if (wave == 0 && t > 0) {               // (all lanes of wave 0, the same words: bsl)
            uint32_t w0;
            if (BS_FLOR) {                        // (the 32 words of iteration t - 1, zeroed again)
                const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                const uint32_t x = ln < 32u ? RED[flor + ln] : 0u;
                if (ln < 32u) RED[flor + ln] = 0u;
                w0 = wave_or(x);
            } else {
                w0 = RED[0];
                RED[0] = 0u;
            }
            RED[16 + t - 1] = w0;                     // (exported after the loop)
            RED[1] &= w0;
        }
        const int nx = (t + 1) & 1;
#pragma unroll
        for (int u = 0; u < VPL; ++u) asm volatile("" : "+s"(dw[u]));
        // (the lane's variables opaque per iteration: [v >= 0], [v < target bits] compared per
        // use, not held through the loop as spilled lane masks; BS_VVO as bsl)
        if (BS_VVO) {
#pragma unroll
            for (int u = 0; u < VPL; ++u) asm volatile("" : "+v"(vv[u]));
        }
        uint32_t rp = rpk;
        asm volatile("" : "+v"(rp));
        if (t + 1 < a.T) {
            // (the lane index made opaque per iteration: the copy addresses are recomputed here
            // rather than hoisted out of the T loop into registers the loop body spills)
            if (BS_GLDS) {            // (async global -> LDS, retired by the next barrier: bsl)
                // (BSC_TOPO: the bounds opaque per iteration, as bsl's BS_TOPO)
                int cw = wave, al = AL, bl = BL, bcl = a.bcols;
                if (BSC_TOPO) asm volatile("" : "+s"(cw), "+s"(al), "+s"(bl), "+s"(bcl));
                copy_async(a.off_alut + 4u * (uint32_t)(nx * al), a.alut + (size_t)(t + 1) * al, al, cw, NT);
                if (bcl > 1)
                    copy_async(a.off_blut + 4u * (uint32_t)(nx * bl), a.blut + (size_t)(t + 1) * bl, bl, cw, NT);
            } else {
                int tl = tid;
                asm volatile("" : "+v"(tl));
                for (int w = tl; w < AL; w += NT) ALUT[nx * AL + w] = a.alut[(size_t)(t + 1) * AL + w];
                if (a.bcols > 1)
                    for (int w = tl; w < BL; w += NT) BLUT[nx * BL + w] = a.blut[(size_t)(t + 1) * BL + w];
            }
        }
        // ======== check nodes ===================================================================
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            if (gchunk[c] < 0) continue;
            // the chunk's check work at L lanes per check (MIX: L = LPC / 2 for the low-degree rows)
            auto chunk = [&](auto LC) __attribute__((always_inline)) {
            constexpr int L = decltype(LC)::value;
            constexpr int OBL = 4 / L;
            const int cjl = lane & (L - 1);
            int gmc = gm[c];
            asm volatile("" : "+s"(gmc));
            uint32_t sbase = gslot[c];
            asm volatile("" : "+v"(sbase));
            auto real = [&](int m) __attribute__((always_inline)) -> bool {
                return ((rp >> (RB * c + m)) & 1u) != 0u;
            };
            const bool has_check = ((rp >> (RB * c + EPL)) & 1u) != 0u;
            // V->C = clamp(Tv - C->V_old, +-15) of the lane's edges (padding: negative, 15)
            v4u q1o = {0u, 0u, 0u, 0u}, q2o = {0u, 0u, 0u, 0u};
            if (t > 0) {
                q1o = lds_q(grec[c]);
                q2o = lds_q(grec[c] + REC_Q2);
            }
            uint32_t Xs[EPL][4], ns[EPL];
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                if (m >= gmc) {                      // padding for the whole chunk
#pragma unroll
                    for (int i = 0; i < 4; ++i) Xs[m][i] = ~0u;
                    ns[m] = ~0u;
                    continue;
                }
                const uint32_t vw = gvar[c][m >> 1];
                const uint32_t vi = (m & 1) ? (vw >> 16) : (vw & 0xFFFFu);
                const uint32_t ta = a.off_tv + 24u * vi;
                const v2u t01 = lds_d(ta), t23 = lds_d(ta + 8), t45 = lds_d(ta + 16);
                const uint32_t Tv[6] = {t01.x, t01.y, t23.x, t23.y, t45.x, t45.y};
                uint32_t x[7];
                if (t == 0) {
#pragma unroll
                    for (int i = 0; i < 7; ++i) x[i] = Tv[i < 6 ? i : 5];
                } else {
                    const uint32_t sa = sbase + m * sstride;
                    const uint32_t so = lds_w(sa), ao = lds_w(sa + a.off_a);
                    uint32_t bo[4];
                    bo[0] = mux(ao, q2o.x, q1o.x) ^ so;
                    bo[1] = mux(ao, q2o.y, q1o.y) ^ so;
                    bo[2] = mux(ao, q2o.z, q1o.z) ^ so;
                    bo[3] = mux(ao, q2o.w, q1o.w) ^ so;
                    sub_tv(x, Tv, bo, so);
                }
                abs_sat(Xs[m], x);
                ns[m] = x[6];
                if (!real(m)) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) Xs[m][i] = ~0u;
                    ns[m] = ~0u;
                }
            }
            // two minima by a tournament (sorted pairs merged, as bsl); positions past the chunk's
            // bound hold the all-ones padding, so a pair that straddles it sorts correctly and its
            // padding sign word, XORed by all L lanes of the group, leaves the parity unchanged
            uint32_t m1[4], m2[4];
            uint32_t cand[BSC_BSMIN ? EPL : 1];
            uint32_t par = ns[0] ^ ns[1];
            if constexpr (BSC_BSMIN) {
                // the bit-serial search of bsl (min2_bits), over the chunk's real positions
#pragma unroll
                for (int m = 2; m < EPL; ++m) par ^= ns[m];
                switch (gmc) {
#define BSC_MIN2_CASE(k)                                                                           \
    case k:                                                                                        \
        if constexpr (k <= EPL) {                                                                  \
            min2_bits<k, L>(m1, m2, cand, Xs);                                                     \
            if (BS_MIN2_Z) {                                                                       \
                _Pragma("unroll") for (int m = k; m < EPL; ++m) cand[m] = 0u;                      \
            }                                                                                      \
        } else if (BSC_MIN2_U) {                                                                   \
            __builtin_unreachable();                                                               \
        }                                                                                          \
        break;
                    BSC_MIN2_CASE(1) BSC_MIN2_CASE(2) BSC_MIN2_CASE(3) BSC_MIN2_CASE(4) BSC_MIN2_CASE(5)
                    BSC_MIN2_CASE(6) BSC_MIN2_CASE(7) BSC_MIN2_CASE(8) BSC_MIN2_CASE(9) BSC_MIN2_CASE(10)
#undef BSC_MIN2_CASE
                    default:
                        if (BSC_MIN2_U) __builtin_unreachable();  // (an active chunk: 1 <= gmc <= EPL)
                        break;
                }
                par ^= qperm<QP_X1>(par);
                if (L == 4) par ^= qperm<QP_X2>(par);
            } else {
            sort2(m1, m2, Xs[0], Xs[1]);
#pragma unroll
            for (int m = 2; m + 1 < EPL; m += 2) {
                if (m >= gmc) continue;
                uint32_t b1[4], b2[4];
                sort2(b1, b2, Xs[m], Xs[m + 1]);
                merge2(m1, m2, b1, b2);
                par ^= ns[m] ^ ns[m + 1];
            }
            if constexpr (EPL & 1) {
                if (EPL - 1 < gmc) {
                    const uint32_t(&X)[4] = Xs[EPL - 1];
                    const uint32_t l1 = lt4(X, m1), l2 = lt4(X, m2);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        m2[i] = mux(l1, m1[i], mux(l2, X[i], m2[i]));
                        m1[i] = mux(l1, X[i], m1[i]);
                    }
                    par ^= ns[EPL - 1];
                }
            }
            par ^= qperm<QP_X1>(par);
            merge_lanes<QP_X1>(m1, m2);
            if (L == 4) {
                par ^= qperm<QP_X2>(par);
                merge_lanes<QP_X2>(m1, m2);
            }
            }
            // weighted, quantized minima (Main_Functions.py:266-316).  One table of the fixed set
            // for the whole iteration (uniform alpha: C5): all 4 bits of both by immediate truth
            // tables (one entry of the jump table for all waves: no instruction-cache churn), the
            // group's first lane writes the record
            bool fixed = false;
            if (BSC_AFIX && a.atid) {
                const int k = __builtin_amdgcn_readfirstlane(a.atid[t]);
                if (k >= 0 && k < kNBetaTab) {
                    fixed = true;
                    uint32_t p1[4], p2[4];
                    table_asm2(p1, p2, m1, m2, k);
                    if (has_check && cjl == 0) {
                        lds_qput(grec[c], p1);
                        lds_qput(grec[c] + REC_Q2, p2);
                    }
                }
            }
            uint32_t qb[OBL][2];
            if (!fixed) {
                const uint32_t mm[2][4] = {{m1[0], m1[1], m1[2], m1[3]}, {m2[0], m2[1], m2[2], m2[3]}};
                const uint32_t tab = gtab[c] + (uint32_t)((t & 1) * AL * 4);
#pragma unroll
                for (int b = 0; b < OBL; ++b) {
                    uint32_t o[2];
                    lut_bit<2>(o, mm, tab + (uint32_t)(b * 64));
                    qb[b][0] = o[0];
                    qb[b][1] = o[1];
                }
            }
            // the record: lane j writes planes OBL j .. of q1 and q2 (the whole group has read the
            // old record above: same wave, LDS operations in program order); idle lanes past
            // the last check (degree 0) share its clamped record address and must not write
            if (!fixed && has_check) {
#pragma unroll
                for (int b = 0; b < OBL; ++b) {
                    lds_put(grec[c] + 4u * (uint32_t)(OBL * cjl + b), qb[b][0]);
                    lds_put(grec[c] + REC_Q2 + 4u * (uint32_t)(OBL * cjl + b), qb[b][1]);
                }
            }
            // per edge: the C->V sign (par ^ own V->C sign, :251-254) and [|V->C| == min]
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                if (real(m)) {
                    const uint32_t sa = sbase + m * sstride;
                    uint32_t eq;
                    if constexpr (BSC_BSMIN) {
                        eq = cand[m];
                    } else {
                    const uint32_t(&X)[4] = Xs[m];
                    uint32_t ne = X[0] ^ m1[0];
#pragma unroll
                    for (int i = 1; i < 4; ++i) ne = B3(T_ORXOR, ne, X[i], m1[i]);
                    eq = ~ne;
                    }
                    lds_put(sa, par ^ ns[m]);
                    lds_put(sa + a.off_a, eq);
                }
            }
                    };
            if (!MIX || gl4[c]) chunk(std::integral_constant<int, LPC>{});
            else if constexpr (MIX) chunk(std::integral_constant<int, LPC / 2>{});
        }
        __syncthreads();
        // ======== variable nodes ================================================================
        const uint32_t bslice = a.off_blut + (uint32_t)(nx * BL * 4);
        if (t == a.T - 1) vn_phase(false, true, bslice, t + 1);
        else vn_phase(false, false, bslice, t + 1);
        __syncthreads();
    }
    if (tid == 0) {
        const uint32_t wl = RED[0] & valid;
        const uint32_t all = RED[1] & RED[0] & valid;
        const uint32_t ap = RED[2] & valid;
        RED[16 + a.T - 1] = RED[0];
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
    if (a.flags || a.iter_wrong) {
        __syncthreads();
        if (a.flags && tid < nvalid)
            a.flags[b0 + tid] = (uint8_t)(((RED[5] >> tid) & 1) | (((RED[6] >> tid) & 1) << 1));
        if (a.iter_wrong)
            for (int t = tid; t < a.T; t += NT)
                a.iter_wrong[(size_t)t * (size_t)((a.B + 31) >> 5) + blockIdx.x] = RED[16 + t] & valid;
    }
}

}  // namespace bs
}  // namespace ldpc

// ---- host: planning, graph tables, launch -------------------------------------------------
namespace ldpc {
namespace bs {

std::vector<int32_t> slot_layout(const host::GraphTables& h, int LPC, size_t* nslot);
std::vector<int32_t> slot_layout_rows(const host::GraphTables& h, const std::vector<int>& rl, size_t* nslot);
std::vector<int32_t> uniform_lanes(const host::GraphTables& h, int LPC, int cn_lanes);
std::vector<int> check_chunk_cost_lanes(const host::GraphTables& h, const std::vector<int32_t>& lanes);
std::vector<int> column_rotation_lanes(const host::GraphTables& h, int EPL, const std::vector<int32_t>& lanes);
std::vector<int> deal_chunks(const std::vector<int>& cost, int nw, int cap);
std::vector<int> check_chunk_cost(const host::GraphTables& h, int LPC, int cch);
std::vector<int> column_rotation(const host::GraphTables& h, int LPC, int EPL, int cn_lanes);
void bs_stagger(bool one_per_cu, int* stagger, int* stagger_n);
int bs_make_tables(const Bufs& b, const DevGraph& g, int arows, int ar, int bcols, float step, int qmax,
                   float cu, bool ucn, FusedWorkspace& ws, uint32_t** alut, uint32_t** blut, hipStream_t s,
                   const int32_t** atid = nullptr);
bool bs_mode(int mode);
float bs_step(int mode);
int bs_qmax(int mode);

constexpr int kBscNInst = sizeof(kBscInst) / sizeof(kBscInst[0]);
constexpr int BSC_NW = 16;
constexpr int BSC_TAG = 100;     // ws.bs_graph_inst of the bsc tables: BSC_TAG + instance

struct BscPlan {
    bool ok = false;
    int inst = -1, nw = BSC_NW, cn_lanes = 0, arows = 1, bcols = 1, cn_dmin = 0;
    float cu = -1.f;
    size_t nslot = 0;
    uint32_t off_a = 0, off_rec = 0, off_tv = 0, off_red = 0, off_alut = 0, off_blut = 0;
    size_t lds = 0;
    std::vector<int32_t> lay;
    std::vector<int> vorder, vslot;      // variables by degree; chunk of each (wave, u) place
    std::vector<int> rl;                 // lanes per check of each row
    std::vector<int32_t> lanes;          // check lane -> check | lane << 16 | lanes per check << 20, -1 idle
};

static BscPlan bsc_plan(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    BscPlan p;
    const char* e = getenv("LDPC_BS");
    if (e && atoi(e) == 0) return p;
    if (!bs_mode(mode)) return p;
    if (ucn || per_edge_w || !g.host || !g.w_beta_nonneg) return p;
    const host::GraphTables& h = *g.host;
    int min_cdeg = 1 << 30;
    for (int i = 0; i < h.M; ++i) min_cdeg = std::min(min_cdeg, h.row_ptr[i + 1] - h.row_ptr[i]);
    if (min_cdeg < 2) return p;
    const int nv = g.n_vars, nc = g.n_checks, z = h.z;
    const char* el = getenv("LDPC_BS_LPC");          // A/B: force 2 or 4 lanes per check
    const int want_lpc = el ? atoi(el) : 0;
    const char* ei = getenv("LDPC_BSC_INST");        // A/B: force one instance (if it fits)
    const int want_inst = ei ? atoi(ei) : -1;
    // the mixed-lane instances first (fewest check chunks per wave first) when the decode takes
    // the beta = 1 build (every beta 1, one column table: bsc_launch's B1), where they run without
    // spills: C5 53.86 -> 52.44 ms (r3zd).  With a beta table they spill 11-19 VGPRs and issue 7 %
    // fewer VALU instructions in the same time as the uniform ones (56.24-56.43 against 56.34 ms,
    // r3w; PMC r3 mixprof): the uniform instances stay the default there.  LDPC_BSC_MIX=0/1
    // forces either.
    const char* em = getenv("LDPC_BSC_MIX");
    const bool mix = em ? atoi(em) != 0 : (g.w_beta_one && g.w_beta_uniform);
    std::vector<int> order(kBscNInst);
    for (int i = 0; i < kBscNInst; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
        const int kx = kBscInst[x].MIX == mix ? 0 : 1, ky = kBscInst[y].MIX == mix ? 0 : 1;
        if (kx != ky) return kx < ky;
        return kBscInst[x].MIX && kBscInst[x].CPL < kBscInst[y].CPL;
    });
    for (const int i : order) {
        const BscInst& k = kBscInst[i];
        if (h.max_cdeg > k.D || h.max_vdeg > k.DVH) continue;
        if (want_lpc != 0 && want_lpc != k.LPC) continue;
        if (want_inst >= 0 && want_inst != i) continue;
        if (want_inst < 0 && k.NW != BSC_NW) continue;          // A/B-only instances
        BscPlan q;
        q.inst = i;
        q.nw = k.NW;
        // rows and check lanes: MIX instances give the rows of degree <= LPC / 2 * EPL half the
        // lanes, in 64-lane chunks of their own after the full-width rows' chunks
        const int EPLk = (k.D + k.LPC - 1) / k.LPC;
        q.rl.assign((size_t)h.M, k.LPC);
        if (k.MIX)
            for (int i = 0; i < h.M; ++i)
                if (h.row_ptr[i + 1] - h.row_ptr[i] <= k.LPC / 2 * EPLk) q.rl[(size_t)i] = k.LPC / 2;
        if (k.MIX) {
            for (const int L : {k.LPC, k.LPC / 2}) {
                for (int i = 0; i < h.M; ++i) {
                    if (q.rl[(size_t)i] != L) continue;
                    for (int hc = 0; hc < z; ++hc)
                        for (int j = 0; j < L; ++j) q.lanes.push_back((i * z + hc) | (j << 16) | (L << 20));
                }
                while (q.lanes.size() % 64) q.lanes.push_back(-1);
            }
            q.cn_lanes = (int)q.lanes.size();
        } else {
            q.cn_lanes = 64 * ((k.LPC * nc + 63) / 64);
            q.lanes = uniform_lanes(h, k.LPC, q.cn_lanes);
        }
        const int vch = (nv + 63) / 64, cch = q.cn_lanes / 64;
        if (k.VPL == 1 && k.CPL == 1) q.nw = std::max(vch, cch);
        if (q.nw > 16 || vch > k.VPL * q.nw || cch > k.CPL * q.nw) continue;
        if (nv > 65535 || nc >= 65535) continue;
        // variables by descending degree in 64-chunks, dealt to (wave, u) places (the first
        // chunk of each wave, u = 0, takes the heaviest: only there may a degree exceed DVL)
        q.vorder.resize(nv);
        for (int v = 0; v < nv; ++v) q.vorder[v] = v;
        auto vdeg = [&](int v) { const int j = v / z; return h.col_ptr[j + 1] - h.col_ptr[j]; };
        std::stable_sort(q.vorder.begin(), q.vorder.end(), [&](int x, int y) { return vdeg(x) > vdeg(y); });
        std::vector<int> cost(vch);
        for (int ch = 0; ch < vch; ++ch) cost[ch] = 3 + vdeg(q.vorder[64 * ch]);
        q.vslot = deal_chunks(cost, q.nw, k.VPL);
        bool fits = true;
        for (int w = 0; w < q.nw; ++w)
            for (int u = 1; u < k.VPL; ++u) {
                const int ch = q.vslot[(size_t)w * k.VPL + u];
                if (ch >= 0 && vdeg(q.vorder[64 * ch]) > k.DVL) fits = false;
            }
        if (!fits) continue;
        q.arows = g.w_alpha_uniform ? 1 : h.M;
        q.bcols = g.w_beta_uniform ? 1 : h.N;
        q.cn_dmin = (!k.MIX && q.cn_lanes == k.LPC * nc) ? min_cdeg : 0;
        const float cu = clip / bs_step(mode);
        q.cu = cu > (float)bs_qmax(mode) ? cu : -1.f;
        q.lay = slot_layout_rows(h, q.rl, &q.nslot);
        // LDS: SGN [nslot + 1] | ARG [nslot + 1] | REC [(nc + 1) / 16 blocks][2][16][4] | TV [nv][6] |
        // RED | ALUT | BLUT
        const size_t sgn = ((q.nslot + 1) * 4 + 127) & ~(size_t)127;
        if (q.nslot + 1 > 65535) continue;
        if (nv > 32767) continue;                // v | Tv index << 16 as a non-negative int
        q.off_a = (uint32_t)sgn;
        size_t o = 2 * sgn;
        q.off_rec = (uint32_t)o;
        o += (size_t)((nc + 1 + 15) / 16) * 512;
        q.off_tv = (uint32_t)o;
        if ((rec_off((uint32_t)nc) >> 4) > 65535) continue;     // 16-bit record field
        o += (size_t)nv * 24;
        o = (o + 15) & ~(size_t)15;
        q.off_red = (uint32_t)o;
        o += 64 + (((size_t)4 * T + 15) & ~(size_t)15) + 4 * BS_FLORW;   // + the frame-error words
                                                                       // (16 B aligned), the OR words
        q.off_alut = (uint32_t)o;
        o += (size_t)2 * q.arows * LUT_W * 4;
        q.off_blut = (uint32_t)o;
        o += (size_t)2 * q.bcols * BLUT_W * 4;
        q.lds = (o + 15) & ~(size_t)15;
        if (q.lds > BS_LDS_MAX) continue;
        q.ok = true;
        return q;
    }
    return p;
}

static int bsc_tables(const DevGraph& g, const BscPlan& p, FusedWorkspace& ws, hipStream_t s) {
    if (ws.bs_graph && ws.bs_graph_inst == BSC_TAG + p.inst) return LDPC_OK;
    if (ws.bs_graph) {
        (void)hipFree(ws.bs_graph);
        ws.bs_graph = nullptr;
    }
    const host::GraphTables& h = *g.host;
    const BscInst& k = kBscInst[p.inst];
    const int nv = g.n_vars, nc = g.n_checks, z = h.z, LPC = k.LPC;
    const int VNW = k.DVH + 1, EPL = (k.D + LPC - 1) / LPC, CVW = (EPL + 1) / 2;
    const int NWp = p.nw, nl = 64 * NWp;
    auto slot_of = [&](int i, int kk, int hc) {
        const int L = p.rl[(size_t)i];
        return (uint32_t)((size_t)p.lay[2 * i] + (size_t)(kk % L) * p.lay[2 * i + 1] + (size_t)(kk / L) * z + hc);
    };
    // Tv slots: variable (column j, index hh) keeps its Tv at j z + (hh + toff_j) mod z.  The
    // check phase reads the Tv of each lane's edge m (ds_read_b64, bank = dword mod 64, 6 dwords
    // per variable: 32 lanes are conflict-free when their Tv indices differ mod 32); a half-wave
    // holds 8 consecutive checks of 4 edges, i.e. 4 runs of 8 consecutive indices from 4
    // columns, which overlap mod 32 for most column offsets.  A hill climb over the per-column
    // rotations toff_j spreads them (BG1: 695 -> ~514 LDS cycles per Tv read round of a
    // check pass in tools/bank_model's terms); the variable phase writes the same slot.
    const char* etv = getenv("LDPC_BSC_TVPERM");
    const std::vector<int> toff = (etv && atoi(etv) == 0) ? std::vector<int>(h.N, 0)
                                                           : column_rotation_lanes(h, EPL, p.lanes);
    auto tv_index = [&](int v) -> uint32_t {
        const int j = v / z, hh = v - j * z;
        return (uint32_t)(j * z + (hh + toff[j]) % z);
    };
    const uint32_t pad_word = (uint32_t)p.nslot | ((rec_off((uint32_t)nc) >> 4) << 16);    // zero slot, zero record
    std::vector<uint32_t> vn((size_t)k.VPL * nl * VNW, 0u);
    std::vector<int32_t> wdeg((size_t)2 * k.VPL * NWp, 0);
    for (int u = 0; u < k.VPL; ++u)
        for (int l = 0; l < nl; ++l) {
            uint32_t* q = &vn[((size_t)u * nl + l) * VNW];
            for (int f = 0; f < k.DVH; ++f) q[f] = pad_word;
            q[k.DVH] = 0xFFFFFFFFu;
        }
    for (int w = 0; w < NWp; ++w)
        for (int u = 0; u < k.VPL; ++u) {
            const int ch = p.vslot[(size_t)w * k.VPL + u];
            int dmax = ch < 0 ? -1 : 0, dmin = ch < 0 ? 0 : 1 << 30;     // -1: no chunk (skipped)
            for (int l = 0; ch >= 0 && l < 64; ++l) {
                const int o = 64 * ch + l;
                if (o >= nv) { dmin = 0; continue; }
                uint32_t* q = &vn[((size_t)u * nl + 64 * w + l) * VNW];
                const int v = p.vorder[o], j = v / z, hh = v - j * z;
                const int c0 = h.col_ptr[j], dv = h.col_ptr[j + 1] - c0;
                for (int f = 0; f < dv; ++f) {
                    const int pe = h.col_pe[c0 + f], i = h.pe_row[pe];
                    int hc = hh - h.pe_shift[pe];
                    hc = hc < 0 ? hc + z : hc;
                    q[f] = slot_of(i, pe - h.row_ptr[i], hc) | ((rec_off((uint32_t)(i * z + hc)) >> 4) << 16);
                }
                q[k.DVH] = (uint32_t)v | (tv_index(v) << 16);
                dmax = std::max(dmax, dv);
                dmin = std::min(dmin, dv);
            }
            wdeg[2 * ((size_t)u * NWp + w)] = dmax;
            wdeg[2 * ((size_t)u * NWp + w) + 1] = dmin;
        }
    const int cch = p.cn_lanes / 64;
    std::vector<int32_t> cchunk((size_t)NWp * k.CPL, -1);
    if (k.CPL == 1 && k.VPL == 1) {
        for (int w = 0; w < NWp; ++w) cchunk[w] = w < cch ? w : -1;
    } else {
        const std::vector<int> cs = deal_chunks(check_chunk_cost_lanes(h, p.lanes), NWp, k.CPL);
        for (size_t x = 0; x < cs.size(); ++x) cchunk[x] = cs[x];
    }
    std::vector<uint32_t> cvar((size_t)p.cn_lanes * CVW, 0u);
    for (int ql = 0; ql < p.cn_lanes; ++ql) {
        const int32_t dl = p.lanes[(size_t)ql];
        if (dl < 0) continue;
        const int cc = dl & 0xFFFF, cj = (dl >> 16) & 15, L = (dl >> 20) & 15;
        const int i = cc / z, hc = cc - i * z;
        for (int m = 0; m < EPL; ++m) {
            const int kk = L * m + cj;
            if (kk >= h.row_ptr[i + 1] - h.row_ptr[i]) continue;
            const int pe = h.row_ptr[i] + kk;
            const uint32_t v = tv_index(h.pe_col[pe] * z + (hc + h.pe_shift[pe]) % z);
            cvar[(size_t)ql * CVW + (m >> 1)] |= v << (16 * (m & 1));
        }
    }
    const size_t nwords = vn.size() + wdeg.size() + p.lay.size() + cchunk.size() + cvar.size() + p.lanes.size();
    void* d = nullptr;
    if (hipMalloc(&d, nwords * 4) != hipSuccess) { (void)hipGetLastError(); return LDPC_ERR_OOM; }
    uint32_t* dp = reinterpret_cast<uint32_t*>(d);
    size_t at = 0;
    bool ok = true;
    auto up = [&](const void* src, size_t n) {
        if (n) ok = ok && hipMemcpyAsync(dp + at, src, n * 4, hipMemcpyHostToDevice, s) == hipSuccess;
        at += n;
    };
    up(vn.data(), vn.size());
    up(wdeg.data(), wdeg.size());
    up(p.lay.data(), p.lay.size());
    up(cchunk.data(), cchunk.size());
    up(cvar.data(), cvar.size());
    up(p.lanes.data(), p.lanes.size());
    if (!ok || hipStreamSynchronize(s) != hipSuccess) {
        (void)hipFree(d);
        return LDPC_ERR_HIP;
    }
    ws.bs_graph = d;
    ws.bs_graph_inst = BSC_TAG + p.inst;
    return LDPC_OK;
}

template <int I, bool XP, bool B1, bool Q8>
static int bsc_launch1(const BscArgs& a, int nblocks, int nw, size_t lds, hipStream_t s) {
    constexpr BscInst k = kBscInst[I];
    auto* fn = &k_bsc<k.D, k.DVH, k.DVL, k.LPC, k.VPL, k.CPL, k.WPE, XP, 64 * k.NW, k.MIX, B1, Q8>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)BS_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(nblocks), dim3(64 * nw), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
template <int I, bool XP>
static int bsc_launch(const BscArgs& a, int nblocks, int nw, size_t lds, hipStream_t s, bool q8) {
    // (LDPC_BSC_B1=0: the general channel path for a B1 decode too, an A/B switch)
    static const bool b1_on = [] { const char* e = getenv("LDPC_BSC_B1"); return !(e && atoi(e) == 0); }();
    const bool b1 = b1_on && a.beta_id && a.bcols == 1;
    if constexpr (XP) {
        // (the generated channel comes from ldpc_decode_awgn, which exports no hard bits)
        if (q8) return LDPC_ERR_UNSUPPORTED;
    } else {
        if (q8) return b1 ? bsc_launch1<I, false, true, true>(a, nblocks, nw, lds, s)
                            : bsc_launch1<I, false, false, true>(a, nblocks, nw, lds, s);
    }
    if (b1) return bsc_launch1<I, XP, true, false>(a, nblocks, nw, lds, s);
    return bsc_launch1<I, XP, false, false>(a, nblocks, nw, lds, s);
}

}  // namespace bs

using namespace bs;

// Host-side bounds check of the bsc plan for this graph (test infrastructure, through
// ldpc_debug_bs_bounds): the in-prologue channel's tables at LDS byte 0 end inside the SGN
// region they borrow, and every check chunk's count of real edge positions -- the kernel's
// wave_or / popc over its lanes, restated -- is in 1 .. EPL, the range the min2 switch covers
// (its other cases are marked unreachable: BSC_MIN2_U).  Returns 1 if a plan was checked, 0 if
// none serves the graph; violations / first as BoundsReport.
int bsc_debug_bounds(const DevGraph& g, int mode, float clip, int T, int& violations, std::string& first) {
    const BscPlan p = bsc_plan(g, mode, false, false, clip, T);
    if (!p.ok) return 0;
    auto fail = [&](const char* what, long long idx, long long lo, long long hi) {
        if (violations++ == 0) {
            char buf[160];
            snprintf(buf, sizeof(buf), "%s: %lld outside [%lld, %lld)", what, idx, lo, hi);
            first = buf;
        }
    };
    const host::GraphTables& h = *g.host;
    const BscInst& k = kBscInst[p.inst];
    const int LPC = k.LPC, EPL = (k.D + LPC - 1) / LPC, z = h.z, nc = g.n_checks;
    if ((size_t)p.off_a >= sizeof(uint32_t) * AWGN_TAB_W && 4LL * AWGN_TAB_W > (long long)p.off_a)
        fail("channel tables", 4LL * AWGN_TAB_W, 0, p.off_a);
    for (int ch = 0; ch < p.cn_lanes / 64; ++ch) {
        const int32_t d0 = p.lanes[(size_t)ch * 64];
        const int Lc = (!k.MIX || d0 < 0 || ((d0 >> 20) & 15) == LPC) ? LPC : LPC / 2;
        uint32_t any = 0u;
        for (int l = 0; l < 64; ++l) {
            const int32_t d = p.lanes[(size_t)ch * 64 + l];
            const int cc = d < 0 ? nc : (d & 0xFFFF);
            const int ci = std::min(cc / z, nc / z - 1);
            const int gdeg = cc < nc ? h.row_ptr[ci + 1] - h.row_ptr[ci] : 0;
            const int npos = (gdeg + Lc - 1) / Lc;
            if (npos > 31) { fail("real positions of a lane", npos, 0, 32); continue; }
            any |= (1u << npos) - 1u;
        }
        const int gm = __builtin_popcount(any);
        if (gm < 1 || gm > EPL) fail("real positions of a chunk (the min2 switch)", gm, 1, EPL + 1);
    }
    return 1;
}

bool bsc_q8_ok(const DevGraph& g, int mode, bool ucn, float clip, int T, bool has_short) {
    const BscPlan p = bsc_plan(g, mode, ucn, false, clip, T);
    // (the in-prologue channel's tables borrow the SGN region at LDS byte 0)
    return p.ok && (!has_short || p.cu > 0.f) && (size_t)p.off_a >= sizeof(uint32_t) * AWGN_TAB_W;
}

bool bsc_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    return bsc_plan(g, mode, ucn, per_edge_w, clip, T).ok;
}

const char* bsc_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T) {
    static thread_local char buf[64];
    const BscPlan p = bsc_plan(g, mode, ucn, per_edge_w, clip, T);
    if (!p.ok) return "";
    const BscInst& k = kBscInst[p.inst];
    snprintf(buf, sizeof(buf), "bsc[p32,w%d,d%d,v%d/%d,l%d%s,x%d/%d]", p.nw, k.D, k.DVH, k.DVL, k.LPC,
             k.MIX ? "/2" : "", k.VPL, k.CPL);
    return buf;
}

int bsc_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
               bool ucn, int64_t* counters, uint8_t* flags, uint32_t* bad, uint32_t* hdx, hipStream_t s) {
    const BscPlan p = bsc_plan(g, mode, ucn, false, b.clip, b.T);
    if (!p.ok) return LDPC_ERR_UNSUPPORTED;
    int st = bsc_tables(g, p, ws, s);
    if (st != LDPC_OK) return st;
    const BscInst& k = kBscInst[p.inst];
    const float step = bs_step(mode);
    uint32_t *alut = nullptr, *blut = nullptr;
    const int32_t* atid = nullptr;
    st = bs_make_tables(b, g, p.arows, p.arows, p.bcols, step, bs_qmax(mode), p.cu, false, ws, &alut, &blut, s, &atid);
    if (st != LDPC_OK) return st;
    const uint32_t* gt = reinterpret_cast<const uint32_t*>(ws.bs_graph);
    const int VNW = k.DVH + 1;
    BscArgs a{};
    const bool q8 = b.q8 != nullptr;
    a.llr = llr;
    if (b.q8) {                          // the in-prologue channel (ldpc_decode_awgn)
        const AwgnParams& g8 = *reinterpret_cast<const AwgnParams*>(b.gen8);
        a.gen.tab = b.q8;
        a.gen.k0 = g8.k0;
        a.gen.k1 = g8.k1;
        a.gen.offset = g8.offset;
        a.gen.nb = g8.nb;
        a.gen.kmin = g8.kmin;
        a.gen.ps = g8.ps;
        a.gen.pe = g8.pe;
        a.gen.ss = g8.ss;
        a.gen.se = g8.se;
        a.gen.lds = 0u;
    }

    a.B = b.B;
    a.n_vars = g.n_vars;
    a.n_checks = g.n_checks;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.cn_dmin = p.cn_dmin;
    a.z = g.z;
    a.inv = 1.0f / step;
    a.cu = p.cu;
    a.qmax = bs_qmax(mode);
    a.beta_id = g.w_beta_one ? 1 : 0;
    a.row_ptr = g.row_ptr;
    a.vn_tab = gt;
    const size_t nvt = (size_t)k.VPL * 64 * p.nw * VNW;
    a.vn_wdeg = reinterpret_cast<const int32_t*>(gt + nvt);
    a.row_lay = a.vn_wdeg + 2 * (size_t)k.VPL * p.nw;
    a.cn_chunk = a.row_lay + 2 * (size_t)g.M;
    a.cn_var = reinterpret_cast<const uint32_t*>(a.cn_chunk + (size_t)p.nw * k.CPL);
    a.cn_lane = reinterpret_cast<const int32_t*>(a.cn_var + (size_t)p.cn_lanes * ((((k.D + k.LPC - 1) / k.LPC) + 1) / 2));
    bs_stagger(false, &a.stagger, &a.stagger_n);     // (LDPC_BS_STAGGER still applies; C5: no gain)
    a.alut = alut;
    a.atid = (p.arows == 1 && !getenv("LDPC_BS_NOAFIX")) ? atid : nullptr;
    a.blut = blut;
    a.arows = p.arows;
    a.bcols = p.bcols;
    a.counters = counters;
    a.flags = flags;
    a.bad = bad;
    a.iter_wrong = b.iter_wrong;
    a.hdx = hdx;
    a.off_a = p.off_a;
    a.off_rec = p.off_rec;
    a.off_tv = p.off_tv;
    a.off_red = p.off_red;
    a.off_alut = p.off_alut;
    a.off_blut = p.off_blut;
    const int nblocks = (int)((b.B + PACK - 1) / PACK);
    switch (p.inst) {
        case 1: return hdx ? bsc_launch<1, true>(a, nblocks, p.nw, p.lds, s, q8) : bsc_launch<1, false>(a, nblocks, p.nw, p.lds, s, q8);
        case 2: return hdx ? bsc_launch<2, true>(a, nblocks, p.nw, p.lds, s, q8) : bsc_launch<2, false>(a, nblocks, p.nw, p.lds, s, q8);
        case 3: return hdx ? bsc_launch<3, true>(a, nblocks, p.nw, p.lds, s, q8) : bsc_launch<3, false>(a, nblocks, p.nw, p.lds, s, q8);
        case 4: return hdx ? bsc_launch<4, true>(a, nblocks, p.nw, p.lds, s, q8) : bsc_launch<4, false>(a, nblocks, p.nw, p.lds, s, q8);
        default: return hdx ? bsc_launch<0, true>(a, nblocks, p.nw, p.lds, s, q8) : bsc_launch<0, false>(a, nblocks, p.nw, p.lds, s, q8);
    }
}

}  // namespace ldpc
