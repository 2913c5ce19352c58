// ldpc_bs_kernel.h — bit-sliced fused QMS decoder ("bsl"): 32 codewords per 32-bit word.
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
// LDS holds one 5-word SLOT per lifted edge:
//   between the variable and the check phase: V->C = clamp(Tv - C->V, +-15), as a negative flag
//     and 4 magnitude planes (the nudged zero is positive, Main_Functions.py:229-230);
//   between the check and the variable phase: C->V, as a negative flag and 4 magnitude planes.
// Each slot is read and then rewritten by exactly one lane per phase, so the two share it.
// Check phase: LPC lanes per check (padding edges read the all-ones PAD slot: negative,
// magnitude 15, so they change neither minimum nor parity).  Variable phase: one lane per
// variable (variables ordered by degree so a wave's loop bound is tight; padding edges read the
// all-zero ZERO slot); the channel stays in the lane's registers for the whole decode.
//
// Instances (kBsInst): the small graphs (wman, all variables and check lanes of a pack in one
// <= 16-wave workgroup, 16-bit packed slot addresses, 64 VGPRs: three workgroups per CU) and
// the large ones (5G BG2: VPL variables and CPL check groups per lane, 32-bit addresses, one
// 16-wave workgroup per CU), with or without UCN (Main_Functions.py:180-209: the syndrome of the
// previous hard decisions selects alpha' on unsatisfied checks) and shortened bits (LLR = the
// clip value, off the quantizer grid: Q(ch) = +-15, |Q(beta ch)| from a per-column table).
// Packs with any other LLR off the quantizer grid are flagged in `bad` and decoded by the v5
// kernel instead, so the result is exact for any input.
#pragma once
#include <type_traits>
#include <cstdint>

#include "ldpc_beta_tabs.h"
#include "ldpc_fused.h"
#include "ldpc_fused5_kernel.h"
#include "ldpc_bitplane.h"

namespace ldpc {
namespace bs {

constexpr int PACK = 32;                 // codewords per workgroup
constexpr int SLOT_W = 5;                // words per edge slot: negative flag, magnitude 0..3
constexpr int SLOT_B = SLOT_W * 4;
constexpr int LUT_W = 64;                // words per 16-entry table: [bit j][pair p] {X, Y}
constexpr int BLUT_W = LUT_W + 4;        // beta tables: + |Q(beta clip)| planes (shortened bits)
constexpr int QMAX = 15;
constexpr size_t BS_LDS_MAX = 160 * 1024;

// kernel instances: D = check-degree bound, DV = variable-degree bound, LPC = lanes per check,
// VPL / CPL = variables / 64-lane check chunks per lane, UCN / BIG = unsatisfied-check weights /
// shortened bits supported, PK = 16-bit packed slot addresses, WPE = waves per SIMD (registers),
// NW = waves of the multi-chunk instances (VPL / CPL > 1)
struct BsInst { int D, DV, LPC, VPL, CPL; bool UCN, BIG, PK; int WPE; int NW = 16; };
// cache policy of the LLR loads (the aux operand of the buffer loads: 2 = nt, streaming: the
// read-once LLR blocks then leave the graph tables in L2; A/B switch)
#ifndef BS_LLR_CPOL
#define BS_LLR_CPOL 0
#endif
#ifndef BS_WMAN_WPE
#define BS_WMAN_WPE 8
#endif
constexpr BsInst kBsInst[] = {
    {15, 6, 4, 1, 1, false, false, true, BS_WMAN_WPE},     // wman (C2), LPC 4 measured 6.31 ms vs 6.73
    {16, 8, 4, 1, 1, false, false, true, 8},
    {15, 6, 2, 1, 1, false, false, true, 8},     // LDPC_BS_LPC=2 A/B
    {24, 4, 4, 1, 1, true, true, true, 6},       // 802.11n (C3): degree 22, UCN
    {10, 8, 2, 2, 2, false, true, false, 4},     // 5G BG2 without UCN weighting (C4's trained
                                                 // alpha' = alpha folds to it)
    {10, 8, 2, 2, 2, true, true, false, 4},      // 5G BG2 (C4): 1,280 variables, 640 checks;
                                                 // 18.2 ms vs 21.2 for LPC 4 (CPL 3), same box
    {10, 8, 4, 2, 3, true, true, false, 4},      // LDPC_BS_LPC=4 A/B
    // 5G BG2 with 10 waves (20 variable and 20 check chunks, no idle place) at up to 168 VGPRs
    // (no spills, 2-3 waves per SIMD): LDPC_BS_INST=7 A/B
    {10, 8, 2, 2, 2, true, true, false, 3, 10},
    // 802.11n as a multi-chunk instance: two variables and two check chunks per lane on 8 waves,
    // two workgroups per CU at up to 128 VGPRs (the 80-VGPR one-chunk build spills 7): A/B only
    // (LDPC_BS_INST=8)
    {24, 4, 4, 2, 2, true, true, false, 4, 8},
};
constexpr int kBsNInst = sizeof(kBsInst) / sizeof(kBsInst[0]);

// The QMS channel generated in the kernel's prologue (Q8 builds; ldpc_decode_awgn, SURVEY 8 f
// rank 1): the byte each LLR would have on the q-bit grid (level + 16 + kmin), from the same
// Philox stream and level sampler as ldpc_channel_awgn (ldpc_awgn.h), so the decode is
// bit-identical to ldpc_channel_awgn + ldpc_decode.  The sampler's tables (awgn_gen_table,
// 8.25 KB) are copied into LDS at `lds`, a region the kernel writes only after the prologue.
struct BsGen {
    const uint32_t* tab;         // [AWGN_TAB_W] (awgn_gen_table)
    uint32_t k0, k1;             // Philox key (the seed)
    int64_t offset;              // global index of the batch's first codeword
    int nb, kmin;                // level count - 1, grid index of level 0
    int ps, pe, ss, se;          // 1-based puncture / shorten ranges (0: none)
    uint32_t lds;                // LDS byte address of the tables
};

struct BsArgs {
    const float* llr;            // (Q8 builds: unused, the channel is generated: gen)
    int64_t B;
    int n_vars, n_checks, T, target_bits, cn_lanes, cn_dmin;
    float inv;
    float cu;                    // |LLR| / step of a shortened bit (BIG instances), > qmax
    int qmax;                    // the grid's largest magnitude in grid units (15, 7 or 3)
    int ucn;                     // UCN weights present (UCN instances)
    uint64_t beta_id;            // bit t: iteration t's channel table is the identity (skipped)
    const int32_t* row_ptr;      // [M + 1] proto edges of each row (the check degrees)
    const int32_t* row_lay;      // [M][2] slot layout of each proto row: first slot, j-block stride
    int z;
    const uint32_t* vn_tab;      // [VPL][64 nw][VNW]: slot byte addresses (2 per word if PK), variable (-1 idle)
    const int32_t* vn_wdeg;      // [VPL][nw][3] most and fewest edges of a variable of each wave,
                                 // the chunk's column when it has one (else -1)
    const int32_t* cn_chunk;     // [nw][CPL] 64-lane check chunk of each wave's group (-1 idle)
    const uint32_t* cn_hd;       // [chunks * 64][HDW] UCN: LDS byte addresses of the edges' hard decisions
    const uint32_t* alut;        // [T][AR][LUT_W]: Q(relu(alpha m step)) for m = 0..15 (AR = arows, x2 with UCN)
    const uint32_t* blut;        // [T][bcols][BLUT_W]: |Q(beta m)| for m = 0..15 (grid units), |Q(beta cu)|
    int arows, bcols;
    const int32_t* atid;         // [T][AR] kBetaTab index of each row's check table (-1: not in
                                 // the set; AR = arows, x2 with UCN), or null
    const int32_t* btid;         // [T][btid_n] kBetaTab index of each column's channel table
    int btid_n;                  // (-1: evaluate from the table words), or null
    int64_t* counters;
    uint8_t* flags;
    uint32_t* bad;               // [packs] 1: decoded by the v5 fixup instead
    uint32_t* iter_wrong;        // [T][packs] per-iteration frame-error words, or null
    int stagger, stagger_n;      // start offsets of workgroups 0 .. stagger_n - 1 (the first
                                 // generation, one per CU), spread over 0 .. stagger x 512 clocks
    uint32_t* hdx;               // XP builds: [T][packs][n_vars] hard decisions (bit r = codeword
                                 // 32 pack + r), the hard-bit / syndrome export
    uint32_t off_slots, off_pad, off_zero, off_red, off_alut, off_blut, off_hdz, off_btid;   // LDS byte offsets
    uint32_t off_ch;             // per-lane LDS words: BS_CH_LDS the channel's magnitude planes,
                                 // [lane][VPL][4]; else (BS_GBLDS, one-chunk instances) the check
                                 // lane's slot base (| alpha-table address << 16), [lane]
                                 // (RED: 16 words, then T words: iteration t's frame-error word)
    int ablate;   // timing diagnostics, builds with -DBS_DIAG only (LDPC_DIAG_ABLATE, wrong
                  // results): 1 no check phase, 2 no beta table, 4 no V->C pass, 8 no frame
                  // flags, 16 no iterations, 32 no LLR loads.  (Compiled in, the uniform
                  // tests alone cost 4 %.)
    uint64_t ucn_iter;           // bit t (t < 64): iteration t's alpha' differs from alpha (its
                                 // check phase needs the syndromes); iterations >= 64: on
    uint32_t off_hdl;            // BS_HDLDS (one-chunk UCN instances): the check lanes' packed
                                 // hard-decision addresses, [HDW][lane] words
    uint32_t off_preb;           // (PREB) |Q(beta ch)| of the check-idle waves' variables, 16 B per
                                 // lane from wave cn_lanes / 64 on; 0: none
    BsGen gen;                   // Q8 builds: the in-prologue channel
    unsigned long long* stamps;  // -DBS_STAMP builds only: [16 waves][16] shader-clock sums per
                                 // phase (0 check, 1 check barrier, 2 variable, 3 variable barrier,
                                 // 4 prologue's check setup, 5 epilogue, 8 entry, 9 channel, 10 its
                                 // barrier, 11 tables, 12 first variable phase; 15 packs), timing
                                 // diagnostics
};

// bit-plane arithmetic (B3, the truth tables, add_b / set_b / sub_tv / abs_sat / lt4 / clamp6):
// ldpc_bitplane.h
// LDS accesses by byte address (all slots and tables are LDS-absolute: the kernel's dynamic
// LDS starts at 0, checked at entry)
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t LdsW;
typedef __attribute__((address_space(3))) v4u LdsQ;

__device__ __forceinline__ uint32_t lds_w(uint32_t addr) { return *reinterpret_cast<const LdsW*>(addr); }
__device__ __forceinline__ v4u lds_q(uint32_t addr) { return *reinterpret_cast<const LdsQ*>(addr); }
__device__ __forceinline__ void lds_put(uint32_t addr, uint32_t x) { *reinterpret_cast<LdsW*>(addr) = x; }

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
// (m & X) ^ Y with X, Y in SGPRs as two VOP2 instructions (the compiler's own form is a v_mov
// of one SGPR plus a v_bitop3 reading the other: the same issue cost, every VALU op with an
// SGPR operand takes ~4.2 cycles against 2.4 for VGPR-only ones; tools/valu_rate.hip)
__device__ __forceinline__ uint32_t leaf_s(uint32_t m, uint32_t X, uint32_t Y) {
    uint32_t t, l;
    asm("v_and_b32 %0, %1, %2" : "=v"(t) : "s"(X), "v"(m));
    asm("v_xor_b32 %0, %1, %2" : "=v"(l) : "s"(Y), "v"(t));
    return l;
}
__device__ __forceinline__ void lut_s(uint32_t (&o)[4], const uint32_t (&a)[4], const ConstW* tab) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t l0 = leaf_s(a[0], tab[j * 16 + 4 * q], tab[j * 16 + 4 * q + 1]);
            const uint32_t l1 = leaf_s(a[0], tab[j * 16 + 4 * q + 2], tab[j * 16 + 4 * q + 3]);
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

// n consecutive words src[0..n) to LDS byte address lds (a table for the next iteration),
// global -> LDS without registers (global_load_lds_dword: lane l of the wave whose first word is
// w0 writes word w0 + l).  Nothing waits for the loads here: the next __syncthreads (vmcnt(0))
// retires them, before any wave reads the table.
__device__ __forceinline__ void copy_async(uint32_t lds, const uint32_t* src, int n, int wave, int NT) {
    // (wave-uniform loop; the lane index from mbcnt, so no thread index is kept live for it)
    for (int w0 = wave * 64; w0 < n; w0 += NT) {
        const int w = w0 + (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        if (w < n)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + w),
                                             (__attribute__((address_space(3))) void*)(uintptr_t)(lds + 4u * (uint32_t)w0),
                                             4, 0, 0);
    }
}

// Fixed-set weight tables (ldpc_beta_tabs.h) by a computed call: the wave-uniform table index k
// selects an entry of a jump table (s_getpc + offset, s_swappc); the entry computes the output
// planes with immediate truth tables (v_bitop3) and returns (s_setpc to s[44:45]).  With
// BS_TAB_OOL the table of each call site is assembled into a section of its own, out of the
// kernel's instruction stream, so the loop body stays contiguous; else it follows the call and
// the call skips it.  s40-s45 are the call's scratch.  The caller keeps k in [0, kNBetaTab).
// (A/B, same box, r3i: out of line C2 5.31 against 5.26 ms in line, C4 14.66 both, C3 17.00
// against 17.07 — the instruction stream is not the bottleneck; in line is the default)
#ifndef BS_TAB_OOL
#define BS_TAB_OOL 0
#endif
#if BS_TAB_OOL
#define LDPC_TAB_CALL(SH, AL, TABLE)                                                              \
    "s_getpc_b64 s[40:41]\n\t"                                                                   \
    "s_add_u32 s40, s40, .Lbtab%=@rel32@lo+4\n\t"                                                \
    "s_addc_u32 s41, s41, .Lbtab%=@rel32@hi+12\n\t"                                              \
    "s_lshl_b32 s42, %[k], " SH "\n\t"                                                           \
    "s_add_u32 s40, s40, s42\n\t"                                                                \
    "s_addc_u32 s41, s41, 0\n\t"                                                                 \
    "s_swappc_b64 s[44:45], s[40:41]\n"                                                          \
    "\t.pushsection .text.ldpc_tables,\"ax\",@progbits\n"                                         \
    "\t.p2align " AL "\n"                                                                        \
    ".Lbtab%=:\n" TABLE "\t.popsection\n"
#else
#define LDPC_TAB_CALL(SH, AL, TABLE)                                                              \
    "s_getpc_b64 s[40:41]\n"                                                                      \
    ".Lbpc%=:\n\t"                                                                                \
    "s_lshl_b32 s42, %[k], " SH "\n\t"                                                           \
    "s_add_u32 s40, s40, s42\n\t"                                                                \
    "s_addc_u32 s41, s41, 0\n\t"                                                                 \
    "s_add_u32 s40, s40, .Lbtab%=-.Lbpc%=\n\t"                                                    \
    "s_addc_u32 s41, s41, 0\n\t"                                                                 \
    "s_swappc_b64 s[44:45], s[40:41]\n\t"                                                        \
    "s_branch .Lbend%=\n"                                                                        \
    "\t.p2align " AL "\n"                                                                        \
    ".Lbtab%=:\n" TABLE ".Lbend%=:\n"
#endif

// The channel-weight table |Q(beta_t ch)| (Main_Functions.py:164-177) when beta_t's table is
// table k of the fixed set: each output bit j is mux(m3, f_hi(m2, m1, m0), f_lo(m2, m1, m0))
// with compile-time truth tables, at most three v_bitop3 with immediates, against 16 leaves with
// SGPR operands (4.2-cycle forms) and 7 muxes per bit for a table held in SGPRs.  (A C++ switch
// over the 210 tables, a binary tree of scalar branches with 210 leaves, made the register
// allocator spill 291 VGPRs.)
__device__ __forceinline__ void beta_asm(uint32_t (&o)[4], const uint32_t (&m)[4], int k) {
    uint32_t t0, t1;
    asm volatile(LDPC_TAB_CALL("7", "7", LDPC_BETA_ASM_TABLE)
        : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]),
          [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [m0] "v"(m[0]), [m1] "v"(m[1]), [m2] "v"(m[2]), [m3] "v"(m[3]), [k] "s"(k)
        : "s40", "s41", "s42", "s43", "s44", "s45", "scc");
}
#ifndef BS_BFIX
#define BS_BFIX 1       // the fixed-table channel weighting (A/B switch)
#endif
// The table ids staged in LDS per iteration (one global_load_lds by wave 0 at the iteration
// start) instead of a global load after the barrier (A/B switch, off: same box, r3k, C3 18.29
// against 16.60 ms, C2 5.41 against 5.26)
#ifndef BS_BTID_LDS
#define BS_BTID_LDS 0
#endif

// The check phase's two weighted minima through table k of the fixed set, all 4 output bits of
// both (<= 24 v_bitop3 with immediates, 256-byte entries of LDPC_BETA_ASM_TABLE2)
__device__ __forceinline__ void table_asm2(uint32_t (&p)[4], uint32_t (&q)[4], const uint32_t (&a)[4],
                                           const uint32_t (&b)[4], int k) {
    uint32_t t0, t1;
    asm volatile(LDPC_TAB_CALL("8", "8", LDPC_BETA_ASM_TABLE2)
        : [p0] "=&v"(p[0]), [p1] "=&v"(p[1]), [p2] "=&v"(p[2]), [p3] "=&v"(p[3]),
          [q0] "=&v"(q[0]), [q1] "=&v"(q[1]), [q2] "=&v"(q[2]), [q3] "=&v"(q[3]),
          [t0] "=&v"(t0), [t1] "=&v"(t1)
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]),
          [b0] "v"(b[0]), [b1] "v"(b[1]), [b2] "v"(b[2]), [b3] "v"(b[3]), [k] "s"(k)
        : "s40", "s41", "s42", "s43", "s44", "s45", "scc");
}
// a chunk of check lanes whose checks lie in two rows (lanes < split: table k0, the others k1)
__device__ __forceinline__ void alpha_fixed(uint32_t (&p)[4], uint32_t (&q)[4], const uint32_t (&a)[4],
                                            const uint32_t (&b)[4], int k0, int k1, int split) {
    if (k0 == k1) {
        table_asm2(p, q, a, b, k0);
    } else {
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        if (ln < split) table_asm2(p, q, a, b, k0);
        else table_asm2(p, q, a, b, k1);
    }
}
// The fixed-table check weighting (A/B switch, off).  Measured on one box (r3g): C3 20.1
// against 18.9 ms, C4 16.2 against 15.2, C2 5.69 against 5.71; compiled in but disabled, the
// others ran 3-7 % slower than without it.  Not the instruction cache (the out-of-line tables
// changed nothing, r3i): the table call holds 18 operands live at once, and the higher register
// pressure of the whole check phase costs more than the table words and the lane exchange.
#ifndef BS_AFIX
#define BS_AFIX 0
#endif
// DPP moves with bound_ctrl (A/B switch; see qperm)
#ifndef BS_DPP_BC
#define BS_DPP_BC true
#endif
// wave priorities (A/B switch): 2 runs each check phase at priority 1 and each variable phase at
// 0, so that the check phase — the one with idle waves (C3: 7 of 12 waves hold check lanes) —
// wins issue slots from the other resident workgroups' variable phases; -1 (default) picks 2 for
// the one-chunk instances (several workgroups per CU; same box, r5j: C2 4.71 -> 4.64 ms, C3
// 13.56 -> 12.99) and 0 for the multi-chunk ones (one workgroup per CU: C4 11.32 against 11.38)
#ifndef BS_PRIO
#define BS_PRIO -1
#endif

// lane permutation inside each group of 4 lanes (DPP quad_perm, a VALU move).  bound_ctrl on:
// every lane of a quad_perm / row mirror has a source lane, so the "old" operand is dead — with
// it off the compiler materialised the old value 0 in the destination first (one v_mov_b32 0
// per DPP move: 26 of the ~200 VALU of a C2 check lane), and with it on a DPP move whose
// consumer is a VOP2 op folds into it (v_xor_b32_dpp)
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, BS_DPP_BC);
}
constexpr int QP_X1 = 0xB1;          // [1, 0, 3, 2]
constexpr int QP_X2 = 0x4E;          // [2, 3, 0, 1]

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, BS_DPP_BC);
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
// lo = min(A, B), hi = max(A, B) (4-plane magnitudes)
__device__ __forceinline__ void sort2(uint32_t (&lo)[4], uint32_t (&hi)[4], const uint32_t (&A)[4],
                                      const uint32_t (&B)[4]) {
    const uint32_t l = lt4(B, A);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        lo[i] = mux(l, B[i], A[i]);
        hi[i] = mux(l, A[i], B[i]);
    }
}
// AND over the LPC lanes of a check's group: one v_and_b32_dpp per step.  (Each step's result
// goes through an empty asm, so the two ANDs are not reassociated into one v_bitop3 AND3 — which
// left both DPP moves unfolded: 2 DPP moves + 2 VALU per step pair instead of 2 DPP ANDs.)
template <int LPC>
__device__ __forceinline__ uint32_t grp_and(uint32_t a) {
    a &= qperm<QP_X1>(a);
    asm("" : "+v"(a));
    if (LPC == 4) {
        a &= qperm<QP_X2>(a);
        asm("" : "+v"(a));
    }
    return a;
}
// The check's two minima by a bit-serial search over the whole lane group, most significant
// plane first: plane i of the minimum is the AND over the edges still tied with it on the planes
// above (cand), taken across the group by DPP; cand ends as [|V->C| = m1], the edges that get the
// second minimum in pass 2.  The second minimum is the same search over the other edges, or m1
// where two or more edges tie at it.  (Against the pair tournament and the two lane-group merges:
// C2, 4 edges per lane, 98 VALU with 22 DPP per lane against 117 with 18, and pass 2 no longer
// compares each edge with m1.)  Padding slots (all ones) are magnitude 15: with degree >= 2 they
// change neither minimum.
// (the first K of the EPL slots: the multi-chunk instances skip the positions that are padding
// for the whole chunk, K = gm by a switch)
template <int K, int LPC, int EPL>
__device__ __forceinline__ void min2_bits(uint32_t (&m1)[4], uint32_t (&m2)[4], uint32_t (&cand)[EPL],
                                          const uint32_t (&X)[EPL][4]) {
    static_assert(K >= 1 && K <= EPL, "active slots");
    constexpr unsigned T_ANDORN = (TA & (TB | ~TC)) & 0xFF;      // a & (b | ~c)
    constexpr unsigned T_ANDOR = (TA & (TB | TC)) & 0xFF;        // a & (b | c)
    constexpr unsigned T_ANDEQ = (TA & ~(TB ^ TC)) & 0xFF;       // a & (b == c)
    constexpr unsigned T_NANDEQ = (~TA & ~(TB ^ TC)) & 0xFF;     // ~a & (b == c)
    constexpr unsigned T_ORAND = (TA | (TB & TC)) & 0xFF;        // a | (b & c)
    // m1, most significant plane first
    uint32_t a = X[0][3];
#pragma unroll
    for (int m = 1; m < K; ++m) a &= X[m][3];
    a = grp_and<LPC>(a);
    m1[3] = a;
#pragma unroll
    for (int m = 0; m < K; ++m) cand[m] = ~(X[m][3] ^ a);
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        a = X[0][i] | ~cand[0];
#pragma unroll
        for (int m = 1; m < K; ++m) a = B3(T_ANDORN, a, X[m][i], cand[m]);
        a = grp_and<LPC>(a);
        m1[i] = a;
#pragma unroll
        for (int m = 0; m < K; ++m) cand[m] = B3(T_ANDEQ, cand[m], X[m][i], a);
    }
    // two or more edges of the group at the minimum
    uint32_t one = cand[0], two = 0u;
#pragma unroll
    for (int m = 1; m < K; ++m) {
        two = B3(T_ORAND, two, one, cand[m]);
        one |= cand[m];
    }
    {
        const uint32_t op = qperm<QP_X1>(one);
        two = qperm<QP_X1>(two) | B3(T_ORAND, two, one, op);
        one |= op;
    }
    if (LPC == 4) {
        const uint32_t op = qperm<QP_X2>(one);
        two = qperm<QP_X2>(two) | B3(T_ORAND, two, one, op);
    }
    // the minimum of the other edges (c2: not at m1, tied with the search so far)
    uint32_t c2[K];
    a = X[0][3] | cand[0];
#pragma unroll
    for (int m = 1; m < K; ++m) a = B3(T_ANDOR, a, X[m][3], cand[m]);
    a = grp_and<LPC>(a);
    m2[3] = a;
#pragma unroll
    for (int m = 0; m < K; ++m) c2[m] = B3(T_NANDEQ, cand[m], X[m][3], a);
#pragma unroll
    for (int i = 2; i >= 0; --i) {
        a = X[0][i] | ~c2[0];
#pragma unroll
        for (int m = 1; m < K; ++m) a = B3(T_ANDORN, a, X[m][i], c2[m]);
        a = grp_and<LPC>(a);
        m2[i] = a;
        if (i > 0) {
#pragma unroll
            for (int m = 0; m < K; ++m) c2[m] = B3(T_ANDEQ, c2[m], X[m][i], a);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) m2[i] = mux(two, m1[i], m2[i]);
}
#ifndef BS_BSMIN
#define BS_BSMIN 1      // the bit-serial two minima (A/B switch)
#endif
#ifndef BS_BSMIN_MC
#define BS_BSMIN_MC 1   // ... on the multi-chunk instances too (A/B switch)
#endif
// The switch over a chunk's real positions (1 <= gmc <= EPL for every active chunk, by
// construction: ceil(degree / lanes per check) of its widest check) may mark every other count
// unreachable (U), and zero the tie words of the positions past it (Z).  Without U the compiler
// keeps the search's inputs and outputs alive through the empty cases and copies them at the join
// (C4, static: 39 v_mov per chunk, 2.47 -> 2.28 VALU per pack-edge-iteration).  bsc's C5 gains
// (48.4 -> 47.9 ms, r5o); the bsl C4 build ran slower with U+Z before the plane-count copies
// (r5o: 11.48 against 11.30 ms) and equal after them (r5w: 11.17-11.22 against 11.21-11.22), for
// fewer instructions: on for both
#ifndef BS_MIN2_U
#define BS_MIN2_U 1
#endif
#ifndef BS_MIN2_Z
#define BS_MIN2_Z 1
#endif
#ifndef BSC_MIN2_U
#define BSC_MIN2_U 1
#endif
// the variable phase at the fewest planes of S for each place's largest degree: 7 where
// 15 dw + 15 <= 63, 8 where <= 127, else 9 (one copy of the phase per plane count; BS_SBV 0 off).
// BS_SBV_SET: the plane counts below the instance's that get a copy (1 seven, 2 eight); -1
// (default): both on the one-chunk instances (same box, r5p: C2 4.66 -> 4.61 ms, C3 12.99 ->
// 12.60), eight only on the multi-chunk ones (r5r: C4 11.33 -> 11.20; with both its 128-VGPR
// build spilled 17 VGPRs and ran 11.74)
#ifndef BS_SBV
#define BS_SBV 1
#endif
#ifndef BS_SBV_SET
#define BS_SBV_SET -1
#endif
// instances whose variables have at most BS_KEEP_DV edges keep all of them (0: none — 802.11n's
// choice before the plane-count copies, three of four and the fourth read again; with them the C3
// build keeps all four at the same 69-75 VGPRs: same box, r5s, 12.60 -> 12.40 ms)
#ifndef BS_KEEP_DV
#define BS_KEEP_DV 4
#endif

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

#ifdef BS_DIAG
#define ABL(bit) (a.ablate & (bit))
#else
#define ABL(bit) 0
#endif
// Phase markers for the ISA attribution (tools/isa_phase_table.py), analysis builds only
// (-DBS_MARK: an assembler comment ";@ph NAME.K" at each phase start; the product build has none)
// PH4 / PH8 / PH9 tie the marker to the values the phase starts from ("+v"), so the phase's first
// instructions cannot be scheduled above it
#ifdef BS_MARK
#define PH(name, k) asm volatile(";@ph " name ".%0" ::"i"(k))
#define PH4(name, k, x) asm volatile(";@ph " name ".%4" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "i"(k))
#define PH8(name, k, x, y)                                                                        \
    asm volatile(";@ph " name ".%8" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]),  \
                 "+v"(y[1]), "+v"(y[2]), "+v"(y[3]) : "i"(k))
#define PH9(name, k, x, y, z)                                                                     \
    asm volatile(";@ph " name ".%9" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]),  \
                 "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(z) : "i"(k))
#else
#define PH(name, k) ((void)0)
#define PH4(name, k, x) ((void)0)
#define PH8(name, k, x, y) ((void)0)
#define PH9(name, k, x, y, z) ((void)0)
#endif
// C->V messages of a variable lane's first BS_KEEP edges kept in registers from the sum pass to
// the V->C pass (the others are read from their slots again).  Measured per instance, same box,
// 2 rounds (tools/bs_variant.sh -DBS_KEEP=k): C2 5.79 (0) / 5.70 (1) / 5.58 (2) / 5.56 (3) /
// 5.55 (4) / 5.71 ms (6); C3 18.75 / 18.53 / 18.25 / 17.80 / 17.76 / 17.75; C4 18.15 / 17.97 /
// 17.81 / 17.76 / 17.67 / 17.62 ms (round 3; round 5 with the plane-count copies: C2 takes 3,
// C3 all four, profiles/r5/ab_sbv.log).
// the channel's 4 magnitude planes of each variable kept in LDS (one ds_read_b128 per variable
// and iteration) instead of 4 registers held through the whole decode (A/B switch)
#ifndef BS_CH_LDS
#define BS_CH_LDS 0
#endif
// the one-chunk instances' check-lane slot base (packed with the alpha-table address) kept in
// one LDS word per lane and read at each check phase, instead of a register held through the T
// loop (which the 64- and 80-VGPR builds spilled: a scratch reload + vmcnt(0) per iteration)
#ifndef BS_GBLDS
#define BS_GBLDS 1
#endif
// with it, the check lane's EPL slot addresses themselves (16 bits each, the PAD slot in place of
// a padding edge), two per LDS word after the slot-base word: the check phase reads them instead
// of computing base + m stride and selecting PAD by lane masks (VALU with SGPR operands, ~4
// cycles each) (A/B switch, off: 0.05 fewer VALU per pack-edge-iteration on C2, but the words
// push C2's LDS over a third of the CU (two workgroups per CU: 4.81 against 4.69 ms) and C3's
// over a half (20.2 against 13.5 ms), r5c)
#ifndef BS_ALDS
#define BS_ALDS 0
#endif
// The channel planes of one variable for the 32 codewords of a pack: sign cs, magnitude planes
// cm[0..3] of Q(ch) in grid units, shortened-bit flags bg (BIG); returns 1 when a row is off the
// grid (the pack then goes to the v5 fixup).  Per row: x = llr / step, q = clamp(rint(x), +-qmax)
// — on the grid iff q == x, or a shortened bit (|x| == cu, decoded as +-qmax) — and q is stored
// as the byte q + 16 (+ 32 for a shortened bit) by v_cvt_pk_u8_f32, four rows per word.  The 32
// bytes become bit planes by four 8x8 bit-matrix transposes (three delta swaps each) and a 4x4
// byte transpose (v_perm); offset binary q + 16 gives the sign (NOT bit 4) and, bit-sliced, the
// magnitude (the low 4 bits, negated mod 16 where negative).  About 300 VALU per variable against
// ~750 for a per-row insertion of each bit into each plane (2 ops per bit and plane).
// (valid: the pack's codewords; rows past it read 0 and are masked)
__device__ __forceinline__ void t8x8(uint32_t& lo, uint32_t& hi) {
    uint32_t t;
    t = B3((TA ^ TB) & TC, lo, lo >> 7, 0x00AA00AAu);
    lo = B3(T_XOR3, lo, t, t << 7);
    t = B3((TA ^ TB) & TC, hi, hi >> 7, 0x00AA00AAu);
    hi = B3(T_XOR3, hi, t, t << 7);
    t = B3((TA ^ TB) & TC, lo, lo >> 14, 0x0000CCCCu);
    lo = B3(T_XOR3, lo, t, t << 14);
    t = B3((TA ^ TB) & TC, hi, hi >> 14, 0x0000CCCCu);
    hi = B3(T_XOR3, hi, t, t << 14);
    t = B3((TA ^ TB) & TC, lo, hi << 4, 0xF0F0F0F0u);
    lo ^= t;
    hi ^= t >> 4;
}
// the 32 bytes (byte r of D[r / 4]: q + 16, + 32 on a shortened bit) -> sign / magnitude /
// shortened planes
template <bool BIG>
__device__ __forceinline__ void pack_bytes(const uint32_t (&D)[8], uint32_t valid, uint32_t& cs,
                                           uint32_t (&cm)[4], uint32_t& bg) {
    uint32_t lo[4], hi[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        lo[g] = D[2 * g];
        hi[g] = D[2 * g + 1];
        t8x8(lo[g], hi[g]);
    }
    // byte p of lo[g] (p < 4) / hi[g] (p >= 4): plane p of rows 8 g .. 8 g + 7
    const uint32_t a = __builtin_amdgcn_perm(lo[1], lo[0], 0x06020400u), b = __builtin_amdgcn_perm(lo[1], lo[0], 0x07030501u);
    const uint32_t c = __builtin_amdgcn_perm(lo[3], lo[2], 0x06020400u), d = __builtin_amdgcn_perm(lo[3], lo[2], 0x07030501u);
    const uint32_t L0 = __builtin_amdgcn_perm(c, a, 0x05040100u) & valid, L2 = __builtin_amdgcn_perm(c, a, 0x07060302u) & valid;
    const uint32_t L1 = __builtin_amdgcn_perm(d, b, 0x05040100u) & valid, L3 = __builtin_amdgcn_perm(d, b, 0x07060302u) & valid;
    const uint32_t e = __builtin_amdgcn_perm(hi[1], hi[0], 0x05010400u), f = __builtin_amdgcn_perm(hi[3], hi[2], 0x05010400u);
    const uint32_t n = ~__builtin_amdgcn_perm(f, e, 0x05040100u) & valid;
    bg = BIG ? (__builtin_amdgcn_perm(f, e, 0x07060302u) & valid) : 0u;
    cs = n;
    cm[0] = L0;
    cm[1] = B3(T_XAND, L1, n, L0);
    cm[2] = B3(T_XAND, L2, n, L0 | L1);
    cm[3] = B3(T_XAND, L3, n, L0 | L1 | L2);
}
template <bool BIG>
__device__ __forceinline__ int pack_channel(const float (&xv)[PACK], float inv, int qmax, float cu,
                                            uint32_t valid, uint32_t& cs, uint32_t (&cm)[4], uint32_t& bg) {
    const float qf = (float)qmax;
    uint32_t D[8];
    int off = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) D[k] = 0u;
#pragma unroll
    for (int r = 0; r < PACK; ++r) {
        const float x = xv[r] * inv;
        const float q = __builtin_amdgcn_fmed3f(rintf(x), -qf, qf);
        const bool big = BIG && fabsf(x) == cu;
        off |= (q != x && !big) ? 1 : 0;
        D[r >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(q + (big ? 48.f : 16.f), r & 3, D[r >> 2]);
    }
    pack_bytes<BIG>(D, valid, cs, cm, bg);
    return off;
}
// The bytes of variable v for the 32 codewords of pack pk, generated (Q8 builds): byte r of
// D[r / 4] = level + 16 + kmin of codeword offset + 32 pk + r (a shortened bit: 48 - qmax, a
// punctured one: 16; oracle/philox_oracle.py awgn_q8).  Four codewords per Philox call; a batch offset
// off the quads takes two quads per word and a byte funnel shift (wave-uniform).
typedef unsigned int v2u_g __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const v2u_g LdsU2;
__device__ __forceinline__ void gen_bytes(const BsGen& g, int64_t pk, int v, int qmax, uint32_t (&D)[8]) {
    const int bit = v + 1;
    if (g.ss > 0 && bit >= g.ss && bit <= g.se) {
#pragma unroll
        for (int i = 0; i < 8; ++i) D[i] = (uint32_t)(48 - qmax) * 0x01010101u;
        return;
    }
    if (g.ps > 0 && bit >= g.ps && bit <= g.pe) {
#pragma unroll
        for (int i = 0; i < 8; ++i) D[i] = 0x10101010u;
        return;
    }
    LdsU2* bucket = reinterpret_cast<LdsU2*>((uintptr_t)g.lds);
    const LdsW* thi = reinterpret_cast<const LdsW*>((uintptr_t)(g.lds + 8u * (1u << AWGN_KB)));
    const LdsW* tlo = thi + AWGN_NB_MAX;
    const uint64_t g0 = (uint64_t)g.offset + (uint64_t)pk * 32u;
    const int sh = (int)(g.offset & 3);
    const uint32_t boff = (uint32_t)(16 + g.kmin);
    auto word = [&](const int (&l)[4]) __attribute__((always_inline)) -> uint32_t {
        return ((uint32_t)l[0] + boff) | ((uint32_t)l[1] + boff) << 8 | ((uint32_t)l[2] + boff) << 16 |
               ((uint32_t)l[3] + boff) << 24;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint64_t gq = (g0 + 4u * (uint32_t)i) >> 2;
        int la[4];
        awgn_levels4b(g, bucket, thi, tlo, (uint32_t)v, gq, la);
        uint32_t w = word(la);
        if (sh) {
            int lb[4];
            awgn_levels4b(g, bucket, thi, tlo, (uint32_t)v, gq + 1, lb);
            w = __builtin_amdgcn_alignbyte(word(lb), w, (uint32_t)sh);
        }
        D[i] = w;
    }
}
// the generator's tables into LDS (every thread of the workgroup; the caller's barrier follows
// and, with BS_GENASYNC, retires the global -> LDS copies by its vmcnt(0): one L2 round trip
// instead of one per 64 NT words, each waited before its store)
#ifndef BS_GENASYNC
#define BS_GENASYNC 1
#endif
__device__ __forceinline__ void gen_tables(const BsGen& g, int tid, int NT) {
    if (BS_GENASYNC) {
        copy_async(g.lds, g.tab, AWGN_TAB_W, __builtin_amdgcn_readfirstlane(tid >> 6), NT);
        return;
    }
    for (int w = tid; w < AWGN_TAB_W; w += NT) lds_put(g.lds + 4u * (uint32_t)w, g.tab[w]);
}
#ifndef BS_PACKT
#define BS_PACKT 1      // pack_channel (A/B switch; 0: per-row bit insertion)
#endif

// first-generation start spread of the one-workgroup-per-CU instances, microseconds (bs_stagger)
// (bsl's one-workgroup-per-CU instances: 5G BG2 (C4) 13.93 -> 13.78 ms at 100 us, 50 / 200 us
// in between, same box, r3ze; bsc: no effect, so it passes one_per_cu = false and starts at 0).
// Round 6, with C4's packs at ~82 us: 60 us 10.47 / 10.53 ms against 100 us 10.52 and 0 us 10.56
// (two boxes, profiles/r6/session_r6l.log, r6m; 30-80 us equal within 0.2 %; C5 no gain at 180 /
// 360 us)
#ifndef BS_STAGGER_US
#define BS_STAGGER_US 60.0
#endif
// the check lane's slot base and alpha-table address packed in one register (16-bit-address
// one-chunk instances; ldpc_bs.hip checks that the tables end below 64 KB)
#ifndef BS_PKG
#define BS_PKG 1
#endif
// column-aligned variable lanes (ldpc_bs.hip, colalign_fits): 1 on where it fits
#ifndef BS_COLALIGN
#define BS_COLALIGN 1
#endif
// (A/B switch, off: C3 spill-free at 72 VGPRs with it, and slower: 17.37 against 16.07 ms on one
// box, r3q — pass 2 then waits on its LDS reads, where the spills it removes were reloaded once
// per iteration)
#ifndef BS_REREAD
#define BS_REREAD 0
#endif
// (the multi-chunk instances, one workgroup per CU with registers to spare: BS_KEEP_MC; 5G BG2
// keeps 7 of its 8: C4 11.85-11.88 -> 11.60-11.65 ms, 6: 11.76-11.79, same box, r4f)
// the multi-chunk instances' real-edge-position word, read per iteration through an opaque copy
// (A/B switch; see rpk in k_bs)
#ifndef BS_RPW
#define BS_RPW 1
#endif
#ifndef BS_VVO
#define BS_VVO 1
#endif
// the one-chunk UCN instances' packed hard-decision addresses (HDW words per check lane) in LDS,
// read at each check phase, instead of registers the 80-VGPR build spilled (A/B switch)
// the one-chunk instances' channel-table ids by scalar loads (s_load from the constant address
// space: an SGPR result, no vector-memory round trip and vmcnt wait per variable phase) (A/B)
#ifndef BS_BTID_S
#define BS_BTID_S 1
#endif
#ifndef BS_HDLDS
#define BS_HDLDS 1
#endif
#ifndef BS_KEEP_MC
#define BS_KEEP_MC 7
#endif
#ifndef BS_KEEP
#define BS_KEEP 3       // (wman: 3 against 4, same box r5u, 4.63 -> 4.59 ms over five pairs)
#endif
#ifndef BS_KEEP_MCU
#define BS_KEEP_MCU 4
#endif
// variable places without a chunk skipped (A/B switch: -DBS_VSKIP=0 runs their table work)
#ifndef BS_VSKIP
#define BS_VSKIP 1
#endif
// lanes with several variables issue all their LLR loads before converting any (A/B switch)
#ifndef BS_LLR_ALL
#define BS_LLR_ALL 0
#endif
// LLR loads through a buffer descriptor (A/B switch; 0: 64-bit pointer loads)
#ifndef BS_BUFLD
#define BS_BUFLD 1
#endif
// fold / check-lane / table-copy tests on the wave index instead of the thread index (A/B)
#ifndef BS_TIDFREE
#define BS_TIDFREE 1
#endif
// the next iteration's weight tables copied global -> LDS asynchronously (global_load_lds: the
// wave does not wait for the load; the barrier after the check phase retires it) instead of
// through registers, which stalled every wave for an L2 round trip at each iteration start
// (A/B switch)
#ifndef BS_GLDS
#define BS_GLDS 1
#endif
// UCN: a wave's alpha' table evaluation skipped when all its checks are satisfied (A/B switch;
// the multi-chunk instances only: C4 17.96 against 18.03 ms, C3 17.54 against 17.31 without)
#ifndef BS_USKIP
#define BS_USKIP 1
#endif
// the variable phase's channel-table ids (a.btid, one global load per variable place and
// iteration, whose result the table jump waits for) loaded before the check phase instead of
// at their use: 1 for the multi-chunk instances (one workgroup per CU, so nothing else hides a
// wave's L2 round trip after the barrier), 2 for every instance, 0 off (A/B switch)
// loop-top table copies with opaque bounds (hoisted, their compares were 64-bit lane masks held
// through the loop and spilled: C2's in-loop v_readlane 35 -> 24 static; same box,
// profiles/r6/session_r6x.log: C2 4.427 -> 4.406 ms, C4 10.542 -> 10.447, C3 12.451 -> 12.378).
// Not in wman's in-prologue channel build (Q8): there it cost the sweep step 1.1 % (4.651
// against 4.599 ms, session_r6ac.log), where the other Q8 builds gained (sweep step without /
// with it, two boxes each: C3 80.5 / 83.1 M cw/s, C4 94.5 / 96.0 M; session_r6ad, r6z, r6ab)
#ifndef BS_TOPO
#define BS_TOPO 1
#endif
// loop-top table addresses reloaded from the kernel arguments per iteration (scalar loads from
// the kernarg segment, whose pointer stays in its SGPRs) instead of held through the T loop:
// C3's loop spill reloads 16 -> 0, C2's 8 -> 3; same box, profiles/r6/session_r6ah.log: C2
// 4.406 -> 4.322 ms, C3 12.361 -> 12.157 (sweep step 12.628 -> 12.464)
#ifndef BS_KARG
#define BS_KARG 1
#endif
// the epilogue's output pointers loaded from the kernel arguments after the T loop, so the
// loop does not hold them from the kernel's entry (C2's channel-build loop reloads 20 -> 11;
// same box, profiles/r6/session_r6ak.log: C3 12.124 -> 12.052 ms, sweep steps C2 4.604 ->
// 4.561, C3 12.44 -> 12.34)
#ifndef BS_KEPI
#define BS_KEPI 1
#endif
// (PREB) the check-idle waves' next channel tables evaluated in the check phase: -1 the one-chunk
// UCN instance, 0 off, 1 every one-chunk instance.  Off: on 802.11n (C3) it cost 2 % (same box,
// profiles/r6/session_r6w.log: 12.67 against 12.41 ms, counters equal) -- the second inlined
// copy of the table code doubled the loop's SGPR spills (30 -> 56) for ~12 % of five waves'
// variable phase
#ifndef BS_PREB
#define BS_PREB 0
#endif
#ifndef BS_BKPF
#define BS_BKPF 1
#endif
// iteration 0's tables copied asynchronously behind the channel loads (A/B switch; 0: through
// registers after the channel barrier, with a barrier of their own; -1, default: on for the
// one-chunk instances -- with BS_EB C2 4.519 -> 4.482 ms, r6c -- off for the multi-chunk ones,
// one workgroup per CU, where the two together cost C4 2.2 %: 11.26 against 11.51 ms, r6d)
#ifndef BS_T0ASYNC
#define BS_T0ASYNC -1
#endif
// the prologue's first barrier after the first LLR loads are issued (A/B switch; 0: before them;
// -1: as BS_T0ASYNC)
#ifndef BS_EB
#define BS_EB -1
#endif
// the multi-chunk instances' 32-bit edge addresses not made opaque per use (A/B switch, off: 16
// fewer v_mov per wave and iteration on C4, but 12.04 against 11.26 ms, r6d)
#ifndef BS_VAO
#define BS_VAO 0
#endif
// the multi-chunk instances read the PAD slot at the positions past a chunk's real ones instead
// of filling their registers with ~0 behind a branch (C4 11.26 -> 10.84 ms, r6d)
#ifndef BS_SKRD
#define BS_SKRD 1
#endif
// the variable phases' frame-error words: every lane ORs its word into one of BS_FLORW LDS words
// (lane & 31: two lanes per word, distinct banks) and wave 0 folds them at the next iteration's
// top, instead of a wave_or (4 DPP + 4 readlane, ~34 issue cycles) and a lane-0 atomic in every
// wave (A/B switch; the last iteration keeps the wave reduction, with its APP and bit counts)
#ifndef BS_FLOR
#define BS_FLOR 1
#endif
static_assert(!BS_FLOR || BS_TIDFREE, "BS_FLOR: wave 0 folds the words with all its lanes");
#define BS_FLORW 32
// the prologue's wave priority (A/B switch): the channel, tables and first variable phase of a
// new workgroup compete with the other resident workgroups' iterations, whose check phases run
// at priority 1-2, and at 0 take only the issue slots those leave (-1, default: 3 on the
// instances whose loop runs PRIO 4 -- wman: same box, r6c, 4.482 -> 4.454 ms over three rounds --
// 0 elsewhere: C3 12.71 against 12.75 ms)
#ifndef BS_PROPRIO
#define BS_PROPRIO -1
#endif

// Register budget: the small instances run at 64 VGPRs (WPE 8: three 9-wave workgroups per CU).
// At a 72-register budget only two were resident (the waves of a workgroup are not spread evenly
// over the SIMDs): measured 7.56 ms (72 VGPRs) -> 6.51 ms (64) per 2^20-codeword C2 decode.
// XP: the hard-bit export build (a.hdx: every iteration's hard decisions, for the hard_bits /
// synd_bits outputs); the counters-only build is the one the bench and the sweeps run.
// LB: the workgroup size bound (64 NW for the multi-chunk instances: the register budget is
// 512 / (waves per SIMD), which a 1024-lane bound would fix at 128)
// Q8: the channel generated in the prologue (a.gen: ldpc_decode_awgn) instead of read as float
// LLRs; a build of its own (a run-time branch moved the register allocation of the whole kernel: C3's
// spills 5 -> 9 VGPRs)
template <int D, int DV, int LPC, int VPL, int CPL, bool UCN, bool BIG, bool PK, int WPE, bool XP, int LB, bool Q8>
__global__ void __launch_bounds__(LB) __attribute__((amdgpu_waves_per_eu(WPE)))
k_bs(BsArgs a) {
    static_assert(LPC == 2 || LPC == 4, "lanes per check");
    constexpr int SB = (DV * QMAX + QMAX <= 127) ? 8 : 9;     // planes of S and of lw + S
    constexpr int EPL = (D + LPC - 1) / LPC;                     // edge slots per check lane
    constexpr bool SKIPM = CPL > 1;                              // chunk-wide padding skipped
    constexpr int OB = 4 / LPC;                                  // alpha-table output bits per lane
    constexpr int VNA = PK ? (DV + 1) / 2 : DV;                  // address words per variable
    constexpr int VNW = VNA + 1;
    constexpr int HDW = (EPL + 1) / 2;                           // packed hd addresses per check lane
    constexpr bool PKG = PK && CPL == 1 && BS_PKG;               // slot base | alpha table << 16
    // pass 2 reads its slots again instead of holding all EPL of them from pass 1 (wide checks:
    // 30 registers at the check phase's peak, where the 80-register C3 build spilled)
    constexpr bool RR = BS_REREAD && EPL >= 6;
    // the multi-chunk instances read the PAD slot at the positions past a chunk's real ones
    constexpr bool SKRD = BS_SKRD && CPL > 1 && BS_BSMIN && BS_BSMIN_MC && !RR;
    constexpr bool T0A = BS_T0ASYNC < 0 ? (VPL == 1 && CPL == 1) : BS_T0ASYNC != 0;
    constexpr bool EBR = BS_EB < 0 ? T0A : BS_EB != 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if ((uint32_t)(uintptr_t)smem != 0u) __builtin_trap();          // slots are LDS-absolute
#ifdef BS_STAMP
    // per-wave phase times (wave-uniform, s_memtime shader clocks): where a wave's time goes,
    // barrier waits included (diagnostic builds only)
    uint64_t sacc[13] = {};
    uint64_t sts = __builtin_amdgcn_s_memtime();
#define BS_ST(i)                                                                                   \
    do {                                                                                           \
        const uint64_t tn_ = __builtin_amdgcn_s_memtime();                                         \
        sacc[i] += tn_ - sts;                                                                      \
        sts = tn_;                                                                                 \
    } while (0)
#else
#define BS_ST(i) ((void)0)
#endif
    const int tid = threadIdx.x;
    const int NT = blockDim.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwv = NT >> 6;
    const int nv = a.n_vars;
    const int64_t b0 = (int64_t)blockIdx.x * PACK;
    const int nvalid = (int)min<int64_t>(PACK, a.B - b0);
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);   // [0] wrong_t, [1] all t, [2] APP > 0, [3] bits
    const int flor = 16 + ((a.T + 3) & ~3);                         // (BS_FLOR) the 32 OR words
    const int AR = UCN ? 2 * a.arows : a.arows;
    const int AL = AR * LUT_W, BL = a.bcols * BLUT_W;
    uint32_t* ALUT = reinterpret_cast<uint32_t*>(smem + a.off_alut);   // [2][AR][LUT_W]
    uint32_t* BLUT = reinterpret_cast<uint32_t*>(smem + a.off_blut);   // [2][bcols][BLUT_W]
    const bool ucn = UCN && a.ucn;
    // UCN work of iteration t's check phase (the syndromes, the alpha' table) and of the hard
    // decisions the variable phase writes for it: skipped where alpha'_t = alpha_t
    auto ucn_on = [&](int t) __attribute__((always_inline)) -> bool {
        return ucn && (t >= 64 || ((a.ucn_iter >> t) & 1));
    };

    constexpr int PROPRIO = BS_PROPRIO >= 0 ? BS_PROPRIO
                            : ((BS_PRIO < 0 && VPL == 1 && CPL == 1 && DV >= 6) || BS_PRIO == 4 ? 3 : 0);
    if (PROPRIO > 0) __builtin_amdgcn_s_setprio(PROPRIO);
    // ---- per-lane variables: slot addresses, variable index, degree bounds of the wave ----------
    uint32_t va[VPL][VNA];
    int vv[VPL], dw[VPL], dwmin[VPL], pcol[VPL];
    uint32_t tab_b[VPL];
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        const uint32_t* vt = a.vn_tab + ((size_t)u * NT + tid) * VNW;
        // (the slot addresses: loaded after the LLR prologue when the lane holds several
        // variables, where they would only add to the registers the LLR loads hold)
        if (!(BS_LLR_ALL && VPL > 1)) {
#pragma unroll
            for (int p = 0; p < VNA; ++p) va[u][p] = vt[p];
        }
        vv[u] = (int)vt[VNA];                                // -1: no variable (UCN: v | HD index << 16)
        dw[u] = __builtin_amdgcn_readfirstlane(a.vn_wdeg[3 * (u * nwv + wave)]);
        dwmin[u] = __builtin_amdgcn_readfirstlane(a.vn_wdeg[3 * (u * nwv + wave) + 1]);
        pcol[u] = __builtin_amdgcn_readfirstlane(a.vn_wdeg[3 * (u * nwv + wave) + 2]);
        tab_b[u] = (a.bcols > 1 && vv[u] >= 0) ? (uint32_t)(((UCN ? (vv[u] & 0xFFFF) : vv[u]) / (nv / a.bcols)) * BLUT_W * 4) : 0u;
    }
    int cn_dmin = a.cn_dmin;

    // ---- channel planes: the lane's variables for the 32 codewords of the pack ------------------
    // (no __syncthreads_or: it allocates static LDS, which would move the dynamic LDS base
    // away from 0; the flag word lives in RED)
    // one workgroup per CU: the first generation starts in lockstep, and with every pack taking
    // the same time, each later generation again fetches its LLR blocks in one chip-wide burst
    // while HBM idles the rest of the pack.  Spreading the first starts over a pack's duration
    // keeps the fetches apart for the whole grid (later workgroups inherit the offsets).
    if (a.stagger > 0 && (int)blockIdx.x < a.stagger_n) {
        const int n = (int)(((uint32_t)blockIdx.x * 97u % (uint32_t)a.stagger_n) * (uint32_t)a.stagger /
                            (uint32_t)a.stagger_n);
        for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(8);
    }
    // PAD slot (all ones: V->C negative, magnitude 15), ZERO slot (a zero C->V), the zero hard
    // decision word of UCN padding edges, the counters and the off-grid flag RED[7]; iteration
    // 0's tables are copied global -> LDS asynchronously (global_load_lds) behind the channel
    // loads, retired by the channel barrier (through registers, each thread's loads waited in
    // turn: three L2 round trips and a barrier of their own per pack)
    if (tid < SLOT_W) {
        reinterpret_cast<uint32_t*>(smem + a.off_pad)[tid] = 0xFFFFFFFFu;
        reinterpret_cast<uint32_t*>(smem + a.off_zero)[tid] = 0u;
    }
    if (UCN && tid == 0) lds_put(a.off_hdz, 0u);
    if (tid < 8) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
#ifdef BS_STAMP
    if (tid == 0) {
        uint32_t hw0;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw0));
        RED[12] = (hw0 >> 4) & 3u;
    }
#endif
    if (BS_FLOR && tid < BS_FLORW) RED[flor + tid] = 0u;
    // (the barrier that orders these writes before the channel's flag updates: here when the
    // channel is generated from the sampler's tables; else after the first variable's LLR loads
    // are issued, so that it waits beside their HBM round trip, BS_EB)
    if constexpr (Q8) gen_tables(a.gen, tid, NT);
    if (Q8 || !EBR) __syncthreads();
    BS_ST(8);
    uint32_t cs[VPL], cm[VPL][4], bg[VPL];
    int off = 0;
    if (T0A) {                           // (retired by the channel barrier's vmcnt(0))
        copy_async(a.off_alut, a.alut, AL, wave, NT);
        copy_async(a.off_blut, a.blut, BL, wave, NT);
    }
    // all 32 loads of a variable issued before any use: one HBM round trip per workgroup
    // prologue (with batches of 8 the LLR fetch cost 0.75 ms of a 6.5 ms C2 decode, with this
    // 0.44 ms: the workgroups stay in step, so every pack boundary is a chip-wide HBM burst; a
    // persistent grid prefetching the next pack during the check phases needed 6 more
    // loop-carried registers and spilled: 7.56 ms).
    // the pack's LLR rows through a buffer descriptor (wave-uniform base and size): each load is
    // buffer_load_dword with the lane's 4 v in voffset and the row's 4 r nv in soffset, so no
    // load needs a 64-bit VGPR address (with them the multi-variable lanes spilled the loaded
    // values and waited for each load in turn); rows past the batch read 0
    const __amdgpu_buffer_rsrc_t llr_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.llr + b0 * nv), 0, nvalid * nv * 4, 0x00020000);
    auto llr_at = [&](int r, int v) __attribute__((always_inline)) -> float {
        if (BS_BUFLD)
            return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(llr_rs, 4 * v, 4 * r * nv, BS_LLR_CPOL));
        return a.llr[(b0 + min(r, nvalid - 1)) * nv + v];
    };
    auto var_of = [&](int u) __attribute__((always_inline)) -> int {
        return (UCN && vv[u] >= 0) ? (vv[u] & 0xFFFF) : vv[u];
    };
    // lanes with several variables (VPL > 1, one workgroup per CU: nothing else hides the fetch)
    // issue variable u + 1's loads while converting variable u's (BS_LLR_ALL), so the fetch is
    // one round trip without holding every variable's 32 values at once
    float xv[VPL][PACK];
    if constexpr (Q8) {
        // generated channel (ldpc_decode_awgn): the grid bytes of the lane's variables from the
        // Philox stream, packed into planes as pack_channel's; never off the grid
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            cs[u] = 0u;
            bg[u] = 0u;
#pragma unroll
            for (int p = 0; p < 4; ++p) cm[u][p] = 0u;
            const int v = var_of(u);
            if (v >= 0 && !ABL(32)) {
                uint32_t Dq[8];
                gen_bytes(a.gen, blockIdx.x, v, a.qmax, Dq);
                pack_bytes<BIG>(Dq, valid, cs[u], cm[u], bg[u]);
            }
        }
    } else {
    if (var_of(0) >= 0 && !ABL(32)) {
#pragma unroll
        for (int r = 0; r < PACK; ++r) xv[0][r] = llr_at(r, var_of(0));
    }
    if (EBR) {
        // (a workgroup barrier without __syncthreads' fence, whose vmcnt(0) would wait for the
        // loads just issued: the LDS writes above complete (lgkmcnt(0)) and the compiler keeps
        // every memory access on its side)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0), vmcnt / expcnt untouched
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        cs[u] = 0u;
        bg[u] = 0u;
#pragma unroll
        for (int p = 0; p < 4; ++p) cm[u][p] = 0u;
        const int v = var_of(u);
        const int u1 = u + 1 < VPL ? u + 1 : u;
        const int vn = (u + 1 < VPL && !ABL(32)) ? var_of(u1) : -1;
        const bool inter = BS_LLR_ALL && v >= 0 && vn >= 0 && !ABL(32);   // next loads interleaved
        if (BS_PACKT && v >= 0 && !ABL(32)) {
            if (inter) {
#pragma unroll
                for (int r = 0; r < PACK; ++r) xv[u1][r] = llr_at(r, vn);
            }
            off |= pack_channel<BIG>(xv[u], a.inv, a.qmax, a.cu, valid, cs[u], cm[u], bg[u]);
        } else if (v >= 0 && !ABL(32)) {
#pragma unroll
            for (int r = 0; r < PACK; ++r) {
                if (inter) xv[u1][r] = llr_at(r, vn);
                const float x = xv[u][r] * a.inv;
                const float xr = rintf(x);
                const bool big = BIG && fabsf(x) == a.cu;       // a shortened bit (a.cu > qmax)
                off |= ((xr != x || fabsf(xr) > (float)a.qmax) && !big) ? 1 : 0;
                const int xi = (r < nvalid) ? (big ? (x < 0.f ? -a.qmax : a.qmax) : (int)xr) : 0;
                const uint32_t m = (uint32_t)(xi < 0 ? -xi : xi);
                cs[u] |= (xi < 0 ? 1u : 0u) << r;
                if (BIG) bg[u] |= (big && r < nvalid ? 1u : 0u) << r;
#pragma unroll
                for (int p = 0; p < 4; ++p) cm[u][p] |= ((m >> p) & 1u) << r;
            }
        }
        if (vn >= 0 && !inter) {
#pragma unroll
            for (int r = 0; r < PACK; ++r) xv[u1][r] = llr_at(r, vn);
        }
    }
    }
    if (off) atomicOr(&RED[7], 1u);
    BS_ST(9);
    __syncthreads();
    BS_ST(10);
    if (RED[7]) {                              // off the grid: the v5 fixup decodes this pack
        if (tid == 0) a.bad[blockIdx.x] = 1u;
        return;
    }
    if (tid == 0) a.bad[blockIdx.x] = 0u;
    if (BS_CH_LDS) {
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            v4u c4;
            c4.x = cm[u][0];
            c4.y = cm[u][1];
            c4.z = cm[u][2];
            c4.w = cm[u][3];
            *reinterpret_cast<LdsQ*>(a.off_ch + 16u * (uint32_t)(tid * VPL + u)) = c4;
        }
    }
    if (!T0A) {
        for (int w = tid; w < AL; w += NT) ALUT[w] = a.alut[w];
        for (int w = tid; w < BL; w += NT) BLUT[w] = a.blut[w];
        __syncthreads();
    }
    BS_ST(11);

    // ---- variable phase -------------------------------------------------------------------------
    //   first: lw_0 as every edge's V->C (no C->V yet);
    //   else:  S = sum of the C->V, APP_t = Q(ch) + S (hard decision, counters); unless last,
    //          Tv = clamp(Q(beta_{t+1} ch) + S) and V->C_e = clamp(Tv - C->V_e, +-15) per edge
    //   UCN:   the hard decision (APP_t >= 0; first: lw_0 >= 0) to HD[v] for the next check phase
    constexpr bool BKPF = !XP && BS_BFIX && !BS_BTID_LDS && (BS_BKPF == 2 || (BS_BKPF == 1 && VPL > 1));
    // the one-chunk UCN instance (802.11n: 108 checks x 4 lanes fill 7 of 12 waves): the
    // check-idle waves evaluate the next variable phase's channel tables during the check phase
    constexpr bool PREB = (BS_PREB < 0 ? (UCN && VPL == 1 && CPL == 1) : BS_PREB != 0) && VPL == 1 &&
                          CPL == 1 && !XP && !BS_BTID_LDS;
    int bkp[VPL];                        // (BKPF) the ids of iteration tb's tables, loaded early
#pragma unroll
    for (int u = 0; u < VPL; ++u) bkp[u] = -1;
    // |Q(beta_tb ch)| (4 planes) of the lane's variable u: the identity table, one of the fixed
    // set (wave-uniform id: a jump into immediate truth tables), the iteration's table in
    // constant memory (one beta per iteration) or the LDS table words (bslice).  pre: evaluated
    // ahead, in the check phase, where the LDS tables of iteration tb may still be in flight:
    // returns false (nothing done) for the paths that read them
    auto beta_lw = [&](const int u, const uint32_t bslice, const int tb, const uint32_t (&cmu)[4],
                       uint32_t (&lw)[4], const bool use_bk, const bool pre, const bool nobig)
                       __attribute__((always_inline)) -> bool {
        int bk = -1;
        if constexpr (!XP && BS_BFIX) {
            if (use_bk && a.btid) {
                const int col = (a.bcols == 1) ? 0 : pcol[u];
                if (BKPF) bk = __builtin_amdgcn_readfirstlane(bkp[u]);
                else if (col >= 0)   // (BS_BTID_S: a scalar load, through the constant address space)
                    bk = __builtin_amdgcn_readfirstlane(
                        BS_BTID_LDS ? (int)lds_w(a.off_btid + 4u * (uint32_t)col)
                        : BS_BTID_S ? (int)((const ConstW*)a.btid)[(size_t)tb * a.btid_n + col]
                                    : a.btid[(size_t)tb * a.btid_n + col]);
            }
        }
        // identity table: |Q(beta ch)| = |ch| (the mask covers iterations 0..63)
        if (ABL(2) || (tb < 64 && ((a.beta_id >> tb) & 1))) {
            PH("vn_beta_id", u);
#pragma unroll
            for (int i = 0; i < 4; ++i) lw[i] = cmu[i];
        } else if (bk >= 0 && bk < kNBetaTab) {   // a table of the fixed set
            if (pre && BIG && a.bcols > 1 && !nobig) return false;
            PH("vn_beta_fix", u);
            beta_asm(lw, cmu, bk);
            if constexpr (BIG) {            // shortened bits: |Q(beta cu)| from the table words
                if (a.bcols == 1) {
                    const ConstW* tg = (const ConstW*)(a.blut) + (size_t)tb * BLUT_W;
#pragma unroll
                    for (int i = 0; i < 4; ++i) lw[i] = mux(bg[u], tg[LUT_W + i], lw[i]);
                } else if (!pre) {          // (pre: no shortened bit in the wave)
                    const v4u gb = lds_q(bslice + tab_b[u] + LUT_W * 4);
                    lw[0] = mux(bg[u], gb.x, lw[0]);
                    lw[1] = mux(bg[u], gb.y, lw[1]);
                    lw[2] = mux(bg[u], gb.z, lw[2]);
                    lw[3] = mux(bg[u], gb.w, lw[3]);
                }
            }
        } else if (a.bcols == 1) {          // one beta per iteration: table in SGPRs
            PH("vn_beta_sg", u);
            const ConstW* tg = (const ConstW*)(a.blut) + (size_t)tb * BLUT_W;
            lut_s(lw, cmu, tg);
            if constexpr (BIG) {
#pragma unroll
                for (int i = 0; i < 4; ++i) lw[i] = mux(bg[u], tg[LUT_W + i], lw[i]);
            }
        } else {
            if (pre) return false;
            PH("vn_beta_lds", u);
            const uint32_t btab = bslice + tab_b[u];
            const uint32_t cmi[1][4] = {{cmu[0], cmu[1], cmu[2], cmu[3]}};
            uint32_t lo[1][4];
            lut<1>(lo, cmi, btab);
#pragma unroll
            for (int i = 0; i < 4; ++i) lw[i] = lo[0][i];
            if constexpr (BIG) {
                const v4u gb = lds_q(btab + LUT_W * 4);
                lw[0] = mux(bg[u], gb.x, lw[0]);
                lw[1] = mux(bg[u], gb.y, lw[1]);
                lw[2] = mux(bg[u], gb.z, lw[2]);
                lw[3] = mux(bg[u], gb.w, lw[3]);
            }
        }
        return true;
    };
    // (PREB) the check-idle waves' |Q(beta_{t+1} ch)|, evaluated during the check phase of
    // iteration t (their lanes hold no check), read back by the variable phase
    bool preb_done = false;
    // (no shortened bit in any lane of the wave: the fixed tables' shortened-bit planes unneeded)
    const bool nobig = !BIG || __builtin_amdgcn_ballot_w64(bg[0] != 0u) == 0ull;
    // (the lane's 16 B, recomputed at each use from the lane id: no address held through the loop)
    auto pre_addr = [&]() __attribute__((always_inline)) -> uint32_t {
        const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        return a.off_preb + 16u * ((uint32_t)(wave * 64 - a.cn_lanes) + ln);
    };
    auto vn_phase = [&](const bool first, const bool last, const uint32_t bslice, const int tb)
                        __attribute__((always_inline)) {
        uint32_t wr = 0u, apos = 0u, nb = 0u;
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            // a (wave, u) place without a variable chunk (dw = -1, wave-uniform): nothing to do
            // (5G BG2: 20 chunks on 32 places; their beta table and Tv work used to run anyway)
            if (BS_VSKIP && VPL > 1 && dw[u] < 0) continue;
            PH("vn_setup", (last ? 100 : 0) + u);
#pragma unroll
            for (int p = 0; p < VNA; ++p) {
                // (PK: unpacked per use, not hoisted as twice the registers; the 32-bit
                // addresses of the multi-chunk instances need no unpacking, and the opaque copy
                // made them loop-carried values the allocator moved at every iteration's end:
                // 16 v_mov per wave on C4, BS_VAO)
                if (PK || !BS_VAO) asm volatile("" : "+v"(va[u][p]));
            }
            auto vaddr = [&](int f) __attribute__((always_inline)) -> uint32_t {
                if constexpr (PK) return (f & 1) ? (va[u][f >> 1] >> 16) : (va[u][f >> 1] & 0xFFFFu);
                else return va[u][f];
            };
            const int v = (UCN && vv[u] >= 0) ? (vv[u] & 0xFFFF) : vv[u];
            const uint32_t hda = UCN ? 4u * ((uint32_t)vv[u] >> 16) : 0u;     // HD slot (rotated)
            uint32_t cmu[4] = {cm[u][0], cm[u][1], cm[u][2], cm[u][3]};
            if (BS_CH_LDS) {
                int tl = tid;
                asm volatile("" : "+v"(tl));
                const v4u c4 = lds_q(a.off_ch + 16u * (uint32_t)(tl * VPL + u));
                cmu[0] = c4.x;
                cmu[1] = c4.y;
                cmu[2] = c4.z;
                cmu[3] = c4.w;
            }
            const bool counted = v >= 0 && v < a.target_bits;
            uint32_t lw[1][4];                   // |Q(beta_{t+1} ch)| (before the C->V: fewer live registers)
            PH("vn_beta", (last ? 100 : 0) + u);
            if (!last) {
                if (PREB && !first && preb_done) {          // (evaluated in the check phase)
                    const v4u q = lds_q(pre_addr());
                    lw[0][0] = q.x;
                    lw[0][1] = q.y;
                    lw[0][2] = q.z;
                    lw[0][3] = q.w;
                } else {
                    (void)beta_lw(u, bslice, tb, cmu, lw[0], !first, false, false);
                }
            }
            // C->V of the first KEEP edges stay in registers for the V->C pass, the others are read
            // again: wman 3 of 6 (BS_KEEP), 802.11n all four (BS_KEEP_DV; three and the fourth
            // read again before round 5, 14.48 -> 14.41 ms, r3zh), 5G BG2 7 of 8 (BS_KEEP_MC), 4
            // with UCN (BS_KEEP_MCU)
            constexpr int KEEP0 = (VPL > 1 || CPL > 1) ? (UCN ? BS_KEEP_MCU : BS_KEEP_MC) : BS_KEEP;
            constexpr int KEEP = DV <= BS_KEEP_DV ? DV : (KEEP0 < DV ? KEEP0 : DV - 1);
            const int dwu = dw[u];
            // the rest at SBX planes of S: the fewest that hold 15 dw + 15 for the place's largest
            // degree dw (wave-uniform), BS_SBV
            auto vbody = [&](auto sbc) __attribute__((always_inline)) {
                constexpr int SB = decltype(sbc)::value;
                uint32_t mn[KEEP > 0 ? KEEP : 1], mb[KEEP > 0 ? KEEP : 1][4];
                uint32_t S[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) S[i] = 0u;
                if (!first) {
#pragma unroll
                    for (int f = 0; f < DV; ++f) {
                        if (f < dwu) {
                            PH("vn_sum", 1000 * (SB - 6) + (last ? 100 : 0) + 10 * u + f);
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
                    if constexpr (SB == 8) PH8("vn_app", 1000 * (SB - 6) + (last ? 100 : 0) + u, S, (S + 4));
                    else PH("vn_app", 1000 * (SB - 6) + (last ? 100 : 0) + u);
                    // APP_t = Q(ch) + S: the sign (hard decision) from the carry chain alone, the full
                    // sum only in the last iteration (APP > 0 for the loss counter)
                    uint32_t hd, nz = 0u;
                    const uint32_t c_s = cs[u];
                    if (last) {
                        uint32_t A[SB];
#pragma unroll
                        for (int i = 0; i < SB; ++i) A[i] = S[i];
                        const uint32_t cb[4] = {cmu[0] ^ c_s, cmu[1] ^ c_s, cmu[2] ^ c_s, cmu[3] ^ c_s};
                        add_b<SB>(A, cb, c_s);
                        hd = ~A[SB - 1];
#pragma unroll
                        for (int i = 0; i < SB; ++i) nz |= A[i];
                    } else {
                        uint32_t c = c_s;
#pragma unroll
                        for (int i = 0; i < SB - 1; ++i) c = B3(T_MAJ, S[i], i < 4 ? (cmu[i] ^ c_s) : c_s, c);
                        hd = B3(T_XNOR3, S[SB - 1], c_s, c);
                    }
                    if (UCN && !last && v >= 0 && ucn_on(tb)) lds_put(hda, hd);   // HD[v] (Main_Functions.py:184-188)
                    hd &= valid;                                     // APP >= 0 -> hard decision 1
                    if constexpr (XP) {                              // iteration tb - 1's hard decisions
                        if (v >= 0) a.hdx[((size_t)(tb - 1) * (size_t)((a.B + 31) >> 5) + blockIdx.x) * nv + v] = hd;
                    }
                    if (ABL(8)) hd = 0u;
                    if (counted) {
                        wr |= hd;
                        if (last) {
                            apos |= hd & nz;
                            nb += (uint32_t)__popc(hd);
                        }
                    }
                }
                if (last) return;
                if constexpr (SB == 8) PH8("vn_tv", 1000 * (SB - 6) + (last ? 100 : 0) + u, S, (S + 4));
                else PH("vn_tv", 1000 * (SB - 6) + (last ? 100 : 0) + u);
                // Tv = clamp(Q(beta ch) + S): the table gives |Q(beta ch)|, the channel the sign
                uint32_t lb[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) lb[i] = lw[0][i] ^ cs[u];
                add_b<SB>(S, lb, cs[u]);
                uint32_t Tv[6];
                clamp6<SB>(Tv, S);
                const int dwm = dwmin[u];
                if (first) {
                    // UCN at t = 0: the hard decision of x~ = Q(beta_0 ch) (Main_Functions.py:181-182)
                    if (UCN && v >= 0 && ucn_on(0)) lds_put(hda, ~Tv[5]);
                    uint32_t x[7], X[4];
#pragma unroll
                    for (int i = 0; i < 7; ++i) x[i] = Tv[i < 6 ? i : 5];
                    abs_sat(X, x);
#pragma unroll
                    for (int f = 0; f < DV; ++f)
                        if (f < dwu && (f < dwm || vaddr(f) != a.off_zero)) write_slot(vaddr(f), x[6], X);
                } else {
#pragma unroll
                    for (int f = 0; f < DV; ++f) {
                        if (f < dwu) {
                            if (ABL(4)) continue;
                            PH("vn_vc", 1000 * (SB - 6) + (last ? 100 : 0) + 10 * u + f);
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
                            if (f < dwm || vaddr(f) != a.off_zero) write_slot(vaddr(f), x[6], X);
                        }
                    }
                }
            };
            constexpr int SBSET = BS_SBV_SET >= 0 ? BS_SBV_SET : ((VPL == 1 && CPL == 1) ? 3 : 2);
            if constexpr (BS_SBV && SB >= 8) {
                if ((SBSET & 1) && dwu * QMAX + QMAX <= 63) vbody(std::integral_constant<int, 7>{});
                else if ((SBSET & 2) && SB == 9 && dwu * QMAX + QMAX <= 127) vbody(std::integral_constant<int, (SB == 9 ? 8 : SB)>{});
                else vbody(std::integral_constant<int, SB>{});
            } else {
                vbody(std::integral_constant<int, SB>{});
            }
        }
        if (!first && BS_FLOR && !last) {
            PH("vn_flags", 0);
            if (!ABL(8)) {
                const uint32_t la = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) & 31u;
                __hip_atomic_fetch_or(RED + flor + la, wr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else if (!first) {
            PH("vn_flags", last ? 100 : 0);
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
    };

    if (BS_LLR_ALL && VPL > 1) {
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
            const uint32_t* vt = a.vn_tab + ((size_t)u * NT + tid) * VNW;
#pragma unroll
            for (int p = 0; p < VNA; ++p) va[u][p] = vt[p];
        }
    }
    vn_phase(true, false, a.off_blut, 0);
    BS_ST(12);
    // check groups: chunk k of 64 check lanes; lane LPC c + j of it (check c = row i, index h)
    // takes edges k = LPC m + j, at slots first_i + j A_i + m z + h (a.row_lay); edges past the
    // degree read the all-ones PAD slot and are not written; idle lanes (c >= n_checks) read PAD
    // only.  (Lane j of a check's group evaluates alpha-table output bits OB j .. OB j + OB - 1:
    // 16 words per bit, at 64 B per bit.)
    const int cj = lane % LPC;
    int gchunk[CPL], gdeg[CPL], gm[CPL];
    // fixed-set check tables: the chunk's first row | (first lane of the next row) << 16 (64: one
    // row); -1: its checks span more than two rows (the table words then)
    int grow[CPL];
    uint32_t gbase[CPL], gtab[CPL], ghd[CPL][UCN ? HDW : 1];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        gchunk[c] = (CPL == 1) ? wave : __builtin_amdgcn_readfirstlane(a.cn_chunk[wave * CPL + c]);
        const int ql = max(gchunk[c], 0) * 64 + lane;
        const int cc = ql / LPC;
        const int ci = min(cc / a.z, a.n_checks / a.z - 1);
        gdeg[c] = (cc < a.n_checks) ? a.row_ptr[ci + 1] - a.row_ptr[ci] : 0;
        // edge positions m holding a real edge for some lane of the chunk (wave-uniform): the
        // positions past them are padding for every lane and skipped (LPC, an even count, lanes
        // of each group skip together, so the group's [V->C >= 0] parity is unchanged)
        // (the instances with several check chunks per lane: 5G-type graphs, whose rows differ
        // in degree; the one-chunk instances serve near-regular rows and keep their registers)
        gm[c] = SKIPM ? (int)__popc(wave_or((1u << ((gdeg[c] + LPC - 1) / LPC)) - 1u)) : EPL;
        gbase[c] = a.off_slots + (uint32_t)((a.row_lay[2 * ci] + cj * a.row_lay[2 * ci + 1] + (cc - ci * a.z)) * SLOT_B);
        gtab[c] = a.off_alut + (uint32_t)((a.arows > 1 ? ci : 0) * LUT_W * 4) + (uint32_t)(cj * OB * 64);
        // (16-bit LDS addresses: the slot base and the alpha-table address share one register
        // through the T loop, unpacked per iteration)
        if constexpr (PKG) gbase[c] |= gtab[c] << 16;
        {
            const int ch = max(gchunk[c], 0), mr = a.n_checks / a.z - 1;
            const int c0 = ch * (64 / LPC);
            const int r0 = min(c0 / a.z, mr), r1 = min((c0 + 64 / LPC - 1) / a.z, mr);
            const int split = (r1 == r0) ? 64 : LPC * (r1 * a.z - c0);
            grow[c] = __builtin_amdgcn_readfirstlane(a.arows == 1 ? (64 << 16) : (r1 - r0 > 1 ? -1 : (r0 | split << 16)));
        }
        if constexpr (UCN) {
#pragma unroll
            // (the table holds the cn_lanes check lanes: a one-chunk instance's waves past them
            // read nothing -- their reads ran off the end of the allocation)
            for (int p = 0; p < HDW; ++p) ghd[c][p] = (ucn && gchunk[c] >= 0 && ql < a.cn_lanes) ? a.cn_hd[(size_t)ql * HDW + p] : 0u;
        }
    }
    // the lane's real edge positions, one word for all its chunks (bit RB c + m: position m of
    // chunk c holds an edge of the lane's check), read through an opaque copy per iteration so
    // [LPC m + j < degree] is not hoisted out of the T loop as CPL x EPL 64-bit lane masks whose
    // SGPR pairs the loop spilled (bsc: 166 v_readlane reloads in the loop body before).  The
    // multi-chunk instances only: the one-chunk builds spill VGPRs with it (C2 3 -> 9, C3 7 -> 10)
    constexpr bool RPW = BS_RPW && CPL > 1;
    constexpr int RB = EPL;
    static_assert(CPL * RB <= 32, "real-position word");
    static_assert(!SKIPM || EPL <= 8, "BS_MIN2_CASE covers 1..8");
    uint32_t rpk = 0u;
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
        for (int m = 0; m < EPL; ++m)
            if (RPW && (LPC * m + LPC - 1 < cn_dmin || LPC * m + cj < gdeg[c])) rpk |= 1u << (RB * c + m);
    const uint32_t cstride = (uint32_t)(a.z * SLOT_B);
    const uint32_t tabu = (uint32_t)(a.arows * LUT_W * 4);        // alpha' tables after the alpha ones
    constexpr bool GBL = BS_GBLDS && CPL == 1 && !BS_CH_LDS;
    constexpr bool ALDS = GBL && PK && BS_ALDS;
    constexpr int HWA = (EPL + 1) / 2;                            // (ALDS) address words per check lane
    // words per lane (ALDS: [lane][GW], an odd count, so a 32-lane group's reads of one word hit
    // 32 distinct banks; all of a lane's words read with immediate offsets from one address)
    constexpr int GW = ALDS ? ((1 + HWA) | 1) : 1;
    if constexpr (GBL) lds_put(a.off_ch + 4u * (uint32_t)(tid * GW), gbase[0]);
    if constexpr (ALDS) {
        const uint32_t b = gbase[0] & 0xFFFFu;
#pragma unroll
        for (int p = 0; p < HWA; ++p) {
            uint32_t w = 0u;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int m = 2 * p + h;
                const bool re = m < EPL && (LPC * m + LPC - 1 < cn_dmin || LPC * m + cj < gdeg[0]);
                w |= (re ? b + (uint32_t)m * (uint32_t)(a.z * SLOT_B) : a.off_pad) << (16 * h);
            }
            lds_put(a.off_ch + 4u * (uint32_t)(tid * GW + 1 + p), w);
        }
    }
    constexpr bool HDL = BS_HDLDS && UCN && CPL == 1;
    if constexpr (HDL) {
#pragma unroll
        for (int p = 0; p < HDW; ++p) lds_put(a.off_hdl + 4u * (uint32_t)(p * NT + tid), ghd[0][p]);
    }
    __syncthreads();

    // wave priorities (BS_PRIO: 1 the younger half of the workgroup at priority 1 for the whole
    // decode; 2 the check phase at priority 1, the variable phase at 0; 3 the reverse; 4 the
    // check phase at 2, the variable phase at 1 on the waves whose first place has degree >= DV - 1
    // and 0 on the others; 6 as 4 with the check phase at 1; 8 as 6 with those waves at 2; 9 the
    // waves with more than the mean work of each phase at 1)
    // (default: 4 on the one-chunk instances with DV >= 6 — wman, whose three degree-6 waves hold
    // twice the variable work of the other six: same box, r5aa, 4.59 -> 4.52 ms — 2 on the other
    // one-chunk instances — 802.11n, where nearly every wave is that heavy: 12.37 against 12.70 —
    // and 0 on the multi-chunk ones)
    constexpr int PRIO = BS_PRIO >= 0 ? BS_PRIO : ((VPL == 1 && CPL == 1) ? (DV >= 6 ? 4 : 2) : 0);
    if (PRIO == 1 && wave >= (nwv >> 1)) __builtin_amdgcn_s_setprio(1);
    // PRIO 9: in each phase the waves with more than the mean work at priority 1 (variable phase:
    // 3 + the degree of each chunk the wave holds, from the dealing table; check phase: its chunks)
    bool heavy_v = false, heavy_c = false;
    if constexpr (PRIO == 9) {
        int own = 0, sum = 0, cown = 0, csum = 0;
        for (int w = 0; w < nwv; ++w) {      // (wave-uniform: scalar loads)
            int cw = 0, cc = 0;
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                const int d = __builtin_amdgcn_readfirstlane(a.vn_wdeg[3 * (u * nwv + w)]);
                cw += d >= 0 ? 3 + d : 0;
            }
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                cc += (CPL == 1 ? w * 64 < a.cn_lanes : __builtin_amdgcn_readfirstlane(a.cn_chunk[w * CPL + c]) >= 0) ? 1 : 0;
            sum += cw;
            csum += cc;
            if (w == wave) {
                own = cw;
                cown = cc;
            }
        }
        heavy_v = own * nwv > sum;
        heavy_c = cown * nwv > csum;
    }
    BS_ST(4);
    for (int t = 0; t < (ABL(16) ? 0 : a.T); ++t) {
        PH("top", 0);
        if ((BS_TIDFREE ? wave == 0 : tid == 0) && t > 0) {   // fold iteration t-1's frame flags
            // (every lane of wave 0 writes the same words: a wave-uniform branch, no thread
            // index kept live through the loop; kept in LDS for the iter_wrong export after the
            // loop: a global pointer held through it cost the 64-VGPR build 17 SGPR spill moves)
            uint32_t w0;
            if (BS_FLOR) {                    // (the 32 words of iteration t - 1, zeroed again)
                const uint32_t ln = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
                uint32_t x = ln < 32u ? RED[flor + ln] : 0u;
                if (ln < 32u) RED[flor + ln] = 0u;
                w0 = wave_or(x);
            } else {
                w0 = RED[0];
                RED[0] = 0u;
            }
            RED[16 + t - 1] = w0;
            RED[1] &= w0;
        }
        const int nx = (t + 1) & 1;
#pragma unroll
        for (int u = 0; u < VPL; ++u) asm volatile("" : "+s"(dw[u]), "+s"(dwmin[u]));   // compared per use, not hoisted as masks
        if (!RPW) asm volatile("" : "+s"(cn_dmin));
        // (the lane's variable made opaque per iteration on the multi-chunk instances: [v >= 0]
        // and [v < target bits] are compared per use, not held through the loop as spilled
        // 64-bit lane masks)
        if (BS_VVO == 2 || (BS_VVO && RPW)) {
#pragma unroll
            for (int u = 0; u < VPL; ++u) asm volatile("" : "+v"(vv[u]));
        }
        // next iteration's tables (their slots were last read two phases ago)
        if (t + 1 < a.T) {
            // (the lane index made opaque per iteration: the copy addresses are recomputed here
            // rather than hoisted out of the T loop into registers the loop body spills)
            if (BS_GLDS) {
                int cw = wave;
                if (!BS_TIDFREE) {                  // (the wave from an opaque thread index)
                    int tl = tid;
                    asm volatile("" : "+v"(tl));
                    cw = __builtin_amdgcn_readfirstlane(tl >> 6);
                }
                // (BS_TOPO: the copies' wave-uniform bounds made opaque per iteration, so their
                // compares are redone here instead of held through the loop as 64-bit lane masks)
                int al = AL, bl = BL, bcl = a.bcols;
                if (BS_TOPO && !(Q8 && VPL == 1 && CPL == 1 && !UCN))
                    asm volatile("" : "+s"(cw), "+s"(al), "+s"(bl), "+s"(bcl));
                // (BS_KARG: the tables' addresses loaded again from the kernel arguments each
                // iteration (scalar loads) instead of held through the loop, where they were
                // spilled to VGPR lanes and reloaded by v_readlane)
                const uint32_t* alut_p = a.alut;
                const uint32_t* blut_p = a.blut;
                uint32_t off_al = a.off_alut, off_bl = a.off_blut;
                // (one-chunk instances: the multi-chunk build spilled more with it, C4's loop
                // reloads 4 -> 44; wman's in-prologue channel build: its sweep step 0.4 % slower)
                if constexpr (BS_KARG && VPL == 1 && CPL == 1 && !(Q8 && !UCN)) {
                    typedef __attribute__((address_space(4))) const BsArgs ConstArgs;
                    ConstArgs* ka = (ConstArgs*)__builtin_amdgcn_kernarg_segment_ptr();
                    asm volatile("" : "+s"(ka));
                    alut_p = ka->alut;
                    blut_p = ka->blut;
                    off_al = ka->off_alut;
                    off_bl = ka->off_blut;
                }
                copy_async(off_al + 4u * (uint32_t)(nx * al), alut_p + (size_t)(t + 1) * al, al, cw, NT);
                if (bcl > 1)
                    copy_async(off_bl + 4u * (uint32_t)(nx * bl), blut_p + (size_t)(t + 1) * bl, bl, cw, NT);
                if (!XP && BS_BFIX && BS_BTID_LDS && a.btid)   // this iteration's variable phase: ids of row t + 1
                    copy_async(a.off_btid, reinterpret_cast<const uint32_t*>(a.btid) + (size_t)(t + 1) * a.btid_n,
                               a.bcols == 1 ? 1 : a.btid_n, cw, NT);
            } else {
                int tl = tid;
                asm volatile("" : "+v"(tl));
                for (int w = tl; w < AL; w += NT) ALUT[nx * AL + w] = a.alut[(size_t)(t + 1) * AL + w];
                if (a.bcols > 1)
                    for (int w = tl; w < BL; w += NT) BLUT[nx * BL + w] = a.blut[(size_t)(t + 1) * BL + w];
                if (!XP && BS_BFIX && BS_BTID_LDS && a.btid)
                    for (int w = tl; w < (a.bcols == 1 ? 1 : a.btid_n); w += NT)
                        lds_put(a.off_btid + 4u * (uint32_t)w, (uint32_t)a.btid[(size_t)(t + 1) * a.btid_n + w]);
            }
        }
        if constexpr (BKPF) {                // this iteration's variable phase: ids of row t + 1
            if (t + 1 < a.T && a.btid) {     // (the last variable phase takes no table)
#pragma unroll
                for (int u = 0; u < VPL; ++u) {
                    const int col = (a.bcols == 1) ? 0 : pcol[u];
                    bkp[u] = col >= 0 ? a.btid[(size_t)(t + 1) * a.btid_n + col] : -1;
                }
            }
        }
        // ======== check nodes ===================================================================
        if (PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if (PRIO == 3) __builtin_amdgcn_s_setprio(0);
        if (PRIO == 4) __builtin_amdgcn_s_setprio(2);
        if (PRIO == 6 || PRIO == 8) __builtin_amdgcn_s_setprio(1);
        if (PRIO == 9) {
            if (heavy_c) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if constexpr (PREB) {
            preb_done = false;
            if (a.off_preb && wave * 64 >= a.cn_lanes && t + 1 < a.T) {
                uint32_t cmu[4] = {cm[0][0], cm[0][1], cm[0][2], cm[0][3]};
                if (BS_CH_LDS) {
                    int tl = tid;
                    asm volatile("" : "+v"(tl));
                    const v4u c4 = lds_q(a.off_ch + 16u * (uint32_t)tl);
                    cmu[0] = c4.x;
                    cmu[1] = c4.y;
                    cmu[2] = c4.z;
                    cmu[3] = c4.w;
                }
                uint32_t lwp[4];
                if (beta_lw(0, 0u, t + 1, cmu, lwp, true, true, nobig)) {
                    v4u q;
                    q.x = lwp[0];
                    q.y = lwp[1];
                    q.z = lwp[2];
                    q.w = lwp[3];
                    *reinterpret_cast<LdsQ*>(pre_addr()) = q;
                    preb_done = true;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const bool active = (CPL == 1) ? (BS_TIDFREE ? wave * 64 < a.cn_lanes : tid < a.cn_lanes)
                                           : (gchunk[c] >= 0);   // (cn_lanes: 64 k)
            if (!active || ABL(1)) continue;
            PH("ck_addr", c);
            uint32_t cbase;
            uint32_t aw[ALDS ? HWA : 1];
            if constexpr (GBL) {
                // (the lane index from an operand the loop cannot hoist: a hoisted address was
                // itself held through the loop and spilled)
                uint32_t all = ~0u;
                asm volatile("" : "+s"(all));
                const uint32_t ln = __builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
                const uint32_t la = a.off_ch + ((uint32_t)wave << 8) * GW + 4u * GW * ln;
                cbase = lds_w(la);
                if constexpr (ALDS) {
#pragma unroll
                    for (int p = 0; p < HWA; ++p) aw[p] = lds_w(la + 4u * (uint32_t)(1 + p));
                }
            } else {
                cbase = gbase[c];
                asm volatile("" : "+v"(cbase));
            }
            uint32_t ctab = PKG ? (cbase >> 16) : gtab[c];
            if constexpr (PKG) cbase &= 0xFFFFu;
            int gmc = gm[c];
            asm volatile("" : "+s"(gmc));
            uint32_t rp = rpk;
            if (RPW) asm volatile("" : "+v"(rp));
            const int cdeg = gdeg[c];
            // slot m of the lane: a real edge (always while LPC m + LPC - 1 < cn_dmin)
            auto real = [&](int m) __attribute__((always_inline)) -> bool {
                if constexpr (RPW) return ((rp >> (RB * c + m)) & 1u) != 0u;
                else return LPC * m + LPC - 1 < cn_dmin || LPC * m + cj < cdeg;
            };
            auto caddr = [&](int m) __attribute__((always_inline)) -> uint32_t {
                if constexpr (ALDS) return (m & 1) ? (aw[m >> 1] >> 16) : (aw[m >> 1] & 0xFFFFu);
                else return real(m) ? cbase + m * cstride : a.off_pad;
            };
            // (ALDS) pass 2's test: real for the whole wave while LPC m + LPC - 1 < cn_dmin, else
            // the lane's address is not the PAD slot's
            auto real2 = [&](int m) __attribute__((always_inline)) -> bool {
                if constexpr (ALDS) return LPC * m + LPC - 1 < cn_dmin || caddr(m) != a.off_pad;
                else return real(m);
            };
            // pass 1: two minima of |V->C| and the parity of [V->C >= 0] over the lane's edges
            // (padding edges: negative, magnitude 15), then merged across the lane group
            // (the lane's EPL slots are read once, all loads issued before any use, and kept
            // in registers for pass 2)
            uint32_t Xs[EPL][4], ns[EPL];
            PH("ck_read", c);
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                if (SKIPM && !SKRD && m >= gmc) {    // padding for the whole chunk
                    // (SKRD: read like the others -- the PAD slot, every lane the same address,
                    // a broadcast -- instead of a branch that fills 5 registers per position with
                    // ~0 at every check phase: 54 v_mov per C4 chunk pair.  Left unset instead,
                    // the 128-VGPR build spilled)
#pragma unroll
                    for (int i = 0; i < 4; ++i) Xs[m][i] = ~0u;
                    ns[m] = ~0u;
                } else {
                    read_slot(ns[m], Xs[m], caddr(m));
                }
            }
            // UCN: syndrome of the previous hard decisions over the check (padding edges read a
            // zero word): odd -> the check is unsatisfied, its messages weighted by alpha'
            uint32_t syn = 0u;
            PH("ck_syn", c);
            const bool ucn_t = ucn_on(t);
            if constexpr (UCN) {
                if (ucn_t) {
                    // (the packed addresses made opaque per iteration: unpacked per use, not
                    // hoisted out of the T loop as EPL registers that the loop then spilled;
                    // HDL: read from LDS, through a lane index the loop cannot hoist)
                    uint32_t hwv[HDW];
                    if constexpr (HDL) {
                        uint32_t all = ~0u;
                        asm volatile("" : "+s"(all));
                        const uint32_t ln = __builtin_amdgcn_mbcnt_hi(all, __builtin_amdgcn_mbcnt_lo(all, 0u));
#pragma unroll
                        for (int p = 0; p < HDW; ++p)
                            hwv[p] = lds_w(a.off_hdl + 4u * (uint32_t)(p * NT) + ((uint32_t)wave << 8) + 4u * ln);
                    } else {
#pragma unroll
                        for (int p = 0; p < HDW; ++p) {
                            asm volatile("" : "+v"(ghd[c][p]));
                            hwv[p] = ghd[c][p];
                        }
                    }
#pragma unroll
                    for (int m = 0; m < EPL; ++m) {
                        if (SKIPM && m >= gmc) continue;
                        const uint32_t hw = hwv[m >> 1];
                        syn ^= lds_w((m & 1) ? (hw >> 16) : (hw & 0xFFFFu));
                    }
                    syn ^= qperm<QP_X1>(syn);
                    if (LPC == 4) syn ^= qperm<QP_X2>(syn);
                }
            }
            PH4("ck_min", c, Xs[EPL - 1]);
            uint32_t m1[4] = {Xs[0][0], Xs[0][1], Xs[0][2], Xs[0][3]}, m2[4] = {~0u, ~0u, ~0u, ~0u};
            uint32_t par = ns[0];
            // (BSM: the bit-serial search; cand[m] = [|V->C| of slot m = m1] for pass 2)
            constexpr bool BSM = BS_BSMIN && !RR && (!SKIPM || BS_BSMIN_MC);
            uint32_t cand[BSM ? EPL : 1];
            if constexpr (BSM) {
                // (padding positions: ~0, an even count of them over the LPC lanes of a group)
#pragma unroll
                for (int m = 1; m < EPL; ++m) par ^= ns[m];
                if constexpr (SKIPM) {
                    switch (gmc) {                   // wave-uniform: the chunk's real positions
#define BS_MIN2_CASE(k)                                                                            \
    case k:                                                                                        \
        if constexpr (k <= EPL) {                                                                  \
            PH("ck_mink", 16 * c + k);                                                             \
            min2_bits<k, LPC>(m1, m2, cand, Xs);                                                   \
            if (BS_MIN2_Z) {                                                                       \
                _Pragma("unroll") for (int m = k; m < EPL; ++m) cand[m] = 0u;                      \
            }                                                                                      \
        } else if (BS_MIN2_U) {                                                                    \
            __builtin_unreachable();                                                               \
        }                                                                                          \
        break;
                        BS_MIN2_CASE(1) BS_MIN2_CASE(2) BS_MIN2_CASE(3) BS_MIN2_CASE(4) BS_MIN2_CASE(5)
                        BS_MIN2_CASE(6) BS_MIN2_CASE(7) BS_MIN2_CASE(8)
#undef BS_MIN2_CASE
                        default:
                            if (BS_MIN2_U) __builtin_unreachable();   // (an active chunk: 1 <= gmc <= EPL)
                            break;
                    }
                } else {
                    min2_bits<EPL, LPC>(m1, m2, cand, Xs);
                }
            } else if constexpr (!SKIPM && EPL >= 2) {
                // tournament: sort pairs (12 ops), merge sorted pairs (24) — 48 ops for four
                // edges against 56 for the running two-minima update (only the two values matter)
                sort2(m1, m2, Xs[0], Xs[1]);
                par ^= ns[1];
#pragma unroll
                for (int m = 2; m + 1 < EPL; m += 2) {
                    uint32_t b1[4], b2[4];
                    sort2(b1, b2, Xs[m], Xs[m + 1]);
                    merge2(m1, m2, b1, b2);
                    par ^= ns[m] ^ ns[m + 1];
                }
                if constexpr (EPL & 1) {
                    const uint32_t(&X)[4] = Xs[EPL - 1];
                    const uint32_t l1 = lt4(X, m1), l2 = lt4(X, m2);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        m2[i] = mux(l1, m1[i], mux(l2, X[i], m2[i]));
                        m1[i] = mux(l1, X[i], m1[i]);
                    }
                    par ^= ns[EPL - 1];
                }
            } else {
#pragma unroll
            for (int m = 1; m < EPL; ++m) {
                if (SKIPM && m >= gmc) continue;
                const uint32_t(&X)[4] = Xs[m];
                const uint32_t l1 = lt4(X, m1), l2 = lt4(X, m2);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    m2[i] = mux(l1, m1[i], mux(l2, X[i], m2[i]));
                    m1[i] = mux(l1, X[i], m1[i]);
                }
                par ^= ns[m];
            }
            }
            PH9("ck_merge", c, m1, m2, par);
            par ^= qperm<QP_X1>(par);
            if (!BSM) merge_lanes<QP_X1>(m1, m2);
            if (LPC == 4) {
                par ^= qperm<QP_X2>(par);
                if (!BSM) merge_lanes<QP_X2>(m1, m2);
            }
            // message k is negative iff an even number of the OTHER edges have V->C >= 0
            // (Main_Functions.py:251-254): par ^ n_k, par the parity of [V->C >= 0] over the
            // LPC EPL slots (an even count, padding included)
            // weighted, quantized minima: each lane evaluates OB output bits, the group shares them
            uint32_t q1[4], q2[4];
            PH9("ck_tab", c, m1, m2, par);
            {
                const uint32_t mm[2][4] = {{m1[0], m1[1], m1[2], m1[3]}, {m2[0], m2[1], m2[2], m2[3]}};
                const uint32_t tab = ctab + (uint32_t)((t & 1) * AL * 4);
                uint32_t qb[OB][2];
                // alpha' is needed only where a check is unsatisfied for some codeword: a wave
                // whose checks are all satisfied in all 32 codewords (most waves once the
                // frames have converged) skips its table (the same messages, exactly)
                bool any_unsat = false;
                if constexpr (UCN) any_unsat = ucn_t && (!(BS_USKIP && CPL > 1) || __builtin_amdgcn_ballot_w64(syn != 0u) != 0ull);
                // tables of the fixed set: every lane evaluates all 4 bits of both minima with
                // immediate truth tables (no table words, no lane exchange)
                bool fixed = false;
                if (BS_AFIX && a.atid && grow[c] >= 0) {
                    const int r0 = grow[c] & 0xFFFF, split = grow[c] >> 16;
                    const int32_t* at = a.atid + (size_t)t * AR;
                    const int k0 = __builtin_amdgcn_readfirstlane(at[r0]);
                    const int k1 = split < 64 ? __builtin_amdgcn_readfirstlane(at[r0 + 1]) : k0;
                    int u0 = 0, u1 = 0;
                    if (UCN && any_unsat) {
                        u0 = __builtin_amdgcn_readfirstlane(at[a.arows + r0]);
                        u1 = split < 64 ? __builtin_amdgcn_readfirstlane(at[a.arows + r0 + 1]) : u0;
                    }
                    fixed = min(min(k0, k1), min(u0, u1)) >= 0 && max(max(k0, k1), max(u0, u1)) < kNBetaTab;
                    if (fixed) {
                        alpha_fixed(q1, q2, m1, m2, k0, k1, split);
                        if (UCN && any_unsat) {             // alpha' where the check is unsatisfied
                            uint32_t v1[4], v2[4];
                            alpha_fixed(v1, v2, m1, m2, u0, u1, split);
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                q1[i] = mux(syn, v1[i], q1[i]);
                                q2[i] = mux(syn, v2[i], q2[i]);
                            }
                        }
                    }
                }
                if (!fixed) {
#pragma unroll
                for (int b = 0; b < OB; ++b) {
                    uint32_t o[2];
                    lut_bit<2>(o, mm, tab + (uint32_t)(b * 64));
                    if constexpr (UCN) {
                        if (any_unsat) {              // alpha' where the check is unsatisfied
                            uint32_t ou[2];
                            lut_bit<2>(ou, mm, tab + tabu + (uint32_t)(b * 64));
                            o[0] = mux(syn, ou[0], o[0]);
                            o[1] = mux(syn, ou[1], o[1]);
                        }
                    }
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
            }
            // pass 2: an edge whose |V->C| equals the minimum gets the weighted second minimum
            // (if it is not the only one, the two minima are equal), the others the minimum
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                if (m == 0) PH8("ck_pass2", 16 * c, q1, q2);
                if (real2(m)) {
                    if (m > 0) PH("ck_pass2", 16 * c + m);
                    const uint32_t addr = ALDS ? caddr(m) : cbase + m * cstride;
                    uint32_t Mg[4];
                    if constexpr (BSM) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) Mg[i] = mux(cand[m], q2[i], q1[i]);
                        write_slot(addr, par ^ ns[m], Mg);
                    } else {
                    uint32_t X[4], n;
                    if constexpr (RR) {
                        read_slot(n, X, addr);       // (the slot still holds this edge's V->C)
                    } else {
                        n = ns[m];
#pragma unroll
                        for (int i = 0; i < 4; ++i) X[i] = Xs[m][i];
                    }
                    uint32_t ne = X[0] ^ m1[0];
#pragma unroll
                    for (int i = 1; i < 4; ++i) ne = B3(T_ORXOR, ne, X[i], m1[i]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) Mg[i] = mux(ne, q1[i], q2[i]);
                    write_slot(addr, par ^ n, Mg);
                    }
                }
            }
        }
        BS_ST(0);
        __syncthreads();
        BS_ST(1);
        // ======== variable nodes ================================================================
        if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
        if (PRIO == 3) __builtin_amdgcn_s_setprio(1);
        if (PRIO == 9) {
            if (heavy_v) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (PRIO == 4 || PRIO == 6 || PRIO == 8) {   // the waves of the heaviest variables first
            if (dw[0] >= DV - 1) __builtin_amdgcn_s_setprio(PRIO == 8 ? 2 : 1);
            else __builtin_amdgcn_s_setprio(0);
        }
        const uint32_t bslice = a.off_blut + (uint32_t)(nx * BL * 4);
        if (t == a.T - 1) vn_phase(false, true, bslice, t + 1);
        else vn_phase(false, false, bslice, t + 1);
        BS_ST(2);
        __syncthreads();
        BS_ST(3);
    }
    // the epilogue's output pointers (BS_KEPI: loaded from the kernel arguments here, not held
    // through the T loop from the kernel's entry)
    int64_t* e_counters = a.counters;
    uint8_t* e_flags = a.flags;
    uint32_t* e_iter_wrong = a.iter_wrong;
    int64_t e_B = a.B;
    // (not C4's decode build: more loop spills; not wman's decode build: 0.5 % slower)
    if constexpr (BS_KEPI && (Q8 || (VPL == 1 && CPL == 1 && UCN))) {
        typedef __attribute__((address_space(4))) const BsArgs ConstArgs;
        ConstArgs* ka = (ConstArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));
        e_counters = ka->counters;
        e_flags = ka->flags;
        e_iter_wrong = ka->iter_wrong;
        e_B = ka->B;
    }
    if (tid == 0) {
        const uint32_t wl = RED[0] & valid;
        const uint32_t all = RED[1] & RED[0] & valid;
        const uint32_t ap = RED[2] & valid;
        RED[16 + a.T - 1] = RED[0];
        if (e_counters) {
            unsigned long long* cc = reinterpret_cast<unsigned long long*>(e_counters);
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
    if (e_flags || e_iter_wrong) {
        __syncthreads();
        if (e_flags && tid < nvalid)
            e_flags[b0 + tid] = (uint8_t)(((RED[5] >> tid) & 1) | (((RED[6] >> tid) & 1) << 1));
        if (e_iter_wrong)                   // [T][packs]: iteration t's frame-error word
            for (int t = tid; t < a.T; t += NT)
                e_iter_wrong[(size_t)t * (size_t)((e_B + 31) >> 5) + blockIdx.x] = RED[16 + t] & valid;
    }
#ifdef BS_STAMP
    BS_ST(5);
    if (a.stamps && lane == 0 && wave < 16) {
#pragma unroll
        for (int i = 0; i < 13; ++i) atomicAdd(a.stamps + 16 * wave + i, (unsigned long long)sacc[i]);
        atomicAdd(a.stamps + 16 * wave + 15, 1ull);
        // the SIMD this wave ran on (HW_ID bits 5:4) relative to wave 0's (RED[12]): counts in
        // 32-bit fields, offsets 0-1 in word 13, 2-3 in word 14
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const uint32_t simd = (((hw >> 4) & 3u) - RED[12]) & 3u;
        atomicAdd(a.stamps + 16 * wave + 13 + (simd >> 1), 1ull << (32 * (simd & 1)));
    }
#endif
#undef BS_ST
}

template <int I, bool XP, bool Q8>
int launch_bs_x(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s) {
    constexpr BsInst k = kBsInst[I];
    constexpr int LB = (k.VPL > 1 || k.CPL > 1) ? 64 * k.NW : 1024;
    auto* fn = &k_bs<k.D, k.DV, k.LPC, k.VPL, k.CPL, k.UCN, k.BIG, k.PK, k.WPE, XP, LB, Q8>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)BS_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3(nblocks), dim3(64 * nw), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
template <int I>
int launch_bs(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s, bool q8) {
    // (the generated channel comes from ldpc_decode_awgn, which exports no hard bits)
    if (a.hdx) return q8 ? LDPC_ERR_UNSUPPORTED : launch_bs_x<I, true, false>(a, nblocks, nw, lds, s);
    return q8 ? launch_bs_x<I, false, true>(a, nblocks, nw, lds, s) : launch_bs_x<I, false, false>(a, nblocks, nw, lds, s);
}

// per-instance translation units (ldpc_bs_inst.hip, -DBS_INST=i)
template <int I>
int bs_launch(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s, bool q8);

}  // namespace bs
}  // namespace ldpc
