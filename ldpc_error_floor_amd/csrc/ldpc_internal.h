// ldpc_internal.h — shared device-side types of the MI355X NMS decoder (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "ldpc_host.h"
#include "ldpc_nms.h"

namespace ldpc {

constexpr int TILE = 256;          // codewords per tile: 64 lanes x float4
constexpr int VN_PER_WAVE = 8;     // variables handled by one wave in vn_update

// Graph tables on the device (E(C) = row-major proto-edge order).
struct DevGraph {
    int M, N, z, E;
    int n_checks, n_vars, n_edges, max_cdeg;
    const int32_t* row_ptr;    // [M+1]
    const int32_t* pe_row;     // [E]
    const int32_t* pe_col;     // [E]
    const int32_t* pe_shift;   // [E]  P[i,j] mod z
    const int32_t* col_ptr;    // [N+1]
    const int32_t* col_pe;     // [E]  proto edges of each column, ascending row
    const int4* vn_edge;       // [E]  column order: {r0*z + (pe - r0), row degree, shift, (i*z) << 6 | (pe - r0)}
    const int32_t* h_row_ptr;  // [M+1] host copy of row_ptr (kernel planning)
    // [M] row i may share check groups with row i-1 (equal degree and weights; set by
    // ldpc_weights_set): host copy for planning, device copy for the address tables
    const int32_t* h_row_merge;
    const int32_t* row_merge;
    const host::GraphTables* host;   // host tables (ldpc_host.h)
    // weight properties of the current weights (host::WeightInfo, set by ldpc_weights_set)
    int w_alpha_uniform, w_beta_uniform, w_beta_nonneg, w_beta_one;
    int w_alpha_pair_uniform;            // alpha and alpha_ucn: one value per iteration each
    uint64_t w_beta_id_mask;     // iterations whose q5 channel table is the identity
    uint64_t w_ucn_iter;         // bit t (t < 64): iteration t's alpha' differs from its alpha
                                 // somewhere (UCN weighting matters); iterations >= 64: assumed
    const int32_t* beta_tid;     // [T][N] kBetaTab index of each column's q5 channel table, -1
    uint64_t w_version;          // incremented by every ldpc_weights_set (table caches)
};

// Per-decode buffers and scalars.
struct Bufs {
    float* ch;                 // [tiles][n_vars][256]  channel LLR
    float* Tv;                 // [tiles][n_vars][256]  lw + S (next iteration's VN total)
    float* c2v;                // [tiles][n_edges][256] C->V messages (check-major rows)
    uint64_t* hd;              // [slots][tiles][n_vars][4] hard decisions, ballot layout
    uint64_t* wrong;           // [T][tiles][4] frame has a 1 among target bits at t
    uint64_t* anypos;          // [tiles][4]    frame has APP > 0 among target bits at T-1
    int32_t* biterr;           // [tiles]       target bits = 1 at T-1
    float* app_out;            // [T][B][target_bits] or null
    const float* alpha;        // [T][E]
    const float* alpha_ucn;    // [T][E] or null
    const float* beta;         // [T][N]
    int64_t B;
    int ntiles, T, n_vars, target_bits;
    int hd_all;                // 1: hd kept for every iteration (slots T+1), 0: ring of 2
    int store_hd, count;
    float clip;
    const void* awgn;          // AwgnParams* (ldpc_awgn.h): generate the LLRs in the fused
                               // prologue instead of reading them (fused v5 only), or null
    uint32_t* iter_wrong;      // [T][ceil(B/32)] per-iteration frame-error words, or null
                               // (ldpc_decode_outputs::iter_wrong; zeroed before the decode)
    const uint32_t* q8;        // the bit-sliced kernels' in-prologue channel: its sampler tables
                               // (awgn_gen_table, device), with gen8, instead of LLRs; or null
    const void* gen8;          // AwgnParams* of that channel (with q8)
};

// Sum-product check update pieces (decoding_type 0, Main_Functions.py:238-245) shared by flood
// and the fused SP kernel, in the oracle's float32 arithmetic (oracle/nms_oracle.py _sp_check):
// t = fl32(tanh(fl32(-x / 2))) with t == 0 -> 1 (the reference's masking also swallows exact-
// zero messages), the product over the other edges in edge order in float32 (the caller's
// prefix x later edges), o = -2 fl32(atanh(clip(product, +-fl32(1 - 1e-7)))).  tanh and atanh
// are evaluated in float64 and rounded once, so they are the correctly rounded float32 values
// (the float32 library functions were a few ulps off, which atanh near the clip amplified to
// differences up to ~0.7 in an APP against the oracle).
__device__ __forceinline__ float sp_t(float x) {
    const float y = (float)tanh((double)(-0.5f * x));
    return (y != 0.f) ? y : 1.f;                                               // :240
}
__device__ __forceinline__ float sp_o(float others) {
    constexpr float SP_EPS = 1.0f - 1e-7f;            // float32(1 - 1e-7) = 0.99999988
    others = fminf(fmaxf(others, -SP_EPS), SP_EPS);                            // :243
    return -2.0f * (float)atanh((double)others);                               // :244
}

// per-iteration frame-error words (ldpc_decode_outputs::iter_wrong) of one block of codewords
// b0 .. b0 + CW - 1 (CW a power of two <= 64, b0 a multiple of CW) at iteration t: `m` holds
// bit r = codeword b0 + r (already masked to the valid codewords).  Blocks narrower than a word
// share it, so they OR into the zeroed buffer.
__device__ inline void put_iter_wrong(uint32_t* iw, int64_t B, int t, int64_t b0, int CW,
                                      unsigned long long m) {
    const int64_t nwd = (B + 31) >> 5;
    uint32_t* row = iw + (size_t)t * nwd;
    if (CW >= 32) {
        row[b0 >> 5] = (uint32_t)m;
        if (CW == 64 && (b0 >> 5) + 1 < nwd) row[(b0 >> 5) + 1] = (uint32_t)(m >> 32);
    } else if (m) {
        atomicOr(row + (b0 >> 5), (uint32_t)m << (b0 & 31));
    }
}

// hard decisions of iteration s (s = -1: prologue's lw_0) live in slot s+1 (or ring (s+1)&1)
__host__ __device__ inline size_t hd_index(const Bufs& p, int s, int64_t tile, int v) {
    const int slot = p.hd_all ? s + 1 : ((s + 1) & 1);
    return (((size_t)slot * p.ntiles + tile) * p.n_vars + v) * 4;
}

inline int64_t round_up8(int64_t x) { return (x + 7) & ~int64_t(7); }

int flood_decode(const DevGraph& g, const Bufs& b, const float* llr, int mode, bool ucn,
                 hipStream_t s);

}  // namespace ldpc
