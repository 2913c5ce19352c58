// ldpc_host.h — the host-only half of the C ABI: graph tables, weight analysis and argument
// validation.  Plain C++17 with no HIP dependency, so that it builds with g++ under
// -fsanitize=address,undefined (tests/native/host_check.cpp, tests/test_host_sanitized.py) and
// is the same code ldpc_capi.hip runs before it touches the device.
//
// What it replaces in the reference: init_parameter / init_connecting_matrix
// (Main_Functions.py:8-150) build the lifted Tanner graph as dense (E z)^2 matrices; here the
// same graph is a row-major proto-edge list E(C) (the weight order, :69-71) with CSR offsets
// per proto row and column.  check_params (:498-523) is the reference's only validation; the
// decode-argument checks below are the ABI's own.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "ldpc_nms.h"

namespace ldpc {

// decoding modes (decoding_type x q_bit)
enum Mode : int { MODE_Q6 = 0, MODE_Q5, MODE_QM5, MODE_Q4, MODE_Q3, MODE_MS, MODE_MSNN, MODE_SP };
constexpr bool mode_is_qms(int m) { return m >= 0 && m <= MODE_Q3; }

inline int mode_of(int decoding_type, int q_bit) {
    if (decoding_type == LDPC_DEC_SP) return MODE_SP;
    if (decoding_type == LDPC_DEC_MS) return MODE_MS;
    if (decoding_type == LDPC_DEC_MS_NONUDGE) return MODE_MSNN;
    if (decoding_type != LDPC_DEC_QMS) return -1;
    switch (q_bit) {
        case 6: return MODE_Q6;
        case 5: return MODE_Q5;
        case -5: return MODE_QM5;
        case 4: return MODE_Q4;
        case 3: return MODE_Q3;
        default: return -1;
    }
}

namespace host {

constexpr int kMaxCheckDegree = 64;

// Lifted graph of a QC proto matrix (-1 = no edge, else cyclic shift, taken mod z).
struct GraphTables {
    int M = 0, N = 0, z = 0, E = 0;
    int max_cdeg = 0, max_vdeg = 0;
    std::vector<int32_t> row_ptr;    // [M+1] proto edges of row i: row_ptr[i] .. row_ptr[i+1]-1
    std::vector<int32_t> pe_row;     // [E] E(C) order (row-major)
    std::vector<int32_t> pe_col;     // [E]
    std::vector<int32_t> pe_shift;   // [E] P[i,j] mod z
    std::vector<int32_t> col_ptr;    // [N+1]
    std::vector<int32_t> col_pe;     // [E] proto edges of each column, ascending row
    // the device image: row_ptr | pe_row | pe_col | pe_shift | col_ptr | col_pe | pad to 16 B |
    // vn_edge [E] int4 {r0*z + (pe - r0), row degree, shift, (i*z) << 6 | (pe - r0)} in column order
    std::vector<int32_t> device_block;
    size_t off_vn = 0;               // int32 offset of vn_edge inside device_block
};

// LDPC_OK, LDPC_ERR_ARG (null / non-positive sizes / entry < -1 / no edge / sizes whose lifted
// counts overflow int32) or LDPC_ERR_UNSUPPORTED (check degree above kMaxCheckDegree).
int build_graph(const int32_t* proto, int32_t M, int32_t N, int32_t z, GraphTables& out);

// Per-iteration weight tables alpha [T][E], alpha_ucn [T][E] or null, beta [T][N]:
// per_edge_w = some row's CN / UCN weights differ inside the row at some t (sharing 1 / 4);
// row_merge[i] = row i may share fused-kernel check groups with row i-1 (equal degree, uniform
// row weights, the previous row's weights at every t).
// alpha_uniform = one CN weight for every edge at each t (sharing type 3, no UCN weights);
// beta_uniform = one VN weight for every column at each t; beta_nonneg = no beta below 0
// (the bit-sliced kernel takes the sign of Q(beta ch) from the channel); beta_one = every beta
// is 1 (flat weights: Q(beta ch) = Q(ch)).
struct WeightInfo {
    int per_edge_w = 0;
    int alpha_uniform = 0, beta_uniform = 0, beta_nonneg = 0, beta_one = 0;
    // alpha and (if given) alpha_ucn each one value per iteration (UCN decoders: one table pair
    // per iteration instead of one per row)
    int alpha_pair_uniform = 0;
    // bit t (t < 64): every column's q5/q-5 channel table of iteration t is the identity,
    // min(15, |rint(fl32(m beta))|) == m for m = 0..15 (the bit-sliced kernels skip it)
    uint64_t beta_id_mask = 0;
    // bit t (t < 64): alpha_ucn[t] differs from alpha[t] for some edge (with equal tables the
    // unsatisfied-check weighting of that iteration is the identity, Main_Functions.py:266-304)
    uint64_t ucn_iter_mask = 0;
    std::vector<int32_t> row_merge;
    // [T][N]: index into kBetaTab (ldpc_beta_tabs.h) of column j's q5 / q-5 channel table at
    // iteration t, min(15, |rint(fl32(m beta))|) for m = 0..15; -1 when beta < 0 or the table is
    // not in the set (the bit-sliced kernel then evaluates it from its table words)
    std::vector<int32_t> beta_tid;
};
// kBetaTab index of beta's q5 / q-5 channel table, or -1
int beta_table_id(float beta);
int analyze_weights(const GraphTables& g, int32_t T, const float* alpha, const float* alpha_ucn,
                    const float* beta, WeightInfo& out);

// ldpc_decode / ldpc_decode_awgn argument checks.  Returns LDPC_OK and the mode, or the status
// the ABI reports: LDPC_ERR_ARG (null params, bad mode, target_bits, clip_llr, kernel) or
// LDPC_ERR_STATE (B or T outside the context limits, weights missing or shorter than T).
int check_decode(const GraphTables& g, int64_t B, int64_t B_max, int32_t T_max, int32_t T_w,
                 const ldpc_decode_params* p, int* mode);

// ldpc_channel_awgn argument checks (LDPC_OK or LDPC_ERR_ARG).
int check_channel(int64_t B, int32_t n_vars, double sigma, int64_t offset, int32_t decoding_type,
                  int32_t q_bit, int32_t punct_start, int32_t punct_end, int32_t short_start,
                  int32_t short_end, float clip_llr);

// Variable-phase edge order.  A variable lane reads (and rewrites) its slots in edge order f, one
// LDS instruction per f for the whole wave; a half-wave (32 lanes) is served in one pass only
// when its 32 dword addresses fall in distinct banks (dword mod 32; identical addresses
// broadcast).  The slot layout is fixed by the check phase, but each lane may visit its own
// edges in any order (S is a sum; the V->C write-back is per edge), so the order is chosen per
// lane to minimise, over the rounds f, the largest number of distinct addresses sharing a bank:
// a deterministic hill climb over swaps of two edges of one lane.  Real edges stay in positions
// [0, degree) (the kernel treats positions below the wave's smallest degree as real).
// A[l * DV + f]: byte address of lane l's edge f; deg[l]: its degree; rounds: the wave's largest
// degree.  Returns the summed cost (cycles) before and after.
std::pair<int, int> order_variable_edges(std::vector<uint32_t>& A, const std::vector<int>& deg, int DV,
                                         int rounds);

// QMS channel level sampler (ldpc_awgn.h): the levels of Cal_MSA_Q (Print_Functions.py:12-25)
// for q_bit, their rounding boundaries x_j in LLR units, and the 64-bit fixed-point CDF
// thresholds T_j = P(LLR < x_j) 2^64 of the channel LLR = 2 (sigma n - 1) / sigma^2, n ~ N(0, 1)
// (create_mix_epoch, :29-72), from erfc in float64: for n_j = (x_j sigma^2 / 2 + 1) / sigma,
// T_j = floor(ldexp(erfc(-n_j / sqrt 2) / 2, 64)) when n_j < 0, else 2^64 - floor(ldexp(erfc(n_j /
// sqrt 2) / 2, 64)) (2^64 - 1 when that tail is 0; float64 erfc: about 2^-53 relative).  Writes nb (at most 32) boundaries, level
// values val[0..nb] and kmin = val[0] / grid step (the bit-sliced kernels' byte offset; 0 for
// q = 6, whose levels are not on one grid).  oracle/philox_oracle.py restates it.
void awgn_qms_levels(double sigma, int q_bit, int* nb, int* kmin, uint32_t* thr_hi, uint32_t* thr_lo,
                     float* val);

}  // namespace host
}  // namespace ldpc
