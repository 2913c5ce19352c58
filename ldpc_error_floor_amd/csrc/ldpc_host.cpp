// ldpc_host.cpp — host-only graph tables, weight analysis and argument validation of the C ABI
// (see ldpc_host.h).  No HIP: built into libldpc_nms.so by hipcc and, for the sanitized check,
// by g++ -fsanitize=address,undefined.
#include "ldpc_host.h"
#include "ldpc_beta_tabs.h"

#include <algorithm>
#include <climits>
#include <cmath>

namespace ldpc {
namespace host {

int build_graph(const int32_t* proto, int32_t M, int32_t N, int32_t z, GraphTables& g) {
    g = GraphTables{};
    if (!proto || M <= 0 || N <= 0 || z <= 0) return LDPC_ERR_ARG;
    // every lifted count the device code indexes with int: checks, variables, edges (<= M*N*z)
    if ((int64_t)M * N * z > INT32_MAX) return LDPC_ERR_ARG;
    g.M = M;
    g.N = N;
    g.z = z;
    g.row_ptr.assign((size_t)M + 1, 0);
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            const int32_t s = proto[(size_t)i * N + j];
            if (s < -1) return LDPC_ERR_ARG;
            if (s != -1) {
                g.pe_row.push_back(i);
                g.pe_col.push_back(j);
                g.pe_shift.push_back(s % z);
            }
        }
    g.E = (int)g.pe_row.size();
    if (g.E == 0) return LDPC_ERR_ARG;
    for (int e = 0; e < g.E; ++e) g.row_ptr[(size_t)g.pe_row[e] + 1]++;
    for (int i = 0; i < M; ++i) {
        g.max_cdeg = std::max(g.max_cdeg, g.row_ptr[(size_t)i + 1]);
        g.row_ptr[(size_t)i + 1] += g.row_ptr[i];
    }
    if (g.max_cdeg > kMaxCheckDegree) return LDPC_ERR_UNSUPPORTED;
    g.col_ptr.assign((size_t)N + 1, 0);
    for (int e = 0; e < g.E; ++e) g.col_ptr[(size_t)g.pe_col[e] + 1]++;
    for (int j = 0; j < N; ++j) {
        g.max_vdeg = std::max(g.max_vdeg, g.col_ptr[(size_t)j + 1]);
        g.col_ptr[(size_t)j + 1] += g.col_ptr[j];
    }
    g.col_pe.assign((size_t)g.E, 0);
    {
        std::vector<int32_t> fill(g.col_ptr.begin(), g.col_ptr.end() - 1);
        for (int e = 0; e < g.E; ++e) g.col_pe[(size_t)fill[(size_t)g.pe_col[e]]++] = e;   // ascending row
    }
    std::vector<int32_t>& h = g.device_block;
    h.insert(h.end(), g.row_ptr.begin(), g.row_ptr.end());
    h.insert(h.end(), g.pe_row.begin(), g.pe_row.end());
    h.insert(h.end(), g.pe_col.begin(), g.pe_col.end());
    h.insert(h.end(), g.pe_shift.begin(), g.pe_shift.end());
    h.insert(h.end(), g.col_ptr.begin(), g.col_ptr.end());
    h.insert(h.end(), g.col_pe.begin(), g.col_pe.end());
    while (h.size() % 4) h.push_back(0);
    g.off_vn = h.size();
    for (int e = 0; e < g.E; ++e) {
        const int pe = g.col_pe[(size_t)e], i = g.pe_row[(size_t)pe], r0 = g.row_ptr[(size_t)i];
        h.push_back(r0 * z + (pe - r0));
        h.push_back(g.row_ptr[(size_t)i + 1] - r0);
        h.push_back(g.pe_shift[(size_t)pe]);
        h.push_back(((i * z) << 6) | (pe - r0));      // first check of the row, position (ffl)
    }
    return LDPC_OK;
}

int beta_table_id(float b) {
    if (!(b >= 0.f)) return -1;
    uint8_t t[16];
    for (int m = 0; m < 16; ++m)
        t[m] = (uint8_t)std::min(15.f, std::fabs(std::nearbyint((float)m * b)));   // fp32 product, half to even
    int lo = 0, hi = kNBetaTab;             // (the set is in ascending order of the table sums)
    int sum = 0;
    for (int m = 0; m < 16; ++m) sum += t[m];
    for (int k = lo; k < hi; ++k) {
        int s = 0;
        for (int m = 0; m < 16; ++m) s += kBetaTab[k][m];
        if (s != sum) continue;
        if (std::equal(t, t + 16, kBetaTab[k])) return k;
    }
    return -1;
}

int analyze_weights(const GraphTables& g, int32_t T, const float* alpha, const float* alpha_ucn,
                    const float* beta, WeightInfo& w) {
    w = WeightInfo{};
    if (T <= 0 || !alpha || !beta || g.E <= 0) return LDPC_ERR_ARG;
    if ((int64_t)T * g.E > INT32_MAX || (int64_t)T * g.N > INT32_MAX) return LDPC_ERR_ARG;
    for (int t = 0; t < T && !w.per_edge_w; ++t)
        for (int i = 0; i < g.M && !w.per_edge_w; ++i)
            for (int e = g.row_ptr[(size_t)i] + 1; e < g.row_ptr[(size_t)i + 1]; ++e) {
                const size_t a0 = (size_t)t * g.E + g.row_ptr[(size_t)i], a1 = (size_t)t * g.E + e;
                if (alpha[a1] != alpha[a0] || (alpha_ucn && alpha_ucn[a1] != alpha_ucn[a0])) {
                    w.per_edge_w = 1;
                    break;
                }
            }
    w.row_merge.assign((size_t)g.M, 0);
    for (int i = 1; i < g.M && !w.per_edge_w; ++i) {
        const int deg = g.row_ptr[(size_t)i + 1] - g.row_ptr[(size_t)i];
        bool same = deg == g.row_ptr[(size_t)i] - g.row_ptr[(size_t)i - 1];
        // (an all -1 proto row has no weights to compare: row_ptr[i] may then be E, one past
        // the last weight of the iteration — found by the sanitized host check)
        for (int t = 0; t < T && same && deg > 0; ++t) {
            const size_t a0 = (size_t)t * g.E + g.row_ptr[(size_t)i - 1];
            const size_t a1 = (size_t)t * g.E + g.row_ptr[(size_t)i];
            same = alpha[a1] == alpha[a0] && (!alpha_ucn || alpha_ucn[a1] == alpha_ucn[a0]);
        }
        w.row_merge[(size_t)i] = same ? 1 : 0;
    }
    w.alpha_uniform = (!w.per_edge_w && !alpha_ucn) ? 1 : 0;
    w.alpha_pair_uniform = !w.per_edge_w ? 1 : 0;
    for (int t = 0; t < T && w.alpha_pair_uniform; ++t) {
        const size_t a0 = (size_t)t * g.E;
        for (int e = 1; e < g.E && w.alpha_pair_uniform; ++e)
            if (alpha[a0 + e] != alpha[a0] || (alpha_ucn && alpha_ucn[a0 + e] != alpha_ucn[a0]))
                w.alpha_pair_uniform = 0;
    }
    w.beta_uniform = 1;
    w.beta_nonneg = 1;
    w.beta_one = 1;
    for (int t = 0; t < T && t < 64; ++t) {
        bool id = true;
        for (int j = 0; j < g.N && id; ++j) {
            const float b = beta[(size_t)t * g.N + j];
            for (int m = 0; m <= 15 && id; ++m) {
                const float q = std::nearbyint((float)m * b);     // round half to even, fp32 product
                id = std::min(15.f, std::fabs(q)) == (float)m && !(b < 0.f);
            }
        }
        if (id) w.beta_id_mask |= (uint64_t)1 << t;
    }
    if (alpha_ucn)
        for (int t = 0; t < T && t < 64; ++t)
            for (int e = 0; e < g.E; ++e)
                if (alpha_ucn[(size_t)t * g.E + e] != alpha[(size_t)t * g.E + e]) {
                    w.ucn_iter_mask |= (uint64_t)1 << t;
                    break;
                }
    w.beta_tid.resize((size_t)T * g.N);
    for (size_t x = 0; x < (size_t)T * g.N; ++x) w.beta_tid[x] = beta_table_id(beta[x]);
    for (int t = 0; t < T; ++t) {
        const float a0 = alpha[(size_t)t * g.E], b0 = beta[(size_t)t * g.N];
        for (int e = 1; e < g.E && w.alpha_uniform; ++e)
            if (alpha[(size_t)t * g.E + e] != a0) w.alpha_uniform = 0;
        for (int j = 0; j < g.N; ++j) {
            const float b = beta[(size_t)t * g.N + j];
            if (b != b0) w.beta_uniform = 0;
            if (!(b >= 0.f)) w.beta_nonneg = 0;
            if (b != 1.f) w.beta_one = 0;
        }
    }
    return LDPC_OK;
}

int check_decode(const GraphTables& g, int64_t B, int64_t B_max, int32_t T_max, int32_t T_w,
                 const ldpc_decode_params* p, int* mode) {
    if (!p) return LDPC_ERR_ARG;
    if (B <= 0 || B > B_max || p->T <= 0 || p->T > T_max) return LDPC_ERR_STATE;
    if (T_w < p->T) return LDPC_ERR_STATE;
    const int m = mode_of(p->decoding_type, p->q_bit);
    if (m < 0) return LDPC_ERR_ARG;
    if (p->target_bits <= 0 || p->target_bits > g.N * g.z) return LDPC_ERR_ARG;
    if (!(p->clip_llr > 0.f) || !std::isfinite(p->clip_llr)) return LDPC_ERR_ARG;
    if (p->kernel != LDPC_KERNEL_AUTO && p->kernel != LDPC_KERNEL_FLOOD &&
        p->kernel != LDPC_KERNEL_FUSED)
        return LDPC_ERR_ARG;
    if (mode) *mode = m;
    return LDPC_OK;
}

int check_channel(int64_t B, int32_t n_vars, double sigma, int64_t offset, int32_t decoding_type,
                  int32_t q_bit, int32_t punct_start, int32_t punct_end, int32_t short_start,
                  int32_t short_end, float clip_llr) {
    if (B <= 0 || n_vars <= 0 || !(sigma > 0.0) || !std::isfinite(sigma) || offset < 0)
        return LDPC_ERR_ARG;
    if (mode_of(decoding_type, q_bit) < 0) return LDPC_ERR_ARG;
    if (punct_start < 0 || short_start < 0) return LDPC_ERR_ARG;
    if (punct_start > 0 && punct_end < punct_start) return LDPC_ERR_ARG;
    if (short_start > 0 && short_end < short_start) return LDPC_ERR_ARG;
    if (!(clip_llr > 0.f) || !std::isfinite(clip_llr)) return LDPC_ERR_ARG;
    return LDPC_OK;
}

std::pair<int, int> order_variable_edges(std::vector<uint32_t>& A, const std::vector<int>& deg, int DV,
                                         int rounds) {
    // cost of round f of the half-wave at lane h0: the most distinct addresses on one bank (the
    // cycles the access takes), and the sum of squared bank loads as the tie-break that lets the
    // climb leave plateaus of equal maxima
    auto round_cost = [&](int h0, int f) {
        uint32_t seen[32];
        int ns = 0, cnt[32] = {0}, mx = 0, sq = 0;
        for (int l = h0; l < h0 + 32; ++l) {
            const uint32_t ad = A[(size_t)l * DV + f];
            bool dup = false;
            for (int i = 0; i < ns && !dup; ++i) dup = seen[i] == ad;
            if (dup) continue;
            seen[ns++] = ad;
            const int c = ++cnt[(ad >> 2) & 31];
            mx = std::max(mx, c);
            sq += 2 * c - 1;
        }
        return mx * 4096 + sq;
    };
    int before = 0, after = 0;
    uint64_t rng = 0x9E3779B97F4A7C15ull;
    for (int h0 = 0; h0 < 64; h0 += 32) {
        std::vector<int> cost(rounds);
        std::vector<int> movable;
        for (int l = h0; l < h0 + 32; ++l)
            if (deg[l] >= 2) movable.push_back(l);
        for (int f = 0; f < rounds; ++f) {
            cost[f] = round_cost(h0, f);
            before += cost[f] / 4096;
        }
        for (int it = 0; it < 4000 && !movable.empty(); ++it) {
            rng = rng * 6364136223846793005ull + 1442695040888963407ull;
            const int l = movable[(rng >> 33) % movable.size()];
            const int f1 = (int)((rng >> 17) % (uint64_t)deg[l]);
            int f2 = (int)((rng >> 45) % (uint64_t)(deg[l] - 1));
            if (f2 >= f1) ++f2;
            std::swap(A[(size_t)l * DV + f1], A[(size_t)l * DV + f2]);
            const int c1 = round_cost(h0, f1), c2 = round_cost(h0, f2);
            if (c1 + c2 <= cost[f1] + cost[f2]) {
                cost[f1] = c1;
                cost[f2] = c2;
            } else {
                std::swap(A[(size_t)l * DV + f1], A[(size_t)l * DV + f2]);
            }
        }
        for (int f = 0; f < rounds; ++f) after += cost[f] / 4096;
    }
    return {before, after};
}

void awgn_qms_levels(double sigma, int q_bit, int* nb, int* kmin, uint32_t* thr_hi, uint32_t* thr_lo,
                     float* val) {
    double u, cmax;                       // grid step and clip of Cal_MSA_Q
    switch (q_bit) {
        case 6: u = 1.0; cmax = 15.5; break;
        case 5: u = 0.5; cmax = 7.5; break;
        case -5: u = 1.0; cmax = 15.0; break;
        case 4: u = 1.0; cmax = 7.0; break;
        default: u = 2.0; cmax = 6.0; break;
    }
    const int K = (int)std::ceil(cmax / u) + 1;
    auto Q = [&](int k) { return std::min(std::max(k * u, -cmax), cmax); };
    int n = 0;
    val[0] = (float)Q(-K);
    const double s2 = sigma * sigma;
    for (int k = -K + 1; k <= K; ++k) {
        if (Q(k) == Q(k - 1)) continue;
        const double x = (k - 0.5) * u;                       // rounding boundary, LLR units
        const double nz = (x * s2 * 0.5 + 1.0) / sigma;       // noise value at the boundary
        uint64_t T;
        if (nz < 0.0) {
            T = (uint64_t)std::ldexp(0.5 * std::erfc(-nz * 0.7071067811865476), 64);
        } else {
            const uint64_t tail = (uint64_t)std::ldexp(0.5 * std::erfc(nz * 0.7071067811865476), 64);
            // (a tail below 2^-64 rounds to 0: the threshold 2^64 - 1 gives that level
            // probability 2^-64 instead of its < 2^-64; oracle/philox_oracle.py does the same)
            T = tail == 0 ? ~(uint64_t)0 : (uint64_t)0 - tail;
        }
        thr_hi[n] = (uint32_t)(T >> 32);
        thr_lo[n] = (uint32_t)T;
        ++n;
        val[n] = (float)Q(k);
    }
    *nb = n;
    *kmin = q_bit == 6 ? 0 : (int)std::lround(-cmax / u);
}

}  // namespace host
}  // namespace ldpc
