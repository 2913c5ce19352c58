// host_check.cpp — drives the host-only half of the C ABI (ldpc_host.cpp: graph tables, weight
// analysis, argument validation) under -fsanitize=address,undefined on the CPU.
// Built and run by tests/test_host_sanitized.py; test infrastructure, not product code.
//
//   host_check selftest              argument-validation cases + randomized graphs / weights
//   host_check tables FILE Z         the tables of a BaseGraph/*.txt proto as JSON on stdout
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <limits>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "ldpc_host.h"

using namespace ldpc;

static int failures = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                          \
        }                                                                        \
    } while (0)

// structural invariants of a built graph against the proto matrix it came from
static void check_tables(const std::vector<int32_t>& P, int M, int N, int z, const host::GraphTables& g) {
    int E = 0;
    for (int v : P) E += v != -1;
    CHECK(g.E == E && g.M == M && g.N == N && g.z == z);
    CHECK((int)g.row_ptr.size() == M + 1 && g.row_ptr[0] == 0 && g.row_ptr[M] == E);
    CHECK((int)g.col_ptr.size() == N + 1 && g.col_ptr[0] == 0 && g.col_ptr[N] == E);
    int e = 0, maxc = 0, maxv = 0;
    for (int i = 0; i < M; ++i) {
        CHECK(g.row_ptr[i] <= g.row_ptr[i + 1]);
        maxc = std::max(maxc, g.row_ptr[i + 1] - g.row_ptr[i]);
        for (int j = 0; j < N; ++j) {
            const int s = P[(size_t)i * N + j];
            if (s == -1) continue;
            CHECK(g.pe_row[e] == i && g.pe_col[e] == j && g.pe_shift[e] == s % z);
            CHECK(g.pe_shift[e] >= 0 && g.pe_shift[e] < z);
            ++e;
        }
    }
    for (int j = 0; j < N; ++j) {
        maxv = std::max(maxv, g.col_ptr[j + 1] - g.col_ptr[j]);
        for (int k = g.col_ptr[j]; k < g.col_ptr[j + 1]; ++k) {
            const int pe = g.col_pe[k];
            CHECK(pe >= 0 && pe < E && g.pe_col[pe] == j);
            if (k > g.col_ptr[j]) CHECK(g.pe_row[g.col_pe[k - 1]] < g.pe_row[pe]);
        }
    }
    CHECK(g.max_cdeg == maxc && g.max_vdeg == maxv);
    CHECK(g.off_vn % 4 == 0 && g.device_block.size() == g.off_vn + 4 * (size_t)E);
    for (int k = 0; k < E; ++k) {
        const int32_t* q = g.device_block.data() + g.off_vn + 4 * (size_t)k;
        const int pe = g.col_pe[k], i = g.pe_row[pe], r0 = g.row_ptr[i];
        CHECK(q[0] == r0 * z + (pe - r0) && q[1] == g.row_ptr[i + 1] - r0 && q[2] == g.pe_shift[pe] &&
              q[3] == (((i * z) << 6) | (pe - r0)));
    }
}

static void validation_cases() {
    host::GraphTables g;
    const int32_t p4[4] = {0, -1, 1, 0};
    CHECK(host::build_graph(nullptr, 2, 2, 4, g) == LDPC_ERR_ARG);
    CHECK(host::build_graph(p4, 0, 2, 4, g) == LDPC_ERR_ARG);
    CHECK(host::build_graph(p4, 2, -1, 4, g) == LDPC_ERR_ARG);
    CHECK(host::build_graph(p4, 2, 2, 0, g) == LDPC_ERR_ARG);
    const int32_t bad[4] = {-3, -1, 1, 0};
    CHECK(host::build_graph(bad, 2, 2, 4, g) == LDPC_ERR_ARG);
    const int32_t none[4] = {-1, -1, -1, -1};
    CHECK(host::build_graph(none, 2, 2, 4, g) == LDPC_ERR_ARG);
    // lifted sizes beyond int32 are refused (M*N*z bounds the edge count)
    CHECK(host::build_graph(p4, 2, 2, 1 << 29, g) == LDPC_ERR_ARG);
    CHECK(host::build_graph(p4, 2, 2, INT32_MAX, g) == LDPC_ERR_ARG);
    // check degree 65 > 64
    std::vector<int32_t> wide(65, 0);
    CHECK(host::build_graph(wide.data(), 1, 65, 1, g) == LDPC_ERR_UNSUPPORTED);
    std::vector<int32_t> w64(64, 3);
    CHECK(host::build_graph(w64.data(), 1, 64, 2, g) == LDPC_OK);
    check_tables(w64, 1, 64, 2, g);
    CHECK(host::build_graph(p4, 2, 2, 4, g) == LDPC_OK);
    check_tables(std::vector<int32_t>(p4, p4 + 4), 2, 2, 4, g);

    // weights
    host::WeightInfo wi;
    std::vector<float> a(3 * g.E, 0.75f), b(3 * g.N, 1.0f);
    CHECK(host::analyze_weights(g, 0, a.data(), nullptr, b.data(), wi) == LDPC_ERR_ARG);
    CHECK(host::analyze_weights(g, 3, nullptr, nullptr, b.data(), wi) == LDPC_ERR_ARG);
    CHECK(host::analyze_weights(g, 3, a.data(), nullptr, nullptr, wi) == LDPC_ERR_ARG);
    CHECK(host::analyze_weights(g, INT32_MAX, a.data(), nullptr, b.data(), wi) == LDPC_ERR_ARG);
    CHECK(host::analyze_weights(g, 3, a.data(), nullptr, b.data(), wi) == LDPC_OK);
    CHECK(wi.per_edge_w == 0 && (int)wi.row_merge.size() == g.M);
    CHECK(wi.beta_one == 1 && wi.beta_id_mask == 7u);          // beta = 1: identity tables
    // identity iff min(15, rint(15 beta)) == 15 and rint(m beta) == m below: 0.98 is (15 * 0.98
    // = 14.7), 0.96 is not (rint(14.4) = 14), 1.04 is not (rint(12 * 1.04 = 12.48) = 12 but
    // rint(13 * 1.04 = 13.52) = 14); one column off spoils the iteration
    for (int j = 0; j < g.N; ++j) {
        b[(size_t)0 * g.N + j] = 0.98f;
        b[(size_t)1 * g.N + j] = 0.96f;
        b[(size_t)2 * g.N + j] = j == 0 ? 1.04f : 1.0f;
    }
    CHECK(host::analyze_weights(g, 3, a.data(), nullptr, b.data(), wi) == LDPC_OK);
    CHECK(wi.beta_one == 0 && wi.beta_id_mask == 1u);
    std::fill(b.begin(), b.end(), 1.0f);
    // UCN iterations: bit t set when alpha'_t differs from alpha_t at some edge (the kernels
    // skip the unsatisfied-check work of the others); no alpha' -> no bit
    CHECK(host::analyze_weights(g, 3, a.data(), nullptr, b.data(), wi) == LDPC_OK && wi.ucn_iter_mask == 0u);
    {
        std::vector<float> u(a);
        u[(size_t)1 * g.E + (g.E - 1)] = 0.5f;               // iteration 1, last edge
        CHECK(host::analyze_weights(g, 3, a.data(), u.data(), b.data(), wi) == LDPC_OK);
        CHECK(wi.ucn_iter_mask == 2u);
        u[0] = 0.25f;                                         // iteration 0, first edge
        CHECK(host::analyze_weights(g, 3, a.data(), u.data(), b.data(), wi) == LDPC_OK);
        CHECK(wi.ucn_iter_mask == 3u);
        CHECK(host::analyze_weights(g, 3, a.data(), a.data(), b.data(), wi) == LDPC_OK);
        CHECK(wi.ucn_iter_mask == 0u);
    }

    // decode parameters
    ldpc_decode_params p{};
    p.T = 3; p.decoding_type = LDPC_DEC_QMS; p.q_bit = 5; p.target_bits = g.N * g.z;
    p.clip_llr = 20.f; p.kernel = LDPC_KERNEL_AUTO;
    int mode = -1;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &p, &mode) == LDPC_OK && mode == MODE_Q5);
    CHECK(host::check_decode(g, 10, 16, 5, 3, nullptr, &mode) == LDPC_ERR_ARG);
    CHECK(host::check_decode(g, 0, 16, 5, 3, &p, &mode) == LDPC_ERR_STATE);
    CHECK(host::check_decode(g, 17, 16, 5, 3, &p, &mode) == LDPC_ERR_STATE);
    CHECK(host::check_decode(g, 10, 16, 2, 3, &p, &mode) == LDPC_ERR_STATE);   // T > T_max
    CHECK(host::check_decode(g, 10, 16, 5, 2, &p, &mode) == LDPC_ERR_STATE);   // T > T_w
    ldpc_decode_params q = p;
    q.q_bit = 7;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.decoding_type = 9;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.target_bits = g.N * g.z + 1;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.target_bits = 0;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.clip_llr = std::numeric_limits<float>::quiet_NaN();
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.clip_llr = std::numeric_limits<float>::infinity();
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.kernel = 3;
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_ERR_ARG);
    q = p; q.decoding_type = LDPC_DEC_SP; q.q_bit = 99;     // q_bit is ignored outside QMS
    CHECK(host::check_decode(g, 10, 16, 5, 3, &q, &mode) == LDPC_OK && mode == MODE_SP);

    // channel parameters
    CHECK(host::check_channel(4, 10, 0.5, 0, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_OK);
    CHECK(host::check_channel(0, 10, 0.5, 0, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 0, 0.5, 0, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.0, 0, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, std::nan(""), 0, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, -1, 2, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, 0, 2, 2, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, 0, 5, 5, 0, 0, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, 0, 2, 5, 5, 3, 0, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, 0, 2, 5, 0, 0, -1, 0, 20.f) == LDPC_ERR_ARG);
    CHECK(host::check_channel(4, 10, 0.5, 0, 2, 5, 1, 2, 3, 4, 0.f) == LDPC_ERR_ARG);
}

// randomized protos (including empty rows / columns, shifts >= z, z = 1) and weight tables
static void fuzz(int rounds) {
    std::mt19937 rng(20251016);
    for (int r = 0; r < rounds; ++r) {
        const int M = 1 + rng() % 12, N = 1 + rng() % 40, z = 1 + rng() % 80;
        const double dens = (rng() % 100) / 100.0;
        std::vector<int32_t> P((size_t)M * N);
        for (auto& v : P) v = (rng() % 1000) / 1000.0 < dens ? (int32_t)(rng() % 400) : -1;
        host::GraphTables g;
        const int st = host::build_graph(P.data(), M, N, z, g);
        int E = 0;
        for (int v : P) E += v != -1;
        if (E == 0) { CHECK(st == LDPC_ERR_ARG); continue; }
        CHECK(st == LDPC_OK);
        if (st != LDPC_OK) continue;
        check_tables(P, M, N, z, g);
        const int T = 1 + rng() % 6;
        std::vector<float> a((size_t)T * g.E), u((size_t)T * g.E), b((size_t)T * g.N, 1.f);
        const bool per_row = rng() % 2;
        for (int t = 0; t < T; ++t)
            for (int e = 0; e < g.E; ++e) {
                const float w = per_row ? 0.5f + 0.01f * (float)(g.pe_row[e] % 3) : 0.5f + 0.01f * (float)(rng() % 50);
                a[(size_t)t * g.E + e] = w;
                u[(size_t)t * g.E + e] = w * 0.5f;
            }
        host::WeightInfo wi;
        CHECK(host::analyze_weights(g, T, a.data(), (rng() % 2) ? u.data() : nullptr, b.data(), wi) == LDPC_OK);
        CHECK((int)wi.row_merge.size() == M);
        if (per_row) CHECK(wi.per_edge_w == 0);
        for (int i = 1; i < M; ++i)
            if (wi.row_merge[i])
                CHECK(g.row_ptr[i + 1] - g.row_ptr[i] == g.row_ptr[i] - g.row_ptr[i - 1]);
    }
}

static int tables(const char* path, int z) {
    std::ifstream f(path);
    std::vector<int32_t> P;
    std::string line;
    int M = 0, N = -1;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        int v, n = 0;
        while (ss >> v) { P.push_back(v); ++n; }
        if (n == 0) continue;
        if (N < 0) N = n;
        if (n != N) { std::fprintf(stderr, "ragged proto\n"); return 2; }
        ++M;
    }
    host::GraphTables g;
    const int st = host::build_graph(P.data(), M, N, z, g);
    if (st != LDPC_OK) { std::printf("{\"status\": %d}\n", st); return 0; }
    check_tables(P, M, N, z, g);
    auto arr = [](const std::vector<int32_t>& v) {
        std::string s = "[";
        for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
        return s + "]";
    };
    std::printf("{\"status\": 0, \"M\": %d, \"N\": %d, \"E\": %d, \"max_cdeg\": %d, \"max_vdeg\": %d, "
                "\"row_ptr\": %s, \"pe_col\": %s, \"pe_shift\": %s, \"col_ptr\": %s, \"col_pe\": %s}\n",
                g.M, g.N, g.E, g.max_cdeg, g.max_vdeg, arr(g.row_ptr).c_str(), arr(g.pe_col).c_str(),
                arr(g.pe_shift).c_str(), arr(g.col_ptr).c_str(), arr(g.col_pe).c_str());
    return failures ? 1 : 0;
}


// bit-sliced variable-phase edge order (order_variable_edges): every lane keeps its edges, real
// edges stay in positions [0, degree), padding positions are untouched, the bank cost never rises,
// and a half-wave of one cyclic column block plus a second block's lanes is made conflict-free
static void vorder_cases(int rounds) {
    uint64_t r = 12345;
    auto rnd = [&](int n) { r = r * 6364136223846793005ull + 1442695040888963407ull; return (int)((r >> 33) % n); };
    auto cost = [](const std::vector<uint32_t>& A, int DV, int nr) {
        int c = 0;
        for (int h0 = 0; h0 < 64; h0 += 32)
            for (int f = 0; f < nr; ++f) {
                std::vector<uint32_t> seen;
                int cnt[32] = {0}, mx = 0;
                for (int l = h0; l < h0 + 32; ++l) {
                    const uint32_t a = A[(size_t)l * DV + f];
                    if (std::find(seen.begin(), seen.end(), a) != seen.end()) continue;
                    seen.push_back(a);
                    mx = std::max(mx, ++cnt[(a >> 2) & 31]);
                }
                c += mx;
            }
        return c;
    };
    for (int it = 0; it < rounds; ++it) {
        const int DV = 2 + rnd(7), nr = 1 + rnd(DV);
        const uint32_t zero = 4u * 100000u;
        std::vector<uint32_t> A((size_t)64 * DV, zero);
        std::vector<int> deg(64, 0);
        uint32_t next = 0;
        for (int l = 0; l < 64; ++l) {
            deg[l] = rnd(nr + 1);
            for (int f = 0; f < deg[l]; ++f) { next += 1 + rnd(40); A[(size_t)l * DV + f] = 20u * next; }
        }
        const std::vector<uint32_t> A0 = A;
        const int c0 = cost(A, DV, nr);
        const std::pair<int, int> c = host::order_variable_edges(A, deg, DV, nr);
        CHECK(c.first == c0 && c.second == cost(A, DV, nr) && c.second <= c.first);
        for (int l = 0; l < 64; ++l) {
            std::vector<uint32_t> a(A.begin() + (size_t)l * DV, A.begin() + (size_t)l * DV + deg[l]);
            std::vector<uint32_t> b(A0.begin() + (size_t)l * DV, A0.begin() + (size_t)l * DV + deg[l]);
            std::sort(a.begin(), a.end());
            std::sort(b.begin(), b.end());
            CHECK(a == b);
            for (int f = deg[l]; f < DV; ++f) CHECK(A[(size_t)l * DV + f] == zero);
        }
    }
    // lanes 0..23 of one column take banks 5l and 5(l + 8); lanes 24 + i of another column hold
    // an edge on bank 5i and one on bank 5(24 + i), in the order that collides in both rounds
    // (4 cycles); the reordered lanes 24..31 are conflict-free (2)
    const int DV = 2;
    std::vector<uint32_t> A((size_t)64 * DV, 4u * 100000u);
    std::vector<int> deg(64, 0);
    for (int l = 0; l < 32; ++l) {
        deg[l] = 2;
        const uint32_t i = (uint32_t)(l - 24);
        A[(size_t)l * DV] = 20u * (l < 24 ? (uint32_t)l : 32u * 50u + i);
        A[(size_t)l * DV + 1] = 20u * (l < 24 ? 32u * 70u + (uint32_t)l + 8u : 32u * 60u + 24u + i);
    }
    const std::pair<int, int> c = host::order_variable_edges(A, deg, DV, 2);
    CHECK(c.first == 4 + 2 && c.second == 2 + 2);   // (the empty second half-wave: 1 per round)
}

// the QMS level sampler's thresholds and level values (host::awgn_qms_levels) as JSON, for
// tests/test_host_sanitized.py to compare with oracle/philox_oracle.qms_levels
static int qms(double sigma, int q_bit) {
    int nb = 0, kmin = 0;
    uint32_t hi[64], lo[64];
    float val[65];
    host::awgn_qms_levels(sigma, q_bit, &nb, &kmin, hi, lo, val);
    std::printf("{\"nb\": %d, \"kmin\": %d, \"thr\": [", nb, kmin);
    for (int j = 0; j < nb; ++j)
        std::printf("%s%llu", j ? ", " : "", (unsigned long long)(((uint64_t)hi[j] << 32) | lo[j]));
    std::printf("], \"val\": [");
    for (int j = 0; j <= nb; ++j) std::printf("%s%.9g", j ? ", " : "", (double)val[j]);
    std::printf("]}\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "tables") return tables(argv[2], std::atoi(argv[3]));
    if (argc >= 4 && std::string(argv[1]) == "qms") return qms(std::atof(argv[2]), std::atoi(argv[3]));
    if (argc >= 2 && std::string(argv[1]) == "selftest") {
        validation_cases();
        fuzz(argc >= 3 ? std::atoi(argv[2]) : 3000);
        vorder_cases(500);
        std::printf("host_check: %d failures\n", failures);
        return failures ? 1 : 0;
    }
    std::fprintf(stderr, "usage: host_check selftest [rounds] | tables FILE Z\n");
    return 2;
}
