// ldpc_fused5.hip — fused QMS decoder v5: per-decode tables, shape planning and dispatch.
// The kernel is in ldpc_fused5_kernel.h; each shape is compiled in its own translation unit
// (ldpc_fused5_shape.hip, -DF5_SHAPE=<index>) so the shapes build in parallel.
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldpc_fused5_kernel.h"

namespace ldpc {

namespace f5 {

// Per-decode weight table shared by every workgroup (beta needs none: the kernel keeps ch / step
// and reads beta as given, fl32(ch*beta)/step == fl32((ch/step)*beta)):
//   qtab[t][tab][row][m] = [+q, -q] bytes, q = Q(relu(|o| * w)), |o| = min(m, qmax) grid units
//                     for m <= 3 qmax (the kernel indexes by the unclamped |Tv - m|), m = 3 qmax
//                     + 1 stands for "no other edge" (the 10000 value), w = alpha_t,row
//                     (tab 0) or alpha_ucn_t,row (tab 1, UCN only); qslice halfwords per t
__global__ void k_f5_tables(const float* __restrict__ alpha, const float* __restrict__ alpha_ucn,
                            const int32_t* __restrict__ row_ptr, int T, int Mp, int E, int qmax,
                            float step, float inv, int qslice, uint16_t* qtab) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    const int nq = 3 * qmax + 2;               // |o| = 0 .. 3 qmax (min(|o|, qmax) used), none
    if (qtab && f < T * qslice) {
        const int tt = f / qslice, rem = f - tt * qslice;
        const int tab = rem / (Mp * nq), r2 = rem - tab * (Mp * nq);
        const int row = r2 / nq, m = r2 - row * nq;
        uint16_t v = 0;
        if (tab == 0 || (tab == 1 && alpha_ucn)) {
            const float w = (tab ? alpha_ucn : alpha)[(size_t)tt * E + row_ptr[row]];
            const int q = q_mag5(m == nq - 1 ? F5_BIG_U : min(m, qmax), w, step, inv, qmax);
            v = (uint16_t)(((uint32_t)q & 0xFFu) | (((uint32_t)(-q) & 0xFFu) << 8));
        }
        qtab[f] = v;
    }
}

// Check groups.  A run is a maximal range of consecutive proto rows that may share a group:
// row i continues row i-1's run when merge[i] != 0 (equal degree and, every iteration, equal
// CN / UCN weights: ldpc_weights_set).  A run's checks, row-major (z per row), are cut into
// groups of SLOTS consecutive checks, so only a run's last group idles lanes (one row per run:
// the last group of every row).  Groups are numbered run by run ("canonical" order).
__host__ __device__ inline int f5_run_groups(int nrows, int z, int slots) {
    return (nrows * z + slots - 1) / slots;
}
// f(first_row, nrows, degree) for every run, in row order; stops when f returns true
template <class F>
__host__ __device__ inline void f5_for_runs(const int32_t* row_ptr, const int32_t* merge, int M, F f) {
    for (int i = 0; i < M;) {
        int j = i + 1;
        while (j < M && merge && merge[j]) ++j;
        if (f(i, j - i, row_ptr[i + 1] - row_ptr[i])) return;
        i = j;
    }
}
inline int f5_ngroups(const int32_t* row_ptr, const int32_t* merge, int M, int z, int slots) {
    int n = 0;
    f5_for_runs(row_ptr, merge, M, [&](int, int nr, int) { n += f5_run_groups(nr, z, slots); return false; });
    return n;
}

// Table position s is what wave s % nw runs as its group s / nw.  bal = 0: position s is
// canonical group s.  bal = 1 (graphs with very unequal row degrees): groups are ranked by
// degree, heaviest first (ties in row order), and dealt to the waves in snake order (round r
// left to right when r is even, right to left when odd), so every wave's edge count is within
// one row's degree of the others'.
__device__ int f5_group_of(int s, const int32_t* __restrict__ row_ptr, const int32_t* merge, int M,
                           int z, int slots, int ngroups, int nw, int bal) {
    if (!bal) return s;
    const int r = s / nw, w = s - r * nw;
    const int nr = min(nw, ngroups - r * nw);               // groups dealt in round r
    const int rank = r * nw + ((r & 1) ? nr - 1 - w : w);
    int canon = 0, res = s;
    f5_for_runs(row_ptr, merge, M, [&](int i0, int n, int d) {
        const int ng = f5_run_groups(n, z, slots);
        int before = 0;                                     // groups ranked ahead of this run's
        f5_for_runs(row_ptr, merge, M, [&](int j0, int m, int d2) {
            if (d2 > d || (d2 == d && j0 < i0)) before += f5_run_groups(m, z, slots);
            return false;
        });
        if (rank >= before && rank < before + ng) {
            res = canon + (rank - before);
            return true;
        }
        canon += ng;
        return false;
    });
    return res;
}

// Edge addresses per (table position, lane): lane = slot * CW + cw serves check c = off * SLOTS
// + slot of its group's run (off: the group's index inside the run), i.e. circulant row h = c
// mod z of proto row i = first + c / z; edge k of that row reads W[(pe_col * z + (h + shift) mod
// z) * CW + cw], packed as byte offsets two per word.  Lanes past the run's last check point
// every edge at the lane's own dummy word (no two lanes' pass-2 atomics on one LDS word) and are
// masked out of the results.  grow: the run's first row (its weights stand for the run's),
// degree and the lane-valid mask.
__global__ void k_f5_gad(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ pe_col,
                         const int32_t* __restrict__ pe_shift, const int32_t* __restrict__ merge,
                         int M, int ngroups, int z, int logcw, int maxdeg, int npk, int total,
                         int nw, int bal, uint32_t* gad, uint4* grow) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= ngroups * 64) return;
    const int grp = f >> 6, lane = f & 63;
    const int cwn = 1 << logcw, slots = 64 >> logcw;
    const int slot = lane >> logcw, cw = lane & (cwn - 1);
    const int rg = f5_group_of(grp, row_ptr, merge, M, z, slots, ngroups, nw, bal);
    int first = 0, nrows = 1, off = rg;
    f5_for_runs(row_ptr, merge, M, [&](int i0, int n, int) {
        const int ng = f5_run_groups(n, z, slots);
        if (off < ng) {
            first = i0;
            nrows = n;
            return true;
        }
        off -= ng;
        return false;
    });
    const int deg = row_ptr[first + 1] - row_ptr[first];
    const int c = off * slots + slot;
    const bool valid = c < nrows * z;
    const int i = first + (valid ? c / z : 0);
    const int h = valid ? c - (c / z) * z : 0;
    const int r0 = row_ptr[i];
    for (int p = 0; p < npk; ++p) {
        uint32_t word = 0;
        for (int j = 0; j < 2; ++j) {
            const int k = 2 * p + j;
            uint32_t byte = (uint32_t)(total + lane) * 4u;            // dummy word of this lane
            if (valid && k < deg && k < maxdeg) {
                int hs = h + pe_shift[r0 + k];
                hs = (hs >= z) ? hs - z : hs;
                byte = (uint32_t)(((pe_col[r0 + k] * z + hs) << logcw) + cw) * 4u;
            }
            word |= byte << (16 * j);
        }
        gad[((size_t)grp * npk + p) * 64 + lane] = word;
    }
    if (lane == 0) {
        uint32_t lo = 0, hi = 0;
        for (int l = 0; l < 64; ++l)
            if (off * slots + (l >> logcw) < nrows * z) (l < 32 ? lo : hi) |= 1u << (l & 31);
        grow[grp] = make_uint4((uint32_t)row_ptr[first] | ((uint32_t)deg << 16) | ((uint32_t)first << 24),
                               lo, hi, 0u);
    }
}


size_t f5_lds(int nv, int cw, int T, int N) {
    (void)T;
    return ((((size_t)nv * cw + F5_NDUMMY) * 4 + (size_t)nv * cw * 4 + (size_t)2 * N * 4 + 15) & ~(size_t)15) + 8 * 8;
}

struct Plan5 {
    int shape = -1, nw = 0, ngroups = 0;
    const int32_t* merge = nullptr;      // device row-merge flags used (null: one row per run)
    size_t lds = 0;
};

Plan5 plan5(const DevGraph& g, int T) {
    Plan5 best;
    double best_score = 0;
    const char* force = getenv("LDPC_F5_SHAPE");
    const int forced = force ? atoi(force) : -1;
    const char* me = getenv("LDPC_F5_MERGE");            // 0: one proto row per run (A/B runs)
    const bool use_merge = g.h_row_merge && g.row_merge && !(me && atoi(me) == 0);
    const int32_t* hm = use_merge ? g.h_row_merge : nullptr;
    for (int si = 0; si < (int)(sizeof(kShapes5) / sizeof(kShapes5[0])); ++si) {
        const Shape5& sh = kShapes5[si];
        if (forced >= 0 ? si != forced : !sh.autosel) continue;
        if ((g.z == 1) != (sh.cw == 64)) continue;
        if (g.max_cdeg > sh.maxdeg) continue;
        const int slots = 64 / sh.cw;
        const int ngroups = f5_ngroups(g.h_row_ptr, hm, g.M, g.z, slots);
        // waves: enough for MAXG groups each, rounded up to a multiple of 4 (a workgroup's
        // busiest SIMD holds ceil(nw / 4) waves either way; the extra waves share the VN phase)
        const int nw0 = (ngroups + sh.maxg - 1) / sh.maxg;
        const int nw = std::min(16, (nw0 + 3) & ~3);
        if (nw * sh.maxg < ngroups || nw < 1) continue;
        if (sh.hg > 0 && sh.hg < sh.maxg) {      // groups too heavy for a light slot must fit the heavy ones
            int heavy = 0;
            f5_for_runs(g.h_row_ptr, hm, g.M, [&](int, int n, int d) {
                heavy += (d > sh.ldeg) ? f5_run_groups(n, g.z, slots) : 0;
                return false;
            });
            if (heavy > sh.hg * nw) continue;
        }
        if (g.N > 64 * nw) continue;                                    // beta slice copy
        const size_t lds = f5_lds(g.n_vars, sh.cw, T, g.N);
        if (lds > F5_LDS_MAX) continue;
        if (((size_t)g.n_vars * sh.cw + F5_NDUMMY) * 4 > 65536) continue;    // 16-bit addresses
        // resident workgroups per CU: LDS and the shape's VGPR budget (Shape5::wpe waves per SIMD;
        // a workgroup puts ceil(nw/4) waves on its busiest SIMD and the next workgroup starts
        // on the same SIMD: measured, a 14-wave group at 7 waves/SIMD runs alone).  VALU issue
        // saturates around 6 waves per SIMD, so waves beyond 24 per CU earn nothing.
        const int wg_lds = (int)(F5_LDS_MAX / lds);
        const int wpe = std::max(sh.wpe, 4);
        const int wg_waves = wpe / ((nw + 3) / 4);
        const int wgs = std::max(1, std::min(wg_lds, wg_waves));
        const double eff = (double)g.max_cdeg / (double)(((g.max_cdeg + 7) / 8) * 8);
        const double util = (double)(g.M * g.z) / (double)(ngroups * slots);    // lanes on real checks
        const double score = (double)std::min(wgs * nw0, 24) * eff * util + 1e-3 * sh.cw;
        if (score > best_score) {
            best_score = score;
            best.shape = si;
            best.nw = nw;
            best.merge = use_merge ? g.row_merge : nullptr;
            best.ngroups = ngroups;
            best.lds = lds;
        }
    }
    return best;
}

// LDPC_DIAG_STAMPS=<file>: raw per-workgroup marks of one launch, [nblocks][32] u64 (100 MHz
// s_memrealtime: 0 start, 1 after the LLR/CH prologue, 2 after the edge-address setup, 5 after
// iteration 0's pass 1, 6 after its pass-2 barrier, 8 + t start of iteration t, 30 end; slot 31
// = XCC_ID << 32 | HW_ID), appended to <file>.  Analysis: tools/stamps.py.
void report_stamps(const unsigned long long* d, int nblocks, hipStream_t s, const char* path) {
    std::vector<unsigned long long> h((size_t)nblocks * 32);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    if (FILE* f = fopen(path, "ab")) {
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
    }
}

}  // namespace f5

using namespace f5;

bool fused5_supported(const DevGraph& g, int T) { return plan5(g, T).shape >= 0; }

const char* fused5_shape_name(const DevGraph& g, int T) {
    static thread_local char buf[64];
    const Plan5 p = plan5(g, T);
    if (p.shape < 0) return "";
    const Shape5& sh = kShapes5[p.shape];
    snprintf(buf, sizeof(buf), "fused5[cw%d,g%d,d%d,w%d]", sh.cw, sh.maxg, sh.maxdeg, p.nw);
    return buf;
}

int fused5_cw(const DevGraph& g, int T) {
    const Plan5 p = plan5(g, T);
    return p.shape < 0 ? 0 : kShapes5[p.shape].cw;
}

int fused5_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr,
                  int qmax, float step, int clip_u, bool per_edge_w, uint64_t* hd_out,
                  int64_t* counters, uint8_t* flags, hipStream_t s, const uint32_t* only) {
    Plan5 p = plan5(g, b.T);
    if (p.shape < 0 || qmax > 31) return LDPC_ERR_UNSUPPORTED;   // pass 1's 8-bit V->C range
    const Shape5& sh = kShapes5[p.shape];
    // weight tables (uniform row weights): only if they cost no workgroup slot per CU
    // per-iteration slices of the weight tables, double-buffered in LDS
    const int qrow = 3 * qmax + 2;
    const int qucn = g.M * qrow;
    const int qslice = ((b.alpha_ucn ? 2 : 1) * qucn + 1) & ~1;
    bool lut = !per_edge_w && g.M < 256 && (qslice >> 1) <= 64 * p.nw &&
               getenv("LDPC_F5_NOLUT") == nullptr;
    if (lut) {
        const size_t lds_lut = p.lds + (((size_t)2 * qslice * 2 + 15) & ~(size_t)15);
        if (lds_lut > F5_LDS_MAX || F5_LDS_MAX / lds_lut < F5_LDS_MAX / p.lds) lut = false;
        else p.lds = lds_lut;
    }
    F5Args a{};
    a.llr = llr;
    a.beta = b.beta;
    a.app_out = b.app_out;
    a.hd_out = hd_out;
    a.counters = counters;
    a.flags = flags;
    a.row_ptr = g.row_ptr;
    a.pe_col = g.pe_col;
    a.pe_shift = g.pe_shift;
    a.B = b.B;
    a.ntiles = b.ntiles;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.clip_u = clip_u;
    a.qmax = qmax;
    a.step = step;
    a.inv = 1.0f / step;
    a.n_vars = g.n_vars;
    a.N = g.N;
    a.E = g.E;
    a.z = g.z;
    a.ngroups = p.ngroups;
    a.nent = (g.n_vars * sh.cw + 64 * p.nw - 1) / (64 * p.nw);
    a.nfull = g.n_vars * sh.cw / 64;
    a.cpw = (a.nfull + p.nw - 1) / p.nw;
    a.Mp = g.M;
    if (b.awgn) {
        a.gen = 1;
        a.awgn = *reinterpret_cast<const AwgnParams*>(b.awgn);
    }
    a.zmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.z - 1) / (uint64_t)g.z);
    a.only = only;
    a.iter_wrong = b.iter_wrong;
    if (const char* e = getenv("LDPC_DIAG_ABLATE")) a.ablate = atoi(e);   // timing only
    // shared tables: one small launch per decode instead of per-workgroup dependent loads
    const size_t nqt = (size_t)b.T * qslice;
    const int npk = (sh.maxdeg + 1) / 2;
    const size_t off_qt = 0;
    const size_t off_gad = (off_qt + nqt * 2 + 255) & ~(size_t)255;
    const size_t off_grow = off_gad + (size_t)p.ngroups * npk * 64 * 4;
    const size_t tbytes = off_grow + (size_t)p.ngroups * 16;
    if (tbytes > ws.tables_bytes) {
        if (ws.tables) (void)hipFree(ws.tables);
        ws.tables = nullptr;
        ws.tables_bytes = 0;
        ws.key_gad[0] = ws.key_qtab[0] = ~0ull;
        if (hipMalloc(&ws.tables, tbytes) != hipSuccess) {
            (void)hipGetLastError();
            return LDPC_ERR_OOM;
        }
        ws.tables_bytes = tbytes;
    }
    uint16_t* qtab = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(ws.tables) + off_qt);
    uint32_t* gad = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ws.tables) + off_gad);
    uint4* grow = reinterpret_cast<uint4*>(reinterpret_cast<char*>(ws.tables) + off_grow);
    {
        // (skipped when the same tables are already in place: same weights, T, shape, grouping)
        const uint64_t kq[4] = {g.w_version, (uint64_t)b.T << 32 | (uint32_t)qmax,
                                (uint64_t)__builtin_bit_cast(uint32_t, step) << 32 | (uint32_t)qslice,
                                (uint64_t)(b.alpha_ucn != nullptr)};
        if (lut && !std::equal(kq, kq + 4, ws.key_qtab)) {
            hipLaunchKernelGGL(k_f5_tables, dim3((unsigned)((nqt + 255) / 256)), dim3(256), 0, s,
                               b.alpha, b.alpha_ucn, g.row_ptr, b.T, g.M, g.E, qmax, step,
                               1.0f / step, qslice, qtab);
            std::copy(kq, kq + 4, ws.key_qtab);
        }
        const int lcw = f5_logcw(sh.cw);
        const char* be = getenv("LDPC_F5_BALANCE");
        const bool hetero = sh.hg > 0 && sh.hg < sh.maxg;
        const bool bal = hetero || (be ? atoi(be) != 0 : sh.bal);
        const uint64_t kg[4] = {g.w_version, (uint64_t)p.shape << 32 | (uint32_t)p.ngroups,
                                (uint64_t)(p.merge != nullptr) << 1 | (bal ? 1u : 0u),
                                (uint64_t)off_gad << 32 | (uint32_t)p.nw};
        if (!std::equal(kg, kg + 4, ws.key_gad)) {
            hipLaunchKernelGGL(k_f5_gad, dim3((unsigned)((p.ngroups * 64 + 255) / 256)), dim3(256), 0, s,
                               g.row_ptr, g.pe_col, g.pe_shift, p.merge, g.M, p.ngroups, g.z, lcw,
                               sh.maxdeg, npk, g.n_vars * sh.cw, p.nw, bal ? 1 : 0, gad, grow);
            std::copy(kg, kg + 4, ws.key_gad);
        }
        if (hipGetLastError() != hipSuccess) return LDPC_ERR_HIP;
    }
    a.betas = b.beta;      // [T][N] as given (the kernel keeps ch / step)
    a.qtab = qtab;
    a.qslice = qslice;
    a.qucn = qucn;
    a.qrow = qrow;
    a.gad = gad;
    a.grow = grow;
    const int nblocks = (int)((b.B + sh.cw - 1) / sh.cw);
    const float* au = b.alpha_ucn;
    const char* diag = getenv("LDPC_DIAG_STAMPS");   // timing investigation only
    if (diag && (hipMalloc(&a.stamps, (size_t)nblocks * 32 * sizeof(unsigned long long)) != hipSuccess ||
                 hipMemsetAsync(a.stamps, 0, (size_t)nblocks * 32 * 8, s) != hipSuccess))
        return LDPC_ERR_OOM;
    int rc;
    switch (p.shape) {
        case 0: rc = f5_launch<0>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 1: rc = f5_launch<1>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 2: rc = f5_launch<2>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 3: rc = f5_launch<3>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 4: rc = f5_launch<4>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 5: rc = f5_launch<5>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 6: rc = f5_launch<6>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 7: rc = f5_launch<7>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 8: rc = f5_launch<8>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        case 9: rc = f5_launch<9>(a, nblocks, p.nw, p.lds, lut, b.alpha, au, per_edge_w, s); break;
        default: rc = LDPC_ERR_UNSUPPORTED;
    }
    if (diag) {
        if (rc == LDPC_OK) report_stamps(a.stamps, nblocks, s, diag);
        (void)hipFree(a.stamps);
    }
    return rc;
}

}  // namespace ldpc
