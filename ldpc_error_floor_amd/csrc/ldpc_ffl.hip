// ldpc_ffl.hip — fused decoder for the floating-point modes ("ffl"): min-sum fp32
// (decoding_type 1), min-sum without the zero nudge (3) and QMS q = 6 (whose +-15.5 grid the
// integer kernels do not cover).  All T flooding iterations of a block of CW codewords in one
// launch, counters / frame flags only; the arithmetic is the flood kernel's (ldpc_flood.hip,
// Main_Functions.py:212-335) operation for operation, so the counters equal flood's exactly.
//
// State in LDS, per codeword of the block (w = codeword within the block, innermost):
//   TV[v][w]       Tv = Q(beta_{t+1} ch) + S, the variable's total (the check side subtracts
//                  its own old message: V->C = Q(Tv - C->V_old), as in flood's k_cn_update);
//   REC[f][c][w]   the check's messages in compressed form: R1 (the message of every edge but
//                  the argmin), R2 (the argmin's), the [V->C > 0] bits of the edges, and
//                  argmin | parity << 8.  Edge k's C->V is (odd_k ? R : -R) with
//                  R = (k == argmin ? R2 : R1) and odd_k = parity ^ bit k — exactly flood's
//                  r = sign(o) Q(relu(|o| w)) for o = odd ? m' : -m' (m' = the adjusted
//                  minimum, Main_Functions.py:250-254), since the weight is one per row;
//   HD[v][w]       (UCN) the previous hard decision, for the check's syndrome.
// The channel stays in registers (each lane owns its variables for the whole decode).  LDS per
// codeword: 4 (N z) + 16 (M z) [+ 4 (N z)] bytes: wman 4.6 KB, so a 16-codeword block fits two
// workgroups per CU.
//
// Work mapping: a wave takes G = 64 / CW consecutive checks (variables) of one proto row
// (column) for the CW codewords (lane = g CW + w), so the graph and the weights are
// wave-uniform (scalar loads) and a half-wave's LDS words are contiguous (consecutive checks
// read consecutive Tv rows: conflict-free banks).  z is padded to a multiple of G per row/column.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "ldpc_fused.h"
#include "ldpc_quant.h"

namespace ldpc {
namespace ffl {

constexpr int NW = 16;                   // waves per workgroup
constexpr int KVMAX = 12;                // variable wave-tasks per wave (channel registers)
constexpr size_t LDS_MAX = 160 * 1024;

struct FflArgs {
    const float* llr;
    int64_t B;
    int n_vars, n_checks, z, hq, M, N, E, T, target_bits;   // hq = padded z / G
    float clip;
    const int32_t* row_ptr;
    const int32_t* pe_col;
    const int32_t* pe_shift;
    const int32_t* pe_row;
    const int32_t* col_ptr;
    const int32_t* col_pe;
    const int4* vn_edge;         // [E] column order (DevGraph::vn_edge)
    const float* alpha;          // [T][E] (one value per row used: the row's first edge)
    const float* alpha_ucn;      // [T][E] or null
    const float* beta;           // [T][N]
    int64_t* counters;
    uint8_t* flags;
    uint32_t* iter_wrong;        // [T][ceil(B/32)] per-iteration frame-error words (zeroed), or null
    uint32_t off_tv, off_rec, off_hd, off_red;
};

__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// OR of the CW-bit groups of a 64-lane ballot (bit w of the result: some lane g CW + w)
template <int CW>
__device__ __forceinline__ uint32_t fold(uint64_t m) {
    uint32_t r = 0;
#pragma unroll
    for (int g = 0; g < 64 / CW; ++g) r |= (uint32_t)(m >> (g * CW));
    return CW == 32 ? r : (r & ((1u << CW) - 1u));
}

// frame flags / counters of the block from the LDS reductions (RED[0]: some bit wrong at the
// last iteration, RED[1]: wrong at every earlier one, RED[2]: some app > 0, RED[3]: bit errors)
template <int CW>
__device__ __forceinline__ void block_finish(const FflArgs& a, uint32_t* RED, int tid, int64_t b0,
                                             int nvalid, uint32_t valid) {
    if (tid == 0) {
        const uint32_t wl = RED[0] & valid;
        const uint32_t all = RED[1] & RED[0] & valid;
        const uint32_t ap = RED[2] & valid;
        if (a.iter_wrong) put_iter_wrong(a.iter_wrong, a.B, a.T - 1, b0, CW, wl);
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

template <int MODE, int CW, bool UCN>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(8)))
k_ffl(FflArgs a) {
    constexpr int G = 64 / CW;
    constexpr bool nudge = (MODE != MODE_MSNN);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* TV = reinterpret_cast<float*>(smem + a.off_tv);
    float* R1 = reinterpret_cast<float*>(smem + a.off_rec);
    float* R2 = R1 + (size_t)a.n_checks * CW;
    uint32_t* SG = reinterpret_cast<uint32_t*>(R2 + (size_t)a.n_checks * CW);
    uint32_t* XW = SG + (size_t)a.n_checks * CW;
    uint32_t* HD = reinterpret_cast<uint32_t*>(smem + a.off_hd);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uni(tid >> 6);
    const int g = lane / CW, w = lane % CW;
    const int z = a.z, hq = a.hq, nv = a.n_vars;
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nvalid = (int)min<int64_t>(CW, a.B - b0);
    const bool wvalid = w < nvalid;
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    const int nvt = a.N * hq, nct = a.M * hq;          // wave-tasks

    // ---- prologue: the channel of the lane's variables, Tv_0 = lw_0, hd_{-1} = [lw_0 >= 0] ----
    float ch[KVMAX];
#pragma unroll
    for (int kk = 0; kk < KVMAX; ++kk) {
        ch[kk] = 0.f;
        const int q = wave + kk * NW;
        if (q < nvt) {
            const int j = q / hq, h = (q - j * hq) * G + g;
            if (h < z && wvalid) ch[kk] = a.llr[(b0 + w) * nv + j * z + h];
        }
    }
#pragma unroll
    for (int kk = 0; kk < KVMAX; ++kk) {
        const int q = wave + kk * NW;
        if (q < nvt) {
            const int j = q / hq, h = (q - j * hq) * G + g;
            if (h < z) {
                const int v = j * z + h;
                const float lw = qchan<MODE>(ch[kk] * a.beta[j]);
                TV[v * CW + w] = lw;
                if (UCN) HD[v * CW + w] = lw >= 0.f ? 1u : 0u;
            }
        }
    }
    if (tid < 8) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
    __syncthreads();

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {            // fold iteration t-1's frame flags
            if (a.iter_wrong) put_iter_wrong(a.iter_wrong, a.B, t - 1, b0, CW, RED[0] & valid);
            RED[1] &= RED[0];
            RED[0] = 0u;
        }
        // ======== check nodes (flood's k_cn_update on the compressed records) ==================
        for (int q = wave; q < nct; q += NW) {
            const int i = uni(q / hq);
            const int h = (q - i * hq) * G + g;
            const bool act = h < z;
            const int hh = act ? h : z - 1;
            const int c = i * z + hh;
            const int r0 = a.row_ptr[i], deg = a.row_ptr[i + 1] - r0;
            float o1 = 0.f, o2 = 0.f;
            uint32_t osg = 0u, oxw = 0u;
            if (t > 0) {
                o1 = R1[c * CW + w];
                o2 = R2[c * CW + w];
                osg = SG[c * CW + w];
                oxw = XW[c * CW + w];
            }
            const int oix = (int)(oxw & 0xFFu);
            const uint32_t opar = (oxw >> 8) & 1u;
            float mn1 = 10000.f, mn2 = 10000.f;
            int ix = 0;
            uint32_t sg = 0u, syn = 0u;
            // four edges at a time: their Tv (and hard decision) reads in flight together
            for (int k0 = 0; k0 < deg; k0 += 4) {
                float tv[4];
                uint32_t hdv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (k0 + u < deg) {
                        const int pe = r0 + k0 + u;
                        const int s = hh + a.pe_shift[pe];
                        const int v = a.pe_col[pe] * z + (s >= z ? s - z : s);
                        tv[u] = TV[v * CW + w];
                        if (UCN) hdv[u] = HD[v * CW + w];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + u;
                    if (k < deg) {
                        float cv = 0.f;
                        if (t > 0) {
                            const float R = (k == oix) ? o2 : o1;
                            cv = (opar ^ ((osg >> k) & 1u)) ? R : -R;
                        }
                        float x = qmsg<MODE>(tv[u] - cv, a.clip);
                        if (nudge && x == 0.f) x = 1e-4f;               // Main_Functions.py:229-230
                        float am = fabsf(x);
                        if (!(am > 0.f)) am = 10000.f;                    // zeros never the min (:248)
                        if (am < mn1) { mn2 = mn1; mn1 = am; ix = k; }
                        else if (am < mn2) { mn2 = am; }
                        sg |= (uint32_t)(x > 0.f) << k;
                        if (UCN) syn ^= hdv[u];
                    }
                }
            }
            // the two possible messages R(m') = sign(m') Q(relu(|m'| w)) (:250-316)
            const float al = a.alpha[(size_t)t * a.E + r0];
            const float w_ = (UCN && (syn & 1u)) ? a.alpha_ucn[(size_t)t * a.E + r0] : al;
            float rr[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                float m = u ? mn2 : mn1;
                if (m <= 1e-4f) m = m - 1e-4f;                          // :250
                float xx = fabsf(m) * w_;
                xx = (xx > 0.f) ? xx : 0.f;                             // :308
                xx = qmsg<MODE>(xx, a.clip);                            // :310-313
                rr[u] = (m > 0.f) ? xx : ((m < 0.f) ? -xx : 0.f);
            }
            if (act) {
                R1[c * CW + w] = rr[0];
                R2[c * CW + w] = rr[1];
                SG[c * CW + w] = sg;
                XW[c * CW + w] = (uint32_t)ix | ((uint32_t)(__popc(sg) & 1) << 8);
            }
        }
        __syncthreads();
        // ======== variable nodes (flood's k_vn_update) ==========================================
        const bool last = (t == a.T - 1);
        uint32_t wr = 0u, apos = 0u, nb = 0u;
#pragma unroll
        for (int kk = 0; kk < KVMAX; ++kk) {
            const int q = wave + kk * NW;
            if (q >= nvt) continue;          // (wave-uniform; not a break: the loop must unroll)
            const int j = uni(q / hq);
            const int h = (q - j * hq) * G + g;
            const bool act = h < z;
            const int hh = act ? h : z - 1;
            const int e0 = a.col_ptr[j], e1 = a.col_ptr[j + 1];
            float S = 0.f;
            // four edges at a time (16 record reads in flight), summed in column order as flood
            for (int e = e0; e < e1; e += 4) {
                float r1[4], r2[4];
                uint32_t xw[4], sgw[4];
                int kk4[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (e + u < e1) {
                        const int4 ve = a.vn_edge[e + u];     // {., ., shift, (i z) << 6 | k}
                        int hc = hh - ve.z;
                        hc = hc < 0 ? hc + z : hc;
                        const int c = (ve.w >> 6) + hc;
                        kk4[u] = ve.w & 63;
                        xw[u] = XW[c * CW + w];
                        sgw[u] = SG[c * CW + w];
                        r1[u] = R1[c * CW + w];
                        r2[u] = R2[c * CW + w];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (e + u < e1) {
                        const float R = ((int)(xw[u] & 0xFFu) == kk4[u]) ? r2[u] : r1[u];
                        const uint32_t odd = ((xw[u] >> 8) ^ (sgw[u] >> kk4[u])) & 1u;
                        S += odd ? R : -R;
                    }
                }
            }
            const int v = j * z + hh;
            const float app = fminf(fmaxf(qchan<MODE>(ch[kk]) + S, -a.clip), a.clip);
            const bool counted = act && wvalid && v < a.target_bits;
            const bool hd = app >= 0.f;
            wr |= fold<CW>(__ballot(counted && hd));
            if (last) {
                apos |= fold<CW>(__ballot(counted && app > 0.f));
                nb += (uint32_t)__popcll(__ballot(counted && hd));
            } else if (act) {
                const float beta = a.beta[(size_t)(t + 1) * a.N + j];
                TV[v * CW + w] = qchan<MODE>(ch[kk] * beta) + S;
                if (UCN) HD[v * CW + w] = hd ? 1u : 0u;
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
    block_finish<CW>(a, RED, tid, b0, nvalid, valid);
}

// ---- sum-product (decoding_type 0): flood's cn_update_sp / k_vn_update on LDS ---------------
// The sum-product messages do not compress (every edge's C->V differs), so the state is flood's
// own: C2V[(pe z + h)][w] per edge (proto edge pe in row order, check h of the row: a wave's
// consecutive checks are consecutive words) and TV[v][w]; pass 1 parks t_k = tanh(-x_k/2) in
// the edge's slot after reading the old message there, pass 2 overwrites it with the new one.
// LDS per codeword: 4 (N z + E z) [+ 4 N z] bytes.  Per-edge weights are read as flood reads them.
template <int CW, bool UCN>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(8)))
k_ffs(FflArgs a) {
    constexpr int G = 64 / CW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* TV = reinterpret_cast<float*>(smem + a.off_tv);
    float* C2V = reinterpret_cast<float*>(smem + a.off_rec);
    uint32_t* HD = reinterpret_cast<uint32_t*>(smem + a.off_hd);
    uint32_t* RED = reinterpret_cast<uint32_t*>(smem + a.off_red);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = uni(tid >> 6);
    const int g = lane / CW, w = lane % CW;
    const int z = a.z, hq = a.hq, nv = a.n_vars;
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int nvalid = (int)min<int64_t>(CW, a.B - b0);
    const bool wvalid = w < nvalid;
    const uint32_t valid = (nvalid >= 32) ? 0xFFFFFFFFu : ((1u << nvalid) - 1u);
    const int nvt = a.N * hq, nct = a.M * hq;

    float ch[KVMAX];
#pragma unroll
    for (int kk = 0; kk < KVMAX; ++kk) {
        ch[kk] = 0.f;
        const int q = wave + kk * NW;
        if (q < nvt) {
            const int j = q / hq, h = (q - j * hq) * G + g;
            if (h < z && wvalid) ch[kk] = a.llr[(b0 + w) * nv + j * z + h];
        }
    }
#pragma unroll
    for (int kk = 0; kk < KVMAX; ++kk) {
        const int q = wave + kk * NW;
        if (q < nvt) {
            const int j = q / hq, h = (q - j * hq) * G + g;
            if (h < z) {
                const int v = j * z + h;
                const float lw = ch[kk] * a.beta[j];
                TV[v * CW + w] = lw;
                if (UCN) HD[v * CW + w] = lw >= 0.f ? 1u : 0u;
            }
        }
    }
    if (tid < 8) RED[tid] = (tid == 1) ? 0xFFFFFFFFu : 0u;
    __syncthreads();

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {
            if (a.iter_wrong) put_iter_wrong(a.iter_wrong, a.B, t - 1, b0, CW, RED[0] & valid);
            RED[1] &= RED[0];
            RED[0] = 0u;
        }
        // ======== check nodes (flood's cn_update_sp) =========================================
        for (int q = wave; q < nct; q += NW) {
            const int i = uni(q / hq);
            const int h = (q - i * hq) * G + g;
            const bool act = h < z;
            const int hh = act ? h : z - 1;
            const int r0 = a.row_ptr[i], deg = a.row_ptr[i + 1] - r0;
            uint32_t syn = 0u;
            for (int k0 = 0; k0 < deg; k0 += 4) {
                float tv[4], cv[4];
                uint32_t hdv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (k0 + u < deg) {
                        const int pe = r0 + k0 + u;
                        const int s = hh + a.pe_shift[pe];
                        const int v = a.pe_col[pe] * z + (s >= z ? s - z : s);
                        tv[u] = TV[v * CW + w];
                        cv[u] = (t > 0) ? C2V[(pe * z + hh) * CW + w] : 0.f;
                        if (UCN) hdv[u] = HD[v * CW + w];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (k0 + u < deg) {
                        const float y = sp_t(fminf(fmaxf(tv[u] - cv[u], -a.clip), a.clip));   // :227
                        if (act) C2V[((r0 + k0 + u) * z + hh) * CW + w] = y;
                        if (UCN) syn ^= hdv[u];
                    }
                }
            }
            const float* at = a.alpha + (size_t)t * a.E + r0;
            const float* au = UCN ? a.alpha_ucn + (size_t)t * a.E + r0 : nullptr;
            // edge k's product over the others in the oracle's order (as flood's cn_update_sp)
            float pre = 1.f;
            for (int k = 0; k < deg; ++k) {
                const int slot = ((r0 + k) * z + hh) * CW + w;
                const float y = act ? C2V[slot] : 1.f;
                float others = pre;
                for (int j = k + 1; j < deg; ++j) others *= act ? C2V[((r0 + j) * z + hh) * CW + w] : 1.f;
                pre *= y;
                const float o = sp_o(others);
                const float wt = (UCN && (syn & 1u)) ? au[k] : at[k];
                float x = fabsf(o) * wt;
                x = (x > 0.f) ? x : 0.f;                                               // :308
                x = fminf(fmaxf(x, -a.clip), a.clip);                                  // :313
                if (act) C2V[slot] = (o > 0.f) ? x : ((o < 0.f) ? -x : 0.f);           // :316
            }
        }
        __syncthreads();
        // ======== variable nodes (flood's k_vn_update) ========================================
        const bool last = (t == a.T - 1);
        uint32_t wr = 0u, apos = 0u, nb = 0u;
#pragma unroll
        for (int kk = 0; kk < KVMAX; ++kk) {
            const int q = wave + kk * NW;
            if (q >= nvt) continue;
            const int j = uni(q / hq);
            const int h = (q - j * hq) * G + g;
            const bool act = h < z;
            const int hh = act ? h : z - 1;
            const int e0 = a.col_ptr[j], e1 = a.col_ptr[j + 1];
            float S = 0.f;
            for (int e = e0; e < e1; e += 4) {
                float cv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (e + u < e1) {
                        const int pe = a.col_pe[e + u];
                        int hc = hh - a.pe_shift[pe];
                        hc = hc < 0 ? hc + z : hc;
                        cv[u] = C2V[(pe * z + hc) * CW + w];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (e + u < e1) S += cv[u];
            }
            const int v = j * z + hh;
            const float app = fminf(fmaxf(ch[kk] + S, -a.clip), a.clip);
            const bool counted = act && wvalid && v < a.target_bits;
            const bool hd = app >= 0.f;
            wr |= fold<CW>(__ballot(counted && hd));
            if (last) {
                apos |= fold<CW>(__ballot(counted && app > 0.f));
                nb += (uint32_t)__popcll(__ballot(counted && hd));
            } else if (act) {
                const float beta = a.beta[(size_t)(t + 1) * a.N + j];
                TV[v * CW + w] = ch[kk] * beta + S;
                if (UCN) HD[v * CW + w] = hd ? 1u : 0u;
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
    block_finish<CW>(a, RED, tid, b0, nvalid, valid);
}

struct FflPlan {
    bool ok = false;
    int cw = 0, hq = 0;
    uint32_t off_tv = 0, off_rec = 0, off_hd = 0, off_red = 0;
    size_t lds = 0;
};

// min-sum modes: CW 16 (else 4) with the compressed records, one weight per row; sum-product:
// CW 8 (else 4, 2) with per-edge messages, any weights
static FflPlan plan(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    FflPlan p;
    const char* e = getenv("LDPC_FFL");
    if (e && atoi(e) == 0) return p;
    const bool sp = (mode == MODE_SP);
    if (!g.host || (!sp && (per_edge_w || g.max_cdeg > 32))) return p;
    const host::GraphTables& h = *g.host;
    // (sum-product: CW 8 first — no idle check lanes when 8 | z; 3.64 M against 3.34 M cw/s at
    // CW 4 on wman, one box)
    const int cws_ms[3] = {16, 4, 0}, cws_sp[3] = {8, 4, 2};
    for (int cw : sp ? cws_sp : cws_ms) {
        if (cw == 0) break;
        const int G = 64 / cw;
        const int hq = (h.z + G - 1) / G;
        if ((h.N * hq + NW - 1) / NW > KVMAX) continue;
        size_t o = 0;
        p.off_tv = 0;
        o += (size_t)g.n_vars * cw * 4;
        p.off_rec = (uint32_t)o;
        o += sp ? (size_t)g.n_edges * cw * 4 : (size_t)4 * g.n_checks * cw * 4;
        p.off_hd = (uint32_t)o;
        if (ucn) o += (size_t)g.n_vars * cw * 4;
        p.off_red = (uint32_t)o;
        o += 64;
        if (o > LDS_MAX) continue;
        p.ok = true;
        p.cw = cw;
        p.hq = hq;
        p.lds = o;
        return p;
    }
    return FflPlan{};
}

template <int CW, bool UCN>
static int launch_sp(const FflArgs& a, int nblocks, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ffs<CW, UCN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_ffs<CW, UCN>), dim3(nblocks), dim3(64 * NW), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

template <int MODE, int CW, bool UCN>
static int launch(const FflArgs& a, int nblocks, size_t lds, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ffl<MODE, CW, UCN>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL((k_ffl<MODE, CW, UCN>), dim3(nblocks), dim3(64 * NW), lds, s, a);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

template <int MODE>
static int launch_mode(const FflArgs& a, int cw, bool ucn, int nblocks, size_t lds, hipStream_t s) {
    if (cw == 16) return ucn ? launch<MODE, 16, true>(a, nblocks, lds, s) : launch<MODE, 16, false>(a, nblocks, lds, s);
    return ucn ? launch<MODE, 4, true>(a, nblocks, lds, s) : launch<MODE, 4, false>(a, nblocks, lds, s);
}

}  // namespace ffl

bool ffl_mode(int mode) {
    return mode == MODE_MS || mode == MODE_MSNN || mode == MODE_Q6 || mode == MODE_SP;
}

bool ffl_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    return ffl_mode(mode) && ffl::plan(g, mode, ucn, per_edge_w).ok;
}

const char* ffl_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w) {
    static thread_local char buf[48];
    const ffl::FflPlan p = ffl::plan(g, mode, ucn, per_edge_w);
    snprintf(buf, sizeof(buf), "ffl[%scw%d,w%d%s]", mode == MODE_SP ? "sp," : "", p.cw, ffl::NW,
             ucn ? ",ucn" : "");
    return buf;
}

int ffl_decode(const DevGraph& g, const Bufs& b, const float* llr, int mode, bool ucn, bool per_edge_w,
               int64_t* counters, uint8_t* flags, hipStream_t s) {
    const ffl::FflPlan p = ffl::plan(g, mode, ucn, per_edge_w);
    if (!p.ok || !ffl_mode(mode)) return LDPC_ERR_UNSUPPORTED;
    ffl::FflArgs a{};
    a.llr = llr;
    a.B = b.B;
    a.n_vars = g.n_vars;
    a.n_checks = g.n_checks;
    a.z = g.z;
    a.hq = p.hq;
    a.M = g.M;
    a.N = g.N;
    a.E = g.E;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.clip = b.clip;
    a.row_ptr = g.row_ptr;
    a.pe_col = g.pe_col;
    a.pe_shift = g.pe_shift;
    a.pe_row = g.pe_row;
    a.col_ptr = g.col_ptr;
    a.col_pe = g.col_pe;
    a.vn_edge = g.vn_edge;
    a.alpha = b.alpha;
    a.alpha_ucn = ucn ? b.alpha_ucn : nullptr;
    a.beta = b.beta;
    a.counters = counters;
    a.flags = flags;
    a.iter_wrong = b.iter_wrong;
    a.off_tv = p.off_tv;
    a.off_rec = p.off_rec;
    a.off_hd = p.off_hd;
    a.off_red = p.off_red;
    const int nblocks = (int)((b.B + p.cw - 1) / p.cw);
    switch (mode) {
        case MODE_MS: return ffl::launch_mode<MODE_MS>(a, p.cw, ucn, nblocks, p.lds, s);
        case MODE_MSNN: return ffl::launch_mode<MODE_MSNN>(a, p.cw, ucn, nblocks, p.lds, s);
        case MODE_SP:
            if (p.cw == 8) return ucn ? ffl::launch_sp<8, true>(a, nblocks, p.lds, s) : ffl::launch_sp<8, false>(a, nblocks, p.lds, s);
            if (p.cw == 4) return ucn ? ffl::launch_sp<4, true>(a, nblocks, p.lds, s) : ffl::launch_sp<4, false>(a, nblocks, p.lds, s);
            return ucn ? ffl::launch_sp<2, true>(a, nblocks, p.lds, s) : ffl::launch_sp<2, false>(a, nblocks, p.lds, s);
        default: return ffl::launch_mode<MODE_Q6>(a, p.cw, ucn, nblocks, p.lds, s);
    }
}

}  // namespace ldpc
