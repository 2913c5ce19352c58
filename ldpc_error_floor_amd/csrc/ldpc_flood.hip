// ldpc_flood.hip — flooding NMS/QMS decoder as two edge-parallel kernels per iteration.
//
// Semantics: build_neural_network (Main_Functions.py:157-385), restated in edge form in
// SURVEY.md Appendix A and oracle/nms_oracle.py.  One iteration t:
//   cn_update(t): per check c, over its edges e=(c,v):  v2c = Q(Tv[v] - C2V_t[e]) (+nudge),
//                 two-minima + sign parity, C2V_{t+1}[e] = Q(relu(|o| * w)) * sign(o)
//   vn_update(t): per variable v: S = sum_e C2V_{t+1}[e];  APP_t = clip(Qch(ch)+S);
//                 hard bit; Tv[v] = Q(beta_{t+1} ch) + S for the next iteration.
// Tv[v] = lw[v] + S[v] fuses the VN-weighted channel (Main_Functions.py:168-177) with the
// VN sum so the check kernel reads one value per edge.
//
// Layout in HBM ("batch-innermost tiles"): every per-codeword array is
// [tile][row][256] with 256 codewords per tile; lane l of a wave holds codewords
// 4l..4l+3 as one float4, so every row access of a wave is one contiguous 1 KiB.
// The Tanner graph (check/variable ids, shifts, weights) is wave-uniform: all lanes of a
// wave work on the same check / variable for different codewords, so the graph lives in
// scalar registers and costs no vector memory traffic.
#include "ldpc_internal.h"
#include "ldpc_quant.h"

namespace ldpc {

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ int64_t xcd_block() {
    // XCD-aware remap: blocks b and b+8 share an XCD; give each XCD a contiguous range of
    // work items so the checks of one tile (which share Tv rows) hit the same L2.
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    return (nb & 7) ? b : (int64_t)(b & 7) * (nb >> 3) + (b >> 3);
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float f4(const float4& v, int q) {
    return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
}

// ----------------------------------------------------------------------------------------
// prologue: llr [B][n_vars] -> ch [tile][v][256], Tv_0 = lw_0, hd_{-1} = (lw_0 >= 0)
template <int MODE, bool UCN>
__global__ void __launch_bounds__(256) k_prologue(DevGraph g, Bufs p, const float* __restrict__ llr) {
    __shared__ float sm[32][TILE + 1];
    const int nchunks = (g.n_vars + 31) / 32;
    const int64_t tile = blockIdx.x / nchunks;
    const int v0 = (int)(blockIdx.x - tile * nchunks) * 32;
    const int tid = threadIdx.x;
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
        const int bl = r * 8 + (tid >> 5);
        const int vl = tid & 31;
        const int64_t b = tile * TILE + bl;
        const int v = v0 + vl;
        sm[vl][bl] = (b < p.B && v < g.n_vars) ? llr[b * g.n_vars + v] : 0.f;
    }
    __syncthreads();
    const int wave = tid >> 6, lane = tid & 63;
    for (int vl = wave * 8; vl < wave * 8 + 8; ++vl) {
        const int v = v0 + vl;
        if (v >= g.n_vars) break;
        const float4 x = make_float4(sm[vl][4 * lane], sm[vl][4 * lane + 1], sm[vl][4 * lane + 2],
                                     sm[vl][4 * lane + 3]);
        const size_t row = ((size_t)tile * g.n_vars + v) * TILE + 4 * lane;
        st4(p.ch + row, x);
        const float beta = p.beta[v / g.z];             // t = 0
        float4 lw;
        lw.x = qchan<MODE>(x.x * beta);
        lw.y = qchan<MODE>(x.y * beta);
        lw.z = qchan<MODE>(x.z * beta);
        lw.w = qchan<MODE>(x.w * beta);
        st4(p.Tv + row, lw);
        if (UCN) {
            const uint64_t b0 = __ballot(lw.x >= 0.f), b1 = __ballot(lw.y >= 0.f);
            const uint64_t b2 = __ballot(lw.z >= 0.f), b3 = __ballot(lw.w >= 0.f);
            uint64_t* hw = p.hd + hd_index(p, -1, tile, v);
            if (lane == 0) { hw[0] = b0; hw[1] = b1; hw[2] = b2; hw[3] = b3; }
        }
    }
}

// ----------------------------------------------------------------------------------------
// check-node update (Main_Functions.py:213-316)
// Sum-product check update (decoding_type 0, Main_Functions.py:238-245), 4 codewords per
// lane like the min-sum path, in the oracle's float32 order (sp_t / sp_o, ldpc_internal.h):
// pass 1 parks t_k in the edge's C->V slot (after reading the old message there); pass 2 takes
// edge k's product over the others as (t_0 ... t_{k-1}) t_{k+1} ... t_{d-1} left to right
// (the running prefix, then the later slots, which still hold t), writes its message into slot
// k, then extends the prefix with t_k; then weight, relu, clip and sign as the min-sum path.
template <bool UCN>
__device__ __forceinline__ void cn_update_sp(const DevGraph& g, const Bufs& p, int t, int64_t tile,
                                             int c, int lane, int i, int h, int r0, int deg,
                                             const float* Tt, float* Ct) {
    (void)c; (void)i;
    uint32_t syn = 0;
    for (int k = 0; k < deg; ++k) {
        const int pe = r0 + k;
        const int s = h + g.pe_shift[pe];
        const int v = g.pe_col[pe] * g.z + (s >= g.z ? s - g.z : s);
        const float4 tv = ld4(Tt + (size_t)v * TILE);
        const float4 cv = (t == 0) ? make_float4(0.f, 0.f, 0.f, 0.f) : ld4(Ct + (size_t)k * TILE);
        float th[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            th[q] = sp_t(fminf(fmaxf(f4(tv, q) - f4(cv, q), -p.clip), p.clip));   // :227
        st4(Ct + (size_t)k * TILE, make_float4(th[0], th[1], th[2], th[3]));
        if (UCN) {
            const uint64_t* hw = p.hd + hd_index(p, t - 1, tile, v);
            syn ^= (uint32_t)((hw[0] >> lane) & 1) | ((uint32_t)((hw[1] >> lane) & 1) << 1) |
                   ((uint32_t)((hw[2] >> lane) & 1) << 2) | ((uint32_t)((hw[3] >> lane) & 1) << 3);
        }
    }
    const float* at = p.alpha + (size_t)t * g.E;
    const float* au = UCN ? p.alpha_ucn + (size_t)t * g.E : nullptr;
    float pre[4] = {1.f, 1.f, 1.f, 1.f};
    for (int k = 0; k < deg; ++k) {
        const float a = at[r0 + k];
        const float u = UCN ? au[r0 + k] : 0.f;
        const float4 tk = ld4(Ct + (size_t)k * TILE);
        float others[4] = {pre[0], pre[1], pre[2], pre[3]};
        for (int j = k + 1; j < deg; ++j) {
            const float4 tj = ld4(Ct + (size_t)j * TILE);
#pragma unroll
            for (int q = 0; q < 4; ++q) others[q] *= f4(tj, q);
        }
        float r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float o = sp_o(others[q]);
            const float w = (UCN && ((syn >> q) & 1)) ? u : a;
            float x = fabsf(o) * w;
            x = (x > 0.f) ? x : 0.f;                                              // :308
            x = fminf(fmaxf(x, -p.clip), p.clip);                                 // :313
            r[q] = (o > 0.f) ? x : ((o < 0.f) ? -x : 0.f);                        // :316
            pre[q] *= f4(tk, q);
        }
        st4(Ct + (size_t)k * TILE, make_float4(r[0], r[1], r[2], r[3]));
    }
}

template <int MODE, bool FIRST, bool UCN>
__global__ void __launch_bounds__(256) k_cn_update(DevGraph g, Bufs p, int t) {
    const int64_t item = xcd_block() * 4 + uniform(threadIdx.x >> 6);
    const int64_t tile = item / g.n_checks;
    if (tile >= p.ntiles) return;
    const int c = uniform((int)(item - tile * g.n_checks));
    const int lane = threadIdx.x & 63;
    const int i = c / g.z, h = c - i * g.z;
    const int r0 = g.row_ptr[i];
    const int deg = g.row_ptr[i + 1] - r0;
    const float* Tt = p.Tv + (size_t)tile * g.n_vars * TILE + 4 * lane;
    float* Ct = p.c2v + ((size_t)tile * g.n_edges + (size_t)r0 * g.z + (size_t)h * deg) * TILE + 4 * lane;
    constexpr bool nudge = (MODE != MODE_MSNN && MODE != MODE_SP);
    if constexpr (MODE == MODE_SP) {
        cn_update_sp<UCN>(g, p, t, tile, c, lane, i, h, r0, deg, Tt, Ct);
        return;
    }

    float mn1[4], mn2[4];
    int ix[4];
    uint64_t sg[4];
    uint32_t syn = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { mn1[q] = 10000.f; mn2[q] = 10000.f; ix[q] = 0; sg[q] = 0; }

    // pass 1: V->C messages, two minima, sign bits
    for (int k = 0; k < deg; ++k) {
        const int pe = r0 + k;
        const int s = h + g.pe_shift[pe];
        const int v = g.pe_col[pe] * g.z + (s >= g.z ? s - g.z : s);
        const float4 tv = ld4(Tt + (size_t)v * TILE);
        float4 cv = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!FIRST) cv = ld4(Ct + (size_t)k * TILE);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float x = qmsg<MODE>(f4(tv, q) - f4(cv, q), p.clip);
            if (nudge && x == 0.f) x = 1e-4f;                   // Main_Functions.py:229-230
            float a = fabsf(x);
            if (!(a > 0.f)) a = 10000.f;                          // zeros never the min (:248)
            if (a < mn1[q]) { mn2[q] = mn1[q]; mn1[q] = a; ix[q] = k; }
            else if (a < mn2[q]) { mn2[q] = a; }
            sg[q] |= (uint64_t)(x > 0.f) << k;
        }
        if (UCN) {
            const uint64_t* hw = p.hd + hd_index(p, t - 1, tile, v);
            syn ^= (uint32_t)((hw[0] >> lane) & 1) | ((uint32_t)((hw[1] >> lane) & 1) << 1) |
                   ((uint32_t)((hw[2] >> lane) & 1) << 2) | ((uint32_t)((hw[3] >> lane) & 1) << 3);
        }
    }
    // pass 2: C->V messages (Main_Functions.py:250-316)
    const float* at = p.alpha + (size_t)t * g.E;
    const float* au = UCN ? p.alpha_ucn + (size_t)t * g.E : nullptr;
    int par[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) par[q] = __popcll(sg[q]) & 1;
    for (int k = 0; k < deg; ++k) {
        const float a = at[r0 + k];
        const float u = UCN ? au[r0 + k] : 0.f;
        float r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float m = (k == ix[q]) ? mn2[q] : mn1[q];
            if (m <= 1e-4f) m = m - 1e-4f;                          // :250
            const int odd = par[q] ^ (int)((sg[q] >> k) & 1);       // positives among others
            const float o = odd ? m : -m;                           // :251-254
            const float w = (UCN && ((syn >> q) & 1)) ? u : a;      // :275, :285, :295
            float x = fabsf(o) * w;
            x = (x > 0.f) ? x : 0.f;                                // :308
            x = qmsg<MODE>(x, p.clip);                              // :310-313
            r[q] = (o > 0.f) ? x : ((o < 0.f) ? -x : 0.f);          // :316 x * sign(o)
        }
        st4(Ct + (size_t)k * TILE, make_float4(r[0], r[1], r[2], r[3]));
    }
}

// ----------------------------------------------------------------------------------------
// variable-node update (Main_Functions.py:317-335), hard decisions, FER/BER accumulation
template <int MODE, bool LAST>
__global__ void __launch_bounds__(256) k_vn_update(DevGraph g, Bufs p, int t) {
    const int ngroups = (g.n_vars + VN_PER_WAVE - 1) / VN_PER_WAVE;
    const int64_t item = xcd_block() * 4 + uniform(threadIdx.x >> 6);
    const int64_t tile = item / ngroups;
    if (tile >= p.ntiles) return;
    const int grp = uniform((int)(item - tile * ngroups));
    const int lane = threadIdx.x & 63;
    const float* Ct = p.c2v + (size_t)tile * g.n_edges * TILE + 4 * lane;
    const bool count = p.count != 0;
    bool valid[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) valid[q] = (int64_t)(tile * TILE + 4 * lane + q) < p.B;
    uint32_t any_hd = 0, any_pos = 0;
    int nbits = 0;

    const int vbeg = grp * VN_PER_WAVE;
    const int vend = min(vbeg + VN_PER_WAVE, g.n_vars);
    for (int v = vbeg; v < vend; ++v) {
        const int j = v / g.z;
        const int gg = v - j * g.z;
        float4 S = make_float4(0.f, 0.f, 0.f, 0.f);
        // the column's edges four at a time: one scalar table load per edge and all four
        // message rows in flight before the (in-order, as before) sum
        const int e0 = g.col_ptr[j], e1 = g.col_ptr[j + 1];
        for (int e = e0; e < e1; e += 4) {
            float4 cv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e + u < e1) {
                    const int4 ve = g.vn_edge[e + u];
                    int h = gg - ve.z;
                    if (h < 0) h += g.z;
                    cv[u] = ld4(Ct + ((size_t)ve.x + (size_t)h * ve.y) * TILE);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (e + u < e1) { S.x += cv[u].x; S.y += cv[u].y; S.z += cv[u].z; S.w += cv[u].w; }
            }
        }
        const size_t vrow = ((size_t)tile * g.n_vars + v) * TILE + 4 * lane;
        const float4 ch = ld4(p.ch + vrow);
        float app[4];
        app[0] = fminf(fmaxf(qchan<MODE>(ch.x) + S.x, -p.clip), p.clip);
        app[1] = fminf(fmaxf(qchan<MODE>(ch.y) + S.y, -p.clip), p.clip);
        app[2] = fminf(fmaxf(qchan<MODE>(ch.z) + S.z, -p.clip), p.clip);
        app[3] = fminf(fmaxf(qchan<MODE>(ch.w) + S.w, -p.clip), p.clip);
        if (p.store_hd) {
            const uint64_t b0 = __ballot(app[0] >= 0.f), b1 = __ballot(app[1] >= 0.f);
            const uint64_t b2 = __ballot(app[2] >= 0.f), b3 = __ballot(app[3] >= 0.f);
            uint64_t* hw = p.hd + hd_index(p, t, tile, v);
            if (lane == 0) { hw[0] = b0; hw[1] = b1; hw[2] = b2; hw[3] = b3; }
        }
        if (!LAST) {
            const float beta = p.beta[(size_t)(t + 1) * g.N + j];
            float4 tn;
            tn.x = qchan<MODE>(ch.x * beta) + S.x;
            tn.y = qchan<MODE>(ch.y * beta) + S.y;
            tn.z = qchan<MODE>(ch.z * beta) + S.z;
            tn.w = qchan<MODE>(ch.w * beta) + S.w;
            st4(p.Tv + vrow, tn);
        }
        if (v < p.target_bits) {
            if (p.app_out) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (valid[q]) {
                        const int64_t b = tile * TILE + 4 * lane + q;
                        p.app_out[((size_t)t * p.B + b) * p.target_bits + v] = app[q];
                    }
                }
            }
            if (count) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool hd = valid[q] && app[q] >= 0.f;
                    any_hd |= (uint32_t)hd << q;
                    if (LAST) {
                        any_pos |= (uint32_t)(valid[q] && app[q] > 0.f) << q;
                        nbits += hd;
                    }
                }
            }
        }
    }
    if (count) {
        uint64_t* wr = p.wrong + ((size_t)t * p.ntiles + tile) * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t m = __ballot((any_hd >> q) & 1);
            if (lane == q && m) atomicOr(reinterpret_cast<unsigned long long*>(wr + q), (unsigned long long)m);
        }
        if (LAST) {
            uint64_t* ap = p.anypos + (size_t)tile * 4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint64_t m = __ballot((any_pos >> q) & 1);
                if (lane == q && m) atomicOr(reinterpret_cast<unsigned long long*>(ap + q), (unsigned long long)m);
            }
            for (int off = 32; off > 0; off >>= 1) nbits += __shfl_xor(nbits, off);
            if (lane == 0 && nbits) atomicAdd(p.biterr + tile, nbits);
        }
    }
}

// ----------------------------------------------------------------------------------------
template <int MODE>
static int launch_iterations(const DevGraph& g, const Bufs& b, const float* llr, bool ucn,
                             hipStream_t s) {
    const int T = b.T;
    const int nchunks = (g.n_vars + 31) / 32;
    const dim3 blk(256);
    if (ucn) hipLaunchKernelGGL((k_prologue<MODE, true>), dim3(b.ntiles * nchunks), blk, 0, s, g, b, llr);
    else hipLaunchKernelGGL((k_prologue<MODE, false>), dim3(b.ntiles * nchunks), blk, 0, s, g, b, llr);
    const int64_t cn_waves = (int64_t)b.ntiles * g.n_checks;
    const int ngroups = (g.n_vars + VN_PER_WAVE - 1) / VN_PER_WAVE;
    const int64_t vn_waves = (int64_t)b.ntiles * ngroups;
    const dim3 cn_grid(round_up8((cn_waves + 3) / 4));
    const dim3 vn_grid(round_up8((vn_waves + 3) / 4));
    for (int t = 0; t < T; ++t) {
        if (t == 0) {
            if (ucn) hipLaunchKernelGGL((k_cn_update<MODE, true, true>), cn_grid, blk, 0, s, g, b, t);
            else hipLaunchKernelGGL((k_cn_update<MODE, true, false>), cn_grid, blk, 0, s, g, b, t);
        } else {
            if (ucn) hipLaunchKernelGGL((k_cn_update<MODE, false, true>), cn_grid, blk, 0, s, g, b, t);
            else hipLaunchKernelGGL((k_cn_update<MODE, false, false>), cn_grid, blk, 0, s, g, b, t);
        }
        if (t == T - 1) hipLaunchKernelGGL((k_vn_update<MODE, true>), vn_grid, blk, 0, s, g, b, t);
        else hipLaunchKernelGGL((k_vn_update<MODE, false>), vn_grid, blk, 0, s, g, b, t);
    }
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

int flood_decode(const DevGraph& g, const Bufs& b, const float* llr, int mode, bool ucn,
                 hipStream_t s) {
    switch (mode) {
        case MODE_Q6: return launch_iterations<MODE_Q6>(g, b, llr, ucn, s);
        case MODE_Q5: return launch_iterations<MODE_Q5>(g, b, llr, ucn, s);
        case MODE_QM5: return launch_iterations<MODE_QM5>(g, b, llr, ucn, s);
        case MODE_Q4: return launch_iterations<MODE_Q4>(g, b, llr, ucn, s);
        case MODE_Q3: return launch_iterations<MODE_Q3>(g, b, llr, ucn, s);
        case MODE_MS: return launch_iterations<MODE_MS>(g, b, llr, ucn, s);
        case MODE_MSNN: return launch_iterations<MODE_MSNN>(g, b, llr, ucn, s);
        case MODE_SP: return launch_iterations<MODE_SP>(g, b, llr, ucn, s);
        default: return LDPC_ERR_ARG;
    }
}

}  // namespace ldpc
