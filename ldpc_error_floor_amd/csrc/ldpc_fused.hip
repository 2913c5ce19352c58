// ldpc_fused.hip — all T flooding iterations of the QMS decoder in ONE launch.
//
// Same algorithm as ldpc_flood.hip / oracle/nms_oracle.py (Main_Functions.py:157-385), but a
// workgroup owns CW codewords for the whole decode, so nothing but the input LLRs and the
// final counters touches HBM:
//
//   LDS  W[v][cw]   int32: low 16 bits = Tv = lw + S (the VN total the check side reads),
//                          high 16 bits = S_{t+1} accumulated by ds_add from the check side
//        CH[v][cw]  f32 channel LLR (Q(beta_t * ch) needs the raw value every iteration)
//        HD[...]    hard-decision bits of the previous iteration (UCN only)
//   VGPR per check group: the compressed C->V state of min-sum — the quantized output
//        magnitude of the argmin edge and of the others, the argmin index, and the mask of
//        edges with an odd number of other positive inputs; every C->V message is re-derived
//        from these (per-edge weights keep the raw minima instead).
//
// Arithmetic is integer in units of the q-bit grid step (q=5: 0.5, q=-5/4: 1, q=3: 2):
// sums/differences of grid values stay on the grid, so Q() of them is a clamp, and the only
// real roundings — Q(beta * ch) and Q(alpha * m) — use the same fp32 multiply +
// round-half-even as the reference.  Results are bit-identical to the fp32 reference.
//
// Lanes: lane = slot * CW + cw.  The SLOTS = 64/CW slots of a wave work on SLOTS checks of
// the same proto row (h = hg + slot*hstep), so the row's degree, columns, shifts and weights
// stay wave-uniform (scalar registers) while each slot gathers its own variables.
#include <cstdlib>

#include "ldpc_fused.h"

namespace ldpc {

constexpr int FUSED_THREADS = 1024;
constexpr int FUSED_NW = FUSED_THREADS / 64;
constexpr int FUSED_MAXG = 8;          // check groups per wave (state registers)
constexpr int FUSED_MAXDEG = 32;       // sign masks are 32-bit
constexpr int BIG_U = 1023;            // "no other edge": value 10000 (Main_Functions.py:248)
constexpr size_t FUSED_LDS_MAX = 160 * 1024;

template <int MODE> struct Grid;
template <> struct Grid<MODE_Q5> { static constexpr float step = 0.5f, inv = 2.0f; static constexpr int qmax = 15; };
template <> struct Grid<MODE_QM5> { static constexpr float step = 1.0f, inv = 1.0f; static constexpr int qmax = 15; };
template <> struct Grid<MODE_Q4> { static constexpr float step = 1.0f, inv = 1.0f; static constexpr int qmax = 7; };
template <> struct Grid<MODE_Q3> { static constexpr float step = 2.0f, inv = 0.5f; static constexpr int qmax = 3; };

// Q(x) in grid units: clamp(rint(x / step), +-qmax)  (== Cal_MSA_Q_TF(x) / step)
template <int MODE>
__device__ __forceinline__ int qunits(float x) {
    const float r = fminf(fmaxf(rintf(x * Grid<MODE>::inv), -(float)Grid<MODE>::qmax),
                          (float)Grid<MODE>::qmax);
    return (int)r;
}
// quantized C->V magnitude for a check-side minimum of m units and weight w (:266-313)
template <int MODE>
__device__ __forceinline__ int qmag(int m, float w) {
    const float mv = (m >= BIG_U) ? 10000.0f : (float)m * Grid<MODE>::step;
    float x = mv * w;                          // fl32(|o| * w)
    x = (x > 0.f) ? x : 0.f;                   // x * [x > 0]
    return qunits<MODE>(x);
}

struct FusedArgs {
    DevGraph g;
    const float* llr;          // [B][n_vars]
    const float* alpha;        // [T][E]
    const float* alpha_ucn;    // [T][E] or null
    const float* beta;         // [T][N]
    float* app_out;            // [T][B][target_bits] or null
    uint64_t* hd_out;          // flood ballot layout, slots T+1 (compat bit export) or null
    int64_t* counters;         // [4] or null
    uint8_t* flags;            // [B] or null
    int64_t B;
    int ntiles;                // ceil(B/256), for hd_out indexing
    int T, target_bits;
    int per_edge_w;            // weights differ inside a proto row
    int clip_u;                // clip_LLR in grid units
    int hstep, ngroups, nent;
    uint32_t zmagic;           // ceil(2^32 / z)
};

// C->V message (grid units) of edge k from a check-group state
struct CState {
    int mA, mB, idx;           // magnitudes (quantized, or raw minima with per-edge weights)
    uint32_t osg;              // bit k: odd number of OTHER positive inputs -> sign +
    int ucn;                   // syndrome of the previous hard decision (per lane)
};

template <int MODE, bool PEW>
__device__ __forceinline__ int c2v_msg(const CState& s, int k, float w, float wu) {
    int m = (k == s.idx) ? s.mB : s.mA;
    if constexpr (PEW) m = qmag<MODE>(m, s.ucn ? wu : w);
    return ((s.osg >> k) & 1u) ? m : -m;
}

template <int MODE, int CW, bool UCN, bool PEW>
__global__ void __launch_bounds__(FUSED_THREADS)
k_fused(FusedArgs a, const float* __restrict__ alpha, const float* __restrict__ alpha_ucn) {
    constexpr int SLOTS = 64 / CW;
    constexpr int qmax = Grid<MODE>::qmax;
    constexpr float step = Grid<MODE>::step;
    const DevGraph& g = a.g;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nv = g.n_vars;
    const int z = g.z;
    uint32_t* W = reinterpret_cast<uint32_t*>(smem);                         // [nv][CW]
    float* CH = reinterpret_cast<float*>(smem + (size_t)nv * CW * 4);         // [nv][CW]
    uint64_t* HD = reinterpret_cast<uint64_t*>(smem + (size_t)nv * CW * 8);   // entry bits
    const int hd_words = (nv * CW + 63) / 64;
    float* BETA = reinterpret_cast<float*>(HD + hd_words);                   // [T][N]
    unsigned long long* RED =
        reinterpret_cast<unsigned long long*>(BETA + (((size_t)a.T * g.N + 1) & ~(size_t)1));
    // RED: 0 wrong_t, 1 all_wrong, 2 any_pos (last t), 3 bit errors (last t), 5/6 flags

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int slot = lane / CW;
    const int cw = lane - slot * CW;
    const int64_t b0 = (int64_t)blockIdx.x * CW;
    const int64_t nvalid = (b0 + CW <= a.B) ? CW : (a.B - b0);
    constexpr bool ucn = UCN;
    constexpr bool pew = PEW;
    const unsigned long long cwmask = (CW == 64) ? ~0ull : ((1ull << CW) - 1);
    const unsigned long long valid_cw = (nvalid >= 64) ? ~0ull : ((1ull << nvalid) - 1);
    const uint32_t zmagic = a.zmagic;                 // v / z == umulhi(v, zmagic) for v < 2^16

    // ---- per-group graph info, kept in VGPRs for the whole decode -------------------------
    // einf: lane k < deg holds edge k of the group's proto row: (col*z) << 16 | shift
    // hinf: this lane's check index h (or a valid stand-in) | valid << 16
    // rinf: lane-uniform r0 | deg << 16
    uint32_t einf[FUSED_MAXG], hinf[FUSED_MAXG], rinf[FUSED_MAXG];
#pragma unroll
    for (int gi = 0; gi < FUSED_MAXG; ++gi) {
        einf[gi] = 0; hinf[gi] = 0; rinf[gi] = 0;
        const int grp = wave + gi * FUSED_NW;
        if (grp < a.ngroups) {
            const int i = grp / a.hstep;
            const int hg = grp - i * a.hstep;
            const int r0 = g.row_ptr[i];
            const int deg = g.row_ptr[i + 1] - r0;
            if (lane < deg)
                einf[gi] = ((uint32_t)(g.pe_col[r0 + lane] * z) << 16) | (uint32_t)g.pe_shift[r0 + lane];
            const int h = hg + slot * a.hstep;
            const bool valid = h < z;
            hinf[gi] = (uint32_t)(valid ? h : hg) | ((uint32_t)valid << 16);
            rinf[gi] = (uint32_t)r0 | ((uint32_t)deg << 16);
        }
    }

    // ---- prologue: LLRs -> CH (transposed), beta table, W = Tv_0, HD = (lw_0 >= 0) ---------
    for (int f = tid; f < CW * nv; f += FUSED_THREADS) {
        const int r = f / nv, v = f - r * nv;                 // coalesced global read
        CH[v * CW + r] = (r < nvalid) ? a.llr[(b0 + r) * nv + v] : 0.f;
    }
    for (int f = tid; f < a.T * g.N; f += FUSED_THREADS) BETA[f] = a.beta[f];
    if (tid < 8) RED[tid] = (tid == 1) ? ~0ull : 0ull;
    __syncthreads();
    const int total = nv * CW;
    for (int r = 0; r < a.nent; ++r) {
        const int e = tid + r * FUSED_THREADS;
        const bool in = e < total;
        int tv = 0;
        if (in) {
            const uint32_t v = (uint32_t)e / CW;
            tv = qunits<MODE>(CH[e] * BETA[__umulhi(v, zmagic)]);   // lw_0 = Q(beta_0 * ch)
            W[e] = (uint32_t)tv & 0xFFFFu;
        }
        if (ucn) {
            const uint64_t bal = __ballot(in && tv >= 0);
            if (lane == 0 && e - lane < total) HD[(e - lane) >> 6] = bal;
        }
    }
    __syncthreads();

    // ---- check-group state ---------------------------------------------------------------
    CState st[FUSED_MAXG];
#pragma unroll
    for (int gi = 0; gi < FUSED_MAXG; ++gi) { st[gi].mA = 0; st[gi].mB = 0; st[gi].idx = 0; st[gi].osg = 0; st[gi].ucn = 0; }

    for (int t = 0; t < a.T; ++t) {
        if (tid == 0 && t > 0) {   // fold iteration t-1's frame flags (its VN phase is done)
            RED[1] &= RED[0];
            RED[0] = 0;
        }
        // ======== check nodes: V->C from Tv and C2V_t, two minima, new state, S scatter =====
        const float* at = alpha + (size_t)t * g.E;
        const float* au = ucn ? alpha_ucn + (size_t)t * g.E : nullptr;
        const float* at_prev = alpha + (size_t)(t > 0 ? t - 1 : 0) * g.E;
        const float* au_prev = ucn ? alpha_ucn + (size_t)(t > 0 ? t - 1 : 0) * g.E : nullptr;
#pragma unroll
        for (int gi = 0; gi < FUSED_MAXG; ++gi) {
            const int grp = wave + gi * FUSED_NW;
            if (grp >= a.ngroups) break;
            const uint32_t ri = __builtin_amdgcn_readfirstlane(rinf[gi]);
            const int r0 = (int)(ri & 0xFFFFu);
            const int deg = (int)(ri >> 16);
            const uint32_t hl = hinf[gi] & 0xFFFFu;
            const bool valid = (hinf[gi] >> 16) != 0;
            const uint32_t ei = einf[gi];
            uint32_t k1 = ((uint32_t)BIG_U << 6) | 63u, k2 = k1;
            uint32_t neg = 0, syn = 0;
            CState& s = st[gi];

            for (int k = 0; k < deg; ++k) {
                const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)ei, k);
                const uint32_t a1 = hl + (info & 0xFFFFu);
                const uint32_t hs = min(a1, a1 - (uint32_t)z);          // (h + shift) mod z
                const int e = (int)(((info >> 16) + hs) * CW) + cw;
                const int tv = (int)(int16_t)(W[e] & 0xFFFFu);
                // C2V_t from the previous state (all-zero state at t = 0 gives 0)
                const float w = pew ? at_prev[r0 + k] : 0.f;
                const float wu = (pew && ucn) ? au_prev[r0 + k] : 0.f;
                const int cold = c2v_msg<MODE, PEW>(s, k, w, wu);
                int x = tv - cold;
                x = min(max(x, -qmax), qmax);                         // Q(v2c) on the grid
                const uint32_t mag = (uint32_t)(x < 0 ? -x : x);      // 0 == nudged +1e-4
                const uint32_t key = (mag << 6) | (uint32_t)k;
                k2 = max(k1, min(k2, key));
                k1 = min(k1, key);
                neg |= ((uint32_t)x >> 31) << k;                      // 0 -> +1e-4: positive
                if (ucn) syn ^= (uint32_t)(HD[e >> 6] >> (e & 63)) & 1u;
            }
            const uint32_t dmask = (deg >= 32) ? 0xFFFFFFFFu : ((1u << deg) - 1u);
            const uint32_t pos = ~neg & dmask;
            const uint32_t par = __popc(pos) & 1u;
            s.osg = pos ^ (par ? 0xFFFFFFFFu : 0u);
            s.idx = (int)(k1 & 63u);
            s.ucn = (int)syn;
            const int m1 = (int)(k1 >> 6), m2 = (int)(k2 >> 6);
            if (pew) {
                s.mA = m1;
                s.mB = m2;
            } else {
                const float w = (ucn && syn) ? au[r0] : at[r0];
                s.mA = qmag<MODE>(m1, w);
                s.mB = qmag<MODE>(m2, w);
            }
            if (valid) {

                for (int k = 0; k < deg; ++k) {
                    const uint32_t info = (uint32_t)__builtin_amdgcn_readlane((int)ei, k);
                    const uint32_t a1 = hl + (info & 0xFFFFu);
                    const uint32_t hs = min(a1, a1 - (uint32_t)z);
                    const int e = (int)(((info >> 16) + hs) * CW) + cw;
                    const float w = pew ? at[r0 + k] : 0.f;
                    const float wu = (pew && ucn) ? au[r0 + k] : 0.f;
                    const int c = c2v_msg<MODE, PEW>(s, k, w, wu);
                    atomicAdd(&W[e], (uint32_t)c << 16);
                }
            }
        }
        __syncthreads();
        // ======== variable nodes: APP, hard decision, Tv for the next iteration ============
        const bool last = (t == a.T - 1);
        const float* bnext = BETA + (size_t)(last ? t : t + 1) * g.N;
        uint32_t any_hd = 0, any_pos = 0, nbits = 0;
        for (int r = 0; r < a.nent; ++r) {
            const int e = tid + r * FUSED_THREADS;
            const bool in = e < total;
            int app = -1;
            if (in) {
                const uint32_t v = (uint32_t)e / CW;
                const uint32_t wv = W[e];
                const int S = (int)wv >> 16;
                const float ch = CH[e];
                app = qunits<MODE>(ch) + S;                           // Q(xa) + sum C2V
                app = min(max(app, -a.clip_u), a.clip_u);             // clip +-clip_LLR
                if (!last) {
                    const int tn = qunits<MODE>(ch * bnext[__umulhi(v, zmagic)]) + S;
                    W[e] = (uint32_t)tn & 0xFFFFu;
                }
                if ((int)v < a.target_bits) {
                    any_hd |= (uint32_t)(app >= 0);
                    if (last) { any_pos |= (uint32_t)(app > 0); nbits += (uint32_t)(app >= 0); }
                    if (a.app_out && cw < nvalid)
                        a.app_out[((size_t)t * a.B + b0 + cw) * a.target_bits + v] = (float)app * step;
                }
                if (a.hd_out && app >= 0 && cw < nvalid) {
                    const int64_t b = b0 + cw;
                    const int64_t tile = b / TILE;
                    const int bl = (int)(b - tile * TILE);
                    const size_t idx = ((((size_t)(t + 1) * a.ntiles + tile) * nv + v) * 4) + (bl & 3);
                    atomicOr(reinterpret_cast<unsigned long long*>(a.hd_out + idx), 1ull << (bl >> 2));
                }
            }
            if (ucn) {
                const uint64_t bal = __ballot(in && app >= 0);
                if (lane == 0 && e - lane < total) HD[(e - lane) >> 6] = bal;
            }
        }
        // per-codeword OR over this wave's entries (lanes l, l+CW, ... share codeword l%CW)
        unsigned long long bw = __ballot(any_hd);
        unsigned long long m = 0;
#pragma unroll
        for (int s2 = 0; s2 < SLOTS; ++s2) m |= (bw >> (s2 * CW)) & cwmask;
        if (lane == 0 && m) atomicOr(&RED[0], m);
        if (last) {
            bw = __ballot(any_pos);
            m = 0;
#pragma unroll
            for (int s2 = 0; s2 < SLOTS; ++s2) m |= (bw >> (s2 * CW)) & cwmask;
            if (lane == 0 && m) atomicOr(&RED[2], m);
            uint32_t nb = (cw < nvalid) ? nbits : 0u;
            for (int off = 32; off > 0; off >>= 1) nb += __shfl_xor(nb, off);
            if (lane == 0 && nb) atomicAdd(&RED[3], (unsigned long long)nb);
        }
        __syncthreads();
    }
    if (tid == 0) {
        const unsigned long long wl = RED[0] & valid_cw;
        const unsigned long long all = RED[1] & RED[0] & valid_cw;
        const unsigned long long ap = RED[2] & valid_cw;
        if (a.counters) {
            const unsigned long long c0 = RED[3];
            const unsigned long long c1 = __popcll(wl);
            const unsigned long long c2 = __popcll(all);
            const unsigned long long c3 = 2ull * __popcll(ap) + __popcll(wl & ~ap);
            unsigned long long* cc = reinterpret_cast<unsigned long long*>(a.counters);
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

// ---- host side ---------------------------------------------------------------------------
namespace {

int fused_cw(const DevGraph& g, int T) {
    if (g.z == 1) return 64;
    for (int cw : {32, 16, 8}) {
        const size_t lds = (size_t)g.n_vars * cw * 8 + (size_t)((g.n_vars * cw + 63) / 64) * 8 +
                           (((size_t)T * g.N + 1) & ~(size_t)1) * 4 + 8 * 8;
        if (lds <= FUSED_LDS_MAX) return cw;
    }
    return 0;
}

size_t fused_lds(const DevGraph& g, int T, int cw) {
    return (size_t)g.n_vars * cw * 8 + (size_t)((g.n_vars * cw + 63) / 64) * 8 +
           (((size_t)T * g.N + 1) & ~(size_t)1) * 4 + 8 * 8;
}

template <int MODE, int CW, bool UCN, bool PEW>
int launch_k(const FusedArgs& a, int nblocks, size_t lds, hipStream_t s) {
    static bool attr_set = false;
    if (!attr_set) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused<MODE, CW, UCN, PEW>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)FUSED_LDS_MAX);
        attr_set = true;
    }
    hipLaunchKernelGGL((k_fused<MODE, CW, UCN, PEW>), dim3(nblocks), dim3(FUSED_THREADS), lds, s, a,
                       a.alpha, a.alpha_ucn);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

template <int MODE, int CW>
int launch(const FusedArgs& a, int nblocks, size_t lds, hipStream_t s) {
    const bool ucn = a.alpha_ucn != nullptr;
    if (a.per_edge_w)
        return ucn ? launch_k<MODE, CW, true, true>(a, nblocks, lds, s)
                   : launch_k<MODE, CW, false, true>(a, nblocks, lds, s);
    return ucn ? launch_k<MODE, CW, true, false>(a, nblocks, lds, s)
               : launch_k<MODE, CW, false, false>(a, nblocks, lds, s);
}

template <int MODE>
int launch_mode(const FusedArgs& a, int cw, int nblocks, size_t lds, hipStream_t s) {
    switch (cw) {
        case 64: return launch<MODE, 64>(a, nblocks, lds, s);
        case 32: return launch<MODE, 32>(a, nblocks, lds, s);
        case 16: return launch<MODE, 16>(a, nblocks, lds, s);
        case 8: return launch<MODE, 8>(a, nblocks, lds, s);
        default: return LDPC_ERR_UNSUPPORTED;
    }
}

float mode_step(int mode) {
    switch (mode) {
        case MODE_Q5: return 0.5f;
        case MODE_QM5: case MODE_Q4: return 1.0f;
        case MODE_Q3: return 2.0f;
        default: return 0.f;
    }
}

}  // namespace

static int fused_version() {
    const char* e = getenv("LDPC_FUSED_VERSION");
    return e ? atoi(e) : 5;   // 5: v5 (fallback v3), 4: v4 packed experiment, 3: v3, 2: v2
}

static bool fused2_supported(const DevGraph& g, int T);

static int mode_qmax(int mode) { return (mode == MODE_Q4) ? 7 : (mode == MODE_Q3) ? 3 : 15; }

bool fused_supported(const DevGraph& g, int mode, int T) {
    if (mode != MODE_Q5 && mode != MODE_QM5 && mode != MODE_Q4 && mode != MODE_Q3) return false;
    if (g.n_vars >= 32768) return false;
    if (fused_version() >= 5 && fused5_supported(g, T)) return true;
    if (fused_version() >= 3 && fused3_supported(g, T)) return true;
    return fused2_supported(g, T);
}

const char* fused_kernel_name(const DevGraph& g, int mode, int T, bool per_edge_w) {
    if (!fused_supported(g, mode, T)) return "";
    if (fused_version() >= 5 && fused5_supported(g, T)) return fused5_shape_name(g, T);
    if (fused_version() == 4 && fused4_supported(g, T, mode_qmax(mode), per_edge_w))
        return fused4_shape_name(g, T);
    if (fused_version() >= 3 && fused3_supported(g, T)) return fused3_shape_name(g, T);
    return "fused2";
}

static bool fused2_supported(const DevGraph& g, int T) {
    if (g.max_cdeg > FUSED_MAXDEG) return false;
    if (g.n_vars >= 65536 || g.z >= 65536) return false;      // 16-bit packed graph info
    const int cw = fused_cw(g, T);
    if (cw == 0) return false;
    const int slots = 64 / cw;
    const int hstep = (g.z + slots - 1) / slots;
    if ((int64_t)g.M * hstep > (int64_t)FUSED_NW * FUSED_MAXG) return false;
    return true;
}

int64_t fused_bytes_per_cw(const DevGraph& g, int T) {
    (void)T;
    // compulsory: the channel LLRs are read once; outputs are counters only
    return (int64_t)g.n_vars * 4;
}

int fused_decode(const DevGraph& g, Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
                 bool ucn, bool want_bits, int ntiles_max, int T_max, int per_edge_w,
                 int64_t* counters, uint8_t* flags, hipStream_t s) {
    if (!fused_supported(g, mode, b.T)) return LDPC_ERR_UNSUPPORTED;
    const float step = mode_step(mode);
    const float cu = b.clip / step;
    if (cu != rintf(cu) || cu > 32000.f) return LDPC_ERR_UNSUPPORTED;
    uint64_t* hd_out = nullptr;
    if (want_bits) {
        const size_t elems = (size_t)(T_max + 1) * ntiles_max * g.n_vars * 4;
        if ((int64_t)elems > ws.hd_elems) {
            if (ws.hd) (void)hipFree(ws.hd);
            ws.hd = nullptr;
            ws.hd_elems = 0;
            if (hipMalloc(reinterpret_cast<void**>(&ws.hd), elems * sizeof(uint64_t)) != hipSuccess) {
                (void)hipGetLastError();
                return LDPC_ERR_OOM;
            }
            ws.hd_elems = (int64_t)elems;
        }
        if (hipMemsetAsync(ws.hd, 0, (size_t)(b.T + 1) * b.ntiles * g.n_vars * 4 * sizeof(uint64_t), s) != hipSuccess)
            return LDPC_ERR_HIP;
        hd_out = ws.hd;
    }
    if (fused_version() >= 5 && fused5_supported(g, b.T))
        return fused5_decode(g, b, ws, llr, mode_qmax(mode), step, (int)cu, per_edge_w != 0, hd_out,
                             counters, flags, s);
    if (b.awgn) return LDPC_ERR_UNSUPPORTED;          // in-kernel channel: v5 only
    if (fused_version() == 4 && fused4_supported(g, b.T, mode_qmax(mode), per_edge_w != 0))
        return fused4_decode(g, b, llr, mode_qmax(mode), step, (int)cu, hd_out, counters, flags, s);
    if (fused_version() >= 3 && fused3_supported(g, b.T)) {
        const int qmax = mode_qmax(mode);
        return fused3_decode(g, b, llr, qmax, step, (int)cu, per_edge_w != 0, hd_out, counters,
                             flags, s);
    }
    const int cw = fused_cw(g, b.T);
    FusedArgs a{};
    a.g = g;
    a.llr = llr;
    a.alpha = b.alpha;
    a.alpha_ucn = ucn ? b.alpha_ucn : nullptr;
    a.beta = b.beta;
    a.app_out = b.app_out;
    a.counters = nullptr;
    a.flags = nullptr;
    a.B = b.B;
    a.ntiles = b.ntiles;
    a.T = b.T;
    a.target_bits = b.target_bits;
    a.per_edge_w = per_edge_w;
    a.clip_u = (int)cu;
    const int slots = 64 / cw;
    a.hstep = (g.z + slots - 1) / slots;
    a.ngroups = g.M * a.hstep;
    a.nent = (g.n_vars * cw + FUSED_THREADS - 1) / FUSED_THREADS;
    a.zmagic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.z - 1) / (uint64_t)g.z);
    a.hd_out = hd_out;
    a.counters = counters;
    a.flags = flags;
    const int nblocks = (int)((b.B + cw - 1) / cw);
    const size_t lds = fused_lds(g, b.T, cw);
    switch (mode) {
        case MODE_Q5: return launch_mode<MODE_Q5>(a, cw, nblocks, lds, s);
        case MODE_QM5: return launch_mode<MODE_QM5>(a, cw, nblocks, lds, s);
        case MODE_Q4: return launch_mode<MODE_Q4>(a, cw, nblocks, lds, s);
        case MODE_Q3: return launch_mode<MODE_Q3>(a, cw, nblocks, lds, s);
        default: return LDPC_ERR_UNSUPPORTED;
    }
}

void fused_bits_view(const FusedWorkspace& ws, Bufs& b) {
    b.hd = ws.hd;
    b.hd_all = 1;
}

void fused_free(FusedWorkspace& ws) {
    if (ws.hd) (void)hipFree(ws.hd);
    ws.hd = nullptr;
    ws.hd_elems = 0;
    if (ws.tables) (void)hipFree(ws.tables);
    ws.tables = nullptr;
    ws.tables_bytes = 0;
}

}  // namespace ldpc
