// ldpc_capi.hip — C ABI (include/ldpc_nms.h): graph/weights/context management, decode
// dispatch, and the small compat kernels (output export, FER/BER counter finalisation).
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "ldpc_awgn.h"
#include "ldpc_internal.h"
#include "ldpc_fused.h"

using namespace ldpc;

struct ldpc_graph {
    int device = 0;
    host::GraphTables h;       // host tables (ldpc_host.cpp), also the device image
    int32_t* d_tables = nullptr;
    DevGraph dev{};
    int T_w = 0;
    int per_edge_w = 0;        // CN weights differ inside a proto row (sharing 1/4)
    std::vector<int32_t> row_merge;   // [M] DevGraph::h_row_merge
    int32_t* d_row_merge = nullptr;
    float* d_alpha = nullptr;
    float* d_alpha_ucn = nullptr;
    float* d_beta = nullptr;
    int32_t* d_beta_tid = nullptr;   // [T][N] host::WeightInfo::beta_tid
};

struct ldpc_ctx {
    ldpc_graph* g = nullptr;
    int64_t B_max = 0;
    int T_max = 0;
    int ntiles_max = 0;
    // flooding workspace (allocated on first use)
    float* ch = nullptr;
    float* Tv = nullptr;
    float* c2v = nullptr;
    uint64_t* hd = nullptr;
    // counters workspace (always)
    uint64_t* wrong = nullptr;
    uint64_t* anypos = nullptr;
    int32_t* biterr = nullptr;
    // fused workspace
    FusedWorkspace fused{};
    // LLR buffer for ldpc_decode_awgn when the kernel cannot generate in its prologue
    float* llr_scratch = nullptr;
    int64_t llr_scratch_n = 0;
    // the bit-sliced kernels' in-prologue channel: the level sampler's tables (awgn_gen_table),
    // on the device and the host copy last uploaded
    uint32_t* gen_tab = nullptr;
    uint32_t gen_host[AWGN_TAB_W] = {};
    bool gen_valid = false;
    // recorded on the decode's stream after every decode that reads gen_tab: a table change
    // waits for it, so a decode still running on another stream keeps the tables it started with
    hipEvent_t gen_done = nullptr;
    bool gen_pending = false;
    char last_kernel[64] = {0};   // ldpc_ctx_last_kernel
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename T>
int dev_alloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) return LDPC_OK;
    if (hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        *p = nullptr;
        return LDPC_ERR_OOM;
    }
    return LDPC_OK;
}

template <typename T>
void dev_free(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

// ---- compat kernels --------------------------------------------------------------------
// The hard decision of codeword b, variable v at iteration t, wherever the decode left it: the
// tile layout of flood / v5 (Bufs::hd, slot t + 1), or the bit-sliced kernels' packed words
// (except packs the v5 fixup decoded, which are in the tile layout).
struct HdSrc {
    const uint64_t* tile;
    const uint32_t* pack;
    const uint32_t* bad;
    int64_t npk;
    int ntiles, n_vars;
    __device__ uint32_t bit(int t, int64_t b, int v) const {
        const int64_t pk = b >> 5;
        if (pack && !bad[pk]) return (pack[((size_t)t * npk + pk) * n_vars + v] >> (b & 31)) & 1u;
        const int64_t ti = b / TILE;
        const int bl = (int)(b - ti * TILE);
        return (uint32_t)((tile[(((size_t)(t + 1) * ntiles + ti) * n_vars + v) * 4 + (bl & 3)] >> (bl >> 2)) & 1u);
    }
};

__global__ void k_export_hard(HdSrc src, int64_t B, uint32_t* __restrict__ out, int T, int nwords) {
    const int64_t total = (int64_t)T * B * nwords;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int w = (int)(id % nwords);
        const int64_t b = (id / nwords) % B;
        const int t = (int)(id / ((int64_t)nwords * B));
        uint32_t word = 0;
        for (int k = 0; k < 32; ++k) {
            const int v = w * 32 + k;
            if (v >= src.n_vars) break;
            word |= src.bit(t, b, v) << k;
        }
        out[id] = word;
    }
}

// syndrome H hd_t mod 2 per check (the quantity the reference computes as the UCN indicator of
// iteration t + 1, Main_Functions.py:180-209)
__global__ void k_export_synd(DevGraph g, HdSrc src, int64_t B, uint32_t* __restrict__ out, int T, int nwords) {
    const int64_t total = (int64_t)T * B * nwords;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int w = (int)(id % nwords);
        const int64_t b = (id / nwords) % B;
        const int t = (int)(id / ((int64_t)nwords * B));
        uint32_t word = 0;
        for (int k = 0; k < 32; ++k) {
            const int c = w * 32 + k;
            if (c >= g.n_checks) break;
            const int i = c / g.z, h = c - i * g.z;
            uint32_t par = 0;
            for (int pe = g.row_ptr[i]; pe < g.row_ptr[i + 1]; ++pe) {
                const int s = h + g.pe_shift[pe];
                const int v = g.pe_col[pe] * g.z + (s >= g.z ? s - g.z : s);
                par ^= src.bit(t, b, v);
            }
            word |= par << k;
        }
        out[id] = word;
    }
}

// flood's per-iteration frame flags (Bufs::wrong, [T][tiles][4] ballot words) -> iter_wrong
__global__ void k_iter_wrong(Bufs p, uint32_t* __restrict__ out) {
    const int64_t npk = (p.B + 31) >> 5;
    const int64_t total = (int64_t)p.T * npk;
    for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < total;
         id += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(id / npk);
        const int64_t pk = id - (int64_t)t * npk;
        uint32_t word = 0;
        for (int r = 0; r < 32; ++r) {
            const int64_t b = 32 * pk + r;
            if (b >= p.B) break;
            const int64_t ti = b / TILE;
            const int bl = (int)(b - ti * TILE);
            word |= (uint32_t)((p.wrong[((size_t)t * p.ntiles + ti) * 4 + (bl & 3)] >> (bl >> 2)) & 1u) << r;
        }
        out[id] = word;
    }
}

__global__ void k_finalize(Bufs p, int64_t* __restrict__ counters, uint8_t* __restrict__ flags) {
    __shared__ unsigned long long red[4][256];
    unsigned long long c[4] = {0, 0, 0, 0};
    for (int64_t tile = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tile < p.ntiles;
         tile += (int64_t)gridDim.x * blockDim.x) {
        uint64_t wl[4], all[4], ap[4];
        for (int q = 0; q < 4; ++q) {
            uint64_t valid = 0;
            for (int l = 0; l < 64; ++l)
                if (tile * TILE + 4 * l + q < p.B) valid |= 1ull << l;
            wl[q] = p.wrong[((size_t)(p.T - 1) * p.ntiles + tile) * 4 + q] & valid;
            uint64_t a = valid;
            for (int t = 0; t < p.T; ++t) a &= p.wrong[((size_t)t * p.ntiles + tile) * 4 + q];
            all[q] = a;
            ap[q] = p.anypos[(size_t)tile * 4 + q] & valid;
            c[1] += __popcll(wl[q]);
            c[2] += __popcll(all[q]);
            c[3] += 2 * __popcll(ap[q]) + __popcll(wl[q] & ~ap[q]);
        }
        c[0] += (unsigned long long)p.biterr[tile];
        if (flags) {
            for (int bl = 0; bl < TILE; ++bl) {
                const int64_t b = tile * TILE + bl;
                if (b >= p.B) break;
                const int lane = bl >> 2, q = bl & 3;
                flags[b] = (uint8_t)(((all[q] >> lane) & 1) | (((wl[q] >> lane) & 1) << 1));
            }
        }
    }
    for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = c[k];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && counters)
        for (int k = 0; k < 4; ++k)
            if (red[k][0]) atomicAdd(reinterpret_cast<unsigned long long*>(counters + k), red[k][0]);
}

int ensure_counters(ldpc_ctx* c) {
    if (c->wrong) return LDPC_OK;
    const size_t nt = (size_t)c->ntiles_max;
    int st = dev_alloc(&c->wrong, (size_t)c->T_max * nt * 4);
    if (st == LDPC_OK) st = dev_alloc(&c->anypos, nt * 4);
    if (st == LDPC_OK) st = dev_alloc(&c->biterr, nt);
    return st;
}

int ensure_flood(ldpc_ctx* c) {
    if (c->ch) return LDPC_OK;
    const ldpc_graph* g = c->g;
    const size_t nt = (size_t)c->ntiles_max;
    const size_t nv = (size_t)g->h.N * g->h.z, ne = (size_t)g->h.E * g->h.z;
    int st = dev_alloc(&c->ch, nt * nv * TILE);
    if (st == LDPC_OK) st = dev_alloc(&c->Tv, nt * nv * TILE);
    if (st == LDPC_OK) st = dev_alloc(&c->c2v, nt * ne * TILE);
    if (st == LDPC_OK) st = dev_alloc(&c->hd, (size_t)(c->T_max + 1) * nt * nv * 4);
    if (st != LDPC_OK) {
        dev_free(c->ch); dev_free(c->Tv); dev_free(c->c2v); dev_free(c->hd);
    }
    return st;
}

}  // namespace

extern "C" {

int ldpc_abi_version(void) { return LDPC_NMS_ABI_VERSION; }

const char* ldpc_status_string(int status) {
    switch (status) {
        case LDPC_OK: return "ok";
        case LDPC_ERR_ARG: return "invalid argument";
        case LDPC_ERR_HIP: return "HIP runtime error";
        case LDPC_ERR_OOM: return "device out of memory";
        case LDPC_ERR_STATE: return "invalid state (weights not set or limits exceeded)";
        case LDPC_ERR_UNSUPPORTED: return "unsupported configuration";
        default: return "unknown status";
    }
}

int ldpc_graph_create(const int32_t* proto, int32_t M, int32_t N, int32_t z, int32_t device,
                      ldpc_graph** out) {
    if (!out) return LDPC_ERR_ARG;
    *out = nullptr;
    ldpc_graph* g = new (std::nothrow) ldpc_graph();
    if (!g) return LDPC_ERR_OOM;
    const int st = host::build_graph(proto, M, N, z, g->h);
    if (st != LDPC_OK) { delete g; return st; }
    g->device = device;
    const host::GraphTables& h = g->h;
    {
        DeviceGuard dg(device);
        if (dev_alloc(&g->d_tables, h.device_block.size()) != LDPC_OK) { delete g; return LDPC_ERR_OOM; }
        if (hipMemcpy(g->d_tables, h.device_block.data(), h.device_block.size() * sizeof(int32_t),
                      hipMemcpyHostToDevice) != hipSuccess) {
            dev_free(g->d_tables);
            delete g;
            return LDPC_ERR_HIP;
        }
    }
    DevGraph& d = g->dev;
    d.M = M; d.N = N; d.z = z; d.E = h.E;
    d.n_checks = M * z; d.n_vars = N * z; d.n_edges = h.E * z; d.max_cdeg = h.max_cdeg;
    const int32_t* p = g->d_tables;
    d.row_ptr = p; p += M + 1;
    d.pe_row = p; p += h.E;
    d.pe_col = p; p += h.E;
    d.pe_shift = p; p += h.E;
    d.col_ptr = p; p += N + 1;
    d.col_pe = p;
    d.vn_edge = reinterpret_cast<const int4*>(g->d_tables + h.off_vn);
    d.h_row_ptr = h.row_ptr.data();
    d.host = &g->h;
    *out = g;
    return LDPC_OK;
}

int ldpc_graph_destroy(ldpc_graph* g) {
    if (!g) return LDPC_ERR_ARG;
    DeviceGuard dg(g->device);
    dev_free(g->d_tables);
    dev_free(g->d_alpha);
    dev_free(g->d_alpha_ucn);
    dev_free(g->d_beta);
    dev_free(g->d_beta_tid);
    dev_free(g->d_row_merge);
    delete g;
    return LDPC_OK;
}

int ldpc_graph_query(const ldpc_graph* g, int32_t* dims) {
    if (!g || !dims) return LDPC_ERR_ARG;
    const host::GraphTables& h = g->h;
    const int32_t v[8] = {h.M, h.N, h.z, h.E, h.M * h.z, h.N * h.z, h.E * h.z, h.max_cdeg};
    std::memcpy(dims, v, sizeof(v));
    return LDPC_OK;
}

int ldpc_weights_set(ldpc_graph* g, int32_t T, const float* alpha, const float* alpha_ucn,
                     const float* beta) {
    if (!g) return LDPC_ERR_ARG;
    // alpha' equal to alpha bit for bit at every iteration: the unsatisfied-check weighting
    // (Main_Functions.py:266-304) selects between equal weights, so every kernel decodes it as a
    // decoder without UCN (no syndrome / hard-decision work; the same outputs exactly).  The
    // 5G BG2 trained weights of C4 are such a table.
    if (alpha && alpha_ucn && T > 0 && g->h.E > 0 &&
        std::memcmp(alpha, alpha_ucn, (size_t)T * g->h.E * sizeof(float)) == 0)
        alpha_ucn = nullptr;
    host::WeightInfo wi;
    const int sta = host::analyze_weights(g->h, T, alpha, alpha_ucn, beta, wi);
    if (sta != LDPC_OK) return sta;
    DeviceGuard dg(g->device);
    dev_free(g->d_alpha);
    dev_free(g->d_alpha_ucn);
    dev_free(g->d_beta);
    dev_free(g->d_beta_tid);
    g->dev.beta_tid = nullptr;
    g->T_w = 0;
    const size_t ne = (size_t)T * g->h.E, nn = (size_t)T * g->h.N;
    int st = dev_alloc(&g->d_alpha, ne);
    if (st == LDPC_OK && alpha_ucn) st = dev_alloc(&g->d_alpha_ucn, ne);
    if (st == LDPC_OK) st = dev_alloc(&g->d_beta, nn);
    if (st == LDPC_OK) st = dev_alloc(&g->d_beta_tid, nn);
    if (st != LDPC_OK) return st;
    bool ok = hipMemcpy(g->d_alpha, alpha, ne * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
    if (alpha_ucn)
        ok = ok && hipMemcpy(g->d_alpha_ucn, alpha_ucn, ne * sizeof(float),
                             hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(g->d_beta, beta, nn * sizeof(float), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(g->d_beta_tid, wi.beta_tid.data(), nn * sizeof(int32_t), hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) return LDPC_ERR_HIP;
    g->dev.beta_tid = g->d_beta_tid;
    g->T_w = T;
    g->per_edge_w = wi.per_edge_w;
    g->row_merge = wi.row_merge;
    g->dev.h_row_merge = nullptr;
    g->dev.row_merge = nullptr;
    if (!g->d_row_merge) {
        const int st2 = dev_alloc(&g->d_row_merge, (size_t)g->h.M);
        if (st2 != LDPC_OK) return st2;
    }
    if (hipMemcpy(g->d_row_merge, g->row_merge.data(), (size_t)g->h.M * sizeof(int32_t),
                  hipMemcpyHostToDevice) != hipSuccess)
        return LDPC_ERR_HIP;
    g->dev.h_row_merge = g->row_merge.data();
    g->dev.row_merge = g->d_row_merge;
    g->dev.w_alpha_uniform = wi.alpha_uniform;
    g->dev.w_alpha_pair_uniform = wi.alpha_pair_uniform;
    g->dev.w_beta_uniform = wi.beta_uniform;
    g->dev.w_beta_nonneg = wi.beta_nonneg;
    g->dev.w_beta_one = wi.beta_one;
    g->dev.w_beta_id_mask = wi.beta_id_mask;
    g->dev.w_ucn_iter = wi.ucn_iter_mask;
    g->dev.w_version++;
    return LDPC_OK;
}

int ldpc_ctx_create(ldpc_graph* g, int64_t B_max, int32_t T_max, ldpc_ctx** out) {
    if (!out) return LDPC_ERR_ARG;
    *out = nullptr;
    if (!g || B_max <= 0 || T_max <= 0) return LDPC_ERR_ARG;
    ldpc_ctx* c = new (std::nothrow) ldpc_ctx();
    if (!c) return LDPC_ERR_OOM;
    c->g = g;
    c->B_max = B_max;
    c->T_max = T_max;
    c->ntiles_max = (int)((B_max + TILE - 1) / TILE);
    DeviceGuard dg(g->device);
    const int st = ensure_counters(c);
    if (st != LDPC_OK) { ldpc_ctx_destroy(c); return st; }
    *out = c;
    return LDPC_OK;
}

int ldpc_ctx_destroy(ldpc_ctx* c) {
    if (!c) return LDPC_ERR_ARG;
    DeviceGuard dg(c->g->device);
    dev_free(c->ch); dev_free(c->Tv); dev_free(c->c2v); dev_free(c->hd);
    dev_free(c->wrong); dev_free(c->anypos); dev_free(c->biterr);
    fused_free(c->fused);
    if (c->llr_scratch) (void)hipFree(c->llr_scratch);
    if (c->gen_done) (void)hipEventSynchronize(c->gen_done);
    if (c->gen_tab) (void)hipFree(c->gen_tab);
    if (c->gen_done) (void)hipEventDestroy(c->gen_done);
    delete c;
    return LDPC_OK;
}

static int decode_impl(ldpc_ctx* c, const float* llr_dev, int64_t B, const ldpc_decode_params* p,
                       const ldpc_decode_outputs* o, void* stream, const AwgnParams* gen,
                       const uint32_t* q8 = nullptr, const AwgnParams* gen8 = nullptr);

// LDPC_KERNEL_AUTO takes the fused kernel when it serves the request, except for sum-product:
// its check update is bound by the tanh / atanh / divide VALU work, which flood's four codewords
// per lane amortize better (wman T=20: flood 3.98 M against 3.64 M codewords/s for the fused
// kernel, one box), so the fused SP kernel runs only when asked for
static bool auto_fused(int mode) { return mode != MODE_SP; }

int ldpc_decode(ldpc_ctx* c, const float* llr_dev, int64_t B, const ldpc_decode_params* p,
                const ldpc_decode_outputs* o, void* stream) {
    if (!llr_dev) return LDPC_ERR_ARG;
    return decode_impl(c, llr_dev, B, p, o, stream, nullptr);
}

// ldpc_decode_awgn's byte channel in the bit-sliced kernels' prologue (their Q8 build) serves a
// counters-only decode with these parameters (LDPC_AWGN_Q8=0: never, an A/B and test switch)
static bool q8_serves(const ldpc_ctx* c, const ldpc_decode_params* p, bool has_short) {
    static const bool q8_on = [] { const char* e = getenv("LDPC_AWGN_Q8"); return !(e && atoi(e) == 0); }();
    const ldpc_graph* g = c->g;
    return q8_on && p->decoding_type == LDPC_DEC_QMS && p->kernel != LDPC_KERNEL_FLOOD &&
           fused_q8_ok(g->dev, mode_of(p->decoding_type, p->q_bit), p->T, p->clip_llr,
                       g->d_alpha_ucn != nullptr, g->per_edge_w != 0, has_short);
}

int ldpc_awgn_in_kernel(const ldpc_ctx* c, const ldpc_decode_params* p, int32_t has_short, int32_t app) {
    if (!c || !p) return LDPC_ERR_ARG;
    const ldpc_graph* g = c->g;
    const int mode = mode_of(p->decoding_type, p->q_bit);
    if (mode < 0) return LDPC_ERR_ARG;
    if (!app && q8_serves(c, p, has_short != 0)) return 1;
    // decode_impl with a generator: the fused v5 kernel's prologue, unless the counters-only
    // decode is the bit-sliced kernels' (which read LLRs when Q8 does not serve) or the kernel
    // is flood / ffl (the channel kernel first)
    if (ffl_mode(mode) || !fused_supported(g->dev, mode, p->T, p->clip_llr)) return 0;
    int kern = p->kernel;
    if (kern == LDPC_KERNEL_AUTO) kern = auto_fused(mode) ? LDPC_KERNEL_FUSED : LDPC_KERNEL_FLOOD;
    if (kern != LDPC_KERNEL_FUSED) return 0;
    return fused_awgn_v5(g->dev, mode, p->T, p->clip_llr, g->d_alpha_ucn != nullptr, g->per_edge_w != 0,
                         app != 0) ? 1 : 0;
}

int ldpc_decode_awgn(ldpc_ctx* c, int64_t B, const ldpc_decode_params* p,
                     const ldpc_channel_params* ch, const ldpc_decode_outputs* o, void* stream) {
    if (!c || !p || !ch || !(ch->sigma > 0.0) || ch->offset < 0) return LDPC_ERR_ARG;
    if (B <= 0 || B > c->B_max) return LDPC_ERR_STATE;
    const AwgnParams a = make_awgn(ch->sigma, ch->seed, ch->offset, p->decoding_type, p->q_bit,
                                   ch->punct_start, ch->punct_end, ch->short_start, ch->short_end,
                                   p->clip_llr);
    int st = decode_impl(c, nullptr, B, p, o, stream, &a);
    if (st != LDPC_ERR_UNSUPPORTED) return st;
    ldpc_graph* g = c->g;
    // counters-only QMS decodes the bit-sliced kernels serve: the channel generated in their
    // prologue (SURVEY 8 f rank 1) -- the LLRs never touch HBM (oracle/philox_oracle.awgn_q8); the
    // sampler's tables (8.25 KB) are uploaded when the channel parameters change
    // (counters / flags / iter_wrong only: hard-bit and syndrome exports take the export build,
    // which reads its LLRs)
    if ((!o || (!o->app_all && !o->hard_bits && !o->synd_bits)) && q8_serves(c, p, ch->short_start > 0)) {
        DeviceGuard dg(g->device);
        if (!c->gen_tab) {
            if (hipMalloc(reinterpret_cast<void**>(&c->gen_tab), sizeof(c->gen_host)) != hipSuccess) {
                (void)hipGetLastError();
                return LDPC_ERR_OOM;
            }
            c->gen_valid = false;
        }
        uint32_t tab[AWGN_TAB_W];
        awgn_gen_table(a, tab);
        if (!c->gen_done && hipEventCreateWithFlags(&c->gen_done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            c->gen_done = nullptr;
            return LDPC_ERR_HIP;
        }
        if (!c->gen_valid || std::memcmp(tab, c->gen_host, sizeof(tab)) != 0) {
            // a decode still reading the previous tables may run on another stream: wait for the
            // last one that used them (gen_done) before the copy overwrites them; the stream wait
            // keeps the host copy stable until the transfer has read it
            if (c->gen_pending && hipEventSynchronize(c->gen_done) != hipSuccess) return LDPC_ERR_HIP;
            c->gen_pending = false;
            std::memcpy(c->gen_host, tab, sizeof(tab));
            c->gen_valid = false;
            if (hipMemcpyAsync(c->gen_tab, c->gen_host, sizeof(tab), hipMemcpyHostToDevice,
                               reinterpret_cast<hipStream_t>(stream)) != hipSuccess ||
                hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
                return LDPC_ERR_HIP;
            c->gen_valid = true;
        }
        st = decode_impl(c, nullptr, B, p, o, stream, nullptr, c->gen_tab, &a);
        if (st == LDPC_OK) {
            if (hipEventRecord(c->gen_done, reinterpret_cast<hipStream_t>(stream)) != hipSuccess) return LDPC_ERR_HIP;
            c->gen_pending = true;
        }
        if (st != LDPC_ERR_UNSUPPORTED) return st;
    }
    // this kernel reads its LLRs: generate them into the context's buffer, then decode
    const int64_t n = c->B_max * (int64_t)g->h.N * g->h.z;
    if (c->llr_scratch_n < n) {
        DeviceGuard dg(g->device);
        if (c->llr_scratch) (void)hipFree(c->llr_scratch);
        c->llr_scratch = nullptr;
        c->llr_scratch_n = 0;
        if (hipMalloc(reinterpret_cast<void**>(&c->llr_scratch), (size_t)n * sizeof(float)) != hipSuccess) {
            (void)hipGetLastError();
            return LDPC_ERR_OOM;
        }
        c->llr_scratch_n = n;
    }
    {
        DeviceGuard dg(g->device);
        st = ldpc_channel_awgn(c->llr_scratch, B, g->h.N * g->h.z, ch->sigma, ch->seed, ch->offset,
                               p->decoding_type, p->q_bit, ch->punct_start, ch->punct_end,
                               ch->short_start, ch->short_end, p->clip_llr, stream);
    }
    if (st != LDPC_OK) return st;
    return decode_impl(c, c->llr_scratch, B, p, o, stream, nullptr);
}

int ldpc_kernel_info(const ldpc_ctx* c, const ldpc_decode_params* p, int64_t* bytes_per_cw,
                     char* name, int32_t name_len) {
    if (!c || !p) return LDPC_ERR_ARG;
    const ldpc_graph* g = c->g;
    const int mode = mode_of(p->decoding_type, p->q_bit);
    if (mode < 0) return LDPC_ERR_ARG;
    const bool ucn = g->d_alpha_ucn != nullptr;
    int kern = p->kernel;
    // the float modes' fused kernel (ffl) serves counters-only decodes; it is the one reported
    const bool fl = ffl_mode(mode) && ffl_supported(g->dev, mode, ucn, g->per_edge_w != 0);
    const bool fok = fl || fused_supported(g->dev, mode, p->T, p->clip_llr);
    if (kern == LDPC_KERNEL_AUTO) kern = (fok && auto_fused(mode)) ? LDPC_KERNEL_FUSED : LDPC_KERNEL_FLOOD;
    if (kern == LDPC_KERNEL_FUSED && !fok) return LDPC_ERR_UNSUPPORTED;
    if (kern != LDPC_KERNEL_FLOOD && kern != LDPC_KERNEL_FUSED) return LDPC_ERR_ARG;
    const int64_t nv = (int64_t)g->h.N * g->h.z, ne = (int64_t)g->h.E * g->h.z;
    int64_t bytes = 0;
    const char* nm = "";
    if (kern == LDPC_KERNEL_FLOOD) {
        // per iteration: CN reads Tv (once per variable) and C2V_t (not at t=0), writes
        // C2V_{t+1}; VN reads C2V_{t+1} and ch, writes Tv (not at T-1) and hard bits;
        // UCN adds the hard-bit read.  Plus the prologue transpose (llr in, ch + Tv out).
        for (int t = 0; t < p->T; ++t) {
            bytes += nv * 4 + (t > 0 ? ne * 4 : 0) + ne * 4;
            bytes += ne * 4 + nv * 4 + (t < p->T - 1 ? nv * 4 : 0) + nv / 8 + (ucn ? nv / 8 : 0);
        }
        bytes += nv * 4 * 3;
        nm = "flood";
    } else {
        bytes = fused_bytes_per_cw(g->dev, p->T);
        nm = fl ? ffl_kernel_name(g->dev, mode, ucn, g->per_edge_w != 0)
                : fused_kernel_name(g->dev, mode, p->T, p->clip_llr, ucn, g->per_edge_w != 0);
    }
    if (bytes_per_cw) *bytes_per_cw = bytes;
    if (name && name_len > 0) {
        std::strncpy(name, nm, (size_t)name_len - 1);
        name[name_len - 1] = 0;
    }
    return LDPC_OK;
}

static int decode_impl(ldpc_ctx* c, const float* llr_dev, int64_t B, const ldpc_decode_params* p,
                       const ldpc_decode_outputs* o, void* stream, const AwgnParams* gen,
                       const uint32_t* q8, const AwgnParams* gen8) {
    if (!c || !p || (!llr_dev && !gen && !q8)) return LDPC_ERR_ARG;
    ldpc_graph* g = c->g;
    if (!g->d_alpha || !g->d_beta) return LDPC_ERR_STATE;
    int mode = -1;
    const int chk = host::check_decode(g->h, B, c->B_max, c->T_max, g->T_w, p, &mode);
    if (chk != LDPC_OK) return chk;
    // the caller's outputs struct, never read past the size it declares (ABI 1: five pointers)
    ldpc_decode_outputs out{};
    if (o) {
        if (p->outputs_size == (int32_t)sizeof(ldpc_decode_outputs)) {
            out = *o;
        } else if (p->outputs_size == 0) {
            out.app_all = o->app_all;
            out.hard_bits = o->hard_bits;
            out.synd_bits = o->synd_bits;
            out.counters = o->counters;
            out.frame_flags = o->frame_flags;
        } else {
            return LDPC_ERR_ARG;
        }
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    DeviceGuard dg(g->device);
    const bool ucn = g->d_alpha_ucn != nullptr;

    const bool want_bits = out.hard_bits || out.synd_bits;
    int kern = p->kernel;
    // float modes: the ffl kernel serves counters-only decodes of LLRs in HBM (AUTO takes flood
    // for APP / bit exports; an in-kernel channel is generated first by the caller)
    const bool fl = ffl_mode(mode);
    const bool fok = fl ? (!want_bits && !out.app_all && ffl_supported(g->dev, mode, ucn, g->per_edge_w != 0))
                        : fused_supported(g->dev, mode, p->T, p->clip_llr);
    if (kern == LDPC_KERNEL_AUTO) kern = (fok && auto_fused(mode)) ? LDPC_KERNEL_FUSED : LDPC_KERNEL_FLOOD;
    if (kern != LDPC_KERNEL_FLOOD && kern != LDPC_KERNEL_FUSED) return LDPC_ERR_ARG;
    if (kern == LDPC_KERNEL_FUSED && !fok) return LDPC_ERR_UNSUPPORTED;
    if (gen && (kern != LDPC_KERNEL_FUSED || fl)) return LDPC_ERR_UNSUPPORTED;   // caller falls back
    if (q8 && (kern != LDPC_KERNEL_FUSED || fl)) return LDPC_ERR_UNSUPPORTED;

    const int ntiles = (int)((B + TILE - 1) / TILE);
    const bool count = out.counters || out.frame_flags || out.iter_wrong;
    Bufs b{};
    b.B = B;
    b.ntiles = ntiles;
    b.T = p->T;
    b.n_vars = g->h.N * g->h.z;
    b.target_bits = p->target_bits;
    b.clip = p->clip_llr;
    b.alpha = g->d_alpha;
    b.alpha_ucn = g->d_alpha_ucn;
    b.beta = g->d_beta;
    b.app_out = out.app_all;
    b.count = count ? 1 : 0;
    b.wrong = c->wrong;
    b.anypos = c->anypos;
    b.biterr = c->biterr;
    b.awgn = gen;
    b.iter_wrong = out.iter_wrong;
    b.q8 = q8;
    b.gen8 = gen8;
    if (out.iter_wrong &&
        hipMemsetAsync(out.iter_wrong, 0, (size_t)p->T * ((B + 31) / 32) * sizeof(uint32_t), s) != hipSuccess)
        return LDPC_ERR_HIP;

    if (count && kern == LDPC_KERNEL_FLOOD) {
        if (hipMemsetAsync(c->wrong, 0, (size_t)p->T * ntiles * 4 * sizeof(uint64_t), s) != hipSuccess ||
            hipMemsetAsync(c->anypos, 0, (size_t)ntiles * 4 * sizeof(uint64_t), s) != hipSuccess ||
            hipMemsetAsync(c->biterr, 0, (size_t)ntiles * sizeof(int32_t), s) != hipSuccess)
            return LDPC_ERR_HIP;
    }

    int st;
    if (kern == LDPC_KERNEL_FLOOD) {
        st = ensure_flood(c);
        if (st != LDPC_OK) return st;
        b.ch = c->ch;
        b.Tv = c->Tv;
        b.c2v = c->c2v;
        b.hd = c->hd;
        b.hd_all = want_bits ? 1 : 0;
        b.store_hd = (ucn || want_bits) ? 1 : 0;
        st = flood_decode(g->dev, b, llr_dev, mode, ucn, s);
    } else if (fl) {
        st = ffl_decode(g->dev, b, llr_dev, mode, ucn, g->per_edge_w != 0, out.counters,
                        out.frame_flags, s);
    } else {
        st = fused_decode(g->dev, b, c->fused, llr_dev, mode, ucn, want_bits, c->ntiles_max,
                          c->T_max, g->per_edge_w, out.counters, out.frame_flags, s);
    }
    if (st != LDPC_OK) return st;
    const char* served = kern == LDPC_KERNEL_FLOOD ? "flood"
                         : fl ? ffl_kernel_name(g->dev, mode, ucn, g->per_edge_w != 0)
                              : c->fused.last_kernel;
    // (a channel generated inside the decoding kernel -- the bit-sliced Q8 build or the v5
    // prologue -- is marked "+gen", so a caller can tell it from a decode of LLRs in HBM)
    std::snprintf(c->last_kernel, sizeof(c->last_kernel), "%s%s", served,
                  (q8 || (gen && kern == LDPC_KERNEL_FUSED)) ? "+gen" : "");

    if (count && kern == LDPC_KERNEL_FLOOD) {
        hipLaunchKernelGGL(k_finalize, dim3(std::min(1024, (ntiles + 255) / 256)), dim3(256), 0, s, b,
                           out.counters, out.frame_flags);
        if (out.iter_wrong) {
            const int64_t total = (int64_t)p->T * ((B + 31) / 32);
            hipLaunchKernelGGL(k_iter_wrong, dim3((unsigned)std::min<int64_t>(4096, (total + 255) / 256)),
                               dim3(256), 0, s, b, out.iter_wrong);
        }
    }
    if (want_bits) {
        HdSrc src{};
        src.npk = (B + 31) / 32;
        src.ntiles = ntiles;
        src.n_vars = g->h.N * g->h.z;
        if (kern == LDPC_KERNEL_FUSED) {
            const HdView v = fused_bits_view(c->fused);
            src.tile = v.tile;
            src.pack = v.pack;
            src.bad = v.bad;
        } else {
            src.tile = c->hd;
        }
        if (out.hard_bits) {
            const int nw = (g->h.N * g->h.z + 31) / 32;
            const int64_t total = (int64_t)p->T * B * nw;
            hipLaunchKernelGGL(k_export_hard, dim3((unsigned)std::min<int64_t>(4096, (total + 255) / 256)),
                               dim3(256), 0, s, src, B, out.hard_bits, p->T, nw);
        }
        if (out.synd_bits) {
            const int nw = (g->h.M * g->h.z + 31) / 32;
            const int64_t total = (int64_t)p->T * B * nw;
            hipLaunchKernelGGL(k_export_synd, dim3((unsigned)std::min<int64_t>(4096, (total + 255) / 256)),
                               dim3(256), 0, s, g->dev, src, B, out.synd_bits, p->T, nw);
        }
    }
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

int ldpc_ctx_last_kernel(const ldpc_ctx* c, char* name, int32_t name_len) {
    if (!c || !name || name_len <= 0) return LDPC_ERR_ARG;
    std::strncpy(name, c->last_kernel, (size_t)name_len - 1);
    name[name_len - 1] = 0;
    return LDPC_OK;
}

}  // extern "C"
