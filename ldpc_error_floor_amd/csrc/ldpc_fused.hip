// ldpc_fused.hip — dispatch of the fused decoder (all T flooding iterations in ONE launch).
//
// Same algorithm as ldpc_flood.hip / oracle/nms_oracle.py (Main_Functions.py:157-385), but a
// workgroup owns CW codewords for the whole decode, so nothing but the input LLRs and the
// final counters touches HBM.  The kernel is v5 (ldpc_fused5_kernel.h, planning and tables in
// ldpc_fused5.hip).  It serves the integer QMS modes (q in {5, -5, 4, 3}) of every graph that
// plan5 can map to a shape; everything else (q = 6, the float modes, graphs no shape fits, a
// clip_LLR off the quantizer grid) is the flood kernel's, which the AUTO selection falls back
// to.  There are no other fused variants: only kernels with parity tests can be selected.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "ldpc_fused.h"

namespace ldpc {

namespace {

float mode_step(int mode) {
    switch (mode) {
        case MODE_Q5: return 0.5f;
        case MODE_QM5: case MODE_Q4: return 1.0f;
        case MODE_Q3: return 2.0f;
        default: return 0.f;
    }
}

int mode_qmax(int mode) { return (mode == MODE_Q4) ? 7 : (mode == MODE_Q3) ? 3 : 15; }

// clip_LLR in grid units: the APP clip (Main_Functions.py:322-325) is a clamp in the kernel's
// integer domain only when clip / step is an integer; 0 when it is not representable
int clip_units(int mode, float clip) {
    const float step = mode_step(mode);
    if (!(step > 0.f) || !(clip > 0.f)) return 0;
    const float cu = clip / step;
    if (cu != rintf(cu) || cu > 32000.f) return 0;
    return (int)cu;
}

}  // namespace

bool fused_supported(const DevGraph& g, int mode, int T, float clip_llr) {
    if (mode != MODE_Q5 && mode != MODE_QM5 && mode != MODE_Q4 && mode != MODE_Q3) return false;
    if (g.n_vars >= 32768) return false;
    if (clip_units(mode, clip_llr) == 0) return false;
    return fused5_supported(g, T);
}

// counters-only decodes (throughput mode) run the bit-sliced kernel when it applies
static bool use_bs(const DevGraph& g, int mode, int T, bool ucn, bool per_edge_w, float clip) {
    const int cw = fused5_cw(g, T);
    return cw > 0 && cw <= 32 && bs_supported(g, mode, ucn, per_edge_w, clip, T);
}

// the kernel a counters-only decode runs (the throughput / roofline report)
const char* fused_kernel_name(const DevGraph& g, int mode, int T, float clip_llr, bool ucn,
                              bool per_edge_w) {
    if (!fused_supported(g, mode, T, clip_llr)) return "";
    if (use_bs(g, mode, T, ucn, per_edge_w, clip_llr)) return bs_kernel_name(g, mode, ucn, per_edge_w, clip_llr, T);
    return fused5_shape_name(g, T);
}

bool fused_q8_ok(const DevGraph& g, int mode, int T, float clip, bool ucn, bool per_edge_w, bool has_short) {
    return fused_supported(g, mode, T, clip) && use_bs(g, mode, T, ucn, per_edge_w, clip) &&
           bs_q8_ok(g, mode, ucn, clip, T, has_short);
}

bool fused_awgn_v5(const DevGraph& g, int mode, int T, float clip, bool ucn, bool per_edge_w, bool app) {
    // fused_decode with a generator: the v5 prologue, except counters-only decodes the
    // bit-sliced kernels serve (UNSUPPORTED there: ldpc_decode_awgn then generates into HBM)
    return fused_supported(g, mode, T, clip) && (app || !use_bs(g, mode, T, ucn, per_edge_w, clip));
}

int64_t fused_bytes_per_cw(const DevGraph& g, int T) {
    (void)T;
    // compulsory: the channel LLRs are read once; outputs are counters only
    return (int64_t)g.n_vars * 4;
}

int fused_decode(const DevGraph& g, Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
                 bool ucn, bool want_bits, int ntiles_max, int T_max, int per_edge_w,
                 int64_t* counters, uint8_t* flags, hipStream_t s) {
    if (!fused_supported(g, mode, b.T, b.clip)) return LDPC_ERR_UNSUPPORTED;
    // counters-only decodes the bit-sliced kernel serves read their LLRs: with an in-kernel
    // channel requested, the caller (ldpc_decode_awgn) generates them into HBM first — the
    // channel kernel plus the bit-sliced decode beat the v5 kernel's in-prologue channel
    if (b.awgn && !b.app_out && use_bs(g, mode, b.T, ucn, per_edge_w != 0, b.clip))
        return LDPC_ERR_UNSUPPORTED;
    const float step = mode_step(mode);
    const int cu = clip_units(mode, b.clip);
    uint64_t* hd_out = nullptr;
    // counters / frame flags / bit exports without APP: the bit-sliced kernel when it applies
    // (its export build stores every iteration's hard decisions, bit-sliced, in ws.hdx)
    const bool bs = !b.app_out && !b.awgn && use_bs(g, mode, b.T, ucn, per_edge_w != 0, b.clip);
    if (b.q8 && !bs) return LDPC_ERR_UNSUPPORTED;          // the in-prologue channel is the bit-sliced kernels'

    ws.bits_packed = false;
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
        // the v5 export ORs its bits into a zeroed buffer; a bit-sliced decode reads the tile
        // buffer only for the packs its v5 fixup decodes, and the fixup clears those blocks'
        // bits itself (f5_block), so the (T + 1) x tiles x n_vars x 32 B memset is skipped
        if (!bs &&
            hipMemsetAsync(ws.hd, 0, (size_t)(b.T + 1) * b.ntiles * g.n_vars * 4 * sizeof(uint64_t), s) != hipSuccess)
            return LDPC_ERR_HIP;
        hd_out = ws.hd;
    }
    if (bs) {
        // bit-sliced kernel; packs whose LLRs are off the quantizer grid go to the v5 kernel
        const int64_t npk = (b.B + 31) / 32;
        uint32_t* hdx = nullptr;
        if (want_bits) {
            const int64_t n = (int64_t)b.T * npk * g.n_vars;
            if (n > ws.hdx_elems) {
                if (ws.hdx) (void)hipFree(ws.hdx);
                ws.hdx = nullptr;
                ws.hdx_elems = 0;
                if (hipMalloc(reinterpret_cast<void**>(&ws.hdx), (size_t)n * 4) != hipSuccess) {
                    (void)hipGetLastError();
                    return LDPC_ERR_OOM;
                }
                ws.hdx_elems = n;
            }
            hdx = ws.hdx;
        }
        if (npk > ws.bs_bad_n) {
            if (ws.bs_bad) (void)hipFree(ws.bs_bad);
            ws.bs_bad = nullptr;
            ws.bs_bad_n = 0;
            const int64_t n = std::max<int64_t>(npk, (int64_t)(ntiles_max) * 8);
            if (hipMalloc(reinterpret_cast<void**>(&ws.bs_bad), (size_t)n * 4) != hipSuccess) {
                (void)hipGetLastError();
                return LDPC_ERR_OOM;
            }
            ws.bs_bad_n = n;
        }
        int st = bs_decode(g, b, ws, llr, mode, ucn, counters, flags, ws.bs_bad, hdx, s);
        if (st != LDPC_OK) return st;
        ws.last_kernel = fused_kernel_name(g, mode, b.T, b.clip, ucn, per_edge_w != 0);
        ws.bits_packed = want_bits;
        if (b.q8) return LDPC_OK;      // generated channel: every pack is on the grid, nothing to fix up
        // test hook: LDPC_BS_FIXUP=0 skips the v5 fixup, so a test can tell that a batch was
        // decoded by the bit-sliced kernel alone (flagged packs then contribute nothing).  Read
        // per decode (a test sets it after other decodes ran in the same process).
        const char* fx = getenv("LDPC_BS_FIXUP");
        if (fx && atoi(fx) == 0) return LDPC_OK;
        return fused5_decode(g, b, ws, llr, mode_qmax(mode), step, cu, per_edge_w != 0, hd_out,
                             counters, flags, s, ws.bs_bad);
    }
    ws.last_kernel = fused5_shape_name(g, b.T);
    return fused5_decode(g, b, ws, llr, mode_qmax(mode), step, cu, per_edge_w != 0, hd_out,
                         counters, flags, s);
}

HdView fused_bits_view(const FusedWorkspace& ws) {
    HdView v{};
    v.tile = ws.hd;
    if (ws.bits_packed) {
        v.pack = ws.hdx;
        v.bad = ws.bs_bad;
    }
    return v;
}

void fused_free(FusedWorkspace& ws) {
    if (ws.hd) (void)hipFree(ws.hd);
    ws.hd = nullptr;
    ws.hd_elems = 0;
    if (ws.tables) (void)hipFree(ws.tables);
    ws.tables = nullptr;
    ws.tables_bytes = 0;
    if (ws.bs_graph) (void)hipFree(ws.bs_graph);
    ws.bs_graph = nullptr;
    if (ws.bs_lut) (void)hipFree(ws.bs_lut);
    ws.bs_lut = nullptr;
    ws.bs_lut_bytes = 0;
    if (ws.bs_bad) (void)hipFree(ws.bs_bad);
    ws.bs_bad = nullptr;
    ws.bs_bad_n = 0;
    if (ws.hdx) (void)hipFree(ws.hdx);
    ws.hdx = nullptr;
    ws.hdx_elems = 0;
    ws.bits_packed = false;
    ws.key_gad[0] = ws.key_qtab[0] = ws.key_bslut[0] = ~0ull;
}

}  // namespace ldpc
