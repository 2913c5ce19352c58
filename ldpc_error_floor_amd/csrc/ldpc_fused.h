// ldpc_fused.h — fused (all iterations in one launch, LDS/register-resident) decoder.
#pragma once
#include <string>

#include "ldpc_internal.h"

namespace ldpc {

struct FusedWorkspace {
    uint64_t* hd = nullptr;        // [T][tiles][n_vars][4] hard decisions (only for bit export)
    int64_t hd_elems = 0;
    void* tables = nullptr;        // per-decode tables shared by all workgroups (v5)
    size_t tables_bytes = 0;
    void* bs_graph = nullptr;      // bit-sliced kernel: graph tables (built once per context)
    int bs_graph_inst = -1;        // the kernel instance they were built for
    void* bs_lut = nullptr;        // bit-sliced kernel: per-decode weight tables
    size_t bs_lut_bytes = 0;
    uint32_t* bs_bad = nullptr;    // [packs] 1: pack decoded by the v5 fixup
    int64_t bs_bad_n = 0;
    uint32_t* hdx = nullptr;       // [T][packs][n_vars] bit-sliced hard decisions (bit export of
    int64_t hdx_elems = 0;         // the bit-sliced kernels; fixup packs are in `hd` instead)
    bool bits_packed = false;      // the last bit-exporting decode wrote hdx (+ hd for bad packs)
    const char* last_kernel = "";  // the kernel that served the last decode (ldpc_ctx_last_kernel)
    // what the per-decode table kernels last wrote (they depend only on the graph, the weights
    // and T): a decode with the same key skips them
    uint64_t key_gad[4] = {~0ull, 0, 0, 0}, key_qtab[4] = {~0ull, 0, 0, 0}, key_bslut[4] = {~0ull, 0, 0, 0};
};

// fused v5 serves this request (QMS q in {5,-5,4,3}, clip_llr on the grid, a shape fits)
bool fused_supported(const DevGraph& g, int mode, int T, float clip_llr);
int64_t fused_bytes_per_cw(const DevGraph& g, int T);
int fused_decode(const DevGraph& g, Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
                 bool ucn, bool want_bits, int ntiles_max, int T_max, int per_edge_w,
                 int64_t* counters, uint8_t* flags, hipStream_t s);
// where the last bit-exporting fused decode left its hard decisions (ldpc_capi.hip's HdSrc)
struct HdView {
    const uint64_t* tile;      // [T+1][tiles][n_vars][4] (Bufs::hd layout, slot t + 1), or null
    const uint32_t* pack;      // [T][packs][n_vars] bit-sliced, or null
    const uint32_t* bad;       // [packs] 1: this pack's bits are in `tile` (v5 fixup)
};
HdView fused_bits_view(const FusedWorkspace& ws);
const char* fused_kernel_name(const DevGraph& g, int mode, int T, float clip_llr, bool ucn,
                              bool per_edge_w);

// v5 (ldpc_fused5.hip): byte-packed check state, default when a shape fits
bool fused5_supported(const DevGraph& g, int T);
const char* fused5_shape_name(const DevGraph& g, int T);
// only: null, or per-32-codeword pack flags: decode just the blocks of flagged packs (the
// bit-sliced kernel's fixup; needs a shape with CW <= 32, fused5_cw)
int fused5_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr,
                  int qmax, float step, int clip_u, bool per_edge_w, uint64_t* hd_out,
                  int64_t* counters, uint8_t* flags, hipStream_t s, const uint32_t* only = nullptr);
int fused5_cw(const DevGraph& g, int T);

// bit-sliced (ldpc_bs.hip): 32 codewords per word, counters / flags only, QMS q = 5 / -5
// (clip: clip_LLR, the LLR of shortened bits)
// (T: the iteration count, whose per-iteration frame words take 4 T bytes of LDS)
bool bs_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T);
const char* bs_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T);
// hdx: null, or [T][packs][n_vars] u32: also store every iteration's hard decisions (bit r of
// word (t, pack, v) = codeword 32 pack + r; the export build of the kernel)
int bs_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
              bool ucn, int64_t* counters, uint8_t* flags, uint32_t* bad, uint32_t* hdx, hipStream_t s);
// the in-prologue channel (Bufs::q8 / gen8) serves this counters-only decode: the bit-sliced
// kernel applies, has room for the sampler's tables in its slot region and, with shortened bits
// in the channel, has the shortened-bit marker (a BIG instance)
bool bs_q8_ok(const DevGraph& g, int mode, bool ucn, float clip, int T, bool has_short);
bool bsc_q8_ok(const DevGraph& g, int mode, bool ucn, float clip, int T, bool has_short);
// host-side bounds check of the bsc plan (test infrastructure, ldpc_debug_bs_bounds)
int bsc_debug_bounds(const DevGraph& g, int mode, float clip, int T, int& violations, std::string& first);
// (fused_decode with it: the bit-sliced kernel or LDPC_ERR_UNSUPPORTED)
bool fused_q8_ok(const DevGraph& g, int mode, int T, float clip, bool ucn, bool per_edge_w, bool has_short);
// a decode with an in-kernel generator (Bufs::awgn) runs the v5 kernel's prologue channel
bool fused_awgn_v5(const DevGraph& g, int mode, int T, float clip, bool ucn, bool per_edge_w, bool app);
// compressed bit-sliced kernel (ldpc_bsc.hip): the graphs whose per-edge slots exceed the LDS
bool bsc_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T);
const char* bsc_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w, float clip, int T);
int bsc_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
               bool ucn, int64_t* counters, uint8_t* flags, uint32_t* bad, uint32_t* hdx, hipStream_t s);
void fused_free(FusedWorkspace& ws);

// float-mode fused decoder (ldpc_ffl.hip): MS, MS without nudge, QMS q = 6, sum-product; counters / flags
// only, row-uniform CN weights
bool ffl_mode(int mode);
bool ffl_supported(const DevGraph& g, int mode, bool ucn, bool per_edge_w);
const char* ffl_kernel_name(const DevGraph& g, int mode, bool ucn, bool per_edge_w);
int ffl_decode(const DevGraph& g, const Bufs& b, const float* llr, int mode, bool ucn, bool per_edge_w,
               int64_t* counters, uint8_t* flags, hipStream_t s);

}  // namespace ldpc
