// ldpc_fused.h — fused (all iterations in one launch, LDS/register-resident) decoder.
#pragma once
#include "ldpc_internal.h"

namespace ldpc {

struct FusedWorkspace {
    uint64_t* hd = nullptr;        // [T][tiles][n_vars][4] hard decisions (only for bit export)
    int64_t hd_elems = 0;
    void* tables = nullptr;        // per-decode tables shared by all workgroups (v5)
    size_t tables_bytes = 0;
};

bool fused_supported(const DevGraph& g, int mode, int T);
int64_t fused_bytes_per_cw(const DevGraph& g, int T);
int fused_decode(const DevGraph& g, Bufs& b, FusedWorkspace& ws, const float* llr, int mode,
                 bool ucn, bool want_bits, int ntiles_max, int T_max, int per_edge_w,
                 int64_t* counters, uint8_t* flags, hipStream_t s);
void fused_bits_view(const FusedWorkspace& ws, Bufs& b);
const char* fused_kernel_name(const DevGraph& g, int mode, int T, bool per_edge_w);

// v4 (ldpc_fused4.hip): two codewords per lane (packed 16-bit), preferred when it fits
bool fused4_supported(const DevGraph& g, int T, int qmax, bool per_edge_w);
const char* fused4_shape_name(const DevGraph& g, int T);
int fused4_decode(const DevGraph& g, const Bufs& b, const float* llr, int qmax, float step,
                  int clip_u, uint64_t* hd_out, int64_t* counters, uint8_t* flags, hipStream_t s);

// v3 (ldpc_fused3.hip): shape-specialised variant, preferred when a shape fits
bool fused3_supported(const DevGraph& g, int T);
const char* fused3_shape_name(const DevGraph& g, int T);
int fused3_decode(const DevGraph& g, const Bufs& b, const float* llr, int qmax, float step,
                  int clip_u, bool per_edge_w, uint64_t* hd_out, int64_t* counters,
                  uint8_t* flags, hipStream_t s);
// v5 (ldpc_fused5.hip): byte-packed check state, default when a shape fits
bool fused5_supported(const DevGraph& g, int T);
const char* fused5_shape_name(const DevGraph& g, int T);
int fused5_decode(const DevGraph& g, const Bufs& b, FusedWorkspace& ws, const float* llr,
                  int qmax, float step, int clip_u, bool per_edge_w, uint64_t* hd_out,
                  int64_t* counters, uint8_t* flags, hipStream_t s);
void fused_free(FusedWorkspace& ws);

}  // namespace ldpc
