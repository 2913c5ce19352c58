// ldpc_fused.hip — placeholder until the fused kernel lands.
#include "ldpc_fused.h"

namespace ldpc {
bool fused_supported(const DevGraph&, int, int) { return false; }
int64_t fused_bytes_per_cw(const DevGraph&, int) { return 0; }
int fused_decode(const DevGraph&, Bufs&, FusedWorkspace&, const float*, int, bool, bool, int, int,
                 hipStream_t) { return LDPC_ERR_UNSUPPORTED; }
void fused_bits_view(const FusedWorkspace& ws, Bufs& b) { b.hd = ws.hd; b.hd_all = 1; }
void fused_free(FusedWorkspace& ws) { if (ws.hd) (void)hipFree(ws.hd); ws.hd = nullptr; }
}  // namespace ldpc
