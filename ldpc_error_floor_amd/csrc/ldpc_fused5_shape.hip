// ldpc_fused5_shape.hip — one fused v5 shape per translation unit: built once per entry of
// kShapes5 with -DF5_SHAPE=<index> (ldpc_error_floor_amd/build.py), instantiating the kernel
// builds (UCN x per-edge weights x APP export x weight table) of that shape only.
#include "ldpc_fused5_kernel.h"

#ifndef F5_SHAPE
#error "build with -DF5_SHAPE=<index into kShapes5>"
#endif

namespace ldpc {
namespace f5 {

template <int S>
int f5_launch(const F5Args& a, int nblocks, int nw, size_t lds, bool lut, const float* alpha,
              const float* alpha_ucn, bool pew, hipStream_t s) {
    constexpr Shape5 sh = kShapes5[S];
    constexpr int hg = sh.hg > 0 ? sh.hg : sh.maxg;
    constexpr int ldeg = sh.hg > 0 ? sh.ldeg : sh.maxdeg;
    return launch5s<sh.cw, sh.maxg, sh.maxdeg, hg, ldeg, sh.wpe>(a, nblocks, nw, lds, lut, alpha, alpha_ucn,
                                                          pew, s);
}

template int f5_launch<F5_SHAPE>(const F5Args&, int, int, size_t, bool, const float*, const float*,
                                 bool, hipStream_t);

}  // namespace f5
}  // namespace ldpc
