// ldpc_bs_inst.hip — one bit-sliced kernel instance per translation unit: built once per entry
// of kBsInst with -DBS_INST=i (ldpc_error_floor_amd/build.py), so the instances compile in
// parallel.
#include "ldpc_bs_kernel.h"

#ifndef BS_INST
#error "build with -DBS_INST=<index into kBsInst>"
#endif

namespace ldpc {
namespace bs {

template <>
int bs_launch<BS_INST>(const BsArgs& a, int nblocks, int nw, size_t lds, hipStream_t s, bool q8) {
    return launch_bs<BS_INST>(a, nblocks, nw, lds, s, q8);
}

}  // namespace bs
}  // namespace ldpc
