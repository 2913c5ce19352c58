// ldpc_quant.h — the reference's message quantizers on the device (flood and ffl kernels).
#pragma once
#include "ldpc_internal.h"

namespace ldpc {

// quantizers (Main_Functions.py:475-494 forward values; Print_Functions.py:12-25)
template <int MODE>
__device__ __forceinline__ float qmsg(float x, float clip) {
    if constexpr (MODE == MODE_Q6) return fminf(fmaxf(rintf(x), -15.5f), 15.5f);
    else if constexpr (MODE == MODE_Q5) return fminf(fmaxf(rintf(x * 2.0f) * 0.5f, -7.5f), 7.5f);
    else if constexpr (MODE == MODE_QM5) return fminf(fmaxf(rintf(x), -15.0f), 15.0f);
    else if constexpr (MODE == MODE_Q4) return fminf(fmaxf(rintf(x), -7.0f), 7.0f);
    else if constexpr (MODE == MODE_Q3) return fminf(fmaxf(rintf(x * 0.5f) * 2.0f, -6.0f), 6.0f);
    else return fminf(fmaxf(x, -clip), clip);            // MS: clip_by_value(+-clip_LLR)
}
template <int MODE>
__device__ __forceinline__ float qchan(float x) {       // Q on the channel (QMS only)
    if constexpr (mode_is_qms(MODE)) return qmsg<MODE>(x, 0.f);
    else return x;
}

}  // namespace ldpc
