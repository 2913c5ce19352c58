// ldpc_collect.hip — on-device collection of uncorrected frames (SURVEY §8 f rank 2).
//
// The reference appends every frame that is wrong at every iteration (calc_ber_fer's
// uncor_flag, Print_Functions.py:100-118) to Uncor.txt as 3 zero columns + the negated LLRs
// (write_uncor_file, Print_Functions.py:120-126).  On the GPU sweep the LLRs never leave the
// device, so the failing frames are compacted here: one ballot per wave, one atomic per wave,
// indices in wave order within a wave (the host sorts the few of them), then a row gather.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "ldpc_nms.h"

namespace ldpc {

__global__ void k_collect(const uint8_t* __restrict__ flags, int64_t B, uint32_t mask,
                          uint32_t want, int64_t* __restrict__ idx, int64_t cap,
                          unsigned long long* __restrict__ count) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool hit = b < B && ((uint32_t)flags[b] & mask) == want;
    const unsigned long long bal = __ballot(hit);
    if (bal == 0) return;
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (lane == __ffsll((long long)bal) - 1) base = atomicAdd(count, (unsigned long long)__popcll(bal));
    base = __shfl(base, __ffsll((long long)bal) - 1);
    if (hit) {
        const unsigned long long r = base + __popcll(bal & ((1ull << lane) - 1));
        if ((int64_t)r < cap) idx[r] = b;
    }
}

__global__ void k_gather_rows(const float* __restrict__ src, int64_t n_cols,
                              const int64_t* __restrict__ idx, int64_t n, float* __restrict__ dst) {
    const int64_t r = blockIdx.y;
    if (r >= n) return;
    const float* s = src + idx[r] * n_cols;
    float* d = dst + r * n_cols;
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n_cols;
         c += (int64_t)gridDim.x * blockDim.x)
        d[c] = s[c];
}

}  // namespace ldpc

extern "C" int ldpc_collect_frames(const uint8_t* flags_dev, int64_t B, uint32_t mask,
                                   uint32_t want, int64_t* idx_dev, int64_t cap,
                                   int64_t* count_dev, void* stream) {
    if (!flags_dev || !count_dev || B < 0 || cap < 0 || (cap > 0 && !idx_dev)) return LDPC_ERR_ARG;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (hipMemsetAsync(count_dev, 0, sizeof(int64_t), s) != hipSuccess) return LDPC_ERR_HIP;
    if (B == 0) return LDPC_OK;
    const unsigned grid = (unsigned)((B + 255) / 256);
    hipLaunchKernelGGL(ldpc::k_collect, dim3(grid), dim3(256), 0, s, flags_dev, B, mask, want,
                       idx_dev, cap, reinterpret_cast<unsigned long long*>(count_dev));
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}

// One value of write_uncor_file's row text: "%.1f" of v (Python's rendering, which is what
// np.savetxt calls: nan without a sign).  v = -(double)x for a float32 x, so v * 10 is exact
// in a double (24-bit significand x 10) and rounding it to an integer half to even (adding
// and taking away 2^52 + 2^51 in the default rounding mode, exact below 2^51) gives the
// correctly rounded tenths "%.1f" prints.  From 1e14 on (and for inf) the C library's
// correctly rounded "%.1f" is used instead.
constexpr uint64_t kTenthsLut = 10000;
struct TenthsLut {
    char s[kTenthsLut][8];
    uint8_t len[kTenthsLut];
    TenthsLut() {
        for (uint64_t a = 0; a < kTenthsLut; ++a)
            len[a] = (uint8_t)std::snprintf(s[a], 8, "%llu.%llu", (unsigned long long)(a / 10),
                                            (unsigned long long)(a % 10));
    }
};
static const TenthsLut& tenths_lut() {
    static const TenthsLut lut;
    return lut;
}

static inline char* put_tenths(char* p, double v) {
    const double av = std::fabs(v);
    if (!(av < 1e14)) {
        if (std::isnan(v)) {
            std::memcpy(p, "nan", 3);
            return p + 3;
        }
        return p + std::snprintf(p, 48, "%.1f", v);
    }
    const double m = 6755399441055744.0;               // 2^52 + 2^51 (no -ffast-math here)
    const double t = (av * 10.0 + m) - m;
    if (std::signbit(v)) *p++ = '-';
    uint64_t a = (uint64_t)t;
    if (a < kTenthsLut) {                              // |v| < 1000: "ddd.d" from the table
        std::memcpy(p, tenths_lut().s[a], 8);
        return p + tenths_lut().len[a];
    }
    const char frac = (char)('0' + a % 10);
    a /= 10;
    char d[20];
    int k = 0;
    do {
        d[k++] = (char)('0' + a % 10);
        a /= 10;
    } while (a);
    while (k) *p++ = d[--k];
    *p++ = '.';
    *p++ = frac;
    return p;
}

extern "C" int ldpc_format_uncor_rows(const float* rows, int64_t n, int64_t n_cols, char* out,
                                      int64_t cap, int64_t* len) {
    if (!len || n < 0 || n_cols <= 0 || (n > 0 && (!rows || !out))) return LDPC_ERR_ARG;
    *len = 0;
    if (cap < n * LDPC_UNCOR_ROW_BOUND(n_cols)) return LDPC_ERR_ARG;
    char* p = out;
    const TenthsLut& lut = tenths_lut();
    (void)lut;
    for (int64_t r = 0; r < n; ++r) {
        std::memcpy(p, "0.0\t0.0\t0.0\t", 12);
        p += 12;
        const float* x = rows + r * n_cols;
        for (int64_t c = 0; c < n_cols; ++c) {
            p = put_tenths(p, -(double)x[c]);
            *p++ = c + 1 < n_cols ? '\t' : '\n';
        }
    }
    *len = (int64_t)(p - out);
    return LDPC_OK;
}

extern "C" int ldpc_gather_rows(const float* src_dev, int64_t n_cols, const int64_t* idx_dev,
                                int64_t n, float* dst_dev, void* stream) {
    if (n < 0 || n_cols <= 0 || (n > 0 && (!src_dev || !idx_dev || !dst_dev))) return LDPC_ERR_ARG;
    if (n == 0) return LDPC_OK;
    if (n > 65535) return LDPC_ERR_ARG;                       // grid.y limit; call in slices
    const unsigned gx = (unsigned)std::min<int64_t>(64, (n_cols + 255) / 256);
    hipLaunchKernelGGL(ldpc::k_gather_rows, dim3(gx, (unsigned)n), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), src_dev, n_cols, idx_dev, n, dst_dev);
    return hipGetLastError() == hipSuccess ? LDPC_OK : LDPC_ERR_HIP;
}
