// v_sad_u16 semantics probe: gfx950 sums |a - b| over BOTH 16-bit halves, plus c
// (expected last two: 0x105 and 0x1_0204 = 0x200 + 0xFFFF + 5)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* a, const unsigned* b, unsigned* o, int n) {
    int i = threadIdx.x;
    if (i < n) o[i] = __builtin_amdgcn_sad_u16(a[i], b[i], 5u);
}
int main() {
    const int n = 8;
    unsigned ha[n] = {0x0100u, 0xFF00u, 0x8100u, 0x7F00u, 0x8000u, 0xFFFF8100u, 0xFFFF8100u, 0x00007E00u};
    unsigned hb[n] = {0x8000u, 0x8000u, 0x8000u, 0x8000u, 0x0000u, 0x0000u, 0xFFFF8000u, 0xFFFF8000u};
    unsigned *da, *db, *dout, ho[n];
    hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dout, sizeof ho);
    hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
    k<<<1, 64>>>(da, db, dout, n);
    hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i) printf("sad_u16(%08x, %08x, 5) = %08x\n", ha[i], hb[i], ho[i]);
    return 0;
}
