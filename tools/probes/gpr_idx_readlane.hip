// Probe (round 3): with GPR indexing on for VSRC2 and VDST only, is v_readlane_b32's SGPR
// destination or its VGPR source moved by the index?  The global-table phase B
// (kernels.hip) reads each output's jump target with v_readlane while indexing is on.
// Prints s80 and s88 after a readlane of v10 lane 5 with index 8 (v10 = 100 + lane,
// v18 = 200 + lane): expected "s80=105 s88=7".
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *out) {
    unsigned a = 100 + threadIdx.x, b = 200 + threadIdx.x, s80, s88;
    asm volatile(
        "s_mov_b32 s97, m0\n"
        "s_mov_b32 s80, 3\n"
        "s_mov_b32 s88, 7\n"
        "s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)\n"
        "s_set_gpr_idx_idx 8\n"
        "s_nop 1\n"
        "v_readlane_b32 s80, v10, 5\n"
        "s_set_gpr_idx_off\n"
        "s_mov_b32 m0, s97\n"
        "s_nop 4\n"
        "s_mov_b32 %0, s80\n"
        "s_mov_b32 %1, s88\n"
        : "=s"(s80), "=s"(s88), "+{v10}"(a), "+{v18}"(b)
        :
        : "s80", "s97", "s88", "scc");
    if (threadIdx.x == 0) {
        out[0] = s80;
        out[1] = s88;
        out[2] = a + b;
    }
}

int main() {
    unsigned *d, h[3];
    if (hipMalloc(&d, 12) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 12, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("s80=%u s88=%u (v10+v18 lane0 %u)\n", h[0], h[1], h[2]);
    return (h[0] == 105 && h[1] == 7) ? 0 : 1;
}
