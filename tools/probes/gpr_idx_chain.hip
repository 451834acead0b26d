// Probe (round 3): with GPR indexing on for VSRC0 and VDST, (1) v_readlane_b32's VGPR source
// follows the index, (2) `s_add_u32 m0, m0, 9` moves the index by 9 while indexing stays on.
// The chained phase B (kernels.hip lh_inverse_ch_kernel) relies on both.  v10 / v19 / v28 =
// 100 / 200 / 300 + lane; reads lane 5 at index 0, 9, 18: expected "105 205 305".
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(unsigned *out) {
    unsigned a = 100 + threadIdx.x, b = 200 + threadIdx.x, c = 300 + threadIdx.x, r0, r1, r2;
    asm volatile(
        "s_mov_b32 s97, m0\n"
        "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n"
        "s_nop 1\n"
        "v_readlane_b32 s80, v10, 5\n"
        "s_add_u32 m0, m0, 9\n"
        "s_nop 1\n"
        "v_readlane_b32 s81, v10, 5\n"
        "s_add_u32 m0, m0, 9\n"
        "s_nop 1\n"
        "v_readlane_b32 s82, v10, 5\n"
        "s_set_gpr_idx_off\n"
        "s_mov_b32 m0, s97\n"
        "s_nop 4\n"
        "s_mov_b32 %0, s80\n"
        "s_mov_b32 %1, s81\n"
        "s_mov_b32 %2, s82\n"
        : "=s"(r0), "=s"(r1), "=s"(r2), "+{v10}"(a), "+{v19}"(b), "+{v28}"(c)
        :
        : "s80", "s81", "s82", "s97", "scc");
    if (threadIdx.x == 0) {
        out[0] = r0;
        out[1] = r1;
        out[2] = r2;
    }
}

int main() {
    unsigned *d, h[3];
    if (hipMalloc(&d, 12) != hipSuccess) return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 12, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    printf("%u %u %u\n", h[0], h[1], h[2]);
    return (h[0] == 105 && h[1] == 205 && h[2] == 305) ? 0 : 1;
}
