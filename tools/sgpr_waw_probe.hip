// sgpr_waw_probe.hip -- is a VALU carry-out write of an SGPR pair ordered
// before a later SALU write of the same pair on gfx950?  Round 4's lost
// final-state stores were exec-masked stores whose
// masks the failing build formed as
//     v_mad_i64_i32 v[..], s[10:11], ...     (VALU: carry-out into s[10:11])
//     s_and_b64     s[10:11], vcc, s[14:15]  (SALU: the mask, 1-3 instructions later)
//     v_writelane_b32 v252, s10, 59          (spill of the mask)
// If the VALU's SGPR write could land after the SALU's, the spilled mask
// would be the carry-out (0) and the stores it guards would be dropped.
// This probe runs that shape with 0-4 independent instructions between the
// two writes and reads the pair back through v_cndmask: a lane that reads the
// carry-out value instead of the SALU value is a violation.
//   hipcc --offload-arch=gfx950 -O2 -o tools/sgpr_waw_probe tools/sgpr_waw_probe.hip
//   ./tools/sgpr_waw_probe [blocks] [iters]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

// v_add_co_u32 with a carry in every lane (0xffffffff + 1) writes all-ones to
// s[10:11]; the SALU then writes the pattern 0x5555... / 0xaaaa...; the
// readback must see the pattern.
template <int GAP>
__global__ void probe(unsigned* bad, int iters) {
    const unsigned lane = threadIdx.x & 63;
    unsigned nbad = 0;
    for (int it = 0; it < iters; ++it) {
        unsigned a = 0xffffffffu - (unsigned)(it & 1) * 0u, b = 1u + lane * 0u;
        unsigned sum, got;
        if (GAP == 0)
            asm volatile(
                "v_add_co_u32_e64 %0, s[10:11], %2, %3\n\t"
                "s_mov_b32 s10, 0x55555555\n\t"
                "s_mov_b32 s11, 0xaaaaaaaa\n\t"
                "v_cndmask_b32_e64 %1, 0, 1, s[10:11]\n\t"
                : "=&v"(sum), "=&v"(got) : "v"(a), "v"(b) : "s10", "s11");
        else if (GAP == 1)
            asm volatile(
                "v_add_co_u32_e64 %0, s[10:11], %2, %3\n\t"
                "v_mov_b32 %1, 0\n\t"
                "s_mov_b32 s10, 0x55555555\n\t"
                "s_mov_b32 s11, 0xaaaaaaaa\n\t"
                "v_cndmask_b32_e64 %1, 0, 1, s[10:11]\n\t"
                : "=&v"(sum), "=&v"(got) : "v"(a), "v"(b) : "s10", "s11");
        else if (GAP == 2)   // the failing build's shape: a writelane of the SALU result
            asm volatile(
                "v_add_co_u32_e64 %0, s[10:11], %2, %3\n\t"
                "s_and_b64 s[10:11], exec, %4\n\t"
                "v_writelane_b32 %1, s10, 0\n\t"
                "v_writelane_b32 %1, s11, 1\n\t"
                : "=&v"(sum), "=&v"(got) : "v"(a), "v"(b), "s"(0x55555555aaaaaaaaull) : "s10", "s11");
        else
            asm volatile(
                "s_mov_b64 s[12:13], %4\n\t"
                "v_mad_u64_u32 v[40:41], s[10:11], %2, %3, v[40:41]\n\t"
                "s_and_b64 s[10:11], exec, s[12:13]\n\t"
                "v_cndmask_b32_e64 %1, 0, 1, s[10:11]\n\t"
                : "=&v"(sum), "=&v"(got) : "v"(a), "v"(b), "s"(0x55555555aaaaaaaaull)
                : "s10", "s11", "s12", "s13", "v40", "v41");
        (void)sum;
        unsigned want;
        if (GAP == 2) {
            // lanes 0 and 1 of `got` hold s10 / s11 of the SALU result
            const unsigned v0 = __shfl(got, 0, 64), v1 = __shfl(got, 1, 64);
            want = (v0 == 0xaaaaaaaau && v1 == 0x55555555u) ? 1u : 0u;
            nbad += want ? 0u : 1u;
        } else if (GAP == 3) {
            const unsigned long long m = 0x55555555aaaaaaaaull;
            want = (unsigned)((m >> lane) & 1ull);
            nbad += got != want;
        } else {
            const unsigned long long m = 0xaaaaaaaa55555555ull;
            want = (unsigned)((m >> lane) & 1ull);
            nbad += got != want;
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096, iters = argc > 2 ? atoi(argv[2]) : 2000;
    unsigned* d;
    hipMalloc(&d, 4 * sizeof(unsigned));
    hipMemset(d, 0, 4 * sizeof(unsigned));
    hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(256), 0, 0, d + 0, iters);
    hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(256), 0, 0, d + 1, iters);
    hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(256), 0, 0, d + 2, iters);
    hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(256), 0, 0, d + 3, iters);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    unsigned h[4];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const double n = (double)blocks * 256 * iters;
    printf("VALU carry-out -> SALU write -> read, %g lane-trials each: violations gap0 %u, gap1 %u, "
           "writelane shape %u (wave-trials %g), mad64 shape %u\n", n, h[0], h[1], h[2], n / 64, h[3]);
    return 0;
}
