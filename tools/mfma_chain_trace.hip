// mfma_chain_trace.hip -- the split-bf16 chain of ONE output on the bf16
// MFMA, with the accumulator dumped after every MFMA, for pinning a model
// mismatch to its step.  Input file: int32 n, then the
// x parts and the alpha parts as uint16 [3][n] each, k in the order the
// hardware consumes them (per 16-deep block: lane half 0's 8 values, then
// lane half 1's).  Output: float32 [n/16 * 6] accumulators.
//   hipcc --offload-arch=gfx950 -O2 -o tools/mfma_chain_trace tools/mfma_chain_trace.hip
//   ./tools/mfma_chain_trace in.bin out.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void chain(const uint16_t* xp, const uint16_t* ap, float* out, int n) {
    const int l = threadIdx.x;
    const int pi[6] = {0, 0, 1, 0, 1, 2}, pj[6] = {0, 1, 0, 2, 1, 0};
    f32x16 acc;
    for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
    for (int b = 0; b < n / 16; ++b)
        for (int q = 0; q < 6; ++q) {
            bf16x8 a, c;
            for (int i = 0; i < 8; ++i) {
                const int k = 16 * b + 8 * (l / 32) + i;
                const uint16_t xv = (l % 32 == 0) ? xp[pi[q] * n + k] : 0;
                const uint16_t yv = (l % 32 == 0) ? ap[pj[q] * n + k] : 0;
                a[i] = __builtin_bit_cast(__bf16, xv);
                c[i] = __builtin_bit_cast(__bf16, yv);
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, c, acc, 0, 0, 0);
            if (l == 0) out[b * 6 + q] = acc[0];
        }
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    int n = 0;
    if (fread(&n, 4, 1, f) != 1 || n <= 0 || n % 16 || n > (1 << 20)) return 1;
    uint16_t* h = (uint16_t*)malloc((size_t)6 * n * 2);
    if (fread(h, 2, (size_t)6 * n, f) != (size_t)6 * n) return 1;
    fclose(f);
    uint16_t* d;
    float* o;
    hipMalloc(&d, (size_t)6 * n * 2);
    hipMalloc(&o, (size_t)n / 16 * 6 * 4);
    hipMemcpy(d, h, (size_t)6 * n * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, d, d + 3 * n, o, n);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float* ho = (float*)malloc((size_t)n / 16 * 6 * 4);
    hipMemcpy(ho, o, (size_t)n / 16 * 6 * 4, hipMemcpyDeviceToHost);
    FILE* g = fopen(argv[2], "wb");
    if (!g) return 1;
    fwrite(ho, 4, (size_t)n / 16 * 6, g);
    fclose(g);
    printf("ok %d\n", n);
    return 0;
}
