// mfma_case_probe.hip -- v_mfma_f32_32x32x16_bf16 on given cases: for each
// (x[16], y[16], c) the output D[0][0] (A row 0 = x, B column 0 = y, C[0][0]
// = c; k = 8*(lane/32) + i), for targeted probes of the accumulation model
// (DESIGN.md section 9).  Input: int32 n, uint16 x[n][16], uint16 y[n][16],
// float c[n].  Output: float d[n].
//   hipcc --offload-arch=gfx950 -O2 -o tools/mfma_case_probe tools/mfma_case_probe.hip
//   ./tools/mfma_case_probe in.bin out.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(const uint16_t* x, const uint16_t* y, const float* c, float* out, int n) {
    const int l = threadIdx.x;
    for (int t = blockIdx.x; t < n; t += gridDim.x) {
        bf16x8 a, b;
        for (int i = 0; i < 8; ++i) {
            const int k = 8 * (l / 32) + i;
            a[i] = __builtin_bit_cast(__bf16, (uint16_t)(l % 32 == 0 ? x[t * 16 + k] : 0));
            b[i] = __builtin_bit_cast(__bf16, (uint16_t)(l % 32 == 0 ? y[t * 16 + k] : 0));
        }
        f32x16 acc;
        for (int j = 0; j < 16; ++j) acc[j] = 0.0f;
        if (l == 0) acc[0] = c[t];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        if (l == 0) out[t] = acc[0];
    }
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 1;
    int n = 0;
    if (fread(&n, 4, 1, f) != 1 || n <= 0 || n > (1 << 22)) return 1;
    uint16_t* h = (uint16_t*)malloc((size_t)n * 64);
    float* c = (float*)malloc((size_t)n * 4);
    if (fread(h, 2, (size_t)n * 32, f) != (size_t)n * 32 || fread(c, 4, (size_t)n, f) != (size_t)n) return 1;
    fclose(f);
    uint16_t* d;
    float *dc, *dout;
    hipMalloc(&d, (size_t)n * 64);
    hipMalloc(&dc, (size_t)n * 4);
    hipMalloc(&dout, (size_t)n * 4);
    hipMemcpy(d, h, (size_t)n * 64, hipMemcpyHostToDevice);
    hipMemcpy(dc, c, (size_t)n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1024), dim3(64), 0, 0, d, d + (size_t)n * 16, dc, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    float* o = (float*)malloc((size_t)n * 4);
    hipMemcpy(o, dout, (size_t)n * 4, hipMemcpyDeviceToHost);
    FILE* g = fopen(argv[2], "wb");
    if (!g) return 1;
    fwrite(o, 4, (size_t)n, g);
    fclose(g);
    printf("ok %d\n", n);
    return 0;
}
