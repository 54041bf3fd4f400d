// Compiler probe: does LLVM keep raw buffer stores/loads
// (address space 8 resource) ordered against global (address space 1)
// accesses of the same memory?  Build the ISA and read it:
//   hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -o aa.s tools/aa_probe.hip
// Result (ROCm 7.2, gfx950): t1 reloads the global value after the buffer
// store (no store-to-load forwarding of 1.0), t2 issues the buffer load after
// both stores, t3 keeps store -> load -> store in program order.  The compiler
// treats the two address spaces as may-alias, so mixing the store forms
// cannot reorder record traffic.
#include <hip/hip_runtime.h>
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) float gfloat;
// T1: global store, buffer store to the same address, global load -> forwarded?
extern "C" __global__ void t1(float* p, float* out) {
  gfloat* g = (gfloat*)p;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 1024, 0x00020000);
  g[threadIdx.x] = 1.0f;
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 2.0f), rs, threadIdx.x * 4, 0, 0);
  out[threadIdx.x] = g[threadIdx.x];
}
// T2: buffer store then global store then buffer load -> forwarded?
extern "C" __global__ void t2(float* p, float* out) {
  gfloat* g = (gfloat*)p;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 1024, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 2.0f), rs, threadIdx.x * 4, 0, 0);
  g[threadIdx.x] = 1.0f;
  out[threadIdx.x] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, threadIdx.x * 4, 0, 0));
}
// T3: buffer store, buffer store (same rsrc, same offset), buffer load
extern "C" __global__ void t3(float* p, float* out, int o) {
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 1024, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 2.0f), rs, threadIdx.x * 4, o, 0);
  float x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, threadIdx.x * 4, 0, 0));
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 3.0f), rs, threadIdx.x * 4, 0, 0);
  out[threadIdx.x] = x;
}
