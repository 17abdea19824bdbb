// Standalone check of the primitives used by the streaming graph operator:
// raw buffer load/store with (voffset, soffset) and DPP wave_shr:1 / wave_shl:1.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__device__ __forceinline__ float lane_prev(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_next(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, false));
}
__global__ void k(const float* x, float* y, int W, int rows) {
  auto r = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, W * rows * 4, 0x00020000);
  auto w = __builtin_amdgcn_make_buffer_rsrc((void*)y, (short)0, 3 * W * rows * 4, 0x00020000);
  int lane = threadIdx.x & 63;
  for (int t = 0; t < rows; ++t) {
    float v = __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4, t * W * 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(v, w, lane * 4, t * W * 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(lane_prev(v), w, lane * 4, (rows + t) * W * 4, 0);
    __builtin_amdgcn_raw_buffer_store_b32(lane_next(v), w, lane * 4, (2 * rows + t) * W * 4, 0);
  }
}
int main() {
  const int W = 64, R = 3;
  std::vector<float> h(W * R), o(3 * W * R, -1.f);
  for (int i = 0; i < W * R; ++i) h[i] = i;
  float *dx, *dy;
  hipMalloc(&dx, h.size() * 4); hipMalloc(&dy, o.size() * 4);
  hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, o.data(), o.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dx, dy, W, R);
  hipMemcpy(o.data(), dy, o.size() * 4, hipMemcpyDeviceToHost);
  for (int blk = 0; blk < 3; ++blk) {
    printf("%s:", blk == 0 ? "copy" : blk == 1 ? "prev" : "next");
    for (int t = 0; t < R; ++t) printf(" [row%d: %g %g %g .. %g %g]", t, o[(blk*R+t)*W+0], o[(blk*R+t)*W+1], o[(blk*R+t)*W+2], o[(blk*R+t)*W+62], o[(blk*R+t)*W+63]);
    printf("\n");
  }
  return 0;
}
