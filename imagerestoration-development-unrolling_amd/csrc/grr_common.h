// Shared helpers for the gfx950 kernels of libgrr.so (status plumbing, indexing,
// XCD-aware block remap).  Written for CDNA4 only: wave64, 8 XCDs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/grr.h"

namespace grr {

// thread-local last error (grr_last_error)
void set_error(const char* fmt, ...);
void clear_error();

#define GRR_REQUIRE(cond, code, ...)        \
  do {                                      \
    if (!(cond)) {                          \
      ::grr::set_error(__VA_ARGS__);        \
      return code;                          \
    }                                       \
  } while (0)

// Check the launch that was just queued on the stream.
grr_status launch_status(const char* what);

constexpr int kWave = 64;
constexpr int kXcd = 8;

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch);
// re-label them so each XCD walks one contiguous chunk of the logical grid, i.e.
// neighbouring tiles (which share halo lines) share that XCD's L2.  Bijective for
// any n (cdna_hip_programming.md, "XCD swizzle must be bijective").  Speed only.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t n) {
  const uint32_t xcd = bid % kXcd, q = n / kXcd, r = n % kXcd;
  const uint32_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / kXcd;
}

// LocalNonLinearBlock on the split-bf16 MFMA kernels (lnb_ops.hip), C <= 128
int64_t lnb_mfma_workspace_floats(int B, int C, int hid, int H, int W);
int64_t fused_pack_floats(int C, int hid);   // the fused block's chunk images + W2 row scales
bool lnb_fused(int C, int hid);
// C <= 96 runs the whole block as one fused pass (lnb_fused16_kernel); keep_g: it also stores the gated
// activation g [B, hid, H, W] at the workspace's start (where the two-kernel path leaves it anyway)
bool lnb_fused(int C, int hid);
grr_status lnb_forward_mfma(const float* x, const float* ln_w, const float* w1, const float* wdw, const float* w2,
                            const float* skip, float* out, float* ws, int B, int C, int hid, int H, int W,
                            hipStream_t s, bool keep_g = false, int io = 0);
// the same block when x holds R stacked copies of the Ch-channel image xh (GEMM1 runs on xh)
grr_status lnb_forward_mfma_rep(const float* xh, int Ch, int R, const float* x, const float* ln_w, const float* w1,
                                const float* wdw, const float* w2, const float* skip, float* out, float* ws, int B,
                                int hid, int H, int W, hipStream_t s);

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// ---------------------------------------------------------------------------
// Fixed-order reductions of the training reverse (per-graph scalars, stencil / depthwise taps,
// multiM): no float atomics.  A reduced value idx has one partial slot per contributor (a wave or
// a workgroup of the launch) in a scratch array [n][nslot]; each contributor stores its partial
// into its own slot, and red_finish_kernel then adds each row, in slot order, to the destination
// (dst[idx] += sum).  The result is the same on every run, whatever the schedule or the stream
// interleaving.
// ---------------------------------------------------------------------------
struct Red {
  float* p;          // [n][nslot] partials; nullptr: the value is not wanted
  uint32_t nslot;
};
__device__ __forceinline__ void red_put(const Red& r, int idx, uint32_t slot, float v) {
  if (r.p) r.p[(size_t)idx * r.nslot + slot] = v;
}

// Host side: the partial arrays of one launch, carved from a scratch buffer leased for the stream (a
// per-stream grow-only buffer from the registered allocator -- PyTorch's caching allocator in the
// Python package -- or hipMalloc; grr_set_scratch_allocator, graph_bwd.hip), then finished (one launch
// for all of them) and returned.  Every kernel stores every slot of its plan (zero partials included),
// so the scratch needs no fill.
class RedScratch {
 public:
  static constexpr int kMax = 4;
  explicit RedScratch(hipStream_t s) : s_(s) {}
  RedScratch(const RedScratch&) = delete;
  RedScratch& operator=(const RedScratch&) = delete;
  ~RedScratch();
  int plan(float* dst, int n, uint32_t nslot);   // before alloc(); dst == nullptr: not wanted
  grr_status alloc(const char* what);
  Red red(int i) const { return Red{dst_[i] ? part_[i] : nullptr, nslot_[i]}; }
  grr_status finish(const char* what);            // dst[idx] += sum over slots; frees the scratch

 private:
  hipStream_t s_;
  int k_ = 0;
  float* dst_[kMax] = {};
  float* part_[kMax] = {};
  int n_[kMax] = {};
  uint32_t nslot_[kMax] = {};
  void* base_ = nullptr;
};

}  // namespace grr
