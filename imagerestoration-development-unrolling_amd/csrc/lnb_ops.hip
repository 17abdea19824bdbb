// LocalNonLinearBlock (nsubnets = 1) on gfx950 — REF:911-964, REF13:541-575.
//
//   n   = ln_w * x / sqrt(var_c x + 1e-5)            CustomLayerNorm (unbiased var over C)
//   h   = W1 n                                        1x1, C -> 2 hid
//   m,v = dw3x3_replicate(h)[:hid], [hid:]            depthwise 3x3
//   g   = sigmoid(m) * m * v                          gate
//   out = skip0 * x + skip1 * W2 g                    1x1, hid -> C
//
// Two kernels.  The 2*hid-channel hidden tensor h never reaches HBM:
//
//  lnb_head_kernel  LN + W1 + depthwise 3x3 + gate, x -> g [B, hid, H, W].
//    A 512-thread workgroup owns a 32-column x TH-row output tile and recomputes W1 on
//    its (TH+2) x 34 halo (replicate padding = clamped halo coordinates).  Every wave keeps
//    the x / sigma columns of its halo pixels as an exact 3-term bf16 split in registers (B
//    operand of v_mfma_f32_16x16x32_bf16; LN folded: W1 (ln_w * x / sigma) = (W1 diag ln_w)
//    (x / sigma)); the hidden channels are walked in
//    chunks of 8 (mask, value) pairs = 16 GEMM rows.  A chunk's W1.diag(ln_w) fragments
//    arrive by LDS-DMA in a 3-slot ring two chunks ahead; its 16 x halo h image goes to a double-buffered LDS plane set, from
//    which the next iteration evaluates the depthwise 3x3 + gate (one wave per hidden
//    channel, lane = output column) while the matrix cores run the following chunk.  One
//    barrier per chunk; every wave issues a fixed sequence of memory operations per
//    iteration (dummy DMA / out-of-range buffer stores at the edges), so the ring is
//    waited on with a counted vmcnt.  The K = 3 head (the image filter's replicated first block,
//    110 VGPRs) keeps one chunk in flight instead of two and runs two workgroups per CU.
//
//  lnb_mix_kernel   W2 g + skip, g, x -> out.  256 pixels x all C rows per workgroup,
//    W2 (split, fragment order) streamed through a 4-slot LDS-DMA ring per 16-deep k-step,
//    g loaded two k-steps ahead and split in registers (B operand of
//    v_mfma_f32_32x32x16_bf16, 32 consecutive pixels per 32-lane half = 128-B loads).
//
// Arithmetic: both GEMMs use the exact 3-term bf16 split of feature_ops.hip (six products,
// fp32-accurate); depthwise 3x3 and the gate in fp32 with the reference's tap order.
#include <cstdlib>

#include "grr_common.h"

namespace grr {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// exact split v = v0 + v1 + v2 of 8 values into bf16 terms (RNE casts: v_cvt_pk_bf16_f32)
__device__ __forceinline__ void split3x8(const float (&v)[8], bf16x8& t0, bf16x8& t1, bf16x8& t2) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h0 = (__bf16)v[j];
    const float r1 = v[j] - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    const float r2 = r1 - (float)h1;
    t0[j] = h0;
    t1[j] = h1;
    t2[j] = (__bf16)r2;
  }
}
__host__ __device__ inline uint16_t bf16_bits_rne(float v) {
  uint32_t u;
  __builtin_memcpy(&u, &v, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_bits_val(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t split_term(float v, int q) {
  const uint16_t h0 = bf16_bits_rne(v);
  if (q == 0) return h0;
  const float r1 = v - bf16_bits_val(h0);
  const uint16_t h1 = bf16_bits_rne(r1);
  if (q == 1) return h1;
  return bf16_bits_rne(r1 - bf16_bits_val(h1));
}

// six-product accumulation of (a0+a1+a2)(b0+b1+b2), smallest terms first
#define GRR_X3_MFMA(FN, acc, a0, a1, a2, b0, b1, b2) \
  do {                                               \
    acc = FN(a1, b1, acc, 0, 0, 0);                  \
    acc = FN(a2, b0, acc, 0, 0, 0);                  \
    acc = FN(a0, b2, acc, 0, 0, 0);                  \
    acc = FN(a1, b0, acc, 0, 0, 0);                  \
    acc = FN(a0, b1, acc, 0, 0, 0);                  \
    acc = FN(a0, b0, acc, 0, 0, 0);                  \
  } while (0)

__device__ __forceinline__ void dma16(const void* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (lds_ptr_t)lds_wave_base, 16, 0, 0);
}
// The same 16-byte LDS-DMA as an asm statement.  hipcc answers every LDS-DMA builtin with
// lgkmcnt(0) waits at all later LDS reads (it cannot order the DMA's LDS write against them);
// the head kernel orders its ring itself (counted vmcnt + barrier), so it issues the DMA
// opaquely and keeps the compiler's counted lgkmcnt waits.  The compiler does not count these
// operations: they are only issued where no compiler-visible vector-memory load is pending
// behind them.
typedef __attribute__((address_space(3))) float* lds_f32_t;
__device__ __forceinline__ void dma16_opaque(const void* src, float* lds_wave_base) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(lds_f32_t)lds_wave_base;
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(__builtin_amdgcn_readfirstlane(m0v)) : "memory");
}

// ---------------------------------------------------------------------------
// head: LN + W1 + dw3x3 + gate
constexpr int LH_TW = 32;           // output columns per tile
constexpr int LH_HWD = LH_TW + 2;   // halo columns
constexpr int LH_JC = 8;            // (mask, value) pairs per chunk -> 16 GEMM rows

template <int NB>
struct HeadGeom {
  static constexpr int NH = 8 * NB * 16;     // halo pixels held by the 8 waves
  static constexpr int HR = NH / LH_HWD;     // halo rows
  static constexpr int TH = HR - 2;          // output rows
  static constexpr int RA = (TH + 1) / 2;    // output rows per half-wave in the gate phase
  static constexpr int HP = NH + 4;          // LDS pitch of one h row (== 4 mod 8: conflict-free writes)
};

struct LnbHeadArgs {
  const float* x;        // [B, C, H, W]
  const char* w1f;       // [nch][KS*3 + 1] images of 1 KB: W1 diag(ln_w) fragments, then the chunk's taps
  float* g;              // [B, hid, H, W]
  float var_den;         // unbiased-variance denominator: C - 1, or (R C - 1) / R for an R-fold replicated x
  int C, hid, H, W, tiles_x, tiles_y, nch;
  uint32_t nblk;
};

// Per chunk c (8 hidden channels): KS*3 bf16 images of 16x16x32 A fragments of W1 diag(ln_w)
// (k-step s, term q, lane l, element j: row r = l & 15 -- r < 8: mask channel 8c + r, else
// value channel hid + 8c + r - 8 -- and k = 32 s + 8 (l >> 4) + j), then one fp32 image with
// the depthwise taps: [w][2 t], [w][2 t + 1] = tap t of mask channel 8c + w and of value channel hid + 8c + w.
__host__ __device__ inline int head_images(int KS) { return KS * 3 + 1; }

// R > 1: the block's input is R stacked copies of a C-channel image (MultiScaleGraphFilter's
// graph replicas, REF13:918-921); W1 diag(ln_w) is folded over the copies (w1 rows have R*C
// entries), so GEMM1 runs with K = C instead of R*C.
__global__ void lnb_w1_pack_kernel(const float* __restrict__ w1, const float* __restrict__ ln_w,
                                   const float* __restrict__ wdw, char* __restrict__ out, int C, int hid, int KS,
                                   int nch, int R) {
  const int NI = head_images(KS);
  const int64_t n = (int64_t)nch * NI * 256;        // 32-bit words
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i >> 8;
    const int e = (int)(i & 255), c = (int)(img / NI), im = (int)(img % NI);
    uint32_t word = 0;
    if (im < KS * 3) {
      const int q = im % 3, s = im / 3, l = e >> 2, r = l & 15, jj = LH_JC * c + (r & 7);
      uint16_t h[2] = {0, 0};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = 32 * s + 8 * (l >> 4) + 2 * (e & 3) + u;
        if (jj < hid && k < C) {
          const float* wr = w1 + (int64_t)((r < 8 ? 0 : hid) + jj) * (R * C);
          float v = wr[k] * ln_w[k];
          for (int rep = 1; rep < R; ++rep) v += wr[rep * C + k] * ln_w[rep * C + k];
          h[u] = split_term(v, q);
        }
      }
      word = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
    } else if (e < LH_JC * 18) {   // taps of chunk channel w: (mask, value) pairs, tap by tap
      const int w = e / 18, t = (e % 18) >> 1, comp = e & 1, jj = LH_JC * c + w;
      if (jj < hid) word = __float_as_uint(wdw[(int64_t)((comp ? hid : 0) + jj) * 9 + t]);
    }
    reinterpret_cast<uint32_t*>(out)[i] = word;
  }
}

// chunks of W1 fragments in flight ahead of GEMM1; the K = 3 head (110 VGPRs) runs two workgroups
// per CU with one chunk ahead (3-slot ring: 78 KB of LDS per workgroup)
__host__ __device__ constexpr int head_ahead(int KS) { return KS == 1 ? 1 : 2; }
__host__ __device__ constexpr int head_wgs(int KS) { return KS == 1 ? 2 : 1; }

template <int KS, int NB>
__global__ __launch_bounds__(512, head_wgs(KS)) void lnb_head_kernel(LnbHeadArgs a) {
  using Geo = HeadGeom<NB>;
  constexpr int NI = KS * 3 + 1;        // images per chunk (fragments + taps)
  constexpr int DPW = (NI + 7) / 8;     // LDS-DMA instructions per wave per chunk
  constexpr int SLOTF = NI * 256;       // floats per ring slot
  constexpr int AHEAD = head_ahead(KS);
  constexpr int NSLOT = AHEAD + 2;      // chunks in flight + GEMM1(c) + gate(c - 1)
  constexpr int HBUF = 2 * LH_JC * Geo::HP;
  constexpr int RA = Geo::RA;
  __shared__ __attribute__((aligned(16))) float smem[2 * HBUF + NSLOT * SLOTF];
  float* const ring = smem + 2 * HBUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int tx = lb % a.tiles_x; lb /= a.tiles_x;
  const int ty = lb % a.tiles_y;
  const int b = lb / a.tiles_y;
  const int H = a.H, W = a.W, C = a.C, hid = a.hid, nch = a.nch;
  const int HW = H * W;
  const int y0 = ty * Geo::TH, x0 = tx * LH_TW;

  auto issue = [&](int chunk, int slot_idx) {
    float* slot = ring + slot_idx * SLOTF;
    const char* src = a.w1f + (int64_t)chunk * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int img = min(i * 8 + wave, NI - 1);   // surplus waves repeat the last image
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };
  issue(0, 0);
  if constexpr (AHEAD == 2) issue(min(1, nch - 1), 1);

  // this wave's halo pixels: raw x column split into bf16 terms, and 1/sigma (REF:916-922)
  const int kq = lane >> 4;
  bf16x8 xf[NB][KS][3];
  float rstd[NB];
  float xv[NB][KS][8];
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    const int q = min((wave * NB + blk) * 16 + (lane & 15), Geo::HR * LH_HWD - 1);
    const int hy = q / LH_HWD, hx = q - hy * LH_HWD;
    const int gy = clampi(y0 - 1 + hy, 0, H - 1), gx = clampi(x0 - 1 + hx, 0, W - 1);
    const float* xp = a.x + (int64_t)b * C * HW + gy * W + gx;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[blk][s][j] = xp[(int64_t)min(32 * s + 8 * kq + j, C - 1) * HW];
  }
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (32 * s + 8 * kq + j >= C) xv[blk][s][j] = 0.f;
        sum += xv[blk][s][j];
      }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float mean = sum / (float)C;
    float sq = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = 32 * s + 8 * kq + j < C ? xv[blk][s][j] - mean : 0.f;
        sq += d * d;
      }
    sq += __shfl_xor(sq, 16);
    sq += __shfl_xor(sq, 32);
    rstd[blk] = 1.0f / sqrtf(sq / a.var_den + 1e-5f);
    // x / sigma first (REF:921), so h = (W1 diag ln_w) (x / sigma) leaves GEMM1 unscaled
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[blk][s][j] *= rstd[blk];
#pragma unroll
    for (int s = 0; s < KS; ++s) split3x8(xv[blk][s], xf[blk][s][0], xf[blk][s][1], xf[blk][s][2]);
  }

  // chunks 0 and 1 landed (this wave's DMAs), then every wave's: the ring is shared
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // gate phase mapping: wave = hidden channel of the chunk, lane = (output column, row half)
  const int col = lane & 31, r0 = (lane >> 5) * RA;
  const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
      a.g + (int64_t)b * hid * HW, 0, (int)((int64_t)hid * HW * 4), 0x00020000);
  const int gx = x0 + col;

  auto gemm1 = [&](int c) {
    if (c >= nch) return;
    const float* slot = ring + (c % NSLOT) * SLOTF + lane * 4;
    f32x4 acc[NB];
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) acc[blk] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 0) * 256);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 1) * 256);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 2) * 256);
#pragma unroll
      for (int blk = 0; blk < NB; ++blk)
        GRR_X3_MFMA(__builtin_amdgcn_mfma_f32_16x16x32_bf16, acc[blk], a0, a1, a2, xf[blk][s][0],
                    xf[blk][s][1], xf[blk][s][2]);
    }
    // h rows 4 kq + i (0..7 mask, 8..15 value) of the halo pixels -> LDS plane set c & 1
    float* hb = smem + (c & 1) * HBUF;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      const int q = (wave * NB + blk) * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) hb[(4 * kq + i) * Geo::HP + q] = acc[blk][i];
    }
  };
  // depthwise 3x3 (REF:946) + gate sigmoid(m) m v (REF:947) of chunk c - 1
  auto gate = [&](int c) {
    const int jj = LH_JC * (c - 1) + wave;
    const bool live = c >= 1 && jj < hid;
    const bool lane_ok = live && gx < W;
    const int nrow = min(Geo::TH, H - y0) - r0;   // output rows of this lane's half inside the tile and image
    const uint32_t off0 = (uint32_t)(jj * HW + (y0 + r0) * W + gx) * 4u;
    const float* hb = smem + ((c + 1) & 1) * HBUF;
    const float* mp = hb + wave * Geo::HP + col;
    const float* vp = hb + (LH_JC + wave) * Geo::HP + col;
    const float* taps = ring + ((c + NSLOT - 1) % NSLOT) * SLOTF + KS * 3 * 256 + wave * 18;
    float km[9], kv[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      km[t] = taps[2 * t];
      kv[t] = taps[2 * t + 1];
    }
    float mw[3][3], vw[3][3];
#pragma unroll
    for (int i = 0; i < RA + 2; ++i) {
      const int hrow = min(r0 + i, Geo::HR - 1) * LH_HWD;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        mw[i % 3][d] = mp[hrow + d];
        vw[i % 3][d] = vp[hrow + d];
      }
      if (i >= 2) {
        float m = 0.f, v = 0.f;
#pragma unroll
        for (int ay = 0; ay < 3; ++ay)
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) {
            m += km[ay * 3 + ax] * mw[(i - 2 + ay) % 3][ax];
            v += kv[ay * 3 + ax] * vw[(i - 2 + ay) % 3][ax];
          }
        const float gv = (m * v) * __builtin_amdgcn_rcpf(1.0f + __expf(-m));   // sigmoid(m) m v
        const bool ok = lane_ok && i - 2 < nrow;
        const uint32_t off = ok ? off0 + (uint32_t)((i - 2) * W) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gv), grs, off, 0, 0);
      }
    }
  };

  // Iteration c: GEMM1 of chunk c and the gate of chunk c - 1 (independent LDS planes).  The two
  // waves sharing a SIMD (w, w + 4) run them in opposite orders, so one wave's matrix work
  // overlaps the other's vector / LDS work (MI355X_MICROARCH.md, two waves per SIMD: stagger).
  const bool gate_first = wave < 4;
  for (int c = 0; c <= nch; ++c) {
    // chunk c + AHEAD -> slot (c + AHEAD) % NSLOT, last read (gate of chunk c - 2) before the previous barrier
    issue(min(c + AHEAD, nch - 1), (c + AHEAD) % NSLOT);
    if (gate_first) {
      gate(c);
      gemm1(c);
    } else {
      gemm1(c);
      gate(c);
    }
    // chunk c + 1 landed: after its DMA this wave issued RA stores (iteration c - 1),
    // DPW DMAs and RA stores (iteration c) -- AHEAD = 1: RA stores (iteration c); then every
    // wave's part (barrier)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(AHEAD == 2 ? 2 * RA + DPW : RA) : "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// ---------------------------------------------------------------------------
// head16: LN + W1 + dw3x3 + gate with GEMM1 on fp16 two-term splits (C <= 96)
//
// GEMM1 h = (W1 diag ln_w)(x / sigma) runs on v_mfma_f32_32x32x16_f16 with both operands as
// exact two-term fp16 splits a = a_hi + a_lo (22 significant bits) and three products
// (a_lo b_hi, a_hi b_lo, a_hi b_hi; the dropped a_lo b_lo is below 2^-22 |a b|): the products
// are exact in the fp32 accumulator, so each term's error is the 2^-22 representation error,
// the order of fp32 rounding in a K-deep fp32 sum (tests/test_gpu_parity.py:
// test_x3_gemm_is_fp32_accurate bounds the block against float64).  fp16 has a narrow exponent
// range, so both operands are power-of-two scaled, exactly: every W1 row by 2^s_row (its largest
// entry into [2^13, 2^14)), every halo pixel's x / sigma by 2^XE (2^e_p for a pixel whose
// largest |x / sigma| leaves [2^-10, 2^4)).  h is stored as 2^(s_row + XE) h (pixels with
// e_p != XE are rescaled once when their h goes to LDS) and the depthwise taps are packed as
// tap 2^-(s_row + XE), so the depthwise sums -- and everything after -- are the unscaled values.
//
// Against the bf16 head (lnb_head_kernel): half the MFMA products for the same fp32-class
// accuracy, and 32x32x16 MFMAs (they hold the SIMD's vector issue 8 of 32 cycles instead of
// 8 of 16), so the partner wave's depthwise + gate gets the issue slots.  Tile as before (32 x
// 13 outputs, 34 x 15 halo pixels); a chunk is 16 (mask, value) pairs = 32 GEMM rows; the h of
// a chunk lives in LDS as 16 pair planes ((m, v) interleaved per halo pixel: one ds_write_b64
// per pair of accumulator registers, one ds_read_b64 per tap column in the gate), double
// buffered (2 x 64 KB); the W1 fragments + taps of a chunk arrive by LDS-DMA in a 2-slot ring
// one chunk ahead (the taps of the chunk the gate needs next are copied to registers first).
constexpr int L6_NP = 16;                   // (mask, value) pairs per chunk
constexpr int L6_NB = 2;                    // 32-pixel GEMM1 blocks per wave
constexpr int L6_NH = 8 * L6_NB * 32;       // halo pixels of a tile (512; 510 used)
constexpr int L6_HR = L6_NH / LH_HWD;       // halo rows (15)
constexpr int L6_TH = L6_HR - 2;            // output rows (13)
constexpr int L6_PP = 2 * L6_NH;            // floats per pair plane
constexpr int L6_HBUF = L6_NP * L6_PP;      // floats per h buffer (64 KB)
constexpr int L6_XE = 10;                   // common power-of-two scale of the fp16 x operand
constexpr int L6_TAPF = L6_NP * 18;         // tap floats per chunk
__host__ __device__ constexpr int head16_images(int KS) { return 2 * KS + 2; }   // fp16 hi/lo per k-step + 2 tap images

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// largest |W1 diag(ln_w)| entry of GEMM row `row` (folded over the R replicas) -> its scale exponent
__device__ __forceinline__ int head16_row_exp(const float* __restrict__ w1, const float* __restrict__ ln_w, int row,
                                              int C, int R) {
  const float* wr = w1 + (int64_t)row * (R * C);
  float mx = 0.f;
  for (int k = 0; k < C; ++k) {
    float v = wr[k] * ln_w[k];
    for (int rep = 1; rep < R; ++rep) v += wr[rep * C + k] * ln_w[rep * C + k];
    mx = fmaxf(mx, fabsf(v));
  }
  if (mx == 0.f) return 0;
  int e;
  frexpf(mx, &e);                 // mx < 2^e
  return clampi(14 - e, -60, 60); // mx 2^s in [2^13, 2^14)
}

// Per chunk c (16 pairs): for k-step s (16 deep) two 1-KB images of 32x32x16 A fragments
// (term q = 0 hi, 1 lo; lane l, element j: GEMM row r = l & 31 -- pair 16 c + (r >> 1), mask
// (r even) or value (r odd) channel -- and k = 16 s + 8 (l >> 5) + j), then two fp32 images with
// the depthwise taps, [pair w][tap t][mask, value], scaled by 2^-(s_row + XE).
__global__ void lnb_w1_pack16_kernel(const float* __restrict__ w1, const float* __restrict__ ln_w,
                                     const float* __restrict__ wdw, char* __restrict__ out, int C, int hid, int KS,
                                     int nch, int R) {
  const int NI = head16_images(KS);
  const int64_t n = (int64_t)nch * NI * 256;        // 32-bit words
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i >> 8;
    const int e = (int)(i & 255), c = (int)(img / NI), im = (int)(img % NI);
    uint32_t word = 0;
    if (im < 2 * KS) {
      const int q = im & 1, s = im >> 1, l = e >> 2, r = l & 31, pj = L6_NP * c + (r >> 1);
      if (pj < hid) {
        const int row = (r & 1 ? hid : 0) + pj;
        const int sc = head16_row_exp(w1, ln_w, row, C, R);
        const float* wr = w1 + (int64_t)row * (R * C);
        uint16_t hb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int k = 16 * s + 8 * (l >> 5) + 2 * (e & 3) + u;
          float v = 0.f;
          if (k < C) {
            v = wr[k] * ln_w[k];
            for (int rep = 1; rep < R; ++rep) v += wr[rep * C + k] * ln_w[rep * C + k];
          }
          const float vs = ldexpf(v, sc);
          const _Float16 h0 = (_Float16)vs;
          const _Float16 t = q == 0 ? h0 : (_Float16)(vs - (float)h0);
          hb[u] = __builtin_bit_cast(uint16_t, t);
        }
        word = (uint32_t)hb[0] | ((uint32_t)hb[1] << 16);
      }
    } else {
      const int e2 = (im - 2 * KS) * 256 + e;
      if (e2 < L6_TAPF) {
        const int w = e2 / 18, t = (e2 % 18) >> 1, comp = e2 & 1, pj = L6_NP * c + w;
        if (pj < hid) {
          const int row = (comp ? hid : 0) + pj;
          const int sc = head16_row_exp(w1, ln_w, row, C, R);
          // the gate's exp2 argument and product fold in here (lnb_head16_kernel, gate): mask taps
          // carry -log2(e), value taps -ln(2), so m' = -log2(e) m, v' = -ln(2) v, m' v' = m v and
          // sigmoid(m) = 1 / (1 + 2^m')
          const float fold = comp ? -0.69314718055994531f : -1.44269504088896341f;
          word = __float_as_uint(ldexpf(wdw[(int64_t)row * 9 + t], -(sc + L6_XE)) * fold);
        }
      }
    }
    reinterpret_cast<uint32_t*>(out)[i] = word;
  }
}

// NW = 8 waves per workgroup: each computes GEMM1 for NB = 2 blocks of 32 halo pixels and the gate of
// PPW = 2 pairs per chunk (a 16-wave workgroup, one block and one pair per wave, measured within 2 %)
template <int KS, int NW>
__global__ __launch_bounds__(64 * NW, 1) void lnb_head16_kernel(LnbHeadArgs a) {
  static_assert(NW == 8, "lnb_head16_kernel: 8 waves");
  constexpr int NB = L6_NB * 8 / NW, PPW = L6_NP / NW;
  constexpr int NI = head16_images(KS);
  constexpr int DPW = (NI + NW - 1) / NW;  // LDS-DMA instructions per wave per chunk
  constexpr int SLOTF = NI * 256;        // floats per ring slot
  __shared__ __attribute__((aligned(16))) float smem[2 * L6_HBUF + 2 * SLOTF];
  float* const ring = smem + 2 * L6_HBUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int tx = lb % a.tiles_x; lb /= a.tiles_x;
  const int ty = lb % a.tiles_y;
  const int b = lb / a.tiles_y;
  const int H = a.H, W = a.W, C = a.C, hid = a.hid, nch = a.nch;
  const int HW = H * W;
  const int y0 = ty * L6_TH, x0 = tx * LH_TW;

  auto issue = [&](int chunk, int slot_idx) {
    float* slot = ring + slot_idx * SLOTF;
    const char* src = a.w1f + (int64_t)chunk * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int img = min(i * NW + wave, NI - 1);   // surplus waves repeat the last image
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };
  issue(0, 0);

  // this wave's halo pixels (block blk: pixel q = (wave NB + blk) 32 + (lane & 31)); lane half kh
  // holds channels 16 s + 8 kh + j of it
  const int kh = lane >> 5;
  f16x8 xh[NB][KS], xl[NB][KS];
  float corr[NB];
  bool any_corr = false;
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    const int q = min((wave * NB + blk) * 32 + (lane & 31), L6_HR * LH_HWD - 1);
    const int hy = q / LH_HWD, hx = q - hy * LH_HWD;
    const int gy = clampi(y0 - 1 + hy, 0, H - 1), gx = clampi(x0 - 1 + hx, 0, W - 1);
    const float* xp = a.x + (int64_t)b * C * HW + gy * W + gx;
    float xv[KS][8];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * kh + j;
        const float v = xp[(int64_t)min(k, C - 1) * HW];
        xv[s][j] = k < C ? v : 0.f;
      }
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += xv[s][j];
    sum += __shfl_xor(sum, 32);
    const float mean = sum / (float)C;
    float sq = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = 16 * s + 8 * kh + j < C ? xv[s][j] - mean : 0.f;
        sq += d * d;
      }
    sq += __shfl_xor(sq, 32);
    const float rstd = 1.0f / sqrtf(sq / a.var_den + 1e-5f);
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xv[s][j] *= rstd;                       // x / sigma (REF:921)
        mx = fmaxf(mx, fabsf(xv[s][j]));
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    int ep = L6_XE;
    if (mx != 0.f) {
      int e;
      frexpf(mx, &e);                         // mx < 2^e
      if (e > 14 - L6_XE || e < -L6_XE) ep = clampi(14 - e, -100, 100);
    }
    corr[blk] = ldexpf(1.0f, L6_XE - ep);
    any_corr |= ep != L6_XE;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = ldexpf(xv[s][j], ep);
        const _Float16 h0 = (_Float16)v;
        xh[blk][s][j] = h0;
        xl[blk][s][j] = (_Float16)(v - (float)h0);
      }
  }
  // wave-uniform (scalar branch at the h store; almost never taken on LayerNorm'd inputs)
  const bool wave_corr = __builtin_amdgcn_readfirstlane((int)__any(any_corr)) != 0;

  // GEMM1 of chunk c (ring slot c & 1) -> pair planes of h buffer c & 1
  auto gemm1_mma = [&](int c, f32x16 (&acc)[NB]) {
    const float* slot = ring + (c & 1) * SLOTF + lane * 4;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) acc[blk] = f32x16{};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(slot + (2 * s + 0) * 256);
      const f16x8 al = *reinterpret_cast<const f16x8*>(slot + (2 * s + 1) * 256);
#pragma unroll
      for (int blk = 0; blk < NB; ++blk) {
        acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh[blk][s], acc[blk], 0, 0, 0);
        acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl[blk][s], acc[blk], 0, 0, 0);
        acc[blk] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh[blk][s], acc[blk], 0, 0, 0);
      }
    }
  };
  auto gemm1_store = [&](int c, f32x16 (&acc)[NB]) {
    float* hb = smem + (c & 1) * L6_HBUF;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      if (wave_corr) acc[blk] *= corr[blk];
      const int q = (wave * NB + blk) * 32 + (lane & 31);
      // registers 2u, 2u + 1 = rows r, r + 1 (r even: mask, value of pair r / 2)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = ((2 * u) & 3) + 8 * ((2 * u) >> 2) + 4 * kh;
        *reinterpret_cast<f32x2*>(hb + (r >> 1) * L6_PP + 2 * q) = f32x2{acc[blk][2 * u], acc[blk][2 * u + 1]};
      }
    }
  };
  auto gemm1 = [&](int c) {
    if (c >= nch) return;
    f32x16 acc[NB];
    gemm1_mma(c, acc);
    gemm1_store(c, acc);
  };

  // gate phase mapping: lane = (output column, pair kh of the wave's two); every lane runs all L6_TH output
  // rows of its pair (15 halo rows read for 13 outputs, against 18 for 14 with a lane per half column:
  // 1.7 % faster at C = 96, 5.6 % on the replicated block, round 4)
  const int col = lane & 31;
  const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
      a.g + (int64_t)b * hid * HW, 0, (int)((int64_t)hid * HW * 4), 0x00020000);
  const int gx = x0 + col;
  // g stores: the lane's byte offset of output row k (row y0 + k, its column, its pair's plane kh HW) in
  // voffset -- out of range for rows past the tile or the image and for columns past the image, fixed for
  // the whole kernel (vrow) -- and the wave's first pair plane and the row, wave-uniform, in soffset
  static_assert(PPW == 2, "lnb_head16_kernel: the gate maps the wave's two pairs to its lane halves");
  constexpr uint32_t kOut = 0x80000000u;
  constexpr int GR = L6_TH;                      // output rows per lane
  const int nrow = min(L6_TH, H - y0);           // output rows inside the tile and image
  const uint32_t vcol = gx < W ? (uint32_t)(kh * HW + y0 * W + gx) * 4u : kOut;
  uint32_t vrow[GR];
#pragma unroll
  for (int k = 0; k < GR; ++k) vrow[k] = k < nrow ? vcol : kOut;
  constexpr int kGateStores = GR;                // g stores per wave and iteration
  float tk[18];                                  // taps of the lane's pair in the chunk the next gate evaluates
  auto load_taps = [&](int c) {
    const float* t = ring + (c & 1) * SLOTF + 2 * KS * 256 + (PPW * wave + kh) * 18;
#pragma unroll
    for (int i = 0; i < 18; ++i) tk[i] = t[i];
  };
  // depthwise 3x3 (REF:946) + gate sigmoid(m) m v (REF:947) of chunk c, h buffer c & 1.  The taps carry
  // the exp2 fold of lnb_w1_pack16_kernel: m' = -log2(e) m, v' = -ln(2) v, g = m' v' / (1 + 2^m').
  auto gate = [&](int c) {
    const float* hbuf = smem + (c & 1) * L6_HBUF;
    const int jj0 = L6_NP * c + PPW * wave;        // the wave's first pair (lane half kh: pair jj0 + kh)
    const bool all_live = jj0 + 1 < hid;           // wave-uniform
    const bool live = jj0 + kh < hid;
    // soffset is not range-checked: a pair past the hidden channels stores out of range through voffset
    const int soff0 = jj0 < hid ? jj0 * HW * 4 : 0;
    const float* hp = hbuf + (PPW * wave + kh) * L6_PP + 2 * col;
    f32x2 win[3][3];                               // rows (i mod 3) x halo columns col .. col + 2
#pragma unroll
    for (int i = 0; i < GR + 2; ++i) {
      const int hrow = i * LH_HWD;
#pragma unroll
      for (int d = 0; d < 3; ++d) win[i % 3][d] = *reinterpret_cast<const f32x2*>(hp + 2 * (hrow + d));
      if (i >= 2) {
        const f32x2 h0 = win[(i - 2) % 3][0];
        float m = tk[0] * h0[0], v = tk[1] * h0[1];
#pragma unroll
        for (int t = 1; t < 9; ++t) {
          const f32x2 hv = win[(i - 2 + t / 3) % 3][t % 3];
          m = __builtin_fmaf(tk[2 * t], hv[0], m);
          v = __builtin_fmaf(tk[2 * t + 1], hv[1], v);
        }
        const float gv = (m * v) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(m));
        const uint32_t vo = all_live || live ? vrow[i - 2] : kOut;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(gv), grs, vo, soff0 + (i - 2) * W * 4, 0);
      }
    }
  };

  // prologue: chunk 0's fragments landed -> GEMM1(0), its taps, chunk 1 into slot 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  gemm1(0);
  load_taps(0);
  issue(min(1, nch - 1), 1);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  // Iteration c: gate of chunk c - 1 (h buffer (c - 1) & 1, taps in registers) and GEMM1 of chunk c
  // (slot c & 1 -> h buffer c & 1); the waves of a SIMD (w, w + 4) run them in opposite orders.  Slot
  // (c + 1) & 1 last served GEMM1(c - 1) and load_taps(c - 1), both before the previous barrier.
  const bool gate_first = wave < NW / 2;
  for (int c = 1; c <= nch; ++c) {
    issue(min(c + 1, nch - 1), (c + 1) & 1);
    if (gate_first) {
      gate(c - 1);
      gemm1(c);
    } else {
      gemm1(c);
      gate(c - 1);
    }
    if (c < nch) load_taps(c);
    // chunk c + 1 landed (after its DMAs this wave issued the GR gate stores), then every wave's
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(kGateStores) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
}

// ---------------------------------------------------------------------------
// rep: the image filter's first block -- input = the C_s-channel image replicated over the graphs
// (REF13:918-921), C_s <= 3 -- in one pass, LN through the skip, without g in HBM or h in LDS.
//
// The depthwise 3x3 is linear in h = W1' n, so it folds into GEMM1 as an im2col GEMM:
//   d[j, p] = sum_t tap[j, t] h[j, p + delta_t] = sum_{c, t} (tap[j, t] W1'[j, c]) n[c, p + delta_t]
// (W1' = W1 diag(ln_w) folded over the replicas, n = x / sigma, the replicate padding = clamped
// neighbour coordinates), K = 9 C_s <= 32: two 16-deep k-steps of v_mfma_f32_32x32x16_f16 on exact
// two-term fp16 splits (three products, head16's arithmetic and scaling: rows of the folded matrix by
// 2^s_row, each pixel's im2col column by 2^XE, corrected per column when its largest entry leaves the
// range).  The 32 x 32 accumulator of a chunk (16 (mask, value) pairs x 32 pixels) holds both halves
// of every pair in one lane, so the gate runs on it in registers, and the lane's eight gated values
// are already the B operand of GEMM2 (W2 g, v_mfma_f32_32x32x16_f16 on two-term splits) once W2's k
// order is permuted to the accumulator's pair order (lnb_rep_pack_kernel).  GEMM2's fp16 operands are
// power-of-two scaled: W2 rows by 2^s2_row, each pixel's gated values by a running exponent E (set by
// the first chunk's largest |g| of the pixel into [2^13, 2^14); a later chunk with larger values lowers
// E and scales the pixel's accumulators down by the exact power of two), undone in the epilogue.
// A workgroup = 8 waves x 32 pixels; the chunk's fragments (both GEMMs) and its per-row constants
// arrive by LDS-DMA in a 4-slot ring three chunks ahead; four waves per SIMD (two workgroups per CU)
// overlap one another's matrix and vector phases.  Against head16 + mix for
// this block: no g round trip (4 KB per pixel of HBM traffic), no h planes in LDS, no depthwise FMAs.
constexpr int LR_NW = 8;                  // waves per workgroup
constexpr int LR_PX = LR_NW * 32;         // pixels per workgroup (one 32-pixel block per wave)
constexpr int LR_XE = 10;                 // common power-of-two scale of the im2col operand
constexpr int LR_NSLOT = 4;               // ring slots (three chunks in flight ahead of GEMM2)
// A1 (2 k-steps x hi / lo), A2 (MT row tiles x hi / lo), the gate's row constants, the W2 row scales
__host__ __device__ constexpr int rep_images(int MT) { return 4 + 2 * MT + 1; }

struct LnbRepArgs {
  const float* xs;      // [B, Cs, P]: the image the block input replicates
  const char* pack;     // [nch][rep_images(MT)] 1-KB images
  const float* skip;    // [2]
  float* out;           // [B, C, P]
  float var_den;        // (C - 1) / R: the unbiased variance over the C replicated channels from the Cs sources
  int Cs, C, hid, H, W, nch, tiles;
  uint32_t nblk;
};

// scale exponent of a row whose largest |entry| is mx: mx 2^s in [2^13, 2^14)
__device__ __forceinline__ int rep_scale_exp(float mx) {
  if (mx == 0.f) return 0;
  int e;
  frexpf(mx, &e);
  return clampi(14 - e, -60, 60);
}
__device__ __forceinline__ float rep_w1f(const float* __restrict__ w1, const float* __restrict__ ln_w, int row, int c,
                                         int Cs, int R) {
  float w = 0.f;
  for (int rep = 0; rep < R; ++rep) w += w1[(int64_t)row * (R * Cs) + rep * Cs + c] * ln_w[rep * Cs + c];
  return w;
}
// largest |tap[row, t] W1'[row, c]| over the folded row (C_s channels x 9 taps) -> its scale exponent
__device__ __forceinline__ int rep_row_exp(const float* __restrict__ w1, const float* __restrict__ ln_w,
                                           const float* __restrict__ wdw, int row, int Cs, int R) {
  float mx = 0.f;
  for (int c = 0; c < Cs; ++c) {
    const float w = rep_w1f(w1, ln_w, row, c, Cs, R);
    for (int t = 0; t < 9; ++t) mx = fmaxf(mx, fabsf(wdw[(int64_t)row * 9 + t] * w));
  }
  return rep_scale_exp(mx);
}
__device__ __forceinline__ int rep_w2_exp(const float* __restrict__ w2, int m, int hid) {
  float mx = 0.f;
  for (int k = 0; k < hid; ++k) mx = fmaxf(mx, fabsf(w2[(int64_t)m * hid + k]));
  return rep_scale_exp(mx);
}
__device__ __forceinline__ uint32_t f16_pair_word(float a, float b, int q) {   // term q (0 hi, 1 lo) of a, b
  const _Float16 ha = (_Float16)a, hb = (_Float16)b;
  const _Float16 ta = q == 0 ? ha : (_Float16)(a - (float)ha), tb = q == 0 ? hb : (_Float16)(b - (float)hb);
  return (uint32_t)__builtin_bit_cast(uint16_t, ta) | ((uint32_t)__builtin_bit_cast(uint16_t, tb) << 16);
}

// Per chunk c (16 pairs): images 0..3 = A1 (k-step s = im >> 1, term hi / lo = im & 1; lane l, element j:
// GEMM row r = l & 31 -- pair 16 c + (r >> 1), mask (r even) or value -- and k = 16 s + 8 (l >> 5) + j =
// 9 c_s + t), scaled by 2^s_row; images 4 + 2 mt + q = A2 (W2 rows 32 mt + (l & 31) scaled by 2^s2_row,
// term q; k = 8 (l >> 5) + j is pair pi = 4 (j >> 1) + (j & 1) + 2 (l >> 5) of the chunk: the
// accumulator's pair order); image 4 + 2 MT: words 16 kh + i = the gate's constant of accumulator
// register i of lane half kh (row (i & 3) + 8 (i >> 2) + 4 kh): -log2(e) 2^-(s_row + XE) (mask rows),
// -ln(2) 2^-(s_row + XE) (value rows); words 32 + m = 2^-s2_row of output row m (C <= 128).
__global__ void lnb_rep_pack_kernel(const float* __restrict__ w1, const float* __restrict__ ln_w,
                                    const float* __restrict__ wdw, const float* __restrict__ w2,
                                    char* __restrict__ out, int Cs, int R, int C, int hid, int MT, int nch) {
  const int NI = rep_images(MT);
  const int64_t n = (int64_t)nch * NI * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t img = i >> 8;
    const int e = (int)(i & 255), c = (int)(img / NI), im = (int)(img % NI);
    const int l = e >> 2;
    uint32_t word = 0;
    if (im < 4) {
      const int s = im >> 1, q = im & 1, r = l & 31, pj = 16 * c + (r >> 1);
      if (pj < hid) {
        const int row = (r & 1 ? hid : 0) + pj;
        const int sc = rep_row_exp(w1, ln_w, wdw, row, Cs, R);
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int k = 16 * s + 8 * (l >> 5) + 2 * (e & 3) + u;
          v[u] = 0.f;
          if (k < 9 * Cs) v[u] = ldexpf(wdw[(int64_t)row * 9 + k % 9] * rep_w1f(w1, ln_w, row, k / 9, Cs, R), sc);
        }
        word = f16_pair_word(v[0], v[1], q);
      }
    } else if (im < 4 + 2 * MT) {
      const int mt = (im - 4) >> 1, q = (im - 4) & 1, m = 32 * mt + (l & 31);
      if (m < C) {
        const int sc = rep_w2_exp(w2, m, hid);
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int j = 2 * (e & 3) + u;
          const int pj = 16 * c + 4 * (j >> 1) + (j & 1) + 2 * (l >> 5);
          v[u] = pj < hid ? ldexpf(w2[(int64_t)m * hid + pj], sc) : 0.f;
        }
        word = f16_pair_word(v[0], v[1], q);
      }
    } else if (e < 32) {
      const int kh = e >> 4, ii = e & 15, r = (ii & 3) + 8 * (ii >> 2) + 4 * kh, pj = 16 * c + (r >> 1);
      if (pj < hid) {
        const int row = (r & 1 ? hid : 0) + pj;
        const float fold = r & 1 ? -0.69314718055994531f : -1.44269504088896341f;
        word = __float_as_uint(ldexpf(fold, -(rep_row_exp(w1, ln_w, wdw, row, Cs, R) + LR_XE)));
      }
    } else if (e < 32 + C) {
      word = __float_as_uint(ldexpf(1.0f, -rep_w2_exp(w2, e - 32, hid)));
    }
    reinterpret_cast<uint32_t*>(out)[i] = word;
  }
}

template <int MT, int CS>
// four waves per SIMD (two workgroups per CU): <= 128 VGPRs; the four-tile instance (C > 96) three
__global__ __launch_bounds__(64 * LR_NW, MT <= 3 ? 4 : 3) void lnb_rep_kernel(LnbRepArgs a) {
  constexpr int NI = rep_images(MT), SLOTF = NI * 256;
  constexpr int DPW = (NI + LR_NW - 1) / LR_NW;   // LDS-DMA instructions per wave per chunk
  constexpr int CI = 4 + 2 * MT;                   // the constants image
  __shared__ __attribute__((aligned(16))) float smem[LR_NSLOT * SLOTF];
  const int lane = threadIdx.x & 63, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int b = (int)(lb / (uint32_t)a.tiles), tile = (int)(lb % (uint32_t)a.tiles);
  const int H = a.H, W = a.W, C = a.C, nch = a.nch;
  const int P = H * W;
  const int p = tile * LR_PX + wave * 32 + (lane & 31);   // this lane's pixel (column of every MFMA block)

  auto issue = [&](int c) {
    float* slot = smem + (c % LR_NSLOT) * SLOTF;
    const char* src = a.pack + (int64_t)min(c, nch - 1) * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int img = min(i * LR_NW + wave, NI - 1);   // surplus waves repeat the last image
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };

  // im2col column of pixel p: n = x / sigma at the 9 replicate-clamped neighbours, k = 9 c + t; this lane
  // half holds k = 16 s + 8 kh + j
  const int pc = min(p, P - 1), py = pc / W, px = pc - py * W;
  const float* xb = a.xs + (int64_t)b * CS * P;
  float nb[9][CS];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = clampi(py + t / 3 - 1, 0, H - 1), xx = clampi(px + t % 3 - 1, 0, W - 1);
    float v[CS], sum = 0.f;
#pragma unroll
    for (int c = 0; c < CS; ++c) {
      v[c] = xb[(int64_t)c * P + yy * W + xx];
      sum += v[c];
    }
    const float mean = sum / (float)CS;
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < CS; ++c) {
      const float d = v[c] - mean;
      sq += d * d;
    }
    const float rstd = 1.0f / sqrtf(sq / a.var_den + 1e-5f);
#pragma unroll
    for (int c = 0; c < CS; ++c) nb[t][c] = v[c] * rstd;   // x / sigma (REF:921)
  }
  // the entry of either lane half is a compile-time (c, t); one select per entry
  auto im2col = [&](int k) -> float {
    if (k >= 9 * CS) return 0.f;
    return nb[k % 9][k / 9];
  };
  float nv[2][8];
  float mx = 0.f;
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = kh ? im2col(16 * s2 + 8 + j) : im2col(16 * s2 + j);
      nv[s2][j] = v;
      mx = fmaxf(mx, fabsf(v));
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  int ep = LR_XE;
  if (mx != 0.f) {
    int e;
    frexpf(mx, &e);
    if (e > 14 - LR_XE || e < -LR_XE) ep = clampi(14 - e, -100, 100);
  }
  const float corr = ldexpf(1.0f, LR_XE - ep);
  const bool wave_corr = __builtin_amdgcn_readfirstlane((int)__any(ep != LR_XE)) != 0;
  f16x8 xh[2], xl[2];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = ldexpf(nv[s2][j], ep);
      const _Float16 h0 = (_Float16)v;
      xh[s2][j] = h0;
      xl[s2][j] = (_Float16)(v - (float)h0);
    }

  issue(0);
  issue(1);
  issue(2);

  // GEMM1 of chunk c (LN, W1, depthwise in one accumulation), from its ring slot
  auto gemm1 = [&](int c) -> f32x16 {
    const float* slot = smem + (c % LR_NSLOT) * SLOTF + lane * 4;
    f32x16 acc = f32x16{};
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(slot + (2 * s2 + 0) * 256);
      const f16x8 al = *reinterpret_cast<const f16x8*>(slot + (2 * s2 + 1) * 256);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl[s2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh[s2], acc, 0, 0, 0);
    }
    return acc;
  };

  // chunk 0 landed (this wave's DMAs; after them chunks 1 and 2's), then every wave's
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * DPW) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  f32x16 acc2[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc2[t] = f32x16{};
  int E = 1000;                                     // the pixel's GEMM2 scale exponent (none yet)

  // gate of the chunk whose GEMM1 accumulator is acc (ring slot of chunk c), then its GEMM2
  auto gate_gemm2 = [&](int c, f32x16 acc) {
    if (wave_corr) acc *= corr;
    // gate sigmoid(m) m v (REF:947) on the accumulator: registers 2q, 2q + 1 = mask, value of chunk pair
    // 4 (q >> 1) + (q & 1) + 2 kh; the row constants undo the scales and carry the exp2 fold
    const float* cslot = smem + (c % LR_NSLOT) * SLOTF;
    const float* cst = cslot + CI * 256 + kh * 16;
    float gq[8];
    float gm = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float m = acc[2 * q] * cst[2 * q], v = acc[2 * q + 1] * cst[2 * q + 1];
      gq[q] = (m * v) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(m));
      gm = fmaxf(gm, fabsf(gq[q]));
    }
    // the pixel's running exponent: largest |g| so far into [2^13, 2^14); lowering it scales the
    // accumulated sums down by the exact power of two
    gm = fmaxf(gm, __shfl_xor(gm, 32));
    int eg = E;
    if (gm != 0.f) {
      int e;
      frexpf(gm, &e);
      eg = min(E, clampi(14 - e, -100, 100));
    }
    if (__builtin_amdgcn_readfirstlane((int)__any(eg != E && E != 1000)) != 0) {
      const float f = E != 1000 ? ldexpf(1.0f, eg - E) : 1.0f;
#pragma unroll
      for (int t = 0; t < MT; ++t) acc2[t] *= f;
    }
    E = eg;
    const int Eu = E == 1000 ? 0 : E;
    f16x8 gh, gl;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float v = ldexpf(gq[q], Eu);
      const _Float16 h0 = (_Float16)v;
      gh[q] = h0;
      gl[q] = (_Float16)(v - (float)h0);
    }
    // GEMM2: W2 (k permuted to the accumulator's pair order) g, three products of two-term splits
    const float* slot = cslot + lane * 4;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(slot + (4 + 2 * t + 0) * 256);
      const f16x8 al = *reinterpret_cast<const f16x8*>(slot + (4 + 2 * t + 1) * 256);
      acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, gh, acc2[t], 0, 0, 0);
      acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gl, acc2[t], 0, 0, 0);
      acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gh, acc2[t], 0, 0, 0);
    }
  };

  // (Measured on the bench shape, round 4: staggering the two waves of a SIMD -- half of them running
  // gate(c), GEMM2(c), GEMM1(c + 1) -- spills at the 128-VGPR bound of four waves per SIMD, and GEMM1 of
  // chunk c + 1 beside the gate of chunk c fits only three waves per SIMD: 1.73 ms against 1.52.)
  for (int c = 0; c < nch; ++c) {
    // chunk c + 1 landed (this wave's DMAs; after them only chunk c + 2's), then every wave's
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DPW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(c + 3);                                   // slot (c + 3) % 4 was last read in iteration c - 1
    gate_gemm2(c, gemm1(c));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue (REF:962-964): out[m, p] = skip0 x[m mod Cs, p] + skip1 (W2 g)[m, p] 2^-(s2_row + E).  Row m =
  // 32 t + (i & 3) + 8 (i >> 2) + 4 kh: the wave-uniform part in soffset, the lane's 4 kh rows and its
  // pixel in voffset (out of range past the image's pixels).  The W2 row scales come from the last
  // chunk's slot (every slot holds them).
  const float* rs2 = smem + ((nch - 1) % LR_NSLOT) * SLOTF + CI * 256 + 32;
  const float s0 = a.skip[0], s1 = a.skip[1] * ldexpf(1.0f, E == 1000 ? 0 : -E);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)b * C * P, 0,
                                                                        (int)((int64_t)C * P * 4), 0x00020000);
  float xo[CS];
#pragma unroll
  for (int c = 0; c < CS; ++c) xo[c] = xb[(int64_t)c * P + pc];
  const uint32_t vb = p < P ? (uint32_t)(4 * kh * P + p) * 4u : 0x80000000u;
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m0 = 32 * t + (i & 3) + 8 * (i >> 2);          // row of lane half 0; lane half 1: m0 + 4
      const float xv = kh ? xo[(m0 + 4) % CS] : xo[m0 % CS];   // source channel of replica row m
      const float r2 = rs2[min(m0 + 4 * kh, C - 1)];
      const uint32_t vo = m0 + 4 < C ? vb : (m0 < C && !kh ? vb : 0x80000000u);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0 * xv + s1 * (acc2[t][i] * r2)), ors, vo, m0 * P * 4, 0);
    }
}

// ---------------------------------------------------------------------------
// fused16: the whole block for C <= 96 in one pass -- LN + W1 + depthwise 3x3 + gate + W2 + skip --
// with the gated activation kept on chip (no g round trip through HBM, no mix launch).
//
// Persistent, wave-specialised workgroups (8 waves, one workgroup per CU, 148 KB of LDS): waves 0-3 are
// producers, waves 4-7 consumers; wave w and w + 4 share a SIMD.  A tile is 32 output columns x 8 output
// rows with its 34 x 10 halo (340 pixels in 11 blocks of 32); hidden channels go in chunks of 16 (mask,
// value) pairs.  A workgroup walks its tiles' chunks as one sequence of steps; step i:
//   producers  GEMM1 of step i's (tile, chunk) (v_mfma_f32_32x32x16_f16 on exact two-term fp16 splits,
//              head16's arithmetic and scaling; x / sigma of the wave's halo blocks in registers, loaded,
//              normalised and split at the tile's first chunk) -> the chunk's h planes in LDS buffer i & 1;
//   consumers  depthwise 3x3 + gate of step i - 1 (buffer (i - 1) & 1) in the GEMM2 B-operand layout:
//              lane = (column l % 32, pair half l / 32), two output rows per wave, the half's 8 pairs in
//              turn (taps from the ring, the same for a lane half; the window of both rows' pixels, 4 x 3
//              h pairs, read once); GEMM2 (W2 g, v_mfma_f32_32x32x16_f16, two-term fp16 splits) with rep's
//              running per-pixel exponent (largest |g| so far into [2^13, 2^14); a lower one scales the
//              pixel's accumulators down exactly); the W2 accumulators (2 rows x MT tiles) stay in the
//              consumer's registers over the tile's chunks; after the tile's last chunk the epilogue
//              out = skip0 x + skip1 2^-(s2_row + E) acc, while the producers already load the next tile;
//   one barrier; the W1 / W2 fragments and taps of step i + 1 arrive by LDS-DMA in a 3-slot ring meanwhile.
// With a gate buffer given (training's kept gate) the consumers also store g [B, hid, H, W] (fp32).
// Against head16 + mix: no g write + read (2 KB per pixel at hid 256), half the GEMM2 products (fp16
// two-term instead of the bf16 three-term split), one launch, and the x prologue / output epilogue of a
// tile overlap the other role's work.
constexpr int LF_TW = 32;                   // output columns per tile
constexpr int LF_TH = 8;                    // output rows per tile (2 per consumer wave)
constexpr int LF_HWD = LF_TW + 2;           // halo columns
constexpr int LF_HR = LF_TH + 2;            // halo rows
constexpr int LF_NQ = LF_HWD * LF_HR;       // halo pixels (340)
constexpr int LF_NBLK = (LF_NQ + 31) / 32;  // 32-pixel GEMM1 blocks (11)
constexpr int LF_PP = 2 * LF_NBLK * 32;     // floats per pair plane (m, v interleaved)
constexpr int LF_HBUF = 16 * LF_PP;         // floats per h buffer
constexpr int LF_NSLOT = 3;                 // ring slots (step i + 1 loading, GEMM1(i), GEMM2(i - 1))
constexpr int LF_XE = 10;                   // common power-of-two scale of the fp16 x operand
// h planes and taps in pair duos: per halo pixel the (mask, value) of pairs 2d, 2d + 1 in 16 bytes, as GEMM1's
// accumulator holds them (registers 4q .. 4q + 3 = pairs 4q + 2 kh, + 1), so the gate reads its window and taps
// as ds_read_b128 -- 21 reads per two pairs; one pair at a time took 2 x (12 ds_read_b64 + 5): 64 x 256^2
// 3.71 -> 3.67 ms (with the b64 reads merged into ds_read2_b64, which run at half the LDS rate: 3.76)
constexpr int LF_DSTR = 36;                 // tap floats per duo: 9 taps x (m_a, v_a, m_b, v_b)
constexpr int LF_TAPS = 8 * LF_DSTR;        // tap floats per chunk (two 1-KB images)
__host__ __device__ constexpr int fused_images(int KS, int MT) { return 2 * KS + 2 * MT + 2; }

struct LnbFusedArgs {
  const float* x;        // [B, C, H, W]
  const char* pack;      // [nch][fused_images] 1-KB images: W1 frags (hi, lo per k-step), W2 frags (hi, lo per
                         // row tile), taps ([pair][tap][mask, value], scaled and exp2-folded)
  const float* r2;       // [C]: 2^-s2_row
  const float* skip;     // [2]
  float* out;            // [B, C, H, W]
  float* g;              // [B, hid, H, W] or nullptr
  float var_den;
  int C, hid, H, W, tiles_x, tiles_y, nch, ntiles;
};

// W1 images as lnb_w1_pack16_kernel's (rows 2^s_row-scaled, fp16 hi / lo); W2 images: row tile t, term q,
// lane l, element j: m = 32 t + (l & 31), k = 8 (l >> 5) + j = pair 16 c + k, W2[m][16 c + k] 2^s2_row(m);
// taps as head16's (2^-(s_row + XE), exp2 fold); r2[m] = 2^-s2_row(m)
__global__ void lnb_fused_pack_kernel(const float* __restrict__ w1, const float* __restrict__ ln_w,
                                      const float* __restrict__ wdw, const float* __restrict__ w2,
                                      char* __restrict__ pack, float* __restrict__ r2, int C, int hid, int KS,
                                      int MT, int nch) {
  const int NI = fused_images(KS, MT);
  const int64_t n_img = (int64_t)nch * NI * 256;
  const int64_t n = n_img + C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (i >= n_img) {
      const int m = (int)(i - n_img);
      r2[m] = ldexpf(1.0f, -rep_w2_exp(w2, m, hid));
      continue;
    }
    const int64_t img = i >> 8;
    const int e = (int)(i & 255), c = (int)(img / NI), im = (int)(img % NI), l = e >> 2;
    uint32_t word = 0;
    if (im < 2 * KS) {
      const int q = im & 1, s = im >> 1, r = l & 31, pj = 16 * c + (r >> 1);
      if (pj < hid) {
        const int row = (r & 1 ? hid : 0) + pj;
        const int sc = head16_row_exp(w1, ln_w, row, C, 1);
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int k = 16 * s + 8 * (l >> 5) + 2 * (e & 3) + u;
          v[u] = k < C ? ldexpf(w1[(int64_t)row * C + k] * ln_w[k], sc) : 0.f;
        }
        word = f16_pair_word(v[0], v[1], q);
      }
    } else if (im < 2 * KS + 2 * MT) {
      const int t = (im - 2 * KS) >> 1, q = (im - 2 * KS) & 1, m = 32 * t + (l & 31);
      if (m < C) {
        const int sc = rep_w2_exp(w2, m, hid);
        float v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int pj = 16 * c + 8 * (l >> 5) + 2 * (e & 3) + u;
          v[u] = pj < hid ? ldexpf(w2[(int64_t)m * hid + pj], sc) : 0.f;
        }
        word = f16_pair_word(v[0], v[1], q);
      }
    } else {
      const int r = (im - 2 * KS - 2 * MT) * 256 + e;
      if (r < LF_TAPS) {
        const int w = 2 * (r / LF_DSTR) + ((r >> 1) & 1), t = (r % LF_DSTR) >> 2, comp = r & 1, pj = 16 * c + w;
        if (pj < hid && t < 9) {
          const int row = (comp ? hid : 0) + pj;
          const float fold = comp ? -0.69314718055994531f : -1.44269504088896341f;
          word = __float_as_uint(ldexpf(wdw[(int64_t)row * 9 + t], -(head16_row_exp(w1, ln_w, row, C, 1) + LF_XE)) *
                                 fold);
        }
      }
    }
    reinterpret_cast<uint32_t*>(pack)[i] = word;
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const float* const_f32_t;
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
// exact two-term fp16 split of (a, b) with packed round-to-nearest conversions (v_cvt_pk_f16_f32): hi, lo
__device__ __forceinline__ void split2_f16(float a, float b, uint32_t& hi, uint32_t& lo) {
  const f32x2v v = f32x2v{a, b};
  const f16x2 h = __builtin_convertvector(v, f16x2);
  const f16x2 l = __builtin_convertvector(v - __builtin_convertvector(h, f32x2v), f16x2);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, l);
}
// consumer mapping: lane per (column, pair half), two rows per lane, taps from the LDS ring (a lane per
// pixel with scalar taps and B operands by v_permlane32_swap measured slower)

// timing-only diagnostic builds (wrong results): 1 = consumers skip their work, 2 = producers skip theirs,
// 8 = the gate without its exp / rcp
#ifndef GRR_FUSED_DIAG
#define GRR_FUSED_DIAG 0
#endif
// GRR_FUSED_STAMP=1: diagnostic build -- each wave sums s_memtime deltas of its phases (producer: DMA issue,
// x prologue, GEMM1, h stores, wait, barrier; consumer: DMA issue, gate, GEMM2, epilogue, wait, barrier)
// into g_fused_stamps[workgroup][wave][phase] (grr_lnb_fused_stamps copies them out)
#ifndef GRR_FUSED_STAMP
#define GRR_FUSED_STAMP 0
#endif
#if GRR_FUSED_STAMP
__device__ unsigned long long g_fused_stamps[1024 * 8 * 8];
#define FSTAMP(k)                                              \
  do {                                                         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_prev;                                 \
    st_prev = t_;                                              \
  } while (0)
#else
#define FSTAMP(k) \
  do {            \
  } while (0)
#endif

// tile t of the launch -> (b, ty, tx): consecutive tiles of a workgroup walk along rows of one image
struct FusedTile {
  int b, y0, x0;
};
__device__ __forceinline__ FusedTile fused_tile(const LnbFusedArgs& a, int t) {
  const int tx = t % a.tiles_x, r = t / a.tiles_x;
  return FusedTile{r / a.tiles_y, (r % a.tiles_y) * LF_TH, tx * LF_TW};
}

// IO: bit 0 -- x (and the skip operand) in the channel-blocked layout [B][NB][H][W][8] (NB = ceil(C / 8), the
// pad channels 0; grr_lnb_forward_c8), bit 1 -- out in it; else [B, C, H, W].  The blocked layout serves the
// kernel's memory instructions: the producer's 8 channels of a pixel per k-step are 32 contiguous bytes (two
// dwordx4 loads instead of eight dword loads) and the consumer's four consecutive accumulator rows of a pixel
// are 16 contiguous bytes (one dwordx4 load / store instead of four).  Measured per 64 x 256^2 block: blocked
// input 3.91 -> 3.74 ms, blocked output unchanged.  Same values in the same registers
// either way: the results are bitwise equal.
template <int KS, int MT, int IO>
__global__ __launch_bounds__(512, 1) void lnb_fused16_kernel(LnbFusedArgs a) {
  constexpr bool IN8 = (IO & 1) != 0, OUT8 = (IO & 2) != 0;
  constexpr int NI = fused_images(KS, MT), SLOTF = NI * 256;
  constexpr int DPW = (NI + 7) / 8;      // LDS-DMA instructions per wave per step
  __shared__ __attribute__((aligned(16))) float smem[2 * LF_HBUF + LF_NSLOT * SLOTF + 32 * MT];
  float* const ring = smem + 2 * LF_HBUF;
  float* const r2s = ring + LF_NSLOT * SLOTF;    // 2^-s2_row of the W2 rows (0 past C)

  const int tid = threadIdx.x, lane = tid & 63, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, W = a.W, C = a.C, hid = a.hid, nch = a.nch;
  if (tid < 32 * MT) r2s[tid] = tid < C ? a.r2[tid] : 0.f;   // read after the first barrier
  const int HW = H * W;
  // the workgroup's tiles: blockIdx.x, + gridDim.x, ...; steps = tiles x chunks (+ 1: the last gate)
  const int G = gridDim.x, wg = blockIdx.x;
  const int my_tiles = wg < a.ntiles ? (a.ntiles - wg + G - 1) / G : 0;
  const int nsteps = my_tiles * nch;

  // the chunk `chunk` into ring slot `sl` (the offsets recomputed per call: hoisted out of the step loop
  // they would hold 2 DPW x 3 SGPRs for the whole kernel)
  auto issue = [&](int sl, int chunk) {
    int sv = __builtin_amdgcn_readfirstlane(sl), cv = __builtin_amdgcn_readfirstlane(chunk), wv = wave;
    asm volatile("" : "+s"(sv), "+s"(cv), "+s"(wv));
    float* slot = ring + sv * SLOTF;
    const char* src = a.pack + (int64_t)cv * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int img = min(i * 8 + wv, NI - 1);   // surplus waves repeat the last image
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };
  // step counters without divisions: (chunk, ring slot) of the next step's DMA
  int dch = nch > 1 ? 1 : 0, dsl = 1;
  auto advance_dma = [&]() {
    dch = dch + 1 == nch ? 0 : dch + 1;
    dsl = dsl == LF_NSLOT - 1 ? 0 : dsl + 1;
  };
  if (nsteps == 0) return;   // workgroup-uniform: no barrier is left waiting
#if GRR_FUSED_STAMP
  unsigned long long st_acc[8] = {}, st_prev = __builtin_amdgcn_s_memtime();
  auto stamp_out = [&]() {
    if (lane < 8 && blockIdx.x < 1024) {
      unsigned long long v = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) v = lane == k ? st_acc[k] : v;
      g_fused_stamps[(blockIdx.x * 8 + wave) * 8 + lane] = v;
    }
  };
#endif
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  if (wave < 4) {
    // ---------------- producer: GEMM1 of the halo blocks wave, wave + 4, wave + 8 (< LF_NBLK)
    constexpr int NBW = (LF_NBLK + 3) / 4;
    const bool has_last = wave + 4 * (NBW - 1) < LF_NBLK;   // wave-uniform
    f16x8 xh[NBW][KS], xl[NBW][KS];
    float corr[NBW];
    bool wave_corr = false;
    int c = 0, tile = wg, sl = 0;                  // step i's chunk, tile and ring slot
    for (int i = 0; i <= nsteps; ++i) {
      issue(dsl, dch);                             // slot of step i + 1 last served step i - 2 (steps i - 2, i - 1)
      advance_dma();
      FSTAMP(0);
      if (i < nsteps && !(GRR_FUSED_DIAG & 2)) {
        if (c == 0) {
          // the tile's halo pixels: raw x, LayerNorm statistics (REF:916-922), x / sigma split in fp16 terms
          const FusedTile T = fused_tile(a, tile);
          // x of the image through a buffer descriptor: channel 16 s + 8 kh + j of the lane's pixel at
          // voffset (pixel + 8 kh HW) 4 + soffset (16 s + j) HW 4 -- the uniform part in an SGPR, no
          // per-element address arithmetic -- and channels >= C past num_records read as 0
          const int cx = IN8 ? 8 * ((C + 7) / 8) : C;   // channels of one image in x (blocked: the pads too)
          const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(a.x + (int64_t)T.b * cx * HW), 0, (int)((int64_t)cx * HW * 4), 0x00020000);
          bool any_corr = false;
#pragma unroll
          for (int k = 0; k < NBW; ++k) {
            const int q = min((wave + 4 * k) * 32 + (lane & 31), LF_NQ - 1);
            const int hy = q / LF_HWD, hx = q - hy * LF_HWD;
            const int gy = clampi(T.y0 - 1 + hy, 0, H - 1), gx = clampi(T.x0 - 1 + hx, 0, W - 1);
            const int vo = (8 * kh * HW + gy * W + gx) * 4;
            // (a copy per block the compiler cannot see through: otherwise it hoists the 8 KS soffsets out
            // of the step loop and holds them in SGPRs for the whole kernel)
            int hw4 = HW * 4;
            asm volatile("" : "+s"(hw4));
            float xv[KS][8];
            if constexpr (IN8) {
              // blocked: channels 16 s + 8 kh + j = block 2 s + kh, lane j of it -- 32 bytes at voffset
              // (kh HW + pixel) 32 + soffset 2 s HW 32; blocks >= NB past num_records read as 0
              const uint32_t vo8 = (uint32_t)((kh * HW + gy * W + gx) * 32);
#pragma unroll
              for (int s = 0; s < KS; ++s) {
                const u32x4 lo = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo8, 16 * s * hw4, 0));
                const u32x4 hi = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo8 + 16, 16 * s * hw4, 0));
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  xv[s][j] = __uint_as_float(lo[j]);
                  xv[s][4 + j] = __uint_as_float(hi[j]);
                }
              }
            } else {
#pragma unroll
              for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j)
                  xv[s][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, (16 * s + j) * hw4, 0));
            }
            float sum = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
              for (int j = 0; j < 8; ++j) sum += xv[s][j];
            sum += __shfl_xor(sum, 32);
            const float mean = sum / (float)C;
            float sq = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const float d = 16 * s + 8 * kh + j < C ? xv[s][j] - mean : 0.f;
                sq += d * d;
              }
            sq += __shfl_xor(sq, 32);
            const float rstd = 1.0f / sqrtf(sq / a.var_den + 1e-5f);
            float mx = 0.f;
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                xv[s][j] *= rstd;                       // x / sigma (REF:921)
                mx = fmaxf(mx, fabsf(xv[s][j]));
              }
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            int ep = LF_XE;
            if (mx != 0.f) {
              int e;
              frexpf(mx, &e);
              if (e > 14 - LF_XE || e < -LF_XE) ep = clampi(14 - e, -100, 100);
            }
            corr[k] = ldexpf(1.0f, LF_XE - ep);
            any_corr |= ep != LF_XE;
#pragma unroll
            for (int s = 0; s < KS; ++s) {
              uint32_t hw[4], lw[4];
#pragma unroll
              for (int j = 0; j < 4; ++j)
                split2_f16(ldexpf(xv[s][2 * j], ep), ldexpf(xv[s][2 * j + 1], ep), hw[j], lw[j]);
              xh[k][s] = __builtin_bit_cast(f16x8, u32x4{hw[0], hw[1], hw[2], hw[3]});
              xl[k][s] = __builtin_bit_cast(f16x8, u32x4{lw[0], lw[1], lw[2], lw[3]});
            }
          }
          wave_corr = __builtin_amdgcn_readfirstlane((int)__any(any_corr)) != 0;
        }
        FSTAMP(1);
        const float* slot = ring + sl * SLOTF + lane * 4;
        f32x16 acc[NBW];
#pragma unroll
        for (int k = 0; k < NBW; ++k) acc[k] = f32x16{};
        // k-step s's W1 fragments in registers while step s + 1's load (the scheduling barrier keeps the
        // compiler from reading every k-step's fragments up front: 8 KS registers on top of the x operands)
        f16x8 ah = *reinterpret_cast<const f16x8*>(slot);
        f16x8 al = *reinterpret_cast<const f16x8*>(slot + 256);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          f16x8 bh, bl;
          if (s + 1 < KS) {
            bh = *reinterpret_cast<const f16x8*>(slot + (2 * s + 2) * 256);
            bl = *reinterpret_cast<const f16x8*>(slot + (2 * s + 3) * 256);
          }
#pragma unroll
          for (int k = 0; k < NBW; ++k) {
            if (k == NBW - 1 && !has_last) continue;
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh[k][s], acc[k], 0, 0, 0);
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl[k][s], acc[k], 0, 0, 0);
            acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh[k][s], acc[k], 0, 0, 0);
          }
          if (s + 1 < KS) {
            ah = bh;
            al = bl;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        FSTAMP(2);
        float* hb = smem + (i & 1) * LF_HBUF;
#pragma unroll
        for (int k = 0; k < NBW; ++k) {
          if (k == NBW - 1 && !has_last) continue;
          if (wave_corr) acc[k] *= corr[k];
          const int q = (wave + 4 * k) * 32 + (lane & 31);
          // registers 4u .. 4u + 3 = rows 8 u + 4 kh .. + 3: (mask, value) of pairs 4 u + 2 kh, + 1 = duo 2 u + kh
#pragma unroll
          for (int u = 0; u < 4; ++u)
            *reinterpret_cast<f32x4*>(hb + (2 * u + kh) * 2 * LF_PP + 4 * q) =
                f32x4{acc[k][4 * u], acc[k][4 * u + 1], acc[k][4 * u + 2], acc[k][4 * u + 3]};
        }
        if (++c == nch) {
          c = 0;
          tile += G;
        }
        sl = sl == LF_NSLOT - 1 ? 0 : sl + 1;
      }
      FSTAMP(3);
      // step i + 1's chunk landed (this wave's DMAs), h(i) written; then every wave's
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      FSTAMP(4);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      FSTAMP(5);
    }
#if GRR_FUSED_STAMP
    stamp_out();
#endif
    return;
  }

  // ---------------- consumer: depthwise + gate + GEMM2 of output rows 2 cw, 2 cw + 1 of the tile
  __builtin_amdgcn_s_setprio(1);   // the VALU-bound role first at the SIMD's issue arbiter (3 % at 256^2, 128^2)
  const int cw = wave - 4;
  const int col = lane & 31;
  f32x16 acc2[2][MT];
  int E[2] = {1000, 1000};                           // the column pixel's GEMM2 scale exponent per row (none yet)
  int ch = 0, ctile = wg, csl = 0;                   // step i - 1's chunk, tile and ring slot
  for (int i = 0; i <= nsteps; ++i) {
    issue(dsl, dch);
    advance_dma();
    FSTAMP(0);
    if (i >= 1 && !(GRR_FUSED_DIAG & 1)) {
      const int st = i - 1;
      if (ch == 0) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
#pragma unroll
          for (int t = 0; t < MT; ++t) acc2[rb][t] = f32x16{};
          E[rb] = 1000;
        }
      }
      const float* slot = ring + csl * SLOTF;
      const FusedTile T = fused_tile(a, ctile);
      const int gxo = T.x0 + col;
      const float* w2s = slot + 2 * KS * 256 + lane * 4;
      float g[2][8];
      // the gate, a pair duo at a time (taps and window of both output rows as 16-byte reads): the window is
      // halo rows 2 cw .. 2 cw + 3, columns col .. col + 2; the two planes' depthwise sums of both pairs run
      // as packed FMA chains (v_pk_fma_f32: the same fp32 fma per component)
      // duo dd = pairs 8 kh + 2 dd, + 1
      const float* hwin4 = smem + (st & 1) * LF_HBUF + 4 * kh * 2 * LF_PP + 4 * (2 * cw * LF_HWD + col);
      const float* tapd = slot + (2 * KS + 2 * MT) * 256 + 4 * kh * LF_DSTR;
      // Software-pipelined over (duo, tap row): stage r of a duo adds tap row r's products with window rows r
      // (output row 0) and r + 1 (output row 1) -- the same fma order as all nine taps at once -- while the
      // next stage's 16-byte reads (tap row r + 1 and window row r + 2, or the next duo's tap row 0 and window
      // rows 0, 1) are in flight: <= 80 registers live, no read waits behind more than 9 newer ones.  (A duo at
      // a time with all 21 reads up front: 3.53 ms at 64 x 256^2, this 3.48; the next duo's reads in flight
      // beside the current duo's spill at the 256-register bound)
      f32x4 tc[4][9], wc[4][12];
      auto ld_taps = [&](int dd, int r) __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < 3; ++x) tc[dd][3 * r + x] = *reinterpret_cast<const f32x4*>(tapd + dd * LF_DSTR + 4 * (3 * r + x));
      };
      auto ld_row = [&](int dd, int r) __attribute__((always_inline)) {
#pragma unroll
        for (int x = 0; x < 3; ++x)
          wc[dd][3 * r + x] = *reinterpret_cast<const f32x4*>(hwin4 + dd * 2 * LF_PP + 4 * (r * LF_HWD + x));
      };
      auto gate2 = [&](const f32x4& mv, int rb, int dd) __attribute__((always_inline)) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          // m' = -log2(e) m, v' = -ln(2) v (the taps' fold): sigmoid(m) m v = m' v' / (1 + 2^m')
          const float m = mv[2 * e], v = mv[2 * e + 1];
          g[rb][2 * dd + e] = (GRR_FUSED_DIAG & 8) ? (m * v) : (m * v) * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(m));
        }
      };
      ld_taps(0, 0);
      ld_row(0, 0);
      ld_row(0, 1);
#pragma unroll
      for (int dd = 0; dd < 4; ++dd) {
        f32x4 mv0, mv1;
        ld_taps(dd, 1);
        ld_row(dd, 2);
        __builtin_amdgcn_sched_barrier(0);
        mv0 = tc[dd][0] * wc[dd][0];
        mv1 = tc[dd][0] * wc[dd][3];
#pragma unroll
        for (int x = 1; x < 3; ++x) {
          mv0 = __builtin_elementwise_fma(tc[dd][x], wc[dd][x], mv0);
          mv1 = __builtin_elementwise_fma(tc[dd][x], wc[dd][3 + x], mv1);
        }
        __builtin_amdgcn_sched_barrier(0);
        ld_taps(dd, 2);
        ld_row(dd, 3);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          mv0 = __builtin_elementwise_fma(tc[dd][3 + x], wc[dd][3 + x], mv0);
          mv1 = __builtin_elementwise_fma(tc[dd][3 + x], wc[dd][6 + x], mv1);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (dd < 3) {
          ld_taps(dd + 1, 0);
          ld_row(dd + 1, 0);
          ld_row(dd + 1, 1);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int x = 0; x < 3; ++x) {
          mv0 = __builtin_elementwise_fma(tc[dd][6 + x], wc[dd][6 + x], mv0);
          mv1 = __builtin_elementwise_fma(tc[dd][6 + x], wc[dd][9 + x], mv1);
        }
        gate2(mv0, 0, dd);
        gate2(mv1, 1, dd);
        __builtin_amdgcn_sched_barrier(0);
      }
      FSTAMP(1);
      if (a.g) {   // kept gate (training): the unscaled fp32 values, [B, hid, H, W]
        float* gb = a.g + (int64_t)T.b * hid * HW;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int yy = T.y0 + 2 * cw + rb;
          if (yy < H && gxo < W) {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              const int pj = 16 * ch + 8 * kh + jj;
              if (pj < hid) gb[(int64_t)pj * HW + yy * W + gxo] = g[rb][jj];
            }
          }
        }
      }
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        // the pixel's running exponent: largest |g| over the chunk's 16 pairs (both lane halves) into
        // [2^13, 2^14); a lower one scales the pixel's accumulated sums down by the exact power of two
        float gm = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) gm = fmaxf(gm, fabsf(g[rb][jj]));
        const auto gs = __builtin_amdgcn_permlane32_swap(__float_as_uint(gm), __float_as_uint(gm), false, false);
        gm = fmaxf(__uint_as_float(gs[0]), __uint_as_float(gs[1]));
        int eg = E[rb];
        if (gm != 0.f) {
          int e;
          frexpf(gm, &e);
          eg = min(E[rb], clampi(14 - e, -100, 100));
        }
        if (__builtin_amdgcn_readfirstlane((int)__any(eg != E[rb] && E[rb] != 1000)) != 0) {
          const float f = E[rb] != 1000 ? ldexpf(1.0f, eg - E[rb]) : 1.0f;
#pragma unroll
          for (int t = 0; t < MT; ++t) acc2[rb][t] *= f;
        }
        E[rb] = eg;
        const int Eu = eg == 1000 ? 0 : eg;
        f16x8 gh, gl;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const float v = ldexpf(g[rb][jj], Eu);
          const _Float16 h0 = (_Float16)v;
          gh[jj] = h0;
          gl[jj] = (_Float16)(v - (float)h0);
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const f16x8 ah = *reinterpret_cast<const f16x8*>(w2s + (2 * t + 0) * 256);
          const f16x8 al = *reinterpret_cast<const f16x8*>(w2s + (2 * t + 1) * 256);
          acc2[rb][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, gh, acc2[rb][t], 0, 0, 0);
          acc2[rb][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gl, acc2[rb][t], 0, 0, 0);
          acc2[rb][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gh, acc2[rb][t], 0, 0, 0);
        }
      }
      FSTAMP(2);
      if (ch == nch - 1) {
        // epilogue (REF:962-964): out[m, p] = skip0 x[m, p] + skip1 2^-E_p r2[m] acc; accumulator block rb
        // holds output row 2 cw + rb, column lane % 32, rows m = 32 t + (i & 3) + 8 (i >> 2) + 4 kh
        const float s0 = a.skip[0], s1 = a.skip[1];
        // skip operand and output through buffer descriptors: row m = 32 t + (u & 3) + 8 (u >> 2) + 4 kh of
        // the lane's pixel at voffset (pixel + 4 kh HW) 4 + soffset (32 t + (u & 3) + 8 (u >> 2)) HW 4; rows
        // >= C fall past num_records (loads 0, stores dropped), pixels outside the image take an
        // out-of-range voffset
        const int c8 = 8 * ((C + 7) / 8);
        const int cx = IN8 ? c8 : C, co = OUT8 ? c8 : C;
        const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.x + (int64_t)T.b * cx * HW), 0, (int)((int64_t)cx * HW * 4), 0x00020000);
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)T.b * co * HW, 0,
                                                                              (int)((int64_t)co * HW * 4), 0x00020000);
        const int Eb[2] = {E[0], E[1]};
        // the W2 row scales and 2^-E into the accumulators first, then every skip operand of both rows in one
        // round of loads (the gate's registers are dead here: acc2 + 2 MT x 16 fit), then the stores
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const float sc = s1 * ldexpf(1.0f, Eb[rb] == 1000 ? 0 : -Eb[rb]);
#pragma unroll
          for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int u = 0; u < 16; ++u) acc2[rb][t][u] *= sc * r2s[32 * t + (u & 3) + 8 * (u >> 2) + 4 * kh];
        }
        __builtin_amdgcn_sched_barrier(0);
        int hw4 = __builtin_amdgcn_readfirstlane(HW * 4);   // (not hoisted: see the producer's x loads)
        asm volatile("" : "+s"(hw4));
        // NCHW: row m at voffset (pixel + 4 kh HW) 4 + soffset (32 t + (u & 3) + 8 (u >> 2)) HW 4; blocked: rows
        // 32 t + 8 q + 4 kh + 0..3 (u = 4 q + 0..3) are block 4 t + q, lanes 4 kh .. 4 kh + 3 of the pixel --
        // 16 bytes at voffset pixel 32 + 16 kh + soffset (4 t + q) HW 32
        uint32_t vx[2], vo[2], vx8[2], vo8[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
          const int yy = T.y0 + 2 * cw + rb;
          const uint32_t pix = (uint32_t)(min(yy, H - 1) * W + min(gxo, W - 1));
          const bool in = yy < H && gxo < W;
          vx[rb] = (uint32_t)(4 * kh * HW + pix) * 4u;
          vo[rb] = in ? vx[rb] : 0x80000000u;
          vx8[rb] = pix * 32u + 16u * kh;
          vo8[rb] = in ? vx8[rb] : 0x80000000u;
        }
        float xv[2][MT][16];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            if constexpr (IN8) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const u32x4 v = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, vx8[rb], (4 * t + q) * 8 * hw4, 0));
#pragma unroll
                for (int r = 0; r < 4; ++r) xv[rb][t][4 * q + r] = __uint_as_float(v[r]);
              }
            } else {
#pragma unroll
              for (int u = 0; u < 16; ++u)
                xv[rb][t][u] = __uint_as_float(
                    __builtin_amdgcn_raw_buffer_load_b32(xrs, vx[rb], (32 * t + (u & 3) + 8 * (u >> 2)) * hw4, 0));
            }
          }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
          for (int t = 0; t < MT; ++t) {
            if constexpr (OUT8) {
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                u32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = __float_as_uint(s0 * xv[rb][t][4 * q + r] + acc2[rb][t][4 * q + r]);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b128(
                                                           ors, 0, 0, 0)), v),
                                                       ors, vo8[rb], (4 * t + q) * 8 * hw4, 0);
              }
            } else {
#pragma unroll
              for (int u = 0; u < 16; ++u)
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0 * xv[rb][t][u] + acc2[rb][t][u]), ors, vo[rb],
                                                      (32 * t + (u & 3) + 8 * (u >> 2)) * hw4, 0);
            }
          }
      }
      if (++ch == nch) {
        ch = 0;
        ctile += G;
      }
      csl = csl == LF_NSLOT - 1 ? 0 : csl + 1;
    }
    FSTAMP(3);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    FSTAMP(4);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    FSTAMP(5);
  }
#if GRR_FUSED_STAMP
  stamp_out();
#endif
}

#if GRR_FUSED_STAMP
extern "C" int grr_lnb_fused_stamps(unsigned long long* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fused_stamps), sizeof(unsigned long long) * std::min(n, 1024 * 64),
                             0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

// ---------------------------------------------------------------------------
// mix: out = skip0 x + skip1 W2 g
constexpr int LM_NBB = 2;                 // 32-pixel blocks per wave
constexpr int LM_PX = 4 * LM_NBB * 32;    // pixels per workgroup
constexpr int LM_KD = 16;                 // hidden channels per k-step

struct LnbMixArgs {
  const float* g;         // [B, hid, P]
  const char* w2f;        // [KS2][MT][3] fragment images of W2
  const float* x;         // [B, C, P], or [B, xs_c, P] read at channel m mod xs_c when xs_c > 0
  int xs_c;
  const float* skip;      // [2]
  float* out;             // [B, C, P]
  int64_t P;
  int C, hid, KS2, tiles;
  uint32_t nblk;
};

// W2 [C, hid] -> 32x32x16 A fragments.  k-step s, row tile t, term q, lane l, element j:
// m = 32 t + (l & 31), k = 16 s + 8 (l >> 5) + j.
__global__ void lnb_w2_pack_kernel(const float* __restrict__ w2, uint16_t* __restrict__ frag, int C, int hid,
                                   int MT, int KS2) {
  const int64_t n = (int64_t)KS2 * MT * 3 * 512;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i & 7), l = (int)((i >> 3) & 63);
    const int64_t img = i >> 9;
    const int q = (int)(img % 3), t = (int)((img / 3) % MT), s = (int)(img / (3 * MT));
    const int m = 32 * t + (l & 31), k = 16 * s + 8 * (l >> 5) + j;
    frag[i] = (m < C && k < hid) ? split_term(w2[(int64_t)m * hid + k], q) : (uint16_t)0;
  }
}

// A k-step's operands -- the W2 fragment images and the [16][256-pixel] g tile -- arrive by
// LDS-DMA in a 3-slot ring two k-steps ahead.  V4 (P % 4 == 0): one 16-byte DMA per g row.
template <int MT, bool V4>
__global__ __launch_bounds__(256, MT >= 4 ? 1 : 2) void lnb_mix_kernel(LnbMixArgs a) {
  constexpr int NI = MT * 3;
  constexpr int WPW = (NI + 3) / 4;                 // W2 image DMAs per wave per k-step
  constexpr int GPW = V4 ? LM_KD / 4 : LM_KD;       // g DMAs per wave per k-step
  constexpr int DPW = WPW + GPW;
  constexpr int WF = NI * 256;                      // floats of W2 images per slot
  constexpr int SLOTF = WF + LM_KD * LM_PX;
  constexpr int NSLOT = 3;
  __shared__ __attribute__((aligned(16))) float smem[NSLOT * SLOTF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int b = lb / a.tiles, tile = lb - b * a.tiles;
  const int64_t P = a.P;
  const int C = a.C, hid = a.hid, KS2 = a.KS2;
  const int r = lane & 31, hh = lane >> 5;
  const int64_t p0 = (int64_t)tile * LM_PX;

  const float* gb = a.g + (int64_t)b * hid * P;
  // per-lane source column of the g tile (clamped into the image)
  const int64_t gcol = V4 ? min(p0 + 4 * lane, P - 4) : 0;
  auto issue = [&](int s) {
    const int ss = min(s, KS2 - 1);
    float* slot = smem + (s % NSLOT) * SLOTF;
    const char* src = a.w2f + (int64_t)ss * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < WPW; ++i) {
      const int img = min(i * 4 + wave, NI - 1);
      dma16(src + img * 1024, slot + img * 256);
    }
    float* gs = slot + WF;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      if constexpr (V4) {
        const int kr = wave * GPW + i;                       // tile row 0..15
        const int k = min(LM_KD * ss + kr, hid - 1);         // k >= hid: zero W2 columns
        dma16(gb + (int64_t)k * P + gcol, gs + kr * LM_PX);
      } else {
        const int kr = wave * 4 + (i >> 2), part = i & 3;    // 4 dword DMAs per row
        const int k = min(LM_KD * ss + kr, hid - 1);
        const int64_t pc = min(p0 + part * 64 + lane, P - 1);
        __builtin_amdgcn_global_load_lds(gb + (int64_t)k * P + pc, (lds_ptr_t)(gs + kr * LM_PX + part * 64), 4, 0,
                                         0);
      }
    }
  };

  f32x16 acc[MT][LM_NBB];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int nb = 0; nb < LM_NBB; ++nb) acc[t][nb] = f32x16{};

  issue(0);
  issue(1);
  for (int s = 0; s < KS2; ++s) {
    // k-step s landed (this wave's DMAs; after them only step s + 1's), then every wave's
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(DPW) : "memory");
    __builtin_amdgcn_s_barrier();
    issue(s + 2);                                  // slot (s + 2) % 3 was last read in step s - 1
    const float* slot = smem + (s % NSLOT) * SLOTF;
    const float* gs = slot + WF + (8 * hh) * LM_PX + wave * LM_NBB * 32 + r;
    bf16x8 bq[LM_NBB][3];
#pragma unroll
    for (int nb = 0; nb < LM_NBB; ++nb) {
      float gv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = gs[j * LM_PX + nb * 32];
      split3x8(gv, bq[nb][0], bq[nb][1], bq[nb][2]);
    }
    const float* ws = slot + lane * 4;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(ws + (3 * t + 0) * 256);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(ws + (3 * t + 1) * 256);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(ws + (3 * t + 2) * 256);
#pragma unroll
      for (int nb = 0; nb < LM_NBB; ++nb)
        GRR_X3_MFMA(__builtin_amdgcn_mfma_f32_32x32x16_bf16, acc[t][nb], a0, a1, a2, bq[nb][0], bq[nb][1],
                    bq[nb][2]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue (REF:962-964): rows m = 32 t + (i & 3) + 8 (i >> 2) + 4 hh, pixel = lane column;
  // x / out through buffer descriptors (32-bit offsets; rows >= C or pixels >= P not stored)
  const float s0 = a.skip[0], s1 = a.skip[1];
  const int img_bytes = (int)((int64_t)C * P * 4);
  const int XC = a.xs_c > 0 ? a.xs_c : C;   // skip operand: x, or the image x replicates (channel m mod XC)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x + (int64_t)b * XC * P), 0, (int)((int64_t)XC * P * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)b * C * P, 0, img_bytes,
                                                                        0x00020000);
  const int Pi = (int)P;
#pragma unroll
  for (int nb = 0; nb < LM_NBB; ++nb) {
    const int p = (int)p0 + (wave * LM_NBB + nb) * 32 + r;
    const int pc = min(p, Pi - 1);
    // one 32-row tile of x at a time (the skip operand): 16 loads in flight, not MT x 16 live registers
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float xv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = min(32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh, C - 1);
        const int mx = XC == C ? m : m % XC;
        xv[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, (mx * Pi + pc) * 4, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hh;
        const uint32_t off = (m < C && p < Pi) ? (uint32_t)(m * Pi + p) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0 * xv[i] + s1 * acc[t][nb][i]), ors, off, 0, 0);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side
static int head_ks(int C) { return (C + 31) / 32; }
static int head_nb(int KS) { return KS <= 3 ? 4 : 3; }
static int64_t align64(int64_t n) { return (n + 63) / 64 * 64; }
// GEMM1 on the fp16 two-term head (lnb_head16_kernel): C <= 96 (its 2-slot ring + 2 x 64 KB of
// h planes fill the CU's LDS at 6 k-steps); 96 < C <= 128 runs the split-bf16 head (lnb_head_kernel)
static int head16_ks(int C) { return (C + 15) / 16; }
static bool head16_enabled(int C) { return head16_ks(C) <= 6; }
static int64_t head_pack_floats(int C, int hid) {
  const int64_t bf = (int64_t)((hid + LH_JC - 1) / LH_JC) * head_images(head_ks(C)) * 256;
  const int64_t f16 = (int64_t)((hid + L6_NP - 1) / L6_NP) * head16_images(head16_ks(C)) * 256;
  return align64(std::max(bf, f16));
}
static int64_t mix_pack_floats(int C, int hid) {
  return align64((int64_t)((hid + LM_KD - 1) / LM_KD) * ((C + 31) / 32) * 3 * 256);
}

// the fused block (lnb_fused16_kernel): C <= 96 (GEMM1's x of three halo blocks, 6 k-steps, in registers)
int g_lnb_fused_on = 1;   // grr_lnb_set_fused (A/B measurement knob)
bool lnb_fused(int C, int hid) { return g_lnb_fused_on && C >= 2 && C <= 96 && hid >= 1; }
int64_t fused_pack_floats(int C, int hid) {
  const int KS = (C + 15) / 16, MT = (C + 31) / 32, nch = (hid + 15) / 16;
  return align64((int64_t)nch * fused_images(KS, MT) * 256) + align64(C);
}

// workspace (floats): [g: B*hid*P][W1 images][W2 images], each 256-B aligned; the fused block's images,
// taps and W2 row scales where the two-kernel path keeps its W1 images (after the g region, which the
// fused block fills only for grr_lnb_forward_keep)
int64_t lnb_mfma_workspace_floats(int B, int C, int hid, int H, int W) {
  const int64_t two_kernel = align64((int64_t)B * hid * H * W) +
                             std::max(head_pack_floats(C, hid) + mix_pack_floats(C, hid), fused_pack_floats(C, hid));
  const int64_t rep = align64((int64_t)((hid + 15) / 16) * rep_images((C + 31) / 32) * 256);   // lnb_rep_kernel's chunk images
  return std::max(two_kernel, rep);
}

template <int KS, int NB>
static void launch_head(const LnbHeadArgs& h, hipStream_t s) {
  hipLaunchKernelGGL((lnb_head_kernel<KS, NB>), dim3(h.nblk), dim3(512), 0, s, h);
}
template <int KS>
static void launch_head16(const LnbHeadArgs& h, hipStream_t s) {
  hipLaunchKernelGGL((lnb_head16_kernel<KS, 8>), dim3(h.nblk), dim3(512), 0, s, h);
}
template <int MT>
static void launch_mix(const LnbMixArgs& m, bool v4, hipStream_t s) {
  if (v4) hipLaunchKernelGGL((lnb_mix_kernel<MT, true>), dim3(m.nblk), dim3(256), 0, s, m);
  else hipLaunchKernelGGL((lnb_mix_kernel<MT, false>), dim3(m.nblk), dim3(256), 0, s, m);
}

// measurement knob (grr_lnb_set_phases): which of pack (1) / head (2) / mix (4) a forward launches, so
// a caller can time the head and the mix of one block apart on a shared workspace
int g_lnb_phases = 7;

template <int KS>
static void launch_fused(const LnbFusedArgs& f, unsigned grid, int io, hipStream_t s) {
  switch (io) {
    case 1: hipLaunchKernelGGL((lnb_fused16_kernel<KS, (KS + 1) / 2, 1>), dim3(grid), dim3(512), 0, s, f); break;
    case 2: hipLaunchKernelGGL((lnb_fused16_kernel<KS, (KS + 1) / 2, 2>), dim3(grid), dim3(512), 0, s, f); break;
    case 3: hipLaunchKernelGGL((lnb_fused16_kernel<KS, (KS + 1) / 2, 3>), dim3(grid), dim3(512), 0, s, f); break;
    default: hipLaunchKernelGGL((lnb_fused16_kernel<KS, (KS + 1) / 2, 0>), dim3(grid), dim3(512), 0, s, f);
  }
}
// compute units of the current device (cached per device)
static int num_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

grr_status lnb_forward_mfma(const float* x, const float* ln_w, const float* w1, const float* wdw, const float* w2,
                            const float* skip, float* out, float* ws, int B, int C, int hid, int H, int W,
                            hipStream_t s, bool keep_g, int io) {
  GRR_REQUIRE(io == 0 || (lnb_fused(C, hid) && !keep_g), GRR_ERR_UNSUPPORTED,
              "grr_lnb_forward_c8: the channel-blocked layout needs the fused pass (C <= 96) without the kept gate");
  if (!lnb_fused(C, hid)) {
    // the two-kernel path leaves g at the workspace's start anyway
    return lnb_forward_mfma_rep(x, C, 1, x, ln_w, w1, wdw, w2, skip, out, ws, B, hid, H, W, s);
  }
  GRR_REQUIRE((int64_t)std::max(hid, C) * H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_forward: max(hid, C)*H*W too large for one image's 32-bit offsets");
  const int KS = (C + 15) / 16, MT = (C + 31) / 32, nch = (hid + 15) / 16;
  const int64_t P = (int64_t)H * W;
  // the chunk images at the workspace's start (grr_lnb_fused_workspace_bytes), after the g region when the
  // pass also keeps g
  float* base = keep_g ? ws + align64((int64_t)B * hid * P) : ws;
  char* pack = reinterpret_cast<char*>(base);
  float* r2 = base + align64((int64_t)nch * fused_images(KS, MT) * 256);
  if (g_lnb_phases & 1) {
    const int64_t n = (int64_t)nch * fused_images(KS, MT) * 256 + C;
    hipLaunchKernelGGL(lnb_fused_pack_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256),
                       0, s, w1, ln_w, wdw, w2, pack, r2, C, hid, KS, MT, nch);
    grr_status st = launch_status("grr_lnb_forward/fused_pack");
    if (st != GRR_OK) return st;
  }
  if (!(g_lnb_phases & 2)) return GRR_OK;
  LnbFusedArgs f{};
  f.x = x; f.pack = pack; f.r2 = r2; f.skip = skip; f.out = out;
  f.g = keep_g ? ws : nullptr;
  f.var_den = (float)(C - 1);
  f.C = C; f.hid = hid; f.H = H; f.W = W; f.nch = nch;
  f.tiles_x = (W + LF_TW - 1) / LF_TW;
  f.tiles_y = (H + LF_TH - 1) / LF_TH;
  const uint64_t nt = (uint64_t)B * f.tiles_x * f.tiles_y;
  GRR_REQUIRE(nt < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
  f.ntiles = (int)nt;
  // persistent: one workgroup per CU (its LDS), each walking tiles blockIdx.x, + gridDim.x, ...
  const unsigned grid = (unsigned)std::min<uint64_t>(nt, (uint64_t)num_cus());
  switch (KS) {
    case 1: launch_fused<1>(f, grid, io, s); break;
    case 2: launch_fused<2>(f, grid, io, s); break;
    case 3: launch_fused<3>(f, grid, io, s); break;
    case 4: launch_fused<4>(f, grid, io, s); break;
    case 5: launch_fused<5>(f, grid, io, s); break;
    default: launch_fused<6>(f, grid, io, s); break;
  }
  return launch_status("grr_lnb_forward/fused");
}

// the replicated first block runs as one fused pass (lnb_rep_kernel) when its im2col depth 9 Cs fits two
// k-steps (else head16 + mix on the Cs-channel source)
bool lnb_rep_fused(int Ch, int R, int C, int hid) {
  return R > 1 && Ch >= 1 && Ch <= 3 && C <= 128 && hid >= 1;
}

template <int MT>
static void launch_rep(const LnbRepArgs& r, hipStream_t s) {
  switch (r.Cs) {
    case 1: hipLaunchKernelGGL((lnb_rep_kernel<MT, 1>), dim3(r.nblk), dim3(64 * LR_NW), 0, s, r); break;
    case 2: hipLaunchKernelGGL((lnb_rep_kernel<MT, 2>), dim3(r.nblk), dim3(64 * LR_NW), 0, s, r); break;
    default: hipLaunchKernelGGL((lnb_rep_kernel<MT, 3>), dim3(r.nblk), dim3(64 * LR_NW), 0, s, r); break;
  }
}

grr_status lnb_forward_mfma_rep(const float* xh, int Ch, int R, const float* x, const float* ln_w, const float* w1,
                                const float* wdw, const float* w2, const float* skip, float* out, float* ws, int B,
                                int hid, int H, int W, hipStream_t s) {
  const int C = R * Ch;   // channels of x / out; the head reads the Ch-channel xh
  GRR_REQUIRE(C >= 2 && C <= 128 && Ch >= 1, GRR_ERR_UNSUPPORTED, "grr_lnb_forward: C=%d outside [2, 128]", C);
  GRR_REQUIRE((int64_t)std::max(hid, C) * H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_forward: max(hid, C)*H*W too large for one image's 32-bit offsets");
  if (lnb_rep_fused(Ch, R, C, hid)) {
    // workspace: the chunk images at its start (the g region the two-kernel path would use is not needed)
    const int MT = (C + 31) / 32, nch = (hid + 15) / 16;
    char* pack = reinterpret_cast<char*>(ws);
    if (g_lnb_phases & 1) {
      const int64_t n = (int64_t)nch * rep_images(MT) * 256;
      hipLaunchKernelGGL(lnb_rep_pack_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256), 0,
                         s, w1, ln_w, wdw, w2, pack, Ch, R, C, hid, MT, nch);
      grr_status st = launch_status("grr_lnb_forward/rep_pack");
      if (st != GRR_OK) return st;
    }
    if (!(g_lnb_phases & 2)) return GRR_OK;
    LnbRepArgs r{};
    r.xs = xh; r.pack = pack; r.skip = skip; r.out = out;
    r.var_den = (float)(C - 1) / (float)R;
    r.Cs = Ch; r.C = C; r.hid = hid; r.H = H; r.W = W; r.nch = nch;
    r.tiles = (int)(((int64_t)H * W + LR_PX - 1) / LR_PX);
    const uint64_t nb = (uint64_t)B * r.tiles;
    GRR_REQUIRE(nb < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
    r.nblk = (uint32_t)nb;
    switch (MT) {
      case 1: launch_rep<1>(r, s); break;
      case 2: launch_rep<2>(r, s); break;
      case 3: launch_rep<3>(r, s); break;
      default: launch_rep<4>(r, s); break;
    }
    return launch_status("grr_lnb_forward/rep");
  }
  const bool h16 = head16_enabled(Ch);
  const int KS = h16 ? head16_ks(Ch) : head_ks(Ch), NB = head_nb(head_ks(Ch));
  const int nch = h16 ? (hid + L6_NP - 1) / L6_NP : (hid + LH_JC - 1) / LH_JC;
  const int MT = (C + 31) / 32, KS2 = (hid + LM_KD - 1) / LM_KD;
  const int64_t P = (int64_t)H * W;
  float* g = ws;
  char* w1f = reinterpret_cast<char*>(ws + align64((int64_t)B * hid * P));
  uint16_t* w2f = reinterpret_cast<uint16_t*>(ws + align64((int64_t)B * hid * P) + head_pack_floats(Ch, hid));
  if (g_lnb_phases & 1) {
    const int64_t n1 = (int64_t)nch * (h16 ? head16_images(KS) : head_images(KS)) * 256;
    const int64_t n2 = (int64_t)KS2 * MT * 3 * 512;
    const dim3 g1((unsigned)std::min<int64_t>((n1 + 255) / 256, 4096));
    if (h16) hipLaunchKernelGGL(lnb_w1_pack16_kernel, g1, dim3(256), 0, s, w1, ln_w, wdw, w1f, Ch, hid, KS, nch, R);
    else hipLaunchKernelGGL(lnb_w1_pack_kernel, g1, dim3(256), 0, s, w1, ln_w, wdw, w1f, Ch, hid, KS, nch, R);
    hipLaunchKernelGGL(lnb_w2_pack_kernel, dim3((unsigned)std::min<int64_t>((n2 + 255) / 256, 4096)), dim3(256), 0,
                       s, w2, w2f, C, hid, MT, KS2);
    grr_status st = launch_status("grr_lnb_forward/pack");
    if (st != GRR_OK) return st;
  }
  LnbHeadArgs h{};
  h.x = xh; h.w1f = w1f; h.g = g;
  h.var_den = R == 1 ? (float)(C - 1) : (float)(C - 1) / (float)R;
  h.C = Ch; h.hid = hid; h.H = H; h.W = W; h.nch = nch;
  const int TH = h16 ? L6_TH : (NB == 4 ? HeadGeom<4>::TH : HeadGeom<3>::TH);
  h.tiles_x = (W + LH_TW - 1) / LH_TW;
  h.tiles_y = (H + TH - 1) / TH;
  const uint64_t nh = (uint64_t)B * h.tiles_x * h.tiles_y;
  GRR_REQUIRE(nh < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
  h.nblk = (uint32_t)nh;
  if (!(g_lnb_phases & 2)) {
  } else if (h16) {
    switch (KS) {
      case 1: launch_head16<1>(h, s); break;
      case 2: launch_head16<2>(h, s); break;
      case 3: launch_head16<3>(h, s); break;
      case 4: launch_head16<4>(h, s); break;
      case 5: launch_head16<5>(h, s); break;
      default: launch_head16<6>(h, s); break;
    }
  } else {
    switch (KS) {
      case 1: launch_head<1, 4>(h, s); break;
      case 2: launch_head<2, 4>(h, s); break;
      case 3: launch_head<3, 4>(h, s); break;
      default: launch_head<4, 3>(h, s); break;
    }
  }
  grr_status st = launch_status("grr_lnb_forward/head");
  if (st != GRR_OK) return st;
  if (!(g_lnb_phases & 4)) return GRR_OK;
  LnbMixArgs m{};
  m.g = g; m.w2f = reinterpret_cast<const char*>(w2f); m.skip = skip; m.out = out;
  m.x = x ? x : xh;           // x == NULL: the skip reads the replicated image itself
  m.xs_c = x ? 0 : Ch;
  m.P = P; m.C = C; m.hid = hid; m.KS2 = KS2;
  m.tiles = (int)((P + LM_PX - 1) / LM_PX);
  const uint64_t nm = (uint64_t)B * m.tiles;
  GRR_REQUIRE(nm < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
  m.nblk = (uint32_t)nm;
  const bool v4 = P % 4 == 0;
  switch (MT) {
    case 1: launch_mix<1>(m, v4, s); break;
    case 2: launch_mix<2>(m, v4, s); break;
    case 3: launch_mix<3>(m, v4, s); break;
    default: launch_mix<4>(m, v4, s); break;
  }
  return launch_status("grr_lnb_forward/mix");
}

}  // namespace grr

extern "C" int grr_lnb_rep_fused(int Cs, int R, int C, int hid) { return grr::lnb_rep_fused(Cs, R, C, hid) ? 1 : 0; }
extern "C" int grr_lnb_fused(int C, int hid) { return grr::lnb_fused(C, hid) ? 1 : 0; }

extern "C" grr_status grr_lnb_set_fused(int enable) {
  grr::clear_error();
  GRR_REQUIRE(enable == 0 || enable == 1, GRR_ERR_INVALID_ARG, "grr_lnb_set_fused: 0 or 1");
  grr::g_lnb_fused_on = enable;
  return GRR_OK;
}

extern "C" grr_status grr_lnb_set_phases(int mask) {
  grr::clear_error();
  GRR_REQUIRE(mask >= 1 && mask <= 7, GRR_ERR_INVALID_ARG, "grr_lnb_set_phases: mask %d outside [1, 7]", mask);
  grr::g_lnb_phases = mask;
  return GRR_OK;
}

