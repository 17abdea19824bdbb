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
#ifndef GRR_HEAD_OPAQUE_DMA
#define GRR_HEAD_OPAQUE_DMA 1
#endif

#ifdef GRR_FUSED_STAMP
// per-phase cycle totals of the first 64 workgroups' waves of the head or fused kernel (timing builds
// only; ordinary vector stores): gate, GEMM1, GEMM2, barrier 1 / vmcnt wait, h store, (wait +) barrier,
// total, iterations
__device__ unsigned long long g_fused_stamps[64 * 8 * 8];
#endif

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
      if constexpr (GRR_HEAD_OPAQUE_DMA) dma16_opaque(src + img * 1024, slot + img * 256);
      else dma16(src + img * 1024, slot + img * 256);
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
#ifndef GRR_HEAD_STAGGER
#define GRR_HEAD_STAGGER 1
#endif
  const bool gate_first = GRR_HEAD_STAGGER ? wave < 4 : true;
#ifdef GRR_FUSED_STAMP
  uint64_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#define GRR_STAMP(k, t) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); st[k] += t_ - (t); (t) = t_; } while (0)
#else
#define GRR_STAMP(k, t) do { } while (0)
#endif
  for (int c = 0; c <= nch; ++c) {
#ifdef GRR_FUSED_STAMP
    uint64_t tt = __builtin_amdgcn_s_memtime();
#endif
    // chunk c + AHEAD -> slot (c + AHEAD) % NSLOT, last read (gate of chunk c - 2) before the previous barrier
    issue(min(c + AHEAD, nch - 1), (c + AHEAD) % NSLOT);
    if (gate_first) {
      gate(c);
      GRR_STAMP(0, tt);
      gemm1(c);
      GRR_STAMP(1, tt);
    } else {
      gemm1(c);
      GRR_STAMP(1, tt);
      gate(c);
      GRR_STAMP(0, tt);
    }
    // chunk c + 1 landed: after its DMA this wave issued RA stores (iteration c - 1),
    // DPW DMAs and RA stores (iteration c) -- AHEAD = 1: RA stores (iteration c); then every
    // wave's part (barrier)
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(AHEAD == 2 ? 2 * RA + DPW : RA) : "memory");
    GRR_STAMP(3, tt);
    __builtin_amdgcn_s_barrier();
    GRR_STAMP(5, tt);
  }
#ifdef GRR_FUSED_STAMP
  st[6] = __builtin_amdgcn_s_memtime() - t_begin;
  st[7] = (uint64_t)(nch + 1);
  if (blockIdx.x < 64 && lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g_fused_stamps[(blockIdx.x * 8 + wave) * 8 + k] = st[k];
  }
#endif
#undef GRR_STAMP
}

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
// fused: LN + W1 + dw3x3 + gate + W2 + skip in ONE kernel; the gated activations g stay in LDS.
//
// The head kernel's tile (32 columns x TH rows, W1 recomputed on the (TH+2) x 34 halo) and its
// hidden-channel chunk loop (8 (mask, value) pairs per chunk), plus the second GEMM: every chunk
// pair's g (16 hidden channels x TH x 32 pixels, fp32 in LDS) is multiplied into per-wave
// accumulators of the output tile (C rows x TH x 32 pixels, v_mfma_f32_32x32x16_bf16 on the
// exact 3-term split, 6 products) that stay in registers across the whole hidden loop; the
// epilogue adds the skip and writes out.  Per iteration c: gate of chunk c - 1 (LDS h -> LDS g),
// GEMM1 of chunk c (registers), GEMM2 of the pair gated two iterations earlier; barrier; h of
// chunk c to LDS; barrier.  W1 chunks (+ taps) arrive by LDS-DMA in a 4-slot ring two chunks
// ahead, W2 pair fragments in a 2-slot ring; every wave issues the same DMA count per iteration,
// so the ring waits are one counted vmcnt.  Nothing of the 2 hid x HW hidden state or the hid x HW
// gated state reaches HBM: the block reads x (with halo) and writes out.
struct LnbFusedArgs {
  const float* x;        // GEMM1 input [B, Ch, H, W] (Ch = C, or the replicated image's channels)
  const char* w1f;       // W1 diag(ln_w) chunk images + taps (lnb_w1_pack_kernel)
  const char* w2f;       // W2 pair images [npairs][MT][3] (lnb_w2_pack_kernel, 16-deep k-steps)
  const float* xs;       // skip operand [B, XC, H, W]: x, or the image it replicates (channel m mod XC)
  int XC;
  const float* skip;     // [2]
  float* out;            // [B, C, H, W]
  float var_den;
  int Ch, C, hid, H, W, tiles_x, tiles_y, nch, npairs;
  uint32_t nblk;
};


template <int KS, int NB, int MT>
__global__ __launch_bounds__(512, 1) void lnb_fused_kernel(LnbFusedArgs a) {
  using Geo = HeadGeom<NB>;
  constexpr int TH = Geo::TH, RA = Geo::RA, HP = Geo::HP;
  constexpr int NI = KS * 3 + 1;        // W1 images per chunk (fragments + taps)
  constexpr int DPW = (NI + 7) / 8;     // W1 LDS-DMAs per wave per iteration
  constexpr int SLOTF = NI * 256;
  constexpr int NSLOT = 4;
  constexpr int HBUF = 2 * LH_JC * HP;  // one h plane set: 8 mask + 8 value rows of halo pixels
  constexpr int W2I = MT * 3;           // W2 fragment images per chunk pair
  constexpr int W2PW = (W2I + 7) / 8;   // W2 LDS-DMAs per wave per iteration
  constexpr int GPX = TH * LH_TW;       // output pixels of the tile
  // g of one chunk, already split for the GEMM2 B operand: [term][pixel][8 channels] bf16 = 4 floats
  // per (term, pixel); the two 32-lane halves of a B read hit chunk slots 16 floats apart mod 64
  constexpr int GCH = 3 * GPX * 4 + 16;
  constexpr int NT2 = MT * TH;          // GEMM2 output tiles (32 channels x 32 pixels of one output row)
  constexpr int TPW = (NT2 + 7) / 8;    // tiles per wave
  __shared__ __attribute__((aligned(16))) float smem[HBUF + NSLOT * SLOTF + 2 * W2I * 256 + 3 * GCH];
  float* const hb = smem;               // h of one chunk: [channel 0..7][halo pixel][mask, value]
  float* const ring = smem + HBUF;
  float* const w2ring = ring + NSLOT * SLOTF;
  float* const gring = w2ring + 2 * W2I * 256;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int tx = lb % a.tiles_x; lb /= a.tiles_x;
  const int ty = lb % a.tiles_y;
  const int b = lb / a.tiles_y;
  const int H = a.H, W = a.W, Ch = a.Ch, C = a.C, hid = a.hid, nch = a.nch, npairs = a.npairs;
  const int HW = H * W;
  const int y0 = ty * TH, x0 = tx * LH_TW;

  auto issue_w1 = [&](int chunk, int slot_idx) {
    float* slot = ring + slot_idx * SLOTF;
    const char* src = a.w1f + (int64_t)chunk * NI * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int img = min(i * 8 + wave, NI - 1);   // surplus waves repeat the last image
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };
  auto issue_w2 = [&](int pair) {
    float* slot = w2ring + (pair & 1) * W2I * 256;
    const char* src = a.w2f + (int64_t)pair * W2I * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < W2PW; ++i) {
      const int img = min(i * 8 + wave, W2I - 1);
      dma16_opaque(src + img * 1024, slot + img * 256);
    }
  };
  issue_w1(0, 0);
  issue_w1(min(1, nch - 1), 1);
  issue_w2(0);

  // this wave's halo pixels: raw x column split into bf16 terms, and 1/sigma (REF:916-922)
  const int kq = lane >> 4;
  bf16x8 xf[NB][KS][3];
  float rstd[NB];
  {
    float xv[NB][KS][8];
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      const int q = min((wave * NB + blk) * 16 + (lane & 15), Geo::HR * LH_HWD - 1);
      const int hy = q / LH_HWD, hx = q - hy * LH_HWD;
      const int gy = clampi(y0 - 1 + hy, 0, H - 1), gx = clampi(x0 - 1 + hx, 0, W - 1);
      const float* xp = a.x + (int64_t)b * Ch * HW + gy * W + gx;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[blk][s][j] = xp[(int64_t)min(32 * s + 8 * kq + j, Ch - 1) * HW];
    }
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      float sum = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (32 * s + 8 * kq + j >= Ch) xv[blk][s][j] = 0.f;
          sum += xv[blk][s][j];
        }
      sum += __shfl_xor(sum, 16);
      sum += __shfl_xor(sum, 32);
      const float mean = sum / (float)Ch;
      float sq = 0.f;
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = 32 * s + 8 * kq + j < Ch ? xv[blk][s][j] - mean : 0.f;
          sq += d * d;
        }
      sq += __shfl_xor(sq, 16);
      sq += __shfl_xor(sq, 32);
      rstd[blk] = 1.0f / sqrtf(sq / a.var_den + 1e-5f);
#pragma unroll
      for (int s = 0; s < KS; ++s) split3x8(xv[blk][s], xf[blk][s][0], xf[blk][s][1], xf[blk][s][2]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // W1 chunks 0, 1 and W2 pair 0 landed (this wave's part)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  f32x4 acc1[NB];
  f32x16 acc2[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc2[i] = f32x16{};

  auto gemm1 = [&](int c) {
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) acc1[blk] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (c >= nch) return;
    const float* slot = ring + (c % NSLOT) * SLOTF + lane * 4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 0) * 256);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 1) * 256);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(slot + (3 * s + 2) * 256);
#pragma unroll
      for (int blk = 0; blk < NB; ++blk)
        GRR_X3_MFMA(__builtin_amdgcn_mfma_f32_16x16x32_bf16, acc1[blk], a0, a1, a2, xf[blk][s][0],
                    xf[blk][s][1], xf[blk][s][2]);
      // the next k-step's fragments are read while these MFMAs run (not all hoisted: registers)
      asm volatile("" ::: "memory");
    }
  };
  // GEMM1 rows 4 kq + i: kq < 2 mask channels 4 kq + i, kq >= 2 value channels 4 (kq - 2) + i
  auto store_h = [&](int c) {
    if (c >= nch) return;
    const int ch0 = 4 * (kq & 1), comp = kq >> 1;
#pragma unroll
    for (int blk = 0; blk < NB; ++blk) {
      const int q = (wave * NB + blk) * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) hb[((ch0 + i) * HP + q) * 2 + comp] = acc1[blk][i] * rstd[blk];
    }
  };
  // depthwise 3x3 (REF:946) + gate sigmoid(m) m v (REF:947) of chunk c - 1 -> g slot (c - 1) mod 3.
  // Mask and value run as one packed pair (v_pk_fma_f32; each component the same fma chain in the
  // reference's tap order); g goes to LDS as its exact 3-term bf16 split, in the GEMM2 B layout.
  const int col = lane & 31, r0 = (lane >> 5) * RA;
  auto gate = [&](int c) {
    const int jj = LH_JC * (c - 1) + wave;
    const bool live = c >= 1 && jj < hid;
    const f32x2* hp = reinterpret_cast<const f32x2*>(hb) + wave * HP + col;
    const float* taps = ring + ((c + NSLOT - 1) % NSLOT) * SLOTF + KS * 3 * 256 + wave * 18;
    __bf16* gdst = reinterpret_cast<__bf16*>(gring + ((c + 2) % 3) * GCH) + wave;
    const f32x2* k2 = reinterpret_cast<const f32x2*>(taps);   // (mask, value) tap pairs, broadcast LDS reads
    f32x2 hw[3][3];
#pragma unroll
    for (int i = 0; i < RA + 2; ++i) {
      const int hrow = min(r0 + i, Geo::HR - 1) * LH_HWD;
#pragma unroll
      for (int d = 0; d < 3; ++d) hw[i % 3][d] = hp[hrow + d];
      if (i >= 2) {
        f32x2 mv = f32x2{0.f, 0.f};
#pragma unroll
        for (int ay = 0; ay < 3; ++ay)
#pragma unroll
          for (int ax = 0; ax < 3; ++ax) mv = __builtin_elementwise_fma(k2[ay * 3 + ax], hw[(i - 2 + ay) % 3][ax], mv);
        const float m = mv.x, v = mv.y;
        const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-m));
        const float g = live ? (sg * m) * v : 0.f;   // 0 for padding channels
        const int orow = r0 + i - 2;
        if (orow < TH) {
          const __bf16 h0 = (__bf16)g;
          const float r1 = g - (float)h0;
          const __bf16 h1 = (__bf16)r1;
          const __bf16 h2 = (__bf16)(r1 - (float)h1);
          __bf16* d = gdst + (orow * LH_TW + col) * 8;
          d[0] = h0;
          d[GPX * 8] = h1;
          d[2 * GPX * 8] = h2;
        }
      }
    }
  };
  // out tile rows += W2[:, 16 p .. 16 p + 15] g(pair p): tile t = wave + 8 i -> (output row t / MT, rows 32 (t % MT) ..)
  auto gemm2 = [&](int p) {
    const float* w2 = w2ring + (p & 1) * W2I * 256 + lane * 4;
    const float* gsrc = gring + ((2 * p + (lane >> 5)) % 3) * GCH + col * 4;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + 8 * i;
      if (t < NT2) {
        const int orow = t / MT, mt = t - orow * MT;
        const float* gp = gsrc + orow * LH_TW * 4;
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(gp);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(gp + GPX * 4);
        const bf16x8 b2 = *reinterpret_cast<const bf16x8*>(gp + 2 * GPX * 4);
        const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(w2 + (3 * mt + 0) * 256);
        const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(w2 + (3 * mt + 1) * 256);
        const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(w2 + (3 * mt + 2) * 256);
        GRR_X3_MFMA(__builtin_amdgcn_mfma_f32_32x32x16_bf16, acc2[i], a0, a1, a2, b0, b1, b2);
      }
    }
  };

  // iteration c: gate(c - 1 chunk), GEMM1(c), GEMM2 of the pair gated in iterations c - 2, c - 1
  const bool gate_first = wave < 4;   // SIMD partners (w, w + 4) overlap one's MFMA with the other's VALU
  const int cmax = 2 * npairs + 1;
#ifdef GRR_FUSED_STAMP
  uint64_t st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t_begin = __builtin_amdgcn_s_memtime();
#define GRR_STAMP(k, t) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); st[k] += t_ - (t); (t) = t_; } while (0)
#else
#define GRR_STAMP(k, t) do { } while (0)
#endif
  for (int c = 0; c <= cmax; ++c) {
#ifdef GRR_FUSED_STAMP
    uint64_t tt = __builtin_amdgcn_s_memtime();
#endif
    issue_w1(min(c + 2, nch - 1), (c + 2) % NSLOT);   // slot last read by gate(c - 1) (taps of chunk c - 2)
    issue_w2(min(c >> 1, npairs - 1));                // slot last read by gemm2 of iteration c - 1 or earlier
    if (gate_first) {
      gate(c);
      GRR_STAMP(0, tt);
      gemm1(c);
      GRR_STAMP(1, tt);
    } else {
      gemm1(c);
      GRR_STAMP(1, tt);
      gate(c);
      GRR_STAMP(0, tt);
    }
    if ((c & 1) && c >= 3) gemm2((c - 3) >> 1);
    GRR_STAMP(2, tt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                     // h of chunk c - 1 and the g slots read: reusable
    asm volatile("" ::: "memory");
    GRR_STAMP(3, tt);
    store_h(c);
    GRR_STAMP(4, tt);
    // everything issued before this iteration landed (this wave's part), then every wave's
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(DPW + W2PW) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    GRR_STAMP(5, tt);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef GRR_FUSED_STAMP
  st[6] = __builtin_amdgcn_s_memtime() - t_begin;
  st[7] = (uint64_t)(cmax + 1);
  if (blockIdx.x < 64 && lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g_fused_stamps[(blockIdx.x * 8 + wave) * 8 + k] = st[k];
  }
#endif
#undef GRR_STAMP

  // epilogue (REF:962-964): out = skip0 x + skip1 W2 g.  acc2[i] element e: channel
  // 32 mt + (e & 3) + 8 (e >> 2) + 4 (lane >> 5), pixel (y0 + orow, x0 + lane & 31)
  const float s0 = a.skip[0], s1 = a.skip[1];
  const int XC = a.XC;
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.xs + (int64_t)b * XC * HW), 0, (int)((int64_t)XC * HW * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)b * C * HW, 0,
                                                                        (int)((int64_t)C * HW * 4), 0x00020000);
  const int gx = x0 + col;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 8 * i;
    if (t < NT2) {
      const int orow = t / MT, mt = t - orow * MT;
      const int gy = y0 + orow;
      const bool pix = gy < H && gx < W;
      const int p = min(gy, H - 1) * W + min(gx, W - 1);
      float xv[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = min(32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5), C - 1);
        const int mx = XC == C ? m : m % XC;
        xv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, (uint32_t)(mx * HW + p) * 4u, 0, 0));
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = 32 * mt + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const uint32_t off = (m < C && pix) ? (uint32_t)(m * HW + p) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(s0 * xv[e] + s1 * acc2[i][e]), ors, off, 0, 0);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side
static int head_ks(int C) { return (C + 31) / 32; }
static int head_nb(int KS) { return KS <= 3 ? 4 : 3; }
static int64_t align64(int64_t n) { return (n + 63) / 64 * 64; }
static int64_t head_pack_floats(int C, int hid) {
  return align64((int64_t)((hid + LH_JC - 1) / LH_JC) * head_images(head_ks(C)) * 256);
}
static int64_t mix_pack_floats(int C, int hid) {
  return align64((int64_t)((hid + LM_KD - 1) / LM_KD) * ((C + 31) / 32) * 3 * 256);
}

// workspace (floats): [g: B*hid*P][W1 images][W2 images], each 256-B aligned
int64_t lnb_mfma_workspace_floats(int B, int C, int hid, int H, int W) {
  return align64((int64_t)B * hid * H * W) + head_pack_floats(C, hid) + mix_pack_floats(C, hid);
}

template <int KS, int NB>
static void launch_head(const LnbHeadArgs& h, hipStream_t s) {
  hipLaunchKernelGGL((lnb_head_kernel<KS, NB>), dim3(h.nblk), dim3(512), 0, s, h);
}
template <int MT>
static void launch_mix(const LnbMixArgs& m, bool v4, hipStream_t s) {
  if (v4) hipLaunchKernelGGL((lnb_mix_kernel<MT, true>), dim3(m.nblk), dim3(256), 0, s, m);
  else hipLaunchKernelGGL((lnb_mix_kernel<MT, false>), dim3(m.nblk), dim3(256), 0, s, m);
}

// GRR_LNB_FUSED=1 selects the single fused kernel (A/B measurements).  Default: head + mix -- the
// fused kernel keeps the GEMM2 accumulators in the registers the gate phase needs for latency
// hiding and measured slower
static bool lnb_fused_enabled() {
  static const bool on = [] {
    const char* e = getenv("GRR_LNB_FUSED");
    return e && e[0] == '1';
  }();
  return on;
}

// halo pixel blocks per wave of the fused kernel: its GEMM2 accumulators share the 256 registers
// of a 2-waves-per-SIMD kernel with the x fragments, so deeper / wider blocks run 3 blocks (9-row
// tiles); the shapes that would still spill (K > 96 with C > 32, or C > 96 with K > 32) keep the
// two-kernel head + mix path
static constexpr int fused_nb(int KS, int MT) { return (KS == 1 || (KS == 2 && MT <= 2)) ? 4 : 3; }
static bool fused_ok(int KS, int MT) { return KS <= MT && (KS == 1 || MT <= 3); }
template <int KS, int MT>
static void launch_fused_t(const LnbFusedArgs& f, hipStream_t s) {
  constexpr int NB = fused_nb(KS, MT);
  hipLaunchKernelGGL((lnb_fused_kernel<KS, NB, MT>), dim3(f.nblk), dim3(512), 0, s, f);
}
static void launch_fused(const LnbFusedArgs& f, int KS, int MT, hipStream_t s) {
  switch (MT * 8 + KS) {
    case 1 * 8 + 1: launch_fused_t<1, 1>(f, s); break;
    case 2 * 8 + 1: launch_fused_t<1, 2>(f, s); break;
    case 2 * 8 + 2: launch_fused_t<2, 2>(f, s); break;
    case 3 * 8 + 1: launch_fused_t<1, 3>(f, s); break;
    case 3 * 8 + 2: launch_fused_t<2, 3>(f, s); break;
    case 3 * 8 + 3: launch_fused_t<3, 3>(f, s); break;
    default: launch_fused_t<1, 4>(f, s); break;
  }
}

grr_status lnb_forward_mfma(const float* x, const float* ln_w, const float* w1, const float* wdw, const float* w2,
                            const float* skip, float* out, float* ws, int B, int C, int hid, int H, int W,
                            hipStream_t s) {
  return lnb_forward_mfma_rep(x, C, 1, x, ln_w, w1, wdw, w2, skip, out, ws, B, hid, H, W, s);
}

grr_status lnb_forward_mfma_rep(const float* xh, int Ch, int R, const float* x, const float* ln_w, const float* w1,
                                const float* wdw, const float* w2, const float* skip, float* out, float* ws, int B,
                                int hid, int H, int W, hipStream_t s) {
  const int C = R * Ch;   // channels of x / out; the head reads the Ch-channel xh
  GRR_REQUIRE(C >= 2 && C <= 128 && Ch >= 1, GRR_ERR_UNSUPPORTED, "grr_lnb_forward: C=%d outside [2, 128]", C);
  GRR_REQUIRE((int64_t)std::max(hid, C) * H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_forward: max(hid, C)*H*W too large for one image's 32-bit offsets");
  const int KS = head_ks(Ch), NB = head_nb(KS), nch = (hid + LH_JC - 1) / LH_JC;
  const int MT = (C + 31) / 32, KS2 = (hid + LM_KD - 1) / LM_KD;
  const int64_t P = (int64_t)H * W;
  float* g = ws;
  char* w1f = reinterpret_cast<char*>(ws + align64((int64_t)B * hid * P));
  uint16_t* w2f = reinterpret_cast<uint16_t*>(ws + align64((int64_t)B * hid * P) + head_pack_floats(Ch, hid));
  {
    const int64_t n1 = (int64_t)nch * head_images(KS) * 256, n2 = (int64_t)KS2 * MT * 3 * 512;
    hipLaunchKernelGGL(lnb_w1_pack_kernel, dim3((unsigned)std::min<int64_t>((n1 + 255) / 256, 4096)), dim3(256), 0,
                       s, w1, ln_w, wdw, w1f, Ch, hid, KS, nch, R);
    hipLaunchKernelGGL(lnb_w2_pack_kernel, dim3((unsigned)std::min<int64_t>((n2 + 255) / 256, 4096)), dim3(256), 0,
                       s, w2, w2f, C, hid, MT, KS2);
    grr_status st = launch_status("grr_lnb_forward/pack");
    if (st != GRR_OK) return st;
  }
  if (lnb_fused_enabled() && fused_ok(KS, MT)) {
    LnbFusedArgs f{};
    f.x = xh; f.w1f = w1f; f.w2f = reinterpret_cast<const char*>(w2f);
    f.xs = x ? x : xh;          // x == NULL: the skip reads the replicated image itself
    f.XC = x ? C : Ch;
    f.skip = skip; f.out = out;
    f.var_den = R == 1 ? (float)(C - 1) : (float)(C - 1) / (float)R;
    f.Ch = Ch; f.C = C; f.hid = hid; f.H = H; f.W = W; f.nch = nch; f.npairs = KS2;
    const int TH = fused_nb(KS, MT) == 4 ? HeadGeom<4>::TH : HeadGeom<3>::TH;
    f.tiles_x = (W + LH_TW - 1) / LH_TW;
    f.tiles_y = (H + TH - 1) / TH;
    const uint64_t nf = (uint64_t)B * f.tiles_x * f.tiles_y;
    GRR_REQUIRE(nf < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
    f.nblk = (uint32_t)nf;
    launch_fused(f, KS, MT, s);
    return launch_status("grr_lnb_forward/fused");
  }
  LnbHeadArgs h{};
  h.x = xh; h.w1f = w1f; h.g = g;
  h.var_den = R == 1 ? (float)(C - 1) : (float)(C - 1) / (float)R;
  h.C = Ch; h.hid = hid; h.H = H; h.W = W; h.nch = nch;
  const int TH = NB == 4 ? HeadGeom<4>::TH : HeadGeom<3>::TH;
  h.tiles_x = (W + LH_TW - 1) / LH_TW;
  h.tiles_y = (H + TH - 1) / TH;
  const uint64_t nh = (uint64_t)B * h.tiles_x * h.tiles_y;
  GRR_REQUIRE(nh < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_lnb_forward: grid too large");
  h.nblk = (uint32_t)nh;
  switch (KS) {
    case 1: launch_head<1, 4>(h, s); break;
    case 2: launch_head<2, 4>(h, s); break;
    case 3: launch_head<3, 4>(h, s); break;
    default: launch_head<4, 3>(h, s); break;
  }
  grr_status st = launch_status("grr_lnb_forward/head");
  if (st != GRR_OK) return st;
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

#ifdef GRR_FUSED_STAMP
extern "C" grr_status grr_debug_fused_stamps(unsigned long long* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(grr::g_fused_stamps), sizeof(grr::g_fused_stamps)) == hipSuccess
             ? GRR_OK : GRR_ERR_HIP;
}
#endif
