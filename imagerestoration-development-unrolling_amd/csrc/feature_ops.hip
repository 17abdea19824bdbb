// gfx950 kernels of the feature CNN that produces the graph features
// (a13 of SURVEY.md §8; REF13 = lib/model_GLR_GTV_deep_v13_no_latent.py).
//
// Dense channel mixing (1x1 and 2x2/s2 convolutions) is a batched GEMM
//   out[b] (M x P) = Wt (M x K) * Bop[b] (K x P),   P = pixels,
// computed on the matrix cores with the exact-fp32 MFMA v_mfma_f32_32x32x2_f32
// (gfx950 has no xf32; f32-in MFMA is bit-for-bit an fmaf chain, so the result
// stays within fp32 rounding of the reference's CPU conv).  The B-operand loader
// fuses CustomLayerNorm's normalisation (LN GEMM) or the 2x2/s2 im2col gather.
// Depthwise 3x3 + gating and the LayerNorm statistics are memory-bound kernels.
#include "grr_common.h"

namespace grr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GT = 256;                    // threads per GEMM workgroup (4 waves, 2x2)
constexpr int BM = 128, BN = 128, BK = 16;  // block tile; each wave owns a 64x64 quadrant
constexpr int APAD = BM + 2;                // 130: conflict-free transposed A stores (8*130 = 16 mod 32)
constexpr int BPAD = BN + 4;

enum { LD_PLAIN = 0, LD_LN = 1, LD_IM2COL = 2 };
enum { EP_STORE = 0, EP_SKIP = 1 };

struct GemmArgs {
  const float* x;      // activations [B, K, P]  (im2col: [B, Cin, H, W])
  const float* wt;     // [M, K]
  const float* ln_sd;  // LD_LN: [B, P] 1 / sqrt(var + eps)
  const float* ln_w;   // LD_LN: [K]
  const float* res;    // EP_SKIP: [B, M, P]
  const float* skip;   // EP_SKIP: [2]
  float* out;          // [B, M, P]
  int K, M;
  int64_t P;
  int Hin, Win, Wo;    // im2col geometry
  int mt, nt;
  uint32_t nblk;
};

// Block tile 128 (out channels) x 128 (pixels), K in chunks of 16 staged through a
// double-buffered LDS image; the next chunk is fetched into registers while the
// current one feeds the matrix cores (v_mfma_f32_32x32x2_f32, 4 accumulators/wave).
template <int LOADER, int EPI, bool VEC>
__global__ __launch_bounds__(GT) void gemm_f32_kernel(GemmArgs a) {
  // one LDS image: double-buffered A / B staging during the K loop, reused by the epilogue
  __shared__ __attribute__((aligned(16))) float smem[2 * BK * APAD + 2 * BK * BPAD + 512];
  auto As = reinterpret_cast<float(*)[BK][APAD]>(smem);
  auto Bs = reinterpret_cast<float(*)[BK][BPAD]>(smem + 2 * BK * APAD);
  float* lnw = smem + 2 * BK * APAD + 2 * BK * BPAD;   // LD_LN: CustomLayerNorm scale, K <= 512
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int mtile = lb % a.mt; lb /= a.mt;       // M tiles of one pixel tile are neighbours (shared B)
  const int ntile = lb % a.nt;
  const int b = lb / a.nt;
  const int m0 = mtile * BM;
  const int64_t n0 = (int64_t)ntile * BN;
  const int K = a.K, M = a.M;
  const int64_t P = a.P;
  const float* xb = a.x + (int64_t)b * (LOADER == LD_IM2COL ? (int64_t)(K / 4) * a.Hin * a.Win : (int64_t)K * P);

  // A staging: thread -> row am, 8 consecutive k;  B staging: thread -> row bk, 8 consecutive n
  const int am = tid >> 1, ak = (tid & 1) * 8;
  const int bk = tid >> 4, bn = (tid & 15) * 8;
  float ra[8], rb[8];
  auto load_chunk = [&](int k0) {
    const int mm = m0 + am;
    if (VEC && mm < M && k0 + ak + 8 <= K) {
      const float4* src = reinterpret_cast<const float4*>(a.wt + (int64_t)mm * K + k0 + ak);
      const float4 v0 = src[0], v1 = src[1];
      ra[0] = v0.x; ra[1] = v0.y; ra[2] = v0.z; ra[3] = v0.w;
      ra[4] = v1.x; ra[5] = v1.y; ra[6] = v1.z; ra[7] = v1.w;
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = k0 + ak + q;
        ra[q] = (mm < M && k < K) ? a.wt[(int64_t)mm * K + k] : 0.f;
      }
    }
    if constexpr (LOADER == LD_LN) {
      // CustomLayerNorm's per-channel scale folded into W1's columns (REF:925); the per-pixel
      // 1/sigma is applied in the epilogue: W1 (g * x / sigma) = (W1 diag g) x / sigma
#pragma unroll
      for (int q = 0; q < 8; ++q) ra[q] *= lnw[k0 + ak + q];
    }
    const int k = k0 + bk;
    if constexpr (LOADER == LD_IM2COL) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t n = n0 + bn + q;
        float v = 0.f;
        if (k < K && n < P) {
          const int ci = k >> 2, ay = (k >> 1) & 1, ax = k & 1;
          const int oy = (int)(n / a.Wo), ox = (int)(n - (int64_t)oy * a.Wo);
          v = xb[((int64_t)ci * a.Hin + 2 * oy + ay) * a.Win + 2 * ox + ax];
        }
        rb[q] = v;
      }
    } else {
      if (VEC && k < K && n0 + bn + 8 <= P) {
        const float4* src = reinterpret_cast<const float4*>(xb + (int64_t)k * P + n0 + bn);
        const float4 v0 = src[0], v1 = src[1];
        rb[0] = v0.x; rb[1] = v0.y; rb[2] = v0.z; rb[3] = v0.w;
        rb[4] = v1.x; rb[5] = v1.y; rb[6] = v1.z; rb[7] = v1.w;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int64_t n = n0 + bn + q;
          rb[q] = (k < K && n < P) ? xb[(int64_t)k * P + n] : 0.f;
        }
      }
    }
  };
  auto store_chunk = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) As[buf][ak + q][am] = ra[q];
    *reinterpret_cast<float4*>(&Bs[buf][bk][bn]) = make_float4(rb[0], rb[1], rb[2], rb[3]);
    *reinterpret_cast<float4*>(&Bs[buf][bk][bn + 4]) = make_float4(rb[4], rb[5], rb[6], rb[7]);
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int nchunks = (K + BK - 1) / BK;
  if constexpr (LOADER == LD_LN) {
    for (int k = tid; k < nchunks * BK; k += GT) lnw[k] = k < K ? a.ln_w[k] : 0.f;
    __syncthreads();
  }
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunks) load_chunk((c + 1) * BK);   // in flight during this chunk's MFMAs
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int kr = kk + (lane >> 5);
      const float a0 = As[buf][kr][wm * 64 + (lane & 31)];
      const float a1 = As[buf][kr][wm * 64 + 32 + (lane & 31)];
      const float b0 = Bs[buf][kr][wn * 64 + (lane & 31)];
      const float b1 = Bs[buf][kr][wn * 64 + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (c + 1 < nchunks) store_chunk(buf ^ 1);
    __syncthreads();
  }
  // Epilogue: each 32x32 accumulator tile goes through a per-wave LDS slab (rows m, 32
  // columns n, padded) and leaves as 16-byte row segments: 4 dwordx4 stores per lane
  // instead of 16 dword stores (the store-issue rate, not HBM, bounds a scalar epilogue).
  float s0 = 0.f, s1 = 1.f;
  if constexpr (EPI == EP_SKIP) { s0 = a.skip[0]; s1 = a.skip[1]; }
  constexpr int TP = 36;                                   // slab row pitch (floats)
  float* slab = smem + wave * 32 * TP;                     // 4 x 4.5 KB, inside the A/B image
  const int rr = lane >> 3, cq = (lane & 7) * 4;           // read-back: row group, 4-column chunk
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        slab[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * TP + (lane & 31)] = acc[i][j][r];
      __builtin_amdgcn_s_waitcnt(0xc07f);                   // lgkmcnt(0): this wave's slab writes
      const int64_t nb = n0 + wn * 64 + j * 32 + cq;
      float cs[4] = {1.f, 1.f, 1.f, 1.f};
      if constexpr (LOADER == LD_LN) {                     // 1/sigma per pixel column (REF:921-922)
#pragma unroll
        for (int q = 0; q < 4; ++q) cs[q] = nb + q < P ? a.ln_sd[(int64_t)b * P + nb + q] : 0.f;
      }
#pragma unroll
      for (int pass = 0; pass < 4; ++pass) {
        const int row = pass * 8 + rr;
        const int m = m0 + wm * 64 + i * 32 + row;
        const float4 v4 = *reinterpret_cast<const float4*>(&slab[row * TP + cq]);
        float v[4] = {v4.x, v4.y, v4.z, v4.w};
        if (m < M) {
          const int64_t o = ((int64_t)b * M + m) * P + nb;
          if (VEC && nb + 4 <= P) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if constexpr (LOADER == LD_LN) v[q] *= cs[q];
            }
            if constexpr (EPI == EP_SKIP) {
              const float4 r4 = *reinterpret_cast<const float4*>(a.res + o);
              v[0] = s0 * r4.x + s1 * v[0]; v[1] = s0 * r4.y + s1 * v[1];
              v[2] = s0 * r4.z + s1 * v[2]; v[3] = s0 * r4.w + s1 * v[3];   // REF:962-964
            }
            *reinterpret_cast<float4*>(a.out + o) = make_float4(v[0], v[1], v[2], v[3]);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              if (nb + q < P) {
                float w = v[q];
                if constexpr (LOADER == LD_LN) w *= cs[q];
                if constexpr (EPI == EP_SKIP) w = s0 * a.res[o + q] + s1 * w;
                a.out[o + q] = w;
              }
            }
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);                   // slab reads done before reuse
    }
}

template <int LOADER, int EPI>
static grr_status launch_gemm(GemmArgs a, int B, hipStream_t s, const char* name) {
  a.mt = (a.M + BM - 1) / BM;
  const int64_t nt = (a.P + BN - 1) / BN;
  GRR_REQUIRE(nt < (1ll << 30), GRR_ERR_UNSUPPORTED, "%s: too many pixels", name);
  a.nt = (int)nt;
  const uint64_t n = (uint64_t)B * a.mt * a.nt;
  GRR_REQUIRE(n < (1ull << 31), GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  a.nblk = (uint32_t)n;
  // 16-byte vector staging needs 4-aligned row strides (and base pointers, which torch provides)
  const bool vec = (a.K % 4 == 0) && (a.P % 4 == 0) && ((uintptr_t)a.x % 16 == 0) && ((uintptr_t)a.wt % 16 == 0);
  if (vec) hipLaunchKernelGGL((gemm_f32_kernel<LOADER, EPI, true>), dim3(a.nblk), dim3(GT), 0, s, a);
  else hipLaunchKernelGGL((gemm_f32_kernel<LOADER, EPI, false>), dim3(a.nblk), dim3(GT), 0, s, a);
  return launch_status(name);
}

// CustomLayerNorm statistics: sd[b,p] = 1/sqrt(var_c x[b,c,p] + 1e-5), unbiased (REF:919-922).
// One workgroup = 64 consecutive pixels x LN_G channel groups (one wave each, channels
// c = grp, grp + LN_G, ...; 256-B coalesced row loads, 4 independent accumulators per lane);
// two passes (mean, then squared deviations) as the reference's var, partials via LDS.
constexpr int LN_G = 4;
__global__ __launch_bounds__(64 * LN_G) void ln_stats_kernel(const float* __restrict__ x, float* __restrict__ sd,
                                                             int B, int C, int64_t P) {
  __shared__ float part[LN_G][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t tiles = (P + 63) / 64;
  const int64_t b = blockIdx.x / tiles, p = (blockIdx.x - b * tiles) * 64 + lane;
  const bool ok = p < P;
  const float* xp = x + b * C * P + (ok ? p : 0);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int c = grp;
  for (; c + 3 * LN_G < C; c += 4 * LN_G) {
    a0 += xp[(int64_t)c * P];
    a1 += xp[(int64_t)(c + LN_G) * P];
    a2 += xp[(int64_t)(c + 2 * LN_G) * P];
    a3 += xp[(int64_t)(c + 3 * LN_G) * P];
  }
  for (; c < C; c += LN_G) a0 += xp[(int64_t)c * P];
  part[grp][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < LN_G; ++g) s += part[g][lane];
  const float mean = s / (float)C;
  __syncthreads();
  a0 = a1 = a2 = a3 = 0.f;
  c = grp;
  for (; c + 3 * LN_G < C; c += 4 * LN_G) {
    const float d0 = xp[(int64_t)c * P] - mean, d1 = xp[(int64_t)(c + LN_G) * P] - mean;
    const float d2 = xp[(int64_t)(c + 2 * LN_G) * P] - mean, d3 = xp[(int64_t)(c + 3 * LN_G) * P] - mean;
    a0 += d0 * d0; a1 += d1 * d1; a2 += d2 * d2; a3 += d3 * d3;
  }
  for (; c < C; c += LN_G) {
    const float d = xp[(int64_t)c * P] - mean;
    a0 += d * d;
  }
  part[grp][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (grp == 0 && ok) {
    float q = 0.f;
#pragma unroll
    for (int g = 0; g < LN_G; ++g) q += part[g][lane];
    sd[b * P + p] = 1.0f / sqrtf(q / (float)(C - 1) + 1e-5f);
  }
}

// depthwise 3x3 on the 2*hid GEMM output, then the gate.  One workgroup = (b, j, 32x32 tile).
//   FFN = false: LocalNonLinearBlock, replicate padding, g = sigmoid(mask) * mask * value (REF:934-947)
//   FFN = true:  the window models' FeedForward (REF7:29-48), zero padding (Conv2d padding=1),
//                g = gelu(x1) * x2 with the exact erf gelu of nn.functional.gelu
constexpr int DT = 32, DS = DT + 2, DA = DS * DS;
template <bool FFN>
__global__ __launch_bounds__(256) void dw_gate_kernel(const float* __restrict__ h, const float* __restrict__ wdw,
                                                      float* __restrict__ gout, int hid, int H, int W,
                                                      int tiles_x, int tiles_y, uint32_t nblk) {
  __shared__ float Ms[DA];
  __shared__ float Vs[DA];
  uint32_t lb = xcd_remap(blockIdx.x, nblk);
  const int tx = lb % tiles_x; lb /= tiles_x;
  const int ty = lb % tiles_y; lb /= tiles_y;
  const int j = lb % hid;
  const int b = lb / hid;
  const int y0 = ty * DT, x0 = tx * DT;
  const int64_t HW = (int64_t)H * W;
  const float* mp = h + ((int64_t)b * 2 * hid + j) * HW;
  const float* vp = h + ((int64_t)b * 2 * hid + hid + j) * HW;
  for (int i = threadIdx.x; i < DA; i += 256) {
    const int ry = i / DS, rx = i - ry * DS;
    const int yy = y0 - 1 + ry, xx = x0 - 1 + rx;
    const int64_t o = (int64_t)clampi(yy, 0, H - 1) * W + clampi(xx, 0, W - 1);
    const bool in = !FFN || (yy >= 0 && yy < H && xx >= 0 && xx < W);
    Ms[i] = in ? mp[o] : 0.f;
    Vs[i] = in ? vp[o] : 0.f;
  }
  float km[9], kv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    km[t] = wdw[j * 9 + t];
    kv[t] = wdw[(hid + j) * 9 + t];
  }
  __syncthreads();
  float* gp = gout + ((int64_t)b * hid + j) * HW;
  for (int i = threadIdx.x; i < DT * DT; i += 256) {
    const int oy = i / DT, ox = i - oy * DT;
    const int gy = y0 + oy, gx = x0 + ox;
    if (gy >= H || gx >= W) continue;
    float m = 0.f, v = 0.f;
#pragma unroll
    for (int ay = 0; ay < 3; ++ay)
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        const int li = (oy + ay) * DS + ox + ax;
        m += km[ay * 3 + ax] * Ms[li];
        v += kv[ay * 3 + ax] * Vs[li];
      }
    if constexpr (FFN) {
      gp[(int64_t)gy * W + gx] = (m * 0.5f * (1.0f + erff(m * 0.70710678118654752440f))) * v;
    } else {
      const float sg = 1.0f / (1.0f + expf(-m));
      gp[(int64_t)gy * W + gx] = (sg * m) * v;
    }
  }
}

// ---------------------------------------------------------------------------
// fp32-accurate 1x1 convolution on bf16 MFMA ("x3 split").
//
// Every fp32 operand is split EXACTLY into three bf16 terms, v = v0 + v1 + v2
// (v0 = rne(v), v1 = rne(v - v0), v2 = v - v0 - v1: the 24 significand bits as 3 x 8),
// and the six products above 2^-24 |a b| are accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16: a0b0 + a0b1 + a1b0 + a0b2 + a2b0 + a1b1 (the dropped
// a1b2 + a2b1 + a2b2 are below fp32 rounding).  Six bf16 MFMAs cost 6 x 32 cycles per
// 32x32x16 block against 8 x 64 for v_mfma_f32_32x32x2_f32: 2.7x the fp32 MFMA rate.
//
// out[b][m][p] = rstd(b,p) * sum_k A[m][k] x[b][k][p]   (rstd = 1 without LN)
// With LN (CustomLayerNorm folded, REF:911-925): A = W1 . diag(ln_w) and
// rstd = 1 / sqrt(var_unbiased_k(x[b][:][p]) + 1e-5), computed in-kernel from the
// x column the wave already holds.
//
// Workgroup = 4 waves x 32 pixels; every wave keeps its pixels' K-column as split B
// fragments in registers and walks ALL M rows in chunks of 64 (two 32-row MFMA
// tiles).  A (pre-split, fragment order, lnb_x3_pack_kernel) streams through a 2-slot
// LDS-DMA ring shared by the 4 waves.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t bf16_rne(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_val(uint32_t h) { return __builtin_bit_cast(float, h << 16); }
// exact 3-term split: returns the bf16 bit patterns of v0, v1, v2
__device__ __forceinline__ void split3(float v, uint32_t& h0, uint32_t& h1, uint32_t& h2) {
  h0 = bf16_rne(v);
  const float r1 = v - bf16_val(h0);
  h1 = bf16_rne(r1);
  const float r2 = r1 - bf16_val(h1);
  h2 = bf16_rne(r2);
}

// the same exact split of 8 values with the hardware RNE conversion (v_cvt_pk_bf16_f32: two values per
// instruction; the residuals come back through a shift / mask): about half the vector instructions of
// the integer-rounding split3 above, the same bits for finite values
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

#ifndef GRR_X3_TILES
#define GRR_X3_TILES 1   // 32-row chunks: 36 KB LDS ring at K = 96 -> 4 workgroups per CU (2 tiles: 2.38 -> 1 tile: 1.88 ms per bench step)
#endif
constexpr int X3_NT = GRR_X3_TILES;  // 32-row MFMA tiles per chunk
constexpr int X3_MCH = 32 * X3_NT;   // output rows per chunk

// frag images per chunk: [tile t][k-step s][term q] x 64 lanes x 8 bf16 (1 KB each),
// padded to a whole number of 16-byte DMA instructions per wave (4 waves)
__host__ __device__ inline int x3_imgs(int KS) { return X3_NT * KS * 3; }
__host__ __device__ inline int x3_niw(int KS) { return (x3_imgs(KS) + 3) / 4; }
__host__ __device__ inline int64_t x3_chunk_bytes(int KS) { return (int64_t)x3_niw(KS) * 4 * 1024; }

// A[m][k] = W[m][k] * (ln_w ? ln_w[k] : 1), split and laid out in fragment order
__global__ void x3_pack_kernel(const float* __restrict__ w, const float* __restrict__ ln_w,
                               uint16_t* __restrict__ frag, int M, int K, int KS, int nch) {
  const int64_t per = x3_chunk_bytes(KS) / 2;        // bf16 per chunk image
  const int64_t n = per * nch;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i / per);
    const int e = (int)(i - (int64_t)c * per);
    const int img = e >> 9, lane = (e >> 3) & 63, j = e & 7;
    uint16_t out = 0;
    if (img < x3_imgs(KS)) {
      const int q = img % 3, s = (img / 3) % KS, t = img / (3 * KS);
      const int m = c * X3_MCH + t * 32 + (lane & 31), k = 16 * s + 8 * (lane >> 5) + j;
      if (m < M && k < K) {
        const float v = ln_w ? w[(int64_t)m * K + k] * ln_w[k] : w[(int64_t)m * K + k];
        uint32_t h0, h1, h2;
        split3(v, h0, h1, h2);
        out = (uint16_t)(q == 0 ? h0 : q == 1 ? h1 : h2);
      }
    }
    frag[i] = out;
  }
}

struct X3Args {
  const float* x;          // [B, K, P]
  const uint16_t* frag;    // [nch][x3_chunk_bytes / 2]
  float* out;              // [B, M, P]
  int64_t P;
  int K, M, nch, tiles;    // tiles: X3_PX-pixel tiles per image
  uint32_t nblk;
};


#ifndef GRR_X3_WAVES   // waves (32-pixel columns) per workgroup: the W chunk images DMA'd once serve them all
#define GRR_X3_WAVES 8
#endif
constexpr int X3_WV = GRR_X3_WAVES, X3_PX = 32 * X3_WV;   // pixels per workgroup
template <int KS, bool LN>
__global__ __launch_bounds__(64 * X3_WV) void gemm_x3_kernel(X3Args a) {
  extern __shared__ __attribute__((aligned(16))) float x3_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int b = lb / a.tiles, tile = lb - b * a.tiles;
  const int64_t P = a.P;
  const int K = a.K, M = a.M, r = lane & 31, hf = lane >> 5;
  const int64_t p = (int64_t)tile * X3_PX + wave * 32 + r;
  const bool pin = p < P;
  const int64_t pc = pin ? p : P - 1;
  const int NIW = x3_niw(KS);
  const int64_t CB = x3_chunk_bytes(KS);
  const int nch = a.nch;
  const char* fragb = reinterpret_cast<const char*>(a.frag);

  auto issue = [&](int c) {        // chunk c -> slot c & 1 (16-byte LDS-DMA, lane-linear)
    float* slot = x3_lds + (c & 1) * (CB / 4);
    const char* src = fragb + (int64_t)c * CB;
    for (int i = 0; i < (NIW * 4 + X3_WV - 1) / X3_WV; ++i) {
      const int img = i * X3_WV + wave;
      if (X3_WV > 4 && img >= NIW * 4) break;   // the chunk holds NIW * 4 images
      __builtin_amdgcn_global_load_lds((const void*)(src + img * 1024 + lane * 16),
                                       (__attribute__((address_space(3))) void*)(slot + img * 256), 16, 0, 0);
    }
  };
  issue(0);

  // this lane's K column: k = 16 s + 8 hf + j
  float xv[KS][8];
  // wave-uniform slab base + 32-bit lane offsets (K P < 2^30, checked on the host); rows past K load
  // row K - 1 and are zeroed by a select (no per-load branches)
  // (through a buffer descriptor: row 16 s + j in soffset, rows >= K past num_records read 0)
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(a.x + (int64_t)b * K * P), (short)0, (int)(4u * (uint32_t)K * (uint32_t)P), 0x00020000);
  const uint32_t xvo = 4u * ((uint32_t)(8 * hf) * (uint32_t)P + (uint32_t)pc), xPb = 4u * (uint32_t)P;
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      xv[s][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, xvo, (uint32_t)(16 * s + j) * xPb, 0));
  float rstd = 1.f;
  if constexpr (LN) {                          // CustomLayerNorm statistics (REF:916-922)
    float sum = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += xv[s][j];
    sum += __shfl_xor(sum, 32);
    const float mean = sum / (float)K;
    float sq = 0.f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = 16 * s + 8 * hf + j < K ? xv[s][j] - mean : 0.f;
        sq += d * d;
      }
    sq += __shfl_xor(sq, 32);
    rstd = 1.0f / sqrtf(sq / (float)(K - 1) + 1e-5f);
  }
  bf16x8 bq[KS][3];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    split3x8(xv[s], bq[s][0], bq[s][1], bq[s][2]);

  // the image's [M, P] output slab as a buffer resource ((M + 32) P < 2^30, checked on the host)
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)b * M * P, (short)0,
                                                                       (int)(4u * (uint32_t)M * (uint32_t)P), 0x00020000);
  const uint32_t Pb = 4u * (uint32_t)P;
  const uint32_t so = (uint32_t)((4 * hf) * P + pc) * 4u;
  for (int c = 0; c < nch; ++c) {
    // chunk c landed (this wave's DMAs; later ops: the previous chunk's stores), then all waves'
    if (c == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"i"(16 * X3_NT) : "memory");
    __builtin_amdgcn_s_barrier();
    if (c + 1 < nch) issue(c + 1);             // slot (c+1)&1 was last read in chunk c-1
    const float* slot = x3_lds + (c & 1) * (CB / 4);
    f32x16 acc[X3_NT];
#pragma unroll
    for (int t = 0; t < X3_NT; ++t) {
      acc[t] = f32x16{};
      const float* im = slot + (t * KS * 3) * 256 + lane * 4;
      bf16x8 a0 = *reinterpret_cast<const bf16x8*>(im);
      bf16x8 a1 = *reinterpret_cast<const bf16x8*>(im + 256);
      bf16x8 a2 = *reinterpret_cast<const bf16x8*>(im + 512);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        // prefetch the next k-step's fragments behind this step's six MFMAs
        bf16x8 n0 = a0, n1 = a1, n2 = a2;
        if (s + 1 < KS) {
          n0 = *reinterpret_cast<const bf16x8*>(im + (s + 1) * 768);
          n1 = *reinterpret_cast<const bf16x8*>(im + (s + 1) * 768 + 256);
          n2 = *reinterpret_cast<const bf16x8*>(im + (s + 1) * 768 + 512);
        }
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[s][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, bq[s][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[s][2], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq[s][0], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[s][1], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq[s][0], acc[t], 0, 0, 0);
        a0 = n0; a1 = n1; a2 = n2;
      }
    }
    // epilogue: 16 buffer stores per tile, row m0 in soffset; rows >= M fall past num_records and are
    // dropped; lanes past P (the image's last pixel tile) computed pixel P - 1 from the same x column
    // and store that same value there
#pragma unroll
    for (int t = 0; t < X3_NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t m0 = (uint32_t)(c * X3_MCH + t * 32 + (i & 3) + 8 * (i >> 2));
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[t][i] * rstd), ors, so, m0 * Pb, 0);
      }
  }
}

template <bool LN>
static grr_status launch_x3(const float* x, const uint16_t* frag, float* out, int B, int K, int M, int64_t P,
                            hipStream_t s, const char* name) {
  GRR_REQUIRE(K >= 1 && K <= 128, GRR_ERR_UNSUPPORTED, "%s: K=%d outside [1, 128]", name, K);
  GRR_REQUIRE((int64_t)(K + 16) * P < (1ll << 30) && (int64_t)(M + 32) * P < (1ll << 30), GRR_ERR_UNSUPPORTED,
              "%s: K*P or M*P too large for 32-bit offsets", name);
  X3Args a{};
  a.x = x; a.frag = frag; a.out = out; a.P = P; a.K = K; a.M = M;
  a.nch = (M + X3_MCH - 1) / X3_MCH;
  a.tiles = (int)((P + X3_PX - 1) / X3_PX);
  const uint64_t n = (uint64_t)B * a.tiles;
  GRR_REQUIRE(n < (1ull << 31), GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  a.nblk = (uint32_t)n;
  const int KS = (K + 15) / 16;
  const size_t lds = 2 * (size_t)x3_chunk_bytes(KS);
  switch (KS) {
#define GRR_X3_CASE(ks) \
    case ks: hipLaunchKernelGGL((gemm_x3_kernel<ks, LN>), dim3(a.nblk), dim3(64 * X3_WV), lds, s, a); break;
    GRR_X3_CASE(1) GRR_X3_CASE(2) GRR_X3_CASE(3) GRR_X3_CASE(4)
    GRR_X3_CASE(5) GRR_X3_CASE(6) GRR_X3_CASE(7) GRR_X3_CASE(8)
#undef GRR_X3_CASE
  }
  return launch_status(name);
}

// ---------------------------------------------------------------------------
// The same fp32-accurate 1x1 convolution for deep inputs (K > 128: the training reverse's
// W1^T gh (K = 2 hid), the v1.0 widths): a wave can no longer hold its pixels' K column, so the
// loop order flips.  A workgroup = 8 waves x 32 pixels x one M tile of 32 TM rows; the
// accumulators of all TM row tiles stay in registers while K streams by 16-deep k-steps: each
// wave loads its pixels' 16 x rows two steps ahead (rows 16 s + 8 hf + j, 128-B coalesced per
// half-wave), splits them in registers, and multiplies them with the row tiles' split W
// fragments (x3_pack_kernel's images, [32-row group][k-step][term]), which arrive by LDS-DMA in
// a 3-slot ring of X3K_KC k-steps shared by the 8 waves, two chunks ahead.
// ---------------------------------------------------------------------------
constexpr int X3K_KC = 2;   // k-steps per ring slot (3 slots: 72 KB at 4 row tiles, two workgroups per CU)

// 16-byte LDS-DMA (lane l -> LDS m0 + 16 l) as an asm statement: hipcc answers the LDS-DMA builtin with
// vmcnt(0) before every later LDS read (it cannot order the DMA's LDS write against them), which drains
// the x loads the k-loop keeps two steps ahead.  The ring is ordered by the kernel itself (counted
// vmcnt + barrier per chunk); the compiler's own counted waits stay correct with these extra,
// uncounted operations in flight (vmcnt retires loads in order: a wait only gets stricter).
typedef __attribute__((address_space(3))) float* x3_lds_t;
__device__ __forceinline__ void x3_dma16(const void* src, const float* lds_wave_base) {
  const uint32_t m0v = (uint32_t)(uintptr_t)(x3_lds_t)lds_wave_base;
  asm volatile("global_load_lds_dwordx4 %0, off" ::"v"(src), "{m0}"(__builtin_amdgcn_readfirstlane(m0v)) : "memory");
}

enum { X3K_STORE = 0, X3K_LN = 1, X3K_SKIP = 2 };
struct X3KArgs {
  const float* x;          // [B, K, P]
  const float* sd;         // X3K_LN: [B, P] per-pixel scale 1 / sqrt(var + eps) (ln_stats_kernel)
  const float* res;        // X3K_SKIP: [B, M, P]
  const float* skip;       // X3K_SKIP: [2], out = skip0 res + skip1 acc
  const uint16_t* frag;    // x3_pack_kernel layout, X3_NT = 1: [32-row group][x3_chunk_bytes(KS) / 2]
  float* out;              // [B, M, P]
  int64_t P;
  int K, M, KS, ngroups, nmt, tiles;
  int64_t CB;              // bytes per 32-row group image
  uint32_t nblk;
};

template <int TM, int EPI>
__global__ __launch_bounds__(64 * X3_WV, 4) void gemm_x3k_kernel(X3KArgs a) {
  static_assert(X3_NT == 1, "gemm_x3k_kernel reads the one-tile pack layout");
  extern __shared__ __attribute__((aligned(16))) float x3_lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  uint32_t lb = xcd_remap(blockIdx.x, a.nblk);
  const int mt = (int)(lb % (uint32_t)a.nmt);   // the M tiles of one pixel tile are neighbours (shared x rows)
  lb /= (uint32_t)a.nmt;
  const int tile = (int)(lb % (uint32_t)a.tiles), b = (int)(lb / (uint32_t)a.tiles);
  const int64_t P = a.P;
  const int K = a.K, M = a.M, KS = a.KS, r = lane & 31, hf = lane >> 5;
  const int64_t p = (int64_t)tile * X3_PX + wave * 32 + r;
  const bool pin = p < P;
  const int64_t pc = pin ? p : P - 1;
  const char* fragb = reinterpret_cast<const char*>(a.frag);
  constexpr int SLOT = X3K_KC * TM * 3 * 256;    // floats per ring slot (1 KB images)
  const int nch = (KS + X3K_KC - 1) / X3K_KC;

  // chunk c -> slot c % 3: images [s][t][q] for k-steps c KC .. c KC + KC - 1, row tiles t < TM.  This
  // wave's images i = wave + X3_WV n and their fragment offsets are fixed across chunks (computed once:
  // the per-chunk address is one clamp and one multiply-add, not a div / mod chain in the scalar unit)
  constexpr int NIMG = X3K_KC * TM * 3, NI = (NIMG + X3_WV - 1) / X3_WV;
  int64_t img_src[NI];                          // wave-uniform (the lane's 16 bytes added at issue)
  int img_si[NI];
#pragma unroll
  for (int n = 0; n < NI; ++n) {
    const int i = wave + X3_WV * n;
    const int q = i % 3, t = (i / 3) % TM;
    int g = mt * TM + t;
    if (g >= a.ngroups) g = a.ngroups - 1;     // rows past M: any valid image (never stored)
    img_src[n] = (int64_t)g * a.CB + q * 1024;
    img_si[n] = i / (3 * TM);
  }
  auto issue = [&](int c, int slot_idx) {
    float* slot = x3_lds + slot_idx * SLOT;
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const int i = wave + X3_WV * n;
      if (NIMG % X3_WV == 0 || i < NIMG) {
        const int s = c * X3K_KC + img_si[n];
        const int ss = s < KS ? s : KS - 1;
        x3_dma16(fragb + img_src[n] + (int64_t)ss * 3072 + lane * 16, slot + i * 256);
      }
    }
  };

  // the image's [K, P] slab as a buffer resource: row 16 s + j + 8 hf of pixel pc at voffset
  // 4 (8 hf P + pc) + soffset 4 (16 s + j) P (wave-uniform, SGPR) -- no per-row address arithmetic in
  // the vector or scalar units; rows past K fall past num_records and read 0 ((K + 16) P < 2^30,
  // checked on the host)
  const float* xs = a.x + (int64_t)b * K * P;
  const uint32_t P32 = (uint32_t)P, pc32 = (uint32_t)pc;
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xs), (short)0, (int)(4u * (uint32_t)K * P32), 0x00020000);
  const uint32_t voff = 4u * ((uint32_t)(8 * hf) * P32 + pc32), Pb = 4u * P32;
  auto load = [&](int s, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, voff, (uint32_t)(16 * s + j) * Pb, 0));
  };

  f32x16 acc[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) acc[t] = f32x16{};

  // 3-slot ring, chunks two ahead.  Per wave and chunk: its DMAs of chunk c + 2 (at least DMIN),
  // then 8 KC dword x loads (the k-steps one chunk ahead), in that order.
  constexpr int DMIN = X3K_KC * TM * 3 / X3_WV;
  issue(0, 0);
  if (nch > 1) issue(1, 1);
  float x0[8], x1[8];
  load(0, x0);
  load(1 < KS ? 1 : 0, x1);
  static_assert(X3K_KC == 2, "two k-steps per chunk: x0 / x1 alternate by step parity");
  // one k-step: split this step's x (loaded two steps ago), reload the buffer two steps ahead, multiply
  auto kstep = [&](const float* slot, int s, int si, float (&xb)[8]) __attribute__((always_inline)) {
    bf16x8 bq0, bq1, bq2;
    split3x8(xb, bq0, bq1, bq2);
    // the scheduler would otherwise sink the reload below the other buffer's split (which then waits on
    // loads issued just before it, vmcnt(0))
    __builtin_amdgcn_sched_barrier(0);
    load(s + 2 < KS ? s + 2 : KS - 1, xb);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const float* im = slot + (si * TM * 3 + t * 3) * 256 + lane * 4;
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(im);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(im + 256);
      const bf16x8 a2 = *reinterpret_cast<const bf16x8*>(im + 512);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq1, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, bq0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq2, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bq0, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq1, acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bq0, acc[t], 0, 0, 0);
    }
  };
  // chunk c: this wave's DMAs of chunk c landed (younger: chunk c - 2's x loads, chunk c + 1's DMAs if
  // any, chunk c - 1's x loads), then every wave's; one barrier per chunk: a wave at it has finished
  // reading the slot the next issue() overwrites
  auto chunk_top = [&](int c) __attribute__((always_inline)) {
    if (c == 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (c + 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(32 + DMIN) : "memory");
    else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");               // the slot's LDS reads stay below the barrier
    const int sc = c % 3;
    if (c + 2 < nch) issue(c + 2, sc == 0 ? 2 : sc - 1);   // slot (c + 2) % 3 was last read in chunk c - 1
    return x3_lds + sc * SLOT;
  };
  // whole chunks in a branch-free body (x0 / x1 always in the same order, so the compiler's counted
  // waits before each split allow the other buffer's eight loads in flight), the odd k-step after
  const int nfull = KS / X3K_KC;
  for (int c = 0; c < nfull; ++c) {
    const float* slot = chunk_top(c);
    kstep(slot, c * X3K_KC, 0, x0);
    kstep(slot, c * X3K_KC + 1, 1, x1);
  }
  if (nfull < nch) {
    const float* slot = chunk_top(nfull);
    kstep(slot, nfull * X3K_KC, 0, x0);
  }
  float cs = 1.f, s0 = 0.f, s1 = 1.f;
  if constexpr (EPI == X3K_LN) cs = a.sd[(int64_t)b * P + pc];   // CustomLayerNorm 1/sigma (REF:921-922)
  if constexpr (EPI == X3K_SKIP) { s0 = a.skip[0]; s1 = a.skip[1]; }
  // row m = 32 g + (i & 3) + 8 (i >> 2) + 4 hf through buffer descriptors of the image's [M, P] slabs: the
  // lane's 4 (4 hf P + pc) in voffset, the row's 4 m P in soffset ((M + 32) P < 2^30, checked on the
  // host); rows >= M fall past num_records (stores dropped); lanes past P computed pixel P - 1 from the
  // same x column and store that same value there
  const uint32_t MPb = 4u * (uint32_t)M * P32;
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(a.out + (int64_t)b * M * P, (short)0, (int)MPb,
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t rrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(EPI == X3K_SKIP ? a.res + (int64_t)b * M * P : a.out), (short)0,
      EPI == X3K_SKIP ? (int)MPb : 0, 0x00020000);
  const uint32_t eoff = 4u * ((uint32_t)(4 * hf) * P32 + pc32);
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t mr = (uint32_t)((mt * TM + t) * 32 + (i & 3) + 8 * (i >> 2));
      float v = acc[t][i];
      if constexpr (EPI == X3K_LN) v *= cs;
      if constexpr (EPI == X3K_SKIP)   // REF:962-964
        v = s0 * __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, eoff, mr * Pb, 0)) + s1 * v;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ors, eoff, mr * Pb, 0);
    }
}

template <int EPI = X3K_STORE>
static grr_status launch_x3k(const float* x, const uint16_t* frag, float* out, int B, int K, int M, int64_t P,
                             hipStream_t s, const char* name, const float* sd = nullptr, const float* res = nullptr,
                             const float* skip = nullptr) {
  GRR_REQUIRE((int64_t)(K + 16) * P < (1ll << 30) && (int64_t)(M + 128) * P < (1ll << 30), GRR_ERR_UNSUPPORTED,
              "%s: K*P or M*P too large for 32-bit offsets", name);
  X3KArgs a{};
  a.x = x; a.frag = frag; a.out = out; a.P = P; a.K = K; a.M = M; a.sd = sd; a.res = res; a.skip = skip;
  a.KS = (K + 15) / 16;
  a.ngroups = (M + 31) / 32;
  a.CB = x3_chunk_bytes(a.KS);
  a.tiles = (int)((P + X3_PX - 1) / X3_PX);
  // row tiles per workgroup: all of M up to 128 rows, else 4 (128-row M tiles)
  const int TM = a.ngroups >= 4 ? 4 : a.ngroups;
  a.nmt = (a.ngroups + TM - 1) / TM;
  const uint64_t n = (uint64_t)B * a.tiles * a.nmt;
  GRR_REQUIRE(n < (1ull << 31), GRR_ERR_UNSUPPORTED, "%s: grid too large", name);
  a.nblk = (uint32_t)n;
  const size_t lds = 3 * (size_t)X3K_KC * TM * 3 * 1024;
  switch (TM) {
    case 1: hipLaunchKernelGGL((gemm_x3k_kernel<1, EPI>), dim3(a.nblk), dim3(64 * X3_WV), lds, s, a); break;
    case 2: hipLaunchKernelGGL((gemm_x3k_kernel<2, EPI>), dim3(a.nblk), dim3(64 * X3_WV), lds, s, a); break;
    case 3: hipLaunchKernelGGL((gemm_x3k_kernel<3, EPI>), dim3(a.nblk), dim3(64 * X3_WV), lds, s, a); break;
    default: hipLaunchKernelGGL((gemm_x3k_kernel<4, EPI>), dim3(a.nblk), dim3(64 * X3_WV), lds, s, a); break;
  }
  return launch_status(name);
}

// out[b, g Cin + c] = img[b, c]: one thread per 4 consecutive pixels of one (b, c) plane reads
// them once (16-byte load) and writes the G copies (16-byte stores); store-bandwidth bound.
__global__ void repeat_graphs_kernel(const float* __restrict__ img, float* __restrict__ out, int Cin, int G,
                                     int64_t P, int64_t nq) {
  const int64_t P4 = P / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t plane = i / P4, q = i - plane * P4;      // plane = b Cin + c
    const int64_t b = plane / Cin, c = plane - b * Cin;
    const float4 v = reinterpret_cast<const float4*>(img + plane * P)[q];
    float4* o = reinterpret_cast<float4*>(out + (b * G * Cin + c) * P) + q;
    for (int g = 0; g < G; ++g) o[g * Cin * P4] = v;
  }
}
__global__ void repeat_graphs_scalar_kernel(const float* __restrict__ img, float* __restrict__ out, int Cin, int G,
                                            int64_t P, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % P, plane = i / P;
    const int64_t b = plane / Cin, c = plane - b * Cin;
    const float v = img[i];
    for (int g = 0; g < G; ++g) out[((b * G + g) * Cin + c) * P + p] = v;
  }
}

}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_conv1x1(const float* x, const float* wt, float* out, int B, int K, int M, int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(x && wt && out && B > 0 && K > 0 && M > 0 && P > 0, GRR_ERR_INVALID_ARG, "grr_conv1x1: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_conv1x1: out aliases x");
  GemmArgs a{};
  a.x = x; a.wt = wt; a.out = out; a.K = K; a.M = M; a.P = P;
  return launch_gemm<LD_PLAIN, EP_STORE>(a, B, (hipStream_t)stream, "grr_conv1x1");
}

int64_t grr_conv1x1_workspace_bytes(int K, int M) {
  if (K < 1 || K > 4096 || M < 1) return 0;
  const int KS = (K + 15) / 16, nch = (M + X3_MCH - 1) / X3_MCH;
  return (int64_t)nch * x3_chunk_bytes(KS);
}

grr_status grr_conv1x1_ws(const float* x, const float* wt, float* out, void* workspace, int B, int K, int M,
                          int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(x && wt && out && workspace && B > 0 && K > 0 && M > 0 && P > 0, GRR_ERR_INVALID_ARG,
              "grr_conv1x1_ws: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_conv1x1_ws: out aliases x");
  GRR_REQUIRE(K <= 4096, GRR_ERR_UNSUPPORTED, "grr_conv1x1_ws: K=%d > 4096", K);
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0, GRR_ERR_INVALID_ARG, "grr_conv1x1_ws: workspace not 256-B aligned");
  GRR_REQUIRE(P * 16 < (1ll << 31), GRR_ERR_UNSUPPORTED, "grr_conv1x1_ws: P too large");
  hipStream_t s = (hipStream_t)stream;
  const int KS = (K + 15) / 16, nch = (M + X3_MCH - 1) / X3_MCH;
  uint16_t* frag = (uint16_t*)workspace;
  const int64_t nf = (int64_t)nch * x3_chunk_bytes(KS) / 2;
  hipLaunchKernelGGL(x3_pack_kernel, dim3((unsigned)std::min<int64_t>((nf + 255) / 256, 1 << 16)), dim3(256), 0, s,
                     wt, nullptr, frag, M, K, KS, nch);
  grr_status st = launch_status("grr_conv1x1_ws/pack");
  if (st != GRR_OK) return st;
  if ((int64_t)K * P >= (1ll << 30) || (int64_t)M * P >= (1ll << 30)) {   // past the 32-bit lane offsets
    GemmArgs g{};
    g.x = x; g.wt = wt; g.out = out; g.K = K; g.M = M; g.P = P;
    return launch_gemm<LD_PLAIN, EP_STORE>(g, B, s, "grr_conv1x1_ws/fp32");
  }
  if (K > 128) return launch_x3k(x, frag, out, B, K, M, P, s, "grr_conv1x1_ws");
  return launch_x3<false>(x, frag, out, B, K, M, P, s, "grr_conv1x1_ws");
}

grr_status grr_conv2x2s2(const float* x, const float* wt, float* out, int B, int K, int M, int H, int W,
                         void* stream) {
  clear_error();
  GRR_REQUIRE(x && wt && out && B > 0 && K > 0 && M > 0 && H > 1 && W > 1, GRR_ERR_INVALID_ARG,
              "grr_conv2x2s2: bad args");
  GemmArgs a{};
  a.x = x; a.wt = wt; a.out = out; a.K = 4 * K; a.M = M; a.P = (int64_t)(H / 2) * (W / 2);
  a.Hin = H; a.Win = W; a.Wo = W / 2;
  return launch_gemm<LD_IM2COL, EP_STORE>(a, B, (hipStream_t)stream, "grr_conv2x2s2");
}

}  // extern "C"

namespace grr {

// Unfused block pipeline for the wide blocks:
//   FFN = true:  FeedForward block of the window models' feature CNN (FFBlock, REF7:13-67):
//                n = ln_w * x / sqrt(var_c x + 1e-5);  h = W_in n;  x1, x2 = dwconv3x3_zero(h);
//                out = s0 x + s1 W_out (gelu(x1) * x2)
//   FFN = false: LocalNonLinearBlock with C > 128 (the v1.0 widths 192 / 384; REF:911-964): replicate
//                depthwise, g = sigmoid(m) m v  (C <= 128 runs the fused head / mix kernels, lnb_ops.hip)
// W_in on the split-bf16 GEMM with the LN folded (K = C <= 128: statistics in-kernel; deeper: the
// K-streaming kernel with ln_stats' per-pixel scale in its epilogue), the depthwise + gate as one
// memory-bound pass, W_out + skip on the K-streaming kernel's skip epilogue.
// Workspace (floats, 64-aligned pieces): sd [B P], h [B 2hid P], g [B hid P], W_in / W_out fragments.
struct FfnLayout {
  int64_t sd, h, g, f1, f2, total;
  int KS1, nch1, KS2, nch2;
};
static int64_t a64(int64_t n) { return (n + 63) / 64 * 64; }
static FfnLayout ffn_layout(int B, int C, int hid, int64_t P) {
  FfnLayout L{};
  L.KS1 = (C + 15) / 16; L.nch1 = (2 * hid + 31) / 32;
  L.KS2 = (hid + 15) / 16; L.nch2 = (C + 31) / 32;
  L.sd = 0;
  L.h = a64((int64_t)B * P);
  L.g = L.h + a64((int64_t)B * 2 * hid * P);
  L.f1 = L.g + a64((int64_t)B * hid * P);
  L.f2 = L.f1 + a64((int64_t)L.nch1 * x3_chunk_bytes(L.KS1) / 4);
  L.total = L.f2 + a64((int64_t)L.nch2 * x3_chunk_bytes(L.KS2) / 4);
  return L;
}

template <bool FFN>
static grr_status block_x3_forward(const float* x, const float* ln_w, const float* w_in, const float* w_dw,
                                   const float* w_out, const float* skip, float* out, float* ws, int B, int C,
                                   int hid, int H, int W, hipStream_t s) {
  const int64_t P = (int64_t)H * W;
  const FfnLayout L = ffn_layout(B, C, hid, P);
  float* sd = ws + L.sd;
  float* hbuf = ws + L.h;
  float* gbuf = ws + L.g;
  uint16_t* f1 = reinterpret_cast<uint16_t*>(ws + L.f1);
  uint16_t* f2 = reinterpret_cast<uint16_t*>(ws + L.f2);
  auto pack = [&](const float* w, const float* lw, uint16_t* frag, int M, int K, int KS, int nch) {
    const int64_t nf = (int64_t)nch * x3_chunk_bytes(KS) / 2;
    hipLaunchKernelGGL(x3_pack_kernel, dim3((unsigned)std::min<int64_t>((nf + 255) / 256, 1 << 16)), dim3(256), 0, s,
                       w, lw, frag, M, K, KS, nch);
    return launch_status("grr_ffn_forward/pack");
  };
  grr_status st = pack(w_in, ln_w, f1, 2 * hid, C, L.KS1, L.nch1);
  if (st != GRR_OK) return st;
  st = pack(w_out, nullptr, f2, C, hid, L.KS2, L.nch2);
  if (st != GRR_OK) return st;
  if (C <= 128) {
    st = launch_x3<true>(x, f1, hbuf, B, C, 2 * hid, P, s, "grr_ffn_forward/w_in");
  } else {
    GRR_REQUIRE((int64_t)B * ((P + 63) / 64) < (1ll << 31), GRR_ERR_UNSUPPORTED, "grr_ffn_forward: grid too large");
    hipLaunchKernelGGL(ln_stats_kernel, dim3((unsigned)((int64_t)B * ((P + 63) / 64))), dim3(64 * LN_G), 0, s, x, sd,
                       B, C, P);
    st = launch_status("grr_ffn_forward/ln_stats");
    if (st != GRR_OK) return st;
    st = launch_x3k<X3K_LN>(x, f1, hbuf, B, C, 2 * hid, P, s, "grr_ffn_forward/w_in", sd);
  }
  if (st != GRR_OK) return st;
  const int tx = (W + DT - 1) / DT, ty = (H + DT - 1) / DT;
  const uint64_t nb = (uint64_t)B * hid * tx * ty;
  GRR_REQUIRE(nb < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_ffn_forward: grid too large");
  hipLaunchKernelGGL(dw_gate_kernel<FFN>, dim3((unsigned)nb), dim3(256), 0, s, hbuf, w_dw, gbuf, hid, H, W, tx, ty,
                     (uint32_t)nb);
  st = launch_status("grr_ffn_forward/dw_gate");
  if (st != GRR_OK) return st;
  return launch_x3k<X3K_SKIP>(gbuf, f2, out, B, hid, C, P, s, "grr_ffn_forward/w_out", nullptr, x, skip);
}

}  // namespace grr

extern "C" {

int64_t grr_lnb_workspace_bytes(int B, int C, int hid, int H, int W) {
  if (B <= 0 || C <= 0 || hid <= 0 || H <= 0 || W <= 0) return 0;
  const int64_t f = C <= 128 ? grr::lnb_mfma_workspace_floats(B, C, hid, H, W)
                             : grr::ffn_layout(B, C, hid, (int64_t)H * W).total;
  return f * (int64_t)sizeof(float);
}

int64_t grr_lnb_fused_workspace_bytes(int C, int hid) {
  if (!grr::lnb_fused(C, hid)) return 0;
  return grr::fused_pack_floats(C, hid) * (int64_t)sizeof(float);
}

grr_status grr_lnb_forward(const float* x, const float* ln_w, const float* w1, const float* wdw, const float* w2,
                           const float* skip, float* out, void* workspace, int B, int C, int hid, int H, int W,
                           void* stream) {
  grr::clear_error();
  GRR_REQUIRE(x && ln_w && w1 && wdw && w2 && skip && out && workspace && B > 0 && C > 1 && hid > 0 && H > 0 &&
                  W > 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_forward: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_lnb_forward: out aliases x");
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0, GRR_ERR_INVALID_ARG, "grr_lnb_forward: workspace not 256-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (C <= 128)
    return grr::lnb_forward_mfma(x, ln_w, w1, wdw, w2, skip, out, (float*)workspace, B, C, hid, H, W, s);
  GRR_REQUIRE(C <= 4096 && hid <= 4096, GRR_ERR_UNSUPPORTED, "grr_lnb_forward: C=%d, hid=%d > 4096", C, hid);
  return grr::block_x3_forward<false>(x, ln_w, w1, wdw, w2, skip, out, (float*)workspace, B, C, hid, H, W, s);
}

grr_status grr_lnb_forward_c8(const float* x, const float* ln_w, const float* w1, const float* wdw, const float* w2,
                              const float* skip, float* out, void* workspace, int B, int C, int hid, int H, int W,
                              int layout, void* stream) {
  grr::clear_error();
  GRR_REQUIRE(x && ln_w && w1 && wdw && w2 && skip && out && workspace && B > 0 && C > 1 && hid > 0 && H > 0 &&
                  W > 0 && layout >= 0 && layout <= 3,
              GRR_ERR_INVALID_ARG, "grr_lnb_forward_c8: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_lnb_forward_c8: out aliases x");
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_forward_c8: workspace 256-B, x and out 16-B aligned");
  GRR_REQUIRE(grr_lnb_fused(C, hid) && (int64_t)((C + 7) / 8) * 8 * H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_lnb_forward_c8: needs the fused pass (grr_lnb_fused) and 2^31 bytes per blocked image");
  return grr::lnb_forward_mfma(x, ln_w, w1, wdw, w2, skip, out, (float*)workspace, B, C, hid, H, W,
                               (hipStream_t)stream, false, layout);
}

// [B, C, H, W] <-> [B, ceil(C / 8), H, W, 8] (pad channels written as 0 / skipped)
namespace grr {
__global__ __launch_bounds__(256) void c8_pack_kernel(const float* __restrict__ x, float* __restrict__ y, int C, int64_t HW,
                                                     int64_t n) {   // n = B * NB * HW (one thread: 8 channels)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % HW, r = i / HW;
    const int nb = (C + 7) / 8, blk = (int)(r % nb);
    const int64_t b = r / nb;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * blk + j;
      v[j] = c < C ? x[(b * C + c) * HW + p] : 0.f;
    }
    float4* o = reinterpret_cast<float4*>(y + i * 8);
    o[0] = make_float4(v[0], v[1], v[2], v[3]);
    o[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}
__global__ __launch_bounds__(256) void c8_unpack_kernel(const float* __restrict__ y, float* __restrict__ x, int C,
                                                       int64_t HW, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i % HW, r = i / HW;
    const int nb = (C + 7) / 8, blk = (int)(r % nb);
    const int64_t b = r / nb;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 8 * blk + j;
      if (c < C) x[(b * C + c) * HW + p] = y[i * 8 + j];
    }
  }
}
}  // namespace grr

grr_status grr_c8_convert(const float* src, float* dst, int B, int C, int H, int W, int to_blocked, void* stream) {
  grr::clear_error();
  GRR_REQUIRE(src && dst && src != dst && B > 0 && C > 0 && H > 0 && W > 0 && ((uintptr_t)(to_blocked ? dst : src) & 15) == 0,
              GRR_ERR_INVALID_ARG, "grr_c8_convert: bad args (the blocked tensor 16-B aligned)");
  const int64_t HW = (int64_t)H * W, n = (int64_t)B * ((C + 7) / 8) * HW;
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
  if (to_blocked)
    hipLaunchKernelGGL(grr::c8_pack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src, dst, C, HW, n);
  else
    hipLaunchKernelGGL(grr::c8_unpack_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, src, dst, C, HW, n);
  return grr::launch_status("grr_c8_convert");
}

grr_status grr_lnb_forward_keep(const float* x, const float* ln_w, const float* w1, const float* wdw,
                                const float* w2, const float* skip, float* out, void* workspace, int B, int C,
                                int hid, int H, int W, void* stream) {
  grr::clear_error();
  GRR_REQUIRE(x && ln_w && w1 && wdw && w2 && skip && out && workspace && B > 0 && C > 1 && hid > 0 && H > 0 &&
                  W > 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_forward_keep: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_lnb_forward_keep: out aliases x");
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0, GRR_ERR_INVALID_ARG,
              "grr_lnb_forward_keep: workspace not 256-B aligned");
  GRR_REQUIRE(C <= 128, GRR_ERR_UNSUPPORTED, "grr_lnb_forward_keep: C=%d > 128", C);
  return grr::lnb_forward_mfma(x, ln_w, w1, wdw, w2, skip, out, (float*)workspace, B, C, hid, H, W,
                               (hipStream_t)stream, true);
}

grr_status grr_lnb_forward_rep(const float* src, int Cs, int R, const float* x, const float* ln_w, const float* w1,
                               const float* wdw, const float* w2, const float* skip, float* out, void* workspace,
                               int B, int hid, int H, int W, void* stream) {
  grr::clear_error();
  GRR_REQUIRE(src && ln_w && w1 && wdw && w2 && skip && out && workspace && B > 0 && Cs > 0 && R > 0 &&
                  hid > 0 && H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_lnb_forward_rep: bad args");
  GRR_REQUIRE(out != x && out != src, GRR_ERR_INVALID_ARG, "grr_lnb_forward_rep: out aliases an input");
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0, GRR_ERR_INVALID_ARG,
              "grr_lnb_forward_rep: workspace not 256-B aligned");
  GRR_REQUIRE(R * Cs <= 128, GRR_ERR_UNSUPPORTED, "grr_lnb_forward_rep: R*Cs=%d > 128", R * Cs);
  return grr::lnb_forward_mfma_rep(src, Cs, R, x, ln_w, w1, wdw, w2, skip, out, (float*)workspace, B, hid, H, W,
                                   (hipStream_t)stream);
}

int64_t grr_ffn_workspace_bytes(int B, int C, int hid, int H, int W) {
  if (B <= 0 || C <= 1 || hid <= 0 || H <= 0 || W <= 0) return 0;
  return grr::ffn_layout(B, C, hid, (int64_t)H * W).total * (int64_t)sizeof(float);
}

grr_status grr_ffn_forward(const float* x, const float* ln_w, const float* w_in, const float* w_dw, const float* w_out,
                           const float* skip, float* out, void* workspace, int B, int C, int hid, int H, int W,
                           void* stream) {
  grr::clear_error();
  GRR_REQUIRE(x && ln_w && w_in && w_dw && w_out && skip && out && workspace && B > 0 && C > 1 && hid > 0 &&
                  H > 0 && W > 0,
              GRR_ERR_INVALID_ARG, "grr_ffn_forward: bad args");
  GRR_REQUIRE(out != x, GRR_ERR_INVALID_ARG, "grr_ffn_forward: out aliases x");
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0, GRR_ERR_INVALID_ARG, "grr_ffn_forward: workspace not 256-B aligned");
  GRR_REQUIRE(C <= 4096 && hid <= 4096, GRR_ERR_UNSUPPORTED, "grr_ffn_forward: C=%d, hid=%d > 4096", C, hid);
  return grr::block_x3_forward<true>(x, ln_w, w_in, w_dw, w_out, skip, out, (float*)workspace, B, C, hid, H, W,
                                     (hipStream_t)stream);
}

grr_status grr_repeat_graphs(const float* img, float* out, int B, int Cin, int G, int64_t P, void* stream) {
  clear_error();
  GRR_REQUIRE(img && out && B > 0 && Cin > 0 && G > 0 && P > 0, GRR_ERR_INVALID_ARG, "grr_repeat_graphs: bad args");
  const int64_t n = (int64_t)B * Cin * P;   // input elements
  if (P % 4 == 0 && (uintptr_t)img % 16 == 0 && (uintptr_t)out % 16 == 0) {
    const int64_t nq = n / 4;
    const int blocks = (int)std::min<int64_t>((nq + 255) / 256, 1 << 16);
    hipLaunchKernelGGL(repeat_graphs_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, img, out, Cin, G, P, nq);
  } else {
    const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1 << 16);
    hipLaunchKernelGGL(repeat_graphs_scalar_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, img, out, Cin,
                       G, P, n);
  }
  return launch_status("grr_repeat_graphs");
}

}  // extern "C"
