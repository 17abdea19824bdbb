// gfx950 weight-gradient reductions of the training step (reverse of the feature CNN's 1x1 / 2x2-s2
// convolutions and of LocalNonLinearBlock's W1 / W2; REF:556-612, REF13:564-575 under autograd):
//
//   out[m][k] = sum_b sum_p A[b][m][p] * Bop[b][k][p]      A [B, M, P], Bop [B, K, P]
//
// a reduction over all B*P pixels into a small M x K matrix.  Both operands are pixel-contiguous,
// which is the layout v_mfma_f32_32x32x16_bf16 consumes without any LDS staging: lane l of a wave holds
// A[row l & 31][8 consecutive pixels] and Bop[row l & 31][the same pixels], the pixels being the MFMA's
// k index (two dwordx4 loads per row and step).  Both operands are split exactly into three bf16 terms
// in registers (six products, fp32-accurate: the arithmetic class of the reference's fp32 autograd
// GEMM), summed in a fixed order.
//
// Work split: one wave = one (32 TA x 32 TB) output tile x one pixel chunk of one image; the tiles of
// a chunk are neighbouring waves (xcd_remap keeps them on one XCD, so the chunk's rows are read from
// HBM once and served to the other tiles from L2).  Each wave writes its partial tile to a workspace
// [chunks][M][K]; a second kernel adds the chunks in index order.  No atomics and no wave ever waits
// on another: the result is deterministic and the kernel cannot stall behind a concurrent launch on
// another stream (the library GEMMs it replaces are stream-K kernels whose workgroups wait on each
// other's partial tiles).
#include "grr_common.h"

#include <cstdlib>

namespace grr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct WgArgs {
  const float* a;      // [B, M, P]
  const float* bop;    // [B, K, P]
  float* ws;           // [nchunk, M, K]
  int M, K;            // rows of a, rows of bop
  int64_t osa, osb;    // ws element (row of a, row of bop) at ra * osa + rb * osb within a chunk
  int64_t P;
  int64_t CP;          // pixels per chunk (multiple of 32)
  int cpi;             // chunks per image
  int nta, ntb;        // output tiles along M (32 TA rows) and K (32 TB columns)
  uint32_t nblk;
};

// output tile per wave: 32 TA x 32 TB (TA TB accumulators in AGPRs); wgrad_plan picks the tile.  (A
// 64 x 96 tile at two waves per SIMD measured slower than 128 x 96 on a 512 x 96 output, 1.03 vs 0.86 ms,
// it is taken only where 128 x 96 would be mostly padding.)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// exact split v = v0 + v1 + v2 of 8 values into bf16 terms (RNE casts: v_cvt_pk_bf16_f32)
__device__ __forceinline__ void wg_split3x8(const float (&v)[8], bf16x8& t0, bf16x8& t1, bf16x8& t2) {
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

// 16 pixels per step on v_mfma_f32_32x32x16_bf16: lane l holds k = 8 (l >> 5) + j, i.e. half-wave h
// takes pixels p0 + 8 h + j (one 32-B run per row and lane; the two halves cover 64 B of each row).
// Both operands are split exactly into three bf16 terms and the six products above 2^-24 |a b| are
// accumulated in fp32, smallest first (the x3 GEMM of feature_ops.hip / lnb_ops.hip: fp32-accurate,
// 2.7x the v_mfma_f32_32x32x2_f32 rate).  Row loads run two steps ahead.
template <int TA, int TB, bool VEC, int WPS>
__global__ __launch_bounds__(64, WPS) void wgrad_x3_kernel(WgArgs a) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const uint32_t id = xcd_remap(blockIdx.x, a.nblk);
  const int ntile = a.nta * a.ntb;
  const int tile = (int)(id % (uint32_t)ntile), chunk = (int)(id / (uint32_t)ntile);
  const int ta = tile % a.nta, tb = tile / a.nta;
  const int b = chunk / a.cpi, c = chunk - b * a.cpi;
  const int64_t P = a.P;
  const int64_t p_begin = (int64_t)c * a.CP;
  const int64_t p_end = p_begin + a.CP < P ? p_begin + a.CP : P;
  const int M = a.M, K = a.K;

  // rows of this lane, advanced to the chunk and the lane's 8-pixel run (rows past M / K are
  // clamped: they only feed accumulator rows that are never stored)
  const float* arow[TA];
  const float* brow[TB];
#pragma unroll
  for (int t = 0; t < TA; ++t) {
    const int m = ta * 32 * TA + 32 * t + r;
    arow[t] = a.a + ((int64_t)b * M + (m < M ? m : M - 1)) * P + p_begin + 8 * h;
  }
#pragma unroll
  for (int t = 0; t < TB; ++t) {
    const int k = tb * 32 * TB + 32 * t + r;
    brow[t] = a.bop + ((int64_t)b * K + (k < K ? k : K - 1)) * P + p_begin + 8 * h;
  }

  // full step at chunk offset o (wave-uniform; every lane's 8 pixels inside the chunk)
  auto load = [&](int o, float (&xa)[TA][8], float (&xb)[TB][8]) {
#pragma unroll
    for (int t = 0; t < TA; ++t) {
      if constexpr (VEC) {
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const float4 f = *reinterpret_cast<const float4*>(arow[t] + o + 4 * v);
          xa[t][4 * v] = f.x; xa[t][4 * v + 1] = f.y; xa[t][4 * v + 2] = f.z; xa[t][4 * v + 3] = f.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xa[t][j] = arow[t][o + j];
      }
    }
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      if constexpr (VEC) {
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const float4 f = *reinterpret_cast<const float4*>(brow[t] + o + 4 * v);
          xb[t][4 * v] = f.x; xb[t][4 * v + 1] = f.y; xb[t][4 * v + 2] = f.z; xb[t][4 * v + 3] = f.w;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xb[t][j] = brow[t][o + j];
      }
    }
  };

  f32x16 acc[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = f32x16{};

  bf16x8 fa[TA][3], fb[TB][3];
  auto split = [&](const float (&xa)[TA][8], const float (&xb)[TB][8]) {
#pragma unroll
    for (int t = 0; t < TA; ++t) wg_split3x8(xa[t], fa[t][0], fa[t][1], fa[t][2]);
#pragma unroll
    for (int t = 0; t < TB; ++t) wg_split3x8(xb[t], fb[t][0], fb[t][1], fb[t][2]);
  };
  auto mma = [&]() {
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
      }
  };

  // full steps, two load buffers: a buffer is refilled right after its split (the refill offset is
  // clamped to the last full step, so the loop body has no branches; surplus loads are discarded)
  const int ns = (int)((p_end - p_begin) / 16);
  const int last = ns > 0 ? 16 * (ns - 1) : 0;
  float ra0[TA][8], rb0[TB][8], ra1[TA][8], rb1[TB][8];
  if (ns > 0) {
    load(0, ra0, rb0);
    load(min(16, last), ra1, rb1);
    int i = 0;
    // split a buffer, refill it, then multiply: the refill is in flight for two steps of MFMAs.
    // sched_barrier: the scheduler would otherwise sink the refills below the MFMAs (loads one
    // step ahead instead of two, every load waited on at the loop top)
    for (; i + 1 < ns; i += 2) {
      const int o = 16 * i;
      split(ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);
      load(min(o + 32, last), ra0, rb0);
      __builtin_amdgcn_sched_barrier(0);
      mma();
      split(ra1, rb1);
      __builtin_amdgcn_sched_barrier(0);
      load(min(o + 48, last), ra1, rb1);
      __builtin_amdgcn_sched_barrier(0);
      mma();
    }
    if (i < ns) {
      split(ra0, rb0);
      mma();
    }
  }
  // ragged tail (< 16 pixels): guarded loads, pixels past the chunk read as zero
  const int rem = (int)(p_end - p_begin) - 16 * ns;
  if (rem > 0) {
    const int o = 16 * ns;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = 8 * h + j < rem;
#pragma unroll
      for (int t = 0; t < TA; ++t) ra0[t][j] = ok ? arow[t][o + j] : 0.f;
#pragma unroll
      for (int t = 0; t < TB; ++t) rb0[t][j] = ok ? brow[t][o + j] : 0.f;
    }
    split(ra0, rb0);
    mma();
  }

  // partial tile -> ws[chunk][m][k]; accumulator element e of lane l is row (e & 3) + 8 (e >> 2) + 4 h,
  // column l & 31: the 32 lanes of a half-wave store 128 contiguous bytes of one row
  float* wsc = a.ws + (int64_t)chunk * M * K;
  const int64_t osa = a.osa, osb = a.osb;
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) {
      const int k = tb * 32 * TB + 32 * j + r;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = ta * 32 * TA + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M && k < K) wsc[m * osa + k * osb] = acc[i][j][e];
      }
    }
}

// out[i] = sum_c ws[c][i]: a workgroup = 64 consecutive outputs x RW waves; wave w adds chunks
// w, w + RW, ... (four running sums, fixed order), then the RW partials are added in wave order:
// deterministic.  (One thread per output looping over all chunks left ~3 waves per CU with one
// dependent-load chain each: 0.2-0.4 ms per call at the msgf shapes.)
constexpr int WG_RW = 16;
__global__ __launch_bounds__(64 * WG_RW) void wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                   float* __restrict__ out, int64_t n, int nchunk) {
  __shared__ float part[WG_RW][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    int c = w;
    for (; c + 3 * WG_RW < nchunk; c += 4 * WG_RW) {
      s0 += ws[(int64_t)c * n + i];
      s1 += ws[(int64_t)(c + WG_RW) * n + i];
      s2 += ws[(int64_t)(c + 2 * WG_RW) * n + i];
      s3 += ws[(int64_t)(c + 3 * WG_RW) * n + i];
    }
    for (; c < nchunk; c += WG_RW) s0 += ws[(int64_t)c * n + i];
  }
  part[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && i < n) {
    float t = part[0][lane];
#pragma unroll
    for (int q = 1; q < WG_RW; ++q) t += part[q][lane];
    out[i] = t;
  }
}

struct WgPlan {
  int ta, tb;          // 32-row tiles per wave along the a / bop rows
  int wps;             // waves per SIMD the instance is built for
  bool swap;           // operands exchanged (out^T = sum bop a^T): less tile padding
  int64_t CP;
  int cpi, nta, ntb;
  int64_t nchunk, nwaves;
};

// wave tiles built: 128 x 96 (the default), 192 x 64 (M x K = 192 x 48, the v1.0 model's first-level
// W1 gradient: one tile holds the whole output at 75 % use instead of two at 37.5 %) and 64 x 96 at
// two waves per SIMD (48 x 96, its W2 gradient).  The plan takes the cover of the output with the
// least measured cost: tiles x the tile's cost per pixel step relative to 128 x 96 (192 x 64: 1.05,
// its MFMA work plus eight operand blocks to split; 64 x 96: 0.8, measured at 96 x 192 on 256^2 x 32,
// where three of them ran 0.754 ms against two 128 x 96 tiles' 0.657 ms; profiles/r05/wgrad).
struct WgTile {
  int ta, tb, wps;
  float cost;
};
static constexpr WgTile kWgTiles[] = {{4, 3, 1, 1.0f}, {6, 2, 1, 1.05f}, {2, 3, 2, 0.8f}};
// 0: the 128 x 96 tile only (A/B and test knob; GRR_WGRAD_TILES=0 sets it for a whole run)
static int g_wgrad_tiles = [] {
  const char* e = std::getenv("GRR_WGRAD_TILES");
  return e && *e ? (std::atoi(e) != 0 ? 1 : 0) : 1;
}();

// chunks of whole 32-pixel steps sized for ~3 rounds of waves over the SIMDs, at most 4096 chunks and
// kWgradWsBudget bytes of workspace (the wide v1.0 LNB weights, 2 hid x C = 1536 x 384, would otherwise
// take 1024 x 2.4 MB); the operand order that pads the output tiles least
static constexpr int64_t kWgradWsBudget = 128ll << 20;

static WgPlan wgrad_plan(int B, int M, int K, int64_t P) {
  WgPlan p{};
  double best = 0.0;
  const int ntiles = g_wgrad_tiles ? (int)(sizeof(kWgTiles) / sizeof(kWgTiles[0])) : 1;
  for (int ti = 0; ti < ntiles; ++ti) {
    const WgTile t = kWgTiles[ti];
    for (int sw = 0; sw < 2; ++sw) {
      const int ma = sw ? K : M, kb = sw ? M : K;
      const int64_t na = (ma + 32 * t.ta - 1) / (32 * t.ta), nb = (kb + 32 * t.tb - 1) / (32 * t.tb);
      const double cost = (double)(na * nb) * t.cost;
      if (best == 0.0 || cost < best) {
        best = cost;
        p.ta = t.ta; p.tb = t.tb; p.wps = t.wps; p.swap = sw != 0;
        p.nta = (int)na; p.ntb = (int)nb;
      }
    }
  }
  const int64_t tiles = (int64_t)p.nta * p.ntb;
  const int64_t target = 3072 * p.wps;
  int64_t cp = ((int64_t)B * P * tiles + target - 1) / target;
  cp = (cp + 31) / 32 * 32;
  const int64_t pmax = (P + 31) / 32 * 32;
  if (cp < 512) cp = 512;
  if (cp > pmax) cp = pmax;
  for (;;) {
    p.cpi = (int)((P + cp - 1) / cp);
    p.nchunk = (int64_t)B * p.cpi;
    if ((p.nchunk <= 4096 && p.nchunk * (int64_t)M * K * (int64_t)sizeof(float) <= kWgradWsBudget) || cp >= pmax)
      break;
    cp = std::min<int64_t>(pmax, cp * 2);
  }
  p.CP = cp;
  p.nwaves = p.nchunk * tiles;
  return p;
}

}  // namespace grr

using namespace grr;

extern "C" {

grr_status grr_wgrad_set_tiles(int enable) {
  g_wgrad_tiles = enable ? 1 : 0;
  return GRR_OK;
}

int64_t grr_wgrad_workspace_bytes(int B, int M, int K, int64_t P) {
  if (B <= 0 || M <= 0 || K <= 0 || P <= 0) return 0;
  const WgPlan p = wgrad_plan(B, M, K, P);
  return p.nchunk * (int64_t)M * K * (int64_t)sizeof(float);
}

grr_status grr_wgrad(const float* a, const float* bop, float* out, void* workspace, int B, int M, int K, int64_t P,
                     void* stream) {
  clear_error();
  GRR_REQUIRE(a && bop && out && workspace && B > 0 && M > 0 && K > 0 && P > 0, GRR_ERR_INVALID_ARG,
              "grr_wgrad: bad args");
  GRR_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)bop & 15) == 0, GRR_ERR_INVALID_ARG,
              "grr_wgrad: operands not 16-B aligned");
  const WgPlan p = wgrad_plan(B, M, K, P);
  GRR_REQUIRE(p.nwaves < (1ll << 31), GRR_ERR_UNSUPPORTED, "grr_wgrad: grid too large");
  hipStream_t s = (hipStream_t)stream;
  WgArgs w{};
  w.a = p.swap ? bop : a; w.bop = p.swap ? a : bop; w.ws = (float*)workspace;
  w.M = p.swap ? K : M; w.K = p.swap ? M : K;
  w.osa = p.swap ? 1 : K; w.osb = p.swap ? K : 1;
  w.P = P; w.CP = p.CP; w.cpi = p.cpi; w.nta = p.nta; w.ntb = p.ntb; w.nblk = (uint32_t)p.nwaves;
  // 16-byte row loads need 4-aligned rows and chunk starts (CP is a multiple of 32)
  const dim3 g(w.nblk), t(64);
  const bool vec = P % 4 == 0;
#define GRR_WG_LAUNCH(TA, TB, WPS)                                                       \
  if (p.ta == TA && p.tb == TB) {                                                        \
    if (vec) hipLaunchKernelGGL((wgrad_x3_kernel<TA, TB, true, WPS>), g, t, 0, s, w);   \
    else hipLaunchKernelGGL((wgrad_x3_kernel<TA, TB, false, WPS>), g, t, 0, s, w);      \
  }
  GRR_WG_LAUNCH(4, 3, 1)
  else GRR_WG_LAUNCH(6, 2, 1)
  else GRR_WG_LAUNCH(2, 3, 2)
#undef GRR_WG_LAUNCH
  grr_status st = launch_status("grr_wgrad");
  if (st != GRR_OK) return st;
  const int64_t n = (int64_t)M * K;
  GRR_REQUIRE((n + 63) / 64 < (1ll << 31), GRR_ERR_UNSUPPORTED, "grr_wgrad: output too large");
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((uint32_t)((n + 63) / 64)), dim3(64 * WG_RW), 0, s,
                     (const float*)workspace, out, n, (int)p.nchunk);
  return launch_status("grr_wgrad/reduce");
}

}  // extern "C"
