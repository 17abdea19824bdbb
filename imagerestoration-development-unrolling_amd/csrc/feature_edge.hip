// The image filter's last feature 1x1 conv and the edge weights of both graph modules of a level in one pass
// (REF:146-175 extract_edge_weights / normalize_and_transform_features on the features of REF13:887-926's
// patchs_features_extraction 1x1 output).  Before, the 1x1 conv (C -> 2C, gemm_x3_kernel) wrote the [B, 2C, H, W]
// feature tensor and the edge-row kernel read it back: 768 + 768 B per pixel of HBM traffic between two
// launches.  Here the features never leave the CU.
//
// Workgroup = (b, 32-column strip, row segment), 9 waves:
//  * wave 8 (loader) streams the strip's input rows (the LocalNonLinearBlock output x, [B, C, H, W] or the
//    channel-blocked [B, C/8, H, W, 8] of grr_lnb_forward_c8) one row ahead, scales each pixel by a power of two
//    (its largest |x| into [2^13, 2^14)), splits it into exact-sum fp16 hi / lo terms in the layout of the
//    32x32x16 MFMA's B operand and writes them into a 2-slot LDS ring -- for the strip's 32 columns (main image)
//    and for its halo columns x0 - 1, x0 + 32, x0 + 33 (halo image, lanes 0, 31, 30);
//  * waves 0..7 each own 8 graphs of one slab (4 tiles of GTV features, 4 of GLR features; lane half kh
//    holds graphs 8 t + 4 kh .. + 3): per row, the 1x1 conv of both images on v_mfma_f32_32x32x16_f16 (three
//    products of the two-term splits; A = the wave's weight rows, staged in LDS, scaled by a power of two per
//    (slab, graph)) leaves each lane the 12 features (4 graphs x 3) of its column; normalisation (F.normalize *
//    multiM), the four neighbour similarities (left / right by DPP lane shifts, the strip-edge lanes from the
//    halo features, which a small per-wave LDS ring keeps for three rows; up / down from the previous rows'
//    registers), the softmax and (GTV) the pair weights follow in registers -- edge_row_kernel's expressions
//    with hardware reciprocal / sqrt / exp2 in place of the IEEE division sequences and expf (<= 2 ulp; the
//    conv's fp16 splits already make the weights fp32-class, not bitwise).
// Strips are 32-column aligned so that every store fills whole 128-B lines: 29-column strips (halo inside the
// window) wrote each line from two workgroups and ran 3.19 ms against 1.57 ms aligned (64 x 256^2).
// The power-of-two scales need no undoing: F.normalize is exact under them (sqrt and division commute with a
// power-of-two factor; the 1e-12 floor is scaled alike).
#include <type_traits>

#include "grr_common.h"

namespace grr {
namespace {

typedef _Float16 fe_f16x8 __attribute__((ext_vector_type(8)));
typedef float fe_f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t fe_u32x4 __attribute__((ext_vector_type(4)));
typedef float fe_f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 fe_f16x2 __attribute__((ext_vector_type(2)));

constexpr int FE_KS = 6;                 // k-steps of 16: input channels <= 96
constexpr int FE_GH = 4;                 // graphs per lane half (12 of the 16 accumulator rows)
constexpr int FE_TPS = 4;                // tiles (waves) per slab: G <= 32
constexpr int FE_NT = 2 * FE_TPS;        // compute waves
constexpr int FE_THREADS = 64 * (FE_NT + 1);
constexpr int FE_OWN = 32;                      // output columns per strip (32-aligned: whole 128-B lines)
constexpr int FE_IMG = FE_KS * 2 * 256;         // floats of one B image set (hi, lo per k-step)
constexpr int FE_SLOT = FE_IMG + 32;            // image set + the ep of its 32 pixels
constexpr int FE_AIMG = FE_KS * 2 * 256;        // floats of one tile's A images
constexpr int FE_HB = 8;                        // conv rows per halo batch (3 halo pixels a row: 24 B columns)
constexpr int FE_HR = FE_HB + 3, FE_HROW = 2 * 3 * 12;   // halo feature ring: rows, floats per row ([kh][L, R1, R2][12])
// A images, 2 main ring slots, 1 halo batch slot, per-wave halo feature rings
constexpr int FE_LDS = FE_NT * FE_AIMG + 3 * FE_SLOT + FE_NT * FE_HR * FE_HROW;
static_assert(FE_LDS * 4 <= 163840, "feature_edges LDS");
constexpr uint32_t FE_OOB = 0x80000000u;
// features carry sqrt(log2 e) (folded into multiM): a similarity is then log2(e) times REF's, the argument of
// v_exp_f32 (2^x) directly
constexpr float FE_SQRT_L2E = 1.2011224087864498f;
#ifndef FE_REMAP
#define FE_REMAP 1   // GLR tiles on the loader's SIMD (the compute waves' role map): 1.637 -> 1.604 ms at 64 x 256^2
#endif
#ifndef FE_SWAP
#define FE_SWAP 1   // GLR waves: edges before the conv (see iteration)
#endif
#ifndef FE_DIAG
#define FE_DIAG 0   // timing-only builds: 1 no stores, 2 no edge arithmetic, 4 no loads (loader), 8 no conv
#endif

struct FeArgs {
  const float* x;          // [B, C, H, W], or channel-blocked
  const char* pack;        // [tile][k-step][term] 1-KB A images (fe_pack_kernel)
  const int* sexp;         // [2][G] power-of-two scale of each (slab, graph)'s weight rows
  const float* multiM[2];  // [G, 3] per slab (GTV, GLR)
  float* w[2];             // raw weights [B, G, 4, H, W] per slab
  float* c;                // GTV pair weights [B, G, 2, H, W]
  int C, G, H, W, nstrips, sseg, nsegs;
  uint32_t nblk;
};

__device__ __forceinline__ int fe_scale_exp(float mx) {   // mx 2^s in [2^13, 2^14)
  if (mx == 0.f) return 0;
  int e;
  frexpf(mx, &e);
  return clampi(14 - e, -100, 100);
}
// (slab, graph) -> the exponent of its three weight rows
__device__ __forceinline__ int fe_graph_exp(const float* __restrict__ wf, int slab, int g, int G, int K) {
  float mx = 0.f;
  for (int f = 0; f < 3; ++f) {
    const float* row = wf + (int64_t)(slab * 3 * G + 3 * g + f) * K;
    for (int k = 0; k < K; ++k) mx = fmaxf(mx, fabsf(row[k]));
  }
  return fe_scale_exp(mx);
}

// A images: tile T (slab T / 4, graphs 8 (T % 4) ..), k-step s, term q; lane l, element j: A row i = l & 31
// (lane half kh = (i >> 2) & 1, accumulator register r = ((i >> 3) << 2) | (i & 3): graph 8 (T % 4) + 4 kh + r / 3,
// feature r % 3 for r < 12, else zero), k = 16 s + 8 (l >> 5) + j
__global__ void fe_pack_kernel(const float* __restrict__ wf, char* __restrict__ pack, int* __restrict__ sexp, int G,
                               int K) {
  const int n_img = FE_NT * FE_KS * 2 * 256;
  const int n = n_img + 2 * G;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (i >= n_img) {
      const int sg = i - n_img;
      sexp[sg] = fe_graph_exp(wf, sg / G, sg % G, G, K);
      continue;
    }
    const int img = i >> 8, e = i & 255;
    const int T = img / (FE_KS * 2), s = (img >> 1) % FE_KS, q = img & 1;
    const int l = e >> 2, jw = e & 3;
    const int ir = l & 31, khr = (ir >> 2) & 1, r = ((ir >> 3) << 2) | (ir & 3);
    const int slab = T / FE_TPS, g = 8 * (T % FE_TPS) + 4 * khr + r / 3;
    uint32_t word = 0;
    if (r < 3 * FE_GH && g < G) {
      const int row = slab * 3 * G + 3 * g + r % 3, sc = fe_graph_exp(wf, slab, g, G, K);
      float v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = 16 * s + 8 * (l >> 5) + 2 * jw + u;
        v[u] = k < K ? ldexpf(wf[(int64_t)row * K + k], sc) : 0.f;
      }
      const _Float16 h0 = (_Float16)v[0], h1 = (_Float16)v[1];
      const _Float16 t0 = q == 0 ? h0 : (_Float16)(v[0] - (float)h0), t1 = q == 0 ? h1 : (_Float16)(v[1] - (float)h1);
      word = (uint32_t)__builtin_bit_cast(uint16_t, t0) | ((uint32_t)__builtin_bit_cast(uint16_t, t1) << 16);
    }
    reinterpret_cast<uint32_t*>(pack)[i] = word;
  }
}

// (DPP moves are convergent: never sunk into a branch, where inactive lanes would read as 0.  No inline asm in
// the edge arithmetic: an asm statement ends the scheduling region and the conv MFMAs could not be spread over it)
__device__ __forceinline__ float fe_prev(float v) {   // lane - 1 (DPP wave shift; whole wave active)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float fe_next(float v) {   // lane + 1
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
}
template <int E>
__device__ __forceinline__ float fe_quad_e(float v) {   // every lane of a quad takes the quad's element E
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), E * 0x55, 0xF, 0xF, true));
}
__device__ __forceinline__ float fe_quad(float v, int e) {   // e a compile-time constant after unrolling
  return e == 0 ? fe_quad_e<0>(v) : e == 1 ? fe_quad_e<1>(v) : e == 2 ? fe_quad_e<2>(v) : fe_quad_e<3>(v);
}

template <bool IN8>
__global__ __launch_bounds__(FE_THREADS, 1) void feat_edge_kernel(FeArgs a) {
  // Explicit fmas only: an iteration is instantiated several times (phase, edge / conv flags), and contraction
  // left to the backend fused differently per instance -- a row's weights then depended on where its segment
  // started (1 ulp), which breaks bitwise batch independence (the segment length follows the batch size)
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float lds[FE_LDS];
  float* const aimg = lds;                         // [tile][k-step][term] A images
  float* const ring = aimg + FE_NT * FE_AIMG;      // [slot 0, 1]: main images + ep of their pixels
  float* const himg = ring + 2 * FE_SLOT;          // the halo batch image + ep
  float* const hring = himg + FE_SLOT;             // [wave][conv row % FE_HR][kh][L, R1, R2][12]: halo features
  const int lane = threadIdx.x & 63, kh = lane >> 5, n = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t unit = xcd_remap(blockIdx.x, a.nblk);
  const int strip = unit % a.nstrips;
  unit /= a.nstrips;
  const int seg = unit % a.nsegs;
  const int b = unit / a.nsegs;
  const int H = a.H, W = a.W, G = a.G, C = a.C;
  const int HW = H * W;
  const int x0 = strip * FE_OWN, col = x0 + n;     // the lane's column (main image)
  const int colc = clampi(col, 0, W - 1);
  const int r0 = seg * a.sseg, r1 = min(r0 + a.sseg, H);
  // a segment ending inside the image runs one more edge row (not stored) for its last row's c_v
  const int rend = r1 < H ? r1 + 1 : H;
  // iteration k: the conv of row r0 - 1 + k (clamped into the image; k <= rend - r0 + 1) and the edges of row
  // r0 - 3 + k (k >= 3)
  const int NI = rend - r0 + 3;
  const int NI3 = (NI + 2) / 3 * 3;

  // the tiles' A images into LDS (every workgroup reads the same 96 KB: L2)
  for (int i = threadIdx.x; i < FE_NT * FE_AIMG / 4; i += FE_THREADS)
    reinterpret_cast<fe_u32x4*>(aimg)[i] = reinterpret_cast<const fe_u32x4*>(a.pack)[i];

  if (wave == FE_NT) {
    // ---------------- loader: the main pixels of a row, one row ahead; the halo pixels of FE_HB rows at a time
    // halo batch m = conv rows (iterations) FE_HB m .. + FE_HB - 1: lane n < 24 holds row FE_HB m + n / 3, column
    // x0 - 1 (n % 3 = 0, the left neighbour L), x0 + 32 (1, the right neighbour R1), x0 + 33 (2, R1's right
    // neighbour R2, for the pair weight of column x0 + 31); lanes 24..31 repeat lane 23's pixel
    const int hn = min(n, 3 * FE_HB - 1);
    const int hcol = clampi(hn % 3 == 0 ? x0 - 1 : (hn % 3 == 1 ? x0 + 32 : x0 + 33), 0, W - 1);
    const int cx = IN8 ? 8 * ((C + 7) / 8) : C;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x + (int64_t)b * cx * HW), 0, (int)((int64_t)cx * HW * 4), 0x00020000);
    float v[2][FE_KS][8];
    auto load = [&](int set, int gy, int cc) __attribute__((always_inline)) {
      if (FE_DIAG & 4) return;
      int hw4 = __builtin_amdgcn_readfirstlane(HW * 4);
      asm volatile("" : "+s"(hw4));
      if constexpr (IN8) {
        const uint32_t vo = (uint32_t)((kh * HW + gy * W + cc) * 32);
#pragma unroll
        for (int s = 0; s < FE_KS; ++s) {
          const fe_u32x4 lo =
              __builtin_bit_cast(fe_u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, 16 * s * hw4, 0));
          const fe_u32x4 hi =
              __builtin_bit_cast(fe_u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, vo + 16, 16 * s * hw4, 0));
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[set][s][j] = __uint_as_float(lo[j]);
            v[set][s][4 + j] = __uint_as_float(hi[j]);
          }
        }
      } else {
        const uint32_t vo = (uint32_t)((8 * kh * HW + gy * W + cc) * 4);
#pragma unroll
        for (int s = 0; s < FE_KS; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[set][s][j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, (16 * s + j) * hw4, 0));
      }
    };
    auto issue_main = [&](int k) { load(0, clampi(r0 - 1 + k, 0, H - 1), colc); };
    auto issue_halo = [&](int m) { load(1, clampi(r0 - 1 + FE_HB * m + hn / 3, 0, H - 1), hcol); };
    auto put = [&](int set, float* slot) __attribute__((always_inline)) {   // the loaded pixels of set -> a slot
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      float mx = 0.f;
#pragma unroll
      for (int s = 0; s < FE_KS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(v[set][s][j]));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const int ep = fe_scale_exp(mx);
#pragma unroll
      for (int s = 0; s < FE_KS; ++s) {
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const fe_f32x2 p = fe_f32x2{ldexpf(v[set][s][2 * j], ep), ldexpf(v[set][s][2 * j + 1], ep)};
          const fe_f16x2 h = __builtin_convertvector(p, fe_f16x2);
          const fe_f16x2 l = __builtin_convertvector(p - __builtin_convertvector(h, fe_f32x2), fe_f16x2);
          hw[j] = __builtin_bit_cast(uint32_t, h);
          lw[j] = __builtin_bit_cast(uint32_t, l);
        }
        *reinterpret_cast<fe_u32x4*>(slot + (2 * s) * 256 + 4 * lane) = fe_u32x4{hw[0], hw[1], hw[2], hw[3]};
        *reinterpret_cast<fe_u32x4*>(slot + (2 * s + 1) * 256 + 4 * lane) = fe_u32x4{lw[0], lw[1], lw[2], lw[3]};
      }
      if (kh == 0) reinterpret_cast<int*>(slot + FE_IMG)[n] = ep;
    };
    issue_main(0);
    issue_halo(0);
    put(0, ring);
    put(1, himg);
    issue_main(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // A images, slot 0 and halo batch 0
    asm volatile("" ::: "memory");
    for (int k = 0; k < NI3; ++k) {
      if (k + 1 <= NI - 2) {   // uniform: iterations 0 .. NI - 2 run a conv
        put(0, ring + ((k + 1) & 1) * FE_SLOT);
        if ((k + 1) % FE_HB == 0) put(1, himg);   // read by the compute waves in iteration k + 1 only
        if (k + 2 <= NI - 2) {
          issue_main(k + 2);
          if ((k + 2) % FE_HB == 0) issue_halo((k + 2) / FE_HB);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }

  // ---------------- compute wave: slab, tile
  // wave -> (slab, tile): waves w and w + 4 share a SIMD (a workgroup's waves cycle over the four), and the
  // loader (wave 8) joins waves 0 and 4 -- so those two take the lighter GLR tiles (no pair weights, no R1
  // softmax) and the GTV tiles go to the loader-free SIMDs
#if FE_REMAP
  const int slab = (0xD1 >> wave) & 1;                 // GLR: waves 0, 4, 6, 7 (tiles 0..3), GTV: 1, 5, 2, 3
  const int t4 = (0xE5E0 >> (2 * wave)) & 3;
#else
  const int slab = wave >> 2, t4 = wave & 3;
#endif
  const int gbase = 8 * t4 + 4 * kh;                 // the lane half's first graph
  if (8 * t4 >= G) {                                 // no graph in this tile: the barriers only
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    for (int k = 0; k <= NI3; ++k) __builtin_amdgcn_s_barrier();
    return;
  }
  // the compute of one slab, slab a compile-time constant so that a steady-state iteration (conv MFMAs, edge
  // arithmetic) is one basic block and the scheduler can overlap the MFMAs with the edges' VALU work
  auto run = [&](auto sl_tag) __attribute__((always_inline)) {
  constexpr int slab = decltype(sl_tag)::value;
  constexpr bool EDGES_FIRST = FE_SWAP && slab == 1;
  float M[FE_GH][3];
  int sg[FE_GH];
#pragma unroll
  for (int gi = 0; gi < FE_GH; ++gi) {
    const int g = min(gbase + gi, G - 1);
    sg[gi] = a.sexp[slab * G + g];
#pragma unroll
    for (int f = 0; f < 3; ++f) M[gi][f] = a.multiM[slab][g * 3 + f] * FE_SQRT_L2E;
  }
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      a.w[slab] + (int64_t)b * G * 4 * HW, 0, (int)((int64_t)G * 4 * HW * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      slab == 0 ? a.c + (int64_t)b * G * 2 * HW : nullptr, 0, slab == 0 ? (int)((int64_t)G * 2 * HW * 4) : 0,
      0x00020000);
  const bool lane_out = col < W;
  const float* const at = aimg + (4 * slab + t4) * FE_AIMG + 4 * lane;   // the tile's A images
  float* const hw_wave = hring + wave * FE_HR * FE_HROW;
  float fw[3][FE_GH][3];   // normalised features of three consecutive rows (rotating)
  float wdn_prev[FE_GH];
#pragma unroll
  for (int gi = 0; gi < FE_GH; ++gi) wdn_prev[gi] = 0.f;

  // F.normalize * multiM of one pixel's 4 x 3 features (REF:146-157): one hardware reciprocal per (pixel,
  // graph) instead of three IEEE divisions (the IEEE sequence serialises on VCC); <= 1.5 ulp
  auto norm4 = [&](const fe_f32x16& acc, int ep, float (&out)[FE_GH][3]) __attribute__((always_inline)) {
#pragma unroll
    for (int gi = 0; gi < FE_GH; ++gi) {
      const float f0 = acc[3 * gi], f1 = acc[3 * gi + 1], f2 = acc[3 * gi + 2];
      float ss = __builtin_fmaf(f0, f0, 0.f);
      ss = __builtin_fmaf(f1, f1, ss);
      ss = __builtin_fmaf(f2, f2, ss);
      const float den = fmaxf(__builtin_amdgcn_sqrtf(ss), ldexpf(1e-12f, ep + sg[gi]));   // the scaled 1e-12 floor
      const float inv = __builtin_amdgcn_rcpf(den);
      out[gi][0] = (f0 * inv) * M[gi][0];
      out[gi][1] = (f1 * inv) * M[gi][1];
      out[gi][2] = (f2 * inv) * M[gi][2];
    }
  };
  // softmax of four (log2(e)-scaled) similarities with v_exp_f32 (2^x, x <= 0) and one reciprocal
  auto softmax4 = [&](float s0, float s1, float s2, float s3, float& w0, float& w1, float& w2, float& w3)
      __attribute__((always_inline)) {
    const float m = fmaxf(fmaxf(s0, s1), fmaxf(s2, s3));
    const float e0 = __builtin_amdgcn_exp2f(s0 - m), e1 = __builtin_amdgcn_exp2f(s1 - m);
    const float e2 = __builtin_amdgcn_exp2f(s2 - m), e3 = __builtin_amdgcn_exp2f(s3 - m);
    const float sum = ((e0 + e1) + e2) + e3;
    const float rs = __builtin_amdgcn_rcpf(sum);
    w0 = e0 * rs;
    w1 = e1 * rs;
    w2 = e2 * rs;
    w3 = e3 * rs;
  };
  // edges of row ey from the main rows P (ey - 1), Q (ey), N (ey + 1) and the halo ring rows hP, hQ, hN
  auto edges = [&](int ey, auto p_tag, auto q_tag, auto n_tag, const float* hP, const float* hQ, const float* hN)
      __attribute__((always_inline)) {
    constexpr int P = decltype(p_tag)::value, Q = decltype(q_tag)::value, N = decltype(n_tag)::value;
    const bool own = ey < r1 && !(FE_DIAG & 1);
    const uint32_t row_off = (uint32_t)(ey * W + col);
    const uint32_t vo = lane_out && own ? (row_off + 16u * kh * HW) * 4u : FE_OOB;
    const uint32_t voc = lane_out && own ? (row_off + 8u * kh * HW) * 4u : FE_OOB;
    const uint32_t vcv = lane_out && ey > r0 && !(FE_DIAG & 1) ? (row_off - W + 8u * kh * HW) * 4u : FE_OOB;   // row ey - 1
    const int hw4 = __builtin_amdgcn_readfirstlane(HW * 4);
    // the lane's neighbour across the strip edge, row ey: lane 0 the left pixel L, lane 31 the right R1
    const float* hq = hQ + kh * 36;
    float hb[FE_GH][3];
    {
      const float* src = hq + (n == 31 ? 12 : 0);
#pragma unroll
      for (int gi = 0; gi < FE_GH; ++gi)
#pragma unroll
        for (int f = 0; f < 3; ++f) hb[gi][f] = src[3 * gi + f];
    }
    // GTV: the softmax of R1 = x0 + 32 (lane 31's right neighbour, whose w_left lane 31's pair weight needs), one
    // graph per lane of the DPP quad 28..31 (lane 28 + j: graph 3 - j) instead of all four graphs in every lane.
    // Inputs: R1's rows ey - 1, ey, ey + 1 and R2 = x0 + 33 (R1 itself at the image's right edge) from the halo
    // ring; R1 . (x0 + 31) from lane 31 (its hb and its own features) by a quad broadcast
    float w1r[FE_GH];
    if constexpr (slab == 0) {
      const int gl = 3 - (n & 3);
      float t1 = 0.f;
#pragma unroll
      for (int gi = 0; gi < FE_GH; ++gi) {
        float d = 0.f;
#pragma unroll
        for (int f = 0; f < 3; ++f) d = __builtin_fmaf(hb[gi][f], fw[Q][gi][f], d);
        const float b31 = fe_quad(d, 3);
        t1 = gl == gi ? b31 : t1;
      }
      const float* r1q = hq + 12 + 3 * gl;
      const float* r1p = hP + kh * 36 + 12 + 3 * gl;
      const float* r1n = hN + kh * 36 + 12 + 3 * gl;
      const float* r2 = hq + (x0 + 32 < W - 1 ? 24 : 12) + 3 * gl;
      float t0 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const float v = r1q[f];
        t0 = __builtin_fmaf(v, r1p[f], t0);
        t2 = __builtin_fmaf(v, r2[f], t2);
        t3 = __builtin_fmaf(v, r1n[f], t3);
      }
      float u0, u1, u2, u3;
      softmax4(t0, t1, t2, t3, u0, u1, u2, u3);
#pragma unroll
      for (int gi = 0; gi < FE_GH; ++gi) w1r[gi] = fe_quad(u1, 3 - gi);   // lane 31: graph gi from lane 31 - gi
    }
#pragma unroll
    for (int gi = 0; gi < FE_GH; ++gi) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        const float v = fw[Q][gi][f];
        const float pl = fe_prev(v), pr = fe_next(v);
        // at the image's edges the neighbour is the pixel itself (REF's replicate padding): the halo columns and
        // the lanes past W are clamped into the image, so their features already equal v bitwise
        const float lv = n == 0 ? hb[gi][f] : pl;
        const float rv = n == 31 ? hb[gi][f] : pr;
        s0 = __builtin_fmaf(v, fw[P][gi][f], s0);
        s1 = __builtin_fmaf(v, lv, s1);
        s2 = __builtin_fmaf(v, rv, s2);
        s3 = __builtin_fmaf(v, fw[N][gi][f], s3);
      }
      float w0, w1, w2, w3;
      softmax4(s0, s1, s2, s3, w0, w1, w2, w3);
      const bool gok = gbase + gi < G;
      const uint32_t so = (uint32_t)((8 * t4 + gi) * 4) * hw4;
      const uint32_t vg = gok ? vo : FE_OOB;
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w0), wr, vg, so, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w1), wr, vg, so + hw4, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w2), wr, vg, so + 2 * hw4, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(w3), wr, vg, so + 3 * hw4, 0);
      if (slab == 0) {   // wave-uniform: pair weights (REF:452-516's C^T C as pair weights)
        // w_left(p + right): lane n + 1's w1; for lane 31 the softmax of R1 = x0 + 32 from the halo rows (R1's
        // up / down rows, R2 = x0 + 33 to its right, this lane's column to its left)
        const float w1n = fe_next(w1);   // (outside the select: a DPP read in a branch sees inactive lanes as 0)
        const float wln = n == 31 ? w1r[gi] : w1n;
        const float ch = col + 1 < W ? __builtin_fmaf(w2, w2, wln * wln) : 0.f;
        // row ey - 1: w_down(p)^2 + w_up(p + down)^2
        const float cv = __builtin_fmaf(wdn_prev[gi], wdn_prev[gi], w0 * w0);
        wdn_prev[gi] = w3;
        const uint32_t soc = (uint32_t)((8 * t4 + gi) * 2) * hw4;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(ch), crs, gok ? voc : FE_OOB, soc, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cv), crs, gok ? vcv : FE_OOB, soc + hw4, 0);
      }
    }
  };

  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // A images, ring slot 0 (row r0 - 1), halo batch 0
  asm volatile("" ::: "memory");
  // the halo batch of conv rows k .. k + FE_HB - 1 into the halo feature ring (the main image's product order)
  auto halo = [&](int k) __attribute__((always_inline)) {
    fe_f32x16 ax = fe_f32x16{};
    const float* hs = himg + 4 * lane;
#pragma unroll
    for (int s = 0; s < FE_KS; ++s) {
      const fe_f16x8 ah = *reinterpret_cast<const fe_f16x8*>(at + (2 * s) * 256);
      const fe_f16x8 al = *reinterpret_cast<const fe_f16x8*>(at + (2 * s + 1) * 256);
      const fe_f16x8 ch = *reinterpret_cast<const fe_f16x8*>(hs + (2 * s) * 256);
      const fe_f16x8 cl = *reinterpret_cast<const fe_f16x8*>(hs + (2 * s + 1) * 256);
      ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, ch, ax, 0, 0, 0);
      ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, cl, ax, 0, 0, 0);
      ax = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, ch, ax, 0, 0, 0);
    }
    float hf[FE_GH][3];
    norm4(ax, reinterpret_cast<const int*>(himg + FE_IMG)[n], hf);
    if (n < 3 * FE_HB) {   // lane n: conv row k + n / 3, pixel L / R1 / R2
      float* dst = hw_wave + ((k + n / 3) % FE_HR) * FE_HROW + kh * 36 + 12 * (n % 3);
#pragma unroll
      for (int gi = 0; gi < FE_GH; ++gi)
#pragma unroll
        for (int f = 0; f < 3; ++f) dst[3 * gi + f] = hf[gi][f];
    }
  };
  // iteration k: phase PH = k mod 3: the row of iteration k goes to fw[PH]; the edge row's rows are slot PH
  // (= k - 3), (PH + 1) % 3 (k - 2), (PH + 2) % 3 (k - 1).  The halo features of conv row j sit in halo ring row
  // j % FE_HR: iteration FE_HB m writes rows FE_HB m .. + FE_HB - 1 while rows FE_HB m - 3 .. - 1 are still read
  // (FE_HR = FE_HB + 3 keeps them apart).  EDGE / CONV are compile-time (k >= 3 / k <= NI - 2).
  auto iteration = [&](int k, auto ph_tag, auto edge_tag, auto conv_tag) __attribute__((always_inline)) {
    constexpr int PH = decltype(ph_tag)::value;
    constexpr bool EDGE = decltype(edge_tag)::value, CONV = decltype(conv_tag)::value;
    using IP = std::integral_constant<int, PH>;
    using IQ = std::integral_constant<int, (PH + 1) % 3>;
    using IN = std::integral_constant<int, (PH + 2) % 3>;
    fe_f32x16 am = fe_f32x16{};
    int epm = 0;
    auto conv = [&]() __attribute__((always_inline)) {
      if (CONV && !(FE_DIAG & 8)) {
        const float* slot = ring + (k & 1) * FE_SLOT + 4 * lane;
#pragma unroll
        for (int s = 0; s < FE_KS; ++s) {
          const fe_f16x8 ah = *reinterpret_cast<const fe_f16x8*>(at + (2 * s) * 256);
          const fe_f16x8 al = *reinterpret_cast<const fe_f16x8*>(at + (2 * s + 1) * 256);
          const fe_f16x8 bh = *reinterpret_cast<const fe_f16x8*>(slot + (2 * s) * 256);
          const fe_f16x8 bl = *reinterpret_cast<const fe_f16x8*>(slot + (2 * s + 1) * 256);
          am = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, am, 0, 0, 0);
          am = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, am, 0, 0, 0);
          am = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, am, 0, 0, 0);
        }
        epm = reinterpret_cast<const int*>(ring + (k & 1) * FE_SLOT + FE_IMG)[n];
      }
    };
    auto edge = [&]() __attribute__((always_inline)) {
      if (EDGE && !(FE_DIAG & 2)) {   // rows k - 3, k - 2, k - 1
        const int j = k % FE_HR;
        const int jp = j >= 3 ? j - 3 : j + FE_HR - 3, jq = j >= 2 ? j - 2 : j + FE_HR - 2, jn = j >= 1 ? j - 1 : FE_HR - 1;
        edges(r0 - 3 + k, IP{}, IQ{}, IN{}, hw_wave + jp * FE_HROW, hw_wave + jq * FE_HROW, hw_wave + jn * FE_HROW);
      }
    };
    // GTV waves conv first, GLR waves edges first: where a SIMD holds one of each, one's dependent MFMA chain
    // overlaps the other's edge arithmetic (both in lockstep after the barrier)
    if constexpr (!EDGES_FIRST) {
      conv();
      __builtin_amdgcn_sched_barrier(0);
      edge();
    } else {
      edge();
      __builtin_amdgcn_sched_barrier(0);
      conv();
    }
    if (CONV) {
      if (k % FE_HB == 0 && !(FE_DIAG & 8)) halo(k);   // uniform
      norm4(am, epm, fw[PH]);                           // row k replaces row k - 3
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using T = std::true_type;
  using F = std::false_type;
  // NI >= 4: iterations 0..2 conv only, 3..NI-2 both, NI-1 edges only
  iteration(0, I0{}, F{}, T{});
  iteration(1, I1{}, F{}, T{});
  iteration(2, I2{}, F{}, T{});
  int k = 3;
  for (; k + 2 <= NI - 2; k += 3) {
    iteration(k, I0{}, T{}, T{});
    iteration(k + 1, I1{}, T{}, T{});
    iteration(k + 2, I2{}, T{}, T{});
  }
  const int rem = NI - 1 - k;   // 0..2 conv rows left (k % 3 == 0), then the edge-only iteration NI - 1
  if (rem == 0) {
    iteration(k, I0{}, T{}, F{});
  } else if (rem == 1) {
    iteration(k, I0{}, T{}, T{});
    iteration(k + 1, I1{}, T{}, F{});
  } else {
    iteration(k, I0{}, T{}, T{});
    iteration(k + 1, I1{}, T{}, T{});
    iteration(k + 2, I2{}, T{}, F{});
  }
  for (int i = NI; i < NI3; ++i) __builtin_amdgcn_s_barrier();   // the loader's NI3 iteration barriers
  if (slab == 0 && r1 == H) {   // the image's last row: no lower neighbour, c_v = 0
    int hw4 = __builtin_amdgcn_readfirstlane(HW * 4);
    const uint32_t vz = lane_out ? ((uint32_t)((H - 1) * W + col) + 8u * kh * HW) * 4u : FE_OOB;
#pragma unroll
    for (int gi = 0; gi < FE_GH; ++gi)
      __builtin_amdgcn_raw_buffer_store_b32(0u, crs, gbase + gi < G ? vz : FE_OOB, (uint32_t)((8 * t4 + gi) * 2 + 1) * hw4,
                                            0);
  }
  };
  if (slab == 0)
    run(std::integral_constant<int, 0>{});
  else
    run(std::integral_constant<int, 1>{});
}

}  // namespace
}  // namespace grr

using namespace grr;

extern "C" {

int64_t grr_feature_edges_workspace_bytes(int G) {
  return G <= 0 ? 0 : (int64_t)FE_NT * FE_KS * 2 * 1024 + 256 * (((int64_t)2 * G * 4 + 255) / 256);
}

int grr_feature_edges_supported(int C, int G, int F, int H, int W) {
  return F == 3 && G >= 1 && G <= FE_TPS * 8 && C == G * F && C <= 16 * FE_KS && H >= 1 && W >= 1 &&
                 (int64_t)G * 4 * H * W * 4 < (1ll << 31)
             ? 1
             : 0;
}

grr_status grr_feature_edges(const float* x, int x_blocked, const float* wf, const float* multiM_gtv,
                             const float* multiM_glr, float* wG, float* cG, float* wL, void* workspace, int B, int C,
                             int G, int F, int H, int W, void* stream) {
  clear_error();
  GRR_REQUIRE(x && wf && multiM_gtv && multiM_glr && wG && cG && wL && workspace && B > 0, GRR_ERR_INVALID_ARG,
              "grr_feature_edges: bad args");
  GRR_REQUIRE(grr_feature_edges_supported(C, G, F, H, W), GRR_ERR_UNSUPPORTED,
              "grr_feature_edges: needs F = 3, G <= %d, C = G F <= %d (got C %d, G %d, F %d)", FE_TPS * 8, 16 * FE_KS, C,
              G, F);
  GRR_REQUIRE(((uintptr_t)workspace & 255) == 0 && (!x_blocked || ((uintptr_t)x & 15) == 0), GRR_ERR_INVALID_ARG,
              "grr_feature_edges: workspace 256-B aligned, a blocked x 16-B aligned");
  GRR_REQUIRE((int64_t)((C + 7) / 8) * 8 * H * W * 4 < (1ll << 31), GRR_ERR_UNSUPPORTED,
              "grr_feature_edges: image too large for 32-bit offsets");
  hipStream_t s = (hipStream_t)stream;
  char* pack = static_cast<char*>(workspace);
  int* sexp = reinterpret_cast<int*>(pack + (int64_t)FE_NT * FE_KS * 2 * 1024);
  {
    const int n = FE_NT * FE_KS * 2 * 256 + 2 * G;
    hipLaunchKernelGGL(fe_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, s, wf, pack, sexp, G, C);
    grr_status st = launch_status("grr_feature_edges/pack");
    if (st != GRR_OK) return st;
  }
  FeArgs a{};
  a.x = x;
  a.pack = pack;
  a.sexp = sexp;
  a.multiM[0] = multiM_gtv;
  a.multiM[1] = multiM_glr;
  a.w[0] = wG;
  a.w[1] = wL;
  a.c = cG;
  a.C = C;
  a.G = G;
  a.H = H;
  a.W = W;
  a.nstrips = (W + FE_OWN - 1) / FE_OWN;
  // row segments: >= 4 workgroups per CU where the batch allows, segments of >= 32 rows (each costs 3 extra
  // conv rows and 1 extra edge row)
  int sseg = H;
  const int64_t strips = (int64_t)B * a.nstrips;
  while (sseg > 32 && strips * ((H + sseg - 1) / sseg) < 1024) sseg = (sseg + 1) / 2;
  a.sseg = sseg;
  a.nsegs = (H + sseg - 1) / sseg;
  const uint64_t nblk = (uint64_t)strips * a.nsegs;
  GRR_REQUIRE(nblk < (1ull << 31), GRR_ERR_UNSUPPORTED, "grr_feature_edges: grid too large");
  a.nblk = (uint32_t)nblk;
  if (x_blocked)
    hipLaunchKernelGGL(feat_edge_kernel<true>, dim3(a.nblk), dim3(FE_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL(feat_edge_kernel<false>, dim3(a.nblk), dim3(FE_THREADS), 0, s, a);
  return launch_status("grr_feature_edges");
}

}  // extern "C"
