// K10 — implicit-GEMM convolution of the UNet3D's InflatedConv3d / resnet convs (tuneavideo
// resnet.py:11-19 applies nn.Conv2d per frame on '(b f) c h w'), channels-last bf16, with the bias
// and the resnet's shortcut add (resnet.py:196-205, 'output_tensor = input_tensor + hidden_states')
// fused into the epilogue.
//
//   y[p, co] = bias[co] + sum_{kh, kw, c} x[n, oy*s - pad + kh, ox*s - pad + kw, c] * w[co, kh, kw, c]
//              (+ residual[p, co])
// with p = (n, oy, ox).  As a GEMM: M = N*Ho*Wo pixels, N = Cout, K = KH*KW*Cin, both operands
// K-contiguous in memory (x is NHWC; the channels-last conv weight is [Cout][KH][KW][Cin]).
//
// MI355X design:
//  * 128 x 160 output tile per 256-thread workgroup, 2 x 2 waves of 64 x 80 = 4 x 5 tiles of
//    v_mfma_f32_16x16x32_bf16 (Cout = 320 / 640 / 1280 are whole multiples of 160, no ragged
//    column tiles);
//  * K in steps of 64 channels at one (kh, kw): every A row is one 128-byte segment of an input
//    pixel (or zeros in the padding), every B row 128 bytes of a weight row, staged through LDS
//    with register prefetch (issue the next step's global loads before this step's MFMAs, write
//    them after the barrier);
//  * LDS rows padded to 144 bytes: the 16 rows a 16-lane group reads with ds_read_b128 fall in 16
//    distinct 4-bank groups;
//  * epilogue: accumulators + bias -> bf16 tile in LDS, then each thread writes whole 16-byte
//    channel vectors (adding the residual vector), fully coalesced.
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {
namespace conv {

constexpr int BN = 160, BK = 64;
constexpr int WTM = 4, WTN = 5;                 // 16x16 MFMA tiles per wave (64 x 80)
constexpr int ROW = BK + 8;                     // LDS row (elements): 144 bytes
constexpr int CROW = BN + 8;                    // epilogue tile row (elements)

// BM = 128 (4 waves, 2 workgroups per CU) or 256 (8 waves, one per CU); waves are (BM/64) x 2
template <int BM>
struct Cfg {
  static constexpr int NT = BM * 2;                       // threads
  static constexpr int A_CH = BM * BK / 8 / NT;           // 16-byte chunks per thread per step: 4
  static constexpr int B_CH = (BN * BK / 8 + NT - 1) / NT;
  static constexpr int LDS_AB = (BM + BN) * ROW * 2;
  static constexpr int LDS_C = BM * CROW * 2;
  static constexpr int LDS_BYTES = LDS_AB > LDS_C ? LDS_AB : LDS_C;
};

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(bf16x8 a, bf16x8 b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int KS, int BM>
__global__ __launch_bounds__(BM * 2, BM == 128 ? 2 : 1) void conv_kernel(const vp2p_conv_args a) {
  constexpr int NT = Cfg<BM>::NT, A_CH = Cfg<BM>::A_CH, B_CH = Cfg<BM>::B_CH;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* As = reinterpret_cast<bf16*>(smem);
  bf16* Bs = As + BM * ROW;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;           // wave grid (BM/64) x 2
  const int M = a.batch * a.out_h * a.out_w;
  const int ntn = a.cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const bf16* x = static_cast<const bf16*>(a.x);
  const bf16* wt = static_cast<const bf16*>(a.w);
  const int Kw = KS * KS * a.cin;               // weight row length

  // A rows owned by this thread for staging: row = tid / 8 + 32 i, chunk = tid % 8
  const int ach = tid & 7;
  int a_n[A_CH], a_iy[A_CH], a_ix[A_CH];
  bool a_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int p = m0 + (tid >> 3) + (NT / 8) * i;
    a_ok[i] = p < M;
    const int pp = a_ok[i] ? p : 0;
    const int n = pp / (a.out_h * a.out_w), rem = pp - n * a.out_h * a.out_w;
    const int oy = rem / a.out_w, ox = rem - oy * a.out_w;
    a_n[i] = n;
    a_iy[i] = oy * a.stride - a.pad;
    a_ix[i] = ox * a.stride - a.pad;
  }
  u32x4 areg[A_CH], breg[B_CH];
  const int csteps = a.cin / BK;
  const int nsteps = KS * KS * csteps;

  auto load = [&](int step) {
    const int tap = step / csteps, c0 = (step - tap * csteps) * BK;
    const int kh = tap / KS, kw = tap - kh * KS;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
      const bool ok = a_ok[i] && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      // branch-free: padding taps load a valid address (pixel 0) and are zeroed by a select
      const int64_t pix = ok ? ((int64_t)a_n[i] * a.in_h + iy) * a.in_w + ix : 0;
      const u32x4 v = *reinterpret_cast<const u32x4*>(x + pix * a.cin + c0 + ach * 8);
      areg[i] = ok ? v : u32x4{0, 0, 0, 0};
    }
    const int64_t kofs = (int64_t)tap * a.cin + c0;
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int c = tid + NT * i, row = c >> 3, ch = c & 7;
      if (c < BN * 8) breg[i] = *reinterpret_cast<const u32x4*>(wt + (int64_t)(n0 + row) * Kw + kofs + ch * 8);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<u32x4*>(As + ((tid >> 3) + (NT / 8) * i) * ROW + ach * 8) = areg[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int c = tid + NT * i, row = c >> 3, ch = c & 7;
      if (c < BN * 8) *reinterpret_cast<u32x4*>(Bs + row * ROW + ch * 8) = breg[i];
    }
  };

  f32x4v acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int fr = l & 15, fk = (l >> 4) * 8;     // fragment row / k offset of this lane
  load(0);
  for (int step = 0; step < nsteps; ++step) {
    __syncthreads();
    store();
    __syncthreads();
    if (step + 1 < nsteps) load(step + 1);
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 af[WTM], bfr[WTN];
#pragma unroll
      for (int i = 0; i < WTM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + 16 * i + fr) * ROW + ks + fk);
#pragma unroll
      for (int j = 0; j < WTN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 80 + 16 * j + fr) * ROW + ks + fk);
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  // epilogue: (acc + bias) -> bf16 tile in LDS (lane holds rows 4*(l>>4)+e of column l&15)
  __syncthreads();
  bf16* Cs = reinterpret_cast<bf16*>(smem);
  const bf16* bias = static_cast<const bf16*>(a.bias);
#pragma unroll
  for (int j = 0; j < WTN; ++j) {
    const int col = wn * 80 + 16 * j + fr;
    const float bv = bias ? (float)bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wm * 64 + 16 * i + 4 * (l >> 4) + e) * CROW + col] = (bf16)(acc[i][j][e] + bv);
  }
  __syncthreads();
  // 128 rows x 20 chunks of 8 channels; residual added per 16-byte vector
  const bf16* res = static_cast<const bf16*>(a.residual);
  bf16* y = static_cast<bf16*>(a.y);
  for (int c = tid; c < BM * (BN / 8); c += NT) {
    const int row = c / (BN / 8), ch = c - row * (BN / 8);
    const int p = m0 + row;
    if (p >= M) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + ch * 8);
    const int64_t o = (int64_t)p * a.cout + n0 + ch * 8;
    if (res) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)rv[j]);
    }
    *reinterpret_cast<bf16x8*>(y + o) = v;
  }
}

// ------------------------------------------------------------------------------------------------
// conv_kernel_g: the same 128 x 160 tile, staged by LDS-DMA (global_load_lds_dwordx4) into two LDS
// stages, one barrier per K-step (the DMA of step s+1 runs under the MFMAs of step s; no VGPRs
// hold the tile in flight).  A DMA instruction writes 64 x 16 B lane-linearly = 8 rows of 128 B;
// the XOR swizzle lives in the per-lane SOURCE address: LDS slot j of row r holds global chunk
// j ^ ((r >> 1) & 7), which makes the 16 rows of a 16-lane ds_read_b128 hit 16 distinct 4-bank
// groups.  Padding taps and rows past M read a 16-byte zero vector in global memory.
// ------------------------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) unsigned int kZero16[4] = {0, 0, 0, 0};

// GBM = 128 (4 waves, 2 workgroups per CU) or 256 (8 waves, one per CU); waves (GBM/64) x 2
template <int GBM, int NS = 2>
struct GCfg {
  static constexpr int NW = GBM / 32;
  static constexpr int STAGE = (GBM + BN) * BK * 2;              // bytes per stage (A then B)
  static constexpr int LDS = NS * STAGE > GBM * CROW * 2 ? NS * STAGE : GBM * CROW * 2;
  static constexpr int ADMA = GBM / 8 / NW;                      // A DMA instructions per wave per step: 4
  static constexpr int BDMA = (BN / 8 + NW - 1) / NW;            // B: 5 (4 waves) or 3 (8 waves, last ragged)
};

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

// NS = 2: one step in flight, __syncthreads per step.  NS = 3: two steps in flight; each wave
// waits (counted vmcnt) only for its own DMA of the step it is about to read, then a raw
// s_barrier -- the newer step's DMA stays in flight across it.
// EPI = 1 (GEGLU, 1x1 only): the weight rows come interleaved per 160-column tile as [80 "a" rows,
// the 80 matching "gate" rows], and the epilogue writes y[p, nt*80 + j] = a * gelu(g) (exact erf,
// each step rounded to bf16 as torch's eager GEGLU does) into a (M, cout/2) output.
template <int KS, int GBM, int NS, int EPI = 0>
__global__ __launch_bounds__(GBM * 2, GBM == 128 && NS == 2 ? 2 : 1) void conv_kernel_g(const vp2p_conv_args a) {
  using G = GCfg<GBM, NS>;
  constexpr int NW = G::NW, G_STAGE = G::STAGE, G_ADMA = G::ADMA, G_BDMA = G::BDMA;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int M = a.batch * a.out_h * a.out_w;
  const int ntn = a.cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = bid / ntn, nt = bid - mt * ntn;
  const int m0 = mt * GBM, n0 = nt * BN;
  const bf16* x = static_cast<const bf16*>(a.x);
  const bf16* wt = static_cast<const bf16*>(a.w);
  const int Kw = KS * KS * a.cin;
  const bf16* zero = reinterpret_cast<const bf16*>(kZero16);

  // this lane's rows: A instruction i of wave w covers rows 8*(w + 4i) .. +7, lane row l / 8
  const int lr = l >> 3, lj = l & 7;
  int a_n[G_ADMA], a_iy[G_ADMA], a_ix[G_ADMA], a_c[G_ADMA];
  bool a_ok[G_ADMA];
#pragma unroll
  for (int i = 0; i < G_ADMA; ++i) {
    const int r = 8 * (w + NW * i) + lr;
    const int p = m0 + r;
    a_ok[i] = p < M;
    const int pp = a_ok[i] ? p : 0;
    const int n = pp / (a.out_h * a.out_w), rem = pp - n * a.out_h * a.out_w;
    const int oy = rem / a.out_w, ox = rem - oy * a.out_w;
    a_n[i] = n;
    a_iy[i] = oy * a.stride - a.pad;
    a_ix[i] = ox * a.stride - a.pad;
    a_c[i] = swz(r, lj) * 8;                                  // source channel offset of this lane
  }
  int b_c[G_BDMA];
#pragma unroll
  for (int i = 0; i < G_BDMA; ++i) b_c[i] = swz(8 * (w + NW * i) + lr, lj) * 8;

  const int csteps = a.cin / BK;
  const int nsteps = KS * KS * csteps;
  auto dma = [&](int step, int stage) {
    const int tap = step / csteps, c0 = (step - tap * csteps) * BK;
    const int kh = tap / KS, kw = tap - kh * KS;
    char* As = smem + stage * G_STAGE;
    char* Bs = As + GBM * BK * 2;
#pragma unroll
    for (int i = 0; i < G_ADMA; ++i) {
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
      const bool ok = a_ok[i] && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      const bf16* src = ok ? x + (((int64_t)a_n[i] * a.in_h + iy) * a.in_w + ix) * a.cin + c0 + a_c[i] : zero;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(As + 8 * (w + NW * i) * BK * 2),
                                       16, 0, 0);
    }
    const int64_t kofs = (int64_t)tap * a.cin + c0;
#pragma unroll
    for (int i = 0; i < G_BDMA; ++i) {
      if (BN / 8 % NW && w + NW * i >= BN / 8) break;           // 8-wave tile: 20 row groups over 8 waves
      const int row = 8 * (w + NW * i) + lr;
      const bf16* src = wt + (int64_t)(n0 + row) * Kw + kofs + b_c[i];
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(Bs + 8 * (w + NW * i) * BK * 2),
                                       16, 0, 0);
    }
  };

  f32x4v acc[WTM][WTN];
#pragma unroll
  for (int i = 0; i < WTM; ++i)
#pragma unroll
    for (int j = 0; j < WTN; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int fr = l & 15, fq = l >> 4;           // fragment row / 16-byte chunk within the 32-wide k-step
  // DMA instructions this wave issues per step (the last B row groups are ragged over 8 waves)
  const int ndma = G_ADMA + ((BN / 8 % NW) ? (w < BN / 8 % NW ? G_BDMA : G_BDMA - 1) : G_BDMA);
  dma(0, 0);
  if (NS == 3 && nsteps > 1) dma(1, 1);
  for (int step = 0; step < nsteps; ++step) {
    if constexpr (NS == 2) {
      __syncthreads();                            // vmcnt(0): step's DMA landed; step-1's reads done
      if (step + 1 < nsteps) dma(step + 1, (step + 1) & 1);
    } else {
      // own DMA of `step` landed (the newer step's may still fly), then everyone's
      if (step + 1 < nsteps) {
        if (ndma == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else if (ndma == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (step + 2 < nsteps) dma(step + 2, (step + 2) % 3);
    }
    const char* As = smem + (NS == 2 ? (step & 1) : (step % 3)) * G_STAGE;
    const char* Bs = As + GBM * BK * 2;
#pragma unroll
    for (int ks = 0; ks < BK / 8; ks += 4) {      // chunk index of the k-step (0 or 4)
      bf16x8 af[WTM], bfr[WTN];
#pragma unroll
      for (int i = 0; i < WTM; ++i) {
        const int r = wm * 64 + 16 * i + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * BK * 2 + swz(r, ks + fq) * 16);
      }
#pragma unroll
      for (int j = 0; j < WTN; ++j) {
        const int r = wn * 80 + 16 * j + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + r * BK * 2 + swz(r, ks + fq) * 16);
      }
#pragma unroll
      for (int i = 0; i < WTM; ++i)
#pragma unroll
        for (int j = 0; j < WTN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  __syncthreads();
  bf16* Cs = reinterpret_cast<bf16*>(smem);
  const bf16* bias = static_cast<const bf16*>(a.bias);
#pragma unroll
  for (int j = 0; j < WTN; ++j) {
    const int col = wn * 80 + 16 * j + fr;
    const float bv = bias ? (float)bias[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < WTM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wm * 64 + 16 * i + 4 * fq + e) * CROW + col] = (bf16)(acc[i][j][e] + bv);
  }
  __syncthreads();
  const bf16* res = static_cast<const bf16*>(a.residual);
  bf16* y = static_cast<bf16*>(a.y);
  if constexpr (EPI == 1) {
#pragma clang fp contract(off)
    constexpr float kAlpha = 0.70710678118654752440f;
    const int half = a.cout / 2;
    for (int c = tid; c < GBM * (BN / 16); c += GBM * 2) {
      const int row = c / (BN / 16), ch = c - row * (BN / 16);
      const int p = m0 + row;
      if (p >= M) continue;
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + ch * 8);
      const bf16x8 gv = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + BN / 2 + ch * 8);
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float g = (float)gv[j];
        const float ge = (float)(bf16)(g * 0.5f * (1.f + erff(g * kAlpha)));
        v[j] = (bf16)((float)av[j] * ge);
      }
      *reinterpret_cast<bf16x8*>(y + (int64_t)p * half + nt * (BN / 2) + ch * 8) = v;
    }
    return;
  }
  for (int c = tid; c < GBM * (BN / 8); c += GBM * 2) {
    const int row = c / (BN / 8), ch = c - row * (BN / 8);
    const int p = m0 + row;
    if (p >= M) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + row * CROW + ch * 8);
    const int64_t o = (int64_t)p * a.cout + n0 + ch * 8;
    if (res) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)rv[j]);
    }
    *reinterpret_cast<bf16x8*>(y + o) = v;
  }
}

}  // namespace conv
}  // namespace vp2p

using namespace vp2p;

extern "C" int vp2p_conv2d_supported(const vp2p_conv_args* a) {
  if (!a) return 0;
  if (a->dtype != VP2P_BF16) return 0;
  if (a->kernel != 1 && a->kernel != 3) return 0;
  if (a->pad != (a->kernel - 1) / 2 || (a->stride != 1 && a->stride != 2)) return 0;
  if (a->cin <= 0 || a->cin % conv::BK || a->cout <= 0 || a->cout % conv::BN) return 0;
  if (a->batch <= 0 || a->in_h <= 0 || a->in_w <= 0) return 0;
  if (a->out_h != (a->in_h + 2 * a->pad - a->kernel) / a->stride + 1) return 0;
  if (a->out_w != (a->in_w + 2 * a->pad - a->kernel) / a->stride + 1) return 0;
  if (a->epilogue != VP2P_CONV_EPI_NONE &&
      (a->epilogue != VP2P_CONV_EPI_GEGLU || a->kernel != 1 || a->stride != 1 || a->residual)) return 0;
  return 1;
}

extern "C" int vp2p_conv2d_fwd(const vp2p_conv_args* a, void* stream) {
  if (!a || !a->x || !a->w || !a->y) return VP2P_E_ARG;
  if (a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (!vp2p_conv2d_supported(a)) return VP2P_E_SHAPE;
  for (const void* p : {a->x, a->w, static_cast<const void*>(a->y), a->residual})
    if (reinterpret_cast<uintptr_t>(p) & 15) return VP2P_E_ARG;
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  if (M * a->cout > ((int64_t)1 << 40)) return VP2P_E_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // default (1): the LDS-DMA kernel conv_kernel_g with 128-row tiles; 2: its 256-row (8-wave) form;
  // 3: 256-row tiles with three LDS stages (two steps in flight);
  // 128 / 256: the register-staged kernels (A/B experiments)
  const char* e = getenv("VP2P_CONV_BM");
  const int bm = e ? atoi(e) : 1;
  if (a->epilogue != VP2P_CONV_EPI_NONE && !(bm >= 1 && bm <= 3)) return VP2P_E_SHAPE;
  if (bm >= 1 && bm <= 3) {
    auto launch_g = [&](auto gbm_tag, auto ns_tag) {
      constexpr int GBM = decltype(gbm_tag)::value, NS = decltype(ns_tag)::value;
      constexpr int lds = conv::GCfg<GBM, NS>::LDS;
      const int64_t nwg = (M + GBM - 1) / GBM * (a->cout / conv::BN);
      if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
      static const bool attr =
          hipFuncSetAttribute(reinterpret_cast<const void*>(&conv::conv_kernel_g<3, GBM, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(&conv::conv_kernel_g<1, GBM, NS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
          hipFuncSetAttribute(reinterpret_cast<const void*>(&conv::conv_kernel_g<1, GBM, NS, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
      if (!attr) return VP2P_E_LAUNCH;
      if (a->epilogue == VP2P_CONV_EPI_GEGLU)
        hipLaunchKernelGGL((conv::conv_kernel_g<1, GBM, NS, 1>), dim3((unsigned)nwg), dim3(2 * GBM), lds, s, *a);
      else if (a->kernel == 3)
        hipLaunchKernelGGL((conv::conv_kernel_g<3, GBM, NS>), dim3((unsigned)nwg), dim3(2 * GBM), lds, s, *a);
      else
        hipLaunchKernelGGL((conv::conv_kernel_g<1, GBM, NS>), dim3((unsigned)nwg), dim3(2 * GBM), lds, s, *a);
      return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
    };
    if (bm == 3) return launch_g(std::integral_constant<int, 256>{}, std::integral_constant<int, 3>{});
    if (bm == 2) return launch_g(std::integral_constant<int, 256>{}, std::integral_constant<int, 2>{});
    return launch_g(std::integral_constant<int, 128>{}, std::integral_constant<int, 2>{});
  }
  auto launch = [&](auto bm_tag) {
    constexpr int BM = decltype(bm_tag)::value;
    constexpr int lds = conv::Cfg<BM>::LDS_BYTES;
    const int64_t nwg = (M + BM - 1) / BM * (a->cout / conv::BN);
    if (nwg <= 0 || nwg > 0x7fffffff) return VP2P_E_SHAPE;
    static const bool attr =
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv::conv_kernel<3, BM>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess &&
        hipFuncSetAttribute(reinterpret_cast<const void*>(&conv::conv_kernel<1, BM>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    if (!attr) return VP2P_E_LAUNCH;
    if (a->kernel == 3)
      hipLaunchKernelGGL((conv::conv_kernel<3, BM>), dim3((unsigned)nwg), dim3(2 * BM), lds, s, *a);
    else
      hipLaunchKernelGGL((conv::conv_kernel<1, BM>), dim3((unsigned)nwg), dim3(2 * BM), lds, s, *a);
    return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
  };
  return bm == 256 ? launch(std::integral_constant<int, 256>{}) : launch(std::integral_constant<int, 128>{});
}
