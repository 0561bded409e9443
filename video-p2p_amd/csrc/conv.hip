// K10 — implicit-GEMM convolution of the UNet3D's InflatedConv3d / resnet convs (tuneavideo
// resnet.py:11-19 applies nn.Conv2d per frame on '(b f) c h w'), channels-last bf16, with the bias
// and the resnet's shortcut add (resnet.py:196-205, 'output_tensor = input_tensor + hidden_states')
// fused into the epilogue; the same GEMM core with K = Cin runs the FeedForward projection with the
// GEGLU gate fused (attention.py:190, 259).
//
//   y[p, co] = bias[co] + sum_{kh, kw, c} x[n, oy*s - pad + kh, ox*s - pad + kw, c] * w[co, kh, kw, c]
//              (+ residual[p, co])
// with p = (n, oy, ox).  As a GEMM: M = N*Ho*Wo pixels, N = Cout, K = KH*KW*Cin, both operands
// K-contiguous in memory (x is NHWC; the channels-last conv weight is [Cout][KH][KW][Cin]).
//
// MI355X design:
//  * 128 x 160 output tile per 256-thread workgroup, 2 x 2 waves of 64 x 80 = 4 x 5 tiles of
//    v_mfma_f32_16x16x32_bf16 (Cout = 320 / 640 / 1280 are whole multiples of 160, no ragged
//    column tiles); two workgroups per CU;
//  * K in steps of 64 channels at one (kh, kw): A rows are 128-byte segments of input pixels (a
//    16-byte zero vector for padding taps), B rows 128 bytes of weight rows, moved by LDS-DMA
//    (global_load_lds_dwordx4) into two LDS stages; one barrier per step, the DMA of step s+1 runs
//    under the MFMAs of step s and no VGPR holds the tile in flight;
//  * K order channel-major (round 5): the nine taps of one 64-channel chunk in consecutive steps,
//    so a chunk's shifted re-reads (one 128-B line per pixel) hit L2.  Tap-major (all channels of
//    a tap, then the next) spans 640-2560 B per pixel between re-reads, over the 4 MB L2 of an XCD
//    at 32 concurrent tiles: FETCH + WRITE 934 -> 281 MB per 64^2 320 -> 320 launch (3.7x -> 1.1x the
//    algorithmic bytes), 0.238 -> 0.222 ms, whole edit +1.4 % (profiles/r05_k10_cmajor_*);
//  * LDS rows are unpadded 128 B; the XOR swizzle (slot j of row r holds chunk j ^ ((r >> 1) & 7))
//    is applied on the per-lane DMA source address, so the 16 rows a 16-lane ds_read_b128 touches
//    fall in 16 distinct 4-bank groups;
//  * epilogue: accumulators + bias -> bf16 tile in LDS, then whole 16-byte channel vectors out
//    (residual added per vector), fully coalesced;
//  * split-K for the small-M shapes (the 8x8 latents: 128 tiles for 256 CUs): each workgroup sums a
//    slice of the K-steps into an fp32 workspace and a second pass adds the slices, the bias and the
//    residual with the same roundings as the one-pass epilogue.
//  * DMA addressing: each lane's byte offset of its pixel at tap (0, 0) and a 9-bit mask of the taps
//    that fall outside the image are computed once; a K-step's address is one add of a wave-uniform
//    tap/channel offset, and an out-of-image tap sets bit 31 so the buffer load (raw buffer
//    resource, num_records < 2^31) delivers the zero padding.  Rebuilding 64-bit pointers per step
//    (~130 VALU per step per wave) was the limiter of the first form: 830-930 -> 1020-1150 TF/s.
// Measured (profiles/r02_conv_bench_fastaddr.jsonl): 1020-1150 TF/s on the large 3x3 convs; the
// Upsample3D convs on the same buffer form (AM 2): 835-964 -> 1008-1192 TF/s, bit-equal
// (profiles/r02_conv_up_bench.jsonl).  Tried and
// dropped: register staging (~800), 256-row tiles with three LDS stages and a counted-vmcnt barrier
// span (-5 %), one wave per 32 rows x 160 columns on 32x32x16 MFMAs (-9 %: every wave reads all of B).
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "common.hpp"
#include "vp2p.h"

namespace vp2p {
namespace conv {

// the main loop's fragment reads software-pipelined against the MFMAs (conv_tile; 0: the compiler's
// order, kept for A/B)
#ifndef VP2P_K10_PIPE
#define VP2P_K10_PIPE 1
#endif
constexpr bool kPipe = VP2P_K10_PIPE;
// K order of the KS x KS convs: 0 tap-major (all channels of one tap, then the next tap), 1
// channel-major (the taps of one 64-channel chunk in consecutive steps)
#ifndef VP2P_K10_CMAJOR
#define VP2P_K10_CMAJOR 1
#endif
// tile raster of the one-pass grids (split-K keeps row-major): 0 row tile major (all column tiles
// of a row tile in consecutive workgroups), G > 0 grouped (G row tiles per group, row tile
// fastest), so an XCD's contiguous share of the grid reads fewer weight columns.  Same tiles, so
// bit-equal; 8 measured 0-5 % faster per launch (res-32 GEGLU 0.242 -> 0.231 ms, 64^2 640 -> 320
// 3x3 0.401 -> 0.391 ms; profiles/r05_k10_groupm_ab.jsonl), the whole edit +0.3 %
#ifndef VP2P_K10_GROUPM
#define VP2P_K10_GROUPM 8
#endif
#ifndef VP2P_K10_SPLIT_RASTER
#define VP2P_K10_SPLIT_RASTER 1
#endif

constexpr int BN = 160, BK = 64;
constexpr int CROW = BN + 8;                    // epilogue tile row (elements)

typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v mfma16(bf16x8 a, bf16x8 b, f32x4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
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

constexpr int GBM = 128, NW = 4;                               // the split-K / small-M tile
// Tile configurations of conv_tile (CF):
//  0: 128 x 160, 4 waves (2 x 2 of 64 x 80), two LDS stages, one __syncthreads per K-step, two
//     workgroups per CU -- the default;
//  1: 256 x 160, 8 waves (4 x 2 of 64 x 80), THREE LDS stages (3 x 52 KB), one workgroup per CU;
//     the DMA of steps s+1 and s+2 in flight under step s's MFMAs (counted vmcnt + raw s_barrier,
//     so the barrier does not drain the ring) -- the long-K 1x1 GEMMs;
//  2: 256 x 320 "wide", 8 waves (2 x 4 of 128 x 80: 8 x 5 MFMA tiles, every A fragment used 5x,
//     every B fragment 8x), two stages (2 x 72 KB), one workgroup per CU: twice the MFMAs per LDS
//     byte read and per barrier of 0 / 1 (Cout % 320 == 0; the epilogue runs in two 128-row passes);
//  3: 64 x 160 "short", 4 waves (2 x 2 of 32 x 80), two stages: the small-clip shapes whose 128-row
//     grid would leave CUs idle (1-2 frame edits), one pass where 0 needed a split-K second pass;
//  4: 192 x 320 "mid", 8 waves (2 x 4 of 96 x 80), two stages (2 x 64 KB), one workgroup per CU:
//     the grids whose 192-row tiles come out at whole waves of 256 where 0 / 2 leave a part-filled
//     last wave (the 3-frame clip's 64x64 convs: M 49152, 256 tiles, against 768 of 0 = 3 per CU);
// All: the same per-output K order and MFMA sequence (one 16x16x32 MFMA per 32 channels), so
// bit-equal results.
template <int TBM_, int TBN_, int WTM_, int NST_, int KB_ = 64, int WTN_ = 5> struct GTile {
  static constexpr int TBM = TBM_, TBN = TBN_, WTM = WTM_, WTN = WTN_, NSTAGE = NST_;
  static constexpr int WN = 16 * WTN;                             // output columns per wave
  static constexpr int KB = KB_;                                  // channels per K-step
  static constexpr int RB = KB * 2;                               // LDS row bytes
  static constexpr int CPW = KB / 8;                              // 16-byte chunks per row
  static constexpr int RPI = 64 / CPW;                            // rows per LDS-DMA instruction
  __device__ static __forceinline__ int swz(int r, int c) {
    if constexpr (KB == 64) return c ^ ((r >> 1) & 7);
    else return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3);
  }
  static constexpr int WR = 16 * WTM;                             // output rows per wave
  static constexpr int WCOL = TBN / WN;                           // waves along N
  static constexpr int NWV = (TBM / WR) * WCOL;                   // waves
  static constexpr int NT = 64 * NWV;                             // threads
  static constexpr int STAGE = (TBM + TBN) * RB;                  // bytes per LDS stage (A then B)
  static constexpr int CROWV = TBN + 8;                           // epilogue tile row (elements)
  static constexpr int EROWS = TBM * CROWV * 2 <= NSTAGE * STAGE ? TBM : WR;   // epilogue rows per pass
  static constexpr int LDS = NSTAGE * STAGE > EROWS * CROWV * 2 ? NSTAGE * STAGE : EROWS * CROWV * 2;
  static constexpr int ADMA = TBM / RPI / NWV;                    // A DMA instructions per wave per step
  static constexpr int BBLK = TBN / RPI;                          // RPI-row B blocks per step
  static constexpr int BDMA = (BBLK + NWV - 1) / NWV;             // B DMA slots per wave
};
template <int CF> struct GCfg;
template <> struct GCfg<0> : GTile<128, 160, 4, 2> {};
template <> struct GCfg<1> : GTile<256, 160, 4, 3> {};
template <> struct GCfg<2> : GTile<256, 320, 8, 2> {};
template <> struct GCfg<3> : GTile<64, 160, 2, 2> {};
template <> struct GCfg<4> : GTile<192, 320, 6, 2> {};
// The GEGLU epilogue's form of each tile: the same block, threads, stages and LDS, with every wave
// 160 columns wide (10 16-column tiles = 5 (value, gate) pairs of the same 16 channels: the weights
// come interleaved per 16 as [16 value rows | 16 gate rows]), so a lane holds a channel's value and
// gate for the same four rows itself -- no cross-lane exchange.
template <int CF> struct GCfgG;
template <> struct GCfgG<0> : GTile<128, 160, 2, 2, 64, 10> {};
template <> struct GCfgG<1> : GTile<256, 160, 2, 3, 64, 10> {};
template <> struct GCfgG<2> : GTile<256, 320, 4, 2, 64, 10> {};
template <> struct GCfgG<3> : GTile<64, 160, 1, 2, 64, 10> {};
constexpr int G_STAGE = GCfg<0>::STAGE;
constexpr int G_LDS = GCfg<0>::LDS;


struct Welford {
  float n, mean, m2;
};
// Chan's merge of two (count, mean, M2) summaries (the K7 GroupNorm partial format, norm.hip)
__device__ __forceinline__ Welford wmerge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  return {n, a.mean + d * fb, a.m2 + b.m2 + d * d * a.n * fb};
}

// LDS-DMA destination (a non-template helper: the address-space cast of a TBM-dependent expression
// inside the kernel template makes hipcc's host pass silently drop the kernel's launch stub)
__device__ __forceinline__ __attribute__((address_space(3))) void* to_lds(const char* p) {
  return (__attribute__((address_space(3))) void*)(p);
}

// erf for the GEGLU epilogue, branch-free: Abramowitz & Stegun 7.1.28,
//   erf(|x|) = 1 - (1 + a1|x| + ... + a6|x|^6)^-16   (|error| <= 3e-7; <= 1.8e-6 in fp32 arithmetic),
// 6 FMAs, 4 multiplies and one v_rcp.  ocml's erff branches at |x| = 1 and runs both sides on
// mixed waves (~45 VALU per element): res-64 GEGLU projection 0.483 -> 0.432 ms, res-32 0.315 ->
// 0.284 (profiles/r02_k10_epilogue_ab.jsonl; a transposed-accumulator epilogue with 8-byte LDS
// writes measured no faster and was dropped).
typedef float f32x2v __attribute__((ext_vector_type(2)));

// erf_fast on a pair: the same fp32 operations per element, on packed FMAs / multiplies (v_pk_fma_f32,
// v_pk_mul_f32: two lanes' worth per instruction), so the GEGLU epilogue's polynomial costs half
__device__ __forceinline__ f32x2v erf_fast2(f32x2v x) {
  const f32x2v ax = __builtin_elementwise_abs(x);
  f32x2v p = __builtin_elementwise_fma(ax, (f32x2v)(4.30638e-5f), (f32x2v)(2.765672e-4f));
  p = __builtin_elementwise_fma(p, ax, (f32x2v)(1.520143e-4f));
  p = __builtin_elementwise_fma(p, ax, (f32x2v)(9.2705272e-3f));
  p = __builtin_elementwise_fma(p, ax, (f32x2v)(4.22820123e-2f));
  p = __builtin_elementwise_fma(p, ax, (f32x2v)(7.05230784e-2f));
  p = __builtin_elementwise_fma(p, ax, (f32x2v)(1.f));
  p *= p;
  p *= p;
  p *= p;
  p *= p;
  const f32x2v r = {__builtin_amdgcn_rcpf(p.x), __builtin_amdgcn_rcpf(p.y)};
  return __builtin_elementwise_copysign((f32x2v)(1.f) - r, x);
}

typedef bf16 bf16x2v __attribute__((ext_vector_type(2)));
// both lanes of a pair rounded to bf16 (round to nearest even) and back: one v_cvt_pk_bf16_f32, the
// two halves unpacked by a shift and a mask
__device__ __forceinline__ f32x2v round_bf16x2(f32x2v x) {
  const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2v));
  return f32x2v{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}

__device__ __forceinline__ f32x4v round_bf16x4(f32x4v x) {
  const f32x2v lo = round_bf16x2(f32x2v{x[0], x[1]}), hi = round_bf16x2(f32x2v{x[2], x[3]});
  return f32x4v{lo[0], lo[1], hi[0], hi[1]};
}

// erf_fast2 on four values (two independent packed chains)
__device__ __forceinline__ f32x4v erf_fast4(f32x4v x) {
  const f32x4v ax = __builtin_elementwise_abs(x);
  f32x4v p = __builtin_elementwise_fma(ax, (f32x4v)(4.30638e-5f), (f32x4v)(2.765672e-4f));
  p = __builtin_elementwise_fma(p, ax, (f32x4v)(1.520143e-4f));
  p = __builtin_elementwise_fma(p, ax, (f32x4v)(9.2705272e-3f));
  p = __builtin_elementwise_fma(p, ax, (f32x4v)(4.22820123e-2f));
  p = __builtin_elementwise_fma(p, ax, (f32x4v)(7.05230784e-2f));
  p = __builtin_elementwise_fma(p, ax, (f32x4v)(1.f));
  p *= p;
  p *= p;
  p *= p;
  p *= p;
  const f32x4v r = {__builtin_amdgcn_rcpf(p[0]), __builtin_amdgcn_rcpf(p[1]), __builtin_amdgcn_rcpf(p[2]),
                    __builtin_amdgcn_rcpf(p[3])};
  return __builtin_elementwise_copysign((f32x4v)(1.f) - r, x);
}

__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  float p = __builtin_fmaf(ax, 4.30638e-5f, 2.765672e-4f);
  p = __builtin_fmaf(p, ax, 1.520143e-4f);
  p = __builtin_fmaf(p, ax, 9.2705272e-3f);
  p = __builtin_fmaf(p, ax, 4.22820123e-2f);
  p = __builtin_fmaf(p, ax, 7.05230784e-2f);
  p = __builtin_fmaf(p, ax, 1.f);
  p *= p;
  p *= p;
  p *= p;
  p *= p;                                                   // inf for large |x|: rcp -> 0, erf -> 1
  return copysignf(1.f - __builtin_amdgcn_rcpf(p), x);
}

// EPI = 0: bf16 output (+ residual, or + a per-image vector; optionally the GroupNorm partials of the
// stored tile).  EPI = 1 (GEGLU, 1x1 only): the weight rows come interleaved per 32 as [16 value
// rows | the 16 matching gate rows] (GCfgG), and the epilogue writes y[p, c] = value * gelu(gate) of
// channel c (erf to 1.8e-6, each step rounded to bf16 as torch's eager GEGLU does) into a (M, cout/2)
// output.  EPI = 2: split-K slice, fp32 accumulators to workspace[split].
// AM (addressing): 1 = 32-bit buffer offsets precomputed per DMA row (input below 2^31 bytes): the
// per-step address is one add + the padding mask; 2 = the same with the x2 nearest upsample read on
// the fly (per row: the source pixel's offset and the output pixel's parities; a tap's source row /
// column step is -1, 0 or +1 by parity, two selects + adds per row and step); 0 = 64-bit pointers
// rebuilt per step (inputs beyond 2^31 bytes).
template <int KS, int EPI, int AM, int CF>
__device__ __forceinline__ void conv_tile(const vp2p_conv_args& a) {
  using Cfg = std::conditional_t<EPI == 1, GCfgG<CF>, GCfg<CF>>;
  static_assert(Cfg::NWV == GCfg<CF>::NWV && Cfg::LDS <= GCfg<CF>::LDS, "the launch's block and LDS");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / Cfg::WCOL, wn = w - (w / Cfg::WCOL) * Cfg::WCOL;
  // B blocks of this wave: 8 * (w + Cfg::NWV * i) for i < nbd (8 waves: waves 0-3 take three, 4-7 two)
  const int nbd = (Cfg::BBLK - w + Cfg::NWV - 1) / Cfg::NWV;
  const int M = a.batch * a.out_h * a.out_w;
  const int ntn = a.cout / Cfg::TBN;
  const int ks_n = EPI == 2 ? a.ksplit : 1;
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid0 % ks_n, bid = bid0 / ks_n;
#if VP2P_K10_GROUPM > 0
  // grouped raster: GROUPM row tiles x all column tiles per group, row tile fastest, so an XCD's
  // contiguous share of the grid covers GROUPM rows x a few columns (fewer weight bytes per XCD)
  int mt, nt;
  if (ks_n == 1) {
    const int mtn = (M + Cfg::TBM - 1) / Cfg::TBM;
    const int per = VP2P_K10_GROUPM * ntn, g = bid / per, first = g * VP2P_K10_GROUPM;
    const int gs = min(mtn - first, VP2P_K10_GROUPM), in = bid - g * per;
    mt = first + in % gs;
    nt = in / gs;
  } else {
    if (KS > 1 && VP2P_K10_SPLIT_RASTER) {
      // split-K 3x3: one group of all row tiles, row tile fastest (the K slices of a tile adjacent),
      // so an XCD's share covers whole column tiles and each weight column is fetched by one XCD:
      // the 8x8 / 16x16-latent convs 7-22 % faster (profiles/r05_k10_split_raster*_ab.jsonl; the
      // split-K 1x1 GEMMs 2-4 % slower that way, so they keep row-major)
      const int mtn = (M + Cfg::TBM - 1) / Cfg::TBM;
      nt = bid / mtn;
      mt = bid - nt * mtn;
    } else {
      mt = bid / ntn;
      nt = bid - mt * ntn;
    }
  }
#else
  const int mt = bid / ntn, nt = bid - mt * ntn;
#endif
  const int m0 = mt * Cfg::TBM, n0 = nt * Cfg::TBN;
  const bf16* x = static_cast<const bf16*>(a.x);
  const bf16* wt = static_cast<const bf16*>(a.w);
  const int Kw = KS * KS * a.cin;
  const bf16* zero = reinterpret_cast<const bf16*>(kZero16);

  // this lane's rows: A instruction i of wave w covers rows RPI*(w + NWV*i) .. +RPI-1, lane row l / CPW
  const int lr = l / Cfg::CPW, lj = l % Cfg::CPW;
  int a_n[Cfg::ADMA], a_iy[Cfg::ADMA], a_ix[Cfg::ADMA], a_c[Cfg::ADMA];
  bool a_ok[Cfg::ADMA];
#pragma unroll
  for (int i = 0; i < Cfg::ADMA; ++i) {
    const int r = Cfg::RPI * (w + Cfg::NWV * i) + lr;
    const int p = m0 + r;
    a_ok[i] = p < M;
    const int pp = a_ok[i] ? p : 0;
    const int n = pp / (a.out_h * a.out_w), rem = pp - n * a.out_h * a.out_w;
    const int oy = rem / a.out_w, ox = rem - oy * a.out_w;
    a_n[i] = n;
    a_iy[i] = oy * a.stride - a.pad;
    a_ix[i] = ox * a.stride - a.pad;
    a_c[i] = Cfg::swz(r, lj) * 8;                             // source channel offset of this lane
  }
  int b_c[Cfg::BDMA];
#pragma unroll
  for (int i = 0; i < Cfg::BDMA; ++i) b_c[i] = Cfg::swz(Cfg::RPI * (w + Cfg::NWV * i) + lr, lj) * 8;
  // buffer forms: byte offsets at tap (0, 0) (AM 2: of the source pixel under the output pixel) and
  // the out-of-image tap masks (bit kh * KS + kw; AM 2: the output pixel's parities in bits 16, 17)
  uint32_t a_off[Cfg::ADMA], a_bad[Cfg::ADMA], b_off[Cfg::BDMA];
  __amdgpu_buffer_rsrc_t xr, wr;
  const int sh = a.in_h >> (AM == 2), sw = a.in_w >> (AM == 2);   // stored image
  const int cin1 = a.cin - a.cin2;       // channels (and row stride) of x; x2 holds the last cin2
  if constexpr (AM != 0) {
    xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0,
                                           (uint32_t)a.batch * sh * sw * cin1 * 2u, 0x00020000);
    wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, (uint32_t)a.cout * Kw * 2u, 0x00020000);
#pragma unroll
    for (int i = 0; i < Cfg::ADMA; ++i) {
      if constexpr (AM == 2) {
        const int oy = a_iy[i] + a.pad, ox = a_ix[i] + a.pad;       // stride 1
        a_off[i] = (uint32_t)((((a_n[i] * sh + (oy >> 1)) * sw + (ox >> 1)) * a.cin + a_c[i]) * 2);
      } else {
        a_off[i] = (uint32_t)((((a_n[i] * a.in_h + a_iy[i]) * a.in_w + a_ix[i]) * cin1 + a_c[i]) * 2);
      }
      uint32_t bad = 0;
#pragma unroll
      for (int kh = 0; kh < KS; ++kh)
#pragma unroll
        for (int kw = 0; kw < KS; ++kw) {
          const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
          if (!a_ok[i] || iy < 0 || iy >= a.in_h || ix < 0 || ix >= a.in_w) bad |= 1u << (kh * KS + kw);
        }
      if constexpr (AM == 2) bad |= ((uint32_t)((a_iy[i] + a.pad) & 1) << 16) | ((uint32_t)((a_ix[i] + a.pad) & 1) << 17);
      a_bad[i] = bad;
    }
#pragma unroll
    for (int i = 0; i < Cfg::BDMA; ++i) {
      const int row = Cfg::RPI * (w + Cfg::NWV * i) + lr < Cfg::TBN ? Cfg::RPI * (w + Cfg::NWV * i) + lr : Cfg::TBN - 1;
      b_off[i] = (uint32_t)(((n0 + row) * Kw + b_c[i]) * 2);
    }
  }

  // two-source 1x1 input: the pixel's offsets in x2 (row stride cin2) for the K-steps past cin1
  uint32_t a_off2[Cfg::ADMA];
  __amdgpu_buffer_rsrc_t xr2 = xr;
  if constexpr (AM == 1 && KS == 1) {
    if (a.x2) {
      xr2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x2), 0,
                                              (uint32_t)a.batch * a.in_h * a.in_w * a.cin2 * 2u, 0x00020000);
#pragma unroll
      for (int i = 0; i < Cfg::ADMA; ++i)
        a_off2[i] = (uint32_t)((((a_n[i] * a.in_h + a_iy[i]) * a.in_w + a_ix[i]) * a.cin2 + a_c[i]) * 2);
    }
  }
  const int csteps = a.cin / Cfg::KB;
  const int nall = KS * KS * csteps;
  const int s_begin = (int)((int64_t)nall * split / ks_n), s_end = (int)((int64_t)nall * (split + 1) / ks_n);
  auto dma = [&](int step, int stage) {
#if VP2P_K10_CMAJOR
    // channel-major K order: the KS x KS taps of one 64-channel chunk in consecutive steps, so the
    // shifted re-reads of a chunk's rows (128 B, one L2 line) hit L2
    const int cs = KS == 1 ? step : step / (KS * KS), tap = step - cs * (KS * KS), c0 = cs * Cfg::KB;
#else
    const int tap = step / csteps, c0 = (step - tap * csteps) * Cfg::KB;
#endif
    const int kh = tap / KS, kw = tap - kh * KS;
    char* As = smem + stage * Cfg::STAGE;
    char* Bs = As + Cfg::TBM * Cfg::RB;
    if constexpr (AM != 0) {
      if constexpr (AM == 2) {
        // source row step of tap row kh for output-row parity py: kh 0 -> py - 1, 1 -> 0, 2 -> py
        const uint32_t rs = (uint32_t)(sw * a.cin * 2), cs = (uint32_t)(a.cin * 2);
        const uint32_t ry0 = kh == 0 ? 0u - rs : 0u, ry1 = kh == 2 ? rs : 0u;
        const uint32_t cx0 = kw == 0 ? 0u - cs : 0u, cx1 = kw == 2 ? cs : 0u;
        const uint32_t xs = (uint32_t)(c0 * 2);
#pragma unroll
        for (int i = 0; i < Cfg::ADMA; ++i) {
          const uint32_t o = a_off[i] + xs + ((a_bad[i] >> 16) & 1 ? ry1 : ry0) + ((a_bad[i] >> 17) & 1 ? cx1 : cx0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, to_lds(As + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                                   16, o | ((a_bad[i] >> tap) << 31), 0, 0, 0);
        }
      } else if (KS == 1 && a.x2 && c0 >= cin1) {           // 1x1, second source (wave-uniform)
        const uint32_t xs = (uint32_t)((c0 - cin1) * 2);
#pragma unroll
        for (int i = 0; i < Cfg::ADMA; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr2, to_lds(As + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                                   16, (a_off2[i] + xs) | ((a_bad[i] >> tap) << 31), 0, 0, 0);
      } else {
        const uint32_t xs = (uint32_t)(((kh * a.in_w + kw) * cin1 + c0) * 2);
#pragma unroll
        for (int i = 0; i < Cfg::ADMA; ++i)
#if defined(VP2P_K10_DIAG) && (VP2P_K10_DIAG & 4)      // lab: no A DMA
          if (false)
#endif
          __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, to_lds(As + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                                   16, (a_off[i] + xs) | ((a_bad[i] >> tap) << 31), 0, 0, 0);
      }
      const uint32_t ws = (uint32_t)((tap * a.cin + c0) * 2);
#pragma unroll
      for (int i = 0; i < Cfg::BDMA; ++i)
#if defined(VP2P_K10_DIAG) && (VP2P_K10_DIAG & 8)      // lab: no B DMA
        if (false)
#endif
        if (Cfg::BDMA * Cfg::NWV == Cfg::BBLK || i < nbd)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, to_lds(Bs + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                                   16, b_off[i] + ws, 0, 0, 0);
      return;
    }
#pragma unroll
    for (int i = 0; i < Cfg::ADMA; ++i) {
      const int iy = a_iy[i] + kh, ix = a_ix[i] + kw;
      const bool ok = a_ok[i] && iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w;
      // upsample = 1: the input is nearest-upsampled x2 on the fly (Upsample3D, resnet.py:79-99):
      // (iy, ix) of the virtual in_h x in_w image reads source pixel (iy/2, ix/2)
      const int up = a.upsample;
      const bf16* src = ok ? x + (((int64_t)a_n[i] * (a.in_h >> up) + (iy >> up)) * (a.in_w >> up) + (ix >> up)) *
                                     a.cin + c0 + a_c[i]
                           : zero;
      __builtin_amdgcn_global_load_lds(src, to_lds(As + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                       16, 0, 0);
    }
    const int64_t kofs = (int64_t)tap * a.cin + c0;
#pragma unroll
    for (int i = 0; i < Cfg::BDMA; ++i) {
      if (Cfg::BDMA * Cfg::NWV != Cfg::BBLK && i >= nbd) continue;
      const int row = Cfg::RPI * (w + Cfg::NWV * i) + lr;
      const bf16* src = wt + (int64_t)(n0 + row) * Kw + kofs + b_c[i];
      __builtin_amdgcn_global_load_lds(src, to_lds(Bs + Cfg::RPI * (w + Cfg::NWV * i) * Cfg::RB),
                                       16, 0, 0);
    }
  };

  f32x4v acc[Cfg::WTM][Cfg::WTN];
#pragma unroll
  for (int i = 0; i < Cfg::WTM; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::WTN; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int fr = l & 15, fq = l >> 4;           // fragment row / 16-byte chunk within the 32-wide k-step
  // prologue: the first NSTAGE - 1 steps' DMA in flight (one step for the two-stage tiles)
#pragma unroll
  for (int k = 0; k < Cfg::NSTAGE - 1; ++k)
    if (s_begin + k < s_end) dma(s_begin + k, k);
  // this wave's LDS-DMA instructions per step (the B blocks do not always split evenly over waves)
  constexpr int CNT_HI = Cfg::ADMA + Cfg::BDMA, CNT_LO = Cfg::BBLK % Cfg::NWV == 0 ? CNT_HI : CNT_HI - 1;
  const bool hi = w < Cfg::BBLK % Cfg::NWV || Cfg::BBLK % Cfg::NWV == 0;
  int cur = 0;                                    // LDS stage of this step
  for (int step = s_begin; step < s_end; ++step) {
    if constexpr (Cfg::NSTAGE == 2) {
#ifndef VP2P_K10_DIAG
      __syncthreads();                            // vmcnt(0): step's DMA landed; step-1's reads done
      if (step + 1 < s_end) dma(step + 1, cur ^ 1);
#else   // lab diagnostics only (wrong results): 1 = no main-loop DMA, 2 = no barrier, 4 / 8 = no A / B DMA
      if (!(VP2P_K10_DIAG & 2)) __syncthreads();
      if (!(VP2P_K10_DIAG & 1) && step + 1 < s_end) dma(step + 1, cur ^ 1);
#endif
    } else {
      // this wave's DMA of `step` landed (the ones of the next steps may stay in flight: in-order
      // vmcnt), then every wave's: the barrier also orders all reads of stage (step - 1) % NSTAGE
      // before the DMA of step + NSTAGE - 1 overwrites it.  A raw s_barrier: __syncthreads() would
      // drain the ring.
      const int ahead = min(Cfg::NSTAGE - 2, s_end - 1 - step);   // later steps already issued
      if (ahead >= 2) {
        if (hi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * CNT_HI) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * CNT_LO) : "memory");
      } else if (ahead == 1) {
        if (hi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT_HI) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CNT_LO) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (step + Cfg::NSTAGE - 1 < s_end)
        dma(step + Cfg::NSTAGE - 1, cur == 0 ? Cfg::NSTAGE - 1 : cur - 1);
    }
    const char* As = smem + cur * Cfg::STAGE;
    const char* Bs = As + Cfg::TBM * Cfg::RB;
    cur = cur + 1 == Cfg::NSTAGE ? 0 : cur + 1;
    if constexpr (kPipe && Cfg::NSTAGE == 2 && Cfg::CPW == 8 && (AM != 0 || Cfg::NWV <= 4)) {
      // Fragment reads software-pipelined against the MFMAs, slot by slot.  Per 32-channel k-step
      // the smaller operand set is held (H: the wave's B fragments when WTN <= WTM, else its A
      // fragments) and the larger one rotates through three registers (R): group g issues the
      // NH MFMAs of rotating fragment g and the read of fragment g + 2; the second k-step's held
      // set is read during the first k-step's groups.  Every read is then >= 2 groups (>= 2 NH
      // MFMAs) ahead of its first use instead of just before it, and each group is pinned by a
      // sched_barrier (left to itself hipcc issued the A reads in pairs right before their MFMAs:
      // s_waitcnt lgkmcnt(1 / 0) every 5 MFMAs).
      constexpr bool HB = Cfg::WTN <= Cfg::WTM;
      constexpr int NH = HB ? Cfg::WTN : Cfg::WTM, NR = HB ? Cfg::WTM : Cfg::WTN;
      auto ldA = [&](int ks, int i) {
        const int r = wm * Cfg::WR + 16 * i + fr;
        return *reinterpret_cast<const bf16x8*>(As + r * Cfg::RB + Cfg::swz(r, 4 * ks + fq) * 16);
      };
      auto ldB = [&](int ks, int j) {
        const int r = wn * Cfg::WN + 16 * j + fr;
        return *reinterpret_cast<const bf16x8*>(Bs + r * Cfg::RB + Cfg::swz(r, 4 * ks + fq) * 16);
      };
      auto ldH = [&](int ks, int k) { return HB ? ldB(ks, k) : ldA(ks, k); };
      auto ldR = [&](int ks, int k) { return HB ? ldA(ks, k) : ldB(ks, k); };
      // R[1] below is fragment (ks 0, idx 1): the rotation assumes two fragments per k-step
      static_assert(NR >= 2, "pipelined fragment reads need NR = max(WTM, WTN) >= 2");
      bf16x8 H[2][NH], R[3];
#pragma unroll
      for (int k = 0; k < NH; ++k) H[0][k] = ldH(0, k);
      R[0] = ldR(0, 0);
      R[1] = ldR(0, 1);
#pragma unroll
      for (int g = 0; g < 2 * NR; ++g) {
        const int ks = g / NR, rr = g - ks * NR, gn = g + 2;
        if (gn < 2 * NR) R[gn % 3] = ldR(gn / NR, gn % NR);
        if (ks == 0 && rr < NH) H[1][rr] = ldH(1, rr);
#pragma unroll
        for (int k = 0; k < NH; ++k) {
          if constexpr (HB) acc[rr][k] = mfma16(R[g % 3], H[ks][k], acc[rr][k]);
          else acc[k][rr] = mfma16(H[ks][k], R[g % 3], acc[k][rr]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      continue;
    }
#pragma unroll
    for (int ks = 0; ks < Cfg::CPW; ks += 4) {   // chunk index of the 32-channel MFMA k-step (0 or 4)
      bf16x8 af[Cfg::WTM], bfr[Cfg::WTN];
#pragma unroll
      for (int i = 0; i < Cfg::WTM; ++i) {
        const int r = wm * Cfg::WR + 16 * i + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * Cfg::RB + Cfg::swz(r, ks + fq) * 16);
      }
#pragma unroll
      for (int j = 0; j < Cfg::WTN; ++j) {
        const int r = wn * Cfg::WN + 16 * j + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + r * Cfg::RB + Cfg::swz(r, ks + fq) * 16);
      }
#pragma unroll
      for (int i = 0; i < Cfg::WTM; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::WTN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  }

  if constexpr (EPI == 2) {
    // fp32 slice: lane holds rows 4*fq+e of column fr of each 16x16 tile
    float* ws = a.workspace + (int64_t)split * M * a.cout;
#pragma unroll
    for (int i = 0; i < Cfg::WTM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int p = m0 + wm * Cfg::WR + 16 * i + 4 * fq + e;
        if (p < M) {
#pragma unroll
          for (int j = 0; j < Cfg::WTN; ++j) ws[(int64_t)p * a.cout + n0 + wn * Cfg::WN + 16 * j + fr] = acc[i][j][e];
        }
      }
    return;
  }
  const bf16* bias = static_cast<const bf16*>(a.bias);
  if constexpr (EPI == 1) {
    // GEGLU straight from the accumulators: tile 2q of the wave holds the values and tile 2q + 1 the
    // gates of the same 16 channels (weights interleaved per 32 rows), so lane l has a channel's value and
    // gate for rows 4 * fq + e, e = 0..3, and forms those four outputs on packed FP32 -- the
    // projection rounded to bf16, gelu rounded, the product rounded, exactly K9's order.  The
    // (TBM, TBN / 2) output tile is staged in LDS (free after the last K-step) and leaves as whole
    // 16-byte row segments.
#pragma clang fp contract(off)
    constexpr float kAlpha = 0.70710678118654752440f;
    constexpr int OW = Cfg::TBN / 2, OROW = OW + 8;                 // output tile row (elements)
    static_assert(Cfg::TBM * OROW * 2 <= Cfg::LDS, "GEGLU output tile in LDS");
    const int half = a.cout / 2;
    bf16* Os = reinterpret_cast<bf16*>(smem);
    __syncthreads();                                                // every wave done with the stages
#pragma unroll
    for (int q = 0; q < Cfg::WTN / 2; ++q) {
      const int gv = n0 + wn * Cfg::WN + 32 * q + fr;               // value column; gate: gv + 16
      const float bv = bias ? (float)bias[gv] : 0.f, bg = bias ? (float)bias[gv + 16] : 0.f;
      const int oc = wn * (Cfg::WN / 2) + 16 * q + fr;              // output channel within the tile
#pragma unroll
      for (int i = 0; i < Cfg::WTM; ++i) {
        const int rb = wm * Cfg::WR + 16 * i + 4 * fq;
        {
          // the lane's four rows as one 4-vector: every step is two independent packed ops, so the
          // dependent-issue wait of packed FP32 never stalls
          const f32x4v val = round_bf16x4(acc[i][2 * q] + bv);
          const f32x4v g = round_bf16x4(acc[i][2 * q + 1] + bg);
          const f32x4v ge = round_bf16x4(g * 0.5f * (1.f + erf_fast4(g * kAlpha)));
          const f32x4v o = val * ge;
#pragma unroll
          for (int e = 0; e < 4; ++e) Os[(rb + e) * OROW + oc] = (bf16)o[e];
        }
      }
    }
    __syncthreads();
    bf16* y = static_cast<bf16*>(a.y);
    for (int c = tid; c < Cfg::TBM * (OW / 8); c += Cfg::NT) {
      const int row = c / (OW / 8), ch = c - row * (OW / 8);
      const int p = m0 + row;
      if (p < M)
        *reinterpret_cast<bf16x8*>(y + (int64_t)p * half + n0 / 2 + ch * 8) =
            *reinterpret_cast<const bf16x8*>(Os + row * OROW + ch * 8);
    }
    return;
  }
  bf16* Cs = reinterpret_cast<bf16*>(smem);
  const float al = a.alpha == 0.f ? 1.f : a.alpha;     // x 1.0f is exact: alpha-free callers unchanged
  const bf16* res = static_cast<const bf16*>(a.residual);
  const bf16* iadd = static_cast<const bf16*>(a.img_add);
  const int hw = a.out_h * a.out_w;
  bf16* y = static_cast<bf16*>(a.y);
  // GroupNorm statistics of the stored tile (vp2p_conv2d_gn_parts checked the geometry): the tile
  // holds GT whole groups of cg channels; tpg threads per group, each summing fixed channel pairs over
  // a stride of rows (shifted sums, the shift its first value), merged (Chan) across the tpg lanes
  const bool gn = a.gn_partials != nullptr;
  const int cg = gn ? a.cout / a.gn_groups : 2, GT = Cfg::TBN / cg, tpg = Cfg::NT / GT, hc = cg >> 1;
  const int gi = tid / tpg, gk = tid - gi * tpg, grs = tpg / hc;          // rows per step
  const bool gact = gk < grs * hc;
  const int gcp = gk % hc, gr0 = gk / hc;
  float gK = 0.f, gs1 = 0.f, gs2 = 0.f;
  int gn_n = 0;
  // rows [pass * EROWS, (pass + 1) * EROWS) of the tile go through the LDS tile at a time
  for (int pass = 0; pass < Cfg::TBM / Cfg::EROWS; ++pass) {
  __syncthreads();
  if (wm * Cfg::WR / Cfg::EROWS == pass) {
    const int rb = wm * Cfg::WR - pass * Cfg::EROWS;
#pragma unroll
    for (int j = 0; j < Cfg::WTN; ++j) {
      const int col = wn * Cfg::WN + 16 * j + fr;
      const float bv = bias ? (float)bias[n0 + col] : 0.f;
#pragma unroll
      for (int i = 0; i < Cfg::WTM; ++i) {
        // the lane's four rows of the column as a 4-vector: packed adds / multiplies / conversions
        const f32x4v v = (acc[i][j] + bv) * al;
        const bf16x2v lo = __builtin_convertvector(f32x2v{v[0], v[1]}, bf16x2v);
        const bf16x2v hi = __builtin_convertvector(f32x2v{v[2], v[3]}, bf16x2v);
        bf16* c = Cs + (rb + 16 * i + 4 * fq) * Cfg::CROWV + col;
        c[0] = lo.x;
        c[Cfg::CROWV] = lo.y;
        c[2 * Cfg::CROWV] = hi.x;
        c[3 * Cfg::CROWV] = hi.y;
      }
    }
  }
  __syncthreads();
  const int mp = m0 + pass * Cfg::EROWS;
  for (int c = tid; c < Cfg::EROWS * (Cfg::TBN / 8); c += Cfg::NT) {
    const int row = c / (Cfg::TBN / 8), ch = c - row * (Cfg::TBN / 8);
    const int p = mp + row;
    if (p >= M) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(Cs + row * Cfg::CROWV + ch * 8);
    const int64_t o = (int64_t)p * a.cout + n0 + ch * 8;
    if (res) {
      const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)rv[j]);
    }
    if (iadd) {        // h + temb: the image's vector, one more rounding (resnet.py:149-156)
      const bf16x8 tv = *reinterpret_cast<const bf16x8*>(iadd + (int64_t)(p / hw) * a.cout + n0 + ch * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)tv[j]);
    }
    *reinterpret_cast<bf16x8*>(y + o) = v;
    if (gn) *reinterpret_cast<bf16x8*>(Cs + row * Cfg::CROWV + ch * 8) = v;   // the stored values
  }
  if (gn) {
    __syncthreads();
    if (gact) {
      for (int r = gr0; r < Cfg::EROWS; r += grs) {
        const bf16x2v t = *reinterpret_cast<const bf16x2v*>(Cs + r * Cfg::CROWV + gi * cg + 2 * gcp);
        const float x0 = (float)t.x, x1 = (float)t.y;
        if (gn_n == 0) gK = x0;
        const float d0 = x0 - gK, d1 = x1 - gK;
        gs1 += d0 + d1;
        gs2 = fmaf(d0, d0, fmaf(d1, d1, gs2));
        gn_n += 2;
      }
    }
  }
  }
  if (gn) {
    const float fn = (float)gn_n, inv = gn_n ? 1.f / fn : 0.f;
    Welford w = {fn, gK + gs1 * inv, fmaxf(gs2 - gs1 * gs1 * inv, 0.f)};
    for (int off = tpg >> 1; off > 0; off >>= 1) {
      const Welford o = {__shfl_xor(w.n, off), __shfl_xor(w.mean, off), __shfl_xor(w.m2, off)};
      w = wmerge(w, o);
    }
    if (gk == 0) {
      const int parts = a.gn_rows / Cfg::TBM, smp = m0 / a.gn_rows, t = (m0 - smp * a.gn_rows) / Cfg::TBM;
      float* o = a.gn_partials + (((int64_t)smp * parts + t) * a.gn_groups + n0 / cg + gi) * 3;
      o[0] = w.n;
      o[1] = w.mean;
      o[2] = w.m2;
    }
  }
}

template <int KS, int EPI = 0, int AM = 1>
__global__ __launch_bounds__(256, 2) void conv_kernel_g(const vp2p_conv_args a) {
  conv_tile<KS, EPI, AM, 0>(a);
}

template <int KS, int EPI = 0, int AM = 1>
__global__ __launch_bounds__(512, 1) void conv_kernel_b(const vp2p_conv_args a) {
  conv_tile<KS, EPI, AM, 1>(a);
}

template <int KS, int EPI = 0, int AM = 1>
__global__ __launch_bounds__(512, 1) void conv_kernel_w(const vp2p_conv_args a) {
  conv_tile<KS, EPI, AM, 2>(a);
}

template <int KS, int EPI = 0, int AM = 1>
__global__ __launch_bounds__(256, 2) void conv_kernel_s(const vp2p_conv_args a) {
  conv_tile<KS, EPI, AM, 3>(a);
}

template <int KS, int EPI = 0, int AM = 1>
__global__ __launch_bounds__(512, 1) void conv_kernel_m(const vp2p_conv_args a) {
  conv_tile<KS, EPI, AM, 4>(a);
}

// ------------------------------------------------------------------------------------------------
// K10s: the K = 320 1x1 GEMMs of the 64x64-latent transformer blocks as a persistent stream --
// proj_in, to_q, to_out, proj_out, attn_temp's to_out (N = 320: y = x W^T (+ bias) (* alpha)
// (+ residual)), attn_temp's q|k|v (N = 960) and the GEGLU projection (N = 2560 interleaved, the
// GEGLU epilogue); M = B f 4096 rows.  The N = 320 ones are HBM-bound (640 B in and 640 B out per
// row against 205 KFLOP), and the tiled kernels ran them at ~2.9 TB/s: each 256 x 320 tile is 5
// K-steps between a prologue and an epilogue that nothing overlaps.  Here a workgroup per CU keeps
// one 320-column group of W in registers (10 waves x 32 output columns x K 320: 80 VGPRs a lane,
// read once) and streams 32-row blocks of x through a 4-slot LDS ring by LDS-DMA, three blocks in
// flight, each block's output staged in LDS and stored as whole row segments.  N = 320 NG: NG
// workgroups share each row block (consecutive logical ids, so one XCD and its L2), each with its
// column group.  Per output the same 16x16x32 MFMAs in the same K order as the tiled kernels (one per
// 32 channels, ascending) and the same epilogue roundings: bit-equal.
// ------------------------------------------------------------------------------------------------
#ifndef VP2P_K10_SKINNY
#define VP2P_K10_SKINNY 1
#endif
#ifndef VP2P_K10S_MINBLK      // the fewest 32-row blocks the stream takes (fewer: the tiled kernels)
#define VP2P_K10S_MINBLK 1024
#endif
constexpr int SK_R = 32;
// ring slots: x (and, with a residual, the residual's rows too, also by LDS-DMA: a register load of
// it would be the youngest vector-memory operation, and waiting for it drains the x prefetch).
// Without a residual the output tile is double-buffered and block li's rows are stored after the
// NEXT iteration's barrier: one barrier per block; the residual variant's ring leaves no room for a
// second tile and keeps a barrier before its stores.  EPI 1 (GEGLU): a wave's 32 columns are 16
// value and the 16 matching gate rows of the interleaved weight, its 16 output channels' value and
// gate in the same lanes; a group writes 160 output channels.
// KK = 640 (the 32x32-latent projections, W 640 x 640): 16 weight rows a wave (the same 80 VGPRs),
// 160-column groups, 40 KB blocks in a 3-slot ring; a wave's A fragments then feed one 16-column
// tile each, so that stream is bound by LDS reads at half the MFMA rate (measured level with the
// tiled kernels; not dispatched, see skinny_kind).
template <int KK, int CW, bool RES, int EPI, int NW_ = 10> struct SkCfg {
  static constexpr int NW = NW_, NT = 64 * NW;                   // waves, threads
  static constexpr int CT = CW / 16;                             // 16-column MFMA tiles per wave
  static constexpr int GW = NW * CW;                             // weight rows (columns) per group
  static constexpr int BLK = SK_R * KK * 2;                      // one block of x rows
  static constexpr int CH = KK * 2 / 16;                         // 16-byte chunks per row
  static constexpr int DPW = SK_R * CH / (64 * NW);              // x DMA instructions per wave per block
  static constexpr int ST = (RES || KK > 320) ? 3 : 4;           // slots: ST - 1 blocks in flight
  static constexpr int SLOT = (RES ? 2 : 1) * BLK;
  static constexpr int OB = RES ? 1 : 2;                         // output tiles
  static constexpr int ON = EPI == 1 ? GW / 2 : GW;              // output columns per group
  static constexpr int OROW = ON + 8;                            // output tile row (elements)
  static constexpr int EPC = SK_R * (ON / 8) / NT;               // output chunks per thread per block
  static constexpr int LDS = ST * SLOT + OB * SK_R * OROW * 2;
  static constexpr int D = (RES ? 2 : 1) * DPW;                  // DMA instructions per wave per block
  // the in-order vmcnt that retires a wave's DMA of block li counts everything issued after it; in the
  // steady state: for each of the next ST - 2 iterations its DMA and its EPC stores (and, with the
  // residual's barrier before the stores, the stores of the iteration that issued it)
  static constexpr int YOUNG = (RES ? EPC : 0) + (ST - 2) * (D + EPC);
  static_assert(SK_R * CH == DPW * 64 * NW && SK_R * (ON / 8) == EPC * NT, "whole instructions / chunks");
  static_assert(!RES || (KK == 320 && CW == 32 && EPI == 0), "a residual on the 320 x 320 stream only");
  static_assert(EPI == 0 || (KK == 320 && CW == 32), "GEGLU: value and gate tiles in one wave");
  static_assert(LDS <= 160 * 1024, "LDS");
  // LDS slot of chunk c of row r: an XOR within aligned groups of 8 chunks (640-B rows: the 16 rows of
  // a quarter-wave alternate two bank halves) or 16 (1280-B rows all start on bank 0)
  __device__ static __forceinline__ int swz(int r, int c) {
    if constexpr (KK == 320) return c ^ ((r >> 1) & 7);
    else return c ^ (r & 15);
  }
};

// one 1 KB lane-linear LDS-DMA (a non-template helper: see to_lds)
__device__ __forceinline__ void sk_dma(__amdgpu_buffer_rsrc_t r, char* dst, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, to_lds(dst), 16, off, 0, 0, 0);
}

template <int KK, int CW, bool RES, int EPI, int NW = 10>
__global__ __launch_bounds__(64 * NW, 1) void conv_kernel_k320(const vp2p_conv_args a) {
  using S = SkCfg<KK, CW, RES, EPI, NW>;
  constexpr int CT = S::CT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, l = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = l & 15, fq = l >> 4;
  const int nblk = a.batch * a.out_h * a.out_w / SK_R;
  const int NG = a.cout / S::GW;                                   // column groups
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int cg = lid % NG, g = lid / NG, G = gridDim.x / NG;       // group, row-stream index, streams
  const int nmine = g < nblk ? (nblk - g + G - 1) / G : 0;
  bf16* Os = reinterpret_cast<bf16*>(smem + S::ST * S::SLOT);
  const int ncol = cg * S::GW + CW * w;                            // this wave's first weight row

  // this wave's CW weight rows: all of K for them, as 16x16x32 B fragments (row ncol + 16 t + fr,
  // channels 32 s + 8 fq .. + 7)
  const bf16* wt = static_cast<const bf16*>(a.w);
  bf16x8 wf[CT][KK / 32];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int s = 0; s < KK / 32; ++s)
      wf[t][s] = *reinterpret_cast<const bf16x8*>(wt + (int64_t)(ncol + 16 * t + fr) * KK + 32 * s + 8 * fq);
  const bf16* bias = static_cast<const bf16*>(a.bias);
  float bv[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) bv[t] = bias ? (float)bias[ncol + 16 * t + fr] : 0.f;
  const float al = a.alpha == 0.f ? 1.f : a.alpha;

  // LDS-DMA: the block's 16-byte slots q = row * CH + j, slot j of a row holding chunk swz(row, j);
  // this wave fills DPW lane-linear 1 KB instructions.  The residual's rows land unswizzled (the
  // epilogue reads them as whole 16-byte chunks).
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (uint32_t)nblk * S::BLK,
                                                                0x00020000);
  __amdgpu_buffer_rsrc_t rr = xr;
  if constexpr (RES)
    rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.residual), 0, (uint32_t)nblk * S::BLK, 0x00020000);
  uint32_t loff[S::DPW];
#pragma unroll
  for (int k = 0; k < S::DPW; ++k) {
    const int q = (S::DPW * w + k) * 64 + l, row = q / S::CH, j = q - row * S::CH;
    loff[k] = (uint32_t)(row * KK * 2 + S::swz(row, j) * 16);
  }
  auto dma = [&](int li) {
    const uint32_t base = (uint32_t)(g + li * G) * S::BLK;
    char* st = smem + (li % S::ST) * S::SLOT;
#pragma unroll
    for (int k = 0; k < S::DPW; ++k) sk_dma(xr, st + (S::DPW * w + k) * 1024, base + loff[k]);
    if constexpr (RES)
#pragma unroll
      for (int k = 0; k < S::DPW; ++k)
        sk_dma(rr, st + S::BLK + (S::DPW * w + k) * 1024, base + ((S::DPW * w + k) * 64 + l) * 16);
  };
  static_assert(S::YOUNG == 10 || S::YOUNG == 8 || S::YOUNG == 6, "the immediates below");
#pragma unroll
  for (int p = 0; p < S::ST - 1; ++p)
    if (p < nmine) dma(p);

  bf16* y = static_cast<bf16*>(a.y);
  const int ystride = EPI == 1 ? a.cout / 2 : a.cout;
  const int ycol = cg * S::ON;
  // block lj's rows from output tile ob (+ its residual from ring slot sl) as whole 16-byte chunks
  auto store = [&](int lj, int ob, const char* sl) {
    const bf16* O = Os + ob * SK_R * S::OROW;
    const int64_t r0 = (int64_t)(g + lj * G) * SK_R;
#pragma unroll
    for (int k = 0; k < S::EPC; ++k) {
      const int c = tid + k * S::NT, row = c / (S::ON / 8), ch = c - row * (S::ON / 8);
      bf16x8 v = *reinterpret_cast<const bf16x8*>(O + row * S::OROW + ch * 8);
      if constexpr (RES) {
        const bf16x8 rv = *reinterpret_cast<const bf16x8*>(sl + S::BLK + c * 16);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)rv[j]);
      }
      *reinterpret_cast<bf16x8*>(y + (r0 + row) * ystride + ycol + ch * 8) = v;
    }
  };
  for (int li = 0; li < nmine; ++li) {
    if (li >= S::ST - 1 && li + S::ST - 2 < nmine) {             // wave-uniform
      if constexpr (S::YOUNG == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if constexpr (S::YOUNG == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();             // every wave's DMA of block li landed, block li - 1's tile written
    if constexpr (!RES)
      if (li > 0) store(li - 1, (li - 1) & 1, nullptr);
    if (li + S::ST - 1 < nmine) dma(li + S::ST - 1);               // into the slot block li - 1 used
    const char* st = smem + (li % S::ST) * S::SLOT;
    f32x4v acc[2][CT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < CT; ++t) acc[i][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KK / 32; ++s) {
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = 16 * i + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(st + row * KK * 2 + S::swz(row, 4 * s + fq) * 16);
      }
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        acc[0][t] = mfma16(af[0], wf[t][s], acc[0][t]);
        acc[1][t] = mfma16(af[1], wf[t][s], acc[1][t]);
      }
    }
    bf16* O = Os + (S::OB == 2 ? (li & 1) : 0) * SK_R * S::OROW;
    if constexpr (EPI == 1) {
      // the tiled kernels' GEGLU epilogue: value and gate rounded to bf16, gelu rounded, the product
      // rounded (K9's order)
#pragma clang fp contract(off)
      constexpr float kAlpha = 0.70710678118654752440f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4v val = round_bf16x4(acc[i][0] + bv[0]);
        const f32x4v gt = round_bf16x4(acc[i][CT - 1] + bv[CT - 1]);
        const f32x4v ge = round_bf16x4(gt * 0.5f * (1.f + erf_fast4(gt * kAlpha)));
        const f32x4v o = val * ge;
#pragma unroll
        for (int e = 0; e < 4; ++e) O[(16 * i + 4 * fq + e) * S::OROW + 16 * w + fr] = (bf16)o[e];
      }
    } else {
      // the tiled kernels' epilogue roundings: (acc + bias) * alpha -> bf16, then + residual -> bf16
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < CT; ++t) {
          const f32x4v v = (acc[i][t] + bv[t]) * al;
          const bf16x2v lo = __builtin_convertvector(f32x2v{v[0], v[1]}, bf16x2v);
          const bf16x2v hi = __builtin_convertvector(f32x2v{v[2], v[3]}, bf16x2v);
          bf16* c = O + (16 * i + 4 * fq) * S::OROW + CW * w + 16 * t + fr;
          c[0] = lo.x;
          c[S::OROW] = lo.y;
          c[2 * S::OROW] = hi.x;
          c[3 * S::OROW] = hi.y;
        }
    }
    if constexpr (RES) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      store(li, 0, st);
    }
  }
  if constexpr (!RES) {
    if (nmine > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      store(nmine - 1, (nmine - 1) & 1, nullptr);
    }
  }
}

template <int KK, int CW, bool RES, int EPI, int NW = 10>
static int launch_k320(const vp2p_conv_args& a, hipStream_t s, int n_cu) {
  using S = SkCfg<KK, CW, RES, EPI, NW>;
  constexpr int lds = S::LDS;
  static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_kernel_k320<KK, CW, RES, EPI, NW>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return VP2P_E_LAUNCH;
  const int ng = a.cout / S::GW;
  const int64_t nblk = (int64_t)a.batch * a.out_h * a.out_w / SK_R;
  int64_t streams = n_cu / ng > 0 ? n_cu / ng : 1;                 // row streams per column group
  if (streams > nblk) streams = nblk;
  hipLaunchKernelGGL((conv_kernel_k320<KK, CW, RES, EPI, NW>), dim3((unsigned)(streams * ng)), dim3(S::NT), lds, s, a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

// the K10s shapes, on whole 32-row blocks, enough of them to give every CU a stream: 1x1, K = 320 and
// N = 320 NG (NG <= 8; a residual only at N = 320; the plain or the GEGLU epilogue).  (K = 640 forms,
// bit-equal, measured level with the tiled kernels on M 32768 K 640 N 640 and are not dispatched:
// 10 waves x 16 rows (SkCfg<640, 16, ...>, LDS-read bound) 39.4 vs 39.7 us,
// profiles/r05_k10s_k640_level.jsonl; 5 waves x 32 rows (SkCfg<640, 32, false, 0, 5>, W in 160 VGPRs,
// one SIMD with two waves against three with one) 39.0 vs 39.2 us and the edit 0.5 % slower,
// profiles/r05_k10s_k640_5w_rejected.jsonl.)
static int skinny_kind(const vp2p_conv_args* a, int64_t M) {
  if (!VP2P_K10_SKINNY || a->kernel != 1 || a->stride != 1 || a->x2 || a->cin2 || a->upsample || a->gn_partials ||
      a->img_add || M % SK_R || M / SK_R < VP2P_K10S_MINBLK || M * a->cin * 2 >= ((int64_t)1 << 31))   // 32-bit offsets
    return 0;
  const bool plain = a->epilogue == VP2P_CONV_EPI_NONE;
  if (a->cin == 320 && a->cout % 320 == 0 && a->cout <= 2560 && (plain || a->epilogue == VP2P_CONV_EPI_GEGLU) &&
      (!a->residual || (a->cout == 320 && plain)))
    return 320;
  return 0;
}

template <int KS, int EPI, int AM, int CF> struct ConvKernel;
template <int KS, int EPI, int AM> struct ConvKernel<KS, EPI, AM, 0> {
  static const void* fn() { return reinterpret_cast<const void*>(&conv_kernel_g<KS, EPI, AM>); }
};
template <int KS, int EPI, int AM> struct ConvKernel<KS, EPI, AM, 1> {
  static const void* fn() { return reinterpret_cast<const void*>(&conv_kernel_b<KS, EPI, AM>); }
};
template <int KS, int EPI, int AM> struct ConvKernel<KS, EPI, AM, 2> {
  static const void* fn() { return reinterpret_cast<const void*>(&conv_kernel_w<KS, EPI, AM>); }
};
template <int KS, int EPI, int AM> struct ConvKernel<KS, EPI, AM, 3> {
  static const void* fn() { return reinterpret_cast<const void*>(&conv_kernel_s<KS, EPI, AM>); }
};
template <int KS, int EPI, int AM> struct ConvKernel<KS, EPI, AM, 4> {
  static const void* fn() { return reinterpret_cast<const void*>(&conv_kernel_m<KS, EPI, AM>); }
};

// split-K second pass: y = round(round(sum_s ws[s] + bias) + residual), the one-pass roundings
__global__ __launch_bounds__(256) void conv_splitk_reduce(const vp2p_conv_args a) {
  const int64_t M = (int64_t)a.batch * a.out_h * a.out_w;
  const int nv = a.cout / 8;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= M * nv) return;
  const int64_t p = e / nv;
  const int c0 = (int)(e - p * nv) * 8;
  const int64_t o = p * a.cout + c0;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  for (int sp = 0; sp < a.ksplit; ++sp) {
    const f32x4v* q = reinterpret_cast<const f32x4v*>(a.workspace + (int64_t)sp * M * a.cout + o);
    const f32x4v lo = q[0], hi = q[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] += lo[j]; v[4 + j] += hi[j]; }
  }
  const bf16* bias = static_cast<const bf16*>(a.bias);
  const bf16* res = static_cast<const bf16*>(a.residual);
  const bf16* iadd = static_cast<const bf16*>(a.img_add);
  const int64_t hw = (int64_t)a.out_h * a.out_w;
  const float al = a.alpha == 0.f ? 1.f : a.alpha;
  bf16x8 out;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = (float)(bf16)((v[j] + (bias ? (float)bias[c0 + j] : 0.f)) * al);
    if (res) t = t + (float)res[o + j];
    if (iadd) t = t + (float)iadd[(p / hw) * a.cout + c0 + j];
    out[j] = (bf16)t;
  }
  *reinterpret_cast<bf16x8*>(static_cast<bf16*>(a.y) + o) = out;
}

template <int KS, int EPI, int AM, int CF>
static int launch_g1(const vp2p_conv_args& a, dim3 grid, hipStream_t s) {
  using Cfg = GCfg<CF>;
  static const bool attr = hipFuncSetAttribute(ConvKernel<KS, EPI, AM, CF>::fn(),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Cfg::LDS) == hipSuccess;
  if (!attr) return VP2P_E_LAUNCH;
  if constexpr (CF == 0)
    hipLaunchKernelGGL((conv_kernel_g<KS, EPI, AM>), grid, dim3(Cfg::NT), Cfg::LDS, s, a);
  else if constexpr (CF == 1)
    hipLaunchKernelGGL((conv_kernel_b<KS, EPI, AM>), grid, dim3(Cfg::NT), Cfg::LDS, s, a);
  else if constexpr (CF == 2)
    hipLaunchKernelGGL((conv_kernel_w<KS, EPI, AM>), grid, dim3(Cfg::NT), Cfg::LDS, s, a);
  else if constexpr (CF == 3)
    hipLaunchKernelGGL((conv_kernel_s<KS, EPI, AM>), grid, dim3(Cfg::NT), Cfg::LDS, s, a);
  else
    hipLaunchKernelGGL((conv_kernel_m<KS, EPI, AM>), grid, dim3(Cfg::NT), Cfg::LDS, s, a);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

// am: addressing form (see conv_kernel_g); the upsampling form exists for the 3x3 one-pass kernel only
template <int KS, int EPI, int CF = 0>
static int launch_g(const vp2p_conv_args& a, dim3 grid, int am, hipStream_t s) {
  if constexpr (KS == 3 && EPI == 0)
    if (am == 2) return launch_g1<KS, EPI, 2, CF>(a, grid, s);
  return am == 1 ? launch_g1<KS, EPI, 1, CF>(a, grid, s) : launch_g1<KS, EPI, 0, CF>(a, grid, s);
}

// Tile choice for one-pass launches (split-K launches always take CF 0).
// CF 1 (256 x 160, 3 stages): measured (profiles/r03_k10_tile_ab.jsonl, bit-equal) to win only on the
// long-K 1x1 GEMMs (M 131072, K 1280, N 320: 185.5 -> 170.2 us), 2-8 % slower on the 3x3 convs and
// the K = 320 GEMM / GEGLU shapes.  CF 2 (256 x 320 wide): Cout % 320 == 0 and enough
// tiles to give every CU one.  (A wide tile on 32-channel K-steps in a four-stage ring, three steps'
// DMA in flight, measured bit-equal but 4-10 % slower on every shape:
// profiles/r03_k10_deep_rejected.jsonl.)
// The wide tile wherever it gives every CU a tile (measured, profiles/r03_k10_wide_ab.jsonl, bit-equal:
// 3x3 convs at 64^2 / 32^2 -6..-13 %, 1x1 GEMMs M 131072 K 320 / 1280 N 320 -5 / -21 %, M 32768 K 640
// N 640 -10 %; slower where it leaves CUs idle: 128-tile grids +3..+50 %) -- unless its grid ends in a
// part-filled wave that the 128 x 160 grid (two workgroups per CU) does not: the wide tile's ~12 %
// per-tile advantage against the two grids' last-wave fill (M 8192 K 1280 N 3840: 384 wide tiles =
// 1.5 waves, 1536 128-row tiles = 3 full waves).
static double wave_fill(int64_t tiles, int64_t slots) {
  return (double)tiles / (double)(((tiles + slots - 1) / slots) * slots);
}

static int pick_tile(const vp2p_conv_args* a, int64_t M) {
#ifdef VP2P_K10_FORCE_CF   // lab A/B builds only (tools/lab_build.sh)
  if (VP2P_K10_FORCE_CF != 2 || a->cout % 320 == 0) return VP2P_K10_FORCE_CF;
#endif
  const int64_t tiles_b = (M + 255) / 256 * (a->cout / BN);
  const int64_t tiles_0 = (M + GBM - 1) / GBM * (a->cout / BN);
  const bool wide_ok = a->cout % 320 == 0;    // plain and GEGLU epilogues (GEGLU: profiles/r03_k10_geglu_wide_ab.jsonl)
  const int64_t tiles_w = (M + 255) / 256 * (a->cout / 320);
  if (wide_ok && tiles_w >= 256 && 1.12 * wave_fill(tiles_w, 256) >= wave_fill(tiles_0, 512)) return 2;
  return (tiles_b >= 256 && a->kernel == 1 && a->cin >= 1280) ? 1 : 0;
}

// the 64-row tile where the 128-row grid leaves CUs idle (< 384 tiles) and the 64-row one fills
// them: >= 384 tiles, or >= 256 on short K (<= 48 K-steps; longer K keeps split-K, which measured
// faster there).  Small-clip shapes, profiles/r04_k10_short_tile.jsonl: 1-frame res-64 3x3
// 56.2 -> 43.4 us, 2-frame res-32 3x3 (320 -> 640) 50.5 -> 35.2 us, M 4096 K 640 N 640 14.4 -> 10.0 us.
// Not for a long-K 3x3 (> 96 steps) whose 64-row grid still ends in a part-filled wave: split-K over
// 128-row tiles measured faster there (profiles/r06_k10_plan_sweep.jsonl, the 3-frame clip's 16x16
// convs, M 3072 N 1280 K 1280 / 1920 / 2560 x 9: 114.7 / 161.1 / 224.2 -> 101.2 / 135.9 / 171.6 us at
// 4 slices), except on the upsampling form, which split-K would give up.
static bool short_tile(const vp2p_conv_args* a, int64_t M) {
  const int64_t tiles = (M + GBM - 1) / GBM * (a->cout / BN);
  const int64_t tiles_s = (M + 63) / 64 * (a->cout / BN);
  const int nsteps = a->kernel * a->kernel * (a->cin / BK);
  if (a->kernel == 3 && nsteps > 96 && tiles_s < 512 && !a->upsample) return false;
  // short-K projections (<= 30 K-steps) on however few tiles: one pass beat the 2-slice split there
  // (M 1024 / 768 / 256, K 1280, N 1280: 19.0 / 17.9 / 14.8 -> 13.1 / 12.9 / 12.3 us, r06 sweep)
  if (a->kernel == 1 && nsteps <= 30 && tiles < 384) return true;
  return tiles < 384 && (tiles_s >= 384 || (tiles_s >= 256 && nsteps <= 48));
}

// The 192 x 320 tile (CF 4) for a plain conv / projection whose 192-row grid is one or two whole waves
// of 256 where the others end part-filled or run 3+ tiles per CU (profiles/r06_k10_plan_sweep.jsonl,
// the 3-frame clip: 64x64 3x3 N 320 K 320 / 640 / 960 x 9: 85.0 / 156.4 / 224.9 -> 73.1 / 132.5 /
// 193.6 us; the Upsample3D convs 64x64 N 640 296.2 -> 270.7, 32x32 N 1280 301.3 -> 266.3;
// r06_k10_plan_linear.jsonl: M 49152 N 320 K 640 / 960 / 1280 30.7 / 40.3 / 59.0 -> 26.0 / 33.2 / 40.2)
static bool mid_tile(const vp2p_conv_args* a, int64_t M) {
  if (a->epilogue != VP2P_CONV_EPI_NONE || a->cout % 320) return false;
  const int64_t tiles = (M + 191) / 192 * (a->cout / 320);
  return tiles <= 512 && wave_fill(tiles, 256) >= 0.95;
}

// K-split for this shape: 1 unless the grid would leave most CUs idle (the 8x8-latent convs)
static int pick_ksplit(const vp2p_conv_args* a) {
  if (a->epilogue != VP2P_CONV_EPI_NONE) return 1;
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  if (short_tile(a, M)) return 1;
  const int64_t tiles = (M + GBM - 1) / GBM * (a->cout / BN);
  const int nsteps = a->kernel * a->kernel * (a->cin / BK);
  if (tiles >= 384) return 1;
  // at most 8 slices, 16 where 8 would leave half the CUs without a workgroup (<= 16 tiles: the
  // 8x8-latent convs of a 1-frame clip; profiles/r04_k10_ksplit16.jsonl: M 256 K 2560*9 N 1280
  // 46.1 -> 35.0 us, K 1280*9 29.1 -> 25.4 us; 16 slices of the 32-tile grids measured slower)
  int kmax = tiles <= 16 ? 16 : 8;
  if (nsteps / 8 < kmax) kmax = nsteps / 8;                      // keep >= 8 steps per slice
  if (kmax < 2) return 1;
  int k0 = (int)((512 + tiles - 1) / tiles);
  if (k0 > kmax) k0 = kmax;
  // of k0 - 1, k0, k0 + 1 the one whose grid best fills its last wave of 512 (ties: more slices):
  // 192 tiles take 4 slices (768 = 1.5 waves), not 3 (576: a 64-workgroup second wave), measured
  // 101.2 / 135.9 / 171.6 vs 117.0 / 160.9 / 206.4 us (profiles/r06_k10_plan_sweep.jsonl)
  int k = k0;
  double best = -1.0;
  for (int c = k0 - 1; c <= k0 + 1; ++c) {
    if (c < 2 || c > kmax) continue;
    const double f = wave_fill(tiles * c, 512);
    if (f >= best) { best = f; k = c; }
  }
  return k;
}

// K-split on the 192 x 320 tile where its slices make exactly one wave of 256 workgroups (>= 32 K-steps
// a slice) in the small-M regime (< 384 128 x 160 tiles): the 3-frame clip's 16x16 3x3 convs, M 3072
// N 1280, 4 slices of 64 tiles -- K 1280 / 1920 / 2560 x 9 98.7 / 132.1 / 170.1 -> 91.9 / 122.9 / 154.2 us,
// and the Upsample3D conv there (otherwise the one-pass short tile) 113.8 -> 98.0
// (profiles/r06_k10_plan_split4.jsonl)
static int mid_split(const vp2p_conv_args* a, int64_t M) {
  if (a->kernel != 3 || a->epilogue != VP2P_CONV_EPI_NONE || a->cout % 320) return 0;
  if ((M + GBM - 1) / GBM * (a->cout / BN) >= 384) return 0;
  const int64_t tiles = (M + 191) / 192 * (a->cout / 320);
  const int nsteps = a->kernel * a->kernel * (a->cin / BK);
  for (int k = 2; k <= 8; ++k)
    if (tiles * k == 256 && nsteps / k >= 32) return k;
  return 0;
}

// The launch plan of a shape: tile configuration cf and K-split k (1: one pass).
struct Plan {
  int cf, k;
};

static bool plan_valid(const vp2p_conv_args* a, int cf, int k) {
  if (cf < 0 || cf > 4 || k < 1 || k > 16) return false;
  if ((cf == 2 || cf == 4) && a->cout % 320) return false;
  if (cf == 4 && a->epilogue != VP2P_CONV_EPI_NONE) return false;
  if (k > 1 && (a->epilogue != VP2P_CONV_EPI_NONE || (cf != 0 && cf != 3 && cf != 4))) return false;
  return a->kernel * a->kernel * (a->cin / BK) >= k;
}

// VP2P_K10_PLAN="CF,K" (tools/k10_plan_sweep.py: A/B only) forces both wherever they are valid for the
// shape; read on every call, so a sweep can change it between launches
static Plan plan_of(const vp2p_conv_args* a) {
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  Plan p{0, pick_ksplit(a)};
  if (const int km = mid_split(a, M)) p = Plan{4, km};
  else if (p.k == 1) p.cf = short_tile(a, M) ? 3 : mid_tile(a, M) ? 4 : pick_tile(a, M);
  if (const char* e = getenv("VP2P_K10_PLAN")) {
    int cf = -1, k = 0;
    if (sscanf(e, "%d,%d", &cf, &k) == 2 && plan_valid(a, cf, k)) p = Plan{cf, k};
  }
  return p;
}

static void tile_dims(int cf, int* tbm, int* tbn, int* nt) {
  switch (cf) {
    case 1: *tbm = GCfg<1>::TBM; *tbn = GCfg<1>::TBN; *nt = GCfg<1>::NT; break;
    case 2: *tbm = GCfg<2>::TBM; *tbn = GCfg<2>::TBN; *nt = GCfg<2>::NT; break;
    case 3: *tbm = GCfg<3>::TBM; *tbn = GCfg<3>::TBN; *nt = GCfg<3>::NT; break;
    case 4: *tbm = GCfg<4>::TBM; *tbn = GCfg<4>::TBN; *nt = GCfg<4>::NT; break;
    default: *tbm = GCfg<0>::TBM; *tbn = GCfg<0>::TBN; *nt = GCfg<0>::NT; break;
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
  // an output scale only on the plain epilogue without a residual (the scaled projection)
  if (a->alpha != 0.f && a->alpha != 1.f && (a->residual || a->epilogue != VP2P_CONV_EPI_NONE)) return 0;
  if (!(a->alpha == a->alpha) || a->alpha > 3.0e38f || a->alpha < -3.0e38f) return 0;   // NaN / inf
  if (a->upsample != 0 && (a->upsample != 1 || a->stride != 1 || (a->in_h & 1) || (a->in_w & 1))) return 0;
  if (a->img_add && (a->residual || a->epilogue != VP2P_CONV_EPI_NONE)) return 0;
  if (a->x2 || a->cin2) {   // two-source input: 1x1 convs on the buffer-offset form only
    if (!a->x2 || a->cin2 <= 0 || a->cin2 >= a->cin || a->cin2 % conv::BK || a->kernel != 1 || a->stride != 1 ||
        a->upsample || a->epilogue != VP2P_CONV_EPI_NONE)
      return 0;
    if ((int64_t)a->batch * a->in_h * a->in_w * a->cin * 2 >= ((int64_t)1 << 31)) return 0;
  }
  return 1;
}

extern "C" int32_t vp2p_conv2d_gn_parts(const vp2p_conv_args* a) {
  if (!a || !vp2p_conv2d_supported(a)) return 0;
  if (a->epilogue != VP2P_CONV_EPI_NONE || (a->alpha != 0.f && a->alpha != 1.f)) return 0;
  const conv::Plan pl = conv::plan_of(a);
  if (pl.k > 1) return 0;                                       // statistics in the one-pass epilogue only
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  if (a->gn_groups <= 0 || a->cout % a->gn_groups || a->gn_rows <= 0 || M % a->gn_rows) return 0;
  const int cg = a->cout / a->gn_groups;
  int tbm, tbn, nt;
  conv::tile_dims(pl.cf, &tbm, &tbn, &nt);
  if (cg % 2 || tbn % cg || a->gn_rows % tbm) return 0;
  const int gt = tbn / cg;
  if (nt % gt) return 0;
  const int tpg = nt / gt;
  if (tpg > 64 || (tpg & (tpg - 1)) || tpg < cg / 2) return 0;   // one wave per group, >= one row of pairs
  return a->gn_rows / tbm;
}

extern "C" int vp2p_conv2d_plan(const vp2p_conv_args* a, int32_t* tile, int32_t* ksplit) {
  if (!a || !tile || !ksplit) return VP2P_E_ARG;
  if (!vp2p_conv2d_supported(a)) return VP2P_E_SHAPE;
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  if (conv::skinny_kind(a, M)) {
    *tile = 5;
    *ksplit = 1;
    return VP2P_OK;
  }
  const conv::Plan pl = conv::plan_of(a);
  *tile = pl.cf;
  *ksplit = pl.k;
  return VP2P_OK;
}

extern "C" int64_t vp2p_conv2d_workspace_bytes(const vp2p_conv_args* a) {
  if (!a || !vp2p_conv2d_supported(a)) return 0;
  const int k = conv::plan_of(a).k;
  return k > 1 ? (int64_t)k * a->batch * a->out_h * a->out_w * a->cout * 4 : 0;
}

extern "C" int vp2p_conv2d_fwd(const vp2p_conv_args* a, void* stream) {
  if (!a || !a->x || !a->w || !a->y) return VP2P_E_ARG;
  if (a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (!vp2p_conv2d_supported(a)) return VP2P_E_SHAPE;
  for (const void* p : {a->x, a->w, static_cast<const void*>(a->y), a->residual,
                        static_cast<const void*>(a->workspace), a->x2, a->img_add})
    if (reinterpret_cast<uintptr_t>(p) & 15) return VP2P_E_ARG;
  if (a->gn_partials && vp2p_conv2d_gn_parts(a) <= 0) return VP2P_E_SHAPE;
  const int64_t M = (int64_t)a->batch * a->out_h * a->out_w;
  if (M * a->cout > ((int64_t)1 << 40)) return VP2P_E_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  conv::Plan pl = conv::plan_of(a);
  if (pl.k > 1 && !a->workspace) {                      // no workspace given: one pass
    pl.k = 1;
    pl.cf = conv::short_tile(a, M) ? 3 : conv::mid_tile(a, M) ? 4 : conv::pick_tile(a, M);
  }
  const int k = pl.k;
  int tbm, tbn, nt_;
  conv::tile_dims(pl.cf, &tbm, &tbn, &nt_);
  const int64_t tiles = (M + tbm - 1) / tbm * (a->cout / tbn);
  // addressing: 32-bit buffer offsets when the stored input is below 2^31 bytes (the upsampling
  // form for the one-pass 3x3 kernel), 64-bit pointers otherwise
  const int64_t in_bytes = (int64_t)a->batch * (a->in_h >> a->upsample) * (a->in_w >> a->upsample) * a->cin * 2;
  const int fast = in_bytes >= ((int64_t)1 << 31) ? 0
                   : !a->upsample ? 1
                   : (a->kernel == 3 && k == 1 && a->epilogue == VP2P_CONV_EPI_NONE) ? 2 : 0;
  if (tiles * k > 0x7fffffff) return VP2P_E_SHAPE;
  const dim3 grid((unsigned)(tiles * k));
  int rc;
  if (const int sk = conv::skinny_kind(a, M); sk) {
    // the persistent grid is sized by the CU count of the device this launch runs on (cached per
    // device id: a process may drive several devices)
    static int n_cu_of[64] = {};
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    if (dev < 64) n_cu = n_cu_of[dev];
    if (!n_cu) {
      if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
        n_cu = 256;
      if (dev < 64) n_cu_of[dev] = n_cu;
    }
    if (a->epilogue == VP2P_CONV_EPI_GEGLU) rc = conv::launch_k320<320, 32, false, 1>(*a, s, n_cu);
    else if (a->residual) rc = conv::launch_k320<320, 32, true, 0>(*a, s, n_cu);
    else rc = conv::launch_k320<320, 32, false, 0>(*a, s, n_cu);
  } else if (k > 1) {
    vp2p_conv_args b = *a;
    b.ksplit = k;
    if (pl.cf == 3)
      rc = a->kernel == 3 ? conv::launch_g<3, 2, 3>(b, grid, fast, s) : conv::launch_g<1, 2, 3>(b, grid, fast, s);
    else if (pl.cf == 4)
      rc = a->kernel == 3 ? conv::launch_g<3, 2, 4>(b, grid, fast, s) : conv::launch_g<1, 2, 4>(b, grid, fast, s);
    else
      rc = a->kernel == 3 ? conv::launch_g<3, 2>(b, grid, fast, s) : conv::launch_g<1, 2>(b, grid, fast, s);
    if (rc != VP2P_OK) return rc;
    const int64_t n = M * (a->cout / 8);
    hipLaunchKernelGGL(conv::conv_splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, b);
  } else if (pl.cf == 3) {
    if (a->epilogue == VP2P_CONV_EPI_GEGLU) rc = conv::launch_g<1, 1, 3>(*a, grid, fast, s);
    else rc = a->kernel == 3 ? conv::launch_g<3, 0, 3>(*a, grid, fast, s) : conv::launch_g<1, 0, 3>(*a, grid, fast, s);
  } else if (pl.cf == 1) {
    if (a->epilogue == VP2P_CONV_EPI_GEGLU) rc = conv::launch_g<1, 1, 1>(*a, grid, fast, s);
    else rc = a->kernel == 3 ? conv::launch_g<3, 0, 1>(*a, grid, fast, s) : conv::launch_g<1, 0, 1>(*a, grid, fast, s);
  } else if (pl.cf == 2) {
    if (a->epilogue == VP2P_CONV_EPI_GEGLU) rc = conv::launch_g<1, 1, 2>(*a, grid, fast, s);
    else rc = a->kernel == 3 ? conv::launch_g<3, 0, 2>(*a, grid, fast, s) : conv::launch_g<1, 0, 2>(*a, grid, fast, s);
  } else if (pl.cf == 4) {     // plain epilogue only (plan_valid)
    rc = a->kernel == 3 ? conv::launch_g<3, 0, 4>(*a, grid, fast, s) : conv::launch_g<1, 0, 4>(*a, grid, fast, s);
  } else if (a->epilogue == VP2P_CONV_EPI_GEGLU) {
    rc = conv::launch_g<1, 1>(*a, grid, fast, s);
  } else {
    rc = a->kernel == 3 ? conv::launch_g<3, 0>(*a, grid, fast, s) : conv::launch_g<1, 0>(*a, grid, fast, s);
  }
  if (rc != VP2P_OK) return rc;
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}
