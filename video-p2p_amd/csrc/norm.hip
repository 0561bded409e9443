// K7 (5-D GroupNorm + channel add + SiLU), K8 (LayerNorm), K9 (GEGLU gate): the HBM-bound
// normalisation / activation work of the UNet3D around the attention kernels.
//
// All three read channels-last activations in 16-byte vectors of 8 channels.  A thread owns one
// 8-channel vector of a row and walks rows, so per-channel parameters (affine, fused scale/shift)
// stay in registers and every global access is a full, coalesced 16-byte load/store.
//
// GroupNorm statistics span (c/G, f, h, w) of one batch element (tuneavideo resnet.py:142,158 runs
// nn.GroupNorm on the 5-D tensor).  At B=4, f=8, 64x64, C=320 one group is 327,680 elements, so the
// reduction is split over ~1000 row chunks per launch: gn_stats_kernel writes one
// (count, mean, M2) partial per (chunk, group) from shifted per-thread sums, gn_apply_kernel merges
// all partials of its batch element with Chan's formula (parallel over threads, then one merge per
// group) and applies y = x * a_c + b_c with a_c = rstd_g * w_c, b_c = bias_c - mean_g * a_c.
// Traffic: x read twice (the second read is usually an Infinity-Cache hit), y written once.
#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

template <typename T> struct V8;
template <> struct V8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[8]) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)r[j];
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j];
    *reinterpret_cast<bf16x8*>(p) = r;
  }
  static __device__ __forceinline__ float round(float x) { return (float)(bf16)x; }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    f32x4 a, b;
#pragma unroll
    for (int j = 0; j < 4; ++j) { a[j] = v[j]; b[j] = v[4 + j]; }
    reinterpret_cast<f32x4*>(p)[0] = a;
    reinterpret_cast<f32x4*>(p)[1] = b;
  }
  static __device__ __forceinline__ float round(float x) { return x; }
};

template <typename T> __device__ __forceinline__ float ld1(const void* p, int i) {
  return (float)static_cast<const T*>(p)[i];
}

struct Welford {
  float n, mean, m2;
};

__device__ __forceinline__ Welford wmerge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (b.n == 0.f) return a;
  if (a.n == 0.f) return b;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  return {n, a.mean + d * fb, a.m2 + b.m2 + d * d * a.n * fb};
}

// ------------------------------------------------------------------------------------------------
// GroupNorm geometry (host and device agree on it): block = nvec * R threads, thread t owns channel
// vector t % nvec of rows r = t / nvec, r + R, ...; a chunk is `chunk` consecutive rows of one
// batch element (frames * rows rows in total).
// ------------------------------------------------------------------------------------------------
struct GnGeom {
  int nvec, R, threads, chunk, parts, cg;
  int64_t L;
};

static bool gn_geom(const vp2p_group_norm_args* a, GnGeom* g) {
  if (!a || a->batch <= 0 || a->frames <= 0 || a->rows <= 0 || a->channels <= 0 || a->groups <= 0)
    return false;
  if (a->channels % 8 || a->channels % a->groups || a->groups > 64 || a->channels > 4096) return false;
  g->nvec = a->channels / 8;
  g->R = a->channels / 8 >= 512 ? 1 : 512 / (a->channels / 8);
  g->threads = g->nvec * g->R;
  if (g->threads > 512) return false;
  g->cg = a->channels / a->groups;
  g->L = (int64_t)a->frames * a->rows;
  if (g->L >= ((int64_t)1 << 31)) return false;
  // ~1024 blocks per launch, 8..16 rows per thread (2..4 rounds of kUnroll loads in flight).  The
  // floor of 8 keeps the partial count (which every apply block merges) small at the 8x8 / 16x16
  // latents (171 -> 22 partials per group at 8x8x1280).
  const int64_t all = g->L * a->batch;
  int64_t rpt = (all + (int64_t)g->R * 1024 - 1) / ((int64_t)g->R * 1024);
  if (rpt < 8) rpt = 8;
  if (rpt > 16) rpt = 16;
  const int64_t chunk = rpt * g->R;
  g->chunk = (int)chunk;
  g->parts = (int)((g->L + chunk - 1) / chunk);
  return true;
}

constexpr int kUnroll = 4;

// This thread's input column (8-channel vector v of batch element b) and its row stride: x, or x2
// for the channels of a two-source input's second part
template <typename T>
__device__ __forceinline__ const T* gn_src(const vp2p_group_norm_args& a, const GnGeom& g, int b, int v, int& stride) {
  const int c1 = a.channels - a.channels2;
  if (a.x2 && v * 8 >= c1) {
    stride = a.channels2;
    return static_cast<const T*>(a.x2) + (int64_t)b * g.L * a.channels2 + (v * 8 - c1);
  }
  stride = c1;
  return static_cast<const T*>(a.x) + (int64_t)b * g.L * c1 + v * 8;
}

// x (+ add of the row's sample) of one 8-channel vector, rounded to T like torch's h + temb;
// x points at the thread's column, xs is its row stride
template <typename T, bool ADD>
__device__ __forceinline__ void load_row(const vp2p_group_norm_args& a, const T* x, int xs, int b, int64_t row,
                                         int v, float (&val)[8]) {
  V8<T>::load(x + row * xs, val);
  if (ADD) {
    float ad[8];
    const int fr = (int)((uint32_t)row / (uint32_t)a.rows);     // L = frames * rows < 2^31 (gn_geom)
    V8<T>::load(static_cast<const T*>(a.add) + ((int64_t)b * a.frames + fr) * a.channels + v * 8, ad);
#pragma unroll
    for (int j = 0; j < 8; ++j) val[j] = V8<T>::round(val[j] + ad[j]);
  }
}

template <typename T, bool ADD>
__global__ __launch_bounds__(512) void gn_stats_kernel(const vp2p_group_norm_args a, const GnGeom g) {
  extern __shared__ float sm[];
  const int C = a.channels, G = a.groups, R = g.R, nvec = g.nvec, cg = g.cg;
  float* s_mean = sm;                       // [R][C]
  float* s_m2 = sm + R * C;                 // [R][C]
  float* s_cnt = sm + 2 * R * C;            // [R]
  float* s_w = s_cnt + R;                   // [3][threads] second-stage partials
  const int b = blockIdx.y, part = blockIdx.x, tid = threadIdx.x;
  const int v = tid % nvec, r = tid / nvec;
  const int64_t row0 = (int64_t)part * g.chunk;
  const int64_t row1 = row0 + g.chunk < g.L ? row0 + g.chunk : g.L;
  int xs;
  const T* x = gn_src<T>(a, g, b, v, xs);
  float K[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { K[j] = 0.f; s1[j] = 0.f; s2[j] = 0.f; }
  int n = 0;
  int64_t row = row0 + r;
  if (row < row1) load_row<T, ADD>(a, x, xs, b, row, v, K);     // shift: the thread's first value
  // kUnroll rows in flight per thread: all loads issued before any is consumed
  for (; row + (kUnroll - 1) * R < row1; row += kUnroll * R) {
    float val[kUnroll][8];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) load_row<T, ADD>(a, x, xs, b, row + u * R, v, val[u]);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = val[u][j] - K[j];
        s1[j] += d;
        s2[j] = fmaf(d, d, s2[j]);
      }
    n += kUnroll;
  }
  for (; row < row1; row += R) {
    float val[8];
    load_row<T, ADD>(a, x, xs, b, row, v, val);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = val[j] - K[j];
      s1[j] += d;
      s2[j] = fmaf(d, d, s2[j]);
    }
    ++n;
  }
  const float fn = (float)n, inv = n ? 1.f / fn : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_mean[r * C + v * 8 + j] = K[j] + s1[j] * inv;
    s_m2[r * C + v * 8 + j] = fmaxf(s2[j] - s1[j] * s1[j] * inv, 0.f);
  }
  if (v == 0) s_cnt[r] = fn;
  __syncthreads();
  // stage 2: tpg threads per group merge the group's R * cg (row-lane, channel) entries
  const int tpg = g.threads / G;
  const int gi = tid / tpg, k = tid - gi * tpg;
  Welford w = {0.f, 0.f, 0.f};
  if (gi < G) {
    for (int e = k; e < R * cg; e += tpg) {
      const int rr = e / cg, c = gi * cg + (e - rr * cg);
      w = wmerge(w, {s_cnt[rr], s_mean[rr * C + c], s_m2[rr * C + c]});
    }
  }
  s_w[tid] = w.n;
  s_w[g.threads + tid] = w.mean;
  s_w[2 * g.threads + tid] = w.m2;
  __syncthreads();
  if (tid < G) {
    Welford t = {0.f, 0.f, 0.f};
    for (int e = 0; e < tpg; ++e) {
      const int i = tid * tpg + e;
      t = wmerge(t, {s_w[i], s_w[g.threads + i], s_w[2 * g.threads + i]});
    }
    float* o = a.partials + (((int64_t)b * g.parts + part) * G + tid) * 3;
    o[0] = t.n;
    o[1] = t.mean;
    o[2] = t.m2;
  }
}

// Finalize: one 256-thread block per (group, batch element) merges that group's nsets x parts
// partials -- one load per thread in flight, then a fixed-order tree in LDS -- into {mean, rstd}
// (TRIPLE: into the merged (count, mean, M2), the frame-sharded exchange).
template <bool TRIPLE = false>
__global__ __launch_bounds__(256) void gn_finalize_kernel(const vp2p_group_norm_args a, const GnGeom g,
                                                          const float* __restrict__ partials, int nsets,
                                                          float* __restrict__ stats) {
  __shared__ float s_n[256], s_mean[256], s_m2[256];
  const int G = a.groups, gi = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int total = nsets * g.parts;
  Welford w = {0.f, 0.f, 0.f};
  for (int e = tid; e < total; e += 256) {
    const int set = e / g.parts, p = e - set * g.parts;
    const float* q = partials + ((((int64_t)set * a.batch + b) * g.parts + p) * G + gi) * 3;
    w = wmerge(w, {q[0], q[1], q[2]});
  }
  s_n[tid] = w.n;
  s_mean[tid] = w.mean;
  s_m2[tid] = w.m2;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
      const Welford t = wmerge({s_n[tid], s_mean[tid], s_m2[tid]}, {s_n[tid + st], s_mean[tid + st], s_m2[tid + st]});
      s_n[tid] = t.n;
      s_mean[tid] = t.mean;
      s_m2[tid] = t.m2;
    }
    __syncthreads();
  }
  if (tid == 0) {
    if constexpr (TRIPLE) {
      float* o = stats + ((int64_t)b * G + gi) * 3;
      o[0] = s_n[0];
      o[1] = s_mean[0];
      o[2] = s_m2[0];
    } else {
      stats[((int64_t)b * G + gi) * 2] = s_mean[0];
      stats[((int64_t)b * G + gi) * 2 + 1] = rsqrtf(s_m2[0] / s_n[0] + a.eps);
    }
  }
}

// FIN: statistics already finalized (`stats`, (batch, groups, 2)); otherwise every block merges all
// partials itself (the ABI's vp2p_group_norm_apply)
template <typename T, bool ADD, bool SILU, bool FIN = false>
__global__ __launch_bounds__(512) void gn_apply_kernel(const vp2p_group_norm_args a, const GnGeom g,
                                                        const float* __restrict__ partials, int nsets, int mparts) {
  __shared__ float s_w[FIN ? 1 : 3 * 512];
  __shared__ float s_mean[64], s_rstd[64];
  const int C = a.channels, G = a.groups, R = g.R, nvec = g.nvec, cg = g.cg;
  const int b = blockIdx.y, part = blockIdx.x, tid = threadIdx.x;
  if constexpr (FIN) {
    if (tid < G) {
      s_mean[tid] = partials[((int64_t)b * G + tid) * 2];
      s_rstd[tid] = partials[((int64_t)b * G + tid) * 2 + 1];
    }
  } else {
    const int tpg = g.threads / G;
    const int gi = tid / tpg, k = tid - gi * tpg;
    Welford w = {0.f, 0.f, 0.f};
    if (gi < G) {
      const int P = mparts > 0 ? mparts : g.parts;     // partials per (set, sample): _stats' or a producer's
      const int total = nsets * P;
      for (int e = k; e < total; e += tpg) {
        const int set = e / P, p = e - set * P;
        const float* q = partials + ((((int64_t)set * a.batch + b) * P + p) * G + gi) * 3;
        w = wmerge(w, {q[0], q[1], q[2]});
      }
    }
    s_w[tid] = w.n;
    s_w[512 + tid] = w.mean;
    s_w[1024 + tid] = w.m2;
    __syncthreads();
    if (tid < G) {
      Welford t = {0.f, 0.f, 0.f};
      for (int e = 0; e < tpg; ++e) {
        const int i = tid * tpg + e;
        t = wmerge(t, {s_w[i], s_w[512 + i], s_w[1024 + i]});
      }
      s_mean[tid] = t.mean;
      s_rstd[tid] = rsqrtf(t.m2 / t.n + a.eps);
    }
  }
  __syncthreads();
  const int v = tid % nvec, r = tid / nvec;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = v * 8 + j, q = c / cg;
    const float wt = a.weight ? ld1<T>(a.weight, c) : 1.f;
    const float bs = a.bias ? ld1<T>(a.bias, c) : 0.f;
    sc[j] = s_rstd[q] * wt;
    sh[j] = fmaf(-s_mean[q], sc[j], bs);
  }
  const int64_t row0 = (int64_t)part * g.chunk;
  const int64_t row1 = row0 + g.chunk < g.L ? row0 + g.chunk : g.L;
  const int64_t base = (int64_t)b * g.L * C + v * 8;
  int xs;
  const T* x = gn_src<T>(a, g, b, v, xs);
  T* y = static_cast<T*>(a.y) + base;
  auto finish = [&](float (&val)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = fmaf(val[j], sc[j], sh[j]);
      if (SILU) t = t * __builtin_amdgcn_rcpf(1.f + __expf(-t));   // v_rcp, not the IEEE divide sequence
      val[j] = t;
    }
  };
  int64_t row = row0 + r;
  for (; row + (kUnroll - 1) * R < row1; row += kUnroll * R) {
    float val[kUnroll][8];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) load_row<T, ADD>(a, x, xs, b, row + u * R, v, val[u]);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      finish(val[u]);
      V8<T>::store(y + (row + u * R) * C, val[u]);
    }
  }
  for (; row < row1; row += R) {
    float val[8];
    load_row<T, ADD>(a, x, xs, b, row, v, val);
    finish(val);
    V8<T>::store(y + row * C, val);
  }
}

static int gn_check(const vp2p_group_norm_args* a, GnGeom* g) {
  if (!a || !a->x || !a->y) return VP2P_E_ARG;
  if (a->x2 ? (a->channels2 <= 0 || a->channels2 >= a->channels || a->channels2 % 8) : a->channels2 != 0)
    return VP2P_E_ARG;
  if (a->dtype != VP2P_F32 && a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (!gn_geom(a, g)) return VP2P_E_SHAPE;
  return VP2P_OK;
}

template <typename T>
static void gn_stats_launch(const vp2p_group_norm_args& a, const GnGeom& g, hipStream_t s) {
  const dim3 grid(g.parts, a.batch);
  const size_t lds = (size_t)(2 * g.R * a.channels + g.R + 3 * g.threads) * sizeof(float);
  if (a.add)
    hipLaunchKernelGGL((gn_stats_kernel<T, true>), grid, dim3(g.threads), lds, s, a, g);
  else
    hipLaunchKernelGGL((gn_stats_kernel<T, false>), grid, dim3(g.threads), lds, s, a, g);
}

// parts = the partial sets (FIN = false) or the finalized (batch, groups, 2) statistics (FIN = true)
template <typename T, bool FIN = false>
static void gn_apply_launch(const vp2p_group_norm_args& a, const GnGeom& g, const float* parts, int nsets,
                            hipStream_t s, int mparts = 0) {
  const dim3 grid(g.parts, a.batch), block(g.threads);
  const bool add = a.add != nullptr, silu = a.silu != 0;
  if (add && silu) hipLaunchKernelGGL((gn_apply_kernel<T, true, true, FIN>), grid, block, 0, s, a, g, parts, nsets, mparts);
  else if (add) hipLaunchKernelGGL((gn_apply_kernel<T, true, false, FIN>), grid, block, 0, s, a, g, parts, nsets, mparts);
  else if (silu) hipLaunchKernelGGL((gn_apply_kernel<T, false, true, FIN>), grid, block, 0, s, a, g, parts, nsets, mparts);
  else hipLaunchKernelGGL((gn_apply_kernel<T, false, false, FIN>), grid, block, 0, s, a, g, parts, nsets, mparts);
}

// ------------------------------------------------------------------------------------------------
// K8 LayerNorm: one wave per row, NV 8-channel vectors per lane held in registers (exact two-pass
// mean / variance), 4 rows per 256-thread block.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}

// ADD: the block's residual add fused in front (BasicTransformerBlock, attention.py:247-268:
// 'hidden_states = attn(norm(hidden_states)) + hidden_states'): x_new = x + res, rounded to T and
// written to sum (as the reference stores the sum), then normalised.
template <typename T, int NV, int RPW, bool ADD = false>
__global__ __launch_bounds__(256) void ln_kernel(const vp2p_layer_norm_args a, const T* res = nullptr,
                                                 T* sum = nullptr) {
  const int lane = lane_id();
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (row0 >= a.rows) return;
  const int C = a.channels, nvec = C / 8;
  float v[RPW][NV][8];
  // every load of the wave's RPW rows is issued before the first reduction
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = row0 + rr < a.rows ? row0 + rr : a.rows - 1;
    const T* x = static_cast<const T*>(a.x) + row * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nvec) {
        V8<T>::load(x + vi * 8, v[rr][i]);
        if constexpr (ADD) {
          float rv[8];
          V8<T>::load(res + row * C + vi * 8, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[rr][i][j] = (float)(T)(v[rr][i][j] + rv[j]);
          if (row0 + rr < a.rows) V8<T>::store(sum + row * C + vi * 8, v[rr][i]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[rr][i][j] = 0.f;
      }
    }
  }
  float w[NV][8], bs[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < 8; ++j) { w[i][j] = 1.f; bs[i][j] = 0.f; }
    if (vi < nvec) {
      if (a.weight) V8<T>::load(static_cast<const T*>(a.weight) + vi * 8, w[i]);
      if (a.bias) V8<T>::load(static_cast<const T*>(a.bias) + vi * 8, bs[i]);
    }
  }
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int64_t row = row0 + rr;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[rr][i][j];
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (lane + 64 * i < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[rr][i][j] -= mean;
          q = fmaf(v[rr][i][j], v[rr][i][j], q);
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / (float)C + a.eps);
    if (row >= a.rows) continue;
    T* y = static_cast<T*>(a.y) + row * C;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + 64 * i;
      if (vi < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[rr][i][j] = v[rr][i][j] * rstd * w[i][j] + bs[i][j];
        V8<T>::store(y + vi * 8, v[rr][i]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// K9 GEGLU gate: y = a * gelu(g) with a = x[:, :inner], g = x[:, inner:]; gelu rounded to the
// storage type before the product, as torch's eager F.gelu followed by a * (...) does.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void geglu_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t rows,
                                                    int inner) {
#pragma clang fp contract(off)
  const int nv = inner / 8;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * nv) return;
  const int64_t row = e / nv;
  const int col = (int)(e - row * nv) * 8;
  const T* xr = x + row * 2 * inner;
  float av[8], gv[8];
  V8<T>::load(xr + col, av);
  V8<T>::load(xr + inner + col, gv);
  constexpr float kAlpha = 0.70710678118654752440f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float ge = V8<T>::round(gv[j] * 0.5f * (1.f + erff(gv[j] * kAlpha)));
    av[j] = av[j] * ge;
  }
  V8<T>::store(y + row * inner + col, av);
}


// ================================================================================================
// Backward of K7-K9 (input gradients only: the null-text optimisation differentiates the UNet
// w.r.t. the unconditional embedding with every weight frozen, run_videop2p.py:580-612).
// ================================================================================================

// mean / rstd of every group of batch element b from the forward partials (all nsets merged)
__device__ __forceinline__ void gn_group_stats(const vp2p_group_norm_args& a, const GnGeom& g,
                                               const float* __restrict__ partials, int nsets, int b, float* s_w,
                                               float* s_mean, float* s_rstd, float* s_n) {
  const int G = a.groups, tid = threadIdx.x, tpg = g.threads / G;
  const int gi = tid / tpg, k = tid - gi * tpg;
  Welford w = {0.f, 0.f, 0.f};
  if (gi < G) {
    const int total = nsets * g.parts;
    for (int e = k; e < total; e += tpg) {
      const int set = e / g.parts, p = e - set * g.parts;
      const float* q = partials + ((((int64_t)set * a.batch + b) * g.parts + p) * G + gi) * 3;
      w = wmerge(w, {q[0], q[1], q[2]});
    }
  }
  s_w[tid] = w.n;
  s_w[512 + tid] = w.mean;
  s_w[1024 + tid] = w.m2;
  __syncthreads();
  if (tid < G) {
    Welford t = {0.f, 0.f, 0.f};
    for (int e = 0; e < tpg; ++e) {
      const int i = tid * tpg + e;
      t = wmerge(t, {s_w[i], s_w[512 + i], s_w[1024 + i]});
    }
    s_mean[tid] = t.mean;
    s_rstd[tid] = rsqrtf(t.m2 / t.n + a.eps);
    s_n[tid] = t.n;
  }
  __syncthreads();
}

// g = dL/d(normalised x) * weight, through the SiLU when it was fused: a = xhat*w + bias,
// silu'(a) = s(a) (1 + a (1 - s(a)))
template <bool SILU>
__device__ __forceinline__ float gn_grad(float dy, float xhat, float wt, float bs) {
  if (SILU) {
    const float av = fmaf(xhat, wt, bs);
    const float sg = 1.f / (1.f + __expf(-av));
    dy = dy * sg * (1.f + av * (1.f - sg));
  }
  return dy * wt;
}

// per (chunk, group): sum g and sum g * xhat -> bwd partials (batch, parts, groups, 2)
template <typename T, bool ADD, bool SILU>
__global__ __launch_bounds__(512) void gn_bwd_reduce_kernel(const vp2p_group_norm_args a, const GnGeom g,
                                                            const float* __restrict__ partials, int nsets,
                                                            const T* __restrict__ dy, float* __restrict__ bpart) {
  extern __shared__ float sm[];
  const int C = a.channels, G = a.groups, R = g.R, nvec = g.nvec, cg = g.cg;
  float* s_w = sm;                      // [3 * 512]
  float* s_mean = sm + 1536;            // [64]
  float* s_rstd = s_mean + 64;
  float* s_n = s_rstd + 64;
  float* s_a = s_n + 64;                // [R][C]
  float* s_b = s_a + R * C;             // [R][C]
  const int b = blockIdx.y, part = blockIdx.x, tid = threadIdx.x;
  gn_group_stats(a, g, partials, nsets, b, s_w, s_mean, s_rstd, s_n);
  const int v = tid % nvec, r = tid / nvec;
  float mu[8], rs[8], wt[8], bs[8], s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = v * 8 + j, q = c / cg;
    mu[j] = s_mean[q];
    rs[j] = s_rstd[q];
    wt[j] = a.weight ? ld1<T>(a.weight, c) : 1.f;
    bs[j] = a.bias ? ld1<T>(a.bias, c) : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
  const int64_t row0 = (int64_t)part * g.chunk;
  const int64_t row1 = row0 + g.chunk < g.L ? row0 + g.chunk : g.L;
  const int64_t base = (int64_t)b * g.L * C + v * 8;
  const T* x = static_cast<const T*>(a.x) + base;
  const int xs = C;
  for (int64_t row = row0 + r; row < row1; row += R) {
    float xv[8], dv[8];
    load_row<T, ADD>(a, x, xs, b, row, v, xv);
    V8<T>::load(dy + base + row * C, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mu[j]) * rs[j];
      const float gg = gn_grad<SILU>(dv[j], xh, wt[j], bs[j]);
      s1[j] += gg;
      s2[j] = fmaf(gg, xh, s2[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s_a[r * C + v * 8 + j] = s1[j];
    s_b[r * C + v * 8 + j] = s2[j];
  }
  __syncthreads();
  const int tpg = g.threads / G;
  const int gi = tid / tpg, k = tid - gi * tpg;
  float t1 = 0.f, t2 = 0.f;
  if (gi < G) {
    for (int e = k; e < R * cg; e += tpg) {
      const int rr = e / cg, c = gi * cg + (e - rr * cg);
      t1 += s_a[rr * C + c];
      t2 += s_b[rr * C + c];
    }
  }
  __syncthreads();
  s_w[tid] = t1;
  s_w[512 + tid] = t2;
  __syncthreads();
  if (tid < G) {
    float u1 = 0.f, u2 = 0.f;
    for (int e = 0; e < tpg; ++e) {
      u1 += s_w[tid * tpg + e];
      u2 += s_w[512 + tid * tpg + e];
    }
    float* o = bpart + (((int64_t)b * g.parts + part) * G + tid) * 2;
    o[0] = u1;
    o[1] = u2;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) per group
template <typename T, bool ADD, bool SILU>
__global__ __launch_bounds__(512) void gn_bwd_apply_kernel(const vp2p_group_norm_args a, const GnGeom g,
                                                           const float* __restrict__ partials, int nsets,
                                                           const T* __restrict__ dy, const float* __restrict__ bpart,
                                                           int bsets, T* __restrict__ dx) {
  __shared__ float s_w[3 * 512];
  __shared__ float s_mean[64], s_rstd[64], s_n[64], s_m1[64], s_m2[64];
  const int C = a.channels, G = a.groups, R = g.R, nvec = g.nvec, cg = g.cg;
  const int b = blockIdx.y, part = blockIdx.x, tid = threadIdx.x;
  gn_group_stats(a, g, partials, nsets, b, s_w, s_mean, s_rstd, s_n);
  {  // tpg threads per group sum a strided share of the (set, part) partials, then one add per group
    const int tpg = g.threads / G;
    const int gi = tid / tpg, k = tid - gi * tpg;
    float u1 = 0.f, u2 = 0.f;
    if (gi < G) {
      for (int e = k; e < bsets * g.parts; e += tpg) {
        const int set = e / g.parts, p = e - set * g.parts;
        const float* q = bpart + ((((int64_t)set * a.batch + b) * g.parts + p) * G + gi) * 2;
        u1 += q[0];
        u2 += q[1];
      }
    }
    s_w[tid] = u1;
    s_w[512 + tid] = u2;
    __syncthreads();
    if (tid < G) {
      float v1 = 0.f, v2 = 0.f;
      for (int e = 0; e < tpg; ++e) {
        v1 += s_w[tid * tpg + e];
        v2 += s_w[512 + tid * tpg + e];
      }
      s_m1[tid] = v1 / s_n[tid];
      s_m2[tid] = v2 / s_n[tid];
    }
    __syncthreads();
  }
  const int v = tid % nvec, r = tid / nvec;
  float mu[8], rs[8], wt[8], bs[8], m1[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = v * 8 + j, q = c / cg;
    mu[j] = s_mean[q];
    rs[j] = s_rstd[q];
    m1[j] = s_m1[q];
    m2[j] = s_m2[q];
    wt[j] = a.weight ? ld1<T>(a.weight, c) : 1.f;
    bs[j] = a.bias ? ld1<T>(a.bias, c) : 0.f;
  }
  const int64_t row0 = (int64_t)part * g.chunk;
  const int64_t row1 = row0 + g.chunk < g.L ? row0 + g.chunk : g.L;
  const int64_t base = (int64_t)b * g.L * C + v * 8;
  const T* x = static_cast<const T*>(a.x) + base;
  const int xs = C;
  for (int64_t row = row0 + r; row < row1; row += R) {
    float xv[8], dv[8];
    load_row<T, ADD>(a, x, xs, b, row, v, xv);
    V8<T>::load(dy + base + row * C, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xh = (xv[j] - mu[j]) * rs[j];
      const float gg = gn_grad<SILU>(dv[j], xh, wt[j], bs[j]);
      xv[j] = rs[j] * (gg - m1[j] - xh * m2[j]);
    }
    V8<T>::store(dx + base + row * C, xv);
  }
}

template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const vp2p_layer_norm_args a, const T* __restrict__ dy,
                                                     T* __restrict__ dx) {
  const int lane = lane_id();
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.rows) return;
  const int C = a.channels, nvec = C / 8;
  float xv[NV][8], gv[NV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = lane + 64 * i;
#pragma unroll
    for (int j = 0; j < 8; ++j) { xv[i][j] = 0.f; gv[i][j] = 0.f; }
    if (vi < nvec) {
      V8<T>::load(static_cast<const T*>(a.x) + row * C + vi * 8, xv[i]);
      V8<T>::load(dy + row * C + vi * 8, gv[i]);
      float w[8];
      if (a.weight) {
        V8<T>::load(static_cast<const T*>(a.weight) + vi * 8, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[i][j] *= w[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += xv[i][j];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xv[i][j] -= mean;
        q = fmaf(xv[i][j], xv[i][j], q);
      }
    }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + a.eps);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      xv[i][j] *= rstd;
      s1 += gv[i][j];
      s2 = fmaf(gv[i][j], xv[i][j], s2);
    }
  const float m1 = wave_sum(s1) / (float)C, m2 = wave_sum(s2) / (float)C;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int vi = lane + 64 * i;
    if (vi < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) xv[i][j] = rstd * (gv[i][j] - m1 - xv[i][j] * m2);
      V8<T>::store(dx + row * C + vi * 8, xv[i]);
    }
  }
}

// y = a * ge, ge = round(gelu(g)):  da = dy * ge,  dg = round(dy * a) * gelu'(g),
// gelu'(g) = Phi(g) + g * phi(g)  (torch's autograd of the eager a * F.gelu(g))
template <typename T>
__global__ __launch_bounds__(256) void geglu_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                        T* __restrict__ dx, int64_t rows, int inner) {
#pragma clang fp contract(off)
  const int nv = inner / 8;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * nv) return;
  const int64_t row = e / nv;
  const int col = (int)(e - row * nv) * 8;
  const T* xr = x + row * 2 * inner;
  float av[8], gv[8], dv[8];
  V8<T>::load(xr + col, av);
  V8<T>::load(xr + inner + col, gv);
  V8<T>::load(dy + row * inner + col, dv);
  constexpr float kAlpha = 0.70710678118654752440f;
  constexpr float kBeta = 0.39894228040143267794f;   // 1/sqrt(2 pi)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float cdf = 0.5f * (1.f + erff(gv[j] * kAlpha));
    const float ge = V8<T>::round(gv[j] * cdf);
    const float dge = V8<T>::round(dv[j] * av[j]);
    const float pdf = kBeta * __expf(-0.5f * gv[j] * gv[j]);
    av[j] = dv[j] * ge;
    gv[j] = dge * (cdf + gv[j] * pdf);
  }
  T* dr = dx + row * 2 * inner;
  V8<T>::store(dr + col, av);
  V8<T>::store(dr + inner + col, gv);
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int32_t vp2p_group_norm_parts(const vp2p_group_norm_args* a) {
  GnGeom g;
  const int rc = gn_check(a, &g);
  return rc == VP2P_OK ? g.parts : rc;
}

extern "C" int vp2p_group_norm_stats(const vp2p_group_norm_args* a, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!a->partials) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a->dtype == VP2P_BF16) gn_stats_launch<bf16>(*a, g, s);
  else gn_stats_launch<float>(*a, g, s);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_apply(const vp2p_group_norm_args* a, const float* partials, int32_t nsets,
                                     void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || nsets <= 0) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a->dtype == VP2P_BF16) gn_apply_launch<bf16>(*a, g, partials, nsets, s);
  else gn_apply_launch<float>(*a, g, partials, nsets, s);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_finalize(const vp2p_group_norm_args* a, const float* partials, int32_t nsets,
                                        float* stats, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || !stats || nsets <= 0) return VP2P_E_ARG;
  if ((int64_t)nsets * g.parts >= ((int64_t)1 << 31)) return VP2P_E_SHAPE;
  hipLaunchKernelGGL(gn_finalize_kernel<false>, dim3(a->groups, a->batch), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a, g, partials, nsets, stats);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_merge(const vp2p_group_norm_args* a, const float* partials, float* triples,
                                     void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || !triples) return VP2P_E_ARG;
  hipLaunchKernelGGL(gn_finalize_kernel<true>, dim3(a->groups, a->batch), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a, g, partials, 1, triples);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_apply_parts(const vp2p_group_norm_args* a, const float* partials, int32_t parts,
                                           void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || parts <= 0) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a->dtype == VP2P_BF16) gn_apply_launch<bf16>(*a, g, partials, 1, s, parts);
  else gn_apply_launch<float>(*a, g, partials, 1, s, parts);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_finalize_parts(const vp2p_group_norm_args* a, const float* partials, int32_t parts,
                                              float* stats, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || !stats || parts <= 0) return VP2P_E_ARG;
  g.parts = parts;
  hipLaunchKernelGGL(gn_finalize_kernel<false>, dim3(a->groups, a->batch), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a, g, partials, 1, stats);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_merge_parts(const vp2p_group_norm_args* a, const float* partials, int32_t parts,
                                           float* triples, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!partials || !triples || parts <= 0) return VP2P_E_ARG;
  g.parts = parts;
  hipLaunchKernelGGL(gn_finalize_kernel<true>, dim3(a->groups, a->batch), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a, g, partials, 1, triples);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_finalize_merged(const vp2p_group_norm_args* a, const float* triples, int32_t nsets,
                                               float* stats, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!triples || !stats || nsets <= 0) return VP2P_E_ARG;
  g.parts = 1;                                          // one merged triple per (set, batch, group)
  hipLaunchKernelGGL(gn_finalize_kernel<false>, dim3(a->groups, a->batch), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a, g, triples, nsets, stats);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_apply_stats(const vp2p_group_norm_args* a, const float* stats, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (!stats) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a->dtype == VP2P_BF16) gn_apply_launch<bf16, true>(*a, g, stats, 1, s);
  else gn_apply_launch<float, true>(*a, g, stats, 1, s);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_fwd(const vp2p_group_norm_args* a, void* stream) {
  int rc = vp2p_group_norm_stats(a, stream);
  if (rc != VP2P_OK) return rc;
  return vp2p_group_norm_apply(a, a->partials, 1, stream);
}

extern "C" int vp2p_add_layer_norm_fwd(const vp2p_layer_norm_args* a, const void* residual, void* sum,
                                       void* stream) {
  if (!a || !a->x || !a->y || !residual || !sum || a->rows < 0) return VP2P_E_ARG;
  if (a->dtype != VP2P_F32 && a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (a->channels <= 0 || a->channels % 8 || a->channels > 2048) return VP2P_E_SHAPE;
  if (a->rows == 0) return VP2P_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nv = (a->channels / 8 + 63) / 64;
  const int rpw = nv == 1 ? 4 : nv == 2 ? 2 : 1;
  const dim3 grid((unsigned)((a->rows + 4 * rpw - 1) / (4 * rpw))), block(256);
#define VP2P_ALN(T)                                                                                          \
  {                                                                                                          \
    const T* r = static_cast<const T*>(residual);                                                            \
    T* o = static_cast<T*>(sum);                                                                             \
    switch (nv) {                                                                                            \
      case 1: hipLaunchKernelGGL((ln_kernel<T, 1, 4, true>), grid, block, 0, s, *a, r, o); break;            \
      case 2: hipLaunchKernelGGL((ln_kernel<T, 2, 2, true>), grid, block, 0, s, *a, r, o); break;            \
      case 3: hipLaunchKernelGGL((ln_kernel<T, 3, 1, true>), grid, block, 0, s, *a, r, o); break;            \
      default: hipLaunchKernelGGL((ln_kernel<T, 4, 1, true>), grid, block, 0, s, *a, r, o); break;           \
    }                                                                                                        \
  }
  if (a->dtype == VP2P_BF16) VP2P_ALN(bf16) else VP2P_ALN(float)
#undef VP2P_ALN
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_layer_norm_fwd(const vp2p_layer_norm_args* a, void* stream) {
  if (!a || !a->x || !a->y || a->rows < 0) return VP2P_E_ARG;
  if (a->dtype != VP2P_F32 && a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (a->channels <= 0 || a->channels % 8 || a->channels > 2048) return VP2P_E_SHAPE;
  if (a->rows == 0) return VP2P_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nv = (a->channels / 8 + 63) / 64;
  const int rpw = nv == 1 ? 4 : nv == 2 ? 2 : 1;          // rows per wave: ~4 vector loads in flight per lane
  const dim3 grid((unsigned)((a->rows + 4 * rpw - 1) / (4 * rpw))), block(256);
#define VP2P_LN(T)                                                                           \
  switch (nv) {                                                                              \
    case 1: hipLaunchKernelGGL((ln_kernel<T, 1, 4>), grid, block, 0, s, *a); break;          \
    case 2: hipLaunchKernelGGL((ln_kernel<T, 2, 2>), grid, block, 0, s, *a); break;          \
    case 3: hipLaunchKernelGGL((ln_kernel<T, 3, 1>), grid, block, 0, s, *a); break;          \
    default: hipLaunchKernelGGL((ln_kernel<T, 4, 1>), grid, block, 0, s, *a); break;         \
  }
  if (a->dtype == VP2P_BF16) { VP2P_LN(bf16) } else { VP2P_LN(float) }
#undef VP2P_LN
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_geglu_fwd(const void* x, void* y, int64_t rows, int32_t inner, int32_t dtype, void* stream) {
  if (!x || !y || rows < 0 || inner <= 0) return VP2P_E_ARG;
  if (dtype != VP2P_F32 && dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (inner % 8) return VP2P_E_SHAPE;
  if (rows == 0) return VP2P_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = rows * (inner / 8);
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (dtype == VP2P_BF16)
    hipLaunchKernelGGL((geglu_kernel<bf16>), grid, block, 0, s, static_cast<const bf16*>(x), static_cast<bf16*>(y),
                       rows, inner);
  else
    hipLaunchKernelGGL((geglu_kernel<float>), grid, block, 0, s, static_cast<const float*>(x),
                       static_cast<float*>(y), rows, inner);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_bwd_reduce(const vp2p_group_norm_args* a, const float* partials, int32_t nsets,
                                          const void* dy, float* bwd_partials, void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (a->x2) return VP2P_E_ARG;                       // forward only
  if (!partials || nsets <= 0 || !dy || !bwd_partials) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(g.parts, a->batch), block(g.threads);
  const size_t lds = (size_t)(1536 + 192 + 2 * g.R * a->channels) * sizeof(float);
  const bool add = a->add != nullptr, silu = a->silu != 0;
#define VP2P_GNB(T)                                                                                          \
  {                                                                                                          \
    const T* d = static_cast<const T*>(dy);                                                                  \
    if (add && silu) hipLaunchKernelGGL((gn_bwd_reduce_kernel<T, true, true>), grid, block, lds, s, *a, g, partials, nsets, d, bwd_partials); \
    else if (add) hipLaunchKernelGGL((gn_bwd_reduce_kernel<T, true, false>), grid, block, lds, s, *a, g, partials, nsets, d, bwd_partials); \
    else if (silu) hipLaunchKernelGGL((gn_bwd_reduce_kernel<T, false, true>), grid, block, lds, s, *a, g, partials, nsets, d, bwd_partials); \
    else hipLaunchKernelGGL((gn_bwd_reduce_kernel<T, false, false>), grid, block, lds, s, *a, g, partials, nsets, d, bwd_partials); \
  }
  if (a->dtype == VP2P_BF16) VP2P_GNB(bf16) else VP2P_GNB(float)
#undef VP2P_GNB
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_group_norm_bwd_apply(const vp2p_group_norm_args* a, const float* partials, int32_t nsets,
                                         const void* dy, const float* bwd_partials, int32_t bsets, void* dx,
                                         void* stream) {
  GnGeom g;
  int rc = gn_check(a, &g);
  if (rc != VP2P_OK) return rc;
  if (a->x2) return VP2P_E_ARG;                       // forward only
  if (!partials || nsets <= 0 || !dy || !bwd_partials || bsets <= 0 || !dx) return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(g.parts, a->batch), block(g.threads);
  const bool add = a->add != nullptr, silu = a->silu != 0;
#define VP2P_GNA(T)                                                                                          \
  {                                                                                                          \
    const T* d = static_cast<const T*>(dy);                                                                  \
    T* o = static_cast<T*>(dx);                                                                              \
    if (add && silu) hipLaunchKernelGGL((gn_bwd_apply_kernel<T, true, true>), grid, block, 0, s, *a, g, partials, nsets, d, bwd_partials, bsets, o); \
    else if (add) hipLaunchKernelGGL((gn_bwd_apply_kernel<T, true, false>), grid, block, 0, s, *a, g, partials, nsets, d, bwd_partials, bsets, o); \
    else if (silu) hipLaunchKernelGGL((gn_bwd_apply_kernel<T, false, true>), grid, block, 0, s, *a, g, partials, nsets, d, bwd_partials, bsets, o); \
    else hipLaunchKernelGGL((gn_bwd_apply_kernel<T, false, false>), grid, block, 0, s, *a, g, partials, nsets, d, bwd_partials, bsets, o); \
  }
  if (a->dtype == VP2P_BF16) VP2P_GNA(bf16) else VP2P_GNA(float)
#undef VP2P_GNA
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_layer_norm_bwd(const vp2p_layer_norm_args* a, const void* dy, void* dx, void* stream) {
  if (!a || !a->x || !dy || !dx || a->rows < 0) return VP2P_E_ARG;
  if (a->dtype != VP2P_F32 && a->dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (a->channels <= 0 || a->channels % 8 || a->channels > 2048) return VP2P_E_SHAPE;
  if (a->rows == 0) return VP2P_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nv = (a->channels / 8 + 63) / 64;
  const dim3 grid((unsigned)((a->rows + 3) / 4)), block(256);
#define VP2P_LNB(T)                                                                                      \
  {                                                                                                      \
    const T* d = static_cast<const T*>(dy);                                                              \
    T* o = static_cast<T*>(dx);                                                                          \
    switch (nv) {                                                                                        \
      case 1: hipLaunchKernelGGL((ln_bwd_kernel<T, 1>), grid, block, 0, s, *a, d, o); break;             \
      case 2: hipLaunchKernelGGL((ln_bwd_kernel<T, 2>), grid, block, 0, s, *a, d, o); break;             \
      case 3: hipLaunchKernelGGL((ln_bwd_kernel<T, 3>), grid, block, 0, s, *a, d, o); break;             \
      default: hipLaunchKernelGGL((ln_bwd_kernel<T, 4>), grid, block, 0, s, *a, d, o); break;            \
    }                                                                                                    \
  }
  if (a->dtype == VP2P_BF16) VP2P_LNB(bf16) else VP2P_LNB(float)
#undef VP2P_LNB
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_geglu_bwd(const void* x, const void* dy, void* dx, int64_t rows, int32_t inner, int32_t dtype,
                              void* stream) {
  if (!x || !dy || !dx || rows < 0 || inner <= 0) return VP2P_E_ARG;
  if (dtype != VP2P_F32 && dtype != VP2P_BF16) return VP2P_E_DTYPE;
  if (inner % 8) return VP2P_E_SHAPE;
  if (rows == 0) return VP2P_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t n = rows * (inner / 8);
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (dtype == VP2P_BF16)
    hipLaunchKernelGGL((geglu_bwd_kernel<bf16>), grid, block, 0, s, static_cast<const bf16*>(x),
                       static_cast<const bf16*>(dy), static_cast<bf16*>(dx), rows, inner);
  else
    hipLaunchKernelGGL((geglu_bwd_kernel<float>), grid, block, 0, s, static_cast<const float*>(x),
                       static_cast<const float*>(dy), static_cast<float*>(dx), rows, inner);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}
