// K5 + K6 — classifier-free guidance, DDIM update and LocalBlend in one launch.
//
// Reference, per denoising step (pipeline_tuneavideo.py:409-424):
//   noise_pred = u + g * (t - u); fast: noise_pred[0] = t[0]                   (:409-415)
//   latents = scheduler.step(noise_pred, t, latents)  (eta = 0)                 (dependent_ddim.py:268-309)
//       x0 = (x - sqrt(1 - a_t) * e) / sqrt(a_t);  x' = sqrt(a_prev) * x0 + sqrt(1 - a_prev) * e
//   latents = controller.step_callback(latents) -> LocalBlend                   (run_videop2p.py:142-155)
//       m_p  = nearest_up(maxpool3x3(mean_40 sum_w alpha_p[w] * maps_p)) / max  > th
//       x_t  = x_t[:1] + (m_0 | m_p) * (x_t - x_t[:1])
// NullInversion.next_step / prev_step (run_videop2p.py:445-463) are the same update with other
// constants (cfg = 0).
//
// The reference runs these as ~20 separate torch kernels plus the mask pipeline; here one launch
// reads the UNet output once and writes the new latents once.  Every arithmetic op is rounded
// separately (fp contract off) so the DDIM/CFG/blend results match torch's fp32 eager ops bit for bit.
#include "common.hpp"
#include "vp2p.h"

namespace vp2p {

constexpr int kMaxLbPix = 1024;
constexpr int kMaxPrompts = 4;

template <typename TN>
__global__ __launch_bounds__(256) void step_kernel(const vp2p_step_args a) {
#pragma clang fp contract(off)
  __shared__ float pooled[kMaxPrompts * kMaxLbPix];
  __shared__ float pmax[kMaxPrompts];
  __shared__ float submax[kMaxPrompts];
  const int P = a.prompts, Cc = a.channels, F = a.frames, H = a.height, W = a.width;
  const int fr = blockIdx.x % F, c = blockIdx.x / F;
  const bool lb = a.lb_acc != nullptr;
  const int LH = a.lb_h, LW = a.lb_w, LHW = LH * LW;
  const int tid = threadIdx.x;

  if (lb) {
    for (int idx = tid; idx < P * LHW; idx += blockDim.x) {
      const int p = idx / LHW, k = idx - p * LHW, y = k / LW, x = k - y * LW;
      const float* src = a.lb_acc + ((int64_t)p * F + fr) * LHW;
      float m = kNegInf;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int yy = y + dy, xx = x + dx;
          if (yy >= 0 && yy < LH && xx >= 0 && xx < LW) m = fmaxf(m, src[yy * LW + xx] / a.lb_count);
        }
      pooled[p * kMaxLbPix + k] = m;
    }
    __syncthreads();
    const int wv = tid >> 6, ln = tid & 63;
    for (int p = wv; p < P; p += blockDim.x >> 6) {
      float m = kNegInf, ms = kNegInf;
      for (int k = ln; k < LHW; k += 64) {
        m = fmaxf(m, pooled[p * kMaxLbPix + k]);
        if (a.lb_sub) ms = fmaxf(ms, a.lb_sub[((int64_t)p * F + fr) * LHW + k] / a.lb_count);
      }
      for (int off = 32; off > 0; off >>= 1) {
        m = fmaxf(m, __shfl_xor(m, off));
        ms = fmaxf(ms, __shfl_xor(ms, off));
      }
      if (ln == 0) {
        pmax[p] = m;
        submax[p] = ms;
      }
    }
    __syncthreads();
  }
  // substruct_words mask (run_videop2p.py:149-151): get_mask(maps, substruct_layers, use_pool=False),
  // i.e. no pooling and threshold th[1]; it removes pixels from the blend mask
  auto sub_at = [&](int p, int k) {
    return a.lb_sub[((int64_t)p * F + fr) * LHW + k] / a.lb_count / submax[p] > a.lb_sub_th;
  };

  const float sy_scale = (float)LH / (float)H, sx_scale = (float)LW / (float)W;
  const int64_t HW = (int64_t)H * W;
  const TN* noise = static_cast<const TN*>(a.noise);
  for (int e = tid; e < HW; e += blockDim.x) {
    float prev[kMaxPrompts];
    for (int p = 0; p < P; ++p) {
      float eps;
      if (a.cfg) {
        const float u = (float)noise[(((int64_t)p * Cc + c) * F + fr) * HW + e];
        const float t = (float)noise[(((int64_t)(P + p) * Cc + c) * F + fr) * HW + e];
        eps = (a.fast && p == 0) ? t : u + a.guidance * (t - u);
      } else {
        eps = (float)noise[(((int64_t)p * Cc + c) * F + fr) * HW + e];
      }
      const float x = a.latents[(((int64_t)p * Cc + c) * F + fr) * HW + e];
      const float x0 = (x - a.c1 * eps) / a.c2;
      prev[p] = a.c4 * x0 + a.c3 * eps;
    }
    if (lb) {
      const int y = (int)(e / W), x = (int)(e - (int64_t)y * W);
      const int sy = min((int)floorf((float)y * sy_scale), LH - 1);
      const int sx = min((int)floorf((float)x * sx_scale), LW - 1);
      const int k = sy * LW + sx;
      const bool m0 = pooled[k] / pmax[0] > a.lb_th;
      const bool s0 = a.lb_sub && sub_at(0, k);
      for (int p = 0; p < P; ++p) {
        bool mp = m0 || (pooled[p * kMaxLbPix + k] / pmax[p] > a.lb_th);
        if (a.lb_sub) mp = mp && !(s0 || sub_at(p, k));
        const float mf = mp ? 1.f : 0.f;
        if (a.mask_out && c == 0) a.mask_out[((int64_t)p * F + fr) * HW + e] = mp ? 1 : 0;
        a.out[(((int64_t)p * Cc + c) * F + fr) * HW + e] = prev[0] + mf * (prev[p] - prev[0]);
      }
    } else {
      for (int p = 0; p < P; ++p) a.out[(((int64_t)p * Cc + c) * F + fr) * HW + e] = prev[p];
    }
  }
}

// Null-text inner loss (run_videop2p.py:594-599) and its gradient w.r.t. the unconditional noise:
//   e = u + g (c - u),  rec = c4 ((x - c1 e) / c2) + c3 e,  loss = mean((rec - x_prev)^2)
//   dloss/du = (2 / n) (rec - x_prev) (c3 - c4 c1 / c2) (1 - g)
// Pass 1 writes the gradient and one partial sum per block; pass 2 sums the partials in a fixed
// order (deterministic loss, compared against the early-stop epsilon every inner iteration).
constexpr int kLossBlocks = 1024;

template <typename TN>
__global__ __launch_bounds__(256) void nulltext_loss_kernel(const vp2p_nulltext_loss_args a) {
#pragma clang fp contract(off)
  __shared__ float red[4];
  const TN* u = static_cast<const TN*>(a.noise_uncond);
  const TN* c = static_cast<const TN*>(a.noise_cond);
  TN* gout = static_cast<TN*>(a.grad_uncond);
  const float de = a.c3 - a.c4 * a.c1 / a.c2;
  const float gscale = 2.f / (float)a.n * de * (1.f - a.guidance);
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const float uu = (float)u[i], cc = (float)c[i];
    const float e = uu + a.guidance * (cc - uu);
    const float x0 = (a.latents[i] - a.c1 * e) / a.c2;
    const float rec = a.c4 * x0 + a.c3 * e;
    const float d = rec - a.latents_prev[i];
    acc += d * d;
    gout[i] = (TN)(d * gscale);
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) a.partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void nulltext_loss_final_kernel(const vp2p_nulltext_loss_args a, int nblocks) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += blockDim.x) acc += a.partials[i];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) a.loss[0] = ((red[0] + red[1]) + (red[2] + red[3])) / (float)a.n;
}

}  // namespace vp2p

using namespace vp2p;

extern "C" int vp2p_nulltext_loss(const vp2p_nulltext_loss_args* a, void* stream) {
  if (!a || !a->noise_uncond || !a->noise_cond || !a->latents || !a->latents_prev || !a->grad_uncond ||
      !a->partials || !a->loss || a->n <= 0)
    return VP2P_E_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t want = (a->n + 255) / 256;
  const int blocks = (int)(want < kLossBlocks ? want : kLossBlocks);
  if (a->noise_dtype == VP2P_BF16)
    hipLaunchKernelGGL(nulltext_loss_kernel<bf16>, dim3(blocks), dim3(256), 0, s, *a);
  else if (a->noise_dtype == VP2P_F32)
    hipLaunchKernelGGL(nulltext_loss_kernel<float>, dim3(blocks), dim3(256), 0, s, *a);
  else
    return VP2P_E_DTYPE;
  hipLaunchKernelGGL(nulltext_loss_final_kernel, dim3(1), dim3(256), 0, s, *a, blocks);
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int32_t vp2p_nulltext_loss_partials(void) { return kLossBlocks; }

extern "C" int vp2p_step_fused(const vp2p_step_args* a, void* stream) {
  if (!a || !a->noise || !a->latents || !a->out) return VP2P_E_ARG;
  if (a->prompts <= 0 || a->channels <= 0 || a->frames <= 0 || a->height <= 0 || a->width <= 0)
    return VP2P_E_ARG;
  if (a->prompts > kMaxPrompts) return VP2P_E_SHAPE;
  if (a->lb_acc) {
    if (a->lb_h <= 0 || a->lb_w <= 0 || a->lb_count <= 0.f) return VP2P_E_ARG;
    if (a->lb_h * a->lb_w > kMaxLbPix) return VP2P_E_SHAPE;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid(a->frames * a->channels), block(256);
  if (a->noise_dtype == VP2P_BF16)
    hipLaunchKernelGGL(step_kernel<bf16>, grid, block, 0, s, *a);
  else if (a->noise_dtype == VP2P_F32)
    hipLaunchKernelGGL(step_kernel<float>, grid, block, 0, s, *a);
  else
    return VP2P_E_DTYPE;
  return hipGetLastError() == hipSuccess ? VP2P_OK : VP2P_E_LAUNCH;
}

extern "C" int vp2p_abi_version(void) { return VP2P_ABI_VERSION; }

extern "C" int vp2p_supported_head_dims(int32_t* out, int32_t capacity) {
  static const int32_t dims[] = {32, 40, 64, 80, 128, 160};
  const int n = (int)(sizeof(dims) / sizeof(dims[0]));
  for (int i = 0; i < n && out && i < capacity; ++i) out[i] = dims[i];
  return n;
}
