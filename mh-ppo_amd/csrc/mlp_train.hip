// mlp_train.hip — fused forward + loss gradient + backward + weight gradient of
// one continuous-head Model_PPO (13 -> 32 -> 64 -> 32 -> 1, ReLU;
// Coop-MH-PPO-scalable.py:42-93) over M rows, on f32 MFMA (v_mfma_f32_32x32x2_f32,
// exact fp32 products/sums).  Replaces, per epoch and head, the torch forward
// GEMMs, autograd backward and weight-gradient GEMMs of train_model_c
// (:778-815) whose K = M reductions ran at ~15 % of HBM bandwidth.
//
// Geometry: one wave owns a 32-row tile at a time (grid-stride over tiles) and
// keeps its running weight gradient in registers; 4 waves per block share the
// weights staged in LDS (padded strides, conflict-free operand reads).
// Orientation: activations are held TRANSPOSED, H^T [features x 32 rows]: the
// MFMA C tile then has the row on the lane (l & 31) and the features in the 16
// registers (feature(r, l) = (r&3) + 8(r>>2) + 4(l>>5)), so register s of a
// layer's output is the B operand of k-step s of the next layer (k order
// feature(s, l), matched by the A-operand weight reads) — no data movement
// between layers, forward or backward.  Weight gradients sum over rows, i.e.
// need rows on the K axis: the delta and activation tiles go through a
// wave-local LDS transpose [feature][row] (stride 33) for those MFMAs; bias
// gradients are row sums of the same LDS tiles.
//
// KIND 0 (critic pass): V = net(x); writes V, accumulates (sum A, sum A^2) of
//   A = ret - V (advantage statistics, :786-787) and the MSE loss; dV = 2(V-ret)/M.
// KIND 1 (actor pass): mu = tanh(y)*std + mean; A = ((ret - V) - mean_A) /
//   (std_A + 1e-10) from the global statistics; PPO clip surrogate with float64
//   ratio (:795-806); dy = dL/dmu * std * (1 - tanh^2).
// Outputs per wave: the packed torch-layout gradient (4673 floats) and float64
// partial sums; k_grad_stage1/2 sum the per-wave partials in fixed order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/mhppo.h"
#include "common.h"
#include "rollout_dev.h"

using namespace mhppo;

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 4;
constexpr int NIN = 13;
constexpr int NW = 32 * NIN + 32 + 64 * 32 + 64 + 32 * 64 + 32 + 32 + 1;  // 4673 packed params
constexpr int S1 = 15, S2 = 33, S3 = 65, ST = 33;                          // LDS row strides
// LDS layout (floats)
constexpr int O_W1 = 0, O_B1 = O_W1 + 32 * S1, O_W2 = O_B1 + 32, O_B2 = O_W2 + 64 * S2, O_W3 = O_B2 + 64,
              O_B3 = O_W3 + 32 * S3, O_W4 = O_B3 + 32, O_B4 = O_W4 + 32, O_WEND = O_B4 + 4;
constexpr int TILE = 32 * ST;                   // one transposed 32x32 tile
constexpr int O_X = 0, O_T = 32 * NIN;          // per-wave scratch: X tile, then 3 tiles
constexpr int WAVE_LDS = O_T + 3 * TILE + 32;   // + dy row
constexpr int LDS_FLOATS = O_WEND + WAVES * WAVE_LDS;
// packed gradient offsets (torch layout)
constexpr int G_W1 = 0, G_B1 = 32 * NIN, G_W2 = G_B1 + 32, G_B2 = G_W2 + 64 * 32, G_W3 = G_B2 + 64,
              G_B3 = G_W3 + 32 * 64, G_W4 = G_B3 + 32, G_B4 = G_W4 + 32;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int feat(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

// store a C tile (lane = row j, registers = feature(r,l)) as T[feature][row]
__device__ __forceinline__ void put_tile(float *T, const f32x16 &v, int l) {
#pragma unroll
  for (int r = 0; r < 16; r++) T[feat(r, l) * ST + (l & 31)] = v[r];
}
// row sum of T[f][0..31] for f = l & 31 (lanes >= 32 return the same sum)
__device__ __forceinline__ float row_sum(const float *T, int l) {
  const float *p = T + (l & 31) * ST;
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 32; c++) s += p[c];
  return s;
}

template <int KIND>
__global__ void __launch_bounds__(64 * WAVES)
    k_mlp_train(const float *__restrict__ W, const float *__restrict__ X, int64_t M, const float *__restrict__ ret,
                float *__restrict__ V, const float *__restrict__ act, const float *__restrict__ lp_old,
                const double *__restrict__ stats, double m_global, float out_mean, float out_std,
                float *__restrict__ gpart, double *__restrict__ dpart) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  // ---- stage weights (padded strides)
  for (int i = tid; i < 32 * NIN; i += 64 * WAVES) lds[O_W1 + (i / NIN) * S1 + i % NIN] = W[i];
  for (int i = tid; i < 32 * S1; i += 64 * WAVES)
    if (i % S1 >= NIN) lds[O_W1 + i] = 0.0f;
  for (int i = tid; i < 32; i += 64 * WAVES) lds[O_B1 + i] = W[G_B1 + i];
  for (int i = tid; i < 64 * 32; i += 64 * WAVES) lds[O_W2 + (i >> 5) * S2 + (i & 31)] = W[G_W2 + i];
  for (int i = tid; i < 64; i += 64 * WAVES) lds[O_B2 + i] = W[G_B2 + i];
  for (int i = tid; i < 32 * 64; i += 64 * WAVES) lds[O_W3 + (i >> 6) * S3 + (i & 63)] = W[G_W3 + i];
  for (int i = tid; i < 32; i += 64 * WAVES) {
    lds[O_B3 + i] = W[G_B3 + i];
    lds[O_W4 + i] = W[G_W4 + i];
  }
  if (tid == 0) lds[O_B4] = W[G_B4];
  __syncthreads();
  float *ws = lds + O_WEND + w * WAVE_LDS;
  float *Xs = ws + O_X, *T0 = ws + O_T, *T1 = T0 + TILE, *T2 = T1 + TILE, *dys = T2 + TILE;
  const float b4 = lds[O_B4];
  const int j = l & 31;
  const int kh = l >> 5;

  // persistent accumulators
  f32x16 gW1 = zero16(), gW2a = zero16(), gW2b = zero16(), gW3a = zero16(), gW3b = zero16();
  float gB1 = 0.f, gB2 = 0.f, gB3 = 0.f, gW4 = 0.f, gB4 = 0.f;
  double acc_loss = 0.0, acc_a = 0.0, acc_a2 = 0.0;
  float meanf = 0.f, stdf = 1.f;
  if (KIND == 1) {
    double mean = stats[0] / m_global;
    double var = (stats[1] - stats[0] * mean) / (m_global - 1.0);
    meanf = (float)mean;
    stdf = (float)sqrt(var > 0 ? var : 0.0);
  }
  const double inv_m = 1.0 / m_global;
  const int64_t ntiles = (M + 31) / 32;
  const int64_t gw = (int64_t)blockIdx.x * WAVES + w, nw = (int64_t)gridDim.x * WAVES;

  for (int64_t tile = gw; tile < ntiles; tile += nw) {
    const int64_t row0 = tile * 32;
    const int nrows = (int)min((int64_t)32, M - row0);
    // ---- X tile -> LDS [row][13]
    for (int q = l; q < 32 * NIN; q += 64) Xs[q] = (q / NIN < nrows) ? X[row0 * NIN + q] : 0.0f;
    wave_sync();
    // ---- forward
    f32x16 h1 = zero16();
#pragma unroll
    for (int s = 0; s < 7; s++) {
      int k = 2 * s + kh;
      float a = lds[O_W1 + j * S1 + k];
      float b = (k < NIN) ? Xs[j * NIN + k] : 0.0f;
      h1 = mfma(a, b, h1);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) h1[r] = relu(h1[r] + lds[O_B1 + feat(r, l)]);
    f32x16 h2a = zero16(), h2b = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = feat(s, l);
      h2a = mfma(lds[O_W2 + j * S2 + k], h1[s], h2a);
      h2b = mfma(lds[O_W2 + (32 + j) * S2 + k], h1[s], h2b);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
      h2a[r] = relu(h2a[r] + lds[O_B2 + feat(r, l)]);
      h2b[r] = relu(h2b[r] + lds[O_B2 + 32 + feat(r, l)]);
    }
    f32x16 h3 = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[O_W3 + j * S3 + feat(s, l)], h2a[s], h3);
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[O_W3 + j * S3 + 32 + feat(s, l)], h2b[s], h3);
    float part = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      h3[r] = relu(h3[r] + lds[O_B3 + feat(r, l)]);
      part = fmaf(lds[O_W4 + feat(r, l)], h3[r], part);
    }
    float y = (part + __shfl_xor(part, 32)) + b4;
    // ---- loss gradient dL/dy for this lane's row
    const int64_t row = row0 + j;
    const bool valid = j < nrows;
    float dy = 0.0f;
    if (valid) {
      float rt = ret[row];
      if (KIND == 0) {
        float v = y;
        if (kh == 0) V[row] = v;
        float a = rt - v;
        float d = v - rt;
        if (kh == 0) {
          acc_a += (double)a;
          acc_a2 += (double)a * (double)a;
          acc_loss += (double)d * (double)d;
        }
        dy = (float)(2.0 * inv_m * (double)d);
      } else {
        float t = tanhf(y);
        float mu = t * out_std + out_mean;
        float a = rt - V[row];
        float A = (a - meanf) / (stdf + 1e-10f);
        float diff = (float)((double)act[row] - (double)mu);
        float x = diff * MVN_INV_L;
        float lp = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HALF_LOGDET;
        double r = exp((double)lp - (double)lp_old[row]);
        double Ad = (double)A;
        double rc = r < 0.8 ? 0.8 : (r > 1.2 ? 1.2 : r);
        double s1 = r * Ad, s2 = rc * Ad, in = (r >= 0.8 && r <= 1.2) ? 1.0 : 0.0;
        double g = (s1 < s2) ? Ad : ((s2 < s1) ? in * Ad : 0.5 * Ad + 0.5 * in * Ad);
        if (kh == 0) acc_loss += -(s1 < s2 ? s1 : s2);
        float dmu = (float)(inv_m * (-g) * r * (double)x * (double)MVN_INV_L);
        dy = (dmu * out_std) * (1.0f - t * t);
      }
    }
    gB4 += (kh == 0) ? dy : 0.0f;
    // ---- layer 4 backward: dW4 = rowsum(dy * h3), dH3 = w4 * dy masked
    f32x16 g = zero16();
#pragma unroll
    for (int r = 0; r < 16; r++) {
      g[r] = dy * h3[r];
      h3[r] = (h3[r] > 0.0f) ? lds[O_W4 + feat(r, l)] * dy : 0.0f;  // h3 := dH3^T
    }
    put_tile(T0, g, l);
    put_tile(T1, h3, l);
    put_tile(T2, h2a, l);
    wave_sync();
    if (kh == 0) {
      gW4 += row_sum(T0, l);
      gB3 += row_sum(T1, l);
    }
    // dW3[:, 0:32] += dH3^T . H2a
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      gW3a = mfma(T1[j * ST + k], T2[j * ST + k], gW3a);
    }
    wave_sync();
    put_tile(T2, h2b, l);
    wave_sync();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      gW3b = mfma(T1[j * ST + k], T2[j * ST + k], gW3b);
    }
    // dH2^T = W3^T . dH3^T, masked by h2 > 0
    f32x16 d2a = zero16(), d2b = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int f = feat(s, l);
      d2a = mfma(lds[O_W3 + f * S3 + j], h3[s], d2a);
      d2b = mfma(lds[O_W3 + f * S3 + 32 + j], h3[s], d2b);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
      d2a[r] = (h2a[r] > 0.0f) ? d2a[r] : 0.0f;
      d2b[r] = (h2b[r] > 0.0f) ? d2b[r] : 0.0f;
    }
    wave_sync();
    put_tile(T0, d2a, l);
    put_tile(T1, d2b, l);
    put_tile(T2, h1, l);
    wave_sync();
    gB2 += row_sum(kh ? T1 : T0, l);
    // dW2 += dH2^T . H1
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      float b = T2[j * ST + k];
      gW2a = mfma(T0[j * ST + k], b, gW2a);
      gW2b = mfma(T1[j * ST + k], b, gW2b);
    }
    // dH1^T = W2^T . dH2^T, masked by h1 > 0
    f32x16 d1 = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) d1 = mfma(lds[O_W2 + feat(s, l) * S2 + j], d2a[s], d1);
#pragma unroll
    for (int s = 0; s < 16; s++) d1 = mfma(lds[O_W2 + (32 + feat(s, l)) * S2 + j], d2b[s], d1);
#pragma unroll
    for (int r = 0; r < 16; r++) d1[r] = (h1[r] > 0.0f) ? d1[r] : 0.0f;
    wave_sync();
    put_tile(T0, d1, l);
    wave_sync();
    if (kh == 0) gB1 += row_sum(T0, l);
    // dW1 += dH1^T . X
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      float b = (j < NIN) ? Xs[k * NIN + j] : 0.0f;
      gW1 = mfma(T0[j * ST + k], b, gW1);
    }
    wave_sync();
  }
  // ---- write this wave's partial gradient (packed torch layout)
  float *gp = gpart + (size_t)gw * NW;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    int f = feat(r, l);
    if (j < NIN) gp[G_W1 + f * NIN + j] = gW1[r];
    gp[G_W2 + f * 32 + j] = gW2a[r];
    gp[G_W2 + (32 + f) * 32 + j] = gW2b[r];
    gp[G_W3 + f * 64 + j] = gW3a[r];
    gp[G_W3 + f * 64 + 32 + j] = gW3b[r];
  }
  if (kh == 0) {
    gp[G_B1 + j] = gB1;
    gp[G_B3 + j] = gB3;
    gp[G_W4 + j] = gW4;
  }
  gp[G_B2 + l] = gB2;  // lanes 0-31: features 0-31 (T0), lanes 32-63: 32-63 (T1)
  // b4 and float64 sums: wave reductions
  float b4s = gB4;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) b4s += __shfl_xor(b4s, o);
  double s0 = acc_loss, s1 = acc_a, s2 = acc_a2;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (l == 0) {
    gp[G_B4] = b4s;
    dpart[gw * 3 + 0] = s0;
    dpart[gw * 3 + 1] = s1;
    dpart[gw * 3 + 2] = s2;
  }
}

// Deterministic two-stage gradient reduction over the per-wave partials (fixed order,
// float64): stage 1 sums contiguous groups of waves, stage 2 sums the RG group totals.
constexpr int RG = 32;
constexpr int NWD = NW + 3;  // gradient + (loss, sum A, sum A^2)

__global__ void __launch_bounds__(256)
    k_grad_stage1(const float *gpart, const double *dpart, int nw, double *tmp) {
  int k = blockIdx.x * 256 + threadIdx.x;
  int g = blockIdx.y;
  int i0 = (int)((int64_t)g * nw / RG), i1 = (int)((int64_t)(g + 1) * nw / RG);
  double s = 0.0;
  if (k < NW) {
    for (int i = i0; i < i1; i++) s += (double)gpart[(size_t)i * NW + k];
  } else if (k < NWD) {
    for (int i = i0; i < i1; i++) s += dpart[(size_t)i * 3 + (k - NW)];
  } else {
    return;
  }
  tmp[(size_t)g * NWD + k] = s;
}

__global__ void __launch_bounds__(256) k_grad_stage2(const double *tmp, float *grad, double *out3) {
  int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= NWD) return;
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < RG; g++) s += tmp[(size_t)g * NWD + k];
  if (k < NW)
    grad[k] = (float)s;
  else if (out3)
    out3[k - NW] += s;
}

struct Work {  // per-device partial buffers (calls on one device must share one stream)
  float *g = nullptr;
  double *d = nullptr;
  double *t = nullptr;
  int nw = 0;
};
Work g_work[16];

int grid_waves() {
  int dev = 0, cus = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus * 2 * WAVES;  // 2 blocks of 4 waves per CU
}
}  // namespace

extern "C" int mhppo_mlp_train_cont(int kind, const float *packed, const float *X, int64_t M, const float *ret,
                                    float *value, const float *act, const float *logp_old, const double *stats,
                                    double m_global, float out_mean, float out_std, float *grad, double *sums,
                                    void *stream) {
  if (!packed || !X || !ret || !value || !grad || M < 0 || (kind != 0 && kind != 1))
    return set_error(MHPPO_EINVAL, "bad argument");
  if (kind == 1 && (!act || !logp_old || !stats)) return set_error(MHPPO_EINVAL, "actor pass needs act/logp/stats");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  hipGetDevice(&dev);
  Work &wk = g_work[dev & 15];
  int nw = grid_waves();
  if (M > 0) nw = (int)min((int64_t)nw, ((M + 31) / 32 + WAVES - 1) / WAVES * WAVES);
  if (nw < WAVES) nw = WAVES;
  if (wk.nw < nw) {
    if (wk.g) (void)hipFree(wk.g);
    if (wk.d) (void)hipFree(wk.d);
    if (wk.t) (void)hipFree(wk.t);
    if (hipMalloc(&wk.g, sizeof(float) * (size_t)nw * NW) != hipSuccess ||
        hipMalloc(&wk.d, sizeof(double) * (size_t)nw * 3) != hipSuccess ||
        hipMalloc(&wk.t, sizeof(double) * (size_t)RG * NWD) != hipSuccess) {
      wk = Work{};
      return set_error(MHPPO_ENOMEM, "mlp_train partials");
    }
    wk.nw = nw;
  }
  dim3 grid(nw / WAVES), blk(64 * WAVES);
  size_t shm = sizeof(float) * LDS_FLOATS;
  if (kind == 0)
    hipLaunchKernelGGL(k_mlp_train<0>, grid, blk, shm, s, packed, X, M, ret, value, act, logp_old, stats, m_global,
                       out_mean, out_std, wk.g, wk.d);
  else
    hipLaunchKernelGGL(k_mlp_train<1>, grid, blk, shm, s, packed, X, M, ret, value, act, logp_old, stats, m_global,
                       out_mean, out_std, wk.g, wk.d);
  hipLaunchKernelGGL(k_grad_stage1, dim3((NWD + 255) / 256, RG), dim3(256), 0, s, wk.g, wk.d, nw, wk.t);
  hipLaunchKernelGGL(k_grad_stage2, dim3((NWD + 255) / 256), dim3(256), 0, s, wk.t, grad, sums);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}
