// Fused EgoAttention-2h Q-value forward for config 5 (policy in the loop), float32.
//
// Restates ttrl_agent/agents/common/models.py: MultiLayerPerceptron (:50-76), EgoAttention
// (:157-194), EgoAttentionNetwork.forward (:237-312), attention (:370-388) for
// ego_attention_2h.json (embeddings 7->64->64 ReLU, 2 heads of 32, output 64->64->64->A).
//
// Two launches, no intermediate round trip through torch:
//   rows_kernel  one lane per entity row (ego rows and other rows in separate blocks, so every
//                block reads one weight set and the weights are wave-uniform scalar loads):
//                embedding MLP, then the row's key and value; K^T, V^T [64][rows] and the ego
//                embeddings E^T [64][B] are written feature-major (coalesced across lanes).
//   env_kernel   one wave per 4 envs, lane o = feature o: query, masked softmax over the
//                entities per head, the value mix, the combine + residual, the output MLP.
// The forward is a dense contraction, but on gfx950 float32 MFMA issues at the float32
// vector rate, so the rows are plain FMAs fed by scalar-cached weights; the win over the torch
// graph is fusion (no HBM round trips of the [B*15, 64] activations) and launch count.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ttrl_mi355x.h"

namespace {

constexpr int HD = 64;  // hidden width of every layer

// Offsets (in floats) of each tensor in the packed weight buffer, see ttrl_mi355x.h.
struct PolicyLayout {
  int e1w, e1b, e2w, e2b, o1w, o1b, o2w, o2b, wv, wk, wq, wc, h1w, h1b, h2w, h2b, pw, pb, total;
};
__host__ __device__ inline PolicyLayout policy_layout(int F, int A) {
  PolicyLayout L;
  int p = 0;
  auto take = [&](int n) { const int r = p; p += n; return r; };
  L.e1w = take(HD * F); L.e1b = take(HD); L.e2w = take(HD * HD); L.e2b = take(HD);
  L.o1w = take(HD * F); L.o1b = take(HD); L.o2w = take(HD * HD); L.o2b = take(HD);
  L.wv = take(HD * HD); L.wk = take(HD * HD); L.wq = take(HD * HD); L.wc = take(HD * HD);
  L.h1w = take(HD * HD); L.h1b = take(HD); L.h2w = take(HD * HD); L.h2b = take(HD);
  L.pw = take(A * HD); L.pb = take(A);
  L.total = p;
  return L;
}

constexpr int RB = 256;  // rows (lanes) per rows_kernel block

// acc[o] += sum_k Wt[k][o] * in[k] in outer-product order: each k step is 64 independent FMAs
// (no serial accumulation chain) fed by broadcast float4 reads of the [in][out] weights.
__device__ __forceinline__ void dense64(const float4* __restrict__ wt, const float (&in)[HD], float (&acc)[HD]) {
#pragma unroll
  for (int k = 0; k < HD; ++k) {
#pragma unroll
    for (int o = 0; o < HD; o += 4) {
      const float4 w = wt[(k * HD + o) / 4];
      acc[o] = fmaf(w.x, in[k], acc[o]);
      acc[o + 1] = fmaf(w.y, in[k], acc[o + 1]);
      acc[o + 2] = fmaf(w.z, in[k], acc[o + 2]);
      acc[o + 3] = fmaf(w.w, in[k], acc[o + 3]);
    }
  }
}

template <int F>
__global__ void __launch_bounds__(RB) rows_kernel(const float* __restrict__ obs, int B, int NE,
                                                  const float* __restrict__ W, int A, float* __restrict__ KT,
                                                  float* __restrict__ VT, float* __restrict__ ET) {
  // the block's weights (embedding W1, b1, W2, b2, then key / value), transposed to [in][out]
  // in LDS once; every lane of the block multiplies by the same weights (broadcast reads)
  __shared__ float4 w2t[HD * HD / 4], wkt[HD * HD / 4], wvt[HD * HD / 4];
  __shared__ float w1t[F * HD], b1s[HD], b2s[HD];
  const PolicyLayout L = policy_layout(F, A);
  const int ego_blocks = (B + RB - 1) / RB;
  const bool ego = (int)blockIdx.x < ego_blocks;
  const float* w1 = W + (ego ? L.e1w : L.o1w);
  const float* b1 = W + (ego ? L.e1b : L.o1b);
  const float* w2 = W + (ego ? L.e2w : L.o2w);
  const float* b2 = W + (ego ? L.e2b : L.o2b);
  const int tid = threadIdx.x;
  float* w2f = reinterpret_cast<float*>(w2t);
  float* wkf = reinterpret_cast<float*>(wkt);
  float* wvf = reinterpret_cast<float*>(wvt);
  for (int i = tid; i < HD * HD; i += RB) {  // packed matrices are [in][out] already
    w2f[i] = w2[i];
    wkf[i] = W[L.wk + i];
    wvf[i] = W[L.wv + i];
  }
  for (int i = tid; i < HD * F; i += RB) w1t[i] = w1[i];
  if (tid < HD) { b1s[tid] = b1[tid]; b2s[tid] = b2[tid]; }
  __syncthreads();
  const long t = ego ? (long)blockIdx.x * RB + tid : (long)(blockIdx.x - ego_blocks) * RB + tid;
  const long n_rows = ego ? B : (long)B * (NE - 1);
  if (t >= n_rows) return;
  const long env = ego ? t : t / (NE - 1);
  const int j = ego ? 0 : 1 + (int)(t % (NE - 1));
  const long row = env * NE + j;
  const long R = (long)B * NE;
  float x[F];
#pragma unroll
  for (int k = 0; k < F; ++k) x[k] = obs[row * F + k];
  float h1[HD], acc[HD];
#pragma unroll
  for (int o = 0; o < HD; ++o) h1[o] = b1s[o];
#pragma unroll
  for (int k = 0; k < F; ++k)
#pragma unroll
    for (int o = 0; o < HD; ++o) h1[o] = fmaf(w1t[k * HD + o], x[k], h1[o]);
#pragma unroll
  for (int o = 0; o < HD; ++o) { h1[o] = h1[o] > 0.0f ? h1[o] : 0.0f; acc[o] = b2s[o]; }
  dense64(w2t, h1, acc);
  float h2[HD];
#pragma unroll
  for (int o = 0; o < HD; ++o) h2[o] = acc[o] > 0.0f ? acc[o] : 0.0f;
  if (ego)
#pragma unroll
    for (int o = 0; o < HD; ++o) ET[(long)o * B + env] = h2[o];
#pragma unroll
  for (int o = 0; o < HD; ++o) acc[o] = 0.0f;
  dense64(wkt, h2, acc);
#pragma unroll
  for (int o = 0; o < HD; ++o) { KT[(long)o * R + row] = acc[o]; acc[o] = 0.0f; }
  dense64(wvt, h2, acc);
#pragma unroll
  for (int o = 0; o < HD; ++o) VT[(long)o * R + row] = acc[o];
}

constexpr int EPB = 8;  // envs per wave in env_kernel

template <int F>
__global__ void __launch_bounds__(64) env_kernel(const float* __restrict__ obs, int B, int NE, int heads,
                                                 const float* __restrict__ W, int A, const float* __restrict__ KT,
                                                 const float* __restrict__ VT, const float* __restrict__ ET,
                                                 float* __restrict__ Q) {
  const PolicyLayout L = policy_layout(F, A);
  __shared__ float vec[EPB][HD];       // the vector being multiplied (q input, value mix, ...)
  __shared__ float prob[EPB][8][32];   // softmax weights [head][entity] (heads * NE <= 64)
  const int o = threadIdx.x;
  const int dph = HD / heads;
  const long R = (long)B * NE;
  const float scale = 1.0f / sqrtf((float)dph);
  float e[EPB];
#pragma unroll
  for (int u = 0; u < EPB; ++u) {
    const long b = (long)blockIdx.x * EPB + u;
    e[u] = b < B ? ET[(long)o * B + b] : 0.0f;
    vec[u][o] = e[u];
  }
  __syncthreads();
  // query_ego: q[o] = Wq[o] . e
  float q[EPB];
#pragma unroll
  for (int u = 0; u < EPB; ++u) q[u] = 0.0f;
  for (int k = 0; k < HD; ++k) {
    const float w = W[L.wq + k * HD + o];  // [in][out]: coalesced across lanes
#pragma unroll
    for (int u = 0; u < EPB; ++u) q[u] = fmaf(w, vec[u][k], q[u]);
  }
  __syncthreads();
  // scores per (head, entity): lane o < heads*NE takes one; masked_fill(presence < 0.5, -1e9)
  const int h = o / NE, jj = o % NE;
#pragma unroll
  for (int u = 0; u < EPB; ++u) {
    vec[u][o] = q[u];
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < EPB; ++u) {
    const long b = (long)blockIdx.x * EPB + u;
    if (o < heads * NE && b < B) {
      float s = 0.0f;
      for (int d = 0; d < dph; ++d) s = fmaf(vec[u][h * dph + d], KT[(long)(h * dph + d) * R + b * NE + jj], s);
      s = s * scale;
      if (obs[(b * NE + jj) * F + 0] < 0.5f) s = -1e9f;
      prob[u][h][jj] = s;
    }
  }
  __syncthreads();
  if (o < heads * EPB) {  // softmax over the entities of one (env, head)
    const int u = o / heads, hh = o % heads;
    float m = -3.4e38f;
    for (int k = 0; k < NE; ++k) m = fmaxf(m, prob[u][hh][k]);
    float sum = 0.0f;
    for (int k = 0; k < NE; ++k) {
      const float p = expf(prob[u][hh][k] - m);
      prob[u][hh][k] = p;
      sum += p;
    }
    for (int k = 0; k < NE; ++k) prob[u][hh][k] /= sum;
  }
  __syncthreads();
  // value mix: out[o] = sum_j p[head(o)][j] V[j][o]
  float mix[EPB];
#pragma unroll
  for (int u = 0; u < EPB; ++u) {
    const long b = (long)blockIdx.x * EPB + u;
    float a = 0.0f;
    if (b < B)
      for (int k = 0; k < NE; ++k) a = fmaf(prob[u][o / dph][k], VT[(long)o * R + b * NE + k], a);
    mix[u] = a;
  }
#pragma unroll
  for (int u = 0; u < EPB; ++u) vec[u][o] = mix[u];
  __syncthreads();
  // attention_combine + residual: (Wc . out + ego) / 2
  float att[EPB];
#pragma unroll
  for (int u = 0; u < EPB; ++u) att[u] = 0.0f;
  for (int k = 0; k < HD; ++k) {
    const float w = W[L.wc + k * HD + o];
#pragma unroll
    for (int u = 0; u < EPB; ++u) att[u] = fmaf(w, vec[u][k], att[u]);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < EPB; ++u) vec[u][o] = (att[u] + e[u]) / 2.0f;
  __syncthreads();
  // output MLP 64 -> 64 -> 64 (ReLU) -> A
  const int offs_w[2] = {L.h1w, L.h2w}, offs_b[2] = {L.h1b, L.h2b};
  for (int layer = 0; layer < 2; ++layer) {
    float a[EPB];
#pragma unroll
    for (int u = 0; u < EPB; ++u) a[u] = W[offs_b[layer] + o];
    for (int k = 0; k < HD; ++k) {
      const float w = W[offs_w[layer] + k * HD + o];
#pragma unroll
      for (int u = 0; u < EPB; ++u) a[u] = fmaf(w, vec[u][k], a[u]);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < EPB; ++u) vec[u][o] = a[u] > 0.0f ? a[u] : 0.0f;
    __syncthreads();
  }
  if (o < A * EPB) {
    const int u = o / A, act = o % A;
    const long b = (long)blockIdx.x * EPB + u;
    if (b < B) {
      float a = W[L.pb + act];
      for (int k = 0; k < HD; ++k) a = fmaf(W[L.pw + k * A + act], vec[u][k], a);
      Q[b * A + act] = a;
    }
  }
}

template <int F>
int launch(const float* obs, int B, int NE, int heads, const float* W, int A, float* scratch, float* Q,
           hipStream_t st) {
  const long R = (long)B * NE;
  float* KT = scratch;
  float* VT = KT + HD * R;
  float* ET = VT + HD * R;
  const int blocks1 = (B + RB - 1) / RB + (int)((B * (long)(NE - 1) + RB - 1) / RB);
  hipLaunchKernelGGL(rows_kernel<F>, dim3(blocks1), dim3(RB), 0, st, obs, B, NE, W, A, KT, VT, ET);
  hipLaunchKernelGGL(env_kernel<F>, dim3((B + EPB - 1) / EPB), dim3(64), 0, st, obs, B, NE, heads, W, A, KT, VT,
                     ET, Q);
  return hipGetLastError() == hipSuccess ? TTRL_OK : TTRL_E_LAUNCH;
}

}  // namespace

extern "C" {

int64_t ttrl_ego_attention_sizes(int32_t n_features, int32_t n_actions, int32_t batch, int32_t n_entities,
                                 int64_t* scratch_floats) {
  if (n_features < 1 || n_features > 16 || n_actions < 1 || n_actions > 16) return TTRL_E_ARG;
  if (scratch_floats) *scratch_floats = (int64_t)HD * batch * (2 * (int64_t)n_entities + 1);
  return policy_layout(n_features, n_actions).total;
}

int ttrl_ego_attention_q(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features, int32_t heads,
                         const float* weights, int32_t n_actions, float* scratch, float* q, void* stream) {
  if (!obs || !weights || !scratch || !q || batch < 0 || n_entities < 2 || n_entities > 32 || n_actions < 1 ||
      n_actions > 16 || (heads != 1 && heads != 2 && heads != 4 && heads != 8) || heads * n_entities > 64)
    return TTRL_E_ARG;
  if (batch == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (n_features) {
    case 5: return launch<5>(obs, batch, n_entities, heads, weights, n_actions, scratch, q, st);
    case 7: return launch<7>(obs, batch, n_entities, heads, weights, n_actions, scratch, q, st);
    case 8: return launch<8>(obs, batch, n_entities, heads, weights, n_actions, scratch, q, st);
    default: return TTRL_E_UNSUPPORTED;
  }
}

}  // extern "C"
