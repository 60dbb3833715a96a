// Fused EgoAttention-2h Q-value forward for config 5 (policy in the loop), float32.
//
// Restates ttrl_agent/agents/common/models.py: MultiLayerPerceptron (:50-76), EgoAttention
// (:157-194), EgoAttentionNetwork.forward (:237-312), attention (:370-388) for
// ego_attention_2h.json (embeddings 7->64->64 ReLU, 2 heads of 32, output 64->64->64->A).
//
// One launch (ego_attention_kernel below): a wave per 4 envs, lane k = feature k, the key and
// value projections moved out of the entity loop by linearity, the per-entity scores summed over
// the lanes by one transposing butterfly; only the Q-values reach HBM.
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

constexpr int EPWV = 4;  // envs per wave of ego_attention_kernel

#ifdef TTRL_POL_CLOCKS  // diagnostic build: shader-clock stamps at the phase boundaries of each wave
constexpr int POL_CLK_BLOCKS = 4096;
__device__ long long g_pol_clk[POL_CLK_BLOCKS * 9];
#define POL_T(n) (pol_clk[n] = clock64())
#else
#define POL_T(n) ((void)0)
#endif

// acc[u] += sum_k W[k][o] * v[k].u for the wave's EPWV vectors staged in LDS as one float4 per
// feature (env u in component u). Lane o's whole weight column (the [in][out] rows are coalesced
// across lanes) is requested before the first FMA, so one memory latency covers the 64 loads;
// each weight is used EPWV times.
__device__ __forceinline__ void matvec4(const float* __restrict__ w, const float4* v, int o, float (&acc)[EPWV]) {
  float col[HD];
#pragma unroll
  for (int k = 0; k < HD; ++k) col[k] = w[k * HD + o];
#pragma unroll
  for (int k = 0; k < HD; ++k) {
    const float4 x = v[k];
    acc[0] = fmaf(col[k], x.x, acc[0]);
    acc[1] = fmaf(col[k], x.y, acc[1]);
    acc[2] = fmaf(col[k], x.z, acc[2]);
    acc[3] = fmaf(col[k], x.w, acc[3]);
  }
}

__device__ __forceinline__ float4 f4(const float (&a)[EPWV]) { return make_float4(a[0], a[1], a[2], a[3]); }

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// v from the lane whose index differs in bit B (quad_perm / ds_swizzle / row_ror:8 / bpermute)
template <int B>
__device__ __forceinline__ float lane_xor(float v) {
  if constexpr (B == 0) return dpp_f<0xB1>(v);
  else if constexpr (B == 1) return dpp_f<0x4E>(v);
  else if constexpr (B == 2) return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x101F));
  else if constexpr (B == 3) return dpp_f<0x128>(v);
  else if constexpr (B == 4) return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F));
  else return __int_as_float(__builtin_amdgcn_ds_bpermute((int)((threadIdx.x ^ 32) << 2), __float_as_int(v)));
}

// Sums over the wave's 64 lanes of N values at once (a transposing butterfly): at lane bit B the
// lanes with the bit set keep the upper half of their values and send the lower half, so N values
// take N - 1 + (6 - log2 N) exchanges instead of 6 N. Afterwards v[0] of lane L is the sum of value
// fold_index<N>(L); lanes 0 .. N-1 hold every index once.
template <int B, int N>
__device__ __forceinline__ void fold(float* v, int lane) {
  if constexpr (N > 1) {
    const bool hi = (lane >> B) & 1;
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float keep = hi ? v[i + N / 2] : v[i];
      const float send = hi ? v[i] : v[i + N / 2];
      v[i] = keep + lane_xor<B>(send);
    }
    fold<B + 1, N / 2>(v, lane);
  } else if constexpr (B < 6) {
    v[0] += lane_xor<B>(v[0]);
    fold<B + 1, 1>(v, lane);
  }
}

template <int N>
__device__ __forceinline__ int fold_index(int lane) {
  int idx = 0;
#pragma unroll
  for (int b = 0, n = N; n > 1; ++b, n >>= 1) idx += ((lane >> b) & 1) * (n / 2);
  return idx;
}

// LDS of one wave (floats): the broadcast vectors, the wave's observations, the ego embeddings,
// qk_h (then the per-head weighted embedding sums), the ego scores
struct PolLds {
  int ob, es, qk, s0, total;
};
__host__ __device__ inline PolLds pol_lds(int NE, int F, int H) {
  PolLds P;
  P.ob = HD * 4;
  P.es = P.ob + ((EPWV * NE * F + 3) & ~3);
  P.qk = P.es + HD * 4;
  P.s0 = P.qk + H * HD * 4;
  P.total = P.s0 + EPWV * (H > 16 ? H : 16);  // the ego scores, later the Q rows of the argmax (A <= 16)
  return P;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// D = A B + C on a 16 x 16 x 4 float32 tile (exact fmaf chain over k). Lane l holds A[l & 15][l >> 4],
// B[l >> 4][l & 15] and D[4 (l >> 4) + r][l & 15] in register r.
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// EpsilonGreedy acting fused into the forward (epsilon_greedy.py:32-48 with DiscreteDistribution.sample,
// exploration/abstract.py:20-25; AbstractDQNAgent.act, dqn/abstract.py:65-83): the greedy action is
// np.argmax(Q) (the first maximum; a NaN wins, as in numpy), and with probability epsilon a uniform
// action replaces it -- the distribution {a: epsilon / A + (1 - epsilon) [a == greedy]} the reference
// samples.  The draws are counter-based, Philox4x32-10 keyed on the seed with counter (env, step):
// any batch split or replay order gives each env the same action.  epsilon / step come from device
// scalars when given (a captured HIP graph refreshes them between replays).
struct Explore {
  int64_t* act;            // [B] actions out (int64); both null: Q-values only
  int32_t* act32;          // [B] the same actions as int32 (the env's action index type)
  float eps;
  const float* eps_dev;    // overrides eps when set
  long long step;
  const int64_t* step_dev; // overrides step when set
  unsigned seed_lo, seed_hi;
  long long env_offset;    // global env id of row 0: the draws are keyed on (env_offset + row, step)
};

__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    c = make_uint4((unsigned)(p1 >> 32) ^ c.y ^ key.x, (unsigned)p1, (unsigned)(p0 >> 32) ^ c.w ^ key.y, (unsigned)p0);
    key.x += 0x9E3779B9u; key.y += 0xBB67AE85u;
  }
  return c;
}

// One wave per EPWV envs, lane k = feature k. Linearity moves the key and value projections
// out of the entity loop: with x_j the 64-wide embedding of entity j,
//   score_hj = q_h . (Wk x_j)_h / sqrt(d) = x_j . qk_h,      qk_h = Wk_h^T q_h / sqrt(d)
//   mix_h    = sum_j p_hj (Wv x_j)_h      = (Wv (sum_j p_hj x_j))_h
// so an entity costs only its embedding, and the value projection runs once per env on the
// weighted embedding sum.
//   1. ego embeddings, queries, qk_h, the ego's scores (VALU, lane k = feature k; env-level
//      weights loaded once per wave, used EPWV times)
//   2. the other entities, 4 at a time for the wave's 4 envs: a 16-column tile (column c = entity
//      c >> 2, env c & 3) through both embedding layers on float32 MFMA 16x16x4 (the first
//      layer's output tile is the second's B operand in place: its k order is permuted, and the
//      register-resident weight fragments follow that order), scores from the tile rows each
//      lane holds, masked_fill(presence < 0.5, -1e9) (models.py:383), and an online softmax over
//      the entities (models.py:384): running max / sum / weighted embedding sum per (env, head)
//   3. the value projection, attention_combine + residual (att + ego) / 2, output MLP, predict
// No [B*NE, 64] activation reaches HBM; f32 MFMA is exact f32 (an fmaf chain) at the f32 vector
// rate, but it needs no LDS broadcast of the activations, which bounded the VALU form.
template <int F, int H>
__global__ void __launch_bounds__(64, 2) ego_attention_kernel(const float* __restrict__ obs, int B, int NE,
                                                              const float* __restrict__ W, int A,
                                                              float* __restrict__ Q, Explore ex) {
  constexpr int DPH = HD / H, NV = EPWV * H;
  const PolicyLayout L = policy_layout(F, A);
  const PolLds P = pol_lds(NE, F, H);
#ifdef TTRL_POL_CLOCKS
  long long pol_clk[9];
  pol_clk[0] = clock64();
#endif
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  float4* bc = lds4;                                 // [HD] vectors broadcast to the wave
  const float* ob = lds + P.ob;                      // [EPWV][NE][F]
  float4* es = reinterpret_cast<float4*>(lds + P.es);  // [HD] ego embeddings
  float4* qks = reinterpret_cast<float4*>(lds + P.qk);  // [H][HD] qk_h; then the weighted sums
  float* s0s = lds + P.s0;                           // [EPWV][H] the ego's scores
  const int k = threadIdx.x;
  const long b0 = (long)blockIdx.x * EPWV;
  {  // one coalesced copy of the wave's EPWV consecutive [NE][F] observations
    const long avail = ((long)B - b0) * NE * F;  // a partial last wave repeats env b0 (never stored)
    const int n = EPWV * NE * F;
    for (int i = k; i < n; i += HD) lds[P.ob + i] = obs[b0 * NE * F + (i < avail ? i : i % (NE * F))];
  }
  __syncthreads();
  // 1. ego embeddings (MultiLayerPerceptron, ReLU after both layers), queries, qk_h
  POL_T(1);
  float e[EPWV], t[EPWV];
#pragma unroll
  for (int u = 0; u < EPWV; ++u) {
    float h = W[L.e1b + k];
#pragma unroll
    for (int f = 0; f < F; ++f) h = fmaf(W[L.e1w + f * HD + k], ob[u * NE * F + f], h);
    t[u] = h > 0.0f ? h : 0.0f;
    e[u] = W[L.e2b + k];
  }
  bc[k] = f4(t);
  __syncthreads();
  matvec4(W + L.e2w, bc, k, e);
  POL_T(2);
#pragma unroll
  for (int u = 0; u < EPWV; ++u) {
    e[u] = e[u] > 0.0f ? e[u] : 0.0f;
    t[u] = 0.0f;
  }
  __syncthreads();
  bc[k] = f4(e);
  __syncthreads();
  matvec4(W + L.wq, bc, k, t);  // t = q (lane o = query feature o)
  POL_T(3);
  __syncthreads();
  bc[k] = f4(t);
  __syncthreads();
  float qk[EPWV][H];
#pragma unroll
  for (int u = 0; u < EPWV; ++u)
#pragma unroll
    for (int h = 0; h < H; ++h) qk[u][h] = 0.0f;
  const float4* wrow = reinterpret_cast<const float4*>(W + L.wk + k * HD);  // Wk[k][.]: row k
#pragma unroll
  for (int o4 = 0; o4 < HD / 4; ++o4) {
    const float4 w = wrow[o4];
    const int h = o4 * 4 / DPH;
    const float4 q0 = bc[o4 * 4], q1 = bc[o4 * 4 + 1], q2 = bc[o4 * 4 + 2], q3 = bc[o4 * 4 + 3];
    qk[0][h] = fmaf(w.w, q3.x, fmaf(w.z, q2.x, fmaf(w.y, q1.x, fmaf(w.x, q0.x, qk[0][h]))));
    qk[1][h] = fmaf(w.w, q3.y, fmaf(w.z, q2.y, fmaf(w.y, q1.y, fmaf(w.x, q0.y, qk[1][h]))));
    qk[2][h] = fmaf(w.w, q3.z, fmaf(w.z, q2.z, fmaf(w.y, q1.z, fmaf(w.x, q0.z, qk[2][h]))));
    qk[3][h] = fmaf(w.w, q3.w, fmaf(w.z, q2.w, fmaf(w.y, q1.w, fmaf(w.x, q0.w, qk[3][h]))));
  }
  const float scale = 1.0f / sqrtf((float)DPH);
#pragma unroll
  for (int u = 0; u < EPWV; ++u)
#pragma unroll
    for (int h = 0; h < H; ++h) qk[u][h] *= scale;
  // the ego (entity 0): its score x_0 . qk_h summed over the lanes, masked like the others
  POL_T(4);
  {
    float v[NV];
#pragma unroll
    for (int u = 0; u < EPWV; ++u)
#pragma unroll
      for (int h = 0; h < H; ++h) v[u * H + h] = e[u] * qk[u][h];
    fold<0, NV>(v, k);
    const int idx = fold_index<NV>(k);
    if (k < NV) s0s[idx] = ob[(idx / H) * NE * F] < 0.5f ? -1e9f : v[0];
    es[k] = f4(e);
#pragma unroll
    for (int h = 0; h < H; ++h) qks[h * HD + k] = make_float4(qk[0][h], qk[1][h], qk[2][h], qk[3][h]);
  }
  // 2. the other entities on MFMA. Lane l: column c = l & 15 (entity jj = c >> 2 of the batch,
  // env u = c & 3), row group g = l >> 4; it holds tile rows 16 M + 4 g + r (M, r = 0..3).
  const int g = k >> 4, c = k & 15, jj = c >> 2, u = c & 3;
  constexpr int KS1 = (F + 1 + 3) / 4;  // first-layer k steps: F inputs, then the bias (input = 1)
  float a1[KS1][4], a2[4][4][4], b2[4][4];
#pragma unroll
  for (int st = 0; st < KS1; ++st)
#pragma unroll
    for (int M = 0; M < 4; ++M) {
      const int in = 4 * st + g;
      a1[st][M] = in < F ? W[L.o1w + in * HD + 16 * M + c] : (in == F ? W[L.o1b + 16 * M + c] : 0.0f);
    }
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) a2[M][m][r] = W[L.o2w + (16 * m + 4 * g + r) * HD + 16 * M + c];
#pragma unroll
  for (int M = 0; M < 4; ++M)
#pragma unroll
    for (int r = 0; r < 4; ++r) b2[M][r] = W[L.o2b + 16 * M + 4 * g + r];
  __syncthreads();
  float qf[H][4][4], acc[H][4][4], mx[H], sm[H];
  {
    const float* qkf = reinterpret_cast<const float*>(qks);
    const float* ef = reinterpret_cast<const float*>(es);
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 16 * M + 4 * g + r;
        const float x0 = jj == 0 ? ef[f * 4 + u] : 0.0f;  // the ego's term, counted once per env
#pragma unroll
        for (int h = 0; h < H; ++h) {
          qf[h][M][r] = qkf[(h * HD + f) * 4 + u];
          acc[h][M][r] = x0;
        }
      }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      mx[h] = s0s[u * H + h];
      sm[h] = 1.0f;
    }
  }
  POL_T(5);
  for (int j0 = 1; j0 < NE; j0 += 4) {
    const int j = j0 + jj;
    const bool live = j < NE;
    const float* oj = ob + (u * NE + (live ? j : 0)) * F;
    f32x4 t1[4];
#pragma unroll
    for (int M = 0; M < 4; ++M) t1[M] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int st = 0; st < KS1; ++st) {
      const int in = 4 * st + g;
      const float bv = !live ? 0.0f : (in < F ? oj[in < F ? in : 0] : (in == F ? 1.0f : 0.0f));
#pragma unroll
      for (int M = 0; M < 4; ++M) t1[M] = mfma4(a1[st][M], bv, t1[M]);
    }
    f32x4 t2[4];
#pragma unroll
    for (int M = 0; M < 4; ++M) t2[M] = f32x4{b2[M][0], b2[M][1], b2[M][2], b2[M][3]};
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x1 = t1[m][r] > 0.0f ? t1[m][r] : 0.0f;  // ReLU; k step (m, r) = rows 16 m + 4 g + r
#pragma unroll
        for (int M = 0; M < 4; ++M) t2[M] = mfma4(a2[M][m][r], x1, t2[M]);
      }
    float x[4][4];
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 4; ++r) x[M][r] = t2[M][r] > 0.0f ? t2[M][r] : 0.0f;
    const float presence = oj[0];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float sc = 0.0f;
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc = fmaf(x[M][r], qf[h][M][r], sc);
      sc += lane_xor<4>(sc);  // the other row groups of the column
      sc += lane_xor<5>(sc);
      sc = !live ? -__builtin_inff() : (presence < 0.5f ? -1e9f : sc);
      float bm = fmaxf(sc, lane_xor<2>(sc));  // the batch's entities of env u
      bm = fmaxf(bm, lane_xor<3>(bm));
      const float mn = fmaxf(mx[h], bm), corr = expf(mx[h] - mn), p = expf(sc - mn);
      float ps = p + lane_xor<2>(p);
      ps += lane_xor<3>(ps);
      sm[h] = fmaf(sm[h], corr, ps);
      mx[h] = mn;
#pragma unroll
      for (int M = 0; M < 4; ++M)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[h][M][r] = fmaf(acc[h][M][r], corr, p * x[M][r]);
    }
  }
  // the weighted sums of env u over the batch columns (lanes differing in bits 2, 3), to LDS
  __syncthreads();
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int M = 0; M < 4; ++M)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = acc[h][M][r];
        a += lane_xor<2>(a);
        a += lane_xor<3>(a);
        if (jj == 0) reinterpret_cast<float*>(qks)[(h * HD + 16 * M + 4 * g + r) * 4 + u] = a / sm[h];
      }
  // 3. value projection per head, attention_combine, residual, output MLP, predict
  POL_T(6);
#pragma unroll
  for (int v = 0; v < EPWV; ++v) t[v] = 0.0f;
  __syncthreads();
  matvec4(W + L.wv, qks + (k / DPH) * HD, k, t);  // output feature k belongs to head k / DPH
  __syncthreads();
  float y[EPWV];
#pragma unroll
  for (int u = 0; u < EPWV; ++u) y[u] = 0.0f;
  bc[k] = f4(t);
  __syncthreads();
  matvec4(W + L.wc, bc, k, y);
  POL_T(7);
#pragma unroll
  for (int u = 0; u < EPWV; ++u) y[u] = (y[u] + e[u]) / 2.0f;
  const int offs_w[2] = {L.h1w, L.h2w}, offs_b[2] = {L.h1b, L.h2b};
#pragma unroll
  for (int layer = 0; layer < 2; ++layer) {
    __syncthreads();
    bc[k] = f4(y);
#pragma unroll
    for (int u = 0; u < EPWV; ++u) y[u] = W[offs_b[layer] + k];
    __syncthreads();
    matvec4(W + offs_w[layer], bc, k, y);
#pragma unroll
    for (int u = 0; u < EPWV; ++u) y[u] = y[u] > 0.0f ? y[u] : 0.0f;
  }
  __syncthreads();
  bc[k] = f4(y);
  __syncthreads();
  if (k < A) {
    float a[EPWV];
#pragma unroll
    for (int u = 0; u < EPWV; ++u) a[u] = W[L.pb + k];
#pragma unroll 16
    for (int i = 0; i < HD; ++i) {
      const float w = W[L.pw + i * A + k];
      const float4 v = bc[i];
      a[0] = fmaf(w, v.x, a[0]);
      a[1] = fmaf(w, v.y, a[1]);
      a[2] = fmaf(w, v.z, a[2]);
      a[3] = fmaf(w, v.w, a[3]);
    }
#pragma unroll
    for (int u = 0; u < EPWV; ++u) {
      if (b0 + u < B) Q[(b0 + u) * A + k] = a[u];
      if (ex.act || ex.act32) s0s[u * 16 + k] = a[u];  // the ego scores' LDS is dead: the env's Q row for the argmax
    }
  }
  if (ex.act || ex.act32) {  // 4. epsilon-greedy: lane u acts for env b0 + u
    __syncthreads();
    if (k < EPWV && b0 + k < B) {
      const float* qrow = s0s + k * 16;
      int best = 0;
      float bq = qrow[0];
      for (int i = 1; i < A; ++i) {
        const float v = qrow[i];
        if (bq == bq && (v > bq || v != v)) { bq = v; best = i; }  // np.argmax: first max, first NaN
      }
      const float eps = ex.eps_dev ? *ex.eps_dev : ex.eps;
      const unsigned long long step = ex.step_dev ? (unsigned long long)*ex.step_dev : (unsigned long long)ex.step;
      const unsigned long long env = (unsigned long long)ex.env_offset + (unsigned long long)(b0 + k);
      const uint4 r = philox4x32(make_uint4((unsigned)env, (unsigned)(env >> 32), (unsigned)step, (unsigned)(step >> 32)),
                                 make_uint2(ex.seed_lo, ex.seed_hi));
      const float uni = (float)(r.x >> 8) * 0x1p-24f;                       // U[0, 1)
      const int rnd = (int)(((unsigned long long)r.y * (unsigned)A) >> 32);  // U{0 .. A-1}
      const int pick = uni < eps ? rnd : best;
      if (ex.act) ex.act[b0 + k] = pick;
      if (ex.act32) ex.act32[b0 + k] = pick;
    }
  }
  POL_T(8);
#ifdef TTRL_POL_CLOCKS
  if (k == 0 && blockIdx.x < POL_CLK_BLOCKS)
    for (int n = 0; n < 9; ++n) g_pol_clk[blockIdx.x * 9 + n] = pol_clk[n] - pol_clk[0];
#endif
}

template <int F, int H>
int launch(const float* obs, int B, int NE, const float* W, int A, float* Q, const Explore& ex, hipStream_t st) {
  const size_t lds = pol_lds(NE, F, H).total * sizeof(float);
  hipLaunchKernelGGL((ego_attention_kernel<F, H>), dim3((B + EPWV - 1) / EPWV), dim3(64), lds, st, obs, B, NE,
                     W, A, Q, ex);
  return hipGetLastError() == hipSuccess ? TTRL_OK : TTRL_E_LAUNCH;
}

template <int F>
int launch_heads(const float* obs, int B, int NE, int heads, const float* W, int A, float* Q, const Explore& ex,
                 hipStream_t st) {
  switch (heads) {
    case 1: return launch<F, 1>(obs, B, NE, W, A, Q, ex, st);
    case 2: return launch<F, 2>(obs, B, NE, W, A, Q, ex, st);
    case 4: return launch<F, 4>(obs, B, NE, W, A, Q, ex, st);
    case 8: return launch<F, 8>(obs, B, NE, W, A, Q, ex, st);
    default: return TTRL_E_ARG;
  }
}

int forward(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features, int32_t heads,
            const float* weights, int32_t n_actions, float* q, const Explore& ex, void* stream) {
  if (!obs || !weights || !q || batch < 0 || n_entities < 2 || n_entities > 32 || n_actions < 1 ||
      n_actions > 16 || (heads != 1 && heads != 2 && heads != 4 && heads != 8) || heads * n_entities > 64)
    return TTRL_E_ARG;
  if (batch == 0) return TTRL_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (n_features) {
    case 5: return launch_heads<5>(obs, batch, n_entities, heads, weights, n_actions, q, ex, st);
    case 7: return launch_heads<7>(obs, batch, n_entities, heads, weights, n_actions, q, ex, st);
    case 8: return launch_heads<8>(obs, batch, n_entities, heads, weights, n_actions, q, ex, st);
    default: return TTRL_E_UNSUPPORTED;
  }
}

}  // namespace

extern "C" {

int64_t ttrl_ego_attention_sizes(int32_t n_features, int32_t n_actions, int32_t batch, int32_t n_entities,
                                 int64_t* scratch_floats) {
  if (n_features < 1 || n_features > 16 || n_actions < 1 || n_actions > 16) return TTRL_E_ARG;
  if (scratch_floats) *scratch_floats = 1;  // the fused kernel keeps every activation on chip
  return policy_layout(n_features, n_actions).total;
}

int ttrl_ego_attention_q(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features, int32_t heads,
                         const float* weights, int32_t n_actions, float* scratch, float* q, void* stream) {
  if (!scratch) return TTRL_E_ARG;
  return forward(obs, batch, n_entities, n_features, heads, weights, n_actions, q, Explore{}, stream);
}

int ttrl_ego_attention_act(const float* obs, int32_t batch, int32_t n_entities, int32_t n_features, int32_t heads,
                           const float* weights, int32_t n_actions, float epsilon, const float* epsilon_dev,
                           uint64_t seed, int64_t step, const int64_t* step_dev, int64_t env_offset, float* q,
                           int64_t* actions, int32_t* actions32, void* stream) {
  if ((!actions && !actions32) || !(epsilon >= 0.0f && epsilon <= 1.0f) || env_offset < 0) return TTRL_E_ARG;
  Explore ex{};
  ex.env_offset = env_offset;
  ex.act = actions; ex.act32 = actions32;
  ex.eps = epsilon; ex.eps_dev = epsilon_dev; ex.step = step; ex.step_dev = step_dev;
  ex.seed_lo = (unsigned)seed; ex.seed_hi = (unsigned)(seed >> 32);
  return forward(obs, batch, n_entities, n_features, heads, weights, n_actions, q, ex, stream);
}

#ifdef TTRL_POL_CLOCKS
int ttrl_diag_policy_clocks(long long* out, int32_t n) {
  if (n > POL_CLK_BLOCKS * 9) n = POL_CLK_BLOCKS * 9;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pol_clk), n * sizeof(long long)) == hipSuccess ? TTRL_OK
                                                                                              : TTRL_E_LAUNCH;
}
#endif

}  // extern "C"
