// Phase timing of the LDS-resident attention forward (reference shape B8 T512 H16 hd32):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 benchmarks/attn_phase_micro.hip -o /tmp/ap && /tmp/ap
// Variants: full kernel, staging only, staging + QK^T/PV MFMAs without softmax transcendentals.
#include "../distributed_training_compare_jax_amd/csrc/attention.hip"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace {
template <int MODE>  // 0: stage only, 1: stage + MFMAs (no exp), 2: stage + one 64-key tile per wave
__global__ void __launch_bounds__(RES_THREADS) fwd_variant(const bf16* __restrict__ qkv, bf16* __restrict__ o, int B,
                                                          int T, int H, float scale) {
  constexpr int HD = 32, KC = 1, HT = 2;
  using L = AttnLds<HD>;
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, j = lane & 15;
  const int half = blockIdx.x & 1, bh = blockIdx.x >> 1, b = bh / H, h = bh % H;
  const int Tp = (T + 63) / 64 * 64;
  bf16* sK = lds;
  bf16* sV = lds + Tp * L::KLD;
  const long ts = 3L * H * HD;
  const bf16* Qb = qkv + (long)b * T * ts + (0 * H + h) * HD;
  const bf16* Kb = qkv + (long)b * T * ts + (1 * H + h) * HD;
  const bf16* Vb = qkv + (long)b * T * ts + (2 * H + h) * HD;
  stage_rows<L::KLD, HD, RES_MAXT>(sK, Kb, ts, T, Tp, tid);
  stage_rows<L::VLD, HD, RES_MAXT>(sV, Vb, ts, T, Tp, tid);
  __syncthreads();
  const int qg = 2 * w + half;
  const int q = qg * 16 + j;
  bf16x8 qf = *(const bf16x8*)(Qb + (long)q * ts + 8 * g);
  f32x4 acc[HT] = {};
  const int ntile = MODE == 2 ? 1 : (MODE == 0 ? 0 : (qg * 16 + 16 + 63) / 64);
  for (int kt = 0; kt < ntile; ++kt) {
    const bf16* tK = sK + kt * 64 * L::KLD;
    const bf16* tV = sV + kt * 64 * L::VLD;
    f32x4 sc[4];
    for (int st = 0; st < 4; ++st) sc[st] = mfma(row_frag(tK, L::KLD, st * 16, 0, lane), qf, f32x4{0.f, 0.f, 0.f, 0.f});
    const bf16x8 pf0 = pack_p(sc[0], sc[1]), pf1 = pack_p(sc[2], sc[3]);
    for (int t = 0; t < HT; ++t) {
      acc[t] = mfma(tr_frag(tV, L::VLD, 0, t * 16, lane), pf0, acc[t]);
      acc[t] = mfma(tr_frag(tV, L::VLD, 32, t * 16, lane), pf1, acc[t]);
    }
  }
  bf16* orow = o + ((long)b * T + q) * H * HD + h * HD;
  for (int t = 0; t < HT; ++t) *(bf16x4*)(orow + t * 16 + 4 * g) = bf16x4{f2bf(acc[t][0]), f2bf(acc[t][1]), f2bf(acc[t][2]), f2bf(acc[t][3])};
}
}  // namespace

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

int main() {
  const int B = 8, T = 512, H = 16, HD = 32;
  bf16 *qkv, *o; float* lse;
  CK(hipMalloc(&qkv, (size_t)B * T * 3 * H * HD * 2)); CK(hipMalloc(&o, (size_t)B * T * H * HD * 2));
  CK(hipMalloc(&lse, (size_t)B * H * T * 4));
  std::vector<uint16_t> hbuf((size_t)B * T * 3 * H * HD, 0x3c00);
  CK(hipMemcpy(qkv, hbuf.data(), hbuf.size() * 2, hipMemcpyHostToDevice));
  const long lds = res_lds_fwd(T, HD);
  allow_lds(attn_fwd_res_kernel<32>, lds);
  allow_lds(fwd_variant<0>, lds); allow_lds(fwd_variant<1>, lds); allow_lds(fwd_variant<2>, lds);
  const float sc = 0.17f;
  dim3 grid(B * H * 2), blk(RES_THREADS);
  float t_full = timeit([&] { hipLaunchKernelGGL(attn_fwd_res_kernel<32>, grid, blk, lds, 0, qkv, o, lse, B, T, H, sc); }, 50);
  float t0 = timeit([&] { hipLaunchKernelGGL(fwd_variant<0>, grid, blk, lds, 0, qkv, o, B, T, H, sc); }, 50);
  float t1 = timeit([&] { hipLaunchKernelGGL(fwd_variant<1>, grid, blk, lds, 0, qkv, o, B, T, H, sc); }, 50);
  float t2 = timeit([&] { hipLaunchKernelGGL(fwd_variant<2>, grid, blk, lds, 0, qkv, o, B, T, H, sc); }, 50);
  printf("full %.1f us | stage only %.1f | stage+1 tile %.1f | stage+MFMA (no softmax) %.1f\n", t_full, t0, t2, t1);
  return 0;
}
