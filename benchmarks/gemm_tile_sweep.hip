// Tile-shape sweep for every layer GEMM of the reference step (built and run on the GPU box):
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I distributed_training_compare_jax_amd/csrc \
//         benchmarks/gemm_tile_sweep.hip -o /tmp/ts && /tmp/ts
// For each shape: the production dispatch (dtc_gemm) and candidate tilings on the two kernel bodies
// of csrc/gemm.hip — register-staged gemm_kernel<BM,BN,64> and the DMA-ring gemm_dma_kernel<BM,BN,NS>
// — with split-K 1/2/4 (split > 1: fp32 slabs + the deterministic slab reduce, timed separately and
// together).  Prints us per call, back to back (L2-warm), median of 5 rounds of 40 reps.
#include "../distributed_training_compare_jax_amd/csrc/gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static float timeit(const std::function<void()>& f, int reps = 40) {
  for (int i = 0; i < 3; ++i) f();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> r;
  for (int round = 0; round < 5; ++round) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    r.push_back(ms * 1e3f / reps);
  }
  std::sort(r.begin(), r.end());
  return r[2];
}

// grid geometry exactly as launch_t computes it
struct Geo { int tm, tn, gm, kps, nb; };
static Geo geo(const GemmArgs& a, int BM, int BN, int split) {
  Geo g;
  g.tm = (a.M + BM - 1) / BM; g.tn = (a.N + BN - 1) / BN;
  const int nt = g.tm * g.tn;
  g.gm = g.tm;
  if (g.tn <= 16) g.gm = std::max(1, std::min(g.tm, (nt / 8 + g.tn - 1) / g.tn));
  const int nk = a.K / 64;
  g.kps = ((nk + split - 1) / split) * 64;
  g.nb = nt * split;
  return g;
}
static Epi mkepi(const GemmArgs& a, int tn) {
  Epi e;
  e.M = a.M; e.N = a.N; e.C = a.C; e.ldc = a.ldc; e.bias = a.bias; e.aux = a.aux; e.ldaux = a.ldaux;
  e.aux_out = a.aux_out; e.alpha = a.alpha; e.beta = a.beta; e.labels = a.labels; e.vocab_start = a.vocab_start;
  e.n_valid = a.n_valid; e.part = a.part; e.label_out = a.label_out; e.colsum = nullptr; e.nparts = tn * 2;
  return e;
}

template <int BM, int BN, bool AK, bool BKM, int EPI, bool F32>
void run_reg(const GemmArgs& a, int split) {
  Geo g = geo(a, BM, BN, split);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, 64, AK, BKM, EPI, F32>), dim3(g.nb), dim3(NT), 0, 0, (const bf16*)a.A, a.lda,
                     operand_bytes(AK, a.M, a.K, a.lda), (const bf16*)a.B, a.ldb, operand_bytes(BKM, a.N, a.K, a.ldb),
                     a.M, a.N, a.K, g.tm, g.tn, g.gm, split, g.kps, (float*)a.workspace, mkepi(a, g.tn));
}
template <int BM, int BN, int NS, bool AK, bool BKM, int EPI, bool F32>
void run_dma(const GemmArgs& a, int split) {
  Geo g = geo(a, BM, BN, split);
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, NS, AK, BKM, EPI, F32>), dim3(g.nb), dim3(NT), 0, 0, (const bf16*)a.A,
                     a.lda, (const bf16*)a.B, a.ldb, a.M, a.N, a.K, g.tm, g.tn, g.gm, split, g.kps,
                     (float*)a.workspace, mkepi(a, g.tn));
}
static void run_reduce(const GemmArgs& a, int split) {
  long MN = (long)a.M * a.N;
  hipLaunchKernelGGL(splitk_reduce, dim3((int)((MN / 4 + 255) / 256)), dim3(256), 0, 0, (const float*)a.workspace,
                     split, MN, (float*)a.C, a.ldc, a.N, 0.f);
}

struct Variant { std::string name; std::function<void(const GemmArgs&, int)> fn; };

template <bool AK, bool BKM, int EPI, bool F32>
std::vector<Variant> variants() {
  return {
      {"reg 128x128", run_reg<128, 128, AK, BKM, EPI, F32>},
      {"reg  64x64 ", run_reg<64, 64, AK, BKM, EPI, F32>},
      {"reg 128x64 ", run_reg<128, 64, AK, BKM, EPI, F32>},
      {"reg  64x128", run_reg<64, 128, AK, BKM, EPI, F32>},
      {"dma  64x64 s4", run_dma<64, 64, 4, AK, BKM, EPI, F32>},
      {"dma 128x128 s2", run_dma<128, 128, 2, AK, BKM, EPI, F32>},
      {"dma 128x128 s3", run_dma<128, 128, 3, AK, BKM, EPI, F32>},
      {"dma 128x64 s3", run_dma<128, 64, 3, AK, BKM, EPI, F32>},
      {"dma  64x128 s3", run_dma<64, 128, 3, AK, BKM, EPI, F32>},
      {"dma 256x128 s2", run_dma<256, 128, 2, AK, BKM, EPI, F32>},
      {"dma 256x128 s3", run_dma<256, 128, 3, AK, BKM, EPI, F32>},
      {"dma 128x256 s2", run_dma<128, 256, 2, AK, BKM, EPI, F32>},
  };
}

int main() {
  const int M = 4096, KMAX = 4096, NMAX = 2048;
  std::vector<uint16_t> h((size_t)M * KMAX);
  uint32_t x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; float f = ((x >> 9) & 0xFFFF) / 65536.f - 0.5f; uint32_t u; memcpy(&u, &f, 4); v = u >> 16; }
  bf16 *A, *B, *C2, *U; float *C, *bias, *R, *WS;
  CK(hipMalloc(&A, (size_t)M * KMAX * 2)); CK(hipMalloc(&B, (size_t)M * KMAX * 2));
  CK(hipMalloc(&C, (size_t)M * NMAX * 4)); CK(hipMalloc(&C2, (size_t)M * NMAX * 2)); CK(hipMalloc(&U, (size_t)M * NMAX * 2));
  CK(hipMalloc(&bias, NMAX * 4)); CK(hipMalloc(&R, (size_t)M * NMAX * 4));
  CK(hipMalloc(&WS, (size_t)8 * M * NMAX * 4));
  CK(hipMemcpy(A, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), (size_t)M * KMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(U, h.data(), (size_t)M * NMAX * 2, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, NMAX * 4)); CK(hipMemset(R, 0, (size_t)M * NMAX * 4));

  struct Shape { const char* name; int layout, M, N, K, epi, f32; };
  const Shape shapes[] = {
      {"fwd   qkv ", 0, M, 1536, 512, EPI_STORE, 0}, {"fwd   fc1 ", 0, M, 2048, 512, EPI_GELU, 0},
      {"fwd   out ", 0, M, 512, 512, EPI_RESID, 1},  {"fwd   fc2 ", 0, M, 512, 2048, EPI_RESID, 1},
      {"dgrad qkv ", 1, M, 512, 1536, EPI_STORE, 1}, {"dgrad out ", 1, M, 512, 512, EPI_STORE, 0},
      {"dgrad fc1 ", 1, M, 512, 2048, EPI_STORE, 1}, {"dgrad fc2 ", 1, M, 2048, 512, EPI_DGELU, 0},
      {"wgrad qkv ", 2, 1536, 512, M, EPI_STORE, 1}, {"wgrad out ", 2, 512, 512, M, EPI_STORE, 1},
      {"wgrad fc1 ", 2, 2048, 512, M, EPI_STORE, 1}, {"wgrad fc2 ", 2, 512, 2048, M, EPI_STORE, 1},
  };
  for (const Shape& s : shapes) {
    GemmArgs a{};
    a.layout = s.layout; a.M = s.M; a.N = s.N; a.K = s.K;
    // operands: K-major [rows][K] (ld = K) or MN-major [K][rows] (ld = rows)
    const bool ak = s.layout != 2, bk = s.layout == 0;
    a.A = A; a.lda = ak ? s.K : s.M;
    a.B = B; a.ldb = bk ? s.K : s.N;
    a.C = s.f32 ? (void*)C : (void*)C2; a.ldc = s.N; a.c_f32 = s.f32; a.epi = s.epi; a.alpha = 1.f;
    a.bias = s.layout == 0 ? bias : nullptr;
    if (s.epi == EPI_RESID) { a.aux = R; a.ldaux = s.N; }
    if (s.epi == EPI_DGELU) { a.aux = U; a.ldaux = s.N; }
    if (s.epi == EPI_GELU) a.aux_out = U;
    a.workspace = WS; a.ws_bytes = (long)8 * M * NMAX * 4;
    const double fl = 2.0 * s.M * s.N * s.K;
    GemmArgs ap = a;
    if (s.layout == 2) ap.defer_reduce = 0;
    float tp = timeit([&] { dtc_gemm(&ap, 0); });
    printf("%s [%5d x %5d x %5d] production %7.2f us (%6.1f TF/s)\n", s.name, s.M, s.N, s.K, tp, fl / tp * 1e-6);
    std::vector<Variant> vs;
    if (s.layout == 0 && s.epi == EPI_STORE) vs = variants<true, true, EPI_STORE, false>();
    if (s.layout == 0 && s.epi == EPI_GELU) vs = variants<true, true, EPI_GELU, false>();
    if (s.layout == 0 && s.epi == EPI_RESID) vs = variants<true, true, EPI_RESID, true>();
    if (s.layout == 1 && s.epi == EPI_STORE && s.f32) vs = variants<true, false, EPI_STORE, true>();
    if (s.layout == 1 && s.epi == EPI_STORE && !s.f32) vs = variants<true, false, EPI_STORE, false>();
    if (s.layout == 1 && s.epi == EPI_DGELU) vs = variants<true, false, EPI_DGELU, false>();
    if (s.layout == 2) vs = variants<false, false, EPI_STORE, true>();
    for (auto& v : vs) {
      for (int split : {1, 2, 4, 8}) {
        const int nk = s.K / 64;
        if (nk / split < 2) continue;
        if (split > 1 && !s.f32 && s.layout != 2 && s.epi != EPI_RESID) continue;  // bf16 outputs: whole-K only
        Geo g = geo(a, 128, 128, 1);
        (void)g;
        float t = timeit([&] { v.fn(a, split); });
        float tr = split > 1 ? timeit([&] { run_reduce(a, split); }) : 0.f;
        printf("    %-15s split %d: %7.2f us%s", v.name.c_str(), split, t, split > 1 ? "" : "\n");
        if (split > 1) printf(" + reduce %6.2f = %7.2f us\n", tr, t + tr);
      }
    }
    fflush(stdout);
  }
  return 0;
}
