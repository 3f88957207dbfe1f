// GEMM lab: the production 256x256 ping-pong kernel (csrc/gemm_bf16.hip tiles pp / ppp, the round-5 tile
// order, and the ablations: no staging / MFMAs only / no MFMAs) timed in one process at a set of shapes.
// pp is checked against a naive fp32-accumulate reference; ppp and the round-5 order are screened for races
// (their outputs over 20 repeated launches must stay bit-identical to pp's).
//
//   hipcc --offload-arch=gfx950 -O3 -Icsrc -o tools/ubench/gemm_lab.bin tools/ubench/gemm_lab.hip
//   tools/ubench/gemm_lab.bin
#include "../../csrc/gemm_bf16.hip"
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(size_t)m * K + k]) * bf2f(B[(size_t)n * K + k]);
  C[(size_t)m * N + n] = fmaxf(s, 0.f);
}

static unsigned short host_bf(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}
static float host_f(unsigned short h) {
  unsigned u = (unsigned)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

typedef hipError_t (*launch_t)(const st::GemmArgs&, hipStream_t);

int main(int argc, char** argv) {
  const int shapes[][3] = {{16384, 1024, 1024}, {16384, 1024, 4096}, {8192, 8192, 8192}, {4096, 4096, 4096},
                           {8192, 4096, 1024}, {4096, 1024, 1024}};
  // "pmc V": only variant V at the act step's shape, 20 launches, no checks (one kernel for rocprofv3 --pmc)
  if (argc > 2 && std::strcmp(argv[1], "pmc") == 0) {
    const int v = std::atoi(argv[2]);
    launch_t f[] = {st::launch_gemm_pp<st::EPI_BF16, 0>, st::launch_gemm_pp<st::EPI_BF16, 0, 1>,
                    st::launch_gemm_pp<st::EPI_BF16, 0, 2>, st::launch_gemm_pp<st::EPI_BF16, 0, 3>};
    const int M = 16384, N = 1024, K = 1024;
    bf16_t *A, *B, *C;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMemset(A, 0x3c, (size_t)M * K * 2));   // 0x3c3c: a small positive bf16 everywhere
    CK(hipMemset(B, 0x3c, (size_t)N * K * 2));
    st::GemmArgs a{};
    a.A = A; a.B = B; a.out = C; a.M = M; a.N = N; a.K = K; a.lda = K; a.ldb = K; a.ldo = N;
    a.relu = 1; a.alpha = 1.f; a.splitk = 1;
    for (int i = 0; i < 20; ++i) CK(f[v](a, nullptr));
    CK(hipDeviceSynchronize());
    std::printf("pmc variant %d done\n", v);
    return 0;
  }
  const char* names[] = {"pp", "ppp", "pp-rowmajor", "pp-nostage", "pp-mfma-only", "pp-no-mfma"};
  launch_t fns[] = {st::launch_gemm_pp<st::EPI_BF16, 0>, st::launch_gemm_pp<st::EPI_BF16, 1>,
                    st::launch_gemm_pp<st::EPI_BF16, 0, 0, 0>, st::launch_gemm_pp<st::EPI_BF16, 0, 1>,
                    st::launch_gemm_pp<st::EPI_BF16, 0, 2>, st::launch_gemm_pp<st::EPI_BF16, 0, 3>};
  constexpr int NV = 6, NCHECK = 3;   // the ablations (wrong results by design) are timed only
  int bad = 0;
  for (const auto& sh : shapes) {
    const int M = sh[0], N = sh[1], K = sh[2];
    std::vector<unsigned short> hA((size_t)M * K), hB((size_t)N * K);
    unsigned s = 12345u;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (float)(s >> 8) / 16777216.f * 2.f - 1.f; };
    for (auto& x : hA) x = host_bf(rnd());
    for (auto& x : hB) x = host_bf(rnd() * 0.05f);
    bf16_t *A, *B, *C, *C0;
    float* R;
    CK(hipMalloc(&A, hA.size() * 2));
    CK(hipMalloc(&B, hB.size() * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&C0, (size_t)M * N * 2));
    CK(hipMalloc(&R, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
    st::GemmArgs a{};
    a.A = A; a.B = B; a.M = M; a.N = N; a.K = K; a.lda = K; a.ldb = K; a.ldo = N;
    a.relu = 1; a.alpha = 1.f; a.splitk = 1;
    // reference (fp32 accumulate) vs pp, then every variant bit-identical to pp over repeated launches
    ref_kernel<<<dim3((N + 255) / 256, M), 256>>>(A, B, R, M, N, K);
    a.out = C0;
    CK(fns[0](a, nullptr));
    CK(hipDeviceSynchronize());
    std::vector<unsigned short> hC((size_t)M * N), h0((size_t)M * N);
    std::vector<float> hR((size_t)M * N);
    CK(hipMemcpy(h0.data(), C0, h0.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hR.data(), R, hR.size() * 4, hipMemcpyDeviceToHost));
    double maxerr = 0.0;
    for (size_t i = 0; i < h0.size(); ++i) maxerr = std::fmax(maxerr, std::fabs(host_f(h0[i]) - hR[i]));
    std::printf("%dx%dx%d  pp max |C - ref| = %.4g\n", M, N, K, maxerr);
    if (maxerr > 0.05) bad = 1;
    a.out = C;
    for (int v = 0; v < NV; ++v) {
      int mism = 0;
      for (int r = 0; r < (v < NCHECK ? 20 : 0); ++r) {
        CK(hipMemset(C, 0xFF, (size_t)M * N * 2));
        CK(fns[v](a, nullptr));
        CK(hipMemcpy(hC.data(), C, hC.size() * 2, hipMemcpyDeviceToHost));
        if (std::memcmp(hC.data(), h0.data(), hC.size() * 2)) ++mism;
      }
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      for (int i = 0; i < 5; ++i) CK(fns[v](a, nullptr));
      const int iters = K >= 4096 ? 20 : 50;
      CK(hipEventRecord(e0, nullptr));
      for (int i = 0; i < iters; ++i) CK(fns[v](a, nullptr));
      CK(hipEventRecord(e1, nullptr));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      std::printf("  %-5s %8.2f us  %6.0f TF/s  mismatching runs %d/20\n", names[v], us, 2.0 * M * N * K / us / 1e6, mism);
      if (mism) bad = 1;
    }
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(C0)); CK(hipFree(R));
  }
  return bad;
}
