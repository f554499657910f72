// Experiment: decoder skinny GEMM (M = 24 rows) weight layouts. Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/gemv_bench.hip -o /tmp/gemv_bench && /tmp/gemv_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

// V1: row-major W [N][K]; block = 4 waves = 16 cols, K split over waves (the product kernel's structure)
__global__ __launch_bounds__(256) void v1(const bf16_t* A, const bf16_t* W, int M, int N, int K, float* out) {
  __shared__ float red[4][32][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n0 = blockIdx.x * 16, ns = K >> 5, s0 = wid * ns / 4, s1 = (wid + 1) * ns / 4;
  const int col = min(n0 + (lane & 15), N - 1), ksub = 8 * (lane >> 4);
  const bf16_t* wp = W + (size_t)col * K + ksub;
  const bf16_t* ap0 = A + (size_t)min(lane & 15, M - 1) * K + ksub;
  const bf16_t* ap1 = A + (size_t)min(16 + (lane & 15), M - 1) * K + ksub;
  f32x4 c0 = {0}, c1 = {0};
  int s = s0;
  for (; s + 8 <= s1; s += 8) {
    bf16x8 bw[8], a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { bw[u] = *(const bf16x8*)(wp + 32 * (s + u)); a0[u] = *(const bf16x8*)(ap0 + 32 * (s + u)); a1[u] = *(const bf16x8*)(ap1 + 32 * (s + u)); }
#pragma unroll
    for (int u = 0; u < 8; ++u) { c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0); }
  }
  for (; s < s1; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 32 * s), a0 = *(const bf16x8*)(ap0 + 32 * s), a1 = *(const bf16x8*)(ap1 + 32 * s);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  for (int r = 0; r < 4; ++r) { red[wid][rb + r][cc] = c0[r]; red[wid][16 + rb + r][cc] = c1[r]; }
  __syncthreads();
  for (int e = tid; e < 32 * 16; e += 256) {
    int m = e >> 4, c = e & 15, n = n0 + c;
    if (m < M && n < N) out[(size_t)m * N + n] = red[0][m][c] + red[1][m][c] + red[2][m][c] + red[3][m][c];
  }
}

// packed W: [N/16][K/32][64 lanes][8]: the (col group, step) fragment is 1 KB contiguous.
// packed A: [K/32][2][64][8]: the 2 m-tile fragments of a step are 2 KB contiguous.
// V2: block = 4 waves = 16 cols, K split over waves
__global__ __launch_bounds__(256) void v2(const bf16_t* Ap, const bf16_t* Wp, int M, int N, int K, float* out) {
  __shared__ float red[4][32][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.x, n0 = g * 16, ns = K >> 5, s0 = wid * ns / 4, s1 = (wid + 1) * ns / 4;
  const bf16_t* wp = Wp + ((size_t)g * ns) * 512 + lane * 8;
  const bf16_t* ap = Ap + lane * 8;
  f32x4 c0 = {0}, c1 = {0};
  int s = s0;
  for (; s + 8 <= s1; s += 8) {
    bf16x8 bw[8], a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { bw[u] = *(const bf16x8*)(wp + 512 * (s + u)); a0[u] = *(const bf16x8*)(ap + 1024 * (s + u)); a1[u] = *(const bf16x8*)(ap + 1024 * (s + u) + 512); }
#pragma unroll
    for (int u = 0; u < 8; ++u) { c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0); }
  }
  for (; s < s1; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 512 * s), a0 = *(const bf16x8*)(ap + 1024 * s), a1 = *(const bf16x8*)(ap + 1024 * s + 512);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  for (int r = 0; r < 4; ++r) { red[wid][rb + r][cc] = c0[r]; red[wid][16 + rb + r][cc] = c1[r]; }
  __syncthreads();
  for (int e = tid; e < 32 * 16; e += 256) {
    int m = e >> 4, c = e & 15, n = n0 + c;
    if (m < M && n < N) out[(size_t)m * N + n] = red[0][m][c] + red[1][m][c] + red[2][m][c] + red[3][m][c];
  }
}

// V3: packed; one wave = one 16-col group, full K (no cross-wave reduction); block = 4 waves = 4 groups
template <int UNR>
__global__ __launch_bounds__(256) void v3(const bf16_t* Ap, const bf16_t* Wp, int M, int N, int K, float* out) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.x * 4 + wid, ns = K >> 5;
  if (g * 16 >= N) return;
  const bf16_t* wp = Wp + ((size_t)g * ns) * 512 + lane * 8;
  const bf16_t* ap = Ap + lane * 8;
  f32x4 c0 = {0}, c1 = {0};
  int s = 0;
  for (; s + UNR <= ns; s += UNR) {
    bf16x8 bw[UNR], a0[UNR], a1[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) { bw[u] = *(const bf16x8*)(wp + 512 * (s + u)); a0[u] = *(const bf16x8*)(ap + 1024 * (s + u)); a1[u] = *(const bf16x8*)(ap + 1024 * (s + u) + 512); }
#pragma unroll
    for (int u = 0; u < UNR; ++u) { c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0); }
  }
  for (; s < ns; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 512 * s), a0 = *(const bf16x8*)(ap + 1024 * s), a1 = *(const bf16x8*)(ap + 1024 * s + 512);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
  }
  const int n = g * 16 + (lane & 15), rb = (lane >> 4) * 4;
  if (n < N)
    for (int r = 0; r < 4; ++r) {
      if (rb + r < M) out[(size_t)(rb + r) * N + n] = c0[r];
      if (16 + rb + r < M) out[(size_t)(16 + rb + r) * N + n] = c1[r];
    }
}

// V4: packed, W-only stream test (A from LDS: one block stages the 2 KB/step A fragments once) -- split K in-wave
// groups: block = 4 waves, each wave its own 16-col group, full K; A fragments read from LDS (staged once per block)
__global__ __launch_bounds__(256) void v4(const bf16_t* Ap, const bf16_t* Wp, int M, int N, int K, float* out) {
  extern __shared__ __attribute__((aligned(16))) bf16_t asm_[];  // [ns][2][64][8]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ns = K >> 5;
  for (int i = tid; i < ns * 128; i += 256) ((uint4*)asm_)[i] = ((const uint4*)Ap)[i];
  __syncthreads();
  const int g = blockIdx.x * 4 + wid;
  if (g * 16 >= N) return;
  const bf16_t* wp = Wp + ((size_t)g * ns) * 512 + lane * 8;
  f32x4 c0 = {0}, c1 = {0};
  int s = 0;
  for (; s + 8 <= ns; s += 8) {
    bf16x8 bw[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) bw[u] = *(const bf16x8*)(wp + 512 * (s + u));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      bf16x8 a0 = *(const bf16x8*)(asm_ + 1024 * (s + u) + lane * 8), a1 = *(const bf16x8*)(asm_ + 1024 * (s + u) + 512 + lane * 8);
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw[u], c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw[u], c1, 0, 0, 0);
    }
  }
  for (; s < ns; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 512 * s);
    bf16x8 a0 = *(const bf16x8*)(asm_ + 1024 * s + lane * 8), a1 = *(const bf16x8*)(asm_ + 1024 * s + 512 + lane * 8);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
  }
  const int n = g * 16 + (lane & 15), rb = (lane >> 4) * 4;
  if (n < N)
    for (int r = 0; r < 4; ++r) {
      if (rb + r < M) out[(size_t)(rb + r) * N + n] = c0[r];
      if (16 + rb + r < M) out[(size_t)(16 + rb + r) * N + n] = c1[r];
    }
}


// V5: packed W, row-major A [M][K] (as the decoder's LN / attention kernels write it); split-K over 4 waves
__global__ __launch_bounds__(256) void v5(const bf16_t* A, const bf16_t* Wp, int M, int N, int K, float* out) {
  __shared__ float red[4][32][17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.x, n0 = g * 16, ns = K >> 5, s0 = wid * ns / 4, s1 = (wid + 1) * ns / 4;
  const bf16_t* wp = Wp + ((size_t)g * ns) * 512 + lane * 8;
  const int ksub = 8 * (lane >> 4);
  const bf16_t* ap0 = A + (size_t)min(lane & 15, M - 1) * K + ksub;
  const bf16_t* ap1 = A + (size_t)min(16 + (lane & 15), M - 1) * K + ksub;
  f32x4 c0 = {0}, c1 = {0};
  int s = s0;
  for (; s + 8 <= s1; s += 8) {
    bf16x8 bw[8], a0[8], a1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { bw[u] = *(const bf16x8*)(wp + 512 * (s + u)); a0[u] = *(const bf16x8*)(ap0 + 32 * (s + u)); a1[u] = *(const bf16x8*)(ap1 + 32 * (s + u)); }
#pragma unroll
    for (int u = 0; u < 8; ++u) { c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[u], bw[u], c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[u], bw[u], c1, 0, 0, 0); }
  }
  for (; s < s1; ++s) {
    bf16x8 bw = *(const bf16x8*)(wp + 512 * s), a0 = *(const bf16x8*)(ap0 + 32 * s), a1 = *(const bf16x8*)(ap1 + 32 * s);
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, c0, 0, 0, 0); c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bw, c1, 0, 0, 0);
  }
  const int cc = lane & 15, rb = (lane >> 4) * 4;
  for (int r = 0; r < 4; ++r) { red[wid][rb + r][cc] = c0[r]; red[wid][16 + rb + r][cc] = c1[r]; }
  __syncthreads();
  for (int e = tid; e < 32 * 16; e += 256) {
    int m = e >> 4, c = e & 15, n = n0 + c;
    if (m < M && n < N) out[(size_t)m * N + n] = red[0][m][c] + red[1][m][c] + red[2][m][c] + red[3][m][c];
  }
}

template <typename F>
float time_graph(F launch, hipStream_t s, int n) {
  hipGraph_t g; hipGraphExec_t ge;
  launch(); CK(hipStreamSynchronize(s));
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < n; ++i) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s)); CK(hipStreamSynchronize(s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, s)); CK(hipGraphLaunch(ge, s)); CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); best = std::min(best, ms * 1000.f / n);
  }
  return best;
}

int main() {
  const int M = 24;
  struct Sh { const char* name; int N, K; } shapes[] = {{"lm_head", 51872, 1280}, {"fc1", 5120, 1280}, {"fc2", 1280, 5120}, {"qkv", 3840, 1280}, {"o", 1280, 1280}};
  hipStream_t s; CK(hipStreamCreate(&s));
  // a large buffer to flush caches between shapes: weights are streamed from HBM in the decoder (4 layers x 85 MB + 133 MB)
  for (auto sh : shapes) {
    const int N = sh.N, K = sh.K;
    // several weight copies so that back-to-back launches stream from HBM, not the 256 MB Infinity Cache
    const int copies = std::max(1, (int)(600e6 / ((double)N * K * 2)));
    size_t wn = (size_t)N * K;
    std::vector<bf16_t> h(wn);
    for (size_t i = 0; i < wn; ++i) h[i] = (bf16_t)(0x3c00 + (i * 2654435761u >> 20) % 256);
    bf16_t *W, *Wp, *A, *Ap; float* out;
    CK(hipMalloc(&W, wn * 2 * copies)); CK(hipMalloc(&Wp, wn * 2 * copies));
    for (int c = 0; c < copies; ++c) { CK(hipMemcpy(W + c * wn, h.data(), wn * 2, hipMemcpyHostToDevice)); CK(hipMemcpy(Wp + c * wn, h.data(), wn * 2, hipMemcpyHostToDevice)); }
    CK(hipMalloc(&A, (size_t)32 * K * 2)); CK(hipMalloc(&Ap, (size_t)32 * K * 2)); CK(hipMemset(A, 0x3c, 32 * K * 2)); CK(hipMemset(Ap, 0x3c, 32 * K * 2));
    CK(hipMalloc(&out, (size_t)M * N * 4));
    int it = 0;
    auto L1 = [&]() { hipLaunchKernelGGL(v1, dim3(N / 16), dim3(256), 0, s, A, W + (size_t)(it++ % copies) * wn, M, N, K, out); };
    auto L2 = [&]() { hipLaunchKernelGGL(v2, dim3(N / 16), dim3(256), 0, s, Ap, Wp + (size_t)(it++ % copies) * wn, M, N, K, out); };
    auto L3 = [&]() { hipLaunchKernelGGL(v3<8>, dim3((N / 16 + 3) / 4), dim3(256), 0, s, Ap, Wp + (size_t)(it++ % copies) * wn, M, N, K, out); };
    auto L3b = [&]() { hipLaunchKernelGGL(v3<16>, dim3((N / 16 + 3) / 4), dim3(256), 0, s, Ap, Wp + (size_t)(it++ % copies) * wn, M, N, K, out); };
    auto L5 = [&]() { hipLaunchKernelGGL(v5, dim3(N / 16), dim3(256), 0, s, A, Wp + (size_t)(it++ % copies) * wn, M, N, K, out); };
    auto L4 = [&]() { hipLaunchKernelGGL(v4, dim3((N / 16 + 3) / 4), dim3(256), (K / 32) * 2048, s, Ap, Wp + (size_t)(it++ % copies) * wn, M, N, K, out); };
    const int n = 4 * copies;
    float t1 = time_graph(L1, s, n), t2 = time_graph(L2, s, n), t3 = time_graph(L3, s, n), t3b = time_graph(L3b, s, n), t4 = K <= 2048 ? time_graph(L4, s, n) : 0.f, t5 = time_graph(L5, s, n);
    double gb = wn * 2 / 1e3;
    printf("%-8s N=%6d K=%5d copies=%d | v1 rowmajor %7.2f us %6.0f GB/s | v2 packed splitK %7.2f us %6.0f | v3 packed fullK u8 %7.2f us %6.0f | u16 %7.2f us %6.0f | v4 A in LDS %7.2f us %6.0f | v5 packedW rowA %7.2f us %6.0f\n",
           sh.name, N, K, copies, t1, gb / t1, t2, gb / t2, t3, gb / t3, t3b, gb / t3b, t4, gb / t4, t5, gb / t5);
    CK(hipFree(W)); CK(hipFree(Wp)); CK(hipFree(A)); CK(hipFree(Ap)); CK(hipFree(out));
  }
  return 0;
}
