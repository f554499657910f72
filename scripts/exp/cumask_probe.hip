// Experiment (not product code): which physical CUs does a CU-masked stream's kernel land on?
//   hipcc --offload-arch=gfx950 -O2 scripts/exp/cumask_probe.hip -o scripts/exp/cumask_probe && ./scripts/exp/cumask_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <set>
#include <vector>

__global__ void probe(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
    unsigned cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    out[blockIdx.x] = (xcc << 16) | (se << 8) | (sh << 4) | cu;
    // keep the CU busy a little so the dispatcher spreads blocks
    for (volatile int i = 0; i < 2000; i++) {}
  }
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", ncu);
  const int nb = 4096;
  unsigned* d;
  hipMalloc(&d, nb * 4);
  std::vector<unsigned> h(nb);
  int words = (ncu + 31) / 32;
  auto run = [&](std::vector<unsigned> mask, const char* name) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, words, mask.data()) != hipSuccess) { printf("mask fail\n"); return; }
    hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, nb * 4, hipMemcpyDeviceToHost);
    std::set<unsigned> cus, xccs;
    for (unsigned v : h) { cus.insert(v); xccs.insert(v >> 16); }
    printf("%-28s -> %3zu CUs, xccs:", name, cus.size());
    for (unsigned x : xccs) {
      int c = 0;
      for (unsigned v : cus) c += (v >> 16) == x;
      printf(" %u(%d)", x, c);
    }
    printf("\n");
    hipStreamDestroy(s);
  };
  std::vector<unsigned> m(words, 0);
  for (int b = 0; b < 16; b++) {
    std::fill(m.begin(), m.end(), 0);
    m[b / 32] |= 1u << (b % 32);
    char nm[64];
    snprintf(nm, 64, "bit %d", b);
    run(m, nm);
  }
  for (int b : {32, 33, 64, 100, 128, 255}) {
    std::fill(m.begin(), m.end(), 0);
    m[b / 32] |= 1u << (b % 32);
    char nm[64];
    snprintf(nm, 64, "bit %d", b);
    run(m, nm);
  }
  std::fill(m.begin(), m.end(), 0); m[0] = 0xffffffffu; run(m, "word0 all");
  std::fill(m.begin(), m.end(), 0); m[0] = 0xffu; run(m, "bits 0-7");
  std::fill(m.begin(), m.end(), 0); for (int w = 0; w < words; w++) m[w] = 0xffu; run(m, "bits 0-7 of each word");
  std::fill(m.begin(), m.end(), 0); for (int w = 0; w < words; w++) m[w] = 0xffffff00u; run(m, "bits 8-31 of each word");
  std::fill(m.begin(), m.end(), 0); for (int i = 0; i < 64; i++) m[i / 32] |= 1u << (i % 32); run(m, "bits 0-63");
  std::fill(m.begin(), m.end(), 0xffffffffu); run(m, "all");
  return 0;
}
