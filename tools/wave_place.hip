// Probe: where the waves of a 512-thread workgroup land (HW_ID: SIMD and CU
// of each wave), to choose the role split of a two-role kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void probe(unsigned *out) {
  unsigned id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = id;
}

int main() {
  const int nb = 256;
  unsigned *d;
  hipMalloc(&d, nb * 8 * 4);
  hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 40000, 0, d);
  std::vector<unsigned> h(nb * 8);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  int same_pairs = 0, rr = 0;
  for (int b = 0; b < nb; b++) {
    int simd[8];
    for (int w = 0; w < 8; w++) simd[w] = (h[b * 8 + w] >> 4) & 3;
    bool ok = true;
    for (int w = 0; w < 4; w++) ok &= simd[w] == simd[w + 4];
    same_pairs += ok;
    bool r = true;
    for (int w = 0; w < 8; w++) r &= simd[w] == (w & 3);
    rr += r;
    if (b < 4) {
      printf("block %d:", b);
      for (int w = 0; w < 8; w++) printf(" w%d:simd%d,cu%u", w, simd[w], (h[b * 8 + w] >> 8) & 15);
      printf("\n");
    }
  }
  printf("blocks where wave w and w+4 share a SIMD: %d of %d; round-robin w&3: %d\n", same_pairs, nb, rr);
  return 0;
}
