// vit_micro.hip — DIAGNOSTIC: the Viterbi decoder (viterbi_dev.h) alone on
// random soft symbols, one wave per codeword, at several grid sizes, to tell
// a per-wave latency bound (time flat in the wave count up to the resident
// limit) from a throughput bound (time proportional to waves per SIMD).
// Prints one line per grid: waves, ms, cycles per trellis step per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../aero-cli_amd/csrc/viterbi_dev.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("hip %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int NSOFT = 62 + 4992 + 24;

__global__ __launch_bounds__(64) void vit(const uint8_t *soft, uint64_t *out, unsigned long long *cyc, int reps) {
  __shared__ uint8_t sbuf[NSOFT + 2];
  const int lane = threadIdx.x;
  const uint8_t *src = soft + (size_t)blockIdx.x * NSOFT;
  for (int i = lane; i < NSOFT; i += 64) sbuf[i] = src[i];
  __syncthreads();
  uint64_t acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
    uint64_t obw;
    aero::viterbi_decode_regs(sbuf, NSOFT, obw, lane);
    acc ^= obw;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[(size_t)blockIdx.x * 64 + lane] = acc;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 1;
  const int maxw = 65536;
  std::vector<uint8_t> h((size_t)maxw * NSOFT);
  srand(7);
  for (auto &v : h) v = (uint8_t)(rand() & 255);
  uint8_t *d;
  uint64_t *o;
  unsigned long long *cy;
  CK(hipMalloc(&d, h.size()));
  CK(hipMalloc(&o, (size_t)maxw * 64 * 8));
  CK(hipMalloc(&cy, (size_t)maxw * 8));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grids[] = {256, 1024, 2048, 4096, 6144, 8192, 12288, 16384, 32768};
  std::vector<unsigned long long> hc(maxw);
  for (int g : grids) {
    hipLaunchKernelGGL(vit, dim3(g), dim3(64), 0, 0, d, o, cy, reps);  // warm
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(vit, dim3(g), dim3(64), 0, 0, d, o, cy, reps);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipMemcpy(hc.data(), cy, (size_t)g * 8, hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < g; ++i) s += (double)hc[i];
    const double steps = (double)reps * (NSOFT / 2);
    printf("{\"waves\": %d, \"ms\": %.4f, \"wave_cycles_per_step\": %.1f, \"ns_per_wave_step_chip\": %.4f}\n", g, ms,
           s / g / steps, ms * 1e6 / (g * steps));
  }
  return 0;
}
