// mfma_add_probe.hip — can v_mfma_f64_4x4x4_4b_f64 serve as a per-lane FP64
// add whose accumulator stays in an AGPR?  With A the identity of each 4x4
// block, D = A B + C = B + C element by element, and if B and C/D share
// their lane layout every lane gets b + c of its own operands.  The sum holds
// b and three exact zeros besides c, so IEEE rounding of any order gives
// RN(b + c), the same double as v_add_f64.  This probe (1) prints the lane
// maps with the identity guess, (2) compares D with the host's b + c on
// random operands of the demodulator's magnitudes and signs, bit for bit.
// Diagnostic for DESIGN.md §4; not part of the product.
//
// hipcc -O3 --offload-arch=gfx950 tools/mfma_add_probe.hip -o tools/mfma_add_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

// measured lane maps (block b, row i, column j, inner k): A[b][i][k] in lane
// 16k + 4b + i, B[b][k][j] in lane 16k + 4b + j, C/D[b][i][j] in lane
// 16i + 4b + j; so B and D share lanes and the identity has A = 1 where
// i == k, i.e. lane & 3 == lane >> 4
__device__ __forceinline__ double ident(int l) { return (l & 3) == (l >> 4) ? 1.0 : 0.0; }

// mode 0: A = identity guess; 1: A = all ones; 2: A = lane, B = ones
__global__ void map_kernel(double *out, int mode) {
  const int l = threadIdx.x;
  double a = ident(l), b = (double)l, c = 0.0;
  if (mode == 1) a = 1.0;
  if (mode == 2) {
    a = (double)l;
    b = 1.0;
  }
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

__global__ void add_kernel(const double *b, const double *c, double *d, long n) {
  const long base = (long)blockIdx.x * 64 * 16;
  const double a = ident(threadIdx.x);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long i = base + r * 64 + threadIdx.x;
    if (base + r * 64 < n) d[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b[i], c[i], 0, 0, 0);
  }
}

int main() {
  double *dout;
  CK(hipMalloc(&dout, 64 * sizeof(double)));
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(map_kernel, dim3(1), dim3(64), 0, 0, dout, mode);
    double h[64];
    CK(hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost));
    printf("mode %d:", mode);
    for (int l = 0; l < 64; ++l) printf(" %g", h[l]);
    printf("\n");
  }
  const long n = 1L << 24;  // multiple of 1024
  std::vector<double> b(n), c(n), d(n);
  std::mt19937_64 g(12345);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  std::uniform_int_distribution<int> ex(-40, 2);
  for (long i = 0; i < n; ++i) {
    // products tap * pcm/32768 * cis and partial sums of them: mixed signs,
    // magnitudes 2^-40 .. 4, some exact zeros and exact negatives of each other
    b[i] = std::ldexp(u(g), ex(g));
    c[i] = std::ldexp(u(g), ex(g));
    if ((i & 1023) == 7) b[i] = 0.0;
    if ((i & 1023) == 9) c[i] = -b[i];
    if ((i & 1023) == 11) b[i] = -0.0;
  }
  double *db, *dc, *dd;
  CK(hipMalloc(&db, n * 8));
  CK(hipMalloc(&dc, n * 8));
  CK(hipMalloc(&dd, n * 8));
  CK(hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dc, c.data(), n * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(add_kernel, dim3(n / 1024), dim3(64), 0, 0, db, dc, dd, n);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(d.data(), dd, n * 8, hipMemcpyDeviceToHost));
  long bad = 0, badz = 0;
  for (long i = 0; i < n; ++i) {
    volatile double ref = b[i] + c[i];
    uint64_t x, y;
    double r = ref;
    memcpy(&x, &r, 8);
    memcpy(&y, &d[i], 8);
    if (x != y) {
      if (r == d[i]) badz++;  // only the sign of a zero differs
      else if (bad++ < 5) printf("mismatch %ld: %.17g + %.17g = %.17g, mfma %.17g\n", i, b[i], c[i], r, d[i]);
    }
  }
  printf("mfma add vs host add on %ld pairs: %ld value mismatches, %ld zero-sign mismatches\n", n, bad, badz);
  return 0;
}
