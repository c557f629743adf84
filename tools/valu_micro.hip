// valu_micro.hip — how much of a SIMD's FP64 issue one wave can use.
//
// Each wave runs a long unrolled stream of FP64 VALU instructions (IND
// independent accumulators, or one dependent chain) and the kernel is timed
// at 1, 2, 3 and 4 waves per SIMD (256-thread workgroups = one wave per SIMD
// of a CU, 1..4 workgroups per CU).  If the chip's time stays flat from one
// wave per SIMD to two, a lone wave leaves half the SIMD's issue idle and a
// second resident wave doubles throughput.  Diagnostic for DESIGN.md §4
// (the demodulators run one wave per SIMD); not part of the product.
//
// hipcc -O3 --offload-arch=gfx950 tools/valu_micro.hip -o tools/valu_micro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int IND, int OP>  // OP 0: v_add_f64, 1: v_mul_f64, 2: v_fma_f64, 3: v_add_f32
__global__ __launch_bounds__(256) void stream_kernel(double *out, int iters, double a, double b) {
  double acc[IND];
  float accf[IND];
#pragma unroll
  for (int k = 0; k < IND; ++k) {
    acc[k] = threadIdx.x + k;
    accf[k] = threadIdx.x + k;
  }
  const float af = (float)a, bf = (float)b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int k = 0; k < IND; ++k) {
        if (OP == 0)
          acc[k] = acc[k] + a;
        else if (OP == 1)
          acc[k] = acc[k] * b;
        else if (OP == 2)
          acc[k] = __builtin_fma(acc[k], b, a);
        else
          accf[k] = accf[k] + af;
      }
    }
    (void)bf;
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < IND; ++k) s += acc[k] + accf[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int IND, int OP>
void run(const char *name, double *out, int cus) {
  const int iters = 2000;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int wps = 1; wps <= 4; ++wps) {
    const int grid = cus * wps;
    hipLaunchKernelGGL((stream_kernel<IND, OP>), dim3(grid), dim3(256), 0, 0, out, iters, 1e-300, 1.0000001);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((stream_kernel<IND, OP>), dim3(grid), dim3(256), 0, 0, out, iters, 1e-300, 1.0000001);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double insts = (double)iters * 16 * IND;  // per wave
    // ns per instruction per wave, and chip-wide wave-instructions per SIMD per ns
    printf("%-12s ind=%d waves/SIMD=%d  %.3f ms  %.3f ns/inst per wave  %.3f wave-inst/ns per SIMD\n", name, IND,
           wps, ms, ms * 1e6 / insts, insts * wps / (ms * 1e6));
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  double *out;
  CK(hipMalloc(&out, sizeof(double) * 256 * cus * 4));
  run<8, 0>("add_f64", out, cus);
  run<1, 0>("add_f64 dep", out, cus);
  run<8, 1>("mul_f64", out, cus);
  run<8, 2>("fma_f64", out, cus);
  run<1, 2>("fma_f64 dep", out, cus);
  run<8, 3>("add_f32", out, cus);
  run<1, 3>("add_f32 dep", out, cus);
  CK(hipFree(out));
  return 0;
}
