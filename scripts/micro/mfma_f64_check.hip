// Checks the operand/result lane maps of v_mfma_f64_16x16x4_f64 on gfx950 with
// exact integer data: lane l = 16h + c holds A[c][4s+h] and B[4s+h][c] at
// k-step s, and D[h+4m][c] in result register m.  Prints max |D - A.B|.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(const double* A, const double* B, double* D) {
  const int l = threadIdx.x, h = l >> 4, c = l & 15;
  d4 acc = {0, 0, 0, 0};
  for (int s = 0; s < 4; ++s)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[c * 16 + 4 * s + h], B[(4 * s + h) * 16 + c], acc, 0, 0, 0);
  for (int m = 0; m < 4; ++m) D[(h + 4 * m) * 16 + c] = acc[m];
}
// throughput: every wave issues 4 independent accumulator chains
__global__ void tput(double* out, int iters) {
  const double a = 1.0 + 1e-9 * threadIdx.x, b = 1.0 - 1e-9 * threadIdx.x;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  if (s[0] == 12345.0) out[0] = s[1];
}
int main() {
  double A[256], B[256], D[256], R[256];
  for (int i = 0; i < 256; ++i) { A[i] = (i * 7) % 13 - 6; B[i] = (i * 5) % 11 - 5; }
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double t = 0;
      for (int k = 0; k < 16; ++k) t += A[i * 16 + k] * B[k * 16 + j];
      R[i * 16 + j] = t;
    }
  double *dA, *dB, *dD;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dD, 2048);
  hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(D, dD, 2048, hipMemcpyDeviceToHost);
  double e = 0;
  for (int i = 0; i < 256; ++i) e = fmax(e, fabs(D[i] - R[i]));
  printf("mfma_f64_16x16x4 layout check: max |D - AB| = %g\n", e);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const int iters = 4000, blocks = 1024 * 4, threads = 64;
  hipLaunchKernelGGL(tput, dim3(blocks), dim3(threads), 0, 0, dD, 10);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(tput, dim3(blocks), dim3(threads), 0, 0, dD, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
  const double flop = 2048.0 * 4 * iters * blocks;
  printf("mfma_f64_16x16x4 throughput: %.1f TFLOP/s (%d waves x %d MFMA, %.3f ms)\n", flop / ms / 1e9, blocks, 4 * iters, ms);
  return e != 0.0;
}
