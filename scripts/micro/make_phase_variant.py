"""Write an instrumented copy of hd_kernels.hip whose layer_body records, per wave,
the s_memtime cycles of each phase (HD_TICK) and adds them into d_phase[] at the end
(one atomicAdd per phase from lane 0), plus extern "C" hd_debug_phase() to read them.

    python scripts/micro/make_phase_variant.py OUT.hip
    bash scripts/ab/kvariant.sh inst OUT.hip hd_kernels.hip
    HD_LIB_PATH=mb/inst/libhdisort.so python scripts/micro/phase_time.py

Timing only (the instrumentation itself shifts the schedule a little); profiles/r06/
layer_phase_cycles*.txt came from it.
"""
import os
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "pyharp_amd", "csrc",
                   "hd_kernels.hip")
s = open(SRC).read()
i0 = s.index("__device__ __forceinline__ int layer_body(")
end = s.index("  return st;\n}", i0)
head, body, tail = s[:i0], s[i0:end], s[end:]


def tick(anchor, k, after=False):
    global body
    assert body.count(anchor) == 1, anchor
    t = f"  HD_TICK({k});\n"
    body = body.replace(anchor, anchor + t if after else t + anchor)


body = body.replace("  int st = 0;\n",
                    "  int st = 0;\n  long long ph_[20] = {};\n  long long t_prev_ = clock64();\n", 1)
tick("  const double rf = om / (1.0 - f);\n", 16, after=True)
tick("  const double mub = beam ? mu0 : 0.0;\n", 17, after=True)
tick("  // L L^T = -A-  (lower triangle of lch)\n", 1)
tick("  // thermal: cvec = dB + 2 (dB/tau') h,  h = W^-1 D^1/2 L^-T L^-1 D^1/2 mu\n", 2)
tick("  // ---- eigenpairs (c_soleig)", 3)
tick("  // L is not needed again until the beam solution: park it", 4)
tick("  if (!jacobi_os<NN>(v, A.max_sweeps)) st |= kStEigen;\n", 5)
tick("  jacobi_os_polish<NN>(v, beam && near_resonance<NN>(v, rmu0 * rmu0, kResPolish));\n", 6,
     after=True)
tick("  // beam, the part that needs only B and k", 7)
tick("  // ---- beam particular solution Z+/- (c_upbeam)", 8)
tick("  // ---- layer operators in the flux-weighted basis ----\n", 9)
tick("  // Psi^T = L^-T V Gamma^1/2 = L^-T B Delta^1/2 -> LDS", 10)
tick("  // Omega = U Delta^1/2 = L B K^-1 Delta^1/2, in place", 11)
tick("  using RL = RecL<NN>;\n", 12)
tick("  double ap_[NN][NN], qvec[NN];\n", 13)
tick("  // ---- store: R~ = A+ - A-", 14)
leg_end = """  }
#pragma unroll
  for (int i = 0; i < NN; ++i)
#pragma unroll
    for (int j = i; j < NN; ++j) {
      const double diag = (i == j) ? Qc.rmu[i] : 0.0;"""
assert body.count(leg_end) == 1
body = body.replace(leg_end, leg_end.replace("  }\n", "  }\n  HD_TICK(18);\n", 1))
body += """  HD_TICK(15);
  if ((threadIdx.x & 63) == 0)
    for (int k_ = 1; k_ < 20; ++k_) atomicAdd(&d_phase[k_], (unsigned long long)ph_[k_]);
"""
macro = """
__device__ unsigned long long d_phase[32];
#define HD_TICK(k) do { __builtin_amdgcn_sched_barrier(0); const long long now_ = clock64(); \\
  ph_[k] = now_ - t_prev_; t_prev_ = now_; __builtin_amdgcn_sched_barrier(0); } while (0)
"""
anchor = "// one wave per block: a layer-kernel wave can take any SIMD"
head = head.replace(anchor, macro + "\n" + anchor, 1)
tail += """
extern "C" int hd_debug_phase(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hd::d_phase), sizeof(unsigned long long) * 32);
  if (e == hipSuccess && reset) {
    unsigned long long z[32] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(hd::d_phase), z, sizeof(z));
  }
  return (int)e;
}
"""
open(sys.argv[1], "w").write(head + body + tail)
