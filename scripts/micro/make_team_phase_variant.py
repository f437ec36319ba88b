"""Instrumented copy of hd_team_mfma.hip: per-wave s_memtime cycles of each phase of
hd_team_mfma_layer_kernel added into d_phase_t[] (lane 0, once per wave at the end),
read by extern "C" hd_debug_phase() (same interface as make_phase_variant.py).

    python scripts/micro/make_team_phase_variant.py OUT.hip
    bash scripts/ab/kvariant.sh tinst OUT.hip hd_team_mfma.hip
    HD_LIB_PATH=mb/tinst/libhdisort.so PHASE_NSTR=32 python scripts/micro/phase_time.py
"""
import os
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "pyharp_amd", "csrc",
                   "hd_team_mfma.hip")
s = open(SRC).read()
i0 = s.index("__global__ __launch_bounds__(64, 2) void hd_team_mfma_layer_kernel(LayerArgs A) {")
i1 = s.index("#if HD_AB_VARIANTS  // the one-wave team sweep")
head, body, tail = s[:i0], s[i0:i1], s[i1:]


def tick(anchor, k, after=False):
    global body
    assert body.count(anchor) == 1, anchor
    t = f"  HD_TICK({k});\n"
    body = body.replace(anchor, anchor + t if after else t + anchor)


body = body.replace("  int st = 0;\n",
                    "  int st = 0;\n  long long ph_[20] = {};\n  long long t_prev_ = clock64();\n", 1)
tick("  // L L^T = S-\n", 1)
tick("  // ---- pre-Jacobi vectors (depend on L only) ----\n", 2)
tick("  double cvec = 0.0, db = 0.0, bsum = 0.0;\n", 3)
tick("  // ---- C C^T = S+ ; B0 = C^T L (lane j: column j) ; C^-1 to LDS ----\n", 4)
tick("    // Warm start (hd_kernels.hpp): B0 <- B0 V0 on the matrix core, V0 the\n", 5)
tick("  // ---- eigenpairs (c_soleig): Sym = L^T S+ L = B0^T B0 = V diag(k^2) V^T ----\n", 6)
tick("  double kk;\n", 7)
tick("  // ---- the dense products on the matrix core; vectors of the beam solution ----\n", 8)
tick("    // beam (c_upbeam): tt = U^T w2 / (1/mu0^2 - k^2), sv = W^-1 D^1/2 U tt, then\n", 9)
tick("    get_m(S0, h, c, Y);            // W (M)\n", 10)
tick("  const double ga = g_i * (cvec - fma(-zp, e0, zm));\n", 11)
tick("    get_rows<NN>(S1, t, i, hr);\n    if (!team_chol<NN, false>(hr, unused, jrd)) st |= kStEigen;\n", 12)
tick("  // ---- store: R~ = A+ - A-, T~ = A- + A+ - I (M layout), S~+, S~-, tau' (T) ----\n", 13)
end = body.rindex("}\n")
body = body[:end] + """  HD_TICK(15);
  if (lane == 0)
    for (int k_ = 1; k_ < 20; ++k_) atomicAdd(&d_phase_t[k_], (unsigned long long)ph_[k_]);
""" + body[end:]
macro = """
__device__ unsigned long long d_phase_t[32];
#define HD_TICK(k) do { __builtin_amdgcn_sched_barrier(0); const long long now_ = clock64(); \\
  ph_[k] = now_ - t_prev_; t_prev_ = now_; __builtin_amdgcn_sched_barrier(0); } while (0)
"""
head = head.replace("// XCD-aware block numbering", macro + "\n// XCD-aware block numbering", 1)
tail += """
extern "C" int hd_debug_phase(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(hd::d_phase_t), sizeof(unsigned long long) * 32);
  if (e == hipSuccess && reset) {
    unsigned long long z[32] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(hd::d_phase_t), z, sizeof(z));
  }
  return (int)e;
}
"""
open(sys.argv[1], "w").write(head + body + tail)
