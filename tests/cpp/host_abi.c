/* Plain-C caller of the drop-in boundary (include/hdisort.h) on host arrays:
 * no torch, no HIP headers -- what a cgo / JNI / N-API / ctypes binding links.
 * A 3-wave x 5-column batch (nstr 8, 12 layers, beam + Lambert), solved by
 * hd_solve_host and by hd_solve_band_host; prints "flux <w> <c> <lev> <up> <dn>"
 * for every level and "band <c> <lev> <up> <dn>", which tests/test_gpu_host_abi.py
 * compares with the CPU oracle.  Exit code = the first non-OK return code. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "hdisort.h"

enum { NW = 3, NC = 5, NL = 12, NSTR = 8, NPROP = 2 + NSTR };

int main(void) {
  static double prop[NW][NC][NL][NPROP], fbeam[NW][NC], umu0[NW][NC], alb[NW][NC];
  static double flux[NW][NC][NL + 1][2], bflux[NC][NL + 1][2], flux2[NW][NC][NL + 1][2];
  static int status[NW][NC];
  const double wt[NW] = {0.2, 0.3, 0.5};
  for (int w = 0; w < NW; ++w)
    for (int c = 0; c < NC; ++c) {
      fbeam[w][c] = 1.0 + 0.1 * w;
      umu0[w][c] = 0.3 + 0.12 * c;
      alb[w][c] = 0.05 + 0.15 * c;
      for (int l = 0; l < NL; ++l) {
        double *p = prop[w][c][l];
        const double g = 0.1 + 0.06 * ((w + c + l) % 10);
        p[0] = 0.01 * pow(1.7, (double)((l + 2 * w + c) % 11));
        p[1] = 0.3 + 0.05 * ((3 * l + w) % 13);
        for (int k = 1; k <= NSTR; ++k) p[1 + k] = pow(g, k);
      }
    }
  hd_context *ctx = NULL;
  int rc = hd_context_create(&ctx, 0);
  if (rc) {
    fprintf(stderr, "hd_context_create: %s\n", hd_last_error(NULL));
    return rc;
  }
  hd_config cfg = {NSTR, NSTR, NL, NPROP, HD_FLAG_LAMBER | HD_FLAG_ONLYFL};
  hd_inputs in = {NW, NC, &prop[0][0][0][0], &fbeam[0][0], &umu0[0][0], &alb[0][0],
                  NULL, NULL, NULL, NULL, NULL, NULL, NULL};
  rc = hd_solve_host(ctx, &cfg, &in, &flux[0][0][0][0], &status[0][0]);
  if (rc) {
    fprintf(stderr, "hd_solve_host: %s\n", hd_last_error(ctx));
    return rc;
  }
  rc = hd_solve_band_host(ctx, &cfg, &in, wt, &bflux[0][0][0], &flux2[0][0][0][0], NULL);
  if (rc) {
    fprintf(stderr, "hd_solve_band_host: %s\n", hd_last_error(ctx));
    return rc;
  }
  for (int w = 0; w < NW; ++w)
    for (int c = 0; c < NC; ++c)
      for (int v = 0; v <= NL; ++v) {
        printf("flux %d %d %d %.17g %.17g\n", w, c, v, flux[w][c][v][0], flux[w][c][v][1]);
        if (flux2[w][c][v][0] != flux[w][c][v][0] || flux2[w][c][v][1] != flux[w][c][v][1]) {
          fprintf(stderr, "band call's per-point fluxes differ from hd_solve_host's\n");
          return 9;
        }
      }
  for (int c = 0; c < NC; ++c)
    for (int v = 0; v <= NL; ++v) printf("band %d %d %.17g %.17g\n", c, v, bflux[c][v][0], bflux[c][v][1]);
  hd_context_destroy(ctx);
  return 0;
}
