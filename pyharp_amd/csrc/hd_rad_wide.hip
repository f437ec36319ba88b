// hd_rad_wide.hip -- the intensity-path kernels of hd_rad.hip for nstr 18..32
// (NN 9..16), compiled with their NN-loops rolled: one lane per (solve, mode)
// problem as at nstr <= 16, with the per-lane NN x NN matrices in private
// memory instead of registers.  Same arithmetic, same record layouts; it is
// the coverage path of radiances at large nstr (every harp flux call site uses
// the team kernels of hd_team*.hip instead).  Symbols live in hd::wide.
#define HD_RAD_WIDE 1
#define HD_RUNROLL _Pragma("nounroll")
#define HD_UNROLL_NN _Pragma("nounroll")
#include "hd_rad.hip"
