#!/bin/bash
# both A/B scripts in one box session:  gpurun -- bash scripts/ab/lean_quad_ab.sh TAG [ROUNDS]
export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
bash scripts/ab/quad_ab.sh $1_quad ${2:-2}
bash scripts/ab/lean_ab.sh $1_lean ${2:-2}
