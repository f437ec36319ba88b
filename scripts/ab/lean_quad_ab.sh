#!/bin/bash
# both A/B scripts in one box session:  gpurun -- bash scripts/ab/lean_quad_ab.sh TAG [ROUNDS]
set -e -o pipefail
bash scripts/ab/quad_ab.sh $1_quad ${2:-2}
bash scripts/ab/lean_ab.sh $1_lean ${2:-2}
