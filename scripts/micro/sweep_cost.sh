# marginal wall time of one Jacobi sweep in the layer kernel: layer kernel alone with
# the sweep cap at 1..5 (the debug cap; results unconverged) for library variants
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  for k in 1 2 3 4 5; do
    HD_MAX_SWEEPS=$k timeout -k 10 120 python scripts/micro/layer_alone.py $v 2>/dev/null | tee -a gpurun_out/$TAG/sweep_cost.txt
  done
done
