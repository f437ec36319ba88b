# layer kernel alone (scripts/micro/layer_alone.py) for library variants mb/<name> ("cur" = in-tree)
#   gpurun -- bash scripts/micro/layer_alone.sh TAG v1 v2 v1 v2 ...
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 120 python scripts/micro/layer_alone.py $v 2>/dev/null | tee -a gpurun_out/$TAG/layer_alone.txt
done
