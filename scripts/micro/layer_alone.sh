set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06e
for v in r05 tj st nomom r05 tj st nomom; do
  HD_LIB_PATH=$PWD/mb/$v/libhdisort.so timeout -k 10 120 python scripts/micro/layer_alone.py $v 2>/dev/null | tee -a gpurun_out/r06e/layer_alone.txt
done
