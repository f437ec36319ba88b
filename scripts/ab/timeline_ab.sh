export HD_AB=1  # the A/B switches below are read only with this opt-in
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in cur head; do
  unset HD_LIB_PATH
  if [ $v != cur ]; then export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl_$v -o kt --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tl_$v.json 2> gpurun_out/tl_$v.err
  echo "$v done"
done
