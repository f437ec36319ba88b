# Jacobi sweeps per layer item and per 64-lane wave on the GPU (device status bits,
# scripts/micro/sweep_count.py) for the in-tree library and mb/<name> variants
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:?tag}; shift; mkdir -p $OUT
for v in "$@"; do
  if [ $v = cur ]; then unset HD_LIB_PATH; else export HD_LIB_PATH=$PWD/mb/$v/libhdisort.so; fi
  echo "== $v" >> $OUT/sweeps.txt
  timeout -k 10 120 python scripts/micro/sweep_count.py 16 2>/dev/null >> $OUT/sweeps.txt
  timeout -k 10 120 python scripts/micro/sweep_count.py 8 2>/dev/null >> $OUT/sweeps.txt
done
cat $OUT/sweeps.txt
