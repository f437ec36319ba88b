# C4 and its 8-GPU rank shape with the fused band sum (default) and with --no-fuse (hd_solve with
# per-g fluxes stored, then hd_band_flux) as the timed step, interleaved on one box:
#   gpurun -- bash scripts/micro/fuse_ab.sh TAG
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:?tag}; mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for mode in fused nofuse; do
    for shape in c4 g8; do
      a="--steps 10 --warmup 3 --no-cpu-baseline --no-extra"
      [ $mode = nofuse ] && a="$a --no-fuse"
      [ $shape = g8 ] && a="$a --ngpoint 8"
      f=gpurun_out/$TAG/${shape}_${mode}_$rep.json
      timeout -k 10 200 python bench.py $a > $f 2>/dev/null
      python -c "import json; d=json.load(open('$f')); print('$shape $mode', d['value'], d['ms_per_step'])"
    done
  done
done
