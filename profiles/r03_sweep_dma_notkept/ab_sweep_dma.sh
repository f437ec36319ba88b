set -e -o pipefail
mkdir -p gpurun_out/sd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_band.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sd/pytest.log 2>&1 || { tail -30 gpurun_out/sd/pytest.log; exit 1; }
tail -2 gpurun_out/sd/pytest.log
run() {  # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $EXTRA > gpurun_out/sd/$tag.json 2>gpurun_out/sd/$tag.err
  echo "$tag $(python -c "import json;d=json.load(open('gpurun_out/sd/$tag.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['path_roofline']['sweep_ms_per_step'])")"
}
EXTRA=""
run c4_plain HD_SWEEP_DMA=0
run c4_dma_g1 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=1
run c4_dma_g2 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=2
run c4_dma_g4 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=4
run c4_dma_g3 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=3
EXTRA="--ngpoint 8"
run g8_plain HD_SWEEP_DMA=0
run g8_dma_g1 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=1
run g8_dma_g2 HD_SWEEP_DMA=1 HD_SWEEP_GROUPS=2
