#!/bin/bash
# N>1 rehearsal on a 1-GPU box: 2-rank GPU test (gloo) + bench.py under torchrun with 2 ranks
set -e -o pipefail
OUT=gpurun_out/${1:-dist}
mkdir -p "$OUT"
timeout -k 10 300 python -m pytest tests/test_gpu_distributed.py -x -q > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
HD_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > "$OUT/bench2.json" 2> "$OUT/bench2.err" || { tail -30 "$OUT/bench2.err"; exit 1; }
cat "$OUT/bench2.json"
